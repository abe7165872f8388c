// Experiment: gemm_wgrad (gemm.hpp) with the slab stored TRANSPOSED in LDS (Gt[n][r], Xt[k][r], 16 rows per slab,
// 80-B pitch) so that a lane's 8 k-slot values (rows 8 lh .. 8 lh + 7 of its column) come as two ds_read_b128
// instead of eight ds_read_b32.  Global loads: thread f reads row m = f % MR, float4 column c = f / MR (a wave's lanes
// cover 16 rows x 4 float4 columns), written as four ds_write_b32 to Gt[4c + j][m]: bank (16 c + 20 j + m) mod 64,
// conflict-free.  MFMA ss of a 16-row sub-slab consumes rows (ss, 8 + ss) exactly like the library kernel, so P is
// bitwise the library's.
#pragma once
#include "../../nerf-sys_amd/csrc/gemm.hpp"

template <int BN, int BK, int WAVES_N, int MINW = 1>
__global__ __launch_bounds__(256, MINW) void gemm_wgrad_t_kernel(const float* __restrict__ G, int ldg,
                                                                const float* __restrict__ X, int ldx,
                                                                float* __restrict__ P, int ldp, float* __restrict__ Pb,
                                                                int64_t slab, int64_t rows_per_split, int64_t M,
                                                                int n_ktiles, int n_tiles) {
  constexpr int MR = 16, PR = 20;
  constexpr int WAVES_K = 4 / WAVES_N;
  constexpr int WTN = BN / WAVES_N, WTK = BK / WAVES_K;
  constexpr int TM = WTN / 32, TN = WTK / 32;
  constexpr int G_F4 = MR * BN / 4, X_F4 = MR * BK / 4;
  static_assert(G_F4 % 256 == 0 && X_F4 % 256 == 0, "whole passes");
  constexpr int G_PER = G_F4 / 256, X_PER = X_F4 / 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * (BN + BK) * PR];
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int s = lin / n_tiles;
  const int tile = lin - s * n_tiles;
  const int nt = tile / n_ktiles, kt = tile - nt * n_ktiles;
  const int n0 = nt * BN, k0 = kt * BK;
  const int64_t r0 = (int64_t)s * rows_per_split;
  int64_t r1 = r0 + rows_per_split;
  if (r1 > M) r1 = M;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave / WAVES_K, wk = wave % WAVES_K;
  const int li = lane & 31, lh = lane >> 5;
  const bool do_bias = (Pb != nullptr) && kt == 0 && wk == 0;
  float4 rg[G_PER], rx[X_PER];
#define WT_GLOAD(m_)                                                                           \
  _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    rg[i] = *reinterpret_cast<const float4*>(G + ((m_) + f % MR) * ldg + n0 + (f / MR) * 4);   \
  }                                                                                            \
  _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    rx[i] = *reinterpret_cast<const float4*>(X + ((m_) + f % MR) * ldx + k0 + (f / MR) * 4);   \
  }
#define WT_SSTORE(buf_)                                                                        \
  {                                                                                            \
    float* Gs_ = smem + (buf_) * (BN + BK) * PR;                                               \
    float* Xs_ = Gs_ + BN * PR;                                                                \
    _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      float* d = Gs_ + (4 * (f / MR)) * PR + f % MR;                                           \
      d[0] = rg[i].x; d[PR] = rg[i].y; d[2 * PR] = rg[i].z; d[3 * PR] = rg[i].w;               \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      float* d = Xs_ + (4 * (f / MR)) * PR + f % MR;                                           \
      d[0] = rx[i].x; d[PR] = rx[i].y; d[2 * PR] = rx[i].z; d[3 * PR] = rx[i].w;               \
    }                                                                                          \
  }
  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  float bsum[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) bsum[a] = 0.f;
  const int64_t nit = (r1 - r0) / MR;
  if (nit > 0) {
    WT_GLOAD(r0);
    WT_SSTORE(0);
  }
  __syncthreads();
  for (int64_t it = 0; it < nit; ++it) {
    const int cur = (int)(it & 1);
    WT_GLOAD(r0 + (it + 1 < nit ? it + 1 : it) * MR);
    const float* Gs = smem + cur * (BN + BK) * PR;
    const float* Xs = Gs + BN * PR;
    float4 ga[TM][2], xb[TN][2];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) ga[a][hq] = *reinterpret_cast<const float4*>(Gs + (wn * WTN + a * 32 + li) * PR + 8 * lh + 4 * hq);
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) xb[b][hq] = *reinterpret_cast<const float4*>(Xs + (wk * WTK + b * 32 + li) * PR + 8 * lh + 4 * hq);
#pragma unroll
    for (int ss = 0; ss < 8; ++ss) {
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const float af = ga[a][ss >> 2][ss & 3];
        if (do_bias) bsum[a] += af;
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af, xb[b][ss >> 2][ss & 3], acc[a][b], 0, 0, 0);
      }
    }
    WT_SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef WT_GLOAD
#undef WT_SSTORE
  float* Ps = P + (int64_t)s * slab;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int k = k0 + wk * WTK + b * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * WTN + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        Ps[(int64_t)n * ldp + k] = acc[a][b][r];
      }
    }
  if (do_bias) {
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const float v = bsum[a] + __shfl_xor(bsum[a], 32, 64);
      if (lh == 0) Pb[(int64_t)s * slab + n0 + wn * WTN + a * 32 + li] = v;
    }
  }
}

// Measured (tools/gemm_bench16.hip, 9 interleaved rounds): this kernel 0.867-0.873 ms vs the library's 0.861-0.874 (no
// gain: ds_read instruction count does not bound the weight gradient); the same transposed slab feeding 16x16x4 MFMAs
// (one ds_read_b128 per 16-row slab and block) 0.854 at MINW 2 / 0.932 at 3 / 0.977 at 1 — not kept either.
