// Measured and not kept (tools/gemm_bench16.hip, C2 fine-net shape): the weight-gradient GEMM on 16x16x4 MFMAs ran
// 0.887-0.962 ms per 256x256 launch against 0.857 ms for the library's 32x32x2 gemm_wgrad_kernel (MINW 2 / 1, MR 32).
#pragma once
#include "../../nerf-sys_amd/csrc/gemm.hpp"

// gemm_wgrad (gemm.hpp) on v_mfma_f32_16x16x4_f32.  P[s][n][k] = sum over the rows m of split s of
// G[m][n] X[m][k] (+ bias column sums).  MFMA A = G^T (i = n, k-slot = row), B = X (k-slot = row, j = k); MFMA s of a
// 16-row sub-slab takes rows 4s .. 4s+3 (k-slot g = row 4s + g), so every element accumulates its rows in sequential
// order.  LDS row pitch = width + 16 floats (= 16 mod 64 banks): the four k-slot groups of a ds_read_b32 (16
// consecutive floats of rows 4s .. 4s+3) hit 64 distinct banks.  Lane l holds P[n = .. + 4g + r][k = .. + (l & 15)].
template <int BN, int BK, int WAVES_N, int MR = 16, int MINW = 1>
__global__ __launch_bounds__(256, MINW) void gemm_wgrad16_kernel(const float* __restrict__ G, int ldg,
                                                                 const float* __restrict__ X, int ldx,
                                                                 float* __restrict__ P, int ldp, float* __restrict__ Pb,
                                                                 int64_t slab, int64_t rows_per_split, int64_t M,
                                                                 int n_ktiles, int n_tiles) {
  constexpr int WAVES_K = 4 / WAVES_N;
  constexpr int WTN = BN / WAVES_N, WTK = BK / WAVES_K;
  constexpr int TM = WTN / 16, TN = WTK / 16;
  constexpr int PG = BN + 16, PX = BK + 16;
  constexpr int G_F4 = MR * BN / 4, X_F4 = MR * BK / 4;
  constexpr int G_PER = (G_F4 + 255) / 256, X_PER = (X_F4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * MR * (PG + PX)];
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
  const int lr = lane & 15, lg = lane >> 4;
  const bool do_bias = (Pb != nullptr) && kt == 0 && wk == 0;
  float4 rg[G_PER], rx[X_PER];
#define W16_GLOAD(m_)                                                                          \
  _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    if (G_F4 % 256 == 0 || f < G_F4)                                                           \
      rg[i] = *reinterpret_cast<const float4*>(G + ((m_) + f / (BN / 4)) * ldg + n0 + (f % (BN / 4)) * 4); \
  }                                                                                            \
  _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    if (X_F4 % 256 == 0 || f < X_F4)                                                           \
      rx[i] = *reinterpret_cast<const float4*>(X + ((m_) + f / (BK / 4)) * ldx + k0 + (f % (BK / 4)) * 4); \
  }
#define W16_SSTORE(buf_)                                                                       \
  {                                                                                            \
    float* Gs_ = smem + (buf_) * MR * (PG + PX);                                               \
    float* Xs_ = Gs_ + MR * PG;                                                                \
    _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (G_F4 % 256 == 0 || f < G_F4)                                                         \
        *reinterpret_cast<float4*>(Gs_ + (f / (BN / 4)) * PG + (f % (BN / 4)) * 4) = rg[i];   \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (X_F4 % 256 == 0 || f < X_F4)                                                         \
        *reinterpret_cast<float4*>(Xs_ + (f / (BK / 4)) * PX + (f % (BK / 4)) * 4) = rx[i];   \
    }                                                                                          \
  }
  nerf_f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = nerf_f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) bsum[a] = 0.f;
  const int64_t nit = (r1 - r0) / MR;
  if (nit > 0) {
    W16_GLOAD(r0);
    W16_SSTORE(0);
  }
  __syncthreads();
  for (int64_t it = 0; it < nit; ++it) {
    const int cur = (int)(it & 1);
    W16_GLOAD(r0 + (it + 1 < nit ? it + 1 : it) * MR);
    const float* Gs = smem + cur * MR * (PG + PX);
    const float* Xs = Gs + MR * PG;
#pragma unroll
    for (int ss = 0; ss < MR / 4; ++ss) {
      const int row = 4 * ss + lg;
      float af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = Gs[row * PG + wn * WTN + a * 16 + lr];
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = Xs[row * PX + wk * WTK + b * 16 + lr];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        if (do_bias) bsum[a] += af[a];
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a], bf[b], acc[a][b], 0, 0, 0);
      }
    }
    W16_SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef W16_GLOAD
#undef W16_SSTORE
  float* Ps = P + (int64_t)s * slab;
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int k = k0 + wk * WTK + b * 16 + lr;
#pragma unroll
      for (int r = 0; r < 4; ++r) Ps[(int64_t)(n0 + wn * WTN + a * 16 + 4 * lg + r) * ldp + k] = acc[a][b][r];
    }
  if (do_bias) {
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      float v = bsum[a];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lg == 0) Pb[(int64_t)s * slab + n0 + wn * WTN + a * 16 + lr] = v;
    }
  }
}

