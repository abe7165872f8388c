// Experiment: gemm_wgrad (gemm.hpp) with 8-wave workgroups (512 threads) owning a BN x BK = 128 x 256 tile of a split:
// the G slab rows are loaded once for both 128-column halves of X (25 % fewer global-load bytes per MFMA than the
// 4-wave 128 x 128 tile), two workgroups per CU (LDS 49 KB each), waves 2 (n) x 4 (k) with 64 x 64 wave tiles and the
// library kernel's per-element accumulation order (P bitwise equal).
// Measured (tools/gemm_bench16.hip): 0.893 ms vs 0.854 for the library's 4-wave 128 x 128 kernel — not kept.
#pragma once
#include "../../nerf-sys_amd/csrc/gemm.hpp"

template <int BN, int BK, int WAVES_N, int MR = 16>
__global__ __launch_bounds__(512) void gemm_wgrad8_kernel(const float* __restrict__ G, int ldg,
                                                          const float* __restrict__ X, int ldx,
                                                          float* __restrict__ P, int ldp, float* __restrict__ Pb,
                                                          int64_t slab, int64_t rows_per_split, int64_t M,
                                                          int n_ktiles, int n_tiles) {
  constexpr int NT = 512, NWAVE = NT / 64;
  constexpr int WAVES_K = NWAVE / WAVES_N;
  constexpr int WTN = BN / WAVES_N, WTK = BK / WAVES_K;
  constexpr int TM = WTN / 32, TN = WTK / 32;
  constexpr int G_F4 = MR * BN / 4, X_F4 = MR * BK / 4;
  constexpr int G_PER = (G_F4 + NT - 1) / NT, X_PER = (X_F4 + NT - 1) / NT;
  __shared__ __attribute__((aligned(16))) float smem[2 * MR * (BN + BK)];
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
#define W8_GLOAD(m_)                                                                           \
  _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                         \
    const int f = tid + NT * i;                                                                \
    if (G_F4 % NT == 0 || f < G_F4)                                                            \
      rg[i] = *reinterpret_cast<const float4*>(G + ((m_) + f / (BN / 4)) * ldg + n0 + (f % (BN / 4)) * 4); \
  }                                                                                            \
  _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                         \
    const int f = tid + NT * i;                                                                \
    if (X_F4 % NT == 0 || f < X_F4)                                                            \
      rx[i] = *reinterpret_cast<const float4*>(X + ((m_) + f / (BK / 4)) * ldx + k0 + (f % (BK / 4)) * 4); \
  }
#define W8_SSTORE(buf_)                                                                        \
  {                                                                                            \
    float* Gs_ = smem + (buf_) * MR * (BN + BK);                                               \
    float* Xs_ = Gs_ + MR * BN;                                                                \
    _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                       \
      const int f = tid + NT * i;                                                              \
      if (G_F4 % NT == 0 || f < G_F4) *reinterpret_cast<float4*>(Gs_ + f * 4) = rg[i];         \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                       \
      const int f = tid + NT * i;                                                              \
      if (X_F4 % NT == 0 || f < X_F4) *reinterpret_cast<float4*>(Xs_ + f * 4) = rx[i];         \
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
    W8_GLOAD(r0);
    W8_SSTORE(0);
  }
  __syncthreads();
  for (int64_t it = 0; it < nit; ++it) {
    const int cur = (int)(it & 1);
    W8_GLOAD(r0 + (it + 1 < nit ? it + 1 : it) * MR);
    const float* Gs = smem + cur * MR * (BN + BK);
    const float* Xs = Gs + MR * BN;
#pragma unroll
    for (int ss = 0; ss < MR / 2; ++ss) {
      const int row = 16 * (ss >> 3) + 8 * lh + (ss & 7);
      float af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = Gs[row * BN + wn * WTN + a * 32 + li];
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = Xs[row * BK + wk * WTK + b * 32 + li];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        if (do_bias) bsum[a] += af[a];
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[a], bf[b], acc[a][b], 0, 0, 0);
      }
    }
    W8_SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef W8_GLOAD
#undef W8_SSTORE
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
