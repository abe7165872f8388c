// Weights-stationary fp32 MFMA NT GEMM for the NeRF MLP layers:   C[m][n] = epi( sum_k A[m][k] * W[n][k] )
//
// The layer shapes are tall and thin (M = 10^5..10^6 samples, N <= 256, K <= 320), so a block keeps its
// NB x K slice of the weights resident in LDS for its whole life (loaded once per launch, 133 KB at
// NB = 128, K = 256) and streams row panels of the activations straight from HBM into registers:
//   * no LDS staging of the activations and no barrier in the main loop -- each wave runs on its own,
//     with a D-deep register ring of activation k-slabs in flight (the counted waits are the compiler's);
//   * one 512-thread block per CU (LDS-bound), 8 waves = 2 per SIMD, so one wave's load or epilogue
//     bubbles are covered by its SIMD partner's MFMAs;
//   * static row-panel partition (persistent blocks), the NB-column blocks of one panel on one XCD.
// MFMA: v_mfma_f32_32x32x2_f32 with swapped operands (tile = C^T: lane li holds output row m, 16 columns in
// its registers) and the k order k = 8 h + 4 j + s of gemm.hpp, so results are bitwise identical to
// gemm_nt_kernel.  LDS row pitch K + 4 floats: the 16 lanes of a ds_read_b128 group hit 16 distinct slots.
#pragma once
#include "../../nerf-sys_amd/csrc/gemm.hpp"

template <int K, int NB, int TM, int TN, int WAVES_N, int EPI, int D>
__global__ __launch_bounds__(512, 1) void gemm_ws_kernel(const float* __restrict__ A, int lda,
                                                         const float* __restrict__ W, int ldw,
                                                         const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                                         const uint32_t* __restrict__ mbits, int ldmb,
                                                         uint32_t* __restrict__ mbits_out, int n_panels, int n_groups,
                                                         int n_cblk) {
  constexpr int WAVES_M = 8 / WAVES_N;
  constexpr int PM = WAVES_M * TM * 32;  // rows per panel
  static_assert(NB == WAVES_N * TN * 32, "column block");
  static_assert(K % 16 == 0, "k");
  constexpr int NK = K / 16;
  constexpr int LW = K + 4;
  __shared__ __attribute__((aligned(16))) float sW[NB * LW];

  const int b = blockIdx.x;
  const int cb = (b >> 3) % n_cblk;
  const int g = (b & 7) + 8 * (b / (8 * n_cblk));
  const int n0 = cb * NB;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;

  // resident weights
  {
    constexpr int NF4 = NB * (K / 4);
    constexpr int PER = (NF4 + 511) / 512;
    float4 t[PER];  // all loads in flight before the first store
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + 512 * j;
      if (NF4 % 512 == 0 || i < NF4) {
        const int r = i / (K / 4), c = i - r * (K / 4);
        t[j] = *reinterpret_cast<const float4*>(W + (int64_t)(n0 + r) * ldw + 4 * c);
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + 512 * j;
      if (NF4 % 512 == 0 || i < NF4) {
        const int r = i / (K / 4), c = i - r * (K / 4);
        *reinterpret_cast<float4*>(sW + r * LW + 4 * c) = t[j];
      }
    }
  }
  __syncthreads();
  if (g >= n_groups) return;

  const float* wl[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) wl[t] = sW + (wn * TN * 32 + t * 32 + li) * LW + 8 * lh;

  for (int p = g; p < n_panels; p += n_groups) {
    const int64_t mw = (int64_t)p * PM + wm * TM * 32;
    const float* al[TM];
#pragma unroll
    for (int a = 0; a < TM; ++a) al[a] = A + (mw + a * 32 + li) * lda + 8 * lh;

    float4 ra[D][TM][2];
#pragma unroll
    for (int s = 0; s < D - 1; ++s)
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        ra[s][a][0] = *reinterpret_cast<const float4*>(al[a] + 16 * s);
        ra[s][a][1] = *reinterpret_cast<const float4*>(al[a] + 16 * s + 4);
      }
    float4 wf[2][TN][2];
#pragma unroll
    for (int t = 0; t < TN; ++t) {
      wf[0][t][0] = *reinterpret_cast<const float4*>(wl[t]);
      wf[0][t][1] = *reinterpret_cast<const float4*>(wl[t] + 4);
    }

    nerf_f32x16 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int t = 0; t < TN; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][t][r] = 0.f;

#pragma unroll
    for (int kt = 0; kt < NK; ++kt) {
      // activation slab kt + D - 1 into the ring, weight fragments of slab kt + 1 from LDS
      if (kt + D - 1 < NK) {
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          ra[(kt + D - 1) % D][a][0] = *reinterpret_cast<const float4*>(al[a] + 16 * (kt + D - 1));
          ra[(kt + D - 1) % D][a][1] = *reinterpret_cast<const float4*>(al[a] + 16 * (kt + D - 1) + 4);
        }
      }
      if (kt + 1 < NK) {
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          wf[(kt + 1) & 1][t][0] = *reinterpret_cast<const float4*>(wl[t] + 16 * (kt + 1));
          wf[(kt + 1) & 1][t][1] = *reinterpret_cast<const float4*>(wl[t] + 16 * (kt + 1) + 4);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int t = 0; t < TN; ++t)
              acc[a][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(wf[kt & 1][t][h][s], ra[kt % D][a][h][s], acc[a][t], 0, 0,
                                                               0);
      __builtin_amdgcn_sched_barrier(0);
    }
    nt_epilogue<TM, TN, TM * 32, TN * 32, EPI>(acc, mw, n0 + wn * TN * 32, li, lh, bias, C, ldc, mbits, ldmb, mbits_out);
  }
}
