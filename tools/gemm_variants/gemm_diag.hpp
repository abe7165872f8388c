// Diagnostic copies of gemm_nt_body (gemm.hpp) with parts of the k-loop removed, to locate the fp32 GEMM's
// non-MFMA cycles: D = 0 library loop; 1 no global loads / LDS stores in the loop (LDS reads + MFMA only);
// 2 no LDS reads (fragments read once before the loop; global loads + LDS stores + MFMA); 3 MFMA only;
// 4 no barrier in the loop (results wrong, timing only).  Outputs of D > 0 are wrong by construction.
#pragma once
#include "../../nerf-sys_amd/csrc/gemm.hpp"

template <int BM, int BN, int WAVES_M, int EPI, int D, int MINW = 4>
__global__ __launch_bounds__(256, MINW) void gemm_diag_kernel(const float* __restrict__ A, int lda,
                                                             const float* __restrict__ B, int ldb,
                                                             const float* __restrict__ bias, float* __restrict__ C,
                                                             int ldc, const uint32_t* __restrict__ mbits, int ldmb,
                                                             uint32_t* __restrict__ mbits_out, int K, int n_ntiles) {
  constexpr int BK = 16, LS = BK + 4, C4 = BK / 4, HK = BK / 2;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int A_F4 = BM * C4, B_F4 = BN * C4;
  constexpr int A_PER = (A_F4 + 255) / 256, B_PER = (B_F4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LS];
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;
  const float* Ab = A + m0 * lda;
  const float* Bb = B + (int64_t)n0 * ldb;
  float4 ra[A_PER], rb[B_PER];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_PER; ++i) { const int f = tid + 256 * i; ra[i] = *reinterpret_cast<const float4*>(Ab + (int64_t)(f / C4) * lda + k0 + (f % C4) * 4); }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) { const int f = tid + 256 * i; rb[i] = *reinterpret_cast<const float4*>(Bb + (int64_t)(f / C4) * ldb + k0 + (f % C4) * 4); }
  };
  auto sstore = [&](int buf) {
    float* As_ = smem + buf * (BM + BN) * LS;
    float* Bs_ = As_ + BM * LS;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) { const int f = tid + 256 * i; *reinterpret_cast<float4*>(As_ + (f / C4) * LS + (f % C4) * 4) = ra[i]; }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) { const int f = tid + 256 * i; *reinterpret_cast<float4*>(Bs_ + (f / C4) * LS + (f % C4) * 4) = rb[i]; }
  };
  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int nk = K / BK;
  gload(0);
  sstore(0);
  __syncthreads();
  float4 af0[TM][2], bf0[TN][2];
  if (D == 2 || D == 3) {
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
#pragma unroll
      for (int a = 0; a < TM; ++a) af0[a][hh] = *reinterpret_cast<const float4*>(smem + (wm * WTM + a * 32 + li) * LS + HK * lh + 4 * hh);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf0[b][hh] = *reinterpret_cast<const float4*>(smem + BM * LS + (wn * WTN + b * 32 + li) * LS + HK * lh + 4 * hh);
    }
  }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (D == 0 || D == 2 || D == 4) gload((kt + 1 < nk ? kt + 1 : kt) * BK);
    const float* As = smem + cur * (BM + BN) * LS;
    const float* Bs = As + BM * LS;
#pragma unroll
    for (int hh = 0; hh < HK / 4; ++hh) {
      float4 af[TM], bf[TN];
      if (D == 2 || D == 3) {
#pragma unroll
        for (int a = 0; a < TM; ++a) af[a] = af0[a][hh];
#pragma unroll
        for (int b = 0; b < TN; ++b) bf[b] = bf0[b][hh];
      } else {
#pragma unroll
        for (int a = 0; a < TM; ++a) af[a] = *reinterpret_cast<const float4*>(As + (wm * WTM + a * 32 + li) * LS + HK * lh + 4 * hh);
#pragma unroll
        for (int b = 0; b < TN; ++b) bf[b] = *reinterpret_cast<const float4*>(Bs + (wn * WTN + b * 32 + li) * LS + HK * lh + 4 * hh);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(bf[b][s], af[a][s], acc[a][b], 0, 0, 0);
    }
    if (D == 0 || D == 2 || D == 4) sstore(cur ^ 1);
    if (D != 4 && D != 3) __syncthreads();
  }
  nt_epilogue<TM, TN, WTM, WTN, EPI>(acc, m0 + wm * WTM, n0 + wn * WTN, li, lh, bias, C, ldc, mbits, ldmb, mbits_out);
}
