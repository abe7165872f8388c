// Experiment: persistent gemm_nt16 — each workgroup walks tiles t = blockIdx.x + k * gridDim.x (same XCD for a grid
// that is a multiple of 8), and the last k-slab of tile t loads slab 0 of tile t + G, so the next tile's prologue
// (first global load, LDS store, barrier) overlaps the current tile's last MFMA block and epilogue.
// Measured (tools/gemm_bench16.hip): with an if/else between the two loads, dgrad 1.786 ms at 1024 workgroups, 1.491
// at 768, vs 0.826 for gemm_nt16_kernel; with the branch-free selects below 0.907 / 0.890 vs 0.825.
#pragma once
#include "../../nerf-sys_amd/csrc/gemm.hpp"

template <int BM, int BN, int WAVES_M, int EPI, int MINW = 3>
__global__ __launch_bounds__(256, MINW) void gemm_nt16p_kernel(const float* __restrict__ A, int lda,
                                                              const float* __restrict__ B, int ldb,
                                                              const float* __restrict__ bias, float* __restrict__ C,
                                                              int ldc, const uint32_t* __restrict__ mbits, int ldmb,
                                                              uint32_t* __restrict__ mbits_out, int K, int n_ntiles,
                                                              int ntiles) {
  constexpr int BK = 16, LS = BK + 4, C4 = BK / 4;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_F4 = BM * C4, B_F4 = BN * C4;
  constexpr int A_PER = (A_F4 + 255) / 256, B_PER = (B_F4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LS];
  const int G = gridDim.x;
  int t = blockIdx.x;
  if (t >= ntiles) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int lr = lane & 15, lg = lane >> 4;
  auto tile_of = [&](int tt, int64_t& m0, int& n0) {
    const int tile = xcd_remap(tt, ntiles);
    const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
    m0 = (int64_t)mt * BM;
    n0 = nt * BN;
  };
  int64_t m0;
  int n0;
  tile_of(t, m0, n0);
  const float* Ab = A + m0 * lda;
  const float* Bb = B + (int64_t)n0 * ldb;
  float4 ra[A_PER], rb[B_PER];
#define P16_GLOAD(Ap_, Bp_, k0_)                                                               \
  _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    ra[i] = *reinterpret_cast<const float4*>((Ap_) + (int64_t)(f / C4) * lda + (k0_) + (f % C4) * 4); \
  }                                                                                            \
  _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    rb[i] = *reinterpret_cast<const float4*>((Bp_) + (int64_t)(f / C4) * ldb + (k0_) + (f % C4) * 4); \
  }
#define P16_SSTORE(buf_)                                                                       \
  {                                                                                            \
    float* As_ = smem + (buf_) * (BM + BN) * LS;                                               \
    float* Bs_ = As_ + BM * LS;                                                                \
    _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      *reinterpret_cast<float4*>(As_ + (f / C4) * LS + (f % C4) * 4) = ra[i];                  \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      *reinterpret_cast<float4*>(Bs_ + (f / C4) * LS + (f % C4) * 4) = rb[i];                  \
    }                                                                                          \
  }
  const int nk = K / BK;
  P16_GLOAD(Ab, Bb, 0);
  P16_SSTORE(0);
  __syncthreads();
  int cur = 0;
  for (;;) {
    const int tn = t + G;
    const bool more = tn < ntiles;
    int64_t m0n = m0;
    int n0n = n0;
    if (more) tile_of(tn, m0n, n0n);
    const float* An = A + m0n * lda;
    const float* Bn = B + (int64_t)n0n * ldb;
    nerf_f32x4 acc[TM][TN];
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] = nerf_f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk; ++kt) {
      {
        const bool last = kt + 1 == nk;  // branch-free: the last slab loads slab 0 of the next tile
        const float* Ap = last ? An : Ab;
        const float* Bp = last ? Bn : Bb;
        const int k0 = last ? 0 : (kt + 1) * BK;
        P16_GLOAD(Ap, Bp, k0);
      }
      const float* As = smem + cur * (BM + BN) * LS;
      const float* Bs = As + BM * LS;
      float4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = *reinterpret_cast<const float4*>(As + (wm * WTM + a * 16 + lr) * LS + 4 * lg);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = *reinterpret_cast<const float4*>(Bs + (wn * WTN + b * 16 + lr) * LS + 4 * lg);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf[b][s], af[a][s], acc[a][b], 0, 0, 0);
      P16_SSTORE(cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
    // epilogue of tile t (same as gemm_nt16_kernel)
    const int64_t mw = m0 + wm * WTM;
    const int nw = n0 + wn * WTN;
#pragma unroll
    for (int bp = 0; bp < TN / 2; ++bp) {
      const int g = (nw + 32 * bp) >> 5;
      float4 bv[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bv[h] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) bv[h] = *reinterpret_cast<const float4*>(bias + nw + 32 * bp + 16 * h + 4 * lg);
      }
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const int64_t m = mw + a * 16 + lr;
        uint32_t word = 0;
        if (EPI == EPI_MASK) word = mbits[m * ldmb + g];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const nerf_f32x4 v0 = acc[a][2 * bp + h];
          float v[4] = {v0[0], v0[1], v0[2], v0[3]};
          const float bb[4] = {bv[h].x, bv[h].y, bv[h].z, bv[h].w};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int bit = 16 * h + 4 * lg + r;
            if (EPI == EPI_BIAS) v[r] += bb[r];
            if (EPI == EPI_BIAS_RELU) {
              v[r] = fmaxf(v[r] + bb[r], 0.f);
              word |= (v[r] > 0.f ? 1u : 0u) << bit;
            }
            if (EPI == EPI_MASK) v[r] = ((word >> bit) & 1u) ? v[r] : 0.f;
          }
          *reinterpret_cast<float4*>(C + m * ldc + nw + 32 * bp + 16 * h + 4 * lg) = make_float4(v[0], v[1], v[2], v[3]);
        }
        if (EPI == EPI_BIAS_RELU && mbits_out) {
          word |= __shfl_xor(word, 16, 64);
          word |= __shfl_xor(word, 32, 64);
          if (lg == 0) mbits_out[m * ldmb + g] = word;
        }
      }
    }
    if (!more) break;
    t = tn;
    m0 = m0n;
    n0 = n0n;
    Ab = An;
    Bb = Bn;
  }
#undef P16_GLOAD
#undef P16_SSTORE
}
