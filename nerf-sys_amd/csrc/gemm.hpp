// fp32-input MFMA GEMMs for the NeRF MLP (gfx950 `v_mfma_f32_32x32x2_f32`, exact fp32 fmaf chains).
//
// Three shapes cover the whole MLP forward/backward (weights PyTorch (out,in) row-major):
//   gemm_nt     C[m][n] = epi( sum_k A[m][k] * B[n][k] )      forward  (B = W)      and
//                                                             dgrad    (B = W^T, copied once per step)
//   gemm_wgrad  P[s][n][k] = sum_{m in split s} G[m][n] * X[m][k]   (+ column sums of G -> bias grad)
//   reduce      dW = sum_s P[s]                                deterministic split-M reduction
//
// Tiling (one 256-thread workgroup = 4 waves, fp32 MFMA runs at the fp32 vector rate, 64 FLOP/clk/SIMD):
//   * BK = 16 k-slab, double-buffered in LDS, register-staged float4 global loads issued before the
//     MFMA block of the current slab and written to the other LDS buffer after it (one barrier / slab).
//   * lane l of a 32x32x2 MFMA supplies A[i=l&31][k-slot h=l>>5]; the slab's 16 k are split as
//     k = 8h + s for MFMA s = 0..7, so each lane reads its 8 k-values as two ds_read_b128 from a row of
//     the [rows][20]-float LDS tile (80-B row pitch: 16 consecutive rows hit 16 distinct 16-B bank slots).
//   * XCD-aware bijective blockIdx remap so that the column tiles of one row panel share an XCD L2.
#pragma once
#include "common.hpp"

typedef float nerf_f32x16 __attribute__((ext_vector_type(16)));

enum NerfEpi { EPI_BIAS = 0, EPI_BIAS_RELU = 1, EPI_MASK = 2, EPI_NONE = 3 };

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = bid & 7, loc = bid >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

template <int TM, int TN, int WTM, int WTN, int EPI>
__device__ __forceinline__ void nt_epilogue(const nerf_f32x16 (&acc)[TM][TN], int64_t mw, int nw, int li, int lh,
                                            const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                            const uint32_t* __restrict__ mbits, int ldmb,
                                            uint32_t* __restrict__ mbits_out);

// ------------------------------------------------------------------------------------------ gemm_nt
// Requirements (checked by the host wrapper): M % BM == 0, N % BN == 0, K % 16 == 0, lda/ldb/ldc/ldm % 4
// == 0, 16-byte aligned A/B.
//
// Measured alternatives (tools/gemm_bench2.hip, tools/gemm_variants/, MI355X, C2 trunk shape; this kernel
// runs at 79 % of the fp32 MFMA peak at its in-kernel clock of 2.3 GHz, tools/clock_probe.hip): an
// LDS-DMA (global_load_lds) ring with counted vmcnt, a weights-stationary persistent kernel with
// activations streamed to registers, prefetch loads pinned above the MFMA block (inline asm), BK = 32,
// a 128x256 tile and 2..3 waves/SIMD were all 2-13 % slower; so were (C2 step, 27.5 ms base) s_setprio 1 over
// the MFMA block (28.5 ms) and iglp_opt(0) / iglp_opt(1) in the k-loop (30.4 / 30.2 ms).
template <int BM, int BN, int WAVES_M, int EPI, int BK = 16, int NBUF = 2>
__device__ __forceinline__ void gemm_nt_body(const float* __restrict__ A, int lda, const float* __restrict__ B, int ldb,
                                             const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                             const uint32_t* __restrict__ mbits, int ldmb,
                                             uint32_t* __restrict__ mbits_out, int K, int n_ntiles) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wave tile");
  static_assert(BK == 16 || BK == 32, "k-slab");
  constexpr int LS = BK + 4;         // LDS row pitch (floats): 80 / 144 B, 16 rows -> 16 distinct bank slots
  constexpr int C4 = BK / 4;         // float4 per row per slab
  constexpr int HK = BK / 2;         // k per lane half per slab
  constexpr int A_F4 = BM * C4, B_F4 = BN * C4;
  constexpr int A_PER = (A_F4 + 255) / 256, B_PER = (B_F4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[NBUF * (BM + BN) * LS];

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
#define NT_GLOAD(k0_)                                                                          \
  _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    if (A_F4 % 256 == 0 || f < A_F4)                                                           \
      ra[i] = *reinterpret_cast<const float4*>(Ab + (int64_t)(f / C4) * lda + (k0_) + (f % C4) * 4); \
  }                                                                                            \
  _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    if (B_F4 % 256 == 0 || f < B_F4)                                                           \
      rb[i] = *reinterpret_cast<const float4*>(Bb + (int64_t)(f / C4) * ldb + (k0_) + (f % C4) * 4); \
  }
#define NT_SSTORE(buf_)                                                                        \
  {                                                                                            \
    float* As_ = smem + (buf_) * (BM + BN) * LS;                                               \
    float* Bs_ = As_ + BM * LS;                                                                \
    _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (A_F4 % 256 == 0 || f < A_F4)                                                         \
        *reinterpret_cast<float4*>(As_ + (f / C4) * LS + (f % C4) * 4) = ra[i];                \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (B_F4 % 256 == 0 || f < B_F4)                                                         \
        *reinterpret_cast<float4*>(Bs_ + (f / C4) * LS + (f % C4) * 4) = rb[i];                \
    }                                                                                          \
  }

  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = K / BK;
  NT_GLOAD(0);
  NT_SSTORE(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = NBUF == 2 ? (kt & 1) : 0;
    NT_GLOAD((kt + 1 < nk ? kt + 1 : kt) * BK);
    const float* As = smem + cur * (BM + BN) * LS;
    const float* Bs = As + BM * LS;
    // lane half h owns k = h*HK + s of the slab; its k-values of a row are read 4 at a time
#pragma unroll
    for (int hh = 0; hh < HK / 4; ++hh) {
      float4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[a] = *reinterpret_cast<const float4*>(As + (wm * WTM + a * 32 + li) * LS + HK * lh + 4 * hh);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[b] = *reinterpret_cast<const float4*>(Bs + (wn * WTN + b * 32 + li) * LS + HK * lh + 4 * hh);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)  // swapped operands: the tile is C^T (i = n, j = m)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(bf[b][s], af[a][s], acc[a][b], 0, 0, 0);
    }
    if (NBUF == 1) __syncthreads();  // single buffer: every wave done reading before the overwrite
    NT_SSTORE(NBUF == 2 ? (cur ^ 1) : 0);
    __syncthreads();
  }
#undef NT_GLOAD
#undef NT_SSTORE
  nt_epilogue<TM, TN, WTM, WTN, EPI>(acc, m0 + wm * WTM, n0 + wn * WTN, li, lh, bias, C, ldc, mbits, ldmb, mbits_out);
}

template <int BM, int BN, int WAVES_M, int EPI, int MINW = 1, int BK = 16, int NBUF = 2>
__global__ __launch_bounds__(256, MINW) void gemm_nt_kernel(const float* __restrict__ A, int lda,
                                                      const float* __restrict__ B, int ldb,
                                                      const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                                      const uint32_t* __restrict__ mbits, int ldmb,
                                                      uint32_t* __restrict__ mbits_out, int K, int n_ntiles) {
  gemm_nt_body<BM, BN, WAVES_M, EPI, BK, NBUF>(A, lda, B, ldb, bias, C, ldc, mbits, ldmb, mbits_out, K, n_ntiles);
}

// epilogue.  The MFMA computed C^T, so lane li holds ONE output row m = ... + li and register
// r = 4q + e holds column 8q + 4 lh + e of the 32-column tile: four float4 runs per row -> 16-B stores.
// ReLU masks travel as bits: the forward writes word g = column/32 of row m (the lane's 16 bits OR'd
// with its partner lane's li+32), the input-gradient GEMM reads one word per row instead of 32 floats.
template <int TM, int TN, int WTM, int WTN, int EPI>
__device__ __forceinline__ void nt_epilogue(const nerf_f32x16 (&acc)[TM][TN], int64_t mw, int nw, int li, int lh,
                                            const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                            const uint32_t* __restrict__ mbits, int ldmb,
                                            uint32_t* __restrict__ mbits_out) {
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int nb = nw + b * 32;
    const int g = nb >> 5;
    float4 bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) bv[q] = *reinterpret_cast<const float4*>(bias + nb + 8 * q + 4 * lh);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int64_t m = mw + a * 32 + li;
      uint32_t word = 0;
      if (EPI == EPI_MASK) word = mbits[m * ldmb + g];
      float* crow = C + m * ldc + nb + 4 * lh;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[a][b][4 * q + e];
          const float bb = e == 0 ? bv[q].x : (e == 1 ? bv[q].y : (e == 2 ? bv[q].z : bv[q].w));
          if (EPI == EPI_BIAS) v[e] += bb;
          if (EPI == EPI_BIAS_RELU) {
            v[e] = fmaxf(v[e] + bb, 0.f);
            word |= (v[e] > 0.f ? 1u : 0u) << (8 * q + 4 * lh + e);
          }
          if (EPI == EPI_MASK) v[e] = ((word >> (8 * q + 4 * lh + e)) & 1u) ? v[e] : 0.f;
        }
        *reinterpret_cast<float4*>(crow + 8 * q) = make_float4(v[0], v[1], v[2], v[3]);
      }
      if (EPI == EPI_BIAS_RELU && mbits_out) {
        word |= __shfl_xor(word, 32, 64);
        if (lh == 0) mbits_out[m * ldmb + g] = word;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ gemm_wgrad
// P[s][n][k] (row pitch ldp) = sum over rows m of split s of G[m][n] * X[m][k]; the tile of column
// block 0 also writes Pb[s][n] = sum_m G[m][n] (bias gradient).  MFMA A = G^T (i = n, k-slot = m),
// B = X (k-slot = m, j = k).  LDS tiles [16 rows][cols] read with ds_read_b32 (32 consecutive floats per
// half-wave: conflict-free).
// MR = rows per LDS slab (16, 32 or 64; rows_per_split % MR == 0).  The narrow tiles (one or two tiles
// per split: 256 or 512 workgroups) are latency-bound at MR = 16 (too few bytes in flight per CU), so they
// stage 32 / 64 rows; each slab is consumed as MR/16 sub-slabs of 16 rows in the MR = 16 row order, so the
// per-element accumulation order, and hence every bit of P, does not depend on MR.
template <int BN, int BK, int WAVES_N, int MR = 16>
__global__ __launch_bounds__(256) void gemm_wgrad_kernel(const float* __restrict__ G, int ldg,
                                                         const float* __restrict__ X, int ldx,
                                                         float* __restrict__ P, int ldp, float* __restrict__ Pb,
                                                         int64_t slab, int64_t rows_per_split, int64_t M,
                                                         int n_ktiles, int n_tiles) {
  constexpr int WAVES_K = 4 / WAVES_N;
  constexpr int WTN = BN / WAVES_N, WTK = BK / WAVES_K;
  constexpr int TM = WTN / 32, TN = WTK / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  static_assert(MR == 16 || MR == 32 || MR == 64, "rows per slab");
  constexpr int G_F4 = MR * BN / 4, X_F4 = MR * BK / 4;
  constexpr int G_PER = (G_F4 + 255) / 256, X_PER = (X_F4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * MR * (BN + BK)];

  // 1-D grid of (split, tile) pairs, tile fastest, remapped so that the output tiles of one split are
  // consecutive on ONE XCD: they stream the same G / X rows, which then come from that XCD's L2 once.
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
#define WG_GLOAD(m_)                                                                           \
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
#define WG_SSTORE(buf_)                                                                        \
  {                                                                                            \
    float* Gs_ = smem + (buf_) * MR * (BN + BK);                                               \
    float* Xs_ = Gs_ + MR * BN;                                                                \
    _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (G_F4 % 256 == 0 || f < G_F4) *reinterpret_cast<float4*>(Gs_ + f * 4) = rg[i];        \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (X_F4 % 256 == 0 || f < X_F4) *reinterpret_cast<float4*>(Xs_ + f * 4) = rx[i];        \
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
    WG_GLOAD(r0);
    WG_SSTORE(0);
  }
  __syncthreads();
  for (int64_t it = 0; it < nit; ++it) {
    const int cur = (int)(it & 1);
    WG_GLOAD(r0 + (it + 1 < nit ? it + 1 : it) * MR);
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
    WG_SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef WG_GLOAD
#undef WG_SSTORE

  float* Ps = P + (int64_t)s * slab;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int k = k0 + wk * WTK + b * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = n0 + wn * WTN + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        Ps[(int64_t)n * ldp + k] = acc[a][b][r];
      }
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

// ------------------------------------------------------------------------------------------ 16x16x4 forms
// The same GEMMs on v_mfma_f32_16x16x4_f32 (equal FLOP per cycle, exact fp32 fmaf chains like the 32x32x2 form).
// MI355X_MICROARCH.md "DVFS give-back" (7): under load the 16x16 shape holds a higher clock than the 32x32 one;
// measured at the C2 fine-net trunk shape in tools/gemm_bench16.hip (interleaved with the 32x32x2 kernels above).
// gemm_nt16_kernel: 128x128 block tile, BK-deep LDS slabs (80-B / 144-B row pitch), register staging and XCD remap
// as gemm_nt_body; each wave owns 64x64 as 4x4 16x16 blocks.  Lane l supplies row (l & 15) and k-slot g = l >> 4;
// a 16-k half-slab is split k = 4g + s for MFMA s = 0..3, so one ds_read_b128 per row fragment feeds four MFMAs.
// Operands swapped (the tile is C^T): lane l holds output row m = .. + (l & 15), columns n = .. + 4g + r (r = 0..3)
// -> one float4 store per 16x16 block; ReLU bitmask words OR'd over the four k-slot groups.
typedef float nerf_f32x4 __attribute__((ext_vector_type(4)));

template <int BM, int BN, int WAVES_M, int EPI, int MINW = 4, int BK = 16>
__global__ __launch_bounds__(256, MINW) void gemm_nt16_kernel(const float* __restrict__ A, int lda,
                                                             const float* __restrict__ B, int ldb,
                                                             const float* __restrict__ bias, float* __restrict__ C,
                                                             int ldc, const uint32_t* __restrict__ mbits, int ldmb,
                                                             uint32_t* __restrict__ mbits_out, int K, int n_ntiles) {
  constexpr int LS = BK + 4, C4 = BK / 4;
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  static_assert(TN % 2 == 0, "mask words span two 16-column blocks");
  constexpr int A_F4 = BM * C4, B_F4 = BN * C4;
  constexpr int A_PER = (A_F4 + 255) / 256, B_PER = (B_F4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LS];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int lr = lane & 15, lg = lane >> 4;
  const float* Ab = A + m0 * lda;
  const float* Bb = B + (int64_t)n0 * ldb;

  float4 ra[A_PER], rb[B_PER];
#define N16_GLOAD(k0_)                                                                         \
  _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    if (A_F4 % 256 == 0 || f < A_F4)                                                           \
      ra[i] = *reinterpret_cast<const float4*>(Ab + (int64_t)(f / C4) * lda + (k0_) + (f % C4) * 4); \
  }                                                                                            \
  _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    if (B_F4 % 256 == 0 || f < B_F4)                                                           \
      rb[i] = *reinterpret_cast<const float4*>(Bb + (int64_t)(f / C4) * ldb + (k0_) + (f % C4) * 4); \
  }
#define N16_SSTORE(buf_)                                                                       \
  {                                                                                            \
    float* As_ = smem + (buf_) * (BM + BN) * LS;                                               \
    float* Bs_ = As_ + BM * LS;                                                                \
    _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (A_F4 % 256 == 0 || f < A_F4)                                                         \
        *reinterpret_cast<float4*>(As_ + (f / C4) * LS + (f % C4) * 4) = ra[i];                \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (B_F4 % 256 == 0 || f < B_F4)                                                         \
        *reinterpret_cast<float4*>(Bs_ + (f / C4) * LS + (f % C4) * 4) = rb[i];                \
    }                                                                                          \
  }

  nerf_f32x4 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) acc[a][b] = nerf_f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = K / BK;
  N16_GLOAD(0);
  N16_SSTORE(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    N16_GLOAD((kt + 1 < nk ? kt + 1 : kt) * BK);
    const float* As = smem + cur * (BM + BN) * LS;
    const float* Bs = As + BM * LS;
#pragma unroll
    for (int hh = 0; hh < BK / 16; ++hh) {  // k = 16 hh + 4 g + s
      float4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a] = *reinterpret_cast<const float4*>(As + (wm * WTM + a * 16 + lr) * LS + 16 * hh + 4 * lg);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b] = *reinterpret_cast<const float4*>(Bs + (wn * WTN + b * 16 + lr) * LS + 16 * hh + 4 * lg);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(bf[b][s], af[a][s], acc[a][b], 0, 0, 0);
    }
    N16_SSTORE(cur ^ 1);
    __syncthreads();
  }

#undef N16_GLOAD
#undef N16_SSTORE
  // epilogue: lane holds row m = mw + 16a + lr, columns nb + 4lg + r of 16-column block b
  const int64_t mw = m0 + wm * WTM;
  const int nw = n0 + wn * WTN;
#pragma unroll
  for (int bp = 0; bp < TN / 2; ++bp) {
    const int g = (nw + 32 * bp) >> 5;  // mask word of columns [32 g, 32 g + 32)
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
}

// Split-M reduce (round 4): a float4 element's S slab terms in RG consecutive groups of slabs, one wave per group (64
// elements per 256-thread block), each group summed in slab order from 0, then the group sums added in group order onto
// the initial value by wave 0.  A fixed order — bitwise reproducible, and the same in every reduce kernel (the layered
// and the fused bf16 backward stay bitwise equal) — with RG times the loads in flight of one thread walking all S
// slabs: that walk is latency-bound (the 131-MB bf16 reduce ran at ~1 TB/s, 130 us per call).
constexpr int RG = 4;
__device__ __forceinline__ float4 rg_group_sum(const float* __restrict__ base, int64_t stride, int S, int g) {
  const int s0 = (int)((int64_t)S * g / RG), s1 = (int)((int64_t)S * (g + 1) / RG);
  const float4* p = reinterpret_cast<const float4*>(base);
  const int64_t st = stride / 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 16
  for (int s = s0; s < s1; ++s) {  // loads batched by the unroll, adds kept in split order
    const float4 v = p[s * st];
    a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
  }
  return a;
}
__device__ __forceinline__ void rg_add(float4& a, const float4& v) {
  a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
}

// dst[i] = (acc ? dst[i] : 0) + sum_{s<S} src[s*slab + i]   (float4 lanes, the RG-group order above); grid cdiv(n4, 64)
static __global__ __launch_bounds__(256) void reduce_splits_kernel(const float* __restrict__ src, int64_t slab, int S,
                                                                   float* __restrict__ dst, int64_t n4,
                                                                   int accumulate) {
  __shared__ float4 part[RG][64];
  const int e = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + e;
  part[g][e] = i < n4 ? rg_group_sum(src + 4 * i, slab, S, g) : make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  if (g == 0 && i < n4) {
    float4 a = accumulate ? reinterpret_cast<const float4*>(dst)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int k = 0; k < RG; ++k) rg_add(a, part[k][e]);
    reinterpret_cast<float4*>(dst)[i] = a;
  }
}
