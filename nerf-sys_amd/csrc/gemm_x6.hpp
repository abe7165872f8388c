// fp32 trunk GEMMs on the bf16 matrix cores: every fp32 operand is split into three bf16 pieces x = hi + mid + lo
// (round-to-nearest at each step; 3 x 8 significant bits cover fp32's 24, so the split is exact for normal numbers)
// and A.B^T is accumulated in fp32 from the six piece products whose magnitude is >= 2^-16 of the leading one:
//   lo.hi + mid.mid + hi.lo + mid.hi + hi.mid + hi.hi     (smallest first, one fp32 accumulator per output)
// The three dropped products (mid.lo, lo.mid, lo.lo) are <= 2^-24 relative — fp32 rounding size.  Measured on
// MI355X (tools/split_probe.hip, K = 256, forward- and backward-like data, error / sum_k |a_k b_k| against fp64):
// max 5.71 / mean 0.347 x 2^-24 for this scheme against 5.78 / 0.307 for the 16x16x4 fp32 MFMA and for a sequential
// fp32 fmaf chain (the two are bitwise equal) — the same accuracy as the fp32 path, at six `v_mfma_f32_32x32x16_bf16`
// (16 cycles per 16K MACs each) instead of sixteen `v_mfma_f32_16x16x4_f32` (8 cycles per 1K MACs each): 2.7x the
// MAC rate of the fp32 matrix cores, which moves the 256x256 trunk layers from MFMA-bound to HBM-bound.
//
//   gemm_nt_x6     C[m][n] = epi( sum_k A[m][k] B[n][k] ): A fp32 activations (split while staged into LDS), B the
//                  layer weights (forward) or their transpose (input gradient) as three pre-split bf16 planes
//   gemm_wgrad_x6  P[s][n][k] = sum_{m in split s} G[m][n] X[m][k] (+ bias column sums): both operands fp32
//                  activations, split while staged; fp32 slabs, deterministic reduce as in gemm.hpp
// Fragment / LDS conventions are gemm_bf16.hpp's (NT: [rows][BK] tiles, ds_read_b128 per fragment, C^T so a lane
// owns one output row; wgrad: row-major [m][cols] tiles read with ds_read_b64_tr_b16), one image per piece plane.
#pragma once
#include "gemm_bf16.hpp"

// two fp32 -> one packed bf16 pair in ONE v_cvt_pk_bf16_f32 (round to nearest even); the scalar-cast form
// (nerf_pack_bf16x2) compiles to two converts plus a repack
typedef float x6_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 x6_bf16x2 __attribute__((ext_vector_type(2)));
typedef float x6_f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint32_t x6_pack(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(x6_f32x2{a, b}, x6_bf16x2));
}

// four fp32 values -> their hi / mid / lo bf16 pieces, packed in pairs (v_cvt_pk_bf16_f32 rounds to nearest even).
// DOT2: each residual x - piece by one v_dot2c_f32_bf16 against (-1, 0) / (0, -1) instead of widening the piece
// (shift / mask) and a packed subtract: 7 VALU instructions per pair instead of 9, exact (the difference is an fp32
// number), so the pieces are bitwise the same.  Measured (C2, profiles/r05/x6_variants_ab.txt): on every split kernel
// forward 0.574 -> 0.566 ms, input gradient unchanged, weight gradient 0.479 -> 0.515 ms (its split sits in the staging
// path, where the dot's longer latency shows); on the forward alone within the noise (C2 224.0-224.9k either way).
// Off by default (NERF_X6_DOT2_FWD=1: the forward on the dot form).
#ifndef NERF_X6_DOT2_FWD
#define NERF_X6_DOT2_FWD 0
#endif
template <bool DOT2 = false>
__device__ __forceinline__ void x6_split4(const float4 v, uint2& h, uint2& m, uint2& l) {
#ifdef NERF_X6_NOSPLIT  // ablation builds only: split cost probe (wrong results)
  h = m = l = make_uint2(__float_as_uint(v.x), __float_as_uint(v.y));
  return;
#endif
#ifdef NERF_X6_CHEAPSPLIT  // ablation builds only: the hi pieces as all three (realistic operand values, 1/5 of the
  // split's VALU; wrong results) — does the split's VALU hold the kernels?
  h = m = l = make_uint2(x6_pack(v.x, v.y), x6_pack(v.z, v.w));
  return;
#endif
#ifdef NERF_X6_DOT2SPLIT  // A/B builds: every split kernel on the dot form
  if constexpr (true) {
#else
  if constexpr (DOT2) {
#endif
    typedef __bf16 b2_ __attribute__((ext_vector_type(2)));
    // the (-1, 0) / (0, -1) pairs as SGPR values: as a VOP2 inline constant "-1.0" the hardware does not read (-1, 0)
    uint32_t c0_, c1_;
    asm("s_mov_b32 %0, 0xbf80" : "=s"(c0_));  // (not volatile: hoisted out of the loops)
    asm("s_mov_b32 %0, 0xbf800000" : "=s"(c1_));
    const b2_ e0 = __builtin_bit_cast(b2_, c0_), e1 = __builtin_bit_cast(b2_, c1_);
    auto res = [&](uint32_t p, float x0, float x1, float& y0, float& y1) __attribute__((always_inline)) {
      const b2_ q = __builtin_bit_cast(b2_, p);
      y0 = __builtin_amdgcn_fdot2_f32_bf16(q, e0, x0, false);
      y1 = __builtin_amdgcn_fdot2_f32_bf16(q, e1, x1, false);
    };
    const uint32_t h0 = x6_pack(v.x, v.y), h1 = x6_pack(v.z, v.w);
    float r0, r1, r2, r3, s0, s1, s2, s3;
    res(h0, v.x, v.y, r0, r1);
    res(h1, v.z, v.w, r2, r3);
    const uint32_t m0 = x6_pack(r0, r1), m1 = x6_pack(r2, r3);
    res(m0, r0, r1, s0, s1);
    res(m1, r2, r3, s2, s3);
    h = make_uint2(h0, h1);
    m = make_uint2(m0, m1);
    l = make_uint2(x6_pack(s0, s1), x6_pack(s2, s3));
    return;
  }
  const uint32_t h0 = x6_pack(v.x, v.y), h1 = x6_pack(v.z, v.w);
  const float r0 = v.x - nerf_bf16_lo(h0), r1 = v.y - nerf_bf16_hi(h0);
  const float r2 = v.z - nerf_bf16_lo(h1), r3 = v.w - nerf_bf16_hi(h1);
  const uint32_t m0 = x6_pack(r0, r1), m1 = x6_pack(r2, r3);
  const uint32_t l0 = x6_pack(r0 - nerf_bf16_lo(m0), r1 - nerf_bf16_hi(m0));
  const uint32_t l1 = x6_pack(r2 - nerf_bf16_lo(m1), r3 - nerf_bf16_hi(m1));
  h = make_uint2(h0, h1);
  m = make_uint2(m0, m1);
  l = make_uint2(l0, l1);
}

// the six piece products, smallest first: term t multiplies A piece X6_PA[t] by B piece X6_PB[t] (0 = hi, 1 = mid,
// 2 = lo).  One term is issued for every accumulator of the wave before the next term, so consecutive MFMAs never
// chain on one accumulator (a dependent 32x32x16 MFMA waits for its predecessor's result).
__device__ constexpr int X6_PA[6] = {2, 1, 0, 1, 0, 0};
__device__ constexpr int X6_PB[6] = {0, 1, 2, 0, 1, 0};
// the forward kernels' order: the same as X6_PA / X6_PB (lo.hi first).  A hi.lo-first order measured 0.635 -> 0.629 ms
// per fine layer in round 3; with the LDS epilogue (round 4) its training run is slower (227.9k vs 229.3k rays/s) and
// its 3000-step PSNR (25.93 dB, sd 0.30 over 3 jitter seeds, 8 views) sits inside the default's band (26.12 dB, sd
// 0.16): decided by speed, lo.hi first is kept (profiles/r04/psnr_band.txt)
#ifdef NERF_X6_FWD_HIFIRST  // A/B builds: the hi.lo-first forward order (PSNR noise-band study, round 4)
__device__ constexpr int X6F_PA[6] = {0, 2, 1, 1, 0, 0};
__device__ constexpr int X6F_PB[6] = {2, 0, 1, 0, 1, 0};
#else
__device__ constexpr int X6F_PA[6] = {2, 1, 0, 1, 0, 0};
__device__ constexpr int X6F_PB[6] = {0, 1, 2, 0, 1, 0};
#endif
// acc_[TM_][TN_] += over the six terms; MFMA(first_, second_) operands: NT passes (B fragment, A fragment) so the
// accumulator is C^T (gemm_bf16.hpp); the weight gradient passes (G^T fragment, X fragment)
#ifndef NERF_X6_TERMS  // ablation builds only (tools/build_exp.sh): fewer terms -> wrong results, MFMA cost probe
#define NERF_X6_TERMS 6
#endif
#define X6_MFMA_BLOCK(acc_, TM_, TN_, FIRST_, SECOND_)                                                      \
  _Pragma("unroll") for (int t_ = 6 - NERF_X6_TERMS; t_ < 6; ++t_)                                        \
    _Pragma("unroll") for (int a_ = 0; a_ < TM_; ++a_)                                                    \
      _Pragma("unroll") for (int b_ = 0; b_ < TN_; ++b_)                                                  \
        acc_[a_][b_] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(FIRST_, SECOND_, acc_[a_][b_], 0, 0, 0);

// ------------------------------------------------------------------------------------------ weight planes
// dst plane p (p = hi, mid, lo) of job j: [rows_out][cols_out] bf16 at dst + p * plane, where for a plain job
// rows_out x cols_out = rows x cols of src (row pitch lds) and for a transposed job dst[c][r] = src[r][c]
struct X6Job {
  const float* src;
  nerf_bf16* dst;
  int rows, cols, lds, transpose;
  int64_t plane;
};
struct X6Jobs {
  X6Job j[16];
};
static __global__ void x6_planes_kernel(X6Jobs jobs) {
  const X6Job J = jobs.j[blockIdx.z];
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  if (r0 >= J.rows || c0 >= J.cols) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < J.rows && c < J.cols) ? J.src[(int64_t)r * J.lds + c] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    // plain: element (r0 + y, c0 + tx); transposed: element (r0 + tx, c0 + y) written to row c0 + y
    const float v = J.transpose ? tile[tx][y] : tile[y][tx];
    const int orow = J.transpose ? c0 + y : r0 + y, ocol = J.transpose ? r0 + tx : c0 + tx;
    const int orows = J.transpose ? J.cols : J.rows, ocols = J.transpose ? J.rows : J.cols;
    if (orow < orows && ocol < ocols) {
      const nerf_bf16 h = (nerf_bf16)v;
      const float r1 = v - (float)h;
      const nerf_bf16 m = (nerf_bf16)r1;
      const nerf_bf16 l = (nerf_bf16)(r1 - (float)m);
      const int64_t o = (int64_t)orow * ocols + ocol;
      J.dst[o] = h;
      J.dst[J.plane + o] = m;
      J.dst[2 * J.plane + o] = l;
    }
  }
}

// ------------------------------------------------------------------------------------------ gemm_nt_x6
// 128 x 128 output tile per 256-thread workgroup (four 64 x 64 wave tiles of 2 x 2 MFMA tiles), BK = 32 (two MFMA
// k-steps per slab).  The activation operand goes HBM -> registers in fragment layout (lane (r, h) of row block a:
// row r, k = 8 h .. 8 h + 7 of each 16-k step = two float4) and is split there, so only the pre-split weight planes
// pass through LDS: a first version that staged all six piece images through LDS ran at MFMA busy 0.31 with the LDS
// pipe as busy as the matrix cores (12 ds_read_b128 + 9 ds_write per 24 MFMAs, PMC 4e7 bank-conflict cycles per
// launch).  Weight planes: [3][128][40] bf16 per stage (80-B pitch: 16 consecutive rows hit 16 distinct 16-B bank
// slots), double-buffered, 60 KiB per workgroup -> two workgroups per CU.  The activation loads of slab k + 2 are
// issued as slab k's registers are consumed (two register sets); the weight slab k + 1 (L2-resident) is staged in
// registers during slab k and written to LDS after it (one barrier per slab).
// B: three planes of [N][ldb] bf16, plane stride bplane.  Requirements (host): M % 128 == 0, N % 128 == 0,
// K % 32 == 0, lda % 4 == 0, ldb % 8 == 0.
template <int EPI, int BK = 32, int MINW = 2>
__global__ __launch_bounds__(256, MINW) void gemm_nt_x6_kernel(const float* __restrict__ A, int lda,
                                                              const nerf_bf16* __restrict__ Bp, int ldb, int64_t bplane,
                                                              const float* __restrict__ bias, float* __restrict__ C,
                                                              int ldc, const uint32_t* __restrict__ mbits, int ldmb,
                                                              uint32_t* __restrict__ mbits_out, int K, int n_ntiles) {
  constexpr int BM = 128, BN = 128, WTM = 64, WTN = 64, TM = 2, TN = 2;
  constexpr int KS = BK / 16;   // MFMA k-steps per slab
  constexpr int CPR = BK / 8;   // 16-B weight chunks per row per slab
  static_assert(BK == 16 || BK == 32, "slab");
  constexpr int LS = BK + 8;    // 48 / 80-B pitch: 16 consecutive rows hit 16 distinct 16-B bank slots
  constexpr int PL = BN * LS;  // one weight piece image
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[2 * 3 * PL];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  const nerf_bf16* Bb = Bp + (int64_t)n0 * ldb;
  // this lane's activation rows (uniform tile base + 32-bit lane offsets)
  const float* At = A + (m0 + wm * WTM) * lda;
  int aoff[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) aoff[a] = (a * 32 + li) * lda + 8 * lh;

  // register sets: ra[set][a][ks] = the 8 fp32 of row block a, k-step ks (two float4)
  float4 ra[2][TM][KS][2];
  uint4 rb[3][KS];  // weight slab: 3 planes x 128 rows x CPR chunks of 16 B (thread: chunks t + 256 i)
#define X6_ALOAD(set_, k0_)                                                                                \
  _Pragma("unroll") for (int a = 0; a < TM; ++a)                                                          \
    _Pragma("unroll") for (int ks = 0; ks < KS; ++ks)                                                     \
      _Pragma("unroll") for (int hf = 0; hf < 2; ++hf)                                                    \
        ra[set_][a][ks][hf] = *reinterpret_cast<const float4*>(At + aoff[a] + (k0_) + 16 * ks + 4 * hf);
#define X6_BLOAD(k0_)                                                                                      \
  _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                           \
    _Pragma("unroll") for (int i = 0; i < KS; ++i) {                                                      \
      const int c = tid + 256 * i;                                                                        \
      rb[p][i] = *reinterpret_cast<const uint4*>(Bb + p * bplane + (int64_t)(c / CPR) * ldb + (k0_) + 8 * (c % CPR)); \
    }
#define X6_BSTORE(buf_)                                                                                    \
  _Pragma("unroll") for (int p = 0; p < 3; ++p)                                                           \
    _Pragma("unroll") for (int i = 0; i < KS; ++i) {                                                      \
      const int c = tid + 256 * i;                                                                        \
      *reinterpret_cast<uint4*>(smem + ((buf_) * 3 + p) * PL + (c / CPR) * LS + 8 * (c % CPR)) = rb[p][i]; \
    }

  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = K / BK;
  X6_ALOAD(0, 0);
  X6_ALOAD(1, (nk > 1 ? 1 : 0) * BK);
  X6_BLOAD(0);
  X6_BSTORE(0);
  __syncthreads();
  for (int kt0 = 0; kt0 < nk; kt0 += 2) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // slab kt = kt0 + j: LDS buffer j, activation register set j
      const int kt = kt0 + j;
      if (kt < nk) {
        X6_BLOAD((kt + 1 < nk ? kt + 1 : kt) * BK);
        const nerf_bf16* S = smem + j * 3 * PL;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          nerf_bf16x8 af[TM][3], bf[TN][3];
#pragma unroll
          for (int a = 0; a < TM; ++a) {
            uint2 h0, m0_, l0, h1, m1, l1;
            x6_split4(ra[j][a][ks][0], h0, m0_, l0);
            x6_split4(ra[j][a][ks][1], h1, m1, l1);
            af[a][0] = __builtin_bit_cast(nerf_bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
            af[a][1] = __builtin_bit_cast(nerf_bf16x8, make_uint4(m0_.x, m0_.y, m1.x, m1.y));
            af[a][2] = __builtin_bit_cast(nerf_bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
          }
#pragma unroll
          for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int b = 0; b < TN; ++b)
              bf[b][p] = *reinterpret_cast<const nerf_bf16x8*>(S + p * PL + (wn * WTN + b * 32 + li) * LS + 16 * ks +
                                                               8 * lh);
          X6_MFMA_BLOCK(acc, TM, TN, bf[b_][X6F_PB[t_]], af[a_][X6F_PA[t_]])  // the forward order (as gemm_nt_x6w)
        }
        // set j is consumed: slab kt + 2 streams into it while slab kt + 1 is computed
        X6_ALOAD(j, (kt + 2 < nk ? kt + 2 : nk - 1) * BK);
        X6_BSTORE(j ^ 1);
        __syncthreads();
      }
    }
  }
#undef X6_ALOAD
#undef X6_BLOAD
#undef X6_BSTORE

#ifdef NERF_X6_NOSTORE  // ablation builds only: the epilogue's cost (outputs left stale)
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b) asm volatile("" ::"v"(acc[a][b]));
#else
  ntb_epilogue<TM, TN, WTM, WTN, EPI, 0>(acc, m0 + wm * WTM, n0 + wn * WTN, li, lh, bias, C, ldc, mbits, ldmb,
                                         mbits_out);
#endif
}

// ------------------------------------------------------------------------------------------ LDS-staged epilogue
// The C^T accumulator leaves lane (li, lh) with row li, columns 8q + 4lh .. + 3 of each 32 x 32 block: the direct
// store (ntb_epilogue) writes 32 rows x 32 B per instruction, and with one workgroup per CU the 256 KiB of a tile's
// outputs leave at the store-issue rate while the matrix cores idle (cdna_hip_programming.md T21).  Here each block
// goes registers -> a private [32][36] fp32 LDS tile (144-B pitch) -> registers as 8 lanes per row, so every store
// instruction writes 8 whole 128-B lines.  Bias / ReLU / mask words are applied in registers first, exactly as
// ntb_epilogue does (same fp32 operations, bitwise the same outputs).
constexpr int X6E_PITCH = 36;
constexpr int X6E_WAVE_FLOATS = 32 * X6E_PITCH;
template <int TM, int TN, int EPI>
__device__ __forceinline__ void x6_epilogue_lds(nerf_f32x16 (&acc)[TM][TN], int64_t mw, int n0, int lane,
                                                const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                                const uint32_t* __restrict__ mbits, int ldmb,
                                                uint32_t* __restrict__ mbits_out, float* E) {
  const int li = lane & 31, lh = lane >> 5;
  const int rr = lane >> 3, cc = 4 * (lane & 7);  // read-back: row rr + 8 i, columns cc .. cc + 3
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int nb = n0 + b * 32;
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
        *reinterpret_cast<float4*>(E + li * X6E_PITCH + 8 * q + 4 * lh) = make_float4(v[0], v[1], v[2], v[3]);
      }
      if (EPI == EPI_BIAS_RELU && mbits_out) {
        word |= __shfl_xor(word, 32, 64);
        if (lh == 0) mbits_out[m * ldmb + g] = word;
      }
      // The read-back takes rows other lanes wrote.  What orders it: the wave's LDS operations execute in issue order,
      // and the write and read addresses (lane-dependent offsets into the same tile) may alias for the compiler, so it
      // can move neither the reads above these writes nor the next block's writes above these reads.  Explicit
      // barriers were built and measured (round 5, profiles/r05/x6_epi_fence_ab.txt): wavefront-scope release / acquire
      // fences cost 17 % of the launch (they wait for the block's global stores); "memory" asm clobbers and
      // sched_barriers here stop SROA from keeping o in registers (80 B of scratch per lane, or 32 KiB of LDS once
      // promoted).  Neither is kept.
      float4 o[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = *reinterpret_cast<const float4*>(E + (rr + 8 * i) * X6E_PITCH + cc);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<float4*>(C + (mw + a * 32 + rr + 8 * i) * ldc + nb + cc) = o[i];
    }
  }
}

#ifdef NERF_X6W_STAMPS  // diagnostic builds only (tools/x6_stamps.py): s_memtime per pipeline point, one workgroup
__device__ unsigned long long nerf_x6_stamps[2][8][128];
#define X6W_STAMP()                                                                                       \
  if (stamp_on) {                                                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();                                           \
    if (lane == 0 && si_ < 128) nerf_x6_stamps[BIGSMALL ? 1 : 0][wave][si_] = t_;                          \
    ++si_;                                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                                    \
  }
#else
#define X6W_STAMP()
#endif
// ------------------------------------------------------------------------------------------ gemm_nt_x6w
// Wide-wave form of gemm_nt_x6: a (64 NW) x 128 workgroup tile whose NW waves each own 64 rows x ALL 128 columns
// (2 x 4 MFMA tiles), so every activation row is loaded and split by exactly one wave (gemm_nt_x6's 64 x 64 waves
// split each row twice) and the split VALU work per MFMA halves.  Weight planes [3][128][BK + 8] bf16
// double-buffered in LDS; B fragments are read per pair of column blocks so that at most 24 VGPRs of them are live.
// Requirements as gemm_nt_x6 with M % (32 TM NW) == 0 and K % BK == 0.  Default BK = 32, NW = 8 (512 x 128 tiles, one
// workgroup per CU): C2 step 204.0k -> 207.5-209.0k rays/s over BK = 16, NW = 4 (fwd / dgrad 0.65 -> 0.63 ms).
// TM = 1 (32-row waves; the BIGSMALL input gradients, whose 256 accumulator registers per 64-row wave allowed only one
// wave per SIMD): 256 x 128 tiles at two waves per SIMD.
#ifndef NERF_X6W_PAIRB
#define NERF_X6W_PAIRB 0
#endif
#ifndef NERF_X6W_PAIRB3
#define NERF_X6W_PAIRB3 0
#endif
constexpr bool defined_regb() {
#ifdef NERF_X6W_REGB
  return true;
#else
  return false;
#endif
}
// TN_: 32-column blocks per wave (= the workgroup's columns / 32).  TN_ = 8 with TM = 1 (A/B builds,
// NERF_X6_FWD_TN8): 256 x 256 tiles of 32 x 256 waves, so each activation row is split by ONE workgroup instead of one
// per 128-column tile, at the same per-accumulator MFMA order (bitwise the same outputs).
template <int EPI, int BK = 32, int NW = 8, bool BIGSMALL = false, int TM = 2, int MINW = (BIGSMALL ? 1 : 8 / NW),
          int NKC = 0, int TN_ = 4>
__global__ __launch_bounds__(64 * NW, MINW) void gemm_nt_x6w_kernel(const float* __restrict__ A, int lda,
                                                                     const nerf_bf16* __restrict__ Bp, int ldb,
                                                                     int64_t bplane, const float* __restrict__ bias,
                                                                     float* __restrict__ C, int ldc,
                                                                     const uint32_t* __restrict__ mbits, int ldmb,
                                                                     uint32_t* __restrict__ mbits_out, int K,
                                                                     int n_ntiles) {
  constexpr int NT = 64 * NW;                     // threads
  constexpr int WTM = 32 * TM, BM = WTM * NW, TN = TN_, BN = 32 * TN_, WTN = BN;
  constexpr int KS = BK / 16, CPR = BK / 8;       // MFMA k-steps / 16-B weight chunks per row, per slab
  constexpr int BCH = 3 * BN * CPR / NT;          // weight chunks per thread per slab
#ifdef NERF_X6W_REGB  // register staging: whole 16-B chunks per thread (the GLDS DMA groups are checked below)
  static_assert((3 * BN * CPR) % NT == 0 && (BN * CPR) % NT == 0, "weight staging");
#endif
#if !defined(NERF_X6W_REGB) || defined(NERF_X6W_SWIZZLE)
  // weight images [BN][BK] bf16 unpadded, 16-B chunk q of row r in slot q ^ ((r >> 2) & 3) (BK = 32: four chunks per
  // 64-B row): the staging writes (4 rows x 4 chunks per 16-lane group) and the fragment reads (16 consecutive rows,
  // one chunk) both hit 16 distinct 16-B bank slots.  The 80-B padded pitch it replaces was 2-way conflicted on the
  // staging writes (PMC SQ_LDS_BANK_CONFLICT 8.5e6 cycles per fine forward launch, profiles/r04/pmc_split.txt).
  constexpr int LS = BK;
  static_assert(BK == 32, "the swizzle assumes four 16-B chunks per row");
  auto sw = [](int r, int q) { return q ^ ((r >> 2) & 3); };
#else  // A/B builds: the 80-B padded pitch
  constexpr int LS = BK + 8;
  auto sw = [](int r, int q) { return q; };
#endif
  constexpr int PL = BN * LS;
  // PB: one workgroup barrier per PAIR of slabs (four weight buffers: the next pair is DMA'd into the two the previous
  // pair read, released by that pair's barrier) instead of one per slab — the waves arrive at a slab barrier skewed
  // (s_memtime stamps, round 4: ~1.9k of a 9.55k-cycle forward slab), and a barrier every other slab pays that wait
  // once per two slabs.  The two-set, non-A3 loop only.
  constexpr bool PB = NERF_X6W_PAIRB && !(NKC > 0) && !defined_regb();
  // the same for the three-set (A3) input-gradient loop: pairs of the fully unrolled slab sequence
  constexpr bool PB3 = NERF_X6W_PAIRB3 && (NKC > 0) && !defined_regb();
  constexpr int NBUF = (PB || PB3) ? 4 : 2;
  // the epilogue tiles reuse the weight images (12-wave workgroups: a little more than the two buffers)
  constexpr int SMEM_E = (NBUF * 3 * PL > NW * X6E_WAVE_FLOATS * 2) ? NBUF * 3 * PL : NW * X6E_WAVE_FLOATS * 2;
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[SMEM_E];

#ifdef NERF_X6W_STAGGER  // probe builds: every other workgroup starts ~NERF_X6W_STAGGER x 64 clocks late
  if ((blockIdx.x >> 3) & 1) __builtin_amdgcn_s_sleep(NERF_X6W_STAGGER);
#endif
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const nerf_bf16* Bb = Bp + (int64_t)n0 * ldb;
  const float* At = A + (m0 + wave * WTM) * lda;
  int aoff[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) aoff[a] = (a * 32 + li) * lda + 8 * lh;

#ifndef NERF_X6W_REGB  // NERF_X6W_REGB (A/B builds): register-staged weight slabs
  constexpr bool GLDS = true;
#else
  constexpr bool GLDS = false;
#endif
  // NKC > 0 (K = NKC BK at compile time, TM = 1): three activation register sets, the slab loop fully unrolled — slab
  // kt + 2's loads are issued at the start of slab kt, after its weight DMA, so the end-of-slab weight wait leaves them
  // in flight (two slabs of latency instead of one)
  constexpr bool A3 = NKC > 0;
  static_assert(!A3 || TM == 1, "three activation sets: 32-row waves");
  float4 ra[A3 ? 3 : 2][TM][KS][2];
  const uint32_t bofs = (uint32_t)(((tid / CPR) * ldb + 8 * (tid % CPR)) * (int)sizeof(nerf_bf16));  // bytes
  uint4 rb[GLDS ? 1 : BCH];
  // GLDS: the weight slab DMA'd straight into the LDS image (global_load_lds_dwordx4, no VGPRs): one wave-instruction
  // fills 16 rows x 64 B of a piece image, lane l -> row l / 4, slot l % 4, so the swizzle goes on the source: lane l
  // reads chunk (l % 4) ^ ((row >> 2) & 3) = (l & 3) ^ ((l >> 4) & 3) of its row.  Issued as inline asm after the touch
  // of the slab's activation registers (hipcc neither counts these loads nor drains them at its own waits).  Against
  // register staging (profiles/r04/x6_glds_ab.txt, C2 on MI355X): fwd 0.595 -> 0.572-0.583 ms, dgrad 0.614 ->
  // 0.588-0.594 ms per fine launch, 218.5k -> 221k rays/s, the same loss bits; s_memtime stamps of the forward: slab
  // 11.4k -> 9.6k cycles, its "weight store + barrier" tail 3.5k -> 1.9k
  constexpr int GPP = BN * BK * 2 / 1024, GPW = 3 * GPP / NW;  // 1-KiB groups per piece image / per wave
  // GLDS: the NW waves' GPW groups each must cover the three piece images' 3 GPP 1-KiB groups exactly
  static_assert(!GLDS || (BK == 32 && GPW * NW == 3 * GPP && GPP * 1024 == BN * BK * 2), "GLDS staging");
  const int wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t gofs = (uint32_t)((((lane >> 2) * ldb) + 8 * ((lane & 3) ^ ((lane >> 4) & 3))) * 2);
  const uint32_t smem_u32 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;  // chunk c = tid + NT i: plane c / (BN CPR), row (c / CPR) % BN, chunk c % CPR
#define X6W_ALOAD(set_, k0_)                                                                              \
  _Pragma("unroll") for (int a = 0; a < TM; ++a)                                                         \
    _Pragma("unroll") for (int ks = 0; ks < KS; ++ks)                                                    \
      _Pragma("unroll") for (int hf = 0; hf < 2; ++hf)                                                   \
        ra[set_][a][ks][hf] = *reinterpret_cast<const float4*>(At + aoff[a] + (k0_) + 16 * ks + 4 * hf);
  // ASMB: the weight-slab loads as inline asm.  The compiler sinks plain loads to just before their LDS writes, which
  // exposes an L2 round trip per slab; in the BIGSMALL input-gradient kernel that cost 0.78 -> 0.72 ms per fine layer
  // (64-row waves, one per SIMD; measured on MI355X).  Issued after the wave's activation registers of the slab have landed
  // (the touch below), so the compiler's counted waits on its own activation loads never wait on these as well.  At two
  // waves per SIMD the extra live registers spill (fwd 0.62 -> 0.65 ms): plain loads there.  32-row waves (TM = 1) have
  // the registers: a forward of that shape went 0.76 -> 0.655 ms with them, still behind 0.63 ms for 64-row waves.
  constexpr bool ASMB = !GLDS && (BIGSMALL || TM == 1);
  constexpr bool ASML = ASMB || GLDS;  // weight loads hipcc does not count
  // B fragments are read per pair of column blocks (2 x 3 fragments live).  Measured and not kept (round 4,
  // profiles/r04/x6_bfrag_ab.txt): one block at a time (fwd 0.603 -> 0.612 ms), with the next block read under the
  // current block's MFMAs (0.613-0.619), and one block at a time with inline-asm weight loads (0.599-0.601).  Also not
  // kept: the two 4-wave halves staggered by one barrier (ping-pong: one half's 24-MFMA cluster under the other's split
  // and fragment reads, three DMA'd weight buffers, two barriers per cluster): fwd 0.58 -> 0.64, dgrad 0.59 -> 0.67 ms
  // (profiles/r04/x6_pingpong_ab.txt)
  constexpr int BPG = 2;
#define X6W_BLOAD(k0_, dbuf_)                                                                             \
  if constexpr (GLDS) {                                                                                   \
    _Pragma("unroll") for (int a = 0; a < TM; ++a)                                                       \
      _Pragma("unroll") for (int ks = 0; ks < KS; ++ks)                                                  \
        asm volatile("" ::"v"(__builtin_bit_cast(x6_f32x4, ra[j][a][ks][0])),                            \
                     "v"(__builtin_bit_cast(x6_f32x4, ra[j][a][ks][1])) : "memory");                     \
    _Pragma("unroll") for (int i = 0; i < GPW; ++i) {                                                    \
      const int g_ = wave_u + NW * i, p_ = g_ / GPP, rb_ = (g_ % GPP) * 16;                              \
      const nerf_bf16* sb_ = Bb + p_ * bplane + (int64_t)rb_ * ldb + (k0_);                              \
      const uint32_t dst_ = smem_u32 + (uint32_t)((((dbuf_) * 3 + p_) * PL + rb_ * LS) * 2);             \
      unsigned keep_;                                                                                     \
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t" \
                   "s_mov_b32 m0, %0" : "=&s"(keep_) : "v"(gofs), "s"(sb_), "s"(dst_) : "memory");       \
    }                                                                                                     \
  } else if constexpr (ASMB) {                                                                            \
    _Pragma("unroll") for (int a = 0; a < TM; ++a)                                                       \
      _Pragma("unroll") for (int ks = 0; ks < KS; ++ks)                                                  \
        asm volatile("" ::"v"(__builtin_bit_cast(x6_f32x4, ra[j][a][ks][0])),                            \
                     "v"(__builtin_bit_cast(x6_f32x4, ra[j][a][ks][1])) : "memory");                     \
    _Pragma("unroll") for (int i = 0; i < BCH; ++i) {                                                    \
      /* NT divides BN CPR: chunk c's plane and the row base of its NT-chunk group are uniform, so the     \
         address is a uniform SGPR base plus one 32-bit lane offset (bofs) instead of a VGPR pair a chunk */ \
      const int pu = (NT * i) / (BN * CPR), ru = ((NT * i) % (BN * CPR)) / CPR;                          \
      const nerf_bf16* sb_ = Bb + pu * bplane + (int64_t)ru * ldb + (k0_);                              \
      x6_f32x4 v_;                                                                                        \
      asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(v_) : "v"(bofs), "s"(sb_) : "memory");       \
      rb[i] = __builtin_bit_cast(uint4, v_);                                                              \
    }                                                                                                     \
  } else {                                                                                                \
    _Pragma("unroll") for (int i = 0; i < BCH; ++i) {                                                    \
      const int c = tid + NT * i, p = c / (BN * CPR), r = (c / CPR) % BN, q = c % CPR;                   \
      rb[i] = *reinterpret_cast<const uint4*>(Bb + p * bplane + (int64_t)r * ldb + (k0_) + 8 * q);       \
    }                                                                                                     \
  }
#define X6W_BWAIT()                                                                                       \
  if constexpr (GLDS) {                                                                                   \
    if constexpr (TM * KS * 2 == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                    \
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");                                                \
  } else if constexpr (ASMB) {                                                                            \
    static_assert(TM * KS * 2 == 8 || TM * KS * 2 == 4, "vmcnt: the activation loads after the weight loads"); \
    if constexpr (TM * KS * 2 == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");                    \
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");                                                \
    _Pragma("unroll") for (int i = 0; i < BCH; ++i) {                                                    \
      x6_f32x4 v_ = __builtin_bit_cast(x6_f32x4, rb[i]);                                                  \
      asm volatile("" : "+v"(v_));                                                                        \
      rb[i] = __builtin_bit_cast(uint4, v_);                                                              \
    }                                                                                                     \
  }
#define X6W_BSTORE(buf_)                                                                                  \
  if constexpr (!GLDS) _Pragma("unroll") for (int i = 0; i < BCH; ++i) {                                 \
    const int c = tid + NT * i, p = c / (BN * CPR), r = (c / CPR) % BN, q = c % CPR;                     \
    *reinterpret_cast<uint4*>(smem + ((buf_) * 3 + p) * PL + r * LS + 8 * sw(r, q)) = rb[i];             \
  }

  // BIGSMALL: the five small piece products accumulate in their own registers (2^-8 of the hi.hi sum, so the bf16
  // MFMA's one-guard-bit accumulator update loses 2^8 less there) and hi.hi gets 1 update per k-step instead of 6
  nerf_f32x16 acc[TM][TN], accs[BIGSMALL ? TM : 1][BIGSMALL ? TN : 1];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        acc[a][b][r] = 0.f;
        if constexpr (BIGSMALL) accs[a][b][r] = 0.f;
      }

  const int nk = A3 ? NKC : K / BK;
  X6W_ALOAD(0, 0);
  X6W_ALOAD(1, (nk > 1 ? 1 : 0) * BK);
  {
    const int j = 0;
    X6W_BLOAD(0, 0);
    if constexpr (PB || PB3) {  // host: K % (2 BK) == 0, so slab 1 exists
      X6W_BLOAD(BK, 1);
    }
    if constexpr (ASML) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  X6W_BSTORE(0);
  __syncthreads();
#ifdef NERF_X6W_STAMPS
  const bool stamp_on = blockIdx.x == 777 && (BIGSMALL || EPI == EPI_BIAS_RELU);
  int si_ = 0;
#endif
  // one slab's k-steps on activation register set rj and weight buffer S
  auto slab_mfma = [&](const float4 (&rj)[TM][KS][2], const nerf_bf16* S, auto&& after_split) __attribute__((always_inline)) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          nerf_bf16x8 af[TM][3];
#pragma unroll
          for (int a = 0; a < TM; ++a) {
            uint2 h0, m0_, l0, h1, m1, l1;
            x6_split4<NERF_X6_DOT2_FWD && !BIGSMALL>(rj[a][ks][0], h0, m0_, l0);
            x6_split4<NERF_X6_DOT2_FWD && !BIGSMALL>(rj[a][ks][1], h1, m1, l1);
            af[a][0] = __builtin_bit_cast(nerf_bf16x8, make_uint4(h0.x, h0.y, h1.x, h1.y));
            af[a][1] = __builtin_bit_cast(nerf_bf16x8, make_uint4(m0_.x, m0_.y, m1.x, m1.y));
            af[a][2] = __builtin_bit_cast(nerf_bf16x8, make_uint4(l0.x, l0.y, l1.x, l1.y));
          }
          if (ks == KS - 1) after_split();  // the slab's activation registers are all split
          X6W_STAMP();
#pragma unroll
          for (int bp = 0; bp < TN / BPG; ++bp) {  // groups of BPG column blocks: BPG x 3 B fragments live
            nerf_bf16x8 bf[BPG][3];
#pragma unroll
            for (int p = 0; p < 3; ++p)
#pragma unroll
              for (int b = 0; b < BPG; ++b)
                bf[b][p] = *reinterpret_cast<const nerf_bf16x8*>(S + p * PL + ((BPG * bp + b) * 32 + li) * LS +
                                                                 8 * sw((BPG * bp + b) * 32 + li, 2 * ks + lh));
#pragma unroll
            for (int t = 0; t < 6; ++t)
#pragma unroll
              for (int a = 0; a < TM; ++a)
#pragma unroll
                for (int b = 0; b < BPG; ++b) {
                  if constexpr (BIGSMALL) {
                    if (t < 5)
                      accs[a][BPG * bp + b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                          bf[b][X6_PB[t]], af[a][X6_PA[t]], accs[a][BPG * bp + b], 0, 0, 0);
                    else
                      acc[a][BPG * bp + b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                          bf[b][X6_PB[t]], af[a][X6_PA[t]], acc[a][BPG * bp + b], 0, 0, 0);
                  } else {
                    acc[a][BPG * bp + b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        bf[b][X6F_PB[t]], af[a][X6F_PA[t]], acc[a][BPG * bp + b], 0, 0, 0);
                  }
                }
          }
          X6W_STAMP();
        }
  };
  X6W_STAMP();
  if constexpr (PB3) {
    static_assert(NKC % 2 == 0, "slab pairs");
    // pair (kt0, kt0 + 1) in buffers b0, b0 + 1: the next pair's DMAs and slab kt0 + 2's activations go out at the
    // pair's start (after the touch of set kt0 % 3), slab kt0 + 3's after slab kt0 (into the set it freed); one
    // barrier per pair, which the next pair's DMAs wait on (vmcnt(8): the 8 activation loads issued after them stay
    // in flight); the last pair loads nothing and drains
#pragma unroll
    for (int p = 0; p < NKC / 2; ++p) {
      const int kt0 = 2 * p, b0 = kt0 & 3;
      const bool more = kt0 + 2 < NKC;  // compile time (unrolled)
      {
        const int j = kt0 % 3;
        if (more) {
          X6W_BLOAD((kt0 + 2) * BK, b0 ^ 2);
          X6W_BLOAD((kt0 + 3) * BK, (b0 ^ 2) + 1);
        }
      }
      if (more) X6W_ALOAD((kt0 + 2) % 3, (kt0 + 2) * BK);
      asm volatile("" ::: "memory");
      slab_mfma(ra[kt0 % 3], smem + b0 * 3 * PL, [] {});
      if (more) X6W_ALOAD((kt0 + 3) % 3, (kt0 + 3) * BK);
      asm volatile("" ::: "memory");
      slab_mfma(ra[(kt0 + 1) % 3], smem + (b0 + 1) * 3 * PL, [] {});
      if (more) {
        if constexpr (TM * KS * 2 == 4) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      X6W_STAMP();
      __syncthreads();
      X6W_STAMP();
    }
  } else if constexpr (A3) {
#pragma unroll
    for (int kt = 0; kt < NKC; ++kt) {
      const int j = kt % 3;
      X6W_BLOAD((kt + 1 < NKC ? kt + 1 : kt) * BK, (kt + 1) & 1);
      // set (kt + 2) % 3 was consumed by slab kt - 1; the last two slabs load nothing (a dead load would be deleted by the
      // compiler and leave the counted weight wait short), so their weight wait drains the queue
      if (kt + 2 < NKC) X6W_ALOAD((kt + 2) % 3, (kt + 2) * BK);
      asm volatile("" ::: "memory");  // pinned here: hipcc otherwise sinks the loads to the end of the slab
      slab_mfma(ra[j], smem + (kt & 1) * 3 * PL, [] {});
      if (kt + 2 < NKC) {
        X6W_BWAIT();
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      X6W_STAMP();
      __syncthreads();
      X6W_STAMP();
    }
  } else if constexpr (PB) {
    for (int kt0 = 0; kt0 < nk; kt0 += 2) {
      const int b0 = kt0 & 3;  // this pair's buffers b0, b0 + 1; the next pair's b0 ^ 2, (b0 ^ 2) + 1
      {
        const int j = 0;  // (the DMA's touch: set 0 feeds this pair's first slab)
        // past the end the last pair is DMA'd again into buffers nobody reads (the drain below covers it)
        X6W_BLOAD((kt0 + 2 < nk ? kt0 + 2 : nk - 2) * BK, b0 ^ 2);
        X6W_BLOAD((kt0 + 3 < nk ? kt0 + 3 : nk - 1) * BK, (b0 ^ 2) + 1);
      }
      asm volatile("" ::: "memory");
      slab_mfma(ra[0], smem + b0 * 3 * PL, [&]() __attribute__((always_inline)) {
        X6W_ALOAD(0, (kt0 + 2 < nk ? kt0 + 2 : nk - 1) * BK);
        asm volatile("" ::: "memory");
      });
      slab_mfma(ra[1], smem + (b0 + 1) * 3 * PL, [&]() __attribute__((always_inline)) {
        X6W_ALOAD(1, (kt0 + 3 < nk ? kt0 + 3 : nk - 1) * BK);
        asm volatile("" ::: "memory");
      });
      // the next pair's two DMAs done; the two activation sets issued after them stay in flight
      if constexpr (TM * KS * 2 == 8) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      X6W_STAMP();
      __syncthreads();
      X6W_STAMP();
    }
  } else
  for (int kt0 = 0; kt0 < nk; kt0 += 2) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {  // slab kt = kt0 + j: LDS buffer j, activation register set j
      const int kt = kt0 + j;
      // ASMB: nk is even (host: K % (2 BK) == 0), so no guard — every path into the loop header then has the same
      // loads in flight and the compiler's counted wait there stays vmcnt(8) instead of draining to vmcnt(0)
      if (ASML || kt < nk) {
        X6W_BLOAD((kt + 1 < nk ? kt + 1 : kt) * BK, j ^ 1);
        const nerf_bf16* S = smem + j * 3 * PL;
#ifndef NERF_X6W_LATE_A  // set j's next loads issued right after its last split, pinned before the last k-step's MFMAs
        // (profiles/r04/x6_early_a_ab.txt: fwd 0.582 -> 0.578 ms, C2 +0.5 %; with register-staged weights the same move
        // was slower, x6_early_ab.txt).  NERF_X6W_LATE_A (A/B builds): after the slab's MFMAs
        slab_mfma(ra[j], S, [&] {
          X6W_ALOAD(j, (kt + 2 < nk ? kt + 2 : nk - 1) * BK);
          asm volatile("" ::: "memory");
        });
#else
        slab_mfma(ra[j], S, [] {});
        X6W_ALOAD(j, (kt + 2 < nk ? kt + 2 : nk - 1) * BK);  // set j consumed: slab kt + 2 streams into it
#endif
        X6W_BWAIT();
        X6W_STAMP();
        X6W_BSTORE(j ^ 1);
        __syncthreads();
        X6W_STAMP();
      }
    }
  }
#undef X6W_ALOAD
#undef X6W_BLOAD
#undef X6W_BWAIT
#undef X6W_BSTORE

  if constexpr (GLDS && !A3) {
    // the two-set loop's last slab re-issued slab nk - 1's weight DMA into buffer 0, which the epilogue tiles below
    // reuse; the loop's counted vmcnt covered it only while the (dead) activation loads after it were still issued.
    // Drain every wave's DMA and meet before any wave writes its epilogue tile, independent of what hipcc keeps.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if constexpr (BIGSMALL) {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) acc[a][b] += accs[a][b];
  }
#if defined(NERF_X6W_REGEPI)  // A/B builds: the direct row-per-lane stores (32 rows x 32 B per store instruction)
  ntb_epilogue<TM, TN, WTM, WTN, EPI, 0>(acc, m0 + wave * WTM, n0, li, lh, bias, C, ldc, mbits, ldmb, mbits_out);
#else
  // the loop's last barrier freed the weight images: every wave stages its 32 x 32 blocks through a private LDS
  // tile and stores whole 128-B row lines (8 lanes per row).  C2 bench on MI355X (profiles/r04/x6_epilogue_ab.txt):
  // fwd 0.625 -> 0.591 ms, dgrad 0.669 -> 0.610 ms per fine layer, 208.0k -> 217.0k rays/s, bitwise the same loss
  x6_epilogue_lds<TM, TN, EPI>(acc, m0 + wave * WTM, n0, lane, bias, C, ldc, mbits, ldmb, mbits_out,
                               reinterpret_cast<float*>(smem) + wave * X6E_WAVE_FLOATS);
#endif
  X6W_STAMP();
}

// ------------------------------------------------------------------------------------------ gemm_wgrad_x6
// gemm_wgrad_bf16_kernel's tiling with fp32 operands split while staged: 16-row slabs (one MFMA k-step), per stage
// three G piece images [16][PG] and three X images [16][PX] (pitch = 64 B mod 256 B for the transposing reads),
// double-buffered: 60 KiB for 128 x 128 tiles -> two workgroups per CU.  Bias column sums (tiles of k-block 0) add
// the three pieces of every G value, which sum to it exactly.  Requirements: rows_per_split % 16 == 0, M % 16 == 0,
// ldg / ldx % 4 == 0.
template <int BN, int BK, int WAVES_N>
__global__ __launch_bounds__(256, 2) void gemm_wgrad_x6_kernel(const float* __restrict__ G, int ldg,
                                                              const float* __restrict__ X, int ldx,
                                                              float* __restrict__ P, int ldp, float* __restrict__ Pb,
                                                              int64_t slab, int64_t rows_per_split, int64_t M,
                                                              int n_ktiles, int n_tiles) {
  constexpr int MR = 16;
  constexpr int WAVES_K = 4 / WAVES_N;
  constexpr int WTN = BN / WAVES_N, WTK = BK / WAVES_K;
  constexpr int TM = WTN / 32, TN = WTK / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  constexpr int PG = ((BN + 127) / 128) * 128 + 32, PX = ((BK + 127) / 128) * 128 + 32;
  constexpr int IG = MR * PG, IX = MR * PX;       // one piece image
  constexpr int STAGE = 3 * (IG + IX);
  constexpr int G_F4 = MR * BN / 4, X_F4 = MR * BK / 4;
  constexpr int G_PER = (G_F4 + 255) / 256, X_PER = (X_F4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[2 * STAGE];

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

  constexpr int PF = 4;  // register sets in flight, as in gemm_nt_x6_kernel
  float4 rg[PF][G_PER], rx[PF][X_PER];
#define WX6_GLOAD(set_, m_)                                                                                \
  {                                                                                                        \
    _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                                    \
      const int f = tid + 256 * i;                                                                         \
      if (G_F4 % 256 == 0 || f < G_F4)                                                                     \
        rg[set_][i] = *reinterpret_cast<const float4*>(G + ((m_) + f / (BN / 4)) * ldg + n0 + (f % (BN / 4)) * 4); \
    }                                                                                                      \
    _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                                    \
      const int f = tid + 256 * i;                                                                         \
      if (X_F4 % 256 == 0 || f < X_F4)                                                                     \
        rx[set_][i] = *reinterpret_cast<const float4*>(X + ((m_) + f / (BK / 4)) * ldx + k0 + (f % (BK / 4)) * 4); \
    }                                                                                                      \
  }
#define WX6_SSTORE(set_, buf_)                                                                             \
  {                                                                                                        \
    nerf_bf16* Gs_ = smem + (buf_) * STAGE;                                                                \
    nerf_bf16* Xs_ = Gs_ + 3 * IG;                                                                         \
    _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                                    \
      const int f = tid + 256 * i;                                                                         \
      if (G_F4 % 256 == 0 || f < G_F4) {                                                                   \
        uint2 h, m, l;                                                                                     \
        x6_split4(rg[set_][i], h, m, l);                                                                   \
        const int o = (f / (BN / 4)) * PG + (f % (BN / 4)) * 4;                                            \
        *reinterpret_cast<uint2*>(Gs_ + o) = h;                                                            \
        *reinterpret_cast<uint2*>(Gs_ + IG + o) = m;                                                       \
        *reinterpret_cast<uint2*>(Gs_ + 2 * IG + o) = l;                                                   \
      }                                                                                                    \
    }                                                                                                      \
    _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                                    \
      const int f = tid + 256 * i;                                                                         \
      if (X_F4 % 256 == 0 || f < X_F4) {                                                                   \
        uint2 h, m, l;                                                                                     \
        x6_split4(rx[set_][i], h, m, l);                                                                   \
        const int o = (f / (BK / 4)) * PX + (f % (BK / 4)) * 4;                                            \
        *reinterpret_cast<uint2*>(Xs_ + o) = h;                                                            \
        *reinterpret_cast<uint2*>(Xs_ + IX + o) = m;                                                       \
        *reinterpret_cast<uint2*>(Xs_ + 2 * IX + o) = l;                                                   \
      }                                                                                                    \
    }                                                                                                      \
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

  // transposing-read addressing (gemm_bf16.hpp): lane 4q + p of 16-lane group g reads row 8 (g >> 1) + 4 t + q,
  // columns 16 (g & 1) + 4 p .. + 3; lane i of the group receives column 16 (g & 1) + i
  const int grp = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int trow = 8 * (grp >> 1) + q, tcol = 16 * (grp & 1) + 4 * p4;
  auto tr_frag = [&](const nerf_bf16* base, int pitch) {
    const nerf_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) nerf_s16x4*)(base));
    const nerf_s16x4 hi =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) nerf_s16x4*)(base + 4 * pitch));
    const short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(nerf_bf16x8, v8);
  };

  const int64_t nit = (r1 - r0) / MR;
  if (nit > 0) {
#pragma unroll
    for (int j = 0; j < PF; ++j) WX6_GLOAD(j, r0 + (j < nit ? j : nit - 1) * MR);
    WX6_SSTORE(0, 0);
  }
  __syncthreads();
  for (int64_t it0 = 0; it0 < nit; it0 += PF) {
#pragma unroll
   for (int j = 0; j < PF; ++j) {  // slab it = it0 + j: LDS buffer j & 1, register set j
    const int64_t it = it0 + j;
    if (it >= nit) break;
    WX6_GLOAD(j, r0 + (it + PF < nit ? it + PF : nit - 1) * MR);
    const nerf_bf16* Gs = smem + (j & 1) * STAGE;
    const nerf_bf16* Xs = Gs + 3 * IG;
    nerf_bf16x8 af[TM][3], bf[TN][3];
#pragma unroll
    for (int pc = 0; pc < 3; ++pc) {
#pragma unroll
      for (int a = 0; a < TM; ++a) af[a][pc] = tr_frag(Gs + pc * IG + trow * PG + wn * WTN + a * 32 + tcol, PG);
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[b][pc] = tr_frag(Xs + pc * IX + trow * PX + wk * WTK + b * 32 + tcol, PX);
    }
    if (do_bias) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
        {  // the slab's 8 rows summed first, then added to the running sum (64x fewer additions to the large sum)
          float t8 = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) t8 += ((float)af[a][0][j] + (float)af[a][1][j]) + (float)af[a][2][j];
          bsum[a] += t8;
        }
    }
    // A = G^T (rows n, piece X6_PA), B = X (columns k, piece X6_PB); P itself is accumulated (not transposed)
    // the next slab's split + LDS stores interleaved with this slab's MFMAs (as gemm_wgrad_x6w; unconditional: past the
    // last slab they fill the free buffer): C2 208.8k -> 209.6k rays/s on one box, bitwise the same
    // (profiles/r03/x6_wgrad_interleave_ab.txt)
    WX6_SSTORE((j + 1) % PF, (j + 1) & 1);
    X6_MFMA_BLOCK(acc, TM, TN, af[a_][X6_PA[t_]], bf[b_][X6_PB[t_]])
#pragma unroll
    for (int q = 0; q < 6 * TM * TN; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
    __syncthreads();
   }
  }
#undef WX6_GLOAD
#undef WX6_SSTORE

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

// ------------------------------------------------------------------------------------------ gemm_wgrad_x6w
// The 256 x 256 weight gradient of one split in ONE 512-thread workgroup: G and X are each read once per split (the
// 128 x 128-tile form reads them twice, PMC 2.30 GB against 1.68 GB algorithmic per fine launch) and every element is
// split once; eight waves of 64 (n) x 128 (k) (2 x 4 MFMA tiles) amortise each G fragment over four X fragments.
// 16-row slabs, six piece images [16][288] bf16 per stage, double-buffered (108 KiB: one workgroup per CU, two waves
// per SIMD); the loads of slab it + 2 are issued at iteration it (two register sets; three were slower,
// 0.477 -> 0.512 ms in a round-4 A/B build, not kept).  The bias columns are summed from the raw staging registers.  Requirements: rows_per_split % 16 == 0, M % 16 == 0, ldg / ldx % 4 == 0, K >= 256 (the first
// 256 columns of X).
__global__ __launch_bounds__(512, 1) void gemm_wgrad_x6w_kernel(const float* __restrict__ G, int ldg,
                                                               const float* __restrict__ X, int ldx,
                                                               float* __restrict__ P, int ldp, float* __restrict__ Pb,
                                                               int64_t slab, int64_t rows_per_split, int64_t M) {
  constexpr int MR = 16, TM = 2, TN = 4, WTN = 64, WTK = 128;
  constexpr int PT = 256 + 32;                   // pitch = 64 B mod 256 B (transposing reads, gemm_bf16.hpp)
  constexpr int IMG = MR * PT;                   // one piece image
  constexpr int STAGE = 6 * IMG;                 // G hi / mid / lo, X hi / mid / lo
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[2 * STAGE];

  const int s = blockIdx.x;
  const int64_t r0 = (int64_t)s * rows_per_split;
  int64_t r1 = r0 + rows_per_split;
  if (r1 > M) r1 = M;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave >> 1, wk = wave & 1;
  const int li = lane & 31, lh = lane >> 5;
  // bias columns: summed from the raw fp32 G values in the staging registers, 8 FMAs per thread and slab (thread tid
  // holds columns 4 (tid & 63) .. + 3 of rows tid >> 6 (mod 8)), the eight waves' partials added in wave order at the
  // end.  Round 4 summed the three pieces of each MFMA fragment in the wk == 0 waves (48 VALU per tile and slab, the
  // wk == 1 waves idle at the barrier meanwhile): 0.477 ms per fine layer -> 0.445 with the tiles shared by both waves
  // -> 0.426 ms summed raw (profiles/r05/x6_variants_ab.txt; the bias gradients' summation order changed, ~1e-7 of
  // their scale)
  const bool braw = Pb != nullptr;
  float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);

  // staging: a 16 x 256 fp32 slab = 1024 float4, thread f = tid + 512 i: row f >> 6, float4 f & 63
  constexpr int PF = 2;  // register sets (three, loads issued three slabs ahead, were slower: call 29)
  float4 rg[PF][2], rx[PF][2];
#define WX6W_GLOAD(set_, m_)                                                                               \
  _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                                          \
    const int f = tid + 512 * i;                                                                           \
    rg[set_][i] = *reinterpret_cast<const float4*>(G + ((m_) + (f >> 6)) * ldg + 4 * (f & 63));            \
    rx[set_][i] = *reinterpret_cast<const float4*>(X + ((m_) + (f >> 6)) * ldx + 4 * (f & 63));            \
  }
#define WX6W_SSTORE(set_, buf_)                                                                            \
  _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                                          \
    const int f = tid + 512 * i;                                                                           \
    const int o = (f >> 6) * PT + 4 * (f & 63);                                                            \
    nerf_bf16* S_ = smem + (buf_) * STAGE;                                                                 \
    uint2 h, m, l;                                                                                         \
    x6_split4(rg[set_][i], h, m, l);                                                                       \
    *reinterpret_cast<uint2*>(S_ + o) = h;                                                                 \
    *reinterpret_cast<uint2*>(S_ + IMG + o) = m;                                                           \
    *reinterpret_cast<uint2*>(S_ + 2 * IMG + o) = l;                                                       \
    x6_split4(rx[set_][i], h, m, l);                                                                       \
    *reinterpret_cast<uint2*>(S_ + 3 * IMG + o) = h;                                                       \
    *reinterpret_cast<uint2*>(S_ + 4 * IMG + o) = m;                                                       \
    *reinterpret_cast<uint2*>(S_ + 5 * IMG + o) = l;                                                       \
  }
#define WX6W_BACC(set_, sc_)                                                                               \
  _Pragma("unroll") for (int i = 0; i < 2; ++i) {                                                          \
    b4.x = fmaf(rg[set_][i].x, (sc_), b4.x);                                                               \
    b4.y = fmaf(rg[set_][i].y, (sc_), b4.y);                                                               \
    b4.z = fmaf(rg[set_][i].z, (sc_), b4.z);                                                               \
    b4.w = fmaf(rg[set_][i].w, (sc_), b4.w);                                                               \
  }

  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int grp = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
  const int trow = 8 * (grp >> 1) + q, tcol = 16 * (grp & 1) + 4 * p4;
  auto tr_frag = [&](const nerf_bf16* base) {
    const nerf_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) nerf_s16x4*)(base));
    const nerf_s16x4 hi =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) nerf_s16x4*)(base + 4 * PT));
    const short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(nerf_bf16x8, v8);
  };

  const int64_t nit = (r1 - r0) / MR;
  if (nit > 0) {
#pragma unroll
    for (int j = 0; j < PF; ++j) WX6W_GLOAD(j, r0 + (j < nit ? j : nit - 1) * MR);
    WX6W_SSTORE(0, 0);
    if (braw) WX6W_BACC(0, 1.f);
  }
  __syncthreads();
  // slab it: LDS buffer j = it & 1, register set j.  Whole rounds of the two sets run in the loop and a last odd slab
  // is peeled after it: with a break inside the unrolled round, a path with set 0's loads still in flight reached the
  // loop header and the compiler's wait counting drained every load (vmcnt(0)) at the top of each round; 0.425 ->
  // 0.421 ms per fine layer, bitwise the same (profiles/r05/x6_variants_ab.txt, call 34)
  auto do_slab = [&](auto J, const int64_t it) __attribute__((always_inline)) {
      constexpr int j = decltype(J)::value;
      WX6W_GLOAD(j, r0 + (it + PF < nit ? it + PF : nit - 1) * MR);
      const int buf = j;
      const nerf_bf16* Gs = smem + buf * STAGE;
      const nerf_bf16* Xs = Gs + 3 * IMG;
      nerf_bf16x8 af[TM][3];
#pragma unroll
      for (int pc = 0; pc < 3; ++pc)
#pragma unroll
        for (int a = 0; a < TM; ++a) af[a][pc] = tr_frag(Gs + pc * IMG + trow * PT + wn * WTN + a * 32 + tcol);
#pragma unroll
      for (int bp = 0; bp < TN / 2; ++bp) {  // column-block pairs: 2 x 3 X fragments live
        // the next slab's split + LDS stores go between the two column-block pairs (unconditionally: past the last
        // slab they fill the free buffer), and the group barriers below interleave their VALU work one MFMA at a time
        // with the second pair's MFMAs instead of leaving it between the last MFMA and the barrier: 0.52 -> 0.47 ms
        // per fine layer on MI355X (profiles/r03/x6_wgrad_interleave_ab.txt), bitwise the same results
        if (bp == 1) WX6W_SSTORE((j + 1) % PF, buf ^ 1);
        // slab it + 1's G values (a clamped repeat past the last slab: weight 0); x * 1 + s is the exact sum
        if (bp == 1 && braw) WX6W_BACC((j + 1) % PF, it + 1 < nit ? 1.f : 0.f);
        nerf_bf16x8 bf[2][3];
#pragma unroll
        for (int pc = 0; pc < 3; ++pc)
#pragma unroll
          for (int b = 0; b < 2; ++b)
            bf[b][pc] = tr_frag(Xs + pc * IMG + trow * PT + wk * WTK + (2 * bp + b) * 32 + tcol);
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
              acc[a][2 * bp + b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[a][X6_PA[t]], bf[b][X6_PB[t]],
                                                                         acc[a][2 * bp + b], 0, 0, 0);
        if (bp == 1) {  // the pair's fragment reads first, then one MFMA per ~4 VALU of the split, LDS writes spread
          __builtin_amdgcn_sched_group_barrier(0x100, 6, 0);
#pragma unroll
          for (int q = 0; q < 24; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);
            if (q & 1) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
          }
        }
      }
      __syncthreads();
  };
  int64_t it0 = 0;
  for (; it0 + PF <= nit; it0 += PF) {
    do_slab(std::integral_constant<int, 0>{}, it0);
    do_slab(std::integral_constant<int, 1>{}, it0 + 1);
  }
  if (it0 < nit) do_slab(std::integral_constant<int, 0>{}, it0);
#undef WX6W_GLOAD
#undef WX6W_SSTORE
#undef WX6W_BACC
  if (braw) {  // the eight waves' partials meet in LDS (free after the loop's last barrier), added in wave order
    float* part = reinterpret_cast<float*>(smem);
    *reinterpret_cast<float4*>(part + wave * 256 + 4 * lane) = b4;
    __syncthreads();
    if (tid < 256) {
      float v = part[tid];
#pragma unroll
      for (int w = 1; w < 8; ++w) v += part[w * 256 + tid];
      Pb[(int64_t)s * slab + tid] = v;
    }
  }

  float* Ps = P + (int64_t)s * slab;
#pragma unroll
  for (int a = 0; a < TM; ++a) {
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int k = wk * WTK + b * 32 + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = wn * WTN + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        Ps[(int64_t)n * ldp + k] = acc[a][b][r];
      }
    }
  }
}

