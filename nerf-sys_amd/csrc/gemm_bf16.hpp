// bf16 MFMA GEMMs for the C3 configuration ("bf16 MLP with fp32 compositing", BASELINE.json configs[2]):
// bf16 operands in HBM and LDS, fp32 accumulation on gfx950 `v_mfma_f32_32x32x16_bf16`, fp32 master
// weights and gradients.  Same three shapes as the fp32 path (gemm.hpp):
//   gemm_nt_bf16     C[m][n] = epi( sum_k A[m][k] * B[n][k] )   forward (B = W) / input gradient (B = W^T)
//   gemm_wgrad_bf16  P[s][n][k] = sum_{m in split s} G[m][n] * X[m][k]  (+ bias column sums), fp32 slabs
//
// At these layer shapes (M ~ 10^6 rows, N, K <= 320) the bf16 layers are HBM-bound (1 KB/row/layer of bf16
// activations in + out against ~0.26 MFLOP/row), so the tiles are the fp32 kernel's: 128 x 128 blocks of
// four 64 x 64 wave tiles (2 x 2 MFMA tiles), one barrier per k-slab, register-staged 16-B loads.
//
// Fragments.  32x32x16 bf16 MFMA: lane l (r = l & 31, h = l >> 5) supplies A[i = r][k = 8 h + j] and
// B[k = 8 h + j][col r], j = 0..7 (8 bf16 = 4 VGPRs).
//  * NT: operands are rows with k contiguous -> one ds_read_b128 per fragment from a [rows][BK] LDS tile
//    with a 16-B row pad (pitch BK + 8 bf16: 16 consecutive rows hit 16 distinct 16-B bank slots).
//    As in the fp32 kernel the MFMA computes C^T (i = n from W, j = m from the activations), so lane r
//    owns one output row and the epilogue stores runs of 4 consecutive columns.
//  * wgrad: both operands are indexed by the contraction index m = the ROW of G and X, so a fragment is a
//    column of a row-major [m][cols] LDS tile: two ds_read_b64_tr_b16 (gfx950 transposing read: a
//    16-lane group reads a 4-row x 16-column block and lane i receives column i) give the 8 rows.
//    Row pitch 160 bf16 (320 B = 64 B mod 256 B): the four rows of a block sit in disjoint bank quarters.
#pragma once
#include "gemm.hpp"

// The 16-bit MLP element of this translation unit.  mlp_bf16.hip is compiled twice: as mlp_bf16.o (bf16, the C3 engine
// and autocast(bfloat16)) and with -DNERF_F16=1 as mlp_f16.o (fp16: the operands of the reference's AMP loop,
// torch.autocast(float16), pipelines/online_stage/runtime_adapt.py:291-310, models/metamodule/metamodule.py:150-156).
// Everything below and in the mlp_bf16_*.hpp kernels lives in a namespace named after the element, so the two builds'
// kernels and helpers never meet at link time; "nerf_bf16" names the element type of the build.
#ifndef NERF_F16
#define NERF_F16 0
#endif
#if NERF_F16
#define NERF_H16NS nerf_h16_f16
#else
#define NERF_H16NS nerf_h16_bf16
#endif

namespace NERF_H16NS {

// nerf_bf16: the scalar element (memory arrays, conversions).  nerf_bf16x8: eight 16-bit elements as a REGISTER
// CONTAINER, the bf16 vector type in both builds — the fp16 build reinterprets it only inside h16_mfma and the element
// accessors below.  (As a half vector, hipcc treated the fragments as packed-fp16 values and the fused layer backward
// spilled 70 VGPRs where the bf16 build spills none.)
#if NERF_F16
typedef _Float16 nerf_bf16;
#else
typedef __bf16 nerf_bf16;
#endif
typedef __bf16 nerf_bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 nerf_f16x8 __attribute__((ext_vector_type(8)));
typedef short nerf_s16x4 __attribute__((ext_vector_type(4)));

#if NERF_F16
typedef float nerf_f32x2h __attribute__((ext_vector_type(2)));
typedef _Float16 nerf_f16x2 __attribute__((ext_vector_type(2)));
#endif
__device__ __forceinline__ uint32_t nerf_pack_bf16x2(float a, float b) {
#if NERF_F16  // one v_cvt_pk_f16_f32 (round to nearest even); the scalar casts became two converts and a repack
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(nerf_f32x2h{a, b}, nerf_f16x2));
#else
  const nerf_bf16 x = (nerf_bf16)a, y = (nerf_bf16)b;  // v_cvt_pk_bf16_f32, round to nearest even
  return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
#endif
}
// sin / cos of the frequency encoding for the bf16 path, whose encoding is rounded to bf16 (8-bit mantissa): the
// argument is reduced to [-1/2, 1/2] revolutions and fed to v_sin_f32 / v_cos_f32 (absolute error ~ |x| 6e-8 rad from
// the fp32 product, 5e-5 rad at the top band of |x| = 1.5, far below the 2e-3 bf16 rounding of the result).  The fp32
// path keeps the libm sincosf (pinned to the reference's torch.sin / torch.cos at 1e-5), and so does the fp16 build:
// the reference's encoding is fp32 torch.sin / torch.cos, rounded to fp16 only at the matmul (11-bit significand, so
// the hardware sine's 5e-5 rad would move one rounding in ten at the top band).
__device__ __forceinline__ void pe_sincos_bf16(float x, float* s, float* c) {
#if NERF_F16
  sincosf(x, s, c);
#else
  const float r = x * 0.15915494309189535f;
  const float f = r - rintf(r);
  *s = __builtin_amdgcn_sinf(f);
  *c = __builtin_amdgcn_cosf(f);
#endif
}
// the low / high element of a packed pair as fp32
__device__ __forceinline__ float nerf_bf16_lo(uint32_t u) {
#if NERF_F16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(u & 0xffffu));
#else
  return __uint_as_float(u << 16);
#endif
}
__device__ __forceinline__ float nerf_bf16_hi(uint32_t u) {
#if NERF_F16
  return (float)__builtin_bit_cast(_Float16, (uint16_t)(u >> 16));
#else
  return __uint_as_float(u & 0xffff0000u);
#endif
}
// 32x32x16 MFMA of the build's element (fp32 accumulation): v_mfma_f32_32x32x16_bf16 / v_mfma_f32_32x32x16_f16
__device__ __forceinline__ nerf_f32x16 h16_mfma(nerf_bf16x8 a, nerf_bf16x8 b, nerf_f32x16 c) {
#if NERF_F16
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(nerf_f16x8, a), __builtin_bit_cast(nerf_f16x8, b), c,
                                                0, 0, 0);
#else
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
#endif
}
// element j of a container as fp32 / element j := round(x) (the build's element type); macros, so the bf16 build's
// expressions are the round-4 ones token for token (same ISA)
#if NERF_F16
// through a u16 view: hipcc (ROCm 7.2) folds a bit_cast of a __bf16 vector element to _Float16 into element 0 for every
// j (the narrow weight gradient's bias summed element 0 eight times: trunk.0 bias 2.5x off)
typedef unsigned short nerf_u16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ float h16_get_f16(const nerf_bf16x8 v, int j) {
  return (float)__builtin_bit_cast(_Float16, (unsigned short)__builtin_bit_cast(nerf_u16x8, v)[j]);
}
__device__ __forceinline__ void h16_set_f16(nerf_bf16x8& v, int j, float x) {
  nerf_u16x8 t = __builtin_bit_cast(nerf_u16x8, v);
  t[j] = __builtin_bit_cast(unsigned short, (_Float16)x);
  v = __builtin_bit_cast(nerf_bf16x8, t);
}
#define H16_GET(v, j) h16_get_f16((v), (j))
#define H16_SET(v, j, x) h16_set_f16((v), (j), (x))
#else
#define H16_GET(v, j) ((float)(v)[j])
#define H16_SET(v, j, x) ((v)[j] = (nerf_bf16)(x))
#endif
// The layer output before its bias.  fp16 build: the reference's autocast matmul returns an fp16 tensor and the fp32
// bias is added after it (metamodule.py:153-155: fp16 + fp32 promotes to fp32), so the accumulator is rounded to fp16
// first and the bias added in fp32 (the accumulators start at zero, not at the bias).  bf16 build (the C3 engine's own
// arithmetic): the accumulators start at the bias and nothing is rounded here.
constexpr bool H16_BIAS_AFTER = NERF_F16 != 0;
__device__ __forceinline__ float h16_out(float acc, float bias) {
#if NERF_F16
  return (float)(_Float16)acc + bias;
#else
  return acc;
#endif
}

// epilogue of the bf16 NT GEMMs (C^T: lane li owns row mw + a*32 + li; register r = 4q + e is column
// 8q + 4lh + e of the 32-column tile b).  bf16 outputs leave as one 16-B store per (q, q+1) pair after a
// v_permlane32_swap exchange between the lane halves (cdna_hip_programming.md T21).
template <int TM, int TN, int WTM, int WTN, int EPI, int OUT_BF16>
__device__ __forceinline__ void ntb_epilogue(nerf_f32x16 (&acc)[TM][TN], int64_t mw, int nw, int li, int lh,
                                             const float* __restrict__ bias, void* __restrict__ Cv, int ldc,
                                             const uint32_t* __restrict__ mbits, int ldmb,
                                             uint32_t* __restrict__ mbits_out, const uint32_t* pre_words = nullptr) {
  const int64_t m0 = mw;
  const int n0 = nw;
  constexpr int wm = 0, wn = 0;
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int nb = n0 + wn * WTN + b * 32;
    const int g = nb >> 5;
    float4 bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) bv[q] = *reinterpret_cast<const float4*>(bias + nb + 8 * q + 4 * lh);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int64_t m = m0 + wm * WTM + a * 32 + li;
      uint32_t word = 0;
      if (EPI == EPI_MASK) word = pre_words ? pre_words[a * TN + b] : mbits[m * ldmb + g];
      uint2 pk[4];
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
        if constexpr (OUT_BF16) {
          pk[q] = make_uint2(nerf_pack_bf16x2(v[0], v[1]), nerf_pack_bf16x2(v[2], v[3]));
        } else {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(Cv) + m * ldc + nb + 8 * q + 4 * lh) =
              make_float4(v[0], v[1], v[2], v[3]);
        }
      }
      if constexpr (OUT_BF16) {
        // T21 (cdna_hip_programming.md): lanes li / li + 32 hold columns 8q..8q+3 / 8q+4..8q+7 of the same row;
        // one v_permlane32_swap per dword of the (q, q + 1) pair leaves 16 contiguous bytes in every lane
        // (low half: columns 16p..16p+7, high half: 16p+8..16p+15) -> one 16-B store per pair.
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) {
          uint2 x = pk[2 * pr], y = pk[2 * pr + 1];
          const auto r0 = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
          const auto r1 = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
          x.x = r0[0]; y.x = r0[1];
          x.y = r1[0]; y.y = r1[1];
          *reinterpret_cast<uint4*>(reinterpret_cast<nerf_bf16*>(Cv) + m * ldc + nb + 16 * pr + 8 * lh) =
              make_uint4(x.x, x.y, y.x, y.y);
        }
      }
      if (EPI == EPI_BIAS_RELU && mbits_out) {
        word |= __shfl_xor(word, 32, 64);
        if (lh == 0) mbits_out[m * ldmb + g] = word;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------ gemm_nt_bf16
// EPI as in gemm.hpp.  OUT_BF16: store C as bf16 (activations / activation gradients) or fp32 (head outputs).
// Requirements (host wrapper): M % BM == 0, N % BN == 0, K % BK == 0, lda/ldb % 8 == 0, ldc % 4 == 0.
template <int BM, int BN, int WAVES_M, int EPI, int OUT_BF16, int BK = 64, int MINW = 2>
__global__ __launch_bounds__(256, MINW) void gemm_nt_bf16_kernel(const nerf_bf16* __restrict__ A, int lda,
                                                                const nerf_bf16* __restrict__ B, int ldb,
                                                                const float* __restrict__ bias, void* __restrict__ Cv,
                                                                int ldc, const uint32_t* __restrict__ mbits, int ldmb,
                                                                uint32_t* __restrict__ mbits_out, int K, int n_ntiles) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wave tile");
  static_assert(BK % 16 == 0, "k-slab");
  constexpr int LS = BK + 8;              // LDS row pitch (bf16)
  constexpr int C8 = BK / 8;              // 16-B chunks per row per slab
  constexpr int A_CH = BM * C8, B_CH = BN * C8;
  constexpr int A_PER = (A_CH + 255) / 256, B_PER = (B_CH + 255) / 256;
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[2 * (BM + BN) * LS];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;
  const nerf_bf16* Ab = A + m0 * lda;
  const nerf_bf16* Bb = B + (int64_t)n0 * ldb;

  uint4 ra[A_PER], rb[B_PER];
#define NTB_GLOAD(k0_)                                                                                  \
  _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                                  \
    const int f = tid + 256 * i;                                                                        \
    if (A_CH % 256 == 0 || f < A_CH)                                                                    \
      ra[i] = *reinterpret_cast<const uint4*>(Ab + (int64_t)(f / C8) * lda + (k0_) + (f % C8) * 8);     \
  }                                                                                                     \
  _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                                  \
    const int f = tid + 256 * i;                                                                        \
    if (B_CH % 256 == 0 || f < B_CH)                                                                    \
      rb[i] = *reinterpret_cast<const uint4*>(Bb + (int64_t)(f / C8) * ldb + (k0_) + (f % C8) * 8);     \
  }
#define NTB_SSTORE(buf_)                                                                                \
  {                                                                                                     \
    nerf_bf16* As_ = smem + (buf_) * (BM + BN) * LS;                                                    \
    nerf_bf16* Bs_ = As_ + BM * LS;                                                                     \
    _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                                \
      const int f = tid + 256 * i;                                                                      \
      if (A_CH % 256 == 0 || f < A_CH) *reinterpret_cast<uint4*>(As_ + (f / C8) * LS + (f % C8) * 8) = ra[i]; \
    }                                                                                                   \
    _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                                \
      const int f = tid + 256 * i;                                                                      \
      if (B_CH % 256 == 0 || f < B_CH) *reinterpret_cast<uint4*>(Bs_ + (f / C8) * LS + (f % C8) * 8) = rb[i]; \
    }                                                                                                   \
  }

  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = K / BK;
  NTB_GLOAD(0);
  NTB_SSTORE(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    NTB_GLOAD((kt + 1 < nk ? kt + 1 : kt) * BK);
    const nerf_bf16* As = smem + cur * (BM + BN) * LS;
    const nerf_bf16* Bs = As + BM * LS;
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      nerf_bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[a] = *reinterpret_cast<const nerf_bf16x8*>(As + (wm * WTM + a * 32 + li) * LS + 16 * ks + 8 * lh);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[b] = *reinterpret_cast<const nerf_bf16x8*>(Bs + (wn * WTN + b * 32 + li) * LS + 16 * ks + 8 * lh);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)  // swapped operands: the tile is C^T (i = n, j = m)
          acc[a][b] = h16_mfma(bf[b], af[a], acc[a][b]);
    }
    NTB_SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef NTB_GLOAD
#undef NTB_SSTORE

  ntb_epilogue<TM, TN, WTM, WTN, EPI, OUT_BF16>(acc, m0 + wm * WTM, n0 + wn * WTN, li, lh, bias, Cv, ldc, mbits, ldmb,
                                                mbits_out);
}

// ------------------------------------------------------------------------------------------ gemm_nt_bf16_ring
// Persistent NT GEMM with an LDS-DMA ring: the bf16 layers are HBM-bound, and the register-staged kernel
// above keeps one 32-deep k-slab per block in flight (latency-bound at ~3.4 TB/s).  Here every block walks
// a strided list of output tiles as ONE stream of k-slabs (tile t0, slabs 0..nk-1, tile t0 + grid, ...)
// and the DMA engine (global_load_lds_dwordx4, no VGPR staging) keeps STAGES-1 slabs in flight across
// tile boundaries; a counted `s_waitcnt vmcnt` + raw barrier retire one slab per iteration.
// LDS image per stage: A [BM][32] then B [BN][32] bf16, 64-B rows of four 16-B chunks; DMA writes are
// lane-linear, so chunk c of row r is fetched into slot c ^ ((r >> 2) & 3) by permuting the SOURCE
// address, and a fragment read of chunk c = 2 ks + h finds it there (16 lanes of a ds_read_b128 group:
// 16 distinct bank slots).  Fragment reads are inline asm: a compiler-visible LDS read of the DMA target
// would be preceded by `s_waitcnt vmcnt(0)`, draining the ring.
__device__ __forceinline__ nerf_bf16x8 ntb_lds_read(uint32_t byte_addr) {
  nerf_bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(byte_addr));
  return v;
}
__device__ __forceinline__ void ntb_wait_vmcnt(int n) {
  // s_waitcnt needs an immediate: dispatch the (wave-uniform) count to one of the encodings
  switch (n) {
#define NTB_W(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    NTB_W(0) NTB_W(1) NTB_W(2) NTB_W(3) NTB_W(4) NTB_W(5) NTB_W(6) NTB_W(7) NTB_W(8) NTB_W(9) NTB_W(10) NTB_W(11)
    NTB_W(12) NTB_W(13) NTB_W(14) NTB_W(15) NTB_W(16) NTB_W(17) NTB_W(18) NTB_W(19) NTB_W(20) NTB_W(21) NTB_W(22)
    NTB_W(23) NTB_W(24) NTB_W(25) NTB_W(26) NTB_W(27) NTB_W(28) NTB_W(29) NTB_W(30) NTB_W(31) NTB_W(32)
#undef NTB_W
    default: asm volatile("s_waitcnt vmcnt(32)" ::: "memory"); break;
  }
}

template <int BM, int BN, int WAVES_M, int EPI, int OUT_BF16, int STAGES, int MINW>
__global__ __launch_bounds__(256, MINW) void gemm_nt_bf16_ring_kernel(const nerf_bf16* __restrict__ A, int lda,
                                                                     const nerf_bf16* __restrict__ B, int ldb,
                                                                     const float* __restrict__ bias,
                                                                     void* __restrict__ Cv, int ldc,
                                                                     const uint32_t* __restrict__ mbits, int ldmb,
                                                                     uint32_t* __restrict__ mbits_out, int K,
                                                                     int n_ntiles, int n_tiles) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wave tile");
  constexpr int BK = 32;                          // bf16 per row per slab: 64 B
  constexpr int STAGE_E = (BM + BN) * BK;         // bf16 elements per stage
  constexpr int NPIECE = (BM + BN) / 16;          // 1 KiB DMA pieces per stage (16 rows each)
  constexpr int PPW = (NPIECE + 3) / 4;
  static_assert(STAGES >= 2 && (STAGES - 2) * PPW <= 12, "ring depth");
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[STAGES * STAGE_E];

  const int grid = gridDim.x;
  const int t0 = xcd_remap(blockIdx.x, grid);
  if (t0 >= n_tiles) return;
  const int my_tiles = (n_tiles - t0 + grid - 1) / grid;
  const int nk = K / BK;
  const int total = my_tiles * nk;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;
  const int MYP = (NPIECE % 4 == 0) ? PPW : (NPIECE - wave + 3) / 4;

  // this lane's piece rows (A rows first, then B rows) and swizzled source chunk
  int prow[PPW], pch[PPW];
  bool pa[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int piece = wave + 4 * j;
    const int r = piece * 16 + (lane >> 2);
    pa[j] = r < BM;
    prow[j] = pa[j] ? r : r - BM;
    pch[j] = (lane & 3) ^ ((prow[j] >> 2) & 3);
  }
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;

  auto issue = [&](int g) {
    const int ti = g / nk, kt = g - ti * nk;
    const int tile = t0 + ti * grid;
    const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
    nerf_bf16* st = smem + (g % STAGES) * STAGE_E;
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      const int piece = wave + 4 * j;
      if (NPIECE % 4 == 0 || piece < NPIECE) {
        const nerf_bf16* src = pa[j] ? A + ((int64_t)mt * BM + prow[j]) * lda + kt * BK + 8 * pch[j]
                                     : B + ((int64_t)nt * BN + prow[j]) * ldb + kt * BK + 8 * pch[j];
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(st + piece * 512),
                                         16, 0, 0);
      }
    }
  };

  uint32_t a_off[TM], b_off[TN];
  int a_sw[TM], b_sw[TN];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const int r = wm * WTM + a * 32 + li;
    a_off[a] = (uint32_t)(r * BK * 2);
    a_sw[a] = (r >> 2) & 3;
  }
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int r = wn * WTN + b * 32 + li;
    b_off[b] = (uint32_t)((BM + r) * BK * 2);
    b_sw[b] = (r >> 2) & 3;
  }

  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < total) issue(s0);

  for (int g = 0; g < total; ++g) {
    // retire slab g: this wave's pieces of the younger in-flight slabs (at most STAGES-2) may stay outstanding
    const int younger = (total - 1 - g) < (STAGES - 2) ? (total - 1 - g) : (STAGES - 2);
    ntb_wait_vmcnt(younger * MYP);
    __builtin_amdgcn_s_barrier();  // every wave's pieces of slab g landed; every wave done reading slab g-1
    if (g + STAGES - 1 < total) issue(g + STAGES - 1);
    const uint32_t st = sbase + (uint32_t)((g % STAGES) * STAGE_E * 2);
    nerf_bf16x8 af[2][TM], bf[2][TN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int a = 0; a < TM; ++a) af[ks][a] = ntb_lds_read(st + a_off[a] + 16 * ((2 * ks + lh) ^ a_sw[a]));
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[ks][b] = ntb_lds_read(st + b_off[b] + 16 * ((2 * ks + lh) ^ b_sw[b]));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int a = 0; a < TM; ++a) asm volatile("" : "+v"(af[ks][a]));
#pragma unroll
      for (int b = 0; b < TN; ++b) asm volatile("" : "+v"(bf[ks][b]));
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = h16_mfma(bf[ks][b], af[ks][a], acc[a][b]);
    const int ti = g / nk;
    if (g - ti * nk == nk - 1) {
      const int tile = t0 + ti * grid;
      const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
      ntb_epilogue<TM, TN, WTM, WTN, EPI, OUT_BF16>(acc, (int64_t)mt * BM + wm * WTM, nt * BN + wn * WTN, li, lh, bias,
                                                    Cv, ldc, mbits, ldmb, mbits_out);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------------ gemm_nt_bf16_wsr
// Weights-stationary variant of the ring kernel: a persistent 512-thread block owns ONE BN-column slice of
// B (the layer weights, BN x K bf16, loaded once into LDS) and streams 256-row panels of A through an
// LDS-DMA ring.  Per output row the CUs then ingest only the 2K bytes of A (the ring kernel also re-reads
// a 128-row B tile per 128-row A tile).  B image: row r (K/8 16-B chunks) keeps chunk c in slot
// c ^ (r & 15) within its 256-B group (wsr_slot) -> the 16 rows of a ds_read_b128 group hit 16 distinct
// bank slots (K = 64 and the K = 320 tail: 8-chunk groups, 2-way).
// 8 waves = 4 (m) x 2 (n) of 64 x 64; blocks b and b + 8 (one XCD) take the two column slices of the same
// panels.  LDS: B 2 K * BN bytes + STAGES * 16 KiB.
// slot of 16-B chunk c of B row r: XOR-swizzled inside its aligned group of 16 chunks (8 for a row's
// 8-chunk tail, K % 128 == 64), so the swizzle never leaves the row
template <int KC>
__device__ __forceinline__ int wsr_slot(int c, int r) {
  static_assert(KC % 8 == 0, "K % 64");
  const int base = c & ~15;
  const int gmask = (base + 16 <= KC) ? 15 : 7;
  return base | ((c ^ r) & gmask);
}

template <int K, int BN, int EPI, int OUT_BF16, int STAGES>
__global__ __launch_bounds__(512, 1) void gemm_nt_bf16_wsr_kernel(const nerf_bf16* __restrict__ A, int lda,
                                                                 const nerf_bf16* __restrict__ B, int ldb,
                                                                 const float* __restrict__ bias,
                                                                 void* __restrict__ Cv, int ldc,
                                                                 const uint32_t* __restrict__ mbits, int ldmb,
                                                                 uint32_t* __restrict__ mbits_out, int n_ntiles,
                                                                 int n_panels) {
  constexpr int BM = 256, WAVES_M = 4, WAVES_N = 2;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  constexpr int BK = 32;
  constexpr int NK = K / BK;
  static_assert(K % BK == 0, "k");
  constexpr int STAGE_E = BM * BK;                // A only: 16 KiB
  constexpr int B_E = BN * K;
  constexpr int KC = K / 8;                       // 16-B chunks per B row
  static_assert(STAGES >= 2 && (STAGES - 2) * 2 <= 12, "ring depth");
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[B_E + STAGES * STAGE_E];

  const int b = blockIdx.x;
  const int cb = (b >> 3) % n_ntiles;
  const int grp = (b & 7) + 8 * (b / (8 * n_ntiles));
  const int n_groups = (gridDim.x / (8 * n_ntiles)) * 8;
  const int n0 = cb * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;

  // resident weight slice (plain loads + swizzled ds_write; once per block)
  {
    constexpr int NCH = BN * KC, PER = (NCH + 511) / 512;
    uint4 v[PER];  // every load in flight before the first LDS write
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + 512 * j;
      if (NCH % 512 == 0 || i < NCH) {
        const int r = i / KC, c = i - r * KC;
        v[j] = *reinterpret_cast<const uint4*>(B + (int64_t)(n0 + r) * ldb + 8 * c);
      }
    }
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int i = tid + 512 * j;
      if (NCH % 512 == 0 || i < NCH) {
        const int r = i / KC, c = i - r * KC;
        *reinterpret_cast<uint4*>(smem + r * K + 8 * wsr_slot<KC>(c, r)) = v[j];
      }
    }
  }
  __syncthreads();
  if (grp >= n_groups) return;
  const int my_panels = grp < n_panels ? (n_panels - grp + n_groups - 1) / n_groups : 0;
  const int total = my_panels * NK;

  // A ring pieces: wave w loads rows [32 w, 32 w + 32) of each 256-row slab as two 1 KiB pieces
  int prow[2], pch[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    prow[j] = 32 * wave + 16 * j + (lane >> 2);
    pch[j] = (lane & 3) ^ ((prow[j] >> 2) & 3);
  }
  nerf_bf16* const ring = smem + B_E;
  const uint32_t rbase = (uint32_t)(uintptr_t)ring, bbase = (uint32_t)(uintptr_t)smem;
  auto issue = [&](int g) {
    const int pi = g / NK, kt = g - pi * NK;
    const int64_t m0 = (int64_t)(grp + pi * n_groups) * BM;
    nerf_bf16* st = ring + (g % STAGES) * STAGE_E;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const nerf_bf16* src = A + (m0 + prow[j]) * lda + kt * BK + 8 * pch[j];
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(st + (2 * wave + j) * 512), 16, 0, 0);
    }
  };

  uint32_t a_off[TM];
  int a_sw[TM];
#pragma unroll
  for (int a = 0; a < TM; ++a) {
    const int r = wm * WTM + a * 32 + li;
    a_off[a] = (uint32_t)(r * BK * 2);
    a_sw[a] = (r >> 2) & 3;
  }
  uint32_t b_row[TN];
  int b_sw[TN];
#pragma unroll
  for (int t = 0; t < TN; ++t) {
    const int r = wn * WTN + t * 32 + li;
    b_row[t] = bbase + (uint32_t)(r * K * 2);
    b_sw[t] = r & 15;
  }

  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int t = 0; t < TN; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][t][r] = 0.f;

#pragma unroll
  for (int s0 = 0; s0 < STAGES - 1; ++s0)
    if (s0 < total) issue(s0);

  // epilogue stores per lane (bf16 outputs: one 16-B store per pair of 32-column halves; fp32: 4 per tile) plus the
  // ReLU bitmask word stores of the forward; they are younger than the DMA of the next STAGES - 1 slabs, and vmcnt
  // counts in issue order, so a wait that ignored them would drain the stores at every panel boundary
#ifndef NERF_WSR_STORE_AWARE
#define NERF_WSR_STORE_AWARE 1
#endif
  // exact count only: an over-count would let a wait pass before its slab landed
  const int NST = TM * TN * (OUT_BF16 ? 2 : 4) + ((EPI == EPI_BIAS_RELU && mbits_out) ? TM * TN : 0);
  constexpr int NML = (EPI == EPI_MASK) ? TM * TN : 0;  // mask-word loads issued at each panel start
  uint32_t words[TM * TN];
  for (int g = 0; g < total; ++g) {
    const int younger = (total - 1 - g) < (STAGES - 2) ? (total - 1 - g) : (STAGES - 2);
    // vector-memory ops issued after slab g's DMA (at iteration g - STAGES + 1) and still possibly in flight:
    // the DMA of the younger slabs, the epilogue stores of iterations g - STAGES + 1 .. g - 1 and the mask-word
    // loads of panel starts g - STAGES + 2 .. g - 1
    int extra = 0;
    if (NERF_WSR_STORE_AWARE) {
#pragma unroll
      for (int e = 1; e <= STAGES - 1; ++e) {
        if (g - e >= 0 && (g - e) % NK == NK - 1) extra += NST;
        if (e <= STAGES - 2 && g - e >= 0 && (g - e) % NK == 0) extra += NML;
      }
    }
    ntb_wait_vmcnt(younger * 2 + extra);
    __builtin_amdgcn_s_barrier();
    const int pi = g / NK, kt = g - pi * NK;
    if (EPI == EPI_MASK && kt == 0) {  // this panel's ReLU mask words, long before its epilogue needs them
      const int64_t mp = (int64_t)(grp + pi * n_groups) * BM + wm * WTM;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int t = 0; t < TN; ++t) {
          // inline-asm load: a compiler-visible load used NK - 1 iterations later makes the waitcnt pass emit
          // vmcnt(0) at the epilogue (it cannot count across the loop back-edge), draining the DMA ring every panel;
          // the slab waits above already cover it (it is older than the DMA of slab kt = NK - 1)
          const uint32_t* pm = mbits + (mp + a * 32 + li) * ldmb + ((n0 + wn * WTN + t * 32) >> 5);
          asm volatile("global_load_dword %0, %1, off" : "=v"(words[a * TN + t]) : "v"(pm) : "memory");
        }
    }
    if (g + STAGES - 1 < total) issue(g + STAGES - 1);
    const uint32_t st = rbase + (uint32_t)((g % STAGES) * STAGE_E * 2);
    nerf_bf16x8 af[2][TM], bf[2][TN];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int a = 0; a < TM; ++a) af[ks][a] = ntb_lds_read(st + a_off[a] + 16 * ((2 * ks + lh) ^ a_sw[a]));
#pragma unroll
      for (int t = 0; t < TN; ++t) {
        const int c = 4 * kt + 2 * ks + lh;  // chunk of the B row
        bf[ks][t] = ntb_lds_read(b_row[t] + 16 * wsr_slot<KC>(c, b_sw[t]));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int a = 0; a < TM; ++a) asm volatile("" : "+v"(af[ks][a]));
#pragma unroll
      for (int t = 0; t < TN; ++t) asm volatile("" : "+v"(bf[ks][t]));
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int t = 0; t < TN; ++t)
          acc[a][t] = h16_mfma(bf[ks][t], af[ks][a], acc[a][t]);
    if (kt == NK - 1) {
      const int64_t m0 = (int64_t)(grp + pi * n_groups) * BM;
      if (EPI == EPI_MASK) {
#pragma unroll
        for (int i = 0; i < TM * TN; ++i) asm volatile("" : "+v"(words[i]));  // uses stay behind the slab wait
      }
      ntb_epilogue<TM, TN, WTM, WTN, EPI, OUT_BF16>(acc, m0 + wm * WTM, n0 + wn * WTN, li, lh, bias, Cv, ldc, mbits,
                                                    ldmb, mbits_out, EPI == EPI_MASK ? words : nullptr);
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int t = 0; t < TN; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[a][t][r] = 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------------ gemm_wgrad_bf16
// P[s][n][k] (row pitch ldp, fp32) = sum over rows m of split s of G[m][n] * X[m][k]; the tiles of column
// block 0 also write Pb[s][n] = sum_m G[m][n].  MFMA A = G^T (i = n, k-slot = m), B = X (k-slot = m, j = k).
// Requirements: rows_per_split % MR == 0, M % 32 == 0, ldg/ldx % 8 == 0.  MR = rows per LDS slab: the
// narrow launches (one or two tiles per split) stage 64 rows to keep enough bytes in flight per CU; the
// 16-row MFMA k-steps run in the same row order for every MR, so P does not depend on it.
template <int BN, int BK, int WAVES_N, int MR = 32>
__global__ __launch_bounds__(256, 2) void gemm_wgrad_bf16_kernel(const nerf_bf16* __restrict__ G, int ldg,
                                                                const nerf_bf16* __restrict__ X, int ldx,
                                                                float* __restrict__ P, int ldp, float* __restrict__ Pb,
                                                                int64_t slab, int64_t rows_per_split, int64_t M,
                                                                int n_ktiles, int n_tiles) {
  constexpr int WAVES_K = 4 / WAVES_N;
  constexpr int WTN = BN / WAVES_N, WTK = BK / WAVES_K;
  constexpr int TM = WTN / 32, TN = WTK / 32;
  static_assert(TM >= 1 && TN >= 1, "wave tile");
  static_assert(MR == 32 || MR == 64, "rows per slab");
  constexpr int PG = ((BN + 127) / 128) * 128 + 32, PX = ((BK + 127) / 128) * 128 + 32;  // pitch = 64 B mod 256 B
  constexpr int G_CH = MR * BN / 8, X_CH = MR * BK / 8;
  constexpr int G_PER = (G_CH + 255) / 256, X_PER = (X_CH + 255) / 256;
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[2 * MR * (PG + PX)];

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

  uint4 rg[G_PER], rx[X_PER];
#define WGB_GLOAD(m_)                                                                                   \
  _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                                  \
    const int f = tid + 256 * i;                                                                        \
    if (G_CH % 256 == 0 || f < G_CH)                                                                    \
      rg[i] = *reinterpret_cast<const uint4*>(G + ((m_) + f / (BN / 8)) * ldg + n0 + (f % (BN / 8)) * 8); \
  }                                                                                                     \
  _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                                  \
    const int f = tid + 256 * i;                                                                        \
    if (X_CH % 256 == 0 || f < X_CH)                                                                    \
      rx[i] = *reinterpret_cast<const uint4*>(X + ((m_) + f / (BK / 8)) * ldx + k0 + (f % (BK / 8)) * 8); \
  }
#define WGB_SSTORE(buf_)                                                                                \
  {                                                                                                     \
    nerf_bf16* Gs_ = smem + (buf_) * MR * (PG + PX);                                                    \
    nerf_bf16* Xs_ = Gs_ + MR * PG;                                                                     \
    _Pragma("unroll") for (int i = 0; i < G_PER; ++i) {                                                \
      const int f = tid + 256 * i;                                                                      \
      if (G_CH % 256 == 0 || f < G_CH)                                                                  \
        *reinterpret_cast<uint4*>(Gs_ + (f / (BN / 8)) * PG + (f % (BN / 8)) * 8) = rg[i];              \
    }                                                                                                   \
    _Pragma("unroll") for (int i = 0; i < X_PER; ++i) {                                                \
      const int f = tid + 256 * i;                                                                      \
      if (X_CH % 256 == 0 || f < X_CH)                                                                  \
        *reinterpret_cast<uint4*>(Xs_ + (f / (BK / 8)) * PX + (f % (BK / 8)) * 8) = rx[i];              \
    }                                                                                                   \
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

  // transposing-read addressing: lane 4q + p of 16-lane group g reads row 8 h + 4 t + q (h = g >> 1, t = read
  // 0/1 of the pair), columns c0 + 16 (g & 1) + 4 p .. + 3; lane i of the group receives column c0 + 16 (g & 1) + i
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int trow = 8 * (grp >> 1) + q, tcol = 16 * (grp & 1) + 4 * p;

  const int64_t nit = (r1 - r0) / MR;
  if (nit > 0) {
    WGB_GLOAD(r0);
    WGB_SSTORE(0);
  }
  __syncthreads();
  for (int64_t it = 0; it < nit; ++it) {
    const int cur = (int)(it & 1);
    WGB_GLOAD(r0 + (it + 1 < nit ? it + 1 : it) * MR);
    const nerf_bf16* Gs = smem + cur * MR * (PG + PX);
    const nerf_bf16* Xs = Gs + MR * PG;
#pragma unroll
    for (int ks = 0; ks < MR / 16; ++ks) {
      nerf_bf16x8 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        const nerf_bf16* base = Gs + (16 * ks + trow) * PG + wn * WTN + a * 32 + tcol;
        const nerf_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) nerf_s16x4*)(base));
        const nerf_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) nerf_s16x4*)(base + 4 * PG));
        const short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        af[a] = __builtin_bit_cast(nerf_bf16x8, v8);
      }
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const nerf_bf16* base = Xs + (16 * ks + trow) * PX + wk * WTK + b * 32 + tcol;
        const nerf_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) nerf_s16x4*)(base));
        const nerf_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            (__attribute__((address_space(3))) nerf_s16x4*)(base + 4 * PX));
        const short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        bf[b] = __builtin_bit_cast(nerf_bf16x8, v8);
      }
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        if (do_bias) {
#pragma unroll
          for (int j = 0; j < 8; ++j) bsum[a] += H16_GET(af[a], j);
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) acc[a][b] = h16_mfma(af[a], bf[b], acc[a][b]);
      }
    }
    WGB_SSTORE(cur ^ 1);
    __syncthreads();
  }
#undef WGB_GLOAD
#undef WGB_SSTORE

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

}  // namespace NERF_H16NS
using namespace NERF_H16NS;
