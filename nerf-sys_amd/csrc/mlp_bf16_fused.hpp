// Fused bf16 forward of the whole vanilla NeRF MLP (BASELINE.json configs[2]) — ONE launch per pass instead of
// one GEMM launch per layer with every activation through HBM.  models/inr/meta_vanilla.py:109-154:
//   enc (xyz PE) -> 8 x [Linear + ReLU] (skip cat([h, enc]) at trunk.4) -> head (sigma | 15 geo)
//   -> cat([geo, dir PE]) -> Linear 42->128 + ReLU -> Linear 128->3 -> sigmoid ; sigma = trunc_exp
//
// A workgroup (4 waves, one per SIMD) owns a tile of 128 sample rows for the whole network.  The tile's
// activations stay in LDS across the layers (H [128][256] bf16; E [128][64] holds the xyz encoding for trunk.0
// / trunk.4 and then the colour input); the MFMA accumulators hold one layer's output tile (wave w: output
// columns 64w..64w+63 of all 128 rows, 4 x 2 `v_mfma_f32_32x32x16_bf16` tiles of C^T as in gemm_bf16.hpp).
// Weights stream from L2 in a fragment-major bf16 image (frag_pack_kernel): the 16-B A-operand fragment of
// lane l for (32-row block nb, 16-deep k-step ks) sits at ((nb * KS + ks) * 64 + l) * 8, so one wave-load
// reads 1 KiB contiguous.  Four k-steps of fragments are kept in flight in a register ring that runs across
// layer boundaries (the next layer's first fragments load under the current layer's last MFMAs).  Biases
// initialise the accumulators.  Epilogue per layer: barrier, ReLU + bf16 into H (16-B LDS stores after the
// v_permlane32_swap pairing of gemm_bf16.hpp), barrier; in training the tile is then copied H -> HBM with
// coalesced 512-B row stores (the activations nerf_mlp_bwd_bf16 reads) and the ReLU bitmask words go out from
// the accumulator registers.
//
// HBM per sample row: reads enc (128 B, written by pe_prefill_bf16_kernel with the colour-input prefill,
// 128 B), writes rgb_sigma (16 B); training adds the saved activations (8 x 512 B + heads ~0.5 KB).
// MFMA work per 128-row tile: 4,112 32x32x16 MFMAs (trunk 3,840, heads 272); weights read from L2 once per
// tile (~1 MB).
#pragma once
#include "gemm_bf16.hpp"
#include "mlp_common.hpp"

namespace NERF_H16NS {
namespace nerf_fused {
using namespace nerf_mlp;

constexpr int FT = 11;                      // fragment tensors: trunk.0..7, head, colour0, colour1
constexpr int BMF = 128;                    // rows per tile
constexpr int HP = 264, EP = 72, CP = 136;  // LDS row pitches (bf16): 16 rows -> 16 distinct 16-B bank slots
constexpr int FN[FT] = {256, 256, 256, 256, 256, 256, 256, 256, 32, 128, 32};
constexpr int FK[FT] = {64, 256, 256, 256, 320, 256, 256, 256, 256, 64, 128};
constexpr int FSRC[FT] = {0, 2, 4, 6, 8, 10, 12, 14, 16, 18, 20};  // weight tensor index in the packed layout

struct FragTab {
  int64_t off[FT + 1];  // bf16 element offsets of each tensor's fragment image (off[FT] = total)
  int64_t src[FT];      // fp32 offsets of the source tensors in the packed layout
};

inline FragTab frag_tab() {
  const Layout& L = layout();
  FragTab T{};
  int64_t o = 0;
  for (int t = 0; t < FT; ++t) {
    T.off[t] = o;
    T.src[t] = L.off[FSRC[t]];
    o += (int64_t)FN[t] * FK[t];
  }
  T.off[FT] = o;
  return T;
}

// fp32 packed [N][K] -> fragment-major bf16: chunk c (8 values) = tensor t, (nb, ks) = c/64 split, lane c%64
__global__ void frag_pack_kernel(const float* __restrict__ w, nerf_bf16* __restrict__ wf, FragTab T) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c * 8 >= T.off[FT]) return;
  int t = 0;
#pragma unroll
  for (int i = 1; i < FT; ++i)
    if (c * 8 >= T.off[i]) t = i;
  const int K = FK[t], KS = K / 16;
  const int64_t lc = c - T.off[t] / 8;
  const int lane = (int)(lc & 63);
  const int64_t fr = lc >> 6;
  const int nb = (int)(fr / KS), ks = (int)(fr - (int64_t)nb * KS);
  const int row = 32 * nb + (lane & 31), k0 = 16 * ks + 8 * (lane >> 5);
  const float4* s = reinterpret_cast<const float4*>(w + T.src[t] + (int64_t)row * K + k0);
  const float4 a = s[0], b = s[1];
  *reinterpret_cast<uint4*>(wf + c * 8) = make_uint4(nerf_pack_bf16x2(a.x, a.y), nerf_pack_bf16x2(a.z, a.w),
                                                     nerf_pack_bf16x2(b.x, b.y), nerf_pack_bf16x2(b.z, b.w));
}

// xyz PE (models/encodings.py:437-444, L = 10, include_input) -> X3E cols 256..319 (bf16) and the colour-input
// prefill CIN[m] = [0 x 15, d, dir PE (L = 4), 0 ...] (meta_vanilla.py:109-121; the fused kernel fills the
// 15 geo columns).  Rows M..Mp-1 are zero.
__global__ __launch_bounds__(256) void pe_prefill_bf16_kernel(const float* __restrict__ xd, int64_t M, int64_t Mp, nerf_bf16* __restrict__ X3E,
                                       nerf_bf16* __restrict__ CIN) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= Mp) return;
  // two phases (xyz encoding, then the colour-input prefill), each packed and stored before the next: one 64-value
  // array live at a time (the fp16 build's libm sincosf spilled 60 VGPRs with both arrays live)
  float v[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) v[i] = 0.f;
  if (m < M) {
    const float x[3] = {xd[m * 6], xd[m * 6 + 1], xd[m * 6 + 2]};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v[k] = x[k];
      float band = 1.0f;
#pragma unroll
      for (int l = 0; l < 10; ++l) {
        float s, cs;
        pe_sincos_bf16(x[k] * band, &s, &cs);
        v[3 + k * 20 + l] = cs;
        v[3 + k * 20 + 10 + l] = s;
        band *= 2.0f;
      }
    }
  }
  uint4* q = reinterpret_cast<uint4*>(X3E + m * 320 + 256);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    q[i] = make_uint4(nerf_pack_bf16x2(v[8 * i], v[8 * i + 1]), nerf_pack_bf16x2(v[8 * i + 2], v[8 * i + 3]),
                      nerf_pack_bf16x2(v[8 * i + 4], v[8 * i + 5]), nerf_pack_bf16x2(v[8 * i + 6], v[8 * i + 7]));
#pragma unroll
  for (int i = 0; i < 64; ++i) v[i] = 0.f;
  if (m < M) {
    const float d[3] = {xd[m * 6 + 3], xd[m * 6 + 4], xd[m * 6 + 5]};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v[15 + k] = d[k];
      float band = 1.0f;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        float s, cs;
        pe_sincos_bf16(d[k] * band, &s, &cs);
        v[18 + k * 8 + l] = cs;
        v[18 + k * 8 + 4 + l] = s;
        band *= 2.0f;
      }
    }
  }
  uint4* r = reinterpret_cast<uint4*>(CIN + m * 64);
#pragma unroll
  for (int i = 0; i < 8; ++i)
    r[i] = make_uint4(nerf_pack_bf16x2(v[8 * i], v[8 * i + 1]), nerf_pack_bf16x2(v[8 * i + 2], v[8 * i + 3]),
                      nerf_pack_bf16x2(v[8 * i + 4], v[8 * i + 5]), nerf_pack_bf16x2(v[8 * i + 6], v[8 * i + 7]));
}

struct FusedArgs {
  const nerf_bf16* wf;   // fragment image (frag_pack_kernel)
  const float* w;        // fp32 packed parameters (biases)
  nerf_bf16* X3E;        // [Mp][320]: cols 256..319 = enc (read); training: cols 0..255 = trunk.3 output
  nerf_bf16* Y;          // training: Y0, Y1, Y2, Y4, ..., Y7 back to back ([Mp][256] each; Y3 lives in X3E)
  uint32_t* MB;          // training: MB0..MB7 back to back ([Mp][8] ReLU bitmask words each)
  float* O16;            // [Mp][32] fp32: col 0 = sigma pre-activation (training, layered backward only)
  nerf_bf16* CIN;        // [Mp][64] colour input (prefill read; training: written back complete)
  nerf_bf16* C0;         // [Mp][128] (training)
  uint32_t* MC0;         // [Mp][4] (training)
  float* O3;             // [Mp][32] fp32 colour-out pre-activations, cols 0..3 (training, layered backward only)
  float* HO;             // [Mp][4] fp32 (o3_0, o3_1, o3_2, sigma_raw): what the fused tail reads (training)
  float* out;            // [M][4] rgb_sigma
  const float* xd;       // [M][6] sample points + directions (the io waves encode them: no prefill launch)
  int64_t M, Mp;
  int ntiles;
};

__device__ __forceinline__ void bar() { __syncthreads(); }

typedef nerf_bf16x8 Ring[4][2];
typedef unsigned short nerf_u16x2 __attribute__((ext_vector_type(2)));

// Fragment (nb, kk) of a tensor with KS k-steps.  Loads go through a buffer resource built once per kernel (raw
// buffer over the 1 MB image): voffset = lane * 16 + the wave's fragment column (VGPR), soffset = tensor + k-step
// (wave-uniform SGPR, a few scalar ops next to the load) — plain pointers made the compiler precompute ~250 64-bit
// addresses per tile and spill them.
typedef unsigned int nerf_u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ nerf_bf16x8 frag_ld(__amdgpu_buffer_rsrc_t rs, int tensor_off, int nb, int kk, int KS,
                                               int lane) {
  const nerf_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + nb * KS * 1024, tensor_off + kk * 1024, 0);
  return __builtin_bit_cast(nerf_bf16x8, v);
}

__device__ __forceinline__ nerf_bf16x8 lds_frag(const nerf_bf16* p) { return *reinterpret_cast<const nerf_bf16x8*>(p); }

// accumulator init with the bias of columns 8q + 4lh + e of the 32-column block starting at col0
// biases of every layer, staged in LDS once per workgroup: trunk.i at 256 i, head 2048, colour0 2080, colour1 2208
constexpr int BOFF[FT] = {0, 256, 512, 768, 1024, 1280, 1536, 1792, 2048, 2080, 2208};
constexpr int BTOT = 2240;
// (fp16 build: zero — the bias is added after the matmul output's fp16 rounding, gemm_bf16.hpp h16_out)
__device__ __forceinline__ void acc_bias(nerf_f32x16& acc, const float* bias, int col0, int lh) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if constexpr (H16_BIAS_AFTER) {
      acc[4 * q + 0] = acc[4 * q + 1] = acc[4 * q + 2] = acc[4 * q + 3] = 0.f;
    } else {
      const float4 b = *reinterpret_cast<const float4*>(bias + col0 + 8 * q + 4 * lh);
      acc[4 * q + 0] = b.x; acc[4 * q + 1] = b.y; acc[4 * q + 2] = b.z; acc[4 * q + 3] = b.w;
    }
  }
}
// the layer output of accumulator register 4 q + e of a 32-column block starting at col0 (fp16 build: fp16-rounded
// matmul output + fp32 bias; bf16 build: the accumulator, which started at the bias)
__device__ __forceinline__ float acc_out(const nerf_f32x16& acc, int r, const float* bias, int col0, int lh) {
  if constexpr (H16_BIAS_AFTER) return h16_out(acc[r], bias[col0 + 8 * (r >> 2) + 4 * lh + (r & 3)]);
  return acc[r];
}

// k-step order of a stage (position p -> k-step kk), so that a wave starts on the columns IT wrote in the previous
// epilogue and the barrier that publishes everyone else's columns overlaps those MFMAs:
//   K_ID    identity (inputs already published: trunk.0 / colour 0 read E)
//   K_ROT16 (p + 4 w) & 15        a 256-wide H input: wave w wrote columns 64w..64w+63 = k-steps 4w..4w+3
//   K_L4    trunk.4 (K = 320): the own 4 h k-steps, the 4 enc k-steps (E, k-steps 16..19), the other 12 h k-steps
//   K_ROT8  (p + 2 w) & 7         colour out over C0: wave w wrote columns 32w..32w+31 = k-steps 2w, 2w+1
#ifndef NERF_FUSED_ROT
#define NERF_FUSED_ROT 0
#endif
enum { K_ID = 0, K_ROT16 = 1, K_L4 = 2, K_ROT8 = 3 };
template <int KIND>
__device__ __forceinline__ int kpos(int p, int w) {
  if (!NERF_FUSED_ROT) return p;
  if (KIND == K_ROT16) return (p + 4 * w) & 15;
  if (KIND == K_L4) return p < 4 ? 4 * w + p : (p < 8 ? 12 + p : ((4 * w + p - 4) & 15));
  if (KIND == K_ROT8) return (p + 2 * w) & 7;
  return p;
}
// A operand source of position p: 0 = H (k-step kk of the Hs tile), 1 = E (k-step kk - EOFF of the Es tile)
template <int KIND, int ESRC>
__device__ __forceinline__ constexpr bool from_e(int p) {
  return ESRC == 1 || (KIND == K_L4 && (NERF_FUSED_ROT ? (p >= 4 && p < 8) : p >= 16));
}
// position of the in-stage barrier: after the wave's own k-steps with rotation, before position 0 without
template <int BARROT>
__device__ __forceinline__ constexpr int barpos() { return BARROT < 0 ? -1 : (NERF_FUSED_ROT ? BARROT : 0); }

// One stage of the pipeline: KS positions over the fragments of tensor `wcur` (NBW fragment columns per wave from nb0)
// in KIND order; A operands from LDS (TA 32-row blocks, rows ar0 + 32 a + li).  The ring holds positions 0..3 on
// entry; consuming position p refills its slot with position p + 4 of this stage or, past the end, with position
// p + 4 - KS of the NEXT stage (KSN positions in KINDN order, NBWN columns from nbn0 of tensor wnext).  BAR >= 0:
// the workgroup barrier that publishes the other waves' epilogue sits between positions BAR - 1 and BAR.
template <int KS, int NBW, int TA, int KIND, int ESRC, int BARROT, int KSN, int NBWN, int KINDN>
__device__ __forceinline__ void stage(nerf_f32x16 (&acc)[4][2], Ring& ring, __amdgpu_buffer_rsrc_t rs, int wcur,
                                      int nb0, int wnext, int nbn0, const nerf_bf16* Hs, const nerf_bf16* Es,
                                      int pitch_h, int pitch_e, int ar0, int li, int lh, int lane, int w) {
  static_assert(KS % 4 == 0 && KSN % 4 == 0, "ring slot alignment across stages");
  constexpr int EOFF = (KIND == K_L4) ? 16 : 0;
  constexpr int BAR = barpos<BARROT>();
  auto afrag = [&](int p, int a) {
    const int r = ar0 + 32 * a + li;
    const int kk = kpos<KIND>(p, w);
    return from_e<KIND, ESRC>(p) ? lds_frag(Es + r * pitch_e + 16 * (kk - EOFF) + 8 * lh)
                                 : lds_frag(Hs + r * pitch_h + 16 * kk + 8 * lh);
  };
  nerf_bf16x8 af[TA];
  if (BAR != 0) {
#pragma unroll
    for (int a = 0; a < TA; ++a) af[a] = afrag(0, a);
  }
#pragma unroll
  for (int p = 0; p < KS; ++p) {
    if (p == BAR) {  // everyone's previous epilogue is in LDS past this point
      bar();
#pragma unroll
      for (int a = 0; a < TA; ++a) af[a] = afrag(p, a);
    }
    nerf_bf16x8 an[TA];  // A fragments of the next position, read under this position's MFMAs
    if (p + 1 < KS && p + 1 != BAR) {
#pragma unroll
      for (int a = 0; a < TA; ++a) an[a] = afrag(p + 1, a);
    }
    nerf_bf16x8 bf[NBW];
#pragma unroll
    for (int b = 0; b < NBW; ++b) bf[b] = ring[p & 3][b];
#ifdef NERF_EXP_FWD_NOWLOAD
    if (false) {
#else
    if (p + 4 < KS) {
#endif
      const int kk = kpos<KIND>(p + 4, w);
#pragma unroll
      for (int b = 0; b < NBW; ++b) ring[p & 3][b] = frag_ld(rs, wcur, nb0 + b, kk, KS, lane);
    } else if (p + 4 - KS < KSN) {
      const int kk = kpos<KINDN>(p + 4 - KS, w);
#pragma unroll
      for (int b = 0; b < NBWN; ++b) ring[p & 3][b] = frag_ld(rs, wnext, nbn0 + b, kk, KSN, lane);
    }
#ifdef NERF_EXP_FWD_NOMFMA
#pragma unroll
    for (int a = 0; a < TA; ++a) asm volatile("" ::"v"(af[a]));
#pragma unroll
    for (int b = 0; b < NBW; ++b) asm volatile("" ::"v"(bf[b]));
#else
#pragma unroll
    for (int a = 0; a < TA; ++a)
#pragma unroll
      for (int b = 0; b < NBW; ++b)
        acc[a][b] = h16_mfma(bf[b], af[a], acc[a][b]);
#endif
    if (p + 1 < KS && p + 1 != BAR) {
#pragma unroll
      for (int a = 0; a < TA; ++a) af[a] = an[a];
    }
  }
}

// ReLU + bf16 of accumulator tiles acc[a][b] (rows ar0 + 32 a + li, cols c0 + 32 b + (C^T register layout)) into an
// LDS tile (pitch): two values per v_cvt_pk_bf16_f32, ReLU as v_pk_max_i16 on the bf16 bit patterns (rounding keeps
// the sign, so round-then-clamp == clamp-then-round), 16-B stores after pairing the lane halves (gemm_bf16.hpp).
typedef float nerf_f32x2 __attribute__((ext_vector_type(2)));
typedef nerf_bf16 nerf_bf16x2 __attribute__((ext_vector_type(2)));
typedef short nerf_s16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t relu_pk(float x, float y) {
  const nerf_f32x2 f = {x, y};
  const nerf_s16x2 z = {0, 0};
  const nerf_s16x2 r = __builtin_elementwise_max(__builtin_bit_cast(nerf_s16x2, __builtin_convertvector(f, nerf_bf16x2)), z);
  return __builtin_bit_cast(uint32_t, r);
}

// fp16 build: the output pair of accumulator registers (r, r + 1) — both fp16-rounded in one v_cvt_pk_f16_f32,
// widened, the fp32 bias pair added in one v_pk_add_f32 — then relu_pk.  (hipcc had already paired the scalar form
// the same way; written on pairs, 5 spilled VGPRs went away and the time stayed: 750 us per training launch against
// 656 us for the bf16 build, whose bias sits in the accumulators — profiles/r05/prof_amp_summary.txt)
// bf16 build: relu_pk of the accumulators.
__device__ __forceinline__ uint32_t relu_pk_out(float a0, float a1, float b0, float b1) {
#if NERF_F16 && !defined(NERF_F16_NOMIX)
  // fp32(fp16 value) + bias in ONE v_fma_mix_f32 per element (f16 source x 1.0 + f32 bias, one fp32 rounding of the
  // exact sum = the fp32 add), instead of a widening convert + half a v_pk_add_f32: hipcc folds fmaf(x, 1, b) into an
  // add and never selects the mixed form
  const uint32_t hb = __builtin_bit_cast(uint32_t, __builtin_convertvector(nerf_f32x2{a0, a1}, nerf_f16x2));
  float z0, z1;
  asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(z0) : "v"(hb), "v"(b0));
  asm("v_fma_mix_f32 %0, %1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(z1) : "v"(hb), "v"(b1));
  return relu_pk(z0, z1);
#elif NERF_F16
  const nerf_f16x2 h = __builtin_convertvector(nerf_f32x2{a0, a1}, nerf_f16x2);
  const nerf_f32x2 x = __builtin_convertvector(h, nerf_f32x2) + nerf_f32x2{b0, b1};
  return relu_pk(x[0], x[1]);
#else
  return relu_pk(a0, a1);
#endif
}

template <int TA, int NB>
__device__ __forceinline__ void relu_to_lds(const nerf_f32x16 (&acc)[4][2], nerf_bf16* dst, int pitch, int ar0, int c0,
                                            int li, int lh, const float* bias) {
#ifdef NERF_EXP_FWD_NOEPI
#pragma unroll
  for (int a = 0; a < TA; ++a)
#pragma unroll
    for (int b = 0; b < NB; ++b) asm volatile("" ::"v"(acc[a][b]));
  return;
#endif
#pragma unroll
  for (int a = 0; a < TA; ++a) {
    const int r = ar0 + 32 * a + li;
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      uint2 pk[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);  // columns c0 + 32 b + 8 q + 4 lh .. + 3
        if constexpr (H16_BIAS_AFTER) b4 = *reinterpret_cast<const float4*>(bias + c0 + 32 * b + 8 * q + 4 * lh);
        pk[q] = make_uint2(relu_pk_out(acc[a][b][4 * q], acc[a][b][4 * q + 1], b4.x, b4.y),
                           relu_pk_out(acc[a][b][4 * q + 2], acc[a][b][4 * q + 3], b4.z, b4.w));
      }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        uint2 x = pk[2 * pr], y = pk[2 * pr + 1];
        const auto r0 = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
        const auto r1 = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
        x.x = r0[0]; y.x = r0[1];
        x.y = r1[0]; y.y = r1[1];
        *reinterpret_cast<uint4*>(dst + r * pitch + c0 + 32 * b + 16 * pr + 8 * lh) = make_uint4(x.x, x.y, y.x, y.y);
      }
    }
  }
}

// copy ROWS x COLS bf16 from an LDS tile (pitch) to global rows m0.. (ld), 16 B per lane, row-contiguous
template <int ROWS, int COLS>
__device__ __forceinline__ void lds_to_global(const nerf_bf16* src, int pitch, nerf_bf16* __restrict__ dst, int64_t ld,
                                              int64_t m0, int tid) {
  constexpr int CH = COLS / 8, TOT = ROWS * CH;
  static_assert(TOT % 256 == 0, "whole passes");
#pragma unroll
  for (int i = 0; i < TOT / 256; ++i) {
    const int f = tid + 256 * i;
    const int r = f / CH, c = f - r * CH;
    *reinterpret_cast<uint4*>(dst + (m0 + r) * ld + 8 * c) = *reinterpret_cast<const uint4*>(src + r * pitch + 8 * c);
  }
}

// global rows m0.. (ld) -> LDS tile (pitch), ROWS x COLS bf16, via registers (loads issued first)
template <int ROWS, int COLS>
struct TileLoad {
  static constexpr int CH = COLS / 8, PER = ROWS * CH / 256;
  uint4 v[PER];
  __device__ __forceinline__ void issue(const nerf_bf16* __restrict__ src, int64_t ld, int64_t m0, int tid) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int f = tid + 256 * i;
      const int r = f / CH, c = f - r * CH;
      v[i] = *reinterpret_cast<const uint4*>(src + (m0 + r) * ld + 8 * c);
    }
  }
  __device__ __forceinline__ void store(nerf_bf16* dst, int pitch, int tid) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int f = tid + 256 * i;
      const int r = f / CH, c = f - r * CH;
      *reinterpret_cast<uint4*>(dst + r * pitch + 8 * c) = v[i];
    }
  }
};

// ---------------------------------------------------------------------------------------------- the kernel
// Workgroup = 8 waves: waves 0-3 compute (MFMA), waves 4-7 move bytes ("io" waves, one per SIMD beside a compute
// wave).  The compute waves issue no global stores on the layer path: every vector-memory op counts in one
// in-order vmcnt, so a burst of activation stores in front of the next layer's weight-fragment loads would make
// each of those loads wait for the stores to drain.  The io waves copy every finished layer tile LDS -> HBM
// (with its ReLU bitmask words) while the compute waves run the next layer, and stage the next tile's
// encoding / colour-input prefill into E.  Persistent: one workgroup per CU walks tiles blockIdx.x + k * grid.
// Both roles pass the same 20 barriers per tile (2 per trunk layer, 2 around the head, 1 after colour layer 0,
// 1 at the end of the tile) plus one in the prologue.
constexpr int NCW = 4;  // compute waves; io waves NCW..2*NCW-1, io wave j owns tile rows 32 j .. 32 j + 31

// compile-time offsets: packed fp32 layout (mlp_common.hpp make_layout) and the fragment image
constexpr int64_t lay_off(int t) {
  int64_t o = 0;
  for (int i = 0; i < t; ++i) {
    int r = 256, c = 1;
    if (i < 16) {
      c = (i % 2 == 0) ? KPAD[i / 2] : 1;
    } else {
      const int R[6] = {32, 32, 128, 128, 32, 32}, C[6] = {256, 1, 64, 1, 128, 1};
      r = R[i - 16];
      c = C[i - 16];
    }
    o += (int64_t)r * c;
    o = (o + 31) & ~int64_t(31);
  }
  return o;
}
constexpr int64_t frag_off(int t) {
  int64_t o = 0;
  for (int i = 0; i < t; ++i) o += (int64_t)FN[i] * FK[i];
  return o;
}

// io wave j: copy rows 32 j .. 32 j + 31 of an LDS tile (COLS bf16 wide, pitch) to global rows m0 + r (ld); with
// MB, also the ReLU bitmask word of every 32 columns (bit = value > 0) to MB[(m0 + r) * (COLS / 32) + g]
typedef unsigned int nerf_u32x4t __attribute__((ext_vector_type(4)));
template <int COLS, bool MASK_>
__device__ __forceinline__ void io_copy(const nerf_bf16* src, int pitch, nerf_bf16* __restrict__ dst, int64_t ld,
                                        int64_t m0, uint32_t* __restrict__ mb, int j, int lane) {
#ifdef NERF_EXP_NOMASK
  constexpr bool MASK = false;
#else
  constexpr bool MASK = MASK_;
#endif
  constexpr int CH = COLS / 8, RPI = 64 / CH, IT = 32 / RPI, B = IT < 8 ? IT : 8;
  const int rl = lane / CH, c = lane - rl * CH;
#pragma unroll
  for (int i0 = 0; i0 < IT; i0 += B) {
    uint4 v[B];
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int r = 32 * j + (i0 + i) * RPI + rl;
      v[i] = *reinterpret_cast<const uint4*>(src + r * pitch + 8 * c);
    }
#pragma unroll
    for (int i = 0; i < B; ++i) {
      const int64_t m = m0 + 32 * j + (i0 + i) * RPI + rl;
#ifdef NERF_EXP_NOSTORE
      if (v[i].x == 0x12345678u && v[i].y == 0x9abcdef0u) *reinterpret_cast<uint4*>(dst + m * ld + 8 * c) = v[i];
#elif defined(NERF_IO_PLAIN_STORES)
      *reinterpret_cast<uint4*>(dst + m * ld + 8 * c) = v[i];
#else
      // non-temporal: the saved activations are read back only by the backward, long after (measured on the fine-net
      // training forward: 1.27 -> 1.06 ms against plain stores)
      __builtin_nontemporal_store(__builtin_bit_cast(nerf_u32x4t, v[i]), reinterpret_cast<nerf_u32x4t*>(dst + m * ld + 8 * c));
#endif
      if (MASK) {
        // post-ReLU bf16: bit = value != 0 (a -0 is 0x8000); 2 values per v_pk_min_u16, quads combined by DPP
        const uint32_t u[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
        uint32_t bits = 0;
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const uint32_t nz = __builtin_bit_cast(uint32_t, __builtin_elementwise_min(
              __builtin_bit_cast(nerf_u16x2, u[h] & 0x7fff7fffu), nerf_u16x2{1, 1}));
          bits |= ((nz & 1u) | (nz >> 15)) << (2 * h);
        }
        bits <<= 8 * (c & 3);
        bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0xB1, 0xf, 0xf, true);  // quad_perm [1,0,3,2]
        bits |= (uint32_t)__builtin_amdgcn_mov_dpp((int)bits, 0x4E, 0xf, 0xf, true);  // quad_perm [2,3,0,1]
        if ((c & 3) == 0) mb[m * (COLS / 32) + (c >> 2)] = bits;
      }
    }
  }
}

// io wave j: 32 rows x 64 bf16 (128 B) of a [rows][ld] global array -> registers -> LDS (four named registers, not
// an array: held across barriers and loop iterations, an array is left in scratch / promoted to LDS)
struct IoRows64 {
  uint4 v0, v1, v2, v3;
  __device__ __forceinline__ void load(const nerf_bf16* __restrict__ src, int64_t ld, int64_t m0, int j, int lane) {
    const nerf_bf16* p = src + (m0 + 32 * j + (lane >> 3)) * ld + 8 * (lane & 7);
    v0 = *reinterpret_cast<const uint4*>(p);
    v1 = *reinterpret_cast<const uint4*>(p + 8 * ld);
    v2 = *reinterpret_cast<const uint4*>(p + 16 * ld);
    v3 = *reinterpret_cast<const uint4*>(p + 24 * ld);
  }
  __device__ __forceinline__ void store(nerf_bf16* dst, int pitch, int j, int lane) const {
    nerf_bf16* p = dst + (32 * j + (lane >> 3)) * pitch + 8 * (lane & 7);
    *reinterpret_cast<uint4*>(p) = v0;
    *reinterpret_cast<uint4*>(p + 8 * pitch) = v1;
    *reinterpret_cast<uint4*>(p + 16 * pitch) = v2;
    *reinterpret_cast<uint4*>(p + 24 * pitch) = v3;
  }
};

// The encodings of rows 32 j + (lane >> 3) + 8 i (i = 0..3) of the tile at m0, computed by io wave j from x_d (lane:
// columns 8 (lane & 7) .. + 7), exactly what pe_prefill_bf16_kernel writes (same sin / cos and bf16 packing, so the
// bits are the same): XYZ — the xyz encoding [x, cos / sin 2^0..2^9 per dimension, 0] (X3E columns 256..319; also
// stored to HBM for the backward's narrow weight gradients); else the colour-input prefill [0 x 15 (geo: the
// compute waves), d, cos / sin 2^0..2^3 per dimension, 0 ...].  Rows >= M are zero.  Replaces the prefill launch and
// its 256 B per row of HBM round trip (round 6).
template <bool XYZ>
__device__ __forceinline__ void io_encode(IoRows64& R, const float* __restrict__ xd, int64_t M, int64_t m0, int j,
                                          int lane, nerf_bf16* __restrict__ x3e) {
  const int cb = 8 * (lane & 7);
  uint4 out[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t m = m0 + 32 * j + (lane >> 3) + 8 * i;
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = 0.f;
    if (m < M) {
      const float* r = xd + m * 6 + (XYZ ? 0 : 3);
      const float x[3] = {r[0], r[1], r[2]};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = cb + e;
        if (XYZ) {
          if (c < 3) {
            v[e] = x[c];
          } else if (c < 63) {
            const int q = c - 3, k = q / 20, rr = q - 20 * k, l = rr < 10 ? rr : rr - 10;
            float sn, cs;
            pe_sincos_bf16(x[k] * (float)(1 << l), &sn, &cs);
            v[e] = rr < 10 ? cs : sn;
          }
        } else {
          if (c >= 15 && c < 18) {
            v[e] = x[c - 15];
          } else if (c >= 18 && c < 42) {
            const int q = c - 18, k = q >> 3, wi = q & 7, l = wi & 3;
            float sn, cs;
            pe_sincos_bf16(x[k] * (float)(1 << l), &sn, &cs);
            v[e] = wi < 4 ? cs : sn;
          }
        }
      }
    }
    out[i] = make_uint4(nerf_pack_bf16x2(v[0], v[1]), nerf_pack_bf16x2(v[2], v[3]), nerf_pack_bf16x2(v[4], v[5]),
                        nerf_pack_bf16x2(v[6], v[7]));
    if (XYZ)  // the backward's copy (read only by the narrow weight gradients, at the end of the backward)
      __builtin_nontemporal_store(__builtin_bit_cast(nerf_u32x4t, out[i]),
                                  reinterpret_cast<nerf_u32x4t*>(x3e + m * 320 + 256 + cb));
  }
  R.v0 = out[0]; R.v1 = out[1]; R.v2 = out[2]; R.v3 = out[3];
}

// Barriers per tile (compute and io waves pass the same sequence): B_k (k = 0..7, "every trunk epilogue k is in
// LDS"; B_k sits inside the stage after k), H2 (colour input complete), C (colour layer 0 output complete, inside
// colour out), D (end of tile: the next tile's encoding is in E).  Trunk epilogue k writes H[k & 1]; the io waves
// copy it to HBM after B_k and must be done before it is overwritten (epilogue k + 2, after B_{k+1}).
template <bool TRAIN, bool MASKS>
__device__ __forceinline__ void io_role(const FusedArgs& A, nerf_bf16* Hs, nerf_bf16* Es, int tile, int G, int j,
                                        int lane) {
  const int64_t Mp = A.Mp;
  IoRows64 enc, cin;
  io_encode<true>(enc, A.xd, A.M, (int64_t)tile * BMF, j, lane, A.X3E);
  enc.store(Es, EP, j, lane);
  bar();  // prologue
  for (int t = tile; t < A.ntiles; t += G) {
    const int64_t m0 = (int64_t)t * BMF;
    const bool next = t + G < A.ntiles;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      bar();  // B_k
      if (k == 4) {  // trunk.4 (the last reader of the encoding) is done: colour-input prefill -> E
        cin.store(Es, EP, j, lane);
        if (next) io_encode<true>(enc, A.xd, A.M, m0 + (int64_t)G * BMF, j, lane, A.X3E);
      }
#ifdef NERF_EXP_ODD_NOSTORE
      // probe of the odd-layer recompute: X1, X3, X5, X7 (epilogues k = 0, 2, 4, 6) not saved
      if (TRAIN && (k & 1)) {
#else
      if (TRAIN) {
#endif
        nerf_bf16* Y = (k == 3) ? A.X3E : A.Y + (int64_t)(k < 3 ? k : k - 1) * Mp * 256;
        io_copy<256, MASKS>(Hs + (k & 1) * BMF * HP, HP, Y, k == 3 ? 320 : 256, m0, MASKS ? A.MB + (int64_t)k * Mp * 8 : nullptr, j,
                            lane);
      }
      if (k == 0) io_encode<false>(cin, A.xd, A.M, m0, j, lane, nullptr);
    }
    bar();  // H2: colour input complete in E
    if (TRAIN) io_copy<64, false>(Es, EP, A.CIN, 64, m0, nullptr, j, lane);
    bar();  // C: colour layer 0 output in H[1]; colour 0 done reading E
    if (next) enc.store(Es, EP, j, lane);
    // C0 (+ its mask words) only for the LAYERED backward: the fused tail recomputes it from CIN (mlp_bf16_tail.hpp)
    if (TRAIN && MASKS) io_copy<128, MASKS>(Hs + BMF * HP, CP, A.C0, 128, m0, A.MC0, j, lane);
    bar();  // D
  }
}

template <bool TRAIN, bool MASKS>
__device__ __forceinline__ void compute_role(const FusedArgs& A, nerf_bf16* Hs, nerf_bf16* Es, float* Ssig,
                                             const float* Bs, int tile, int G, int w, int li, int lh, int lane) {
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc((void*)A.wf, 0, (int)(frag_off(FT) * 2), 0x00020000);
#define F(t) ((int)(frag_off(t) * 2))
#define BI(t) (Bs + BOFF[t])
  nerf_bf16* H0 = Hs;
  nerf_bf16* H1 = Hs + BMF * HP;
  Ring ring;
  nerf_f32x16 acc[4][2];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int b = 0; b < 2; ++b) ring[s][b] = frag_ld(rs, F(0), 2 * w + b, s, 4, lane);
  bar();  // prologue: the first tile's encoding is in E, the biases in Bs

  auto bias_trunk = [&](int t) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) acc_bias(acc[a][b], BI(t), 64 * w + 32 * b, lh);
  };
  for (int t = tile; t < A.ntiles; t += G) {
    const int64_t m0 = (int64_t)t * BMF;
    // trunk: <KS, NBW, TA, KIND, ESRC, BAR, KSN, NBWN, KINDN>; epilogue k -> H[k & 1]
    bias_trunk(0);
    stage<4, 2, 4, K_ID, 1, -1, 16, 2, K_ROT16>(acc, ring, rs, F(0), 2 * w, F(1), 2 * w, H1, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 2>(acc, H0, HP, 0, 64 * w, li, lh, BI(0));
    bias_trunk(1);
    stage<16, 2, 4, K_ROT16, 0, 4, 16, 2, K_ROT16>(acc, ring, rs, F(1), 2 * w, F(2), 2 * w, H0, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 2>(acc, H1, HP, 0, 64 * w, li, lh, BI(1));
    bias_trunk(2);
    stage<16, 2, 4, K_ROT16, 0, 4, 16, 2, K_ROT16>(acc, ring, rs, F(2), 2 * w, F(3), 2 * w, H1, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 2>(acc, H0, HP, 0, 64 * w, li, lh, BI(2));
    bias_trunk(3);
    stage<16, 2, 4, K_ROT16, 0, 4, 20, 2, K_L4>(acc, ring, rs, F(3), 2 * w, F(4), 2 * w, H0, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 2>(acc, H1, HP, 0, 64 * w, li, lh, BI(3));
    bias_trunk(4);
    stage<20, 2, 4, K_L4, 2, 8, 16, 2, K_ROT16>(acc, ring, rs, F(4), 2 * w, F(5), 2 * w, H1, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 2>(acc, H0, HP, 0, 64 * w, li, lh, BI(4));
    bias_trunk(5);
    stage<16, 2, 4, K_ROT16, 0, 4, 16, 2, K_ROT16>(acc, ring, rs, F(5), 2 * w, F(6), 2 * w, H0, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 2>(acc, H1, HP, 0, 64 * w, li, lh, BI(5));
    bias_trunk(6);
    stage<16, 2, 4, K_ROT16, 0, 4, 16, 2, K_ROT16>(acc, ring, rs, F(6), 2 * w, F(7), 2 * w, H1, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 2>(acc, H0, HP, 0, 64 * w, li, lh, BI(6));
    bias_trunk(7);
    // the head's fragments are one 32-column block shared by every wave (nb 0)
    stage<16, 2, 4, K_ROT16, 0, 4, 16, 1, K_ROT16>(acc, ring, rs, F(7), 2 * w, F(8), 0, H0, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 2>(acc, H1, HP, 0, 64 * w, li, lh, BI(7));

    // ---- head: O16 = h7 W_head^T + b (sigma | 15 geo | 0), wave w -> rows 32w..32w+31 (own trunk.7 columns first)
    acc_bias(acc[0][0], BI(8), 0, lh);
    stage<16, 1, 1, K_ROT16, 0, 4, 4, 1, K_ID>(acc, ring, rs, F(8), 0, F(9), w, H1, Es, HP, EP, 32 * w, li, lh, lane, w);
    const int r = 32 * w + li;
    if (lh == 0) Ssig[r] = acc_out(acc[0][0], 0, BI(8), 0, lh);
#pragma unroll
    for (int q = 0; q < 2; ++q)  // geo (cols 1..15) -> colour input cols 0..14 (E holds the prefill since B_4)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = 8 * q + 4 * lh + e;
        if (c >= 1) Es[r * EP + c - 1] = (nerf_bf16)acc_out(acc[0][0], 4 * q + e, BI(8), 0, lh);
      }
    bar();  // H2: colour input complete; every wave done reading H[1] (trunk.7 output)

    // ---- colour layer 0: C0 = ReLU(CIN W_c0^T + b), wave w -> cols 32w..32w+31 of all rows, tile in H[1] (pitch CP)
#pragma unroll
    for (int a = 0; a < 4; ++a) acc_bias(acc[a][0], BI(9), 32 * w, lh);
    stage<4, 1, 4, K_ID, 1, -1, 8, 1, K_ROT8>(acc, ring, rs, F(9), w, F(10), 0, H1, Es, HP, EP, 0, li, lh, lane, w);
    relu_to_lds<4, 1>(acc, H1, CP, 0, 32 * w, li, lh, BI(9));

    // ---- colour out: O3 = C0 W_c1^T + b, wave w -> rows 32w..32w+31 (barrier C after its own 2 k-steps);
    // the next tile's trunk.0 fragments are prefetched into the ring
    acc_bias(acc[0][0], BI(10), 0, lh);
    stage<8, 1, 1, K_ROT8, 0, 2, 4, 2, K_ID>(acc, ring, rs, F(10), 0, F(0), 2 * w, H1, Es, CP, EP, 32 * w, li, lh, lane, w);
    const int64_t m = m0 + r;
    if (lh == 0) {
      const float sraw = Ssig[r];
      if constexpr (H16_BIAS_AFTER)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[0][0][e] = acc_out(acc[0][0], e, BI(10), 0, 0);
      if (TRAIN) {
        // the fused tail reads the colour-out pre-activations and sigma_raw as ONE dense 16-B row (round 6; the two
        // [Mp][32] rows below, 20 B used of two 128-B lines, stay for the layered backward)
        *reinterpret_cast<float4*>(A.HO + m * 4) = make_float4(acc[0][0][0], acc[0][0][1], acc[0][0][2], sraw);
        if (MASKS) {
          A.O16[m * 32] = sraw;
          *reinterpret_cast<float4*>(A.O3 + m * 32) = make_float4(acc[0][0][0], acc[0][0][1], acc[0][0][2], acc[0][0][3]);
        }
      }
      if (m < A.M) {
        const float sg = expf(fminf(fmaxf(sraw, -EXP_MAX), EXP_MAX));
        reinterpret_cast<float4*>(A.out)[m] =
            make_float4(sigmoidf_(acc[0][0][0]), sigmoidf_(acc[0][0][1]), sigmoidf_(acc[0][0][2]), sg);
      }
    }
    bar();  // D: the next tile's encoding is in E
  }
#undef F
#undef BI
}

// MASKS: also write the ReLU bitmask words the LAYERED backward reads (the fused backward, mlp_bf16_bwd.hpp /
// mlp_bf16_tail.hpp, takes its masks from the saved activations themselves; measured: 1.50 -> 1.33 ms per fine-net
// training forward without them)
template <bool TRAIN, bool MASKS>
__global__ __launch_bounds__(512, 1) void mlp_fwd_fused_bf16_kernel(FusedArgs A) {
  __shared__ __attribute__((aligned(16))) nerf_bf16 Hs[2 * BMF * HP];  // H[0], H[1]: trunk epilogues alternate
  __shared__ __attribute__((aligned(16))) nerf_bf16 Es[BMF * EP];
  __shared__ float Ssig[BMF];
  __shared__ __attribute__((aligned(16))) float Bs[BTOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tile = blockIdx.x;
  if (tile >= A.ntiles) return;
  for (int i = tid; i < BTOT; i += 512) {  // biases -> LDS (read by the compute waves after the prologue barrier)
    int t = 0;
#pragma unroll
    for (int k = 1; k < FT; ++k)
      if (i >= BOFF[k]) t = k;
    Bs[i] = A.w[lay_off(FSRC[t] + 1) + (i - BOFF[t])];
  }
  if (w >= NCW)
    io_role<TRAIN, MASKS>(A, Hs, Es, tile, gridDim.x, w - NCW, lane);
  else
    compute_role<TRAIN, MASKS>(A, Hs, Es, Ssig, Bs, tile, gridDim.x, w, lane & 31, lane >> 5, lane);
}

}  // namespace nerf_fused
}  // namespace NERF_H16NS
