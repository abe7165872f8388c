// Fused bf16 backward of one 256 x 256 trunk layer (BASELINE.json configs[2]; models/inr/meta_vanilla.py:123-141,
// the backward of `h = relu(linear_i(h))`): input gradient AND weight gradient in ONE pass over the layer's rows.
//
//   G = dZ_i   [Mp][256] bf16   gradient of the layer's pre-activation (this launch's input)
//   X = X_i    [Mp][ldx] bf16   the layer's input = relu(Z_{i-1}) saved by the forward
//   dZ_{i-1} = (G W_i) * [X_i > 0]                      -> D [Mp][256] bf16 (next launch's G)
//   P[s][n][k] = sum_{m in split s} G[m][n] X[m][k],  Pb[s][n] = sum_m G[m][n]     fp32 split-M slabs
//
// The layered path (gemm_bf16.hpp) runs this as two HBM-bound launches: dgrad reads G + a ReLU bitmask and writes
// D (1,056 B/row), wgrad re-reads G and X (1,024 B/row).  Here each row's G and X are read ONCE (1,536 B/row with
// the D write): the ReLU mask of dZ_{i-1} is X_i > 0, the same X_i tile the weight gradient consumes, and the
// split's weight-gradient accumulators stay in registers across all its rows.
//
// Work split: the 256 x 256 fp32 accumulators of a split (256 KiB) are more than one workgroup can hold next to its
// other state, so a split is served by a PAIR of workgroups, h = 0 / 1 owning input columns k in [128 h, 128 h + 128)
// of both dW and dX.  Blocks b and b + 8 form a pair (round-robin XCD dealing puts them on one XCD: the G tile both
// stream is then read from HBM once and hit in L2 by the partner — PMC: 788 MB fetched per fine launch against
// 806 MB of G + X; speed only, never correctness).
// Workgroup = 12 waves (3 per SIMD, <= 168 VGPRs each):
//   compute waves c = 0..7 own input-column block kb = 4 h + (c & 3) (32 columns) and half mh = c >> 2:
//     wgrad  acc[j] (j = 0..3) = dW[32 (4 mh + j)..][32 kb..]: 4 x v_mfma_f32_32x32x16_bf16 accumulators (64 VGPRs),
//            A = G^T, B = X^T fragments by ds_read_b64_tr_b16 (transposing reads, gfx950);
//     dgrad  dX[rows 32 mh..][32 kb..] = G W_i[:, kb]: 1 accumulator, A = W_i^T fragments from the workgroup's
//            LDS-resident W^T half (64 KiB, loaded once), B = G row fragments;
//     epilogue: ReLU mask from the X tile in LDS, bf16, 16-B stores of D.
//     A compute wave issues no global load at all: its only vector-memory operations are the D stores.  (A first
//     version streamed W^T fragments from L2 through a register ring; queued behind the CU's tile traffic an L2 hit
//     took longer than the ring's 4 k-steps of cover and the kernel ran at 332 us per fine launch.)
//   io waves j = 0..3 (waves 8..11) stream the tiles HBM -> registers -> LDS: two register sets of one tile each
//     (48 VGPRs); a set is written into the free LDS stage and reloaded at once, so two tiles are always in flight.
// Tiles of 64 rows: G [64][256] (32 KiB) + X half [64][128] (16 KiB) per stage, 2 stages + W^T half = 160 KiB;
// one workgroup barrier per tile.
// LDS images are unpadded and XOR-swizzled per 16-B chunk: chunk c of row r sits at slot c ^ swz(r),
// swz(r) = 4 (r & 3) + ((r >> 2) & 3).  Conflict-free for all three access shapes: a ds_read_b128 lane group (16
// rows, one chunk: 16 distinct swz), a ds_read_b64_tr_b16 half-wave (4 rows r0..r0+3, r0 % 4 == 0, x 4 aligned
// chunks: slot = (c ^ 4 q) + (p ^ k) -> 16 distinct slots) and the epilogue's mask reads (as the first).
//
// MFMA order: the weight-gradient k-steps walk the split's rows 16 at a time in row order and the input gradient
// contracts n in 16-wide steps in order, exactly as gemm_wgrad_bf16 / gemm_nt_bf16_wsr do: the result is bitwise
// the layered path's (tests/test_gpu_bf16.py::test_fused_backward_matches_layered).
#pragma once
#include <type_traits>

#include "gemm_bf16.hpp"
#include "mlp_common.hpp"

namespace NERF_H16NS {
namespace nerf_bwd {

constexpr int TR = 64;                  // rows per tile
constexpr int GBY = TR * 512;           // G tile bytes (64 rows x 256 bf16)
constexpr int XBY = TR * 256;           // X half tile bytes (64 rows x 128 bf16)
constexpr int STB = GBY + XBY;          // 48 KiB per stage
constexpr int NSTG = 2;
constexpr int WOFF = NSTG * STB;        // W^T half: [128 k][256 n] bf16, 64 KiB
constexpr int LDS_BYTES = WOFF + 128 * 512;
static_assert(LDS_BYTES <= 163840, "LDS");
constexpr int WT_LAYER = 256 * 256;     // bf16 elements of one layer's W^T image

__device__ __forceinline__ int swz(int r) { return 4 * (r & 3) + ((r >> 2) & 3); }

// W_i^T of trunk layers i = 1..7 (image i - 1), row-major bf16: WT[k][n] = W_i[n][k] for k < 256 (trunk.4: its first
// 256 input columns, the trunk.3 output; the encoding columns need no input gradient) — mlp_bf16.hip builds it with the
// tiled transpose kernel.
typedef unsigned int io_u32x4 __attribute__((ext_vector_type(4)));  // a vector value (uint4 copies become memcpy)

struct LayerArgs {
  const nerf_bf16* G;    // dZ_i [Mp][256]
  const nerf_bf16* X;    // X_i, row pitch ldx (cols 0..255 used)
  const nerf_bf16* WT;   // this layer's W^T image [256][256]
  nerf_bf16* D;          // dZ_{i-1} [Mp][256]
  float* P;              // weight-gradient slab 0 of this tensor (row pitch ldp)
  float* Pb;             // bias-gradient slab 0
  int64_t slab;          // floats between consecutive splits' slabs
  int64_t rps, Mp;       // rows per split (multiple of 64), padded rows (multiple of 256)
  int ldx, ldp, S;
};

// inline-asm LDS reads (byte address + immediate offset); the caller waits lgkmcnt before the use
template <int OFF>
__device__ __forceinline__ nerf_bf16x8 tr_frag_asm(uint32_t a0, uint32_t a1) {
  nerf_s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a0), "i"(OFF) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "i"(OFF) : "memory");
  const short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(nerf_bf16x8, v8);
}
__device__ __forceinline__ nerf_bf16x8 lds_b128(uint32_t a) {
  nerf_bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

typedef unsigned short nerf_u16x2b __attribute__((ext_vector_type(2)));
// keep the bf16 pair v where the matching bf16 of x is nonzero (x is post-ReLU: +0 / -0 both count as zero)
__device__ __forceinline__ uint32_t relu_mask2(uint32_t v, uint32_t x) {
  const nerf_u16x2b nz = __builtin_elementwise_min(__builtin_bit_cast(nerf_u16x2b, x & 0x7fff7fffu), nerf_u16x2b{1, 1});
  const nerf_u16x2b m = nerf_u16x2b{0, 0} - nz;
  return v & __builtin_bit_cast(uint32_t, m);
}

// raw workgroup barrier (no fence): every wave waits for its own LDS writes before it; the empty asm statements keep
// memory operations from being moved across it at the IR level, the sched_barriers at the machine level
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

// every wave: this workgroup's W^T half (rows k = 128 h .. 128 h + 127 of the image) -> LDS, swizzled by row
__device__ __forceinline__ void load_wt(const LayerArgs& A, char* lds, int h, int tid) {
  constexpr int CH = 128 * 32;  // 16-B chunks
  for (int i0 = 0; i0 < CH; i0 += 768 * 4) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 768 + tid;
      if (i < CH) v[u] = *reinterpret_cast<const uint4*>(A.WT + (int64_t)(128 * h + (i >> 5)) * 256 + 8 * (i & 31));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + u * 768 + tid;
      if (i < CH) {
        const int r = i >> 5, c = i & 31;
        *reinterpret_cast<uint4*>(lds + WOFF + r * 512 + 16 * (c ^ swz(r))) = v[u];
      }
    }
  }
}

__device__ __forceinline__ void bwd_compute(const LayerArgs& A, char* lds, int s, int h, int c, int nT,
                                            int64_t r0, int lane) {
  const int li = lane & 31, lh = lane >> 5;
  const int kl = c & 3, mh = c >> 2;  // local 32-column block, row half / n-block half
  const int kb = 4 * h + kl;          // global 32-column block of this wave

  nerf_f32x16 acc[4];  // dW[32 (4 mh + j)..][32 kb..], j = 0..3
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  // LDS byte offsets, split into a per-lane register part and a compile-time part (the swizzle of every row this
  // lane touches depends only on the lane: rows r = 16 ks + trow + 4 t with trow % 4 == q, and r = 32 mh + li).
  // Transposing reads (gemm_bf16.hpp, gemm_wgrad_bf16): lane 4 q + p of 16-lane group g reads row 8 (g >> 1) + 4 t + q,
  // columns 16 (g & 1) + 4 p .. + 3 of a 32-column block; chunk (4 nb + tc) ^ swz(r) = 4 (nb ^ q) + (tc ^ e_t).
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int trow = 8 * (grp >> 1) + q;
  const int tc = 2 * (grp & 1) + (p >> 1), tbyte = 8 * (p & 1);
  int ga[2][4], xa[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int e = (2 * (grp >> 1) + tt) & 3;  // (r >> 2) & 3 of the row read by read tt
    const int base = (trow + 4 * tt) * 512 + 256 * mh + 16 * (tc ^ e) + tbyte;
#pragma unroll
    for (int j = 0; j < 4; ++j) ga[tt][j] = base + 64 * (j ^ q);  // n-block 4 mh + j, + 8192 ks
    xa[tt] = GBY + (trow + 4 * tt) * 256 + 64 * (kl ^ q) + 16 * (tc ^ e) + tbyte;  // + 4096 ks
  }
  // row fragments: G row 32 mh + li and W^T row 32 kl + li, chunk 2 ks + lh -> slot (2 ks) ^ u with u = lh ^ swz(li)
  // (swz(32 a + li) = swz(li)); the X mask reads: X row 32 mh + li, chunk 4 kl + 2 pr + lh -> (4 kl + 2 pr) ^ u
  const int u = lh ^ swz(li);
  const uint32_t lbase = (uint32_t)(uintptr_t)lds;
  const uint32_t wrow = lbase + WOFF + (32 * kl + li) * 512;

  // The pipeline below is ordered by hand: LDS reads are inline asm with immediate offsets and counted lgkmcnt waits
  // (the ds_read_tr intrinsic got no offset folding: one address VGPR per read), each wait asm passes the fragments
  // it covers through "+v" so no MFMA can be hoisted above it, and sched_barrier fences keep the stages in order.
  for (int t = 0; t < nT; ++t) {
    raw_barrier();  // T_t: tile t is in stage t % 2; every wave is done with tile t - 1
    const uint32_t Lb = lbase + (uint32_t)((t % NSTG) * STB);
    uint32_t gat[2][4], xat[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      xat[tt] = Lb + xa[tt];
#pragma unroll
      for (int j = 0; j < 4; ++j) gat[tt][j] = Lb + ga[tt][j];
    }
    const uint32_t rg = Lb + (32 * mh + li) * 512, rx = Lb + GBY + (32 * mh + li) * 256;
    nerf_bf16x8 wfr[4], gfr[4];  // input-gradient fragments, read 3 k-steps ahead
    auto dg_reads = [&](int ks) {
      const uint32_t o = 16 * ((2 * ks) ^ u);
      wfr[ks & 3] = lds_b128(wrow + o);
      gfr[ks & 3] = lds_b128(rg + o);
    };
    // ---- weight gradient: 4 k-steps of 16 rows, fragments of k-step ks + 1 read under the MFMAs of ks (10 reads)
    nerf_bf16x8 xf[2], gf[2][4];
    auto wg_reads = [&](auto KS, int b) {
      constexpr int ks = decltype(KS)::value;
      xf[b] = tr_frag_asm<4096 * ks>(xat[0], xat[1]);
#pragma unroll
      for (int j = 0; j < 4; ++j) gf[b][j] = tr_frag_asm<8192 * ks>(gat[0][j], gat[1][j]);
    };
    wg_reads(std::integral_constant<int, 0>{}, 0);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      constexpr int cb = ks & 1;
      if constexpr (ks + 1 < 4) {
        wg_reads(std::integral_constant<int, ks + 1>{}, cb ^ 1);
        asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(xf[cb]), "+v"(gf[cb][0]), "+v"(gf[cb][1]), "+v"(gf[cb][2]),
                     "+v"(gf[cb][3])::"memory");
      } else {  // the input gradient's first three fragment pairs go out under the last weight-gradient MFMAs
        dg_reads(0);
        dg_reads(1);
        dg_reads(2);
        asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(xf[cb]), "+v"(gf[cb][0]), "+v"(gf[cb][1]), "+v"(gf[cb][2]),
                     "+v"(gf[cb][3])::"memory");
      }
      SCHED_FENCE();
#ifdef NERF_EXP_BWD_NOWG
      asm volatile("" ::"v"(gf[cb][0]), "v"(gf[cb][1]), "v"(gf[cb][2]), "v"(gf[cb][3]), "v"(xf[cb]));
#else
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = h16_mfma(gf[cb][j], xf[cb], acc[j]);
#endif
      SCHED_FENCE();
    });
    // ---- input gradient: dX^T[32 kb..][rows 32 mh..] over n in 16 k-steps
    nerf_f32x16 dacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) dacc[r] = 0.f;
#ifdef NERF_EXP_BWD_XMFMA
    nerf_f32x16 dacc2;  // probe of the odd-layer recompute's MFMA work: one more 16-step chain per tile (no LDS reads)
#pragma unroll
    for (int r = 0; r < 16; ++r) dacc2[r] = 0.f;
#endif
    nerf_bf16x8 xm[2];
    static_for<0, 16>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      nerf_bf16x8& wf = wfr[ks & 3];
      nerf_bf16x8& g = gfr[ks & 3];
      if constexpr (ks + 3 < 16) {
        dg_reads(ks + 3);
        asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(wf), "+v"(g)::"memory");
      } else if constexpr (ks == 13) {  // the epilogue's ReLU-mask chunks
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) xm[pr] = lds_b128(rx + 16 * ((4 * kl + 2 * pr) ^ u));
        asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(wf), "+v"(g)::"memory");
      } else if constexpr (ks == 14) {
        asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(wf), "+v"(g)::"memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(wf), "+v"(g)::"memory");
      }
      SCHED_FENCE();
#ifdef NERF_EXP_BWD_NODG
      asm volatile("" ::"v"(wf), "v"(g));
#else
      dacc = h16_mfma(wf, g, dacc);
#endif
#ifdef NERF_EXP_BWD_XMFMA
      dacc2 = h16_mfma(g, wf, dacc2);
#endif
      SCHED_FENCE();
    });
#ifdef NERF_EXP_BWD_XMFMA
    if (dacc2[0] == 1.2345e-30f) dacc[0] += 1.f;  // keeps the probe chain live
#endif
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(xm[0]), "+v"(xm[1])::"memory");
    // ---- epilogue: lane li owns row 32 mh + li, register 4 q + e = column 8 q + 4 lh + e of the wave's block
    nerf_bf16* Dt = A.D + (r0 + (int64_t)t * TR + 32 * mh + li) * 256 + 32 * kb + 8 * lh;
    uint2 pk[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
      pk[qq] = make_uint2(nerf_pack_bf16x2(dacc[4 * qq], dacc[4 * qq + 1]), nerf_pack_bf16x2(dacc[4 * qq + 2], dacc[4 * qq + 3]));
#pragma unroll
    for (int pr = 0; pr < 2; ++pr) {
      uint2 x = pk[2 * pr], y = pk[2 * pr + 1];
      const auto s0 = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
      const auto s1 = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
      x.x = s0[0]; y.x = s0[1];
      x.y = s1[0]; y.y = s1[1];
      // this lane now holds columns 16 pr + 8 lh .. + 7 of the block
      const uint4 xv = __builtin_bit_cast(uint4, xm[pr]);
      const uint4 o = make_uint4(relu_mask2(x.x, xv.x), relu_mask2(x.y, xv.y), relu_mask2(y.x, xv.z), relu_mask2(y.y, xv.w));
#if defined(NERF_EXP_BWD_NOSTORE)
      asm volatile("" ::"v"(o.x), "v"(o.y), "v"(o.z), "v"(o.w));
#elif defined(NERF_EXP_BWD_NT)
      __builtin_nontemporal_store(io_u32x4{o.x, o.y, o.z, o.w}, reinterpret_cast<io_u32x4*>(Dt + 16 * pr));
#else
      *reinterpret_cast<uint4*>(Dt + 16 * pr) = o;
#endif
    }
    SCHED_FENCE();
  }

  // ---- the split's slab (rows n = 32 (4 mh + j) + 8 (r >> 2) + 4 lh + (r & 3), column k = 32 kb + li)
  float* Ps = A.P + (int64_t)s * A.slab + (int64_t)(128 * mh + 4 * lh) * A.ldp + 32 * kb + li;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float* Pn = Ps + (int64_t)(32 * j) * A.ldp;
#pragma unroll
    for (int r = 0; r < 16; ++r) Pn[((r & 3) + 8 * (r >> 2)) * A.ldp] = acc[j][r];
  }
}

// io wave j: rows 16 j .. 16 j + 15 of every tile, HBM -> registers (one tile per register set, 12 x 16 B per lane:
// 8 G pieces of 2 rows, 4 X-half pieces of 4 rows, each wave-instruction 1 KiB contiguous) -> swizzled LDS stage
// Named members, not arrays: an array member of a set held across loop iterations stays a stack object (scratch),
// with every load waited on before its scratch store.
struct IoSet {
  io_u32x4 v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10, v11;  // 0..7: G pieces, 8..11: X-half pieces
  template <int I>
  __device__ __forceinline__ io_u32x4& at() {
    if constexpr (I == 0) return v0;
    else if constexpr (I == 1) return v1;
    else if constexpr (I == 2) return v2;
    else if constexpr (I == 3) return v3;
    else if constexpr (I == 4) return v4;
    else if constexpr (I == 5) return v5;
    else if constexpr (I == 6) return v6;
    else if constexpr (I == 7) return v7;
    else if constexpr (I == 8) return v8;
    else if constexpr (I == 9) return v9;
    else if constexpr (I == 10) return v10;
    else return v11;
  }
};
__device__ __forceinline__ void io_load(IoSet& S, const LayerArgs& A, int64_t m0, int h, int j, int lane) {
  const nerf_bf16* g = A.G + (m0 + 16 * j + (lane >> 5)) * 256 + 8 * (lane & 31);
  const nerf_bf16* x = A.X + (m0 + 16 * j + (lane >> 4)) * (int64_t)A.ldx + 128 * h + 8 * (lane & 15);
  static_for<0, 8>([&](auto I) {
    constexpr int i = decltype(I)::value;
    S.template at<i>() = *reinterpret_cast<const io_u32x4*>(g + 2 * i * 256);
  });
  static_for<0, 4>([&](auto I) {
    constexpr int i = decltype(I)::value;
    S.template at<8 + i>() = *reinterpret_cast<const io_u32x4*>(x + 4 * i * (int64_t)A.ldx);
  });
}
__device__ __forceinline__ void io_store(IoSet& S, char* st, int j, int lane) {
  static_for<0, 8>([&](auto I) {
    constexpr int i = decltype(I)::value;
    const int r = 16 * j + 2 * i + (lane >> 5), c = lane & 31;
    *reinterpret_cast<io_u32x4*>(st + r * 512 + 16 * (c ^ swz(r))) = S.template at<i>();
  });
  static_for<0, 4>([&](auto I) {
    constexpr int i = decltype(I)::value;
    const int r = 16 * j + 4 * i + (lane >> 4), c = lane & 15;
    *reinterpret_cast<io_u32x4*>(st + GBY + r * 256 + 16 * (c ^ swz(r))) = S.template at<8 + i>();
  });
}

// io wave j also accumulates (workgroup h = 0 only) the bias gradient Pb[n] = sum_m G[m][n] from the G pieces it has in
// registers before they go to LDS: lane (r1, cc) = (lane >> 5, lane & 31) sums rows 16 j + 2 i + r1 of every tile for
// columns 8 cc .. 8 cc + 7; at the end the two row parities are added (shuffle), the four io waves' partials meet in
// LDS and io wave 0 adds them in wave order: a fixed order (bitwise reproducible), but not the layered kernel's.
__device__ __forceinline__ void bias_acc(const IoSet& R, float (&bs)[8]) {
  static_for<0, 8>([&](auto I) {
    constexpr int i = decltype(I)::value;
    const io_u32x4 v = const_cast<IoSet&>(R).template at<i>();
#if NERF_F16
    // fp16 build: each dword as a half2 added to the two fp32 sums with v_dot2c_f32_f16 against (1, 0) / (0, 1) (the
    // exact x + sum with one rounding, no conversion temporaries).  The dword goes through a scalar first: hipcc
    // compiled __builtin_bit_cast(half2, v[d]) on the vector-element lvalue as a read of v[0] for every d (all four
    // column pairs summed column pair 0: trunk bias 1.18 relative error; the fault H16_GET avoids, gemm_bf16.hpp).
    // Measured and not kept: v_cvt_f32_f16 + fp32 adds (hipcc hoists the 64 conversions of a tile set: 70 VGPRs of the
    // io register sets spilled), integer fp16 -> fp32 decoding (296 VGPRs spilled)
    static_for<0, 4>([&](auto D) {
      constexpr int d = decltype(D)::value;
      typedef _Float16 h2_ __attribute__((ext_vector_type(2)));
      const unsigned int u = v[d];
      const h2_ x = __builtin_bit_cast(h2_, u);
      bs[2 * d] = __builtin_amdgcn_fdot2(x, h2_{(_Float16)1.0f, (_Float16)0.0f}, bs[2 * d], false);
      bs[2 * d + 1] = __builtin_amdgcn_fdot2(x, h2_{(_Float16)0.0f, (_Float16)1.0f}, bs[2 * d + 1], false);
    });
#else
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      bs[2 * d] += nerf_bf16_lo(v[d]);
      bs[2 * d + 1] += nerf_bf16_hi(v[d]);
    }
#endif
  });
}

// Two named register sets (an array of sets held across loop iterations is left in scratch): tile k lives in set k % 2.
// Step t stores tile t + 1 into the stage tile t - 1 held, then reloads that set with tile t + 3, so tiles t + 2 and
// t + 3 are in flight while tile t is computed.  Inside the loop every step stores and loads unconditionally (past the
// end: the last tile again, into a stage nobody reads), so the compiler's vmcnt bookkeeping sees one fixed pattern —
// with conditional loads it fell back to draining (vmcnt(0)) before every store.
__device__ __forceinline__ void io_step(IoSet& R, const LayerArgs& A, char* lds, int h, int j, int t, int nT,
                                        int64_t r0, int lane, float (&bs)[8]) {
  raw_barrier();  // T_t: tile t in stage t % 2 is complete; every wave is done with tile t - 1
#ifndef NERF_EXP_BWD_NOIO
  if (h == 0 && t + 1 < nT) bias_acc(R, bs);
  io_store(R, lds + ((t + 1) % NSTG) * STB, j, lane);
  const int tl = t + 3 < nT ? t + 3 : nT - 1;
  io_load(R, A, r0 + (int64_t)tl * TR, h, j, lane);
#endif
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // tile t + 1's LDS writes are done before T_{t+1}
}

#ifndef NERF_BWD_IOSETS
#define NERF_BWD_IOSETS 2
#endif
// NERF_BWD_IOSETS == 3: three register sets, tile k in set k % 3; step t stores tile t + 1 and reloads its set with
// tile t + 4 (three tiles in flight while tile t is computed)
__device__ __forceinline__ void io_step3(IoSet& R, const LayerArgs& A, char* lds, int h, int j, int t, int nT,
                                         int64_t r0, int lane, float (&bs)[8]) {
  raw_barrier();
  if (h == 0 && t + 1 < nT) bias_acc(R, bs);
  io_store(R, lds + ((t + 1) % NSTG) * STB, j, lane);
  const int tl = t + 4 < nT ? t + 4 : nT - 1;
  io_load(R, A, r0 + (int64_t)tl * TR, h, j, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

__device__ __forceinline__ void bwd_io(const LayerArgs& A, char* lds, int h, int j, int nT, int64_t r0, int lane,
                                       float (&bs)[8]) {
  if (nT == 0) return;
#if NERF_BWD_IOSETS == 3
  {
    IoSet R0, R1, R2;
    io_load(R0, A, r0, h, j, lane);
    io_load(R1, A, r0 + (int64_t)(nT > 1 ? 1 : nT - 1) * TR, h, j, lane);
    io_load(R2, A, r0 + (int64_t)(nT > 2 ? 2 : nT - 1) * TR, h, j, lane);
    if (h == 0) bias_acc(R0, bs);
    io_store(R0, lds, j, lane);
    io_load(R0, A, r0 + (int64_t)(nT > 3 ? 3 : nT - 1) * TR, h, j, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    int t = 0;
    for (; t + 2 < nT; t += 3) {
      io_step3(R1, A, lds, h, j, t, nT, r0, lane, bs);
      io_step3(R2, A, lds, h, j, t + 1, nT, r0, lane, bs);
      io_step3(R0, A, lds, h, j, t + 2, nT, r0, lane, bs);
    }
    if (t < nT) io_step3(R1, A, lds, h, j, t, nT, r0, lane, bs);
    if (t + 1 < nT) io_step3(R2, A, lds, h, j, t + 1, nT, r0, lane, bs);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    return;
  }
#endif
  IoSet R0, R1;
  io_load(R0, A, r0, h, j, lane);
  io_load(R1, A, r0 + (int64_t)(nT > 1 ? 1 : 0) * TR, h, j, lane);
  if (h == 0) bias_acc(R0, bs);
  io_store(R0, lds, j, lane);
  io_load(R0, A, r0 + (int64_t)(nT > 2 ? 2 : nT - 1) * TR, h, j, lane);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int t = 0;
  for (; t + 1 < nT; t += 2) {
    io_step(R1, A, lds, h, j, t, nT, r0, lane, bs);
    io_step(R0, A, lds, h, j, t + 1, nT, r0, lane, bs);
  }
  if (t < nT) io_step(R1, A, lds, h, j, t, nT, r0, lane, bs);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's redundant loads land before the wave retires
}

__global__ __launch_bounds__(768, 3) void bwd_layer_bf16_kernel(LayerArgs A) {
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];
  const int b = blockIdx.x;
  const int h = (b >> 3) & 1;
  const int s = (b >> 4) * 8 + (b & 7);
  if (s >= A.S) return;  // whole workgroup: no barrier is left waiting
  const int64_t r0 = (int64_t)s * A.rps;
  int64_t r1 = r0 + A.rps;
  if (r1 > A.Mp) r1 = A.Mp;
  const int nT = r1 > r0 ? (int)((r1 - r0) / TR) : 0;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  load_wt(A, lds, h, (int)threadIdx.x);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // W^T in LDS before T_0 (the loop's first barrier)
  float bs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (w >= 8)
    bwd_io(A, lds, h, w - 8, nT, r0, lane, bs);
  else
    bwd_compute(A, lds, s, h, w, nT, r0, lane);
  if (h == 0) {  // bias gradient: parities by shuffle, the io waves' partials through LDS (stage 0 is free now)
    raw_barrier();
    float* part = reinterpret_cast<float*>(lds);
    if (w >= 8) {
#pragma unroll
      for (int d = 0; d < 8; ++d) {
        const float v = bs[d] + __shfl_xor(bs[d], 32, 64);
        if (lane < 32) part[(w - 8) * 256 + 8 * lane + d] = v;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    if (w == 8) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int n = 64 * e + lane;
        A.Pb[(int64_t)s * A.slab + n] = ((part[n] + part[256 + n]) + part[512 + n]) + part[768 + n];
      }
    }
  }
}

}  // namespace nerf_bwd
}  // namespace NERF_H16NS
