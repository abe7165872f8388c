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
// stream is then read from HBM once and hit in L2 by the partner — speed only, never correctness).
// Workgroup = 12 waves (3 per SIMD, <= 168 VGPRs each):
//   compute waves c = 0..7 own input-column block kb = 4 h + (c & 3) (32 columns) and half mh = c >> 2:
//     wgrad  acc[j] (j = 0..3) = dW[32 (4 mh + j)..][32 kb..]: 4 x v_mfma_f32_32x32x16_bf16 accumulators (64 VGPRs),
//            A = G^T, B = X^T fragments by ds_read_b64_tr_b16 (transposing reads, gfx950);
//     dgrad  dX[rows 32 mh..][32 kb..] = G W_i[:, kb]: 1 accumulator, A = W_i^T fragments streamed from L2 (a
//            fragment-major image, one contiguous KiB per wave-load) through a 4-deep register ring, B = G row fragments;
//     epilogue: ReLU mask from the X tile in LDS, bf16, 16-B stores of D.
//   io waves j = 0..3 (waves 8..11) move the tiles HBM -> LDS by LDS-DMA (global_load_lds_dwordx4): a compute wave then holds
//     only L2-latency loads in its in-order vmcnt queue (a wait on a weight fragment never waits for HBM).
// Tiles of 64 rows: G [64][256] (32 KiB) + X half [64][128] (16 KiB) per stage, 3 stages (144 KiB) -> two tiles in
// flight while one is computed; one workgroup barrier per tile.
// LDS images are unpadded and XOR-swizzled per 16-B chunk: chunk c of row r sits at slot c ^ swz(r),
// swz(r) = 4 (r & 3) + ((r >> 2) & 3).  Conflict-free for all three access shapes: a ds_read_b128 lane group (16
// rows, one chunk: 16 distinct swz), a ds_read_b64_tr_b16 half-wave (4 rows r0..r0+3, r0 % 4 == 0, x 4 aligned
// chunks: slot = (c ^ 4 q) + (p ^ k) -> 16 distinct slots) and the epilogue's mask reads (as the first).  The DMA
// writes lane-linear 1-KiB pieces, so the permutation is applied to the SOURCE address.
//
// MFMA order: the weight-gradient k-steps walk the split's rows 16 at a time in row order and the input gradient
// contracts n in 16-wide steps in order, exactly as gemm_wgrad_bf16 / gemm_nt_bf16_wsr do: the result is bitwise
// the layered path's.
#pragma once
#include <type_traits>

#include "gemm_bf16.hpp"
#include "mlp_common.hpp"

namespace nerf_bwd {

constexpr int TR = 64;                  // rows per tile
constexpr int GBY = TR * 512;           // G tile bytes (64 rows x 256 bf16)
constexpr int XBY = TR * 256;           // X half tile bytes (64 rows x 128 bf16)
constexpr int STB = GBY + XBY;          // 48 KiB per stage
constexpr int NSTG = 3;
constexpr int FRAG_LAYER = 8 * 16 * 64 * 8;  // bf16 elements of one layer's W^T fragment image (128 KiB)

__device__ __forceinline__ int swz(int r) { return 4 * (r & 3) + ((r >> 2) & 3); }

// W_i^T fragment image of trunk layers i = 1..7 (image i - 1): fragment (kb, ks), lane l, element j holds
// W_i[n = 16 ks + 8 (l >> 5) + j][k = 32 kb + (l & 31)] (bf16) — the A operand of dX^T = W^T G^T; for trunk.4 only
// the first 256 input columns (the trunk.3 output; the encoding columns need no input gradient).
struct WTSrc {
  int64_t off[7];  // fp32 offset of W_i (i = 1..7) in the packed layout
  int ld[7];       // its row pitch (KPAD[i])
};
__global__ void wt_frag_pack_kernel(const float* __restrict__ w, nerf_bf16* __restrict__ wf, WTSrc S) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // 16-B chunk index
  if (c >= 7 * FRAG_LAYER / 8) return;
  const int img = (int)(c / (FRAG_LAYER / 8));
  const int r = (int)(c - (int64_t)img * (FRAG_LAYER / 8));
  const int lane = r & 63, ks = (r >> 6) & 15, kb = r >> 10;
  const float* src = w + S.off[img] + (int64_t)(16 * ks + 8 * (lane >> 5)) * S.ld[img] + 32 * kb + (lane & 31);
  float v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = src[(int64_t)j * S.ld[img]];
  *reinterpret_cast<uint4*>(wf + c * 8) = make_uint4(nerf_pack_bf16x2(v[0], v[1]), nerf_pack_bf16x2(v[2], v[3]),
                                                     nerf_pack_bf16x2(v[4], v[5]), nerf_pack_bf16x2(v[6], v[7]));
}

typedef unsigned int nerf_bwd_u32x4 __attribute__((ext_vector_type(4)));

struct LayerArgs {
  const nerf_bf16* G;    // dZ_i [Mp][256]
  const nerf_bf16* X;    // X_i, row pitch ldx (cols 0..255 used)
  const nerf_bf16* WTf;  // this layer's W^T fragment image (FRAG_LAYER bf16)
  nerf_bf16* D;          // dZ_{i-1} [Mp][256]
  float* P;              // weight-gradient slab 0 of this tensor (row pitch ldp)
  float* Pb;             // bias-gradient slab 0
  int64_t slab;          // floats between consecutive splits' slabs
  int64_t rps, Mp;       // rows per split (multiple of 64), padded rows (multiple of 256)
  int ldx, ldp, S;
};

// io wave j: DMA pieces of tile t (rows m0 .. m0 + 63) into stage st: G pieces 8 j .. 8 j + 7 (2 rows each), X-half
// pieces 4 j .. 4 j + 3 (4 rows each); lane L of a piece writes LDS slot L, so it fetches the chunk that the swizzle
// puts there.
__device__ __forceinline__ void io_issue(const LayerArgs& A, char* st, int64_t m0, int h, int j, int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = 8 * j + i;
    const int row = 2 * p + (lane >> 5);
    const int c = (lane & 31) ^ swz(row);
    const nerf_bf16* src = A.G + (m0 + row) * 256 + 8 * c;
    __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(st + p * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = 4 * j + i;
    const int row = 4 * p + (lane >> 4);
    const int c = (lane & 15) ^ swz(row);
    const nerf_bf16* src = A.X + (m0 + row) * (int64_t)A.ldx + 128 * h + 8 * c;
    __builtin_amdgcn_global_load_lds((const void*)src,
                                     (__attribute__((address_space(3))) void*)(st + GBY + p * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ nerf_bf16x8 tr_frag(const char* base, int o0, int o1) {
  typedef __attribute__((address_space(3))) nerf_s16x4 lds_s16x4;
  const nerf_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + o0));
  const nerf_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + o1));
  const short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(nerf_bf16x8, v8);
}

// inline-asm LDS reads (byte address + immediate offset); the caller waits lgkmcnt before the use
template <int OFF>
__device__ __forceinline__ nerf_bf16x8 tr_frag_asm(uint32_t a0, uint32_t a1) {
  nerf_s16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a0), "i"(OFF) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "i"(OFF) : "memory");
  const short v8 __attribute__((ext_vector_type(8))) = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(nerf_bf16x8, v8);
}
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}
__device__ __forceinline__ nerf_bf16x8 lds_b128(uint32_t a) {
  nerf_bf16x8 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
  return v;
}

typedef unsigned short nerf_u16x2b __attribute__((ext_vector_type(2)));
// keep the bf16 pair v where the matching bf16 of x is nonzero (x is post-ReLU: +0 / -0 both count as zero)
__device__ __forceinline__ uint32_t relu_mask2(uint32_t v, uint32_t x) {
  const nerf_u16x2b nz = __builtin_elementwise_min(__builtin_bit_cast(nerf_u16x2b, x & 0x7fff7fffu), nerf_u16x2b{1, 1});
  const nerf_u16x2b m = nerf_u16x2b{0, 0} - nz;
  return v & __builtin_bit_cast(uint32_t, m);
}

// raw workgroup barrier: __syncthreads() carries a workgroup fence, and the io waves' outstanding LDS-DMA would make
// that fence wait for vmcnt(0) (draining the prefetch); the empty asm statements keep memory operations from being
// moved across it at the IR level, the sched_barriers at the machine level
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
}
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

__device__ __forceinline__ void bwd_compute(const LayerArgs& A, const char* lds, int s, int h, int c, int nT,
                                            int64_t r0, int lane) {
  const int li = lane & 31, lh = lane >> 5;
  const int kl = c & 3, mh = c >> 2;  // local 32-column block, row half / n-block half
  const int kb = 4 * h + kl;          // global 32-column block of this wave
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)A.WTf, 0, FRAG_LAYER * 2, 0x00020000);
  auto wfrag = [&](int ks) {
    const nerf_bwd_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, lane * 16 + kb * 16 * 1024, ks * 1024, 0);
    return __builtin_bit_cast(nerf_bf16x8, v);
  };
  nerf_bf16x8 ring[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) ring[i] = wfrag(i);

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
  // row fragments of G (dgrad B operand) and the X mask reads: row 32 mh + li, chunk ch -> slot ch ^ swz(li)
  const int gs = swz(li);
  const int rowg = (32 * mh + li) * 512, rowx = GBY + (32 * mh + li) * 256;

  // The pipeline below is ordered by hand: LDS reads are inline asm with immediate offsets and counted lgkmcnt waits
  // (the ds_read_tr intrinsic got no offset folding: one address VGPR per read), each wait asm passes the fragments
  // it covers through "+v" so no MFMA can be hoisted above it, and sched_barrier fences keep the stages in order (the
  // default scheduler, minimising registers for 3 waves per SIMD, sank every weight-fragment load next to its MFMA).
  const uint32_t lbase = (uint32_t)(uintptr_t)lds;
  const int u = lh ^ gs;  // row-fragment chunk 2 ks + lh -> slot (2 ks) ^ u
  for (int t = 0; t < nT; ++t) {
    raw_barrier();  // tile t is in stage t % 3; every wave is done with tile t - 1
    const uint32_t Lb = lbase + (uint32_t)((t % NSTG) * STB);
    uint32_t gat[2][4], xat[2];
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      xat[tt] = Lb + xa[tt];
#pragma unroll
      for (int j = 0; j < 4; ++j) gat[tt][j] = Lb + ga[tt][j];
    }
    const uint32_t rg = Lb + rowg, rx = Lb + rowx;
    // ---- weight gradient: 4 k-steps of 16 rows, fragments of k-step ks + 1 read under the MFMAs of ks (10 reads)
    nerf_bf16x8 xf[2], gf[2][4];
    auto wg_reads = [&](auto KS, int b) {
      constexpr int ks = decltype(KS)::value;
      xf[b] = tr_frag_asm<4096 * ks>(xat[0], xat[1]);
#pragma unroll
      for (int j = 0; j < 4; ++j) gf[b][j] = tr_frag_asm<8192 * ks>(gat[0][j], gat[1][j]);
    };
    nerf_bf16x8 gr[3];
    auto grow = [&](int ks) { return lds_b128(rg + 16 * ((2 * ks) ^ u)); };
    wg_reads(std::integral_constant<int, 0>{}, 0);
    static_for<0, 4>([&](auto KS) {
      constexpr int ks = decltype(KS)::value;
      constexpr int cb = ks & 1;
      if constexpr (ks + 1 < 4) {
        wg_reads(std::integral_constant<int, ks + 1>{}, cb ^ 1);
        asm volatile("s_waitcnt lgkmcnt(10)" : "+v"(xf[cb]), "+v"(gf[cb][0]), "+v"(gf[cb][1]), "+v"(gf[cb][2]),
                     "+v"(gf[cb][3])::"memory");
      } else {  // the input gradient's first two row fragments go out under the last weight-gradient MFMAs
        gr[0] = grow(0);
        gr[1] = grow(1);
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(xf[cb]), "+v"(gf[cb][0]), "+v"(gf[cb][1]), "+v"(gf[cb][2]),
                     "+v"(gf[cb][3])::"memory");
      }
      SCHED_FENCE();
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(gf[cb][j], xf[cb], acc[j], 0, 0, 0);
      SCHED_FENCE();
    });
    // ---- input gradient: dX^T[32 kb..][rows 32 mh..] over n in 16 k-steps; row fragments read 2 k-steps ahead,
    // weight fragments 4 k-steps ahead (the ring runs on into the next tile: W is the same for every tile)
    nerf_f32x16 dacc;
#pragma unroll
    for (int r = 0; r < 16; ++r) dacc[r] = 0.f;
    nerf_bf16x8 xm[2];
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) {
      const nerf_bf16x8 wf = ring[ks & 3];
      ring[ks & 3] = wfrag((ks + 4) & 15);
      nerf_bf16x8& g = gr[ks % 3];
      if (ks + 2 < 16) {
        gr[(ks + 2) % 3] = grow(ks + 2);
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(g)::"memory");
      } else if (ks == 14) {  // the epilogue's ReLU-mask chunks (local chunk 4 kl + 2 pr + lh of the X half)
#pragma unroll
        for (int pr = 0; pr < 2; ++pr) xm[pr] = lds_b128(rx + 16 * ((4 * kl + 2 * pr) ^ u));
        asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(g)::"memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(g)::"memory");
      }
      SCHED_FENCE();
      dacc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, g, dacc, 0, 0, 0);
      SCHED_FENCE();
    }
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
      *reinterpret_cast<uint4*>(Dt + 16 * pr) = o;
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

// io wave j: the DMA stream, plus (workgroup h = 0 only) the bias gradient Pb[n] = sum_m G[m][n] of columns
// n = 64 j + 32 e + (lane & 31), e = 0 / 1, from the G tile already in LDS: lane half lh sums the rows 16 ks + 8 lh + jj
// of every 16-row k-step in row order and the halves are added at the end — the summation order of gemm_wgrad_bf16's
// bias column sums (its G^T fragment of lane (li, lh) holds those 8 rows), so Pb is bitwise the layered path's.
__device__ __forceinline__ void bwd_io(const LayerArgs& A, char* lds, int s, int h, int j, int nT, int64_t r0, int lane) {
  const int lh = lane >> 5;
  float bs[2] = {0.f, 0.f};
  if (nT > 0) io_issue(A, lds, r0, h, j, lane);
  if (nT > 1) io_issue(A, lds + STB, r0 + TR, h, j, lane);
  for (int t = 0; t < nT; ++t) {
    if (t + 1 < nT)
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // tile t + 1's 12 pieces may stay in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier();  // tile t visible to every wave; every wave is done with tile t - 1 (stage (t + 2) % 3)
    if (t + 2 < nT) io_issue(A, lds + ((t + 2) % NSTG) * STB, r0 + (int64_t)(t + 2) * TR, h, j, lane);
    if (h == 0) {
      // tile t stays in its stage until the DMA issued after the NEXT barrier, which this wave only passes after these
      // reads.  Inline-asm LDS reads: a compiler-visible LDS read would be preceded by vmcnt(0) (the DMA in flight)
      const uint32_t Gs = (uint32_t)(uintptr_t)(lds + (t % NSTG) * STB);
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        uint32_t u[8][2];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
          const int row = 16 * ks + 8 * lh + jj;
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            const int n = 64 * j + 32 * e + (lane & 31);
            const uint32_t ad = Gs + row * 512 + 16 * ((n >> 3) ^ swz(row)) + 2 * (n & 7);
            asm volatile("ds_read_u16 %0, %1" : "=v"(u[jj][e]) : "v"(ad) : "memory");
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int jj = 0; jj < 8; ++jj)
#pragma unroll
          for (int e = 0; e < 2; ++e) bs[e] += __uint_as_float(u[jj][e] << 16);
      }
    }
  }
  if (h == 0) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float v = bs[e] + __shfl_xor(bs[e], 32, 64);
      if (lh == 0) A.Pb[(int64_t)s * A.slab + 64 * j + 32 * e + (lane & 31)] = v;
    }
  }
}

__global__ __launch_bounds__(768, 3) void bwd_layer_bf16_kernel(LayerArgs A) {
  __shared__ __attribute__((aligned(1024))) char lds[NSTG * STB];
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
  if (w >= 8)
    bwd_io(A, lds, s, h, w - 8, nT, r0, lane);
  else
    bwd_compute(A, lds, s, h, w, nT, r0, lane);
}

}  // namespace nerf_bwd
