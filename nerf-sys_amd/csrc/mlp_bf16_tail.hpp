// Fused bf16 backward of the MLP "tail" (BASELINE.json configs[2]; models/inr/meta_vanilla.py:109-154): everything
// between d_rgb_sigma and dZ7 (the gradient of the trunk.7 pre-activation) in ONE launch.  The layered path runs it as
// eight launches through HBM (head_out_bwd, colour_out dgrad + wgrad, colour layer 0 dgrad + wgrad, geo_bwd, head
// dgrad + wgrad: 1.2 ms per fine-net backward at the C2 size).  Per 64-row tile:
//   P0  dO3   = g.rgb * s(1-s) (bf16, cols 0..2),  ds = g.sigma * exp(clamp(sigma_raw))          (wave 0, lane = row)
//   P1  dC0   = (dO3 Wc1) * [C0 > 0]   -> LDS (bf16)                               MFMA, 8 waves x 2
//       dWc1 += dO3^T C0,  dbc1 += sum dO3                                          MFMA, waves 0-3 x 4
//   P2  dO16  = [ds | dC0 Wc0[:, :15] | 0]  -> LDS (bf16; the shifted Wc0 image puts dCIN col c at dO16 col c+1)
//                                                                                   MFMA, waves 0-1 x 8
//       dWc0 += dC0^T CIN,  dbc0 += sum dC0                                         MFMA, 8 waves x 4
//   P3  dZ7   = (dO16 Wh) * [Y7 > 0]   -> HBM (bf16)                               MFMA, 8 waves x 4
//       dWh  += dO16^T Y7,  dbh += sum dO16                                         MFMA, 8 waves x 4
// with the layered path's bf16 rounding points and MFMA k order, so dZ7 — and with it every trunk gradient — is
// bitwise the layered path's; the head / colour weight sums run over the two halves of each split (two workgroups,
// the second half's sums in partial2, added by reduce_splits2 after the slab terms): a fixed order, not the layered one.
// HBM per row: Y7 512 + CIN 128 + g / HO 32 B read, dZ7 512 B written (~1.2 KB; the chain moved
// ~3.6 KB).  Round 6: C0 (the colour layer-0 output, 256 B per row) is no longer written by the fused forward and read
// back here — each compute wave recomputes its 32 x 32 block of the tile's C0 from the CIN tile with the forward's
// fragments, bias-initialised accumulators, k order and ReLU / rounding (mlp_bf16_fused.hpp colour layer 0): bitwise
// the forward's C0, for 4 MFMAs per wave and tile.  Workgroup = 12 waves: 8 compute + 4 io waves that stage tiles
// through two register sets into two LDS stages (mlp_bf16_bwd.hpp's scheme).
#pragma once
#include "mlp_bf16_bwd.hpp"
#include "mlp_bf16_fused.hpp"

namespace NERF_H16NS {
namespace nerf_tail {
using nerf_bwd::raw_barrier;
using nerf_bwd::static_for;
using nerf_bwd::swz;
typedef nerf_bwd::io_u32x4 u32x4;

constexpr int TR = 64;
// stage (bytes): Y7 [64][256] bf16 | C0 [64][128] (written by the compute waves) | CIN [64][64] | g [64] float4 |
// O3 cols 0..3 [64] float4 | sraw [64]
constexpr int Y_OFF = 0, C_OFF = 64 * 512, I_OFF = C_OFF + 64 * 256, G_OFF = I_OFF + 64 * 128;
constexpr int O_OFF = G_OFF + 1024, S_OFF = O_OFF + 1024, STB = S_OFF + 256;
constexpr int NSTG = 2;
// work area: dO3 [64][32] bf16 | dO16 [64][32] bf16 | dC0 [64][128] bf16 | ds [64] f32 | shifted Wc0^T fragments (8 KiB)
constexpr int D3_OFF = NSTG * STB, D16_OFF = D3_OFF + 4096, DC_OFF = D16_OFF + 4096, DS_OFF = DC_OFF + 16384;
// (fp16 build: + the sigma head's weight row as fp16, WS_OFF, 512 B)
constexpr int WC0_OFF = DS_OFF + 256, WS_OFF = WC0_OFF + 8192, LDS_BYTES = WS_OFF + (NERF_F16 ? 512 : 0);
static_assert(LDS_BYTES <= 163840, "LDS");

__device__ __forceinline__ int swz8(int r) { return 4 * ((r >> 1) & 1); }  // CIN rows (8 chunks): tr reads only
__device__ __forceinline__ int swz4(int r) { return (r >> 2) & 3; }        // dO3 / dO16 rows (4 chunks)
__device__ __forceinline__ int ay(int r, int c) { return Y_OFF + r * 512 + 16 * (c ^ swz(r)); }
__device__ __forceinline__ int ac(int r, int c) { return C_OFF + r * 256 + 16 * (c ^ swz(r)); }
__device__ __forceinline__ int ai(int r, int c) { return I_OFF + r * 128 + 16 * (c ^ swz8(r)); }
__device__ __forceinline__ int a3(int r, int c) { return D3_OFF + r * 64 + 16 * (c ^ swz4(r)); }
__device__ __forceinline__ int a16(int r, int c) { return D16_OFF + r * 64 + 16 * (c ^ swz4(r)); }
__device__ __forceinline__ int adc(int r, int c) { return DC_OFF + r * 256 + 16 * (c ^ swz(r)); }

struct TailArgs {
  const float* w;      // fp32 packed parameters
  const float* g;      // d_rgb_sigma [M][4]
  const float* HO;     // [Mp][4] colour-out pre-activations 0..2, sigma_raw (the fused forward's dense row)
  const nerf_bf16* Y7; // trunk.7 output [Mp][256]
  const nerf_bf16* CIN;// colour input [Mp][64]
  const nerf_bf16* wfc0;// colour layer 0's fragment image (frag_pack_kernel, tensor 9: 128 x 64, 2 x 4 fragments)
  nerf_bf16* dZ7;      // [Mp][256]
  float* partial;      // slab s of the packed gradient (split s, first half)
  float* partial2;     // [S][cslab] second halves: packed offsets off16 .. total
  int64_t slab, cslab, rps, M, Mp;
  int64_t off16, off17, off18, off19, off20, off21;  // head W / b, colour0 W / b, colour_out W / b
  int S;
};

// transposing-read fragments (A = G^T or B = X^T of a weight gradient; lane geometry as gemm_wgrad_bf16) by inline asm:
// two per-lane base addresses (rows +0 / +4 of k-step 0) and the k-step as an immediate offset (the intrinsic got no
// offset folding: one address VGPR per read, which spilled here); the caller waits lgkmcnt(0) and passes the
// fragments through "+v" before the MFMAs
template <typename AD>
__device__ __forceinline__ void tr_bases(uint32_t base, AD ad, int cb, int lane, uint32_t& b0, uint32_t& b1) {
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int r = 8 * (grp >> 1) + q, c = 4 * cb + 2 * (grp & 1) + (p >> 1);
  b0 = base + (uint32_t)(ad(r, c) + 8 * (p & 1));
  b1 = base + (uint32_t)(ad(r + 4, c) + 8 * (p & 1));
}
__device__ __forceinline__ nerf_bf16x8 ld16(const char* p) { return *reinterpret_cast<const nerf_bf16x8*>(p); }

// A-operand fragment of a weight matrix read from fp32 memory: element (i, kk) = src[kk * ld_k + i * ld_i] for lane row
// i = i0 + (lane & 31), kk = 16 ks + 8 (lane >> 5) + j; bf16 round-to-nearest-even like the layered path's transposes
__device__ __forceinline__ nerf_bf16x8 wfrag(const float* src, int ld_k, int ld_i, int i0, int ks, int lane) {
  nerf_bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) H16_SET(v, j, src[(int64_t)(16 * ks + 8 * (lane >> 5) + j) * ld_k + (int64_t)(i0 + (lane & 31)) * ld_i]);
  return v;
}

// C^T accumulator (lane li = row, register 4 q + e = column 8 q + 4 lh + e) -> bf16, paired so that lane (li, lh) holds
// columns 16 pr + 8 lh .. + 7 of the 32-column block in out[pr] (gemm_bf16.hpp epilogue)
__device__ __forceinline__ void pack_pairs(const nerf_f32x16& a, uint4 (&out)[2]) {
  uint2 pk[4];
#pragma unroll
  for (int qq = 0; qq < 4; ++qq)
    pk[qq] = make_uint2(nerf_pack_bf16x2(a[4 * qq], a[4 * qq + 1]), nerf_pack_bf16x2(a[4 * qq + 2], a[4 * qq + 3]));
#pragma unroll
  for (int pr = 0; pr < 2; ++pr) {
    uint2 x = pk[2 * pr], y = pk[2 * pr + 1];
    const auto s0 = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
    const auto s1 = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
    out[pr] = make_uint4(s0[0], s1[0], s0[1], s1[1]);
  }
}
__device__ __forceinline__ uint4 mask4(uint4 v, uint4 x) {
  return make_uint4(nerf_bwd::relu_mask2(v.x, x.x), nerf_bwd::relu_mask2(v.y, x.y), nerf_bwd::relu_mask2(v.z, x.z),
                    nerf_bwd::relu_mask2(v.w, x.w));
}
__device__ __forceinline__ void wait_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

__device__ __forceinline__ void tail_compute(const TailArgs& A, char* lds, float* P, int w, int nT, int64_t r0,
                                             int lane) {
  const int li = lane & 31, lh = lane >> 5;
  const float* W = A.w;
  // register-resident weight fragments: colour_out^T for dC0 (cols 32 (w & 3)..), head^T for dZ7 (cols 32 w..)
  nerf_bf16x8 wc1[2], wh[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    wc1[ks] = wfrag(W + A.off20, 128, 1, 32 * (w & 3), ks, lane);  // A[i = C0 col][kk = dO3 col] = Wc1[kk][i]
    wh[ks] = wfrag(W + A.off16, 256, 1, 32 * w, ks, lane);        // A[i = Y7 col][kk = dO16 col] = Wh[kk][i]
  }

  if constexpr (NERF_F16)  // geo only: the sigma row (kk = 0: k-step 0, lane half 0, element 0) is added apart
    if (lh == 0) H16_SET(wh[0], 0, 0.f);
  nerf_f32x16 ac1, ac0, ahd;  // dWc1 (waves 0-3: k-block w), dWc0 (n-block w >> 1, k-block w & 1), dWh (k-block w)
#pragma unroll
  for (int r = 0; r < 16; ++r) ac1[r] = ac0[r] = ahd[r] = 0.f;
  float b1 = 0.f, b0 = 0.f, bh = 0.f;
  // fp16 build: the sigma-head and colour-out bias gradients are sums of the fp32 pre-activation gradients (the bias
  // add is fp32 in the reference, metamodule.py:153-155; only the matmul's operand is fp16), kept by wave 0 in P0
  float fa = 0.f, fb = 0.f, fc = 0.f, fs = 0.f;
  // transposing-read bases (k-step 0): work tiles absolute, stage tiles relative to the stage (+ Lo per tile)
  const uint32_t lb = (uint32_t)(uintptr_t)lds;
  uint32_t t3a0, t3a1, tca0, tca1, tda0, tda1, tia0, tia1, t16a0, t16a1, tya0, tya1;
  tr_bases(lb, a3, 0, lane, t3a0, t3a1);
  tr_bases(lb, ac, w & 3, lane, tca0, tca1);
  tr_bases(lb, adc, w >> 1, lane, tda0, tda1);
  tr_bases(lb, ai, w & 1, lane, tia0, tia1);
  tr_bases(lb, a16, 0, lane, t16a0, t16a1);
  tr_bases(lb, ay, w, lane, tya0, tya1);

  for (int t = 0; t < nT; ++t) {
    raw_barrier();  // T_t
    const char* L = lds + (t % NSTG) * STB;
    const uint32_t Lo = (uint32_t)((t % NSTG) * STB);
    // ---- C0 of the tile (rows 32 (w >> 2).., cols 32 (w & 3)..) from its CIN rows: the fused forward's colour layer 0
    // (acc_bias, 4 k-steps in order, relu_pk_out, the lane-half pairing of relu_to_lds) -> the stage's C0 slot
    {
      const int cb = w & 3, row = 32 * (w >> 2) + li;
      // the weights: A[i = C0 col 32 cb + i][kk = CIN col] = Wc0[col][kk], fragment (nb = cb, ks) of the fused forward's
      // image of colour layer 0 (frag_pack_kernel: ((nb * 4 + ks) * 64 + lane) * 8), loaded per tile from uniform bases
      // laundered per tile (hoisted out of the tile loop, the fragments and the bias held 32 VGPRs across it: the
      // compute waves sit at 166 of 168 without them)
      uint64_t wp_ = (uint64_t)(uintptr_t)A.wfc0, bp_ = (uint64_t)(uintptr_t)(W + A.off19);
      asm volatile("" : "+s"(wp_), "+s"(bp_));
      const nerf_bf16* wcp = reinterpret_cast<const nerf_bf16*>(wp_) + ((int64_t)cb * 256 + lane) * 8;
      const float* bc0 = reinterpret_cast<const float*>(bp_);
      nerf_f32x16 c;
      nerf_fused::acc_bias(c, bc0, 32 * cb, lh);
#pragma unroll
      for (int k2 = 0; k2 < 4; k2 += 2) {  // two fragments in flight at a time (register pressure: 168 VGPRs)
        const nerf_bf16x8 wa = *reinterpret_cast<const nerf_bf16x8*>(wcp + k2 * 64 * 8);
        const nerf_bf16x8 wb = *reinterpret_cast<const nerf_bf16x8*>(wcp + (k2 + 1) * 64 * 8);
        c = h16_mfma(wa, ld16(L + ai(row, 2 * k2 + lh)), c);
        c = h16_mfma(wb, ld16(L + ai(row, 2 * k2 + 2 + lh)), c);
      }
      uint2 pk[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float4 b4 = make_float4(0.f, 0.f, 0.f, 0.f);
        if constexpr (H16_BIAS_AFTER) b4 = *reinterpret_cast<const float4*>(bc0 + 32 * cb + 8 * q + 4 * lh);
        pk[q] = make_uint2(nerf_fused::relu_pk_out(c[4 * q], c[4 * q + 1], b4.x, b4.y),
                           nerf_fused::relu_pk_out(c[4 * q + 2], c[4 * q + 3], b4.z, b4.w));
      }
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        uint2 x = pk[2 * pr], y = pk[2 * pr + 1];
        const auto r0_ = __builtin_amdgcn_permlane32_swap(x.x, y.x, false, false);
        const auto r1_ = __builtin_amdgcn_permlane32_swap(x.y, y.y, false, false);
        *reinterpret_cast<uint4*>(lds + (t % NSTG) * STB + ac(row, 4 * cb + 2 * pr + lh)) =
            make_uint4(r0_[0], r1_[0], r0_[1], r1_[1]);
      }
    }
    // ---- P0: head-output derivatives of the tile's rows (wave 0, lane = row)
    if (w == 0) {
      const int64_t m = r0 + (int64_t)t * TR + lane;
      const float4 g = *reinterpret_cast<const float4*>(L + G_OFF + 16 * lane);
      const float4 o = *reinterpret_cast<const float4*>(L + O_OFF + 16 * lane);
      const float sr = *reinterpret_cast<const float*>(L + S_OFF + 4 * lane);
      float a = 0.f, b = 0.f, c = 0.f, ds = 0.f;
      if (m < A.M) {  // trunc_exp' / sigmoid' (mlp_bf16.hip head_out_bwd_bf16_kernel)
        const float s0 = nerf_mlp::sigmoidf_(o.x), s1 = nerf_mlp::sigmoidf_(o.y), s2 = nerf_mlp::sigmoidf_(o.z);
        a = g.x * (s0 * (1.0f - s0));
        b = g.y * (s1 * (1.0f - s1));
        c = g.z * (s2 * (1.0f - s2));
        ds = g.w * expf(fminf(fmaxf(sr, -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
      }
      if constexpr (NERF_F16) {
        fa += a; fb += b; fc += c; fs += ds;
      }
      *reinterpret_cast<uint4*>(lds + a3(lane, 0)) = make_uint4(nerf_pack_bf16x2(a, b), nerf_pack_bf16x2(c, 0.f), 0u, 0u);
      *reinterpret_cast<float*>(lds + DS_OFF + 4 * lane) = ds;
    }
    wait_lds();
    raw_barrier();  // B1: dO3 / ds of the tile are in LDS
    // ---- P1: dC0 (wave w: C0 cols 32 (w & 3).., rows 32 (w >> 2)..) and the colour_out weight gradient
    {
      const int nb = w & 3, row = 32 * (w >> 2) + li;
      nerf_f32x16 d;
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) d = h16_mfma(wc1[ks], ld16(lds + a3(row, 2 * ks + lh)), d);
      uint4 o[2];
      pack_pairs(d, o);
#pragma unroll
      for (int pr = 0; pr < 2; ++pr) {
        const int ch = 4 * nb + 2 * pr + lh;
        *reinterpret_cast<uint4*>(lds + adc(row, ch)) = mask4(o[pr], *reinterpret_cast<const uint4*>(L + ac(row, ch)));
      }
    }
    if (w < 4) {
      nerf_bf16x8 ga[4], gb[4];
      static_for<0, 4>([&](auto KS) {
        constexpr int ks = decltype(KS)::value;
        ga[ks] = nerf_bwd::tr_frag_asm<1024 * ks>(t3a0, t3a1);
        gb[ks] = nerf_bwd::tr_frag_asm<4096 * ks>(tca0 + Lo, tca1 + Lo);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ga[0]), "+v"(ga[1]), "+v"(ga[2]), "+v"(ga[3]), "+v"(gb[0]), "+v"(gb[1]),
                   "+v"(gb[2]), "+v"(gb[3])::"memory");
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (w == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) b1 += H16_GET(ga[ks], j);
        }
        ac1 = h16_mfma(ga[ks], gb[ks], ac1);
      }
    }
    wait_lds();
    raw_barrier();  // B2: dC0 in LDS
    // ---- P2: dO16 = [ds | dCIN cols 0..14 | 0] (waves 0-1: rows 32 w..) and the colour layer-0 weight gradient
    if (w < 2) {
      const int row = 32 * w + li;
      nerf_f32x16 d;
#pragma unroll
      for (int r = 0; r < 16; ++r) d[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        d = h16_mfma(ld16(lds + WC0_OFF + ks * 1024 + 16 * lane), ld16(lds + adc(row, 2 * ks + lh)),
                                                    d);
      uint4 o[2];
      pack_pairs(d, o);
      uint4 v = o[0];  // dO16 cols 8 lh .. 8 lh + 7 (col 0 = ds)
      if (lh == 0) {
        const float ds = *reinterpret_cast<const float*>(lds + DS_OFF + 4 * row);
        v.x = (v.x & 0xffff0000u) | (uint32_t)__builtin_bit_cast(uint16_t, (nerf_bf16)ds);
      }
      *reinterpret_cast<uint4*>(lds + a16(row, lh)) = v;
    }
    {
      nerf_bf16x8 ga[4], gb[4];
      static_for<0, 4>([&](auto KS) {
        constexpr int ks = decltype(KS)::value;
        ga[ks] = nerf_bwd::tr_frag_asm<4096 * ks>(tda0, tda1);
        gb[ks] = nerf_bwd::tr_frag_asm<2048 * ks>(tia0 + Lo, tia1 + Lo);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ga[0]), "+v"(ga[1]), "+v"(ga[2]), "+v"(ga[3]), "+v"(gb[0]), "+v"(gb[1]),
                   "+v"(gb[2]), "+v"(gb[3])::"memory");
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if ((w & 1) == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) b0 += H16_GET(ga[ks], j);
        }
        ac0 = h16_mfma(ga[ks], gb[ks], ac0);
      }
    }
    wait_lds();
    raw_barrier();  // B3: dO16 in LDS
    // ---- P3: dZ7 (wave w: trunk.7 cols 32 w.., both row blocks) -> HBM, and the head weight gradient
    {
#pragma unroll
      for (int mb = 0; mb < 2; ++mb) {
        const int row = 32 * mb + li;
        nerf_f32x16 d;
#pragma unroll
        for (int r = 0; r < 16; ++r) d[r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) d = h16_mfma(wh[ks], ld16(lds + a16(row, 2 * ks + lh)), d);
        if constexpr (NERF_F16) {
          // the reference's h7 feeds two fp16 matmuls (sigma_head, geo_head): each input gradient is rounded to fp16,
          // the two are added in fp32 and the sum rounded again where it enters trunk.7's matmul backward.  wh has its
          // sigma row zeroed (geo only); the sigma part is the rank-1 product ds16 * Ws16 (exact in fp32), rounded
          const float ds16 = (float)(nerf_bf16)*reinterpret_cast<const float*>(lds + DS_OFF + 4 * row);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const uint2 wv = *reinterpret_cast<const uint2*>(lds + WS_OFF + 2 * (32 * w + 8 * q + 4 * lh));
            const float ws4[4] = {nerf_bf16_lo(wv.x), nerf_bf16_hi(wv.x), nerf_bf16_lo(wv.y), nerf_bf16_hi(wv.y)};
#pragma unroll
            for (int e = 0; e < 4; ++e)
              d[4 * q + e] = (float)(nerf_bf16)d[4 * q + e] + (float)(nerf_bf16)(ds16 * ws4[e]);
          }
        }
        uint4 o[2];
        pack_pairs(d, o);
        nerf_bf16* dst = A.dZ7 + (r0 + (int64_t)t * TR + row) * 256 + 32 * w + 8 * lh;
#pragma unroll
        for (int pr = 0; pr < 2; ++pr)
        {
          const uint4 v = mask4(o[pr], *reinterpret_cast<const uint4*>(L + ay(row, 4 * w + 2 * pr + lh)));
#ifdef NERF_EXP_BWD_NT
          __builtin_nontemporal_store(u32x4{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4*>(dst + 16 * pr));
#else
          *reinterpret_cast<uint4*>(dst + 16 * pr) = v;
#endif
        }
      }
      nerf_bf16x8 ga[4], gb[4];
      static_for<0, 4>([&](auto KS) {
        constexpr int ks = decltype(KS)::value;
        ga[ks] = nerf_bwd::tr_frag_asm<1024 * ks>(t16a0, t16a1);
        gb[ks] = nerf_bwd::tr_frag_asm<8192 * ks>(tya0 + Lo, tya1 + Lo);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(ga[0]), "+v"(ga[1]), "+v"(ga[2]), "+v"(ga[3]), "+v"(gb[0]), "+v"(gb[1]),
                   "+v"(gb[2]), "+v"(gb[3])::"memory");
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        if (w == 0) {
#pragma unroll
          for (int j = 0; j < 8; ++j) bh += H16_GET(ga[ks], j);
        }
        ahd = h16_mfma(ga[ks], gb[ks], ahd);
      }
    }
  }
  // ---- slabs (C^T accumulators: row n = 8 (r >> 2) + 4 lh + (r & 3) of the block, column = lane li)
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = 8 * (r >> 2) + 4 * lh + (r & 3);
    if (w < 4) P[A.off20 + (int64_t)n * 128 + 32 * w + li] = ac1[r];
    P[A.off18 + (int64_t)(32 * (w >> 1) + n) * 64 + 32 * (w & 1) + li] = ac0[r];
    P[A.off16 + (int64_t)n * 256 + 32 * w + li] = ahd[r];
  }
  b1 += __shfl_xor(b1, 32, 64);
  b0 += __shfl_xor(b0, 32, 64);
  bh += __shfl_xor(bh, 32, 64);
  if constexpr (NERF_F16) {
    if (w == 0) {
      fa = wave_sum(fa); fb = wave_sum(fb); fc = wave_sum(fc); fs = wave_sum(fs);
      if (li == 0) { b1 = fa; bh = fs; }
      if (li == 1) b1 = fb;
      if (li == 2) b1 = fc;
    }
  }
  if (lh == 0) {
    if (w == 0) {
      P[A.off21 + li] = b1;
      P[A.off17 + li] = bh;
    }
    if ((w & 1) == 0) P[A.off19 + 32 * (w >> 1) + li] = b0;
  }
}

// ---- io waves: two named register sets of one tile each (11 x 16 B per lane)
struct TailSet {
  u32x4 v0, v1, v2, v3, v4, v5, v6, v7, v8, v9, v10;
  template <int I>
  __device__ __forceinline__ u32x4& at() {
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
    else return v10;
  }
};
// io wave j, rows 16 j .. 16 j + 15 of the tile: Y7 (8 pieces of 2 rows), CIN (2 pieces of 8 rows); plus one per-row
// vector of all 64 rows: j = 0 g, j = 1 HO (O3 cols 0..2 + sigma_raw), j = 2 sigma_raw (HO col 3)
__device__ __forceinline__ void tail_load(TailSet& S, const TailArgs& A, int64_t m0, int j, int lane) {
  const nerf_bf16* y = A.Y7 + (m0 + 16 * j + (lane >> 5)) * 256 + 8 * (lane & 31);
  const nerf_bf16* x = A.CIN + (m0 + 16 * j + (lane >> 3)) * 64 + 8 * (lane & 7);
  static_for<0, 8>([&](auto I) { S.template at<decltype(I)::value>() = *reinterpret_cast<const u32x4*>(y + 512 * decltype(I)::value); });
  static_for<0, 2>([&](auto I) { S.template at<8 + decltype(I)::value>() = *reinterpret_cast<const u32x4*>(x + 512 * decltype(I)::value); });
  // one unconditional 16-B load per lane for every io wave (a conditional load left the compiler unable to count the
  // set's loads: it drained vmcnt(0) before the stores); g is [M][4]: rows past M read row M - 1 and are zeroed
  const int64_t m = m0 + lane;
  const float* pv = j == 0 ? A.g + (m < A.M ? m : A.M - 1) * 4 : A.HO + m * 4;
  S.v10 = *reinterpret_cast<const u32x4*>(pv);
  if (j == 0 && m >= A.M) S.v10 = u32x4{0u, 0u, 0u, 0u};
}
__device__ __forceinline__ void tail_store(TailSet& S, char* st, int j, int lane) {
  static_for<0, 8>([&](auto I) {
    constexpr int i = decltype(I)::value;
    *reinterpret_cast<u32x4*>(st + ay(16 * j + 2 * i + (lane >> 5), lane & 31)) = S.template at<i>();
  });
  static_for<0, 2>([&](auto I) {
    constexpr int i = decltype(I)::value;
    *reinterpret_cast<u32x4*>(st + ai(16 * j + 8 * i + (lane >> 3), lane & 7)) = S.template at<8 + i>();
  });
  if (j == 0) *reinterpret_cast<u32x4*>(st + G_OFF + 16 * lane) = S.v10;
  if (j == 1) *reinterpret_cast<u32x4*>(st + O_OFF + 16 * lane) = S.v10;
  if (j == 2) *reinterpret_cast<uint32_t*>(st + S_OFF + 4 * lane) = S.v10.w;
}
__device__ __forceinline__ void tail_step(TailSet& R, const TailArgs& A, char* lds, int j, int t, int nT, int64_t r0,
                                          int lane) {
  raw_barrier();  // T_t
  tail_store(R, lds + ((t + 1) % NSTG) * STB, j, lane);  // tile t + 1 (past the end: a stage nobody reads)
  const int tl = t + 3 < nT ? t + 3 : nT - 1;
  tail_load(R, A, r0 + (int64_t)tl * TR, j, lane);
  wait_lds();
  raw_barrier();  // B1
  raw_barrier();  // B2
  raw_barrier();  // B3
}
__device__ __forceinline__ void tail_io(const TailArgs& A, char* lds, int j, int nT, int64_t r0, int lane) {
  if (nT == 0) return;
  TailSet R0, R1;
  tail_load(R0, A, r0, j, lane);
  tail_load(R1, A, r0 + (int64_t)(nT > 1 ? 1 : 0) * TR, j, lane);
  tail_store(R0, lds, j, lane);
  tail_load(R0, A, r0 + (int64_t)(nT > 2 ? 2 : nT - 1) * TR, j, lane);
  wait_lds();
  int t = 0;
  for (; t + 1 < nT; t += 2) {
    tail_step(R1, A, lds, j, t, nT, r0, lane);
    tail_step(R0, A, lds, j, t + 1, nT, r0, lane);
  }
  if (t < nT) tail_step(R1, A, lds, j, t, nT, r0, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// grid = 2 S8 workgroups: split s = (b >> 4) * 8 + (b & 7), half h = (b >> 3) & 1 takes rows [s rps + h rph, ...)
__global__ __launch_bounds__(768, 3) void bwd_tail_bf16_kernel(TailArgs A) {
  __shared__ __attribute__((aligned(1024))) char lds[LDS_BYTES];
  const int b = blockIdx.x;
  const int h = (b >> 3) & 1;
  const int s = (b >> 4) * 8 + (b & 7);
  if (s >= A.S) return;
  const int64_t rph = ((A.rps / 2 + TR - 1) / TR) * TR;
  const int64_t r0 = (int64_t)s * A.rps + h * rph;
  int64_t r1 = h ? (int64_t)s * A.rps + A.rps : r0 + rph;
  if (r1 > A.Mp) r1 = A.Mp;
  const int nT = r1 > r0 ? (int)((r1 - r0) / TR) : 0;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // constant parts of the work tiles (dO3 chunks 1..3, dO16 chunks 2..3: zero columns) and the shifted colour layer-0
  // image for dO16: fragment ks, lane l holds A[i = l & 31][kk = 16 ks + 8 (l >> 5) + j] = Wc0[kk][i - 1] (i = 1..15)
  for (int i = tid; i < 64 * 5; i += 768) {
    const int r = i / 5, k = i % 5;
    const int off = k < 3 ? a3(r, 1 + k) : a16(r, k - 1);
    *reinterpret_cast<uint4*>(lds + off) = make_uint4(0u, 0u, 0u, 0u);
  }
  for (int i = tid; i < 8 * 64; i += 768) {
    const int ks = i >> 6, l = i & 63, col = l & 31;
    nerf_bf16x8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int kk = 16 * ks + 8 * (l >> 5) + j;
      H16_SET(v, j, (col >= 1 && col <= 15) ? A.w[A.off18 + (int64_t)kk * 64 + col - 1] : 0.f);
    }
    *reinterpret_cast<nerf_bf16x8*>(lds + WC0_OFF + ks * 1024 + 16 * l) = v;
  }
  if constexpr (NERF_F16)
    for (int i = tid; i < 256; i += 768) reinterpret_cast<nerf_bf16*>(lds + WS_OFF)[i] = (nerf_bf16)A.w[A.off16 + i];
  wait_lds();
  if (w >= 8) {
    tail_io(A, lds, w - 8, nT, r0, lane);
  } else {
    float* P = h ? A.partial2 + (int64_t)s * A.cslab - A.off16 : A.partial + (int64_t)s * A.slab;
    tail_compute(A, lds, P, w, nT, r0, lane);
  }
}

}  // namespace nerf_tail
}  // namespace NERF_H16NS
