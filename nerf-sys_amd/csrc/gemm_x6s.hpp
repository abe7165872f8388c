// Input-gradient split GEMM with the activation split SHARED by two column groups (A/B builds: NERF_X6_DG_SHARED).
//
// gemm_nt_x6w's input gradient (BIGSMALL, 32-row waves, 256 x 128 tiles) splits every row of dZ once per 128-column
// tile, i.e. twice per layer, and its two accumulator sets leave no registers for 32 x 256 waves (measured at one
// wave per SIMD: slower, profiles/r05/x6_variants_ab.txt).  Here a 512-thread workgroup owns 128 rows x 256 columns:
// wave w computes rows 32 (w & 3) .. + 31 of column half w >> 2 (32 x 128, the same 4 MFMA tiles and two accumulator
// sets as gemm_nt_x6w's input gradient), and splits only ONE of each slab's two 16-deep k-steps of its rows — k-step
// w >> 2 — into a swizzled LDS image of the three pieces, which both column halves read.  So each activation value is
// split once per layer; the price is the piece image (24 KiB per slab buffer) and three ds_read_b128 per k-step for
// the A fragments.  Every accumulator sees the same MFMA sequence as in gemm_nt_x6w (k-step order, six terms in
// X6_PA / X6_PB order, small terms in their own accumulators): the outputs are bitwise the same.
//
// Pipeline (K = NKC 32-deep slabs, fully unrolled): raw activations of slab s land in register set s & 1 two slabs
// ahead; at slab kt a wave splits slab kt + 1 into piece buffer (kt + 1) & 1 and DMAs weight slab kt + 1 into weight
// buffer (kt + 1) & 1 (global_load_lds_dwordx4, as gemm_nt_x6w), then runs slab kt's MFMAs from buffers kt & 1; one
// barrier per slab publishes both.  Requirements (host): M % 128 == 0, N == 256, K == 32 NKC, lda % 4 == 0.
#pragma once
#include "gemm_x6.hpp"

template <int EPI, int NKC>
__global__ __launch_bounds__(512, 1) void gemm_nt_x6s_kernel(const float* __restrict__ A, int lda,
                                                            const nerf_bf16* __restrict__ Bp, int ldb, int64_t bplane,
                                                            float* __restrict__ C, int ldc,
                                                            const uint32_t* __restrict__ mbits, int ldmb) {
  constexpr int NW = 8, BK = 32, KS = 2, BN = 256, TN = 4, LS = 32;
  constexpr int PL = BN * LS;        // one weight piece image [256][32] bf16
  constexpr int PA = 128 * LS;       // one activation piece image [128][32] bf16
  constexpr int GPP = BN * BK * 2 / 1024, GPW = 3 * GPP / NW;  // 1-KiB DMA groups per weight piece / per wave
  static_assert((3 * GPP) % NW == 0, "weight DMA groups");
  static_assert(NW * X6E_WAVE_FLOATS * 2 <= 2 * 3 * PL, "epilogue tiles fit in the weight images");
  __shared__ __attribute__((aligned(16))) nerf_bf16 smem[2 * 3 * PL];  // weight images, then the epilogue tiles
  __shared__ __attribute__((aligned(16))) nerf_bf16 apc[2 * 3 * PA];   // activation piece images
  auto sw = [](int r, int q) { return q ^ ((r >> 2) & 3); };

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t m0 = (int64_t)tile * 128;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 31, lh = lane >> 5;
  const int rb = wave & 3, ch = wave >> 2;  // row block, column half (= the k-step of each slab this wave splits)
  const int ar = 32 * rb + li;              // this lane's row in the tile
  // raw activations of a slab: row ar, k = 32 kt + 16 ch + 8 lh .. + 7 (two float4)
  const float* Ar = A + (m0 + ar) * lda + 16 * ch + 8 * lh;
  const int wave_u = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t gofs = (uint32_t)((((lane >> 2) * ldb) + 8 * ((lane & 3) ^ ((lane >> 4) & 3))) * 2);
  const uint32_t smem_u32 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;

  float4 ra[2][2];
  auto aload = [&](int set, int kt) __attribute__((always_inline)) {
    ra[set][0] = *reinterpret_cast<const float4*>(Ar + BK * kt);
    ra[set][1] = *reinterpret_cast<const float4*>(Ar + BK * kt + 4);
  };
  auto touch = [&](int set) __attribute__((always_inline)) {
    asm volatile("" ::"v"(__builtin_bit_cast(x6_f32x4, ra[set][0])), "v"(__builtin_bit_cast(x6_f32x4, ra[set][1]))
                 : "memory");
  };
  auto bdma = [&](int kt, int buf) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < GPW; ++i) {
      const int g_ = wave_u + NW * i, p_ = g_ / GPP, rb_ = (g_ % GPP) * 16;
      const nerf_bf16* sb_ = Bp + p_ * bplane + (int64_t)rb_ * ldb + BK * kt;
      const uint32_t dst_ = smem_u32 + (uint32_t)(((buf * 3 + p_) * PL + rb_ * LS) * 2);
      unsigned keep_;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\t"
                   "s_mov_b32 m0, %0" : "=&s"(keep_) : "v"(gofs), "s"(sb_), "s"(dst_) : "memory");
    }
  };
  // split the raw set into the three piece images of buffer buf: row ar, 16-B chunk 2 ch + lh
  auto split_store = [&](int set, int buf) __attribute__((always_inline)) {
    uint2 h0, m0_, l0, h1, m1, l1;
    x6_split4(ra[set][0], h0, m0_, l0);
    x6_split4(ra[set][1], h1, m1, l1);
    const int o = ar * LS + 8 * sw(ar, 2 * ch + lh);
    *reinterpret_cast<uint4*>(apc + (buf * 3 + 0) * PA + o) = make_uint4(h0.x, h0.y, h1.x, h1.y);
    *reinterpret_cast<uint4*>(apc + (buf * 3 + 1) * PA + o) = make_uint4(m0_.x, m0_.y, m1.x, m1.y);
    *reinterpret_cast<uint4*>(apc + (buf * 3 + 2) * PA + o) = make_uint4(l0.x, l0.y, l1.x, l1.y);
  };

  nerf_f32x16 acc[TN], accs[TN];
#pragma unroll
  for (int b = 0; b < TN; ++b)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc[b][r] = 0.f;
      accs[b][r] = 0.f;
    }

  // prologue: raw slabs 0, 1; pieces of slab 0; weights of slab 0
  aload(0, 0);
  aload(1, NKC > 1 ? 1 : 0);
  touch(0);
  bdma(0, 0);
  split_store(0, 0);
  if (NKC > 2) aload(0, 2);
  asm volatile("" ::: "memory");
  if constexpr (NKC > 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // the DMA; slab 2's two loads in flight
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

#pragma unroll
  for (int kt = 0; kt < NKC; ++kt) {
    const int cur = kt & 1, nxt = cur ^ 1;
    const bool more = kt + 1 < NKC;  // compile time (unrolled)
    if (more) {
      touch(nxt);          // slab kt + 1's raw values have landed (the compiler waits for its own loads here)
      bdma(kt + 1, nxt);   // weight slab kt + 1
#ifndef NERF_X6S_LATE_SPLIT
      split_store(nxt, nxt);
      if (kt + 3 < NKC) aload(nxt, kt + 3);  // set nxt is free again: slab kt + 3 streams into it
#endif
      asm volatile("" ::: "memory");
    }
    // slab kt's MFMAs: A fragments from the piece image (row ar, chunk 2 ks + lh), B fragments as gemm_nt_x6w
    const nerf_bf16* S = smem + cur * 3 * PL;
    const nerf_bf16* P = apc + cur * 3 * PA;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#ifdef NERF_X6S_LATE_SPLIT  // A/B builds: the next slab's split between this slab's two k-steps (under the MFMAs)
      if (ks == 1 && more) {
        split_store(nxt, nxt);
        if (kt + 3 < NKC) aload(nxt, kt + 3);
        asm volatile("" ::: "memory");
      }
#endif
      nerf_bf16x8 af[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        af[p] = *reinterpret_cast<const nerf_bf16x8*>(P + p * PA + ar * LS + 8 * sw(ar, 2 * ks + lh));
#pragma unroll
      for (int bp = 0; bp < TN / 2; ++bp) {
        nerf_bf16x8 bf[2][3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            const int row = 128 * ch + (2 * bp + b) * 32 + li;
            bf[b][p] = *reinterpret_cast<const nerf_bf16x8*>(S + p * PL + row * LS + 8 * sw(row, 2 * ks + lh));
          }
#pragma unroll
        for (int t = 0; t < 6; ++t)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (t < 5)
              accs[2 * bp + b] =
                  __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[b][X6_PB[t]], af[X6_PA[t]], accs[2 * bp + b], 0, 0, 0);
            else
              acc[2 * bp + b] =
                  __builtin_amdgcn_mfma_f32_32x32x16_bf16(bf[b][X6_PB[t]], af[X6_PA[t]], acc[2 * bp + b], 0, 0, 0);
          }
      }
    }
    if (more) {
      // weight slab kt + 1 done (slab kt + 3's two loads, issued after it, may stay in flight); piece writes done
      if (kt + 3 < NKC) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave is done with the weight images before they become epilogue tiles
  nerf_f32x16 accw[1][TN];
#pragma unroll
  for (int b = 0; b < TN; ++b) accw[0][b] = acc[b] + accs[b];
  x6_epilogue_lds<1, TN, EPI>(accw, m0 + 32 * rb, 128 * ch, lane, nullptr, C, ldc, mbits, ldmb, nullptr,
                               reinterpret_cast<float*>(smem) + wave * X6E_WAVE_FLOATS);
}
