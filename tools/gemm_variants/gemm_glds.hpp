// fp32 MFMA NT GEMM with LDS-DMA staging (gfx950 `global_load_lds_dwordx4`) and a multi-stage ring:
//   C[m][n] = epi( sum_k A[m][k] * B[n][k] )
//
// Why: the register-staged kernel of gemm.hpp has its next-slab global loads sunk by hipcc below the MFMA
// block and waited on at once (exposed L2/HBM latency every slab).  Here the loads for slab kt+STAGES-1
// are issued by the DMA engine right after the barrier that retires slab kt, and only a counted
// `s_waitcnt vmcnt(N)` (never 0 inside the loop) waits for slab kt+1 one iteration later.
//
// LDS image: per stage A [BM][16] then B [BN][16] fp32, rows of 64 B = four 16-B chunks.  DMA writes are
// lane-linear (lane L -> byte 16 L of its 1 KiB piece = row L/4, chunk slot L%4), so the bank swizzle
// lives in the per-lane SOURCE address: slot p of row r holds k-chunk p ^ ((r >> 2) & 3).  A reading lane
// (row = 32-aligned base + li, chunk c) then finds its chunk at slot c ^ ((li >> 2) & 3): within every
// 16-lane ds_read_b128 group the (li & 3, (li >> 2) & 3) pairs are distinct -> 16 distinct 16-B bank slots.
#pragma once
#include "../../nerf-sys_amd/csrc/gemm.hpp"

#define NERF_LDS __attribute__((address_space(3)))

// s_waitcnt vmcnt(n) for a runtime n (the count is an immediate): n is wave-uniform and small.
__device__ __forceinline__ void nerf_wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
  }
}

typedef float nerf_f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ nerf_f32x4 lds_read_f4(uint32_t byte_addr) {
  nerf_f32x4 v;
  asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(byte_addr));
  return v;
}
// wait until at most N LDS reads of this wave are outstanding
template <int N>
__device__ __forceinline__ void nerf_wait_lgkmcnt_half() {
  if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(2)" ::: "memory");
  else if constexpr (N == 3) asm volatile("s_waitcnt lgkmcnt(3)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt lgkmcnt(5)" ::: "memory");
  else if constexpr (N == 6) asm volatile("s_waitcnt lgkmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

template <int BM, int BN, int WAVES_M, int EPI, int STAGES = 3, int MINW = 2>
__global__ __launch_bounds__(256, MINW) void gemm_nt_glds_kernel(const float* __restrict__ A, int lda,
                                                                const float* __restrict__ B, int ldb,
                                                                const float* __restrict__ bias, float* __restrict__ C,
                                                                int ldc, const uint32_t* __restrict__ mbits, int ldmb,
                                                                uint32_t* __restrict__ mbits_out, int K, int n_ntiles) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wave tile");
  constexpr int BK = 16;
  constexpr int STAGE_F = (BM + BN) * BK;         // floats per stage
  constexpr int NPIECE = (BM + BN) / 16;          // 1 KiB DMA pieces per stage
  constexpr int PPW = (NPIECE + 3) / 4;           // pieces per wave (upper bound)
  __shared__ __attribute__((aligned(16))) float smem[STAGES * STAGE_F];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;

  // per-lane DMA source pointers (k = 0) and wave-uniform LDS piece offsets
  const float* src[PPW];
  int dst[PPW];
#pragma unroll
  for (int j = 0; j < PPW; ++j) {
    const int piece = wave + 4 * j;
    const int r = piece * 16 + (lane >> 2);  // row of the stage image (A rows first, then B rows)
    const int p = lane & 3;
    const int rr = r < BM ? r : r - BM;
    const int c = p ^ ((rr >> 2) & 3);
    if (piece < NPIECE) {
      src[j] = (r < BM) ? A + (m0 + rr) * (int64_t)lda + 4 * c : B + (int64_t)(n0 + rr) * ldb + 4 * c;
      dst[j] = piece * 256;  // floats
    } else {
      src[j] = A;
      dst[j] = -1;
    }
  }
  auto issue = [&](int stage, int k0) {
#pragma unroll
    for (int j = 0; j < PPW; ++j) {
      if (NPIECE % 4 == 0 || dst[j] >= 0)
        __builtin_amdgcn_global_load_lds((const void*)(src[j] + k0), (NERF_LDS void*)(smem + stage * STAGE_F + dst[j]),
                                         16, 0, 0);
    }
  };

  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = K / BK;
  // prologue: STAGES-1 slabs in flight
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) issue(s, s * BK);

  const int sw = (li >> 2) & 3;
  // byte offsets (within a stage) of this lane's fragment rows and of its two k-chunks
  uint32_t a_off[TM], b_off[TN];
#pragma unroll
  for (int a = 0; a < TM; ++a) a_off[a] = (uint32_t)((wm * WTM + a * 32 + li) * BK * 4);
#pragma unroll
  for (int b = 0; b < TN; ++b) b_off[b] = (uint32_t)((BM + wn * WTN + b * 32 + li) * BK * 4);
  const uint32_t slot0 = (uint32_t)((((2 * lh) ^ sw)) * 16), slot1 = (uint32_t)((((2 * lh + 1) ^ sw)) * 16);
  const int MYP = (NPIECE % 4 == 0) ? PPW : (NPIECE - wave + 3) / 4;  // this wave's pieces per slab
  for (int kt = 0; kt < nk; ++kt) {
    // retire slab kt: this wave's pieces of the slabs issued after it (at most STAGES-2) may stay in flight
    if (kt + STAGES - 2 < nk) nerf_wait_vmcnt((STAGES - 2) * MYP);
    else nerf_wait_vmcnt(0);
    __builtin_amdgcn_s_barrier();  // every wave's DMA of slab kt landed; every wave done with slab kt-1
    if (kt + STAGES - 1 < nk) issue((kt + STAGES - 1) % STAGES, (kt + STAGES - 1) * BK);
    // fragment reads are inline asm: a compiler-visible ds_read of the DMA-written array would get an
    // `s_waitcnt vmcnt(0)` (the waitcnt pass cannot tell the stages apart), draining the ring.
    const uint32_t sbase = (uint32_t)(uintptr_t)(smem + (kt % STAGES) * STAGE_F);
    nerf_f32x4 af[2][TM], bf[2][TN];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int a = 0; a < TM; ++a) af[h][a] = lds_read_f4(sbase + a_off[a] + (h ? slot1 : slot0));
#pragma unroll
      for (int b = 0; b < TN; ++b) bf[h][b] = lds_read_f4(sbase + b_off[b] + (h ? slot1 : slot0));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // tie the fragments to the wait so no MFMA is hoisted above it
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int a = 0; a < TM; ++a) asm volatile("" : "+v"(af[h][a]));
#pragma unroll
      for (int b = 0; b < TN; ++b) asm volatile("" : "+v"(bf[h][b]));
    }
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(bf[h][b][s], af[h][a][s], acc[a][b], 0, 0, 0);
  }
  nt_epilogue<TM, TN, WTM, WTN, EPI>(acc, m0 + wm * WTM, n0 + wn * WTN, li, lh, bias, C, ldc, mbits, ldmb, mbits_out);
}
