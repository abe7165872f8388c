// Fused colour-branch backward of the vanilla MLP (fp32 path, mlp.hip).  The activations C0 / CIN may be read as
// fp32 or bf16 (TA) and dO16 written as fp32 or bf16 (TD); all arithmetic and the weight-gradient sums are fp32.
// Measured: fp32 path 28.2 -> 28.0 ms/step (six launches and ~1.7 GB of HBM traffic per step removed); the bf16
// path keeps its bf16-MFMA chain, which is faster there (8.36 vs 8.74 ms/step with this kernel: one 256-thread
// workgroup per CU walking 48 tiles is latency-bound at ~11 us per tile; the two-workgroups-per-split version
// below still measured 8.23 ms there against 8.15-8.18 ms for the chain, whose launches overlap the coarse
// backward better).
#pragma once
#include "gemm.hpp"
#include "mlp_common.hpp"

// ------------------------------------------------------------------ fused colour-branch backward
// One kernel for everything between d_rgb_sigma and dO16 (the gradient of the [sigma | geo] head output):
// sigmoid' and trunc_exp' (head_out), the colour_out and colour layer-0 weight / bias gradients and the
// geo-feature input gradient.  Grid = the S row splits of the packed weight-gradient slabs; each
// workgroup walks its split in 64-row tiles (the next tile's C0 / CIN rows are prefetched into registers
// while the current one is computed), keeps its weight-gradient sums in registers across the tiles and
// writes them into its slab once.  Per row it reads C0 / CIN / O3 / O16[0] / d_rgb_sigma (~1 KB) and writes
// one 128-B dO16 row; the unfused chain moved ~2.7 KB per row through six launches.
//   dO3   = g.rgb * s(1-s)                   (3 columns; VALU)
//   dWc1 += dO3^T C0, dbc1 += sum dO3        (3 x 128: VALU, thread = output column x row half, in the same pass
//   dC0   = (dO3 Wc1[:3]) * (C0 > 0)          as dC0; the forward ReLU mask is C0 > 0)
//   dWc0 += dC0^T CIN, dbc0 += sum dC0       (128 x 64: MFMA 32x32x2, wave w -> rows 32w.., both 32-col blocks)
//   dgeo  = dC0 Wc0[:, :15]                  (MFMA 16x16x4, wave w -> rows 16w.., Wc0 in registers)
//   dO16  = [g.sigma * exp(clamp(sigma_raw)), dgeo, 0...]   (stored from the dgeo accumulators)
// Round 4: the dC0 pass was 4-way LDS bank-conflicted (row-per-lane-group mapping), the dWc0 k-steps 2-way, and dgeo
// ran on 32x32x2 tiles with 17 of 32 columns unused plus an LDS sum of two contraction halves (5 barriers per tile,
// now 3).
namespace nerf_mlp {
// row parts per split of color_bwd / head_bwd: part 0 writes its sums into the split's slab, parts 1 .. TAIL_NQ - 1
// into rows (q - 1) S + s of partial2, added by reduce_splits2 after the slab terms.  Measured (C2, one box,
// profiles/r05/x6_variants_ab.txt): 2 parts 224.4-225.4k, 4 parts 224.0-224.1k, 8 parts 222.7-223.2k rays/s — the
// extra parts' partial slabs and reduce terms cost more than the second workgroup per CU gains; 2 is kept
#ifndef NERF_TAIL_NQ
#define NERF_TAIL_NQ 2
#endif
constexpr int TAIL_NQ = NERF_TAIL_NQ;
// rows [r0, r1) of part q of split sp (rps and the part length are multiples of `unit` rows)
__device__ __forceinline__ void tail_part_rows(int64_t sp, int q, int64_t rps, int64_t Mp, int unit, int64_t& r0,
                                               int64_t& r1) {
  const int64_t rpq = ((rps + (int64_t)TAIL_NQ * unit - 1) / ((int64_t)TAIL_NQ * unit)) * unit;
  const int64_t s0 = sp * rps, s1 = s0 + rps;
  r0 = s0 + q * rpq;
  r1 = (q == TAIL_NQ - 1) ? s1 : r0 + rpq;
  if (r1 > s1) r1 = s1;
  if (r1 > Mp) r1 = Mp;
  if (r0 > r1) r0 = r1;
}
constexpr int CB_ROWS = 64;
constexpr int CB_C0 = 132, CB_CIN = 68;

// 4 consecutive activations as fp32 (fp32 or bf16 storage) and 4 fp32 values stored as T
__device__ __forceinline__ float4 tail_ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float4 tail_ld4(const __bf16* p) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                     __uint_as_float(u.y & 0xffff0000u));
}
__device__ __forceinline__ void tail_st4(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
__device__ __forceinline__ void tail_st4(__bf16* p, float4 v) {
  p[0] = (__bf16)v.x; p[1] = (__bf16)v.y; p[2] = (__bf16)v.z; p[3] = (__bf16)v.w;
}

template <typename TA, typename TD>
__global__ __launch_bounds__(256, 2) void color_bwd_kernel(const float* __restrict__ g, const float* __restrict__ HO,
                                                        const TA* __restrict__ C0,
                                                        const TA* __restrict__ CIN,
                                                        const float* __restrict__ Wc0,  // [128][64]
                                                        const float* __restrict__ Wc1,  // [32][128]
                                                        TD* __restrict__ dO16, float* __restrict__ partial,
                                                        int64_t slab, int64_t off_w0, int64_t off_b0,
                                                        int64_t off_w1, int64_t off_b1, int64_t rps, int64_t M,
                                                        int64_t Mp, float* __restrict__ partial2, int64_t cslab,
                                                        int64_t p2base, int ldd) {
  // dC0 overwrites C0 in place (each element by the thread that read it, so without a barrier between): 52 KB of LDS,
  // two workgroups per CU, three barriers per tile.  Workgroup TAIL_NQ s + q walks part q of split s; part 0 writes the
  // colour sums into slab s, part q > 0 into row (q - 1) S + s of partial2 (cslab floats: packed offsets p2base ..
  // total of one slab; p2base <= off_w0).  dO16 rows have pitch ldd: 32 (columns 16..31 written as zeros) or 16.
  __shared__ __attribute__((aligned(16))) float s_c0[CB_ROWS * CB_C0];
  float* const s_dc0 = s_c0;
  __shared__ __attribute__((aligned(16))) float s_cin[CB_ROWS * CB_CIN];
  __shared__ __attribute__((aligned(16))) float s_do3[CB_ROWS * 4];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, li = lane & 31, lh = lane >> 5;
  const int64_t sp = blockIdx.x / TAIL_NQ, S = gridDim.x / TAIL_NQ;
  const int q = blockIdx.x % TAIL_NQ;
  int64_t r0, r1;
  tail_part_rows(sp, q, rps, Mp, CB_ROWS, r0, r1);

  // register prefetch of one tile: C0 = 2048 float4 (8 / thread), CIN = 1024 float4 (4 / thread); wave 0 also
  // prefetches the tile's head outputs: d_rgb_sigma (M rows: the row index is clamped, the value zeroed below for
  // m >= M) and the HO row (the three colour pre-activations, sigma_raw).
  float4 pc[8], pi[4], pg = make_float4(0.f, 0.f, 0.f, 0.f), po = pg;
  // r0, r1, rps and the part length are multiples of CB_ROWS (the host rounds rps to 64; Mp is a multiple of 256),
  // so every row of a tile is < r1 and the loads carry no row guard (a guarded load became a branch with a
  // vmcnt(0) drain after it); a uniform tile base + 32-bit lane offsets keeps no 64-bit address per load live
  auto fetch = [&](int64_t t0) {
    const TA* c0t = C0 + t0 * 128;
    const TA* cit = CIN + t0 * 64;
#pragma unroll
    for (int u = 0; u < 8; ++u) pc[u] = tail_ld4(c0t + (tid + 256 * u) * 4);  // row f >> 5, float4 f & 31
#pragma unroll
    for (int u = 0; u < 4; ++u) pi[u] = tail_ld4(cit + (tid + 256 * u) * 4);  // row f >> 4, float4 f & 15
    if (tid < CB_ROWS) {  // wave 0 (uniform branch)
      const int64_t m = t0 + tid, mc = m < M ? m : M - 1;
      pg = reinterpret_cast<const float4*>(g)[mc];
      po = reinterpret_cast<const float4*>(HO)[m];
    }
  };

  // colour_out / dC0 phase: thread (column jw, row half rh); its colour_out weight column lives in registers
  const int jw = tid & 127, rh = tid >> 7;
  const float w10 = Wc1[jw], w11 = Wc1[128 + jw], w12 = Wc1[256 + jw];
  float w1a = 0.f, w1b = 0.f, w1c = 0.f, b1a = 0.f, b1b = 0.f, b1c = 0.f;  // b1*: kept by jw == 0
  // dgeo phase (16x16x4 MFMA, wave w -> rows 16w..16w+15, all 128 contraction columns): lane group kg = lane >> 4
  // owns contraction columns 32 kg + kk; its B operand Wc0[32 kg + kk][c = lane & 15] lives in registers
  const int gc = lane & 15, kg = lane >> 4;
  float wg[32];
#pragma unroll
  for (int kk = 0; kk < 32; ++kk) wg[kk] = Wc0[(32 * kg + kk) * 64 + gc];
  nerf_f32x16 acc0[2];
  for (int r = 0; r < 16; ++r) { acc0[0][r] = 0.f; acc0[1][r] = 0.f; }
  float bsum0 = 0.f;

  if (r0 < r1) fetch(r0);
  for (int64_t t0 = r0; t0 < r1; t0 += CB_ROWS) {
    __syncthreads();  // previous tile's LDS readers are done
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int f = tid + 256 * u;
      *reinterpret_cast<float4*>(s_c0 + (f >> 5) * CB_C0 + 4 * (f & 31)) = pc[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int f = tid + 256 * u;
      *reinterpret_cast<float4*>(s_cin + (f >> 4) * CB_CIN + 4 * (f & 15)) = pi[u];
    }
    if (tid < CB_ROWS) {
      const int64_t m = t0 + tid;
      float a = 0.f, b = 0.f, c = 0.f, ds = 0.f;
      if (m < M) {
        const float s0 = sigmoidf_(po.x), s1 = sigmoidf_(po.y), s2 = sigmoidf_(po.z);
        a = pg.x * (s0 * (1.0f - s0));
        b = pg.y * (s1 * (1.0f - s1));
        c = pg.z * (s2 * (1.0f - s2));
        ds = pg.w * expf(fminf(fmaxf(po.w, -EXP_MAX), EXP_MAX));
      }
      *reinterpret_cast<float4*>(s_do3 + tid * 4) = make_float4(a, b, c, ds);
    }
    __syncthreads();
    if (t0 + CB_ROWS < r1) fetch(t0 + CB_ROWS);  // in flight during this tile's compute
    // ---- VALU: dWc1 / dbc1 sums over the thread's 32 rows, then its dC0 element written over the C0 element it read
#pragma unroll 8
    for (int rr = 0; rr < CB_ROWS / 2; ++rr) {
      const int r = 32 * rh + rr;
      const float c0 = s_c0[r * CB_C0 + jw];
      const float4 d = *reinterpret_cast<const float4*>(s_do3 + r * 4);
      w1a += d.x * c0;
      w1b += d.y * c0;
      w1c += d.z * c0;
      if (jw == 0) { b1a += d.x; b1b += d.y; b1c += d.z; }
      const float v = d.x * w10 + d.y * w11 + d.z * w12;
      s_dc0[r * CB_C0 + jw] = c0 > 0.f ? v : 0.f;
    }
    __syncthreads();
    // ---- MFMA: dWc0 (wave w -> rows 32w..), bias sums.  k-step st pairs rows r and r + 8 (lane halves): 8 rows apart
    // the two halves' LDS reads sit 32 banks apart (pitches 132 / 68), conflict-free
#pragma unroll 16
    for (int st = 0; st < CB_ROWS / 2; ++st) {
      const int row = (st & 7) + 16 * (st >> 3) + 8 * lh;
      const float av = s_dc0[row * CB_C0 + 32 * wave + li];
      bsum0 += av;
      acc0[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, s_cin[row * CB_CIN + li], acc0[0], 0, 0, 0);
      acc0[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, s_cin[row * CB_CIN + 32 + li], acc0[1], 0, 0, 0);
    }
    // ---- dgeo = dC0 Wc0[:, :15] (16x16x4: A lane (row gc, k 32 kg + kk), B lane (k, column gc)), then the dO16 rows
    //      [ds, dgeo, 0...] straight from the accumulator (lane (kg, gc) holds rows 4 kg + v, column gc)
    {
      nerf_f32x4 accg = {0.f, 0.f, 0.f, 0.f};
      const float* arow = s_dc0 + (16 * wave + gc) * CB_C0 + 32 * kg;
#pragma unroll
      for (int k4 = 0; k4 < 8; ++k4) {
        const float4 a4 = *reinterpret_cast<const float4*>(arow + 4 * k4);
        accg = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, wg[4 * k4 + 0], accg, 0, 0, 0);
        accg = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, wg[4 * k4 + 1], accg, 0, 0, 0);
        accg = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, wg[4 * k4 + 2], accg, 0, 0, 0);
        accg = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, wg[4 * k4 + 3], accg, 0, 0, 0);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int r = 16 * wave + 4 * kg + v;
        TD* drow = dO16 + (t0 + r) * ldd;
        if (gc < 15) drow[gc + 1] = (TD)accg[v];
        else drow[0] = (TD)s_do3[r * 4 + 3];
        if (ldd == 32) drow[16 + gc] = (TD)0.f;
      }
    }
  }
  // ---- this split's slab: weight sums, bias sums (lane halves combined); the dWc1 row halves combined through LDS
  __syncthreads();
  if (rh == 1) {
    s_c0[jw * 4 + 0] = w1a; s_c0[jw * 4 + 1] = w1b; s_c0[jw * 4 + 2] = w1c;
    if (jw == 0) { s_c0[512] = b1a; s_c0[513] = b1b; s_c0[514] = b1c; }
  }
  __syncthreads();
  float* P = q ? partial2 + ((q - 1) * S + sp) * cslab - p2base : partial + sp * slab;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int n = (r & 3) + 8 * (r >> 2) + 4 * lh;
    P[off_w0 + (int64_t)(32 * wave + n) * 64 + li] = acc0[0][r];
    P[off_w0 + (int64_t)(32 * wave + n) * 64 + 32 + li] = acc0[1][r];
  }
  const float v0 = bsum0 + __shfl_xor(bsum0, 32, 64);
  if (lh == 0) P[off_b0 + 32 * wave + li] = v0;
  // colour_out: rows 0..2 from the VALU sums, rows 3..31 zero; its bias likewise
  for (int i = tid; i < 32 * 128; i += 256) {
    const int n = i >> 7;
    if (n >= 3) P[off_w1 + i] = 0.f;
  }
  if (rh == 0) {
    P[off_w1 + jw] = w1a + s_c0[jw * 4 + 0];
    P[off_w1 + 128 + jw] = w1b + s_c0[jw * 4 + 1];
    P[off_w1 + 256 + jw] = w1c + s_c0[jw * 4 + 2];
    if (jw == 0) {
      P[off_b1 + 0] = b1a + s_c0[512];
      P[off_b1 + 1] = b1b + s_c0[513];
      P[off_b1 + 2] = b1c + s_c0[514];
    }
  }
  if (tid >= 3 && tid < 32) P[off_b1 + tid] = 0.f;
}
// ------------------------------------------------------------------ fused head backward (fp32 path)
// dZ7 = (dO16 Wh) * [Y7 > 0] and the head sums dWh += dO16^T Y7, dbh += colsum(dO16) in ONE pass over Y7: the one
// read of a Y7 float4 is both the ReLU mask of the lane's own dZ7 float4 and a weight-gradient MFMA operand.  It
// replaces the head input-gradient GEMM and the head weight-gradient GEMM, which streamed Y7 / dZ7 separately
// (fine net, round 3: 258 + 216 us; this pass moves 2.1 KB per row: dO16 64 B + Y7 1 KB in, dZ7 1 KB out).
// Same split walk as color_bwd (workgroup TAIL_NQ s + q, 64-row tiles, sums in registers, parts q > 0 into partial2).  Lane
// (g, j) of wave w owns columns hc = 64 w + 4 j .. + 3 and, in row group u, row 4 u + g: its dZ7 float4 is a
// 16-term VALU dot against its register slice of Wh, and its Y7 float4 is the B operand of four 16x16x4 MFMAs
// (column hc + q, q = 0..3) whose A operand is dO16[4 u + g][n = j] — output lane (g, j) register v then holds
// dWh[4 g + v][hc + q].  dO16 tiles are double-buffered in LDS (one barrier per tile); Y7 streams in two 32-row
// halves, each issued one half ahead, from a uniform tile base with 32-bit lane offsets.
constexpr int HB_ROWS = 64;
static __global__ __launch_bounds__(256, 2) void head_bwd_kernel(const float* __restrict__ dO16,  // [Mp][16]
                                                       const float* __restrict__ Y7,    // [Mp][256]
                                                       const float* __restrict__ Wh,    // [32][256], rows < 16 live
                                                       float* __restrict__ dZ7,         // [Mp][256]
                                                       float* __restrict__ partial, int64_t slab,
                                                       float* __restrict__ partial2, int64_t cslab, int64_t p2base,
                                                       int64_t off_wh, int64_t off_bh, int64_t rps, int64_t Mp) {
  __shared__ __attribute__((aligned(16))) float s_d[2][HB_ROWS * 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, g = lane >> 4, j = lane & 15;
  const int hc = 64 * wave + 4 * j;
  const int64_t sp = blockIdx.x / TAIL_NQ, S = gridDim.x / TAIL_NQ;
  const int q = blockIdx.x % TAIL_NQ;
  int64_t r0, r1;
  tail_part_rows(sp, q, rps, Mp, HB_ROWS, r0, r1);
  // every tile row is < r1 (r0, r1 multiples of 64, as in color_bwd); "next tile" loads past the last tile re-read it
  const int64_t last = r1 - HB_ROWS;

  float4 wh[16];
#pragma unroll
  for (int n = 0; n < 16; ++n) wh[n] = *reinterpret_cast<const float4*>(Wh + n * 256 + hc);
  nerf_f32x4 acc[4], accb;
#pragma unroll
  for (int q = 0; q < 4; ++q) acc[q] = nerf_f32x4{0.f, 0.f, 0.f, 0.f};
  accb = nerf_f32x4{0.f, 0.f, 0.f, 0.f};

  float4 dd = make_float4(0.f, 0.f, 0.f, 0.f), ya[8], yb[8];
  auto load_y = [&](float4 (&y)[8], int64_t t0, int rb) {
    const float* yt = Y7 + t0 * 256;
#pragma unroll
    for (int u = 0; u < 8; ++u) y[u] = *reinterpret_cast<const float4*>(yt + ((rb + 4 * u + g) * 256 + hc));
  };
  auto rows = [&](const float4 (&y)[8], int64_t t0, int rb, const float* sd) {
    float* zt = dZ7 + t0 * 256;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = rb + 4 * u + g;
      const float* drow = sd + r * 16;
      float z0 = 0.f, z1 = 0.f, z2 = 0.f, z3 = 0.f;
#pragma unroll
      for (int n4 = 0; n4 < 4; ++n4) {
        const float4 d = *reinterpret_cast<const float4*>(drow + 4 * n4);
        const float dn[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float4 w4 = wh[4 * n4 + e];
          z0 = fmaf(dn[e], w4.x, z0);
          z1 = fmaf(dn[e], w4.y, z1);
          z2 = fmaf(dn[e], w4.z, z2);
          z3 = fmaf(dn[e], w4.w, z3);
        }
      }
      const float4 yy = y[u];
      *reinterpret_cast<float4*>(zt + (r * 256 + hc)) =
          make_float4(yy.x > 0.f ? z0 : 0.f, yy.y > 0.f ? z1 : 0.f, yy.z > 0.f ? z2 : 0.f, yy.w > 0.f ? z3 : 0.f);
      const float a = drow[j];
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, yy.x, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, yy.y, acc[1], 0, 0, 0);
      acc[2] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, yy.z, acc[2], 0, 0, 0);
      acc[3] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, yy.w, acc[3], 0, 0, 0);
      if (wave == 0) accb = __builtin_amdgcn_mfma_f32_16x16x4f32(a, 1.0f, accb, 0, 0, 0);
    }
  };

  if (r0 < r1) {
    dd = *reinterpret_cast<const float4*>(dO16 + r0 * 16 + tid * 4);  // 64 rows x 16 = one float4 per thread
    load_y(ya, r0, 0);
  }
  int buf = 0;
  for (int64_t t0 = r0; t0 < r1; t0 += HB_ROWS) {
    const int64_t tn = t0 < last ? t0 + HB_ROWS : last;
    float* sd = s_d[buf];
    *reinterpret_cast<float4*>(sd + tid * 4) = dd;
    __syncthreads();  // (the other buffer's readers finished before the previous tile's barrier)
    dd = *reinterpret_cast<const float4*>(dO16 + tn * 16 + tid * 4);
    load_y(yb, t0, 32);
    rows(ya, t0, 0, sd);
    load_y(ya, tn, 0);
    rows(yb, t0, 32, sd);
    buf ^= 1;
  }

  float* P = q ? partial2 + ((q - 1) * S + sp) * cslab - p2base : partial + sp * slab;
#pragma unroll
  for (int v = 0; v < 4; ++v)
    *reinterpret_cast<float4*>(P + off_wh + (int64_t)(4 * g + v) * 256 + hc) =
        make_float4(acc[0][v], acc[1][v], acc[2][v], acc[3][v]);
  for (int i = tid; i < 16 * 256; i += 256) P[off_wh + 16 * 256 + i] = 0.f;  // head rows 16..31: padding
  if (wave == 0 && j == 0) {
#pragma unroll
    for (int v = 0; v < 4; ++v) P[off_bh + 4 * g + v] = accb[v];
  }
  if (tid >= 16 && tid < 32) P[off_bh + tid] = 0.f;
}

// reduce_splits plus the colour / head sums of parts 1.. : float4 i >= c0 of the packed gradient also adds the S terms of src2
// (src2[s][i - c0]) after the slab terms, both in gemm.hpp's RG-group order (bitwise reproducible); grid cdiv(n4, 64)
// (TAIL_NQ - 1 sets of S rows in src2: parts 1, 2, ... of color_bwd / head_bwd, each added in that order)
static __global__ __launch_bounds__(256) void reduce_splits2_kernel(const float* __restrict__ src, int64_t slab, int S,
                                                                    float* __restrict__ dst, int64_t n4, int accumulate,
                                                                    const float* __restrict__ src2, int64_t slab2,
                                                                    int64_t c0) {
  __shared__ float4 part[TAIL_NQ][RG][64];
  const int e = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + e;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  part[0][g][e] = i < n4 ? rg_group_sum(src + 4 * i, slab, S, g) : z;
#pragma unroll
  for (int q = 1; q < TAIL_NQ; ++q)
    part[q][g][e] = (i < n4 && i >= c0) ? rg_group_sum(src2 + (int64_t)(q - 1) * S * slab2 + 4 * (i - c0), slab2, S, g)
                                        : z;
  __syncthreads();
  if (g == 0 && i < n4) {
    float4 a = accumulate ? reinterpret_cast<const float4*>(dst)[i] : z;
#pragma unroll
    for (int k = 0; k < RG; ++k) rg_add(a, part[0][k][e]);
    if (i >= c0) {
#pragma unroll
      for (int q = 1; q < TAIL_NQ; ++q)
#pragma unroll
        for (int k = 0; k < RG; ++k) rg_add(a, part[q][k][e]);
    }
    reinterpret_cast<float4*>(dst)[i] = a;
  }
}

}  // namespace nerf_mlp

