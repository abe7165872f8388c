// Fused forward "tail" of the vanilla MLP (fp32 path, mlp.hip): everything after the trunk.7 output in ONE launch —
// models/inr/meta_vanilla.py:109-154 (MetaNeRF.color / forward):
//   O16 = h7 W_head^T + b           [sigma_raw | geo 0..14]                       (sigma_head + geo_head)
//   CIN = [geo, d, FrequencyEncoder(d, L = 4)]  (42 columns)                      (models/encodings.py:437-444)
//   C0  = relu(CIN W_c0^T + b_c0)    (128)
//   O3  = C0 W_c1^T + b_c1           (3)
//   rgb_sigma = [sigmoid(O3), trunc_exp(sigma_raw)]                              (models/trunc_exp.py:30-61)
// The unfused chain ran five launches per net (two N = 32 GEMMs, the colour-input build, the colour layer-0 GEMM and
// the head activation) and moved ~2.9 KB per sample row through HBM; this kernel reads the trunk.7 row (1 KB) and
// the direction, and writes what the backward reads (HO 16 B, CIN 256 B, C0 512 B) and rgb_sigma.
//
// Geometry: a 256-thread workgroup (4 waves) walks 64-row tiles (persistent, two workgroups per CU); wave w owns rows
// 16 w .. 16 w + 15 of the tile through all three layers.  Every product is v_mfma_f32_16x16x4_f32 (exact fp32 fmaf
// chains) with the operands swapped as in gemm_nt16_kernel: lane l supplies activation row (l & 15) and k-slot
// g = l >> 4 (one float4 per lane feeds four MFMAs over a 16-deep k chunk, k = 16 hh + 4 g + s) and receives row
// (l & 15), columns 4 g + r of the 16-column output block — which is exactly the A-operand layout of the next layer,
// so the head output and C0 stay in registers as the next layer's input fragments:
//   * head -> colour layer 0: the colour input is taken in the head's column alignment ([sigma_raw | geo | d | PE])
//     against a colour-0 weight image shifted by one column with a zero first column (sigma_raw contributes 0 x
//     sigma_raw = 0); the direction encoding of the lane's columns is computed in place (libm sincosf, as
//     build_cin_kernel);
//   * colour 0 -> colour out: C0 column block cb is k chunk cb of the colour-out product.
// Weights (head rows 0..15, the shifted colour-0 image, colour-out rows 0..15) and biases sit in LDS once per
// workgroup; the next tile's trunk.7 fragments are loaded while the colour-out layer of the current tile runs.
#pragma once
#include "gemm.hpp"
#include "mlp_common.hpp"

namespace nerf_mlp {

constexpr int FT_ROWS = 64;
// LDS pitches (floats).  A ds_read_b128 of lane (lr = l & 15, g = l >> 4) reads 16-B slot (lr * P / 4 + g) mod 16 of the
// 64-bank array; its lane groups {0-3,12-15,20-27}, ... mix (lr, g) with (lr - 4 .. lr + 7, g + 1), which are all
// distinct for P / 4 = 2 (mod 16) (slots 2 lr + g): 264 / 72 / 136.  The round-4 pitches 260 / 52 / 132 (P / 4 odd)
// put two lanes of every group on one slot: 1.4e7 conflict cycles per fine launch (profiles/r05/pmc_mfma.txt).
// The CIN staging pitch 68 keeps its scalar writes at most 2-way (free for ds_write_b32).
constexpr int FT_WH = 264, FT_WC0 = 72, FT_WC1 = 136, FT_CIN = 68;

struct FwdTailArgs {
  const float* Y7;   // [Mp][ldy] trunk.7 output (ldy 256 in training, 320 in the inference ping-pong)
  const float* xd;   // [M][6] (directions in cols 3..5)
  const float* w;    // packed fp32 parameters
  int64_t off_wh, off_bh, off_wc0, off_bc0, off_wc1, off_bc1;
  float *HO, *CIN, *C0;        // [Mp][4] (o3_0..2, sigma_raw), [Mp][64], [Mp][128] (training: what the backward reads)
  float* out;                  // [M][4] rgb_sigma
  int64_t M, Mp;
  int ntiles, ldy;
};

// canonical colour-input column c (0..63) of a row: geo (from the head, handled by the caller), d, its encoding
// [cos 2^0..2^3, sin 2^0..2^3] per dimension (build_cin_kernel's order), zeros from column 42
__device__ __forceinline__ float cin_dir_value(int c, const float (&d)[3]) {
  if (c < 15 || c >= 42) return 0.f;
  if (c < 18) return d[c - 15];
  const int q = c - 18, k = q >> 3, wi = q & 7, l = wi & 3;
  float s, co;
  sincosf(d[k] * (float)(1 << l), &s, &co);
  return wi < 4 ? co : s;
}

template <bool TRAIN>
__global__ __launch_bounds__(256, 2) void fwd_tail_kernel(FwdTailArgs A) {
  __shared__ __attribute__((aligned(16))) float sWh[16 * FT_WH];
  __shared__ __attribute__((aligned(16))) float sWc0[128 * FT_WC0];
  __shared__ __attribute__((aligned(16))) float sWc1[16 * FT_WC1];
  __shared__ __attribute__((aligned(16))) float sB[16 + 128 + 16];
  __shared__ __attribute__((aligned(16))) float sCIN[FT_ROWS * FT_CIN];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int lr = lane & 15, g = lane >> 4;

  for (int i = tid; i < 16 * 256; i += 256) sWh[(i >> 8) * FT_WH + (i & 255)] = A.w[A.off_wh + i];
  for (int i = tid; i < 128 * 48; i += 256) {
    const int n = i / 48, j = i - n * 48;  // shifted image: column j <- Wc0 column j - 1, column 0 = 0
    sWc0[n * FT_WC0 + j] = j == 0 ? 0.f : A.w[A.off_wc0 + n * 64 + j - 1];
  }
  for (int i = tid; i < 16 * 128; i += 256) sWc1[(i >> 7) * FT_WC1 + (i & 127)] = A.w[A.off_wc1 + i];
  if (tid < 16) sB[tid] = A.w[A.off_bh + tid];
  if (tid < 128) sB[16 + tid] = A.w[A.off_bc0 + tid];
  if (tid < 16) sB[144 + tid] = A.w[A.off_bc1 + tid];
  __syncthreads();

  int t = blockIdx.x;
  if (t >= A.ntiles) return;
  float4 yf[16];  // trunk.7 fragments of the tile: row 16 w + lr, columns 16 hh + 4 g .. + 3
  auto load_y = [&](int tile) {
    const float* y = A.Y7 + ((int64_t)tile * FT_ROWS + 16 * w + lr) * A.ldy + 4 * g;
#pragma unroll
    for (int hh = 0; hh < 16; ++hh) yf[hh] = *reinterpret_cast<const float4*>(y + 16 * hh);
  };
  load_y(t);
  for (; t < A.ntiles; t += gridDim.x) {
    const int64_t m = (int64_t)t * FT_ROWS + 16 * w + lr;  // this lane's row
    // ---- head: O16[m][4g + r], columns 0..15 (rows 16..31 of the packed head are zero padding)
    nerf_f32x4 ah = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int hh = 0; hh < 16; ++hh) {
      const float4 wf = *reinterpret_cast<const float4*>(sWh + lr * FT_WH + 16 * hh + 4 * g);
      ah = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.x, yf[hh].x, ah, 0, 0, 0);
      ah = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.y, yf[hh].y, ah, 0, 0, 0);
      ah = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.z, yf[hh].z, ah, 0, 0, 0);
      ah = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.w, yf[hh].w, ah, 0, 0, 0);
    }
    float o16[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) o16[r] = ah[r] + sB[4 * g + r];
    const float sigma_raw = o16[0];  // meaningful in lanes g == 0
    // ---- colour input in the head's alignment: chunk 0 = O16 columns 0..15, chunks 1, 2 = canonical CIN
    // columns 15 + 4g + s and 31 + 4g + s (direction and its encoding); rows >= M are all zero (build_cin_kernel)
    const bool real = m < A.M;
    float d[3] = {0.f, 0.f, 0.f};
    if (real) {
      d[0] = A.xd[m * 6 + 3];
      d[1] = A.xd[m * 6 + 4];
      d[2] = A.xd[m * 6 + 5];
    }
    float4 cin[3];
    cin[0] = real ? make_float4(o16[0], o16[1], o16[2], o16[3]) : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int ch = 1; ch < 3; ++ch) {
      float v[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {  // one sincosf at a time: interleaved, their slow paths exhaust the registers
        v[s] = real ? cin_dir_value(16 * ch - 1 + 4 * g + s, d) : 0.f;
        __builtin_amdgcn_sched_barrier(0);
      }
      cin[ch] = make_float4(v[0], v[1], v[2], v[3]);
    }
    if (TRAIN) {  // the canonical CIN row (geo | d | PE | 0) for the backward, staged per wave through LDS
      float* sr = sCIN + (16 * w + lr) * FT_CIN;
      const float c0v[4] = {cin[0].x, cin[0].y, cin[0].z, cin[0].w};
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (4 * g + r >= 1) sr[4 * g + r - 1] = c0v[r];
      const float c1v[4] = {cin[1].x, cin[1].y, cin[1].z, cin[1].w}, c2v[4] = {cin[2].x, cin[2].y, cin[2].z, cin[2].w};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sr[15 + 4 * g + s] = c1v[s];
        sr[31 + 4 * g + s] = c2v[s];
        sr[47 + 4 * g + s] = 0.f;
      }
      if (g == 3) sr[63] = 0.f;
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave reads back only its own 16 rows
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = (lane >> 4) + 4 * i, c4 = lane & 15;
        *reinterpret_cast<float4*>(A.CIN + ((int64_t)t * FT_ROWS + 16 * w + row) * 64 + 4 * c4) =
            *reinterpret_cast<const float4*>(sCIN + (16 * w + row) * FT_CIN + 4 * c4);
      }
    }
    // ---- colour layer 0: C0 = relu(CIN Wc0^T + b), 8 column blocks of 16, K = 48 (3 chunks)
    nerf_f32x4 ac[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) ac[cb] = nerf_f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
#pragma unroll
      for (int cb = 0; cb < 8; ++cb) {
        const float4 wf = *reinterpret_cast<const float4*>(sWc0 + (16 * cb + lr) * FT_WC0 + 16 * ch + 4 * g);
        ac[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.x, cin[ch].x, ac[cb], 0, 0, 0);
        ac[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.y, cin[ch].y, ac[cb], 0, 0, 0);
        ac[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.z, cin[ch].z, ac[cb], 0, 0, 0);
        ac[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.w, cin[ch].w, ac[cb], 0, 0, 0);
      }
    }
    float4 c0[8];
#pragma unroll
    for (int cb = 0; cb < 8; ++cb) {
      const float* b = sB + 16 + 16 * cb + 4 * g;
      c0[cb] = make_float4(fmaxf(ac[cb][0] + b[0], 0.f), fmaxf(ac[cb][1] + b[1], 0.f), fmaxf(ac[cb][2] + b[2], 0.f),
                           fmaxf(ac[cb][3] + b[3], 0.f));
      if (TRAIN) *reinterpret_cast<float4*>(A.C0 + m * 128 + 16 * cb + 4 * g) = c0[cb];
    }
    // the next tile's trunk.7 rows, under colour out (issued right after the head MFMAs instead, pinned there: 214 -> 218
    // us per launch, round 4 — not kept)
    if (t + (int)gridDim.x < A.ntiles) load_y(t + gridDim.x);
    // ---- colour out: O3 = C0 Wc1^T + b (16 columns, 3 real), K = 128: C0 block cb is k chunk cb
    nerf_f32x4 ao = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < 8; ++ch) {
      const float4 wf = *reinterpret_cast<const float4*>(sWc1 + lr * FT_WC1 + 16 * ch + 4 * g);
      ao = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.x, c0[ch].x, ao, 0, 0, 0);
      ao = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.y, c0[ch].y, ao, 0, 0, 0);
      ao = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.z, c0[ch].z, ao, 0, 0, 0);
      ao = __builtin_amdgcn_mfma_f32_16x16x4f32(wf.w, c0[ch].w, ao, 0, 0, 0);
    }
    float o3[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) o3[r] = ao[r] + sB[144 + 4 * g + r];
    // the backward's head-output inputs, one 16-B row (round 4; the [Mp][32] O16 / O3 rows, 256 B written and read
    // back at line granularity for 16 used bytes, are gone): the colour pre-activations and sigma_raw
    if (TRAIN && g == 0) reinterpret_cast<float4*>(A.HO)[m] = make_float4(o3[0], o3[1], o3[2], sigma_raw);
    if (g == 0 && real) {
      const float sg = expf(fminf(fmaxf(sigma_raw, -EXP_MAX), EXP_MAX));
      reinterpret_cast<float4*>(A.out)[m] = make_float4(sigmoidf_(o3[0]), sigmoidf_(o3[1]), sigmoidf_(o3[2]), sg);
    }
  }
}

}  // namespace nerf_mlp
