// The vanilla NeRF expert in bf16 (BASELINE.json configs[2], "bf16 MLP with fp32 compositing"): the same
// network and packed fp32 parameters as mlp.hip (models/inr/meta_vanilla.py:109-154), with every layer's
// GEMM on gfx950 bf16 MFMA (fp32 accumulate) and the activations kept in HBM as bf16:
//   forward  x_d -> PE (bf16) -> 8 x [bf16 GEMM + bias + ReLU -> bf16 + bitmask] -> heads (fp32 out)
//            -> colour input (bf16) -> colour MLP -> sigmoid / trunc_exp (fp32)        rgb_sigma fp32
//   backward activation gradients bf16, weight gradients fp32 (fp32 split-M slabs, deterministic reduce)
// The compositing, loss, sampling and optimiser stay fp32.  Parameters stay fp32 masters; each call
// converts them once to a packed bf16 copy (and bf16 transposes for the input-gradient GEMMs) in the
// caller's workspace.
//
// Workspace (Mp = M rounded up to 256): Wb [total] bf16, X3E [Mp][320] bf16 (trunk.3 output | xyz PE),
// Y0..Y7 [Mp][256] bf16, O16 [Mp][32] fp32, CIN [Mp][64] bf16, C0 [Mp][128] bf16, O3 [Mp][32] fp32,
// bitmasks; backward: dA/dB [Mp][256] bf16, dO16/dO3 [Mp][32] bf16, dCIN [Mp][32] fp32, dC0 [Mp][128]
// bf16, bf16 transposed weights, S fp32 partial slabs of the packed gradient.
#include "gemm_bf16.hpp"
#include "mlp_bf16_fused.hpp"
#include "mlp_bf16_bwd.hpp"
#include "mlp_bf16_tail.hpp"
#include "mlp_tail.hpp"
#include "mlp_common.hpp"

// entry-point names of this build (gemm_bf16.hpp NERF_F16): nerf_mlp_*_bf16 or nerf_mlp_*_f16
#if NERF_F16
#define NERF_H16_FN(name) name##_f16
#else
#define NERF_H16_FN(name) name##_bf16
#endif

namespace NERF_H16NS {
namespace {
using namespace nerf_mlp;

// narrow slab of the fused backward: trunk.0 W [256][64] | trunk.4 W[:, 256:320] [256][64] | trunk.0 b [256]
constexpr int64_t NPS = 2 * 256 * 64 + 256;
constexpr int64_t WTB_ELEMS = 7 * 65536 + 256 * 32 + 128 * 32 + 32 * 128;

struct WSB {
  int64_t Mp;
  nerf_bf16 *Wb, *Wf, *X3E, *Y[8], *CIN, *C0;
  float *O16, *O3, *HO;
  uint32_t *MB[8], *MC0;
  nerf_bf16 *dA, *dB, *dO16, *dO3, *dC0, *WTb, *WTf;
  float *dCIN, *partial, *partial2, *np;
  int S, S2;
  int64_t rps, rps2;
  int64_t bytes;
};

// split-M partial slabs of the weight gradient: one per >= 1024 rows, at most NERF_BF16_MAX_SPLITS (128) — the fused
// backward runs two workgroups per split, so 128 splits fill the 256 CUs in one round (256 splits took two rounds and
// doubled the slab traffic: 526 MB of partials per fine-net backward).  A compile-time constant (tools/ A/B builds
// pass -DNERF_BF16_MAX_SPLITS=...), so the workspace query and the kernels always agree.
#ifndef NERF_BF16_MAX_SPLITS
#define NERF_BF16_MAX_SPLITS 128
#endif
#ifndef NERF_BF16_NARROW_MUL
#define NERF_BF16_NARROW_MUL 2  // sub-splits per split of the narrow trunk.0 / trunk.4-encoding weight gradients
#endif
int bf16_splits(int64_t Mp) {
  const int mx = NERF_BF16_MAX_SPLITS;
  int64_t sp = Mp / 1024;
  return (int)(sp < 1 ? 1 : (sp > mx ? mx : sp));
}

WSB carve_b(void* base, int64_t M, int training) {
  WSB w{};
  w.Mp = round_up(M < 1 ? 1 : M, 256);
  const int64_t Mp = w.Mp;
  char* p = reinterpret_cast<char*>(base);
  auto take = [&](int64_t bytes) {
    char* q = p;
    p += round_up(bytes, 256);
    return q;
  };
  const Layout& L = layout();
  w.Wb = (nerf_bf16*)take(L.total * 2);
  w.Wf = (nerf_bf16*)take(nerf_fused::frag_tab().off[nerf_fused::FT] * 2);
  w.X3E = (nerf_bf16*)take(Mp * 320 * 2);
  if (training) {
    for (int i = 0; i < 8; ++i) w.Y[i] = (i == 3) ? w.X3E : (nerf_bf16*)take(Mp * 256 * 2);
  } else {
    nerf_bf16* q = (nerf_bf16*)take(Mp * 256 * 2);
    for (int i = 0; i < 8; ++i) w.Y[i] = (i % 2 == 0) ? q : w.X3E;  // ping-pong
  }
  w.O16 = (float*)take(Mp * 32 * 4);
  w.CIN = (nerf_bf16*)take(Mp * 64 * 2);
  w.C0 = (nerf_bf16*)take(Mp * 128 * 2);
  w.O3 = (float*)take(Mp * 32 * 4);
  w.HO = (float*)take(Mp * 4 * 4);
  if (training) {
    for (int i = 0; i < 8; ++i) w.MB[i] = (uint32_t*)take(Mp * 8 * 4);
    w.MC0 = (uint32_t*)take(Mp * 4 * 4);
    w.dA = (nerf_bf16*)take(Mp * 256 * 2);
    w.dB = (nerf_bf16*)take(Mp * 256 * 2);
    w.dO16 = (nerf_bf16*)take(Mp * 32 * 2);
    w.dO3 = (nerf_bf16*)take(Mp * 32 * 2);
    w.dC0 = (nerf_bf16*)take(Mp * 128 * 2);
    w.dCIN = (float*)take(Mp * 32 * 4);
    w.WTb = (nerf_bf16*)take(WTB_ELEMS * 2);
    w.WTf = (nerf_bf16*)take(7 * nerf_bwd::WT_LAYER * 2);
    w.S = bf16_splits(Mp);
    w.rps = round_up(nerf_cdiv(Mp, w.S), 64);  // whole slabs for every wgrad MR
    w.partial = (float*)take((int64_t)w.S * L.total * 4);
    w.partial2 = (float*)take((int64_t)w.S * (L.total - L.off[16]) * 4);  // second-half tail sums (fused backward)
    // the narrow weight gradients of the fused backward (trunk.0, trunk.4's encoding columns) over S2 = 4 S sub-splits
    {
      int64_t s2 = (int64_t)NERF_BF16_NARROW_MUL * w.S, cap = Mp / 256;
      w.S2 = (int)(s2 > cap ? (cap < 1 ? 1 : cap) : s2);
      w.rps2 = round_up(nerf_cdiv(Mp, w.S2), 64);
    }
    w.np = (float*)take((int64_t)w.S2 * NPS * 4);
  }
  w.bytes = (int64_t)(p - (char*)base);
  return w;
}

// ------------------------------------------------------------------ elementwise kernels

__global__ void to_bf16_kernel(const float* __restrict__ src, int64_t n, nerf_bf16* __restrict__ dst) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  if (i + 4 <= n) {
    const float4 v = *reinterpret_cast<const float4*>(src + i);
    *reinterpret_cast<uint2*>(dst + i) = make_uint2(nerf_pack_bf16x2(v.x, v.y), nerf_pack_bf16x2(v.z, v.w));
  } else {
    for (int64_t k = i; k < n; ++k) dst[k] = (nerf_bf16)src[k];
  }
}

// batched transpose fp32 -> bf16: dst_i[c][r] = src_i[r][c] (src pitch lds_i)
struct TJobB {
  const float* src;
  nerf_bf16* dst;
  int rows, cols, lds;
};
struct TJobsB {
  TJobB j[10];
};
__global__ void transpose_bf16_kernel(TJobsB jobs) {
  const TJobB J = jobs.j[blockIdx.z];
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  if (r0 >= J.rows || c0 >= J.cols) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < J.rows && c < J.cols) ? J.src[(int64_t)r * J.lds + c] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < J.cols && r < J.rows) J.dst[(int64_t)c * J.rows + r] = (nerf_bf16)tile[tx][y];
  }
}

// xyz PE (models/encodings.py:437-444, L = 10, include_input) of x_d[:, :3] into X3E cols 256..319 (bf16).
__global__ void pe_xyz_bf16_kernel(const float* __restrict__ xd, int64_t M, int64_t Mp, nerf_bf16* __restrict__ X3E) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= Mp) return;
  uint4* q = reinterpret_cast<uint4*>(X3E + m * 320 + 256);
  float v[64];
  if (m >= M) {
#pragma unroll
    for (int c = 0; c < 64; ++c) v[c] = 0.f;
  } else {
    const float x[3] = {xd[m * 6], xd[m * 6 + 1], xd[m * 6 + 2]};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v[k] = x[k];
      float band = 1.0f;
#pragma unroll
      for (int l = 0; l < 10; ++l) {
        float s, c;
        pe_sincos_bf16(x[k] * band, &s, &c);
        v[3 + k * 20 + l] = c;
        v[3 + k * 20 + 10 + l] = s;
        band *= 2.0f;
      }
    }
    v[63] = 0.f;
  }
#pragma unroll
  for (int c = 0; c < 8; ++c)
    q[c] = make_uint4(nerf_pack_bf16x2(v[8 * c], v[8 * c + 1]), nerf_pack_bf16x2(v[8 * c + 2], v[8 * c + 3]),
                      nerf_pack_bf16x2(v[8 * c + 4], v[8 * c + 5]), nerf_pack_bf16x2(v[8 * c + 6], v[8 * c + 7]));
}

// CIN[m] = [O16[m][1..15], d, dir PE (L = 4), 0...] in bf16 (meta_vanilla.py:109-121)
__global__ void build_cin_bf16_kernel(const float* __restrict__ xd, const float* __restrict__ O16, int64_t M,
                                      int64_t Mp, nerf_bf16* __restrict__ CIN) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= Mp) return;
  uint4* q = reinterpret_cast<uint4*>(CIN + m * 64);
  float v[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) v[c] = 0.f;
  if (m < M) {
    const float* o = O16 + m * 32;
#pragma unroll
    for (int c = 0; c < 15; ++c) v[c] = o[1 + c];
    const float d[3] = {xd[m * 6 + 3], xd[m * 6 + 4], xd[m * 6 + 5]};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v[15 + k] = d[k];
      float band = 1.0f;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        float s, c;
        pe_sincos_bf16(d[k] * band, &s, &c);
        v[18 + k * 8 + l] = c;
        v[18 + k * 8 + 4 + l] = s;
        band *= 2.0f;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 8; ++c)
    q[c] = make_uint4(nerf_pack_bf16x2(v[8 * c], v[8 * c + 1]), nerf_pack_bf16x2(v[8 * c + 2], v[8 * c + 3]),
                      nerf_pack_bf16x2(v[8 * c + 4], v[8 * c + 5]), nerf_pack_bf16x2(v[8 * c + 6], v[8 * c + 7]));
}

// (HO, training: the dense (o3, sigma_raw) row the fused tail reads, so a layered forward feeds the fused backward)
__global__ void head_out_b_kernel(const float* __restrict__ O3, const float* __restrict__ O16, int64_t M,
                                  float* __restrict__ out, float* __restrict__ HO) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const float* c = O3 + m * 32;
  const float sr = O16[m * 32];
  if (HO) reinterpret_cast<float4*>(HO)[m] = make_float4(c[0], c[1], c[2], sr);
  const float sg = expf(fminf(fmaxf(sr, -EXP_MAX), EXP_MAX));
  reinterpret_cast<float4*>(out)[m] = make_float4(sigmoidf_(c[0]), sigmoidf_(c[1]), sigmoidf_(c[2]), sg);
}

// d_rgb_sigma -> dO3 (bf16, cols 0..2) and dO16 col 0 (sigma); all other columns zero
__global__ void head_out_bwd_bf16_kernel(const float* __restrict__ g, const float* __restrict__ O3,
                                         const float* __restrict__ O16, int64_t M, int64_t Mp,
                                         nerf_bf16* __restrict__ dO3, nerf_bf16* __restrict__ dO16) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= Mp) return;
  float a = 0.f, b = 0.f, c = 0.f, ds = 0.f;
  if (m < M) {
    const float4 gg = reinterpret_cast<const float4*>(g)[m];
    const float* o = O3 + m * 32;
    const float s0 = sigmoidf_(o[0]), s1 = sigmoidf_(o[1]), s2 = sigmoidf_(o[2]);
    a = gg.x * (s0 * (1.0f - s0));
    b = gg.y * (s1 * (1.0f - s1));
    c = gg.z * (s2 * (1.0f - s2));
    ds = gg.w * expf(fminf(fmaxf(O16[m * 32], -EXP_MAX), EXP_MAX));
  }
  uint4* q3 = reinterpret_cast<uint4*>(dO3 + m * 32);
  uint4* q16 = reinterpret_cast<uint4*>(dO16 + m * 32);
  const uint4 z = make_uint4(0, 0, 0, 0);
  q3[0] = make_uint4(nerf_pack_bf16x2(a, b), nerf_pack_bf16x2(c, 0.f), 0, 0);
  q3[1] = z; q3[2] = z; q3[3] = z;
  // dO16: col 0 = d sigma_raw; cols 1..15 are written by geo_bwd, cols 16..31 zero
  reinterpret_cast<nerf_bf16*>(q16)[0] = (nerf_bf16)ds;
  q16[2] = z; q16[3] = z;
}

// dO16[m][1..15] = dCIN[m][0..14] (bf16)
__global__ void geo_bwd_bf16_kernel(const float* __restrict__ dCIN, int64_t Mp, nerf_bf16* __restrict__ dO16) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= Mp * 15) return;
  const int64_t m = idx / 15;
  const int c = (int)(idx - m * 15);
  dO16[m * 32 + 1 + c] = (nerf_bf16)dCIN[m * 32 + c];
}

// ------------------------------------------------------------------ launch helpers

template <int BM, int BN, int WAVES_M, int EPI, int OUT_BF16>
int launch_ntb(const nerf_bf16* A, int lda, const nerf_bf16* B, int ldb, const float* bias, void* C, int ldc,
               const uint32_t* mbits, uint32_t* mbits_out, int64_t M, int N, int K, hipStream_t st) {
  if (M % BM || N % BN || K % 32) return NERF_E_ARG;
  const int ntn = N / BN;
  const int64_t nblk = (M / BM) * ntn;
  gemm_nt_bf16_kernel<BM, BN, WAVES_M, EPI, OUT_BF16, 32, 3><<<(unsigned)nblk, 256, 0, st>>>(
      A, lda, B, ldb, bias, C, ldc, mbits, N / 32, mbits_out, K, ntn);
  return NERF_OK;
}

// weights-stationary persistent kernel (gemm_bf16.hpp, gemm_nt_bf16_wsr): one 512-thread block per CU
template <int K, int EPI, int OUT_BF16, int STAGES>
int launch_wsr(const nerf_bf16* A, int lda, const nerf_bf16* B, int ldb, const float* bias, void* C, int ldc,
               const uint32_t* mbits, uint32_t* mbits_out, int64_t M, int N, hipStream_t st) {
  if (M % 256 || N % 128) return NERF_E_ARG;
  const int ntn = N / 128;
  gemm_nt_bf16_wsr_kernel<K, 128, EPI, OUT_BF16, STAGES><<<256, 512, 0, st>>>(A, lda, B, ldb, bias, C, ldc, mbits, N / 32,
                                                                             mbits_out, ntn, (int)(M / 256));
  return NERF_OK;
}

template <int EPI, int OUT_BF16>
int ntb(const nerf_bf16* A, int lda, const nerf_bf16* B, int ldb, const float* bias, void* C, int ldc,
        const uint32_t* mbits, uint32_t* mbits_out, int64_t M, int N, int K, hipStream_t st) {
  if ((N == 256 || N == 128) && OUT_BF16) {  // the trunk / colour-0 layers: HBM-bound, weights stationary
    if (K == 256) return launch_wsr<256, EPI, OUT_BF16, 5>(A, lda, B, ldb, bias, C, ldc, mbits, mbits_out, M, N, st);
    if (K == 320) return launch_wsr<320, EPI, OUT_BF16, 4>(A, lda, B, ldb, bias, C, ldc, mbits, mbits_out, M, N, st);
    if (K == 64) return launch_wsr<64, EPI, OUT_BF16, 5>(A, lda, B, ldb, bias, C, ldc, mbits, mbits_out, M, N, st);
  }
  if (N == 256 || N == 128)
    return launch_ntb<128, 128, 2, EPI, OUT_BF16>(A, lda, B, ldb, bias, C, ldc, mbits, mbits_out, M, N, K, st);
  if (N == 32) return launch_ntb<256, 32, 4, EPI, OUT_BF16>(A, lda, B, ldb, bias, C, ldc, mbits, mbits_out, M, N, K, st);
  return NERF_E_ARG;
}

// one 64-column block of K (trunk.0, the K = 320 remainder of trunk.4, colour.0)
int narrowb(const nerf_bf16* G, int ldg, const nerf_bf16* X, int ldx, float* P, int ldp, float* Pb, int64_t slab,
            const WSB& w, int N, hipStream_t st) {
  // 128 x 64 tiles, 64 rows per slab; measured per fine launch on MI355X: 111 us vs 64 x 64 tiles at 32 / 64
  // rows 119 / 133 us (the fp32 path prefers the smaller tile)
  gemm_wgrad_bf16_kernel<128, 64, 2, 64><<<(N / 128) * w.S, 256, 0, st>>>(G, ldg, X, ldx, P, ldp, Pb, slab, w.rps,
                                                                         w.Mp, 1, N / 128);
  return NERF_OK;
}

int wgradb(const nerf_bf16* G, int ldg, const nerf_bf16* X, int ldx, int tensor_w, const WSB& w, int N, int K,
           hipStream_t st) {
  const Layout& L = layout();
  float* P = w.partial + L.off[tensor_w];
  float* Pb = w.partial + L.off[tensor_w + 1];
  const int ldp = L.cols[tensor_w];
  const int64_t slab = L.total;
  if (N % 32 || K % 32) return NERF_E_ARG;
  if (N >= 128 && K > 128 && K % 128 == 64) {  // trunk.4 (K = 320): 128x128 tiles + a 128x64 column
    const int kb = K - 64;
    TRY(wgradb(G, ldg, X, ldx, tensor_w, w, N, kb, st));
    return narrowb(G, ldg, X + kb, ldx, P + kb, ldp, nullptr, slab, w, N, st);
  }
  if (N >= 128 && K % 128 == 0) {
    const int nt = (N / 128) * (K / 128);
#ifndef NERF_WGRAD_MR
#define NERF_WGRAD_MR 32
#endif
    gemm_wgrad_bf16_kernel<128, 128, 2, NERF_WGRAD_MR><<<nt * w.S, 256, 0, st>>>(G, ldg, X, ldx, P, ldp, Pb, slab, w.rps, w.Mp,
                                                                 K / 128, nt);
  } else if (N >= 128 && K == 64) {
    return narrowb(G, ldg, X, ldx, P, ldp, Pb, slab, w, N, st);
  } else if (N == 32 && K % 128 == 0) {
    const int nt = K / 128;
    gemm_wgrad_bf16_kernel<32, 128, 1, 64><<<nt * w.S, 256, 0, st>>>(G, ldg, X, ldx, P, ldp, Pb, slab, w.rps, w.Mp,
                                                                K / 128, nt);
  } else {
    return NERF_E_ARG;
  }
  return NERF_OK;
}

}  // namespace

// Path selection is an explicit argument (include/nerf_amd.h NERF_BF16_LAYERED_*): NERF_BF16_LAYERED_BWD selects the
// layered backward (a dgrad and a wgrad GEMM launch per trunk layer; its forward also writes the ReLU bitmasks),
// NERF_BF16_LAYERED_FWD the layer-by-layer forward (one GEMM launch per layer, activations through HBM).  The
// defaults are the fused kernels (mlp_bf16_fused.hpp, mlp_bf16_bwd.hpp); the layered launches are their bitwise
// references in the tests.

// The fused backward's W_i^T images of trunk layers 1..7 (bf16 [k][n], first 256 input columns; W.WTf) through 32 x 32
// LDS tiles, coalesced on both sides.  Made by the training FORWARD, with the colour layer-0 fragments the fused tail
// reads (W.Wf), so that the backward launches no weight preparation of its own: on the two-stream schedule (coarse
// backward beside the fine backward) each such small launch queued behind the other net's persistent workgroups for
// ~90 us of the fine chain (profiles/r06/a17/step_bf16.txt).  The backward's weights are the forward's (the
// workspace holds that forward's activations), so the images are this call's.
void bwd_weight_images(const float* w, const WSB& W, hipStream_t st) {
  const Layout& L = layout();
  TJobsB jobs{};
  for (int i = 1; i < 8; ++i)
    jobs.j[i - 1] = TJobB{w + L.off[2 * i], W.WTf + (int64_t)(i - 1) * nerf_bwd::WT_LAYER, 256, 256, KPAD[i]};
  transpose_bf16_kernel<<<dim3(8, 8, 7), 256, 0, st>>>(jobs);
}

int fused_forward(const float* w, const float* x_d, int64_t M, float* rgb_sigma, const WSB& W, int training,
                  bool layered_bwd, hipEvent_t* ev, hipStream_t st) {
  using namespace nerf_fused;
  const Layout& L = layout();
  const FragTab T = frag_tab();
  const int64_t Mp = W.Mp;
  for (int t = 0; t < NT; ++t)
    if (L.off[t] != lay_off(t)) return NERF_E_ARG;  // device-side compile-time offsets must match the layout
  if (training) {  // the kernel addresses Y[i] / MB[i] from one base each
    for (int i = 0; i < 8; ++i) {
      if (i != 3 && W.Y[i] != W.Y[0] + (int64_t)(i < 3 ? i : i - 1) * Mp * 256) return NERF_E_ARG;
      if (W.MB[i] != W.MB[0] + (int64_t)i * Mp * 8) return NERF_E_ARG;
    }
  }
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu <= 0) n_cu = 256;
  }
  frag_pack_kernel<<<(unsigned)nerf_cdiv(T.off[FT] / 8, 256), 256, 0, st>>>(w, W.Wf, T);
  if (training) bwd_weight_images(w, W, st);  // (also beside a layered backward's masks: either backward may follow)
  FusedArgs A{};  // (the io waves encode x_d themselves: io_encode, no pe_prefill_bf16_kernel launch)
  A.xd = x_d;
  A.wf = W.Wf;
  A.w = w;
  A.X3E = W.X3E;
  A.Y = training ? W.Y[0] : nullptr;
  A.MB = training ? W.MB[0] : nullptr;
  A.O16 = W.O16; A.CIN = W.CIN; A.C0 = W.C0; A.MC0 = training ? W.MC0 : nullptr; A.O3 = W.O3; A.HO = W.HO;
  A.out = rgb_sigma;
  A.M = M;
  A.Mp = Mp;
  A.ntiles = (int)(Mp / BMF);  // Mp is a multiple of 256: whole 128-row tiles
  const int grid = A.ntiles < n_cu ? A.ntiles : n_cu;  // persistent, one workgroup per CU (LDS ~87 KB)
  if (ev) (void)hipEventRecord(ev[0], st);
  if (training && layered_bwd)  // the layered backward reads ReLU bitmasks
    mlp_fwd_fused_bf16_kernel<true, true><<<grid, 512, 0, st>>>(A);
  else if (training)
    mlp_fwd_fused_bf16_kernel<true, false><<<grid, 512, 0, st>>>(A);
  else
    mlp_fwd_fused_bf16_kernel<false, false><<<grid, 512, 0, st>>>(A);
  if (ev)
    for (int i = 1; i < 16; ++i) (void)hipEventRecord(ev[i], st);  // ev[0] -> ev[1] brackets the fused launch
  return nerf_launch_status();
}

// the 11 bias tensors of the packed layout (packed offsets / lengths): the fp16 build rounds every other sum
struct BiasTab {
  int64_t off[11];
  int len[11];
};
inline BiasTab bias_tab() {
  const Layout& L = layout();
  BiasTab b{};
  for (int t = 0; t < 11; ++t) {
    b.off[t] = L.off[2 * t + 1];
    b.len[t] = L.rows[2 * t + 1];
  }
  return b;
}

// Final reduce of the fused backward (fixed order, bitwise reproducible): element e of the packed gradient =
//   trunk.0 W / b and trunk.4 W[:, 256:320]  sum over the S2 narrow sub-slabs (np);
//   everything else                          sum over the S split slabs, plus (e >= off16: head / colour) the S
//                                            second-half tail slabs after them.
__global__ __launch_bounds__(256) void reduce_fused_bf16_kernel(const float* __restrict__ partial, int64_t slab, int S,
                                                                const float* __restrict__ partial2, int64_t slab2,
                                                                int64_t off16, const float* __restrict__ np, int S2,
                                                                float* __restrict__ dst, int64_t n4, int accumulate,
                                                                int64_t off0, int64_t off1, int64_t off8, BiasTab bt) {
  // gemm.hpp's RG-group order (one wave per group of slabs, 64 elements per block; grid cdiv(n4, 64)): the 256-wide
  // trunk weights sum exactly as the layered path's reduce_splits_kernel does
  __shared__ float4 part[2][RG][64];
  const int el = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 64 + el;
  const int64_t e = 4 * i;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  int64_t nofs = -1;  // offset in the narrow slab, or -1
  if (e >= off0 && e < off0 + 256 * 64) nofs = e - off0;
  else if (e >= off1 && e < off1 + 256) nofs = 32768 + (e - off1);
  else if (e >= off8 && e < off8 + 256 * 320 && (e - off8) % 320 >= 256) {
    const int64_t n = (e - off8) / 320, k = (e - off8) % 320 - 256;
    nofs = 16384 + n * 64 + k;
  }
  const bool live = i < n4, two = live && nofs < 0 && e >= off16;
  part[0][g][el] = !live ? z : (nofs >= 0 ? rg_group_sum(np + nofs, NPS, S2, g) : rg_group_sum(partial + e, slab, S, g));
  part[1][g][el] = two ? rg_group_sum(partial2 + (e - off16), slab2, S, g) : z;
  __syncthreads();
  if (g == 0 && live) {
    if constexpr (NERF_F16) {
      // the reference's weight gradient is an fp16 matmul output, cast to fp32 and then accumulated in fp32: this
      // call's sum is rounded to fp16 once (overflow -> inf, which GradScaler then sees), biases stay fp32 sums
      float4 a = z;
#pragma unroll
      for (int k = 0; k < RG; ++k) rg_add(a, part[0][k][el]);
      if (two) {
#pragma unroll
        for (int k = 0; k < RG; ++k) rg_add(a, part[1][k][el]);
      }
      bool bias = false;
#pragma unroll
      for (int t = 0; t < 11; ++t) bias |= e >= bt.off[t] && e < bt.off[t] + bt.len[t];
      if (!bias) {
        a.x = (float)(_Float16)a.x; a.y = (float)(_Float16)a.y; a.z = (float)(_Float16)a.z; a.w = (float)(_Float16)a.w;
      }
      if (accumulate) {
        const float4 d = reinterpret_cast<const float4*>(dst)[i];
        a = make_float4(d.x + a.x, d.y + a.y, d.z + a.z, d.w + a.w);
      }
      reinterpret_cast<float4*>(dst)[i] = a;
    } else {
      float4 a = accumulate ? reinterpret_cast<const float4*>(dst)[i] : z;
#pragma unroll
      for (int k = 0; k < RG; ++k) rg_add(a, part[0][k][el]);
      if (two) {
#pragma unroll
        for (int k = 0; k < RG; ++k) rg_add(a, part[1][k][el]);
      }
      reinterpret_cast<float4*>(dst)[i] = a;
    }
  }
}

// The fused bf16 backward: ONE tail launch (mlp_bf16_tail.hpp: head-output derivatives, colour branch, head dgrad +
// wgrad -> dZ7), ONE launch per 256-wide trunk layer 7..1 (mlp_bf16_bwd.hpp: input + weight gradient), the narrow
// wgrads of trunk.0 and of trunk.4's encoding columns, then one deterministic split reduce (the tail's second-half
// sums added after the slab terms).
int fused_backward(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, const WSB& W,
                   hipEvent_t* ev, hipStream_t st) {
  const Layout& L = layout();
  const int64_t Mp = W.Mp;
  if (W.rps % nerf_bwd::TR) return NERF_E_ARG;
  const int S8 = (W.S + 7) / 8 * 8;
  // the fused tail recomputes C0 with the forward's colour layer-0 fragments (W.Wf) and the layers read the W_i^T
  // images (W.WTf): both made by the training forward, fused or layered (bwd_weight_images)
  const nerf_fused::FragTab FT_ = nerf_fused::frag_tab();
  nerf_tail::TailArgs T{};
  T.w = w; T.g = d_rgb_sigma; T.HO = W.HO; T.Y7 = W.Y[7]; T.CIN = W.CIN;
  T.wfc0 = W.Wf + FT_.off[9];
  T.dZ7 = W.dA; T.partial = W.partial; T.partial2 = W.partial2;
  T.slab = L.total; T.off16 = L.off[16]; T.cslab = L.total - L.off[16];
  T.off17 = L.off[17]; T.off18 = L.off[18]; T.off19 = L.off[19]; T.off20 = L.off[20]; T.off21 = L.off[21];
  T.rps = W.rps; T.M = M; T.Mp = Mp; T.S = W.S;
  if (ev) (void)hipEventRecord(ev[2], st);
  nerf_tail::bwd_tail_bf16_kernel<<<2 * S8, 768, 0, st>>>(T);
  if (ev) (void)hipEventRecord(ev[3], st);
  nerf_bf16* dcur = W.dA;
  nerf_bf16* dnext = W.dB;
  for (int i = 7; i >= 1; --i) {
    nerf_bwd::LayerArgs A{};
    A.G = dcur;
    A.X = (i == 4) ? W.X3E : W.Y[i - 1];
    A.ldx = (i == 4 || i - 1 == 3) ? 320 : 256;
    A.WT = W.WTf + (int64_t)(i - 1) * nerf_bwd::WT_LAYER;
    A.D = dnext;
    A.P = W.partial + L.off[2 * i];
    A.Pb = W.partial + L.off[2 * i + 1];
    A.ldp = L.cols[2 * i];
    A.slab = L.total;
    A.rps = W.rps;
    A.Mp = Mp;
    A.S = W.S;
    if (ev) (void)hipEventRecord(ev[4 * i], st);
    nerf_bwd::bwd_layer_bf16_kernel<<<2 * S8, 768, 0, st>>>(A);
    if (ev) {
      (void)hipEventRecord(ev[4 * i + 1], st);
      (void)hipEventRecord(ev[4 * i + 2], st);
      (void)hipEventRecord(ev[4 * i + 3], st);
    }
    if (i == 4)  // the encoding columns of trunk.4 (no input gradient): narrow wgrad over the S2 sub-splits
      gemm_wgrad_bf16_kernel<128, 64, 2, 64><<<2 * W.S2, 256, 0, st>>>(dcur, 256, W.X3E + 256, 320, W.np + 16384, 64,
                                                                      nullptr, NPS, W.rps2, Mp, 1, 2);
    nerf_bf16* t = dcur; dcur = dnext; dnext = t;
  }
  if (ev) (void)hipEventRecord(ev[0], st);
  gemm_wgrad_bf16_kernel<128, 64, 2, 64><<<2 * W.S2, 256, 0, st>>>(dcur, 256, W.X3E + 256, 320, W.np, 64, W.np + 32768,
                                                                  NPS, W.rps2, Mp, 1, 2);
  if (ev) (void)hipEventRecord(ev[1], st);
  const int64_t n4 = L.total / 4;
  reduce_fused_bf16_kernel<<<(unsigned)nerf_cdiv(n4, 64), 256, 0, st>>>(
      W.partial, L.total, W.S, W.partial2, L.total - L.off[16], L.off[16], W.np, W.S2, d_w, n4, accumulate, L.off[0],
      L.off[1], L.off[8], bias_tab());
  return nerf_launch_status();
}

}  // namespace NERF_H16NS
using namespace NERF_H16NS;

extern "C" int64_t NERF_H16_FN(nerf_mlp_workspace_bytes)(int64_t M, int training) {
  if (M < 0) return -1;
  return carve_b(nullptr, M, training).bytes + 256;
}

extern "C" int NERF_H16_FN(nerf_mlp_fwd)(const float* w, const float* x_d, int64_t M, float* rgb_sigma, void* ws,
                                 int64_t ws_bytes, int training, int flags, hipEvent_t* ev, hipStream_t st) {
  NERF_CHECK_ARG(w && ws && M >= 0 && (M == 0 || (x_d && rgb_sigma)));  // an empty batch may pass null rows
  if (flags & ~(NERF_F16 ? 0 : (NERF_BF16_LAYERED_FWD | NERF_BF16_LAYERED_BWD))) return NERF_E_ENUM;
  if (!nerf_aligned16(w) || !nerf_aligned16(ws) || !nerf_aligned16(rgb_sigma)) return NERF_E_ALIGN;
  const WSB W = carve_b(ws, M, training);
  if (ws_bytes < W.bytes) return NERF_E_WORKSPACE;
  if (M == 0) return NERF_OK;
  const Layout& L = layout();
  const int64_t Mp = W.Mp;
  auto Wb = [&](int t) { return W.Wb + L.off[t]; };
  auto Bias = [&](int t) { return w + L.off[t]; };
  if (!(flags & NERF_BF16_LAYERED_FWD))
    return fused_forward(w, x_d, M, rgb_sigma, W, training, (flags & NERF_BF16_LAYERED_BWD) != 0, ev, st);

  to_bf16_kernel<<<(unsigned)nerf_cdiv(L.total / 4 + 1, 256), 256, 0, st>>>(w, L.total, W.Wb);
  pe_xyz_bf16_kernel<<<(unsigned)nerf_cdiv(Mp, 256), 256, 0, st>>>(x_d, M, Mp, W.X3E);
  const nerf_bf16* in = W.X3E + 256;
  int ld_in = 320;
  for (int i = 0; i < 8; ++i) {
    nerf_bf16* out = W.Y[i];
    const int ld_out = training ? (i == 3 ? 320 : 256) : ((i % 2 == 0) ? 256 : 320);
    if (i == 4) { in = W.X3E; ld_in = 320; }
    if (ev) (void)hipEventRecord(ev[2 * i], st);
    TRY((ntb<EPI_BIAS_RELU, 1>(in, ld_in, Wb(2 * i), KPAD[i], Bias(2 * i + 1), out, ld_out, nullptr,
                               training ? W.MB[i] : nullptr, Mp, 256, KPAD[i], st)));
    if (ev) (void)hipEventRecord(ev[2 * i + 1], st);
    in = out;
    ld_in = ld_out;
  }
  TRY((ntb<EPI_BIAS, 0>(in, ld_in, Wb(16), 256, Bias(17), W.O16, 32, nullptr, nullptr, Mp, 32, 256, st)));
  build_cin_bf16_kernel<<<(unsigned)nerf_cdiv(Mp, 256), 256, 0, st>>>(x_d, W.O16, M, Mp, W.CIN);
  TRY((ntb<EPI_BIAS_RELU, 1>(W.CIN, 64, Wb(18), 64, Bias(19), W.C0, 128, nullptr, training ? W.MC0 : nullptr, Mp,
                             128, 64, st)));
  TRY((ntb<EPI_BIAS, 0>(W.C0, 128, Wb(20), 128, Bias(21), W.O3, 32, nullptr, nullptr, Mp, 32, 128, st)));
  head_out_b_kernel<<<(unsigned)nerf_cdiv(M, 256), 256, 0, st>>>(W.O3, W.O16, M, rgb_sigma, training ? W.HO : nullptr);
  if (training) {  // the fused backward's weight images (bwd_weight_images): either backward may follow
    const nerf_fused::FragTab T = nerf_fused::frag_tab();
    nerf_fused::frag_pack_kernel<<<(unsigned)nerf_cdiv(T.off[nerf_fused::FT] / 8, 256), 256, 0, st>>>(w, W.Wf, T);
    bwd_weight_images(w, W, st);
  }
  return nerf_launch_status();
}

extern "C" int NERF_H16_FN(nerf_mlp_bwd)(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate,
                                 void* ws, int64_t ws_bytes, int flags, hipEvent_t* ev, hipStream_t st) {
  NERF_CHECK_ARG(w && d_w && ws && M >= 0 && (M == 0 || d_rgb_sigma));
  if (flags & ~(NERF_F16 ? 0 : (NERF_BF16_LAYERED_FWD | NERF_BF16_LAYERED_BWD))) return NERF_E_ENUM;
  if (!nerf_aligned16(w) || !nerf_aligned16(ws) || !nerf_aligned16(d_w) || !nerf_aligned16(d_rgb_sigma))
    return NERF_E_ALIGN;
  const WSB W = carve_b(ws, M, 1);
  if (ws_bytes < W.bytes) return NERF_E_WORKSPACE;
  const Layout& L = layout();
  if (M == 0) {
    if (!accumulate) (void)hipMemsetAsync(d_w, 0, L.total * sizeof(float), st);
    return nerf_launch_status();
  }
  const int64_t Mp = W.Mp;
  auto Wt = [&](int t) { return w + L.off[t]; };

  if (!(flags & NERF_BF16_LAYERED_BWD)) return fused_backward(w, M, d_rgb_sigma, d_w, accumulate, W, ev, st);
  // bf16 transposed weights for the input-gradient GEMMs (the bf16 forward copy W.Wb is reused for nothing
  // here: the backward GEMMs contract over the output dimension)
  nerf_bf16* T = W.WTb;
  nerf_bf16* WTi[8] = {nullptr};
  TJobsB jobs{};
  int nj = 0;
  for (int i = 1; i < 8; ++i) {
    WTi[i] = T;
    jobs.j[nj++] = TJobB{Wt(2 * i), T, 256, 256, KPAD[i]};
    T += 65536;
  }
  nerf_bf16* Wht = T;  jobs.j[nj++] = TJobB{Wt(16), Wht, 32, 256, 256};  T += 256 * 32;
  nerf_bf16* Wc1t = T; jobs.j[nj++] = TJobB{Wt(20), Wc1t, 32, 128, 128}; T += 128 * 32;
  nerf_bf16* Wc0t = T; jobs.j[nj++] = TJobB{Wt(18), Wc0t, 128, 32, 64};
  transpose_bf16_kernel<<<dim3(8, 8, nj), 256, 0, st>>>(jobs);

  head_out_bwd_bf16_kernel<<<(unsigned)nerf_cdiv(Mp, 256), 256, 0, st>>>(d_rgb_sigma, W.O3, W.O16, M, Mp, W.dO3,
                                                                         W.dO16);
  // colour MLP
  TRY((ntb<EPI_MASK, 1>(W.dO3, 32, Wc1t, 32, nullptr, W.dC0, 128, W.MC0, nullptr, Mp, 128, 32, st)));
  TRY(wgradb(W.dO3, 32, W.C0, 128, 20, W, 32, 128, st));
  TRY((ntb<EPI_NONE, 0>(W.dC0, 128, Wc0t, 128, nullptr, W.dCIN, 32, nullptr, nullptr, Mp, 32, 128, st)));
  TRY(wgradb(W.dC0, 128, W.CIN, 64, 18, W, 128, 64, st));
  geo_bwd_bf16_kernel<<<(unsigned)nerf_cdiv(Mp * 15, 256), 256, 0, st>>>(W.dCIN, Mp, W.dO16);
  // heads -> dZ7
  nerf_bf16* dcur = W.dA;
  nerf_bf16* dnext = W.dB;
  if (ev) (void)hipEventRecord(ev[2], st);
  TRY((ntb<EPI_MASK, 1>(W.dO16, 32, Wht, 32, nullptr, dcur, 256, W.MB[7], nullptr, Mp, 256, 32, st)));
  if (ev) (void)hipEventRecord(ev[3], st);
  TRY(wgradb(W.dO16, 32, W.Y[7], 256, 16, W, 32, 256, st));
  // trunk
  for (int i = 7; i >= 0; --i) {
    const nerf_bf16* X = (i == 0) ? W.X3E + 256 : (i == 4 ? W.X3E : W.Y[i - 1]);
    const int ldx = (i == 0 || i == 4) ? 320 : ((i - 1) == 3 ? 320 : 256);
    if (ev) (void)hipEventRecord(ev[4 * i], st);
    TRY(wgradb(dcur, 256, X, ldx, 2 * i, W, 256, KPAD[i], st));
    if (ev) (void)hipEventRecord(ev[4 * i + 1], st);
    if (i > 0) {
      if (ev) (void)hipEventRecord(ev[4 * i + 2], st);
      TRY((ntb<EPI_MASK, 1>(dcur, 256, WTi[i], 256, nullptr, dnext, 256, W.MB[i - 1], nullptr, Mp, 256, 256, st)));
      if (ev) (void)hipEventRecord(ev[4 * i + 3], st);
      nerf_bf16* t = dcur; dcur = dnext; dnext = t;
    }
  }
  const int64_t n4 = L.total / 4;
  reduce_splits_kernel<<<(unsigned)nerf_cdiv(n4, 64), 256, 0, st>>>(W.partial, L.total, W.S, d_w, n4, accumulate);
  return nerf_launch_status();
}
