// The vanilla NeRF expert — 8x256 ReLU trunk with the [h|enc] skip at layer 4, sigma/geo heads,
// 2-layer colour MLP — forward and backward on fp32 MFMA (gfx950).
//
// Restates (psklavos1/NeRF-Sys adaptive_nerf/):
//   MetaNeRF.density / color / forward   models/inr/meta_vanilla.py:109-154 (ctor :36-97)
//   MetaLinear.forward (x W^T + b)       models/metamodule/metamodule.py:140-156
//   FrequencyEncoder (xyz L=10, dir L=4) models/encodings.py:437-444
//   trunc_exp fwd/bwd                    models/trunc_exp.py:30-61
// as the expert contract x_d (M,6) -> (M,4) of models/inr/meta_ngp.py:226-241.
//
// Activation layout in the caller's workspace (Mp = M rounded up to 256, row-major, fp32):
//   X3E [Mp][320] : cols 0..255 = trunk.3 output, cols 256..318 = xyz encoding, col 319 = 0
//                   (so trunk.4 reads cat([h, enc]) with K = 320 and no copy; trunk.0 reads cols 256..319)
//   Y0..Y2, Y4..Y7 [Mp][256], HO [Mp][4] (colour pre-activations 0..2, sigma_raw), CIN [Mp][64] (geo | dir-enc |
//   0), C0 [Mp][128].  Backward adds dA/dB [Mp][256], dO16 [Mp][16] (from the fused colour-branch backward),
//   transposed trunk weights, and S split-M partial slabs of the packed gradient.
#include "gemm.hpp"
#include "gemm_x6.hpp"
#include "gemm_x6s.hpp"
#include "mlp_common.hpp"
#include "mlp_tail.hpp"
#include "mlp_fwd_tail.hpp"

namespace {
using namespace nerf_mlp;

struct WS {
  int64_t Mp;
  float *X3E, *Y[8], *HO, *CIN, *C0;
  uint32_t* MB[8];  // ReLU bitmasks of the trunk outputs [Mp][8] (colour layer 0 re-derives its mask from C0 > 0)
  // backward
  float *dA, *dB, *dO16, *WT, *partial, *partial2;
  float* dZ[8];  // two-stream backward (training == 2): one input-gradient buffer per trunk layer (dZ_i of trunk.i)
  nerf_bf16* WPf;  // bf16 piece planes of the trunk weights (split GEMMs): layer i at x6_fwd_off(i), [3][256][KPAD_i]
  nerf_bf16* WPb;  // ... of the transposed trunk weights (input gradients): layer i >= 1 at 3 * 65536 * (i - 1)
  int S;
  int64_t rps;
  int64_t bytes;
};

constexpr int64_t WT_FLOATS = 7 * 65536;
// bf16 piece planes (gemm_x6.hpp): forward 3 x 256 x sum(KPAD) bf16, input gradient 7 x 3 x 256 x 256 bf16
inline int64_t x6_fwd_off(int i) {
  int64_t o = 0;
  for (int j = 0; j < i; ++j) o += 3 * 256 * (int64_t)KPAD[j];
  return o;
}
constexpr int64_t X6_BWD_BF16 = 7 * 3 * 65536;
// the head backward (dZ7, head weight / bias sums) is one pass (head_bwd_kernel); the second-half sums of the split
// walks (head + colour tensors) start at P2BASE
#define P2BASE (layout().off[16])

WS carve(void* base, int64_t M, int training) {
  WS w{};
  w.Mp = round_up(M < 1 ? 1 : M, 256);
  const int64_t Mp = w.Mp;
  float* p = reinterpret_cast<float*>(base);
  auto take = [&](int64_t n) {
    float* q = p;
    p += round_up(n, 64);
    return q;
  };
  w.X3E = take(Mp * 320);
  w.WPf = reinterpret_cast<nerf_bf16*>(take(x6_fwd_off(8) / 2));
  if (training) {
    for (int i = 0; i < 8; ++i) w.Y[i] = (i == 3) ? w.X3E : take(Mp * 256);
  } else {
    float* q = take(Mp * 256);
    for (int i = 0; i < 8; ++i) w.Y[i] = (i % 2 == 0) ? q : w.X3E;  // ping-pong
  }
  w.HO = take(Mp * 4);
  w.CIN = take(Mp * 64);
  w.C0 = take(Mp * 128);
  if (training) {
    for (int i = 0; i < 8; ++i) w.MB[i] = reinterpret_cast<uint32_t*>(take(Mp * 8));
    if (training == 2) {  // the weight-gradient stream reads dZ_i while the input-gradient chain runs ahead
      for (int i = 0; i < 8; ++i) w.dZ[i] = take(Mp * 256);
      w.dA = w.dZ[7];
      w.dB = w.dZ[6];
    } else {
      w.dA = take(Mp * 256);
      w.dB = take(Mp * 256);
    }
    w.dO16 = take(Mp * 16);  // [Mp][16]: the head-output gradient, written by color_bwd, read by head_bwd
    w.WT = take(WT_FLOATS);
    w.WPb = reinterpret_cast<nerf_bf16*>(take(X6_BWD_BF16 / 2));
    w.S = n_splits(Mp);
    w.rps = round_up(nerf_cdiv(Mp, w.S), 64);  // whole slabs for every wgrad MR
    w.partial = take((int64_t)w.S * layout().total);
    w.partial2 = take((int64_t)(TAIL_NQ - 1) * w.S * (layout().total - P2BASE));  // head + colour sums, parts 1..
  }
  w.bytes = (int64_t)((char*)p - (char*)base);
  return w;
}

inline int ld_of(const WS& w, int i) { return (i == 3) ? 320 : 256; }

// ------------------------------------------------------------------ elementwise kernels

// xyz positional encoding of x_d[:, :3] into X3E cols 256..319 (pad col 319 = 0; rows >= M zero).
// One thread per sample row computes its 64 values; a wave's 64 rows then leave through a per-wave LDS tile, 32 columns
// at a time, so that each store instruction writes 8 rows x 128 B (whole lines) instead of one 16-B piece of each of
// 64 rows 1280 B apart.  Same values, same bits.  Against the row-per-lane stores it measured within the noise (C2
// 225.3k vs 225.2k, profiles/r05/x6_variants_ab.txt): the kernel is bound by its 30 libm sincosf per row.  Tile pitch
// 33 floats: the row-per-lane writes of a column hit 64 distinct banks.
constexpr int PE_TP = 33;
__global__ __launch_bounds__(256) void pe_xyz_kernel(const float* __restrict__ xd, int64_t M, int64_t Mp,
                                                     float* __restrict__ X3E) {
  __shared__ float tile[4][64 * PE_TP];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t m0 = ((int64_t)blockIdx.x * 4 + wv) * 64;  // this wave's first row (Mp is a multiple of 256)
  if (m0 >= Mp) return;  // wave-uniform
  const int64_t m = m0 + lane;
  float v[64];
#pragma unroll
  for (int c = 0; c < 64; ++c) v[c] = 0.f;
  if (m < M) {
    const float x[3] = {xd[m * 6], xd[m * 6 + 1], xd[m * 6 + 2]};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v[k] = x[k];
      float band = 1.0f;
#pragma unroll
      for (int l = 0; l < 10; ++l) {
        float s, c;
        sincosf(x[k] * band, &s, &c);
        v[3 + k * 20 + l] = c;
        v[3 + k * 20 + 10 + l] = s;
        band *= 2.0f;
      }
    }
  }
  float* t = tile[wv];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int c = 0; c < 32; ++c) t[lane * PE_TP + c] = v[32 * hf + c];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // store i: rows 8 i + (lane >> 3), float4 (lane & 7) of the half
      const int r = 8 * i + (lane >> 3), q = lane & 7;
      const float* src = t + r * PE_TP + 4 * q;
      *reinterpret_cast<float4*>(X3E + (m0 + r) * 320 + 256 + 32 * hf + 4 * q) =
          make_float4(src[0], src[1], src[2], src[3]);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// batched transpose: dst_i[c][r] = src_i[r][c] for r < rows_i, c < cols_i  (src pitch lds_i)
struct TJob {
  const float* src;
  float* dst;
  int rows, cols, lds;
};
struct TJobs {
  TJob j[10];
};
__global__ void transpose_kernel(TJobs jobs) {
  const TJob J = jobs.j[blockIdx.z];
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  if (r0 >= J.rows || c0 >= J.cols) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int y = ty; y < 32; y += 8) {
    const int r = r0 + y, c = c0 + tx;
    tile[y][tx] = (r < J.rows && c < J.cols) ? J.src[(int64_t)r * J.lds + c] : 0.f;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int c = c0 + y, r = r0 + tx;
    if (c < J.cols && r < J.rows) J.dst[(int64_t)c * J.rows + r] = tile[tx][y];
  }
}

// ------------------------------------------------------------------ launch helpers

// 16x16x4 trunk forward / input-gradient GEMMs (gemm.hpp): waves per SIMD the register budget is sized for.
// tools/gemm_bench16.hip (MI355X, C2 fine-net shape, 9 interleaved rounds): fwd 0.839 / dgrad 0.817 ms per 256x256
// launch at 3 against 0.901 / 0.874 for the 32x32x2 kernel (2: 0.861 / 0.821, 4: 0.858; BK = 32: 0.957 / 0.940).
#ifndef NERF_NT16_MINW
#define NERF_NT16_MINW 3
#endif

// MINW = 4 waves per SIMD: the register budget (128 unified VGPR+AGPR per lane) that lets four 256-thread
// workgroups share a CU; measured +9..12 % over the unconstrained allocation (tools/gemm_bench.hip).
template <int BM, int BN, int WAVES_M, int EPI>
int launch_nt(const float* A, int lda, const float* B, int ldb, const float* bias, float* C, int ldc,
              const uint32_t* mbits, uint32_t* mbits_out, int64_t M, int N, int K, hipStream_t st) {
  if (M % BM || N % BN || K % 16) return NERF_E_ARG;
  const int ntn = N / BN;
  const int64_t nblk = (M / BM) * ntn;
#ifndef NERF_GEMM32
  if constexpr (BM == 128 && BN == 128 && WAVES_M == 2) {  // the trunk GEMMs: 16x16x4 form (gemm.hpp)
    gemm_nt16_kernel<128, 128, 2, EPI, NERF_NT16_MINW><<<(unsigned)nblk, 256, 0, st>>>(A, lda, B, ldb, bias, C, ldc, mbits,
                                                                                       N / 32, mbits_out, K, ntn);
    return NERF_OK;
  }
#endif
  gemm_nt_kernel<BM, BN, WAVES_M, EPI, (BN >= 128 ? 4 : 1)><<<(unsigned)nblk, 256, 0, st>>>(A, lda, B, ldb, bias, C, ldc, mbits,
                                                                           N / 32, mbits_out, K, ntn);
  return NERF_OK;
}

// dispatch on N for the trunk-like GEMMs.  mbits: ReLU bitmask [M][N/32] read by EPI_MASK; mbits_out:
// bitmask written by EPI_BIAS_RELU (nullable).
template <int EPI>
int nt(const float* A, int lda, const float* B, int ldb, const float* bias, float* C, int ldc, const uint32_t* mbits,
       uint32_t* mbits_out, int64_t M, int N, int K, hipStream_t st) {
  if (N == 256 || N == 128)
    return launch_nt<128, 128, 2, EPI>(A, lda, B, ldb, bias, C, ldc, mbits, mbits_out, M, N, K, st);
  if (N == 32) return launch_nt<256, 32, 4, EPI>(A, lda, B, ldb, bias, C, ldc, mbits, mbits_out, M, N, K, st);
  return NERF_E_ARG;
}

int wgrad(const float* G, int ldg, const float* X, int ldx, int tensor_w, const WS& w, int N, int K, hipStream_t st) {
  const Layout& L = layout();
  float* P = w.partial + L.off[tensor_w];
  float* Pb = w.partial + L.off[tensor_w + 1];
  const int ldp = L.cols[tensor_w];
  const int64_t slab = L.total;
  if (N % 32 || K % 32) return NERF_E_ARG;
  // one 256 x 64 block (trunk.0 and the K = 320 remainder of trunk.4): four 64 x 64 tiles per split (1024
  // workgroups) staging 32 rows per slab.  Measured on MI355X at the fine net's M (per launch): 256x64 tiles
  // at 16 / 32 rows 398 / 358 us, 128x64 323 us, 128x32 309 us, 64x64 at 16 rows 272 us, this 252 us.
  auto narrow = [&](const float* Xn, float* Pn, float* Pbn) {
    gemm_wgrad_kernel<64, 64, 2, 32><<<4 * w.S, 256, 0, st>>>(G, ldg, Xn, ldx, Pn, ldp, Pbn, slab, w.rps, w.Mp, 1, 4);
  };
  if (N == 256 && K == 64) {  // trunk.0
    narrow(X, P, Pb);
    return NERF_OK;
  }
  if (N >= 128 && K > 128 && K % 128 == 64) {  // trunk.4 (K = 320): 128x128 tiles + one 256x64 block
    if (N != 256) return NERF_E_ARG;
    const int kb = K - 64;
    const int e = wgrad(G, ldg, X, ldx, tensor_w, w, N, kb, st);
    if (e != NERF_OK) return e;
    narrow(X + kb, P + kb, nullptr);
    return NERF_OK;
  }
  if (N >= 128 && K % 128 == 0) {
    const int nt = (N / 128) * (K / 128);
    gemm_wgrad_kernel<128, 128, 2><<<nt * w.S, 256, 0, st>>>(G, ldg, X, ldx, P, ldp, Pb, slab, w.rps, w.Mp, K / 128, nt);
  } else if (N >= 128 && K % 64 == 0) {
    const int nt = (N / 128) * (K / 64);
    gemm_wgrad_kernel<128, 64, 2><<<nt * w.S, 256, 0, st>>>(G, ldg, X, ldx, P, ldp, Pb, slab, w.rps, w.Mp, K / 64, nt);
  } else if (N == 32 && K % 128 == 0) {
    const int nt = K / 128;
    gemm_wgrad_kernel<32, 128, 1, 64><<<nt * w.S, 256, 0, st>>>(G, ldg, X, ldx, P, ldp, Pb, slab, w.rps, w.Mp, K / 128, nt);
  } else {
    return NERF_E_ARG;
  }
  return NERF_OK;
}

// split-product (bf16 x 6) forms of the trunk GEMMs (gemm_x6.hpp)
template <int EPI>
int nt_x6(const float* A, int lda, const nerf_bf16* Bp, int ldb, int64_t bplane, const float* bias, float* C, int ldc,
          const uint32_t* mbits, uint32_t* mbits_out, int64_t M, int N, int K, hipStream_t st) {
  if (M % 128 || N % 128 || K % 32 || lda % 4 || ldb % 8) return NERF_E_ARG;
  const int ntn = N / 128;
#ifndef NERF_X6_SQUARE  // (64 NW) x 128 tiles of 64 x 128 waves (gemm_nt_x6w); NERF_X6_SQUARE: 128 x 128 (A/B builds)
#ifndef NERF_X6W_BK
#define NERF_X6W_BK 32
#endif
#ifndef NERF_X6W_NW
#define NERF_X6W_NW 8
#endif
  if constexpr (EPI == EPI_MASK) {
    // input gradients: split accumulators (gemm_x6.hpp BIGSMALL) on 32-row waves, two per SIMD (256 x 128 tiles of 8
    // waves): 0.73-0.75 -> 0.665 ms per fine layer against 64-row waves at one per SIMD, bitwise the same results
#ifndef NERF_X6_DG_NW  // A/B builds: waves per input-gradient workgroup (4: two workgroups per CU)
#define NERF_X6_DG_NW 8
#endif
    constexpr int DGM = 32 * NERF_X6_DG_NW;
#ifdef NERF_X6_DG_SHARED  // A/B builds: 128 x 256 tiles, each activation slab split once and shared (gemm_x6s.hpp)
    if (M % 128 == 0 && K == 256 && N == 256 && EPI == EPI_MASK) {
      gemm_nt_x6s_kernel<EPI, 8><<<(unsigned)(M / 128), 512, 0, st>>>(A, lda, Bp, ldb, bplane, C, ldc, mbits, N / 32);
      return NERF_OK;
    }
#endif
#ifdef NERF_X6_DG_TN8  // A/B builds: input gradient on 128 x 256 tiles of 32 x 256 waves, one wave per SIMD (both
    // accumulator sets, 256 registers, need the whole register file): each row split once instead of twice
    if (M % 128 == 0 && K == 256 && N % 256 == 0) {
      gemm_nt_x6w_kernel<EPI, 32, 4, true, 1, 1, 8, 8><<<(unsigned)((M / 128) * (N / 256)), 256, 0, st>>>(
          A, lda, Bp, ldb, bplane, bias, C, ldc, mbits, N / 32, mbits_out, K, N / 256);
      return NERF_OK;
    }
#endif
#ifndef NERF_X6W_NOA3  // three activation register sets, K = 256 unrolled (NERF_X6W_NOA3: the two-set loop, A/B builds)
    // (profiles/r04/x6_a3_ab.txt: 0.597 -> 0.584 ms per fine launch, C2 +0.5 %, bitwise the same)
    if (M % DGM == 0 && K == 256) {
      gemm_nt_x6w_kernel<EPI, 32, NERF_X6_DG_NW, true, 1, 8 / NERF_X6_DG_NW, 8><<<(unsigned)((M / DGM) * ntn),
                                                                                64 * NERF_X6_DG_NW, 0, st>>>(
          A, lda, Bp, ldb, bplane, bias, C, ldc, mbits, N / 32, mbits_out, K, ntn);
      return NERF_OK;
    }
#endif
    if (M % DGM == 0 && K % 64 == 0) {  // gemm_nt_x6w walks the slabs in pairs
      gemm_nt_x6w_kernel<EPI, 32, NERF_X6_DG_NW, true, 1, 8 / NERF_X6_DG_NW><<<(unsigned)((M / DGM) * ntn),
                                                                             64 * NERF_X6_DG_NW, 0, st>>>(
          A, lda, Bp, ldb, bplane, bias, C, ldc, mbits, N / 32, mbits_out, K, ntn);
      return NERF_OK;
    }
  }
#ifndef NERF_X6_K64_NW  // trunk.0 (K = 64: two slabs, the tile's 256 KiB of stores dominate): waves per workgroup
#define NERF_X6_K64_NW 8
#endif
  if constexpr (NERF_X6_K64_NW != NERF_X6W_NW) {
    if (K == 64 && EPI == EPI_BIAS_RELU && M % (64 * NERF_X6_K64_NW) == 0) {
      gemm_nt_x6w_kernel<EPI, NERF_X6W_BK, NERF_X6_K64_NW><<<(unsigned)((M / (64 * NERF_X6_K64_NW)) * ntn),
                                                             64 * NERF_X6_K64_NW, 0, st>>>(
          A, lda, Bp, ldb, bplane, bias, C, ldc, mbits, N / 32, mbits_out, K, ntn);
      return NERF_OK;
    }
  }
#ifndef NERF_X6_FWD_TN8  // forward on 256 x 256 tiles of 32 x 256 waves: each activation row is split by one workgroup
// instead of two (one per 128-column tile), at the same per-accumulator MFMA order — bitwise the same outputs.  C2 on
// one box (profiles/r05/x6_variants_ab.txt): fwd 0.572 -> 0.539 ms per fine layer, 228.6k -> 233.0k rays/s.
// NERF_X6_FWD_TN8=0 (A/B builds): the 512 x 128 tiles of 64 x 128 waves.
#define NERF_X6_FWD_TN8 1
#endif
#if NERF_X6_FWD_TN8
#ifdef NERF_X6_FWD_A3  // A/B builds: the K = 256 forward layers on three activation register sets (the A3 loop)
  if (EPI == EPI_BIAS_RELU && N % 256 == 0 && M % 256 == 0 && K == 256) {
    gemm_nt_x6w_kernel<EPI, 32, 8, false, 1, 1, 8, 8><<<(unsigned)((M / 256) * (N / 256)), 512, 0, st>>>(
        A, lda, Bp, ldb, bplane, bias, C, ldc, mbits, N / 32, mbits_out, K, N / 256);
    return NERF_OK;
  }
#endif
  if (EPI == EPI_BIAS_RELU && N % 256 == 0 && M % 256 == 0 && K % 64 == 0) {
    gemm_nt_x6w_kernel<EPI, 32, 8, false, 1, 1, 0, 8><<<(unsigned)((M / 256) * (N / 256)), 512, 0, st>>>(
        A, lda, Bp, ldb, bplane, bias, C, ldc, mbits, N / 32, mbits_out, K, N / 256);
    return NERF_OK;
  }
#endif
#ifdef NERF_X6_FWD_W12  // A/B builds: forward on 32-row waves, NERF_X6_FWD_W12 (12 or 16) per workgroup (3 / 4 per SIMD)
  if (EPI == EPI_BIAS_RELU && M % (32 * NERF_X6_FWD_W12) == 0 && K % 64 == 0) {
    gemm_nt_x6w_kernel<EPI, 32, NERF_X6_FWD_W12, false, 1, 1><<<(unsigned)((M / (32 * NERF_X6_FWD_W12)) * ntn),
                                                                64 * NERF_X6_FWD_W12, 0, st>>>(
        A, lda, Bp, ldb, bplane, bias, C, ldc, mbits, N / 32, mbits_out, K, ntn);
    return NERF_OK;
  }
#endif
  if (M % (64 * NERF_X6W_NW) == 0 && K % (2 * NERF_X6W_BK) == 0) {
    gemm_nt_x6w_kernel<EPI, NERF_X6W_BK, NERF_X6W_NW><<<(unsigned)((M / (64 * NERF_X6W_NW)) * ntn), 64 * NERF_X6W_NW, 0,
                                                        st>>>(A, lda, Bp, ldb, bplane, bias, C, ldc, mbits, N / 32,
                                                              mbits_out, K, ntn);
    return NERF_OK;
  }
#endif
#ifndef NERF_X6_NT_BK  // ablation / tuning builds: slab depth and workgroups per CU of the split NT GEMM
#define NERF_X6_NT_BK 32
#define NERF_X6_NT_MINW 2
#endif
  gemm_nt_x6_kernel<EPI, NERF_X6_NT_BK, NERF_X6_NT_MINW><<<(unsigned)((M / 128) * ntn), 256, 0, st>>>(A, lda, Bp, ldb, bplane, bias, C, ldc, mbits,
                                                                      N / 32, mbits_out, K, ntn);
  return NERF_OK;
}

// trunk weight gradient, N = 256: 128 x 128 tiles over the first 256 input columns, 128 x 64 tiles over K = 64
// (trunk.0) and the K = 320 remainder of trunk.4 (its encoding columns)
int wgrad_x6(const float* G, int ldg, const float* X, int ldx, int tensor_w, const WS& w, int N, int K, hipStream_t st) {
  const Layout& L = layout();
  float* P = w.partial + L.off[tensor_w];
  float* Pb = w.partial + L.off[tensor_w + 1];
  const int ldp = L.cols[tensor_w];
  const int64_t slab = L.total;
  if (N != 256 || ldg % 4 || ldx % 4) return NERF_E_ARG;
  auto t128 = [&](const float* Xk, float* Pk, float* Pbk) {
#ifndef NERF_X6_WGRAD_TILES  // one 512-thread workgroup per split (gemm_wgrad_x6w); the A/B form: 4 x 128x128 tiles
    gemm_wgrad_x6w_kernel<<<w.S, 512, 0, st>>>(G, ldg, Xk, ldx, Pk, ldp, Pbk, slab, w.rps, w.Mp);
#else
    gemm_wgrad_x6_kernel<128, 128, 2><<<4 * w.S, 256, 0, st>>>(G, ldg, Xk, ldx, Pk, ldp, Pbk, slab, w.rps, w.Mp, 2, 4);
#endif
  };
  auto t64 = [&](const float* Xk, float* Pk, float* Pbk) {
    // (a one-workgroup-per-split form reading G and X once, as gemm_wgrad_x6w, measured 185 -> 191 us per launch:
    // profiles/r04/x6_narrow_wgrad_ab.txt)
    gemm_wgrad_x6_kernel<128, 64, 4><<<2 * w.S, 256, 0, st>>>(G, ldg, Xk, ldx, Pk, ldp, Pbk, slab, w.rps, w.Mp, 1, 2);
  };
  if (K == 64) {
    t64(X, P, Pb);
  } else if (K == 256) {
    t128(X, P, Pb);
  } else if (K == 320) {
    t128(X, P, Pb);
    t64(X + 256, P + 256, nullptr);
  } else {
    return NERF_E_ARG;
  }
  return NERF_OK;
}

}  // namespace

extern "C" int64_t nerf_mlp_layout(int64_t* table) {
  const Layout& L = layout();
  if (table) {
    for (int t = 0; t < NT; ++t) {
      table[4 * t + 0] = L.off[t];
      table[4 * t + 1] = L.rows[t];
      table[4 * t + 2] = L.cols[t];
      table[4 * t + 3] = L.creal[t];
    }
  }
  return L.total;
}

extern "C" int64_t nerf_mlp_workspace_bytes(int64_t M, int training) {
  if (M < 0) return -1;
  return carve(nullptr, M, training).bytes + 256;
}

extern "C" int nerf_mlp_fwd_ex(const float* w, const float* x_d, int64_t M, float* rgb_sigma, void* ws,
                               int64_t ws_bytes, int training, int flags, hipEvent_t* ev, hipStream_t st) {
  NERF_CHECK_ARG(w && ws && M >= 0 && (M == 0 || (x_d && rgb_sigma)));  // an empty batch may pass null rows
  if (flags & ~NERF_MLP_NATIVE_FP32) return NERF_E_ENUM;
  const bool native = flags & NERF_MLP_NATIVE_FP32;
  if (!nerf_aligned16(w) || !nerf_aligned16(ws) || !nerf_aligned16(rgb_sigma)) return NERF_E_ALIGN;
  const WS W = carve(ws, M, training);
  if (ws_bytes < W.bytes) return NERF_E_WORKSPACE;
  if (M == 0) return NERF_OK;
  const Layout& L = layout();
  const int64_t Mp = W.Mp;
  auto Wt = [&](int t) { return w + L.off[t]; };

  pe_xyz_kernel<<<(unsigned)nerf_cdiv(Mp, 256), 256, 0, st>>>(x_d, M, Mp, W.X3E);  // 4 waves x 64 rows
  if (!native) {  // this call's weights as bf16 piece planes
    X6Jobs jobs{};
    for (int i = 0; i < 8; ++i)
      jobs.j[i] = X6Job{Wt(2 * i), W.WPf + x6_fwd_off(i), 256, KPAD[i], KPAD[i], 0, 256 * (int64_t)KPAD[i]};
    x6_planes_kernel<<<dim3(10, 8, 8), 256, 0, st>>>(jobs);
  }
  // trunk
  const float* in = W.X3E + 256;
  int ld_in = 320;
  for (int i = 0; i < 8; ++i) {
    float* out = W.Y[i];
    const int ld_out = training ? ld_of(W, i) : ((i % 2 == 0) ? 256 : 320);
    if (i == 4) { in = W.X3E; ld_in = 320; }  // cat([h3, enc]) lives in X3E
    if (ev) (void)hipEventRecord(ev[2 * i], st);
    if (native)
      TRY(nt<EPI_BIAS_RELU>(in, ld_in, Wt(2 * i), KPAD[i], Wt(2 * i + 1), out, ld_out, nullptr,
                            training ? W.MB[i] : nullptr, Mp, 256, KPAD[i], st));
    else
      TRY(nt_x6<EPI_BIAS_RELU>(in, ld_in, W.WPf + x6_fwd_off(i), KPAD[i], 256 * (int64_t)KPAD[i], Wt(2 * i + 1), out,
                               ld_out, nullptr, training ? W.MB[i] : nullptr, Mp, 256, KPAD[i], st));
    if (ev) (void)hipEventRecord(ev[2 * i + 1], st);
    in = out;
    ld_in = ld_out;
  }
  // heads + colour MLP + output activations in ONE launch (mlp_fwd_tail.hpp)
  {
    FwdTailArgs T{};
    T.Y7 = in; T.ldy = ld_in; T.xd = x_d; T.w = w;
    T.off_wh = L.off[16]; T.off_bh = L.off[17]; T.off_wc0 = L.off[18]; T.off_bc0 = L.off[19];
    T.off_wc1 = L.off[20]; T.off_bc1 = L.off[21];
    T.HO = W.HO; T.CIN = W.CIN; T.C0 = W.C0; T.out = rgb_sigma;
    T.M = M; T.Mp = Mp; T.ntiles = (int)(Mp / FT_ROWS);
    const int n_cu = nerf_cu_count();
    const int grid = T.ntiles < 2 * n_cu ? T.ntiles : 2 * n_cu;
    if (training)
      fwd_tail_kernel<true><<<grid, 256, 0, st>>>(T);
    else
      fwd_tail_kernel<false><<<grid, 256, 0, st>>>(T);
  }
  return nerf_launch_status();
}

#ifdef NERF_X6W_STAMPS  // diagnostic builds only: the split NT kernels' pipeline stamps (tools/x6_stamps.py)
extern "C" int nerf_debug_x6_stamps(unsigned long long* out, int clear) {
  if (clear) {
    static unsigned long long zero[2 * 8 * 128] = {};
    return nerf_hip_status(hipMemcpyToSymbol(HIP_SYMBOL(nerf_x6_stamps), zero, sizeof(zero)));
  }
  return nerf_hip_status(hipMemcpyFromSymbol(out, HIP_SYMBOL(nerf_x6_stamps), sizeof(nerf_x6_stamps)));
}
#endif

extern "C" int nerf_mlp_fwd(const float* w, const float* x_d, int64_t M, float* rgb_sigma, void* ws, int64_t ws_bytes,
                            int training, hipEvent_t* ev, hipStream_t st) {
  return nerf_mlp_fwd_ex(w, x_d, M, rgb_sigma, ws, ws_bytes, training, 0, ev, st);
}

extern "C" int64_t nerf_mlp_workspace_bytes_2s(int64_t M) {
  if (M < 0) return -1;
  return carve(nullptr, M, 2).bytes + 256;
}

namespace {
// The backward of nerf_mlp_fwd.  stw == nullptr: every launch on st (nerf_mlp_bwd).  Otherwise the weight-gradient
// GEMMs go to stw, each behind an event recorded on st after the launch that produced its input (sync[1]: colour
// branch + head dgrad -> head and trunk.7 wgrads; sync[8 - i], i < 7: trunk.(i+1) dgrad -> trunk.i wgrad), and st
// waits for stw (sync[9]) before the split reduce; sync[0] is unused.  The same kernels, grids and slabs: bitwise the
// one-stream result.
int mlp_bwd_impl(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                 int64_t ws_bytes, int flags, hipEvent_t* ev, hipStream_t st, hipStream_t stw, hipEvent_t* sync) {
  NERF_CHECK_ARG(w && d_w && ws && M >= 0 && (M == 0 || d_rgb_sigma));
  NERF_CHECK_ARG(!stw || sync);
  if (flags & ~(NERF_MLP_NATIVE_FP32 | NERF_MLP_NATIVE_DGRAD)) return NERF_E_ENUM;
  const bool native = flags & NERF_MLP_NATIVE_FP32;
  // input gradients: split products with the small terms in their own accumulators (gemm_nt_x6w BIGSMALL) unless
  // NERF_MLP_NATIVE_DGRAD keeps them on the fp32 MFMA
  const bool split_dgrad = !native && !(flags & NERF_MLP_NATIVE_DGRAD);
  if (!nerf_aligned16(w) || !nerf_aligned16(ws) || !nerf_aligned16(d_w) || !nerf_aligned16(d_rgb_sigma))
    return NERF_E_ALIGN;
  const bool two = stw != nullptr;
  const WS W = carve(ws, M, two ? 2 : 1);
  if (ws_bytes < W.bytes) return NERF_E_WORKSPACE;
  hipStream_t sw = two ? stw : st;  // the weight-gradient stream
  auto handoff = [&](int k) -> int {  // sw waits for everything issued on st so far
    if (!two) return NERF_OK;
    hipError_t e = hipEventRecord(sync[k], st);
    if (e == hipSuccess) e = hipStreamWaitEvent(stw, sync[k], 0);
    return nerf_hip_status(e);
  };
  const Layout& L = layout();
  if (M == 0) {
    if (!accumulate) (void)hipMemsetAsync(d_w, 0, L.total * sizeof(float), st);
    return nerf_launch_status();
  }
  const int64_t Mp = W.Mp;
  auto Wt = [&](int t) { return w + L.off[t]; };

  // transposed weights for the dgrad GEMMs: bf16 piece planes (split) or fp32 (NERF_MLP_NATIVE_DGRAD / native)
  float* T = W.WT;
  float* WTi[8] = {nullptr};
  TJobs jobs{};
  int nj = 0;
  if (!split_dgrad) {
    for (int i = 1; i < 8; ++i) {
      WTi[i] = T;
      jobs.j[nj++] = TJob{Wt(2 * i), T, 256, 256, KPAD[i]};  // first 256 input cols (h part for trunk.4)
      T += 65536;
    }
  } else {
    X6Jobs xj{};
    for (int i = 1; i < 8; ++i)
      xj.j[i - 1] = X6Job{Wt(2 * i), W.WPb + 3 * 65536 * (int64_t)(i - 1), 256, 256, KPAD[i], 1, 65536};
    x6_planes_kernel<<<dim3(8, 8, 7), 256, 0, st>>>(xj);
  }
  if (nj) transpose_kernel<<<dim3(8, 8, nj), 256, 0, st>>>(jobs);

  // colour branch + head activations in one kernel: dO16 and the colour weight / bias slabs (TAIL_NQ workgroups per
  // split; the colour sums of parts 1.. go to W.partial2 and are added by the final reduce)
  float* dcur = W.dA;
  float* dnext = W.dB;
  // events 2/3 (layer 0 has no input gradient) bracket the backward tail (colour branch + heads -> dZ7)
  if (ev) (void)hipEventRecord(ev[2], st);
  // colour branch -> dO16 [Mp][16]; then ONE pass over Y7 for dZ7 and the head weight / bias sums (mlp_tail.hpp)
  color_bwd_kernel<float, float><<<TAIL_NQ * W.S, 256, 0, st>>>(d_rgb_sigma, W.HO, W.C0, W.CIN, Wt(18), Wt(20), W.dO16,
                                                          W.partial, L.total, L.off[18], L.off[19], L.off[20], L.off[21],
                                                          W.rps, M, Mp, W.partial2, L.total - P2BASE, P2BASE, 16);
  head_bwd_kernel<<<TAIL_NQ * W.S, 256, 0, st>>>(W.dO16, W.Y[7], Wt(16), dcur, W.partial, L.total, W.partial2,
                                           L.total - P2BASE, P2BASE, L.off[16], L.off[17], W.rps, Mp);
  if (ev) (void)hipEventRecord(ev[3], st);
  TRY(handoff(1));  // dZ7 and the head / colour slabs are complete
  // trunk
  for (int i = 7; i >= 0; --i) {
    const float* X = (i == 0) ? W.X3E + 256 : (i == 4 ? W.X3E : W.Y[i - 1]);
    const int ldx = (i == 0 || i == 4) ? 320 : ld_of(W, i - 1);
    if (two && i < 7) TRY(handoff(8 - i));  // dZ_i, written by the trunk.(i+1) dgrad: sync[8 - i]
    if (ev) (void)hipEventRecord(ev[4 * i], sw);
    if (native)
      TRY(wgrad(dcur, 256, X, ldx, 2 * i, W, 256, KPAD[i], sw));
    else
      TRY(wgrad_x6(dcur, 256, X, ldx, 2 * i, W, 256, KPAD[i], sw));
    if (ev) (void)hipEventRecord(ev[4 * i + 1], sw);
    if (i > 0) {
      if (two) dnext = W.dZ[i - 1];  // never the buffer a trailing weight gradient still reads
      if (ev) (void)hipEventRecord(ev[4 * i + 2], st);
      if (!split_dgrad)
        TRY(nt<EPI_MASK>(dcur, 256, WTi[i], 256, nullptr, dnext, 256, W.MB[i - 1], nullptr, Mp, 256, 256, st));
      else
        TRY(nt_x6<EPI_MASK>(dcur, 256, W.WPb + 3 * 65536 * (int64_t)(i - 1), 256, 65536, nullptr, dnext, 256,
                            W.MB[i - 1], nullptr, Mp, 256, 256, st));
      if (ev) (void)hipEventRecord(ev[4 * i + 3], st);
      float* t = dcur; dcur = dnext; dnext = t;
    }
  }
  if (two) {  // join: the split reduce reads every weight-gradient slab
    TRY(nerf_hip_status(hipEventRecord(sync[9], stw)));
    TRY(nerf_hip_status(hipStreamWaitEvent(st, sync[9], 0)));
  }
  const int64_t n4 = L.total / 4;
  reduce_splits2_kernel<<<(unsigned)nerf_cdiv(n4, 64), 256, 0, st>>>(W.partial, L.total, W.S, d_w, n4, accumulate,
                                                                      W.partial2, L.total - P2BASE, P2BASE / 4);
  return nerf_launch_status();
}
}  // namespace

extern "C" int nerf_mlp_bwd_ex(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate,
                               void* ws, int64_t ws_bytes, int flags, hipEvent_t* ev, hipStream_t st) {
  return mlp_bwd_impl(w, M, d_rgb_sigma, d_w, accumulate, ws, ws_bytes, flags, ev, st, nullptr, nullptr);
}

extern "C" int nerf_mlp_bwd(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                            int64_t ws_bytes, hipEvent_t* ev, hipStream_t st) {
  return mlp_bwd_impl(w, M, d_rgb_sigma, d_w, accumulate, ws, ws_bytes, 0, ev, st, nullptr, nullptr);
}

extern "C" int nerf_mlp_bwd_2s_ex(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate,
                                  void* ws, int64_t ws_bytes, int flags, hipEvent_t* ev, hipStream_t st,
                                  hipStream_t wgrad_stream, hipEvent_t* sync) {
  NERF_CHECK_ARG(wgrad_stream && sync && wgrad_stream != st);
  return mlp_bwd_impl(w, M, d_rgb_sigma, d_w, accumulate, ws, ws_bytes, flags, ev, st, wgrad_stream, sync);
}

extern "C" int nerf_mlp_bwd_2s(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                               int64_t ws_bytes, hipEvent_t* ev, hipStream_t st, hipStream_t wgrad_stream,
                               hipEvent_t* sync) {
  return nerf_mlp_bwd_2s_ex(w, M, d_rgb_sigma, d_w, accumulate, ws, ws_bytes, 0, ev, st, wgrad_stream, sync);
}
