// Micro-benchmark of the MLP GEMM kernels at the C2 fine-net shape (M = 4096*192 = 786,432 rows,
// 256x256 layers), interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_bench.hip -o tools/gemm_bench
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
#include "../nerf-sys_amd/csrc/gemm.hpp"

template <int BM, int BN, int WAVES_M, int EPI, int MINW, int BK, int NBUF, int ABL>
__global__ __launch_bounds__(256, MINW) void gemm_abl(const float* __restrict__ A, int lda,
                                                      const float* __restrict__ B, int ldb,
                                                      const float* __restrict__ bias, float* __restrict__ C, int ldc,
                                                      const uint32_t* __restrict__ mbits, int ldmb,
                                                      uint32_t* __restrict__ mbits_out, int K, int n_ntiles) {
  constexpr int WAVES_N = 4 / WAVES_M;
  constexpr int WTM = BM / WAVES_M, WTN = BN / WAVES_N;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wave tile");
  static_assert(BK == 16 || BK == 32, "k-slab");
  constexpr int LS = BK + 4;         // LDS row pitch (floats): 80 / 144 B, 16 rows -> 16 distinct bank slots
  constexpr int C4 = BK / 4;         // float4 per row per slab
  constexpr int HK = BK / 2;         // k per lane half per slab
  constexpr int A_F4 = BM * C4, B_F4 = BN * C4;
  constexpr int A_PER = (A_F4 + 255) / 256, B_PER = (B_F4 + 255) / 256;
  __shared__ __attribute__((aligned(16))) float smem[NBUF * (BM + BN) * LS];

  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int mt = tile / n_ntiles, nt = tile - mt * n_ntiles;
  const int64_t m0 = (int64_t)mt * BM;
  const int n0 = nt * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int li = lane & 31, lh = lane >> 5;

  const float* Ab = A + m0 * lda;
  const float* Bb = B + (int64_t)n0 * ldb;

  float4 ra[A_PER], rb[B_PER];
#define AB_GLOAD(k0_)                                                                          \
  _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    if (A_F4 % 256 == 0 || f < A_F4)                                                           \
      ra[i] = *reinterpret_cast<const float4*>(Ab + (int64_t)(f / C4) * lda + (k0_) + (f % C4) * 4); \
  }                                                                                            \
  _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                         \
    const int f = tid + 256 * i;                                                               \
    if (B_F4 % 256 == 0 || f < B_F4)                                                           \
      rb[i] = *reinterpret_cast<const float4*>(Bb + (int64_t)(f / C4) * ldb + (k0_) + (f % C4) * 4); \
  }
#define AB_SSTORE(buf_)                                                                        \
  {                                                                                            \
    float* As_ = smem + (buf_) * (BM + BN) * LS;                                               \
    float* Bs_ = As_ + BM * LS;                                                                \
    _Pragma("unroll") for (int i = 0; i < A_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (A_F4 % 256 == 0 || f < A_F4)                                                         \
        *reinterpret_cast<float4*>(As_ + (f / C4) * LS + (f % C4) * 4) = ra[i];                \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < B_PER; ++i) {                                       \
      const int f = tid + 256 * i;                                                             \
      if (B_F4 % 256 == 0 || f < B_F4)                                                         \
        *reinterpret_cast<float4*>(Bs_ + (f / C4) * LS + (f % C4) * 4) = rb[i];                \
    }                                                                                          \
  }

  nerf_f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int nk = K / BK;
  AB_GLOAD(0);
  AB_SSTORE(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = NBUF == 2 ? (kt & 1) : 0;
    if (!(ABL & 1)) { AB_GLOAD((kt + 1 < nk ? kt + 1 : kt) * BK); }
    const float* As = smem + cur * (BM + BN) * LS;
    const float* Bs = As + BM * LS;
    // lane half h owns k = h*HK + s of the slab; its k-values of a row are read 4 at a time
#pragma unroll
    for (int hh = 0; hh < HK / 4; ++hh) {
      float4 af[TM], bf[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a)
        af[a] = *reinterpret_cast<const float4*>(As + (wm * WTM + a * 32 + li) * LS + HK * lh + 4 * hh);
#pragma unroll
      for (int b = 0; b < TN; ++b)
        bf[b] = *reinterpret_cast<const float4*>(Bs + (wn * WTN + b * 32 + li) * LS + HK * lh + 4 * hh);
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)  // swapped operands: the tile is C^T (i = n, j = m)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(bf[b][s], af[a][s], acc[a][b], 0, 0, 0);
    }
    if (!(ABL & 2)) {
      if (NBUF == 1) __syncthreads();
      AB_SSTORE(NBUF == 2 ? (cur ^ 1) : 0);
      __syncthreads();
    }
  }
#undef AB_GLOAD
#undef AB_SSTORE

  // epilogue.  The MFMA computed C^T, so lane li holds ONE output row m = ... + li and register
  // r = 4q + e holds column 8q + 4 lh + e of the 32-column tile: four float4 runs per row -> 16-B stores.
  // ReLU masks travel as bits: the forward writes word g = column/32 of row m (the lane's 16 bits OR'd
  // with its partner lane's li+32), the input-gradient GEMM reads one word per row instead of 32 floats.
#pragma unroll
  for (int b = 0; b < TN; ++b) {
    const int nb = n0 + wn * WTN + b * 32;
    const int g = nb >> 5;
    float4 bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      bv[q] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) bv[q] = *reinterpret_cast<const float4*>(bias + nb + 8 * q + 4 * lh);
    }
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      const int64_t m = m0 + wm * WTM + a * 32 + li;
      uint32_t word = 0;
      if (EPI == EPI_MASK) word = mbits[m * ldmb + g];
      float* crow = C + m * ldc + nb + 4 * lh;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          v[e] = acc[a][b][4 * q + e];
          const float bb = e == 0 ? bv[q].x : (e == 1 ? bv[q].y : (e == 2 ? bv[q].z : bv[q].w));
          if (EPI == EPI_BIAS) v[e] += bb;
          if (EPI == EPI_BIAS_RELU) {
            v[e] = fmaxf(v[e] + bb, 0.f);
            word |= (v[e] > 0.f ? 1u : 0u) << (8 * q + 4 * lh + e);
          }
          if (EPI == EPI_MASK) v[e] = ((word >> (8 * q + 4 * lh + e)) & 1u) ? v[e] : 0.f;
        }
        if (!(ABL & 4)) *reinterpret_cast<float4*>(crow + 8 * q) = make_float4(v[0], v[1], v[2], v[3]);
        else asm volatile("" :: "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]));
      }
      if (EPI == EPI_BIAS_RELU && mbits_out) {
        word |= __shfl_xor(word, 32, 64);
        if (lh == 0) mbits_out[m * ldmb + g] = word;
      }
    }
  }
}


#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
  const int64_t M = 4096LL * 192;
  const int N = 256, K = 256;
  const int rounds = argc > 1 ? atoi(argv[1]) : 5;
  std::vector<float> h((size_t)M * K);
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (auto& x : h) x = U(rng);
  float *A, *B, *C, *bias, *P;
  uint32_t *mb;
  CK(hipMalloc(&A, M * K * 4)); CK(hipMalloc(&B, N * K * 4)); CK(hipMalloc(&C, M * N * 4));
  CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&mb, M * 8 * 4));
  const int S = 256; const int64_t slab = 256 * 256 + 256;
  CK(hipMalloc(&P, (int64_t)S * slab * 4));
  CK(hipMemcpy(A, h.data(), M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data(), N * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemset(mb, 0xff, M * 8 * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double flop = 2.0 * M * N * K;
  struct V { const char* name; std::vector<float> ms; };
  std::vector<V> vs = {{"fwd relu+bits (lib)", {}}, {"dgrad bits (lib)", {}}, {"wgrad (lib)", {}},
                       {"fwd abl: no gload", {}}, {"fwd abl: no lds-store+bar", {}}, {"fwd abl: no C store", {}},
                       {"fwd abl: mfma+lds-read only", {}}};
  auto run = [&](int v) {
    const int ntn = N / 128; const unsigned nb = (unsigned)((M / 128) * ntn);
    switch (v) {
      case 0: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 1: gemm_nt_kernel<128, 128, 2, EPI_MASK, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 2: { const int nt = 4; const int64_t rps = M / S;
        gemm_wgrad_kernel<128, 128, 2><<<nt * S, 256>>>(A, K, C, N, P, 256, P + 65536, slab, rps, M, 2, nt); break; }
      case 3: gemm_abl<128, 128, 2, EPI_BIAS_RELU, 4, 16, 2, 1><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 4: gemm_abl<128, 128, 2, EPI_BIAS_RELU, 4, 16, 2, 2><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 5: gemm_abl<128, 128, 2, EPI_BIAS_RELU, 4, 16, 2, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 6: gemm_abl<128, 128, 2, EPI_BIAS_RELU, 4, 16, 2, 7><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
    }
  };
  for (int v = 0; v < (int)vs.size(); ++v) run(v);
  CK(hipDeviceSynchronize());
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < (int)vs.size(); ++v) {
      CK(hipEventRecord(e0)); run(v); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); vs[v].ms.push_back(ms);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%-28s median %.4f ms  min %.4f  -> %.1f TFLOP/s (%.1f%% of 157.3)\n", v.name, med, v.ms[0],
           flop / med * 1e-9, flop / med * 1e-9 / 157.3 * 100);
  }
  return 0;
}
