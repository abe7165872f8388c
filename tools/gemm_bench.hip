// Micro-benchmark of the MLP GEMM kernels at the C2 fine-net shape (M = 4096*192 = 786,432 rows,
// 256x256 layers), interleaved rounds in one process (cdna_hip_programming.md §5.4 rule 24).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_bench.hip -o tools/gemm_bench
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
#include "../nerf-sys_amd/csrc/gemm.hpp"

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
  std::vector<V> vs = {{"nt fwd relu+bits 128x128", {}}, {"nt fwd relu 128x128", {}}, {"nt none 128x128", {}},
                       {"nt dgrad bits 128x128", {}}, {"wgrad 128x128", {}},
                       {"nt fwd relu+bits lb4", {}}, {"nt dgrad bits lb4", {}},
                       {"fwd lb4 BK32 1buf", {}}, {"fwd lb2 BK32 2buf", {}}, {"dgrad lb4 BK32 1buf", {}},
                       {"fwd lb4 BK16 1buf", {}}, {"none lb4 BK32 1buf", {}}};
  auto run = [&](int v) {
    const int ntn = N / 128; const unsigned nb = (unsigned)((M / 128) * ntn);
    switch (v) {
      case 0: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 1: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, nullptr, K, ntn); break;
      case 2: gemm_nt_kernel<128, 128, 2, EPI_NONE><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, nullptr, K, ntn); break;
      case 3: gemm_nt_kernel<128, 128, 2, EPI_MASK><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 4: { const int nt = 4; const int64_t rps = M / S;
        gemm_wgrad_kernel<128, 128, 2><<<nt * S, 256>>>(A, K, C, N, P, 256, P + 65536, slab, rps, M, 2, nt); break; }
      case 5: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 6: gemm_nt_kernel<128, 128, 2, EPI_MASK, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 7: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 4, 32, 1><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 8: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 2, 32, 2><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 9: gemm_nt_kernel<128, 128, 2, EPI_MASK, 4, 32, 1><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 10: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 4, 16, 1><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn); break;
      case 11: gemm_nt_kernel<128, 128, 2, EPI_NONE, 4, 32, 1><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, nullptr, K, ntn); break;
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
