// Micro-benchmark: the library's register-staged fp32 MFMA GEMMs (gemm.hpp) vs the measured alternatives of
// tools/gemm_variants/ (LDS-DMA ring, weights-stationary, barrier-free wgrad) and tile/occupancy variants at the
// C2 fine-net trunk shape (M = 4096*192 rows, 256x256 layers), interleaved rounds in one process
// (cdna_hip_programming.md §5.4 rule 24); every variant's output is compared bitwise with the library's.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_bench2.hip -o tools/gemm_bench2
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>
#include <random>
#include <cmath>
#include "gemm_variants/gemm_glds.hpp"
#include "gemm_variants/gemm_ws.hpp"
#include "gemm_variants/gemm_wgrad_os.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
  const int64_t M = 4096LL * 192;
  const int N = 256, K = 256;
  const int rounds = argc > 1 ? atoi(argv[1]) : 7;
  std::vector<float> h((size_t)M * K);
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (auto& x : h) x = U(rng);
  float *A, *B, *C, *bias;
  uint32_t *mb, *mbo;
  CK(hipMalloc(&A, M * K * 4)); CK(hipMalloc(&B, N * K * 4)); CK(hipMalloc(&C, M * N * 4));
  CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&mb, M * 8 * 4)); CK(hipMalloc(&mbo, M * 8 * 4));
  CK(hipMemcpy(A, h.data(), M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data() + 12345, N * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h.data() + 777, N * 4, hipMemcpyHostToDevice));
  {
    std::vector<uint32_t> bits((size_t)M * 8);
    for (auto& b : bits) b = rng();
    CK(hipMemcpy(mb, bits.data(), M * 8 * 4, hipMemcpyHostToDevice));
  }
  const int64_t slab = 256 * 256 + 256;
  float* P;
  CK(hipMalloc(&P, 256 * slab * 4));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double flop = 2.0 * M * N * K;
  const int ntn = N / 128;
  const unsigned nb = (unsigned)((M / 128) * ntn);
  struct V { const char* name; int cls; std::vector<float> ms; };
  std::vector<V> vs = {
      {"fwd  lib regstage", 0, {}},
      {"fwd  MINW=2", 0, {}},
      {"fwd  BK=32 MINW=2", 0, {}},
      {"fwd  BN=256 MINW=2", 0, {}},
      {"fwd  glds ring S=4", 0, {}},
      {"fwd  weights-stat D=2", 0, {}},
      {"dgrd lib regstage", 1, {}},
      {"dgrd BN=256", 1, {}},
      {"wgrd lib lds", 2, {}},
      {"wgrd barrier-free R=8", 2, {}},
      {"wgrd 256x256 tile", 2, {}},
      {"wgrd 256x128 tile", 2, {}},
      {"wgrd 128x256 tile", 2, {}},
  };
  const unsigned nb256 = (unsigned)(M / 128);
  auto run = [&](int v) {
    switch (v) {
      case 0: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 1: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 2><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 2: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 2, 32><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 3: gemm_nt_kernel<128, 256, 2, EPI_BIAS_RELU, 2><<<nb256, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, 1); break;
      case 4: gemm_nt_glds_kernel<128, 128, 2, EPI_BIAS_RELU, 4, 2><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 5: gemm_ws_kernel<256, 128, 2, 2, 2, EPI_BIAS_RELU, 2><<<256, 512>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, (int)(M / 256), 128, 2); break;
      case 6: gemm_nt_kernel<128, 128, 2, EPI_MASK, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 7: gemm_nt_kernel<128, 256, 2, EPI_MASK, 2><<<nb256, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, 1); break;
      case 8: gemm_wgrad_kernel<128, 128, 2><<<4 * 256, 256>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 2, 4); break;
      case 9: gemm_wgrad_os_kernel<4, 2, 8, 8><<<256, 512>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 4); break;
      case 10: gemm_wgrad_kernel<256, 256, 2><<<256, 256>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 1, 1); break;
      case 11: gemm_wgrad_kernel<256, 128, 2><<<2 * 256, 256>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 2, 2); break;
      case 12: gemm_wgrad_kernel<128, 256, 2><<<2 * 256, 256>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 1, 2); break;
    }
  };
  // correctness: each variant vs the library variant of its class, bitwise (same k order, same fmaf chain)
  std::vector<float> ref((size_t)M * N), out((size_t)M * N);
  std::vector<uint32_t> refb((size_t)M * 8), outb((size_t)M * 8);
  int bad = 0;
  std::vector<float> pref((size_t)256 * slab), pout((size_t)256 * slab);
  for (int v = 0; v < (int)vs.size(); ++v) {
    if (vs[v].cls == 2) {
      // wgrad reads C as its X operand: fill C with the activations once
      if (v == 8) CK(hipMemcpy(C, h.data() + 4321, M * N * 4, hipMemcpyHostToDevice));
      CK(hipMemset(P, 0, 256 * slab * 4));
      run(v);
      CK(hipDeviceSynchronize());
      std::vector<float>& dst = (v == 8) ? pref : pout;
      CK(hipMemcpy(dst.data(), P, 256 * slab * 4, hipMemcpyDeviceToHost));
      if (v != 8) {
        // compare the reduced sums over splits (the split partition is the same; summation order differs)
        double maxrel = 0;
        for (int64_t i = 0; i < slab; ++i) {
          double a = 0, b = 0, sc = 0;
          for (int sp = 0; sp < 256; ++sp) { a += pref[sp * slab + i]; b += pout[sp * slab + i]; sc += fabs(pref[sp * slab + i]); }
          maxrel = std::max(maxrel, fabs(a - b) / (sc + 1e-30));
        }
        printf("check %-20s: max |diff| / sum|partials| = %.3e\n", vs[v].name, maxrel);
        bad += maxrel > 1e-5;
      }
      continue;
    }
    CK(hipMemset(C, 0, M * N * 4)); CK(hipMemset(mbo, 0, M * 8 * 4));
    run(v);
    CK(hipDeviceSynchronize());
    const bool is_ref = (v == 0 || v == 6);
    std::vector<float>& dst = is_ref ? ref : out;
    std::vector<uint32_t>& dstb = is_ref ? refb : outb;
    CK(hipMemcpy(dst.data(), C, M * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(dstb.data(), mbo, M * 8 * 4, hipMemcpyDeviceToHost));
    if (!is_ref) {
      size_t nd = 0;
      for (size_t i = 0; i < ref.size(); ++i) nd += (memcmp(&ref[i], &out[i], 4) != 0);
      size_t ndb = 0;
      if (vs[v].cls == 0) for (size_t i = 0; i < refb.size(); ++i) ndb += (refb[i] != outb[i]);
      printf("check %-20s: %zu differing outputs, %zu differing mask words\n", vs[v].name, nd, ndb);
      bad += (nd != 0 || ndb != 0);
    }
  }
  CK(hipMemcpy(C, h.data() + 4321, M * N * 4, hipMemcpyHostToDevice));
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < (int)vs.size(); ++v) {
      CK(hipEventRecord(e0)); run(v); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); vs[v].ms.push_back(ms);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%-22s median %.4f ms  min %.4f  -> %.1f TFLOP/s (%.1f%% of 157.3)\n", v.name, med, v.ms[0],
           flop / med * 1e-9, flop / med * 1e-9 / 157.3 * 100);
  }
  return bad;
}
