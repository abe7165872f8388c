// Micro-benchmark: the library's fp32 gemm_nt (32x32x2 MFMA) vs the 16x16x4 variant (gemm_variants/gemm_nt16.hpp)
// at the C2 fine-net trunk shape (M = 4096*192, 256x256), forward (bias + ReLU + mask words) and dgrad (mask),
// interleaved rounds in one process, random data.  The k order inside a slab differs (k = 4g + s), so outputs are
// compared by max |diff| / sum |a||b| and mask words by count.
// Measured (MI355X, 7 interleaved rounds, median ms; 103.1 GFLOP per launch):
//   fwd lib 0.863-0.916 (0.72-0.76 of peak), dgrad lib 0.858-0.875; 16x16x4 fwd 1.204-1.211, dgrad 1.190-1.200 (0.54)
//   diagnostics (gemm_diag.hpp, lambda-based loop; its D = 0 copy of the library loop already runs 1.21-1.23):
//     no global loads / LDS stores in the loop 0.806-0.815; MFMA only 0.819-0.826; MFMA only at K = 2048 (1/8 of the
//     tiles, same FLOP) 0.712-0.720 (0.91 of peak): ~13 % of the K = 256 launch is the per-tile prologue / epilogue.
//   16x16x4 in the macro-staged loop (gemm.hpp gemm_nt16_kernel, now the library's trunk fwd / dgrad): fwd 0.839-0.852
//   at MINW 3 vs 0.897-0.901; dgrad 0.817-0.827 vs 0.874-0.894; BK = 32 0.94-0.96; the weight gradient on 16x16x4
//   (gemm_variants/gemm_wgrad16.hpp) 0.887-0.962 vs 0.857-0.874, with the slab transposed in LDS (gemm_wgrad_t.hpp)
//   0.867-0.873.  (The 1.2 ms of the first 16x16x4 build and of the D = 0 diagnostic came from lambda-based
//   staging loads, which the compiler sank behind the MFMA block.)
//   Keeping the staging loads in front of the MFMA block (the compiler sinks them behind it): sched_barrier after the
//   loads — the IR has already sunk them, so it only fences the scheduler — wgrad 0.923 vs 0.862, nt16 fwd 0.853 vs
//   0.838; loads for slab k + 2 issued before the barrier that ends slab k (software pipelined): wgrad 0.923, nt16 fwd
//   1.036 / dgrad 1.017 (slower: the wait for the older loads then counts the newer ones in flight).
//   A persistent 16x16x4 kernel whose last k-slab loads slab 0 of the workgroup's next tile (gemm_nt16p.hpp): dgrad
//   1.786 ms at 1024 workgroups / 1.491 at 768 vs 0.826 with an if/else between the two loads, 0.907 / 0.890 vs 0.825
//   with branch-free pointer selects: the prologue of a new tile is not what the ~13 % per-tile cost is made of.
//   Chunk-major LDS slabs ([4-float chunk][row], conflict-free for every ds_read_b128 phase; PMC: the 16x16x4 kernel
//   shows 5.2e7 LDS bank-conflict cycles per launch vs 2.7e7 for the 32x32x2 one): fwd 0.866 vs 0.837, dgrad 0.833 vs
//   0.831 — the conflicts do not bound it (PMC: MFMA busy 0.80 for fwd / dgrad at 2.3-2.4 GHz, wgrad 0.77).
//   Tried on the library kernel and not kept: staggering the first generation of workgroups by s_sleep (slot or
//   hashed, 0.886-0.946: slower), an epilogue staged through LDS so that every store writes whole 128-B lines
//   (fwd 0.875 vs 0.863, dgrad 0.851 vs 0.858: within noise).
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_bench16.hip -o tools/gemm_bench16
#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>
#include <random>
#include <cmath>
#include "gemm_variants/gemm_nt16.hpp"
#include "gemm_variants/gemm_wgrad_t.hpp"
#include "gemm_variants/gemm_wgrad8.hpp"
#include "gemm_variants/gemm_diag.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
  const int64_t M = 4096LL * 192;
  const int N = 256, K = 256;
  const int rounds = argc > 1 ? atoi(argv[1]) : 9;
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
  struct V { const char* name; int ref; std::vector<float> ms; };
  std::vector<V> vs = {
      {"fwd  lib 32x32x2", -1, {}},
      {"fwd  16x16x4 MINW=2", 0, {}},
      {"fwd  16x16x4 MINW=3", 0, {}},
      {"fwd  16x16x4 BK=32 MINW=2", 0, {}},
      {"fwd  16x16x4 MINW=4", 0, {}},
      {"dgrd lib 32x32x2", -1, {}},
      {"dgrd 16x16x4 MINW=2", 5, {}},
      {"dgrd 16x16x4 MINW=3", 5, {}},
      {"dgrd 16x16x4 BK=32 MINW=2", 5, {}},
      {"wgrd lib 32x32x2", -3, {}},
      {"wgrd LDS-transposed", -5, {}},
      {"wgrd LDS-transposed MINW=2", -5, {}},
      {"wgrd 8 waves 128x256", -5, {}},
  };
  auto run = [&](int v) {
    switch (v) {
      case 0: gemm_nt_kernel<128, 128, 2, EPI_BIAS_RELU, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 1: gemm_nt16_kernel<128, 128, 2, EPI_BIAS_RELU, 2><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 2: gemm_nt16_kernel<128, 128, 2, EPI_BIAS_RELU, 3><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 3: gemm_nt16_kernel<128, 128, 2, EPI_BIAS_RELU, 2, 32><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 4: gemm_nt16_kernel<128, 128, 2, EPI_BIAS_RELU, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mbo, K, ntn); break;
      case 5: gemm_nt_kernel<128, 128, 2, EPI_MASK, 4><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 6: gemm_nt16_kernel<128, 128, 2, EPI_MASK, 2><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 7: gemm_nt16_kernel<128, 128, 2, EPI_MASK, 3><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 8: gemm_nt16_kernel<128, 128, 2, EPI_MASK, 2, 32><<<nb, 256>>>(A, K, B, K, bias, C, N, mb, 8, nullptr, K, ntn); break;
      case 9: gemm_wgrad_kernel<128, 128, 2><<<4 * 256, 256>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 2, 4); break;
      case 10: gemm_wgrad_t_kernel<128, 128, 2><<<4 * 256, 256>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 2, 4); break;
      case 12: gemm_wgrad8_kernel<128, 256, 2><<<2 * 256, 512>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 1, 2); break;
      case 11: gemm_wgrad_t_kernel<128, 128, 2, 2><<<4 * 256, 256>>>(A, K, C, N, P, 256, P + 65536, slab, M / 256, M, 2, 4); break;
    }
  };
  // bound on |sum_k a_k b_k| rounding: sum_k |a_k||b_k| <= K (|a|, |b| <= 1)
  std::vector<float> ref((size_t)M * N), out((size_t)M * N);
  std::vector<uint32_t> refb((size_t)M * 8), outb((size_t)M * 8);
  int bad = 0;
  std::vector<float> pref((size_t)256 * slab), pout((size_t)256 * slab);
  for (int v = 0; v < (int)vs.size(); ++v) {
    if (vs[v].ref == -2) continue;
    if (vs[v].ref <= -3) {  // wgrad: C holds the X operand
      CK(hipMemcpy(C, h.data() + 4321, M * N * 4, hipMemcpyHostToDevice));
      CK(hipMemset(P, 0, 256 * slab * 4));
      run(v);
      CK(hipDeviceSynchronize());
      std::vector<float>& dst = vs[v].ref == -3 ? pref : pout;
      CK(hipMemcpy(dst.data(), P, 256 * slab * 4, hipMemcpyDeviceToHost));
      if (vs[v].ref == -5) {
        size_t nd = 0;
        for (size_t i = 0; i < pref.size(); ++i) nd += memcmp(&pref[i], &pout[i], 4) != 0;
        printf("check %-22s: %zu of %zu partial-slab values differ from the library's (bitwise)\n", vs[v].name, nd, pref.size());
        bad += nd != 0;
      }
      if (vs[v].ref == -4) {
        double maxrel = 0;
        for (int64_t i = 0; i < slab; ++i) {
          double a = 0, b = 0, sc = 0;
          for (int sp = 0; sp < 256; ++sp) { a += pref[sp * slab + i]; b += pout[sp * slab + i]; sc += fabs(pref[sp * slab + i]); }
          maxrel = std::max(maxrel, fabs(a - b) / (sc + 1e-30));
        }
        printf("check %-22s: max |diff| / sum|partials| = %.3e\n", vs[v].name, maxrel);
        bad += maxrel > 1e-5;
      }
      continue;
    }
    CK(hipMemset(C, 0, M * N * 4)); CK(hipMemset(mbo, 0, M * 8 * 4));
    run(v);
    CK(hipDeviceSynchronize());
    if (vs[v].ref == -2) continue;  // diagnostics: timing only
    const bool is_ref = vs[v].ref < 0;
    std::vector<float>& dst = is_ref ? ref : out;
    std::vector<uint32_t>& dstb = is_ref ? refb : outb;
    CK(hipMemcpy(dst.data(), C, M * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(dstb.data(), mbo, M * 8 * 4, hipMemcpyDeviceToHost));
    if (!is_ref) {
      double md = 0; size_t nd = 0;
      for (size_t i = 0; i < ref.size(); ++i) { md = std::max(md, (double)fabsf(ref[i] - out[i])); nd += ref[i] != out[i]; }
      size_t ndb = 0;
      if (v < 5) for (size_t i = 0; i < refb.size(); ++i) ndb += __builtin_popcount(refb[i] ^ outb[i]);
      printf("check %-22s: max|diff| %.3e (bound ~K*eps = %.1e), %zu of %zu outputs differ, %zu mask bits differ\n",
             vs[v].name, md, 256 * 1.2e-7, nd, ref.size(), ndb);
      bad += md > 1e-4;
    }
  }
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < (int)vs.size(); ++v) {
      for (int w = 0; w < 3; ++w) run(v);  // back-to-back launches: the clock under sustained load
      CK(hipEventRecord(e0));
      for (int w = 0; w < 5; ++w) run(v);
      CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
      float ms; CK(hipEventElapsedTime(&ms, e0, e1)); vs[v].ms.push_back(ms / 5);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    printf("%-24s median %.4f ms  min %.4f  -> %.1f TFLOP/s (%.1f%% of 157.3)\n", v.name, med, v.ms[0],
           flop / med * 1e-9, flop / med * 1e-9 / 157.3 * 100);
  }
  return bad;
}
