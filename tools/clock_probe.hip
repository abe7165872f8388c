// Diagnostic build (never shipped): the in-kernel clock the chip holds under (1) a bare fp32-MFMA loop on
// random operands and (2) the library's trunk forward GEMM, from s_memtime / s_memrealtime stamps taken by
// wave 0 of every block at entry and exit (MI355X_MICROARCH.md 'DVFS give-back' item 6). Stamps go to a
// debug buffer only.  Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/clock_probe.hip -o tools/clock_probe
#include <cstdio>
#include <vector>
#include <algorithm>
#include <random>
#include "../nerf-sys_amd/csrc/gemm.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ __forceinline__ void stamp(unsigned long long* dbg, int slot) {
  if (threadIdx.x == 0) {
    const unsigned long long t = __builtin_amdgcn_s_memtime();
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    dbg[4 * blockIdx.x + 2 * slot] = t;
    dbg[4 * blockIdx.x + 2 * slot + 1] = r;
  }
}

__global__ __launch_bounds__(256, 4) void mfma_loop(const float* __restrict__ in, float* out, int iters,
                                                    unsigned long long* dbg) {
  stamp(dbg, 0);
  float a = in[threadIdx.x], b = in[threadIdx.x + 256];
  nerf_f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int i = 0; i < iters; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(b, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  stamp(dbg, 1);
}

template <int EPI>
__global__ __launch_bounds__(256, 4) void gemm_probe(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                     int ldb, const float* __restrict__ bias, float* __restrict__ C,
                                                     int ldc, const uint32_t* __restrict__ mbits, int ldmb,
                                                     uint32_t* __restrict__ mbits_out, int K, int n_ntiles,
                                                     unsigned long long* dbg) {
  stamp(dbg, 0);
  gemm_nt_body<128, 128, 2, EPI>(A, lda, B, ldb, bias, C, ldc, mbits, ldmb, mbits_out, K, n_ntiles);
  stamp(dbg, 1);
}

static void report(const char* name, std::vector<unsigned long long>& h, int nblk, double flop, float ms) {
  std::vector<double> ghz;
  for (int b = 0; b < nblk; ++b) {
    const double dt = (double)(h[4 * b + 2] - h[4 * b]);
    const double dr = (double)(h[4 * b + 3] - h[4 * b + 1]);
    if (dr > 0) ghz.push_back(dt / dr * 0.1);
  }
  std::sort(ghz.begin(), ghz.end());
  printf("%-34s %.4f ms  %.1f TFLOP/s  in-kernel clock median %.3f GHz (p10 %.3f, p90 %.3f)  -> %.1f%% of peak at that clock\n",
         name, ms, flop / ms * 1e-9, ghz[ghz.size() / 2], ghz[ghz.size() / 10], ghz[ghz.size() * 9 / 10],
         flop / ms * 1e-9 / (256 * 4 * 64 * ghz[ghz.size() / 2] * 1e-3) * 100);
}

int main() {
  const int64_t M = 4096LL * 192;
  const int N = 256, K = 256;
  std::vector<float> h((size_t)M * K);
  std::mt19937 rng(1);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  for (auto& x : h) x = U(rng);
  float *A, *B, *C, *bias;
  uint32_t* mb;
  unsigned long long* dbg;
  CK(hipMalloc(&A, M * K * 4)); CK(hipMalloc(&B, N * K * 4)); CK(hipMalloc(&C, M * N * 4));
  CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&mb, M * 8 * 4)); CK(hipMalloc(&dbg, 4 * 16384 * 8));
  CK(hipMemcpy(A, h.data(), M * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(B, h.data() + 999, N * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, h.data(), N * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<unsigned long long> hd(4 * 16384);
  const int ntn = 2; const int nb = (int)((M / 128) * ntn);
  const int iters = 4096, nbl = 1024;
  for (int rep = 0; rep < 3; ++rep) {
    // warm: ~2 s of back-to-back launches before each measurement
    for (int w = 0; w < 200; ++w) gemm_probe<EPI_BIAS_RELU><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn, dbg);
    CK(hipEventRecord(e0));
    gemm_probe<EPI_BIAS_RELU><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, ntn, dbg);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(hd.data(), dbg, 4 * nb * 8, hipMemcpyDeviceToHost));
    report("trunk fwd GEMM (lib body)", hd, nb, 2.0 * M * N * K, ms);
    for (int w = 0; w < 20; ++w) mfma_loop<<<nbl, 256>>>(A, C, iters, dbg);
    CK(hipEventRecord(e0));
    mfma_loop<<<nbl, 256>>>(A, C, iters, dbg);
    CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipMemcpy(hd.data(), dbg, 4 * nbl * 8, hipMemcpyDeviceToHost));
    report("bare fp32 MFMA loop (random regs)", hd, nbl, 2.0 * 32 * 32 * 2 * 4 * iters * 4.0 * nbl, ms);
  }
  return 0;
}
