// Correctness (vs a host fp64 reference on the same bf16-rounded operands) and speed of the bf16 MFMA
// GEMMs (nerf-sys_amd/csrc/gemm_bf16.hpp) at the C3 fine-net trunk shape.
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/gemm_bf16_test.hip -o tools/gemm_bf16_test
#include <cstdio>
#include <cstring>
#include <cmath>
#include <vector>
#include <algorithm>
#include <random>
#include "../nerf-sys_amd/csrc/gemm_bf16.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static uint16_t f2bf(float f) {  // round to nearest even (finite inputs)
  uint32_t u; memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) { uint32_t u = (uint32_t)h << 16; float f; memcpy(&f, &u, 4); return f; }

int main(int argc, char** argv) {
  int bad = 0;
  std::mt19937 rng(7);
  std::uniform_real_distribution<float> U(-1.f, 1.f);
  // ---------------- correctness, small shapes
  {
    const int M = 512, N = 256, K = 320;
    std::vector<uint16_t> a(M * K), b(N * K);
    for (auto& x : a) x = f2bf(U(rng));
    for (auto& x : b) x = f2bf(U(rng));
    std::vector<float> bias(N);
    for (auto& x : bias) x = U(rng);
    nerf_bf16 *dA, *dB; float* dbias; void* dC; uint32_t* dm;
    CK(hipMalloc(&dA, M * K * 2)); CK(hipMalloc(&dB, N * K * 2)); CK(hipMalloc(&dbias, N * 4));
    CK(hipMalloc(&dC, M * N * 4)); CK(hipMalloc(&dm, M * 8 * 4));
    CK(hipMemcpy(dA, a.data(), M * K * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, b.data(), N * K * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dbias, bias.data(), N * 4, hipMemcpyHostToDevice));
    const int ntn = N / 128;
    gemm_nt_bf16_kernel<128, 128, 2, EPI_BIAS_RELU, 0><<<(M / 128) * ntn, 256>>>(dA, K, dB, K, dbias, dC, N, nullptr, 8, dm, K, ntn);
    CK(hipDeviceSynchronize());
    std::vector<float> c(M * N);
    std::vector<uint32_t> mb(M * 8);
    CK(hipMemcpy(c.data(), dC, M * N * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(mb.data(), dm, M * 8 * 4, hipMemcpyDeviceToHost));
    double maxerr = 0; int maskbad = 0;
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < N; ++n) {
        double s = bias[n], sa = fabs(bias[n]);
        for (int k = 0; k < K; ++k) { s += (double)bf2f(a[m * K + k]) * bf2f(b[n * K + k]); sa += fabs((double)bf2f(a[m * K + k]) * bf2f(b[n * K + k])); }
        const double r = s > 0 ? s : 0;
        maxerr = std::max(maxerr, fabs(r - c[m * N + n]) / (sa + 1e-30));
        const int bit = (mb[m * 8 + n / 32] >> (n % 32)) & 1;
        maskbad += (bit != (c[m * N + n] > 0.f));
      }
    printf("nt_bf16 fwd fp32-out M=%d N=%d K=%d: max |err|/sum|a b| = %.3e, mask mismatches %d\n", M, N, K, maxerr, maskbad);
    bad += (maxerr > 1e-6) || maskbad;
    // bf16 output + mask epilogue
    gemm_nt_bf16_kernel<128, 128, 2, EPI_MASK, 1><<<(M / 128) * ntn, 256>>>(dA, K, dB, K, nullptr, dC, N, dm, 8, nullptr, K, ntn);
    CK(hipDeviceSynchronize());
    std::vector<uint16_t> cb(M * N);
    CK(hipMemcpy(cb.data(), dC, M * N * 2, hipMemcpyDeviceToHost));
    maxerr = 0;
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < N; ++n) {
        double s = 0, sa = 0;
        for (int k = 0; k < K; ++k) { s += (double)bf2f(a[m * K + k]) * bf2f(b[n * K + k]); sa += fabs((double)bf2f(a[m * K + k]) * bf2f(b[n * K + k])); }
        const int bit = (mb[m * 8 + n / 32] >> (n % 32)) & 1;
        const double r = bit ? s : 0.0;
        maxerr = std::max(maxerr, fabs(r - bf2f(cb[m * N + n])) / (sa + 1e-30));
      }
    printf("nt_bf16 dgrad bf16-out: max |err|/sum|a b| = %.3e (bf16 output rounding ~4e-3 of |value|)\n", maxerr);
    bad += maxerr > 8e-3;
    // N = 32 head tile (fp32 out, K = 256)
    gemm_nt_bf16_kernel<256, 32, 4, EPI_BIAS, 0><<<M / 256, 256>>>(dA, K, dB, K, dbias, dC, 32, nullptr, 1, nullptr, 256, 1);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(c.data(), dC, M * 32 * 4, hipMemcpyDeviceToHost));
    maxerr = 0;
    for (int m = 0; m < M; ++m)
      for (int n = 0; n < 32; ++n) {
        double s = bias[n], sa = fabs(bias[n]);
        for (int k = 0; k < 256; ++k) { s += (double)bf2f(a[m * K + k]) * bf2f(b[n * K + k]); sa += fabs((double)bf2f(a[m * K + k]) * bf2f(b[n * K + k])); }
        maxerr = std::max(maxerr, fabs(s - c[m * 32 + n]) / (sa + 1e-30));
      }
    printf("nt_bf16 head N=32: max |err|/sum|a b| = %.3e\n", maxerr);
    bad += maxerr > 1e-6;
    // wgrad: P[n][k] = sum_m G[m][n] X[m][k], G = A[:, :256] viewed with ld K, X = B-like [M][K]
    std::vector<uint16_t> x(M * K);
    for (auto& v : x) v = f2bf(U(rng));
    nerf_bf16* dX; float* dP;
    CK(hipMalloc(&dX, M * K * 2));
    CK(hipMemcpy(dX, x.data(), M * K * 2, hipMemcpyHostToDevice));
    const int S = 4; const int64_t rps = M / S; const int64_t slab = 256 * 320 + 256;
    CK(hipMalloc(&dP, S * slab * 4));
    // N = 256 (G cols 0..255 of A, ld K), K = 256 (X cols 0..255): 2 x 2 tiles of 128
    gemm_wgrad_bf16_kernel<128, 128, 2><<<4 * S, 256>>>(dA, K, dX, K, dP, 320, dP + 256 * 320, slab, rps, M, 2, 4);
    CK(hipDeviceSynchronize());
    std::vector<float> P(S * slab);
    CK(hipMemcpy(P.data(), dP, S * slab * 4, hipMemcpyDeviceToHost));
    maxerr = 0; double bmax = 0;
    for (int n = 0; n < 256; ++n) {
      for (int k = 0; k < 256; ++k) {
        double ref = 0, sa = 0, got = 0;
        for (int m = 0; m < M; ++m) { const double t = (double)bf2f(a[m * K + n]) * bf2f(x[m * K + k]); ref += t; sa += fabs(t); }
        for (int sp = 0; sp < S; ++sp) got += P[sp * slab + n * 320 + k];
        maxerr = std::max(maxerr, fabs(ref - got) / (sa + 1e-30));
      }
      double rb = 0, sb = 0, gb = 0;
      for (int m = 0; m < M; ++m) { rb += bf2f(a[m * K + n]); sb += fabs(bf2f(a[m * K + n])); }
      for (int sp = 0; sp < S; ++sp) gb += P[sp * slab + 256 * 320 + n];
      bmax = std::max(bmax, fabs(rb - gb) / (sb + 1e-30));
    }
    printf("wgrad_bf16 N=K=256: max |err|/sum|g x| = %.3e, bias %.3e\n", maxerr, bmax);
    bad += (maxerr > 1e-6) || (bmax > 1e-6);
  }
  // ---------------- speed at the C3 fine trunk shape
  {
    const int64_t M = 4096LL * 192;
    const int N = 256, K = 256;
    std::vector<uint16_t> h((size_t)M * K);
    for (auto& v : h) v = f2bf(U(rng));
    nerf_bf16 *A, *B, *C; float *bias, *P; uint32_t* mb;
    CK(hipMalloc(&A, M * K * 2)); CK(hipMalloc(&B, N * K * 2)); CK(hipMalloc(&C, M * N * 2));
    CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&mb, M * 8 * 4));
    const int S = 256; const int64_t slab = 256 * 256 + 256;
    CK(hipMalloc(&P, S * slab * 4));
    CK(hipMemcpy(A, h.data(), M * K * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(C, h.data(), M * N * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data() + 999, N * K * 2, hipMemcpyHostToDevice));
    CK(hipMemset(bias, 0, N * 4)); CK(hipMemset(mb, 0xff, M * 32));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const unsigned nb = (unsigned)((M / 128) * 2);
    auto run = [&](int v) {
      switch (v) {
        case 0: gemm_nt_bf16_kernel<128, 128, 2, EPI_BIAS_RELU, 1><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, 2); break;
        case 1: gemm_nt_bf16_kernel<128, 128, 2, EPI_MASK, 1><<<nb, 256>>>(A, K, B, K, nullptr, C, N, mb, 8, nullptr, K, 2); break;
        case 2: gemm_wgrad_bf16_kernel<128, 128, 2><<<4 * S, 256>>>(A, K, C, N, P, 256, P + 65536, slab, M / S, M, 2, 4); break;
        case 3: gemm_nt_bf16_kernel<128, 128, 2, EPI_BIAS_RELU, 1, 32, 3><<<nb, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, 2); break;
        case 4: gemm_nt_bf16_ring_kernel<128, 128, 2, EPI_BIAS_RELU, 1, 4, 2><<<512, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, 2, (int)nb); break;
        case 5: gemm_nt_bf16_ring_kernel<128, 128, 2, EPI_BIAS_RELU, 1, 3, 3><<<768, 256>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, K, 2, (int)nb); break;
        case 6: gemm_nt_bf16_ring_kernel<128, 128, 2, EPI_MASK, 1, 4, 2><<<512, 256>>>(A, K, B, K, nullptr, C, N, mb, 8, nullptr, K, 2, (int)nb); break;
        case 7: gemm_nt_bf16_wsr_kernel<256, 128, EPI_BIAS_RELU, 1, 5><<<256, 512>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, 2, (int)(M / 256)); break;
        case 8: gemm_nt_bf16_wsr_kernel<256, 128, EPI_MASK, 1, 5><<<256, 512>>>(A, K, B, K, nullptr, C, N, mb, 8, nullptr, 2, (int)(M / 256)); break;
        case 9: gemm_nt_bf16_wsr_kernel<256, 128, EPI_BIAS_RELU, 1, 4><<<256, 512>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, 2, (int)(M / 256)); break;
        case 10: gemm_nt_bf16_wsr_kernel<256, 128, EPI_BIAS_RELU, 1, 5><<<256, 512>>>(A, K, B, K, bias, C, 0, nullptr, 8, nullptr, 2, (int)(M / 256)); break;
        case 11: gemm_nt_bf16_wsr_kernel<256, 128, EPI_BIAS_RELU, 1, 5><<<512, 512>>>(A, K, B, K, bias, C, N, nullptr, 8, mb, 2, (int)(M / 256)); break;
      }
    };
    const int NV = 12;
    const char* names[NV] = {"nt_bf16 fwd bias+relu", "nt_bf16 dgrad mask", "wgrad_bf16 split-M", "nt_bf16 fwd BK=32 w3",
                             "ring fwd S=4 x2", "ring fwd S=3 x3", "ring dgrad S=4 x2", "wsr fwd S=5", "wsr dgrad S=5",
                             "wsr fwd S=4", "wsr fwd no-store", "wsr fwd grid512"};
    const double fb = M * 256.0 * 2 * 2 + M * 32.0;
    const double bytes[NV] = {fb, fb, M * 256.0 * 2 * 2, fb, fb, fb, fb, fb, fb, fb, M * 256.0 * 2, fb};
    for (int v = 0; v < NV; ++v) run(v);
    CK(hipDeviceSynchronize());
    std::vector<float> ms[NV];
    for (int r = 0; r < 9; ++r)
      for (int v = 0; v < NV; ++v) {
        CK(hipEventRecord(e0)); run(v); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
        float t; CK(hipEventElapsedTime(&t, e0, e1)); ms[v].push_back(t);
      }
    for (int v = 0; v < NV; ++v) {
      std::sort(ms[v].begin(), ms[v].end());
      const double t = ms[v][ms[v].size() / 2];
      printf("%-24s median %.4f ms  %.0f TFLOP/s (%.1f%% of 2500)  %.2f TB/s algorithmic (%.1f%% of 8)\n", names[v], t,
             2.0 * M * N * K / t * 1e-9, 2.0 * M * N * K / t * 1e-9 / 2500 * 100, bytes[v] / t * 1e-9,
             bytes[v] / t * 1e-9 / 8 * 100);
    }
  }
  // ring kernel == register-staged kernel, bitwise (same k order), bf16 relu out + mask, at C3 size
  {
    const int64_t M = 4096LL * 48;
    const int N = 256, K = 256;
    std::vector<uint16_t> h((size_t)M * K);
    for (auto& v : h) v = f2bf(U(rng));
    nerf_bf16 *A, *B, *C1, *C2; float* bias; uint32_t *m1, *m2;
    // B also serves the K = 320 case (ldb 320)
    CK(hipMalloc(&A, M * K * 2)); CK(hipMalloc(&B, N * 320 * 2)); CK(hipMalloc(&C1, M * N * 2)); CK(hipMalloc(&C2, M * N * 2));
    CK(hipMalloc(&bias, N * 4)); CK(hipMalloc(&m1, M * 32)); CK(hipMalloc(&m2, M * 32));
    CK(hipMemcpy(A, h.data(), M * K * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, h.data() + 77, N * 320 * 2, hipMemcpyHostToDevice));
    std::vector<float> bb(N); for (auto& v : bb) v = U(rng);
    CK(hipMemcpy(bias, bb.data(), N * 4, hipMemcpyHostToDevice));
    const int nt = (int)((M / 128) * 2);
    gemm_nt_bf16_kernel<128, 128, 2, EPI_BIAS_RELU, 1, 32, 3><<<nt, 256>>>(A, K, B, K, bias, C1, N, nullptr, 8, m1, K, 2);
    gemm_nt_bf16_ring_kernel<128, 128, 2, EPI_BIAS_RELU, 1, 4, 2><<<300, 256>>>(A, K, B, K, bias, C2, N, nullptr, 8, m2, K, 2, nt);
    CK(hipDeviceSynchronize());
    std::vector<uint16_t> c1(M * N), c2(M * N); std::vector<uint32_t> k1(M * 8), k2(M * 8);
    CK(hipMemcpy(c1.data(), C1, M * N * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(c2.data(), C2, M * N * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(k1.data(), m1, M * 32, hipMemcpyDeviceToHost)); CK(hipMemcpy(k2.data(), m2, M * 32, hipMemcpyDeviceToHost));
    size_t nd = 0, ndm = 0;
    for (size_t i = 0; i < c1.size(); ++i) nd += c1[i] != c2[i];
    for (size_t i = 0; i < k1.size(); ++i) ndm += k1[i] != k2[i];
    // EPI_MASK ring vs register-staged
    gemm_nt_bf16_kernel<128, 128, 2, EPI_MASK, 1, 32, 3><<<nt, 256>>>(A, K, B, K, nullptr, C1, N, m1, 8, nullptr, K, 2);
    gemm_nt_bf16_ring_kernel<128, 128, 2, EPI_MASK, 1, 3, 3><<<257, 256>>>(A, K, B, K, nullptr, C2, N, m1, 8, nullptr, K, 2, nt);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(c1.data(), C1, M * N * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(c2.data(), C2, M * N * 2, hipMemcpyDeviceToHost));
    size_t nd2 = 0;
    for (size_t i = 0; i < c1.size(); ++i) nd2 += c1[i] != c2[i];
    printf("ring vs register-staged: fwd %zu differing outputs, %zu mask words; dgrad %zu differing\n", nd, ndm, nd2);
    bad += (nd || ndm || nd2);
    gemm_nt_bf16_kernel<128, 128, 2, EPI_BIAS_RELU, 1, 32, 3><<<nt, 256>>>(A, K, B, K, bias, C1, N, nullptr, 8, m1, K, 2);
    gemm_nt_bf16_wsr_kernel<256, 128, EPI_BIAS_RELU, 1, 5><<<256, 512>>>(A, K, B, K, bias, C2, N, nullptr, 8, m2, 2, (int)(M / 256));
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(c1.data(), C1, M * N * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(c2.data(), C2, M * N * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(k1.data(), m1, M * 32, hipMemcpyDeviceToHost)); CK(hipMemcpy(k2.data(), m2, M * 32, hipMemcpyDeviceToHost));
    nd = 0; ndm = 0;
    for (size_t i = 0; i < c1.size(); ++i) nd += c1[i] != c2[i];
    for (size_t i = 0; i < k1.size(); ++i) ndm += k1[i] != k2[i];
    printf("wsr vs register-staged: fwd %zu differing outputs, %zu mask words\n", nd, ndm);
    bad += (nd || ndm);
    // K = 320 (trunk.4, lda 320) and K = 64 (trunk.0 / colour layer 0)
    for (int KK : {320, 64}) {
      // only the first M/2 rows: A holds M x 256 elements, so M/2 rows of 320 (or 64) fit
      gemm_nt_bf16_kernel<128, 128, 2, EPI_BIAS_RELU, 1, 32, 3><<<nt / 2, 256>>>(A, KK, B, KK, bias, C1, N, nullptr, 8, m1, KK, 2);
      if (KK == 320)
        gemm_nt_bf16_wsr_kernel<320, 128, EPI_BIAS_RELU, 1, 4><<<256, 512>>>(A, KK, B, KK, bias, C2, N, nullptr, 8, m2, 2, (int)(M / 256 / 2));
      else
        gemm_nt_bf16_wsr_kernel<64, 128, EPI_BIAS_RELU, 1, 5><<<256, 512>>>(A, KK, B, KK, bias, C2, N, nullptr, 8, m2, 2, (int)(M / 256 / 2));
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(c1.data(), C1, M / 2 * N * 2, hipMemcpyDeviceToHost)); CK(hipMemcpy(c2.data(), C2, M / 2 * N * 2, hipMemcpyDeviceToHost));
      nd = 0;
      for (size_t i = 0; i < (size_t)(M / 2 * N); ++i) nd += c1[i] != c2[i];
      printf("wsr K=%d vs register-staged: %zu differing outputs (first M/2 rows)\n", KK, nd);
      bad += nd != 0;
    }
  }
  printf(bad ? "FAILED\n" : "OK\n");
  return bad;
}
