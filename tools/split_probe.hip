// Accuracy probe for fp32 GEMMs computed from bf16 split products on gfx950 (`v_mfma_f32_32x32x16_bf16`, fp32
// accumulation): every fp32 operand x = hi + mid + lo exactly (three round-to-nearest bf16 pieces of 8 significant
// bits each), and A.B^T = sum over the piece pairs.  Compared against an fp64 reference next to the two fp32 paths the
// repo uses today (16x16x4 fp32 MFMA, and a sequential fp32 fmaf chain like the CPU reference's), on the trunk-GEMM
// shape (K = 256) with forward-like data (ReLU activations x Kaiming weights) and backward-like data (masked small
// gradients).  Error metric per output: |C - C64| / sum_k |a_k b_k| (the scale any fp32 dot product's rounding error
// is bounded by); reported as max and mean over the outputs.
//   hipcc -O3 --offload-arch=gfx950 tools/split_probe.hip -o /tmp/split_probe && /tmp/split_probe
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int M = 8192, N = 256, K = 256;

__global__ void ref64_kernel(const float* A, const float* B, double* C, double* S) {
  const int m = blockIdx.x, n = threadIdx.x;
  double s = 0.0, a = 0.0;
  for (int k = 0; k < K; ++k) {
    const double p = (double)A[m * K + k] * (double)B[n * K + k];
    s += p;
    a += fabs(p);
  }
  C[m * N + n] = s;
  S[m * N + n] = a;
}

__global__ void fma_chain_kernel(const float* A, const float* B, float* C) {
  const int m = blockIdx.x, n = threadIdx.x;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s = fmaf(A[m * K + k], B[n * K + k], s);
  C[m * N + n] = s;
}

// one wave per 16x16 output block, k in steps of 4 (lane l: row / col l & 15, k-slot l >> 4)
__global__ void mfma_f32_kernel(const float* A, const float* B, float* C) {
  const int l = threadIdx.x, m0 = blockIdx.x * 16, n0 = blockIdx.y * 16;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += 4) {
    const float a = A[(m0 + (l & 15)) * K + k0 + (l >> 4)];
    const float b = B[(n0 + (l & 15)) * K + k0 + (l >> 4)];
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  }
  for (int v = 0; v < 4; ++v) C[(m0 + 4 * (l >> 4) + v) * N + n0 + (l & 15)] = acc[v];
}

__device__ inline void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
  h = (__bf16)x;
  const float r1 = x - (float)h;
  m = (__bf16)r1;
  const float r2 = r1 - (float)m;
  l = (__bf16)r2;
}

// one wave per 32x32 output block; NT = number of piece products (3: hh hm mh, 6: + hl mm lh, 9: all)
template <int NT>
__global__ void mfma_split_kernel(const float* A, const float* B, float* C) {
  const int l = threadIdx.x, m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int k0 = 0; k0 < K; k0 += 16) {
    bf16x8 a[3], b[3];
    for (int t = 0; t < 8; ++t) {
      __bf16 h, md, lo;
      split3(A[(m0 + (l & 31)) * K + k0 + 8 * (l >> 5) + t], h, md, lo);
      a[0][t] = h; a[1][t] = md; a[2][t] = lo;
      split3(B[(n0 + (l & 31)) * K + k0 + 8 * (l >> 5) + t], h, md, lo);
      b[0][t] = h; b[1][t] = md; b[2][t] = lo;
    }
    // smallest terms first
    if (NT >= 9) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[2], acc, 0, 0, 0);
    if (NT >= 9) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[2], acc, 0, 0, 0);
    if (NT >= 9) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[1], acc, 0, 0, 0);
    if (NT >= 6) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
    if (NT >= 6) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
    if (NT >= 6) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  }
  // 32x32 accumulator: register r of lane l holds row 8 (r / 4) + 4 (l / 32) + r % 4, column l % 32
  for (int r = 0; r < 16; ++r) C[(m0 + 8 * (r / 4) + 4 * (l >> 5) + (r & 3)) * N + n0 + (l & 31)] = acc[r];
}

// the same with the small terms accumulated in their own register set (added at the end): the large hh term then
// does not swamp the small ones inside the fp32 accumulator at every k step
template <int NT>
__global__ void mfma_split2_kernel(const float* A, const float* B, float* C) {
  const int l = threadIdx.x, m0 = blockIdx.x * 32, n0 = blockIdx.y * 32;
  f32x16 big, small;
  for (int r = 0; r < 16; ++r) big[r] = small[r] = 0.f;
  for (int k0 = 0; k0 < K; k0 += 16) {
    bf16x8 a[3], b[3];
    for (int t = 0; t < 8; ++t) {
      __bf16 h, md, lo;
      split3(A[(m0 + (l & 31)) * K + k0 + 8 * (l >> 5) + t], h, md, lo);
      a[0][t] = h; a[1][t] = md; a[2][t] = lo;
      split3(B[(n0 + (l & 31)) * K + k0 + 8 * (l >> 5) + t], h, md, lo);
      b[0][t] = h; b[1][t] = md; b[2][t] = lo;
    }
    if (NT >= 9) small = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[2], small, 0, 0, 0);
    if (NT >= 9) small = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[2], small, 0, 0, 0);
    if (NT >= 9) small = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[1], small, 0, 0, 0);
    if (NT >= 6) small = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], small, 0, 0, 0);
    if (NT >= 6) small = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], small, 0, 0, 0);
    if (NT >= 6) small = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], small, 0, 0, 0);
    small = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], small, 0, 0, 0);
    small = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], small, 0, 0, 0);
    big = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], big, 0, 0, 0);
  }
  for (int r = 0; r < 16; ++r) C[(m0 + 8 * (r / 4) + 4 * (l >> 5) + (r & 3)) * N + n0 + (l & 31)] = big[r] + small[r];
}

static float urand(unsigned& s) {
  s = s * 1664525u + 1013904223u;
  return ((s >> 8) + 0.5f) / 16777216.0f;
}
static float nrand(unsigned& s) {
  const float u1 = urand(s), u2 = urand(s);
  return sqrtf(-2.f * logf(u1)) * cosf(6.2831853f * u2);
}

int main() {
  std::vector<float> hA(M * K), hB(N * K);
  float *A, *B, *C;
  double *C64, *S64;
  (void)hipMalloc(&A, M * K * 4);
  (void)hipMalloc(&B, N * K * 4);
  (void)hipMalloc(&C, M * N * 4);
  (void)hipMalloc(&C64, M * N * 8);
  (void)hipMalloc(&S64, M * N * 8);
  std::vector<float> hC(M * N);
  std::vector<double> hR(M * N), hS(M * N);
  for (int data = 0; data < 2; ++data) {
    unsigned s = 12345u + data;
    for (int i = 0; i < M * K; ++i) {
      const float v = nrand(s);
      hA[i] = data == 0 ? fmaxf(v, 0.f) * 0.7f : (v > 0.3f ? v * 3e-7f : 0.f);  // activations / masked gradients
    }
    for (int i = 0; i < N * K; ++i) hB[i] = (urand(s) * 2.f - 1.f) * 0.0625f;  // U(-1/sqrt(K), 1/sqrt(K))
    (void)hipMemcpy(A, hA.data(), M * K * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(B, hB.data(), N * K * 4, hipMemcpyHostToDevice);
    ref64_kernel<<<M, N>>>(A, B, C64, S64);
    (void)hipMemcpy(hR.data(), C64, M * N * 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(hS.data(), S64, M * N * 8, hipMemcpyDeviceToHost);
    auto report = [&](const char* what) {
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(hC.data(), C, M * N * 4, hipMemcpyDeviceToHost);
      double mx = 0, mean = 0, mxrel = 0;
      for (int i = 0; i < M * N; ++i) {
        if (hS[i] == 0) continue;
        const double e = fabs((double)hC[i] - hR[i]) / hS[i];
        mx = fmax(mx, e);
        mean += e;
        if (fabs(hR[i]) > 1e-3 * hS[i]) mxrel = fmax(mxrel, fabs((double)hC[i] - hR[i]) / fabs(hR[i]));
      }
      printf("%-10s %-34s max %.3e  mean %.3e  (x 2^-24: max %.2f mean %.3f)  max rel(|C| > 1e-3 scale) %.3e\n",
             data == 0 ? "forward" : "backward", what, mx, mean / (M * N), mx * 16777216.0, mean / (M * N) * 16777216.0,
             mxrel);
    };
    fma_chain_kernel<<<M, N>>>(A, B, C);
    report("fp32 fmaf chain (CPU-like)");
    mfma_f32_kernel<<<dim3(M / 16, N / 16), 64>>>(A, B, C);
    report("fp32 MFMA 16x16x4");
    mfma_split_kernel<3><<<dim3(M / 32, N / 32), 64>>>(A, B, C);
    report("bf16 x3 (hh hm mh)");
    mfma_split_kernel<6><<<dim3(M / 32, N / 32), 64>>>(A, B, C);
    report("bf16 x6 one accumulator");
    mfma_split_kernel<9><<<dim3(M / 32, N / 32), 64>>>(A, B, C);
    report("bf16 x9 one accumulator");
    mfma_split2_kernel<6><<<dim3(M / 32, N / 32), 64>>>(A, B, C);
    report("bf16 x6 big/small accumulators");
    mfma_split2_kernel<9><<<dim3(M / 32, N / 32), 64>>>(A, B, C);
    report("bf16 x9 big/small accumulators");
  }
  return 0;
}
