// clip_grad_norm_ + torch.optim.Adam over the flat packed parameter buffer (gfx950).
//
// Restates the plain train step of pipelines/online_stage/runtime_adapt.py:300-310
// (clip_grad_norm_(1.0), scaler.step(Adam)) with the param groups of common/utils.py:16-76
// (per-group learning rate).  Update order follows torch's single-tensor Adam:
//   m = lerp(m, g, 1-b1); v = v*b2 + (1-b2) g^2; p += -(lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps).
// The global norm is reduced deterministically: pass 1 writes 256 block partials, the Adam kernel
// re-sums them in a fixed order in every block (no host sync, graph-capturable).
#include <cmath>
#include "common.hpp"

namespace {

constexpr int NPART = 256;

struct Segs {
  int64_t off[9];
  float lr[8];
  int n;
};

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
    red[16] = s;
  }
  __syncthreads();
  return red[16];
}

// 256 blocks x 1024 threads, float4 loads, two independent accumulators: the pass is HBM-bound (a
// 256 x 256 scalar version ran at 0.8 TB/s on 134 M floats).
__global__ __launch_bounds__(1024) void sqnorm_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
  __shared__ float red[17];
  float s0 = 0.f, s1 = 0.f;
  const int64_t n4 = ((uintptr_t)g & 15u) ? 0 : n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + stride < n4; i += 2 * stride) {
    const float4 a = g4[i], b = g4[i + stride];
    s0 += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
    s1 += b.x * b.x + b.y * b.y + b.z * b.z + b.w * b.w;
  }
  for (; i < n4; i += stride) {
    const float4 a = g4[i];
    s0 += a.x * a.x + a.y * a.y + a.z * a.z + a.w * a.w;
  }
  for (int64_t j = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += stride) s1 += g[j] * g[j];
  const float s = block_sum(s0 + s1, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n, Segs segs,
                                                   float b2, float omb1, float omb2, float eps, float wd, float bc2s,
                                                   const float* __restrict__ part, float max_norm) {
  __shared__ float red[17];
  float scale = 1.0f;
  if (part && max_norm > 0.f) {
    const float s = block_sum(threadIdx.x < NPART ? part[threadIdx.x] : 0.f, red);
    const float norm = sqrtf(s);
    scale = fminf(max_norm / (norm + 1e-6f), 1.0f);
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int sgi = 0;
    while (sgi + 1 < segs.n && i >= segs.off[sgi + 1]) ++sgi;
    if (i < segs.off[0] || i >= segs.off[segs.n]) continue;
    const float lr = segs.lr[sgi];
    float gi = g[i] * scale;
    float pi = p[i];
    if (wd != 0.f) gi = gi + wd * pi;
    float mi = m[i];
    mi = mi + omb1 * (gi - mi);
    float vi = v[i] * b2 + omb2 * (gi * gi);
    const float denom = sqrtf(vi) / bc2s + eps;
    pi = pi + (-lr) * (mi / denom);  // lr here is the step size lr/bc1
    m[i] = mi;
    v[i] = vi;
    p[i] = pi;
  }
}

}  // namespace

extern "C" int nerf_grad_sqnorm(const float* g, int64_t n, float* partials, hipStream_t stream) {
  NERF_CHECK_ARG(g && partials && n >= 0);
  sqnorm_kernel<<<NPART, 1024, 0, stream>>>(g, n, partials);
  return nerf_launch_status();
}

extern "C" int nerf_adam(float* p, const float* g, float* m, float* v, int64_t n, const int64_t* seg_off_host,
                         const double* seg_lr_host, int n_seg, double beta1, double beta2, float eps, float weight_decay,
                         int step, const float* partials, float max_norm, hipStream_t stream) {
  NERF_CHECK_ARG(p && g && m && v && n >= 0 && seg_off_host && seg_lr_host && n_seg >= 1 && n_seg <= 8 && step >= 1);
  Segs s{};
  s.n = n_seg;
  for (int i = 0; i <= n_seg; ++i) s.off[i] = seg_off_host[i];
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  for (int i = 0; i < n_seg; ++i) s.lr[i] = (float)(seg_lr_host[i] / bc1);
  for (int i = 0; i < n_seg; ++i) NERF_CHECK_ARG(s.off[i] <= s.off[i + 1]);
  NERF_CHECK_ARG(s.off[0] >= 0 && s.off[n_seg] <= n);
  const float bc2s = (float)std::sqrt(bc2);
  int64_t blocks = nerf_cdiv(n, 256);
  if (blocks > 2048) blocks = 2048;
  if (blocks < 1) blocks = 1;
  adam_kernel<<<(unsigned)blocks, 256, 0, stream>>>(p, g, m, v, n, s, (float)beta2, (float)(1.0 - beta1),
                                                      (float)(1.0 - beta2), eps, weight_decay, bc2s, partials,
                                                      max_norm);
  return nerf_launch_status();
}

