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
  float lr[8];      // lr / bc1 of the step (host-counted steps)
  double lr0[8];    // the groups' base learning rates (device-counted steps: lr / bc1 formed in the kernel)
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

__device__ __forceinline__ float clip_scale(const float* __restrict__ part, float max_norm, float* red) {
  if (!(part && max_norm > 0.f)) return 1.0f;
  const float s = block_sum(threadIdx.x < NPART ? part[threadIdx.x] : 0.f, red);
  return fminf(max_norm / (sqrtf(s) + 1e-6f), 1.0f);
}

struct AdamHyper {
  float b2, omb1, omb2, eps, wd, bc2s;
};

// one element, torch's single-tensor Adam order; elements outside every segment are returned unchanged
__device__ __forceinline__ void adam_elem(int64_t i, const Segs& segs, const AdamHyper& h, float scale, float g,
                                          float& p, float& m, float& v) {
  if (i < segs.off[0] || i >= segs.off[segs.n]) return;
  int sgi = 0;
  while (sgi + 1 < segs.n && i >= segs.off[sgi + 1]) ++sgi;
  const float lr = segs.lr[sgi];  // the step size lr / bc1
  float gi = g * scale;
  if (h.wd != 0.f) gi = gi + h.wd * p;
  m = m + h.omb1 * (gi - m);
  v = v * h.b2 + h.omb2 * (gi * gi);
  const float denom = sqrtf(v) / h.bc2s + h.eps;
  p = p + (-lr) * (m / denom);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_load(const float4* q) {
  const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(q));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store(float4 a, float4* q) {
  f32x4 v;
  v.x = a.x; v.y = a.y; v.z = a.z; v.w = a.w;
  __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(q));
}

__device__ __forceinline__ void adam4(int64_t e0, const Segs& segs, const AdamHyper& h, float scale, float4 g,
                                      float4& p, float4& m, float4& v) {
  if (e0 + 4 <= segs.off[0] || e0 >= segs.off[segs.n]) return;
  adam_elem(e0, segs, h, scale, g.x, p.x, m.x, v.x);
  adam_elem(e0 + 1, segs, h, scale, g.y, p.y, m.y, v.y);
  adam_elem(e0 + 2, segs, h, scale, g.z, p.z, m.z, v.z);
  adam_elem(e0 + 3, segs, h, scale, g.w, p.w, m.w, v.w);
}

// VEC: p, g, m, v 16-byte aligned -> float4 streams (28 B/element of HBM traffic; the scalar form ran at 4.7 TB/s
// over 134 M elements), the n % 4 tail element-wise.  step_dev (graph-captured steps): the step count is read from
// device memory and the bias corrections are formed here, in double as nerf_adam does on the host.
template <bool VEC>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n, Segs segs,
                                                   AdamHyper h, const float* __restrict__ part, float max_norm,
                                                   const int64_t* __restrict__ step_dev, double beta1, double beta2) {
  __shared__ float red[17];
  if (step_dev) {
    const double st = (double)step_dev[0];
    const double bc1 = 1.0 - pow(beta1, st), bc2 = 1.0 - pow(beta2, st);
    for (int i = 0; i < segs.n; ++i) segs.lr[i] = (float)(segs.lr0[i] / bc1);
    h.bc2s = (float)sqrt(bc2);
  }
  const float scale = clip_scale(part, max_norm, red);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i0 = 0;
  if (VEC) {
    const int64_t n4 = n / 4;
    float4* p4 = reinterpret_cast<float4*>(p);
    float4* m4 = reinterpret_cast<float4*>(m);
    float4* v4 = reinterpret_cast<float4*>(v);
    const float4* g4 = reinterpret_cast<const float4*>(g);
    // two float4 groups per thread per iteration (8 independent 16-B loads in flight), streaming stores
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + stride < n4; i += 2 * stride) {
      const int64_t j = i + stride;
      float4 pa = p4[i], ga = nt_load(g4 + i), ma = m4[i], va = v4[i];
      float4 pb = p4[j], gb = nt_load(g4 + j), mb = m4[j], vb = v4[j];
      adam4(4 * i, segs, h, scale, ga, pa, ma, va);
      adam4(4 * j, segs, h, scale, gb, pb, mb, vb);
      p4[i] = pa; nt_store(ma, m4 + i); nt_store(va, v4 + i);
      p4[j] = pb; nt_store(mb, m4 + j); nt_store(vb, v4 + j);
    }
    for (; i < n4; i += stride) {
      float4 pa = p4[i], ga = g4[i], ma = m4[i], va = v4[i];
      adam4(4 * i, segs, h, scale, ga, pa, ma, va);
      p4[i] = pa; m4[i] = ma; v4[i] = va;
    }
    i0 = 4 * n4;
  }
  for (int64_t i = i0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float pp = p[i], mm = m[i], vv = v[i];
    adam_elem(i, segs, h, scale, g[i], pp, mm, vv);
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
  }
}

}  // namespace

extern "C" int nerf_grad_sqnorm(const float* g, int64_t n, float* partials, hipStream_t stream) {
  NERF_CHECK_ARG(g && partials && n >= 0);
  sqnorm_kernel<<<NPART, 1024, 0, stream>>>(g, n, partials);
  return nerf_launch_status();
}

static int adam_launch(float* p, const float* g, float* m, float* v, int64_t n, const int64_t* seg_off_host,
                       const double* seg_lr_host, int n_seg, double beta1, double beta2, float eps, float weight_decay,
                       int step, const int64_t* step_dev, const float* partials, float max_norm, hipStream_t stream) {
  NERF_CHECK_ARG(p && g && m && v && n >= 0 && seg_off_host && seg_lr_host && n_seg >= 1 && n_seg <= 8 &&
                 (step >= 1 || step_dev));
  Segs s{};
  s.n = n_seg;
  for (int i = 0; i <= n_seg; ++i) s.off[i] = seg_off_host[i];
  const double bc1 = step_dev ? 1.0 : 1.0 - std::pow(beta1, (double)step);
  const double bc2 = step_dev ? 1.0 : 1.0 - std::pow(beta2, (double)step);
  for (int i = 0; i < n_seg; ++i) s.lr[i] = (float)(seg_lr_host[i] / bc1);
  for (int i = 0; i < n_seg; ++i) s.lr0[i] = seg_lr_host[i];
  for (int i = 0; i < n_seg; ++i) NERF_CHECK_ARG(s.off[i] <= s.off[i + 1]);
  NERF_CHECK_ARG(s.off[0] >= 0 && s.off[n_seg] <= n);
  const AdamHyper h{(float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), eps, weight_decay,
                    (float)std::sqrt(bc2)};
  const bool vec = nerf_aligned16(p) && nerf_aligned16(g) && nerf_aligned16(m) && nerf_aligned16(v);
  int64_t blocks = nerf_cdiv(vec ? n / 4 : n, 256);
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  if (vec)
    adam_kernel<true><<<(unsigned)blocks, 256, 0, stream>>>(p, g, m, v, n, s, h, partials, max_norm, step_dev, beta1,
                                                             beta2);
  else
    adam_kernel<false><<<(unsigned)blocks, 256, 0, stream>>>(p, g, m, v, n, s, h, partials, max_norm, step_dev, beta1,
                                                              beta2);
  return nerf_launch_status();
}

extern "C" int nerf_adam(float* p, const float* g, float* m, float* v, int64_t n, const int64_t* seg_off_host,
                         const double* seg_lr_host, int n_seg, double beta1, double beta2, float eps, float weight_decay,
                         int step, const float* partials, float max_norm, hipStream_t stream) {
  return adam_launch(p, g, m, v, n, seg_off_host, seg_lr_host, n_seg, beta1, beta2, eps, weight_decay, step, nullptr,
                     partials, max_norm, stream);
}

// nerf_adam with the step count in device memory (*step_dev >= 1, read by the kernel): a captured hipGraph replays
// it with the count its own increment node advanced (the step closure of nerf_amd/graph_step.py)
extern "C" int nerf_adam_dstep(float* p, const float* g, float* m, float* v, int64_t n, const int64_t* seg_off_host,
                               const double* seg_lr_host, int n_seg, double beta1, double beta2, float eps,
                               float weight_decay, const int64_t* step_dev, const float* partials, float max_norm,
                               hipStream_t stream) {
  NERF_CHECK_ARG(step_dev);
  return adam_launch(p, g, m, v, n, seg_off_host, seg_lr_host, n_seg, beta1, beta2, eps, weight_decay, 0, step_dev,
                     partials, max_norm, stream);
}

