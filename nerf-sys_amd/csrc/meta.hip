// Meta-learning inner / outer updates on fast weights.
//
// nerf_sgd_multi: task_adapt's functional SGD step (adaptive_nerf/pipelines/offline_stage/meta_core.py:61-64),
//   out_i = w_i - lr * g_i for every fast tensor i in ONE launch (blockIdx.y = tensor). torch computes
//   `inner_lr * g` and the subtraction as two rounded fp32 ops; this file is built with -ffp-contract=off so the
//   result is bit-identical.
// nerf_reptile_update: reptile_meta_update (meta_core.py:145-176): per tensor, delta = (sum_f (fast_f - theta)) / n
//   accumulated in fast-list order, and theta += lr * delta only when every element of delta is finite and
//   sum |delta| > 0 (the reference's per-tensor guard) — pass 1 sets the guard flags, pass 2 applies.
#include "common.hpp"

namespace {
constexpr int META_MAX = 64;   // tensors per launch
constexpr int REPTILE_MAX_FAST = 16;

struct SgdList {
  const float* w[META_MAX];
  const float* g[META_MAX];
  float* o[META_MAX];
  int64_t n[META_MAX];
};

__global__ void sgd_multi_kernel(SgdList L, float lr) {
  const int t = blockIdx.y;
  const float* w = L.w[t];
  const float* g = L.g[t];
  float* o = L.o[t];
  const int64_t n = L.n[t];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (g) {
      const float step = lr * g[i];
      o[i] = w[i] - step;
    } else {
      o[i] = w[i];
    }
  }
}

// one launch covers up to REPTILE_PTRS (tensor, fast copy) pointers; the host loops over tensor chunks
constexpr int REPTILE_PTRS = 128;
struct ReptileList {
  float* theta[META_MAX];
  int64_t n[META_MAX];
  const float* fast[REPTILE_PTRS];  // fast[t * n_fast + f] = the f-th fast copy of chunk tensor t
  int n_fast;
};

__device__ __forceinline__ float reptile_delta(const ReptileList& L, int t, int64_t i, float th) {
  float s = 0.f;  // sum_delta starts at zeros and gets add_(v - theta) per fast copy, in order
  for (int f = 0; f < L.n_fast; ++f) s = s + (L.fast[t * L.n_fast + f][i] - th);
  return s / (float)L.n_fast;
}

__global__ void reptile_check_kernel(ReptileList L, int32_t* flags) {
  const int t = blockIdx.y;
  const float* th = L.theta[t];
  int bad = 0, nz = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < L.n[t]; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = reptile_delta(L, t, i, th[i]);
    bad |= !isfinite(d);
    nz |= (d != 0.f);
  }
  const unsigned long long b = __ballot(bad), z = __ballot(nz);  // one atomic per wave
  if ((threadIdx.x & 63) == 0) {
    if (b) atomicOr(&flags[2 * t], 1);
    if (z) atomicOr(&flags[2 * t + 1], 1);
  }
}

__global__ void reptile_apply_kernel(ReptileList L, float lr, const int32_t* flags) {
  const int t = blockIdx.y;
  if (flags[2 * t] || !flags[2 * t + 1]) return;  // non-finite or all-zero delta: tensor left as is
  float* th = L.theta[t];
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < L.n[t]; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = reptile_delta(L, t, i, th[i]);
    const float step = lr * d;
    th[i] = th[i] + step;
  }
}

unsigned grid_x(int64_t mx) {
  const int64_t b = nerf_cdiv(mx, 256);
  return (unsigned)(b < 1 ? 1 : (b > 1024 ? 1024 : b));
}
}  // namespace

extern "C" int nerf_sgd_multi(int n_tensors, const float* const* w, const float* const* g, float* const* out,
                              const int64_t* numel, float lr, hipStream_t stream) {
  if (n_tensors < 0 || n_tensors > META_MAX) return NERF_E_ARG;
  if (n_tensors == 0) return NERF_OK;
  if (!w || !g || !out || !numel) return NERF_E_ARG;
  SgdList L{};
  int64_t mx = 0;
  for (int i = 0; i < n_tensors; ++i) {
    if (numel[i] < 0 || (numel[i] > 0 && (!w[i] || !out[i]))) return NERF_E_ARG;
    L.w[i] = w[i]; L.g[i] = g[i]; L.o[i] = out[i]; L.n[i] = numel[i];
    if (numel[i] > mx) mx = numel[i];
  }
  if (mx == 0) return NERF_OK;
  sgd_multi_kernel<<<dim3(grid_x(mx), n_tensors), 256, 0, stream>>>(L, lr);
  return nerf_launch_status();
}

extern "C" int64_t nerf_reptile_workspace_bytes(int n_tensors) {
  return n_tensors < 0 ? -1 : (int64_t)2 * n_tensors * (int64_t)sizeof(int32_t);
}

extern "C" int nerf_reptile_update(int n_tensors, float* const* theta, const float* const* fast, int n_fast,
                                   const int64_t* numel, float lr, int32_t* flags, int64_t ws_bytes,
                                   hipStream_t stream) {
  if (n_tensors < 0 || n_fast < 1 || n_fast > REPTILE_PTRS) return NERF_E_ARG;
  if (n_tensors == 0) return NERF_OK;
  if (!theta || !fast || !numel || !flags) return NERF_E_ARG;
  if (ws_bytes < nerf_reptile_workspace_bytes(n_tensors)) return NERF_E_WORKSPACE;
  for (int i = 0; i < n_tensors; ++i) {
    if (numel[i] < 0 || (numel[i] > 0 && !theta[i])) return NERF_E_ARG;
    for (int f = 0; f < n_fast; ++f)
      if (numel[i] > 0 && !fast[(int64_t)i * n_fast + f]) return NERF_E_ARG;
  }
  if (hipMemsetAsync(flags, 0, (size_t)2 * n_tensors * sizeof(int32_t), stream) != hipSuccess) return NERF_E_ARG;
  int per = REPTILE_PTRS / n_fast;
  if (per > META_MAX) per = META_MAX;
  for (int c0 = 0; c0 < n_tensors; c0 += per) {
    const int nt = n_tensors - c0 < per ? n_tensors - c0 : per;
    ReptileList L{};
    L.n_fast = n_fast;
    int64_t mx = 0;
    for (int t = 0; t < nt; ++t) {
      L.theta[t] = theta[c0 + t];
      L.n[t] = numel[c0 + t];
      for (int f = 0; f < n_fast; ++f) L.fast[t * n_fast + f] = fast[(int64_t)(c0 + t) * n_fast + f];
      if (L.n[t] > mx) mx = L.n[t];
    }
    if (mx == 0) continue;
    const dim3 grid(grid_x(mx), nt);
    reptile_check_kernel<<<grid, 256, 0, stream>>>(L, flags + 2 * c0);
    reptile_apply_kernel<<<grid, 256, 0, stream>>>(L, lr, flags + 2 * c0);
    const int st = nerf_launch_status();
    if (st != NERF_OK) return st;
  }
  return NERF_OK;
}
