// The MoE container of the reference on gfx950: point routing to K experts,
// order-preserving per-expert dispatch lists, the weighted mix of expert outputs and the background MLP.
//
// Restates (psklavos1/NeRF-Sys adaptive_nerf/):
//   MetaContainer._routing            models/inr/meta_container.py:97-134
//   MetaContainer.forward (mix)       models/inr/meta_container.py:266-330  (index_add_ / index_copy_)
//   MetaContainer.background_color    models/inr/meta_container.py:334-363  (SH -> Linear-ReLU-Linear-Sigmoid)
//
// Data layout: routing weights W [M][K] fp32 (one-hot for hard routing), dispatch lists expert-major
// (rows of expert 0 in ascending order, then expert 1, ...; offsets[K+1]), so expert k evaluates the
// contiguous gather X[idx[off_k .. off_{k+1})] and the mix adds w * y back in expert order — the
// reference's summation order, bit for bit.  All kernels are HBM-bound row passes.
#include "common.hpp"

// the mix must round like the reference's index_add_(y * w): no fma contraction in this file
#pragma clang fp contract(off)

namespace {

constexpr int MOE_MAX_K = 32;

struct Cent {
  float c[MOE_MAX_K][3];
};

__global__ void route_kernel(const float* __restrict__ x, int64_t xs, int64_t M, Cent cen, int K, int c2d, float bm,
                             const int32_t* __restrict__ m_dev, float* __restrict__ W) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  if (m_dev && m >= *m_dev) {  // capacity rows past the device-side count: no expert
    for (int k = 0; k < K; ++k) W[m * K + k] = 0.f;
    return;
  }
  const float px = x[m * xs], py = x[m * xs + 1], pz = x[m * xs + 2];
  float dist[MOE_MAX_K];
  float mind = INFINITY;
  int arg = 0;
  for (int k = 0; k < K; ++k) {
    const float dy = py - cen.c[k][1], dz = pz - cen.c[k][2];
    float s = dy * dy + dz * dz;
    if (!c2d) {
      const float dx = px - cen.c[k][0];
      s = dx * dx + dy * dy + dz * dz;
    }
    const float dd = sqrtf(s);
    dist[k] = dd;
    if (dd < mind) { mind = dd; arg = k; }  // first minimum, as torch.argmin
  }
  float* w = W + m * K;
  if (bm > 1.0f) {
    float md = INFINITY;
    for (int k = 0; k < K; ++k) { dist[k] = fmaxf(dist[k], 1e-6f); md = fminf(md, dist[k]); }
    const float lim = bm * md;
    float inv[MOE_MAX_K];
    float den = 0.f;
    for (int k = 0; k < K; ++k) {
      inv[k] = dist[k] <= lim ? 1.0f / dist[k] : 0.f;
      den += inv[k];
    }
    den = fmaxf(den, 1e-6f);
    for (int k = 0; k < K; ++k) w[k] = inv[k] / den;
  } else {
    for (int k = 0; k < K; ++k) w[k] = k == arg ? 1.0f : 0.f;
  }
}

// per-block counts of routed rows per expert
__global__ void dispatch_count_kernel(const float* __restrict__ W, int64_t M, int K, float eps,
                                      int32_t* __restrict__ bcnt, const int32_t* __restrict__ m_dev) {
  __shared__ int cnt[MOE_MAX_K];
  if (m_dev && *m_dev < M) M = *m_dev;  // device-sized (nerf_moe_dispatch_n): rows past the count route nowhere
  if (threadIdx.x < MOE_MAX_K) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = 0; k < K; ++k) {
    const bool f = m < M && W[m * K + k] > eps;
    const uint64_t b = __ballot(f);
    if ((threadIdx.x & 63) == 0) atomicAdd(&cnt[k], (int)__popcll(b));
  }
  __syncthreads();
  if (threadIdx.x < K) bcnt[(int64_t)blockIdx.x * K + threadIdx.x] = cnt[threadIdx.x];
}

// one 256-thread workgroup per expert: exclusive scan of the per-block counts (each thread a contiguous run of
// blocks), per-expert totals -> tot[k].  A one-thread-per-expert loop took 0.54 ms at 5,700 blocks.
__global__ __launch_bounds__(256) void dispatch_scan_kernel(int32_t* __restrict__ bcnt, int64_t nblk, int K,
                                                            int32_t* __restrict__ tot) {
  __shared__ int ts[256];
  const int k = blockIdx.x;
  const int64_t chunk = (nblk + 255) / 256;
  const int64_t b0 = threadIdx.x * chunk, b1 = (b0 + chunk < nblk) ? b0 + chunk : nblk;
  int s = 0;
  for (int64_t b = b0; b < b1; ++b) s += bcnt[b * K + k];
  ts[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // Hillis-Steele inclusive scan
    const int v = threadIdx.x >= d ? ts[threadIdx.x - d] : 0;
    __syncthreads();
    ts[threadIdx.x] += v;
    __syncthreads();
  }
  int run = ts[threadIdx.x] - s;
  for (int64_t b = b0; b < b1; ++b) {
    const int c = bcnt[b * K + k];
    bcnt[b * K + k] = run;
    run += c;
  }
  if (threadIdx.x == 255) tot[k] = ts[255];
}

__global__ void dispatch_offsets_kernel(const int32_t* __restrict__ tot, int K, int32_t* __restrict__ offsets) {
  if (threadIdx.x != 0) return;
  int o = 0;
  offsets[0] = 0;
  for (int j = 0; j < K; ++j) { o += tot[j]; offsets[j + 1] = o; }
}

__global__ void dispatch_write_kernel(const float* __restrict__ W, int64_t M, int K, float eps,
                                      const int32_t* __restrict__ bbase, const int32_t* __restrict__ offsets,
                                      int32_t* __restrict__ idx, const int32_t* __restrict__ m_dev) {
  __shared__ int wcnt[MOE_MAX_K][4];
  if (m_dev && *m_dev < M) M = *m_dev;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (int k = 0; k < K; ++k) {
    const bool f = m < M && W[m * K + k] > eps;
    const uint64_t b = __ballot(f);
    if (lane == 0) wcnt[k][wave] = (int)__popcll(b);
  }
  __syncthreads();
  for (int k = 0; k < K; ++k) {
    const bool f = m < M && W[m * K + k] > eps;
    const uint64_t b = __ballot(f);
    if (f) {
      int pos = offsets[k] + bbase[(int64_t)blockIdx.x * K + k];
      for (int w = 0; w < wave; ++w) pos += wcnt[k][w];
      pos += (int)__popcll(b & ((1ull << lane) - 1ull));
      idx[pos] = (int32_t)m;
    }
  }
}

__global__ void gather_rows_kernel(const float* __restrict__ src, int64_t ss, const int32_t* __restrict__ idx, int64_t n,
                                   int cols, float* __restrict__ dst, int64_t ds, const int32_t* __restrict__ rng) {
  if (rng) {  // device-sized (nerf_gather_rows_rng): idx entries rng[0] .. rng[1] - 1 -> dst rows 0 ..
    const int64_t c = (int64_t)rng[1] - rng[0];
    n = c < n ? (c < 0 ? 0 : c) : n;
    idx += rng[0];
  }
  // grid-stride: the device-sized form launches a bounded grid over the capacity (most of it past the count)
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * cols; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / cols;
    const int c = (int)(t - i * cols);
    dst[i * ds + c] = src[(int64_t)idx[i] * ss + c];
  }
}

__global__ void combine_kernel(const float* __restrict__ y, int64_t n, int C, const int32_t* __restrict__ idx,
                               const float* __restrict__ W, int K, int k, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * C) return;
  const int64_t i = t / C;
  const int c = (int)(t - i * C);
  const int64_t m = idx[i];
  out[m * C + c] = out[m * C + c] + y[i * C + c] * W[m * K + k];
}

__global__ void combine_bwd_kernel(const float* __restrict__ dout, int64_t n, int C, const int32_t* __restrict__ idx,
                                   const float* __restrict__ W, int K, int k, float* __restrict__ dy) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * C) return;
  const int64_t i = t / C;
  const int c = (int)(t - i * C);
  const int64_t m = idx[i];
  dy[i * C + c] = dout[m * C + c] * W[m * K + k];
}

// ------------------------------------------------------------------ background MLP

constexpr int BG_MAXH = 64;

__device__ __forceinline__ void bg_enc(const float* __restrict__ d, int64_t ds, int64_t r, float e[16]) {
  float x = d[r * ds], y = d[r * ds + 1], z = d[r * ds + 2];
  // F.normalize (eps 1e-12) then SHEncoder.forward's own normalisation (clamp 1e-9)
  for (int pass = 0; pass < 2; ++pass) {
    const float n = fmaxf(sqrtf(x * x + y * y + z * z), pass == 0 ? 1e-12f : 1e-9f);
    x = x / n; y = y / n; z = z / n;
  }
  const float xx = x * x, yy = y * y, zz = z * z;
  e[0] = 0.28209479177387814f;
  e[1] = 0.4886025119029199f * y;
  e[2] = 0.4886025119029199f * z;
  e[3] = 0.4886025119029199f * x;
  e[4] = 1.0925484305920792f * x * y;
  e[5] = 1.0925484305920792f * y * z;
  e[6] = 0.9461746957575601f * zz - 0.31539156525251999f;
  e[7] = 1.0925484305920792f * x * z;
  e[8] = 0.5462742152960396f * (xx - yy);
  e[9] = 0.5900435899266435f * y * (3.0f * xx - yy);
  e[10] = 2.890611442640554f * x * y * z;
  e[11] = 0.4570457994644658f * y * (5.0f * zz - 1.0f);
  e[12] = 0.3731763325901154f * z * (5.0f * zz - 3.0f);
  e[13] = 0.4570457994644658f * x * (5.0f * zz - 1.0f);
  e[14] = 1.445305721320277f * z * (xx - yy);
  e[15] = 0.5900435899266435f * x * (xx - 3.0f * yy);
}

// packed weights: W1 [H][16] | b1 [H] | W2 [3][H] | b2 [3].  The hidden layer is consumed as it is produced (o
// accumulates h_j in j order, the same order as a separate second loop) so no H-long register array is indexed
// with a runtime bound (that spills to scratch); hs (LDS, may be null) keeps h for the backward.
__device__ __forceinline__ void bg_forward_row(const float* sw, int H, const float e[16], float o[3], float* hs) {
  const float* W1 = sw;
  const float* b1 = sw + 16 * H;
  const float* W2 = b1 + H;
  const float* b2 = W2 + 3 * H;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  for (int j = 0; j < H; ++j) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += W1[j * 16 + i] * e[i];
    const float h = fmaxf(s + b1[j], 0.f);
    if (hs) hs[j] = h;
    s0 += W2[j] * h;
    s1 += W2[H + j] * h;
    s2 += W2[2 * H + j] * h;
  }
  o[0] = s0 + b2[0];
  o[1] = s1 + b2[1];
  o[2] = s2 + b2[2];
}

__global__ __launch_bounds__(256) void bg_fwd_kernel(const float* __restrict__ d, int64_t ds, int64_t N,
                                                     const float* __restrict__ w, int H, float* __restrict__ out) {
  __shared__ float sw[16 * BG_MAXH + BG_MAXH + 3 * BG_MAXH + 3];
  const int P = 20 * H + 3;
  for (int i = threadIdx.x; i < P; i += blockDim.x) sw[i] = w[i];
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  float e[16], o[3];
  bg_enc(d, ds, r, e);
  bg_forward_row(sw, H, e, o, nullptr);
  for (int c = 0; c < 3; ++c) out[r * 3 + c] = 1.0f / (1.0f + expf(-o[c]));
}

// Backward over BG_RAYS rays per workgroup: wave 0 recomputes each ray's row (e, h, dz, dh) into LDS, then the
// 256 threads own parameters and sum their per-ray contributions over the block's rays in ray order (one slab per
// block, deterministic).  The previous form (every thread looping over all 20H+3 parameters with a wave reduction
// per parameter and runtime-indexed register arrays) took 0.22 ms for 4096 rays.
constexpr int BG_RAYS = 64;
__global__ __launch_bounds__(256) void bg_bwd_kernel(const float* __restrict__ d, int64_t ds, int64_t N,
                                                     const float* __restrict__ w, int H,
                                                     const float* __restrict__ gout, float* __restrict__ slab) {
  __shared__ float sw[16 * BG_MAXH + BG_MAXH + 3 * BG_MAXH + 3];
  __shared__ float es[BG_RAYS][17];
  __shared__ float hs[BG_RAYS][BG_MAXH + 1];
  __shared__ float dhs[BG_RAYS][BG_MAXH + 1];
  __shared__ float dzs[BG_RAYS][4];
  const int P = 20 * H + 3;
  for (int i = threadIdx.x; i < P; i += blockDim.x) sw[i] = w[i];
  __syncthreads();
  if (threadIdx.x < BG_RAYS) {
    const int q = threadIdx.x;
    const int64_t r = (int64_t)blockIdx.x * BG_RAYS + q;
    float e[16], o[3], dz[3] = {0.f, 0.f, 0.f};
    if (r < N) {
      bg_enc(d, ds, r, e);
      bg_forward_row(sw, H, e, o, hs[q]);
      for (int c = 0; c < 3; ++c) {
        const float sg = 1.0f / (1.0f + expf(-o[c]));
        dz[c] = gout[r * 3 + c] * (sg * (1.0f - sg));
      }
      const float* W2 = sw + 17 * H;
      for (int j = 0; j < H; ++j) {
        const float g = W2[j] * dz[0] + W2[H + j] * dz[1] + W2[2 * H + j] * dz[2];
        dhs[q][j] = hs[q][j] > 0.f ? g : 0.f;
      }
    } else {  // rows past N contribute zero
#pragma unroll
      for (int i = 0; i < 16; ++i) e[i] = 0.f;
      for (int j = 0; j < H; ++j) { hs[q][j] = 0.f; dhs[q][j] = 0.f; }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) es[q][i] = e[i];
    for (int c = 0; c < 3; ++c) dzs[q][c] = dz[c];
  }
  __syncthreads();
  for (int p = threadIdx.x; p < P; p += blockDim.x) {
    float v = 0.f;
    if (p < 16 * H) {
      const int j = p >> 4, i = p & 15;
      for (int q = 0; q < BG_RAYS; ++q) v += dhs[q][j] * es[q][i];
    } else if (p < 17 * H) {
      const int j = p - 16 * H;
      for (int q = 0; q < BG_RAYS; ++q) v += dhs[q][j];
    } else if (p < 20 * H) {
      const int c = (p - 17 * H) / H, j = (p - 17 * H) - c * H;
      for (int q = 0; q < BG_RAYS; ++q) v += dzs[q][c] * hs[q][j];
    } else {
      const int c = p - 20 * H;
      for (int q = 0; q < BG_RAYS; ++q) v += dzs[q][c];
    }
    slab[(int64_t)blockIdx.x * P + p] = v;
  }
}

__global__ void bg_reduce_kernel(const float* __restrict__ slab, int nblk, int P, float* __restrict__ dw) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= P) return;
  float s = 0.f;
  for (int b = 0; b < nblk; ++b) s += slab[(int64_t)b * P + p];
  dw[p] = s;
}

}  // namespace

extern "C" int nerf_moe_route(const float* x, int64_t x_stride, int64_t M, const float* centroids, int K,
                              int cluster_2d, float boundary_margin, float* weights, hipStream_t st) {
  if (M < 0 || K < 1 || K > MOE_MAX_K || x_stride < 3 || !centroids) return NERF_E_ARG;
  if (M == 0) return NERF_OK;
  if (!x || !weights) return NERF_E_ARG;
  Cent c{};
  for (int k = 0; k < K; ++k)
    for (int j = 0; j < 3; ++j) c.c[k][j] = centroids[3 * k + j];
  route_kernel<<<(unsigned)nerf_cdiv(M, 256), 256, 0, st>>>(x, x_stride, M, c, K, cluster_2d, boundary_margin,
                                                            nullptr, weights);
  return nerf_launch_status();
}

extern "C" int nerf_moe_route_n(const float* x, int64_t x_stride, int64_t capacity, const int32_t* m_dev,
                                const float* centroids, int K, int cluster_2d, float boundary_margin, float* weights,
                                hipStream_t st) {
  if (capacity < 0 || K < 1 || K > MOE_MAX_K || x_stride < 3 || !centroids || !m_dev) return NERF_E_ARG;
  if (capacity == 0) return NERF_OK;
  if (!x || !weights) return NERF_E_ARG;
  Cent c{};
  for (int k = 0; k < K; ++k)
    for (int j = 0; j < 3; ++j) c.c[k][j] = centroids[3 * k + j];
  route_kernel<<<(unsigned)nerf_cdiv(capacity, 256), 256, 0, st>>>(x, x_stride, capacity, c, K, cluster_2d,
                                                                   boundary_margin, m_dev, weights);
  return nerf_launch_status();
}

extern "C" int64_t nerf_moe_dispatch_workspace_bytes(int64_t M, int K) {
  if (M < 0 || K < 1 || K > MOE_MAX_K) return NERF_E_ARG;
  return nerf_cdiv(M < 1 ? 1 : M, 256) * K * 4 + MOE_MAX_K * 4 + 256;
}

static int moe_dispatch_impl(const float* weights, int64_t M, const int32_t* m_dev, int K, float eps, int32_t* offsets,
                             int32_t* idx, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (M < 0 || K < 1 || K > MOE_MAX_K || !offsets) return NERF_E_ARG;
  if (M == 0) {
    (void)hipMemsetAsync(offsets, 0, (K + 1) * sizeof(int32_t), st);
    return nerf_launch_status();
  }
  if (!weights || !idx || !ws) return NERF_E_ARG;
  const int64_t nblk = nerf_cdiv(M, 256);
  if (ws_bytes < nblk * K * 4 + MOE_MAX_K * 4) return NERF_E_WORKSPACE;
  int32_t* bcnt = reinterpret_cast<int32_t*>(ws);
  dispatch_count_kernel<<<(unsigned)nblk, 256, 0, st>>>(weights, M, K, eps, bcnt, m_dev);
  int32_t* tot = bcnt + nblk * K;
  dispatch_scan_kernel<<<K, 256, 0, st>>>(bcnt, nblk, K, tot);
  dispatch_offsets_kernel<<<1, 64, 0, st>>>(tot, K, offsets);
  dispatch_write_kernel<<<(unsigned)nblk, 256, 0, st>>>(weights, M, K, eps, bcnt, offsets, idx, m_dev);
  return nerf_launch_status();
}

extern "C" int nerf_moe_dispatch(const float* weights, int64_t M, int K, float eps, int32_t* offsets, int32_t* idx,
                                 void* ws, int64_t ws_bytes, hipStream_t st) {
  return moe_dispatch_impl(weights, M, nullptr, K, eps, offsets, idx, ws, ws_bytes, st);
}

extern "C" int nerf_moe_dispatch_n(const float* weights, int64_t cap, const int32_t* m_dev, int K, float eps,
                                   int32_t* offsets, int32_t* idx, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (!m_dev) return NERF_E_ARG;
  return moe_dispatch_impl(weights, cap, m_dev, K, eps, offsets, idx, ws, ws_bytes, st);
}

extern "C" int nerf_gather_rows(const float* src, int64_t src_stride, const int32_t* idx, int64_t n, int cols,
                                float* dst, int64_t dst_stride, hipStream_t st) {
  if (n < 0 || cols < 1 || src_stride < cols || dst_stride < cols) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!src || !idx || !dst) return NERF_E_ARG;
  gather_rows_kernel<<<(unsigned)nerf_cdiv(n * cols, 256), 256, 0, st>>>(src, src_stride, idx, n, cols, dst, dst_stride,
                                                                         nullptr);
  return nerf_launch_status();
}

extern "C" int nerf_gather_rows_rng(const float* src, int64_t src_stride, const int32_t* idx, const int32_t* rng,
                                    int64_t cap, int cols, float* dst, int64_t dst_stride, hipStream_t st) {
  if (cap < 0 || cols < 1 || src_stride < cols || dst_stride < cols || !rng) return NERF_E_ARG;
  if (cap == 0) return NERF_OK;
  if (!src || !idx || !dst) return NERF_E_ARG;
  const int64_t blocks = nerf_cdiv(cap * cols, 256);
  gather_rows_kernel<<<(unsigned)(blocks < 4096 ? blocks : 4096), 256, 0, st>>>(src, src_stride, idx, cap, cols, dst,
                                                                                dst_stride, rng);
  return nerf_launch_status();
}

extern "C" int nerf_moe_combine(const float* y, int64_t n, int C, const int32_t* idx, const float* weights, int K,
                                int k, float* out, hipStream_t st) {
  if (n < 0 || C < 1 || K < 1 || k < 0 || k >= K) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!y || !idx || !weights || !out) return NERF_E_ARG;
  combine_kernel<<<(unsigned)nerf_cdiv(n * C, 256), 256, 0, st>>>(y, n, C, idx, weights, K, k, out);
  return nerf_launch_status();
}

extern "C" int nerf_moe_combine_bwd(const float* d_out, int64_t n, int C, const int32_t* idx, const float* weights,
                                    int K, int k, float* d_y, hipStream_t st) {
  if (n < 0 || C < 1 || K < 1 || k < 0 || k >= K) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!d_out || !idx || !weights || !d_y) return NERF_E_ARG;
  combine_bwd_kernel<<<(unsigned)nerf_cdiv(n * C, 256), 256, 0, st>>>(d_out, n, C, idx, weights, K, k, d_y);
  return nerf_launch_status();
}

extern "C" int nerf_bg_mlp_fwd(const float* d, int64_t d_stride, int64_t N, const float* w, int H, float* out,
                               hipStream_t st) {
  if (N < 0 || H < 1 || H > BG_MAXH || d_stride < 3) return NERF_E_ARG;
  if (N == 0) return NERF_OK;
  if (!d || !w || !out) return NERF_E_ARG;
  bg_fwd_kernel<<<(unsigned)nerf_cdiv(N, 256), 256, 0, st>>>(d, d_stride, N, w, H, out);
  return nerf_launch_status();
}

extern "C" int64_t nerf_bg_mlp_workspace_bytes(int64_t N, int H) {
  if (N < 0 || H < 1 || H > BG_MAXH) return NERF_E_ARG;
  return nerf_cdiv(N < 1 ? 1 : N, BG_RAYS) * (20 * H + 3) * 4 + 256;
}

extern "C" int nerf_bg_mlp_bwd(const float* d, int64_t d_stride, int64_t N, const float* w, int H,
                               const float* d_out, float* d_w, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (N < 0 || H < 1 || H > BG_MAXH || d_stride < 3 || !d_w) return NERF_E_ARG;
  const int P = 20 * H + 3;
  if (N == 0) {
    (void)hipMemsetAsync(d_w, 0, P * sizeof(float), st);
    return nerf_launch_status();
  }
  if (!d || !w || !d_out || !ws) return NERF_E_ARG;
  const int64_t nblk = nerf_cdiv(N, BG_RAYS);
  if (ws_bytes < nblk * P * 4) return NERF_E_WORKSPACE;
  float* slab = reinterpret_cast<float*>(ws);
  bg_bwd_kernel<<<(unsigned)nblk, 256, 0, st>>>(d, d_stride, N, w, H, d_out, slab);
  bg_reduce_kernel<<<(unsigned)nerf_cdiv(P, 256), 256, 0, st>>>(slab, (int)nblk, P, d_w);
  return nerf_launch_status();
}

// ==================================================================================== occupancy MoE path
// render_rays_occ for a full container (nerfs/ray_rendering.py:384-481): per-expert AABB prefilter
// (_intersect_rays_aabb :171-190), union of the experts' marched segments per ray (_merge_segments_union
// :193-258, a per-ray Python loop in the reference), and the soft blend of sigma / rgb BEFORE integration.

namespace {

__global__ void rays_aabb_hit_kernel(const float* __restrict__ rays, int64_t N, float x0, float y0, float z0, float x1,
                                     float y1, float z1, int32_t* __restrict__ hit) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= N) return;
  const float* ry = rays + r * 8;
  const float mn[3] = {x0, y0, z0}, mx[3] = {x1, y1, z1};
  float tmin = -INFINITY, tmax = INFINITY;
  for (int a = 0; a < 3; ++a) {
    const float d = ry[3 + a];
    const float inv = fabsf(d) > 1e-9f ? 1.0f / d : 1.0f / 1e-9f;
    const float t0 = (mn[a] - ry[a]) * inv, t1 = (mx[a] - ry[a]) * inv;
    tmin = fmaxf(tmin, fminf(t0, t1));
    tmax = fminf(tmax, fmaxf(t0, t1));
  }
  hit[r] = fminf(tmax, ry[7]) > fmaxf(tmin, ry[6]) ? 1 : 0;
}

// idx of the set flags (order preserving): pos = exclusive scan of flags
__global__ void flag_compact_kernel(const int32_t* __restrict__ flag, const int32_t* __restrict__ pos, int64_t n,
                                    int32_t* __restrict__ idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && flag[i]) idx[pos[i]] = (int32_t)i;
}

// Per ray: K-way merge of the experts' sorted boundary lists (t0 list and t1 list of every expert), unique,
// -> segments between consecutive distinct boundaries.  seg (K*2 lists): for expert k the ray's samples are
// [s0k, s1k) of its packed arrays.  Count pass (out_off == nullptr) or write pass.
struct ExpertLists {
  const float* t0[8];
  const float* t1[8];
  const int32_t* off[8];   // per-expert offsets over the GLOBAL rays (N+1)
};

constexpr int UNION_CAP = 2048;  // boundaries per ray sorted in LDS; longer rays take the sequential merge

// sequential K-way merge of the ray's 2K sorted lists (t0 list and t1 list of every expert), exact-equality
// unique; calls emit(prev, cur) for each segment.  Returns the segment count.
template <typename Emit>
__device__ int merge_seq(const ExpertLists& E, int K, int64_t r, Emit emit) {
  int pa[8], pb[8], end[8];
  for (int k = 0; k < K; ++k) {
    pa[k] = E.off[k][r];
    pb[k] = pa[k];
    end[k] = E.off[k][r + 1];
  }
  float prev = 0.f;
  bool have = false;
  int nb = 0;
  while (true) {
    float best = INFINITY;
    int bk = -1, which = 0;
    for (int k = 0; k < K; ++k) {
      if (pa[k] < end[k] && E.t0[k][pa[k]] < best) { best = E.t0[k][pa[k]]; bk = k; which = 0; }
      if (pb[k] < end[k] && E.t1[k][pb[k]] < best) { best = E.t1[k][pb[k]]; bk = k; which = 1; }
    }
    if (bk < 0) break;
    if (which == 0) ++pa[bk]; else ++pb[bk];
    if (have && best == prev) continue;
    if (have) { emit(nb, prev, best); ++nb; }
    prev = best;
    have = true;
  }
  return nb;
}

// One wave (= one 64-thread workgroup) per ray: gather all boundaries into LDS, bitonic sort, unique by
// adjacent comparison + ballot prefix counts.  Count pass (out_off == nullptr) or write pass.
__global__ __launch_bounds__(64) void union_kernel(ExpertLists E, int K, int64_t N, int32_t* __restrict__ counts,
                                                   const int32_t* __restrict__ out_off, int32_t* __restrict__ ri_o,
                                                   float* __restrict__ t0_o, float* __restrict__ t1_o) {
  __shared__ float buf[UNION_CAP];
  const int64_t r = blockIdx.x;
  const int lane = threadIdx.x;
  int nb = 0;
  for (int k = 0; k < K; ++k) nb += 2 * (E.off[k][r + 1] - E.off[k][r]);
  if (nb > UNION_CAP) {  // rare: sequential merge on lane 0
    if (lane == 0) {
      const int64_t w0 = out_off ? out_off[r] : 0;
      const int n = merge_seq(E, K, r, [&](int j, float a, float b) {
        if (out_off) { ri_o[w0 + j] = (int32_t)r; t0_o[w0 + j] = a; t1_o[w0 + j] = b; }
      });
      if (!out_off) counts[r] = n;
    }
    return;
  }
  int P = 64;
  while (P < nb) P <<= 1;
  // gather: expert k's t0 list then its t1 list
  int base = 0;
  for (int k = 0; k < K; ++k) {
    const int s0 = E.off[k][r], c = E.off[k][r + 1] - s0;
    for (int i = lane; i < c; i += 64) {
      buf[base + i] = E.t0[k][s0 + i];
      buf[base + c + i] = E.t1[k][s0 + i];
    }
    base += 2 * c;
  }
  for (int i = nb + lane; i < P; i += 64) buf[i] = INFINITY;
  __syncthreads();
  for (int size = 2; size <= P; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = lane; i < P / 2; i += 64) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const bool up = (lo & size) == 0;
        const float a = buf[lo], b = buf[hi];
        if ((a > b) == up) { buf[lo] = b; buf[hi] = a; }
      }
      __syncthreads();
    }
  }
  // distinct boundaries: element i (< nb) is new if i == 0 or buf[i] != buf[i-1]
  int D = 0;
  for (int c0 = 0; c0 < nb; c0 += 64) {
    const int i = c0 + lane;
    D += (int)__popcll(__ballot(i < nb && (i == 0 || buf[i] != buf[i - 1])));
  }
  if (out_off && D >= 2) {
    const int64_t w0 = out_off[r];
    int j0 = 0;
    for (int c0 = 0; c0 < nb; c0 += 64) {
      const int i = c0 + lane;
      const bool isnew = i < nb && (i == 0 || buf[i] != buf[i - 1]);
      const uint64_t m = __ballot(isnew);
      if (isnew) {
        const int j = j0 + (int)__popcll(m & ((1ull << lane) - 1ull));  // index of this distinct boundary
        if (j > 0) t1_o[w0 + j - 1] = buf[i];                         // ends segment j-1
        if (j < D - 1) { ri_o[w0 + j] = (int32_t)r; t0_o[w0 + j] = buf[i]; }  // starts segment j
      }
      j0 += (int)__popcll(m);
    }
  }
  if (!out_off && lane == 0) counts[r] = D >= 2 ? D - 1 : 0;
}

// per-expert ray counts on the global ray index: cnt[hit_idx[i]] = counts_k[i]
__global__ void scatter_counts_kernel(const int32_t* __restrict__ hit_idx, const int32_t* __restrict__ cnt_k,
                                      int64_t n, int32_t* __restrict__ cnt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) cnt[hit_idx[i]] = cnt_k[i];
}

// blend of expert k's (rgb, sigma) rows into the mix accumulators (expert order, as the reference's sums):
// s[m] += W[m,k] * sigma ; c[m] += (W[m,k] * sigma) * rgb
// device-sized (rng): y rows 0 .. rng[1] - rng[0] - 1 pair with idx entries rng[0] ..
__device__ __forceinline__ const int32_t* rng_rows(const int32_t* __restrict__ rng, int64_t& n, const int32_t* idx) {
  if (rng) {
    const int64_t c = (int64_t)rng[1] - rng[0];
    n = c < n ? (c < 0 ? 0 : c) : n;
    idx += rng[0];
  }
  return idx;
}
__global__ void blend_kernel(const float* __restrict__ y, int64_t n, const int32_t* __restrict__ idx,
                             const float* __restrict__ W, int K, int k, float* __restrict__ s, float* __restrict__ c,
                             const int32_t* __restrict__ rng) {
  idx = rng_rows(rng, n, idx);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t m = idx[i];
  const float4 v = reinterpret_cast<const float4*>(y)[i];
  const float ws = W[m * K + k] * v.w;
  s[m] = s[m] + ws;
  c[m * 3] = c[m * 3] + ws * v.x;
  c[m * 3 + 1] = c[m * 3 + 1] + ws * v.y;
  c[m * 3 + 2] = c[m * 3 + 2] + ws * v.z;
}

// rs_mix[m] = [c / max(s, 1e-12), max(s, 1e-12)]
__global__ void blend_finish_kernel(const float* __restrict__ s, const float* __restrict__ c, int64_t M,
                                    float* __restrict__ rs, const int32_t* __restrict__ m_dev) {
  if (m_dev && *m_dev < M) M = *m_dev;
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  const float sn = fmaxf(s[m], 1e-12f);
  reinterpret_cast<float4*>(rs)[m] = make_float4(c[m * 3] / sn, c[m * 3 + 1] / sn, c[m * 3 + 2] / sn, sn);
}

// backward of the blend for expert k: given d rs_mix (M,4) and the raw sums, d y_k (n,4)
__global__ void blend_bwd_kernel(const float* __restrict__ y, int64_t n, const int32_t* __restrict__ idx,
                                 const float* __restrict__ W, int K, int k, const float* __restrict__ s,
                                 const float* __restrict__ rs, const float* __restrict__ drs, float* __restrict__ dy,
                                 const int32_t* __restrict__ rng) {
  idx = rng_rows(rng, n, idx);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t m = idx[i];
  const float4 v = reinterpret_cast<const float4*>(y)[i];
  const float4 mix = reinterpret_cast<const float4*>(rs)[m];
  const float4 g = reinterpret_cast<const float4*>(drs)[m];
  const float w = W[m * K + k];
  const bool live = s[m] >= 1e-12f;  // clamp_min(1e-12) passes the gradient only above the bound
  const float sn = fmaxf(s[m], 1e-12f);
  // rgb_mix = sum_k w_k sig_k c_k / sn ; sigma_mix = sn
  const float dc = w * v.w / sn;
  float dsig = (live ? g.w : 0.f) * w;
  const float gdot = g.x * (v.x - (live ? mix.x : 0.f)) + g.y * (v.y - (live ? mix.y : 0.f)) +
                     g.z * (v.z - (live ? mix.z : 0.f));
  dsig += w * gdot / sn;
  reinterpret_cast<float4*>(dy)[i] = make_float4(dc * g.x, dc * g.y, dc * g.z, dsig);
}

}  // namespace

extern "C" int nerf_rays_aabb_hit(const float* rays, int64_t N, const float* box, int32_t* hit, hipStream_t st) {
  if (N < 0 || !box) return NERF_E_ARG;
  if (N == 0) return NERF_OK;
  if (!rays || !hit) return NERF_E_ARG;
  rays_aabb_hit_kernel<<<(unsigned)nerf_cdiv(N, 256), 256, 0, st>>>(rays, N, box[0], box[1], box[2], box[3], box[4],
                                                                    box[5], hit);
  return nerf_launch_status();
}

extern "C" int nerf_flag_compact(const int32_t* flags, const int32_t* pos, int64_t n, int32_t* idx, hipStream_t st) {
  if (n < 0) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!flags || !pos || !idx) return NERF_E_ARG;
  flag_compact_kernel<<<(unsigned)nerf_cdiv(n, 256), 256, 0, st>>>(flags, pos, n, idx);
  return nerf_launch_status();
}

extern "C" int nerf_scatter_counts(const int32_t* hit_idx, const int32_t* counts_k, int64_t n, int32_t* counts,
                                   hipStream_t st) {
  if (n < 0) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!hit_idx || !counts_k || !counts) return NERF_E_ARG;
  scatter_counts_kernel<<<(unsigned)nerf_cdiv(n, 256), 256, 0, st>>>(hit_idx, counts_k, n, counts);
  return nerf_launch_status();
}

extern "C" int nerf_segments_union(const float* const* t0s, const float* const* t1s, const int32_t* const* offs, int K,
                                   int64_t N, int32_t* counts, const int32_t* out_off, int32_t* ray_idx, float* t0,
                                   float* t1, hipStream_t st) {
  if (K < 1 || K > 8 || N < 0 || !t0s || !t1s || !offs) return NERF_E_ARG;
  if (N == 0) return NERF_OK;
  if (!out_off && !counts) return NERF_E_ARG;
  ExpertLists E{};
  for (int k = 0; k < K; ++k) { E.t0[k] = t0s[k]; E.t1[k] = t1s[k]; E.off[k] = offs[k]; }
  union_kernel<<<(unsigned)N, 64, 0, st>>>(E, K, N, counts, out_off, ray_idx, t0, t1);
  return nerf_launch_status();
}

extern "C" int nerf_moe_blend(const float* y, int64_t n, const int32_t* idx, const float* weights, int K, int k,
                              float* s_acc, float* c_acc, hipStream_t st) {
  if (n < 0 || K < 1 || k < 0 || k >= K) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!y || !idx || !weights || !s_acc || !c_acc) return NERF_E_ARG;
  blend_kernel<<<(unsigned)nerf_cdiv(n, 256), 256, 0, st>>>(y, n, idx, weights, K, k, s_acc, c_acc, nullptr);
  return nerf_launch_status();
}

extern "C" int nerf_moe_blend_rng(const float* y, int64_t cap, const int32_t* idx, const int32_t* rng,
                                  const float* weights, int K, int k, float* s_acc, float* c_acc, hipStream_t st) {
  if (cap < 0 || K < 1 || k < 0 || k >= K || !rng) return NERF_E_ARG;
  if (cap == 0) return NERF_OK;
  if (!y || !idx || !weights || !s_acc || !c_acc) return NERF_E_ARG;
  blend_kernel<<<(unsigned)nerf_cdiv(cap, 256), 256, 0, st>>>(y, cap, idx, weights, K, k, s_acc, c_acc, rng);
  return nerf_launch_status();
}

extern "C" int nerf_moe_blend_finish(const float* s_acc, const float* c_acc, int64_t M, float* rgb_sigma,
                                     hipStream_t st) {
  if (M < 0) return NERF_E_ARG;
  if (M == 0) return NERF_OK;
  if (!s_acc || !c_acc || !rgb_sigma) return NERF_E_ARG;
  blend_finish_kernel<<<(unsigned)nerf_cdiv(M, 256), 256, 0, st>>>(s_acc, c_acc, M, rgb_sigma, nullptr);
  return nerf_launch_status();
}

extern "C" int nerf_moe_blend_finish_n(const float* s_acc, const float* c_acc, int64_t cap, const int32_t* m_dev,
                                       float* rgb_sigma, hipStream_t st) {
  if (cap < 0 || !m_dev) return NERF_E_ARG;
  if (cap == 0) return NERF_OK;
  if (!s_acc || !c_acc || !rgb_sigma) return NERF_E_ARG;
  blend_finish_kernel<<<(unsigned)nerf_cdiv(cap, 256), 256, 0, st>>>(s_acc, c_acc, cap, rgb_sigma, m_dev);
  return nerf_launch_status();
}

extern "C" int nerf_moe_blend_bwd(const float* y, int64_t n, const int32_t* idx, const float* weights, int K, int k,
                                  const float* s_acc, const float* rgb_sigma, const float* d_rgb_sigma, float* d_y,
                                  hipStream_t st) {
  if (n < 0 || K < 1 || k < 0 || k >= K) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!y || !idx || !weights || !s_acc || !rgb_sigma || !d_rgb_sigma || !d_y) return NERF_E_ARG;
  blend_bwd_kernel<<<(unsigned)nerf_cdiv(n, 256), 256, 0, st>>>(y, n, idx, weights, K, k, s_acc, rgb_sigma,
                                                                d_rgb_sigma, d_y, nullptr);
  return nerf_launch_status();
}

extern "C" int nerf_moe_blend_bwd_rng(const float* y, int64_t cap, const int32_t* idx, const int32_t* rng,
                                      const float* weights, int K, int k, const float* s_acc, const float* rgb_sigma,
                                      const float* d_rgb_sigma, float* d_y, hipStream_t st) {
  if (cap < 0 || K < 1 || k < 0 || k >= K || !rng) return NERF_E_ARG;
  if (cap == 0) return NERF_OK;
  if (!y || !idx || !weights || !s_acc || !rgb_sigma || !d_rgb_sigma || !d_y) return NERF_E_ARG;
  blend_bwd_kernel<<<(unsigned)nerf_cdiv(cap, 256), 256, 0, st>>>(y, cap, idx, weights, K, k, s_acc, rgb_sigma,
                                                                  d_rgb_sigma, d_y, rng);
  return nerf_launch_status();
}
