// Ray generation, near/far clamping, NDC, stratified sampling, point construction and the
// Fourier positional encoding — the HBM-bound front of the NeRF hot path (gfx950, fp32).
//
// Reference behaviour restated (paths in psklavos1/NeRF-Sys adaptive_nerf/):
//   get_ray_directions  nerfs/ray_sampling.py:111-136     get_rays  :50-108 (+ :10-24)
//   ray_aabb_intersect  nerfs/scene_box.py:45-107         clamp_rays_near_far  ray_sampling.py:139-176
//   stratified_t_vals   nerfs/ray_rendering.py:262-287    point build  ray_rendering.py:317-319
//   FrequencyEncoder    models/encodings.py:437-444
#include "common.hpp"

namespace {

__device__ __forceinline__ void aabb_slab(const float o[3], const float d[3], const float* aabb, float max_bound,
                                          float invalid, float& tn, float& tf) {
  const float eps = 1e-8f;
  float tmin = -INFINITY, tmax = INFINITY;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    float rd = d[k];
    if (fabsf(rd) < eps) rd = rd >= 0.f ? eps : -eps;
    const float inv = 1.0f / rd;
    const float t0 = (aabb[k] - o[k]) * inv;
    const float t1 = (aabb[3 + k] - o[k]) * inv;
    tmin = fmaxf(tmin, fminf(t0, t1));
    tmax = fminf(tmax, fmaxf(t0, t1));
  }
  tmin = fminf(fmaxf(tmin, 0.f), max_bound);
  tmax = fminf(fmaxf(tmax, 0.f), max_bound);
  if (tmax <= tmin) { tmin = invalid; tmax = invalid; }
  tn = tmin;
  tf = tmax;
}

__global__ void rays_gen_kernel(const float* __restrict__ c2w, const int32_t* __restrict__ pix, int64_t n, int H,
                                int W, float fx, float fy, float cx, float cy, int center, float near_v,
                                float far_v, const float* __restrict__ aabb, float max_bound, float invalid,
                                const uint8_t* __restrict__ img, float* __restrict__ rays,
                                float* __restrict__ rgb) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  int im, row, col;
  if (pix) {
    im = pix[3 * p];
    row = pix[3 * p + 1];
    col = pix[3 * p + 2];
  } else {
    im = 0;
    row = (int)(p / W);
    col = (int)(p % W);
  }
  float i = (float)col, j = (float)row;
  if (center) { i += 0.5f; j += 0.5f; }
  float x = (i - cx) / fx, y = -((j - cy) / fy), z = -1.0f;
  float nrm = sqrtf(x * x + y * y + z * z);
  nrm = fmaxf(nrm, 1e-12f);
  x = x / nrm; y = y / nrm; z = z / nrm;
  const float* M = c2w + 12 * (int64_t)im;
  float o[3] = {M[3], M[7], M[11]};
  float d[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) d[r] = x * M[4 * r + 0] + y * M[4 * r + 1] + z * M[4 * r + 2];
  float tn = near_v, tf = far_v;
  if (aabb) aabb_slab(o, d, aabb, max_bound, invalid, tn, tf);
  float4* out = reinterpret_cast<float4*>(rays + 8 * p);
  out[0] = make_float4(o[0], o[1], o[2], d[0]);
  out[1] = make_float4(d[1], d[2], tn, tf);
  if (img && rgb) {
    const uint8_t* px = img + (((int64_t)im * H + row) * W + col) * 3;
    rgb[3 * p + 0] = px[0] / 255.0f;
    rgb[3 * p + 1] = px[1] / 255.0f;
    rgb[3 * p + 2] = px[2] / 255.0f;
  }
}

__global__ void pick_pixels_kernel(int64_t n, int n_images, int H, int W, uint64_t seed, int32_t* __restrict__ pix) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const uint64_t z = nerf_mix64(seed * 0x9e3779b97f4a7c15ULL + nerf_mix64((uint64_t)p + 0x632be59bd9b4e019ULL));
  const uint64_t tot = (uint64_t)n_images * (uint64_t)H * (uint64_t)W;
  const uint64_t k = (uint64_t)(((unsigned __int128)z * tot) >> 64);  // unbiased-enough multiply-shift
  const uint64_t hw = (uint64_t)H * W;
  pix[3 * p] = (int32_t)(k / hw);
  pix[3 * p + 1] = (int32_t)((k % hw) / W);
  pix[3 * p + 2] = (int32_t)(k % W);
}

__global__ void clamp_kernel(float* __restrict__ rays, int64_t n, int has_near, float nv, int has_far, float fv,
                             float eps, float invalid, uint8_t* __restrict__ valid) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  float a = rays[8 * p + 6], b = rays[8 * p + 7];
  if (has_near) a = fmaxf(a, nv);
  if (has_far) b = fminf(b, fv);
  const bool ok = isfinite(a) && isfinite(b) && (b > a + eps);
  if (has_near || has_far) {
    rays[8 * p + 6] = ok ? a : invalid;
    rays[8 * p + 7] = ok ? b : invalid;
  }
  if (valid) valid[p] = ok ? 1 : 0;
}

__global__ void ndc_kernel(const float* __restrict__ in, int64_t n, float H, float W, float focal, float nearp,
                           float* __restrict__ out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  const float* r = in + 8 * p;
  float o0 = r[0], o1 = r[1], o2 = r[2];
  const float d0 = r[3], d1 = r[4], d2 = r[5];
  const float t = -(nearp + o2) / d2;
  o0 = o0 + t * d0; o1 = o1 + t * d1; o2 = o2 + t * d2;
  const float ax = -1.0f / (W / (2.0f * focal)), ay = -1.0f / (H / (2.0f * focal));
  float* q = out + 8 * p;
  q[0] = ax * o0 / o2;
  q[1] = ay * o1 / o2;
  q[2] = 1.0f + 2.0f * nearp / o2;
  q[3] = ax * (d0 / d2 - o0 / o2);
  q[4] = ay * (d1 / d2 - o1 / o2);
  q[5] = -2.0f * nearp / o2;
  q[6] = 0.0f;
  q[7] = 1.0f;
}

// torch.linspace(0,1,S)[s] on the CPU: symmetric evaluation around the midpoint.
__device__ __forceinline__ float linspace01(int s, int S) {
  if (S == 1) return 0.0f;
  const float step = 1.0f / (float)(S - 1);
  return (s < S / 2) ? step * (float)s : 1.0f - step * (float)(S - 1 - s);
}

__device__ __forceinline__ float t_lin_at(float nr, float fr, int s, int S) {
  const float tl = linspace01(s, S);
  const float a = nr * (1.0f - tl);
  const float b = fr * tl;
  return a + b;
}

// one thread per (ray, sample)
__global__ void stratified_kernel(const float* __restrict__ rays, int64_t n, int S, int randomized,
                                  const float* __restrict__ u, uint64_t seed, float* __restrict__ t) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * S) return;
  const int64_t r = idx / S;
  const int s = (int)(idx - r * S);
  const float nr = rays[8 * r + 6], fr = rays[8 * r + 7];
  float tv = t_lin_at(nr, fr, s, S);
  if (randomized) {
    const float tp = s > 0 ? t_lin_at(nr, fr, s - 1, S) : tv;
    const float tn = s < S - 1 ? t_lin_at(nr, fr, s + 1, S) : tv;
    const float low = s > 0 ? 0.5f * (tp + tv) : tv;
    const float high = s < S - 1 ? 0.5f * (tv + tn) : tv;
    const float uu = u ? u[idx] : nerf_uniform(seed, (uint64_t)r, (uint64_t)s);
    tv = low + (high - low) * uu;
  }
  t[idx] = tv;
}

__global__ void build_xd_kernel(const float* __restrict__ rays, const float* __restrict__ t, int64_t n, int S,
                                float* __restrict__ xd) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * S) return;
  const int64_t r = idx / S;
  const float* ry = rays + 8 * r;
  const float tv = t[idx];
  float* q = xd + 6 * idx;
  q[0] = ry[0] + ry[3] * tv;
  q[1] = ry[1] + ry[4] * tv;
  q[2] = ry[2] + ry[5] * tv;
  q[3] = ry[3];
  q[4] = ry[4];
  q[5] = ry[5];
}

__global__ void freq_encode_kernel(const float* __restrict__ x, int64_t n, int D, int L, int inc,
                                   float* __restrict__ out, int ld) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * D) return;
  const int64_t r = idx / D;
  const int k = (int)(idx - r * D);
  const float v = x[r * D + k];
  float* q = out + r * ld;
  if (inc) q[k] = v;
  float* pe = q + (inc ? D : 0) + k * 2 * L;
  float band = 1.0f;
  for (int l = 0; l < L; ++l) {
    float s, c;
    sincosf(v * band, &s, &c);
    pe[l] = c;
    pe[L + l] = s;
    band *= 2.0f;
  }
}

inline unsigned blocks_for(int64_t n, int bs) { return (unsigned)nerf_cdiv(n, bs); }

}  // namespace

extern "C" int nerf_rays_gen(const float* c2w, int n_poses, const int32_t* pix, int64_t n, int H, int W, float fx,
                             float fy, float cx, float cy, int center_pixels, float near_v, float far_v,
                             const float* aabb, float aabb_max_bound, float aabb_invalid, const uint8_t* images_u8,
                             float* rays_out, float* rgb_out, hipStream_t stream) {
  NERF_CHECK_ARG(c2w && rays_out && n >= 0 && n_poses >= 1 && H > 0 && W > 0);
  if (!nerf_aligned16(rays_out)) return NERF_E_ALIGN;
  if (!pix && n != (int64_t)H * W) return NERF_E_ARG;
  if (images_u8 && !rgb_out) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  rays_gen_kernel<<<blocks_for(n, 256), 256, 0, stream>>>(c2w, pix, n, H, W, fx, fy, cx, cy, center_pixels, near_v,
                                                           far_v, aabb, aabb_max_bound, aabb_invalid, images_u8,
                                                           rays_out, rgb_out);
  return nerf_launch_status();
}

extern "C" int nerf_pick_pixels(int64_t n, int n_images, int H, int W, uint64_t seed, int32_t* pix_out,
                                hipStream_t stream) {
  NERF_CHECK_ARG(pix_out && n >= 0 && n_images > 0 && H > 0 && W > 0);
  if (n == 0) return NERF_OK;
  pick_pixels_kernel<<<blocks_for(n, 256), 256, 0, stream>>>(n, n_images, H, W, seed, pix_out);
  return nerf_launch_status();
}

extern "C" int nerf_clamp_near_far(float* rays, int64_t n, int has_near, float near_v, int has_far, float far_v,
                                   float eps, float invalid_value, uint8_t* valid_out, hipStream_t stream) {
  NERF_CHECK_ARG(rays && n >= 0);
  if (n == 0) return NERF_OK;
  clamp_kernel<<<blocks_for(n, 256), 256, 0, stream>>>(rays, n, has_near, near_v, has_far, far_v, eps,
                                                        invalid_value, valid_out);
  return nerf_launch_status();
}

extern "C" int nerf_rays_ndc(const float* rays_in, int64_t n, int H, int W, float focal, float near_plane,
                             float* rays_out, hipStream_t stream) {
  NERF_CHECK_ARG(rays_in && rays_out && n >= 0 && H > 0 && W > 0 && focal > 0.f);
  if (n == 0) return NERF_OK;
  ndc_kernel<<<blocks_for(n, 256), 256, 0, stream>>>(rays_in, n, (float)H, (float)W, focal, near_plane, rays_out);
  return nerf_launch_status();
}

extern "C" int nerf_sample_stratified(const float* rays, int64_t n, int S, int randomized, const float* u,
                                      uint64_t seed, float* t_out, hipStream_t stream) {
  NERF_CHECK_ARG(rays && t_out && n >= 0 && S >= 1);
  if (n == 0) return NERF_OK;
  stratified_kernel<<<blocks_for(n * S, 256), 256, 0, stream>>>(rays, n, S, randomized, u, seed, t_out);
  return nerf_launch_status();
}

extern "C" int nerf_build_xd(const float* rays, const float* t, int64_t n, int S, float* xd_out,
                             hipStream_t stream) {
  NERF_CHECK_ARG(rays && t && xd_out && n >= 0 && S >= 1);
  if (n == 0) return NERF_OK;
  build_xd_kernel<<<blocks_for(n * S, 256), 256, 0, stream>>>(rays, t, n, S, xd_out);
  return nerf_launch_status();
}

extern "C" int nerf_freq_encode(const float* x, int64_t n, int D, int L, int include_input, float* out, int ld_out,
                                hipStream_t stream) {
  NERF_CHECK_ARG(x && out && n >= 0 && D >= 1 && L >= 0 && L <= 24);
  NERF_CHECK_ARG(ld_out >= D * (2 * L + (include_input ? 1 : 0)));
  if (n == 0) return NERF_OK;
  freq_encode_kernel<<<blocks_for(n * D, 256), 256, 0, stream>>>(x, n, D, L, include_input, out, ld_out);
  return nerf_launch_status();
}

extern "C" const char* nerf_version(void) { return "nerf_amd 0.1 gfx950"; }
