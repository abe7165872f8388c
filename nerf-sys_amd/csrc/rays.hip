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

// One ray of get_ray_directions + get_rays (+ the AABB slab test): pixel (row, col) of the camera c2w M (3x4)
// -> o[3], d[3], near, far. Shared by the batch / dense generator and the dataset build so both give the same bits.
__device__ __forceinline__ void make_ray(const float* M, int row, int col, float fx, float fy, float cx, float cy,
                                         int center, float near_v, float far_v, const float* aabb, float max_bound,
                                         float invalid, float o[3], float d[3], float& tn, float& tf) {
  float i = (float)col, j = (float)row;
  if (center) { i += 0.5f; j += 0.5f; }
  float x = (i - cx) / fx, y = -((j - cy) / fy), z = -1.0f;
  float nrm = sqrtf(x * x + y * y + z * z);
  nrm = fmaxf(nrm, 1e-12f);
  x = x / nrm; y = y / nrm; z = z / nrm;
  o[0] = M[3]; o[1] = M[7]; o[2] = M[11];
#pragma unroll
  for (int r = 0; r < 3; ++r) d[r] = x * M[4 * r + 0] + y * M[4 * r + 1] + z * M[4 * r + 2];
  tn = near_v;
  tf = far_v;
  if (aabb) aabb_slab(o, d, aabb, max_bound, invalid, tn, tf);
}

// clamp_rays_near_far (nerfs/ray_sampling.py:139-176) of one ray; returns valid
__device__ __forceinline__ bool clamp_ray(float& a, float& b, int has_near, float nv, int has_far, float fv, float eps,
                                          float invalid) {
  if (has_near) a = fmaxf(a, nv);
  if (has_far) b = fminf(b, fv);
  const bool ok = isfinite(a) && isfinite(b) && (b > a + eps);
  if (has_near || has_far) {
    a = ok ? a : invalid;
    b = ok ? b : invalid;
  }
  return ok;
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
  float o[3], d[3], tn, tf;
  make_ray(c2w + 12 * (int64_t)im, row, col, fx, fy, cx, cy, center, near_v, far_v, aabb, max_bound, invalid, o, d,
           tn, tf);
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

// RamRaysDataset build (data/ram_rays_dataset.py:46-121) for a run of same-size images, two passes around one
// exclusive scan. Count pass (pos == NULL): flags[g] = mask && valid-after-clamp for every pixel g of the run.
// Write pass: a pixel is kept iff pos[g+1] > pos[g]; its ray is recomputed (ALU is free here, the 44-byte
// intermediate row is not) and written with its colour / 255 and image index at row pos[g]. HBM per pixel:
// mask 1 B + flags 4 B (count), scan 8 B, pos 4 B + pixel 3 B + 48 B per kept row (write).
struct DatasetArgs {
  const float* c2w;         // n_images x 12
  const float* intr;        // n_images x 4: fx fy cx cy
  const int32_t* image_index;
  int H, W, center;
  const float* aabb;
  int has_near, has_far;
  float near_v, far_v;
  const uint8_t* images;    // n_images x H x W x 3
  const uint8_t* masks;     // n_images x H x W, or NULL
};

__device__ __forceinline__ bool dataset_ray(const DatasetArgs& A, int64_t g, int& im, float o[3], float d[3],
                                            float& tn, float& tf) {
  const int64_t hw = (int64_t)A.H * A.W;
  im = (int)(g / hw);
  const int64_t q = g - (int64_t)im * hw;
  const int row = (int)(q / A.W), col = (int)(q - (int64_t)row * A.W);
  const float* K = A.intr + 4 * (int64_t)im;
  make_ray(A.c2w + 12 * (int64_t)im, row, col, K[0], K[1], K[2], K[3], A.center, 0.f, 0.f, A.aabb, 1e10f, 1e10f, o,
           d, tn, tf);
  return clamp_ray(tn, tf, A.has_near, A.near_v, A.has_far, A.far_v, 1e-6f, INFINITY);
}

__global__ void dataset_count_kernel(DatasetArgs A, int64_t n, int32_t* __restrict__ flags) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  int keep = 0;
  if (A.masks == nullptr || A.masks[g]) {
    int im;
    float o[3], d[3], tn, tf;
    keep = dataset_ray(A, g, im, o, d, tn, tf) ? 1 : 0;
  }
  flags[g] = keep;
}

__global__ void dataset_write_kernel(DatasetArgs A, int64_t n, const int32_t* __restrict__ pos,
                                     float* __restrict__ out_rays, float* __restrict__ out_rgb,
                                     int32_t* __restrict__ out_idx) {
  const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const int32_t r = pos[g];
  if (pos[g + 1] == r) return;
  int im;
  float o[3], d[3], tn, tf;
  dataset_ray(A, g, im, o, d, tn, tf);
  float4* w = reinterpret_cast<float4*>(out_rays + 8 * (int64_t)r);
  w[0] = make_float4(o[0], o[1], o[2], d[0]);
  w[1] = make_float4(d[1], d[2], tn, tf);
  const uint8_t* px = A.images + 3 * g;
  out_rgb[3 * (int64_t)r + 0] = px[0] / 255.0f;
  out_rgb[3 * (int64_t)r + 1] = px[1] / 255.0f;
  out_rgb[3 * (int64_t)r + 2] = px[2] / 255.0f;
  out_idx[r] = A.image_index[im];
}

// step_dev (graph-captured steps): the stream's seed is seed + *step_dev * seed_mul, read from device memory
__global__ void pick_pixels_kernel(int64_t n, int n_images, int H, int W, uint64_t seed,
                                   const int64_t* __restrict__ step_dev, uint64_t seed_mul, int32_t* __restrict__ pix) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n) return;
  if (step_dev) seed += (uint64_t)step_dev[0] * seed_mul;
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
  const bool ok = clamp_ray(a, b, has_near, nv, has_far, fv, eps, invalid);
  if (has_near || has_far) {
    rays[8 * p + 6] = a;
    rays[8 * p + 7] = b;
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
  pick_pixels_kernel<<<blocks_for(n, 256), 256, 0, stream>>>(n, n_images, H, W, seed, nullptr, 0, pix_out);
  return nerf_launch_status();
}

extern "C" int nerf_pick_pixels_dseed(int64_t n, int n_images, int H, int W, uint64_t seed_base, uint64_t seed_mul,
                                      const int64_t* step_dev, int32_t* pix_out, hipStream_t stream) {
  NERF_CHECK_ARG(pix_out && step_dev && n >= 0 && n_images > 0 && H > 0 && W > 0);
  if (n == 0) return NERF_OK;
  pick_pixels_kernel<<<blocks_for(n, 256), 256, 0, stream>>>(n, n_images, H, W, seed_base, step_dev, seed_mul, pix_out);
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

extern "C" int nerf_dataset_rays(const float* c2w, const float* intrinsics, const int32_t* image_index,
                                 int n_images, int H, int W, int center_pixels, const float* aabb, int has_near,
                                 float near_v, int has_far, float far_v, const uint8_t* images, const uint8_t* masks,
                                 int32_t* flags, const int32_t* pos, float* out_rays, float* out_rgb,
                                 int32_t* out_idx, hipStream_t stream) {
  NERF_CHECK_ARG(n_images >= 0 && H > 0 && W > 0);
  if (n_images == 0) return NERF_OK;
  NERF_CHECK_ARG(c2w && intrinsics && image_index && aabb);
  const int64_t n = (int64_t)n_images * H * W;
  NERF_CHECK_ARG(n < INT32_MAX);  // row positions are an int32 scan
  DatasetArgs A{c2w, intrinsics, image_index, H, W, center_pixels, aabb, has_near, has_far, near_v, far_v, images,
                masks};
  if (pos == nullptr) {
    NERF_CHECK_ARG(flags);
    dataset_count_kernel<<<blocks_for(n, 256), 256, 0, stream>>>(A, n, flags);
  } else {
    NERF_CHECK_ARG(images && out_rays && out_rgb && out_idx);
    if (!nerf_aligned16(out_rays)) return NERF_E_ALIGN;
    dataset_write_kernel<<<blocks_for(n, 256), 256, 0, stream>>>(A, n, pos, out_rays, out_rgb, out_idx);
  }
  return nerf_launch_status();
}

// nerf_version() is generated by the Makefile (build/version.cpp): it carries the hash of the sources it was built from
