// Ray-dataset build on the GPU: _process_single_image
// (adaptive_nerf/data/ram_rays_dataset.py:46-121) after ray generation. The reference masks the (H*W, 8) rays
// and the uint8 pixels with the keep mask (:97-104), clamps near/far (:107-109) and keeps the valid rays
// (:114-115), then attaches the image index (:117). The two boolean filters commute with the row-wise clamp,
// so one keep flag per pixel (mask && valid) + an exclusive scan + one compaction pass gives the same rows in the
// same order. The compaction writes rays (8 floats), rgb (3 floats, already /255 by nerf_rays_gen) and the
// int32 image index straight into the dataset's concatenated arrays at a caller-given row offset.
#include "common.hpp"

namespace {
__global__ void keep_flags_kernel(const uint8_t* __restrict__ valid, const uint8_t* __restrict__ mask, int64_t n,
                                  int32_t* __restrict__ flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  flags[i] = (valid[i] != 0) && (mask == nullptr || mask[i] != 0);
}

// one thread per source pixel; kept rows are written as two float4 (rays) + 3 floats + 1 int
__global__ void compact_kernel(const float* __restrict__ rays, const float* __restrict__ rgb,
                               const int32_t* __restrict__ flags, const int32_t* __restrict__ pos, int64_t n,
                               int32_t image_index, float* __restrict__ out_rays, float* __restrict__ out_rgb,
                               int32_t* __restrict__ out_idx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || !flags[i]) return;
  const int64_t o = pos[i];
  const float4* r = reinterpret_cast<const float4*>(rays + 8 * i);
  float4* w = reinterpret_cast<float4*>(out_rays + 8 * o);
  w[0] = r[0];
  w[1] = r[1];
  out_rgb[3 * o + 0] = rgb[3 * i + 0];
  out_rgb[3 * o + 1] = rgb[3 * i + 1];
  out_rgb[3 * o + 2] = rgb[3 * i + 2];
  out_idx[o] = image_index;
}
}  // namespace

extern "C" int nerf_ray_keep_flags(const uint8_t* valid, const uint8_t* mask, int64_t n, int32_t* flags,
                                   hipStream_t stream) {
  if (n < 0) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!valid || !flags) return NERF_E_ARG;
  keep_flags_kernel<<<(unsigned)nerf_cdiv(n, 256), 256, 0, stream>>>(valid, mask, n, flags);
  return nerf_launch_status();
}

extern "C" int nerf_rays_compact(const float* rays, const float* rgb, const int32_t* flags, const int32_t* pos,
                                 int64_t n, int32_t image_index, float* out_rays, float* out_rgb, int32_t* out_idx,
                                 hipStream_t stream) {
  if (n < 0) return NERF_E_ARG;
  if (n == 0) return NERF_OK;
  if (!rays || !rgb || !flags || !pos || !out_rays || !out_rgb || !out_idx) return NERF_E_ARG;
  if ((reinterpret_cast<uintptr_t>(rays) | reinterpret_cast<uintptr_t>(out_rays)) & 15) return NERF_E_ALIGN;
  compact_kernel<<<(unsigned)nerf_cdiv(n, 256), 256, 0, stream>>>(rays, rgb, flags, pos, n, image_index, out_rays,
                                                                   out_rgb, out_idx);
  return nerf_launch_status();
}
