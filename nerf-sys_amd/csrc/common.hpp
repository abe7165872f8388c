// Shared helpers for the gfx950 NeRF kernels (wave64, fp32).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/nerf_amd.h"

#define NERF_WAVE 64

// Compute units of the current device (256 on MI355X), read once per process (one process per GPU).
static inline int nerf_cu_count() {
  static int n_cu = 0;
  if (!n_cu) {
    int dev = 0, v = 0;
    (void)hipGetDevice(&dev);
    n_cu = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  return n_cu;
}

// Return the launch status of the last kernel as the C-ABI int convention.
static inline int nerf_launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? NERF_OK : (int)e;
}

// A HIP runtime call's result as the C-ABI int convention (include/nerf_amd.h: 0 ok, <0 NERF_E_*, >0 the hipError_t
// passed through — hipError_t values are positive, so they never collide with a NERF_E_* code).
static inline int nerf_hip_status(hipError_t e) { return e == hipSuccess ? NERF_OK : (int)e; }

#define NERF_CHECK_ARG(cond) \
  do {                       \
    if (!(cond)) return NERF_E_ARG; \
  } while (0)

static inline bool nerf_aligned16(const void* p) { return (((uintptr_t)p) & 15u) == 0; }

static inline int64_t nerf_cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ---------------------------------------------------------------- counter RNG
// splitmix64 finaliser over (seed, stream id, index) -> uniform float in [0,1) with 24 bits.
__device__ __forceinline__ uint64_t nerf_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
__device__ __forceinline__ float nerf_uniform(uint64_t seed, uint64_t a, uint64_t b) {
  uint64_t z = nerf_mix64(seed * 0x9e3779b97f4a7c15ULL + nerf_mix64(a * 0xd1b54a32d192ed03ULL + b));
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// ---------------------------------------------------------------- wave scans (64 lanes)
__device__ __forceinline__ int nerf_lane() { return (int)(threadIdx.x & 63); }

// inclusive prefix product across the wave
__device__ __forceinline__ float wave_incl_prod(float v) {
  const int lane = nerf_lane();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    float o = __shfl_up(v, d, 64);
    if (lane >= d) v *= o;
  }
  return v;
}
// inclusive prefix sum across the wave
__device__ __forceinline__ float wave_incl_sum(float v) {
  const int lane = nerf_lane();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    float o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}
