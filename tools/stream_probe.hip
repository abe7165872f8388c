// HBM streaming probe: the achievable rate of the bf16 layer-backward traffic mix on this GPU (1,024 B/row read as
// two 512-B rows, 512 B/row written, 786,432 rows) — the practical roofline the fused layer kernels are compared
// against (the nominal 8 TB/s is a peak).  Variants: plain vs non-temporal loads / stores, unroll depth, grid.
//   hipcc -O3 --offload-arch=gfx950 tools/stream_probe.hip -o /tmp/stream_probe && /tmp/stream_probe
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int MODE, int U, bool NTL, bool NTS>  // MODE 0: read G + X, write D; 1: read only; 2: write only
__global__ __launch_bounds__(256) void stream_kernel(const u32x4* __restrict__ g, const u32x4* __restrict__ x,
                                                     u32x4* __restrict__ d, long n16, int sink) {
  const long stride = (long)gridDim.x * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += U * stride) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * stride;
      if (MODE != 2 && j < n16) {
        if (NTL) {
          a[u] = __builtin_nontemporal_load(g + j);
          b[u] = __builtin_nontemporal_load(x + j);
        } else {
          a[u] = g[j];
          b[u] = x[j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long j = i + u * stride;
      if (j < n16) {
        u32x4 v = MODE == 2 ? u32x4{(unsigned)j, 1u, 2u, 3u} : a[u] ^ b[u];
        if (MODE == 1) {
          acc ^= v;
        } else if (NTS) {
          __builtin_nontemporal_store(v, d + j);
        } else {
          d[j] = v;
        }
      }
    }
  }
  if (MODE == 1 && acc.x == 0x12345u && sink) d[0] = acc;
}

static hipEvent_t e0, e1;
template <int MODE, int U, bool NTL, bool NTS>
float run(int grid, const u32x4* g, const u32x4* x, u32x4* d, long n16) {
  float best = 1e9f;
  for (int it = 0; it < 10; ++it) {
    (void)hipEventRecord(e0);
    stream_kernel<MODE, U, NTL, NTS><<<grid, 256>>>(g, x, d, n16, 0);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (it >= 2 && ms < best) best = ms;
  }
  return best;
}

int main() {
  const long rows = 786432, n16 = rows * 512 / 16;  // 512-B rows
  u32x4 *g, *x, *d;
  (void)hipMalloc(&g, n16 * 16);
  (void)hipMalloc(&x, n16 * 16);
  (void)hipMalloc(&d, n16 * 16);
  (void)hipMemset(g, 1, n16 * 16);
  (void)hipMemset(x, 2, n16 * 16);
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double B0 = rows * 1536.0, B1 = rows * 1024.0, B2 = rows * 512.0;
  auto rep = [&](const char* what, int grid, double bytes, float ms) {
    printf("%-46s grid %5d %7.1f us %6.2f TB/s\n", what, grid, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
  };
  for (int grid : {1024, 4096, 8192}) {
    rep("mix plain U4", grid, B0, run<0, 4, false, false>(grid, g, x, d, n16));
    rep("mix plain U8", grid, B0, run<0, 8, false, false>(grid, g, x, d, n16));
    rep("mix nt-load U4", grid, B0, run<0, 4, true, false>(grid, g, x, d, n16));
    rep("mix nt-store U4", grid, B0, run<0, 4, false, true>(grid, g, x, d, n16));
    rep("mix nt-load nt-store U4", grid, B0, run<0, 4, true, true>(grid, g, x, d, n16));
    rep("mix nt-load nt-store U8", grid, B0, run<0, 8, true, true>(grid, g, x, d, n16));
    rep("read plain U4", grid, B1, run<1, 4, false, false>(grid, g, x, d, n16));
    rep("read nt U8", grid, B1, run<1, 8, true, false>(grid, g, x, d, n16));
    rep("write plain U4", grid, B2, run<2, 4, false, false>(grid, g, x, d, n16));
    rep("write nt U4", grid, B2, run<2, 4, false, true>(grid, g, x, d, n16));
  }
  return 0;
}
