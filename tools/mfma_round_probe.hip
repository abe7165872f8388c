// How v_mfma_f32_32x32x16_bf16 rounds its fp32 accumulation (MI355X): C = +-1.0, sixteen equal exact products whose
// sum is 1.5 ulp(1.0) (round-to-nearest-even -> 2 ulp, round-toward-zero -> 1 ulp), 0.75 ulp (RNE -> 1, RTZ -> 0) and
// 0.25 ulp (RNE -> 0, RTZ -> 0); the same for v_mfma_f32_16x16x4_f32 (four products), and the plain VALU fmaf.
//   hipcc -O3 --offload-arch=gfx950 tools/mfma_round_probe.hip -o /tmp/mfma_round_probe && /tmp/mfma_round_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// out[0] = bf16 MFMA result (row 0 / col 0), out[1] = f32 16x16x4 MFMA result, out[2] = fmaf chain
__global__ void probe(float c0, float prod_sum_ulps, float* out) {
  const int l = threadIdx.x;
  // bf16: every lane's 8 A values and 8 B values: a * b per product, 16 products per output (k = 16)
  // product p = prod_sum_ulps * 2^-23 / 16: take a = 2^-8, b = prod_sum_ulps * 2^-19 (exact in bf16 for 1.5, 0.75, 0.25)
  const float a = 0.00390625f, b = prod_sum_ulps * 1.9073486328125e-06f * (c0 < 0 ? -1.f : 1.f);
  bf16x8 av, bv;
  for (int t = 0; t < 8; ++t) { av[t] = (__bf16)a; bv[t] = (__bf16)b; }
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = c0;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av, bv, acc, 0, 0, 0);
  // f32 16x16x4: four products of a * (4 b)
  f32x4 acc2 = {c0, c0, c0, c0};
  acc2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, 4.f * b, acc2, 0, 0, 0);
  if (l == 0) {
    out[0] = acc[0];
    out[1] = acc2[0];
    float s = c0;
    s = fmaf(a * 16.f, b, s);
    out[2] = s;
  }
}

int main() {
  float* d;
  (void)hipMalloc(&d, 16);
  float h[3];
  for (float c0 : {1.f, -1.f})
    for (float u : {1.5f, 0.75f, 0.25f}) {
      probe<<<1, 64>>>(c0, u, d);
      (void)hipMemcpy(h, d, 12, hipMemcpyDeviceToHost);
      const float ulp = 1.1920928955078125e-07f;
      printf("C=%+.0f products sum %.2f ulp: bf16 32x32x16 -> %+.2f ulp, f32 16x16x4 -> %+.2f ulp, fmaf -> %+.2f ulp\n", c0, u,
             (h[0] - c0) / ulp, (h[1] - c0) / ulp, (h[2] - c0) / ulp);
    }
  return 0;
}
