// Hierarchical inverse-CDF resampling + sorted merge of coarse and fine depths (gfx950).
//
// ABSENT in the reference (psklavos1/NeRF-Sys has no sample_pdf) — canonical NeRF
// formulation (Mildenhall et al. 2020): interior coarse weights + 1e-5 -> pdf over the S-1 t-midpoints,
// cdf with a leading 0, u -> searchsorted(right=True), linear interpolation inside the bin (denominator
// < 1e-5 -> 1), then the union with the coarse t sorted.  Parity is pinned against the CPU oracle
// (oracle/nerf_oracle.py hierarchical_t_vals) on identical u, not against the reference.
//
// One wave64 per ray: wave scan for the cdf, binary search in LDS per fine sample, then a register
// bitonic sort of the 64*P (coarse + fine + inf padding) values, lane-blocked (element e = lane*P + p).
#include "common.hpp"

namespace {

constexpr int MAXS = 256;

__device__ __forceinline__ float linspace01(int s, int S) {
  if (S == 1) return 0.0f;
  const float step = 1.0f / (float)(S - 1);
  return (s < S / 2) ? step * (float)s : 1.0f - step * (float)(S - 1 - s);
}

template <int P>
__global__ __launch_bounds__(256) void sample_pdf_kernel(const float* __restrict__ t, const float* __restrict__ w,
                                                         int64_t n, int S, int n_imp, const float* __restrict__ u,
                                                         int det, uint64_t seed, float* __restrict__ t_out) {
  __shared__ float s_cdf[4][MAXS];
  __shared__ float s_edge[4][MAXS];
  __shared__ float s_stage[4][64 * P];
  const int wv = threadIdx.x >> 6;
  const int lane = nerf_lane();
  const int64_t r = (int64_t)blockIdx.x * 4 + wv;
  if (r >= n) return;
  const float* tr = t + r * S;
  const float* wr = w + r * S;
  const int B = S - 2;  // interior weights -> bins between the S-1 midpoints
  float* cdf = s_cdf[wv];
  float* edge = s_edge[wv];
  float* stage = s_stage[wv];

  // ---- pdf / cdf.  torch's CPU sum/cumsum accumulate float in double (at::acc_type<float>), so the
  // reduction and the scan run in fp64 and each cdf entry is rounded to fp32 once, like the oracle.
  double totd = 0.0;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int b = b0 + lane;
    totd += (b < B) ? (double)(wr[1 + b] + 1e-5f) : 0.0;
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) totd += __shfl_xor(totd, d, 64);
  const float tot = (float)totd;
  double carry = 0.0;
  if (lane == 0) cdf[0] = 0.f;
  for (int b0 = 0; b0 < B; b0 += 64) {
    const int b = b0 + lane;
    double v = (b < B) ? (double)((wr[1 + b] + 1e-5f) / tot) : 0.0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const double o = __shfl_up(v, d, 64);
      if (lane >= d) v += o;
    }
    v += carry;
    if (b < B) cdf[b + 1] = (float)v;
    carry = __shfl(v, 63, 64);
  }
  for (int j = lane; j < S - 1; j += 64) edge[j] = 0.5f * (tr[j + 1] + tr[j]);
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

  // ---- fine samples -> stage[S + q]; coarse t -> stage[0..S)
  const int NC = S - 1;  // cdf entries
  for (int q = lane; q < n_imp; q += 64) {
    float uu;
    if (u) uu = u[r * n_imp + q];
    else if (det) uu = linspace01(q, n_imp);
    else uu = nerf_uniform(seed, (uint64_t)r, (uint64_t)q + 0x5bd1e995ULL);
    // searchsorted(cdf, u, right=True): first index with cdf[idx] > u
    int lo = 0, hi = NC;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid] <= uu) lo = mid + 1;
      else hi = mid;
    }
    const int below = lo - 1 < 0 ? 0 : lo - 1;
    const int above = lo > NC - 1 ? NC - 1 : lo;
    const float c0 = cdf[below], c1 = cdf[above];
    float den = c1 - c0;
    if (den < 1e-5f) den = 1.0f;
    const float tt = (uu - c0) / den;
    const float e0 = edge[below], e1 = edge[above];
    stage[S + q] = e0 + tt * (e1 - e0);
  }
  for (int j = lane; j < S; j += 64) stage[j] = tr[j];
  const int TOT = S + n_imp;
  for (int j = TOT + lane; j < 64 * P; j += 64) stage[j] = INFINITY;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");

  float v[P];
#pragma unroll
  for (int p = 0; p < P; ++p) v[p] = stage[lane * P + p];

  // ---- bitonic sort of 64*P values, element e = lane*P + p
#pragma unroll
  for (int k = 2; k <= 64 * P; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= P) {
        const int lx = j / P;
#pragma unroll
        for (int p = 0; p < P; ++p) {
          const int e = lane * P + p;
          const float o = __shfl_xor(v[p], lx, 64);
          const bool asc = (e & k) == 0;
          const bool lower = (e & j) == 0;
          v[p] = (asc == lower) ? fminf(v[p], o) : fmaxf(v[p], o);
        }
      } else {
#pragma unroll
        for (int p = 0; p < P; ++p) {
          if ((p & j) == 0) {
            const int q = p | j;
            const int e = lane * P + p;
            const bool asc = (e & k) == 0;
            const float a = v[p], b = v[q];
            v[p] = asc ? fminf(a, b) : fmaxf(a, b);
            v[q] = asc ? fmaxf(a, b) : fminf(a, b);
          }
        }
      }
    }
  }
  float* out = t_out + r * TOT;
#pragma unroll
  for (int p = 0; p < P; ++p) {
    const int e = lane * P + p;
    if (e < TOT) out[e] = v[p];
  }
}

}  // namespace

extern "C" int nerf_sample_pdf(const float* t, const float* w, int64_t n, int S, int n_imp, const float* u, int det,
                               uint64_t seed, float* t_out, hipStream_t stream) {
  NERF_CHECK_ARG(t && w && t_out && n >= 0 && S >= 3 && S <= MAXS && n_imp >= 1 && S + n_imp <= 512);
  if (n == 0) return NERF_OK;
  const int tot = S + n_imp;
  const unsigned blocks = (unsigned)nerf_cdiv(n, 4);
  if (tot <= 64) sample_pdf_kernel<1><<<blocks, 256, 0, stream>>>(t, w, n, S, n_imp, u, det, seed, t_out);
  else if (tot <= 128) sample_pdf_kernel<2><<<blocks, 256, 0, stream>>>(t, w, n, S, n_imp, u, det, seed, t_out);
  else if (tot <= 256) sample_pdf_kernel<4><<<blocks, 256, 0, stream>>>(t, w, n, S, n_imp, u, det, seed, t_out);
  else sample_pdf_kernel<8><<<blocks, 256, 0, stream>>>(t, w, n, S, n_imp, u, det, seed, t_out);
  return nerf_launch_status();
}
