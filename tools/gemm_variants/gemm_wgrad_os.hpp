// Barrier-free weight-gradient GEMM (fp32 MFMA):  P[s][n][k] = sum_{m in split s} G[m][n] * X[m][k]
// (+ Pb[s][n] = sum_m G[m][n] for the bias), one partial slab per row split s, reduced deterministically
// by reduce_splits_kernel.
//
// Every wave owns a (32 NT_N) x (32 NT_K) output tile and streams its split's rows straight from HBM/L2
// into registers -- no LDS, no barrier: lane l reads row m = 2t + (l >> 5) of the pair t, NT_N consecutive
// G values at column nb + NT_N (l & 31) (one dwordx4 at NT_N = 4) and NT_K consecutive X values at column
// kb + NT_K (l & 31).  Component c of those vectors is the A (resp. B) operand of MFMA tile c, i.e. tile
// (cn, ck) accumulates P[nb + NT_N i + cn][kb + NT_K j + ck] (i, j = the 32x32 row / column) -- a strided
// column set per tile that makes every operand load a single wide, coalesced access.
// The waves of a block cover the whole N x K output for the same rows, so each row is fetched from HBM
// once and served to the other waves from L1/L2.  An R-deep register ring keeps R row pairs in flight.
// Requirement (host wrapper): every split's row count is a multiple of 2 R (rows_per_split and M are).
#pragma once
#include "../../nerf-sys_amd/csrc/gemm.hpp"

template <int N>
struct nerf_fvec;
template <>
struct nerf_fvec<1> { typedef float T; };
template <>
struct nerf_fvec<2> { typedef float T __attribute__((ext_vector_type(2))); };
template <>
struct nerf_fvec<4> { typedef float T __attribute__((ext_vector_type(4))); };

template <int N>
__device__ __forceinline__ float nerf_comp(const typename nerf_fvec<N>::T& v, int c) {
  if constexpr (N == 1) return v;
  else return v[c];
}

template <int NT_N, int NT_K, int R, int MAXW>
__global__ __launch_bounds__(MAXW * 64) void gemm_wgrad_os_kernel(const float* __restrict__ G, int ldg,
                                                                  const float* __restrict__ X, int ldx,
                                                                  float* __restrict__ P, int ldp,
                                                                  float* __restrict__ Pb, int64_t slab,
                                                                  int64_t rows_per_split, int64_t M, int n_kblk) {
  typedef typename nerf_fvec<NT_N>::T GV;
  typedef typename nerf_fvec<NT_K>::T XV;
  const int s = blockIdx.x;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int nblk = wave / n_kblk, kblk = wave - nblk * n_kblk;
  const int nb = nblk * 32 * NT_N, kb = kblk * 32 * NT_K;
  const int lr = lane >> 5, lc = lane & 31;
  const int64_t r0 = (int64_t)s * rows_per_split;
  int64_t r1 = r0 + rows_per_split;
  if (r1 > M) r1 = M;
  const int64_t npairs = r1 > r0 ? (r1 - r0) >> 1 : 0;
  const bool do_bias = (Pb != nullptr) && kblk == 0;

  const float* gp = G + (r0 + lr) * ldg + nb + NT_N * lc;
  const float* xp = X + (r0 + lr) * ldx + kb + NT_K * lc;
  const int64_t gstep = 2 * (int64_t)ldg, xstep = 2 * (int64_t)ldx;

  nerf_f32x16 acc[NT_N][NT_K];
#pragma unroll
  for (int a = 0; a < NT_N; ++a)
#pragma unroll
    for (int b = 0; b < NT_K; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  float bsum[NT_N];
#pragma unroll
  for (int a = 0; a < NT_N; ++a) bsum[a] = 0.f;

  if (npairs > 0) {
    GV gq[R];
    XV xq[R];
    const int64_t last = npairs - 1;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t t = i < last ? i : last;
      gq[i] = *reinterpret_cast<const GV*>(gp + t * gstep);
      xq[i] = *reinterpret_cast<const XV*>(xp + t * xstep);
    }
    for (int64_t t0 = 0; t0 < npairs; t0 += R) {
#pragma unroll
      for (int i = 0; i < R; ++i) {
        const GV g = gq[i];
        const XV x = xq[i];
        // refill this ring slot with pair t0 + R + i (clamped: a harmless re-read past the end)
        int64_t tn = t0 + R + i;
        tn = tn < last ? tn : last;
        gq[i] = *reinterpret_cast<const GV*>(gp + tn * gstep);
        xq[i] = *reinterpret_cast<const XV*>(xp + tn * xstep);
#pragma unroll
        for (int a = 0; a < NT_N; ++a) {
          if (do_bias) bsum[a] += nerf_comp<NT_N>(g, a);
#pragma unroll
          for (int b = 0; b < NT_K; ++b)
            acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(nerf_comp<NT_N>(g, a), nerf_comp<NT_K>(x, b), acc[a][b], 0,
                                                             0, 0);
        }
      }
    }
  }

  float* Ps = P + (int64_t)s * slab;
#pragma unroll
  for (int a = 0; a < NT_N; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int i = (r & 3) + 8 * (r >> 2) + 4 * lr;
      const int n = nb + NT_N * i + a;
      float* row = Ps + (int64_t)n * ldp + kb + NT_K * lc;
      if constexpr (NT_K == 2) {
        *reinterpret_cast<float2*>(row) = make_float2(acc[a][0][r], acc[a][1][r]);
      } else {
#pragma unroll
        for (int b = 0; b < NT_K; ++b) row[b] = acc[a][b][r];
      }
    }
  }
  if (do_bias) {
#pragma unroll
    for (int a = 0; a < NT_N; ++a) {
      const float v = bsum[a] + __shfl_xor(bsum[a], 32, 64);
      if (lr == 0) Pb[(int64_t)s * slab + nb + NT_N * lc + a] = v;
    }
  }
}
