// Alpha-composited volume integration (forward + analytic backward) with the fused MSE loss head.
//
// Restates volume_render (psklavos1/NeRF-Sys adaptive_nerf/nerfs/ray_rendering.py:114-165, called with
// raw_rgb = raw_sigma = False at :336-343):
//   rgb = clamp(rgb,0,1); sigma = clamp_min(sigma,0)*scale; delta_i = clamp_min(t_{i+1}-t_i, 1e-4),
//   last delta = previous delta;  alpha = clamp(1-exp(-sigma delta), 0, 1-1e-7);
//   T = exclusive cumprod(1-alpha+1e-10);  w = alpha T;  rgb_map = sum w rgb (+ (1-acc) bg),
//   depth = sum w t,  acc = sum w.
// and the loss head compute_mse_loss (nerfs/losses.py:10-32) + color_space_transformer
// (nerfs/color_space.py:22-66).
//
// One wave64 per ray; lane l owns samples [l*SPL, l*SPL+SPL) (coalesced float4 (rgb,sigma) loads),
// the transmittance is a wave-wide multiplicative scan, the backward is a division-free affine
// suffix scan:  Q_i = sum_{k>i} e_k alpha_k prod_{i<j<k} f_j,   dL/dalpha_i = T_i (e_i - Q_i),
// with e_k = dL/dw_k and f_j = 1 - alpha_j + 1e-10.  HBM-bound: 20 B/sample in, 4 B/sample weights out.
#include "common.hpp"

namespace {

constexpr float AMAX = (float)(1.0 - 1e-7);

struct SampleState {
  float4 rs;
  float t, delta, e_s;  // e_s = exp(-sigma*delta)
  float x;              // 1 - exp(-sigma delta) before the clamp
  float alpha, f;
};

template <int SPL>
__device__ __forceinline__ void load_ray(const float* __restrict__ rgb_sigma, const float* __restrict__ t, int64_t r,
                                         int S, float sigma_scale, SampleState (&st)[SPL]) {
  const int lane = nerf_lane();
  const float4* rs4 = reinterpret_cast<const float4*>(rgb_sigma) + r * S;
  const float* tr = t + r * S;
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int i = lane * SPL + j;
    const bool v = i < S;
    st[j].rs = v ? rs4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    st[j].t = v ? tr[i] : 0.f;
  }
  // neighbours' t for the interval lengths
  const float t_next_lane = __shfl_down(st[0].t, 1, 64);
  const float t_prev_lane = __shfl_up(st[SPL - 1].t, 1, 64);
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int i = lane * SPL + j;
    const float tn = (j + 1 < SPL) ? st[j + 1 < SPL ? j + 1 : j].t : t_next_lane;
    const float tp = (j > 0) ? st[j > 0 ? j - 1 : 0].t : t_prev_lane;
    float d;
    if (i < S - 1) d = fmaxf(tn - st[j].t, 1e-4f);
    else d = fmaxf(st[j].t - tp, 1e-4f);  // last interval copies the previous one
    st[j].delta = d;
    float sg = fmaxf(st[j].rs.w, 0.f);
    if (sigma_scale != 1.0f) sg = sg * sigma_scale;
    st[j].e_s = expf(-sg * d);
    st[j].x = 1.0f - st[j].e_s;
    const float a = fminf(fmaxf(st[j].x, 0.f), AMAX);
    st[j].alpha = (i < S) ? a : 0.f;
    st[j].f = (i < S) ? (1.0f - a) + 1e-10f : 1.0f;
  }
}

// exclusive transmittance T for each local sample
template <int SPL>
__device__ __forceinline__ void transmittance(const SampleState (&st)[SPL], float (&T)[SPL]) {
  float loc = 1.0f;
#pragma unroll
  for (int j = 0; j < SPL; ++j) loc *= st[j].f;
  const float incl = wave_incl_prod(loc);
  float excl = __shfl_up(incl, 1, 64);
  if (nerf_lane() == 0) excl = 1.0f;
  float run = excl;
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    T[j] = run;
    run *= st[j].f;
  }
}

__device__ __forceinline__ float srgb_to_linear(float x) {
  return x <= 0.04045f ? x / 12.92f : powf((x + 0.055f) / 1.055f, 2.4f);
}

// The loss head's sum: one float atomic per workgroup of FWD_RAYS rays (the per-ray partials meet in LDS first).  With
// one atomic per ray the 4096 same-address atomics of a C2 batch serialised at the L2: 56-61 us per fine / coarse
// launch on MI355X (profiles/r03/prof_fp32_summary.txt) for ~15 MB of data.
constexpr int FWD_RAYS = 16;
template <int SPL>
__global__ __launch_bounds__(64 * FWD_RAYS) void composite_fwd_kernel(const float* __restrict__ rgb_sigma,
                                                            const float* __restrict__ t, const float* __restrict__ bg,
                                                            int64_t n, int S, float sigma_scale,
                                                            float* __restrict__ rgb, float* __restrict__ depth,
                                                            float* __restrict__ weights, float* __restrict__ acc,
                                                            const float* __restrict__ gt, int cs, float inv_count,
                                                            float* __restrict__ loss_sum, float* __restrict__ d_rgb) {
  __shared__ float s_loss[FWD_RAYS];
  const int wv = threadIdx.x >> 6;
  const int64_t r = (int64_t)blockIdx.x * FWD_RAYS + wv;
  const int lane = nerf_lane();
  if (gt && lane == 0) s_loss[wv] = 0.f;
  if (r < n) {
    SampleState st[SPL];
    load_ray<SPL>(rgb_sigma, t, r, S, sigma_scale, st);
    float T[SPL];
    transmittance<SPL>(st, T);
    float cr = 0.f, cg = 0.f, cb = 0.f, dd = 0.f, aa = 0.f;
#pragma unroll
    for (int j = 0; j < SPL; ++j) {
      const int i = lane * SPL + j;
      const float w = st[j].alpha * T[j];
      if (i < S) weights[r * S + i] = w;
      cr += w * fminf(fmaxf(st[j].rs.x, 0.f), 1.f);
      cg += w * fminf(fmaxf(st[j].rs.y, 0.f), 1.f);
      cb += w * fminf(fmaxf(st[j].rs.z, 0.f), 1.f);
      dd += w * st[j].t;
      aa += w;
    }
    cr = wave_sum(cr); cg = wave_sum(cg); cb = wave_sum(cb); dd = wave_sum(dd); aa = wave_sum(aa);
    if (bg) {
      const float k = 1.0f - aa;
      cr = cr + k * bg[3 * r];
      cg = cg + k * bg[3 * r + 1];
      cb = cb + k * bg[3 * r + 2];
    }
    if (lane == 0) {
      rgb[3 * r] = cr; rgb[3 * r + 1] = cg; rgb[3 * r + 2] = cb;
      if (depth) depth[r] = dd;
      if (acc) acc[r] = aa;
    }
    if (gt && lane < 3) {
      const float p = lane == 0 ? cr : (lane == 1 ? cg : cb);
      float g = fminf(fmaxf(gt[3 * r + lane], 0.f), 1.f);
      float pp, dp;
      if (cs == 0) {  // linear: compare clamp(pred) with clamp(srgb_to_linear(gt))
        pp = fminf(fmaxf(p, 0.f), 1.f);
        dp = (p >= 0.f && p <= 1.f) ? 1.f : 0.f;
        g = fminf(fmaxf(srgb_to_linear(g), 0.f), 1.f);
      } else if (cs == 1) {  // srgb: compare clamp(linear_to_srgb(pred)) with gt
        const float xc = fminf(fmaxf(p, 0.f), 1.f);
        const float y = xc <= 0.0031308f ? 12.92f * xc : 1.055f * powf(xc, 1.0f / 2.4f) - 0.055f;
        const float dy = xc <= 0.0031308f ? 12.92f : (1.055f / 2.4f) * powf(xc, 1.0f / 2.4f - 1.0f);
        pp = fminf(fmaxf(y, 0.f), 1.f);
        dp = ((y >= 0.f && y <= 1.f) ? 1.f : 0.f) * ((p >= 0.f && p <= 1.f) ? dy : 0.f);
      } else {  // identity
        pp = p;
        dp = 1.f;
      }
      const float diff = pp - g;
      d_rgb[3 * r + lane] = 2.0f * diff * inv_count * dp;
      float l = diff * diff * inv_count;
      l += __shfl_down(l, 1, 64) + __shfl_down(l, 2, 64);
      if (lane == 0) s_loss[wv] = l;
    }
  }
  if (gt) {  // uniform: every wave reaches the barrier
    __syncthreads();
    if (threadIdx.x == 0) {
      float l = 0.f;
#pragma unroll
      for (int k = 0; k < FWD_RAYS; ++k) l += s_loss[k];
      atomicAdd(loss_sum, l);
    }
  }
}

template <int SPL>
__global__ __launch_bounds__(256) void composite_bwd_kernel(const float* __restrict__ rgb_sigma,
                                                            const float* __restrict__ t, const float* __restrict__ bg,
                                                            int64_t n, int S, float sigma_scale,
                                                            const float* __restrict__ g_rgb,
                                                            const float* __restrict__ g_depth,
                                                            const float* __restrict__ g_acc,
                                                            const float* __restrict__ g_w, float* __restrict__ d_out) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  const int lane = nerf_lane();
  SampleState st[SPL];
  load_ray<SPL>(rgb_sigma, t, r, S, sigma_scale, st);
  float T[SPL];
  transmittance<SPL>(st, T);
  const float gr = g_rgb[3 * r], gg = g_rgb[3 * r + 1], gb = g_rgb[3 * r + 2];
  const float gd = g_depth ? g_depth[r] : 0.f;
  float ga = g_acc ? g_acc[r] : 0.f;
  if (bg) ga -= gr * bg[3 * r] + gg * bg[3 * r + 1] + gb * bg[3 * r + 2];
  float e[SPL], A[SPL];
#pragma unroll
  for (int j = 0; j < SPL; ++j) {
    const int i = lane * SPL + j;
    const float c0 = fminf(fmaxf(st[j].rs.x, 0.f), 1.f), c1 = fminf(fmaxf(st[j].rs.y, 0.f), 1.f),
                c2 = fminf(fmaxf(st[j].rs.z, 0.f), 1.f);
    float ej = gr * c0 + gg * c1 + gb * c2 + gd * st[j].t + ga;
    if (g_w && i < S) ej += g_w[r * S + i];
    e[j] = (i < S) ? ej : 0.f;
    A[j] = e[j] * st[j].alpha;
  }
  // lane segment as an affine map  V_start = Aseg + Bseg * V_after
  float Aseg = 0.f, Bseg = 1.f;
#pragma unroll
  for (int j = SPL - 1; j >= 0; --j) {
    Aseg = A[j] + st[j].f * Aseg;
    Bseg = st[j].f * Bseg;
  }
  // inclusive suffix scan over lanes: (A,B)_l <- (A_l + B_l A_{l+d}, B_l B_{l+d})
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const float oa = __shfl_down(Aseg, d, 64), ob = __shfl_down(Bseg, d, 64);
    if (lane + d < 64) {
      Aseg = Aseg + Bseg * oa;
      Bseg = Bseg * ob;
    }
  }
  float Vnext = __shfl_down(Aseg, 1, 64);
  if (lane == 63) Vnext = 0.f;
  float4* out = reinterpret_cast<float4*>(d_out) + r * S;
#pragma unroll
  for (int j = SPL - 1; j >= 0; --j) {
    const int i = lane * SPL + j;
    const float Q = Vnext;
    Vnext = A[j] + st[j].f * Vnext;
    if (i >= S) continue;
    const float dalpha = T[j] * (e[j] - Q);
    const float x = st[j].x;
    const float dx = (x >= 0.f && x <= AMAX) ? dalpha : 0.f;
    float dsig = dx * st[j].delta * st[j].e_s;
    if (sigma_scale != 1.0f) dsig *= sigma_scale;
    if (!(st[j].rs.w >= 0.f)) dsig = 0.f;
    const float w = st[j].alpha * T[j];
    const float4 c = st[j].rs;
    float4 o;
    o.x = (c.x >= 0.f && c.x <= 1.f) ? w * gr : 0.f;
    o.y = (c.y >= 0.f && c.y <= 1.f) ? w * gg : 0.f;
    o.z = (c.z >= 0.f && c.z <= 1.f) ? w * gb : 0.f;
    o.w = dsig;
    out[i] = o;
  }
}

template <int SPL>
void launch_fwd(const float* rs, const float* t, const float* bg, int64_t n, int S, float sc, float* rgb, float* depth,
                float* w, float* acc, const float* gt, int cs, float ic, float* ls, float* drgb, hipStream_t st) {
  composite_fwd_kernel<SPL><<<(unsigned)nerf_cdiv(n, FWD_RAYS), 64 * FWD_RAYS, 0, st>>>(rs, t, bg, n, S, sc, rgb, depth,
                                                                                      w, acc, gt, cs, ic, ls, drgb);
}
template <int SPL>
void launch_bwd(const float* rs, const float* t, const float* bg, int64_t n, int S, float sc, const float* gr,
                const float* gd, const float* ga, const float* gw, float* d, hipStream_t st) {
  composite_bwd_kernel<SPL><<<(unsigned)nerf_cdiv(n, 4), 256, 0, st>>>(rs, t, bg, n, S, sc, gr, gd, ga, gw, d);
}

int spl_for(int S) {
  const int need = (S + 63) / 64;
  if (need <= 1) return 1;
  if (need <= 2) return 2;
  if (need <= 3) return 3;
  if (need <= 4) return 4;
  if (need <= 8) return 8;
  if (need <= 16) return 16;
  return -1;
}

}  // namespace

extern "C" int nerf_composite_fwd(const float* rgb_sigma, const float* t, const float* bg, int64_t n, int S,
                                  float sigma_scale, float* rgb, float* depth, float* weights, float* acc,
                                  const float* gt, int color_space, float inv_count, float* loss_sum, float* d_rgb,
                                  hipStream_t stream) {
  if (color_space < 0 || color_space > 2) return NERF_E_ENUM;
  NERF_CHECK_ARG(n >= 0 && S >= 2);
  if (n == 0) return NERF_OK;
  NERF_CHECK_ARG(rgb_sigma && t && rgb && weights);
  if (gt) NERF_CHECK_ARG(loss_sum && d_rgb);
  if (!nerf_aligned16(rgb_sigma)) return NERF_E_ALIGN;
  switch (spl_for(S)) {
    case 1: launch_fwd<1>(rgb_sigma, t, bg, n, S, sigma_scale, rgb, depth, weights, acc, gt, color_space, inv_count, loss_sum, d_rgb, stream); break;
    case 2: launch_fwd<2>(rgb_sigma, t, bg, n, S, sigma_scale, rgb, depth, weights, acc, gt, color_space, inv_count, loss_sum, d_rgb, stream); break;
    case 3: launch_fwd<3>(rgb_sigma, t, bg, n, S, sigma_scale, rgb, depth, weights, acc, gt, color_space, inv_count, loss_sum, d_rgb, stream); break;
    case 4: launch_fwd<4>(rgb_sigma, t, bg, n, S, sigma_scale, rgb, depth, weights, acc, gt, color_space, inv_count, loss_sum, d_rgb, stream); break;
    case 8: launch_fwd<8>(rgb_sigma, t, bg, n, S, sigma_scale, rgb, depth, weights, acc, gt, color_space, inv_count, loss_sum, d_rgb, stream); break;
    case 16: launch_fwd<16>(rgb_sigma, t, bg, n, S, sigma_scale, rgb, depth, weights, acc, gt, color_space, inv_count, loss_sum, d_rgb, stream); break;
    default: return NERF_E_ARG;
  }
  return nerf_launch_status();
}

extern "C" int nerf_composite_bwd(const float* rgb_sigma, const float* t, const float* bg, int64_t n, int S,
                                  float sigma_scale, const float* g_rgb, const float* g_depth, const float* g_acc,
                                  const float* g_weights, float* d_rgb_sigma, hipStream_t stream) {
  NERF_CHECK_ARG(n >= 0 && S >= 2);
  if (n == 0) return NERF_OK;
  NERF_CHECK_ARG(rgb_sigma && t && g_rgb && d_rgb_sigma);
  if (!nerf_aligned16(rgb_sigma) || !nerf_aligned16(d_rgb_sigma)) return NERF_E_ALIGN;
  switch (spl_for(S)) {
    case 1: launch_bwd<1>(rgb_sigma, t, bg, n, S, sigma_scale, g_rgb, g_depth, g_acc, g_weights, d_rgb_sigma, stream); break;
    case 2: launch_bwd<2>(rgb_sigma, t, bg, n, S, sigma_scale, g_rgb, g_depth, g_acc, g_weights, d_rgb_sigma, stream); break;
    case 3: launch_bwd<3>(rgb_sigma, t, bg, n, S, sigma_scale, g_rgb, g_depth, g_acc, g_weights, d_rgb_sigma, stream); break;
    case 4: launch_bwd<4>(rgb_sigma, t, bg, n, S, sigma_scale, g_rgb, g_depth, g_acc, g_weights, d_rgb_sigma, stream); break;
    case 8: launch_bwd<8>(rgb_sigma, t, bg, n, S, sigma_scale, g_rgb, g_depth, g_acc, g_weights, d_rgb_sigma, stream); break;
    case 16: launch_bwd<16>(rgb_sigma, t, bg, n, S, sigma_scale, g_rgb, g_depth, g_acc, g_weights, d_rgb_sigma, stream); break;
    default: return NERF_E_ARG;
  }
  return nerf_launch_status();
}
