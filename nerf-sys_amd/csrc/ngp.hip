// The Instant-NGP expert on gfx950: multiresolution hash-grid encoding
// (gather / scatter-add), spherical-harmonics direction encoding, and the small MetaNGP MLPs as ONE fused
// kernel per pass (all layers on fp32 MFMA, activations resident in LDS, weights streamed from L2).
//
// Restates (psklavos1/NeRF-Sys adaptive_nerf/):
//   HashGridEncoder ctor / _hash / _gather / _torch_forward   models/encodings.py:175-270, :288-381
//   components_from_spherical_harmonics / SHEncoder.forward   models/encodings.py:27-81, :133-151
//   FrequencyEncoder.torch_forward (dir option)               models/encodings.py:437-444
//   MetaNGP _world_to_unit / density / color / forward        models/inr/meta_ngp.py:166-255 (ctor :21-105)
//   MetaLinear.forward (x W^T + b), trunc_exp                 models/metamodule/metamodule.py:140-156,
//                                                             models/trunc_exp.py:30-61
//
// Fused MLP (nerf_ngp_fwd / nerf_ngp_bwd): a workgroup of 4 waves owns a tile of 64 samples.  Every layer
// is <= 64 wide, so one layer is at most 2x2 blocks of 32x32 (`v_mfma_f32_32x32x2_f32`, exact fp32 fmaf
// chains): wave w computes rows 32*(w&1).., columns 32*(w>>1)...  Activations live in LDS as [64][ld]
// fp32 tiles (ld = width + 4: the 8 k-values a lane reads per 16-k slab are two conflict-free
// ds_read_b128).  Weights (PyTorch (out,in) layout, zero padded to 32) are read straight from L2.
// The backward recomputes the forward into per-layer LDS tiles (no activation round trip through HBM),
// then walks the layers in reverse: weight gradients accumulate in registers across all the tiles a
// persistent workgroup visits (one 32x32 accumulator block per (layer, n-block, k-block), dealt to the 4
// waves), input gradients go tile-to-tile in LDS, d_enc leaves to HBM for the hash-grid scatter.  Each
// workgroup writes ONE slab of the packed gradient; a deterministic reduce sums the slabs.
#include <cstdlib>
#include <mutex>
#include <set>
#include <type_traits>

#include "mlp_common.hpp"

// hipcc contracts a*b-c into one fma by default; the hash-grid math must round every product like the
// reference's torch ops (e.g. frac = x*res - floor(x*res) with x*res rounded first).  The pragma covers this
// file; the Makefile adds -ffp-contract=off for the HIP-header helpers (__fmul_rn, ...) inlined here.
#pragma clang fp contract(off)

typedef float ngp_f32x16 __attribute__((ext_vector_type(16)));
typedef float ngp_f32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int NGP_ROWS = 64;   // forward / density tile (32x32 MFMA blocks)
constexpr int NGP_BROWS = 32;  // backward tile (16x16 MFMA blocks; half the LDS, so two workgroups fit per CU)
constexpr int NGP_MAX_LAYERS = 12;
constexpr int NGP_MAX_SB = 32;

struct NgpLayer {
  int w_off, b_off;  // packed offsets (floats)
  int Kpad, Npad;    // padded to multiples of 32, <= 64
  int relu;          // ReLU on the output
  int in_buf, in_ld; // LDS tile of the input (float offset, row pitch)
  int out_buf, out_ld;
  int in_relu;       // the input is a ReLU output (mask for the input gradient)
};

struct NgpPlan {
  int nl, head, n_trunk, n_color;
  NgpLayer ly[NGP_MAX_LAYERS];
  int enc_buf, enc_ld, in_dim;
  int cin_buf, cin_ld, cin_kpad, geo, dir_mode, sh_levels, dir_dim;
  int sigmoid;
  int g0, g1;            // gradient tiles (ld 68)
  int dsig;              // d sigma_raw per tile row (64 floats; backward plan)
  int sraw;              // sigma_raw per tile row (64 floats; forward plan, -1 in the backward plan)
  int bsum;              // bias-gradient partials [4 waves][nl][64] (backward plan)
  int smem_floats;
  int nsb;               // weight-gradient 32x32 blocks: layer, n-block, k-block
  int sb_layer[NGP_MAX_SB], sb_nb[NGP_MAX_SB], sb_kb[NGP_MAX_SB];
  int64_t total;         // packed floats
};

inline int pad32(int x) { return (x + 31) / 32 * 32; }

// Builds the packed layout and the LDS plan.  save != 0: every layer input keeps its own tile (backward);
// else trunk/colour activations ping-pong.  Returns false for an unsupported configuration.
bool make_plan(const NerfNgpNet& n, bool save, NgpPlan& P) {
  P = NgpPlan{};
  const int dir_dim = n.dir_encoding == 0 ? n.sh_levels * n.sh_levels : 27;
  if (n.in_dim < 1 || n.in_dim > 64 || n.hidden < 1 || n.hidden > 64 || n.color_hidden < 1 || n.color_hidden > 64)
    return false;
  if (n.geo_feat_dim < 0 || n.geo_feat_dim + 1 > 32 || n.sigma_depth < 0 || n.color_depth < 0) return false;
  if (n.dir_encoding == 0 && (n.sh_levels < 1 || n.sh_levels > 5)) return false;
  if (n.dir_encoding != 0 && n.dir_encoding != 1) return false;
  if (n.geo_feat_dim + dir_dim > 64) return false;
  if (n.generic_kernels != 0 && n.generic_kernels != 1) return false;
  P.nl = n.sigma_depth + n.color_depth + 2;
  if (P.nl > NGP_MAX_LAYERS) return false;
  P.n_trunk = n.sigma_depth;
  P.n_color = n.color_depth;
  P.head = n.sigma_depth;
  P.in_dim = n.in_dim;
  P.geo = n.geo_feat_dim;
  P.dir_mode = n.dir_encoding;
  P.sh_levels = n.sh_levels;
  P.dir_dim = dir_dim;
  P.sigmoid = n.use_sigmoid_rgb;
  P.cin_kpad = pad32(n.geo_feat_dim + dir_dim);
  // packed layout
  int64_t o = 0;
  int last = n.in_dim;
  for (int l = 0; l < P.nl; ++l) {
    NgpLayer& L = P.ly[l];
    int N, K;
    if (l < P.head) { N = n.hidden; K = last; L.relu = 1; }
    else if (l == P.head) { N = 1 + n.geo_feat_dim; K = last; L.relu = 0; }
    else if (l < P.nl - 1) { N = n.color_hidden; K = (l == P.head + 1) ? n.geo_feat_dim + dir_dim : last; L.relu = 1; }
    else { N = 3; K = (l == P.head + 1) ? n.geo_feat_dim + dir_dim : last; L.relu = 0; }
    L.Npad = pad32(N);
    L.Kpad = pad32(K);
    L.w_off = (int)o; o += (int64_t)L.Npad * L.Kpad;
    L.b_off = (int)o; o += L.Npad;
    if (l < P.head) last = n.hidden;
    else if (l > P.head) last = n.color_hidden;
    L.in_relu = (l > 0 && l != P.head + 1 && P.ly[l - 1].relu) ? 1 : 0;
  }
  P.total = o;
  // LDS plan (floats)
  int s = 0;
  const int rows = save ? NGP_BROWS : NGP_ROWS;
  auto take = [&](int ld) { int b = s; s += rows * ld; return b; };
  P.enc_ld = pad32(n.in_dim) + 4;
  P.enc_buf = take(P.enc_ld);
  P.cin_ld = P.cin_kpad + 4;
  P.cin_buf = take(P.cin_ld);
  // backward plan: two gradient tiles (g0 also holds the raw head output, g1 the rgb logits) and d sigma_raw.
  // forward plan: activations ping-pong through two tiles (the head output too; its sigma_raw column is copied
  // to sraw before the colour layers overwrite it), which halves the LDS of a workgroup so two fit per CU.
  int pp[2] = {-1, -1};
  if (save) {
    P.g0 = take(68);
    P.g1 = take(68);
    P.dsig = s; s += NGP_BROWS;
    P.sraw = -1;
    P.bsum = -1;
  } else {
    pp[0] = take(68);
    pp[1] = take(68);
    P.g0 = P.g1 = P.dsig = P.bsum = -1;
    P.sraw = s; s += NGP_ROWS;
  }
  int prev_out = P.enc_buf, prev_ld = P.enc_ld;
  for (int l = 0; l < P.nl; ++l) {
    NgpLayer& L = P.ly[l];
    if (l == P.head + 1) { prev_out = P.cin_buf; prev_ld = P.cin_ld; }
    L.in_buf = prev_out;
    L.in_ld = prev_ld;
    if (!save) { L.out_buf = pp[l & 1]; L.out_ld = 68; }
    else if (l == P.head) { L.out_buf = P.g0; L.out_ld = 68; }           // raw [sigma, geo]: aliases a grad tile
    else if (l == P.nl - 1) { L.out_buf = P.g1; L.out_ld = 68; }    // raw rgb logits
    else { L.out_buf = take(L.Npad + 4); L.out_ld = L.Npad + 4; }
    prev_out = L.out_buf;
    prev_ld = L.out_ld;
  }
  // bias-gradient partials last, only when two workgroups still fit per CU (deep nets: one wave per layer sums all
  // rows in registers)
  if (save && (int64_t)(s + 4 * P.nl * 64) * 4 <= 80 * 1024) { P.bsum = s; s += 4 * P.nl * 64; }
  P.smem_floats = s;
  if ((int64_t)s * 4 > 160 * 1024) return false;
  // weight-gradient blocks (32x32, 16 MFMAs of 64 cycles per 32-row tile), dealt to the 4 waves: slot sb = wave + 4 j.
  // A layer's wgrad blocks run in the same barrier interval as its input-gradient MFMAs (16x16 blocks: every wave
  // owns Kpad / 32 of them, Npad / 4 MFMAs of 32 cycles each), so each block goes to the wave with the least work in
  // that interval (then the fewest slots used).  Costs in units of 32 cycles.
  int nblk = 0;
  for (int l = 0; l < P.nl; ++l) nblk += (P.ly[l].Npad / 32) * (P.ly[l].Kpad / 32);
  const int per_wave = (nblk + 3) / 4;
  if (4 * per_wave > NGP_MAX_SB) return false;
  int used[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4 * per_wave; ++i) P.sb_layer[i] = -1;
  for (int l = 0; l < P.nl; ++l) {
    const NgpLayer& L = P.ly[l];
    int cost[4];
    for (int w = 0; w < 4; ++w) cost[w] = (L.Kpad / 32) * (L.Npad / 4);
    for (int nb = 0; nb < L.Npad / 32; ++nb)
      for (int kb = 0; kb < L.Kpad / 32; ++kb) {
        int best = -1;
        for (int w = 0; w < 4; ++w) {
          if (used[w] >= per_wave) continue;
          if (best < 0 || cost[w] < cost[best] || (cost[w] == cost[best] && used[w] < used[best])) best = w;
        }
        const int sb = best + 4 * used[best];
        P.sb_layer[sb] = l; P.sb_nb[sb] = nb; P.sb_kb[sb] = kb;
        ++used[best];
        cost[best] += 32;  // 16 MFMAs x 64 cycles
      }
  }
  P.nsb = 4 * per_wave;
  return true;
}

// ---------------------------------------------------------------------------------------- hash grid

struct HashArgs {
  int L, F, log2T, interp;
  int res[NERF_HASH_MAX_LEVELS];
  float mn[3], inv_unused[3], ext[3];
  int has_aabb;
  float eps;
};

__device__ __forceinline__ uint32_t ngp_hash(int ix, int iy, int iz, uint32_t mask) {
  // (ix*1 ^ iy*2654435761 ^ iz*805459861) mod 2^log2T — the low bits of the reference's int64 products
  return ((uint32_t)ix ^ ((uint32_t)iy * 2654435761u) ^ ((uint32_t)iz * 805459861u)) & mask;
}

__device__ __forceinline__ void load_x01(const HashArgs& a, const float* __restrict__ x, int64_t xs, int64_t m,
                                         float p[3]) {
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float v = x[m * xs + c];
    if (a.has_aabb) {
      v = __fdiv_rn(__fsub_rn(v, a.mn[c]), a.ext[c]);
      v = fminf(fmaxf(v, a.eps), 1.0f - a.eps);
    }
    p[c] = v;
  }
}

// corner weights in the reference's autograd product order: ((g*(1-wz))*(1-wy))*(1-wx) etc.  For the
// forward the blend is c00 = f000*(1-wx) + f100*wx, ... (no fma contraction: bit-exact with torch).
// the F features of one level at unit-cube point p (shared by hash_fwd_kernel and the fused density kernel)
template <int F>
__device__ __forceinline__ void hash_level(const HashArgs& a, const float* __restrict__ table, const float p[3], int l,
                                           float acc[F]) {
  const float r = (float)a.res[l];
  const uint32_t mask = (1u << a.log2T) - 1u;
  const float* tb = table + ((int64_t)l << a.log2T) * F;
  if (a.interp == 0) {  // Nearest: torch.round = round half to even
    const int ix = (int)rintf(__fmul_rn(p[0], r)), iy = (int)rintf(__fmul_rn(p[1], r)), iz = (int)rintf(__fmul_rn(p[2], r));
    const float* e = tb + (int64_t)ngp_hash(ix, iy, iz, mask) * F;
#pragma unroll
    for (int f = 0; f < F; ++f) acc[f] = e[f];
  } else {
    float s[3], w[3];
    int i0[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      s[c] = __fmul_rn(p[c], r);
      const float fl = floorf(s[c]);
      w[c] = __fsub_rn(s[c], fl);
      i0[c] = (int)fl;
      if (a.interp == 2) w[c] = __fmul_rn(__fmul_rn(w[c], w[c]), __fsub_rn(3.0f, __fmul_rn(2.0f, w[c])));
    }
    float f[8][F];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // k bits: x = 4, y = 2, z = 1
      const float* e = tb + (int64_t)ngp_hash(i0[0] + ((k >> 2) & 1), i0[1] + ((k >> 1) & 1), i0[2] + (k & 1), mask) * F;
      if (F == 2) {
        const float2 v = *reinterpret_cast<const float2*>(e);
        f[k][0] = v.x;
        f[k][F > 1 ? 1 : 0] = v.y;
      } else if (F == 4) {
        const float4 v = *reinterpret_cast<const float4*>(e);
        f[k][0] = v.x; f[k][F > 1 ? 1 : 0] = v.y; f[k][F > 2 ? 2 : 0] = v.z; f[k][F > 3 ? 3 : 0] = v.w;
      } else {
#pragma unroll
        for (int q = 0; q < F; ++q) f[k][q] = e[q];
      }
    }
    const float ux = __fsub_rn(1.0f, w[0]), uy = __fsub_rn(1.0f, w[1]), uz = __fsub_rn(1.0f, w[2]);
#pragma unroll
    for (int q = 0; q < F; ++q) {
      // k index: (dx, dy, dz) -> 4dx + 2dy + dz ; c_yz = f[0yz]*(1-wx) + f[1yz]*wx
      const float c00 = __fadd_rn(__fmul_rn(f[0][q], ux), __fmul_rn(f[4][q], w[0]));
      const float c01 = __fadd_rn(__fmul_rn(f[1][q], ux), __fmul_rn(f[5][q], w[0]));
      const float c10 = __fadd_rn(__fmul_rn(f[2][q], ux), __fmul_rn(f[6][q], w[0]));
      const float c11 = __fadd_rn(__fmul_rn(f[3][q], ux), __fmul_rn(f[7][q], w[0]));
      const float c0 = __fadd_rn(__fmul_rn(c00, uy), __fmul_rn(c10, w[1]));
      const float c1 = __fadd_rn(__fmul_rn(c01, uy), __fmul_rn(c11, w[1]));
      acc[q] = __fadd_rn(__fmul_rn(c0, uz), __fmul_rn(c1, w[2]));
    }
  }
}

template <int F>
__global__ void hash_fwd_kernel(HashArgs a, const float* __restrict__ table, const float* __restrict__ x, int64_t xs,
                                int64_t M, float* __restrict__ out, int os) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = gid / a.L;
  const int l = (int)(gid - m * a.L);
  if (m >= M) return;
  float p[3];
  load_x01(a, x, xs, m, p);
  float acc[F];
  hash_level<F>(a, table, p, l, acc);
  float* o = out + m * os + l * F;
  if (F == 2) {
    *reinterpret_cast<float2*>(o) = make_float2(acc[0], acc[F > 1 ? 1 : 0]);
  } else {
#pragma unroll
    for (int q = 0; q < F; ++q) o[q] = acc[q];
  }
  // zero the row's pad columns [L*F, os): spread over the row's L threads
  for (int c = a.L * F + l; c < os; c += a.L) out[m * os + c] = 0.f;
}

template <int F>
__global__ void hash_bwd_kernel(HashArgs a, const float* __restrict__ x, int64_t xs, int64_t M,
                                const float* __restrict__ g, int gs, float* __restrict__ dtab) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = gid / a.L;
  const int l = (int)(gid - m * a.L);
  if (m >= M) return;
  float p[3];
  load_x01(a, x, xs, m, p);
  const float r = (float)a.res[l];
  const uint32_t mask = (1u << a.log2T) - 1u;
  float* tb = dtab + ((int64_t)l << a.log2T) * F;
  float gg[F];
#pragma unroll
  for (int q = 0; q < F; ++q) gg[q] = g[m * gs + l * F + q];
  if (a.interp == 0) {
    const int ix = (int)rintf(__fmul_rn(p[0], r)), iy = (int)rintf(__fmul_rn(p[1], r)), iz = (int)rintf(__fmul_rn(p[2], r));
    float* e = tb + (int64_t)ngp_hash(ix, iy, iz, mask) * F;
#pragma unroll
    for (int q = 0; q < F; ++q) unsafeAtomicAdd(e + q, gg[q]);
    return;
  }
  float w[3];
  int i0[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float s = __fmul_rn(p[c], r);
    const float fl = floorf(s);
    w[c] = __fsub_rn(s, fl);
    i0[c] = (int)fl;
    if (a.interp == 2) w[c] = __fmul_rn(__fmul_rn(w[c], w[c]), __fsub_rn(3.0f, __fmul_rn(2.0f, w[c])));
  }
  const float u[3] = {__fsub_rn(1.0f, w[0]), __fsub_rn(1.0f, w[1]), __fsub_rn(1.0f, w[2])};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int dx = (k >> 2) & 1, dy = (k >> 1) & 1, dz = k & 1;
    float* e = tb + (int64_t)ngp_hash(i0[0] + dx, i0[1] + dy, i0[2] + dz, mask) * F;
#pragma unroll
    for (int q = 0; q < F; ++q) {
      const float v = __fmul_rn(__fmul_rn(__fmul_rn(gg[q], dz ? w[2] : u[2]), dy ? w[1] : u[1]), dx ? w[0] : u[0]);
      unsafeAtomicAdd(e + q, v);
    }
  }
}

// F = 2 backward, shaped for the memory-side atomic unit: float atomics execute at the memory side at one
// rate of 64-B requests chip-wide (MI355X_MICROARCH.md § Global float atomics), so a wave-instruction whose
// 64 lanes hit 64 scattered entries costs 16x one that hits 4 segments.  Four lanes cooperate on one
// (sample, level): lane q adds feature f = q & 1 of the x-corner dx = q >> 1 for each of the four (y,z)
// corners.  With the reference's x-prime of 1 the two x-corners hash to h and h ^ (ix ^ (ix+1)), the same
// 64-B segment 7 times in 8, so each instruction carries ~16 requests instead of 64.
__global__ void hash_bwd_f2_kernel(HashArgs a, const float* __restrict__ x, int64_t xs, int64_t M,
                                   const float* __restrict__ g, int gs, float* __restrict__ dtab) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int q = (int)(gid & 3);
  const int64_t pair = gid >> 2;
  const int64_t m = pair / a.L;
  const int l = (int)(pair - m * a.L);
  if (m >= M) return;
  float p[3];
  load_x01(a, x, xs, m, p);
  const float r = (float)a.res[l];
  const uint32_t mask = (1u << a.log2T) - 1u;
  float* tb = dtab + ((int64_t)l << a.log2T) * 2;
  const int dx = q >> 1, f = q & 1;
  const float gg = g[m * gs + l * 2 + f];
  if (a.interp == 0) {
    if (dx == 0) {
      const int ix = (int)rintf(__fmul_rn(p[0], r)), iy = (int)rintf(__fmul_rn(p[1], r)),
                iz = (int)rintf(__fmul_rn(p[2], r));
      unsafeAtomicAdd(tb + (int64_t)ngp_hash(ix, iy, iz, mask) * 2 + f, gg);
    }
    return;
  }
  float w[3];
  int i0[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float s = __fmul_rn(p[c], r);
    const float fl = floorf(s);
    w[c] = __fsub_rn(s, fl);
    i0[c] = (int)fl;
    if (a.interp == 2) w[c] = __fmul_rn(__fmul_rn(w[c], w[c]), __fsub_rn(3.0f, __fmul_rn(2.0f, w[c])));
  }
  const float u[3] = {__fsub_rn(1.0f, w[0]), __fsub_rn(1.0f, w[1]), __fsub_rn(1.0f, w[2])};
  const float wx = dx ? w[0] : u[0];
#pragma unroll
  for (int yz = 0; yz < 4; ++yz) {
    const int dy = yz >> 1, dz = yz & 1;
    const float v = __fmul_rn(__fmul_rn(__fmul_rn(gg, dz ? w[2] : u[2]), dy ? w[1] : u[1]), wx);
    unsafeAtomicAdd(tb + (int64_t)ngp_hash(i0[0] + dx, i0[1] + dy, i0[2] + dz, mask) * 2 + f, v);
  }
}

// F = 2 with run aggregation.  Lanes: q = lane & 3 (feature q & 1, x-corner q >> 1), sample m = global lane / 4,
// so a wave holds 16 consecutive samples — consecutive samples of one ray in the packed (ray-major, t-sorted)
// order.  Each thread walks the L levels; at coarse levels neighbouring samples share cells, so before every
// atomic the lanes of one (feature, x-corner) sub-sequence holding the same table entry are summed with a
// segmented suffix scan (runs of equal index) and only the run head issues the atomic: the atomic count drops
// where samples per cell > 1 (levels with res * step < 1), the result is the same sum in another order.
__global__ __launch_bounds__(256) void hash_bwd_f2_agg_kernel(HashArgs a, const float* __restrict__ x, int64_t xs,
                                                              int64_t M, const float* __restrict__ g, int gs,
                                                              float* __restrict__ dtab) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int q = lane & 3, grp = lane >> 2;
  const int64_t m = gid >> 2;
  const bool valid = m < M;
  if (__ballot(valid) == 0) return;
  float p[3] = {0.f, 0.f, 0.f};
  if (valid) load_x01(a, x, xs, m, p);
  const uint32_t mask = (1u << a.log2T) - 1u;
  const int dx = q >> 1, f = q & 1;
  const unsigned long long qmask = 0x1111111111111111ull << q;
  const unsigned long long after = lane == 63 ? 0ull : ~((2ull << lane) - 1ull);
  for (int l = 0; l < a.L; ++l) {
    const float r = (float)a.res[l];
    float w[3];
    int i0[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float sc = __fmul_rn(p[c], r);
      const float fl = floorf(sc);
      w[c] = __fsub_rn(sc, fl);
      i0[c] = (int)fl;
      if (a.interp == 2) w[c] = __fmul_rn(__fmul_rn(w[c], w[c]), __fsub_rn(3.0f, __fmul_rn(2.0f, w[c])));
    }
    const float u[3] = {__fsub_rn(1.0f, w[0]), __fsub_rn(1.0f, w[1]), __fsub_rn(1.0f, w[2])};
    const float wx = dx ? w[0] : u[0];
    const float gg = valid ? g[m * gs + l * 2 + f] : 0.f;
    float* tb = dtab + ((int64_t)l << a.log2T) * 2;
#pragma unroll
    for (int yz = 0; yz < 4; ++yz) {
      const int dy = yz >> 1, dz = yz & 1;
      const float v = __fmul_rn(__fmul_rn(__fmul_rn(gg, dz ? w[2] : u[2]), dy ? w[1] : u[1]), wx);
      const uint32_t idx = valid ? ngp_hash(i0[0] + dx, i0[1] + dy, i0[2] + dz, mask) * 2u + (uint32_t)f
                                 : 0xFFFFFFFFu;
      const uint32_t prev = __shfl_up(idx, 4, 64);
      const bool head = grp == 0 || prev != idx;
      const unsigned long long nxt = __ballot(head) & qmask & after;  // heads after me in my sub-sequence
      const int run_end = nxt ? (int)__builtin_ctzll(nxt) - 4 : 60 + q;
      float sum = v;
#pragma unroll
      for (int off = 4; off < 64; off <<= 1) {
        const float o = __shfl_down(sum, off, 64);
        if (lane + off <= run_end) sum += o;
      }
      if (head && valid) unsafeAtomicAdd(tb + idx, sum);
    }
  }
}

// ---------------------------------------------------------------------------------------- direction encodings

// SH components of degree `deg` of a unit direction into v[0..(deg+1)^2) (models/encodings.py:27-81; the
// products are evaluated left to right as torch does).
__device__ __forceinline__ void sh_eval(int deg, float x, float y, float z, float* v) {
  const float xx = x * x, yy = y * y, zz = z * z;
  v[0] = 0.28209479177387814f;
  if (deg > 0) {
    v[1] = 0.4886025119029199f * y;
    v[2] = 0.4886025119029199f * z;
    v[3] = 0.4886025119029199f * x;
  }
  if (deg > 1) {
    v[4] = __fmul_rn(1.0925484305920792f * x, y);
    v[5] = __fmul_rn(1.0925484305920792f * y, z);
    v[6] = __fsub_rn(__fmul_rn(0.9461746957575601f, zz), 0.31539156525251999f);
    v[7] = __fmul_rn(1.0925484305920792f * x, z);
    v[8] = __fmul_rn(0.5462742152960396f, __fsub_rn(xx, yy));
  }
  if (deg > 2) {
    v[9] = __fmul_rn(0.5900435899266435f * y, __fsub_rn(3.0f * xx, yy));
    v[10] = __fmul_rn(__fmul_rn(2.890611442640554f * x, y), z);
    v[11] = __fmul_rn(0.4570457994644658f * y, __fsub_rn(5.0f * zz, 1.0f));
    v[12] = __fmul_rn(0.3731763325901154f * z, __fsub_rn(5.0f * zz, 3.0f));
    v[13] = __fmul_rn(0.4570457994644658f * x, __fsub_rn(5.0f * zz, 1.0f));
    v[14] = __fmul_rn(1.445305721320277f * z, __fsub_rn(xx, yy));
    v[15] = __fmul_rn(0.5900435899266435f * x, __fsub_rn(xx, 3.0f * yy));
  }
  if (deg > 3) {
    v[16] = __fmul_rn(__fmul_rn(2.5033429417967046f * x, y), __fsub_rn(xx, yy));
    v[17] = __fmul_rn(__fmul_rn(1.7701307697799304f * y, z), __fsub_rn(3.0f * xx, yy));
    v[18] = __fmul_rn(__fmul_rn(0.9461746957575601f * x, y), __fsub_rn(7.0f * zz, 1.0f));
    v[19] = __fmul_rn(__fmul_rn(0.6690465435572892f * y, z), __fsub_rn(7.0f * zz, 3.0f));
    v[20] = __fmul_rn(0.10578554691520431f, __fadd_rn(__fsub_rn(__fmul_rn(35.0f * zz, zz), 30.0f * zz), 3.0f));
    v[21] = __fmul_rn(__fmul_rn(0.6690465435572892f * x, z), __fsub_rn(7.0f * zz, 3.0f));
    v[22] = __fmul_rn(__fmul_rn(0.47308734787878004f, __fsub_rn(xx, yy)), __fsub_rn(7.0f * zz, 1.0f));
    v[23] = __fmul_rn(__fmul_rn(1.7701307697799304f * x, z), __fsub_rn(xx, 3.0f * yy));
    v[24] = __fmul_rn(0.6258357354491761f,
                      __fsub_rn(__fmul_rn(xx, __fsub_rn(xx, 3.0f * yy)), __fmul_rn(yy, __fsub_rn(3.0f * xx, yy))));
  }
}

// d / max(|d|, eps) with |d| = sqrt(x^2 + y^2 + z^2)
__device__ __forceinline__ void unit3(float& x, float& y, float& z, float eps) {
  const float n = fmaxf(__fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(x, x), __fmul_rn(y, y)), __fmul_rn(z, z))), eps);
  x = __fdiv_rn(x, n);
  y = __fdiv_rn(y, n);
  z = __fdiv_rn(z, n);
}

__global__ void sh_kernel(const float* __restrict__ d, int64_t ds, int64_t M, int levels, float* __restrict__ out,
                          int os) {
  const int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= M) return;
  float x = d[m * ds], y = d[m * ds + 1], z = d[m * ds + 2];
  unit3(x, y, z, 1e-9f);
  float v[25];
  sh_eval(levels - 1, x, y, z, v);
  const int nc = levels * levels;
  for (int c = 0; c < os; ++c) out[m * os + c] = c < nc ? v[c] : 0.f;
}

// ---------------------------------------------------------------------------------------- fused MLP

__device__ __forceinline__ ngp_f32x16 zero16() {
  ngp_f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// Y = act(X W^T + b) for one 64-row tile.  Lane li of wave (rb, cb) owns row rb*32+li; register 4q+e of its
// accumulator is column cb*32 + 8q + 4lh + e (C^T tile: the weight is the MFMA's A operand).
__device__ __forceinline__ void layer_fwd(const NgpLayer& L, float* smem, const float* __restrict__ w, int wave,
                                          int li, int lh) {
  const int rb = wave & 1, cb = wave >> 1;
  if (cb * 32 >= L.Npad) return;
  const float* X = smem + L.in_buf + (rb * 32 + li) * L.in_ld + 8 * lh;
  const float* Wr = w + L.w_off + (int64_t)(cb * 32 + li) * L.Kpad + 8 * lh;
  ngp_f32x16 acc = zero16();
  const int ns = L.Kpad / 16;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s < ns) {
      const float4 w0 = *reinterpret_cast<const float4*>(Wr + 16 * s);
      const float4 w1 = *reinterpret_cast<const float4*>(Wr + 16 * s + 4);
      const float4 x0 = *reinterpret_cast<const float4*>(X + 16 * s);
      const float4 x1 = *reinterpret_cast<const float4*>(X + 16 * s + 4);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w0.x, x0.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w0.y, x0.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w0.z, x0.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w0.w, x0.w, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1.x, x1.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1.y, x1.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1.z, x1.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(w1.w, x1.w, acc, 0, 0, 0);
    }
  }
  float* Y = smem + L.out_buf + (rb * 32 + li) * L.out_ld + cb * 32 + 4 * lh;
  const float* bias = w + L.b_off + cb * 32 + 4 * lh;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 b = *reinterpret_cast<const float4*>(bias + 8 * q);
    float v0 = acc[4 * q] + b.x, v1 = acc[4 * q + 1] + b.y, v2 = acc[4 * q + 2] + b.z, v3 = acc[4 * q + 3] + b.w;
    if (L.relu) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
    *reinterpret_cast<float4*>(Y + 8 * q) = make_float4(v0, v1, v2, v3);
  }
}

// enc tile (rows >= M and pad columns zero)
__device__ __forceinline__ void load_enc(const NgpPlan& P, float* smem, const float* __restrict__ enc, int es,
                                         int64_t m0, int64_t M) {
  const int kp = P.enc_ld - 4;
  for (int i = threadIdx.x; i < NGP_ROWS * kp; i += blockDim.x) {
    const int r = i / kp, c = i - r * kp;
    const int64_t m = m0 + r;
    smem[P.enc_buf + r * P.enc_ld + c] = (m < M && c < P.in_dim) ? enc[m * es + c] : 0.f;
  }
}

// direction encoding of one row into v[0..dir_dim): MetaNGP._enc_dir (meta_ngp.py:176-179) then SHEncoder.forward
// (encodings.py:133-151, normalises again) or the dir FrequencyEncoder (encodings.py:437-444)
__device__ __forceinline__ void dir_encode(const NgpPlan& P, float x, float y, float z, float v[27]) {
  unit3(x, y, z, 1e-9f);
  if (P.dir_mode == 0) {
    unit3(x, y, z, 1e-9f);
    sh_eval(P.sh_levels - 1, x, y, z, v);
  } else {
    const float d[3] = {x, y, z};
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      v[k] = d[k];
      float band = 1.0f;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        float s, cc;
        sincosf(d[k] * band, &s, &cc);
        v[3 + k * 8 + l] = cc;
        v[3 + k * 8 + 4 + l] = s;
        band *= 2.0f;
      }
    }
  }
}

// cin = [geo (head cols 1..geo) | dir encoding | 0] for row r (one thread per row)
__device__ __forceinline__ void build_cin_row(const NgpPlan& P, float* smem, const float* __restrict__ x_d, int64_t m,
                                              int64_t M, int r) {
  float* c = smem + P.cin_buf + r * P.cin_ld;
  const float* h = smem + P.ly[P.head].out_buf + r * P.ly[P.head].out_ld;
  if (P.sraw >= 0) smem[P.sraw + r] = h[0];
  for (int k = 0; k < P.geo; ++k) c[k] = h[1 + k];
  float v[27];
  float x = 0.f, y = 0.f, z = 1.f;
  if (m < M) { x = x_d[m * 6 + 3]; y = x_d[m * 6 + 4]; z = x_d[m * 6 + 5]; }
  dir_encode(P, x, y, z, v);
  for (int k = 0; k < P.dir_dim; ++k) c[P.geo + k] = v[k];
  for (int k = P.geo + P.dir_dim; k < P.cin_kpad; ++k) c[k] = 0.f;
}

__device__ __forceinline__ void forward_tile(const NgpPlan& P, float* smem, const float* __restrict__ w,
                                             const float* __restrict__ enc, int es, const float* __restrict__ x_d,
                                             int64_t m0, int64_t M, int wave, int li, int lh) {
  load_enc(P, smem, enc, es, m0, M);
  __syncthreads();
  for (int l = 0; l <= P.head; ++l) {
    layer_fwd(P.ly[l], smem, w, wave, li, lh);
    __syncthreads();
  }
  if (threadIdx.x < NGP_ROWS) build_cin_row(P, smem, x_d, m0 + threadIdx.x, M, threadIdx.x);
  __syncthreads();
  for (int l = P.head + 1; l < P.nl; ++l) {
    layer_fwd(P.ly[l], smem, w, wave, li, lh);
    __syncthreads();
  }
}

__global__ __launch_bounds__(256) void ngp_fwd_kernel(NgpPlan P, const float* __restrict__ w,
                                                      const float* __restrict__ enc, int es,
                                                      const float* __restrict__ x_d, int64_t M,
                                                      float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * NGP_ROWS;
  forward_tile(P, smem, w, enc, es, x_d, m0, M, wave, li, lh);
  if (threadIdx.x < NGP_ROWS) {
    const int r = threadIdx.x;
    const int64_t m = m0 + r;
    if (m < M) {
      const float* o = smem + P.ly[P.nl - 1].out_buf + r * P.ly[P.nl - 1].out_ld;
      const float sr = P.sraw >= 0 ? smem[P.sraw + r] : smem[P.ly[P.head].out_buf + r * P.ly[P.head].out_ld];
      float c0 = o[0], c1 = o[1], c2 = o[2];
      if (P.sigmoid) { c0 = nerf_mlp::sigmoidf_(c0); c1 = nerf_mlp::sigmoidf_(c1); c2 = nerf_mlp::sigmoidf_(c2); }
      const float sg = expf(fminf(fmaxf(sr, -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
      reinterpret_cast<float4*>(out)[m] = make_float4(c0, c1, c2, sg);
    }
  }
}

// MetaNGP.density (meta_ngp.py:192-224): the sigma trunk and head only — sigma = trunc_exp(raw) per row; the
// colour branch (direction encoding + colour MLP, about half the network) is skipped.  Used by the visibility
// filter of the occupancy marcher and the occupancy-grid update, which need sigma only.
__global__ __launch_bounds__(256) void ngp_density_kernel(NgpPlan P, const float* __restrict__ w,
                                                          const float* __restrict__ enc, int es, int64_t M,
                                                          float* __restrict__ sigma) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * NGP_ROWS;
  load_enc(P, smem, enc, es, m0, M);
  __syncthreads();
  for (int l = 0; l <= P.head; ++l) {
    layer_fwd(P.ly[l], smem, w, wave, li, lh);
    __syncthreads();
  }
  if (threadIdx.x < NGP_ROWS) {
    const int64_t m = m0 + threadIdx.x;
    if (m < M) {
      const float sr = smem[P.ly[P.head].out_buf + threadIdx.x * P.ly[P.head].out_ld];
      sigma[m] = expf(fminf(fmaxf(sr, -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
    }
  }
}

// ---- backward: 32-row tiles, 16x16x4 f32 MFMA blocks for the recomputed forward and the input gradients, 32x32x2
// blocks for the weight gradients.  Two workgroups share a CU (LDS ~68 KB each), so one workgroup's barrier and L2
// waits hide behind the other's MFMAs.  A wave's weight operands of the NEXT layer step are loaded into registers
// while the current step computes (the fragment stream of a tile: forward layers 0..nl-1, then input-gradient
// layers nl-1..0, wrapping to the next tile), and the barriers are plain s_barriers behind an LDS wait, so the
// prefetch stays in flight across them.

// one wave's weight operands for one step: a[j] = 4 k-values of its 16-row A fragment for k-slab j (16 k), b = bias
struct NgpFrag {
  float4 a[4];
  float4 b;
};

// 16x16 blocks of a [32 x N] output (N = 32 or 64): wave w owns column block w (both row blocks) when N = 64, else
// the block (column w & 1, row w >> 1).
__device__ __forceinline__ void blk16(int N, int wave, int& cb, int& rb0, int& nrb) {
  if (N == 64) { cb = wave; rb0 = 0; nrb = 2; }
  else { cb = wave & 1; rb0 = wave >> 1; nrb = 1; }
}

// Step i < nl: forward of layer i, A = W rows (n = 16 cb + c16), k = 16 j + 4 g + e.  Step i >= nl: input gradient
// of layer 2 nl - 1 - i, A = W^T rows (k = 16 kb + c16) of the transposed image wt, n = 16 j + 4 g + e.  Both are
// five unconditional float4 loads (slabs past the layer's width re-read slab 0; the input-gradient step re-reads a
// bias it ignores): with a fixed count the compiler waits for the current fragment with vmcnt(5), not vmcnt(0).
__device__ __forceinline__ void load_frag(const NgpPlan& P, const float* __restrict__ w, const float* __restrict__ wt,
                                          int i, int wave, int lane, NgpFrag& f) {
  const int g = lane >> 4, c16 = lane & 15;
  const bool fw = i < P.nl;
  const NgpLayer& L = P.ly[fw ? i : 2 * P.nl - 1 - i];
  const int width = fw ? L.Npad : L.Kpad;   // output width of the step
  const int depth = fw ? L.Kpad : L.Npad;   // reduction length
  const int cb = width == 64 ? wave : (wave & 1);
  const float* src = (fw ? w : wt) + L.w_off + (cb * 16 + c16) * depth + 4 * g;
  const int ns = depth / 16;
#pragma unroll
  for (int j = 0; j < 4; ++j) f.a[j] = *reinterpret_cast<const float4*>(src + 16 * (j < ns ? j : 0));
  f.b = *reinterpret_cast<const float4*>(w + L.b_off + (fw ? cb * 16 : 0) + 4 * g);
}

// W^T image of every layer (Kpad x Npad at the layer's packed weight offset) for the input-gradient fragments
__global__ __launch_bounds__(256) void ngp_wt_kernel(NgpPlan P, const float* __restrict__ w, float* __restrict__ wt) {
  const NgpLayer& L = P.ly[blockIdx.x];
  for (int i = threadIdx.x; i < L.Kpad * L.Npad; i += 256) {
    const int k = i / L.Npad, n = i - k * L.Npad;
    wt[L.w_off + i] = w[L.w_off + n * L.Kpad + k];
  }
}

// acc[b] (16x16) += A(16 x 4 KS) B_b for NRB row blocks whose B rows come from LDS (4 k-values per lane per 16-k
// slab).  Compile-time KS / NRB: every LDS read is issued before the first MFMA, and the row blocks' accumulator
// chains interleave (16x16x4 has 40 cycles of dependent latency against 32 of issue).
template <int KS, int NRB>
__device__ __forceinline__ void mfma16_tile(float4 (&acc)[2], const NgpFrag& f, const float* row0, int ld) {
  typedef float f32x4 __attribute__((ext_vector_type(4)));
  float4 x[NRB][KS];
#pragma unroll
  for (int b = 0; b < NRB; ++b)
#pragma unroll
    for (int j = 0; j < KS; ++j) x[b][j] = *reinterpret_cast<const float4*>(row0 + 16 * b * ld + 16 * j);
  f32x4 c[NRB];
#pragma unroll
  for (int b = 0; b < NRB; ++b) c[b] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < KS; ++j) {
    const float av[4] = {f.a[j].x, f.a[j].y, f.a[j].z, f.a[j].w};
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int b = 0; b < NRB; ++b) {
        const float xv = e == 0 ? x[b][j].x : e == 1 ? x[b][j].y : e == 2 ? x[b][j].z : x[b][j].w;
        c[b] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[e], xv, c[b], 0, 0, 0);
      }
  }
#pragma unroll
  for (int b = 0; b < NRB; ++b) acc[b] = make_float4(c[b][0], c[b][1], c[b][2], c[b][3]);
}

// Y[32 x Npad] = act(X W^T + b): lane (g, c16) of a block holds Y[16 rb + c16][16 cb + 4 g .. + 3]
template <int KS, int NRB>
__device__ __forceinline__ void layer_fwd16_t(const NgpLayer& L, float* smem, const NgpFrag& f, int wave, int lane) {
  const int g = lane >> 4, c16 = lane & 15;
  const int cb = NRB == 2 ? wave : (wave & 1), rb0 = NRB == 2 ? 0 : (wave >> 1);
  float4 acc[2];
  mfma16_tile<KS, NRB>(acc, f, smem + L.in_buf + (16 * rb0 + c16) * L.in_ld + 4 * g, L.in_ld);
#pragma unroll
  for (int b = 0; b < NRB; ++b) {
    float v0 = acc[b].x + f.b.x, v1 = acc[b].y + f.b.y, v2 = acc[b].z + f.b.z, v3 = acc[b].w + f.b.w;
    if (L.relu) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
    *reinterpret_cast<float4*>(smem + L.out_buf + (16 * (rb0 + b) + c16) * L.out_ld + cb * 16 + 4 * g) =
        make_float4(v0, v1, v2, v3);
  }
}

__device__ __forceinline__ void layer_fwd16(const NgpLayer& L, float* smem, const NgpFrag& f, int wave, int lane) {
  // Kpad, Npad in {32, 64}: uniform dispatch to the four compile-time shapes
  if (L.Kpad == 64) {
    if (L.Npad == 64) layer_fwd16_t<4, 2>(L, smem, f, wave, lane);
    else layer_fwd16_t<4, 1>(L, smem, f, wave, lane);
  } else {
    if (L.Npad == 64) layer_fwd16_t<2, 2>(L, smem, f, wave, lane);
    else layer_fwd16_t<2, 1>(L, smem, f, wave, lane);
  }
}

// Gnext[r][k] = sum_n G[r][n] W[n][k]  (masked by X > 0 when the input is a ReLU output).  If dst_global the
// result goes to d_enc rows m < M, columns < ncols instead of LDS.
template <int KS, int NRB>
__device__ __forceinline__ void layer_dgrad16_t(const NgpLayer& L, float* smem, const NgpFrag& f, int G, int Gn,
                                                int wave, int lane, float* __restrict__ dst_global, int ds, int ncols,
                                                int64_t m0, int64_t M) {
  const int g = lane >> 4, c16 = lane & 15;
  const int kb = NRB == 2 ? wave : (wave & 1), rb0 = NRB == 2 ? 0 : (wave >> 1);
  float4 acc[2];
  mfma16_tile<KS, NRB>(acc, f, smem + G + (16 * rb0 + c16) * 68 + 4 * g, 68);
  const int k0 = kb * 16 + 4 * g;
#pragma unroll
  for (int b = 0; b < NRB; ++b) {
    const int r = 16 * (rb0 + b) + c16;
    float v0 = acc[b].x, v1 = acc[b].y, v2 = acc[b].z, v3 = acc[b].w;
    if (dst_global) {
      const int64_t m = m0 + r;
      if (m < M) {
        float* o = dst_global + m * ds + k0;
        if (k0 < ncols) o[0] = v0;
        if (k0 + 1 < ncols) o[1] = v1;
        if (k0 + 2 < ncols) o[2] = v2;
        if (k0 + 3 < ncols) o[3] = v3;
      }
    } else {
      if (L.in_relu) {
        const float4 x = *reinterpret_cast<const float4*>(smem + L.in_buf + r * L.in_ld + k0);
        v0 = x.x > 0.f ? v0 : 0.f; v1 = x.y > 0.f ? v1 : 0.f; v2 = x.z > 0.f ? v2 : 0.f; v3 = x.w > 0.f ? v3 : 0.f;
      }
      *reinterpret_cast<float4*>(smem + Gn + r * 68 + k0) = make_float4(v0, v1, v2, v3);
    }
  }
}

__device__ __forceinline__ void layer_dgrad16(const NgpLayer& L, float* smem, const NgpFrag& f, int G, int Gn,
                                              int wave, int lane, float* __restrict__ dst_global, int ds, int ncols,
                                              int64_t m0, int64_t M) {
  // reduction over Npad, output width Kpad
  if (L.Npad == 64) {
    if (L.Kpad == 64) layer_dgrad16_t<4, 2>(L, smem, f, G, Gn, wave, lane, dst_global, ds, ncols, m0, M);
    else layer_dgrad16_t<4, 1>(L, smem, f, G, Gn, wave, lane, dst_global, ds, ncols, m0, M);
  } else {
    if (L.Kpad == 64) layer_dgrad16_t<2, 2>(L, smem, f, G, Gn, wave, lane, dst_global, ds, ncols, m0, M);
    else layer_dgrad16_t<2, 1>(L, smem, f, G, Gn, wave, lane, dst_global, ds, ncols, m0, M);
  }
}

// acc += G[:, nb-block]^T X[:, kb-block] over the tile's 32 rows; lane li <-> k = kb*32 + li, register
// 4q+e <-> n = nb*32 + 8q + 4lh + e.  Operands of 8 MFMAs are read ahead of them.
__device__ __forceinline__ void wgrad_block(ngp_f32x16& acc, const NgpLayer& L, const float* smem, int G, int nb,
                                            int kb, int li, int lh) {
  const float* Gc = smem + G + nb * 32 + li + 8 * lh * 68;
  const float* Xc = smem + L.in_buf + kb * 32 + li + 8 * lh * L.in_ld;
#pragma unroll
  for (int s = 0; s < NGP_BROWS / 16; ++s) {
    float gv[8], xv[8];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      gv[t] = Gc[(16 * s + t) * 68];
      xv[t] = Xc[(16 * s + t) * L.in_ld];
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(gv[t], xv[t], acc, 0, 0, 0);
  }
}

// LDS writes of every wave visible, then s_barrier — without the release fence of __syncthreads, which would also
// wait for the weight prefetch in flight
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int NSB>
__global__ __launch_bounds__(256, 2) void ngp_bwd_kernel(NgpPlan P, const float* __restrict__ w,
                                                         const float* __restrict__ enc, int es,
                                                         const float* __restrict__ x_d, int64_t M,
                                                         const float* __restrict__ gout, float* __restrict__ d_enc,
                                                         float* __restrict__ partial,
                                                         const float* __restrict__ wt, int64_t ntiles) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* dsig = smem + P.dsig;
  // wave index in an SGPR: the plan's per-wave tables (sb_layer, ...) are then scalar kernarg loads, not vector
  // loads that the compiler would wait for with vmcnt(0) (draining the weight prefetch)
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, li = lane & 31,
            lh = lane >> 5;
  ngp_f32x16 accw[NSB];
#pragma unroll
  for (int j = 0; j < NSB; ++j) accw[j] = zero16();
  // bias gradients: wave w sums rows 8w..8w+7 of every tile into its own LDS partial (column = lane); without
  // room for the partials (P.bsum < 0) wave l&3 sums all rows of layer l into bacc[l>>2]
  float* bsum = smem + (P.bsum >= 0 ? P.bsum : 0) + wave * P.nl * 64;
  if (P.bsum >= 0)
    for (int l = 0; l < P.nl; ++l) bsum[l * 64 + lane] = 0.f;
  float bacc[3] = {0.f, 0.f, 0.f};
  const int nsteps = 2 * P.nl;
  // fragment ping-pong: step s computes with (s even ? fa : fb) and prefetches step s + 1 into the other (2 nl steps
  // per tile, so the parity carries over to the next tile); no register copies, which would wait for the prefetch
  NgpFrag fa, fb;
  load_frag(P, w, wt, 0, wave, lane, fa);

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t m0 = tile * NGP_BROWS;
    // ---- tile inputs, spread over the workgroup: thread (r = tid / 8, p = tid % 8) owns row r's columns
    // p, p + 8, ... of the enc tile and of the direction encoding (cin columns geo..), and keeps the row's output
    // gradient.  Loads are unconditional (rows clamped to M - 1, masked after), so none of them drains the weight
    // prefetch with vmcnt(0).
    const int pr = tid >> 3, pp = tid & 7;
    {
      const int64_t m = m0 + pr;
      const int64_t mc = m < M ? m : M - 1;
      const int kp = P.enc_ld - 4;
      const float* src = enc + mc * es;
      float* erow = smem + P.enc_buf + pr * P.enc_ld;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = pp + 8 * i;
        const float v = src[c < P.in_dim ? c : 0];
        if (c < kp) erow[c] = (m < M && c < P.in_dim) ? v : 0.f;
      }
      const float* dr = x_d + mc * 6 + 3;
      const float dx = dr[0], dy = dr[1], dz = dr[2];
      float v[27];
      dir_encode(P, m < M ? dx : 0.f, m < M ? dy : 0.f, m < M ? dz : 1.f, v);
      float* crow = smem + P.cin_buf + pr * P.cin_ld;
#pragma unroll
      for (int k = 0; k < 27; ++k)
        if (k < P.dir_dim && (k & 7) == pp) crow[P.geo + k] = v[k];
      for (int c = P.geo + P.dir_dim + pp; c < P.cin_kpad; c += 8) crow[c] = 0.f;
    }
    lds_barrier();
    int G = P.g0, Gn = P.g1;
    // step s < nl: forward of layer s; the last forward step also forms the output gradients.  Step s >= nl: layer
    // l = 2 nl - 1 - s in reverse (weight gradient, bias partials, input gradient).
    auto step = [&](int s, const NgpFrag& use, NgpFrag& pre) {
      // lane-derived values recomputed per step from an opaque copy: otherwise the compiler hoists every per-lane
      // LDS address of every layer shape out of the tile loop and holds them all in VGPRs (spilling past 256)
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      const int li = lane & 31, lh = lane >> 5, pr = 8 * wave + (lane >> 3), pp = lane & 7;
      // the row's output gradient, issued before the weight prefetch so that waiting for it leaves that in flight
      float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
      if (s == P.nl - 1) gv = reinterpret_cast<const float4*>(gout)[m0 + pr < M ? m0 + pr : M - 1];
      load_frag(P, w, wt, s + 1 == nsteps ? 0 : s + 1, wave, lane, pre);
      if (s < P.nl) {
        layer_fwd16(P.ly[s], smem, use, wave, lane);
        lds_barrier();
        if (s == P.head) {  // cin columns 0..geo-1 = head output columns 1..geo
          const float* hrow = smem + P.ly[P.head].out_buf + pr * P.ly[P.head].out_ld;
          float* crow = smem + P.cin_buf + pr * P.cin_ld;
          for (int c = pp; c < P.geo; c += 8) crow[c] = hrow[1 + c];
          lds_barrier();
        }
        if (s == P.nl - 1) {
          // output gradients: rgb through the sigmoid, sigma through trunc_exp (trunc_exp.py:54-57); thread p = 0 of
          // each row (8 rows per wave, so all four waves share the work)
          const NgpLayer& Lo = P.ly[P.nl - 1];
          const NgpLayer& Lh = P.ly[P.head];
          float4 gq = make_float4(0.f, 0.f, 0.f, 0.f);
          if (m0 + pr >= M) gv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (pp == 0) {
            const float* o = smem + Lo.out_buf + pr * Lo.out_ld;
            const float gg[3] = {gv.x, gv.y, gv.z};
            float gc[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              if (P.sigmoid) {
                const float sg = nerf_mlp::sigmoidf_(o[c]);
                gc[c] = gg[c] * (sg * (1.0f - sg));
              } else {
                gc[c] = gg[c];
              }
            }
            gq = make_float4(gc[0], gc[1], gc[2], 0.f);
            const float sr = smem[Lh.out_buf + pr * Lh.out_ld];
            dsig[pr] = gv.w * expf(fminf(fmaxf(sr, -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
          }
          lds_barrier();  // the raw head/out tiles alias the gradient tiles
          *reinterpret_cast<float4*>(smem + P.g0 + pr * 68 + 4 * pp) = gq;
          lds_barrier();
          G = P.g0; Gn = P.g1;
        }
        return;
      }
      const int l = 2 * P.nl - 1 - s;
      const NgpLayer& L = P.ly[l];
      // weight gradient blocks of this layer owned by this wave
#pragma unroll
      for (int j = 0; j < NSB; ++j) {
        const int sb = wave + 4 * j;
        if (sb < P.nsb && P.sb_layer[sb] == l) wgrad_block(accw[j], L, smem, G, P.sb_nb[sb], P.sb_kb[sb], li, lh);
      }
      if (P.bsum >= 0 && lane < L.Npad) {
        const float* gcol = smem + G + (8 * wave) * 68 + lane;
        float sum = 0.f;
#pragma unroll
        for (int r = 0; r < 8; ++r) sum += gcol[r * 68];
        bsum[l * 64 + lane] += sum;
      } else if (P.bsum < 0 && (l & 3) == wave && lane < L.Npad) {
        float sum = 0.f;
        for (int r = 0; r < NGP_BROWS; ++r) sum += smem[G + r * 68 + lane];
        bacc[l >> 2] += sum;
      }
      // input gradient
      const bool to_enc = (l == 0);
      layer_dgrad16(L, smem, use, G, Gn, wave, lane, to_enc ? d_enc : nullptr, es, P.in_dim, m0, M);
      lds_barrier();
      if (l == P.head + 1) {
        // Gn holds d cin: the head's gradient is [d sigma_raw, d geo, 0...] (thread (r, p): columns 4p..4p+3)
        {
          const float* dc = smem + Gn + pr * 68;
          float hv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int c = 4 * pp + e;
            hv[e] = c == 0 ? dsig[pr] : (c <= P.geo ? dc[c - 1] : 0.f);
          }
          *reinterpret_cast<float4*>(smem + G + pr * 68 + 4 * pp) = make_float4(hv[0], hv[1], hv[2], hv[3]);
        }
        lds_barrier();
      } else {
        const int t = G; G = Gn; Gn = t;
      }
    };
    // pairs of steps with fixed operands (2 nl steps per tile): no selects or copies between the two fragments
    for (int s = 0; s < nsteps; s += 2) {
      step(s, fa, fb);
      step(s + 1, fb, fa);
    }
  }
  // slab of this workgroup: every packed float is written exactly once
  float* slab = partial + (int64_t)blockIdx.x * P.total;
#pragma unroll
  for (int j = 0; j < NSB; ++j) {
    const int sb = wave + 4 * j;
    if (sb < P.nsb && P.sb_layer[sb] >= 0) {
      const NgpLayer& L = P.ly[P.sb_layer[sb]];
      const int k = P.sb_kb[sb] * 32 + li;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int n = P.sb_nb[sb] * 32 + 8 * q + 4 * lh + e;
          slab[L.w_off + (int64_t)n * L.Kpad + k] = accw[j][4 * q + e];
        }
    }
  }
  if (P.bsum >= 0) {
    __syncthreads();
    for (int l = wave; l < P.nl; l += 4) {
      if (lane < P.ly[l].Npad) {
        const float* b = smem + P.bsum + l * 64 + lane;
        const int ws = P.nl * 64;
        slab[P.ly[l].b_off + lane] = (b[0] + b[ws]) + (b[2 * ws] + b[3 * ws]);
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int l = wave + 4 * j;
      if (l < P.nl && lane < P.ly[l].Npad) slab[P.ly[l].b_off + lane] = bacc[j];
    }
  }
}

// ---- the production expert's backward.  MetaNGP's defaults (nerf_runner.py:103-121; meta_ngp.py:21-105): hash
// encoding <= 32 wide, sigma trunk 2 x 64, head 1 + 15, SH degree-4 directions (16), colour 2 x 64, rgb.  The same
// algorithm as ngp_bwd_kernel with every shape, LDS offset and weight-gradient block fixed at compile time: the whole
// tile is straight-line code (no plan lookups, no branches on the layer shape, no conditional accumulator updates),
// the head / rgb layers compute only their live 16 columns, and the weight gradients use balanced 16x16 blocks (each
// wave owns a quarter of every layer's live blocks, so no wave idles through a layer's barrier interval).
namespace ngp_prod {
constexpr int NL = 6, HEAD = 2;
constexpr int KP[NL] = {32, 64, 64, 32, 64, 64};    // padded fan-in
constexpr int NP[NL] = {64, 64, 32, 64, 64, 32};    // padded fan-out (packed layout)
constexpr int NE[NL] = {64, 64, 16, 64, 64, 16};    // live fan-out: head 1 + 15, rgb 3 -> 16
constexpr int RELU[NL] = {1, 1, 0, 1, 1, 0};
constexpr int INRELU[NL] = {0, 1, 1, 0, 1, 1};
constexpr int WOFF[NL] = {0, 2112, 6272, 8352, 10464, 14624};
constexpr int BOFF[NL] = {2048, 6208, 8320, 10400, 14560, 16672};
constexpr int TOTAL = 16704;
// LDS (floats; the backward plan of make_plan for this shape, checked on the host)
constexpr int ENC = 0, CIN = 1152, G0 = 2304, G1 = 4480, DSIG = 6656, BSUM = 15392, SMEM = 16928;
constexpr int OUTB[NL] = {6688, 8864, G0, 11040, 13216, G1};
constexpr int INB[NL] = {ENC, 6688, 8864, CIN, 11040, 13216};
constexpr int INLD[NL] = {36, 68, 68, 36, 68, 68};
constexpr int GEO = 15, DIRD = 16;
// gradient tile read (G) and written (GN) by the input-gradient step of layer l (g0 holds the output gradients)
constexpr int GB[NL] = {G0, G1, G0, G0, G1, G0};
constexpr int GNB[NL] = {-1, G0, G1, G1, G0, G1};
// weight-gradient 16x16 blocks: layer l has (NE/16) x (KP/16) live blocks, block i = wave + 4 q -> (i / (KP/16),
// i % (KP/16)); NBW[l] blocks per wave in accumulator slots SLOT0[l]..
constexpr int NBW[NL] = {2, 4, 1, 2, 4, 1};
constexpr int SLOT0[NL] = {0, 2, 6, 7, 9, 13};
constexpr int NSLOT = 14;

template <int B, int E, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

// weights of step s (forward layer s < NL, else the input gradient of layer 2 NL - 1 - s): a fixed, per-step load
// count, so the compiler's waits for the current fragment are exact
template <int S>
__device__ __forceinline__ void load_frag(const float* __restrict__ w, const float* __restrict__ wt, int wave, int lane,
                                          NgpFrag& f) {
  constexpr bool fw = S < NL;
  constexpr int l = fw ? S : 2 * NL - 1 - S;
  constexpr int width = fw ? NE[l] : KP[l], depth = fw ? KP[l] : NE[l], pitch = fw ? KP[l] : NP[l];
  const int g = lane >> 4, c16 = lane & 15;
  const int cb = width == 64 ? wave : width == 32 ? (wave & 1) : 0;
  const float* src = (fw ? w : wt) + WOFF[l] + (cb * 16 + c16) * pitch + 4 * g;
#pragma unroll
  for (int j = 0; j < depth / 16; ++j) f.a[j] = *reinterpret_cast<const float4*>(src + 16 * j);
  if constexpr (fw) f.b = *reinterpret_cast<const float4*>(w + BOFF[l] + cb * 16 + 4 * g);
}

template <int l, int IN = INB[l], int IN_LD = INLD[l], int OUT = OUTB[l]>
__device__ __forceinline__ void fwd(float* smem, const NgpFrag& f, int wave, int lane) {
  constexpr int NRB = NE[l] == 64 ? 2 : 1;
  if (NE[l] == 16 && wave >= 2) return;  // 16 live columns: one column block, waves 0-1 take its row blocks
  const int g = lane >> 4, c16 = lane & 15;
  const int cb = NE[l] == 64 ? wave : 0, rb0 = NE[l] == 64 ? 0 : wave;
  float4 acc[2];
  mfma16_tile<KP[l] / 16, NRB>(acc, f, smem + IN + (16 * rb0 + c16) * IN_LD + 4 * g, IN_LD);
#pragma unroll
  for (int b = 0; b < NRB; ++b) {
    float v0 = acc[b].x + f.b.x, v1 = acc[b].y + f.b.y, v2 = acc[b].z + f.b.z, v3 = acc[b].w + f.b.w;
    if (RELU[l]) { v0 = fmaxf(v0, 0.f); v1 = fmaxf(v1, 0.f); v2 = fmaxf(v2, 0.f); v3 = fmaxf(v3, 0.f); }
    *reinterpret_cast<float4*>(smem + OUT + (16 * (rb0 + b) + c16) * 68 + cb * 16 + 4 * g) =
        make_float4(v0, v1, v2, v3);
  }
}

template <int l, bool ENC_TO_LDS = false>
__device__ __forceinline__ void dgrad(float* smem, const NgpFrag& f, int wave, int lane, float* __restrict__ d_enc,
                                      int es, int in_dim, int64_t m0, int64_t M) {
  constexpr int NRB = KP[l] == 64 ? 2 : 1;
  const int g = lane >> 4, c16 = lane & 15;
  const int kb = KP[l] == 64 ? wave : (wave & 1), rb0 = KP[l] == 64 ? 0 : (wave >> 1);
  float4 acc[2];
  mfma16_tile<NE[l] / 16, NRB>(acc, f, smem + GB[l] + (16 * rb0 + c16) * 68 + 4 * g, 68);
  const int k0 = kb * 16 + 4 * g;
#pragma unroll
  for (int b = 0; b < NRB; ++b) {
    const int r = 16 * (rb0 + b) + c16;
    float v0 = acc[b].x, v1 = acc[b].y, v2 = acc[b].z, v3 = acc[b].w;
    if constexpr (l == 0 && ENC_TO_LDS) {  // d_enc tile -> the free gradient tile (G1) for the fused table scatter
      *reinterpret_cast<float4*>(smem + G1 + r * 68 + k0) = make_float4(v0, v1, v2, v3);
    } else if constexpr (l == 0) {
      const int64_t m = m0 + r;
      if (m < M) {
        float* o = d_enc + m * es + k0;
        if (k0 < in_dim) o[0] = v0;
        if (k0 + 1 < in_dim) o[1] = v1;
        if (k0 + 2 < in_dim) o[2] = v2;
        if (k0 + 3 < in_dim) o[3] = v3;
      }
    } else {
      if (INRELU[l]) {
        const float4 x = *reinterpret_cast<const float4*>(smem + INB[l] + r * INLD[l] + k0);
        v0 = x.x > 0.f ? v0 : 0.f; v1 = x.y > 0.f ? v1 : 0.f; v2 = x.z > 0.f ? v2 : 0.f; v3 = x.w > 0.f ? v3 : 0.f;
      }
      *reinterpret_cast<float4*>(smem + GNB[l] + r * 68 + k0) = make_float4(v0, v1, v2, v3);
    }
  }
}

// acc[slot] (16x16: n = 16 nb + 4 g + e, k = 16 kb + c16) += sum over the tile's 32 rows of G[r][n] X[r][k];
// MFMA s reduces rows 8 g + s (lane group g), the wave's blocks of the layer interleaved
template <int l>
__device__ __forceinline__ void wgrad(ngp_f32x4 (&acc)[NSLOT], const float* smem, int wave, int lane) {
  constexpr int KB = KP[l] / 16;
  const int g = lane >> 4, c16 = lane & 15;
  float gv[NBW[l]][8], xv[NBW[l]][8];
#pragma unroll
  for (int q = 0; q < NBW[l]; ++q) {
    const int i = wave + 4 * q, nb = i / KB, kb = i % KB;
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      gv[q][s] = smem[GB[l] + (8 * g + s) * 68 + nb * 16 + c16];
      xv[q][s] = smem[INB[l] + (8 * g + s) * INLD[l] + kb * 16 + c16];
    }
  }
#pragma unroll
  for (int s = 0; s < 8; ++s)
#pragma unroll
    for (int q = 0; q < NBW[l]; ++q)
      acc[SLOT0[l] + q] = __builtin_amdgcn_mfma_f32_16x16x4f32(gv[q][s], xv[q][s], acc[SLOT0[l] + q], 0, 0, 0);
}

// one tile's inputs for thread (row pr, part pp): enc columns pp + 8 i and the ray direction; rows clamped to M - 1
struct TileIn {
  float e[4];
  float d[3];
};

__device__ __forceinline__ void load_tile_in(const float* __restrict__ enc, int es, int in_dim,
                                             const float* __restrict__ x_d, int64_t M, int64_t tile, int pr, int pp,
                                             TileIn& t) {
  const int64_t m = tile * NGP_BROWS + pr;
  const int64_t mc = m < M ? m : M - 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = pp + 8 * i;
    t.e[i] = enc[mc * es + (c < in_dim ? c : 0)];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) t.d[c] = x_d[mc * 6 + 3 + c];
}

}  // namespace ngp_prod

// HB: the hash-table gradient is scattered from the kernel itself — d_enc of a tile goes to LDS (never to HBM) and
// the four waves issue hash_bwd_f2_agg_kernel's run-aggregated atomics for it (wave w: samples 16 (w & 1) .. + 15 of
// the tile, levels 8 (w >> 1) .. + 7; the same 16-consecutive-sample grouping, so the same request count), while the
// other workgroup on the CU runs its MFMAs: the MLP backward hides under the memory-side atomic traffic.
template <int SIGMOID, bool HB = false>
__global__ __launch_bounds__(256, 2) void ngp_bwd_prod_kernel(const float* __restrict__ w, const float* __restrict__ wt,
                                                              const float* __restrict__ enc, int es, int in_dim,
                                                              const float* __restrict__ x_d, int64_t M,
                                                              const float* __restrict__ gout,
                                                              float* __restrict__ d_enc, float* __restrict__ partial,
                                                              int64_t ntiles, HashArgs ha = HashArgs{},
                                                              float* __restrict__ dtab = nullptr,
                                                              const int32_t* __restrict__ rng = nullptr) {
  using namespace ngp_prod;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (rng) {  // device-sized launch (nerf_ngp_bwd_hash_n): M is the capacity, the rows are rng[1] - rng[0]
    const int64_t n = (int64_t)rng[1] - rng[0];
    M = n < 0 ? 0 : (n < M ? n : M);
    ntiles = (M + NGP_BROWS - 1) / NGP_BROWS;
  }
  ngp_f32x4 acc[NSLOT];
#pragma unroll
  for (int j = 0; j < NSLOT; ++j) acc[j] = ngp_f32x4{0.f, 0.f, 0.f, 0.f};
  float bacc[NL];  // bias gradient of column `lane`, this wave's rows 8 wave .. 8 wave + 7 of every tile
#pragma unroll
  for (int l = 0; l < NL; ++l) bacc[l] = 0.f;
  NgpFrag fa, fb;
  load_frag<0>(w, wt, wave, tid & 63, fa);
  TileIn nx;
  if (M > 0) load_tile_in(enc, es, in_dim, x_d, M, blockIdx.x, tid >> 3, tid & 7, nx);

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t m0 = tile * NGP_BROWS;
    // ---- tile inputs (prefetched during the previous tile's backward) -> enc tile, cin direction columns
    {
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      const int pr = 8 * wave + (lane >> 3), pp = lane & 7;
      const bool ok = m0 + pr < M;
      float* erow = smem + ENC + pr * 36;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = pp + 8 * i;
        erow[c] = (ok && c < in_dim) ? nx.e[i] : 0.f;
      }
      float v[27];
      float x = ok ? nx.d[0] : 0.f, y = ok ? nx.d[1] : 0.f, z = ok ? nx.d[2] : 1.f;
      unit3(x, y, z, 1e-9f);  // MetaNGP._enc_dir (meta_ngp.py:176-179)
      unit3(x, y, z, 1e-9f);  // SHEncoder.forward normalises again (encodings.py:141)
      sh_eval(3, x, y, z, v);
      float v0 = v[0], v8 = v[8];  // components pp and 8 + pp (selects: a runtime index would put v in scratch)
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if (pp == k) { v0 = v[k]; v8 = v[8 + k]; }
      float* crow = smem + CIN + pr * 36;
      crow[GEO + pp] = v0;
      crow[GEO + 8 + pp] = v8;
      if (pp == 0) crow[GEO + DIRD] = 0.f;
    }
    lds_barrier();
    sfor<0, 2 * NL>([&](auto S) {
      constexpr int s = decltype(S)::value;
      NgpFrag& use = (s & 1) ? fb : fa;
      NgpFrag& pre = (s & 1) ? fa : fb;
      int lane = tid & 63;
      asm volatile("" : "+v"(lane));
      const int pr = 8 * wave + (lane >> 3), pp = lane & 7;
      float4 gv = make_float4(0.f, 0.f, 0.f, 0.f);
      if constexpr (s == NL - 1) gv = reinterpret_cast<const float4*>(gout)[m0 + pr < M ? m0 + pr : M - 1];
      if constexpr (s == NL) load_tile_in(enc, es, in_dim, x_d, M, tile + gridDim.x, pr, pp, nx);
      load_frag<(s + 1) % (2 * NL)>(w, wt, wave, lane, pre);
      if constexpr (s < NL) {
        fwd<s>(smem, use, wave, lane);
        lds_barrier();
        if constexpr (s == HEAD) {  // cin columns 0..14 = head output columns 1..15
          const float* hrow = smem + G0 + pr * 68;
          float* crow = smem + CIN + pr * 36;
          crow[pp] = hrow[1 + pp];
          if (pp < GEO - 8) crow[8 + pp] = hrow[9 + pp];
          lds_barrier();
        }
        if constexpr (s == NL - 1) {
          // output gradients: rgb through the sigmoid, sigma through trunc_exp (trunc_exp.py:54-57)
          float4 gq = make_float4(0.f, 0.f, 0.f, 0.f);
          if (m0 + pr >= M) gv = make_float4(0.f, 0.f, 0.f, 0.f);
          if (pp == 0) {
            const float* o = smem + G1 + pr * 68;
            if (SIGMOID) {
              const float s0 = nerf_mlp::sigmoidf_(o[0]), s1 = nerf_mlp::sigmoidf_(o[1]),
                          s2 = nerf_mlp::sigmoidf_(o[2]);
              gq = make_float4(gv.x * (s0 * (1.0f - s0)), gv.y * (s1 * (1.0f - s1)), gv.z * (s2 * (1.0f - s2)), 0.f);
            } else {
              gq = make_float4(gv.x, gv.y, gv.z, 0.f);
            }
            const float sr = smem[G0 + pr * 68];
            smem[DSIG + pr] = gv.w * expf(fminf(fmaxf(sr, -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
          }
          lds_barrier();  // the raw head / rgb tiles alias the gradient tiles
          *reinterpret_cast<float4*>(smem + G0 + pr * 68 + 4 * pp) = gq;
          lds_barrier();
        }
      } else {
        constexpr int l = 2 * NL - 1 - s;
        wgrad<l>(acc, smem, wave, lane);
        if (lane < NP[l]) {
          const float* gcol = smem + GB[l] + (8 * wave) * 68 + lane;
          float sum = 0.f;
#pragma unroll
          for (int r = 0; r < 8; ++r) sum += gcol[r * 68];
          bacc[l] += sum;
        }
        dgrad<l, HB>(smem, use, wave, lane, d_enc, es, in_dim, m0, M);
        lds_barrier();
        if constexpr (HB && l == 0) {
          // table scatter of this tile (hash_bwd_f2_agg_kernel's lanes: q = (x-corner, feature), 16 samples)
          const int q = lane & 3, grp = lane >> 2;
          const int r = 16 * (wave & 1) + grp;
          const int64_t m = m0 + r;
          const bool valid = m < M;
          float p[3] = {0.f, 0.f, 0.f};
          if (valid) load_x01(ha, x_d, 6, m, p);
          const uint32_t mask = (1u << ha.log2T) - 1u;
          const int dx = q >> 1, f = q & 1;
          const unsigned long long qmask = 0x1111111111111111ull << q;
          const unsigned long long after = lane == 63 ? 0ull : ~((2ull << lane) - 1ull);
          const float* drow = smem + G1 + r * 68;
          // a fixed count of 32 atomic instructions per wave (8 levels x 4 corners, lanes masked): with a variable
          // count the compiler would wait for the next tile's first weight fragments with vmcnt(0), behind them
#pragma unroll
          for (int li2 = 0; li2 < 8; ++li2) {
            const int l2 = 8 * (wave >> 1) + li2;
            const bool lvalid = valid && l2 < ha.L;
            const float rr = (float)ha.res[l2 < ha.L ? l2 : 0];
            float wv[3];
            int i0[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
              const float sc = __fmul_rn(p[c], rr);
              const float fl = floorf(sc);
              wv[c] = __fsub_rn(sc, fl);
              i0[c] = (int)fl;
              if (ha.interp == 2) wv[c] = __fmul_rn(__fmul_rn(wv[c], wv[c]), __fsub_rn(3.0f, __fmul_rn(2.0f, wv[c])));
            }
            const float u[3] = {__fsub_rn(1.0f, wv[0]), __fsub_rn(1.0f, wv[1]), __fsub_rn(1.0f, wv[2])};
            const float wx = dx ? wv[0] : u[0];
            const float gg = lvalid ? drow[2 * l2 + f] : 0.f;
            float* tb = dtab + ((int64_t)l2 << ha.log2T) * 2;
#pragma unroll
            for (int yz = 0; yz < 4; ++yz) {
              const int dy = yz >> 1, dz = yz & 1;
              const float v = __fmul_rn(__fmul_rn(__fmul_rn(gg, dz ? wv[2] : u[2]), dy ? wv[1] : u[1]), wx);
              const uint32_t idx = lvalid ? ngp_hash(i0[0] + dx, i0[1] + dy, i0[2] + dz, mask) * 2u + (uint32_t)f
                                          : 0xFFFFFFFFu;
              const uint32_t prev = __shfl_up(idx, 4, 64);
              const bool head = grp == 0 || prev != idx;
              const unsigned long long nxt = __ballot(head) & qmask & after;
              const int run_end = nxt ? (int)__builtin_ctzll(nxt) - 4 : 60 + q;
              float sum = v;
#pragma unroll
              for (int off = 4; off < 64; off <<= 1) {
                const float o = __shfl_down(sum, off, 64);
                if (lane + off <= run_end) sum += o;
              }
              if (head && lvalid) unsafeAtomicAdd(tb + idx, sum);
            }
          }
        }
        if constexpr (l == HEAD + 1) {
          // GNB holds d cin: the head's gradient is [d sigma_raw, d geo, 0...] (thread (r, p): columns 4p..4p+3)
          const float* dc = smem + GNB[l] + pr * 68;
          float hv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int c = 4 * pp + e;
            hv[e] = c == 0 ? smem[DSIG + pr] : (c <= GEO ? dc[c - 1] : 0.f);
          }
          *reinterpret_cast<float4*>(smem + GB[HEAD] + pr * 68 + 4 * pp) = make_float4(hv[0], hv[1], hv[2], hv[3]);
          lds_barrier();
        }
      }
    });
  }
  // ---- this workgroup's slab: every packed float written exactly once
  const int lane = tid & 63, g = lane >> 4, c16 = lane & 15;
  float* slab = partial + (int64_t)blockIdx.x * TOTAL;
  sfor<0, NL>([&](auto Lc) {
    constexpr int l = decltype(Lc)::value;
    constexpr int KB = KP[l] / 16;
#pragma unroll
    for (int q = 0; q < NBW[l]; ++q) {
      const int i = wave + 4 * q, nb = i / KB, kb = i % KB;
#pragma unroll
      for (int e = 0; e < 4; ++e) slab[WOFF[l] + (nb * 16 + 4 * g + e) * KP[l] + kb * 16 + c16] = acc[SLOT0[l] + q][e];
    }
    if constexpr (NE[l] < NP[l])  // dead rows of the head / rgb weights
      for (int i = tid; i < (NP[l] - NE[l]) * KP[l]; i += 256) slab[WOFF[l] + NE[l] * KP[l] + i] = 0.f;
    smem[BSUM + (wave * NL + l) * 64 + lane] = bacc[l];
  });
  __syncthreads();
  for (int l = wave; l < NL; l += 4) {
    if (lane < NP[l]) {
      const float* b = smem + BSUM + l * 64 + lane;
      constexpr int ws = NL * 64;
      slab[BOFF[l] + lane] = (b[0] + b[ws]) + (b[2 * ws] + b[3 * ws]);
    }
  }
}

// The production expert's forward (MODE 0: rgb + sigma, nerf_ngp_fwd) and density (MODE 1: sigma trunk + head only,
// nerf_ngp_density): one 32-row tile per workgroup, the same compile-time layer code as the backward's recompute,
// activations ping-ponging through two LDS tiles (27 KB per workgroup: six workgroups per CU hide the weight loads).
namespace ngp_prod {
constexpr int F_ENC = 0, F_CIN = 1152, F_PA = 2304, F_PB = 4480, F_SRAW = 6656, F_SMEM = 6688;
}

// HASH: the enc tile is computed from the sample positions (x_d cols 0..2) in the prologue — the hash_fwd_kernel
// arithmetic, (row, level) pairs t and t + 256 — and also written to enc [M][es] for the backward (one launch for the
// expert's encoding + MLP forward, the gathers of one workgroup overlapping another's MFMAs); else read from enc.
template <int MODE, int SIGMOID, bool HASH = false>
__global__ __launch_bounds__(256) void ngp_fwd_prod_kernel(const float* __restrict__ w, const float* __restrict__ enc,
                                                           int es, int in_dim, const float* __restrict__ x_d,
                                                           int64_t M, float* __restrict__ out, HashArgs ha = HashArgs{},
                                                           const float* __restrict__ table = nullptr,
                                                           float* __restrict__ enc_out = nullptr,
                                                           const int32_t* __restrict__ rng = nullptr) {
  using namespace ngp_prod;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int pr = tid >> 3, pp = tid & 7;
  if (rng) {  // device-sized launch (nerf_ngp_fwd_enc_n): the grid covers the capacity M, the rows are rng[1] - rng[0]
    const int64_t n = (int64_t)rng[1] - rng[0];
    M = n < 0 ? 0 : (n < M ? n : M);
  }
  if ((int64_t)blockIdx.x * NGP_BROWS >= M) return;  // whole workgroup: no barrier is left waiting
  const int64_t m0 = (int64_t)blockIdx.x * NGP_BROWS, m = m0 + pr, mc = m < M ? m : M - 1;
  const bool ok = m < M;
  NgpFrag fa, fb;
  load_frag<0>(w, nullptr, wave, lane, fa);
  {
    if constexpr (HASH) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int pair = tid + 256 * u, r = pair >> 4, l = pair & 15;
        const int64_t mr = m0 + r;
        float2 v = make_float2(0.f, 0.f);
        if (mr < M && l < ha.L) {
          float p[3], acc[2];
          load_x01(ha, x_d, 6, mr, p);
          hash_level<2>(ha, table, p, l, acc);
          v = make_float2(acc[0], acc[1]);
          *reinterpret_cast<float2*>(enc_out + mr * es + 2 * l) = v;
        }
        *reinterpret_cast<float2*>(smem + F_ENC + r * 36 + 2 * l) = v;
      }
      for (int i = tid; i < NGP_BROWS * (es - 2 * ha.L); i += 256) {  // enc pad columns, as hash_fwd_kernel
        const int r = i / (es - 2 * ha.L), c = 2 * ha.L + i % (es - 2 * ha.L);
        if (m0 + r < M) enc_out[(m0 + r) * es + c] = 0.f;
      }
    } else {
      float* erow = smem + F_ENC + pr * 36;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = pp + 8 * i;
        const float v = enc[mc * es + (c < in_dim ? c : 0)];
        erow[c] = (ok && c < in_dim) ? v : 0.f;
      }
    }
    if constexpr (MODE == 0) {
      const float* dr = x_d + mc * 6 + 3;
      float x = ok ? dr[0] : 0.f, y = ok ? dr[1] : 0.f, z = ok ? dr[2] : 1.f;
      float v[27];
      unit3(x, y, z, 1e-9f);  // MetaNGP._enc_dir (meta_ngp.py:176-179)
      unit3(x, y, z, 1e-9f);  // SHEncoder.forward normalises again (encodings.py:141)
      sh_eval(3, x, y, z, v);
      float v0 = v[0], v8 = v[8];
#pragma unroll
      for (int k = 1; k < 8; ++k)
        if (pp == k) { v0 = v[k]; v8 = v[8 + k]; }
      float* crow = smem + F_CIN + pr * 36;
      crow[GEO + pp] = v0;
      crow[GEO + 8 + pp] = v8;
      if (pp == 0) crow[GEO + DIRD] = 0.f;
    }
  }
  lds_barrier();
  load_frag<1>(w, nullptr, wave, lane, fb);
  fwd<0, F_ENC, 36, F_PA>(smem, fa, wave, lane);
  lds_barrier();
  load_frag<2>(w, nullptr, wave, lane, fa);
  fwd<1, F_PA, 68, F_PB>(smem, fb, wave, lane);
  lds_barrier();
  if constexpr (MODE == 0) load_frag<3>(w, nullptr, wave, lane, fb);
  fwd<2, F_PB, 68, F_PA>(smem, fa, wave, lane);
  lds_barrier();
  if constexpr (MODE == 1) {
    if (pp == 0 && ok) {
      const float sr = smem[F_PA + pr * 68];
      out[m] = expf(fminf(fmaxf(sr, -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
    }
    return;
  } else {
    {  // cin columns 0..14 = head output columns 1..15; sigma_raw aside (PA is reused by colour layer 1)
      const float* hrow = smem + F_PA + pr * 68;
      float* crow = smem + F_CIN + pr * 36;
      crow[pp] = hrow[1 + pp];
      if (pp < GEO - 8) crow[8 + pp] = hrow[9 + pp];
      if (pp == 0) smem[F_SRAW + pr] = hrow[0];
    }
    lds_barrier();
    load_frag<4>(w, nullptr, wave, lane, fa);
    fwd<3, F_CIN, 36, F_PB>(smem, fb, wave, lane);
    lds_barrier();
    load_frag<5>(w, nullptr, wave, lane, fb);
    fwd<4, F_PB, 68, F_PA>(smem, fa, wave, lane);
    lds_barrier();
    fwd<5, F_PA, 68, F_PB>(smem, fb, wave, lane);
    lds_barrier();
    if (pp == 0 && ok) {
      const float* o = smem + F_PB + pr * 68;
      float c0 = o[0], c1 = o[1], c2 = o[2];
      if (SIGMOID) { c0 = nerf_mlp::sigmoidf_(c0); c1 = nerf_mlp::sigmoidf_(c1); c2 = nerf_mlp::sigmoidf_(c2); }
      const float sg = expf(fminf(fmaxf(smem[F_SRAW + pr], -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
      reinterpret_cast<float4*>(out)[m] = make_float4(c0, c1, c2, sg);
    }
  }
}


// Density straight from world points for the production expert (occupancy-grid updates and the visibility filter's
// sigma): the hash-grid encoding of the tile's 32 rows is computed into the LDS enc tile (thread t: (row, level)
// pairs t and t + 256 — 16 levels x 2 features; the same arithmetic as hash_fwd_kernel, so the bits match the
// two-launch path) and the sigma trunk + head run on it at once: no enc round trip through HBM, and one
// workgroup's gathers overlap another's MFMAs (six per CU).
__global__ __launch_bounds__(256) void ngp_density_enc_prod_kernel(HashArgs a, const float* __restrict__ table,
                                                                   const float* __restrict__ w,
                                                                   const float* __restrict__ x, int64_t xs,
                                                                   int64_t M, float* __restrict__ sigma,
                                                                   const int32_t* __restrict__ rng = nullptr) {
  using namespace ngp_prod;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if (rng) {  // device-sized launch (nerf_ngp_density_enc_rng): rows rng[0] .. rng[1] - 1 of x and sigma
    const int64_t lo = rng[0], n = (int64_t)rng[1] - lo;
    M = n < 0 ? 0 : (n < M ? n : M);
    x += lo * xs;
    sigma += lo;
  }
  if ((int64_t)blockIdx.x * NGP_BROWS >= M) return;
  const int64_t m0 = (int64_t)blockIdx.x * NGP_BROWS;
  NgpFrag fa, fb;
  load_frag<0>(w, nullptr, wave, lane, fa);
  load_frag<1>(w, nullptr, wave, lane, fb);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int pair = tid + 256 * u, r = pair >> 4, l = pair & 15;
    const int64_t m = m0 + r;
    float2 v = make_float2(0.f, 0.f);
    if (m < M && l < a.L) {
      float p[3], acc[2];
      load_x01(a, x, xs, m, p);
      hash_level<2>(a, table, p, l, acc);
      v = make_float2(acc[0], acc[1]);
    }
    *reinterpret_cast<float2*>(smem + F_ENC + r * 36 + 2 * l) = v;
  }
  lds_barrier();
  fwd<0, F_ENC, 36, F_PA>(smem, fa, wave, lane);
  lds_barrier();
  load_frag<2>(w, nullptr, wave, lane, fa);
  fwd<1, F_PA, 68, F_PB>(smem, fb, wave, lane);
  lds_barrier();
  fwd<2, F_PB, 68, F_PA>(smem, fa, wave, lane);
  lds_barrier();
  if (tid < NGP_BROWS && m0 + tid < M) {
    const float sr = smem[F_PA + tid * 68];
    sigma[m0 + tid] = expf(fminf(fmaxf(sr, -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
  }
}

// dw = sum over the workgroup slabs.  A block owns 64 consecutive columns (16 float4) and 16 slab groups: thread
// (g, c) sums slabs g, g+16, ... of its column in order, then column c's 16 group sums are added in order g = 0..15
// (deterministic).  One thread per column over all slabs ran at 0.3 TB/s (256 dependent adds per thread).
constexpr int RED_COLS4 = 16, RED_GROUPS = 16;
template <bool VEC_OUT>
__global__ __launch_bounds__(256) void ngp_reduce_kernel(const float* __restrict__ partial, int64_t total, int nslab,
                                                         float* __restrict__ dw, int accumulate) {
  __shared__ float4 red[RED_GROUPS][RED_COLS4];
  const int c = threadIdx.x % RED_COLS4, g = threadIdx.x / RED_COLS4;
  const int64_t i4 = (int64_t)blockIdx.x * RED_COLS4 + c;  // float4 column (total % 32 == 0)
  const int64_t n4 = total / 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4) {
    const float4* p = reinterpret_cast<const float4*>(partial) + i4;
#pragma unroll 4
    for (int b = g; b < nslab; b += RED_GROUPS) {
      const float4 v = p[(int64_t)b * n4];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && i4 < n4) {
    float4 a = red[0][c];
#pragma unroll
    for (int k = 1; k < RED_GROUPS; ++k) {
      const float4 v = red[k][c];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    if (VEC_OUT) {
      float4* o = reinterpret_cast<float4*>(dw) + i4;
      if (accumulate) { const float4 d = *o; a.x = d.x + a.x; a.y = d.y + a.y; a.z = d.z + a.z; a.w = d.w + a.w; }
      *o = a;
    } else {
      float* o = dw + 4 * i4;
      const float v[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = accumulate ? o[e] + v[e] : v[e];
    }
  }
}

// dynamic LDS above 64 KB must be allowed per kernel, once per process.  Keyed by the kernel's address: the
// ngp_bwd_kernel<NSB> instantiations share one function type, so a per-type once_flag would set only the first.
template <typename K>
void allow_lds(K kernel) {
  static std::mutex mu;
  static std::set<const void*> done;
  const void* f = reinterpret_cast<const void*>(kernel);
  std::lock_guard<std::mutex> lock(mu);
  if (done.insert(f).second)
    (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
}

int bwd_grid(int64_t M) {
  const int64_t ntiles = nerf_cdiv(M, NGP_BROWS);
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
  }
  ncu *= 2;  // two workgroups per CU
  return (int)(ntiles < ncu ? (ntiles < 1 ? 1 : ntiles) : ncu);
}

// the plan is the production expert's (ngp_bwd_prod_kernel's compile-time shape and LDS layout);
// net.generic_kernels = 1 keeps the generic kernel (its reference in the tests, A/B measurements)
bool is_prod_plan(const NerfNgpNet& net, const NgpPlan& P) {
  using namespace ngp_prod;
  if (net.generic_kernels || P.nl != NL || P.head != HEAD || P.total != TOTAL || P.dir_mode != 0 || P.sh_levels != 4 ||
      P.geo != GEO || P.dir_dim != DIRD || P.in_dim > 32 || P.enc_buf != ENC || P.enc_ld != 36 ||
      P.cin_buf != CIN || P.cin_ld != 36 || P.g0 != G0 || P.g1 != G1 || P.dsig != DSIG || P.bsum != BSUM ||
      P.smem_floats != SMEM)
    return false;
  for (int l = 0; l < NL; ++l) {
    const NgpLayer& L = P.ly[l];
    if (L.Kpad != KP[l] || L.Npad != NP[l] || L.w_off != WOFF[l] || L.b_off != BOFF[l] || L.relu != RELU[l] ||
        L.in_relu != INRELU[l] || L.in_buf != INB[l] || L.in_ld != INLD[l] || L.out_buf != OUTB[l] ||
        (L.out_ld != 68))
      return false;
  }
  return true;
}

bool hash_args(const NerfHashGrid* g, const float* aabb_host_unused, HashArgs& a) {
  if (!g || g->levels < 1 || g->levels > NERF_HASH_MAX_LEVELS) return false;
  const int F = g->features_per_level;
  if (!(F == 1 || F == 2 || F == 4 || F == 8)) return false;
  if (g->log2_hashmap_size < 1 || g->log2_hashmap_size > 26) return false;
  if (g->interpolation < 0 || g->interpolation > 2) return false;
  a = HashArgs{};
  a.L = g->levels;
  a.F = F;
  a.log2T = g->log2_hashmap_size;
  a.interp = g->interpolation;
  for (int l = 0; l < a.L; ++l) {
    if (g->resolutions[l] < 1) return false;
    a.res[l] = g->resolutions[l];
  }
  return true;
}

}  // namespace

// aabb is a HOST pointer here (6 floats): the box is part of the expert's configuration, like the resolutions.
extern "C" int nerf_hash_encode(const NerfHashGrid* grid, const float* table, const float* x, int64_t x_stride,
                                int64_t M, const float* aabb, float enc_eps, float* out, int out_stride,
                                hipStream_t st) {
  HashArgs a;
  if (!hash_args(grid, nullptr, a) || M < 0 || x_stride < 3 || out_stride < a.L * a.F) return NERF_E_ARG;
  if (M == 0) return NERF_OK;
  if (!table || !x || !out) return NERF_E_ARG;
  if (aabb) {
    a.has_aabb = 1;
    for (int c = 0; c < 3; ++c) { a.mn[c] = aabb[c]; a.ext[c] = aabb[3 + c] - aabb[c]; }
    a.eps = enc_eps;
  }
  if (M == 0) return NERF_OK;
  if ((a.F == 2 || a.F == 4) && (!nerf_aligned16(table) || (out_stride % 2))) return NERF_E_ALIGN;
  const int64_t n = M * a.L;
  const unsigned blocks = (unsigned)nerf_cdiv(n, 256);
  switch (a.F) {
    case 1: hash_fwd_kernel<1><<<blocks, 256, 0, st>>>(a, table, x, x_stride, M, out, out_stride); break;
    case 2: hash_fwd_kernel<2><<<blocks, 256, 0, st>>>(a, table, x, x_stride, M, out, out_stride); break;
    case 4: hash_fwd_kernel<4><<<blocks, 256, 0, st>>>(a, table, x, x_stride, M, out, out_stride); break;
    default: hash_fwd_kernel<8><<<blocks, 256, 0, st>>>(a, table, x, x_stride, M, out, out_stride); break;
  }
  return nerf_launch_status();
}

// -DNERF_HASH_BWD_NOAGG builds the per-(sample, level) kernel without run aggregation (tools/ A/B builds)
static constexpr bool hash_bwd_aggregate() {
#ifdef NERF_HASH_BWD_NOAGG
  return false;
#else
  return true;
#endif
}

extern "C" int nerf_hash_encode_bwd(const NerfHashGrid* grid, const float* x, int64_t x_stride, int64_t M,
                                    const float* aabb, float enc_eps, const float* d_out, int d_stride,
                                    float* d_table, hipStream_t st) {
  HashArgs a;
  if (!hash_args(grid, nullptr, a) || M < 0 || x_stride < 3 || d_stride < a.L * a.F) return NERF_E_ARG;
  if (M == 0) return NERF_OK;
  if (!x || !d_out || !d_table) return NERF_E_ARG;
  if (aabb) {
    a.has_aabb = 1;
    for (int c = 0; c < 3; ++c) { a.mn[c] = aabb[c]; a.ext[c] = aabb[3 + c] - aabb[c]; }
    a.eps = enc_eps;
  }
  if (M == 0) return NERF_OK;
  const int64_t n = M * a.L;
  const unsigned blocks = (unsigned)nerf_cdiv(n, 256);
  switch (a.F) {
    case 1: hash_bwd_kernel<1><<<blocks, 256, 0, st>>>(a, x, x_stride, M, d_out, d_stride, d_table); break;
    case 2:
      if (a.interp != 0 && hash_bwd_aggregate())
        hash_bwd_f2_agg_kernel<<<(unsigned)nerf_cdiv(4 * M, 256), 256, 0, st>>>(a, x, x_stride, M, d_out, d_stride,
                                                                                d_table);
      else
        hash_bwd_f2_kernel<<<(unsigned)nerf_cdiv(4 * n, 256), 256, 0, st>>>(a, x, x_stride, M, d_out, d_stride,
                                                                            d_table);
      break;
    case 4: hash_bwd_kernel<4><<<blocks, 256, 0, st>>>(a, x, x_stride, M, d_out, d_stride, d_table); break;
    default: hash_bwd_kernel<8><<<blocks, 256, 0, st>>>(a, x, x_stride, M, d_out, d_stride, d_table); break;
  }
  return nerf_launch_status();
}

extern "C" int nerf_sh_encode(const float* d, int64_t d_stride, int64_t M, int levels, float* out, int out_stride,
                              hipStream_t st) {
  if (M < 0 || d_stride < 3 || levels < 1 || levels > 5 || out_stride < levels * levels) return NERF_E_ARG;
  if (M == 0) return NERF_OK;
  if (!d || !out) return NERF_E_ARG;
  sh_kernel<<<(unsigned)nerf_cdiv(M, 256), 256, 0, st>>>(d, d_stride, M, levels, out, out_stride);
  return nerf_launch_status();
}

extern "C" int64_t nerf_ngp_layout(const NerfNgpNet* net, int64_t* table, int32_t* n_tensors) {
  NgpPlan P;
  if (!net || !make_plan(*net, true, P)) return NERF_E_ARG;
  if (n_tensors) *n_tensors = 2 * P.nl;
  if (table) {
    for (int l = 0; l < P.nl; ++l) {
      const NgpLayer& L = P.ly[l];
      int real_k;
      if (l == 0) real_k = net->in_dim;
      else if (l <= P.head) real_k = net->hidden;
      else if (l == P.head + 1) real_k = net->geo_feat_dim + P.dir_dim;
      else real_k = net->color_hidden;
      int64_t* t = table + 8 * l;
      t[0] = L.w_off; t[1] = L.Npad; t[2] = L.Kpad; t[3] = real_k;
      t[4] = L.b_off; t[5] = L.Npad; t[6] = 1; t[7] = 1;
    }
  }
  return P.total;
}

extern "C" int64_t nerf_ngp_workspace_bytes(const NerfNgpNet* net, int64_t M) {
  NgpPlan P;
  if (!net || M < 0 || !make_plan(*net, true, P)) return NERF_E_ARG;
  return ((int64_t)bwd_grid(M) + 1) * P.total * 4 + 256;  // slabs + the W^T image
}

extern "C" int nerf_ngp_fwd(const NerfNgpNet* net, const float* w, const float* enc, int enc_stride,
                            const float* x_d, int64_t M, float* rgb_sigma, hipStream_t st) {
  NgpPlan P;
  if (!net || M < 0 || !make_plan(*net, false, P) || enc_stride < net->in_dim) return NERF_E_ARG;
  if (M == 0) return NERF_OK;
  if (!w || !enc || !x_d || !rgb_sigma) return NERF_E_ARG;
  if (!nerf_aligned16(w) || !nerf_aligned16(rgb_sigma)) return NERF_E_ALIGN;
  NgpPlan Pb;  // the production shape runs the compile-time kernel (its check is on the backward plan's layout)
  if (make_plan(*net, true, Pb) && is_prod_plan(*net, Pb)) {
    const unsigned blocks = (unsigned)nerf_cdiv(M, NGP_BROWS);
    const size_t smp = (size_t)ngp_prod::F_SMEM * 4;
    if (P.sigmoid)
      ngp_fwd_prod_kernel<0, 1><<<blocks, 256, smp, st>>>(w, enc, enc_stride, P.in_dim, x_d, M, rgb_sigma);
    else
      ngp_fwd_prod_kernel<0, 0><<<blocks, 256, smp, st>>>(w, enc, enc_stride, P.in_dim, x_d, M, rgb_sigma);
    return nerf_launch_status();
  }
  const size_t sm = (size_t)P.smem_floats * 4;
  allow_lds(ngp_fwd_kernel);
  ngp_fwd_kernel<<<(unsigned)nerf_cdiv(M, NGP_ROWS), 256, sm, st>>>(P, w, enc, enc_stride, x_d, M, rgb_sigma);
  return nerf_launch_status();
}

extern "C" int nerf_ngp_density(const NerfNgpNet* net, const float* w, const float* enc, int enc_stride, int64_t M,
                                float* sigma, hipStream_t st) {
  NgpPlan P;
  if (!net || M < 0 || !make_plan(*net, false, P) || enc_stride < net->in_dim) return NERF_E_ARG;
  if (M == 0) return NERF_OK;
  if (!w || !enc || !sigma) return NERF_E_ARG;
  if (!nerf_aligned16(w)) return NERF_E_ALIGN;
  NgpPlan Pb;
  if (make_plan(*net, true, Pb) && is_prod_plan(*net, Pb)) {
    ngp_fwd_prod_kernel<1, 0><<<(unsigned)nerf_cdiv(M, NGP_BROWS), 256, (size_t)ngp_prod::F_SMEM * 4, st>>>(
        w, enc, enc_stride, P.in_dim, nullptr, M, sigma);
    return nerf_launch_status();
  }
  const size_t sm = (size_t)P.smem_floats * 4;
  allow_lds(ngp_density_kernel);
  ngp_density_kernel<<<(unsigned)nerf_cdiv(M, NGP_ROWS), 256, sm, st>>>(P, w, enc, enc_stride, M, sigma);
  return nerf_launch_status();
}

static int ngp_density_enc_impl(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table, const float* w,
                                const float* x, int64_t x_stride, int64_t M, const int32_t* rng, const float* aabb,
                                float enc_eps, float* sigma, hipStream_t st) {
  NgpPlan P, Pb;
  HashArgs a;
  if (!net || !grid || M < 0 || x_stride < 3 || !make_plan(*net, false, P) || !hash_args(grid, nullptr, a))
    return NERF_E_ARG;
  if (a.F != 2 || a.L > 16 || a.L * a.F != net->in_dim || !make_plan(*net, true, Pb) || !is_prod_plan(*net, Pb))
    return NERF_E_UNSUPPORTED;
  if (M == 0) return NERF_OK;
  if (!table || !w || !x || !sigma) return NERF_E_ARG;
  if (!nerf_aligned16(w) || !nerf_aligned16(table)) return NERF_E_ALIGN;
  if (aabb) {
    a.has_aabb = 1;
    for (int c = 0; c < 3; ++c) { a.mn[c] = aabb[c]; a.ext[c] = aabb[3 + c] - aabb[c]; }
    a.eps = enc_eps;
  }
  ngp_density_enc_prod_kernel<<<(unsigned)nerf_cdiv(M, NGP_BROWS), 256, (size_t)ngp_prod::F_SMEM * 4, st>>>(
      a, table, w, x, x_stride, M, sigma, rng);
  return nerf_launch_status();
}

extern "C" int nerf_ngp_density_enc(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table,
                                    const float* w, const float* x, int64_t x_stride, int64_t M, const float* aabb,
                                    float enc_eps, float* sigma, hipStream_t st) {
  return ngp_density_enc_impl(net, grid, table, w, x, x_stride, M, nullptr, aabb, enc_eps, sigma, st);
}

extern "C" int nerf_ngp_density_enc_rng(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table,
                                        const float* w, const float* x, int64_t x_stride, int64_t cap,
                                        const int32_t* rng, const float* aabb, float enc_eps, float* sigma,
                                        hipStream_t st) {
  if (!rng) return NERF_E_ARG;
  return ngp_density_enc_impl(net, grid, table, w, x, x_stride, cap, rng, aabb, enc_eps, sigma, st);
}

static int ngp_fwd_enc_impl(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table, const float* w,
                            const float* x_d, int64_t M, const int32_t* rng, const float* aabb, float enc_eps,
                            float* enc, int enc_stride, float* rgb_sigma, hipStream_t st) {
  NgpPlan P, Pb;
  HashArgs a;
  if (!net || !grid || M < 0 || !make_plan(*net, false, P) || !hash_args(grid, nullptr, a)) return NERF_E_ARG;
  if (enc_stride < a.L * a.F) return NERF_E_ARG;
  if (a.F != 2 || a.L > 16 || a.L * a.F != net->in_dim || !make_plan(*net, true, Pb) || !is_prod_plan(*net, Pb))
    return NERF_E_UNSUPPORTED;
  if (M == 0) return NERF_OK;
  if (!table || !w || !x_d || !enc || !rgb_sigma) return NERF_E_ARG;
  if (!nerf_aligned16(w) || !nerf_aligned16(table) || !nerf_aligned16(rgb_sigma) || (enc_stride % 2) ||
      !nerf_aligned16(enc))
    return NERF_E_ALIGN;
  if (aabb) {
    a.has_aabb = 1;
    for (int c = 0; c < 3; ++c) { a.mn[c] = aabb[c]; a.ext[c] = aabb[3 + c] - aabb[c]; }
    a.eps = enc_eps;
  }
  const unsigned blocks = (unsigned)nerf_cdiv(M, NGP_BROWS);
  const size_t smp = (size_t)ngp_prod::F_SMEM * 4;
  if (P.sigmoid)
    ngp_fwd_prod_kernel<0, 1, true><<<blocks, 256, smp, st>>>(w, nullptr, enc_stride, P.in_dim, x_d, M, rgb_sigma, a,
                                                                table, enc, rng);
  else
    ngp_fwd_prod_kernel<0, 0, true><<<blocks, 256, smp, st>>>(w, nullptr, enc_stride, P.in_dim, x_d, M, rgb_sigma, a,
                                                                table, enc, rng);
  return nerf_launch_status();
}

extern "C" int nerf_ngp_fwd_enc(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table,
                                const float* w, const float* x_d, int64_t M, const float* aabb, float enc_eps,
                                float* enc, int enc_stride, float* rgb_sigma, hipStream_t st) {
  return ngp_fwd_enc_impl(net, grid, table, w, x_d, M, nullptr, aabb, enc_eps, enc, enc_stride, rgb_sigma, st);
}

extern "C" int nerf_ngp_fwd_enc_n(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table, const float* w,
                                  const float* x_d, int64_t cap, const int32_t* rng, const float* aabb, float enc_eps,
                                  float* enc, int enc_stride, float* rgb_sigma, hipStream_t st) {
  if (!rng) return NERF_E_ARG;
  return ngp_fwd_enc_impl(net, grid, table, w, x_d, cap, rng, aabb, enc_eps, enc, enc_stride, rgb_sigma, st);
}

extern "C" int nerf_ngp_bwd(const NerfNgpNet* net, const float* w, const float* enc, int enc_stride,
                            const float* x_d, int64_t M, const float* d_rgb_sigma, float* d_enc, float* d_w,
                            int accumulate, void* ws, int64_t ws_bytes, hipStream_t st) {
  NgpPlan P;
  if (!net || !d_w || M < 0 || !make_plan(*net, true, P) || enc_stride < net->in_dim) return NERF_E_ARG;
  if (M == 0) {
    if (!accumulate) (void)hipMemsetAsync(d_w, 0, P.total * sizeof(float), st);
    return nerf_launch_status();
  }
  if (!w || !enc || !x_d || !d_rgb_sigma || !d_enc || !ws) return NERF_E_ARG;
  if (!nerf_aligned16(w) || !nerf_aligned16(d_rgb_sigma) || !nerf_aligned16(ws)) return NERF_E_ALIGN;
  const int grid = bwd_grid(M);
  if (ws_bytes < ((int64_t)grid + 1) * P.total * 4) return NERF_E_WORKSPACE;
  const int64_t ntiles = nerf_cdiv(M, NGP_BROWS);
  const int nsbw = (P.nsb + 3) / 4;
  const size_t sm = (size_t)P.smem_floats * 4;
  float* partial = reinterpret_cast<float*>(ws);
  float* wt = partial + (int64_t)grid * P.total;
  ngp_wt_kernel<<<P.nl, 256, 0, st>>>(P, w, wt);
  if (is_prod_plan(*net, P)) {
    const size_t smp = (size_t)ngp_prod::SMEM * 4;
    if (P.sigmoid) {
      allow_lds(ngp_bwd_prod_kernel<1>);
      ngp_bwd_prod_kernel<1><<<grid, 256, smp, st>>>(w, wt, enc, enc_stride, P.in_dim, x_d, M, d_rgb_sigma, d_enc,
                                                      partial, ntiles);
    } else {
      allow_lds(ngp_bwd_prod_kernel<0>);
      ngp_bwd_prod_kernel<0><<<grid, 256, smp, st>>>(w, wt, enc, enc_stride, P.in_dim, x_d, M, d_rgb_sigma, d_enc,
                                                      partial, ntiles);
    }
  } else {
  allow_lds(ngp_bwd_kernel<4>);
  allow_lds(ngp_bwd_kernel<6>);
  allow_lds(ngp_bwd_kernel<8>);
  if (nsbw <= 4)
    ngp_bwd_kernel<4><<<grid, 256, sm, st>>>(P, w, enc, enc_stride, x_d, M, d_rgb_sigma, d_enc, partial, wt,
                                                 ntiles);
  else if (nsbw <= 6)
    ngp_bwd_kernel<6><<<grid, 256, sm, st>>>(P, w, enc, enc_stride, x_d, M, d_rgb_sigma, d_enc, partial, wt,
                                                 ntiles);
  else
    ngp_bwd_kernel<8><<<grid, 256, sm, st>>>(P, w, enc, enc_stride, x_d, M, d_rgb_sigma, d_enc, partial, wt,
                                                 ntiles);
  }
  const unsigned rblocks = (unsigned)nerf_cdiv(P.total / 4, RED_COLS4);
  if (nerf_aligned16(d_w))
    ngp_reduce_kernel<true><<<rblocks, 256, 0, st>>>(partial, P.total, grid, d_w, accumulate);
  else
    ngp_reduce_kernel<false><<<rblocks, 256, 0, st>>>(partial, P.total, grid, d_w, accumulate);
  return nerf_launch_status();
}

// nerf_ngp_bwd + nerf_hash_encode_bwd in one launch for the production shape with a linear / smoothstep F = 2 grid:
// the table gradient is scatter-added into d_table from inside the MLP backward (no d_enc in HBM).
static int ngp_bwd_hash_impl(const NerfNgpNet* net, const NerfHashGrid* hgrid, const float* w, const float* enc,
                             int enc_stride, const float* x_d, int64_t M, const int32_t* rng, const float* d_rgb_sigma,
                             const float* aabb, float enc_eps, float* d_table, float* d_w, int accumulate, void* ws,
                             int64_t ws_bytes, hipStream_t st) {
  NgpPlan P;
  HashArgs a;
  if (!net || !hgrid || !d_w || M < 0 || !make_plan(*net, true, P) || enc_stride < net->in_dim ||
      !hash_args(hgrid, nullptr, a))
    return NERF_E_ARG;
  if (a.F != 2 || a.interp == 0 || a.L > 16 || a.L * a.F != net->in_dim || !is_prod_plan(*net, P)) return NERF_E_UNSUPPORTED;
  if (M == 0) {
    if (!accumulate) (void)hipMemsetAsync(d_w, 0, P.total * sizeof(float), st);
    return nerf_launch_status();
  }
  if (!w || !enc || !x_d || !d_rgb_sigma || !d_table || !ws) return NERF_E_ARG;
  if (!nerf_aligned16(w) || !nerf_aligned16(d_rgb_sigma) || !nerf_aligned16(ws)) return NERF_E_ALIGN;
  if (aabb) {
    a.has_aabb = 1;
    for (int c = 0; c < 3; ++c) { a.mn[c] = aabb[c]; a.ext[c] = aabb[3 + c] - aabb[c]; }
    a.eps = enc_eps;
  }
  const int grid = bwd_grid(M);
  if (ws_bytes < ((int64_t)grid + 1) * P.total * 4) return NERF_E_WORKSPACE;
  const int64_t ntiles = nerf_cdiv(M, NGP_BROWS);
  float* partial = reinterpret_cast<float*>(ws);
  float* wt = partial + (int64_t)grid * P.total;
  ngp_wt_kernel<<<P.nl, 256, 0, st>>>(P, w, wt);
  const size_t smp = (size_t)ngp_prod::SMEM * 4;
  if (P.sigmoid) {
    allow_lds(ngp_bwd_prod_kernel<1, true>);
    ngp_bwd_prod_kernel<1, true><<<grid, 256, smp, st>>>(w, wt, enc, enc_stride, P.in_dim, x_d, M, d_rgb_sigma,
                                                           nullptr, partial, ntiles, a, d_table, rng);
  } else {
    allow_lds(ngp_bwd_prod_kernel<0, true>);
    ngp_bwd_prod_kernel<0, true><<<grid, 256, smp, st>>>(w, wt, enc, enc_stride, P.in_dim, x_d, M, d_rgb_sigma,
                                                           nullptr, partial, ntiles, a, d_table, rng);
  }
  const unsigned rblocks = (unsigned)nerf_cdiv(P.total / 4, RED_COLS4);
  if (nerf_aligned16(d_w))
    ngp_reduce_kernel<true><<<rblocks, 256, 0, st>>>(partial, P.total, grid, d_w, accumulate);
  else
    ngp_reduce_kernel<false><<<rblocks, 256, 0, st>>>(partial, P.total, grid, d_w, accumulate);
  return nerf_launch_status();
}

extern "C" int nerf_ngp_bwd_hash(const NerfNgpNet* net, const NerfHashGrid* hgrid, const float* w, const float* enc,
                                 int enc_stride, const float* x_d, int64_t M, const float* d_rgb_sigma,
                                 const float* aabb, float enc_eps, float* d_table, float* d_w, int accumulate,
                                 void* ws, int64_t ws_bytes, hipStream_t st) {
  return ngp_bwd_hash_impl(net, hgrid, w, enc, enc_stride, x_d, M, nullptr, d_rgb_sigma, aabb, enc_eps, d_table, d_w,
                           accumulate, ws, ws_bytes, st);
}

extern "C" int nerf_ngp_bwd_hash_n(const NerfNgpNet* net, const NerfHashGrid* hgrid, const float* w, const float* enc,
                                   int enc_stride, const float* x_d, int64_t cap, const int32_t* rng,
                                   const float* d_rgb_sigma, const float* aabb, float enc_eps, float* d_table,
                                   float* d_w, int accumulate, void* ws, int64_t ws_bytes, hipStream_t st) {
  if (!rng) return NERF_E_ARG;
  return ngp_bwd_hash_impl(net, hgrid, w, enc, enc_stride, x_d, cap, rng, d_rgb_sigma, aabb, enc_eps, d_table, d_w,
                           accumulate, ws, ws_bytes, st);
}
