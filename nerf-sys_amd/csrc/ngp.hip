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

#include "mlp_common.hpp"

// hipcc contracts a*b-c into one fma by default; the hash-grid math must round every product like the
// reference's torch ops (e.g. frac = x*res - floor(x*res) with x*res rounded first).  The pragma covers this
// file; the Makefile adds -ffp-contract=off for the HIP-header helpers (__fmul_rn, ...) inlined here.
#pragma clang fp contract(off)

typedef float ngp_f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int NGP_ROWS = 64;
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
  auto take = [&](int ld) { int b = s; s += NGP_ROWS * ld; return b; };
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
    P.dsig = s; s += NGP_ROWS;
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
  // bias-gradient partials last, only when they fit (deep nets: one wave per layer sums all rows in registers)
  if (save && (int64_t)(s + 4 * P.nl * 64) * 4 <= 160 * 1024) { P.bsum = s; s += 4 * P.nl * 64; }
  P.smem_floats = s;
  if ((int64_t)s * 4 > 160 * 1024) return false;
  // weight-gradient blocks, dealt to the 4 waves: slot sb = wave + 4 j.  In the backward a layer's wgrad blocks run
  // in the same barrier interval as its input-gradient MFMAs (wave (rb, kb) busy iff kb*32 < Kpad, Npad/2 MFMAs), so
  // each block goes to the wave with the least work in that interval (then the fewest slots used): the critical
  // MFMA chain of the production net drops from 352 to 288 per tile versus a layer-major deal.
  int nblk = 0;
  for (int l = 0; l < P.nl; ++l) nblk += (P.ly[l].Npad / 32) * (P.ly[l].Kpad / 32);
  const int per_wave = (nblk + 3) / 4;
  if (4 * per_wave > NGP_MAX_SB) return false;
  int used[4] = {0, 0, 0, 0};
  for (int i = 0; i < 4 * per_wave; ++i) P.sb_layer[i] = -1;
  for (int l = 0; l < P.nl; ++l) {
    const NgpLayer& L = P.ly[l];
    int cost[4];
    for (int w = 0; w < 4; ++w) cost[w] = ((w >> 1) * 32 < L.Kpad) ? L.Npad / 2 : 0;
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
        cost[best] += 32;  // 64 rows / 2 per MFMA
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
template <int F>
__global__ void hash_fwd_kernel(HashArgs a, const float* __restrict__ table, const float* __restrict__ x, int64_t xs,
                                int64_t M, float* __restrict__ out, int os) {
  const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t m = gid / a.L;
  const int l = (int)(gid - m * a.L);
  if (m >= M) return;
  float p[3];
  load_x01(a, x, xs, m, p);
  const float r = (float)a.res[l];
  const uint32_t mask = (1u << a.log2T) - 1u;
  const float* tb = table + ((int64_t)l << a.log2T) * F;
  float acc[F];
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
  unit3(x, y, z, 1e-9f);  // MetaNGP._enc_dir (meta_ngp.py:176-179)
  if (P.dir_mode == 0) {
    unit3(x, y, z, 1e-9f);  // SHEncoder.forward normalises again (encodings.py:141)
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

// Gnext[r][k] = sum_n G[r][n] W[n][k]  (masked by X > 0 when the input is a ReLU output).  If dst_global the
// result goes to d_enc rows m < M, columns < ncols instead of LDS.
__device__ __forceinline__ void layer_dgrad(const NgpLayer& L, float* smem, const float* __restrict__ w, int G,
                                            int Gn, int wave, int li, int lh, float* __restrict__ dst_global,
                                            int ds, int ncols, int64_t m0, int64_t M) {
  const int rb = wave & 1, kb = wave >> 1;
  if (kb * 32 >= L.Kpad) return;
  const float* Gr = smem + G + (rb * 32 + li) * 68 + 8 * lh;
  const float* Wc = w + L.w_off + kb * 32 + li;  // column k = kb*32 + li, row n = 16 s + 8 lh + t
  ngp_f32x16 acc = zero16();
  const int ns = L.Npad / 16;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s < ns) {
      const float4 g0 = *reinterpret_cast<const float4*>(Gr + 16 * s);
      const float4 g1 = *reinterpret_cast<const float4*>(Gr + 16 * s + 4);
      const float* wc = Wc + (int64_t)(16 * s + 8 * lh) * L.Kpad;
      float wv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) wv[t] = wc[(int64_t)t * L.Kpad];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[0], g0.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[1], g0.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[2], g0.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[3], g0.w, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[4], g1.x, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[5], g1.y, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[6], g1.z, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wv[7], g1.w, acc, 0, 0, 0);
    }
  }
  const int r = rb * 32 + li;
  const int k0 = kb * 32 + 4 * lh;
  if (dst_global) {
    const int64_t m = m0 + r;
    if (m < M) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = k0 + 8 * q + e;
          if (k < ncols) dst_global[m * ds + k] = acc[4 * q + e];
        }
    }
    return;
  }
  const float* X = smem + L.in_buf + r * L.in_ld + k0;
  float* Y = smem + Gn + r * 68 + k0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float v0 = acc[4 * q], v1 = acc[4 * q + 1], v2 = acc[4 * q + 2], v3 = acc[4 * q + 3];
    if (L.in_relu) {
      const float4 x = *reinterpret_cast<const float4*>(X + 8 * q);
      v0 = x.x > 0.f ? v0 : 0.f; v1 = x.y > 0.f ? v1 : 0.f; v2 = x.z > 0.f ? v2 : 0.f; v3 = x.w > 0.f ? v3 : 0.f;
    }
    *reinterpret_cast<float4*>(Y + 8 * q) = make_float4(v0, v1, v2, v3);
  }
}

// acc += G[:, nb-block]^T X[:, kb-block] over the tile's 64 rows; lane li <-> k = kb*32 + li, register
// 4q+e <-> n = nb*32 + 8q + 4lh + e.
__device__ __forceinline__ void wgrad_block(ngp_f32x16& acc, const NgpLayer& L, const float* smem, int G, int nb,
                                            int kb, int li, int lh) {
  const float* Gc = smem + G + nb * 32 + li;
  const float* Xc = smem + L.in_buf + kb * 32 + li;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int r = 16 * s + 8 * lh + t;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(Gc[r * 68], Xc[r * L.in_ld], acc, 0, 0, 0);
    }
  }
}

template <int NSB>
__global__ __launch_bounds__(256) void ngp_bwd_kernel(NgpPlan P, const float* __restrict__ w,
                                                      const float* __restrict__ enc, int es,
                                                      const float* __restrict__ x_d, int64_t M,
                                                      const float* __restrict__ gout, float* __restrict__ d_enc,
                                                      float* __restrict__ partial, int64_t ntiles) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* dsig = smem + P.dsig;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, li = lane & 31, lh = lane >> 5;
  ngp_f32x16 accw[NSB];
#pragma unroll
  for (int j = 0; j < NSB; ++j) accw[j] = zero16();
  // bias gradients: wave w sums rows 16w..16w+15 of every tile into its own LDS partial (column = lane); without
  // room for the partials (P.bsum < 0) wave l&3 sums all rows of layer l into bacc[l>>2]
  float* bsum = smem + (P.bsum >= 0 ? P.bsum : 0) + wave * P.nl * 64;
  if (P.bsum >= 0)
    for (int l = 0; l < P.nl; ++l) bsum[l * 64 + lane] = 0.f;
  float bacc[3] = {0.f, 0.f, 0.f};

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t m0 = tile * NGP_ROWS;
    forward_tile(P, smem, w, enc, es, x_d, m0, M, wave, li, lh);
    // output gradients: rgb through the sigmoid, sigma through trunc_exp (trunc_exp.py:54-57)
    const NgpLayer& Lo = P.ly[P.nl - 1];
    const NgpLayer& Lh = P.ly[P.head];
    float gc[3] = {0.f, 0.f, 0.f};
    if (threadIdx.x < NGP_ROWS) {
      const int r = threadIdx.x;
      const int64_t m = m0 + r;
      float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
      if (m < M) g = reinterpret_cast<const float4*>(gout)[m];
      const float* o = smem + Lo.out_buf + r * Lo.out_ld;
      const float gg[3] = {g.x, g.y, g.z};
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        if (P.sigmoid) {
          const float s = nerf_mlp::sigmoidf_(o[c]);
          gc[c] = gg[c] * (s * (1.0f - s));
        } else {
          gc[c] = gg[c];
        }
      }
      const float sr = smem[Lh.out_buf + r * Lh.out_ld];
      dsig[r] = g.w * expf(fminf(fmaxf(sr, -nerf_mlp::EXP_MAX), nerf_mlp::EXP_MAX));
    }
    __syncthreads();  // the raw head/out tiles alias the gradient tiles
    if (threadIdx.x < NGP_ROWS) {
      float* gr = smem + P.g0 + threadIdx.x * 68;
      gr[0] = gc[0]; gr[1] = gc[1]; gr[2] = gc[2];
      for (int c = 3; c < 32; ++c) gr[c] = 0.f;
    }
    __syncthreads();
    int G = P.g0, Gn = P.g1;
    for (int l = P.nl - 1; l >= 0; --l) {
      const NgpLayer& L = P.ly[l];
      // weight gradient blocks of this layer owned by this wave
#pragma unroll
      for (int j = 0; j < NSB; ++j) {
        const int sb = wave + 4 * j;
        if (sb < P.nsb && P.sb_layer[sb] == l) wgrad_block(accw[j], L, smem, G, P.sb_nb[sb], P.sb_kb[sb], li, lh);
      }
      if (P.bsum >= 0 && lane < L.Npad) {
        const float* gc = smem + G + (16 * wave) * 68 + lane;
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) s += gc[r * 68];
        bsum[l * 64 + lane] += s;
      } else if (P.bsum < 0 && (l & 3) == wave && lane < L.Npad) {
        float s = 0.f;
        for (int r = 0; r < NGP_ROWS; ++r) s += smem[G + r * 68 + lane];
        bacc[l >> 2] += s;
      }
      // input gradient
      const bool to_enc = (l == 0);
      layer_dgrad(L, smem, w, G, Gn, wave, li, lh, to_enc ? d_enc : nullptr, es, P.in_dim, m0, M);
      __syncthreads();
      if (l == P.head + 1) {
        // Gn holds d cin: the head's gradient is [d sigma_raw, d geo, 0...]
        if (threadIdx.x < NGP_ROWS) {
          const int r = threadIdx.x;
          const float* dc = smem + Gn + r * 68;
          float* gh = smem + G + r * 68;
          gh[0] = dsig[r];
          for (int c = 0; c < P.geo; ++c) gh[1 + c] = dc[c];
          for (int c = 1 + P.geo; c < 32; ++c) gh[c] = 0.f;
        }
        __syncthreads();
      } else {
        const int t = G; G = Gn; Gn = t;
      }
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
  const int64_t ntiles = nerf_cdiv(M, NGP_ROWS);
  int dev = 0, ncu = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ncu = v;
  }
  return (int)(ntiles < ncu ? (ntiles < 1 ? 1 : ntiles) : ncu);
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

// NERF_HASH_BWD_AGG=0 selects the per-(sample, level) kernel without run aggregation (A/B measurements)
static bool hash_bwd_aggregate() {
  static const bool on = [] {
    const char* e = getenv("NERF_HASH_BWD_AGG");
    return !(e && e[0] == '0');
  }();
  return on;
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
  return (int64_t)bwd_grid(M) * P.total * 4 + 256;
}

extern "C" int nerf_ngp_fwd(const NerfNgpNet* net, const float* w, const float* enc, int enc_stride,
                            const float* x_d, int64_t M, float* rgb_sigma, hipStream_t st) {
  NgpPlan P;
  if (!net || M < 0 || !make_plan(*net, false, P) || enc_stride < net->in_dim) return NERF_E_ARG;
  if (M == 0) return NERF_OK;
  if (!w || !enc || !x_d || !rgb_sigma) return NERF_E_ARG;
  if (!nerf_aligned16(w) || !nerf_aligned16(rgb_sigma)) return NERF_E_ALIGN;
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
  const size_t sm = (size_t)P.smem_floats * 4;
  allow_lds(ngp_density_kernel);
  ngp_density_kernel<<<(unsigned)nerf_cdiv(M, NGP_ROWS), 256, sm, st>>>(P, w, enc, enc_stride, M, sigma);
  return nerf_launch_status();
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
  if (ws_bytes < (int64_t)grid * P.total * 4) return NERF_E_WORKSPACE;
  const int64_t ntiles = nerf_cdiv(M, NGP_ROWS);
  const int nsbw = (P.nsb + 3) / 4;
  const size_t sm = (size_t)P.smem_floats * 4;
  float* partial = reinterpret_cast<float*>(ws);
  allow_lds(ngp_bwd_kernel<4>);
  allow_lds(ngp_bwd_kernel<6>);
  allow_lds(ngp_bwd_kernel<8>);
  if (nsbw <= 4)
    ngp_bwd_kernel<4><<<grid, 256, sm, st>>>(P, w, enc, enc_stride, x_d, M, d_rgb_sigma, d_enc, partial, ntiles);
  else if (nsbw <= 6)
    ngp_bwd_kernel<6><<<grid, 256, sm, st>>>(P, w, enc, enc_stride, x_d, M, d_rgb_sigma, d_enc, partial, ntiles);
  else
    ngp_bwd_kernel<8><<<grid, 256, sm, st>>>(P, w, enc, enc_stride, x_d, M, d_rgb_sigma, d_enc, partial, ntiles);
  const unsigned rblocks = (unsigned)nerf_cdiv(P.total / 4, RED_COLS4);
  if (nerf_aligned16(d_w))
    ngp_reduce_kernel<true><<<rblocks, 256, 0, st>>>(partial, P.total, grid, d_w, accumulate);
  else
    ngp_reduce_kernel<false><<<rblocks, 256, 0, st>>>(partial, P.total, grid, d_w, accumulate);
  return nerf_launch_status();
}
