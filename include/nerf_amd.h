/*
 * nerf_amd.h — C-ABI of the MI355X (gfx950) NeRF hot-path library  libnerf_amd.so
 *
 * Every entry point is `extern "C"`, takes plain device pointers + sizes + a hipStream_t,
 * never allocates device memory, never synchronises the device, and returns an int status:
 *     0  ok
 *    <0  invalid argument (shape / alignment / enum)  — see NERF_E_* below
 *    >0  hipError_t of the failed launch (passthrough)
 * All buffers are caller-owned (PyTorch allocates them).  All floating point is fp32.
 * Thread-safe and re-entrant: no mutable global state.
 *
 * Each function names the reference interface it replaces (paths relative to
 * psklavos1/NeRF-Sys adaptive_nerf/).  INTEGRATION.md shows the ctypes binding.
 */
#ifndef NERF_AMD_H
#define NERF_AMD_H

#include <stdint.h>
#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NERF_OK 0
#define NERF_E_ARG (-1)      /* bad size / pointer */
#define NERF_E_ALIGN (-2)    /* pointer not 16-byte aligned */
#define NERF_E_ENUM (-3)     /* unknown enum value */
#define NERF_E_WORKSPACE (-4)/* workspace too small */
#define NERF_E_UNSUPPORTED (-5) /* valid arguments, but no kernel for this configuration (use the general path) */

/* ------------------------------------------------------------------ rays */

/* get_ray_directions (nerfs/ray_sampling.py:111-136) + get_rays (:50-108, _rays_cam_to_world :10-24)
 * + SceneBox.ray_aabb_intersect (nerfs/scene_box.py:45-107).
 * Pixel p of the batch is (img, row, col) = pix[3p..3p+2] (pix may be NULL: dense H*W image of
 * pose 0, row-major).  c2w: n_poses x 3 x 4 row-major.  aabb (6 floats min,max) or NULL for the
 * constant [near,far].  Writes rays (n,8) = [o, d, near, far].  If images_u8 != NULL (n_poses x H x
 * W x 3 bytes) the gathered pixel colour /255 is written to rgb_out (n,3). */
int nerf_rays_gen(const float* c2w, int n_poses, const int32_t* pix, int64_t n, int H, int W,
                  float fx, float fy, float cx, float cy, int center_pixels, float near_v, float far_v,
                  const float* aabb, float aabb_max_bound, float aabb_invalid,
                  const uint8_t* images_u8, float* rays_out, float* rgb_out, hipStream_t stream);

/* Random training batch: draws n (img,row,col) triplets with a counter-based RNG (seed) into
 * pix_out (n,3) — the data path of RamRaysDataset/DataLoader (pipelines/online_stage/runtime_adapt.py:76-86). */
int nerf_pick_pixels(int64_t n, int n_images, int H, int W, uint64_t seed, int32_t* pix_out,
                     hipStream_t stream);

/* nerf_pick_pixels with the seed seed_base + (*step_dev) * seed_mul read on the device (*step_dev: int64 step
 * counter in HBM), so a captured hipGraph draws a new batch per replay (tools/bench_container.py --graph; the
 * reference draws each batch from its host RNG, runtime_adapt.py:286-296). */
int nerf_pick_pixels_dseed(int64_t n, int n_images, int H, int W, uint64_t seed_base, uint64_t seed_mul,
                           const int64_t* step_dev, int32_t* pix_out, hipStream_t stream);

/* clamp_rays_near_far (nerfs/ray_sampling.py:139-176), in place; valid_out (n) bytes or NULL.
 * has_near/has_far select the overrides. */
int nerf_clamp_near_far(float* rays, int64_t n, int has_near, float near_v, int has_far, float far_v,
                        float eps, float invalid_value, uint8_t* valid_out, hipStream_t stream);

/* Forward-facing NDC rays (canonical NeRF; absent in the reference).  rays_in/out (n,8); output
 * near=0, far=1. */
int nerf_rays_ndc(const float* rays_in, int64_t n, int H, int W, float focal, float near_plane,
                  float* rays_out, hipStream_t stream);

/* ------------------------------------------------------------------ sampling */

/* stratified_t_vals (nerfs/ray_rendering.py:262-287).  randomized!=0 jitters each interval with u
 * (n,S) if given, else with the counter RNG (seed).  t_out (n,S). */
int nerf_sample_stratified(const float* rays, int64_t n, int S, int randomized, const float* u,
                           uint64_t seed, float* t_out, hipStream_t stream);

/* Point construction of render_rays_stratified (nerfs/ray_rendering.py:317-319):
 * x_d[r*S+s] = [o + d t, d]  (n*S, 6). */
int nerf_build_xd(const float* rays, const float* t, int64_t n, int S, float* xd_out, hipStream_t stream);

/* Hierarchical inverse-CDF resampling (canonical NeRF sample_pdf; ABSENT in the reference).
 * t (n,S) sorted coarse depths, w (n,S) coarse weights.  Draws n_imp samples from the pdf of the
 * interior weights over the S-1 t-midpoints (u (n,n_imp) in [0,1) if given, else linspace when
 * det!=0, else counter RNG(seed)), and writes the sorted union t_out (n, S+n_imp).
 * Requires S+n_imp <= 512 and S >= 3. */
int nerf_sample_pdf(const float* t, const float* w, int64_t n, int S, int n_imp, const float* u, int det,
                    uint64_t seed, float* t_out, hipStream_t stream);

/* ------------------------------------------------------------------ encoding */

/* FrequencyEncoder.torch_forward (models/encodings.py:437-444): out (n, D*(2L+inc)) with row
 * stride ld_out floats; per dim [cos 2^0..2^{L-1}, sin ...] after the optional raw input. */
int nerf_freq_encode(const float* x, int64_t n, int D, int L, int include_input, float* out, int ld_out,
                     hipStream_t stream);

/* ------------------------------------------------------------------ MLP (vanilla expert) */

/* Packed weight layout of the 8x256 NeRF MLP (models/inr/meta_vanilla.py:13-154, frequency dirs):
 * tensors (PyTorch (out,in) row-major, zero-padded):  trunk.i W (256 x Kpad_i) b(256), i=0..7 with
 * Kpad = 64 / 256 / 320 (skip, [h|enc] hidden first) ; head W (32 x 256) rows [sigma, geo0..14, 0..]
 * b(32) ; color0 W (128 x 64) cols [geo 15 | dir-enc 27 | 0] b(128) ; color1 W (32 x 128) b(32).
 * nerf_mlp_layout fills table[t*4 + {offset, rows, cols_padded, cols_real}] for t < 22 tensors
 * (order: W0,b0,...,W7,b7, Wh,bh, Wc0,bc0, Wc1,bc1) and returns the total packed floats. */
int64_t nerf_mlp_layout(int64_t* table);

/* Workspace (bytes) needed by nerf_mlp_fwd/bwd for M samples.  training!=0 keeps every
 * activation for nerf_mlp_bwd. */
int64_t nerf_mlp_workspace_bytes(int64_t M, int training);

/* expert(x_d (M,6), params) -> (M,4) [sigmoid rgb, trunc_exp sigma]  (meta_vanilla.py:123-154,
 * metamodule.py:140-156, trunc_exp.py:43-61).  w: packed weights.  ws: workspace (16B aligned).
 * M = 0 is an empty call: x_d / rgb_sigma (and the backward's d_rgb_sigma) may be null; the backward then zero-fills
 * d_w (accumulate = 0) or leaves it untouched.  The same holds for the _bf16 / _f16 entry points. */
int nerf_mlp_fwd(const float* w, const float* x_d, int64_t M, float* rgb_sigma, void* ws, int64_t ws_bytes,
                 int training, hipEvent_t* events, hipStream_t stream);

/* events: NULL, or 16 caller-created hipEvent_t recorded on `stream` around each trunk layer's GEMM
 * (events[2i], events[2i+1] bracket trunk.i) — for live per-kernel timing (bench.py roofline). */

/* Backward of nerf_mlp_fwd (autograd of the same modules).  Needs the workspace of a training
 * forward on the same x_d/w.  d_w (packed layout) is overwritten, or accumulated into if
 * accumulate!=0. */
int nerf_mlp_bwd(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                 int64_t ws_bytes, hipEvent_t* events, hipStream_t stream);
/* events: NULL, or 32 hipEvent_t: events[4i+0/1] bracket the weight-gradient GEMM of trunk.i,
 * events[4i+2/3] its input-gradient GEMM (i >= 1); events[2/3] bracket the backward tail (colour branch + head -> dZ7). */

/* nerf_mlp_bwd with the weight-gradient GEMMs on a second stream: the input-gradient chain (colour branch, head and
 * trunk dgrads) stays on `stream`; each weight-gradient GEMM runs on `wgrad_stream` behind an event recorded on
 * `stream` after the launch that produced its input; `stream` waits for `wgrad_stream` before the final split reduce,
 * so d_w is complete in `stream` order.  sync: 10 caller-created hipEvent_t (hipEventDisableTiming is fine).  The
 * workspace keeps one input-gradient buffer per trunk layer: nerf_mlp_workspace_bytes_2s(M) bytes, filled by a
 * training nerf_mlp_fwd (the forward part of it is nerf_mlp_workspace_bytes(M, 1)'s).  Same kernels, grids and split
 * slabs as nerf_mlp_bwd: d_w is bitwise equal.  The events[4i+0/1] of a weight-gradient GEMM are recorded on
 * wgrad_stream. */
int64_t nerf_mlp_workspace_bytes_2s(int64_t M);
int nerf_mlp_bwd_2s(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                    int64_t ws_bytes, hipEvent_t* events, hipStream_t stream, hipStream_t wgrad_stream, hipEvent_t* sync);

/* fp32 GEMM engine of the three calls above.  Default (flags 0, and the un-suffixed entry points): the 256-wide
 * trunk GEMMs (forward, input gradient, weight gradient) run on the bf16 matrix cores as split products — every fp32
 * operand is cut into three bf16 pieces hi + mid + lo that sum to it exactly, and the six piece products down to
 * 2^-16 of the leading one are accumulated in fp32 (v_mfma_f32_32x32x16_bf16); measured error against fp64 equals the
 * fp32 MFMA's and a sequential fp32 fmaf chain's (tools/split_probe.hip); the input-gradient GEMMs keep the small
 * products in separate accumulators (see NERF_MLP_NATIVE_DGRAD).  NERF_MLP_NATIVE_FP32 selects the
 * v_mfma_f32_16x16x4_f32 kernels instead.  Unknown flag bits: NERF_E_ENUM.  Replaces the same reference interfaces as
 * nerf_mlp_fwd / nerf_mlp_bwd (MetaNeRF forward / autograd, models/inr/meta_vanilla.py:123-154). */
#define NERF_MLP_NATIVE_FP32 1
/* NERF_MLP_NATIVE_DGRAD (backward, with the split engine): the input-gradient GEMMs on the fp32 MFMA kernels.  By
 * default they are split products too, with the five small products in accumulators of their own: the bf16 MFMA adds
 * each 16-product sum to its fp32 accumulator with one guard bit (tools/mfma_round_probe.hip), and with ONE accumulator
 * that biased the long signed input-gradient chain (weight gradients 1.3-20x the fp32 engine's error); with separate
 * small-term accumulators they are as accurate as the fp32 engine's (tests/test_gpu_split_gemm.py). */
#define NERF_MLP_NATIVE_DGRAD 2
int nerf_mlp_fwd_ex(const float* w, const float* x_d, int64_t M, float* rgb_sigma, void* ws, int64_t ws_bytes,
                    int training, int flags, hipEvent_t* events, hipStream_t stream);
int nerf_mlp_bwd_ex(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                    int64_t ws_bytes, int flags, hipEvent_t* events, hipStream_t stream);
int nerf_mlp_bwd_2s_ex(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                       int64_t ws_bytes, int flags, hipEvent_t* events, hipStream_t stream, hipStream_t wgrad_stream,
                       hipEvent_t* sync);

/* bf16 variants (BASELINE configs[2]: "bf16 MLP with fp32 compositing"): the same network, packed fp32
 * parameters, inputs and outputs as nerf_mlp_fwd/bwd; the layer GEMMs run on bf16 MFMA with fp32
 * accumulation and the activations / activation gradients live in the workspace as bf16.  The weight
 * gradient d_w is fp32.  Not bit-compatible with the fp32 path (tolerance: bf16 rounding).
 * flags (0 = the production kernels; a bitwise OR of):
 *   NERF_BF16_LAYERED_FWD  one GEMM launch per layer instead of the fused single-launch forward;
 *   NERF_BF16_LAYERED_BWD  one dgrad + one wgrad GEMM launch per layer instead of the fused per-layer backward.
 *                          The backward of a workspace must be called with the same NERF_BF16_LAYERED_BWD bit as
 *                          the training forward that filled it (the layered backward reads ReLU bitmasks that only
 *                          such a forward writes).
 * The layered launches are the bitwise references of the fused kernels (tests/test_gpu_bf16.py); unknown bits ->
 * NERF_E_ENUM.  The split counts are compile-time constants (NERF_BF16_MAX_SPLITS, NERF_BF16_NARROW_MUL). */
#define NERF_BF16_LAYERED_FWD 1
#define NERF_BF16_LAYERED_BWD 2
int64_t nerf_mlp_workspace_bytes_bf16(int64_t M, int training);
int nerf_mlp_fwd_bf16(const float* w, const float* x_d, int64_t M, float* rgb_sigma, void* ws, int64_t ws_bytes,
                      int training, int flags, hipEvent_t* events, hipStream_t stream);
int nerf_mlp_bwd_bf16(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                      int64_t ws_bytes, int flags, hipEvent_t* events, hipStream_t stream);
/* events: as for nerf_mlp_fwd / nerf_mlp_bwd. */

/* fp16 variants: the reference's AMP training loop (pipelines/online_stage/runtime_adapt.py:291-310,
 * configs/train.json "use_amp": torch.autocast(float16) + GradScaler) on the same fused kernels as the bf16 entry
 * points, with fp16 operands on v_mfma_f32_32x32x16_f16 (fp32 accumulation) and the reference's rounding points under
 * autocast (models/metamodule/metamodule.py:150-156: `inputs.matmul(weight.t()) + bias`):
 *   forward   every layer output = fp32(fp16(x16 W16^T)) + bias (fp32), ReLU, then fp16 as the next matmul's operand;
 *             the heads / colour-out pre-activations (sigma's trunc_exp input, clamp 88.72) stay fp32;
 *   backward  activation gradients fp16 (the matmul backward's fp16 outputs), weight gradients summed in fp32 and
 *             rounded to fp16 once per call (the fp16 grad of the autocast weight cast, then fp32), bias gradients
 *             fp32 sums; d_w is fp32 and accumulates in fp32 after the rounding.
 * Workspace as nerf_mlp_workspace_bytes_bf16.  flags: 0 only (no layered form; other bits NERF_E_ENUM). */
int64_t nerf_mlp_workspace_bytes_f16(int64_t M, int training);
int nerf_mlp_fwd_f16(const float* w, const float* x_d, int64_t M, float* rgb_sigma, void* ws, int64_t ws_bytes,
                     int training, int flags, hipEvent_t* events, hipStream_t stream);
int nerf_mlp_bwd_f16(const float* w, int64_t M, const float* d_rgb_sigma, float* d_w, int accumulate, void* ws,
                     int64_t ws_bytes, int flags, hipEvent_t* events, hipStream_t stream);

/* ------------------------------------------------------------------ compositing + loss */

/* volume_render (nerfs/ray_rendering.py:114-165, raw_rgb=raw_sigma=False).  rgb_sigma (n,S,4),
 * t (n,S), bg (n,3) or NULL.  Outputs rgb (n,3), depth (n), weights (n,S), acc (n).
 * Optional fused loss head (nerfs/losses.py:10-32 + color_space.py:22-66): if gt != NULL,
 * loss_sum[0] += inv_count * sum((cs(pred)-cs(gt))^2) and d_rgb (n,3) = dloss/drgb.
 * color_space: 0 linear, 1 srgb, 2 identity.  S <= 1024. */
int nerf_composite_fwd(const float* rgb_sigma, const float* t, const float* bg, int64_t n, int S,
                       float sigma_scale, float* rgb, float* depth, float* weights, float* acc,
                       const float* gt, int color_space, float inv_count, float* loss_sum, float* d_rgb,
                       hipStream_t stream);

/* Backward of volume_render: upstream grads g_rgb (n,3) [required], g_depth (n), g_acc (n),
 * g_weights (n,S) [each nullable] -> d_rgb_sigma (n,S,4). */
int nerf_composite_bwd(const float* rgb_sigma, const float* t, const float* bg, int64_t n, int S,
                       float sigma_scale, const float* g_rgb, const float* g_depth, const float* g_acc,
                       const float* g_weights, float* d_rgb_sigma, hipStream_t stream);

/* ------------------------------------------------------------------ optimiser */

/* Per-block partial sums of squares of g (n) into partials[256] (first pass of
 * clip_grad_norm_, pipelines/online_stage/runtime_adapt.py:305-307). */
int nerf_grad_sqnorm(const float* g, int64_t n, float* partials, hipStream_t stream);

/* torch.optim.Adam step (common/utils.py:16-76 param groups) over a flat buffer split into
 * n_seg segments [seg_off[i], seg_off[i+1]) with learning rate seg_lr[i] (n_seg <= 8).
 * If partials != NULL and max_norm > 0 the gradient is first scaled by
 * min(1, max_norm / (sqrt(sum(partials)) + 1e-6))  (clip_grad_norm_). step is 1-based. */
int nerf_adam(float* p, const float* g, float* m, float* v, int64_t n, const int64_t* seg_off_host,
              const double* seg_lr_host, int n_seg, double beta1, double beta2, float eps, float weight_decay,
              int step, const float* partials, float max_norm, hipStream_t stream);

/* nerf_adam with the step count read from device memory (*step_dev >= 1; the bias corrections are formed in the
 * kernel in double, as nerf_adam forms them on the host): the optimiser node of a captured train-step hipGraph. */
int nerf_adam_dstep(float* p, const float* g, float* m, float* v, int64_t n, const int64_t* seg_off_host,
                    const double* seg_lr_host, int n_seg, double beta1, double beta2, float eps, float weight_decay,
                    const int64_t* step_dev, const float* partials, float max_norm, hipStream_t stream);

/* ------------------------------------------------------------------ Instant-NGP expert */

#define NERF_HASH_MAX_LEVELS 32

/* HashGridEncoder configuration (models/encodings.py:175-270).  resolutions[l] are the integers the
 * reference computes, floor(min_res * growth**l) in fp32 (:205-209).  interpolation: 0 Nearest,
 * 1 Linear, 2 Smoothstep (:331-361).  levels*features_per_level <= 64, features_per_level in {1,2,4,8}. */
typedef struct {
  int32_t levels;
  int32_t features_per_level;
  int32_t log2_hashmap_size;
  int32_t interpolation;
  int32_t resolutions[NERF_HASH_MAX_LEVELS];
} NerfHashGrid;

/* HashGridEncoder._torch_forward (models/encodings.py:313-381) with _hash/_gather (:288-311): table
 * (levels * 2^log2 , F) fp32.  Positions x (M rows, pitch x_stride floats, first 3 used).  If aabb (HOST
 * pointer, 6 floats: min xyz, max xyz — part of the expert's configuration) is non-NULL the positions are world coordinates mapped as
 * MetaNGP._world_to_unit (models/inr/meta_ngp.py:166-169): clamp((x-min)/extent, eps, 1-eps); else x is
 * used as given.  out (M rows, pitch out_stride >= levels*F): cols [0, L*F) = [level0 f0..fF-1, level1 ...],
 * cols [L*F, out_stride) zero. */
int nerf_hash_encode(const NerfHashGrid* grid, const float* table, const float* x, int64_t x_stride, int64_t M,
                     const float* aabb, float enc_eps, float* out, int out_stride, hipStream_t stream);

/* Backward of nerf_hash_encode w.r.t. the table (autograd of the reference's gather + trilinear blend):
 * d_table += scatter of d_out (M rows, pitch d_stride).  Accumulates with fp32 atomics (the caller zeroes
 * d_table first); the order of the additions is not deterministic. */
int nerf_hash_encode_bwd(const NerfHashGrid* grid, const float* x, int64_t x_stride, int64_t M, const float* aabb,
                         float enc_eps, const float* d_out, int d_stride, float* d_table, hipStream_t stream);

/* SHEncoder.forward (models/encodings.py:133-151, components :27-81): normalise (clamp 1e-9), real SH of
 * degree levels-1 (levels 1..5) -> out (M rows, pitch out_stride >= levels^2). */
int nerf_sh_encode(const float* d, int64_t d_stride, int64_t M, int levels, float* out, int out_stride,
                   hipStream_t stream);

/* MetaNGP networks (models/inr/meta_ngp.py:75-105): sigma trunk of sigma_depth ReLU layers (hidden),
 * sigma_head (1) + geo_head (geo_feat_dim), colour MLP of color_depth ReLU layers (color_hidden) on
 * cat([geo, dir-enc]) and a 3-wide output (sigmoid if use_sigmoid_rgb).  dir_encoding: 0 spherical
 * harmonics (sh_levels), 1 FrequencyEncoder(3, 4, include_input).  Every width <= 64, 1+geo <= 32. */
typedef struct {
  int32_t in_dim;
  int32_t hidden;
  int32_t sigma_depth;
  int32_t geo_feat_dim;
  int32_t color_hidden;
  int32_t color_depth;
  int32_t dir_encoding;
  int32_t sh_levels;
  int32_t use_sigmoid_rgb;
  int32_t generic_kernels; /* 0: the compile-time production-shape kernels when the shape is MetaNGP's default (the
                              fused *_enc / bwd_hash entry points need them); 1: always the plan-driven generic
                              kernels (their reference in the tests; the fused entry points return NERF_E_UNSUPPORTED) */
} NerfNgpNet;

/* Packed parameter layout: per layer (trunk 0..sd-1, head, colour 0..cd-1, out) W (Npad x Kpad) then
 * b (Npad), PyTorch (out,in) row-major, zero padded to multiples of 32; the head's rows are [sigma, geo...].
 * table (may be NULL) receives 4 int64 per tensor {offset, rows_pad, cols_pad, cols_real}; *n_tensors the
 * tensor count.  Returns the packed float count, or <0 for an unsupported configuration. */
int64_t nerf_ngp_layout(const NerfNgpNet* net, int64_t* table, int32_t* n_tensors);

/* Workspace (bytes) of nerf_ngp_bwd for M samples (per-workgroup weight-gradient slabs). */
int64_t nerf_ngp_workspace_bytes(const NerfNgpNet* net, int64_t M);

/* MetaNGP.forward after the xyz encoding (meta_ngp.py:182-255): enc (M rows, pitch enc_stride) from
 * nerf_hash_encode, directions x_d[:,3:6] (x_d (M,6)) -> rgb_sigma (M,4).  One fused kernel: all layers
 * run on fp32 MFMA with the activations in LDS. */
int nerf_ngp_fwd(const NerfNgpNet* net, const float* w, const float* enc, int enc_stride, const float* x_d,
                 int64_t M, float* rgb_sigma, hipStream_t stream);
/* MetaNGP.density (models/inr/meta_ngp.py:192-224): sigma (M) = trunc_exp of the sigma head after the trunk;
 * the colour branch is not evaluated. */
int nerf_ngp_density(const NerfNgpNet* net, const float* w, const float* enc, int enc_stride, int64_t M,
                     float* sigma, hipStream_t stream);
/* sigma from world points in ONE launch (hash-grid encoding into LDS + sigma trunk + head; bitwise the
 * nerf_hash_encode + nerf_ngp_density pair) for the production expert shape (16 x 2 hash features, 2 x 64 sigma
 * trunk, 1 + 15 head, SH degree 4 colour input — MetaNGP's defaults); NERF_E_UNSUPPORTED for other shapes. */
/* the expert's forward in ONE launch for the production shape: hash encoding of x_d's positions into LDS (also
 * written to enc [M][enc_stride] for nerf_ngp_bwd, bitwise nerf_hash_encode's) + the fused MLP -> rgb_sigma (bitwise
 * nerf_ngp_fwd's); NERF_E_UNSUPPORTED for other shapes. */
int nerf_ngp_fwd_enc(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table, const float* w,
                     const float* x_d, int64_t M, const float* aabb, float enc_eps, float* enc, int enc_stride,
                     float* rgb_sigma, hipStream_t stream);
int nerf_ngp_density_enc(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table, const float* w,
                         const float* x, int64_t x_stride, int64_t M, const float* aabb, float enc_eps, float* sigma,
                         hipStream_t stream);

/* Backward of nerf_ngp_fwd (recomputes the forward on chip): d_enc (M rows, pitch enc_stride; cols
 * >= in_dim untouched) and d_w (packed layout; overwritten, or accumulated into if accumulate != 0). */
int nerf_ngp_bwd(const NerfNgpNet* net, const float* w, const float* enc, int enc_stride, const float* x_d,
                 int64_t M, const float* d_rgb_sigma, float* d_enc, float* d_w, int accumulate, void* ws,
                 int64_t ws_bytes, hipStream_t stream);
/* nerf_ngp_bwd + nerf_hash_encode_bwd(d_table += ...) in ONE launch for the production expert shape with a
 * Linear / Smoothstep F = 2 grid (d_enc never leaves the chip; the table scatter runs beside the MLP backward);
 * NERF_E_UNSUPPORTED otherwise.  d_table accumulates (atomics), d_w as nerf_ngp_bwd. */
int nerf_ngp_bwd_hash(const NerfNgpNet* net, const NerfHashGrid* grid, const float* w, const float* enc,
                      int enc_stride, const float* x_d, int64_t M, const float* d_rgb_sigma, const float* aabb,
                      float enc_eps, float* d_table, float* d_w, int accumulate, void* ws, int64_t ws_bytes,
                      hipStream_t stream);

/* Device-sized forms (the container's sync-free train step, meta_container.py:275-343 with the sizes never read on
 * the host): every buffer is sized for `cap` rows and the row count is read on the device from rng (int32 pair,
 * device): rows = min(rng[1] - rng[0], cap).  The grids cover the capacity; workgroups past the count exit.
 *   _fwd_enc_n / _bwd_hash_n: rows 0 .. rows - 1 of x_d / enc / rgb_sigma / d_rgb_sigma (an expert's gathered samples,
 *                             rng = that expert's dispatch offsets); ws sized by nerf_ngp_workspace_bytes(net, cap)
 *   _density_enc_rng:         rows rng[0] .. rng[1] - 1 of x and sigma (one expert's slice of a packed march) */
int nerf_ngp_fwd_enc_n(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table, const float* w,
                       const float* x_d, int64_t cap, const int32_t* rng, const float* aabb, float enc_eps, float* enc,
                       int enc_stride, float* rgb_sigma, hipStream_t stream);
int nerf_ngp_density_enc_rng(const NerfNgpNet* net, const NerfHashGrid* grid, const float* table, const float* w,
                             const float* x, int64_t x_stride, int64_t cap, const int32_t* rng, const float* aabb,
                             float enc_eps, float* sigma, hipStream_t stream);
int nerf_ngp_bwd_hash_n(const NerfNgpNet* net, const NerfHashGrid* grid, const float* w, const float* enc,
                        int enc_stride, const float* x_d, int64_t cap, const int32_t* rng, const float* d_rgb_sigma,
                        const float* aabb, float enc_eps, float* d_table, float* d_w, int accumulate, void* ws,
                        int64_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------------------------ MoE container */

/* MetaContainer._routing (models/inr/meta_container.py:97-134): distances of x[:, :3] (rows of pitch
 * x_stride) to K <= 32 centroids (HOST array K x 3) on (y,z) if cluster_2d else (x,y,z).  boundary_margin
 * > 1: soft inverse-distance weights of the experts within margin x the nearest distance; else one-hot
 * argmin.  weights (M, K) fp32. */
int nerf_moe_route(const float* x, int64_t x_stride, int64_t M, const float* centroids, int K, int cluster_2d,
                   float boundary_margin, float* weights, hipStream_t stream);
/* nerf_moe_route over `capacity` rows of which the first *m_dev (device int32) are real: rows past it get all-zero
 * weights (no expert), so a following nerf_moe_dispatch over the capacity needs no host read of the count. */
int nerf_moe_route_n(const float* x, int64_t x_stride, int64_t capacity, const int32_t* m_dev, const float* centroids,
                     int K, int cluster_2d, float boundary_margin, float* weights, hipStream_t stream);

/* Order-preserving per-expert dispatch (the `(w[:,k] > 0).nonzero()` of meta_container.py:288-296):
 * idx (up to M*K int32) receives the rows with weights[m][k] > eps, expert-major and ascending within an
 * expert; offsets (K+1 int32, device) the exclusive expert offsets.  ws: nerf_moe_dispatch_workspace_bytes. */
int64_t nerf_moe_dispatch_workspace_bytes(int64_t M, int K);
int nerf_moe_dispatch(const float* weights, int64_t M, int K, float eps, int32_t* offsets, int32_t* idx, void* ws,
                      int64_t ws_bytes, hipStream_t stream);

/* dst[i][c] = src[idx[i]][c], c < cols (the expert's x.index_select rows). */
int nerf_gather_rows(const float* src, int64_t src_stride, const int32_t* idx, int64_t n, int cols, float* dst,
                     int64_t dst_stride, hipStream_t stream);
/* Device-sized forms (see nerf_ngp_fwd_enc_n): dispatch over `cap` rows of which the first *m_dev are real; gather
 * of idx entries rng[0] .. rng[1] - 1 (rng = an expert's device offsets) into dst rows 0 .. */
int nerf_moe_dispatch_n(const float* weights, int64_t cap, const int32_t* m_dev, int K, float eps, int32_t* offsets,
                        int32_t* idx, void* ws, int64_t ws_bytes, hipStream_t stream);
int nerf_gather_rows_rng(const float* src, int64_t src_stride, const int32_t* idx, const int32_t* rng, int64_t cap,
                         int cols, float* dst, int64_t dst_stride, hipStream_t stream);

/* The mix of expert k (meta_container.py:304-318): out[idx[i]][c] += y[i][c] * weights[idx[i]][k] for the
 * n rows of the expert (rows unique within a call; call k = 0..K-1 in order for the reference's sum order;
 * one-hot weights reproduce index_copy_).  Backward: d_y[i][c] = d_out[idx[i]][c] * weights[idx[i]][k]. */
int nerf_moe_combine(const float* y, int64_t n, int C, const int32_t* idx, const float* weights, int K, int k,
                     float* out, hipStream_t stream);
int nerf_moe_combine_bwd(const float* d_out, int64_t n, int C, const int32_t* idx, const float* weights, int K,
                         int k, float* d_y, hipStream_t stream);

/* MetaContainer.background_color (meta_container.py:334-363, bg_encoding "spherical"): F.normalize(d),
 * SHEncoder(levels=4), Linear(16,H)-ReLU-Linear(H,3)-Sigmoid, H <= 64.  w packed [W1 (H,16) | b1 (H) |
 * W2 (3,H) | b2 (3)] (PyTorch layouts).  Backward: d_w (20H+3 floats, overwritten) from d_out (N,3);
 * per-workgroup slabs + deterministic reduce. */
int nerf_bg_mlp_fwd(const float* d, int64_t d_stride, int64_t N, const float* w, int H, float* out,
                    hipStream_t stream);
int64_t nerf_bg_mlp_workspace_bytes(int64_t N, int H);
int nerf_bg_mlp_bwd(const float* d, int64_t d_stride, int64_t N, const float* w, int H, const float* d_out,
                    float* d_w, void* ws, int64_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------------------------ occupancy rendering */
/* nerfacc 0.5.3 pieces the reference calls (nerfs/ray_rendering.py:349-558, models/inr/meta_ngp.py:108-145,
 * 318-443), rebuilt from the published algorithms (oracle/occ_oracle.py; nerfacc's source is not in the
 * image: PARITY UNPINNED).  Grid: levels x R^3 cells, id = l*R^3 + (ix*R + iy)*R + iz; level l covers the
 * ROI box scaled by 2^l about its centre.  Packed samples are ray-major with offsets[N+1]. */
typedef struct {
  int32_t levels;
  int32_t resolution;
  float roi[6];
} NerfOccGrid;

/* OccGridEstimator.sampling marching: per ray, t from max(near_plane, rays[:,6]) (+ u*step when stratified;
 * u (N) or the counter RNG) to min(far_plane, rays[:,7]) clipped to the outermost level; dt =
 * clamp(t*cone_angle, step, 1e10); [t, t+dt) is emitted when the cell of its midpoint is occupied, empty
 * cells are skipped on the dt lattice.  Count pass (offsets == NULL): counts[N].  Write pass: offsets (N+1)
 * from nerf_exclusive_scan_i32(counts) -> ray_idx / t0 / t1. */
int nerf_occ_march(const NerfOccGrid* grid, const uint8_t* binaries, const float* rays, int64_t N, float near_plane,
                   float far_plane, float step, float cone_angle, int stratified, const float* u, uint64_t seed,
                   int max_steps, int32_t* counts, const int32_t* offsets, int32_t* ray_idx, float* t0, float* t1,
                   hipStream_t stream);

/* nerf_occ_march for every expert of a container in one launch (render_rays_occ, nerfs/ray_rendering.py:397-422):
 * ray r is marched through expert k's grid only when it hits boxes[6k..6k+5] (_intersect_rays_aabb, :171-190).
 * grids (K), binaries (K device pointers), boxes (K x 6), steps (K): HOST arrays; K <= 8.  Count pass:
 * counts[k*N + r]; write pass: offsets (K*N+1, exclusive scan of counts) -> ray_idx (= r) / t0 / t1, so expert
 * k's samples are the contiguous range [offsets[k*N], offsets[(k+1)*N]).  Jitter: counter RNG (seed, k, r). */
int nerf_occ_march_multi(const NerfOccGrid* grids, const uint8_t* const* binaries, const float* boxes,
                         const float* steps, int K, const float* rays, int64_t N, float near_plane, float far_plane,
                         float cone_angle, int stratified, uint64_t seed, int max_steps, int32_t* counts,
                         const int32_t* offsets, int32_t* ray_idx, float* t0, float* t1, hipStream_t stream);

/* nerf_occ_march_multi with the write pass replaced by a copy.  Count pass (offsets == NULL): counts as above, and
 * the first `cap` segments [t0, t1] of pair j = k*N + r are kept in stage (K*N*cap float pairs, 8-byte aligned).
 * Emit pass (offsets given, same arguments and seed): pairs with counts[j] <= cap are copied from stage, longer
 * pairs are marched again; the output equals nerf_occ_march_multi's write pass exactly. */
int nerf_occ_march_multi_staged(const NerfOccGrid* grids, const uint8_t* const* binaries, const float* boxes,
                                const float* steps, int K, const float* rays, int64_t N, float near_plane,
                                float far_plane, float cone_angle, int stratified, uint64_t seed, int max_steps,
                                int32_t* counts, float* stage, int cap, const int32_t* offsets, int32_t* ray_idx,
                                float* t0, float* t1, hipStream_t stream);

/* nerf_occ_march_multi_staged with the jitter seed seed + (*step_dev) * seed_mul read on the device (captured
 * train-step graphs: one marching jitter stream per replay). */
int nerf_occ_march_multi_staged_dseed(const NerfOccGrid* grids, const uint8_t* const* binaries, const float* boxes,
                                      const float* steps, int K, const float* rays, int64_t N, float near_plane,
                                      float far_plane, float cone_angle, int stratified, uint64_t seed, int max_steps,
                                      int32_t* counts, float* stage, int cap, const int32_t* offsets,
                                      int32_t* ray_idx, float* t0, float* t1, const int64_t* step_dev,
                                      uint64_t seed_mul, hipStream_t stream);

/* Exclusive scan of n int32 into out[n+1] (out[n] = total); in / out 16-byte aligned. Reduce-then-scan over
 * 2048-element tiles: 3 launches, 12 B of HBM traffic per element. */
int64_t nerf_scan_workspace_bytes(int64_t n);
int nerf_exclusive_scan_i32(const int32_t* in, int64_t n, int32_t* out, void* ws, int64_t ws_bytes,
                            hipStream_t stream);

/* render_weight_from_density + accumulate_along_rays (+ background): w_i = exp(-sum_{j<i} s_j) (1-exp(-s_i)),
 * s = sigma (t1 - t0); rgb = sum w c + (1-acc) bg, depth = sum w (t0+t1)/2, acc = sum w.  rgb_sigma (M,4). */
int nerf_packed_composite_fwd(const float* rgb_sigma, const float* t0, const float* t1, const int32_t* offsets,
                              int64_t N, const float* bg, float* rgb, float* depth, float* acc, float* weights,
                              hipStream_t stream);
/* Backward: g_rgb (N,3) required; g_depth, g_acc (N), g_weights (M) nullable -> d_rgb_sigma (M,4). */
int nerf_packed_composite_bwd(const float* rgb_sigma, const float* t0, const float* t1, const int32_t* offsets,
                              int64_t N, const float* bg, const float* g_rgb, const float* g_depth, const float* g_acc,
                              const float* g_weights, float* d_rgb_sigma, hipStream_t stream);

/* render_visibility_from_density: keep[j] = T_j >= early_stop_eps && (alpha_thre <= 0 || alpha_j >= alpha_thre). */
/* nerf_packed_visibility over n_seg segments in groups of `group` consecutive segments (one group per expert of
 * a multi-expert march): segment s uses min(alpha_thre, alpha_groups[s / group]) (alpha_groups: device). */
int nerf_packed_visibility_groups(const float* t0, const float* t1, const float* sigmas, const int32_t* offsets,
                                  int64_t n_seg, int64_t group, float early_stop_eps, float alpha_thre,
                                  const float* alpha_groups, int32_t* keep, hipStream_t stream);
int nerf_packed_visibility(const float* t0, const float* t1, const float* sigmas, const int32_t* offsets, int64_t N,
                           float early_stop_eps, float alpha_thre, int32_t* keep, hipStream_t stream);
/* Compaction of the kept samples (pos = exclusive scan of keep); counts_out (N, zeroed by the caller, or NULL)
 * receives the per-ray kept counts. */
int nerf_packed_compact(const int32_t* keep, const int32_t* pos, int64_t M, const int32_t* ray_idx, const float* t0,
                        const float* t1, int32_t* ray_idx_out, float* t0_out, float* t1_out, int32_t* counts_out,
                        hipStream_t stream);

/* OccGridEstimator update: jittered points of the given cells (n,3); EMA update occs[c] = max(occs[c]*decay,
 * value) for visible cells; threshold thre[0] = min(mean(occs >= 0), occ_thre), thre[1] = mean(occs)
 * (device, no host sync); binaries = occs > thre[0]. */
int nerf_occ_cell_points(const NerfOccGrid* grid, const int32_t* cells, int64_t n, uint64_t seed, float* x,
                         hipStream_t stream);
int nerf_occ_update(float* occs, const int32_t* cells, const float* values, int64_t n, float ema_decay,
                    hipStream_t stream);
/* The cell draw of OccGridEstimator._update after warm-up (nerfacc _sample_uniform_and_occupied_cells) with no
 * host read: occ_list / pos = nerf_flag_compact / exclusive scan of the binaries (levels x cells_per_level) as
 * int32 flags.  Per level: n uniform cells, then every occupied cell if there are <= n of them (other slots
 * -1), else n draws with replacement.  cells: levels x 2n global ids; cell_points / update skip ids < 0. */
int nerf_occ_sample_cells(const int32_t* occ_list, const int32_t* pos, int levels, int64_t cells_per_level,
                          int64_t n, uint64_t seed, int32_t* cells, hipStream_t stream);
int nerf_occ_threshold(const float* occs, int64_t n, float occ_thre, float* thre_out, hipStream_t stream);
/* thre_out must hold nerf_occ_threshold_floats() floats (2 results + 16-B pad + fp64 block partials). */
int64_t nerf_occ_threshold_floats(void);
int nerf_occ_binarize(const float* occs, int64_t n, const float* thre, uint8_t* binaries, hipStream_t stream);

/* OccGridEstimator.mark_invisible_cells: cells whose centre no camera sees (K (n_cam,3,3), c2w (n_cam,3,4) RDF,
 * depth > near_plane, inside W x H) get occs = -1. */
int nerf_occ_mark_invisible(const NerfOccGrid* grid, const float* K, const float* c2w, int n_cam, int W, int H,
                            float near_plane, float* occs, hipStream_t stream);

/* nerfacc.pack_info: per-ray sample counts of a packed ray_idx (M) -> counts (N, zeroed here). */
int nerf_ray_counts(const int32_t* ray_idx, int64_t M, int64_t N, int32_t* counts, hipStream_t stream);
/* Sample points of packed intervals (render_expert_occ, ray_rendering.py:523-525): x_d[j] = [o + d t_mid, d]. */
int nerf_packed_points(const float* rays, const int32_t* ray_idx, const float* t0, const float* t1, int64_t M,
                       float* x_d, hipStream_t stream);
/* nerf_packed_points for the first *m_dev (device int32) of `capacity` rows; the rest are left untouched. */
int nerf_packed_points_n(const float* rays, const int32_t* ray_idx, const float* t0, const float* t1,
                         int64_t capacity, const int32_t* m_dev, float* x_d, hipStream_t stream);

/* Full-container occupancy rendering (render_rays_occ, nerfs/ray_rendering.py:384-481).
 * nerf_rays_aabb_hit: _intersect_rays_aabb (:171-190) of rays (N,8) with box (HOST, 6 floats) -> hit (N) int32.
 * nerf_flag_compact: idx[pos[i]] = i for flags[i] != 0 (pos = exclusive scan of flags).
 * nerf_scatter_counts: counts[hit_idx[i]] = counts_k[i] (an expert's per-ray counts on the global rays).
 * nerf_segments_union: _merge_segments_union (:193-258): per ray, the sorted distinct union of every expert's
 *   t0 and t1 boundaries (t0s / t1s / offs: HOST arrays of K <= 8 device pointers; offs[k] (N+1) per-expert
 *   offsets over the global rays) -> the segments between consecutive boundaries.  Count pass (out_off NULL)
 *   -> counts (N); write pass -> ray_idx / t0 / t1 at out_off.
 * nerf_moe_blend / _finish / _bwd: sigma and rgb blended BEFORE integration (:441-471): s += w_k sigma_k,
 *   c += (w_k sigma_k) rgb_k over the rows expert k evaluated (call in expert order), then
 *   rgb_sigma = [c / max(s, 1e-12), max(s, 1e-12)]; backward per expert -> d_y (n,4). */
int nerf_rays_aabb_hit(const float* rays, int64_t N, const float* box, int32_t* hit, hipStream_t stream);
int nerf_flag_compact(const int32_t* flags, const int32_t* pos, int64_t n, int32_t* idx, hipStream_t stream);
int nerf_scatter_counts(const int32_t* hit_idx, const int32_t* counts_k, int64_t n, int32_t* counts, hipStream_t stream);
int nerf_segments_union(const float* const* t0s, const float* const* t1s, const int32_t* const* offs, int K, int64_t N,
                        int32_t* counts, const int32_t* out_off, int32_t* ray_idx, float* t0, float* t1,
                        hipStream_t stream);
int nerf_moe_blend(const float* y, int64_t n, const int32_t* idx, const float* weights, int K, int k, float* s_acc,
                   float* c_acc, hipStream_t stream);
int nerf_moe_blend_finish(const float* s_acc, const float* c_acc, int64_t M, float* rgb_sigma, hipStream_t stream);
int nerf_moe_blend_bwd(const float* y, int64_t n, const int32_t* idx, const float* weights, int K, int k,
                       const float* s_acc, const float* rgb_sigma, const float* d_rgb_sigma, float* d_y,
                       hipStream_t stream);
/* Device-sized blend (see nerf_ngp_fwd_enc_n): y / d_y rows 0 .. rng[1] - rng[0] - 1 pair with idx entries rng[0] ..;
 * _finish_n over `cap` rows of which the first *m_dev are real. */
int nerf_moe_blend_rng(const float* y, int64_t cap, const int32_t* idx, const int32_t* rng, const float* weights, int K,
                       int k, float* s_acc, float* c_acc, hipStream_t stream);
int nerf_moe_blend_finish_n(const float* s_acc, const float* c_acc, int64_t cap, const int32_t* m_dev, float* rgb_sigma,
                            hipStream_t stream);
int nerf_moe_blend_bwd_rng(const float* y, int64_t cap, const int32_t* idx, const int32_t* rng, const float* weights,
                           int K, int k, const float* s_acc, const float* rgb_sigma, const float* d_rgb_sigma,
                           float* d_y, hipStream_t stream);

/* ------------------------------------------------------------------ meta-learning updates (§8f row 4) */

/* task_adapt's inner update (adaptive_nerf/pipelines/offline_stage/meta_core.py:61-64):
 * out_i = w_i - lr * g_i (two rounded fp32 ops, like torch) for up to 64 fast tensors in one launch.
 * w / g / out / numel are HOST arrays; g[i] NULL -> out_i = w_i (a parameter autograd left unused). */
int nerf_sgd_multi(int n_tensors, const float* const* w, const float* const* g, float* const* out,
                   const int64_t* numel, float lr, hipStream_t stream);

/* reptile_meta_update (meta_core.py:145-176): per tensor t, delta = (sum_f (fast[t*n_fast+f] - theta_t)) / n_fast
 * (summed in fast-list order) and theta_t += lr * delta, skipped when delta has a non-finite element or is all
 * zero (the reference's per-tensor guard). theta / fast / numel are HOST arrays of device pointers / sizes;
 * flags: device int32 workspace of nerf_reptile_workspace_bytes(n_tensors) bytes. */
int64_t nerf_reptile_workspace_bytes(int n_tensors);
int nerf_reptile_update(int n_tensors, float* const* theta, const float* const* fast, int n_fast,
                        const int64_t* numel, float lr, int32_t* flags, int64_t ws_bytes, hipStream_t stream);

/* ------------------------------------------------------------------ ray dataset build (§8f row 4) */

/* _process_single_image (adaptive_nerf/data/ram_rays_dataset.py:46-121) for n_images same-size (H x W) images in
 * two passes around nerf_exclusive_scan_i32 (n = n_images*H*W pixels, image-major, row-major):
 *   count pass (pos == NULL): flags[n] = keep-mask (:97-104; masks NULL = keep all) && valid after
 *     get_rays with the AABB near/far (:88-92, max_bound = invalid = 1e10) and clamp_rays_near_far (:104-106,
 *     has_near / has_far = the override; eps 1e-6, invalid -> inf);
 *   write pass (pos = exclusive scan of flags, n+1 entries): kept pixel g -> row pos[g] of out_rays (8 floats,
 *     16-byte aligned), out_rgb (3 floats, pixel / 255, :112) and out_idx (image_index[image of g], :117).
 * c2w (n_images x 12), intrinsics (n_images x 4: fx fy cx cy), image_index (n_images), aabb (6): device.
 * n_images * H * W < 2^31 (int32 row positions; RamRaysDataset builds runs of <= 2^26 pixels). */
int nerf_dataset_rays(const float* c2w, const float* intrinsics, const int32_t* image_index, int n_images, int H,
                      int W, int center_pixels, const float* aabb, int has_near, float near_v, int has_far,
                      float far_v, const uint8_t* images, const uint8_t* masks, int32_t* flags, const int32_t* pos,
                      float* out_rays, float* out_rgb, int32_t* out_idx, hipStream_t stream);

/* Library build identification (string, static). */
const char* nerf_version(void);

#ifdef __cplusplus
}
#endif
#endif /* NERF_AMD_H */
