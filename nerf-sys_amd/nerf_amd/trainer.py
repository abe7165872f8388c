"""Fused NeRF training engine on flat packed buffers — the benchmarked train step.

Same step as the reference's plain train loop (pipelines/online_stage/runtime_adapt.py:278-313):
rays -> render (coarse 64 stratified + fine 64+128 hierarchical) -> MSE (linear colour space,
coarse + fine terms) -> backward -> clip_grad_norm_(1.0) -> Adam (per-group lr, common/utils.py:16-76),
but every stage is a HIP launch on one stream with no host synchronisation:

  pick_pixels+rays_gen(+gt gather) -> sample_stratified -> build_xd -> mlp_fwd(coarse)
  -> composite_fwd(+loss, dL/drgb) -> sample_pdf -> build_xd -> mlp_fwd(fine) -> composite_fwd(+loss)
  -> composite_bwd -> mlp_bwd(fine) -> composite_bwd -> mlp_bwd(coarse)
  -> [RCCL all_reduce(SUM) of the flat gradient (+ loss) buffer, data parallel: the coarse net's bucket as soon as
      its side-stream backward ends, the fine net's + loss after the fine backward]
  -> grad_sqnorm -> adam

Both networks live in ONE flat fp32 buffer [coarse | fine] (kernel packed layout), so the data-parallel
exchange is a single all-reduce of ~4 MB per step; the loss normaliser is 1/(3 N_global), so a SUM
all-reduce yields exactly the global-batch mean gradient.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import kernels as K
from .dp import allreduce_flat, inv_count as _inv_count
from .vanilla import PackedLayout, VanillaNeRF

_CS = ("linear", "srgb", "identity")
ENGINE_PRECISIONS = ("fp32", "bf16")


class RayBatcher:
    """Random pixel batches from images resident in HBM (uint8) -> rays (N,8) + gt (N,3)."""

    def __init__(self, scene, device):
        self.scene = scene
        self.poses = scene.poses.to(device).float().contiguous()
        self.images = scene.images.to(device).contiguous()
        self.device = device

    def batch(self, n, seed, shard=None, step_dev=None, seed_mul=0):
        """n random pixels from the counter RNG stream ``seed``.  ``shard=(rank, world)`` keeps the rank-strided
        slice pix[rank::world] of that draw (an/scripts/create_clusters.py:799), so every world size sees
        the same global batch (strong scaling).  ``step_dev`` (int64 device counter): the stream is
        seed + step_dev * seed_mul, read on the device (captured train-step graphs, graph_step.py)."""
        s = self.scene
        pix = K.pick_pixels(n, self.poses.shape[0], s.H, s.W, seed, self.device, step_dev=step_dev,
                            seed_mul=seed_mul)
        if shard is not None and shard[1] > 1:
            pix = pix[shard[0]::shard[1]].contiguous()
        fx, fy, cx, cy = s.intrinsics
        rays, gt = K.rays_gen(self.poses, s.H, s.W, fx, fy, cx, cy, pix=pix, near=s.near if not s.ndc else 0.0,
                              far=s.far if not s.ndc else 1.0, images_u8=self.images)
        if s.ndc:
            rays = K.rays_ndc(rays, s.H, s.W, s.focal, 1.0)
        return rays, gt


class NeRFTrainer:
    def __init__(self, coarse: VanillaNeRF, fine: Optional[VanillaNeRF] = None, *, n_samples: int = 64,
                 n_importance: int = 128, lr_sigma: float = 2e-3, lr_color: float = 2e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, grad_clip: Optional[float] = 1.0,
                 color_space: str = "linear", bg: str = "white", sigma_scale: float = 1.0,
                 world_size: int = 1, device="cuda", overlap: bool = True, precision: str = "fp32",
                 overlap_with: str = "bwd", bf16_flags: int = 0, split_wgrad: bool = False,
                 fp32_gemm: str = "split"):
        L = PackedLayout.get()
        self.L = L
        self.P = L.total
        self.nets = [coarse] + ([fine] if fine is not None else [])
        self.n_nets = len(self.nets)
        self.device = torch.device(device)
        P = self.P
        with torch.no_grad():
            self.params = torch.cat([n.packed().detach().to(self.device) for n in self.nets]).contiguous()
        # grads + 1 trailing float for the loss, all-reduced together
        self.gbuf = torch.zeros(self.n_nets * P + 4, dtype=torch.float32, device=self.device)
        self.grads = self.gbuf[: self.n_nets * P]
        self.loss_buf = self.gbuf[self.n_nets * P: self.n_nets * P + 1]
        self.m = torch.zeros_like(self.params)
        self.v = torch.zeros_like(self.params)
        self.partials = torch.empty(256, dtype=torch.float32, device=self.device)
        cs = L.color_start
        self.seg_off, self.seg_lr = [0], []
        for k in range(self.n_nets):
            self.seg_off += [k * P + cs, (k + 1) * P]
            self.seg_lr += [lr_sigma, lr_color]
        self.S, self.n_imp = n_samples, n_importance
        # fp32 (configs[1]) or bf16 (configs[2]); compositing stays fp32.  The fp16 build of the MLP kernels
        # (K.PRECISIONS has "fp16") is the reference's autocast(float16) loop on the drop-in surface, where
        # GradScaler supplies the loss scale and the inf/nan step skip; this engine has neither, so unscaled
        # ~1/(3 N) gradients would underflow in its fp16 backward: refused here
        if precision not in ENGINE_PRECISIONS:
            raise ValueError(f"precision must be one of {ENGINE_PRECISIONS} (fp16 runs only under autocast + "
                             f"GradScaler on the drop-in render_rays / VanillaNeRF surface)")
        self.precision = precision
        self.bf16_flags = int(bf16_flags)  # K.BF16_LAYERED_* (A/B runs of the layered bf16 launches)
        # fp32 trunk GEMMs: "split" = every trunk GEMM as bf16 piece products (gemm_x6.hpp; the input gradients with
        # separate small-term accumulators), the default; "native_dgrad" = input gradients on the fp32 MFMA;
        # "native" = every GEMM on the fp32 MFMA kernels
        flags = {"split": 0, "native_dgrad": K.MLP_NATIVE_DGRAD, "native": K.MLP_NATIVE_FP32}
        if fp32_gemm not in flags:
            raise ValueError(f"fp32_gemm must be one of {sorted(flags)}, got {fp32_gemm!r}")
        self.fp32_gemm = fp32_gemm
        self.fp32_flags = flags[fp32_gemm]
        self.betas, self.eps, self.wd = betas, eps, weight_decay
        self.grad_clip = grad_clip
        if color_space not in _CS:
            raise ValueError(f"Invalid color_space={color_space!r}")
        self.color_space = color_space
        if bg not in ("white", "black", "none"):
            raise ValueError("trainer background must be 'white', 'black' or 'none'")
        self.bg_policy = bg
        self.sigma_scale = sigma_scale
        self.world_size = world_size
        # False only for the bench's exposed-exchange measurement (bench.py dp record): the step then skips the
        # all-reduce, so each rank applies its own gradient — a timing device, never a training mode
        self.exchange_enabled = True
        self.step_count = 0
        self._ws = {}
        self._bg = {}
        self.timing = None  # dict of event lists when timing is enabled
        # coarse-net backward on a second HIP stream, concurrent with the fine net's forward/backward
        # (independent work once the coarse forward and its loss head are done; two nets only, since a
        # shared net accumulates both passes into one gradient segment).  Measured on MI355X (C2 step):
        # 28.1-28.5 ms vs 29.6 ms on one stream; joining the streams before the fine backward instead of at
        # the end of the step serialises it (34.2 ms); stream priorities change nothing.
        self.overlap = bool(overlap) and self.n_nets == 2 and self.device.type == "cuda"
        # what the coarse backward runs beside: the fine backward (default) or the fine forward (overlap_with="fwd").
        # Measured on MI355X with the round-6 kernels, three alternated rounds on one box (profiles/r06/overlap_ab.txt):
        # bf16 (C3) 4.51-4.53 ms beside the backward vs 4.66-4.67 beside the forward and 4.66-4.68 on one stream; fp32
        # (C2) 17.10-17.13 vs 17.15 vs 17.32-17.34 ms.  The fused bf16 forward is one persistent launch holding every
        # CU's LDS: the coarse layer backward beside it got the CUs only between its tiles (1.08 ms for a 0.10 ms
        # launch) and slowed it by 0.16 ms; beside the fine layer backward (byte-bound, one workgroup pair per split)
        # the coarse launches fill the CUs' idle issue slots.  (Rounds 2-3, on the earlier kernels, measured the
        # opposite: fp32 27.4 (fwd) vs 28.4 ms (bwd), bf16 7.30 vs 7.36 ms.)
        if overlap_with not in ("fwd", "bwd"):
            raise ValueError("overlap_with must be 'fwd' or 'bwd'")
        self.overlap_with = overlap_with
        self._side = torch.cuda.Stream(device=self.device) if self.overlap else None
        # fp32, opt-in: the fine net's weight-gradient GEMMs on their own stream beside its input-gradient chain
        # (nerf_mlp_bwd_2s: bitwise the one-stream gradient).  Measured on MI355X (C2, two A/B rounds on one box):
        # 152.3k / 152.2k rays/s against 151.9k / 152.0k in line — both chains are MFMA-bound at ~0.8 busy and
        # share the CUs, so the overlap buys ~0.2 % for 6.4 GB more workspace; off by default.
        self.split_wgrad = bool(split_wgrad) and precision == "fp32" and self.device.type == "cuda"
        if self.split_wgrad:
            self._wg = torch.cuda.Stream(device=self.device)
            self._wg_sync = [torch.cuda.Event() for _ in range(10)]
            for e in self._wg_sync:
                e.record()  # materialise the handles

    # ---- helpers
    def w(self, k):
        return self.params[k * self.P:(k + 1) * self.P]

    def g(self, k):
        return self.grads[k * self.P:(k + 1) * self.P]

    def _workspace(self, key, M, two_stream=False):
        ws = self._ws.get(key)
        need = K.mlp_workspace_bytes_2s(M) if two_stream else K.mlp_workspace_bytes(M, 1, self.precision)
        if ws is None or ws.numel() < need:
            ws = torch.empty(need, dtype=torch.uint8, device=self.device)
            self._ws[key] = ws
        return ws

    def _background(self, n):
        if self.bg_policy == "none":
            return None
        b = self._bg.get(n)
        if b is None:
            b = torch.full((n, 3), 1.0 if self.bg_policy == "white" else 0.0, device=self.device)
            self._bg[n] = b
        return b

    def enable_timing(self, n_steps: int = 1, skip: int = 0):
        """Pre-create one set of HIP events per instrumented step (no host sync inside the timed steps): the
        library records them around the fine net's trunk GEMM launches of the n_steps steps that follow the next
        `skip` steps.  Each recorded event costs the stream ~10-25 us (a gap before the next launch), so a bench
        instruments a few of its timed steps, not all of them."""
        if n_steps <= 0:
            self.timing = None
            return
        mk = lambda k: [torch.cuda.Event(enable_timing=True) for _ in range(k)]
        sets = [{"fwd": mk(16), "bwd": mk(32), "ar": mk(4)} for _ in range(n_steps)]
        for st in sets:
            for e in st["fwd"] + st["bwd"] + st["ar"]:
                e.record()  # materialise the event handles
        torch.cuda.synchronize()
        self.timing = {"pool": sets, "used": [], "M": None, "skip": int(skip)}

    def enable_exchange_timing(self, n_steps: int):
        """HIP events around the all-reduce buckets only (no GEMM events), for n_steps steps run as in production
        (the coarse backward and its bucket on the side stream): collect_exchange_timing() then gives each step's
        bucket times.  The kernel-timing pass (enable_timing) runs without the side stream, so its steps have ONE
        exchange of the whole buffer."""
        mk = lambda k: [torch.cuda.Event(enable_timing=True) for _ in range(k)]
        sets = [{"fwd": None, "bwd": None, "ar": mk(4)} for _ in range(max(0, n_steps))]
        for st in sets:
            for e in st["ar"]:
                e.record()
        torch.cuda.synchronize()
        self.timing = {"pool": sets, "used": [], "M": None, "skip": 0} if sets else None

    def collect_exchange_timing(self):
        """[[bucket-0 ms or None, bucket-1 ms or None] per step] of the enable_exchange_timing steps."""
        out = []
        for ev in self.timing["used"]:
            used = ev.get("ar_used", 0)
            out.append([ev["ar"][2 * b].elapsed_time(ev["ar"][2 * b + 1]) if used >> b & 1 else None for b in range(2)])
        self.timing = None
        return out

    def _next_events(self):
        if not self.timing or not self.timing["pool"]:
            return None
        if self.timing["skip"] > 0:
            self.timing["skip"] -= 1
            return None
        ev = self.timing["pool"].pop(0)
        self.timing["used"].append(ev)
        return ev

    # ---- the step
    def step(self, rays: torch.Tensor, gt: torch.Tensor, seed: int, u_strat=None, u_pdf=None) -> torch.Tensor:
        """One train step on this rank's rays; returns the (global) loss as a device scalar.
        u_strat (N,S) / u_pdf (N,n_importance) replace the in-kernel RNG (parity tests)."""
        N = rays.shape[0]
        S, NI = self.S, self.n_imp
        bg = self._background(N)
        inv_count = _inv_count(N, self.world_size)
        self.gbuf.zero_()
        fine_k = 1 if self.n_nets > 1 else 0
        # coarse forward
        t_c = K.sample_stratified(rays, S, True, u_strat, seed)
        xd_c = K.build_xd(rays, t_c)
        ws_c = self._workspace("c", N * S)
        rs_c = K.mlp_fwd(self.w(0), xd_c, ws_c, True, precision=self.precision, bf16_flags=self.bf16_flags,
                          fp32_flags=self.fp32_flags)
        _, _, w_c, _, _, drgb_c = K.composite_fwd(rs_c, t_c, bg, self.sigma_scale, gt=gt,
                                                  color_space=self.color_space, inv_count=inv_count,
                                                  loss_sum=self.loss_buf)
        side_done = None
        P = self.P
        ev_box = [self._next_events() if NI > 0 else None]  # HIP events of this step (timed steps only)

        def coarse_bwd_on_side():
            main = torch.cuda.current_stream(self.device)
            fork = torch.cuda.Event()
            fork.record(main)
            self._side.wait_event(fork)
            with torch.cuda.stream(self._side):
                d_rs_c = K.composite_bwd(rs_c, t_c, bg, drgb_c, sigma_scale=self.sigma_scale)
                K.mlp_bwd(self.w(0), N * S, d_rs_c, ws_c, d_w=self.g(0), accumulate=False, precision=self.precision,
                          bf16_flags=self.bf16_flags,
                          fp32_flags=self.fp32_flags)
                # bucket 1 of the data-parallel exchange: the coarse net's gradient is final here, so its all-reduce
                # starts now and runs beside the rest of the fine net's pass (bucket 2 trails the backward)
                self._exchange(self.gbuf[:P], ev_box[0], 0)
                done = torch.cuda.Event()
                done.record(self._side)
            return done

        if self.overlap and NI > 0 and self.overlap_with == "fwd":
            side_done = coarse_bwd_on_side()
        if NI > 0:
            t_f = K.sample_pdf(t_c, w_c, NI, u=u_pdf, det=False, seed=seed ^ 0x5EED)
            xd_f = K.build_xd(rays, t_f)
            ws_f = self._workspace("f", N * (S + NI), two_stream=self.split_wgrad)
            ev = ev_box[0]
            rs_f = K.mlp_fwd(self.w(fine_k), xd_f, ws_f, True, events=ev["fwd"] if ev and ev["fwd"] else None,
                             precision=self.precision, bf16_flags=self.bf16_flags,
                          fp32_flags=self.fp32_flags)
            if self.overlap and self.overlap_with == "bwd":
                side_done = coarse_bwd_on_side()
            _, _, _, _, _, drgb_f = K.composite_fwd(rs_f, t_f, bg, self.sigma_scale, gt=gt,
                                                    color_space=self.color_space, inv_count=inv_count,
                                                    loss_sum=self.loss_buf)
            d_rs_f = K.composite_bwd(rs_f, t_f, bg, drgb_f, sigma_scale=self.sigma_scale)
            K.mlp_bwd(self.w(fine_k), N * (S + NI), d_rs_f, ws_f, d_w=self.g(fine_k), accumulate=False,
                      events=ev["bwd"] if ev and ev["bwd"] else None, precision=self.precision, bf16_flags=self.bf16_flags,
                      fp32_flags=self.fp32_flags, wgrad_stream=self._wg if self.split_wgrad else None,
                      sync=self._wg_sync if self.split_wgrad else None)
            if ev:
                self.timing["M"] = N * (S + NI)
        if side_done is not None:
            torch.cuda.current_stream(self.device).wait_event(side_done)
            self._exchange(self.gbuf[P:], ev_box[0], 1)   # bucket 2: fine gradient + loss
        else:
            d_rs_c = K.composite_bwd(rs_c, t_c, bg, drgb_c, sigma_scale=self.sigma_scale)
            K.mlp_bwd(self.w(0), N * S, d_rs_c, ws_c, d_w=self.g(0), accumulate=(fine_k == 0 and NI > 0),
                      precision=self.precision, bf16_flags=self.bf16_flags,
                          fp32_flags=self.fp32_flags)
            self._exchange(self.gbuf, ev_box[0], 1)
        self.step_count += 1
        if self.grad_clip is not None and self.grad_clip > 0:
            K.grad_sqnorm(self.grads, self.partials)
            parts, mx = self.partials, float(self.grad_clip)
        else:
            parts, mx = None, 0.0
        K.adam(self.params, self.grads, self.m, self.v, self.seg_off, self.seg_lr, self.step_count, self.betas,
               self.eps, self.wd, parts, mx)
        return self.loss_buf

    def _exchange(self, buf, ev, bucket):
        """SUM all-reduce of one bucket of the flat [grad_coarse | grad_fine | loss] buffer over RCCL, issued with
        async_op=True and waited on the current (consuming) stream; with timing events, events["ar"][2 bucket] is
        recorded before the issue and [2 bucket + 1] after work.wait() on the same stream, so the pair brackets the
        collective as that stream sees it (RCCL: its stream waits for the RCCL kernel; gloo rehearsal: the host copy
        round trip), including the wait for the slowest rank."""
        if self.world_size <= 1 or not self.exchange_enabled:
            return
        cur = torch.cuda.current_stream(self.device)
        if ev:
            ev["ar"][2 * bucket].record(cur)
        work = allreduce_flat(buf, self.world_size, async_op=True)
        if work is not None:
            work.wait()
        if ev:
            ev["ar"][2 * bucket + 1].record(cur)
            ev["ar_used"] = ev.get("ar_used", 0) | (1 << bucket)

    def collect_timing(self):
        """Per-launch durations (ms) of the fine net's trunk GEMMs over every timed step:
        {"fwd": [[8 layers] per step], "wgrad": [[8]], "dgrad": [[7: layers 1..7]], "dgrad_head": [1 per step],
        "M": samples}."""
        out = {"fwd": [], "wgrad": [], "dgrad": [], "dgrad_head": [], "M": self.timing["M"]}
        for ev in self.timing["used"]:
            out["fwd"].append([ev["fwd"][2 * i].elapsed_time(ev["fwd"][2 * i + 1]) for i in range(8)])
            out["wgrad"].append([ev["bwd"][4 * i].elapsed_time(ev["bwd"][4 * i + 1]) for i in range(8)])
            out["dgrad"].append([ev["bwd"][4 * i + 2].elapsed_time(ev["bwd"][4 * i + 3]) for i in range(1, 8)])
            out["dgrad_head"].append(ev["bwd"][2].elapsed_time(ev["bwd"][3]))  # head -> trunk.7 input gradient
            used = ev.get("ar_used", 0)
            out.setdefault("allreduce", []).append([ev["ar"][2 * b].elapsed_time(ev["ar"][2 * b + 1])
                                                    for b in range(2) if used >> b & 1])
        return out

    @torch.no_grad()
    def sync_to_modules(self):
        for k, net in enumerate(self.nets):
            vals = self.L.unpack(self.w(k))
            for n, p in net.named_parameters():
                p.copy_(vals[n])
