"""Ray datasets built on the GPU — the reference's DRZ data path
(adaptive_nerf/data/{image_metadata,dataset,ram_rays_dataset}.py) with its per-image ray generation on HIP.

The reference decodes each image on the CPU, builds (H*W, 8) rays with torch, masks, clamps and filters them
there (a process pool of up to 8 workers, ram_rays_dataset.py:151-204) and keeps the dataset in host RAM.
Here the host only decodes the file (PIL, as the reference) and uploads the uint8 pixels; one fused kernel
(nerf_rays_gen) makes every pixel's ray with the AABB near/far and gathers its colour / 255, nerf_clamp_near_far
applies the override in place, and a keep-flag / exclusive-scan / compaction pass writes the kept rows straight
into the dataset's concatenated device arrays. The dataset lives in HBM (32 + 12 + 4 B per ray), which is where
the training loop consumes it.

Mirrors: ImageMetadata (image_metadata.py:41-121), get_image_metadata / get_metadata_item / cap_metadata /
get_meta_lookups (dataset.py:148-291), load_coordinates (dataset.py:20-24) and RamRaysDataset
(ram_rays_dataset.py:127-260) with the same constructor, item dict and validation balancing.
"""
from __future__ import annotations

from pathlib import Path
from typing import Dict, List, Optional, Tuple
from zipfile import ZipFile

import numpy as np
import torch
import torch.nn.functional as F

from ._lib import check, lib, ptr, stream
from .occupancy import exclusive_scan


class ImageMetadata:
    """image_metadata.py:41-121: one posed image of a DRZ scene (c2w (3,4) or (4,4), intrinsics [fx,fy,cx,cy])."""

    def __init__(self, image_path: Path, c2w: torch.Tensor, W: int, H: int, intrinsics: torch.Tensor,
                 image_index: int, is_val: bool = False, mask_dir: Optional[Path] = None):
        self.image_path = Path(image_path) if image_path is not None else None
        self.c2w = c2w
        self.W = W
        self.H = H
        self.intrinsics = intrinsics
        self.image_index = image_index
        self.is_val = is_val
        self.mask_path = (Path(mask_dir) / f"{self.image_path.stem}.pt") if mask_dir is not None else None

    def __repr__(self):
        return (f"ImageMetadata(path={self.image_path}, image_index={self.image_index}, W={self.W}, H={self.H}, "
                f"intrinsics={self.intrinsics.tolist()}, c2w={self.c2w.tolist()})")

    def load_image(self) -> torch.Tensor:
        """(H, W, 3) uint8 RGB; resized with LANCZOS when the file's size differs (image_metadata.py:73-78)."""
        from PIL import Image
        img = Image.open(self.image_path).convert("RGB")
        if img.size != (self.W, self.H):
            img = img.resize((self.W, self.H), Image.LANCZOS)
        return torch.from_numpy(np.array(img, dtype=np.uint8))

    def load_mask(self) -> Optional[torch.Tensor]:
        """(H, W) bool keep mask from masks/<stem>.pt (plain or zipped), nearest-resized (image_metadata.py:80-121).
        Loaded with ``weights_only=True``: a mask is a tensor, never a pickled object."""
        if self.mask_path is None or not self.mask_path.exists():
            return None
        try:
            m = torch.load(self.mask_path, map_location="cpu", weights_only=True)
        except Exception:
            with ZipFile(self.mask_path, "r") as zf:
                with zf.open(zf.namelist()[0]) as f:
                    m = torch.load(f, map_location="cpu", weights_only=True)
        if m.ndim == 1:
            if m.numel() != self.H * self.W:
                return None
            m = m.view(self.H, self.W)
        if m.ndim != 2:
            return None
        if (m.shape[0], m.shape[1]) != (self.H, self.W):
            m = F.interpolate(m[None, None].float(), size=(self.H, self.W), mode="nearest")[0, 0]
        return m.bool()


# ---------------------------------------------------------------- DRZ layout (dataset.py:148-291)

def load_coordinates(data_path) -> Tuple[torch.Tensor, float]:
    """coordinates.pt -> (origin_drb (3,), pose_scale_factor) (dataset.py:20-24)."""
    info = torch.load(Path(data_path) / "coordinates.pt", map_location="cpu", weights_only=True)
    return info["origin_drb"], info["pose_scale_factor"]


def _list_metadata_files(d: Path) -> List[Path]:
    if not d.exists() or not d.is_dir():
        return []
    return sorted((p for p in d.iterdir() if p.is_file() and p.suffix == ".pt"), key=lambda x: x.name)


def get_metadata_item(metadata_path: Path, image_index: int, scale_factor: float, is_val: bool = False,
                      mask_dir: Optional[Path] = None) -> Optional[ImageMetadata]:
    """dataset.py:257-291: <root>/metadata/<stem>.pt {W, H, c2w, intrinsics} + <root>/rgbs/<stem>.{jpg,png}."""
    image_path = None
    for ext in (".jpg", ".JPG", ".png", ".PNG"):
        cand = metadata_path.parent.parent / "rgbs" / f"{metadata_path.stem}{ext}"
        if cand.exists():
            image_path = cand
            break
    if image_path is None:
        return None
    md = torch.load(metadata_path, map_location="cpu", weights_only=True)
    return ImageMetadata(image_path, md["c2w"], int(round(md["W"] * scale_factor)), int(round(md["H"] * scale_factor)),
                         md["intrinsics"] * scale_factor, image_index, is_val, mask_dir)


def get_image_metadata(data_path, scale_factor: float, mask_dir=None,
                       only_test: bool = False) -> Tuple[List[ImageMetadata], List[ImageMetadata]]:
    """dataset.py:185-254: flat layout <root>/{metadata,rgbs} (all validation) or split layout
    <root>/{train,val|test}/metadata with image indices over the union sorted by file name."""
    root = Path(data_path)
    flat = _list_metadata_files(root / "metadata")
    if flat and (root / "rgbs").exists():
        idx = {p.name: i for i, p in enumerate(sorted(flat, key=lambda x: x.name))}
        return [], [get_metadata_item(p, idx[p.name], scale_factor, True, mask_dir) for p in flat]
    train = _list_metadata_files(root / "train" / "metadata")
    ev = _list_metadata_files(root / "val" / "metadata") or _list_metadata_files(root / "test" / "metadata")
    if train or ev:
        idx = {p.name: i for i, p in enumerate(sorted(train + ev, key=lambda x: x.name))}
        tr = [] if only_test else [get_metadata_item(p, idx[p.name], scale_factor, False, mask_dir) for p in train]
        return tr, [get_metadata_item(p, idx[p.name], scale_factor, True, mask_dir) for p in ev]
    return [], []


def cap_metadata(md_list, cap_images):
    """dataset.py:148-156."""
    if cap_images is None or cap_images <= 0 or len(md_list) <= cap_images:
        return md_list
    return [md_list[i] for i in torch.randperm(len(md_list))[:cap_images].tolist()]


def get_meta_lookups(train_md, val_md):
    """dataset.py:159-173: {image_index: {"H", "W"}} for train and val."""
    def lut(mds):
        return {m.image_index: {"H": m.H, "W": m.W} for m in mds} if mds else None
    return lut(train_md), lut(val_md)


# ---------------------------------------------------------------- GPU ray build

def _image_rays(md, img_u8_dev, mask_dev, aabb_dev, center_pixels, override):
    """Per image: fused rays + colours (HBM), clamp in place, keep flags -> (rays, rgb, flags, pos, n_kept)."""
    H, W = int(md.H), int(md.W)
    n = H * W
    dev = img_u8_dev.device
    c2w = md.c2w[:3, :4].to(dev, torch.float32).contiguous()
    fx, fy, cx, cy = [float(v) for v in md.intrinsics]
    rays = torch.empty((n, 8), dtype=torch.float32, device=dev)
    rgb = torch.empty((n, 3), dtype=torch.float32, device=dev)
    L = lib()
    check(L.nerf_rays_gen(ptr(c2w), 1, None, n, H, W, fx, fy, cx, cy, int(center_pixels), 0.0, 0.0, ptr(aabb_dev),
                          1e10, 1e10, ptr(img_u8_dev), ptr(rays), ptr(rgb), stream()), "nerf_rays_gen")
    valid = torch.empty(n, dtype=torch.uint8, device=dev)
    if override is None:
        has_n, nv, has_f, fv = 0, 0.0, 0, 0.0
    else:
        no, fo = override
        # an override tuple always rewrites invalid rays to inf (ray_sampling.py:169-176), even (None, None):
        # max(near, -inf) is the identity
        has_n, nv = 1, (float("-inf") if no is None else float(no))
        has_f, fv = (0, 0.0) if fo is None else (1, float(fo))
    check(L.nerf_clamp_near_far(ptr(rays), n, has_n, nv, has_f, fv, 1e-6, float("inf"), ptr(valid), stream()),
          "nerf_clamp_near_far")
    flags = torch.empty(n, dtype=torch.int32, device=dev)
    check(L.nerf_ray_keep_flags(ptr(valid), ptr(mask_dev), n, ptr(flags), stream()), "nerf_ray_keep_flags")
    pos = exclusive_scan(flags)
    return rays, rgb, flags, pos


class RamRaysDataset(torch.utils.data.Dataset):
    """ram_rays_dataset.py:127-233 — every kept ray of every image, resident in HBM.

    Items are dicts {"rgbs" (3), "rays" (8), "img_indices"} as in the reference (:222-229); ``batch(n, seed)``
    draws a random batch with one device gather (the DataLoader-with-shuffle of the reference's train loops).
    ``num_workers`` is accepted for signature parity; the per-image work runs on the GPU."""

    def __init__(self, metadata_items: List[ImageMetadata], center_pixels: bool, val_balancing: bool = False,
                 ray_gen_kwargs: Optional[dict] = None, num_workers: Optional[int] = None, device=None):
        super().__init__()
        if ray_gen_kwargs is None or "scene_box" not in ray_gen_kwargs:
            raise ValueError("ray_gen_kwargs must contain keys: 'scene_box' and 'near_far_override'")
        box = ray_gen_kwargs["scene_box"]
        if box is None:
            raise ValueError("Provide near/far when scene_box is None")  # get_rays without near/far (:91-92)
        override = ray_gen_kwargs.get("near_far_override", None)
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        aabb = box.aabb.reshape(6).to(dev, torch.float32).contiguous()
        chunks, kept_ids, pending, pending_px = [], [], [], 0
        with torch.no_grad():
            for md in metadata_items:
                if md is None:
                    continue
                img = md.load_image()
                if img is None:
                    continue
                if img.ndim == 3 and img.shape[0] == 3 and img.shape[-1] != 3:
                    img = img.permute(1, 2, 0)
                if img.ndim == 2 and img.shape[-1] == 3:
                    img = img.view(md.H, md.W, 3)
                if not (img.ndim == 3 and img.shape[-1] == 3) or img.numel() != md.H * md.W * 3:
                    continue
                keep = md.load_mask()
                if keep is not None and keep.ndim == 1:
                    keep = keep.view(md.H, md.W)
                if md.is_val and val_balancing:
                    if keep is None:
                        keep = torch.ones(md.H, md.W, dtype=torch.bool)
                    keep = self._apply_meganerf_val_balancing_static(keep, md.H, md.W)
                if keep is not None and int(keep.sum()) == 0:
                    continue
                img_d = img.contiguous().to(dev)
                mask_d = None if keep is None else keep.reshape(-1).to(torch.uint8).to(dev)
                rays, rgb, flags, pos = _image_rays(md, img_d, mask_d, aabb, center_pixels, override)
                pending.append((md.image_index, rays, rgb, flags, pos))
                pending_px += rays.shape[0]
                if pending_px >= self.FLUSH_PIXELS:
                    chunks.append(self._compact(pending, dev, kept_ids))
                    pending, pending_px = [], 0
            if pending or not chunks:
                chunks.append(self._compact(pending, dev, kept_ids))
        if len(chunks) == 1:
            self._rays, self._rgbs, self._img_indices = chunks[0]
        else:
            self._rays, self._rgbs, self._img_indices = (torch.cat([c[i] for c in chunks]) for i in range(3))
        total = self._rays.shape[0]
        self._num_images = len(kept_ids)
        self._img_unique_ids = sorted(set(kept_ids))
        if total == 0:
            print("Warning: MemoryDataset ended up empty. Check masks/val logic.")

    # per-image full-resolution ray buffers (44 B / pixel) are compacted once this many pixels are pending
    FLUSH_PIXELS = 1 << 26

    @staticmethod
    def _compact(pending, dev, kept_ids):
        """One host read of the pending images' kept counts, then compaction into one set of arrays."""
        counts = torch.stack([p[4][-1] for p in pending]).cpu().tolist() if pending else []
        total = int(sum(counts))
        rays_o = torch.empty((total, 8), dtype=torch.float32, device=dev)
        rgbs_o = torch.empty((total, 3), dtype=torch.float32, device=dev)
        idx_o = torch.empty((total,), dtype=torch.int32, device=dev)
        o = 0
        for (iid, rays, rgb, flags, pos), c in zip(pending, counts):
            if c == 0:  # no valid ray: the image is dropped (ram_rays_dataset.py:107-108)
                continue
            check(lib().nerf_rays_compact(ptr(rays), ptr(rgb), ptr(flags), ptr(pos), rays.shape[0], int(iid),
                                          ptr(rays_o[o:]), ptr(rgbs_o[o:]), ptr(idx_o[o:]), stream()),
                  "nerf_rays_compact")
            o += c
            kept_ids.append(int(iid))
        return rays_o, rgbs_o, idx_o

    def __len__(self) -> int:
        return self._rgbs.shape[0]

    def __getitem__(self, idx) -> Dict[str, torch.Tensor]:
        return {"rgbs": self._rgbs[idx], "rays": self._rays[idx], "img_indices": self._img_indices[idx]}

    def batch(self, n: int, seed: int) -> Dict[str, torch.Tensor]:
        """A random batch of n rays (with replacement), drawn and gathered on the device."""
        g = torch.Generator(device=self._rays.device).manual_seed(int(seed))
        idx = torch.randint(0, len(self), (n,), device=self._rays.device, generator=g)
        return self[idx]

    @staticmethod
    def _apply_meganerf_val_balancing_static(keep_mask: torch.Tensor, H: int, W: int) -> torch.Tensor:
        """ram_rays_dataset.py:236-260 (host: a per-image mask edit with a torch.randperm draw)."""
        keep_mask = keep_mask.reshape(H, W).clone()
        left = keep_mask[:, : W // 2]
        n_right = int(keep_mask[:, W // 2:].sum())
        if n_right > 0:
            cand = torch.arange(H * W, device=keep_mask.device).view(H, W)[:, : W // 2][~left]
            if cand.numel() > 0:
                add = cand[torch.randperm(cand.numel(), device=keep_mask.device)[:n_right]]
                flat = keep_mask.view(-1)
                flat.scatter_(0, add, torch.ones_like(add, dtype=torch.bool))
                keep_mask = flat.view(H, W)
        keep_mask[:, W // 2:] = False
        return keep_mask.reshape(-1).bool()
