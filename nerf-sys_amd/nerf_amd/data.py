"""Ray datasets built on the GPU — the reference's DRZ data path
(adaptive_nerf/data/{image_metadata,dataset,ram_rays_dataset}.py) with its per-image ray generation on HIP.

The reference decodes each image on the CPU, builds (H*W, 8) rays with torch, masks, clamps and filters them
there (a process pool of up to 8 workers, ram_rays_dataset.py:151-204) and keeps the dataset in host RAM.
Here the host only decodes the file (PIL, as the reference) and uploads the uint8 pixels of a run of same-size
images in one copy; nerf_dataset_rays then makes every pixel's ray (directions, cam->world, AABB near/far, the
near/far override) in a count pass that writes only a keep flag, one exclusive scan places the kept rows, and
a write pass recomputes the kept rays and writes them with their colour / 255 and image index straight into the
dataset's device arrays — one host read per run. The dataset lives in HBM (32 + 12 + 4 B per ray), which is where
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

def _override_args(override):
    if override is None:
        return 0, 0.0, 0, 0.0
    no, fo = override
    # an override tuple always rewrites invalid rays to inf (ray_sampling.py:169-176), even (None, None):
    # max(near, -inf) is the identity
    return 1, (float("-inf") if no is None else float(no)), (0 if fo is None else 1), (0.0 if fo is None else float(fo))


def build_run(run, aabb_dev, center_pixels, override, dev):
    """One run of same-size images -> (rays (n,8), rgbs (n,3), img_indices (n,), kept image ids): nerf_dataset_rays
    count pass, exclusive scan, ONE host read (per-image kept counts), write pass."""
    H, W = int(run[0][0].H), int(run[0][0].W)
    n_img = len(run)
    imgs = torch.from_numpy(np.stack([np.asarray(img, dtype=np.uint8).reshape(H, W, 3) for _, img, _ in run]))
    masks = None
    if any(k is not None for _, _, k in run):
        masks = torch.stack([torch.ones(H * W, dtype=torch.bool) if k is None else k.reshape(-1).bool()
                             for _, _, k in run]).to(torch.uint8).to(dev)
    imgs = imgs.to(dev)
    c2w = torch.stack([md.c2w[:3, :4].float().reshape(12) for md, _, _ in run]).to(dev)
    intr = torch.stack([torch.as_tensor(md.intrinsics, dtype=torch.float32).reshape(4) for md, _, _ in run]).to(dev)
    ids = torch.tensor([int(md.image_index) for md, _, _ in run], dtype=torch.int32).to(dev)
    hn, nv, hf, fv = _override_args(override)
    n = n_img * H * W
    flags = torch.empty(n, dtype=torch.int32, device=dev)
    L = lib()
    args = (ptr(c2w), ptr(intr), ptr(ids), n_img, H, W, int(center_pixels), ptr(aabb_dev), hn, nv, hf, fv, ptr(imgs),
            ptr(masks))
    check(L.nerf_dataset_rays(*args, ptr(flags), None, None, None, None, stream()), "nerf_dataset_rays(count)")
    pos = exclusive_scan(flags)
    bounds = pos[:: H * W].cpu().tolist()           # n_img + 1 image boundaries (the last one = total)
    total = bounds[-1]
    rays = torch.empty((total, 8), dtype=torch.float32, device=dev)
    rgbs = torch.empty((total, 3), dtype=torch.float32, device=dev)
    idx = torch.empty((total,), dtype=torch.int32, device=dev)
    if total:
        check(L.nerf_dataset_rays(*args, None, ptr(pos), ptr(rays), ptr(rgbs), ptr(idx), stream()),
              "nerf_dataset_rays(write)")
    kept = [int(md.image_index) for (md, _, _), a, b in zip(run, bounds[:-1], bounds[1:]) if b > a]
    return rays, rgbs, idx, kept


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
        chunks, kept_ids, run, run_px = [], [], [], 0

        def flush():
            nonlocal run, run_px
            if run:
                r, c, i, k = build_run(run, aabb, center_pixels, override, dev)
                chunks.append((r, c, i))
                kept_ids.extend(k)
            run, run_px = [], 0

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
                if run and ((run[0][0].H, run[0][0].W) != (md.H, md.W) or run_px >= self.FLUSH_PIXELS):
                    flush()
                run.append((md, img.contiguous().numpy() if isinstance(img, torch.Tensor) else img, keep))
                run_px += md.H * md.W
            flush()
        if not chunks:
            self._rays = torch.zeros((0, 8), dtype=torch.float32, device=dev)
            self._rgbs = torch.zeros((0, 3), dtype=torch.float32, device=dev)
            self._img_indices = torch.zeros((0,), dtype=torch.int32, device=dev)
        elif len(chunks) == 1:
            self._rays, self._rgbs, self._img_indices = chunks[0]
        else:
            self._rays, self._rgbs, self._img_indices = (torch.cat([c[i] for c in chunks]) for i in range(3))
        self._num_images = len(kept_ids)
        self._img_unique_ids = sorted(set(kept_ids))
        if len(self) == 0:
            print("Warning: MemoryDataset ended up empty. Check masks/val logic.")

    # images of one size are built together, up to this many pixels per run (HBM scratch: 12 B / pixel)
    FLUSH_PIXELS = 1 << 26

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
