"""FrequencyEncoder on the HIP kernel — models/encodings.py:387-444 of the reference.

API: forward(x (...,D)) -> (..., D*(2L + include_input)); per input dim [cos 2^0..2^{L-1} x, sin ...]
after the raw input.  No gradient w.r.t. x (the reference never differentiates sample positions on
this path); raises if one is requested.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import kernels as K


class FrequencyEncoder(nn.Module):
    def __init__(self, in_dim: int, pe_dim: int, include_input: bool = True, use_pi: bool = False):
        super().__init__()
        self.in_dim = int(in_dim)
        self.pe_dim = int(pe_dim)
        self.include_input = bool(include_input)
        self.use_pi = bool(use_pi)

    @property
    def out_dim(self) -> int:
        return self.in_dim * (2 * self.pe_dim + (1 if self.include_input else 0))

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        assert x.shape[-1] == self.in_dim, f"Expected (...,{self.in_dim}), got {tuple(x.shape)}"
        if x.requires_grad and torch.is_grad_enabled():
            raise NotImplementedError("FrequencyEncoder (HIP) has no input gradient")
        xin = x.float().contiguous()
        if self.use_pi:
            xin = xin * torch.pi
        return K.freq_encode(xin, self.pe_dim, self.include_input)
