"""Host-path helper shared by the experts: a cached ``dict(named_parameters())``.

Every expert call packs its weights (``tensors()`` -> ``pack``), and the module traversal behind
``named_parameters()`` costs ~40 us per call — ~0.5 ms of host time per production container step (4 experts,
~12 packs; ``tools/cpu_profile_container.py``), on the host path that feeds the GPU after each size read.  The
parameter objects of an expert do not change between calls (``load_state_dict`` and ``.to()`` update them in
place), so the dict is kept until an attribute of the module is assigned or ``_apply`` (.to / .cuda / .float)
runs; replacing a parameter of a SUBmodule afterwards needs ``expert.drop_param_cache()``."""
import torch.nn as nn


class OwnParamCache(nn.Module):
    def own_params(self):
        c = self.__dict__.get("_own_param_cache")
        if c is None:
            c = dict(self.named_parameters())
            object.__setattr__(self, "_own_param_cache", c)
        return c

    def drop_param_cache(self):
        self.__dict__.pop("_own_param_cache", None)

    def __setattr__(self, name, value):
        self.__dict__.pop("_own_param_cache", None)
        super().__setattr__(name, value)

    def _apply(self, fn, *args, **kwargs):
        self.__dict__.pop("_own_param_cache", None)
        return super()._apply(fn, *args, **kwargs)
