"""Load the committed golden fixtures (tests/golden/*.npz, produced by tools/gen_golden.py)."""
import os
from collections import OrderedDict

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: torch.from_numpy(z[k].copy()) for k in z.files}


def mlp_params(prefix="w/"):
    z = load("mlp")
    return OrderedDict((k[len(prefix):], v) for k, v in z.items() if k.startswith(prefix))
