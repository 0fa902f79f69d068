"""Shared helpers for the test-suite (models with synthetic weights, golden configs)."""
import json

import numpy as np
import torch

from yolo_hip import synth
from yolo_hip.variants import VARIANTS

# (variant, size, batch) of every forward golden in tests/golden/
FORWARD_GOLDENS = [("n", 640, 1), ("n", 320, 2), ("t", 256, 1), ("s", 256, 1), ("m", 256, 1),
                   ("l", 256, 1), ("x", 320, 1)]
GOLDEN_INPUT_SEED = 5


def golden_name(v, size, b):
    return f"forward_{v}_{size}_b{b}.npz"


def make_model(variant, fused=True):
    """Drop-in nets.nn model of a variant with the synthetic (calibrated) weights, eval mode."""
    from nets import nn

    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{variant}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    return model.fuse() if fused else model


def synth_sd(variant):
    from nets import nn
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{variant}")(80)
    return synth.synth_state_dict(model.state_dict(), seed=0)


def oracle_for(variant, dtype=torch.float64, fold_bn=True):
    from oracle.forward import Oracle
    v = VARIANTS[variant]
    return Oracle(synth_sd(variant), v.width, v.depth, v.csp, 80, dtype=dtype, fold_bn=fold_bn)


def anchor_strides(height, width):
    from oracle.forward import strides_per_anchor
    return strides_per_anchor(height, width)


def grid_unit_error(y, ref, height, width):
    """Max |Δ| of box coordinates in grid units (pixels / stride, i.e. before nets/nn.py:270's
    stride multiply) and of class scores."""
    y = torch.as_tensor(y, dtype=torch.float64)
    ref = torch.as_tensor(ref, dtype=torch.float64)
    s = anchor_strides(height, width).double()
    dbox = ((y[:, :4] - ref[:, :4]).abs() / s).max().item()
    dcls = (y[:, 4:] - ref[:, 4:]).abs().max().item()
    return dbox, dcls


def noise_floor(g, key):
    """Reference's own deviation from its float64 forward (box max px, box mean, cls max, cls mean)."""
    return np.asarray(g[key], dtype=np.float64)


def meta(g):
    return json.loads(str(g["meta"]))
