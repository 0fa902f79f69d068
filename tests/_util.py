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


def box_iou(a, b):
    """IoU matrix of (n, 4) and (m, 4) x1y1x2y2 boxes (float64 numpy)."""
    a = np.asarray(a, dtype=np.float64)[:, None, :]
    b = np.asarray(b, dtype=np.float64)[None, :, :]
    iw = np.clip(np.minimum(a[..., 2], b[..., 2]) - np.maximum(a[..., 0], b[..., 0]), 0, None)
    ih = np.clip(np.minimum(a[..., 3], b[..., 3]) - np.maximum(a[..., 1], b[..., 1]), 0, None)
    inter = iw * ih
    area = lambda x: (x[..., 2] - x[..., 0]) * (x[..., 3] - x[..., 1])
    return inter / np.maximum(area(a) + area(b) - inter, 1e-12)


def detection_match(got, want, top=100, iou_min=0.5):
    """Detection-set match of `got` against the reference detections `want` ((k, 6) rows
    x1 y1 x2 y2 score class, score-descending): each of want's `top` highest-scoring
    detections is matched greedily (in score order) to an unused detection of the same class
    in got with the highest IoU. Returns (fraction matched with IoU >= iou_min, mean IoU over
    want's top detections, unmatched counting 0)."""
    got = np.asarray(got, dtype=np.float64)
    want = np.asarray(want, dtype=np.float64)[:top]
    if len(want) == 0:
        return 1.0, 1.0
    used = np.zeros(len(got), dtype=bool)
    ious = np.zeros(len(want))
    if len(got):
        iou = box_iou(want[:, :4], got[:, :4])
        for i in range(len(want)):
            cand = np.where((got[:, 5] == want[i, 5]) & ~used)[0]
            if len(cand):
                j = cand[np.argmax(iou[i, cand])]
                if iou[i, j] > 0:
                    ious[i] = iou[i, j]
                    used[j] = True
    return float((ious >= iou_min).mean()), float(ious.mean())
