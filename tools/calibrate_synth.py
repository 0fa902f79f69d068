"""Calibrate the synthetic weights so the random network behaves like a trained one.

Random conv weights alone put a 90-conv SiLU network either in the vanishing or
the exploding regime (global gain 1.45 -> outputs independent of the image,
1.6 -> saturated DFL and class scores). A trained detector avoids both because
its BatchNorm running statistics match the activations they normalise. This
tool recreates that: one train-mode forward (BatchNorm momentum 1.0) of the
drop-in module tree on synthetic scenes (yolo_hip.synth.synth_scenes) sets every running_mean/running_var to
the batch statistics it sees, then the class-logit bias of the head is shifted
so that ~2% of (anchor, class) pairs clear the 0.001 NMS threshold.

The resulting statistics are stored as data (yolo_hip/synth_calib/v11_<v>.npz)
and applied by yolo_hip.synth.synth_state_dict, so every machine rebuilds
bit-identical weights without re-running this tool.

Usage: python tools/calibrate_synth.py [n t s m l x]
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))

from nets import nn  # noqa: E402
from yolo_hip import synth  # noqa: E402

OUT = os.path.join(ROOT, "yolo-infer-pt_amd", "yolo_hip", "synth_calib")
TARGET_FRACTION = 0.02


def calibrate(variant):
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{variant}")(80)
    sd = synth.synth_state_dict(model.state_dict(), seed=0, calib=False, cls_bias=0.0)
    model.load_state_dict(sd)
    for m in model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.momentum = 1.0
    model.train()
    x = synth.synth_scenes(8, 640, 640, seed=123)
    with torch.no_grad():
        model(x)
        model.eval()
        y = model(synth.synth_scenes(4, 640, 640, seed=321))
    scores = y[:, 4:].double().clamp(1e-12, 1 - 1e-12)
    logits = torch.log(scores / (1 - scores)).flatten()
    thr = float(np.log(0.001 / 0.999))
    q = float(torch.quantile(logits[torch.randperm(logits.numel())[:500000]], 1 - TARGET_FRACTION))
    shift = thr - q
    stats = {}
    for name, t in model.state_dict().items():
        if name.endswith("running_mean") or name.endswith("running_var"):
            stats[name] = t.detach().float().numpy()
    stats["cls_shift"] = np.array([shift], dtype=np.float32)
    path = os.path.join(OUT, f"v11_{variant}.npz")
    np.savez_compressed(path, **stats)
    print(f"v11_{variant}: {len(stats) - 1} BN stat tensors, cls logit shift {shift:+.3f} -> {path}")


if __name__ == "__main__":
    torch.set_num_threads(os.cpu_count() or 8)
    for v in (sys.argv[1:] or ["n", "t", "s", "m", "l", "x"]):
        calibrate(v)
