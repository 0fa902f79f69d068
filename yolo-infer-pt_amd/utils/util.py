"""Drop-in for the hot-path helpers of the reference's `utils/util.py`.

  make_anchors          reference utils/util.py:85-96 (grid centres + stride per anchor)
  wh2xy                 reference utils/util.py:76-82
  non_max_suppression   reference utils/util.py:123-169, run on device by the gfx950
                        kernels behind include/yolo_hip.h (yh_nms)
  setup_seed            reference utils/util.py:12-20
  load_weight           reference utils/util.py:345-355 } yolo_hip.weights: safe checkpoint
  load_ultralytics_weight  utils/util.py:358-516       } reading + key mapping; the HIP
                        engine re-packs the new parameters on the next device forward
  compute_metric, compute_ap, smooth   utils/util.py:99-120, 225-300, 172-177: the eval
                        loop's metrics on the device (yolo_hip.metrics)

non_max_suppression semantics: candidate (anchor, class) pairs with score >
threshold (compared in the tensor dtype), score-descending order with ties
broken by the lower anchor*nc + class index (the reference's argsort is
unstable, util.py:157), first 30000 kept, class-offset boxes (class * 7680),
greedy IoU > threshold suppression (torchvision.ops.nms contract), first 300
kept. As in the reference, the rows come back as float32 (util.py:148: torch.cat
with `j.float()` promotes box and score to float32, so the class offset and the
IoU run in float32 too; the wh2xy corners are rounded to the input dtype first).
Head outputs on a cuda device run on the MI355X kernels (yh_nms); on the CPU
device (main.py:20 falls back to "cpu") the library's C++ host implementation
(yh_nms_host) runs the same contract. Deliberate difference: no wall-clock
cutoff (util.py:133-134,166-167 silently truncates batches).
"""
import math
import os
import random

import numpy
import torch

from yolo_hip.metrics import compute_ap, compute_metric, smooth  # noqa: F401

__all__ = ["setup_seed", "setup_multi_processes", "wh2xy", "make_anchors", "non_max_suppression", "load_weight",
           "load_ultralytics_weight", "compute_metric", "compute_ap", "smooth", "AverageMeter"]

# Training-side names of the reference's utils/util.py (losses, label assigner, EMA, LR
# schedules, optimizer groups, plots, ONNX export) are outside this build's scope
#  and deliberately absent: training keeps the reference's own utils.


class AverageMeter:
    """Running mean of per-batch values weighted by batch size, NaNs skipped
    (reference utils/util.py:630-640; main.py:119-121 logs losses with it)."""

    def __init__(self):
        self.num = 0
        self.sum = 0
        self.avg = 0

    def update(self, v, n):
        if math.isnan(float(v)):
            return
        self.num += n
        self.sum += v * n
        self.avg = self.sum / self.num

MAX_WH = 7680
MAX_DET = 300
MAX_NMS = 30000


def setup_seed():
    random.seed(0)
    numpy.random.seed(0)
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True


def setup_multi_processes():
    """Process settings of the reference's entry point (utils/util.py:23-44, called by main.py:354):
    the `fork` start method, OpenCV's own threading off when cv2 is installed, and OMP / MKL
    thread counts of 1 unless the environment sets them."""
    import platform
    if platform.system() != "Windows":
        torch.multiprocessing.set_start_method("fork", force=True)
    try:
        import cv2
        cv2.setNumThreads(0)
    except ImportError:
        pass
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    os.environ.setdefault("MKL_NUM_THREADS", "1")


def wh2xy(x):
    """(cx, cy, w, h) -> (x1, y1, x2, y2) for an (n, 4+) tensor or array."""
    y = x.clone() if isinstance(x, torch.Tensor) else numpy.copy(x)
    half_w, half_h = x[:, 2] / 2, x[:, 3] / 2
    y[:, 0] = x[:, 0] - half_w
    y[:, 1] = x[:, 1] - half_h
    y[:, 2] = x[:, 0] + half_w
    y[:, 3] = x[:, 1] + half_h
    return y


def make_anchors(x, strides, offset=0.5):
    """Per-level grid centres (x + offset, y + offset), row-major, and the level stride per anchor."""
    assert x is not None
    points, stride_col = [], []
    dtype, device = x[0].dtype, x[0].device
    for level, stride in enumerate(strides):
        h, w = x[level].shape[-2:]
        gx = torch.arange(end=w, device=device, dtype=dtype) + offset
        gy = torch.arange(end=h, device=device, dtype=dtype) + offset
        gy, gx = torch.meshgrid(gy, gx, indexing="ij")
        points.append(torch.stack((gx, gy), -1).view(-1, 2))
        stride_col.append(torch.full((h * w, 1), stride, dtype=dtype, device=device))
    return torch.cat(points), torch.cat(stride_col)


def non_max_suppression(outputs, confidence_threshold=0.001, iou_threshold=0.65):
    """(B, 4 + nc, A) head outputs -> list of B float32 tensors (k <= 300, 6) = x1, y1, x2, y2, score, class."""
    from yolo_hip.engine import nms, nms_host

    run = nms if outputs.is_cuda else nms_host
    dets, counts = run(outputs, confidence_threshold, iou_threshold, MAX_DET, MAX_NMS, float(MAX_WH))
    kept = counts.tolist()
    return [dets[i, :k] for i, k in enumerate(kept)]


def load_weight(model, ckpt, trusted=False):
    """Keep the checkpoint tensors whose key and shape match the model; load non-strictly."""
    from yolo_hip.weights import load_weight as _lw
    return _lw(model, ckpt, trusted=trusted)


def load_ultralytics_weight(model, ckpt_path, mapping="reference", trusted=False):
    """Ultralytics YOLO11 checkpoint -> model (mapping "reference" = the reference's key map, "exact" = all keys)."""
    from yolo_hip.weights import load_ultralytics_weight as _lu
    return _lu(model, ckpt_path, mapping=mapping, trusted=trusted)
