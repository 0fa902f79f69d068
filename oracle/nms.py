"""NumPy restatement of the reference NMS (TEST INFRASTRUCTURE ONLY).

non_max_suppression   reference utils/util.py:123-169
torchvision_nms       the torchvision.ops.nms contract the reference calls at
                      util.py:162 (torchvision is not installed, its version is
                      unpinned in README.md:8): boxes sorted by score, keep the
                      best, drop every later box whose IoU with it is > thr,
                      IoU = inter / (area_a + area_b - inter), area = (x2-x1)*(y2-y1)
                      (no +1), all in the boxes' dtype; kept indices returned in
                      score order.

Deterministic tie rule (the reference's argsort at util.py:157 is unstable):
equal scores keep the row-major (anchor, class) candidate order.
"""
import numpy as np


def wh2xy(x):                                                   # util.py:76-82
    y = x.copy()
    y[:, 0] = x[:, 0] - x[:, 2] / 2
    y[:, 1] = x[:, 1] - x[:, 3] / 2
    y[:, 2] = x[:, 0] + x[:, 2] / 2
    y[:, 3] = x[:, 1] + x[:, 3] / 2
    return y


def torchvision_nms(boxes, scores, iou_threshold, limit=None):
    """Greedy NMS; returns kept indices in descending-score order (stable for ties).

    `limit` stops after that many keeps (the caller only uses the first max_det).
    """
    dt = boxes.dtype
    order = np.argsort(-scores.astype(np.float64), kind="stable")
    b = boxes[order]
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    area = (x2 - x1) * (y2 - y1)
    alive = np.ones(len(order), dtype=bool)
    keep = []
    zero = dt.type(0)
    for i in range(len(order)):
        if not alive[i]:
            continue
        keep.append(order[i])
        if limit is not None and len(keep) >= limit:
            break
        j = np.nonzero(alive[i + 1:])[0] + i + 1
        if j.size == 0:
            break
        xx1 = np.maximum(x1[i], x1[j])
        yy1 = np.maximum(y1[i], y1[j])
        xx2 = np.minimum(x2[i], x2[j])
        yy2 = np.minimum(y2[i], y2[j])
        w = np.maximum(zero, xx2 - xx1)
        h = np.maximum(zero, yy2 - yy1)
        inter = w * h
        ovr = inter / (area[i] + area[j] - inter)
        alive[j[ovr > iou_threshold]] = False
    return np.asarray(keep, dtype=np.int64)


def _round_to(a, half):
    """Round float32 values to a 16-bit float type and back (None = keep float32)."""
    if half is None:
        return a
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(half).float().numpy()


def non_max_suppression(outputs, confidence_threshold=0.001, iou_threshold=0.65,
                        max_det=300, max_nms=30000, max_wh=7680, half=None):
    """(B, 4+nc, A) float32 array -> list of (k, 6) float32 arrays (util.py:123-169).

    `half` (torch.float16 / torch.bfloat16) describes head outputs that were
    produced in that dtype: the threshold is rounded to it (torch compares a
    tensor with a Python float in the tensor's dtype) and the wh2xy corners are
    rounded to it, while the class-offset IoU geometry stays in float32 (the
    documented deviation of the HIP path for 16-bit inputs).
    """
    outputs = np.asarray(outputs, dtype=np.float32)
    bs, no, _ = outputs.shape
    nc = no - 4
    thr = np.float32(_round_to(np.array([confidence_threshold], np.float32), half)[0])
    res = []
    for xi in outputs:                                          # util.py:136
        x = xi.T                                                # (A, 4+nc)
        keep_anchor = x[:, 4:].max(1) > thr                     # util.py:130
        x = x[keep_anchor]
        if not x.shape[0]:
            res.append(np.zeros((0, 6), np.float32))
            continue
        box = _round_to(wh2xy(x[:, :4]), half)                  # util.py:144-145
        i, j = np.nonzero(x[:, 4:] > thr)                       # util.py:147, row-major
        det = np.concatenate((box[i], x[i, 4 + j, None], j[:, None].astype(np.float32)), 1)
        if not det.shape[0]:
            res.append(np.zeros((0, 6), np.float32))
            continue
        det = det[np.argsort(-det[:, 4].astype(np.float64), kind="stable")[:max_nms]]  # util.py:157
        c = det[:, 5:6] * np.float32(max_wh)                    # util.py:160
        keep = torchvision_nms(det[:, :4] + c, det[:, 4], iou_threshold, limit=max_det)  # util.py:161-163
        res.append(det[keep[:max_det]])
    return res
