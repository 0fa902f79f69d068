"""On-device NMS (yh_nms) vs the reference goldens and the oracle. Marked gpu.

Bar: bit-exact kept rows (x1, y1, x2, y2, score, class) and counts for float32
head outputs; for 16-bit outputs, bit-exact against the oracle run with the same
dtype rounding of threshold and wh2xy corners.
"""
import numpy as np
import pytest
import torch

from _util import golden_name
from conftest import load_golden
from oracle import nms as onms
from yolo_hip import synth

pytestmark = pytest.mark.gpu


def _gpu_nms(y, dev, **kw):
    from yolo_hip.engine import nms
    dets, counts = nms(y.to(dev), **kw)
    counts = counts.cpu().tolist()
    dets = dets.cpu().numpy()
    return [dets[i, :c] for i, c in enumerate(counts)]


def _unpack(counts, flat):
    out, o = [], 0
    for c in counts:
        out.append(flat[o:o + c])
        o += c
    return out


def _assert_same(got, want):
    assert len(got) == len(want)
    for i, (a, b) in enumerate(zip(got, want)):
        assert a.shape == b.shape, f"image {i}: kept {a.shape[0]} vs {b.shape[0]}"
        np.testing.assert_array_equal(a, b, err_msg=f"image {i}")


def test_matches_reference_golden_synthetic(gpu):
    g = load_golden("nms_synth.npz")
    y = torch.stack([synth.synth_head_output(8400, 80, seed=int(s), mode=str(m))
                     for m, s in zip(g["modes"], g["seeds"])])
    _assert_same(_gpu_nms(y, gpu), _unpack(g["counts"], g["dets"]))


def test_matches_reference_golden_on_model_output(gpu):
    g = load_golden("nms_forward_n640.npz")
    y = torch.from_numpy(load_golden(golden_name("n", 640, 1))["y"])
    _assert_same(_gpu_nms(y, gpu), _unpack(g["counts"], g["dets"]))


@pytest.mark.parametrize("seed", range(6))
def test_random_cases_vs_oracle(gpu, seed):
    rng = np.random.default_rng(seed)
    B = int(rng.integers(1, 4))
    A = int(rng.integers(50, 3000))
    nc = int(rng.choice([1, 3, 80]))
    y = np.empty((B, 4 + nc, A), np.float32)
    y[:, 0:2] = rng.uniform(0, 320, size=(B, 2, A))
    y[:, 2:4] = rng.uniform(2, 120, size=(B, 2, A))
    s = 1 / (1 + np.exp(-rng.normal(-4, 3, size=(B, nc, A))))
    if seed % 2:  # heavy ties: quantised scores
        s = np.round(s * 64) / 64
    y[:, 4:] = s.astype(np.float32)
    kw = dict(confidence_threshold=float(rng.choice([0.001, 0.05, 0.3])), iou_threshold=float(rng.choice([0.3, 0.5, 0.65, 0.9])),
              max_det=int(rng.choice([1, 17, 300])), max_nms=int(rng.choice([50, 5000, 30000])))
    want = onms.non_max_suppression(y, kw["confidence_threshold"], kw["iou_threshold"], kw["max_det"], kw["max_nms"])
    got = _gpu_nms(torch.from_numpy(y), gpu, **kw)
    _assert_same(got, want)


@pytest.mark.parametrize("case", ["small_max_wh", "huge_boxes"])
def test_cross_class_overlap_vs_oracle(gpu, case):
    """Boxes of different classes overlap after the class offset (max_wh below the coordinate
    range, or boxes wider than max_wh / 2): the same-class shortcut of the IoU mask must not
    apply, and cross-class suppression must match the oracle."""
    rng = np.random.default_rng(7 if case == "huge_boxes" else 8)
    B, A, nc = 2, 2500, 80
    y = np.empty((B, 4 + nc, A), np.float32)
    y[:, 0:2] = rng.uniform(0, 640, size=(B, 2, A))
    y[:, 2:4] = rng.uniform(8, 200, size=(B, 2, A))
    if case == "huge_boxes":
        y[:, 2:4, ::97] = rng.uniform(4000, 20000, size=(B, 2, y[:, 2:4, ::97].shape[-1]))
    y[:, 4:] = (1 / (1 + np.exp(-rng.normal(-5, 2.5, size=(B, nc, A))))).astype(np.float32)
    max_wh = 40.0 if case == "small_max_wh" else 7680.0
    for iou in (0.3, 0.65):
        want = onms.non_max_suppression(y, 0.001, iou, 300, 30000, max_wh=max_wh)
        _assert_same(_gpu_nms(torch.from_numpy(y), gpu, iou_threshold=iou, max_wh=max_wh), want)


def test_empty_and_ragged_batch(gpu):
    y = torch.zeros(3, 84, 500)
    y[:, 2:4] = 20.0
    y[1, 4 + 2, 7] = 0.9
    y[1, 0:2, 7] = 100.0
    got = _gpu_nms(y, gpu)
    assert [g.shape[0] for g in got] == [0, 1, 0]
    np.testing.assert_array_equal(got[1], np.array([[90, 90, 110, 110, 0.9, 2]], np.float32))


def test_many_candidates_multiple_select_batches(gpu):
    """Every pair is a candidate (>4096 per image): exercises radix select + several sorted batches."""
    y = torch.stack([synth.synth_head_output(8400, 80, seed=9, mode="stress"),
                     synth.synth_head_output(8400, 80, seed=10, mode="dense")])
    for kw in (dict(), dict(max_det=1024, max_nms=20000), dict(iou_threshold=0.05, max_det=1024)):
        want = onms.non_max_suppression(y.numpy(), **kw)
        _assert_same(_gpu_nms(y, gpu, **kw), want)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_half_inputs_vs_oracle(gpu, dtype):
    y = torch.stack([synth.synth_head_output(8400, 80, seed=4, mode="typical"),
                     synth.synth_head_output(8400, 80, seed=5, mode="dense")]).to(dtype)
    want = onms.non_max_suppression(y.float().numpy(), half=dtype)
    _assert_same(_gpu_nms(y, gpu), want)


def test_dropin_non_max_suppression(gpu):
    from utils.util import non_max_suppression
    g = load_golden("nms_forward_n640.npz")
    y = torch.from_numpy(load_golden(golden_name("n", 640, 1))["y"]).to(gpu)
    out = non_max_suppression(y)
    assert isinstance(out, list) and len(out) == 1 and out[0].device == y.device
    _assert_same([out[0].cpu().numpy()], _unpack(g["counts"], g["dets"]))


@pytest.mark.parametrize("iou", [-0.1, -0.0, -1e-30])
def test_negative_iou_threshold_vs_oracle(gpu, iou):
    """with iou_threshold < 0 a disjoint pair (IoU 0 > thr) suppresses too, across
    classes, so the same-class shortcut must not apply (torchvision's greedy contract)."""
    rng = np.random.default_rng(11)
    B, A, nc = 2, 900, 80
    y = np.empty((B, 4 + nc, A), np.float32)
    y[:, 0:2] = rng.uniform(0, 640, size=(B, 2, A))
    y[:, 2:4] = rng.uniform(8, 60, size=(B, 2, A))
    y[:, 2:4, ::50] = 0.0   # zero-area boxes: 0 / 0 union, NaN IoU never suppresses
    y[:, 4:] = (1 / (1 + np.exp(-rng.normal(-5, 2.5, size=(B, nc, A))))).astype(np.float32)
    want = onms.non_max_suppression(y, 0.001, iou, 300, 30000)
    _assert_same(_gpu_nms(torch.from_numpy(y), gpu, iou_threshold=iou), want)


@pytest.mark.parametrize("scores", ["spread", "tied"])
def test_few_kept_long_continuation_vs_oracle(gpu, scores):
    """Boxes of each class piled on one spot: an image keeps about one box per class of 67 k
    candidates, so NMS runs later batches until max_nms candidates are processed (the C5
    pattern). 'spread': scores over many bins (the fast path's compact list); 'tied': one score
    for every pair (a single bin past 4096 keys: the radix-select path and its list)."""
    rng = np.random.default_rng(21)
    B, A, nc = 2, 8400, 8
    y = np.empty((B, 4 + nc, A), np.float32)
    y[:, 0:2] = 320.0 + rng.uniform(-2, 2, size=(B, 2, A))
    y[:, 2:4] = 100.0 + rng.uniform(-2, 2, size=(B, 2, A))
    if scores == "spread":
        y[:, 4:] = rng.uniform(0.01, 0.99, size=(B, nc, A)).astype(np.float32)
    else:
        y[:, 4:] = 0.5
    for kw in (dict(), dict(max_nms=50000, max_det=5)):
        want = onms.non_max_suppression(y, 0.001, 0.65, kw.get("max_det", 300), kw.get("max_nms", 30000))
        _assert_same(_gpu_nms(torch.from_numpy(y), gpu, **kw), want)
