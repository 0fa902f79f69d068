"""Host (CPU) NMS yh_nms_host (csrc/nms_host.cpp) vs the reference goldens and the oracle.

The drop-in's CPU device path (utils.util.non_max_suppression on a CPU tensor,
main.py:20) runs this C++ implementation; the oracle is only the checker. Bar:
bit-exact kept rows and counts, as for the device kernel (tests/test_gpu_nms.py).
"""
import numpy as np
import pytest
import torch

from _util import golden_name
from conftest import load_golden
from oracle import nms as onms
from yolo_hip import synth


def _host_nms(y, **kw):
    from yolo_hip.engine import nms_host
    dets, counts = nms_host(y, **kw)
    return [dets[i, :c].numpy() for i, c in enumerate(counts.tolist())]


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


def test_matches_reference_golden_synthetic():
    g = load_golden("nms_synth.npz")
    y = torch.stack([synth.synth_head_output(8400, 80, seed=int(s), mode=str(m))
                     for m, s in zip(g["modes"], g["seeds"])])
    _assert_same(_host_nms(y), _unpack(g["counts"], g["dets"]))


def test_matches_reference_golden_on_model_output():
    g = load_golden("nms_forward_n640.npz")
    y = torch.from_numpy(load_golden(golden_name("n", 640, 1))["y"])
    _assert_same(_host_nms(y), _unpack(g["counts"], g["dets"]))


@pytest.mark.parametrize("seed", range(4))
def test_random_cases_vs_oracle(seed):
    rng = np.random.default_rng(seed)
    B = int(rng.integers(1, 4))
    A = int(rng.integers(50, 3000))
    nc = int(rng.choice([1, 3, 80]))
    y = np.zeros((B, 4 + nc, A), np.float32)
    y[:, 0] = rng.uniform(0, 640, (B, A))
    y[:, 1] = rng.uniform(0, 640, (B, A))
    y[:, 2:4] = np.exp(rng.uniform(np.log(4), np.log(200), (B, 2, A)))
    y[:, 4:] = rng.uniform(0, 1, (B, nc, A)) ** 8      # many below 0.001, a few ties of 0
    y[:, 4:, ::7] = 0.5                                 # exact score ties
    t = torch.from_numpy(y)
    _assert_same(_host_nms(t, iou_threshold=0.5), onms.non_max_suppression(y, iou_threshold=0.5))


@pytest.mark.parametrize("dt", [torch.float16, torch.bfloat16])
def test_half_inputs_vs_oracle(dt):
    y = torch.stack([synth.synth_head_output(8400, 80, seed=s, mode="typical") for s in (3, 4)]).to(dt)
    want = onms.non_max_suppression(y.float().numpy(), half=dt)
    _assert_same(_host_nms(y), want)


def test_stress_every_pair_a_candidate():
    y = synth.synth_head_output(8400, 80, seed=5, mode="stress")[None]
    _assert_same(_host_nms(y), onms.non_max_suppression(y.numpy()))


def test_thread_count_does_not_change_results():
    from yolo_hip.engine import nms_host
    y = torch.stack([synth.synth_head_output(8400, 80, seed=s, mode="typical") for s in range(5)])
    d1, c1 = nms_host(y, threads=1)
    d8, c8 = nms_host(y, threads=8)
    assert torch.equal(c1, c8) and torch.equal(d1, d8)


@pytest.mark.parametrize("iou", [-0.1, -0.0])
def test_negative_iou_threshold_vs_oracle(iou):
    """iou_threshold < 0: disjoint pairs (IoU 0) suppress too, across classes; zero-area boxes
    (NaN IoU) never do."""
    rng = np.random.default_rng(11)
    B, A, nc = 2, 900, 80
    y = np.empty((B, 4 + nc, A), np.float32)
    y[:, 0:2] = rng.uniform(0, 640, size=(B, 2, A))
    y[:, 2:4] = rng.uniform(8, 60, size=(B, 2, A))
    y[:, 2:4, ::50] = 0.0
    y[:, 4:] = (1 / (1 + np.exp(-rng.normal(-5, 2.5, size=(B, nc, A))))).astype(np.float32)
    _assert_same(_host_nms(torch.from_numpy(y), iou_threshold=iou),
                 onms.non_max_suppression(y, 0.001, iou, 300, 30000))
