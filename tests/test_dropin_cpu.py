"""Drop-in API (nets.nn / utils.util) on the CPU: constructor parity with the
reference, module-tree semantics vs the oracle, anchors, public names."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from _util import GOLDEN_INPUT_SEED, golden_name, make_model
from conftest import GOLD, load_golden
from yolo_hip import synth


def test_public_api_names():
    from nets import nn
    from utils import util
    for name in ("fuse_conv", "Conv", "Residual", "CSPModule", "CSP", "SPP", "Attention", "PSABlock", "PSA",
                 "DarkNet", "DarkFPN", "DFL", "Head", "YOLO", "yolo_v11_n", "yolo_v11_t", "yolo_v11_s",
                 "yolo_v11_m", "yolo_v11_l", "yolo_v11_x"):
        assert hasattr(nn, name), name
    for name in ("make_anchors", "wh2xy", "non_max_suppression", "setup_seed"):
        assert hasattr(util, name), name


def test_fresh_construction_is_bit_identical_to_reference():
    """Same module registration order and init as nets/nn.py -> identical state_dict for seed 0."""
    from nets import nn
    with open(os.path.join(GOLD, "construct_v11_n.json")) as f:
        gold = json.load(f)
    torch.manual_seed(0)
    m = nn.yolo_v11_n(80)
    sd = m.state_dict()
    assert list(m.stride.tolist()) == gold["stride"]
    assert sorted(sd.keys()) == sorted(gold["tensors"].keys())
    for k, v in sd.items():
        h = hashlib.sha256(np.ascontiguousarray(v.detach().numpy()).tobytes()).hexdigest()
        assert h == gold["tensors"][k], k


def test_head_attributes():
    m = make_model("n", fused=False)
    assert m.head.nc == 80 and m.head.no == 144 and m.head.ch == 16
    assert m.stride.tolist() == [8.0, 16.0, 32.0]


def test_module_forward_matches_golden_fp32():
    g = load_golden(golden_name("n", 320, 2))
    m = make_model("n")
    x = synth.synth_scenes(2, 320, 320, seed=GOLDEN_INPUT_SEED)
    with torch.no_grad():
        y = m(x).numpy()
    # fp32 CPU forward vs float64 golden: the reference's own fp32 noise level
    np.testing.assert_allclose(y, g["y"], rtol=1e-5, atol=2e-3)


def test_module_forward_matches_golden_fp32_c1():
    """C1's own shape (BASELINE.json configs[0]: v11_n, 1 x 3 x 640 x 640, PyTorch CPU forward)
    through the drop-in module on the CPU, against the reference's float64 golden, within
    2x the reference's own fp32 noise (8 vs 1 thread) in pixels and scores."""
    g = load_golden(golden_name("n", 640, 1))
    m = make_model("n")
    x = synth.synth_scenes(1, 640, 640, seed=GOLDEN_INPUT_SEED)
    with torch.no_grad():
        y = m(x).double().numpy()
    d = np.abs(y - g["y"])
    noise = [float(v) for v in g["dev_fp32_8thr"]]
    assert d[:, :4].max() <= max(1e-3, 2 * noise[0]), (d[:, :4].max(), noise[0])
    assert d[:, 4:].max() <= max(1e-5, 2 * noise[2]), (d[:, 4:].max(), noise[2])


def test_fuse_matches_reference_fold_formula():
    from nets import nn
    conv = torch.nn.Conv2d(8, 16, 3, padding=1, bias=False)
    bn = torch.nn.BatchNorm2d(16, eps=1e-3)
    with torch.no_grad():
        for t in (bn.weight, bn.bias, bn.running_mean):
            t.copy_(torch.randn(16))
        bn.running_var.copy_(torch.rand(16) + 0.5)
    bn.eval()
    f = nn.fuse_conv(conv, bn)
    x = torch.randn(2, 8, 9, 9)
    with torch.no_grad():
        np.testing.assert_allclose(f(x).numpy(), bn(conv(x)).numpy(), rtol=1e-5, atol=1e-5)


def test_make_anchors_layout():
    from utils.util import make_anchors
    feats = [torch.zeros(1, 4, 4, 6), torch.zeros(1, 4, 2, 3)]
    a, s = make_anchors(feats, torch.tensor([8.0, 16.0]))
    assert a.shape == (24 + 6, 2) and s.shape == (30, 1)
    assert a[0].tolist() == [0.5, 0.5] and a[1].tolist() == [1.5, 0.5] and a[6].tolist() == [0.5, 1.5]
    assert s[:24].unique().tolist() == [8.0] and s[24:].unique().tolist() == [16.0]


def test_wh2xy():
    from utils.util import wh2xy
    b = torch.tensor([[10.0, 20.0, 4.0, 6.0]])
    assert wh2xy(b).tolist() == [[8.0, 17.0, 12.0, 23.0]]


def test_cpu_nms_runs_the_native_host_path():
    """main.py:20 falls back to the CPU device: the drop-in NMS runs yh_nms_host (C++),
    returns the reference's float32 rows (util.py:148 promotes through j.float())."""
    from utils.util import non_max_suppression
    from yolo_hip import synth
    y = torch.stack([synth.synth_head_output(8400, 80, seed=1, mode="typical")])
    for dt in (torch.float32, torch.float16, torch.bfloat16):
        out = non_max_suppression(y.to(dt))
        assert len(out) == 1 and out[0].dtype == torch.float32 and out[0].shape[1] == 6 and out[0].shape[0] > 0
    empty = non_max_suppression(torch.zeros(2, 84, 10))
    assert [tuple(o.shape) for o in empty] == [(0, 6), (0, 6)] and empty[0].dtype == torch.float32


def test_training_mode_returns_level_maps():
    m = make_model("n", fused=False).train()
    out = m(torch.zeros(1, 3, 64, 64))
    assert [tuple(t.shape) for t in out] == [(1, 144, 8, 8), (1, 144, 4, 4), (1, 144, 2, 2)]
