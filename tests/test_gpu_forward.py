"""HIP forward parity on an MI355X: every variant vs the reference goldens, the
drop-in nets.nn path, graph replay, batch invariance. Marked gpu.

Tolerances (written here, justified in DESIGN.md §Parity):
  float32: class scores |Δ| <= 1e-3; box coordinates |Δ| <= 1e-3 in grid units
           (pixels / stride = the model's native output before nets/nn.py:270 multiplies
           by the stride), widened to 2x the reference's own fp32 CPU noise where that is
           larger (v11_x). The golden is the reference evaluated in float64.
  bf16/fp16: mean |Δ| (boxes px, scores) <= 2x the reference's own CPU bf16/fp16 forward's
           mean deviation from the same float64 golden; max |Δ| <= 4x its max.
"""
import numpy as np
import pytest
import torch

from _util import FORWARD_GOLDENS, GOLDEN_INPUT_SEED, golden_name, grid_unit_error, make_model
from conftest import load_golden
from yolo_hip import synth

pytestmark = pytest.mark.gpu


def _engine(model, dtype, dev):
    from yolo_hip.engine import Engine
    eng = Engine(*model._yh_arch, dev, dtype)
    eng.load_module(model)
    return eng


@pytest.mark.parametrize("variant,size,batch", FORWARD_GOLDENS)
def test_fp32_matches_reference(gpu, variant, size, batch):
    g = load_golden(golden_name(variant, size, batch))
    model = make_model(variant)
    x = synth.synth_scenes(batch, size, size, seed=GOLDEN_INPUT_SEED)
    eng = _engine(model, torch.float32, gpu)
    y = eng.forward(x.to(gpu)).cpu()
    dbox, dcls = grid_unit_error(y, g["y"], size, size)
    ref_noise_grid = float(g["dev_fp32_8thr"][0]) / 8.0
    tol_box = max(1e-3, 2.0 * ref_noise_grid)
    dpx = (y[:, :4].double() - torch.from_numpy(g["y"][:, :4]).double()).abs().max().item()
    print(f"v11_{variant}@{size} fp32: box {dbox:.2e} grid ({dpx:.2e} px; reference fp32 noise "
          f"{g['dev_fp32_8thr'][0]:.2e} px), cls {dcls:.2e}")
    assert dcls <= 1e-3
    assert dbox <= tol_box


@pytest.mark.parametrize("dtype,key", [(torch.bfloat16, "dev_bf16"), (torch.float16, "dev_fp16")])
@pytest.mark.parametrize("variant,size,batch", [("n", 640, 1), ("s", 256, 1), ("m", 256, 1)])
def test_half_precision_within_reference_noise(gpu, dtype, key, variant, size, batch):
    g = load_golden(golden_name(variant, size, batch))
    model = make_model(variant)
    x = synth.synth_scenes(batch, size, size, seed=GOLDEN_INPUT_SEED)
    eng = _engine(model, dtype, gpu)
    y = eng.forward(x.to(gpu, dtype)).float().cpu().double()
    ref = torch.from_numpy(g["y"]).double()
    d = (y - ref).abs()
    mine = [d[:, :4].max().item(), d[:, :4].mean().item(), d[:, 4:].max().item(), d[:, 4:].mean().item()]
    floor = [float(v) for v in g[key]]
    print(f"v11_{variant}@{size} {dtype}: box max {mine[0]:.3g} mean {mine[1]:.3g} (ref {floor[0]:.3g}/{floor[1]:.3g}); "
          f"cls max {mine[2]:.3g} mean {mine[3]:.3g} (ref {floor[2]:.3g}/{floor[3]:.3g})")
    assert mine[1] <= 2.0 * floor[1] and mine[3] <= 2.0 * floor[3]
    assert mine[0] <= 4.0 * floor[0] and mine[2] <= 4.0 * floor[2]


def test_dropin_module_runs_hip_path(gpu):
    model = make_model("n")
    x = synth.synth_scenes(2, 320, 320, seed=11)
    m = model.to(gpu)
    with torch.no_grad():
        y = m(x.to(gpu))
    assert "_yh_engines" in m.__dict__ and len(m.__dict__["_yh_engines"]) == 1
    from yolo_hip import _lib
    assert _lib._lib is not None, "libyolo_hip.so was not loaded"
    ref = _engine(make_model("n"), torch.float32, gpu).forward(x.to(gpu))
    assert torch.equal(y, ref)


def test_dropin_detects_weight_changes(gpu):
    model = make_model("n").to(gpu)
    x = synth.synth_scenes(1, 256, 256, seed=12).to(gpu)
    with torch.no_grad():
        y0 = model(x).clone()
        model.head.cls[0][4].bias.add_(1.0)
        y1 = model(x)
    assert not torch.equal(y0, y1)


def test_dropin_half_model(gpu):
    model = make_model("n").to(gpu).half()
    x = synth.synth_scenes(1, 320, 320, seed=13).to(gpu).half()
    with torch.no_grad():
        y = model(x)
    assert y.dtype == torch.float16 and y.shape == (1, 84, 2100)
    assert torch.isfinite(y).all()


def test_graph_replay_equals_eager_and_batch_invariance(gpu):
    model = make_model("n")
    x = synth.synth_scenes(3, 320, 320, seed=14).to(gpu, torch.bfloat16)
    eng = _engine(model, torch.bfloat16, gpu)
    eng.set_graph(False)
    eager = eng.forward(x)
    eng.set_graph(True)
    g1 = eng.forward(x)
    g2 = eng.forward(x)
    assert torch.equal(eager, g1) and torch.equal(g1, g2)
    for i in range(3):
        single = eng.forward(x[i:i + 1].contiguous())
        assert torch.equal(single[0], g1[i]), f"image {i} depends on its batch"


def test_rectangular_input(gpu):
    model = make_model("n")
    x = synth.synth_scenes(1, 256, 384, seed=15)
    eng = _engine(model, torch.float32, gpu)
    y = eng.forward(x.to(gpu)).cpu()
    from _util import oracle_for
    ref = oracle_for("n", torch.float64)(x).float()
    dbox, dcls = grid_unit_error(y, ref, 256, 384)
    assert dbox <= 1e-3 and dcls <= 1e-3


def test_unfused_model_folds_batchnorm_on_device(gpu):
    g = load_golden(golden_name("n", 320, 2))
    model = make_model("n", fused=False)
    x = synth.synth_scenes(2, 320, 320, seed=GOLDEN_INPUT_SEED)
    y = _engine(model, torch.float32, gpu).forward(x.to(gpu)).cpu()
    dbox, dcls = grid_unit_error(y, g["y"], 320, 320)
    assert dbox <= 1e-3 and dcls <= 1e-3
