"""HIP forward parity on an MI355X: every variant vs the reference goldens, the
drop-in nets.nn path, graph replay, batch invariance. Marked gpu.

Tolerances (written here, justified in DESIGN.md §Parity):
  float32: class scores |Δ| <= 1e-3; box coordinates |Δ| <= 1e-3 in grid units
           (pixels / stride = the model's native output before nets/nn.py:270 multiplies
           by the stride), widened to 2x the reference's own fp32 CPU noise where that is
           larger (v11_x). The golden is the reference evaluated in float64.
  bf16/fp16: mean |Δ| (boxes px, scores) <= 2x the reference's own CPU bf16/fp16 forward's
           mean deviation from the same float64 golden; box max |Δ| <= 2x its max; class
           scores: the 99.999th percentile of |Δ| <= 2x its max (at most ~7 of the 672 000
           scores of an image above it) and the max <= 3x. Measured r03 (max over the
           reference's max): boxes 0.59-1.22x, scores 0.87-2.16x (n@640 fp16: one score).
"""


def half_bars(d, ref_max_box, ref_mean_box, ref_max_cls, ref_mean_cls):
    """The bf16 / fp16 bar above on |Δ| (N, 4+nc, A) against the reference's own statistics."""
    box, cls = d[:, :4], d[:, 4:]
    q = float(np.quantile(np.asarray(cls).ravel(), 0.99999))
    assert box.mean() <= 2.0 * ref_mean_box and cls.mean() <= 2.0 * ref_mean_cls
    assert box.max() <= 2.0 * ref_max_box, (float(box.max()), ref_max_box)
    assert q <= 2.0 * ref_max_cls and cls.max() <= 3.0 * ref_max_cls, (q, float(cls.max()), ref_max_cls)
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
    # in pixels: within max(1e-3 px, 2x the reference's own fp32 CPU noise)
    assert dpx <= max(1e-3, 2.0 * float(g["dev_fp32_8thr"][0])), dpx
    assert dcls <= max(1e-5, 2.0 * float(g["dev_fp32_8thr"][2])), dcls


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
    half_bars(d.numpy(), floor[0], floor[1], floor[2], floor[3])


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


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("variant,size,batch", [("n", 640, 1), ("n", 320, 2), ("s", 256, 1), ("x", 320, 1)])
def test_half_precision_detection_sets_match(gpu, dtype, variant, size, batch):
    """post-NMS detection-set match of a bf16 / fp16 forward + device NMS
    against the float64 golden's detections (oracle NMS), beside the same measure for the
    reference algorithm run in that dtype on the CPU (oracle forward in bf16 / fp16)."""
    from _util import detection_match, oracle_for
    from oracle import nms as onms
    from yolo_hip.engine import nms
    g = load_golden(golden_name(variant, size, batch))
    want = onms.non_max_suppression(g["y"].astype(np.float32))
    model = make_model(variant)
    x = synth.synth_scenes(batch, size, size, seed=GOLDEN_INPUT_SEED)
    eng = _engine(model, dtype, gpu)
    dets, counts = nms(eng.forward(x.to(gpu, dtype)))
    dets, counts = dets.cpu().numpy(), counts.cpu().numpy()
    ref_half = oracle_for(variant, dtype)(x.to(dtype)).float().numpy()
    ref_dets = onms.non_max_suppression(ref_half, half=dtype)
    for i in range(batch):
        got = dets[i, :counts[i]]
        m50, miou = detection_match(got, want[i])
        r50, riou = detection_match(ref_dets[i], want[i])
        print(f"v11_{variant}@{size} {dtype} image {i}: top-100 match@0.5 {m50:.3f} mean IoU {miou:.4f} "
              f"(reference in {dtype} on CPU: {r50:.3f} / {riou:.4f})")
        # bar: as good as the reference algorithm run in the same dtype, within 3 of 100
        # detections (one-run comparisons of two noisy forwards)
        assert m50 >= min(0.99, r50) - 0.03
        assert miou >= min(0.99, riou) - 0.03


def test_s_fp16_bench_shape(gpu):
    """C3's configuration (v11_s, fp16, 640x640, batch 64): the per-shape tuner's plans for
    batch 64 give each image exactly the output of a batch-1 forward of it (every conv plan
    follows one reduction order), and image 0 is within the reference algorithm's own fp16
    noise of the float64 oracle (oracle run in fp16 on the CPU for the noise floor)."""
    from _util import oracle_for
    model = make_model("s")
    x = synth.synth_scenes(64, 640, 640, seed=21)
    eng = _engine(model, torch.float16, gpu)
    y = eng.forward(x.to(gpu, torch.float16)).clone()
    assert torch.isfinite(y.float()).all()
    for i in (0, 17, 63):
        y1 = eng.forward(x[i:i + 1].to(gpu, torch.float16))
        assert torch.equal(y1[0], y[i]), f"image {i}: batch-64 plan differs from batch-1"
    x0 = x[:1]
    ref = oracle_for("s", torch.float64)(x0).numpy()
    half = oracle_for("s", torch.float16)(x0.half()).float().numpy()
    d = np.abs(y[:1].float().cpu().numpy().astype(np.float64) - ref)
    f = np.abs(half.astype(np.float64) - ref)
    print(f"v11_s@640 fp16 b64: box max {d[:, :4].max():.3g} mean {d[:, :4].mean():.3g} "
          f"(reference fp16 {f[:, :4].max():.3g} / {f[:, :4].mean():.3g}); cls max {d[:, 4:].max():.3g} "
          f"(reference {f[:, 4:].max():.3g})")
    half_bars(d, f[:, :4].max(), f[:, :4].mean(), f[:, 4:].max(), f[:, 4:].mean())


def test_x_1280_c5_shape(gpu):
    """C5's shape (v11_x, 1280x1280: 33600 anchors, PSA attention over 1600 tokens) against
    the subsampled float64 golden (forward_x_1280_b1_sub.npz: 4096 seeded anchors, per-row
    sums over all anchors, the reference NMS detections)."""
    from _util import detection_match
    from yolo_hip.engine import nms
    g = load_golden("forward_x_1280_b1_sub.npz")
    idx = torch.from_numpy(g["idx"])
    ref = g["y_sub"].astype(np.float64)
    x = synth.synth_scenes(1, 1280, 1280, seed=GOLDEN_INPUT_SEED)
    model = make_model("x")
    counts_ref = int(g["counts"][0])
    want = g["dets"][:counts_ref]
    # fp32: within 2x the reference's own fp32 CPU noise (pixels / scores)
    y32 = _engine(model, torch.float32, gpu).forward(x.to(gpu))
    assert y32.shape[2] == int(g["anchors"])
    d = np.abs(y32[:, :, idx].cpu().double().numpy() - ref)
    rs = np.abs(y32.double().sum(dim=2).cpu().numpy() - g["row_sum"])
    print(f"v11_x@1280 fp32: box {d[:, :4].max():.3g} px (reference {g['dev_fp32_8thr'][0]:.3g}), "
          f"cls {d[:, 4:].max():.3g}; row-sum |d| max {rs.max():.3g}")
    assert d[:, :4].max() <= max(1e-3, 2 * float(g["dev_fp32_8thr"][0]))
    assert d[:, 4:].max() <= max(1e-5, 2 * float(g["dev_fp32_8thr"][2]))
    dets, counts = nms(y32)
    m50, miou = detection_match(dets[0, :counts[0]].cpu().numpy(), want)
    print(f"v11_x@1280 fp32 detections: match@0.5 {m50:.3f} mean IoU {miou:.4f}")
    assert m50 >= 0.99 and miou >= 0.99
    # bf16 (C5's dtype): within the reference's own bf16 CPU deviation (the bar above)
    yb = _engine(model, torch.bfloat16, gpu).forward(x.to(gpu, torch.bfloat16)).float()
    assert torch.isfinite(yb).all()
    d = np.abs(yb[:, :, idx].cpu().double().numpy() - ref)
    fl = [float(v) for v in g["dev_bf16"]]
    print(f"v11_x@1280 bf16: box max {d[:, :4].max():.3g} mean {d[:, :4].mean():.3g} (reference {fl[0]:.3g} / "
          f"{fl[1]:.3g}); cls max {d[:, 4:].max():.3g} mean {d[:, 4:].mean():.3g} (reference {fl[2]:.3g} / {fl[3]:.3g})")
    half_bars(d, fl[0], fl[1], fl[2], fl[3])


def test_x_1280_c5_bench_shape(gpu):
    """C5's own configuration (v11_x, bf16, 1280x1280, batch 16): the per-shape tuner's plans
    at batch 16 give every image exactly its batch-1 output (one reduction order for every
    plan), and image 0 is within the reference's own bf16 deviation of the subsampled float64
    golden (the bar above, as the batch-1 test)."""
    from _util import detection_match
    from yolo_hip.engine import nms
    g = load_golden("forward_x_1280_b1_sub.npz")
    idx = torch.from_numpy(g["idx"])
    ref = g["y_sub"].astype(np.float64)
    x0 = synth.synth_scenes(1, 1280, 1280, seed=GOLDEN_INPUT_SEED)
    rest = synth.synth_scenes(15, 1280, 1280, seed=31)
    x = torch.cat([x0, rest]).to(gpu, torch.bfloat16)
    eng = _engine(make_model("x"), torch.bfloat16, gpu)
    y = eng.forward(x).clone()
    assert torch.isfinite(y.float()).all()
    for i in (0, 7, 15):
        y1 = eng.forward(x[i:i + 1].contiguous())
        assert torch.equal(y1[0], y[i]), f"image {i}: batch-16 plans differ from batch-1"
    d = np.abs(y[:1, :, idx].float().cpu().double().numpy() - ref)
    fl = [float(v) for v in g["dev_bf16"]]
    print(f"v11_x@1280 bf16 b16 image 0: box max {d[:, :4].max():.3g} mean {d[:, :4].mean():.3g} (reference "
          f"{fl[0]:.3g} / {fl[1]:.3g}); cls max {d[:, 4:].max():.3g} mean {d[:, 4:].mean():.3g}")
    half_bars(d, fl[0], fl[1], fl[2], fl[3])
    dets, counts = nms(y[:1])
    want = g["dets"][:int(g["counts"][0])]
    m50, miou = detection_match(dets[0, :counts[0]].cpu().numpy(), want)
    # bar: the reference algorithm in bf16 on the CPU (oracle forward + NMS) matches 0.73 / 0.59 of
    # the float64 golden's top 100, and 0.67-0.75 / 0.54-0.59 when ~0.01 % of the bf16 input
    # values move by one ulp (tests/golden/x1280_bf16_ref_match.json, oracle/make_x1280_half_match.py):
    # bf16 v11_x at 1280 is chaotic with the synthetic weights. The device must do no worse than
    # the worst of those equally valid bf16 runs.
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "x1280_bf16_ref_match.json")) as f:
        ref = json.load(f)["bf16"]
    print(f"v11_x@1280 bf16 b16 detections: match@0.5 {m50:.3f} mean IoU {miou:.4f} (reference bf16 "
          f"{ref['match50']:.3f} / {ref['mean_iou']:.3f}, 1-ulp spread {min(ref['perturbed_match50']):.2f}-"
          f"{max(ref['perturbed_match50']):.2f})")
    assert m50 >= min(ref["perturbed_match50"]) and miou >= min(ref["perturbed_mean_iou"]), (m50, miou)


def test_n_bf16_c2_bench_shape(gpu):
    """C2's own configuration (v11_n, bf16, 640x640, batch 32, the headline bench), image 0 = the
    golden's input: the per-shape tuner's plans and the batch-32 fused-kernel choices (c3k,
    head_cls, K-split) give images 0, 17 and 31 exactly their batch-1 outputs, image 0 is within
    the reference's own bf16 deviation of the float64 golden (forward_n_640_b1.npz), and its
    post-NMS detections match the golden's as well as the reference algorithm run in bf16 does."""
    from _util import detection_match, oracle_for
    from oracle import nms as onms
    from yolo_hip.engine import nms
    g = load_golden(golden_name("n", 640, 1))
    x0 = synth.synth_scenes(1, 640, 640, seed=GOLDEN_INPUT_SEED)
    rest = synth.synth_scenes(31, 640, 640, seed=41)
    x = torch.cat([x0, rest]).to(gpu, torch.bfloat16)
    eng = _engine(make_model("n"), torch.bfloat16, gpu)
    y = eng.forward(x).clone()
    assert torch.isfinite(y.float()).all()
    for i in (0, 17, 31):
        y1 = eng.forward(x[i:i + 1].contiguous())
        assert torch.equal(y1[0], y[i]), f"image {i}: batch-32 plans differ from batch-1"
    ref = g["y"].astype(np.float64)
    d = np.abs(y[:1].float().cpu().double().numpy() - ref)
    fl = [float(v) for v in g["dev_bf16"]]
    print(f"v11_n@640 bf16 b32 image 0: box max {d[:, :4].max():.3g} mean {d[:, :4].mean():.3g} (reference "
          f"{fl[0]:.3g} / {fl[1]:.3g}); cls max {d[:, 4:].max():.3g} mean {d[:, 4:].mean():.3g}")
    half_bars(d, fl[0], fl[1], fl[2], fl[3])
    want = onms.non_max_suppression(g["y"].astype(np.float32))[0]
    dets, counts = nms(y[:1])
    m50, miou = detection_match(dets[0, :counts[0]].cpu().numpy(), want)
    ref_half = oracle_for("n", torch.bfloat16)(x0.to(torch.bfloat16)).float().numpy()
    r50, riou = detection_match(onms.non_max_suppression(ref_half, half=torch.bfloat16)[0], want)
    print(f"v11_n@640 bf16 b32 detections: match@0.5 {m50:.3f} mean IoU {miou:.4f} (reference bf16 {r50:.3f} / {riou:.4f})")
    assert m50 >= min(0.99, r50) - 0.03 and miou >= min(0.99, riou) - 0.03
