"""Two-stream DetectPipeline (forward k+1 beside NMS k), and with two forward lanes
(forwards of consecutive batches overlap on two engines), vs the sequential schedule,
at the bench's full size (v11_n, 640x640, batch 32, bf16). Marked gpu.

Bar: bit-identical detections and counts for every batch - the pipeline only
reorders independent work across streams. Plus the on-device NMS of a full
bench batch against the CPU oracle on the same head output (bit-exact).
"""
import numpy as np
import pytest
import torch

from oracle import nms as onms
from yolo_hip import synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine(gpu):
    from nets import nn
    from yolo_hip.engine import Engine
    torch.manual_seed(0)
    model = nn.yolo_v11_n(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    eng = Engine(*model._yh_arch, gpu, torch.bfloat16)
    eng.load_module(model)
    return eng


def test_pipeline_equals_sequential(gpu, engine):
    from yolo_hip.engine import nms
    from yolo_hip.pipeline import DetectPipeline
    B, S = 32, 640
    xs = [synth.synth_scenes(B, S, S, seed=200 + i).to(gpu, torch.bfloat16) for i in range(3)]
    want = []
    for x in xs:
        y = engine.forward(x)
        d, c = nms(y)
        want.append((d.cpu(), c.cpu()))
    pipe = DetectPipeline(engine, B, S, S)
    got = [pipe.submit(x) for x in xs + xs[:1]]   # 4 batches: buffer reuse is exercised
    torch.cuda.synchronize()
    for i, (d, c, _, _) in enumerate(got):
        wd, wc = want[i % 3]
        assert torch.equal(c.cpu(), wc), f"batch {i}: counts differ"
        for j, k in enumerate(wc.tolist()):
            assert torch.equal(d[j, :k].cpu(), wd[j, :k]), f"batch {i} image {j}"


def test_two_lane_pipeline_equals_sequential(gpu, engine):
    from nets import nn
    from yolo_hip.engine import Engine, nms
    from yolo_hip.pipeline import DetectPipeline
    B, S = 32, 640
    torch.manual_seed(0)
    model = nn.yolo_v11_n(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    lane1 = Engine(*model._yh_arch, gpu, torch.bfloat16)
    lane1.load_module(model)
    xs = [synth.synth_scenes(B, S, S, seed=210 + i).to(gpu, torch.bfloat16) for i in range(3)]
    want = []
    for x in xs:
        d, c = nms(engine.forward(x))
        want.append((d.cpu(), c.cpu()))
    pipe = DetectPipeline([engine, lane1], B, S, S)
    got = [pipe.submit(x) for x in xs + xs]   # 6 batches over 2 lanes and 4 head buffers
    pipe.drain()
    torch.cuda.synchronize()
    for i, (d, c, _, _) in enumerate(got):
        wd, wc = want[i % 3]
        assert torch.equal(c.cpu(), wc), f"batch {i}: counts differ"
        for j, k in enumerate(wc.tolist()):
            assert torch.equal(d[j, :k].cpu(), wd[j, :k]), f"batch {i} image {j}"


def test_full_batch_nms_matches_oracle(gpu, engine):
    from yolo_hip.engine import nms
    x = synth.synth_scenes(32, 640, 640, seed=300).to(gpu, torch.bfloat16)
    y = engine.forward(x)
    d, c = nms(y)
    d, c = d.cpu().numpy(), c.cpu().tolist()
    want = onms.non_max_suppression(y.float().cpu().numpy(), half=torch.bfloat16)
    assert len(want) == 32
    for j, w in enumerate(want):
        assert c[j] == w.shape[0], f"image {j}: kept {c[j]} vs {w.shape[0]}"
        np.testing.assert_array_equal(d[j, :c[j]], w, err_msg=f"image {j}")
