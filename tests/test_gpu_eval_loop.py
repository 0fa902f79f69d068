"""The reference's eval loop (main.py:test, 264-300) end to end through the drop-in
on the device. Marked gpu.

What main.py does per batch: uint8 samples -> .half() / 255 -> model(samples) ->
util.non_max_suppression -> per image util.compute_metric against the labels ->
util.compute_ap over everything. Here with synthetic weights, scenes and labels:
  * model(x) on the fp16 drop-in equals yolo_hip.Engine.forward on the uint8
    batch (the fused `/255`, yh_forward_u8) bit for bit;
  * the on-device metrics equal the same code run on CPU tensors; the CPU code
    is pinned to the reference by tests/test_metrics.py.
"""
import numpy as np
import pytest
import torch

from yolo_hip import synth

pytestmark = pytest.mark.gpu


def test_reference_eval_loop_on_device(gpu):
    from nets import nn
    from utils import util
    from yolo_hip.engine import Engine

    torch.manual_seed(0)
    model = nn.yolo_v11_n(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model = model.fuse().half().to(gpu).eval()          # main.py:245-252 order

    B, S = 4, 320
    scenes = synth.synth_scenes(B, S, S, seed=21)        # [0, 1) floats
    samples = (scenes * 255).round().clamp(0, 255).to(torch.uint8).to(gpu)

    with torch.no_grad():
        x = samples.half() / 255.                          # main.py:265-267
        outputs = model(x)
    eng = Engine(*model._yh_arch, gpu, torch.float16)
    eng.load_module(model)
    fused = eng.forward(samples)                           # yh_forward_u8
    assert torch.equal(outputs, fused)

    dets = util.non_max_suppression(outputs, 0.001, 0.65)
    assert len(dets) == B and all(d.shape[1] == 6 for d in dets)

    # synthetic labels: jittered copies of a few detections per image
    g = torch.Generator().manual_seed(3)
    iou_v = torch.linspace(0.5, 0.95, 10).to(gpu)
    metrics_dev, metrics_cpu = [], []
    for i, out in enumerate(dets):
        out = out.float()
        k = min(5, out.shape[0])
        tgt = torch.cat([out[:k, 5:6], out[:k, :4] + torch.randn((k, 4), generator=g).to(gpu) * 2.0], 1)
        m_dev = util.compute_metric(out[:, :6], tgt, iou_v)
        m_cpu = util.compute_metric(out[:, :6].cpu(), tgt.cpu(), iou_v.cpu())
        assert m_dev.device == out.device
        assert torch.equal(m_dev.cpu(), m_cpu)
        metrics_dev.append((m_dev, out[:, 4], out[:, 5], tgt[:, 0]))
        metrics_cpu.append((m_cpu, out[:, 4].cpu(), out[:, 5].cpu(), tgt[:, 0].cpu()))
    r_dev = util.compute_ap(*[torch.cat(x, 0) for x in zip(*metrics_dev)])
    r_cpu = util.compute_ap(*[torch.cat(x, 0).numpy() for x in zip(*metrics_cpu)], device="cpu")
    np.testing.assert_allclose(r_dev[2:], r_cpu[2:], rtol=0, atol=1e-12)
    assert r_dev[4] > 0.0                                  # the jittered labels are found
