"""Eval metrics (yolo_hip.metrics; reference utils/util.py:99-120, 172-177, 225-300)
against the reference's own outputs on a synthetic detection set
(tests/golden/metrics_synth.npz, oracle/make_metric_goldens.py).

compute_metric: bit-exact TP matrices. compute_ap: the scalars within 1e-12
and the per-class TP/FP counts exact. Runs on the CPU; the gpu-marked case runs
the same code on the device.
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from yolo_hip.metrics import compute_ap, compute_metric


def _run(device):
    g = load_golden("metrics_synth.npz")
    iou_v = torch.linspace(0.5, 0.95, 10, device=device)
    metrics = []
    for i in range(int(g["n_img"])):
        out = torch.from_numpy(g[f"out_{i}"]).to(device)
        tgt = torch.from_numpy(g[f"tgt_{i}"]).to(device)
        metric = torch.zeros(out.shape[0], 10, dtype=torch.bool, device=device)
        if out.shape[0] == 0:
            if tgt.shape[0]:
                metrics.append((metric, *torch.zeros((2, 0), device=device), tgt[:, 0]))
            continue
        if tgt.shape[0]:
            metric = compute_metric(out, tgt, iou_v)
        assert metric.device == out.device
        assert np.array_equal(metric.cpu().numpy(), g[f"correct_{i}"]), f"image {i}"
        metrics.append((metric, out[:, 4], out[:, 5], tgt[:, 0]))
    cat = [torch.cat(x, dim=0) for x in zip(*metrics)]
    tp, fp, m_pre, m_rec, map50, mean_ap = compute_ap(*cat)
    assert np.array_equal(tp, g["ap_tp"]) and np.array_equal(fp, g["ap_fp"])
    np.testing.assert_allclose([m_pre, m_rec, map50, mean_ap], g["ap_scalars"], rtol=0, atol=1e-12)
    # numpy inputs, as main.py passes them
    got = compute_ap(*[x.cpu().numpy() for x in cat], device=device)
    np.testing.assert_allclose(got[2:], g["ap_scalars"], rtol=0, atol=1e-12)


def test_metrics_match_reference_cpu():
    _run(torch.device("cpu"))


def test_compute_metric_edge_cases():
    iou_v = torch.linspace(0.5, 0.95, 10)
    out = torch.tensor([[0, 0, 10, 10, 0.9, 1], [0, 0, 10, 10, 0.8, 1], [0, 0, 10, 10, 0.7, 2]])
    tgt = torch.tensor([[1, 0, 0, 10, 10]], dtype=torch.float32)
    m = compute_metric(out.float(), tgt, iou_v)
    # two detections hit the one label at every threshold: only the lower index counts
    assert m[0].all() and not m[1].any() and not m[2].any()
    none = compute_metric(out.float(), torch.zeros((0, 5)), iou_v)
    assert none.shape == (3, 10) and not none.any()


@pytest.mark.gpu
def test_metrics_match_reference_gpu(gpu):
    _run(gpu)
