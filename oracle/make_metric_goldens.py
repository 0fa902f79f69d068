"""Golden fixture for the eval metrics: the reference's own
compute_metric (utils/util.py:99-120) and compute_ap (utils/util.py:225-300) run
in this container on a synthetic detection set (never on the GPU box).

  tests/golden/metrics_synth.npz
      per image i: out_<i> (D, 6) detections [x1, y1, x2, y2, score, cls] and
      tgt_<i> (L, 5) labels [cls, x1, y1, x2, y2]; correct_<i> (D, 10) the
      reference's compute_metric; ap_* the reference's compute_ap over the
      concatenation main.py:296-299 builds.

Detections are jittered copies of the labels (some with the wrong class, some
duplicated, so the greedy matching has work to do) plus random false
positives; scores are distinct (the reference's argsort is unstable on ties).

Usage: PYTHONDONTWRITEBYTECODE=1 python oracle/make_metric_goldens.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True
GOLD = os.path.join(ROOT, "tests", "golden")


def synth_set(n_img=24, seed=0):
    rng = np.random.default_rng(seed)
    imgs = []
    used = set()
    for _ in range(n_img):
        L = int(rng.integers(0, 12))
        c = rng.integers(0, 6, L).astype(np.float32)
        xy = rng.uniform(0, 560, (L, 2))
        wh = rng.uniform(8, 160, (L, 2))
        tgt = np.concatenate([c[:, None], xy, xy + wh], 1).astype(np.float32)
        dets = []
        for k in range(L):
            for _ in range(int(rng.integers(0, 3))):       # 0..2 detections per label
                j = rng.normal(0, 0.08, 4) * np.concatenate([wh[k], wh[k]])
                box = tgt[k, 1:] + j
                cls = c[k] if rng.uniform() < 0.85 else float(rng.integers(0, 6))
                dets.append(np.concatenate([box, [0.0, cls]]))
        for _ in range(int(rng.integers(0, 6))):           # false positives
            xy0 = rng.uniform(0, 560, 2)
            dets.append(np.concatenate([xy0, xy0 + rng.uniform(8, 160, 2), [0.0, float(rng.integers(0, 6))]]))
        out = np.array(dets, dtype=np.float32).reshape(-1, 6)
        for d in range(out.shape[0]):                        # distinct scores
            while True:
                s = np.float32(rng.uniform(0.001, 1.0))
                if s not in used:
                    used.add(s)
                    out[d, 4] = s
                    break
        out = out[np.argsort(-out[:, 4], kind="stable")]
        imgs.append((out, tgt))
    return imgs


def main():
    from oracle.make_goldens import import_reference
    _, ref_util = import_reference()
    iou_v = torch.linspace(0.5, 0.95, 10)
    rec = {}
    metrics = []
    for i, (out, tgt) in enumerate(synth_set()):
        o, t = torch.from_numpy(out), torch.from_numpy(tgt)
        rec[f"out_{i}"] = out
        rec[f"tgt_{i}"] = tgt
        metric = torch.zeros(o.shape[0], 10, dtype=torch.bool)
        if o.shape[0] == 0:
            if t.shape[0]:
                metrics.append((metric, *torch.zeros((2, 0)), t[:, 0]))
            rec[f"correct_{i}"] = metric.numpy()
            continue
        if t.shape[0]:
            metric = ref_util.compute_metric(o, t, iou_v)
        rec[f"correct_{i}"] = metric.numpy()
        metrics.append((metric, o[:, 4], o[:, 5], t[:, 0]))
    cat = [torch.cat(x, dim=0).numpy() for x in zip(*metrics)]
    tp, fp, m_pre, m_rec, map50, mean_ap = ref_util.compute_ap(*cat, plot=False, names={})
    rec.update(ap_tp=tp, ap_fp=fp, ap_scalars=np.array([m_pre, m_rec, map50, mean_ap]), n_img=np.array(len(synth_set())))
    np.savez_compressed(os.path.join(GOLD, "metrics_synth.npz"), **rec)
    print(f"mAP50 {map50:.4f}  mAP {mean_ap:.4f}  P {m_pre:.4f}  R {m_rec:.4f}")


if __name__ == "__main__":
    main()
