"""main.py:test (224-304) through the drop-in modules on the CPU: Dataset + DataLoader with
Dataset.collate_fn (main.py:232-234), the loop body (264-294) with the model, the library's
host NMS (utils.util.non_max_suppression on CPU tensors -> yh_nms_host), compute_metric, and
compute_ap (297-299). The labels are the model's own top detections, clipped to the image
area and written back as YOLO label files in original-image coordinates; inside the loop the
targets main.py builds (`util.wh2xy(box) * scale`) must land on those boxes again. This checks
the label geometry (letterbox scale + border, normalisation) end to end, not only that it runs.
(The synthetic weights' boxes are large, so most cross the image edge: clipped labels are not
IoU-1 copies of the detections, and the mAP itself is only required to be positive.)"""
import os

import numpy as np
import torch
from torch.utils import data

from yolo_hip import synth


def _write_images(root, shapes):
    from PIL import Image
    os.makedirs(os.path.join(root, "images", "val"), exist_ok=True)
    os.makedirs(os.path.join(root, "labels", "val"), exist_ok=True)
    files = []
    for i, (h, w) in enumerate(shapes):
        x = synth.synth_scenes(1, h, w, seed=40 + i)[0]          # (3, h, w) RGB in [0, 1)
        rgb = (x.permute(1, 2, 0) * 255).round().clamp(0, 255).to(torch.uint8).numpy()
        fn = os.path.join(root, "images", "val", f"{i:03d}.png")
        Image.fromarray(rgb).save(fn)
        files.append(fn)
    return files


def test_main_test_loop_on_cpu(tmp_path):
    from nets import nn
    from utils import util
    from utils.dataset import Dataset

    S = 256
    shapes = [(192, 256), (256, 160), (400, 320), (128, 128), (256, 256)]
    files = _write_images(str(tmp_path), shapes)

    torch.manual_seed(0)
    model = nn.yolo_v11_n(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model = model.fuse().eval()

    # pass 1: the model's top-3 detections per image -> label files in original-image coordinates
    ds0 = Dataset(files, S, {}, augment=False)
    want_boxes = []
    for i, fn in enumerate(files):
        sample = ds0[i][0]
        with torch.no_grad():
            out = util.non_max_suppression(model(sample[None].float() / 255.))[0]
        h0, w0 = shapes[i]
        r0 = S / max(h0, w0)
        h, w = (int(h0 * r0), int(w0 * r0)) if r0 != 1 else (h0, w0)
        r = min(S / h, S / w, 1.0)
        dw, dh = (S - round(w * r)) / 2, (S - round(h * r)) / 2
        out = out[:3]
        x1 = ((out[:, 0] - dw) / (r * w)).clamp(0, 1)
        x2 = ((out[:, 2] - dw) / (r * w)).clamp(0, 1)
        y1 = ((out[:, 1] - dh) / (r * h)).clamp(0, 1)
        y2 = ((out[:, 3] - dh) / (r * h)).clamp(0, 1)
        with open(fn.replace("images", "labels").rsplit(".", 1)[0] + ".txt", "w") as f:
            for c, a, b, c2, d in zip(out[:, 5].tolist(), x1.tolist(), y1.tolist(), x2.tolist(), y2.tolist()):
                f.write(f"{int(c)} {(a + c2) / 2:.6f} {(b + d) / 2:.6f} {c2 - a:.6f} {d - b:.6f}\n")
        clipped = torch.stack((x1 * r * w + dw, y1 * r * h + dh, x2 * r * w + dw, y2 * r * h + dh), 1)
        want_boxes.append((out[:, 5], clipped))

    # pass 2: main.py:232-234 and the loop of 264-299, CPU device
    dataset = Dataset(files, S, {}, augment=False)
    loader = data.DataLoader(dataset, batch_size=4, shuffle=False, num_workers=0, collate_fn=Dataset.collate_fn)
    iou_v = torch.linspace(start=0.5, end=0.95, steps=10)
    n_iou = iou_v.numel()
    metrics, n_batches = [], 0
    with torch.no_grad():
        for samples, targets in loader:
            n_batches += 1
            samples = samples.float() / 255.
            _, _, h, w = samples.shape
            scale = torch.tensor((w, h, w, h))
            outputs = util.non_max_suppression(model(samples))
            for i, output in enumerate(outputs):
                idx = targets['idx'] == i
                cls = targets['cls'][idx]
                box = targets['box'][idx]
                metric = torch.zeros(output.shape[0], n_iou, dtype=torch.bool)
                if output.shape[0] == 0:
                    if cls.shape[0]:
                        metrics.append((metric, *torch.zeros((2, 0)), cls.squeeze(-1)))
                    continue
                wc, wb = want_boxes[4 * (n_batches - 1) + i]
                assert torch.equal(cls[:, 0], wc)
                # the canvas corners main.py compares against: within the labels' 6-digit text
                # (1e-6 of a side) plus xy2wh's 1e-3 px clip at the canvas edge
                assert (util.wh2xy(box) * scale - wb).abs().max().item() < 2e-3
                if cls.shape[0]:
                    target = torch.cat(tensors=(cls, util.wh2xy(box) * scale), dim=1)
                    metric = util.compute_metric(output[:, :6], target, iou_v)
                metrics.append((metric, output[:, 4], output[:, 5], cls.squeeze(-1)))
    assert n_batches == 2
    metrics = [torch.cat(x, dim=0).cpu().numpy() for x in zip(*metrics)]
    assert metrics[0].any()
    tp, fp, m_pre, m_rec, map50, mean_ap = util.compute_ap(*metrics, plot=False, names={})
    assert 0 < m_rec <= 1 and 0 < map50 <= 1 and 0 < mean_ap <= map50, (m_pre, m_rec, map50, mean_ap)
    assert tp.shape == fp.shape and np.isfinite(mean_ap)
