"""Eval preprocessing of the loader (the data format before the
path): the library's host letterbox (yh_letterbox_host, yh_resize_linear_host) against
the numpy restatement in oracle/preprocess.py (bit-exact), that restatement against
torch's half-pixel bilinear resize (within one grey level: cv2 itself is absent, so
parity with cv2 is unpinned), and the drop-in utils.dataset on a small on-disk set.
The device kernel (yh_letterbox) is pinned to the host path in test_gpu_preprocess.py.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import preprocess as opre
from yolo_hip import preprocess as pre

from conftest import GOLD

SHAPES = [(480, 640, 640), (1000, 750, 640), (300, 200, 640), (1280, 1280, 640), (1280, 960, 640),
          (1279, 853, 640), (17, 23, 64), (640, 640, 640), (720, 1280, 640), (33, 1000, 320), (2, 3, 64),
          (1, 1, 32), (427, 640, 640), (640, 427, 640), (5000, 40, 640)]


def _img(h, w, seed):
    rng = np.random.default_rng(seed)
    base = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    if h > 4 and w > 4:   # smooth gradients + noise: exercises rounding at every level
        yy, xx = np.mgrid[0:h, 0:w]
        base[..., 0] = ((xx * 255) // max(1, w - 1)).astype(np.uint8)
    return base


def test_geometry_matches_restatement():
    for h in (1, 2, 31, 320, 427, 479, 480, 481, 639, 640, 641, 1000, 1279, 4000):
        for w in (1, 3, 64, 333, 640, 853, 1280, 3000):
            for s in (32, 320, 640, 1280):
                want = opre.geometry(h, w, s)
                if min(want[:2]) < 1:   # the reference's cv2.resize would reject a 0-pixel side
                    with pytest.raises(RuntimeError):
                        pre.geometry(h, w, s)
                    continue
                assert pre.geometry(h, w, s) == want, (h, w, s)


@pytest.mark.parametrize("h,w,s", SHAPES)
def test_host_letterbox_bit_exact_vs_restatement(h, w, s):
    img = _img(h, w, h * 7 + w)
    want = opre.letterbox(img, s)
    assert np.array_equal(pre.letterbox_host(img, s), want)
    assert np.array_equal(pre.letterbox_host(img, s, threads=4), want)
    # strided source (a crop of a wider buffer)
    wide = np.zeros((h, w + 5, 3), dtype=np.uint8)
    wide[:, :w] = img
    assert np.array_equal(pre.letterbox_host(wide[:, :w], s), want)


@pytest.mark.parametrize("h,w,nh,nw", [(480, 640, 240, 320), (480, 640, 479, 641), (100, 100, 37, 211),
                                       (7, 9, 640, 480), (640, 480, 640, 480)])
def test_resize_linear_host_vs_restatement_and_torch(h, w, nh, nw):
    img = _img(h, w, 3)
    got = pre.resize_linear_host(img, nh, nw)
    assert np.array_equal(got, opre.resize_linear(img, nh, nw))
    if (h, w) != (2 * nh, 2 * nw):
        t = torch.from_numpy(img).permute(2, 0, 1)[None].float()
        ref = F.interpolate(t, size=(nh, nw), mode="bilinear", align_corners=False)[0].permute(1, 2, 0)
        assert (torch.from_numpy(got).float() - ref).abs().max().item() <= 1.0 + 1e-3


def test_restatement_within_one_level_of_torch_bilinear():
    for h, w, s in SHAPES:
        img = _img(h, w, 11)
        nh, nw, top, left = opre.geometry(h, w, s)
        if (h, w) == (2 * nh, 2 * nw):
            continue
        t = torch.from_numpy(img).permute(2, 0, 1)[None].float()
        ref = F.interpolate(t, size=(nh, nw), mode="bilinear", align_corners=False)[0].flip(0)
        got = torch.from_numpy(opre.letterbox(img, s)[:, top:top + nh, left:left + nw].astype(np.float32))
        assert (got - ref).abs().max().item() <= 1.0 + 1e-3, (h, w, s)


def test_average_meter():
    from utils import util
    m = util.AverageMeter()
    m.update(2.0, 3)
    m.update(float("nan"), 5)
    m.update(4.0, 1)
    assert m.num == 4 and m.avg == pytest.approx(2.5)


def _write_set(root, shapes):
    from PIL import Image
    imgs, files = [], []
    os.makedirs(os.path.join(root, "images", "val"), exist_ok=True)
    os.makedirs(os.path.join(root, "labels", "val"), exist_ok=True)
    for i, (h, w) in enumerate(shapes):
        rgb = _img(h, w, 100 + i)[:, :, ::-1]
        fn = os.path.join(root, "images", "val", f"{i:03d}.png")
        Image.fromarray(np.ascontiguousarray(rgb)).save(fn)
        with open(os.path.join(root, "labels", "val", f"{i:03d}.txt"), "w") as f:
            for row in _labels_of(i):   # every third image has no labels
                f.write(" ".join(str(v) for v in row) + "\n")
        imgs.append(np.ascontiguousarray(rgb[:, :, ::-1]))
        files.append(fn)
    return files, imgs


def test_dataset_eval_items(tmp_path):
    """dataset.py:30-90 (augment=False): (sample, cls, box, zeros(n)); the sample is the letterbox
    (load_image + resize + CHW/RGB), the labels are moved onto the letterboxed canvas."""
    from utils import dataset
    shapes = [(480, 640), (640, 427), (300, 300), (1280, 960), (200, 640)]
    files, imgs = _write_set(str(tmp_path), shapes)
    ds = dataset.Dataset(files, 640, {}, augment=False)
    assert len(ds) == len(files)
    for i in range(len(ds)):
        sample, cls, box, idx = ds[i]
        assert sample.dtype == torch.uint8 and sample.shape == (3, 640, 640)
        assert np.array_equal(sample.numpy(), opre.letterbox(imgs[i], 640))
        # the reference's two-step route: load_image, resize (pad), CHW + BGR->RGB
        im, (h0, w0) = ds.load_image(i)
        assert (h0, w0) == shapes[i]
        padded, ratio, pad = dataset.resize(im, 640, False)
        assert ratio == (1.0, 1.0)
        assert np.array_equal(np.ascontiguousarray(padded.transpose(2, 0, 1)[::-1]), sample.numpy())
        assert np.array_equal(ds.raw(i).numpy(), imgs[i])
        # labels: class column + normalised (cx, cy, w, h) on the 640 canvas
        want = _expected_targets(shapes[i], _labels_of(i), 640)
        assert cls.shape == (len(want), 1) and box.shape == (len(want), 4) and idx.shape == (len(want),)
        assert torch.equal(idx, torch.zeros(len(want)))
        if len(want):
            np.testing.assert_array_equal(cls.numpy()[:, 0], want[:, 0])
            np.testing.assert_allclose(box.numpy(), want[:, 1:], rtol=0, atol=2e-6)
    with pytest.raises(NotImplementedError):
        dataset.Dataset(files, 640, {}, augment=True)


def _labels_of(i):
    return [] if i % 3 == 2 else [(i % 80, 0.5, 0.5, 0.25, 0.4), (3, 0.2, 0.3, 0.1, 0.1)]


def _expected_targets(shape, labels, S):
    """Restatement of the label path of dataset.py:45-61 for eval: the image is scaled by
    S / max(h, w) (int sizes, load_image), never enlarged, centred with a zero border (resize);
    a normalised label maps to pixels on that canvas, is clipped to [0, S - 1e-3] and
    re-normalised by S. float64 here, float32 in the loader."""
    h0, w0 = shape
    r0 = S / max(h0, w0)
    h, w = (int(h0 * r0), int(w0 * r0)) if r0 != 1 else (h0, w0)
    r = min(S / h, S / w, 1.0)
    dw, dh = (S - round(w * r)) / 2, (S - round(h * r)) / 2
    out = []
    for c, cx, cy, bw, bh in labels:   # file order (numpy.unique's sorted order only when rows repeat)
        x1 = min(max(r * w * (cx - bw / 2) + dw, 0), S - 1e-3)
        x2 = min(max(r * w * (cx + bw / 2) + dw, 0), S - 1e-3)
        y1 = min(max(r * h * (cy - bh / 2) + dh, 0), S - 1e-3)
        y2 = min(max(r * h * (cy + bh / 2) + dh, 0), S - 1e-3)
        out.append((c, (x1 + x2) / 2 / S, (y1 + y2) / 2 / S, (x2 - x1) / S, (y2 - y1) / S))
    return np.array(out, dtype=np.float64).reshape(-1, 5)


def test_load_label_rules(tmp_path):
    """dataset.py:195-236: duplicate rows dropped, malformed label files and tiny images skipped,
    a missing label file gives no labels."""
    from PIL import Image
    from utils import dataset
    root = str(tmp_path)
    os.makedirs(os.path.join(root, "images", "v"))
    os.makedirs(os.path.join(root, "labels", "v"))
    names = ["dup", "bad", "tiny", "nolabel"]
    files = []
    for n in names:
        fn = os.path.join(root, "images", "v", n + ".png")
        size = (8, 8) if n == "tiny" else (32, 24)
        Image.fromarray(np.zeros((size[1], size[0], 3), dtype=np.uint8)).save(fn)
        files.append(fn)
    with open(os.path.join(root, "labels", "v", "dup.txt"), "w") as f:
        f.write("1 0.5 0.5 0.2 0.2\n0 0.1 0.1 0.1 0.1\n1 0.5 0.5 0.2 0.2\n")
    with open(os.path.join(root, "labels", "v", "bad.txt"), "w") as f:
        f.write("1 0.5 0.5 1.2 0.2\n")
    got = dataset.Dataset.load_label(files)
    assert list(got) == [files[0], files[3]]
    np.testing.assert_array_equal(got[files[0]], np.array([[0, .1, .1, .1, .1], [1, .5, .5, .2, .2]], np.float32))
    assert got[files[3]].shape == (0, 5)


def test_collate_fn_targets():
    """dataset.py:178-193: labels concatenated, 'idx' = the image's position in the batch."""
    from utils import dataset
    items = []
    for n in (2, 0, 3):
        items.append((torch.full((3, 4, 4), n, dtype=torch.uint8), torch.arange(n, dtype=torch.float32)[:, None],
                      torch.rand(n, 4), torch.zeros(n)))
    x, t = dataset.Dataset.collate_fn(items)
    assert x.shape == (3, 3, 4, 4) and x[2, 0, 0, 0] == 3
    assert t['idx'].tolist() == [0, 0, 2, 2, 2]
    assert t['cls'][:, 0].tolist() == [0, 1, 0, 1, 2]
    assert torch.equal(t['box'], torch.cat([it[2] for it in items]))
