"""Eval-mode drop-in for the reference's loader `utils/dataset.py`.

main.py:test builds `Dataset(filenames, input_size, params, augment=False)` and a
`DataLoader(..., collate_fn=Dataset.collate_fn)` (main.py:232-234), then reads
`targets['idx' / 'cls' / 'box']` per image (main.py:276-278). This module keeps that
contract for eval:

  Dataset.__getitem__   dataset.py:30-90 (augment=False branch): (sample, cls, box, idx)
                        sample (3, S, S) uint8 RGB letterbox, cls (n, 1), box (n, 4)
                        normalised (cx, cy, w, h) on the letterboxed canvas, idx zeros(n)
  Dataset.collate_fn    dataset.py:178-193: stacked samples + {'cls', 'box', 'idx'}, idx = the
                        image's position in the batch
  Dataset.load_label    dataset.py:195-236: PIL-verified images, YOLO .txt labels from the
                        sibling `labels/` directory, rows de-duplicated
  load_image            dataset.py:95-103: r = input_size / max(h, w), INTER_LINEAR to
                        (int(w r), int(h r)) when r != 1
  resize                dataset.py:292-313 (augment=False): shrink only, centred zero border
  wh2xy / xy2wh         dataset.py:239-262: label box conversions (xy2wh clips in place)

The pixel arithmetic is the library's C++ (yh_letterbox_host / yh_resize_linear_host, the
same __host__ __device__ code as the device kernel yh_letterbox). Deliberate differences:
the label table is not cached to `<dir>.cache` (the reference pickles it with torch.save and
reads it back with weights_only=False; reading the .txt files again is cheap and executes
nothing), and images are decoded with PIL instead of cv2 (absent here; JPEG decoders may
differ in the last bit - parity with cv2.imread is unpinned). Training (augment=True:
mosaic, mix-up, random perspective, HSV, flips, Albumentations) is out of scope and raises.
"""
import os

import numpy
import torch
from torch.utils import data

from yolo_hip import preprocess

FORMATS = 'bmp', 'dng', 'jpeg', 'jpg', 'mpo', 'png', 'tif', 'tiff', 'webp'


def read_bgr(filename):
    """The decoded image as cv2.imread returns it, (h, w, 3) uint8 BGR, EXIF orientation applied."""
    from PIL import Image, ImageOps
    with Image.open(filename) as im:
        rgb = numpy.asarray(ImageOps.exif_transpose(im).convert("RGB"))
    return numpy.ascontiguousarray(rgb[:, :, ::-1])


def _pad_geometry(h, w, input_size):
    """resize()'s arithmetic (dataset.py:297-311) without the pixels: scale r, the resized
    (new_w, new_h), the float half-paddings (dw, dh) and the integer (top, left) border."""
    r = min(input_size / h, input_size / w, 1.0)
    nw, nh = int(round(w * r)), int(round(h * r))
    dw, dh = (input_size - nw) / 2, (input_size - nh) / 2
    return r, nw, nh, dw, dh, int(round(dh - 0.1)), int(round(dw - 0.1))


def resize(image, input_size, augment):
    """dataset.py:292-313 with augment=False: shrink only (INTER_LINEAR), then a zero border that
    centres the image on an input_size square. Returns (canvas, (r, r), (dw, dh))."""
    if augment:
        raise NotImplementedError("resize(augment=True) draws a random interpolation (training only)")
    h, w = image.shape[:2]
    r, nw, nh, dw, dh, top, left = _pad_geometry(h, w, input_size)
    if (nh, nw) != (h, w):
        image = preprocess.resize_linear_host(image, nh, nw)
    canvas = numpy.zeros((nh + top + int(round(dh + 0.1)), nw + left + int(round(dw + 0.1)), 3), dtype=numpy.uint8)
    canvas[top:top + nh, left:left + nw] = image
    return canvas, (r, r), (dw, dh)


def wh2xy(x, w=640, h=640, pad_w=0, pad_h=0):
    """Normalised (cx, cy, bw, bh) rows -> pixel corners (x1, y1, x2, y2) on a w x h image placed
    at (pad_w, pad_h) (dataset.py:239-247)."""
    y = numpy.copy(x)
    half_w, half_h = x[:, 2] / 2, x[:, 3] / 2
    y[:, 0] = w * (x[:, 0] - half_w) + pad_w
    y[:, 1] = h * (x[:, 1] - half_h) + pad_h
    y[:, 2] = w * (x[:, 0] + half_w) + pad_w
    y[:, 3] = h * (x[:, 1] + half_h) + pad_h
    return y


def xy2wh(x, w, h):
    """Pixel corners -> normalised (cx, cy, bw, bh) on a w x h canvas (dataset.py:250-262). As in
    the reference the corners are first clipped IN PLACE to [0, w - 1e-3] / [0, h - 1e-3]."""
    x[:, [0, 2]] = x[:, [0, 2]].clip(0, w - 1E-3)
    x[:, [1, 3]] = x[:, [1, 3]].clip(0, h - 1E-3)
    y = numpy.copy(x)
    y[:, 0] = (x[:, 0] + x[:, 2]) / 2 / w
    y[:, 1] = (x[:, 1] + x[:, 3]) / 2 / h
    y[:, 2] = (x[:, 2] - x[:, 0]) / w
    y[:, 3] = (x[:, 3] - x[:, 1]) / h
    return y


def _label_path(filename):
    """<root>/images/<split>/<name>.<ext> -> <root>/labels/<split>/<name>.txt (dataset.py:212-214:
    the last `/images/` path component becomes `/labels/`, the extension `.txt`)."""
    a, b = f'{os.sep}images{os.sep}', f'{os.sep}labels{os.sep}'
    return b.join(filename.rsplit(a, 1)).rsplit('.', 1)[0] + '.txt'


def _read_label(filename):
    """(n, 5) float32 [class, cx, cy, w, h] rows of an image, or raises AssertionError for a label
    file the reference rejects (negative values, not 5 columns, coordinates above 1)."""
    path = _label_path(filename)
    if not os.path.isfile(path):
        return numpy.zeros((0, 5), dtype=numpy.float32)
    with open(path) as f:
        rows = [line.split() for line in f.read().strip().splitlines() if len(line)]
    label = numpy.array(rows, dtype=numpy.float32)
    if not len(label):
        return numpy.zeros((0, 5), dtype=numpy.float32)
    assert (label >= 0).all(), f'{path}: negative label values'
    assert label.shape[1] == 5, f'{path}: labels need 5 columns'
    assert (label[:, 1:] <= 1).all(), f'{path}: non-normalised coordinates'
    _, first = numpy.unique(label, axis=0, return_index=True)
    if len(first) < len(label):   # duplicate rows dropped (kept in numpy.unique's sorted order)
        label = label[first]
    return label


class Dataset(data.Dataset):
    """The reference's eval dataset: item i is (sample, cls, box, idx) with the letterboxed uint8
    RGB sample and the image's labels on the letterboxed canvas. `raw(i)` returns the decoded
    BGR image instead, for loops that letterbox whole batches on the device
    (yolo_hip.preprocess.letterbox, one kernel per batch)."""

    def __init__(self, filenames, input_size, params=None, augment=False):
        if augment:
            raise NotImplementedError("Dataset(augment=True) is the training pipeline (mosaic, mix-up, random "
                                      "perspective, HSV, flips): use the reference's loader for training")
        self.params = params
        self.mosaic = self.augment = False
        self.input_size = input_size
        labels = self.load_label(filenames)
        self.labels = list(labels.values())
        self.filenames = list(labels.keys())
        self.n = len(self.filenames)
        self.indices = range(self.n)

    def __len__(self):
        return len(self.filenames)

    def load_image(self, i):
        """(resized BGR image, (h0, w0)): dataset.py:95-103 with INTER_LINEAR (eval)."""
        image = read_bgr(self.filenames[i])
        h, w = image.shape[:2]
        r = self.input_size / max(h, w)
        if r != 1:
            image = preprocess.resize_linear_host(image, int(h * r), int(w * r))
        return image, (h, w)

    def __getitem__(self, index):
        index = self.indices[index]
        image = read_bgr(self.filenames[index])
        S = self.input_size
        # load_image's size, then resize()'s scale and border; the pixels of both steps come from
        # one call (yh_letterbox_host, bit-identical to load_image + resize: tests/test_preprocess.py)
        h0, w0 = image.shape[:2]
        r0 = S / max(h0, w0)
        h, w = (int(h0 * r0), int(w0 * r0)) if r0 != 1 else (h0, w0)
        r, _, _, dw, dh, _, _ = _pad_geometry(h, w, S)
        sample = preprocess.letterbox_host(image, S)

        label = self.labels[index].copy()
        if label.size:
            label[:, 1:] = wh2xy(label[:, 1:], r * w, r * h, dw, dh)
        nl = len(label)
        cls = label[:, 0:1]
        box = xy2wh(label[:, 1:5], S, S)
        target_cls = torch.from_numpy(cls) if nl else torch.zeros((0, 1))
        target_box = torch.from_numpy(box) if nl else torch.zeros((0, 4))
        return torch.from_numpy(sample), target_cls, target_box, torch.zeros(nl)

    def raw(self, i):
        return torch.from_numpy(read_bgr(self.filenames[i]))

    @staticmethod
    def collate_fn(batch):
        """Stack the samples; concatenate the labels of the batch, each row tagged with the index
        of its image in the batch (dataset.py:178-193; main.py:276 selects rows by it)."""
        samples, cls, box, indices = zip(*batch)
        idx = torch.cat([ind + i for i, ind in enumerate(indices)], dim=0)
        targets = {'cls': torch.cat(cls, dim=0), 'box': torch.cat(box, dim=0), 'idx': idx}
        return torch.stack(samples, dim=0), targets

    @staticmethod
    def load_label(filenames):
        """{filename: (n, 5) labels} for the images that pass the reference's checks (PIL verify,
        both sides > 9 px, a known format, a well-formed label file); others are skipped, a
        missing image or label file gives no labels (dataset.py:195-236). Nothing is cached."""
        from PIL import Image
        out = {}
        for filename in filenames:
            try:
                with open(filename, 'rb') as f:
                    image = Image.open(f)
                    image.verify()
                shape = image.size
                assert (shape[0] > 9) & (shape[1] > 9), f'image size {shape} <10 pixels'
                assert image.format.lower() in FORMATS, f'invalid image format {image.format}'
                label = _read_label(filename)
            except FileNotFoundError:
                label = numpy.zeros((0, 5), dtype=numpy.float32)
            except AssertionError:
                continue
            out[filename] = label
        return out
