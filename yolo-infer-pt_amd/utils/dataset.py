"""Drop-in for the eval side of the reference's `utils/dataset.py`.

  Dataset(filenames, input_size, params, augment=False)   dataset.py:14-237
      __getitem__ -> (uint8 (3, S, S) RGB CHW sample, cls (n, 1), box (n, 4)
      normalised cx cy w h, zeros(n)), collate_fn, load_label: as the reference.
      The image is decoded with PIL (cv2 is not a dependency of this build) into
      the BGR HWC array cv2.imread returns, and letterboxed by the library's C++
      host path (yh_letterbox_host: load_image's INTER_LINEAR resize + zero border
      + HWC->CHW, BGR->RGB, dataset.py:95-103, 292-313, 86-88).
      `Dataset.raw(index)` returns the decoded BGR image and its canvas-space
      labels instead, for loops that letterbox whole batches on the device
      (yolo_hip.preprocess.letterbox, one kernel per batch).
  wh2xy, xy2wh, resize (augment=False)                      dataset.py:239-262, 292-313

Training-time augmentation (mosaic, mix-up, random perspective, HSV, flips,
Albumentations) is outside this build's scope: Dataset(augment=True) and those
names raise NotImplementedError. Deliberate difference: the label cache lives in
`<images dir>.labels.npz` (numpy, no pickle) instead of the reference's
torch-pickled `<images dir>.cache` (dataset.py:197-199).
"""
import os

import numpy
import torch
from torch.utils import data

from yolo_hip import preprocess

FORMATS = "bmp", "dng", "jpeg", "jpg", "mpo", "png", "tif", "tiff", "webp"

OUT_OF_SCOPE = ("Albumentations", "augment_hsv", "candidates", "mix_up", "random_perspective", "resample")


def _out_of_scope(name, ref):
    def stub(*args, **kwargs):
        raise NotImplementedError(f"utils.dataset.{name} ({ref} in the reference) is training-time augmentation, "
                                  f"outside this inference build's scope")
    stub.__name__ = stub.__qualname__ = name
    stub.__doc__ = f"Out of scope: the reference's {ref} (training augmentation). Raises NotImplementedError."
    return stub


for _name, _ref in zip(OUT_OF_SCOPE, ("utils/dataset.py:390", "utils/dataset.py:274", "utils/dataset.py:316",
                                      "utils/dataset.py:382", "utils/dataset.py:324", "utils/dataset.py:265")):
    globals()[_name] = _out_of_scope(_name, _ref)
del _name, _ref


def read_bgr(filename):
    """Decoded image as cv2.imread(filename) returns it: (h, w, 3) uint8 BGR, EXIF orientation
    applied (PIL's decoders: JPEG pixels may differ from libjpeg-turbo's by the decoder's IDCT /
    chroma upsampling; parity with cv2.imread itself is unpinned)."""
    from PIL import Image, ImageOps
    with Image.open(filename) as im:
        rgb = numpy.asarray(ImageOps.exif_transpose(im).convert("RGB"))
    return numpy.ascontiguousarray(rgb[:, :, ::-1])


def wh2xy(x, w=640, h=640, pad_w=0, pad_h=0):
    """Normalised (cx, cy, w, h) -> pixel (x1, y1, x2, y2) on a w x h image offset by the padding
    (dataset.py:239-247)."""
    y = numpy.copy(x)
    y[:, 0] = w * (x[:, 0] - x[:, 2] / 2) + pad_w
    y[:, 1] = h * (x[:, 1] - x[:, 3] / 2) + pad_h
    y[:, 2] = w * (x[:, 0] + x[:, 2] / 2) + pad_w
    y[:, 3] = h * (x[:, 1] + x[:, 3] / 2) + pad_h
    return y


def xy2wh(x, w, h):
    """Pixel (x1, y1, x2, y2) clipped in place to the image -> normalised (cx, cy, w, h)
    (dataset.py:250-262)."""
    x[:, [0, 2]] = x[:, [0, 2]].clip(0, w - 1e-3)
    x[:, [1, 3]] = x[:, [1, 3]].clip(0, h - 1e-3)
    y = numpy.copy(x)
    y[:, 0] = ((x[:, 0] + x[:, 2]) / 2) / w
    y[:, 1] = ((x[:, 1] + x[:, 3]) / 2) / h
    y[:, 2] = (x[:, 2] - x[:, 0]) / w
    y[:, 3] = (x[:, 3] - x[:, 1]) / h
    return y


def resize(image, input_size, augment):
    """dataset.py:292-313 for augment=False: scale down only (INTER_LINEAR), zero border to a
    centred input_size square. Returns (image, (r, r), (dw, dh))."""
    if augment:
        raise NotImplementedError("resize(augment=True) uses training-time random interpolation (out of scope)")
    shape = image.shape[:2]
    r = min(input_size / shape[0], input_size / shape[1], 1.0)
    pad = int(round(shape[1] * r)), int(round(shape[0] * r))
    w = (input_size - pad[0]) / 2
    h = (input_size - pad[1]) / 2
    if shape[::-1] != pad:
        image = preprocess.resize_linear_host(image, pad[1], pad[0])
    top, bottom = int(round(h - 0.1)), int(round(h + 0.1))
    left, right = int(round(w - 0.1)), int(round(w + 0.1))
    out = numpy.zeros((pad[1] + top + bottom, pad[0] + left + right, 3), dtype=numpy.uint8)
    out[top:top + pad[1], left:left + pad[0]] = image
    return out, (r, r), (w, h)


class Dataset(data.Dataset):
    def __init__(self, filenames, input_size, params, augment):
        if augment:
            raise NotImplementedError("Dataset(augment=True) is the training pipeline (mosaic, mix-up, random "
                                      "perspective, HSV, flips): outside this inference build's scope")
        self.params = params
        self.mosaic = False
        self.augment = False
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

    def _labels_on_canvas(self, index, h0, w0):
        """Labels of image `index` in the letterboxed canvas: (cls (n, 1), box (n, 4) normalised cx cy w h)."""
        S = self.input_size
        nh, nw, _, _ = preprocess.geometry(h0, w0, S)
        dw, dh = (S - nw) / 2, (S - nh) / 2
        label = self.labels[index].copy()
        if label.size:
            label[:, 1:] = wh2xy(label[:, 1:], nw, nh, dw, dh)
        return label[:, 0:1], xy2wh(label[:, 1:5], S, S)

    def __getitem__(self, index):
        index = self.indices[index]
        image = read_bgr(self.filenames[index])
        h0, w0 = image.shape[:2]
        cls, box = self._labels_on_canvas(index, h0, w0)
        sample = preprocess.letterbox_host(image, self.input_size)
        nl = len(cls)
        target_cls = torch.from_numpy(cls) if nl else torch.zeros((nl, 1))
        target_box = torch.from_numpy(box) if nl else torch.zeros((nl, 4))
        return torch.from_numpy(sample), target_cls, target_box, torch.zeros(nl)

    def raw(self, index):
        """(decoded BGR HWC uint8 tensor, cls, box, zeros(n)): the letterbox left to the device
        (yolo_hip.preprocess.letterbox of a list of these images gives the batch __getitem__
        and collate_fn would)."""
        index = self.indices[index]
        image = read_bgr(self.filenames[index])
        cls, box = self._labels_on_canvas(index, *image.shape[:2])
        nl = len(cls)
        return (torch.from_numpy(image), torch.from_numpy(cls) if nl else torch.zeros((nl, 1)),
                torch.from_numpy(box) if nl else torch.zeros((nl, 4)), torch.zeros(nl))

    def load_mosaic(self, index, params):
        raise NotImplementedError("load_mosaic (dataset.py:105-176) is training-time augmentation (out of scope)")

    @staticmethod
    def collate_fn(batch):
        """dataset.py:178-193: stacked samples + {'cls', 'box', 'idx'} with per-image indices.
        Samples of different shapes (Dataset.raw images) stay a list."""
        samples, cls, box, indices = zip(*batch)
        cls = torch.cat(cls, dim=0)
        box = torch.cat(box, dim=0)
        new_indices = [t + i for i, t in enumerate(indices)]
        indices = torch.cat(new_indices, dim=0)
        targets = {"cls": cls, "box": box, "idx": indices}
        if all(s.shape == samples[0].shape for s in samples):
            return torch.stack(samples, dim=0), targets
        return list(samples), targets

    @staticmethod
    def load_label(filenames):
        """{image filename: (n, 5) float32 labels (cls, cx, cy, w, h)} (dataset.py:195-237): the
        images/ -> labels/ sibling .txt of each image, images PIL-verified; cached per image
        directory in `<dir>.labels.npz`."""
        if not filenames:
            return {}
        path = f"{os.path.dirname(filenames[0])}.labels.npz"
        if os.path.exists(path):
            with numpy.load(path, allow_pickle=False) as z:
                if [str(s) for s in z["inputs"]] == list(filenames):
                    return {str(n): z[f"l{i}"] for i, n in enumerate(z["filenames"])}
        from PIL import Image
        x = {}
        for filename in filenames:
            try:
                with open(filename, "rb") as f:
                    image = Image.open(f)
                    image.verify()
                shape = image.size
                assert (shape[0] > 9) & (shape[1] > 9), f"image size {shape} <10 pixels"
                assert image.format.lower() in FORMATS, f"invalid image format {image.format}"
                a, b = f"{os.sep}images{os.sep}", f"{os.sep}labels{os.sep}"
                txt = b.join(filename.rsplit(a, 1)).rsplit(".", 1)[0] + ".txt"
                label = numpy.zeros((0, 5), dtype=numpy.float32)
                if os.path.isfile(txt):
                    with open(txt) as f:
                        rows = [r.split() for r in f.read().strip().splitlines() if len(r)]
                    if rows:
                        label = numpy.array(rows, dtype=numpy.float32)
                        assert (label >= 0).all()
                        assert label.shape[1] == 5
                        assert (label[:, 1:] <= 1).all()
                        _, i = numpy.unique(label, axis=0, return_index=True)
                        if len(i) < len(label):
                            label = label[i]
            except FileNotFoundError:
                label = numpy.zeros((0, 5), dtype=numpy.float32)
            except AssertionError:
                continue
            x[filename] = label
        try:
            numpy.savez(path, inputs=numpy.array(list(filenames)), filenames=numpy.array(list(x.keys())),
                        **{f"l{i}": v for i, v in enumerate(x.values())})
        except OSError:
            pass
        return x
