"""Eval-time image preparation of the reference's data loader.

Only the part of `utils/dataset.py` that produces the network input is in scope:

  load_image   dataset.py:95-103   r = input_size / max(h, w); INTER_LINEAR resize to
                                   (int(w r), int(h r)) when r != 1
  resize       dataset.py:292-313  augment=False: zero border to a centred square canvas
  (channels)   dataset.py:86-88    HWC -> CHW, BGR -> RGB

The pixel arithmetic is the library's C++ (yh_resize_linear_host / yh_letterbox_host,
the same __host__ __device__ function as the device kernel yh_letterbox). Labels,
the label cache, collation and every training-time augmentation stay with the
reference: this module deliberately does not reimplement them.
"""
import numpy
import torch
from torch.utils import data

from yolo_hip import preprocess


def read_bgr(filename):
    """The decoded image as cv2.imread returns it, (h, w, 3) uint8 BGR, EXIF orientation applied.
    PIL decodes it (cv2 is not a dependency here): JPEG pixels may differ from libjpeg-turbo's
    by the decoder's IDCT / chroma upsampling, so parity with cv2.imread itself is unpinned."""
    from PIL import Image, ImageOps
    with Image.open(filename) as im:
        rgb = numpy.asarray(ImageOps.exif_transpose(im).convert("RGB"))
    return numpy.ascontiguousarray(rgb[:, :, ::-1])


def resize(image, input_size, augment):
    """dataset.py:292-313 with augment=False: shrink only (INTER_LINEAR), then a zero border that
    centres the image on an input_size square. Returns (canvas, (r, r), (dw, dh))."""
    if augment:
        raise NotImplementedError("resize(augment=True) draws a random interpolation (training only)")
    h, w = image.shape[:2]
    r = min(input_size / h, input_size / w, 1.0)
    nw, nh = int(round(w * r)), int(round(h * r))
    dw, dh = (input_size - nw) / 2, (input_size - nh) / 2
    if (nh, nw) != (h, w):
        image = preprocess.resize_linear_host(image, nh, nw)
    top, left = int(round(dh - 0.1)), int(round(dw - 0.1))
    canvas = numpy.zeros((nh + top + int(round(dh + 0.1)), nw + left + int(round(dw + 0.1)), 3), dtype=numpy.uint8)
    canvas[top:top + nh, left:left + nw] = image
    return canvas, (r, r), (dw, dh)


class Dataset(data.Dataset):
    """Eval images in the reference's network-input form: item i is the (3, S, S) uint8 RGB
    letterboxed image (what the reference's __getitem__ returns as its sample) and the original
    (h, w). `raw(i)` returns the decoded BGR image instead, for loops that letterbox whole
    batches on the device (yolo_hip.preprocess.letterbox, one kernel per batch)."""

    def __init__(self, filenames, input_size, params=None, augment=False):
        if augment:
            raise NotImplementedError("Dataset(augment=True) is the training pipeline (mosaic, mix-up, random "
                                      "perspective, HSV, flips): use the reference's loader for training")
        self.filenames = list(filenames)
        self.input_size = input_size
        self.params = params

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

    def __getitem__(self, i):
        image = read_bgr(self.filenames[i])
        return torch.from_numpy(preprocess.letterbox_host(image, self.input_size)), image.shape[:2]

    def raw(self, i):
        return torch.from_numpy(read_bgr(self.filenames[i]))
