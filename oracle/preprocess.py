"""CPU restatement of the reference loader's eval preprocessing (TEST INFRASTRUCTURE ONLY).

  utils/dataset.py:95-103   load_image: r = input_size / max(h, w); cv2.resize to
                            (int(w * r), int(h * r)), INTER_LINEAR, when r != 1
  utils/dataset.py:292-313  resize(augment=False): r <= 1 -> no second resize; border
                            top = round(dh - 0.1), bottom = round(dh + 0.1) (same for
                            left / right), cv2.BORDER_CONSTANT = 0
  utils/dataset.py:86-88    image.transpose((2, 0, 1))[::-1]: HWC -> CHW, BGR -> RGB

cv2.resize's INTER_LINEAR for 8-bit images, vectorised here with numpy from
OpenCV's published algorithm (imgproc/resize.cpp): 11-bit coefficients from the
float source coordinate, an exact integer horizontal pass, and the vertical pass
as its SIMD kernel rounds (VResizeLinearVec_32s8u: (S >> 4) * beta >> 16, + 2,
>> 2) over the bytes its 128-bit vector loops cover, and the scalar FixedPtCast
((S0 b0 + S1 b1 + 2^21) >> 22) on the row's tail bytes (see `vtail`); an exact 2x downscale is routed to INTER_AREA's fast path. cv2 is absent
from this image and no fixture of cv2 output exists in the reference: PARITY
UNPINNED against cv2 itself. The kernels are pinned to this restatement, and this
restatement to torch's half-pixel bilinear resize within one grey level.
"""
import numpy as np


def geometry(h, w, size):
    r = size / max(h, w)                       # dataset.py:97
    nh, nw = (int(h * r), int(w * r)) if r != 1 else (h, w)
    dw, dh = (size - nw) / 2, (size - nh) / 2  # dataset.py:302-304
    return nh, nw, int(round(dh - 0.1)), int(round(dw - 0.1))   # dataset.py:310-311


def _axis(n_dst, n_src, clamp):
    scale = 1.0 / (n_dst / n_src)
    f = ((np.arange(n_dst, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if clamp:   # x axis: coordinates outside the image take the edge pixel with weight 1
        lo, hi = s < 0, s >= n_src - 1
        s = np.where(lo, 0, np.where(hi, n_src - 1, s))
        f = np.where(lo | hi, np.float32(0), f)
    a0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048)).astype(np.int64)
    return np.clip(s, 0, n_src - 1), np.clip(s + 1, 0, n_src - 1), a0, a1


def vtail(width):
    """First byte of a resized row that OpenCV's vertical pass computes in its scalar loop:
    VResizeLinearVec_32s8u steps 16 bytes while x <= width - 16, then 8 bytes while
    x < width - 8 (128-bit universal intrinsics); the rest is scalar."""
    x = ((width - 16) // 16 + 1) * 16 if width >= 16 else 0
    if x < width - 8:
        x += 8
    return x


def resize_linear(img, nh, nw):
    """cv2.resize(img, (nw, nh), interpolation=INTER_LINEAR) for an (h, w, 3) uint8 image."""
    h, w = img.shape[:2]
    if (h, w) == (nh, nw):
        return img.copy()
    src = img.astype(np.int64)
    if h == 2 * nh and w == 2 * nw:            # INTER_AREA fast path
        s = src[0::2, 0::2] + src[0::2, 1::2] + src[1::2, 0::2] + src[1::2, 1::2]
        return ((s + 2) >> 2).astype(np.uint8)
    xs0, xs1, xa0, xa1 = _axis(nw, w, True)
    ys0, ys1, ya0, ya1 = _axis(nh, h, False)
    horiz = src[:, xs0] * xa0[None, :, None] + src[:, xs1] * xa1[None, :, None]   # (h, nw, 3)
    t0 = ((horiz[ys0] >> 4) * ya0[:, None, None]) >> 16
    t1 = ((horiz[ys1] >> 4) * ya1[:, None, None]) >> 16
    vec = (t0 + t1 + 2) >> 2
    sca = (horiz[ys0] * ya0[:, None, None] + horiz[ys1] * ya1[:, None, None] + (1 << 21)) >> 22
    byte = (np.arange(nw)[:, None] * 3 + np.arange(3)[None, :])[None]   # byte index within the row
    return np.clip(np.where(byte < vtail(3 * nw), vec, sca), 0, 255).astype(np.uint8)


def letterbox(img, size):
    """(h, w, 3) uint8 BGR -> (3, size, size) uint8 RGB: the network input of one image."""
    nh, nw, top, left = geometry(img.shape[0], img.shape[1], size)
    out = np.zeros((size, size, 3), dtype=np.uint8)
    out[top:top + nh, left:left + nw] = resize_linear(img, nh, nw)
    return np.ascontiguousarray(out.transpose(2, 0, 1)[::-1])
