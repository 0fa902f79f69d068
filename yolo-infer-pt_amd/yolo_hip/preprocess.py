"""Eval-mode image preprocessing of the reference's loader (yh_letterbox / _host).

The reference's Dataset (utils/dataset.py:30-90, augment=False) turns a decoded
BGR image into the network input in three steps: load_image's cv2.resize to
int(w r) x int(h r) with r = input_size / max(h, w) (dataset.py:95-103),
resize()'s zero border to a centred square canvas (dataset.py:292-313) and the
HWC -> CHW, BGR -> RGB flip (dataset.py:86-88). `letterbox` runs all three for a
whole batch in one kernel on the device; `letterbox_host` runs the same per-pixel
code on the host (C++). The resize restates OpenCV's INTER_LINEAR 8-bit algorithm
(csrc/preprocess.hip); cv2 is not in this image, so parity against cv2 itself is
unpinned - the tests pin the kernels to the independent numpy restatement in
oracle/preprocess.py and to torch's bilinear resize within one level.
"""
from ctypes import byref, c_int, c_void_p

import numpy as np
import torch

from ._lib import check, lib


def geometry(height, width, size):
    """(new_h, new_w, top, left) of the letterbox of an height x width image on a size x size canvas."""
    nh, nw, top, left = c_int(), c_int(), c_int(), c_int()
    check(lib().yh_letterbox_geometry(int(height), int(width), int(size), byref(nh), byref(nw), byref(top),
                                      byref(left)), "letterbox_geometry")
    return nh.value, nw.value, top.value, left.value


def letterbox_host(image, size, threads=1):
    """uint8 HWC BGR numpy image -> uint8 (3, size, size) RGB CHW numpy array (host C++)."""
    img = np.ascontiguousarray(image)
    if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
        raise ValueError("letterbox_host needs an (h, w, 3) uint8 image")
    out = np.empty((3, size, size), dtype=np.uint8)
    check(lib().yh_letterbox_host(c_void_p(img.ctypes.data), img.shape[0], img.shape[1], img.strides[0], int(size),
                                  c_void_p(out.ctypes.data), int(threads)), "letterbox_host")
    return out


def resize_linear_host(image, new_h, new_w):
    """cv2.resize(image, (new_w, new_h), interpolation=cv2.INTER_LINEAR) of a uint8 (h, w, 3) image (host C++)."""
    img = np.ascontiguousarray(image)
    if img.dtype != np.uint8 or img.ndim != 3 or img.shape[2] != 3:
        raise ValueError("resize_linear_host needs an (h, w, 3) uint8 image")
    out = np.empty((int(new_h), int(new_w), 3), dtype=np.uint8)
    check(lib().yh_resize_linear_host(c_void_p(img.ctypes.data), img.shape[0], img.shape[1], img.strides[0],
                                      int(new_h), int(new_w), c_void_p(out.ctypes.data)), "resize_linear_host")
    return out


def letterbox(images, size, device=None, out=None):
    """Batch of uint8 HWC BGR images (tensors or arrays, any sizes) -> uint8 (B, 3, size, size) RGB
    CHW cuda tensor, on the current stream of `device` (default: the first cuda image's device,
    else cuda:0). Host images are copied to the device first."""
    if device is None:
        device = next((im.device for im in images if isinstance(im, torch.Tensor) and im.is_cuda),
                      torch.device("cuda", 0))
    device = torch.device(device)
    srcs = []
    for im in images:
        t = torch.as_tensor(im)
        if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
            raise ValueError("letterbox needs (h, w, 3) uint8 images")
        if t.stride(2) != 1 or t.stride(1) != 3:
            t = t.contiguous()
        srcs.append(t.to(device, non_blocking=True))
    B = len(srcs)
    if out is None:
        out = torch.empty((B, 3, size, size), dtype=torch.uint8, device=device)
    elif out.shape != (B, 3, size, size) or out.dtype != torch.uint8 or not out.is_contiguous():
        raise ValueError("letterbox: bad out tensor")
    if B == 0:
        return out
    ptrs = (c_void_p * B)(*[t.data_ptr() for t in srcs])
    hs = (c_int * B)(*[t.shape[0] for t in srcs])
    ws = (c_int * B)(*[t.shape[1] for t in srcs])
    st = (c_int * B)(*[t.stride(0) for t in srcs])
    with torch.cuda.device(device):
        check(lib().yh_letterbox(ptrs, hs, ws, st, B, int(size), c_void_p(out.data_ptr()),
                                 c_void_p(torch.cuda.current_stream(device).cuda_stream)), "letterbox")
    for t in srcs:   # keep the sources alive for the queued kernel
        t.record_stream(torch.cuda.current_stream(device))
    return out
