"""Deterministic synthetic weights, images and head outputs.

There are no checkpoints or datasets on the build or GPU boxes, so parity
fixtures, tests and the bench all draw their data from here. Every tensor is
keyed by its state_dict name through numpy's PCG64, so the same name always
gets the same values on any machine (the golden generator feeds exactly these
weights to the reference model, the tests feed them to the HIP engine).

Weight recipe: conv weights ~ N(0, (gain^2 / fan_in)),
BatchNorm gamma, running_var ~ U(0.75, 1.25), beta, running_mean ~ N(0, 0.1),
head output biases ~ N(0, 0.1) with the class-logit biases shifted so that
a realistic share of (anchor, class) pairs clears the 0.001 confidence
threshold (trained detectors keep a few thousand candidates per image). The
BatchNorm running statistics and that shift are calibrated once by
tools/calibrate_synth.py (a random SiLU stack is otherwise in the vanishing or
exploding regime) and stored in synth_calib/; inputs for parity and bench are
structured synthetic scenes (synth_scenes). The DFL projection (head.dfl.conv.weight,
nets/nn.py:219-220) is fixed to 0..15 and is never randomised.
"""
import hashlib
import os
import zlib

import numpy as np
import torch

CONV_GAIN = 1.0
CLS_BIAS = -9.0
# DFL logit convs (head.box.<l>.2) at half gain: moderate bin distributions, as in
# a trained head, which keeps the fp32 forward's own rounding noise on box
# coordinates (stride x DFL expectation) well below the 1e-3 px parity bar.
BOX_LOGIT_GAIN = 0.5


def _rng(seed, name):
    return np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(name.encode())]))


def synth_tensor(name, shape, seed=0, gain=CONV_GAIN, cls_bias=CLS_BIAS):
    """Value of one state_dict entry."""
    rng = _rng(seed, name)
    shape = tuple(int(s) for s in shape)
    if name.endswith("num_batches_tracked"):
        return np.zeros(shape, dtype=np.int64)
    if name == "head.dfl.conv.weight":
        return np.arange(shape[1], dtype=np.float32).reshape(shape)
    if name.endswith("norm.weight") or name.endswith("norm.running_var"):
        return rng.uniform(0.75, 1.25, size=shape).astype(np.float32)
    if name.endswith("norm.bias") or name.endswith("norm.running_mean"):
        return rng.normal(0.0, 0.1, size=shape).astype(np.float32)
    if name.endswith(".bias"):
        b = rng.normal(0.0, 0.1, size=shape).astype(np.float32)
        if name.startswith("head.cls.") and name.endswith(".4.bias"):
            b += np.float32(cls_bias)
        return b
    if name.endswith("weight") and len(shape) == 4:
        fan_in = shape[1] * shape[2] * shape[3]
        if name.startswith("head.box.") and name.endswith(".2.weight"):
            gain = gain * BOX_LOGIT_GAIN
        return (rng.standard_normal(size=shape) * (gain / np.sqrt(fan_in))).astype(np.float32)
    raise KeyError(f"no synthetic rule for {name} {shape}")


CALIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "synth_calib")


def variant_of(template):
    """Name of the reference variant a state_dict template belongs to (by stem/stage widths)."""
    w1 = tuple(template["net.p1.0.conv.weight"].shape)[0]
    w5 = tuple(template["net.p5.0.conv.weight"].shape)[0]
    deep = "net.p2.1.res_m.0.conv3.conv.weight" in template
    two = "net.p2.1.res_m.1.conv1.conv.weight" in template
    table = {(16, 256, False, False): "n", (24, 384, False, False): "t", (32, 512, False, False): "s",
             (64, 512, True, False): "m", (64, 512, True, True): "l", (96, 768, True, True): "x"}
    return table.get((w1, w5, deep, two))


def load_calibration(variant):
    path = os.path.join(CALIB_DIR, f"v11_{variant}.npz")
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def synth_state_dict(template, seed=0, calib=True, gain=CONV_GAIN, cls_bias=None):
    """Synthetic values for every entry of a state_dict template (name -> tensor).

    With calib=True (default) the BatchNorm running statistics and the class
    bias shift come from tools/calibrate_synth.py's stored calibration.
    """
    cal = None
    if calib:
        v = variant_of(template)
        if v is None:
            raise ValueError("no synthetic calibration for this architecture; use calib=False")
        cal = load_calibration(v)
    shift = float(cal["cls_shift"][0]) if cal is not None else (CLS_BIAS if cls_bias is None else cls_bias)
    out = {}
    for name, t in template.items():
        if cal is not None and name in cal:
            v = cal[name].astype(np.float32)
        else:
            v = synth_tensor(name, tuple(t.shape), seed, gain=gain, cls_bias=shift)
        out[name] = torch.from_numpy(np.ascontiguousarray(v))
        if v.dtype != np.int64:
            out[name] = out[name].to(t.dtype)
    return out


def synth_images(batch, height, width, seed=0):
    """(B, 3, H, W) float32 in [0, 1): the letterboxed-image range after /255 (main.py:265-267)."""
    rng = np.random.Generator(np.random.PCG64([int(seed), 0x1A6E5]))
    return torch.from_numpy(rng.random((batch, 3, height, width), dtype=np.float32))


def synth_scenes(batch, height, width, seed=0, shapes=24):
    """(B, 3, H, W) float32 in [0, 1]: piecewise-constant "scenes" (random coloured
    rectangles and discs over a colour gradient, light noise). Unlike iid noise
    they have image-scale structure, so deep features vary between images the way
    real photos make them vary."""
    rng = np.random.Generator(np.random.PCG64([int(seed), 0x5CE7E]))
    out = np.empty((batch, 3, height, width), dtype=np.float32)
    yy, xx = np.meshgrid(np.linspace(0, 1, height, dtype=np.float32),
                         np.linspace(0, 1, width, dtype=np.float32), indexing="ij")
    for b in range(batch):
        c0, c1 = rng.random(3), rng.random(3)
        ang = rng.uniform(0, 2 * np.pi)
        t = (np.cos(ang) * xx + np.sin(ang) * yy)
        t = (t - t.min()) / max(float(t.max() - t.min()), 1e-6)
        img = c0[:, None, None] * (1 - t) + c1[:, None, None] * t
        for _ in range(shapes):
            col = rng.random(3)
            cx, cy = rng.uniform(0, width), rng.uniform(0, height)
            rw, rh = np.exp(rng.uniform(np.log(8), np.log(width / 2), size=2))
            if rng.random() < 0.5:
                m = (np.abs(xx * width - cx) < rw / 2) & (np.abs(yy * height - cy) < rh / 2)
            else:
                m = ((xx * width - cx) / rw) ** 2 + ((yy * height - cy) / rh) ** 2 < 0.25
            img[:, m] = col[:, None]
        img += rng.normal(0, 0.03, size=img.shape)
        out[b] = np.clip(img, 0.0, 1.0)
    return torch.from_numpy(out)


def synth_head_output(anchors=8400, nc=80, seed=0, mode="typical", img=640.0):
    """A (4 + nc, A) float32 head output with DISTINCT class scores.

    modes: "typical" - logits ~ N(-10, 1.5) (~2% of pairs above 0.001),
           "dense"   - boxes clustered on a few centres (heavy suppression),
           "stress"  - logits ~ N(0, 2) (every pair a candidate).
    Scores are made pairwise distinct (argsort in the reference is unstable,
    so only distinct scores pin an order).
    """
    rng = np.random.Generator(np.random.PCG64([int(seed), zlib.crc32(mode.encode())]))
    out = np.empty((4 + nc, anchors), dtype=np.float32)
    if mode == "dense":
        centres = rng.uniform(64, img - 64, size=(12, 2))
        pick = rng.integers(0, len(centres), size=anchors)
        out[0] = centres[pick, 0] + rng.normal(0, 6, size=anchors)
        out[1] = centres[pick, 1] + rng.normal(0, 6, size=anchors)
        out[2] = np.exp(rng.uniform(np.log(40), np.log(120), size=anchors))
        out[3] = np.exp(rng.uniform(np.log(40), np.log(120), size=anchors))
        logits = rng.normal(-8.0, 2.0, size=(nc, anchors))
    else:
        out[0] = rng.uniform(0, img, size=anchors)
        out[1] = rng.uniform(0, img, size=anchors)
        out[2] = np.exp(rng.uniform(np.log(4), np.log(320), size=anchors))
        out[3] = np.exp(rng.uniform(np.log(4), np.log(320), size=anchors))
        mu, sd = (-10.0, 1.5) if mode == "typical" else (0.0, 2.0)
        logits = rng.normal(mu, sd, size=(nc, anchors))
    scores = (1.0 / (1.0 + np.exp(-logits))).astype(np.float32)
    out[4:] = _make_distinct(scores)
    return torch.from_numpy(out)


def _make_distinct(s):
    flat = s.reshape(-1).copy()
    while True:
        order = np.argsort(flat, kind="stable")
        srt = flat[order]
        dup = np.nonzero(srt[1:] == srt[:-1])[0]
        if dup.size == 0:
            return flat.reshape(s.shape)
        idx = order[dup + 1]
        flat[idx] = np.nextafter(flat[idx], np.float32(np.inf))


def sha256(t):
    a = t.detach().cpu().contiguous().numpy()
    return hashlib.sha256(a.tobytes()).hexdigest()
