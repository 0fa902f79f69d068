"""Per-op interval oracle of the 16-bit kernels (TEST INFRASTRUCTURE ONLY).

tests/test_gpu_op_parity.py steps the forward op by op through the parity taps
(yh_debug_run_ops / yh_debug_operand) and hands each op's *device-produced* 16-bit inputs
to the functions here. For every output element they compute, in float64, the exact result
of the reference computation of that op (nets/nn.py:28-270, utils/util.py:85-96 — the
functions named per op below) on those inputs, with the op's weights as the device holds
them (dense / stem weights rounded once to the dtype, depthwise / positional weights and
biases fp32), and with one rounding to the dtype at every layer output the reference
materialises (each Conv's output, the Residual sum nets/nn.py:49, the attention output
before the positional term, the class / box logits before the decode).

The device computes in fp32; its documented arithmetic (fp32 MFMA K-sums, fp32 FMA chains,
hardware exp / reciprocal) departs from the exact result by a bounded amount E. So the
oracle returns, per element, the interval [rnd(v - E), rnd(v + E)] of dtype values a
correct kernel may produce, where v is the exact value and E the bound below. Wherever v
lies farther than E from a rounding boundary (almost everywhere) the interval is a single
value: the device must be bit-exact there. In fused multi-layer ops a layer output whose
interval holds two values carries both into the next layer (interval arithmetic), so the
check stays exact downstream of every undecided rounding.

Error bounds (u = 2^-24, fp32 unit roundoff; |.| = magnitudes of the exact terms):
  * K-term sum + bias (MFMA fp32 accumulate or an fp32 FMA chain, any order, round-to-
    nearest or truncating adds): (2K + 4) u (sum |x w| + |b|);
  * SiLU x * rcp(1 + exp(-x)) and sigmoid rcp(1 + exp(-x)) with __expf / v_rcp_f32:
    relative (2|x| + 16) u of the result, plus 1e-35 absolute (exp overflow below -88);
  * the residual / positional adds and the DFL / box arithmetic: a few u of the magnitudes;
  * attention: the 16-bit rounding of the softmax weights before the P.V MFMA (relative
    2^-8 bf16, 2^-11 fp16) and the fp32 online-softmax terms, see attention_op().
Every endpoint is further widened by 2u of its magnitude before the rounding (so the
fp64 -> fp32 -> dtype conversion of an endpoint can never narrow the interval).
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

U = 2.0 ** -24
ERR = [1.0]   # 0 inside exact_values(): every bound dropped (the correctly rounded exact result)
SILU_XMIN = -1.2784645427610738    # argmin of x * sigmoid(x)
ABS = 1e-35


# ------------------------------------------------------------------ rounding / intervals
def rnd(t, dtype):
    """float64 tensor -> nearest dtype value (as float64)."""
    return t.to(torch.float32).to(dtype).to(torch.float64)


def rnd_iv(lo, hi, dtype):
    """[lo, hi] (float64, exact bounds) -> the interval of dtype values it rounds into."""
    lo = lo - ERR[0] * (2 * U * lo.abs() + ABS)
    hi = hi + ERR[0] * (2 * U * hi.abs() + ABS)
    return rnd(lo, dtype), rnd(hi, dtype)


class exact_values:
    """Within this context every op function returns (v, v): its exact result, rounded
    once per layer output like the device rounds (no error bound)."""

    def __enter__(self):
        ERR[0] = 0.0

    def __exit__(self, *a):
        ERR[0] = 1.0


def half_u(dtype):
    """unit roundoff of the 16-bit dtype"""
    return 2.0 ** -8 if dtype == torch.bfloat16 else 2.0 ** -11


def silu_iv(lo, hi):
    """SiLU over [lo, hi] (exact extremes, x * sigmoid(x) has one minimum) + device error."""
    a, b = F.silu(lo), F.silu(hi)
    mn, mx = torch.minimum(a, b), torch.maximum(a, b)
    inside = (lo < SILU_XMIN) & (hi > SILU_XMIN)
    mn = torch.where(inside, torch.full_like(mn, float(F.silu(torch.tensor(SILU_XMIN, dtype=torch.float64)))), mn)
    x = torch.maximum(lo.abs(), hi.abs())
    m = torch.maximum(mn.abs(), mx.abs())
    e = ERR[0] * ((2 * x + 16) * U * m + ABS)
    return mn - e, mx + e


def sigmoid_iv(lo, hi):
    """sigmoid over [lo, hi] (monotone) + the device's rcp(1 + exp(-x)) error."""
    a, b = torch.sigmoid(lo), torch.sigmoid(hi)
    x = torch.maximum(lo.abs(), hi.abs())
    return a - ERR[0] * ((2 * x + 16) * U * a + ABS), b + ERR[0] * ((2 * x + 16) * U * b + ABS)


# ------------------------------------------------------------------ parameters
class Params:
    """Conv parameters as the device holds them, from the (fused) reference state_dict the
    engine was loaded from: nets/nn.py Conv blocks (`name.conv.weight` / `.bias`, BN already
    folded by fuse_conv nets/nn.py:8-25) or plain nn.Conv2d (`name.weight` / `.bias`)."""

    def __init__(self, state_dict, dtype):
        self.sd = state_dict
        self.dtype = dtype
        self._c = {}

    def __call__(self, desc):
        name = desc["name"]
        if name in self._c:
            return self._c[name]
        sd = self.sd
        if f"{name}.conv.weight" in sd:
            w, b = sd[f"{name}.conv.weight"], sd.get(f"{name}.conv.bias")
        else:
            w, b = sd[f"{name}.weight"], sd.get(f"{name}.bias")
        assert f"{name}.norm.weight" not in sd, "Params expects a fused state_dict"
        w = w.detach().float().cpu()
        b = torch.zeros(w.shape[0]) if b is None else b.detach().float().cpu()
        if desc["g"] == 1:       # dense / stem convs: MFMA operands rounded to the dtype once
            w = w.to(self.dtype)
        out = (w.double(), b.double())
        self._c[name] = out
        return out


# ------------------------------------------------------------------ one conv layer
def conv_pre(xlo, xhi, desc, params, rows=None, couts=None):
    """Pre-activation interval of Conv `desc` (nets/nn.py:28-39, BN folded) for inputs in
    [xlo, xhi] (NCHW float64): exact conv of the midpoint +- the conv of the radius with |w|,
    widened by the K-sum bound. rows = (r0, r1) restricts to those output rows, couts to
    those output channels (the result then has only those)."""
    w, b = params(desc)
    k, s, g = desc["k"], desc["s"], desc["g"]
    if couts is not None:
        w, b = w[couts], b[couts]
        assert g == 1
    p = k // 2
    mid = (xlo + xhi) * 0.5
    rad = (xhi - xlo) * 0.5
    mag = torch.maximum(xlo.abs(), xhi.abs())
    if rows is not None:
        r0, r1 = rows
        sl = lambda t: F.pad(t, (0, 0, p, p))[:, :, r0 * s:(r1 - 1) * s + k]
        mid, rad, mag = sl(mid), sl(rad), sl(mag)
        pad = (0, p)
    else:
        pad = p
    c = F.conv2d(mid, w, b, s, pad, groups=g)
    m = F.conv2d(mag, w.abs(), b.abs(), s, pad, groups=g)
    K = (w.shape[1]) * k * k
    e = ERR[0] * (2 * K + 4) * U * m
    if bool((rad > 0).any()):
        e = e + F.conv2d(rad, w.abs(), None, s, pad, groups=g)
    return c - e, c + e


def layer(xlo, xhi, desc, params, dtype, res=None, rows=None, couts=None):
    """Conv + activation + one rounding (+ Residual add nets/nn.py:49 and its rounding):
    the rounded output interval."""
    lo, hi = conv_pre(xlo, xhi, desc, params, rows, couts)
    if desc["act"]:
        lo, hi = silu_iv(lo, hi)
    lo, hi = rnd_iv(lo, hi, dtype)
    if res is not None:
        rlo, rhi = res
        m = ERR[0] * U * (torch.maximum(lo.abs(), hi.abs()) + torch.maximum(rlo.abs(), rhi.abs()))
        lo, hi = rnd_iv(lo + rlo - m, hi + rhi + m, dtype)
    return lo, hi


def exact(t):
    return t, t


# ------------------------------------------------------------------ ops
def conv_op(ins, d, params, dtype, rows=None, couts=None):
    """OP_CONV: Conv (nets/nn.py:28-39) over the concat of its input segments (DarkFPN's
    nearest x2 upsample + torch.cat, nn.py:203-209, for segments with up = 1), optional
    Residual add (nn.py:49, PSABlock nn.py:135-136)."""
    segs = []
    for i, o in enumerate(d["operands"]):
        if o["role"].startswith("in"):
            t = ins[o["role"]][:, :o["logical"]]
            if o["up"]:
                t = t.repeat_interleave(2, 2).repeat_interleave(2, 3)
            segs.append(t)
    x = torch.cat(segs, 1)
    res = None
    if "res" in ins:
        r = ins["res"][:, :d["convs"][0]["cout"]]
        if rows is not None:
            r = r[:, :, rows[0]:rows[1]]
        if couts is not None:
            r = r[:, couts]
        res = exact(r)
    return layer(x, x, d["convs"][0], params, dtype, res=res, rows=rows, couts=couts)


def stem_op(x, d, params, dtype):
    """OP_STEM2 / OP_FIRST: net.p1.0 Conv(3, c1, 3, 2) (+ net.p2.0 Conv(c1, c2, 3, 2)),
    nets/nn.py:160-163."""
    lo, hi = exact(x)
    for c in d["convs"]:
        lo, hi = layer(lo, hi, c, params, dtype)
    return lo, hi


def dw_op(ins, d, params, dtype):
    """OP_DW: DWConv 3x3 + SiLU (head cls branch, nets/nn.py:248-252)."""
    x = ins["in0"]
    return layer(x, x, d["convs"][0], params, dtype)


def sppf_op(ins, d):
    """OP_SPPF: y1 = m(x), y2 = m(y1), y3 = m(y2), 5x5 max pools (nets/nn.py:90-94) - exact."""
    x = ins["in0"]
    ys = []
    for _ in range(3):
        x = F.max_pool2d(x, 5, 1, 2)
        ys.append(x)
    y = torch.cat(ys, 1)
    return y, y


def csp_op(ins, d, params, dtype):
    """OP_CSP (fused C3k2 with one Residual, nets/nn.py:66-80, 42-49): conv1 -> chunk(2) ->
    [a | b] -> r = b + conv2(conv1(b)) -> conv2(cat(a, b, r)). Tail mode (no conv1 in the op):
    the input is conv1's output."""
    c1, r1, r2, c2 = d["convs"]
    x = ins["in0"]
    if c1 is not None:
        tlo, thi = layer(x, x, c1, params, dtype)
    else:
        tlo, thi = exact(x)
    c = r1["cin"]
    blo, bhi = tlo[:, c:2 * c], thi[:, c:2 * c]
    mlo, mhi = layer(blo, bhi, r1, params, dtype)
    rlo, rhi = layer(mlo, mhi, r2, params, dtype, res=(blo, bhi))
    return layer(torch.cat([tlo, rlo], 1), torch.cat([thi, rhi], 1), c2, params, dtype)


def c3k_op(ins, d, params, dtype):
    """OP_C3K (CSPModule / C3k, nets/nn.py:52-63): conv3(cat(res_m(conv1(x)), conv2(x)))
    with two Residual(h, e=1.0)."""
    cv1, cv2, a1, a2, b1, b2, cv3 = d["convs"]
    x = ins["in0"]
    plo, phi = layer(x, x, cv1, params, dtype)
    qlo, qhi = layer(x, x, cv2, params, dtype)
    for r1, r2 in ((a1, a2), (b1, b2)):
        mlo, mhi = layer(plo, phi, r1, params, dtype)
        plo, phi = layer(mlo, mhi, r2, params, dtype, res=(plo, phi))
    return layer(torch.cat([plo, qlo], 1), torch.cat([phi, qhi], 1), cv3, params, dtype)


def attention_op(ins, d, params, dtype, heads):
    """OP_ATTN (Attention nets/nn.py:97-123 up to the projection): per head
    o = V softmax(Q^T K * dk^-0.5)^T, rounded, + pe(v) (the positional DWConv 3x3, BN folded),
    rounded. The device keeps scores and softmax sums in fp32, rounds each softmax weight to
    the dtype before the P.V MFMA (misc.hip psa_attention_*), and rescales online per block of
    16 keys; its departure from the exact o is bounded by
        (u16 + 2 eps + (4T + 8) u) (sum_j p_j |v_j| / D + |o|) + ds_max sum_j p_j |v_j - o| / D
    (+ T 2^-25 max|v| / D for fp16 subnormal weights), eps = (max_j |s_j - m| + 8) u the exp
    error, ds_max the fp32 score error (scale (2 dk + 4) u sum |q k| + 2 u |s|)."""
    qkv = ins["in0"]
    B, _, H, W = qkv.shape
    T = H * W
    dk, dh = 32, 64
    u16 = half_u(dtype)
    pe_desc = d["convs"][0]
    pw, pb = params(pe_desc)
    outs_lo, outs_hi = [], []
    t = qkv.reshape(B, heads, 2 * dk + dh, T)
    q, k, v = t[:, :, :dk], t[:, :, dk:2 * dk], t[:, :, 2 * dk:]
    scale = dk ** -0.5
    s = torch.einsum("bhcq,bhck->bhqk", q, k) * scale
    sabs = torch.einsum("bhcq,bhck->bhqk", q.abs(), k.abs()) * scale
    m = s.amax(-1, keepdim=True)
    p = torch.exp(s - m)
    D = p.sum(-1, keepdim=True)
    o = torch.einsum("bhqk,bhck->bhqc", p, v) / D                       # (B, h, T, dh)
    pv = torch.einsum("bhqk,bhck->bhqc", p, v.abs()) / D
    # sum_j p_j |v_j - o| / D <= sum_j p_j |v_j| / D + |o|
    ds = ((2 * dk + 4) * U * sabs + 2 * U * s.abs()).amax(-1, keepdim=True)
    eps = ((s - m).abs().amax(-1, keepdim=True) + 8) * U
    e = (u16 + 2 * eps + (4 * T + 8) * U + ds) * (pv + o.abs())
    if dtype == torch.float16:
        e = e + T * 2.0 ** -25 * v.abs().amax(-1)[:, :, None, :] / D
    e = ERR[0] * e
    olo, ohi = rnd_iv(o - e, o + e, dtype)
    to_nchw = lambda z: z.permute(0, 1, 3, 2).reshape(B, heads * dh, H, W)
    olo, ohi = to_nchw(olo), to_nchw(ohi)
    vv = v.reshape(B, heads * dh, H, W)
    pe = F.conv2d(vv, pw, pb, 1, 1, groups=heads * dh)
    pm = F.conv2d(vv.abs(), pw.abs(), pb.abs(), 1, 1, groups=heads * dh)
    em = ERR[0] * 24 * U * (pm + torch.maximum(olo.abs(), ohi.abs()))
    return rnd_iv(olo + pe - em, ohi + pe + em, dtype)


def head_cls_level(x, convs, params, dtype):
    """One level of the cls branch (nets/nn.py:248-252): DWConv -> Conv 1x1 -> DWConv ->
    Conv 1x1 -> Conv2d 1x1 (+ bias): the rounded class-logit interval."""
    lo, hi = exact(x)
    for c in convs:
        lo, hi = layer(lo, hi, c, params, dtype)
    return lo, hi


def dfl_box(llo, lhi, stride, dtype):
    """DFL (nets/nn.py:222-225) + make_anchors (utils/util.py:85-96) + dist2bbox
    (nets/nn.py:264-268) on rounded box logits in [llo, lhi] (B, 64, h, w): the interval of
    the four rounded output rows (cx, cy, w, h) * stride, (B, 4, h*w)."""
    B, _, h, w = llo.shape
    mid = (llo + lhi) * 0.5
    rad = (lhi - llo) * 0.5
    lg = mid.reshape(B, 4, 16, h * w)
    rd = rad.reshape(B, 4, 16, h * w)
    p = torch.softmax(lg, 2)
    bins = torch.arange(16, dtype=torch.float64).view(1, 1, 16, 1)
    dist = (p * bins).sum(2)                                             # (B, 4, A)
    rng = (lg.amax(2) - lg.amin(2))
    # sensitivity to the logits (first order, 5 % slack) + the fp32 softmax / FMA chain
    dr = 1.05 * (p * (bins - dist[:, :, None]).abs() * rd).sum(2) + ERR[0] * (15 * (2 * (rng + 4) + 20) + 240) * U
    gy, gx = torch.meshgrid(torch.arange(h, dtype=torch.float64) + 0.5, torch.arange(w, dtype=torch.float64) + 0.5,
                            indexing="ij")
    ax, ay = gx.reshape(1, -1), gy.reshape(1, -1)
    lt, rb = dist[:, :2], dist[:, 2:]
    x1, y1 = ax - lt[:, 0], ay - lt[:, 1]
    x2, y2 = ax + rb[:, 0], ay + rb[:, 1]
    st = float(stride)
    cx, cy = (x1 + x2) / 2 * st, (y1 + y2) / 2 * st
    bw, bh = (x2 - x1) * st, (y2 - y1) * st
    ex = ((dr[:, 0] + dr[:, 2]) * st + ERR[0] * 4 * U * (x1.abs() + x2.abs()) * st)
    ey = ((dr[:, 1] + dr[:, 3]) * st + ERR[0] * 4 * U * (y1.abs() + y2.abs()) * st)
    c = torch.stack([cx, cy, bw, bh], 1)
    e = torch.stack([ex / 2, ey / 2, ex, ey], 1)
    return rnd_iv(c - e, c + e, dtype)


# ------------------------------------------------------------------ comparison
def ordered(t16):
    """16-bit values -> integers ordered like the values (for ulp distances)."""
    i = t16.view(torch.int16).to(torch.int32)
    return torch.where(i < 0, -(i & 0x7FFF), i)


def ulp_width(lo, hi, dtype):
    """(hi - lo) in units of the dtype's ulp at max(|lo|, |hi|) (float64 tensor)"""
    p, emin = (8, -126) if dtype == torch.bfloat16 else (11, -14)
    m = torch.maximum(lo.abs(), hi.abs())
    e = torch.floor(torch.log2(torch.where(m > 0, m, torch.ones_like(m)))).clamp(min=emin)
    return torch.where(m > 0, (hi - lo) / torch.exp2(e - (p - 1)), torch.zeros_like(m))


def compare(dev, lo, hi, ref, dtype, what):
    """dev (dtype tensor) within [lo, hi] everywhere; ref = the correctly rounded exact result
    (exact_values()). Returns a stats dict: elements, out-of-interval count, share of pinned
    (one-value) intervals, share equal to ref, ulps from ref (max, share above 1)."""
    dev = dev.cpu()
    assert dev.shape == lo.shape == ref.shape, (what, tuple(dev.shape), tuple(lo.shape), tuple(ref.shape))
    d64 = dev.to(torch.float64)
    finite = torch.isfinite(d64)
    ok = (d64 >= lo) & (d64 <= hi) & finite
    pinned = lo == hi
    ulps = (ordered(dev) - ordered(ref.to(dtype))).abs()
    # interval width in ulps of the dtype at the interval's magnitude: (hi - lo) / ulp(max(|lo|, |hi|))
    # (0: pinned, 1: two adjacent values). How much freedom the proven bound leaves a kernel: a wide
    # interval could hide a few-ulp error. Intervals that straddle zero (the cancellation elements)
    # measure about 2^p (p = 8 bf16, 11 fp16): their width is set by the magnitudes summed, not by |y|.
    width = ulp_width(lo, hi, dtype)
    wq = width.flatten()
    if wq.numel() > 1 << 22:   # torch.quantile's size limit: a seeded sample
        wq = wq[torch.randperm(wq.numel(), generator=torch.Generator().manual_seed(0))[:1 << 22]]
    st = dict(what=what, n=int(dev.numel()), bad=int((~ok).sum()), pinned=float(pinned.double().mean()),
              exact=float((ulps == 0).double().mean()), max_ulp=int(ulps.max()) if dev.numel() else 0,
              over1=float((ulps > 1).double().mean()),
              w50=float(wq.quantile(0.5)) if wq.numel() else 0.0,
              w99=float(wq.quantile(0.99)) if wq.numel() else 0.0,
              w999=float(wq.quantile(0.999)) if wq.numel() else 0.0,
              wide=float((width > 4).double().mean()) if dev.numel() else 0.0,
              wmax=float(width.max()) if dev.numel() else 0.0)
    if st["bad"]:
        idx = torch.nonzero(~ok)[:5].tolist()
        st["examples"] = [(tuple(i), float(d64[tuple(i)]), float(lo[tuple(i)]), float(hi[tuple(i)])) for i in idx]
    return st
