"""The per-op interval oracle (tests/_opcheck.py) itself, on the CPU: it accepts an fp32
evaluation of each op (torch's own fp32 kernels, a different summation order than the
device's) rounded like the device rounds, and it rejects a one-ulp change of a pinned
element. Runs the oracle on the v11_n synthetic weights at small shapes."""
import pytest
import torch
import torch.nn.functional as F

import _opcheck as oc
from _util import make_model


def _fp32_layer(x, desc, params, dtype, res=None):
    w, b = params(desc)
    y = F.conv2d(x.float(), w.float(), b.float(), desc["s"], desc["k"] // 2, groups=desc["g"])
    if desc["act"]:
        y = F.silu(y)
    y = y.to(dtype)
    if res is not None:
        y = (y.float() + res.float()).to(dtype)
    return y


def _desc(name, model, act=1, s=1):
    m = model.get_submodule(name)
    conv = getattr(m, "conv", m)
    return dict(name=name, k=conv.kernel_size[0], s=s, g=conv.groups, act=act, cin=conv.in_channels,
                cout=conv.out_channels, bias=int(conv.bias is not None))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16])
def test_interval_oracle_accepts_fp32_and_rejects_an_ulp(dtype):
    model = make_model("n")
    params = oc.Params(model.state_dict(), dtype)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(2, 64, 20, 20, generator=g).to(dtype)
    d1 = _desc("head.box.0.0", model)
    d2 = _desc("head.box.0.1", model)
    # one layer, and a chain with a residual
    y1 = _fp32_layer(x, d1, params, dtype)
    lo, hi = oc.layer(x.double(), x.double(), d1, params, dtype)
    with oc.exact_values():
        ref, _ = oc.layer(x.double(), x.double(), d1, params, dtype)
    st = oc.compare(y1, lo, hi, ref, dtype, "layer")
    assert st["bad"] == 0 and st["exact"] > 0.99 and st["over1"] < 1e-3, st
    y2 = _fp32_layer(y1, d2, params, dtype, res=y1)
    lo2, hi2 = oc.layer(lo, hi, d2, params, dtype, res=(lo, hi))
    with oc.exact_values():
        ref2, _ = oc.layer(ref, ref, d2, params, dtype, res=(ref, ref))
    st = oc.compare(y2, lo2, hi2, ref2, dtype, "chain")
    assert st["bad"] == 0 and st["over1"] < 5e-3, st
    # a one-ulp change of a pinned element is caught
    idx = torch.nonzero(lo2 == hi2)[len(torch.nonzero(lo2 == hi2)) // 2].tolist()
    bad = y2.clone()
    bits = bad.view(torch.int16)
    bits[tuple(idx)] += 1
    assert oc.compare(bad, lo2, hi2, ref2, dtype, "perturbed")["bad"] == 1


def test_attention_and_dfl_intervals_hold_fp32_evaluations():
    dtype = torch.bfloat16
    model = make_model("n")
    params = oc.Params(model.state_dict(), dtype)
    g = torch.Generator().manual_seed(4)
    heads, T, H, W = 2, 64, 8, 8
    qkv = torch.randn(1, heads * 128, H, W, generator=g).to(dtype)
    pe = dict(name="net.p5.3.res_m.0.conv1.conv1", k=3, s=1, g=heads * 64, act=0, cin=heads * 64,
              cout=heads * 64, bias=0)
    lo, hi = oc.attention_op({"in0": qkv.double()}, {"convs": [pe]}, params, dtype, heads)
    # fp32 evaluation with the softmax weights rounded to the dtype before P.V (as the device)
    t = qkv.float().reshape(1, heads, 128, T)
    q, k, v = t[:, :, :32], t[:, :, 32:64], t[:, :, 64:]
    s = torch.einsum("bhcq,bhck->bhqk", q, k) * (32 ** -0.5)
    p = torch.exp(s - s.amax(-1, keepdim=True))
    o = torch.einsum("bhqk,bhck->bhqc", p.to(dtype).float(), v) / p.sum(-1, keepdim=True)
    o = o.to(dtype).float().permute(0, 1, 3, 2).reshape(1, heads * 64, H, W)
    pw, pb = params(pe)
    y = (o + F.conv2d(v.reshape(1, heads * 64, H, W), pw.float(), pb.float(), 1, 1, groups=heads * 64)).to(dtype)
    with oc.exact_values():
        ref, _ = oc.attention_op({"in0": qkv.double()}, {"convs": [pe]}, params, dtype, heads)
    st = oc.compare(y, lo, hi, ref, dtype, "attention")
    assert st["bad"] == 0, st
    # DFL box rows from logits
    lg = torch.randn(1, 64, 4, 4, generator=g).to(dtype)
    blo, bhi = oc.dfl_box(lg.double(), lg.double(), 8, dtype)
    pr = torch.softmax(lg.float().view(1, 4, 16, 16), 2)
    dist = (pr * torch.arange(16.).view(1, 1, 16, 1)).sum(2)
    gy, gx = torch.meshgrid(torch.arange(4.) + 0.5, torch.arange(4.) + 0.5, indexing="ij")
    ax, ay = gx.reshape(1, -1), gy.reshape(1, -1)
    x1, y1, x2, y2 = ax - dist[:, 0], ay - dist[:, 1], ax + dist[:, 2], ay + dist[:, 3]
    box = torch.stack([(x1 + x2) / 2 * 8, (y1 + y2) / 2 * 8, (x2 - x1) * 8, (y2 - y1) * 8], 1).to(dtype)
    with oc.exact_values():
        bref, _ = oc.dfl_box(lg.double(), lg.double(), 8, dtype)
    st = oc.compare(box, blo, bhi, bref, dtype, "dfl")
    assert st["bad"] == 0, st
