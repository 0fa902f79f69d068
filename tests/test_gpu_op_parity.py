"""Op-by-op parity of the benchmarked 16-bit kernels against the fp64 oracle. Marked gpu.

The forward of a bench configuration is stepped one op at a time through the parity taps
(include/yolo_hip.h: yh_debug_run_ops, yh_debug_operand). Each op's inputs are taken from the
workspace exactly as the device produced them; tests/_opcheck.py evaluates that one op in
float64 on them (nets/nn.py:28-270, utils/util.py:85-96) and returns, per output element, the
interval of dtype values a correct kernel may produce: the exact result rounded once per layer
output, widened only by the proven bound of the kernel's fp32 arithmetic (K-sum, exp /
reciprocal, the attention's 16-bit softmax weights). Every device output must lie in its
interval; where the exact value is not within that bound of a rounding boundary the interval
is one value and the device must be bit-exact. The printed line per op gives the share of
such pinned elements, the share equal to the correctly rounded exact value (oc.exact_values:
the exact result with every error bound dropped, rounded per layer), the share more than one
ulp from it and the largest distance in ulps (near-zero outputs of opposite sign count the
whole range between them), and the interval width (p50 / p99 / max, in ulps). Single-layer
ops must keep the share beyond one ulp under 0.1 % (measured r05: at most 8e-5); the fused kinds
have per-kind ceilings (OVER1_MAX), and every kind a ceiling on its interval widths (WIDTH_MAX).

Covered kernels (by configuration):
  * C2 v11_n bf16 640 b32 (images 0, 17, 31): the tuned conv_mx / conv_mxr / conv_rw plans incl.
    the K-split ones (20x20 / 40x40 layers), stem_fused, csp_fused (whole-block and tail mode),
    c3k_fused in row bands and in SPLIT mode, sppf_fused, psa_attention_full, head_cls (all three
    levels, scores written straight into y), box_dfl; with YH_BOXCHAIN=1 (n bf16 b2) the opt-in
    fused box branch of the three levels (boxc.hip);
  * C2 unfused (YH_FUSE=0 YH_PWCHAIN=0 YH_C3K=0 YH_HCLS_WIDE=0): the per-layer launches each
    fused kernel is bit-identical to, at v11_n's shapes, under the single-layer bar;
  * v11_n fp16 640 b2: the same kernels in fp16;
  * C3 v11_s fp16 640 b64 (images 0, 63): wider conv plans, seven-launch C3k, per-layer cls
    branches (dwconv3x3_c4) and the class-rows decode (head_decode_lds);
  * C5 v11_x bf16 1280 b1: the 256-cout staged plans, conv_first_tile, the seven-launch C3k,
    psa_attention_lds + pe_add (1600 tokens), dwconv3x3_c4, head_decode_lds, box_dfl (96-channel
    K). Large conv layers are checked on three 4-row bands (top, middle, bottom) and 32 of
    their output channels; every other op on its whole output.
The stepped forward must leave y bit-identical to the graph forward.
"""
import numpy as np
import pytest
import torch

import _opcheck as oc
from _util import make_model
from yolo_hip import synth

pytestmark = pytest.mark.gpu

IN_ROLES = ("in0", "in1", "res", "x0", "x1", "x2", "L0", "L1", "L2")


def _nchw(t):
    return t.permute(0, 3, 1, 2).contiguous()


def _anchor_off(l, H, W):
    return sum((H >> (3 + k)) * (W >> (3 + k)) for k in range(l))


def _bands(Ho):
    if Ho <= 24:
        return [(0, Ho)]
    m = Ho // 2 - 2
    return [(0, 4), (m, m + 4), (Ho - 4, Ho)]


def _check_op(d, ins, outs, x, y, H, W, nc, params, dtype):
    """Stats of every output of op `d` (one entry per compared tensor): each output's interval
    and, with the error bounds dropped (oc.exact_values), its correctly rounded exact value."""
    kind = d["kind"]
    cases = []   # (what, device tensor, oracle function -> (lo, hi))
    if kind == "conv":
        conv = d["convs"][0]
        dev = _nchw(outs["out"])[:, :conv["cout"]]
        Ho = dev.shape[2]
        cost = dev.shape[0] * Ho * dev.shape[3] * conv["cout"] * conv["cin"] * conv["k"] ** 2
        if cost <= 3e9:
            cases.append(("out", dev, lambda: oc.conv_op(ins, d, params, dtype)))
        else:
            couts = None
            if conv["cout"] > 64:
                couts = torch.unique(torch.linspace(0, conv["cout"] - 1, 32).round().long())
            for r0, r1 in _bands(Ho):
                dv = dev[:, :, r0:r1]
                if couts is not None:
                    dv = dv[:, couts]
                cases.append((f"out rows {r0}-{r1}", dv,
                              lambda r0=r0, r1=r1: oc.conv_op(ins, d, params, dtype, rows=(r0, r1), couts=couts)))
    elif kind in ("stem", "stem_fused"):
        cases.append(("out", _nchw(outs["out"])[:, :d["convs"][-1]["cout"]],
                      lambda: oc.stem_op(x.double(), d, params, dtype)))
    elif kind == "dwconv":
        cases.append(("out", _nchw(outs["out"])[:, :d["convs"][0]["cout"]], lambda: oc.dw_op(ins, d, params, dtype)))
    elif kind == "sppf":
        cases.append(("out", _nchw(outs["out"]), lambda: oc.sppf_op(ins, d)))
    elif kind == "attention":
        cases.append(("out", _nchw(outs["out"]), lambda: oc.attention_op(ins, d, params, dtype, d["heads"])))
    elif kind == "c3k2":
        cases.append(("out", _nchw(outs["out"]), lambda: oc.csp_op(ins, d, params, dtype)))
    elif kind == "c3k":
        cases.append(("out", _nchw(outs["out"]), lambda: oc.c3k_op(ins, d, params, dtype)))
    elif kind == "head_cls":
        for l in range(3):
            if f"x{l}" not in ins:
                continue
            cv = d["convs"][5 * l:5 * l + 5]
            if d["direct"]:
                h, w = H >> (3 + l), W >> (3 + l)
                a0 = _anchor_off(l, H, W)
                dev = y[:, 4:4 + nc, a0:a0 + h * w].reshape(y.shape[0], nc, h, w)
                fn = lambda l=l, cv=cv: oc.rnd_iv(*oc.sigmoid_iv(*oc.head_cls_level(ins[f"x{l}"], cv, params, dtype)),
                                                  dtype)
                cases.append((f"level {l} scores", dev, fn))
            else:
                cases.append((f"level {l} logits", _nchw(outs[f"y{l}"])[:, :nc],
                              lambda l=l, cv=cv: oc.head_cls_level(ins[f"x{l}"], cv, params, dtype)))
    elif kind == "box_dfl":
        for l in range(3):
            h, w = H >> (3 + l), W >> (3 + l)
            a0 = _anchor_off(l, H, W)
            fn = lambda l=l: oc.dfl_box(*oc.layer(ins[f"x{l}"], ins[f"x{l}"], d["convs"][l], params, dtype), 8 << l,
                                        dtype)
            cases.append((f"level {l} boxes", y[:, 0:4, a0:a0 + h * w], fn))
    elif kind == "box_chain":
        for l in range(3):
            h, w = H >> (3 + l), W >> (3 + l)
            a0 = _anchor_off(l, H, W)
            c0, c1, c2 = d["convs"][3 * l:3 * l + 3]

            def fn(l=l, c0=c0, c1=c1, c2=c2):
                lo, hi = oc.layer(ins[f"x{l}"], ins[f"x{l}"], c0, params, dtype)
                lo, hi = oc.layer(lo, hi, c1, params, dtype)
                return oc.dfl_box(*oc.layer(lo, hi, c2, params, dtype), 8 << l, dtype)
            cases.append((f"level {l} boxes", y[:, 0:4, a0:a0 + h * w], fn))
    elif kind == "pw_chain":
        # stage by stage: inputs from the device operands (captured before the chain ran) or from
        # an earlier stage's output interval; compared where no later stage overwrote the output
        def chain_iv():
            iv = []
            for k, stg in enumerate(d["stages"]):
                conv = d["convs"][k]
                los, his = [], []
                for r in stg["runs"]:
                    if r["src"] < 0:
                        t = ins[f"s{k}.in{r['seg']}"][:, r["off"]:r["off"] + r["n"]]
                        los.append(t)
                        his.append(t)
                    else:
                        lo, hi = iv[r["src"]]
                        los.append(lo[:, r["soff"]:r["soff"] + r["n"]])
                        his.append(hi[:, r["soff"]:r["soff"] + r["n"]])
                res = None
                if stg["res"] == -1:
                    res = oc.exact(ins[f"s{k}.res"][:, :conv["cout"]])
                elif stg["res"] >= 0:
                    lo, hi = iv[stg["res"]]
                    o = stg["res_off"]
                    res = (lo[:, o:o + conv["cout"]], hi[:, o:o + conv["cout"]])
                iv.append(oc.layer(torch.cat(los, 1), torch.cat(his, 1), conv, params, dtype, res=res))
            return iv
        for k, stg in enumerate(d["stages"]):
            if stg["final"]:
                cases.append((f"stage {k} out", _nchw(outs[f"s{k}.out"])[:, :d["convs"][k]["cout"]],
                              lambda k=k: chain_iv()[k]))
    elif kind == "decode":
        for l in range(3):
            L = ins[f"L{l}"]
            h, w = H >> (3 + l), W >> (3 + l)
            a0 = _anchor_off(l, H, W)
            if l >= d["dlo"]:
                lg = L[:, 64:64 + nc]
                dev = y[:, 4:4 + nc, a0:a0 + h * w].reshape(y.shape[0], nc, h, w)
                cases.append((f"level {l} scores", dev, lambda lg=lg: oc.rnd_iv(*oc.sigmoid_iv(lg, lg), dtype)))
            if d["dbox"]:
                cases.append((f"level {l} boxes", y[:, 0:4, a0:a0 + h * w],
                              lambda L=L, l=l: oc.dfl_box(L[:, :64], L[:, :64], 8 << l, dtype)))
    else:
        raise AssertionError(f"no oracle for op kind {kind}")
    st = []
    for what, dev, fn in cases:
        lo, hi = fn()
        with oc.exact_values():
            ref, _ = fn()
        st.append(oc.compare(dev, lo, hi, ref, dtype, what))
    return st


# Share of elements more than one ulp from the correctly rounded exact result, per op kind.
# Single-layer ops: 0.1 % (measured r05: at most 8e-5, the cancellation elements). Fused chains
# carry a layer's undecided roundings (1 ulp either way, both legitimate) into the next layer's
# K-sum, and attention rounds its softmax weights to the dtype for the P.V MFMA, so those kinds
# get a ceiling of about twice the largest share measured over C2 / n fp16 / C3 / C5 in r05
# (gpurun_out r5final2: c3k 4.8e-2, attention 1.04e-2, pw_chain 4.9e-3, c3k2 4.1e-3, head_cls
# 1.1e-3, stem_fused 8.6e-4, box_chain 0): a regression that stays inside the (wider) propagated
# intervals still shows up here.
OVER1_MAX = {"c3k": 0.10, "attention": 0.025, "pw_chain": 0.012, "c3k2": 0.01, "head_cls": 0.003,
             "stem_fused": 0.002, "box_chain": 1e-3}
# Interval width (tests/_opcheck.py ulp_width: (hi - lo) in ulps of the dtype at the interval's
# magnitude; 0 = pinned, 1 = two adjacent values), (p50, p99) per op kind: the freedom the proven
# bound leaves a kernel. It is the oracle's looseness, not the device's error: the (2K + 4) u
# K-sum bound grows with K and with cancellation (|y| << sum |x w|), so the long 3x3 K-sums of C5
# (K up to 3456) reach p99 ~1800, and fused chains carry every layer's interval into the next
# (c3k: six layers, p50 ~1800). The device's own error is what over1 measures (share beyond one
# ulp of the correctly rounded exact value). Bounds: ~1.5x the r06 maxima over C2 / C2 unfused /
# n fp16 / C3 / C5 / box chain (gpurun_out r6b), so a loosened oracle shows up as well.
# The fused kinds are pinned transitively rather than by their own intervals: each is bit-identical
# to its per-layer launches (tests/test_gpu_fusion.py), and those launches meet the single-layer
# bar (over1 <= 0.1 %, every element in its interval) at v11_n's shapes in test_op_parity_c2_unfused.
WIDTH_MAX = {"conv": (128, 2700), "stem": (1, 4), "dwconv": (1, 4), "decode": (1, 2), "box_dfl": (1, 2),
             "sppf": (0, 0), "stem_fused": (8, 360), "attention": (6, 240), "c3k2": (96, 2400),
             "c3k": (2700, 5300), "pw_chain": (600, 4200), "head_cls": (36, 128), "box_chain": (24, 264)}


def run_op_parity(gpu, variant, dtype, batch, size, images, seed):
    from yolo_hip.engine import Engine
    model = make_model(variant)
    params = oc.Params(model.state_dict(), dtype)
    x = synth.synth_scenes(batch, size, size, seed=seed).to(gpu, dtype)
    eng = Engine(*model._yh_arch, gpu, dtype)
    eng.load_module(model)
    y = eng.forward(x).clone()
    torch.cuda.synchronize()
    nc = eng.num_classes
    H = W = size
    kernels = {i: o["kernel"] for i, o in enumerate(eng.ops(batch, H, W))}
    yd = torch.full_like(y, float("nan"))
    img = torch.tensor(images)
    x_sel = x[img].cpu()
    kinds, failures = set(), []
    n_checked = 0
    for i in range(len(kernels)):
        d = eng.debug_op_desc(i, batch, H, W)
        if d["active"] != 1:
            continue
        ins = {}
        for s, o in enumerate(d["operands"]):
            if o["role"] in IN_ROLES or o["role"].split(".")[-1] in IN_ROLES:
                ins[o["role"]] = _nchw(eng.debug_operand(i, s, batch, d)[img].cpu()).double()
        eng.debug_run(x, yd, i, i + 1)
        outs = {}
        for s, o in enumerate(d["operands"]):
            if not (o["role"] in IN_ROLES or o["role"].split(".")[-1] in IN_ROLES):
                outs[o["role"]] = eng.debug_operand(i, s, batch, d)[img].cpu()
        torch.cuda.synchronize()
        st = _check_op(d, ins, outs, x_sel, yd[img].cpu(), H, W, nc, params, dtype)
        kinds.add(d["kind"])
        for s in st:
            n_checked += s["n"]
            print(f"{d['label']:<28} {kernels[i] or d['kind']:<36} {s['what']:<18} n={s['n']:<9} "
                  f"pinned {s['pinned']:.5f} exact {s['exact']:.5f} >1ulp {s['over1']:.2e} max_ulp {s['max_ulp']} "
                  f"width p50 {s['w50']:.2f} p99 {s['w99']:.2f} p99.9 {s['w999']:.1f} >4 {s['wide']:.2e} "
                  f"max {s['wmax']:.0f} bad {s['bad']}")
            # every element within its proven interval; the share beyond one ulp and the
            # interval width under the op kind's ceilings (OVER1_MAX, WIDTH_MAX)
            w50, w99 = WIDTH_MAX[d["kind"]]
            if s["bad"] or s["over1"] > OVER1_MAX.get(d["kind"], 1e-3) or s["w50"] > w50 or s["w99"] > w99:
                failures.append((d["label"], kernels[i], s))
    assert not failures, failures[:4]
    # the stepped forward reproduces the graph forward bit for bit
    assert torch.equal(yd, y)
    return kinds, n_checked


def test_op_parity_c2_n_bf16_b32(gpu):
    kinds, n = run_op_parity(gpu, "n", torch.bfloat16, 32, 640, (0, 17, 31), seed=21)
    assert {"stem_fused", "conv", "c3k2", "c3k", "sppf", "attention", "head_cls", "box_dfl", "pw_chain"} <= kinds, kinds


def test_op_parity_c2_unfused(gpu, monkeypatch):
    """C2 with every cross-layer fusion off (at handle creation): the per-layer launches that
    each fused kernel is bit-identical to (tests/test_gpu_fusion.py) run at v11_n's fused shapes
    and must meet the single-layer bar themselves (<= 0.1 % beyond one ulp, interval p99 width
    <= 4 ulps), which closes the transitive pin of the fused kernels."""
    for k in ("YH_FUSE", "YH_PWCHAIN", "YH_C3K", "YH_HCLS_WIDE"):
        monkeypatch.setenv(k, "0")
    kinds, n = run_op_parity(gpu, "n", torch.bfloat16, 32, 640, (0, 17, 31), seed=21)
    assert not kinds & {"stem_fused", "c3k2", "c3k", "head_cls", "pw_chain", "box_chain"}, kinds
    assert {"stem", "conv", "dwconv", "sppf", "attention", "decode"} <= kinds, kinds


def test_op_parity_n_fp16(gpu):
    kinds, n = run_op_parity(gpu, "n", torch.float16, 2, 640, (0, 1), seed=22)
    assert {"stem_fused", "conv", "c3k2", "c3k", "sppf", "attention", "head_cls", "box_dfl"} <= kinds, kinds


def test_op_parity_c3_s_fp16_b64(gpu):
    kinds, n = run_op_parity(gpu, "s", torch.float16, 64, 640, (0, 63), seed=23)
    assert {"stem_fused", "conv", "c3k2", "dwconv", "decode", "box_dfl", "attention", "sppf"} <= kinds, kinds


def test_op_parity_c5_x_bf16_1280(gpu):
    kinds, n = run_op_parity(gpu, "x", torch.bfloat16, 1, 1280, (0,), seed=24)
    assert {"stem", "conv", "dwconv", "decode", "box_dfl", "attention", "sppf"} <= kinds, kinds
    # (x: 96 box channels, the per-layer box convs + box_dfl)


def test_op_parity_box_chain_n_bf16(gpu, monkeypatch):
    """The opt-in fused box branch (boxc.hip, YH_BOXCHAIN=1 at handle creation) op by op."""
    monkeypatch.setenv("YH_BOXCHAIN", "1")
    kinds, n = run_op_parity(gpu, "n", torch.bfloat16, 2, 640, (0, 1), seed=25)
    assert "box_chain" in kinds, kinds
