"""Fused launches (csrc/head.hip) are bit-identical to the per-layer launches they replace.
Marked gpu.

The fused op recomputes the same layers in the same arithmetic order (per-channel depthwise
FMA chains, conv_mx's K order on v_mfma_f32_32x32x16, one rounding per layer output), so the
head output must be exactly equal with fusion on (default) and off (YH_FUSE=0 at handle
creation), for every shape: whole and partial tiles, every level, both 16-bit dtypes. The same holds
for the folded decode (box_dfl writes the box rows, head_cls or a class-rows decode the
scores), including anchor counts that are not a multiple of 8 (96 x 160: A = 315), and for
the fused C3k2 blocks (c3k2.hip: conv1 -> Residual -> conv2 in one launch), whole and
partial tiles, and for the fused stem (conv.hip stem_fused: the stem and net.p2.0 in one
launch, the stem output only in LDS), with the engine-dtype and the uint8 input.
"""
import os

import pytest
import torch

from _util import make_model
from yolo_hip import synth

pytestmark = pytest.mark.gpu


def _engine(model, dtype, dev, fuse, **env):
    """Engine built with YH_FUSE (and any extra YH_* settings) set at handle creation."""
    from yolo_hip.engine import Engine
    env = {"YH_FUSE": "1" if fuse else "0", **env}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        eng = Engine(*model._yh_arch, dev, dtype)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    eng.load_module(model)
    return eng


@pytest.mark.parametrize("variant,dtype,batch,h,w", [("n", torch.bfloat16, 4, 640, 640), ("n", torch.float16, 2, 320, 256),
                                                     ("s", torch.bfloat16, 2, 384, 640), ("x", torch.bfloat16, 1, 320, 320),
                                                     ("n", torch.float16, 3, 96, 160)])
def test_fused_head_equals_per_layer_launches(gpu, variant, dtype, batch, h, w):
    model = make_model(variant)
    x = synth.synth_scenes(batch, h, w, seed=31).to(gpu, dtype)
    fused = _engine(model, dtype, gpu, True)
    plain = _engine(model, dtype, gpu, False)
    kinds_f = {o["cls"] for o in fused.ops(batch, h, w)}
    kinds_p = {o["cls"] for o in plain.ops(batch, h, w)}
    assert "head_cls" not in kinds_p and "box_dfl" not in kinds_p
    assert "box_dfl" in kinds_f   # decode folded into the box tail (+ head_cls / class-rows decode)
    if variant in ("n", "s"):   # C3k2 blocks with one Residual: net.p2.1 (n, s), net.p3.1 (n)
        assert "c3k2" in kinds_f and "c3k2" not in kinds_p
        # stem + net.p2.0 (16 -> 32 / 32 -> 64) in one launch
        assert "net.p1.0+p2.0" in [o["label"] for o in fused.ops(batch, h, w)]
        assert "net.p1.0+p2.0" not in [o["label"] for o in plain.ops(batch, h, w)]
    if variant == "n":   # s (128) / x (384) cls branches keep the per-layer launches
        assert "head_cls" in kinds_f
        assert len(fused.ops(batch, h, w)) < len(plain.ops(batch, h, w))
    yf = fused.forward(x).clone()
    yp = plain.forward(x).clone()
    assert torch.isfinite(yf.float()).all()
    assert torch.equal(yf, yp), (yf.float() - yp.float()).abs().max().item()
    fused.set_graph(False)
    assert torch.equal(fused.forward(x), yp)


@pytest.mark.parametrize("dtype,batch,h,w", [(torch.bfloat16, 2, 640, 640), (torch.float16, 3, 96, 160)])
def test_csp_tail_mode_equals_per_layer_launches(gpu, dtype, batch, h, w):
    """C3k2 tail mode (conv1 launched alone, Residual + conv2 fused; the default for
    fpn.h2's two-segment input) forced on every eligible block of v11_n."""
    model = make_model("n")
    x = synth.synth_scenes(batch, h, w, seed=37).to(gpu, dtype)
    tail = _engine(model, dtype, gpu, True, YH_CSP_TAIL="1")
    plain = _engine(model, dtype, gpu, False)
    labels = [o["label"] for o in tail.ops(batch, h, w) if o["cls"] == "c3k2"]
    assert "net.p3.1.tail" in labels and "fpn.h2.tail" in labels, labels
    yt = tail.forward(x).clone()
    yp = plain.forward(x).clone()
    assert torch.equal(yt, yp), (yt.float() - yp.float()).abs().max().item()


@pytest.mark.parametrize("variant,dtype,batch,h,w", [("n", torch.float16, 2, 640, 640), ("s", torch.bfloat16, 3, 96, 160)])
def test_fused_stem_uint8_input(gpu, variant, dtype, batch, h, w):
    """The fused stem stages the loader's uint8 image with main.py:265-267's `/ 255` exactly
    like the per-layer stem: uint8 forwards with fusion on and off are bit-identical."""
    model = make_model(variant)
    g = torch.Generator().manual_seed(5)
    x8 = torch.randint(0, 256, (batch, 3, h, w), dtype=torch.uint8, generator=g).to(gpu)
    fused = _engine(model, dtype, gpu, True)
    plain = _engine(model, dtype, gpu, False)
    yf = fused.forward(x8).clone()
    yp = plain.forward(x8).clone()
    assert torch.equal(yf, yp), (yf.float() - yp.float()).abs().max().item()
    assert torch.equal(fused.forward(x8.to(dtype) / 255), yf)


@pytest.mark.parametrize("variant,dtype,batch,h,w,nfused", [("n", torch.bfloat16, 2, 640, 640, 3),
                                                           ("n", torch.float16, 3, 96, 160, 3),
                                                           ("n", torch.bfloat16, 2, 608, 480, 3),
                                                           ("n", torch.bfloat16, 1, 1280, 1280, 0),
                                                           ("s", torch.float16, 2, 640, 640, 0),
                                                           ("s", torch.bfloat16, 1, 1280, 1280, 0)])
def test_c3k_block_equals_per_layer_launches(gpu, variant, dtype, batch, h, w, nfused):
    """c3k.hip: a CSPModule(c, c) block with c = 64 or 128 in one launch wherever bands of at
    least 4 rows (+ the 4-row halo) fit a workgroup's LDS, for c = 128 only where the bands allow
    the SPLIT mode (phases within 8 pixel tiles): v11_n's 40x40 (c = 64) net.p4.1 and 20x20
    (c = 128) net.p5.1 / fpn.h6 at 640 and 608x480 / 96x160, none at 1280 (80x80 c = 64 bands
    are too wide, 40x40 c = 128 ones too tall for SPLIT); none for v11_s (40x40 c = 128, 20x20
    c = 256). YH_C3K=0 keeps the seven per-layer launches everywhere. Bit-identical either way."""
    model = make_model(variant)
    x = synth.synth_scenes(batch, h, w, seed=37).to(gpu, dtype)
    # pointwise chains off in both: with YH_C3K=0 the per-layer C3k 1x1 convs would form chains
    # of their own and change the launch count this test compares
    fused = _engine(model, dtype, gpu, True, YH_PWCHAIN="0")
    plain = _engine(model, dtype, gpu, True, YH_C3K="0", YH_PWCHAIN="0")
    yf = fused.forward(x).clone()
    yp = plain.forward(x).clone()
    kinds_f = [u["cls"] for u in fused.units(batch, h, w)]
    kinds_p = [u["cls"] for u in plain.units(batch, h, w)]
    assert "c3k" not in kinds_p
    assert kinds_f.count("c3k") == nfused, kinds_f
    assert len(kinds_p) - len(kinds_f) == 6 * nfused   # seven launches -> one per fused block
    assert torch.isfinite(yf.float()).all()
    assert torch.equal(yf, yp), (yf.float() - yp.float()).abs().max().item()


@pytest.mark.parametrize("dtype,batch,h,w", [(torch.bfloat16, 2, 640, 640), (torch.float16, 3, 96, 160),
                                             (torch.bfloat16, 1, 352, 480)])
def test_head_cls_wide_level_equals_per_layer_launches(gpu, dtype, batch, h, w):
    """head.hip: v11_n's 20x20 cls branch (256 input channels: four 64-channel dw1 chunks, pw1
    over 16 K blocks in two halves) joins the fused head_cls launch, and with every level fused
    the class-rows decode disappears (5 + 1 launches fewer); YH_HCLS_WIDE=0 keeps its per-layer
    launches. Bit-identical either way."""
    model = make_model("n")
    x = synth.synth_scenes(batch, h, w, seed=41).to(gpu, dtype)
    wide = _engine(model, dtype, gpu, True)
    plain = _engine(model, dtype, gpu, True, YH_HCLS_WIDE="0")
    yf = wide.forward(x).clone()
    yp = plain.forward(x).clone()
    lf = [u["label"] for u in wide.units(batch, h, w)]
    lp = [u["label"] for u in plain.units(batch, h, w)]
    assert "head.decode_cls" in lp and "head.cls.2.1" in lp, lp
    assert not any(l.startswith("head.cls.") or l.startswith("head.decode") for l in lf), lf
    assert len(lp) - len(lf) == 6
    assert torch.isfinite(yf.float()).all()
    assert torch.equal(yf, yp), (yf.float() - yp.float()).abs().max().item()


@pytest.mark.parametrize("variant,dtype,batch,size", [("n", torch.bfloat16, 4, 640), ("s", torch.float16, 2, 320),
                                                      ("x", torch.bfloat16, 1, 1280), ("n", torch.float16, 2, 224)])
def test_attention_lds_kernel_equals_per_wave_kernel(gpu, variant, dtype, batch, size):
    """misc.hip psa_attention_lds (K / V staged in LDS once per workgroup, chunks of 256 keys)
    runs psa_attention_mfma's per-16-key-block arithmetic in the same order: bit-identical, also
    over several chunks (x at 1280: 1600 tokens) and with a partial last block (224: 49 tokens).
    YH_ATTN_LDS is read at launch, so each engine captures its own kernel."""
    model = make_model(variant)
    x = synth.synth_scenes(batch, size, size, seed=33).to(gpu, dtype)
    ys = []
    old_full = os.environ.get("YH_ATTN_FULL")
    os.environ["YH_ATTN_FULL"] = "0"   # the chunked kernel, not the whole-K/V one, where both apply
    try:
        for v in ("0", "1"):
            old = os.environ.get("YH_ATTN_LDS")
            os.environ["YH_ATTN_LDS"] = v
            try:
                eng = _engine(model, dtype, gpu, True)
                ys.append(eng.forward(x).clone())
                torch.cuda.synchronize()
            finally:
                if old is None:
                    del os.environ["YH_ATTN_LDS"]
                else:
                    os.environ["YH_ATTN_LDS"] = old
    finally:
        if old_full is None:
            del os.environ["YH_ATTN_FULL"]
        else:
            os.environ["YH_ATTN_FULL"] = old_full
    assert torch.isfinite(ys[0].float()).all()
    assert torch.equal(ys[0], ys[1])


@pytest.mark.parametrize("variant,dtype,batch,size", [("n", torch.bfloat16, 4, 640), ("s", torch.float16, 2, 320),
                                                      ("n", torch.float16, 2, 224), ("m", torch.bfloat16, 2, 480)])
def test_attention_full_kernel_equals_chunked_kernel_and_pe_add(gpu, variant, dtype, batch, size):
    """misc.hip psa_attention_full (one workgroup per (image, head), the whole K / V in LDS, the
    positional term added in the epilogue) is bit-identical to the chunked kernel followed by
    pe_add (YH_ATTN_FULL=0), including partial key blocks (224: 49 tokens) and several heads
    (m: 4 heads at 480 -> 225 tokens). Both workgroup shapes of the full kernel: these small
    batches pick 8 waves with one 16-query block per wave, YH_ATTN_NW=16 forces the 16-wave shape
    the large batches use (YH_ATTN_QS=1: several query blocks per wave)."""
    model = make_model(variant)
    x = synth.synth_scenes(batch, size, size, seed=34).to(gpu, dtype)
    ys = []
    for env in ({"YH_ATTN_FULL": "0"}, {"YH_ATTN_FULL": "1"}, {"YH_ATTN_FULL": "1", "YH_ATTN_NW": "16", "YH_ATTN_QS": "1"}):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            eng = _engine(model, dtype, gpu, True)
            ys.append(eng.forward(x).clone())
            torch.cuda.synchronize()
        finally:
            for k, v in old.items():
                if v is None:
                    del os.environ[k]
                else:
                    os.environ[k] = v
    assert torch.isfinite(ys[0].float()).all()
    for y in ys[1:]:
        assert torch.equal(ys[0], y), (ys[0].float() - y.float()).abs().max().item()


@pytest.mark.parametrize("variant,dtype,batch,size", [("n", torch.bfloat16, 4, 640), ("s", torch.float16, 2, 320),
                                                      ("x", torch.bfloat16, 1, 1280), ("n", torch.float16, 2, 224)])
def test_sppf_kernel_equals_three_maxpools(gpu, variant, dtype, batch, size):
    """misc.hip sppf_fused (CPW 8-channel chunks of one image per workgroup: 1 or 2 by default,
    halved until the planes fit the LDS) with the default and 1, 2, 4 and 8 chunks (YH_SPPF_CPW;
    8 fits at 20x20, 40x40 falls back to 2) is bit-identical to three maxpool5 launches
    (YH_SPPF_FUSED=0).
    Both switches are read at launch."""
    model = make_model(variant)
    x = synth.synth_scenes(batch, size, size, seed=35).to(gpu, dtype)
    ys = []
    for env in ({"YH_SPPF_FUSED": "0"}, {"YH_SPPF_CPW": "1"}, {}, {"YH_SPPF_CPW": "2"}, {"YH_SPPF_CPW": "4"},
                {"YH_SPPF_CPW": "8"}):
        old = {k: os.environ.get(k) for k in ("YH_SPPF_FUSED", "YH_SPPF_CPW")}
        os.environ.update(env)
        try:
            eng = _engine(model, dtype, gpu, True)
            ys.append(eng.forward(x).clone())
            torch.cuda.synchronize()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    assert torch.isfinite(ys[0].float()).all()
    for yv in ys[1:]:
        assert torch.equal(ys[0], yv)


@pytest.mark.parametrize("bands", ["1", "2", "3", "5", "7", "20"])
def test_c3k_row_bands_equal_per_layer_launches(gpu, bands):
    """c3k.hip row bands: each image's block is split over `bands` workgroups that recompute the
    4-row halo of the chain of four 3x3 convs; every split (1 = one workgroup per image where the
    region fits, 20 = one row each at 20x20, uneven splits, a last band with no rows; the 40x40
    h = 32 block takes at least the 10 bands its regions need and the 20x20 h = 64 blocks at least
    the 4 bands of their SPLIT mode, the only mode h = 64 runs in) is bit-identical to the seven
    per-layer launches. YH_C3K_BANDS is read at launch."""
    model = make_model("n")
    x = synth.synth_scenes(2, 640, 640, seed=38).to(gpu, torch.bfloat16)
    plain = _engine(model, torch.bfloat16, gpu, True, YH_C3K="0")
    yp = plain.forward(x).clone()
    old = os.environ.get("YH_C3K_BANDS")
    os.environ["YH_C3K_BANDS"] = bands
    try:
        fused = _engine(model, torch.bfloat16, gpu, True)
        yf = fused.forward(x).clone()
        torch.cuda.synchronize()
    finally:
        if old is None:
            del os.environ["YH_C3K_BANDS"]
        else:
            os.environ["YH_C3K_BANDS"] = old
    assert [u["cls"] for u in fused.units(2, 640, 640)].count("c3k") == 3
    assert torch.equal(yf, yp), (yf.float() - yp.float()).abs().max().item()


@pytest.mark.parametrize("variant,dtype,batch,h,w", [("n", torch.bfloat16, 4, 640, 640), ("n", torch.float16, 3, 96, 160),
                                                     ("n", torch.bfloat16, 2, 608, 480), ("n", torch.bfloat16, 1, 1280, 1280),
                                                     ("s", torch.float16, 2, 384, 640), ("m", torch.bfloat16, 1, 320, 320)])
def test_box_chain_equals_per_layer_launches(gpu, variant, dtype, batch, h, w):
    """boxc.hip (opt-in, YH_BOXCHAIN=1): the box branch of all three levels (box.l.0 3x3 -> box.l.1 3x3
    -> box.l.2 1x1 + DFL + anchors + dist2bbox) in one launch, the 64-channel intermediates in LDS, is
    bit-identical to the seven per-layer launches (YH_BOXCHAIN=0): whole and partial tiles, level inputs of 64 / 128 / 256
    (n) and 128 / 256 / 512 (s) channels, K-split (mx_kchunks: 640, 40x40 / 20x20 levels) and
    unsplit box.l.0 shapes (1280: 80x80 / 40x40), an anchor count that is not a multiple of 8."""
    model = make_model(variant)
    x = synth.synth_scenes(batch, h, w, seed=43).to(gpu, dtype)
    fused = _engine(model, dtype, gpu, True, YH_BOXCHAIN="1")   # opt-in (slower than the per-layer launches)
    plain = _engine(model, dtype, gpu, True, YH_BOXCHAIN="0")
    yf = fused.forward(x).clone()
    yp = plain.forward(x).clone()
    lf = [u["label"] for u in fused.units(batch, h, w)]
    lp = [u["label"] for u in plain.units(batch, h, w)]
    assert "head.box" in lf and "head.box_dfl" not in lf and not any(l.startswith("head.box.") for l in lf), lf
    assert "head.box" not in lp and "head.box_dfl" in lp
    assert len(lp) - len(lf) == 6
    assert torch.isfinite(yf.float()).all()
    assert torch.equal(yf, yp), (yf.float() - yp.float()).abs().max().item()


@pytest.mark.parametrize("variant,dtype,batch,h,w,nchain", [("n", torch.bfloat16, 2, 640, 640, 3),
                                                           ("n", torch.float16, 3, 96, 160, 3),
                                                           ("n", torch.bfloat16, 32, 640, 640, 3),
                                                           ("s", torch.float16, 2, 640, 640, 3),
                                                           ("x", torch.bfloat16, 1, 640, 640, 3),
                                                           ("n", torch.bfloat16, 1, 1280, 1280, 3)])
def test_pw_chain_equals_per_layer_launches(gpu, variant, dtype, batch, h, w, nchain):
    """pwchain.hip: runs of consecutive 1x1 convs on a 40x40-or-smaller map (the C3k2 conv2 ->
    SPPF conv1 pair, SPPF conv2 -> C2PSA conv1 -> qkv, and the PSABlock after the attention core:
    proj (+x) -> ffn -> ffn (+x) -> C2PSA conv2 over [a | b]) as one launch each, the stage
    outputs a later stage reads kept in LDS, are bit-identical to the per-layer launches
    (YH_PWCHAIN=0): 64- and 32-pixel workgroups (s, x: the wider stages take 32), a partial last
    workgroup (96x160: a 3x5 map at the coarsest level), concat inputs split between LDS and global
    sources, residuals from LDS and from global."""
    model = make_model(variant)
    x = synth.synth_scenes(batch, h, w, seed=47).to(gpu, dtype)
    fused = _engine(model, dtype, gpu, True)
    plain = _engine(model, dtype, gpu, True, YH_PWCHAIN="0")
    yf = fused.forward(x).clone()
    yp = plain.forward(x).clone()
    uf = fused.units(batch, h, w)
    up = plain.units(batch, h, w)
    chains = [u["label"] for u in uf if u["cls"] == "pw_chain"]
    print(variant, h, w, chains)
    assert len(chains) >= nchain, [u["label"] for u in uf]   # s / x: more runs at 40x40 too
    assert "pw_chain" not in [u["cls"] for u in up]
    assert len(up) > len(uf)
    assert torch.isfinite(yf.float()).all()
    assert torch.equal(yf, yp), (yf.float() - yp.float()).abs().max().item()
