"""Every conv_mx plan gives bit-identical forwards. Marked gpu.

The per-shape autotuner (csrc/engine.cpp ensure_tuned) picks, per layer, one of
the layer's conv_mx candidate plans (csrc/conv_mx.hip: conv_mx with staged
weights, conv_mxr with resident weights; csrc/conv_rw.hip: weights in VGPRs with a
shared patch ring; different tile shapes, cout slices and 16-channel blocks per stage). That is only valid because every plan follows one
reduction order (conv_mx.h: for each 16-channel block, for each tap, one
32x32x16 MFMA step): this test forces candidate k on every layer (clamped to the
layer's last candidate) and requires the exact same head output for every k and
for the tuned choice. The forward parity tests pin that output to the oracle.
"""
import pytest
import torch

from yolo_hip import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("variant,dtype,batch,size", [("n", torch.bfloat16, 32, 640), ("n", torch.float16, 4, 640),
                                                      ("s", torch.float16, 64, 640), ("x", torch.bfloat16, 1, 1280)])
def test_all_conv_plans_bit_identical(gpu, variant, dtype, batch, size):
    from nets import nn
    from yolo_hip.engine import Engine
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{variant}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    eng = Engine(*model._yh_arch, gpu, dtype)
    eng.load_module(model)
    x = synth.synth_scenes(batch, size, size, seed=11).to(gpu, dtype)
    outs, names = {}, set()
    for k in range(18):
        eng.force_conv_kernel(k)
        outs[k] = eng.forward(x).clone()
        names |= {o["kernel"] for o in eng.ops(batch, size, size) if o["cls"] in ("conv1x1", "conv3x3")}
    eng.force_conv_kernel(-1)
    outs["tuned"] = eng.forward(x).clone()
    names |= {o["kernel"] for o in eng.ops(batch, size, size) if o["cls"] in ("conv1x1", "conv3x3")}
    assert any(n.startswith("mxr") for n in names) and any(n.startswith("mx_") for n in names), names
    if variant in ("n", "s"):
        assert any(n.startswith("rw_") for n in names), names
    ref = outs[0]
    assert torch.isfinite(ref.float()).all()
    for k, y in outs.items():
        assert torch.equal(y, ref), f"plan {k}: {(y.float() - ref.float()).abs().max().item()} max diff vs plan 0"
