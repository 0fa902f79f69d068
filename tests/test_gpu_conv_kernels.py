"""Every dense-conv kernel implementation gives bit-identical forwards. Marked gpu.

The per-shape autotuner (csrc/engine.cpp ensure_tuned) may pick any of
conv_gemm2 (3 tile shapes), conv_stream (2-, 4- and 8-slot rings),
conv_direct and conv_tiny per layer. That is only valid because they all accumulate K in the
same order (32-deep MFMA steps, increasing k): this test forces each one on
every layer that supports it and requires the exact same head output as the
reference kernel (conv_gemm2), which the forward parity tests pin to the oracle.
"""
import pytest
import torch

from yolo_hip import synth

pytestmark = pytest.mark.gpu

KERNELS = ["gemm", "gemm64", "gemm128", "stream", "direct", "stream4", "stream8", "tiny"]


@pytest.mark.parametrize("dtype,batch", [(torch.bfloat16, 32), (torch.float16, 4)])
def test_all_conv_kernels_bit_identical(gpu, dtype, batch):
    from nets import nn
    from yolo_hip.engine import Engine
    torch.manual_seed(0)
    model = nn.yolo_v11_n(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    eng = Engine(*model._yh_arch, gpu, dtype)
    eng.load_module(model)
    x = synth.synth_scenes(batch, 640, 640, seed=11).to(gpu, dtype)
    outs = {}
    for k, name in enumerate(KERNELS):
        eng.force_conv_kernel(k)
        outs[name] = eng.forward(x).clone()
        used = {o["kernel"] for o in eng.ops(batch, 640, 640) if o["cls"] in ("conv1x1", "conv3x3")}
        assert name in used, f"kernel {name} ran on no layer ({used})"
    eng.force_conv_kernel(-1)
    outs["tuned"] = eng.forward(x).clone()
    ref = outs["gemm"]
    assert torch.isfinite(ref.float()).all()
    for name, y in outs.items():
        assert torch.equal(y, ref), f"{name}: {(y.float() - ref.float()).abs().max().item()} max diff vs gemm"
