"""Fused preprocessing: the loader's uint8 image batch
goes straight into the forward (yh_forward_u8); the stem applies main.py:265-267's
`samples.half() / 255.` while staging its input. Marked gpu.

Parity bar: bit-identical head output to the same engine fed torch's own
`x.to(dtype) / 255.` on the device, for every handle dtype, graph on and off.
"""
import pytest
import torch

from yolo_hip import synth

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float16, torch.float32])
def test_uint8_input_matches_torch_preprocessing(gpu, dtype):
    from nets import nn
    from yolo_hip.engine import Engine
    torch.manual_seed(0)
    model = nn.yolo_v11_n(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    eng = Engine(*model._yh_arch, gpu, dtype)
    eng.load_module(model.eval())
    g = torch.Generator().manual_seed(5)
    x8 = torch.randint(0, 256, (3, 3, 320, 288), generator=g, dtype=torch.uint8)
    x8[0, :, :20] = 114   # letterbox-style flat border rows
    x8 = x8.to(gpu)
    want = eng.forward(x8.to(dtype) / 255.).clone()
    got = eng.forward(x8).clone()
    assert torch.equal(got, want), (got.float() - want.float()).abs().max().item()
    eng.set_graph(False)
    assert torch.equal(eng.forward(x8), want)
    # both input kinds keep their own captured graph
    eng.set_graph(True)
    assert torch.equal(eng.forward(x8.to(dtype) / 255.), want)
    assert torch.equal(eng.forward(x8), want)
