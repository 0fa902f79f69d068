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


def test_device_letterbox_matches_host_path(gpu):
    """yh_letterbox (one kernel per 32 images) == yh_letterbox_host per image (same per-pixel
    code), for a batch of mixed sizes larger than one launch, host and device sources."""
    import numpy as np
    from yolo_hip import preprocess as pre
    rng = np.random.default_rng(3)
    shapes = [(480, 640), (640, 427), (1280, 1280), (1280, 960), (17, 23), (640, 640), (720, 1280), (33, 1000)]
    imgs = [rng.integers(0, 256, shapes[i % len(shapes)] + (3,), dtype=np.uint8) for i in range(37)]
    want = np.stack([pre.letterbox_host(im, 640) for im in imgs])
    got = pre.letterbox([torch.from_numpy(im).to(gpu) for im in imgs], 640)
    torch.cuda.synchronize()
    assert got.shape == (37, 3, 640, 640) and got.dtype == torch.uint8
    assert np.array_equal(got.cpu().numpy(), want)
    got2 = pre.letterbox(imgs[:3], 320, device=gpu)
    assert np.array_equal(got2.cpu().numpy(), np.stack([pre.letterbox_host(im, 320) for im in imgs[:3]]))


def test_letterboxed_batch_runs_through_forward_u8(gpu):
    import numpy as np
    from nets import nn
    from yolo_hip import preprocess as pre
    from yolo_hip.engine import Engine
    torch.manual_seed(0)
    model = nn.yolo_v11_n(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    eng = Engine(*model._yh_arch, gpu, torch.bfloat16)
    eng.load_module(model.eval())
    rng = np.random.default_rng(4)
    imgs = [rng.integers(0, 256, s + (3,), dtype=np.uint8) for s in ((480, 640), (640, 480), (300, 500))]
    x8 = pre.letterbox([torch.from_numpy(im).to(gpu) for im in imgs], 640)
    y = eng.forward(x8).clone()
    ref = eng.forward(torch.from_numpy(np.stack([pre.letterbox_host(im, 640) for im in imgs])).to(gpu)).clone()
    assert torch.equal(y, ref)


@pytest.mark.parametrize("size", [320, 640, 1280])
def test_device_letterbox_matches_restatement(gpu, size):
    """yh_letterbox on the device against oracle/preprocess.py (the numpy restatement of
    dataset.py:95-103, 292-313, 86-88 with OpenCV's INTER_LINEAR / INTER_AREA arithmetic)
    directly, bit for bit, on a mixed-size batch larger than one launch (37 images: up- and
    down-scales, exact 2x downscales, no-resize, tiny and extreme aspect ratios)."""
    import numpy as np
    from oracle import preprocess as opre
    from yolo_hip import preprocess as pre
    rng = np.random.default_rng(size)
    shapes = [(480, 640), (640, 427), (1280, 1280), (1280, 960), (17, 23), (640, 640), (720, 1280), (33, 1000),
              (2 * size, 2 * size), (size, size // 2), (2560, 1440), (12, 3000)]
    imgs = []
    for i in range(37):
        h, w = shapes[i % len(shapes)]
        im = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        if h > 4 and w > 4:   # smooth gradient in one channel: rounding at every level
            im[..., 1] = ((np.arange(w)[None, :] * 255) // max(1, w - 1)).astype(np.uint8)
        imgs.append(im)
    got = pre.letterbox([torch.from_numpy(im).to(gpu) for im in imgs], size).cpu().numpy()
    for i, im in enumerate(imgs):
        assert np.array_equal(got[i], opre.letterbox(im, size)), (i, im.shape, size)
