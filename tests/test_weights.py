"""Weight ingest (yolo_hip.weights; reference utils/util.py:345-516).

CPU: the "reference" Ultralytics mapping reproduces, key for key, what the
reference's own load_ultralytics_weight did (tests/golden/ultralytics_map_*.json,
oracle/make_weight_goldens.py); load_weight loads exactly the reference's key
set; the "exact" mapping round-trips every tensor; checkpoints that pickle
objects are refused unless trusted. GPU: weights loaded from a checkpoint file
give the bit-identical HIP forward of the model they came from, and re-loading
re-packs the device weights.
"""
import json
import os

import pytest
import torch

from conftest import GOLD
from yolo_hip import synth
from yolo_hip.weights import (load_ultralytics_weight, load_weight, map_ultralytics, read_checkpoint,
                              ultralytics_names)


def _model(v="n", seed=0):
    from nets import nn
    torch.manual_seed(0)
    m = getattr(nn, f"yolo_v11_{v}")(80)
    if seed is not None:
        m.load_state_dict(synth.synth_state_dict(m.state_dict(), seed=seed))
    return m.eval()


def _ultra_sd(model):
    names = ultralytics_names(model)
    return {names[k]: v.clone() for k, v in model.state_dict().items()}


@pytest.mark.parametrize("v", ["n", "m", "x"])
def test_reference_mapping_matches_reference_loader(v):
    with open(os.path.join(GOLD, f"ultralytics_map_{v}.json")) as f:
        gold = json.load(f)
    model = _model(v, seed=None)
    src = _ultra_sd(model)
    assert sorted(src) == gold["src_keys"], "Ultralytics key schema changed since the golden was made"
    mapped = map_ultralytics(src, model, "reference")
    back = {id(t): k for k, t in src.items()}
    got = sorted([back[id(t)], k] for k, t in mapped.items())
    assert got == gold["mapped"]


@pytest.mark.parametrize("v", ["n", "x"])
def test_exact_mapping_round_trips_every_tensor(v, tmp_path):
    src_model = _model(v, seed=3)
    path = tmp_path / "ultra.pt"
    torch.save({"model": _ultra_sd(src_model)}, path)
    dst = _model(v, seed=None)
    load_ultralytics_weight(dst, str(path), mapping="exact")
    a, b = src_model.state_dict(), dst.state_dict()
    assert a.keys() == b.keys()
    for k in a:
        assert torch.equal(a[k], b[k]), k


def test_load_weight_matches_reference_key_set(tmp_path):
    with open(os.path.join(GOLD, "load_weight_n.json")) as f:
        gold = json.load(f)
    model = _model("n", seed=None)
    sd = {k: t.clone() for k, t in model.state_dict().items()}
    sd.pop("net.p1.0.conv.weight")
    sd["head.box.0.2.weight"] = torch.zeros(3, 3)
    sd["not.a.key"] = torch.zeros(2)
    assert sorted(sd) == gold["ckpt_keys"]
    seen = []
    orig = model.load_state_dict

    def spy(state_dict, strict=True):
        seen.extend(state_dict)
        return orig(state_dict, strict=strict)
    model.load_state_dict = spy
    path = tmp_path / "own.pt"
    torch.save({"model": sd}, path)
    load_weight(model, str(path))
    assert sorted(seen) == gold["loaded"]


def test_checkpoint_formats(tmp_path):
    model = _model("n", seed=1)
    sd = model.state_dict()
    from safetensors.torch import save_file
    save_file({k: v.contiguous() for k, v in sd.items()}, str(tmp_path / "w.safetensors"))
    torch.save(sd, tmp_path / "raw.pt")
    torch.save({"ema": sd, "model": None}, tmp_path / "ema.pt")
    for name in ("w.safetensors", "raw.pt", "ema.pt"):
        got = read_checkpoint(str(tmp_path / name))
        assert got.keys() == sd.keys() and all(torch.equal(got[k], sd[k]) for k in sd), name
    # a pickled module executes code on load: refused unless trusted
    torch.save({"model": model}, tmp_path / "module.pt")
    with pytest.raises(RuntimeError, match="trusted=True"):
        read_checkpoint(str(tmp_path / "module.pt"))
    got = read_checkpoint(str(tmp_path / "module.pt"), trusted=True)
    assert all(torch.equal(got[k], sd[k]) for k in sd)


def test_utils_util_exports_loaders():
    from utils import util
    assert util.load_weight and util.load_ultralytics_weight


@pytest.mark.gpu
def test_loaded_weights_drive_the_hip_forward(gpu, tmp_path):
    src = _model("n", seed=7)
    path = tmp_path / "ultra.pt"
    torch.save({"model": _ultra_sd(src)}, path)
    x = synth.synth_scenes(2, 256, 256, seed=4).to(gpu, torch.bfloat16)
    with torch.no_grad():
        want = src.to(gpu)(x).clone()
    dst = _model("n", seed=1).to(gpu)
    with torch.no_grad():
        before = dst(x).clone()          # engine packed with the old weights
    assert not torch.equal(before, want)
    load_ultralytics_weight(dst, str(path), mapping="exact")
    with torch.no_grad():
        got = dst(x)                     # new parameter versions -> re-pack on device
    assert torch.equal(got, want)
