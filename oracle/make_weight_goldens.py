"""Golden fixtures for weight ingest, made by running the
reference's own loaders in this container (never on the GPU box).

  tests/golden/ultralytics_map_<v>.json
      The reference's load_ultralytics_weight (utils/util.py:358-516) applied to
      an Ultralytics-YOLO11-named checkpoint of variant <v>: which checkpoint key
      landed on which model key ("mapped"), out of all keys ("src_keys").
      The checkpoint's key set comes from yolo_hip.weights.ultralytics_names (our
      restatement of the Ultralytics YOLO11 module tree, yolo11.yaml layers
      0-23); its values are distinct per key so a wrong landing is visible.
  tests/golden/load_weight_n.json
      The reference's load_weight (utils/util.py:345-355) on a checkpoint with
      extra keys and shape-mismatched keys: the set of model keys it loaded.

The checkpoints are files this script writes itself ({"model": module}); the
reference unpickles them with torch.load (weights_only=False in
load_ultralytics_weight; load_weight's bare torch.load defaults to
weights_only=True on torch >= 2.6 and cannot read its own module checkpoints,
so it is called with torch.load forced to weights_only=False for this file).

Usage: PYTHONDONTWRITEBYTECODE=1 python oracle/make_weight_goldens.py
"""
import contextlib
import io
import json
import os
import sys
import tempfile

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))
sys.dont_write_bytecode = True
GOLD = os.path.join(ROOT, "tests", "golden")


class Holder(torch.nn.Module):
    """A pickled 'model' whose state_dict is an arbitrary key -> tensor map."""

    def __init__(self, sd):
        super().__init__()
        self.sd = sd

    def state_dict(self, *a, **k):  # noqa: D401
        return dict(self.sd)


def ultra_checkpoint(model):
    from yolo_hip.weights import ultralytics_names
    names = ultralytics_names(model)
    sd = {}
    for i, (k, v) in enumerate(model.state_dict().items()):
        t = v.clone()
        if t.is_floating_point():
            t = torch.full_like(t, float(i) + 0.25)   # distinct value per key
        sd[names[k]] = t
    return sd


def main():
    from oracle.make_goldens import import_reference
    ref_nn, ref_util = import_reference()
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for v in ("n", "m", "x"):
            torch.manual_seed(0)
            model = getattr(ref_nn, f"yolo_v11_{v}")(80)
            src = ultra_checkpoint(model)
            path = os.path.join(tmp, f"ultra_{v}.pt")
            torch.save({"model": Holder(src)}, path)
            before = {k: t.clone() for k, t in model.state_dict().items()}
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                ref_util.load_ultralytics_weight(model, path)
            after = model.state_dict()
            # a model key was loaded iff its value now equals a checkpoint tensor's marker
            by_val = {}
            for k, t in src.items():
                if t.is_floating_point() and t.numel():
                    by_val.setdefault(float(t.flatten()[0]), []).append(k)
            mapped = []
            for k, t in after.items():
                if t.is_floating_point() and t.numel() and not torch.equal(t, before[k]):
                    cands = by_val.get(float(t.flatten()[0]), [])
                    assert len(cands) == 1, (k, cands)
                    mapped.append([cands[0], k])
            lines = [ln for ln in buf.getvalue().splitlines() if ln.startswith("Successfully mapped")]
            # integer buffers (num_batches_tracked) carry no marker: take them from the log
            for ln in lines:
                s, d = ln[len("Successfully mapped "):].split(" -> ")
                if not src[s].is_floating_point():
                    mapped.append([s, d])
            assert len(lines) == len(mapped), (len(lines), len(mapped))
            rec = dict(variant=v, src_keys=sorted(src), mapped=sorted(mapped))
            with open(os.path.join(GOLD, f"ultralytics_map_{v}.json"), "w") as f:
                json.dump(rec, f, indent=0)
            out[v] = len(mapped)
            print(f"v11_{v}: reference mapped {len(mapped)} of {len(src)} Ultralytics keys")

        # load_weight: extra keys + a shape mismatch + a missing key
        torch.manual_seed(0)
        model = ref_nn.yolo_v11_n(80)
        sd = {k: t.clone() for k, t in model.state_dict().items()}
        sd.pop("net.p1.0.conv.weight")
        sd["head.box.0.2.weight"] = torch.zeros(3, 3)              # wrong shape
        sd["not.a.key"] = torch.zeros(2)                            # extra key
        path = os.path.join(tmp, "own.pt")
        torch.save({"model": Holder(sd)}, path)
        orig = torch.load
        ref_util.torch.load = lambda f, *a, **k: orig(f, weights_only=False)
        seen = []

        def spy(state_dict, strict=True):
            seen.extend(state_dict.keys())
            return torch.nn.Module.load_state_dict(model, state_dict, strict=strict)
        model.load_state_dict = spy
        try:
            ref_util.load_weight(model, path)
        finally:
            ref_util.torch.load = orig
        with open(os.path.join(GOLD, "load_weight_n.json"), "w") as f:
            json.dump(dict(ckpt_keys=sorted(sd), loaded=sorted(seen)), f, indent=0)
        print(f"load_weight: {len(seen)} of {len(sd)} keys loaded")


if __name__ == "__main__":
    main()
