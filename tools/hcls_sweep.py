"""Per-op time of the fused head.cls launch (HIP events, eager) under several workgroup
splits over the levels (YH_HCLS_SPLIT=g0,g1,g2; "" = the engine's cost model).

python tools/hcls_sweep.py [variant] [batch] "g0,g1,g2" ...
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))

from yolo_hip import synth  # noqa: E402
from yolo_hip.engine import Engine  # noqa: E402


def main():
    v = sys.argv[1] if len(sys.argv) > 1 else "n"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    splits = sys.argv[3:] or [""]
    from nets import nn
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, torch.bfloat16)
    eng.load_module(model)
    x = synth.synth_scenes(B, 640, 640, seed=3).to(dev, torch.bfloat16)
    y = eng.forward(x)
    for sp in splits:   # "g0,g1,g2" or "g0,g1,g2/dbg"
        sp, _, dbg = sp.partition("/")
        os.environ["YH_HCLS_DBG"] = dbg or "0"
        if sp:
            os.environ["YH_HCLS_SPLIT"] = sp
        else:
            os.environ.pop("YH_HCLS_SPLIT", None)
        eng.profile(True)
        eng.profile_reset()
        for _ in range(10):
            eng.forward(x, out=y)
        eng.profile(False)
        for u in eng.units(B, 640, 640):
            if u["cls"] == "head_cls":
                print(f"split {sp or 'model':12s} dbg {dbg or 0:3} head.cls {u['ms'] / max(1, u['calls']) * 1e3:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
