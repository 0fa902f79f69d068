"""Run the HIP forward and save the output, for comparing conv kernel modes (YH_CONV) bitwise.

python tools/conv_compare.py save OUT.pt [variant] [size] [batch] [dtype]
python tools/conv_compare.py diff A.pt B.pt
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))


def save(out, v="n", size=640, B=8, dt="bf16"):
    from nets import nn
    from yolo_hip import synth
    from yolo_hip.engine import Engine
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16}[dt]
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, dtype)
    eng.load_module(model)
    x = synth.synth_scenes(B, size, size, seed=5).to(dev, dtype)
    y = eng.forward(x)
    torch.save(y.cpu(), out)


def diff(a, b):
    ya, yb = torch.load(a, weights_only=True).float(), torch.load(b, weights_only=True).float()
    d = (ya - yb).abs()
    neq = (ya != yb).sum().item()
    print(f"{a} vs {b}: {neq} of {ya.numel()} values differ, max |d| {d.max().item():.3g}")
    return neq


if __name__ == "__main__":
    if sys.argv[1] == "save":
        a = sys.argv[2:] + [None] * 5
        save(a[0], a[1] or "n", int(a[2] or 640), int(a[3] or 8), a[4] or "bf16")
    else:
        sys.exit(1 if diff(sys.argv[2], sys.argv[3]) else 0)
