"""Run one level-program case (fused vs unfused compare) with diagnostics.
python tools/level_case.py variant dtype batch h w"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))
from yolo_hip import synth  # noqa: E402
from yolo_hip.engine import Engine  # noqa: E402


def main():
    v, dt, B, h, w = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
    dtype = {"bf16": torch.bfloat16, "fp16": torch.float16}[dt]
    from nets import nn
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, dtype)
    eng.load_module(model)
    x = synth.synth_scenes(B, h, w, seed=21).to(dev, dtype)
    eng.set_level_fusion(False)
    ref = eng.forward(x).clone()
    torch.cuda.synchronize()
    print("unfused ok", flush=True)
    eng.set_level_fusion(True)
    eng.set_graph(False)
    got = eng.forward(x).clone()
    torch.cuda.synchronize()
    print("fused ok; status", flush=True)
    eng.level_status()
    d = (got.float() - ref.float()).abs()
    print("max diff", d.max().item(), "n diff", int((d > 0).sum()))


if __name__ == "__main__":
    main()
