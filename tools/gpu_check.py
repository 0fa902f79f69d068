"""Developer smoke check on a GPU box: HIP forward vs the CPU module forward.

python tools/gpu_check.py [variant] [size] [batch]
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))

from nets import nn  # noqa: E402
from yolo_hip import synth  # noqa: E402
from yolo_hip.engine import Engine, nms  # noqa: E402


def main():
    v = sys.argv[1] if len(sys.argv) > 1 else "n"
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 320
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval().fuse()
    x = synth.synth_scenes(B, size, size, seed=5)
    with torch.no_grad():
        ref = model(x)
    print("cpu ref", tuple(ref.shape), float(ref[:, :4].abs().max()), flush=True)
    dev = torch.device("cuda", 0)
    for dt in (torch.float32, torch.bfloat16, torch.float16):
        eng = Engine(*model._yh_arch, dev, dt)
        eng.load_module(model)
        xd = x.to(dev, dt)
        eng.set_graph(False)
        y = eng.forward(xd)
        torch.cuda.synchronize()
        yf = y.float().cpu()
        dbox = (yf[:, :4] - ref[:, :4]).abs().max().item()
        dcls = (yf[:, 4:] - ref[:, 4:]).abs().max().item()
        print(f"{dt}: box max|d| {dbox:.3e}  cls max|d| {dcls:.3e}", flush=True)
        eng.set_graph(True)
        y2 = eng.forward(xd)
        torch.cuda.synchronize()
        print(f"   graph vs eager identical: {torch.equal(y, y2)}", flush=True)
        t0 = time.time()
        for _ in range(10):
            eng.forward(xd, out=y2)
        torch.cuda.synchronize()
        print(f"   {(time.time() - t0) / 10 * 1e3:.3f} ms/forward (B={B}, {size}^2)", flush=True)
        dets, counts = nms(y)
        torch.cuda.synchronize()
        print(f"   nms counts {counts.tolist()}", flush=True)


if __name__ == "__main__":
    main()
