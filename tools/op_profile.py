"""Per-op kernel times (HIP events) of the forward, sorted by time.

python tools/op_profile.py [variant] [size] [batch] [dtype] [steps]
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
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 640
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}[sys.argv[4] if len(sys.argv) > 4 else "bf16"]
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 10
    from nets import nn
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, dt)
    eng.load_module(model)
    x = synth.synth_scenes(B, size, size, seed=3).to(dev, dt)
    for _ in range(3):
        y = eng.forward(x)
    eng.profile(True)
    eng.profile_reset()
    for _ in range(steps):
        eng.forward(x, out=y)
    eng.profile(False)
    from yolo_hip.engine import nms
    for _ in range(3):
        nms(y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        dets, counts = nms(y)
    e1.record()
    torch.cuda.synchronize()
    print(f"nms: {e0.elapsed_time(e1) / steps * 1e3:.1f} us per batch of {B} (kept {counts.tolist()[:4]})")
    ops = eng.ops(B, size, size)
    tot = sum(o["ms"] / o["calls"] for o in ops)
    print(f"v11_{v} {size}^2 B={B} {dt}: forward kernels {tot * 1e3:.1f} us")
    if os.environ.get("YH_PROF_OUT"):
        import json
        with open(os.environ["YH_PROF_OUT"], "w") as f:
            json.dump({"nms_us": e0.elapsed_time(e1) / steps * 1e3, "fwd_us": tot * 1e3,
                       "ops": [dict(label=o["label"], cls=o["cls"], us=o["ms"] / o["calls"] * 1e3,
                                    bytes=o["bytes"], flops=o["flops"], kernel=o["kernel"]) for o in ops]}, f)
    rows = sorted(ops, key=lambda o: -o["ms"] / o["calls"])
    for o in rows:
        ms = o["ms"] / o["calls"]
        print(f"{ms * 1e3:8.1f} us {100 * ms / tot:5.1f}%  {o['bytes'] / ms / 1e6:7.0f} GB/s "
              f"{o['flops'] / ms / 1e9:7.1f} TF/s  {o['bytes'] / 1e6:8.1f} MB  {o['cls']:9s} {o['kernel'] or '':9s} {o['label']}")


if __name__ == "__main__":
    main()
