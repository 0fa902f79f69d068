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
    units = eng.units(B, size, size)
    tot = sum(u["ms"] / max(1, u["calls"]) for u in units)
    print(f"v11_{v} {size}^2 B={B} {dt}: forward kernels {tot * 1e3:.1f} us in {len(units)} launch units")
    if os.environ.get("YH_PROF_OUT"):
        import json
        with open(os.environ["YH_PROF_OUT"], "w") as f:
            json.dump({"nms_us": e0.elapsed_time(e1) / steps * 1e3, "fwd_us": tot * 1e3,
                       "ops": [dict(label=u["label"], cls=u["cls"], us=u["ms"] / max(1, u["calls"]) * 1e3,
                                    bytes=u["bytes"], flops=u["flops"], kernel=u["kernel"]) for u in units]}, f)
    rows = sorted(units, key=lambda u: -u["ms"] / max(1, u["calls"]))
    for u in rows:
        ms = u["ms"] / max(1, u["calls"])
        print(f"{ms * 1e3:8.1f} us {100 * ms / tot:5.1f}%  {u['bytes'] / ms / 1e6:7.0f} GB/s "
              f"{u['flops'] / ms / 1e9:7.1f} TF/s  {u['bytes'] / 1e6:8.1f} MB  {u['cls']:9s} {u['kernel'] or '':9s} {u['label']}")


if __name__ == "__main__":
    main()
