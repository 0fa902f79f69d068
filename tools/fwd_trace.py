"""Workload for `rocprofv3 --kernel-trace`: serial graph-replayed forwards of the bench
configuration (one forward at a time, nothing overlapping), so every dispatch record
is one kernel of the real forward with its in-network inputs (tools/trace_ops.py
maps them to ops).

  rocprofv3 --kernel-trace -f csv -d gpurun_out/ft -o run -- python3 tools/fwd_trace.py
  python tools/trace_ops.py gpurun_out/ft

Env: YH_VARIANT (n), YH_SIZE (640), YH_BATCH (32), YH_DTYPE (bf16), YH_FWD (5 forwards).
Writes the op list to $YH_OPS_OUT (default gpurun_out/ft_ops.json).
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))

from yolo_hip import synth  # noqa: E402
from yolo_hip.engine import Engine  # noqa: E402

DT = {"bf16": torch.bfloat16, "fp16": torch.float16, "fp32": torch.float32}


def main():
    v = os.environ.get("YH_VARIANT", "n")
    size = int(os.environ.get("YH_SIZE", "640"))
    B = int(os.environ.get("YH_BATCH", "32"))
    dt = DT[os.environ.get("YH_DTYPE", "bf16")]
    nf = int(os.environ.get("YH_FWD", "5"))
    from nets import nn
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, dt)
    eng.load_module(model)
    x = synth.synth_scenes(B, size, size, seed=100).to(dev, dt)
    y = eng.forward(x)          # autotune + graph capture
    for _ in range(3):
        eng.forward(x, out=y)
    torch.cuda.synchronize()
    torch.zeros(1, device=dev).fill_(7.0)   # marker dispatch: the traced forwards follow it
    torch.cuda.synchronize()
    for _ in range(nf):
        eng.forward(x, out=y)
        torch.cuda.synchronize()
    out = os.environ.get("YH_OPS_OUT", os.path.join(ROOT, "gpurun_out", "ft_ops.json"))
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(dict(forwards=nf, ops=[dict(label=o["label"], cls=o["cls"], bytes=o["bytes"], flops=o["flops"],
                                              kernel=o["kernel"]) for o in (u["ops"][0] for u in eng.units(B, size, size))]), f)
    print("fwd_trace done", flush=True)


if __name__ == "__main__":
    main()
