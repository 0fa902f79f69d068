"""Workload for rocprofv3 --pmc passes: eager (non-graph) forwards of the bench
configuration, so every kernel is its own dispatch record.

  rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run -f csv -- python3 tools/pmc_run.py
  python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/ops.json

Writes the op list (label, class, algorithmic bytes) of the profiled shape to
$YH_OPS_OUT so tools/pmc_traffic.py can map the dispatches after the marker (one
eager forward) to ops.
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


def main():
    v = os.environ.get("YH_VARIANT", "n")
    size = int(os.environ.get("YH_SIZE", "640"))
    B = int(os.environ.get("YH_BATCH", "32"))
    dname = os.environ.get("YH_DTYPE", "bf16")
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[dname]
    from nets import nn
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, dt)
    eng.load_module(model)
    x = synth.synth_scenes(B, size, size, seed=100).to(dev, dt)
    eng.forward(x)          # autotune (many candidate launches)
    eng.set_graph(False)
    y = eng.forward(x)
    eng.forward(x, out=y)
    torch.cuda.synchronize()
    torch.zeros(1, device=dev).fill_(7.0)   # marker dispatch: the measured forward follows it
    torch.cuda.synchronize()
    eng.forward(x, out=y)
    torch.cuda.synchronize()
    out = os.environ.get("YH_OPS_OUT")
    if out:
        with open(out, "w") as f:
            json.dump(dict(config=dict(variant=v, size=size, batch=B, dtype=dname),
                           ops=[dict(label=o["label"], cls=o["cls"], bytes=o["bytes"], kernel=o["kernel"])
                                for o in (u["ops"][0] for u in eng.units(B, size, size))]), f)
    print("pmc workload done", flush=True)


if __name__ == "__main__":
    main()
