"""Back-to-back on-device NMS of one batch of synthetic scenes (default v11_n bf16 640x640, 32
images), for rocprofv3 --kernel-trace --stats (per-kernel durations of nms_zero/emit/gather/prep/
mask/finish).

  python tools/nms_bench.py [variant size batch dtype]     e.g. x 1280 16 bf16 (C5)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))

from yolo_hip import synth  # noqa: E402
from yolo_hip.engine import Engine, nms  # noqa: E402


def main():
    from nets import nn
    v = sys.argv[1] if len(sys.argv) > 1 else "n"
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 640
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[sys.argv[4] if len(sys.argv) > 4 else "bf16"]
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    eng = Engine(*model._yh_arch, dev, dt)
    eng.load_module(model)
    ys = [eng.forward(synth.synth_scenes(B, S, S, seed=300 + i).to(dev, dt)).clone() for i in range(2)]
    for _ in range(3):
        nms(ys[0])
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(30):
        nms(ys[i % 2])
    e1.record()
    torch.cuda.synchronize()
    print(f"nms per batch of {B}: {e0.elapsed_time(e1) / 30 * 1e3:.1f} us (HIP events, back to back)")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        nms(ys[0])
        with torch.cuda.graph(g, stream=s):
            nms(ys[0])
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(30):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"nms per batch of {B}: {e0.elapsed_time(e1) / 30 * 1e3:.1f} us (one captured graph, replayed back to back)")


if __name__ == "__main__":
    main()
