"""Phase timing of the NMS kernels on a real v11_n bf16 head output (debug hook yh_debug_nms_trace).

  python tools/nms_trace.py [variant size batch dtype [scene seed]]

Needs the diagnostic build of the library: make EXTRA=-DYH_ABLATION OUT=exp_lib/libyolo_hip.so
OBJDIR=build/abl, then run with YH_LIB=exp_lib/libyolo_hip.so."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))

from yolo_hip import synth  # noqa: E402
from yolo_hip._lib import lib  # noqa: E402
from yolo_hip.engine import Engine, nms  # noqa: E402


def main():
    from nets import nn
    v = sys.argv[1] if len(sys.argv) > 1 else "n"
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 640
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    dt = {"bf16": torch.bfloat16, "fp16": torch.float16}[sys.argv[4] if len(sys.argv) > 4 else "bf16"]
    seed = int(sys.argv[5]) if len(sys.argv) > 5 else 100
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, dt)
    eng.load_module(model)
    x = synth.synth_scenes(B, S, S, seed=seed).to(dev, dt)
    y = eng.forward(x)
    if os.environ.get("YH_NMS_Y"):   # a head output saved by the shipped library (torch.save)
        y = torch.load(os.environ["YH_NMS_Y"], weights_only=True).to(dev)
    for _ in range(3):
        nms(y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        nms(y)
    e1.record()
    torch.cuda.synchronize()
    print(f"nms (zero + emit + gather + prep + mask + finish) per batch of {B}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us (HIP events, back to back)")
    tr = torch.zeros((B, 16), dtype=torch.int64, device=dev)
    lib().yh_debug_nms_trace(ctypes.c_void_p(tr.data_ptr()))
    nms(y)
    torch.cuda.synchronize()
    lib().yh_debug_nms_trace(None)
    t = tr.cpu()
    # marks: 0-3 nms_prep (start, start, gathered keys loaded, sorted + decoded), 4-6 nms_finish
    # (start, first batch resolved, end); 3 -> 4 is nms_mask plus the launch gaps
    ph = ["-", "load batch", "sort+decode", "mask(+gaps)", "resolve", "outputs+rest"]
    d = (t[:, 1:7] - t[:, 0:6]).double() * 10.0  # 100 MHz ticks -> ns
    print("per-image phase us (mean / max):")
    for i, name in enumerate(ph):
        print(f"  {name:16s} {d[:, i].mean().item() / 1e3:8.2f} {d[:, i].max().item() / 1e3:8.2f}")
    total = (t[:, 6] - t[:, 0]).double() * 10.0 / 1e3
    print(f"  total            {total.mean().item():8.2f} {total.max().item():8.2f}")
    k = int((t[:, 6] - t[:, 0]).argmax())
    if t[k, 8] > 0:   # the slowest image continued past the first batch: nms_rest's summed parts
        r = [int(v) for v in t[k].tolist()]
        lo40 = (1 << 40) - 1
        print(f"image {k} continuation: {r[9] >> 40} later batches, {r[15] >> 40} sub-batches; us: "
              f"select/scan {(r[9] & lo40) / 100:.1f} sort {r[11] / 100:.1f} | sub-batches: decode {r[12] / 100:.1f} "
              f"kept+pairwise {r[13] / 100:.1f} resolve {r[14] / 100:.1f} out {(r[15] & lo40) / 100:.1f} | "
              f"finish total {(r[6] - r[4]) / 100:.1f}")
    print("kernel spans us: prep", ((t[:, 3] - t[:, 0]).max().item() * 10 / 1e3),
          "finish", ((t[:, 6] - t[:, 4]).max().item() * 10 / 1e3),
          "prep end -> finish start", ((t[:, 4].min() - t[:, 3].max()).item() * 10 / 1e3))
    start = t[:, 0].min()
    print("block start spread us", ((t[:, 0] - start).double() * 10 / 1e3).max().item())


if __name__ == "__main__":
    main()
