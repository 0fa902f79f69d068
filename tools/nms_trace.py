"""Phase timing of the NMS kernels on a real v11_n bf16 head output (debug hook yh_debug_nms_trace).

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
    B = 32
    torch.manual_seed(0)
    model = nn.yolo_v11_n(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, torch.bfloat16)
    eng.load_module(model)
    x = synth.synth_scenes(B, 640, 640, seed=100).to(dev, torch.bfloat16)
    y = eng.forward(x)
    for _ in range(3):
        nms(y)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        nms(y)
    e1.record()
    torch.cuda.synchronize()
    print(f"nms (emit + image) per batch of {B}: {e0.elapsed_time(e1) / 20 * 1e3:.1f} us (HIP events, back to back)")
    tr = torch.zeros((B, 16), dtype=torch.int64, device=dev)
    lib().yh_debug_nms_trace(ctypes.c_void_p(tr.data_ptr()))
    nms(y)
    torch.cuda.synchronize()
    lib().yh_debug_nms_trace(None)
    t = tr.cpu()
    ph = ["hist-scan", "select+gather", "sort", "greedy(batch0)", "rest", "end"]
    d = (t[:, 1:7] - t[:, 0:6]).double() * 10.0  # 100 MHz ticks -> ns
    print("per-image phase us (mean / max):")
    for i, name in enumerate(ph):
        print(f"  {name:16s} {d[:, i].mean().item() / 1e3:8.2f} {d[:, i].max().item() / 1e3:8.2f}")
    total = (t[:, 6] - t[:, 0]).double() * 10.0 / 1e3
    print(f"  total            {total.mean().item():8.2f} {total.max().item():8.2f}")
    sb = (t[:, 12:16] - torch.cat((t[:, 3:4], t[:, 12:15]), 1)).double() * 10.0
    for i, name in enumerate(["sb0 decode", "sb0 kept+pairwise", "sb0 resolve", "sb0 outputs"]):
        print(f"  {name:16s} {sb[:, i].mean().item() / 1e3:8.2f} {sb[:, i].max().item() / 1e3:8.2f}")
    print("batches", t[:, 8].tolist()[:8], "processed", t[:, 9].tolist()[:8], "cands", t[:, 11].tolist()[:8])
    ghz = (t[:, 10] - t[:, 7]).double() / ((t[:, 6] - t[:, 0]).double() * 10.0)
    print(f"shader clock during nms_image: {ghz.mean().item():.3f} GHz (s_memtime / s_memrealtime)")
    start = t[:, 0].min()
    print("block start spread us", ((t[:, 0] - start).double() * 10 / 1e3).max().item())


if __name__ == "__main__":
    main()
