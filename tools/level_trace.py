"""Per-op timeline of the level programs (block 0's barrier arrival / departure,
s_memrealtime at 100 MHz): python tools/level_trace.py [variant] [size] [batch]."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))

from yolo_hip import synth  # noqa: E402
from yolo_hip._lib import lib  # noqa: E402
from yolo_hip.engine import Engine  # noqa: E402


def main():
    v = sys.argv[1] if len(sys.argv) > 1 else "n"
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 640
    B = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    from nets import nn
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, torch.bfloat16)
    eng.load_module(model)
    x = synth.synth_scenes(B, size, size, seed=3).to(dev, torch.bfloat16)
    y = eng.forward(x)
    buf = torch.zeros(16384, dtype=torch.int64, device=dev)
    L = lib()
    L.yh_debug_level_trace.argtypes = [ctypes.c_void_p]
    L.yh_debug_level_op_label.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                          ctypes.POINTER(ctypes.c_char_p)]
    L.yh_debug_level_trace(ctypes.c_void_p(buf.data_ptr()))
    eng.set_graph(False)
    for _ in range(3):
        eng.forward(x, out=y)
    torch.cuda.synchronize()
    L.yh_debug_level_trace(None)
    t = buf.cpu().tolist()
    k = 0
    tot = 0.0
    print("op  label                                     start->koff  koff->patch+w0  kloop  store  barrier   (us)")
    while True:
        lab = ctypes.c_char_p()
        if L.yh_debug_level_op_label(eng._h, B, size, size, k, ctypes.byref(lab)) != 0:
            break
        r = t[8 * k:8 * k + 8]
        d = lambda a, b: (r[b] - r[a]) / 100.0 if r[a] and r[b] else float("nan")
        seg = [d(1, 2), d(2, 3), d(3, 4), d(4, 5), d(5, 6)]
        tot += d(1, 6)
        print(f"{k:3d} {lab.value.decode():40s} " + " ".join(f"{x:7.2f}" for x in seg) + f"   total {d(1, 6):7.2f}")
        k += 1
    print(f"sum {tot:.1f} us")


if __name__ == "__main__":
    main()
