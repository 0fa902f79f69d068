"""head_cls phase stamps (YH_LIB=scratch/libs/libhctrace.so, built with -DYH_HC_TRACE)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "yolo-infer-pt_amd"))

from yolo_hip import synth  # noqa: E402
from yolo_hip.engine import Engine  # noqa: E402
from yolo_hip import _lib  # noqa: E402


def main():
    v = sys.argv[1] if len(sys.argv) > 1 else "n"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    from nets import nn
    torch.manual_seed(0)
    model = getattr(nn, f"yolo_v11_{v}")(80)
    model.load_state_dict(synth.synth_state_dict(model.state_dict(), seed=0))
    model.eval()
    dev = torch.device("cuda", 0)
    eng = Engine(*model._yh_arch, dev, torch.bfloat16)
    eng.load_module(model)
    x = synth.synth_scenes(B, 640, 640, seed=3).to(dev, torch.bfloat16)
    y = eng.forward(x)
    for _ in range(3):
        eng.forward(x, out=y)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(os.environ["YH_LIB"])
    n = 8192 * 10
    buf = np.zeros(n, dtype=np.uint64)
    rc = lib.yh_debug_hc_trace(ctypes.c_void_p(buf.ctypes.data), ctypes.c_int(n))
    assert rc == 0, rc
    t = buf.reshape(8192, 10).astype(np.int64)
    used = t[:, 8] > 0
    t = t[used]
    print(f"workgroups traced: {len(t)}")
    rt0 = t[:, 0].min()
    span = (t[:, 8].max() - rt0) * 10e-3
    print(f"kernel span (s_memrealtime, 100 MHz): {span:.1f} us")
    life = (t[:, 8] - t[:, 0]) * 10e-3
    lv = (t[:, 9] >> 40) & 0xff
    names = ["land", "dw1", "pw1", "dw2", "pw2", "pw3"]
    for L in sorted(set(lv.tolist())):
        m = lv == L
        d = np.diff(t[m][:, 1:8], axis=1)   # cycles per phase
        tot = t[m][:, 7] - t[m][:, 1]
        print(f"level {L}: {m.sum()} wgs, life {np.median(life[m]):.2f} us median ({life[m].mean():.2f} mean), "
              f"cycles {np.median(tot):.0f} median; start {(t[m][:, 0].min() - rt0) * 1e-2:.1f}..{(t[m][:, 0].max() - rt0) * 1e-2:.1f} us")
        print("   phase  " + " ".join(f"{s:>7s}" for s in names))
        print("   median " + " ".join(f"{x:7.0f}" for x in np.median(d, axis=0)))
        print("   mean   " + " ".join(f"{x:7.0f}" for x in d.mean(axis=0)))
        print("   p90    " + " ".join(f"{x:7.0f}" for x in np.percentile(d, 90, axis=0)))
    # residency: workgroups alive over time, and per-CU counts
    ev = sorted([(a, 1) for a in t[:, 0]] + [(b, -1) for b in t[:, 8]])
    cur = 0
    mx = 0
    hist = []
    for tt, dlt in ev:
        cur += dlt
        mx = max(mx, cur)
        hist.append((tt, cur))
    hist = np.array(hist)
    print(f"max concurrent workgroups: {mx}")
    for q in (0.1, 0.25, 0.5, 0.75, 0.9):
        tq = rt0 + q * (t[:, 8].max() - rt0)
        i = np.searchsorted(hist[:, 0], tq)
        print(f"  at {q:.2f} of span: {hist[min(i, len(hist) - 1), 1]} alive")
    hw = t[:, 9] & 0xffffffff
    cu = (hw >> 8) & 0xf
    se = (hw >> 13) & 0x7
    sh = (hw >> 12) & 1
    xcc = (t[:, 9] >> 32) & 0xff
    key = xcc * 1000 + se * 100 + sh * 20 + cu
    ks, cnt = np.unique(key, return_counts=True)
    print(f"distinct CUs: {len(ks)}, workgroups per CU min/median/max {cnt.min()}/{np.median(cnt):.0f}/{cnt.max()}")
    # clock: cycles per us from memtime vs realtime
    cyc = (t[:, 7] - t[:, 1]).astype(np.float64)
    us = (t[:, 8] - t[:, 0]) * 1e-2
    ok = us > 1
    print(f"shader clock estimate: {np.median(cyc[ok] / us[ok]):.0f} cycles/us")


if __name__ == "__main__":
    main()
