"""Per-batch timeline of bench.py's pipelined steps (diagnostic, GPU).

Runs the bench's default schedule (three forward lanes + one NMS stream, yolo_hip.pipeline)
for --steps steps after a synchronize, exactly as bench.py's timed region, and records HIP
events on each lane stream around every forward and on the NMS stream after every NMS. Prints
per batch: lane, forward start / end and NMS end relative to the region start (us), and the
region's total, so the fill (lanes starting in phase) and the drain (the last forwards running
with fewer partners) can be read off.

  python tools/lane_timeline.py [--steps 20] [--warmup 5] [--lanes 3]
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "yolo-infer-pt_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--lanes", type=int, default=3)
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    import bench
    from yolo_hip import synth
    from yolo_hip.engine import Engine, nms

    dev = torch.device("cuda", 0)
    dtype = torch.bfloat16
    model = bench.build_model("n")
    B, S = 32, 640
    engs = []
    for _ in range(a.lanes):
        e = Engine(*model._yh_arch, dev, dtype)
        e.load_module(model)
        e.reserve(B, S, S)
        engs.append(e)
    xs = [synth.synth_scenes(B, S, S, seed=100 + 1000 * k).to(dev, dtype) for k in range(4)]
    A = engs[0].num_anchors(S, S)
    ys = [torch.empty((B, 84, A), dtype=dtype, device=dev) for _ in range(2 * a.lanes)]
    for e in engs:
        e.forward(xs[0], out=ys[0])
        torch.cuda.synchronize()
    lanes = [torch.cuda.Stream(device=dev) for _ in engs]
    ns = torch.cuda.Stream(device=dev)
    free = [None] * len(ys)

    def run(n, rec):
        main = torch.cuda.current_stream(dev)
        evs = []
        for k in range(n):
            lane, i = k % len(engs), k % len(ys)
            fs = lanes[lane]
            ready = torch.cuda.Event()
            ready.record(main)
            fs.wait_event(ready)
            if free[i] is not None:
                fs.wait_event(free[i])
            e0, e1, e2 = (torch.cuda.Event(enable_timing=rec) for _ in range(3))
            with torch.cuda.stream(fs):
                e0.record(fs)
                engs[lane].forward(xs[k % 4], out=ys[i])
                e1.record(fs)
            with torch.cuda.stream(ns):
                ns.wait_event(e1)
                nms(ys[i])
                e2.record(ns)
            free[i] = e2
            evs.append((lane, e0, e1, e2))
        return evs

    for r in range(a.repeat):
        run(a.warmup, False)
        torch.cuda.synchronize()
        t_start = torch.cuda.Event(enable_timing=True)
        t_start.record()
        t0 = time.perf_counter()
        evs = run(a.steps, True)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        print(f"repeat {r}: {a.steps} steps, wall {wall * 1e3:.3f} ms, {B * a.steps / wall:.0f} img/s")
        print("  batch lane   fwd_start   fwd_end   fwd_len   nms_end")
        for k, (lane, e0, e1, e2) in enumerate(evs):
            s0, s1, s2 = (t_start.elapsed_time(e) * 1e3 for e in (e0, e1, e2))
            print(f"  {k:5d} {lane:4d} {s0:10.1f} {s1:9.1f} {s1 - s0:9.1f} {s2:9.1f}")


if __name__ == "__main__":
    main()
