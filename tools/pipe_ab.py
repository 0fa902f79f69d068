"""A/B of the bench schedule's host side (diagnostic, GPU): bench.py's timed region (20 steps
after 5 warm-up steps, synchronize on both sides) with yolo_hip.pipeline.DetectPipeline as
bench.py built it up to round 5 ("pipe": a `ready` marker on the caller's stream every step),
without the marker when the caller's stream is idle ("skip"), with its result ring ("ring": per-slot dets / counts and one NMS
workspace, no per-batch allocation or record_stream), both ("ringskip"), and a bare loop of the same launches
("raw"). Modes alternate; per run: img/s and the host time of the submit loop.

  python tools/pipe_ab.py [--steps 20] [--warmup 5] [--rounds 4] [--modes pipe,ring,raw]
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
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--lanes", type=int, default=3)
    ap.add_argument("--modes", default="pipe,ring,skip,ringskip,raw")
    a = ap.parse_args()
    import bench
    from yolo_hip import synth
    from yolo_hip.engine import Engine, nms
    from yolo_hip.pipeline import DetectPipeline

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
    y0 = torch.empty((B, 84, A), dtype=dtype, device=dev)
    for e in engs:
        e.forward(xs[0], out=y0)
        torch.cuda.synchronize()
    # only the modes asked for create streams (a process per mode keeps the stream -> hardware
    # queue mapping the same as bench.py's)
    opts = {"pipe": dict(idle_skip=False), "ring": dict(result_ring=True, idle_skip=False),
            "skip": dict(idle_skip=True), "ringskip": dict(result_ring=True, idle_skip=True)}
    modes = a.modes.split(",")
    pipes = {m: DetectPipeline(engs, B, S, S, **opts[m]) for m in modes if m in opts}
    if "raw" in modes:
        lanes = [torch.cuda.Stream(device=dev) for _ in engs]
        ns = torch.cuda.Stream(device=dev)
    ys = [torch.empty((B, 84, A), dtype=dtype, device=dev) for _ in range(2 * a.lanes)]
    free = [None] * len(ys)

    def raw_step(k):
        main = torch.cuda.current_stream(dev)
        lane, i = k % len(engs), k % len(ys)
        fs = lanes[lane]
        ready = torch.cuda.Event()
        ready.record(main)
        fs.wait_event(ready)
        if free[i] is not None:
            fs.wait_event(free[i])
        with torch.cuda.stream(fs):
            engs[lane].forward(xs[k % 4], out=ys[i])
            e1 = torch.cuda.Event()
            e1.record(fs)
        with torch.cuda.stream(ns):
            ns.wait_event(e1)
            out = nms(ys[i])
            e2 = torch.cuda.Event()
            e2.record(ns)
        free[i] = e2
        return out

    res = {m: [] for m in modes}
    for r in range(a.rounds):
        for mode in res:
            it = [0]

            def step():
                k = it[0]
                it[0] += 1
                if mode == "raw":
                    return raw_step(k)
                return pipes[mode].submit(xs[k % 4])[:3]

            for _ in range(a.warmup):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                last = step()
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            del last
            res[mode].append((B * a.steps / el, (t1 - t0) * 1e3))
            print(f"round {r} {mode:5s} {B * a.steps / el:8.0f} img/s  {el / a.steps * 1e3:.4f} ms/step  "
                  f"host submit {(t1 - t0) * 1e3:.2f} ms", flush=True)
    for mode, v in res.items():
        vals = sorted(x[0] for x in v)
        print(f"{mode:5s} median {vals[len(vals) // 2]:.0f} img/s  runs {[round(x) for x in vals]}")


if __name__ == "__main__":
    main()
