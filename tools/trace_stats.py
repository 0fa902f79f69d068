"""Kernel statistics of the timed region of a `rocprofv3 --kernel-trace` run of bench.py.

python tools/trace_stats.py TRACE_DIR [steps]

bench.py launches a marker fill kernel right after its timed steps (and none before them: see
bench.py); the timed steps are the dispatches from the `steps`-th last forward's first
dispatch (set_io) before that marker up to the marker (the tuner's trial launches, the
warm-up steps and the roofline's eager forwards are excluded). Prints per kernel name: calls, calls per step, total and
average duration, and the busy time of the whole region (union of kernel intervals).
"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    rows = []
    for fn in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    marks = [i for i, r in enumerate(rows) if "fill" in r[2].lower()]
    # the end marker is torch.zeros(1) + fill_(8): the first fill dispatch of its cluster
    clusters = []
    for i in marks:
        if clusters and i == clusters[-1][-1] + 1:
            clusters[-1].append(i)
        else:
            clusters.append([i])
    if not clusters:
        raise SystemExit("end marker not found")
    b = clusters[-1][0]
    # every forward starts with one set_io dispatch: the region starts at the `steps`-th last
    # set_io before b (the earlier ones are the warm-up steps')
    sio = [i for i in range(b) if "set_io" in rows[i][2]]
    if len(sio) < steps:
        raise SystemExit(f"only {len(sio)} forwards before the end marker")
    a = sio[-steps]
    region = rows[a:b]
    t0, t1 = rows[a][0], rows[b][0]
    stats = {}
    for s, e, n in region:
        k = n.split("(")[0][:90]
        c = stats.setdefault(k, [0, 0])
        c[0] += 1
        c[1] += e - s
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in region:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    print(f"timed region: {(t1 - t0) / 1e6:.3f} ms for {steps} steps ({(t1 - t0) / 1e3 / steps:.1f} us/step), "
          f"{len(region)} dispatches, GPU busy {busy / 1e6:.3f} ms ({100.0 * busy / max(1, t1 - t0):.1f} %)")
    print(f"{'calls':>7} {'/step':>6} {'total ms':>9} {'avg us':>8}  kernel")
    for k, (c, t) in sorted(stats.items(), key=lambda kv: -kv[1][1]):
        print(f"{c:7d} {c / steps:6.2f} {t / 1e6:9.3f} {t / c / 1e3:8.2f}  {k}")


if __name__ == "__main__":
    main()
