"""Compare per-op JSON dumps of tools/op_profile.py (YH_PROF_OUT)."""
import json
import sys

names = sys.argv[2:]
d = {n: json.load(open(f"{sys.argv[1]}/{n}.json")) for n in names}
for n in names:
    by = {}
    for o in d[n]["ops"]:
        by[o["cls"]] = by.get(o["cls"], 0) + o["us"]
    print(f"{n:8s} fwd {d[n]['fwd_us']:7.1f} nms {d[n]['nms_us']:6.1f}", {k: round(v, 1) for k, v in sorted(by.items())})
rows = []
for i, o in enumerate(d[names[0]]["ops"]):
    if o["cls"] not in ("conv1x1", "conv3x3"):
        continue
    ts = {n: round(d[n]["ops"][i]["us"], 1) for n in names}
    rows.append((max(ts.values()), o["label"], o["cls"], o["bytes"] / 1e6, ts))
for r in sorted(rows, reverse=True)[:int(40)]:
    best = min(r[4].values())
    print(f"{r[1]:32s} {r[2]} {r[3]:6.1f}MB {r[3] * 1e3 / best:6.0f}GB/s", r[4])
