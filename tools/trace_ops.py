"""Map a rocprofv3 kernel trace of tools/fwd_trace.py to the forward's ops.

python tools/trace_ops.py TRACE_DIR [OPS_JSON] [--json OUT]

Prints per-op kernel durations (median over the traced forwards), the per-class sums,
and the gaps between consecutive dispatches (launch bubbles inside the graph).
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

FAMILY = {  # dispatch-name patterns per op class (yolo_hip.engine.OP_CLASSES); convs take exactly one dispatch
    "stem": r"conv_first|stem_fused",
    "dwconv": r"dwconv",
    "sppf": r"sppf|maxpool",
    "attention": r"psa_attention|pe_add",
    "decode": r"head_decode",
    "head_cls": r"head_cls",
    "box_dfl": r"box_dfl",
    "c3k2": r"csp_fused",
    "c3k": r"c3k_fused",
    "box_chain": r"box_chain",
    "pw_chain": r"pw_chain",
}


def load_trace(d):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return rows


def main():
    d = sys.argv[1]
    ops_json = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else None
    ops_json = ops_json or os.path.join(os.path.dirname(d.rstrip("/")), "ft_ops.json")
    meta = json.load(open(ops_json))
    ops, nf = meta["ops"], meta["forwards"]
    rows = load_trace(d)
    mk = max(i for i, r in enumerate(rows) if "fill" in r[2].lower() or "Fill" in r[2])
    disp = [r for r in rows[mk + 1:] if "set_io" not in r[2]]
    per = len(disp) // nf
    times = [[] for _ in ops]
    names = [None] * len(ops)
    gaps = []
    for f in range(nf):
        seq = disp[f * per:(f + 1) * per]
        j = 0
        for i, o in enumerate(ops):
            if j >= len(seq):
                raise SystemExit(f"forward {f}: ran out of dispatches at op {i} {o['label']}")
            t0, t1 = seq[j][0], seq[j][1]
            names[i] = names[i] or seq[j][2].split("(")[0][:60]
            j += 1
            if o["cls"] not in ("conv1x1", "conv3x3"):
                pat = FAMILY.get(o["cls"])
                while pat and j < len(seq) and re.search(pat, seq[j][2]) and \
                        (i + 1 >= len(ops) or ops[i + 1]["cls"] != o["cls"]):
                    t1 = seq[j][1]
                    j += 1
            times[i].append((t1 - t0) / 1e3)
        gaps.append((seq[-1][1] - seq[0][0]) / 1e3 - sum(t[-1] for t in times))
    med = [statistics.median(t) for t in times]
    tot = sum(med)
    cls = {}
    for o, m in zip(ops, med):
        cls[o["cls"]] = cls.get(o["cls"], 0) + m
    print(f"{len(ops)} ops, {per} dispatches/forward, kernels {tot:.1f} us, "
          f"span-minus-kernels {statistics.median(gaps):.1f} us")
    print({k: round(v, 1) for k, v in sorted(cls.items())})
    for i in sorted(range(len(ops)), key=lambda i: -med[i]):
        o = ops[i]
        print(f"{med[i]:8.1f} us {o['bytes'] / med[i] / 1e3:7.0f} GB/s {o['flops'] / med[i] / 1e6:7.1f} TF/s "
              f"{o['bytes'] / 1e6:7.1f} MB  {o['cls']:8s} {o['label']:28s} {o['kernel'] or names[i]}")
    if "--json" in sys.argv:
        out = sys.argv[sys.argv.index("--json") + 1]
        with open(out, "w") as f:
            json.dump(dict(kernels_us=tot, classes=cls, ops=[dict(o, us=m) for o, m in zip(ops, med)]), f)


if __name__ == "__main__":
    main()
