"""Any rocprofv3 --pmc counters per op (one eager forward of tools/pmc_run.py),
with the dispatch -> op mapping of tools/pmc_traffic.py.

  python tools/pmc_ops.py <pmc_dir> <ops.json> [label-regex]

Prints one row per op: every counter of the pass and, when the pass holds
SQ_WAVE_CYCLES, the wait / active counters as shares of it; with
SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE, MFMA busy per SIMD-cycle.
"""
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import per_op  # noqa: E402


def counters(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = {}
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                did = int(r["Dispatch_Id"])
                rec = rows.setdefault(did, dict(name=r["Kernel_Name"], c={}))
                rec["c"][r["Counter_Name"]] = rec["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = [rows[k] for k in sorted(rows)]
    mk = max(i for i, r in enumerate(out) if "fill" in r["name"].lower())
    return [r for r in out[mk + 1:] if "set_io" not in r["name"]]


def main():
    d, opsf = sys.argv[1:3]
    pat = re.compile(sys.argv[3]) if len(sys.argv) > 3 else None
    ops = json.load(open(opsf))["ops"]
    disp = counters(d)
    names = sorted({k for r in disp for k in r["c"]})
    cols = {}
    for n in names:
        cols[n] = per_op([dict(name=r["name"], value=r["c"].get(n, 0.0)) for r in disp], ops)
    hdr = "op".ljust(34) + "".join(f"{n.replace('SQ_', '')[:14]:>15s}" for n in names)
    print(hdr)
    for i, o in enumerate(ops):
        if pat and not pat.search(o["label"]):
            continue
        wc = cols.get("SQ_WAVE_CYCLES", [0] * len(ops))[i]
        cells = []
        for n in names:
            v = cols[n][i]
            if wc and n.startswith(("SQ_WAIT", "SQ_ACTIVE")) and n != "SQ_WAVE_CYCLES":
                cells.append(f"{100 * v / wc:14.1f}%")
            else:
                cells.append(f"{v:15.0f}")
        print(o["label"][:33].ljust(34) + "".join(cells))


if __name__ == "__main__":
    main()
