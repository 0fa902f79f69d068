"""Per-conv-op SQ counters from a rocprofv3 --pmc pass over tools/pmc_run.py.

  python tools/pmc_sq.py <pmc_dir> <ops.json> [label ...]

Maps the last forward's conv dispatches onto the engine's conv ops (one
dispatch per conv op, in op order) and prints every counter of the pass per op.
"""
import csv
import glob
import json
import os
import re
import sys

CONV_RE = re.compile(r"conv_(direct|gemm2|gemm|stream|patch)(<|I)")


def main():
    d, ops_json = sys.argv[1:3]
    want = set(sys.argv[3:])
    ops = [o for o in json.load(open(ops_json)) if o["cls"] in ("conv3x3", "conv1x1")]
    rows = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                did = int(r["Dispatch_Id"])
                rec = rows.setdefault(did, dict(name=r["Kernel_Name"], c={}))
                rec["c"][r["Counter_Name"]] = rec["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    conv = [rows[k] for k in sorted(rows) if CONV_RE.search(rows[k]["name"])][-len(ops):]
    names = sorted({k for r in conv for k in r["c"]})
    print("label".ljust(34) + "".join(n[-14:].rjust(16) for n in names))
    for o, r in zip(ops, conv):
        if want and o["label"] not in want:
            continue
        print(o["label"][:33].ljust(34) + "".join(f"{r['c'].get(n, 0):16.0f}" for n in names) + "  " + r["name"][:40])


if __name__ == "__main__":
    main()
