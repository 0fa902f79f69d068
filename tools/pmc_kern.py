"""SQ counters per kernel of the last eager forward of tools/pmc_run.py.

  python tools/pmc_kern.py <pmc_dir> [regex ...]

Prints, for the last dispatch of each kernel whose name matches a regex (default:
the fused kernels), every counter of the pass, plus the derived shares of
SQ_WAVE_CYCLES when the pass holds the wait / active counters.
"""
import csv
import glob
import os
import re
import sys


def main():
    d = sys.argv[1]
    pats = [re.compile(p) for p in (sys.argv[2:] or ["head_cls", "csp_fused", "box_dfl", "conv_first", "stem_fused", "psa_attention"])]
    rows = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                did = int(r["Dispatch_Id"])
                rec = rows.setdefault(did, dict(name=r["Kernel_Name"], c={}))
                rec["c"][r["Counter_Name"]] = rec["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    last = {}
    for did in sorted(rows):
        for p in pats:
            if p.search(rows[did]["name"]):
                last[(p.pattern, rows[did]["name"][:80])] = rows[did]["c"]
    for (p, name), c in last.items():
        print(name)
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        for k in sorted(c):
            share = f"  ({100 * c[k] / wc:5.1f} % of wave cycles)" if wc and k.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
            print(f"   {k:28s} {c[k]:16.0f}{share}")


if __name__ == "__main__":
    main()
