"""Every dispatch of the last eager forward from a rocprofv3 --pmc pass over
tools/pmc_run.py, with all counters of the pass (SQ units).

  python tools/pmc_all.py <pmc_dir> <n_last>
"""
import csv
import glob
import os
import sys


def main():
    d, n = sys.argv[1], int(sys.argv[2])
    rows = {}
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for r in csv.DictReader(f):
                did = int(r["Dispatch_Id"])
                rec = rows.setdefault(did, dict(name=r["Kernel_Name"], c={}))
                rec["c"][r["Counter_Name"]] = rec["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    last = [rows[k] for k in sorted(rows)][-n:]
    names = sorted({k for r in last for k in r["c"]})
    print("kernel".ljust(48) + "".join(x[-14:].rjust(16) for x in names))
    for r in last:
        print(r["name"][:47].ljust(48) + "".join(f"{r['c'].get(x, 0):16.0f}" for x in names))


if __name__ == "__main__":
    main()
