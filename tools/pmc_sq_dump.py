"""Every counter of one or more rocprofv3 --pmc passes of tools/pmc_run.py, per op of the given
classes (default conv3x3): raw totals, and per wave (counter / SQ_WAVES) where the pass has
SQ_WAVES. For the SQ breakdowns DESIGN.md quotes (wave cycles parked at s_waitcnt / barriers,
LDS instructions and their issue stalls, vector-memory instructions, MFMA busy).

  python tools/pmc_sq_dump.py <ops.json> <pmc_dir> [<pmc_dir> ...] [--cls=conv3x3,c3k2]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_sq_ops import dispatches, per_op  # noqa: E402
import json  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cls = {"conv3x3"}
    for a in sys.argv[1:]:
        if a.startswith("--cls="):
            cls = set(a.split("=", 1)[1].split(","))
    opsf, dirs = args[0], args[1:]
    ops = json.load(open(opsf))["ops"]
    tables = [per_op(dispatches(d), ops) for d in dirs]
    for i, o in enumerate(ops):
        if o["cls"] not in cls:
            continue
        c = {}
        us = None
        for groups in tables:   # a counter repeated in several passes (SQ_WAVES) is taken once
            cp = {}
            for r in groups[i]:
                for k, v in r["c"].items():
                    cp[k] = cp.get(k, 0.0) + v
            for k, v in cp.items():
                c.setdefault(k, v)
            us = sum((r["t1"] - r["t0"]) for r in groups[i]) / 1e3
        waves = c.get("SQ_WAVES", 0.0)
        print(f"{o['label']} [{o.get('kernel') or o['cls']}] {us:.1f} us (last pass)")
        for k in sorted(c):
            per = f"  per wave {c[k] / waves:12.1f}" if waves else ""
            print(f"    {k:32s} {c[k]:16.0f}{per}")


if __name__ == "__main__":
    main()
