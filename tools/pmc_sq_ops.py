"""Per-op SQ counters (MFMA busy, wave / wait cycles, LDS) from one rocprofv3 --pmc pass of
tools/pmc_run.py, mapped onto the engine's ops the way tools/pmc_traffic.py maps traffic.

  python tools/pmc_sq_ops.py <pmc_dir> <ops.json> [class ...]   (default: conv3x3 conv1x1)

MFMA utilisation of an op = SQ_VALU_MFMA_BUSY_CYCLES / (SIMDs x the op's duration in
cycles), the duration taken from the pass's own dispatch timestamps (one eager forward,
counters serialise the dispatches) at the measured shader clock (--mhz, default 2400), and,
as a duration-free figure, MFMA busy / (SQ_BUSY_CYCLES x SIMDs per SE-counter).
Also printed: SQ_VALU_MFMA_BUSY_CYCLES / 32 = 32x32x16 MFMA instructions (MI355X_MICROARCH.md:
"= 32 x N_mfma for 32x32x16 bf16").
"""
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import FAMILY  # noqa: E402


def dispatches(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    rows = {}
    for fn in files:
        with open(fn) as f:
            for r in csv.DictReader(f):
                did = int(r["Dispatch_Id"])
                rec = rows.setdefault(did, dict(name=r["Kernel_Name"], c={}, t0=int(r["Start_Timestamp"]),
                                                t1=int(r["End_Timestamp"])))
                rec["c"][r["Counter_Name"]] = rec["c"].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    out = [rows[k] for k in sorted(rows)]
    mk = max(i for i, r in enumerate(out) if "fill" in r["name"].lower())
    return [r for r in out[mk + 1:] if "set_io" not in r["name"]]


def per_op(disp, ops):
    res, j = [], 0
    for i, o in enumerate(ops):
        group = [disp[j]]
        j += 1
        pat = FAMILY.get(o["cls"])
        if o["cls"] not in ("conv1x1", "conv3x3"):
            while pat and j < len(disp) and re.search(pat, disp[j]["name"]) and \
                    (i + 1 >= len(ops) or ops[i + 1]["cls"] != o["cls"]):
                group.append(disp[j])
                j += 1
        res.append(group)
    if j != len(disp):
        raise SystemExit(f"mapped {j} of {len(disp)} dispatches")
    return res


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    mhz = 2400.0
    for a in sys.argv[1:]:
        if a.startswith("--mhz="):
            mhz = float(a.split("=", 1)[1])
    d, opsf = args[:2]
    classes = set(args[2:]) or {"conv3x3", "conv1x1"}
    meta = json.load(open(opsf))
    ops = meta["ops"]
    groups = per_op(dispatches(d), ops)
    simds = 256 * 4
    fam = {}
    print(f"{'op':36s} {'cls':9s} {'us':>7s} {'mfma':>9s} {'mfma_util':>9s} {'wait_any':>8s} {'wait_inst':>9s} {'active':>7s}")
    for o, g in zip(ops, groups):
        if o["cls"] not in classes:
            continue
        c = {}
        for r in g:
            for k, v in r["c"].items():
                c[k] = c.get(k, 0.0) + v
        us = sum((r["t1"] - r["t0"]) for r in g) / 1e3
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        util = busy / (simds * us * mhz) if us > 0 else 0.0
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        f = fam.setdefault(o["cls"], dict(launches=0, us=0.0, busy=0.0))
        f["launches"] += 1
        f["us"] += us
        f["busy"] += busy
        print(f"{o['label']:36s} {o['cls']:9s} {us:7.1f} {busy / 32:9.0f} {util:9.3f} {c.get('SQ_WAIT_ANY', 0) / wc:8.2f} "
              f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:9.2f} {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:7.2f}")
    for k, f in fam.items():
        print(f"family {k}: {f['launches']} launches, {f['us']:.1f} us, MFMA busy {f['busy'] / (simds * f['us'] * mhz):.3f} "
              f"of the SIMDs' cycles over the family's time")


if __name__ == "__main__":
    main()
