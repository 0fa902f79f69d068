"""One line per op from tools/pmc_sq_dump.py's output (the SQ breakdowns DESIGN.md quotes).

SQ_WAVE_CYCLES / SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY count quad-cycles (4 clk);
SQ_VALU_MFMA_BUSY_CYCLES counts clk. wait% = SQ_WAIT_ANY (parked at s_waitcnt / s_barrier),
winst% = SQ_WAIT_INST_ANY (issue stalls), act% = SQ_ACTIVE_INST_ANY, each over SQ_WAVE_CYCLES;
mfma/w = MFMA busy clk per wave, mfma% = that over the wave's clk (times the waves a SIMD holds for the
SIMD's share); ldsconf% = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.

  python tools/sq_table.py <sq_dump.txt>
"""
import re
import sys


def main():
    ops, cur = [], None
    for line in open(sys.argv[1]):
        m = re.match(r"^(\S.*?) \[(.*)\] ([\d.]+) us \(last pass\)", line)
        if m:
            cur = dict(name=m.group(1), kernel=m.group(2), us=float(m.group(3)), c={})
            ops.append(cur)
            continue
        m = re.match(r"^\s+(SQ_\w+)\s+([\d.]+)", line)
        if m and cur is not None:
            cur["c"][m.group(1)] = float(m.group(2))
    print(f"{'op':34s} {'us':>6s} {'waves':>6s} {'clk/w':>8s} {'wait%':>6s} {'winst%':>6s} {'act%':>5s} "
          f"{'mfma/w':>7s} {'mfma%':>6s} {'valu/w':>7s} {'lds/w':>6s} {'ldsconf%':>8s}  kernel")
    for o in ops:
        c = o["c"]
        w = c.get("SQ_WAVES", 0.0)
        cyc = c.get("SQ_WAVE_CYCLES", 0.0)
        if not w or not cyc:
            continue
        clk = 4 * cyc / w
        pct = lambda k: 100.0 * c.get(k, 0.0) / cyc
        mf = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / w
        lds_act = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        conf = 100.0 * c.get("SQ_LDS_BANK_CONFLICT", 0.0) / lds_act if lds_act else 0.0
        print(f"{o['name'][:34]:34s} {o['us']:6.1f} {w:6.0f} {clk:8.0f} {pct('SQ_WAIT_ANY'):6.1f} "
              f"{pct('SQ_WAIT_INST_ANY'):6.1f} {pct('SQ_ACTIVE_INST_ANY'):5.1f} {mf:7.0f} {100 * mf / clk:6.1f} "
              f"{c.get('SQ_INSTS_VALU', 0.0) / w:7.0f} {c.get('SQ_INSTS_LDS', 0.0) / w:6.0f} {conf:8.1f}  {o['kernel']}")


if __name__ == "__main__":
    main()
