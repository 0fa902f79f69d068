#!/bin/bash
# A/B of the in-tree library against exp_lib/base (YH_LIB) on one box: optional GPU tests
# ($TESTS, -k $KEXPR; a plain test failure does not stop the A/B, a crash / timeout does),
# per-op HIP-event profiles and benches of both, alternating.
set -o pipefail
O=gpurun_out/${1:-ab}; mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -k "${KEXPR:-not nothing_deselected}" -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
  rc=$?
  tail -3 $O/tests.log
  if [ $rc -ge 124 ]; then echo "TESTS_CRASH rc=$rc"; tail -30 $O/tests.log; exit 1; fi
fi
B=exp_lib/base/libyolo_hip.so
YH_LIB=$B timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > $O/op_base.txt 2>&1 || { echo OPB_FAIL; tail $O/op_base.txt; exit 1; }
timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > $O/op_new.txt 2>&1 || { echo OPN_FAIL; tail $O/op_new.txt; exit 1; }
for r in 1 2; do
  YH_LIB=$B timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_base$r.json 2>$O/b_base$r.err || { echo BB_FAIL; tail $O/b_base$r.err; exit 1; }
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_new$r.json 2>$O/b_new$r.err || { echo BN_FAIL; tail $O/b_new$r.err; exit 1; }
done
python - "$O" <<'PY'
import json, sys
O = sys.argv[1]
for n in ("base1", "new1", "base2", "new2"):
    r = json.load(open(f"{O}/b_{n}.json"))
    rf = r["roofline"]
    print(n, r["value"], "img/s", "3x3 frac", rf["frac"], "fwd_kernel_ms", rf["forward_kernel_ms"],
          {k: v["us"] for k, v in rf["per_class"].items()})
PY
