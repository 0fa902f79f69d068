#!/bin/bash
# Quick GPU iteration: selected gpu tests, per-op profile, bench (no CPU baseline).
#   bash tools/quick.sh OUTNAME "tests/test_a.py tests/test_b.py" [extra bench args]
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-quick}
TESTS=${2:-tests}
shift 2
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTS_FAIL; tail -40 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
YH_PROF_OUT="$OUT/ops.json" timeout -k 10 300 python tools/op_profile.py n 640 32 bf16 10 > "$OUT/ops.log" 2>&1 || { echo OPS_FAIL; tail -20 "$OUT/ops.log"; exit 1; }
head -3 "$OUT/ops.log" | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
grep -v amdgpu.ids "$OUT/bench.err"; cat "$OUT/bench.json"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --serial "$@" > "$OUT/bench_serial.json" 2> "$OUT/bench_serial.err" || { echo BENCH_SERIAL_FAIL; tail -20 "$OUT/bench_serial.err"; exit 1; }
cat "$OUT/bench_serial.json"
