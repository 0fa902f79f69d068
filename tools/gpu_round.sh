#!/bin/bash
# One GPU round on the box: gpu tests, serial forward trace (per-op kernel times),
# bench. Each GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo "TESTS FAILED"; tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
bash tools/ft.sh "$(basename $OUT)/ft" > /dev/null || { echo "TRACE FAILED"; exit 1; }
head -2 "$OUT/ft/ops.txt"
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "BENCH FAILED"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
