#!/bin/bash
# One GPU round on the box: gpu tests, per-op profile, bench. Each GPU step has its
# own time limit; the chain stops at the first failure.
set -o pipefail
OUT=${1:-gpurun_out/round}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > "$OUT/tests.log" 2>&1 || { echo "TESTS FAILED"; tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 300 python tools/op_profile.py n 640 32 bf16 10 > "$OUT/ops.log" 2>&1 || { echo "OPS FAILED"; tail -20 "$OUT/ops.log"; exit 1; }
head -3 "$OUT/ops.log"
timeout -k 10 400 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "BENCH FAILED"; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.err" | grep -v amdgpu.ids; cat "$OUT/bench.json"
