#!/bin/bash
# Full GPU round: gpu tests, per-op profile, bench (with CPU baseline), rocprofv3
# kernel-trace stats of the bench, and FETCH_SIZE / WRITE_SIZE PMC passes.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r10}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTS_FAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
timeout -k 10 300 python tools/op_profile.py n 640 32 bf16 10 > "$OUT/ops.log" 2>&1 || { echo OPS_FAIL; tail -20 "$OUT/ops.log"; exit 1; }
head -2 "$OUT/ops.log"
timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
grep -v amdgpu.ids "$OUT/bench.err"; cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof_bench.err" || { echo PROF_FAIL; tail -20 "$OUT/prof_bench.err"; exit 1; }
cat "$OUT/prof_bench.json"
YH_OPS_OUT="$OUT/ops.json" timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 "$R/tools/pmc_run.py" > "$OUT/pmc_fetch.log" 2>&1 || { echo PMC_FETCH_FAIL; tail -20 "$OUT/pmc_fetch.log"; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- python3 "$R/tools/pmc_run.py" > "$OUT/pmc_write.log" 2>&1 || { echo PMC_WRITE_FAIL; tail -20 "$OUT/pmc_write.log"; exit 1; }
cd "$R"
python tools/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/ops.json" "$OUT/pmc_traffic.json" || echo PMC_PARSE_FAIL
find "$OUT" -name "*stats.csv" | head
