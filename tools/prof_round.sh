#!/bin/bash
# Measurement round on the box: PMC traffic passes (installed as profiles/pmc_traffic_latest.json,
# which bench.py's roofline reads), the default bench command (with the CPU baseline), the same
# bench under rocprofv3 --kernel-trace --stats, the serial per-op trace.
# Outputs under gpurun_out/$1; copy what is judged into profiles/.
set -o pipefail
OUT=gpurun_out/${1:-prof}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/pmc_round.sh "${OUT#gpurun_out/}/pmc" > "$OUT/pmc.txt" 2>&1 || { echo PMC_FAIL; tail "$OUT/pmc.txt"; exit 1; }
cp "$OUT/pmc/pmc_traffic.json" profiles/pmc_traffic_latest.json || { echo PMC_COPY_FAIL; exit 1; }
head -12 "$OUT/pmc.txt"
timeout -k 10 500 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/rp" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/bench_rocprof.json" 2> "$OUT/bench_rocprof.err" || { echo PROF_FAIL; tail -20 "$OUT/bench_rocprof.err"; exit 1; }
python tools/trace_stats.py "$OUT/rp" 50 > "$OUT/bench_trace_stats.txt"; head -3 "$OUT/bench_trace_stats.txt"
bash tools/ft.sh "${OUT#gpurun_out/}/ft" > /dev/null || { echo TRACE_FAIL; exit 1; }
