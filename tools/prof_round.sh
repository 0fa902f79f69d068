# rocprofv3 kernel trace + stats of the default bench command (no CPU baseline);
# summaries go to gpurun_out/$1 (copy what is judged into profiles/).
set -o pipefail
OUT=${1:-gpurun_out/prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d "$OUT" -o run -- python3 bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo PROF_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
find "$OUT" -name "*.csv" | head -20
