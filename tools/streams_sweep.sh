#!/bin/bash
# bench (no roofline / CPU baseline) for several forward stream counts
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-ss}; mkdir -p "$OUT"; cd "$R"
for n in 1 2 3 4 6 8; do
  YH_STREAMS=$n timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --serial > "$OUT/s$n.json" 2>/dev/null || { echo "FAIL $n"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/s$n.json'));print($n, d['ms_per_step'], d['value'])"
done
