#!/bin/bash
# bench (no roofline / CPU baseline) under several schedules
set -o pipefail
OUT=${1:-gpurun_out/sched}; mkdir -p "$OUT"
for a in "--serial" "--lanes 1" "--lanes 2" "--lanes 3" "--lanes 4" "--lanes 3 --nms-on-lane"; do
  n=$(echo "$a" | tr -d ' -')
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $a > "$OUT/$n.json" 2>/dev/null || { echo "FAIL $a"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$n.json'));print('$a', d['ms_per_step'], d['value'])"
done
