#!/bin/bash
# bench (no roofline / CPU baseline) under several conv_mx LDS budgets (YH_MX_LDS_MAX)
set -o pipefail
OUT=${1:-gpurun_out/lds}; shift; mkdir -p "$OUT"
for v in "$@"; do
  YH_MX_LDS_MAX=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline > "$OUT/b$v.json" 2>/dev/null || { echo "FAIL $v"; exit 1; }
  python -c "import json;d=json.load(open('$OUT/b$v.json'));print('$v', d['ms_per_step'], d['value'])"
done
