#!/bin/bash
# Fused C3k2 (c3k2.hip) tile / workgroups-per-CU sweep: per-op eager times of the two
# fused blocks (tools/op_profile.py) for each setting. Output under gpurun_out/$1.
set -o pipefail
O=gpurun_out/${1:-csp}; mkdir -p $O
for cfg in "8x16 1" "8x16 2" "8x8 2" "8x8 3" "16x16 1" "4x16 2"; do
  set -- $cfg
  YH_CSP_TILE=$1 YH_CSP_WG_PER_CU=$2 timeout -k 10 120 python tools/op_profile.py n 640 32 bf16 10 > $O/op_$1_$2.txt 2>&1 || { echo "FAIL $cfg"; tail $O/op_$1_$2.txt; exit 1; }
  echo "tile $1 per_cu $2: $(grep -E 'net.p2.1 |net.p3.1 ' $O/op_$1_$2.txt | tr -s ' ' | tr '\n' '|')"
done
