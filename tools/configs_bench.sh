#!/bin/bash
# Bench lines for the other BASELINE.json configs (C3: v11_s fp16 b64 640; C5:
# v11_x bf16 b16 1280) - same bench.py, one GPU, each step under its own limit.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-cfg}; mkdir -p "$OUT"; cd "$R"
timeout -k 10 400 python bench.py --variant s --dtype fp16 --batch 64 --no-cpu-baseline > "$OUT/c3.json" 2> "$OUT/c3.err" || { echo C3_FAIL; tail -20 "$OUT/c3.err"; exit 1; }
cat "$OUT/c3.json"
timeout -k 10 500 python bench.py --variant x --size 1280 --batch 16 --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/c5.json" 2> "$OUT/c5.err" || { echo C5_FAIL; tail -20 "$OUT/c5.err"; exit 1; }
cat "$OUT/c5.json"
