#!/bin/bash
# Kernel iteration: conv-kernel bit-identity tests, tuning log + per-op profile, bench.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-it}; mkdir -p "$OUT"; cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv_kernels.py tests/test_gpu_forward.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTS_FAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
YH_TUNE_LOG=1 YH_PROF_OUT="$OUT/ops.json" timeout -k 10 300 python tools/op_profile.py n 640 32 bf16 10 > "$OUT/ops.log" 2> "$OUT/tune.log" || { echo OPS_FAIL; tail -20 "$OUT/tune.log"; exit 1; }
head -3 "$OUT/ops.log" | grep -v amdgpu.ids
timeout -k 10 300 python bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo BENCH_FAIL; tail -20 "$OUT/bench.err"; exit 1; }
grep -E "conv3x3|conv1x1" "$OUT/bench.err"; python -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'])"
