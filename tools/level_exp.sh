#!/bin/bash
# Level-program timing experiments: correctness test, then op profiles with
# debug skip masks (YH_LEVEL_SKIP bit k skips LevelOpKind k: 1 conv, 2 dw, 4 pool, 8 attn).
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-lexp}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_level.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1 || { echo TESTS_FAIL; tail -30 "$OUT/tests.log"; exit 1; }
tail -1 "$OUT/tests.log"
for m in 0 15 14 1; do
  YH_LEVEL_SKIP=$m timeout -k 10 200 python tools/op_profile.py n 640 32 bf16 10 > "$OUT/ops_skip$m.log" 2>&1 || { echo "OPS_FAIL $m"; tail -20 "$OUT/ops_skip$m.log"; exit 1; }
  echo "== skip $m"; grep -E "forward kernels|level" "$OUT/ops_skip$m.log" | head -4
done
