#!/bin/bash
# End-of-round evidence in one call: every GPU test, smoke(), tools/prof_round.sh (PMC traffic,
# bench with the CPU baseline, rocprofv3 kernel stats, forward trace), the C3 / C5 bench lines.
# Outputs under gpurun_out/$1; copy what is judged into profiles/.
set -o pipefail
T=${1:-final}; O=gpurun_out/$T; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/gpu_tests.log; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
bash tools/prof_round.sh $T/prof > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof.log; exit 1; }
bash tools/configs_bench.sh $T/cfg > $O/cfg.log 2>&1 || { echo CFG_FAIL; tail -20 $O/cfg.log; exit 1; }
echo FINAL_OK
