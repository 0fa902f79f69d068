#!/bin/bash
# Round-6 evidence in one call: every GPU test, smoke(), tools/prof_round.sh (PMC traffic, bench with
# the CPU baseline, rocprofv3 kernel stats, forward trace), round-6 PMC summaries of C3 / C5, their
# bench lines, NMS kernel stats, and the driver's 20-step bench command twice.
# Outputs under gpurun_out/$1; tools/collect_round6.sh copies what is judged into profiles/.
set -o pipefail
T=${1:-r6final}; O=gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo TESTS_FAIL; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench20_$r.json 2> $O/bench20_$r.err || { echo BENCH20_FAIL; tail -20 $O/bench20_$r.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench20_$r.json'));print('bench20', d['value'], d['roofline']['frac'])"
done
bash tools/prof_round.sh $T/prof > $O/prof.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof.log; exit 1; }
head -3 $O/prof/bench_trace_stats.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/nb -o run -- python3 tools/nms_bench.py > $O/nb.log 2>&1 || { echo NMSB_FAIL; tail $O/nb.log; exit 1; }
bash tools/pmc_config.sh s 640 64 fp16 > $O/pmc_c3.log 2>&1 || { echo PMC_C3_FAIL; tail $O/pmc_c3.log; exit 1; }
bash tools/pmc_config.sh x 1280 16 bf16 > $O/pmc_c5.log 2>&1 || { echo PMC_C5_FAIL; tail $O/pmc_c5.log; exit 1; }
bash tools/configs_bench.sh $T/cfg > $O/cfg.log 2>&1 || { echo CFG_FAIL; tail -20 $O/cfg.log; exit 1; }
grep -h '"value"' $O/cfg/c3.json $O/cfg/c5.json | python -c "import sys,json; [print(json.loads(l)['config']['workload'], json.loads(l)['value']) for l in sys.stdin]"
echo FINAL_OK
