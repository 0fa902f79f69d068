set -o pipefail
mkdir -p gpurun_out/r9
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/r9/tests.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r9/tests.log; exit 1; }
tail -1 gpurun_out/r9/tests.log
bash tools/conv_sweep.sh gpurun_out/r9 "auto:X=1" "g2:YH_CONV=0" || exit 1
grep -c direct gpurun_out/r9/auto.txt; 
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r9/bench.json 2> gpurun_out/r9/bench.err || { echo BENCH_FAIL; tail -20 gpurun_out/r9/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r9/bench.err; cat gpurun_out/r9/bench.json
