#!/bin/bash
# split-greedy NMS check: bit-exact tests, phase trace, per-kernel rocprof durations
set -o pipefail
mkdir -p gpurun_out/r3n
timeout -k 10 300 python -u -m pytest tests/test_gpu_nms.py tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r3n/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r3n/tests.log; exit 1; }
YH_LIB=exp_lib/libyolo_hip.so timeout -k 10 120 python -u tools/nms_trace.py > gpurun_out/r3n/nms_trace.txt 2>&1 || { echo "trace failed"; tail -20 gpurun_out/r3n/nms_trace.txt; exit 1; }
rm -rf gpurun_out/r3n/prof
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3n/prof -o nms -- python3 tools/nms_bench.py > gpurun_out/r3n/nms_bench.txt 2>&1 || { echo "prof failed"; tail -20 gpurun_out/r3n/nms_bench.txt; exit 1; }
echo ok
