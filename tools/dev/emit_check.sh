# nms_emit rework: bit-exact NMS tests, per-kernel durations of back-to-back NMS calls
set -o pipefail
mkdir -p gpurun_out/em
timeout -k 10 300 python -u -m pytest tests/test_gpu_nms.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/em/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/em/tests.log; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/em/prof -o nms -- python3 tools/nms_bench.py > gpurun_out/em/nms_bench.txt 2>&1 || { echo "prof failed"; tail -20 gpurun_out/em/nms_bench.txt; exit 1; }
echo ok
