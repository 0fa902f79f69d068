set -o pipefail
mkdir -p gpurun_out/r8
YH_CONV=2 timeout -k 10 300 python -m pytest tests/test_gpu_forward.py -x -q > gpurun_out/r8/tests_direct.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r8/tests_direct.log; exit 1; }
tail -1 gpurun_out/r8/tests_direct.log
bash tools/conv_sweep.sh gpurun_out/r8 "nosk:YH_CONV=2 YH_SPLITK_MAX=0" "sk2k:YH_CONV=2 YH_SPLITK_MAX=2048" "sk4k:YH_CONV=2 YH_SPLITK_MAX=4096" "sk16k:YH_CONV=2 YH_SPLITK_MAX=16384"
