set -o pipefail
mkdir -p gpurun_out/r7
YH_CONV=2 timeout -k 10 300 python -m pytest tests/test_gpu_forward.py -x -q > gpurun_out/r7/tests_direct.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r7/tests_direct.log; exit 1; }
tail -1 gpurun_out/r7/tests_direct.log
for v in n s; do
  YH_CONV=0 timeout -k 10 120 python tools/conv_compare.py save /tmp/y0_$v.pt $v 640 8 bf16 && \
  YH_CONV=2 timeout -k 10 120 python tools/conv_compare.py save /tmp/y2_$v.pt $v 640 8 bf16 || exit 1
  python tools/conv_compare.py diff /tmp/y0_$v.pt /tmp/y2_$v.pt
done
bash tools/conv_sweep.sh gpurun_out/r7 "g2:YH_CONV=0" "d2:YH_CONV=2"
