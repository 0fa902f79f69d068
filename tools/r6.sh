set -o pipefail
mkdir -p gpurun_out/r6
YH_CONV=2 timeout -k 10 300 python -m pytest tests/test_gpu_forward.py -x -q > gpurun_out/r6/tests_direct.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/r6/tests_direct.log; exit 1; }
tail -1 gpurun_out/r6/tests_direct.log
for v in n s; do for dt in bf16 fp16; do
  YH_CONV=0 timeout -k 10 120 python tools/conv_compare.py save gpurun_out/r6/y0_$v$dt.pt $v 640 8 $dt && \
  YH_CONV=2 timeout -k 10 120 python tools/conv_compare.py save gpurun_out/r6/y2_$v$dt.pt $v 640 8 $dt || exit 1
  python tools/conv_compare.py diff gpurun_out/r6/y0_$v$dt.pt gpurun_out/r6/y2_$v$dt.pt
done; done
rm -f gpurun_out/r6/*.pt
bash tools/conv_sweep.sh gpurun_out/r6 "g2:YH_CONV=0" "d2:YH_CONV=2"
