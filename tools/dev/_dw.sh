timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dw_tests.log 2>&1; rc=$?; tail -2 gpurun_out/dw_tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/dw_tests.log | head; exit 1; }
for v in new base; do
  L=""; [ $v = base ] && L="YH_LIB=exp_lib/base/libyolo_hip.so"
  env $L timeout -k 10 300 python -u tools/op_profile.py x 1280 16 bf16 5 > gpurun_out/dw_x_$v.txt 2>&1 || exit 1
  env $L timeout -k 10 300 python -u tools/op_profile.py s 640 64 fp16 5 > gpurun_out/dw_s_$v.txt 2>&1 || exit 1
done
for f in gpurun_out/dw_x_new.txt gpurun_out/dw_x_base.txt gpurun_out/dw_s_new.txt gpurun_out/dw_s_base.txt; do echo $f; grep "forward kernels" $f; grep " dwconv " $f | awk '{s+=$1} END {print "dwconv total", s}'; done
