timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -k "sppf or attention_full" -q --timeout 300 --timeout-method thread > gpurun_out/sppf.log 2>&1; rc=$?; tail -3 gpurun_out/sppf.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/sppf.log | head; exit 1; }
CFGS="base:YH_LIB=exp_lib/base/libyolo_hip.so;new:X=1;cpw1:YH_SPPF_CPW=1;cpw4:YH_SPPF_CPW=4" REPS=1 bash tools/dev/envab.sh sppf
for f in base new cpw1 cpw4; do grep -E " sppf " gpurun_out/sppf/op_$f.txt | awk -v f=$f '{print f, $0}'; done
