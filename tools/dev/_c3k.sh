

timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -q --timeout 300 --timeout-method thread > gpurun_out/fus.log 2>&1; rc=$?; tail -3 gpurun_out/fus.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/fus.log | head; exit 1; }

[ $rc -lt 124 ] && CFGS="base:YH_LIB=exp_lib/base/libyolo_hip.so;new:X=1;nopersist:YH_STEM_PERSIST=0;hc1024:YH_LIB=exp_lib/hc1024/libyolo_hip.so" bash tools/dev/envab.sh c3kp
for f in base new nopersist hc1024; do grep -E " c3k  | stem | head_cls " gpurun_out/c3kp/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
