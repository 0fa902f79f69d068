YH_CSP_TILE=16x16 timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -k "fused_equals or csp" -q --timeout 300 --timeout-method thread > gpurun_out/csp.log 2>&1; rc=$?; tail -3 gpurun_out/csp.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/csp.log | head; exit 1; }
CFGS="base:YH_LIB=exp_lib/base/libyolo_hip.so;new:X=1;t16:YH_CSP_TILE=16x16;t16w:YH_LIB=exp_lib/csp1024/libyolo_hip.so YH_CSP_TILE=16x16;t816w:YH_LIB=exp_lib/csp1024/libyolo_hip.so YH_CSP_TILE=8x32" REPS=1 bash tools/dev/envab.sh csp
for f in base new t16 t16w t816w; do grep -E " c3k2 " gpurun_out/csp/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
