timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -k "head" -q --timeout 300 --timeout-method thread > gpurun_out/hcp.log 2>&1; rc=$?; tail -2 gpurun_out/hcp.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/hcp.log | head; exit 1; }
CFGS="base:YH_LIB=exp_lib/base/libyolo_hip.so;new:X=1" REPS=3 bash tools/dev/envab.sh hcp
for f in base new; do grep -E " head_cls " gpurun_out/hcp/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
