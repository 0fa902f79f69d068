timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py -q --timeout 300 --timeout-method thread > gpurun_out/xcd2.log 2>&1; rc=$?; tail -2 gpurun_out/xcd2.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/xcd2.log | head; exit 1; }
O=gpurun_out/xcd_pmc
python tools/pmc_traffic.py $O/fnew $O/wnew $O/ops.json 2>/dev/null | grep -E "stem|c3k2" | head -4
CFGS="base:YH_LIB=exp_lib/base/libyolo_hip.so;new:X=1" REPS=1 bash tools/dev/envab.sh xcd2
for f in base new; do grep -E " stem | c3k2 " gpurun_out/xcd2/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
