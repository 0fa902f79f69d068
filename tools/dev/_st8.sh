YH_LIB=exp_lib/st8/libyolo_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py -k "stem or fused_head" -q --timeout 300 --timeout-method thread > gpurun_out/st8.log 2>&1; rc=$?; tail -2 gpurun_out/st8.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/st8.log | head; exit 1; }
CFGS="st4:X=1;st8:YH_LIB=exp_lib/st8/libyolo_hip.so" REPS=3 bash tools/dev/envab.sh st8
for f in st4 st8; do grep -E " stem " gpurun_out/st8/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
