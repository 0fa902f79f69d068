YH_LIB=exp_lib/bd2/libyolo_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py -k "fused_head" -q --timeout 300 --timeout-method thread 2>&1 | tail -1
YH_LIB=exp_lib/bd8/libyolo_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fusion.py -k "fused_head" -q --timeout 300 --timeout-method thread 2>&1 | tail -1
CFGS="t4:X=1;t2:YH_LIB=exp_lib/bd2/libyolo_hip.so;t8:YH_LIB=exp_lib/bd8/libyolo_hip.so" REPS=2 bash tools/dev/envab.sh bd
for f in t4 t2 t8; do grep -E " box_dfl " gpurun_out/bd/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
