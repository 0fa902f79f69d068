timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -k "attention" -q --timeout 300 --timeout-method thread > gpurun_out/attn4.log 2>&1; rc=$?; tail -2 gpurun_out/attn4.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/attn4.log | head; exit 1; }
timeout -k 10 300 python -u tools/op_profile.py x 1280 16 bf16 5 > gpurun_out/attn4_x_new.txt 2>&1 && YH_LIB=exp_lib/base/libyolo_hip.so timeout -k 10 300 python -u tools/op_profile.py x 1280 16 bf16 5 > gpurun_out/attn4_x_base.txt 2>&1
grep -E "attention|forward kernels" gpurun_out/attn4_x_new.txt gpurun_out/attn4_x_base.txt
