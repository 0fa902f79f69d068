timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -k "c3k" -q --timeout 300 --timeout-method thread > gpurun_out/c3ks.log 2>&1; rc=$?; tail -2 gpurun_out/c3ks.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/c3ks.log | head; exit 1; }
timeout -k 10 300 python -u tools/op_profile.py n 640 32 bf16 5 > gpurun_out/c3ks_ops.txt 2>&1; grep -E "forward kernels| c3k  " gpurun_out/c3ks_ops.txt
