timeout -k 10 300 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/ops_c2.txt 2>&1 && timeout -k 10 300 python -u tools/op_profile.py s 640 64 fp16 5 > gpurun_out/ops_c3.txt 2>&1 && timeout -k 10 400 python -u tools/op_profile.py x 1280 16 bf16 3 > gpurun_out/ops_c5.txt 2>&1
grep "forward kernels" gpurun_out/ops_c*.txt
