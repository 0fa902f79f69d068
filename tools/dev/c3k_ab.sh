# A/B of the fused C3k blocks in one process pair on the same box
timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_c3k_on.txt 2>&1 || exit 1
YH_C3K=0 timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_c3k_off.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_c3k_on.json 2>/dev/null || exit 1
YH_C3K=0 timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_c3k_off.json 2>/dev/null || exit 1
