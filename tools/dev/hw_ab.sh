# same-box A/B of the wide head_cls level (YH_HCLS_WIDE): op profile and bench, both ways
timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_hw_on.txt 2>&1 || exit 1
YH_HCLS_WIDE=0 timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_hw_off.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_hw_on.json 2>/dev/null || exit 1
YH_HCLS_WIDE=0 timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_hw_off.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_hw_on2.json 2>/dev/null || exit 1
