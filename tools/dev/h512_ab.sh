# same-box A/B: default head_cls (4-wave workgroups) vs the 8-wave build in tools/dev/libyh512.so
L=$GRAFT_REPO_ROOT/tools/dev/libyh512.so
YH_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fusion.py -k "head" > gpurun_out/t_h512.txt 2>&1 || { tail gpurun_out/t_h512.txt; exit 1; }
timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_h256.txt 2>&1 || exit 1
YH_LIB=$L timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_h512.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_h256.json 2>/dev/null || exit 1
YH_LIB=$L timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_h512.json 2>/dev/null || exit 1
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_h256b.json 2>/dev/null || exit 1
YH_LIB=$L timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_h512b.json 2>/dev/null || exit 1
