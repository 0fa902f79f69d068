# same-box A/B of the depthwise item height (YH_HC_RB builds in tools/dev/libyh_rb*.so) vs the default
D=$GRAFT_REPO_ROOT/tools/dev
for v in rb2 rb5; do YH_LIB=$D/libyh_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fusion.py -k "head" > gpurun_out/t_$v.txt 2>&1 || { tail gpurun_out/t_$v.txt; exit 1; }; done
timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_rb4.txt 2>&1 || exit 1
for v in rb2 rb5; do YH_LIB=$D/libyh_$v.so timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_$v.txt 2>&1 || exit 1; done
for r in a b; do
timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_rb4$r.json 2>/dev/null || exit 1
for v in rb2 rb5; do YH_LIB=$D/libyh_$v.so timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/b_$v$r.json 2>/dev/null || exit 1; done
done
