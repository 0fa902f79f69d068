# 256-cout staged conv_mx plans: bit-identity of every plan, then C5 bench new vs tools/dev/libyh_cmxold.so, alternating
set -o pipefail
mkdir -p gpurun_out/cmx
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv_kernels.py -x -q --timeout 400 --timeout-method thread > gpurun_out/cmx/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/cmx/tests.log; exit 1; }
for r in a b; do for v in new old; do L=; [ $v = old ] && L=$GRAFT_REPO_ROOT/tools/dev/libyh_cmxold.so
YH_LIB=$L timeout -k 10 400 python -u bench.py --variant x --size 1280 --batch 16 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/cmx/c5_$v$r.json 2> gpurun_out/cmx/c5_$v$r.err || { tail gpurun_out/cmx/c5_$v$r.err; exit 1; }
done; done
echo ok
