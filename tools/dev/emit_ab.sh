# same-box A/B of nms_emit: default library vs tools/dev/libyh_nmsold.so (round-3 emit), alternating
set -o pipefail
mkdir -p gpurun_out/em
timeout -k 10 300 python -u -m pytest tests/test_gpu_nms.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/em/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/em/tests.log; exit 1; }
for r in a b; do
for v in new old; do
L=; [ $v = old ] && L=$GRAFT_REPO_ROOT/tools/dev/libyh_nmsold.so
rm -rf gpurun_out/em/p_$v$r
YH_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/em/p_$v$r -o nms -- python3 tools/nms_bench.py > gpurun_out/em/nb_$v$r.txt 2>&1 || { echo "prof failed"; tail -20 gpurun_out/em/nb_$v$r.txt; exit 1; }
done; done
for r in a b; do for v in new old; do L=; [ $v = old ] && L=$GRAFT_REPO_ROOT/tools/dev/libyh_nmsold.so
YH_LIB=$L timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/em/b_$v$r.json 2>/dev/null || exit 1
done; done
echo ok
