timeout -k 10 600 python -u -m pytest tests/test_gpu_fusion.py -k "c3k or head" -q --timeout 300 --timeout-method thread > gpurun_out/xcd.log 2>&1; rc=$?; tail -2 gpurun_out/xcd.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/xcd.log | head; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/xcd_pmc; mkdir -p $O
for v in base new; do
  L=""; [ $v = base ] && L="YH_LIB=exp_lib/base/libyolo_hip.so"
  env $L YH_OPS_OUT=$O/ops.json timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/f$v -o run -- python3 tools/pmc_run.py > $O/f$v.log 2>&1 || { echo F_FAIL; tail $O/f$v.log; exit 1; }
  env $L timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/w$v -o run -- python3 tools/pmc_run.py > $O/w$v.log 2>&1 || { echo W_FAIL; exit 1; }
  python tools/pmc_traffic.py $O/f$v $O/w$v $O/ops.json > $O/t$v.txt; echo $v; grep -E "head_cls|c3k |forward" $O/t$v.txt | head -4
done
CFGS="base:YH_LIB=exp_lib/base/libyolo_hip.so;new:X=1" REPS=3 bash tools/dev/envab.sh xcd
for f in base new; do grep -E " c3k  | head_cls " gpurun_out/xcd/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
