timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -k "attention" -q --timeout 300 --timeout-method thread > gpurun_out/attn3.log 2>&1; rc=$?; tail -2 gpurun_out/attn3.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/attn3.log | head; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/attn_pmc; mkdir -p $O
for q in 1 2; do
YH_ATTN_QS=$q YH_OPS_OUT=$O/ops.json timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/f$q -o run -- python3 tools/pmc_run.py > $O/f$q.log 2>&1 || { echo F_FAIL; tail $O/f$q.log; exit 1; }
YH_ATTN_QS=$q timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/w$q -o run -- python3 tools/pmc_run.py > $O/w$q.log 2>&1 || { echo W_FAIL; exit 1; }
python tools/pmc_traffic.py $O/f$q $O/w$q $O/ops.json > $O/t$q.txt; grep -E "attention|forward" $O/t$q.txt | head -3
done
CFGS="qs1:YH_ATTN_QS=1;qs2:YH_ATTN_QS=2" REPS=2 bash tools/dev/envab.sh attn3
for f in qs1 qs2; do grep -E " attention " gpurun_out/attn3/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
