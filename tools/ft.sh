# Serial forward kernel trace (tools/fwd_trace.py) mapped to ops; with MX="<filter>"
# also the conv_mx micro bench (MX_ABL / MX_TRACE pass through).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ft}; mkdir -p $O
if [ -n "$MX" ]; then for f in $MX; do timeout -k 10 200 tools/micro/mx_bench "$f" >> $O/mx.txt 2>&1 || { echo MX_FAIL; tail $O/mx.txt; exit 1; }; done; fi
YH_OPS_OUT=$O/ops_meta.json timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $O/tr -o run -- python3 tools/fwd_trace.py > $O/run.log 2>&1 || { echo FT_FAIL; tail -20 $O/run.log; exit 1; }
python tools/trace_ops.py $O/tr $O/ops_meta.json --json $O/ops.json > $O/ops.txt 2>&1; head -45 $O/ops.txt
