#!/bin/bash
# PMC HBM-traffic passes (FETCH_SIZE, WRITE_SIZE; one counter group per run) of one eager
# v11_n b32 forward, mapped to ops by tools/pmc_traffic.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pmc}; mkdir -p $O
YH_OPS_OUT=$O/ops.json timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 tools/pmc_run.py > $O/fetch.log 2>&1 || { echo FETCH_FAIL; tail $O/fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- python3 tools/pmc_run.py > $O/write.log 2>&1 || { echo WRITE_FAIL; tail $O/write.log; exit 1; }
python tools/pmc_traffic.py $O/fetch $O/write $O/ops.json $O/pmc_traffic.json
