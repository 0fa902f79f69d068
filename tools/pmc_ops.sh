#!/bin/bash
# SQ counter passes over one eager v11_n b32 forward (tools/pmc_run.py), per op
# (tools/pmc_ops.py). Optional $2: label regex.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-po}; mkdir -p $O
export YH_OPS_OUT=$O/ops.json
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -f csv -d $O/p1 -o run -- python3 tools/pmc_run.py > $O/p1.log 2>&1 || { echo P1_FAIL; tail -5 $O/p1.log; exit 1; }
python tools/pmc_ops.py $O/p1 $O/ops.json $2 > $O/p1.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d $O/p2 -o run -- python3 tools/pmc_run.py > $O/p2.log 2>&1 || { echo P2_FAIL; tail -5 $O/p2.log; exit 1; }
python tools/pmc_ops.py $O/p2 $O/ops.json $2 > $O/p2.txt
cat $O/p1.txt $O/p2.txt
