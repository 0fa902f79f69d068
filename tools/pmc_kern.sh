#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, 8 SQ counters max) over one eager
# v11_n b32 forward (tools/pmc_run.py), printed per fused kernel by tools/pmc_kern.py.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-pk}; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -f csv -d $O/p1 -o run -- python3 tools/pmc_run.py > $O/p1.log 2>&1 || { echo P1_FAIL; tail -5 $O/p1.log; exit 1; }
python tools/pmc_kern.py $O/p1 > $O/p1.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $O/p2 -o run -- python3 tools/pmc_run.py > $O/p2.log 2>&1 || { echo P2_FAIL; tail -5 $O/p2.log; exit 1; }
python tools/pmc_kern.py $O/p2 > $O/p2.txt
cat $O/p1.txt $O/p2.txt
