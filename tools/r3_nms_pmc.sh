#!/bin/bash
# PMC passes over tools/nms_bench.py (one rocprofv3 --pmc run each)
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r3p; rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $OUT/sq -o run -- python3 $R/tools/nms_bench.py > $OUT/sq.log 2>&1 || { echo PMC_FAIL sq; tail -5 $OUT/sq.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/tools/nms_bench.py > $OUT/fetch.log 2>&1 || { echo PMC_FAIL fetch; tail -5 $OUT/fetch.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/write -o run -- python3 $R/tools/nms_bench.py > $OUT/write.log 2>&1 || { echo PMC_FAIL write; tail -5 $OUT/write.log; exit 1; }
echo ok
