#!/bin/bash
# SQ-counter passes (one rocprofv3 --pmc run each) over the eager bench forward with
# every eligible conv forced to kernel $2 and $3.
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/${1:-sq}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for k in $2 $3; do
  YH_CONV=$k YH_OPS_OUT=$OUT/ops$k.json timeout -s KILL 150 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d $OUT/p$k -o run -- python3 $R/tools/pmc_run.py > $OUT/p$k.log 2>&1 || { echo PMC_FAIL $k; tail -5 $OUT/p$k.log; exit 1; }
  python3 $R/tools/pmc_sq.py $OUT/p$k $OUT/ops$k.json head.box.0.0 net.p3.0 head.box.1.1 net.p5.1.res_m.0.res_m.0.conv1 fpn.h1.res_m.0.conv1
done
