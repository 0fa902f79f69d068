#!/bin/bash
# SQ-counter pass (MFMA busy, wave / wait cycles) over one eager forward of a bench configuration,
# per op: bash tools/pmc_sq_cfg.sh x 1280 16 bf16 [out]
set -o pipefail
V=$1; S=$2; B=$3; D=$4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${5:-sq_${V}_${S}_b${B}_${D}}; mkdir -p $O
export YH_VARIANT=$V YH_SIZE=$S YH_BATCH=$B YH_DTYPE=$D
YH_OPS_OUT=$O/ops.json timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -f csv -d $O/sq -o run -- python3 tools/pmc_run.py > $O/sq.log 2>&1 || { echo SQ_FAIL; tail $O/sq.log; exit 1; }
python tools/pmc_sq_ops.py $O/sq $O/ops.json conv3x3 conv1x1 > $O/sq_ops.txt || { echo MAP_FAIL; exit 1; }
tail -3 $O/sq_ops.txt
