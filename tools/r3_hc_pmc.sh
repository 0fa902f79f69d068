#!/bin/bash
# SQ counter passes over head_cls (tools/op_profile.py: eager v11_n b32 bf16 forwards)
set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/hcp; rm -rf "$OUT"; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 150 rocprofv3 --kernel-include-regex "$1" --pmc $3 --output-format csv -d $OUT/$2 -o run -- python3 $R/tools/op_profile.py n 640 32 bf16 2 > $OUT/$2.log 2>&1 || { echo PMC_FAIL $2; tail -5 $OUT/$2.log; exit 1; }
}
run head_cls a "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_WAVE_CYCLES"
run head_cls b "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_ANY"
run head_cls c "SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_EXP SQ_INSTS_SMEM SQ_INSTS_FLAT"
echo ok
