cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
O=gpurun_out/pmc_c3k; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d $O/p1 -o p1 -- tools/micro/c3k_bench 32 20 20 64 32 40 40 32 > $O/p1.log 2>&1 || { echo P1_FAIL; tail $O/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_INSTS_VMEM SQ_WAVES SQ_INST_LEVEL_LDS --output-format csv -d $O/p2 -o p2 -- tools/micro/c3k_bench 32 20 20 64 32 40 40 32 > $O/p2.log 2>&1 || { echo P2_FAIL; tail $O/p2.log; exit 1; }
find $O -name "*counter_collection.csv" | head
