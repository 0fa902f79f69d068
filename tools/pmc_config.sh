#!/bin/bash
# PMC HBM-traffic passes for a non-headline bench configuration; installs the summary as
# profiles/pmc_traffic_<variant>_<size>_b<batch>_<dtype>.json, which bench.py's roofline reads
# for that configuration.   bash tools/pmc_config.sh x 1280 16 bf16
set -o pipefail
V=$1; S=$2; B=$3; D=$4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pmc_${V}_${S}_b${B}_${D}; mkdir -p $O
export YH_VARIANT=$V YH_SIZE=$S YH_BATCH=$B YH_DTYPE=$D
YH_OPS_OUT=$O/ops.json timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d $O/fetch -o run -- python3 tools/pmc_run.py > $O/fetch.log 2>&1 || { echo FETCH_FAIL; tail $O/fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d $O/write -o run -- python3 tools/pmc_run.py > $O/write.log 2>&1 || { echo WRITE_FAIL; tail $O/write.log; exit 1; }
python tools/pmc_traffic.py $O/fetch $O/write $O/ops.json $O/pmc_traffic.json > $O/pmc.txt || { echo MAP_FAIL; exit 1; }
cp $O/pmc_traffic.json profiles/pmc_traffic_${V}_${S}_b${B}_${D}.json
head -14 $O/pmc.txt
