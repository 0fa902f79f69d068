set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/stem
for tr in 2 4 8; do
  YH_STEM_TR=$tr YH_PROF_OUT=gpurun_out/stem/ops_$tr.json timeout -k 10 200 python tools/op_profile.py n 640 32 bf16 10 > gpurun_out/stem/ops_$tr.log 2>&1 || exit 1
done
YH_STEM=1 YH_PROF_OUT=gpurun_out/stem/ops_old.json timeout -k 10 200 python tools/op_profile.py n 640 32 bf16 10 > gpurun_out/stem/ops_old.log 2>&1
