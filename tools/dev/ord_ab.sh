# head_cls workgroup order A/B: 20x20 level first (default) vs levels in order (tools/dev/libyh_ord.so)
set -o pipefail
L=$GRAFT_REPO_ROOT/tools/dev/libyh_ord.so
timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_ord_def.txt 2>&1 || exit 1
YH_LIB=$L timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_ord_seq.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_ord_def2.txt 2>&1 || exit 1
YH_LIB=$L timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > gpurun_out/op_ord_seq2.txt 2>&1 || exit 1
