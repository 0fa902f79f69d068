timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -k "c3k" -q --timeout 300 --timeout-method thread > gpurun_out/split.log 2>&1; rc=$?; tail -2 gpurun_out/split.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/split.log | head; exit 1; }
(cd tools/micro && timeout -k 10 60 ./c3k_bench 32 20 20 64 32 40 40 32 && YH_C3K_SPLIT=0 timeout -k 10 60 ./c3k_bench 32 20 20 64) > gpurun_out/split_micro.txt 2>&1; grep "per launch" gpurun_out/split_micro.txt
CFGS="nosplit:YH_C3K_SPLIT=0;split:X=1" REPS=2 bash tools/dev/envab.sh split
for f in nosplit split; do grep -E " c3k  " gpurun_out/split/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
