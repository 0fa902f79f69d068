YH_ATTN_QS=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_fusion.py -k "attention_full" -q --timeout 300 --timeout-method thread > gpurun_out/attn.log 2>&1; rc=$?; tail -3 gpurun_out/attn.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/attn.log | head; exit 1; }
CFGS="qs1:X=1;qs2:YH_ATTN_QS=2;qs4:YH_ATTN_QS=4;nofull:YH_ATTN_FULL=0" REPS=2 bash tools/dev/envab.sh attn2
for f in qs1 qs2 qs4 nofull; do grep -E " attention " gpurun_out/attn2/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
