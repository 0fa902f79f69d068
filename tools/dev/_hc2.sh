CFGS="new:X=1;hc1024:YH_LIB=exp_lib/hc1024/libyolo_hip.so" REPS=3 bash tools/dev/envab.sh hc2
for f in new hc1024; do grep -E " head_cls " gpurun_out/hc2/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
