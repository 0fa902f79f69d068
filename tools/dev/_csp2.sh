CFGS="new:X=1;t16w:YH_LIB=exp_lib/csp1024/libyolo_hip.so YH_CSP_TILE=16x16;t816w:YH_LIB=exp_lib/csp1024/libyolo_hip.so YH_CSP_TILE=8x32" REPS=3 bash tools/dev/envab.sh csp2
for f in new t16w t816w; do grep -E " c3k2 " gpurun_out/csp2/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
