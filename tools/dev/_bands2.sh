CFGS="b4:X=1;b5:YH_C3K_BANDS=5;b7:YH_C3K_BANDS=7" REPS=3 bash tools/dev/envab.sh bands2
for f in b4 b5 b7; do grep -E " c3k  " gpurun_out/bands2/op_$f.txt | awk -v f=$f '{print f, $1, $NF}'; done
