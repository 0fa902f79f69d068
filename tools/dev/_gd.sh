CFGS="base:X=1;g5:YH_TUNE_GDIV=5;g15:YH_TUNE_GDIV=15" REPS=3 bash tools/dev/envab.sh gd
