CFGS="base:X=1;g5:YH_TUNE_GDIV=5;g3:YH_TUNE_GDIV=3" REPS=4 bash tools/dev/envab.sh gd2
