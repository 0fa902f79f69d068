set -o pipefail
bash tools/conv_sweep.sh gpurun_out/r6 "g2:YH_CONV=0" "d2:YH_CONV=2"
