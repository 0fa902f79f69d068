cd tools/micro
for b in 4 5 7 10; do YH_C3K_BANDS=$b timeout -k 10 60 ./c3k_bench 32 20 20 64 | grep "per launch"; done
for b in 8 10 13; do YH_C3K_BANDS=$b timeout -k 10 60 ./c3k_bench 32 40 40 32 | grep "per launch"; done
