for r in 1 2; do
for v in 0 1; do
YH_TUNE_READS1=$v timeout -k 10 400 python -u bench.py --variant x --size 1280 --batch 16 --steps 10 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r1_x_$v.json 2>/dev/null || exit 1
YH_TUNE_READS1=$v timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline > gpurun_out/r1_n_$v.json 2>/dev/null || exit 1
python -c "import json;print('reads1=$v', 'x', json.load(open('gpurun_out/r1_x_$v.json'))['value'], 'n', json.load(open('gpurun_out/r1_n_$v.json'))['value'])"
done
done
