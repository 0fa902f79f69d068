for r in 1 2; do
for L in 2 3 4 6; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --lanes $L > gpurun_out/lanes_$L_$r.json 2>/dev/null || { echo FAIL $L; exit 1; }
  python -c "import json;r=json.load(open('gpurun_out/lanes_$L_$r.json'));print('lanes $L', r['value'], r['ms_per_step'])"
done
done
