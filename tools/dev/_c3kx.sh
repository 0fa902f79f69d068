YH_C3K=0 timeout -k 10 300 python -u tools/op_profile.py s 640 64 fp16 5 > gpurun_out/ops_c3_noc3k.txt 2>&1
grep "forward kernels" gpurun_out/ops_c3_noc3k.txt; grep "net.p4.1.res_m.0" gpurun_out/ops_c3_noc3k.txt | awk '{s+=$1} END {print "per-layer sum", s}'
for b in 1 2; do
timeout -k 10 300 python -u bench.py --variant s --dtype fp16 --batch 64 --no-cpu-baseline --no-roofline > gpurun_out/c3_on_$b.json 2>/dev/null
YH_C3K=0 timeout -k 10 300 python -u bench.py --variant s --dtype fp16 --batch 64 --no-cpu-baseline --no-roofline > gpurun_out/c3_off_$b.json 2>/dev/null
python -c "import json;print('on', json.load(open('gpurun_out/c3_on_$b.json'))['value'], 'off', json.load(open('gpurun_out/c3_off_$b.json'))['value'])"
done
