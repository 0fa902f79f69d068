#!/bin/bash
# Op profiles and benches of the in-tree library under several env settings ($CFGS: ';'-separated
# "name:VAR=val VAR2=val" entries; "base" = exp_lib/base via YH_LIB), alternating benches.
set -o pipefail
O=gpurun_out/${1:-envab}; mkdir -p $O
IFS=';' read -ra C <<< "$CFGS"
for c in "${C[@]}"; do
  n=${c%%:*}; e=${c#*:}
  env $e timeout -k 10 200 python -u tools/op_profile.py n 640 32 bf16 10 > $O/op_$n.txt 2>&1 || { echo "OP_FAIL $n"; tail $O/op_$n.txt; exit 1; }
  grep "forward kernels" $O/op_$n.txt | sed "s/^/$n: /"
done
for r in $(seq 1 ${REPS:-1}); do
  for c in "${C[@]}"; do
    n=${c%%:*}; e=${c#*:}
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b_${n}_$r.json 2>$O/b_${n}_$r.err || { echo "B_FAIL $n"; tail $O/b_${n}_$r.err; exit 1; }
    python -c "import json;r=json.load(open('$O/b_${n}_$r.json'));print('$n', r['value'], r['roofline']['frac'], r['roofline']['forward_kernel_ms'])"
  done
done
