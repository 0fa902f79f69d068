O=gpurun_out/rep; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" $O/tests.log | head -20; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
for r in 1 2 3 4 5; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/b$r.json 2>/dev/null || exit 1
  python -c "import json;r=json.load(open('$O/b$r.json'));print('run $r', r['value'], 'img/s', r['ms_per_step'], 'ms/step', 'frac', r['roofline']['frac'])" | tee -a $O/summary.txt
done
