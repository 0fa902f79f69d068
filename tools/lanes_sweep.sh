#!/bin/bash
# Sweep forward lanes (and the NMS placement) for bench.py (v11_n b32 bf16).
set -o pipefail
O=gpurun_out/${1:-lanes}
mkdir -p $O
run() {   # name, then bench args
    local n=$1; shift
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 40 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'])"
}
run l2 --lanes 2
run l3 --lanes 3
run l4 --lanes 4
run l3nms --lanes 3 --nms-on-lane
run l4nms --lanes 4 --nms-on-lane
run l3b --lanes 3
