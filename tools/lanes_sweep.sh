#!/bin/bash
# Sweep forward lanes x segment split x HW queues for bench.py (v11_n b32 bf16).
set -o pipefail
O=gpurun_out/lanes3
mkdir -p $O
run() {   # name, then KEY=VAL env settings, then bench args
    local n=$1; shift
    local envs=(); while [[ "$1" == *=* ]]; do envs+=("$1"); shift; done
    env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 40 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'])"
}
run l3_hs0 YH_HEADSPLIT=0 --lanes 3
run l3_hs0_nl YH_HEADSPLIT=0 --lanes 3 --nms-on-lane
run l4_hs0_nl YH_HEADSPLIT=0 --lanes 4 --nms-on-lane
run l2_hs0_nl YH_HEADSPLIT=0 --lanes 2 --nms-on-lane
run l4_hs0 YH_HEADSPLIT=0 --lanes 4
run l2_hs1_nl YH_HEADSPLIT=1 --lanes 2 --nms-on-lane
run l3_hs0_b YH_HEADSPLIT=0 --lanes 3
