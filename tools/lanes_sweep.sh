#!/bin/bash
# Sweep forward lanes x segment split x HW queues for bench.py (v11_n b32 bf16).
set -o pipefail
O=gpurun_out/lanes5
mkdir -p $O
run() {   # name, then KEY=VAL env settings, then bench args
    local n=$1; shift
    local envs=(); while [[ "$1" == *=* ]]; do envs+=("$1"); shift; done
    env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 40 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['ms_per_step'])"
}
run t0 --lanes 3
run t3 YH_TUNE_TPUT=3 --lanes 3
run t2 YH_TUNE_TPUT=2 --lanes 3
run t0b --lanes 3
run t3b YH_TUNE_TPUT=3 --lanes 3
