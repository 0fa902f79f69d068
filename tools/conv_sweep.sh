#!/bin/bash
# Per-op timing of the forward under several conv kernel configurations.
# usage: bash tools/conv_sweep.sh OUTDIR "NAME:ENV=.. ENV=.." ...
set -o pipefail
out=$1; shift
mkdir -p "$out"
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  echo "== $name ($envs)"
  env $envs YH_PROF_OUT="$out/$name.json" timeout -k 10 240 python tools/op_profile.py n 640 32 bf16 10 > "$out/$name.txt" 2>&1 || { echo "FAILED $name rc=$?"; tail -5 "$out/$name.txt"; exit 1; }
  head -2 "$out/$name.txt"
done
