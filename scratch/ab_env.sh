#!/bin/bash
# A/B of environment knobs on the in-tree library: scratch/ab_env.sh CONFIG "VAR=val ..." ...   ("-" = none)
CFG=$1; shift
mkdir -p gpurun_out/ab
i=0
for E in "$@"; do
  i=$((i+1))
  [ "$E" = "-" ] && E=""
  env $E timeout -k 10 200 python bench.py --config $CFG --steps 200 --no-c3 --no-cpu-baseline --kernel-table gpurun_out/ab/${CFG}_env$i.txt > gpurun_out/ab/${CFG}_env$i.log 2>/dev/null || { echo "$E failed"; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab/${CFG}_env$i.log').readlines()[-1]); print('$CFG', '$E', d['value'], d['ms_per_step'])"
done
