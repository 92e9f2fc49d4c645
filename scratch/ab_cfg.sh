#!/bin/bash
# A/B of environment settings on one bench config: scratch/ab_cfg.sh CONFIG TAG1 "VAR=v" TAG2 "..." ...
CFG=$1; shift
while [ $# -ge 2 ]; do
  TAG=$1; ENVS=$2; shift 2
  env $ENVS timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline --steps 60 --warmup 10 --kernel-table gpurun_out/ktable_${CFG}_$TAG.txt > gpurun_out/bench_${CFG}_$TAG.json 2> gpurun_out/bench_${CFG}_$TAG.err || { echo "bench $TAG failed"; tail -5 gpurun_out/bench_${CFG}_$TAG.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/bench_${CFG}_$TAG.json').read().strip().splitlines()[-1]); print('$CFG $TAG', d['value'], d['ms_per_step'])"
done
