#!/bin/bash
# A/B of environment settings on the default bench (MNIST + weak-scaling keys) with kernel tables:
#   scratch/ab_env.sh TAG1 "VAR=v VAR2=v" TAG2 "..." ...   (empty string = defaults)
while [ $# -ge 2 ]; do
  TAG=$1; ENVS=$2; shift 2
  env $ENVS timeout -k 10 300 python bench.py --no-c3 --no-cpu-baseline --kernel-table gpurun_out/ktable_$TAG.txt > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench $TAG failed"; tail -5 gpurun_out/bench_$TAG.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1]); print('$TAG', d['value'], d['ms_per_step'], {k: (d[k].get('value'), d[k].get('ms_per_step')) for k in ('celeba','pacs','camelyon_bf16') if k in d})"
done
