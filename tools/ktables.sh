#!/bin/bash
# Per-call in-step kernel tables of the bench configs under env A/B settings.
# Usage: tools/ktables.sh TAG "cfg1 cfg2 ..." "ENV_A" "ENV_B" ...   (ENV "-" = no extra env)
TAG=$1; CFGS=$2; shift 2
mkdir -p gpurun_out/kt
export TMPDIR=/tmp
for cfg in $CFGS; do
  i=0
  for envs in "$@"; do
    [ "$envs" = "-" ] && envs=""
    out=gpurun_out/kt/${TAG}_${cfg}_$i
    env $envs timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --no-c3 --no-cpu-baseline \
      --kernel-table $out.txt > $out.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "$cfg [$envs] rc=$rc"; tail -5 $out.log; exit $rc; fi
    python -c "import json; d=json.loads(open('$out.log').read().strip().splitlines()[-1]); print('$cfg', '[$envs]', d['value'], d['ms_per_step'])"
    i=$((i+1))
  done
done
