#!/bin/bash
# A/B of whole libraries on one box, alternating: tools/ab_libs.sh TAG "CFGS" ROUNDS LIB_A LIB_B ...
TAG=$1; CFGS=$2; ROUNDS=$3; shift 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for r in $(seq $ROUNDS); do
  for cfg in $CFGS; do
    for lib in "$@"; do
      n=$(basename $lib .so)
      out=gpurun_out/ab/${TAG}_${cfg}_${n}_$r
      CVHIP_LIB=$lib timeout -k 10 300 python -u bench.py --config $cfg --steps 100 --no-c3 --no-cpu-baseline \
        --kernel-table $out.txt > $out.log 2>&1 || { echo "$cfg $lib failed"; tail -5 $out.log; exit 1; }
      python -c "import json; d=json.loads(open('$out.log').read().strip().splitlines()[-1]); print('$r', '$cfg', '$n', d['value'], d['ms_per_step'])"
    done
  done
done
