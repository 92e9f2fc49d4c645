#!/bin/bash
# A/B of kernel-variant libraries: scratch/ab.sh CONFIG lib1 lib2 ...   (lib "base" = in-tree)
CFG=$1; shift
mkdir -p gpurun_out/ab
for L in "$@"; do
  if [ "$L" = base ]; then LIB=""; else LIB=$PWD/scratch/lib_$L.so; fi
  CVHIP_LIB=$LIB CVHIP_SIDE_STREAM=0 timeout -k 10 200 python bench.py --config $CFG --steps 200 --no-c3 --no-cpu-baseline --kernel-table gpurun_out/ab/${CFG}_$L.txt > gpurun_out/ab/${CFG}_$L.log 2>/dev/null || { echo "$L failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab/${CFG}_$L.log').readlines()[-1]); print('$CFG $L', d['value'], d['ms_per_step'])"
done
