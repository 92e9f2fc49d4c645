#!/bin/bash
# SQ counters of single step-program calls: scratch/pmc_sq.sh CONFIG CALL [CALL...]
CFG=$1; shift
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for C in "$@"; do
  D=gpurun_out/pmc_sq/${CFG}_$(echo $C | tr -d '[]')
  mkdir -p $D
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d $D -o run -- python3 bench.py --config $CFG --only-call "$C" --reps 20 --warmup 3 > $D/log.txt 2>&1 || { echo "pmc $C failed"; tail -5 $D/log.txt; exit 1; }
done
echo done
