#!/bin/bash
# SQ counters of one step-program call: tools/pmc_one.sh CONFIG CALL TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=$1; C=$2; TAG=$3
D=gpurun_out/pmc_sq/${TAG}_${CFG}_$(echo $C | tr -d '[]')
mkdir -p $D
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $D -o run -- python3 bench.py --config $CFG --only-call "$C" --reps 20 --warmup 3 --no-cpu-baseline --no-kernel-pass > $D/log.txt 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 bench.py --config $CFG --only-call "$C" --reps 20 --warmup 3 --no-cpu-baseline --no-kernel-pass > $D/log2.txt 2>&1
echo ok $D
