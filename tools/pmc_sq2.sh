#!/bin/bash
# Instruction mix and stall split of step-program calls, two SQ passes + a kernel trace per call:
#   tools/pmc_sq2.sh CONFIG TAG CALL [CALL...]      (env passes through, e.g. CV_DIRECT=0)
# pass A: SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS
#         SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU
# pass B: SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU
# summary: python tools/sq_summary.py gpurun_out/pmc_sq/TAG_CONFIG_CALL
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CFG=$1; TAG=$2; shift 2
for C in "$@"; do
  D=gpurun_out/pmc_sq/${TAG}_${CFG}_$(echo $C | tr -d '[]')
  rm -rf $D; mkdir -p $D
  B="python3 bench.py --config $CFG --only-call $C --reps 20 --warmup 3 --no-cpu-baseline --no-kernel-pass"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU --output-format csv -d $D/a -o run -- $B > $D/log_a.txt 2>&1
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_INSTS_SALU \
    --output-format csv -d $D/b -o run -- $B > $D/log_b.txt 2>&1
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- $B > $D/log_t.txt 2>&1
  python3 tools/sq_summary.py $D
done
