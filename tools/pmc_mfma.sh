#!/bin/bash
# MFMA busy cycles of one step-program call: SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE in one rocprofv3 pass
# usage: tools/pmc_mfma.sh <config> <call, e.g. 'enc[4]'>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cfg=$1; call=$2
d=gpurun_out/mfma_${cfg}_${call//[\[\]]/_}
rm -rf "$d"
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$d" -o run -- \
  python bench.py --config "$cfg" --only-call "$call" --reps 50 --warmup 5 --no-cpu-baseline --no-kernel-pass
python profiles/pmc_mfma.py "$d" "$cfg $call" 50 | tee -a gpurun_out/mfma_util.jsonl
