#!/bin/bash
# Round-3 session-3 evidence: rocprofv3 kernel-trace summaries of the bench configs (part "trace"), PMC HBM traffic
# of the priced calls and of the edge calls, SQ / MFMA counters (part "pmc").  Every pass is its own run.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
part=$1
if [ "$part" = trace ]; then
  for cfg in mnist celeba-mim camelyon-bf16; do
    steps=50; [ $cfg = celeba-mim ] && steps=30
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$cfg -o run -- \
      python3 bench.py --config $cfg --steps $steps --warmup 10 --no-cpu-baseline --no-c3 --no-kernel-pass \
      > gpurun_out/prof_$cfg.log 2>&1
    echo "trace $cfg done"
  done
fi
if [ "$part" = pmc ]; then
  while read cfg label; do
    bash tools/pmc_traffic.sh $cfg "$label" > gpurun_out/pmct_${cfg}_$(echo ${label%%:*} | tr -d '[]').log 2>&1
    echo "traffic $cfg $label done"
  done <<'LIST'
mnist enc[3]:cv_conv_backward_data
celeba-mim enc[7]:cv_conv_backward_data
celeba enc[7]:cv_conv_backward_data
pacs fwd[5]:cv_conv_forward
camelyon-bf16 enc[7]:cv_conv_backward_data
mnist fwd[1]:cv_conv_forward
mnist fwd[8]:cv_conv_forward
mnist dec[0]:cv_conv_backward_deferred
mnist enc[5]:cv_conv_backward_weight_deferred
celeba fwd[1]:cv_conv_forward
celeba fwd[12]:cv_conv_forward
LIST
  bash tools/pmc_mfma.sh mnist 'enc[3]' > gpurun_out/mfma_mnist.log 2>&1
  echo "mfma done"
fi
if [ "$part" = sq ]; then
  while read cfg call; do
    D=gpurun_out/pmc_sq/${cfg}_$(echo $call | tr -d '[]')
    mkdir -p $D
    timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $D -o run -- \
      python3 bench.py --config $cfg --only-call "$call" --reps 20 --warmup 3 --no-cpu-baseline --no-kernel-pass \
      > $D/log.txt 2>&1
    echo "sq $cfg $call done"
  done <<'LIST'
mnist fwd[1]
mnist fwd[8]
mnist dec[0]
mnist enc[5]
celeba fwd[1]
celeba fwd[12]
mnist enc[3]
LIST
fi
echo ALLDONE
