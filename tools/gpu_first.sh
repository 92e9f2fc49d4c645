#!/bin/bash
# New-kernel gate, then the full session: tools/gpu_first.sh TAG FIRST_TEST_FILE
TAG=$1; FIRST=$2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest $FIRST -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/gputest_${TAG}_first.txt 2>&1
rc=$?
tail -5 gpurun_out/gputest_${TAG}_first.txt
if [ $rc -ne 0 ]; then echo "first gate rc=$rc: stopping"; exit $rc; fi
exec_rc=0
bash tools/gpu_round.sh $TAG
