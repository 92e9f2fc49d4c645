#!/bin/bash
# One GPU-box session: the -m gpu suite (optionally a subset), then (if the suite ended normally: all passed or
# assertion failures only) the default bench line.  Usage: tools/gpu_round.sh TAG [pytest selection...]
# Outputs: gpurun_out/gputest_TAG.txt, gpurun_out/bench_TAG.json (+ .log)
TAG=$1; shift
SEL=${@:-tests}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/gputest_$TAG.txt 2>&1
rc=$?
tail -3 gpurun_out/gputest_$TAG.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
if [ -n "$NOBENCH" ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.log 2>&1
brc=$?
tail -1 gpurun_out/bench_$TAG.log > gpurun_out/bench_$TAG.json
echo "bench rc=$brc"; head -c 600 gpurun_out/bench_$TAG.json; echo
exit $brc
