#!/bin/bash
# The direct-conv plans (tile, fragments, stages, grid) of every bench config's stride-2 calls: one eager step each
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in ${1:-mnist celeba pacs camelyon}; do
  echo "== $cfg"
  CV_DIRECT_LOG=1 timeout -k 10 200 python -u bench.py --config $cfg --steps 1 --warmup 0 --no-c3 --no-cpu-baseline \
    --no-kernel-pass 2>&1 >/dev/null | grep "^direct" | sort | uniq -c
done
