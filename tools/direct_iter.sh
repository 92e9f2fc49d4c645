#!/bin/bash
# Direct-conv iteration on the box: kernel tests, in-step phase stamps of the given MNIST calls, kernel tables.
#   tools/direct_iter.sh TAG "CALLS" "CFGS"
TAG=$1; CALLS=${2:-"enc[3] fwd[3] enc[1]"}; CFGS=${3:-"mnist celeba"}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_direct.py -m gpu -x -q -p no:cacheprovider --timeout 120 \
  --timeout-method thread > gpurun_out/direct_${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/direct_${TAG}_tests.txt; exit 1; }
tail -1 gpurun_out/direct_${TAG}_tests.txt
CVHIP_LIB=scratch/libclearvae_stamps.so timeout -k 10 200 python tools/stamps_direct.py mnist $CALLS \
  > gpurun_out/stamps_${TAG}.txt 2>&1 || { tail -20 gpurun_out/stamps_${TAG}.txt; exit 1; }
python - gpurun_out/stamps_${TAG}.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d = json.loads(l); r = d["runs"][-1]
    print(d["call"], d["name"], "wgs", r["wgs"], "span", r["span_us"],
          " ".join(f"{k[:-2]}={v[1]}" for k, v in r.items() if k.endswith("_q")))
PY
bash tools/ktables.sh $TAG "$CFGS" -
