#!/bin/bash
# direct-kernel stage-loop ablations (stamps build): none / no weight DMA / no MFMA / no fragment reads
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for d in 0 1 2 4 3 6; do
  CV_DIRECT_DBG=$d CVHIP_LIB=scratch/libclearvae_stamps.so timeout -k 10 200 python tools/stamps_direct.py mnist "enc[3]" "enc[1]" \
    > gpurun_out/stamps_dbg$d.txt 2>&1 || { tail -20 gpurun_out/stamps_dbg$d.txt; exit 1; }
  python - gpurun_out/stamps_dbg$d.txt $d <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d = json.loads(l); r = d["runs"][-1]
    print("dbg", sys.argv[2], d["call"], "span", r["span_us"], " ".join(f"{k[:-2]}={v[1]}" for k, v in r.items() if k.endswith("_q")))
PY
done
