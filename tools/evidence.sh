#!/bin/bash
# Round evidence on one box: the default bench line, the rocprofv3 kernel summaries of every bench config, the PMC
# HBM traffic and MFMA utilisation of every key's priced call, and the SQ instruction mix of the MNIST direct
# backward-data call against the GEMM core.   tools/evidence.sh TAG [parts: bench trace pmc sq]
TAG=$1; shift
PARTS=${@:-bench trace pmc sq}
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ev_$TAG
O=gpurun_out/ev_$TAG
for part in $PARTS; do
case $part in
bench)
  timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  tail -c 600 $O/bench.json; echo
  ;;
trace)
  for cfg in mnist celeba-mim celeba pacs camelyon-bf16 camelyon-fp32; do
    steps=50; [ $cfg = celeba-mim ] && steps=30
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$cfg -o run -- \
      python3 bench.py --config $cfg --steps $steps --warmup 10 --no-cpu-baseline --no-c3 --no-kernel-pass \
      > $O/trace_$cfg.log 2>&1 || { tail -5 $O/trace_$cfg.log; exit 1; }
    echo "trace $cfg done"
  done
  ;;
pmc)
  # every key's priced call, from this tag's bench line
  python - $O/bench.json > $O/priced.txt <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = [("mnist", d), ("celeba-mim", d.get("c3") or {}), ("celeba", d.get("celeba") or {}),
        ("pacs", d.get("pacs") or {}), ("camelyon-bf16", d.get("camelyon_bf16") or {}),
        ("camelyon-fp32", d.get("camelyon_fp32") or {})]
for cfg, e in keys:
    r = e.get("roofline") or {}
    if r.get("kernel"):
        print(cfg, r["kernel"])
PY
  cat $O/priced.txt
  while read cfg label; do
    call=${label%%:*}
    bash tools/pmc_traffic.sh $cfg "$label" > $O/pmct_${cfg}.log 2>&1 || { tail -5 $O/pmct_${cfg}.log; exit 1; }
    tail -1 $O/pmct_${cfg}.log
    bash tools/pmc_mfma.sh $cfg "$call" > $O/mfma_${cfg}.log 2>&1 || { tail -5 $O/mfma_${cfg}.log; exit 1; }
    tail -1 $O/mfma_${cfg}.log
  done < $O/priced.txt
  ;;
sq)
  bash tools/pmc_sq2.sh mnist ${TAG}_direct "enc[3]" > $O/sq_direct.log 2>&1 || { tail -5 $O/sq_direct.log; exit 1; }
  CV_DIRECT=0 bash tools/pmc_sq2.sh mnist ${TAG}_core "enc[3]" > $O/sq_core.log 2>&1 || { tail -5 $O/sq_core.log; exit 1; }
  tail -1 $O/sq_direct.log; tail -1 $O/sq_core.log
  ;;
esac
done
echo EVIDENCE_DONE
