#!/bin/bash
# scatter band-rows sweep: isolated time of the scatter call for several CV_EDGE_SCATTER_RB
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg_call in "celeba-mim fwd[14]" "mnist fwd[10]" "camelyon-bf16 fwd[14]"; do
  set -- $cfg_call
  for rb in 0 2 3 4 5 6 7 9 15; do
    D=gpurun_out/sweep/${1}_rb$rb
    mkdir -p $D
    CV_EDGE_SCATTER_RB=$rb timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $D -o run -- python3 bench.py --config $1 --only-call "$2" --reps 30 --warmup 3 --no-cpu-baseline --no-kernel-pass > $D/log.txt 2>&1 || { echo fail $D; tail -3 $D/log.txt; exit 1; }
    python3 - "$D" <<'PY'
import csv, glob, sys
for p in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "edge_scatter" in r["Name"]:
            print(sys.argv[1], r["Name"][:45], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2))
PY
  done
done
