#!/bin/bash
# HBM traffic of one step-program call: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes
# usage: tools/pmc_traffic.sh <config> <full call label, e.g. 'enc[4]:cv_conv_backward_data'>
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
cfg=$1; label=$2; call=${label%%:*}
d=gpurun_out/pmc_${cfg}_${call//[\[\]]/_}
rm -rf "$d"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$d/fetch" -o run -- \
  python bench.py --config "$cfg" --only-call "$call" --reps 50 --warmup 5 --no-cpu-baseline --no-kernel-pass
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$d/write" -o run -- \
  python bench.py --config "$cfg" --only-call "$call" --reps 50 --warmup 5 --no-cpu-baseline --no-kernel-pass
[ -f "gpurun_out/${cfg}_traffic.json" ] || { [ -f "profiles/${cfg}_traffic.json" ] && cp "profiles/${cfg}_traffic.json" gpurun_out/; } || true
python profiles/pmc_traffic.py "$d" "$label" call 50 "gpurun_out/${cfg}_traffic.json"
