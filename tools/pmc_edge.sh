#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, SQ occupancy) of the edge-kernel calls (<= 4 image-side channels)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in mnist celeba-mim; do
  timeout -k 5 150 python tools/list_calls.py $cfg > gpurun_out/calls_$cfg.txt 2>/dev/null
done
cat gpurun_out/calls_*.txt
# edge calls: image-side conv geometry (c_in or c_out <= 4); celeba-mim: the forward ones only
python - > gpurun_out/edge_calls.txt <<'PY'
import re
for cfg in ("mnist", "celeba-mim"):
    for ln in open(f"gpurun_out/calls_{cfg}.txt"):
        m = re.search(r"n=\d+ (\d+)x\d+ -> (\d+)x\d+", ln)
        if not m or min(int(m.group(1)), int(m.group(2))) > 4:
            continue
        lab = ln.split()[1]
        if cfg == "celeba-mim" and not lab.startswith("fwd"):
            continue
        print(cfg, lab)
PY
cat gpurun_out/edge_calls.txt
while read cfg label; do
  call=${label%%:*}
  echo "== $cfg $label"
  bash tools/pmc_traffic.sh $cfg "$label" > gpurun_out/pmc_edge_${cfg}_${call//[\[\]]/_}.log 2>&1 || { echo failed; tail -3 gpurun_out/pmc_edge_${cfg}_${call//[\[\]]/_}.log; exit 1; }
  D=gpurun_out/pmc_sq/${cfg}_$(echo $call | tr -d '[]')
  mkdir -p $D
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d $D -o run -- python3 bench.py --config $cfg --only-call "$call" --reps 20 --warmup 3 --no-cpu-baseline --no-kernel-pass > $D/log.txt 2>&1 || { echo "sq pmc $call failed"; tail -5 $D/log.txt; exit 1; }
done < gpurun_out/edge_calls.txt
echo ALLDONE
