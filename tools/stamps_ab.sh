cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in stamps stamps_nsl6; do
  CVHIP_LIB=scratch/libclearvae_$v.so timeout -k 10 200 python tools/stamps_direct.py mnist "enc[3]" "enc[1]" > gpurun_out/stamps_$v.txt 2>&1 || { tail -20 gpurun_out/stamps_$v.txt; exit 1; }
  echo "== $v"
  python - gpurun_out/stamps_$v.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d = json.loads(l); r = d["runs"][-1]
    print(d["call"], d["name"], "wgs", r["wgs"], "span", r["span_us"],
          " ".join(f"{k[:-2]}={v[1]}" for k, v in r.items() if k.endswith("_q")))
PY
done
