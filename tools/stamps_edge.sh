cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for spec in "mnist @edge" "celeba @edge"; do
  set -- $spec
  CVHIP_LIB=scratch/libclearvae_stamps.so timeout -k 10 200 python tools/stamps_direct.py $1 "$2" > gpurun_out/stamps_edge_$1.txt 2>&1 || { tail -20 gpurun_out/stamps_edge_$1.txt; exit 1; }
  python - gpurun_out/stamps_edge_$1.txt <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if not l.startswith("{"): continue
    d = json.loads(l); r = d["runs"][-1]
    print(d["call"], d["name"], "wgs", r["wgs"], "span", r["span_us"], " ".join(f"{k[:-2]}={v}" for k, v in r.items() if k.endswith("_q")))
PY
done
