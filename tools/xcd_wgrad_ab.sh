cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
for v in 0 1; do
  d=gpurun_out/xcdw_$v
  rm -rf $d
  CV_XCD_WGRAD=$v timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o run -- python bench.py --config celeba --only-call "enc[1]" --reps 50 --warmup 5 --no-cpu-baseline --no-kernel-pass > $d.log 2>&1
  CV_XCD_WGRAD=$v timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o run -- python bench.py --config celeba --only-call "enc[1]" --reps 50 --warmup 5 --no-cpu-baseline --no-kernel-pass >> $d.log 2>&1
  python - $d <<'PY'
import csv, glob, statistics, sys
d = sys.argv[1]
for cnt, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
    vals, names = {}, {}
    for p in glob.glob(f"{d}/{sub}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] != cnt: continue
            i = int(r["Dispatch_Id"]); vals[i] = vals.get(i, 0) + float(r["Counter_Value"]); names[i] = r["Kernel_Name"]
    ids = sorted(vals)[-100:]
    by = {}
    for i in ids: by.setdefault(names[i][:60], []).append(vals[i])
    for k, v in by.items(): print(d, cnt, k, round(statistics.median(v) * (2 if cnt == "FETCH_SIZE" else 1) / 1024, 1), "MB")
PY
done
bash tools/ktables.sh xcdw "celeba celeba-mim" - CV_XCD_WGRAD=1 2>&1 || true
