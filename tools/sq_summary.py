import csv, glob, statistics, sys
for D in sys.argv[1:]:
    vals = {}
    rows = []
    for p in glob.glob(D + "/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(p)))
    last = max(int(r["Dispatch_Id"]) for r in rows)
    kname = [r["Kernel_Name"] for r in rows if int(r["Dispatch_Id"]) == last][0]
    disp = sorted({int(r["Dispatch_Id"]) for r in rows if r["Kernel_Name"] == kname})[-10:]
    for c in {r["Counter_Name"] for r in rows}:
        xs = [sum(float(r["Counter_Value"]) for r in rows if r["Counter_Name"] == c and int(r["Dispatch_Id"]) == dd) for dd in disp]
        vals[c] = statistics.median(xs)
    dur = None
    for p in glob.glob(D + "/trace/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Name"] == kname:
                dur = float(r["AverageNs"]) / 1e3
    print(D, kname[:60], "avg_us", dur, {k: round(v) for k, v in sorted(vals.items())})
