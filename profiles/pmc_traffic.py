"""HBM traffic per launch of one step-program call from rocprofv3 PMC passes (MI355X_MICROARCH.md,
"HBM"): FETCH_SIZE and WRITE_SIZE are collected in SEPARATE passes (they do not fit one TCC pass),
each run as

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir>/fetch -o run -- \
        python bench.py --only-call 'enc[4]' --reps 50 --warmup 5 --no-cpu-baseline --no-kernel-pass
    rocprofv3 --pmc WRITE_SIZE ... -d <dir>/write ...

FETCH_SIZE is in KiB and on gfx950 counts half the bytes of 16-B-per-lane streaming reads (128-B
requests tallied at 64 B), so it is doubled; WRITE_SIZE (KiB) is exact for 16-B stores and float
atomics.  The per-launch figure is the median over the last --reps dispatches of the call's dominant
kernel (the warmup steps dispatch the same kernel for other layers first).

    python profiles/pmc_traffic.py <dir> 'enc[4]:cv_conv_backward_data' <kernel-name-substring|auto> <reps> <out.json>

(merges into out.json, keyed by the bench's full call label "program[index]:c_function", so a stale entry
from an older program layout is never matched).  `auto`: the kernel of the trace's last dispatch — in
--only-call mode the last --reps dispatches are the call's own launches.  `call`: every kernel the call
launches, summed per repetition (the unit the bench's roofline prices).
"""

import csv
import glob
import json
import statistics
import sys


def per_dispatch(path_glob, counter, kernel_sub):
    vals = {}
    for path in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != counter or kernel_sub not in r.get("Kernel_Name", ""):
                continue
            d = int(r["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def per_call(path_glob, counter, reps):
    """`call` mode: a call that launches K kernels per repetition (e.g. the direct backward-data + the deferred
    weight gradient of cv_conv_backward_deferred_kpack) — the period K of the last dispatches' kernel names,
    the counter summed over each repetition's K dispatches; (per-repetition sums, kernel names of one period)."""
    vals, names = {}, {}
    for path in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get("Counter_Name") != counter:
                continue
            d = int(r["Dispatch_Id"])
            vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
    ids = sorted(vals)
    seq = [names[i] for i in ids]
    for k in range(1, 9):
        tail = seq[-k * reps:]
        if len(tail) == k * reps and all(tail[i] == tail[i % k] for i in range(len(tail))):
            break
    else:
        raise SystemExit("no periodic tail of call dispatches")
    v = [vals[i] for i in ids[-k * reps:]]
    return [sum(v[r * k:(r + 1) * k]) for r in range(reps)], seq[-k:]


def main():
    d, call, ksub, reps, out = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), sys.argv[5]
    if ksub == "call":
        fetch, kn = per_call(f"{d}/fetch/**/*counter_collection.csv", "FETCH_SIZE", reps)
        write, _ = per_call(f"{d}/write/**/*counter_collection.csv", "WRITE_SIZE", reps)
        f_kib, w_kib = statistics.median(fetch), statistics.median(write)
        rec = {"kernels": kn, "dispatches_per_call": len(kn), "fetch_size_kib_median": f_kib,
               "write_size_kib_median": w_kib, "traffic_bytes": 2 * f_kib * 1024 + w_kib * 1024}
        try:
            db = json.load(open(out))
        except (OSError, ValueError):
            db = {"note": "per launch: traffic = 2*FETCH_SIZE (gfx950 16B-load correction) + WRITE_SIZE", "calls": {}}
        db["calls"][call] = rec
        json.dump(db, open(out, "w"), indent=1)
        print(json.dumps({call: rec}))
        return
    if ksub == "auto":
        last = (-1, None)
        for path in glob.glob(f"{d}/fetch/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(path)):
                if int(r["Dispatch_Id"]) > last[0]:
                    last = (int(r["Dispatch_Id"]), r["Kernel_Name"])
        ksub = last[1]
        if ksub is None:
            raise SystemExit(f"no dispatches under {d}")
    fetch = per_dispatch(f"{d}/fetch/**/*counter_collection.csv", "FETCH_SIZE", ksub)[-reps:]
    write = per_dispatch(f"{d}/write/**/*counter_collection.csv", "WRITE_SIZE", ksub)[-reps:]
    if not fetch or not write:
        raise SystemExit(f"no dispatches of {ksub!r} found under {d}")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    rec = {"kernel": ksub, "dispatches": [len(fetch), len(write)],
           "fetch_size_kib_median": f_kib, "write_size_kib_median": w_kib,
           "traffic_bytes": 2 * f_kib * 1024 + w_kib * 1024}
    try:
        db = json.load(open(out))
    except (OSError, ValueError):
        db = {"note": "per launch: traffic = 2*FETCH_SIZE (gfx950 16B-load correction) + WRITE_SIZE", "calls": {}}
    db["calls"][call] = rec
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps({call: rec}))


if __name__ == "__main__":
    main()
