"""MFMA utilisation of one step-program call from one rocprofv3 pass (tools/pmc_mfma.sh):
SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over the SIMDs (MI355X_MICROARCH.md: = 32 x N_mfma for
a 32-cycle MFMA), GRBM_GUI_ACTIVE the active cycles summed over the 8 XCDs, so

    utilisation = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)

per repetition of the call (its K kernels summed), median over the last `reps` repetitions.

    python profiles/pmc_mfma.py <dir> <label> <reps>
"""
import csv
import glob
import json
import statistics
import sys


def main():
    d, label, reps = sys.argv[1], sys.argv[2], int(sys.argv[3])
    rows = []
    for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(path)))
    by = {}
    for r in rows:
        k = int(r["Dispatch_Id"])
        e = by.setdefault(k, {"kernel": r["Kernel_Name"]})
        e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ids = sorted(by)
    seq = [by[i]["kernel"] for i in ids]
    # the call's K kernels per repetition (the period of the dispatch tail); each repetition summed
    for k in range(1, 9):
        tail = seq[-k * reps:]
        if len(tail) == k * reps and all(tail[i] == tail[i % k] for i in range(len(tail))):
            break
    else:
        raise SystemExit("no periodic tail of call dispatches")
    tail_ids = ids[-k * reps:]
    sel = []
    for r in range(reps):
        grp = [by[i] for i in tail_ids[r * k:(r + 1) * k]]
        sel.append({c: sum(e[c] for e in grp) for c in ("SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")})
    util = [e["SQ_VALU_MFMA_BUSY_CYCLES"] / (e["GRBM_GUI_ACTIVE"] / 8 * 1024) for e in sel]
    print(json.dumps({label: {"kernels": seq[-k:], "dispatches": len(sel), "mfma_util_median": statistics.median(util),
                              "mfma_busy_median": statistics.median(e["SQ_VALU_MFMA_BUSY_CYCLES"] for e in sel),
                              "grbm_gui_active_median": statistics.median(e["GRBM_GUI_ACTIVE"] for e in sel)}}))


if __name__ == "__main__":
    main()
