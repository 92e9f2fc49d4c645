"""MFMA utilisation of one step-program call from one rocprofv3 pass (scratch/pmc_mfma.sh):
SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over the SIMDs (MI355X_MICROARCH.md: = 32 x N_mfma for
a 32-cycle MFMA), GRBM_GUI_ACTIVE the active cycles summed over the 8 XCDs, so

    utilisation = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)

per dispatch, median over the call's last `reps` dispatches (the kernel of the trace's last dispatch).

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
    kern = by[ids[-1]]["kernel"]
    sel = [by[i] for i in ids if by[i]["kernel"] == kern][-reps:]
    util = [e["SQ_VALU_MFMA_BUSY_CYCLES"] / (e["GRBM_GUI_ACTIVE"] / 8 * 1024) for e in sel]
    print(json.dumps({label: {"kernel": kern, "dispatches": len(sel), "mfma_util_median": statistics.median(util),
                              "mfma_busy_median": statistics.median(e["SQ_VALU_MFMA_BUSY_CYCLES"] for e in sel),
                              "grbm_gui_active_median": statistics.median(e["GRBM_GUI_ACTIVE"] for e in sel)}}))


if __name__ == "__main__":
    main()
