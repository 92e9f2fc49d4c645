"""Timeline of one replayed step from a rocprofv3 kernel trace (profiling aid, reads only the CSV).

usage: python tools/step_timeline.py run_kernel_trace.csv [first-kernel-substring] [step index from the end]

A step starts at each dispatch whose name contains the first-kernel substring (default: the step-start pack launch).
Prints every dispatch of the chosen step: start offset, duration, end offset, queue, short name; then the busy union
of the step (time with at least one kernel running) against its wall span, and the gaps longer than 3 us."""

import csv
import sys


def main():
    path = sys.argv[1]
    first = sys.argv[2] if len(sys.argv) > 2 else "pack"
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if first in r[3]]
    if len(starts) < back + 1:
        print("not enough steps", len(starts))
        return
    a, b = starts[-back - 1], starts[-back]
    step = rows[a:b]
    t0 = step[0][0]
    for s, e, q, name in step:
        short = name.split("(")[0]
        if len(short) > 90:
            short = short[:90]
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} {(e - t0) / 1e3:9.1f}  q{q}  {short}")
    # busy union
    iv = sorted((s, e) for s, e, _, _ in step)
    busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
    for s, e in iv[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            if s - cur_e > 3000:
                gaps.append(((cur_e - t0) / 1e3, (s - cur_e) / 1e3))
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[b][0] - t0
    print(f"step span {span / 1e3:.1f} us, busy union {busy / 1e3:.1f} us, kernels {len(step)}")
    for at, g in gaps:
        print(f"  gap {g:6.1f} us at {at:8.1f}")


if __name__ == "__main__":
    main()
