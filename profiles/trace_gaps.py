#!/usr/bin/env python3
"""Per-launch duration and the gap to the next launch of one kernel, from a
rocprofv3 --kernel-trace CSV (run_kernel_trace.csv): the device time between two
back-to-back launches on one stream (dispatch + cache write-back/invalidate at
the kernel boundary).  usage: trace_gaps.py <run_kernel_trace.csv> [name substring]"""
import csv
import statistics as S
import sys


def main(path, sub="copy_kernel"):
    rows = [r for r in csv.DictReader(open(path)) if sub in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    gaps = []
    for a, b in zip(rows, rows[1:]):
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        if 0 <= g < 50:            # back-to-back launches (not across host phases)
            gaps.append(g)
    names = sorted({r["Kernel_Name"] for r in rows})
    print("kernel(s): %s" % "; ".join(names))
    print("launches %d  duration us: mean %.2f median %.2f min %.2f max %.2f" %
          (len(dur), S.mean(dur), S.median(dur), min(dur), max(dur)))
    if gaps:
        print("back-to-back gaps %d  us: mean %.2f median %.2f min %.2f max %.2f" %
              (len(gaps), S.mean(gaps), S.median(gaps), min(gaps), max(gaps)))


if __name__ == "__main__":
    main(*sys.argv[1:3])
