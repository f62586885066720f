#!/usr/bin/env python3
"""configs[4]'s GPU-0 share (profiles/configs4_share.py, one (method, -c) cell, REPS runs) under
rocprofv3 --kernel-trace: split each run's device time into kernel time and the gaps between
consecutive launches, per launch class.  With the PMC passes (FETCH_SIZE, WRITE_SIZE; separate
runs) the HBM bytes of the copy launches against their algorithmic bytes.
usage: share_trace_summary.py <kernel_trace.csv> <reps> [fetch_counter.csv write_counter.csv]"""
import collections
import csv
import sys


def launches(path):
    rows = []
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("xgk::", "")
        wg = int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, wg))
    rows.sort()
    return rows


def main(trace, reps, fetch=None, write=None):
    rows = [x for x in launches(trace) if "copy_kernel" in x[2] or "clock_kernel" in x[2] or "engine" in x[2]]
    reps = int(reps)
    per_run = len(rows) // reps
    print("launches in the trace: %d (%d runs of %d)" % (len(rows), reps, per_run))
    for k in range(reps):
        run = rows[k * per_run:(k + 1) * per_run]
        span = (run[-1][1] - run[0][0]) / 1e3
        busy = sum(e - s for s, e, _n, _w in run) / 1e3
        gaps = [(run[i + 1][0] - run[i][1]) / 1e3 for i in range(len(run) - 1)]
        gaps.sort()
        print("run %d: first launch start -> last launch end %.1f us; kernels %.1f us (%.1f %%); gaps %.1f us "
              "(median %.2f, max %.2f us over %d boundaries)" % (k, span, busy, 100 * busy / span, sum(gaps),
                                                                  gaps[len(gaps) // 2] if gaps else 0,
                                                                  gaps[-1] if gaps else 0, len(gaps)))
    by = collections.defaultdict(list)
    for s, e, n, w in rows:
        by[(n, w)].append((e - s) / 1e3)
    print("%-34s %10s %8s %10s %10s" % ("kernel", "workgroups", "launches", "median_us", "mean_us"))
    for (n, w), ds in sorted(by.items()):
        ds.sort()
        print("%-34s %10d %8d %10.2f %10.2f" % (n, w, len(ds), ds[len(ds) // 2], sum(ds) / len(ds)))
    if fetch and write:
        f = sum(float(r["Counter_Value"]) for r in csv.DictReader(open(fetch))
                if r["Counter_Name"] == "FETCH_SIZE" and "copy_kernel" in r["Kernel_Name"])
        w = sum(float(r["Counter_Value"]) for r in csv.DictReader(open(write))
                if r["Counter_Name"] == "WRITE_SIZE" and "copy_kernel" in r["Kernel_Name"])
        print("PMC over the profiled run(s), copy kernels: read 2 x FETCH_SIZE = %.3f GiB, WRITE_SIZE = %.3f GiB "
              "(gfx950 wide-stream correction on FETCH_SIZE, MI355X_MICROARCH.md)" % (2 * f * 1024 / 2 ** 30,
                                                                                   w * 1024 / 2 ** 30))


if __name__ == "__main__":
    main(*sys.argv[1:])
