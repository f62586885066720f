#!/usr/bin/env python3
"""Round 6: does a cross-GPU step's local part (the copy launch on the side stream) run while the
step's RCCL kernel runs?  Reads one rank's rocprofv3 kernel trace; per copy-kernel class (kernel,
grid, stream): launches, how many start inside an RCCL kernel's [start, end] on another stream, and
the share of their device time spent inside one.  usage: overlap_summary.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rccl = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]) for r in rows
              if "nccl" in r["Kernel_Name"].lower())
print("RCCL kernels: %d on streams %s" % (len(rccl), sorted({s for _a, _b, s in rccl})))
by = collections.defaultdict(lambda: [0, 0, 0.0, 0.0])
for r in rows:
    name = r["Kernel_Name"]
    if "copy_kernel" not in name:
        continue
    a, b, st = int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"]
    short = name.split("(")[0].replace("void ", "").replace("xgk::", "")
    wg = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    inside = 0
    starts_in = False
    for ra, rb, rs in rccl:
        if rs == st or rb <= a or ra >= b:
            continue
        inside += min(b, rb) - max(a, ra)
        starts_in |= ra <= a < rb
    k = by[(short, wg, st)]
    k[0] += 1
    k[1] += starts_in
    k[2] += (b - a) / 1e3
    k[3] += inside / 1e3
print("%-28s %6s %6s %8s %12s %10s %14s" % ("kernel", "wgs", "stream", "launches", "start_in_rccl", "device_us",
                                             "us_inside_rccl"))
for (k, wg, st), (n, si, us, ins) in sorted(by.items()):
    print("%-28s %6d %6s %8d %12d %10.1f %14.1f" % (k, wg, st, n, si, us, ins))
