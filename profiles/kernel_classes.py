#!/usr/bin/env python3
"""Reduce a rocprofv3 kernel trace to copy-kernel launch classes: per (kernel, grid size), the
number of launches and their median / mean duration.  usage: kernel_classes.py <run_kernel_trace.csv>"""
import collections
import csv
import sys

by = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"]
    if "copy_kernel" not in name:
        continue
    short = name.split("(")[0].replace("void ", "").replace("xgk::", "")
    wg = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    by[(short, wg)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print("%-28s %10s %8s %10s %10s" % ("kernel", "workgroups", "launches", "median_us", "mean_us"))
for (k, wg), ds in sorted(by.items()):
    ds.sort()
    print("%-28s %10d %8d %10.2f %10.2f" % (k, wg, len(ds), ds[len(ds) // 2], sum(ds) / len(ds)))
