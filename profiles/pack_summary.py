#!/usr/bin/env python3
# HISTORICAL RECIPE: it sets XG_* knobs folded into constants by commit 88b890f (round 4);
# rerun now, those arms are identical (libxg warns about each such variable).  Kept as the record.
"""Reduce a rocprofv3 kernel trace of profiles/pack_virtual.py to copy-kernel HBM GB/s per
launch size class.  Every transfer there is a whole number of 32 KiB pieces (256 KiB
segments), one workgroup per piece, so a launch of W workgroups moves W * 32 KiB and reads +
writes 2 * W * 32 KiB -- unless the launch is too small for 2 x CUs workgroups of 32 KiB, which
then get smaller pieces (round 3): pass those classes as "W=bytes,..." (e.g. 512=4194304).
usage: pack_summary.py <run_kernel_trace.csv> [W=bytes,...]"""
import collections
import csv
import os
import sys

CHUNK = int(os.environ.get("XG_COPY_CHUNK", "32768"))
CLASSES = dict(tuple(map(int, kv.split("="))) for kv in sys.argv[2].split(",")) if len(sys.argv) > 2 else {}
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "copy_kernel" in r["Kernel_Name"]]
by = collections.defaultdict(list)
for r in rows:
    wg = int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"])
    by[wg].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
print("workgroups  bytes_moved  launches  avg_us  HBM_GBps(read+write)")
for wg, ds in sorted(by.items()):
    avg = sum(ds) / len(ds)
    nb = CLASSES.get(wg, wg * CHUNK)
    print("%10d  %11d  %8d  %6.2f  %8.1f" % (wg, nb, len(ds), avg / 1e3, 2.0 * nb / avg))
