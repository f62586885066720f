"""Per-method copy-launch durations of a bench run from a rocprofv3 kernel trace: the timed
region's launches cycle through methods 1..4 (one launch each per step), so launch i of the
back-to-back run belongs to method (i mod 4) + 1.  usage: bench_per_method.py <run_kernel_trace.csv>"""
import csv
import statistics as S
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1])) if "copy_kernel" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 4*K launches are the timed region (K steps); take the final 80
tail = rows[-80:]
for m in range(4):
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in tail[m::4]]
    print("method %d: launches %d  mean %.1f us  median %.1f  min %.1f  max %.1f  -> %.0f GB/s of traffic"
          % (m + 1, len(d), S.mean(d), S.median(d), min(d), max(d), 939524096 / S.median(d) / 1e3))
