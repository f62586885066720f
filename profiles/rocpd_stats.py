#!/usr/bin/env python3
"""Per-kernel summary (calls, total / mean / min / max ns) of a rocprofv3 rocpd database -- what
`--stats` writes as run_kernel_stats.csv when the output format is csv -- so a run recorded in the
default SQLite format yields the same table.  usage: rocpd_stats.py <run_results.db> [out.csv]"""
import collections
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute("select s.display_name, d.end - d.start from rocpd_kernel_dispatch d "
                  "join rocpd_info_kernel_symbol s on s.id = d.kernel_id").fetchall()
per = collections.defaultdict(list)
for name, ns in rows:
    per[name].append(ns)
out = ['"Name","Calls","TotalDurationNs","AverageNs","Percentage","MinNs","MaxNs"']
total = sum(sum(v) for v in per.values()) or 1
for name, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    out.append('"%s",%d,%d,%.1f,%.2f,%d,%d' % (name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / total,
                                               min(v), max(v)))
text = "\n".join(out) + "\n"
if len(sys.argv) > 2:
    open(sys.argv[2], "w").write(text)
print(text)
