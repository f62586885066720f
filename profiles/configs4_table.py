#!/usr/bin/env python3
"""configs[4] side by side: the HIP path at -d 8 MiB on one MI355X (configs4_sweep.py output) and
the reference under MPICH (configs4_ref.py outputs) at reduced -d, per (method, -c), with the
aggregate GB/s each implies (P*A*d / max total time).  Every one of the 24 cells has a
reference figure or says it did not finish.
usage: configs4_table.py <gpu.txt> <ref_a.txt> [ref_b.txt ...]"""
import re
import sys

P, A = 256, 64
gpu = {}
for line in open(sys.argv[1]):
    g = re.match(r"m(\d+)\s+c(\d) steps\s+(\d+).*max total ([0-9.]+) s\s+([0-9.]+) GB/s\s+bad (\d+)", line)
    if g:
        gpu[(int(g.group(1)), int(g.group(2)))] = (float(g.group(4)), float(g.group(5)), int(g.group(6)), int(g.group(3)))
refs = []
for path in sys.argv[2:]:
    cells, head, d = {}, "", None
    for line in open(path):
        if line.startswith("#"):
            head = line.strip("# \n")
            continue
        g = re.match(r"m(\d+) c(\d) d(\d+): (.*)", line)
        if not g:
            continue
        d = int(g.group(3))
        t = re.search(r"max total time = ([0-9.]+)", g.group(4))
        cells[(int(g.group(1)), int(g.group(2)))] = float(t.group(1)) if t else None
    refs.append((path, head, d, cells))
print("# configs[4] (P256 A64, half-sync m7 / m11 / m12, -c 1..8): max total time (s) and aggregate GB/s")
print("# HIP path: %s (one MI355X, -d 8 MiB = the largest -d one GPU holds, every byte verified)" % sys.argv[1])
for path, head, d, _ in refs:
    print("# reference -d %d: %s -- %s" % (d, path, head))
hdr = "%-4s %-3s %22s" % ("m", "-c", "HIP -d 8MiB s / GB/s")
for _p, _h, d, _c in refs:
    hdr += " %24s" % ("ref -d %d s / GB/s" % d)
print(hdr)
for c in range(1, 9):
    for m in (7, 11, 12):
        t, gbs, bad, _st = gpu.get((m, c), (float("nan"), float("nan"), -1, 0))
        row = "m%-3d c%-2d %10.6f / %8.1f" % (m, c, t, gbs)
        for _p, _h, d, cells in refs:
            v = cells.get((m, c), "missing")
            if v is None:
                row += " %24s" % "did not finish"
            elif v == "missing":
                row += " %24s" % "not run"
            else:
                row += " %12.3f / %9.4f" % (v, P * A * d / v / 1e9)
        print(row + ("" if bad == 0 else "  BAD %d" % bad))
