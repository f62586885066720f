#!/usr/bin/env python3
"""Tabulate profiles/chain_modes.sh output: per method label and experiment, the median over
repetitions of the CLI's 'max total time' in each mode, the reference's beside it, and the
ratio of the default mode (the first present: launch, then the round-2 solo_armed) to the
reference.  usage: chain_summary.py <outdir>"""
import glob
import os
import re
import statistics as S
import sys


def parse(path):
    out = []   # [(label, t)] in print order; -i 2 prints every label twice
    for line in open(path):
        m = re.match(r"\| (.*) max total time = ([0-9.]+)", line)
        if m:
            out.append((m.group(1).strip(), float(m.group(2))))
    return out


def main(d):
    modes = [m for m in ["launch", "armed", "grid_launch", "copy1", "graph", "nograph", "solo_armed", "solo1_armed", "grid_armed",
                         "solo_launch"] if glob.glob(os.path.join(d, m + "_*.txt"))]
    runs = {m: [parse(f) for f in sorted(glob.glob(os.path.join(d, m + "_*.txt")))] for m in modes}
    refs = [parse(f) for f in sorted(glob.glob(os.path.join(d, "ref*.txt")))]   # ref.txt or ref_<r>.txt
    base = runs[modes[0]][0]
    print(("%-36s %4s" + " %11s" * len(modes) + " %10s %7s") % ("method", "exp", *modes, "reference", "ratio"))
    seen = {}
    for i, (lab, _t) in enumerate(base):
        e = seen.get(lab, 0)
        seen[lab] = e + 1
        med = [S.median(r[i][1] for r in runs[m]) * 1e6 for m in modes]
        rv = []
        for ref in refs:
            rf = [t for (l, t) in ref if l == lab]
            if e < len(rf):
                rv.append(rf[e] * 1e6)
        rv = S.median(rv) if rv else float("nan")
        print(("%-36s %4d" + " %11.1f" * len(modes) + " %10.1f %7.2f") % (lab, e, *med, rv, med[0] / rv))
    print("(us, median over %d repetitions, reference median over %d runs; ratio = %s / reference)"
          % (len(runs[modes[0]]), len(refs), modes[0]))


if __name__ == "__main__":
    main(sys.argv[1])
