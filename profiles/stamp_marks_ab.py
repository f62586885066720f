#!/usr/bin/env python3
"""A/B (round 4): a step boundary of an eager run marked by a timing event (the default) or by a
one-lane clock kernel stamp (XG_STAMP_MARKS=1, the form graph replays use).  Multi-step plans whose
steps are not chained: GPU 0's local-only share of 8-GPU jobs (cross-GPU steps: fork / join + the
step mark) and one-GPU plans outside the engine and graphs.  Per cell, interleaved A/B, the device
time of the run (done[-1]) and the host wall time, min over REPS; every run verified.
usage: python3 profiles/stamp_marks_ab.py
The A/B ran at a build that read XG_STAMP_MARKS (profiles/r04/stamp_marks/ab.txt); stamps then
became the only step mark and the knob was removed, so at HEAD both columns are stamps
(profiles/r04/stamp_marks/after.txt: the same cells, a check that nothing regressed)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["XG_SELF_MAX"] = "0"
os.environ["XG_GRAPH"] = "0"
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
REPS = int(os.environ.get("REPS", "5"))
# (label, G, method, P, A, d, c)
CELLS = [("configs[3] m9 share", 8, 9, 256, 32, 4 << 20, 200000000),
         ("configs[3] m10 share", 8, 10, 256, 32, 4 << 20, 200000000),
         ("configs[4] m12 -c 8 share d1M", 8, 12, 256, 64, 1 << 20, 8),
         ("configs[4] m11 -c 1 share d1M", 8, 11, 256, 64, 1 << 20, 1),
         ("README m3 share", 8, 3, 32, 14, 2048, 3),
         ("README m6 share", 8, 6, 32, 14, 2048, 3),
         ("README m7 share", 8, 7, 32, 14, 2048, 3),
         ("P64 A16 256K m9 1gpu", 1, 9, 64, 16, 256 << 10, 200000000),
         ("P256 A64 1M m12 -c 8 1gpu", 1, 12, 256, 64, 1 << 20, 8)]
ctxs = {}
for label, g, m, P, A, d, c in CELLS:
    if g not in ctxs:
        ctxs[g] = xg.Context.virtual(0, g, device=0) if g > 1 else xg.Context(rank=0, nranks=1, device=0)
    ctx = ctxs[g]
    s = xg.Schedule(m, P, A, d, c, xg.aggregator_list(P, A), ntimes=1)
    run = xg.MethodRun(ctx, s, it=0, mode=0)
    try:
        if g > 1:
            run.set_local_only()
        best = {0: [1e9, 1e9], 1: [1e9, 1e9]}
        for _ in range(REPS):
            for mk in (0, 1):
                os.environ["XG_STAMP_MARKS"] = str(mk)
                done, _post, wall = run.run_timed()
                best[mk] = [min(best[mk][0], done[-1]), min(best[mk][1], wall)]
        os.environ["XG_STAMP_MARKS"] = "0"
        _chk, bad, _f = run.verify()
        lo, hi = s.block_range(g, 0)
        if g == 1:
            assert not any(bad)
        print("%-30s G%d steps=%-4d launches=%-4d events: dev %8.1f us wall %8.1f us | stamps: dev %8.1f us wall %8.1f us"
              % (label, g, s.nsteps, run.launches, best[0][0] * 1e6, best[0][1] * 1e6, best[1][0] * 1e6, best[1][1] * 1e6),
              flush=True)
    finally:
        run.close()
for c in ctxs.values():
    c.close()
print("stamp_marks_ab ok", flush=True)
