#!/usr/bin/env python3
"""A/B (round 4): a timed run marking every step vs only the steps a Timer reads
(xg_sched_timed_steps -> xg_plan_set_step_marks, the default since).  Same cells as
stamp_marks_ab.py: GPU 0's local-only share of 8-GPU plans and one-GPU plans; per cell,
interleaved, min over REPS of the device time of the run (done[-1]) and the host wall time, and
the max total time of the reference's report over GPU 0's ranks (must not grow).
usage: python3 profiles/timed_steps_ab.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
os.environ["XG_SELF_MAX"] = "0"
os.environ["XG_GRAPH"] = "0"
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
REPS = int(os.environ.get("REPS", "5"))
CELLS = [("configs[3] m9 share", 8, 9, 256, 32, 4 << 20, 200000000),
         ("configs[3] m10 share", 8, 10, 256, 32, 4 << 20, 200000000),
         ("configs[4] m12 -c 8 share d1M", 8, 12, 256, 64, 1 << 20, 8),
         ("configs[4] m11 -c 1 share d1M", 8, 11, 256, 64, 1 << 20, 1),
         ("README m6 share", 8, 6, 32, 14, 2048, 3),
         ("README m12 share", 8, 12, 32, 14, 2048, 3),
         ("README m9 share", 8, 9, 32, 14, 2048, 3)]
ctxs = {}
for label, g, m, P, A, d, c in CELLS:
    if g not in ctxs:
        ctxs[g] = xg.Context.virtual(0, g, device=0) if g > 1 else xg.Context(rank=0, nranks=1, device=0)
    ctx = ctxs[g]
    s = xg.Schedule(m, P, A, d, c, xg.aggregator_list(P, A), ntimes=1)
    need = s.timed_steps()
    lo, hi = s.block_range(g, 0)
    run = xg.MethodRun(ctx, s, it=0, mode=0)
    try:
        if g > 1:
            run.set_local_only()
        best = {}
        for _ in range(REPS):
            for name, mk in (("all", None), ("read", need)):
                run.set_step_marks(mk)
                done, post, wall = run.run_timed()
                tmax = max(s.rank_timer(q, done, post, g).total_time for q in range(lo, hi))
                b = best.setdefault(name, [1e9, 1e9, 1e9])
                best[name] = [min(b[0], done[-1]), min(b[1], wall), min(b[2], tmax)]
        print("%-30s G%d steps=%-4d marked=%-4d | every step: dev %8.1f us wall %8.1f us total %8.1f us"
              " | read steps: dev %8.1f us wall %8.1f us total %8.1f us"
              % (label, g, s.nsteps, sum(need), *[x * 1e6 for x in best["all"]], *[x * 1e6 for x in best["read"]]),
              flush=True)
    finally:
        run.close()
for c in ctxs.values():
    c.close()
print("timed_steps_ab ok", flush=True)
