"""Armed solo engine under repetition: the README-config chains (m6, m9, m12) run 2000 times
each on the default rails, every run checked for a timed-out rail (xg_plan_check inside
run_timed) and the bytes verified at the end; prints the spread of the run times."""
import os
import statistics as S
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as G

xg = G.load_package().xg
P, A, d, c = 32, 14, 2048, 3
N = int(os.environ.get("REPS", "2000"))
rl = xg.aggregator_list(P, A)
ctx = xg.Context(0, 1, device=0)
for m in (6, 9, 12):
    s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
    run = xg.MethodRun(ctx, s, it=0, mode=1)
    t0, walls = time.time(), []
    for i in range(N):
        done, _post, wall = run.run_timed()
        walls.append(done[-1])
        if time.time() - t0 > 60:
            break
    _chk, bad, _f = run.verify()
    nbad = sum(1 for b in bad if b)
    walls.sort()
    print("m%d runs %d  bad slots %d  total us: min %.1f median %.1f p99 %.1f max %.1f" % (
        m, len(walls), nbad, walls[0] * 1e6, S.median(walls) * 1e6, walls[int(0.99 * (len(walls) - 1))] * 1e6,
        walls[-1] * 1e6), flush=True)
    run.close()
    if nbad:
        sys.exit(1)
ctx.close()
