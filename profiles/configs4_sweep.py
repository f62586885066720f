#!/usr/bin/env python3
"""BASELINE configs[4] (P256 A64, half-sync m7 / m11 / m12, -c 1..8) on ONE MI355X at the
largest -d it holds (8 MiB: 128 GiB SEND + 128 GiB RECV; one allocation reused across the
sweep).  Per (method, c): every byte verified on the device, then the reference's report
quantities -- max over all 256 logical ranks of total time (median of 3 timed runs) -- and the
aggregate GB/s = P*A*d / max total time.  usage: configs4_sweep.py [d]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
P, A = 256, 64
d = int(sys.argv[1]) if len(sys.argv) > 1 else 8 << 20
rl = xg.aggregator_list(P, A)
ctx = xg.Context(0, 1, device=0)
R = xg.Regions(ctx, [P * A * d, P * A * d, 0, 0, 0])
print("P%d A%d -d %d on one MI355X: method, -c, steps, engine, max total time (s), aggregate GB/s, bad slots" % (P, A, d))
for c in range(1, 9):
    for m in (7, 11, 12):
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
        run = xg.MethodRun(ctx, s, it=0, mode=0, regions=R)
        tot = []
        for _ in range(3):
            done, post, _w = run.run_timed()
            tot.append(max(s.rank_timer(q, done, post).total_time for q in range(P)))
        _chk, bad, _f = run.verify()
        t = sorted(tot)[1]
        print("m%-2d c%d steps %4d engine %3d  max total %.6f s  %8.1f GB/s  bad %d" % (
            m, c, s.nsteps, run.engine_workgroups, t, P * A * d / t / 1e9, sum(1 for b in bad if b)), flush=True)
        run.close()
R.close()
ctx.close()
