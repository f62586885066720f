"""Theta-scale plans (P16384 A256 d2048, m1) on one MI355X under each execution form:
default (split solo launches / engine choice), grid engine (XG_ENGINE_SOLO=0), per-step
launch chains (XG_ENGINE_MAX_STEP=0).  usage: python3 profiles/theta_probe.py [c ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as G

xg = G.load_package().xg
P, A, d = 16384, 256, 2048
rl = xg.aggregator_list(P, A)
cs = [int(x) for x in sys.argv[1:]] or [8, 1]
for c in cs:
    s = xg.Schedule(1, P, A, d, c, rl, ntimes=1)
    for name, env in (("default", {}), ("grid", {"XG_ENGINE_SOLO": "0"}), ("chains", {"XG_ENGINE_MAX_STEP": "0"})):
        os.environ.update(env)
        cx = xg.Context(rank=0, nranks=1, device=0)
        for key in env:
            del os.environ[key]
        t0 = time.time()
        run = xg.MethodRun(cx, s, it=0, mode=0)
        tl = time.time() - t0
        n, nseg, nh = run.engine_steps()
        ts = []
        for _ in range(3):
            done, _post, wall = run.run_timed()
            ts.append(done[-1])
        _chk, bad, _f = run.verify()
        print("c %5d %-8s steps %5d engine steps %5d segments %3d rails %3d launches %5d load %.1f s  total %.3f ms "
              "(best of 3)  bad slots %d" % (c, name, run.nsteps, n, nseg, run.engine_rails, run.launches, tl,
                                             min(ts) * 1e3, sum(1 for b in bad if b)), flush=True)
        run.close()
        cx.close()
