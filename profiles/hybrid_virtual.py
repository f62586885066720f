#!/usr/bin/env python3
"""Engine segments inside multi-GPU plans: the README configuration (P32 A14 -d 2048 -c 3)
as an 8-GPU job on one MI355X (virtual GPUs, cross-GPU pairs through RCCL self send/recv,
xg_vplans_run_rccl), m6 / m9 / m12, with the step engine on (default) or off
(XG_ENGINE_MAX_STEP=0).  Prints the plans' kernel launches per run and the run time; a
rocprofv3 kernel trace of the same command counts the launches the device saw."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
P, A, d, c, GPUS, REPS = 32, 14, 2048, 3, 8, int(os.environ.get("REPS", "5"))
PACK = int(os.environ.get("PACK", 4 << 20))     # 0: direct (one RCCL call per segment)
PACK_MIN = int(os.environ.get("PACK_MIN", 0))    # pack only (step, peer) lists of >= this many bytes
rl = xg.aggregator_list(P, A)
ctxs = [xg.Context.virtual(g, GPUS, device=0) for g in range(GPUS)]
for m in (6, 9, 12):
    s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
    runs = [xg.MethodRun(cx, s, it=0, mode=0, pack_max_seg=PACK, pack_min=PACK_MIN) for cx in ctxs]
    xg.run_virtual(runs, rccl=True)
    bad = sum(sum(1 for b in r.verify()[1] if b) for r in runs)
    if bad:
        raise SystemExit("m%d: %d bad slots" % (m, bad))
    t0 = time.perf_counter()
    for _ in range(REPS):
        xg.run_virtual(runs, rccl=True)
    dt = (time.perf_counter() - t0) / REPS
    seg = [r.engine_steps() for r in runs]
    print("m%-2d pack %d/%d steps %d  launches per run (all GPUs) %3d  engine steps %3d in %d segments  %.1f us per run"
          % (m, PACK, PACK_MIN, s.nsteps, sum(r.launches for r in runs), sum(x[0] for x in seg), sum(x[1] for x in seg),
             dt * 1e6), flush=True)
    for r in runs:
        r.close()
for cx in ctxs:
    cx.close()
