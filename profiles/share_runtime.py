#!/usr/bin/env python3
"""Device time of one GPU's share of the 8-GPU configs[2] plans (P64 A16 -d 256 KiB, m5 / m8,
two-sided packing) run alone (xg_plan_set_local_only: pack, the local part on the side stream,
unpack; RCCL left out): median over REPS timed runs of the step's completion.  Run it with
XG_SPLIT_AFTER_PACK=0 and =1 to compare the local part forking beside the packs (both share HBM)
with forking after them (it overlaps the unpack here, the transfer on a real node)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
P, A, d, GPUS, REPS = 64, 16, 256 << 10, 8, int(os.environ.get("REPS", "50"))
rl = xg.aggregator_list(P, A)
ctx = xg.Context.virtual(0, GPUS, device=0)
for m in (5, 8):
    s = xg.Schedule(m, P, A, d, 200000000, rl, ntimes=1)
    run = xg.MethodRun(ctx, s, it=0, mode=0, pack_max_seg=4 << 20)
    try:
        run.set_local_only()
        for _ in range(5):
            run.run_timed()
        t = sorted(run.run_timed()[0][-1] for _ in range(REPS))
        print("m%d split_after_pack=%s: GPU 0's share alone %.2f us median (p10 %.2f, p90 %.2f) over %d runs" % (
            m, os.environ.get("XG_SPLIT_AFTER_PACK", "1"), t[len(t) // 2] * 1e6, t[len(t) // 10] * 1e6,
            t[9 * len(t) // 10] * 1e6, REPS), flush=True)
    finally:
        run.close()
ctx.close()
