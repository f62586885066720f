"""The Theta sweep's shape (P16384 A256 d2048, m1 / m2) as an 8-GPU job on ONE MI355X
(virtual GPUs: each GPU's plan, regions and launches; RCCL pairs moved as device copies):
the multi-GPU planner and packing at that scale, every received segment verified.
usage: python3 profiles/theta_virtual8.py [c ...]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as G

xg = G.load_package().xg
P, A, d, NG = 16384, 256, 2048, 8
rl = xg.aggregator_list(P, A)
ctxs = [xg.Context.virtual(g, NG, device=0) for g in range(NG)]
for c in [int(x) for x in sys.argv[1:]] or [16384]:
    for m in (1, 2):
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
        for pack in (0, 4 << 20):
            t0 = time.time()
            runs = [xg.MethodRun(cx, s, it=0, mode=1, pack_max_seg=pack) for cx in ctxs]
            tl = time.time() - t0
            done = xg.run_virtual(runs)
            bad = 0
            for r in runs:
                _chk, b, _f = r.verify()
                bad += sum(1 for x in b if x)
            cross = sum(r.view.remote_send_bytes for r in runs)
            print("m%d c %5d %-6s steps %5d load %.1f s  virtual run %.3f ms (8 GPUs' steps serialized on one device)  "
                  "cross-GPU %.2f GiB  bad slots %d" % (m, c, "packed" if pack else "direct", s.nsteps, tl,
                                                        done[-1] * 1e3, cross / 2**30, bad), flush=True)
            for r in runs:
                r.close()
for cx in ctxs:
    cx.close()
