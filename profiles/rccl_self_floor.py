#!/usr/bin/env python3
"""RCCL's floor on one MI355X: one group of a self ncclSend + ncclRecv on a 1-rank communicator
(XG_SELF_COMM=1, xg_p2p_bench), per message size -- what one RCCL launch of a latency-bound
step costs before any xGMI hop.  usage: XG_SELF_COMM=1 python3 profiles/rccl_self_floor.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
ctx = xg.Context(0, 1, device=0)
print("bytes  reps  us_per_group  GB/s")
for nb in (4096, 65536, 1 << 20, 16 << 20, 256 << 20):
    reps = 200 if nb <= 65536 else (50 if nb <= 1 << 20 else 10)
    gbps, sec = ctx.p2p_bench(nb, mode=2, reps=reps)
    print("%9d  %4d  %10.2f  %8.1f" % (nb, reps, sec * 1e6, gbps), flush=True)
ctx.close()
