#!/usr/bin/env python3
"""Pack / unpack kernels of the 8-GPU plans on one MI355X (virtual GPUs, xg_vplans_run).

BASELINE configs[2] shape: 64 logical ranks, 16 aggregators, -d 256 KiB, methods 5 and 8
(MPI_Alltoallw -> per-peer pack into one staging buffer, grouped send/recv, unpack).  All 8
GPUs' plans run on this device, every cross-GPU segment packed (pack_max_seg = 1 GiB), each
RCCL pair moved as one device copy.  Run under rocprofv3 --kernel-trace; pack_summary.py
reduces the trace to HBM GB/s per launch class (local gather, pack, unpack).  The local
gather of a step that also exchanges runs on a side stream beside the packs (as on real
GPUs), so its launches overlap others.  Delivery is verified before the profiled
repetitions."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
P, A, d, GPUS, REPS = 64, 16, 256 << 10, 8, int(os.environ.get("REPS", "10"))
PACK = int(os.environ.get("PACK", 1 << 30))      # 0: direct (one RCCL call per 256 KiB segment)
RCCL = os.environ.get("RCCL") == "1"             # the pairs through RCCL (self send/recv) instead of copies
rl = xg.aggregator_list(P, A)
ctxs = [xg.Context.virtual(g, GPUS, device=0) for g in range(GPUS)]
for m in (5, 8):
    s = xg.Schedule(m, P, A, d, 200000000, rl, ntimes=1)
    runs = [xg.MethodRun(c, s, it=0, mode=0, pack_max_seg=PACK) for c in ctxs]
    xg.run_virtual(runs, rccl=RCCL)
    bad = sum(sum(1 for b in r.verify()[1] if b) for r in runs)
    if bad:
        raise SystemExit("m%d: %d bad slots" % (m, bad))
    t0 = time.perf_counter()
    dev = []
    for _ in range(REPS):
        dev.append(xg.run_virtual(runs, rccl=RCCL)[-1])
    dt = (time.perf_counter() - t0) / REPS
    dev.sort()
    print("m%d pack %d rccl %d: %.1f us per virtual run (host), device %.1f us (median), launches per run %d" % (
        m, PACK, RCCL, dt * 1e6, dev[len(dev) // 2] * 1e6, sum(r.launches for r in runs)), flush=True)
    for r in runs:
        r.close()
    print("m%d ok: %d GPUs x %d reps, %s" % (m, GPUS, REPS, "every cross-GPU segment packed" if PACK else
                                             "one RCCL call per cross-GPU segment"), flush=True)
for c in ctxs:
    c.close()
