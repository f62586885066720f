#!/usr/bin/env python3
"""The three forms of a cross-GPU transfer list on the 8-GPU configs[2] plans, on one MI355X.

BASELINE configs[2]: 64 logical ranks, 16 aggregators, -d 256 KiB, methods 5 and 8
(MPI_Alltoallw, mpi_test.c:599-654, :885-940) as an 8-GPU job on this device (virtual GPUs,
xg_vplans_run_rccl: every pair through RCCL on a 1-rank communicator).  Per GPU and step, the
28 MiB it sends to its 7 peers (16 segments of 256 KiB per peer) go
  direct            one RCCL call per segment, no copy;
  packed_two_sided  one staging buffer per peer and direction: pack 28 MiB, 7 calls, unpack 28 MiB;
  packed_one_sided  runs contiguous at one end (2 per peer, 2 MiB each), the other end staged:
                    m8 packs 28 MiB on the sender and receives straight into the slots, m5
                    sends straight from the aggregators' segments and unpacks on the receiver.
Printed per method and form: the virtual run's host and device time (median of REPS), kernel
launches per run, and the copy launches by class (HIP events around every launch of GPU 0:
bytes, mean us, TB/s of read + write).  Every byte is verified before timing."""
import collections
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg
P, A, d, GPUS, REPS = 64, 16, 256 << 10, 8, int(os.environ.get("REPS", "20"))
RCCL = os.environ.get("RCCL", "1") == "1"
FORMS = [("direct", 0, -1), ("packed_one_sided", 1 << 30, xg.PACK_ONE_SIDED),
         ("packed_two_sided", 1 << 30, xg.PACK_TWO_SIDED)]
only = os.environ.get("FORMS")
if only:
    FORMS = [f for f in FORMS if f[0] in only.split(",")]
rl = xg.aggregator_list(P, A)
ctxs = [xg.Context.virtual(g, GPUS, device=0) for g in range(GPUS)]
for m in [int(x) for x in os.environ.get("METHODS", "5,8").split(",")]:
    s = xg.Schedule(m, P, A, d, 200000000, rl, ntimes=1)
    for name, pack, form in FORMS:
        runs = [xg.MethodRun(c, s, it=0, mode=1, pack_max_seg=pack, pack_form=form) for c in ctxs]
        xg.run_virtual(runs, rccl=RCCL)
        bad = sum(sum(1 for b in r.verify()[1] if b) for r in runs)
        if bad:
            raise SystemExit("m%d %s: %d bad slots" % (m, name, bad))
        for _ in range(3):
            xg.run_virtual(runs, rccl=RCCL)
        host, dev = [], []
        for _ in range(REPS):
            t0 = time.perf_counter()
            dev.append(xg.run_virtual(runs, rccl=RCCL)[-1])
            host.append(time.perf_counter() - t0)
        host.sort()
        dev.sort()
        v = runs[0].view
        copied = (sum(c[4] for c in v.copies if c[2] == 2), sum(c[4] for c in v.copies if c[0] == 3))
        calls = sum(1 for o in v.p2p)
        print("m%d %-17s host %7.1f us  device %7.1f us per virtual run (median of %d), launches/run %d, "
              "GPU 0: %d RCCL calls, packs %d B, unpacks %d B" % (
                  m, name, host[len(host) // 2] * 1e6, dev[len(dev) // 2] * 1e6, REPS,
                  sum(r.launches for r in runs), calls, copied[0], copied[1]), flush=True)
        # GPU 0's copy launches, each between HIP events on the stream it runs on
        ctxs[0].ktime_begin(per_launch=True)
        for _ in range(5):
            xg.run_virtual(runs, rccl=RCCL)
        _ms, n, _b = ctxs[0].ktime_end()
        cls = collections.defaultdict(list)
        for ms, b in ctxs[0].ktime_launches(n):
            cls[b].append(ms)
        for b, ts in sorted(cls.items()):
            ts.sort()
            us = ts[len(ts) // 2] * 1e3
            print("    launch class %10d B (read+write)  %3d launches  median %6.2f us  %5.2f TB/s" % (
                b, len(ts), us, b / us / 1e6), flush=True)
        for r in runs:
            r.close()
for c in ctxs:
    c.close()
print("pack_forms ok", flush=True)
