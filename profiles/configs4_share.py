#!/usr/bin/env python3
"""configs[4] at its stated size, one GPU's share: P256 A64 -d 64 MiB on 8 GPUs is 256 GiB of
SEND + RECV per GPU -- only one GPU of the job fits on this device, so GPU 0's plan runs alone
(xg_plan_set_local_only: every copy launch of its plan, its RCCL calls left out) for m7 / m11 /
m12 at every -c in 1..8 (script_theta_all_to_many_256.sh:33-106 sweeps -c).  Per run: the
regions it holds, its steps and launches, the bytes it keeps on the GPU and the bytes it would
send over xGMI, the device time of its local share (min of REPS), and the delivery check: every
slot whose source lives on GPU 0 bit-exact (and two sampled against the oracle's closed form),
every other slot still unwritten.  usage: python3 profiles/configs4_share.py   (CELLS=11:1,12:8 runs only those (method, -c) cells)"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
os.environ["XG_SELF_MAX"] = "0"          # local parts as copy launches (set before the context)
import __graft_entry__ as G  # noqa: E402
import xg_oracle as O  # noqa: E402

xg = G.load_package().xg
P, A, d, GPUS, REPS = 256, 64, 64 << 20, 8, int(os.environ.get("REPS", "3"))
rl = xg.aggregator_list(P, A)
ctx = xg.Context.virtual(0, GPUS, device=0)
_arch, _cus, hbm = ctx.info()
need = [0] * xg.NBUF
for m in (7, 11, 12):
    s = xg.Schedule(m, P, A, d, 1, rl, ntimes=1)
    v = s.devplan(GPUS, 0)
    need = [max(a, b) for a, b in zip(need, v.region_bytes)]
print("GPU 0 of %d, P%d A%d -d %d: regions %s = %.1f GiB of %.1f GiB HBM" % (
    GPUS, P, A, d, need, sum(need) / 2 ** 30, hbm / 2 ** 30), flush=True)
R = xg.Regions(ctx, need)
lo, hi = 0, 0
CELLS = [tuple(map(int, x.split(":"))) for x in os.environ.get("CELLS", "").split(",") if x.strip()]
try:
    for m in (7, 11, 12):
        for c in range(1, 9):
            if CELLS and (m, c) not in CELLS:
                continue
            s = xg.Schedule(m, P, A, d, c, rl, ntimes=1, iteration=1)
            lo, hi = s.block_range(GPUS, 0)
            run = xg.MethodRun(ctx, s, it=1, mode=1, regions=R)
            try:
                run.set_local_only()
                t = min(run.run_timed()[0][-1] for _ in range(REPS))
                chk, bad, _first = run.verify()
                local = [i for i, sl in enumerate(run.slots) if lo <= sl[0] < hi]
                other = [i for i in range(len(run.slots)) if not lo <= run.slots[i][0] < hi]
                assert local and all(bad[i] == 0 for i in local), (m, c)
                assert all(bad[i] > d // 2 for i in other), (m, c)
                for i in ((local[0], local[-1]) if c == 1 else (local[c % len(local)],)):
                    src, seed, _dst, _off = run.slots[i]
                    assert chk[i] == O.chk64(O.fingerprint(1, src, seed, 1, d)), (m, c, i)
                v = run.view
                print("m%-2d c=%d steps=%-4d launches=%-4d local=%6.1f GiB  xGMI out=%6.1f GiB  local share %8.3f ms"
                      " = %6.2f TB/s delivered (%5.2f TB/s of HBM traffic)  slots: %d local bit-exact, %d from peers"
                      " unwritten" % (m, c, s.nsteps, run.launches, v.local_bytes / 2 ** 30,
                                      v.remote_send_bytes / 2 ** 30, t * 1e3, v.local_bytes / t / 1e12,
                                      2 * v.local_bytes / t / 1e12, len(local), len(other)), flush=True)
            finally:
                run.close()
finally:
    R.close()
    ctx.close()
print("configs4_share ok", flush=True)
