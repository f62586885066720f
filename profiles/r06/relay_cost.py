#!/usr/bin/env python3
"""Round 6: what the relay form's extra RCCL calls cost, measured on one GPU.

1. RCCL's cost per call inside a group: xg_p2p_split_bench on a one-rank communicator
   (XG_SELF_COMM=1: rank 0 sends to itself) -- the same bytes posted as 1, 2, 4, 8, 16, 32 calls;
   the slope of time against calls is the per-call cost, the intercept the one-call time.
2. The relay form and the coalesced relay form (XG_RELAY_COALESCED: one call per hop and kind)
   against direct on configs[3] m9 / m10 (P256 A32, the pairwise XOR rounds the relay
   form reroutes) as a virtual 8-GPU job whose pairs go through RCCL (xg_vplans_run_rccl: every
   GPU's calls of a step in one group on one device): device time per run, calls per step of
   GPU 0 in each form.  On one device no link is crossed, so the relay form's 4x link-time gain
   is absent here and what remains is its cost: 1.75x the posted bytes and G x the calls.
Prints one JSON object per measurement and a summary.
"""
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
os.environ["XG_SELF_COMM"] = "1"
import __graft_entry__ as G  # noqa: E402

xg = G.load_package().xg


def split_costs():
    ctx = xg.Context(rank=0, nranks=1, device=0)
    rows = []
    try:
        for nbytes in (128 << 10, 1 << 20, 4 << 20, 16 << 20):
            for calls in (1, 2, 4, 8, 16, 32):
                reps = 50 if nbytes <= 1 << 20 else 20
                ts = []
                for _ in range(3):
                    _g, sec = ctx.p2p_split_bench(nbytes, calls, reps)
                    ts.append(sec)
                row = {"what": "split", "bytes": nbytes, "calls": calls, "us_per_rep_median": round(statistics.median(ts) * 1e6, 2),
                       "us_min": round(min(ts) * 1e6, 2), "us_max": round(max(ts) * 1e6, 2)}
                rows.append(row)
                print(json.dumps(row), flush=True)
    finally:
        ctx.close()
    # least-squares slope per size: us per extra call
    fit = {}
    for nbytes in sorted({r["bytes"] for r in rows}):
        pts = [(r["calls"], r["us_per_rep_median"]) for r in rows if r["bytes"] == nbytes]
        n = len(pts)
        mx = sum(x for x, _ in pts) / n
        my = sum(y for _, y in pts) / n
        slope = sum((x - mx) * (y - my) for x, y in pts) / sum((x - mx) ** 2 for x, _ in pts)
        fit[nbytes] = {"us_per_call": round(slope, 3), "us_one_call": round(my - slope * (mx - 1), 2)}
    print(json.dumps({"what": "split_fit", "fit": fit}), flush=True)
    return fit


def calls_per_step(s, form):
    v = s.devplan(8, 0, form[0], 0, form[1])
    n = [sum(1 for k, peer, *_ in v.calls(st) if k in (xg.CALL_SEND, xg.CALL_RECV) and peer != 0)
         for st in range(v.nsteps)]
    return sum(n) / max(1, sum(1 for x in n if x)), v.nsteps


CASES = [(256, 32, d, 200000000, m) for d in (1 << 20, 4 << 20) for m in (9, 10)]
# CASES=m7: configs[4]'s m7 (P256 A64) at -d 1 / 8 MiB, which only the coalesced form's weighted
# two-hop split reroutes
M7_CASES = [(256, 64, d, 1, 7) for d in (1 << 20, 8 << 20)]


def relay_vs_direct(reps=3, cases=CASES):
    it = 1
    ctxs = [xg.Context.virtual(g, 8, device=0) for g in range(8)]
    out = []
    try:
        for P, A, d, comm, m in cases:
            rl = xg.aggregator_list(P, A)
            s = xg.Schedule(m, P, A, d, comm, rl, ntimes=1, iteration=it)
            forms = {"direct": (0, -1), "relay": (0, 2), "coalesced": (0, 3)}
            need = [[0] * xg.NBUF for _ in range(8)]
            for f in forms.values():
                for g in range(8):
                    need[g] = [max(a, b) for a, b in zip(need[g], s.devplan(8, g, f[0], 0, f[1]).region_bytes)]
            regs = [xg.Regions(c, n) for c, n in zip(ctxs, need)]
            try:
                row = {"what": "virtual8_rccl", "P": P, "A": A, "d": d, "c": comm, "method": m}
                for name, f in forms.items():
                    runs = [xg.MethodRun(c, s, it=it, mode=1, pack_max_seg=f[0], pack_form=f[1], regions=regs[g])
                            for g, c in enumerate(ctxs)]
                    try:
                        xg.run_virtual(runs, rccl=True)          # warm-up (connection set-up)
                        ts = []
                        for _ in range(reps):
                            t0 = time.perf_counter()
                            done = xg.run_virtual(runs, rccl=True)
                            ts.append((done[-1], time.perf_counter() - t0))
                        bad = sum(sum(1 for b in r.verify()[1] if b) for r in runs)
                    finally:
                        for r in runs:
                            r.close()
                    cps, nst = calls_per_step(s, f)
                    row[name] = {"device_ms_median": round(statistics.median(t for t, _ in ts) * 1e3, 3),
                                 "device_ms_min": round(min(t for t, _ in ts) * 1e3, 3),
                                 "device_ms_max": round(max(t for t, _ in ts) * 1e3, 3),
                                 "host_ms_median": round(statistics.median(w for _, w in ts) * 1e3, 3),
                                 "gpu0_cross_calls_per_busy_step": round(cps, 2), "steps": nst, "bad_slots": bad}
                for f in ("relay", "coalesced"):
                    row[f + "_over_direct"] = round(row[f]["device_ms_median"] / row["direct"]["device_ms_median"], 3)
                out.append(row)
                print(json.dumps(row), flush=True)
            finally:
                for r in regs:
                    r.close()
    finally:
        for c in ctxs:
            c.close()
    return out


if __name__ == "__main__":
    if os.environ.get("SPLIT", "1") == "1":
        split_costs()
    relay_vs_direct(cases=M7_CASES if os.environ.get("CASES") == "m7" else CASES)
    print("relay_cost ok", flush=True)
