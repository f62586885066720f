#!/usr/bin/env python3
"""How far is the relay form (XG_RELAY) from the best possible two-hop routing?  CPU only.

For every step of the BASELINE 8-GPU plans whose messages cross GPUs, the GPU-pair traffic matrix
D[a][b] (bytes) is routed four ways and the step's link time summed over the run:

  direct   busiest GPU pair (one link carries each pair's bytes)
  relay    the relay form where it applies: (max egress + max ingress) / G, kept only when lower
           (devplan.c relay_step; the real form also requires >= 1 MiB messages)
  LP       the optimum of ANY two-hop routing in two sequential RCCL groups: each pair's bytes
           split over G paths -- straight in group 0, straight in group 1, or via relay h (a -> h
           in group 0, h -> b in group 1) -- minimising max group-0 link + max group-1 link
           (scipy linprog / HiGHS)
  FW       a non-uniform split anyone could compute per step without an LP solver: Frank-Wolfe on
           a soft-max of the two groups' busiest links (300 iterations, numpy) -- what a weighted
           relay form would send; kept per step only where it beats the relay form

A permutation step (m9 / m10, most of m11) is provably at its two-hop optimum under the relay
form: with d bytes straight and r through each of the G - 2 relays, every link of the source
carries 2r (its own first hops plus what it forwards) and the straight link d, so the group pair
costs >= M / 4 for an M-byte message at G = 8, which is what the relay form achieves.
Writes the table to stdout.
"""
import os
import sys

import numpy as np
from scipy.optimize import linprog

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

G = 8
CONFIGS = [("configs[3]", 256, 32, 4 << 20, 200000000, (9, 10))] + \
          [("configs[4] -c %d" % c, 256, 64, 64 << 20, c, (7, 11, 12)) for c in (1, 8)]


def lp_two_hop(D):
    """min T0 + T1 over two-hop routings of the pair matrix D (MiB)"""
    pairs = [(a, b) for a in range(G) for b in range(G) if a != b and D[a][b] > 0]
    nv = len(pairs) * G + 2
    cost = np.zeros(nv)
    cost[-2] = cost[-1] = 1.0
    a_ub, b_ub = [], []
    for u in range(G):
        for v in range(G):
            if u == v:
                continue
            r0, r1 = np.zeros(nv), np.zeros(nv)
            for k, (a, b) in enumerate(pairs):
                for h in range(G):
                    if a == u and h == v:          # group-0 hop a -> h (h == b: straight)
                        r0[k * G + h] = 1.0
                    if h == u and b == v:          # group-1 hop h -> b (h == a: straight)
                        r1[k * G + h] = 1.0
            r0[-2] = r1[-1] = -1.0
            a_ub += [r0, r1]
            b_ub += [0.0, 0.0]
    a_eq, b_eq = [], []
    for k, (a, b) in enumerate(pairs):
        r = np.zeros(nv)
        r[k * G:(k + 1) * G] = 1.0
        a_eq.append(r)
        b_eq.append(D[a][b])
    res = linprog(cost, A_ub=np.array(a_ub), b_ub=b_ub, A_eq=np.array(a_eq), b_eq=b_eq,
                  bounds=[(0, None)] * nv, method="highs")
    assert res.status == 0, res.message
    return res.fun


def fw_two_hop(D, iters=300, sharp=40.0):
    """Frank-Wolfe on softmax(group-0 link loads) + softmax(group-1 link loads): per pair, move a
    2 / (t + 3) share of its bytes onto its cheapest path under the current gradient; -> the best
    T0 + T1 seen (MiB)"""
    pairs = [(a, b) for a in range(G) for b in range(G) if a != b and D[a][b] > 0]
    dem = np.array([D[a][b] for a, b in pairs], float)
    y = np.zeros((len(pairs), G))
    for i, (a, b) in enumerate(pairs):
        y[i, a] = y[i, b] = dem[i] / 2                 # straight, half in each group

    def loads(y):
        l0, l1 = np.zeros((G, G)), np.zeros((G, G))
        for i, (a, b) in enumerate(pairs):
            for h in range(G):
                if h != a:
                    l0[a, h] += y[i, h]
                if h != b:
                    l1[h, b] += y[i, h]
        return l0, l1

    best = None
    for t in range(iters + 1):
        l0, l1 = loads(y)
        cost = l0.max() + l1.max()
        best = cost if best is None else min(best, cost)
        if t == iters:
            break
        beta = sharp / cost
        g0 = np.exp(beta * (l0 - l0.max()))
        g1 = np.exp(beta * (l1 - l1.max()))
        g0, g1 = g0 / g0.sum(), g1 / g1.sum()
        s = np.zeros_like(y)
        for i, (a, b) in enumerate(pairs):
            c = [(g0[a, h] if h != a else 0.0) + (g1[h, b] if h != b else 0.0) for h in range(G)]
            s[i, int(np.argmin(c))] = dem[i]
        y = y + 2.0 / (t + 3) * (s - y)
    return best


def main():
    import __graft_entry__ as GE
    xg = GE.load_package().xg
    print("two-hop routing of the BASELINE 8-GPU plans, link time summed over the run (MiB on the busiest link)")
    print("%-16s %-4s %10s %10s %10s %10s %12s %12s" % ("config", "m", "direct", "relay", "FW", "LP", "relay / LP",
                                                        "min(relay, FW) / direct"))
    for name, P, A, d, c, methods in CONFIGS:
        rl = xg.aggregator_list(P, A)
        for m in methods:
            s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
            by = {}
            for src, _ss, dst, _ds, ln, st, flags in s.messages():
                a, b = s.gpu_of(G, src), s.gpu_of(G, dst)
                if flags & 4 or a == b or ln <= 0:
                    continue
                by.setdefault(st, [[0.0] * G for _ in range(G)])[a][b] += ln / 2 ** 20
            direct = relay = best = fwr = 0.0
            memo = {}
            for D in by.values():
                key = tuple(map(tuple, D))
                if key not in memo:
                    dd = max(max(r) for r in D)
                    eg = max(sum(r) for r in D)
                    ig = max(sum(D[a][b] for a in range(G)) for b in range(G))
                    rr = min(dd, (eg + ig) / G)
                    memo[key] = (dd, rr, lp_two_hop(D), min(rr, fw_two_hop(D)))
                dd, rr, ll, ff = memo[key]
                direct += dd
                relay += rr
                best += ll
                fwr += ff
            print("%-16s %-4d %10.0f %10.0f %10.0f %10.0f %12.3f %12.3f"
                  % (name, m, direct, relay, fwr, best, relay / best, fwr / direct))
            sys.stdout.flush()


if __name__ == "__main__":
    main()
