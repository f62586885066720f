#!/usr/bin/env python3
"""How far is the relay form (XG_RELAY) from the best possible two-hop routing?  CPU only.

For every step of the BASELINE 8-GPU plans whose messages cross GPUs, the GPU-pair traffic matrix
D[a][b] (bytes) is routed three ways and the step's link time summed over the run:

  direct   busiest GPU pair (one link carries each pair's bytes)
  relay    the relay form where it applies: (max egress + max ingress) / G, kept only when lower
           (devplan.c relay_step; the real form also requires >= 1 MiB messages)
  LP       the optimum of ANY two-hop routing in two sequential RCCL groups: each pair's bytes
           split over G paths -- straight in group 0, straight in group 1, or via relay h (a -> h
           in group 0, h -> b in group 1) -- minimising max group-0 link + max group-1 link
           (scipy linprog / HiGHS)

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


def main():
    import __graft_entry__ as GE
    xg = GE.load_package().xg
    print("two-hop routing of the BASELINE 8-GPU plans, link time summed over the run (MiB on the busiest link)")
    print("%-16s %-4s %10s %10s %10s %12s" % ("config", "m", "direct", "relay", "LP", "relay / LP"))
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
            direct = relay = best = 0.0
            memo = {}
            for D in by.values():
                key = tuple(map(tuple, D))
                if key not in memo:
                    dd = max(max(r) for r in D)
                    eg = max(sum(r) for r in D)
                    ig = max(sum(D[a][b] for a in range(G)) for b in range(G))
                    memo[key] = (dd, min(dd, (eg + ig) / G), lp_two_hop(D))
                dd, rr, ll = memo[key]
                direct += dd
                relay += rr
                best += ll
            print("%-16s %-4d %10.0f %10.0f %10.0f %12.3f" % (name, m, direct, relay, best, relay / best))
            sys.stdout.flush()


if __name__ == "__main__":
    main()
