#!/usr/bin/env python3
"""Round 6: seeded random shapes (tests/test_relay.py _random_shapes) through both relay forms on the CPU executor:
pairing proof, race check, every byte against the oracle.  usage: relay_random.py <seed> <shapes>"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")):
    sys.path.insert(0, p)
import __graft_entry__ as G  # noqa: E402
from plan_exec import check_recv, simulate  # noqa: E402  (CPU executor: test infrastructure)
from test_relay import _random_shapes  # noqa: E402

xg = G.load_package().xg
seed, n = int(sys.argv[1]), int(sys.argv[2])
runs = fenced = refused = 0
for P, A, Gn, d, c, m in _random_shapes(seed, n):
    rl = xg.aggregator_list(P, A)
    try:
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=1, iteration=1)
    except xg.XGError:
        refused += 1; continue
    for f in (2, 3):
        s.check_pairing(Gn, 0, 0, f)
        views, regs = simulate(s, Gn, it=1, mode=1, pack=0, form=f)
        check_recv(s, Gn, regs, it=1, mode=1)
        runs += 1
        fenced += any(4 in [x[0] for x in views[0].calls(st)] for st in range(views[0].nsteps))
print("seed", seed, "shapes", n, "runs", runs, "plans with a relayed/weighted step", fenced, "refused", refused)
