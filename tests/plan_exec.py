"""CPU executor of xg_devplan (TEST DOUBLE, never part of the product).

Runs GPU g's plan on numpy regions exactly as libxg does on HBM: per step,
stage copies (TAM memcpy's through SCRATCH), pre copies (local gather/scatter
+ packs), the grouped p2p exchange (matched per ordered GPU pair in issue
order, as RCCL does), then post copies (unpacks).  Every copy of one launch
runs concurrently on the GPU, so each launch is first checked for races: no
copy may write bytes another copy of the same launch reads or writes.
"""
import numpy as np

import xg_oracle as O


def make_regions(s, view, G, g, it, mode):
    d = s.d
    reg = [np.zeros(max(0, b), np.uint8) for b in view.region_bytes]
    reg[1][:] = 0xA5
    for rank, seed0, off, nsegs in s.fill_runs(G, g):
        for k in range(nsegs):
            reg[0][off + k * d: off + (k + 1) * d] = O.fingerprint(mode, rank, seed0 + k, it, d)
    return reg


def check_races(lst, what=""):
    """Writes of one launch must not overlap each other or another copy's reads."""
    ev = []
    for i, (sb, so, db, do, ln) in enumerate(lst):
        if ln > 0:
            ev.append((db, do, do + ln, i, "w"))
            ev.append((sb, so, so + ln, i, "r"))
    ev.sort()
    # sweep per buffer: any write interval overlapping an interval of another copy
    by_buf = {}
    for b, lo, hi, i, k in ev:
        by_buf.setdefault(b, []).append((lo, hi, i, k))
    for b, iv in by_buf.items():
        active = []
        for lo, hi, i, k in iv:
            active = [a for a in active if a[1] > lo]
            for alo, ahi, ai, ak in active:
                if ai != i and ("w" in (k, ak)):
                    raise AssertionError("race in launch %s: copies %d and %d overlap in buffer %d" % (what, ai, i, b))
            active.append((lo, hi, i, k))


def copies(reg, lst, what=""):
    check_races(lst, what)
    for sb, so, db, do, ln in lst:
        assert 0 <= so and so + ln <= reg[sb].size and 0 <= do and do + ln <= reg[db].size
        reg[db][do:do + ln] = reg[sb][so:so + ln]


def step_parts(view, st):
    """(stage copies, pre copies, p2p ops, post copies) of one step."""
    pb, pc, qb, qc, ob, oc = view.steps[st]
    sc = view.stage_count[st]
    return (view.copies[pb:pb + sc], view.copies[pb + sc:pb + pc], view.p2p[qb:qb + qc],
            view.copies[ob:ob + oc])


def simulate(s, G, it=0, mode=0, pack=1 << 20, form=-1):
    views = [s.devplan(G, g, pack, 0, form) for g in range(G)]
    regs = [make_regions(s, v, G, g, it, mode) for g, v in enumerate(views)]
    for st in range(views[0].nsteps):
        parts = [step_parts(v, st) for v in views]
        for g in range(G):
            copies(regs[g], parts[g][0], "stage")
            copies(regs[g], parts[g][1], "pre")
        # the step's RCCL groups in order (a relay step: group 1 forwards what group 0 delivered)
        for grp in sorted({o[5] for g in range(G) for o in parts[g][2]}):
            for g in range(G):   # a recv of the group must not land on bytes a send of the group reads
                ops = [o for o in parts[g][2] if o[5] == grp]
                check_races([(o[2], o[3], o[2], o[3], o[4]) if o[1] else (-1, 0, o[2], o[3], o[4]) for o in ops],
                            "p2p group %d" % grp)
            for g in range(G):
                for p in range(G):
                    if p == g:
                        continue
                    sends = [o for o in parts[g][2] if o[0] == p and o[1] and o[5] == grp]
                    recvs = [o for o in parts[p][2] if o[0] == g and not o[1] and o[5] == grp]
                    assert len(sends) == len(recvs), (st, grp, g, p)
                    for (_, _, sb, so, sl, _g), (_, _, rb, ro, rl, _h) in zip(sends, recvs):
                        assert sl == rl, (st, grp, g, p)
                        regs[p][rb][ro:ro + rl] = regs[g][sb][so:so + sl]
        for g in range(G):
            copies(regs[g], parts[g][3], "post")
    return views, regs


def check_recv(s, G, regs, it=0, mode=0):
    exp = O.expected_recv(s.method, s.P, s.A, s.d, s.rank_list, it, mode)
    for r, buf in exp.items():
        g = s.gpu_of(G, r)
        off = s.recv_offset(G, r)
        got = regs[g][1][off: off + buf.size]
        assert (got == buf).all(), (s.method, G, r)
