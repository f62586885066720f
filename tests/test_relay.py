"""The relay form (XG_RELAY, devplan.c relay_calls) on the CPU: a step whose cross-GPU messages form a
permutation of the GPUs -- pairwise m9 / m10's XOR rounds (mpi_test.c:510-597, :421-508; partner
rank ^ i at :531-545) -- sends every message over all G - 1 links of its source in two RCCL groups
instead of over one link.  Every byte still lands where the reference puts it (race-checked CPU
executor, oracle closed form), RCCL pairs the calls within one step AND one group, the other steps
stay exactly the direct form's, and the busiest link of configs[3]'s pairwise rounds carries a
quarter of what it carries direct (profiles/r05/link_load.txt)."""
import pytest

import xg_oracle as O
from plan_exec import check_recv, simulate

DIRECT, RELAY, COALESCED = (0, -1), (0, 2), (0, 3)
SEND, RECV, BARRIER, FENCE = 1, 2, 3, 4


@pytest.mark.parametrize("G, d, form", [(3, 1 << 20, RELAY), (4, (1 << 20) + 48, RELAY), (8, (1 << 20) + 3, RELAY),
                                        (3, 1 << 20, COALESCED), (8, (1 << 20) + 3, COALESCED)])
def test_relay_plans_deliver_every_byte(xg, G, d, form):
    """P16 A8 (lists of >= 1 MiB per XOR round at every G), every method the relay form changes,
    collision-free fingerprint; 16-B aligned cuts of an unaligned -d ((1 << 20) + 3) included.
    (A plan the relay form leaves alone is the direct form's, call for call:
    test_relay_decision_follows_the_link_model.)"""
    P, A = 16, 8
    rl = xg.aggregator_list(P, A)
    relayed = set()
    for m in O.METHODS:
        s = xg.Schedule(m, P, A, d, 3, rl, ntimes=1, iteration=1)
        if not any(o[5] == 1 for g in range(G) for o in s.devplan(G, g, form[0], 0, form[1]).p2p):
            continue
        relayed.add(m)
        assert s.check_pairing(G, form[0], 0, form[1]) > 0
        _views, regs = simulate(s, G, it=1, mode=1, pack=form[0], form=form[1])
        check_recv(s, G, regs, it=1, mode=1)
    assert {3, 4, 6, 9, 10, 11, 12} <= relayed, relayed


def _ref_group_pairs(views):
    """independent restatement: in each step and each group of it (calls split at the fence), the
    k-th send of g to h with the k-th receive of h from g -> {(step, group, g, h, len)} counts"""
    from collections import Counter
    G = len(views)
    out = Counter()
    for st in range(views[0].nsteps):
        groups = []
        for v in views:
            gs, cur = [], []
            for c in v.calls(st):
                if c[0] == FENCE:
                    gs.append(cur)
                    cur = []
                elif c[0] in (SEND, RECV):
                    cur.append(c)
            gs.append(cur)
            groups.append(gs)
        for q in range(max(len(x) for x in groups)):
            for g in range(G):
                for h in range(G):
                    sends = [c for c in (groups[g][q] if q < len(groups[g]) else []) if c[0] == SEND and c[1] == h]
                    recvs = [c for c in (groups[h][q] if q < len(groups[h]) else []) if c[0] == RECV and c[1] == g]
                    assert len(sends) == len(recvs), (st, q, g, h)
                    for a, b in zip(sends, recvs):
                        assert a[4] == b[4], (st, q, g, h)
                        out[(st, q, g, h, a[4])] += 1
    return out


@pytest.mark.parametrize("m", [9, 10, 12])
def test_relay_pairs_by_step_and_group(xg, m):
    from collections import Counter
    P, A, d, G = 16, 8, 1 << 20, 8
    s = xg.Schedule(m, P, A, d, 3, xg.aggregator_list(P, A), ntimes=1)
    views = [s.devplan(G, g, RELAY[0], 0, RELAY[1]) for g in range(G)]
    pairs = xg.devplans_match(views, groups=True)
    got = Counter((st, grp, src, dst, ln) for st, grp, src, dst, _sc, _rc, ln in pairs)
    assert got == _ref_group_pairs(views)
    # pairs come in (step, group) order; a relay step's group 1 forwards what group 0 delivered
    assert [(p[0], p[1]) for p in pairs] == sorted((p[0], p[1]) for p in pairs)
    for v in views:
        for st in range(v.nsteps):
            c = v.calls(st)
            assert [x[0] for x in c].count(FENCE) <= 1
            if FENCE in [x[0] for x in c]:
                f = [x[0] for x in c].index(FENCE)
                assert all(x[0] in (SEND, RECV) for x in c[f + 1:] if x[0] != BARRIER)
    if m in (9, 10):
        assert any(p[1] == 1 for p in pairs)


def test_relay_refused_when_a_pair_spans_two_groups(xg):
    """the matcher's new rule: a send in a step's first group whose receive sits in the second
    group is refused (the two groups are separate ncclGroupEnd launches: such a pair could wait
    for a group its peer posts later)"""
    S, R, F = SEND, RECV, FENCE
    calls = [[[(S, 1, 0, 0, 8), (F, -1, -1, 0, 0)]],
             [[(F, -1, -1, 0, 0), (R, 0, 1, 0, 8)]]]
    with pytest.raises(xg.XGError) as e:
        xg.calls_match(calls, 1)
    assert "group 0, its receive in group 1" in str(e.value)
    ok = [[[(S, 1, 0, 0, 8), (F, -1, -1, 0, 0), (S, 1, 0, 8, 8)]],
          [[(R, 0, 1, 0, 8), (F, -1, -1, 0, 0), (R, 0, 1, 8, 8)]]]
    assert len(xg.calls_match(ok, 1)) == 2


def _busiest(views, xg):
    """sum over steps and groups of the busiest directed link's bytes"""
    tot = 0
    for st in range(views[0].nsteps):
        per = {}
        for g, v in enumerate(views):
            q = 0
            for kind, peer, _b, _o, ln in v.calls(st):
                if kind == FENCE:
                    q += 1
                elif kind == SEND and peer != g:
                    per[(q, g, peer)] = per.get((q, g, peer), 0) + ln
        for q in {k[0] for k in per}:
            tot += max(b for k, b in per.items() if k[0] == q)
    return tot


@pytest.mark.parametrize("m", [9, 10])
def test_relay_at_configs3_full_size(xg, m):
    """configs[3] (P256 A32 -d 4 MiB) on 8 GPUs: the 224 cross-GPU XOR rounds are relayed, the 32
    GPU-local ones are not; RCCL pairs every call; the busiest link carries 1/4 of the direct form's
    bytes (3584 -> 896 MiB over the run: DESIGN.md's link-load table)"""
    P, A, d, G = 256, 32, 4 << 20, 8
    s = xg.Schedule(m, P, A, d, 200000000, xg.aggregator_list(P, A), ntimes=1)
    assert s.check_pairing(G, RELAY[0], 0, RELAY[1]) > 0
    relay = [s.devplan(G, g, RELAY[0], 0, RELAY[1]) for g in range(G)]
    direct = [s.devplan(G, g, DIRECT[0], 0, DIRECT[1]) for g in range(G)]
    steps = sum(1 for st in range(relay[0].nsteps) if FENCE in [c[0] for c in relay[0].calls(st)])
    assert steps == 224
    assert _busiest(direct, xg) == 3584 << 20 and _busiest(relay, xg) == 896 << 20
    assert [v.remote_send_bytes for v in relay] == [v.remote_send_bytes for v in direct]
    # relay staging: a relay holds one 1/8 piece of each of the 6 other sources' 16 MiB -> 12 MiB
    assert max(v.region_bytes[3] for v in relay) == 12 << 20


def _relay_model(s, G, st_msgs):
    """the relay decision restated: (max egress + max ingress) / G <= 0.8 x the busiest GPU pair,
    every cross-GPU message >= 1 MiB (XG_RELAY_GAIN, XG_RELAY_MIN_BYTES)"""
    eg, ig, pair = [0] * G, [0] * G, {}
    for src, dst, ln in st_msgs:
        a, b = s.gpu_of(G, src), s.gpu_of(G, dst)
        if a == b or ln <= 0:
            continue
        if ln < 1 << 20:
            return False
        eg[a] += ln
        ig[b] += ln
        pair[(a, b)] = pair.get((a, b), 0) + ln
    return bool(pair) and G >= 3 and (max(eg) + max(ig)) / G <= 0.8 * max(pair.values())


@pytest.mark.parametrize("m", [1, 2, 5, 7, 9, 11, 12])
@pytest.mark.parametrize("P, A, d", [(16, 8, 1 << 20), (16, 8, 64 << 10), (24, 6, 2 << 20)])
def test_relay_decision_follows_the_link_model(xg, m, P, A, d):
    """a step is relayed exactly when the two-phase link model beats the direct form's busiest GPU
    pair by 20 % and its messages are >= 1 MiB; every other step is the direct form's, call for
    call (unordered / alltoallw steps -- every GPU to every GPU -- stay direct: no gain there)"""
    G = 8
    s = xg.Schedule(m, P, A, d, 3, xg.aggregator_list(P, A), ntimes=1)
    by_step = {}
    for src, _ss, dst, _ds, ln, st, flags in s.messages():
        if not flags & 4:
            by_step.setdefault(st, []).append((src, dst, ln))
    relay = [s.devplan(G, g, RELAY[0], 0, RELAY[1]) for g in range(G)]
    direct = [s.devplan(G, g, DIRECT[0], 0, DIRECT[1]) for g in range(G)]
    for st in range(relay[0].nsteps):
        want = _relay_model(s, G, by_step.get(st, []))
        for g in range(G):
            got = FENCE in [c[0] for c in relay[g].calls(st)]
            assert got == want, (m, P, A, d, st, g)
            if not got:
                assert relay[g].calls(st) == direct[g].calls(st), (m, st, g)
    if d < 1 << 20:
        assert not any(o[5] for v in relay for o in v.p2p)


def _link_bytes_by_step(views):
    """{(step, group, src GPU, dst GPU): bytes} of every cross-GPU send"""
    out = {}
    for st in range(views[0].nsteps):
        for g, v in enumerate(views):
            q = 0
            for kind, peer, _b, _o, ln in v.calls(st):
                if kind == FENCE:
                    q += 1
                elif kind == SEND and peer != g:
                    out[(st, q, g, peer)] = out.get((st, q, g, peer), 0) + ln
    return out


@pytest.mark.parametrize("m, P, A, d, c", [(9, 256, 32, 4 << 20, 200000000), (10, 256, 32, 4 << 20, 200000000),
                                           (11, 256, 64, 8 << 20, 1), (12, 256, 64, 8 << 20, 8)])
def test_coalesced_relay_same_links_fewer_calls(xg, m, P, A, d, c):
    """the coalesced relay form (XG_RELAY_COALESCED) at configs[3] / configs[4]'s shapes on 8 GPUs:
    the same steps relayed, every directed link carrying the same bytes in every step and group as the
    relay form, every other step the direct form's call for call -- and a pairwise round (m9 / m10)
    posts G - 1 sends + G - 1 receives per group on every GPU, where the relay form posts 112 calls
    (4 messages per GPU pair, G calls per message and direction)"""
    G = 8
    s = xg.Schedule(m, P, A, d, c, xg.aggregator_list(P, A), ntimes=1)
    assert s.check_pairing(G, COALESCED[0], 0, COALESCED[1]) > 0
    direct = [s.devplan(G, g, DIRECT[0], 0, DIRECT[1]) for g in range(G)]
    relay = [s.devplan(G, g, RELAY[0], 0, RELAY[1]) for g in range(G)]
    coal = [s.devplan(G, g, COALESCED[0], 0, COALESCED[1]) for g in range(G)]
    assert _link_bytes_by_step(coal) == _link_bytes_by_step(relay)
    ncalls = {"relay": 0, "coalesced": 0}
    for g in range(G):
        for st in range(coal[g].nsteps):
            cc, rc = coal[g].calls(st), relay[g].calls(st)
            assert (FENCE in [x[0] for x in cc]) == (FENCE in [x[0] for x in rc]), (g, st)
            if FENCE not in [x[0] for x in cc]:
                assert cc == direct[g].calls(st), (g, st)
                continue
            ncalls["coalesced"] += sum(1 for x in cc if x[0] in (SEND, RECV))
            ncalls["relay"] += sum(1 for x in rc if x[0] in (SEND, RECV))
            if m in (9, 10):
                f = [x[0] for x in cc].index(FENCE)
                for grp in (cc[:f], cc[f + 1:]):
                    assert sum(1 for x in grp if x[0] == SEND) == G - 1, (g, st)
                    assert sum(1 for x in grp if x[0] == RECV) == G - 1, (g, st)
                    assert len({x[1] for x in grp if x[0] == SEND}) == G - 1
    assert ncalls["coalesced"] * 4 <= ncalls["relay"], ncalls
    assert [v.remote_send_bytes for v in coal] == [v.remote_send_bytes for v in direct]


@pytest.mark.parametrize("m", [9, 11, 12])
def test_coalesced_relay_packs_and_unpacks(xg, m):
    """P32 A16 on 8 GPUs (4 ranks per GPU: several messages per GPU pair, so calls carry several
    pieces -- packed by the sender, unpacked by the receiver -- next to one-piece calls that move in
    place), -d (1 << 20) + 3 (every piece at an odd address): every byte where the reference puts it,
    no launch races (CPU executor), staging laid out as the device displacement scan rebuilds it"""
    P, A, d, G = 32, 16, (1 << 20) + 3, 8
    s = xg.Schedule(m, P, A, d, 3, xg.aggregator_list(P, A), ntimes=1, iteration=1)
    views, regs = simulate(s, G, it=1, mode=1, pack=COALESCED[0], form=COALESCED[1])
    check_recv(s, G, regs, it=1, mode=1)
    packed = unpacked = 0
    for v in views:
        for st in range(v.nsteps):
            pb, pc, _qb, _qc, ob, oc = v.steps[st]
            packs = [c for c in v.copies[pb:pb + pc] if c[2] == 2]
            unpacks = v.copies[ob:ob + oc]
            # the displacement scan's layout: every step's packs / unpacks tile staging from 0, in order
            off = 0
            for c in packs:
                assert c[3] == off
                off += c[4]
            off = 0
            for c in unpacks:
                assert c[0] == 3 and c[1] == off
                off += c[4]
            packed += len(packs)
            unpacked += len(unpacks)
    assert packed > 0 and unpacked > 0


def _groups_busiest(views, st):
    """sum over the RCCL groups of step st of its busiest directed link's bytes"""
    per = {}
    for g, v in enumerate(views):
        q = 0
        for kind, peer, _b, _o, ln in v.calls(st):
            if kind == FENCE:
                q += 1
            elif kind == SEND and peer != g:
                per[(q, g, peer)] = per.get((q, g, peer), 0) + ln
    return sum(max(b for k, b in per.items() if k[0] == q) for q in {k[0] for k in per}) if per else 0


@pytest.mark.parametrize("c", [1, 8])
def test_weighted_split_of_configs4_m7(xg, c):
    """configs[4]'s m7 (P256 A64, here -d 8 MiB) on 8 GPUs: no step is a permutation, so the uniform
    cut gains nothing (the relay form leaves it direct), but the coalesced form's weighted two-hop
    split (devplan.c weighted_step, Frank-Wolfe) reroutes all 64 of its cross-GPU steps: each weighted
    step's busiest group-0 + group-1 links carry <= 0.85 of its busiest pair's bytes, the run 0.81 of
    the direct form's (4096 -> 3302 MiB; the LP optimum of two-hop routing is 0.78,
    profiles/r05/relay_lp.txt); RCCL pairs every call, within 10 % of direct's call count (a share of
    >= 4 MiB a piece goes one call per piece, in place: rc_split)"""
    P, A, d, G = 256, 64, 8 << 20, 8
    s = xg.Schedule(7, P, A, d, c, xg.aggregator_list(P, A), ntimes=1)
    assert s.check_pairing(G, COALESCED[0], 0, COALESCED[1]) > 0
    direct = [s.devplan(G, g, DIRECT[0], 0, DIRECT[1]) for g in range(G)]
    relay = [s.devplan(G, g, RELAY[0], 0, RELAY[1]) for g in range(G)]
    coal = [s.devplan(G, g, COALESCED[0], 0, COALESCED[1]) for g in range(G)]
    tot_d = tot_c = weighted = 0
    for st in range(direct[0].nsteps):
        assert relay[0].calls(st) == direct[0].calls(st)
        bd, bc = _groups_busiest(direct, st), _groups_busiest(coal, st)
        if FENCE in [x[0] for x in coal[0].calls(st)]:
            weighted += 1
            assert bc <= 0.85 * bd, (st, bc, bd)
        else:
            assert bc == bd
        tot_d += bd
        tot_c += bc
    assert weighted == 64 and tot_d == 4096 << 20 and tot_c <= 0.81 * tot_d, (weighted, tot_d >> 20, tot_c >> 20)
    for g in range(G):
        n = lambda v: sum(1 for st in range(v.nsteps) for x in v.calls(st) if x[0] in (SEND, RECV))
        assert n(coal[g]) <= 1.1 * n(direct[g])


def test_weighted_split_matches_the_python_frank_wolfe(xg):
    """the C split (quantised to 1/1024ths) against profiles/relay_lp.py's fw_two_hop, an independent
    numpy statement of the same Frank-Wolfe, on every weighted step of configs[4] m7 at -c 1 and
    P24 A6 m1 on 4 GPUs (an uneven all-to-all): within 5 % of its best (continuous) link time -- the C
    split folds shares under 16/1024 of a pair into its largest (one call fewer per dropped hop)"""
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location("relay_lp", os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "relay_lp.py"))
    lp = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(lp)
    for P, A, d, c, m, G in [(256, 64, 8 << 20, 1, 7, 8), (24, 6, 1 << 20, 3, 1, 4)]:
        lp.G = G
        s = xg.Schedule(m, P, A, d, c, xg.aggregator_list(P, A), ntimes=1)
        coal = [s.devplan(G, g, COALESCED[0], 0, COALESCED[1]) for g in range(G)]
        mats = {}
        for src, _ss, dst, _ds, ln, st, flags in s.messages():
            a, b = s.gpu_of(G, src), s.gpu_of(G, dst)
            if flags & 4 or a == b or ln <= 0:
                continue
            mats.setdefault(st, [[0.0] * G for _ in range(G)])[a][b] += ln / 2 ** 20
        seen = 0
        for st, D in mats.items():
            if FENCE not in [x[0] for x in coal[0].calls(st)] or seen >= 4:
                continue
            seen += 1
            got = _groups_busiest(coal, st) / 2 ** 20
            assert got <= 1.05 * lp.fw_two_hop(D), (m, st, got)
        assert seen


@pytest.mark.parametrize("P, A, G, methods", [(32, 16, 3, (7, 9, 12)), (24, 6, 4, (1, 2, 12)), (32, 8, 8, (7,)),
                                              (16, 8, 3, (5, 8, 15, 16))])
def test_weighted_split_delivers_every_byte(xg, P, A, G, methods):
    """steps the coalesced form splits by weight (the uneven block maps of 3 / 4 GPUs, m7's matrices,
    m5 / m8's alltoallw, TAM m15 / m16's aggregation) at -d (1 << 20) + 3: every byte where the
    reference puts it, no launch races, RCCL pairs every call; every such step has a second group"""
    d = (1 << 20) + 3
    rl = xg.aggregator_list(P, A)
    for m in methods:
        s = xg.Schedule(m, P, A, d, 3, rl, ntimes=1, iteration=1)
        relay = s.devplan(G, 0, RELAY[0], 0, RELAY[1])
        coal = s.devplan(G, 0, COALESCED[0], 0, COALESCED[1])
        fences = lambda v: sum(1 for st in range(v.nsteps) if FENCE in [x[0] for x in v.calls(st)])
        assert fences(coal) > fences(relay), (P, A, G, m)      # some step is weighted, not uniform
        assert s.check_pairing(G, COALESCED[0], 0, COALESCED[1]) > 0
        _views, regs = simulate(s, G, it=1, mode=1, pack=COALESCED[0], form=COALESCED[1])
        check_recv(s, G, regs, it=1, mode=1)


def _random_shapes(seed, n):
    import random
    rnd = random.Random(seed)
    out = []
    while len(out) < n:
        P = rnd.randint(6, 40)
        A = rnd.randint(1, min(P, 16))
        G = rnd.randint(3, min(8, P))
        d = rnd.choice([1 << 20, (1 << 20) + 3, (1 << 20) + 48, (2 << 20) + 5])
        c = rnd.choice([1, 2, 3, 8, 200000000])
        m = rnd.randint(1, 20)
        out.append((P, A, G, d, c, m))
    return out


@pytest.mark.parametrize("P, A, G, d, c, m", _random_shapes(2026, 6))    # 450 more: profiles/r06/relay_random.py
def test_relay_forms_random_shapes(xg, P, A, G, d, c, m):
    """random shapes (P 6-40, A 1-16, G 3-8, -d 1-2 MiB aligned and not, -c 1-8 / default, methods
    1-20): both relay forms (uniform cuts, coalesced calls, weighted splits) deliver every byte
    where the reference puts it, race-free, and RCCL pairs every call; a schedule MPI itself would
    deadlock on (m6 at some -c) is refused alike in every form"""
    rl = xg.aggregator_list(P, A)
    try:
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=1, iteration=1)
    except xg.XGError as e:
        assert "deadlock" in str(e).lower() or "hang" in str(e).lower(), str(e)
        return
    for form in (RELAY, COALESCED):
        assert s.check_pairing(G, form[0], 0, form[1]) >= 0
        _views, regs = simulate(s, G, it=1, mode=1, pack=form[0], form=form[1])
        check_recv(s, G, regs, it=1, mode=1)


def test_coalesced_form_goes_in_place_for_large_pieces(xg):
    """a coalesced call whose pieces average >= 4 MiB goes one call per piece, in place
    (devplan.c rc_split): at configs[4]'s stated -d 64 MiB (8 MiB pieces) m11's coalesced plan posts
    the relay form's calls in every step and group (bench.plan_signature: in another order, its
    relayed pieces elsewhere in STAGE_RECV), with no pack or unpack; at -d 8 MiB (1 MiB pieces) it packs and
    posts 4x fewer calls; RCCL pairs both"""
    P, A, G = 256, 64, 8
    rl = xg.aggregator_list(P, A)
    for d, same in ((64 << 20, True), (8 << 20, False)):
        s = xg.Schedule(11, P, A, d, 1, rl, ntimes=1)
        assert s.check_pairing(G, COALESCED[0], 0, COALESCED[1]) > 0
        for g in (0, 5):
            r = s.devplan(G, g, RELAY[0], 0, RELAY[1])
            c = s.devplan(G, g, COALESCED[0], 0, COALESCED[1])
            calls = lambda v: [v.calls(st) for st in range(v.nsteps)]
            if same:         # the same calls in every step and group, up to where a relay keeps its pieces
                import bench
                assert bench.plan_signature(c) == bench.plan_signature(r)
                assert not [x for x in c.copies if x[2] == 2 or x[0] == 3]
            else:
                n = lambda v: sum(1 for cs in calls(v) for x in cs if x[0] in (SEND, RECV))
                assert 4 * n(c) <= n(r) and [x for x in c.copies if x[2] == 2]


def test_relay_forms_with_large_pieces_deliver_every_byte(xg):
    """P8 A4 -d (12 << 20) + 3 on 3 GPUs (pieces of 4 MiB and up: the coalesced form's calls go one
    per piece, in place, its relayed pieces received and forwarded piece by piece -- rc_split -- as at
    configs[4]'s stated size): half-sync and pairwise; every byte where the reference puts it (the
    GPU test runs unordered and TAM too)"""
    P, A, d, G = 8, 4, (12 << 20) + 3, 3
    rl = xg.aggregator_list(P, A)
    n = 0
    for m in (7, 9, 12):
        try:
            s = xg.Schedule(m, P, A, d, 3, rl, ntimes=1, iteration=1)
        except xg.XGError:
            continue
        for form in (RELAY, COALESCED):
            v = s.devplan(G, 0, form[0], 0, form[1])
            if not any(FENCE in [x[0] for x in v.calls(st)] for st in range(v.nsteps)):
                continue
            n += 1
            assert s.check_pairing(G, form[0], 0, form[1]) > 0
            _views, regs = simulate(s, G, it=1, mode=1, pack=form[0], form=form[1])
            check_recv(s, G, regs, it=1, mode=1)
    assert n >= 4, n
