"""Multi-GPU device plans (libxghost xg_devplan_build), executed on the CPU.

Block mapping of logical ranks onto G GPUs, local copies vs grouped p2p,
pack/unpack staging vs one op per segment: every received byte must equal
the oracle's closed form, for every method, G in 1..8 and both p2p modes.
"""
import pytest

import xg_oracle as O
from plan_exec import check_recv, simulate

# direct (one call per segment), packed two-sided (pack + unpack), packed one-sided (runs)
FORMS = ((0, -1), (1 << 20, 0), (1 << 20, 1))

CASES = [  # P, A, d, c, ntimes, type, proc_node
    (32, 14, 40, 3, 2, 1, 1),      # README shape (reduced d), throttled
    (20, 6, 24, 7, 3, 1, 1),
    (24, 7, 16, 1, 1, 3, 4),       # unsorted aggregator list
    (16, 16, 8, 5, 1, 0, 1),       # every rank an aggregator
    (13, 4, 33, 200000000, 2, 1, 1),
    (18, 5, 20, 4, 2, 1, 5),       # TAM nodes of 5, 5, 5, 3 ranks
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("G", [1, 2, 3, 4, 8])
def test_plans_deliver_every_byte(xg, case, G):
    P, A, d, c, k, t, pn = case
    if G > P:
        pytest.skip("more GPUs than ranks")
    rl = xg.aggregator_list(P, A, pn, t)
    for m in O.METHODS:
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=k, proc_node=pn, barrier_type=(m * G) % 3)
        for pack, form in FORMS:
            views, regs = simulate(s, G, it=1, mode=1, pack=pack, form=form)
            check_recv(s, G, regs, it=1, mode=1)
            if G > 1 and m in (13, 17, 19):     # in-loop barriers become device-side barriers
                assert all(v.sync_after == views[0].sync_after for v in views)
                assert sum(views[0].sync_after) >= 1 or m == 13


P256_CASES = [  # (A, d, c, methods): configs[3] and configs[4]'s shapes at reduced -d
    (32, 48, 200000000, (1, 2, 9, 10)),
    (64, 16, 1, (7, 11, 12)),
    (64, 16, 3, (7, 11, 12)),
    (64, 16, 8, (7, 11, 12)),
]


@pytest.mark.parametrize("case", P256_CASES, ids=lambda c: "A%d_d%d_c%d" % c[:3])
def test_p256_plans_deliver_every_byte(xg, case):
    """The plans the 8-GPU run of configs[3] / configs[4] executes (P = 256, 32 or 64 ranks per
    GPU, 32 / 64 aggregators), at a reduced -d, through the race-checked executor: direct,
    two-sided and one-sided, every received byte against the closed form"""
    A, d, c, methods = case
    P, G = 256, 8
    rl = xg.aggregator_list(P, A)
    for m in methods:
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=2, iteration=1)
        for pack, form in FORMS:
            _views, regs = simulate(s, G, it=1, mode=1, pack=pack, form=form)
            check_recv(s, G, regs, it=1, mode=1)


def test_pack_decision_and_volume(xg):
    """Two-sided packing: >= 2 segments to a peer with mean < pack_max_seg -> one RCCL op per
    peer and direction."""
    P, A, d = 32, 14, 1024
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(1, P, A, d, 200000000, rl)
    G = 8
    tot_local = tot_remote = 0
    for g in range(G):
        packed = s.devplan(G, g, pack_max_seg=1 << 20, pack_form=xg.PACK_TWO_SIDED)
        direct = s.devplan(G, g, pack_max_seg=0)
        peers = {o[0] for o in packed.p2p}
        # one send and one recv per peer in the single step when packed
        assert len(packed.p2p) == 2 * len(peers)
        assert len(direct.p2p) > len(packed.p2p)
        assert packed.remote_send_bytes == direct.remote_send_bytes
        assert packed.region_bytes[2] == packed.remote_send_bytes
        tot_local += packed.local_bytes
        tot_remote += packed.remote_send_bytes
    assert tot_local + tot_remote == P * A * d


def test_region_sizes(xg):
    P, A, d = 32, 14, 4096
    rl = xg.aggregator_list(P, A)
    for m in (1, 2):
        s = xg.Schedule(m, P, A, d, 200000000, rl)
        for G in (1, 2, 4, 8):
            tot_send = sum(s.region_bytes(G, g, 0) for g in range(G))
            tot_recv = sum(s.region_bytes(G, g, 1) for g in range(G))
            assert tot_send == tot_recv == P * A * d


def _random_cases(seed, n):
    import random
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        P = rng.choice([2, 3, 5, 7, 9, 12, 16, 19, 24])
        out.append((rng.randint(1, 20), P, rng.randint(1, P), rng.choice([1, 5, 16, 24, 40]),
                    rng.choice([1, 2, 3, 5, 200000000]), rng.randint(1, 3), rng.randint(0, 3),
                    rng.choice([1, 2, 3, 4]), rng.randint(0, 2), rng.choice([2, 3, 4, 8])))
    return out


@pytest.mark.parametrize("case", _random_cases(11, 200), ids=lambda c: "m%d_P%d_A%d_d%d_c%d_k%d_t%d_pn%d_b%d_G%d" % c)
def test_random_plans_deliver_every_byte(xg, case):
    """Seeded random shapes (every method, placement type, barrier type, -c, -k, proc_node)
    as G-GPU jobs, packed and direct, through the race-checked executor."""
    m, P, A, d, c, k, t, pn, b, G = case
    G = min(G, P)
    rl = xg.aggregator_list(P, A, pn, t)
    try:
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=k, proc_node=pn, barrier_type=b, iteration=2)
    except xg.XGError as e:
        pytest.skip("refused schedule: %s" % e)
    for pack, form in FORMS:
        _views, regs = simulate(s, G, it=2, mode=1, pack=pack, form=form)
        check_recv(s, G, regs, it=2, mode=1)


def test_pack_min_keeps_small_peer_lists_direct(xg):
    """pack_min (the CLI default 64 KiB): a (step, peer) list of >= 2 segments is packed only
    when it also moves >= pack_min bytes; both ends decide alike, so the plans still pair and
    deliver every byte"""
    P, A = 32, 14
    rl = xg.aggregator_list(P, A)
    for d, expect_packed in ((2048, False), (1 << 20, True)):
        s = xg.Schedule(1, P, A, d, 200000000, rl)
        G = 8
        views = [s.devplan(G, g, 4 << 20, 64 << 10) for g in range(G)]
        packed = any(o[2] == 2 for v in views for o in v.p2p)          # a send from STAGE_SEND
        assert packed == expect_packed, d
        s.check_pairing(G, 4 << 20, 64 << 10)
    s = xg.Schedule(6, P, A, 40, 3, rl, ntimes=2)
    _views, regs = simulate_min(s, 8)
    check_recv(s, 8, regs)


def simulate_min(s, G):
    import plan_exec
    orig = s.devplan
    s.devplan = lambda ng, g, pack=1 << 20, _pm=0, form=-1: orig(ng, g, pack, 64 << 10, form)
    try:
        return plan_exec.simulate(s, G)
    finally:
        s.devplan = orig


def _copied(view):
    """bytes a plan copies through staging: (packed, unpacked)"""
    return (sum(c[4] for c in view.copies if c[2] == 2), sum(c[4] for c in view.copies if c[0] == 3))


@pytest.mark.parametrize("m", [5, 8, 1, 2])
def test_one_sided_runs_at_configs2(xg, m):
    """configs[2] (P64 A16, -d 256 KiB) on 8 GPUs: the one-sided form sends, per peer, one run per
    receiving aggregator (all-to-many: 8 senders' segments land contiguous in its slots) or per
    sending aggregator (many-to-all), copies every cross-GPU byte on ONE side only -- half the
    two-sided form's pack + unpack bytes -- and still delivers every byte."""
    P, A, d, G = 64, 16, 256 << 10, 8
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(m, P, A, d, 200000000, rl)
    a2m = m in (1, 8)
    for g in range(G):
        one = s.devplan(G, g, 4 << 20, 0, xg.PACK_ONE_SIDED)
        two = s.devplan(G, g, 4 << 20, 0, xg.PACK_TWO_SIDED)
        assert one.remote_send_bytes == two.remote_send_bytes == 7 * 8 * 2 * d
        pk1, up1 = _copied(one)
        pk2, up2 = _copied(two)
        assert pk2 == up2 == one.remote_send_bytes
        # a2m: gathered by the sender, received straight into the slots; m2a: sent straight
        # from the aggregator's segments, scattered by the receiver
        assert (pk1, up1) == ((one.remote_send_bytes, 0) if a2m else (0, one.remote_send_bytes))
        for peer in range(G):
            if peer == g:
                continue
            sends = [o for o in one.p2p if o[0] == peer and o[1]]
            recvs = [o for o in one.p2p if o[0] == peer and not o[1]]
            # 2 aggregators per GPU: 2 runs of 8 segments (2 MiB) each way
            assert [o[4] for o in sends] == [o[4] for o in recvs] == [8 * d, 8 * d]
            assert all(o[2] == (2 if a2m else 0) for o in sends)
            assert all(o[2] == (1 if a2m else 3) for o in recvs)
    s.check_pairing(G, 4 << 20, 0, xg.PACK_ONE_SIDED)
    _views, regs = simulate(s, G, it=1, mode=1, pack=4 << 20, form=xg.PACK_ONE_SIDED)
    check_recv(s, G, regs, it=1, mode=1)


def test_one_sided_moves_contiguous_runs_without_copies(xg):
    """A run contiguous at both ends moves as one call straight between the regions: one
    aggregator (rank 0) and 8 ranks on 2 GPUs -- GPU 1's four senders hold their one segment
    each back to back, and they land in four consecutive slots of the aggregator."""
    P, A, d, G = 8, 1, 4096, 2
    rl = xg.aggregator_list(P, A)
    for m in (8, 1):
        s = xg.Schedule(m, P, A, d, 200000000, rl)
        v0, v1 = (s.devplan(G, g, 4 << 20, 0, xg.PACK_ONE_SIDED) for g in range(G))
        assert _copied(v0) == _copied(v1) == (0, 0)
        assert [o[1:5] for o in v1.p2p] == [(1, 0, 0, 4 * d)]                      # SEND, offset 0
        assert [o[1:5] for o in v0.p2p] == [(0, 1, s.recv_offset(G, 0) + 4 * d, 4 * d)]
        _views, regs = simulate(s, G, it=0, mode=1, pack=4 << 20, form=xg.PACK_ONE_SIDED)
        check_recv(s, G, regs, it=0, mode=1)
