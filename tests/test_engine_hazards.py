"""Step-engine barrier flags (xg_engine_hazards, csrc/host/hazard.c) on the CPU.

The engine arrives at a step barrier as soon as its stores are issued and loads
the next step's first unit early; that is only valid when the next step reads
nothing written since the last ordering point and rewrites such bytes only with
identical bytes.  Flag 2 marks every other boundary (drain + release/acquire, no
early load), flag 1 the last step (its stamp anchors the step times).
"""
import pytest

SEND, RECV = 0, 1 << 40          # stand-in base addresses of two regions


def test_identical_rewrites_are_not_hazards(xg):
    s = [(SEND, RECV, 4096)]
    flags, n = xg.engine_hazards([s, s, s])
    assert flags == [0, 0, 1] and n == 0


def test_read_after_write_is_a_hazard(xg):
    flags, n = xg.engine_hazards([[(SEND, RECV, 4096)], [(RECV + 100, RECV + 8192, 16)]])
    assert flags == [2, 1] and n == 1


def test_rewrite_with_other_bytes_is_a_hazard(xg):
    flags, n = xg.engine_hazards([[(SEND, RECV, 4096)], [(SEND + 4096, RECV + 2048, 4096)]])
    assert flags == [2, 1] and n == 1


def test_partial_rewrite_same_offset_is_not(xg):
    # the second step rewrites half the slot from the matching half of the same source
    flags, n = xg.engine_hazards([[(SEND, RECV, 8192)], [(SEND + 4096, RECV + 4096, 4096)]])
    assert flags == [0, 1] and n == 0


def test_write_after_read_needs_no_flag(xg):
    # loads of a step have returned before its stores issue, so the barrier orders them
    flags, _ = xg.engine_hazards([[(RECV, RECV + 65536, 4096)], [(SEND, RECV, 4096)]])
    assert flags == [0, 1]


def test_hazard_point_clears_pending_writes(xg):
    a = [(SEND, RECV, 4096)]
    b = [(RECV, RECV + 8192, 4096)]          # reads a's output: hazard after step 0
    c = [(SEND + 8192, RECV, 4096)]          # rewrites a's bytes, but a was ordered: only b pending
    flags, n = xg.engine_hazards([a, b, c])
    assert flags == [2, 0, 1] and n == 1


def test_force_drains_every_step_and_keeps_hazards(xg):
    flags, n = xg.engine_hazards([[(SEND, RECV, 64)], [(RECV, RECV + 64, 64)], [(SEND, RECV + 128, 64)]], force=True)
    assert flags == [2, 1, 1] and n == 1


def test_empty_transfers_are_ignored(xg):
    flags, n = xg.engine_hazards([[(SEND, RECV, 0)], [(RECV, RECV, 0)], []])
    assert flags == [0, 0, 1] and n == 0


def _spans(view, base):
    steps = []
    for (pb, pc, _q, _n, _b, _c) in view.steps:
        steps.append([(base[sb] + so, base[db] + do, ln) for (sb, so, db, do, ln) in view.copies[pb:pb + pc]])
    return steps


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("method", [1, 3, 6, 7, 9, 10, 11, 12, 13, 18])
def test_real_plans_have_no_hazards(xg, method, k):
    """Every GPU-local schedule only reads SEND and writes RECV; the -k repetitions
    rewrite the same slots with the same bytes -- so no engine barrier needs more
    than the last step's drain (the property the engine's early loads rest on)."""
    P, A, d, c = 32, 14, 2048, 3
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=4, barrier_type=1)
    v = s.devplan(1, 0)
    base = {b: (b + 1) << 40 for b in range(xg.NBUF)}
    flags, n = xg.engine_hazards(_spans(v, base))
    assert n == 0 and flags[-1] == 1 and all(f == 0 for f in flags[:-1]), (method, k, flags)


@pytest.mark.parametrize("method", [15, 16])
def test_tam_plans_have_hazards_where_scratch_is_read_back(xg, method):
    """TAM stages rank data in SCRATCH and reads it back later.  With each plan step cut
    into its stage copies, then its local copies, the scan puts a hazard barrier before
    every step that reads SCRATCH written since the previous hazard point (checked
    against a direct interval walk).  Those barriers are why TAM plans stay outside the
    engine: in the grid engine they cost 59-61 us at the README size against 29 us for
    per-step launches (profiles/r02/tam_engine/)."""
    P, A, d, c = 32, 14, 2048, 3
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=2, proc_node=4)
    v = s.devplan(1, 0)
    base = {b: (b + 1) << 40 for b in range(xg.NBUF)}
    steps = []
    for i, (pb, pc, _q, _n, _b, _c) in enumerate(v.steps):
        cp = [(base[sb] + so, base[db] + do, ln) for (sb, so, db, do, ln) in v.copies[pb:pb + pc]]
        ns = v.stage_count[i]
        if ns:
            steps.append(cp[:ns])
        if pc > ns or not ns:
            steps.append(cp[ns:])
    flags, n = xg.engine_hazards(steps)
    assert n > 0 and flags[-1] >= 1
    # reference walk: pending written bytes since the last flag-2 barrier
    pend = []
    for t, st in enumerate(steps):
        if t and any(lo < sa + ln and sa < hi for (sa, _da, ln) in st if ln for (lo, hi) in pend):
            assert flags[t - 1] == 2, (t, flags)
            pend = []
        if flags[t] == 2:
            pend = []
        else:
            pend += [(da, da + ln) for (_sa, da, ln) in st if ln]
