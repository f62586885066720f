"""The solo engine's tables (csrc/host/solo.c xg_solo_tables) on the CPU: an interpreter
that executes them exactly as kernels.h solo_engine_kernel does -- per rail, rows of 16
pieces, `before` barriers ahead of each wave's store, the row's barrier count in all,
barrier k stamping the step meta lists for it, the spare chunk never stored -- checks
that every piece of every step is stored exactly once, by some rail, between the barrier
closing the rail's previous step and the one closing its own, and that the rails stay
balanced.  Random segments and the real G = 1 plans of the README-config chains."""
import random

import pytest


PIECE, K, MAXP = 1024, 8, 4608
LEN_BITS = {16: 7, 4: 9, 1: 11}      # kernels.h SoloFmt


def decode(d, G=16, row_word=None):
    """(src, dst, len in granules, before); row_word given: the WIDE form of one-wave rails
    (32-bit offsets in the descriptor, the length in the row's barrier word, every barrier
    of the row before its one piece)"""
    if row_word is not None:
        return d & 0xFFFFFFFF, d >> 32, (row_word >> 8) & 0xFFF, row_word & 0xFF
    L = LEN_BITS[G]
    return d & 0xFFFFFF, (d >> 24) & 0xFFFFFF, (d >> 48) & ((1 << L) - 1), d >> (48 + L)


def interpret(steps, rails_max, sbase, dbase, xg, WAVES=16, G=16):
    """WAVES: pieces per row = waves per rail (16: a workgroup; 1: a single wave);
    G: the descriptors' granule (offsets and lengths in G-byte units)"""
    rc, shape, descs, close, csteps, rows = xg.solo_tables(steps, rails_max, sbase, dbase, waves=WAVES, granule=G)
    assert rc == 0, (rc, shape)
    R, npc, nr = shape["rails"], shape["npieces"], shape["nrows"]
    n = len(steps)
    total = sum((x[2] + PIECE - 1) // PIECE for st in steps for x in st)
    assert R == max(1, min(rails_max, total // WAVES))
    assert npc % (WAVES * K) == 0 and (npc // (WAVES * K)) % 2 == 1      # even chunks + the spare
    # the steps each (src, dst) piece belongs to (the -k repetitions move identical pieces)
    owner = {}
    for t, st in enumerate(steps):
        for (s, d, ln) in st:
            for o in range(0, ln, PIECE):
                owner.setdefault((s + o, d + o), []).append((t, min(PIECE, ln - o)))
    left = {key: list(v) for key, v in owner.items()}
    per_rail = []
    for r in range(R):
        nb = sum((x & 0xFF) if WAVES == 1 else x for x in close[r])
        cs = csteps[r]
        assert all(c >= 0 for c in cs[:nb]) and all(c == -1 for c in cs[nb:]), cs
        assert all(a < b for a, b in zip(cs[:nb], cs[1:nb])), cs       # closed steps increase
        assert nr - K >= 0
        k0 = 0                       # barriers before this row
        real = 0
        rail_steps = []
        for row in range(nr):
            nrow = close[r][row] & 0xFF if WAVES == 1 else close[r][row]
            assert nrow <= WAVES
            prev_bf = 0
            for w in range(WAVES):
                so, do, l16, bf = decode(descs[r][row * WAVES + w], G, close[r][row] if WAVES == 1 else None)
                assert bf <= nrow and bf >= prev_bf
                prev_bf = bf
                if l16 == 0:
                    assert so == 0 and do == 0
                    continue
                assert row < nr - K, "a piece in the spare chunk is never stored"
                assert row < rows[r], "the kernel stops after the rows the table says are real"
                real += 1
                key = (sbase + so * G, dbase + do * G)
                assert key in owner, key
                kb = k0 + bf                 # barriers executed before this store
                lo = cs[kb - 1] + 1 if kb > 0 else 0          # it must belong to a step in [lo, hi]
                hi = cs[kb] if kb < nb else n - 1
                # a barrier closes the step of every piece stored since the one before it; the
                # -k repetitions hold identical pieces in several steps, so pick by that rule
                # (after the rail's last barrier: its final step, the latest candidate)
                fit = [x for x in left[key] if (x[0] == hi if kb < nb else lo <= x[0] <= hi)]
                assert fit, ("stored outside its step's barriers, or twice", r, row, w, lo, hi, owner[key])
                pick = fit[0] if kb < nb else max(fit)
                t, ln = pick
                left[key].remove(pick)
                assert l16 * G == ln
                rail_steps.append(t)
            assert nrow == 0 or row < rows[r], "a barrier in a row the kernel skips"
            k0 += nrow
        assert k0 == nb
        assert rows[r] == (real + WAVES - 1) // WAVES
        assert rail_steps == sorted(rail_steps), "a rail stores its steps in order"
        # every step the rail had pieces in is closed by a barrier, or is its last one
        used = sorted(set(rail_steps))
        assert used[:-1] == [c for c in cs[:nb] if c in used[:-1]] and set(cs[:nb]) == set(used[:-1])
        per_rail.append(real)
    assert not any(left.values()), "every piece stored"
    assert max(per_rail) - min(per_rail) <= 1, per_rail
    return shape


def random_steps(rng, nsteps, sbase, dbase, G=16):
    steps, so, do = [], 0, 0
    for _ in range(nsteps):
        st = []
        for _ in range(rng.choice([0, 1, 1, 2, 3, 5])):
            ln = G * rng.randint(1, 300 * 16 // G)
            st.append((sbase + so, dbase + do, ln))
            so += ln + G * rng.randint(0, 4)
            do += ln + G * rng.randint(0, 4)
        steps.append(st)
    return steps


@pytest.mark.parametrize("seed", range(10))
@pytest.mark.parametrize("G", [4, 1])
@pytest.mark.parametrize("rails", [1, 7, 64, 512])
def test_random_segments_fine_granules(xg, seed, G, rails):
    """segments whose sizes are not multiples of 16 (any -d): descriptors in 4-B or 1-B
    units on one-wave rails, executed by the same interpreter"""
    rng = random.Random(seed * 131 + G * 7 + rails)
    sbase, dbase = (1 << 32) + G * 3, (3 << 32) + G
    steps = random_steps(rng, rng.randint(1, 60), sbase, dbase, G)
    if not any(steps):
        steps[0].append((sbase, dbase, 1000))
    interpret(steps, rails, sbase, dbase, xg, WAVES=1, G=G)


@pytest.mark.parametrize("seed", range(12))
@pytest.mark.parametrize("rails,waves", [(1, 16), (3, 16), (8, 16), (16, 16), (1, 1), (7, 1), (64, 1), (256, 1)])
def test_random_segments(xg, seed, rails, waves):
    rng = random.Random(seed * 31 + rails + waves)
    sbase, dbase = 1 << 32, 3 << 32
    steps = random_steps(rng, rng.randint(1, 60), sbase, dbase)
    if not any(steps):
        steps[0].append((sbase, dbase, 4096))
    interpret(steps, rails, sbase, dbase, xg, WAVES=waves)


@pytest.mark.parametrize("method", [6, 9, 10, 11, 12, 18])
@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("rails,waves,d", [(16, 16, 2048), (256, 1, 2048), (512, 1, 1000), (512, 1, 33)])
def test_readme_chain_plans(xg, method, k, rails, waves, d):
    """the G = 1 plans of the README configuration (P32 A14 c3; d = 2048, and d = 1000 / 33
    on 4-B / 1-B granules), as build_segments hands them over: one transfer per local
    copy, SEND and RECV at 1 GiB apart"""
    P, A, c = 32, 14, 3
    G = 16 if d % 16 == 0 else 4 if d % 4 == 0 else 1
    s = xg.Schedule(method, P, A, d, c, xg.aggregator_list(P, A), ntimes=k)
    v = s.devplan(1, 0)
    base = {b: (1 << 32) + (b << 30) for b in range(xg.NBUF)}
    steps = []
    for (pb, pn, _qb, _qn, _ob, _on) in v.steps:
        steps.append([(base[sb] + so, base[db] + do, ln) for (sb, so, db, do, ln) in v.copies[pb:pb + pn]])
    while steps and not steps[-1]:
        steps.pop()
    srcs = [x[0] for st in steps for x in st]
    dsts = [x[1] for st in steps for x in st]
    shape = interpret(steps, rails, min(srcs), min(dsts), xg, WAVES=waves, G=G)
    assert shape["rails"] == min(rails, sum((x[2] + PIECE - 1) // PIECE for st in steps for x in st))


def test_rejects(xg):
    sb, db = 1 << 32, 3 << 32
    rc, _s, *_ = xg.solo_tables([[(sb + 8, db, 64)]], 8, sb, db)            # misaligned
    assert rc == 3
    rc, _s, *_ = xg.solo_tables([[(sb, db, 64)]], 8, sb + 16, db)           # below the base
    assert rc == 3
    rc, _s, *_ = xg.solo_tables([[(sb + (1 << 28), db, 64)]], 8, sb, db)   # past the 24-bit window
    assert rc == 3
    rc, shape, *_ = xg.solo_tables([[(sb, db, 1024 * MAXP * 2)]], 1, sb, db)    # too many pieces per rail
    assert rc == 3 and shape["npieces"] > MAXP
    rc, shape, *_ = xg.solo_tables([[(sb, db, 1024 * MAXP * 2)]], 8, sb, db)    # ... which rails spread
    assert rc == 0 and shape["rails"] == 8
    rc, _s, *_ = xg.solo_tables([[(sb, db, 64)]] * 2049, 8, sb, db)         # too many steps
    assert rc == 3
    rc, _s, *_ = xg.solo_tables([[(sb, db, 64)]], 8, sb, db, waves=4)       # rails are 16 waves or 1
    assert rc == 3
    rc, _s, *_ = xg.solo_tables([[(sb, db, 64)]], 513, sb, db, waves=1)     # at most 512 rails
    assert rc == 3
    rc, _s, *_ = xg.solo_tables([[(sb + 2, db, 64)]], 8, sb, db, waves=1, granule=4)   # not 4-B aligned
    assert rc == 3
    rc, _s, *_ = xg.solo_tables([[(sb + 4, db, 68)]], 8, sb, db, waves=1, granule=4)
    assert rc == 0
    rc, _s, *_ = xg.solo_tables([[(sb + 3, db + 1, 1001)]], 8, sb, db, waves=1, granule=1)
    assert rc == 0
    rc, _s, *_ = xg.solo_tables([[(sb + (1 << 24), db, 64)]], 8, sb, db, waves=1, granule=1)   # wide: 4 GiB window
    assert rc == 0
    rc, _s, *_ = xg.solo_tables([[(sb + (1 << 32), db, 64)]], 8, sb, db, waves=1, granule=1)
    assert rc == 3
    rc, _s, *_ = xg.solo_tables([[(sb + (1 << 28), db, 64)]], 8, sb, db, waves=1)             # wide: 64 GiB window
    assert rc == 0
    rc, _s, *_ = xg.solo_tables([[(sb, db, 64)]], 8, sb, db, waves=16, granule=4)   # fine granules: one-wave rails
    assert rc == 3
    rc, _s, *_ = xg.solo_tables([[(sb, db, 64)]], 8, sb, db, waves=1, granule=8)    # 16, 4 or 1
    assert rc == 3


@pytest.mark.parametrize("seed", range(8))
def test_reduce_stamps(xg, seed):
    """step t of a solo segment is over when every rail is: each rail's latest stamp at or
    before t (0 = the rail closed nothing there), MAX over rails; steps outside [s0, s1)
    untouched (0)"""
    rng = random.Random(seed)
    R, n = rng.randint(1, 20), rng.randint(1, 50)
    stamps = [[0] * n for _ in range(R)]
    for r in range(R):
        t0 = rng.randint(1000, 2000)
        for t in range(n):
            t0 += rng.randint(1, 50)
            if rng.random() < 0.3:
                stamps[r][t] = t0
    s0 = rng.randint(0, n - 1)
    s1 = rng.randint(s0 + 1, n)
    got = xg.solo_reduce_stamps(stamps, s0, s1)
    for t in range(n):
        if not s0 <= t < s1:
            assert got[t] == 0
            continue
        exp = max(max([x for x in stamps[r][s0:t + 1] if x] or [0]) for r in range(R))
        assert got[t] == exp, (t, got[t], exp)
    assert all(a <= b for a, b in zip(got[s0:s1], got[s0 + 1:s1]))


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("G", [16, 4, 1])
def test_wide_windows_one_wave_rails(xg, seed, G):
    """one-wave rails address 32-bit granule offsets: transfers spread over GiBs (16384
    logical ranks on one GPU) fit one table"""
    rng = random.Random(seed * 7 + G)
    sbase, dbase = 1 << 40, 1 << 44
    span = min(1 << 32, (1 << 32) * G) - (1 << 20)          # stay inside the window
    steps = []
    for _ in range(rng.randint(2, 40)):
        st = []
        for _ in range(rng.randint(1, 4)):
            ln = G * rng.randint(1, 200 * 16 // G)
            so = rng.randrange(0, span - ln, G)
            do = rng.randrange(0, span - ln, G)
            st.append((sbase + so, dbase + do, ln))
        steps.append(st)
    srcs = [x[0] for st in steps for x in st]
    dsts = [x[1] for st in steps for x in st]
    assert max(srcs) - min(srcs) > (1 << 28) or G == 1     # past the packed form's window
    interpret(steps, rng.choice([1, 16, 512]), min(srcs), min(dsts), xg, WAVES=1, G=G)
