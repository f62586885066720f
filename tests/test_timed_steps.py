"""A timed run marks only the steps whose completion time some rank's Timer reads
(xg_sched_timed_steps -> xg_plan_set_step_marks); every other step is reported as done with the
next marked one.  That must change no Timer field of any rank: checked here for every method of
every reference-captured configuration (golden and BASELINE shapes) on random non-decreasing step
times, method Timer and m13's per-repetition timers alike (exact equality, not a tolerance: the
clock of a rank at a bracket is the time of the one step it reads there)."""
import random

import pytest

from conftest import baseline_configs, golden_configs, load_baseline, load_golden


def _filled(done, need):
    out = list(done)
    for s in range(len(out) - 2, -1, -1):
        if not need[s]:
            out[s] = out[s + 1]
    return out


def _check(xg, s, rng, tag, trials=3, gpus=(1, 4)):
    need = s.timed_steps()
    assert len(need) == s.nsteps and (not need or need[-1] == 1), tag
    for _trial in range(trials):
        done = [0.0] * s.nsteps
        t = 0.0
        for i in range(s.nsteps):
            t += rng.choice([0.0, rng.random()])
            done[i] = t
        post = [rng.random() * 1e-3 for _ in range(s.nsteps)]
        fill = _filled(done, need)
        for r in range(s.P):
            for G in gpus:
                a, b = s.rank_timer(r, done, post, G), s.rank_timer(r, fill, post, G)
                assert a.as_tuple() == b.as_tuple(), (tag, r, G)
            if s.method == 13:
                ra = [x.as_tuple() for x in s.rank_rep_timers(r, done, post)]
                rb = [x.as_tuple() for x in s.rank_rep_timers(r, fill, post)]
                assert ra == rb, (tag, r)
    return need


@pytest.mark.parametrize("cfg", golden_configs())
def test_unmarked_steps_change_no_timer(xg, cfg):
    meta, _, _ = load_golden(cfg)
    rng = random.Random(cfg)
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"], ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"], barrier_type=meta["barrier"])
        _check(xg, s, rng, (cfg, m))


@pytest.mark.parametrize("cfg", baseline_configs())
def test_unmarked_steps_change_no_timer_at_baseline_shapes(xg, cfg):
    meta, _, _ = load_baseline(cfg)
    rng = random.Random(cfg)
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"], ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"])
        need = _check(xg, s, rng, (cfg, m), trials=1, gpus=(8,))
        if m in (9, 10):      # pairwise: only the total is timed -- one mark for the whole run
            assert sum(need) == 1 and s.nsteps == meta["P"] * meta["ntimes"], (cfg, m, sum(need), s.nsteps)


def test_readme_configuration_marks(xg):
    """README configuration (P32 A14 -d 2048 -c 3): the unordered / balanced / half-sync methods
    read every step, pairwise only its last, and m6's blocking rounds -- spread by the step
    compiler over 38 steps -- only the 21 that close some rank's round"""
    rl = xg.aggregator_list(32, 14)
    got = {}
    for m in (1, 2, 3, 4, 6, 7, 9, 10, 11, 12):
        s = xg.Schedule(m, 32, 14, 2048, 3, rl)
        got[m] = (s.nsteps, sum(s.timed_steps()))
        _check(xg, s, random.Random(m), m)
    assert got == {1: (11, 11), 2: (11, 11), 3: (11, 11), 4: (11, 11), 6: (38, 21), 7: (5, 5), 9: (32, 1),
                   10: (32, 1), 11: (22, 22), 12: (38, 29)}, got
