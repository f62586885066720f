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


@pytest.mark.parametrize("cfg", ["readme_p32_a14", "p20_a6_c7", "p24_a7_t3_c1"])
def test_graph_replay_post_time_reaches_every_post(xg, cfg):
    """a graph replay posts the whole run in one launch; xg_plan_run shares that launch
    time out over the steps in proportion to xg_stepplan.posts (the request posts of the GPU's
    ranks in each step).  Then every post costs the same share, a step without posts gets none
    (no Timer would read it), and for the methods whose post bracket holds all of a rank's posts
    the GPU's ranks' post_request_time sum to the launch time exactly."""
    meta, _, _ = load_golden(cfg)
    whole = {1, 2, 4, 13, 14, 17, 18}            # post bracket around every request post
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"], ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"], barrier_type=meta["barrier"])
        for G in (1, 2, 4):
            for g in range(G):
                v = s.devplan(G, g)
                tot = sum(v.posts)
                lo, hi = s.block_range(G, g)
                if not tot or hi <= lo:
                    continue
                T = 2.5e-5                                    # the replay's launch time
                post = [T * x / tot for x in v.posts]         # exec.hip, graph branch of xg_plan_run
                assert abs(sum(post) - T) < 1e-15 and all(p == 0 for p, x in zip(post, v.posts) if not x)
                done = [0.0] * v.nsteps
                got = sum(s.rank_timer(r, done, post, G).post_request_time for r in range(lo, hi))
                assert got <= T * (1 + 1e-9), (cfg, m, G, g, got)
                if m in whole:
                    assert abs(got - T) < 1e-12, (cfg, m, G, g, got)
