"""libxghost (the product's C host side) against the reference traces and the oracle."""
import subprocess
import os

import pytest

import xg_oracle as O
from conftest import REPO, GOLDEN, golden_configs, load_golden

CONFIGS = golden_configs()


@pytest.mark.parametrize("cfg", CONFIGS)
def test_traces_match_reference(xg, cfg):
    meta, traces, _ = load_golden(cfg)
    rl = xg.aggregator_list(meta["P"], meta["A"], meta["proc_node"], meta["type"])
    assert rl == meta["aggregators"]
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], rl, ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"], barrier_type=meta["barrier"])
        for r in range(meta["P"]):
            assert s.trace(r) == traces[(m, r)], (cfg, m, r)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_steps_match_oracle(xg, cfg):
    meta, _, _ = load_golden(cfg)
    rl = meta["aggregators"]
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], rl, ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"], barrier_type=meta["barrier"])
        progs = O.programs(m, meta["P"], meta["A"], meta["d"], meta["c"], rl, meta["ntimes"], meta["proc_node"],
                           meta["barrier"])
        om = O.match(progs)
        info = {}
        ost, ons = O.asap_steps(progs, om, info=info)
        assert s.barrier_epochs()[1:] == info["barrier_epochs"][1:], (cfg, m)
        mine = sorted((a, b, c, d, n, st) for a, b, c, d, n, st, fl in s.messages() if not fl & 1)
        ref = sorted((a, b, c, d, n, st) for (a, b, c, d, n, _sp, _rp), st in zip(om, ost))
        assert mine == ref, (cfg, m)
        assert s.nsteps >= ons


def test_deadlock_is_reported_not_hung(xg):
    rl = xg.aggregator_list(32, 14)
    xg.Schedule(6, 32, 14, 65424, 3, rl)
    with pytest.raises(xg.XGError, match="deadlocks"):
        xg.Schedule(6, 32, 14, 65425, 3, rl)


@pytest.mark.parametrize("t", [0, 1, 2, 3])
def test_aggregator_types(xg, t):
    for P, A, p in [(32, 14, 1), (24, 7, 4), (256, 64, 8), (12, 5, 3), (7, 7, 2)]:
        assert xg.aggregator_list(P, A, p, t) == O.aggregator_list(P, A, p, t)


def test_labels(xg):
    for m, lab in O.LABELS.items():
        assert xg.method_label(m) == lab
    assert xg.method_label(15) == "All to many TAM" and xg.method_label(21) is None


def test_timer_semantics(xg):
    """Logical clock: each wait advances a rank's clock to the completion time of the
    step it waits on; the reference's MPI_Wtime brackets become clock intervals."""
    rl = xg.aggregator_list(8, 3)
    # m1 unordered: one step; every rank: post bracket, then recv bracket over the waitall
    s = xg.Schedule(1, 8, 3, 64, 1000, rl)
    assert s.nsteps == 1
    t = s.rank_timer(0, [0.005], [0.001])
    assert t.recv_wait_all_time == pytest.approx(0.005) and t.total_time == pytest.approx(0.005)
    assert t.send_wait_all_time == 0
    # m1 throttled (c=2 -> 4 receive phases): aggregator recv_wait = last phase end;
    # a non-aggregator only waits for its sends (send_wait)
    s = xg.Schedule(1, 8, 3, 64, 2, rl)
    done = [0.001 * (i + 1) for i in range(s.nsteps)]
    t_agg = s.rank_timer(0, done)
    assert t_agg.recv_wait_all_time == pytest.approx(done[-1])
    t_non = s.rank_timer(1, done)
    assert t_non.recv_wait_all_time == 0 and t_non.send_wait_all_time > 0
    assert t_non.total_time <= t_agg.total_time + 1e-12


def test_post_time_is_shared_over_posted_requests(xg):
    """A step's host enqueue time is shared over the requests posted in it, so the
    post times of all ranks of one GPU sum to the GPU's enqueue time."""
    rl = xg.aggregator_list(8, 3)
    s = xg.Schedule(1, 8, 3, 64, 1000, rl)       # one step; 8*3 sends + 3*8 recvs = 48 posts
    posts = [s.rank_timer(r, [0.002], [0.008]).post_request_time for r in range(8)]
    assert sum(posts) == pytest.approx(0.008)
    assert posts[0] == pytest.approx(0.008 * 11 / 48)          # aggregator: 8 recvs + 3 sends
    assert posts[1] == pytest.approx(0.008 * 3 / 48)           # non-aggregator: 3 sends
    # two GPUs: each GPU's enqueue time is shared over its own ranks' posts
    posts2 = [s.rank_timer(r, [0.002], [0.008], ngpus=2).post_request_time for r in range(8)]
    assert sum(posts2[:4]) == pytest.approx(0.008) and sum(posts2[4:]) == pytest.approx(0.008)


def test_summarize_results_format(xg, tmp_path, capfd):
    """xg_summarize_results prints exactly the reference's report lines (masked golden)."""
    import re
    T = xg.Timer(0.1, 0.2, 0.3, 0.0, 0.4)
    csvp = str(tmp_path / "results.csv")
    import ctypes
    xg.host().xg_summarize_results(32, 14, 2048, 3, 2, 1, csvp.encode(), b"All to many", T, T)
    ctypes.CDLL(None).fflush(None)
    out = capfd.readouterr().out
    golden = open(os.path.join(GOLDEN, "readme_p32_a14", "report_m1.txt")).read().splitlines()
    # golden = header (2 lines) + per-iteration blocks; one method block = 9 lines
    block = golden[2:11]
    assert re.sub(r"\d+(\.\d+)?", "#", out).splitlines() == block
    rows = open(csvp).read().splitlines()
    assert rows[0].startswith("Method,# of processes,# of aggregators,data size,max comm,ntimes,aggregator type")
    assert rows[1].startswith("All to many,32,14,2048,3,2,1,0.100000,")


def test_cli_usage_matches_reference(pkg):
    exe = os.path.join(os.path.dirname(pkg.__file__), "bin", "test")
    out = subprocess.run([exe, "-h"], capture_output=True, text=True, timeout=30)
    assert out.returncode == 0
    ref = open(os.path.join(GOLDEN, "usage.txt")).read().replace("{argv0}", exe)
    assert out.stderr == ref


def _pairwise(xg, method, P, A, d, k, fast, pn=1, t=1):
    import os
    old = os.environ.get("XG_PAIRWISE_FAST")
    os.environ["XG_PAIRWISE_FAST"] = "1" if fast else "0"
    try:
        return xg.Schedule(method, P, A, d, 8, xg.aggregator_list(P, A, pn, t), ntimes=k)
    finally:
        if old is None:
            del os.environ["XG_PAIRWISE_FAST"]
        else:
            os.environ["XG_PAIRWISE_FAST"] = old


@pytest.mark.parametrize("method", [9, 10])
@pytest.mark.parametrize("P,A,d,k", [(64, 8, 4096, 1), (64, 64, 100, 2), (100, 7, 70000, 2), (37, 5, 1000, 3),
                                     (128, 3, 65424, 1), (48, 48, 8, 1)])
def test_pairwise_fast_form_equals_full_form(xg, method, P, A, d, k):
    """Large-P pairwise leaves out the 0-byte MPI_Sendrecv rounds (P^2 of them) and syncs each
    rank to the round before its next exchange instead: the same messages in the same steps,
    the same step count and the same rank timers as the full form, for power-of-two (XOR)
    and shift rounds, both directions, eager and rendezvous sizes, -k repetitions."""
    import random
    full = _pairwise(xg, method, P, A, d, k, fast=False)
    fast = _pairwise(xg, method, P, A, d, k, fast=True)
    assert fast.nsteps == full.nsteps == k * P
    key = lambda m: (m[0], m[2], m[1], m[3], m[5])
    want = sorted((m for m in full.messages() if m[4] > 0), key=key)
    got = sorted(fast.messages(), key=key)
    assert [m[:6] for m in got] == [m[:6] for m in want]
    rng = random.Random(P * 31 + k)
    done, t = [], 0.0
    for _ in range(full.nsteps):
        t += rng.uniform(0.0, 2e-6)
        done.append(t)
    for r in range(P):
        a, b = full.rank_timer(r, done).as_tuple(), fast.rank_timer(r, done).as_tuple()
        assert a == b, (r, a, b)


@pytest.mark.parametrize("method", [9, 10])
def test_pairwise_fast_form_trace_is_not_the_reference_trace(xg, method):
    """XG_PAIRWISE_FAST=1 (the default above P = 1024) drops the 0-byte MPI_Sendrecv rounds, so
    xg_sched_trace is then NOT the reference's call trace (include/xg_sched.h says so): pinned
    here at the README size, where the full form reproduces the golden trace.  The fast trace
    is exactly the reference trace's byte-carrying posts (a one-sided round becomes a single
    blocking send or receive), with its own completion tokens."""
    meta, traces, _ = load_golden("readme_p32_a14")
    P, A = meta["P"], meta["A"]
    full = _pairwise(xg, method, P, A, meta["d"], meta["ntimes"], fast=False)
    fast = _pairwise(xg, method, P, A, meta["d"], meta["ntimes"], fast=True)
    posts = lambda tr: [t for t in tr.split() if t[0] in "sir" and not t.endswith(":0")]
    differs = 0
    for r in range(P):
        ref = traces[(method, r)]
        assert full.trace(r) == ref
        assert posts(fast.trace(r)) == posts(ref), r
        differs += fast.trace(r) != ref
    assert differs > 0
