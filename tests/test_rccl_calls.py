"""The RCCL calls of a multi-GPU job (libxghost calls.c) -- the code the driver's 8-GPU run
executes and no one-GPU box can: what each GPU posts per step (xg_devplan_step_calls, the
list enqueue_step posts) and whether RCCL pairs those calls step by step (xg_calls_match:
per ordered GPU pair, the k-th send with the k-th receive over the whole run, as RCCL's
per-peer FIFO does).  Every golden configuration x method, every BASELINE configuration,
G = 2..8, direct and packed; bench.py's own call sequence (tuning passes included) on G
processes; and the matcher's refusals."""
import json
import hashlib
import os
import subprocess
import sys

import pytest

from conftest import REPO, golden_configs, load_golden

CONFIGS = golden_configs()
# direct (one call per segment), packed one-sided (runs; the default packed form), packed
# two-sided (one staging buffer per peer and direction)
PACKS = ((0, -1), (4 << 20, 1), (4 << 20, 0))
# ... and the relay forms (two RCCL groups in a permutation step; tests/test_relay.py)
PACKS_RELAY = PACKS + ((0, 2), (0, 3))


def _ref_pairs(views):
    """Independent restatement of the pairing, per step (tests/plan_exec.py's rule): in
    each step, the k-th send of g to h with the k-th receive of h from g."""
    G = len(views)
    out = []
    for st in range(views[0].nsteps):
        calls = [v.calls(st) for v in views]
        for g in range(G):
            for h in range(G):
                sends = [i for i, c in enumerate(calls[g]) if c[0] == 1 and c[1] == h]
                recvs = [i for i, c in enumerate(calls[h]) if c[0] == 2 and c[1] == g]
                assert len(sends) == len(recvs), (st, g, h)
                b0, b1 = views[g].steps[st][2], views[h].steps[st][2]
                for si, ri in zip(sends, recvs):
                    assert calls[g][si][4] == calls[h][ri][4]
                    out.append((st, g, h, b0 + si + sum(views[g].sync_after[:st]),
                                b1 + ri + sum(views[h].sync_after[:st]), calls[g][si][4]))
    return out


@pytest.mark.parametrize("cfg", CONFIGS)
def test_golden_jobs_pair_step_by_step(xg, cfg):
    """every golden config x method x G = 2..8 x {direct, packed}: RCCL's whole-run FIFO
    pairing puts every send and its receive in the same step, with the same length, and
    every GPU ends the same steps with a barrier"""
    meta, _, _ = load_golden(cfg)
    rl = meta["aggregators"]
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], rl, ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"], barrier_type=meta["barrier"])
        for G in range(2, min(8, meta["P"]) + 1):
            for pack, form in PACKS_RELAY:
                n = s.check_pairing(G, pack, 0, form)
                views = [s.devplan(G, g, pack, 0, form) for g in range(G)]
                assert n == sum(1 for v in views for st in range(v.nsteps) for c in v.calls(st) if c[0] == 1)
                assert all(v.sync_after == views[0].sync_after for v in views)


@pytest.mark.parametrize("cfg", ["readme_p32_a14", "p16_a5_c3_b1", "p24_a7_t3_c1", "p8_a3_d1m_c2"])
def test_pairs_equal_the_per_step_rule(xg, cfg):
    """the C matcher's pairs = an independent per-step pairing, call for call; the step's
    calls are its p2p list then the barrier; the pairs carry every cross-GPU byte"""
    meta, _, _ = load_golden(cfg)
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"], ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"], barrier_type=meta["barrier"])
        for G in (2, 3, 8):
            if G > meta["P"]:
                continue
            for pack, form in PACKS:
                views = [s.devplan(G, g, pack, 0, form) for g in range(G)]
                for v in views:
                    for st in range(v.nsteps):
                        c = v.calls(st)
                        qb, qc = v.steps[st][2], v.steps[st][3]
                        assert [(x[1], x[0] == 1, x[2], x[3], x[4]) for x in c if x[0] != 3] == \
                            [(o[0], bool(o[1]), o[2], o[3], o[4]) for o in v.p2p[qb:qb + qc]]
                        assert [x[0] for x in c].count(3) == v.sync_after[st]
                        assert all(x[0] != 3 for x in c[:-1])          # the barrier is the step's last call
                pairs = xg.devplans_match(views)
                assert pairs == _ref_pairs(views), (cfg, m, G, pack, form)
                assert sum(p[5] for p in pairs) == sum(v.remote_send_bytes for v in views)


# BASELINE.json configs[1..4] at full size (host plans only: nothing is allocated)
BASELINE = [
    ("configs1", 32, 14, 1 << 20, [200000000], (1, 2, 3, 4)),
    ("configs2", 64, 16, 256 << 10, [200000000], (5, 8)),
    ("configs3", 256, 32, 4 << 20, [200000000], (1, 2, 9, 10)),
    ("configs4", 256, 64, 64 << 20, list(range(1, 9)), (7, 11, 12)),
]


@pytest.mark.parametrize("case", BASELINE, ids=[b[0] for b in BASELINE])
def test_baseline_configs_pair_on_2_to_8_gpus(xg, case):
    _, P, A, d, cs, methods = case
    rl = xg.aggregator_list(P, A)
    for m in methods:
        for c in cs:
            s = xg.Schedule(m, P, A, d, c, rl)
            for G in (2, 3, 4, 8):
                for pack, form in PACKS_RELAY:
                    assert s.check_pairing(G, pack, 0, form) > 0


# ---------------------------------------------------------------- the matcher's refusals
S, R, B = 1, 2, 3


def _refused(xg, calls, nsteps, what):
    with pytest.raises(xg.XGError) as e:
        xg.calls_match(calls, nsteps)
    assert what in str(e.value), str(e.value)


def test_matcher_accepts_and_orders_a_valid_job(xg):
    calls = [[[(S, 1, 0, 0, 8), (R, 1, 1, 0, 4)], [(S, 1, 0, 8, 8), (B, -1, -1, 0, 0)]],
             [[(S, 0, 0, 0, 4), (R, 0, 1, 0, 8)], [(R, 0, 1, 8, 8), (B, -1, -1, 0, 0)]]]
    assert xg.calls_match(calls, 2) == [(0, 0, 1, 0, 1, 8), (0, 1, 0, 0, 1, 4), (1, 0, 1, 2, 2, 8)]


def test_matcher_refuses_mismatches(xg):
    # a send nobody receives
    _refused(xg, [[[(S, 1, 0, 0, 8)]], [[]]], 1, "sends and 0 receives")
    # equal counts per channel but the receive one step late: RCCL would pair them across steps
    _refused(xg, [[[(S, 1, 0, 0, 8)], [(S, 1, 0, 8, 8)]], [[], [(R, 0, 1, 0, 8), (R, 0, 1, 8, 8)]]], 2,
             "is posted in step 0, its receive in step 1")
    # lengths differ
    _refused(xg, [[[(S, 1, 0, 0, 8)]], [[(R, 0, 1, 0, 16)]]], 1, "carries 8 bytes, its receive 16")
    # one GPU's in-loop barrier missing
    _refused(xg, [[[(B, -1, -1, 0, 0)]], [[]]], 1, "GPU 0 ends with a barrier")
    # a send posted after the step's barrier
    _refused(xg, [[[(B, -1, -1, 0, 0), (S, 1, 0, 0, 8)]], [[(R, 0, 1, 0, 8), (B, -1, -1, 0, 0)]]], 1,
             "after the step's barrier")
    # per channel: the job's totals agree (3 sends, 3 receives) but GPU 1 takes one receive
    # from GPU 0 for GPU 0's two sends
    _refused(xg, [[[(S, 1, 0, 0, 8), (S, 1, 0, 8, 8)]], [[(R, 0, 1, 0, 8), (R, 2, 1, 8, 8), (R, 2, 1, 16, 8)]],
                  [[(S, 1, 0, 0, 8)]]], 1, "posts 2 sends to GPU 1, which posts 1 receives")
    # a peer out of range
    _refused(xg, [[[(S, 5, 0, 0, 8)]], [[]]], 1, "to peer 5")


# ---------------------------------------------------------------- bench.py's call sequence on G processes
DRIVER = r'''
import os, sys, json
sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "tests"))
import __graft_entry__ as G
import fake_xg
real = G.load_package()
fx = fake_xg.install(real)
sys.argv = ["bench.py"] + {argv!r}
import bench
rc = bench.main()
print("TRACE " + json.dumps(fx.trace))
sys.exit(rc)
'''


@pytest.mark.parametrize("world", [2, 4])
def test_bench_ranks_issue_the_same_collectives(tmp_path, world):
    """bench.py as a G-process job (fake device layer whose barrier and MAX really span the
    processes; REAL host plans): every rank issues the same sequence of barriers, MAX
    reductions, RCCL ceiling runs and plan runs, tuning passes included -- the plans it runs
    are refused up front unless their calls pair (check_pairing in MethodRun)."""
    key = "calls_%s_%s_%d" % (tmp_path.name, hashlib.sha1(str(tmp_path).encode()).hexdigest()[:10], world)
    argv = ["--gpus", str(world), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--watchdog", "200"]
    code = DRIVER.format(repo=REPO, argv=argv)
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), XG_RDZV_KEY=key,
                   XG_FAKE_BARRIER_DIR=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    traces = [json.loads([l for l in o.splitlines() if l.startswith("TRACE ")][0][6:]) for o, _ in outs]
    for r in range(1, world):
        assert traces[r] == traces[0], "rank %d's collective sequence differs from rank 0's" % r
    kinds = [t[0] for t in traces[0]]
    assert kinds.count("plan") == 12              # 4 methods x {direct, packed one-sided, two-sided} candidates
    assert "p2p_bench" in kinds and "allreduce_max" in kinds
    line = json.loads([l for l in outs[0][0].splitlines() if l.startswith("{")][0])
    assert line["n_gpus"] == world and line["pack_autotune_ms_per_run"]


@pytest.mark.parametrize("cfg", ["readme_p32_a14", "p20_a6_c7", "p16_a4_t2_c5"])
def test_self_calls_carry_the_local_part(xg, cfg):
    """XG_SELF_MAX: a cross-GPU step whose local copies move <= self_max bytes lists them as
    self send + receive pairs (peer = its own GPU) after its cross-GPU calls, before the
    barrier; the job still pairs step by step, and the self pairs are exactly those copies"""
    meta, _, _ = load_golden(cfg)
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"], ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"], barrier_type=meta["barrier"])
        for G in (2, 8):
            for pack, form in PACKS:
                views = [s.devplan(G, g, pack, 0, form) for g in range(G)]
                pairs = xg.devplans_match(views, self_max=1 << 30)
                cross = xg.devplans_match(views)
                assert [(p[0], p[1], p[2], p[5]) for p in pairs if p[1] != p[2]] == \
                    [(p[0], p[1], p[2], p[5]) for p in cross]
                for g, v in enumerate(views):
                    for st in range(v.nsteps):
                        c = v.calls(st, self_max=1 << 30)
                        own = [x for x in c if x[0] != 3 and x[1] == g]
                        pb, pc = v.steps[st][0], v.steps[st][1]
                        sc = v.stage_count[st]
                        local = [cp for cp in v.copies[pb + sc: pb + pc] if cp[2] != 2 and cp[4] > 0]
                        if not v.steps[st][3]:              # no cross-GPU call: nothing moves into a group
                            assert not own
                            continue
                        assert [(x[0], x[2], x[3], x[4]) for x in own] == \
                            [t for cp in local for t in ((1, cp[0], cp[1], cp[4]), (2, cp[2], cp[3], cp[4]))]
                        assert [x for x in c if x[0] == 3 or x[1] != g] == v.calls(st)   # cross calls + barrier as before
                        assert not own or c.index(own[0]) == len(v.calls(st)) - v.sync_after[st]   # after the cross calls


def test_bench_ranks_with_different_arguments_refuse_alike(tmp_path):
    """ranks started with different arguments would plan different RCCL calls and hang: every
    rank compares a digest of its arguments (one MAX reduction) and all stop with the reason"""
    key = "calls_args_%s_%s" % (tmp_path.name, hashlib.sha1(str(tmp_path).encode()).hexdigest()[:10])
    procs = []
    for r, steps in ((0, "2"), (1, "3")):
        argv = ["--gpus", "2", "--steps", steps, "--warmup", "1", "--no-cpu-baseline", "--watchdog", "120"]
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE="2", XG_RDZV_KEY=key,
                   XG_FAKE_BARRIER_DIR=str(tmp_path))
        procs.append(subprocess.Popen([sys.executable, "-c", DRIVER.format(repo=REPO, argv=argv)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (_o, e) in zip(procs, outs):
        assert p.returncode != 0 and "different arguments" in e, e[-2000:]
