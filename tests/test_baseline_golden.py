"""The BASELINE.json configuration shapes pinned to the REAL reference.

tests/golden/baseline/ holds the reference binary (oracle/_ref/test_capture: the unmodified
mpi_test.c + lustre_driver_test.c objects and the PMPI capture layer) run under MPICH at
configs[1] and configs[2] at full size, configs[3]'s shape (P256 A32) at -d 64 KiB and
configs[4]'s shape (P256 A64) at -d 4 KiB for every -c in 1..8 (tests/golden/make_baseline.py).
Every rank's whole MPI call trace is kept as a sha1 digest, so the product's C scheduler
(libxghost) and the oracle are compared with the reference rank by rank at P = 256 -- the
m7 / m11 / m12 -c caps and their never-reset last-round shrink across -k
(mpi_test.c:1070-1081, :956-967, :1014-1025), pairwise m9 / m10's shift rounds (:421-597).
The GPU side of the same fixtures is tests/test_gpu_baseline.py.
"""
import hashlib

import pytest

import xg_oracle as O
from conftest import baseline_configs, load_baseline

CONFIGS = baseline_configs()


def _sha1(s):
    return hashlib.sha1(s.encode()).hexdigest()


def test_every_baseline_shape_is_captured():
    names = set(CONFIGS)
    assert {"cfg1_p32_a14_d1m", "cfg2_p64_a16_d256k", "cfg3_p256_a32_d64k"} <= names
    assert {"cfg4_p256_a64_d4k_c%d" % c for c in range(1, 9)} <= names
    for name, methods in (("cfg1", [1, 2, 3, 4, 5, 7, 8, 9, 10, 11, 12]), ("cfg2", list(range(1, 13))),
                          ("cfg3", [1, 2, 9, 10]), ("cfg4", [7, 11, 12])):
        for cfg in baseline_configs(name):
            assert load_baseline(cfg)[0]["method_list"] == methods, cfg


@pytest.mark.parametrize("cfg", CONFIGS)
def test_placement(xg, cfg):
    meta, _, _ = load_baseline(cfg)
    P, A = meta["P"], meta["A"]
    assert xg.aggregator_list(P, A, meta["proc_node"], meta["type"]) == meta["aggregators"]
    assert O.aggregator_list(P, A, meta["proc_node"], meta["type"]) == meta["aggregators"]


@pytest.mark.parametrize("cfg", CONFIGS)
def test_c_scheduler_traces_match_reference(xg, cfg):
    """libxghost's per-rank MPI program of every method = the reference's, every rank"""
    meta, samples, _ = load_baseline(cfg)
    rl = meta["aggregators"]
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], rl, ntimes=meta["ntimes"],
                        proc_node=meta["proc_node"])
        for r in range(meta["P"]):
            t = s.trace(r)
            if (m, r) in samples:
                assert t == samples[(m, r)], (cfg, m, r)
            assert _sha1(t) == meta["trace_sha1"][str(m)][r], (cfg, m, r)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_oracle_traces_match_reference(cfg):
    meta, _, _ = load_baseline(cfg)
    rl = meta["aggregators"]
    for m in meta["method_list"]:
        progs = O.programs(m, meta["P"], meta["A"], meta["d"], meta["c"], rl, meta["ntimes"], meta["proc_node"])
        for r in range(meta["P"]):
            assert _sha1(O.trace_tokens(progs[r])) == meta["trace_sha1"][str(m)][r], (cfg, m, r)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_closed_form_checksums_match_reference(cfg):
    """every captured segment: the reference's checksum = chk64 of the oracle's MAP_DATA
    fingerprint (mpi_test.c:71-77; one checksum per (rank + seed + iter) mod 256 and -d), and
    the union over methods covers every (rank, aggregator) pair of every iteration"""
    meta, _, data = load_baseline(cfg)
    P, A, d, rl = meta["P"], meta["A"], meta["d"], meta["aggregators"]
    aggidx = {g: i for i, g in enumerate(rl)}
    memo = {}
    for direction, table in data.items():
        assert len(table) == P * A * meta["iters"], (cfg, direction)
        for (it, src, dst), (n, chk) in table.items():
            seed = aggidx[dst] if direction == "a2m" else dst
            key = (src + seed + it) & 0xFF
            if key not in memo:
                memo[key] = O.chk64(O.map_data(src, seed, it, d))
            assert n == d and chk == memo[key], (cfg, direction, it, src, dst)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_uncaptured_pairs_are_self_copies(cfg):
    """PMPI sees every pair except the aggregator self-memcpys of m3 / m4 (mpi_test.c:1473, :1646)"""
    meta, _, _ = load_baseline(cfg)
    for m, info in meta["methods"].items():
        if info["status"] == "timeout":
            continue
        assert info["status"] == "ok" and info["layout_ok"], (cfg, m)
        want = meta["A"] * meta["iters"] if int(m) in (3, 4, 6) else 0      # m6's memcpy: mpi_test.c:1714
        assert info["uncaptured_pairs"] == want, (cfg, m)


def test_reference_hangs_where_the_step_compiler_predicts_a_deadlock(xg):
    """configs[1] m6 (all_to_many_sync, 1 MiB segments past MPICH's 65,424-byte eager limit): the
    reference run did not finish in 90 s, and the step compiler refuses the schedule as deadlocked
    (so does the oracle); configs[2] m6 (256 KiB, also past the limit) the reference completes
    and the compiler accepts.  Every other captured method completes and is accepted."""
    hung = []
    for cfg in CONFIGS:
        meta, _, _ = load_baseline(cfg)
        rl = meta["aggregators"]
        for m, info in meta["methods"].items():
            m = int(m)
            args = (m, meta["P"], meta["A"], meta["d"], meta["c"], rl)
            if info["status"] == "timeout":
                hung.append((cfg, m))
                with pytest.raises(xg.XGError, match="deadlocks"):
                    xg.Schedule(*args, ntimes=meta["ntimes"])
                with pytest.raises(RuntimeError, match="deadlock"):
                    O.asap_steps(O.programs(*args, meta["ntimes"]))
            else:
                xg.Schedule(*args, ntimes=meta["ntimes"])
    assert hung == [("cfg1_p32_a14_d1m", 6)]


@pytest.mark.parametrize("cfg", baseline_configs("cfg4"))
def test_steps_match_oracle_at_p256(xg, cfg):
    """the step compiler's schedule of the -c sweep (P256 A64) = the oracle's earliest-step
    schedule of the reference-pinned programs, message for message, barrier epochs included"""
    meta, _, _ = load_baseline(cfg)
    rl = meta["aggregators"]
    for m in meta["method_list"]:
        s = xg.Schedule(m, meta["P"], meta["A"], meta["d"], meta["c"], rl, ntimes=meta["ntimes"])
        progs = O.programs(m, meta["P"], meta["A"], meta["d"], meta["c"], rl, meta["ntimes"])
        om = O.match(progs)
        info = {}
        ost, ons = O.asap_steps(progs, om, info=info)
        assert s.barrier_epochs()[1:] == info["barrier_epochs"][1:], (cfg, m)
        mine = sorted((a, b, c, d, n, st) for a, b, c, d, n, st, fl in s.messages() if not fl & 1)
        ref = sorted((a, b, c, d, n, st) for (a, b, c, d, n, _sp, _rp), st in zip(om, ost))
        assert mine == ref, (cfg, m)
        assert s.nsteps >= ons


def _counts_as_d(trace, d):
    """a trace with every message count equal to the segment size written as 'D'"""
    import re
    return re.sub(r":%d(?=[@# ]|$)" % d, ":D", trace)


@pytest.mark.parametrize("cfg,d_full", [("cfg3_p256_a32_d64k", 4 << 20)] +
                         [("cfg4_p256_a64_d4k_c%d" % c, 64 << 20) for c in range(1, 9)])
def test_stated_size_schedules_are_the_captured_ones(xg, cfg, d_full):
    """configs[3] (-d 4 MiB) and configs[4] (-d 64 MiB) were captured at a reduced -d (host RAM).
    The MPI program of every rank at the stated size is the captured one with every segment
    count scaled: the product's schedule at the stated -d, counts written as 'D', equals its
    schedule at the captured -d (whose every rank equals the reference's by digest, above)."""
    meta, _, _ = load_baseline(cfg)
    rl, d = meta["aggregators"], meta["d"]
    for m in meta["method_list"]:
        small = xg.Schedule(m, meta["P"], meta["A"], d, meta["c"], rl, ntimes=meta["ntimes"])
        full = xg.Schedule(m, meta["P"], meta["A"], d_full, meta["c"], rl, ntimes=meta["ntimes"])
        for r in range(meta["P"]):
            ts = small.trace(r)
            assert _sha1(ts) == meta["trace_sha1"][str(m)][r], (cfg, m, r)
            assert _counts_as_d(full.trace(r), d_full) == _counts_as_d(ts, d), (cfg, m, r)
