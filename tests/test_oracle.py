"""The oracle (oracle/xg_oracle.py) pinned against the REAL reference.

tests/golden/ was produced by running the reference binary (built from
/root/reference by oracle/Makefile) under MPICH with the PMPI capture shim
(oracle/pmpi_capture.c); see tests/golden/make_golden.py.
"""
import pytest

import xg_oracle as O
from conftest import golden_configs, load_golden

CONFIGS = golden_configs()


def test_readme_aggregator_list():
    # the reference's own known answer: README.md:42
    assert O.aggregator_list(32, 14) == [0, 3, 6, 8, 10, 12, 14, 16, 18, 20, 22, 24, 26, 28]


@pytest.mark.parametrize("cfg", CONFIGS)
def test_placement(cfg):
    meta, _, _ = load_golden(cfg)
    assert O.aggregator_list(meta["P"], meta["A"], meta["proc_node"], meta["type"]) == meta["aggregators"]


@pytest.mark.parametrize("cfg", CONFIGS)
def test_traces_match_reference(cfg):
    meta, traces, _ = load_golden(cfg)
    P = meta["P"]
    rl = meta["aggregators"]
    for m in meta["method_list"]:
        progs = O.programs(m, P, meta["A"], meta["d"], meta["c"], rl, meta["ntimes"], meta["proc_node"],
                           meta["barrier"])
        for r in range(P):
            assert O.trace_tokens(progs[r]) == traces[(m, r)], (cfg, m, r)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_bytes_match_reference(cfg):
    meta, _, data = load_golden(cfg)
    P, A, d = meta["P"], meta["A"], meta["d"]
    rl = meta["aggregators"]
    aggidx = {g: i for i, g in enumerate(rl)}
    for m in meta["method_list"]:
        if m in O.TAM_METHODS:
            continue
        direction = O.direction(m)
        progs = O.programs(m, P, A, d, meta["c"], rl, meta["ntimes"], meta["proc_node"], meta["barrier"])
        for it in range(meta["iters"]):
            recv = O.execute(m, P, A, d, rl, progs, it)
            exp = O.expected_recv(m, P, A, d, rl, it)
            for r, buf in exp.items():
                assert (recv[r] == buf).all(), (cfg, m, it, r)
            for (git, src, dst), (glen, gchk) in data[direction].items():
                if git != it:
                    continue
                slot = src if direction == "a2m" else aggidx[src]
                assert glen == d
                assert O.chk64(recv[dst][slot * d:(slot + 1) * d]) == gchk, (cfg, m, it, src, dst)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_tam_messages_match_reference(cfg):
    """m15/m16 (lustre_driver_test.c collective_write): every message each rank received, in
    completion order, with the checksum of its bytes -- the intermediate aggregation buffers
    included -- and the final receive buffers equal to the closed form."""
    meta, _, data = load_golden(cfg)
    P, A, d = meta["P"], meta["A"], meta["d"]
    rl = meta["aggregators"]
    for m in O.TAM_METHODS:
        if m not in meta["method_list"]:
            continue
        for it in range(meta["iters"]):
            progs = O.programs(m, P, A, d, meta["c"], rl, meta["ntimes"], meta["proc_node"], meta["barrier"], it=it)
            rec = {}
            recv = O.execute(m, P, A, d, rl, progs, it, record=rec)
            for r, buf in O.expected_recv(m, P, A, d, rl, it).items():
                assert (recv[r] == buf).all(), (cfg, m, it, r)
            for r in range(P):
                # one reference run holds ntimes repetitions; the oracle replays them all
                assert rec[r] == data["tam"].get((m, it, r), []), (cfg, m, it, r)


@pytest.mark.parametrize("cfg", CONFIGS)
def test_uncaptured_pairs_are_self_copies(cfg):
    """The only pairs PMPI could not see are the aggregator self-memcpys of m3/m4/m6
    (and, at -d 0, every pair: a 0-byte segment has nothing to checksum)."""
    meta, _, _ = load_golden(cfg)
    rl = meta["aggregators"]
    for m, info in meta["methods"].items():
        assert info["status"] == "ok" and info["layout_ok"]
        if meta["d"] == 0:
            continue
        for it, src, dst in info["uncaptured_pairs"]:
            assert int(m) in (3, 4, 6, 18, 20) and src == dst and dst in rl


def test_asap_schedules_exist_for_goldens():
    for cfg in CONFIGS:
        meta, _, _ = load_golden(cfg)
        for m in meta["method_list"]:
            progs = O.programs(m, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"], meta["ntimes"],
                               meta["proc_node"], meta["barrier"])
            steps, n = O.asap_steps(progs)
            assert all(s is not None and 0 <= s < n for s in steps)


def test_m6_deadlock_boundary_matches_mpich():
    """Measured on the reference binary: m6 at P32 A14 c3 completes at d <= 65424 (MPICH eager)
    and hangs at d >= 65425 (rendezvous).  The oracle predicts the same."""
    rl = O.aggregator_list(32, 14)
    O.asap_steps(O.programs(6, 32, 14, 65424, 3, rl, 1), eager_limit=65424)
    with pytest.raises(RuntimeError, match="deadlock"):
        O.asap_steps(O.programs(6, 32, 14, 65425, 3, rl, 1), eager_limit=65424)


def test_chk64_known_answers():
    import numpy as np
    assert O.chk64(np.zeros(0, np.uint8)) == 0
    # position matters, length matters
    a = O.map_data(3, 5, 1, 64)
    b = a.copy(); b[[0, 8]] = b[[8, 0]]
    assert O.chk64(a) != O.chk64(b)
    assert O.chk64(a[:63]) != O.chk64(np.concatenate([a[:63], [0]]).astype(np.uint8))


def test_map_data_is_mod256_ramp():
    v = O.map_data(200, 60, 1, 300)
    assert v[0] == (200 + 60 + 1) % 256 and all(int(v[i + 1]) == (int(v[i]) + 1) % 256 for i in range(299))
