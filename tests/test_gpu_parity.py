"""GPU parity: the HIP path (libxg.so) vs the oracle and the reference's captured bytes.

Every received segment is checked twice on the device (xg_verify): against the
closed-form fingerprint (byte-exact mismatch count) and by its xg_chk64, which
must equal the checksum the PMPI capture recorded from the REAL reference for
the same (method, iter, src, dst).  Bit-exact is the bar (integer/byte work).
"""
import pytest

from conftest import golden_configs, load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(xg):
    c = xg.Context(rank=0, nranks=1, device=0)
    yield c
    c.close()


def _run(xg, ctx, meta, method, it, mode=0, pack=1 << 20):
    P, A, d, c, k = meta["P"], meta["A"], meta["d"], meta["c"], meta["ntimes"]
    rl = xg.aggregator_list(P, A, meta["proc_node"], meta["type"])
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=meta["proc_node"],
                    barrier_type=meta.get("barrier", 0))
    run = xg.MethodRun(ctx, s, it=it, mode=mode, pack_max_seg=pack)
    done, post, wall = run.run_timed()
    chk, bad, first = run.verify()
    return s, run, (done, post, wall), chk, bad, first


@pytest.mark.parametrize("cfg", golden_configs())
def test_golden_all_methods(xg, ctx, cfg):
    meta, _traces, data = load_golden(cfg)
    import xg_oracle as O
    for method in meta["method_list"]:
        direction = O.direction(method)
        for it in range(meta["iters"]):
            s, run, _t, chk, bad, first = _run(xg, ctx, meta, method, it)
            try:
                assert len(run.slots) == sum(1 for k in data[direction] if k[0] == it)
                for (src, seed, dst, off), ck, nb, fb in zip(run.slots, chk, bad, first):
                    assert nb == 0, "%s m%d it%d %d->%d: %d bad bytes from %d" % (cfg, method, it, src, dst, nb, fb)
                    glen, gchk = data[direction][(it, src, dst)]
                    assert glen == meta["d"] and ck == gchk, (cfg, method, it, src, dst, hex(ck), hex(gchk))
            finally:
                run.close()


@pytest.mark.parametrize("method", list(range(1, 21)))
def test_strong_fingerprint(xg, ctx, method):
    """Collision-free fingerprint: catches misroutes MAP_DATA cannot (equal rank+seed)."""
    import xg_oracle as O
    meta = {"P": 20, "A": 6, "d": 1000, "c": 7, "ntimes": 2, "proc_node": 3, "type": 1, "barrier": 2}
    s, run, _t, chk, bad, _f = _run(xg, ctx, meta, method, it=3, mode=1)
    try:
        exp = O.expected_recv(method, 20, 6, 1000, s.rank_list, 3, mode=1)
        for (src, seed, dst, off), ck, nb in zip(run.slots, chk, bad):
            assert nb == 0
            local = off - s.recv_offset(1, dst)
            assert ck == O.chk64(exp[dst][local: local + 1000])
    finally:
        run.close()


def test_readback_matches_oracle_bytes(xg, ctx):
    """Read the receive region back and compare with the oracle's executed MPI program."""
    import numpy as np
    import xg_oracle as O
    P, A, d, c, k = 16, 5, 1000, 3, 2
    rl = xg.aggregator_list(P, A)
    for method in (3, 4, 6, 11):
        s = xg.Schedule(method, P, A, d, c, rl, ntimes=k)
        run = xg.MethodRun(ctx, s, it=1, mode=0)
        run.run_timed()
        progs = O.programs(method, P, A, d, c, rl, k)
        ref = O.execute(method, P, A, d, rl, progs, 1)
        try:
            for r, buf in ref.items():
                if buf.size == 0:
                    continue
                got = np.frombuffer(run.read(1, s.recv_offset(1, r), buf.size), dtype=np.uint8)
                assert (got == buf).all(), (method, r)
        finally:
            run.close()


@pytest.mark.parametrize("method", [15, 16])
def test_tam_aggregation_buffers_match_oracle(xg, ctx, method):
    """TAM (collective_write): besides the receive slots, the intermediate aggregation
    buffers of every rank (aggregate_buf | send_buf2 | recv_buf in SCRATCH) hold exactly
    what the oracle's MPI execution leaves in them -- the same bytes the PMPI capture of
    the reference checksums message by message (tests/test_oracle.py)."""
    import numpy as np
    import xg_oracle as O
    P, A, d, c, k, pn, it = 18, 5, 1000, 3, 2, 5, 1
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=pn, iteration=it)
    run = xg.MethodRun(ctx, s, it=it, mode=1)
    try:
        run.run_timed()
        _chk, bad, _f = run.verify()
        assert all(b == 0 for b in bad)
        bufs = {}
        O.execute(method, P, A, d, rl, O.programs(method, P, A, d, c, rl, k, pn, it=it), it, mode=1, buffers=bufs)
        for r in range(P):
            base = s.scratch_offset(1, r)
            off = 0
            for name in ("AGG", "SBUF2", "RBUF"):
                ref = bufs[r].get(name, np.zeros(0, np.uint8))
                if ref.size:
                    got = np.frombuffer(run.read(xg.BUF_SCRATCH, base + off, ref.size), dtype=np.uint8)
                    assert (got == ref).all(), (method, r, name)
                off += (ref.size + 255) // 256 * 256
    finally:
        run.close()


@pytest.mark.parametrize("d", [2048, 1000])
@pytest.mark.parametrize("method", [15, 16])
def test_tam_stage_copies_share_a_launch(xg, method, d):
    """XG_FUSE_STAGE: a TAM step whose stage copies nothing else of the step touches
    (xg_step_stage_meets_rest) runs them in the same launch as its local copies -- one launch
    fewer per run at the README configuration -- and every receive slot and aggregation buffer
    is the same as with the stage copies in a launch of their own."""
    import os
    import xg_oracle as O
    P, A, c, k, it = 32, 14, 3, 2, 1
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, iteration=it)
    exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
    runs = {}
    ctxs = []
    try:
        for fuse in ("1", "0"):
            old = os.environ.get("XG_FUSE_STAGE")
            os.environ["XG_FUSE_STAGE"] = fuse
            try:
                cx = xg.Context(rank=0, nranks=1, device=0)
            finally:
                if old is None:
                    del os.environ["XG_FUSE_STAGE"]
                else:
                    os.environ["XG_FUSE_STAGE"] = old
            ctxs.append(cx)
            run = xg.MethodRun(cx, s, it=it, mode=1)
            runs[fuse] = run
            for _ in range(2):
                done, _post, wall = run.run_timed()
                assert all(0 <= a <= b for a, b in zip(done, done[1:])) and done[-1] <= wall + 1e-4
            chk, bad, _first = run.verify()
            assert not any(bad), (method, d, fuse)
            for (src, seed, dst, off), ck in zip(run.slots, chk):
                local = off - s.recv_offset(1, dst)
                assert ck == O.chk64(exp[dst][local: local + d]), (method, d, fuse, src, dst)
        assert runs["1"].launches < runs["0"].launches, (runs["1"].launches, runs["0"].launches)
        scr = s.region_bytes(1, 0, xg.BUF_SCRATCH)
        assert runs["1"].read(xg.BUF_SCRATCH, 0, scr) == runs["0"].read(xg.BUF_SCRATCH, 0, scr)
    finally:
        for r in runs.values():
            r.close()
        for cx in ctxs:
            cx.close()


@pytest.mark.parametrize("d", [1000, 2048])
@pytest.mark.parametrize("method", [1, 6, 9, 10, 11, 12, 13, 18])
def test_step_engine_matches_per_step_launches(xg, ctx, method, d):
    """GPU-local plans of small steps run as ONE persistent launch (step engine: grid
    barrier + wall-clock stamp per step; d = 1000: byte path, d = 2048: 16-B buffer
    loads/stores with partial units).  Same bytes as one launch per step, every slot
    checked against the oracle with the strong fingerprint; step times ordered and
    inside the run's wall time."""
    import os
    import xg_oracle as O
    P, A, c, k, it = 20, 6, 3, 2, 1
    rl = xg.aggregator_list(P, A)
    os.environ["XG_ENGINE_MAX_STEP"] = "0"
    try:
        ctx_eager = xg.Context(rank=0, nranks=1, device=0)
    finally:
        del os.environ["XG_ENGINE_MAX_STEP"]
    try:
        s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=3, barrier_type=1, iteration=it)
        exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
        res = {}
        for name, cx in (("engine", ctx), ("eager", ctx_eager)):
            run = xg.MethodRun(cx, s, it=it, mode=1)
            try:
                if name == "eager" or run.nsteps >= 2:     # one-step plans: armed solo when small enough
                    assert (run.engine_workgroups > 0) == (name != "eager"), (name, run.nsteps)
                done, post, wall = run.run_timed()
                assert all(0 <= a <= b for a, b in zip(done, done[1:])), done
                assert done[-1] <= wall + 1e-4
                chk, bad, _f = run.verify()
                assert all(b == 0 for b in bad), name
                for (src, seed, dst, off), ck in zip(run.slots, chk):
                    local = off - s.recv_offset(1, dst)
                    assert ck == O.chk64(exp[dst][local: local + d]), (name, method, src, dst)
                res[name] = chk
            finally:
                run.close()
        assert res["engine"] == res["eager"]
    finally:
        ctx_eager.close()


ENGINE_MODES = {
    "solo_armed": {"XG_ENGINE_ARM": "1"},                       # 512 one-wave rails, doorbell-armed
    "solo64_armed": {"XG_SOLO_RAILS": "64", "XG_ENGINE_ARM": "1"},
    "solo37_launch": {"XG_SOLO_RAILS": "37", "XG_ENGINE_ARM": "0"},
    "solo16_armed": {"XG_SOLO_RAILS": "16", "XG_ENGINE_ARM": "1"},
    "wg_armed": {"XG_SOLO_WAVES": "16", "XG_ENGINE_ARM": "1"},  # 16 workgroup rails of 16 waves
    "wg1_launch": {"XG_SOLO_WAVES": "16", "XG_SOLO_RAILS": "1", "XG_ENGINE_ARM": "0"},
    "grid_armed": {"XG_ENGINE_SOLO": "0", "XG_ENGINE_ARM": "1"},
    "solo_launch": {},                                          # the default: launched inside the timed region
    "grid_drain": {"XG_ENGINE_SOLO": "0", "XG_ENGINE_DRAIN": "1", "XG_ENGINE_ARM": "0"},
}


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("method", [6, 9, 12, 18])
def test_step_engine_modes(xg, method, k):
    """The README-sized chains under every engine form: solo rails (one-wave or 16-wave)
    or a grid barrier per step, armed by the doorbell or launched inside the timed region, and
    the grid engine draining at every step (XG_ENGINE_DRAIN=1).  Same bytes (strong
    fingerprint, every slot against the oracle), step times ordered and within the
    run's wall time, repeated runs stay correct."""
    import os
    import xg_oracle as O
    P, A, d, c, it = 32, 14, 2048, 3, 0
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, iteration=it)
    exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
    res = {}
    for name, env in ENGINE_MODES.items():
        old = {key: os.environ.get(key) for key in env}
        os.environ.update(env)
        try:
            cx = xg.Context(rank=0, nranks=1, device=0)
        finally:
            for key, v in old.items():
                if v is None:
                    del os.environ[key]
                else:
                    os.environ[key] = v
        try:
            run = xg.MethodRun(cx, s, it=it, mode=1)
            try:
                assert run.engine_workgroups > 0
                rails = {"solo_armed": 512, "solo64_armed": 64, "solo37_launch": 37, "solo16_armed": 16, "wg_armed": 16,
                         "wg1_launch": 1, "solo_launch": 512}.get(name, 0)
                assert run.engine_rails == rails, (name, run.engine_rails)
                for _rep in range(3):
                    done, _post, wall = run.run_timed()
                    assert all(0 <= a <= b for a, b in zip(done, done[1:])), (name, done)
                    assert done[-1] <= wall + 1e-4
                chk, bad, _f = run.verify()
                assert all(b == 0 for b in bad), name
                for (src, seed, dst, off), ck in zip(run.slots, chk):
                    local = off - s.recv_offset(1, dst)
                    assert ck == O.chk64(exp[dst][local: local + d]), (name, method, src, dst)
                res[name] = chk
            finally:
                run.close()
        finally:
            cx.close()
    assert all(v == res["solo_armed"] for v in res.values())


@pytest.mark.parametrize("k", [1, 3])
@pytest.mark.parametrize("d", [1000, 100, 24, 33, 1])
@pytest.mark.parametrize("method", [6, 9, 12, 18, 1, 4])
def test_solo_engine_fine_granules(xg, method, d, k):
    """Segment sizes that are not multiples of 16 run on the solo engine's 4-B (d = 1000,
    100, 24) or 1-B (d = 33, 1) granules: armed one-wave rails, the same bytes as one
    launch per step, every slot against the oracle with the strong fingerprint."""
    import os
    import xg_oracle as O
    P, A, c, it = 32, 14, 3, 1
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, iteration=it)
    exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
    res = {}
    for name, env in (("solo", {}), ("eager", {"XG_ENGINE_MAX_STEP": "0"})):
        os.environ.update(env)
        try:
            cx = xg.Context(rank=0, nranks=1, device=0)
        finally:
            for key in env:
                del os.environ[key]
        try:
            run = xg.MethodRun(cx, s, it=it, mode=1)
            try:
                if name == "solo" and run.nsteps >= 2:
                    assert run.engine_rails > 0, (method, d, k, run.nsteps)
                for _rep in range(3):
                    done, _post, wall = run.run_timed()
                    assert all(0 <= a <= b for a, b in zip(done, done[1:])), (name, done)
                    assert done[-1] <= wall + 1e-4
                chk, bad, _f = run.verify()
                assert all(b == 0 for b in bad), (name, method, d)
                for (src, seed, dst, off), ck in zip(run.slots, chk):
                    local = off - s.recv_offset(1, dst)
                    assert ck == O.chk64(exp[dst][local: local + d]), (name, method, d, src, dst)
                res[name] = chk
            finally:
                run.close()
        finally:
            cx.close()
    assert res["solo"] == res["eager"]


@pytest.mark.parametrize("method,k,env", [(6, 60, {}), (9, 70, {}), (12, 2, {"XG_ENGINE_SOLO_MAX": "262144"}),
                                          (18, 3, {"XG_ENGINE_SOLO_MAX": "1048576"}), (1, 200, {})])
def test_long_runs_split_into_solo_launches(xg, method, k, env):
    """A hazard-free run too long for one solo launch (more than 2048 steps at a large -k,
    or more bytes than XG_ENGINE_SOLO_MAX) becomes consecutive solo launches instead of
    one grid launch with a barrier per step: same bytes as per-step launches, step times
    ordered, every slot against the oracle."""
    import os
    import xg_oracle as O
    P, A, d, c, it = 32, 14, 2048, 3, 0
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, iteration=it)
    exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
    res = {}
    for name, extra in (("split", env), ("grid", {"XG_ENGINE_SOLO": "0"}), ("eager", {"XG_ENGINE_MAX_STEP": "0"})):
        os.environ.update(extra)
        try:
            cx = xg.Context(rank=0, nranks=1, device=0)
        finally:
            for key in extra:
                del os.environ[key]
        try:
            run = xg.MethodRun(cx, s, it=it, mode=1)
            try:
                if name == "split":
                    n_eng, nseg, nhaz = run.engine_steps()
                    assert nseg >= 2 and nhaz == 0 and run.engine_rails > 0, (n_eng, nseg, nhaz, run.nsteps)
                for _rep in range(2):
                    done, _post, wall = run.run_timed()
                    assert all(0 <= a <= b for a, b in zip(done, done[1:])), name
                    assert done[-1] <= wall + 1e-4
                chk, bad, _f = run.verify()
                assert all(b == 0 for b in bad), name
                for (src, seed, dst, off), ck in zip(run.slots, chk):
                    local = off - s.recv_offset(1, dst)
                    assert ck == O.chk64(exp[dst][local: local + d]), (name, method, src, dst)
                res[name] = (chk, done[-1])
            finally:
                run.close()
        finally:
            cx.close()
    assert res["split"][0] == res["eager"][0] == res["grid"][0]
    print("method %d -k %d: split solo %.1f us, grid engine %.1f us, per-step launches %.1f us"
          % (method, k, res["split"][1] * 1e6, res["grid"][1] * 1e6, res["eager"][1] * 1e6))


GRAPH_FORMS = {
    "chains": {"XG_GRAPH": "1", "XG_ENGINE_MAX_STEP": "0"},                  # chained step launches, stamps
    "grid_and_launches": {"XG_GRAPH": "1", "XG_ENGINE_SOLO": "0", "XG_ENGINE_MAX_STEP": str(64 << 10)},
    "solo_and_launches": {"XG_GRAPH": "1", "XG_ENGINE_MAX_STEP": str(64 << 10)},
}


@pytest.mark.parametrize("form", list(GRAPH_FORMS))
@pytest.mark.parametrize("method", [1, 4, 6, 9, 12, 13, 15])
def test_graph_replay_one_gpu(xg, form, method):
    """XG_GRAPH=1: a multi-launch plan is captured once (copy launches, chain stamps, engine
    segments -- the grid engine's ticket counter reset inside the graph) and every later run
    replays it.  Three runs, the receive slots re-poisoned between them: every replay delivers
    every byte (strong fingerprint, against the oracle), step times ordered inside the wall
    time."""
    import os
    import xg_oracle as O
    P, A, d, c, k, it = 24, 7, 48 << 10, 3, 2, 1
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=4, barrier_type=1, iteration=it)
    exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
    env = GRAPH_FORMS[form]
    old = {key: os.environ.get(key) for key in env}
    os.environ.update(env)
    try:
        cx = xg.Context(rank=0, nranks=1, device=0)
    finally:
        for key, v in old.items():
            if v is None:
                del os.environ[key]
            else:
                os.environ[key] = v
    try:
        run = xg.MethodRun(cx, s, it=it, mode=1)
        try:
            for rep in range(3):
                if rep:
                    run.poison()
                done, post, wall = run.run_timed()
                assert all(0 <= a <= b for a, b in zip(done, done[1:])), (form, done)
                assert done[-1] <= wall + 1e-4
                chk, bad, _f = run.verify()
                assert all(b == 0 for b in bad), (form, method, rep)
                for (src, seed, dst, off), ck in zip(run.slots, chk):
                    local = off - s.recv_offset(1, dst)
                    assert ck == O.chk64(exp[dst][local: local + d]), (form, method, rep, src, dst)
            run.poison()
            run.enqueue()                     # the enqueue graph (bench loops) delivers too
            cx.sync()
            run.check()
            assert all(b == 0 for b in run.verify()[1]), (form, method)
        finally:
            run.close()
    finally:
        cx.close()
