"""GPU: the step engine's ordering, the LDS realignment copy, the device
displacement scan, engine segments inside multi-GPU plans, and check_buffer's
negative path.

Synthetic plans are built directly as xg_devplan structures (include/xg_sched.h)
and executed through the C-ABI (xg_plan_load / xg_plan_run); the expected bytes
come from executing the same steps in order with numpy.
"""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx(xg):
    c = xg.Context(rank=0, nranks=1, device=0)
    yield c
    c.close()


def _ctx_env(xg, **env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return xg.Context(rank=0, nranks=1, device=0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


class Synth:
    """regions (SEND random bytes, RECV poisoned) + a synthetic one-GPU plan"""

    def __init__(self, xg, ctx, send_bytes, recv_bytes, steps, seed=0):
        d = xg.device()
        self.xg, self.d = xg, d
        rb = (C.c_int64 * xg.NBUF)(send_bytes, recv_bytes, 0, 0, 0)
        self.r = C.c_void_p()
        assert d.xg_regions_alloc(ctx.handle, rb, C.byref(self.r)) == 0
        rng = np.random.default_rng(seed)
        self.send = rng.integers(0, 256, send_bytes, dtype=np.uint8)
        self.recv = np.full(recv_bytes, 0xA5, np.uint8)
        buf = self.send.tobytes()
        assert d.xg_regions_write(self.r, xg.BUF_SEND, 0, buf, len(buf)) == 0
        copies = [c for st in steps for c in st]
        self.copies = (xg.Copy * max(1, len(copies)))(
            *[xg.Copy(so, do, ln, sb, db) for (sb, so, db, do, ln) in copies])
        sp, b = [], 0
        for st in steps:
            sp.append(xg.StepPlan(b, len(st), 0, 0, 0, 0, 0, 0))
            b += len(st)
        self.sp = (xg.StepPlan * len(sp))(*sp)
        self.p2p = (xg.P2P * 1)()
        dp = xg.DevPlan()
        dp.gpu, dp.ngpus, dp.nsteps = 0, 1, len(steps)
        for i, v in enumerate((send_bytes, recv_bytes, 0, 0, 0)):
            dp.region_bytes[i] = v
        dp.ncopy, dp.np2p = len(copies), 0
        dp.copies = C.cast(self.copies, C.POINTER(xg.Copy))
        dp.p2p = C.cast(self.p2p, C.POINTER(xg.P2P))
        dp.steps = C.cast(self.sp, C.POINTER(xg.StepPlan))
        self.dp = dp
        self.p = C.c_void_p()
        assert d.xg_plan_load(ctx.handle, self.r, C.byref(dp), C.byref(self.p)) == 0
        self.steps = steps

    def expected(self, recv=None):
        """RECV after one run that starts from `recv` (default: the poisoned region)"""
        bufs = {0: self.send.copy(), 1: (self.recv if recv is None else recv).copy()}
        for st in self.steps:
            # one step = simultaneous copies (the generator keeps them independent)
            vals = [bufs[sb][so:so + ln].copy() for (sb, so, db, do, ln) in st]
            for (sb, so, db, do, ln), v in zip(st, vals):
                bufs[db][do:do + ln] = v
        return bufs[1]

    def run(self):
        n = max(1, len(self.steps))
        done, post, wall = (C.c_double * n)(), (C.c_double * n)(), C.c_double()
        assert self.d.xg_plan_run(self.p, done, post, C.byref(wall)) == 0
        out = C.create_string_buffer(len(self.recv))
        assert self.d.xg_regions_read(self.r, 1, 0, out, len(self.recv)) == 0
        return np.frombuffer(out.raw, np.uint8)

    def close(self):
        self.d.xg_plan_free(self.p)
        self.d.xg_regions_free(self.r)


def _hazard_steps(unit, n_units, shift):
    """A: prime the consumer CUs' L1 with the slot's old bytes; B: write the slot from
    SEND; C: copy the slot on, shifted by `shift` units (each unit read by another
    workgroup than the one that wrote it, on another XCD); D: rewrite the slot with
    OTHER bytes; E: copy it again."""
    L = unit * n_units
    S, R = 0, 1
    return [
        [(R, shift * unit, R, 4 * L, L - shift * unit)],       # A: C's reads, of the poisoned slot
        [(S, 0, R, 0, L)],                                     # B
        [(R, shift * unit, R, L, L - shift * unit)],           # C: read-after-write (B)
        [(S, L, R, 0, L)],                                     # D: rewrite with other bytes
        [(R, 0, R, 2 * L, L)],                                 # E: read-after-write (D)
    ]


@pytest.mark.parametrize("unit_kib,n_units", [(4, 64), (4, 256), (16, 128)])
def test_engine_orders_hazards(xg, ctx, unit_kib, n_units):
    """Steps that read what an earlier step wrote, or rewrite it with other bytes, run
    inside ONE engine launch with the release/acquire barrier (flag 2) and still give
    exactly the bytes of in-order execution -- 20 runs each, consumer L1 primed."""
    unit = unit_kib << 10
    steps = _hazard_steps(unit, n_units, 1)
    L = unit * n_units
    sy = Synth(xg, ctx, 2 * L, 5 * L, steps)
    try:
        assert xg.device().xg_plan_engine(sy.p) > 0
        ns, nh = C.c_int(), C.c_int()
        assert xg.device().xg_plan_engine_steps(sy.p, C.byref(ns), C.byref(nh)) == len(steps)
        assert nh.value == 2 and ns.value == 1
        want = None
        for i in range(20):
            want = sy.expected(want)           # each run starts from the previous run's RECV
            got = sy.run()
            assert (got == want).all(), "run %d: %d bytes differ" % (i, int((got != want).sum()))
    finally:
        sy.close()


def test_graph_replays_alternate_with_eager_runs(xg):
    """XG_GRAPH=1 on a plan of a grid-engine segment (flag-2 hazard steps, which the solo engine
    never takes) and one step too large for the engine: runs replayed from the captured graph
    alternate with runs under a kernel-timing session (launched eagerly).  A replay restarts the
    device ticket counter inside the graph, so every replay leaves the host's ticket base stale;
    the next eager launch must zero the engine state again -- otherwise its grid
    barrier waits for tickets that never come and the run fails.  Every run's bytes checked."""
    unit, n_units, big = 4 << 10, 64, 32 << 20
    L = unit * n_units
    steps = _hazard_steps(unit, n_units, 1) + [[(0, 0, 1, 5 * L, big)]]
    cx = _ctx_env(xg, XG_GRAPH=1, XG_ENGINE_SOLO=0)
    try:
        sy = Synth(xg, cx, big, 5 * L + big, steps)
        try:
            d = xg.device()
            assert d.xg_plan_engine(sy.p) > 0 and d.xg_plan_engine_rails(sy.p) == 0
            assert d.xg_plan_launches(sy.p) == 2
            want = None
            for i in range(8):
                want = sy.expected(want)
                timed = i % 2 == 1               # odd runs: eager, inside a kernel-timing session
                if timed:
                    cx.ktime_begin(per_launch=True)
                got = sy.run()
                if timed:
                    _ms, n, _b = cx.ktime_end()
                    assert n == 2
                assert (got == want).all(), "run %d (%s): %d bytes differ" % (
                    i, "eager" if timed else "graph", int((got != want).sum()))
        finally:
            sy.close()
    finally:
        cx.close()


def _random_steps(rng, send_bytes, recv_bytes, nsteps, align):
    steps = []
    for _ in range(nsteps):
        st, dst_used, src_ranges = [], [], []
        for _k in range(rng.integers(1, 6)):
            ln = int(rng.integers(1, 600)) * 16 + (0 if align == 16 else int(rng.integers(0, 16)))
            for _try in range(20):
                do = int(rng.integers(0, (recv_bytes - ln) // align)) * align + (0 if align == 16 else int(rng.integers(0, 16)))
                do = min(do, recv_bytes - ln)
                if all(do + ln <= a or do >= b for a, b in dst_used + src_ranges):
                    break
            else:
                continue
            if rng.random() < 0.4:     # RECV -> RECV: must not meet this step's destinations
                for _try in range(20):
                    so = min(int(rng.integers(0, recv_bytes - ln)), recv_bytes - ln)
                    if all(so + ln <= a or so >= b for a, b in dst_used + [(do, do + ln)]):
                        st.append((1, so, 1, do, ln))
                        src_ranges.append((so, so + ln))
                        dst_used.append((do, do + ln))
                        break
            else:
                so = min(int(rng.integers(0, send_bytes - ln)), send_bytes - ln)
                st.append((0, so, 1, do, ln))
                dst_used.append((do, do + ln))
        steps.append(st)
    return steps


@pytest.mark.parametrize("align", [16, 1])
@pytest.mark.parametrize("seed", range(6))
def test_random_plans_engine_and_launches(xg, ctx, seed, align):
    """Random step lists (SEND->RECV and RECV->RECV copies, reads of earlier steps'
    output, rewrites; 16-B aligned or any phase) give the in-order bytes both in the
    step engine and as one copy launch per step (the LDS realignment path for the
    misaligned pieces)."""
    rng = np.random.default_rng(seed)
    send_bytes, recv_bytes = 1 << 20, 1 << 20
    steps = _random_steps(rng, send_bytes, recv_bytes, 12, align)
    eager = _ctx_env(xg, XG_ENGINE_MAX_STEP=0)
    try:
        for cx, engine in ((ctx, True), (eager, False)):
            sy = Synth(xg, cx, send_bytes, recv_bytes, steps, seed=seed)
            try:
                assert (xg.device().xg_plan_engine(sy.p) > 0) == engine
                want = None
                for _ in range(3):
                    want = sy.expected(want)
                    got = sy.run()
                    assert (got == want).all(), (engine, int((got != want).sum()))
            finally:
                sy.close()
    finally:
        eager.close()


@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 6])
def test_copy_variants_every_phase(xg, variant):
    """Every copy-kernel variant moves pieces at every (source, destination) phase mod
    16 and lengths around the 4 KiB tile, byte-exact (misaligned ones through LDS)."""
    cx = _ctx_env(xg, XG_ENGINE_MAX_STEP=0, XG_COPY_VARIANT=variant)
    try:
        steps, do = [], 0
        st = []
        for sp in range(16):
            for dp_ in range(16):
                i = sp * 16 + dp_
                ln = 4096 + (37 * i) % 9000 - (i % 7)
                st.append((0, 9600 * i + sp, 1, do + dp_, ln))
                do += ((ln + dp_ + 64) // 16 + 1) * 16
        steps.append(st)
        sy = Synth(xg, cx, 9600 * 256 + 13200, do + 64, steps, seed=variant)
        try:
            want = sy.expected()
            got = sy.run()
            assert (got == want).all(), int((got != want).sum())
        finally:
            sy.close()
    finally:
        cx.close()


@pytest.mark.parametrize("d", [4096, 1000])
def test_verify_reports_a_corrupted_byte(xg, ctx, d):
    """check_buffer's negative path (mpi_test.c:83-92): one overwritten byte of a
    receive slot is reported as exactly one bad byte at its offset, in that slot only."""
    P, A = 12, 5
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(1, P, A, d, 3, rl, ntimes=1)
    run = xg.MethodRun(ctx, s, it=1, mode=0)
    try:
        run.run_timed()
        _c, bad, first = run.verify()
        assert all(b == 0 for b in bad) and all(f == -1 for f in first)
        for victim, at in ((0, 0), (7, d - 1), (len(run.slots) - 1, d // 2 + 3)):
            off = run.slots[victim][3] + at
            (orig,) = run.read(xg.BUF_RECV, off, 1)
            run.write(xg.BUF_RECV, off, bytes([orig ^ 0x5A]))
            _c, bad, first = run.verify()
            assert bad[victim] == 1 and first[victim] == at, (victim, bad[victim], first[victim])
            assert sum(bad) == 1
            run.write(xg.BUF_RECV, off, bytes([orig]))
        _c, bad, _f = run.verify()
        assert all(b == 0 for b in bad)
    finally:
        run.close()


@pytest.mark.parametrize("method,d", [(5, 2048), (8, 2048), (5, 1000), (8, 24), (1, 1000), (2, 4096)])
def test_device_displacements_match_host_layout(xg, method, d):
    """The staging displacements of the packed segments are computed at plan load by
    the wavefront prefix scan (displ_scan_kernel); they equal the host layout's
    exclusive prefix sums (xg_devplan_build), and the packed plans stay bit-exact."""
    import xg_oracle as O
    P, A, c, k, G = 16, 4, 200000000, 2, 4      # default -c: one step, several segments per peer
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k)
    ctxs = [xg.Context.virtual(g, G) for g in range(G)]
    runs, total = [], 0
    try:
        for g in range(G):
            r = xg.MethodRun(ctxs[g], s, it=1, mode=1, pack_max_seg=1 << 20)
            runs.append(r)
            v = r.view
            host = []
            for (pb, pc, _q, _n, qb, qc) in v.steps:
                host += [do for (sb, so, db, do, ln) in v.copies[pb:pb + pc] if db == xg.BUF_STAGE_SEND and ln > 0]
                host += [so for (sb, so, db, do, ln) in v.copies[qb:qb + qc] if sb == xg.BUF_STAGE_RECV and ln > 0]
            assert r.displs() == host, g
            total += len(host)
        assert total > 0
        xg.run_virtual(runs)
        exp = O.expected_recv(method, P, A, d, rl, 1, mode=1)
        for g, r in enumerate(runs):
            chk, bad, _f = r.verify()
            assert all(b == 0 for b in bad), g
            for (src, seed, dst, off), ck in zip(r.slots, chk):
                local = off - s.recv_offset(G, dst)
                assert ck == O.chk64(exp[dst][local: local + d]), (g, src, dst)
    finally:
        for r in runs:
            r.close()
        for cx in ctxs:
            cx.close()


@pytest.mark.parametrize("method", [6, 9, 12, 18])
def test_engine_segments_in_multi_gpu_plans(xg, method):
    """Multi-GPU plans: every run of >= 2 steps in which a GPU only copies locally is ONE
    engine launch; the virtual 8-GPU job (RCCL self send/recv for the cross-GPU pairs)
    is bit-exact and needs fewer launches than one per step part."""
    import xg_oracle as O
    P, A, d, c, k, G = 32, 14, 2048, 3, 2, 8
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k)
    os.environ["XG_ENGINE_MAX_STEP"] = "0"
    try:
        ectxs = [xg.Context.virtual(g, G) for g in range(G)]
    finally:
        del os.environ["XG_ENGINE_MAX_STEP"]
    ctxs = [xg.Context.virtual(g, G) for g in range(G)]
    runs = []
    try:
        eager = sum(xg.MethodRun(ectxs[g], s, it=0, mode=1).launches for g in range(G))
        runs = [xg.MethodRun(ctxs[g], s, it=0, mode=1) for g in range(G)]
        xg.run_virtual(runs, rccl=True)
        exp = O.expected_recv(method, P, A, d, rl, 0, mode=1)
        for g, r in enumerate(runs):
            chk, bad, _f = r.verify()
            assert all(b == 0 for b in bad), g
            for (src, seed, dst, off), ck in zip(r.slots, chk):
                local = off - s.recv_offset(G, dst)
                assert ck == O.chk64(exp[dst][local: local + d]), (g, src, dst)
        seg_steps = sum(r.engine_steps()[0] for r in runs)
        launches = sum(r.launches for r in runs)
        assert launches <= eager
        if seg_steps:
            assert launches < eager, (launches, eager, seg_steps)
    finally:
        for r in runs:
            r.close()
        for cx in ctxs + ectxs:
            cx.close()


@pytest.mark.parametrize("method,d", [(11, 1 << 20), (12, 1 << 20), (9, 4 << 20), (15, 2048), (16, 2048),
                                      (16, 1000), (15, 1 << 20)])
def test_step_chains_time_like_events(xg, method, d):
    """Runs of one-launch local steps (large steps, outside the engine; TAM steps: a stage
    launch and/or a local launch) are timed by in-kernel start stamps of each step's
    first launch instead of a step mark after every step (XG_STEP_CHAIN; the marks were HIP
    events until round 4, clock stamps since -- the test keeps its name): same delivered
    bytes as the run marked step by step, step times ordered and inside the run's wall time,
    and no later than that run's by more than noise."""
    import xg_oracle as O
    P, A, c = 32, 14, 3
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=2)
    exp = O.expected_recv(method, P, A, d, rl, 0, mode=1)
    res = {}
    for name, env in (("chain", {}), ("events", {"XG_STEP_CHAIN": "0"})):
        cx = _ctx_env(xg, XG_ENGINE_MAX_STEP=0, **env)
        try:
            run = xg.MethodRun(cx, s, it=0, mode=1)
            try:
                best = None
                for _rep in range(3):
                    done, _post, wall = run.run_timed()
                    assert all(0 <= a <= b for a, b in zip(done, done[1:])), (name, done)
                    assert done[-1] <= wall + 1e-4
                    best = done[-1] if best is None else min(best, done[-1])
                chk, bad, _f = run.verify()
                assert all(b == 0 for b in bad), name
                for (src, seed, dst, off), ck in zip(run.slots, chk):
                    local = off - s.recv_offset(1, dst)
                    assert ck == O.chk64(exp[dst][local: local + d]), (name, src, dst)
                res[name] = (chk, best)
            finally:
                run.close()
        finally:
            cx.close()
    assert res["chain"][0] == res["events"][0]
    print("method %d d %d: chained %.1f us, evented %.1f us" % (method, d, res["chain"][1] * 1e6,
                                                                res["events"][1] * 1e6))
    assert res["chain"][1] <= res["events"][1] * 1.10 + 20e-6
