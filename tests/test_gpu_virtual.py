"""Multi-GPU device plans on one MI355X: every GPU of a G-GPU job is emulated on
the one device (xg_init_virtual), each with its own regions, fill, plan and
copy-kernel launches; the RCCL send/recv pairs of each step are moved as device
copies in RCCL's per-peer order (xg_vplans_run).  This runs the exact per-GPU
plans the driver's 2/4/8-GPU bench executes (local gather/scatter, packing
into per-peer staging, unpacking) on the hardware, and checks every received
segment against the checksums captured from the real reference.

RCCL refuses two ranks on one device, so the box cannot run a 2-rank
communicator; test_golden_multi_gpu_rccl instead moves the same pairs through
RCCL on a 1-rank communicator (self ncclSend/ncclRecv in one group per step,
ncclAllReduce for the in-loop barriers): RCCL's p2p calls with the plans' real
buffers, offsets and lengths.  tests/test_plan_gloo.py runs the same plans
across two processes on CPU.
"""
import pytest

from conftest import golden_configs, load_golden

pytestmark = pytest.mark.gpu

GPUS = (2, 3, 8)
# (pack_max_seg, pack form): never pack / pack every multi-segment peer list one-sided (runs,
# staged on one side) / two-sided (one staging buffer per peer and direction)
PACKINGS = ((0, -1), (1 << 30, 1), (1 << 30, 0))


@pytest.fixture(scope="module")
def worlds(xg):
    w = {G: [xg.Context.virtual(g, G, device=0) for g in range(G)] for G in GPUS}
    yield w
    for ctxs in w.values():
        for c in ctxs:
            c.close()


def _run_job(xg, ctxs, s, it, mode, pack, rccl=False, reps=1, form=-1):
    runs = [xg.MethodRun(c, s, it=it, mode=mode, pack_max_seg=pack, pack_form=form) for c in ctxs]
    try:
        for rep in range(reps):           # reps > 1: a replay (graph mode) must deliver again
            if rep:
                for r in runs:
                    r.poison()
            done = xg.run_virtual(runs, rccl=rccl)
            assert all(b >= a for a, b in zip(done, done[1:]))
        out = []
        for r in runs:
            chk, bad, first = r.verify()
            out += list(zip(r.slots, chk, bad, first))
        return out
    finally:
        for r in runs:
            r.close()


@pytest.mark.parametrize("G", GPUS)
@pytest.mark.parametrize("cfg", golden_configs())
def test_golden_multi_gpu(xg, worlds, cfg, G):
    _golden_job(xg, worlds, cfg, G, rccl=False)


@pytest.mark.parametrize("G", (2, 8))
@pytest.mark.parametrize("cfg", golden_configs())
def test_golden_multi_gpu_rccl(xg, worlds, cfg, G):
    _golden_job(xg, worlds, cfg, G, rccl=True)


def _golden_job(xg, worlds, cfg, G, rccl):
    meta, _traces, data = load_golden(cfg)
    import xg_oracle as O
    P, A, d, c, k = meta["P"], meta["A"], meta["d"], meta["c"], meta["ntimes"]
    if G > P:
        pytest.skip("more GPUs than ranks")
    rl = xg.aggregator_list(P, A, meta["proc_node"], meta["type"])
    it = meta["iters"] - 1
    for method in meta["method_list"]:
        direction = O.direction(method)
        s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=meta["proc_node"],
                        barrier_type=meta.get("barrier", 0), iteration=it)
        for pack, form in PACKINGS:
            res = _run_job(xg, worlds[G], s, it, 0, pack, rccl, form=form)
            assert len(res) == sum(1 for key in data[direction] if key[0] == it), (cfg, method, G)
            for (src, seed, dst, off), ck, nb, fb in res:
                assert nb == 0, "%s G%d m%d pack%d/%d %d->%d: %d bad bytes from %d" % (
                    cfg, G, method, pack, form, src, dst, nb, fb)
                glen, gchk = data[direction][(it, src, dst)]
                assert ck == gchk, (cfg, G, method, pack, form, src, dst, hex(ck), hex(gchk))


@pytest.mark.parametrize("G", GPUS)
@pytest.mark.parametrize("method", list(range(1, 21)))
def test_strong_fingerprint_multi_gpu(xg, worlds, G, method):
    """Collision-free fingerprint across GPU boundaries (unaligned d, packed staging, one- and
    two-sided)."""
    import xg_oracle as O
    P, A, d, c, k, it = 20, 6, 1000, 7, 2, 3
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=3, barrier_type=2, iteration=it)
    exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
    for form in (1, 0):
        res = _run_job(xg, worlds[G], s, it, 1, 1 << 20, form=form)
        assert res
        for (src, seed, dst, off), ck, nb, _fb in res:
            assert nb == 0, (method, G, form, src, dst)
            local = off - s.recv_offset(G, dst)
            assert ck == O.chk64(exp[dst][local: local + d]), (method, G, form, src, dst)


@pytest.mark.parametrize("G", (2, 8))
@pytest.mark.parametrize("method", [1, 2, 5, 8, 9, 10])
def test_config2_full_size_through_rccl(xg, worlds, G, method):
    """BASELINE configs[2] at full size (P64 A16 -d 256 KiB) as a G-GPU job on this device,
    every cross-GPU segment through RCCL (1-rank communicator), packed and direct: zero
    mismatching bytes against the closed-form strong fingerprint, sampled checksums equal
    the oracle's (size-independent check: the CPU oracle does not replay 256 MiB here)."""
    import xg_oracle as O
    P, A, d, it = 64, 16, 256 << 10, 2
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, 200000000, rl, ntimes=1, iteration=it)
    for pack, form in PACKINGS:
        res = _run_job(xg, worlds[G], s, it, 1, pack, rccl=True, form=form)
        assert len(res) == P * A
        assert all(nb == 0 for _slot, _ck, nb, _fb in res), (method, G, pack, form)
        for (src, seed, _dst, _off), ck, _nb, _fb in res[:: max(1, len(res) // 6)]:
            assert ck == O.chk64(O.fingerprint(1, src, seed, it, d)), (method, G, pack, form, src, seed)


STEP_FORMS = {
    "split": {"XG_SELF_MAX": "0", "XG_SPLIT_MIN": "0"},       # local part on the side stream, after the packs
    "split_with_packs": {"XG_SELF_MAX": "0", "XG_SPLIT_MIN": "0", "XG_SPLIT_AFTER_PACK": "0"},   # round 2: together
    "self_in_group": {"XG_SELF_MAX": str(1 << 30)},          # local part as self send/recv in the RCCL group
    "local_in_fused": {"XG_SELF_MAX": "0", "XG_SPLIT_MIN": str(1 << 40)},   # in the (fused) pack launch
    "graph": {"XG_GRAPH": "1", "XG_SELF_MAX": "0"},           # the whole job captured once, replayed
    "graph_self": {"XG_GRAPH": "1", "XG_SELF_MAX": str(1 << 30)},
}


@pytest.mark.parametrize("form", list(STEP_FORMS))
@pytest.mark.parametrize("rccl", [False, True])
@pytest.mark.parametrize("G", (2, 8))
def test_cross_gpu_step_forms(xg, form, rccl, G):
    """The two cheaper forms of a cross-GPU step (one launch fewer than the split local
    gather + its fork/join): every method, packed and direct, collision-free fingerprint,
    unaligned d, every slot against the oracle."""
    import os
    import xg_oracle as O
    env = STEP_FORMS[form]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ctxs = [xg.Context.virtual(g, G, device=0) for g in range(G)]
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        P, A, d, c, k, it = 20, 6, 1000, 7, 2, 3
        rl = xg.aggregator_list(P, A)
        for method in range(1, 21):
            s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=3, barrier_type=2, iteration=it)
            exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
            for pack, pform in PACKINGS:
                res = _run_job(xg, ctxs, s, it, 1, pack, rccl=rccl, reps=2 if "graph" in form else 1, form=pform)
                for (src, seed, dst, off), ck, nb, _fb in res:
                    assert nb == 0, (form, method, G, pack, pform, src, dst)
                    local = off - s.recv_offset(G, dst)
                    assert ck == O.chk64(exp[dst][local: local + d]), (form, method, G, pack, pform, src, dst)
    finally:
        for cx in ctxs:
            cx.close()


@pytest.mark.parametrize("graph", [False, True])
@pytest.mark.parametrize("rccl", [False, True])
@pytest.mark.parametrize("G", (2, 8))
def test_wave_copy_on_every_cross_gpu_launch(xg, rccl, G, graph):
    """XG_COPY_WAVE_MIN=0: every plain, 16-B aligned copy launch of a cross-GPU step (packs,
    unpacks, fused unpack + pack, the local part) runs copy_kernel_w (these launches are small:
    2 KiB pieces, wave_kib_for) -- every method, direct and both packed forms, a power-of-two -d
    and a ragged one (pieces of every length below the piece size), every slot against the
    oracle."""
    _wave_copy_jobs(xg, rccl, G, graph, {})


@pytest.mark.parametrize("kib", ["4", "8"])
def test_wave_copy_piece_sizes(xg, kib):
    """the same jobs with copy_kernel_w's piece size forced (XG_WAVE_KIB) to the 4 and 8 KiB
    forms larger launches pick (wave_kib_for): 8 GPUs, copies"""
    _wave_copy_jobs(xg, False, 8, False, {"XG_WAVE_KIB": kib})


def _wave_copy_jobs(xg, rccl, G, graph, extra):
    import os
    import xg_oracle as O
    env = dict(extra, XG_COPY_WAVE_MIN="0")
    if graph:
        env["XG_GRAPH"] = "1"           # the whole job captured once and replayed (twice below)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ctxs = [xg.Context.virtual(g, G, device=0) for g in range(G)]
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        P, A, c, k, it = 20, 6, 7, 2, 3
        rl = xg.aggregator_list(P, A)
        for d in (4096, 20000):
            for method in range(1, 21):
                s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, proc_node=3, barrier_type=2, iteration=it)
                exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
                for pack, pform in PACKINGS:
                    res = _run_job(xg, ctxs, s, it, 1, pack, rccl=rccl, form=pform, reps=2 if graph else 1)
                    for (src, seed, dst, off), ck, nb, _fb in res:
                        assert nb == 0, (d, method, G, pack, pform, src, dst)
                        local = off - s.recv_offset(G, dst)
                        assert ck == O.chk64(exp[dst][local: local + d]), (d, method, G, pack, pform, src, dst)
    finally:
        for cx in ctxs:
            cx.close()


@pytest.mark.parametrize("method", [7, 11, 12, 5, 8])
def test_one_gpu_share_alone(xg, method):
    """xg_plan_set_local_only: GPU 0 of an 8-GPU job runs its share alone (copy launches only,
    no RCCL).  Every slot whose source lives on GPU 0 is delivered bit-exact; every slot whose
    source is another GPU stays unwritten -- so the hook really leaves the exchange out (the
    full-size configs[4] share in profiles/ rests on this)."""
    import os
    import xg_oracle as O
    old = os.environ.get("XG_SELF_MAX")
    os.environ["XG_SELF_MAX"] = "0"           # local parts as copy launches, not self calls
    try:
        ctx = xg.Context.virtual(0, 8, device=0)
    finally:
        if old is None:
            del os.environ["XG_SELF_MAX"]
        else:
            os.environ["XG_SELF_MAX"] = old
    try:
        P, A, d, c, it, G = 64, 16, 65536, 3, 1, 8
        rl = xg.aggregator_list(P, A)
        s = xg.Schedule(method, P, A, d, c, rl, ntimes=1, iteration=it)
        for pack in (0, 1 << 30):
            run = xg.MethodRun(ctx, s, it=it, mode=1, pack_max_seg=pack)
            try:
                run.set_local_only()
                done, _post, wall = run.run_timed()
                assert all(0 <= a <= b for a, b in zip(done, done[1:])) and done[-1] <= wall + 1e-4
                chk, bad, _first = run.verify()
                lo, hi = s.block_range(G, 0)
                local = [lo <= src < hi for (src, _seed, _dst, _off) in run.slots]
                assert any(local) and not all(local)
                for (src, seed, dst, off), ck, nb, loc in zip(run.slots, chk, bad, local):
                    if loc:
                        assert nb == 0, (method, pack, src, dst)
                        assert ck == O.chk64(O.fingerprint(1, src, seed, it, d)), (method, pack, src, dst)
                    else:     # never received (poison, or unpacked from staging nobody filled)
                        assert nb > d // 2, (method, pack, src, dst, nb)
            finally:
                run.close()
    finally:
        ctx.close()


RELAYS = ((0, 2), (0, 3))           # XG_RELAY, XG_RELAY_COALESCED


@pytest.mark.parametrize("rccl", [False, True])
@pytest.mark.parametrize("G", (3, 8))
def test_relay_forms_every_method(xg, worlds, G, rccl):
    """both relay forms on every method 1-20 (TAM included) at P32 A16 -d (1 << 20) + 3 -- every
    relayed piece at an odd address, the coalesced form's packs and unpacks through the LDS realign
    path -- as a G-GPU job through copies and through RCCL: every slot byte-exact on the device,
    sampled checksums equal the oracle's closed form; the methods the relay forms reroute include
    the pairwise and half-sync ones"""
    import xg_oracle as O
    P, A, d, it = 32, 16, (1 << 20) + 3, 1
    rl = xg.aggregator_list(P, A)
    relayed = set()
    for method in range(1, 21):
        s = xg.Schedule(method, P, A, d, 3, rl, ntimes=1, iteration=it)
        for pack, form in RELAYS:
            v = s.devplan(G, 0, pack, 0, form)
            if any(k == xg.CALL_FENCE for st in range(v.nsteps) for k, *_ in v.calls(st)):
                relayed.add(method)
            res = _run_job(xg, worlds[G], s, it, 1, pack, rccl=rccl, form=form)
            assert res and all(nb == 0 for _slot, _ck, nb, _fb in res), (method, G, form, rccl)
            for (src, seed, _dst, _off), ck, _nb, _fb in res[:: max(1, len(res) // 5)]:
                assert ck == O.chk64(O.fingerprint(1, src, seed, it, d)), (method, G, form, src, seed)
    assert {9, 10, 11, 12} <= relayed, relayed


@pytest.mark.parametrize("step_form", ["split", "self_in_group", "local_in_fused", "graph"])
def test_relay_forms_under_every_step_form(xg, worlds, step_form):
    """the relay forms' steps (two RCCL groups; the coalesced form's packs, unpacks and in-place
    pieces) beside each way a cross-GPU step's local part can travel -- side stream, self send/recv
    in the first group, inside the fused pack launch -- and under graph replay: 8 GPUs through
    RCCL, pairwise / half-sync / TAM methods, every slot byte-exact"""
    import os
    P, A, d, it = 32, 16, 1 << 20, 1
    env = STEP_FORMS[step_form]
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        ctxs = [xg.Context.virtual(g, 8, device=0) for g in range(8)]     # the knobs are read at init
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v
    try:
        rl = xg.aggregator_list(P, A)
        for method in (9, 11, 12, 15):
            s = xg.Schedule(method, P, A, d, 3, rl, ntimes=1, iteration=it)
            for pack, form in RELAYS:
                res = _run_job(xg, ctxs, s, it, 1, pack, rccl=True, reps=2, form=form)
                assert res and all(nb == 0 for _slot, _ck, nb, _fb in res), (method, form, step_form)
    finally:
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("rccl", [False, True])
def test_relay_forms_large_pieces(xg, worlds, rccl):
    """P8 A4 -d (12 << 20) + 3 on 3 GPUs: pieces of 4 MiB and up, so the coalesced form's calls go one
    per piece, in place, and its relayed pieces are received and forwarded piece by piece (rc_split,
    as at configs[4]'s stated size) -- unordered, half-sync, pairwise, TAM; every slot byte-exact on
    the device, sampled checksums against the oracle's closed form"""
    import xg_oracle as O
    P, A, d, it, G = 8, 4, (12 << 20) + 3, 1, 3
    rl = xg.aggregator_list(P, A)
    for method in (1, 7, 9, 12, 15):
        s = xg.Schedule(method, P, A, d, 3, rl, ntimes=1, iteration=it)
        for pack, form in RELAYS:
            res = _run_job(xg, worlds[G], s, it, 1, pack, rccl=rccl, form=form)
            assert res and all(nb == 0 for _slot, _ck, nb, _fb in res), (method, form, rccl)
            for (src, seed, _dst, _off), ck, _nb, _fb in res[:: max(1, len(res) // 4)]:
                assert ck == O.chk64(O.fingerprint(1, src, seed, it, d)), (method, form, src, seed)
