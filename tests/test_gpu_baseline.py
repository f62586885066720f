"""GPU parity at the BASELINE.json configuration shapes, against the REAL reference.

1. test_baseline_one_gpu / test_baseline_virtual8_rccl: every fixture of tests/golden/baseline/
   (the reference captured under MPICH at configs[1] and configs[2] at full size, configs[3]'s
   P256 A32 at -d 64 KiB, configs[4]'s P256 A64 at -d 4 KiB for -c 1..8; make_baseline.py) run
   through libxg with the reference's own MAP_DATA bytes, on one GPU and as an 8-GPU job on this
   device whose cross-GPU pairs go through RCCL (self ncclSend / ncclRecv on a 1-rank
   communicator), direct and both packed forms: every received segment's xg_chk64 equals the
   checksum the reference's receive buffer had, and no byte differs from the closed form.
2. test_config3_full_size_virtual8 / test_config4_d8m_virtual8: every byte of the 8-GPU plans
   of configs[3] (P256 A32 -d 4 MiB, m1 / m2 / m9 / m10) and configs[4] (P256 A64, m7 / m11 /
   m12, -c 1..8, at -d 8 MiB: 256 GiB for the 8 GPUs' regions) moved on the device as an 8-GPU
   job, verified slot by slot (collision-free fingerprint) -- configs[4]'s m11 / m12 in both relay
   forms too, m7 in the coalesced form's weighted split (profiles/r06/relay_c4.log, split_tests.log).
3. test_config4_stated_size_gpu0_share: configs[4] at its stated -d 64 MiB, GPU 0's share of the
   8-GPU job (256 GiB of regions) run alone, every -c.
Reference: mpi_test.c:1748-1950 (m1 / m2), :421-597 (m9 / m10), :942-1114 (m11 / m12 / m7).
"""
import pytest

import xg_oracle as O
from conftest import baseline_configs, load_baseline

pytestmark = pytest.mark.gpu

# (pack_max_seg, pack form): direct / one-sided / two-sided
PACKINGS = ((0, -1), (1 << 30, 1), (1 << 30, 0))


@pytest.fixture(scope="module")
def ctx(xg):
    c = xg.Context(rank=0, nranks=1, device=0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def world8(xg):
    w = [xg.Context.virtual(g, 8, device=0) for g in range(8)]
    yield w
    for c in w:
        c.close()


def _sched(xg, meta, method, it):
    return xg.Schedule(method, meta["P"], meta["A"], meta["d"], meta["c"], meta["aggregators"],
                       ntimes=meta["ntimes"], proc_node=meta["proc_node"], iteration=it)


def _check_golden(cfg, meta, data, method, it, results, tag):
    direction = O.direction(method)
    assert len(results) == sum(1 for key in data[direction] if key[0] == it), (cfg, method, tag)
    for (src, _seed, dst, _off), ck, nb, fb in results:
        assert nb == 0, "%s m%d it%d %s %d->%d: %d bad bytes from %d" % (cfg, method, it, tag, src, dst, nb, fb)
        glen, gchk = data[direction][(it, src, dst)]
        assert glen == meta["d"] and ck == gchk, (cfg, method, it, tag, src, dst, hex(ck), hex(gchk))


@pytest.mark.parametrize("cfg", baseline_configs())
def test_baseline_one_gpu(xg, ctx, cfg):
    meta, _, data = load_baseline(cfg)
    for method in meta["method_list"]:
        for it in range(meta["iters"]):
            run = xg.MethodRun(ctx, _sched(xg, meta, method, it), it=it, mode=0)
            try:
                done, _post, wall = run.run_timed()
                assert all(0 <= a <= b for a, b in zip(done, done[1:])) and done[-1] <= wall + 1e-4
                chk, bad, first = run.verify()
                _check_golden(cfg, meta, data, method, it, list(zip(run.slots, chk, bad, first)), "1gpu")
            finally:
                run.close()


def _run_job(xg, ctxs, s, it, mode, pack, form, rccl, regions=None):
    runs = []
    try:
        for g, c in enumerate(ctxs):
            runs.append(xg.MethodRun(c, s, it=it, mode=mode, pack_max_seg=pack, pack_form=form,
                                     regions=regions[g] if regions else None))
        done = xg.run_virtual(runs, rccl=rccl)
        assert all(0 <= a <= b for a, b in zip(done, done[1:]))
        out = []
        for r in runs:
            chk, bad, first = r.verify()
            out += list(zip(r.slots, chk, bad, first))
        return out
    finally:
        for r in runs:
            r.close()


@pytest.mark.parametrize("cfg", baseline_configs())
def test_baseline_virtual8_rccl(xg, world8, cfg):
    """every capture as an 8-GPU job over RCCL in every form; at configs[1]'s full size (1 MiB
    segments) the relay forms reroute m9 / m10's cross-GPU XOR rounds (and the steps of other
    methods their link model favours) over every link -- the reference's checksums still hold"""
    meta, _, data = load_baseline(cfg)
    it = meta["iters"] - 1
    forms = PACKINGS + (((0, 2), (0, 3)) if meta["d"] >= 1 << 20 else ())
    for method in meta["method_list"]:
        s = _sched(xg, meta, method, it)
        for pack, form in forms:
            res = _run_job(xg, world8, s, it, 0, pack, form, rccl=True)
            _check_golden(cfg, meta, data, method, it, res, "G8 rccl pack%d/%d" % (pack, form))


@pytest.mark.parametrize("G", [2, 4])
@pytest.mark.parametrize("cfg", ["cfg1_p32_a14_d1m", "cfg2_p64_a16_d256k"])
def test_baseline_scaling_jobs_rccl(xg, cfg, G):
    """the bench's N = 2 and 4 workloads (configs[1], and configs[2]'s shape) as G-GPU jobs over
    RCCL, direct / one-sided / two-sided, every slot against the reference's checksums"""
    meta, _, data = load_baseline(cfg)
    it = meta["iters"] - 1
    ctxs = [xg.Context.virtual(g, G, device=0) for g in range(G)]
    try:
        for method in meta["method_list"]:
            s = _sched(xg, meta, method, it)
            for pack, form in PACKINGS:
                res = _run_job(xg, ctxs, s, it, 0, pack, form, rccl=True)
                _check_golden(cfg, meta, data, method, it, res, "G%d rccl pack%d/%d" % (G, pack, form))
    finally:
        for c in ctxs:
            c.close()


def _shared_regions(xg, ctxs, scheds, packings):
    """one Regions per virtual GPU, sized for every (schedule, packing) it will run"""
    G = len(ctxs)
    need = [[0] * xg.NBUF for _ in range(G)]
    for s in scheds:
        for pack, form in packings:
            for g in range(G):
                rb = s.devplan(G, g, pack, 0, form).region_bytes
                need[g] = [max(a, b) for a, b in zip(need[g], rb)]
    return [xg.Regions(c, n) for c, n in zip(ctxs, need)]


def _check_strong(s, res, d, it, tag, sample=7):
    assert len(res) == s.P * s.A, tag
    assert all(nb == 0 for _sl, _ck, nb, _fb in res), (tag, [(sl, nb, fb) for sl, _ck, nb, fb in res if nb][:3])
    for (src, seed, _dst, _off), ck, _nb, _fb in res[:: max(1, len(res) // sample)]:
        assert ck == O.chk64(O.fingerprint(1, src, seed, it, d)), (tag, src, seed)


@pytest.mark.parametrize("method", [1, 2, 9, 10])
def test_config3_full_size_virtual8(xg, world8, method):
    """configs[3] at full size (P256 A32 -d 4 MiB: 32 GiB per direction) as an 8-GPU job: the
    cross-GPU pairs as device copies in RCCL's pairing for direct / one-sided / two-sided / relay /
    coalesced relay, and through RCCL itself for the direct and both relay forms"""
    P, A, d, it = 256, 32, 4 << 20, 1
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, 200000000, rl, ntimes=1, iteration=it)
    relay = (0, 2)           # XG_RELAY: m9 / m10's cross-GPU rounds over every link, two RCCL groups
    coal = (0, 3)            # XG_RELAY_COALESCED: the same hops, one call per hop and kind
    regions = _shared_regions(xg, world8, [s], PACKINGS + (relay, coal))
    try:
        for (pack, form), rccl in [(p, False) for p in PACKINGS + (relay, coal)] + \
                [(PACKINGS[0], True), (relay, True), (coal, True)]:
            res = _run_job(xg, world8, s, it, 1, pack, form, rccl, regions)
            _check_strong(s, res, d, it, ("m%d" % method, pack, form, rccl))
    finally:
        for r in regions:
            r.close()


def _relayed_steps(xg, s, G, form):
    """steps of GPU 0's plan in `form` that post a second RCCL group (the relay form's forwards)"""
    v = s.devplan(G, 0, form[0], 0, form[1])
    return sum(1 for st in range(v.nsteps) if any(k == xg.CALL_FENCE for k, *_ in v.calls(st)))


@pytest.mark.parametrize("cs", [(1, 2, 3, 4), (5, 6, 7, 8)], ids=["c1-4", "c5-8"])
def test_config4_d8m_virtual8(xg, world8, cs):
    """configs[4] (P256 A64, m7 / m11 / m12) at -d 8 MiB -- 16 GiB of SEND + 16 GiB of RECV per
    GPU, 256 GiB for the job -- as an 8-GPU job at every -c in 1..8 (device copies in RCCL's
    pairing), and through RCCL itself at -c 1 and -c 8; regions allocated once per GPU and half of
    the sweep.  m11 / m12 also in the relay form (XG_RELAY) and the coalesced relay form
    (XG_RELAY_COALESCED), the forms the N = 8 BASELINE phase times beside direct on exactly these
    plans (profiles/r05/link_load.txt): every -c through copies (the coalesced form at -c 1 and 8),
    -c 1 and 8 through RCCL.  m7, which no uniform cut helps, runs in the coalesced form's weighted
    two-hop split (every step) at -c 1 and 8."""
    P, A, d, it = 256, 64, 8 << 20, 1
    rl = xg.aggregator_list(P, A)
    scheds = {(m, c): xg.Schedule(m, P, A, d, c, rl, ntimes=1, iteration=it) for m in (7, 11, 12)
              for c in cs}
    pack = (4 << 20, -1)              # the default: 8 MiB segments are never packed
    relay, coal = (0, 2), (0, 3)
    regions = _shared_regions(xg, world8, list(scheds.values()), (pack, relay, coal))
    try:
        for (m, c), s in scheds.items():
            # the coalesced form at the -c the N = 8 bench reaches first (the suite's time: 1 and 8)
            forms = [pack] + ([relay] if m != 7 else []) + ([coal] if c in (1, 8) else [])
            # the relay forms must reroute these plans, or this test checks nothing new: m11 / m12
            # in both (the same steps), m7 only in the coalesced form's weighted two-hop split
            assert _relayed_steps(xg, s, 8, pack) == 0, (m, c)
            if m != 7:
                assert _relayed_steps(xg, s, 8, relay) == _relayed_steps(xg, s, 8, coal) > 0, (m, c)
            else:
                assert _relayed_steps(xg, s, 8, relay) == 0 and _relayed_steps(xg, s, 8, coal) == 64
            for form in forms:
                for rccl in ((False, True) if c in (1, 8) else (False,)):
                    res = _run_job(xg, world8, s, it, 1, form[0], form[1], rccl, regions)
                    _check_strong(s, res, d, it, ("m%d" % m, c, form, rccl), sample=5)
    finally:
        for r in regions:
            r.close()


def test_config4_stated_size_gpu0_share(xg):
    """configs[4] at its stated size (P256 A64 -d 64 MiB on 8 GPUs: 128 GiB SEND + 128 GiB RECV
    per GPU): GPU 0's plan run alone on this device (xg_plan_set_local_only: its copy launches,
    its RCCL calls left out) for m7 / m11 / m12 at every -c -- the 64 MiB per-GPU plan the
    driver's 8-GPU run executes.  Every slot whose source lives on GPU 0 is bit-exact, every
    slot a peer would fill is still unwritten."""
    import os
    P, A, d, G, it = 256, 64, 64 << 20, 8, 1
    old = os.environ.get("XG_SELF_MAX")
    os.environ["XG_SELF_MAX"] = "0"          # local parts as copy launches (no RCCL self calls)
    try:
        ctx = xg.Context.virtual(0, G, device=0)
    finally:
        if old is None:
            del os.environ["XG_SELF_MAX"]
        else:
            os.environ["XG_SELF_MAX"] = old
    rl = xg.aggregator_list(P, A)
    R = None
    try:
        scheds = {(m, c): xg.Schedule(m, P, A, d, c, rl, ntimes=1, iteration=it) for m in (7, 11, 12)
                  for c in range(1, 9)}
        need = [0] * xg.NBUF
        for m in (7, 11, 12):
            need = [max(a, b) for a, b in zip(need, scheds[(m, 1)].devplan(G, 0).region_bytes)]
        _arch, _cus, hbm = ctx.info()
        assert sum(need) == 2 * (P // G) * A * d < hbm, (need, hbm)
        R = [xg.Regions(ctx, need)]
        lo, hi = scheds[(7, 1)].block_range(G, 0)
        for (m, c), s in scheds.items():
            run = xg.MethodRun(ctx, s, it=it, mode=1, regions=R[0])
            try:
                run.set_local_only()
                done, _post, wall = run.run_timed()
                assert all(0 <= a <= b for a, b in zip(done, done[1:])) and done[-1] <= wall + 1e-4
                chk, bad, _first = run.verify()
                local = [i for i, sl in enumerate(run.slots) if lo <= sl[0] < hi]
                assert local and len(local) < len(run.slots)
                assert all(bad[i] == 0 for i in local), (m, c)
                lset = set(local)
                assert all(bad[i] > d // 2 for i in range(len(run.slots)) if i not in lset), (m, c)
                for i in (local[0], local[len(local) // 2], local[-1]):
                    src, seed, _dst, _off = run.slots[i]
                    assert chk[i] == O.chk64(O.fingerprint(1, src, seed, it, d)), (m, c, i)
            finally:
                run.close()
    finally:
        if R:
            R[0].close()
        ctx.close()
