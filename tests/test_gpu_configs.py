"""BASELINE.json configs as GPU parity cases (1 MI355X hosts every logical rank).

At these sizes the oracle cannot replay the bytes on the CPU in seconds, so the
checks are size-independent: every received byte is compared on the device with
the closed-form fingerprint (xg_verify: zero mismatching bytes, strong mode so a
misroute cannot hide), the CPU oracle confirms the schedule (every rank's MPI
call trace equals the oracle's restatement), and the sum of the per-slot
checksums equals the oracle's closed-form value for a sample of slots.

The oracle's traces at these P = 256 shapes are themselves pinned to the reference: every rank's
whole MPI program at configs[3]'s and configs[4]'s shapes equals the reference's by digest
(tests/test_baseline_golden.py, captured at a reduced -d for every -c), and the programs at the
stated -d are those with every count scaled (test_stated_size_schedules_are_the_captured_ones).
"""
import pytest

import xg_oracle as O

pytestmark = pytest.mark.gpu

CASES = [
    # (name, P, A, d, c, methods, k)
    ("config2_p32_a14_d1m", 32, 14, 1 << 20, 200000000, range(1, 13), 2),
    ("config3_p64_a16_d256k", 64, 16, 256 << 10, 200000000, range(1, 13), 1),
    ("config4_p256_a32_d4m", 256, 32, 4 << 20, 200000000, (1, 2, 9, 10), 1),
    ("config5_p256_a64_d256k_c1", 256, 64, 256 << 10, 1, (7, 11, 12), 1),
    ("config5_p256_a64_d256k_c3", 256, 64, 256 << 10, 3, (7, 11, 12), 1),
    ("config5_p256_a64_d256k_c8", 256, 64, 256 << 10, 8, (7, 11, 12), 1),
]


@pytest.fixture(scope="module")
def ctx(xg):
    c = xg.Context(rank=0, nranks=1, device=0)
    yield c
    c.close()


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_config(xg, ctx, case):
    _name, P, A, d, c, methods, k = case
    rl = xg.aggregator_list(P, A)
    for m in methods:
        try:
            s = xg.Schedule(m, P, A, d, c, rl, ntimes=k)
        except xg.XGError as e:
            # the only refusal allowed: a schedule the reference itself deadlocks on
            assert "deadlocks" in str(e) and m == 6, e
            with pytest.raises(RuntimeError, match="deadlock"):
                O.asap_steps(O.programs(m, P, A, d, c, rl, k))
            continue
        run = xg.MethodRun(ctx, s, it=1, mode=1)
        try:
            done, _post, _wall = run.run_timed()
            assert len(done) == s.nsteps and all(t >= 0 for t in done)
            chk, bad, first = run.verify()
            assert sum(1 for b in bad if b) == 0, (m, [(sl, b, f) for sl, b, f in zip(run.slots, bad, first) if b][:3])
            # sampled slots: checksum equals the oracle closed form
            for i in range(0, len(run.slots), max(1, len(run.slots) // 7)):
                src, seed, dst, _off = run.slots[i]
                assert chk[i] == O.chk64(O.fingerprint(1, src, seed, 1, d)), (m, i)
        finally:
            run.close()
        # the schedule: per-rank trace identical to the oracle's restatement (sampled ranks)
        progs = O.programs(m, P, A, d, c, rl, k)
        for r in range(0, P, max(1, P // 16)):
            assert s.trace(r) == O.trace_tokens(progs[r]), (m, r)


@pytest.mark.parametrize("method", [5, 8])
def test_alltoallw_beyond_int32_displacements(xg, ctx, method):
    """(P-1)*d >= 2^31: the reference's int displacement arrays (*_alltoall_translate,
    mpi_test.c:233-302) overflow and it segfaults (P5 A2 -d 512 MiB, MPICH here); this build
    keeps 64-bit offsets and delivers every segment.  No reference output exists, so the
    check is the closed form: zero mismatching bytes on the device (strong fingerprint), and
    the checksums of the segments whose offsets pass 2^31 equal the oracle's."""
    P, A, d = 5, 2, 512 << 20
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, 200000000, rl, ntimes=1)
    run = xg.MethodRun(ctx, s, it=1, mode=1)
    try:
        run.run_timed()
        chk, bad, first = run.verify()
        assert len(run.slots) == P * A and not any(bad), [(sl, b, f) for sl, b, f in zip(run.slots, bad, first) if b]
        far = [i for i, (_src, _seed, _dst, off) in enumerate(run.slots) if off >= 1 << 31][:2]
        assert far
        for i in far:
            src, seed, _dst, _off = run.slots[i]
            assert chk[i] == O.chk64(O.fingerprint(1, src, seed, 1, d)), (method, run.slots[i])
    finally:
        run.close()


@pytest.fixture(scope="module")
def big_regions(xg, ctx):
    """one 256 GiB SEND + RECV allocation for the whole -c sweep (last tests of the module)"""
    P, A, d = 256, 64, 8 << 20
    r = xg.Regions(ctx, [P * A * d, P * A * d, 0, 0, 0])
    yield r
    r.close()


@pytest.mark.parametrize("c", range(1, 9))
def test_config5_largest_single_gpu_size(xg, ctx, big_regions, c):
    """configs[4] (P256 A64, half-sync m7 / m11 / m12) at the largest -d one MI355X
    holds -- 8 MiB: 128 GiB SEND + 128 GiB RECV in HBM -- at every -c of the
    reference's sweep (script_theta_all_to_many_256.sh:33-106 sweeps -c; here 1..8).
    Every received byte checked on the device (strong fingerprint), sampled slot
    checksums against the oracle's closed form."""
    P, A, d = 256, 64, 8 << 20
    _arch, _cus, hbm = ctx.info()
    rl = xg.aggregator_list(P, A)
    for m in (7, 11, 12):
        s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
        need = sum(s.region_bytes(1, 0, b) for b in range(xg.NBUF))
        assert need == 2 * P * A * d and need < hbm, (need, hbm)
        run = xg.MethodRun(ctx, s, it=1, mode=1, regions=big_regions)
        try:
            done, _post, _wall = run.run_timed()
            assert len(done) == s.nsteps and all(0 <= a <= b for a, b in zip(done, done[1:]))
            chk, bad, first = run.verify()
            assert len(run.slots) == P * A
            assert not any(bad), (m, c, [(sl, b, f) for sl, b, f in zip(run.slots, bad, first) if b][:3])
            for i in range(0, len(run.slots), len(run.slots) // 5):
                src, seed, _dst, _off = run.slots[i]
                assert chk[i] == O.chk64(O.fingerprint(1, src, seed, 1, d)), (m, c, i)
        finally:
            run.close()
