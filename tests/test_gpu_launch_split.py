"""Copy launches cut into back-to-back dispatches (XG_COPY_LAUNCH_MAX, launch_cuts in
runtime/exec.hip).  By default only launches above 768 MiB are cut, which no ordinary test
plan reaches; here the cap is 64 KiB, so every launch of these plans is cut: local
gather/scatter launches, chained launches whose first dispatch stamps the previous step's
completion, and the fused unpack + pack launches of a packed multi-GPU plan.  Every
received byte is checked against the oracle, and the launch counts (xg_plan_launches and
the kernel-timing session) count the dispatches."""
import os

import pytest

pytestmark = pytest.mark.gpu

CAP = 64 << 10


def _ctx(xg, env, virtual=None):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        if virtual:
            return [xg.Context.virtual(g, virtual, device=0) for g in range(virtual)]
        return xg.Context(rank=0, nranks=1, device=0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _check(O, s, run, exp, d, G=1):
    chk, bad, first = run.verify()
    assert all(b == 0 for b in bad), [(sl, b, f) for sl, b, f in zip(run.slots, bad, first) if b][:3]
    for (src, seed, dst, off), ck in zip(run.slots, chk):
        local = off - s.recv_offset(G, dst)
        assert ck == O.chk64(exp[dst][local: local + d]), (s.method, src, dst)


@pytest.mark.parametrize("method", [1, 2, 3, 4, 6, 12])
def test_cut_launches_deliver_every_byte(xg, method):
    """one GPU, engine off (every step its own launches; m6 / m12 as chained launches): the
    same bytes as the uncut plan, and the cut plan dispatches more kernels"""
    import xg_oracle as O
    P, A, d, c, k, it = 32, 14, 48 << 10, 3, 2, 1      # m6 deadlocks above the eager limit (65424 B)
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, iteration=it)
    exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
    cut = _ctx(xg, {"XG_COPY_LAUNCH_MAX": str(CAP), "XG_ENGINE_MAX_STEP": "0"})
    whole = _ctx(xg, {"XG_ENGINE_MAX_STEP": "0"})
    try:
        rc, rw = xg.MethodRun(cut, s, it=it, mode=1), xg.MethodRun(whole, s, it=it, mode=1)
        try:
            assert rc.launches > rw.launches, (rc.launches, rw.launches)
            for _ in range(2):
                done, _post, wall = rc.run_timed()
                assert all(0 <= a <= b for a, b in zip(done, done[1:])), done
                assert done[-1] <= wall + 1e-4
            _check(O, s, rc, exp, d)
            rc.poison()
            # the kernel-timing session counts every dispatch, as rocprofv3 would
            cut.ktime_begin(per_launch=False)
            rc.enqueue()
            _ms, n, nbytes = cut.ktime_end()
            rc.check()
            assert n == rc.launches
            assert nbytes == 2 * k * P * A * d         # read + write of every delivered byte
            _check(O, s, rc, exp, d)
        finally:
            rc.close()
            rw.close()
    finally:
        cut.close()
        whole.close()


@pytest.mark.parametrize("method", [1, 6, 9, 12])
def test_cut_fused_unpack_pack_launches(xg, method):
    """a packed 2-GPU job on this device: packs, unpacks and the fused unpack + pack launches
    all cut at 64 KiB; every slot against the oracle"""
    import xg_oracle as O
    P, A, d, c, k, it = 32, 14, 16 << 10, 3, 2, 2
    rl = xg.aggregator_list(P, A)
    s = xg.Schedule(method, P, A, d, c, rl, ntimes=k, iteration=it)
    exp = O.expected_recv(method, P, A, d, rl, it, mode=1)
    ctxs = _ctx(xg, {"XG_COPY_LAUNCH_MAX": str(CAP), "XG_ENGINE_MAX_STEP": "0"}, virtual=2)
    try:
        runs = [xg.MethodRun(cx, s, it=it, mode=1, pack_max_seg=1 << 30) for cx in ctxs]
        try:
            assert any(r.view.p2p for r in runs)
            xg.run_virtual(runs)
            for r in runs:
                _check(O, s, r, exp, d, G=2)
        finally:
            for r in runs:
                r.close()
    finally:
        for cx in ctxs:
            cx.close()
