"""GPU: a timed run marks only the steps a Timer reads (xg_plan_set_step_marks, set by every
MethodRun and xg_run_method from xg_sched_timed_steps).  On GPU 0's local-only share of 8-GPU
plans (per-step launches, the path real multi-GPU runs take): every byte still lands, step times
stay ordered and every hosted rank's total lies inside the run, with every step marked and with
only the read ones (an unmarked per-step launch reads as the next marked step; steps inside an
engine segment keep their own stamps either way).  That no Timer field changes is proven on the
CPU for every captured configuration (tests/test_timed_steps.py)."""
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("method,P,A,d,c", [(9, 64, 16, 256 << 10, 200000000), (10, 64, 16, 65536, 200000000),
                                            (6, 32, 14, 2048, 3), (12, 32, 14, 4096, 3)])
def test_only_read_steps_are_marked(xg, method, P, A, d, c):
    import os
    G = 8
    old = os.environ.get("XG_SELF_MAX")
    os.environ["XG_SELF_MAX"] = "0"          # local parts as copy launches: the share runs alone
    try:
        ctx = xg.Context.virtual(0, G, device=0)
    finally:
        if old is None:
            del os.environ["XG_SELF_MAX"]
        else:
            os.environ["XG_SELF_MAX"] = old
    try:
        s = xg.Schedule(method, P, A, d, c, xg.aggregator_list(P, A), ntimes=2)
        need = s.timed_steps()
        assert 0 < sum(need) <= s.nsteps and need[-1] == 1
        run = xg.MethodRun(ctx, s, it=0, mode=1)
        try:
            run.set_local_only()
            lo, hi = s.block_range(G, 0)
            for marks in (None, need, None):
                run.set_step_marks(marks)
                for _ in range(2):
                    done, _post, wall = run.run_timed()
                    assert all(0 <= a <= b for a, b in zip(done, done[1:])) and done[-1] <= wall + 1e-4, done
                    for q in range(lo, hi):      # every hosted rank's report: inside the run
                        t = s.rank_timer(q, done, _post, G)
                        assert 0 <= t.total_time <= done[-1] + 1e-9, (q, t.as_tuple())
                _chk, bad, _f = run.verify()
                assert all(bad[i] == 0 for i, sl in enumerate(run.slots) if lo <= sl[0] < hi)
        finally:
            run.close()
    finally:
        ctx.close()
