"""A stand-in for the device half of xg.py, for running bench.py's control flow on a
CPU (tests/test_bench_logic.py).  Schedules, device plans, fill/verify descriptors and
timers are the REAL host library (libxghost.so); only what needs a GPU -- contexts,
RCCL, kernels -- is replaced by plausible no-ops.  Never imported by the product."""
import os
import sys
import time
import types


def make(real_xg):
    fake = types.ModuleType("xg")
    for name in ("aggregator_list", "Schedule", "XGError", "NBUF", "BUF_SEND", "BUF_RECV",
                 "BUF_STAGE_SEND", "BUF_STAGE_RECV", "BUF_SCRATCH", "method_label", "host"):
        setattr(fake, name, getattr(real_xg, name))
    calls = {"p2p_bench": 0, "ktime": [], "runs": 0}
    fake.calls = calls

    def unique_id():
        return b"\x01" * 128

    class Context:
        def __init__(self, rank=0, nranks=1, device=None, uid=None, device_index=None):
            assert nranks == 1 or (uid is not None and len(uid) == 128)
            self.rank, self.nranks = rank, nranks
            self._kt = None
            self._nbar = 0
            # like ncclCommInitRank, returns once every rank has joined (file barrier
            # when the test gives one: XG_FAKE_BARRIER_DIR)
            self.barrier()

        def barrier(self):
            """XG_FAKE_BARRIER_DIR set: a real barrier across the job's processes (one
            marker file per rank and barrier); otherwise a no-op"""
            d = os.environ.get("XG_FAKE_BARRIER_DIR")
            if not d or self.nranks == 1:
                return
            i = self._nbar
            self._nbar += 1
            open(os.path.join(d, "b%d_r%d" % (i, self.rank)), "w").close()
            t0 = time.time()
            while not all(os.path.exists(os.path.join(d, "b%d_r%d" % (i, r))) for r in range(self.nranks)):
                if time.time() - t0 > 120:
                    raise RuntimeError("fake barrier %d: peers missing" % i)
                time.sleep(0.01)

        def device_sync(self):
            pass

        def allreduce_max(self, vals):
            return list(vals)

        def info(self):
            return "gfx950:sramecc+:xnack-", 256, 309220868096

        def set_copy_params(self, chunk=0, variant=0):
            pass

        def ktime_begin(self, max_launches=4096, per_launch=True):
            self._kt = (max_launches, per_launch)
            calls["ktime"].append(self._kt)

        def ktime_end(self):
            per_launch = self._kt[1]
            n = self._kt[0] if per_launch else 8
            self._kt = None
            # region mode: a device time well inside the (near-instant) host-timed region
            return (0.15 * n if per_launch else 1e-6 * n), n, n * 1000000

        def p2p_bench(self, nbytes, mode=0, reps=20):
            calls["p2p_bench"] += 1
            return 50.0, nbytes / 50e9

        def close(self):
            pass

    class MethodRun:
        def __init__(self, ctx, sched, it=0, mode=0, pack_max_seg=4 << 20, regions=None):
            self.ctx, self.sched, self.pack_max_seg = ctx, sched, pack_max_seg
            G, g = ctx.nranks, ctx.rank
            self.view = sched.devplan(G, g, pack_max_seg)
            self.nsteps = self.view.nsteps
            self.slots = sched.verify_slots(G, g)
            self.engine_workgroups = 0
            self.engine_rails = 0

        @property
        def launches(self):
            return sum(1 for st in self.view.steps if st[1]) + sum(1 for st in self.view.steps if st[5])

        def run_timed(self):
            calls["runs"] += 1
            done = [1e-5 * (s + 1) for s in range(self.nsteps)]
            return done, [1e-6] * self.nsteps, done[-1] if done else 0.0

        def verify(self):
            n = len(self.slots)
            return [0] * n, [0] * n, [-1] * n

        def enqueue(self):
            pass

        def check(self):
            pass

        def close(self):
            pass

    fake.unique_id = unique_id
    fake.Context = Context
    fake.MethodRun = MethodRun
    return fake


def install(real_pkg):
    """replace sys.modules['xgamd'] by a package whose .xg is the fake"""
    pkg = types.ModuleType("xgamd")
    pkg.xg = make(real_pkg.xg)
    sys.modules["xgamd"] = pkg
    return pkg.xg
