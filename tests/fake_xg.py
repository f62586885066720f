"""A stand-in for the device half of xg.py, for running bench.py's control flow on a
CPU (tests/test_bench_logic.py).  Schedules, device plans, fill/verify descriptors and
timers are the REAL host library (libxghost.so); only what needs a GPU -- contexts,
RCCL, kernels -- is replaced by plausible no-ops.  Never imported by the product."""
import json
import os
import sys
import time
import types


def _faults(var):
    """XG_FAKE_VERIFY_FAIL / XG_FAKE_P2P_FAIL: comma-separated colon tuples of ints"""
    return {tuple(int(x) for x in f.split(":")) for f in os.environ.get(var, "").split(",") if f.strip()}


def make(real_xg):
    """fault injection (bench.py's partial-failure paths), on the rank XG_FAKE_FAIL_RANK names
    (default: every rank): XG_FAKE_VERIFY_FAIL=<method>:<pack_max_seg>:<pack_form>,... makes that
    plan's verify report a wrong slot; XG_FAKE_P2P_FAIL=<n>,... makes the n-th p2p_bench call
    (0-based: 0 = bench.py's xGMI ceiling, 1.. = its sweep) raise XGError; XG_FAKE_P2P_HANG=<n>,...
    makes it never return"""
    fake = types.ModuleType("xg")
    for name in ("aggregator_list", "Schedule", "XGError", "NBUF", "BUF_SEND", "BUF_RECV",
                 "BUF_STAGE_SEND", "BUF_STAGE_RECV", "BUF_SCRATCH", "PACK_TWO_SIDED", "PACK_ONE_SIDED",
                 "RELAY", "RELAY_COALESCED", "CALL_SEND", "CALL_RECV", "CALL_BARRIER", "CALL_FENCE", "method_label", "host"):
        setattr(fake, name, getattr(real_xg, name))
    calls = {"p2p_bench": 0, "ktime": [], "runs": 0}
    fake.calls = calls
    # every collective-level call this rank makes, in order (what its RCCL communicator
    # would see): compared across ranks by tests/test_rccl_calls.py
    trace = []
    fake.trace = trace

    def _on_fail_rank(rank):
        v = os.environ.get("XG_FAKE_FAIL_RANK")
        return v is None or int(v) == rank

    def _wait_all(d, name, nranks):
        t0 = time.time()
        while not all(os.path.exists(os.path.join(d, name % r)) for r in range(nranks)):
            if time.time() - t0 > 120:
                raise RuntimeError("fake collective %s: peers missing" % name)
            time.sleep(0.005)

    def unique_id():
        return b"\x01" * 128

    def _rccl_warn(msg):
        """what RCCL would write under NCCL_DEBUG=WARN when a call fails: one line in this rank's
        NCCL_DEBUG_FILE (bench.py attaches every rank's tail to a failed line)"""
        f = os.environ.get("NCCL_DEBUG_FILE")
        if f:
            with open(f, "a") as fh:
                fh.write("host:1:1 [0] NCCL WARN %s\n" % msg)

    fake.rccl_version = lambda: 22703

    class Context:
        def __init__(self, rank=0, nranks=1, device=None, uid=None, device_index=None):
            assert nranks == 1 or (uid is not None and len(uid) == 128)
            if os.environ.get("XG_FAKE_INIT_FAIL") == "1":     # e.g. RCCL's "Duplicate GPU detected"
                raise real_xg.XGError("xg_init failed with code 2 (injected)")
            self.rank, self.nranks = rank, nranks
            self._kt = None
            self._nbar = 0
            # like ncclCommInitRank, returns once every rank has joined (file barrier
            # when the test gives one: XG_FAKE_BARRIER_DIR)
            self.barrier()

        def barrier(self):
            """XG_FAKE_BARRIER_DIR set: a real barrier across the job's processes (one
            marker file per rank and barrier); otherwise a no-op"""
            trace.append(["barrier"])
            d = os.environ.get("XG_FAKE_BARRIER_DIR")
            if not d or self.nranks == 1:
                return
            i = self._nbar
            self._nbar += 1
            open(os.path.join(d, "b%d_r%d" % (i, self.rank)), "w").close()
            _wait_all(d, "b%d_r%%d" % i, self.nranks)

        def device_sync(self):
            pass

        def allreduce_max(self, vals):
            """XG_FAKE_BARRIER_DIR set: a real MAX over the job's processes (one file per rank
            and call), so every rank takes the same decisions as under RCCL"""
            trace.append(["allreduce_max", len(vals)])
            d = os.environ.get("XG_FAKE_BARRIER_DIR")
            if not d or self.nranks == 1:
                return list(vals)
            i = self._nred = getattr(self, "_nred", -1) + 1
            tmp = os.path.join(d, "a%d_r%d.tmp" % (i, self.rank))
            with open(tmp, "w") as f:
                json.dump(list(vals), f)
            os.replace(tmp, os.path.join(d, "a%d_r%d" % (i, self.rank)))
            _wait_all(d, "a%d_r%%d" % i, self.nranks)
            got = [json.load(open(os.path.join(d, "a%d_r%d" % (i, r)))) for r in range(self.nranks)]
            if any(len(x) != len(vals) for x in got):
                raise RuntimeError("fake allreduce %d: ranks reduce different lengths" % i)
            return [max(col) for col in zip(*got)]

        def info(self):
            return "gfx950:sramecc+:xnack-", 256, 309220868096

        def set_copy_params(self, chunk=0, variant=0):
            pass

        def ktime_begin(self, max_launches=4096, per_launch=True):
            self._kt = (max_launches, per_launch)
            calls["ktime"].append(self._kt)
            trace.append(["ktime_begin", bool(per_launch)])

        def ktime_end(self):
            per_launch = self._kt[1]
            n = self._kt[0] if per_launch else 8
            self._kt = None
            # region mode: a device time well inside the (near-instant) host-timed region
            return (0.15 * n if per_launch else 1e-6 * n), n, n * 1000000

        def p2p_bench(self, nbytes, mode=0, reps=20):
            calls["p2p_bench"] += 1
            trace.append(["p2p_bench", int(nbytes), int(mode), int(reps)])
            if _on_fail_rank(self.rank) and (calls["p2p_bench"] - 1,) in _faults("XG_FAKE_P2P_FAIL"):
                _rccl_warn("xg_p2p_bench: injected RCCL failure on rank %d" % self.rank)
                raise real_xg.XGError("xg_p2p_bench failed with code 5 (injected)")
            if _on_fail_rank(self.rank) and (calls["p2p_bench"] - 1,) in _faults("XG_FAKE_P2P_HANG"):
                while True:          # a peer lost inside RCCL: this call never returns
                    time.sleep(1)
            return 50.0, nbytes / 50e9

        def p2p_split_bench(self, nbytes, ncalls, reps=20):
            calls["split_bench"] = calls.get("split_bench", 0) + 1
            trace.append(["p2p_split_bench", int(nbytes), int(ncalls), int(reps)])
            if _on_fail_rank(self.rank) and (calls["split_bench"] - 1,) in _faults("XG_FAKE_SPLIT_FAIL"):
                _rccl_warn("xg_p2p_split_bench: injected RCCL failure on rank %d" % self.rank)
                raise real_xg.XGError("xg_p2p_split_bench failed with code 2 (injected)")
            sec = nbytes / 50e9 + 5e-6 * ncalls        # 5 us per call: a visible per-call cost
            return nbytes * (self.nranks - 1) / sec / 1e9, sec

        def p2p_pair_bench(self, nbytes, peer, reps=10):
            calls["pair_bench"] = calls.get("pair_bench", 0) + 1
            trace.append(["p2p_pair_bench", int(nbytes), int(reps)])     # the peer differs by rank (pair_rounds)
            if _on_fail_rank(self.rank) and (calls["pair_bench"] - 1,) in _faults("XG_FAKE_PAIR_FAIL"):
                _rccl_warn("xg_p2p_pair_bench: injected RCCL failure on rank %d" % self.rank)
                raise real_xg.XGError("xg_p2p_pair_bench failed with code 2 (injected)")
            if peer < 0:
                return 0.0, 0.0
            return 40.0 + peer + self.rank, nbytes / 40e9      # distinct per link: the spread is visible

        def close(self):
            pass

    class MethodRun:
        def __init__(self, ctx, sched, it=0, mode=0, pack_max_seg=4 << 20, regions=None, pack_min=0, pack_form=-1):
            self.ctx, self.sched, self.pack_max_seg, self.pack_form = ctx, sched, pack_max_seg, pack_form
            if os.environ.get("XG_FAKE_PLAN_FAIL") == "%d:%d" % (sched.method, ctx.rank):
                raise real_xg.XGError("xg_regions_alloc failed with code 4 (injected)")
            G, g = ctx.nranks, ctx.rank
            if G > 1:     # as the real MethodRun: refuse calls RCCL would not pair
                sched.check_pairing(G, pack_max_seg, pack_min, pack_form,
                                    int(os.environ.get("XG_SELF_MAX", 256 << 10)))
            self.view = sched.devplan(G, g, pack_max_seg, pack_min, pack_form)
            if regions is not None and not regions.fits(self.view.region_bytes):     # as the real MethodRun
                raise real_xg.XGError("MethodRun: shared regions too small for this plan")
            # the RCCL calls this GPU's plan posts per run: per step its send/recv group and
            # its barrier (xg_devplan_step_calls), as a signature the ranks must agree on in
            # everything collective (the barriers) -- the p2p pairing is xg_devplans_match's
            self.barrier_steps = [st for st in range(self.view.nsteps) if self.view.sync_after[st]]
            self.key = [sched.method, sched.P, sched.A, sched.d, sched.c, sched.ntimes, pack_max_seg]
            trace.append(["plan"] + self.key + [self.barrier_steps])
            self.nsteps = self.view.nsteps
            self.slots = sched.verify_slots(G, g)
            self.engine_workgroups = 0
            self.engine_rails = 0

        @property
        def launches(self):
            return sum(1 for st in self.view.steps if st[1]) + sum(1 for st in self.view.steps if st[5])

        def run_timed(self):
            calls["runs"] += 1
            trace.append(["run"] + self.key)
            done = [1e-5 * (s + 1) for s in range(self.nsteps)]
            return done, [1e-6] * self.nsteps, done[-1] if done else 0.0

        def verify(self):
            n = len(self.slots)
            bad = [0] * n
            if n and _on_fail_rank(self.ctx.rank) and \
                    (self.sched.method, self.pack_max_seg, self.pack_form) in _faults("XG_FAKE_VERIFY_FAIL"):
                bad[0] = 7
            return [0] * n, bad, [-1] * n

        def enqueue(self):
            trace.append(["enqueue"] + self.key)
            # XG_FAKE_FORM_DELAY=<pack_form>:<ms>,...: a run of that form takes that long (the
            # form-choice rule's integration tests)
            for f in os.environ.get("XG_FAKE_FORM_DELAY", "").split(","):
                if f.strip() and int(f.split(":")[0]) == self.pack_form:
                    time.sleep(float(f.split(":")[1]) / 1e3)

        def check(self):
            pass

        def close(self):
            pass

    class Regions:
        def __init__(self, ctx, region_bytes):
            self.bytes = list(region_bytes)
            lim = os.environ.get("XG_FAKE_REGIONS_FAIL")       # "<max bytes>:<rank>"
            if lim and int(lim.split(":")[1]) == ctx.rank and sum(self.bytes) > int(lim.split(":")[0]):
                raise real_xg.XGError("xg_regions_alloc failed with code 4 (injected: %d B)" % sum(self.bytes))
            trace.append(["regions", [int(b) for b in region_bytes]])

        def fits(self, region_bytes):
            return all(a <= b for a, b in zip(region_bytes, self.bytes))

        def close(self):
            pass

    fake.unique_id = unique_id
    fake.Context = Context
    fake.MethodRun = MethodRun
    fake.Regions = Regions
    return fake


def install(real_pkg):
    """replace sys.modules['xgamd'] by a package whose .xg is the fake"""
    pkg = types.ModuleType("xgamd")
    pkg.xg = make(real_pkg.xg)
    sys.modules["xgamd"] = pkg
    return pkg.xg
