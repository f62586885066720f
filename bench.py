#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric on the MI355X build.

Metric: aggregate exchange GB/s (+ max total time per method), all-to-many /
many-to-all.  Workload (BASELINE.json configs[1], the single-GPU config):
32 logical ranks, 14 aggregators (type-1 placement), -d 1 MiB, methods 1-4,
default -c.  One bench STEP = one -k repetition of each of methods 1, 2, 3, 4,
i.e. 4 x P*A*d = 1.75 GiB of segments delivered.  Inputs (the fingerprinted
send buffers) are resident in HBM before the timed region, as in the
reference (prepare_*_data is untimed).

    python bench.py [--gpus N] [--steps K] [--warmup W]

One process per GPU.  N > 1 either under a launcher that sets RANK /
WORLD_SIZE / LOCAL_RANK (torch.distributed.run, mpiexec) or on its own: with
no WORLD_SIZE in the environment `--gpus N` makes this process a parent that
never touches the GPU -- it runs the host-MPI baseline, starts N child
processes of itself (one per GPU, RANK / LOCAL_RANK / WORLD_SIZE and one
rendezvous key set), waits for all of them, fails with the highest child exit
code if any fails, and prints rank 0's JSON line with the baseline attached.
The same 32 logical ranks are block-mapped onto N GPUs and cross-GPU segments
move with grouped RCCL send/recv (strong scaling).  The processes never import
torch: barrier, MAX-reduction and device sync go through the framework's own
C-ABI (RCCL + hipDeviceSynchronize), and the RCCL id is handed over through a
file.

Before timing, every method's delivery is verified on the GPU (byte-exact
against the fingerprint); the bench aborts on any mismatch.  After timing, the
step engine's timeout word is checked (a timed-out barrier would have moved
only part of the bytes).
"""
import argparse
import json
import os
import re
import shutil
import statistics
import subprocess
import threading
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "aggregate exchange GB/s + max total time, all-to-many/many-to-all, 1–8 GPUs"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md); 6.29 TB/s measured copy


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--procs", type=int, default=32)
    ap.add_argument("--aggs", type=int, default=14)
    ap.add_argument("--size", type=int, default=1 << 20)
    ap.add_argument("--comm-size", type=int, default=200000000)
    ap.add_argument("--methods", default="1,2,3,4")
    ap.add_argument("--pack-max-seg", type=int, default=4 << 20)
    ap.add_argument("--tune-pack", type=int, default=-1,
                    help="1/0: time direct vs packed (one-/two-sided) cross-GPU plans per method and keep the fastest "
                         "(default: on when N > 1 and --pack-max-seg is left at its default)")
    ap.add_argument("--copy-variant", type=int, default=-1)
    ap.add_argument("--chunk", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-ktime", action="store_true",
                    help="N > 1: skip the per-launch roofline pass")
    ap.add_argument("--child-timeout", type=float, default=0,
                    help="parent mode: seconds before the children are stopped (0: none)")
    ap.add_argument("--cpu-reps", type=int, default=10, help="-k of the reference CPU run")
    ap.add_argument("--baseline-configs", choices=("auto", "on", "off"), default="auto",
                    help="after the line's own measurements, run BASELINE.json's 8-GPU configurations "
                         "(configs[2], [3], [4] at their stated sizes) on this job and add them to the line "
                         "(auto: only when the job has 8 GPUs)")
    ap.add_argument("--baseline-budget", type=float, default=130.0,
                    help="seconds the BASELINE-configs phase may take; cells past it are skipped (all ranks "
                         "alike), and a phase still running GUARD_GRACE s later prints the line without the rest")
    ap.add_argument("--xgmi-budget", type=float, default=20.0,
                    help="N > 1: seconds the xGMI ceiling + sweep phase may take before the line is printed "
                         "without the rest of it")
    ap.add_argument("--watchdog", type=float, default=float(os.environ.get("XG_BENCH_WATCHDOG", 110)),
                    help="rank process: seconds from the communicator init to the measured value before a rank "
                         "that is still running reports the phase it is stuck in and exits 124 (0: off) -- a lost "
                         "peer leaves RCCL waiting forever; the phases after the value have guards of their own")
    ap.add_argument("--cpu-budget", type=float, default=30.0,
                    help="seconds the reference's configs[1] run under mpiexec may take in all")
    ap.add_argument("--cpu-configs", choices=("auto", "on", "off"), default="auto",
                    help="run the reference under mpiexec at BASELINE.json's 8-GPU configurations (configs[2] at "
                         "full size, configs[3] and [4] at -d 4 KiB) before the GPUs start (auto: when the job "
                         "has 8 GPUs)")
    ap.add_argument("--cpu-configs-budget", type=float, default=240.0,
                    help="seconds those reference cells may take in all; a cell past it is recorded as skipped")
    return ap.parse_args()


# ---------------------------------------------------------------- watchdog (rank processes)
PHASE = ["start"]
PHASE_LOG = []          # (phase, monotonic start) in order: phase_wall_s in the N > 1 line


def phase(name):
    PHASE[0] = name
    PHASE_LOG.append((name, time.monotonic()))


HEARTBEAT_S = 45.0      # rank 0 names its phase on stderr this often: a long quiet phase (the reference
                        # at the BASELINE cells runs minutes without output) is not taken for a hang


def start_heartbeat(seconds=HEARTBEAT_S):
    """a daemon thread printing `bench: <phase> (<s> s in it, <s> s in all)` to stderr every `seconds`
    -> an Event that stops it"""
    t_start = time.monotonic()
    stop = threading.Event()

    def beat():
        while not stop.wait(seconds):
            now = time.monotonic()
            t_phase = PHASE_LOG[-1][1] if PHASE_LOG else t_start
            sys.stderr.write("bench: %s (%.0f s in it, %.0f s in all)\n" % (PHASE[0], now - t_phase, now - t_start))
            sys.stderr.flush()

    threading.Thread(target=beat, name="bench-heartbeat", daemon=True).start()
    return stop


def phase_walls():
    """seconds spent in each phase so far (a phase entered several times: summed)"""
    out = {}
    marks = PHASE_LOG + [("", time.monotonic())]
    for (name, t0), (_n, t1) in zip(marks, marks[1:]):
        key = re.sub(r"^method \d+: ", "methods: ", name)
        key = re.sub(r"^BASELINE configs: .*", "BASELINE configs", key)
        out[key] = round(out.get(key, 0.0) + (t1 - t0), 2)
    return out


class Watchdog:
    """A rank whose peers died (or never came) waits in RCCL with no timeout of its own: once armed,
    after `seconds` it names the phase the rank is in and ends the process (os._exit: no exec,
    nothing else runs in its place).  It guards the road to the measured value only: main() re-arms
    it at the communicator init and cancels it once `value` is known -- every phase after that has
    a LineGuard of its own, which prints the measured line instead of a null one."""

    def __init__(self, rank):
        self.rank, self.timer, self.seconds = rank, None, 0

    def _fire(self):
        try:
            sys.stderr.write("bench: rank %d still in phase '%s' after %.0f s; exiting\n"
                             % (self.rank, PHASE[0], self.seconds))
            sys.stderr.flush()
            if self.rank == 0:     # no value was measured: say where it stopped
                line = {"metric": METRIC, "value": None, "unit": "GB/s", "higher_is_better": True,
                        "error": "rank 0 still in phase '%s' after %.0f s" % (PHASE[0], self.seconds)}
                tails = rccl_log_tails()
                if tails:
                    line["rccl_log_tail"] = tails
                print(json.dumps(line), flush=True)
        finally:
            os._exit(124)

    def arm(self, seconds):
        self.cancel()
        self.seconds = seconds
        if seconds > 0:
            self.timer = threading.Timer(seconds, self._fire)
            self.timer.daemon = True
            self.timer.start()

    def cancel(self):
        if self.timer:
            self.timer.cancel()
            self.timer = None


def start_watchdog(seconds, rank):
    """a Watchdog armed for `seconds` (0: off)"""
    w = Watchdog(rank)
    w.arm(seconds)
    return w


GUARD_GRACE = 20.0      # a LineGuard fires this long after its phase's own budget
CPU_GRACE = 10.0        # rank 0's reference cells stop at their budget (run_reference kills the mpiexec
                        # session); the other ranks allow this much more for the last kill + the id file


def pre_value_allowance(a, rank, world, parent):
    """seconds a rank may legitimately wait before its communicator exists: under a launcher (no
    parent process) rank 0 runs the reference's CPU phases first and writes the RCCL id only after
    them, so every rank allows their budgets"""
    if parent or a.no_cpu_baseline or world == 1:
        return 0.0
    return a.cpu_budget + (a.cpu_configs_budget + CPU_GRACE if cpu_configs_on(a, world) else 0.0)


def wall_bound(a, world, parent=False):
    """the longest a rank process can run (seconds) with every phase at its budget and every guard
    firing: pre-communicator CPU phases, the watchdog up to the value, then the LineGuarded xGMI and
    BASELINE-configs phases -- INTEGRATION.md states this bound for the driver's 8-GPU run"""
    pre = pre_value_allowance(a, 0, world, parent) if not parent else 0.0
    post = 0.0
    if world > 1:
        post += a.xgmi_budget
    if a.baseline_configs == "on" or (a.baseline_configs == "auto" and world == 8):
        post += a.baseline_budget + GUARD_GRACE
    return pre + a.watchdog + post


def dumps_live(out):
    """json.dumps of a line another thread may still be adding to (a dict that changes size while
    it is serialised raises RuntimeError): retried a few times, then a copy made key by key"""
    for _ in range(20):
        try:
            return json.dumps(out)
        except RuntimeError:
            time.sleep(0.005)
    return json.dumps({k: out.get(k) for k in list(out)}, default=str)


class LineGuard:
    """Once the line's value is measured it must come out: a phase run under this guard that is
    still going `seconds` after it started (a peer lost inside RCCL waits forever) has
    note(message) record why in `out`, rank 0 print `out` as it stands, and the process end
    (os._exit(0): the measured line is the result; nothing else runs in the process's place)."""

    def __init__(self, out, rank, seconds, note):
        self.out, self.rank, self.seconds, self.note = out, rank, seconds, note
        self.timer = None

    def _fire(self):
        try:
            self.note("still in phase '%s' %.0f s after it started; line printed from what was measured"
                      % (PHASE[0], self.seconds))
            if self.rank == 0:
                finish_line(self.out, self.out.get("n_gpus") or 2)
                print(dumps_live(self.out), flush=True)
        finally:                 # whatever happened above, the process ends
            os._exit(0)

    def __enter__(self):
        if self.seconds > 0:
            self.timer = threading.Timer(self.seconds, self._fire)
            self.timer.daemon = True
            self.timer.start()
        return self

    def __exit__(self, *exc):
        if self.timer:
            self.timer.cancel()
        return False


# ---------------------------------------------------------------- CPU baseline (reference)
def host_cpus():
    """CPUs this process may actually use: affinity mask, capped by a cgroup v2 CPU quota
    (cpu.max), which os.cpu_count() does not see -- (cpus, how it was found)"""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    how = "%d in the affinity mask" % n
    quota = period = None
    try:                                               # cgroup v2
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
    except (OSError, ValueError):
        try:                                           # cgroup v1
            quota = open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read().strip()
            period = open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()
        except OSError:
            pass
    try:
        if quota not in (None, "max", "-1") and int(period) > 0:
            q = max(1, int(int(quota) / int(period)))
            if q < n:
                n, how = q, "cgroup CPU quota %s/%s of %d in the affinity mask" % (quota, period, n)
    except ValueError:
        pass
    return n, how


def reference_cpus(pin):
    """CPUs to pin the reference's MPI processes to, or None (not pinned).  pin: the first `quota` CPUs
    of the mask when a cgroup CPU quota sits below the affinity mask (a one-GPU box: 16 CPUs of quota
    over 256 in the mask).  Measured on those boxes, the two settings suit different runs:
      * configs[1]'s 32 ranks (cpu_baseline) run 5-10x FASTER unpinned -- 0.2-0.6 s per method
        (9.2-18 GB/s, BENCH_r05.json, profiles/r06/unpinned/) against 3.1-3.8 s pinned (1.3-1.5 GB/s,
        profiles/r06/torchrun8*/): 32 busy-polling ranks time-slicing 16 CPUs wait out each other's
        slices, while unpinned they run together until the quota throttles them;
      * the 256-rank BASELINE cells (cpu_baseline_configs) take 48-61 s of wall each unpinned, almost
        all of it MPI start-up under the quota, against 2-16 s pinned, for max total times within
        +-30 % of each other (profiles/r06/torchrun8d/ against torchrun8c/): pinned, every 8-GPU
        method gets its cell inside the budget.
    XG_REF_PIN=1 / 0 forces either for both."""
    env = os.environ.get("XG_REF_PIN")
    if env in ("0", "1"):
        pin = env == "1"
    if not pin or not hasattr(os, "sched_getaffinity"):
        return None
    n, _how = host_cpus()
    mask = sorted(os.sched_getaffinity(0))
    return mask[:n] if n < len(mask) else None


def run_reference(args, timeout, cpus=None):
    """one mpiexec of the reference ./test (oracle/_ref/test) in a session of its own, so a run past
    `timeout` ends with every one of its processes (its exact process group) -- busy-polling MPI
    ranks left behind would share the host with everything after.  cpus: the CPU set its processes
    inherit (reference_cpus).  -> (max total time or None, wall seconds, error text)"""
    import signal
    ref = os.path.join(REPO, "oracle", "_ref", "test")
    mpiexec = shutil.which("mpiexec") or "/opt/conda/bin/mpiexec"
    if not (os.path.exists(ref) and os.path.exists(mpiexec)):
        return None, 0.0, "no reference build (oracle/_ref/test) or mpiexec on this host"
    t0 = time.time()
    old = None
    if cpus:                       # the child inherits this thread's affinity at fork
        old = os.sched_getaffinity(0)
        os.sched_setaffinity(0, cpus)
    try:
        p = subprocess.Popen([mpiexec, "-launcher", "fork"] + args[:2] + [ref] + args[2:], stdout=subprocess.PIPE,
                             stderr=subprocess.PIPE, text=True, cwd="/tmp", start_new_session=True)
    finally:
        if old is not None:
            os.sched_setaffinity(0, old)
    try:
        out, err = p.communicate(timeout=max(1.0, timeout))
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return None, time.time() - t0, "over budget: stopped after %.0f s" % (time.time() - t0)
    mt = re.findall(r"max total time = ([0-9.]+)", out)
    if p.returncode != 0 or not mt:
        return None, time.time() - t0, "reference run failed (exit %d): %s" % (p.returncode, err[-200:])
    return float(mt[0]), time.time() - t0, ""


def pinned_text(cpus):
    return ("pinned to the %d CPUs %d-%d of the affinity mask (the cgroup quota's worth)" % (len(cpus), cpus[0], cpus[-1])
            if cpus else "not pinned")


def cpu_baseline(a, methods):
    """The reference ./test (oracle/_ref/test, built from /root/reference by oracle/Makefile)
    under MPICH on this box's host cores, same P/A/d/methods, bounded -k, --cpu-budget s in all."""
    if not os.path.exists(os.path.join(REPO, "oracle", "_ref", "test")):
        return cpu_baseline_port(a, methods)
    tot_bytes, tot_time, per = 0.0, 0.0, {}
    cpus = reference_cpus(pin=False)      # configs[1]: faster unpinned
    t0 = time.time()
    for m in methods:
        args = ["-n", str(a.procs), "-a", str(a.aggs), "-p", "1", "-d", str(a.size), "-m", str(m), "-i", "1",
                "-k", str(a.cpu_reps)]
        if a.comm_size != 200000000:
            args += ["-c", str(a.comm_size)]
        mt, _wall, err = run_reference(args, a.cpu_budget - (time.time() - t0), cpus)
        if err.startswith("over budget"):
            return {"value": None, "unit": "GB/s", "cores": a.procs, "kind": "reference",
                    "sample": "method %d %s (--cpu-budget %.0f s)" % (m, err, a.cpu_budget)}
        if mt is None:
            return cpu_baseline_port(a, methods, note=err)
        per[m] = mt
        tot_time += mt
        tot_bytes += float(a.procs) * a.aggs * a.size * a.cpu_reps
    ncpu, how = host_cpus()
    return {"value": round(tot_bytes / tot_time / 1e9, 4), "unit": "GB/s", "cores": min(a.procs, ncpu),
            "kind": "reference",
            "sample": "reference ./test via MPICH 3.3.2 ch3:nemesis, mpiexec -n %d (one process per logical "
                      "rank) on %d usable host CPUs (%s; %s)%s, -a %d -d %d -k %d, methods %s, aggregate = "
                      "sum(P*A*d*k) / sum(max total time); %.1f s wall"
                      % (a.procs, ncpu, how, pinned_text(cpus),
                         ", oversubscribed: MPICH busy-polls" if a.procs > ncpu else "",
                         a.aggs, a.size, a.cpu_reps, ",".join(map(str, methods)), time.time() - t0),
            "max_total_time_s": per}


# (cell key, P, A, d, -c, method): BASELINE.json's 8-GPU configurations at sizes the host runs --
# configs[2] at its stated size, configs[3]'s and configs[4]'s P256 shapes at -d 4 KiB (64 MiB would be
# 1 TiB per direction in host RAM); the same keys as the GPU cells at the same -d in
# baseline_configs_8gpu, so the two sit side by side.  A P256 cell on a 16-CPU host costs ~6 s of MPI
# start-up and tear-down whatever its -d, and its exchange is latency-bound (256 busy-polling ranks
# time-slicing: the pairwise m9 / m10 post 256 Sendrecv rounds each), so -d 4 KiB is the size at
# which a cell costs what its schedule costs.  Order: every direction and schedule once --
# alltoallw, a2m, m2a, half-sync a2m / m2a, pairwise, then the rest -- before any -c repeats, so a
# budget that runs out still leaves every kind of schedule measured.
def _c3(m):
    return ("configs[3] at -d 4 KiB m%d" % m, 256, 32, 4 << 10, 200000000, m)


def _c4(c, m):
    return ("configs[4] -c %d at -d 4 KiB m%d" % (c, m), 256, 64, 4 << 10, c, m)


def _c2(m):
    return ("configs[2] m%d" % m, 64, 16, 256 << 10, 200000000, m)


CPU_CELLS = [_c2(5), _c3(1), _c3(2), _c4(8, 7), _c4(8, 11), _c3(9), _c2(8), _c4(8, 12), _c3(10),
             _c4(1, 7), _c4(1, 12), _c4(1, 11)]    # the -c 1 repeats shortest first (m11's ~25 s last)


def cell_cap(a):
    """seconds one reference cell may take: a share of the budget, so one slow cell (a pairwise
    schedule on few CPUs) cannot leave the cells after it unmeasured"""
    return round(max(20.0, 0.3 * a.cpu_configs_budget), 1)


def cpu_configs_on(a, world):
    return a.cpu_configs == "on" or (a.cpu_configs == "auto" and world == 8)


def cpu_baseline_configs(a, cells=CPU_CELLS):
    """The reference itself under mpiexec at BASELINE.json's 8-GPU configurations (CPU_CELLS), one
    process per logical rank on this box's host cores, --cpu-configs-budget seconds in all: a cell
    that would start past it, or runs past it, is recorded as skipped.  Run before any process
    touches a GPU (the parent of an N-GPU job, or rank 0 under a launcher)."""
    ncpu, how = host_cpus()
    cpus = reference_cpus(pin=True)       # 256 ranks: start-up fits the budget pinned
    cap = cell_cap(a)
    t0 = time.time()
    res = {"budget_s": a.cpu_configs_budget, "cell_cap_s": cap, "cores": ncpu, "cores_how": how,
           "pinning": pinned_text(cpus), "kind": "reference",
           "launch": "mpiexec -launcher fork -n P oracle/_ref/test -a A -p 1 -d D -m M -i 1 -k 1 [-c C] "
                     "(MPICH 3.3.2 ch3:nemesis, busy-polling ranks)", "cells": {}}
    for key, P, A, d, c, m in cells:
        left = a.cpu_configs_budget - (time.time() - t0)
        if left <= 1:
            res["cells"][key] = "skipped: budget of %.0f s spent" % a.cpu_configs_budget
            continue
        args = ["-n", str(P), "-a", str(A), "-p", "1", "-d", str(d), "-m", str(m), "-i", "1", "-k", "1"]
        if c != 200000000:
            args += ["-c", str(c)]
        mt, wall, err = run_reference(args, min(left, cap), cpus)
        if mt is None:
            res["cells"][key] = ("skipped: " if err.startswith("over budget") else "failed: ") + err
            continue
        res["cells"][key] = {"P": P, "A": A, "d": d, "c": c, "max_total_time_s": mt,
                             "GBps_delivered": round(P * A * d / mt / 1e9, 4) if mt > 0 else None,
                             "wall_s": round(wall, 1), "oversubscription": round(P / max(1, ncpu), 1)}
    res["spent_s"] = round(time.time() - t0, 1)
    return res


def side_by_side(out):
    """the reference's max total time beside the GPU job's at the same cell (same P, A, d, -c,
    method): {cell: {"gpu_max_total_time_s", "reference_max_total_time_s", "speedup"}}"""
    cpu = ((out.get("cpu_baseline_configs") or {}).get("cells")) or {}
    gpu = ((out.get("baseline_configs_8gpu") or {}).get("cells")) or {}
    rows = {}
    for key, c in cpu.items():
        g = gpu.get(key)
        if isinstance(c, dict) and isinstance(g, dict) and g.get("max_total_time_s"):
            rows[key] = {"gpu_max_total_time_s": g["max_total_time_s"],
                         "reference_max_total_time_s": c["max_total_time_s"],
                         "speedup": round(c["max_total_time_s"] / g["max_total_time_s"], 1)}
    return rows or None


def cpu_baseline_port(a, methods, note=""):
    """Fallback: the oracle's numpy restatement (single core), one repetition per method."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import xg_oracle as O   # checker, timed as the CPU port only
    rl = O.aggregator_list(a.procs, a.aggs)
    t_tot, b_tot = 0.0, 0.0
    for m in methods:
        progs = O.programs(m, a.procs, a.aggs, a.size, a.comm_size, rl, 1)
        t0 = time.time()
        O.execute(m, a.procs, a.aggs, a.size, rl, progs, 0)
        t_tot += time.time() - t0
        b_tot += float(a.procs) * a.aggs * a.size
    return {"value": round(b_tot / t_tot / 1e9, 4), "unit": "GB/s", "cores": 1, "kind": "port",
            "sample": "oracle numpy restatement, 1 repetition of methods %s (fill + matched copies). %s"
                      % (",".join(map(str, methods)), note)}


# ---------------------------------------------------------------- xGMI latency / bandwidth floor (N > 1)
SWEEP_SIZES = (4096, 65536, 1 << 20, 16 << 20)


def p2p_sweep(ctx, world, error=RuntimeError):
    """The pt2pt_test analogue (mpi_sendrecv_test.c:15-74) as RCCL p2p over xGMI, a few
    seconds at most: per message size, one direction 1 -> 0 (xg_p2p_bench mode 2: latency
    of one send/recv pair, what a latency-bound step pays per cross-GPU message) and all
    pairs at once (mode 0: every GPU sends `bytes` to each of its N-1 peers).  Every rank
    runs every case (the calls are collective); the figures are MAX time / MIN rate over
    the GPUs taking part.  -> (rows, None) or, when a case fails on some GPU (`error`
    raised), (the rows before it, the error): every rank stops at the same case."""
    out = []
    for nbytes in SWEEP_SIZES:
        reps = 50 if nbytes <= 65536 else (20 if nbytes <= 1 << 20 else 5)
        for mode, name in ((2, "one_way_1_to_0"), (0, "all_pairs")):
            msg = None
            try:
                gbps, sec = ctx.p2p_bench(nbytes, mode=mode, reps=reps)
            except error as e:
                gbps, sec, msg = 0.0, 0.0, str(e)
            part = mode == 0 or ctx.rank < 2          # mode 2 moves bytes between GPUs 1 and 0 only
            t_max, neg_rate, err = ctx.allreduce_max([sec if part else 0.0, -gbps if part else -1e30,
                                                      1.0 if msg else 0.0])
            if err:
                return out, "%s %d B: %s" % (name, nbytes, msg or "failed on another GPU")
            row = {"mode": name, "bytes": nbytes, "reps": reps, "us_per_rep": round(t_max * 1e6, 2)}
            if mode == 2:
                row["GBps"] = round(-neg_rate, 2)
            else:
                row["GBps_per_gpu_egress_min"] = round(-neg_rate, 2)
                row["GBps_aggregate"] = round(-neg_rate * world, 2)
            out.append(row)
    return out, None


def pair_rounds(n):
    """a 1-factorisation of the n ranks (circle method; odd n: one rank idle per round): round k
    -> partner[r] (-1: idle).  Every pair meets exactly once in n - 1 (n odd: n) rounds."""
    m = n + (n % 2)
    rounds = []
    for k in range(m - 1):
        partner = [-1] * n
        ring = [m - 1] + [(k + i) % (m - 1) for i in range(m - 1)]
        for i in range(m // 2):
            x, y = ring[i], ring[m - 1 - i]
            if x < n and y < n:
                partner[x], partner[y] = y, x
        rounds.append(partner)
    return rounds


def link_sweep(ctx, world, nbytes=16 << 20, reps=5, error=RuntimeError):
    """per-link rates: in each round of a 1-factorisation every rank exchanges `nbytes` each way
    with its partner (xg_p2p_pair_bench), all pairs of the round at once -- every link of the node
    measured under its neighbours' load; a min / max spread shows link asymmetry.  -> (result,
    error or None): every rank stops at the same round on an error (its flag is MAX-reduced)."""
    rates = [[None] * world for _ in range(world)]
    res = {"bytes": nbytes, "reps": reps, "rounds": 0, "GBps": rates}
    for partner in pair_rounds(world):
        ctx.barrier()
        msg = None
        try:
            gbps, _sec = ctx.p2p_pair_bench(nbytes, partner[ctx.rank], reps)
        except error as e:
            gbps, msg = 0.0, str(e)
        row = [0.0] * (world * world) + [1.0 if msg else 0.0]
        if partner[ctx.rank] >= 0:
            row[ctx.rank * world + partner[ctx.rank]] = gbps
        got = ctx.allreduce_max(row)
        if got[-1]:
            return res, "round %d: %s" % (res["rounds"], msg or "failed on another GPU")
        for r in range(world):
            if partner[r] >= 0:
                rates[r][partner[r]] = round(got[r * world + partner[r]], 2)
        res["rounds"] += 1
    vals = [v for row in rates for v in row if v is not None]
    if vals:
        res.update(min=min(vals), max=max(vals), spread=round(max(vals) / min(vals), 3) if min(vals) > 0 else None)
    return res, None


def link_bytes(xg, s, world, pack, form):
    """the plan's link traffic from the calls each GPU posts in this form (xg_devplan_step_calls) ->
    (busiest, total): busiest = per step and per RCCL group of it, the most loaded directed GPU link's
    bytes, summed over the run -- what the exchange costs at one link rate however fast the rest of
    the node is (profiles/link_load.py); total = every cross-GPU send's bytes (a relayed byte crosses
    two links and counts twice: the traffic the links carried, beside the logical payload)"""
    views = [s.devplan(world, g, pack, 0, form) for g in range(world)]
    busiest = total = 0
    for st in range(views[0].nsteps):
        per = {}                                  # (group, src GPU, dst GPU) -> bytes
        for g, v in enumerate(views):
            grp = 0
            for kind, peer, _buf, _off, ln in v.calls(st):
                if kind == xg.CALL_FENCE:
                    grp += 1
                elif kind == xg.CALL_SEND and peer != g:
                    per[(grp, g, peer)] = per.get((grp, g, peer), 0) + ln
                    total += ln
        for q in {k[0] for k in per}:
            busiest += max(b for k, b in per.items() if k[0] == q)
    return busiest, total


CALL_COST_BYTES = (1 << 20, 16 << 20)


def call_cost(ctx, world, reps=10, error=RuntimeError):
    """RCCL's cost per call inside a group on this node's links: all pairs at once, every transfer of
    `bytes` posted as 1 call and as `world` calls (xg_p2p_split_bench) -- a relayed message is cut into
    G pieces, so a relayed step posts about G x the calls of direct.  MAX time
    over the GPUs.  -> (result, error or None): every rank stops at the same case on an error."""
    res = {"reps": reps, "rows": []}
    for nbytes in CALL_COST_BYTES:
        t = {}
        for calls in (1, world):
            msg = None
            try:
                _g, sec = ctx.p2p_split_bench(nbytes, calls, reps)
            except error as e:
                sec, msg = 0.0, str(e)
            t_max, err = ctx.allreduce_max([sec, 1.0 if msg else 0.0])
            if err:
                return res, "%d B x %d calls: %s" % (nbytes, calls, msg or "failed on another GPU")
            t[calls] = t_max
            res["rows"].append({"bytes": nbytes, "calls_per_peer": calls, "us_per_rep": round(t_max * 1e6, 2)})
        # per extra send + receive pair: every rank posts (calls - 1) x (world - 1) more of each
        res.setdefault("us_per_extra_call", {})[str(nbytes)] = round(
            (t[world] - t[1]) * 1e6 / max(1, (world - 1) * (world - 1)), 3)
    return res, None


def busiest_link_bytes(xg, s, world, pack, form):
    """link_bytes' busiest-link figure"""
    return link_bytes(xg, s, world, pack, form)[0]


FORM_REPS = 3           # timed runs per plan form wherever forms are compared (median / min / max)
CHOICE_RULE = ("%d timed runs per form; direct is kept unless a form's median beats direct's by more than the "
               "spread (max - min) of either; ms_per_run = the chosen form's median" % FORM_REPS)


def choose_form(samples, default="direct"):
    """The form choice of a BASELINE cell or of a method of the N > 1 line.  samples: {form: [seconds
    of each timed run]} of the forms that verified.  `default` (direct: no staging, no second group)
    is kept unless another form's MEDIAN beats it by more than the spread (max - min) of either form's
    runs; among the forms that do, the lowest median wins.  Without the default, the lowest median.
    -> (chosen, {form: {"median_ms", "min_ms", "max_ms"}}, margin): margin = (the best other median -
    the chosen median) / the chosen median -- negative when a faster median was within the spread."""
    st = {f: (statistics.median(v), min(v), max(v)) for f, v in samples.items() if v}
    if not st:
        return None, {}, None
    if default in st:
        dm, dlo, dhi = st[default]
        win = [f for f, (m, lo, hi) in st.items() if f != default and dm - m > max(dhi - dlo, hi - lo)]
        chosen = min(win, key=lambda f: st[f][0]) if win else default
    else:
        chosen = min(st, key=lambda f: st[f][0])
    stats = {f: {"median_ms": round(m * 1e3, 4), "min_ms": round(lo * 1e3, 4), "max_ms": round(hi * 1e3, 4)}
             for f, (m, lo, hi) in st.items()}
    others = [st[f][0] for f in st if f != chosen]
    cm = st[chosen][0]
    margin = round((min(others) - cm) / cm, 4) if others and cm > 0 else None
    return chosen, stats, margin


def link_rate(out):
    """the median per-link rate (GB/s, one direction) of the per-link sweep, or None"""
    links = ((out.get("xgmi") or {}).get("links")) or {}
    vals = sorted(v for row in links.get("GBps") or [] for v in row if v)
    return vals[len(vals) // 2] if vals else None


# ---------------------------------------------------------------- BASELINE.json's 8-GPU configurations
# (name, P, A, d, -c, methods): configs[2], configs[3], configs[4] at their stated sizes, and
# configs[3] / [4] at the reduced -d (4 KiB) the reference runs at on the host (CPU_CELLS: the same keys),
# ahead of configs[4]'s stated-size cells, which take most of the phase's budget
BASELINE_CELLS = ([  # first a link-level probe of two-hop routing: one rank per GPU, pairwise m9, so every XOR
                   # round is a permutation of 16 MiB messages on one link each direct, on every link
                   # relayed (busiest-link bytes 112 -> 28 MiB); not a BASELINE config, ~1 s
                   ("two-hop probe P8 A8 -d 16 MiB", 8, 8, 16 << 20, 200000000, (9,)),
                   ("configs[2]", 64, 16, 256 << 10, 200000000, (5, 8)),
                   ("configs[3]", 256, 32, 4 << 20, 200000000, (1, 2, 9, 10)),
                   ("configs[3] at -d 4 KiB", 256, 32, 4 << 10, 200000000, (1, 2, 9, 10))] +
                  [("configs[4] -c %d at -d 4 KiB" % c, 256, 64, 4 << 10, c, (7, 11, 12)) for c in (1, 8)] +
                  # the sweep's ends first: a budget that runs out mid-sweep still leaves -c 1 and 8
                  [("configs[4] -c %d" % c, 256, 64, 64 << 20, c, (7, 11, 12)) for c in (1, 8, 2, 3, 4, 5, 6, 7)])


# the cross-GPU plan forms a BASELINE cell is timed in (pack_max_seg, pack_form), direct first: the
# others only where they change the plan
CELL_FORMS = (("direct", (0, -1)), ("packed_one_sided", (4 << 20, 1)), ("packed_two_sided", (4 << 20, 0)),
              ("relay", (0, 2)), ("relay_coalesced", (0, 3)))
# region tiers of a configuration, largest first: when its regions cannot hold every form's staging
# the forms of the next tier run (on every GPU alike), down to direct alone (no staging at all)
CELL_TIERS = (tuple(f for f, _ in CELL_FORMS), tuple(f for f, _ in CELL_FORMS if f != "relay_coalesced"),
              ("direct",))


def plan_signature(v):
    """what a GPU's plan makes the device do, up to order inside a launch or an RCCL group and where
    staged bytes sit in STAGE_SEND / STAGE_RECV: per step its stage / pre / post copies and the calls
    of each group, as sorted lists (staging offsets left out).  Two forms with one signature on every
    GPU are one plan to time."""
    def cp(c):
        return tuple(x if not (k in (1, 3) and c[k - 1] in (2, 3)) else -1 for k, x in enumerate(c))
    out = []
    for st in range(v.nsteps):
        pb, pc, _qb, _qc, ob, oc = v.steps[st]
        groups, cur = [], []
        for kind, peer, buf, off, ln in v.calls(st):
            if kind in (1, 2):
                cur.append((kind, peer, buf, -1 if buf in (2, 3) else off, ln))
            else:
                groups.append(sorted(cur))
                cur = [(kind, -1, -1, -1, 0)]
        groups.append(sorted(cur))
        out.append((sorted(map(cp, v.copies[pb:pb + pc])), sorted(map(cp, v.copies[ob:ob + oc])), groups))
    return out


def cell_estimate_s(links, link_gbps):
    """seconds a BASELINE cell's runs take at least: every form's verified run + FORM_REPS timed runs,
    each its busiest-link bytes at the per-link rate (0 when no rate was measured)"""
    if not link_gbps:
        return 0.0
    return sum((1 + FORM_REPS) * busiest / (link_gbps * 1e9) for busiest, _total in links.values())


def baseline_configs_phase(xg, ctx, world, rank, budget, result, cells=BASELINE_CELLS, link_gbps=None):
    """Every method of BASELINE.json's 8-GPU configurations on this job: per (config, method) one
    verified run (every slot checked on its GPU, bad slots MAX-reduced), FORM_REPS timed runs (device
    time, MAX over GPUs; the median is the figure), delivered, cross-GPU (logical payload) and on-link
    (what the form's calls put on the links) GB/s and the reference's max total time.
    Beside each: the plan's link bound -- its busiest-link bytes (busiest_link_bytes) at the per-link
    sweep's median rate (`link_gbps`) -- and the fraction of it the run reached.
    Every cross-GPU form that changes the cell's plan -- packed one-sided / two-sided (lists of
    segments <= 4 MiB) and the two relay forms (XG_RELAY, XG_RELAY_COALESCED: configs[3]'s pairwise
    m9 / m10, whose XOR rounds put each GPU on one link; configs[4]'s m11 / m12) -- is verified and
    timed beside the direct
    form; choose_form keeps direct unless another form's median beats it by more than the spread
    ("forms": each form's median / min / max, "chosen", "margin").  Collective throughout: every rank takes the same cells
    in the same order, and every decision (budget spent, a plan or allocation that failed on some
    GPU) is MAX-reduced first, so all ranks skip alike.  Fills result["cells"] as it goes (a
    watchdog may print it half done)."""
    t0 = time.time()
    result["cells"] = cells_out = {}
    regions = {}                      # (P, A, d) -> Regions shared by that configuration's cells
    tier_of = {}                      # (P, A, d) -> the CELL_TIERS index its regions hold
    no_room = set()                   # (P, A, d) whose regions could not be allocated on some GPU
    needs = {}                        # (P, A, d, c) -> region bytes of every method and form on this GPU

    def measure(s, P, A, d, c, form, reg, links):
        """one verified run of a plan form, then FORM_REPS timed runs (device time, MAX over GPUs) ->
        (figures, per-run seconds, None) or (None, None, why).  links: link_bytes of the form (rank 0)"""
        run, err = None, ""
        try:
            run = xg.MethodRun(ctx, s, it=0, mode=0, regions=reg, pack_max_seg=form[0], pack_form=form[1])
        except xg.XGError as e:
            err = str(e)
        if ctx.allreduce_max([1.0 if err else 0.0])[0]:
            if run is not None:
                run.close()
            return None, None, "failed: %s" % (err or "on another GPU")
        runs_s = []
        try:
            ctx.barrier()
            done, post, _wall = run.run_timed()
            lo, hi = s.block_range(world, rank)
            tmax = max(s.rank_timer(q, done, post, world).total_time for q in range(lo, hi)) if hi > lo else 0.0
            _chk, bad, _first = run.verify()
            tmax, nbad = ctx.allreduce_max([tmax, float(sum(1 for b in bad if b))])
            for _ in range(FORM_REPS if nbad == 0 else 0):
                ctx.barrier()
                ctx.device_sync()
                t1 = time.perf_counter()
                run.enqueue()
                ctx.device_sync()
                run.check()
                runs_s.append(ctx.allreduce_max([time.perf_counter() - t1])[0])
        finally:
            run.close()
        t_run = statistics.median(runs_s) if runs_s else 0.0
        cross = sum(s.devplan(world, g).remote_send_bytes for g in range(world))
        # (rank 0 prints the line; the other ranks skip the host-side plan walk)
        busiest, on_links = links if rank == 0 else (0, 0)
        fig = {"P": P, "A": A, "d": d, "c": c, "ms_per_run": round(t_run * 1e3, 4),
               "runs_ms": [round(x * 1e3, 4) for x in runs_s],
               "GBps_delivered": round(P * A * d / t_run / 1e9, 2) if t_run > 0 else None,
               "GBps_cross_gpu": round(cross / t_run / 1e9, 2) if t_run > 0 else None, "cross_gpu_bytes": int(cross),
               "link_bytes": int(on_links) if rank == 0 else None,
               "GBps_link": round(on_links / t_run / 1e9, 2) if rank == 0 and t_run > 0 else None,
               "busiest_link_bytes": int(busiest) if rank == 0 else None,
               "max_total_time_s": tmax, "verified": nbad == 0, "bad_slots_max_gpu": int(nbad)}
        if link_gbps and busiest and t_run > 0:
            bound_ms = busiest / (link_gbps * 1e9) * 1e3
            fig["link_bound_ms"] = round(bound_ms, 4)
            fig["link_bound_frac"] = round(bound_ms / (t_run * 1e3), 4)
        return fig, runs_s, None

    try:
        for name, P, A, d, c, methods in cells:
            rl = xg.aggregator_list(P, A)
            for m in methods:
                key = "%s m%d" % (name, m)
                phase("BASELINE configs: %s" % key)
                if ctx.allreduce_max([time.time() - t0])[0] > budget:
                    cells_out[key] = "skipped: phase budget of %.0f s spent" % budget
                    continue
                if (P, A, d) in no_room:
                    cells_out[key] = "skipped: this configuration's regions did not fit"
                    continue
                nf = len(CELL_FORMS) - 1
                err, no_alloc, differs, new_plan = "", False, [0.0] * nf, [0.0] * nf
                try:
                    s = xg.Schedule(m, P, A, d, c, rl, ntimes=1)
                    # which forms change this GPU's plan (packing: lists of small segments; relay: a
                    # permutation step with lists >= 1 MiB), and which of those are a plan no form
                    # before them has (the coalesced form at configs[4]'s 64 MiB segments is the
                    # relay form's plan); MAX-reduced below, so all GPUs agree
                    v0 = s.devplan(world, rank, 0, 0, -1)
                    seen = [plan_signature(v0)]
                    for i, (_fname, f) in enumerate(CELL_FORMS[1:]):
                        plan = plan_signature(s.devplan(world, rank, f[0], 0, f[1]))
                        differs[i] = 1.0 if plan != seen[0] else 0.0
                        new_plan[i] = 1.0 if plan not in seen else 0.0
                        seen.append(plan)
                    if (P, A, d, c) not in needs:   # one allocation per configuration: all its methods, all forms
                        tiers = [[0] * xg.NBUF for _ in CELL_TIERS]
                        for mm in methods:
                            sm = xg.Schedule(mm, P, A, d, c, rl, ntimes=1)
                            for fname, f in CELL_FORMS:
                                v = sm.devplan(world, rank, f[0], 0, f[1])
                                for k, names in enumerate(CELL_TIERS):
                                    if fname in names:
                                        tiers[k] = [max(x, y) for x, y in zip(tiers[k], v.region_bytes)]
                        needs[(P, A, d, c)] = tiers
                    tiers = needs[(P, A, d, c)]
                    rk = (P, A, d)
                    if rk not in regions or not regions[rk].fits(tiers[tier_of[rk]]):
                        # a new configuration, or one whose -c needs more staging than the cells
                        # before it (configs[4] at -d 4 KiB: -c 8 after -c 1): regions sized for both
                        if rk in regions:
                            tiers = [[max(x, y) for x, y in zip(tb, regions[rk].bytes)] for tb in tiers]
                        for old in regions.values():
                            old.close()
                        regions.clear()
                        tier_of.pop(rk, None)
                        no_alloc = True
                        for k, tb in enumerate(tiers):
                            # the coalesced relay form's staging (up to 5.5 GiB beside configs[4]'s
                            # 256 GiB, tests/test_hbm_fit.py), then the other forms', may not fit
                            try:
                                regions[rk] = xg.Regions(ctx, tb)
                                tier_of[rk] = k
                                break
                            except xg.XGError:
                                if k == len(tiers) - 1:
                                    raise
                        no_alloc = False
                except xg.XGError as e:
                    err = str(e)
                failed, unplaced, tier, *flags = ctx.allreduce_max(
                    [1.0 if err else 0.0, 1.0 if no_alloc else 0.0, float(tier_of.get((P, A, d), 0))] + differs +
                    new_plan)
                differs, new_plan = flags[:nf], flags[nf:]
                if failed:
                    cells_out[key] = "failed: %s" % (err or "on another GPU")
                    if unplaced:      # some GPU never got this configuration's regions: the rest would fail alike
                        no_room.add((P, A, d))
                    continue
                held = CELL_TIERS[int(tier)]
                forms = dict(CELL_FORMS[:1])
                forms.update((fname, f) for (fname, f), dif, nw in zip(CELL_FORMS[1:], differs, new_plan)
                             if dif and nw and fname in held)
                same = [fname for (fname, _f), dif, nw in zip(CELL_FORMS[1:], differs, new_plan) if dif and not nw]
                dropped = [fname for (fname, _f), dif in zip(CELL_FORMS[1:], differs) if dif and fname not in held]
                # the cell's runs at the measured link rate: a cell that would still be running when the
                # phase's guard fires is skipped on every GPU alike (the cells after it may be shorter)
                links = {f: link_bytes(xg, s, world, form[0], form[1]) if rank == 0 else (0, 0)
                         for f, form in forms.items()}
                est = cell_estimate_s(links, link_gbps) if rank == 0 else 0.0
                est, spent = ctx.allreduce_max([est, time.time() - t0])
                if spent + est > budget + GUARD_GRACE / 2:
                    cells_out[key] = ("skipped: %.0f s of runs at the measured link rate would pass the phase "
                                      "budget of %.0f s (%.0f s spent)" % (est, budget, spent))
                    continue
                figs, samples = {}, {}
                for fname, form in forms.items():
                    figs[fname], runs_s, why = measure(s, P, A, d, c, form, regions[(P, A, d)], links[fname])
                    if why:
                        figs[fname] = why
                    elif figs[fname]["verified"]:
                        samples[fname] = runs_s
                if not samples:
                    cells_out[key] = figs["direct"] if len(figs) == 1 else {"forms": figs}
                    continue
                # direct stays the cell's form unless another beats its median by more than the spread
                best, stats, margin = choose_form(samples)
                cell = dict(figs[best])
                if dropped:
                    cell["forms_not_run"] = {f: "its staging did not fit beside the regions on some GPU" for f in dropped}
                if same:
                    cell.setdefault("forms_not_run", {}).update(
                        (f, "the plan of a form before it, on every GPU") for f in same)
                if len(figs) > 1:
                    cell["chosen"] = best
                    cell["forms"] = {k: (stats[k] if k in stats else str(v)) for k, v in figs.items()}
                    cell["margin"] = margin
                    cell["choice_rule"] = CHOICE_RULE
                cells_out[key] = cell
    finally:
        for r in regions.values():
            r.close()
    result["spent_s"] = round(time.time() - t0, 1)


# ---------------------------------------------------------------- diagnostics of the N > 1 line
LOG_DIR = [None]        # per-job directory of the ranks' RCCL logs (NCCL_DEBUG_FILE)


def job_key():
    """one name per job, the same on every rank: the parent's rendezvous key, else the launcher's
    port + run id + the launcher's pid (every local rank's parent)"""
    key = os.environ.get("XG_RDZV_KEY")
    if not key:
        key = "%s_%s_pp%d" % (os.environ.get("MASTER_PORT", "0"), os.environ.get("TORCHELASTIC_RUN_ID", ""),
                              os.getppid())
    return re.sub(r"[^A-Za-z0-9_-]", "_", key)


def rccl_log_setup(rank):
    """N > 1: every rank's RCCL warnings into a file of its own (unless NCCL_DEBUG_FILE is set), so
    rank 0 can attach their tails to the line when something fails"""
    d = "/tmp/xg_bench_nccl_%s" % job_key()
    os.makedirs(d, exist_ok=True)
    os.environ.setdefault("NCCL_DEBUG", "WARN")
    if "NCCL_DEBUG_FILE" not in os.environ:
        os.environ["NCCL_DEBUG_FILE"] = os.path.join(d, "rank%d.log" % rank)
        LOG_DIR[0] = d


NOISE = ("LL cutoff points not detected", "Could not read node")


def rccl_log_tails(lines=6):
    """{rank: last RCCL warning lines} of every rank of this job (same host), or None"""
    d = LOG_DIR[0]
    if not d or not os.path.isdir(d):
        return None
    out = {}
    for f in sorted(os.listdir(d)):
        m = re.match(r"rank(\d+)\.log$", f)
        if not m:
            continue
        try:
            txt = [x.strip() for x in open(os.path.join(d, f), errors="replace").read().splitlines()]
        except OSError:
            continue
        txt = [x for x in txt if x and not any(n in x for n in NOISE)]
        if txt:
            out[m.group(1)] = [x[-300:] for x in txt[-lines:]]
    return out or None


def line_failed(out):
    """anything in the line that says a phase or cell failed"""
    x = out.get("xgmi") or {}
    b = out.get("baseline_configs_8gpu") or {}
    return bool(out.get("error") or out.get("xgmi_error") or out.get("failed_methods") or x.get("ceiling_error")
                or x.get("sweep_error") or x.get("links_error") or b.get("error") or
                any(str(v).startswith("failed") for v in (b.get("cells") or {}).values()))


def finish_line(out, world):
    """what every N > 1 line carries at print time, wherever it is printed: the wall time of each
    phase and, when something failed, the tail of every rank's RCCL warnings"""
    if world > 1:
        out["phase_wall_s"] = phase_walls()
        if line_failed(out):
            out["rccl_log_tail"] = rccl_log_tails()
    return out


def transport():
    if os.environ.get("XG_SHARE_GPU") == "1":
        return ("every rank on ONE GPU (XG_SHARE_GPU=1): RCCL's socket transport on loopback, not xGMI -- "
                "the multi-rank path's calls are real, its rates are not the node's")
    return "RCCL p2p between the node's GPUs (xGMI)"


# ---------------------------------------------------------------- N-GPU job without a launcher
def spawn_ranks(a):
    """Parent of an N-GPU job (no WORLD_SIZE in the environment): never touches the GPU.
    Runs the host-MPI baseline, starts one child process of this script per GPU
    (subprocess, not exec), waits, and prints rank 0's JSON line with the baseline
    attached.  Exit code: the highest child exit code (a failed child stops the rest).
    XG_BENCH_CHILD_STUB=1 (test hook): each child prints its rank environment and exits
    with the code XG_BENCH_STUB_RC lists for it; the parent prints them all."""
    stub = os.environ.get("XG_BENCH_CHILD_STUB") == "1"
    methods = [int(x) for x in a.methods.split(",")]
    cpu = cpu_cfg = None
    if not a.no_cpu_baseline and not stub:
        start_heartbeat()             # the children's rank 0 has its own once they start
        phase("cpu baseline")
        cpu = cpu_baseline(a, methods)
        if cpu_configs_on(a, a.gpus):
            phase("cpu baseline at the BASELINE 8-GPU configurations")
            cpu_cfg = cpu_baseline_configs(a)
        phase("children")
    key = "bench%d_%d" % (os.getpid(), int(time.time() * 1e3))
    argv = [x for x in sys.argv[1:]]
    if "--no-cpu-baseline" not in argv:
        argv.append("--no-cpu-baseline")
    procs, outs = [], []
    # ranks sharing one GPU (XG_SHARE_GPU=1, runtime/ctx.hip): 1 hardware queue each, whatever the
    # environment says (the one-GPU boxes export HIP's default 4: 8 ranks x 4 queues time-slice)
    share = {"GPU_MAX_HW_QUEUES": "1"} if os.environ.get("XG_SHARE_GPU") == "1" else {}
    for r in range(a.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                   LOCAL_WORLD_SIZE=str(a.gpus), XG_RDZV_KEY=key, XG_BENCH_PARENT=str(os.getpid()), **share)
        p = subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__)] + argv, env=env,
                             stdout=subprocess.PIPE, text=True)
        procs.append(p)
        outs.append([])
    readers = []
    for p, o in zip(procs, outs):
        t = threading.Thread(target=lambda p=p, o=o: o.extend(p.stdout), daemon=True)
        t.start()
        readers.append(t)
    t0, failed_at = time.time(), None
    while any(p.poll() is None for p in procs):
        time.sleep(0.2)
        rcs = [p.poll() for p in procs]
        if failed_at is None and any(rc not in (None, 0) for rc in rcs):
            failed_at = time.time()
            sys.stderr.write("bench: rank(s) %s failed; stopping the others\n"
                             % [r for r, rc in enumerate(rcs) if rc not in (None, 0)])
        late = a.child_timeout and time.time() - t0 > a.child_timeout
        if (failed_at is not None and time.time() - failed_at > 10) or late:
            if late and failed_at is None:
                failed_at = time.time()
                sys.stderr.write("bench: children still running after %.0f s; stopping them\n" % a.child_timeout)
            for p in procs:            # exact PIDs of this job's children
                if p.poll() is None:
                    p.terminate()
            deadline = time.time() + 10
            while any(p.poll() is None for p in procs) and time.time() < deadline:
                time.sleep(0.2)
            for p in procs:
                if p.poll() is None:
                    p.kill()
    for t in readers:
        t.join(timeout=5)
    rcs = [p.wait() for p in procs]
    rc = max((abs(x) if x < 0 else x) for x in rcs)
    if stub:
        kids = []
        for o in outs:
            kids += [json.loads(line) for line in o if line.startswith("{")]
        print(json.dumps({"stub": True, "children": kids, "rcs": rcs, "rc": rc}))
        return rc
    for r, o in enumerate(outs):          # anything the children printed besides the JSON line
        for line in o:
            if not (r == 0 and line.startswith("{")):
                sys.stderr.write(line)
    lines = [line for line in outs[0] if line.startswith("{")]
    if rc or not lines:
        sys.stderr.write("bench: %d-GPU job failed (child exit codes %s)\n" % (a.gpus, rcs))
    if not lines:
        return rc or 1
    out = json.loads(lines[-1])           # rank 0's line -- a failed job's too (value null + error)
    out["cpu_baseline"] = cpu
    if cpu_cfg is not None:
        out["cpu_baseline_configs"] = cpu_cfg
        out["reference_vs_gpu_max_total_time"] = side_by_side(out)
    out["launch"] = "bench.py parent: %d child processes (subprocess), one per GPU" % a.gpus
    if rc:
        out["child_exit_codes"] = rcs
    print(json.dumps(out))
    return rc


def child_stub():
    """XG_BENCH_CHILD_STUB=1: report the rank environment the parent gave this child."""
    r = int(os.environ["RANK"])
    rcs = [int(x) for x in os.environ.get("XG_BENCH_STUB_RC", "").split(",") if x.strip()]
    print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "XG_RDZV_KEY",
                                                     "XG_BENCH_PARENT")}))
    return rcs[r] if r < len(rcs) else 0


# ---------------------------------------------------------------- rendezvous (no torch)
def rendezvous_uid(xg, rank, world):
    key = os.environ.get("XG_RDZV_KEY")
    if key:
        path = "/tmp/xg_bench_rdzv_%s.bin" % re.sub(r"[^A-Za-z0-9_-]", "_", key)
    else:
        port = os.environ.get("MASTER_PORT", "0")
        run = os.environ.get("TORCHELASTIC_RUN_ID", "")
        # the launcher (torchrun agent) is the parent of every local rank: its pid keeps a
        # stale file of an earlier launch on the same port from matching
        path = "/tmp/xg_bench_rdzv_%s_%s_pp%d.bin" % (port, re.sub(r"[^A-Za-z0-9_-]", "_", run), os.getppid())
    t_start = time.time()
    if rank == 0:
        uid = xg.unique_id()
        tmp = "%s.%d" % (path, os.getpid())
        with open(tmp, "wb") as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid, path
    while True:
        try:
            st = os.stat(path)
            # rank 0 may run the host-MPI baseline before it writes the id (launcher mode)
            if st.st_mtime >= t_start - 900:
                with open(path, "rb") as f:
                    uid = f.read()
                if len(uid) == 128:
                    return uid, None
        except FileNotFoundError:
            pass
        if time.time() - t_start > 900:
            raise RuntimeError("rank %d: no RCCL id at %s" % (rank, path))
        time.sleep(0.01)


def xgmi_phase(xg, ctx, runs, world, nmethods, steps, elapsed, out):
    """N > 1: the timed region's cross-GPU bytes against the measured RCCL all-pairs ceiling, and the
    pt2pt sweep; out["xgmi"] is filled as the figures come in (a guard may print it half done).
    The ceiling and the sweep are measurements beside the exchange, not the exchange: an RCCL error
    in them leaves null + the error in the line (as long as the ranks can still agree on it --
    every rank reduces the error flag with the figures)."""
    phase("xGMI ceiling (RCCL all-pairs send/recv)")
    cross_step = 0      # every rank derives every GPU's plan (deterministic, cheap)
    for r in runs:
        for g in range(world):
            cross_step += r.sched.devplan(world, g, r.pack_max_seg).remote_send_bytes
    per_pair = max(65536, (cross_step // max(1, nmethods * world * (world - 1)) + 4095) & ~4095)
    achieved = cross_step * steps / elapsed / 1e9
    xgmi = out["xgmi"] = {"achieved": round(achieved, 1), "peak": None, "unit": "GB/s", "frac": None,
                          "cross_gpu_bytes_per_step": int(cross_step),
                          "peak_source": "measured: RCCL all-pairs send/recv, %d B per GPU pair, slowest GPU "
                                         "egress x %d (xg_p2p_bench mode 0)" % (per_pair, world),
                          "ceiling_error": None}
    ceil_err = None
    try:
        ceil_gbps, _ = ctx.p2p_bench(per_pair, mode=0, reps=20)
        err = 0.0
    except xg.XGError as e:
        ceil_gbps, err, ceil_err = 0.0, 1.0, str(e)
    neg, err = ctx.allreduce_max([-ceil_gbps, err])
    if err:
        xgmi["ceiling_error"] = ceil_err or "failed on another GPU"
    else:
        ceil_min = -neg                                       # slowest GPU's egress
        xgmi["peak"] = round(ceil_min * world, 1)
        xgmi["frac"] = round(achieved / (ceil_min * world), 4)
    phase("xGMI p2p sweep")
    xgmi["sweep"], xgmi["sweep_error"] = p2p_sweep(ctx, world, xg.XGError)
    phase("xGMI per-link sweep")
    xgmi["links"], xgmi["links_error"] = link_sweep(ctx, world, error=xg.XGError)
    phase("xGMI per-call cost")
    xgmi["per_call"], xgmi["per_call_error"] = call_cost(ctx, world, error=xg.XGError)
    # the timed region's link bound: the chosen plans' busiest-link bytes per step at the median
    # measured link rate, and the share of it the timed steps reached (rank 0 prints the line)
    rate = link_rate(out)
    if rate and ctx.rank == 0:
        lb = [link_bytes(xg, r.sched, world, r.pack_max_seg, r.pack_form) for r in runs]
        busiest = sum(b for b, _ in lb)
        bound_ms = busiest / (rate * 1e9) * 1e3
        xgmi["link_bound"] = {"busiest_link_bytes_per_step": int(busiest), "link_GBps": rate,
                              "link_bytes_per_step": int(sum(x for _, x in lb)),
                              "ms_per_step": round(bound_ms, 4),
                              "frac": round(bound_ms / (elapsed / steps * 1e3), 4)}


def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        return spawn_ranks(a)
    if os.environ.get("XG_BENCH_CHILD_STUB") == "1":
        return child_stub()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", str(a.gpus)))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world != a.gpus:
        raise SystemExit("WORLD_SIZE=%d but --gpus %d" % (world, a.gpus))
    methods = [int(x) for x in a.methods.split(",")]
    parent = "XG_BENCH_PARENT" in os.environ
    # up to the communicator: the reference's CPU phases on rank 0 (under a launcher) come first
    wd = start_watchdog(a.watchdog + pre_value_allowance(a, rank, world, parent) if a.watchdog > 0 else 0, rank)
    phase("start")
    if rank == 0:
        start_heartbeat()

    # host-MPI baselines first, before this process touches the GPU (rank 0; a parent
    # process of an N-GPU job runs them itself and passes --no-cpu-baseline)
    cpu = cpu_cfg = None
    if rank == 0 and not a.no_cpu_baseline:
        phase("cpu baseline")
        cpu = cpu_baseline(a, methods)
        if cpu_configs_on(a, world):
            phase("cpu baseline at the BASELINE 8-GPU configurations")
            cpu_cfg = cpu_baseline_configs(a)
    if world > 1:
        rccl_log_setup(rank)

    import __graft_entry__ as G
    xg = G.load_package().xg
    uid, rdzv = (None, None)
    dev = int(os.environ.get("XG_DEVICE", local))   # XG_DEVICE: test hook (several ranks on one GPU)
    try:
        if world > 1:
            phase("rendezvous (RCCL id file)")
            uid, rdzv = rendezvous_uid(xg, rank, world)
        phase("RCCL communicator init (ncclCommInitRank, %d ranks)" % world)
        ctx = xg.Context(rank=rank, nranks=world, device=dev, uid=uid)
    except xg.XGError as e:
        # no communicator, so nothing to agree over: each rank reports for itself, rank 0 the line
        if rank == 0:
            print(json.dumps(finish_line({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world,
                                          "higher_is_better": True, "dtype": "u8",
                                          "error": "device / RCCL init failed on rank 0 (%s): %s" % (PHASE[0], e),
                                          "cpu_baseline": cpu}, world)), flush=True)
        sys.stderr.write("bench: rank %d: %s\n" % (rank, e))
        return 1
    wd.arm(a.watchdog)              # from the communicator to the measured value
    ctx.barrier()
    if rdzv:
        os.unlink(rdzv)
    if world > 1:
        # every rank plans every GPU's RCCL calls from its own arguments: ranks started with
        # different ones would post calls nobody pairs and hang in RCCL -- compare first
        import hashlib
        keys = sorted(k for k in os.environ if k.startswith("XG_") and k not in ("XG_RDZV_KEY", "XG_DEVICE"))
        blob = repr((vars(a), [(k, os.environ[k]) for k in keys])).encode()
        h = int.from_bytes(hashlib.sha256(blob).digest()[:8], "little")
        parts = [float((h >> (16 * i)) & 0xffff) for i in range(4)]
        got = ctx.allreduce_max(parts + [-x for x in parts])
        if any(got[i] != -got[4 + i] for i in range(4)):
            raise SystemExit("bench: the ranks were started with different arguments or XG_* settings")
    if a.copy_variant >= 0 or a.chunk:
        ctx.set_copy_params(a.chunk, a.copy_variant)
    arch, cus, hbm = ctx.info()

    rl = xg.aggregator_list(a.procs, a.aggs)
    runs, max_total, tune = [], {}, {}

    def timed_reps(r, reps):
        """device time of `reps` back-to-back runs of one method, MAX over GPUs"""
        ctx.barrier()
        ctx.device_sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            r.enqueue()
        ctx.device_sync()
        r.check()
        return ctx.allreduce_max([time.perf_counter() - t0])[0] / reps

    # N > 1: per method, pick by measurement whether cross-GPU segments go to RCCL
    # one op per segment (direct), in runs contiguous at one end with the rest staged on
    # the other (packed one-sided), packed into one staging buffer per peer (pack +
    # unpack launches, two-sided), or -- where it reroutes some step of the method (three or
    # more GPUs, messages >= 1 MiB) -- cut over every link in two groups (relay; relay_coalesced:
    # the same hops, one call per hop and kind).  Every form
    # is timed FORM_REPS times and choose_form keeps direct unless another form's median beats
    # it by more than the spread.  Every GPU sees the same MAX times -> the same choice.
    tune_on = a.tune_pack == 1 or (a.tune_pack < 0 and world > 1 and a.pack_max_seg == 4 << 20)
    names = {(0, -1): "direct", (4 << 20, xg.PACK_ONE_SIDED): "packed_one_sided",
             (4 << 20, xg.PACK_TWO_SIDED): "packed_two_sided", (0, xg.RELAY): "relay",
             (0, xg.RELAY_COALESCED): "relay_coalesced"}
    relays = ((0, xg.RELAY), (0, xg.RELAY_COALESCED))
    base = [k for k in names if k not in relays] if tune_on else [(a.pack_max_seg, -1)]
    failed = {}         # method -> why each of its plan forms was refused (every form failed)
    for m in methods:
        phase("method %d: verify + plan choice" % m)
        s = xg.Schedule(m, a.procs, a.aggs, a.size, a.comm_size, rl, ntimes=1)
        cands = list(base)
        if tune_on and world >= 3:
            # a relay form only where it changes some GPU's plan (MAX over the GPUs: all agree; the
            # coalesced form also reroutes steps the uniform cut does not help, by a weighted split)
            v0 = s.devplan(world, rank, 0, 0, -1)
            vs = [s.devplan(world, rank, pk, 0, form) for pk, form in relays]
            dif = ctx.allreduce_max([1.0 if (v.copies, v.p2p) != (v0.copies, v0.p2p) else 0.0 for v in vs])
            cands.extend(f for f, d in zip(relays, dif) if d)
        passed, samples, why = {}, {}, {}
        for pk, form in cands:
            fname = names.get((pk, form), "plan")
            # a form that cannot be planned, loaded or verified on SOME GPU is left out on every
            # GPU alike (MAX over the GPUs) and recorded; the line is printed from the forms that
            # passed.  Nothing collective is posted with a plan before every GPU has loaded it.
            r, err = None, ""
            try:
                r = xg.MethodRun(ctx, s, it=0, mode=0, pack_max_seg=pk, pack_form=form)
            except xg.XGError as e:
                err = "plan failed: %s" % e
            if ctx.allreduce_max([1.0 if err else 0.0])[0]:
                why[fname] = err or "plan failed on another GPU"
                if r is not None:
                    r.close()
                continue
            # parity gate + the reference's own timing report for this method
            ctx.barrier()
            done, post, _wall = r.run_timed()
            lo, hi = s.block_range(world, rank)
            tmax = max(s.rank_timer(q, done, post, world).total_time for q in range(lo, hi)) if hi > lo else 0.0
            _chk, bad, _first = r.verify()
            nbad = float(sum(1 for b in bad if b))
            tmax, nbad = ctx.allreduce_max([tmax, nbad])
            if nbad:
                why[fname] = "verify failed: %d slots (most on one GPU)" % nbad
                r.close()
                continue
            # the reference's report for a warm method: median of 3 more timed runs
            tw = []
            for _ in range(3):
                ctx.barrier()
                done, post, _wall = r.run_timed()
                tw.append(max(s.rank_timer(q, done, post, world).total_time for q in range(lo, hi)) if hi > lo else 0.0)
            tmax = ctx.allreduce_max([sorted(tw)[1]])[0]
            if len(cands) > 1:
                samples[fname] = [timed_reps(r, 2) for _ in range(FORM_REPS)]
            passed[fname] = (r, tmax, (pk, form))
        if len(cands) > 1:
            tune.setdefault(str(m), {}).update(why)
        if not passed:
            failed[str(m)] = why
            continue
        chosen = next(iter(passed))
        if len(cands) > 1:
            chosen, stats, margin = choose_form(samples)
            tm = tune[str(m)]
            for f, st in stats.items():
                tm[f + "_ms"] = st["median_ms"]
            tm.update(stats={f: stats[f] for f in stats}, chosen=chosen, margin=margin, choice_rule=CHOICE_RULE)
        for f, (r, _t, _k) in passed.items():
            if f != chosen:
                r.close()
        max_total[str(m)] = passed[chosen][1]
        runs.append(passed[chosen][0])
    if failed:
        # a method none of whose forms delivered: no throughput can be quoted for the
        # workload -- say which and why in the line, then fail
        for r in runs:
            r.close()
        if rank == 0:
            print(json.dumps(finish_line({"metric": METRIC, "value": None, "unit": "GB/s", "n_gpus": world,
                                          "steps": a.steps, "warmup": a.warmup, "higher_is_better": True,
                                          "dtype": "u8",
                                          "error": "every plan form of method(s) %s failed" % ",".join(sorted(failed)),
                                          "failed_methods": failed, "pack_autotune_ms_per_run": tune or None,
                                          "cpu_baseline": cpu}, world)))
        ctx.close()
        return 1

    def step():
        for r in runs:
            r.enqueue()

    def check_all():
        for r in runs:
            r.check()

    phase("warm-up")
    for _ in range(a.warmup):
        step()
    ctx.device_sync()
    check_all()

    # timed region: K steps, nothing but the exchange on the stream.  One HIP event
    # pair brackets the whole region on that stream (kernel-timing session, region
    # mode): with nothing but copy launches in it (N = 1) its device time over the
    # number of launches is the copy kernel's average launch duration, gaps between
    # back-to-back launches included.
    phase("timed steps")
    launches_per_step = sum(r.launches for r in runs)
    region = world == 1 and not any(r.view.p2p for r in runs)
    ctx.barrier()
    ctx.device_sync()
    t0 = time.perf_counter()
    if region:
        ctx.ktime_begin(per_launch=False)
    for _ in range(a.steps):
        step()
    # the region's end event goes in right behind the last launch, before the host waits:
    # its device time is then inside the host-timed interval [t0, t1]
    kms, nlaunch, kbytes = ctx.ktime_end() if region else (0.0, 0, 0)
    ctx.device_sync()
    t1 = time.perf_counter()
    check_all()
    ctx.barrier()
    elapsed = ctx.allreduce_max([t1 - t0])[0]
    how = None
    if region:
        how = ("one HIP event pair on the exchange stream around the timed region itself (%d back-to-back "
               "launches; launch gaps included)" % nlaunch)
    elif not a.no_ktime:
        # N > 1 the region also holds RCCL: a second pass of the same K steps with an
        # event pair around every copy launch (the events cost ~7 us of device time
        # per launch, so this pass is kept out of `value`)
        ctx.barrier()
        ctx.device_sync()
        ctx.ktime_begin(max(1, launches_per_step * a.steps), per_launch=True)
        t2 = time.perf_counter()
        for _ in range(a.steps):
            step()
        ctx.device_sync()
        t3 = time.perf_counter()
        kms, nlaunch, kbytes = ctx.ktime_end()
        check_all()
        ctx.barrier()
        how = ("HIP events around every copy launch, on its stream, over a second pass of the same %d steps "
               "(that pass: %.4f ms per step)" % (a.steps, ctx.allreduce_max([t3 - t2])[0] / a.steps * 1e3))

    seg_bytes = float(a.procs) * a.aggs * a.size * len(methods) * a.steps
    value = seg_bytes / elapsed / 1e9
    wd.cancel()      # the value is measured: the LineGuards own every phase after this

    roof = None
    if nlaunch and rank == 0:
        avg_s = kms / nlaunch / 1e3
        per_launch = kbytes / nlaunch
        achieved = per_launch / avg_s / 1e9
        if region and avg_s * launches_per_step > elapsed / a.steps * 1.001:
            raise SystemExit("bench: kernel time %.1f us x %d launches exceeds the step time %.1f us"
                             % (avg_s * 1e6, launches_per_step, elapsed / a.steps * 1e6))
        traffic, traffic_src = None, None
        tf = os.path.join(REPO, "profiles", "pmc_traffic.json")
        if os.path.exists(tf):
            try:
                pm = json.load(open(tf))
                traffic, traffic_src = pm.get("hbm_bytes_per_launch"), pm.get("source")
            except (ValueError, OSError):
                traffic = None
        # the committed PMC figure is per launch of THIS workload at N = 1; any other
        # launch size has not been counted
        if traffic and (world != 1 or abs(traffic - per_launch) > 0.05 * per_launch):
            traffic = None
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "traffic_source": ("committed PMC measurement of this bench command (not counted in this run): "
                                   "profiles/pmc_traffic.json, %s" % traffic_src) if traffic else None,
                "kernel": "copy_kernel (intra-GPU gather/scatter)", "launches": nlaunch,
                "launches_per_step": launches_per_step,
                "avg_launch_us": round(avg_s * 1e6, 2), "algorithmic_bytes_per_launch": int(per_launch),
                "measured": how}
    out = {
        "metric": METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic: reference MAP_DATA fingerprint (mpi_test.c:23), verified on device before timing",
        "config": {"workload": "configs[1]: %d logical ranks, %d aggregators, -d %d, methods %s, -c %d, "
                               "aggregator type 1; one step = one -k repetition of each method"
                               % (a.procs, a.aggs, a.size, ",".join(map(str, methods)), a.comm_size),
                   "procs": a.procs, "cb_nodes": a.aggs, "data_size": a.size, "methods": methods,
                   "ranks_per_gpu": -(-a.procs // world), "device": arch, "cus": cus,
                   "copy_variant": a.copy_variant if a.copy_variant >= 0 else int(os.environ.get("XG_COPY_VARIANT", 0)),
                   "parallelism": "block-mapped logical ranks; intra-GPU copy_kernel + grouped RCCL p2p"},
        "max_total_time_s": max_total,      # per method, one -k repetition, median of 3 warm runs
        "roofline": roof,
        "xgmi": None,
        "pack_autotune_ms_per_run": tune or None,
        "cpu_baseline": cpu,
    }
    if world > 1:
        out["rccl_version"] = xg.rccl_version()
        out["transport"] = transport()
    if cpu_cfg is not None:
        out["cpu_baseline_configs"] = cpu_cfg
    if world > 1:
        # N > 1: cross-GPU (xGMI) bytes of the timed region vs the measured RCCL all-pairs ceiling
        with LineGuard(out, rank, a.xgmi_budget, lambda msg: out.__setitem__("xgmi_error", msg)):
            xgmi_phase(xg, ctx, runs, world, len(methods), a.steps, elapsed, out)
    if a.baseline_configs == "on" or (a.baseline_configs == "auto" and world == 8):
        # BASELINE.json's 8-GPU configurations on this job, after everything above is measured.
        # The line must come out whatever happens in there: a rank still in the phase GUARD_GRACE s past
        # its budget (a peer lost inside RCCL waits forever) prints the line with what was done (rank 0)
        # and ends its process.
        for r in runs:
            r.close()
        runs = []
        extra = out["baseline_configs_8gpu"] = {"budget_s": a.baseline_budget}
        with LineGuard(out, rank, a.baseline_budget + GUARD_GRACE, lambda msg: extra.__setitem__("error", msg)):
            try:
                extra["link_GBps"] = link_rate(out)
                baseline_configs_phase(xg, ctx, world, rank, a.baseline_budget, extra, link_gbps=extra["link_GBps"])
            except xg.XGError as e:
                extra["error"] = str(e)
    if rank == 0:
        if cpu_cfg is not None:
            out["reference_vs_gpu_max_total_time"] = side_by_side(out)
        print(json.dumps(finish_line(out, world)))
    ctx.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
