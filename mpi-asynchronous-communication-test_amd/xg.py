"""ctypes binding of the framework's C-ABI (include/xg_sched.h, include/xg.h).

Python is only the harness here (bench.py, tests): every byte of the exchange
is moved by lib/libxg.so (HIP kernels + RCCL) and every schedule comes from
lib/libxghost.so.  There is no fallback: if a library is missing, loading
fails with an error that says how to build it.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIBDIR = os.environ.get("XG_LIBDIR") or os.path.join(HERE, "lib")   # XG_LIBDIR: e.g. a sanitizer build of libxghost


class XGError(RuntimeError):
    pass


class Timer(C.Structure):
    """Timer of the reference (mpi_test.c:25-31)."""
    _fields_ = [("post_request_time", C.c_double), ("send_wait_all_time", C.c_double),
                ("recv_wait_all_time", C.c_double), ("barrier_time", C.c_double),
                ("total_time", C.c_double)]

    def as_tuple(self):
        return (self.post_request_time, self.send_wait_all_time, self.recv_wait_all_time,
                self.barrier_time, self.total_time)


NBUF = 5   # XG_NBUF


class Msg(C.Structure):
    _fields_ = [("src", C.c_int32), ("sseg", C.c_int32), ("dst", C.c_int32), ("dslot", C.c_int32),
                ("len", C.c_int64), ("step", C.c_int32), ("flags", C.c_int32),
                ("sbuf", C.c_int32), ("dbuf", C.c_int32), ("soff", C.c_int64), ("doff", C.c_int64)]


class Copy(C.Structure):
    _fields_ = [("src_off", C.c_int64), ("dst_off", C.c_int64), ("len", C.c_int64),
                ("src_buf", C.c_int32), ("dst_buf", C.c_int32)]


class P2P(C.Structure):
    _fields_ = [("off", C.c_int64), ("len", C.c_int64), ("peer", C.c_int32), ("buf", C.c_int32),
                ("is_send", C.c_int32), ("group", C.c_int32)]


class StepPlan(C.Structure):
    _fields_ = [("pre_begin", C.c_int32), ("pre_count", C.c_int32), ("p2p_begin", C.c_int32),
                ("p2p_count", C.c_int32), ("post_begin", C.c_int32), ("post_count", C.c_int32),
                ("sync_after", C.c_int32), ("stage_count", C.c_int32), ("posts", C.c_int32)]


class DevPlan(C.Structure):
    _fields_ = [("gpu", C.c_int32), ("ngpus", C.c_int32), ("nsteps", C.c_int32), ("pad", C.c_int32),
                ("region_bytes", C.c_int64 * NBUF), ("ncopy", C.c_int32), ("np2p", C.c_int32),
                ("copies", C.POINTER(Copy)), ("p2p", C.POINTER(P2P)), ("steps", C.POINTER(StepPlan)),
                ("local_bytes", C.c_int64), ("remote_send_bytes", C.c_int64),
                ("remote_recv_bytes", C.c_int64)]


class Call(C.Structure):
    """xg_call: one RCCL call of a step (XG_CALL_SEND / RECV / BARRIER)."""
    _fields_ = [("kind", C.c_int32), ("peer", C.c_int32), ("buf", C.c_int32), ("pad", C.c_int32),
                ("off", C.c_int64), ("len", C.c_int64)]


class CallPair(C.Structure):
    _fields_ = [("step", C.c_int32), ("src", C.c_int32), ("dst", C.c_int32), ("send_call", C.c_int32),
                ("recv_call", C.c_int32), ("group", C.c_int32), ("len", C.c_int64)]


CALL_SEND, CALL_RECV, CALL_BARRIER = 1, 2, 3


class SoloShape(C.Structure):
    _fields_ = [("rails", C.c_int32), ("npieces", C.c_int32), ("nrows", C.c_int32), ("nmeta", C.c_int32)]


class Span(C.Structure):
    _fields_ = [("src", C.c_uint64), ("dst", C.c_uint64), ("len", C.c_uint64)]


class SegRun(C.Structure):
    _fields_ = [("rank", C.c_int32), ("seed0", C.c_int32), ("off", C.c_int64), ("nsegs", C.c_int32),
                ("pad", C.c_int32)]


class Slot(C.Structure):
    _fields_ = [("src", C.c_int32), ("seed", C.c_int32), ("dst", C.c_int32), ("pad", C.c_int32),
                ("off", C.c_int64)]


A2M, M2A = 0, 1
BUF_SEND, BUF_RECV, BUF_STAGE_SEND, BUF_STAGE_RECV, BUF_SCRATCH = 0, 1, 2, 3, 4
PACK_TWO_SIDED, PACK_ONE_SIDED, RELAY, RELAY_COALESCED = 0, 1, 2, 3   # xg_devplan_build_form (xg_sched.h XG_RELAY, XG_RELAY_COALESCED)
CALL_SEND, CALL_RECV, CALL_BARRIER, CALL_FENCE = 1, 2, 3, 4   # xg_call kinds
MSG_COPY, MSG_COLL, MSG_CTRL = 1, 2, 4
TAM_METHODS = (15, 16)
MPICH_EAGER_LIMIT = 65424


def _load(name):
    path = os.path.join(LIBDIR, name)
    if not os.path.exists(path):
        raise XGError("%s not built: run `make -C %s` (or __graft_entry__.build())" % (path, HERE))
    return C.CDLL(path, mode=C.RTLD_GLOBAL)


_host = None
_dev = None


def host():
    global _host
    if _host is None:
        h = _load("libxghost.so")
        h.xg_aggregator_list.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int)]
        h.xg_method_label.restype = C.c_char_p
        h.xg_method_label.argtypes = [C.c_int]
        h.xg_method_direction.argtypes = [C.c_int]
        h.xg_sched_build.restype = C.c_void_p
        h.xg_sched_build.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int, C.POINTER(C.c_int),
                                     C.c_int, C.c_int, C.c_int, C.c_int64, C.c_char_p, C.c_size_t]
        h.xg_sched_build_iter.restype = C.c_void_p
        h.xg_sched_build_iter.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int, C.POINTER(C.c_int),
                                          C.c_int, C.c_int, C.c_int, C.c_int64, C.c_int, C.c_char_p, C.c_size_t]
        h.xg_sched_free.argtypes = [C.c_void_p]
        for fn in ("xg_sched_nmsg", "xg_sched_nsteps", "xg_sched_direction", "xg_sched_procs"):
            getattr(h, fn).argtypes = [C.c_void_p]
        h.xg_sched_msgs.restype = C.POINTER(Msg)
        h.xg_sched_msgs.argtypes = [C.c_void_p]
        h.xg_sched_trace.restype = C.c_size_t
        h.xg_sched_trace.argtypes = [C.c_void_p, C.c_int, C.c_char_p, C.c_size_t]
        h.xg_sched_rank_timer.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double),
                                          C.POINTER(C.c_double), C.POINTER(Timer)]
        h.xg_sched_rank_rep_timers.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(C.c_double),
                                               C.POINTER(C.c_double), C.POINTER(Timer)]
        h.xg_sched_ntimes.argtypes = [C.c_void_p]
        h.xg_sched_timed_steps.argtypes = [C.c_void_p, C.POINTER(C.c_uint8)]
        h.xg_sched_barrier_epochs.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        h.xg_save_all_timing.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(Timer), C.c_char_p]
        h.xg_block_range.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        h.xg_gpu_of.argtypes = [C.c_int, C.c_int, C.c_int]
        for fn in ("xg_send_offset", "xg_recv_offset", "xg_scratch_offset"):
            getattr(h, fn).restype = C.c_int64
            getattr(h, fn).argtypes = [C.c_void_p, C.c_int, C.c_int]
        h.xg_region_bytes.restype = C.c_int64
        h.xg_region_bytes.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int]
        h.xg_devplan_build.restype = C.POINTER(DevPlan)
        h.xg_devplan_build.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int64]
        h.xg_devplan_build_ex.restype = C.POINTER(DevPlan)
        h.xg_devplan_build_ex.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_int64]
        h.xg_devplan_build_form.restype = C.POINTER(DevPlan)
        h.xg_devplan_build_form.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int64, C.c_int64, C.c_int]
        h.xg_devplan_free.argtypes = [C.POINTER(DevPlan)]
        h.xg_devplan_step_calls.argtypes = [C.POINTER(DevPlan), C.c_int, C.c_int64, C.POINTER(Call)]
        h.xg_devplan_step_self_calls.argtypes = [C.POINTER(DevPlan), C.c_int, C.c_int64]
        h.xg_calls_match.restype = C.c_int64
        h.xg_calls_match.argtypes = [C.c_int, C.c_int, C.POINTER(C.POINTER(Call)), C.POINTER(C.POINTER(C.c_int32)),
                                     C.POINTER(CallPair), C.c_int64, C.c_char_p, C.c_size_t]
        h.xg_devplans_match.restype = C.c_int64
        h.xg_devplans_match.argtypes = [C.POINTER(C.POINTER(DevPlan)), C.c_int, C.c_int64, C.POINTER(CallPair),
                                        C.c_int64, C.c_char_p, C.c_size_t]
        h.xg_step_local_meets_unpacks.argtypes = [C.POINTER(DevPlan), C.c_int]
        h.xg_step_stage_meets_rest.argtypes = [C.POINTER(DevPlan), C.c_int]
        h.xg_piece_size.restype = C.c_int64
        h.xg_piece_size.argtypes = [C.POINTER(C.c_int64), C.c_int, C.c_int64, C.c_int, C.c_int64]
        h.xg_fill_runs.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(SegRun)]
        h.xg_verify_slots.argtypes = [C.c_void_p, C.c_int, C.c_int, C.POINTER(Slot)]
        h.xg_engine_hazards.argtypes = [C.POINTER(Span), C.POINTER(C.c_int), C.c_int, C.c_int, C.POINTER(C.c_int)]
        h.xg_solo_reduce_stamps.argtypes = [C.POINTER(C.c_uint64), C.c_int, C.c_int64, C.c_int, C.c_int,
                                            C.POINTER(C.c_uint64)]
        h.xg_solo_reduce_stamps.restype = None
        h.xg_solo_tables.argtypes = [C.POINTER(Span), C.POINTER(C.c_int), C.c_int, C.c_int, C.c_int, C.c_uint64,
                                     C.c_uint64, C.POINTER(SoloShape), C.POINTER(C.c_uint64), C.POINTER(C.c_int)]
        h.xg_solo_tables_g.argtypes = [C.POINTER(Span), C.POINTER(C.c_int), C.c_int, C.c_int, C.c_int, C.c_int,
                                       C.c_uint64, C.c_uint64, C.POINTER(SoloShape), C.POINTER(C.c_uint64),
                                       C.POINTER(C.c_int)]
        h.xg_summarize_results.argtypes = [C.c_int] * 6 + [C.c_char_p, C.c_char_p, Timer, Timer]
        _host = h
    return _host


def aggregator_list(procs, cb_nodes, proc_node=1, agg_type=1):
    rl = (C.c_int * cb_nodes)()
    if host().xg_aggregator_list(procs, cb_nodes, proc_node, agg_type, rl) != 0:
        raise XGError("aggregator type %d is not defined by the reference" % agg_type)
    return list(rl)


def engine_hazards(steps, force=False):
    """xg_engine_hazards over steps = [[(src, dst, len), ...], ...] (byte addresses):
    returns (flags per step, number of hazard points)."""
    spans = [x for st in steps for x in st]
    arr = (Span * max(1, len(spans)))(*[Span(*x) for x in spans])
    beg = [0]
    for st in steps:
        beg.append(beg[-1] + len(st))
    sb = (C.c_int * len(beg))(*beg)
    fl = (C.c_int * max(1, len(steps)))()
    n = host().xg_engine_hazards(arr, sb, len(steps), 1 if force else 0, fl)
    return list(fl)[:len(steps)], n


def solo_tables(steps, rails_max, src_base, dst_base, waves=16, granule=16):
    """xg_solo_tables_g over steps = [[(src, dst, len), ...], ...]: returns (rc, shape dict,
    per-rail descriptor lists, per-rail row barrier counts, per-rail closed-step lists,
    per-rail rows holding real pieces)."""
    spans = [x for st in steps for x in st]
    arr = (Span * max(1, len(spans)))(*[Span(*x) for x in spans])
    beg = [0]
    for st in steps:
        beg.append(beg[-1] + len(st))
    sb = (C.c_int * len(beg))(*beg)
    sh = SoloShape()
    rc = host().xg_solo_tables_g(arr, sb, len(steps), rails_max, waves, granule, src_base, dst_base, C.byref(sh),
                                 None, None)
    shape = {"rails": sh.rails, "npieces": sh.npieces, "nrows": sh.nrows, "nmeta": sh.nmeta}
    if rc:
        return rc, shape, None, None, None, None
    R, npc, nr, n = sh.rails, sh.npieces, sh.nrows, len(steps)
    d = (C.c_uint64 * (R * npc))()
    m = (C.c_int * sh.nmeta)()
    rc = host().xg_solo_tables_g(arr, sb, n, rails_max, waves, granule, src_base, dst_base, C.byref(sh), d, m)
    descs = [list(d[r * npc:(r + 1) * npc]) for r in range(R)]
    close = [list(m[r * (nr + 1):(r + 1) * (nr + 1)]) for r in range(R)]
    off = R * (nr + 1)
    csteps = [list(m[off + r * n: off + (r + 1) * n]) for r in range(R)]
    rows = list(m[off + R * n: off + R * n + R])
    return rc, shape, descs, close, csteps, rows


def solo_reduce_stamps(stamps, s0, s1):
    """xg_solo_reduce_stamps over stamps = [rail][step] (ints, 0 = nothing closed)"""
    R, n = len(stamps), len(stamps[0])
    arr = (C.c_uint64 * (R * n))(*[x for row in stamps for x in row])
    out = (C.c_uint64 * n)()
    host().xg_solo_reduce_stamps(arr, R, n, s0, s1, out)
    return list(out)


def _pairs(n, arr, groups=False):
    if groups:
        return [(q.step, q.group, q.src, q.dst, q.send_call, q.recv_call, q.len) for q in arr[:n]]
    return [(q.step, q.src, q.dst, q.send_call, q.recv_call, q.len) for q in arr[:n]]


def calls_match(calls, nsteps):
    """xg_calls_match over calls[g] = [[(kind, peer, buf, off, len), ...] per step]: RCCL's
    pairing of a G-GPU job's calls; returns [(step, src, dst, send_call, recv_call, len)]
    (step-major) or raises XGError with the reason."""
    G = len(calls)
    arrs, begs = [], []
    for g in range(G):
        flat = [c for st in calls[g] for c in st]
        a = (Call * max(1, len(flat)))(*[Call(k, p, b, 0, o, n) for k, p, b, o, n in flat])
        beg = [0]
        for st in calls[g]:
            beg.append(beg[-1] + len(st))
        arrs.append(a)
        begs.append((C.c_int32 * len(beg))(*beg))
    ca = (C.POINTER(Call) * G)(*[C.cast(a, C.POINTER(Call)) for a in arrs])
    cb = (C.POINTER(C.c_int32) * G)(*[C.cast(b, C.POINTER(C.c_int32)) for b in begs])
    err = C.create_string_buffer(512)
    n = host().xg_calls_match(G, nsteps, ca, cb, None, 0, err, 512)
    if n < 0:
        raise XGError(err.value.decode())
    out = (CallPair * max(1, n))()
    host().xg_calls_match(G, nsteps, ca, cb, out, n, err, 512)
    return _pairs(n, out)


def devplans_match(plans, self_max=0, groups=False):
    """xg_devplans_match over the G device plans (DevicePlanView or raw POINTER(DevPlan)) of one
    job (calls listed with self_max): the pairs (groups: (step, group, src, dst, send_call,
    recv_call, len)), or XGError naming the first call that RCCL would pair differently."""
    ptrs = [p.ptr if isinstance(p, DevicePlanView) else p for p in plans]
    G = len(ptrs)
    arr = (C.POINTER(DevPlan) * G)(*ptrs)
    err = C.create_string_buffer(512)
    n = host().xg_devplans_match(arr, G, self_max, None, 0, err, 512)
    if n < 0:
        raise XGError(err.value.decode())
    out = (CallPair * max(1, n))()
    host().xg_devplans_match(arr, G, self_max, out, n, err, 512)
    return _pairs(n, out, groups)


def piece_size(lens, chunk=32768, cus=256, wg_cost=2048):
    """xg_piece_size: the workgroup piece size of one copy launch over copies of these lengths"""
    arr = (C.c_int64 * max(1, len(lens)))(*lens)
    return host().xg_piece_size(arr, len(lens), chunk, cus, wg_cost)


def method_label(method):
    lab = host().xg_method_label(method)
    return lab.decode() if lab else None


class Schedule:
    """One method run (all -k repetitions), compiled to device-wide steps."""

    def __init__(self, method, procs, cb_nodes, data_size, comm_size, rank_list, ntimes=1,
                 eager_limit=MPICH_EAGER_LIMIT, proc_node=1, barrier_type=0, iteration=0):
        h = host()
        self.method, self.P, self.A, self.d, self.c = method, procs, cb_nodes, data_size, comm_size
        self.rank_list = list(rank_list)
        self.ntimes = ntimes
        err = C.create_string_buffer(512)
        rl = (C.c_int * cb_nodes)(*rank_list)
        self._h = h.xg_sched_build_iter(method, procs, cb_nodes, data_size, comm_size, rl, ntimes,
                                        proc_node, barrier_type, eager_limit, iteration, err, 512)
        if not self._h:
            raise XGError(err.value.decode())
        self.nsteps = h.xg_sched_nsteps(self._h)
        self.direction = h.xg_sched_direction(self._h)

    def __del__(self):
        if getattr(self, "_h", None) and _host is not None:
            _host.xg_sched_free(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def messages(self):
        n = host().xg_sched_nmsg(self._h)
        ptr = host().xg_sched_msgs(self._h)
        return [(m.src, m.sseg, m.dst, m.dslot, m.len, m.step, m.flags) for m in ptr[:n]]

    def locations(self):
        """Per message: (sbuf, soff, dbuf, doff) -- region and offset inside the rank's part."""
        n = host().xg_sched_nmsg(self._h)
        ptr = host().xg_sched_msgs(self._h)
        return [(m.sbuf, m.soff, m.dbuf, m.doff) for m in ptr[:n]]

    def trace(self, rank):
        n = host().xg_sched_trace(self._h, rank, None, 0)
        buf = C.create_string_buffer(n + 1)
        host().xg_sched_trace(self._h, rank, buf, n + 1)
        return buf.value.decode()

    def timed_steps(self):
        """per step 1 if some rank's Timer reads its completion time (the last step always),
        else 0 -- the steps a timed run must mark (xg_sched_timed_steps)"""
        need = (C.c_uint8 * max(1, self.nsteps))()
        if host().xg_sched_timed_steps(self._h, need) < 0:
            raise XGError("xg_sched_timed_steps failed")
        return list(need)[:self.nsteps]

    def rank_timer(self, rank, step_done, step_post=None, ngpus=1):
        nd = (C.c_double * max(1, len(step_done)))(*step_done)
        npost = (C.c_double * max(1, len(step_post)))(*step_post) if step_post is not None else None
        t = Timer()
        if host().xg_sched_rank_timer(self._h, ngpus, rank, nd, npost, C.byref(t)) != 0:
            raise XGError("xg_sched_rank_timer: bad rank/ngpus")
        return t

    def rank_rep_timers(self, rank, step_done, step_post=None, ngpus=1):
        """timers[m] of every repetition (m13)."""
        nd = (C.c_double * max(1, len(step_done)))(*step_done)
        npost = (C.c_double * max(1, len(step_post)))(*step_post) if step_post is not None else None
        reps = (Timer * max(1, self.ntimes))()
        if host().xg_sched_rank_rep_timers(self._h, ngpus, rank, nd, npost, reps) != 0:
            raise XGError("xg_sched_rank_rep_timers: bad rank/ngpus")
        return list(reps)[:self.ntimes]

    def barrier_epochs(self):
        n = host().xg_sched_barrier_epochs(self._h, None)
        out = (C.c_int32 * max(1, n))()
        host().xg_sched_barrier_epochs(self._h, out)
        return list(out)[:n]

    def gpu_of(self, ngpus, rank):
        return host().xg_gpu_of(self.P, ngpus, rank)

    def block_range(self, ngpus, g):
        lo, hi = C.c_int(), C.c_int()
        host().xg_block_range(self.P, ngpus, g, C.byref(lo), C.byref(hi))
        return lo.value, hi.value

    def send_offset(self, ngpus, rank):
        return host().xg_send_offset(self._h, ngpus, rank)

    def recv_offset(self, ngpus, rank):
        return host().xg_recv_offset(self._h, ngpus, rank)

    def scratch_offset(self, ngpus, rank):
        return host().xg_scratch_offset(self._h, ngpus, rank)

    def region_bytes(self, ngpus, g, buf):
        return host().xg_region_bytes(self._h, ngpus, g, buf)

    def devplan(self, ngpus, g, pack_max_seg=4 << 20, pack_min=0, pack_form=-1):
        return DevicePlanView(self, ngpus, g, pack_max_seg, pack_min, pack_form)

    def check_pairing(self, ngpus, pack_max_seg=4 << 20, pack_min=0, pack_form=-1, self_max=0):
        """Refuse (XGError) a job whose GPUs' RCCL calls RCCL would not pair step by step
        (xg_devplans_match over every GPU's plan, built in C, the calls listed with the
        self_max the runtime posts with); returns the number of pairs."""
        h = host()
        plans = [h.xg_devplan_build_form(self._h, ngpus, g, pack_max_seg, pack_min, pack_form)
                 for g in range(ngpus)]
        try:
            if not all(plans):
                raise XGError("method %d on %d GPUs: out of host memory building the device plans"
                              % (self.method, ngpus))
            arr = (C.POINTER(DevPlan) * ngpus)(*plans)
            err = C.create_string_buffer(512)
            n = h.xg_devplans_match(arr, ngpus, self_max, None, 0, err, 512)
            if n < 0:
                raise XGError("method %d on %d GPUs: RCCL calls do not pair: %s"
                              % (self.method, ngpus, err.value.decode()))
            return n
        finally:
            for q in plans:
                if q:
                    h.xg_devplan_free(q)

    def fill_runs(self, ngpus, g):
        n = host().xg_fill_runs(self._h, ngpus, g, None)
        runs = (SegRun * max(1, n))()
        host().xg_fill_runs(self._h, ngpus, g, runs)
        return [(r.rank, r.seed0, r.off, r.nsegs) for r in runs[:n]]

    def verify_slots(self, ngpus, g):
        n = host().xg_verify_slots(self._h, ngpus, g, None)
        sl = (Slot * max(1, n))()
        host().xg_verify_slots(self._h, ngpus, g, sl)
        return [(x.src, x.seed, x.dst, x.off) for x in sl[:n]]


class DevicePlanView:
    """Python view of xg_devplan (host memory), used by the CPU plan tests."""

    def __init__(self, sched, ngpus, g, pack_max_seg, pack_min=0, pack_form=-1):
        self.sched = sched
        # pack_form: PACK_TWO_SIDED, PACK_ONE_SIDED, RELAY, RELAY_COALESCED, or -1 = the library's
        # default (xg_sched.h)
        self._p = host().xg_devplan_build_form(sched.handle, ngpus, g, pack_max_seg, pack_min, pack_form)
        if not self._p:
            self._p = None
            raise XGError("xg_devplan_build_form: out of host memory")
        p = self._p.contents
        self.gpu, self.ngpus, self.nsteps = p.gpu, p.ngpus, p.nsteps
        self.region_bytes = list(p.region_bytes)
        self.copies = [(c.src_buf, c.src_off, c.dst_buf, c.dst_off, c.len) for c in p.copies[:p.ncopy]]
        # (peer, is_send, region, offset, length, group): group 1 = a relay step's second RCCL group
        self.p2p = [(o.peer, o.is_send, o.buf, o.off, o.len, o.group) for o in p.p2p[:p.np2p]]
        self.steps = [(s.pre_begin, s.pre_count, s.p2p_begin, s.p2p_count, s.post_begin, s.post_count)
                      for s in p.steps[:p.nsteps]]
        self.sync_after = [s.sync_after for s in p.steps[:p.nsteps]]
        self.stage_count = [s.stage_count for s in p.steps[:p.nsteps]]
        self.posts = [s.posts for s in p.steps[:p.nsteps]]         # request posts of this GPU's ranks
        self.local_bytes = p.local_bytes
        self.remote_send_bytes = p.remote_send_bytes
        self.remote_recv_bytes = p.remote_recv_bytes

    @property
    def ptr(self):
        return self._p

    def local_meets_unpacks(self, step):
        """xg_step_local_meets_unpacks: may step's local copies share a launch with step-1's unpacks?"""
        return host().xg_step_local_meets_unpacks(self._p, step)

    def stage_meets_rest(self, step):
        """xg_step_stage_meets_rest: must step's stage copies keep a launch of their own?"""
        return host().xg_step_stage_meets_rest(self._p, step)

    def calls(self, step, self_max=0):
        """xg_devplan_step_calls: [(kind, peer, buf, off, len)] this GPU posts in `step`"""
        n = host().xg_devplan_step_calls(self._p, step, self_max, None)
        arr = (Call * max(1, n))()
        host().xg_devplan_step_calls(self._p, step, self_max, arr)
        return [(c.kind, c.peer, c.buf, c.off, c.len) for c in arr[:n]]

    def __del__(self):
        if getattr(self, "_p", None) and _host is not None:
            _host.xg_devplan_free(self._p)
            self._p = None


# --------------------------------------------------------------------------- device (libxg.so)
ROCM_RUNTIME_LIBS = ("libamdhip64.so", "librccl.so", "libhsa-runtime64.so")


def foreign_rocm_runtime():
    """ROCm runtime libraries mapped into this process from outside the ROCm install libxg.so is
    built against (lib/rocm_libdir, /opt/rocm*, or $ROCM_PATH).  torch's wheel bundles its own libamdhip64.so.7,
    librccl.so.1 and libhsa-runtime64.so.1 under the same sonames: once `import torch` has
    loaded them, libxg.so binds to those instead -- another runtime and RCCL than it was built
    and tested with (the full GPU suite hung in RCCL that way, profiles/r04/torch_runtime/)."""
    roots = {os.path.realpath(r) for r in ("/opt/rocm", os.environ.get("ROCM_PATH") or "/opt/rocm")}
    try:        # the library directory of the ROCm libxg.so was linked against (written by the Makefile)
        roots.add(os.path.realpath(open(os.path.join(HERE, "lib", "rocm_libdir")).read().strip()))
    except OSError:
        pass
    try:
        roots |= {os.path.realpath(os.path.join("/opt", n)) for n in os.listdir("/opt") if n.startswith("rocm")}
        maps = open("/proc/self/maps").read().splitlines()
    except OSError:
        return []
    bad = set()
    for line in maps:
        path = line.split(None, 5)[5].strip() if len(line.split(None, 5)) == 6 else ""
        if os.path.basename(path).startswith(ROCM_RUNTIME_LIBS):
            rp = os.path.realpath(path)
            if not any(rp.startswith(r + os.sep) for r in roots):
                bad.add(rp)
    return sorted(bad)


def device():
    """libxg.so -- the HIP/RCCL half.  Loading it does not touch the GPU.  Refused (XGError) in a
    process that already holds another ROCm runtime (foreign_rocm_runtime: e.g. torch's)."""
    global _dev
    if _dev is None:
        host()
        bad = foreign_rocm_runtime()
        if bad:
            raise XGError("libxg.so would bind to the ROCm runtime already loaded in this process from %s "
                          "(e.g. by `import torch`), not the one it is built against: load the framework "
                          "before torch, or in a process without it" % ", ".join(bad))
        d = _load("libxg.so")
        # ... and after loading it: a foreign runtime found first on the library search path
        # (LD_LIBRARY_PATH) binds libxg.so's own dependencies to it
        d.xg_foreign_runtime.argtypes = [C.c_char_p, C.c_size_t]
        buf = C.create_string_buffer(1024)
        if d.xg_foreign_runtime(buf, 1024) > 0:
            raise XGError("libxg.so is bound to a ROCm runtime from outside /opt/rocm (%s): refused"
                          % buf.value.decode())
        vp, ip, i64 = C.c_void_p, C.c_int, C.c_int64
        d.xg_get_unique_id.argtypes = [vp]
        d.xg_init.argtypes = [C.POINTER(vp), ip, ip, ip, vp]
        d.xg_finalize.argtypes = [vp]
        d.xg_init_virtual.argtypes = [C.POINTER(vp), ip, ip, ip]
        d.xg_vplans_run.argtypes = [C.POINTER(vp), ip, C.POINTER(C.c_double)]
        d.xg_vplans_run_rccl.argtypes = [C.POINTER(vp), ip, C.POINTER(C.c_double)]
        d.xg_plan_set_local_only.argtypes = [vp, ip]
        d.xg_plan_set_step_marks.argtypes = [vp, C.POINTER(C.c_uint8)]
        d.xg_self_max.restype = i64
        d.xg_self_max.argtypes = [vp]
        d.xg_barrier.argtypes = [vp]
        d.xg_sync.argtypes = [vp]
        d.xg_device_sync.argtypes = [vp]
        d.xg_allreduce_max.argtypes = [vp, C.POINTER(C.c_double), ip]
        d.xg_device_info.argtypes = [vp, C.c_char_p, C.c_size_t, C.POINTER(ip), C.POINTER(C.c_size_t)]
        d.xg_now.restype = C.c_double
        d.xg_regions_alloc.argtypes = [vp, C.POINTER(i64), C.POINTER(vp)]
        d.xg_regions_free.argtypes = [vp]
        d.xg_regions_poison.argtypes = [vp]
        d.xg_regions_ptr.restype = vp
        d.xg_regions_ptr.argtypes = [vp, ip]
        d.xg_regions_read.argtypes = [vp, ip, i64, vp, i64]
        d.xg_regions_write.argtypes = [vp, ip, i64, vp, i64]
        d.xg_fill.argtypes = [vp, C.POINTER(SegRun), ip, i64, ip, ip]
        d.xg_verify.argtypes = [vp, C.POINTER(Slot), ip, i64, ip, ip, C.POINTER(C.c_uint64),
                                C.POINTER(i64), C.POINTER(i64)]
        d.xg_plan_load.argtypes = [vp, vp, C.POINTER(DevPlan), C.POINTER(vp)]
        d.xg_plan_free.argtypes = [vp]
        d.xg_plan_nsteps.argtypes = [vp]
        d.xg_plan_run.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_double)]
        d.xg_plan_enqueue.argtypes = [vp]
        d.xg_plan_engine.argtypes = [vp]
        d.xg_plan_engine_rails.argtypes = [vp]
        d.xg_plan_check.argtypes = [vp]
        d.xg_plan_launches.argtypes = [vp]
        d.xg_plan_engine_steps.argtypes = [vp, C.POINTER(ip), C.POINTER(ip)]
        d.xg_plan_displs.argtypes = [vp, C.POINTER(i64), ip]
        d.xg_ktime_begin.argtypes = [vp, ip, ip]
        d.xg_ktime_end.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(ip), C.POINTER(i64)]
        d.xg_ktime_launch.argtypes = [vp, ip, C.POINTER(C.c_double), C.POINTER(i64)]
        d.xg_set_copy_params.argtypes = [vp, i64, ip]
        d.xg_p2p_bench.argtypes = [vp, i64, ip, ip, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        d.xg_p2p_pair_bench.argtypes = [vp, i64, ip, ip, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        d.xg_p2p_split_bench.argtypes = [vp, i64, ip, ip, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        d.xg_rccl_version.argtypes = [C.POINTER(C.c_int)]
        _dev = d
    return _dev


def _check(rc, what):
    if rc != 0:
        raise XGError("%s failed with code %d (see stderr)" % (what, rc))


def rccl_version():
    """ncclGetVersion of the RCCL libxg.so runs on, e.g. 22703 (no GPU call)"""
    v = C.c_int()
    _check(device().xg_rccl_version(C.byref(v)), "xg_rccl_version")
    return v.value


def unique_id():
    buf = C.create_string_buffer(128)
    _check(device().xg_get_unique_id(buf), "xg_get_unique_id")
    return buf.raw


class Context:
    """One process = one GPU (xg_init).  nranks > 1 needs rank 0's unique_id()."""

    def __init__(self, rank=0, nranks=1, device_index=None, uid=None, device=None):
        d = globals()["device"]()
        dev = device if device is not None else (device_index if device_index is not None else rank)
        self._c = C.c_void_p()
        ub = C.create_string_buffer(uid, 128) if uid else None
        _check(d.xg_init(C.byref(self._c), rank, nranks, dev, ub), "xg_init")
        self.rank, self.nranks = rank, nranks
        self.is_virtual = False

    @classmethod
    def virtual(cls, rank, nranks, device=0):
        """GPU `rank` of an `nranks`-GPU job emulated on one physical device (test hook,
        xg_init_virtual); run the job's plans together with run_virtual()."""
        self = cls.__new__(cls)
        self._c = C.c_void_p()
        _check(globals()["device"]().xg_init_virtual(C.byref(self._c), rank, nranks, device), "xg_init_virtual")
        self.rank, self.nranks = rank, nranks
        self.is_virtual = True
        return self

    @property
    def handle(self):
        return self._c

    def barrier(self):
        _check(_dev.xg_barrier(self._c), "xg_barrier")

    def sync(self):
        _check(_dev.xg_sync(self._c), "xg_sync")

    def device_sync(self):
        _check(_dev.xg_device_sync(self._c), "xg_device_sync")

    def allreduce_max(self, vals):
        arr = (C.c_double * len(vals))(*vals)
        _check(_dev.xg_allreduce_max(self._c, arr, len(vals)), "xg_allreduce_max")
        return list(arr)

    def info(self):
        name = C.create_string_buffer(64)
        cus, hbm = C.c_int(), C.c_size_t()
        _check(_dev.xg_device_info(self._c, name, 64, C.byref(cus), C.byref(hbm)), "xg_device_info")
        return name.value.decode(), cus.value, hbm.value

    def set_copy_params(self, chunk=0, variant=0):
        _check(_dev.xg_set_copy_params(self._c, chunk, variant), "xg_set_copy_params")

    def p2p_bench(self, nbytes, mode=0, reps=20):
        g, sec = C.c_double(), C.c_double()
        _check(_dev.xg_p2p_bench(self._c, nbytes, mode, reps, C.byref(g), C.byref(sec)), "xg_p2p_bench")
        return g.value, sec.value

    def p2p_split_bench(self, nbytes, calls, reps=20):
        """all pairs, every transfer of `nbytes` posted as `calls` calls -> (GB/s sent, s per rep)"""
        g, sec = C.c_double(), C.c_double()
        _check(_dev.xg_p2p_split_bench(self._c, nbytes, calls, reps, C.byref(g), C.byref(sec)),
               "xg_p2p_split_bench")
        return g.value, sec.value

    def p2p_pair_bench(self, nbytes, peer, reps=10):
        """one link, both directions at once, with `peer` (< 0: idle this round) -> (GB/s sent, s per rep)"""
        g, sec = C.c_double(), C.c_double()
        _check(_dev.xg_p2p_pair_bench(self._c, nbytes, peer, reps, C.byref(g), C.byref(sec)), "xg_p2p_pair_bench")
        return g.value, sec.value

    def ktime_begin(self, max_launches=4096, per_launch=True):
        """per_launch: an event pair around every copy / engine launch; else one pair
        around the whole session on the main stream (launches and bytes counted)."""
        _check(_dev.xg_ktime_begin(self._c, max_launches, 1 if per_launch else 2), "xg_ktime_begin")

    def ktime_end(self):
        ms, n, b = C.c_double(), C.c_int(), C.c_int64()
        _check(_dev.xg_ktime_end(self._c, C.byref(ms), C.byref(n), C.byref(b)), "xg_ktime_end")
        return ms.value, n.value, b.value

    def ktime_launches(self, n):
        """per-launch (ms, algorithmic bytes) of the last kernel-timing session"""
        out = []
        for k in range(n):
            ms, b = C.c_double(), C.c_int64()
            _check(_dev.xg_ktime_launch(self._c, k, C.byref(ms), C.byref(b)), "xg_ktime_launch")
            out.append((ms.value, b.value))
        return out

    def close(self):
        if self._c:
            _check(_dev.xg_finalize(self._c), "xg_finalize")
            self._c = None


def now():
    return device().xg_now()


def run_virtual(runs, rccl=False):
    """Execute the MethodRuns of every GPU of one virtual job (runs[g] on Context.virtual(g, n))
    step by step on one device; returns step_done[] (device seconds).  rccl: move the
    cross-GPU pairs through RCCL (1-rank communicator, self send/recv) instead of copies."""
    n = len(runs)
    arr = (C.c_void_p * n)(*[r._p for r in runs])
    nst = max(1, runs[0].nsteps)
    done = (C.c_double * nst)()
    fn = "xg_vplans_run_rccl" if rccl else "xg_vplans_run"
    _check(getattr(device(), fn)(arr, n, done), fn)
    return list(done)[:runs[0].nsteps]


class Regions:
    """HBM regions (xg_regions_alloc) that several MethodRuns may reuse in turn: at
    hundreds of GiB, allocating and freeing per method costs seconds (the driver
    clears fresh pages), refilling and re-poisoning costs milliseconds."""

    def __init__(self, ctx, region_bytes):
        self.bytes = list(region_bytes)
        rb = (C.c_int64 * NBUF)(*self.bytes)
        self._r = C.c_void_p()
        _check(device().xg_regions_alloc(ctx.handle, rb, C.byref(self._r)), "xg_regions_alloc")

    def fits(self, region_bytes):
        return all(a <= b for a, b in zip(region_bytes, self.bytes))

    def close(self):
        if getattr(self, "_r", None):
            _check(_dev.xg_regions_free(self._r), "xg_regions_free")
            self._r = None


class MethodRun:
    """prepare_*_data + the compiled plan of one method on this GPU:
    HBM regions, fingerprint fill (untimed), plan upload.  regions: a Regions
    object to use (re-poisoned here, not freed by close()) instead of new ones."""

    def __init__(self, ctx, sched, it=0, mode=0, pack_max_seg=4 << 20, regions=None, pack_min=0, pack_form=-1):
        d = device()
        self.ctx, self.sched, self.it, self.mode, self.pack_max_seg = ctx, sched, it, mode, pack_max_seg
        self.pack_min, self.pack_form = pack_min, pack_form
        G, g = ctx.nranks, ctx.rank
        if G > 1 and not getattr(ctx, "is_virtual", False):
            # a real multi-GPU job: refuse, on every rank alike, calls RCCL would not pair
            # step by step, before any rank posts one (xg_devplans_match)
            sched.check_pairing(G, pack_max_seg, pack_min, pack_form, d.xg_self_max(ctx.handle))
        self.view = sched.devplan(G, g, pack_max_seg, pack_min, pack_form)
        self._shared = regions is not None
        if regions is not None:
            if not regions.fits(self.view.region_bytes):
                raise XGError("MethodRun: shared regions too small for this plan")
            self._r = regions._r
            _check(d.xg_regions_poison(self._r), "xg_regions_poison")
        else:
            rb = (C.c_int64 * NBUF)(*self.view.region_bytes)
            self._r = C.c_void_p()
            _check(d.xg_regions_alloc(ctx.handle, rb, C.byref(self._r)), "xg_regions_alloc")
        n = host().xg_fill_runs(sched.handle, G, g, None)
        runs = (SegRun * max(1, n))()
        host().xg_fill_runs(sched.handle, G, g, runs)
        _check(d.xg_fill(self._r, runs, n, sched.d, it, mode), "xg_fill")
        ns = host().xg_verify_slots(sched.handle, G, g, None)
        self._slots = (Slot * max(1, ns))()
        host().xg_verify_slots(sched.handle, G, g, self._slots)
        self.nslots = ns
        self.slots = [(s.src, s.seed, s.dst, s.off) for s in self._slots[:ns]]
        self._p = C.c_void_p()
        _check(d.xg_plan_load(ctx.handle, self._r, self.view.ptr, C.byref(self._p)), "xg_plan_load")
        self.nsteps = d.xg_plan_nsteps(self._p)
        self.set_step_marks(sched.timed_steps())       # as xg_run_method: only the steps a Timer reads
        self.engine_workgroups = d.xg_plan_engine(self._p)   # 0: one launch per step
        self.engine_rails = d.xg_plan_engine_rails(self._p)  # > 0: a solo segment on that many rails

    def run_timed(self):
        """barrier-free timed run; returns (step_done[], step_post[], wall)."""
        n = max(1, self.nsteps)
        done, post, wall = (C.c_double * n)(), (C.c_double * n)(), C.c_double()
        _check(_dev.xg_plan_run(self._p, done, post, C.byref(wall)), "xg_plan_run")
        return list(done)[:self.nsteps], list(post)[:self.nsteps], wall.value

    def enqueue(self):
        _check(_dev.xg_plan_enqueue(self._p), "xg_plan_enqueue")

    def check(self):
        """after a synchronised enqueue(): raise if a step-engine barrier timed out"""
        _check(_dev.xg_plan_check(self._p), "xg_plan_check")

    @property
    def launches(self):
        """kernel launches per run (copy + engine launches)"""
        return _dev.xg_plan_launches(self._p)

    def engine_steps(self):
        """(steps inside engine segments, segments, hazard barriers)"""
        ns, nh = C.c_int(), C.c_int()
        n = _dev.xg_plan_engine_steps(self._p, C.byref(ns), C.byref(nh))
        return n, ns.value, nh.value

    def displs(self):
        """staging displacements of the packed segments, as the device scan computed them"""
        n = _dev.xg_plan_displs(self._p, None, 0)
        out = (C.c_int64 * max(1, n))()
        _check(_dev.xg_plan_displs(self._p, out, n), "xg_plan_displs")
        return list(out)[:n]

    def write(self, buf, off, data):
        """test hook: overwrite bytes of a region"""
        b = C.create_string_buffer(bytes(data), len(data))
        _check(_dev.xg_regions_write(self._r, buf, off, b, len(data)), "xg_regions_write")

    def poison(self):
        _check(_dev.xg_regions_poison(self._r), "xg_regions_poison")

    def set_step_marks(self, need=None):
        """mark only the steps with need[s] set in a timed run (None: every step), the others
        reported as done with the next marked one (xg_plan_set_step_marks)"""
        arr = (C.c_uint8 * max(1, self.nsteps))(*need) if need is not None else None
        _check(_dev.xg_plan_set_step_marks(self._p, arr), "xg_plan_set_step_marks")

    def set_local_only(self, on=True):
        """test hook (virtual GPU): run this GPU's share alone -- copy launches only, its RCCL
        calls and in-loop barriers left out (xg_plan_set_local_only)"""
        _check(_dev.xg_plan_set_local_only(self._p, 1 if on else 0), "xg_plan_set_local_only")

    def verify(self):
        ns = max(1, self.nslots)
        chk, bad, first = (C.c_uint64 * ns)(), (C.c_int64 * ns)(), (C.c_int64 * ns)()
        _check(_dev.xg_verify(self._r, self._slots, self.nslots, self.sched.d, self.it, self.mode,
                              chk, bad, first), "xg_verify")
        return list(chk)[:self.nslots], list(bad)[:self.nslots], list(first)[:self.nslots]

    def read(self, buf, off, length):
        out = C.create_string_buffer(max(1, length))
        _check(_dev.xg_regions_read(self._r, buf, off, out, length), "xg_regions_read")
        return out.raw[:length]

    def close(self):
        if getattr(self, "_p", None):
            _check(_dev.xg_plan_free(self._p), "xg_plan_free")
            self._p = None
        if getattr(self, "_r", None):
            if not self._shared:
                _check(_dev.xg_regions_free(self._r), "xg_regions_free")
            self._r = None
