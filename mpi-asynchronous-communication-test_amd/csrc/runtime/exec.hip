// exec.hip -- execution of a loaded plan: per-step copy launches and RCCL groups, chains of
// stamped launches, engine segments, graph replay, armed (doorbell) runs, step marks.
#include "rt.h"

extern "C" const char *xg_debug_where(void)
{
    static char buf[160];
    snprintf(buf, sizeof buf, "%s: step %d of %d: %s", g_where.fn, g_where.step, g_where.nsteps, g_where.phase);
    return buf;
}

// Execution of one step on GPU g (xg_devplan, built by libxghost):
//   1. one copy_kernel launch over every local gather/scatter piece and every
//      pack into the per-peer staging region                (pre copies)
//   2. one ncclGroupStart .. ncclSend/ncclRecv .. ncclGroupEnd with the <= 7
//      peer GPUs this step talks to (xGMI)                  (p2p)
//   3. one copy_kernel launch unpacking staging into the receive slots (post)
//   4. a clock_kernel stamp (step mark) -- the reference's Waitall boundary
// All on one HIP stream per context, so step s+1 starts after step s; the
// cross-GPU order comes from RCCL send/recv matching.

// step boundary i of a run (-1: its start) on `stream`: a clock stamp (d_gstamp)
int mark(xg_plan *p, int i, hipStream_t stream)
{
    hipLaunchKernelGGL(xgk::clock_kernel, dim3(1), dim3(64), 0, stream, p->d_gstamp + i + 1);
    HIPCHK(hipGetLastError());
    return XG_OK;
}

// the run's step marks, after it: gs[i + 1] = boundary i's stamp, gs[0] the start's
int read_marks(const xg_plan *p, std::vector<unsigned long long> &gs)
{
    gs.resize((size_t)p->nsteps + 1);
    HIPCHK(hipMemcpy(gs.data(), p->d_gstamp, 8 * gs.size(), hipMemcpyDeviceToHost));
    return XG_OK;
}

// seconds from the run's start to boundary i
double mark_elapsed(const xg_plan *p, int i, const std::vector<unsigned long long> &gs)
{
    return (double)(gs[i + 1] - gs[0]) / p->ctx->wall_hz;
}

// Copy kernel per launch.  Variant 0 (default) picks by the launch's bytes: a launch
// whose source + destination exceed the 256 MiB Infinity Cache streams through it with
// non-temporal loads and stores (6.3 TB/s vs 5.5-5.6 plain from 256 MiB up), a smaller
// one keeps the default policy, which re-runs serve from the cache
// (profiles/r02/copy_nt_sizes.txt).  1 / 6 force one form (A/B, tests).
//
// A launch of more than 1.5 x launch_max bytes goes as back-to-back kernel dispatches of
// about launch_max bytes each (its pieces are independent: the same step, a few more
// kernel boundaries).  P256 A32 -d 4 MiB m1 / m2 (one 32 GiB step, 1 M pieces): 12.6 ->
// 11.0 ms at 512 MiB per dispatch, 11.5 at 128 MiB; cutting by piece count instead hurt
// steps of small pieces (profiles/r02/launch_split/).  launch_cuts gives the dispatches
// [first piece, end) of pieces [b, b + n): every count of launches (xg_plan_launches, the
// kernel-timing sessions) counts these dispatches, as rocprofv3 does.
static void launch_cuts(const xg_plan *p, int b, int n, int64_t bytes, std::vector<std::pair<int, int>> &out)
{
    out.clear();
    const int64_t cap = p->ctx->launch_max;
    if (!(cap > 0 && bytes > cap + cap / 2 && (int)p->plen.size() > b + n)) {
        out.push_back({b, b + n});
        return;
    }
    const int64_t *pre = p->plen.data();        // prefix sums of the piece lengths
    for (int o = b; o < b + n;) {
        // the first piece boundary at least cap bytes past o (lower_bound may return b + n + 1
        // when fewer than cap bytes remain: clamp), then no runt dispatch at the end
        int e = (int)(std::lower_bound(pre + o + 1, pre + b + n + 1, pre[o] + cap) - pre);
        if (e > b + n) e = b + n;
        if (b + n - e < 16 || pre[b + n] - pre[e] < cap / 2) e = b + n;
        out.push_back({o, e});
        o = e;
    }
}

int launch_dispatches(const xg_plan *p, int b, int n, int64_t bytes)
{
    std::vector<std::pair<int, int>> cuts;
    launch_cuts(p, b, n, bytes, cuts);
    return (int)cuts.size();
}

static int launch_one(xg_plan *p, int b, int n, int v, hipStream_t st, unsigned long long *start)
{
    const xgk::DCopy *pc = p->d_pieces + b;
    if (v == 1 && p->wave_at[b]) {       // pieces of <= wave_at[b] KiB, 16-B aligned (launch_chunk)
        const int w = std::max(1, std::min(p->ctx->wave_grid, (n + 3) / 4));
        if (p->wave_at[b] == 2)
            hipLaunchKernelGGL((xgk::copy_kernel_w<2>), dim3(w), dim3(xgk::kThreads), 0, st, pc, n, start);
        else if (p->wave_at[b] == 4)
            hipLaunchKernelGGL((xgk::copy_kernel_w<4>), dim3(w), dim3(xgk::kThreads), 0, st, pc, n, start);
        else
            hipLaunchKernelGGL((xgk::copy_kernel_w<xgk::kWaveKiB>), dim3(w), dim3(xgk::kThreads), 0, st, pc, n, start);
    } else if (v == 6) hipLaunchKernelGGL((xgk::copy_kernel_g<4, true>), dim3(n), dim3(xgk::kThreads), 0, st, pc, start);
    else hipLaunchKernelGGL((xgk::copy_kernel_g<4>), dim3(n), dim3(xgk::kThreads), 0, st, pc, start);
    HIPCHK(hipGetLastError());
    return XG_OK;
}

// kernel-timing session bookkeeping around one kernel dispatch of `bytes` copied bytes
static int kt_before(xg_ctx *c, hipStream_t stream, bool *kt)
{
    *kt = c->kt_mode == 1 && 2 * (size_t)c->nk + 1 < c->kev.size();
    if (*kt) HIPCHK(hipEventRecord(c->kev[2 * c->nk], stream));
    return XG_OK;
}

static int kt_after(xg_ctx *c, hipStream_t stream, bool kt, int64_t bytes)
{
    if (kt) {
        HIPCHK(hipEventRecord(c->kev[2 * c->nk + 1], stream));
        c->kbytes[c->nk] = 2 * bytes;      // algorithmic HBM bytes: read + write
    }
    if (kt || c->kt_mode == 2) {
        c->nk++;
        c->kt_bytes += 2 * bytes;
    }
    return XG_OK;
}

// One copy launch of pieces [b, b + n) moving `bytes`, as its dispatches (launch_cuts),
// each bracketed by kernel-timing events when a per-launch session is on.  start: the
// first dispatch stamps its start there (see copy_kernel_g).
static int launch_copy(xg_plan *p, int b, int n, int64_t bytes, hipStream_t st, unsigned long long *start = nullptr,
                       bool reread = false)
{
    const int v = copy_variant(p, bytes, reread);
    if (start && v != 1 && v != 6) return XG_EARG;
    std::vector<std::pair<int, int>> cuts;
    launch_cuts(p, b, n, bytes, cuts);
    int rc;
    for (const auto &q : cuts) {
        const int64_t nb = cuts.size() == 1 ? bytes : p->plen[q.second] - p->plen[q.first];
        bool kt;
        if ((rc = kt_before(p->ctx, st, &kt))) return rc;
        if ((rc = launch_one(p, q.first, q.second - q.first, v, st, q.first == b ? start : nullptr))) return rc;
        if ((rc = kt_after(p->ctx, st, kt, nb))) return rc;
    }
    return XG_OK;
}

// one copy launch, bracketed by kernel-timing events when a per-launch session is on
static int timed_copy(xg_plan *p, int b, int n, int64_t bytes, hipStream_t stream, bool reread = false)
{
    return launch_copy(p, b, n, bytes, stream, nullptr, reread);
}

// step part 1: stage copies, then local gather/scatter + packs.  A split step
// forks its local part onto `side`, where it runs beside the packs and the RCCL
// group on `stream`; enqueue_post joins it back before the step ends.  A fused
// step's first launch also holds the previous step's unpacks: the previous step
// ends with it (its event, when recording, goes right behind it), and the local
// part forks after it, so no message of this step lands before one of the previous.
int enqueue_pre(xg_plan *p, int s, hipStream_t stream, hipStream_t side)
{
    const StepR &st = p->steps[s];
    int rc;
    if (st.stage_n && (rc = timed_copy(p, st.stage_b, st.stage_n, st.stage_bytes, stream, true))) return rc;
    if (st.fused) {
        // the previous step's unpacks, [this step's local copies,] this step's packs: one launch
        const StepR &pv = p->steps[s - 1];
        const int n = pv.post_n + (st.fused_local ? st.local_n : 0) + st.pack_n;
        const int64_t b = pv.post_bytes + (st.fused_local ? st.local_bytes : 0) + st.pack_bytes;
        if ((rc = timed_copy(p, pv.post_b, n, b, stream, true))) return rc;
        if (p->rec_ev && p->need_mark[s - 1] && (rc = mark(p, s - 1, stream))) return rc;
    }
    if (st.split) {
        // the packs feed the RCCL group (the critical path), the local part does not: by default
        // the local part forks after the pack launch, so it overlaps the transfer instead of
        // sharing HBM with the packs (XG_SPLIT_AFTER_PACK=0: both at once, as in round 2)
        const bool pack_here = !st.fused && st.pack_n;
        if (pack_here && p->ctx->split_after_pack &&
            (rc = timed_copy(p, st.pack_b, st.pack_n, st.pack_bytes, stream, true)))
            return rc;
        HIPCHK(hipEventRecord(p->fork[s], stream));
        HIPCHK(hipStreamWaitEvent(side, p->fork[s], 0));
        if ((rc = timed_copy(p, st.local_b, st.local_n, st.local_bytes, side))) return rc;
        HIPCHK(hipEventRecord(p->join[s], side));
        if (pack_here && !p->ctx->split_after_pack &&
            (rc = timed_copy(p, st.pack_b, st.pack_n, st.pack_bytes, stream, true)))
            return rc;
    } else if (!st.fused && st.pre_n &&
               (rc = timed_copy(p, st.local_b, st.pre_n, st.local_bytes + st.pack_bytes, stream,
                                st.pack_n > 0 || st.stage_fused))) {
        return rc;
    }
    return XG_OK;
}

// step part 3: unpack out of staging (unless deferred into the next step's fused
// launch), then wait for the forked local part
int enqueue_post(xg_plan *p, int s, hipStream_t stream)
{
    const StepR &st = p->steps[s];
    int rc;
    if (st.post_n && !st.deferred && (rc = timed_copy(p, st.post_b, st.post_n, st.post_bytes, stream))) return rc;
    if (st.split) HIPCHK(hipStreamWaitEvent(stream, p->join[s], 0));
    return XG_OK;
}

static int enqueue_step(xg_plan *p, int s)
{
    xg_ctx *c = p->ctx;
    const StepR &st = p->steps[s];
    int rc;
    if (c->virt && (st.p2p_n || st.sync_after) && !p->local_only) {
        fprintf(stderr, "xg: a virtual GPU's cross-GPU step runs only through xg_vplans_run\n");
        return XG_EARG;
    }
    if ((rc = enqueue_pre(p, s, c->stream, c->side))) return rc;
    if (p->local_only) return enqueue_post(p, s, c->stream);
    // the step's send/recv calls, in the order libxghost lists them (xg_devplan_step_calls), one
    // group per run of them between fences (a relay step: two, the second forwarding what the
    // first delivered to this GPU's staging -- stream order puts it behind the first); the
    // barrier call, if any, is the step's last and follows the unpacks
    const xg_call *cl = p->calls.data() + st.call_b;
    for (int i = 0; i < st.call_n && st.p2p_n;) {
        int e = i;
        while (e < st.call_n && (cl[e].kind == XG_CALL_SEND || cl[e].kind == XG_CALL_RECV)) ++e;
        if (e > i && (rc = rccl_group(
                          e - i,
                          [&](int k) {
                              const xg_call &o = cl[i + k];
                              uint8_t *ptr = p->reg->ptr[o.buf] + o.off;
                              return o.kind == XG_CALL_SEND
                                         ? ncclSend(ptr, (size_t)o.len, ncclUint8, o.peer, c->comm, c->stream)
                                         : ncclRecv(ptr, (size_t)o.len, ncclUint8, o.peer, c->comm, c->stream);
                          },
                          st.groups > 1 ? "relay step exchange" : "step exchange")))
            return rc;
        i = e + 1;            // past the fence (or the barrier, which ends the list)
    }
    if ((rc = enqueue_post(p, s, c->stream))) return rc;
    if (st.sync_after)   /* in-loop MPI_Barrier: every GPU finishes this step before any goes on */
        NCCLCHK(ncclAllReduce(c->d_red, c->d_red, 1, ncclFloat64, ncclMax, c->comm, c->stream));
    return XG_OK;
}

// one launch of the step engine over segment g (armed: waits for the doorbell `epoch`)
int launch_seg(xg_plan *p, const EngSeg &g, hipStream_t stream, bool armed)
{
    xg_ctx *c = p->ctx;
    int rc;
    if (p->engine_reset) {
        HIPCHK(hipMemsetAsync(p->d_engine, 0, sizeof(xgk::EngineState), stream));
        p->engine_base = 0;
        p->engine_reset = false;
    }
    const int n = g.s1 - g.s0;
    xgk::Doorbell *db = armed ? p->db : nullptr;
    const unsigned epoch = armed ? ++p->epoch : 0;
    const unsigned base = p->engine_base;
    if (!g.solo) p->engine_base += (unsigned)(n + (armed ? 1 : 0)) * (unsigned)g.w;
    bool kt;
    if ((rc = kt_before(c, stream, &kt))) return rc;
    unsigned long long *stamps = reinterpret_cast<unsigned long long *>(p->d_engine + 1) + g.s0;
    const int *sb = p->d_sb + g.sb_off;
    if (g.solo && g.wv == 1 && g.gran == 16)
        hipLaunchKernelGGL((xgk::solo_engine_kernel<xgk::kSoloK, 1>), dim3(g.w), dim3(64), 0, stream,
                           p->d_solo + g.u0, g.npieces, g.sbase, g.dbase, sb, n, p->d_engine, stamps, p->nsteps,
                           db, epoch);
    else if (g.solo && g.wv == 1 && g.gran == 4)
        hipLaunchKernelGGL((xgk::solo_engine_kernel<xgk::kSoloK, 1, 4>), dim3(g.w), dim3(64), 0, stream,
                           p->d_solo + g.u0, g.npieces, g.sbase, g.dbase, sb, n, p->d_engine, stamps, p->nsteps,
                           db, epoch);
    else if (g.solo && g.wv == 1)      // granule 1: 16 registers per piece and lane, half the rows per chunk
        hipLaunchKernelGGL((xgk::solo_engine_kernel<xgk::kSoloK / 2, 1, 1>), dim3(g.w), dim3(64), 0, stream,
                           p->d_solo + g.u0, g.npieces, g.sbase, g.dbase, sb, n, p->d_engine, stamps, p->nsteps,
                           db, epoch);
    else if (g.solo)
        hipLaunchKernelGGL((xgk::solo_engine_kernel<xgk::kSoloK, xgk::kSoloWaves>), dim3(g.w), dim3(xgk::kSoloThreads), 0,
                           stream, p->d_solo + g.u0, g.npieces, g.sbase, g.dbase, sb, n, p->d_engine, stamps, p->nsteps,
                           db, epoch);
    else if (g.b == 1)
        hipLaunchKernelGGL(xgk::step_engine_kernel<1>, dim3(g.w), dim3(xgk::kThreads), 0, stream, p->d_epieces, sb, n,
                           p->d_engine, stamps, base, db, epoch);
    else if (g.b == 4)
        hipLaunchKernelGGL(xgk::step_engine_kernel<4>, dim3(g.w), dim3(xgk::kThreads), 0, stream, p->d_epieces, sb, n,
                           p->d_engine, stamps, base, db, epoch);
    else
        hipLaunchKernelGGL(xgk::step_engine_kernel<16>, dim3(g.w), dim3(xgk::kThreads), 0, stream, p->d_epieces, sb,
                           n, p->d_engine, stamps, base, db, epoch);
    HIPCHK(hipGetLastError());
    return kt_after(c, stream, kt, g.bytes);
}

// every engine step's stamp (wall-clock ticks), after a synchronised run: grid
// segments stamp once per step; a solo segment's rails each stamp the steps they
// closed (0 elsewhere), so a rail's stamp of step t is its latest at or before t
// and the step's is the MAX over rails
static int read_stamps(const xg_plan *p, std::vector<unsigned long long> &st)
{
    const size_t n = (size_t)p->nsteps;
    std::vector<unsigned long long> all(n * p->stamp_rails);
    HIPCHK(hipMemcpy(all.data(), p->d_engine + 1, 8 * all.size(), hipMemcpyDeviceToHost));
    st.assign(all.begin(), all.begin() + n);
    for (const EngSeg &g : p->segs)
        if (g.solo)
            xg_solo_reduce_stamps(reinterpret_cast<const uint64_t *>(all.data()), g.w, (int64_t)n, g.s0, g.s1,
                                  reinterpret_cast<uint64_t *>(st.data()));
    return XG_OK;
}

// after a synchronised run: did an engine workgroup give up at a grid barrier?
// Then the tickets are inconsistent: zero the state before the next launch.
extern "C" int xg_plan_check(xg_plan *p)
{
    if (p->segs.empty()) return XG_OK;
    xgk::EngineState es;
    HIPCHK(hipSetDevice(p->ctx->device));
    HIPCHK(hipStreamSynchronize(p->ctx->stream));
    HIPCHK(hipMemcpy(&es, p->d_engine, sizeof es, hipMemcpyDeviceToHost));
    if (es.tmo) {
        p->engine_reset = true;
        fprintf(stderr, "xg: step engine: a workgroup timed out at a grid barrier (workgroups not co-resident?)\n");
        return XG_EHIP;
    }
    return XG_OK;
}

// step s of this plan as enqueued on (stream, side): an engine segment is one
// launch at its first step and nothing at the others
static int enqueue_unit(xg_plan *p, int s)
{
    const int gi = p->seg_of[s];
    if (gi < 0) return enqueue_step(p, s);
    if (p->segs[gi].s0 != s) return XG_OK;
    return launch_seg(p, p->segs[gi], p->ctx->stream);
}

// Armed run of a one-segment plan: the engine is launched, announces itself
// through the doorbell, and waits; the timed region starts when the host rings
// and ends when the engine reports its last step delivered (system-scope store
// to host memory).  The launch and dispatch latency (several us from an idle
// stream) thus stays outside, like the setup of a persistent MPI request before
// MPI_Start; every byte still moves inside.  Step times: the wall-clock stamps,
// anchored at the host-measured end.
static int run_armed(xg_plan *p, double *step_done, double *step_post, double *wall)
{
    xg_ctx *c = p->ctx;
    const EngSeg &g = p->segs[0];
    int rc;
    if ((rc = launch_seg(p, g, c->stream, true))) return rc;
    const unsigned epoch = p->epoch;
    const double tl = xg_now();
    bool ready;
    while (!(ready = __atomic_load_n(&p->db->ready, __ATOMIC_ACQUIRE) == epoch) && xg_now() - tl < 5.0) {
    }
    const double t0 = xg_now();
    __atomic_store_n(&p->db->ring, epoch, __ATOMIC_RELEASE);
    const double tp = xg_now();
    bool done;
    while (!(done = __atomic_load_n(&p->db->done, __ATOMIC_ACQUIRE) == epoch) && xg_now() - t0 < 10.0) {
    }
    const double t1 = xg_now();
    HIPCHK(hipStreamSynchronize(c->stream));
    if (wall) *wall = xg_now() - t0;
    if ((rc = xg_plan_check(p))) return rc;
    if (!ready || !done) {
        fprintf(stderr, "xg: armed step engine: no %s from the device\n", ready ? "completion" : "ready signal");
        return XG_EHIP;
    }
    if (step_post) {
        step_post[0] = tp - t0;
        for (int s = 1; s < p->nsteps; ++s) step_post[s] = 0;
    }
    if (step_done) {
        std::vector<unsigned long long> st;
        if ((rc = read_stamps(p, st))) return rc;
        const double total = t1 - t0;
        for (int s = 0; s < p->nsteps; ++s) {
            const double x = total - (double)(st[p->nsteps - 1] - st[s]) / c->wall_hz;
            step_done[s] = s == p->nsteps - 1 ? total : (x > 0 ? x : 0);
        }
    }
    return XG_OK;
}

// The timed run's launches: ev0, then every step (a chain's launches stamp the steps'
// completions, an engine segment is one launch), each followed by its step event.
// step_post (may be null): host seconds spent enqueueing each step.
static int enqueue_run(xg_plan *p, double *step_post)
{
    xg_ctx *c = p->ctx;
    int rc;
    if ((rc = mark(p, -1, c->stream))) return rc;
    p->rec_ev = true;
    const bool chains = p->d_cstamp && !c->kt_mode;
    for (int s = 0; s < p->nsteps;) {
        const double tp = xg_now();
        const int gi = p->seg_of[s];
        if (chains && p->chain_end[s]) {
            // a chain: launch t + 1 stamps step t's completion at its start; a clock
            // kernel stamps the last one's, one event after it anchors them all
            const int ce = p->chain_end[s];
            for (int t = s; t < ce; ++t) {
                const double tq = xg_now();
                const StepR &st = p->steps[t];
                // the step's first launch stamps the previous step's completion
                unsigned long long *start = t > s ? p->d_cstamp + t - 1 : nullptr;
                rc = XG_OK;
                if (st.stage_n) {
                    rc = launch_copy(p, st.stage_b, st.stage_n, st.stage_bytes, c->stream, start, true);
                    start = nullptr;
                }
                if (!rc && st.local_n)
                    rc = launch_copy(p, st.local_b, st.local_n, st.local_bytes, c->stream, start, st.stage_fused);
                if (rc) {
                    p->rec_ev = false;
                    return rc;
                }
                if (step_post) step_post[t] = xg_now() - tq;
            }
            hipLaunchKernelGGL(xgk::clock_kernel, dim3(1), dim3(64), 0, c->stream, p->d_cstamp + ce - 1);
            HIPCHK(hipGetLastError());
            if ((rc = mark(p, ce - 1, c->stream))) {
                p->rec_ev = false;
                return rc;
            }
            s = ce;
            continue;
        }
        const int e = gi >= 0 ? p->segs[gi].s1 : s + 1;     // one launch posts a whole segment
        if ((rc = enqueue_unit(p, s))) {
            p->rec_ev = false;
            return rc;
        }
        // a deferred step's unpacks run in the next step's fused launch, which records its event
        if ((gi >= 0 || (!p->steps[s].deferred && p->need_mark[s])) && (rc = mark(p, e - 1, c->stream))) {
            p->rec_ev = false;
            return rc;
        }
        if (step_post) {
            step_post[s] = xg_now() - tp;
            for (int t = s + 1; t < e; ++t) step_post[t] = 0;
        }
        s = e;
    }
    p->rec_ev = false;
    return XG_OK;
}

// graph replay applies: asked for, not inside a kernel-timing session (its per-launch
// events are host bookkeeping), and a plan of more than one launch
static bool use_graph(const xg_plan *p)
{
    const int g = p->ctx->graph;
    return (g == 1 || (g < 0 && p->graph_auto)) && !p->ctx->kt_mode && p->nlaunch > 1 && p->d_gstamp;
}

extern "C" int xg_plan_run(xg_plan *p, double *step_done, double *step_post, double *wall)
{
    xg_ctx *c = p->ctx;
    int rc;
    HIPCHK(hipSetDevice(c->device));
    if (p->db && !c->kt_mode) return run_armed(p, step_done, step_post, wall);
    const bool chains = p->d_cstamp && !c->kt_mode;
    if (use_graph(p) && !p->g_run) {
        // captured once: the grid engine's ticket counter restarts from zero in every replay,
        // the step boundaries are stamps (mark)
        p->engine_reset = true;
        rc = capture(c->stream, &p->g_run, [&] { return enqueue_run(p, nullptr); });
        if (rc) {
            p->engine_reset = true;      // the host's ticket base moved for launches that never ran
            return rc;
        }
    }
    const bool graph = p->g_run && use_graph(p);
    const double t0 = xg_now();
    where("xg_plan_run", 0, p->nsteps, "posting the steps");
    if (graph) {
        HIPCHK(hipGraphLaunch(p->g_run, c->stream));
        // a replay restarts the device ticket counter from zero (the memset captured in the
        // graph) and leaves it at the captured run's count, which the host base does not track:
        // the next eager launch must zero the state again
        p->engine_reset = true;
        if (step_post && p->nsteps > 0) {
            // the whole run is posted by one graph launch: its host time is shared out over the
            // steps in proportion to the request posts this GPU's ranks make in each
            // (xg_stepplan.posts), so xg_sched_rank_timer credits all of it to the ranks that post
            // -- no share lands on a step without posts, where no Timer would read it -- and the
            // shares sum to the launch time (evenly over the steps if nothing is posted)
            const double tl = xg_now() - t0;
            int64_t tot = 0;
            for (int s = 0; s < p->nsteps; ++s) tot += p->steps[s].posts;
            for (int s = 0; s < p->nsteps; ++s)
                step_post[s] = tot > 0 ? tl * p->steps[s].posts / (double)tot : tl / p->nsteps;
        }
    } else if ((rc = enqueue_run(p, step_post))) {
        return rc;
    }
    where("xg_plan_run", p->nsteps, p->nsteps, "waiting for the device (hipStreamSynchronize)");
    HIPCHK(hipStreamSynchronize(c->stream));
    where("idle", -1, 0, "");
    if (wall) *wall = xg_now() - t0;
    if ((rc = xg_plan_check(p))) return rc;
    if (!step_done) return XG_OK;
    std::vector<unsigned long long> st;
    if (!p->segs.empty() && (rc = read_stamps(p, st))) return rc;
    std::vector<unsigned long long> cst, gs;
    if (chains) {
        cst.resize(p->nsteps);
        HIPCHK(hipMemcpy(cst.data(), p->d_cstamp, 8 * (size_t)p->nsteps, hipMemcpyDeviceToHost));
    }
    if ((rc = read_marks(p, gs))) return rc;
    for (int s = 0; s < p->nsteps;) {
        const int gi = p->seg_of[s];
        if (chains && p->chain_end[s]) {
            const int ce = p->chain_end[s];
            const double end = mark_elapsed(p, ce - 1, gs);
            for (int t = s; t < ce; ++t) {
                const double x = end - (double)(cst[ce - 1] - cst[t]) / c->wall_hz;
                step_done[t] = t == ce - 1 ? end : (x > 0 ? x : 0);
            }
            s = ce;
            continue;
        }
        const int e = gi >= 0 ? p->segs[gi].s1 : s + 1;
        if (gi < 0 && !p->need_mark[s]) {     // not marked: the next marked step's time (below)
            step_done[s] = -1;
            s = e;
            continue;
        }
        const double end = mark_elapsed(p, e - 1, gs);
        // inside a segment: the wall-clock stamps, anchored at the mark after its launch
        // (the last step of a segment is drained, so its stamp is a delivered time)
        for (int t = s; t < e; ++t) {
            const double x = end - (double)(st.empty() ? 0 : st[e - 1] - st[t]) / c->wall_hz;
            step_done[t] = t == e - 1 ? end : (x > 0 ? x : 0);
        }
        s = e;
    }
    // an unmarked step is reported as done when the next marked one is: no Timer reads it
    // (xg_sched_timed_steps), and the last step is always marked
    for (int s = p->nsteps - 2; s >= 0; --s)
        if (step_done[s] < 0) step_done[s] = step_done[s + 1];
    return XG_OK;
}

// Which steps an eager or captured run marks with a clock stamp (need[s] != 0; null: all).
// The last step is always marked; captured graphs hold the old marks and are dropped.
extern "C" int xg_plan_set_step_marks(xg_plan *p, const uint8_t *need)
{
    if (!p) return XG_EARG;
    for (int s = 0; s < p->nsteps; ++s) p->need_mark[s] = !need || need[s] || s == p->nsteps - 1;
    for (hipGraphExec_t *g : {&p->g_run, &p->vg.exec})   // captured runs hold the old marks: capture again
        if (*g) {
            HIPCHK(hipGraphExecDestroy(*g));
            *g = nullptr;
        }
    return XG_OK;
}

// Test hook: GPU g of a G-GPU job (a virtual context) runs its own share alone -- every copy
// launch of its plan (stage, local gather/scatter, packs, unpacks) with its RCCL calls and
// in-loop barriers left out, so a share too large to put all G GPUs on one device (configs[4]
// at its stated size: 256 GiB per GPU) still executes, its local slots verifiable.  Refused
// (XG_EARG) for a plan whose local copies travel as self send/recv in an RCCL group
// (XG_SELF_MAX): leaving the group out would drop them.
extern "C" int xg_plan_set_local_only(xg_plan *p, int on)
{
    if (!p || !p->ctx->virt) return XG_EARG;
    for (const StepR &st : p->steps)
        if (on && st.self_local) return XG_EARG;
    p->local_only = on != 0;
    return XG_OK;
}

extern "C" int xg_plan_enqueue(xg_plan *p)
{
    int rc;
    auto body = [&] {
        int r;
        for (int s = 0; s < p->nsteps; ++s)
            if ((r = enqueue_unit(p, s))) return r;
        return XG_OK;
    };
    if (!use_graph(p)) return body();
    if (!p->g_enq) {
        p->engine_reset = true;
        if ((rc = capture(p->ctx->stream, &p->g_enq, body))) {
            p->engine_reset = true;      // the host's ticket base moved for launches that never ran
            return rc;
        }
    }
    HIPCHK(hipGraphLaunch(p->g_enq, p->ctx->stream));
    p->engine_reset = true;          // the replay moved the device counter, not the host base
    return XG_OK;
}

