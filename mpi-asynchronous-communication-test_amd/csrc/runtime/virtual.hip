// virtual.hip -- every GPU of a G-GPU job on one device (xg_init_virtual): the pairs RCCL
// would make of the GPUs' call lists, moved as device copies or as RCCL self send/recv.
#include "rt.h"

// Every GPU of a virtual job (xg_init_virtual), step by step on plans[0]'s
// stream: all pre copies (or a GPU's whole engine segment, at its first step:
// its steps touch only that GPU's regions and hold none of its cross-GPU ops,
// so running them together is what a real GPU does too), then each RCCL
// send/recv pair as one device copy (sends of g to h matched in order with h's
// receives from g -- RCCL's per-peer FIFO inside a group), then all post
// copies, then the step event.  step_done[s] = device seconds from the start to
// the end of step s.
// rccl = true: the same pairs go through RCCL instead -- a 1-rank communicator
// on the device (created once, held by plans[0]'s context), each step's pairs as
// one ncclGroupStart/End of self ncclSend + ncclRecv (matched in issue order),
// and the in-loop barriers as ncclAllReduce: RCCL's p2p and collective calls on
// the real plan buffers, on a box with one GPU.
static int vplans_run(xg_plan *const *plans, int n, double *step_done, bool rccl)
{
    if (!plans || n < 1) return XG_EARG;
    xg_ctx *c0 = plans[0]->ctx;
    const int nst = plans[0]->nsteps;
    for (int g = 0; g < n; ++g) {
        const xg_ctx *c = plans[g]->ctx;
        if (!c->virt || c->nranks != n || c->rank != g || c->device != c0->device || plans[g]->nsteps != nst) {
            fprintf(stderr, "xg_vplans_run: plan %d is not GPU %d of one %d-GPU virtual job\n", g, g, n);
            return XG_EARG;
        }
    }
    int rc;
    hipStream_t st = c0->stream;
    HIPCHK(hipSetDevice(c0->device));
    for (int g = 0; g < n; ++g) HIPCHK(hipStreamSynchronize(plans[g]->ctx->stream));
    if (rccl && !c0->comm) {
        ncclUniqueId id;
        StdoutToStderr quiet;
        NCCLCHK(ncclGetUniqueId(&id));
        NCCLCHK(ncclCommInitRank(&c0->comm, 1, id, 0));
    }
    // RCCL's pairing of every GPU's calls (libxghost, calls.c): the same lists a real rank
    // posts in enqueue_step, paired as RCCL pairs them; refused unless every pair falls in
    // one step with one length and the GPUs agree on the barriers
    std::vector<xg_call_pair> pairs;
    auto pair_calls = [&]() -> int {
        std::vector<const xg_call *> cl(n);
        std::vector<const int32_t *> cb(n);
        for (int g = 0; g < n; ++g) {
            cl[g] = plans[g]->calls.data();
            cb[g] = plans[g]->call_begin.data();
        }
        char err[256];
        const int64_t np = xg_calls_match(n, nst, cl.data(), cb.data(), nullptr, 0, err, sizeof err);
        if (np < 0) {
            fprintf(stderr, "xg_vplans_run: the GPUs' RCCL calls do not pair: %s\n", err);
            return XG_EARG;
        }
        pairs.resize((size_t)np + 1);
        xg_calls_match(n, nst, cl.data(), cb.data(), pairs.data(), np, err, sizeof err);
        pairs.resize((size_t)np);
        return XG_OK;
    };
    // the job's launches, RCCL groups and step events on plans[0]'s stream
    auto body = [&]() -> int {
        if ((rc = mark(plans[0], -1, st))) return rc;
        size_t q0 = 0;
        for (int s = 0; s < nst; ++s) {
            where(rccl ? "xg_vplans_run_rccl" : "xg_vplans_run", s, nst, "posting the pre copies");
            for (int g = 0; g < n; ++g) {
                xg_plan *pg = plans[g];
                const int gi = pg->seg_of[s];
                if (gi < 0) rc = enqueue_pre(pg, s, st, pg->ctx->side);
                else rc = pg->segs[gi].s0 == s ? launch_seg(pg, pg->segs[gi], st) : XG_OK;
                if (rc) return rc;
            }
            size_t q1 = q0;
            while (q1 < pairs.size() && pairs[q1].step == s) ++q1;
            auto ends = [&](const xg_call_pair &q, uint8_t **src, uint8_t **dst) {
                const xg_call &sc = plans[q.src]->calls[q.send_call], &rcv = plans[q.dst]->calls[q.recv_call];
                *src = plans[q.src]->reg->ptr[sc.buf] + sc.off;
                *dst = plans[q.dst]->reg->ptr[rcv.buf] + rcv.off;
            };
            if (!rccl) {
                for (size_t q = q0; q < q1; ++q) {
                    uint8_t *src, *dst;
                    ends(pairs[q], &src, &dst);
                    if (pairs[q].len) HIPCHK(hipMemcpyAsync(dst, src, (size_t)pairs[q].len, hipMemcpyDeviceToDevice, st));
                }
            } else {
                where("xg_vplans_run_rccl", s, nst, "posting the RCCL group (ncclGroupEnd)");
                // every pair of one group of the step (pairs come in (step, group) order; a relay
                // step has two) as a self send + receive in ONE RCCL group (issue order = pair order)
                for (size_t g0 = q0; g0 < q1;) {
                    size_t g1 = g0;
                    while (g1 < q1 && pairs[g1].group == pairs[g0].group) ++g1;
                    if ((rc = rccl_group(
                             (int)(2 * (g1 - g0)),
                             [&](int i) {
                                 uint8_t *src, *dst;
                                 const xg_call_pair &q = pairs[g0 + i / 2];
                                 ends(q, &src, &dst);
                                 return i % 2 == 0 ? ncclSend(src, (size_t)q.len, ncclUint8, 0, c0->comm, st)
                                                   : ncclRecv(dst, (size_t)q.len, ncclUint8, 0, c0->comm, st);
                             },
                             "virtual job step")))
                        return rc;
                    g0 = g1;
                }
            }
            q0 = q1;
            for (int g = 0; g < n; ++g)
                if (plans[g]->seg_of[s] < 0 && (rc = enqueue_post(plans[g], s, st))) return rc;
            if (rccl && plans[0]->steps[s].sync_after)
                NCCLCHK(ncclAllReduce(c0->d_red, c0->d_red, 1, ncclFloat64, ncclMax, c0->comm, st));
            if (plans[0]->need_mark[s] && (rc = mark(plans[0], s, st))) return rc;   // the job's marks: GPU 0's
        }
        return XG_OK;
    };
    if (c0->graph == 1 && !c0->kt_mode) {
        // XG_GRAPH=1: the job captured once (per set of plans and transport) and replayed
        std::vector<uint64_t> ids(n);
        for (int g = 0; g < n; ++g) ids[g] = plans[g]->id;
        xg_plan::VGraph &vg = plans[0]->vg;
        if (!vg.exec || vg.ids != ids || vg.rccl != rccl) {
            if (vg.exec) HIPCHK(hipGraphExecDestroy(vg.exec));
            vg.exec = nullptr;
            if ((rc = pair_calls())) return rc;
            for (int g = 0; g < n; ++g) plans[g]->engine_reset = true;
            rc = capture(st, &vg.exec, body);
            for (int g = 0; g < n; ++g)
                if (rc) plans[g]->engine_reset = true;   // ticket bases moved for launches that never ran
            if (rc) return rc;
            vg.ids = ids;
            vg.rccl = rccl;
        }
        HIPCHK(hipGraphLaunch(vg.exec, st));
        for (int g = 0; g < n; ++g) plans[g]->engine_reset = true;   // device counters moved by the replay
    } else if ((rc = pair_calls()) || (rc = body())) {
        return rc;
    }
    where(rccl ? "xg_vplans_run_rccl" : "xg_vplans_run", nst, nst, "waiting for the device (hipStreamSynchronize)");
    HIPCHK(hipStreamSynchronize(st));
    where("idle", -1, 0, "");
    for (int g = 0; g < n; ++g)
        if ((rc = xg_plan_check(plans[g]))) return rc;
    if (step_done) {
        std::vector<unsigned long long> gs;
        if ((rc = read_marks(plans[0], gs))) return rc;
        for (int s = nst - 1; s >= 0; --s)      // an unmarked step: done with the next marked one
            step_done[s] = plans[0]->need_mark[s] ? mark_elapsed(plans[0], s, gs) : step_done[s + 1];
    }
    return XG_OK;
}

extern "C" int xg_vplans_run(xg_plan *const *plans, int n, double *step_done)
{
    return vplans_run(plans, n, step_done, false);
}

extern "C" int xg_vplans_run_rccl(xg_plan *const *plans, int n, double *step_done)
{
    return vplans_run(plans, n, step_done, true);
}

