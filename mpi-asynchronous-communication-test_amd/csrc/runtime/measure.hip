// measure.hip -- kernel-timing sessions (HIP events around copy launches or a whole region)
// and the RCCL p2p microbenchmark (the rccl-tests sendrecv / pt2pt_test analogue).
#include "rt.h"

// mode 1: an event pair around every copy / engine launch (max_launches of them);
// mode 2: one pair around the whole session on the main stream, launches counted
extern "C" int xg_ktime_begin(xg_ctx *c, int max_launches, int mode)
{
    if (mode != 1 && mode != 2) return XG_EARG;
    if (mode == 1 && max_launches < 1) return XG_EARG;
    HIPCHK(hipSetDevice(c->device));
    const size_t need = mode == 1 ? 2 * (size_t)max_launches : 2;
    while (c->kev.size() < need) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        c->kev.push_back(e);
    }
    c->kbytes.resize(mode == 1 ? max_launches : 0);
    c->nk = 0;
    c->kt_bytes = 0;
    c->kt_mode = mode;
    if (mode == 2) HIPCHK(hipEventRecord(c->kev[0], c->stream));
    return XG_OK;
}

extern "C" int xg_ktime_end(xg_ctx *c, double *total_ms, int *launches, int64_t *bytes)
{
    double tot = 0;
    const int mode = c->kt_mode;
    c->kt_mode = 0;
    if (mode == 2) HIPCHK(hipEventRecord(c->kev[1], c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (mode == 2) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, c->kev[0], c->kev[1]));
        tot = ms;
    } else {
        for (int k = 0; k < c->nk; ++k) {
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, c->kev[2 * k], c->kev[2 * k + 1]));
            tot += ms;
        }
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = c->nk;
    if (bytes) *bytes = c->kt_bytes;
    return XG_OK;
}

extern "C" int xg_ktime_launch(xg_ctx *c, int k, double *ms, int64_t *bytes)
{
    if (k < 0 || k >= c->nk || c->kt_mode || (int)c->kbytes.size() <= k) return XG_EARG;
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, c->kev[2 * k], c->kev[2 * k + 1]));
    if (ms) *ms = t;
    if (bytes) *bytes = c->kbytes[k];
    return XG_OK;
}

// ------------------------------------------------------------------ microbenchmark: RCCL p2p ceiling
// This rank's benchmark buffers (`bytes` each way; 0: an idle rank), then agreement over the
// communicator that every rank has its buffers before any rank posts a call: a rank that failed
// its allocation alone and returned would leave its partners in ncclSend / ncclRecv forever
// (the timing events are made here too, for the same reason).
// Every rank of the job calls this (a MAX all-reduce of the failure flag).
static int bench_buffers(xg_ctx *c, DevMem &sb, DevMem &rb, EventPair &ev, int64_t bytes)
{
    double bad = 0;
    if (bytes > 0) {
        if (hipMalloc(&sb.p, bytes) != hipSuccess || hipMalloc(&rb.p, bytes) != hipSuccess ||
            hipMemsetAsync(sb.p, c->rank & 0xff, bytes, c->stream) != hipSuccess ||
            hipEventCreate(&ev.e[0]) != hipSuccess || hipEventCreate(&ev.e[1]) != hipSuccess) {
            fprintf(stderr, "xg: rank %d: %lld B of p2p benchmark buffers not allocated\n", c->rank, (long long)bytes);
            (void)hipGetLastError();
            bad = 1;
        }
    }
    if (c->nranks > 1 && !c->virt) {
        const int rc = xg_allreduce_max(c, &bad, 1);
        if (rc) return rc;
    }
    return bad ? XG_ENOMEM : XG_OK;
}

// The rccl-tests sendrecv analogue (and the GPU version of pt2pt_test,
// mpi_sendrecv_test.c:15-74).  mode 0: all pairs (every rank sends `bytes` to
// every other rank, one group); mode 1: ring (send to r+1, receive from r-1);
// mode 2: one direction 1 -> 0 (pt2pt_test's Issend/Irecv pair), other ranks idle.
// calls > 1: every (rank, peer) transfer posted as `calls` consecutive ncclSend / ncclRecv of
// 16-B aligned cuts of it (xg_p2p_split_bench: RCCL's per-call cost inside a group).
// *gbps = bytes this rank sent (mode 2: received on rank 0) per second; *sec = seconds per rep.
static int p2p_bench(xg_ctx *c, int64_t bytes, int mode, int calls, int reps, double *gbps, double *sec)
{
    const int n = c->nranks, r = c->rank;
    const bool self = n == 1 && c->comm && !c->virt;      // XG_SELF_COMM: rank 0 sends to itself
    if ((n < 2 && !self) || bytes <= 0 || reps < 1 || mode < 0 || mode > 2 || calls < 1 || calls > 4096)
        return XG_EARG;
    HIPCHK(hipSetDevice(c->device));
    const int npeer = self ? 1 : (mode == 0 ? n - 1 : 1);
    DevMem m_sb, m_rb;                  // freed, and the events destroyed, on every return path
    EventPair ev;
    int rc = bench_buffers(c, m_sb, m_rb, ev, bytes * npeer);
    if (rc) return rc;
    uint8_t *sb = m_sb.as<uint8_t>(), *rb = m_rb.as<uint8_t>();
    // this rank's calls of one repetition: (send?, peer, offset into sb / rb, length)
    struct Op { bool send; int peer; int64_t off, len; };
    std::vector<Op> ops;
    auto both = [&](int to, int from, int64_t off) {
        for (int k = 0; k < calls; ++k) {           // cut k of the transfer: [cut(k), cut(k + 1))
            const int64_t a = k ? (bytes * k / calls) & ~(int64_t)15 : 0;
            const int64_t b = k + 1 < calls ? (bytes * (k + 1) / calls) & ~(int64_t)15 : bytes;
            if (b <= a) continue;
            if (to >= 0) ops.push_back({true, to, off + a, b - a});
            if (from >= 0) ops.push_back({false, from, off + a, b - a});
        }
    };
    if (self) {
        both(0, 0, 0);
    } else if (mode == 0) {
        for (int k = 1; k < n; ++k) both((r + k) % n, (r - k + n) % n, (int64_t)(k - 1) * bytes);
    } else if (mode == 1) {
        both((r + 1) % n, (r - 1 + n) % n, 0);
    } else if (r == 1) {
        both(0, -1, 0);
    } else if (r == 0) {
        both(-1, 1, 0);
    }
    auto one = [&]() -> int {
        return rccl_group(
            (int)ops.size(),
            [&](int i) {
                const Op &o = ops[i];
                return o.send ? ncclSend(sb + o.off, (size_t)o.len, ncclUint8, o.peer, c->comm, c->stream)
                              : ncclRecv(rb + o.off, (size_t)o.len, ncclUint8, o.peer, c->comm, c->stream);
            },
            "xg_p2p_bench");
    };
    for (int w = 0; w < 2 && !rc; ++w) rc = one();          // connection set-up + warm-up
    if (!rc) rc = xg_barrier(c);
    if (rc) return rc;
    HIPCHK(hipEventRecord(ev.e[0], c->stream));
    for (int k = 0; k < reps && !rc; ++k) rc = one();
    HIPCHK(hipEventRecord(ev.e[1], c->stream));
    HIPCHK(hipEventSynchronize(ev.e[1]));
    if (rc) return rc;
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ev.e[0], ev.e[1]));
    const double s_rep = ms * 1e-3 / reps;
    if (sec) *sec = s_rep;
    if (gbps) *gbps = (mode == 2 && !self ? (r < 2 ? (double)bytes : 0.0) : (double)bytes * npeer) / s_rep / 1e9;
    return XG_OK;
}

extern "C" int xg_p2p_bench(xg_ctx *c, int64_t bytes, int mode, int reps, double *gbps, double *sec)
{
    return p2p_bench(c, bytes, mode, 1, reps, gbps, sec);
}

extern "C" int xg_p2p_split_bench(xg_ctx *c, int64_t bytes, int calls, int reps, double *gbps, double *sec)
{
    return p2p_bench(c, bytes, 0, calls, reps, gbps, sec);
}


extern "C" int xg_p2p_pair_bench(xg_ctx *c, int64_t bytes, int peer, int reps, double *gbps, double *sec)
{
    if (bytes <= 0 || reps < 1 || c->virt || !c->comm || peer >= c->nranks) return XG_EARG;
    if (gbps) *gbps = 0;
    if (sec) *sec = 0;
    const bool idle = peer < 0 || peer == c->rank;         // idle this round (still agrees below)
    HIPCHK(hipSetDevice(c->device));
    DevMem m_sb, m_rb;
    EventPair ev;
    int rc = bench_buffers(c, m_sb, m_rb, ev, idle ? 0 : bytes);
    if (rc || idle) return rc;
    uint8_t *sb = m_sb.as<uint8_t>(), *rb = m_rb.as<uint8_t>();
    auto one = [&]() -> int {
        return rccl_group(
            2,
            [&](int i) {
                return i == 0 ? ncclSend(sb, (size_t)bytes, ncclUint8, peer, c->comm, c->stream)
                              : ncclRecv(rb, (size_t)bytes, ncclUint8, peer, c->comm, c->stream);
            },
            "xg_p2p_pair_bench");
    };
    for (int w = 0; w < 2 && !rc; ++w) rc = one();          // connection set-up + warm-up
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipEventRecord(ev.e[0], c->stream));
    for (int k = 0; k < reps && !rc; ++k) rc = one();
    HIPCHK(hipEventRecord(ev.e[1], c->stream));
    HIPCHK(hipEventSynchronize(ev.e[1]));
    if (rc) return rc;
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ev.e[0], ev.e[1]));
    const double s_rep = ms * 1e-3 / reps;
    if (sec) *sec = s_rep;
    if (gbps) *gbps = (double)bytes / s_rep / 1e9;
    return XG_OK;
}
