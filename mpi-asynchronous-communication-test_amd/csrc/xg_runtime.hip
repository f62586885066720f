// xg_runtime.hip -- device half of the C-ABI (include/xg.h): HBM regions,
// kernel launches, grouped RCCL exchange, step timing.  gfx950 only.
//
// Execution of one step on GPU g (xg_devplan, built by libxghost):
//   1. one copy_kernel launch over every local gather/scatter piece and every
//      pack into the per-peer staging region                (pre copies)
//   2. one ncclGroupStart .. ncclSend/ncclRecv .. ncclGroupEnd with the <= 7
//      peer GPUs this step talks to (xGMI)                  (p2p)
//   3. one copy_kernel launch unpacking staging into the receive slots (post)
//   4. hipEventRecord(step event)     -- the reference's Waitall boundary
// All on one HIP stream per context, so step s+1 starts after step s; the
// cross-GPU order comes from RCCL send/recv matching.
#include <hip/hip_runtime.h>
#include <unistd.h>
#include <rccl/rccl.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <vector>

#include "kernels.h"
#include "xg.h"

#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "xg: HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__,   \
                    __LINE__, #x);                                                                 \
            return XG_EHIP;                                                                        \
        }                                                                                          \
    } while (0)

#define NCCLCHK(x)                                                                                 \
    do {                                                                                           \
        ncclResult_t r_ = (x);                                                                     \
        if (r_ != ncclSuccess) {                                                                   \
            fprintf(stderr, "xg: RCCL error %s at %s:%d: %s\n", ncclGetErrorString(r_), __FILE__, \
                    __LINE__, #x);                                                                 \
            return XG_ERCCL;                                                                       \
        }                                                                                          \
    } while (0)

struct xg_ctx {
    int rank, nranks, device;
    bool virt;              // xg_init_virtual: one of nranks GPUs emulated on one device, no RCCL
    hipStream_t stream;
    hipStream_t side;       // local gather/scatter of a step that also talks to other GPUs (overlaps RCCL)
    ncclComm_t comm;
    double *d_red;          // device scratch for barrier / MAX reductions
    int64_t chunk;          // bytes per copy workgroup
    int64_t engine_max_step;   // GPU-local plans whose largest step moves <= this many bytes use the step engine
    int engine_wmax;           // at most this many (co-resident) engine workgroups
    int engine_drain;          // 1: always drain before each barrier arrival (XG_ENGINE_DRAIN=1)
    double wall_hz;            // wall_clock64() rate
    int variant;            // copy kernel variant
    // kernel timing session (xg_ktime_begin/end)
    bool kt_on;
    int nk;
    std::vector<hipEvent_t> kev;   // start/end pairs per copy launch
    std::vector<int64_t> kbytes;   // algorithmic bytes (read + write) per launch
};

struct xg_regions {
    xg_ctx *ctx;
    uint8_t *ptr[XG_NBUF];
    int64_t bytes[XG_NBUF];
};

struct StepR {
    // pre = [local gather/scatter pieces | pack-into-staging pieces], one launch
    // unless the step also has cross-GPU ops: then the local part runs on the side
    // stream beside the RCCL group and only the packs precede it (split).
    int stage_b, stage_n, pre_b, pre_n, local_n, post_b, post_n, p2p_b, p2p_n, sync_after;
    int64_t stage_bytes, local_bytes, pack_bytes, post_bytes;   // bytes copied by each launch (read + written once)
    bool split;
};

struct xg_plan {
    xg_ctx *ctx;
    xg_regions *reg;
    int nsteps;
    xgk::DCopy *d_pieces;
    int npieces;
    std::vector<StepR> steps;
    std::vector<xg_p2p> p2p;
    std::vector<hipEvent_t> ev;
    std::vector<hipEvent_t> fork, join;   // per split step: main -> side, side -> main
    hipEvent_t ev0;
    int variant;
    // step engine (one persistent launch for the whole plan), or engine_w == 0
    int engine_w;
    int engine_b;                  // 16-B loads per lane per unit (1, 4, 16)
    int *d_step_begin;             // nsteps + 1 unit offsets, then nsteps drain flags
    xgk::DCopy *d_epieces;         // the engine's work units, step-major
    int engine_ndrain;             // steps whose barrier arrival waits for the stores (engine_drains)
    xgk::EngineState *d_engine;    // state (16 B, zeroed at load) followed by nsteps stamps
    unsigned engine_base;          // barrier tickets taken by earlier launches (wraps)
    bool engine_reset;             // zero the state before the next launch
    int64_t engine_bytes;          // bytes copied per run
};

extern "C" double xg_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// ------------------------------------------------------------------ context
// RCCL writes its log -- and, under NCCL_DEBUG=WARN/VERSION, a version banner at
// communicator creation -- to stdout unless NCCL_DEBUG_FILE says otherwise; stdout
// here carries the reference's report (bin/test, bin/pt2pt_test) and bench.py's JSON
// line, so send RCCL's output to stderr unless the user chose a file.  Called before
// every first RCCL call (RCCL reads the variable when it first logs).
static void rccl_log_to_stderr()
{
    if (!getenv("NCCL_DEBUG_FILE")) setenv("NCCL_DEBUG_FILE", "/dev/stderr", 0);
}

// RCCL 2.27 also prints a version banner (RCCL/HIP/ROCm version, host, library path)
// straight to stdout when it creates a communicator: fd 1 points at fd 2 for that call.
struct StdoutToStderr {
    int saved;
    StdoutToStderr() : saved(-1)
    {
        fflush(stdout);
        saved = dup(1);
        if (saved >= 0) dup2(2, 1);
    }
    ~StdoutToStderr()
    {
        fflush(stdout);
        if (saved >= 0) {
            dup2(saved, 1);
            close(saved);
        }
    }
};

extern "C" int xg_get_unique_id(void *uid)
{
    rccl_log_to_stderr();
    StdoutToStderr quiet;
    ncclUniqueId id;
    static_assert(sizeof(ncclUniqueId) == XG_UNIQUE_ID_BYTES, "unique id size");
    NCCLCHK(ncclGetUniqueId(&id));
    memcpy(uid, &id, sizeof id);
    return XG_OK;
}

extern "C" int xg_init(xg_ctx **out, int rank, int nranks, int device, const void *uid)
{
    int ndev = 0;
    if (!out || nranks < 1 || rank < 0 || rank >= nranks) return XG_EARG;
    HIPCHK(hipGetDeviceCount(&ndev));
    if (device >= ndev && ndev > 0 && nranks > 1) {
        // a launcher that narrows each rank's view (HIP_VISIBLE_DEVICES per rank) leaves
        // fewer visible GPUs than the local rank index
        fprintf(stderr, "xg: device %d not visible (%d visible): using device %d\n", device, ndev, device % ndev);
        device %= ndev;
    }
    if (device < 0 || device >= ndev) {
        fprintf(stderr, "xg: device %d not present (%d visible)\n", device, ndev);
        return XG_EARG;
    }
    HIPCHK(hipSetDevice(device));
    xg_ctx *c = new xg_ctx();
    c->rank = rank; c->nranks = nranks; c->device = device; c->comm = nullptr; c->virt = false;
    c->chunk = 32768; c->variant = 5; c->kt_on = false; c->nk = 0;   // measured best: profiles/r01_copy_ab.txt
    const char *env = getenv("XG_COPY_CHUNK");
    if (env && atol(env) >= 4096) c->chunk = atol(env) & ~(int64_t)15;
    env = getenv("XG_COPY_VARIANT");
    if (env) c->variant = atoi(env);
    c->engine_max_step = 16 << 20;    // crossover vs one launch per step: profiles/r01_engine_sweep.txt
    env = getenv("XG_ENGINE_MAX_STEP");      // 0: never use the step engine
    if (env) c->engine_max_step = atol(env);
    env = getenv("XG_ENGINE_WG");
    c->engine_wmax = env && atoi(env) > 0 ? atoi(env) : 256;    // one per CU
    if (c->engine_wmax > 1024) c->engine_wmax = 1024;
    env = getenv("XG_ENGINE_DRAIN");         // "1": drain every step even without a hazard
    c->engine_drain = env && !strcmp(env, "1");
    {
        int khz = 0;
        HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
        c->wall_hz = khz > 0 ? khz * 1e3 : 1e8;
    }
    HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    HIPCHK(hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    HIPCHK(hipMalloc(&c->d_red, 64 * sizeof(double)));
    rccl_log_to_stderr();
    if (nranks > 1) {
        ncclUniqueId id;
        if (!uid) return XG_EARG;
        memcpy(&id, uid, sizeof id);
        StdoutToStderr quiet;
        NCCLCHK(ncclCommInitRank(&c->comm, nranks, id, rank));
    } else if (getenv("XG_SELF_COMM") && atoi(getenv("XG_SELF_COMM"))) {
        // test hook: a 1-rank communicator, so the RCCL send/recv paths (xg_p2p_bench,
        // bin/pt2pt_test) run as self send/recv on a one-GPU box
        ncclUniqueId id;
        StdoutToStderr quiet;
        NCCLCHK(ncclGetUniqueId(&id));
        NCCLCHK(ncclCommInitRank(&c->comm, 1, id, 0));
    }
    *out = c;
    return XG_OK;
}

// GPU `rank` of an `nranks`-GPU job, emulated on physical `device` inside this
// process: same regions, plans and kernels as a real rank, no communicator.
// Its cross-GPU ops are executed only by xg_vplans_run (all GPUs of the job
// together), which moves each RCCL send/recv pair as a device copy.
extern "C" int xg_init_virtual(xg_ctx **out, int rank, int nranks, int device)
{
    int rc = xg_init(out, 0, 1, device, nullptr);
    if (rc) return rc;
    if (nranks < 1 || rank < 0 || rank >= nranks) {
        xg_finalize(*out);
        *out = nullptr;
        return XG_EARG;
    }
    (*out)->rank = rank;
    (*out)->nranks = nranks;
    (*out)->virt = true;
    return XG_OK;
}

extern "C" int xg_finalize(xg_ctx *c)
{
    if (!c) return XG_OK;
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->comm) NCCLCHK(ncclCommDestroy(c->comm));
    for (auto &e : c->kev) HIPCHK(hipEventDestroy(e));
    HIPCHK(hipFree(c->d_red));
    HIPCHK(hipStreamSynchronize(c->side));
    HIPCHK(hipStreamDestroy(c->side));
    HIPCHK(hipStreamDestroy(c->stream));
    delete c;
    return XG_OK;
}

extern "C" int xg_rank(const xg_ctx *c) { return c->rank; }
extern "C" int xg_nranks(const xg_ctx *c) { return c->nranks; }

extern "C" int xg_sync(xg_ctx *c)
{
    HIPCHK(hipStreamSynchronize(c->stream));
    return XG_OK;
}

extern "C" int xg_device_sync(xg_ctx *c)
{
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipDeviceSynchronize());
    return XG_OK;
}

extern "C" int xg_allreduce_max(xg_ctx *c, double *vals, int n)
{
    if (n < 0) return XG_EARG;
    if (c->nranks == 1 || n == 0 || c->virt) return XG_OK;   // virtual: one process holds every GPU
    double *buf = c->d_red;
    if (n > 64) HIPCHK(hipMalloc(&buf, sizeof(double) * n));
    HIPCHK(hipMemcpyAsync(buf, vals, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    NCCLCHK(ncclAllReduce(buf, buf, n, ncclFloat64, ncclMax, c->comm, c->stream));
    HIPCHK(hipMemcpyAsync(vals, buf, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (buf != c->d_red) HIPCHK(hipFree(buf));
    return XG_OK;
}

extern "C" int xg_barrier(xg_ctx *c)
{
    HIPCHK(hipStreamSynchronize(c->stream));
    if (c->nranks > 1 && !c->virt) {
        NCCLCHK(ncclAllReduce(c->d_red, c->d_red, 1, ncclFloat64, ncclMax, c->comm, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    return XG_OK;
}

extern "C" int xg_device_info(xg_ctx *c, char *name, size_t namelen, int *cus, size_t *hbm)
{
    hipDeviceProp_t p;
    HIPCHK(hipGetDeviceProperties(&p, c->device));
    if (name && namelen) { strncpy(name, p.gcnArchName, namelen - 1); name[namelen - 1] = 0; }
    if (cus) *cus = p.multiProcessorCount;
    if (hbm) *hbm = p.totalGlobalMem;
    return XG_OK;
}

extern "C" int xg_set_copy_params(xg_ctx *c, int64_t chunk, int variant)
{
    if (chunk >= 4096) c->chunk = chunk & ~(int64_t)15;
    if (variant >= 0) c->variant = variant;
    return XG_OK;
}

// ------------------------------------------------------------------ regions
extern "C" int xg_regions_alloc(xg_ctx *c, const int64_t bytes[XG_NBUF], xg_regions **out)
{
    HIPCHK(hipSetDevice(c->device));
    xg_regions *r = new xg_regions();
    r->ctx = c;
    for (int i = 0; i < XG_NBUF; ++i) {
        r->bytes[i] = bytes[i];
        r->ptr[i] = nullptr;
        if (bytes[i] > 0) {
            hipError_t e = hipMalloc(&r->ptr[i], (size_t)bytes[i]);
            if (e != hipSuccess) {
                fprintf(stderr, "xg: hipMalloc(%lld) for region %d failed: %s\n", (long long)bytes[i], i,
                        hipGetErrorString(e));
                for (int j = 0; j < i; ++j) (void)hipFree(r->ptr[j]);
                delete r;
                return XG_ENOMEM;
            }
        }
    }
    *out = r;
    return xg_regions_poison(r);
}

extern "C" int xg_regions_poison(xg_regions *r)
{
    if (r->bytes[XG_BUF_RECV] > 0)
        HIPCHK(hipMemsetAsync(r->ptr[XG_BUF_RECV], 0xA5, (size_t)r->bytes[XG_BUF_RECV], r->ctx->stream));
    if (r->bytes[XG_BUF_SCRATCH] > 0)   /* TAM aggregation buffers start zeroed (gaps stay deterministic) */
        HIPCHK(hipMemsetAsync(r->ptr[XG_BUF_SCRATCH], 0, (size_t)r->bytes[XG_BUF_SCRATCH], r->ctx->stream));
    HIPCHK(hipStreamSynchronize(r->ctx->stream));
    return XG_OK;
}

extern "C" int xg_regions_free(xg_regions *r)
{
    if (!r) return XG_OK;
    HIPCHK(hipStreamSynchronize(r->ctx->stream));
    for (int i = 0; i < XG_NBUF; ++i)
        if (r->ptr[i]) HIPCHK(hipFree(r->ptr[i]));
    delete r;
    return XG_OK;
}

extern "C" void *xg_regions_ptr(xg_regions *r, int buf) { return buf >= 0 && buf < XG_NBUF ? r->ptr[buf] : nullptr; }

extern "C" int xg_regions_read(xg_regions *r, int buf, int64_t off, void *host, int64_t len)
{
    if (buf < 0 || buf >= XG_NBUF || off < 0 || len < 0 || off + len > r->bytes[buf]) return XG_EARG;
    HIPCHK(hipMemcpyAsync(host, r->ptr[buf] + off, (size_t)len, hipMemcpyDeviceToHost, r->ctx->stream));
    HIPCHK(hipStreamSynchronize(r->ctx->stream));
    return XG_OK;
}

// ------------------------------------------------------------------ fill / verify
extern "C" int xg_fill(xg_regions *r, const xg_segrun *runs, int nruns, int64_t d, int iter, int mode)
{
    xg_ctx *c = r->ctx;
    std::vector<xgk::DSeg> segs;
    for (int i = 0; i < nruns; ++i)
        for (int k = 0; k < runs[i].nsegs; ++k) {
            xgk::DSeg s;
            s.off = runs[i].off + (int64_t)k * d;
            s.rank = runs[i].rank;
            s.seed = runs[i].seed0 + k;
            if (s.off < 0 || s.off + d > r->bytes[XG_BUF_SEND]) {
                fprintf(stderr, "xg_fill: segment outside the send region\n");
                return XG_EARG;
            }
            segs.push_back(s);
        }
    if (segs.empty() || d == 0) return XG_OK;
    const int64_t chunk = 65536;
    const int64_t cps = (d + chunk - 1) / chunk;
    if ((int64_t)segs.size() * cps > 0x7fffffff) return XG_EARG;
    xgk::DSeg *dsegs;
    HIPCHK(hipMalloc(&dsegs, sizeof(xgk::DSeg) * segs.size()));
    HIPCHK(hipMemcpyAsync(dsegs, segs.data(), sizeof(xgk::DSeg) * segs.size(), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(xgk::fill_kernel, dim3((unsigned)(segs.size() * cps)), dim3(xgk::kThreads), 0, c->stream,
                       r->ptr[XG_BUF_SEND], dsegs, (int)cps, d, chunk, iter, mode);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipFree(dsegs));
    return XG_OK;
}

extern "C" int xg_verify(xg_regions *r, const xg_slot *slots, int nslots, int64_t d, int iter, int mode,
                         uint64_t *chk, int64_t *bad, int64_t *first_bad)
{
    xg_ctx *c = r->ctx;
    if (nslots <= 0) return XG_OK;
    std::vector<xgk::DSlot> sl(nslots);
    for (int i = 0; i < nslots; ++i) {
        sl[i].off = slots[i].off; sl[i].src = slots[i].src; sl[i].seed = slots[i].seed;
        if (sl[i].off < 0 || sl[i].off + d > r->bytes[XG_BUF_RECV]) return XG_EARG;
    }
    const int64_t chunk = 65536;
    const int64_t cps = d > 0 ? (d + chunk - 1) / chunk : 1;
    xgk::DSlot *dsl;
    unsigned long long *dout;
    HIPCHK(hipMalloc(&dsl, sizeof(xgk::DSlot) * nslots));
    HIPCHK(hipMalloc(&dout, sizeof(unsigned long long) * 3 * nslots));
    HIPCHK(hipMemcpyAsync(dsl, sl.data(), sizeof(xgk::DSlot) * nslots, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemsetAsync(dout, 0, sizeof(unsigned long long) * 2 * nslots, c->stream));
    HIPCHK(hipMemsetAsync(dout + 2 * nslots, 0xff, sizeof(unsigned long long) * nslots, c->stream));
    if (d > 0) {
        hipLaunchKernelGGL(xgk::verify_kernel, dim3((unsigned)(nslots * cps)), dim3(xgk::kThreads), 0, c->stream,
                           r->ptr[XG_BUF_RECV], dsl, (int)cps, d, chunk, iter, mode, dout, dout + nslots,
                           dout + 2 * nslots);
        HIPCHK(hipGetLastError());
    }
    std::vector<unsigned long long> h(3 * (size_t)nslots);
    HIPCHK(hipMemcpyAsync(h.data(), dout, sizeof(unsigned long long) * 3 * nslots, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipFree(dsl));
    HIPCHK(hipFree(dout));
    const uint64_t lenk = 0xD6E8FEB86659FD93ull * (uint64_t)d;
    for (int i = 0; i < nslots; ++i) {
        if (chk) chk[i] = h[i] + lenk;
        if (bad) bad[i] = (int64_t)h[nslots + i];
        if (first_bad) first_bad[i] = h[2 * nslots + i] == ~0ull ? -1 : (int64_t)h[2 * nslots + i];
    }
    return XG_OK;
}

// ------------------------------------------------------------------ plans
// Per-step drain flags of the step engine: flag[t] = 1 makes every workgroup wait
// for its stores (vmcnt 0) before arriving at step t's barrier, which completes
// every store issued up to step t.  Step t drains when step t+1 writes or reads
// bytes that a step since the previous drain wrote (the same receive slots
// rewritten by the next -k repetition, typically: one drain per repetition);
// the last step always drains (its stamp anchors every step time).  force: all.
static std::vector<int> engine_drains(const std::vector<std::vector<xgk::DCopy>> &xfer, bool force)
{
    const int n = (int)xfer.size();
    std::vector<int> fl(n, force ? 1 : 0);
    std::vector<std::pair<uintptr_t, uintptr_t>> pend;     // writes since the last drain, sorted
    std::vector<uintptr_t> pmax;                             // prefix max of their ends
    auto hits = [&](uintptr_t a, uintptr_t b) {              // does [a, b) meet a pending write?
        const size_t i = std::lower_bound(pend.begin(), pend.end(), std::make_pair(b, (uintptr_t)0)) - pend.begin();
        return i > 0 && pmax[i - 1] > a;
    };
    for (int u = 1; u < n && !force; ++u) {
        const size_t m = pend.size();
        for (const xgk::DCopy &x : xfer[u - 1])
            if (x.len > 0) pend.push_back({(uintptr_t)x.dst, (uintptr_t)x.dst + (uintptr_t)x.len});
        std::sort(pend.begin() + m, pend.end());
        std::inplace_merge(pend.begin(), pend.begin() + m, pend.end());
        pmax.resize(pend.size());
        for (size_t i = 0; i < pend.size(); ++i) pmax[i] = std::max(i ? pmax[i - 1] : 0, pend[i].second);
        bool hit = false;
        for (const xgk::DCopy &x : xfer[u])
            if (x.len > 0 && (hits((uintptr_t)x.dst, (uintptr_t)x.dst + (uintptr_t)x.len) ||
                              hits((uintptr_t)x.src, (uintptr_t)x.src + (uintptr_t)x.len))) {
                hit = true;
                break;
            }
        if (hit) {
            fl[u - 1] = 1;
            pend.clear();
        }
    }
    if (n) fl[n - 1] = 1;
    return fl;
}

extern "C" int xg_plan_load(xg_ctx *c, xg_regions *r, const xg_devplan *dp, xg_plan **out)
{
    if (!c || !r || !dp || !out) return XG_EARG;
    if (dp->ngpus != c->nranks || dp->gpu != c->rank) {
        fprintf(stderr, "xg_plan_load: plan for gpu %d/%d loaded on rank %d/%d\n", dp->gpu, dp->ngpus, c->rank,
                c->nranks);
        return XG_EARG;
    }
    for (int i = 0; i < XG_NBUF; ++i)
        if (dp->region_bytes[i] > r->bytes[i]) {
            fprintf(stderr, "xg_plan_load: region %d too small (%lld < %lld)\n", i, (long long)r->bytes[i],
                    (long long)dp->region_bytes[i]);
            return XG_EARG;
        }
    HIPCHK(hipSetDevice(c->device));
    xg_plan *p = new xg_plan();
    p->ctx = c; p->reg = r; p->nsteps = dp->nsteps; p->variant = c->variant;
    // one piece per workgroup, c->chunk bytes (32 KiB: profiles/r01_copy_ab.txt); smaller
    // pieces for small launches were measured no faster, and slower where they stop
    // dividing the segment size (profiles/r01_min_pieces_ab.txt)
    const int64_t chunk = c->chunk;
    std::vector<xgk::DCopy> pieces;
    auto add = [&](const xg_copy &cp) -> bool {
        if (cp.len <= 0) return true;
        if (cp.src_buf < 0 || cp.src_buf >= XG_NBUF || cp.dst_buf < 0 || cp.dst_buf >= XG_NBUF) return false;
        if (cp.src_off < 0 || cp.dst_off < 0 || cp.src_off + cp.len > r->bytes[cp.src_buf] ||
            cp.dst_off + cp.len > r->bytes[cp.dst_buf])
            return false;
        for (int64_t o = 0; o < cp.len; o += chunk) {
            xgk::DCopy d;
            d.src = r->ptr[cp.src_buf] + cp.src_off + o;
            d.dst = r->ptr[cp.dst_buf] + cp.dst_off + o;
            d.len = cp.len - o < chunk ? cp.len - o : chunk;
            pieces.push_back(d);
        }
        return true;
    };
    p->steps.resize(dp->nsteps);
    for (int s = 0; s < dp->nsteps; ++s) {
        const xg_stepplan &sp = dp->steps[s];
        StepR &st = p->steps[s];
        if (sp.stage_count < 0 || sp.stage_count > sp.pre_count) goto bad;
        st.stage_b = (int)pieces.size();
        for (int i = 0; i < sp.stage_count; ++i)
            if (!add(dp->copies[sp.pre_begin + i])) goto bad;
        st.stage_n = (int)pieces.size() - st.stage_b;
        st.stage_bytes = 0;
        for (int i = st.stage_b; i < st.stage_b + st.stage_n; ++i) st.stage_bytes += pieces[i].len;
        st.pre_b = (int)pieces.size();
        st.local_bytes = st.pack_bytes = 0;
        for (int i = sp.stage_count; i < sp.pre_count; ++i) {
            const xg_copy &cp = dp->copies[sp.pre_begin + i];
            const bool pack = cp.dst_buf == XG_BUF_STAGE_SEND;   // the plan lists local copies, then packs
            const int before = (int)pieces.size();
            if (!pack && st.pack_bytes) goto bad;
            if (!add(cp)) goto bad;
            for (int k = before; k < (int)pieces.size(); ++k) (pack ? st.pack_bytes : st.local_bytes) += pieces[k].len;
            if (!pack) st.local_n = (int)pieces.size() - st.pre_b;
        }
        st.pre_n = (int)pieces.size() - st.pre_b;
        if (!st.local_bytes) st.local_n = 0;
        st.post_b = (int)pieces.size();
        for (int i = 0; i < sp.post_count; ++i)
            if (!add(dp->copies[sp.post_begin + i])) goto bad;
        st.post_n = (int)pieces.size() - st.post_b;
        st.post_bytes = 0;
        for (int i = st.post_b; i < st.post_b + st.post_n; ++i) st.post_bytes += pieces[i].len;
        st.p2p_b = (int)p->p2p.size();
        for (int i = 0; i < sp.p2p_count; ++i) {
            const xg_p2p &o = dp->p2p[sp.p2p_begin + i];
            if (o.peer < 0 || o.peer >= c->nranks || o.peer == c->rank || o.buf < 0 || o.buf >= XG_NBUF || o.off < 0 ||
                o.off + o.len > r->bytes[o.buf])
                goto bad;
            p->p2p.push_back(o);
        }
        st.p2p_n = (int)p->p2p.size() - st.p2p_b;
        st.sync_after = sp.sync_after && c->nranks > 1;
        st.split = st.p2p_n > 0 && st.local_n > 0;
    }
    p->npieces = (int)pieces.size();
    p->d_pieces = nullptr;
    if (p->npieces) {
        HIPCHK(hipMalloc(&p->d_pieces, sizeof(xgk::DCopy) * pieces.size()));
        HIPCHK(hipMemcpy(p->d_pieces, pieces.data(), sizeof(xgk::DCopy) * pieces.size(), hipMemcpyHostToDevice));
    }
    p->ev.resize(dp->nsteps);
    for (auto &e : p->ev) HIPCHK(hipEventCreate(&e));
    p->fork.assign(dp->nsteps, nullptr);
    p->join.assign(dp->nsteps, nullptr);
    for (int s = 0; s < dp->nsteps; ++s)
        if (p->steps[s].split) {
            HIPCHK(hipEventCreateWithFlags(&p->fork[s], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&p->join[s], hipEventDisableTiming));
        }
    HIPCHK(hipEventCreate(&p->ev0));
    p->engine_w = 0; p->d_step_begin = nullptr; p->d_epieces = nullptr; p->d_engine = nullptr; p->engine_bytes = 0;
    {
        bool ok = !c->virt && c->engine_max_step > 0 && p->nsteps >= 2;
        for (const StepR &st : p->steps)
            ok = ok && !st.p2p_n && !st.sync_after && !st.stage_n && !st.post_n &&
                 st.local_bytes + st.pack_bytes <= c->engine_max_step;
        if (ok) {
            // the engine's work units: the step's transfers (chunk-sized pieces re-joined) cut
            // to B * 4 KiB, one burst of B 16-B loads per lane per workgroup visit.  B grows
            // with the largest step so a step spreads over up to ~256 workgroups with bytes
            // enough in flight (profiles/r01_engine_sweep.txt: small units starve big steps,
            // big units leave small steps on a handful of workgroups).  One workgroup for a
            // whole plan of tiny steps (workgroup barrier instead of the grid barrier) was
            // measured 2x slower per step: profiles/r01_engine_wg_probe.txt, r01_engine_sweep.txt
            int64_t maxstep = 0;
            for (const StepR &st : p->steps)
                if (st.local_bytes + st.pack_bytes > maxstep) maxstep = st.local_bytes + st.pack_bytes;
            std::vector<std::vector<xgk::DCopy>> xfer(p->nsteps);
            for (int s = 0; s < p->nsteps; ++s) {
                const StepR &st = p->steps[s];
                for (int i = st.pre_b; i < st.pre_b + st.pre_n;) {
                    const uint8_t *src = pieces[i].src;
                    uint8_t *dst = pieces[i].dst;
                    int64_t len = pieces[i].len;
                    for (++i; i < st.pre_b + st.pre_n && pieces[i].src == src + len && pieces[i].dst == dst + len; ++i)
                        len += pieces[i].len;
                    xfer[s].push_back({src, dst, len});
                }
                p->engine_bytes += st.local_bytes + st.pack_bytes;
            }
            auto cut = [&](int64_t unit, std::vector<xgk::DCopy> &ep, std::vector<int> &sb) -> int {
                int maxu = 0;
                ep.clear();
                sb.assign(p->nsteps + 1, 0);
                for (int s = 0; s < p->nsteps; ++s) {
                    sb[s] = (int)ep.size();
                    for (const xgk::DCopy &x : xfer[s])
                        for (int64_t o = 0; o < x.len; o += unit)
                            ep.push_back({x.src + o, x.dst + o, x.len - o < unit ? x.len - o : unit});
                    if ((int)ep.size() - sb[s] > maxu) maxu = (int)ep.size() - sb[s];
                }
                sb[p->nsteps] = (int)ep.size();
                return maxu;
            };
            std::vector<xgk::DCopy> ep;
            std::vector<int> sb;
            p->engine_b = maxstep <= (1 << 20) ? 1 : (maxstep <= (4 << 20) ? 4 : 16);
            const int maxu = cut((int64_t)p->engine_b * xgk::kThreads * 16, ep, sb);
            p->engine_w = maxu < 1 ? 1 : (maxu > c->engine_wmax ? c->engine_wmax : maxu);
            const std::vector<int> fl = engine_drains(xfer, c->engine_drain);  // after the step begins
            p->engine_ndrain = 0;
            for (int f : fl) p->engine_ndrain += f;
            sb.insert(sb.end(), fl.begin(), fl.end());
            HIPCHK(hipMalloc(&p->d_step_begin, sizeof(int) * sb.size()));
            HIPCHK(hipMemcpy(p->d_step_begin, sb.data(), sizeof(int) * sb.size(), hipMemcpyHostToDevice));
            if (!ep.empty()) {
                HIPCHK(hipMalloc(&p->d_epieces, sizeof(xgk::DCopy) * ep.size()));
                HIPCHK(hipMemcpy(p->d_epieces, ep.data(), sizeof(xgk::DCopy) * ep.size(), hipMemcpyHostToDevice));
            }
            HIPCHK(hipMalloc(&p->d_engine, sizeof(xgk::EngineState) + 8 * (size_t)p->nsteps));
            HIPCHK(hipMemset(p->d_engine, 0, sizeof(xgk::EngineState)));
            p->engine_base = 0;
            p->engine_reset = false;
        }
    }
    *out = p;
    return XG_OK;
bad:
    fprintf(stderr, "xg_plan_load: copy or p2p descriptor outside its region\n");
    delete p;
    return XG_EARG;
}

extern "C" int xg_plan_free(xg_plan *p)
{
    if (!p) return XG_OK;
    HIPCHK(hipStreamSynchronize(p->ctx->stream));
    if (p->d_pieces) HIPCHK(hipFree(p->d_pieces));
    HIPCHK(hipStreamSynchronize(p->ctx->side));
    if (p->d_step_begin) HIPCHK(hipFree(p->d_step_begin));
    if (p->d_epieces) HIPCHK(hipFree(p->d_epieces));
    if (p->d_engine) HIPCHK(hipFree(p->d_engine));
    for (auto &e : p->ev) HIPCHK(hipEventDestroy(e));
    for (auto &e : p->fork) if (e) HIPCHK(hipEventDestroy(e));
    for (auto &e : p->join) if (e) HIPCHK(hipEventDestroy(e));
    HIPCHK(hipEventDestroy(p->ev0));
    delete p;
    return XG_OK;
}

extern "C" int xg_plan_nsteps(const xg_plan *p) { return p->nsteps; }
extern "C" int xg_plan_engine(const xg_plan *p) { return p->engine_w; }

static int launch_copy(xg_plan *p, int b, int n, hipStream_t st)
{
    const xgk::DCopy *pc = p->d_pieces + b;
    switch (p->variant) {
    case 1: hipLaunchKernelGGL((xgk::copy_kernel<4, true>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 2: hipLaunchKernelGGL((xgk::copy_kernel<8, false>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 3: hipLaunchKernelGGL((xgk::copy_kernel<8, true>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 4: hipLaunchKernelGGL((xgk::copy_kernel<2, false>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 5: hipLaunchKernelGGL((xgk::copy_kernel_g<4>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 6: hipLaunchKernelGGL((xgk::copy_kernel_g<2>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 7: hipLaunchKernelGGL((xgk::copy_kernel_g<4, 1, 0>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 8: hipLaunchKernelGGL((xgk::copy_kernel_g<4, 1, 1>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 9: hipLaunchKernelGGL((xgk::copy_kernel_g<4, 0, 1>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 10: hipLaunchKernelGGL((xgk::copy_kernel_g<8>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 11: hipLaunchKernelGGL((xgk::copy_kernel_g<8, 1, 1>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 12: hipLaunchKernelGGL((xgk::copy_kernel_b<8>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 13: hipLaunchKernelGGL((xgk::copy_kernel_b<4>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    case 0: hipLaunchKernelGGL((xgk::copy_kernel<4, false>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    default: hipLaunchKernelGGL((xgk::copy_kernel_g<4>), dim3(n), dim3(xgk::kThreads), 0, st, pc); break;
    }
    HIPCHK(hipGetLastError());
    return XG_OK;
}

// one copy launch, bracketed by kernel-timing events when a session is on
static int timed_copy(xg_plan *p, int b, int n, int64_t bytes, hipStream_t stream)
{
    xg_ctx *c = p->ctx;
    int rc;
    const bool kt = c->kt_on && 2 * (size_t)c->nk + 1 < c->kev.size();
    if (kt) HIPCHK(hipEventRecord(c->kev[2 * c->nk], stream));
    if ((rc = launch_copy(p, b, n, stream))) return rc;
    if (kt) {
        HIPCHK(hipEventRecord(c->kev[2 * c->nk + 1], stream));
        c->kbytes[c->nk] = 2 * bytes;      // algorithmic HBM bytes: read + write
        c->nk++;
    }
    return XG_OK;
}

// step part 1: stage copies, then local gather/scatter + packs.  A split step
// forks its local part onto `side`, where it runs beside the packs and the RCCL
// group on `stream`; enqueue_post joins it back before the step ends.
static int enqueue_pre(xg_plan *p, int s, hipStream_t stream, hipStream_t side)
{
    const StepR &st = p->steps[s];
    int rc;
    if (st.stage_n && (rc = timed_copy(p, st.stage_b, st.stage_n, st.stage_bytes, stream))) return rc;
    if (st.split) {
        HIPCHK(hipEventRecord(p->fork[s], stream));
        HIPCHK(hipStreamWaitEvent(side, p->fork[s], 0));
        if ((rc = timed_copy(p, st.pre_b, st.local_n, st.local_bytes, side))) return rc;
        HIPCHK(hipEventRecord(p->join[s], side));
        if (st.pre_n > st.local_n &&
            (rc = timed_copy(p, st.pre_b + st.local_n, st.pre_n - st.local_n, st.pack_bytes, stream)))
            return rc;
    } else if (st.pre_n && (rc = timed_copy(p, st.pre_b, st.pre_n, st.local_bytes + st.pack_bytes, stream))) {
        return rc;
    }
    return XG_OK;
}

// step part 3: unpack out of staging, then wait for the forked local part
static int enqueue_post(xg_plan *p, int s, hipStream_t stream)
{
    const StepR &st = p->steps[s];
    int rc;
    if (st.post_n && (rc = timed_copy(p, st.post_b, st.post_n, st.post_bytes, stream))) return rc;
    if (st.split) HIPCHK(hipStreamWaitEvent(stream, p->join[s], 0));
    return XG_OK;
}

static int enqueue_step(xg_plan *p, int s)
{
    xg_ctx *c = p->ctx;
    const StepR &st = p->steps[s];
    int rc;
    if (c->virt && (st.p2p_n || st.sync_after)) {
        fprintf(stderr, "xg: a virtual GPU's cross-GPU step runs only through xg_vplans_run\n");
        return XG_EARG;
    }
    if ((rc = enqueue_pre(p, s, c->stream, c->side))) return rc;
    if (st.p2p_n) {
        NCCLCHK(ncclGroupStart());
        for (int i = 0; i < st.p2p_n; ++i) {
            const xg_p2p &o = p->p2p[st.p2p_b + i];
            uint8_t *ptr = p->reg->ptr[o.buf] + o.off;
            if (o.is_send)
                NCCLCHK(ncclSend(ptr, (size_t)o.len, ncclUint8, o.peer, c->comm, c->stream));
            else
                NCCLCHK(ncclRecv(ptr, (size_t)o.len, ncclUint8, o.peer, c->comm, c->stream));
        }
        NCCLCHK(ncclGroupEnd());
    }
    if ((rc = enqueue_post(p, s, c->stream))) return rc;
    if (st.sync_after)   /* in-loop MPI_Barrier: every GPU finishes this step before any goes on */
        NCCLCHK(ncclAllReduce(c->d_red, c->d_red, 1, ncclFloat64, ncclMax, c->comm, c->stream));
    return XG_OK;
}

// one launch of the step engine (state zeroed first); timed as one copy launch
static int launch_engine(xg_plan *p)
{
    xg_ctx *c = p->ctx;
    if (p->engine_reset) {
        HIPCHK(hipMemsetAsync(p->d_engine, 0, sizeof(xgk::EngineState), c->stream));
        p->engine_base = 0;
    }
    const unsigned base = p->engine_base;
    p->engine_base += (unsigned)p->nsteps * (unsigned)p->engine_w;
    const bool kt = c->kt_on && 2 * (size_t)c->nk + 1 < c->kev.size();
    if (kt) HIPCHK(hipEventRecord(c->kev[2 * c->nk], c->stream));
    unsigned long long *stamps = reinterpret_cast<unsigned long long *>(p->d_engine + 1);
    if (p->engine_b == 1)
        hipLaunchKernelGGL(xgk::step_engine_kernel<1>, dim3(p->engine_w), dim3(xgk::kThreads), 0, c->stream,
                           p->d_epieces, p->d_step_begin, p->nsteps, p->d_engine, stamps, base);
    else if (p->engine_b == 4)
        hipLaunchKernelGGL(xgk::step_engine_kernel<4>, dim3(p->engine_w), dim3(xgk::kThreads), 0, c->stream,
                           p->d_epieces, p->d_step_begin, p->nsteps, p->d_engine, stamps, base);
    else
        hipLaunchKernelGGL(xgk::step_engine_kernel<16>, dim3(p->engine_w), dim3(xgk::kThreads), 0, c->stream,
                           p->d_epieces, p->d_step_begin, p->nsteps, p->d_engine, stamps, base);
    HIPCHK(hipGetLastError());
    if (kt) {
        HIPCHK(hipEventRecord(c->kev[2 * c->nk + 1], c->stream));
        c->kbytes[c->nk] = 2 * p->engine_bytes;
        c->nk++;
    }
    return XG_OK;
}

// after a synchronised engine run: per-step completion times from the wall-clock
// stamps, anchored at the stream events around the launch
static int engine_times(xg_plan *p, double *step_done)
{
    std::vector<unsigned long long> h(2 + (size_t)p->nsteps);
    HIPCHK(hipMemcpy(h.data(), p->d_engine, sizeof(xgk::EngineState) + 8 * (size_t)p->nsteps, hipMemcpyDeviceToHost));
    const xgk::EngineState *es = reinterpret_cast<const xgk::EngineState *>(h.data());
    if (es->tmo) {
        p->engine_reset = true;        // the tickets are inconsistent now: zero before every launch
        fprintf(stderr, "xg: step engine: a workgroup timed out at a grid barrier (workgroups not co-resident?)\n");
        return XG_EHIP;
    }
    if (step_done) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, p->ev0, p->ev[p->nsteps - 1]));
        const unsigned long long *st = h.data() + 2;
        const double total = ms * 1e-3, last = (double)st[p->nsteps - 1];
        for (int s = 0; s < p->nsteps; ++s) {
            const double t = total - (last - (double)st[s]) / p->ctx->wall_hz;
            step_done[s] = t > 0 ? t : 0;
        }
    }
    return XG_OK;
}

extern "C" int xg_plan_run(xg_plan *p, double *step_done, double *step_post, double *wall)
{
    xg_ctx *c = p->ctx;
    int rc;
    HIPCHK(hipSetDevice(c->device));
    if (p->engine_w) {
        const double t0 = xg_now();
        HIPCHK(hipEventRecord(p->ev0, c->stream));
        if ((rc = launch_engine(p))) return rc;
        HIPCHK(hipEventRecord(p->ev[p->nsteps - 1], c->stream));
        if (step_post) {               // one launch posts every step
            step_post[0] = xg_now() - t0;
            for (int s = 1; s < p->nsteps; ++s) step_post[s] = 0;
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        if (wall) *wall = xg_now() - t0;
        return engine_times(p, step_done);
    }
    const double t0 = xg_now();
    HIPCHK(hipEventRecord(p->ev0, c->stream));
    for (int s = 0; s < p->nsteps; ++s) {
        const double tp = xg_now();
        if ((rc = enqueue_step(p, s))) return rc;
        HIPCHK(hipEventRecord(p->ev[s], c->stream));
        if (step_post) step_post[s] = xg_now() - tp;
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    if (wall) *wall = xg_now() - t0;
    if (step_done)
        for (int s = 0; s < p->nsteps; ++s) {
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, p->ev0, p->ev[s]));
            step_done[s] = ms * 1e-3;
        }
    return XG_OK;
}

extern "C" int xg_plan_enqueue(xg_plan *p)
{
    int rc;
    if (p->engine_w) return launch_engine(p);
    for (int s = 0; s < p->nsteps; ++s)
        if ((rc = enqueue_step(p, s))) return rc;
    return XG_OK;
}

// Every GPU of a virtual job (xg_init_virtual), step by step on plans[0]'s
// stream: all pre copies, then each RCCL send/recv pair as one device copy
// (sends of g to h matched in order with h's receives from g -- RCCL's
// per-peer FIFO inside a group), then all post copies, then the step event.
// step_done[s] = device seconds from the start to the end of step s.
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
    HIPCHK(hipEventRecord(plans[0]->ev0, st));
    std::vector<std::vector<const xg_p2p *>> sends((size_t)n * n), recvs((size_t)n * n);
    for (int s = 0; s < nst; ++s) {
        for (int g = 0; g < n; ++g)
            if ((rc = enqueue_pre(plans[g], s, st, plans[g]->ctx->side))) return rc;
        for (auto &v : sends) v.clear();
        for (auto &v : recvs) v.clear();
        for (int g = 0; g < n; ++g) {
            const StepR &sr = plans[g]->steps[s];
            for (int i = 0; i < sr.p2p_n; ++i) {
                const xg_p2p &o = plans[g]->p2p[sr.p2p_b + i];
                if (o.is_send) sends[(size_t)g * n + o.peer].push_back(&o);
                else recvs[(size_t)o.peer * n + g].push_back(&o);
            }
        }
        bool grouped = false;
        for (int g = 0; g < n; ++g)
            for (int h = 0; h < n; ++h) {
                const auto &sv = sends[(size_t)g * n + h], &rv = recvs[(size_t)g * n + h];
                if (sv.size() != rv.size()) {
                    fprintf(stderr, "xg_vplans_run: step %d: GPU %d posts %zu sends to %d, which posts %zu receives\n",
                            s, g, sv.size(), h, rv.size());
                    return XG_EARG;
                }
                for (size_t k = 0; k < sv.size(); ++k) {
                    if (sv[k]->len != rv[k]->len) {
                        fprintf(stderr, "xg_vplans_run: step %d: %d->%d op %zu: send %lld B, receive %lld B\n", s,
                                g, h, k, (long long)sv[k]->len, (long long)rv[k]->len);
                        return XG_EARG;
                    }
                    if (!sv[k]->len) continue;
                    uint8_t *dst = plans[h]->reg->ptr[rv[k]->buf] + rv[k]->off;
                    uint8_t *src = plans[g]->reg->ptr[sv[k]->buf] + sv[k]->off;
                    if (!rccl) {
                        HIPCHK(hipMemcpyAsync(dst, src, (size_t)sv[k]->len, hipMemcpyDeviceToDevice, st));
                        continue;
                    }
                    if (!grouped) {
                        NCCLCHK(ncclGroupStart());
                        grouped = true;
                    }
                    NCCLCHK(ncclSend(src, (size_t)sv[k]->len, ncclUint8, 0, c0->comm, st));
                    NCCLCHK(ncclRecv(dst, (size_t)rv[k]->len, ncclUint8, 0, c0->comm, st));
                }
            }
        if (grouped) NCCLCHK(ncclGroupEnd());
        for (int g = 0; g < n; ++g)
            if ((rc = enqueue_post(plans[g], s, st))) return rc;
        if (rccl && plans[0]->steps[s].sync_after)
            NCCLCHK(ncclAllReduce(c0->d_red, c0->d_red, 1, ncclFloat64, ncclMax, c0->comm, st));
        HIPCHK(hipEventRecord(plans[0]->ev[s], st));
    }
    HIPCHK(hipStreamSynchronize(st));
    if (step_done)
        for (int s = 0; s < nst; ++s) {
            float ms = 0;
            HIPCHK(hipEventElapsedTime(&ms, plans[0]->ev0, plans[0]->ev[s]));
            step_done[s] = ms * 1e-3;
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

extern "C" int xg_ktime_begin(xg_ctx *c, int max_launches)
{
    if (max_launches < 1) return XG_EARG;
    HIPCHK(hipSetDevice(c->device));
    while (c->kev.size() < 2 * (size_t)max_launches) {
        hipEvent_t e;
        HIPCHK(hipEventCreate(&e));
        c->kev.push_back(e);
    }
    c->kbytes.resize(max_launches);
    c->nk = 0;
    c->kt_on = true;
    return XG_OK;
}

extern "C" int xg_ktime_end(xg_ctx *c, double *total_ms, int *launches, int64_t *bytes)
{
    double tot = 0;
    int64_t b = 0;
    c->kt_on = false;
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int k = 0; k < c->nk; ++k) {
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, c->kev[2 * k], c->kev[2 * k + 1]));
        tot += ms;
        b += c->kbytes[k];
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = c->nk;
    if (bytes) *bytes = b;
    return XG_OK;
}

extern "C" int xg_ktime_launch(xg_ctx *c, int k, double *ms, int64_t *bytes)
{
    if (k < 0 || k >= c->nk || c->kt_on) return XG_EARG;
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, c->kev[2 * k], c->kev[2 * k + 1]));
    if (ms) *ms = t;
    if (bytes) *bytes = c->kbytes[k];
    return XG_OK;
}

// ------------------------------------------------------------------ microbenchmark: HBM copy ceiling
// kind 0: grid-stride float4 copy (the canonical copy), grid = 256 CUs x 8 blocks
// kind 1: copy_kernel<4> over 64 KiB pieces (the exchange's default)
// kind 2: span_copy_kernel<4>, 2048 workgroups, equal contiguous byte ranges
// gbps = 2 * bytes / average time (read + write)
extern "C" int xg_copy_ceiling(xg_ctx *c, int64_t bytes, int kind, int reps, double *gbps)
{
    HIPCHK(hipSetDevice(c->device));
    bytes &= ~(int64_t)65535;
    if (bytes <= 0 || reps < 1) return XG_EARG;
    uint8_t *a, *b;
    HIPCHK(hipMalloc(&a, bytes));
    HIPCHK(hipMalloc(&b, bytes));
    HIPCHK(hipMemsetAsync(a, 1, bytes, c->stream));
    std::vector<xgk::DCopy> pieces;
    for (int64_t o = 0; o < bytes; o += 65536) pieces.push_back({a + o, b + o, 65536});
    xgk::DCopy *dp;
    xgk::DSpan sp = {a, b, bytes, 0}, *ds;
    HIPCHK(hipMalloc(&dp, sizeof(xgk::DCopy) * pieces.size()));
    HIPCHK(hipMemcpy(dp, pieces.data(), sizeof(xgk::DCopy) * pieces.size(), hipMemcpyHostToDevice));
    HIPCHK(hipMalloc(&ds, sizeof sp));
    HIPCHK(hipMemcpy(ds, &sp, sizeof sp, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    const int nb = 2048;
    const int64_t per = ((bytes + nb - 1) / nb + 4095) & ~(int64_t)4095;
    for (int r = -2; r < reps; ++r) {          // 2 warm-up launches
        if (r == 0) HIPCHK(hipEventRecord(e0, c->stream));
        if (kind == 0)
            hipLaunchKernelGGL(xgk::gridstride_copy_kernel, dim3(nb), dim3(xgk::kThreads), 0, c->stream,
                               (const uint4 *)a, (uint4 *)b, bytes / 16);
        else if (kind == 1)
            hipLaunchKernelGGL((xgk::copy_kernel<4, false>), dim3((unsigned)pieces.size()), dim3(xgk::kThreads), 0,
                               c->stream, dp);
        else if (kind == 2)
            hipLaunchKernelGGL((xgk::span_copy_kernel<4>), dim3(nb), dim3(xgk::kThreads), 0, c->stream, ds, 1, bytes,
                               per);
        else if (kind == 3)
            hipLaunchKernelGGL((xgk::copy_kernel_g<4>), dim3((unsigned)pieces.size()), dim3(xgk::kThreads), 0,
                               c->stream, dp);
        else if (kind == 4)
            hipLaunchKernelGGL((xgk::copy_kernel_g<2>), dim3((unsigned)pieces.size()), dim3(xgk::kThreads), 0,
                               c->stream, dp);
        else if (kind == 5)
            hipLaunchKernelGGL(xgk::read_only_kernel, dim3(nb * 2), dim3(xgk::kThreads), 0, c->stream,
                               (xgk::g_cu4 *)a, bytes / 16, (unsigned *)ds);
        else
            hipLaunchKernelGGL(xgk::write_only_kernel, dim3(nb * 2), dim3(xgk::kThreads), 0, c->stream,
                               (xgk::g_u4 *)b, bytes / 16);
        HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(e1, c->stream));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    *gbps = (kind >= 5 ? 1.0 : 2.0) * (double)bytes * reps / (ms * 1e-3) / 1e9;
    HIPCHK(hipEventDestroy(e0));
    HIPCHK(hipEventDestroy(e1));
    HIPCHK(hipFree(a));
    HIPCHK(hipFree(b));
    HIPCHK(hipFree(dp));
    HIPCHK(hipFree(ds));
    return XG_OK;
}

// ------------------------------------------------------------------ microbenchmark: RCCL p2p ceiling
// The rccl-tests sendrecv analogue (and the GPU version of pt2pt_test,
// mpi_sendrecv_test.c:15-74).  mode 0: all pairs (every rank sends `bytes` to
// every other rank, one group); mode 1: ring (send to r+1, receive from r-1);
// mode 2: one direction 1 -> 0 (pt2pt_test's Issend/Irecv pair), other ranks idle.
// *gbps = bytes this rank sent (mode 2: received on rank 0) per second; *sec = seconds per rep.
extern "C" int xg_p2p_bench(xg_ctx *c, int64_t bytes, int mode, int reps, double *gbps, double *sec)
{
    const int n = c->nranks, r = c->rank;
    const bool self = n == 1 && c->comm && !c->virt;      // XG_SELF_COMM: rank 0 sends to itself
    if ((n < 2 && !self) || bytes <= 0 || reps < 1 || mode < 0 || mode > 2) return XG_EARG;
    HIPCHK(hipSetDevice(c->device));
    const int npeer = self ? 1 : (mode == 0 ? n - 1 : 1);
    uint8_t *sb, *rb;
    HIPCHK(hipMalloc(&sb, bytes * npeer));
    HIPCHK(hipMalloc(&rb, bytes * npeer));
    HIPCHK(hipMemsetAsync(sb, r & 0xff, bytes * npeer, c->stream));
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    int rc = XG_OK;
    auto one = [&]() -> int {
        NCCLCHK(ncclGroupStart());
        if (self) {
            NCCLCHK(ncclSend(sb, (size_t)bytes, ncclUint8, 0, c->comm, c->stream));
            NCCLCHK(ncclRecv(rb, (size_t)bytes, ncclUint8, 0, c->comm, c->stream));
        } else if (mode == 0) {
            for (int k = 1; k < n; ++k) {
                const int to = (r + k) % n, from = (r - k + n) % n;
                NCCLCHK(ncclSend(sb + (int64_t)(k - 1) * bytes, (size_t)bytes, ncclUint8, to, c->comm, c->stream));
                NCCLCHK(ncclRecv(rb + (int64_t)(k - 1) * bytes, (size_t)bytes, ncclUint8, from, c->comm, c->stream));
            }
        } else if (mode == 1) {
            NCCLCHK(ncclSend(sb, (size_t)bytes, ncclUint8, (r + 1) % n, c->comm, c->stream));
            NCCLCHK(ncclRecv(rb, (size_t)bytes, ncclUint8, (r - 1 + n) % n, c->comm, c->stream));
        } else if (r == 1) {
            NCCLCHK(ncclSend(sb, (size_t)bytes, ncclUint8, 0, c->comm, c->stream));
        } else if (r == 0) {
            NCCLCHK(ncclRecv(rb, (size_t)bytes, ncclUint8, 1, c->comm, c->stream));
        }
        NCCLCHK(ncclGroupEnd());
        return XG_OK;
    };
    for (int w = 0; w < 2 && !rc; ++w) rc = one();          // connection set-up + warm-up
    if (!rc) rc = xg_barrier(c);
    if (!rc) {
        HIPCHK(hipEventRecord(e0, c->stream));
        for (int k = 0; k < reps && !rc; ++k) rc = one();
        HIPCHK(hipEventRecord(e1, c->stream));
        HIPCHK(hipEventSynchronize(e1));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, e0, e1));
        const double s_rep = ms * 1e-3 / reps;
        if (sec) *sec = s_rep;
        if (gbps) *gbps = (mode == 2 && !self ? (r < 2 ? (double)bytes : 0.0) : (double)bytes * npeer) / s_rep / 1e9;
    }
    HIPCHK(hipEventDestroy(e0));
    HIPCHK(hipEventDestroy(e1));
    HIPCHK(hipFree(sb));
    HIPCHK(hipFree(rb));
    return rc;
}
