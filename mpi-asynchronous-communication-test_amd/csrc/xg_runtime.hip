// xg_runtime.hip -- device half of the C-ABI (include/xg.h): HBM regions,
// kernel launches, grouped RCCL exchange, step timing.  gfx950 only.
//
// Execution of one step on GPU g (xg_devplan, built by libxghost):
//   1. one copy_kernel launch over every local gather/scatter piece and every
//      pack into the per-peer staging region                (pre copies)
//   2. one ncclGroupStart .. ncclSend/ncclRecv .. ncclGroupEnd with the <= 7
//      peer GPUs this step talks to (xGMI)                  (p2p)
//   3. one copy_kernel launch unpacking staging into the receive slots (post)
//   4. a clock_kernel stamp (step mark) -- the reference's Waitall boundary
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

// On an error, hipGetLastError() is read once more: HIP keeps the last failing call's error
// for it, and a later launch check (hipGetLastError right after a launch) would otherwise
// report this old error as its own.
#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "xg: HIP error %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__,   \
                    __LINE__, #x);                                                                 \
            (void)hipGetLastError();                                                               \
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

// Device scratch freed on every return path (error returns of HIPCHK included).
struct DevMem {
    void *p = nullptr;
    DevMem() = default;
    DevMem(const DevMem &) = delete;
    DevMem &operator=(const DevMem &) = delete;
    ~DevMem()
    {
        if (p) (void)hipFree(p);
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

struct EventPair {
    hipEvent_t e[2] = {nullptr, nullptr};
    ~EventPair()
    {
        for (hipEvent_t x : e)
            if (x) (void)hipEventDestroy(x);
    }
};

// Where the host thread is (diagnostics for a run that does not return: xg_debug_where): the
// entry point, the step it is posting and whether it is waiting for the device.  Plain stores,
// read only by a watchdog after the fact.
static struct {
    const char *fn = "idle";
    int step = -1, nsteps = 0;
    const char *phase = "";
} g_where;
static inline void where(const char *fn, int step, int nsteps, const char *phase)
{
    g_where.fn = fn; g_where.step = step; g_where.nsteps = nsteps; g_where.phase = phase;
}
extern "C" const char *xg_debug_where(void)
{
    static char buf[160];
    snprintf(buf, sizeof buf, "%s: step %d of %d: %s", g_where.fn, g_where.step, g_where.nsteps, g_where.phase);
    return buf;
}

// One RCCL group whose calls come from `post`, a callable returning ncclResult_t for
// call i (i = 0..n-1): the group is closed (ncclGroupEnd) on every path, so an error
// never leaves this rank inside an open group.  Returns XG_OK or XG_ERCCL.
template <class F>
static int rccl_group(int n, F post, const char *what)
{
    ncclResult_t r = ncclGroupStart();
    if (r != ncclSuccess) {
        fprintf(stderr, "xg: RCCL error %s: ncclGroupStart (%s)\n", ncclGetErrorString(r), what);
        return XG_ERCCL;
    }
    int rc = XG_OK;
    for (int i = 0; i < n && rc == XG_OK; ++i) {
        r = post(i);
        if (r != ncclSuccess) {
            fprintf(stderr, "xg: RCCL error %s: call %d of %d in a group (%s)\n", ncclGetErrorString(r), i, n, what);
            rc = XG_ERCCL;
        }
    }
    r = ncclGroupEnd();
    if (r != ncclSuccess) {
        fprintf(stderr, "xg: RCCL error %s: ncclGroupEnd (%s)\n", ncclGetErrorString(r), what);
        rc = XG_ERCCL;
    }
    return rc;
}

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
    int solo;                  // 0: never use the solo engine
    int64_t solo_max;          // solo segments move <= this many bytes per run
    int solo_rails;            // solo segments deal their pieces over up to this many rails
    int solo_waves;            // waves per rail: 16 (a workgroup) or 1
    int64_t launch_max;        // copy launches above this many bytes go as back-to-back launches of ~this size
    int64_t wave_min;          // cross-GPU steps' plain copy launches of >= this many bytes (and <= kWaveMax)
                               // run copy_kernel_w (launch_chunk)
    int wave_grid;             // copy_kernel_w workgroups resident at once (occupancy x CUs)
    int cus;                   // compute units
    int step_chain;            // 1: time runs of one-launch local steps by in-kernel stamps (xg_plan_run)
    int engine_arm;            // 1: xg_plan_run arms single-segment plans (doorbell)
    int64_t split_min;         // a cross-GPU step's local gather of >= this many bytes runs on the side stream
                               // (smaller: in the pack / fused launch)
    int64_t self_max;          // a cross-GPU step's local part of <= this many bytes goes in its RCCL group
    int fuse_stage;            // 1: a step's stage copies launch with its local copies when hazard-free
    int split_after_pack;      // 1: a split step's local part forks after its pack launch
    int graph;                 // hipGraph replay of multi-launch runs: 1 always, 0 never, -1 latency-bound one-GPU runs
    double wall_hz;            // wall_clock64() rate
    int variant;            // copy kernel variant (launch_copy)
    int engine_occ;            // co-resident step-engine workgroups the device admits (plan load caps W)
    // kernel timing session (xg_ktime_begin/end): 1 = an event pair around every
    // copy launch, 2 = one pair around the whole session on the main stream
    int kt_mode;
    int nk;
    std::vector<hipEvent_t> kev;   // start/end pairs per copy launch (mode 1), or the region pair
    std::vector<int64_t> kbytes;   // algorithmic bytes (read + write) per launch (mode 1)
    int64_t kt_bytes;              // their sum (both modes)
};

struct xg_regions {
    xg_ctx *ctx;
    uint8_t *ptr[XG_NBUF];
    int64_t bytes[XG_NBUF];
};

struct StepR {
    // Launches of one step (piece ranges in the plan's piece table):
    //   stage (TAM rank-local copies), then local gather/scatter + packs into staging
    //   (one launch; a step with cross-GPU ops runs its local part on the side stream
    //   beside the packs and the RCCL group: split), the RCCL group, the unpacks.
    //   fused: this step's packs go in ONE launch with the previous step's unpacks
    //   (deferred there); a pack only fills staging and delivers nothing, so every
    //   message of this step is still delivered after every one of the previous step.
    // call_b / call_n: the step's RCCL calls in the plan's call list (xg_devplan_step_calls);
    // p2p_n of them are send/recv (one group), sync_after: the last is the in-loop barrier
    int stage_b, stage_n, local_b, local_n, pack_b, pack_n, post_b, post_n, call_b, call_n, p2p_n, sync_after;
    int pre_n;                       // local_n + pack_n
    int64_t stage_bytes, local_bytes, pack_bytes, post_bytes;   // bytes copied by each part (read + written once)
    bool split, fused, deferred;
    bool self_local;                 // the local copies travel in the RCCL group as self send/recv (XG_SELF_MAX)
    bool fused_local;                // fused, and the local copies join that launch (small, hazard-free)
    bool stage_fused;                // the stage copies join the step's local (+ pack) launch: none of the
                                     // other pre copies meets their bytes (xg_step_stage_meets_rest)
};

// A run of >= 2 consecutive GPU-local steps (no RCCL op, no in-loop barrier, no
// TAM stage copy, no unpack, each <= engine_max_step bytes) executed by ONE
// step_engine_kernel launch; every other step is its own launches.
struct EngSeg {
    int s0, s1;                    // steps [s0, s1)
    int w, b;                      // workgroups; 16-B loads per lane per unit (1, 4, 16)
    int sb_off;                    // its block in d_sb: (n + 1) unit offsets, then n flags
                                   // (solo: per rail nrows + 1 row barrier counts, then per rail
                                   // n closed-step indices)
    int nhaz;                      // hazard points (xg_engine_hazards flag 2)
    bool solo;                     // solo engine (solo_engine_kernel), pieces from u0
    int wv;                        // solo: waves per rail (16 or 1)
    int gran;                      // solo: descriptor granule in bytes (16, or 4 / 1 for segments not 16-B aligned)
    int u0;                        // first unit / piece of the segment in d_epieces
    int npieces;                   // solo: pieces per rail (whole chunks of rows), rail r's from u0 + r * npieces
                                   // in d_solo; w = rails
    const uint8_t *sbase;          // solo: base pointers of the descriptors' offsets
    uint8_t *dbase;
    int64_t bytes;                 // bytes copied per run
};

struct xg_plan {
    xg_ctx *ctx;
    xg_regions *reg;
    int nsteps;
    xgk::DCopy *d_pieces;
    int npieces;
    std::vector<StepR> steps;
    std::vector<xg_call> calls;       // every step's RCCL calls, as xg_devplan_step_calls lists them
    std::vector<int32_t> call_begin;  // nsteps + 1: where each step's calls start
    std::vector<hipEvent_t> fork, join;   // per split step: main -> side, side -> main
    int variant;
    bool streaming;                // one run copies more than the Infinity Cache holds (read + write)
    // step engine segments
    std::vector<int> seg_of;       // per step: index into segs, or -1
    std::vector<EngSeg> segs;
    int *d_sb;
    xgk::DCopy *d_epieces;         // every segment's work units, step-major
    xgk::EngineState *d_engine;    // state (16 B, zeroed at load) followed by stamps: rail r's of step
                                   // s at [r * nsteps + s] (grid segments: rail 0)
    int stamp_rails;               // rails the stamp area holds
    unsigned engine_base;          // barrier tickets taken by earlier launches (wraps)
    bool engine_reset;             // zero the state before the next launch
    xgk::Doorbell *db;             // host-pinned doorbell of armed runs (single-segment plans), or null
    std::vector<unsigned long long> solo_desc;   // solo segments' packed pieces (host copy)
    unsigned long long *d_solo;
    unsigned epoch;                // armed launches so far
    // staging displacements of the packed segments, computed on the device at load
    int64_t *d_disp;
    int ndisp;
    int nlaunch;                   // kernel launches per run (copies + engine), RCCL's aside
    bool rec_ev;                   // xg_plan_run is marking steps (fused launches mark the previous step's end)
    // chains: runs of >= 2 consecutive steps that are each ONE local copy launch, or a TAM
    // stage launch and/or a local launch (outside engine segments, no RCCL, no barrier).  xg_plan_run times them with no
    // mark between launches: launch t+1 stamps its start = step t's completion, a clock kernel
    // closes the chain, the chain's mark after it anchors the stamps.  chain_end[s] = end of s's chain (s = its
    // first step), 0 elsewhere.
    std::vector<int> chain_end;
    unsigned long long *d_cstamp;  // nsteps wall-clock stamps of chained steps
    std::vector<int64_t> plen;     // prefix sums of the piece lengths (npieces + 1), host side
    std::vector<char> wave_at;     // npieces + 1: 1 at the first piece of a copy_kernel_w launch
    // hipGraph replay (XG_GRAPH=1): the launches of one xg_plan_enqueue / one timed xg_plan_run,
    // captured at first use and replayed after (a launch-bound multi-step run then costs one
    // graph launch of host time instead of a launch, an event and an RCCL group per step)
    hipGraphExec_t g_enq, g_run;
    // step marks: mark(i) has a one-lane clock_kernel write the wall clock to d_gstamp[i + 1]
    // (i = -1: the start) once everything before it on the stream is done.  Not timing events:
    // an event record left the device idle ~4.7 us per step against ~2.1 us for the stamp
    // (profiles/r04/stamp_marks/), and captured events are not re-recorded by a graph replay on
    // this stack (tools/graph_probe.hip), so eager runs, graph replays and virtual jobs all stamp
    unsigned long long *d_gstamp;
    std::vector<char> need_mark;   // per step: an eager or captured run marks it (xg_plan_set_step_marks;
                                   // default all) -- engine segments and chains mark their last step always
    bool graph_auto;               // XG_GRAPH unset: this plan replays as a graph (latency-bound, one GPU)
    bool local_only;               // test hook (xg_plan_set_local_only): a virtual GPU runs its share alone,
                                   // its RCCL calls and in-loop barriers left out
    uint64_t id;                   // unique per loaded plan (keys the virtual runner's graphs)
    struct VGraph {
        std::vector<uint64_t> ids;
        bool rccl;
        hipGraphExec_t exec;
    } vg;                          // plans[0] of a virtual job: the job's captured run
};

// step boundary i of a run (-1: its start) on `stream`: a clock stamp (d_gstamp)
static int mark(xg_plan *p, int i, hipStream_t stream)
{
    hipLaunchKernelGGL(xgk::clock_kernel, dim3(1), dim3(64), 0, stream, p->d_gstamp + i + 1);
    HIPCHK(hipGetLastError());
    return XG_OK;
}

// the run's step marks, after it: gs[i + 1] = boundary i's stamp, gs[0] the start's
static int read_marks(const xg_plan *p, std::vector<unsigned long long> &gs)
{
    gs.resize((size_t)p->nsteps + 1);
    HIPCHK(hipMemcpy(gs.data(), p->d_gstamp, 8 * gs.size(), hipMemcpyDeviceToHost));
    return XG_OK;
}

// seconds from the run's start to boundary i
static double mark_elapsed(const xg_plan *p, int i, const std::vector<unsigned long long> &gs)
{
    return (double)(gs[i + 1] - gs[0]) / p->ctx->wall_hz;
}

static uint64_t next_plan_id()
{
    static uint64_t n = 0;
    return __atomic_add_fetch(&n, 1, __ATOMIC_RELAXED);
}

// Capture what `body` enqueues on `stream` into a graph and instantiate it.  The stream
// leaves capture mode on every path; on failure nothing is kept.
template <class F>
static int capture(hipStream_t stream, hipGraphExec_t *out, F body)
{
    *out = nullptr;
    HIPCHK(hipStreamBeginCapture(stream, hipStreamCaptureModeThreadLocal));
    const int rc = body();
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(stream, &g);
    if (rc || e != hipSuccess) {
        if (g) (void)hipGraphDestroy(g);
        if (!rc) fprintf(stderr, "xg: hipStreamEndCapture: %s\n", hipGetErrorString(e));
        return rc ? rc : XG_EHIP;
    }
    const hipError_t ie = hipGraphInstantiate(out, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    if (ie != hipSuccess) {
        *out = nullptr;
        fprintf(stderr, "xg: hipGraphInstantiate: %s\n", hipGetErrorString(ie));
        return XG_EHIP;
    }
    return XG_OK;
}

// Settled tuning, fixed since round 4 (DESIGN.md "Knobs" lists what each was measured against).
constexpr int64_t kNtMin = 128 << 20;      // launches of >= this many bytes stream past the MALL:
                                           // non-temporal (profiles/r02/copy_nt_sizes.txt, copy_ab_nt/)
constexpr int64_t kNtStream = 4 << 20;     // ... and, in a streaming plan, launches of >= this many
constexpr int64_t kGridCacheMax = 256 << 20;   // grid_pays: a run of <= this many bytes stays in the MALL
constexpr int64_t kWgCost = 2048;          // a copy workgroup's fixed start, bytes-equivalent (xg_piece_size)
constexpr int64_t kWaveMax = 32 << 20;     // copy_kernel_w up to this launch size (profiles/r03/wave_local/)

// The copy kernel variant of a launch moving `bytes` (launch_copy).  Variant 0 picks
// non-temporal loads/stores (6) when the bytes cannot come back from the 256 MiB
// Infinity Cache: a launch whose own source + destination exceed it, or a launch of
// >= kNtStream bytes in a plan whose run copies more than it (every step then finds
// its bytes evicted by the steps before) -- unless what it writes is read again at
// once (`reread`: packs feeding RCCL, TAM stage copies), which then may still find
// it in the cache; plain (1) otherwise.
static int copy_variant(const xg_plan *p, int64_t bytes, bool reread = false)
{
    if (p->variant) return p->variant;
    return bytes >= kNtMin || (!reread && p->streaming && bytes >= kNtStream) ? 6 : 1;
}

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

// XG_SHARE_GPU=1 (test harness): several ranks of one job on ONE GPU, each its own process
// (a one-GPU box running the multi-rank path).  RCCL refuses two ranks with the same bus id on
// one host ("Duplicate GPU detected"), so every rank names a host of its own (NCCL_HOSTID):
// the ranks then pair over RCCL's network transport (sockets on loopback) instead of xGMI.
// The calls, groups, pairing and collectives are the real multi-rank ones; the transport and
// its rates are not the node's.  Called before the first RCCL call of the process.
static void share_gpu_env(int rank)
{
    const char *v = getenv("XG_SHARE_GPU");
    if (!v || strcmp(v, "1")) return;
    char id[64];
    snprintf(id, sizeof id, "xg-share-gpu-rank-%d", rank);
    setenv("NCCL_HOSTID", id, 1);
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
}

static int env_rank()
{
    const char *v = getenv("RANK");
    if (!v) v = getenv("PMI_RANK");
    return v ? atoi(v) : 0;
}

extern "C" int xg_get_unique_id(void *uid)
{
    share_gpu_env(env_rank());
    rccl_log_to_stderr();
    StdoutToStderr quiet;
    ncclUniqueId id;
    static_assert(sizeof(ncclUniqueId) == XG_UNIQUE_ID_BYTES, "unique id size");
    NCCLCHK(ncclGetUniqueId(&id));
    memcpy(uid, &id, sizeof id);
    return XG_OK;
}

static int init_ctx(xg_ctx *c, const void *uid);

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
    c->stream = c->side = nullptr; c->d_red = nullptr;
    const int rc = init_ctx(c, uid);
    if (rc) {
        xg_finalize(c);                     // frees what init_ctx got to
        return rc;
    }
    *out = c;
    return XG_OK;
}

// the rest of xg_init: tuning knobs, streams, scratch, the communicator
static int init_ctx(xg_ctx *c, const void *uid)
{
    const int device = c->device, rank = c->rank, nranks = c->nranks;
    (void)rank;
    c->chunk = 32768; c->variant = 0; c->kt_mode = 0; c->nk = 0; c->kt_bytes = 0;   // profiles/r01_copy_ab.txt
    const char *env = getenv("XG_COPY_VARIANT");          // 0 by size (default), 1 plain, 6 non-temporal
    if (env && (atoi(env) == 1 || atoi(env) == 6)) c->variant = atoi(env);
    else if (env && atoi(env) != 0) fprintf(stderr, "xg: XG_COPY_VARIANT=%s ignored (0, 1 or 6)\n", env);
    c->engine_max_step = 16 << 20;    // crossover vs one launch per step: profiles/r01_engine_sweep.txt
    env = getenv("XG_ENGINE_MAX_STEP");      // 0: never use the step engine
    if (env) c->engine_max_step = atol(env);
    {
        // the engine's grid barrier needs every workgroup resident at once: at most one
        // per CU by design, never more than the device admits (a partitioned device has
        // fewer CUs; several ranks per GPU share them)
        int cus = 0, per_cu = 0;
        HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, xgk::step_engine_kernel<16>, xgk::kThreads, 0));
        c->engine_occ = cus * (per_cu < 1 ? 1 : per_cu);
        c->engine_wmax = cus;
        if (c->engine_wmax > c->engine_occ) c->engine_wmax = c->engine_occ;
        if (c->engine_wmax < 1) c->engine_wmax = 1;
    }
    env = getenv("XG_ENGINE_DRAIN");         // "1": drain every step even without a hazard
    c->engine_drain = env && !strcmp(env, "1");
    env = getenv("XG_ENGINE_SOLO");          // "0": never solo (the grid engine runs every segment)
    c->solo = !(env && !strcmp(env, "0"));
    // one solo launch moves <= 1 GiB (2048 pieces per one-wave rail of 512; the wide
    // descriptors have no window below that): the Theta-scale runs split into 8 launches
    // instead of 32, 5-6 % faster (profiles/r02/theta/theta_probe_solo_max.txt)
    c->solo_max = (int64_t)1 << 30;
    env = getenv("XG_ENGINE_SOLO_MAX");
    if (env) c->solo_max = atol(env);
    env = getenv("XG_SOLO_WAVES");           // waves per rail: 1 (default) or 16
    c->solo_waves = env && atoi(env) == xgk::kSoloWaves ? xgk::kSoloWaves : 1;
    // see DESIGN.md (solo engine): profiles/r02/rails/solo_probe.txt
    c->solo_rails = c->solo_waves == 1 ? 512 : 16;     // 512 one-wave rails: 2 per CU by LDS
    env = getenv("XG_SOLO_RAILS");
    if (env && atoi(env) > 0) c->solo_rails = std::min(atoi(env), xgk::kSoloMaxRails);
    env = getenv("XG_COPY_LAUNCH_MAX");      // bytes; 0 = one launch however large
    c->launch_max = env ? atoll(env) : (int64_t)512 << 20;
    {
        int cus = 0;
        HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
        c->cus = cus > 0 ? cus : 256;
        // the wave-persistent copy for the launches of cross-GPU steps (packs, unpacks, the
        // local part): profiles/r03/wave_copy/ -- one GPU's configs[2] pack launch 5.8 ->
        // 6.25 TB/s; the 448 MiB non-temporal launches stay copy_kernel_g (6.0 vs 5.5-5.8);
        // above kWaveMax the one-piece-per-workgroup launch is as fast or faster
        // (profiles/r03/wave_local/: 28 MiB 9.3 vs 9.9 us, 56 MiB 18.7 vs 18.2, 112 MiB equal)
        env = getenv("XG_COPY_WAVE_MIN");     // test hook: 0 puts every cross-GPU launch on the wave copy
        c->wave_min = env ? atoll(env) : (int64_t)1 << 20;
        int per_cu = 0;
        HIPCHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, xgk::copy_kernel_w<xgk::kWaveKiB>, xgk::kThreads,
                                                            0));
        c->wave_grid = c->cus * (per_cu < 1 ? 1 : per_cu);
    }
    env = getenv("XG_STEP_CHAIN");           // "0": a step mark after every step launch
    c->step_chain = !(env && !strcmp(env, "0"));
    // "1": arm single-segment plans (launched before the timed region, started by the host's
    // doorbell ring).  Off by default: the reference's total_time brackets its request posts
    // (mpi_test.c:1444, :1763), so the like-for-like time includes the kernel launch
    env = getenv("XG_ENGINE_ARM");
    c->engine_arm = env && !strcmp(env, "1");
    // a cross-GPU step's local part: <= self_max bytes travels in the step's RCCL group as self
    // send/recv (one RCCL launch carries a latency-bound step), < split_min bytes joins the
    // step's pack / fused launch, larger runs on the side stream beside the exchange (split).
    // README configuration as a virtual 8-GPU job (profiles/r03/hybrid/): m6 direct 49 -> 2
    // launches per run, m12 46 -> 6; configs[1..4]'s bulk local parts (MiBs) stay split
    env = getenv("XG_SPLIT_MIN");            // bytes: a smaller local part is not split off
    c->split_min = env ? atoll(env) : (int64_t)1 << 20;
    env = getenv("XG_SELF_MAX");             // bytes: local part posted as self send/recv (0: never)
    c->self_max = env ? atoll(env) : (int64_t)256 << 10;
    env = getenv("XG_FUSE_STAGE");           // "0": stage copies always in a launch of their own
    c->fuse_stage = !(env && !strcmp(env, "0"));
    env = getenv("XG_SPLIT_AFTER_PACK");     // "0": a split step's local part and its packs start together
    c->split_after_pack = !(env && !strcmp(env, "0"));
    // hipGraph replay: "1" every multi-launch run (and virtual job), "0" never; default (-1):
    // one-GPU latency-bound runs only (xg_plan.graph_auto)
    env = getenv("XG_GRAPH");
    c->graph = env ? (!strcmp(env, "1") ? 1 : 0) : -1;
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
        share_gpu_env(rank);
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
    // release everything even after an error; report the first
    int rc = XG_OK;
    auto keep = [&](hipError_t e, const char *what) {
        if (e != hipSuccess && rc == XG_OK) {
            fprintf(stderr, "xg: HIP error %s in xg_finalize (%s)\n", hipGetErrorString(e), what);
            rc = XG_EHIP;
        }
    };
    keep(hipSetDevice(c->device), "hipSetDevice");
    if (c->stream) keep(hipStreamSynchronize(c->stream), "stream");
    if (c->side) keep(hipStreamSynchronize(c->side), "side stream");
    if (c->comm) {
        const ncclResult_t r = ncclCommDestroy(c->comm);
        if (r != ncclSuccess && rc == XG_OK) {
            fprintf(stderr, "xg: RCCL error %s in ncclCommDestroy\n", ncclGetErrorString(r));
            rc = XG_ERCCL;
        }
    }
    for (auto &e : c->kev) keep(hipEventDestroy(e), "event");
    if (c->d_red) keep(hipFree(c->d_red), "scratch");
    if (c->side) keep(hipStreamDestroy(c->side), "side stream");
    if (c->stream) keep(hipStreamDestroy(c->stream), "stream");
    (void)hipGetLastError();
    delete c;
    return rc;
}

extern "C" int xg_rank(const xg_ctx *c) { return c->rank; }
extern "C" int xg_nranks(const xg_ctx *c) { return c->nranks; }
extern "C" int64_t xg_self_max(const xg_ctx *c) { return c ? c->self_max : 0; }

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
    DevMem big;
    if (n > 64) {
        HIPCHK(hipMalloc(&big.p, sizeof(double) * n));
        buf = big.as<double>();
    }
    HIPCHK(hipMemcpyAsync(buf, vals, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
    NCCLCHK(ncclAllReduce(buf, buf, n, ncclFloat64, ncclMax, c->comm, c->stream));
    HIPCHK(hipMemcpyAsync(vals, buf, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
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
    if (variant > 0 && variant != 1 && variant != 6) return XG_EARG;   // 0 by size, 1 plain, 6 non-temporal
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
    const int rc = xg_regions_poison(r);
    if (rc) {                     /* nothing half made is handed out */
        (void)xg_regions_free(r);
        return rc;
    }
    *out = r;
    return XG_OK;
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

extern "C" int xg_regions_write(xg_regions *r, int buf, int64_t off, const void *host, int64_t len)
{
    if (buf < 0 || buf >= XG_NBUF || off < 0 || len < 0 || off + len > r->bytes[buf]) return XG_EARG;
    HIPCHK(hipMemcpyAsync(r->ptr[buf] + off, host, (size_t)len, hipMemcpyHostToDevice, r->ctx->stream));
    HIPCHK(hipStreamSynchronize(r->ctx->stream));
    return XG_OK;
}

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
    DevMem m_segs;
    HIPCHK(hipMalloc(&m_segs.p, sizeof(xgk::DSeg) * segs.size()));
    xgk::DSeg *dsegs = m_segs.as<xgk::DSeg>();
    HIPCHK(hipMemcpyAsync(dsegs, segs.data(), sizeof(xgk::DSeg) * segs.size(), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(xgk::fill_kernel, dim3((unsigned)(segs.size() * cps)), dim3(xgk::kThreads), 0, c->stream,
                       r->ptr[XG_BUF_SEND], dsegs, (int)cps, d, chunk, iter, mode);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
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
    DevMem m_sl, m_out;
    HIPCHK(hipMalloc(&m_sl.p, sizeof(xgk::DSlot) * nslots));
    HIPCHK(hipMalloc(&m_out.p, sizeof(unsigned long long) * 3 * nslots));
    xgk::DSlot *dsl = m_sl.as<xgk::DSlot>();
    unsigned long long *dout = m_out.as<unsigned long long>();
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
    const uint64_t lenk = 0xD6E8FEB86659FD93ull * (uint64_t)d;
    for (int i = 0; i < nslots; ++i) {
        if (chk) chk[i] = h[i] + lenk;
        if (bad) bad[i] = (int64_t)h[nslots + i];
        if (first_bad) first_bad[i] = h[2 * nslots + i] == ~0ull ? -1 : (int64_t)h[2 * nslots + i];
    }
    return XG_OK;
}

// ------------------------------------------------------------------ plans
// Engine eligibility of one step: GPU-local copies only, small enough that the
// per-launch boundary dominates (profiles/r01_engine_sweep.txt: crossover ~16 MiB).
static bool engine_step(const xg_ctx *c, const StepR &st)
{
    return !st.p2p_n && !st.sync_after && !st.stage_n && !st.stage_fused && !st.post_n && !st.pack_n && !st.fused &&
           !st.deferred && st.local_bytes <= c->engine_max_step;
}

// Build the engine segments of a loaded plan from its host piece table: every
// maximal run of >= 2 eligible steps.  Units: the step's transfers (chunk-sized
// pieces re-joined) cut to B * 4 KiB, one burst of B 16-B loads per lane per
// workgroup visit.  B grows with the segment's largest step so a step spreads
// over up to one workgroup per CU with bytes enough in flight
// (profiles/r01_engine_sweep.txt: small units starve big steps, big units leave
// small steps on a handful of workgroups).  Barrier flags: xg_engine_hazards.
static_assert(xgk::kSoloWaves == XG_SOLO_WAVES && xgk::kSoloMaxRails == XG_SOLO_MAX_RAILS &&
                  xgk::kSoloPiece == XG_SOLO_PIECE && xgk::kSoloK == XG_SOLO_K &&
                  xgk::kSoloMaxSteps == XG_SOLO_MAX_STEPS && xgk::kSoloMaxPieces == XG_SOLO_MAX_PIECES &&
                  xgk::kSoloOffMax == XG_SOLO_OFF_MAX && xgk::kSoloWideOffMax == XG_SOLO_WIDE_OFF_MAX,
              "solo engine constants: kernels.h and xg_sched.h disagree");

// Solo or grid engine for a hazard-free segment of n steps (`busy` of them move
// bytes) moving `bytes`: the cheaper by a model of the measured costs (MI355X,
// profiles/r02/rails/solo_probe*.txt): a workgroup rail (one CU) moves ~120 GB/s of
// load + store traffic and closes a step in ~0.2 us, a one-wave rail ~15 GB/s (up to
// the ~6 TB/s HBM copy rate) and ~0.05 us; the grid engine moves at the copy kernels'
// ~5 TB/s but pays >= 1 us of device-scope barrier per step; a lone busy step outside
// the engine is a copy launch inside the timed region (~8 us).
static bool solo_pays(int64_t bytes, int n, int rails, int wv, int busy, int gran = 16)
{
    const double traffic = 2.0 * (double)bytes;
    // one-wave rails on 4-B / 1-B accesses move a quarter / a sixteenth of the 16-B rate
    const double rail = 15e9 * gran / 16.0;
    const double solo = wv == 1 ? traffic / std::min(rails * rail, 6e12 * gran / 16.0) + n * 0.05e-6
                                : traffic / (rails * 120e9) + n * 0.2e-6;
    const double grid = traffic / 5e12 + n * 1.0e-6 + (busy < 2 ? 8e-6 : 0.0);
    return solo < grid;
}

// One engine segment candidate: steps [s0, s1) with their transfers (chunk-sized pieces
// re-joined), hazard flags, solo granule and shape.  Nothing is committed to the plan.
struct SegCand {
    int s0, s1, n;
    std::vector<std::vector<xgk::DCopy>> xfer;
    std::vector<xg_span> spans;
    std::vector<int> tb, fl;
    int64_t bytes, maxstep;
    int nhaz, gran;
    uintptr_t slo, shi, dlo, dhi;
    xg_solo_shape sh;
    bool fits;                     // the solo tables can be built (limits, alignment, window)
};

static SegCand seg_candidate(const xg_plan *p, const std::vector<xgk::DCopy> &pieces, int s0, int s1)
{
    const xg_ctx *c = p->ctx;
    SegCand k{};
    k.s0 = s0; k.s1 = s1; k.n = s1 - s0;
    k.xfer.resize(k.n);
    for (int t = s0; t < s1; ++t) {
        const StepR &st = p->steps[t];
        for (int i = st.local_b; i < st.local_b + st.local_n;) {     // eligible steps hold no packs
            const uint8_t *src = pieces[i].src;
            uint8_t *dst = pieces[i].dst;
            int64_t len = pieces[i].len;
            for (++i; i < st.local_b + st.local_n && pieces[i].src == src + len && pieces[i].dst == dst + len; ++i)
                len += pieces[i].len;
            k.xfer[t - s0].push_back({src, dst, len});
        }
        k.bytes += st.local_bytes + st.pack_bytes;
        k.maxstep = std::max(k.maxstep, st.local_bytes + st.pack_bytes);
    }
    k.tb.assign(k.n + 1, 0);
    for (int t = 0; t < k.n; ++t) {
        k.tb[t + 1] = k.tb[t] + (int)k.xfer[t].size();
        for (const xgk::DCopy &x : k.xfer[t])
            k.spans.push_back({(uint64_t)(uintptr_t)x.src, (uint64_t)(uintptr_t)x.dst, (uint64_t)x.len});
    }
    // hazards over whole transfers (host scan)
    k.fl.assign(k.n, 0);
    k.nhaz = xg_engine_hazards(k.spans.data(), k.tb.data(), k.n, c->engine_drain, k.fl.data());
    // solo granule: the largest of 16 / 4 / 1 every transfer is aligned to (segment sizes
    // that are not multiples of 16 move on 4-B or 1-B accesses, one-wave rails only)
    uint64_t bits = 0;
    for (const xg_span &x : k.spans) bits |= x.src | x.dst | x.len;
    k.gran = (bits & 15) == 0 ? 16 : (bits & 3) == 0 ? 4 : 1;
    // solo: each step's 1 KiB pieces dealt round-robin over up to solo_rails rails, per
    // rail rows of kSoloWaves pieces (xg_solo_tables_g, host/solo.c)
    k.slo = k.dlo = UINTPTR_MAX;
    k.shi = k.dhi = 0;
    for (const xg_span &x : k.spans)
        if (x.len > 0) {
            k.slo = std::min<uintptr_t>(k.slo, x.src); k.shi = std::max<uintptr_t>(k.shi, x.src + x.len);
            k.dlo = std::min<uintptr_t>(k.dlo, x.dst); k.dhi = std::max<uintptr_t>(k.dhi, x.dst + x.len);
        }
    k.fits = (k.gran == 16 || c->solo_waves == 1) && k.shi > k.slo && k.dhi > k.dlo && k.n <= xgk::kSoloMaxSteps &&
             k.bytes <= c->solo_max &&
             xg_solo_tables_g(k.spans.data(), k.tb.data(), k.n, c->solo_rails, c->solo_waves, k.gran, k.slo, k.dlo,
                              &k.sh, nullptr, nullptr) == XG_OK;
    return k;
}

// Cut a hazard-free run [s0, s1) that is too long for one solo launch (steps, bytes, pieces
// per rail, the descriptors' offset window) into consecutive sub-runs that each fit, greedily
// from per-step totals; empty if some single step does not fit on its own.
static std::vector<std::pair<int, int>> solo_split(const xg_plan *p, const SegCand &k)
{
    const xg_ctx *c = p->ctx;
    std::vector<std::pair<int, int>> out;
    const int64_t rows_cap = xgk::kSoloMaxPieces - 3 * xgk::kSoloK * c->solo_waves;   // padding headroom
    const int64_t pieces_cap = (int64_t)c->solo_rails * rows_cap;
    const uint64_t window = (c->solo_waves == 1 ? xgk::kSoloWideOffMax : xgk::kSoloOffMax) * (uint64_t)k.gran;
    int a = k.s0;
    int64_t bytes = 0, np = 0;
    uintptr_t slo = UINTPTR_MAX, shi = 0, dlo = UINTPTR_MAX, dhi = 0;
    for (int t = k.s0; t < k.s1; ++t) {
        int64_t tb = 0, tp = 0;
        uintptr_t tsl = UINTPTR_MAX, tsh = 0, tdl = UINTPTR_MAX, tdh = 0;
        for (const xgk::DCopy &x : k.xfer[t - k.s0]) {
            if (x.len <= 0) continue;
            tb += x.len;
            tp += (x.len + xgk::kSoloPiece - 1) / xgk::kSoloPiece;
            tsl = std::min<uintptr_t>(tsl, (uintptr_t)x.src); tsh = std::max<uintptr_t>(tsh, (uintptr_t)x.src + x.len);
            tdl = std::min<uintptr_t>(tdl, (uintptr_t)x.dst); tdh = std::max<uintptr_t>(tdh, (uintptr_t)x.dst + x.len);
        }
        auto ok = [&](int steps, int64_t b, int64_t q, uintptr_t sl, uintptr_t sh, uintptr_t dl, uintptr_t dh) {
            return steps <= xgk::kSoloMaxSteps && b <= c->solo_max && q <= pieces_cap &&
                   (sh <= sl || sh - sl <= window) && (dh <= dl || dh - dl <= window);
        };
        if (!ok(1, tb, tp, tsl, tsh, tdl, tdh)) return {};
        if (!ok(t + 1 - a, bytes + tb, np + tp, std::min(slo, tsl), std::max(shi, tsh), std::min(dlo, tdl),
                std::max(dhi, tdh))) {
            out.push_back({a, t});
            a = t;
            bytes = np = 0;
            slo = dlo = UINTPTR_MAX;
            shi = dhi = 0;
        }
        bytes += tb;
        np += tp;
        slo = std::min(slo, tsl); shi = std::max(shi, tsh);
        dlo = std::min(dlo, tdl); dhi = std::max(dhi, tdh);
    }
    out.push_back({a, k.s1});
    return out;
}

// Grid engine vs the same steps as chained copy launches, for a run larger than the
// Infinity Cache (bytes > kGridCacheMax = 256 MiB, the MALL: every
// round of units pays HBM latency and address translation of fresh pages).  Per step, the grid's workgroups take ceil(units / W)
// dependent load -> store rounds of ~2 us each behind a ~0.9 us barrier; a chained
// launch costs a ~2.3 us boundary and moves the step at the copy kernel's rate.  Measured
// (profiles/r02/theta/): P16384 A256 d2048 m1 -c 8 (2048 steps of 2048 two-KiB
// transfers) grid 30.0 ms vs chains 7.0 ms; -c 1 (16384 steps of 256) 60.6 vs 47.3 ms.
static bool grid_pays(const xg_plan *p, const SegCand &k)
{
    const xg_ctx *c = p->ctx;
    if (k.bytes <= kGridCacheMax) return true;
    const int b = k.maxstep <= (1 << 20) ? 1 : (k.maxstep <= (4 << 20) ? 4 : 16);
    const int64_t unit = (int64_t)b * xgk::kThreads * 16;
    std::vector<int64_t> units(k.n, 0);
    int64_t maxu = 0;
    for (int t = 0; t < k.n; ++t) {
        for (const xgk::DCopy &x : k.xfer[t]) units[t] += (x.len + unit - 1) / unit;
        maxu = std::max(maxu, units[t]);
    }
    const int64_t W = std::max<int64_t>(1, std::min<int64_t>(maxu, c->engine_wmax));
    double grid = 0, chain = 0;
    for (int t = 0; t < k.n; ++t) {
        const StepR &st = p->steps[k.s0 + t];
        const double traffic = 2.0 * (double)(st.local_bytes + st.pack_bytes);
        grid += 0.9e-6 + std::max((double)((units[t] + W - 1) / W) * 2e-6, traffic / 5e12);
        chain += 2.3e-6 + traffic / 5.5e12;
    }
    return grid < chain;
}

// Commit a candidate as an engine segment (solo tables or grid units) to the plan.
static int commit_seg(xg_plan *p, SegCand &k, bool solo, std::vector<xgk::DCopy> &ep, std::vector<int> &sb)
{
    xg_ctx *c = p->ctx;
    EngSeg g;
    g.s0 = k.s0; g.s1 = k.s1; g.bytes = k.bytes; g.nhaz = k.nhaz;
    g.solo = solo;
    g.wv = c->solo_waves;
    g.gran = k.gran;
    g.b = k.maxstep <= (1 << 20) ? 1 : (k.maxstep <= (4 << 20) ? 4 : 16);
    g.sb_off = (int)sb.size();
    const int n = k.n;
    if (solo) {
        g.sbase = (const uint8_t *)k.slo;
        g.dbase = (uint8_t *)k.dlo;
        g.u0 = (int)p->solo_desc.size();
        g.w = k.sh.rails;
        g.npieces = k.sh.npieces;
        std::vector<int> meta(k.sh.nmeta);
        p->solo_desc.resize(g.u0 + (size_t)k.sh.rails * k.sh.npieces);
        if (xg_solo_tables_g(k.spans.data(), k.tb.data(), n, c->solo_rails, c->solo_waves, k.gran, k.slo, k.dlo, &k.sh,
                             reinterpret_cast<uint64_t *>(p->solo_desc.data()) + g.u0, meta.data()) != XG_OK)
            return XG_EARG;
        sb.insert(sb.end(), meta.begin(), meta.end());
    } else {
        // grid units: the step's transfers cut to B * 4 KiB, one burst of B 16-B loads per lane
        const int64_t unit = (int64_t)g.b * xgk::kThreads * 16;
        const int u0 = (int)ep.size();
        std::vector<int> beg(n + 1);
        int maxu = 0;
        for (int t = 0; t < n; ++t) {
            beg[t] = (int)ep.size() - u0;
            for (const xgk::DCopy &x : k.xfer[t])
                for (int64_t o = 0; o < x.len; o += unit)
                    ep.push_back({x.src + o, x.dst + o, x.len - o < unit ? x.len - o : unit});
            maxu = std::max(maxu, (int)ep.size() - u0 - beg[t]);
        }
        beg[n] = (int)ep.size() - u0;
        g.w = std::max(1, std::min(maxu, c->engine_wmax));
        g.npieces = 0;
        g.u0 = 0;
        for (int t = 0; t <= n; ++t) sb.push_back(u0 + beg[t]);
        sb.insert(sb.end(), k.fl.begin(), k.fl.end());
    }
    for (int t = k.s0; t < k.s1; ++t) p->seg_of[t] = (int)p->segs.size();
    p->segs.push_back(g);
    return XG_OK;
}

static int build_segments(xg_plan *p, const std::vector<xgk::DCopy> &pieces)
{
    xg_ctx *c = p->ctx;
    p->seg_of.assign(p->nsteps, -1);
    if (c->engine_max_step <= 0) return XG_OK;
    std::vector<xgk::DCopy> ep;
    std::vector<int> sb;
    int rc;
    for (int s = 0; s < p->nsteps;) {
        int e = s;
        const int s_run = s;
        while (e < p->nsteps && engine_step(c, p->steps[e])) ++e;
        // steps where this GPU copies nothing cost nothing as their own "launches": trim
        // them off both ends, and keep the run only if >= 2 steps copy something
        const int run_end = e;
        int busy = 0;
        while (s < e && !p->steps[s].pre_n) ++s;
        while (e > s && !p->steps[e - 1].pre_n) --e;
        for (int t = s; t < e; ++t) busy += p->steps[t].pre_n > 0;
        // one busy step is worth an engine launch only as the whole plan: a small one-step
        // plan on rails takes 5 us armed against 6 us (10-24 us cold) as an event-timed copy
        // launch (profiles/r02/one_step/)
        const bool whole = s_run == 0 && run_end == p->nsteps && !c->virt;
        if (busy < (whole ? 1 : 2)) {
            s = run_end > s ? run_end : s + 1;
            continue;
        }
        SegCand k = seg_candidate(p, pieces, s, e);
        const bool solo = k.nhaz == 0 && k.fits && c->solo &&
                          solo_pays(k.bytes, k.n, k.sh.rails, c->solo_waves, busy, k.gran);
        if (!solo && k.nhaz == 0 && c->solo && !k.fits && k.n >= 2) {
            // too long for one solo launch (more than kSoloMaxSteps steps -- e.g. a large -k --,
            // more bytes or pieces per rail than one launch holds): consecutive solo launches,
            // each a kernel boundary, when that beats one grid launch's barrier per step
            std::vector<std::pair<int, int>> cut = solo_split(p, k);
            std::vector<SegCand> parts;
            bool all = !cut.empty() && cut.size() > 1;
            for (size_t i = 0; all && i < cut.size(); ++i) {
                parts.push_back(seg_candidate(p, pieces, cut[i].first, cut[i].second));
                all = parts.back().fits && parts.back().nhaz == 0;
            }
            const double traffic = 2.0 * (double)k.bytes;
            const double grid = traffic / 5e12 + k.n * 1.0e-6;
            const double split = (double)cut.size() * 6e-6 + traffic / (6e12 * k.gran / 16.0) + k.n * 0.05e-6;
            if (all && split < grid) {
                for (SegCand &q : parts)
                    if ((rc = commit_seg(p, q, true, ep, sb))) return rc;
                s = e;
                continue;
            }
        }
        if (!solo && busy < 2) {      // one busy step: an engine launch only if it runs solo
            s = run_end;
            continue;
        }
        if (!solo && !grid_pays(p, k)) {   // streaming-size run of many small transfers per step
            s = e;
            continue;
        }
        if ((rc = commit_seg(p, k, solo, ep, sb))) return rc;
        s = e;
    }
    if (p->segs.empty()) return XG_OK;
    HIPCHK(hipMalloc(&p->d_sb, sizeof(int) * sb.size()));
    HIPCHK(hipMemcpy(p->d_sb, sb.data(), sizeof(int) * sb.size(), hipMemcpyHostToDevice));
    if (!ep.empty()) {
        HIPCHK(hipMalloc(&p->d_epieces, sizeof(xgk::DCopy) * ep.size()));
        HIPCHK(hipMemcpy(p->d_epieces, ep.data(), sizeof(xgk::DCopy) * ep.size(), hipMemcpyHostToDevice));
    }
    if (!p->solo_desc.empty()) {
        const size_t nb = sizeof(unsigned long long) * p->solo_desc.size();
        HIPCHK(hipMalloc(&p->d_solo, nb));
        HIPCHK(hipMemcpy(p->d_solo, p->solo_desc.data(), nb, hipMemcpyHostToDevice));
    }
    p->stamp_rails = 1;
    for (const EngSeg &g : p->segs)
        if (g.solo) p->stamp_rails = std::max(p->stamp_rails, g.w);
    const size_t eb = sizeof(xgk::EngineState) + 8 * (size_t)p->nsteps * p->stamp_rails;
    HIPCHK(hipMalloc(&p->d_engine, eb));
    HIPCHK(hipMemset(p->d_engine, 0, eb));
    // a plan that is ONE segment can be armed by xg_plan_run (doorbell in host memory)
    if (c->engine_arm && !c->virt && p->segs.size() == 1 && p->segs[0].s0 == 0 && p->segs[0].s1 == p->nsteps) {
        HIPCHK(hipHostMalloc((void **)&p->db, sizeof(xgk::Doorbell), hipHostMallocCoherent));
        memset((void *)p->db, 0, sizeof(xgk::Doorbell));
    }
    return XG_OK;
}

// The staging displacements of the packed segments (alltoallw translate,
// mpi_test.c:233-302) on the device: one scan group per step and direction,
// then the pack pieces' destinations / unpack pieces' sources are patched.
// The host's own layout (xg_devplan_build) is the cross-check: a mismatch
// refuses the plan before any copy runs.
struct DisplScan {
    std::vector<int64_t> len, host;   // per packed copy (in group order): length, host displacement
    std::vector<int> groups{0};
    std::vector<xgk::DFix> fix;
    void close_group()
    {
        if ((int)len.size() > groups.back()) groups.push_back((int)len.size());
    }
};

static int run_displ_scan(xg_plan *p, DisplScan &ds)
{
    xg_ctx *c = p->ctx;
    p->ndisp = (int)ds.len.size();
    if (!p->ndisp) return XG_OK;
    const int ng = (int)ds.groups.size() - 1;
    DevMem m_len, m_base, m_groups, m_fix;     // freed on every return (the cross-check's included)
    const std::vector<int64_t> base(ng, 0);    // every step's staging starts at 0 (xg_devplan_build)
    HIPCHK(hipMalloc(&p->d_disp, sizeof(int64_t) * p->ndisp));   // the plan's (xg_plan_free)
    HIPCHK(hipMalloc(&m_len.p, sizeof(int64_t) * p->ndisp));
    HIPCHK(hipMalloc(&m_base.p, sizeof(int64_t) * ng));
    HIPCHK(hipMalloc(&m_groups.p, sizeof(int) * (ng + 1)));
    HIPCHK(hipMalloc(&m_fix.p, sizeof(xgk::DFix) * ds.fix.size()));
    int64_t *d_len = m_len.as<int64_t>(), *d_base = m_base.as<int64_t>();
    int *d_groups = m_groups.as<int>();
    xgk::DFix *d_fix = m_fix.as<xgk::DFix>();
    HIPCHK(hipMemcpyAsync(d_len, ds.len.data(), sizeof(int64_t) * p->ndisp, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_base, base.data(), sizeof(int64_t) * ng, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_groups, ds.groups.data(), sizeof(int) * (ng + 1), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(d_fix, ds.fix.data(), sizeof(xgk::DFix) * ds.fix.size(), hipMemcpyHostToDevice, c->stream));
    hipLaunchKernelGGL(xgk::displ_scan_kernel, dim3(ng), dim3(xgk::kThreads), 0, c->stream, d_len, d_groups, d_base,
                       p->d_disp);
    HIPCHK(hipGetLastError());
    std::vector<int64_t> got(p->ndisp);
    HIPCHK(hipMemcpyAsync(got.data(), p->d_disp, sizeof(int64_t) * p->ndisp, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    for (int i = 0; i < p->ndisp; ++i)
        if (got[i] != ds.host[i]) {
            fprintf(stderr, "xg_plan_load: device displacement %d = %lld, host layout %lld\n", i, (long long)got[i],
                    (long long)ds.host[i]);
            return XG_EARG;
        }
    const int nfix = (int)ds.fix.size();
    hipLaunchKernelGGL(xgk::displ_apply_kernel, dim3((nfix + xgk::kThreads - 1) / xgk::kThreads), dim3(xgk::kThreads),
                       0, c->stream, p->d_pieces, d_fix, nfix, p->d_disp, p->reg->ptr[XG_BUF_STAGE_SEND],
                       p->reg->ptr[XG_BUF_STAGE_RECV]);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return XG_OK;
}

extern "C" int xg_plan_free(xg_plan *p);
static int launch_dispatches(const xg_plan *p, int b, int n, int64_t bytes);

// Device half of a plan load: the piece table, the step events, the displacement scan
// and the engine segments.  On an error the caller frees the plan (xg_plan_free takes a
// half-loaded one: every handle starts null).
static int plan_upload(xg_plan *p, const std::vector<xgk::DCopy> &pieces, DisplScan &ds)
{
    int rc;
    if (p->npieces) {
        HIPCHK(hipMalloc(&p->d_pieces, sizeof(xgk::DCopy) * pieces.size()));
        HIPCHK(hipMemcpy(p->d_pieces, pieces.data(), sizeof(xgk::DCopy) * pieces.size(), hipMemcpyHostToDevice));
    }
    p->need_mark.assign(p->nsteps, 1);
    p->fork.assign(p->nsteps, nullptr);
    p->join.assign(p->nsteps, nullptr);
    for (int s = 0; s < p->nsteps; ++s)
        if (p->steps[s].split) {
            HIPCHK(hipEventCreateWithFlags(&p->fork[s], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&p->join[s], hipEventDisableTiming));
        }
    HIPCHK(hipMalloc(&p->d_gstamp, 8 * ((size_t)p->nsteps + 1)));
    if ((rc = run_displ_scan(p, ds)) || (rc = build_segments(p, pieces))) return rc;
    return XG_OK;
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
    p->ctx = c; p->reg = r; p->nsteps = dp->nsteps; p->variant = c->variant; p->streaming = false;
    p->d_pieces = nullptr; p->d_sb = nullptr; p->d_epieces = nullptr; p->d_engine = nullptr; p->d_disp = nullptr;
    p->ndisp = 0; p->engine_base = 0; p->engine_reset = false; p->nlaunch = 0;
    p->db = nullptr; p->epoch = 0; p->d_solo = nullptr; p->rec_ev = false; p->stamp_rails = 1; p->d_cstamp = nullptr;
    p->g_enq = p->g_run = nullptr; p->id = next_plan_id(); p->vg.rccl = false; p->vg.exec = nullptr;
    p->d_gstamp = nullptr; p->graph_auto = false; p->local_only = false;
    // One piece per workgroup.  Bytes per piece, per launch (launch_chunk over the launch's
    // copies): c->chunk (32 KiB: profiles/r01_copy_ab.txt) or c->chunk / 2, / 4, / 8 (>= 4 KiB;
    // a halving keeps dividing the power-of-two segment sizes: no ragged tail piece per segment,
    // profiles/r01_min_pieces_ab.txt), whichever gives the least work to the busiest CU: a
    // launch of w pieces of c bytes puts ceil(w / CUs) pieces on some CU, each costing c bytes
    // plus a fixed per-workgroup start (kWgCost = 2 KiB bytes-equivalent); ties
    // keep the larger piece.  A 28 MiB pack of 256 KiB segments: 896 pieces of 32 KiB = 3.5
    // per CU (the busiest 4 x 32 KiB) -> 1792 of 16 KiB = exactly 7 (7 x 16 KiB).  The bench's
    // 448 MiB launches stay 32 KiB (56 per CU).  (A rule
    // forcing >= 2 x CUs pieces on small launches was measured 3-7 % slower and dropped:
    // profiles/r03/min_wg/summary.txt.)
    // A launch of a cross-GPU step (packs, unpacks, its local part), or of a GPU-local step too
    // large for the step engine, that copies with plain loads and stores, every transfer 16-B
    // aligned, of >= wave_min bytes: copy_kernel_w over pieces of kWaveKiB (wave_at marks its
    // first piece; profiles/r03/wave_copy/).
    int64_t chunk = c->chunk;
    std::vector<xgk::DCopy> pieces;
    std::vector<char> wave_at;
    auto launch_chunk = [&](std::initializer_list<std::pair<int, int>> ranges, bool cross = false,
                            bool reread = false) {
        chunk = c->chunk;
        const size_t first = pieces.size();
        if (wave_at.size() <= first) wave_at.resize(first + 1, 0);
        wave_at[first] = 0;
        int64_t bytes = 0;
        uint64_t bits = 0;
        for (const auto &rg : ranges)
            for (int i = 0; i < rg.second; ++i) {
                const xg_copy &cp = dp->copies[rg.first + i];
                if (cp.len <= 0) continue;
                bytes += cp.len;
                bits |= (uint64_t)cp.src_off | (uint64_t)cp.dst_off | (uint64_t)cp.len;
            }
        if (bytes <= 0) return;
        if (cross && bytes >= c->wave_min && bytes <= kWaveMax && (bits & 15) == 0 &&
            copy_variant(p, bytes, reread) == 1) {
            chunk = (int64_t)xgk::kWaveKiB << 10;
            wave_at[first] = 1;
            return;
        }
        std::vector<int64_t> lens;
        for (const auto &rg : ranges)
            for (int i = 0; i < rg.second; ++i) lens.push_back(dp->copies[rg.first + i].len);
        chunk = xg_piece_size(lens.data(), (int)lens.size(), c->chunk, c->cus, kWgCost);
    };
    DisplScan ds;
    int rc;
    // side: -1 plain copy; 0 pack (destination in STAGE_SEND, displacement from the
    // device scan); 1 unpack (source in STAGE_RECV, likewise)
    auto add = [&](const xg_copy &cp, int side) -> bool {
        if (cp.len <= 0) return true;
        if (cp.src_buf < 0 || cp.src_buf >= XG_NBUF || cp.dst_buf < 0 || cp.dst_buf >= XG_NBUF) return false;
        if (cp.src_off < 0 || cp.dst_off < 0 || cp.src_off + cp.len > r->bytes[cp.src_buf] ||
            cp.dst_off + cp.len > r->bytes[cp.dst_buf])
            return false;
        const int ci = (int)ds.len.size();
        if (side >= 0) {
            ds.len.push_back(cp.len);
            ds.host.push_back(side == 0 ? cp.dst_off : cp.src_off);
        }
        for (int64_t o = 0; o < cp.len; o += chunk) {
            xgk::DCopy d;
            // staging side of a packed copy: displacement 0 until the device scan patches it
            d.src = r->ptr[cp.src_buf] + (side == 1 ? 0 : cp.src_off) + o;
            d.dst = r->ptr[cp.dst_buf] + (side == 0 ? 0 : cp.dst_off) + o;
            d.len = cp.len - o < chunk ? cp.len - o : chunk;
            if (side >= 0) ds.fix.push_back({(int)pieces.size(), ci, o, side, 0});
            pieces.push_back(d);
        }
        return true;
    };
    p->steps.resize(dp->nsteps);
    // pass 1: per step, what it holds and how it launches
    for (int s = 0; s < dp->nsteps; ++s) {
        const xg_stepplan &sp = dp->steps[s];
        StepR &st = p->steps[s];
        if (sp.stage_count < 0 || sp.stage_count > sp.pre_count || sp.post_count < 0) goto bad;
        int nloc = 0, npack = 0;
        for (int i = sp.stage_count; i < sp.pre_count; ++i) {
            const bool pack = dp->copies[sp.pre_begin + i].dst_buf == XG_BUF_STAGE_SEND;
            if (!pack && npack) goto bad;                       // the plan lists local copies, then packs
            (pack ? npack : nloc) += dp->copies[sp.pre_begin + i].len > 0;
        }
        for (int i = 0; i < sp.post_count; ++i)
            if (dp->copies[sp.post_begin + i].src_buf != XG_BUF_STAGE_RECV) goto bad;   // post copies unpack
        {
            // the step's RCCL calls: exactly what libxghost says this GPU posts (calls.c)
            const int nc = xg_devplan_step_calls(dp, s, c->self_max, nullptr);
            if (nc < 0) goto bad;
            st.self_local = xg_devplan_step_self_calls(dp, s, c->self_max) > 0;
            st.call_b = (int)p->calls.size();
            st.call_n = nc;
            p->call_begin.push_back(st.call_b);
            p->calls.resize(st.call_b + nc);
            xg_devplan_step_calls(dp, s, c->self_max, p->calls.data() + st.call_b);
            st.p2p_n = 0;
            st.sync_after = 0;
            for (int i = 0; i < nc; ++i) {
                const xg_call &o = p->calls[st.call_b + i];
                if (o.kind == XG_CALL_BARRIER) {
                    st.sync_after = c->nranks > 1;
                    continue;
                }
                if ((o.kind != XG_CALL_SEND && o.kind != XG_CALL_RECV) || o.peer < 0 || o.peer >= c->nranks ||
                    (o.peer == c->rank && !st.self_local) || o.buf < 0 || o.buf >= XG_NBUF || o.off < 0 ||
                    o.len < 0 || o.off + o.len > r->bytes[o.buf])
                    goto bad;
                st.p2p_n++;
            }
        }
        if (st.self_local) nloc = 0;        // the local copies travel in the step's RCCL group
        int64_t b_loc = 0;
        for (int i = sp.stage_count; i < sp.pre_count; ++i)
            if (dp->copies[sp.pre_begin + i].dst_buf != XG_BUF_STAGE_SEND && !st.self_local)
                b_loc += std::max<int64_t>(0, dp->copies[sp.pre_begin + i].len);
        // a cross-GPU step's local part runs on the side stream beside the packs and the RCCL
        // group (split) when it is large enough to pay for the fork / join; a smaller one joins
        // the step's first launch -- the fused one too, if it touches none of the bytes the
        // previous step's unpacks write (then the step is ONE copy launch + its RCCL group)
        st.split = st.p2p_n > 0 && nloc > 0 && b_loc >= c->split_min;
        st.deferred = false;
        const bool prev_ok = s > 0 && npack > 0 && sp.stage_count == 0 &&
                             !p->steps[s - 1].sync_after && dp->steps[s - 1].post_count > 0;
        st.fused = prev_ok && (st.split || nloc == 0 || !xg_step_local_meets_unpacks(dp, s));
        st.fused_local = st.fused && !st.split && nloc > 0;
        // TAM: a step's stage copies share the local (+ pack) launch when none of those meets
        // their bytes -- README m15 / m16 step 3: 6 -> 5 launches per run
        st.stage_fused = c->fuse_stage && sp.stage_count > 0 && (nloc > 0 || npack > 0) && !st.split &&
                         !st.fused && !st.self_local && xg_step_stage_meets_rest(dp, s) == 0;
        if (st.fused) p->steps[s - 1].deferred = true;
    }
    p->call_begin.push_back((int32_t)p->calls.size());
    {
        // the bytes one run copies (as the StepR totals below add them up): whether the plan
        // streams past the Infinity Cache decides each launch's variant (copy_variant)
        int64_t run = 0;
        for (int s = 0; s < dp->nsteps; ++s) {
            const xg_stepplan &sp = dp->steps[s];
            for (int i = 0; i < sp.pre_count; ++i) {
                const xg_copy &cp = dp->copies[sp.pre_begin + i];
                const bool local = i >= sp.stage_count && cp.dst_buf != XG_BUF_STAGE_SEND;
                if (!(local && p->steps[s].self_local)) run += std::max<int64_t>(0, cp.len);
            }
            for (int i = 0; i < sp.post_count; ++i) run += std::max<int64_t>(0, dp->copies[sp.post_begin + i].len);
        }
        // ... and whether its regions could hold in it at all: -k repetitions re-copy the same
        // bytes, so a run of many small repetitions (P32 A14 -d 64 KiB -k 50: 56 MiB of
        // regions, 2.8 GB copied) stays cache-resident and copies with plain stores
        int64_t foot = 0;
        for (int i = 0; i < XG_NBUF; ++i) foot += std::max<int64_t>(0, dp->region_bytes[i]);
        p->streaming = std::min(2 * run, foot) > ((int64_t)256 << 20);
    }
    // pass 2: the piece table, each launch's pieces contiguous (a fused launch: the
    // previous step's unpacks, then this step's packs)
    for (int s = 0; s < dp->nsteps; ++s) {
        const xg_stepplan &sp = dp->steps[s];
        StepR &st = p->steps[s];
        auto span = [&](int b) {
            int64_t n = 0;
            for (int i = b; i < (int)pieces.size(); ++i) n += pieces[i].len;
            return n;
        };
        auto add_post = [&](int t) -> bool {      // (chunk set by the caller for its launch)
            const xg_stepplan &tp = dp->steps[t];
            StepR &tt = p->steps[t];
            tt.post_b = (int)pieces.size();
            for (int i = 0; i < tp.post_count; ++i)
                if (!add(dp->copies[tp.post_begin + i], 1)) return false;
            ds.close_group();
            tt.post_n = (int)pieces.size() - tt.post_b;
            tt.post_bytes = span(tt.post_b);
            return true;
        };
        // each launch's pieces cut for that launch's bytes (launch_chunk): stage | local (+ packs,
        // unless split) | [previous unpacks +] packs | unpacks
        int first_pack = sp.pre_count;
        for (int i = sp.stage_count; i < sp.pre_count; ++i)
            if (dp->copies[sp.pre_begin + i].dst_buf == XG_BUF_STAGE_SEND) {
                first_pack = i;
                break;
            }
        const std::pair<int, int> r_stage{sp.pre_begin, sp.stage_count},
            r_local{sp.pre_begin + sp.stage_count, st.self_local ? 0 : first_pack - sp.stage_count},
            r_pack{sp.pre_begin + first_pack, sp.pre_count - first_pack},
            r_prev{st.fused ? dp->steps[s - 1].post_begin : 0, st.fused ? dp->steps[s - 1].post_count : 0},
            r_post{sp.post_begin, sp.post_count};
        int64_t b_local = 0;
        for (int i = 0; i < r_local.second; ++i) b_local += std::max<int64_t>(0, dp->copies[r_local.first + i].len);
        if (st.stage_fused) {
            // stage | local | packs as ONE launch (the stage pieces count as local ones)
            launch_chunk({r_stage, r_local, r_pack}, st.p2p_n > 0 || r_pack.second > 0 || c->engine_max_step <= 0 ||
                                                         b_local > c->engine_max_step, true);
            st.stage_b = (int)pieces.size();
            for (int i = 0; i < sp.stage_count; ++i)
                if (!add(dp->copies[sp.pre_begin + i], -1)) goto bad;
            st.stage_n = 0;
            st.stage_bytes = 0;
        } else {
            launch_chunk({r_stage});
            st.stage_b = (int)pieces.size();
            for (int i = 0; i < sp.stage_count; ++i)
                if (!add(dp->copies[sp.pre_begin + i], -1)) goto bad;
            st.stage_n = (int)pieces.size() - st.stage_b;
            st.stage_bytes = span(st.stage_b);
        }
        // piece order: stage | local | [previous unpacks] | packs (split or not fused), or
        // stage | previous unpacks | local | packs (fused_local: one launch over all three)
        if (st.fused_local) {
            launch_chunk({r_prev, r_local, r_pack}, true, true);
            if (!add_post(s - 1)) goto bad;
        } else if (!st.stage_fused) {
            // a GPU-local step's launch too, when it cannot be an engine step (larger than
            // engine_max_step, or the engine off): one large one-off launch
            const bool big_local = c->engine_max_step <= 0 || b_local > c->engine_max_step;
            if (st.split) launch_chunk({r_local}, true);
            else launch_chunk({r_local, r_pack}, st.p2p_n > 0 || r_pack.second > 0 || big_local, r_pack.second > 0);
        }
        st.local_b = st.stage_fused ? st.stage_b : (int)pieces.size();
        for (int i = sp.stage_count; i < first_pack && !st.self_local; ++i)
            if (!add(dp->copies[sp.pre_begin + i], -1)) goto bad;
        st.local_n = (int)pieces.size() - st.local_b;
        st.local_bytes = span(st.local_b);
        if (!st.fused_local) {
            if (st.split || st.fused) launch_chunk({r_prev, r_pack}, true, true);
            if (st.fused && !add_post(s - 1)) goto bad;
        }
        st.pack_b = (int)pieces.size();
        for (int i = first_pack; i < sp.pre_count; ++i)
            if (!add(dp->copies[sp.pre_begin + i], 0)) goto bad;
        ds.close_group();
        st.pack_n = (int)pieces.size() - st.pack_b;
        st.pack_bytes = span(st.pack_b);
        st.pre_n = st.local_n + st.pack_n;
        st.post_b = (int)pieces.size();
        st.post_n = 0;
        st.post_bytes = 0;
        launch_chunk({r_post}, true);
        if (!st.deferred && !add_post(s)) goto bad;
    }
    // order of a launch's local pieces (workgroup i copies piece i): by destination address.
    // The workgroups in flight at any moment then write a few consecutive segments instead of
    // one piece in each of dozens of scattered slots -- 7-10 % shorter all-to-many launches
    // (DRAM row locality of the write stream; message or source order measured slower,
    // profiles/r02/piece_order/; so did dealing each XCD its own eighth, 3-8 %,
    // profiles/r04/xcd_order/).  Local pieces carry no displacement fix-ups and a launch's
    // pieces are independent, so any order is valid.
    // Unpack pieces (source in staging, patched by the device scan) are ordered by their
    // destination too, with their fix-ups renumbered.
    {
        auto key_less = [](const xgk::DCopy &x, const xgk::DCopy &y) { return x.dst < y.dst; };
        for (const StepR &st : p->steps)
            std::stable_sort(pieces.begin() + st.local_b, pieces.begin() + st.local_b + st.local_n, key_less);
        std::vector<int> where(pieces.size(), -1);      // old index -> its fix-up
        for (size_t f = 0; f < ds.fix.size(); ++f) where[ds.fix[f].piece] = (int)f;
        for (const StepR &st : p->steps) {
            if (st.post_n < 2) continue;
            std::vector<int> idx(st.post_n);
            for (int i = 0; i < st.post_n; ++i) idx[i] = st.post_b + i;
            std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return pieces[x].dst < pieces[y].dst; });
            std::vector<xgk::DCopy> sorted(st.post_n);
            for (int i = 0; i < st.post_n; ++i) sorted[i] = pieces[idx[i]];
            for (int i = 0; i < st.post_n; ++i) {
                const int f = where[idx[i]];
                if (f >= 0) ds.fix[f].piece = st.post_b + i;
            }
            std::copy(sorted.begin(), sorted.end(), pieces.begin() + st.post_b);
        }
    }
    p->npieces = (int)pieces.size();
    wave_at.resize(pieces.size() + 1, 0);
    p->wave_at.swap(wave_at);
    p->plen.assign(pieces.size() + 1, 0);
    for (size_t i = 0; i < pieces.size(); ++i) p->plen[i + 1] = p->plen[i] + pieces[i].len;
    if ((rc = plan_upload(p, pieces, ds))) {
        xg_plan_free(p);        // frees whatever the upload got to
        return rc;
    }
    for (int s = 0; s < p->nsteps; ++s) {
        const StepR &st = p->steps[s];
        if (p->seg_of[s] >= 0) {
            p->nlaunch += p->segs[p->seg_of[s]].s0 == s;
            continue;
        }
        // kernel dispatches, as enqueue_pre / enqueue_post issue them (launch_cuts)
        auto D = [&](int b, int n, int64_t bytes) { return n > 0 ? launch_dispatches(p, b, n, bytes) : 0; };
        p->nlaunch += D(st.stage_b, st.stage_n, st.stage_bytes);
        if (st.fused) {
            const StepR &pv = p->steps[s - 1];
            p->nlaunch += D(pv.post_b, pv.post_n + (st.fused_local ? st.local_n : 0) + st.pack_n,
                            pv.post_bytes + (st.fused_local ? st.local_bytes : 0) + st.pack_bytes);
        }
        if (st.split)
            p->nlaunch += D(st.local_b, st.local_n, st.local_bytes) + (st.fused ? 0 : D(st.pack_b, st.pack_n, st.pack_bytes));
        else if (!st.fused)
            p->nlaunch += D(st.local_b, st.pre_n, st.local_bytes + st.pack_bytes);
        if (!st.deferred) p->nlaunch += D(st.post_b, st.post_n, st.post_bytes);
    }
    {
        int64_t run = 0;
        for (const StepR &st : p->steps) run += st.stage_bytes + st.local_bytes + st.pack_bytes + st.post_bytes;
        // a one-GPU run of several small launches is bound by launching them, not by their
        // bytes: replayed as one graph (README TAM chains 17-19 -> 15-16 us,
        // profiles/r03/readme_cli/summary.txt).  Multi-GPU and virtual runs stay launched:
        // graphs of RCCL and cross-stream nodes replayed 1.1-5x slower (profiles/r03/hybrid/)
        p->graph_auto = c->nranks == 1 && !c->virt && run <= ((int64_t)16 << 20);
    }
    p->chain_end.assign(p->nsteps, 0);
    if (c->step_chain) {
        // a chain step: its stage copies (TAM) and/or its local copies, each one launch
        // of a variant that can stamp its start, and nothing else
        auto one_launch = [&](int s) {
            const StepR &st = p->steps[s];
            auto stamps = [&](int64_t bytes, bool reread) {
                const int v = copy_variant(p, bytes, reread);
                return v == 1 || v == 6;
            };
            return p->seg_of[s] < 0 && !st.split && !st.fused && !st.deferred && !st.p2p_n && !st.pack_n &&
                   !st.post_n && !st.sync_after && (st.local_n > 0 || st.stage_n > 0) &&
                   (!st.local_n || stamps(st.local_bytes, st.stage_fused)) && (!st.stage_n || stamps(st.stage_bytes, true));
        };
        bool any = false;
        for (int s = 0; s < p->nsteps;) {
            int e = s;
            while (e < p->nsteps && one_launch(e)) ++e;
            if (e - s >= 2) {
                p->chain_end[s] = e;
                any = true;
            }
            s = e > s ? e : s + 1;
        }
        if (any) {
            const hipError_t e = hipMalloc(&p->d_cstamp, 8 * (size_t)p->nsteps);
            if (e != hipSuccess) {
                p->d_cstamp = nullptr;
                fprintf(stderr, "xg: HIP error %s: chain stamps\n", hipGetErrorString(e));
                xg_plan_free(p);
                return XG_EHIP;
            }
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
    // release everything even after an error (a half-loaded plan included); report the first
    hipError_t first = hipSuccess;
    auto keep = [&](hipError_t e) {
        if (e != hipSuccess && first == hipSuccess) first = e;
    };
    keep(hipStreamSynchronize(p->ctx->stream));
    keep(hipStreamSynchronize(p->ctx->side));
    for (void *q : {(void *)p->d_pieces, (void *)p->d_sb, (void *)p->d_epieces, (void *)p->d_engine,
                    (void *)p->d_disp, (void *)p->d_solo, (void *)p->d_cstamp, (void *)p->d_gstamp})
        if (q) keep(hipFree(q));
    if (p->db) keep(hipHostFree((void *)p->db));
    for (auto &e : p->fork) if (e) keep(hipEventDestroy(e));
    for (auto &e : p->join) if (e) keep(hipEventDestroy(e));
    for (hipGraphExec_t g : {p->g_enq, p->g_run, p->vg.exec})
        if (g) keep(hipGraphExecDestroy(g));
    delete p;
    if (first != hipSuccess) {
        fprintf(stderr, "xg: HIP error %s while freeing a plan\n", hipGetErrorString(first));
        return XG_EHIP;
    }
    return XG_OK;
}

extern "C" int xg_plan_nsteps(const xg_plan *p) { return p->nsteps; }
extern "C" int xg_plan_engine(const xg_plan *p) { return p->segs.empty() ? 0 : p->segs[0].w; }
extern "C" int xg_plan_engine_rails(const xg_plan *p)
{
    for (const EngSeg &g : p->segs)
        if (g.solo) return g.w;
    return 0;
}
extern "C" int xg_plan_launches(const xg_plan *p) { return p->nlaunch; }

extern "C" int xg_plan_engine_steps(const xg_plan *p, int *nseg, int *nhaz)
{
    int n = 0, h = 0;
    for (const EngSeg &g : p->segs) {
        n += g.s1 - g.s0;
        h += g.nhaz;
    }
    if (nseg) *nseg = (int)p->segs.size();
    if (nhaz) *nhaz = h;
    return n;
}

extern "C" int xg_plan_displs(const xg_plan *p, int64_t *out, int n)
{
    if (!out) return p->ndisp;
    if (n < p->ndisp) return XG_EARG;
    if (p->ndisp) HIPCHK(hipMemcpy(out, p->d_disp, sizeof(int64_t) * p->ndisp, hipMemcpyDeviceToHost));
    return XG_OK;
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

static int launch_dispatches(const xg_plan *p, int b, int n, int64_t bytes)
{
    std::vector<std::pair<int, int>> cuts;
    launch_cuts(p, b, n, bytes, cuts);
    return (int)cuts.size();
}

static int launch_one(xg_plan *p, int b, int n, int v, hipStream_t st, unsigned long long *start)
{
    const xgk::DCopy *pc = p->d_pieces + b;
    if (v == 1 && p->wave_at[b]) {       // pieces of <= kWaveKiB, 16-B aligned (launch_chunk)
        const int w = std::max(1, std::min(p->ctx->wave_grid, (n + 3) / 4));
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
static int enqueue_pre(xg_plan *p, int s, hipStream_t stream, hipStream_t side)
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
static int enqueue_post(xg_plan *p, int s, hipStream_t stream)
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
    // the step's send/recv calls, in the order libxghost lists them (xg_devplan_step_calls),
    // as one group; the barrier call, if any, is the step's last and follows the unpacks
    const xg_call *cl = p->calls.data() + st.call_b;
    if (st.p2p_n && (rc = rccl_group(
                         st.p2p_n,
                         [&](int i) {
                             const xg_call &o = cl[i];
                             uint8_t *ptr = p->reg->ptr[o.buf] + o.off;
                             return o.kind == XG_CALL_SEND
                                        ? ncclSend(ptr, (size_t)o.len, ncclUint8, o.peer, c->comm, c->stream)
                                        : ncclRecv(ptr, (size_t)o.len, ncclUint8, o.peer, c->comm, c->stream);
                         },
                         "step exchange")))
        return rc;
    if ((rc = enqueue_post(p, s, c->stream))) return rc;
    if (st.sync_after)   /* in-loop MPI_Barrier: every GPU finishes this step before any goes on */
        NCCLCHK(ncclAllReduce(c->d_red, c->d_red, 1, ncclFloat64, ncclMax, c->comm, c->stream));
    return XG_OK;
}

// one launch of the step engine over segment g (armed: waits for the doorbell `epoch`)
static int launch_seg(xg_plan *p, const EngSeg &g, hipStream_t stream, bool armed = false)
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
            // the whole run is posted by one graph launch: its host time is shared evenly over the
            // steps, so each step (and each rank posting in it, xg_sched_rank_timer) keeps a share
            // as under per-step enqueueing, and the shares sum to the launch time
            const double tp = (xg_now() - t0) / p->nsteps;
            for (int s = 0; s < p->nsteps; ++s) step_post[s] = tp;
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

// Test hook: GPU g of a G-GPU job (a virtual context) runs its own share alone -- every copy
// launch of its plan (stage, local gather/scatter, packs, unpacks) with its RCCL calls and
// in-loop barriers left out, so a share too large to put all G GPUs on one device (configs[4]
// at its stated size: 256 GiB per GPU) still executes, its local slots verifiable.  Refused
// (XG_EARG) for a plan whose local copies travel as self send/recv in an RCCL group
// (XG_SELF_MAX): leaving the group out would drop them.
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
            } else if (q1 > q0) {
                where("xg_vplans_run_rccl", s, nst, "posting the RCCL group (ncclGroupEnd)");
                // every pair of the step as a self send + receive in ONE group (issue order = pair order)
                if ((rc = rccl_group(
                         (int)(2 * (q1 - q0)),
                         [&](int i) {
                             uint8_t *src, *dst;
                             const xg_call_pair &q = pairs[q0 + i / 2];
                             ends(q, &src, &dst);
                             return i % 2 == 0 ? ncclSend(src, (size_t)q.len, ncclUint8, 0, c0->comm, st)
                                               : ncclRecv(dst, (size_t)q.len, ncclUint8, 0, c0->comm, st);
                         },
                         "virtual job step")))
                    return rc;
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
    DevMem m_sb, m_rb;                  // freed, and the events destroyed, on every return path
    EventPair ev;
    HIPCHK(hipMalloc(&m_sb.p, bytes * npeer));
    HIPCHK(hipMalloc(&m_rb.p, bytes * npeer));
    uint8_t *sb = m_sb.as<uint8_t>(), *rb = m_rb.as<uint8_t>();
    HIPCHK(hipMemsetAsync(sb, r & 0xff, bytes * npeer, c->stream));
    HIPCHK(hipEventCreate(&ev.e[0]));
    HIPCHK(hipEventCreate(&ev.e[1]));
    // this rank's calls of one repetition: (send?, peer, offset into sb / rb)
    struct Op { bool send; int peer; int64_t off; };
    std::vector<Op> ops;
    if (self) {
        ops = {{true, 0, 0}, {false, 0, 0}};
    } else if (mode == 0) {
        for (int k = 1; k < n; ++k) {
            ops.push_back({true, (r + k) % n, (int64_t)(k - 1) * bytes});
            ops.push_back({false, (r - k + n) % n, (int64_t)(k - 1) * bytes});
        }
    } else if (mode == 1) {
        ops = {{true, (r + 1) % n, 0}, {false, (r - 1 + n) % n, 0}};
    } else if (r == 1) {
        ops = {{true, 0, 0}};
    } else if (r == 0) {
        ops = {{false, 1, 0}};
    }
    auto one = [&]() -> int {
        return rccl_group(
            (int)ops.size(),
            [&](int i) {
                const Op &o = ops[i];
                return o.send ? ncclSend(sb + o.off, (size_t)bytes, ncclUint8, o.peer, c->comm, c->stream)
                              : ncclRecv(rb + o.off, (size_t)bytes, ncclUint8, o.peer, c->comm, c->stream);
            },
            "xg_p2p_bench");
    };
    int rc = XG_OK;
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
