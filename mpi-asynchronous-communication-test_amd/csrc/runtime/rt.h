// rt.h -- internal header of libxg's device half (include/xg.h is the C-ABI): the
// context, region and plan structures every runtime translation unit shares, the error
// macros, and the helpers more than one of them calls.  gfx950 only.
//
//   ctx.hip        context (streams, communicator), HBM regions, fill / verify
//   plan_load.hip  xg_plan_load: piece table, launch forms, engine segments, displacement scan
//   exec.hip       execution: per-step launches + RCCL groups, chains, engine, graph, armed runs
//   virtual.hip    a whole G-GPU job on one device (test hook)
//   measure.hip    kernel-timing sessions and the RCCL p2p microbenchmark
#pragma once

#include <hip/hip_runtime.h>
#include <unistd.h>
#include <rccl/rccl.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <algorithm>
#include <vector>

#include "../kernels.h"
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
struct WhereState {
    const char *fn = "idle";
    int step = -1, nsteps = 0;
    const char *phase = "";
};
inline WhereState g_where;         // one for the library (C++17 inline variable)
static inline void where(const char *fn, int step, int nsteps, const char *phase)
{
    g_where.fn = fn; g_where.step = step; g_where.nsteps = nsteps; g_where.phase = phase;
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
    int wave_kib;              // XG_WAVE_KIB: copy_kernel_w piece KiB forced (2 / 4 / 8), 0 = by launch bytes
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
    int groups;                      // RCCL groups of the step: 1, or 2 for a relay step (XG_CALL_FENCE between)
    int posts;                       // request posts of this GPU's ranks in the step (xg_stepplan.posts)
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
    std::vector<char> wave_at;     // npieces + 1: at the first piece of a copy_kernel_w launch, its
                                   // piece KiB (2 / 4 / 8: the J of copy_kernel_w<J>); else 0
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
// Piece KiB of a copy_kernel_w launch of `bytes`: the largest of 8 / 4 / 2 that still gives every
// CU a 4-wave workgroup (bytes / piece >= 4 x CUs): a 4 MiB launch in 8 KiB pieces is 512 waves =
// 128 workgroups, half the chip (the local part of a configs[2] step, profiles/r05/share_launches/);
// in 4 KiB pieces it is 256 workgroups.  Smaller launches take 2 KiB pieces.
static inline int wave_kib_for(int64_t bytes, int cus)
{
    for (int kib = 8; kib > 2; kib /= 2)
        if (bytes / ((int64_t)kib << 10) >= 4 * (int64_t)cus) return kib;
    return 2;
}

// The copy kernel variant of a launch moving `bytes` (launch_copy).  Variant 0 picks
// non-temporal loads/stores (6) when the bytes cannot come back from the 256 MiB
// Infinity Cache: a launch whose own source + destination exceed it, or a launch of
// >= kNtStream bytes in a plan whose run copies more than it (every step then finds
// its bytes evicted by the steps before) -- unless what it writes is read again at
// once (`reread`: packs feeding RCCL, TAM stage copies), which then may still find
// it in the cache; plain (1) otherwise.
static inline int copy_variant(const xg_plan *p, int64_t bytes, bool reread = false)
{
    if (p->variant) return p->variant;
    return bytes >= kNtMin || (!reread && p->streaming && bytes >= kNtStream) ? 6 : 1;
}

// RCCL writes its log -- and, under NCCL_DEBUG=WARN/VERSION, a version banner at
// communicator creation -- to stdout unless NCCL_DEBUG_FILE says otherwise; stdout
// here carries the reference's report (bin/test, bin/pt2pt_test) and bench.py's JSON
// line, so send RCCL's output to stderr unless the user chose a file.  Called before
// every first RCCL call (RCCL reads the variable when it first logs).
static inline void rccl_log_to_stderr()
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


// ---- shared between the runtime's translation units
// exec.hip
int mark(xg_plan *p, int i, hipStream_t stream);
int read_marks(const xg_plan *p, std::vector<unsigned long long> &gs);
double mark_elapsed(const xg_plan *p, int i, const std::vector<unsigned long long> &gs);
int launch_dispatches(const xg_plan *p, int b, int n, int64_t bytes);
int enqueue_pre(xg_plan *p, int s, hipStream_t stream, hipStream_t side);
int enqueue_post(xg_plan *p, int s, hipStream_t stream);
int launch_seg(xg_plan *p, const EngSeg &g, hipStream_t stream, bool armed = false);
