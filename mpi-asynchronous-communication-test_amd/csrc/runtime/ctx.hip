// ctx.hip -- context (streams, communicator, tuning), HBM regions, fill / verify.
#include "rt.h"

#include <dirent.h>
#include <limits.h>
#include <link.h>

#include <string>

extern "C" double xg_now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

// XG_SHARE_GPU=1 (test harness): several ranks of one job on ONE GPU, each its own process
// (a one-GPU box running the multi-rank path).  RCCL refuses two ranks with the same bus id on
// one host ("Duplicate GPU detected"), so every rank names a host of its own (NCCL_HOSTID):
// the ranks then pair over RCCL's network transport (sockets on loopback) instead of xGMI.
// The calls, groups, pairing and collectives are the real multi-rank ones; the transport and
// its rates are not the node's.  (More than ~16 hardware queues on the device and the command
// processor time-slices them: a README run of m9 took 0.79 s at 8 ranks x HIP's default 4 queues
// against 9 ms at 2 (profiles/r05/share_gpu_queues/), and the 8-rank tests ran 4-7x slower once
// the pytest process itself held 4 queues beside 8 x 2.  HIP reads GPU_MAX_HW_QUEUES when it
// loads, so the launchers -- bench.py, xg_spawn_ranks, the tests -- give every process they start
// on a shared device ONE queue.)  Called before the first RCCL call of the process.
static void share_gpu_env(int rank)
{
    const char *v = getenv("XG_SHARE_GPU");
    if (!v || strcmp(v, "1")) return;
    char id[64];
    snprintf(id, sizeof id, "xg-share-gpu-rank-%d", rank);
    setenv("NCCL_HOSTID", id, 1);
    setenv("NCCL_SOCKET_IFNAME", "lo", 0);
    // every rank's RCCL kernels share the one device's CUs and spin until their peer's proxy
    // delivers: few channels per rank keep all ranks' kernels resident at once
    setenv("NCCL_MAX_NCHANNELS", "2", 0);
}

// ---- the ROCm runtime this process runs on (xg.h: xg_foreign_runtime)
static bool under(const std::string &path, const std::string &root)
{
    return !root.empty() && path.size() > root.size() && path.compare(0, root.size(), root) == 0 &&
           path[root.size()] == '/';
}

static std::string real(const char *p)
{
    char buf[PATH_MAX];
    return p && realpath(p, buf) ? std::string(buf) : std::string();
}

struct Foreign {
    std::vector<std::string> roots, bad;
};

static int foreign_cb(struct dl_phdr_info *info, size_t, void *arg)
{
    Foreign *f = static_cast<Foreign *>(arg);
    const char *name = info->dlpi_name;
    if (!name || !*name) return 0;
    const char *base = strrchr(name, '/');
    base = base ? base + 1 : name;
    static const char *const libs[] = {"libamdhip64.so", "librccl.so", "libhsa-runtime64.so"};
    bool rocm = false;
    for (const char *l : libs) rocm |= strncmp(base, l, strlen(l)) == 0;
    if (!rocm) return 0;
    const std::string rp = real(name);
    for (const std::string &r : f->roots)
        if (under(rp.empty() ? std::string(name) : rp, r)) return 0;
    f->bad.push_back(rp.empty() ? std::string(name) : rp);
    return 0;
}

extern "C" int xg_foreign_runtime(char *buf, size_t len)
{
    Foreign f;
#ifdef XG_ROCM_LIBDIR
    f.roots.push_back(real(XG_ROCM_LIBDIR));        // the build's own ROCm (a distro or conda install too)
#endif
    f.roots.push_back(real("/opt/rocm"));
    if (getenv("ROCM_PATH")) f.roots.push_back(real(getenv("ROCM_PATH")));
    if (DIR *d = opendir("/opt")) {                  // versioned installs (/opt/rocm-7.2.0)
        while (struct dirent *e = readdir(d))
            if (!strncmp(e->d_name, "rocm", 4)) f.roots.push_back(real(("/opt/" + std::string(e->d_name)).c_str()));
        closedir(d);
    }
    dl_iterate_phdr(foreign_cb, &f);
    if (buf && len) {
        std::string all;
        for (const std::string &b : f.bad) all += (all.empty() ? "" : ", ") + b;
        snprintf(buf, len, "%s", all.c_str());
    }
    return (int)f.bad.size();
}

// refuse to start on another ROCm runtime than the one libxg.so is built against
static int check_runtime(const char *who)
{
    char bad[1024];
    if (xg_foreign_runtime(bad, sizeof bad) > 0) {
        fprintf(stderr, "xg: %s refused: a foreign ROCm runtime is mapped in this process (%s), e.g. loaded by "
                        "`import torch` before the framework; libxg.so is built against /opt/rocm\n", who, bad);
        return XG_EARG;
    }
    return XG_OK;
}

extern "C" int xg_rccl_version(int *version)
{
    if (!version) return XG_EARG;
    NCCLCHK(ncclGetVersion(version));
    return XG_OK;
}

static int env_rank()
{
    const char *v = getenv("RANK");
    if (!v) v = getenv("PMI_RANK");
    return v ? atoi(v) : 0;
}

extern "C" int xg_get_unique_id(void *uid)
{
    if (check_runtime("xg_get_unique_id")) return XG_EARG;
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
    if (check_runtime("xg_init")) return XG_EARG;
    if (nranks > 1) share_gpu_env(rank);
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

// Knobs that are constants now (Knobs): a setting left in the environment -- an A/B
// recipe under profiles/ from the round that measured it -- changes nothing, so say so once
static void warn_folded_knobs()
{
    static bool done = false;
    if (done) return;
    done = true;
    static const char *const folded[] = {
        // round 4: settled tuning
        "XG_COPY_BALANCE", "XG_COPY_CHUNK", "XG_COPY_NT_MIN", "XG_COPY_NT_STREAM", "XG_COPY_WAVE",
        "XG_COPY_WAVE_MAX", "XG_COPY_WG_COST", "XG_ENGINE_WG", "XG_FUSE_UNPACK", "XG_GRID_CACHE_MAX",
        "XG_PIECE_ORDER", "XG_SOLO_MIN_STEPS", "XG_SOLO_RELAY", "XG_SPLIT_LOCAL",
        // round 5: environment twins of bin/test options (--fingerprint, --eager-limit, ...)
        "XG_FINGERPRINT", "XG_EAGER_LIMIT", "XG_PACK_MAX_SEG", "XG_PACK_MIN", "XG_PACK_FORM"};
    for (const char *k : folded)
        if (getenv(k)) fprintf(stderr, "xg: %s is set but no longer read (folded into a constant or an option)\n", k);
}

// the rest of xg_init: tuning knobs, streams, scratch, the communicator
static int init_ctx(xg_ctx *c, const void *uid)
{
    warn_folded_knobs();
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
        // piece KiB of a wave-copy launch: 0 = by its bytes (wave_kib_for), 2 / 4 / 8 forced (A/B)
        env = getenv("XG_WAVE_KIB");
        c->wave_kib = env && (atoi(env) == 2 || atoi(env) == 4 || atoi(env) == 8) ? atoi(env) : 0;
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

