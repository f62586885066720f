// plan_load.hip -- xg_plan_load: a device plan (libxghost) becomes the piece table, each step's
// launch form, the engine segments and the staging displacements (device scan).
#include "rt.h"

static uint64_t next_plan_id()
{
    static uint64_t n = 0;
    return __atomic_add_fetch(&n, 1, __ATOMIC_RELAXED);
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
    // first piece with the launch's piece KiB, wave_kib_for; profiles/r03/wave_copy/).
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
            const int kib = c->wave_kib ? c->wave_kib : wave_kib_for(bytes, c->cus);
            chunk = (int64_t)kib << 10;
            wave_at[first] = (char)kib;
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
            st.groups = 1;
            st.posts = sp.posts;
            for (int i = 0; i < nc; ++i) {
                const xg_call &o = p->calls[st.call_b + i];
                if (o.kind == XG_CALL_BARRIER) {
                    st.sync_after = c->nranks > 1;
                    continue;
                }
                if (o.kind == XG_CALL_FENCE) {        // a relay step's second RCCL group follows
                    st.groups++;
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

