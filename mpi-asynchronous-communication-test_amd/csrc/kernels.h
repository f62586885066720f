// kernels.h -- CDNA4 (gfx950) kernels of the aggregator exchange.
//
// All of this path is byte movement, HBM-bound; nothing is GEMM-shaped, so no
// MFMA.  The rules that matter (MI355X_MICROARCH.md, cdna_hip_programming.md):
// 16-B per lane accesses (global_load/store_dwordx4, buffer_load/store_dwordx4),
// several loads in flight per lane before the first store, 256-thread
// workgroups (4 wave64s) and >> 256 workgroups per launch.  No workgroup of a
// copy launch reads another's output, so only the step engine (below) needs an
// inter-workgroup protocol.
//
//  fill_kernel        fill_buffer / MAP_DATA (mpi_test.c:71-77, :23): byte o of a
//                     segment of `rank` with seed `seed` = (rank + o + seed + iter)
//                     mod 256, produced 16 bytes per lane with SWAR byte adds.
//  copy_kernel_g / _b the exchange itself: one workgroup per <= chunk-byte piece of
//                     a segment transfer (local gather/scatter, pack into and unpack
//                     out of RCCL staging).  Replaces the shared-memory copies MPI
//                     does inside Irecv/Issend/Alltoallw.  Misaligned pieces (-d not
//                     a multiple of 16) are realigned through LDS.
//  step_engine_kernel a whole GPU-local run of small steps in one persistent
//                     launch: bursts per step, grid barrier + wall-clock stamp between.
//  solo_engine_kernel the same for small plans in ONE workgroup: workgroup barrier
//                     between steps, loads of later steps in flight ahead of the stores.
//  displ_scan_kernel  staging displacements of packed segments (wave64 prefix scan),
//  displ_apply_kernel the device replacement of *_alltoall_translate (:233-302).
//  verify_kernel      check_buffer (mpi_test.c:83-92) + xg_chk64 per receive slot.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace xgk {

constexpr int kThreads = 256;

struct DCopy {          // one workgroup's piece of a transfer (absolute device pointers)
    const uint8_t *src;
    uint8_t *dst;
    int64_t len;
};

struct DSeg {           // one segment to fingerprint
    int64_t off;
    int32_t rank, seed;
};

struct DSlot {          // one receive slot to verify
    int64_t off;
    int32_t src, seed;
};

constexpr uint64_t kGold = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t mix64(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// byte-wise add of two packed u32 (no carry between bytes)
__device__ __forceinline__ uint32_t add_bytes(uint32_t x, uint32_t y)
{
    return ((x & 0x7f7f7f7fu) + (y & 0x7f7f7f7fu)) ^ ((x ^ y) & 0x80808080u);
}

// 16 reference-fingerprint bytes whose first byte is b (mod 256)
__device__ __forceinline__ uint4 ramp16(uint32_t b)
{
    const uint32_t rep = (b & 0xffu) * 0x01010101u;
    uint4 v;
    v.x = add_bytes(rep, 0x03020100u);
    v.y = add_bytes(rep, 0x07060504u);
    v.z = add_bytes(rep, 0x0b0a0908u);
    v.w = add_bytes(rep, 0x0f0e0d0cu);
    return v;
}

__device__ __forceinline__ uint64_t strong_key(int rank, int seed, int iter)
{
    return ((uint64_t)(uint32_t)rank << 42) ^ ((uint64_t)(uint32_t)seed << 21) ^ (uint64_t)(uint32_t)iter;
}

// expected 8 bytes of word q of a segment (mode 0: reference ramp; 1: strong)
__device__ __forceinline__ uint64_t expect_word(int mode, uint32_t b0, uint64_t key, int64_t q)
{
    if (mode == 0) {
        const uint32_t rep = ((b0 + (uint32_t)(q * 8)) & 0xffu) * 0x01010101u;
        return (uint64_t)add_bytes(rep, 0x03020100u) | ((uint64_t)add_bytes(rep, 0x07060504u) << 32);
    }
    return mix64(key + (uint64_t)q * kGold);
}

// ---------------------------------------------------------------- fill
// The non-template kernels are static: every runtime translation unit that includes this header
// gets its own copy (no duplicate host stubs at link time); templates are merged by the linker.
[[maybe_unused]] static __global__ __launch_bounds__(kThreads) void fill_kernel(uint8_t *__restrict__ base, const DSeg *__restrict__ segs,
                                                        int chunks_per_seg, int64_t d, int64_t chunk, int iter,
                                                        int mode)
{
    const int64_t b = blockIdx.x;
    const DSeg sg = segs[b / chunks_per_seg];
    const int64_t c0 = (b % chunks_per_seg) * chunk;
    const int64_t c1 = c0 + chunk < d ? c0 + chunk : d;
    uint8_t *p = base + sg.off;
    const uint32_t b0 = (uint32_t)(sg.rank + sg.seed + iter);
    const uint64_t key = strong_key(sg.rank, sg.seed, iter);
    if ((((uintptr_t)p | (uint64_t)d) & 15) == 0) {
        for (int64_t o = c0 + (int64_t)threadIdx.x * 16; o < c1; o += kThreads * 16) {
            uint4 v;
            if (mode == 0) {
                v = ramp16(b0 + (uint32_t)o);
            } else {
                const uint64_t w0 = mix64(key + (uint64_t)(o >> 3) * kGold);
                const uint64_t w1 = mix64(key + (uint64_t)((o >> 3) + 1) * kGold);
                v.x = (uint32_t)w0; v.y = (uint32_t)(w0 >> 32); v.z = (uint32_t)w1; v.w = (uint32_t)(w1 >> 32);
            }
            *reinterpret_cast<uint4 *>(p + o) = v;
        }
    } else {
        for (int64_t o = c0 + threadIdx.x; o < c1; o += kThreads) {
            p[o] = mode == 0 ? (uint8_t)(b0 + (uint32_t)o)
                             : (uint8_t)(mix64(key + (uint64_t)(o >> 3) * kGold) >> (8 * (o & 7)));
        }
    }
}

// ---------------------------------------------------------------- copy
// Global-address-space, software-pipelined piece copy: the next U 16-B loads of
// a lane are issued before the current U stores, so U..2U loads stay in flight
// and the compiler emits global_load/store_dwordx4 (vmcnt only).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_cu4;
typedef __attribute__((address_space(1))) u32x4 g_u4;

// NT: non-temporal loads and stores (`nt`: streamed through the caches with an
// early-eviction hint -- every byte of a copy is touched once)
template <bool NT>
__device__ __forceinline__ u32x4 ld16(g_cu4 *p)
{
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

template <bool NT>
__device__ __forceinline__ void st16(g_u4 *p, u32x4 v)
{
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int U, bool NT = false>
__device__ __forceinline__ void pipelined_copy16(g_cu4 *__restrict__ s4, g_u4 *__restrict__ t4, int64_t n4)
{
    int64_t i = threadIdx.x;
    const int64_t step = (int64_t)U * kThreads;
    if (i + (U - 1) * (int64_t)kThreads < n4) {
        u32x4 cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = ld16<NT>(s4 + i + u * kThreads);
        for (; i + step + (U - 1) * (int64_t)kThreads < n4; i += step) {
            u32x4 nxt[U];
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = ld16<NT>(s4 + i + step + u * kThreads);
#pragma unroll
            for (int u = 0; u < U; ++u) st16<NT>(t4 + i + u * kThreads, cur[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st16<NT>(t4 + i + u * kThreads, cur[u]);
        i += step;
    }
    for (; i < n4; i += kThreads) st16<NT>(t4 + i, ld16<NT>(s4 + i));
}

// Raw buffer access (gfx9 buffer resource, stride 0, num_records = bytes): a load
// past num_records returns 0 and a store past it is dropped, so the partial tail
// of a transfer needs no per-lane branch.  Branch-free code matters here: with a
// branch around every load and store the compiler's waitcnt pass can no longer
// count, and puts vmcnt(0) before EVERY store (each store then waits for the
// previous one to be acknowledged).
typedef __amdgpu_buffer_rsrc_t brsrc;
constexpr int kRsrcWord3 = 0x00020000;     // gfx9 (gfx950) raw buffer, as composable_kernel
// store cache-policy bits (the `aux` operand): 0 plain, 2 nt, 16 sc1 (write-through:
// the line leaves the XCD's L2 with the store, so nothing is left dirty at kernel end)
constexpr int kAuxPlain = 0, kAuxNT = 2, kAuxSC1 = 16;

__device__ __forceinline__ brsrc make_rsrc(const void *p, int64_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, kRsrcWord3);
}

__device__ __forceinline__ u32x4 bload16(brsrc r, int off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

template <int AUX = kAuxPlain>
__device__ __forceinline__ void bstore16(brsrc r, int off, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, AUX);
}

// LDS-staged realignment for a piece whose source and destination disagree mod
// 16 (any -d that is not a multiple of 16: segment offsets k*d land on every
// phase).  The destination gets whole aligned 16-B stores: the head (< 16 B) and
// tail (< 16 B) go byte by byte, the body in 4 KiB tiles.  Per tile every lane
// loads one ALIGNED 16-B chunk of the source window into LDS (257 chunks cover a
// 4 KiB window at any phase), then reads back five dwords at its own 16-B
// position shifted by the phase and funnel-shifts them (v_alignbyte) into one
// aligned 16-B store.  Each source byte is read from HBM once; the LDS ring has
// two tiles, so one barrier per tile orders both the fill and the reuse.
constexpr int kTile = kThreads * 16;
constexpr int kTileWords = (kTile + 16) / 4;     // 257 chunks of 16 B

__device__ __forceinline__ void bytes_copy(const uint8_t *s, uint8_t *t, int64_t n)
{
    for (int64_t i = threadIdx.x; i < n; i += kThreads) t[i] = s[i];
}

__device__ void realign_copy(const uint8_t *s, uint8_t *t, int64_t n, uint32_t (*lds)[kTileWords])
{
    const int64_t head = (int64_t)((16 - ((uintptr_t)t & 15)) & 15);
    if (n < head + 16) {
        bytes_copy(s, t, n);
        return;
    }
    const int64_t body = (n - head) & ~(int64_t)15;
    bytes_copy(s, t, head);
    bytes_copy(s + head + body, t + head + body, n - head - body);
    const uint8_t *sb = s + head;                    // body source (any phase)
    uint8_t *tb = t + head;                          // body destination (16-B aligned)
    const int phase = (int)((uintptr_t)sb & 15);
    const uint8_t *sa = sb - phase;                  // aligned source window start
    // whole 16-B chunks up to the one holding the body's last byte (inside the
    // allocation: it is 16-B aligned); chunks past that read 0
    const brsrc rs = make_rsrc(sa, (phase + body + 15) & ~(int64_t)15);
    const brsrc rd = make_rsrc(tb, body);
    const int lane = (int)threadIdx.x;
    const int w0 = 4 * lane + (phase >> 2), sh = phase & 3;
    const int ntiles = (int)((body + kTile - 1) / kTile);
    u32x4 a = bload16(rs, lane * 16), b = bload16(rs, kTile);   // b: chunk 256 (lane 0 keeps it)
    for (int k = 0; k < ntiles; ++k) {
        uint32_t *L = lds[k & 1];
        *reinterpret_cast<u32x4 *>(L + 4 * lane) = a;
        if (lane == 0) *reinterpret_cast<u32x4 *>(L + 4 * kThreads) = b;
        if (k + 1 < ntiles) {                         // next tile's loads fly while this one drains
            a = bload16(rs, (k + 1) * kTile + lane * 16);
            b = bload16(rs, (k + 2) * kTile);
        }
        __syncthreads();
        const uint32_t x0 = L[w0], x1 = L[w0 + 1], x2 = L[w0 + 2], x3 = L[w0 + 3], x4 = L[w0 + 4];
        u32x4 v;
        v.x = __builtin_amdgcn_alignbyte(x1, x0, sh);
        v.y = __builtin_amdgcn_alignbyte(x2, x1, sh);
        v.z = __builtin_amdgcn_alignbyte(x3, x2, sh);
        v.w = __builtin_amdgcn_alignbyte(x4, x3, sh);
        bstore16(rd, k * kTile + lane * 16, v);
    }
}

// One workgroup per DCopy piece (<= the context's chunk bytes): copy_kernel_g<U, NT>,
// global loads/stores, U-deep software pipeline; NT: non-temporal loads and stores.
// Pieces whose pointers or length are not 16-B aligned take realign_copy.
// start != nullptr: workgroup 0 stamps the launch's start (wall clock) there -- in a
// chain of back-to-back step launches that is the time the previous step completed
// (xg_plan_run), so the steps need no timing event between them.
template <int U, bool NT = false>
__global__ __launch_bounds__(kThreads) void copy_kernel_g(const DCopy *__restrict__ pieces,
                                                          unsigned long long *start)
{
    __shared__ uint32_t lds[2][kTileWords];
    if (start && blockIdx.x == 0 && threadIdx.x == 0) *start = (unsigned long long)wall_clock64();
    const DCopy c = pieces[blockIdx.x];
    if ((((uintptr_t)c.src | (uintptr_t)c.dst | (uint64_t)c.len) & 15) == 0)
        pipelined_copy16<U, NT>((g_cu4 *)c.src, (g_u4 *)c.dst, c.len >> 4);
    else
        realign_copy(c.src, c.dst, c.len, lds);
}

// Wave-persistent piece copy: copy_kernel_w<J, NT>.  Every wave of the grid copies pieces
// wv, wv + NW, wv + 2 NW, ... (NW = waves in the grid), each of at most J KiB and 16-B
// aligned: J 16-B buffer accesses per lane, instruction j covering the piece's j-th KiB.
// While it stores piece k, the loads of piece k + 1 are in flight (two register buffers),
// so a wave never idles between pieces the way a one-piece workgroup does (exit, the next
// workgroup's dispatch, its descriptor load, then its first data load).  The descriptors
// come 64 at a time (lane l holds the wave's piece b + l) and are broadcast per piece with
// readlane; a piece's length is its buffer resources' range, so a short piece needs no branch.
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

template <int AUX>
__device__ __forceinline__ u32x4 bload16a(brsrc r, int off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, AUX);
}

constexpr int kWaveKiB = 8;       // the product's copy_kernel_w: pieces of <= 8 KiB, 8 accesses per lane

template <int J, bool NT = false>
__global__ __launch_bounds__(kThreads) void copy_kernel_w(const DCopy *__restrict__ pieces, int np,
                                                          unsigned long long *start)
{
    constexpr int AUX = NT ? kAuxNT : kAuxPlain;
    if (start && blockIdx.x == 0 && threadIdx.x == 0) *start = (unsigned long long)wall_clock64();
    const int lane = (int)(threadIdx.x & 63);
    const int NW = (int)gridDim.x * (kThreads / 64);
    // the wave's index, made provably wave-uniform (readfirstlane): every branch below is then
    // scalar, and the buffer resources stay in SGPRs (no waterfall loop around an access, and
    // the waitcnt pass can count the loads of the next piece past the stores of this one)
    const int wv = __builtin_amdgcn_readfirstlane((int)blockIdx.x * (kThreads / 64) + (int)(threadIdx.x >> 6));
    if (wv >= np) return;
    const int n = (np - 1 - wv) / NW + 1;                  // pieces of this wave
    uint64_t ds = 0, dd = 0;
    int dl = 0;
    auto fetch = [&](int b) {                              // descriptors of pieces b .. b + 63
        const int k = b + lane;
        if (k < n) {
            const DCopy c = pieces[wv + (int64_t)k * NW];
            ds = (uint64_t)c.src; dd = (uint64_t)c.dst; dl = (int)c.len;
        }
    };
    struct Rs { brsrc s, d; };
    auto piece = [&](int k) -> Rs {
        const int l = k & 63, len = __builtin_amdgcn_readlane(dl, l);
        return {make_rsrc((const void *)readlane64(ds, l), len), make_rsrc((const void *)readlane64(dd, l), len)};
    };
    auto load = [&](u32x4 *v, const Rs &p) {
#pragma unroll
        for (int j = 0; j < J; ++j) v[j] = bload16a<AUX>(p.s, lane * 16 + j * 1024);
    };
    auto store = [&](const u32x4 *v, const Rs &p) {
#pragma unroll
        for (int j = 0; j < J; ++j) bstore16<AUX>(p.d, lane * 16 + j * 1024, v[j]);
    };
    auto next = [&](int k) -> Rs {                         // piece k's resources (k < n)
        if ((k & 63) == 0) fetch(k);
        return piece(k);
    };
    u32x4 a[J], b[J];
    fetch(0);
    Rs pa = piece(0), pb;
    load(a, pa);
    for (int k = 0;; k += 2) {
        if (k + 1 < n) {
            pb = next(k + 1);
            load(b, pb);
        }
        store(a, pa);
        if (k + 1 >= n) break;
        if (k + 2 < n) {
            pa = next(k + 2);
            load(a, pa);
        }
        store(b, pb);
        if (k + 2 >= n) break;
    }
}

// the wall clock after everything before it on the stream: closes a chain of step launches
[[maybe_unused]] static __global__ void clock_kernel(unsigned long long *t)
{
    if (threadIdx.x == 0) *t = (unsigned long long)wall_clock64();
}

// ---------------------------------------------------------------- step engine
// A GPU-local plan of many small steps (sync / pairwise / throttled schedules
// at small -d) is bound by the per-step kernel boundary + timing event, not by
// HBM.  The engine runs the whole plan in ONE launch of W co-resident
// workgroups: step s = units [step_begin[s], step_begin[s+1]) strided over the
// workgroups, then a grid barrier whose last arriver stamps the step's
// completion time (wall clock).
//
// What the barrier after step s must order is decided per step by the host
// (xg_engine_hazards, include/xg_sched.h), flag[s]:
//   0  nothing: step s+1 neither reads bytes written since the last ordering
//      point nor rewrites them with different bytes.  A workgroup arrives as
//      soon as its stores of step s are ISSUED (they may still land while step
//      s+1 runs) and loads its first unit of step s+1 while the barrier is
//      pending.  The stamp is then the step's issue time, not its delivery.
//   1  timing: every wave waits for its stores (vmcnt 0) before arriving, so
//      the stamp is a delivered time (the last step: it anchors every step time).
//   2  hazard (step s+1 reads, or rewrites with other bytes, what was written
//      since the last such point): stores drained, then the agent-scope
//      release/acquire pair of cdna_hip_programming.md Guideline 16 around the
//      barrier (release fence by one lane before arriving, acquire fence after
//      the wait, before any load of step s+1), and no early load.
// State: a cumulative ticket counter (never reset between launches: each launch
// gets the tickets taken before it as `base`; the host re-zeroes it only after a
// timeout) and a timeout word.  Spins are bounded: a timed-out workgroup sets
// the word and leaves, so a broken residency assumption ends the launch
// instead of hanging; the host checks the word after the launch (xg_plan_check).
struct EngineState {
    unsigned count;     // arrival tickets, cumulative over every launch of the plan
    unsigned tmo;       // != 0: some workgroup gave up waiting
    // solo engine, armed launches (cumulative counters; a launch adds one per rail):
    unsigned rails;     // rails finished: the last of a launch rings `done`
    unsigned arrive;    // rails resident: the last lets rail 0 announce `ready`
    unsigned pad[4];
    // relay: rail 0 saw the ring of this epoch -- written to kGoLines separate 128-B lines
    // at once (one store per lane), rail r polls line r % kGoLines, so hundreds of
    // polling rails do not queue on one L2 line
    unsigned go[16][32];
    // rails finished, counted on the same 16 lines (rail r on line r % 16); the last of
    // a line counts on `rails`, the last of those rings `done` (two short queues of
    // atomics instead of one of R)
    unsigned fin[16][32];
};
constexpr int kGoLines = 16;


template <int B>
__device__ __forceinline__ void burst_load16(const uint8_t *src, int64_t len, u32x4 *v)
{
    const brsrc r = make_rsrc(src, len);
#pragma unroll
    for (int k = 0; k < B; ++k) v[k] = bload16(r, ((int)threadIdx.x + k * kThreads) * 16);
}

template <int B>
__device__ __forceinline__ void burst_store16(uint8_t *dst, int64_t len, const u32x4 *v)
{
    const brsrc r = make_rsrc(dst, len);
#pragma unroll
    for (int k = 0; k < B; ++k) bstore16(r, ((int)threadIdx.x + k * kThreads) * 16, v[k]);
}

// Doorbell (host-pinned memory, one per plan): an ARMED engine launch announces
// `ready` once it runs and waits for the host to ring before its first step, so
// the launch and dispatch latency falls before the timed region starts (as a
// persistent MPI request is set up before MPI_Start); `done` is written after
// the last step's stores are performed.  Every word is accessed with
// system-scope vector loads/stores by one lane; every wait is bounded.
struct Doorbell {
    unsigned ring, ready, done, pad;
};

typedef __attribute__((address_space(1))) unsigned g_u32;

constexpr unsigned kRingSpins = 1u << 26;     // ~2 s of s_sleep(1) polls: then give up

// lane 0: announce, wait for the ring; false = gave up (the launch does nothing)
__device__ __forceinline__ bool wait_ring(Doorbell *db, unsigned epoch)
{
    g_u32 *ring = (g_u32 *)&db->ring;
    __hip_atomic_store((g_u32 *)&db->ready, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (unsigned spins = 0; __hip_atomic_load(ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != epoch;) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kRingSpins) return false;
    }
    return true;
}

__device__ __forceinline__ void ring_done(Doorbell *db, unsigned epoch)
{
    __hip_atomic_store((g_u32 *)&db->done, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// lane 0: wait until *w == v (SYS: a host-memory word, else device memory) or the
// timeout word is set; false = gave up
template <bool SYS>
__device__ __forceinline__ bool poll_word(g_u32 *w, unsigned v, g_u32 *tmo)
{
    for (unsigned spins = 0;; ++spins) {
        const unsigned x = SYS ? __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                               : __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (x == v) return true;
        if (spins > kRingSpins || __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
        __builtin_amdgcn_s_sleep(1);
    }
}

// lane 0 of a finished rail: count it; the launch's last rail tells the host
__device__ __forceinline__ void rail_finished(EngineState *st, int rail, int R, Doorbell *db, unsigned epoch)
{
    const int L = R < kGoLines ? R : kGoLines;
    const int line = rail % L;
    const unsigned per_line = (unsigned)((R - line - 1) / L + 1);     // rails on this line
    const unsigned a = __hip_atomic_fetch_add((g_u32 *)&st->fin[line][0], 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (a % per_line) return;
    const unsigned b = __hip_atomic_fetch_add((g_u32 *)&st->rails, 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (b % (unsigned)L == 0) ring_done(db, epoch);
}

// B: 16-B loads per lane per unit -> units of B * 4 KiB (the host cuts the step's
// transfers to that size and picks B so that a step has enough units to spread).
// db != nullptr: armed launch -- workgroup 0 waits for the ring, then every
// workgroup passes one extra grid barrier (tickets base .. base + W) before step 0.
template <int B>
__global__ __launch_bounds__(kThreads) void step_engine_kernel(const DCopy *__restrict__ pieces,
                                                               const int *__restrict__ step_begin, int nsteps,
                                                               EngineState *st, unsigned long long *stamps,
                                                               unsigned base, Doorbell *db, unsigned epoch)
{
    // compare tickets by difference, which is wrap-safe
    const unsigned W = gridDim.x;
    g_u32 *count = (g_u32 *)&st->count;
    g_u32 *tmo = (g_u32 *)&st->tmo;
    __shared__ int give_up;
    if (threadIdx.x == 0) give_up = 0;
    __syncthreads();
    if (db) {
        if (threadIdx.x == 0) {
            bool ok = blockIdx.x != 0 || wait_ring(db, epoch);
            if (!ok) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned target = base + W;
            __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            for (unsigned spins = 0;
                 (int)(__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0;) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > kRingSpins || __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
            if (__hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) give_up = 1;
        }
        __syncthreads();
        if (give_up) {
            if (blockIdx.x == 0 && threadIdx.x == 0) ring_done(db, epoch);
            return;
        }
        base += W;
    }
    // This workgroup's first unit of the next step is LOADED while the barrier is
    // pending (into v[]) and stored once it opens: the load latency of each step
    // (HBM + address translation of fresh pages) overlaps the barrier.  pf is
    // workgroup-uniform.
    const int *flag = step_begin + nsteps + 1;     // per-step flags (host: xg_engine_hazards)
    bool pf = false;
    DCopy nc = {nullptr, nullptr, 0};
    u32x4 v[B];
    for (int s = 0; s < nsteps; ++s) {
        const int e = step_begin[s + 1];
        int i = step_begin[s] + (int)blockIdx.x;
        if (pf) {
            burst_store16<B>(nc.dst, nc.len, v);
            i += (int)W;
            pf = false;
        }
        for (; i < e; i += (int)W) {
            const DCopy c = pieces[i];       // <= B * 4 KiB
            if ((((uintptr_t)c.src | (uintptr_t)c.dst | (uint64_t)c.len) & 15) == 0) {
                u32x4 w[B];
                burst_load16<B>(c.src, c.len, w);
                burst_store16<B>(c.dst, c.len, w);
            } else {
                bytes_copy(c.src, c.dst, c.len);
            }
        }
        const int fl = flag[s];
        if (fl) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores performed
        __syncthreads();
        const unsigned target = base + (unsigned)(s + 1) * W;
        bool last = false;
        if (threadIdx.x == 0) {
            if (fl == 2) {               // publish: write the XCD's L2 back before arriving
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const unsigned t = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
            last = t == target;
            if (last) {
                stamps[s] = (unsigned long long)wall_clock64();
                if (db && s + 1 == nsteps) ring_done(db, epoch);
            }
        }
        if (s + 1 < nsteps && fl != 2) {   // step s+1 reads nothing written since the last hazard point
            const int j = step_begin[s + 1] + (int)blockIdx.x;
            if (j < step_begin[s + 2]) {
                nc = pieces[j];
                pf = (((uintptr_t)nc.src | (uintptr_t)nc.dst | (uint64_t)nc.len) & 15) == 0;
                if (pf) burst_load16<B>(nc.src, nc.len, v);
            }
        }
        if (threadIdx.x == 0 && !last) {
            unsigned spins = 0;
            while ((int)(__hip_atomic_load(count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) < 0) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1u << 22) || __hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    give_up = 1;
                    break;
                }
            }
        }
        if (fl == 2 && threadIdx.x == 0) {   // acquire: drop this CU's stale L1 lines
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (give_up) return;
    }
}

// ---------------------------------------------------------------- solo engine
// The same plans when they are small (README-sized latency chains: tens of steps
// of tens of KiB): workgroups of 16 waves -- RAILS -- each run every step on their
// own CU, so the step boundary is a workgroup barrier (tens of ns) instead of a
// grid barrier across CUs (~1 us of device-scope atomics and polling).  The host
// deals each step's 1 KiB pieces round-robin over the rails (a message striped
// over R links, as a multi-rail network does); rail r cuts its share into rows of
// 16 pieces, piece (row, w) moved by wave w (64 lanes x 16 B), rows packed back to
// back across steps.  K rows are loaded at once (every lane has K 16-B loads in
// flight, 16 x K KiB per workgroup) and stored in order, with a barrier + wall-
// clock stamp wherever a step that had pieces on this rail ends: the loads of
// later steps run ahead of the stores of earlier ones -- valid because no step
// reads what another writes (the host uses this engine only for plans without
// hazard points, xg_engine_hazards) -- while each rail's stores keep the step
// order.  Rails never wait for each other: step s is over when every rail has
// closed it, so its time is the MAX over rails of their stamps for it (a rail with
// nothing in step s carries its previous stamp; the host reduces).  Like flag 0 of
// the grid engine a stamp is the time the stores were issued; the last step waits
// for its stores (delivered time).  One CU moves ~120 GB/s of load + store
// traffic, so R rails lift the single-workgroup bound R-fold.  A rail is a
// workgroup of WV = 16 waves (rows of 16 pieces, workgroup barriers between
// steps) or a single wave (WV = 1: rows of one piece; a wave's stores issue in
// program order, so its step boundaries cost no barrier at all).
constexpr int kSoloWaves = 16;
constexpr int kSoloThreads = kSoloWaves * 64;
constexpr int kSoloPiece = 64 * 16;              // bytes per wave per row
constexpr int kSoloK = 8;                        // rows per chunk (2 chunks x 8 x 16 KiB in flight)
constexpr int kSoloMaxSteps = 2048;              // stamps kept in LDS (16 KiB)
constexpr int kSoloMaxPieces = 4608;             // descriptors per rail kept in LDS (36 KiB)

// One solo piece in 64 bits: source and destination offsets (16-B units, 24 bits)
// from the segment's two base pointers, the length (16-B units, <= 64, 7 bits) and
// `before` (5 bits, from bit 55): how many of its row's step barriers come before this
// piece.  Steps are packed back to back, so a row may hold the end of one step and the
// start of the next: every wave executes all of the row's barriers, its store after
// the first `before` of them.  (Other granules: SoloFmt below.)
constexpr uint64_t kSoloOffMax = 1ull << 24;     // offsets < 256 MiB from the bases
constexpr int kSoloMaxRails = 512;

// Granule G of a segment's descriptors (xg_solo_tables_g): offsets and lengths in units of
// G bytes.  G = 16: one 16-B access per lane per piece (the form above); G = 4 / 1, for
// segment sizes that are not multiples of 16: 4 dword / 16 byte accesses per lane, access
// j of lane l at G * (l + 64 j) -- each instruction covers 64 consecutive granules of the
// piece -- and the range check drops the granules past its end exactly.  The length field
// widens (7 / 9 / 11 bits for up to 1 KiB), so `before` moves up (55 / 57 / 59).
// One-wave rails (WV = 1) use the WIDE form instead: a row is one piece, so the row's
// barrier word carries the piece's length (bits 8-19, granules) beside its barrier count
// (bits 0-7; every barrier of the row precedes its one piece, so `before` = the count),
// and the 64-bit descriptor holds two 32-bit offsets in granules: windows of 4 GiB (G = 1)
// to 64 GiB (G = 16) instead of 16-256 MiB, so a run whose sources or destinations span
// a whole large region (16384 logical ranks on one GPU) still fits one table.
constexpr uint64_t kSoloWideOffMax = 1ull << 32;

template <int G>
struct SoloFmt {
    static constexpr int kShift = G == 16 ? 4 : G == 4 ? 2 : 0;       // log2 G
    static constexpr int kLenBits = G == 16 ? 7 : G == 4 ? 9 : 11;
    static constexpr int kBefore = 48 + kLenBits;
    static constexpr int kNV = G == 1 ? 16 : 4;                       // registers per lane per piece
};

// Host contract (build_segments), per rail r of R = gridDim.x: pieces
// desc[r * npieces ..], every piece 16-B aligned, <= 1 KiB, within 256 MiB of the
// bases; rows form an even number of chunks of K plus one spare empty chunk;
// meta = [R][nrows + 1] row_close (step barriers inside or in front of row r, each
// piece's `before` saying where it sits among them), then [R][nsteps] the step
// each barrier closes, in order (-1 past the last); nsteps <= kSoloMaxSteps;
// npieces <= kSoloMaxPieces.  The descriptor table is staged into LDS before the
// doorbell (plan set-up: no payload byte moves before the ring), read back a chunk
// at a time in one batch; each piece becomes a buffer resource whose range check
// drops the lanes past its end (an empty padding piece moves nothing), so the body
// has no branch but the step barriers.  stamps[r * stride + t]: rail r's stamp of
// step t, 0 where it closed nothing (the host carries and reduces).
template <int K, int G = 16>
struct SoloChunk {
    unsigned long long d[K];
    uint32_t v[K][SoloFmt<G>::kNV];
};

// the wave-uniform descriptor of a piece (SGPRs)
__device__ __forceinline__ unsigned long long solo_uniform(unsigned long long d)
{
    return ((unsigned long long)__builtin_amdgcn_readfirstlane((int)(d >> 32)) << 32) |
           (unsigned)__builtin_amdgcn_readfirstlane((int)d);
}

// a piece's source / destination offsets and length in granules, from its descriptor and
// (wide form, WV = 1) its row's barrier word
template <int WV, int G>
__device__ __forceinline__ uint64_t solo_src(unsigned long long d)
{
    return WV == 1 ? (d & 0xFFFFFFFFull) : (d & (kSoloOffMax - 1));
}
template <int WV, int G>
__device__ __forceinline__ uint64_t solo_dst(unsigned long long d)
{
    return WV == 1 ? (d >> 32) : ((d >> 24) & (kSoloOffMax - 1));
}
template <int WV, int G>
__device__ __forceinline__ int64_t solo_len(unsigned long long d, unsigned row_word)
{
    return WV == 1 ? (int64_t)((row_word >> 8) & 0xFFF) : (int64_t)((d >> 48) & ((1u << SoloFmt<G>::kLenBits) - 1));
}
template <int WV>
using SoloRowT = typename std::conditional<WV == 1, unsigned, unsigned short>::type;

// issue the loads of chunk c of this wave (rows of WV pieces)
template <int K, int WV, int G>
__device__ __forceinline__ void solo_load(SoloChunk<K, G> &b, const unsigned long long *ldesc,
                                          const SoloRowT<WV> *lclose, int c, int wave, uint64_t l16,
                                          const uint8_t *src_base)
{
    using F = SoloFmt<G>;
#pragma unroll
    for (int k = 0; k < K; ++k) b.d[k] = ldesc[(c * K + k) * WV + wave];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        // the descriptor is wave-uniform: a buffer resource in SGPRs whose range check
        // (num_records = the piece's bytes) drops the lanes past its end -- an empty
        // padding piece moves nothing
        const unsigned long long d = solo_uniform(b.d[k]);
        const unsigned rw = WV == 1 ? (unsigned)__builtin_amdgcn_readfirstlane((int)lclose[c * K + k]) : 0u;
        const brsrc r = make_rsrc(src_base + (solo_src<WV, G>(d) << F::kShift), solo_len<WV, G>(d, rw) << F::kShift);
        if constexpr (G == 16) {
            const u32x4 x = bload16(r, (int)l16 * 16);
            b.v[k][0] = x.x; b.v[k][1] = x.y; b.v[k][2] = x.z; b.v[k][3] = x.w;
        } else if constexpr (G == 4) {
#pragma unroll
            for (int j = 0; j < 4; ++j) b.v[k][j] = __builtin_amdgcn_raw_buffer_load_b32(r, 4 * ((int)l16 + 64 * j), 0, 0);
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) b.v[k][j] = __builtin_amdgcn_raw_buffer_load_b8(r, (int)l16 + 64 * j, 0, 0);
        }
    }
}

// barrier k of this rail: every wave has issued its stores of the step it closes; stamp it
__device__ __forceinline__ void solo_close(unsigned long long *ts, const short *lcstep, int &k)
{
    __syncthreads();
    if (threadIdx.x == 0) ts[lcstep[k]] = (unsigned long long)wall_clock64();
    ++k;
}

// store chunk c in row order; a row that begins new steps first closes the ones before
// it: barrier (every wave issued their stores), stamp
template <int K, int WV, int G>
__device__ __forceinline__ void solo_store(const SoloChunk<K, G> &b, const SoloRowT<WV> *lclose, const short *lcstep,
                                          unsigned long long *ts, int &s, int c, int rows, uint64_t l16,
                                          uint8_t *dst_base)
{
    using F = SoloFmt<G>;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        if (c * K + k >= rows) break;         // padding rows: no piece, no barrier
        const unsigned rw = (unsigned)__builtin_amdgcn_readfirstlane((int)lclose[c * K + k]);
        const int n = WV == 1 ? (int)(rw & 0xFF) : (int)rw;                      // barriers in this row
        // ... before my piece (wide form: all of them)
        const int bf = WV == 1 ? n : __builtin_amdgcn_readfirstlane((int)(b.d[k] >> F::kBefore));
        int j = 0;
        for (; j < bf; ++j) solo_close(ts, lcstep, s);
        asm volatile("" ::: "memory");        // the store stays between its steps' barriers
        const unsigned long long d = solo_uniform(b.d[k]);
        const brsrc r = make_rsrc(dst_base + (solo_dst<WV, G>(d) << F::kShift), solo_len<WV, G>(d, rw) << F::kShift);
        if constexpr (G == 16) {
            u32x4 x;
            x.x = b.v[k][0]; x.y = b.v[k][1]; x.z = b.v[k][2]; x.w = b.v[k][3];
            bstore16(r, (int)l16 * 16, x);
        } else if constexpr (G == 4) {
#pragma unroll
            for (int q = 0; q < 4; ++q) __builtin_amdgcn_raw_buffer_store_b32(b.v[k][q], r, 4 * ((int)l16 + 64 * q), 0, 0);
        } else {
#pragma unroll
            for (int q = 0; q < 16; ++q)
                __builtin_amdgcn_raw_buffer_store_b8((unsigned char)b.v[k][q], r, (int)l16 + 64 * q, 0, 0);
        }
        asm volatile("" ::: "memory");
        for (; j < n; ++j) solo_close(ts, lcstep, s);
    }
}

template <int K, int WV, int G = 16>
__global__ __launch_bounds__(WV * 64) void solo_engine_kernel(const unsigned long long *__restrict__ desc,
                                                                   int npieces, const uint8_t *src_base,
                                                                   uint8_t *dst_base, const int *__restrict__ meta,
                                                                   int nsteps, EngineState *st,
                                                                   unsigned long long *stamps, int stride,
                                                                   Doorbell *db, unsigned epoch)
{
    const int wave = (int)threadIdx.x >> 6, lane = (int)threadIdx.x & 63;
    const int rail = (int)blockIdx.x, R = (int)gridDim.x;
    __shared__ unsigned long long ldesc[kSoloMaxPieces];
    __shared__ SoloRowT<WV> lclose[kSoloMaxPieces / WV + 1];
    __shared__ short lcstep[kSoloMaxSteps];
    __shared__ unsigned long long ts[kSoloMaxSteps];
    __shared__ int give_up;
    constexpr int kT = WV * 64;
    const int nrows = npieces / WV;
    desc += (size_t)rail * npieces;
    const int *row_close = meta + rail * (nrows + 1);
    const int *cstep = meta + R * (nrows + 1) + rail * nsteps;
    const int rows = meta[R * (nrows + 1) + R * nsteps + rail];     // rows holding real pieces
    const int nreal = (rows + K - 1) / K;                              // ... in that many chunks
    for (int i = (int)threadIdx.x; i < npieces; i += kT) ldesc[i] = desc[i];
    for (int i = (int)threadIdx.x; i <= nrows; i += kT) lclose[i] = (SoloRowT<WV>)row_close[i];
    for (int i = (int)threadIdx.x; i < nsteps; i += kT) {
        lcstep[i] = (short)cstep[i];
        ts[i] = 0;
    }
    // armed: every rail resident, then rail 0 announces `ready`; the ring reaches the
    // rails through rail 0, which alone polls the host and relays the epoch in device memory
    // (hundreds of rails polling host memory take ~45 us to all see it)
    __shared__ int relay_now;
    if (threadIdx.x == 0) {
        bool ok = true, relay_go = false;
        if (db) {
            g_u32 *tmo = (g_u32 *)&st->tmo;
            const unsigned old = __hip_atomic_fetch_add((g_u32 *)&st->arrive, 1u, __ATOMIC_RELAXED,
                                                        __HIP_MEMORY_SCOPE_AGENT);
            if (rail == 0) {
                const unsigned all = (old / (unsigned)R + 1) * (unsigned)R;
                for (unsigned spins = 0; ok && (int)(__hip_atomic_load((g_u32 *)&st->arrive, __ATOMIC_RELAXED,
                                                                       __HIP_MEMORY_SCOPE_AGENT) - all) < 0; ++spins) {
                    __builtin_amdgcn_s_sleep(1);
                    ok = spins < kRingSpins;
                }
                ok = ok && wait_ring(db, epoch);
                if (!ok) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else relay_go = true;
            } else {
                ok = poll_word<false>((g_u32 *)&st->go[rail % kGoLines][0], epoch, tmo);
                if (!ok) __hip_atomic_store(tmo, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        give_up = !ok;
        relay_now = relay_go;
    }
    __syncthreads();
    if (relay_now && threadIdx.x < kGoLines)   // one store per lane: every relay line at once
        __hip_atomic_store((g_u32 *)&st->go[threadIdx.x][0], epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (give_up) {
        if (threadIdx.x == 0) rail_finished(st, rail, R, db, epoch);   // still counted
        return;
    }
    const uint64_t l16 = (uint64_t)lane;
    // double buffer: chunk c+1's loads fly while chunk c stores.  The host pads the
    // table to an even number of chunks plus one spare empty chunk, so the loads below
    // need no bounds branch (a conditional one would make the compiler wait on it);
    // the loop leaves after the last chunk that holds real pieces.
    SoloChunk<K, G> A, B;
    int k = 0;
    solo_load<K, WV, G>(A, ldesc, lclose, 0, wave, l16, src_base);
    for (int c = 0; c < nreal; c += 2) {
        solo_load<K, WV, G>(B, ldesc, lclose, c + 1, wave, l16, src_base);
        solo_store<K, WV, G>(A, lclose, lcstep, ts, k, c, rows, l16, dst_base);
        if (c + 1 >= nreal) break;
        solo_load<K, WV, G>(A, ldesc, lclose, c + 2, wave, l16, src_base);
        solo_store<K, WV, G>(B, lclose, lcstep, ts, k, c + 1, rows, l16, dst_base);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this rail's last steps: delivered
    __syncthreads();
    __shared__ unsigned long long t_end;                // the steps after its last barrier end here
    __shared__ int s_end;
    if (threadIdx.x == 0) {
        t_end = (unsigned long long)wall_clock64();
        s_end = k > 0 ? lcstep[k - 1] + 1 : 0;
        if (db) rail_finished(st, rail, R, db, epoch);      // the last rail to finish tells the host
    }
    __syncthreads();
    for (int i = (int)threadIdx.x; i < nsteps; i += kT) stamps[(size_t)rail * stride + i] = i >= s_end ? t_end : ts[i];
}

// ---------------------------------------------------------------- displacement scan
// The device replacement of *_alltoall_translate's displacement loops
// (mpi_test.c:233-302): staging displacements of the packed per-peer segments of
// one step = exclusive prefix sum of their lengths.  One workgroup per group
// (a step's pack list or unpack list, groups[g] .. groups[g+1]): wave64 inclusive
// scan with shuffles, wave totals through LDS, a carry across 256-entry tiles.  disp[i] = base + sum of len[j] for j < i inside the group.
[[maybe_unused]] static __global__ __launch_bounds__(kThreads) void displ_scan_kernel(const int64_t *__restrict__ len,
                                                              const int *__restrict__ groups,
                                                              const int64_t *__restrict__ group_base,
                                                              int64_t *__restrict__ disp)
{
    __shared__ int64_t wsum[kThreads / 64];
    __shared__ int64_t carry;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = groups[blockIdx.x], e = groups[blockIdx.x + 1];
    if (threadIdx.x == 0) carry = group_base[blockIdx.x];
    __syncthreads();
    for (int t = b; t < e; t += kThreads) {
        const int i = t + (int)threadIdx.x;
        const int64_t x0 = i < e ? len[i] : 0;
        int64_t x = x0;                                // inclusive scan inside the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        int64_t before = carry;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        if (i < e) disp[i] = before + x - x0;
        __syncthreads();
        if (threadIdx.x == kThreads - 1) carry = before + x;
        __syncthreads();
    }
}

// Piece table fix-up after the scan: piece k of a packed copy c moves
// [o, o + len) of it; its staging side (dst of a pack, src of an unpack) is
// staging base + disp[c] + o.
struct DFix {
    int piece;          // index into the plan's piece table
    int copy;           // index into disp[]
    int64_t off;        // byte offset of the piece inside its copy
    int side;           // 0: patch dst (pack), 1: patch src (unpack)
    int pad;
};

[[maybe_unused]] static __global__ __launch_bounds__(kThreads) void displ_apply_kernel(DCopy *__restrict__ pieces, const DFix *__restrict__ fix,
                                                               int nfix, const int64_t *__restrict__ disp,
                                                               uint8_t *stage_send, uint8_t *stage_recv)
{
    const int k = blockIdx.x * kThreads + threadIdx.x;
    if (k >= nfix) return;
    const DFix f = fix[k];
    if (f.side == 0) pieces[f.piece].dst = stage_send + disp[f.copy] + f.off;
    else pieces[f.piece].src = stage_recv + disp[f.copy] + f.off;
}

// ---------------------------------------------------------------- verify
__device__ __forceinline__ uint64_t wave_sum(uint64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ uint64_t wave_min(uint64_t v)
{
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

// grid: slots x chunks; each lane hashes 8-byte words.  chk excludes the
// length term (added on the host); first_bad = UINT64_MAX when clean.
[[maybe_unused]] static __global__ __launch_bounds__(kThreads) void verify_kernel(const uint8_t *__restrict__ base,
                                                          const DSlot *__restrict__ slots, int chunks_per_slot,
                                                          int64_t d, int64_t chunk, int iter, int mode,
                                                          unsigned long long *chk, unsigned long long *bad,
                                                          unsigned long long *first_bad)
{
    const int64_t b = blockIdx.x;
    const int si = (int)(b / chunks_per_slot);
    const DSlot sl = slots[si];
    const int64_t c0 = (b % chunks_per_slot) * chunk;           // chunk is a multiple of 8
    const int64_t c1 = c0 + chunk < d ? c0 + chunk : d;
    const uint8_t *p = base + sl.off;
    const uint32_t b0 = (uint32_t)(sl.src + sl.seed + iter);
    const uint64_t key = strong_key(sl.src, sl.seed, iter);
    const bool aligned = (((uintptr_t)p) & 7) == 0;
    uint64_t sum = 0, nbad = 0, first = ~0ull;
    for (int64_t o = c0 + (int64_t)threadIdx.x * 8; o < c1; o += kThreads * 8) {
        const int64_t q = o >> 3;
        const int nb = c1 - o >= 8 ? 8 : (int)(c1 - o);
        uint64_t w = 0;
        if (aligned && nb == 8) {
            w = *reinterpret_cast<const uint64_t *>(p + o);
        } else {
            for (int j = 0; j < nb; ++j) w |= (uint64_t)p[o + j] << (8 * j);
        }
        uint64_t e = expect_word(mode, b0, key, q);
        if (nb < 8) e &= (1ull << (8 * nb)) - 1;
        sum += mix64(w ^ ((uint64_t)q * kGold));
        uint64_t x = w ^ e;
        if (x) {
            for (int j = 0; j < nb; ++j)
                if ((x >> (8 * j)) & 0xff) {
                    ++nbad;
                    if ((uint64_t)(o + j) < first) first = (uint64_t)(o + j);
                }
        }
    }
    sum = wave_sum(sum);
    nbad = wave_sum(nbad);
    first = wave_min(first);
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&chk[si], (unsigned long long)sum);
        if (nbad) {
            atomicAdd(&bad[si], (unsigned long long)nbad);
            atomicMin(&first_bad[si], (unsigned long long)first);
        }
    }
}

}  // namespace xgk
