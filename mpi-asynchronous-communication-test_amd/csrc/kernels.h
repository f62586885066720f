// kernels.h -- CDNA4 (gfx950) kernels of the aggregator exchange.
//
// All of this path is byte movement, HBM-bound; nothing is GEMM-shaped, so no
// MFMA.  The rules that matter (MI355X_MICROARCH.md, cdna_hip_programming.md):
// 16-B per lane accesses (global_load/store_dwordx4), several loads in flight
// per lane before the first store, 256-thread workgroups (4 wave64s) and
// >> 256 workgroups per launch.  No workgroup reads another's output inside a
// launch, so no inter-workgroup hand-off protocol is needed.
//
//  fill_kernel   fill_buffer / MAP_DATA (mpi_test.c:71-77, :23): byte o of a
//                segment of `rank` with seed `seed` = (rank + o + seed + iter)
//                mod 256, produced 16 bytes per lane with SWAR byte adds.
//  copy_kernel_g the exchange itself (default variant; copy_kernel / copy_kernel_b
//                are measured alternatives): one workgroup per <= chunk-byte piece
//                of a segment transfer (local gather/scatter, pack into and unpack
//                out of RCCL staging).  Replaces the shared-memory copies MPI
//                does inside Irecv/Issend/Alltoallw.
//  step_engine_kernel  a whole GPU-local plan of small steps in one persistent
//                launch: bursts per step, grid barrier + wall-clock stamp between.
//  verify_kernel check_buffer (mpi_test.c:83-92) + xg_chk64 per receive slot.
//  span_*, read_only, write_only, gridstride_copy: HBM ceiling microbenchmarks
//                (xg_copy_ceiling), not on the exchange path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

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
__global__ __launch_bounds__(kThreads) void fill_kernel(uint8_t *__restrict__ base, const DSeg *__restrict__ segs,
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
template <bool NT>
__device__ __forceinline__ void st16(uint4 *p, uint4 v)
{
    if constexpr (NT) {
        __builtin_nontemporal_store(v.x, &p->x);
        __builtin_nontemporal_store(v.y, &p->y);
        __builtin_nontemporal_store(v.z, &p->z);
        __builtin_nontemporal_store(v.w, &p->w);
    } else {
        *p = v;
    }
}

// One workgroup per DCopy piece.  U independent 16-B loads per lane are in
// flight before the first store (4 KiB per wave-group step, U*4 KiB per block
// iteration).
template <int U, bool NT>
__global__ __launch_bounds__(kThreads) void copy_kernel(const DCopy *__restrict__ pieces)
{
    const DCopy c = pieces[blockIdx.x];
    const uint8_t *s = c.src;
    uint8_t *t = c.dst;
    const int64_t n = c.len;
    if ((((uintptr_t)s | (uintptr_t)t | (uint64_t)n) & 15) == 0) {
        const uint4 *__restrict__ s4 = reinterpret_cast<const uint4 *>(s);
        uint4 *__restrict__ t4 = reinterpret_cast<uint4 *>(t);
        const int64_t n4 = n >> 4;
        int64_t i = threadIdx.x;
        for (; i + (int64_t)(U - 1) * kThreads < n4; i += (int64_t)U * kThreads) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = s4[i + u * kThreads];
#pragma unroll
            for (int u = 0; u < U; ++u) st16<NT>(t4 + i + u * kThreads, v[u]);
        }
        for (; i < n4; i += kThreads) st16<NT>(t4 + i, s4[i]);
    } else if ((((uintptr_t)s ^ (uintptr_t)t) & 3) == 0) {
        // same 4-byte phase: byte head, dword body, byte tail
        int64_t head = (4 - ((uintptr_t)s & 3)) & 3;
        if (head > n) head = n;
        if ((int64_t)threadIdx.x < head) t[threadIdx.x] = s[threadIdx.x];
        const int64_t nw = (n - head) >> 2;
        const uint32_t *s1 = reinterpret_cast<const uint32_t *>(s + head);
        uint32_t *t1 = reinterpret_cast<uint32_t *>(t + head);
        for (int64_t i = threadIdx.x; i < nw; i += kThreads) t1[i] = s1[i];
        for (int64_t i = head + nw * 4 + threadIdx.x; i < n; i += kThreads) t[i] = s[i];
    } else {
        for (int64_t i = threadIdx.x; i < n; i += kThreads) t[i] = s[i];
    }
}

// Global-address-space, software-pipelined variant: the next U 16-B loads of a
// lane are issued before the current U stores, so U..2U loads stay in flight
// and the compiler emits global_load/store_dwordx4 (vmcnt only) instead of
// flat ops (which also wait on lgkmcnt).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 g_cu4;
typedef __attribute__((address_space(1))) u32x4 g_u4;

// LP / SP: load / store cache policy, 0 = default, 1 = nontemporal (`nt` bit)
template <int LP>
__device__ __forceinline__ u32x4 ld16(g_cu4 *p)
{
    if constexpr (LP == 1) return __builtin_nontemporal_load(p);
    else return *p;
}

template <int SP>
__device__ __forceinline__ void st16g(g_u4 *p, u32x4 v)
{
    if constexpr (SP == 1) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int U, int LP = 0, int SP = 0>
__device__ __forceinline__ void pipelined_copy16(g_cu4 *__restrict__ s4, g_u4 *__restrict__ t4, int64_t n4)
{
    int64_t i = threadIdx.x;
    const int64_t step = (int64_t)U * kThreads;
    if (i + (U - 1) * (int64_t)kThreads < n4) {
        u32x4 cur[U];
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = ld16<LP>(s4 + i + u * kThreads);
        for (; i + step + (U - 1) * (int64_t)kThreads < n4; i += step) {
            u32x4 nxt[U];
#pragma unroll
            for (int u = 0; u < U; ++u) nxt[u] = ld16<LP>(s4 + i + step + u * kThreads);
#pragma unroll
            for (int u = 0; u < U; ++u) st16g<SP>(t4 + i + u * kThreads, cur[u]);
#pragma unroll
            for (int u = 0; u < U; ++u) cur[u] = nxt[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) st16g<SP>(t4 + i + u * kThreads, cur[u]);
        i += step;
    }
    for (; i < n4; i += kThreads) st16g<SP>(t4 + i, ld16<LP>(s4 + i));
}

template <int U, int LP = 0, int SP = 0>
__global__ __launch_bounds__(kThreads) void copy_kernel_g(const DCopy *__restrict__ pieces)
{
    const DCopy c = pieces[blockIdx.x];
    const int64_t n = c.len;
    if ((((uintptr_t)c.src | (uintptr_t)c.dst | (uint64_t)n) & 15) == 0) {
        pipelined_copy16<U, LP, SP>((g_cu4 *)c.src, (g_u4 *)c.dst, n >> 4);
    } else {
        for (int64_t i = threadIdx.x; i < n; i += kThreads) c.dst[i] = c.src[i];
    }
}

// Raw buffer access (gfx9 buffer resource, stride 0, num_records = bytes): a load
// past num_records returns 0 and a store past it is dropped, so the partial tail
// of a transfer needs no per-lane branch.  Branch-free code matters here: with a
// branch around every load and store the compiler's waitcnt pass can no longer
// count, and puts vmcnt(0) before EVERY store (each store then waits for the
// previous one to be acknowledged).
typedef __amdgpu_buffer_rsrc_t brsrc;
// s_waitcnt immediate (gfx9 encoding): vmcnt(0), expcnt(7) and lgkmcnt(15) = no wait on those
constexpr int kVmcnt0 = 0x0F70;
constexpr int kRsrcWord3 = 0x00020000;     // gfx9 (gfx950) raw buffer, as composable_kernel

__device__ __forceinline__ brsrc make_rsrc(const void *p, int64_t bytes)
{
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0, (int)bytes, kRsrcWord3);
}

__device__ __forceinline__ u32x4 bload16(brsrc r, int off)
{
    return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}

__device__ __forceinline__ void bstore16(brsrc r, int off, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
}

// One workgroup moves up to B*4 KiB (len, 16-B aligned) in one burst: every lane
// issues its B 16-B loads, then its B stores -- B*4 KiB in flight per workgroup, so
// a few hundred resident workgroups keep enough bytes in flight to stream HBM.
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

template <int B>
__device__ __forceinline__ void burst_copy16(const uint8_t *src, uint8_t *dst, int64_t len)
{
    u32x4 v[B];
    burst_load16<B>(src, len, v);
    burst_store16<B>(dst, len, v);
}

// Piece copy in bursts (copy variant 12): one workgroup per DCopy piece, B*4 KiB per
// burst, every load of a burst issued before its first store.
template <int B>
__global__ __launch_bounds__(kThreads) void copy_kernel_b(const DCopy *__restrict__ pieces)
{
    const DCopy c = pieces[blockIdx.x];
    if ((((uintptr_t)c.src | (uintptr_t)c.dst | (uint64_t)c.len) & 15) == 0) {
        constexpr int64_t step = (int64_t)B * kThreads * 16;
        for (int64_t o = 0; o < c.len; o += step)
            burst_copy16<B>(c.src + o, c.dst + o, c.len - o < step ? c.len - o : step);
    } else {
        for (int64_t i = threadIdx.x; i < c.len; i += kThreads) c.dst[i] = c.src[i];
    }
}

// ---------------------------------------------------------------- step engine
// A GPU-local plan of many small steps (sync / pairwise / throttled schedules
// at small -d) is bound by the per-step kernel boundary + timing event, not by
// HBM.  The engine runs the whole plan in ONE launch of W co-resident
// workgroups: step s = pieces [step_begin[s], step_begin[s+1]) strided over the
// workgroups, then a grid barrier whose last arriver stamps the step's
// completion time (wall clock).  No workgroup reads bytes another writes in
// this launch (every piece reads SEND and writes RECV), so the barrier orders
// and times steps but publishes no data, and the kernel end makes the stores
// visible.  A workgroup arrives as soon as its stores of step s are ISSUED
// (they may still land while step s+1 runs: -7..12 % per run of the
// sync/pairwise chains, profiles/r01_engine_drain_ab.txt), except at steps the
// host flags (engine_drains): there it waits for them first, so a step that
// rewrites or reads bytes of an earlier step sees them complete.  The last step
// always drains, so its stamp -- the anchor of every step time -- is a delivered time.
// State (cumulative ticket counter + timeout word) is zeroed by a memset before
// every launch; spins are bounded, and a timed-out workgroup sets *tmo and
// leaves, so a broken residency assumption ends the launch instead of hanging.
struct EngineState {
    unsigned count;     // arrival tickets, cumulative over every launch of the plan
    unsigned tmo;       // != 0: some workgroup gave up waiting
    unsigned pad[2];
};

typedef __attribute__((address_space(1))) unsigned g_u32;

// B: 16-B loads per lane per unit -> units of B * 4 KiB (the host cuts the step's
// transfers to that size and picks B so that a step has enough units to spread).
template <int B>
__global__ __launch_bounds__(kThreads) void step_engine_kernel(const DCopy *__restrict__ pieces,
                                                               const int *__restrict__ step_begin, int nsteps,
                                                               EngineState *st, unsigned long long *stamps,
                                                               unsigned base)
{
    // base: tickets taken by this plan's earlier launches (count is never reset
    // between launches, so no memset precedes a launch); compare by difference,
    // which is wrap-safe
    const unsigned W = gridDim.x;
    g_u32 *count = (g_u32 *)&st->count;
    g_u32 *tmo = (g_u32 *)&st->tmo;
    __shared__ int give_up;
    if (threadIdx.x == 0) give_up = 0;
    __syncthreads();
    // This workgroup's first unit of the next step is LOADED while the barrier is
    // pending (into v[]) and stored once it opens: the load latency of each step
    // (HBM + address translation of fresh pages) overlaps the barrier.  pf is
    // workgroup-uniform.
    const int *drain = step_begin + nsteps + 1;     // per-step flags (host: engine_drains)
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
            if ((((uintptr_t)c.src | (uintptr_t)c.dst | (uint64_t)c.len) & 15) == 0)
                burst_copy16<B>(c.src, c.dst, c.len);
            else
                for (int64_t k = threadIdx.x; k < c.len; k += kThreads) c.dst[k] = c.src[k];
        }
        if (drain[s]) __builtin_amdgcn_s_waitcnt(kVmcnt0);  // this wave's stores so far performed
        __syncthreads();
        const unsigned target = base + (unsigned)(s + 1) * W;
        bool last = false;
        if (threadIdx.x == 0) {
            const unsigned t = __hip_atomic_fetch_add(count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
            last = t == target;
            if (last) stamps[s] = (unsigned long long)wall_clock64();
        }
        if (s + 1 < nsteps) {              // no step reads what another writes: safe to load early
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
        __syncthreads();
        if (give_up) return;
    }
}

// ---------------------------------------------------------------- balanced byte-range copy
// The launch's copies form one virtual byte space [0, total) (prefix[k] =
// start of copy k, an exclusive scan of the lengths).  Workgroup b streams the
// contiguous virtual range [b*per, (b+1)*per) -- equal bytes per workgroup, so
// no tail wave; it crosses copy boundaries as it goes.  per is a multiple of
// 16 and every copy length/pointer is 16-B aligned in this fast path (the
// host falls back to copy_kernel otherwise).
struct DSpan {
    const uint8_t *src;
    uint8_t *dst;
    int64_t len;
    int64_t start;      // exclusive prefix of len
};

template <int U>
__global__ __launch_bounds__(kThreads) void span_copy_kernel(const DSpan *__restrict__ spans, int nspans,
                                                             int64_t total, int64_t per)
{
    int64_t pos = (int64_t)blockIdx.x * per;
    const int64_t end = pos + per < total ? pos + per : total;
    if (pos >= end) return;
    // first span containing pos (binary search, wave-uniform)
    int lo = 0, hi = nspans - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (spans[mid].start <= pos) lo = mid; else hi = mid - 1;
    }
    int k = lo;
    while (pos < end) {
        const DSpan sp = spans[k];
        const int64_t off = pos - sp.start;
        const int64_t stop = (sp.start + sp.len < end ? sp.start + sp.len : end) - sp.start;
        const uint4 *__restrict__ s4 = reinterpret_cast<const uint4 *>(sp.src + off);
        uint4 *__restrict__ t4 = reinterpret_cast<uint4 *>(sp.dst + off);
        const int64_t n4 = (stop - off) >> 4;
        int64_t i = threadIdx.x;
        for (; i + (int64_t)(U - 1) * kThreads < n4; i += (int64_t)U * kThreads) {
            uint4 v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) v[u] = s4[i + u * kThreads];
#pragma unroll
            for (int u = 0; u < U; ++u) t4[i + u * kThreads] = v[u];
        }
        for (; i < n4; i += kThreads) t4[i] = s4[i];
        pos = sp.start + stop;
        ++k;
    }
}

// exclusive prefix scan of span lengths, one workgroup (wave64 shuffles +
// LDS across the 4 waves), carried across 256-span tiles -- the device
// replacement of the displacement loops of *_alltoall_translate (:233-302)
__global__ __launch_bounds__(kThreads) void span_scan_kernel(DSpan *spans, int n, int64_t *total)
{
    __shared__ int64_t wsum[kThreads / 64];
    __shared__ int64_t carry;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int base = 0; base < n; base += kThreads) {
        const int i = base + threadIdx.x;
        const int64_t v = i < n ? spans[i].len : 0;
        int64_t x = v;                                 // inclusive scan inside the wave
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[wave] = x;
        __syncthreads();
        int64_t before = carry;
        for (int w = 0; w < wave; ++w) before += wsum[w];
        if (i < n) spans[i].start = before + x - v;
        __syncthreads();
        if (threadIdx.x == kThreads - 1) carry = before + x;
        __syncthreads();
    }
    if (threadIdx.x == 0) *total = carry;
}

// ---------------------------------------------------------------- microbenchmarks
__global__ __launch_bounds__(kThreads) void read_only_kernel(g_cu4 *__restrict__ s, int64_t n4, unsigned *sink)
{
    uint32_t x = 0;
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
        const u32x4 v = s[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9e3779b9u) atomicAdd(sink, 1u);
}

__global__ __launch_bounds__(kThreads) void write_only_kernel(g_u4 *__restrict__ t, int64_t n4)
{
    const u32x4 v = {1u, 2u, 3u, 4u};
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads)
        t[i] = v;
}

__global__ __launch_bounds__(kThreads) void gridstride_copy_kernel(const uint4 *__restrict__ s, uint4 *__restrict__ t,
                                                                   int64_t n4)
{
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads)
        t[i] = s[i];
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
__global__ __launch_bounds__(kThreads) void verify_kernel(const uint8_t *__restrict__ base,
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
