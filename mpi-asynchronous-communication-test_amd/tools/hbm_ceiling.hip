// hbm_ceiling.hip -- HBM ceiling microbenchmarks (tools/libxgtools.so), kept out of
// the product library: what a copy, a read and a write stream reach on this
// device, next to the exchange's own copy kernels over the same bytes.
//
//   kind 0  grid-stride 16-B copy (the canonical copy), 2048 workgroups
//   kind 1  copy_kernel_g<4> over 32 KiB pieces        (exchange default)
//   kind 2  copy_kernel_b<4, sc1 stores> over 32 KiB pieces
//   kind 3  read-only stream, 4096 workgroups (1 byte counted per byte)
//   kind 4  write-only stream, 4096 workgroups (1 byte counted per byte)
//   kind 5  hipMemcpyAsync device-to-device (the runtime's own copy)
//   kind 6  grid-stride 16-B copy with non-temporal loads and stores, 2048 workgroups
//   kind 7  one 256 KiB span per workgroup, 4 x 16-B loads in flight per lane
//   kind 8  copy_kernel_g<4> over 64 KiB pieces
//   kind 9  copy_kernel_g<4, nt> over 32 KiB pieces (non-temporal loads and stores)
//   kind 10 read-only stream, non-temporal loads      kind 11 write-only stream, non-temporal stores
//   kind 12 grid-stride copy, nt loads + plain stores   kind 13 grid-stride copy, plain loads + nt stores
//   kind 14 copy_kernel_g<8, nt> over 32 KiB pieces   kind 15 copy_kernel_g<2, nt> over 32 KiB pieces
//   kind 16 many-to-all gather, copy_kernel_g<4, nt>: 14 source blocks of 32 x 1 MiB segments at a
//           32 MiB stride, destination segment (r, a) at (r * 14 + a) MiB, pieces in destination order
//   kind 17 the same with the source blocks 32 MiB + 64 KiB apart (stride off a power of two)
//   kind 18 one GPU's pack launch of configs[2] m8 on 8 GPUs (28 MiB gathered out of 32 MiB of
//           256 KiB segments, one-sided order), copy_kernel_g<4> over 16 KiB pieces (the product)
//   kind 19 the same pieces, copy_kernel_p<4> (512 persistent 1024-lane workgroups)
//   kind 20 copy_kernel_p<2>, 512 workgroups    kind 21 copy_kernel_p<8>, 256 workgroups
//   kind 22 the kind-18 gather in 8 KiB pieces, copy_kernel_w<8> (wave-persistent, resident grid)
//   kind 23 the kind-16 gather (448 MiB) in 8 KiB pieces, copy_kernel_w<8, nt>
//   kind 24 the same in 4 KiB pieces, copy_kernel_w<4, nt>   kind 25 16 KiB pieces, copy_kernel_w<16, nt>
//   kind 26 the kind-18 pack in the two-sided order (per peer, per sender), copy_kernel_g<4> 16 KiB
//   kind 27 the same, copy_kernel_w<8> over 8 KiB pieces (the product since call K)
//   round 4, the kind-16 gather (448 MiB) against the piece size, the pipeline depth and the cache
//   policy of the loads and stores (buffer accesses, gfx950 cpol bits: sc0 1, nt 2, sc1 16):
//   kind 28 copy_kernel_g<4, nt> 64 KiB pieces      kind 29 copy_kernel_g<8, nt> 32 KiB
//   kind 30 copy_kernel_g<4, nt> 128 KiB            kind 31 copy_kernel_g<4, nt> 16 KiB
//   kind 32 copy_kernel_bb<4, load nt, store nt>    kind 33 <4, nt, nt|sc1>
//   kind 34 <4, nt|sc0|sc1, nt|sc0|sc1>             kind 35 <4, nt, sc0|sc1>
//   kind 36 <4, plain, nt>                          kind 37 <4, nt, plain>
//   kind 38 the contiguous copy (kind 9's pieces) as copy_kernel_bb<4, nt, nt|sc1>
//   kind 39 the kind-16 gather, copy_kernel_bb<4, nt|sc1, nt|sc1>
// *gbps = counted bytes / average launch time (a copy counts read + write).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "../csrc/kernels.h"

namespace {

// copy_kernel_b<U, AUX>: the exchange's piece copy through buffer resources with store policy
// AUX (an A/B variant measured in round 1/2, kept here for the ceiling tables only)
// Pipelined piece copy through buffer resources (n: bytes, a multiple of 16,
// < 2^31): every lane keeps U 16-B loads of the next block in flight while it
// stores the current block.  The trip count is wave-uniform; out-of-range
// lanes of the last block load 0 and their stores are dropped by the range check.
template <int U, int AUX>
__device__ __forceinline__ void pipelined_copy16_b(const uint8_t *src, uint8_t *dst, int n)
{
    const xgk::brsrc rs = xgk::make_rsrc(src, n), rd = xgk::make_rsrc(dst, n);
    constexpr int blk = U * xgk::kThreads * 16;
    const int lane = (int)threadIdx.x * 16;
    xgk::u32x4 cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = xgk::bload16(rs, lane + u * xgk::kThreads * 16);
    for (int base = 0; base < n; base += blk) {
        xgk::u32x4 nxt[U];
#pragma unroll
        for (int u = 0; u < U; ++u) nxt[u] = xgk::bload16(rs, base + blk + lane + u * xgk::kThreads * 16);
#pragma unroll
        for (int u = 0; u < U; ++u) xgk::bstore16<AUX>(rd, base + lane + u * xgk::kThreads * 16, cur[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
}

// copy_kernel_bb<U, LAUX, SAUX>: the same pipelined piece copy with the cache policy of the
// loads (LAUX) and of the stores (SAUX) chosen (round-4 A/B on the bench's gather, kinds 32-37)
template <int U, int LAUX, int SAUX>
__global__ __launch_bounds__(xgk::kThreads) void copy_kernel_bb(const xgk::DCopy *__restrict__ pieces)
{
    const xgk::DCopy c = pieces[blockIdx.x];
    const int n = (int)c.len;
    const xgk::brsrc rs = xgk::make_rsrc(c.src, n), rd = xgk::make_rsrc(c.dst, n);
    constexpr int blk = U * xgk::kThreads * 16;
    const int lane = (int)threadIdx.x * 16;
    xgk::u32x4 cur[U];
#pragma unroll
    for (int u = 0; u < U; ++u) cur[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, lane + u * xgk::kThreads * 16, 0, LAUX);
    for (int base = 0; base < n; base += blk) {
        xgk::u32x4 nxt[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            nxt[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, base + blk + lane + u * xgk::kThreads * 16, 0, LAUX);
#pragma unroll
        for (int u = 0; u < U; ++u) xgk::bstore16<SAUX>(rd, base + lane + u * xgk::kThreads * 16, cur[u]);
#pragma unroll
        for (int u = 0; u < U; ++u) cur[u] = nxt[u];
    }
}

template <int U, int AUX>
__global__ __launch_bounds__(xgk::kThreads) void copy_kernel_b(const xgk::DCopy *__restrict__ pieces)
{
    __shared__ uint32_t lds[2][xgk::kTileWords];
    const xgk::DCopy c = pieces[blockIdx.x];
    if ((((uintptr_t)c.src | (uintptr_t)c.dst | (uint64_t)c.len) & 15) == 0)
        pipelined_copy16_b<U, AUX>(c.src, c.dst, (int)c.len);
    else
        xgk::realign_copy(c.src, c.dst, c.len, lds);
}


// copy_kernel_p<U>: a probe of a persistent piece copy (kinds 19-20) -- W workgroups of 1024
// lanes, workgroup w copies pieces w, w + W, w + 2W, ... of exactly 16 KiB (one 16-B access
// per lane): U pieces' loads in flight per lane, the store of piece k interleaved with the
// loads of piece k + U*W (no launch-wide load burst followed by a store burst).
template <int U>
__global__ __launch_bounds__(1024) void copy_kernel_p(const xgk::DCopy *__restrict__ pieces, int np)
{
    const int W = (int)gridDim.x, lane = (int)threadIdx.x * 16;
    xgk::u32x4 v[U];
    uint8_t *dst[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int i = (int)blockIdx.x + u * W;
        dst[u] = nullptr;
        if (i < np) {
            const xgk::DCopy c = pieces[i];
            v[u] = *(const xgk::g_cu4 *)(c.src + lane);
            dst[u] = c.dst;
        }
    }
    for (int base = (int)blockIdx.x; base < np; base += U * W) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = base + u * W;
            if (i >= np) break;
            *(xgk::g_u4 *)(dst[u] + lane) = v[u];
            const int j = i + U * W;
            if (j < np) {
                const xgk::DCopy c = pieces[j];
                v[u] = *(const xgk::g_cu4 *)(c.src + lane);
                dst[u] = c.dst;
            }
        }
    }
}

__global__ __launch_bounds__(xgk::kThreads) void gridstride_copy(const xgk::u32x4 *__restrict__ s,
                                                                 xgk::u32x4 *__restrict__ t, int64_t n4)
{
    for (int64_t i = (int64_t)blockIdx.x * xgk::kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * xgk::kThreads)
        t[i] = s[i];
}

__global__ __launch_bounds__(xgk::kThreads) void read_only(const xgk::u32x4 *__restrict__ s, int64_t n4, unsigned *sink)
{
    unsigned x = 0;
    for (int64_t i = (int64_t)blockIdx.x * xgk::kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * xgk::kThreads) {
        const xgk::u32x4 v = s[i];
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9e3779b9u) atomicAdd(sink, 1u);     // keeps the loads alive
}

__global__ __launch_bounds__(xgk::kThreads) void write_only(xgk::u32x4 *__restrict__ t, int64_t n4)
{
    const xgk::u32x4 v = {1u, 2u, 3u, 4u};
    for (int64_t i = (int64_t)blockIdx.x * xgk::kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * xgk::kThreads)
        t[i] = v;
}

__global__ __launch_bounds__(xgk::kThreads) void gridstride_copy_nt(const xgk::u32x4 *__restrict__ s,
                                                                    xgk::u32x4 *__restrict__ t, int64_t n4)
{
    for (int64_t i = (int64_t)blockIdx.x * xgk::kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * xgk::kThreads)
        __builtin_nontemporal_store(__builtin_nontemporal_load(s + i), t + i);
}

__global__ __launch_bounds__(xgk::kThreads) void read_only_nt(const xgk::u32x4 *__restrict__ s, int64_t n4, unsigned *sink)
{
    unsigned x = 0;
    for (int64_t i = (int64_t)blockIdx.x * xgk::kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * xgk::kThreads) {
        const xgk::u32x4 v = __builtin_nontemporal_load(s + i);
        x ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (x == 0x9e3779b9u) atomicAdd(sink, 1u);
}

__global__ __launch_bounds__(xgk::kThreads) void write_only_nt(xgk::u32x4 *__restrict__ t, int64_t n4)
{
    const xgk::u32x4 v = {1u, 2u, 3u, 4u};
    for (int64_t i = (int64_t)blockIdx.x * xgk::kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * xgk::kThreads)
        __builtin_nontemporal_store(v, t + i);
}

template <bool NTL, bool NTS>
__global__ __launch_bounds__(xgk::kThreads) void gridstride_copy_mix(const xgk::u32x4 *__restrict__ s,
                                                                     xgk::u32x4 *__restrict__ t, int64_t n4)
{
    for (int64_t i = (int64_t)blockIdx.x * xgk::kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * xgk::kThreads) {
        const xgk::u32x4 v = NTL ? __builtin_nontemporal_load(s + i) : s[i];
        if (NTS) __builtin_nontemporal_store(v, t + i);
        else t[i] = v;
    }
}

}  // namespace

#define CK(x)                                                                                             \
    do {                                                                                                  \
        hipError_t e_ = (x);                                                                              \
        if (e_ != hipSuccess) {                                                                           \
            fprintf(stderr, "xgt: %s at %s:%d: %s\n", hipGetErrorString(e_), __FILE__, __LINE__, #x);     \
            return 1;                                                                                     \
        }                                                                                                 \
    } while (0)

extern "C" int xgt_copy_ceiling(int device, int64_t bytes, int kind, int reps, double *gbps)
{
    bytes &= ~(int64_t)32767;
    if (bytes <= 0 || reps < 1 || kind < 0 || kind > 39) return 3;
    CK(hipSetDevice(device));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint8_t *a, *b;
    unsigned *sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemsetAsync(a, 1, bytes, st));
    const int64_t piece = kind == 28 ? 65536 : kind == 30 ? 131072 : kind == 31 ? 16384 : kind >= 29 ? 32768
                        : kind == 7 ? 262144 : kind == 8 ? 65536 : kind == 22 || kind == 23 || kind == 27 ? 8192 : kind == 24 ? 4096
                        : kind == 25 ? 16384 : kind >= 18 ? 16384 : 32768;
    std::vector<xgk::DCopy> pieces;
    if (kind == 16 || kind == 17 || kind == 23 || kind == 24 || kind == 25 || (kind >= 28 && kind != 38)) {   // bytes ignored: 14 x 32 one-MiB segments
        const int64_t seg = 1 << 20, stride = 32 * seg + (kind == 17 ? 65536 : 0);
        if (14 * stride > bytes) return 3;
        for (int r = 0; r < 32; ++r)
            for (int g = 0; g < 14; ++g)
                for (int64_t o = 0; o < seg; o += piece)
                    pieces.push_back({a + g * stride + r * seg + o, b + (int64_t)(r * 14 + g) * seg + o, piece});
    } else if (kind == 26 || kind == 27) {     // the same pack in the two-sided order (per peer, per sender)
        const int64_t seg = 256 << 10;
        if (32 * seg * 4 > bytes) return 3;
        int64_t t = 0;
        for (int p = 1; p < 8; ++p)
            for (int s = 0; s < 8; ++s)
                for (int ag = 2 * p; ag < 2 * p + 2; ++ag, t += seg)
                    for (int64_t o = 0; o < seg; o += piece) pieces.push_back({a + (s * 16 + ag) * seg + o, b + t + o, piece});
    } else if (kind >= 18 && kind <= 22) {     // bytes ignored: one GPU's pack launch of configs[2] m8
        // on 8 GPUs: 8 ranks x 16 segments of 256 KiB (rank-major, 32 MiB), the 112 bound for the
        // 7 peers gathered in the one-sided order (per peer, per aggregator, the 8 senders)
        const int64_t seg = 256 << 10;
        if (32 * seg * 4 > bytes) return 3;
        int64_t t = 0;
        for (int p = 1; p < 8; ++p)
            for (int ag = 2 * p; ag < 2 * p + 2; ++ag)
                for (int s = 0; s < 8; ++s, t += seg)
                    for (int64_t o = 0; o < seg; o += piece) pieces.push_back({a + (s * 16 + ag) * seg + o, b + t + o, piece});
    } else {
        for (int64_t o = 0; o < bytes; o += piece) pieces.push_back({a + o, b + o, std::min<int64_t>(piece, bytes - o)});
    }
    xgk::DCopy *dp;
    CK(hipMalloc(&dp, sizeof(xgk::DCopy) * pieces.size()));
    CK(hipMemcpy(dp, pieces.data(), sizeof(xgk::DCopy) * pieces.size(), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int64_t n4 = bytes / 16;
    const unsigned np = (unsigned)pieces.size();
    // wave-persistent kinds: as many workgroups as are resident at once (occupancy x CUs)
    int occ = 1, cus = 1;
    if (kind == 22 || kind == 27) CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, xgk::copy_kernel_w<8, false>, xgk::kThreads, 0));
    if (kind == 23) CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, xgk::copy_kernel_w<8, true>, xgk::kThreads, 0));
    if (kind == 24) CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, xgk::copy_kernel_w<4, true>, xgk::kThreads, 0));
    if (kind == 25) CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, xgk::copy_kernel_w<16, true>, xgk::kThreads, 0));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    const unsigned wgrid = (unsigned)std::max(1, std::min<int>(occ * cus, ((int)np + 3) / 4));
    if (kind >= 22 && kind != 26) fprintf(stderr, "xgt kind %d: %u pieces, %d resident workgroups per CU -> grid %u\n", kind, np, occ, wgrid);
    for (int r = -2; r < reps; ++r) {          // 2 warm-up launches
        if (r == 0) CK(hipEventRecord(e0, st));
        switch (kind) {
        case 0: hipLaunchKernelGGL(gridstride_copy, dim3(2048), dim3(xgk::kThreads), 0, st, (const xgk::u32x4 *)a,
                                   (xgk::u32x4 *)b, n4); break;
        case 1: hipLaunchKernelGGL((xgk::copy_kernel_g<4>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        case 2: hipLaunchKernelGGL((copy_kernel_b<4, xgk::kAuxSC1>), dim3(np), dim3(xgk::kThreads), 0, st, dp);
                break;
        case 3: hipLaunchKernelGGL(read_only, dim3(4096), dim3(xgk::kThreads), 0, st, (const xgk::u32x4 *)a, n4, sink);
                break;
        case 4: hipLaunchKernelGGL(write_only, dim3(4096), dim3(xgk::kThreads), 0, st, (xgk::u32x4 *)b, n4); break;
        case 5: CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, st)); break;
        case 6: hipLaunchKernelGGL(gridstride_copy_nt, dim3(2048), dim3(xgk::kThreads), 0, st, (const xgk::u32x4 *)a,
                                   (xgk::u32x4 *)b, n4); break;
        case 9: hipLaunchKernelGGL((xgk::copy_kernel_g<4, true>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        case 10: hipLaunchKernelGGL(read_only_nt, dim3(4096), dim3(xgk::kThreads), 0, st, (const xgk::u32x4 *)a, n4, sink);
                 break;
        case 11: hipLaunchKernelGGL(write_only_nt, dim3(4096), dim3(xgk::kThreads), 0, st, (xgk::u32x4 *)b, n4); break;
        case 12: hipLaunchKernelGGL((gridstride_copy_mix<true, false>), dim3(2048), dim3(xgk::kThreads), 0, st,
                                    (const xgk::u32x4 *)a, (xgk::u32x4 *)b, n4); break;
        case 13: hipLaunchKernelGGL((gridstride_copy_mix<false, true>), dim3(2048), dim3(xgk::kThreads), 0, st,
                                    (const xgk::u32x4 *)a, (xgk::u32x4 *)b, n4); break;
        case 14: hipLaunchKernelGGL((xgk::copy_kernel_g<8, true>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        case 15: hipLaunchKernelGGL((xgk::copy_kernel_g<2, true>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        case 16:
        case 17: hipLaunchKernelGGL((xgk::copy_kernel_g<4, true>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        case 19: hipLaunchKernelGGL((copy_kernel_p<4>), dim3(512), dim3(1024), 0, st, dp, (int)np); break;
        case 20: hipLaunchKernelGGL((copy_kernel_p<2>), dim3(512), dim3(1024), 0, st, dp, (int)np); break;
        case 21: hipLaunchKernelGGL((copy_kernel_p<8>), dim3(256), dim3(1024), 0, st, dp, (int)np); break;
        case 22: hipLaunchKernelGGL((xgk::copy_kernel_w<8, false>), dim3(wgrid), dim3(xgk::kThreads), 0, st, dp,
                                    (int)np, nullptr); break;
        case 23: hipLaunchKernelGGL((xgk::copy_kernel_w<8, true>), dim3(wgrid), dim3(xgk::kThreads), 0, st, dp,
                                    (int)np, nullptr); break;
        case 24: hipLaunchKernelGGL((xgk::copy_kernel_w<4, true>), dim3(wgrid), dim3(xgk::kThreads), 0, st, dp,
                                    (int)np, nullptr); break;
        case 25: hipLaunchKernelGGL((xgk::copy_kernel_w<16, true>), dim3(wgrid), dim3(xgk::kThreads), 0, st, dp,
                                    (int)np, nullptr); break;
        case 27: hipLaunchKernelGGL((xgk::copy_kernel_w<8, false>), dim3(wgrid), dim3(xgk::kThreads), 0, st, dp,
                                    (int)np, nullptr); break;
        case 28:
        case 30:
        case 31: hipLaunchKernelGGL((xgk::copy_kernel_g<4, true>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        case 29: hipLaunchKernelGGL((xgk::copy_kernel_g<8, true>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        case 32: hipLaunchKernelGGL((copy_kernel_bb<4, 2, 2>), dim3(np), dim3(xgk::kThreads), 0, st, dp); break;
        case 33: hipLaunchKernelGGL((copy_kernel_bb<4, 2, 18>), dim3(np), dim3(xgk::kThreads), 0, st, dp); break;
        case 34: hipLaunchKernelGGL((copy_kernel_bb<4, 19, 19>), dim3(np), dim3(xgk::kThreads), 0, st, dp); break;
        case 35: hipLaunchKernelGGL((copy_kernel_bb<4, 2, 17>), dim3(np), dim3(xgk::kThreads), 0, st, dp); break;
        case 36: hipLaunchKernelGGL((copy_kernel_bb<4, 0, 2>), dim3(np), dim3(xgk::kThreads), 0, st, dp); break;
        case 37: hipLaunchKernelGGL((copy_kernel_bb<4, 2, 0>), dim3(np), dim3(xgk::kThreads), 0, st, dp); break;
        case 38: hipLaunchKernelGGL((copy_kernel_bb<4, 2, 18>), dim3(np), dim3(xgk::kThreads), 0, st, dp); break;
        case 39: hipLaunchKernelGGL((copy_kernel_bb<4, 18, 18>), dim3(np), dim3(xgk::kThreads), 0, st, dp); break;
        default: hipLaunchKernelGGL((xgk::copy_kernel_g<4>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        }
        CK(hipGetLastError());
    }
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double moved = kind == 16 || kind == 17 || (kind >= 23 && kind <= 25) || (kind >= 28 && kind != 38) ? 448.0 * (1 << 20) : kind >= 18 ? 28.0 * (1 << 20)
                                                                                               : (double)bytes;
    *gbps = (kind == 3 || kind == 4 || kind == 10 || kind == 11 ? 1.0 : 2.0) * moved * reps / (ms * 1e-3) / 1e9;
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(dp));
    CK(hipFree(sink));
    CK(hipStreamDestroy(st));
    return 0;
}

// ---------------------------------------------------------------- doorbell round trip
// How fast can the host start a waiting kernel and see its answer?  One lane polls a
// ring word; when it reads r it writes r to a done word in host-pinned memory
// (system scope); the host times ring store -> done seen, reps times.
//   kind 0  ring in host-pinned coherent memory (the armed engine's doorbell)
//   kind 1  ring in fine-grained device memory, stored by the host through its mapping
//   kind 2  ring in uncached device memory, stored by the host through its mapping
// Returns 4 if the device ring is not host-accessible (*us untouched).
namespace {
__global__ void doorbell_pingpong(unsigned *ring, unsigned *done, int reps, int dev_ring)
{
    if (threadIdx.x != 0) return;
    typedef __attribute__((address_space(1))) unsigned gu;
    for (int r = 1; r <= reps; ++r) {
        for (unsigned spins = 0;; ++spins) {
            const unsigned x = dev_ring ? __hip_atomic_load((gu *)ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                        : __hip_atomic_load((gu *)ring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            if (x == (unsigned)r) break;
            if (spins > (1u << 26)) return;
            __builtin_amdgcn_s_sleep(1);
        }
        __hip_atomic_store((gu *)done, (unsigned)r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
}  // namespace

#include <time.h>
static double now_s()
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

extern "C" int xgt_doorbell_rtt(int device, int kind, int reps, double *us)
{
    if (kind < 0 || kind > 2 || reps < 1) return 3;
    CK(hipSetDevice(device));
    unsigned *done = nullptr, *ring = nullptr, *hring = nullptr;
    CK(hipHostMalloc((void **)&done, 64, hipHostMallocCoherent));
    *(volatile unsigned *)done = 0;
    if (kind == 0) {
        CK(hipHostMalloc((void **)&ring, 64, hipHostMallocCoherent));
        hring = ring;
    } else {
        CK(hipExtMallocWithFlags((void **)&ring, 64, kind == 1 ? hipDeviceMallocFinegrained : hipDeviceMallocUncached));
        CK(hipMemset(ring, 0, 64));
        hipPointerAttribute_t at;
        CK(hipPointerGetAttributes(&at, ring));
        hring = (unsigned *)at.hostPointer;
        if (!hring) {
            CK(hipFree(ring));
            CK(hipHostFree(done));
            return 4;
        }
    }
    *(volatile unsigned *)hring = 0;
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipLaunchKernelGGL(doorbell_pingpong, dim3(1), dim3(64), 0, st, ring, done, reps + 8, kind != 0);
    CK(hipGetLastError());
    double tot = 0;
    int got = 0;
    for (int r = 1; r <= reps + 8; ++r) {
        const double t0 = now_s();
        __atomic_store_n(hring, (unsigned)r, __ATOMIC_SEQ_CST);
        __builtin_ia32_sfence();
        bool ok = true;
        while (__atomic_load_n(done, __ATOMIC_ACQUIRE) != (unsigned)r)
            if (now_s() - t0 > 2.0) { ok = false; break; }
        const double t1 = now_s();
        if (!ok) break;
        if (r > 8) { tot += t1 - t0; ++got; }      // 8 warm-up round trips
    }
    CK(hipStreamSynchronize(st));
    CK(hipStreamDestroy(st));
    if (kind == 0) CK(hipHostFree(ring)); else CK(hipFree(ring));
    CK(hipHostFree(done));
    if (got != reps) return 5;
    *us = tot / got * 1e6;
    return 0;
}
