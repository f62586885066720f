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
// *gbps = counted bytes / average launch time (a copy counts read + write).
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

#include "../csrc/kernels.h"

namespace {

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
    if (bytes <= 0 || reps < 1 || kind < 0 || kind > 9) return 3;
    CK(hipSetDevice(device));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    uint8_t *a, *b;
    unsigned *sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 4));
    CK(hipMemsetAsync(a, 1, bytes, st));
    const int64_t piece = kind == 7 ? 262144 : (kind == 8 ? 65536 : 32768);
    std::vector<xgk::DCopy> pieces;
    for (int64_t o = 0; o < bytes; o += piece) pieces.push_back({a + o, b + o, std::min<int64_t>(piece, bytes - o)});
    xgk::DCopy *dp;
    CK(hipMalloc(&dp, sizeof(xgk::DCopy) * pieces.size()));
    CK(hipMemcpy(dp, pieces.data(), sizeof(xgk::DCopy) * pieces.size(), hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int64_t n4 = bytes / 16;
    const unsigned np = (unsigned)pieces.size();
    for (int r = -2; r < reps; ++r) {          // 2 warm-up launches
        if (r == 0) CK(hipEventRecord(e0, st));
        switch (kind) {
        case 0: hipLaunchKernelGGL(gridstride_copy, dim3(2048), dim3(xgk::kThreads), 0, st, (const xgk::u32x4 *)a,
                                   (xgk::u32x4 *)b, n4); break;
        case 1: hipLaunchKernelGGL((xgk::copy_kernel_g<4>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        case 2: hipLaunchKernelGGL((xgk::copy_kernel_b<4, xgk::kAuxSC1>), dim3(np), dim3(xgk::kThreads), 0, st, dp);
                break;
        case 3: hipLaunchKernelGGL(read_only, dim3(4096), dim3(xgk::kThreads), 0, st, (const xgk::u32x4 *)a, n4, sink);
                break;
        case 4: hipLaunchKernelGGL(write_only, dim3(4096), dim3(xgk::kThreads), 0, st, (xgk::u32x4 *)b, n4); break;
        case 5: CK(hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, st)); break;
        case 6: hipLaunchKernelGGL(gridstride_copy_nt, dim3(2048), dim3(xgk::kThreads), 0, st, (const xgk::u32x4 *)a,
                                   (xgk::u32x4 *)b, n4); break;
        case 9: hipLaunchKernelGGL((xgk::copy_kernel_g<4, true>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        default: hipLaunchKernelGGL((xgk::copy_kernel_g<4>), dim3(np), dim3(xgk::kThreads), 0, st, dp, nullptr); break;
        }
        CK(hipGetLastError());
    }
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    *gbps = (kind == 3 || kind == 4 ? 1.0 : 2.0) * (double)bytes * reps / (ms * 1e-3) / 1e9;
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(dp));
    CK(hipFree(sink));
    CK(hipStreamDestroy(st));
    return 0;
}
