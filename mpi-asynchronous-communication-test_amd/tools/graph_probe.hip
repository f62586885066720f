// graph_probe.hip -- can a plan run be a hipGraph on this stack?  (tools/bin/graph_probe,
// not linked into the product).  Captures, on one stream, what xg_plan_run enqueues for a
// multi-GPU plan -- copy-kernel launches, a step event per step, a fork/join onto a second
// stream through events, and an RCCL group (self send/recv on a 1-rank communicator) --
// then replays it and reports: did capture / instantiate / launch succeed, do the captured
// events give elapsed times, and what one run costs as stream launches vs as a graph replay.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <time.h>

#include <vector>

#define CK(x)                                                                                           \
    do {                                                                                                \
        hipError_t e_ = (x);                                                                            \
        if (e_ != hipSuccess) {                                                                         \
            printf("FAIL %s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__);                     \
            return 1;                                                                                   \
        }                                                                                               \
    } while (0)
#define NK(x)                                                                                           \
    do {                                                                                                \
        ncclResult_t r_ = (x);                                                                          \
        if (r_ != ncclSuccess) {                                                                        \
            printf("FAIL %s: %s (line %d)\n", #x, ncclGetErrorString(r_), __LINE__);                    \
            return 1;                                                                                   \
        }                                                                                               \
    } while (0)

__global__ void small_copy(const uint4 *s, uint4 *d, int n)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = s[i];
}

static double now()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

struct Run {
    hipStream_t st, side;
    std::vector<hipEvent_t> ev;
    hipEvent_t ev0;
    std::vector<hipEvent_t> fork, join;
    uint4 *a, *b, *c;
    ncclComm_t comm;
    int nsteps, n;
    bool rccl;
};

// one "plan run": per step a copy launch, a side-stream copy (fork/join), an RCCL group, a step event
static int enqueue(Run &r)
{
    CK(hipEventRecord(r.ev0, r.st));
    for (int s = 0; s < r.nsteps; ++s) {
        hipLaunchKernelGGL(small_copy, dim3((r.n + 255) / 256), dim3(256), 0, r.st, r.a, r.b, r.n);
        CK(hipEventRecord(r.fork[s], r.st));
        CK(hipStreamWaitEvent(r.side, r.fork[s], 0));
        hipLaunchKernelGGL(small_copy, dim3((r.n + 255) / 256), dim3(256), 0, r.side, r.a, r.c, r.n);
        CK(hipEventRecord(r.join[s], r.side));
        if (r.rccl) {
            NK(ncclGroupStart());
            NK(ncclSend(r.b, (size_t)r.n * 16, ncclUint8, 0, r.comm, r.st));
            NK(ncclRecv(r.c, (size_t)r.n * 16, ncclUint8, 0, r.comm, r.st));
            NK(ncclGroupEnd());
        }
        CK(hipStreamWaitEvent(r.st, r.join[s], 0));
        CK(hipEventRecord(r.ev[s], r.st));
    }
    return 0;
}

int main(int argc, char **argv)
{
    Run r;
    r.nsteps = argc > 1 ? atoi(argv[1]) : 38;
    r.n = 2048 / 16 * 4;
    r.rccl = true;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&r.st, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&r.side, hipStreamNonBlocking));
    CK(hipMalloc(&r.a, r.n * 16));
    CK(hipMalloc(&r.b, r.n * 16));
    CK(hipMalloc(&r.c, r.n * 16));
    CK(hipMemset(r.a, 1, r.n * 16));
    r.ev.resize(r.nsteps);
    r.fork.resize(r.nsteps);
    r.join.resize(r.nsteps);
    CK(hipEventCreate(&r.ev0));
    for (int s = 0; s < r.nsteps; ++s) {
        CK(hipEventCreate(&r.ev[s]));
        CK(hipEventCreateWithFlags(&r.fork[s], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&r.join[s], hipEventDisableTiming));
    }
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    NK(ncclCommInitRank(&r.comm, 1, id, 0));
    // stream launches
    for (int w = 0; w < 3; ++w)
        if (enqueue(r)) return 1;
    CK(hipStreamSynchronize(r.st));
    const int reps = 20;
    double t0 = now();
    for (int k = 0; k < reps; ++k) {
        if (enqueue(r)) return 1;
        CK(hipStreamSynchronize(r.st));
    }
    const double t_stream = (now() - t0) / reps;
    float ms_last = 0;
    CK(hipEventElapsedTime(&ms_last, r.ev0, r.ev[r.nsteps - 1]));
    printf("stream: %d steps, %.1f us per run (host clock), device ev0 -> last step %.1f us\n", r.nsteps, t_stream * 1e6,
           ms_last * 1e3);
    // capture
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(r.st, hipStreamCaptureModeThreadLocal));
    if (enqueue(r)) return 1;
    CK(hipStreamEndCapture(r.st, &g));
    size_t nn = 0;
    CK(hipGraphGetNodes(g, nullptr, &nn));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    printf("capture ok: %zu graph nodes\n", nn);
    for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, r.st));
    CK(hipStreamSynchronize(r.st));
    t0 = now();
    for (int k = 0; k < reps; ++k) {
        CK(hipGraphLaunch(ge, r.st));
        CK(hipStreamSynchronize(r.st));
    }
    const double t_graph = (now() - t0) / reps;
    float ms_g = -1, ms_mid = -1;
    hipError_t e1 = hipEventElapsedTime(&ms_g, r.ev0, r.ev[r.nsteps - 1]);
    hipError_t e2 = hipEventElapsedTime(&ms_mid, r.ev0, r.ev[r.nsteps / 2]);
    printf("graph: %.1f us per run (host clock); captured events: elapsed ev0 -> last %s %.1f us, ev0 -> mid %s %.1f us\n",
           t_graph * 1e6, hipGetErrorString(e1), ms_g * 1e3, hipGetErrorString(e2), ms_mid * 1e3);
    // the data moved: c must equal a
    std::vector<uint4> ha(r.n), hc(r.n);
    CK(hipMemset(r.c, 0, r.n * 16));
    CK(hipGraphLaunch(ge, r.st));
    CK(hipStreamSynchronize(r.st));
    CK(hipMemcpy(ha.data(), r.a, r.n * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hc.data(), r.c, r.n * 16, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < r.n; ++i) bad += ha[i].x != hc[i].x || ha[i].w != hc[i].w;
    printf("graph replay delivered: %s\n", bad ? "WRONG" : "ok");
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    NK(ncclCommDestroy(r.comm));
    printf("done\n");
    return 0;
}
