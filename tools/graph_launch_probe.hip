// Probe: the host cost of hipGraphLaunch per node.
// Graphs of N tiny kernels (one 64-thread workgroup each), captured on one
// stream, or split over two streams with a fork at the start and a join at
// the end (the step's two encoder chains), with a small (8 B) or a large
// (512 B, like SlabJobs / AdamTable) kernel argument.  Reported: host
// microseconds per hipGraphLaunch, averaged over 20-launch bursts with a
// sync between bursts (the bench's K = 20 regime: the host never blocks on
// a full queue), and the slope per node.
// Build: hipcc --offload-arch=gfx950 -O2 tools/graph_launch_probe.hip -o tools/graph_launch_probe.bin
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("%s -> %s\n", #x, hipGetErrorString(e));                     \
            return -1.0;                                                        \
        }                                                                       \
    } while (0)

struct Big {
    unsigned long long w[64];
};

__global__ void tiny(unsigned *p) {
    if (threadIdx.x == 0) p[blockIdx.x] += 1u;
}

__global__ void tiny_big(unsigned *p, Big b) {
    if (threadIdx.x == 0) p[blockIdx.x] += static_cast<unsigned>(b.w[63]);
}

static double run(int n, bool two, bool big, unsigned *buf) {
    hipStream_t a, b;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    Big arg{};
    arg.w[63] = 1;
    hipGraph_t g;
    CK(hipStreamBeginCapture(a, hipStreamCaptureModeGlobal));
    if (two) {
        CK(hipEventRecord(fork, a));
        CK(hipStreamWaitEvent(b, fork, 0));
    }
    for (int i = 0; i < n; ++i) {
        hipStream_t s = (two && (i & 1)) ? b : a;
        if (big)
            tiny_big<<<1, 64, 0, s>>>(buf + i, arg);
        else
            tiny<<<1, 64, 0, s>>>(buf + i);
    }
    if (two) {
        CK(hipEventRecord(join, b));
        CK(hipStreamWaitEvent(a, join, 0));
    }
    CK(hipStreamEndCapture(a, &g));
    hipGraphExec_t ex;
    CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ex, a));
    CK(hipStreamSynchronize(a));
    double tot = 0.0;
    int cnt = 0;
    for (int rep = 0; rep < 10; ++rep) {
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < 20; ++i) CK(hipGraphLaunch(ex, a));
        const auto t1 = std::chrono::steady_clock::now();
        CK(hipStreamSynchronize(a));
        if (rep >= 2) {
            tot += std::chrono::duration<double, std::micro>(t1 - t0).count();
            cnt += 20;
        }
    }
    CK(hipGraphExecDestroy(ex));
    CK(hipGraphDestroy(g));
    CK(hipEventDestroy(fork));
    CK(hipEventDestroy(join));
    CK(hipStreamDestroy(a));
    CK(hipStreamDestroy(b));
    return tot / cnt;
}

int main() {
    unsigned *buf;
    if (hipMalloc(&buf, 4096 * sizeof(unsigned)) != hipSuccess) return 1;
    const int ns[] = {8, 24, 48, 96};
    for (int two = 0; two < 2; ++two)
        for (int big = 0; big < 2; ++big) {
            double us[4];
            for (int i = 0; i < 4; ++i) {
                us[i] = run(ns[i], two, big, buf);
                if (us[i] < 0) return 1;
            }
            printf("%-9s arg %-4s  us/launch: N=8 %6.2f  N=24 %6.2f  N=48 %6.2f  N=96 %6.2f   "
                   "slope %.3f us/node\n",
                   two ? "2 streams" : "1 stream", big ? "512B" : "8B", us[0], us[1], us[2], us[3],
                   (us[3] - us[0]) / (96 - 8));
        }
    (void)hipFree(buf);
    return 0;
}
