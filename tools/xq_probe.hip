// Cross-queue synchronisation cost inside a replayed HIP graph: the step's
// two-chain shape (fork, a mid join, a second fork, the final join) with the
// mid join / second fork as graph edges (event) or as a one-wave flag kernel
// pair (flag: the producer queue's signal kernel bumps a counter after its
// chain, a one-wave wait kernel on the consumer queue polls it; no graph edge).
//
//   hipcc --offload-arch=gfx950 -O2 tools/xq_probe.hip -o build/xq_probe
//   build/xq_probe            (prints us per replay for both forms)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::printf("%s -> %s\n", #x, hipGetErrorString(e_));                        \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

__global__ void busy_k(float *x, int iters) {
    float v = x[threadIdx.x & 63] + blockIdx.x;
    for (int i = 0; i < iters; ++i) v = v * 1.0000001f + 1e-7f;
    if (v == 12345.f) x[0] = v;  // never: keeps the loop
}

__global__ void signal_k(unsigned *flag) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(flag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// waits until *flag > *ack (one signal not yet consumed), then consumes it
__global__ void wait_k(unsigned *flag, unsigned *ack, unsigned *err) {
    if (threadIdx.x == 0) {
        const unsigned a = __hip_atomic_load(ack, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = wall_clock64();
        while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <= a) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - t0 > 20000000) {  // 0.2 s
                __hip_atomic_fetch_add(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __hip_atomic_store(ack, a + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

struct Bufs {
    float *x;
    unsigned *w;  // flag0, ack0, flag1, ack1, err
};

static void busy(hipStream_t s, const Bufs &b, int grid, int iters) {
    busy_k<<<grid, 256, 0, s>>>(b.x, iters);
}

static int capture(bool flag, hipStream_t a, hipStream_t bq, const Bufs &b, hipGraphExec_t *ex) {
    hipEvent_t e0, e1, e2, e3;
    CK(hipEventCreateWithFlags(&e0, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e3, hipEventDisableTiming));
    hipGraph_t g;
    CK(hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal));
    CK(hipEventRecord(e0, a));
    CK(hipStreamWaitEvent(bq, e0, 0));  // fork at the start
    busy(a, b, 145, 4000);              // "ego build"
    for (int l = 0; l < 5; ++l) {
        busy(a, b, 452, 3000);  // ego chain
        busy(bq, b, 150, 2500);  // core chain
    }
    if (flag) {
        signal_k<<<1, 64, 0, bq>>>(b.w + 0);
        wait_k<<<1, 64, 0, a>>>(b.w + 0, b.w + 1, b.w + 4);
    } else {
        CK(hipEventRecord(e1, bq));
        CK(hipStreamWaitEvent(a, e1, 0));  // forward join
    }
    for (int l = 0; l < 3; ++l) busy(a, b, 241, 2500);  // loss section
    if (flag) {
        signal_k<<<1, 64, 0, a>>>(b.w + 2);
        wait_k<<<1, 64, 0, bq>>>(b.w + 2, b.w + 3, b.w + 4);
    } else {
        CK(hipEventRecord(e2, a));
        CK(hipStreamWaitEvent(bq, e2, 0));  // backward fork
    }
    for (int l = 0; l < 5; ++l) {
        busy(a, b, 452, 4000);
        busy(bq, b, 150, 3000);
    }
    CK(hipEventRecord(e3, bq));
    CK(hipStreamWaitEvent(a, e3, 0));  // final join
    busy(a, b, 142, 1000);              // "Adam"
    CK(hipStreamEndCapture(a, &g));
    CK(hipGraphInstantiate(ex, g, nullptr, nullptr, 0));
    return 0;
}

int main() {
    Bufs b;
    CK(hipMalloc(&b.x, 4096));
    CK(hipMemset(b.x, 0, 4096));
    CK(hipMalloc(&b.w, 64));
    CK(hipMemset(b.w, 0, 64));
    hipStream_t a, bq;
    CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&bq, hipStreamNonBlocking));
    for (int rep = 0; rep < 2; ++rep) {
        for (int flag = 0; flag < 2; ++flag) {
            hipGraphExec_t ex;
            if (capture(flag != 0, a, bq, b, &ex)) return 1;
            for (int i = 0; i < 3; ++i) CK(hipGraphLaunch(ex, a));
            CK(hipStreamSynchronize(a));
            unsigned err = 0;
            CK(hipMemcpy(&err, b.w + 4, 4, hipMemcpyDeviceToHost));
            if (err) {
                std::printf("flag=%d: %u wait timeouts in 3 replays (the two kernels share a queue?)\n",
                            flag, err);
                return 2;
            }
            const int n = 400;
            auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < n; ++i) CK(hipGraphLaunch(ex, a));
            CK(hipStreamSynchronize(a));
            auto t1 = std::chrono::steady_clock::now();
            CK(hipMemcpy(&err, b.w + 4, 4, hipMemcpyDeviceToHost));
            std::printf("%s: %.2f us per replay (timeouts %u)\n", flag ? "flag " : "event",
                        std::chrono::duration<double, std::micro>(t1 - t0).count() / n, err);
            std::fflush(stdout);
            CK(hipGraphExecDestroy(ex));
        }
    }
    return 0;
}
