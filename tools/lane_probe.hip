// Probe for the two-lane replay (ops.SplitGraph): which side stream runs
// concurrently with a lane launched on the caller's stream?  Two linear
// graphs joined only by flag hand-offs, as scgib_graph_split builds them:
//   lane A: signal(f1), spin 50 us, wait(f2)
//   lane B: wait(f1),   spin 50 us, signal(f2)
// Lane A is launched on the caller's stream (the null stream, as torch's
// default stream, or a non-blocking stream), lane B on a candidate side
// stream.  Waits give up after 20 ms (counted).  Reported per candidate: us
// per replay pair over 50 back-to-back replays and the timed-out waits.
// Build: hipcc --offload-arch=gfx950 -O2 tools/lane_probe.hip -o tools/lane_probe.bin
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

__global__ void sig(unsigned *w) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void wait_k(unsigned *w, unsigned *to) {
    if (threadIdx.x == 0) {
        const unsigned a = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t0 = wall_clock64();
        while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a - 1u >= 0x80000000u) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - t0 > 2000000) {  // 20 ms
                __hip_atomic_fetch_add(to, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                break;
            }
        }
        __hip_atomic_store(w + 1, a + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__global__ void spin(unsigned us) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < 100ull * us) {
    }
}

static hipGraphExec_t lane(bool a, unsigned *f1, unsigned *f2, unsigned *to) {
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    hipGraph_t g;
    (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
    if (a) {
        sig<<<1, 64, 0, s>>>(f1);
        spin<<<1, 64, 0, s>>>(50);
        wait_k<<<1, 64, 0, s>>>(f2, to);
    } else {
        wait_k<<<1, 64, 0, s>>>(f1, to);
        spin<<<1, 64, 0, s>>>(50);
        sig<<<1, 64, 0, s>>>(f2);
    }
    (void)hipStreamEndCapture(s, &g);
    hipGraphExec_t ex;
    (void)hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
    (void)hipStreamDestroy(s);
    return ex;
}

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int ncu = prop.multiProcessorCount;
    unsigned *w;
    if (hipMalloc(&w, 64 * sizeof(unsigned)) != hipSuccess) return 1;
    (void)hipMemset(w, 0, 64 * sizeof(unsigned));
    unsigned *f1 = w, *f2 = w + 4, *to = w + 8;
    hipGraphExec_t ea = lane(true, f1, f2, to), eb = lane(false, f1, f2, to);
    // the null stream has work first (as torch's default stream does)
    spin<<<1, 64, 0, nullptr>>>(1);
    (void)hipDeviceSynchronize();
    // 64 pool-like streams first, as torch's stream pools (32 low + 32 high priority)
    std::vector<hipStream_t> pool(64);
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    for (int i = 0; i < 64; ++i)
        (void)hipStreamCreateWithPriority(&pool[i], hipStreamNonBlocking, i < 32 ? lo : hi);
    for (hipStream_t p : pool) spin<<<1, 64, 0, p>>>(1);
    (void)hipDeviceSynchronize();
    std::vector<unsigned> mask((ncu + 31) / 32, 0u);
    for (int i = 0; i < ncu; ++i) mask[i / 32] |= 1u << (i % 32);
    hipStream_t cand[4], caller_nb;
    (void)hipExtStreamCreateWithCUMask(&cand[0], static_cast<uint32_t>(mask.size()), mask.data());
    (void)hipStreamCreateWithFlags(&cand[1], hipStreamNonBlocking);
    (void)hipStreamCreateWithPriority(&cand[2], hipStreamNonBlocking, hi);
    (void)hipStreamCreateWithPriority(&cand[3], hipStreamNonBlocking, lo);
    (void)hipStreamCreateWithFlags(&caller_nb, hipStreamNonBlocking);
    const char *names[4] = {"CU-mask (blocking)", "non-blocking", "non-blocking high prio",
                            "non-blocking low prio"};
    for (int callers = 0; callers < 2; ++callers) {
        hipStream_t A = callers == 0 ? nullptr : caller_nb;
        for (int c = 0; c < 4; ++c) {
            unsigned t0v = 0;
            (void)hipMemcpy(&t0v, to, 4, hipMemcpyDeviceToHost);
            const auto t0 = std::chrono::steady_clock::now();
            for (int r = 0; r < 50; ++r) {
                (void)hipGraphLaunch(ea, A);
                (void)hipGraphLaunch(eb, cand[c]);
            }
            (void)hipDeviceSynchronize();
            const auto t1 = std::chrono::steady_clock::now();
            unsigned t1v = 0;
            (void)hipMemcpy(&t1v, to, 4, hipMemcpyDeviceToHost);
            printf("caller %-12s side %-24s %8.1f us per replay pair, timed-out waits %u\n",
                   callers == 0 ? "null" : "non-blocking", names[c],
                   std::chrono::duration<double, std::micro>(t1 - t0).count() / 50, t1v - t0v);
        }
    }
    return 0;
}
