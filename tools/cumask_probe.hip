// Probe: does a CU-masked stream's kernel keep its CU
// set when it is captured into a HIP graph and replayed?  Two streams from
// hipExtStreamCreateWithCUMask with disjoint masks (CU bits [0, 64) and
// [64, ncu)) each launch a wide kernel whose workgroups record the CU they
// ran on (HW_ID / XCC_ID); eagerly, then captured (fork / join through
// events, the way the step's two encoder chains are captured) and replayed.
// Reported per launch: the distinct CUs used and the overlap of the two sets.
// Build: hipcc --offload-arch=gfx950 -O2 tools/cumask_probe.hip -o tools/cumask_probe.bin
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <set>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e = (x);                                                     \
        if (e != hipSuccess) {                                                  \
            printf("%s -> %s\n", #x, hipGetErrorString(e));                     \
            return 1;                                                           \
        }                                                                       \
    } while (0)

constexpr int kBlocks = 2048;

// every workgroup: spin ~20 us (so the grid spreads over every CU it may use),
// then thread 0 records (XCC_ID << 32) | HW_ID
__global__ void where(unsigned long long *out) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < 2000) {
    }
    if (threadIdx.x == 0)
        out[blockIdx.x] = (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((31 << 11) | 20)) << 32) |
                          static_cast<unsigned>(__builtin_amdgcn_s_getreg((31 << 11) | 4));
}

static std::set<unsigned long long> cus(const std::vector<unsigned long long> &v) {
    std::set<unsigned long long> s;
    for (unsigned long long x : v) {
        const unsigned long long xcc = (x >> 32) & 0xF, hw = x & 0xFFFFFFFFull;
        const unsigned long long cu = (hw >> 8) & 0xF, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
        s.insert((xcc << 16) | (se << 8) | (sh << 4) | cu);
    }
    return s;
}

static void report(const char *tag, const std::vector<unsigned long long> &a,
                   const std::vector<unsigned long long> &b) {
    const std::set<unsigned long long> sa = cus(a), sb = cus(b);
    int both = 0;
    for (unsigned long long x : sa) both += sb.count(x) ? 1 : 0;
    printf("%-28s stream A (mask CUs [0,64)): %3zu CUs   stream B (mask the rest): %3zu CUs   "
           "shared: %d\n", tag, sa.size(), sb.size(), both);
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int ncu = prop.multiProcessorCount;
    printf("device: %s, %d CUs\n", prop.name, ncu);
    const int words = (ncu + 31) / 32;
    std::vector<uint32_t> ma(words, 0u), mb(words, 0u);
    for (int i = 0; i < ncu; ++i) (i < 64 ? ma : mb)[i / 32] |= 1u << (i % 32);
    hipStream_t sa, sb, plain;
    CK(hipExtStreamCreateWithCUMask(&sa, words, ma.data()));
    CK(hipExtStreamCreateWithCUMask(&sb, words, mb.data()));
    CK(hipStreamCreateWithFlags(&plain, hipStreamNonBlocking));
    unsigned long long *da, *db;
    CK(hipMalloc(&da, kBlocks * sizeof(unsigned long long)));
    CK(hipMalloc(&db, kBlocks * sizeof(unsigned long long)));
    std::vector<unsigned long long> ha(kBlocks), hb(kBlocks);
    auto fetch = [&]() -> int {
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ha.data(), da, kBlocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        CK(hipMemcpy(hb.data(), db, kBlocks * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        return 0;
    };
    // 1. eager, both streams at once
    where<<<kBlocks, 64, 0, sa>>>(da);
    where<<<kBlocks, 64, 0, sb>>>(db);
    if (fetch()) return 1;
    report("eager", ha, hb);
    // 2. captured from A with a fork to B and a join back, replayed on A,
    //    then on a plain stream
    hipEvent_t fork, join;
    CK(hipEventCreateWithFlags(&fork, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&join, hipEventDisableTiming));
    hipGraph_t g;
    CK(hipStreamBeginCapture(sa, hipStreamCaptureModeGlobal));
    CK(hipEventRecord(fork, sa));
    CK(hipStreamWaitEvent(sb, fork, 0));
    where<<<kBlocks, 64, 0, sa>>>(da);
    where<<<kBlocks, 64, 0, sb>>>(db);
    CK(hipEventRecord(join, sb));
    CK(hipStreamWaitEvent(sa, join, 0));
    CK(hipStreamEndCapture(sa, &g));
    hipGraphExec_t ex;
    CK(hipGraphInstantiate(&ex, g, nullptr, nullptr, 0));
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipMemset(da, 0, kBlocks * sizeof(unsigned long long)));
        CK(hipMemset(db, 0, kBlocks * sizeof(unsigned long long)));
        CK(hipGraphLaunch(ex, rep == 0 ? sa : plain));
        if (fetch()) return 1;
        report(rep == 0 ? "graph replayed on A" : "graph replayed on a plain stream", ha, hb);
    }
    CK(hipGraphExecDestroy(ex));
    CK(hipGraphDestroy(g));
    CK(hipFree(da));
    CK(hipFree(db));
    CK(hipStreamDestroy(sa));
    CK(hipStreamDestroy(sb));
    CK(hipStreamDestroy(plain));
    return 0;
}
