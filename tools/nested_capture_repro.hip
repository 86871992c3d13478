// Minimal HIP-only reproduction of the nested-fork stream-capture crash seen
// with torch.cuda.graph (tools/capture_probe.py: every case whose fork is
// taken from a stream that itself joined the capture through a fork crashes
// in capture_end).  No torch: plain hipStreamBeginCapture / event fork-join.
//
//   hipcc --offload-arch=gfx950 -O2 tools/nested_capture_repro.hip -o build/nested_repro
//   build/nested_repro flat      origin -> side -> origin             (one level)
//   build/nested_repro nested    origin -> side -> aux -> side -> origin
//   build/nested_repro sibling   origin -> side, origin -> aux (both from origin)
//   build/nested_repro <mode>_destroy  the same, but every fork/join event is
//        destroyed right after its hipStreamWaitEvent, i.e. during the capture
//        (what torch's Stream.wait_stream does: a temporary Event per call)
//   build/nested_repro <mode>[_destroy]_autofree  instantiate with
//        hipGraphInstantiateFlagAutoFreeOnLaunch
// Each prints the step it reached, so a crash names the failing API call.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::printf("%s -> %s\n", #x, hipGetErrorString(e_));                        \
            return 1;                                                                    \
        }                                                                                \
    } while (0)

__global__ void scale(float *p, float s, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] *= s;
}

static void step(const char *what) {
    std::printf("%s\n", what);
    std::fflush(stdout);
}

static bool g_destroy = false;
static hipEvent_t g_ev[6];

// record on `from`, make `to` wait, optionally destroy the event at once
static hipError_t fork_join(hipStream_t from, hipStream_t to, int i) {
    hipError_t e = hipEventRecord(g_ev[i], from);
    if (e != hipSuccess) return e;
    e = hipStreamWaitEvent(to, g_ev[i], 0);
    if (e != hipSuccess || !g_destroy) return e;
    e = hipEventDestroy(g_ev[i]);
    g_ev[i] = nullptr;
    return e;
}

int main(int argc, char **argv) {
    char mbuf[64];
    std::snprintf(mbuf, sizeof(mbuf), "%s", argc > 1 ? argv[1] : "nested");
    bool autofree = false;
    if (char *suf = std::strstr(mbuf, "_autofree")) {  // torch's instantiate flag
        autofree = true;
        *suf = 0;
    }
    if (char *suf = std::strstr(mbuf, "_destroy")) {
        g_destroy = true;
        *suf = 0;
    }
    const char *mode = mbuf;
    const int n = 1024;
    float *d = nullptr;
    CK(hipMalloc(&d, n * sizeof(float)));
    CK(hipMemset(d, 0, n * sizeof(float)));
    hipStream_t origin, side, aux;
    CK(hipStreamCreateWithFlags(&origin, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&side, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&aux, hipStreamNonBlocking));
    for (auto &e : g_ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));

    CK(hipStreamBeginCapture(origin, hipStreamCaptureModeGlobal));  // as torch.cuda.graph
    step("begin capture");
    scale<<<4, 256, 0, origin>>>(d, 2.f, n);
    CK(fork_join(origin, side, 0));  // side joins the capture
    step("fork origin -> side");
    if (!std::strcmp(mode, "nested")) {
        CK(fork_join(side, aux, 1));  // aux forked from side
        step("fork side -> aux");
        scale<<<4, 256, 0, aux>>>(d, 3.f, n);
        CK(fork_join(aux, side, 2));  // aux joins back into side
        step("join aux -> side");
    } else if (!std::strcmp(mode, "sibling")) {
        CK(fork_join(origin, aux, 4));  // aux forked from origin too
        scale<<<4, 256, 0, aux>>>(d, 3.f, n);
        CK(fork_join(aux, origin, 2));
        step("sibling aux forked and joined at origin");
    }
    scale<<<4, 256, 0, side>>>(d, 5.f, n);
    CK(fork_join(side, origin, 3));  // side joins back into origin
    step("join side -> origin");
    hipGraph_t graph = nullptr;
    step("end capture ...");
    CK(hipStreamEndCapture(origin, &graph));
    step("end capture ok");
    hipGraphExec_t exec = nullptr;
    if (autofree)
        CK(hipGraphInstantiateWithFlags(&exec, graph, hipGraphInstantiateFlagAutoFreeOnLaunch));
    else
        CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    step("instantiate ok");
    CK(hipGraphLaunch(exec, origin));
    CK(hipStreamSynchronize(origin));
    float h = 0.f;
    CK(hipMemcpy(&h, d, sizeof(float), hipMemcpyDeviceToHost));
    std::printf("%s: replay ok (d[0] = %g)\n", mode, h);
    return 0;
}
