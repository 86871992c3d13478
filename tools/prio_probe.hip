// Probe: does a kernel captured from a prioritised stream carry the stream's
// priority as its graph-node attribute (hipLaunchAttributePriority)?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *p) { if (threadIdx.x == 0) p[blockIdx.x] = blockIdx.x; }
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s -> %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
int main() {
    int lo, hi;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    printf("priority range least=%d greatest=%d\n", lo, hi);
    int *d;
    CK(hipMalloc(&d, 4096));
    for (int prio : {lo, hi}) {
        hipStream_t s;
        CK(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, prio));
        hipGraph_t g;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        k<<<4, 64, 0, s>>>(d);
        CK(hipStreamEndCapture(s, &g));
        size_t n = 0;
        CK(hipGraphGetNodes(g, nullptr, &n));
        hipGraphNode_t nodes[4];
        CK(hipGraphGetNodes(g, nodes, &n));
        hipKernelNodeAttrValue v{};
        hipError_t e = hipGraphKernelNodeGetAttribute(nodes[0], hipKernelNodeAttributePriority, &v);
        printf("stream priority %d: node attr rc=%s priority=%d\n", prio, hipGetErrorString(e), v.priority);
        hipGraphExec_t ex;
        e = hipGraphInstantiateWithFlags(&ex, g, hipGraphInstantiateFlagUseNodePriority);
        printf("instantiate with UseNodePriority: %s\n", hipGetErrorString(e));
        if (e == hipSuccess) {
            CK(hipGraphLaunch(ex, s));
            CK(hipStreamSynchronize(s));
            CK(hipGraphExecDestroy(ex));
        }
        CK(hipGraphDestroy(g));
        CK(hipStreamDestroy(s));
    }
    CK(hipFree(d));
    return 0;
}
