// Contrastive loss: standalone kernels and C-ABI (bodies: contrast_body.h;
// the head MLP kernels also run them in extra workgroups, gin_layer.hip).
#include "contrast_body.h"

namespace scgib {

__global__ __launch_bounds__(256) void contrast_fwd_k(ContrastArgs a) {
    __shared__ __attribute__((aligned(16))) float sK1[CT * CLD];
    __shared__ __attribute__((aligned(16))) float sK2[CT * CLD];
    contrast_fwd_body(a, blockIdx.x, blockIdx.y, sK1, sK2);
}

__global__ __launch_bounds__(256) void contrast_bwd_k(ContrastArgs a) {
    __shared__ __attribute__((aligned(16))) float sK1[CT * CLD];
    __shared__ __attribute__((aligned(16))) float sK2[CT * CLD];
    __shared__ __attribute__((aligned(16))) float sW[kContrastBwdW];
    __shared__ float sDj[CT];
    contrast_bwd_body(a, blockIdx.x, blockIdx.y, sK1, sK2, sW, sDj);
}

}  // namespace scgib

using namespace scgib;

extern "C" int64_t scgib_contrastive_workspace_floats(int64_t n_graphs) {
    if (n_graphs <= 0) return 0;
    return contrast_pb_offset(n_graphs) + 128 * n_graphs * static_cast<int64_t>(contrast_splits(n_graphs));
}

extern "C" int64_t scgib_contrastive_counters(int64_t n_graphs) {
    return n_graphs <= 0 ? 0 : 1 + (n_graphs + CR - 1) / CR;
}

extern "C" int scgib_contrastive_fwd(const float *z1, const float *z2, int64_t n_graphs,
                                     float *workspace, float *loss, uint32_t *counters,
                                     scgib_stream_t stream) {
    if (n_graphs <= 0 || !z1 || !z2 || !workspace || !loss || !counters) return SCGIB_EINVAL;
    if (n_graphs > (int64_t{1} << 20)) return SCGIB_EUNSUPPORTED;
    const dim3 grid(static_cast<unsigned>((n_graphs + CR - 1) / CR), contrast_splits(n_graphs));
    ContrastArgs a{z1, z2, n_graphs, workspace, loss, nullptr, nullptr, nullptr, counters,
                   contrast_splits(n_graphs), 0};
    contrast_fwd_k<<<grid, 256, 0, as_stream(stream)>>>(a);
    return launch_status();
}

extern "C" int scgib_contrastive_bwd(const float *z1, const float *z2, int64_t n_graphs,
                                     float *workspace, const float *g_loss, float *dz1,
                                     float *dz2, uint32_t *counters, scgib_stream_t stream) {
    if (n_graphs <= 0 || !z1 || !z2 || !workspace || !g_loss || !dz1 || !dz2 || !counters)
        return SCGIB_EINVAL;
    if (n_graphs > (int64_t{1} << 20)) return SCGIB_EUNSUPPORTED;
    const dim3 grid(static_cast<unsigned>((n_graphs + CR - 1) / CR), contrast_splits(n_graphs));
    ContrastArgs a{z1, z2, n_graphs, workspace, nullptr, g_loss, dz1, dz2, counters + 1,
                   contrast_splits(n_graphs), 0};
    contrast_bwd_k<<<grid, 256, 0, as_stream(stream)>>>(a);
    return launch_status();
}
