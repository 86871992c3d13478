// Fixed-order reduction of per-workgroup weight-gradient slabs (shared by the
// fused GIN layer and dense kernels).
#include "mfma_tile.h"

namespace scgib {

// Fixed-order sum of the per-workgroup weight-gradient slabs, one launch:
// workgroup = 64 consecutive slab elements x 16 slab partitions (coalesced
// 256-byte rows per wave); partition s sums slabs s, s + 16, ... (fp32, 8
// loads in flight), then partition 0 adds the 16 partials in order (fp64).
__global__ __launch_bounds__(1024) void slab_reduce_k(const float *__restrict__ slab, int nslab,
                                                      int64_t width, float *__restrict__ out) {
    const int el = threadIdx.x & 63, sp = threadIdx.x >> 6;
    const int64_t e = static_cast<int64_t>(blockIdx.x) * 64 + el;
    __shared__ float red[16][64];
    float acc = 0.f;
    if (e < width) {
        for (int b0 = sp; b0 < nslab; b0 += 16 * 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                v[u] = ld_ok(slab, static_cast<int64_t>(b0 + 16 * u) * width + e, e, b0 + 16 * u < nslab, 0.f);
#pragma unroll
            for (int u = 0; u < 8; ++u) acc += v[u];
        }
    }
    red[sp][el] = acc;
    __syncthreads();
    if (sp == 0 && e < width) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) s += static_cast<double>(red[k][el]);
        out[e] = static_cast<float>(s);
    }
}

int launch_slab_reduce(const float *slab, int nslab, int64_t width, float *out, hipStream_t st) {
    slab_reduce_k<<<dim3(static_cast<unsigned>((width + 63) / 64)), 1024, 0, st>>>(slab, nslab, width, out);
    return launch_status();
}

}  // namespace scgib

extern "C" int scgib_slab_reduce(const float *slab, int32_t n_slabs, int64_t width, float *out,
                                 scgib_stream_t stream) {
    if (n_slabs <= 0 || width <= 0 || !slab || !out) return SCGIB_EINVAL;
    return scgib::launch_slab_reduce(slab, n_slabs, width, out, scgib::as_stream(stream));
}
