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

// Several independent slab reductions in one launch (e.g. the five layers of
// an encoder's backward, reduced once at its end instead of one launch per
// layer): workgroup -> (job, 64-column block) through the job table in the
// kernel arguments; each job is summed exactly as slab_reduce_k does, over a
// column range of its slabs when the job's row stride exceeds its width.
constexpr int kSlabJobs = 16;

struct SlabJobs {
    scgib_slab_job j[kSlabJobs];
    int32_t blk0[kSlabJobs + 1];  // first column block of job i
    int32_t n;
};

// grid-stride over the column blocks (gridDim.x may be capped so that a
// reduce running beside another chain holds few CU slots)
__global__ __launch_bounds__(1024) void slab_reduce_multi_k(const SlabJobs jobs) {
    const int lane = threadIdx.x & 63;
    const int el = threadIdx.x & 63, sp = threadIdx.x >> 6;
    __shared__ float red[16][64];
    for (int b = blockIdx.x; b < jobs.blk0[jobs.n]; b += gridDim.x) {  // block-uniform
        const bool le = lane < jobs.n && jobs.blk0[lane < jobs.n ? lane : 0] <= b;
        const int i = __popcll(__ballot(le)) - 1;
        const scgib_slab_job &J = jobs.j[i];
        const int64_t e = static_cast<int64_t>(b - jobs.blk0[i]) * 64 + el;
        const int64_t stride = J.stride > 0 ? J.stride : J.width;
        float acc = 0.f;
        if (e < J.width) {
            for (int b0 = sp; b0 < J.n_slabs; b0 += 16 * 8) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    v[u] = ld_ok(J.slab, static_cast<int64_t>(b0 + 16 * u) * stride + e, e,
                                 b0 + 16 * u < J.n_slabs, 0.f);
#pragma unroll
                for (int u = 0; u < 8; ++u) acc += v[u];
            }
        }
        red[sp][el] = acc;
        __syncthreads();
        if (sp == 0 && e < J.width) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 16; ++k) s += static_cast<double>(red[k][el]);
            J.out[e] = static_cast<float>(s);
        }
        __syncthreads();  // red is rewritten by the next column block
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

extern "C" int64_t scgib_slab_reduce_max_jobs(void) { return scgib::kSlabJobs; }

extern "C" int scgib_slab_reduce_multi(const scgib_slab_job *jobs, int32_t n_jobs,
                                       scgib_stream_t stream) {
    return scgib_slab_reduce_multi_ex(jobs, n_jobs, 0, stream);
}

extern "C" int scgib_slab_reduce_multi_ex(const scgib_slab_job *jobs, int32_t n_jobs,
                                          int32_t max_workgroups, scgib_stream_t stream) {
    if (n_jobs < 0 || n_jobs > scgib::kSlabJobs || max_workgroups < 0) return SCGIB_EINVAL;
    if (n_jobs == 0) return SCGIB_OK;
    if (!jobs) return SCGIB_EINVAL;
    scgib::SlabJobs t{};
    t.n = n_jobs;
    int64_t blocks = 0;
    for (int i = 0; i < n_jobs; ++i) {
        const scgib_slab_job &J = jobs[i];
        if (J.n_slabs <= 0 || J.width <= 0 || !J.slab || !J.out) return SCGIB_EINVAL;
        if (J.stride < 0 || (J.stride > 0 && J.stride < J.width)) return SCGIB_EINVAL;
        t.j[i] = J;
        t.blk0[i] = static_cast<int32_t>(blocks);
        blocks += (J.width + 63) / 64;
        if (blocks > 0x7fffffff) return SCGIB_EUNSUPPORTED;
    }
    t.blk0[n_jobs] = static_cast<int32_t>(blocks);
    if (max_workgroups > 0 && blocks > max_workgroups) blocks = max_workgroups;
    scgib::slab_reduce_multi_k<<<dim3(static_cast<unsigned>(blocks)), 1024, 0,
                                 scgib::as_stream(stream)>>>(t);
    return scgib::launch_status();
}
