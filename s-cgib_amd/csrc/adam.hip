// One-launch Adam step over a list of fp32 tensors (gfx950) — the optimizer
// of every reference training script (torch.optim.Adam(model.parameters(),
// lr, weight_decay=5e-5), e.g. exp_pretraining.py / exp_molhiv.py:53), with
// the arithmetic of torch's fused Adam (L2 weight decay added to the
// gradient, no amsgrad / maximize):
//   t = step + 1;  g += wd * p;  m = b1 m + (1 - b1) g;  v = b2 v + (1 - b2) g^2
//   p -= (lr / (1 - b1^t)) * m / (sqrt(v) / sqrt(1 - b2^t) + eps);  step = t
//
// torch's fused / foreach paths need 4-5 launches per step for a model of
// ~75 small tensors (step increments + chunked multi-tensor kernels); here
// the tensor table (up to 80 tensors: one launch for the pretraining model)
// travels by value in the kernel arguments (captured with the launch in a
// HIP graph), every workgroup handles one 1024-element chunk
// of one tensor, and the last workgroup to finish advances every tensor's
// step counter (all workgroups read the step before they arrive).
#include "common.h"

namespace scgib {

constexpr int kAdamMax = 80;       // tensors per launch (kernel-argument table, < 4 KB)
constexpr int kAdamChunk = 1024;   // elements per workgroup

// structure of arrays (no per-entry padding): 80 tensors in 3.8 KB of kernel
// arguments, so a whole model's ~75 hot-path tensors take one launch
struct AdamTable {
    float *param[kAdamMax];
    const float *grad[kAdamMax];
    float *exp_avg[kAdamMax];
    float *exp_avg_sq[kAdamMax];
    float *step[kAdamMax];
    int32_t numel[kAdamMax];
    int32_t chunk0[kAdamMax + 1];  // first chunk of tensor i; chunk0[n] = grid
    int32_t n;
};
static_assert(sizeof(AdamTable) <= 4096, "kernel-argument table");

struct AdamRef {
    float *param;
    const float *grad;
    float *exp_avg, *exp_avg_sq;
    int64_t numel;
};

// Precision mirrors torch's fused Adam (ATen fused_adam_utils.cuh): the
// hyper-parameters are doubles, so the weight decay, both moment updates and
// eps enter in double and round to fp32 on assignment; the bias corrections
// are computed in double and rounded to fp32; the final update is fp32.
// One element (shared by adam_chunk and the fused reduce + Adam launch, so
// both give the same bits).
__device__ __forceinline__ void adam_elem(float p, float g, float m, float v, float step_size,
                                          float bc2_sqrt, double beta1, double beta2, double eps,
                                          double wd, float &pp, float &mm, float &vv) {
    float gg = g;
    if (wd != 0.0) gg = static_cast<float>(gg + p * wd);
    mm = static_cast<float>(beta1 * m + (1 - beta1) * gg);
    vv = static_cast<float>(beta2 * v + (1 - beta2) * gg * gg);
    const float denom = static_cast<float>(sqrtf(vv) / bc2_sqrt + eps);
    pp = p - step_size * mm / denom;
}

// the tensor's bias corrections at its step t = *step + 1
__device__ __forceinline__ void adam_coef(const float *step, double lr, double beta1,
                                          double beta2, float &step_size, float &bc2_sqrt) {
    const float t = *step + 1.f;
    const float bc1 = static_cast<float>(1 - pow(beta1, static_cast<double>(t)));
    bc2_sqrt = static_cast<float>(sqrt(1 - pow(beta2, static_cast<double>(t))));
    step_size = static_cast<float>(lr / bc1);
}

template <int NT, int EPT = 4>  // threads per workgroup; a chunk is EPT * NT elements
__device__ __forceinline__ void adam_chunk(const AdamRef &T, int64_t base,
                                           float step_size, float bc2_sqrt, double beta1,
                                           double beta2, double eps, double wd) {
    float p[EPT], g[EPT], m[EPT], v[EPT];
    int64_t idx[EPT];
#pragma unroll
    for (int k = 0; k < EPT; ++k) {  // clamped loads (all in flight), masked stores
        const int64_t j = base + threadIdx.x + NT * k;
        idx[k] = j < T.numel ? j : T.numel - 1;
        p[k] = T.param[idx[k]];
        g[k] = T.grad[idx[k]];
        m[k] = T.exp_avg[idx[k]];
        v[k] = T.exp_avg_sq[idx[k]];
    }
#pragma unroll
    for (int k = 0; k < EPT; ++k) {
        float pp, mm, vv;
        adam_elem(p[k], g[k], m[k], v[k], step_size, bc2_sqrt, beta1, beta2, eps, wd, pp, mm, vv);
        if (base + threadIdx.x + NT * k < T.numel) {
            T.param[idx[k]] = pp;
            T.exp_avg[idx[k]] = mm;
            T.exp_avg_sq[idx[k]] = vv;
        }
    }
}

__global__ __launch_bounds__(256) void adam_step_k(const AdamTable tab, double lr, double beta1,
                                                   double beta2, double eps, double wd,
                                                   unsigned *__restrict__ counter) {
    const int b = blockIdx.x;
    // tensor of this chunk: one parallel compare over the table (lane q holds
    // chunk0[q]) instead of a dependent scalar-load chain
    const int lane = threadIdx.x & 63;
    int i = -1;
#pragma unroll
    for (int r = 0; r < (kAdamMax + 63) / 64; ++r) {
        const int q = 64 * r + lane;
        const bool le = q < tab.n && tab.chunk0[q < tab.n ? q : 0] <= b;
        i += __popcll(__ballot(le));
    }
    const AdamRef T{tab.param[i], tab.grad[i], tab.exp_avg[i], tab.exp_avg_sq[i], tab.numel[i]};
    float step_size, bc2_sqrt;
    adam_coef(tab.step[i], lr, beta1, beta2, step_size, bc2_sqrt);
    const int64_t base = static_cast<int64_t>(b - tab.chunk0[i]) * kAdamChunk;
    if (T.numel > 0) adam_chunk<256>(T, base, step_size, bc2_sqrt, beta1, beta2, eps, wd);
    __shared__ unsigned s_last;
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 gridDim.x - 1;
    __syncthreads();
    if (s_last) {  // every workgroup has read its step: advance all of them at once
        if (threadIdx.x < tab.n) *tab.step[threadIdx.x] += 1.f;
        if (threadIdx.x == 0) *counter = 0u;
    }
}

// ---------------------------------------------------------------------------
// The step's last weight-gradient reduce and the Adam step in ONE launch
// (scgib_adam_step_reduce): the reduce's column blocks (slab_reduce_multi_k's
// decomposition and fixed order, so every gradient has the same bits) apply
// Adam to the elements of the tensors whose gradients they produce, right
// where the reduced value is in a register; the other tensors' Adam chunks
// run as the launch's remaining workgroups, beside them.  The replayed
// pretraining step ended with the two launches back to back (the ego chain's
// final reduce after the join, then Adam): one launch boundary and the Adam
// launch's latency leave its tail.
// ---------------------------------------------------------------------------
constexpr int kFuseJobs = 8;
constexpr int kFuseSegs = 16;
// Adam elements per thread in the fused launch: one (a chunk per 1024
// elements, ~96 workgroups for the pretraining model) — with four, QM9
// B = 32 ran 0.2537–0.2552 ms against 0.2519–0.2527 (B = 512 unchanged,
// profiles/r06_noise/fuse_ept_ab.txt).  Build-time A/B hook SCGIB_FUSE_EPT.
#ifndef SCGIB_FUSE_EPT
#define SCGIB_FUSE_EPT 1
#endif
constexpr int kFuseEPT = SCGIB_FUSE_EPT;
constexpr int kFuseChunk = kFuseEPT * 1024;  // Adam elements per 1024-thread workgroup

struct FuseTable {
    scgib_slab_job j[kFuseJobs];
    int32_t blk0[kFuseJobs + 1];  // first column block of job i; blk0[nj] = reduce blocks
    int32_t nj;
    // reduced tensors: table entry t's gradient = elements [o0, o0 + numel) of job's output
    int32_t seg_t[kFuseSegs], seg_job[kFuseSegs], seg_o0[kFuseSegs];
    int32_t ns;
};

__global__ __launch_bounds__(1024) void adam_reduce_k(const AdamTable tab, const FuseTable ft,
                                                      double lr, double beta1, double beta2,
                                                      double eps, double wd,
                                                      unsigned *__restrict__ counter) {
    const int b = blockIdx.x;
    const int lane = threadIdx.x & 63;
    const int nred = ft.blk0[ft.nj];
    __shared__ float red[16][64];
    if (b < nred) {  // block-uniform: one column block of one reduce job
        const int el = threadIdx.x & 63, sp = threadIdx.x >> 6;
        const bool le = lane < ft.nj && ft.blk0[lane < ft.nj ? lane : 0] <= b;
        const int i = __popcll(__ballot(le)) - 1;
        const scgib_slab_job &J = ft.j[i];
        const int64_t e = static_cast<int64_t>(b - ft.blk0[i]) * 64 + el;
        const int64_t stride = J.stride > 0 ? J.stride : J.width;
        // the Adam tensor of this element's gradient, its bias corrections and
        // operands: independent of the sums, so in flight with the slab loads
        int t = -1;
        int64_t o = 0;
        float step_size = 0.f, bc2_sqrt = 1.f, p0 = 0.f, m0 = 0.f, v0 = 0.f;
        if (sp == 0 && e < J.width) {
            for (int q = 0; q < ft.ns; ++q) {
                const int64_t oq = e - ft.seg_o0[q];
                if (ft.seg_job[q] == i && oq >= 0 && oq < tab.numel[ft.seg_t[q]]) {
                    t = ft.seg_t[q];
                    o = oq;
                }
            }
            if (t >= 0) {
                p0 = tab.param[t][o];
                m0 = tab.exp_avg[t][o];
                v0 = tab.exp_avg_sq[t][o];
                adam_coef(tab.step[t], lr, beta1, beta2, step_size, bc2_sqrt);
            }
        }
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
            double sum = 0.0;
#pragma unroll
            for (int k = 0; k < 16; ++k) sum += static_cast<double>(red[k][el]);
            const float g = static_cast<float>(sum);
            J.out[e] = g;
            if (t >= 0) {
                float pp, mm, vv;
                adam_elem(p0, g, m0, v0, step_size, bc2_sqrt, beta1, beta2, eps, wd, pp, mm, vv);
                tab.param[t][o] = pp;
                tab.exp_avg[t][o] = mm;
                tab.exp_avg_sq[t][o] = vv;
            }
        }
    } else {  // an Adam chunk of a tensor whose gradient is already complete
        const int c = b - nred;
        int i = -1;
#pragma unroll
        for (int r = 0; r < (kAdamMax + 63) / 64; ++r) {
            const int q = 64 * r + lane;
            const bool le = q < tab.n && tab.chunk0[q < tab.n ? q : 0] <= c;
            i += __popcll(__ballot(le));
        }
        const AdamRef T{tab.param[i], tab.grad[i], tab.exp_avg[i], tab.exp_avg_sq[i], tab.numel[i]};
        float step_size, bc2_sqrt;
        adam_coef(tab.step[i], lr, beta1, beta2, step_size, bc2_sqrt);
        const int64_t base = static_cast<int64_t>(c - tab.chunk0[i]) * kFuseChunk;
        if (T.numel > 0) adam_chunk<1024, kFuseEPT>(T, base, step_size, bc2_sqrt, beta1, beta2, eps, wd);
    }
    __shared__ unsigned s_last;
    __syncthreads();
    if (threadIdx.x == 0)
        s_last = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                 gridDim.x - 1;
    __syncthreads();
    if (s_last) {  // every workgroup has read its steps: advance all of them at once
        if (threadIdx.x < tab.n) *tab.step[threadIdx.x] += 1.f;
        if (threadIdx.x == 0) *counter = 0u;
    }
}

// ---------------------------------------------------------------------------
// Gradient bucket for the data-parallel all-reduce (dist.GradAllReducer): all
// gradients packed into one flat buffer in ONE launch (and unpacked, scaled
// by 1 / world, in one more) instead of a copy launch per tensor.  Same
// chunk -> tensor scheme as the Adam step; the table travels by value.
// ---------------------------------------------------------------------------
constexpr int kPackMax = 96;

struct PackTable {
    scgib_grad_slice t[kPackMax];
    int32_t chunk0[kPackMax + 1];
    int32_t n;
};

template <bool UNPACK>
__global__ __launch_bounds__(256) void grad_pack_k(const PackTable tab, float *__restrict__ flat,
                                                   float scale) {
    const int b = blockIdx.x, lane = threadIdx.x & 63;
    // tensor of this chunk: parallel compare over the table (two 64-wide rounds)
    int i = -1;
#pragma unroll
    for (int r = 0; r < (kPackMax + 63) / 64; ++r) {
        const int q = 64 * r + lane;
        const bool le = q < tab.n && tab.chunk0[q < tab.n ? q : 0] <= b;
        i += __popcll(__ballot(le));
    }
    const scgib_grad_slice &T = tab.t[i];
    const int64_t base = static_cast<int64_t>(b - tab.chunk0[i]) * kAdamChunk;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t j = base + threadIdx.x + 256 * k;
        if (j < T.numel) {
            if (UNPACK) T.data[j] = scale * flat[T.offset + j];
            else flat[T.offset + j] = T.data[j];
        }
    }
}

static int launch_pack(const scgib_grad_slice *tensors, int32_t n, float *flat, float scale,
                       bool unpack, hipStream_t st) {
    if (n < 0 || n > kPackMax) return SCGIB_EINVAL;
    if (n == 0) return SCGIB_OK;
    if (!tensors || !flat) return SCGIB_EINVAL;
    PackTable tab;
    tab.n = n;
    int64_t chunks = 0;
    for (int i = 0; i < n; ++i) {
        const scgib_grad_slice &T = tensors[i];
        if (T.numel < 0 || T.offset < 0 || (T.numel > 0 && !T.data)) return SCGIB_EINVAL;
        tab.t[i] = T;
        tab.chunk0[i] = static_cast<int32_t>(chunks);
        chunks += (T.numel + kAdamChunk - 1) / kAdamChunk;
        if (chunks > 0x7fffffff) return SCGIB_EUNSUPPORTED;
    }
    tab.chunk0[n] = static_cast<int32_t>(chunks);
    for (int i = n; i < kPackMax; ++i) tab.t[i] = scgib_grad_slice{};
    if (chunks == 0) return SCGIB_OK;
    if (unpack)
        grad_pack_k<true><<<dim3(static_cast<unsigned>(chunks)), 256, 0, st>>>(tab, flat, scale);
    else
        grad_pack_k<false><<<dim3(static_cast<unsigned>(chunks)), 256, 0, st>>>(tab, flat, scale);
    return launch_status();
}

}  // namespace scgib

using namespace scgib;

extern "C" int64_t scgib_adam_max_tensors(void) { return kAdamMax; }

extern "C" int scgib_adam_step(const scgib_adam_tensor *tensors, int32_t n_tensors, double lr,
                               double beta1, double beta2, double eps, double weight_decay,
                               uint32_t *counter, scgib_stream_t stream) {
    if (n_tensors < 0 || n_tensors > kAdamMax) return SCGIB_EINVAL;
    if (n_tensors == 0) return SCGIB_OK;
    if (!tensors || !counter) return SCGIB_EINVAL;
    AdamTable tab;
    tab.n = n_tensors;
    int64_t chunks = 0;
    for (int i = 0; i < n_tensors; ++i) {
        const scgib_adam_tensor &T = tensors[i];
        if (T.numel < 0 || !T.step || (T.numel > 0 && (!T.param || !T.grad || !T.exp_avg ||
                                                       !T.exp_avg_sq)))
            return SCGIB_EINVAL;
        if (T.numel > 0x7fffffff) return SCGIB_EUNSUPPORTED;
        tab.param[i] = T.param;
        tab.grad[i] = T.grad;
        tab.exp_avg[i] = T.exp_avg;
        tab.exp_avg_sq[i] = T.exp_avg_sq;
        tab.step[i] = T.step;
        tab.numel[i] = static_cast<int32_t>(T.numel);
        tab.chunk0[i] = static_cast<int32_t>(chunks);
        chunks += (T.numel + kAdamChunk - 1) / kAdamChunk;
        if (chunks > 0x7fffffff) return SCGIB_EUNSUPPORTED;
    }
    tab.chunk0[n_tensors] = static_cast<int32_t>(chunks);
    if (chunks == 0) {  // only empty tensors: just advance the steps
        tab.chunk0[n_tensors] = 1;
        chunks = 1;
    }
    for (int i = n_tensors; i < kAdamMax; ++i) {
        tab.param[i] = tab.exp_avg[i] = tab.exp_avg_sq[i] = tab.step[i] = nullptr;
        tab.grad[i] = nullptr;
        tab.numel[i] = 0;
    }
    adam_step_k<<<dim3(static_cast<unsigned>(chunks)), 256, 0, as_stream(stream)>>>(
        tab, lr, beta1, beta2, eps, weight_decay, counter);
    return launch_status();
}

extern "C" int64_t scgib_grad_pack_max_tensors(void) { return kPackMax; }

extern "C" int scgib_grad_pack(const scgib_grad_slice *tensors, int32_t n_tensors, float *flat,
                               scgib_stream_t stream) {
    return launch_pack(tensors, n_tensors, flat, 1.f, false, as_stream(stream));
}

extern "C" int scgib_grad_unpack(const scgib_grad_slice *tensors, int32_t n_tensors,
                                 const float *flat, float scale, scgib_stream_t stream) {
    return launch_pack(tensors, n_tensors, const_cast<float *>(flat), scale, true,
                       as_stream(stream));
}

extern "C" int64_t scgib_adam_reduce_max_jobs(void) { return scgib::kFuseJobs; }

extern "C" int scgib_adam_step_reduce(const scgib_adam_tensor *tensors, int32_t n_tensors,
                                      const scgib_slab_job *jobs, int32_t n_jobs, double lr,
                                      double beta1, double beta2, double eps, double weight_decay,
                                      uint32_t *counter, scgib_stream_t stream) {
    using namespace scgib;
    if (n_tensors < 0 || n_tensors > kAdamMax || n_jobs < 0 || n_jobs > kFuseJobs) return SCGIB_EINVAL;
    if (n_jobs == 0) return scgib_adam_step(tensors, n_tensors, lr, beta1, beta2, eps, weight_decay,
                                            counter, stream);
    if (!jobs || !counter || (n_tensors > 0 && !tensors)) return SCGIB_EINVAL;
    FuseTable ft{};
    ft.nj = n_jobs;
    int64_t blocks = 0;
    for (int i = 0; i < n_jobs; ++i) {
        const scgib_slab_job &J = jobs[i];
        if (J.n_slabs <= 0 || J.width <= 0 || !J.slab || !J.out) return SCGIB_EINVAL;
        if (J.stride < 0 || (J.stride > 0 && J.stride < J.width)) return SCGIB_EINVAL;
        ft.j[i] = J;
        ft.blk0[i] = static_cast<int32_t>(blocks);
        blocks += (J.width + 63) / 64;
        if (blocks > 0x3fffffff) return SCGIB_EUNSUPPORTED;
    }
    ft.blk0[n_jobs] = static_cast<int32_t>(blocks);
    AdamTable tab{};
    tab.n = n_tensors;
    int64_t chunks = 0;
    for (int t = 0; t < n_tensors; ++t) {
        const scgib_adam_tensor &T = tensors[t];
        if (T.numel < 0 || !T.step || (T.numel > 0 && (!T.param || !T.grad || !T.exp_avg ||
                                                       !T.exp_avg_sq)))
            return SCGIB_EINVAL;
        if (T.numel > 0x7fffffff) return SCGIB_EUNSUPPORTED;
        tab.param[t] = T.param;
        tab.grad[t] = T.grad;
        tab.exp_avg[t] = T.exp_avg;
        tab.exp_avg_sq[t] = T.exp_avg_sq;
        tab.step[t] = T.step;
        tab.numel[t] = static_cast<int32_t>(T.numel);
        tab.chunk0[t] = static_cast<int32_t>(chunks);
        // a gradient inside a job's output: Adam in the reduce (no chunks of its own);
        // one that straddles an output's edge is refused
        int seg = -1;
        for (int i = 0; i < n_jobs && T.numel > 0; ++i) {
            const float *o0 = jobs[i].out, *o1 = jobs[i].out + jobs[i].width;
            const float *g0 = T.grad, *g1 = T.grad + T.numel;
            if (g0 >= o0 && g1 <= o1) {
                seg = i;
                break;
            }
            if (g0 < o1 && g1 > o0) return SCGIB_EINVAL;
        }
        if (seg >= 0) {
            if (ft.ns == kFuseSegs) return SCGIB_EUNSUPPORTED;
            ft.seg_t[ft.ns] = t;
            ft.seg_job[ft.ns] = seg;
            ft.seg_o0[ft.ns] = static_cast<int32_t>(T.grad - jobs[seg].out);
            ++ft.ns;
        } else {
            chunks += (T.numel + kFuseChunk - 1) / kFuseChunk;
        }
    }
    for (int a = 0; a < ft.ns; ++a)  // each reduced element updates one tensor
        for (int c = a + 1; c < ft.ns; ++c)
            if (ft.seg_job[a] == ft.seg_job[c] &&
                ft.seg_o0[a] < ft.seg_o0[c] + tab.numel[ft.seg_t[c]] &&
                ft.seg_o0[c] < ft.seg_o0[a] + tab.numel[ft.seg_t[a]])
                return SCGIB_EINVAL;
    tab.chunk0[n_tensors] = static_cast<int32_t>(chunks);
    adam_reduce_k<<<dim3(static_cast<unsigned>(blocks + chunks)), 1024, 0, as_stream(stream)>>>(
        tab, ft, lr, beta1, beta2, eps, weight_decay, counter);
    return launch_status();
}
