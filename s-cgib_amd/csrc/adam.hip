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
__device__ __forceinline__ void adam_chunk(const AdamRef &T, int64_t base,
                                           float step_size, float bc2_sqrt, double beta1,
                                           double beta2, double eps, double wd) {
    float p[4], g[4], m[4], v[4];
    int64_t idx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // clamped loads (all in flight), masked stores
        const int64_t j = base + threadIdx.x + 256 * k;
        idx[k] = j < T.numel ? j : T.numel - 1;
        p[k] = T.param[idx[k]];
        g[k] = T.grad[idx[k]];
        m[k] = T.exp_avg[idx[k]];
        v[k] = T.exp_avg_sq[idx[k]];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        float gg = g[k];
        if (wd != 0.0) gg = static_cast<float>(gg + p[k] * wd);
        const float mm = static_cast<float>(beta1 * m[k] + (1 - beta1) * gg);
        const float vv = static_cast<float>(beta2 * v[k] + (1 - beta2) * gg * gg);
        const float denom = static_cast<float>(sqrtf(vv) / bc2_sqrt + eps);
        const float pp = p[k] - step_size * mm / denom;
        if (base + threadIdx.x + 256 * k < T.numel) {
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
    const float t = *tab.step[i] + 1.f;
    const float bc1 = static_cast<float>(1 - pow(beta1, static_cast<double>(t)));
    const float bc2_sqrt = static_cast<float>(sqrt(1 - pow(beta2, static_cast<double>(t))));
    const float step_size = static_cast<float>(lr / bc1);
    const int64_t base = static_cast<int64_t>(b - tab.chunk0[i]) * kAdamChunk;
    if (T.numel > 0) adam_chunk(T, base, step_size, bc2_sqrt, beta1, beta2, eps, wd);
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
