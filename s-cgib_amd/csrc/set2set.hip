// Set2Set attention readout (gfx950): the per-graph half of DGL's Set2Set
// (reference models.py:565, used by Mainmodel_finetuning.forward :515 and
// Mainmodel_domainadapt :271-272; DGL 1.1 nn/pytorch/glob.py semantics):
//
//   e_v = <x_v, q_g>;  alpha_v = exp(e_v - max_g e) / sum_g exp(. - max);
//   readout_g = sum_{v in g} x_v alpha_v
//
// and its backward.  The LSTM cell between the rounds stays with the host
// (models.Set2Set: four [B, 4d] products on rocBLAS, no host sync); this
// kernel replaces the per-round scatter_reduce / exp / index_add / segment
// sum chain of the eager form and its host->device copy of the segment ids,
// so the fine-tune step is capturable in a HIP graph.
//
// One wavefront per graph.  Lane l = 16 q + j: row group q (0..3) takes rows
// p0 + q, p0 + q + 4, ...; lane j holds channels j, j + 16, j + 32, j + 48
// (< d, d <= 64: the MLP output d = 64 and the raw feature widths of
// s2s_rev, e.g. 9).  A row dot is a 16-lane butterfly; a per-channel sum
// over the graph's rows is a per-lane accumulator folded over the four row
// groups at the end.  Latency-bound VALU/shuffle work (a few hundred flops
// per row): no MFMA.
#include "common.h"

namespace scgib {

namespace {

constexpr int kS2SMaxD = 64;

__device__ __forceinline__ float s2s_red16(float v) {
    v += __shfl_xor(v, 1, kWave);
    v += __shfl_xor(v, 2, kWave);
    v += __shfl_xor(v, 4, kWave);
    v += __shfl_xor(v, 8, kWave);
    return v;
}
__device__ __forceinline__ float s2s_red_q(float v) {
    v += __shfl_xor(v, 16, kWave);
    v += __shfl_xor(v, 32, kWave);
    return v;
}
__device__ __forceinline__ float s2s_max_all(float v) {
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, kWave));
    return v;
}

// rows [p0, p1) of graph g (capacity mode: graphs past dims-counted rows are
// empty only if their ptr entries say so; graph_ptr is always maintained)
__device__ __forceinline__ void s2s_rows(const int32_t *__restrict__ ptr, int64_t g, int64_t &p0,
                                         int64_t &p1) {
    p0 = ptr[g];
    p1 = ptr[g + 1];
}

// zero rows [ptr[nseg], nrows) of out (the capacity padding of dfeat)
__device__ __forceinline__ void s2s_zero_tail(const int32_t *__restrict__ ptr, int64_t nseg,
                                              int64_t nrows, int d, float *__restrict__ out,
                                              int64_t blk, int64_t nblk) {
    const int64_t r0 = ptr[nseg];
    for (int64_t i = r0 * d + blk * 64 + threadIdx.x; i < nrows * d; i += nblk * 64) out[i] = 0.f;
}

}  // namespace

// the logit e_r = <x_r, q> of row r for the 16 lanes of its row group (every
// lane of the group returns it)
__device__ __forceinline__ float s2s_logit(const float *__restrict__ x, int64_t r, int d, int j,
                                           const float (&qv)[4]) {
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = j + 16 * k;
        dot = fmaf(c < d ? x[r * d + c] : 0.f, qv[k], dot);
    }
    return s2s_red16(dot);
}

// stat[2 g] = max_g e, stat[2 g + 1] = the softmax denominator.  The logits
// are recomputed in each pass (a 16-lane dot per row) rather than kept: a
// graph may hold any number of rows, and registers / LDS would bound it.
__global__ __launch_bounds__(64) void set2set_fwd_k(const float *__restrict__ x,
                                                    const float *__restrict__ q,
                                                    const int32_t *__restrict__ ptr, int64_t nseg,
                                                    int d, float *__restrict__ stat,
                                                    float *__restrict__ out) {
    const int64_t g = blockIdx.x;
    const int l = threadIdx.x, rq = l >> 4, j = l & 15;
    int64_t p0, p1;
    s2s_rows(ptr, g, p0, p1);
    float qv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = j + 16 * k;
        qv[k] = c < d ? q[g * d + c] : 0.f;
    }
    // (a row group's 16 lanes run a row together: the butterflies stay
    // within active lanes whatever the other groups do)
    float mx = -INFINITY;
    for (int64_t r = p0 + rq; r < p1; r += 4) mx = fmaxf(mx, s2s_logit(x, r, d, j, qv));
    mx = s2s_max_all(mx);
    float den = 0.f;
    for (int64_t r = p0 + rq; r < p1; r += 4) {
        const float a = expf(s2s_logit(x, r, d, j, qv) - mx);
        den += j == 0 ? a : 0.f;
    }
    den = s2s_red_q(s2s_red16(den));
    // readout_c = sum_r x_rc (a_r / den), as feat * (a / den) summed per graph
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t r = p0 + rq; r < p1; r += 4) {
        const float alpha = expf(s2s_logit(x, r, d, j, qv) - mx) / den;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = j + 16 * k;
            acc[k] = fmaf(c < d ? x[r * d + c] : 0.f, alpha, acc[k]);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float s = s2s_red_q(acc[k]);
        const int c = j + 16 * k;
        if (rq == 0 && c < d) out[g * d + c] = s;
    }
    if (l == 0) {
        stat[2 * g] = mx;
        stat[2 * g + 1] = den;
    }
}

// d readout -> d x, d q:  dalpha_v = <g_g, x_v>;  s = sum alpha dalpha;
// de_v = alpha_v (dalpha_v - s);  dx_v = alpha_v g_g + de_v q_g;  dq_g = sum de_v x_v
__global__ __launch_bounds__(64) void set2set_bwd_k(
    const float *__restrict__ x, const float *__restrict__ q, const int32_t *__restrict__ ptr,
    int64_t nseg, int d, const float *__restrict__ stat, const float *__restrict__ gout,
    float *__restrict__ dx, float *__restrict__ dq, int64_t nrows) {
    if (static_cast<int64_t>(blockIdx.x) >= nseg) {  // block-uniform: the padding rows
        s2s_zero_tail(ptr, nseg, nrows, d, dx, blockIdx.x - nseg, gridDim.x - nseg);
        return;
    }
    const int64_t g = blockIdx.x;
    const int l = threadIdx.x, rq = l >> 4, j = l & 15;
    int64_t p0, p1;
    s2s_rows(ptr, g, p0, p1);
    const float mx = stat[2 * g], den = stat[2 * g + 1];
    float gv[4], qv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = j + 16 * k;
        gv[k] = c < d ? gout[g * d + c] : 0.f;
        qv[k] = c < d ? q[g * d + c] : 0.f;
    }
    float s = 0.f;
    for (int64_t r = p0 + rq; r < p1; r += 4) {
        const float alpha = expf(s2s_logit(x, r, d, j, qv) - mx) / den;
        const float da = s2s_logit(x, r, d, j, gv);
        s += j == 0 ? alpha * da : 0.f;
    }
    s = s2s_red_q(s2s_red16(s));
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t r = p0 + rq; r < p1; r += 4) {
        const float alpha = expf(s2s_logit(x, r, d, j, qv) - mx) / den;
        const float de = alpha * (s2s_logit(x, r, d, j, gv) - s);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = j + 16 * k;
            if (c < d) {
                dx[r * d + c] = fmaf(de, qv[k], alpha * gv[k]);
                acc[k] = fmaf(de, x[r * d + c], acc[k]);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float t = s2s_red_q(acc[k]);
        const int c = j + 16 * k;
        if (rq == 0 && c < d) dq[g * d + c] = t;
    }
}

}  // namespace scgib

using namespace scgib;

extern "C" int scgib_set2set_fwd(const float *x, const float *q, const int32_t *graph_ptr,
                                 int64_t n_graphs, int32_t dim, float *stat, float *out,
                                 scgib_stream_t stream) {
    if (n_graphs < 0 || dim < 1 || dim > kS2SMaxD) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (!x || !q || !graph_ptr || !stat || !out) return SCGIB_EINVAL;
    set2set_fwd_k<<<static_cast<unsigned>(n_graphs), 64, 0, as_stream(stream)>>>(
        x, q, graph_ptr, n_graphs, dim, stat, out);
    return launch_status();
}

extern "C" int scgib_set2set_bwd(const float *x, const float *q, const int32_t *graph_ptr,
                                 int64_t n_graphs, int32_t dim, const float *stat,
                                 const float *g_out, float *dx, float *dq, int64_t n_rows,
                                 scgib_stream_t stream) {
    if (n_graphs < 0 || dim < 1 || dim > kS2SMaxD || n_rows < 0) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (!x || !q || !graph_ptr || !stat || !g_out || !dx || !dq) return SCGIB_EINVAL;
    const int64_t tail = (n_rows * dim + 64 * 64 - 1) / (64 * 64);  // padding-zero blocks (<= 64 rows of work each)
    const int64_t extra = tail < 1 ? 1 : (tail > 256 ? 256 : tail);
    set2set_bwd_k<<<static_cast<unsigned>(n_graphs + extra), 64, 0, as_stream(stream)>>>(
        x, q, graph_ptr, n_graphs, dim, stat, g_out, dx, dq, n_rows);
    return launch_status();
}
