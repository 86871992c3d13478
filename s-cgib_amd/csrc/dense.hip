// Fused 64 -> 64 Linear (+ bias) of the head (gfx950), exact-f32 MFMA tiles:
// compressor[0] of Mainmodel (models.py:589-592, applied at :596 and for the
// continue wrapper :1081-1084 / :1092):  t = f W^T + b.
//
// Forward: one 64-row tile per workgroup, out = x W^T + b.
// Backward: workgroups loop over tiles (grid <= 256), dW = dy^T x and
// db = sum dy accumulate in MFMA registers and land in one slab per
// workgroup (fixed-order slab reduce after), dx = [add +] dy W per tile —
// `add` folds the other gradient of x (the interaction's d f) into the same
// pass.  Capacity mode (dims): rows >= dims[0] are written as zeros.
#include "mfma_tile.h"

namespace scgib {

__global__ __launch_bounds__(256) void linear_fwd_k(const float *__restrict__ x,
                                                    const float *__restrict__ w,
                                                    const float *__restrict__ b, int64_t ncap,
                                                    float *__restrict__ out,
                                                    const int32_t *__restrict__ dims) {
    __shared__ float sA[TM * LDH];
    __shared__ float sW[64 * LDH];
    const int64_t n = eff_count(dims, 0, ncap);
    const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, wr = wv >> 1, wc = wv & 1;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * TM;
    const int nv = static_cast<int>(n - row0 < TM ? (n - row0 > 0 ? n - row0 : 0) : TM);
    if (dims) {
        const int ncr = static_cast<int>(ncap - row0 < TM ? ncap - row0 : TM);
        for (int idx = nv * 64 + tid; idx < ncr * 64; idx += 256) out[row0 * 64 + idx] = 0.f;
        if (nv == 0) return;
    }
    stage_matrix<64>(w, sW);
    {
        float4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int idx = tid + 256 * k, rr = idx >> 4, cq = idx & 15;
            v[k] = ld_ok(reinterpret_cast<const float4 *>(x), (row0 + rr) * 16 + cq, row0 * 16 + cq,
                         rr < nv, make_float4(0.f, 0.f, 0.f, 0.f));
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int idx = tid + 256 * k, rr = idx >> 4, cq = idx & 15;
            float *d = sA + rr * LDH + 4 * cq;
            d[0] = v[k].x; d[1] = v[k].y; d[2] = v[k].z; d[3] = v[k].w;
        }
    }
    __syncthreads();
    const int ccol = wc * 32 + (l & 31);
    f32x16 acc = mma_nt<64>(sA + wr * 32 * LDH, LDH, sW + wc * 32 * LDH, LDH, zero16());
    const float bias = b ? b[ccol] : 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = wr * 32 + acc_row(reg, l);
        if (row < nv) out[(row0 + row) * 64 + ccol] = acc[reg] + bias;
    }
}

// slab per workgroup: dW[64*64] | db[64]
constexpr int kLinSlab = 64 * 64 + 64;

__global__ __launch_bounds__(256) void linear_bwd_k(
    const float *__restrict__ dy, const float *__restrict__ x, const float *__restrict__ w,
    int64_t ncap, int64_t ntiles, const float *__restrict__ add, float *__restrict__ dx,
    float *__restrict__ slab, const int32_t *__restrict__ dims) {
    __shared__ float sD[TM * LDH];
    __shared__ float sA[TM * LDH];
    __shared__ float sW[64 * LDH];
    const int64_t n = eff_count(dims, 0, ncap);
    const int tid = threadIdx.x, l = tid & 63, wv = tid >> 6, wr = wv >> 1, wc = wv & 1;
    const int ch = tid & 63, q = tid >> 6;
    stage_matrix<64>(w, sW);
    f32x16 accW = zero16();
    float db = 0.f;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row0 = tile * TM;
        const int nv = static_cast<int>(n - row0 < TM ? (n - row0 > 0 ? n - row0 : 0) : TM);
        if (dims) {
            const int ncr = static_cast<int>(ncap - row0 < TM ? ncap - row0 : TM);
            for (int idx = nv * 64 + tid; idx < ncr * 64; idx += 256) dx[row0 * 64 + idx] = 0.f;
            if (nv == 0) continue;  // block-uniform
        }
        float4 vd[4], va[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int idx = tid + 256 * k, rr = idx >> 4, cq = idx & 15;
            const int64_t o = (row0 + rr) * 16 + cq, so = row0 * 16 + cq;
            const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
            vd[k] = ld_ok(reinterpret_cast<const float4 *>(dy), o, so, rr < nv, z4);
            va[k] = ld_ok(reinterpret_cast<const float4 *>(x), o, so, rr < nv, z4);
        }
        __syncthreads();  // previous tile's LDS reads are done
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int idx = tid + 256 * k, rr = idx >> 4, cq = idx & 15;
            float *d = sD + rr * LDH + 4 * cq, *a = sA + rr * LDH + 4 * cq;
            d[0] = vd[k].x; d[1] = vd[k].y; d[2] = vd[k].z; d[3] = vd[k].w;
            a[0] = va[k].x; a[1] = va[k].y; a[2] = va[k].z; a[3] = va[k].w;
        }
        __syncthreads();
        const int ccol = wc * 32 + (l & 31);
        // the addend rows, loaded unconditionally (clamped rows) ahead of the
        // products: behind the store's row predicate each load was waited for
        // on its own
        float addv[16];
        if (add) {
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = wr * 32 + acc_row(reg, l);
                addv[reg] = add[(row0 + (row < nv ? row : nv - 1)) * 64 + ccol];
            }
        }
        accW = mma_tn<TM>(sD + wr * 32, LDH, sA + wc * 32, LDH, accW);
        db = col_sum16(db, sD + q * LDH + ch, 4 * LDH);
        f32x16 g = mma_nn<64>(sD + wr * 32 * LDH, LDH, sW + wc * 32, LDH, zero16());
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = wr * 32 + acc_row(reg, l);
            if (row < nv) dx[(row0 + row) * 64 + ccol] = add ? addv[reg] + g[reg] : g[reg];
        }
    }
    float *sl = slab + static_cast<int64_t>(blockIdx.x) * kLinSlab;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int j = wr * 32 + acc_row(reg, l), k = wc * 32 + (l & 31);
        sl[j * 64 + k] = accW[reg];
    }
    __shared__ float sB[4][64];
    sB[q][ch] = db;
    __syncthreads();
    if (tid < 64) sl[64 * 64 + ch] = ((sB[0][ch] + sB[1][ch]) + sB[2][ch]) + sB[3][ch];
}

static int lin_grid(int64_t ntiles) { return static_cast<int>(ntiles < 256 ? ntiles : 256); }

}  // namespace scgib

using namespace scgib;

extern "C" int64_t scgib_linear_slab_floats(int64_t n_nodes) {
    return n_nodes <= 0 ? 0 : static_cast<int64_t>(lin_grid((n_nodes + TM - 1) / TM)) * kLinSlab;
}

extern "C" int scgib_linear_fwd(const float *x, int64_t n_nodes, const float *w, const float *b,
                                float *out, const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes < 0) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!x || !w || !out) return SCGIB_EINVAL;
    const unsigned grid = static_cast<unsigned>((n_nodes + TM - 1) / TM);
    linear_fwd_k<<<grid, 256, 0, as_stream(stream)>>>(x, w, b, n_nodes, out, dims);
    return launch_status();
}

extern "C" int scgib_linear_bwd(const float *dy, const float *x, const float *w, int64_t n_nodes,
                                const float *add, float *dx, float *slab, float *wgrad,
                                const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes <= 0 || !dy || !x || !w || !dx || !slab) return SCGIB_EINVAL;
    const int64_t nt = (n_nodes + TM - 1) / TM;
    const int grid = lin_grid(nt);
    hipStream_t st = as_stream(stream);
    linear_bwd_k<<<grid, 256, 0, st>>>(dy, x, w, n_nodes, nt, add, dx, slab, dims);
    const int rc = launch_status();
    if (rc != SCGIB_OK || !wgrad) return rc;  // wgrad NULL: the caller reduces the slabs
    return launch_slab_reduce(slab, grid, kLinSlab, wgrad, st);
}
