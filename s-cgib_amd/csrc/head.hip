// Fine-tune prediction head and BCE loss (models.py:510-523): the tail of
// Mainmodel_finetuning.forward after Set2Set,
//   scores = sigmoid(predict(q*)),  predict = Linear(K, 64) - ReLU - Linear(64, C)
// and loss = BCE(scores, targets) (models.py:522-523, mean reduction), with
// their backward.  The torch path issued ~19 launches for this (two rocBLAS
// GEMMs forward and four backward, bias / ReLU / sigmoid / BCE / mean
// elementwise and reduce kernels, copies); here it is four: head forward,
// BCE forward, BCE backward, head backward.  The shapes are tiny (B = 32
// graphs, K = 128, C = 1 or 2), so the kernels are latency work: every
// operand is staged in LDS once, each thread owns a fixed set of outputs and
// sums its terms in a fixed order (deterministic, no atomics).
#include "common.h"
#include "running_update.h"

namespace scgib {

constexpr int kHeadH = 64;      // hidden width (args.dims)
constexpr int kHeadKMax = 128;  // input width (2 * hidden: the Set2Set output)
constexpr int kHeadCMax = 16;   // classes
constexpr int kHeadRows = 16;   // forward: rows per workgroup
constexpr int kHeadChunk = 32;  // backward: rows per chunk
constexpr int kHeadG = 4;       // backward: workgroups (dW1 row / dx column slices)

__device__ __forceinline__ float4 hld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
// K is a multiple of 4 (float4 staging); every operand's loads are issued
// together before its LDS stores (a store-after-load loop waits on each load)

// forward: workgroup = 16 rows; thread (r = tid >> 4, u = tid & 15) owns the
// hidden units u, u + 16, u + 32, u + 48 of row r, then output c of row r for
// c = u, u + 16, ... < C.  LDS rows at stride K + 4 (hidden at 68), read as
// float4 (16-B aligned; lane u's four banks start at 4 u: conflict-free), the
// k order of every sum unchanged (scalar reads at stride K + 1 left ~one LDS
// wait per read: 4.3 us for the hidden units, tools/head_trace.py).  with_ru: one more workgroup runs the
// compressor BatchNorm's running update (running_update.h), which nothing in
// the step reads — instead of its own launch on an aux stream.
__global__ __launch_bounds__(256) void head_fwd_k(const float *__restrict__ x, int64_t B, int K,
                                                  const float *__restrict__ w1,
                                                  const float *__restrict__ b1,
                                                  const float *__restrict__ w2,
                                                  const float *__restrict__ b2, int C, int act,
                                                  float *__restrict__ hid,
                                                  float *__restrict__ out,
                                                  const scgib_running_update ru, int with_ru) {
    if (with_ru && blockIdx.x == gridDim.x - 1) {
        running_update_body<256>(ru);
        return;
    }
    constexpr int LH = kHeadH + 4;
    __shared__ float4 sW1[kHeadH * (kHeadKMax + 4) / 4];
    __shared__ float4 sX[kHeadRows * (kHeadKMax + 4) / 4];
    __shared__ float4 sH[kHeadRows * LH / 4];
    __shared__ float4 sW2[kHeadCMax * LH / 4];
    const int tid = threadIdx.x, K4 = K >> 2, L4 = K4 + 1;  // row strides in float4
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kHeadRows;
    SCGIB_MARK(0);
    const int nv = static_cast<int>(B - row0 < kHeadRows ? B - row0 : kHeadRows);
    // loads: W1 (64 K / 4 <= 2048 float4: 8 per thread), x (16 K / 4: 2), W2 (C 64: 4)
    float4 vw[8], vx[2];
    float vw2[4];
    const int nw = kHeadH * K4, nx = kHeadRows * K4, nw2 = C * kHeadH;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int i = tid + 256 * u;
        vw[u] = hld4(w1 + 4 * (i < nw ? i : nw - 1));
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = tid + 256 * u, ic = i < nx ? i : nx - 1, r = ic / K4;
        vx[u] = hld4(x + (row0 + (r < nv ? r : nv - 1)) * K + 4 * (ic - r * K4));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = tid + 256 * u;
        vw2[u] = w2[i < nw2 ? i : nw2 - 1];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        const int i = tid + 256 * u, j = i / K4;
        if (i < nw) sW1[j * L4 + (i - j * K4)] = vw[u];
    }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int i = tid + 256 * u, r = i / K4;
        if (i < nx) sX[r * L4 + (i - r * K4)] = vx[u];
    }
    float *sW2f = reinterpret_cast<float *>(sW2), *sHf = reinterpret_cast<float *>(sH);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int i = tid + 256 * u;
        if (i < nw2) sW2f[(i / kHeadH) * LH + i % kHeadH] = vw2[u];
    }
    __syncthreads();
    SCGIB_MARK(1);
    const int r = tid >> 4, u = tid & 15;
    float acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = 0.f;
#pragma unroll 4
    for (int k4 = 0; k4 < K4; ++k4) {
        const float4 xv = sX[r * L4 + k4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float4 w = sW1[(u + 16 * i) * L4 + k4];
            acc[i] = fmaf(xv.x, w.x, acc[i]);
            acc[i] = fmaf(xv.y, w.y, acc[i]);
            acc[i] = fmaf(xv.z, w.z, acc[i]);
            acc[i] = fmaf(xv.w, w.w, acc[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = u + 16 * i;
        const float h = fmaxf(acc[i] + b1[j], 0.f);
        sHf[r * LH + j] = h;
        if (r < nv) hid[(row0 + r) * kHeadH + j] = h;
    }
    __syncthreads();
    SCGIB_MARK(2);
    for (int c = u; c < C; c += 16) {
        float o = 0.f;
#pragma unroll 4
        for (int j4 = 0; j4 < kHeadH / 4; ++j4) {
            const float4 h = sH[r * (LH / 4) + j4], w = sW2[c * (LH / 4) + j4];
            o = fmaf(h.x, w.x, o);
            o = fmaf(h.y, w.y, o);
            o = fmaf(h.z, w.z, o);
            o = fmaf(h.w, w.w, o);
        }
        o += b2[c];
        if (act) o = 1.f / (1.f + expf(-o));
        if (r < nv) out[(row0 + r) * C + c] = o;
    }
    SCGIB_MARK(3);
}

// backward, kHeadG workgroups, rows in chunks of 32:
//   do = ds * (act ? s (1 - s) : 1)                      [rows][C]
//   dh = (do W2) [hid > 0]                               [rows][64]  (every workgroup)
//   dW1 += dh^T x, db1 += sum dh   rows j in [16 q, 16 q + 16) of workgroup q
//   dx = dh W1                     columns [kb, ke) of workgroup q (a quarter of the float4 columns)
//   dW2 += do^T hid, db2 += sum do (workgroup 0)
// Output ownership (each thread sums its terms in row / chunk order):
//   dW1[j][k]: j = 16 q + (tid >> 4), k = (tid & 15) + 16 m
//   dx[r][k]:  r = tid >> 3, k = kb + (tid & 7) + 8 m
//   dh[r][j]:  r = tid >> 3, j = (tid & 7) + 8 m;  db1 row j = 16 q + tid (tid < 16);
//   dW2 / db2 column j = tid < 64 (workgroup 0)
// LDS: x rows at stride K + 1, the W1 column slice at stride 33.
constexpr int kHeadSlice = kHeadKMax / kHeadG;  // widest dx column slice

__global__ __launch_bounds__(256) void head_bwd_k(
    const float *__restrict__ x, const float *__restrict__ hid, const float *__restrict__ s,
    const float *__restrict__ ds, int64_t B, int K, const float *__restrict__ w1,
    const float *__restrict__ w2, int C, int act, float *__restrict__ dx,
    float *__restrict__ dw1, float *__restrict__ db1, float *__restrict__ dw2,
    float *__restrict__ db2) {
    __shared__ float sX[kHeadChunk * (kHeadKMax + 1)];
    __shared__ float sW1[kHeadH * (kHeadSlice + 1)];
    __shared__ float sH[kHeadChunk * (kHeadH + 1)];    // hid, then dh
    __shared__ float sDo[kHeadChunk * kHeadCMax];
    __shared__ float sW2[kHeadCMax * kHeadH];
    const int q = blockIdx.x, tid = threadIdx.x, K4 = K >> 2, LK = K + 1;
    constexpr int LS = kHeadSlice + 1;
    // this workgroup's dx columns: float4 columns [q K4 / G, (q + 1) K4 / G)
    const int kb = 4 * ((q * K4) / kHeadG), ke = 4 * (((q + 1) * K4) / kHeadG), s4 = (ke - kb) >> 2;
    auto put4 = [](float *d, const float4 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w; };
    SCGIB_MARK(0);
    {   // once: the W1 column slice (64 x <= 8 float4: 2 per thread) and W2 (C 64: 4)
        const int nw = kHeadH * s4, nw2 = C * kHeadH;
        float4 vw[2];
        float vw2[4];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = tid + 256 * u, ic = i < nw ? i : (nw > 0 ? nw - 1 : 0), j = s4 > 0 ? ic / s4 : 0;
            vw[u] = s4 > 0 ? hld4(w1 + j * K + kb + 4 * (ic - j * s4)) : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + 256 * u;
            vw2[u] = w2[i < nw2 ? i : nw2 - 1];
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = tid + 256 * u;
            if (i < nw) {
                const int j = i / s4;
                put4(sW1 + j * LS + 4 * (i - j * s4), vw[u]);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + 256 * u;
            if (i < nw2) sW2[i] = vw2[u];
        }
    }
    SCGIB_MARK(1);
    const int jw = 16 * q + (tid >> 4), kw = tid & 15;  // dW1 ownership
    const int xr = tid >> 3, kx = tid & 7;              // dx / dh ownership
    float aW1[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) aW1[m] = 0.f;
    float aB1 = 0.f, aB2 = 0.f, aW2[kHeadCMax];
#pragma unroll
    for (int c = 0; c < kHeadCMax; ++c) aW2[c] = 0.f;
    for (int64_t c0 = 0; c0 < B; c0 += kHeadChunk) {
        const int nv = static_cast<int>(B - c0 < kHeadChunk ? B - c0 : kHeadChunk);
        // the chunk's loads: x (32 K / 4 <= 1024 float4: 4 per thread), hid (512: 2),
        // ds / s (32 C <= 512: 2)
        const int nx = nv * K4;
        float4 vx[4], vh[2];
        float vd[2], vs[2];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + 256 * u, ic = i < nx ? i : nx - 1, r = ic / K4;
            vx[u] = hld4(x + (c0 + r) * K + 4 * (ic - r * K4));
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = tid + 256 * u, r = i >> 4;
            vh[u] = hld4(hid + (c0 + (r < nv ? r : nv - 1)) * kHeadH + 4 * (i & 15));
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = tid + 256 * u, ic = i < nv * C ? i : nv * C - 1;
            vd[u] = ds[c0 * C + ic];
            vs[u] = act ? s[c0 * C + ic] : 0.f;
        }
        __syncthreads();  // the previous chunk's reads are done
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int i = tid + 256 * u, r = i / K4;
            if (i < kHeadChunk * K4) {
                float *d = sX + r * LK + 4 * (i - r * K4);
                if (i < nx) put4(d, vx[u]);
                else put4(d, make_float4(0.f, 0.f, 0.f, 0.f));
            }
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = tid + 256 * u, r = i >> 4;
            put4(sH + r * (kHeadH + 1) + 4 * (i & 15), r < nv ? vh[u] : make_float4(0.f, 0.f, 0.f, 0.f));
        }
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int i = tid + 256 * u;
            if (i < kHeadChunk * C) {
                const int r = i / C, c = i - r * C;
                sDo[r * kHeadCMax + c] = i < nv * C ? (act ? vd[u] * (vs[u] * (1.f - vs[u])) : vd[u]) : 0.f;
            }
        }
        __syncthreads();
        if (c0 == 0) SCGIB_MARK(2);
        if (q == 0 && tid < kHeadH) {  // dW2[c][j] += sum_r do[r][c] hid[r][j] (column j = tid); db2 by thread c
#pragma unroll
            for (int c = 0; c < kHeadCMax; ++c) {
                if (c < C) {
                    float a = 0.f;
                    for (int r = 0; r < kHeadChunk; ++r)
                        a = fmaf(sDo[r * kHeadCMax + c], sH[r * (kHeadH + 1) + tid], a);
                    aW2[c] += a;
                }
            }
            if (tid < C) {
                float a = 0.f;
                for (int r = 0; r < kHeadChunk; ++r) a += sDo[r * kHeadCMax + tid];
                aB2 += a;
            }
        }
        float dh[8];  // dh[xr][(tid & 7) + 8 m]
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int j = (tid & 7) + 8 * m;
            float a = 0.f;
            for (int c = 0; c < C; ++c) a = fmaf(sDo[xr * kHeadCMax + c], sW2[c * kHeadH + j], a);
            dh[m] = sH[xr * (kHeadH + 1) + j] > 0.f ? a : 0.f;
        }
        if (c0 == 0) SCGIB_MARK(3);
        __syncthreads();  // every read of hid is done: dh replaces it
#pragma unroll
        for (int m = 0; m < 8; ++m) sH[xr * (kHeadH + 1) + (tid & 7) + 8 * m] = dh[m];
        __syncthreads();
        if (c0 == 0) SCGIB_MARK(4);
        // dW1[jw][k] += dh[r][jw] x[r][k].  Unconditional: a lane-dependent
        // `k < K` here put each FMA and its LDS read in its own exec-masked
        // branch with its own wait (9.3 us of the kernel, tools/head_trace.py);
        // r LK + k < kHeadChunk (kHeadKMax + 1) for every K <= kHeadKMax, and
        // columns k >= K are never written out.  (Rows 4 at a time: fully
        // unrolled, hipcc hoisted all 256 reads into registers and spilled.)
#pragma unroll 4
        for (int r = 0; r < kHeadChunk; ++r) {
            const float d = sH[r * (kHeadH + 1) + jw];
#pragma unroll
            for (int m = 0; m < 8; ++m) aW1[m] = fmaf(d, sX[r * LK + kw + 16 * m], aW1[m]);
        }
        if (tid < 16) {
            float a = 0.f;
            for (int r = 0; r < kHeadChunk; ++r) a += sH[r * (kHeadH + 1) + 16 * q + tid];
            aB1 += a;
        }
        if (c0 == 0) SCGIB_MARK(5);
        if (xr < nv) {  // dx[xr][k] = sum_j dh[xr][j] W1[j][k], k in [kb, ke)
            float a[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) a[m] = 0.f;
            for (int j = 0; j < kHeadH; ++j) {
                const float d = sH[xr * (kHeadH + 1) + j];
#pragma unroll
                for (int m = 0; m < 4; ++m) a[m] = fmaf(d, sW1[j * LS + kx + 8 * m], a[m]);
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int k = kb + kx + 8 * m;
                if (k < ke) dx[(c0 + xr) * K + k] = a[m];
            }
        }
        if (c0 == 0) SCGIB_MARK(6);
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int k = kw + 16 * m;
        if (k < K) dw1[jw * K + k] = aW1[m];
    }
    if (tid < 16) db1[16 * q + tid] = aB1;
    if (q == 0 && tid < kHeadH) {
#pragma unroll
        for (int c = 0; c < kHeadCMax; ++c)
            if (c < C) dw2[c * kHeadH + tid] = aW2[c];
    }
    if (q == 0 && tid < C) db2[tid] = aB2;
    SCGIB_MARK(7);
}

// BCE, mean reduction, as torch's binary_cross_entropy: per element
//   l = (t - 1) max(log(1 - s), -100) - t max(log s, -100)
// summed in a fixed order (fp64) and divided by n; backward
//   ds = g (s - t) / max((1 - s) s, 1e-12) / n.
__global__ __launch_bounds__(256) void bce_fwd_k(const float *__restrict__ s,
                                                 const float *__restrict__ t, int64_t n,
                                                 float *__restrict__ loss) {
    __shared__ double sh[256];
    double a = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += 256) {
        const float sv = s[i], tv = t[i];
        const float l1 = fmaxf(logf(1.f - sv), -100.f), l0 = fmaxf(logf(sv), -100.f);
        a += static_cast<double>((tv - 1.f) * l1 - tv * l0);
    }
    sh[threadIdx.x] = a;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if (static_cast<int>(threadIdx.x) < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) *loss = static_cast<float>(sh[0] / static_cast<double>(n));
}

__global__ __launch_bounds__(256) void bce_bwd_k(const float *__restrict__ s,
                                                 const float *__restrict__ t, int64_t n,
                                                 const float *__restrict__ g,
                                                 float *__restrict__ ds) {
    const float gn = *g / static_cast<float>(n);
    for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
        const float sv = s[i];
        ds[i] = gn * (sv - t[i]) / fmaxf((1.f - sv) * sv, 1e-12f);
    }
}

}  // namespace scgib

using namespace scgib;

static bool head_aligned(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

extern "C" int scgib_head_fwd(const float *x, int64_t n_rows, int32_t k_in, const float *w1,
                              const float *b1, const float *w2, const float *b2, int32_t n_out,
                              int32_t sigmoid, float *hid, float *out,
                              const scgib_running_update *ru, scgib_stream_t stream) {
    if (n_rows < 0 || k_in < 1 || k_in > kHeadKMax || n_out < 1 || n_out > kHeadCMax)
        return SCGIB_EINVAL;
    if (n_rows == 0) return SCGIB_OK;
    if (!x || !w1 || !b1 || !w2 || !b2 || !hid || !out) return SCGIB_EINVAL;
    if (k_in % 4 || !head_aligned(x) || !head_aligned(w1)) return SCGIB_EUNSUPPORTED;
    if (ru && (ru->n_graphs < 1 || !ru->stats || !ru->graph_ptr || !ru->running_mean ||
               !ru->running_var))
        return SCGIB_EINVAL;
    const unsigned grid = static_cast<unsigned>((n_rows + kHeadRows - 1) / kHeadRows + (ru ? 1 : 0));
    head_fwd_k<<<grid, 256, 0, as_stream(stream)>>>(x, n_rows, k_in, w1, b1, w2, b2, n_out,
                                                    sigmoid ? 1 : 0, hid, out,
                                                    ru ? *ru : scgib_running_update{}, ru ? 1 : 0);
    return launch_status();
}

extern "C" int scgib_head_bwd(const float *x, const float *hid, const float *out,
                              const float *d_out, int64_t n_rows, int32_t k_in, const float *w1,
                              const float *w2, int32_t n_out, int32_t sigmoid, float *dx,
                              float *dw1, float *db1, float *dw2, float *db2,
                              scgib_stream_t stream) {
    if (n_rows < 0 || k_in < 1 || k_in > kHeadKMax || n_out < 1 || n_out > kHeadCMax)
        return SCGIB_EINVAL;
    if (n_rows == 0) {  // an empty batch (the forward accepted it): zero weight gradients
        if (!dw1 || !db1 || !dw2 || !db2) return SCGIB_EINVAL;
        hipStream_t st = as_stream(stream);
        hipError_t e = hipMemsetAsync(dw1, 0, sizeof(float) * kHeadH * k_in, st);
        if (e == hipSuccess) e = hipMemsetAsync(db1, 0, sizeof(float) * kHeadH, st);
        if (e == hipSuccess) e = hipMemsetAsync(dw2, 0, sizeof(float) * kHeadH * n_out, st);
        if (e == hipSuccess) e = hipMemsetAsync(db2, 0, sizeof(float) * n_out, st);
        return e == hipSuccess ? SCGIB_OK : static_cast<int>(e);
    }
    if (!x || !hid || !out || !d_out || !w1 || !w2 || !dx || !dw1 || !db1 || !dw2 || !db2)
        return SCGIB_EINVAL;
    if (k_in % 4 || !head_aligned(x) || !head_aligned(w1) || !head_aligned(hid))
        return SCGIB_EUNSUPPORTED;
    head_bwd_k<<<kHeadG, 256, 0, as_stream(stream)>>>(x, hid, out, d_out, n_rows, k_in, w1, w2, n_out,
                                                 sigmoid ? 1 : 0, dx, dw1, db1, dw2, db2);
    return launch_status();
}

extern "C" int scgib_bce_fwd(const float *scores, const float *targets, int64_t n, float *loss,
                             scgib_stream_t stream) {
    if (n < 1 || !scores || !targets || !loss) return SCGIB_EINVAL;
    bce_fwd_k<<<1, 256, 0, as_stream(stream)>>>(scores, targets, n, loss);
    return launch_status();
}

extern "C" int scgib_bce_bwd(const float *scores, const float *targets, int64_t n,
                             const float *g_loss, float *d_scores, scgib_stream_t stream) {
    if (n < 1 || !scores || !targets || !g_loss || !d_scores) return SCGIB_EINVAL;
    const int64_t wg = (n + 255) / 256;
    bce_bwd_k<<<static_cast<unsigned>(wg < 64 ? wg : 64), 256, 0, as_stream(stream)>>>(
        scores, targets, n, g_loss, d_scores);
    return launch_status();
}

#ifdef SCGIB_TRACE
// debug build only: this file's own g_trace (see common.h; scgib_trace_set)
extern "C" int scgib_trace_set_head(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif
