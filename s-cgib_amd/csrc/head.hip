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

namespace scgib {

constexpr int kHeadH = 64;      // hidden width (args.dims)
constexpr int kHeadKMax = 128;  // input width (2 * hidden: the Set2Set output)
constexpr int kHeadCMax = 16;   // classes
constexpr int kHeadRows = 16;   // forward: rows per workgroup
constexpr int kHeadChunk = 32;  // backward: rows per chunk

// forward: workgroup = 16 rows; thread (r = tid >> 4, u = tid & 15) owns the
// hidden units u, u + 16, u + 32, u + 48 of row r (LDS W1 rows at stride
// K + 1: the 16 lanes of a row read 16 different banks), then output c of
// row r for c = u, u + 16, ... < C.
__global__ __launch_bounds__(256) void head_fwd_k(const float *__restrict__ x, int64_t B, int K,
                                                  const float *__restrict__ w1,
                                                  const float *__restrict__ b1,
                                                  const float *__restrict__ w2,
                                                  const float *__restrict__ b2, int C, int act,
                                                  float *__restrict__ hid,
                                                  float *__restrict__ out) {
    __shared__ float sW1[kHeadH * (kHeadKMax + 1)];
    __shared__ float sX[kHeadRows * (kHeadKMax + 1)];
    __shared__ float sH[kHeadRows * (kHeadH + 1)];
    __shared__ float sW2[kHeadCMax * (kHeadH + 1)];
    const int tid = threadIdx.x, LK = K + 1;
    const int64_t row0 = static_cast<int64_t>(blockIdx.x) * kHeadRows;
    const int nv = static_cast<int>(B - row0 < kHeadRows ? B - row0 : kHeadRows);
    for (int i = tid; i < kHeadH * K; i += 256) sW1[(i / K) * LK + i % K] = w1[i];
    for (int i = tid; i < kHeadRows * K; i += 256) {
        const int r = i / K;
        sX[r * LK + i % K] = x[(row0 + (r < nv ? r : nv - 1)) * K + i % K];
    }
    for (int i = tid; i < C * kHeadH; i += 256) sW2[(i / kHeadH) * (kHeadH + 1) + i % kHeadH] = w2[i];
    __syncthreads();
    const int r = tid >> 4, u = tid & 15;
    float acc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = 0.f;
    for (int k = 0; k < K; ++k) {
        const float xv = sX[r * LK + k];
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = fmaf(xv, sW1[(u + 16 * i) * LK + k], acc[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int j = u + 16 * i;
        const float h = fmaxf(acc[i] + b1[j], 0.f);
        sH[r * (kHeadH + 1) + j] = h;
        if (r < nv) hid[(row0 + r) * kHeadH + j] = h;
    }
    __syncthreads();
    for (int c = u; c < C; c += 16) {
        float o = 0.f;
        for (int j = 0; j < kHeadH; ++j) o = fmaf(sH[r * (kHeadH + 1) + j], sW2[c * (kHeadH + 1) + j], o);
        o += b2[c];
        if (act) o = 1.f / (1.f + expf(-o));
        if (r < nv) out[(row0 + r) * C + c] = o;
    }
}

// backward, one workgroup, rows in chunks of 32:
//   do = ds * (act ? s (1 - s) : 1)                      [rows][C]
//   dh = (do W2) [hid > 0]                               [rows][64]
//   dW2 += do^T hid, db2 += sum do, dW1 += dh^T x, db1 += sum dh, dx = dh W1
// Output ownership (each thread sums its terms in row / chunk order):
//   dW1[j][k]: j = tid >> 2, k in [32 (tid & 3), +32)  (8 float4 x reads per row)
//   dx[r][k]:  r = tid >> 3, k in [16 (tid & 7), +16)  (4 float4 W1 reads per j)
//   dh[r][j]:  r = tid >> 3, j = (tid & 7) + 8 m;  db1 / dW2 column j = tid < 64
// LDS rows of x and W1 at stride K + 4 (16-byte aligned float4 runs).
constexpr int kHeadLK = kHeadKMax + 4;

__global__ __launch_bounds__(256) void head_bwd_k(
    const float *__restrict__ x, const float *__restrict__ hid, const float *__restrict__ s,
    const float *__restrict__ ds, int64_t B, int K, const float *__restrict__ w1,
    const float *__restrict__ w2, int C, int act, float *__restrict__ dx,
    float *__restrict__ dw1, float *__restrict__ db1, float *__restrict__ dw2,
    float *__restrict__ db2) {
    __shared__ __attribute__((aligned(16))) float sW1[kHeadH * kHeadLK];
    __shared__ __attribute__((aligned(16))) float sX[kHeadChunk * kHeadLK];
    __shared__ float sH[kHeadChunk * (kHeadH + 1)];    // hid, then dh
    __shared__ float sDo[kHeadChunk * kHeadCMax];
    __shared__ float sW2[kHeadCMax * kHeadH];
    const int tid = threadIdx.x;
    // K padded to a multiple of 32 with zero columns (x and W1), so every
    // thread's k runs are whole float4s
    const int KP = (K + 31) & ~31;
    for (int i = tid; i < kHeadH * KP; i += 256) {
        const int j = i / KP, k = i % KP;
        sW1[j * kHeadLK + k] = k < K ? w1[j * K + k] : 0.f;
    }
    for (int i = tid; i < C * kHeadH; i += 256) sW2[i] = w2[i];
    const int jw = tid >> 2, kb = (tid & 3) * 32;   // dW1 ownership
    const int xr = tid >> 3, kx = (tid & 7) * 16;   // dx / dh ownership
    const bool w_on = kb < KP, x_on = kx < KP;      // (wave-divergent only for K < 128)
    float4 aW1[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) aW1[m] = make_float4(0.f, 0.f, 0.f, 0.f);
    float aB1 = 0.f, aB2 = 0.f, aW2[kHeadCMax];
#pragma unroll
    for (int c = 0; c < kHeadCMax; ++c) aW2[c] = 0.f;
    for (int64_t c0 = 0; c0 < B; c0 += kHeadChunk) {
        const int nv = static_cast<int>(B - c0 < kHeadChunk ? B - c0 : kHeadChunk);
        __syncthreads();  // the previous chunk's reads are done
        for (int i = tid; i < kHeadChunk * KP; i += 256) {
            const int r = i / KP, k = i % KP;
            sX[r * kHeadLK + k] = (r < nv && k < K) ? x[(c0 + r) * K + k] : 0.f;
        }
        for (int i = tid; i < kHeadChunk * kHeadH; i += 256) {
            const int r = i >> 6;
            sH[r * (kHeadH + 1) + (i & 63)] = r < nv ? hid[(c0 + r) * kHeadH + (i & 63)] : 0.f;
        }
        for (int i = tid; i < kHeadChunk * C; i += 256) {
            const int r = i / C, c = i % C;
            float d = 0.f;
            if (r < nv) {
                d = ds[(c0 + r) * C + c];
                if (act) {
                    const float sv = s[(c0 + r) * C + c];
                    d = d * (sv * (1.f - sv));
                }
            }
            sDo[r * kHeadCMax + c] = d;
        }
        __syncthreads();
        if (tid < kHeadH) {  // dW2[c][j] += sum_r do[r][c] hid[r][j] (column j = tid); db2 by thread c
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
        __syncthreads();  // every read of hid is done: dh replaces it
#pragma unroll
        for (int m = 0; m < 8; ++m) sH[xr * (kHeadH + 1) + (tid & 7) + 8 * m] = dh[m];
        __syncthreads();
        if (w_on) {  // dW1[jw][kb..kb+31] += sum_r dh[r][jw] x[r][kb..]
            for (int r = 0; r < kHeadChunk; ++r) {
                const float d = sH[r * (kHeadH + 1) + jw];
                const float4 *xp = reinterpret_cast<const float4 *>(sX + r * kHeadLK + kb);
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    const float4 v = xp[m];
                    aW1[m] = make_float4(fmaf(d, v.x, aW1[m].x), fmaf(d, v.y, aW1[m].y),
                                         fmaf(d, v.z, aW1[m].z), fmaf(d, v.w, aW1[m].w));
                }
            }
        }
        if (tid < kHeadH) {
            float a = 0.f;
            for (int r = 0; r < kHeadChunk; ++r) a += sH[r * (kHeadH + 1) + tid];
            aB1 += a;
        }
        if (x_on && xr < nv) {  // dx[xr][kx..kx+15] = sum_j dh[xr][j] W1[j][kx..]
            float4 a[4];
#pragma unroll
            for (int m = 0; m < 4; ++m) a[m] = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int j = 0; j < kHeadH; ++j) {
                const float d = sH[xr * (kHeadH + 1) + j];
                const float4 *wp = reinterpret_cast<const float4 *>(sW1 + j * kHeadLK + kx);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float4 v = wp[m];
                    a[m] = make_float4(fmaf(d, v.x, a[m].x), fmaf(d, v.y, a[m].y),
                                       fmaf(d, v.z, a[m].z), fmaf(d, v.w, a[m].w));
                }
            }
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const float v[4] = {a[m].x, a[m].y, a[m].z, a[m].w};
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    const int k = kx + 4 * m + t;
                    if (k < K) dx[(c0 + xr) * K + k] = v[t];
                }
            }
        }
    }
    if (w_on) {
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const float v[4] = {aW1[m].x, aW1[m].y, aW1[m].z, aW1[m].w};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int k = kb + 4 * m + t;
                if (k < K) dw1[jw * K + k] = v[t];
            }
        }
    }
    if (tid < kHeadH) {
        db1[tid] = aB1;
#pragma unroll
        for (int c = 0; c < kHeadCMax; ++c)
            if (c < C) dw2[c * kHeadH + tid] = aW2[c];
    }
    if (tid < C) db2[tid] = aB2;
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

extern "C" int scgib_head_fwd(const float *x, int64_t n_rows, int32_t k_in, const float *w1,
                              const float *b1, const float *w2, const float *b2, int32_t n_out,
                              int32_t sigmoid, float *hid, float *out, scgib_stream_t stream) {
    if (n_rows < 0 || k_in < 1 || k_in > kHeadKMax || n_out < 1 || n_out > kHeadCMax)
        return SCGIB_EINVAL;
    if (n_rows == 0) return SCGIB_OK;
    if (!x || !w1 || !b1 || !w2 || !b2 || !hid || !out) return SCGIB_EINVAL;
    const unsigned grid = static_cast<unsigned>((n_rows + kHeadRows - 1) / kHeadRows);
    head_fwd_k<<<grid, 256, 0, as_stream(stream)>>>(x, n_rows, k_in, w1, b1, w2, b2, n_out,
                                                    sigmoid ? 1 : 0, hid, out);
    return launch_status();
}

extern "C" int scgib_head_bwd(const float *x, const float *hid, const float *out,
                              const float *d_out, int64_t n_rows, int32_t k_in, const float *w1,
                              const float *w2, int32_t n_out, int32_t sigmoid, float *dx,
                              float *dw1, float *db1, float *dw2, float *db2,
                              scgib_stream_t stream) {
    if (n_rows < 1 || k_in < 1 || k_in > kHeadKMax || n_out < 1 || n_out > kHeadCMax)
        return SCGIB_EINVAL;
    if (!x || !hid || !out || !d_out || !w1 || !w2 || !dx || !dw1 || !db1 || !dw2 || !db2)
        return SCGIB_EINVAL;
    head_bwd_k<<<1, 256, 0, as_stream(stream)>>>(x, hid, out, d_out, n_rows, k_in, w1, w2, n_out,
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
