// The fine-tune prediction head (gfx950): the reference's
//   predict = Sequential(Linear(2d, d), ReLU, Linear(d, C))   (models.py:386-396)
// applied to the Set2Set readout, then sigmoid for the classification
// datasets (models.py:515-520), forward and backward, each as ONE launch of
// one 256-thread workgroup (the head sees B graph rows: B = 32 in the
// molhiv driver).  It replaces ~14 torch launches per step (two GEMMs, the
// ReLU, the sigmoid and their backward: GEMMs, reductions, masks).
//
// Rows are processed in chunks of kHeadRows staged in LDS; every sum runs in
// a fixed order (weight gradients accumulate over the chunks in row order),
// so the results are deterministic.  Shapes: din <= 128, dh <= 64, C <= 64.
// Latency-bound VALU work on a few thousand rows at most: no MFMA.
#include "common.h"

namespace scgib {

namespace {

constexpr int kHeadRows = 64, kHeadIn = 128, kHeadHid = 64, kHeadOut = 64;

__device__ __forceinline__ float head_sigmoid(float v) { return 1.f / (1.f + expf(-v)); }

}  // namespace

__global__ __launch_bounds__(256) void predict_fwd_k(const float *__restrict__ x, int64_t B,
                                                     int din, const float *__restrict__ w1,
                                                     const float *__restrict__ b1, int dh,
                                                     const float *__restrict__ w2,
                                                     const float *__restrict__ b2, int C,
                                                     int sigmoid, float *__restrict__ hid,
                                                     float *__restrict__ out) {
    __shared__ float sX[kHeadRows * (kHeadIn + 1)], sH[kHeadRows * (kHeadHid + 1)];
    const int tid = threadIdx.x, LX = din + 1, LH = dh + 1;
    for (int64_t r0 = 0; r0 < B; r0 += kHeadRows) {
        const int nr = static_cast<int>(B - r0 < kHeadRows ? B - r0 : kHeadRows);
        for (int i = tid; i < nr * din; i += 256) sX[(i / din) * LX + i % din] = x[r0 * din + i];
        __syncthreads();
        // hidden = relu(x W1^T + b1): thread -> (row, unit), unit fastest
        for (int i = tid; i < nr * dh; i += 256) {
            const int r = i / dh, j = i - r * dh;
            const float *wr = w1 + static_cast<int64_t>(j) * din;
            const float *xr = sX + r * LX;
            float a0 = 0.f, a1 = 0.f;
#pragma unroll 16
            for (int k = 0; k + 1 < din; k += 2) {
                a0 = fmaf(wr[k], xr[k], a0);
                a1 = fmaf(wr[k + 1], xr[k + 1], a1);
            }
            if (din & 1) a0 = fmaf(wr[din - 1], xr[din - 1], a0);
            const float h = fmaxf((a0 + a1) + b1[j], 0.f);
            sH[r * LH + j] = h;
            hid[(r0 + r) * dh + j] = h;
        }
        __syncthreads();
        for (int i = tid; i < nr * C; i += 256) {
            const int r = i / C, c = i - r * C;
            const float *wr = w2 + static_cast<int64_t>(c) * dh;
            const float *hr = sH + r * LH;
            float a = 0.f;
#pragma unroll 16
            for (int j = 0; j < dh; ++j) a = fmaf(wr[j], hr[j], a);
            const float z = a + b2[c];
            out[(r0 + r) * C + c] = sigmoid ? head_sigmoid(z) : z;
        }
        __syncthreads();  // (the next chunk overwrites sX / sH)
    }
}

// d out -> dx [B][din], dW1 [dh][din], db1 [dh], dW2 [C][dh], db2 [C]
__global__ __launch_bounds__(256) void predict_bwd_k(
    const float *__restrict__ x, int64_t B, int din, const float *__restrict__ w1, int dh,
    const float *__restrict__ w2, int C, int sigmoid, const float *__restrict__ hid,
    const float *__restrict__ out, const float *__restrict__ g, float *__restrict__ dx,
    float *__restrict__ dw1, float *__restrict__ db1, float *__restrict__ dw2,
    float *__restrict__ db2) {
    __shared__ float sX[kHeadRows * (kHeadIn + 1)], sH[kHeadRows * (kHeadHid + 1)];
    __shared__ float sDH[kHeadRows * (kHeadHid + 1)], sDZ[kHeadRows * kHeadOut];
    const int tid = threadIdx.x, LX = din + 1, LH = dh + 1;
    // the weight gradients in one flat index space (dW1 | db1 | dW2 | db2),
    // entry e owned by thread e mod 256 and accumulated in LDS over the
    // chunks, rows in order
    __shared__ float sAcc[kHeadHid * kHeadIn + kHeadHid + kHeadOut * kHeadHid + kHeadOut];
    const int nW1 = dh * din, nB1 = dh, nW2 = C * dh, nB2 = C;
    const int nAll = nW1 + nB1 + nW2 + nB2;
    for (int e = tid; e < nAll; e += 256) sAcc[e] = 0.f;
    for (int64_t r0 = 0; r0 < B; r0 += kHeadRows) {
        const int nr = static_cast<int>(B - r0 < kHeadRows ? B - r0 : kHeadRows);
        for (int i = tid; i < nr * din; i += 256) sX[(i / din) * LX + i % din] = x[r0 * din + i];
        for (int i = tid; i < nr * dh; i += 256) sH[(i / dh) * LH + i % dh] = hid[r0 * dh + i];
        for (int i = tid; i < nr * C; i += 256) {  // d(pre-sigmoid)
            const float s = out[r0 * C + i], gi = g[r0 * C + i];
            sDZ[i] = sigmoid ? gi * s * (1.f - s) : gi;
        }
        __syncthreads();
        // d hidden = (dz W2) masked by the ReLU
        for (int i = tid; i < nr * dh; i += 256) {
            const int r = i / dh, j = i - r * dh;
            float a = 0.f;
#pragma unroll 4
            for (int c = 0; c < C; ++c)
                a = fmaf(sDZ[r * C + c], w2[static_cast<int64_t>(c) * dh + j], a);
            sDH[r * LH + j] = sH[r * LH + j] > 0.f ? a : 0.f;
        }
        __syncthreads();
        // dx = dH W1 (rows of the chunk; k fastest: W1 columns read coalesced)
        for (int i = tid; i < nr * din; i += 256) {
            const int r = i / din, k = i - r * din;
            float a = 0.f;
#pragma unroll 16
            for (int j = 0; j < dh; ++j)
                a = fmaf(sDH[r * LH + j], w1[static_cast<int64_t>(j) * din + k], a);
            dx[(r0 + r) * din + k] = a;
        }
        // weight gradients of this chunk's rows, in row order
        for (int e = tid; e < nAll; e += 256) {
            float a = sAcc[e];
            if (e < nW1) {
                const int j = e / din, k = e - j * din;
                for (int r = 0; r < nr; ++r) a = fmaf(sDH[r * LH + j], sX[r * LX + k], a);
            } else if (e < nW1 + nB1) {
                const int j = e - nW1;
                for (int r = 0; r < nr; ++r) a += sDH[r * LH + j];
            } else if (e < nW1 + nB1 + nW2) {
                const int f = e - nW1 - nB1, c = f / dh, j = f - c * dh;
                for (int r = 0; r < nr; ++r) a = fmaf(sDZ[r * C + c], sH[r * LH + j], a);
            } else {
                const int c = e - nW1 - nB1 - nW2;
                for (int r = 0; r < nr; ++r) a += sDZ[r * C + c];
            }
            sAcc[e] = a;
        }
        __syncthreads();  // (the next chunk overwrites the LDS images)
    }
    for (int e = tid; e < nAll; e += 256) {
        if (e < nW1)
            dw1[e] = sAcc[e];
        else if (e < nW1 + nB1)
            db1[e - nW1] = sAcc[e];
        else if (e < nW1 + nB1 + nW2)
            dw2[e - nW1 - nB1] = sAcc[e];
        else
            db2[e - nW1 - nB1 - nW2] = sAcc[e];
    }
}

}  // namespace scgib

using namespace scgib;

static bool head_shape_ok(int64_t B, int32_t din, int32_t dh, int32_t C) {
    return B >= 0 && din >= 1 && din <= kHeadIn && dh >= 1 && dh <= kHeadHid && C >= 1 &&
           C <= kHeadOut;
}

extern "C" int scgib_predict_fwd(const float *x, int64_t n_rows, int32_t d_in, const float *w1,
                                 const float *b1, int32_t d_hidden, const float *w2,
                                 const float *b2, int32_t n_out, int32_t sigmoid, float *hidden,
                                 float *out, scgib_stream_t stream) {
    if (!head_shape_ok(n_rows, d_in, d_hidden, n_out)) return SCGIB_EINVAL;
    if (n_rows == 0) return SCGIB_OK;
    if (!x || !w1 || !b1 || !w2 || !b2 || !hidden || !out) return SCGIB_EINVAL;
    predict_fwd_k<<<1, 256, 0, as_stream(stream)>>>(x, n_rows, d_in, w1, b1, d_hidden, w2, b2,
                                                    n_out, sigmoid, hidden, out);
    return launch_status();
}

extern "C" int scgib_predict_bwd(const float *x, int64_t n_rows, int32_t d_in, const float *w1,
                                 int32_t d_hidden, const float *w2, int32_t n_out,
                                 int32_t sigmoid, const float *hidden, const float *out,
                                 const float *g_out, float *dx, float *dw1, float *db1,
                                 float *dw2, float *db2, scgib_stream_t stream) {
    if (!head_shape_ok(n_rows, d_in, d_hidden, n_out)) return SCGIB_EINVAL;
    if (!x || !w1 || !w2 || !hidden || !out || !g_out || !dx || !dw1 || !db1 || !dw2 || !db2)
        return SCGIB_EINVAL;
    predict_bwd_k<<<1, 256, 0, as_stream(stream)>>>(x, n_rows, d_in, w1, d_hidden, w2, n_out,
                                                    sigmoid, hidden, out, g_out, dx, dw1, db1,
                                                    dw2, db2);
    return launch_status();
}
