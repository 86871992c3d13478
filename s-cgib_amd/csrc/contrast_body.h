// Contrastive loss of the pretraining step (gfx950), device bodies:
//   batched_semi_loss(z1, z2, chunk), tau = 1   (models.py:606-629)
//
//   z1n = z1 / max(|z1|, 1e-12), z2n likewise      (F.normalize)
//   R_i = sum_j exp(z1n_i . z1n_j),  Bt_i = sum_j exp(z1n_i . z2n_j)
//   D_i = R_i + Bt_i - exp(z1n_i . z1n_i)
//   loss = mean_i -log(exp(z1n_i . z2n_i) / D_i)
//
// The per-row value does not depend on the reference's chunking, so the
// B x B similarity blocks are formed on the fly and never stored.
//
// Grid: (row blocks of 16) x (NS column splits); a workgroup takes its rows
// against the 64-row column tiles of its split.  The 16 query rows are held in
// registers (one row per 16 lanes), the column tile is normalised into LDS
// (stride 68: 16-byte reads of 16 different rows hit disjoint banks).
//   forward : per (row, split) partial (R, Bt, e11_ii, e12_ii); the last
//             workgroup to arrive combines the splits in fixed order, writes
//             D_i and the mean (fp64) -> deterministic.
//   backward: g = dL/dloss / B,
//     dz1n_i = sum_{j != i} g e11_ij (1/D_i + 1/D_j) z1n_j + sum_j g (e12_ij/D_i - [i=j]) z2n_j
//     dz2n_i = sum_j g (exp(z1n_j . z2n_i)/D_j - [i=j]) z1n_j
//   per-split partials; the last split to arrive for a row block sums them in
//   fixed order and applies the normalisation backward
//     dz = (dzn - zn (zn . dzn)) / |z|   (|z| > eps; z / eps otherwise).
// The split partials cross workgroups through agent-scope stores/loads and
// block_arrive (common.h): no L2 write-back fence.
//
// Arrival counters: caller-provided, zero on entry, left zero on exit (the
// last arriver resets them), so the launches replay from a HIP graph.
#pragma once
#include "common.h"

namespace scgib {

constexpr int CR = 16;   // rows per workgroup
constexpr int CT = 64;   // column tile
constexpr int CLD = 68;  // LDS row stride (16-byte aligned rows)
constexpr int kMaxSplit = 16;
constexpr float kNormEps = 1e-12f;

__host__ __device__ inline int contrast_splits(int64_t B) {
    const int64_t t = (B + CT - 1) / CT;
    return static_cast<int>(t < kMaxSplit ? t : kMaxSplit);
}

// Stage rows [j0, j0 + 64) of x, normalised, into s (64 x CLD); rows >= B are
// zero.  256 threads: row tid >> 2, 16 channels per thread.
__device__ __forceinline__ void stage_tile(const float *__restrict__ x, int64_t B, int64_t j0,
                                           float *s) {
    const int tid = threadIdx.x, r = tid >> 2, q = tid & 3;
    const int64_t j = j0 + r;
    float4 v[4];
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        v[k] = ld_ok(reinterpret_cast<const float4 *>(x), j * 16 + 4 * q + k, 4 * q + k, j < B,
                     make_float4(0.f, 0.f, 0.f, 0.f));
        ss += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
    }
    ss += __shfl_xor(ss, 1, kWave);
    ss += __shfl_xor(ss, 2, kWave);
    const float inv = 1.f / fmaxf(sqrtf(ss), kNormEps);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        *reinterpret_cast<float4 *>(s + r * CLD + 16 * q + 4 * k) =
            make_float4(v[k].x * inv, v[k].y * inv, v[k].z * inv, v[k].w * inv);
}

// a whole normalised row in registers; returns 1 / max(|x|, eps)
__device__ __forceinline__ float load_row(const float *__restrict__ x, int64_t i, int64_t B,
                                          float4 (&q)[16]) {
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        q[k] = ld_ok(reinterpret_cast<const float4 *>(x), i * 16 + k, k, i < B, make_float4(0.f, 0.f, 0.f, 0.f));
        ss += q[k].x * q[k].x + q[k].y * q[k].y + q[k].z * q[k].z + q[k].w * q[k].w;
    }
    const float inv = 1.f / fmaxf(sqrtf(ss), kNormEps);
#pragma unroll
    for (int k = 0; k < 16; ++k) q[k] = make_float4(q[k].x * inv, q[k].y * inv, q[k].z * inv, q[k].w * inv);
    return inv;
}

__device__ __forceinline__ float dot_row(const float4 (&q)[16], const float *s) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const float4 b = *reinterpret_cast<const float4 *>(s + 4 * k);
        acc += q[k].x * b.x;
        acc += q[k].y * b.y;
        acc += q[k].z * b.z;
        acc += q[k].w * b.w;
    }
    return acc;
}

// sum over the 16 lanes of a row group (lanes 16m .. 16m+15 of the wave)
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// workspace (floats): D[B] | fwd partials [S][B][4] | bwd partials [S][B][128],
// S = contrast_splits(B); a launch may use NS <= S splits.
// The bodies take their workgroup's (row block bx, split by) and LDS buffers
// from the caller, so a kernel of another op can run them in extra
// workgroups (the head MLP: gin_layer.hip, ContrastArgs).
struct ContrastArgs {
    const float *z1, *z2;
    int64_t B;               // 0: no contrastive workgroups
    float *ws;
    float *loss;             // fwd
    const float *g_loss;     // bwd
    float *dz1, *dz2;        // bwd
    unsigned *counters;      // fwd: [1]; bwd: [row blocks]
    int nsplit;              // splits of this launch
    int nmain;               // workgroups of the host kernel before the contrastive ones
};

__host__ __device__ inline int64_t contrast_row_blocks(int64_t B) { return (B + CR - 1) / CR; }

// forward body: sK1, sK2 >= CT * CLD floats each
__device__ __forceinline__ void contrast_fwd_body(const ContrastArgs &a, int64_t bx, int by,
                                                  float *sK1, float *sK2) {
    const float *__restrict__ z1 = a.z1, *__restrict__ z2 = a.z2;
    const int64_t B = a.B;
    float *__restrict__ ws = a.ws;
    const int tid = threadIdx.x, r = tid >> 4, cl = tid & 15;
    const int NS = a.nsplit;
    const int64_t i = bx * CR + r;
    float4 q[16];
    load_row(z1, i, B, q);
    float R = 0.f, Bt = 0.f, e12d = 0.f, e11d = 0.f;
    for (int64_t j0 = static_cast<int64_t>(by) * CT; j0 < B; j0 += static_cast<int64_t>(NS) * CT) {
        __syncthreads();
        stage_tile(z1, B, j0, sK1);
        stage_tile(z2, B, j0, sK2);
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < CT / 16; ++cc) {
            const int jj = cl + 16 * cc;
            const int64_t j = j0 + jj;
            if (j < B) {
                const float e11 = expf(dot_row(q, sK1 + jj * CLD));
                const float e12 = expf(dot_row(q, sK2 + jj * CLD));
                R += e11;
                Bt += e12;
                if (j == i) { e11d = e11; e12d = e12; }
            }
        }
    }
    R = sum16(R);
    Bt = sum16(Bt);
    e11d = sum16(e11d);
    e12d = sum16(e12d);
    float *Dv = ws, *pf = ws + B;
    if (cl == 0 && i < B) st_agent4(pf + (by * B + i) * 4, make_float4(R, Bt, e11d, e12d));
    // two-level combine: the last split of each row block finishes its 16
    // rows (D, the -log terms, their fixed-order sum), then the last row
    // block sums the row-block partials in order.  Counters: a.counters[0]
    // (row blocks) and a.counters[1 + bx] (splits; the backward's counters,
    // idle during the forward), each reset by its last arriver.
    unsigned *counter = a.counters;
    const int64_t nrb = contrast_row_blocks(B);
    int64_t off = B + static_cast<int64_t>(contrast_splits(B)) * B * 4;  // bwd partials, idle here
    off += off & 1;
    double *rbp = reinterpret_cast<double *>(ws + off);
    if (!block_arrive(counter + 1 + bx, static_cast<unsigned>(NS))) return;
    __shared__ double sRow[CR];
    if (tid < CR) {
        const int64_t k = bx * CR + tid;
        const int64_t kc = k < B ? k : B - 1;  // clamped: the loads stay unconditional
        float4 v[kMaxSplit];
#pragma unroll
        for (int y = 0; y < kMaxSplit; ++y)
            v[y] = ld_agent4(pf + ((y < NS ? y : 0) * B + kc) * 4);
        float sm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int y = 0; y < kMaxSplit; ++y) {
            const float w = y < NS ? 1.f : 0.f;
            sm[0] = fmaf(v[y].x, w, sm[0]);
            sm[1] = fmaf(v[y].y, w, sm[1]);
            sm[2] = fmaf(v[y].z, w, sm[2]);
            sm[3] = fmaf(v[y].w, w, sm[3]);
        }
        const float D = sm[0] + sm[1] - sm[2];
        if (k < B) Dv[k] = D;
        sRow[tid] = k < B ? static_cast<double>(-logf(sm[3] / D)) : 0.0;
    }
    __syncthreads();
    if (tid == 0) {
        double t = 0.0;
#pragma unroll
        for (int r2 = 0; r2 < CR; ++r2) t += sRow[r2];
        st_agent(rbp + bx, t);
        counter[1 + bx] = 0u;
    }
    if (!block_arrive(counter, static_cast<unsigned>(nrb))) return;
    __shared__ double red[256];
    double t = 0.0;
    for (int64_t b2 = tid; b2 < nrb; b2 += 256) t += ld_agent(rbp + b2);
    red[tid] = t;
    __syncthreads();
    for (int o = 128; o >= 1; o >>= 1) {
        if (tid < o) red[tid] += red[tid + o];
        __syncthreads();
    }
    if (tid == 0) {
        *a.loss = static_cast<float>(red[0] / static_cast<double>(B));
        *counter = 0u;  // ready for the next launch / graph replay
    }
}

// backward body: sK1, sK2 >= CT * CLD floats, sWf >= 3 * CR * (CT + 1), sDj >= CT
constexpr int kContrastBwdW = 3 * CR * (CT + 1);
__device__ __forceinline__ void contrast_bwd_body(const ContrastArgs &a, int64_t bx, int by,
                                                  float *sK1, float *sK2, float *sWf,
                                                  float *sDj) {
    const float *__restrict__ z1 = a.z1, *__restrict__ z2 = a.z2;
    const int64_t B = a.B;
    const float *__restrict__ ws = a.ws;
    float *__restrict__ dz1 = a.dz1, *__restrict__ dz2 = a.dz2;
    unsigned *counters = a.counters;
    auto sW = reinterpret_cast<float (*)[CR][CT + 1]>(sWf);
    const int tid = threadIdx.x, r = tid >> 4, cl = tid & 15;
    const int NS = a.nsplit;
    const int64_t i = bx * CR + r;
    const float g = *a.g_loss / static_cast<float>(B);
    const float *Dv = ws;
    float *pb = a.ws + B + static_cast<int64_t>(contrast_splits(B)) * B * 4;
    float4 q1[16], q2[16];
    const float inv1 = load_row(z1, i, B, q1);
    const float inv2 = load_row(z2, i, B, q2);
    const float invDi = i < B ? 1.f / Dv[i] : 0.f;
    float4 d1 = make_float4(0.f, 0.f, 0.f, 0.f), d2 = d1;
    for (int64_t j0 = static_cast<int64_t>(by) * CT; j0 < B; j0 += static_cast<int64_t>(NS) * CT) {
        __syncthreads();
        stage_tile(z1, B, j0, sK1);
        stage_tile(z2, B, j0, sK2);
        if (tid < CT) sDj[tid] = j0 + tid < B ? Dv[j0 + tid] : 1.f;
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < CT / 16; ++cc) {
            const int jj = cl + 16 * cc;
            const int64_t j = j0 + jj;
            float w11 = 0.f, w12 = 0.f, w21 = 0.f;
            if (j < B && i < B) {
                const float invDj = 1.f / sDj[jj];
                const float e11 = expf(dot_row(q1, sK1 + jj * CLD));
                const float e12 = expf(dot_row(q1, sK2 + jj * CLD));
                const float e21 = expf(dot_row(q2, sK1 + jj * CLD));
                const float delta = j == i ? 1.f : 0.f;
                w11 = j == i ? 0.f : g * e11 * (invDi + invDj);
                w12 = g * (e12 * invDi - delta);
                w21 = g * (e21 * invDj - delta);
            }
            sW[0][r][jj] = w11;
            sW[1][r][jj] = w12;
            sW[2][r][jj] = w21;
        }
        __syncthreads();
#pragma unroll 4
        for (int jj = 0; jj < CT; ++jj) {
            const float w11 = sW[0][r][jj], w12 = sW[1][r][jj], w21 = sW[2][r][jj];
            const float4 k1 = *reinterpret_cast<const float4 *>(sK1 + jj * CLD + 4 * cl);
            const float4 k2 = *reinterpret_cast<const float4 *>(sK2 + jj * CLD + 4 * cl);
            d1.x += w11 * k1.x + w12 * k2.x; d1.y += w11 * k1.y + w12 * k2.y;
            d1.z += w11 * k1.z + w12 * k2.z; d1.w += w11 * k1.w + w12 * k2.w;
            d2.x += w21 * k1.x; d2.y += w21 * k1.y; d2.z += w21 * k1.z; d2.w += w21 * k1.w;
        }
    }
    if (i < B) {
        float *p = pb + (static_cast<int64_t>(by) * B + i) * 128;
        st_agent4(p + 4 * cl, d1);
        st_agent4(p + 64 + 4 * cl, d2);
    }
    if (!block_arrive(counters + bx, NS)) return;
    if (i < B) {
        d1 = d2 = make_float4(0.f, 0.f, 0.f, 0.f);
        float4 v1[kMaxSplit], v2[kMaxSplit];
#pragma unroll
        for (int y = 0; y < kMaxSplit; ++y) {  // all splits in flight (clamped), summed in order
            const float *p = pb + (static_cast<int64_t>(y < NS ? y : 0) * B + i) * 128 + 4 * cl;
            v1[y] = ld_agent4(p);
            v2[y] = ld_agent4(p + 64);
        }
#pragma unroll
        for (int y = 0; y < kMaxSplit; ++y) {
            const float w = y < NS ? 1.f : 0.f;
            d1.x = fmaf(v1[y].x, w, d1.x); d1.y = fmaf(v1[y].y, w, d1.y);
            d1.z = fmaf(v1[y].z, w, d1.z); d1.w = fmaf(v1[y].w, w, d1.w);
            d2.x = fmaf(v2[y].x, w, d2.x); d2.y = fmaf(v2[y].y, w, d2.y);
            d2.z = fmaf(v2[y].z, w, d2.z); d2.w = fmaf(v2[y].w, w, d2.w);
        }
        // this lane's channels of the normalised rows
        float4 a1 = q1[0], a2 = q2[0];
#pragma unroll
        for (int k = 1; k < 16; ++k)
            if (k == cl) { a1 = q1[k]; a2 = q2[k]; }
        const float p1 = sum16(a1.x * d1.x + a1.y * d1.y + a1.z * d1.z + a1.w * d1.w);
        const float p2 = sum16(a2.x * d2.x + a2.y * d2.y + a2.z * d2.z + a2.w * d2.w);
        const float s1 = inv1 < 1.f / kNormEps ? p1 : 0.f;  // |z| <= eps: z / eps, no projection
        const float s2 = inv2 < 1.f / kNormEps ? p2 : 0.f;
        reinterpret_cast<float4 *>(dz1 + i * 64)[cl] =
            make_float4((d1.x - a1.x * s1) * inv1, (d1.y - a1.y * s1) * inv1,
                        (d1.z - a1.z * s1) * inv1, (d1.w - a1.w * s1) * inv1);
        reinterpret_cast<float4 *>(dz2 + i * 64)[cl] =
            make_float4((d2.x - a2.x * s2) * inv2, (d2.y - a2.y * s2) * inv2,
                        (d2.z - a2.z * s2) * inv2, (d2.w - a2.w * s2) * inv2);
    }
    if (tid == 0) counters[bx] = 0u;
}

}  // namespace scgib
