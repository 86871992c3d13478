// Fused GIN layer (gfx950): forward and backward of
//   h_out = ReLU(BN(W2 ReLU(W1 ((1+eps) h_v + sum_{u->v} h_u) + b1) + b2))
// for one GINConv(MLP) + BatchNorm1d + ReLU block of the reference encoder
// (models.py:52-72 with DGL GINConv semantics).
//
// Why fused: per layer the torch path issued ~25 launches (gather, 2 Linear,
// 2 ReLU, BN stats/apply, and their backward, incl. tall-skinny
// [N,64]^T x [N,64] weight-gradient GEMMs for which the BLAS heuristics pick
// 2-workgroup kernels).  Here a layer is 2 launches forward and 4 backward,
// every intermediate of a 64-row tile stays in LDS, and the four GEMMs of a
// tile run on the exact-f32 MFMA v_mfma_f32_32x32x2_f32 (same result as a
// k-ordered fmaf chain, no precision loss vs the fp32 reference).
//
// Forward (training):
//   gin_fwd_k      : per 64-row tile: gather (+ the previous layer's BN+ReLU
//                    applied on load) -> agg; z1 = agg W1^T + b1; r = relu(z1);
//                    z2 = r W2^T + b2; per-tile (sum, centred M2) of z2.
//   bn_finalize_k  : Chan-combine the tile statistics in fp64 (fixed order),
//                    batch mean / biased var, running-stat update (momentum,
//                    unbiased var), scale = gamma * invstd, shift.
// Backward:
//   gin_bwd_stats_k: dy = dh * [scale z2 + shift > 0] with dh either given or
//                    gathered from the next layer's d(agg) over the transposed
//                    CSR; per-tile sum(dy), sum(dy * xhat).
//   bn_bwd_finalize_k: dbeta, dgamma (fp64, fixed order) and the dz2
//                    coefficients.
//   gin_bwd_k      : per tile: dz2 = scale (dy - dbeta/N - xhat dgamma/N);
//                    dW2 += dz2^T r; dr = dz2 W2; dz1 = dr [r > 0];
//                    dW1 += dz1^T agg; d(agg) = dz1 W1.  Workgroups loop over
//                    tiles and keep dW in MFMA accumulators; one slab each.
//   slab_reduce1/2 : fixed-order two-stage sum of the per-workgroup slabs.
//
// LDS tiles are row-major with a +1-float row pad (stride 65 / 33), which
// makes every MFMA operand read (32 lanes: 32 rows of one column, or 32
// columns of one row) bank-conflict free for ds_read_b32.
#include "common.h"

namespace scgib {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int TM = 64;   // rows per tile
constexpr int LDH = 65;  // LDS stride of 64-wide tiles

__device__ __forceinline__ f32x16 zero16() {
    f32x16 a;
#pragma unroll
    for (int i = 0; i < 16; ++i) a[i] = 0.f;
    return a;
}

// C(i, j) += sum_k A(i, k) B(k, j) over K, 32x32 tile, with
//   NT: A(i,k) = As[i*lda + k],   B(k,j) = Bs[j*ldb + k]
//   NN: A(i,k) = As[i*lda + k],   B(k,j) = Bs[k*ldb + j]
//   TN: A(i,k) = As[k*lda + i],   B(k,j) = Bs[k*ldb + j]   (sum over rows k)
// (lane l supplies i or j = l & 31 and k-offset l >> 5 of each K=2 step)
template <int K>
__device__ __forceinline__ f32x16 mma_nt(const float *As, int lda, const float *Bs, int ldb,
                                         f32x16 acc) {
    const int l = threadIdx.x & 63, i = l & 31, kk = l >> 5;
#pragma unroll 8
    for (int k = 0; k < K; k += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[i * lda + k + kk], Bs[i * ldb + k + kk], acc, 0, 0, 0);
    return acc;
}

template <int K>
__device__ __forceinline__ f32x16 mma_nn(const float *As, int lda, const float *Bs, int ldb,
                                         f32x16 acc) {
    const int l = threadIdx.x & 63, i = l & 31, kk = l >> 5;
#pragma unroll 8
    for (int k = 0; k < K; k += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[i * lda + k + kk], Bs[(k + kk) * ldb + i], acc, 0, 0, 0);
    return acc;
}

template <int K>
__device__ __forceinline__ f32x16 mma_tn(const float *As, int lda, const float *Bs, int ldb,
                                         f32x16 acc) {
    const int l = threadIdx.x & 63, i = l & 31, kk = l >> 5;
#pragma unroll 8
    for (int k = 0; k < K; k += 2)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(As[(k + kk) * lda + i], Bs[(k + kk) * ldb + i], acc, 0, 0, 0);
    return acc;
}

// row of accumulator register `reg` of the 32x32 output tile held by lane l
__device__ __forceinline__ int acc_row(int reg, int l) { return (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5); }

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 xform4(float4 z, float4 a, float4 b) {
    return make_float4(fmaxf(a.x * z.x + b.x, 0.f), fmaxf(a.y * z.y + b.y, 0.f),
                       fmaxf(a.z * z.z + b.z, 0.f), fmaxf(a.w * z.w + b.w, 0.f));
}

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
template <int DIN, bool XFORM>
__global__ __launch_bounds__(256) void gin_fwd_k(
    const float *__restrict__ h, const float *__restrict__ in_scale,
    const float *__restrict__ in_shift, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ col, int64_t ncap, float ope, const float *__restrict__ w1,
    const float *__restrict__ b1, const float *__restrict__ w2, const float *__restrict__ b2,
    float *__restrict__ agg_out, float *__restrict__ r_out, float *__restrict__ z2_out,
    float *__restrict__ part, const int32_t *__restrict__ dims) {
    constexpr int LDA = DIN + 1, LPR = DIN / 4, RPP = 256 / LPR;
    const int64_t n = eff_count(dims, 0, ncap);
    __shared__ float sA[TM * LDA];
    __shared__ float sW1[64 * LDA];
    __shared__ float sW2[64 * LDH];
    __shared__ float sR[TM * LDH];
    __shared__ float sRed[2][64];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int64_t tile = blockIdx.x;
    const int64_t row0 = tile * TM;
    const int nv = static_cast<int>(n - row0 < TM ? (n - row0 > 0 ? n - row0 : 0) : TM);  // valid rows
    if (dims) {  // capacity mode: zero this tile's padded rows [nv, rows in capacity)
        const int ncr = static_cast<int>(ncap - row0 < TM ? ncap - row0 : TM);
        for (int idx = nv * 64 + tid; idx < ncr * 64; idx += 256) {
            r_out[row0 * 64 + idx] = 0.f;
            z2_out[row0 * 64 + idx] = 0.f;
        }
        for (int idx = nv * DIN + tid; idx < ncr * DIN; idx += 256) agg_out[row0 * DIN + idx] = 0.f;
        if (nv == 0) {
            if (tid < 128) part[tile * 128 + tid] = 0.f;
            return;
        }
    }

    for (int idx = tid; idx < 64 * DIN; idx += 256) sW1[(idx / DIN) * LDA + idx % DIN] = w1[idx];
    for (int idx = tid; idx < 64 * 64; idx += 256) sW2[(idx >> 6) * LDH + (idx & 63)] = w2[idx];

    // gather: agg[v] = ope * x[v] + sum_{u->v} x[u], x = relu(scale*h + shift) if XFORM
    {
        const int c = tid % LPR;
        float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
        if (XFORM) {
            sc = ld4(in_scale + 4 * c);
            sh = ld4(in_shift + 4 * c);
        }
        const float4 *h4 = reinterpret_cast<const float4 *>(h);
        for (int rr = tid / LPR; rr < TM; rr += RPP) {
            const int64_t v = row0 + rr;
            float4 out = make_float4(0.f, 0.f, 0.f, 0.f);
            if (rr < nv) {
                const int32_t beg = rowptr[v], end = rowptr[v + 1];
                float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
                int32_t j = beg;
                for (; j + 2 <= end; j += 2) {
                    const int64_t u0 = col[j], u1 = col[j + 1];
                    float4 a0 = h4[u0 * LPR + c], a1 = h4[u1 * LPR + c];
                    if (XFORM) { a0 = xform4(a0, sc, sh); a1 = xform4(a1, sc, sh); }
                    acc = add4(add4(acc, a0), a1);
                }
                if (j < end) {
                    float4 a0 = h4[static_cast<int64_t>(col[j]) * LPR + c];
                    if (XFORM) a0 = xform4(a0, sc, sh);
                    acc = add4(acc, a0);
                }
                float4 self = h4[v * LPR + c];
                if (XFORM) self = xform4(self, sc, sh);
                out = make_float4(ope * self.x + acc.x, ope * self.y + acc.y, ope * self.z + acc.z,
                                  ope * self.w + acc.w);
                st4(agg_out + v * DIN + 4 * c, out);
            }
            float *d = sA + rr * LDA + 4 * c;
            d[0] = out.x; d[1] = out.y; d[2] = out.z; d[3] = out.w;
        }
    }
    __syncthreads();

    const int wr = w >> 1, wc = w & 1;
    const int ccol = wc * 32 + (l & 31);
    // z1 = agg W1^T + b1 ; r = relu(z1)
    {
        f32x16 acc = mma_nt<DIN>(sA + wr * 32 * LDA, LDA, sW1 + wc * 32 * LDA, LDA, zero16());
        const float bias = b1[ccol];
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = wr * 32 + acc_row(reg, l);
            const float v = fmaxf(acc[reg] + bias, 0.f);
            sR[row * LDH + ccol] = v;
            if (row < nv) r_out[(row0 + row) * 64 + ccol] = v;
        }
    }
    __syncthreads();
    // z2 = r W2^T + b2 ; tile statistics of z2 (valid rows only)
    f32x16 acc = mma_nt<64>(sR + wr * 32 * LDH, LDH, sW2 + wc * 32 * LDH, LDH, zero16());
    const float bias2 = b2[ccol];
    float s = 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = wr * 32 + acc_row(reg, l);
        acc[reg] += bias2;
        if (row < nv) {
            z2_out[(row0 + row) * 64 + ccol] = acc[reg];
            s += acc[reg];
        }
    }
    s += __shfl_xor(s, 32, kWave);
    if (l < 32) sRed[wr][ccol] = s;
    __syncthreads();
    const float csum = sRed[0][ccol] + sRed[1][ccol];
    const float cmean = csum / nv;
    float m2 = 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = wr * 32 + acc_row(reg, l);
        const float d = acc[reg] - cmean;
        if (row < nv) m2 += d * d;
    }
    m2 += __shfl_xor(m2, 32, kWave);
    __syncthreads();
    if (l < 32) sRed[wr][ccol] = m2;
    __syncthreads();
    if (wr == 0 && l < 32) {
        part[tile * 128 + ccol] = csum;
        part[tile * 128 + 64 + ccol] = sRed[0][ccol] + sRed[1][ccol];
    }
}

// Batch mean / biased variance from the per-tile (sum, centred M2): two
// parallel fixed-order passes (fp64), 16 partitions x 64 channels:
//   mean = sum_b S_b / N ;  M2 = sum_b [M2_b + n_b (S_b/n_b - mean)^2]
// (exact decomposition of the centred sum of squares).  Loads are issued four
// at a time so the partition loops are not latency chains.
__global__ __launch_bounds__(1024) void bn_finalize_k(
    const float *__restrict__ part, int64_t ncap, const float *__restrict__ gamma,
    const float *__restrict__ beta, float eps, float momentum, int training,
    float *__restrict__ rmean, float *__restrict__ rvar, int64_t *__restrict__ nbt,
    float *__restrict__ stat /* [4][64]: mean, invstd, scale, shift */,
    const int32_t *__restrict__ dims) {
    const int c = threadIdx.x & 63, p = threadIdx.x >> 6;
    const int64_t n = eff_count(dims, 0, ncap), ntiles = (n + TM - 1) / TM;
    __shared__ double sh[16][64];
    __shared__ double s_mean[64];
    double mean = 0.0, var = 0.0, M2 = 0.0;
    if (training) {
        double a = 0.0;
        int64_t t = p;
        for (; t + 48 < ntiles; t += 64) {
            const float v0 = part[t * 128 + c], v1 = part[(t + 16) * 128 + c];
            const float v2 = part[(t + 32) * 128 + c], v3 = part[(t + 48) * 128 + c];
            a += v0; a += v1; a += v2; a += v3;
        }
        for (; t < ntiles; t += 16) a += part[t * 128 + c];
        sh[p][c] = a;
        __syncthreads();
        if (p == 0) {
            double s = 0.0;
            for (int k = 0; k < 16; ++k) s += sh[k][c];
            s_mean[c] = s / static_cast<double>(n);
        }
        __syncthreads();
        mean = s_mean[c];
        double q = 0.0;
        for (t = p; t < ntiles; t += 16) {
            const double nb = static_cast<double>(n - t * TM < TM ? n - t * TM : TM);
            const double d = part[t * 128 + c] / nb - mean;
            q += part[t * 128 + 64 + c] + nb * d * d;
        }
        __syncthreads();
        sh[p][c] = q;
        __syncthreads();
        if (p == 0)
            for (int k = 0; k < 16; ++k) M2 += sh[k][c];
        var = M2 / static_cast<double>(n);
    }
    if (p == 0) {
        if (training) {
            if (rmean) {
                rmean[c] = static_cast<float>((1.0 - momentum) * rmean[c] + momentum * mean);
                rvar[c] = static_cast<float>((1.0 - momentum) * rvar[c] +
                                             momentum * (n > 1 ? M2 / static_cast<double>(n - 1) : M2));
                if (c == 0 && nbt) *nbt += 1;
            }
        } else {
            mean = rmean[c];
            var = rvar[c];
        }
        const double istd = 1.0 / sqrt(var + static_cast<double>(eps));
        const double sc = gamma[c] * istd;
        stat[c] = static_cast<float>(mean);
        stat[64 + c] = static_cast<float>(istd);
        stat[128 + c] = static_cast<float>(sc);
        stat[192 + c] = static_cast<float>(beta[c] - mean * sc);
    }
}

__global__ __launch_bounds__(256) void bn_relu_apply_k(const float4 *__restrict__ z,
                                                       const float *__restrict__ stat,
                                                       int64_t n4, float4 *__restrict__ out,
                                                       const int32_t *__restrict__ dims) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i >= n4) return;
    if (dims && i >= static_cast<int64_t>(dims[0]) * 16) {
        out[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    const int c = static_cast<int>(i & 15) * 4;
    out[i] = xform4(z[i], ld4(stat + 128 + c), ld4(stat + 192 + c));
}

// ---------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------
// dy = dh * [scale z2 + shift > 0]; tile sums of dy and dy * xhat.
// GATHER: dh[v] = ope g[v] + sum_{u in out(v)} g[u]   (transposed aggregation
// of the next layer's d(agg), never materialised)
template <bool GATHER>
__global__ __launch_bounds__(256) void gin_bwd_stats_k(
    const float *__restrict__ dh, const int32_t *__restrict__ rowptr_t,
    const int32_t *__restrict__ col_t, float ope, const float *__restrict__ z2,
    const float *__restrict__ stat, int64_t ncap, float *__restrict__ dy_out,
    float *__restrict__ part, const int32_t *__restrict__ dims) {
    __shared__ float sRed[2][16][64];
    const int64_t n = eff_count(dims, 0, ncap);
    const int tid = threadIdx.x, c = tid & 15, slot = tid >> 4;
    const int64_t tile = blockIdx.x, row0 = tile * TM;
    const float4 mean = ld4(stat + 4 * c), istd = ld4(stat + 64 + 4 * c);
    const float4 sc = ld4(stat + 128 + 4 * c), sh = ld4(stat + 192 + 4 * c);
    const float4 *g4 = reinterpret_cast<const float4 *>(dh);
    float4 sdy = make_float4(0.f, 0.f, 0.f, 0.f), sdx = sdy;
    for (int rr = slot; rr < TM; rr += 16) {
        const int64_t v = row0 + rr;
        if (v >= ncap) break;
        if (v >= n) {
            st4(dy_out + v * 64 + 4 * c, make_float4(0.f, 0.f, 0.f, 0.f));
            continue;
        }
        float4 g;
        if (GATHER) {
            float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
            const int32_t beg = rowptr_t[v], end = rowptr_t[v + 1];
            int32_t j = beg;
            for (; j + 2 <= end; j += 2) {
                const int64_t u0 = col_t[j], u1 = col_t[j + 1];
                acc = add4(add4(acc, g4[u0 * 16 + c]), g4[u1 * 16 + c]);
            }
            if (j < end) acc = add4(acc, g4[static_cast<int64_t>(col_t[j]) * 16 + c]);
            const float4 self = g4[v * 16 + c];
            g = make_float4(ope * self.x + acc.x, ope * self.y + acc.y, ope * self.z + acc.z,
                            ope * self.w + acc.w);
        } else {
            g = g4[v * 16 + c];
        }
        const float4 z = ld4(z2 + v * 64 + 4 * c);
        const float4 dy = make_float4(sc.x * z.x + sh.x > 0.f ? g.x : 0.f, sc.y * z.y + sh.y > 0.f ? g.y : 0.f,
                                      sc.z * z.z + sh.z > 0.f ? g.z : 0.f, sc.w * z.w + sh.w > 0.f ? g.w : 0.f);
        st4(dy_out + v * 64 + 4 * c, dy);
        sdy = add4(sdy, dy);
        sdx = add4(sdx, make_float4(dy.x * (z.x - mean.x) * istd.x, dy.y * (z.y - mean.y) * istd.y,
                                    dy.z * (z.z - mean.z) * istd.z, dy.w * (z.w - mean.w) * istd.w));
    }
    float *a = &sRed[0][slot][4 * c];
    a[0] = sdy.x; a[1] = sdy.y; a[2] = sdy.z; a[3] = sdy.w;
    float *b = &sRed[1][slot][4 * c];
    b[0] = sdx.x; b[1] = sdx.y; b[2] = sdx.z; b[3] = sdx.w;
    __syncthreads();
    if (tid < 128) {
        const int which = tid >> 6, ch = tid & 63;
        float s = 0.f;
        for (int k = 0; k < 16; ++k) s += sRed[which][k][ch];
        part[tile * 128 + which * 64 + ch] = s;
    }
}

// dbeta = sum dy, dgamma = sum dy xhat (fp64, fixed order); coefficients of
// dz2 = scale (dy - c1 - xhat c2): training c1 = dbeta/N, c2 = dgamma/N.
__global__ __launch_bounds__(1024) void bn_bwd_finalize_k(const float *__restrict__ part,
                                                          int64_t ncap, int training,
                                                          float *__restrict__ dgamma,
                                                          float *__restrict__ dbeta,
                                                          float *__restrict__ coef,
                                                          const int32_t *__restrict__ dims) {
    const int c = threadIdx.x & 63, p = threadIdx.x >> 6;
    const int64_t n = eff_count(dims, 0, ncap), ntiles = (n + TM - 1) / TM;
    __shared__ double s1[16][64], s2[16][64];
    double a = 0.0, b = 0.0;
    int64_t t = p;
    for (; t + 16 < ntiles; t += 32) {
        const float a0 = part[t * 128 + c], a1 = part[(t + 16) * 128 + c];
        const float b0 = part[t * 128 + 64 + c], b1 = part[(t + 16) * 128 + 64 + c];
        a += a0; a += a1; b += b0; b += b1;
    }
    for (; t < ntiles; t += 16) {
        a += part[t * 128 + c];
        b += part[t * 128 + 64 + c];
    }
    s1[p][c] = a;
    s2[p][c] = b;
    __syncthreads();
    if (p == 0) {
        double db = 0.0, dg = 0.0;
        for (int k = 0; k < 16; ++k) {
            db += s1[k][c];
            dg += s2[k][c];
        }
        dbeta[c] = static_cast<float>(db);
        dgamma[c] = static_cast<float>(dg);
        coef[c] = training ? static_cast<float>(db / n) : 0.f;
        coef[64 + c] = training ? static_cast<float>(dg / n) : 0.f;
    }
}

// slab layout per workgroup: dW2[64*64] | dW1[64*DIN] | db2[64] | db1[64]
template <int DIN>
__global__ __launch_bounds__(256) void gin_bwd_k(
    const float *__restrict__ dy, const float *__restrict__ z2, const float *__restrict__ r,
    const float *__restrict__ agg, const float *__restrict__ stat,
    const float *__restrict__ coef, const float *__restrict__ w1, const float *__restrict__ w2,
    int64_t ncap, int64_t ntiles, float *__restrict__ dagg_out, float *__restrict__ slab,
    const int32_t *__restrict__ dims) {
    const int64_t n = eff_count(dims, 0, ncap);
    constexpr int LDA = DIN + 1;
    constexpr int SLAB = 64 * 64 + 64 * DIN + 128;
    __shared__ float sD[TM * LDH];   // dz2, then dz1
    __shared__ float sR[TM * LDH];
    __shared__ float sA[TM * LDA];
    __shared__ float sW1[64 * LDA];
    __shared__ float sW2[64 * LDH];
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;
    for (int idx = tid; idx < 64 * DIN; idx += 256) sW1[(idx / DIN) * LDA + idx % DIN] = w1[idx];
    for (int idx = tid; idx < 64 * 64; idx += 256) sW2[(idx >> 6) * LDH + (idx & 63)] = w2[idx];
    const int ch = tid & 63, q = tid >> 6;  // column-sum roles: channel, row quarter
    const float s_mean = stat[ch], s_istd = stat[64 + ch], s_sc = stat[128 + ch];
    const float c1 = coef[ch], c2 = coef[64 + ch];
    f32x16 accW2 = zero16(), accW1 = zero16();
    float db2 = 0.f, db1 = 0.f;
    constexpr int NSUB1 = 2 * (DIN / 32);  // 32x32 sub-tiles of dW1 / d(agg)
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t row0 = tile * TM;
        const int nv = static_cast<int>(n - row0 < TM ? (n - row0 > 0 ? n - row0 : 0) : TM);
        if (dims) {  // capacity mode: zero this tile's padded rows of d(agg)
            const int ncr = static_cast<int>(ncap - row0 < TM ? ncap - row0 : TM);
            for (int idx = nv * DIN + tid; idx < ncr * DIN; idx += 256) dagg_out[row0 * DIN + idx] = 0.f;
            if (nv == 0) continue;  // block-uniform
        }
        __syncthreads();  // previous tile's LDS reads are done
        // stage dz2 (computed), r and agg tiles; rows past n are zero
        for (int rr = q; rr < TM; rr += 4) {
            float d = 0.f, rv = 0.f;
            if (rr < nv) {
                const int64_t v = row0 + rr;
                const float z = z2[v * 64 + ch];
                const float xh = (z - s_mean) * s_istd;
                d = s_sc * (dy[v * 64 + ch] - c1 - xh * c2);
                rv = r[v * 64 + ch];
            }
            sD[rr * LDH + ch] = d;
            sR[rr * LDH + ch] = rv;
        }
        for (int idx = tid; idx < TM * DIN; idx += 256) {
            const int rr = idx / DIN, k = idx % DIN;
            sA[rr * LDA + k] = rr < nv ? agg[(row0 + rr) * DIN + k] : 0.f;
        }
        __syncthreads();
        // dW2 += dz2^T r  (sub-tile j-block wr, k-block wc)
        accW2 = mma_tn<TM>(sD + wr * 32, LDH, sR + wc * 32, LDH, accW2);
        // dr = dz2 W2  (rows wr, cols wc)
        f32x16 dr = mma_nn<64>(sD + wr * 32 * LDH, LDH, sW2 + wc * 32, LDH, zero16());
        for (int rr = q; rr < TM; rr += 4) db2 += sD[rr * LDH + ch];
        __syncthreads();  // all reads of dz2 done
        // dz1 = dr * [r > 0]  -> sD
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = wr * 32 + acc_row(reg, l), cc = wc * 32 + (l & 31);
            sD[row * LDH + cc] = sR[row * LDH + cc] > 0.f ? dr[reg] : 0.f;
        }
        __syncthreads();
        for (int rr = q; rr < TM; rr += 4) db1 += sD[rr * LDH + ch];
        // dW1 += dz1^T agg  (64 x DIN)
        if (w < NSUB1) {
            const int jb = w & 1, kb = w >> 1;  // j-block, k-block
            accW1 = mma_tn<TM>(sD + jb * 32, LDH, sA + kb * 32, LDA, accW1);
        }
        // d(agg) = dz1 W1  (TM x DIN)
        if (w < NSUB1) {
            const int rb = w & 1, kb = w >> 1;
            f32x16 da = mma_nn<64>(sD + rb * 32 * LDH, LDH, sW1 + kb * 32, LDA, zero16());
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = rb * 32 + acc_row(reg, l);
                if (row < nv) dagg_out[(row0 + row) * DIN + kb * 32 + (l & 31)] = da[reg];
            }
        }
    }
    // per-workgroup slab
    float *sl = slab + static_cast<int64_t>(blockIdx.x) * SLAB;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int j = wr * 32 + acc_row(reg, l), k = wc * 32 + (l & 31);
        sl[j * 64 + k] = accW2[reg];
    }
    if (w < NSUB1) {
        const int jb = w & 1, kb = w >> 1;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int j = jb * 32 + acc_row(reg, l), k = kb * 32 + (l & 31);
            sl[64 * 64 + j * DIN + k] = accW1[reg];
        }
    }
    __shared__ float sB[2][4][64];
    sB[0][q][ch] = db2;
    sB[1][q][ch] = db1;
    __syncthreads();
    if (tid < 128) {
        const int which = tid >> 6;
        sl[64 * 64 + 64 * DIN + which * 64 + ch] =
            ((sB[which][0][ch] + sB[which][1][ch]) + sB[which][2][ch]) + sB[which][3][ch];
    }
}

// Fixed-order sum of the per-workgroup weight-gradient slabs in two stages:
// stage 1 = (column block, group of kSlabGroup slabs) -> partial; stage 2 sums
// the partials in group order.  Enough workgroups to spread over the chip and
// at most 16 dependent adds per thread.
constexpr int kSlabGroup = 16;

__global__ __launch_bounds__(256) void slab_reduce1_k(const float *__restrict__ slab, int nslab,
                                                      int64_t width, float *__restrict__ partial) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (e >= width) return;
    const int b0 = blockIdx.y * kSlabGroup;
    const int b1 = b0 + kSlabGroup < nslab ? b0 + kSlabGroup : nslab;
    float v[kSlabGroup];
#pragma unroll
    for (int j = 0; j < kSlabGroup; ++j) v[j] = (b0 + j < b1) ? slab[(int64_t)(b0 + j) * width + e] : 0.f;
    float acc = 0.f;
#pragma unroll
    for (int j = 0; j < kSlabGroup; ++j) acc += v[j];
    partial[(int64_t)blockIdx.y * width + e] = acc;
}

__global__ __launch_bounds__(256) void slab_reduce2_k(const float *__restrict__ partial,
                                                      int ngroups, int64_t width,
                                                      float *__restrict__ out) {
    const int64_t e = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (e >= width) return;
    double acc = 0.0;
    for (int g = 0; g < ngroups; ++g) acc += partial[(int64_t)g * width + e];
    out[e] = static_cast<float>(acc);
}

static int bwd_grid(int64_t ntiles) { return static_cast<int>(ntiles < 256 ? ntiles : 256); }

}  // namespace scgib

using namespace scgib;

extern "C" int64_t scgib_gin_tiles(int64_t n_nodes) { return (n_nodes + TM - 1) / TM; }

extern "C" int64_t scgib_gin_slab_floats(int64_t n_nodes, int32_t d_in) {
    const int64_t g = bwd_grid(scgib_gin_tiles(n_nodes));
    const int64_t groups = (g + kSlabGroup - 1) / kSlabGroup;
    return (g + groups) * (64 * 64 + 64 * d_in + 128);  // slabs + stage-1 partials
}

extern "C" int scgib_gin_layer_fwd(const float *h_in, int32_t d_in, const float *in_stat,
                                   const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                                   float one_plus_eps, const float *w1, const float *b1,
                                   const float *w2, const float *b2, float *agg, float *r,
                                   float *z2, float *tile_stats, const int32_t *dims,
                                   scgib_stream_t stream) {
    if (n_nodes < 0 || (d_in != 32 && d_in != 64)) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!h_in || !rowptr || !col || !w1 || !b1 || !w2 || !b2 || !agg || !r || !z2 || !tile_stats)
        return SCGIB_EINVAL;
    if (in_stat && d_in != 64) return SCGIB_EUNSUPPORTED;
    const int64_t nt = scgib_gin_tiles(n_nodes);
    hipStream_t st = as_stream(stream);
    const float *isc = in_stat ? in_stat + 128 : nullptr, *ish = in_stat ? in_stat + 192 : nullptr;
    if (d_in == 32)
        gin_fwd_k<32, false><<<dim3((unsigned)nt), 256, 0, st>>>(h_in, isc, ish, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2, agg, r, z2, tile_stats, dims);
    else if (in_stat)
        gin_fwd_k<64, true><<<dim3((unsigned)nt), 256, 0, st>>>(h_in, isc, ish, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2, agg, r, z2, tile_stats, dims);
    else
        gin_fwd_k<64, false><<<dim3((unsigned)nt), 256, 0, st>>>(h_in, isc, ish, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2, agg, r, z2, tile_stats, dims);
    return launch_status();
}

extern "C" int scgib_bn_finalize(const float *tile_stats, int64_t n_nodes, const float *gamma,
                                 const float *beta, float eps, float momentum, int32_t training,
                                 float *running_mean, float *running_var,
                                 int64_t *num_batches_tracked, float *stat, const int32_t *dims,
                                 scgib_stream_t stream) {
    if (n_nodes < 0 || !gamma || !beta || !stat) return SCGIB_EINVAL;
    if (training && (n_nodes == 0 || !tile_stats)) return SCGIB_EINVAL;
    if (!training && (!running_mean || !running_var)) return SCGIB_EINVAL;
    bn_finalize_k<<<1, 1024, 0, as_stream(stream)>>>(tile_stats, n_nodes, gamma, beta, eps,
                                                     momentum, training, running_mean,
                                                     running_var, num_batches_tracked, stat, dims);
    return launch_status();
}

extern "C" int scgib_bn_relu_apply(const float *z, const float *stat, int64_t n_nodes,
                                   float *out, const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes < 0) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!z || !stat || !out) return SCGIB_EINVAL;
    const int64_t n4 = n_nodes * 16;
    bn_relu_apply_k<<<dim3((unsigned)((n4 + 255) / 256)), 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4 *>(z), stat, n4, reinterpret_cast<float4 *>(out), dims);
    return launch_status();
}

extern "C" int scgib_gin_bwd_stats(const float *dh, const int32_t *rowptr_t,
                                   const int32_t *col_t, float one_plus_eps, const float *z2,
                                   const float *stat, int64_t n_nodes, float *dy,
                                   float *tile_stats, const int32_t *dims,
                                   scgib_stream_t stream) {
    if (n_nodes < 0) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!dh || !z2 || !stat || !dy || !tile_stats) return SCGIB_EINVAL;
    if ((rowptr_t == nullptr) != (col_t == nullptr)) return SCGIB_EINVAL;
    const int64_t nt = scgib_gin_tiles(n_nodes);
    hipStream_t st = as_stream(stream);
    if (rowptr_t)
        gin_bwd_stats_k<true><<<dim3((unsigned)nt), 256, 0, st>>>(dh, rowptr_t, col_t, one_plus_eps, z2, stat, n_nodes, dy, tile_stats, dims);
    else
        gin_bwd_stats_k<false><<<dim3((unsigned)nt), 256, 0, st>>>(dh, rowptr_t, col_t, one_plus_eps, z2, stat, n_nodes, dy, tile_stats, dims);
    return launch_status();
}

extern "C" int scgib_bn_bwd_finalize(const float *tile_stats, int64_t n_nodes, int32_t training,
                                     float *dgamma, float *dbeta, float *coef,
                                     const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes <= 0 || !tile_stats || !dgamma || !dbeta || !coef) return SCGIB_EINVAL;
    bn_bwd_finalize_k<<<1, 1024, 0, as_stream(stream)>>>(tile_stats, n_nodes, training, dgamma,
                                                         dbeta, coef, dims);
    return launch_status();
}

extern "C" int scgib_gin_layer_bwd(const float *dy, const float *z2, const float *r,
                                   const float *agg, int32_t d_in, const float *stat,
                                   const float *coef, const float *w1, const float *w2,
                                   int64_t n_nodes, float *dagg, float *slab, float *wgrad,
                                   const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes <= 0 || (d_in != 32 && d_in != 64)) return SCGIB_EINVAL;
    if (!dy || !z2 || !r || !agg || !stat || !coef || !w1 || !w2 || !dagg || !slab || !wgrad)
        return SCGIB_EINVAL;
    const int64_t nt = scgib_gin_tiles(n_nodes);
    const int grid = bwd_grid(nt);
    hipStream_t st = as_stream(stream);
    if (d_in == 32)
        gin_bwd_k<32><<<grid, 256, 0, st>>>(dy, z2, r, agg, stat, coef, w1, w2, n_nodes, nt, dagg, slab, dims);
    else
        gin_bwd_k<64><<<grid, 256, 0, st>>>(dy, z2, r, agg, stat, coef, w1, w2, n_nodes, nt, dagg, slab, dims);
    const int64_t width = 64 * 64 + 64 * d_in + 128;
    const int groups = (grid + kSlabGroup - 1) / kSlabGroup;
    float *partial = slab + static_cast<int64_t>(grid) * width;
    const unsigned cb = static_cast<unsigned>((width + 255) / 256);
    slab_reduce1_k<<<dim3(cb, groups), 256, 0, st>>>(slab, grid, width, partial);
    slab_reduce2_k<<<dim3(cb), 256, 0, st>>>(partial, groups, width, wgrad);
    return launch_status();
}
