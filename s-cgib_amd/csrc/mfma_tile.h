// Shared device helpers of the fp32 MFMA tile kernels (gin_layer.hip,
// dense.hip): 64-row tiles in padded LDS, exact-f32 v_mfma_f32_32x32x2_f32
// sub-tile products, latency-batched CSR gathers, weight staging.
#pragma once

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

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }

// The forward layer's saved activations (agg, r, z2: read next by the
// backward, or by the next layer's gather) as non-temporal stores (1.6 % off
// the 1.2 M-row superbatch layer, neutral at QM9 B512: profiles/r05_nt);
// SCGIB_NT_SAVED=0 (build-time A/B hook) for plain ones.
#ifndef SCGIB_NT_SAVED
#define SCGIB_NT_SAVED 1
#endif
typedef float scgib_f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_saved(float *p, float v) {
    if constexpr (SCGIB_NT_SAVED != 0) __builtin_nontemporal_store(v, p);
    else *p = v;
}
__device__ __forceinline__ void st4_saved(float *p, float4 v) {
    if constexpr (SCGIB_NT_SAVED != 0)
        __builtin_nontemporal_store(scgib_f4v{v.x, v.y, v.z, v.w}, reinterpret_cast<scgib_f4v *>(p));
    else
        *reinterpret_cast<float4 *>(p) = v;
}
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 xform4(float4 z, float4 a, float4 b) {
    return make_float4(fmaxf(a.x * z.x + b.x, 0.f), fmaxf(a.y * z.y + b.y, 0.f),
                       fmaxf(a.z * z.z + b.z, 0.f), fmaxf(a.w * z.w + b.w, 0.f));
}

// Stage a [64][COLS] row-major matrix into LDS (row stride COLS + 1).
template <int COLS>
__device__ __forceinline__ void stage_matrix(const float *__restrict__ w, float *s) {
    constexpr int LD = COLS + 1, N = 64 * COLS / 4 / 256;
    const int tid = threadIdx.x;
    float4 a[N];
#pragma unroll
    for (int k = 0; k < N; ++k) a[k] = reinterpret_cast<const float4 *>(w)[tid + 256 * k];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        const int idx = 4 * (tid + 256 * k), row = idx / COLS, cc = idx % COLS;
        float *d = s + row * LD + cc;
        d[0] = a[k].x; d[1] = a[k].y; d[2] = a[k].z; d[3] = a[k].w;
    }
}

// W1 [64][DIN] and W2 [64][64] (torch Linear layout) -> padded LDS tiles, in
// two halves so the global loads can be in flight while the caller issues its
// own loads (gathers, tile rows): load_weights issues 16-byte loads into
// registers, store_weights (later) writes them to LDS.  The hardware counts
// outstanding loads in order, so waiting for the weights does not wait for
// loads issued after them.
template <int DIN>
struct WeightRegs {
    float4 a[64 * DIN / 4 / 256], b[64 * 64 / 4 / 256];
};

template <int DIN>
__device__ __forceinline__ void load_weights(const float *__restrict__ w1,
                                             const float *__restrict__ w2, WeightRegs<DIN> &r) {
    constexpr int N1 = 64 * DIN / 4 / 256, N2 = 64 * 64 / 4 / 256;
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < N1; ++k) r.a[k] = reinterpret_cast<const float4 *>(w1)[tid + 256 * k];
#pragma unroll
    for (int k = 0; k < N2; ++k) r.b[k] = reinterpret_cast<const float4 *>(w2)[tid + 256 * k];
}

template <int DIN>
__device__ __forceinline__ void store_weights(const WeightRegs<DIN> &r, float *sW1, float *sW2) {
    constexpr int LDA = DIN + 1, N1 = 64 * DIN / 4 / 256, N2 = 64 * 64 / 4 / 256;
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < N1; ++k) {
        const int idx = 4 * (tid + 256 * k), row = idx / DIN, cc = idx % DIN;
        float *d = sW1 + row * LDA + cc;
        d[0] = r.a[k].x; d[1] = r.a[k].y; d[2] = r.a[k].z; d[3] = r.a[k].w;
    }
#pragma unroll
    for (int k = 0; k < N2; ++k) {
        const int idx = 4 * (tid + 256 * k), row = idx >> 6, cc = idx & 63;
        float *d = sW2 + row * LDH + cc;
        d[0] = r.b[k].x; d[1] = r.b[k].y; d[2] = r.b[k].z; d[3] = r.b[k].w;
    }
}

template <int DIN>
__device__ __forceinline__ void stage_weights(const float *__restrict__ w1,
                                              const float *__restrict__ w2, float *sW1,
                                              float *sW2) {
    WeightRegs<DIN> r;
    load_weights<DIN>(w1, w2, r);
    store_weights<DIN>(r, sW1, sW2);
}


__device__ __forceinline__ float4 fma4(float4 a, float w, float4 acc) {
    return make_float4(fmaf(a.x, w, acc.x), fmaf(a.y, w, acc.y), fmaf(a.z, w, acc.z),
                       fmaf(a.w, w, acc.w));
}

template <int RPT>
struct GatherHead {  // per-row CSR range and self row, loaded up front
    int32_t beg[RPT], deg[RPT];
    float4 self[RPT];
};

// first load round of gather_rows (row pointers and self rows); split out so
// a caller can put other independent loads in flight before the tail waits
template <int RPT, int RPP, int LPR>
__device__ __forceinline__ void gather_head(const float4 *__restrict__ h4,
                                            const int32_t *__restrict__ rowptr, int64_t row0,
                                            int nv, int rbase, int c, GatherHead<RPT> &hd) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const int rr = rbase + k * RPP;
        const int64_t vrow = row0 + (rr < nv ? rr : nv - 1);
        hd.beg[k] = rowptr[vrow];
        hd.deg[k] = rowptr[vrow + 1];
        hd.self[k] = h4[vrow * LPR + c];
    }
}

// one round of up to 4 neighbours per row: acc += x[u] (slots past the
// row's degree enter with weight 0), and the self term acc = ope x[v] + acc
// (shared by gather_tail and the walking forward, so both are bitwise equal)
template <int RPT, bool XFORM>
__device__ __forceinline__ void gather_round(const float4 (&a)[RPT][4], int j0,
                                             const int32_t (&deg)[RPT], float4 sc, float4 sh,
                                             float4 (&acc)[RPT]) {
#pragma unroll
    for (int k = 0; k < RPT; ++k)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float w = j0 + t < deg[k] ? 1.f : 0.f;
            acc[k] = fma4(XFORM ? xform4(a[k][t], sc, sh) : a[k][t], w, acc[k]);
        }
}

template <int RPT, bool XFORM>
__device__ __forceinline__ void gather_self(const float4 (&self)[RPT], float ope, float4 sc,
                                            float4 sh, float4 (&acc)[RPT]) {
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        const float4 x = XFORM ? xform4(self[k], sc, sh) : self[k];
        acc[k] = make_float4(ope * x.x + acc[k].x, ope * x.y + acc[k].y, ope * x.z + acc[k].z,
                             ope * x.w + acc[k].w);
    }
}

// the first neighbour round's indices of gather_tail (the same clamped
// addresses), loaded ahead so they are in flight across other work (the
// forward's deferred BatchNorm finish); rows with no in-edges: not loaded
template <int RPT>
__device__ __forceinline__ void gather_idx0(const int32_t *__restrict__ col,
                                            const GatherHead<RPT> &hd, int32_t (&u)[RPT][4]) {
    int maxdeg = 0, maxend = 0;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        maxend = hd.deg[k] > maxend ? hd.deg[k] : maxend;
        const int d = hd.deg[k] - hd.beg[k];
        maxdeg = d > maxdeg ? d : maxdeg;
    }
    if (maxdeg > 0) {
#pragma unroll
        for (int k = 0; k < RPT; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int32_t e = hd.beg[k] + t;
                u[k][t] = col[e < maxend ? e : maxend - 1];
            }
    }
}

// U0: round 0's indices come from gather_idx0 (u0) instead of being loaded here
template <int RPT, int LPR, bool XFORM, bool U0 = false>
__device__ __forceinline__ void gather_tail(const float4 *__restrict__ h4,
                                            const int32_t *__restrict__ col, GatherHead<RPT> &hd,
                                            int c, float ope, float4 sc, float4 sh,
                                            float4 (&acc)[RPT],
                                            const int32_t (*u0)[4] = nullptr) {
    int maxdeg = 0, maxend = 0;
#pragma unroll
    for (int k = 0; k < RPT; ++k) {
        acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        maxend = hd.deg[k] > maxend ? hd.deg[k] : maxend;
        hd.deg[k] -= hd.beg[k];
        maxdeg = hd.deg[k] > maxdeg ? hd.deg[k] : maxdeg;
    }
    for (int j0 = 0; j0 < maxdeg; j0 += 4) {
        int32_t u[RPT][4];
#pragma unroll
        for (int k = 0; k < RPT; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int32_t e = hd.beg[k] + j0 + t;
                u[k][t] = (U0 && j0 == 0) ? u0[k][t] : col[e < maxend ? e : maxend - 1];
            }
        float4 a[RPT][4];
#pragma unroll
        for (int k = 0; k < RPT; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t) a[k][t] = h4[static_cast<int64_t>(u[k][t]) * LPR + c];
        gather_round<RPT, XFORM>(a, j0, hd.deg, sc, sh, acc);
    }
    gather_self<RPT, XFORM>(hd.self, ope, sc, sh, acc);
}

// Sum aggregation of RPT rows (row0 + rbase + k * RPP) for one 4-channel
// chunk c: out = ope * x[v] + sum_{u in N(v)} x[u] in CSR order, x optionally
// relu(sc * h + sh).  Requires nv >= 1.
//
// Latency: all rows' row pointers and self rows are loaded together, then per
// round 4 neighbour indices per row, then those neighbour rows — every load
// unconditional so that each batch stays in flight (a load whose value is only
// used under a predicate gets sunk into a branch with its own s_waitcnt):
//   * rows past nv duplicate row nv - 1 (computed, never stored by callers);
//   * neighbour slots past a row's degree read a clamped valid edge of this
//     thread's rows and enter through fmaf(x, 0, acc) — exact: x * 1 and
//     acc + x * 0 round like the plain add for finite x.
template <int RPT, int RPP, int LPR, bool XFORM>
__device__ __forceinline__ void gather_rows(const float4 *__restrict__ h4,
                                            const int32_t *__restrict__ rowptr,
                                            const int32_t *__restrict__ col, int64_t row0, int nv,
                                            int rbase, int c, float ope, float4 sc, float4 sh,
                                            float4 (&acc)[RPT]) {
    GatherHead<RPT> hd;
    gather_head<RPT, RPP, LPR>(h4, rowptr, row0, nv, rbase, c, hd);
    gather_tail<RPT, LPR, XFORM>(h4, col, hd, c, ope, sc, sh, acc);
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

// ---------------------------------------------------------------------------
// Operand-prefetching forms of the three products (same k order per output,
// hence bitwise the results of mma_nt / mma_nn / mma_tn).  The loop forms
// above let hipcc emit "2 x ds_read2_b32, s_waitcnt lgkmcnt(0), 2 MFMA": the
// next reads issue only behind the dependent MFMA, so every MFMA pair pays an
// LDS round trip (measured: ~130 cycles per 64-cycle MFMA, phase trace r02).
// Here the operands of a chunk of C steps are read into registers one chunk
// ahead and the MFMAs of up to two independent products alternate, so the
// matrix pipe sees back-to-back issue.
//   operand X(idx, k) = COL ? Xs[k * ld + idx] : Xs[idx * ld + k]
//   NT = <false, false>, NN = <false, true>, TN = <true, true>
// ---------------------------------------------------------------------------
// pins the software pipeline: without it hipcc hoists every LDS read of the
// product (IR level, across other loops) and the kernel spills
// ds_read_b128-fed products: pin the next k block's operand reads ahead of
// the current block's MFMAs (without the pin the scheduler sinks them behind
// the block's MFMAs into the same registers, and each block then waits out an
// LDS latency).
constexpr bool kMmaPrefetchPin = true;  // (gin_bwd5_k 15.80 -> 15.63 us, round 2)

__device__ __forceinline__ void mma_step_fence() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
}

// lane base of operand X: step s then reads base[s * mma_step<COL>(ld)] — one
// address register per operand, every step an immediate offset (an address
// formed as ((2 s) | kk) * ld + i per step is hoisted per step and spills)
template <bool COL>
__device__ __forceinline__ const float *mma_base(const float *X, int ld) {
    const int l = threadIdx.x & 63, i = l & 31, kk = l >> 5;
    return COL ? X + kk * ld + i : X + i * ld + kk;
}
template <bool COL>
__device__ __forceinline__ int mma_step(int ld) { return COL ? 2 * ld : 2; }

template <int K, bool AC, bool BC, int D = 4>
__device__ __forceinline__ f32x16 mma_pf(const float *As, int lda, const float *Bs, int ldb,
                                         f32x16 acc) {
    constexpr int S = K / 2, R = D + 1;
    const float *pa = mma_base<AC>(As, lda), *pb = mma_base<BC>(Bs, ldb);
    const int sa = mma_step<AC>(lda), sb = mma_step<BC>(ldb);
    float a[R], b[R];
#pragma unroll
    for (int s = 0; s < D; ++s) {
        a[s] = pa[s * sa];
        b[s] = pb[s * sb];
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
        if (s + D < S) {
            a[(s + D) % R] = pa[(s + D) * sa];
            b[(s + D) % R] = pb[(s + D) * sb];
        }
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s % R], b[s % R], acc, 0, 0, 0);
        mma_step_fence();
    }
    return acc;
}

// two independent products over the same K, MFMAs alternating.  asum (if
// given) accumulates this lane's A1 operand values over k: for a TN first
// product (A1 = a tile read by column) that is the column's sum over the
// lane's half of the rows — the bias gradient, free beside the MFMAs
// (add the xor-32 partner lane's value for the full column).
template <int K, bool AC1, bool BC1, bool AC2, bool BC2, int D = 3>
__device__ __forceinline__ void mma_pf2(const float *A1, int la1, const float *B1, int lb1,
                                        f32x16 &c1, const float *A2, int la2, const float *B2,
                                        int lb2, f32x16 &c2, float *asum = nullptr) {
    constexpr int S = K / 2, R = D + 1;
    const float *pa1 = mma_base<AC1>(A1, la1), *pb1 = mma_base<BC1>(B1, lb1);
    const float *pa2 = mma_base<AC2>(A2, la2), *pb2 = mma_base<BC2>(B2, lb2);
    const int sa1 = mma_step<AC1>(la1), sb1 = mma_step<BC1>(lb1);
    const int sa2 = mma_step<AC2>(la2), sb2 = mma_step<BC2>(lb2);
    float a1[R], b1[R], a2[R], b2[R];
#pragma unroll
    for (int s = 0; s < D; ++s) {
        a1[s] = pa1[s * sa1];
        b1[s] = pb1[s * sb1];
        a2[s] = pa2[s * sa2];
        b2[s] = pb2[s * sb2];
    }
#pragma unroll
    for (int s = 0; s < S; ++s) {
        if (s + D < S) {
            const int r = (s + D) % R;
            a1[r] = pa1[(s + D) * sa1];
            b1[r] = pb1[(s + D) * sb1];
            a2[r] = pa2[(s + D) * sa2];
            b2[r] = pb2[(s + D) * sb2];
        }
        c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s % R], b1[s % R], c1, 0, 0, 0);
        if (asum) *asum += a1[s % R];
        c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a2[s % R], b2[s % R], c2, 0, 0, 0);
        mma_step_fence();
    }
    // both chains complete here: otherwise hipcc sinks a chain whose result is
    // only read after the tile loop (a dW accumulator) to the loop latch,
    // behind the next barrier, with all its operands held live meanwhile
    asm volatile("" ::"v"(c1[0]), "v"(c2[0]));
}

// acc + p[0] + p[stride] + ... + p[15 stride], added in that order: the 16
// LDS reads go out together (a loop over a runtime start row is not unrolled
// by hipcc and pays one LDS round trip per row — ~2k cycles per call, phase
// trace r02)
__device__ __forceinline__ float col_sum16(float acc, const float *p, int stride) {
    float v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = p[k * stride];
#pragma unroll
    for (int k = 0; k < 16; ++k) acc += v[k];
    return acc;
}

// ---------------------------------------------------------------------------
// Wide-operand forms (gin_bwd5_k).  ds_read_b32 at one or two waves per SIMD
// delivers a fraction of the LDS rate (MI355X_MICROARCH.md §LDS), so each
// lane reads FOUR k values per ds_read_b128 instead: the k order of the K
// sum is permuted — step s = 4 qb + t of lane half kk covers
//   k(s, kk) = 8 qb + 4 kk + t            (kperm below)
// — identically for both operands, so every product is still the exact
// sum over k (only the association order differs from mma_nt/nn/tn).  An
// operand is "k-contiguous" per lane: A row-major over k (NN / NT rows), or a
// transposed image [col][k] for the TN products over rows.  With row strides
// = 4 (mod 64) floats the 16-lane groups of ds_read_b128 are conflict free.
// ---------------------------------------------------------------------------
__device__ __forceinline__ int kperm(int s, int kk) { return 8 * (s >> 2) + 4 * kk + (s & 3); }

__device__ __forceinline__ float f4at(const float4 &v, int t) {
    return t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w;
}

// acc += A B over K = 8 NB: A k-contiguous per lane (pa = this lane's row
// start + 4 kk), B in registers (b[s] = B(kperm(s, kk), lane's column)).
// One accumulation chain (64-cycle issue = dependent latency of the f32 MFMA).
// STRIDE: floats between the lane's consecutive 4-step blocks — 8 for the
// kperm order; 4 for an image whose lane half kk holds k = 2 s + kk as one
// contiguous run (the even | odd split of gin_bwd5r_k's agg rows), which
// feeds step s the forward's own k pair (2 s, 2 s + 1): mma_nt's order.
// The weights come either as a float array or as two f32x16 (b0: steps
// 0..15, b1: 16..31 — registers a wave of another role uses as accumulators).
__device__ __forceinline__ float wsel(const float *b, int s) { return b[s]; }
struct W32 {
    const f32x16 &lo, &hi;
};
__device__ __forceinline__ float wsel(const W32 &b, int s) { return s < 16 ? b.lo[s] : b.hi[s - 16]; }

template <int NB, int STRIDE = 8, class WB>
__device__ __forceinline__ f32x16 mma_rk4(const float *pa, const WB &b, f32x16 acc) {
    float4 a[2];
    a[0] = *reinterpret_cast<const float4 *>(pa);
#pragma unroll
    for (int qb = 0; qb < NB; ++qb) {
        if (qb + 1 < NB) a[(qb + 1) & 1] = *reinterpret_cast<const float4 *>(pa + STRIDE * (qb + 1));
        if (kMmaPrefetchPin) __builtin_amdgcn_sched_barrier(0);  // the next block's read goes out first
#pragma unroll
        for (int t = 0; t < 4; ++t)
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(f4at(a[qb & 1], t), wsel(b, 4 * qb + t), acc, 0, 0, 0);
        mma_step_fence();
    }
    return acc;
}

// one product of mma_kk4x2 (the same per-element chain as its c1 / c2):
// c += A B over K = 8 NB, both operands k-contiguous per lane; asum += the
// lane's A values when SUM
template <int NB, bool SUM>
__device__ __forceinline__ void mma_kk4(const float *pa, const float *pb, f32x16 &c, float &asum) {
    float4 a[2], b[2];
    a[0] = *reinterpret_cast<const float4 *>(pa);
    b[0] = *reinterpret_cast<const float4 *>(pb);
#pragma unroll
    for (int qb = 0; qb < NB; ++qb) {
        if (qb + 1 < NB) {
            const int o = 8 * (qb + 1), x = (qb + 1) & 1;
            a[x] = *reinterpret_cast<const float4 *>(pa + o);
            b[x] = *reinterpret_cast<const float4 *>(pb + o);
        }
        if (kMmaPrefetchPin) __builtin_amdgcn_sched_barrier(0);
        const int x = qb & 1;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float av = f4at(a[x], t);
            c = __builtin_amdgcn_mfma_f32_32x32x2f32(av, f4at(b[x], t), c, 0, 0, 0);
            if (SUM) asum += av;
        }
        mma_step_fence();
    }
    asm volatile("" ::"v"(c[0]));
}

// two products sharing the A operand, K = 8 NB, both operands k-contiguous
// per lane (pa, pb1, pb2 = lane starts + 4 kk); asum += the lane's A values
// (for a transposed dz image: the column sum over the lane's half of the
// rows — the bias gradient).  The two chains alternate.
template <int NB>
__device__ __forceinline__ void mma_kk4x2(const float *pa, const float *pb1, const float *pb2,
                                          f32x16 &c1, f32x16 &c2, float &asum) {
    float4 a[2], b1[2], b2[2];
    a[0] = *reinterpret_cast<const float4 *>(pa);
    b1[0] = *reinterpret_cast<const float4 *>(pb1);
    b2[0] = *reinterpret_cast<const float4 *>(pb2);
#pragma unroll
    for (int qb = 0; qb < NB; ++qb) {
        if (qb + 1 < NB) {
            const int o = 8 * (qb + 1), x = (qb + 1) & 1;
            a[x] = *reinterpret_cast<const float4 *>(pa + o);
            b1[x] = *reinterpret_cast<const float4 *>(pb1 + o);
            b2[x] = *reinterpret_cast<const float4 *>(pb2 + o);
        }
        if (kMmaPrefetchPin) __builtin_amdgcn_sched_barrier(0);  // the next block's reads go out first
        const int x = qb & 1;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const float av = f4at(a[x], t);
            c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, f4at(b1[x], t), c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(av, f4at(b2[x], t), c2, 0, 0, 0);
            asum += av;
        }
        mma_step_fence();
    }
    asm volatile("" ::"v"(c1[0]), "v"(c2[0]));
}

// s_waitcnt through the builtin (the compiler's wait model sees it, an asm
// statement it does not): vmcnt(0) = 0x0F70, lgkmcnt(0) alone = 0xC07F (gfx9
// encoding: vmcnt [3:0] + [15:14], expcnt [6:4], lgkmcnt [11:8])
__device__ __forceinline__ void vm_wait_all() { __builtin_amdgcn_s_waitcnt(0x0F70); }
// barrier without the vmcnt(0) of a __syncthreads fence (global stores and
// prefetch loads stay in flight across it)
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
}

// row of accumulator register `reg` of the 32x32 output tile held by lane l
__device__ __forceinline__ int acc_row(int reg, int l) { return (reg & 3) + 8 * (reg >> 2) + 4 * (l >> 5); }


}  // namespace scgib
