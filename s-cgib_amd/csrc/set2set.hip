// Set2Set readout (gfx950): DGL Set2Set(d, n_iters, 1) as the reference
// builds it (models.py:565; used by Mainmodel_finetuning.forward :515 and
// Mainmodel_domainadapt :271-272; DGL 1.1 nn/pytorch/glob.py semantics), ALL
// n_iters rounds in one launch per direction:
//
//   gates = W_ih q* + b_ih + W_hh h + b_hh      (PyTorch LSTM gate order i, f, g, o)
//   c = sig(f) c + sig(i) tanh(g);  h = sig(o) tanh(c)
//   e_v = <x_v, h_g>;  alpha = softmax over the graph's rows;  r_g = sum_v alpha_v x_v
//   q* = [h, r]
//
// Every graph's recurrence is independent of the others' (the LSTM runs on
// the B graph rows, one row each), so one 256-thread workgroup per graph runs
// the whole recurrence: thread j < 4d owns gate j (its dot products over the
// 2d + d inputs, held in LDS), and all four waves run the attention over the
// graph's rows (16 row groups of 16 lanes: group G takes rows p0 + G,
// p0 + G + 16, ...; lane j of a group holds channels j, j + 16, j + 32,
// j + 48, d <= 64), the first 64 rows staged in LDS.  This replaces the
// ~13 torch launches per round of the LSTM cell + attention (two GEMMs,
// eight elementwise ops, the readout, the concatenation) and their backward.
//
// Saved per graph and round (the backward's inputs), s2s_save(d) floats:
//   q*_prev [2d] | h_prev [d] | c_prev [d] | act [4d] (sig i, sig f, tanh g, sig o) |
//   c [d] | (max_g e, softmax denominator)
// The backward (one workgroup per graph, rounds in reverse) writes the gates'
// pre-activation gradients dG [B][T][4d]; set2set_wgrad_k then forms
// dW_ih = dG^T q*_prev, dW_hh = dG^T h_prev and db = sum dG (fixed order).
// Latency-bound VALU/shuffle work: no MFMA.
#include "common.h"

namespace scgib {

namespace {

constexpr int kS2SMaxD = 64;

__host__ __device__ constexpr int s2s_save(int d) { return 9 * d + 2; }

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
__device__ __forceinline__ float s2s_sigmoid(float v) { return 1.f / (1.f + expf(-v)); }

// <w[0, n), v[0, n)>, w a weight row in global memory, v in LDS: float4 loads
// when the row is a multiple of 4 floats (it is then 16-B aligned: row j
// starts at j n), four accumulators, unrolled so the row's loads are in
// flight together (a latency-bound dot: one thread per gate)
__device__ __forceinline__ float s2s_dot(const float *__restrict__ w, const float *v, int n) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    if ((n & 3) == 0) {
        const float4 *w4 = reinterpret_cast<const float4 *>(w);
#pragma unroll 16
        for (int k = 0; k < n / 4; ++k) {
            const float4 x = w4[k];
            a0 = fmaf(x.x, v[4 * k], a0);
            a1 = fmaf(x.y, v[4 * k + 1], a1);
            a2 = fmaf(x.z, v[4 * k + 2], a2);
            a3 = fmaf(x.w, v[4 * k + 3], a3);
        }
    } else {
#pragma unroll 4
        for (int k = 0; k < n; ++k) a0 = fmaf(w[k], v[k], a0);
    }
    return (a0 + a1) + (a2 + a3);
}

// The graph's rows: the first kS2SRows staged in LDS by the workgroup (every
// round and pass re-reads them), the rest read from global memory.  Row group
// G (of 16) takes rows p0 + G, p0 + G + 16, ...: its staged rows are the
// kS2SPer slots G + 16 i, read into registers once per attention pass with
// plain LDS loads (a per-element LDS-or-global select made every read a flat
// load, and the second pass recomputed every logit: phase trace r05_s2s); rows
// past kS2SRows go through their own global-memory loop.
constexpr int kS2SRows = 64;
constexpr int kS2SPer = kS2SRows / 16;
struct S2SRows {
    const float *__restrict__ x;  // global [*][d]
    const float *xs;              // LDS copy of rows [p0, p0 + ns)
    int64_t p0;
    int ns, d;
};

// all 256 threads: stage rows [p0, p0 + min(n, kS2SRows)) of x into xs (then a
// barrier).  Every thread's loads (<= 4 float4, or <= 16 floats for a width
// not a multiple of 4) are issued before its LDS stores: a load / wait /
// store loop paid one memory latency per element, before the kernels' first
// phase mark (8 of set2set_fwd_k's 17.6 us in the kernel trace).  Call it
// before issuing other loads whose wait it would otherwise share.
__device__ __forceinline__ int s2s_stage(const float *__restrict__ x, int64_t p0, int64_t p1,
                                         int d, float *xs) {
    const int ns = static_cast<int>(p1 - p0 < kS2SRows ? p1 - p0 : kS2SRows);
    const int tid = threadIdx.x, total = ns * d;
    // float4 staging needs 16-B aligned rows: d % 4 == 0 AND a 16-B aligned
    // base (a tensor view with a storage offset may not be): else scalar loads
    if ((d & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        constexpr int K = kS2SRows * kS2SMaxD / 4 / 256;
        const float4 *x4 = reinterpret_cast<const float4 *>(x + p0 * d);
        float4 *xs4 = reinterpret_cast<float4 *>(xs);
        float4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = tid + 256 * k;
            v[k] = i < total / 4 ? x4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (tid + 256 * k < total / 4) xs4[tid + 256 * k] = v[k];
    } else {
        constexpr int K = kS2SRows * kS2SMaxD / 256;
        float v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = tid + 256 * k;
            v[k] = i < total ? x[p0 * d + i] : 0.f;
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (tid + 256 * k < total) xs[tid + 256 * k] = v[k];
    }
    return ns;
}

// lane j's channels j + 16 k of the row group's staged slots G + 16 i, 0 past
// ns or d.  The index is clamped into the staging array (ns <= 64, d <= 64),
// so the loads are unconditional and go out together.
__device__ __forceinline__ void s2s_rows_lds(const S2SRows &X, int G, int j,
                                             float (&xv)[kS2SPer][4]) {
#pragma unroll
    for (int i = 0; i < kS2SPer; ++i) {
        const int o = G + 16 * i;
        const bool ok = o < X.ns;
        const int oc = ok ? o : 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = j + 16 * k;
            const float v = X.xs[oc * X.d + (c < X.d ? c : 0)];
            xv[i][k] = ok && c < X.d ? v : 0.f;
        }
    }
}

// lane j's channels j + 16 k of global row v, 0 past d
__device__ __forceinline__ void s2s_row_glb(const float *__restrict__ x, int64_t v, int d, int j,
                                            float (&xv)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = j + 16 * k;
        xv[k] = c < d ? x[v * d + c] : 0.f;
    }
}

// the row's logit-style dot <x_v, q> for the 16 lanes of its row group (every
// lane of the group returns it)
__device__ __forceinline__ float s2s_dot16(const float (&xv)[4], const float (&qv)[4]) {
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) dot = fmaf(xv[k], qv[k], dot);
    return s2s_red16(dot);
}

// All four waves: the attention readout of rows [p0, p1) with query q (LDS,
// d floats) into r (LDS) and (max, denominator) into st.  The staged rows'
// logits stay in registers between the two passes; rows past kS2SRows are
// re-read and their logits recomputed (a graph may hold any number of rows).
// red: LDS scratch, kS2SRed floats; the waves' partials combine in fixed
// order.  Call from every thread.
constexpr int kS2SRed = 8 + 4 * kS2SMaxD;
__device__ __forceinline__ void s2s_attend_fwd(const S2SRows &X, int64_t p1, const float *q,
                                               float *r, float *st, float *red) {
    const int64_t p0 = X.p0;
    const int d = X.d;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, j = l & 15;
    const int G = 4 * w + (l >> 4);
    float qv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) qv[k] = j + 16 * k < d ? q[j + 16 * k] : 0.f;
    // (a row group's 16 lanes run a row together: the butterflies stay
    // within active lanes whatever the other groups do)
    float xv[kS2SPer][4], e[kS2SPer];
    s2s_rows_lds(X, G, j, xv);
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < kS2SPer; ++i) {
        e[i] = s2s_dot16(xv[i], qv);
        if (G + 16 * i < X.ns) mx = fmaxf(mx, e[i]);
    }
    for (int64_t v = p0 + kS2SRows + G; v < p1; v += 16) {
        float xg[4];
        s2s_row_glb(X.x, v, d, j, xg);
        mx = fmaxf(mx, s2s_dot16(xg, qv));
    }
    mx = s2s_max_all(mx);
    if (l == 0) red[w] = mx;
    __syncthreads();
    mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    // denominator and the unnormalised readout sum_v exp(e_v - max) x_v in one
    // pass, rows in the first pass's order
    float den = 0.f, acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < kS2SPer; ++i) {
        if (G + 16 * i < X.ns) {
            const float a = expf(e[i] - mx);
            den += j == 0 ? a : 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) acc[k] = fmaf(xv[i][k], a, acc[k]);
        }
    }
    for (int64_t v = p0 + kS2SRows + G; v < p1; v += 16) {
        float xg[4];
        s2s_row_glb(X.x, v, d, j, xg);
        const float a = expf(s2s_dot16(xg, qv) - mx);
        den += j == 0 ? a : 0.f;
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[k] = fmaf(xg[k], a, acc[k]);
    }
    den = s2s_red_q(s2s_red16(den));
    if (l == 0) red[4 + w] = den;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float t = s2s_red_q(acc[k]);
        const int c = j + 16 * k;
        if (l < 16 && c < d) red[8 + w * kS2SMaxD + c] = t;
    }
    __syncthreads();
    const float D = (red[4] + red[5]) + (red[6] + red[7]);
    if (tid < d) {
        const float t = (red[8 + tid] + red[8 + kS2SMaxD + tid]) +
                        (red[8 + 2 * kS2SMaxD + tid] + red[8 + 3 * kS2SMaxD + tid]);
        r[tid] = D > 0.f ? t / D : 0.f;  // (an empty graph reads out zero)
    }
    if (tid == 0) {
        st[0] = mx;
        st[1] = D;
    }
}

// All four waves: the attention backward for d r = gr (LDS) with query q (LDS):
//   dalpha_v = <gr, x_v>;  s = sum alpha dalpha;  de_v = alpha_v (dalpha_v - s)
//   dx_v (+)= alpha_v gr + de_v q (dxs: the staged rows' LDS accumulator);
//   dq = sum de_v x_v  (into dq, LDS).  Row groups and red as s2s_attend_fwd;
// the staged rows' alpha and dalpha stay in registers between the passes.
__device__ __forceinline__ void s2s_attend_bwd(const S2SRows &X, int64_t p1, const float *q,
                                               const float *gr, float mx, float den,
                                               float *__restrict__ dx, float *dxs,
                                               bool accumulate, float *dq, float *red) {
    const int64_t p0 = X.p0;
    const int d = X.d;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, j = l & 15;
    const int G = 4 * w + (l >> 4);
    float gv[4], qv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = j + 16 * k;
        gv[k] = c < d ? gr[c] : 0.f;
        qv[k] = c < d ? q[c] : 0.f;
    }
    float xv[kS2SPer][4], al[kS2SPer], da[kS2SPer];
    s2s_rows_lds(X, G, j, xv);
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < kS2SPer; ++i) {
        al[i] = expf(s2s_dot16(xv[i], qv) - mx) / den;
        da[i] = s2s_dot16(xv[i], gv);
        if (G + 16 * i < X.ns) s += j == 0 ? al[i] * da[i] : 0.f;
    }
    for (int64_t v = p0 + kS2SRows + G; v < p1; v += 16) {
        float xg[4];
        s2s_row_glb(X.x, v, d, j, xg);
        const float alpha = expf(s2s_dot16(xg, qv) - mx) / den;
        const float dalpha = s2s_dot16(xg, gv);  // (all 16 lanes: outside the select)
        s += j == 0 ? alpha * dalpha : 0.f;
    }
    s = s2s_red_q(s2s_red16(s));
    if (l == 0) red[w] = s;
    __syncthreads();
    s = (red[0] + red[1]) + (red[2] + red[3]);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < kS2SPer; ++i) {
        const int o = G + 16 * i;
        if (o < X.ns) {
            const float de = al[i] * (da[i] - s);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int c = j + 16 * k;
                if (c < d) {
                    // staged rows accumulate in LDS (written out once, after the
                    // last round)
                    const float t = fmaf(de, qv[k], al[i] * gv[k]);
                    const float prev = accumulate ? dxs[o * d + c] : 0.f;
                    dxs[o * d + c] = prev + t;
                    acc[k] = fmaf(de, xv[i][k], acc[k]);
                }
            }
        }
    }
    for (int64_t v = p0 + kS2SRows + G; v < p1; v += 16) {
        float xg[4];
        s2s_row_glb(X.x, v, d, j, xg);
        const float alpha = expf(s2s_dot16(xg, qv) - mx) / den;
        const float de = alpha * (s2s_dot16(xg, gv) - s);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int c = j + 16 * k;
            if (c < d) {
                const float t = fmaf(de, qv[k], alpha * gv[k]);
                dx[v * d + c] = accumulate ? dx[v * d + c] + t : t;
                acc[k] = fmaf(de, xg[k], acc[k]);
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float t = s2s_red_q(acc[k]);
        const int c = j + 16 * k;
        if (l < 16 && c < d) red[8 + w * kS2SMaxD + c] = t;
    }
    __syncthreads();
    if (tid < d)
        dq[tid] = (red[8 + tid] + red[8 + kS2SMaxD + tid]) +
                  (red[8 + 2 * kS2SMaxD + tid] + red[8 + 3 * kS2SMaxD + tid]);
}

}  // namespace

// the gate dot of s2s_dot's float4 path with the weight row in registers
// (same four accumulators, same k order: the same bits)
template <int N4>
__device__ __forceinline__ float s2s_dot_reg(const float4 (&w)[N4], const float *v) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int k = 0; k < N4; ++k) {
        a0 = fmaf(w[k].x, v[4 * k], a0);
        a1 = fmaf(w[k].y, v[4 * k + 1], a1);
        a2 = fmaf(w[k].z, v[4 * k + 2], a2);
        a3 = fmaf(w[k].w, v[4 * k + 3], a3);
    }
    return (a0 + a1) + (a2 + a3);
}

// One workgroup per graph: all n_iters rounds.  out [B][2d] = the last q*.
// Round 0 starts from q* = h = 0, so its gate products are exactly +0 and
// z = (0 + b_ih) + (0 + b_hh) is formed without them (the round-0 dots were
// 6 of the kernel's ~20 us, phase trace r04).  REG (d = 64: thread j owns
// gate j of 256): the thread's W_ih / W_hh rows (192 floats) are loaded into
// registers at the kernel's start — their latency hides under round 0 — and
// every later round's dots read them there instead of reloading the rows.
template <bool REG>
__global__ __launch_bounds__(256) void set2set_fwd_k(
    const float *__restrict__ x, const int32_t *__restrict__ ptr, int d, int T,
    const float *__restrict__ w_ih, const float *__restrict__ b_ih,
    const float *__restrict__ w_hh, const float *__restrict__ b_hh, float *__restrict__ save,
    float *__restrict__ out) {
    __shared__ float sQ[2 * kS2SMaxD], sH[kS2SMaxD], sC[kS2SMaxD], sA[4 * kS2SMaxD];
    __shared__ float sX[kS2SRows * kS2SMaxD], sRedA[kS2SRed];
    const int64_t g = blockIdx.x;
    const int tid = threadIdx.x, D2 = 2 * d, G4 = 4 * d, S = s2s_save(d);
    constexpr int NI = REG ? 2 * kS2SMaxD / 4 : 1, NH = REG ? kS2SMaxD / 4 : 1;
    const int64_t p0 = ptr[g], p1 = ptr[g + 1];
    const S2SRows X{x, sX, p0, s2s_stage(x, p0, p1, d, sX), d};
    float4 wi[NI], wh[NH];
    if constexpr (REG) {  // d = 64, G4 = 256: every thread owns a gate
        const float4 *ri = reinterpret_cast<const float4 *>(w_ih + static_cast<int64_t>(tid) * D2);
        const float4 *rh = reinterpret_cast<const float4 *>(w_hh + static_cast<int64_t>(tid) * d);
#pragma unroll
        for (int k = 0; k < NI; ++k) wi[k] = ri[k];
#pragma unroll
        for (int k = 0; k < NH; ++k) wh[k] = rh[k];
    }
    if (tid < D2) sQ[tid] = 0.f;
    if (tid < d) sH[tid] = sC[tid] = 0.f;
    // this thread's gate biases (b_ih + b_hh added after the two products, as
    // F.linear(q, W_ih, b_ih) + F.linear(h, W_hh, b_hh))
    const float bi = tid < G4 ? b_ih[tid] : 0.f, bh = tid < G4 ? b_hh[tid] : 0.f;
    SCGIB_MARK(0);
    __syncthreads();
    SCGIB_MARK(1);
    for (int t = 0; t < T; ++t) {
        float *sv = save + (g * T + t) * S;
        if (tid < D2) sv[tid] = sQ[tid];
        if (tid < d) {
            sv[D2 + tid] = sH[tid];
            sv[3 * d + tid] = sC[tid];
        }
        if (tid < G4) {  // gate tid
            float a = 0.f, b = 0.f;  // round 0: q* = h = 0
            if (t > 0) {
                if constexpr (REG) {
                    a = s2s_dot_reg(wi, sQ);
                    b = s2s_dot_reg(wh, sH);
                } else {
                    a = s2s_dot(w_ih + static_cast<int64_t>(tid) * D2, sQ, D2);
                    b = s2s_dot(w_hh + static_cast<int64_t>(tid) * d, sH, d);
                }
            }
            const float z = (a + bi) + (b + bh);
            const int kind = tid / d;  // 0 i, 1 f, 2 g, 3 o
            const float act = kind == 2 ? tanhf(z) : s2s_sigmoid(z);
            sA[tid] = act;
            sv[4 * d + tid] = act;
        }
        __syncthreads();
        if (t == 0) SCGIB_MARK(2);
        if (tid < d) {
            const float c = sA[d + tid] * sC[tid] + sA[tid] * sA[2 * d + tid];
            const float h = sA[3 * d + tid] * tanhf(c);
            sC[tid] = c;
            sH[tid] = h;
            sQ[tid] = h;
            sv[8 * d + tid] = c;
        }
        __syncthreads();
        if (t == 0) SCGIB_MARK(3);
        s2s_attend_fwd(X, p1, sH, sQ + d, sv + 9 * d, sRedA);
        __syncthreads();
        if (t == 0) SCGIB_MARK(4);
    }
    SCGIB_MARK(5);
    if (tid < D2) out[g * D2 + tid] = sQ[tid];
}

// One workgroup per graph, rounds in reverse: d q*_T = g_out -> dx (rows of
// the graph; capacity rows past ptr[B] are zeroed by the extra workgroups)
// and dG [B][T][4d] for set2set_wgrad_k.  REG (d = 64): the transposed gate
// products' weights (lane l of wave w: columns l, l + 64 of W_ih and l of
// W_hh over gate rows 64 w ..) are loaded into registers at the kernel's
// start, their latency hidden under the last round's attention (loaded at
// the products, four dependent 16-row batches: 3.8 us of the kernel, phase
// trace r05_s2s).
template <bool REG>
__global__ __launch_bounds__(256) void set2set_bwd_k(
    const float *__restrict__ x, const int32_t *__restrict__ ptr, int64_t nseg, int d, int T,
    const float *__restrict__ w_ih, const float *__restrict__ w_hh,
    const float *__restrict__ save, const float *__restrict__ g_out, float *__restrict__ dx,
    float *__restrict__ dG, int64_t nrows) {
    if (static_cast<int64_t>(blockIdx.x) >= nseg) {  // block-uniform: the padding rows
        const int64_t r0 = ptr[nseg], nb = gridDim.x - nseg;
        for (int64_t i = r0 * d + (blockIdx.x - nseg) * 256 + threadIdx.x; i < nrows * d;
             i += nb * 256)
            dx[i] = 0.f;
        return;
    }
    __shared__ float sDQ[2 * kS2SMaxD], sDH[kS2SMaxD], sDC[kS2SMaxD], sDG[4 * kS2SMaxD];
    __shared__ float sHq[kS2SMaxD], sAtt[kS2SMaxD], sPart[4][3 * kS2SMaxD];
    __shared__ float sX[kS2SRows * kS2SMaxD], sDX[kS2SRows * kS2SMaxD], sRedA[kS2SRed];
    const int64_t g = blockIdx.x;
    const int tid = threadIdx.x, D2 = 2 * d, G4 = 4 * d, S = s2s_save(d);
    // a round's saved values this thread reads (its act / c / c_prev slice,
    // the attention's max and denominator), loaded one round ahead — the last
    // round's before the staging — so no phase waits on a save load (at the
    // point of use they were a load round in each round's first phase and cell)
    struct SvRound {
        float i, f, gg, o, c, cp, mx, den;
    };
    auto sv_load = [&](int t) {
        const float *sv = save + (g * T + t) * S;
        const int k = tid < d ? tid : 0;
        return SvRound{sv[4 * d + k], sv[5 * d + k], sv[6 * d + k], sv[7 * d + k],
                       sv[8 * d + k], sv[3 * d + k], sv[9 * d], sv[9 * d + 1]};
    };
    SvRound cur = sv_load(T - 1);
    const int64_t p0 = ptr[g], p1 = ptr[g + 1];
    const S2SRows X{x, sX, p0, s2s_stage(x, p0, p1, d, sX), d};
    float wT[REG ? kS2SMaxD : 1][3];
    if constexpr (REG) {
        if (T > 1) {
            const int64_t w0 = 64 * (tid >> 6);
            const int l = tid & 63;
#pragma unroll
            for (int i = 0; i < kS2SMaxD; ++i) {
                wT[i][0] = w_ih[(w0 + i) * 128 + l];
                wT[i][1] = w_ih[(w0 + i) * 128 + 64 + l];
                wT[i][2] = w_hh[(w0 + i) * 64 + l];
            }
        }
    }
    if (tid < D2) sDQ[tid] = g_out[g * D2 + tid];
    if (tid < d) sDH[tid] = sDC[tid] = 0.f;  // from round t + 1 (none after the last)
    SCGIB_MARK(0);
    __syncthreads();
    SCGIB_MARK(1);
    for (int t = T - 1; t >= 0; --t) {
        const int mk = t == T - 1 ? 2 : 7;  // (trace build: the first two rounds' phases)
        (void)mk;
        const SvRound nxt = t > 0 ? sv_load(t - 1) : cur;  // in flight through this round
        // h_t (the round's query) = q*_t's first half: the next round's q*_prev,
        // or recomputed for the last round from its saved act / c
        if (tid < d) sHq[tid] = cur.o * tanhf(cur.c);
        __syncthreads();
        if (t >= T - 2) SCGIB_MARK(mk);
        s2s_attend_bwd(X, p1, sHq, sDQ + d, cur.mx, cur.den, dx, sDX, t < T - 1, sAtt, sRedA);
        __syncthreads();
        if (t >= T - 2) SCGIB_MARK(mk + 1);
        if (tid < d) {  // the cell: dh_t = d q*_t[:d] + the attention's d query + from round t + 1
            const float dh = (sDQ[tid] + sAtt[tid]) + sDH[tid];
            const float ig = cur.i, fg = cur.f, gg = cur.gg, og = cur.o, c = cur.c, cp = cur.cp;
            const float tc = tanhf(c);
            const float dc = sDC[tid] + dh * og * (1.f - tc * tc);
            sDG[tid] = dc * gg * ig * (1.f - ig);             // i
            sDG[d + tid] = dc * cp * fg * (1.f - fg);         // f
            sDG[2 * d + tid] = dc * ig * (1.f - gg * gg);     // g
            sDG[3 * d + tid] = dh * tc * og * (1.f - og);     // o
            sDC[tid] = dc * fg;                               // -> c_{t-1}
        }
        __syncthreads();
        if (t >= T - 2) SCGIB_MARK(mk + 2);
        if (tid < G4) dG[(g * T + t) * G4 + tid] = sDG[tid];
        // round 0's [d q*_{-1} | d h_{-1}] would be the gradient of the initial
        // state, the constant zeros: nothing reads it (the products were
        // 3.6 us of the kernel, phase trace r04)
        if (t == 0) break;
        // [d q*_{t-1} | d h_{t-1} (gates path)] = [W_ih | W_hh]^T dG: wave w sums
        // the gates of its quarter, lane l the outputs l, l + 64, l + 128 < 3d
        // (coalesced along the weight rows); the quarters combine in fixed order
        if constexpr (REG) {  // (the same row order as below: the same bits)
            const int w = tid >> 6, l = tid & 63;
            float acc[3] = {0.f, 0.f, 0.f};
#pragma unroll
            for (int i = 0; i < kS2SMaxD; ++i) {
                const float gj = sDG[64 * w + i];
#pragma unroll
                for (int u = 0; u < 3; ++u) acc[u] = fmaf(wT[i][u], gj, acc[u]);
            }
#pragma unroll
            for (int u = 0; u < 3; ++u) sPart[w][l + 64 * u] = acc[u];
        } else {
            const int w = tid >> 6, l = tid & 63, D3 = 3 * d;
            const int j0 = (G4 * w) / 4, j1 = (G4 * (w + 1)) / 4;
            // per output slot u: its weight column (base, row stride), chosen
            // once, so the loads below are unconditional and the unrolled
            // rows' loads go out together (a branch per load made hipcc wait
            // for each one: 21 us of a round, tools/s2s_trace.py)
            const float *col[3];
            int64_t rs[3];
#pragma unroll
            for (int u = 0; u < 3; ++u) {
                const int o = l + 64 * u;
                col[u] = o < D2 ? w_ih + o : (o < D3 ? w_hh + (o - D2) : w_ih);
                rs[u] = o < D2 ? D2 : (o < D3 ? d : 0);
            }
            float acc[3] = {0.f, 0.f, 0.f};
            constexpr int kB = 16;  // rows per batch: 3 kB loads issued before their uses
            for (int jb = j0; jb < j1; jb += kB) {
                float wv[kB][3];
#pragma unroll
                for (int i = 0; i < kB; ++i) {
                    const int jc = jb + i < j1 ? jb + i : j1 - 1;  // (clamped: no branch)
#pragma unroll
                    for (int u = 0; u < 3; ++u) wv[i][u] = col[u][jc * rs[u]];
                }
#pragma unroll
                for (int i = 0; i < kB; ++i) {
                    const float gj = jb + i < j1 ? sDG[jb + i] : 0.f;
#pragma unroll
                    for (int u = 0; u < 3; ++u) acc[u] = fmaf(wv[i][u], gj, acc[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < 3; ++u)
                if (l + 64 * u < D3) sPart[w][l + 64 * u] = acc[u];
        }
        __syncthreads();
        if (t >= T - 2) SCGIB_MARK(mk + 3);
        if (tid < 3 * d) {
            const float v = (sPart[0][tid] + sPart[1][tid]) + (sPart[2][tid] + sPart[3][tid]);
            if (tid < D2)
                sDQ[tid] = v;
            else
                sDH[tid - D2] = v;
        }
        __syncthreads();
        cur = nxt;
    }
    SCGIB_MARK(12);
    for (int i = tid; i < X.ns * d; i += 256) dx[p0 * d + i] = sDX[i];
    SCGIB_MARK(13);
}

// dW_ih [4d][2d], dW_hh [4d][d], db_ih = db_hh [4d] (two outputs: two parameters):
// workgroup k < 3d forms column k of [dW_ih | dW_hh] over the R = B T saved
// rounds in order; workgroup 3d the bias.  Thread j = gate.
__global__ __launch_bounds__(256) void set2set_wgrad_k(const float *__restrict__ save,
                                                       const float *__restrict__ dG, int64_t R,
                                                       int d, float *__restrict__ dw_ih,
                                                       float *__restrict__ dw_hh,
                                                       float *__restrict__ db_ih,
                                                       float *__restrict__ db_hh) {
    const int k = blockIdx.x, j = threadIdx.x, D2 = 2 * d, G4 = 4 * d, S = s2s_save(d);
    if (j >= G4) return;
    // (four accumulators over r mod 4, combined in fixed order: the loads of
    // the unrolled rows are in flight together)
    float a[4] = {0.f, 0.f, 0.f, 0.f};
    if (k == 3 * d) {
#pragma unroll 8
        for (int64_t r = 0; r < R; ++r) a[r & 3] += dG[r * G4 + j];
        const float acc = (a[0] + a[1]) + (a[2] + a[3]);
        db_ih[j] = acc;
        db_hh[j] = acc;
        return;
    }
    // save row r starts with [q*_prev (2d) | h_prev (d)]: column k of both inputs
#pragma unroll 8
    for (int64_t r = 0; r < R; ++r) a[r & 3] = fmaf(dG[r * G4 + j], save[r * S + k], a[r & 3]);
    const float acc = (a[0] + a[1]) + (a[2] + a[3]);
    if (k < D2)
        dw_ih[static_cast<int64_t>(j) * D2 + k] = acc;
    else
        dw_hh[static_cast<int64_t>(j) * d + (k - D2)] = acc;
}

}  // namespace scgib

using namespace scgib;

extern "C" int64_t scgib_set2set_save_floats(int64_t n_graphs, int32_t dim, int32_t n_iters) {
    return n_graphs * n_iters * s2s_save(dim);
}

extern "C" int scgib_set2set_fwd(const float *x, const int32_t *graph_ptr, int64_t n_graphs,
                                 int32_t dim, int32_t n_iters, const float *w_ih,
                                 const float *b_ih, const float *w_hh, const float *b_hh,
                                 float *save, float *out, scgib_stream_t stream) {
    if (n_graphs < 0 || dim < 1 || dim > kS2SMaxD || n_iters < 1) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (!x || !graph_ptr || !w_ih || !b_ih || !w_hh || !b_hh || !save || !out)
        return SCGIB_EINVAL;
    if (dim == kS2SMaxD)
        set2set_fwd_k<true><<<static_cast<unsigned>(n_graphs), 256, 0, as_stream(stream)>>>(
            x, graph_ptr, dim, n_iters, w_ih, b_ih, w_hh, b_hh, save, out);
    else
        set2set_fwd_k<false><<<static_cast<unsigned>(n_graphs), 256, 0, as_stream(stream)>>>(
            x, graph_ptr, dim, n_iters, w_ih, b_ih, w_hh, b_hh, save, out);
    return launch_status();
}

extern "C" int scgib_set2set_bwd(const float *x, const int32_t *graph_ptr, int64_t n_graphs,
                                 int32_t dim, int32_t n_iters, const float *w_ih,
                                 const float *w_hh, const float *save, const float *g_out,
                                 float *dx, int64_t n_rows, float *dgates, float *dw_ih,
                                 float *dw_hh, float *db_ih, float *db_hh,
                                 scgib_stream_t stream) {
    if (n_graphs < 0 || dim < 1 || dim > kS2SMaxD || n_iters < 1 || n_rows < 0)
        return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    // the four weight gradients all NULL: the data gradient only (dgates kept
    // for a later scgib_set2set_wgrad)
    const bool wg = dw_ih || dw_hh || db_ih || db_hh;
    if (!x || !graph_ptr || !w_ih || !w_hh || !save || !g_out || !dx || !dgates ||
        (wg && (!dw_ih || !dw_hh || !db_ih || !db_hh)))
        return SCGIB_EINVAL;
    hipStream_t st = as_stream(stream);
    const int64_t tail = (n_rows * dim + 256 * 16 - 1) / (256 * 16);  // padding-zero blocks
    const int64_t extra = tail < 1 ? 1 : (tail > 256 ? 256 : tail);
    if (dim == kS2SMaxD)
        set2set_bwd_k<true><<<static_cast<unsigned>(n_graphs + extra), 256, 0, st>>>(
            x, graph_ptr, n_graphs, dim, n_iters, w_ih, w_hh, save, g_out, dx, dgates, n_rows);
    else
        set2set_bwd_k<false><<<static_cast<unsigned>(n_graphs + extra), 256, 0, st>>>(
            x, graph_ptr, n_graphs, dim, n_iters, w_ih, w_hh, save, g_out, dx, dgates, n_rows);
    int rc = launch_status();
    if (rc != SCGIB_OK || !wg) return rc;
    set2set_wgrad_k<<<static_cast<unsigned>(3 * dim + 1), 256, 0, st>>>(
        save, dgates, n_graphs * n_iters, dim, dw_ih, dw_hh, db_ih, db_hh);
    return launch_status();
}

extern "C" int scgib_set2set_wgrad(const float *save, const float *dgates, int64_t n_graphs,
                                   int32_t dim, int32_t n_iters, float *dw_ih, float *dw_hh,
                                   float *db_ih, float *db_hh, scgib_stream_t stream) {
    if (n_graphs < 0 || dim < 1 || dim > kS2SMaxD || n_iters < 1) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (!save || !dgates || !dw_ih || !dw_hh || !db_ih || !db_hh) return SCGIB_EINVAL;
    set2set_wgrad_k<<<static_cast<unsigned>(3 * dim + 1), 256, 0, as_stream(stream)>>>(
        save, dgates, n_graphs * n_iters, dim, dw_ih, dw_hh, db_ih, db_hh);
    return launch_status();
}

#ifdef SCGIB_TRACE
// debug build only: this file's own g_trace (see common.h; scgib_trace_set)
extern "C" int scgib_trace_set_set2set(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif
