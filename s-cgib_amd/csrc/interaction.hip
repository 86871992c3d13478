// Core <-> subgraph interaction, fused (gfx950): compression (per-graph
// compressor BatchNorm, Gumbel gate, noise injection, last-graph KL) and the
// attention-based interaction, one wavefront per molecule.
//
// Reference: models.py:595-604 (compress), :631-660 (compression loop),
// :714-716 / :732-733 (sum_nodes readouts), :729-749 (attention loop).  The
// reference runs two Python loops over the B graphs of a batch (~15 tiny ops
// each, plus a host->device copy of the gate noise per graph); here the B
// graphs are B independent wavefronts of one launch.
//
// Lane mapping inside the wavefront: lane = 16 q + c4.  Row group q (0..3)
// takes rows r0+q, r0+q+4, ...; lane c4 (0..15) holds hidden channels
// 4c4..4c4+3 as a float4.  So every wave instruction touches four node rows
// with 16-B-per-lane coalesced accesses (4 x 256 B), a dot product over the
// 64 channels of a row is a 16-lane butterfly (red16), and a per-channel
// statistic over the graph's rows is a per-lane float4 accumulator folded
// across the four row groups at the end (red_q).  Every shuffle is executed
// by all 64 lanes (rows past the end are masked, not skipped), so the
// butterflies stay well defined.
//
// The attention logit keeps the z-bar half (w_att[0:64] . z1_i + b_att),
// which is constant per graph and cancels in the softmax:
// computing it costs one red16 per graph and keeps the parameter gradients
// identical in exact arithmetic to the reference's.
//
// Latency-bound VALU/shuffle work (a few hundred FLOP per row): no MFMA.
#include "common.h"
#include "running_update.h"

namespace scgib {

constexpr float kKlEps = 1e-7f;  // models.py:632
// (bias - (1 - bias)) and (1 - bias) with bias = 0.0001 (models.py:598) are
// evaluated in double by Python and rounded to fp32 by torch, as here.
constexpr float kGateScale = static_cast<float>(0.0001 - (1.0 - 0.0001));
constexpr float kGateShift = static_cast<float>(1.0 - 0.0001);

// stats slab layout per graph (SCGIB_STATS_STRIDE floats)
enum : int {
    kStMeanT = 0,      // compressor-BN batch mean of t             [64]
    kStSsqT = 64,      // centred sum of squares of t               [64]
    kStMu = 128,       // std_mean(f).mean                         [64]
    kStSigma = 192,    // std_mean(f).std (unbiased)               [64]
    kStSoftMax = 256,  // softmax max M (of the logits without the z-bar constant)
    kStSoftSum = 257,  // softmax denominator S (relative to M)
    kStConst = 258,    // z-bar logit constant w_lo . z1 + b (cancels in the softmax)
};
// pgrad slab layout per graph (SCGIB_PGRAD_STRIDE floats)
enum : int { kPgW2 = 0, kPgB2 = 64, kPgGamma = 65, kPgBeta = 129, kPgWatt = 193, kPgBatt = 321 };

__device__ __forceinline__ float red16(float v) {
    v += __shfl_xor(v, 1, kWave);
    v += __shfl_xor(v, 2, kWave);
    v += __shfl_xor(v, 4, kWave);
    v += __shfl_xor(v, 8, kWave);
    return v;
}

__device__ __forceinline__ float red_q(float v) {
    v += __shfl_xor(v, 16, kWave);
    v += __shfl_xor(v, 32, kWave);
    return v;
}

__device__ __forceinline__ float4 red_q4(float4 v) {
    return make_float4(red_q(v.x), red_q(v.y), red_q(v.z), red_q(v.w));
}

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }
__device__ __forceinline__ void st4(float *p, float4 v) { *reinterpret_cast<float4 *>(p) = v; }
__device__ __forceinline__ float4 f4(float a) { return make_float4(a, a, a, a); }
__device__ __forceinline__ float4 operator+(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 operator-(float4 a, float4 b) { return make_float4(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
__device__ __forceinline__ float4 operator*(float4 a, float4 b) { return make_float4(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
__device__ __forceinline__ float4 operator*(float s, float4 a) { return make_float4(s * a.x, s * a.y, s * a.z, s * a.w); }
__device__ __forceinline__ float dot4(float4 a, float4 b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
__device__ __forceinline__ float4 relu4(float4 a) { return make_float4(fmaxf(a.x, 0.f), fmaxf(a.y, 0.f), fmaxf(a.z, 0.f), fmaxf(a.w, 0.f)); }
__device__ __forceinline__ float4 sqrt4(float4 a) { return make_float4(sqrtf(a.x), sqrtf(a.y), sqrtf(a.z), sqrtf(a.w)); }
__device__ __forceinline__ float4 rcp_sqrt4(float4 a) { return make_float4(1.f / sqrtf(a.x), 1.f / sqrtf(a.y), 1.f / sqrtf(a.z), 1.f / sqrtf(a.w)); }

// Rows are processed in chunks of 4 * CH (CH rows per row group): all loads
// of a chunk are issued first at clamped, always-valid rows, then used with
// 0/1 weights (macc: fmaf(x, w, acc) — exact for w = 1, and acc + x * 0 = acc
// for finite x), so a chunk costs one memory latency instead of one per row
// (a load consumed only under `if (row valid)` is sunk into that branch with
// its own s_waitcnt).  Per-row-group accumulation order is unchanged.
constexpr int CH = 8;

__device__ __forceinline__ float4 macc(float4 x, float w, float4 acc) {
    return make_float4(fmaf(x.x, w, acc.x), fmaf(x.y, w, acc.y), fmaf(x.z, w, acc.z),
                       fmaf(x.w, w, acc.w));
}

__device__ __forceinline__ float gate_lambda(float u, float p) {
    const float e = kGateScale * u + kGateShift;
    const float g = logf(e) - logf(1.f - e);
    return 1.f / (1.f + expf(-(g + p)));
}

// Device noise (pretraining with noise=None): the reference's torch.rand
// draws (gate u [n,1], models.py:599; feature u [n,64], :650) are replaced by
// counter-based Philox4x32-10 uniforms keyed by a device seed and a per-launch
// offset (NoiseGen): gate of row r = word 0 of counter (r, 16, offset),
// channels 4c..4c+3 = counter (r, c, offset).  noise_uniform_k writes them to
// u_gate / u_feat, which the interaction then reads like explicit noise; it
// runs on the core encoder's stream, off the critical path.  Its last
// workgroup advances the offset, so every launch / graph replay draws fresh
// noise.
struct NoiseGen {
    uint32_t key0, key1, off0, off1;
};

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
        const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
        c = make_uint4(hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0);
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

__device__ __forceinline__ float u01(uint32_t x) { return static_cast<float>(x >> 8) * (1.f / 16777216.f); }

__device__ __forceinline__ float noise_gate(const NoiseGen &ng, int64_t r) {
    return u01(philox4x32_10(make_uint4(static_cast<uint32_t>(r), 16u, ng.off0, ng.off1), ng.key0, ng.key1).x);
}

__device__ __forceinline__ float4 noise_feat(const NoiseGen &ng, int64_t r, int c4) {
    const uint4 v = philox4x32_10(make_uint4(static_cast<uint32_t>(r), static_cast<uint32_t>(c4), ng.off0, ng.off1),
                                  ng.key0, ng.key1);
    return make_float4(u01(v.x), u01(v.y), u01(v.z), u01(v.w));
}


// one thread per (row, channel quad); 256 threads = 16 rows per workgroup per
// pass, grid-stride over at most kNoiseWG workgroups.  The bench's step
// draws one step ahead (ops.NoisePrefetch), at the end of the backward's
// core chain beside the ego chain's last layers: 256 workgroups there
// (B = 512: 588 row groups in 3 passes instead of 10) measured 0.3872–0.3882
// vs 0.3886–0.3902 ms per step, B = 32 unchanged (profiles/r06_noise/).
// Build-time A/B hook SCGIB_NOISE_WG: the draws depend only on (row, quad,
// offset), so the grid does not change a bit.
#ifndef SCGIB_NOISE_WG
#define SCGIB_NOISE_WG 256
#endif
constexpr int kNoiseWG = SCGIB_NOISE_WG;
__global__ __launch_bounds__(256) void noise_uniform_k(float *__restrict__ u_gate,
                                                       float *__restrict__ u_feat, int64_t n,
                                                       uint64_t *__restrict__ rng,
                                                       unsigned *__restrict__ cnt) {
    const uint64_t seed = rng[0];
    const uint64_t off = __hip_atomic_load(rng + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const NoiseGen ng{static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32),
                      static_cast<uint32_t>(off), static_cast<uint32_t>(off >> 32)};
    const int c4 = threadIdx.x & 15;
    for (int64_t r = static_cast<int64_t>(blockIdx.x) * 16 + (threadIdx.x >> 4); r < n;
         r += static_cast<int64_t>(gridDim.x) * 16) {
        st4(u_feat + r * 64 + 4 * c4, noise_feat(ng, r, c4));
        if (c4 == 0) u_gate[r] = noise_gate(ng, r);
    }
    // every workgroup has read the offset: the last one advances it
    if (block_arrive(cnt, gridDim.x) && threadIdx.x == 0) {
        __hip_atomic_store(rng + 1, off + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *cnt = 0u;
    }
}

struct Lanes {
    int q, c4, ch;  // row group, channel quad, first channel
};

__device__ __forceinline__ Lanes lanes() {
    const int l = threadIdx.x & 63;
    return {l >> 4, l & 15, (l & 15) * 4};
}

// Waves per graph (build-time A/B hook SCGIB_INT_NW): a graph's rows are
// spread over 4 NW row groups (row group qg = 4 wave + lane / 16), CH / NW
// rows per lane per 32-row chunk; sums over row groups go through the wave's
// shuffles, then (NW > 1) one LDS exchange in fixed wave order.  The kernels
// are latency-bound per wave (phase trace: two ~5 us passes of dependent
// VALU / shuffle chains at NW = 1), so a shorter chain per wave is what pays.
#ifndef SCGIB_INT_NW
#define SCGIB_INT_NW 4
#endif
constexpr int kIntNW = SCGIB_INT_NW;
static_assert(kIntNW == 1 || kIntNW == 2 || kIntNW == 4, "waves per graph");

// cross-wave sums of per-wave float4 totals (identical in every lane of a
// wave's channel quad): v[i] <- sum over waves 0..NW-1, fixed order
template <int NW, int K>
__device__ __forceinline__ void wave_sum4(float4 (&v)[K], float4 (*sx)[4][16], int w, int q, int c4) {
    if constexpr (NW > 1) {
        if (q == 0) {
#pragma unroll
            for (int i = 0; i < K; ++i) sx[i][w][c4] = v[i];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < K; ++i) {
            float4 a = sx[i][0][c4];
#pragma unroll
            for (int k = 1; k < NW; ++k) a = a + sx[i][k][c4];
            v[i] = a;
        }
        __syncthreads();
    }
}

template <int NW>
__device__ __forceinline__ float wave_sum1(float v, float *sx, int w) {
    if constexpr (NW > 1) {
        if ((threadIdx.x & 63) == 0) sx[w] = v;
        __syncthreads();
        float a = sx[0];
#pragma unroll
        for (int k = 1; k < NW; ++k) a += sx[k];
        __syncthreads();
        return a;
    }
    return v;
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void interaction_fwd_k(
    const float *__restrict__ f, const float *__restrict__ t, const float *__restrict__ s,
    const float *__restrict__ u_gate, const float *__restrict__ u_feat,
    const int32_t *__restrict__ gptr, int64_t B, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ rmean,
    const float *__restrict__ rvar, float bn_eps, int training, const float *__restrict__ w2,
    const float *__restrict__ b2p, const float *__restrict__ watt,
    const float *__restrict__ battp, float *__restrict__ im, float *__restrict__ z1,
    float *__restrict__ z2, float *__restrict__ lam, float *__restrict__ logit,
    float *__restrict__ stats, float *__restrict__ kl, float *__restrict__ kl_mean,
    int64_t n_rows_cap, int pad) {
    constexpr int RS = 4 * NW, CN = CH / NW;  // row stride, rows per lane per chunk
    static_assert(RS * CN == 4 * CH, "32-row chunks");
    __shared__ float4 sX[6][4][16];  // cross-wave exchanges (NW > 1)
    __shared__ float sM[4], sS[4], sK[4];
    const Lanes L = lanes();
    const int w = threadIdx.x >> 6, qg = 4 * w + L.q;
    const int64_t gi = blockIdx.x;
    SCGIB_MARK(0);
    if (gi >= B) {  // padding blocks: zero rows [N, n_rows_cap) of im, lam, logit
        const int64_t r_beg = gptr[B];
        for (int64_t r = r_beg + (gi - B); r < n_rows_cap; r += gridDim.x - B) {
            if (threadIdx.x < 32) st4(im + r * 128 + threadIdx.x * 4, f4(0.f));
            if (threadIdx.x == 0) { lam[r] = 0.f; logit[r] = 0.f; }
        }
        return;
    }
    const int64_t r0 = gptr[gi], r1 = gptr[gi + 1];
    const int n = static_cast<int>(r1 - r0);
    if (n <= 0) {
        if (qg == 0) {
            st4(z1 + gi * 64 + L.ch, f4(0.f));
            st4(z2 + gi * 64 + L.ch, f4(0.f));
        }
        if (gi == B - 1 && kl_mean && threadIdx.x == 0) *kl_mean = 0.f;
        return;
    }
    SCGIB_MARK(1);
    // Two load passes (the first chunk of CN rows per row group — a whole
    // typical molecule — stays in registers between them):
    //   pass A: f / t sums and shifted second moments; the attention logit
    //           w_hi . s_v and its online softmax (the per-graph constant
    //           w_lo . z-bar + b cancels in the softmax, so the stored logit,
    //           max and sum exclude it; the backward only uses differences);
    //   pass B: compressor logit p, gate lambda, noisy features, the attended
    //           s rows, z-bar, and (last graph) the KL sum of squares;
    //   KL store pass for the last graph (lambda of the first chunk from
    //   registers, later chunks recomputed).
    const float4 f0 = ld4(f + r0 * 64 + L.ch), t0 = ld4(t + r0 * 64 + L.ch);
    const float4 whi = ld4(watt + 64 + L.ch);
    float4 acc6[6] = {f4(0.f), f4(0.f), f4(0.f), f4(0.f), f4(0.f), f4(0.f)};  // zf zt sf st qf qt
    float M = -INFINITY, S = 0.f;  // per row group, merged below
    float4 fk[CN], tk[CN], sk[CN];  // first chunk, kept
    auto pass_a = [&](int64_t cb, float4 *fv, float4 *tv, float4 *sv) {
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j, rr = r < r1 ? r : r0;
            fv[j] = ld4(f + rr * 64 + L.ch);
            tv[j] = ld4(t + rr * 64 + L.ch);
            sv[j] = ld4(s + rr * 64 + L.ch);
        }
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j;
            const float wt = r < r1 ? 1.f : 0.f;
            acc6[0] = macc(fv[j], wt, acc6[0]);
            acc6[1] = macc(tv[j], wt, acc6[1]);
            const float4 df = fv[j] - f0, dt = tv[j] - t0;
            acc6[2] = macc(df, wt, acc6[2]);
            acc6[3] = macc(dt, wt, acc6[3]);
            acc6[4] = macc(df * df, wt, acc6[4]);
            acc6[5] = macc(dt * dt, wt, acc6[5]);
            const float lg = red16(dot4(whi, sv[j]));
            if (r < r1) {
                if (L.c4 == 0) logit[r] = lg;
                const float Mn = fmaxf(M, lg);
                S = S * expf(M - Mn) + expf(lg - Mn);
                M = Mn;
            }
        }
    };
    // the first chunk's noise (independent of pass A): in flight with its rows
    float4 uk[CN];
    float ugk[CN];
#pragma unroll
    for (int j = 0; j < CN; ++j) {
        const int64_t r = r0 + qg + RS * j, rr = r < r1 ? r : r0;
        uk[j] = ld4(u_feat + rr * 64 + L.ch);
        ugk[j] = u_gate[rr];
    }
    pass_a(r0, fk, tk, sk);
    for (int64_t cb = r0 + RS * CN; cb < r1; cb += RS * CN) {
        float4 fv[CN], tv[CN], sv[CN];
        pass_a(cb, fv, tv, sv);
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) acc6[i] = red_q4(acc6[i]);
    wave_sum4<NW>(acc6, sX, w, L.q, L.c4);
#pragma unroll
    for (int off = 16; off <= 32; off <<= 1) {  // merge the wave's four row groups' softmax
        const float Mo = __shfl_xor(M, off, kWave), So = __shfl_xor(S, off, kWave);
        const float Mn = fmaxf(M, Mo);
        S = (S == 0.f ? 0.f : S * expf(M - Mn)) + (So == 0.f ? 0.f : So * expf(Mo - Mn));
        M = Mn;
    }
    if constexpr (NW > 1) {  // ... and the waves', in wave order
        if ((threadIdx.x & 63) == 0) {
            sM[w] = M;
            sS[w] = S;
        }
        __syncthreads();
        M = sM[0];
        S = sS[0];
#pragma unroll
        for (int k = 1; k < NW; ++k) {
            const float Mo = sM[k], So = sS[k], Mn = fmaxf(M, Mo);
            S = (S == 0.f ? 0.f : S * expf(M - Mn)) + (So == 0.f ? 0.f : So * expf(Mo - Mn));
            M = Mn;
        }
    }
    const float4 zf = acc6[0], zt = acc6[1], sf = acc6[2], st = acc6[3], qf = acc6[4], qt = acc6[5];
    SCGIB_MARK(2);
    const float invS = 1.f / S;
    const float inv_n = 1.f / n;
    const float4 mu = inv_n * zf, mt = inv_n * zt;
    // centred sums of squares (shifted formula); n == 1 -> 0 / 0 -> NaN std, as torch
    const float4 cf = qf - inv_n * (sf * sf), ct = qt - inv_n * (st * st);
    const float4 sig = sqrt4(make_float4(fmaxf(cf.x, 0.f), fmaxf(cf.y, 0.f), fmaxf(cf.z, 0.f),
                                         fmaxf(cf.w, 0.f)) * f4(1.f / static_cast<float>(n - 1)));
    const float4 ctp = make_float4(fmaxf(ct.x, 0.f), fmaxf(ct.y, 0.f), fmaxf(ct.z, 0.f), fmaxf(ct.w, 0.f));
    const float4 m_use = training ? mt : ld4(rmean + L.ch);
    const float4 v_use = training ? inv_n * ctp : ld4(rvar + L.ch);
    const float4 rstd = rcp_sqrt4(v_use + f4(bn_eps));
    const float4 gm = ld4(gamma + L.ch), bt = ld4(beta + L.ch), w2c = ld4(w2 + L.ch);
    const float b2 = *b2p;
    float *sl = stats + gi * SCGIB_STATS_STRIDE;
    if (qg == 0) {
        st4(z2 + gi * 64 + L.ch, zf);
        st4(sl + kStMeanT + L.ch, mt);
        st4(sl + kStSsqT + L.ch, ctp);
        st4(sl + kStMu + L.ch, mu);
        st4(sl + kStSigma + L.ch, sig);
    }
    SCGIB_MARK(3);
    // ---- pass B: compressor logit p, gate lambda, noisy features, attention ----
    const bool last = gi == B - 1;
    const float4 se = sig + f4(kKlEps);
    float4 acc2[2] = {f4(0.f), f4(0.f)};  // zacc, qacc
    float lmk[CN];  // first chunk's lambda, kept for the KL store pass
    auto pass_b = [&](int64_t cb, const float4 *fv, const float4 *tv, const float4 *sv,
                      float *lmo, const float4 *upre, const float *gpre) {
        float4 uv[CN];
        float ug[CN];
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j, rr = r < r1 ? r : r0;
            uv[j] = upre ? upre[j] : ld4(u_feat + rr * 64 + L.ch);
            ug[j] = gpre ? gpre[j] : u_gate[rr];
        }
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j;
            const float wt = r < r1 ? 1.f : 0.f;
            const float4 y = gm * ((tv[j] - m_use) * rstd) + bt;
            const float p = red16(dot4(w2c, relu4(y))) + b2;
            const float lm = gate_lambda(ug[j], p), ln = 1.f - lm;
            if (lmo) lmo[j] = lm;
            const float4 nz = (lm * fv[j] + ln * mu) + uv[j] * (ln * sig);
            acc2[0] = macc(nz, wt, acc2[0]);
            if (last) {
                const float4 d = (lm * fv[j] + ln * mu) - mu;
                const float4 z = make_float4(d.x / se.x, d.y / se.y, d.z / se.z, d.w / se.w);
                acc2[1] = macc(z * z, wt, acc2[1]);
            }
            const float lg = red16(dot4(whi, sv[j]));
            if (r < r1) {
                st4(im + r * 128 + L.ch, nz);
                st4(im + r * 128 + 64 + L.ch, (expf(lg - M) * invS) * sv[j]);
                if (L.c4 == 0) lam[r] = lm;
            }
        }
    };
    pass_b(r0, fk, tk, sk, lmk, uk, ugk);
    for (int64_t cb = r0 + RS * CN; cb < r1; cb += RS * CN) {
        float4 fv[CN], tv[CN], sv[CN];
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j, rr = r < r1 ? r : r0;
            fv[j] = ld4(f + rr * 64 + L.ch);
            tv[j] = ld4(t + rr * 64 + L.ch);
            sv[j] = ld4(s + rr * 64 + L.ch);
        }
        pass_b(cb, fv, tv, sv, nullptr, nullptr, nullptr);
    }
    acc2[0] = red_q4(acc2[0]);
    acc2[1] = red_q4(acc2[1]);
    wave_sum4<NW>(acc2, sX, w, L.q, L.c4);  // (qacc: only the last graph uses it)
    const float4 zacc = acc2[0], qacc = acc2[1];
    SCGIB_MARK(4);
    if (qg == 0) st4(z1 + gi * 64 + L.ch, zacc);
    // the z-bar half of the attention logit (constant per graph; kept for the
    // record, the softmax above and its backward do not depend on it)
    const float cst = red16(dot4(ld4(watt + L.ch), zacc)) + *battp;
    // ---- KL of the last graph only, duplicated (models.py:657-659) ----
    if (last) {  // (block-uniform)
        const float4 den = se * se;
        float ksum = 0.f;
        auto kl_store = [&](int64_t cb, const float *lmv) {
#pragma unroll
            for (int j = 0; j < CN; ++j) {
                const int64_t r = cb + qg + RS * j;
                const float4 ns = (1.f - lmv[j]) * sig;
                const float4 nn = ns * ns;
                const float4 v = f4(0.5f) * make_float4(nn.x / den.x, nn.y / den.y, nn.z / den.z,
                                                        nn.w / den.w) + qacc;
                if (r < r1) {
                    if (kl) {
                        st4(kl + (r - r0) * 64 + L.ch, v);
                        st4(kl + (r - r0 + n) * 64 + L.ch, v);
                    }
                    ksum += (v.x + v.y) + (v.z + v.w);
                }
            }
        };
        kl_store(r0, lmk);
        for (int64_t cb = r0 + RS * CN; cb < r1; cb += RS * CN) {
            float4 tv[CN];
            float ug[CN], lmv[CN];
#pragma unroll
            for (int j = 0; j < CN; ++j) {
                const int64_t r = cb + qg + RS * j, rr = r < r1 ? r : r0;
                tv[j] = ld4(t + rr * 64 + L.ch);
                ug[j] = u_gate[rr];
            }
#pragma unroll
            for (int j = 0; j < CN; ++j) {
                const float4 y = gm * ((tv[j] - m_use) * rstd) + bt;
                lmv[j] = gate_lambda(ug[j], red16(dot4(w2c, relu4(y))) + b2);
            }
            kl_store(cb, lmv);
        }
        // mean over the duplicated [2n, 64] tensor == mean over [n, 64]
        ksum = wave_sum1<NW>(red_q(red16(ksum)), sK, w);
        if (kl_mean && threadIdx.x == 0) *kl_mean = ksum / (static_cast<float>(n) * 64.f);
    }
    if (threadIdx.x == 0) {
        sl[kStSoftMax] = M;
        sl[kStSoftSum] = S;
        sl[kStConst] = cst;
    }
    SCGIB_MARK(5);
}

// the compressor BatchNorm's running-stat update (running_update.h)
static_assert(kStMeanT == kRuMeanOff && kStSsqT == kRuSsqOff, "stats slab layout");

__global__ __launch_bounds__(1024) void bn_running_update_k(const scgib_running_update a) {
    running_update_body<1024>(a);
}

template <int NW>
__global__ __launch_bounds__(64 * NW) void interaction_bwd_k(
    const float *__restrict__ g_im, const float *__restrict__ g_z1,
    const float *__restrict__ g_z2, const float *__restrict__ g_kl,
    const float *__restrict__ f, const float *__restrict__ t, const float *__restrict__ s,
    const float *__restrict__ u_feat, const int32_t *__restrict__ gptr, int64_t B,
    const float *__restrict__ gamma, const float *__restrict__ beta,
    const float *__restrict__ rmean, const float *__restrict__ rvar, float bn_eps,
    int training, const float *__restrict__ w2, const float *__restrict__ watt,
    const float *__restrict__ z1, const float *__restrict__ lam,
    const float *__restrict__ logit, const float *__restrict__ stats, float *__restrict__ df,
    float *__restrict__ dt, float *__restrict__ ds, float *__restrict__ pgrad,
    const float *__restrict__ g_klmean, int64_t n_rows_cap) {
    constexpr int RS = 4 * NW, CN = CH / NW;  // row stride, rows per lane per chunk
    __shared__ float4 sX[6][4][16];  // cross-wave exchanges (NW > 1)
    __shared__ float sK[4];
    const Lanes L = lanes();
    const int wvi = threadIdx.x >> 6, qg = 4 * wvi + L.q;
    const int64_t gi = blockIdx.x;
    if (gi >= B) {  // padding blocks: zero rows [N, n_rows_cap) of df, dt, ds
        const int64_t r_beg = gptr[B];
        for (int64_t r = r_beg + (gi - B); r < n_rows_cap; r += gridDim.x - B) {
            if (threadIdx.x < 16) {
                st4(df + r * 64 + threadIdx.x * 4, f4(0.f));
                st4(dt + r * 64 + threadIdx.x * 4, f4(0.f));
                st4(ds + r * 64 + threadIdx.x * 4, f4(0.f));
            }
        }
        return;
    }
    SCGIB_MARK(0);
    const int64_t r0 = gptr[gi], r1 = gptr[gi + 1];
    const int n = static_cast<int>(r1 - r0);
    float *pg = pgrad + gi * SCGIB_PGRAD_STRIDE;
    if (n <= 0) {
        for (int j = threadIdx.x; j < SCGIB_PGRAD_STRIDE; j += 64 * NW) pg[j] = 0.f;
        return;
    }
    const float *sl = stats + gi * SCGIB_STATS_STRIDE;
    const float inv_n = 1.f / n;
    const float4 mt = ld4(sl + kStMeanT + L.ch), ssq = ld4(sl + kStSsqT + L.ch);
    const float4 mu = ld4(sl + kStMu + L.ch), sig = ld4(sl + kStSigma + L.ch);
    const float M = sl[kStSoftMax], invS = 1.f / sl[kStSoftSum];
    const float4 m_use = training ? mt : ld4(rmean + L.ch);
    const float4 v_use = training ? inv_n * ssq : ld4(rvar + L.ch);
    const float4 rstd = rcp_sqrt4(v_use + f4(bn_eps));
    const float4 gm = ld4(gamma + L.ch), bt = ld4(beta + L.ch), w2c = ld4(w2 + L.ch);
    const float4 wlo = ld4(watt + L.ch), whi = ld4(watt + 64 + L.ch), zb = ld4(z1 + gi * 64 + L.ch);
    SCGIB_MARK(1);

    // ---- attention backward: a_v = alpha_v s_v, alpha = softmax(logit) ----
    // The first chunk (all rows of a typical molecule's ego-net batch slice)
    // stays in registers across the passes; later chunks are re-loaded.
    auto att_load = [&](int64_t cb, float4 *ga, float4 *sv, float *lg) {
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j, rr = r < r1 ? r : r0;
            ga[j] = ld4(g_im + rr * 128 + 64 + L.ch);
            sv[j] = ld4(s + rr * 64 + L.ch);
            lg[j] = logit[rr];
        }
    };
    float4 ga0[CN], sv0[CN];
    float lg0[CN];
    att_load(r0, ga0, sv0, lg0);
    float sa = 0.f;  // sum alpha * dalpha of this row group (uniform over its lanes)
    auto att_sum = [&](int64_t cb, const float4 *ga, const float4 *sv, const float *lg) {
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const float da = red16(dot4(ga[j], sv[j]));
            sa = fmaf(expf(lg[j] - M) * invS * da, cb + qg + RS * j < r1 ? 1.f : 0.f, sa);
        }
    };
    att_sum(r0, ga0, sv0, lg0);
    for (int64_t cb = r0 + RS * CN; cb < r1; cb += RS * CN) {
        float4 ga[CN], sv[CN];
        float lg[CN];
        att_load(cb, ga, sv, lg);
        att_sum(cb, ga, sv, lg);
    }
    const float SA = wave_sum1<NW>(red_q(sa), sK, wvi);
    float4 dwhi = f4(0.f);
    float dcq = 0.f;
    auto att_grad = [&](int64_t cb, const float4 *ga, const float4 *sv, const float *lg) {
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j;
            const float w = r < r1 ? 1.f : 0.f;
            const float da = red16(dot4(ga[j], sv[j]));
            const float al = expf(lg[j] - M) * invS;
            const float dl = al * (da - SA);
            if (r < r1) st4(ds + r * 64 + L.ch, al * ga[j] + dl * whi);
            dwhi = macc(dl * sv[j], w, dwhi);
            dcq = fmaf(dl, w, dcq);
        }
    };
    att_grad(r0, ga0, sv0, lg0);
    for (int64_t cb = r0 + RS * CN; cb < r1; cb += RS * CN) {
        float4 ga[CN], sv[CN];
        float lg[CN];
        att_load(cb, ga, sv, lg);
        att_grad(cb, ga, sv, lg);
    }
    float4 dwv[1] = {red_q4(dwhi)};
    wave_sum4<NW>(dwv, sX, wvi, L.q, L.c4);
    dwhi = dwv[0];
    const float dc = wave_sum1<NW>(red_q(dcq), sK, wvi);
    SCGIB_MARK(2);
    // (a NULL g_z1 / g_z2: the readouts feed no loss, e.g. in the fine-tune head)
    const float4 gb = (g_z1 ? ld4(g_z1 + gi * 64 + L.ch) : f4(0.f)) + dc * wlo;  // d z-bar -> every node's noisy
    const float4 gz2 = g_z2 ? ld4(g_z2 + gi * 64 + L.ch) : f4(0.f);  // d readout(f) -> every node's f

    // ---- KL (last graph) ----
    // gradient of the KL term: a tensor g_kl [2n, 64] (both copies), or the
    // scalar gradient of KL_Loss = mean(KL_tensor): g / (2n 64) per entry
    const bool has_kl = (g_kl != nullptr || g_klmean != nullptr) && (gi == B - 1);
    const float gk_uniform = g_klmean ? *g_klmean / (static_cast<float>(n) * 64.f) : 0.f;
    float4 Gc = f4(0.f);
    if (has_kl && g_kl) {
        for (int base = 0; base < n; base += RS) {
            const int rl = base + qg;
            if (rl < n) Gc = Gc + ld4(g_kl + rl * 64 + L.ch) + ld4(g_kl + (rl + n) * 64 + L.ch);
        }
        float4 gv[1] = {red_q4(Gc)};
        wave_sum4<NW>(gv, sX, wvi, L.q, L.c4);  // (block-uniform branch: the last graph)
        Gc = gv[0];
    }
    if (has_kl && !g_kl) Gc = f4(gk_uniform * n);
    const float4 se = sig + f4(kKlEps);
    const float4 inv2 = make_float4(1.f / (se.x * se.x), 1.f / (se.y * se.y), 1.f / (se.z * se.z),
                                    1.f / (se.w * se.w));

    // ---- compression backward ----
    float4 dw2 = f4(0.f), dg = f4(0.f), dbe = f4(0.f);
    float db2q = 0.f;
    float4 dy0[CN], xh0[CN];  // first chunk's BN-input gradient and normalised input
    auto comp = [&](int64_t cb, float4 *dyo, float4 *xho) {
        float lm[CN];
        float4 fv[CN], gn[CN], uv[CN], tv[CN], gk[CN];
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j, rr = r < r1 ? r : r0;
            lm[j] = lam[rr];
            fv[j] = ld4(f + rr * 64 + L.ch);
            gn[j] = ld4(g_im + rr * 128 + L.ch);
            uv[j] = ld4(u_feat + rr * 64 + L.ch);
            tv[j] = ld4(t + rr * 64 + L.ch);
            if (has_kl && g_kl) {
                const int rl = static_cast<int>(rr - r0);
                gk[j] = ld4(g_kl + rl * 64 + L.ch) + ld4(g_kl + (rl + n) * 64 + L.ch);
            } else {
                gk[j] = f4(gk_uniform);
            }
        }
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j;
            const float w = r < r1 ? 1.f : 0.f;
            const float4 g = gn[j] + gb;
            const float4 fm = fv[j] - mu;
            float part = dot4(g, fm - uv[j] * sig);
            float4 dfv = lm[j] * g + gz2;
            if (has_kl) {
                part += dot4(gk[j], (-(1.f - lm[j])) * (sig * sig * inv2)) +
                        dot4(Gc, (2.f * lm[j]) * (fm * fm * inv2));
                dfv = dfv + (2.f * lm[j] * lm[j]) * (Gc * fm * inv2);
            }
            const float dp = red16(part) * lm[j] * (1.f - lm[j]);
            const float4 xh = (tv[j] - m_use) * rstd;
            const float4 y = gm * xh + bt;
            dw2 = macc(dp * relu4(y), w, dw2);
            db2q = fmaf(dp, w, db2q);
            const float4 dy = make_float4(y.x > 0.f ? dp * w2c.x : 0.f, y.y > 0.f ? dp * w2c.y : 0.f,
                                          y.z > 0.f ? dp * w2c.z : 0.f, y.w > 0.f ? dp * w2c.w : 0.f);
            dg = macc(dy * xh, w, dg);
            dbe = macc(dy, w, dbe);
            if (dyo) {
                dyo[j] = dy;
                xho[j] = xh;
            }
            if (r < r1) {
                st4(df + r * 64 + L.ch, dfv);
                if (!dyo) st4(dt + r * 64 + L.ch, dy);
            }
        }
    };
    comp(r0, dy0, xh0);
    for (int64_t cb = r0 + RS * CN; cb < r1; cb += RS * CN) comp(cb, nullptr, nullptr);
    float4 dv[3] = {red_q4(dw2), red_q4(dg), red_q4(dbe)};
    wave_sum4<NW>(dv, sX, wvi, L.q, L.c4);
    dw2 = dv[0];
    dg = dv[1];
    dbe = dv[2];
    const float db2 = wave_sum1<NW>(red_q(db2q), sK, wvi);
    SCGIB_MARK(3);
    // BatchNorm backward (this graph's batch statistics, or running stats);
    // chunk 0 from registers, later chunks re-read the dt entries this lane wrote
    const float4 gr = gm * rstd;
    auto bn_bwd = [&](int64_t cb, const float4 *dy, const float4 *xh) {
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j;
            if (r < r1)
                st4(dt + r * 64 + L.ch,
                    training ? gr * (dy[j] - inv_n * dbe - xh[j] * (inv_n * dg)) : gr * dy[j]);
        }
    };
    bn_bwd(r0, dy0, xh0);
    for (int64_t cb = r0 + RS * CN; cb < r1; cb += RS * CN) {
        float4 dy[CN], xh[CN];
#pragma unroll
        for (int j = 0; j < CN; ++j) {
            const int64_t r = cb + qg + RS * j, rr = r < r1 ? r : r0;
            dy[j] = ld4(dt + rr * 64 + L.ch);  // valid rows: written by this lane above
            xh[j] = (ld4(t + rr * 64 + L.ch) - m_use) * rstd;
        }
        bn_bwd(cb, dy, xh);
    }
    if (qg == 0) {
        st4(pg + kPgW2 + L.ch, dw2);
        st4(pg + kPgGamma + L.ch, dg);
        st4(pg + kPgBeta + L.ch, dbe);
        st4(pg + kPgWatt + L.ch, dc * zb);
        st4(pg + kPgWatt + 64 + L.ch, dwhi);
    }
    if (threadIdx.x == 0) {
        pg[kPgB2] = db2;
        pg[kPgBatt] = dc;
        pg[SCGIB_PGRAD_STRIDE - 2] = 0.f;
        pg[SCGIB_PGRAD_STRIDE - 1] = 0.f;
    }
    SCGIB_MARK(4);
}

}  // namespace scgib

using namespace scgib;

extern "C" int scgib_interaction_fwd(
    const float *f, const float *t, const float *s, const float *u_gate, const float *u_feat,
    const int32_t *graph_ptr, int64_t n_graphs, int64_t n_nodes, const float *bn_gamma,
    const float *bn_beta, const float *bn_running_mean, const float *bn_running_var,
    float bn_eps, int32_t training, const float *w2, const float *b2, const float *w_att,
    const float *b_att, float *im, float *z1, float *z2, float *lam, float *logit,
    float *stats, float *kl_tensor, float *kl_mean, int32_t pad_rows, scgib_stream_t stream) {
    if (n_graphs < 0 || n_nodes < 0) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (n_graphs > 0x7fffffff) return SCGIB_EUNSUPPORTED;
    if (!graph_ptr || !bn_gamma || !bn_beta || !w2 || !b2 || !w_att || !b_att || !z1 ||
        !z2 || !stats || (!kl_tensor && !kl_mean))
        return SCGIB_EINVAL;
    if (n_nodes > 0 && (!f || !t || !s || !u_gate || !u_feat || !im || !lam || !logit))
        return SCGIB_EINVAL;
    if (!training && (!bn_running_mean || !bn_running_var)) return SCGIB_EINVAL;
    const unsigned grid = static_cast<unsigned>(n_graphs + (pad_rows ? 64 : 0));
    interaction_fwd_k<kIntNW><<<dim3(grid), 64 * kIntNW, 0, as_stream(stream)>>>(
        f, t, s, u_gate, u_feat, graph_ptr, n_graphs, bn_gamma, bn_beta, bn_running_mean,
        bn_running_var, bn_eps, training, w2, b2, w_att, b_att, im, z1, z2, lam, logit, stats,
        kl_tensor, kl_mean, n_nodes, pad_rows);
    return launch_status();
}

extern "C" int scgib_noise_uniform(float *u_gate, float *u_feat, int64_t n_rows,
                                   uint64_t *rng_state, uint32_t *counter,
                                   scgib_stream_t stream) {
    if (n_rows < 0) return SCGIB_EINVAL;
    if (n_rows == 0) return SCGIB_OK;
    if (!u_gate || !u_feat || !rng_state || !counter) return SCGIB_EINVAL;
    if (n_rows > 0xffffffffLL) return SCGIB_EUNSUPPORTED;
    const int64_t wg = (n_rows + 15) / 16;
    noise_uniform_k<<<dim3(static_cast<unsigned>(wg < kNoiseWG ? wg : kNoiseWG)), 256, 0,
                      as_stream(stream)>>>(
        u_gate, u_feat, n_rows, rng_state, counter);
    return launch_status();
}

extern "C" int scgib_bn_running_update(const float *stats, const int32_t *graph_ptr,
                                       int64_t n_graphs, float momentum, float *running_mean,
                                       float *running_var, int64_t *num_batches_tracked,
                                       scgib_stream_t stream) {
    if (n_graphs < 0) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (!stats || !graph_ptr || !running_mean || !running_var) return SCGIB_EINVAL;
    bn_running_update_k<<<1, 1024, 0, as_stream(stream)>>>(scgib_running_update{
        stats, graph_ptr, n_graphs, momentum, running_mean, running_var, num_batches_tracked});
    return launch_status();
}

extern "C" int scgib_interaction_bwd(
    const float *g_im, const float *g_z1, const float *g_z2, const float *g_kl, const float *f,
    const float *t, const float *s, const float *u_feat, const int32_t *graph_ptr,
    int64_t n_graphs, int64_t n_nodes, const float *bn_gamma, const float *bn_beta,
    const float *bn_running_mean, const float *bn_running_var, float bn_eps, int32_t training,
    const float *w2, const float *w_att, const float *z1, const float *lam,
    const float *logit, const float *stats, float *df, float *dt, float *ds, float *pgrad,
    const float *g_klmean, int32_t pad_rows, float *pgrad_total, scgib_stream_t stream) {
    if (n_graphs < 0 || n_nodes < 0) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (n_graphs > 0x7fffffff) return SCGIB_EUNSUPPORTED;
    if (!graph_ptr || !bn_gamma || !bn_beta || !w2 || !w_att || !z1 || !stats || !pgrad)
        return SCGIB_EINVAL;
    if (n_nodes > 0 && (!g_im || !f || !t || !s || !u_feat || !lam || !logit || !df || !dt ||
                        !ds))
        return SCGIB_EINVAL;
    if (!training && (!bn_running_mean || !bn_running_var)) return SCGIB_EINVAL;
    const unsigned grid = static_cast<unsigned>(n_graphs + (pad_rows ? 64 : 0));
    interaction_bwd_k<kIntNW><<<dim3(grid), 64 * kIntNW, 0, as_stream(stream)>>>(
        g_im, g_z1, g_z2, g_kl, f, t, s, u_feat, graph_ptr, n_graphs, bn_gamma, bn_beta,
        bn_running_mean, bn_running_var, bn_eps, training, w2, w_att, z1, lam, logit, stats,
        df, dt, ds, pgrad, g_klmean, n_nodes);
    if (pgrad_total) {
        const int rc = launch_status();
        if (rc != SCGIB_OK) return rc;
        return launch_slab_reduce(pgrad, static_cast<int>(n_graphs), SCGIB_PGRAD_STRIDE,
                                  pgrad_total, as_stream(stream));
    }
    return launch_status();
}

#ifdef SCGIB_TRACE
// debug build only: this file's own g_trace (see common.h; scgib_trace_set)
extern "C" int scgib_trace_set_interaction(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif
