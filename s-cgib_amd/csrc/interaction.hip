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
// Mapping: lane c of the wavefront owns hidden channel c (hidden = 64 =
// wavefront width), so every per-node row access is one 256-B coalesced
// load, every per-channel statistic (means, stds, BN stats, readouts) lives
// in a register, and every per-node dot product over channels (compressor
// output p, attention logit) is one butterfly wave_sum.  Graph rows are
// re-read from L1/L2 between passes (a molecule is a few KB).
//
// The attention logit keeps the z-bar half (w_att[0:64] . z1_i + b_att),
// which is constant per graph and cancels in the softmax:
// computing it costs one wave_sum per graph and keeps the parameter
// gradients identical in exact arithmetic to the reference's.
//
// This is latency-bound VALU/shuffle work (a few hundred FLOP per row), not
// GEMM-shaped: no MFMA.
#include "common.h"

namespace scgib {

constexpr float kKlEps = 1e-7f;             // models.py:632
constexpr float kGateLo = 0.0001f;          // models.py:598: bias = 0.0 + 0.0001
// (bias - (1 - bias)) and (1 - bias) are evaluated in double by Python and
// rounded to fp32 by torch's scalar multiply/add, as here.
constexpr float kGateScale = static_cast<float>(0.0001 - (1.0 - 0.0001));
constexpr float kGateShift = static_cast<float>(1.0 - 0.0001);

// stats slab layout per graph (SCGIB_STATS_STRIDE floats)
enum : int {
    kStMeanT = 0,     // compressor-BN batch mean of t            [64]
    kStSsqT = 64,     // centred sum of squares of t              [64]
    kStMu = 128,      // std_mean(f).mean                        [64]
    kStSigma = 192,   // std_mean(f).std (unbiased)              [64]
    kStSoftMax = 256, // softmax running max M
    kStSoftSum = 257, // softmax denominator S (relative to M)
    kStConst = 258,   // z-bar logit constant
};
// pgrad slab layout per graph (SCGIB_PGRAD_STRIDE floats)
enum : int { kPgW2 = 0, kPgB2 = 64, kPgGamma = 65, kPgBeta = 129, kPgWatt = 193, kPgBatt = 321 };

struct GraphCtx {
    int64_t r0, r1;
    int n;
    float mt, rstd;  // BN stats used for normalisation (batch or running)
    float mu, sig;   // std_mean of f
};

__device__ __forceinline__ float gate_lambda(float u, float p) {
    const float e = kGateScale * u + kGateShift;
    const float g = logf(e) - logf(1.f - e);
    return 1.f / (1.f + expf(-(g + p)));
}

__global__ __launch_bounds__(256) void interaction_fwd_k(
    const float *__restrict__ f, const float *__restrict__ t, const float *__restrict__ s,
    const float *__restrict__ u_gate, const float *__restrict__ u_feat,
    const int32_t *__restrict__ gptr, int64_t B, const float *__restrict__ gamma,
    const float *__restrict__ beta, const float *__restrict__ rmean,
    const float *__restrict__ rvar, float bn_eps, int training, const float *__restrict__ w2,
    const float *__restrict__ b2p, const float *__restrict__ watt,
    const float *__restrict__ battp, float *__restrict__ im, float *__restrict__ z1,
    float *__restrict__ z2, float *__restrict__ lam, float *__restrict__ logit,
    float *__restrict__ stats, float *__restrict__ kl) {
    const int c = threadIdx.x & 63;
    const int64_t gi = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (gi >= B) return;
    const int64_t r0 = gptr[gi], r1 = gptr[gi + 1];
    const int n = static_cast<int>(r1 - r0);
    if (n <= 0) {
        z1[gi * 64 + c] = 0.f;
        z2[gi * 64 + c] = 0.f;
        return;
    }
    // pass 1: readout of f (= graph_features_readout) and means
    float sf = 0.f, st = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        sf += f[r * 64 + c];
        st += t[r * 64 + c];
    }
    const float mu = sf / n, mt = st / n;
    // pass 2: centred second moments (two-pass, as torch's std/var)
    float qf = 0.f, qt = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float df = f[r * 64 + c] - mu, dt = t[r * 64 + c] - mt;
        qf += df * df;
        qt += dt * dt;
    }
    const float sig = sqrtf(qf / static_cast<float>(n - 1));  // n == 1 -> NaN, as torch
    const float m_use = training ? mt : rmean[c];
    const float v_use = training ? qt / n : rvar[c];
    const float rstd = 1.f / sqrtf(v_use + bn_eps);
    const float gm = gamma[c], bt = beta[c], w2c = w2[c], b2 = *b2p;
    z2[gi * 64 + c] = sf;
    float *sl = stats + gi * SCGIB_STATS_STRIDE;
    sl[kStMeanT + c] = mt;
    sl[kStSsqT + c] = qt;
    sl[kStMu + c] = mu;
    sl[kStSigma + c] = sig;
    // pass 3: compressor logit p, gate lambda, noisy features
    float zacc = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float y = gm * (t[r * 64 + c] - m_use) * rstd + bt;
        const float p = wave_sum(w2c * fmaxf(y, 0.f)) + b2;
        const float lm = gate_lambda(u_gate[r], p);
        const float fv = f[r * 64 + c];
        const float ln = 1.f - lm;
        const float nz = (lm * fv + ln * mu) + u_feat[r * 64 + c] * (ln * sig);
        im[r * 128 + c] = nz;
        zacc += nz;
        if (c == 0) lam[r] = lm;
    }
    z1[gi * 64 + c] = zacc;
    // KL of the last graph only, duplicated (models.py:657-659)
    if (gi == B - 1) {
        const float den = (sig + kKlEps) * (sig + kKlEps);
        float q = 0.f;
        for (int64_t r = r0; r < r1; ++r) {
            const float y = gm * (t[r * 64 + c] - m_use) * rstd + bt;
            const float lm = gate_lambda(u_gate[r], wave_sum(w2c * fmaxf(y, 0.f)) + b2);
            const float d = (lm * f[r * 64 + c] + (1.f - lm) * mu) - mu;
            q += (d / (sig + kKlEps)) * (d / (sig + kKlEps));
        }
        for (int64_t r = r0; r < r1; ++r) {
            const float y = gm * (t[r * 64 + c] - m_use) * rstd + bt;
            const float lm = gate_lambda(u_gate[r], wave_sum(w2c * fmaxf(y, 0.f)) + b2);
            const float ns = (1.f - lm) * sig;
            const float v = 0.5f * ((ns * ns) / den) + q;
            kl[(r - r0) * 64 + c] = v;
            kl[(r - r0 + n) * 64 + c] = v;
        }
    }
    // attention: logit_v = w_lo . z1 + w_hi . s_v + b ; softmax over the graph
    const float cst = wave_sum(watt[c] * zacc) + *battp;
    const float whi = watt[64 + c];
    float M = -INFINITY, S = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float lg = wave_sum(whi * s[r * 64 + c]) + cst;
        if (c == 0) logit[r] = lg;
        const float Mn = fmaxf(M, lg);
        S = S * expf(M - Mn) + expf(lg - Mn);
        M = Mn;
    }
    const float invS = 1.f / S;
    for (int64_t r = r0; r < r1; ++r) {
        const float sv = s[r * 64 + c];
        const float lg = wave_sum(whi * sv) + cst;
        im[r * 128 + 64 + c] = (expf(lg - M) * invS) * sv;
    }
    if (c == 0) {
        sl[kStSoftMax] = M;
        sl[kStSoftSum] = S;
        sl[kStConst] = cst;
    }
}

__global__ __launch_bounds__(64) void bn_running_update_k(const float *__restrict__ stats,
                                                          const int32_t *__restrict__ gptr,
                                                          int64_t B, float momentum,
                                                          float *__restrict__ rm,
                                                          float *__restrict__ rv,
                                                          int64_t *__restrict__ nbt) {
    const int c = threadIdx.x;
    float m = rm[c], v = rv[c];
    for (int64_t i = 0; i < B; ++i) {
        const int n = gptr[i + 1] - gptr[i];
        const float *sl = stats + i * SCGIB_STATS_STRIDE;
        const float uv = sl[kStSsqT + c] / static_cast<float>(n - 1);
        m = momentum * sl[kStMeanT + c] + (1.f - momentum) * m;
        v = momentum * uv + (1.f - momentum) * v;
    }
    rm[c] = m;
    rv[c] = v;
    if (c == 0 && nbt) *nbt += B;
}

__global__ __launch_bounds__(256) void interaction_bwd_k(
    const float *__restrict__ g_im, const float *__restrict__ g_z1,
    const float *__restrict__ g_z2, const float *__restrict__ g_kl,
    const float *__restrict__ f, const float *__restrict__ t, const float *__restrict__ s,
    const float *__restrict__ u_feat, const int32_t *__restrict__ gptr, int64_t B,
    const float *__restrict__ gamma, const float *__restrict__ beta,
    const float *__restrict__ rmean, const float *__restrict__ rvar, float bn_eps,
    int training, const float *__restrict__ w2, const float *__restrict__ watt,
    const float *__restrict__ z1, const float *__restrict__ lam,
    const float *__restrict__ logit, const float *__restrict__ stats, float *__restrict__ df,
    float *__restrict__ dt, float *__restrict__ ds, float *__restrict__ pgrad) {
    const int c = threadIdx.x & 63;
    const int64_t gi = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (gi >= B) return;
    const int64_t r0 = gptr[gi], r1 = gptr[gi + 1];
    const int n = static_cast<int>(r1 - r0);
    float *pg = pgrad + gi * SCGIB_PGRAD_STRIDE;
    if (n <= 0) {
        for (int j = c; j < SCGIB_PGRAD_STRIDE; j += 64) pg[j] = 0.f;
        return;
    }
    const float *sl = stats + gi * SCGIB_STATS_STRIDE;
    const float mt = sl[kStMeanT + c], qt = sl[kStSsqT + c];
    const float mu = sl[kStMu + c], sig = sl[kStSigma + c];
    const float M = sl[kStSoftMax], invS = 1.f / sl[kStSoftSum];
    const float m_use = training ? mt : rmean[c];
    const float v_use = training ? qt / n : rvar[c];
    const float rstd = 1.f / sqrtf(v_use + bn_eps);
    const float gm = gamma[c], bt = beta[c], w2c = w2[c];
    const float wlo = watt[c], whi = watt[64 + c], zb = z1[gi * 64 + c];

    // ---- attention backward: a_v = alpha_v s_v, alpha = softmax(logit) ----
    float SA = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float al = expf(logit[r] - M) * invS;
        SA += al * wave_sum(g_im[r * 128 + 64 + c] * s[r * 64 + c]);
    }
    float dwhi = 0.f, dc = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float al = expf(logit[r] - M) * invS;
        const float ga = g_im[r * 128 + 64 + c], sv = s[r * 64 + c];
        const float dl = al * (wave_sum(ga * sv) - SA);
        ds[r * 64 + c] = al * ga + dl * whi;
        dwhi += dl * sv;
        dc += dl;
    }
    const float gb = g_z1[gi * 64 + c] + dc * wlo;  // d z-bar -> every node's noisy
    const float gz2 = g_z2[gi * 64 + c];            // d readout(f) -> every node's f

    // ---- KL (last graph) ----
    const bool has_kl = (g_kl != nullptr) && (gi == B - 1);
    float Gc = 0.f;
    if (has_kl)
        for (int r = 0; r < n; ++r) Gc += g_kl[r * 64 + c] + g_kl[(r + n) * 64 + c];
    const float inv2 = 1.f / ((sig + kKlEps) * (sig + kKlEps));

    // ---- compression backward ----
    float dw2 = 0.f, db2 = 0.f, dg = 0.f, dbe = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
        const float lm = lam[r];
        const float fv = f[r * 64 + c];
        const float gn = g_im[r * 128 + c] + gb;
        float part = gn * (fv - mu - u_feat[r * 64 + c] * sig);
        float dfv = gn * lm + gz2;
        if (has_kl) {
            const int rl = static_cast<int>(r - r0);
            const float gk = g_kl[rl * 64 + c] + g_kl[(rl + n) * 64 + c];
            const float fm = fv - mu;
            part += gk * (-(1.f - lm) * sig * sig * inv2) + Gc * 2.f * lm * fm * fm * inv2;
            dfv += Gc * 2.f * lm * lm * fm * inv2;
        }
        const float dp = wave_sum(part) * lm * (1.f - lm);
        const float xh = (t[r * 64 + c] - m_use) * rstd;
        const float y = gm * xh + bt;
        dw2 += dp * fmaxf(y, 0.f);
        db2 += dp;
        const float dy = y > 0.f ? dp * w2c : 0.f;
        dg += dy * xh;
        dbe += dy;
        df[r * 64 + c] = dfv;
        dt[r * 64 + c] = dy;
    }
    // BatchNorm backward (batch statistics of this graph, or running stats)
    const float inv_n = 1.f / n;
    for (int64_t r = r0; r < r1; ++r) {
        const float dy = dt[r * 64 + c];
        if (training) {
            const float xh = (t[r * 64 + c] - m_use) * rstd;
            dt[r * 64 + c] = gm * rstd * (dy - dbe * inv_n - xh * dg * inv_n);
        } else {
            dt[r * 64 + c] = gm * rstd * dy;
        }
    }
    pg[kPgW2 + c] = dw2;
    pg[kPgGamma + c] = dg;
    pg[kPgBeta + c] = dbe;
    pg[kPgWatt + c] = dc * zb;
    pg[kPgWatt + 64 + c] = dwhi;
    if (c == 0) {
        pg[kPgB2] = db2;
        pg[kPgBatt] = dc;
        pg[SCGIB_PGRAD_STRIDE - 2] = 0.f;
        pg[SCGIB_PGRAD_STRIDE - 1] = 0.f;
    }
}

}  // namespace scgib

using namespace scgib;

extern "C" int scgib_interaction_fwd(
    const float *f, const float *t, const float *s, const float *u_gate, const float *u_feat,
    const int32_t *graph_ptr, int64_t n_graphs, int64_t n_nodes, const float *bn_gamma,
    const float *bn_beta, const float *bn_running_mean, const float *bn_running_var,
    float bn_eps, int32_t training, const float *w2, const float *b2, const float *w_att,
    const float *b_att, float *im, float *z1, float *z2, float *lam, float *logit,
    float *stats, float *kl_tensor, scgib_stream_t stream) {
    if (n_graphs < 0 || n_nodes < 0) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (!graph_ptr || !bn_gamma || !bn_beta || !w2 || !b2 || !w_att || !b_att || !z1 ||
        !z2 || !stats || !kl_tensor)
        return SCGIB_EINVAL;
    if (n_nodes > 0 && (!f || !t || !s || !u_gate || !u_feat || !im || !lam || !logit))
        return SCGIB_EINVAL;
    if (!training && (!bn_running_mean || !bn_running_var)) return SCGIB_EINVAL;
    const int64_t grid = (n_graphs + 3) / 4;
    interaction_fwd_k<<<dim3((unsigned)grid), 256, 0, as_stream(stream)>>>(
        f, t, s, u_gate, u_feat, graph_ptr, n_graphs, bn_gamma, bn_beta, bn_running_mean,
        bn_running_var, bn_eps, training, w2, b2, w_att, b_att, im, z1, z2, lam, logit, stats,
        kl_tensor);
    return launch_status();
}

extern "C" int scgib_bn_running_update(const float *stats, const int32_t *graph_ptr,
                                       int64_t n_graphs, float momentum, float *running_mean,
                                       float *running_var, int64_t *num_batches_tracked,
                                       scgib_stream_t stream) {
    if (n_graphs < 0) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (!stats || !graph_ptr || !running_mean || !running_var) return SCGIB_EINVAL;
    bn_running_update_k<<<1, 64, 0, as_stream(stream)>>>(stats, graph_ptr, n_graphs, momentum,
                                                         running_mean, running_var,
                                                         num_batches_tracked);
    return launch_status();
}

extern "C" int scgib_interaction_bwd(
    const float *g_im, const float *g_z1, const float *g_z2, const float *g_kl, const float *f,
    const float *t, const float *s, const float *u_feat, const int32_t *graph_ptr,
    int64_t n_graphs, int64_t n_nodes, const float *bn_gamma, const float *bn_beta,
    const float *bn_running_mean, const float *bn_running_var, float bn_eps, int32_t training,
    const float *w2, const float *w_att, const float *z1, const float *lam,
    const float *logit, const float *stats, float *df, float *dt, float *ds, float *pgrad,
    scgib_stream_t stream) {
    if (n_graphs < 0 || n_nodes < 0) return SCGIB_EINVAL;
    if (n_graphs == 0) return SCGIB_OK;
    if (!graph_ptr || !g_z1 || !g_z2 || !bn_gamma || !bn_beta || !w2 || !w_att || !z1 ||
        !stats || !pgrad)
        return SCGIB_EINVAL;
    if (n_nodes > 0 && (!g_im || !f || !t || !s || !u_feat || !lam || !logit || !df || !dt ||
                        !ds))
        return SCGIB_EINVAL;
    if (!training && (!bn_running_mean || !bn_running_var)) return SCGIB_EINVAL;
    const int64_t grid = (n_graphs + 3) / 4;
    interaction_bwd_k<<<dim3((unsigned)grid), 256, 0, as_stream(stream)>>>(
        g_im, g_z1, g_z2, g_kl, f, t, s, u_feat, graph_ptr, n_graphs, bn_gamma, bn_beta,
        bn_running_mean, bn_running_var, bn_eps, training, w2, w_att, z1, lam, logit, stats,
        df, dt, ds, pgrad);
    return launch_status();
}
