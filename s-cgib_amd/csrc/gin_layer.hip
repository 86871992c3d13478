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
//   slab_reduce_k  : fixed-order sum of the per-workgroup slabs.
//
// LDS tiles are row-major with a +1-float row pad (stride 65 / 33), which
// makes every MFMA operand read (32 lanes: 32 rows of one column, or 32
// columns of one row) bank-conflict free for ds_read_b32.
#include "mfma_tile.h"
#include "contrast_body.h"
#include "recon_fin.h"
#include "running_update.h"

namespace scgib {

// ---------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// BatchNorm finalize folded into the producing tile kernel (training mode).
// Hierarchical last-arriver: the tiles of a layer arrive in groups of kGroup; the
// last tile of a group combines the group's 16 tile statistics (fp64) into a
// group partial, then arrives at the layer counter; the last group combines
// the groups and writes the BN record / coefficients.  Two short load rounds
// at the tail of the kernel replace a separate 1-workgroup finalize launch.
// Fixed combination order -> deterministic.  Counters: caller-provided, zero
// on entry; each is reset by its last arriver (graph-replay safe).
// ---------------------------------------------------------------------------
// tiles per BatchNorm statistics group (8 / 32 / 64 measured +1 %, round 1)
constexpr int kGroup = 16;
static_assert(kGroup % 4 == 0 && kGroup <= 64, "group combine: 4 partitions, <= 16 loads each");

struct BnFwdFuse {          // gin_fwd_k: BN statistics + running update
    unsigned *counters;     // [ngr_cap + 1]; nullptr: not fused (separate finalize)
    double *gpart;          // [ngr_cap][128]: group sum, group centred M2
    const float *gamma, *beta;
    float *rmean, *rvar, *stat;
    int64_t *nbt;
    float eps, momentum;
    int ngr_cap;
    int defer;              // stop at the group partials (the consumer finishes)
};

struct BnBwdFuse {          // gin_bwd_stats_k: dgamma, dbeta, dz2 coefficients
    unsigned *counters;
    double *gpart;          // [ngr_cap][128]: group sum dy, group sum dy * xhat
    float *dgamma, *dbeta, *coef;
    int training, ngr_cap;
    int defer;
};

// Cross-workgroup exchange: st_agent / ld_agent / block_arrive (common.h).

// rows of tile t / group g of an n-row layer
__device__ __forceinline__ double rows_in(int64_t n, int64_t first, int64_t span) {
    const int64_t r = n - first;
    return static_cast<double>(r < span ? r : span);
}

// Layer statistics from the ngr group partials (fp64, fixed order; 256
// threads, channel c = tid & 63, partition p = tid >> 6 takes groups p, p + 4,
// ...; one load round while ngr <= 64).  Every thread returns its channel's
// mean and centred M2:  M2 = sum_g [M2_g + (S_g - n_g mean)^2 / n_g].
// AGENT: the partials were written earlier in this kernel (agent-scope loads);
// otherwise by a previous kernel (plain loads: L2-cached after the first
// workgroup of an XCD, coherent across the kernel boundary).
template <bool AGENT>
__device__ __forceinline__ double ld_part(const double *p) {
    if constexpr (AGENT) return ld_agent(p);
    else return *p;
}

// Barrier-free layer combine (wave-local shuffles, no LDS): lane l of wave w
// owns channel c = 16 w + (l & 15) and partition p = l >> 4, which takes
// groups p, p + 4, ... (fp64, fixed order); the four partitions combine as
// (p0 + p1) + (p2 + p3) through two xor shuffles (identical in every lane).
// Split into the load (issue early, registers) and the combine, so other
// loads can be in flight meanwhile; one load round for ngr <= kFinG.  (8:
// the QM9 B512 ego layers' 28 groups in one round, and 32 fewer VGPRs than
// 16 in the forward kernel, which then keeps its first neighbour-index round
// in flight across the finish)
constexpr int kFinR = 8, kFinG = 4 * kFinR;
// backward consumers: 2 partitions x kBFinR groups per load round
constexpr int kBFinR = 16;
// past one round of 64 groups the last-arriver statistics take a third
// level: 64-group supergroups (bn_fwd_hier / bn_bwd_hier)
constexpr int kSuper = 64;

struct FwdFin {
    double vs[kFinR], vq[kFinR];
};

__device__ __forceinline__ int fin_channel() { return 16 * (threadIdx.x >> 6) + (threadIdx.x & 15); }

template <bool AGENT>
__device__ __forceinline__ void bn_fwd_fin_load(const double *__restrict__ gpart, int ngr, int g0,
                                                FwdFin &f) {
    const int c = fin_channel(), p = (threadIdx.x & 63) >> 4;
#pragma unroll
    for (int u = 0; u < kFinR; ++u) {
        if (g0 + 4 * u < ngr) {  // wave-uniform: only rounds with a live group are loaded
            const int64_t gg = g0 + p + 4 * u < ngr ? g0 + p + 4 * u : 0;  // group 0 always exists
            f.vs[u] = ld_part<AGENT>(gpart + gg * 128 + c);
            f.vq[u] = ld_part<AGENT>(gpart + gg * 128 + 64 + c);
        }
    }
}

__device__ __forceinline__ double quad_sum(double a) {
    a = a + __shfl_xor(a, 16, kWave);
    return a + __shfl_xor(a, 32, kWave);
}

// mean and centred M2 of channel fin_channel():
//   mean = sum_g S_g / n,  M2 = sum_g [M2_g + (S_g - n_g mean)^2 / n_g]
// n_g = kGroup * 64 for every group but possibly the last, and dividing by a power
// of two equals multiplying by its reciprocal exactly, so only the last
// group's term (added last by its owner, the same order) divides.
// UNIT: rows of every entry but possibly the last (kGroup tiles; a 64-group
// supergroup at the third level of bn_fwd_hier).  S (or nullptr): the sum.
template <bool AGENT, int64_t UNIT = int64_t(kGroup) * TM>
__device__ void bn_fwd_final(const double *__restrict__ gpart, int64_t n, int ngr, FwdFin &f,
                             double &mean, double &M2, double *S = nullptr) {
    constexpr double kFull = static_cast<double>(UNIT), kInvFull = 1.0 / kFull;
    const int p = (threadIdx.x & 63) >> 4;
    double a = 0.0;
    for (int g0 = 0; g0 < ngr; g0 += kFinG) {
        if (g0 > 0) bn_fwd_fin_load<AGENT>(gpart, ngr, g0, f);
#pragma unroll
        for (int u = 0; u < kFinR; ++u)
            if (g0 + 4 * u < ngr) a += g0 + p + 4 * u < ngr ? f.vs[u] : 0.0;
    }
    const double sum = quad_sum(a);
    if (S) *S = sum;
    mean = sum / static_cast<double>(n);
    const int glast = ngr - 1;
    const double nlast = rows_in(n, int64_t(glast) * UNIT, UNIT);
    const bool last_partial = nlast != kFull;
    double q = 0.0, last_vq = 0.0, last_d = 0.0;
    bool owns_last = false;
    for (int g0 = 0; g0 < ngr; g0 += kFinG) {
        if (ngr > kFinG) bn_fwd_fin_load<AGENT>(gpart, ngr, g0, f);  // else still in registers
#pragma unroll
        for (int u = 0; u < kFinR; ++u) {
            if (g0 + 4 * u < ngr) {
                const int g = g0 + p + 4 * u;
                if (g < ngr) {
                    if (g == glast && last_partial) {
                        owns_last = true;
                        last_vq = f.vq[u];
                        last_d = f.vs[u] - nlast * mean;
                    } else {
                        const double d = f.vs[u] - kFull * mean;
                        q += f.vq[u] + d * d * kInvFull;
                    }
                }
            }
        }
    }
    if (owns_last) q += last_vq + last_d * last_d / nlast;
    M2 = quad_sum(q);
}

// BN record of channel c from (mean, M2): returns scale / shift; with
// `write`, also the [4][64] record and the running-statistics update
// (momentum, unbiased variance, num_batches_tracked += 1).
// (gamma_c / beta_c are passed as values: load them early, a dependent
// global load here costs a full memory latency)
__device__ __forceinline__ float2 bn_fwd_publish(int c, double mean, double M2, int64_t n,
                                                 float gamma_c, float beta_c,
                                                 float eps, float momentum, float *rmean,
                                                 float *rvar, int64_t *nbt, float *stat,
                                                 bool write) {
    const double var = M2 / static_cast<double>(n);
    if (write && rmean) {
        rmean[c] = static_cast<float>((1.0 - momentum) * rmean[c] + momentum * mean);
        rvar[c] = static_cast<float>((1.0 - momentum) * rvar[c] +
                                     momentum * (n > 1 ? M2 / static_cast<double>(n - 1) : M2));
        if (c == 0 && nbt) *nbt += 1;
    }
    const double istd = 1.0 / sqrt(var + static_cast<double>(eps));
    const double sc = gamma_c * istd;
    const float scale = static_cast<float>(sc), shift = static_cast<float>(beta_c - mean * sc);
    if (write) {
        stat[c] = static_cast<float>(mean);
        stat[64 + c] = static_cast<float>(istd);
        stat[128 + c] = scale;
        stat[192 + c] = shift;
    }
    return make_float2(scale, shift);
}

// A consumer of a deferred layer (scgib_bn_pending) that is not a GIN layer
// (the encoder output's BN + ReLU): every 256-thread workgroup finishes the
// statistics from the group partials; workgroup 0 writes the record and the
// running update.  sSS[c] = scale, sSS[64 + c] = shift.  Call from all
// threads, before any early return.
__device__ __forceinline__ void bn_pending_finish(const scgib_bn_pending &pend, int64_t n,
                                                  float *sSS) {
    const int fc = fin_channel();
    const int ngr = static_cast<int>(((n + TM - 1) / TM + kGroup - 1) / kGroup);
    const float gam = pend.gamma[fc], bet = pend.beta[fc];
    FwdFin fin;
    bn_fwd_fin_load<false>(pend.gpart, ngr, 0, fin);
    double mean, M2;
    bn_fwd_final<false>(pend.gpart, n, ngr, fin, mean, M2);
    const bool lead = (threadIdx.x & 63) < 16;
    const float2 ss = bn_fwd_publish(fc, mean, M2, n, gam, bet, pend.eps, pend.momentum,
                                     pend.running_mean, pend.running_var,
                                     pend.num_batches_tracked, pend.stat, blockIdx.x == 0 && lead);
    if (lead) {
        sSS[fc] = ss.x;
        sSS[64 + fc] = ss.y;
    }
    __syncthreads();
}

// 256 threads: channel c = tid & 63, partition p = tid >> 6 (4 partitions).
// Per-tile (S, M2) -> group (S_g, M2_g) -> layer (mean, M2); exact
// decomposition M2 = sum_b [M2_b + (S_b - n_b mean)^2 / n_b] at each level.
// arrivals = tiles of group g whose statistics this workgroup contributes
// (1 per tile kernel; a workgroup running several tiles of one group may
// arrive for all of them at once)
__device__ void bn_fwd_hier(const float *__restrict__ part, int64_t n, int64_t tile,
                            const BnFwdFuse &fz, unsigned arrivals = 1u) {
    const int64_t nt = (n + TM - 1) / TM;
    const int ngr = static_cast<int>((nt + kGroup - 1) / kGroup);
    const int g = static_cast<int>(tile / kGroup);
    const int gsize = static_cast<int>(nt - int64_t(g) * kGroup < kGroup ? nt - int64_t(g) * kGroup : kGroup);
    if (!block_arrive(&fz.counters[g], gsize, arrivals)) return;
    const int c = threadIdx.x & 63, p = threadIdx.x >> 6;
    __shared__ double sh[4][64];
    __shared__ double smean[64];
    {   // group combine: partition p takes tiles g*kGroup + p + 4u
        constexpr int U = kGroup / 4;
        float S[U], Q[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t t = int64_t(g) * kGroup + p + 4 * u;
            const int64_t tc = p + 4 * u < gsize ? t : int64_t(g) * kGroup;
            S[u] = ld_agent(part + tc * 128 + c);
            Q[u] = ld_agent(part + tc * 128 + 64 + c);
        }
        double a = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) a += p + 4 * u < gsize ? static_cast<double>(S[u]) : 0.0;
        sh[p][c] = a;
        __syncthreads();
        if (p == 0) {
            const double sg = ((sh[0][c] + sh[1][c]) + sh[2][c]) + sh[3][c];
            smean[c] = sg / rows_in(n, int64_t(g) * kGroup * TM, kGroup * TM);
            st_agent(fz.gpart + int64_t(g) * 128 + c, sg);
        }
        __syncthreads();
        const double mg = smean[c];
        double q = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (p + 4 * u < gsize) {
                const int64_t t = int64_t(g) * kGroup + p + 4 * u;
                const double nb = rows_in(n, t * TM, TM);
                const double d = static_cast<double>(S[u]) - nb * mg;
                q += static_cast<double>(Q[u]) + d * d / nb;
            }
        }
        __syncthreads();
        sh[p][c] = q;
        __syncthreads();
        if (p == 0) st_agent(fz.gpart + int64_t(g) * 128 + 64 + c, ((sh[0][c] + sh[1][c]) + sh[2][c]) + sh[3][c]);
        if (threadIdx.x == 0) fz.counters[g] = 0u;
    }
    if (fz.defer) return;  // the consumer kernel finishes (bn_fwd_final there)
    double mean, M2;
    FwdFin fin;
    if (ngr > kSuper) {  // block-uniform
        // more groups than one load round: a third level, so that no single
        // workgroup walks every group partial in series at the end of the
        // kernel (1172 groups at 1.2 M rows: ~74 us of dependent load rounds).
        // The last group of each 64-group supergroup combines its groups
        // (one round), the last supergroup combines the supergroups.
        constexpr int64_t kSupRows = int64_t(kSuper) * kGroup * TM;
        const int s = g / kSuper, nsup = (ngr + kSuper - 1) / kSuper;
        const int ssize = ngr - s * kSuper < kSuper ? ngr - s * kSuper : kSuper;
        unsigned *scnt = &fz.counters[fz.ngr_cap + 1 + s];
        if (!block_arrive(scnt, ssize)) return;
        const double *gp = fz.gpart + int64_t(s) * kSuper * 128;
        double *sp = fz.gpart + int64_t(fz.ngr_cap) * 128;
        const int64_t ns = static_cast<int64_t>(rows_in(n, s * kSupRows, kSupRows));
        double S;
        bn_fwd_fin_load<true>(gp, ssize, 0, fin);
        bn_fwd_final<true>(gp, ns, ssize, fin, mean, M2, &S);
        if ((threadIdx.x & 63) < 16) {
            st_agent(sp + int64_t(s) * 128 + fin_channel(), S);
            st_agent(sp + int64_t(s) * 128 + 64 + fin_channel(), M2);
        }
        if (threadIdx.x == 0) *scnt = 0u;
        if (!block_arrive(&fz.counters[fz.ngr_cap], nsup)) return;
        const float gam = fz.gamma[fin_channel()], bet = fz.beta[fin_channel()];
        bn_fwd_fin_load<true>(sp, nsup, 0, fin);
        bn_fwd_final<true, kSupRows>(sp, n, nsup, fin, mean, M2);
        bn_fwd_publish(fin_channel(), mean, M2, n, gam, bet, fz.eps, fz.momentum, fz.rmean,
                       fz.rvar, fz.nbt, fz.stat, (threadIdx.x & 63) < 16);
        if (threadIdx.x == 0) fz.counters[fz.ngr_cap] = 0u;
        return;
    }
    if (!block_arrive(&fz.counters[fz.ngr_cap], ngr)) return;
    const float gam = fz.gamma[fin_channel()], bet = fz.beta[fin_channel()];
    bn_fwd_fin_load<true>(fz.gpart, ngr, 0, fin);
    bn_fwd_final<true>(fz.gpart, n, ngr, fin, mean, M2);
    bn_fwd_publish(fin_channel(), mean, M2, n, gam, bet, fz.eps, fz.momentum, fz.rmean,
                   fz.rvar, fz.nbt, fz.stat, (threadIdx.x & 63) < 16);
    if (threadIdx.x == 0) fz.counters[fz.ngr_cap] = 0u;
}

// Layer sums (dbeta | dgamma, 128 values) from the ngr group partials,
// barrier-free: lane l of wave w owns sum index cs = 32 w + (l & 31) and
// partition p = l >> 5 (groups p, p + 2, ...); p0 + p1 via one xor shuffle.
struct BwdFin {
    double v[kBFinR];
};

__device__ __forceinline__ int bfin_index() { return 32 * (threadIdx.x >> 6) + (threadIdx.x & 31); }

template <bool AGENT>
__device__ __forceinline__ void bn_bwd_fin_load(const double *__restrict__ gpart, int ngr, int g0,
                                                BwdFin &f) {
    const int cs = bfin_index(), p = (threadIdx.x & 63) >> 5;
#pragma unroll
    for (int u = 0; u < kBFinR; ++u) {
        if (g0 + 2 * u < ngr) {  // wave-uniform
            const int64_t gg = g0 + p + 2 * u < ngr ? g0 + p + 2 * u : 0;  // group 0 always exists
            f.v[u] = ld_part<AGENT>(gpart + gg * 128 + cs);
        }
    }
}

template <bool AGENT>
__device__ double bn_bwd_final(const double *__restrict__ gpart, int ngr, BwdFin &f) {
    const int p = (threadIdx.x & 63) >> 5;
    double a = 0.0;
    for (int g0 = 0; g0 < ngr; g0 += 2 * kBFinR) {
        if (g0 > 0) bn_bwd_fin_load<AGENT>(gpart, ngr, g0, f);
#pragma unroll
        for (int u = 0; u < kBFinR; ++u)
            if (g0 + 2 * u < ngr) a += g0 + p + 2 * u < ngr ? f.v[u] : 0.0;
    }
    return a + __shfl_xor(a, 32, kWave);
}

// dbeta = sum dy (c < 64), dgamma = sum dy xhat (c >= 64); dz2 coefficient
// coef[c] = tot / N in training (0 in eval); coef may be nullptr
__device__ __forceinline__ float bn_bwd_publish(int c, double tot, int64_t n, int training,
                                                float *dgamma, float *dbeta, float *coef) {
    const float cf = training ? static_cast<float>(tot / static_cast<double>(n)) : 0.f;
    if (dbeta) {
        if (c < 64) dbeta[c] = static_cast<float>(tot);
        else dgamma[c - 64] = static_cast<float>(tot);
    }
    if (coef) coef[c] = cf;
    return cf;
}

// backward: tile (sum dy, sum dy xhat) -> group -> layer sums (fp64);
// sh: 2 KB of LDS scratch (the caller's, so a kernel near its LDS limit can
// lend a dead tile image)
// (group g, `count` of its tiles arriving at once: gin_bwd_statsz_k's walk)
__device__ __forceinline__ void bn_bwd_hier_gs(const float *__restrict__ part, int64_t n, int g, unsigned count,
                               const BnBwdFuse &bz, double (*sh)[128]) {
    const int64_t nt = (n + TM - 1) / TM;
    const int ngr = static_cast<int>((nt + kGroup - 1) / kGroup);
    const int gsize = static_cast<int>(nt - int64_t(g) * kGroup < kGroup ? nt - int64_t(g) * kGroup : kGroup);
    if (!block_arrive(&bz.counters[g], gsize, count)) return;
    const int c = threadIdx.x & 127, p = threadIdx.x >> 7;  // 128 sums x 2 partitions
    {
        constexpr int U = kGroup / 2;
        float v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = p + 2 * u;
            v[u] = ld_agent(part + (int64_t(g) * kGroup + (k < gsize ? k : 0)) * 128 + c);
        }
        double a = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) a += p + 2 * u < gsize ? static_cast<double>(v[u]) : 0.0;
        sh[p][c] = a;
        __syncthreads();
        if (p == 0) st_agent(bz.gpart + int64_t(g) * 128 + c, sh[0][c] + sh[1][c]);
        if (threadIdx.x == 0) bz.counters[g] = 0u;
    }
    if (bz.defer) return;  // the layer's gin_bwd_k finishes (bn_bwd_final there)
    BwdFin fin;
    if (ngr > kSuper) {  // block-uniform: the third level, as in bn_fwd_hier
        const int s = g / kSuper, nsup = (ngr + kSuper - 1) / kSuper;
        const int ssize = ngr - s * kSuper < kSuper ? ngr - s * kSuper : kSuper;
        unsigned *scnt = &bz.counters[bz.ngr_cap + 1 + s];
        if (!block_arrive(scnt, ssize)) return;
        const double *gp = bz.gpart + int64_t(s) * kSuper * 128;
        double *sp = bz.gpart + int64_t(bz.ngr_cap) * 128;
        bn_bwd_fin_load<true>(gp, ssize, 0, fin);
        const double st = bn_bwd_final<true>(gp, ssize, fin);
        if ((threadIdx.x & 63) < 32) st_agent(sp + int64_t(s) * 128 + bfin_index(), st);
        if (threadIdx.x == 0) *scnt = 0u;
        if (!block_arrive(&bz.counters[bz.ngr_cap], nsup)) return;
        bn_bwd_fin_load<true>(sp, nsup, 0, fin);
        const double tot = bn_bwd_final<true>(sp, nsup, fin);
        if ((threadIdx.x & 63) < 32)
            bn_bwd_publish(bfin_index(), tot, n, bz.training, bz.dgamma, bz.dbeta, bz.coef);
        if (threadIdx.x == 0) bz.counters[bz.ngr_cap] = 0u;
        return;
    }
    if (!block_arrive(&bz.counters[bz.ngr_cap], ngr)) return;
    bn_bwd_fin_load<true>(bz.gpart, ngr, 0, fin);
    const double tot = bn_bwd_final<true>(bz.gpart, ngr, fin);
    if ((threadIdx.x & 63) < 32)
        bn_bwd_publish(bfin_index(), tot, n, bz.training, bz.dgamma, bz.dbeta, bz.coef);
    if (threadIdx.x == 0) bz.counters[bz.ngr_cap] = 0u;
}

__device__ void bn_bwd_hier_s(const float *__restrict__ part, int64_t n, int64_t tile,
                              const BnBwdFuse &bz, double (*sh)[128]) {
    bn_bwd_hier_gs(part, n, static_cast<int>(tile / kGroup), 1u, bz, sh);
}

__device__ void bn_bwd_hier(const float *__restrict__ part, int64_t n, int64_t tile,
                            const BnBwdFuse &bz) {
    __shared__ double sh[2][128];
    bn_bwd_hier_s(part, n, tile, bz, sh);
}

// ---------------------------------------------------------------------------
// transfer_d folded into the first GIN layer (PRE): the reference computes
// h0 = x Wt^T per node (models.py:668-669, :1164-1165) and then aggregates h0;
// by linearity agg0 = (ope x_v + sum_u x_u) Wt^T, so layer 0 gathers the raw
// normalised features (F <= 16 floats per row, optionally through the
// ego -> parent node map, i.e. x_subs = x[ego_nodes] is never materialised)
// and applies Wt on the 64-row tile in LDS (K = 16 MFMA).  Backward adds
// dWt += dagg0^T aggx in the same tile kernel; d(agg0) itself is never stored.
// ---------------------------------------------------------------------------
constexpr int kPreF = 16;       // max raw feature width
constexpr int kPreLD = 17;      // LDS stride of the [64][16] aggx tile
constexpr int kPreSlab = 32 * kPreF;

struct PreArgs {
    const float *x;         // [N_parent][F] raw (normalised) features
    const int32_t *nmap;    // nullptr, or [N] row -> parent row (ego batches)
    const float *wt;        // [32][F] transfer_d.weight
    float *aggx;            // [N][16] saved gathered features (zero-padded)
    int F;
};

// 16 lanes per row (lane c = feature c; c >= F contribute 0), 4 rows per
// thread (rbase + 16 k).  Same latency scheme as gather_rows: every load
// unconditional at a clamped valid address, masked lanes/slots enter through
// fmaf(x, 0, acc).  Requires nv >= 1.
__device__ __forceinline__ void gather_x_rows(const PreArgs &pre, const int32_t *__restrict__ rowptr,
                                              const int32_t *__restrict__ col, int64_t row0,
                                              int nv, int rbase, int c, float ope,
                                              float (&acc)[4]) {
    const int F = pre.F, cc = c < F ? c : F - 1;
    const float cm = c < F ? 1.f : 0.f;
    int32_t beg[4], deg[4];
    int64_t vrow[4], sid[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int rr = rbase + 16 * k;
        vrow[k] = row0 + (rr < nv ? rr : nv - 1);
        beg[k] = rowptr[vrow[k]];
        deg[k] = rowptr[vrow[k] + 1];
    }
    // (the uniform branch outside the rows: as a per-row select, each
    // node-map load sat in its own branch and was waited for alone)
    if (pre.nmap) {
#pragma unroll
        for (int k = 0; k < 4; ++k) sid[k] = pre.nmap[vrow[k]];
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) sid[k] = vrow[k];
    }
    float self[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        self[k] = pre.x[sid[k] * F + cc];
        acc[k] = 0.f;
    }
    int maxdeg = 0, maxend = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        maxend = deg[k] > maxend ? deg[k] : maxend;
        deg[k] -= beg[k];
        maxdeg = deg[k] > maxdeg ? deg[k] : maxdeg;
    }
    for (int j0 = 0; j0 < maxdeg; j0 += 4) {
        int64_t u[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int32_t e = beg[k] + j0 + t;
                u[k][t] = col[e < maxend ? e : maxend - 1];
            }
        if (pre.nmap) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int t = 0; t < 4; ++t) u[k][t] = pre.nmap[u[k][t]];
        }
        float a[4][4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t) a[k][t] = pre.x[u[k][t] * F + cc];
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[k] = fmaf(a[k][t], j0 + t < deg[k] ? cm : 0.f, acc[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = ope * (self[k] * cm) + acc[k];
}

// Reconstruction loss fused into the head MLP (RECON, dense path only):
// forward writes each tile's Gram partial out^T out of the MLP output (the
// interaction map IM fed to loss_recon_adj, models.py:762-768) to gslab;
// backward forms d IM = (g/N) (4 IM G - 2 (A + A^T) IM) of its tile in LDS
// (recon.hip for the derivation) instead of reading dy.
struct ReconArgs {
    float *gslab;                       // fwd: [tiles][64*64] Gram partials
    const float *im, *gram;             // bwd: MLP output [N][64], G [64][64]
    const int32_t *rowptr, *col;        // bwd: dst-major CSR
    const int32_t *rowptr_t, *col_t;    // bwd: src-major CSR, nullptr = symmetric
    const float *g_loss;                // bwd: d loss / d recon (device scalar)
    // the contrastive loss (contrast_body.h) in extra workgroups past the
    // MLP's (con.B = 0: none): it reads only z1 / z2, so it runs beside the
    // MLP instead of as its own launch on the critical chain
    ContrastArgs con;
    // fwd, fin_on: the tiles finish the loss themselves (recon_fin.h) once
    // every tile has published its Gram partial and output rows (write-through
    // stores + one arrival each); the host sets it only when the whole grid is
    // co-resident (one workgroup per CU).  ru_block >= 0: that workgroup runs
    // the compressor BatchNorm's running update (running_update.h)
    ReconFin fin;
    int fin_on, ru_block;
    scgib_running_update ru;
};
constexpr uint64_t kFinWaitTicks = 20000000;  // 0.2 s of the 100 MHz wall clock

// GATHER = false is the dense two-layer MLP of the head (models.py:1055-1057,
// applied at :1174): the tile's input rows are staged directly, agg_out and
// the BN tile statistics are not written, z2_out is the MLP output.
constexpr bool kLateWeights = true;  // (early: 0.4372 vs 0.4355 ms, round 2)

// r aliased onto the agg tile: the gathering d_in = 64 layers write r into
// the agg tile's buffer once every wave's first GEMM is done (one more
// barrier): 53 KB of LDS and <= 168 VGPRs, three workgroups per CU instead
// of two, so an ego layer's 437 tiles and Encoder1's 145 fit the chip at once
// (layer 0 with transfer_d folded: the agg tile and W1 are 32 wide, so r
// takes both of their buffers, contiguous: 59.8 -> 43 KB)
template <int DIN, bool GATHER, bool PRE>
constexpr bool kFwdAlias = ((DIN == 64 && GATHER && !PRE) || (DIN == 32 && GATHER && PRE));

// blockIdx -> 64-row tile of a gathering layer.  The dispatcher deals
// workgroups round-robin over the 8 XCDs (MI355X_MICROARCH.md, "Workgroup
// dispatch"), so with tile = blockIdx consecutive tiles — which share rows:
// the neighbours across a tile edge, the row window's halo — sit in
// different L2s.  SCGIB_XCD_TILES = 1 (default) gives each XCD a contiguous
// run of tiles instead (xcd_remap): speed only, every tile computes the same
// bits wherever it runs.  Measured (profiles/r04_window/xcd_tiles.txt): the
// superbatch backward statistics 258.9 -> 236.5 us (0.76 -> 0.83 of HBM),
// the forward layer 437.9 -> 435.4 us, the QM9 B512 step unchanged.
#ifndef SCGIB_XCD_TILES  // (build-time A/B hook: tools/build_ab_lib.sh EXTRA=-DSCGIB_XCD_TILES=n)
#define SCGIB_XCD_TILES 1
#endif
__device__ __forceinline__ int64_t tile_of_block(int64_t ntiles) {
    return SCGIB_XCD_TILES ? xcd_remap(blockIdx.x, ntiles) : static_cast<int64_t>(blockIdx.x);
}

template <int DIN, bool XFORM, bool GATHER = true, bool PRE = false, bool RECON = false>
__global__ __launch_bounds__(256, (kFwdAlias<DIN, GATHER, PRE> ? 3 : 1)) void gin_fwd_k(
    const float *__restrict__ h, const float *__restrict__ in_scale,
    const float *__restrict__ in_shift, const int32_t *__restrict__ rowptr,
    const int32_t *__restrict__ col, int64_t ncap, float ope, const float *__restrict__ w1,
    const float *__restrict__ b1, const float *__restrict__ w2, const float *__restrict__ b2,
    float *__restrict__ agg_out, float *__restrict__ r_out, float *__restrict__ z2_out,
    float *__restrict__ part, const int32_t *__restrict__ dims, BnFwdFuse fz, PreArgs pre,
    scgib_bn_pending pend, ReconArgs rec) {
    constexpr int LDA = DIN + 1, LPR = DIN / 4, RPP = 256 / LPR;
    static_assert(!RECON || !GATHER, "the recon Gram partial is fused into the dense head MLP");
    static_assert(!PRE || DIN == 32, "transfer_d fold produces the 32-wide layer-0 input");
    const int64_t n = eff_count(dims, 0, ncap);
    // sA | sW1 contiguous (contrastive: float4 tiles in each)
    __shared__ __attribute__((aligned(16))) float sAW1[TM * LDA + 64 * LDA];
    float *const sA = sAW1, *const sW1 = sAW1 + TM * LDA;
    __shared__ float sW2[64 * LDH];
    constexpr bool ALIAS = kFwdAlias<DIN, GATHER, PRE>;
    static_assert(!ALIAS || TM * LDA + 64 * LDA >= TM * LDH, "r takes the agg tile's (and W1's) buffer");
    __shared__ float sROwn[ALIAS ? 1 : TM * LDH];
    float *const sR = ALIAS ? sA : sROwn;
    __shared__ float sRed[2][64];
    __shared__ float sPre[PRE ? (TM + 32) * kPreLD : 1];  // aggx tile | Wt
    if constexpr (RECON && DIN == 128) {  // the pretraining head (interaction map width)
        static_assert(TM * LDA >= CT * CLD, "contrastive tiles in sA / sW1");
        if (static_cast<int>(blockIdx.x) == rec.ru_block) {  // block-uniform
            running_update_body<256>(rec.ru);
            return;
        }
        if (rec.con.B > 0 && static_cast<int>(blockIdx.x) >= rec.con.nmain) {  // block-uniform
            const int64_t b = blockIdx.x - rec.con.nmain, nrb = contrast_row_blocks(rec.con.B);
            SCGIB_MARK(0);
            contrast_fwd_body(rec.con, b % nrb, static_cast<int>(b / nrb), sA, sW1);
            SCGIB_MARK(5);
            return;
        }
    }
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    // (the head MLP's grid carries extra workgroups past its tiles: identity there)
    const int64_t tile = GATHER ? tile_of_block(gridDim.x) : static_cast<int64_t>(blockIdx.x);
    const int64_t row0 = tile * TM;
    const int nv = static_cast<int>(n - row0 < TM ? (n - row0 > 0 ? n - row0 : 0) : TM);  // valid rows
    if (dims) {  // capacity mode: zero this tile's padded rows [nv, rows in capacity)
        const int ncr = static_cast<int>(ncap - row0 < TM ? ncap - row0 : TM);
        for (int idx = nv * 64 + tid; idx < ncr * 64; idx += 256) {
            if (r_out) r_out[row0 * 64 + idx] = 0.f;
            z2_out[row0 * 64 + idx] = 0.f;
        }
        if (GATHER && agg_out)
            for (int idx = nv * DIN + tid; idx < ncr * DIN; idx += 256) agg_out[row0 * DIN + idx] = 0.f;
        if (PRE)
            for (int idx = nv * kPreF + tid; idx < ncr * kPreF; idx += 256) pre.aggx[row0 * kPreF + idx] = 0.f;
        if (nv == 0) {
            if (GATHER && tid < 128) part[tile * 128 + tid] = 0.f;
            return;
        }
    }
    SCGIB_MARK(0);
    SCGIB_MARK_HWID();

    // the previous layer's deferred BN statistics: partial loads go out first
    FwdFin fin;
    float pend_gam = 0.f, pend_bet = 0.f;
    const int pend_ngr = static_cast<int>(((n + TM - 1) / TM + kGroup - 1) / kGroup);
    if (XFORM && pend.gpart) {
        pend_gam = pend.gamma[fin_channel()];
        pend_bet = pend.beta[fin_channel()];
        bn_fwd_fin_load<false>(pend.gpart, pend_ngr, 0, fin);
    }
    // weights: in flight during the gather, to LDS before the first GEMM; with
    // kLateWeights (gathering layers) issued after the gather's loads instead,
    // so the latency chain (BN partials -> neighbour indices -> rows) does not
    // share the start-of-kernel fetch burst with 32 KB of weights
    WeightRegs<DIN> wregs;
    constexpr bool late_w = kLateWeights && GATHER && !PRE;
    if (!late_w) load_weights<DIN>(w1, w2, wregs);
    if constexpr (PRE) {  // transfer_d folded: gather raw features, then agg0 = aggx Wt^T
        float *sXg = sPre, *sWt = sPre + TM * kPreLD;
        for (int idx = tid; idx < 32 * kPreF; idx += 256) {
            const int j = idx / kPreF, k = idx % kPreF;
            sWt[j * kPreLD + k] = pre.wt[j * pre.F + (k < pre.F ? k : 0)] * (k < pre.F ? 1.f : 0.f);
        }
        float ax[4];
        gather_x_rows(pre, rowptr, col, row0, nv, tid >> 4, tid & 15, ope, ax);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rr = (tid >> 4) + 16 * k;
            sXg[rr * kPreLD + (tid & 15)] = ax[k];
            if (rr < nv) pre.aggx[(row0 + rr) * kPreF + (tid & 15)] = ax[k];
        }
        __syncthreads();
        if (w < 2) {  // rows 32w..32w+31, all 32 outputs
            const f32x16 a0 = mma_nt<kPreF>(sXg + w * 32 * kPreLD, kPreLD, sWt, kPreLD, zero16());
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = w * 32 + acc_row(reg, l), cc = l & 31;
                sA[row * LDA + cc] = a0[reg];
                if (row < nv) agg_out[(row0 + row) * DIN + cc] = a0[reg];
            }
        }
    } else if constexpr (!GATHER) {  // dense: the input rows themselves
        constexpr int AQ = DIN / 4, AK = TM * AQ / 256;
        float4 va[AK];
#pragma unroll
        for (int k = 0; k < AK; ++k) {
            const int idx = tid + 256 * k, rr = idx / AQ, cq = idx % AQ;
            va[k] = ld_ok(reinterpret_cast<const float4 *>(h), (row0 + rr) * AQ + cq, row0 * AQ + cq,
                          rr < nv, make_float4(0.f, 0.f, 0.f, 0.f));
        }
#pragma unroll
        for (int k = 0; k < AK; ++k) {
            const int idx = tid + 256 * k, rr = idx / AQ, cq = idx % AQ;
            float *d = sA + rr * LDA + 4 * cq;
            d[0] = va[k].x; d[1] = va[k].y; d[2] = va[k].z; d[3] = va[k].w;
        }
    } else

    // gather: agg[v] = ope * x[v] + sum_{u->v} x[u], x = relu(scale*h + shift) if XFORM.
    // Each thread owns RPT rows of one 4-channel chunk; the loads of all its
    // rows are issued together (row pointers + self rows, then up to 4
    // neighbour indices per row, then those neighbour rows), so a tile costs
    // ~3 memory latencies instead of 3 per row.
    {
        constexpr int RPT = TM / RPP;
        const int c = tid % LPR, rbase = tid / LPR;
        float4 sc = make_float4(1.f, 1.f, 1.f, 1.f), sh = make_float4(0.f, 0.f, 0.f, 0.f);
        const float4 *h4 = reinterpret_cast<const float4 *>(h);
        float4 acc[RPT];
        GatherHead<RPT> hd;
        gather_head<RPT, RPP, LPR>(h4, rowptr, row0, nv, rbase, c, hd);  // in flight meanwhile
        // with a deferred BatchNorm finish ahead, the first neighbour-index
        // round goes out before it too (it needs only the row pointers)
        int32_t u0[RPT][4];
        const bool idx_early = XFORM && pend.gpart != nullptr;  // block-uniform
        if (idx_early) gather_idx0<RPT>(col, hd, u0);
        if (XFORM) {
            if (pend.gpart) {  // finish the previous layer's deferred BatchNorm statistics
                __shared__ float sScSh[128];
                double mean, M2;
                SCGIB_MARK(8);
                bn_fwd_final<false>(pend.gpart, n, pend_ngr, fin, mean, M2);
                SCGIB_MARK(9);
                const int fc = fin_channel();
                const bool lead = (tid & 63) < 16;
                const float2 ss = bn_fwd_publish(
                    fc, mean, M2, n, pend_gam, pend_bet, pend.eps, pend.momentum,
                    pend.running_mean, pend.running_var, pend.num_batches_tracked, pend.stat,
                    blockIdx.x == 0 && lead);
                if (lead) {
                    sScSh[fc] = ss.x;
                    sScSh[64 + fc] = ss.y;
                }
                __syncthreads();
                SCGIB_MARK(6);
                sc = make_float4(sScSh[4 * c], sScSh[4 * c + 1], sScSh[4 * c + 2], sScSh[4 * c + 3]);
                sh = make_float4(sScSh[64 + 4 * c], sScSh[65 + 4 * c], sScSh[66 + 4 * c],
                                 sScSh[67 + 4 * c]);
            } else {
                sc = ld4(in_scale + 4 * c);
                sh = ld4(in_shift + 4 * c);
            }
        }
        if (idx_early)
            gather_tail<RPT, LPR, XFORM, true>(h4, col, hd, c, ope, sc, sh, acc, u0);
        else
            gather_tail<RPT, LPR, XFORM>(h4, col, hd, c, ope, sc, sh, acc);
        if (late_w) load_weights<DIN>(w1, w2, wregs);  // before the agg stores (in-order vmcnt)
#pragma unroll
        for (int k = 0; k < RPT; ++k) {
            const int rr = rbase + k * RPP;
            // agg_out NULL (an agg-free layer: its backward never reads agg,
            // gin_bwd_statsz_k forms dW1 from the gathered dz1 instead)
            if (agg_out && rr < nv) st4_saved(agg_out + (row0 + rr) * DIN + 4 * c, acc[k]);
            float *d = sA + rr * LDA + 4 * c;
            d[0] = acc[k].x; d[1] = acc[k].y; d[2] = acc[k].z; d[3] = acc[k].w;
        }
    }
    store_weights<DIN>(wregs, sW1, sW2);
    __syncthreads();
    SCGIB_MARK(1);

    const int wr = w >> 1, wc = w & 1;
    const int ccol = wc * 32 + (l & 31);
    // z1 = agg W1^T + b1 ; r = relu(z1).  r_out NULL (the model path): r is
    // not stored — the backward recomputes it bit for bit from the saved agg
    // (gin_bwd5r_k, gin_bwd_k<.., RC>: this same MFMA chain, k pairs (2s,
    // 2s + 1) in order from zero, + b1, fmaxf)
    {
        f32x16 acc = mma_pf<DIN, false, false>(sA + wr * 32 * LDA, LDA, sW1 + wc * 32 * LDA, LDA, zero16());
        const float bias = b1[ccol];
        if constexpr (ALIAS) __syncthreads();  // every wave's reads of the agg tile and W1 are done
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = wr * 32 + acc_row(reg, l);
            const float v = fmaxf(acc[reg] + bias, 0.f);
            sR[row * LDH + ccol] = v;
            if (r_out && row < nv) st_saved(&r_out[(row0 + row) * 64 + ccol], v);
        }
    }
    __syncthreads();
    SCGIB_MARK(2);
    // z2 = r W2^T + b2 ; tile statistics of z2 (valid rows only)
    f32x16 acc = mma_pf<64, false, false>(sR + wr * 32 * LDH, LDH, sW2 + wc * 32 * LDH, LDH, zero16());
    const float bias2 = b2[ccol];
    float s = 0.f;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int row = wr * 32 + acc_row(reg, l);
        acc[reg] += bias2;
        if (row < nv) {
            if constexpr (RECON)  // write-through: the fused finish reads it from other CUs
                st_agent(&z2_out[(row0 + row) * 64 + ccol], acc[reg]);
            else
                st_saved(&z2_out[(row0 + row) * 64 + ccol], acc[reg]);
            s += acc[reg];
        }
    }
    if constexpr (!GATHER) {
        if constexpr (RECON) {  // Gram partial of the tile: out^T out (valid rows)
            // sA (the input tile) is dead since the first GEMM's barrier
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = wr * 32 + acc_row(reg, l);
                sA[row * LDH + ccol] = row < nv ? acc[reg] : 0.f;
            }
            __syncthreads();
            const f32x16 g = mma_pf<TM, true, true>(sA + wr * 32, LDH, sA + wc * 32, LDH, zero16());
            float *gs = rec.gslab + tile * 4096;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) st_agent(&gs[(wr * 32 + acc_row(reg, l)) * 64 + ccol], g[reg]);
            if (rec.fin_on) {  // block-uniform
                // publish: every wave's write-through stores drained, one arrival
                const unsigned ntiles = static_cast<unsigned>((n + TM - 1) / TM);
                block_arrive(rec.fin.cnt + 1, ntiles);
                SCGIB_MARK(6);
                // tiles past the virtual blocks (d_in = 64 past 256 tiles) only publish:
                // they never read the counter again, which the last virtual block resets
                if (tile >= kFinBlocks) return;
                if (tid == 0) {  // every tile published (bounded wait), then one acquire
                    const uint64_t t0 = wall_clock64();
                    while (__hip_atomic_load(rec.fin.cnt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ntiles) {
                        __builtin_amdgcn_s_sleep(1);
                        if (wall_clock64() - t0 > kFinWaitTicks) {  // loss -> NaN (recon_fin_block)
                            __hip_atomic_store(rec.fin.cnt + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            break;
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
                __syncthreads();
                SCGIB_MARK(7);
                ReconFin f = rec.fin;
                f.im = z2_out;  // (this kernel's own output, read through the pointer it wrote)
                recon_fin_block(static_cast<int>(tile), f, ncap, dims, true);
                SCGIB_MARK(10);
            }
        }
        return;
    }
    SCGIB_MARK(3);
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
        st_agent(part + tile * 128 + ccol, csum);
        st_agent(part + tile * 128 + 64 + ccol, sRed[0][ccol] + sRed[1][ccol]);
    }
    SCGIB_MARK(4);
    if (fz.counters) {
        bn_fwd_hier(part, n, tile, fz);
        SCGIB_MARK(5);
    }
}

// Batch mean / biased variance from the per-tile (sum, centred M2), fp64,
// two passes over the tile statistics with 8 tiles' loads in flight per
// thread (16 partitions x 64 channels, partitions combined in fixed order):
//   mean = sum_b S_b / N ;  M2 = sum_b [M2_b + (S_b - n_b mean)^2 / n_b]
// (exact decomposition of the centred sum of squares; n_b = 64 except the
// last tile, so only that one divides).
__device__ __forceinline__ double sum16_lds(double (*sh)[64], int c) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += sh[k][c];
    return s;
}

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
        for (int64_t t0 = p; t0 < ntiles; t0 += 16 * 8) {
            float S[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) S[u] = ld_ok(part, (t0 + 16 * u) * 128 + c, c, t0 + 16 * u < ntiles, 0.f);
#pragma unroll
            for (int u = 0; u < 8; ++u) a += static_cast<double>(S[u]);
        }
        sh[p][c] = a;
        __syncthreads();
        if (p == 0) s_mean[c] = sum16_lds(sh, c) / static_cast<double>(n);
        __syncthreads();
        mean = s_mean[c];
        double q = 0.0;
        for (int64_t t0 = p; t0 < ntiles; t0 += 16 * 8) {
            float S[8], Q[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t t = t0 + 16 * u;
                S[u] = ld_ok(part, t * 128 + c, c, t < ntiles, 0.f);
                Q[u] = ld_ok(part, t * 128 + 64 + c, 64 + c, t < ntiles, 0.f);
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int64_t t = t0 + 16 * u;
                if (t < ntiles) {
                    const int64_t nb = n - t * TM < TM ? n - t * TM : TM;
                    const double d = static_cast<double>(S[u]) - static_cast<double>(nb) * mean;
                    const double inv_nb = nb == TM ? 1.0 / TM : 1.0 / static_cast<double>(nb);
                    q += static_cast<double>(Q[u]) + d * d * inv_nb;
                }
            }
        }
        __syncthreads();
        sh[p][c] = q;
        __syncthreads();
        if (p == 0) M2 = sum16_lds(sh, c);
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
                                                       const int32_t *__restrict__ dims,
                                                       scgib_bn_pending pend) {
    const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    const int c = static_cast<int>(i & 15) * 4;
    float4 a, b;
    if (pend.gpart) {  // the last GIN layer's deferred statistics
        __shared__ float sSS[128];
        bn_pending_finish(pend, eff_count(dims, 0, n4 / 16), sSS);
        a = make_float4(sSS[c], sSS[c + 1], sSS[c + 2], sSS[c + 3]);
        b = make_float4(sSS[64 + c], sSS[65 + c], sSS[66 + c], sSS[67 + c]);
    } else {
        a = ld4(stat + 128 + c);
        b = ld4(stat + 192 + c);
    }
    // grid-stride (a multiple of 16 float4: the channel quad stays fixed)
    const int64_t nv4 = dims ? static_cast<int64_t>(dims[0]) * 16 : n4;
    for (int64_t k = i; k < n4; k += static_cast<int64_t>(gridDim.x) * 256)
        out[k] = k < nv4 ? xform4(z[k], a, b) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// ---------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------
// dy = dh * [scale z2 + shift > 0]; tile sums of dy and dy * xhat.
// GATHER: dh[v] = ope g[v] + sum_{u in out(v)} g[u]   (transposed aggregation
// of the next layer's d(agg), never materialised)
// SEG: dh[v] = (dh ? dh[v] : 0) + g_seg[seg[v]] — the encoder output feeds a
// segment-sum readout (dgl.sum_nodes) whose gradient is broadcast here
// instead of by a separate segment_broadcast launch.
// The previous layer's weight-gradient slab reduce folded into this launch:
// workgroups past the tile grid each sum one 64-column block of `fold`
// (every slab, fixed order: partition p = tid >> 6 of 4 takes slabs p, p + 4,
// ... in fp32 with 16 loads in flight, then the 4 partials in order in fp64).
// The stats tiles wait on gathers and leave HBM bandwidth idle; the reduce
// fills it, and the chain loses a separate reduce launch at its end.
constexpr int kFoldCols = 64;

__host__ __device__ inline int slab_fold_blocks(const scgib_slab_job &J) {
    return J.n_slabs > 0 ? static_cast<int>((J.width + kFoldCols - 1) / kFoldCols) : 0;
}

__device__ __forceinline__ void slab_fold_block(const scgib_slab_job &J, int b, float *red) {
    const int el = threadIdx.x & 63, sp = threadIdx.x >> 6;
    const int64_t e = static_cast<int64_t>(b) * kFoldCols + el;
    const int64_t stride = J.stride > 0 ? J.stride : J.width;
    const int64_t ec = e < J.width ? e : J.width - 1;  // clamped: loads stay unconditional
    float acc = 0.f;
    for (int b0 = sp; b0 < J.n_slabs; b0 += 4 * 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int sb = b0 + 4 * u;
            v[u] = J.slab[static_cast<int64_t>(sb < J.n_slabs ? sb : sp) * stride + ec];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += b0 + 4 * u < J.n_slabs ? v[u] : 0.f;
    }
    red[sp * 64 + el] = acc;
    __syncthreads();
    if (sp == 0 && e < J.width)
        J.out[e] = static_cast<float>(((static_cast<double>(red[el]) + red[64 + el]) + red[128 + el]) +
                                      red[192 + el]);
}

// The same over 32 columns x 8 slab partitions per block (partials combined
// in fp64, fixed order): for a job of many slabs — the agg-free statistics
// walk's dW1 partials, one per tile at small batches — folded into
// gin_bwd5z_k, whose grid leaves the CUs room for these blocks.
constexpr int kFold8Cols = 32;

__host__ __device__ inline int slab_fold8_blocks(const scgib_slab_job &J) {
    return J.n_slabs > 0 ? static_cast<int>((J.width + kFold8Cols - 1) / kFold8Cols) : 0;
}

__device__ __forceinline__ void slab_fold8_block(const scgib_slab_job &J, int b, float *red) {
    const int el = threadIdx.x & 31, sp = threadIdx.x >> 5;
    const int64_t e = static_cast<int64_t>(b) * kFold8Cols + el;
    const int64_t stride = J.stride > 0 ? J.stride : J.width;
    const int64_t ec = e < J.width ? e : J.width - 1;  // clamped: loads stay unconditional
    float acc = 0.f;
    for (int b0 = sp; b0 < J.n_slabs; b0 += 8 * 16) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int sb = b0 + 8 * u;
            v[u] = J.slab[static_cast<int64_t>(sb < J.n_slabs ? sb : sp) * stride + ec];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) acc += b0 + 8 * u < J.n_slabs ? v[u] : 0.f;
    }
    red[sp * 32 + el] = acc;
    __syncthreads();
    if (sp == 0 && e < J.width) {
        double t = red[el];
#pragma unroll
        for (int p = 1; p < 8; ++p) t += red[32 * p + el];
        J.out[e] = static_cast<float>(t);
    }
}

template <bool GATHER, bool SEG = false>
__global__ __launch_bounds__(256) void gin_bwd_stats_k(
    const float *__restrict__ dh, const int32_t *__restrict__ rowptr_t,
    const int32_t *__restrict__ col_t, float ope, const float *__restrict__ z2,
    const float *__restrict__ stat, int64_t ncap, float *__restrict__ dy_out,
    float *__restrict__ part, const int32_t *__restrict__ dims, BnBwdFuse bz,
    const float *__restrict__ g_seg, const int32_t *__restrict__ seg, scgib_slab_job fold) {
    static_assert(!(GATHER && SEG), "segment broadcast only on the dense input path");
    __shared__ float sRed[2][16][64];
    const int64_t ntile = (ncap + TM - 1) / TM;
    if (static_cast<int64_t>(blockIdx.x) >= ntile) {  // block-uniform: a folded reduce block
        slab_fold_block(fold, static_cast<int>(blockIdx.x - ntile), &sRed[0][0][0]);
        return;
    }
    const int64_t n = eff_count(dims, 0, ncap);
    const int tid = threadIdx.x, c = tid & 15, slot = tid >> 4;
    const int64_t tile = GATHER ? tile_of_block(ntile) : static_cast<int64_t>(blockIdx.x);
    const int64_t row0 = tile * TM;
    const float4 mean = ld4(stat + 4 * c), istd = ld4(stat + 64 + 4 * c);
    const float4 sc = ld4(stat + 128 + 4 * c), sh = ld4(stat + 192 + 4 * c);
    const float4 *g4 = reinterpret_cast<const float4 *>(dh);
    const int nv = static_cast<int>(n - row0 < TM ? (n - row0 > 0 ? n - row0 : 0) : TM);
    if (nv == 0) {  // capacity mode: a tile of padding rows (block-uniform)
        for (int rr = slot; rr < TM && row0 + rr < ncap; rr += 16)
            st4(dy_out + (row0 + rr) * 64 + 4 * c, make_float4(0.f, 0.f, 0.f, 0.f));
        return;
    }
    SCGIB_MARK(0);
    SCGIB_MARK_HWID();
    float4 g[4];
    if (GATHER) {
        gather_rows<4, 16, 16, false>(g4, rowptr_t, col_t, row0, nv, slot, c, ope, sc, sh, g);
    } else if (SEG) {
        int32_t sg[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rr = slot + 16 * k;
            sg[k] = seg[row0 + (rr < nv ? rr : nv - 1)];
        }
        const float4 *gs4 = reinterpret_cast<const float4 *>(g_seg);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rr = slot + 16 * k;
            const float4 b = gs4[static_cast<int64_t>(sg[k]) * 16 + c];
            g[k] = dh ? add4(g4[(row0 + (rr < nv ? rr : nv - 1)) * 16 + c], b) : b;
        }
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rr = slot + 16 * k;
            g[k] = g4[(row0 + (rr < nv ? rr : nv - 1)) * 16 + c];
        }
    }
    // rows past nv: the gather duplicated row nv - 1; z is read at that row
    // and dy is multiplied by 0 (no predicate, so the loads stay batched)
    float4 z[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int rr = slot + 16 * k;
        z[k] = ld4(z2 + (row0 + (rr < nv ? rr : nv - 1)) * 64 + 4 * c);
    }
    float4 sdy = make_float4(0.f, 0.f, 0.f, 0.f), sdx = sdy;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int rr = slot + 16 * k;
        const int64_t v = row0 + rr;
        const float valid = rr < nv ? 1.f : 0.f;
        const float4 zz = z[k], gg = g[k];
        const float4 dy = make_float4((sc.x * zz.x + sh.x > 0.f ? gg.x : 0.f) * valid,
                                      (sc.y * zz.y + sh.y > 0.f ? gg.y : 0.f) * valid,
                                      (sc.z * zz.z + sh.z > 0.f ? gg.z : 0.f) * valid,
                                      (sc.w * zz.w + sh.w > 0.f ? gg.w : 0.f) * valid);
        if (v < ncap) st4(dy_out + v * 64 + 4 * c, dy);
        sdy = add4(sdy, dy);
        sdx = add4(sdx, make_float4(dy.x * (zz.x - mean.x) * istd.x, dy.y * (zz.y - mean.y) * istd.y,
                                    dy.z * (zz.z - mean.z) * istd.z, dy.w * (zz.w - mean.w) * istd.w));
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
        st_agent(part + tile * 128 + which * 64 + ch, s);
    }
    SCGIB_MARK(1);
    if (bz.counters) {
        bn_bwd_hier(part, n, tile, bz);
        SCGIB_MARK(2);
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
    for (int64_t t0 = p; t0 < ntiles; t0 += 16 * 8) {
        float A[8], Bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t t = t0 + 16 * u;
            A[u] = ld_ok(part, t * 128 + c, c, t < ntiles, 0.f);
            Bv[u] = ld_ok(part, t * 128 + 64 + c, 64 + c, t < ntiles, 0.f);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            a += static_cast<double>(A[u]);
            b += static_cast<double>(Bv[u]);
        }
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
// BN = false is the backward of the dense head MLP: dz2 = dy (the gradient
// of the MLP output); z2 / stat / coef are not read.
// PRE: layer 0 with transfer_d folded in (see gather_x_rows): d(agg0) is not
// stored; dWt += d(agg0)^T aggx is accumulated (slab tail of 32 x 16 floats).
// RC (PRE only): r is not read — the forward did not store it — but
// recomputed per tile from the agg tile (staged in the d(agg0) buffer, dead
// until the tile's last products) with the forward's own call, mma_pf<32>
// over the same [64][33] layouts, + b1, fmaxf: bitwise the forward's r;
// rows past the tile's valid rows are 0, as the stored path loads them.
// WG = false (PRE only): the layer's W1 / W2 / biases are frozen (the
// fine-tune freezing quirk) — dr and d(agg0) by the same chains as with WG
// (mma_pf instead of mma_pf2: one product per call, the same k order), no
// dW1 / dW2 / db products or slab part, no agg tile; dWt is still formed.
template <int DIN, bool BN = true, bool PRE = false, bool RECON = false, bool RC = false,
          bool WG = true>
__global__ __launch_bounds__(256, (DIN <= 64 && !RECON ? 2 : 1)) void gin_bwd_k(
    const float *__restrict__ dy, const float *__restrict__ z2, const float *__restrict__ r,
    const float *__restrict__ agg, const float *__restrict__ stat,
    const float *__restrict__ coef, const float *__restrict__ w1, const float *__restrict__ w2,
    int64_t ncap, int64_t ntiles, float *__restrict__ dagg_out, float *__restrict__ slab,
    const int32_t *__restrict__ dims, const float *__restrict__ aggx, scgib_bn_bwd_pending pend,
    ReconArgs rec, int pre_f = kPreF, const float *__restrict__ b1 = nullptr, int nsplit = 1) {
    static_assert(!PRE || DIN == 32, "transfer_d fold: layer 0 only");
    static_assert(!RC || PRE, "r recomputed in the layer-0 backward only (gin_bwd5r_k: d_in = 64)");
    static_assert(WG || (PRE && !RC), "frozen weights: the layer-0 stored-r backward only");
    static_assert(!RECON || !BN, "the recon backward is fused into the dense head MLP");
    const int64_t n = eff_count(dims, 0, ncap);
    constexpr int LDA = DIN + 1;
    constexpr int SLAB = 64 * 64 + 64 * DIN + 128 + (PRE ? kPreSlab : 0);
    constexpr int LDP = 33;  // [64][32] tiles of d(agg0) and zero-padded aggx
    __shared__ float sPre[PRE ? 2 * TM * LDP : 1];
    float *const sPD = sPre, *const sPX = sPre + TM * LDP;
    // r is dead once dz1 is formed, so the agg tile reuses its buffer: 66.5 KB
    // for DIN <= 64, two workgroups per CU (loads of one overlap the other's MFMA)
    constexpr int RA = (LDA > LDH ? LDA : LDH);
    // 16-byte aligned: the contrastive workgroups read them by ds_read_b128
    __shared__ __attribute__((aligned(16))) float sD[TM * LDH];   // dz2, then dz1
    __shared__ __attribute__((aligned(16))) float sRA[TM * RA];   // r, then agg
    __shared__ __attribute__((aligned(16))) float sW1[64 * LDA];
    __shared__ __attribute__((aligned(16))) float sW2[64 * LDH];
    __shared__ float sG[RECON ? 64 * LDH : 1];  // Gram matrix of the recon loss
    float *const sR = sRA, *const sA = sRA;
    unsigned gsz = gridDim.x;  // workgroups of the tile loop
    if constexpr (RECON && DIN == 128) {  // the pretraining head (interaction map width)
        static_assert(TM * RA >= CT * CLD && 64 * LDA >= CT * CLD && TM * LDH >= kContrastBwdW &&
                      64 * LDH >= CT, "contrastive buffers in sRA / sW1 / sD / sW2");
        if (rec.con.B > 0) {
            gsz = static_cast<unsigned>(rec.con.nmain);
            if (blockIdx.x >= gsz) {  // block-uniform
                const int64_t b = blockIdx.x - gsz, nrb = contrast_row_blocks(rec.con.B);
                SCGIB_MARK(0);
                contrast_bwd_body(rec.con, b % nrb, static_cast<int>(b / nrb), sRA, sW1, sD, sW2);
                SCGIB_MARK(5);
                return;
            }
        }
    }
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int wr = w >> 1, wc = w & 1;
    // nsplit 2 (the dense d_in = 128 MLP on few tiles: scgib_mlp2_bwd): two
    // workgroups per tile, each forming half of the dW1 / d(agg) column blocks
    // (its q1 = half), after the same dz2 / dz1 (the same bits: mma_pf is
    // mma_pf2's second product); half 0 alone adds dW2 / db2 / db1.  Every
    // workgroup writes its whole slab row (zeros where the other half adds).
    const int half = static_cast<int>(blockIdx.x) % nsplit;
    SCGIB_MARK(0);
    SCGIB_MARK_HWID();
    [[maybe_unused]] const float rc_bias = RC ? b1[wc * 32 + (l & 31)] : 0.f;
    [[maybe_unused]] float rscale = 0.f;  // recon: g / N
    if constexpr (RECON) {
        stage_matrix<64>(rec.gram, sG);
        rscale = *rec.g_loss / static_cast<float>(n);
    }
    // this layer's deferred BN-backward sums: partial loads go out with the weights
    BwdFin bfin;
    const int pend_ngr = static_cast<int>(((n + TM - 1) / TM + kGroup - 1) / kGroup);
    if (BN && pend.gpart) bn_bwd_fin_load<false>(pend.gpart, pend_ngr, 0, bfin);
    // weights: in flight during the BN finish and the first tile's loads
    // (PRE, the register-heaviest variant: staged at once, no spill)
    WeightRegs<DIN> wregs;
    load_weights<DIN>(w1, w2, wregs);
    bool wpending = true;
    if constexpr (PRE) {
        store_weights<DIN>(wregs, sW1, sW2);
        wpending = false;
    }
    const int ch = tid & 63, q = tid >> 6;  // column-sum roles: channel, row quarter
    // staging roles: 4-channel chunk c4, rows rs + 16 k
    const int c4 = tid & 15, rs = tid >> 4;
    const float4 zero = make_float4(0.f, 0.f, 0.f, 0.f);
    constexpr int NSUB1 = 2 * (DIN / 32);  // 32x32 sub-tiles of dW1 / d(agg)
    constexpr int NW1 = (NSUB1 + 3) / 4;   // per wave
    f32x16 accW2 = zero16(), accW1[NW1];
#pragma unroll
    for (int q1 = 0; q1 < NW1; ++q1) accW1[q1] = zero16();
    f32x16 accWt = zero16();
    if (PRE)  // columns 16..31 of the aggx tile stay zero
        for (int idx = tid; idx < TM * 16; idx += 256) sPX[(idx >> 4) * LDP + 16 + (idx & 15)] = 0.f;
    float db2 = 0.f, db1 = 0.f;
    constexpr int AQ = DIN / 4, AK = TM * AQ / 256;  // agg tile: float4 per row, per thread
    // (software-pipelining the next tile's loads under this tile's GEMMs
    // measured 1-2 % slower: 20-44 bytes/lane of scratch at 2 workgroups/CU,
    // and at QM9 B512 nearly every workgroup owns a single tile)
    float4 vz[4], vd[4], vr[4], va[AK], vx = zero;
    auto load_rows = [&](int64_t t) {
        const int64_t r0 = t * TM;
        const int m = static_cast<int>(n - r0 < TM ? (n - r0 > 0 ? n - r0 : 0) : TM);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rr = rs + 16 * k;
            const int64_t o = (r0 + rr) * 16 + c4, so = r0 * 16 + c4;
            if (BN) vz[k] = ld_ok(reinterpret_cast<const float4 *>(z2), o, so, rr < m, zero);
            else vz[k] = zero;
            if (!RECON) vd[k] = ld_ok(reinterpret_cast<const float4 *>(dy), o, so, rr < m, zero);
            if (!RC) vr[k] = ld_ok(reinterpret_cast<const float4 *>(r), o, so, rr < m, zero);
        }
        if (PRE)
            vx = ld_ok(reinterpret_cast<const float4 *>(aggx), (r0 + (tid >> 2)) * 4 + (tid & 3),
                       r0 * 4 + (tid & 3), (tid >> 2) < m, zero);
    };
    auto load_agg = [&](int64_t t) {
        if constexpr (!WG) return;  // agg is read only by dW1
        const int64_t r0 = t * TM;
        const int m = static_cast<int>(n - r0 < TM ? (n - r0 > 0 ? n - r0 : 0) : TM);
#pragma unroll
        for (int k = 0; k < AK; ++k) {
            const int idx = tid + 256 * k, rr = idx / AQ, cq = idx % AQ;
            va[k] = ld_ok(reinterpret_cast<const float4 *>(agg), (r0 + rr) * AQ + cq, r0 * AQ + cq,
                          rr < m, zero);
        }
    };
    float4 s_mean = zero, s_istd = zero, s_sc = zero, c1 = zero, c2 = zero;
    if (BN) {
        s_mean = ld4(stat + 4 * c4);
        s_istd = ld4(stat + 64 + 4 * c4);
        s_sc = ld4(stat + 128 + 4 * c4);
        if (!pend.gpart) {
            c1 = ld4(coef + 4 * c4);
            c2 = ld4(coef + 64 + 4 * c4);
        } else {  // finish the sums; workgroup 0 writes dgamma, dbeta
            __shared__ float sCoef[128];
            const double tot = bn_bwd_final<false>(pend.gpart, pend_ngr, bfin);
            const int cs = bfin_index();
            const bool lead = (tid & 63) < 32, w0 = blockIdx.x == 0 && lead;
            const float cf = bn_bwd_publish(cs, tot, n, pend.training, w0 ? pend.dgamma : nullptr,
                                            w0 ? pend.dbeta : nullptr, nullptr);
            if (lead) sCoef[cs] = cf;
            __syncthreads();
            c1 = make_float4(sCoef[4 * c4], sCoef[4 * c4 + 1], sCoef[4 * c4 + 2], sCoef[4 * c4 + 3]);
            c2 = make_float4(sCoef[64 + 4 * c4], sCoef[65 + 4 * c4], sCoef[66 + 4 * c4],
                             sCoef[67 + 4 * c4]);
        }
    }
    for (int64_t tile = blockIdx.x / nsplit; tile < ntiles; tile += gsz / nsplit) {
        const int64_t row0 = tile * TM;
        const int nv = static_cast<int>(n - row0 < TM ? (n - row0 > 0 ? n - row0 : 0) : TM);
        if (dims) {  // capacity mode: zero this tile's padded rows of d(agg)
            const int ncr = static_cast<int>(ncap - row0 < TM ? ncap - row0 : TM);
            if (!PRE)
                for (int idx = nv * DIN + tid; idx < ncr * DIN; idx += 256) dagg_out[row0 * DIN + idx] = 0.f;
            // block-uniform; every later tile of this workgroup is empty too,
            // so the registers are never read again
            if (nv == 0) continue;
        }
        load_rows(tile);
        // recon: own IM rows (vd) and nb = ((A + A^T) IM) rows, same layout
        float4 nb[4];
        if constexpr (RECON) {
            const float4 *im4 = reinterpret_cast<const float4 *>(rec.im);
            const float4 one = make_float4(1.f, 1.f, 1.f, 1.f);
            GatherHead<4> hd;
            gather_head<4, 16, 16>(im4, rec.rowptr, row0, nv, rs, c4, hd);
            gather_tail<4, 16, false>(im4, rec.col, hd, c4, 0.f, one, zero, nb);
            if (rec.rowptr_t) {
                GatherHead<4> ht;
                float4 nt[4];
                gather_head<4, 16, 16>(im4, rec.rowptr_t, row0, nv, rs, c4, ht);
                gather_tail<4, 16, false>(im4, rec.col_t, ht, c4, 0.f, one, zero, nt);
#pragma unroll
                for (int k = 0; k < 4; ++k) nb[k] = add4(nb[k], nt[k]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) nb[k] = add4(nb[k], nb[k]);  // A symmetric
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) vd[k] = rs + 16 * k < nv ? hd.self[k] : zero;
        }
        load_agg(tile);
        if (wpending) {  // first tile: its loads are in flight now
            store_weights<DIN>(wregs, sW1, sW2);
            wpending = false;
        }
        __syncthreads();  // previous tile's LDS reads are done
        if (PRE) {
            float *px = sPX + (tid >> 2) * LDP + 4 * (tid & 3);
            px[0] = vx.x; px[1] = vx.y; px[2] = vx.z; px[3] = vx.w;
        }
        if constexpr (RC) {  // the agg tile for the r recompute (in the d(agg0) buffer)
            static_assert(LDP == LDA, "the forward's agg tile layout");
#pragma unroll
            for (int k = 0; k < AK; ++k) {
                const int idx = tid + 256 * k, rr = idx / AQ, cq = idx % AQ;
                float *pa = sPD + rr * LDP + 4 * cq;
                pa[0] = va[k].x; pa[1] = va[k].y; pa[2] = va[k].z; pa[3] = va[k].w;
            }
        }
        // dz2 = scale (dy - c1 - xhat c2); rows past n are zero
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int rr = rs + 16 * k;
            float4 d = zero;
            if (!BN) {
                d = vd[k];
            } else if (rr < nv) {
                d.x = s_sc.x * (vd[k].x - c1.x - (vz[k].x - s_mean.x) * s_istd.x * c2.x);
                d.y = s_sc.y * (vd[k].y - c1.y - (vz[k].y - s_mean.y) * s_istd.y * c2.y);
                d.z = s_sc.z * (vd[k].z - c1.z - (vz[k].z - s_mean.z) * s_istd.z * c2.z);
                d.w = s_sc.w * (vd[k].w - c1.w - (vz[k].w - s_mean.w) * s_istd.w * c2.w);
            }
            float *pd = sD + rr * LDH + 4 * c4, *pr = sR + rr * LDH + 4 * c4;
            pd[0] = d.x; pd[1] = d.y; pd[2] = d.z; pd[3] = d.w;
            if (!RC) { pr[0] = vr[k].x; pr[1] = vr[k].y; pr[2] = vr[k].z; pr[3] = vr[k].w; }
        }
        __syncthreads();
        if constexpr (RC) {  // r = relu(agg W1^T + b1): the forward's GEMM1, rows >= nv zero
            const f32x16 z = mma_pf<DIN, false, false>(sPD + wr * 32 * LDP, LDP, sW1 + wc * 32 * LDA, LDA, zero16());
            const int cc = wc * 32 + (l & 31);
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = wr * 32 + acc_row(reg, l);
                sR[row * LDH + cc] = row < nv ? fmaxf(z[reg] + rc_bias, 0.f) : 0.f;
            }
            __syncthreads();
        }
        if constexpr (RECON) {  // sD = IM tile -> dz2 = d IM = (g/N) (4 IM G - 2 nb)
            const f32x16 p = mma_pf<64, false, true>(sD + wr * 32 * LDH, LDH, sG + wc * 32, LDH, zero16());
            __syncthreads();
#pragma unroll
            for (int reg = 0; reg < 16; ++reg)
                sD[(wr * 32 + acc_row(reg, l)) * LDH + wc * 32 + (l & 31)] = 4.f * rscale * p[reg];
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int rr = rs + 16 * k;
                if (rr < nv) {  // rows past nv: IM = 0 there, so p = 0 already
                    float *pd = sD + rr * LDH + 4 * c4;
                    pd[0] -= 2.f * rscale * nb[k].x; pd[1] -= 2.f * rscale * nb[k].y;
                    pd[2] -= 2.f * rscale * nb[k].z; pd[3] -= 2.f * rscale * nb[k].w;
                }
            }
            __syncthreads();
        }
        if (tile == blockIdx.x / nsplit) SCGIB_MARK(1);
        // dW2 += dz2^T r  (sub-tile j-block wr, k-block wc)
        // dr = dz2 W2  (rows wr, cols wc); the two products alternate
        f32x16 dr = zero16();
        if (WG && half == 0) {
            mma_pf2<64, true, true, false, true>(sD + wr * 32, LDH, sR + wc * 32, LDH, accW2,
                                                 sD + wr * 32 * LDH, LDH, sW2 + wc * 32, LDH, dr);
            db2 = col_sum16(db2, sD + q * LDH + ch, 4 * LDH);
        } else {
            dr = mma_pf<64, false, true>(sD + wr * 32 * LDH, LDH, sW2 + wc * 32, LDH, zero16());
        }
        __syncthreads();  // all reads of dz2 done
        // dz1 = dr * [r > 0]  -> sD
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int row = wr * 32 + acc_row(reg, l), cc = wc * 32 + (l & 31);
            sD[row * LDH + cc] = sR[row * LDH + cc] > 0.f ? dr[reg] : 0.f;
        }
        __syncthreads();  // r is dead: the agg tile (held in registers) takes its buffer
        if (tile == blockIdx.x / nsplit) SCGIB_MARK(2);
        // RC: the agg tile is already in the d(agg0) buffer (the r recompute's
        // operand), the dead r buffer takes d(agg0) instead — same layouts
        float *const aggT = RC ? sPD : sA, *const daggT = RC ? sRA : sPD;
        if constexpr (!RC && WG) {
#pragma unroll
            for (int k = 0; k < AK; ++k) {
                const int idx = tid + 256 * k, rr = idx / AQ, cq = idx % AQ;
                float *pa = sA + rr * LDA + 4 * cq;
                pa[0] = va[k].x; pa[1] = va[k].y; pa[2] = va[k].z; pa[3] = va[k].w;
            }
            __syncthreads();
        }
        if (WG && half == 0) db1 = col_sum16(db1, sD + q * LDH + ch, 4 * LDH);
        // dW1 += dz1^T agg  (64 x DIN) ; d(agg) = dz1 W1  (TM x DIN)
#pragma unroll
        for (int q1 = 0; q1 < NW1; ++q1) {
            const int sub = w + 4 * q1;
            if (sub < NSUB1 && (nsplit == 1 || q1 == half)) {  // (wave-uniform)
                const int jb = sub & 1, kb = sub >> 1;  // j-block (rows of dW1 / d(agg)), k-block
                f32x16 da = zero16();
                if constexpr (WG)
                    mma_pf2<64, true, true, false, true>(sD + jb * 32, LDH, aggT + kb * 32, LDA, accW1[q1],
                                                         sD + jb * 32 * LDH, LDH, sW1 + kb * 32, LDA, da);
                else
                    da = mma_pf<64, false, true>(sD + jb * 32 * LDH, LDH, sW1 + kb * 32, LDA, zero16());
#pragma unroll
                for (int reg = 0; reg < 16; ++reg) {
                    const int row = jb * 32 + acc_row(reg, l);
                    if (PRE) daggT[row * LDP + kb * 32 + (l & 31)] = da[reg];
                    else if (row < nv) dagg_out[(row0 + row) * DIN + kb * 32 + (l & 31)] = da[reg];
                }
            }
        }
        if (PRE) {  // dWt += d(agg0)^T aggx (32 x 32, columns >= 16 are zero)
            __syncthreads();
            if (w == 0) accWt = mma_tn<TM>(daggT, LDP, sPX, LDP, accWt);
        }
        if (tile == blockIdx.x / nsplit) SCGIB_MARK(3);
    }
    // per-workgroup slab
    float *sl = slab + static_cast<int64_t>(blockIdx.x) * SLAB;
    if constexpr (!WG) {  // frozen W1 / W2: only the dWt part
        if (w == 0) {
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int i = acc_row(reg, l), j = l & 31;
                if (j < pre_f) sl[64 * 64 + 64 * DIN + 128 + i * pre_f + j] = accWt[reg];
            }
        }
        SCGIB_MARK(4);
        return;
    }
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int j = wr * 32 + acc_row(reg, l), k = wc * 32 + (l & 31);
        sl[j * 64 + k] = accW2[reg];
    }
#pragma unroll
    for (int q1 = 0; q1 < NW1; ++q1) {
        const int sub = w + 4 * q1;
        if (sub < NSUB1) {
            const int jb = sub & 1, kb = sub >> 1;
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int j = jb * 32 + acc_row(reg, l), kk = kb * 32 + (l & 31);
                sl[64 * 64 + j * DIN + kk] = accW1[q1][reg];
            }
        }
    }
    if (PRE && w == 0) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int i = acc_row(reg, l), j = l & 31;
            // d Wt as [32][F] row-major: a column range of the slab reduces
            // straight into the contiguous transfer_d.weight gradient
            if (j < pre_f) sl[64 * 64 + 64 * DIN + 128 + i * pre_f + j] = accWt[reg];
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
    SCGIB_MARK(4);
}


// ---------------------------------------------------------------------------
// gin_bwd5_k: the GIN layer backward (BN, d_in = 64) on 32-row sub-tiles,
// TWO workgroups per CU (63 KB LDS, <= 256 VGPRs).
//
// (Round 2 replaced gin_bwd2_k with it: 64-row tiles at one workgroup per
// CU, ~1.7 tiles per CU at QM9 B512, whose per-tile phases left the matrix
// pipe idle ~40 % of a tile and whose dword operand reads ran the GEMMs at
// ~80 % of the MFMA rate; phase trace r02.)  Here:
//   * 32-row sub-tiles, two workgroups per CU: one workgroup's non-MFMA
//     phases run under the other's MFMAs; ~3.4 sub-tiles per CU balance
//     better than 1.7 tiles;
//   * no K split: waves take whole products, 32 MFMAs per wave and pair:
//       pair A: waves 0,1 (N): dr block q = dz2 W2[:, 32q..] (K = 64, one
//               chain), dz1 = dr [r > 0] written straight from the accumulator;
//               waves 2,3 (T): dW2 rows 32q.. += dz2^T r (two blocks, K = 32 rows)
//       pair B: N: dW1 rows 32q.. += dz1^T agg;  T: d(agg) block q = dz1 W1[:, 32q..]
//   * every MFMA operand is fed four k values per ds_read_b128 (mma_rk4 /
//     mma_kk4x2, permuted k order): NN products read dz row-major and take
//     the wave's 32-column weight block from 32 VGPRs held for the whole
//     kernel (no weight image in LDS); TN products read transposed dz, r and
//     agg images [col][row];
//   * the next sub-tile's rows are loaded into registers before pair A and
//     written to the r^T / agg^T images once their last reader has passed a
//     barrier (r after pair A, agg after pair B): three barriers per sub-tile.
// The elementwise steps own one column and eight rows per thread (c = tid &
// 63, rows 8 w..8 w+7), so the transposed images are written as float4 runs
// and the row-major dz images as conflict-free dwords.
// LDS: dz2, dz1 row-major + transposed, r^T, agg^T, d(agg) staging = 63 KB.
// ---------------------------------------------------------------------------
constexpr int SM = 32;   // rows per sub-tile
constexpr int LDR = 68;  // row-major 64-wide images (= 4 mod 64: b128 reads conflict free)
constexpr int LDT = 36;  // transposed [64][32] images (rows k-contiguous)

// WG = false: a frozen layer (the fine-tune freezing quirk, models.py:424-434:
// no parameter of it takes a gradient) — only the data-gradient chains run,
// dr and d(agg), each exactly as with WG (bitwise the same d(agg)); the
// dW products, the agg rows (read only by dW1), the transposed dz images
// and the slab are skipped.
template <int DIN, bool WG = true>
__global__ __launch_bounds__(256, 2) void gin_bwd5_k(
    const float *__restrict__ dy, const float *__restrict__ z2, const float *__restrict__ r,
    const float *__restrict__ agg, const float *__restrict__ stat,
    const float *__restrict__ coef, const float *__restrict__ w1, const float *__restrict__ w2,
    int64_t ncap, int64_t nsub, float *__restrict__ dagg_out, float *__restrict__ slab,
    const int32_t *__restrict__ dims, scgib_bn_bwd_pending pend) {
    static_assert(DIN == 64 && SM == 32, "64-wide rows, 32-row sub-tiles");
    constexpr int SLAB = 64 * 64 + 64 * DIN + 128;
    __shared__ __attribute__((aligned(16))) float sD[SM * LDR];   // dz2 [row][k]
    __shared__ __attribute__((aligned(16))) float sDT[64 * LDT];  // dz2 [col][row]
    __shared__ __attribute__((aligned(16))) float sE[SM * LDR];   // dz1
    __shared__ __attribute__((aligned(16))) float sET[64 * LDT];
    __shared__ __attribute__((aligned(16))) float sRT[64 * LDT];  // r [col][row]
    __shared__ __attribute__((aligned(16))) float sAT[DIN * LDT]; // agg [col][row]
    __shared__ float sG[SM * LDH];                                 // d(agg) staging
    __shared__ float sCoef[128];
    const int64_t n = eff_count(dims, 0, ncap);
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int kk = l >> 5, li = l & 31;
    const bool nw = w < 2;  // wave-uniform role: N (dr, dW1) or T (dW2, d(agg))
    const int q = w & 1;    // the role's 32-wide block
    const int c = l;        // elementwise: column c, rows 8 w .. 8 w + 7
    const int64_t last = ncap - 1;
    const int64_t G = gridDim.x;
    SCGIB_MARK(0);
    SCGIB_MARK_HWID();
    BwdFin bfin;
    const int pend_ngr = static_cast<int>(((n + TM - 1) / TM + kGroup - 1) / kGroup);
    if (pend.gpart) bn_bwd_fin_load<false>(pend.gpart, pend_ngr, 0, bfin);
    const float s_mean = stat[c], s_istd = stat[64 + c], s_sc = stat[128 + c];
    float c1 = 0.f, c2 = 0.f;
    if (!pend.gpart) {
        c1 = coef[c];
        c2 = coef[64 + c];
    }
    // the wave's weight block: N waves W2[:, 32q..] (dr), T waves W1[:, 32q..] (d(agg))
    float wreg[32];
    {
        const float *wm = nw ? w2 : w1;
#pragma unroll
        for (int s = 0; s < 32; ++s) wreg[s] = wm[kperm(s, kk) * 64 + q * 32 + li];
    }
    float nx[4][8];  // a sub-tile's column c, rows 8 w + i: [0] dy, [1] z2, [2] r, [3] agg
    auto load_sub = [&](int64_t s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // in order of use: r, agg, then dy / z2
            int64_t row = s * SM + 8 * w + i;
            row = row < last ? row : last;
            nx[2][i] = r[row * 64 + c];
        }
        if constexpr (WG) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                int64_t row = s * SM + 8 * w + i;
                row = row < last ? row : last;
                nx[3][i] = agg[row * DIN + c];
            }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int64_t row = s * SM + 8 * w + i;
            row = row < last ? row : last;
            nx[0][i] = dy[row * 64 + c];
            nx[1][i] = z2[row * 64 + c];
        }
    };
    auto put_t = [&](float *img, int a) {  // column c, rows 8w..8w+7 -> [c][row]
        float4 *p = reinterpret_cast<float4 *>(img + c * LDT + 8 * w);
        p[0] = make_float4(nx[a][0], nx[a][1], nx[a][2], nx[a][3]);
        p[1] = make_float4(nx[a][4], nx[a][5], nx[a][6], nx[a][7]);
    };
    auto rows_of = [&](int64_t s) {
        const int64_t v = n - s * SM;
        return static_cast<int>(v < SM ? (v > 0 ? v : 0) : SM);
    };
    auto zero_pad = [&](int64_t s, int from) {
        const int64_t row0 = s * SM;
        const int ncr = static_cast<int>(ncap - row0 < SM ? ncap - row0 : SM);
        for (int idx = from * DIN + tid; idx < ncr * DIN; idx += 256) dagg_out[row0 * DIN + idx] = 0.f;
    };
    int64_t s = blockIdx.x;
    int nv = s < nsub ? rows_of(s) : 0;
    if (nv > 0) load_sub(s);
    if (pend.gpart) {  // finish the BN-backward sums; workgroup 0 writes dgamma, dbeta
        const double tot = bn_bwd_final<false>(pend.gpart, pend_ngr, bfin);
        const int cs = bfin_index();
        const bool lead = (tid & 63) < 32, w0 = blockIdx.x == 0 && lead;
        const float cf = bn_bwd_publish(cs, tot, n, pend.training, w0 ? pend.dgamma : nullptr,
                                        w0 ? pend.dbeta : nullptr, nullptr);
        if (lead) sCoef[cs] = cf;
    }
    if (nv > 0) {
        put_t(sRT, 2);
        if (WG) put_t(sAT, 3);
    }
    // the weight registers complete here: a load still counted at the loop
    // entry makes hipcc wait vmcnt(0..3) at their uses in EVERY iteration
    // (then for the next sub-tile's rows)
    vm_wait_all();
    __syncthreads();
    if (pend.gpart) {
        c1 = sCoef[c];
        c2 = sCoef[64 + c];
    }
    const float k1 = s_istd * c2;  // dz2 = sc (dy - c1 - (z2 - mean) istd c2)
    SCGIB_MARK(1);
    // N waves: dW1 blocks (q, 0), (q, 1) and db1; T waves: dW2 blocks and db2
    f32x16 accA = zero16(), accB = zero16();
    float dbias = 0.f;
    for (int it = 0; s < nsub; s += G, ++it) {
        if (nv == 0) {  // capacity tail: this and every later sub-tile is padding
            for (int64_t t = s; t < nsub; t += G) zero_pad(t, rows_of(t));
            break;
        }
        {   // dz2 (rows past nv zero) -> sD row-major and sDT transposed
            float d[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float v = s_sc * (nx[0][i] - c1 - (nx[1][i] - s_mean) * k1);
                d[i] = 8 * w + i < nv ? v : 0.f;
                sD[(8 * w + i) * LDR + c] = d[i];
            }
            if constexpr (WG) {
                float4 *p = reinterpret_cast<float4 *>(sDT + c * LDT + 8 * w);
                p[0] = make_float4(d[0], d[1], d[2], d[3]);
                p[1] = make_float4(d[4], d[5], d[6], d[7]);
            }
        }
        const int64_t next = s + G;
        const int next_nv = next < nsub ? rows_of(next) : 0;  // block-uniform
        if (next_nv > 0) load_sub(next);  // in flight during both product pairs
        lds_barrier();  // dz2 complete
        if (it == 0) SCGIB_MARK(2);
        if (nw) {  // dr block q, dz1 = dr [r > 0] -> sE, sET (mask by multiplication)
            const f32x16 dr = mma_rk4<8>(sD + li * LDR + 4 * kk, wreg, zero16());
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = acc_row(reg, l), col = q * 32 + li;
                const float v = dr[reg] * (sRT[col * LDT + row] > 0.f ? 1.f : 0.f);
                sE[row * LDR + col] = v;
                if (WG) sET[col * LDT + row] = v;
            }
        } else if constexpr (WG) {   // dW2 rows 32q.. += dz2^T r (db2 from the A operand)
            mma_kk4x2<4>(sDT + (q * 32 + li) * LDT + 4 * kk, sRT + li * LDT + 4 * kk,
                         sRT + (32 + li) * LDT + 4 * kk, accA, accB, dbias);
        }
        lds_barrier();  // dz1 complete; r and dz2 consumed
        if (it == 0) SCGIB_MARK(3);
        if (next_nv > 0) put_t(sRT, 2);
        if (nw) {  // dW1 rows 32q.. += dz1^T agg (db1 from the A operand)
            if constexpr (WG)
                mma_kk4x2<4>(sET + (q * 32 + li) * LDT + 4 * kk, sAT + li * LDT + 4 * kk,
                             sAT + (32 + li) * LDT + 4 * kk, accA, accB, dbias);
        } else {   // d(agg) block q = dz1 W1[:, 32q..] -> staging
            const f32x16 da = mma_rk4<8>(sE + li * LDR + 4 * kk, wreg, zero16());
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) sG[acc_row(reg, l) * LDH + q * 32 + li] = da[reg];
        }
        lds_barrier();  // d(agg) staged; agg and dz1 consumed
        if (it == 0) SCGIB_MARK(4);
        if (WG && next_nv > 0) put_t(sAT, 3);
        // d(agg) rows: full-row float4 stores (after the loads: in-order vmcnt)
        {
            const int c4 = tid & 15, rs = tid >> 4;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int rr = rs + 16 * k;
                const float *pg = sG + rr * LDH + 4 * c4;
                const float4 v = make_float4(pg[0], pg[1], pg[2], pg[3]);
                if (rr < nv) st4(dagg_out + (s * SM + rr) * DIN + 4 * c4, v);
            }
        }
        if (dims) zero_pad(s, nv);
        nv = next_nv;
    }
    SCGIB_MARK(5);
    if constexpr (!WG) return;
    // per-workgroup slab: dW2 | dW1 | db2 | db1 (gin_bwd_k layout)
    float *sl = slab + static_cast<int64_t>(blockIdx.x) * SLAB;
    float *dw = nw ? sl + 64 * 64 : sl;  // N: dW1 [64][DIN], T: dW2 [64][64]
    const int ld = nw ? DIN : 64;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int j = q * 32 + acc_row(reg, l);
        dw[j * ld + li] = accA[reg];
        dw[j * ld + 32 + li] = accB[reg];
    }
    dbias += __shfl_xor(dbias, 32, kWave);
    if (l < 32) sl[64 * 64 + 64 * DIN + (nw ? 64 : 0) + q * 32 + l] = dbias;
    SCGIB_MARK(6);
}

// ---------------------------------------------------------------------------
// The agg-free backward of a d_in = 64 GIN layer l >= 1.
// agg_l = (I + A) h_{l-1} is read by exactly one product of the layer's
// backward, dW1 = dz1^T agg.  A is symmetric (the reference's bidirected
// molecule graphs), so with g = (I + A)^T dz1 — the transposed gather the
// NEXT statistics kernel runs anyway, now over dz1 instead of d(agg):
//   dW1_l      = dz1^T (I + A) h_{l-1} = g^T h_{l-1}
//   d h_{l-1}  = (I + A)^T (dz1 W1) = g W1
// and h_{l-1} = relu(scale z2_{l-1} + shift) comes elementwise from the z2
// rows that kernel reads for layer l-1's BatchNorm backward.  So the forward
// stores no agg for these layers (256 B per row less of the 768 B it wrote,
// gin_fwd_k), gin_bwd5z_k runs two of gin_bwd5_k's four products (dr, dW2)
// and writes dz1 where gin_bwd5_k wrote d(agg), reading no agg; and
// gin_bwd_statsz_k gathers dz1 and adds the two products it moved (g W1 and
// g^T h, f32 MFMA), leaving dW1 as per-workgroup partials.  No flops are
// added, only moved; the sums associate differently, so results match the
// stored-agg path to rounding, not bitwise (ops.AGG_FREE selects the path).
// ---------------------------------------------------------------------------
constexpr int kZSlab = 64 * 64 + 128;  // gin_bwd5z_k slab: dW2 [64][64] | db2 | db1

// gin_bwd5z_k: gin_bwd5_k's sub-tile walk with its first product pair only —
//   waves 0,1 (N): dr block q = dz2 W2[:, 32q..] (K = 64), dz1 = dr [r > 0]
//                  -> dz1 staging (row-major) and db1 (column sums of dz1);
//   waves 2,3 (T): dW2 rows 32q.. += dz2^T r (two blocks, K = 32 rows) + db2
// — then the dz1 rows go out as full-row float4 stores: two barriers per
// sub-tile (gin_bwd5_k: three), no agg rows loaded, no W1.
// WG = false: a frozen layer (the fine-tune freezing quirk) — dz1 by the same
// dr chain, no dW2 / db products, no slab.
template <bool WG = true>
__global__ __launch_bounds__(256, 2) void gin_bwd5z_k(
    const float *__restrict__ dy, const float *__restrict__ z2, const float *__restrict__ r,
    const float *__restrict__ stat, const float *__restrict__ coef, const float *__restrict__ w2,
    int64_t ncap, int64_t nsub, int64_t G, float *__restrict__ dz1_out, float *__restrict__ slab,
    const int32_t *__restrict__ dims, scgib_bn_bwd_pending pend, scgib_slab_job fold,
    scgib_slab_job fold2) {
    static_assert(SM == 32, "32-row sub-tiles");
    __shared__ __attribute__((aligned(16))) float sD[SM * LDR];   // dz2 [row][k]
    __shared__ __attribute__((aligned(16))) float sDT[64 * LDT];  // dz2 [col][row]
    __shared__ __attribute__((aligned(16))) float sRT[64 * LDT];  // r [col][row]
    __shared__ float sE[SM * LDH];                                 // dz1 staging
    __shared__ float sCoef[128];
    if (static_cast<int64_t>(blockIdx.x) >= G) {  // block-uniform: a folded reduce block
        const int b = static_cast<int>(blockIdx.x - G), f1 = slab_fold8_blocks(fold);
        if (b < f1) slab_fold8_block(fold, b, sD);
        else slab_fold_block(fold2, b - f1, sD);
        return;
    }
    const int64_t n = eff_count(dims, 0, ncap);
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int kk = l >> 5, li = l & 31;
    const bool nw = w < 2;  // wave-uniform role: N (dr, dz1, db1) or T (dW2, db2)
    const int q = w & 1;    // the role's 32-wide block
    const int c = l;        // elementwise: column c, rows 8 w .. 8 w + 7
    const int64_t last = ncap - 1;
    SCGIB_MARK(0);
    SCGIB_MARK_HWID();
    BwdFin bfin;
    const int pend_ngr = static_cast<int>(((n + TM - 1) / TM + kGroup - 1) / kGroup);
    if (pend.gpart) bn_bwd_fin_load<false>(pend.gpart, pend_ngr, 0, bfin);
    const float s_mean = stat[c], s_istd = stat[64 + c], s_sc = stat[128 + c];
    float c1 = 0.f, c2 = 0.f;
    if (!pend.gpart) {
        c1 = coef[c];
        c2 = coef[64 + c];
    }
    float wreg[32];  // N waves: W2[:, 32q..] (k in kperm order); T waves: unused
#pragma unroll
    for (int s = 0; s < 32; ++s) wreg[s] = nw ? w2[kperm(s, kk) * 64 + q * 32 + li] : 0.f;
    float nx[3][8];  // a sub-tile's column c, rows 8 w + i: [0] dy, [1] z2, [2] r
    auto load_sub = [&](int64_t s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // in order of use: r, then dy / z2
            int64_t row = s * SM + 8 * w + i;
            row = row < last ? row : last;
            nx[2][i] = r[row * 64 + c];
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int64_t row = s * SM + 8 * w + i;
            row = row < last ? row : last;
            nx[0][i] = dy[row * 64 + c];
            nx[1][i] = z2[row * 64 + c];
        }
    };
    auto put_rt = [&]() {  // r: column c, rows 8w..8w+7 -> [c][row]
        float4 *p = reinterpret_cast<float4 *>(sRT + c * LDT + 8 * w);
        p[0] = make_float4(nx[2][0], nx[2][1], nx[2][2], nx[2][3]);
        p[1] = make_float4(nx[2][4], nx[2][5], nx[2][6], nx[2][7]);
    };
    auto rows_of = [&](int64_t s) {
        const int64_t v = n - s * SM;
        return static_cast<int>(v < SM ? (v > 0 ? v : 0) : SM);
    };
    auto zero_pad = [&](int64_t s, int from) {
        const int64_t row0 = s * SM;
        const int ncr = static_cast<int>(ncap - row0 < SM ? ncap - row0 : SM);
        for (int idx = from * 64 + tid; idx < ncr * 64; idx += 256) dz1_out[row0 * 64 + idx] = 0.f;
    };
    int64_t s = blockIdx.x;
    int nv = s < nsub ? rows_of(s) : 0;
    if (nv > 0) load_sub(s);
    if (pend.gpart) {  // finish the BN-backward sums; workgroup 0 writes dgamma, dbeta
        const double tot = bn_bwd_final<false>(pend.gpart, pend_ngr, bfin);
        const int cs = bfin_index();
        const bool lead = (tid & 63) < 32, w0 = blockIdx.x == 0 && lead;
        const float cf = bn_bwd_publish(cs, tot, n, pend.training, w0 ? pend.dgamma : nullptr,
                                        w0 ? pend.dbeta : nullptr, nullptr);
        if (lead) sCoef[cs] = cf;
    }
    if (nv > 0) put_rt();
    vm_wait_all();  // the weight registers complete before the loop (gin_bwd5_k)
    __syncthreads();
    if (pend.gpart) {
        c1 = sCoef[c];
        c2 = sCoef[64 + c];
    }
    const float k1 = s_istd * c2;  // dz2 = sc (dy - c1 - (z2 - mean) istd c2)
    SCGIB_MARK(1);
    f32x16 accA = zero16(), accB = zero16();  // T waves: dW2 blocks (q, 0), (q, 1)
    float dbias = 0.f;                         // N: db1 (column q*32 + li), T: db2
    for (int it = 0; s < nsub; s += G, ++it) {
        if (nv == 0) {  // capacity tail: this and every later sub-tile is padding
            for (int64_t t = s; t < nsub; t += G) zero_pad(t, rows_of(t));
            break;
        }
        {   // dz2 (rows past nv zero) -> sD row-major and sDT transposed
            float d[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float v = s_sc * (nx[0][i] - c1 - (nx[1][i] - s_mean) * k1);
                d[i] = 8 * w + i < nv ? v : 0.f;
                sD[(8 * w + i) * LDR + c] = d[i];
            }
            float4 *p = reinterpret_cast<float4 *>(sDT + c * LDT + 8 * w);
            p[0] = make_float4(d[0], d[1], d[2], d[3]);
            p[1] = make_float4(d[4], d[5], d[6], d[7]);
        }
        const int64_t next = s + G;
        const int next_nv = next < nsub ? rows_of(next) : 0;  // block-uniform
        if (next_nv > 0) load_sub(next);  // in flight during the products
        lds_barrier();  // dz2 complete
        if (it == 0) SCGIB_MARK(2);
        if (nw) {  // dr block q, dz1 = dr [r > 0] (mask by multiplication) -> staging
            const f32x16 dr = mma_rk4<8>(sD + li * LDR + 4 * kk, wreg, zero16());
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
                const int row = acc_row(reg, l), col = q * 32 + li;
                const float v = dr[reg] * (sRT[col * LDT + row] > 0.f ? 1.f : 0.f);
                sE[row * LDH + col] = v;
                dbias += v;
            }
        } else if constexpr (WG) {   // dW2 rows 32q.. += dz2^T r (db2 from the A operand)
            mma_kk4x2<4>(sDT + (q * 32 + li) * LDT + 4 * kk, sRT + li * LDT + 4 * kk,
                         sRT + (32 + li) * LDT + 4 * kk, accA, accB, dbias);
        }
        lds_barrier();  // dz1 staged; r and dz2 consumed
        if (it == 0) SCGIB_MARK(3);
        if (next_nv > 0) put_rt();
        {   // dz1 rows: full-row float4 stores
            const int c4 = tid & 15, rs = tid >> 4;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int rr = rs + 16 * k;
                const float *pg = sE + rr * LDH + 4 * c4;
                const float4 v = make_float4(pg[0], pg[1], pg[2], pg[3]);
                if (rr < nv) st4(dz1_out + (s * SM + rr) * 64 + 4 * c4, v);
            }
        }
        if (dims) zero_pad(s, nv);
        nv = next_nv;
    }
    SCGIB_MARK(5);
    if constexpr (!WG) return;
    // per-workgroup slab: dW2 [64][64] | db2 [64] | db1 [64]
    float *sl = slab + static_cast<int64_t>(blockIdx.x) * kZSlab;
    if (!nw) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
            const int j = q * 32 + acc_row(reg, l);
            sl[j * 64 + li] = accA[reg];
            sl[j * 64 + 32 + li] = accB[reg];
        }
    }
    dbias += __shfl_xor(dbias, 32, kWave);
    if (l < 32) sl[64 * 64 + (nw ? 64 : 0) + q * 32 + l] = dbias;
    SCGIB_MARK(6);
}

// gin_bwd_statsz_k: the backward statistics of layer l below an agg-free layer
// l + 1 — gin_bwd_stats_k<GATHER>'s work with the transposed gather taken over
// dz1_{l+1} and the two products moved out of gin_bwd5z_k:
//   g = ope dz1[v] + sum_{v->u} dz1[u]       (gather_rows, as gin_bwd_stats_k)
//   dh = g W1_{l+1}     (f32 MFMA, W1 staged in LDS once per workgroup)
//   dW1_{l+1} += g^T h, h = relu(scale z2 + shift) (rows past nv: 0)
//   dy = dh [scale z2 + shift > 0]; tile sums of dy and dy xhat -> BN hier
// Each workgroup walks a run of `per` consecutive tiles (the fewest workgroups
// reaching ceil(tiles / kZStatSlots) tiles each) and keeps its 64 x 64 dW1
// block in MFMA accumulators (wave w: rows 32 (w >> 1).., columns 32 (w & 1)..),
// one partial slab per workgroup — per-tile partials would write as many
// bytes as the agg rows this path saves.  Workgroups past the walk reduce up
// to two slab jobs.  LDS: the g, h and z tiles row-major at stride 65 (the
// stats layout's 4-channel runs store conflict free, and both products read
// their operands by column or by row conflict free, mma_pf), W1, the sums.
constexpr int kZStatSlots = 512;    // two walking workgroups per CU

// WG = false: layer l + 1 is frozen — dh and dy exactly as with WG, no h
// image, no dW1 product, no slab.
template <bool WG = true>
__global__ __launch_bounds__(256, 2) void gin_bwd_statsz_k(
    const float *__restrict__ dz1, const int32_t *__restrict__ rowptr_t,
    const int32_t *__restrict__ col_t, float ope, const float *__restrict__ w1,
    const float *__restrict__ z2, const float *__restrict__ stat, int64_t ncap, int per,
    float *__restrict__ dy_out, float *__restrict__ part, const int32_t *__restrict__ dims,
    BnBwdFuse bz, float *__restrict__ wslab, scgib_slab_job fold1, scgib_slab_job fold2) {
    __shared__ float sG[TM * LDH];   // g [row][o]; then dh [row][in] (staging)
    __shared__ float sH[TM * LDH];   // h [row][in]
    __shared__ float sZ[TM * LDH];   // z2 [row][c] (not held in registers across the products)
    __shared__ float sW1[64 * LDH];  // W1 [o][in]
    __shared__ float sRed[2][16][64];
    const int64_t ntc = (ncap + TM - 1) / TM;
    const int64_t G = (ntc + per - 1) / per;
    if (static_cast<int64_t>(blockIdx.x) >= G) {  // block-uniform: a folded reduce block
        const int b = static_cast<int>(blockIdx.x - G), f1 = slab_fold_blocks(fold1);
        if (b < f1) slab_fold_block(fold1, b, &sRed[0][0][0]);
        else slab_fold_block(fold2, b - f1, &sRed[0][0][0]);
        return;
    }
    const int64_t n = eff_count(dims, 0, ncap);
    const int rw = (threadIdx.x >> 6) >> 1, cq = (threadIdx.x >> 6) & 1;  // the wave's 32 x 32
    // block of dh and of dW1 (wave-uniform)
    SCGIB_MARK(0);
    SCGIB_MARK_HWID();
    const float4 *g4 = reinterpret_cast<const float4 *>(dz1);
    f32x16 accW = zero16();
    const int64_t vb = SCGIB_XCD_TILES ? xcd_remap(blockIdx.x, G) : static_cast<int64_t>(blockIdx.x);
    const int64_t t0 = vb * per, t1 = t0 + per < ntc ? t0 + per : ntc;
    bool w1_staged = false;
    for (int64_t tile = t0; tile < t1; ++tile) {
        // lane indices laundered per tile: every LDS / global address below is
        // then formed inside the loop, not hoisted out of it and held in
        // registers across the walk (which ran the kernel out of VGPRs)
        int tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        const int c = tid & 15, slot = tid >> 4, l = tid & 63;
        const int64_t row0 = tile * TM;
        const int nv = static_cast<int>(n - row0 < TM ? (n - row0 > 0 ? n - row0 : 0) : TM);
        if (nv == 0) {  // capacity mode: a tile of padding rows (block-uniform)
            for (int rr = slot; rr < TM && row0 + rr < ncap; rr += 16)
                st4(dy_out + (row0 + rr) * 64 + 4 * c, make_float4(0.f, 0.f, 0.f, 0.f));
            continue;
        }
        float4 g[4], z[4];
        {
            const float4 one4 = make_float4(1.f, 1.f, 1.f, 1.f), zero4 = make_float4(0.f, 0.f, 0.f, 0.f);
            // W1 once per workgroup: its loads go out first, then the gather's
            // first round and the z rows; W1 goes to LDS before the gather's
            // neighbour rounds (in-order completion: waiting for W1 does not
            // wait for the loads behind it), so its registers are free again
            // where the gather holds the most
            GatherHead<4> hd;
            if (!w1_staged) {  // block-uniform
                float4 wv[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) wv[k] = reinterpret_cast<const float4 *>(w1)[tid + 256 * k];
                gather_head<4, 16, 16>(g4, rowptr_t, row0, nv, slot, c, hd);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int rr = slot + 16 * k;
                    z[k] = ld4(z2 + (row0 + (rr < nv ? rr : nv - 1)) * 64 + 4 * c);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k) {  // (sW1 is read only after the image barrier)
                    const int idx = 4 * (tid + 256 * k), row = idx >> 6, cc = idx & 63;
                    float *d = sW1 + row * LDH + cc;
                    d[0] = wv[k].x; d[1] = wv[k].y; d[2] = wv[k].z; d[3] = wv[k].w;
                }
                w1_staged = true;
            } else {
                gather_head<4, 16, 16>(g4, rowptr_t, row0, nv, slot, c, hd);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int rr = slot + 16 * k;
                    z[k] = ld4(z2 + (row0 + (rr < nv ? rr : nv - 1)) * 64 + 4 * c);
                }
            }
            gather_tail<4, 16, false>(g4, col_t, hd, c, ope, one4, zero4, g);
            __syncthreads();  // the previous tile's readers of sG (dh) / sH / sZ are done
        }
        {
            const float4 sc = ld4(stat + 128 + 4 * c), sh = ld4(stat + 192 + 4 * c);
#pragma unroll
            for (int k = 0; k < 4; ++k) {  // g, h (rows past nv: 0), z rows
                const int rr = slot + 16 * k;
                const float valid = rr < nv ? 1.f : 0.f;
                float *pg = sG + rr * LDH + 4 * c, *pz = sZ + rr * LDH + 4 * c;
                pg[0] = g[k].x; pg[1] = g[k].y; pg[2] = g[k].z; pg[3] = g[k].w;
                pz[0] = z[k].x; pz[1] = z[k].y; pz[2] = z[k].z; pz[3] = z[k].w;
                if constexpr (WG) {
                    float *ph = sH + rr * LDH + 4 * c;
                    ph[0] = fmaxf(sc.x * z[k].x + sh.x, 0.f) * valid;
                    ph[1] = fmaxf(sc.y * z[k].y + sh.y, 0.f) * valid;
                    ph[2] = fmaxf(sc.z * z[k].z + sh.z, 0.f) * valid;
                    ph[3] = fmaxf(sc.w * z[k].w + sh.w, 0.f) * valid;
                }
            }
        }
        __syncthreads();
        SCGIB_MARK(1);
        // dh block (rw, cq) = g W1: A(i = row, k = o) = sG[row][o], B(k = o, j = in) = sW1[o][in]
        f32x16 dh = mma_pf<64, false, true, 2>(sG + 32 * rw * LDH, LDH, sW1 + 32 * cq, LDH, zero16());
        // dW1 block (rw, cq) += g^T h over the tile's rows: A(i = o, k = row) = sG[row][o],
        // B(k = row, j = in) = sH[row][in]
        if constexpr (WG) accW = mma_pf<64, true, true, 2>(sG + 32 * rw, LDH, sH + 32 * cq, LDH, accW);
        __syncthreads();  // every read of the g tile done: it stages dh now
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
            sG[(32 * rw + acc_row(reg, l)) * LDH + 32 * cq + (l & 31)] = dh[reg];
        __syncthreads();
        SCGIB_MARK(2);
        {
            const float4 mean = ld4(stat + 4 * c), istd = ld4(stat + 64 + 4 * c);
            const float4 sc = ld4(stat + 128 + 4 * c), sh = ld4(stat + 192 + 4 * c);
            float4 sdy = make_float4(0.f, 0.f, 0.f, 0.f), sdx = sdy;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int rr = slot + 16 * k;
                const int64_t v = row0 + rr;
                const float valid = rr < nv ? 1.f : 0.f;
                const float *pd = sG + rr * LDH + 4 * c, *pz = sZ + rr * LDH + 4 * c;
                const float4 gg = make_float4(pd[0], pd[1], pd[2], pd[3]);
                const float4 zz = make_float4(pz[0], pz[1], pz[2], pz[3]);
                const float4 dyv = make_float4((sc.x * zz.x + sh.x > 0.f ? gg.x : 0.f) * valid,
                                               (sc.y * zz.y + sh.y > 0.f ? gg.y : 0.f) * valid,
                                               (sc.z * zz.z + sh.z > 0.f ? gg.z : 0.f) * valid,
                                               (sc.w * zz.w + sh.w > 0.f ? gg.w : 0.f) * valid);
                if (v < ncap) st4(dy_out + v * 64 + 4 * c, dyv);
                sdy = add4(sdy, dyv);
                sdx = add4(sdx, make_float4(dyv.x * (zz.x - mean.x) * istd.x,
                                            dyv.y * (zz.y - mean.y) * istd.y,
                                            dyv.z * (zz.z - mean.z) * istd.z,
                                            dyv.w * (zz.w - mean.w) * istd.w));
            }
            float *pa = &sRed[0][slot][4 * c];
            pa[0] = sdy.x; pa[1] = sdy.y; pa[2] = sdy.z; pa[3] = sdy.w;
            float *pb = &sRed[1][slot][4 * c];
            pb[0] = sdx.x; pb[1] = sdx.y; pb[2] = sdx.z; pb[3] = sdx.w;
        }
        __syncthreads();
        if (tid < 128) {
            const int which = tid >> 6, ch = tid & 63;
            float s = 0.f;
            for (int k = 0; k < 16; ++k) s += sRed[which][k][ch];
            st_agent(part + tile * 128 + which * 64 + ch, s);
        }
        SCGIB_MARK(3);
        __syncthreads();  // sRed's readers done before the next tile writes it
    }
    // the BatchNorm statistics: this workgroup's tiles arrive at their groups
    // at once, one arrival per group its run touches (the hierarchy inlined
    // in the tile loop held its registers beside the walk's and spilled); the
    // dW1 slab is written after (an arrival waits for every store issued
    // before it)
    // (accW waits in LDS meanwhile — each lane its own 16 slots of the dead
    // g tile — so its registers are free for the hierarchy's)
    if constexpr (WG) {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) sG[threadIdx.x * 16 + reg] = accW[reg];
    }
    if (bz.counters) {
        __shared__ double shh[2][128];
        const int64_t ntv = (n + TM - 1) / TM, e = t1 < ntv ? t1 : ntv;
        for (int64_t gg = t0 / kGroup; gg * kGroup < e; ++gg) {
            const int64_t lo = t0 > gg * kGroup ? t0 : gg * kGroup;
            const int64_t hi = e < (gg + 1) * kGroup ? e : (gg + 1) * kGroup;
            if (hi <= lo) continue;  // (a run of padding tiles only: no arrival)
            bn_bwd_hier_gs(part, n, static_cast<int>(gg), static_cast<unsigned>(hi - lo), bz, shh);
        }
    }
    if constexpr (WG) {  // this workgroup's dW1 partial
        const int l = threadIdx.x & 63, li = l & 31;
        float *sl = wslab + static_cast<int64_t>(blockIdx.x) * 4096;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg)
            sl[(32 * rw + acc_row(reg, l)) * 64 + 32 * cq + li] = sG[threadIdx.x * 16 + reg];
    }
    SCGIB_MARK(4);
}

// ---------------------------------------------------------------------------
// gin_bwd5r_k: gin_bwd5_k without the saved r.  The
// forward no longer writes r = relu(agg W1^T + b1) — one of the three [N,64]
// row sets gin_fwd_k stored, a third of its HBM writes — and this kernel
// recomputes it per sub-tile from the agg rows it stages anyway, with the
// forward's own MFMA chain (v_mfma_f32_32x32x2_f32, step s = k pair (2 s,
// 2 s + 1), s = 0..31 in order from zero, then + b1 and fmaxf 0), so every r
// element is bitwise the one the forward would have stored; every other
// product is one of gin_bwd5_k's chains unchanged (same operands, same order
// per output element), so dW1 / dW2 / db / d(agg) are bitwise gin_bwd5_k's
// (tests/test_gpu_parity.py::test_gin_layer_bwd_recompute_bitwise).
// Roles, 80 MFMAs per wave and sub-tile (gin_bwd5_k: 64) in three phases:
//   1: waves 0,1: r block q = agg W1[32q.., :]^T + b1, relu -> r^T image
//                 (and the block's ReLU mask, 16 bits in one register)
//      waves 2,3: dr block q = dz2 W2[:, 32q..] -> the dz1^T image
//   2: waves 0,1: dz1 = dr [r > 0] (their own block) -> dz1 / dz1^T images
//      every wave: dW2 block (q, w >> 1) += dz2^T r (db2: waves 0,1)
//   3: waves 0,1: d(agg) block q = dz1 W1[:, 32q..] -> staging
//      waves 2,3: dW1 rows 32q.. += dz1^T agg (db1)
//   (+ the next sub-tile's dz2 staged during phase 3: three barriers)
// Registers: waves 0,1 hold W1 rows (r) and W1 columns (d(agg)), waves 2,3
// W2 columns (dr) and two dW1 accumulators — the second weight block and
// those accumulators are the same two f32x16.  LDS: gin_bwd5_k's images
// (r^T now written by phase 1) + the agg rows with each row's k split
// even | odd (lane half kk reads k = 2 s + kk, s = 0..31, as one run: b128
// operand reads) = 72 KB, two workgroups per CU.
// ---------------------------------------------------------------------------
constexpr int kEO = 32;  // even | odd split: k -> (k & 1) * 32 + (k >> 1)

template <int DIN>
__global__ __launch_bounds__(256, 2) void gin_bwd5r_k(
    const float *__restrict__ dy, const float *__restrict__ z2, const float *__restrict__ agg,
    const float *__restrict__ stat, const float *__restrict__ coef, const float *__restrict__ w1,
    const float *__restrict__ b1, const float *__restrict__ w2, int64_t ncap, int64_t nsub,
    float *__restrict__ dagg_out, float *__restrict__ slab, const int32_t *__restrict__ dims,
    scgib_bn_bwd_pending pend) {
    static_assert(DIN == 64 && SM == 32, "64-wide rows, 32-row sub-tiles");
    constexpr int SLAB = 64 * 64 + 64 * DIN + 128;
    __shared__ __attribute__((aligned(16))) float sD[SM * LDR];   // dz2 [row][k]
    __shared__ __attribute__((aligned(16))) float sDT[64 * LDT];  // dz2 [col][row]
    __shared__ __attribute__((aligned(16))) float sE[SM * LDR];   // dz1
    __shared__ __attribute__((aligned(16))) float sET[64 * LDT];
    __shared__ __attribute__((aligned(16))) float sRT[64 * LDT];  // r [col][row] (recomputed)
    __shared__ __attribute__((aligned(16))) float sAT[DIN * LDT]; // agg [col][row]
    __shared__ __attribute__((aligned(16))) float sAR[SM * LDR];  // agg [row][even | odd k]
    __shared__ float sG[SM * LDH];                                 // d(agg) staging
    __shared__ float sCoef[128];
    const int64_t n = eff_count(dims, 0, ncap);
    const int tid = threadIdx.x, l = tid & 63, w = tid >> 6;
    const int kk = l >> 5, li = l & 31;
    const bool ra = w < 2;  // wave-uniform role: r, d(agg) (waves 0,1) or dr, dW1 (2,3)
    const int q = w & 1;    // the role's 32-wide block
    const int c = l;        // elementwise: column c, rows 8 w .. 8 w + 7
    const int64_t last = ncap - 1;
    const int64_t G = gridDim.x;
    SCGIB_MARK(0);
    SCGIB_MARK_HWID();
    BwdFin bfin;
    const int pend_ngr = static_cast<int>(((n + TM - 1) / TM + kGroup - 1) / kGroup);
    if (pend.gpart) bn_bwd_fin_load<false>(pend.gpart, pend_ngr, 0, bfin);
    const float s_mean = stat[c], s_istd = stat[64 + c], s_sc = stat[128 + c];
    float c1 = 0.f, c2 = 0.f;
    if (!pend.gpart) {
        c1 = coef[c];
        c2 = coef[64 + c];
    }
    // wa: waves 0,1 W1[32q + li][2 s + kk] (r, the forward's k order);
    //     waves 2,3 W2[kperm(s, kk)][32q + li] (dr)
    // X0 | X1: waves 0,1 W1[kperm(s, kk)][32q + li] (d(agg));
    //          waves 2,3 the dW1 accumulators (q, 0) | (q, 1)
    float wa[32];
    f32x16 X0 = zero16(), X1 = zero16();
    float bias1 = 0.f;
    if (ra) {
#pragma unroll
        for (int s = 0; s < 32; ++s) wa[s] = w1[(q * 32 + li) * DIN + 2 * s + kk];
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            X0[s] = w1[kperm(s, kk) * DIN + q * 32 + li];
            X1[s] = w1[kperm(s + 16, kk) * DIN + q * 32 + li];
        }
        bias1 = b1[q * 32 + li];
    } else {
#pragma unroll
        for (int s = 0; s < 32; ++s) wa[s] = w2[kperm(s, kk) * 64 + q * 32 + li];
    }
    // a sub-tile's column c, rows 8 w + i: [0] dy, [1] z2, [2] agg.  The next
    // sub-tile's agg rows are loaded a whole sub-tile ahead (its r^T / agg
    // images are written after this one's barriers 1 and 3), its dy / z2 only
    // after barrier 1 (staged in phase 3): fewer registers live across phase 1
    float nx[3][8];
    auto load_agg = [&](int64_t s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int64_t row = s * SM + 8 * w + i;
            row = row < last ? row : last;
            nx[2][i] = agg[row * DIN + c];
        }
    };
    auto load_dz = [&](int64_t s) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            int64_t row = s * SM + 8 * w + i;
            row = row < last ? row : last;
            nx[0][i] = dy[row * 64 + c];
            nx[1][i] = z2[row * 64 + c];
        }
    };
    auto load_sub = [&](int64_t s) {
        load_agg(s);
        load_dz(s);
    };
    auto put_at = [&]() {  // agg column c, rows 8w..8w+7 -> [c][row]
        float4 *p = reinterpret_cast<float4 *>(sAT + c * LDT + 8 * w);
        p[0] = make_float4(nx[2][0], nx[2][1], nx[2][2], nx[2][3]);
        p[1] = make_float4(nx[2][4], nx[2][5], nx[2][6], nx[2][7]);
    };
    auto put_ar = [&]() {  // agg column c -> position (c & 1) * 32 + (c >> 1) of rows 8w..
        const int pos = (c & 1) * kEO + (c >> 1);
#pragma unroll
        for (int i = 0; i < 8; ++i) sAR[(8 * w + i) * LDR + pos] = nx[2][i];
    };
    auto rows_of = [&](int64_t s) {
        const int64_t v = n - s * SM;
        return static_cast<int>(v < SM ? (v > 0 ? v : 0) : SM);
    };
    auto zero_pad = [&](int64_t s, int from) {
        const int64_t row0 = s * SM;
        const int ncr = static_cast<int>(ncap - row0 < SM ? ncap - row0 : SM);
        for (int idx = from * DIN + tid; idx < ncr * DIN; idx += 256) dagg_out[row0 * DIN + idx] = 0.f;
    };
    float k1 = 0.f;
    // dz2 = sc (dy - c1 - (z2 - mean) istd c2), rows past nv zero -> sD, sDT
    auto stage_dz2 = [&](int nvs) {
        float d[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float v = s_sc * (nx[0][i] - c1 - (nx[1][i] - s_mean) * k1);
            d[i] = 8 * w + i < nvs ? v : 0.f;
            sD[(8 * w + i) * LDR + c] = d[i];
        }
        float4 *p = reinterpret_cast<float4 *>(sDT + c * LDT + 8 * w);
        p[0] = make_float4(d[0], d[1], d[2], d[3]);
        p[1] = make_float4(d[4], d[5], d[6], d[7]);
    };
    int64_t s = blockIdx.x;
    int nv = s < nsub ? rows_of(s) : 0;
    if (nv > 0) load_sub(s);
    if (pend.gpart) {  // finish the BN-backward sums; workgroup 0 writes dgamma, dbeta
        const double tot = bn_bwd_final<false>(pend.gpart, pend_ngr, bfin);
        const int cs = bfin_index();
        const bool lead = (tid & 63) < 32, w0 = blockIdx.x == 0 && lead;
        const float cf = bn_bwd_publish(cs, tot, n, pend.training, w0 ? pend.dgamma : nullptr,
                                        w0 ? pend.dbeta : nullptr, nullptr);
        if (lead) sCoef[cs] = cf;
        __syncthreads();
        c1 = sCoef[c];
        c2 = sCoef[64 + c];
    }
    k1 = s_istd * c2;
    if (nv > 0) {
        put_at();
        put_ar();
        stage_dz2(nv);
    }
    // the weight registers complete here (see gin_bwd5_k)
    vm_wait_all();
    __syncthreads();
    // the second sub-tile's agg rows: in flight during the first one's phase 1
    if (nv > 0 && s + G < nsub && rows_of(s + G) > 0) load_agg(s + G);
    SCGIB_MARK(1);
    f32x16 acc0 = zero16();  // waves 0,1: dW2 block (q, 0); waves 2,3: dW2 block (q, 1)
    float dbias = 0.f;       // waves 0,1: db2 [32q + li]; waves 2,3: db1
    for (int it = 0; s < nsub; s += G, ++it) {
        if (nv == 0) {  // capacity tail: this and every later sub-tile is padding
            for (int64_t t = s; t < nsub; t += G) zero_pad(t, rows_of(t));
            break;
        }
        const int64_t next = s + G;
        const int next_nv = next < nsub ? rows_of(next) : 0;  // block-uniform
        // the element (row 8 g + 4 kk + t, column 32 q + li) of block q sits in
        // register 4 g + t of every role: one b128 per g in the [col][row] images
        const int col = q * 32 + li;
        unsigned rmask = 0u;  // waves 0,1: bit 4 g + t = [r > 0] of their r block
        if (ra) {  // phase 1: r block q (the forward's chain), relu -> sRT as [col][row]
            const f32x16 z = mma_rk4<8, 4>(sAR + li * LDR + kk * kEO, wa, zero16());
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float v[4];
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    v[t] = fmaxf(z[4 * g + t] + bias1, 0.f);
                    rmask |= (v[t] > 0.f ? 1u : 0u) << (4 * g + t);
                }
                *reinterpret_cast<float4 *>(sRT + col * LDT + 8 * g + 4 * kk) = make_float4(v[0], v[1], v[2], v[3]);
            }
        } else {   // phase 1: dr block q -> sET [col][row] (masked in phase 2 by waves 0,1)
            const f32x16 dr = mma_rk4<8>(sD + li * LDR + 4 * kk, wa, zero16());
#pragma unroll
            for (int g = 0; g < 4; ++g)
                *reinterpret_cast<float4 *>(sET + col * LDT + 8 * g + 4 * kk) =
                    make_float4(dr[4 * g], dr[4 * g + 1], dr[4 * g + 2], dr[4 * g + 3]);
        }
        lds_barrier();  // r^T and dr complete; the agg rows consumed
        if (it == 0) SCGIB_MARK(2);
        if (next_nv > 0) {
            put_ar();
            load_dz(next);  // staged in phase 3
        }
        if (ra) {  // phase 2: dz1 = dr [r > 0] -> sE, sET in place (mask by multiplication)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                float4 *pt = reinterpret_cast<float4 *>(sET + col * LDT + 8 * g + 4 * kk);
                const float4 d = *pt;
                const float4 v = make_float4(d.x * ((rmask >> (4 * g)) & 1u ? 1.f : 0.f),
                                             d.y * ((rmask >> (4 * g + 1)) & 1u ? 1.f : 0.f),
                                             d.z * ((rmask >> (4 * g + 2)) & 1u ? 1.f : 0.f),
                                             d.w * ((rmask >> (4 * g + 3)) & 1u ? 1.f : 0.f));
                const int row = 8 * g + 4 * kk;
                sE[row * LDR + col] = v.x;
                sE[(row + 1) * LDR + col] = v.y;
                sE[(row + 2) * LDR + col] = v.z;
                sE[(row + 3) * LDR + col] = v.w;
                *pt = v;
            }
        }
        // phase 2: dW2 rows 32q.., columns 32 (w >> 1).. += dz2^T r (db2 on waves 0,1)
        if (ra)
            mma_kk4<4, true>(sDT + (q * 32 + li) * LDT + 4 * kk, sRT + li * LDT + 4 * kk, acc0, dbias);
        else
            mma_kk4<4, false>(sDT + (q * 32 + li) * LDT + 4 * kk, sRT + (32 + li) * LDT + 4 * kk, acc0, dbias);
        lds_barrier();  // dz1 complete; dz2 and r consumed
        if (it == 0) SCGIB_MARK(3);
        if (ra) {  // phase 3: d(agg) block q = dz1 W1[:, 32q..] -> staging
            const f32x16 da = mma_rk4<8>(sE + li * LDR + 4 * kk, W32{X0, X1}, zero16());
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) sG[acc_row(reg, l) * LDH + q * 32 + li] = da[reg];
        } else {   // phase 3: dW1 rows 32q.. += dz1^T agg (db1 from the A operand)
            mma_kk4x2<4>(sET + (q * 32 + li) * LDT + 4 * kk, sAT + li * LDT + 4 * kk,
                         sAT + (32 + li) * LDT + 4 * kk, X0, X1, dbias);
        }
        if (next_nv > 0) stage_dz2(next_nv);  // dz2 and its images are free since the barrier
        lds_barrier();  // d(agg) staged, next dz2 staged; agg^T and dz1 consumed
        if (it == 0) SCGIB_MARK(4);
        if (next_nv > 0) {
            put_at();
            const int64_t nn = next + G;  // the sub-tile after: in flight during the next one
            if (nn < nsub && rows_of(nn) > 0) load_agg(nn);
        }
        {   // d(agg) rows: full-row float4 stores (after the loads: in-order vmcnt)
            const int c4 = tid & 15, rs = tid >> 4;
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const int rr = rs + 16 * k;
                const float *pg = sG + rr * LDH + 4 * c4;
                const float4 v = make_float4(pg[0], pg[1], pg[2], pg[3]);
                if (rr < nv) st4(dagg_out + (s * SM + rr) * DIN + 4 * c4, v);
            }
        }
        if (dims) zero_pad(s, nv);
        nv = next_nv;
    }
    SCGIB_MARK(5);
    // per-workgroup slab: dW2 | dW1 | db2 | db1 (gin_bwd_k layout)
    float *sl = slab + static_cast<int64_t>(blockIdx.x) * SLAB;
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int j = q * 32 + acc_row(reg, l);
        sl[j * 64 + (ra ? 0 : 32) + li] = acc0[reg];
        if (!ra) {
            sl[64 * 64 + j * DIN + li] = X0[reg];
            sl[64 * 64 + j * DIN + 32 + li] = X1[reg];
        }
    }
    dbias += __shfl_xor(dbias, 32, kWave);
    if (l < 32) sl[64 * 64 + 64 * DIN + (ra ? 0 : 64) + q * 32 + l] = dbias;
    SCGIB_MARK(6);
}

// up to two workgroups per CU (66.5 KB LDS each): one tile per workgroup for
// batches up to kBwdGridCap tiles, so every tile of
// an encoder layer runs at once; larger batches loop over tiles
constexpr int kCUs = 256;  // MI355X: 8 XCDs x 32 CUs

constexpr int64_t kBwdGridCap = 512;
static int bwd_grid(int64_t ntiles) {
    return static_cast<int>(ntiles < kBwdGridCap ? ntiles : kBwdGridCap);
}

}  // namespace scgib

using namespace scgib;

extern "C" int64_t scgib_gin_tiles(int64_t n_nodes) { return (n_nodes + TM - 1) / TM; }

#ifdef SCGIB_TRACE
// debug build only: buffer of [grid][16] uint64 phase stamps (see common.h)
extern "C" int scgib_trace_set_egonet(void *buf);   // (egonet.hip's own g_trace)
extern "C" int scgib_trace_set_set2set(void *buf);  // (set2set.hip's)
extern "C" int scgib_trace_set_interaction(void *buf);  // (interaction.hip's)
extern "C" int scgib_trace_set_head(void *buf);  // (head.hip's)
extern "C" int scgib_trace_set(void *buf) {
    if (scgib_trace_set_egonet(buf) != 0 || scgib_trace_set_set2set(buf) != 0 ||
        scgib_trace_set_interaction(buf) != 0 || scgib_trace_set_head(buf) != 0)
        return 1;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif

// scgib_gin_layer_bwd: d_in = 32 runs gin_bwd_k (one workgroup per tile up
// to the cap); d_in = 64 gin_bwd5_k, on the fewest workgroups that reach the
// largest per-workgroup count at one workgroup per CU: the same finish time
// as the full two-per-CU grid (measured), half the slabs.
static int64_t bwd5_subtiles(int64_t n_nodes) { return (n_nodes + SM - 1) / SM; }
#ifndef SCGIB_BWD5_SLOTS  // (build-time A/B hook: tools/build_ab_lib.sh EXTRA=-DSCGIB_BWD5_SLOTS=n)
#define SCGIB_BWD5_SLOTS kCUs
#endif
static int bwd5_grid(int64_t nsub) {
    constexpr int64_t slots = SCGIB_BWD5_SLOTS;
    const int64_t per = (nsub + slots - 1) / slots;
    return static_cast<int>((nsub + per - 1) / per);
}

extern "C" int64_t scgib_gin_layer_bwd_slabs(int64_t n_nodes, int32_t d_in) {
    if (n_nodes <= 0) return 0;
    const int64_t nt = scgib_gin_tiles(n_nodes);
    if (d_in == 64) return bwd5_grid(bwd5_subtiles(n_nodes));
    return bwd_grid(nt);
}

extern "C" int64_t scgib_gin_slab_floats(int64_t n_nodes, int32_t d_in) {
    return scgib_gin_layer_bwd_slabs(n_nodes, d_in) * (64 * 64 + 64 * d_in + 128);
}

// layer 0 (transfer_d folded): one tile per workgroup up to SCGIB_BWD0_CAP
// workgroups; past it, the fewest workgroups with the same per-workgroup tile
// count (build-time A/B hook: tools/build_ab_lib.sh EXTRA=-DSCGIB_BWD0_CAP=n)
#ifndef SCGIB_BWD0_CAP
#define SCGIB_BWD0_CAP kBwdGridCap
#endif
static int bwd0_grid(int64_t nt) {
    constexpr int64_t cap = SCGIB_BWD0_CAP;
    const int64_t per = (nt + cap - 1) / cap;
    return static_cast<int>((nt + per - 1) / per);
}

extern "C" int64_t scgib_gin_bwd_slabs(int64_t n_nodes) {
    return n_nodes <= 0 ? 0 : bwd0_grid(scgib_gin_tiles(n_nodes));
}

static int launch_gin_fwd(const float *h_in, int32_t d_in, const float *in_stat,
                          const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                          float one_plus_eps, const float *w1, const float *b1, const float *w2,
                          const float *b2, float *agg, float *r, float *z2, float *tile_stats,
                          const int32_t *dims, const BnFwdFuse &fz,
                          const scgib_bn_pending *pend, hipStream_t st) {
    const int64_t nt = scgib_gin_tiles(n_nodes);
    const float *isc = in_stat ? in_stat + 128 : nullptr, *ish = in_stat ? in_stat + 192 : nullptr;
    const scgib_bn_pending pd = pend ? *pend : scgib_bn_pending{};
    if (d_in == 32)
        gin_fwd_k<32, false><<<dim3((unsigned)nt), 256, 0, st>>>(h_in, isc, ish, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2, agg, r, z2, tile_stats, dims, fz, PreArgs{}, pd, ReconArgs{});
    else if (in_stat || pend)
        gin_fwd_k<64, true><<<dim3((unsigned)nt), 256, 0, st>>>(h_in, isc, ish, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2, agg, r, z2, tile_stats, dims, fz, PreArgs{}, pd, ReconArgs{});
    else
        gin_fwd_k<64, false><<<dim3((unsigned)nt), 256, 0, st>>>(h_in, isc, ish, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2, agg, r, z2, tile_stats, dims, fz, PreArgs{}, pd, ReconArgs{});
    return launch_status();
}

static int gin_fwd_args_ok(const float *h_in, int32_t d_in, const float *in_stat,
                           const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                           const float *w1, const float *b1, const float *w2, const float *b2,
                           const float *agg, const float *r, const float *z2,
                           const float *tile_stats) {
    if (n_nodes < 0 || (d_in != 32 && d_in != 64)) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!h_in || !rowptr || !col || !w1 || !b1 || !w2 || !b2 || !z2 || !tile_stats)
        return SCGIB_EINVAL;  // (r may be NULL: not stored)
    if (!agg && d_in != 64) return SCGIB_EINVAL;  // (agg NULL: an agg-free d_in = 64 layer)
    if (in_stat && d_in != 64) return SCGIB_EUNSUPPORTED;
    return 1;  // go
}

extern "C" int scgib_gin_layer_fwd(const float *h_in, int32_t d_in, const float *in_stat,
                                   const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                                   float one_plus_eps, const float *w1, const float *b1,
                                   const float *w2, const float *b2, float *agg, float *r,
                                   float *z2, float *tile_stats, const int32_t *dims,
                                   scgib_stream_t stream) {
    const int ok = gin_fwd_args_ok(h_in, d_in, in_stat, rowptr, col, n_nodes, w1, b1, w2, b2, agg,
                                   r, z2, tile_stats);
    if (ok != 1) return ok;
    BnFwdFuse fz{};
    return launch_gin_fwd(h_in, d_in, in_stat, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2,
                          agg, r, z2, tile_stats, dims, fz, nullptr, as_stream(stream));
}

static int64_t bn_groups(int64_t n_nodes) { return (scgib_gin_tiles(n_nodes) + kGroup - 1) / kGroup; }
// 64-group supergroups (the third statistics level past one load round of groups)
static int64_t bn_supergroups(int64_t n_nodes) {
    const int64_t g = bn_groups(n_nodes);
    return g > kSuper ? (g + kSuper - 1) / kSuper : 0;
}

extern "C" int64_t scgib_gin_bn_ws_floats(int64_t n_nodes) {
    if (n_nodes <= 0) return 0;
    // tile stats [tiles][128] f32 | (8-byte aligned) group partials [groups][128] f64
    // | supergroup partials [supergroups][128] f64
    return ((scgib_gin_tiles(n_nodes) * 128 + 1) & ~int64_t(1)) +
           2 * 128 * (bn_groups(n_nodes) + bn_supergroups(n_nodes));
}

// [groups] group counters | [1] the layer counter | [supergroups] supergroup counters
extern "C" int64_t scgib_gin_counters(int64_t n_nodes) {
    return n_nodes <= 0 ? 0 : bn_groups(n_nodes) + 1 + bn_supergroups(n_nodes);
}

extern "C" int64_t scgib_gin_bn_gpart_offset(int64_t n_nodes) {
    return n_nodes <= 0 ? 0 : ((scgib_gin_tiles(n_nodes) * 128 + 1) & ~int64_t(1));
}

// 64 groups of kGroup tiles: the consumers' one-round finish (bn_fwd_final)
extern "C" int64_t scgib_gin_defer_max_nodes(void) { return int64_t(64) * kGroup * TM; }

static double *bn_gpart(float *ws, int64_t n_nodes) {
    return reinterpret_cast<double *>(ws + scgib_gin_bn_gpart_offset(n_nodes));
}

extern "C" int scgib_gin_layer_fwd_bn(const float *h_in, int32_t d_in, const float *in_stat,
                                      const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                                      float one_plus_eps, const float *w1, const float *b1,
                                      const float *w2, const float *b2, float *agg, float *r,
                                      float *z2, const float *gamma, const float *beta,
                                      float bn_eps, float momentum, float *running_mean,
                                      float *running_var, int64_t *num_batches_tracked,
                                      float *stat, float *bn_ws, uint32_t *counters,
                                      const int32_t *dims, const scgib_bn_pending *in_pending,
                                      int32_t defer, scgib_stream_t stream) {
    const int ok = gin_fwd_args_ok(h_in, d_in, in_stat, rowptr, col, n_nodes, w1, b1, w2, b2, agg,
                                   r, z2, bn_ws);
    if (ok != 1) return ok == SCGIB_OK ? SCGIB_EINVAL : ok;  // BN needs rows
    if (!gamma || !beta || !stat || !counters || ((running_mean == nullptr) != (running_var == nullptr)))
        return SCGIB_EINVAL;
    if (in_pending && (d_in != 64 || in_stat || !in_pending->gpart || !in_pending->gamma ||
                       !in_pending->beta || !in_pending->stat ||
                       ((in_pending->running_mean == nullptr) != (in_pending->running_var == nullptr))))
        return SCGIB_EINVAL;
    BnFwdFuse fz{counters, bn_gpart(bn_ws, n_nodes), gamma, beta, running_mean, running_var,
                 stat, num_batches_tracked, bn_eps, momentum, static_cast<int>(bn_groups(n_nodes)),
                 defer ? 1 : 0};
    return launch_gin_fwd(h_in, d_in, in_stat, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2,
                          agg, r, z2, bn_ws, dims, fz, in_pending, as_stream(stream));
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
                                   float *out, const int32_t *dims,
                                   const scgib_bn_pending *in_pending, scgib_stream_t stream) {
    if (n_nodes < 0) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!z || !out || (!stat && !in_pending)) return SCGIB_EINVAL;
    if (in_pending && (!in_pending->gpart || !in_pending->gamma || !in_pending->beta ||
                       !in_pending->stat || n_nodes > scgib_gin_defer_max_nodes()))
        return SCGIB_EINVAL;
    const int64_t n4 = n_nodes * 16, wg = (n4 + 255) / 256;
    // at most 128 workgroups: this kernel runs beside the other encoder's
    // layers, so it should hold few CU slots (each thread loops instead)
    bn_relu_apply_k<<<dim3(static_cast<unsigned>(wg < 128 ? wg : 128)), 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4 *>(z), stat, n4, reinterpret_cast<float4 *>(out), dims,
        in_pending ? *in_pending : scgib_bn_pending{});
    return launch_status();
}

static int launch_gin_bwd_stats(const float *dh, const int32_t *rowptr_t, const int32_t *col_t,
                                float one_plus_eps, const float *z2, const float *stat,
                                int64_t n_nodes, float *dy, float *tile_stats,
                                const int32_t *dims, const BnBwdFuse &bz, hipStream_t st,
                                const float *g_seg = nullptr, const int32_t *seg = nullptr,
                                const scgib_slab_job *fold = nullptr) {
    const scgib_slab_job fj = fold ? *fold : scgib_slab_job{};
    const unsigned grid = static_cast<unsigned>(scgib_gin_tiles(n_nodes) + slab_fold_blocks(fj));
    if (rowptr_t)
        gin_bwd_stats_k<true><<<dim3(grid), 256, 0, st>>>(dh, rowptr_t, col_t, one_plus_eps, z2, stat, n_nodes, dy, tile_stats, dims, bz, nullptr, nullptr, fj);
    else if (g_seg)
        gin_bwd_stats_k<false, true><<<dim3(grid), 256, 0, st>>>(dh, rowptr_t, col_t, one_plus_eps, z2, stat, n_nodes, dy, tile_stats, dims, bz, g_seg, seg, fj);
    else
        gin_bwd_stats_k<false><<<dim3(grid), 256, 0, st>>>(dh, rowptr_t, col_t, one_plus_eps, z2, stat, n_nodes, dy, tile_stats, dims, bz, nullptr, nullptr, fj);
    return launch_status();
}

static bool fold_ok(const scgib_slab_job *f) {
    return !f || (f->n_slabs > 0 && f->width > 0 && f->slab && f->out &&
                  (f->stride == 0 || f->stride >= f->width));
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
    BnBwdFuse bz{};
    return launch_gin_bwd_stats(dh, rowptr_t, col_t, one_plus_eps, z2, stat, n_nodes, dy,
                                tile_stats, dims, bz, as_stream(stream));
}

extern "C" int scgib_gin_bwd_stats_bn_fold(const float *dh, const int32_t *rowptr_t,
                                           const int32_t *col_t, float one_plus_eps,
                                           const float *z2, const float *stat, int64_t n_nodes,
                                           int32_t training, float *dy, float *dgamma,
                                           float *dbeta, float *coef, float *bn_ws,
                                           uint32_t *counters, const int32_t *dims,
                                           int32_t defer, const scgib_slab_job *fold,
                                           scgib_stream_t stream) {
    if (n_nodes <= 0 || !dh || !z2 || !stat || !dy || !bn_ws || !counters) return SCGIB_EINVAL;
    if (!defer && (!dgamma || !dbeta || !coef)) return SCGIB_EINVAL;
    if ((rowptr_t == nullptr) != (col_t == nullptr)) return SCGIB_EINVAL;
    if (!fold_ok(fold)) return SCGIB_EINVAL;
    BnBwdFuse bz{counters, bn_gpart(bn_ws, n_nodes), dgamma, dbeta, coef, training,
                 static_cast<int>(bn_groups(n_nodes)), defer ? 1 : 0};
    return launch_gin_bwd_stats(dh, rowptr_t, col_t, one_plus_eps, z2, stat, n_nodes, dy, bn_ws,
                                dims, bz, as_stream(stream), nullptr, nullptr, fold);
}

extern "C" int scgib_gin_bwd_stats_bn(const float *dh, const int32_t *rowptr_t,
                                      const int32_t *col_t, float one_plus_eps, const float *z2,
                                      const float *stat, int64_t n_nodes, int32_t training,
                                      float *dy, float *dgamma, float *dbeta, float *coef,
                                      float *bn_ws, uint32_t *counters, const int32_t *dims,
                                      int32_t defer, scgib_stream_t stream) {
    return scgib_gin_bwd_stats_bn_fold(dh, rowptr_t, col_t, one_plus_eps, z2, stat, n_nodes,
                                       training, dy, dgamma, dbeta, coef, bn_ws, counters, dims,
                                       defer, nullptr, stream);
}

extern "C" int scgib_gin_bwd_stats_seg_bn(const float *dh, const float *g_seg,
                                          const int32_t *seg, const float *z2, const float *stat,
                                          int64_t n_nodes, int32_t training, float *dy,
                                          float *dgamma, float *dbeta, float *coef, float *bn_ws,
                                          uint32_t *counters, const int32_t *dims, int32_t defer,
                                          scgib_stream_t stream) {
    if (n_nodes <= 0 || !g_seg || !seg || !z2 || !stat || !dy || !bn_ws || !counters)
        return SCGIB_EINVAL;
    if (!defer && (!dgamma || !dbeta || !coef)) return SCGIB_EINVAL;
    BnBwdFuse bz{counters, bn_gpart(bn_ws, n_nodes), dgamma, dbeta, coef, training,
                 static_cast<int>(bn_groups(n_nodes)), defer ? 1 : 0};
    return launch_gin_bwd_stats(dh, nullptr, nullptr, 1.f, z2, stat, n_nodes, dy, bn_ws, dims, bz,
                                as_stream(stream), g_seg, seg);
}

// Encoder output + readout in one pass: out = relu(scale z + shift) (the last
// layer's BatchNorm + ReLU), readout[s] = sum of out over rows [ptr[s],
// ptr[s+1]) in the order of segment_sum_k (so bitwise equal to the two-kernel
// path), seg[row] = s for the backward's broadcast.  16 lanes (float4) per
// segment; capacity mode: rows past the last valid segment are zeroed.
__global__ __launch_bounds__(256) void bn_relu_segsum_k(
    const float4 *__restrict__ z, const float *__restrict__ stat, const int32_t *__restrict__ ptr,
    int64_t nseg, int64_t nrows, float4 *__restrict__ out, float4 *__restrict__ readout,
    int32_t *__restrict__ seg, const int32_t *__restrict__ seg_dims,
    const int32_t *__restrict__ dims, scgib_bn_pending pend) {
    const int64_t blk = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t s = blk * 16 + (threadIdx.x >> 4);
    const int c = threadIdx.x & 15;
    const int64_t ns = eff_count(seg_dims, 0, nseg);
    float4 a, b;
    if (pend.gpart) {  // the last GIN layer's deferred statistics
        __shared__ float sSS[128];
        bn_pending_finish(pend, eff_count(dims, 0, nrows), sSS);
        a = make_float4(sSS[4 * c], sSS[4 * c + 1], sSS[4 * c + 2], sSS[4 * c + 3]);
        b = make_float4(sSS[64 + 4 * c], sSS[65 + 4 * c], sSS[66 + 4 * c], sSS[67 + 4 * c]);
    } else {
        a = ld4(stat + 128 + 4 * c);
        b = ld4(stat + 192 + 4 * c);
    }
    if (seg_dims) {  // zero the rows past the last valid segment (grid-stride)
        const int64_t r0 = ptr[ns];
        const int64_t tot = (nrows - r0) * 16;
        for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < tot;
             i += static_cast<int64_t>(gridDim.x) * 256)
            out[r0 * 16 + i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (s >= nseg) return;
    if (s >= ns) {
        readout[s * 16 + c] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    const int64_t beg = ptr[s], end = ptr[s + 1];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t i = beg;
    for (; i + 4 <= end; i += 4) {
        const float4 v0 = xform4(z[i * 16 + c], a, b), v1 = xform4(z[(i + 1) * 16 + c], a, b);
        const float4 v2 = xform4(z[(i + 2) * 16 + c], a, b), v3 = xform4(z[(i + 3) * 16 + c], a, b);
        out[i * 16 + c] = v0; out[(i + 1) * 16 + c] = v1;
        out[(i + 2) * 16 + c] = v2; out[(i + 3) * 16 + c] = v3;
        if (c == 0) { seg[i] = s; seg[i + 1] = s; seg[i + 2] = s; seg[i + 3] = s; }
        acc = add4(add4(add4(add4(acc, v0), v1), v2), v3);
    }
    for (; i < end; ++i) {
        const float4 v = xform4(z[i * 16 + c], a, b);
        out[i * 16 + c] = v;
        if (c == 0) seg[i] = s;
        acc = add4(acc, v);
    }
    readout[s * 16 + c] = acc;
}

extern "C" int scgib_bn_relu_segment_sum(const float *z, const float *stat, const int32_t *ptr,
                                         int64_t n_seg, int64_t n_rows, float *out,
                                         float *readout, int32_t *seg, const int32_t *seg_dims,
                                         const int32_t *dims, const scgib_bn_pending *in_pending,
                                         scgib_stream_t stream) {
    if (n_seg < 0 || n_rows < 0) return SCGIB_EINVAL;
    if (n_seg == 0) return SCGIB_OK;
    if (!z || !ptr || !out || !readout || !seg || (!stat && !in_pending)) return SCGIB_EINVAL;
    if (in_pending && (!in_pending->gpart || !in_pending->gamma || !in_pending->beta ||
                       !in_pending->stat || n_rows == 0 || n_rows > scgib_gin_defer_max_nodes()))
        return SCGIB_EINVAL;
    bn_relu_segsum_k<<<dim3(static_cast<unsigned>((n_seg + 15) / 16)), 256, 0, as_stream(stream)>>>(
        reinterpret_cast<const float4 *>(z), stat, ptr, n_seg, n_rows,
        reinterpret_cast<float4 *>(out), reinterpret_cast<float4 *>(readout), seg, seg_dims, dims,
        in_pending ? *in_pending : scgib_bn_pending{});
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
                                   const float *coef, const float *w1, const float *b1,
                                   const float *w2, int64_t n_nodes, float *dagg, float *slab,
                                   float *wgrad, int32_t need_w, const int32_t *dims,
                                   const scgib_bn_bwd_pending *pending, scgib_stream_t stream) {
    if (n_nodes <= 0 || (d_in != 32 && d_in != 64)) return SCGIB_EINVAL;
    if (!dy || !z2 || !stat || (!coef && !pending) || !w1 || !w2 || !dagg)
        return SCGIB_EINVAL;
    if (need_w && (!agg || !slab)) return SCGIB_EINVAL;
    if (!r && (d_in != 64 || !b1 || !agg)) return SCGIB_EINVAL;  // recompute: d_in = 64, needs b1
    if (!need_w && (d_in != 64 || !r)) return SCGIB_EUNSUPPORTED;  // frozen: stored-r d_in = 64
    if (pending && (!pending->gpart || !pending->dgamma || !pending->dbeta)) return SCGIB_EINVAL;
    const scgib_bn_bwd_pending pd = pending ? *pending : scgib_bn_bwd_pending{};
    const int64_t nt = scgib_gin_tiles(n_nodes);
    const int grid = static_cast<int>(scgib_gin_layer_bwd_slabs(n_nodes, d_in));
    hipStream_t st = as_stream(stream);
    if (d_in == 32)
        gin_bwd_k<32><<<grid, 256, 0, st>>>(dy, z2, r, agg, stat, coef, w1, w2, n_nodes, nt, dagg, slab, dims, nullptr, pd, ReconArgs{});
    else if (!need_w)
        gin_bwd5_k<64, false><<<grid, 256, 0, st>>>(dy, z2, r, agg, stat, coef, w1, w2, n_nodes, bwd5_subtiles(n_nodes), dagg, slab, dims, pd);
    else if (r)
        gin_bwd5_k<64><<<grid, 256, 0, st>>>(dy, z2, r, agg, stat, coef, w1, w2, n_nodes, bwd5_subtiles(n_nodes), dagg, slab, dims, pd);
    else
        gin_bwd5r_k<64><<<grid, 256, 0, st>>>(dy, z2, agg, stat, coef, w1, b1, w2, n_nodes, bwd5_subtiles(n_nodes), dagg, slab, dims, pd);
    const int rc = launch_status();
    if (rc != SCGIB_OK || !wgrad || !need_w) return rc;  // wgrad NULL: the caller reduces the slabs
    return launch_slab_reduce(slab, grid, 64 * 64 + 64 * static_cast<int64_t>(d_in) + 128, wgrad, st);
}

// ---------------------------------------------------------------------------
// agg-free backward entries (gin_bwd5z_k / gin_bwd_statsz_k)
// ---------------------------------------------------------------------------
extern "C" int64_t scgib_gin_layer_bwd_z_slabs(int64_t n_nodes) {
    return n_nodes <= 0 ? 0 : bwd5_grid(bwd5_subtiles(n_nodes));
}

extern "C" int64_t scgib_gin_layer_bwd_z_width(void) { return kZSlab; }

extern "C" int scgib_gin_layer_bwd_z(const float *dy, const float *z2, const float *r,
                                     const float *stat, const float *coef, const float *w2,
                                     int64_t n_nodes, float *dz1, float *slab, int32_t need_w,
                                     const int32_t *dims, const scgib_bn_bwd_pending *pending,
                                     const scgib_slab_job *fold, const scgib_slab_job *fold2,
                                     scgib_stream_t stream) {
    if (n_nodes <= 0 || !dy || !z2 || !r || !stat || (!coef && !pending) || !w2 || !dz1 ||
        (need_w && !slab))
        return SCGIB_EINVAL;
    if (pending && (!pending->gpart || !pending->dgamma || !pending->dbeta)) return SCGIB_EINVAL;
    if (!fold_ok(fold) || !fold_ok(fold2)) return SCGIB_EINVAL;
    const scgib_bn_bwd_pending pd = pending ? *pending : scgib_bn_bwd_pending{};
    const scgib_slab_job fj = fold ? *fold : scgib_slab_job{};
    const scgib_slab_job fj2 = fold2 ? *fold2 : scgib_slab_job{};
    const int64_t G = scgib_gin_layer_bwd_z_slabs(n_nodes);
    const int grid = static_cast<int>(G + slab_fold8_blocks(fj) + slab_fold_blocks(fj2));
    if (need_w)
        gin_bwd5z_k<true><<<grid, 256, 0, as_stream(stream)>>>(
            dy, z2, r, stat, coef, w2, n_nodes, bwd5_subtiles(n_nodes), G, dz1, slab, dims, pd, fj,
            fj2);
    else
        gin_bwd5z_k<false><<<grid, 256, 0, as_stream(stream)>>>(
            dy, z2, r, stat, coef, w2, n_nodes, bwd5_subtiles(n_nodes), G, dz1, slab, dims, pd, fj,
            fj2);
    return launch_status();
}

static int statsz_per(int64_t n_nodes) {
    const int64_t nt = scgib_gin_tiles(n_nodes);
    return static_cast<int>((nt + kZStatSlots - 1) / kZStatSlots);
}

extern "C" int64_t scgib_gin_bwd_stats_z_slabs(int64_t n_nodes) {
    if (n_nodes <= 0) return 0;
    const int64_t nt = scgib_gin_tiles(n_nodes), per = statsz_per(n_nodes);
    return (nt + per - 1) / per;
}

extern "C" int scgib_gin_bwd_stats_z(const float *dz1, const int32_t *rowptr_t,
                                     const int32_t *col_t, float one_plus_eps, const float *w1,
                                     const float *z2, const float *stat, int64_t n_nodes,
                                     int32_t training, float *dy, float *dgamma, float *dbeta,
                                     float *coef, float *bn_ws, uint32_t *counters,
                                     const int32_t *dims, int32_t defer, float *wslab,
                                     int32_t need_w, const scgib_slab_job *fold, int32_t n_fold,
                                     scgib_stream_t stream) {
    if (n_nodes <= 0 || !dz1 || !rowptr_t || !col_t || !w1 || !z2 || !stat || !dy || !bn_ws ||
        !counters || (need_w && !wslab))
        return SCGIB_EINVAL;
    if (!defer && (!dgamma || !dbeta || !coef)) return SCGIB_EINVAL;
    if (n_fold < 0 || n_fold > 2 || (n_fold > 0 && !fold)) return SCGIB_EINVAL;
    for (int i = 0; i < n_fold; ++i)
        if (!fold_ok(&fold[i])) return SCGIB_EINVAL;
    BnBwdFuse bz{counters, bn_gpart(bn_ws, n_nodes), dgamma, dbeta, coef, training,
                 static_cast<int>(bn_groups(n_nodes)), defer ? 1 : 0};
    const scgib_slab_job f1 = n_fold > 0 ? fold[0] : scgib_slab_job{};
    const scgib_slab_job f2 = n_fold > 1 ? fold[1] : scgib_slab_job{};
    const int per = statsz_per(n_nodes);
    const unsigned grid = static_cast<unsigned>(scgib_gin_bwd_stats_z_slabs(n_nodes) +
                                                slab_fold_blocks(f1) + slab_fold_blocks(f2));
    if (need_w)
        gin_bwd_statsz_k<true><<<dim3(grid), 256, 0, as_stream(stream)>>>(
            dz1, rowptr_t, col_t, one_plus_eps, w1, z2, stat, n_nodes, per, dy, bn_ws, dims, bz,
            wslab, f1, f2);
    else
        gin_bwd_statsz_k<false><<<dim3(grid), 256, 0, as_stream(stream)>>>(
            dz1, rowptr_t, col_t, one_plus_eps, w1, z2, stat, n_nodes, per, dy, bn_ws, dims, bz,
            wslab, f1, f2);
    return launch_status();
}

// workgroups per tile of scgib_mlp2_bwd: 2 for d_in = 128 while the doubled
// grid fits the chip (the fine-tune MLP's ~13 tiles: each workgroup's dW1 /
// d(agg) MFMA chain halves, tools/mlp_trace.py), else 1
static int mlp2_split(int64_t nt, int32_t d_in) {
    return d_in == 128 && 2 * static_cast<int64_t>(bwd_grid(nt)) <= kCUs ? 2 : 1;
}

extern "C" int64_t scgib_mlp2_slab_floats(int64_t n_nodes, int32_t d_in) {
    const int64_t nt = scgib_gin_tiles(n_nodes);
    return static_cast<int64_t>(bwd_grid(nt)) * mlp2_split(nt, d_in) * (64 * 64 + 64 * d_in + 128);
}

// the recon heads' backward (scgib_mlp2_recon_bwd / _contrastive_bwd): one
// slab per tile workgroup, no split (their grid also holds the contrastive
// workgroups)
extern "C" int64_t scgib_mlp2_recon_slab_floats(int64_t n_nodes, int32_t d_in) {
    return static_cast<int64_t>(bwd_grid(scgib_gin_tiles(n_nodes))) * (64 * 64 + 64 * d_in + 128);
}

extern "C" int scgib_mlp2_fwd(const float *x, int32_t d_in, int64_t n_nodes, const float *w1,
                              const float *b1, const float *w2, const float *b2, float *r,
                              float *out, const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes < 0 || (d_in != 64 && d_in != 128)) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!x || !w1 || !b1 || !w2 || !b2 || !r || !out) return SCGIB_EINVAL;
    const unsigned nt = static_cast<unsigned>(scgib_gin_tiles(n_nodes));
    hipStream_t st = as_stream(stream);
    if (d_in == 128)
        gin_fwd_k<128, false, false><<<nt, 256, 0, st>>>(x, nullptr, nullptr, nullptr, nullptr, n_nodes, 0.f, w1, b1, w2, b2, nullptr, r, out, nullptr, dims, BnFwdFuse{}, PreArgs{}, scgib_bn_pending{}, ReconArgs{});
    else
        gin_fwd_k<64, false, false><<<nt, 256, 0, st>>>(x, nullptr, nullptr, nullptr, nullptr, n_nodes, 0.f, w1, b1, w2, b2, nullptr, r, out, nullptr, dims, BnFwdFuse{}, PreArgs{}, scgib_bn_pending{}, ReconArgs{});
    return launch_status();
}

extern "C" int scgib_mlp2_bwd(const float *dout, const float *x, const float *r, int32_t d_in,
                              const float *w1, const float *w2, int64_t n_nodes, float *dx,
                              float *slab, float *wgrad, const int32_t *dims,
                              scgib_stream_t stream) {
    if (n_nodes <= 0 || (d_in != 64 && d_in != 128)) return SCGIB_EINVAL;
    if (!dout || !x || !r || !w1 || !w2 || !dx || !slab) return SCGIB_EINVAL;
    const int64_t nt = scgib_gin_tiles(n_nodes);
    const int ns = mlp2_split(nt, d_in), grid = bwd_grid(nt) * ns;
    hipStream_t st = as_stream(stream);
    if (d_in == 128)
        gin_bwd_k<128, false><<<grid, 256, 0, st>>>(dout, nullptr, r, x, nullptr, nullptr, w1, w2, n_nodes, nt, dx, slab, dims, nullptr, scgib_bn_bwd_pending{}, ReconArgs{}, kPreF, nullptr, ns);
    else
        gin_bwd_k<64, false><<<grid, 256, 0, st>>>(dout, nullptr, r, x, nullptr, nullptr, w1, w2, n_nodes, nt, dx, slab, dims, nullptr, scgib_bn_bwd_pending{}, ReconArgs{});
    const int rc = launch_status();
    if (rc != SCGIB_OK || !wgrad) return rc;  // wgrad NULL: the caller reduces the slabs
    return launch_slab_reduce(slab, grid, 64 * 64 + 64 * static_cast<int64_t>(d_in) + 128, wgrad, st);
}

// ---------------------------------------------------------------------------
// Head MLP + adjacency reconstruction loss, fused (Mainmodel / _continue with
// recons_type 'adj': models.py:1174 then :1256-1262).  Forward: mlp2 with a
// Gram partial per tile, then recon_fin_k (Gram reduce + edge term + loss).
// Backward: mlp2 backward whose tile dy is d IM of the recon loss.
// ---------------------------------------------------------------------------
extern "C" int64_t scgib_mlp2_recon_ws_floats(int64_t n_nodes) {
    // gram slabs [tiles][4096] | gram [4096] | 512 doubles
    return n_nodes <= 0 ? 0 : scgib_gin_tiles(n_nodes) * 4096 + 4096 + 2 * 512;
}

static bool g_recon_fold = true;  // scgib_set_recon_fold (tests: both paths bit-equal)
extern "C" int scgib_set_recon_fold(int on) {
    const int prev = g_recon_fold ? 1 : 0;
    g_recon_fold = on != 0;
    return prev;
}

// co-resident workgroups of the head MLP launch on the current device (the
// fused loss finish makes its tiles wait on each other)
template <int DIN>
static int64_t recon_fold_slots() {
    static int64_t slots = -1;
    if (slots < 0) {
        int dev = 0, cus = 0, per = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(
                &per, gin_fwd_k<DIN, false, false, false, true>, 256, 0) != hipSuccess)
            return 0;
        slots = static_cast<int64_t>(cus) * per;
    }
    return slots;
}

static int mlp2_recon_fwd(const float *x, int32_t d_in, int64_t n_nodes, const float *w1,
                          const float *b1, const float *w2, const float *b2, float *r,
                          float *out, const int32_t *rowptr, const int32_t *col, int64_t n_edges,
                          float *ws, uint32_t *counter, float *loss, const int32_t *dims,
                          const ContrastArgs &con, const scgib_running_update *ru,
                          const uint32_t *fault, scgib_stream_t stream) {
    if (n_nodes <= 0 || n_edges < 0 || (d_in != 64 && d_in != 128)) return SCGIB_EINVAL;
    if (!x || !w1 || !b1 || !w2 || !b2 || !r || !out || !rowptr || (n_edges > 0 && !col) || !ws ||
        !counter || !loss)
        return SCGIB_EINVAL;
    const int64_t nt = scgib_gin_tiles(n_nodes);
    float *gram = ws + nt * 4096;
    double *wsd = reinterpret_cast<double *>(gram + 4096);
    ReconArgs rec{};
    rec.gslab = ws;
    rec.con = con;
    rec.con.nmain = static_cast<int>(nt);
    rec.ru_block = -1;
    const int64_t ncon = con.B > 0 ? contrast_row_blocks(con.B) * con.nsplit : 0;
    const bool with_ru = ru && ru->n_graphs > 0;
    hipStream_t st = as_stream(stream);
    // the loss finish inside this launch when every workgroup is co-resident
    // (the head tiles hold one CU each, 101 + 27 KB of LDS): the tiles wait for
    // each other, so a grid past the co-resident slots would not finish — two
    // launches then
    const int64_t grid = nt + ncon + (with_ru && d_in == 128 ? 1 : 0);
    const bool fold = g_recon_fold && (!with_ru || d_in == 128) &&
                      grid <= (d_in == 128 ? recon_fold_slots<128>() : recon_fold_slots<64>());
    if (fold) {
        rec.fin = ReconFin{ws, out, rowptr, col, n_edges, gram, wsd,
                           reinterpret_cast<unsigned *>(counter), loss,
                           reinterpret_cast<const unsigned *>(fault)};
        rec.fin_on = 1;
        if (with_ru) {
            rec.ru_block = static_cast<int>(nt + ncon);
            rec.ru = *ru;
        }
    }
    if (d_in == 128)
        gin_fwd_k<128, false, false, false, true><<<(unsigned)(fold ? grid : nt + ncon), 256, 0, st>>>(x, nullptr, nullptr, nullptr, nullptr, n_nodes, 0.f, w1, b1, w2, b2, nullptr, r, out, nullptr, dims, BnFwdFuse{}, PreArgs{}, scgib_bn_pending{}, rec);
    else
        gin_fwd_k<64, false, false, false, true><<<(unsigned)nt, 256, 0, st>>>(x, nullptr, nullptr, nullptr, nullptr, n_nodes, 0.f, w1, b1, w2, b2, nullptr, r, out, nullptr, dims, BnFwdFuse{}, PreArgs{}, scgib_bn_pending{}, rec);
    const int rc = launch_status();
    if (rc != SCGIB_OK || fold) return rc;
    return launch_recon_fin(ws, out, rowptr, col, n_nodes, n_edges, gram, wsd, counter, loss, dims,
                            ru, reinterpret_cast<const unsigned *>(fault), st);
}

extern "C" int scgib_mlp2_recon_fwd(const float *x, int32_t d_in, int64_t n_nodes,
                                    const float *w1, const float *b1, const float *w2,
                                    const float *b2, float *r, float *out,
                                    const int32_t *rowptr, const int32_t *col, int64_t n_edges,
                                    float *ws, uint32_t *counter, float *loss,
                                    const int32_t *dims, const uint32_t *fault,
                                    scgib_stream_t stream) {
    return mlp2_recon_fwd(x, d_in, n_nodes, w1, b1, w2, b2, r, out, rowptr, col, n_edges, ws,
                          counter, loss, dims, ContrastArgs{}, nullptr, fault, stream);
}

static bool contrast_ok(const float *z1, const float *z2, int64_t n_graphs, const float *cws,
                        const uint32_t *ccounters, int32_t d_in) {
    return n_graphs > 0 && n_graphs <= (int64_t{1} << 20) && z1 && z2 && cws && ccounters &&
           d_in == 128;
}

extern "C" int scgib_mlp2_recon_contrastive_fwd(
    const float *x, int32_t d_in, int64_t n_nodes, const float *w1, const float *b1,
    const float *w2, const float *b2, float *r, float *out, const int32_t *rowptr,
    const int32_t *col, int64_t n_edges, float *ws, uint32_t *counter, float *loss,
    const int32_t *dims, const float *z1, const float *z2, int64_t n_graphs, float *cws,
    float *closs, uint32_t *ccounters, const scgib_running_update *ru, const uint32_t *fault,
    scgib_stream_t stream) {
    if (!contrast_ok(z1, z2, n_graphs, cws, ccounters, d_in) || !closs) return SCGIB_EINVAL;
    if (ru && ru->n_graphs > 0 && (!ru->stats || !ru->graph_ptr || !ru->running_mean || !ru->running_var))
        return SCGIB_EINVAL;
    ContrastArgs con{z1, z2, n_graphs, cws, closs, nullptr, nullptr, nullptr,
                     reinterpret_cast<unsigned *>(ccounters), contrast_splits(n_graphs), 0};
    // the head tiles hold one CU each (101 KB LDS): the contrastive
    // workgroups take the CUs they leave, with as many column splits as fit
    // (each over more column tiles) rather than a second wave behind the
    // tiles; the loss does not depend on the split count (per-tile partials)
    const int64_t nrb = contrast_row_blocks(n_graphs);
    // (one CU kept for the running-update workgroup, so that the grid stays
    // within the CUs and the loss finish can run inside the launch)
    const int64_t ru_wg = ru && ru->n_graphs > 0 ? 1 : 0;
    const int64_t fit = n_nodes > 0 ? (kCUs - scgib_gin_tiles(n_nodes) - ru_wg) / nrb : con.nsplit;
    if (fit < 1) {  // not even one split fits beside the tiles: the two launches
        const int rc = scgib_contrastive_fwd(z1, z2, n_graphs, cws, closs, ccounters, stream);
        if (rc != SCGIB_OK) return rc;
        con = ContrastArgs{};
    } else if (fit < con.nsplit) {
        con.nsplit = static_cast<int>(fit);
    }
    return mlp2_recon_fwd(x, d_in, n_nodes, w1, b1, w2, b2, r, out, rowptr, col, n_edges, ws,
                          counter, loss, dims, con, ru, fault, stream);
}

static int mlp2_recon_bwd(const float *x, const float *r, const float *out, const float *ws,
                          int32_t d_in, const float *w1, const float *w2, int64_t n_nodes,
                          const int32_t *rowptr, const int32_t *col, const int32_t *rowptr_t,
                          const int32_t *col_t, const float *g_loss, float *dx, float *slab,
                          float *wgrad, const int32_t *dims, const ContrastArgs &con,
                          scgib_stream_t stream) {
    if (n_nodes <= 0 || (d_in != 64 && d_in != 128)) return SCGIB_EINVAL;
    if (!x || !r || !out || !ws || !w1 || !w2 || !rowptr || !col || !g_loss || !dx || !slab ||
        ((rowptr_t == nullptr) != (col_t == nullptr)))
        return SCGIB_EINVAL;
    const int64_t nt = scgib_gin_tiles(n_nodes);
    const int grid = bwd_grid(nt);
    ReconArgs rec{nullptr, out, ws + nt * 4096, rowptr, col, rowptr_t, col_t, g_loss, con};
    rec.con.nmain = grid;
    int64_t ncon = 0;
    if (con.B > 0) {
        // one workgroup per CU at this kernel's 256 VGPRs: the contrastive
        // workgroups take the CUs the MLP tiles leave idle (fewer column
        // splits, each over more column tiles) rather than queue behind them
        // (sized for two per CU instead: 1.3 % slower)
        const int64_t nrb = contrast_row_blocks(con.B);
        const int64_t fit = (kCUs - grid) / nrb;  // >= 1 (scgib_mlp2_recon_contrastive_bwd)
        rec.con.nsplit = static_cast<int>(fit < 1 ? 1 : (fit < con.nsplit ? fit : con.nsplit));
        ncon = nrb * rec.con.nsplit;
    }
    hipStream_t st = as_stream(stream);
    if (d_in == 128)
        gin_bwd_k<128, false, false, true><<<(unsigned)(grid + ncon), 256, 0, st>>>(nullptr, nullptr, r, x, nullptr, nullptr, w1, w2, n_nodes, nt, dx, slab, dims, nullptr, scgib_bn_bwd_pending{}, rec);
    else
        gin_bwd_k<64, false, false, true><<<grid, 256, 0, st>>>(nullptr, nullptr, r, x, nullptr, nullptr, w1, w2, n_nodes, nt, dx, slab, dims, nullptr, scgib_bn_bwd_pending{}, rec);
    const int rc = launch_status();
    if (rc != SCGIB_OK || !wgrad) return rc;  // wgrad NULL: the caller reduces the slabs
    return launch_slab_reduce(slab, grid, 64 * 64 + 64 * static_cast<int64_t>(d_in) + 128, wgrad, st);
}

extern "C" int scgib_mlp2_recon_bwd(const float *x, const float *r, const float *out,
                                    const float *ws, int32_t d_in, const float *w1,
                                    const float *w2, int64_t n_nodes, const int32_t *rowptr,
                                    const int32_t *col, const int32_t *rowptr_t,
                                    const int32_t *col_t, const float *g_loss, float *dx,
                                    float *slab, float *wgrad, const int32_t *dims,
                                    scgib_stream_t stream) {
    return mlp2_recon_bwd(x, r, out, ws, d_in, w1, w2, n_nodes, rowptr, col, rowptr_t, col_t,
                          g_loss, dx, slab, wgrad, dims, ContrastArgs{}, stream);
}

extern "C" int scgib_mlp2_recon_contrastive_bwd(
    const float *x, const float *r, const float *out, const float *ws, int32_t d_in,
    const float *w1, const float *w2, int64_t n_nodes, const int32_t *rowptr, const int32_t *col,
    const int32_t *rowptr_t, const int32_t *col_t, const float *g_loss, float *dx, float *slab,
    float *wgrad, const int32_t *dims, const float *z1, const float *z2, int64_t n_graphs,
    float *cws, const float *g_con, float *dz1, float *dz2, uint32_t *ccounters,
    scgib_stream_t stream) {
    if (!contrast_ok(z1, z2, n_graphs, cws, ccounters, d_in) || !g_con || !dz1 || !dz2)
        return SCGIB_EINVAL;
    ContrastArgs con{z1, z2, n_graphs, cws, nullptr, g_con, dz1, dz2,
                     reinterpret_cast<unsigned *>(ccounters) + 1, contrast_splits(n_graphs), 0};
    if (n_nodes > 0 && bwd_grid(scgib_gin_tiles(n_nodes)) + contrast_row_blocks(n_graphs) > kCUs) {
        // not even one column split fits beside the MLP tiles (one workgroup
        // per CU): the two launches, the contrastive one with all its splits
        const int rc = mlp2_recon_bwd(x, r, out, ws, d_in, w1, w2, n_nodes, rowptr, col, rowptr_t,
                                      col_t, g_loss, dx, slab, wgrad, dims, ContrastArgs{}, stream);
        if (rc != SCGIB_OK) return rc;
        return scgib_contrastive_bwd(z1, z2, n_graphs, cws, g_con, dz1, dz2, ccounters, stream);
    }
    return mlp2_recon_bwd(x, r, out, ws, d_in, w1, w2, n_nodes, rowptr, col, rowptr_t, col_t,
                          g_loss, dx, slab, wgrad, dims, con, stream);
}

// ---------------------------------------------------------------------------
// Layer 0 with transfer_d folded in (see gather_x_rows / gin_bwd_k<.., PRE>)
// ---------------------------------------------------------------------------
extern "C" int64_t scgib_gin_layer0_slab_width(void) {
    return 64 * 64 + 64 * 32 + 128 + kPreSlab;
}

extern "C" int scgib_gin_layer0_fwd(const float *x, int32_t n_feat, const int32_t *node_map,
                                    const float *wt, const int32_t *rowptr, const int32_t *col,
                                    int64_t n_nodes, float one_plus_eps, const float *w1,
                                    const float *b1, const float *w2, const float *b2, float *agg,
                                    float *aggx, float *r, float *z2, const float *gamma,
                                    const float *beta, float bn_eps, float momentum,
                                    float *running_mean, float *running_var,
                                    int64_t *num_batches_tracked, float *stat, float *bn_ws,
                                    uint32_t *counters, const int32_t *dims, int32_t defer,
                                    scgib_stream_t stream) {
    if (n_nodes <= 0 || n_feat < 1 || n_feat > kPreF) return n_nodes == 0 ? SCGIB_OK : SCGIB_EINVAL;
    if (!x || !wt || !rowptr || !col || !w1 || !b1 || !w2 || !b2 || !agg || !aggx || !z2 || !bn_ws)
        return SCGIB_EINVAL;  // (r may be NULL: not stored)
    if (counters && (!gamma || !beta || !stat || ((running_mean == nullptr) != (running_var == nullptr))))
        return SCGIB_EINVAL;
    BnFwdFuse fz{};
    if (counters)
        fz = BnFwdFuse{counters, bn_gpart(bn_ws, n_nodes), gamma, beta, running_mean, running_var,
                       stat, num_batches_tracked, bn_eps, momentum,
                       static_cast<int>(bn_groups(n_nodes)), defer ? 1 : 0};
    const PreArgs pre{x, node_map, wt, aggx, n_feat};
    const int64_t nt = scgib_gin_tiles(n_nodes);
    gin_fwd_k<32, false, true, true><<<dim3((unsigned)nt), 256, 0, as_stream(stream)>>>(
        nullptr, nullptr, nullptr, rowptr, col, n_nodes, one_plus_eps, w1, b1, w2, b2, agg, r, z2,
        bn_ws, dims, fz, pre, scgib_bn_pending{}, ReconArgs{});
    return launch_status();
}

extern "C" int scgib_gin_layer0_bwd(const float *dy, const float *z2, const float *r,
                                    const float *agg, const float *aggx, int32_t n_feat,
                                    const float *stat, const float *coef, const float *w1,
                                    const float *b1, const float *w2, int64_t n_nodes, float *slab,
                                    int32_t need_w, const int32_t *dims,
                                    const scgib_bn_bwd_pending *pending, scgib_stream_t stream) {
    if (n_nodes <= 0 || !dy || !z2 || (!r && !b1) || !aggx || !stat || (!coef && !pending) ||
        !w1 || !w2 || !slab || n_feat < 1 || n_feat > kPreF)
        return SCGIB_EINVAL;
    if ((need_w || !r) && !agg) return SCGIB_EINVAL;
    if (!need_w && !r) return SCGIB_EUNSUPPORTED;  // frozen weights: the stored-r kernel
    if (pending && (!pending->gpart || !pending->dgamma || !pending->dbeta)) return SCGIB_EINVAL;
    const scgib_bn_bwd_pending pd = pending ? *pending : scgib_bn_bwd_pending{};
    const int64_t nt = scgib_gin_tiles(n_nodes);
    if (!need_w)
        gin_bwd_k<32, true, true, false, false, false><<<bwd0_grid(nt), 256, 0, as_stream(stream)>>>(
            dy, z2, r, agg, stat, coef, w1, w2, n_nodes, nt, nullptr, slab, dims, aggx, pd, ReconArgs{},
            n_feat);
    else if (r)
        gin_bwd_k<32, true, true><<<bwd0_grid(nt), 256, 0, as_stream(stream)>>>(
            dy, z2, r, agg, stat, coef, w1, w2, n_nodes, nt, nullptr, slab, dims, aggx, pd, ReconArgs{},
            n_feat);
    else
        gin_bwd_k<32, true, true, false, true><<<bwd0_grid(nt), 256, 0, as_stream(stream)>>>(
            dy, z2, nullptr, agg, stat, coef, w1, w2, n_nodes, nt, nullptr, slab, dims, aggx, pd,
            ReconArgs{}, n_feat, b1);
    return launch_status();
}

// r = relu(agg W1^T + b1) with the forward's MFMA chain, i.e. bitwise the r
// gin_fwd_k computes (and the backward recomputes): one wave per 32 x 32
// block, operands straight from global memory (the chain, not the operand
// path, fixes the bits).  Inspection / tests: the ReLU decisions of a model
// step whose forward did not store r.
__global__ __launch_bounds__(256) void gin_hidden_k(const float *__restrict__ agg, int din,
                                                    const float *__restrict__ w1,
                                                    const float *__restrict__ b1, int64_t n,
                                                    float *__restrict__ r) {
    const int l = threadIdx.x & 63, li = l & 31, kk = l >> 5;
    const int64_t blk = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);  // 32 rows x 32 cols
    const int64_t row0 = (blk >> 1) * 32;
    const int col = static_cast<int>(blk & 1) * 32 + li;
    if (row0 >= n) return;  // wave-uniform
    const int64_t arow = row0 + li < n ? row0 + li : n - 1;
    f32x16 acc = zero16();
    for (int s = 0; s < din / 2; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(agg[arow * din + 2 * s + kk],
                                                  w1[col * din + 2 * s + kk], acc, 0, 0, 0);
    const float bias = b1[col];
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
        const int64_t row = row0 + acc_row(reg, l);
        if (row < n) r[row * 64 + col] = fmaxf(acc[reg] + bias, 0.f);
    }
}

extern "C" int scgib_gin_hidden(const float *agg, int32_t d_in, const float *w1, const float *b1,
                                int64_t n_nodes, float *r, scgib_stream_t stream) {
    if (n_nodes < 0 || (d_in != 32 && d_in != 64)) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!agg || !w1 || !b1 || !r) return SCGIB_EINVAL;
    const int64_t blocks = ((n_nodes + 31) / 32) * 2;
    gin_hidden_k<<<dim3(static_cast<unsigned>((blocks + 3) / 4)), 256, 0, as_stream(stream)>>>(
        agg, d_in, w1, b1, n_nodes, r);
    return launch_status();
}
