// Closed form of the B sequential momentum updates of the per-graph
// compressor BatchNorm (one nn.BatchNorm1d call per graph, models.py:642):
//   r_B = (1-m)^B r_0 + sum_i m (1-m)^(B-1-i) x_i
// in fp64.  NT threads = NT/16 contiguous graph partitions x 16 lanes (float4
// channel quads): partition p runs the recurrence S = (1-m) S + m x_i over its
// graphs (Horner form, a round's loads in flight together), then 64 threads
// (one per channel) chain the partitions in order, T = (1-m)^len_p T + S_p,
// and apply the decay of r_0.  Deterministic; closer to the exact recurrence
// than an fp32 sequential loop.  Used by bn_running_update_k (one 1024-thread
// workgroup) and by an extra 256-thread workgroup of recon_fin_k.
#pragma once
#include "common.h"

namespace scgib {

// the per-graph statistics slab (interaction.hip): batch mean of t at 0,
// centred sum of squares at 64, SCGIB_STATS_STRIDE floats per graph
constexpr int kRuMeanOff = 0, kRuSsqOff = 64;

struct RuD4 {
    double x, y, z, w;
};

template <int NT>
__device__ void running_update_body(const scgib_running_update &a) {
    constexpr int kParts = NT / 16, kRound = NT == 1024 ? 8 : 16;
    const int c4 = threadIdx.x & 15, part = threadIdx.x >> 4;
    const int64_t B = a.n_graphs;
    const double m = a.momentum, keep = 1.0 - static_cast<double>(a.momentum);
    const int64_t chunk = (B + kParts - 1) / kParts;
    const int64_t i0 = part * chunk, i1 = i0 + chunk < B ? i0 + chunk : B;
    __shared__ double sPow[3];  // keep^chunk, keep^(last partial length), keep^B
    if (threadIdx.x == NT - 1) {
        const int64_t last = B - (B - 1) / chunk * chunk;
        sPow[0] = pow(keep, static_cast<double>(chunk));
        sPow[1] = pow(keep, static_cast<double>(last));
        sPow[2] = pow(keep, static_cast<double>(B));
    }
    RuD4 am{0.0, 0.0, 0.0, 0.0}, av{0.0, 0.0, 0.0, 0.0};
    for (int64_t ib = i0; ib < i1; ib += kRound) {
        float4 xm[kRound], xs[kRound];
        int32_t g0[kRound], g1[kRound];
#pragma unroll
        for (int u = 0; u < kRound; ++u) {
            const int64_t i = ib + u < i1 ? ib + u : i1 - 1;  // clamped: loads stay unconditional
            const float *sl = a.stats + i * SCGIB_STATS_STRIDE;
            xm[u] = *reinterpret_cast<const float4 *>(sl + kRuMeanOff + 4 * c4);
            xs[u] = *reinterpret_cast<const float4 *>(sl + kRuSsqOff + 4 * c4);
            g0[u] = a.graph_ptr[i];
            g1[u] = a.graph_ptr[i + 1];
        }
#pragma unroll
        for (int u = 0; u < kRound; ++u) {
            if (ib + u < i1) {
                am.x = keep * am.x + m * static_cast<double>(xm[u].x);
                am.y = keep * am.y + m * static_cast<double>(xm[u].y);
                am.z = keep * am.z + m * static_cast<double>(xm[u].z);
                am.w = keep * am.w + m * static_cast<double>(xm[u].w);
                // unbiased variance = centred sum of squares / (n - 1)
                const double inv = 1.0 / static_cast<double>(g1[u] - g0[u] - 1);
                av.x = keep * av.x + m * (static_cast<double>(xs[u].x) * inv);
                av.y = keep * av.y + m * (static_cast<double>(xs[u].y) * inv);
                av.z = keep * av.z + m * (static_cast<double>(xs[u].z) * inv);
                av.w = keep * av.w + m * (static_cast<double>(xs[u].w) * inv);
            }
        }
    }
    __shared__ double pm[kParts][65], pv[kParts][65];
    pm[part][4 * c4] = am.x; pm[part][4 * c4 + 1] = am.y; pm[part][4 * c4 + 2] = am.z; pm[part][4 * c4 + 3] = am.w;
    pv[part][4 * c4] = av.x; pv[part][4 * c4 + 1] = av.y; pv[part][4 * c4 + 2] = av.z; pv[part][4 * c4 + 3] = av.w;
    __syncthreads();
    if (threadIdx.x < 64) {
        const int c = threadIdx.x;
        double sm = 0.0, sv = 0.0;
        for (int p = 0; p < kParts; ++p) {
            const int64_t b0 = p * chunk, b1 = b0 + chunk < B ? b0 + chunk : B;
            if (b1 <= b0) break;  // partitions past B are empty (and so are all later ones)
            const double d = b1 - b0 == chunk ? sPow[0] : sPow[1];
            sm = d * sm + pm[p][c];
            sv = d * sv + pv[p][c];
        }
        a.running_mean[c] = static_cast<float>(sPow[2] * a.running_mean[c] + sm);
        a.running_var[c] = static_cast<float>(sPow[2] * a.running_var[c] + sv);
        if (c == 0 && a.num_batches_tracked) *a.num_batches_tracked += B;
    }
}

}  // namespace scgib
