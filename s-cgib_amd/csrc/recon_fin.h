// The forward finish of the adjacency-reconstruction loss (recon.hip for the
// Gram form), as one 256-thread workgroup body over a virtual block index, so
// that it runs either as recon_fin_k (one launch of kFinBlocks workgroups) or
// inside the head MLP launch (gin_layer.hip, gin_fwd_k<.., RECON>): the MLP
// tiles, once every tile's Gram partial and output rows are published, work
// through the kFinBlocks virtual blocks themselves.  The same virtual block
// decomposition and fixed-order sums either way: the loss bits do not depend
// on which launch ran it.
//
// V = min(tiles, kFinBlocks) virtual blocks (a function of the actual N only,
// so both launch forms use the same decomposition; inside the MLP launch each
// tile is one virtual block).  Virtual block vb:
//   * the edge term of its row range [vb R, vb R + R), R = ceil(N / V) (one
//     64-row pass while N <= 256 tiles): sum_v <im_v, sum_{u->v} im_u> with
//     the latency-batched CSR gather (16 lanes x float4 per row);
//   * Gram chunks c = vb, vb + V, ... < 256 of 16 entries each, reduced over
//     the tile partials (16 partitions x 8 loads in flight, fp64, fixed
//     order) -> G and its share of ||G||^2;
//   * the last of the V arrivals (block_arrive: agent-scope data, no L2
//     write-back fence) forms loss = (sum ||G||^2 - 2 sum E + |E|) / N in
//     fixed order and resets the counters.
#pragma once
#include "mfma_tile.h"

namespace scgib {

constexpr int kGram = 64 * 64;
// finalize: at most 256 virtual blocks; 256 Gram chunks of 16 entries
constexpr int kFinBlocks = kGram / 16;

struct ReconFin {
    const float *gslab;      // [tiles][4096] Gram partials of the MLP tiles
    const float *im;         // MLP output [N][64]
    const int32_t *rowptr, *col;
    int64_t ecap;
    float *gram;             // G [64][64]
    double *wsd;             // 2 * kFinBlocks doubles
    unsigned *cnt;           // [0] arrivals of the virtual blocks, [1] (fused) tile arrivals,
                             // [2] (fused) wait-timeout flag; all left zero
    float *loss;
    const unsigned *fault;   // sticky hand-off fault word (scgib_stream_wait), or nullptr:
                             // while it is set the loss is NaN
};

__device__ __forceinline__ int recon_fin_vblocks(int64_t n) {
    const int64_t t = (n + TM - 1) / TM;
    return static_cast<int>(t < kFinBlocks ? (t < 1 ? 1 : t) : kFinBlocks);
}

__device__ void recon_fin_block(int vb, const ReconFin &a, int64_t ncap, const int32_t *dims,
                                bool fused) {
    const int64_t n = eff_count(dims, 0, ncap), n_edges = eff_count(dims, 1, a.ecap);
    const int64_t ntiles = (n + TM - 1) / TM;
    const int V = recon_fin_vblocks(n);
    const int tid = threadIdx.x;
    // edge term: this block's rows (issued first: three dependent load rounds)
    const int64_t R = (n + V - 1) / V;
    const int64_t rb = static_cast<int64_t>(vb) * R;
    const int64_t re = rb + R < n ? rb + R : n;
    const float4 *im4 = reinterpret_cast<const float4 *>(a.im);
    const float4 one = make_float4(1.f, 1.f, 1.f, 1.f), zero = make_float4(0.f, 0.f, 0.f, 0.f);
    const int c = tid & 15, rbase = tid >> 4;
    float e = 0.f;
    for (int64_t r0 = rb; r0 < re; r0 += TM) {
        const int nv = static_cast<int>(re - r0 < TM ? re - r0 : TM);
        GatherHead<4> hd;
        float4 nb[4];
        gather_head<4, 16, 16>(im4, a.rowptr, r0, nv, rbase, c, hd);
        gather_tail<4, 16, false>(im4, a.col, hd, c, 0.f, one, zero, nb);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float d = hd.self[k].x * nb[k].x + hd.self[k].y * nb[k].y +
                            hd.self[k].z * nb[k].z + hd.self[k].w * nb[k].w;
            e += rbase + 16 * k < nv ? d : 0.f;
        }
    }
    SCGIB_MARK(8);
    __shared__ double part[16][17];
    __shared__ double sE[256];
    __shared__ double red[16];
    sE[tid] = static_cast<double>(e);
    // Gram chunks over the tile partials
    const int el = tid & 15, sp = tid >> 4;
    double q = 0.0;  // (thread 0) this block's share of ||G||^2, chunks in order
    if (ntiles >= 8 && ntiles <= 64) {  // block-uniform
        // few tiles, so each block has up to 32 chunks: each thread owns whole
        // entries with their tile partials in flight NB at a time, instead of
        // one chunk per load round trip (B = 32: 29 rounds, 21 us).  The same
        // sums in the same order as the loop below: partition k = tiles k,
        // k + 16, k + 32, k + 48 from 0.0, then the 16 partitions in order;
        // ||G||^2 over (chunk, entry) in order
        __shared__ double sq[512];
        const int nent = (kFinBlocks - vb + V - 1) / V * 16;  // <= 32 chunks (V >= 8)
        auto entries = [&](auto nbc) {
            constexpr int NB = decltype(nbc)::value;
            for (int e = tid; e < nent; e += 256) {
                const int ent = (vb + (e >> 4) * V) * 16 + (e & 15);
                double p[16];
#pragma unroll
                for (int k = 0; k < 16; ++k) p[k] = 0.0;
                for (int b0 = 0; b0 < ntiles; b0 += NB) {
                    float v[NB];
#pragma unroll
                    for (int b = 0; b < NB; ++b)
                        v[b] = a.gslab[(b0 + b < ntiles ? b0 + b : 0) * kGram + ent];
#pragma unroll
                    for (int b = 0; b < NB; ++b)
                        if (b0 + b < ntiles) p[b % 16] += static_cast<double>(v[b]);
                }
                double g = 0.0;
#pragma unroll
                for (int k = 0; k < 16; ++k) g += p[k];
                a.gram[ent] = static_cast<float>(g);
                sq[e] = g * g;
            }
        };
        if (ntiles <= 16) entries(std::integral_constant<int, 16>{});
        else entries(std::integral_constant<int, 32>{});
        __syncthreads();
        if (tid == 0)
            for (int e = 0; e < nent; ++e) q += sq[e];
    } else {  // one chunk at a time, 16 partitions x 8 tile loads in flight
        for (int ch = vb; ch < kFinBlocks; ch += V) {
            const int ent = ch * 16 + el;
            double acc = 0.0;
            for (int64_t b0 = sp; b0 < ntiles; b0 += 16 * 8) {
                float v[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int64_t b = b0 + 16 * j < ntiles ? b0 + 16 * j : sp;  // clamped: unconditional
                    v[j] = a.gslab[b * kGram + ent];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (b0 + 16 * j < ntiles) acc += static_cast<double>(v[j]);
            }
            part[sp][el] = acc;
            __syncthreads();
            if (tid < 16) {
                double g = 0.0;
#pragma unroll
                for (int k = 0; k < 16; ++k) g += part[k][tid];
                a.gram[ch * 16 + tid] = static_cast<float>(g);
                red[tid] = g * g;
            }
            __syncthreads();
            if (tid == 0)
                for (int k = 0; k < 16; ++k) q += red[k];
        }
    }
    SCGIB_MARK(9);
    for (int off = 128; off >= 1; off >>= 1) {
        if (tid < off) sE[tid] += sE[tid + off];
        __syncthreads();
    }
    if (tid == 0) {
        st_agent(&a.wsd[vb], q);
        st_agent(&a.wsd[kFinBlocks + vb], sE[0]);
    }
    if (!block_arrive(a.cnt, static_cast<unsigned>(V))) return;  // not the last arrival
    __shared__ double fin[2][256];
    fin[0][tid] = tid < V ? ld_agent(&a.wsd[tid]) : 0.0;
    fin[1][tid] = tid < V ? ld_agent(&a.wsd[kFinBlocks + tid]) : 0.0;
    __syncthreads();
    for (int off = 128; off >= 1; off >>= 1) {
        if (tid < off) {
            fin[0][tid] += fin[0][tid + off];
            fin[1][tid] += fin[1][tid + off];
        }
        __syncthreads();
    }
    if (tid == 0) {
        const double l = (fin[0][0] - 2.0 * fin[1][0] + static_cast<double>(n_edges)) / static_cast<double>(n);
        bool timed_out = false;
        if (fused) {
            // every waiting tile has passed its wait by now (each one ran a
            // virtual block before this last arrival; the tiles past V do not
            // wait): the words can reset
            timed_out = __hip_atomic_load(&a.cnt[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
            __hip_atomic_store(&a.cnt[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&a.cnt[2], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // a cross-queue hand-off of this or an earlier step gave up waiting:
        // some kernel read data before it was written, so no loss is reported
        if (a.fault && __hip_atomic_load(a.fault, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u)
            timed_out = true;
        *a.loss = timed_out ? __builtin_nanf("") : static_cast<float>(l);
        __hip_atomic_store(&a.cnt[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch / replay
    }
}

}  // namespace scgib
