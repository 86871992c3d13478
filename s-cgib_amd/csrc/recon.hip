// Adjacency-reconstruction loss in Gram form (gfx950).
//
// Reference: loss_recon_adj (models.py:762-768, :1256-1262) materialises the
// dense N x N matrix IM IM^T - A of the whole batch (0.3 GB at QM9 B=512,
// ~3 GB at B >= 1024) and reduces it.  For a 0/1 adjacency of a simple graph
//   sum_{u,v} (<im_u,im_v> - A_uv)^2 = ||IM^T IM||_F^2 - 2 sum_E <im_u,im_v> + |E|
// exactly, so the loss needs the 64 x 64 Gram matrix G = IM^T IM plus one dot
// product per edge: O(N d^2) flops over one read of IM (HBM-bound), no N^2.
//
// recon_partial_k: each workgroup reduces a contiguous ~64-row range; its four
//   wavefronts each own one 32x32 quadrant of G and accumulate it with the
//   exact-f32 MFMA v_mfma_f32_32x32x2_f32 (two rows per instruction: lane l
//   feeds row l>>5, channel l&31 of the quadrant's A and B halves), then
//   the same wavefronts sum <im_v, sum_{u->v} im_u> for their rows.
// recon_finalize_k: 256 workgroups each reduce 16 Gram entries over the
//   partial slabs (16 partitions per entry, a few loads each, combined in
//   fixed order in fp64) and publish a partial ||G||^2 (agent-scope store);
//   the last-arriving workgroup (block_arrive, common.h: no L2 write-back
//   fence) forms the loss.  Deterministic for a given N.
// recon_bwd_k: grad_v = (g/N) (4 (IM G)_v - 2 ((A + A^T) IM)_v), G staged in
//   LDS, the row of IM broadcast from LDS.
#include "recon_fin.h"
#include "running_update.h"

namespace scgib {


// ~64 rows per partial workgroup (short dependent MFMA/load chains, enough
// workgroups to spread over the CUs), at most 1024 slabs
__host__ __device__ __forceinline__ int64_t recon_blocks(int64_t n) {
    int64_t g = (n + 63) / 64;
    return g < 1 ? 1 : (g > 1024 ? 1024 : g);
}

// partials layout (floats): [G][4096] gram slabs | edge sums [G, padded to a
// multiple of 4] | 16 doubles ||G||^2 partials | uint32 arrival counter (+pad)
__host__ __device__ __forceinline__ int64_t off_edge(int64_t G) { return G * kGram; }
__host__ __device__ __forceinline__ int64_t off_gsq(int64_t G) { return G * kGram + ((G + 3) & ~int64_t(3)); }
__host__ __device__ __forceinline__ int64_t off_cnt(int64_t G) { return off_gsq(G) + 2 * kFinBlocks; }
__global__ __launch_bounds__(256) void recon_partial_k(const float *__restrict__ im,
                                                       const int32_t *__restrict__ rowptr,
                                                       const int32_t *__restrict__ col,
                                                       int64_t ncap, int64_t rows_per_blk,
                                                       float *__restrict__ partials,
                                                       const int32_t *__restrict__ dims) {
    const int G = gridDim.x;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t n = eff_count(dims, 0, ncap);
    const int64_t rb = static_cast<int64_t>(blockIdx.x) * rows_per_blk;
    const int64_t re = rb + rows_per_blk < n ? rb + rows_per_blk : n;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // arrival counter of the finalize kernel (stream-ordered before it)
        *reinterpret_cast<unsigned *>(partials + off_cnt(G)) = 0u;
    }
    const int ta = w >> 1, tb = w & 1;
    const int kk = lane >> 5, ch = lane & 31;
    f32x16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    int64_t r = rb;
    for (; r + 8 <= re; r += 8) {
        float a[4], b[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int64_t row = r + 2 * q + kk;
            a[q] = im[row * 64 + ta * 32 + ch];
            b[q] = im[row * 64 + tb * 32 + ch];
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[q], b[q], acc, 0, 0, 0);
    }
    for (; r < re; r += 2) {
        const int64_t row = r + kk;
        const float a = row < re ? im[row * 64 + ta * 32 + ch] : 0.f;
        const float b = row < re ? im[row * 64 + tb * 32 + ch] : 0.f;
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    float *slab = partials + static_cast<int64_t>(blockIdx.x) * kGram;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const int row = (j & 3) + 8 * (j >> 2) + 4 * (lane >> 5);
        slab[(ta * 32 + row) * 64 + tb * 32 + (lane & 31)] = acc[j];
    }
    // edge term: sum over rows v of this block of <im_v, sum_{u->v} im_u>
    float e = 0.f;
    for (int64_t v = rb + w; v < re; v += 4) {
        float nb = 0.f;
        for (int32_t j = rowptr[v]; j < rowptr[v + 1]; ++j) nb += im[static_cast<int64_t>(col[j]) * 64 + lane];
        e += im[v * 64 + lane] * nb;
    }
    e = wave_sum(e);
    __shared__ float we[4];
    if (lane == 0) we[w] = e;
    __syncthreads();
    if (threadIdx.x == 0) partials[off_edge(G) + blockIdx.x] = ((we[0] + we[1]) + we[2]) + we[3];
}

__global__ __launch_bounds__(256) void recon_finalize_k(float *__restrict__ partials, int G,
                                                        int64_t ncap, int64_t ecap,
                                                        float *__restrict__ gram,
                                                        float *__restrict__ loss,
                                                        const int32_t *__restrict__ dims) {
    const int64_t n = eff_count(dims, 0, ncap), n_edges = eff_count(dims, 1, ecap);
    const int el = threadIdx.x & 15, sp = threadIdx.x >> 4;
    const int e = blockIdx.x * 16 + el;  // Gram entry
    double acc = 0.0;
    for (int b0 = sp; b0 < G; b0 += 16 * 8) {  // 8 independent loads in flight
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int b = b0 + 16 * j < G ? b0 + 16 * j : sp;  // clamped: unconditional loads
            v[j] = partials[(int64_t)b * kGram + e];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (b0 + 16 * j < G) acc += static_cast<double>(v[j]);
    }
    __shared__ double part[16][17];
    __shared__ double red[16];
    part[sp][el] = acc;
    __syncthreads();
    if (threadIdx.x < 16) {
        double g = 0.0;
#pragma unroll
        for (int k = 0; k < 16; ++k) g += part[k][threadIdx.x];
        gram[blockIdx.x * 16 + threadIdx.x] = static_cast<float>(g);
        red[threadIdx.x] = g * g;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double q = 0.0;
        for (int k = 0; k < 16; ++k) q += red[k];
        red[0] = q;
    }
    __syncthreads();
    double *gsq = reinterpret_cast<double *>(partials + off_gsq(G));
    unsigned *cnt = reinterpret_cast<unsigned *>(partials + off_cnt(G));
    if (threadIdx.x == 0) st_agent(&gsq[blockIdx.x], red[0]);
    if (!block_arrive(cnt, kFinBlocks)) return;  // not the last arriver
    // last arriver: ||G||^2 from the 256 partials and the edge term, fixed order
    __shared__ double fin[2][256];
    fin[0][threadIdx.x] = __hip_atomic_load(&gsq[threadIdx.x], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    double es = 0.0;
    const float *ep = partials + off_edge(G);
    for (int b = threadIdx.x; b < G; b += 256) es += static_cast<double>(ep[b]);
    fin[1][threadIdx.x] = es;
    __syncthreads();
    for (int off = 128; off >= 1; off >>= 1) {
        if (threadIdx.x < off) {
            fin[0][threadIdx.x] += fin[0][threadIdx.x + off];
            fin[1][threadIdx.x] += fin[1][threadIdx.x + off];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        *loss = static_cast<float>((fin[0][0] - 2.0 * fin[1][0] + static_cast<double>(n_edges)) /
                                   static_cast<double>(n));
}

__global__ __launch_bounds__(256) void recon_bwd_k(const float *__restrict__ im,
                                                   const float *__restrict__ gram,
                                                   const int32_t *__restrict__ rp_in,
                                                   const int32_t *__restrict__ c_in,
                                                   const int32_t *__restrict__ rp_out,
                                                   const int32_t *__restrict__ c_out, int64_t ncap,
                                                   const float *__restrict__ g_loss,
                                                   float *__restrict__ out,
                                                   const int32_t *__restrict__ dims) {
    const int64_t n = eff_count(dims, 0, ncap);
    __shared__ float sg[kGram];
    __shared__ float srow[4][64];
    for (int i = threadIdx.x; i < kGram; i += 256) sg[i] = gram[i];
    __syncthreads();
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const float scale = *g_loss / static_cast<float>(n);
    const int64_t rows_per_blk = 32;
    const int64_t rb = xcd_remap(blockIdx.x, gridDim.x) * rows_per_blk;
    for (int64_t v = rb + w; v < rb + rows_per_blk && v < ncap; v += 4) {
        if (v >= n) {
            out[v * 64 + lane] = 0.f;
            continue;
        }
        const float iv = im[v * 64 + lane];
        srow[w][lane] = iv;
        __builtin_amdgcn_wave_barrier();
        float acc = 0.f;
#pragma unroll 16
        for (int k = 0; k < 64; ++k) acc += srow[w][k] * sg[k * 64 + lane];
        float nb = 0.f;
        for (int32_t j = rp_in[v]; j < rp_in[v + 1]; ++j) nb += im[static_cast<int64_t>(c_in[j]) * 64 + lane];
        for (int32_t j = rp_out[v]; j < rp_out[v + 1]; ++j) nb += im[static_cast<int64_t>(c_out[j]) * 64 + lane];
        out[v * 64 + lane] = scale * (4.f * acc - 2.f * nb);
        __builtin_amdgcn_wave_barrier();
    }
}

// ---------------------------------------------------------------------------
// Fused path (the pretraining model's): the head MLP forward already wrote one
// Gram partial per 64-row tile (gin_fwd_k<.., RECON>).  When the MLP launch
// cannot finish the loss itself (more tiles than fit the chip beside its other
// workgroups, gin_layer.hip), this launch does: kFinBlocks workgroups, the
// first V = min(tiles, 256) one virtual block each (recon_fin.h), plus
// optionally one workgroup for the compressor BatchNorm's running update.
// The backward is fused into the head MLP backward (gin_bwd_k<.., RECON>).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void recon_fin_k(const ReconFin a, int64_t ncap,
                                                   const int32_t *__restrict__ dims,
                                                   const scgib_running_update ru) {
    if (blockIdx.x == kFinBlocks) {  // (block-uniform) the extra workgroup: the running update
        running_update_body<256>(ru);
        return;
    }
    if (static_cast<int>(blockIdx.x) >= recon_fin_vblocks(eff_count(dims, 0, ncap))) return;
    recon_fin_block(static_cast<int>(blockIdx.x), a, ncap, dims, false);
}

int launch_recon_fin(const float *gslab, const float *im, const int32_t *rowptr,
                     const int32_t *col, int64_t n_nodes, int64_t n_edges, float *gram,
                     double *wsd, unsigned *cnt, float *loss, const int32_t *dims,
                     const scgib_running_update *ru, const unsigned *fault, hipStream_t st) {
    const bool with_ru = ru && ru->n_graphs > 0;
    const ReconFin a{gslab, im, rowptr, col, n_edges, gram, wsd, cnt, loss, fault};
    recon_fin_k<<<kFinBlocks + (with_ru ? 1 : 0), 256, 0, st>>>(
        a, n_nodes, dims, with_ru ? *ru : scgib_running_update{});
    return launch_status();
}

// ---------------------------------------------------------------------------
// A15: logM reconstruction loss (models.py:770-782), per molecule g with
// X = IM rows of g, h = X X^T and the k targets L_i [n, n]:
//   loss = (1/k) sum_g sum_i sum_uv (h_uv - L_i,uv)^2 / n_g^2
//        = sum_g [k ||h||^2 - 2 <h, S_g> + C_g] / (k n_g^2),
//   S_g = sum_i L_i, C_g = sum_i ||L_i||^2 (precomputed, graph.LogMBatch);
//   d loss / d X = 2 g (2k h - S - S^T) X / (k n_g^2).
// One workgroup per molecule; 16 row groups x 16 lanes (float4 channels):
// h_uv = 16-lane butterfly of the row dots, never materialised.  fp64
// accumulation of the expanded loss (the terms cancel when h ~ L).
// ---------------------------------------------------------------------------
__device__ __forceinline__ float red16_sum(float v) {
    v += __shfl_xor(v, 1, kWave);
    v += __shfl_xor(v, 2, kWave);
    v += __shfl_xor(v, 4, kWave);
    v += __shfl_xor(v, 8, kWave);
    return v;
}

__global__ __launch_bounds__(256) void recon_logm_fwd_k(const float *__restrict__ im,
                                                        const int32_t *__restrict__ gptr,
                                                        const float *__restrict__ S,
                                                        const int64_t *__restrict__ soff,
                                                        const double *__restrict__ C, int kstep,
                                                        float *__restrict__ lossg) {
    const int64_t g = blockIdx.x;
    const int64_t r0 = gptr[g];
    const int n = gptr[g + 1] - static_cast<int>(r0);
    const int grp = threadIdx.x >> 4, lane = threadIdx.x & 15;
    const float *Sg = S + soff[g];
    const float4 *x4 = reinterpret_cast<const float4 *>(im);
    const float k = static_cast<float>(kstep);
    double acc = 0.0;
    for (int u = grp; u < n; u += 16) {
        const float4 xu = x4[(r0 + u) * 16 + lane];
        for (int v = 0; v < n; ++v) {
            const float4 xv = x4[(r0 + v) * 16 + lane];
            const float h = red16_sum(xu.x * xv.x + xu.y * xv.y + xu.z * xv.z + xu.w * xv.w);
            acc += static_cast<double>(k * h * h) - 2.0 * static_cast<double>(h) * Sg[int64_t(u) * n + v];
        }
    }
    __shared__ double red[16];
    if (lane == 0) red[grp] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int q = 0; q < 16; ++q) t += red[q];
        lossg[g] = n > 0 ? static_cast<float>((t + C[g]) / (static_cast<double>(kstep) * n * n)) : 0.f;
    }
}

__global__ __launch_bounds__(256) void recon_logm_bwd_k(const float *__restrict__ im,
                                                        const int32_t *__restrict__ gptr,
                                                        const float *__restrict__ S,
                                                        const int64_t *__restrict__ soff,
                                                        int kstep,
                                                        const float *__restrict__ g_loss,
                                                        float *__restrict__ grad) {
    const int64_t g = blockIdx.x;
    const int64_t r0 = gptr[g];
    const int n = gptr[g + 1] - static_cast<int>(r0);
    const int grp = threadIdx.x >> 4, lane = threadIdx.x & 15;
    const float *Sg = S + soff[g];
    const float4 *x4 = reinterpret_cast<const float4 *>(im);
    const float k2 = 2.f * static_cast<float>(kstep);
    const float coef = n > 0 ? 2.f * *g_loss / (static_cast<float>(kstep) * n * n) : 0.f;
    for (int u = grp; u < n; u += 16) {
        const float4 xu = x4[(r0 + u) * 16 + lane];
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int v = 0; v < n; ++v) {
            const float4 xv = x4[(r0 + v) * 16 + lane];
            const float h = red16_sum(xu.x * xv.x + xu.y * xv.y + xu.z * xv.z + xu.w * xv.w);
            const float w = k2 * h - Sg[int64_t(u) * n + v] - Sg[int64_t(v) * n + u];
            acc.x += w * xv.x; acc.y += w * xv.y; acc.z += w * xv.z; acc.w += w * xv.w;
        }
        reinterpret_cast<float4 *>(grad)[(r0 + u) * 16 + lane] =
            make_float4(coef * acc.x, coef * acc.y, coef * acc.z, coef * acc.w);
    }
}

}  // namespace scgib

using namespace scgib;

extern "C" int scgib_recon_logm_fwd(const float *im, const int32_t *graph_ptr, int64_t n_graphs,
                                    const float *S, const int64_t *s_offsets, const double *C,
                                    int32_t kstep, float *loss_graphs, float *loss,
                                    scgib_stream_t stream) {
    if (n_graphs <= 0 || kstep <= 0 || !im || !graph_ptr || !S || !s_offsets || !C ||
        !loss_graphs || !loss)
        return SCGIB_EINVAL;
    if (n_graphs > 0x7fffffff) return SCGIB_EUNSUPPORTED;
    hipStream_t st = as_stream(stream);
    recon_logm_fwd_k<<<static_cast<unsigned>(n_graphs), 256, 0, st>>>(im, graph_ptr, S, s_offsets,
                                                                      C, kstep, loss_graphs);
    const int rc = launch_status();
    if (rc != SCGIB_OK) return rc;
    return launch_slab_reduce(loss_graphs, static_cast<int>(n_graphs), 1, loss, st);
}

extern "C" int scgib_recon_logm_bwd(const float *im, const int32_t *graph_ptr, int64_t n_graphs,
                                    const float *S, const int64_t *s_offsets, int32_t kstep,
                                    const float *g_loss, float *grad_im, scgib_stream_t stream) {
    if (n_graphs <= 0 || kstep <= 0 || !im || !graph_ptr || !S || !s_offsets || !g_loss ||
        !grad_im)
        return SCGIB_EINVAL;
    if (n_graphs > 0x7fffffff) return SCGIB_EUNSUPPORTED;
    recon_logm_bwd_k<<<static_cast<unsigned>(n_graphs), 256, 0, as_stream(stream)>>>(
        im, graph_ptr, S, s_offsets, kstep, g_loss, grad_im);
    return launch_status();
}

extern "C" int64_t scgib_recon_partials_floats(int64_t n_nodes) {
    return off_cnt(recon_blocks(n_nodes)) + 4;
}

extern "C" int scgib_recon_fwd(const float *im, const int32_t *rowptr, const int32_t *col,
                               int64_t n_nodes, int64_t n_edges, float *partials, float *gram,
                               float *loss, const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes <= 0 || n_edges < 0) return SCGIB_EINVAL;
    if (!im || !rowptr || (n_edges > 0 && !col) || !partials || !gram || !loss) return SCGIB_EINVAL;
    const int64_t G = recon_blocks(n_nodes);
    int64_t rows = (n_nodes + G - 1) / G;
    rows += rows & 1;  // even: the MFMA consumes rows in pairs
    hipStream_t st = as_stream(stream);
    recon_partial_k<<<dim3((unsigned)G), 256, 0, st>>>(im, rowptr, col, n_nodes, rows, partials, dims);
    recon_finalize_k<<<kFinBlocks, 256, 0, st>>>(partials, (int)G, n_nodes, n_edges, gram, loss, dims);
    return launch_status();
}

extern "C" int scgib_recon_bwd(const float *im, const float *gram, const int32_t *rowptr_in,
                               const int32_t *col_in, const int32_t *rowptr_out,
                               const int32_t *col_out, int64_t n_nodes, const float *g_loss,
                               float *grad_im, const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes <= 0) return SCGIB_EINVAL;
    if (!im || !gram || !rowptr_in || !rowptr_out || !g_loss || !grad_im) return SCGIB_EINVAL;
    const int64_t grid = (n_nodes + 31) / 32;
    recon_bwd_k<<<dim3((unsigned)grid), 256, 0, as_stream(stream)>>>(
        im, gram, rowptr_in, col_in, rowptr_out, col_out, n_nodes, g_loss, grad_im, dims);
    return launch_status();
}
