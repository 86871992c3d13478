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
// against the 64-row column tiles of its split.  The column tile is
// normalised into LDS (stride 68: 16-byte reads of 16 different rows hit
// disjoint banks); the similarity blocks and the backward's weighted sums
// are f32 MFMA products (v_mfma_f32_16x16x4_f32, the query rows' operand
// values held in registers, the tiles read by ds_read_b128).
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
// stage_tile in two halves, so the next tile's loads can be in flight while
// the current one is computed on: tile_load (rows -> registers, rows >= B
// zero), tile_store (normalise -> LDS).  256 threads: row tid >> 2, 16
// channels per thread.
struct TileRegs {
    float4 v[4];
};

__device__ __forceinline__ void tile_load(const float *__restrict__ x, int64_t B, int64_t j0,
                                          TileRegs &t) {
    const int tid = threadIdx.x, r = tid >> 2, q = tid & 3;
    const int64_t j = j0 + r;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        t.v[k] = ld_ok(reinterpret_cast<const float4 *>(x), j * 16 + 4 * q + k, 4 * q + k, j < B,
                       make_float4(0.f, 0.f, 0.f, 0.f));
}

__device__ __forceinline__ void tile_store(const TileRegs &t, float *s) {
    const int tid = threadIdx.x, r = tid >> 2, q = tid & 3;
    float ss = 0.f;
#pragma unroll
    for (int k = 0; k < 4; ++k) ss += t.v[k].x * t.v[k].x + t.v[k].y * t.v[k].y + t.v[k].z * t.v[k].z + t.v[k].w * t.v[k].w;
    ss += __shfl_xor(ss, 1, kWave);
    ss += __shfl_xor(ss, 2, kWave);
    const float inv = 1.f / fmaxf(sqrtf(ss), kNormEps);
#pragma unroll
    for (int k = 0; k < 4; ++k)
        *reinterpret_cast<float4 *>(s + r * CLD + 16 * q + 4 * k) =
            make_float4(t.v[k].x * inv, t.v[k].y * inv, t.v[k].z * inv, t.v[k].w * inv);
}

// Stage rows [j0, j0 + 64) of x, normalised, into s (64 x CLD); rows >= B are zero.
__device__ __forceinline__ void stage_tile(const float *__restrict__ x, int64_t B, int64_t j0,
                                           float *s) {
    TileRegs t;
    tile_load(x, B, j0, t);
    tile_store(t, s);
}

// sum over the 16 lanes of a row group (lanes 16m .. 16m+15 of the wave)
__device__ __forceinline__ float sum16(float v) {
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kContrastBwdW = 3 * CR * CLD;

__device__ __forceinline__ int kperm16(int s, int kq) { return 16 * (s >> 2) + 4 * kq + (s & 3); }
__device__ __forceinline__ float f4c(const float4 &v, int t) {
    return t == 0 ? v.x : t == 1 ? v.y : t == 2 ? v.z : v.w;
}

// lane (row li, k quarter kq): the row's normalised values at kperm16(s, kq)
__device__ __forceinline__ void load_row_k(const float *__restrict__ x, int64_t i, int64_t B,
                                           int kq, float (&q)[16]) {
    const int64_t ic = i < B ? i : 0;
    const float m = i < B ? 1.f : 0.f;
    float4 v[4];
    float ss = 0.f;
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) {
        v[mm] = *reinterpret_cast<const float4 *>(x + ic * 64 + 16 * mm + 4 * kq);
        ss += v[mm].x * v[mm].x + v[mm].y * v[mm].y + v[mm].z * v[mm].z + v[mm].w * v[mm].w;
    }
    ss += __shfl_xor(ss, 16, kWave);
    ss += __shfl_xor(ss, 32, kWave);
    const float inv = m / fmaxf(sqrtf(ss), kNormEps);
#pragma unroll
    for (int s = 0; s < 16; ++s) q[s] = f4c(v[s >> 2], s & 3) * inv;
}

// workspace (floats): D[B] | fwd partials [T][B][4] | bwd partials [S][B][128],
// T = contrast_tiles(B), S = contrast_splits(B); a launch may use NS <= S splits.
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
// column tiles; the forward keeps one partial per (tile, row), so the loss
// does not depend on how a launch splits the tiles over workgroups
__host__ __device__ inline int64_t contrast_tiles(int64_t B) { return (B + CT - 1) / CT; }
// workspace offset of the backward's split partials (after D and the
// forward's tile partials)
__host__ __device__ inline int64_t contrast_pb_offset(int64_t B) { return B + 4 * contrast_tiles(B) * B; }

// forward body: sK1, sK2 >= CT * CLD floats each.  S11 = Q1 K1^T and
// S12 = Q1 K2^T per 64-column tile on the f32 MFMA (as the backward: wave w
// takes columns 16w.. of the tile, lanes hold rows 4 kq + r), their
// exponentials summed per lane over the tiles, then over the 16 columns of
// a wave (shuffles) and the 4 waves (LDS, fixed order).
__device__ __forceinline__ void contrast_fwd_body(const ContrastArgs &a, int64_t bx, int by,
                                                  float *sK1, float *sK2) {
    const float *__restrict__ z1 = a.z1, *__restrict__ z2 = a.z2;
    const int64_t B = a.B;
    float *__restrict__ ws = a.ws;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, li = l & 15, kq = l >> 4;
    const int NS = a.nsplit;
    const int64_t row0 = bx * CR;
    float q1[16];
    load_row_k(z1, row0 + li, B, kq, q1);
    float *Dv = ws, *pf = ws + B;
    __shared__ float sPart[4][CR][4];
    const int64_t jstep = static_cast<int64_t>(NS) * CT;
    TileRegs t1, t2;  // the next tile's rows, in flight during this tile
    if (static_cast<int64_t>(by) * CT < B) {
        tile_load(z1, B, static_cast<int64_t>(by) * CT, t1);
        tile_load(z2, B, static_cast<int64_t>(by) * CT, t2);
    }
    for (int64_t j0 = static_cast<int64_t>(by) * CT; j0 < B; j0 += jstep) {
        __syncthreads();
        tile_store(t1, sK1);
        tile_store(t2, sK2);
        if (j0 + jstep < B) {
            tile_load(z1, B, j0 + jstep, t1);
            tile_load(z2, B, j0 + jstep, t2);
        }
        __syncthreads();
        f32x4 s11 = {0.f, 0.f, 0.f, 0.f}, s12 = s11;
        const float *pk1 = sK1 + (16 * w + li) * CLD + 4 * kq, *pk2 = sK2 + (16 * w + li) * CLD + 4 * kq;
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const float4 b1 = *reinterpret_cast<const float4 *>(pk1 + 16 * mm);
            const float4 b2 = *reinterpret_cast<const float4 *>(pk2 + 16 * mm);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                s11 = __builtin_amdgcn_mfma_f32_16x16x4f32(q1[4 * mm + t], f4c(b1, t), s11, 0, 0, 0);
                s12 = __builtin_amdgcn_mfma_f32_16x16x4f32(q1[4 * mm + t], f4c(b2, t), s12, 0, 0, 0);
            }
        }
        // (R, Bt, e11_ii, e12_ii) of this tile for rows 4 kq + r: over the
        // wave's 16 columns (shuffles), then over the waves in order
        const int64_t j = j0 + 16 * w + li;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = row0 + 4 * kq + r;
            const float okj = j < B ? 1.f : 0.f, dg = j == i ? 1.f : 0.f;
            const float e11 = expf(s11[r]) * okj, e12 = expf(s12[r]) * okj;
            float v[4] = {e11, e12, e11 * dg, e12 * dg};
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int off = 8; off >= 1; off >>= 1) v[u] += __shfl_xor(v[u], off, kWave);
            if (li == 0) {
#pragma unroll
                for (int u = 0; u < 4; ++u) sPart[w][4 * kq + r][u] = v[u];
            }
        }
        __syncthreads();
        if (tid < CR) {
            const int64_t i = row0 + tid;
            float4 t4;
            t4.x = ((sPart[0][tid][0] + sPart[1][tid][0]) + sPart[2][tid][0]) + sPart[3][tid][0];
            t4.y = ((sPart[0][tid][1] + sPart[1][tid][1]) + sPart[2][tid][1]) + sPart[3][tid][1];
            t4.z = ((sPart[0][tid][2] + sPart[1][tid][2]) + sPart[2][tid][2]) + sPart[3][tid][2];
            t4.w = ((sPart[0][tid][3] + sPart[1][tid][3]) + sPart[2][tid][3]) + sPart[3][tid][3];
            if (i < B) st_agent4(pf + ((j0 / CT) * B + i) * 4, t4);
        }
    }
    // two-level combine: the last split of each row block finishes its 16
    // rows (the tile partials summed in tile order, D, the -log terms, their
    // fixed-order sum), then the last row block sums the row-block partials
    // in order.  Counters: a.counters[0] (row blocks) and a.counters[1 + bx]
    // (splits; the backward's counters, idle during the forward), each reset
    // by its last arriver.
    unsigned *counter = a.counters;
    const int64_t nrb = contrast_row_blocks(B), T = contrast_tiles(B);
    int64_t off = contrast_pb_offset(B);  // bwd partials, idle here
    off += off & 1;
    double *rbp = reinterpret_cast<double *>(ws + off);
    if (!block_arrive(counter + 1 + bx, static_cast<unsigned>(NS))) return;
    __shared__ double sRow[CR];
    if (tid < CR) {
        const int64_t k = bx * CR + tid;
        const int64_t kc = k < B ? k : B - 1;  // clamped: the loads stay unconditional
        float sm[4] = {0.f, 0.f, 0.f, 0.f};
        for (int64_t y0 = 0; y0 < T; y0 += 16) {
            float4 v[16];
#pragma unroll
            for (int y = 0; y < 16; ++y)
                v[y] = ld_agent4(pf + ((y0 + y < T ? y0 + y : 0) * B + kc) * 4);
#pragma unroll
            for (int y = 0; y < 16; ++y) {
                const float wy = y0 + y < T ? 1.f : 0.f;
                sm[0] = fmaf(v[y].x, wy, sm[0]);
                sm[1] = fmaf(v[y].y, wy, sm[1]);
                sm[2] = fmaf(v[y].z, wy, sm[2]);
                sm[3] = fmaf(v[y].w, wy, sm[3]);
            }
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

// backward body: sK1, sK2 >= CT * CLD floats, sWf >= 3 * CR * CLD, sDj unused.
//
// The similarity blocks and the weighted sums are matrix products, run on
// the f32 MFMA v_mfma_f32_16x16x4_f32 (wave w takes columns 16w.. of each
// 64-column tile for the similarities and channels 16w.. for the sums):
//   S11 = Q1 K1^T, S12 = Q1 K2^T, S21 = Q2 K1^T   (16 x 64 per tile, K = 64)
//   d1 += W11 K1 + W12 K2,  d2 += W21 K1          (16 x 64, K = the tile's 64 j)
// with the weights W formed on the S accumulators and passed through LDS.
// Each lane feeds four k values per ds_read_b128 (the k order of every sum
// permuted identically for both operands, kperm16).  The earlier form (one
// 64-long dependent VALU fma chain per dot product, one wave per SIMD inside
// the head MLP's launch) took ~25 us per workgroup at B = 512 (phase trace).
__device__ __forceinline__ void contrast_bwd_body(const ContrastArgs &a, int64_t bx, int by,
                                                  float *sK1, float *sK2, float *sWf,
                                                  float * /*sDj*/) {
    const float *__restrict__ z1 = a.z1, *__restrict__ z2 = a.z2;
    const int64_t B = a.B;
    const float *__restrict__ ws = a.ws;
    float *__restrict__ dz1 = a.dz1, *__restrict__ dz2 = a.dz2;
    unsigned *counters = a.counters;
    const int tid = threadIdx.x, w = tid >> 6, l = tid & 63, li = l & 15, kq = l >> 4;
    const int NS = a.nsplit;
    const int64_t row0 = bx * CR;
    const float g = *a.g_loss / static_cast<float>(B);
    const float *Dv = ws;
    float *pb = a.ws + contrast_pb_offset(B);
    float q1[16], q2[16];  // A operands: row row0 + li, k = kperm16(s, kq)
    load_row_k(z1, row0 + li, B, kq, q1);
    load_row_k(z2, row0 + li, B, kq, q2);
    float invDi[4];        // output rows 4 kq + r
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = row0 + 4 * kq + r;
        invDi[r] = i < B ? 1.f / Dv[i] : 0.f;
    }
    float *sW = sWf;  // [3][CR][CLD]: W11, W12, W21
    f32x4 d1 = {0.f, 0.f, 0.f, 0.f}, d2 = d1;  // rows 4 kq + r, channel 16 w + li
    const int64_t jstep = static_cast<int64_t>(NS) * CT;
    TileRegs t1, t2;  // the next tile's rows, in flight during this tile
    if (static_cast<int64_t>(by) * CT < B) {
        tile_load(z1, B, static_cast<int64_t>(by) * CT, t1);
        tile_load(z2, B, static_cast<int64_t>(by) * CT, t2);
    }
    for (int64_t j0 = static_cast<int64_t>(by) * CT; j0 < B; j0 += jstep) {
        const int64_t j = j0 + 16 * w + li;  // this lane's similarity column
        const float invDj = j < B ? 1.f / Dv[j] : 0.f;
        __syncthreads();
        tile_store(t1, sK1);
        tile_store(t2, sK2);
        if (j0 + jstep < B) {
            tile_load(z1, B, j0 + jstep, t1);
            tile_load(z2, B, j0 + jstep, t2);
        }
        __syncthreads();
        f32x4 s11 = {0.f, 0.f, 0.f, 0.f}, s12 = s11, s21 = s11;
        const float *pk1 = sK1 + (16 * w + li) * CLD + 4 * kq, *pk2 = sK2 + (16 * w + li) * CLD + 4 * kq;
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const float4 b1 = *reinterpret_cast<const float4 *>(pk1 + 16 * mm);
            const float4 b2 = *reinterpret_cast<const float4 *>(pk2 + 16 * mm);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int s = 4 * mm + t;
                s11 = __builtin_amdgcn_mfma_f32_16x16x4f32(q1[s], f4c(b1, t), s11, 0, 0, 0);
                s12 = __builtin_amdgcn_mfma_f32_16x16x4f32(q1[s], f4c(b2, t), s12, 0, 0, 0);
                s21 = __builtin_amdgcn_mfma_f32_16x16x4f32(q2[s], f4c(b1, t), s21, 0, 0, 0);
            }
        }
        // weights at (row 4 kq + r, column 16 w + li of the tile)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int64_t i = row0 + 4 * kq + r;
            const bool ok = i < B && j < B;
            const float delta = j == i ? 1.f : 0.f;
            const float e11 = expf(s11[r]), e12 = expf(s12[r]), e21 = expf(s21[r]);
            const int o = (4 * kq + r) * CLD + 16 * w + li;
            sW[o] = ok && j != i ? g * e11 * (invDi[r] + invDj) : 0.f;
            sW[CR * CLD + o] = ok ? g * (e12 * invDi[r] - delta) : 0.f;
            sW[2 * CR * CLD + o] = ok ? g * (e21 * invDj - delta) : 0.f;
        }
        __syncthreads();
        // d1 += W11 K1 + W12 K2, d2 += W21 K1 over the tile's 64 columns j
        const float *pw = sW + li * CLD + 4 * kq;
        const float *pc1 = sK1 + 16 * w + li, *pc2 = sK2 + 16 * w + li;
#pragma unroll
        for (int mm = 0; mm < 4; ++mm) {
            const float4 w11 = *reinterpret_cast<const float4 *>(pw + 16 * mm);
            const float4 w12 = *reinterpret_cast<const float4 *>(pw + CR * CLD + 16 * mm);
            const float4 w21 = *reinterpret_cast<const float4 *>(pw + 2 * CR * CLD + 16 * mm);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int jj = kperm16(4 * mm + t, kq);
                const float k1 = pc1[jj * CLD], k2 = pc2[jj * CLD];
                d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(w11, t), k1, d1, 0, 0, 0);
                d2 = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(w21, t), k1, d2, 0, 0, 0);
                d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(f4c(w12, t), k2, d1, 0, 0, 0);
            }
        }
    }
    // this split's partial rows -> [split][B][128] (d1 | d2)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int64_t i = row0 + 4 * kq + r;
        if (i < B) {
            float *p = pb + (static_cast<int64_t>(by) * B + i) * 128 + 16 * w + li;
            st_agent(p, d1[r]);
            st_agent(p + 64, d2[r]);
        }
    }
    if (!block_arrive(counters + bx, NS)) return;
    // last split of the row block: fixed-order sum over the splits, then the
    // normalisation backward; row r = tid >> 4, channels 4 cl .. 4 cl + 3
    const int r = tid >> 4, cl = tid & 15;
    const int64_t i = row0 + r;
    if (i < B) {
        float4 e1 = make_float4(0.f, 0.f, 0.f, 0.f), e2 = e1;
        float4 v1[kMaxSplit], v2[kMaxSplit];
#pragma unroll
        for (int y = 0; y < kMaxSplit; ++y) {  // all splits in flight (clamped), summed in order
            const float *p = pb + (static_cast<int64_t>(y < NS ? y : 0) * B + i) * 128 + 4 * cl;
            v1[y] = ld_agent4(p);
            v2[y] = ld_agent4(p + 64);
        }
#pragma unroll
        for (int y = 0; y < kMaxSplit; ++y) {
            const float wy = y < NS ? 1.f : 0.f;
            e1.x = fmaf(v1[y].x, wy, e1.x); e1.y = fmaf(v1[y].y, wy, e1.y);
            e1.z = fmaf(v1[y].z, wy, e1.z); e1.w = fmaf(v1[y].w, wy, e1.w);
            e2.x = fmaf(v2[y].x, wy, e2.x); e2.y = fmaf(v2[y].y, wy, e2.y);
            e2.z = fmaf(v2[y].z, wy, e2.z); e2.w = fmaf(v2[y].w, wy, e2.w);
        }
        // this lane's channels of the normalised rows and the row norms
        const float4 x1 = reinterpret_cast<const float4 *>(z1 + i * 64)[cl];
        const float4 x2 = reinterpret_cast<const float4 *>(z2 + i * 64)[cl];
        const float inv1 = 1.f / fmaxf(sqrtf(sum16(x1.x * x1.x + x1.y * x1.y + x1.z * x1.z + x1.w * x1.w)), kNormEps);
        const float inv2 = 1.f / fmaxf(sqrtf(sum16(x2.x * x2.x + x2.y * x2.y + x2.z * x2.z + x2.w * x2.w)), kNormEps);
        const float4 a1 = make_float4(x1.x * inv1, x1.y * inv1, x1.z * inv1, x1.w * inv1);
        const float4 a2 = make_float4(x2.x * inv2, x2.y * inv2, x2.z * inv2, x2.w * inv2);
        const float p1 = sum16(a1.x * e1.x + a1.y * e1.y + a1.z * e1.z + a1.w * e1.w);
        const float p2 = sum16(a2.x * e2.x + a2.y * e2.y + a2.z * e2.z + a2.w * e2.w);
        const float s1 = inv1 < 1.f / kNormEps ? p1 : 0.f;  // |z| <= eps: z / eps, no projection
        const float s2 = inv2 < 1.f / kNormEps ? p2 : 0.f;
        reinterpret_cast<float4 *>(dz1 + i * 64)[cl] =
            make_float4((e1.x - a1.x * s1) * inv1, (e1.y - a1.y * s1) * inv1,
                        (e1.z - a1.z * s1) * inv1, (e1.w - a1.w * s1) * inv1);
        reinterpret_cast<float4 *>(dz2 + i * 64)[cl] =
            make_float4((e2.x - a2.x * s2) * inv2, (e2.y - a2.y * s2) * inv2,
                        (e2.z - a2.z * s2) * inv2, (e2.w - a2.w * s2) * inv2);
    }
    if (tid == 0) counters[bx] = 0u;
}

}  // namespace scgib
