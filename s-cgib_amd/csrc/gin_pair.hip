// Persistent forward of the encoder pair (include/scgib.h, scgib_gin_pair_fwd):
// Encoder2 over the ego-nets and Encoder1 over the molecules (models.py:702-716,
// GIN-64 x L of models.py:52-72 with transfer_d folded into layer 0, the ego
// readout dgl.sum_nodes and compressor[0] on Encoder1's output) in ONE launch.
//
// Why: the per-layer kernels (gin_fwd_k) spend ~2/3 of each 18-20 us launch
// outside their GEMMs at QM9 B512 — kernel boundary, the weights and the
// deferred BatchNorm partials arriving at every workgroup's start, and the
// dependent CSR -> neighbour-row gather chain — once per layer.  Here:
//   * chunk c of an encoder = the components (molecules / ego-nets) whose
//     first row lies in rows [80c, 80c + 80): <= 112 rows when no component
//     exceeds 33 rows.  Every neighbour of a chunk row is a row of the same
//     chunk (components are closed), so ONE workgroup per chunk owns all the
//     rows it ever gathers: the chunk's local CSR is loaded once (and handed
//     to the backward as a chunk record), its rows stay in LDS from layer to
//     layer, and no row crosses a workgroup;
//   * per layer: aggregation from LDS (BN + ReLU of the previous layer applied
//     once per row in place, then every row's neighbour reads of one degree
//     step in flight together), z1 = agg W1^T, r = relu(z1 + b1),
//     z2 = r W2^T + b2 on the f32 MFMA v_mfma_f32_16x16x4_f32 (16-row
//     blocks), the wave's 16 weight columns held in VGPRs and the next
//     layer's fetched during the BatchNorm exchange, as are the z2 row stores;
//   * BatchNorm's batch statistics: each chunk's (n, mean, centred M2) ->
//     32-chunk groups combined by the group's last arriver (fp64, fixed
//     order) into tagged words ((launch epoch + 1) << 32 | float bits) ->
//     every chunk polls the groups' words and merges them itself (fp64, fixed
//     order, one division): no publisher, no flag, nothing to re-arm.  Chunk
//     0 writes the stat record and the running statistics.  All
//     cross-workgroup words are agent-scope atomics on both sides
//     (MI355X_MICROARCH.md, valid forms); every spin is bounded (timeout ->
//     sync[1], never a hang).
// The whole grid (both encoders' chunks) must be co-resident: the host
// launches it only when it fits scgib_gin_pair_slots() (2 workgroups per CU:
// 63 KB of LDS, <= 256 VGPRs) and falls back to the per-layer kernels
// otherwise.  Writes what the per-layer path saves for the backward (agg, r,
// z2, stat per layer, aggx).
//
// LDS images are [row][64] floats with the float4 slots XOR-swizzled by the
// row (slot q of row r at q ^ (r & 15)): the MFMA operand reads (16 rows x one
// float4 per lane, ds_read_b128) and the row-wise VALU accesses are both
// bank-conflict free without padding.
#include "mfma_tile.h"

namespace scgib {
namespace pair {

constexpr int kWin = 80;                 // chunk window (rows)
constexpr int kRows = 112;               // max rows per chunk
constexpr int kMaxComp = kRows - kWin + 1;  // max component rows (33)
constexpr int kNrb = kRows / 16;         // 16-row blocks
constexpr int kMaxE = 512;               // chunk edges cached in LDS (else read from global)
constexpr int kGrp = 32;                 // chunk partials per group
constexpr int kPart = 132;               // floats per chunk partial: mean[64] M2[64] n pad[3]
constexpr int kL = SCGIB_PAIR_MAX_LAYERS;
constexpr uint64_t kTimeout = 20000000;  // 0.2 s of the 100 MHz wall clock per spin

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int sidx(int row, int col) {
    return row * 64 + ((((col >> 2) ^ (row & 15)) << 2) | (col & 3));
}

__host__ __device__ inline int64_t n_chunks(int64_t n_cap) { return (n_cap + kWin - 1) / kWin; }
__host__ __device__ inline int64_t n_groups(int64_t n_cap) { return (n_chunks(n_cap) + kGrp - 1) / kGrp; }

constexpr int kMaxGroups = 16;           // groups per encoder (512 co-resident chunks)
constexpr int kGT = 130;                 // tagged words per group partial

// merge (nb rows, sum sb, centred M2 mb) into the running (n, mean, M2)
__device__ __forceinline__ void chan_merge(double &n, double &mean, double &m2, double nb, double sb,
                                           double mb) {
    if (nb <= 0.0) return;
    const double meanb = sb / nb, nn = n + nb, d = meanb - mean;
    mean += d * (nb / nn);
    m2 += mb + d * d * (n * nb / nn);
    n = nn;
}

// workspace (per encoder, any memory): the chunk partials [L][nch][kPart]
__host__ __device__ inline int64_t ws_bytes(int64_t n_cap, int L) {
    return static_cast<int64_t>(L) * n_chunks(n_cap) * kPart * 4 + 64;
}
__device__ inline float *ws_of(void *ws) {
    return reinterpret_cast<float *>((reinterpret_cast<uintptr_t>(ws) + 15) & ~uintptr_t(15));
}
// state (per encoder and call site, zeroed once, kept across launches; a
// fixed layout whatever the graph size): [0] launch epoch | group arrival
// counters [kL][kMaxGroups] | group partials [kL][kMaxGroups][kGT] as tagged
// words (epoch + 1) << 32 | float bits, 8-byte aligned.  A group partial
// carries its launch's tag in every word, so the chunks poll the data
// itself: no flag, nothing to re-arm, and a stale word never matches.
struct Cnt {
    unsigned *epoch, *grp;
    uint64_t *gt;
};
__host__ __device__ inline int64_t n_counters(int64_t, int) {
    return 2 + kL * kMaxGroups + 2 + 2 * kL * kMaxGroups * kGT;
}
__device__ inline Cnt cnt_of(unsigned *base) {
    Cnt k;
    k.epoch = base;
    k.grp = base + 2;
    k.gt = reinterpret_cast<uint64_t *>((reinterpret_cast<uintptr_t>(k.grp + kL * kMaxGroups) + 7) &
                                        ~uintptr_t(7));
    return k;
}

struct Smem {
    alignas(16) float buf0[kRows * 64];   // z2 of the previous layer / aggx / r / z2
    alignas(16) float buf1[kRows * 64];   // agg / the final output; scratch of the BN combines
    int32_t rp[kRows + 1];    // chunk-local row pointers (edge offsets from the chunk's first)
    int32_t colv[kMaxE];      // chunk-local neighbour rows
    int32_t cs[kRows + 2];    // chunk-local component starts (readout)
    float ss[128];            // (scale, shift) of the previous layer's BatchNorm
    int32_t sb[2][4];         // bound searches: lo, hi, first hit; sb[0][3]: max degree
    unsigned flag;            // block-wide broadcast of a ticket / last-arriver flag
    int32_t hdr[16];          // backward: the chunk record's header
    alignas(16) float red[4][128];  // backward: the waves' column sums; exchange scratch
};

__device__ __forceinline__ uint64_t now() { return wall_clock64(); }

// diagnostics: wall-clock stamp i of this workgroup (trace != NULL)
__device__ __forceinline__ void mark(uint64_t *tr, int i) {
    if (tr && threadIdx.x == 0) tr[i] = now();
}

__device__ __forceinline__ void set_err(uint32_t *sync, unsigned code) {
    __hip_atomic_store(sync + 1, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_tagged(uint64_t *p, unsigned tag, float v) {
    __hip_atomic_store(p, (static_cast<uint64_t>(tag) << 32) | __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}


// Count this workgroup in (every wave's stores drained first) and return the
// value the counter held before (block-uniform).
__device__ __forceinline__ unsigned arrive(unsigned *counter, Smem &sm) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        sm.flag = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return sm.flag;
}

// Two lower bounds at once: threads 0..127 find the first i in [0, C] with
// gp[i] >= t0, threads 128..255 with gp[i] >= t1 (gp non-decreasing; C when
// none), by 128-way sampling rounds.  Returns this half's index in sm.sb[h][0].
__device__ void lower_bounds(const int32_t *__restrict__ gp, int64_t C, int t0, int t1, Smem &sm) {
    const int h = threadIdx.x >> 7, j = threadIdx.x & 127;
    const int tgt = h ? t1 : t0;
    if (j == 0) {
        sm.sb[h][0] = 0;
        sm.sb[h][1] = static_cast<int>(C);
    }
    __syncthreads();
    for (int round = 0; round < 5; ++round) {
        const int lo = sm.sb[h][0], hi = sm.sb[h][1];
        const bool more = sm.sb[0][0] < sm.sb[0][1] || sm.sb[1][0] < sm.sb[1][1];
        __syncthreads();
        if (!more) break;  // block-uniform
        if (j == 0) sm.sb[h][2] = 128;
        __syncthreads();
        const int n = hi - lo, step = (n + 127) / 128;
        const int p = lo + j * step;
        if (lo < hi && p < hi && gp[p] >= tgt) atomicMin(&sm.sb[h][2], j);
        __syncthreads();
        if (j == 0 && lo < hi) {
            const int f = sm.sb[h][2];
            if (f < 128) {
                sm.sb[h][1] = lo + f * step;
                sm.sb[h][0] = f > 0 ? lo + (f - 1) * step + 1 : lo;
            } else {
                const int last = (n - 1) / step;  // the last sampled j
                sm.sb[h][0] = lo + last * step + 1;
            }
        }
        __syncthreads();
    }
}

// weight fragments of wave w (output columns 16 w + (lane & 15)) for the
// 16x16x4 MFMA with the k order permuted per ds_read_b128: step 4 j + t of
// lane group g = lane >> 4 covers k = 16 j + 4 g + t
template <int K>
__device__ __forceinline__ void load_frag(const float *__restrict__ W, float (&f)[16]) {
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const float *row = W + static_cast<int64_t>(16 * w + (l & 15)) * K + 4 * (l >> 4);
#pragma unroll
    for (int j = 0; j < K / 16; ++j) {
        const float4 v = *reinterpret_cast<const float4 *>(row + 16 * j);
        f[4 * j] = v.x; f[4 * j + 1] = v.y; f[4 * j + 2] = v.z; f[4 * j + 3] = v.w;
    }
}

// acc[rb] = A[16 rb .. 16 rb + 15][0..K) W^T (wave's 16 columns), rb < nrb
template <int K>
__device__ __forceinline__ void gemm(const float *A, const float (&f)[16], int nrb, f32x4 (&acc)[kNrb]) {
    const int l = threadIdx.x & 63, r16 = l & 15, g = l >> 4;
#pragma unroll
    for (int rb = 0; rb < kNrb; ++rb) {
        acc[rb] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (rb < nrb) {  // block-uniform
            const int row = 16 * rb + r16;
#pragma unroll
            for (int j = 0; j < K / 16; ++j) {
                const float4 a = *reinterpret_cast<const float4 *>(A + sidx(row, 16 * j + 4 * g));
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, f[4 * j], acc[rb], 0, 0, 0);
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, f[4 * j + 1], acc[rb], 0, 0, 0);
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, f[4 * j + 2], acc[rb], 0, 0, 0);
                acc[rb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, f[4 * j + 3], acc[rb], 0, 0, 0);
            }
        }
    }
}

// accumulator element i of row block rb: row 16 rb + 4 (lane >> 4) + i, column
// 16 w + (lane & 15)
__device__ __forceinline__ int acc_row16(int rb, int i) { return 16 * rb + 4 * ((threadIdx.x & 63) >> 4) + i; }
__device__ __forceinline__ int acc_col16() { return 16 * (threadIdx.x >> 6) + (threadIdx.x & 15); }

// copy rows [0, nr) of an LDS image (width cols) to global rows g0.. (float4 lanes)
template <int COLS>
__device__ __forceinline__ void lds_to_global(const float *S, float *__restrict__ dst, int64_t g0, int nr) {
    constexpr int Q = COLS / 4;
    for (int idx = threadIdx.x; idx < nr * Q; idx += 256) {
        const int v = idx / Q, q = idx % Q;
        st4(dst + (g0 + v) * COLS + 4 * q, *reinterpret_cast<const float4 *>(S + sidx(v, 4 * q)));
    }
}

// zero rows [r0, r1) x COLS of a global array
template <int COLS>
__device__ __forceinline__ void zero_rows(float *__restrict__ dst, int64_t r0, int64_t r1) {
    constexpr int Q = COLS / 4;
    for (int64_t idx = threadIdx.x; idx < (r1 - r0) * Q; idx += 256)
        st4(dst + (r0 + idx / Q) * COLS + 4 * (idx % Q), make_float4(0.f, 0.f, 0.f, 0.f));
}

struct Layer {  // this layer's per-encoder constants
    float ope, eps, mom;
    const float *gamma, *beta;
    float *rmean, *rvar, *stat;
    int64_t *nbt;
};

// wait until word w of every group partial of layer l carries this launch's
// tag (wave 0's lanes < ngr poll one word each), then a block barrier
__device__ void await_groups(const Cnt &cnt, int l, int64_t ngr, int w, unsigned tag, uint32_t *sync,
                             unsigned code) {
    const int tid = threadIdx.x;
    if (tid < 64) {
        const uint64_t *q = cnt.gt + (static_cast<int64_t>(l) * kMaxGroups + (tid < ngr ? tid : 0)) * kGT + w;
        const uint64_t t0 = now();
        while (true) {
            const uint64_t v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (__all(tid >= ngr || static_cast<unsigned>(v >> 32) == tag)) break;  // wave-uniform
            __builtin_amdgcn_s_sleep(1);
            if (now() - t0 > kTimeout) {
                set_err(sync, code);
                break;
            }
        }
    }
    __syncthreads();
}

// a tagged word's value once it carries tag (re-polled otherwise; bounded)
__device__ __forceinline__ float ld_tagged(const uint64_t *q, unsigned tag, uint32_t *sync, unsigned code) {
    uint64_t v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (static_cast<unsigned>(v >> 32) != tag) {  // (rare: the group's marker word landed first)
        const uint64_t t0 = now();
        do {
            __builtin_amdgcn_s_sleep(1);
            v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (now() - t0 > kTimeout) {
                set_err(sync, code);
                break;
            }
        } while (static_cast<unsigned>(v >> 32) != tag);
    }
    return __uint_as_float(static_cast<unsigned>(v));
}

// The BatchNorm exchange of layer l for chunk c (rows nr), two levels with no
// publisher: chunk partial (n, column means, centred M2; fp32) -> the 32-chunk
// group's last arriver combines them (fp64, fixed order) and stores the group
// partial (n, mean, centred M2) as tagged words -> EVERY chunk reads all
// group partials and merges them itself (fp64, fixed order, one division:
// every chunk gets the same bits), so the
// statistics cost one arrival and two tagged hand-offs.  Chunk 0 also writes
// the stat record and the running statistics.  (scale, shift) -> sm.ss.
template <class Mid>
__device__ void bn_exchange(const f32x4 (&z)[kNrb], int nrb, int nr, int64_t c, int64_t nch,
                            int64_t ngr, int l, float *ws, const Cnt &cnt, unsigned tag,
                            const Layer &Ly, uint32_t *sync, Smem &sm, uint64_t *tr, Mid mid) {
    const int tid = threadIdx.x, lane = tid & 63, g = lane >> 4;
    const int col = acc_col16();
    const int ch = tid & 63, p = tid >> 6;
    // (gamma, beta) in flight during the exchange
    const float gam = Ly.gamma[ch], bet = Ly.beta[ch];
    // ---- chunk partial: column sum and centred M2 over the valid rows (fp32)
    float s = 0.f;
#pragma unroll
    for (int rb = 0; rb < kNrb; ++rb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (rb < nrb && acc_row16(rb, i) < nr) s += z[rb][i];
    s += __shfl_xor(s, 16, kWave);
    s += __shfl_xor(s, 32, kWave);
    const float mean = nr > 0 ? s / static_cast<float>(nr) : 0.f;
    float q = 0.f;
#pragma unroll
    for (int rb = 0; rb < kNrb; ++rb)
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (rb < nrb && acc_row16(rb, i) < nr) {
                const float d = z[rb][i] - mean;
                q += d * d;
            }
    q += __shfl_xor(q, 16, kWave);
    q += __shfl_xor(q, 32, kWave);
    float *part = ws + (static_cast<int64_t>(l) * nch + c) * kPart;
    if (g == 0) {
        st_agent(part + col, mean);
        st_agent(part + 64 + col, q);
    }
    if (tid == 0) st_agent(part + 128, static_cast<float>(nr));
    // ---- group combine by the group's last arriving chunk -> tagged partial
    const int64_t grp = c / kGrp, g0 = grp * kGrp;
    const int gsize = static_cast<int>(nch - g0 < kGrp ? nch - g0 : kGrp);
    unsigned *gcnt = cnt.grp + l * kMaxGroups + grp;
    double *dscr = reinterpret_cast<double *>(sm.buf1);                 // 6 KB of scratch
    const bool last_in_group = arrive(gcnt, sm) == static_cast<unsigned>(gsize - 1);
    mark(tr, 4);
    if (last_in_group) {
        // partition p takes chunks g0 + p + 4 u (fixed order), channel ch:
        // (rows, mean, centred M2) of each
        constexpr int U = kGrp / 4;
        float M[U], Q[U], N[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int k = p + 4 * u;
            const float *pp = ws + (static_cast<int64_t>(l) * nch + g0 + (k < gsize ? k : 0)) * kPart;
            M[u] = ld_agent(pp + ch);
            Q[u] = ld_agent(pp + 64 + ch);
            N[u] = k < gsize ? ld_agent(pp + 128) : 0.f;
        }
        double ns = 0.0, ss = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            ns += N[u];
            ss += static_cast<double>(N[u]) * M[u];
        }
        dscr[p * 64 + ch] = ss;
        dscr[256 + p * 64 + ch] = ns;
        __syncthreads();
        const double Sg = ((dscr[ch] + dscr[64 + ch]) + dscr[128 + ch]) + dscr[192 + ch];
        const double Ng = ((dscr[256 + ch] + dscr[320 + ch]) + dscr[384 + ch]) + dscr[448 + ch];
        const double mg = Ng > 0.0 ? Sg / Ng : 0.0;
        double qq = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const double d = static_cast<double>(M[u]) - mg;
            qq += N[u] > 0.f ? static_cast<double>(Q[u]) + static_cast<double>(N[u]) * d * d : 0.0;
        }
        __syncthreads();
        dscr[p * 64 + ch] = qq;
        __syncthreads();
        uint64_t *gp = cnt.gt + (static_cast<int64_t>(l) * kMaxGroups + grp) * kGT;
        if (p == 0) {
            st_tagged(gp + ch, tag, static_cast<float>(mg));
            st_tagged(gp + 64 + ch, tag,
                      static_cast<float>(((dscr[ch] + dscr[64 + ch]) + dscr[128 + ch]) + dscr[192 + ch]));
            if (ch == 0) st_tagged(gp + 128, tag, static_cast<float>(Ng));
        }
        if (tid == 0) __hip_atomic_store(gcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mark(tr, 5);
    }
    mid();  // work that needs no statistics (the z2 row stores) while the groups finish
    // ---- every chunk: all group partials (row counts first), merged in order
    await_groups(cnt, l, ngr, 128, tag, sync, 0x100u + l);
    mark(tr, 6);
    constexpr int U = kMaxGroups / 4;
    float gN[U], gm[U], gq[U];  // this thread's groups p + 4 u: rows, mean, centred M2
    {
        uint64_t w[3][U];  // every load in flight at once, tags checked after
        const uint64_t *base = cnt.gt + static_cast<int64_t>(l) * kMaxGroups * kGT;
        auto addr = [&](int u, int k) {
            const int64_t g1 = p + 4 * u;
            return base + (g1 < ngr ? g1 : 0) * kGT + (k == 0 ? 128 : k == 1 ? ch : 64 + ch);
        };
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < 3; ++k) w[k][u] = __hip_atomic_load(addr(u, k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool ok = true;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int k = 0; k < 3; ++k) ok = ok && (p + 4 * u >= ngr || static_cast<unsigned>(w[k][u] >> 32) == tag);
        if (!ok)  // (rare: a group's marker word landed before its other words)
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (p + 4 * u < ngr)
#pragma unroll
                    for (int k = 0; k < 3; ++k)
                        w[k][u] = static_cast<uint64_t>(__float_as_uint(ld_tagged(addr(u, k), tag, sync, 0x100u + l)));
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const bool in = p + 4 * u < ngr;
            gN[u] = in ? __uint_as_float(static_cast<unsigned>(w[0][u])) : 0.f;
            gm[u] = in ? __uint_as_float(static_cast<unsigned>(w[1][u])) : 0.f;
            gq[u] = in ? __uint_as_float(static_cast<unsigned>(w[2][u])) : 0.f;
        }
    }
    // N and the mean: partition sums in order, then the 4 partitions in order
    double pn = 0.0, ps = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        pn += gN[u];
        ps += static_cast<double>(gN[u]) * gm[u];
    }
    dscr[p * 64 + ch] = pn;
    dscr[256 + p * 64 + ch] = ps;
    __syncthreads();
    const double N = ((dscr[ch] + dscr[64 + ch]) + dscr[128 + ch]) + dscr[192 + ch];
    const double m = N > 0.0 ? (((dscr[256 + ch] + dscr[320 + ch]) + dscr[384 + ch]) + dscr[448 + ch]) / N : 0.0;
    // the centred M2 about the batch mean: sum of M2_g + N_g (mean_g - mean)^2
    double pq = 0.0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const double d = static_cast<double>(gm[u]) - m;
        pq += static_cast<double>(gq[u]) + static_cast<double>(gN[u]) * d * d;
    }
    dscr[512 + p * 64 + ch] = pq;
    __syncthreads();
    if (p == 0) {
        const double M2 = ((dscr[512 + ch] + dscr[576 + ch]) + dscr[640 + ch]) + dscr[704 + ch];
        const double var = N > 0.0 ? M2 / N : 0.0;
        const double istd = 1.0 / sqrt(var + static_cast<double>(Ly.eps));
        const double sc = static_cast<double>(gam) * istd;
        const float scale = static_cast<float>(sc);
        const float shift = static_cast<float>(static_cast<double>(bet) - m * sc);
        sm.ss[ch] = scale;
        sm.ss[64 + ch] = shift;
        if (c == 0) {  // one chunk per encoder: the layer's record and running statistics
            if (Ly.rmean) {
                const double mo = static_cast<double>(Ly.mom);
                Ly.rmean[ch] = static_cast<float>((1.0 - mo) * Ly.rmean[ch] + mo * m);
                Ly.rvar[ch] = static_cast<float>((1.0 - mo) * Ly.rvar[ch] +
                                                 mo * (N > 1.0 ? M2 / (N - 1.0) : M2));
                if (ch == 0 && Ly.nbt) *Ly.nbt += 1;
            }
            Ly.stat[ch] = static_cast<float>(m);
            Ly.stat[64 + ch] = static_cast<float>(istd);
            Ly.stat[128 + ch] = scale;
            Ly.stat[192 + ch] = shift;
        }
    }
    __syncthreads();
    mark(tr, 7);
}

// This workgroup's chunk c of a graph: components [i0, i1), rows [rb0, rb1),
// its CSR as chunk-local rows in LDS (sm.rp, sm.colv), the component starts
// (sm.cs, ncomp entries + the end).  With node_map/par, par[v] = the x row of
// chunk row v (layer 0 of the forward).
struct Chunk {
    int64_t i0, i1;
    int rb0, rb1, nr, nrb, ncomp, e0;
    int maxdeg;  // the largest row degree of the chunk
    bool lds_col;
};

// valid components: comp_dims[0] (capacity mode), clamped to the capacity
__device__ __forceinline__ int64_t comp_count(const int32_t *comp_dims, int64_t n_comp) {
    if (!comp_dims) return n_comp;
    const int64_t k = comp_dims[0];
    return k < 0 ? 0 : (k < n_comp ? k : n_comp);
}

__device__ Chunk load_chunk(const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col,
                            const int32_t *__restrict__ comp_ptr, int64_t n_comp, int64_t nch,
                            int64_t c, uint32_t *sync, Smem &sm,
                            const int32_t *__restrict__ node_map = nullptr, int32_t *par = nullptr) {
    const int tid = threadIdx.x;
    Chunk k;
    const int win0 = static_cast<int>(c * kWin), win1 = static_cast<int>(c * kWin + kWin);
    lower_bounds(comp_ptr, n_comp, win0, win1, sm);
    k.i0 = sm.sb[0][0];
    k.i1 = c == nch - 1 ? n_comp : sm.sb[1][0];
    __syncthreads();
    k.rb0 = static_cast<int>(comp_ptr[k.i0]);
    k.rb1 = static_cast<int>(comp_ptr[k.i1]);
    if (k.rb1 - k.rb0 > kRows || k.rb1 < k.rb0) {  // a component over kMaxComp rows: host-checked
        if (tid == 0) set_err(sync, 0x10u);
        k.rb1 = k.rb0;
    }
    k.nr = k.rb1 - k.rb0;
    k.nrb = (k.nr + 15) / 16;
    k.ncomp = static_cast<int>(k.i1 - k.i0 < kRows + 1 ? k.i1 - k.i0 : kRows + 1);
    if (tid <= k.nr) sm.rp[tid] = rowptr[k.rb0 + tid];
    if (par && tid < k.nr) par[tid] = node_map ? node_map[k.rb0 + tid] : k.rb0 + tid;
    if (tid <= k.ncomp) sm.cs[tid] = (tid < k.ncomp ? comp_ptr[k.i0 + tid] : k.rb1) - k.rb0;
    __syncthreads();
    k.e0 = sm.rp[0];
    const int ne = sm.rp[k.nr] - k.e0;
    k.lds_col = ne <= kMaxE;  // block-uniform
    if (k.lds_col)
        for (int i = tid; i < ne; i += 256) sm.colv[i] = col[k.e0 + i] - k.rb0;
    __syncthreads();
    if (tid <= k.nr) sm.rp[tid] -= k.e0;
    if (tid == 0) sm.sb[0][3] = 0;
    __syncthreads();
    if (tid < k.nr) atomicMax(&sm.sb[0][3], sm.rp[tid + 1] - sm.rp[tid]);
    __syncthreads();
    k.maxdeg = sm.sb[0][3];
    return k;
}

// The chunk's description as the forward derived it (header, local row
// pointers, component starts, local columns), saved for the backward so that
// it loads one record instead of repeating the searches and the CSR reads.
constexpr int kRecHdr = 16, kRecRp = kRecHdr, kRecCs = kRecRp + kRows + 1, kRecCol = kRecCs + kRows + 2;
constexpr int kRec = 768;  // ints per chunk record (3 x 256)
static_assert(kRecCol + kMaxE <= kRec, "chunk record");

__device__ void save_chunk(const Chunk &k, const Smem &sm, int32_t *__restrict__ rec) {
    const int tid = threadIdx.x;
    if (tid == 0) {
        rec[0] = static_cast<int32_t>(k.i0);
        rec[1] = static_cast<int32_t>(k.i1);
        rec[2] = k.rb0;
        rec[3] = k.rb1;
        rec[4] = k.nr;
        rec[5] = k.ncomp;
        rec[6] = k.e0;
        rec[7] = k.maxdeg;
        rec[8] = k.lds_col ? 1 : 0;
    }
    if (tid <= k.nr) rec[kRecRp + tid] = sm.rp[tid];
    if (tid <= k.ncomp) rec[kRecCs + tid] = sm.cs[tid];
    if (k.lds_col)
        for (int i = tid; i < sm.rp[k.nr]; i += 256) rec[kRecCol + i] = sm.colv[i];
}

__device__ Chunk load_chunk_rec(const int32_t *__restrict__ rec, Smem &sm) {
    const int tid = threadIdx.x;
    int32_t v[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) v[t] = rec[tid + 256 * t];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
        const int i = tid + 256 * t;
        if (i < kRecHdr) sm.hdr[i] = v[t];
        else if (i < kRecCs) sm.rp[i - kRecRp] = v[t];
        else if (i < kRecCol) sm.cs[i - kRecCs] = v[t];
        else if (i - kRecCol < kMaxE) sm.colv[i - kRecCol] = v[t];
    }
    __syncthreads();
    Chunk k;
    k.i0 = sm.hdr[0];
    k.i1 = sm.hdr[1];
    k.rb0 = sm.hdr[2];
    k.rb1 = sm.hdr[3];
    k.nr = sm.hdr[4];
    k.nrb = (k.nr + 15) / 16;
    k.ncomp = sm.hdr[5];
    k.e0 = sm.hdr[6];
    k.maxdeg = sm.hdr[7];
    k.lds_col = sm.hdr[8] != 0;
    return k;
}

// chunk-local neighbour row of chunk edge ei (clamped into the chunk: a graph
// whose edges left their component would read wrong rows, never outside the
// images)
__device__ __forceinline__ int nbr_of(const Chunk &k, const int32_t *__restrict__ col, const Smem &sm,
                                      int ei) {
    const int u = k.lds_col ? sm.colv[ei] : col[k.e0 + ei] - k.rb0;
    return u < 0 ? 0 : (u < k.nr ? u : k.nr - 1);
}

// out[v] = ope f(S[v]) + sum over v's neighbours u of f(S[u]) for the rows
// v = rs + 16 k (k < kNrb) of this thread's float4 slot q (f: per-column
// transform, e.g. the previous BatchNorm + ReLU); rows >= nr give zeros.  All
// rows' neighbour reads of one degree step go out together (the chunk's max
// degree bounds the steps; a missing neighbour enters as fmaf(x, 0, acc), so
// the sum equals the CSR-order sum bit for bit).  epi(k, v, value).
template <class Fn, class Epi>
__device__ __forceinline__ void aggregate_rows(const Chunk &ck, const int32_t *__restrict__ col,
                                               const Smem &sm, const float *S, float ope, int q,
                                               int rs, Fn f, Epi epi) {
    float4 acc[kNrb];
    int e0[kNrb], dg[kNrb];
#pragma unroll
    for (int k = 0; k < kNrb; ++k) {
        const int v = rs + 16 * k, vv = v < ck.nr ? v : 0;
        e0[k] = sm.rp[vv];
        dg[k] = v < ck.nr ? sm.rp[vv + 1] - e0[k] : 0;
        const float4 x = f(*reinterpret_cast<const float4 *>(S + sidx(vv, 4 * q)));
        acc[k] = make_float4(ope * x.x, ope * x.y, ope * x.z, ope * x.w);
    }
    const int elast = sm.rp[ck.nr] - 1;  // (>= 0 whenever maxdeg > 0)
    int md = 0;  // this lane's steps: the largest degree of its rows
#pragma unroll
    for (int k = 0; k < kNrb; ++k) md = dg[k] > md ? dg[k] : md;
    for (int j = 0; j < md; ++j) {
        int u[kNrb];
#pragma unroll
        for (int k = 0; k < kNrb; ++k) u[k] = nbr_of(ck, col, sm, j < dg[k] ? e0[k] + j : elast);
#pragma unroll
        for (int k = 0; k < kNrb; ++k) {
            const float w = j < dg[k] ? 1.f : 0.f;
            const float4 x = f(*reinterpret_cast<const float4 *>(S + sidx(u[k], 4 * q)));
            acc[k] = make_float4(fmaf(x.x, w, acc[k].x), fmaf(x.y, w, acc[k].y), fmaf(x.z, w, acc[k].z),
                                 fmaf(x.w, w, acc[k].w));
        }
    }
#pragma unroll
    for (int k = 0; k < kNrb; ++k) {
        const int v = rs + 16 * k;
        epi(k, v, v < ck.nr ? acc[k] : make_float4(0.f, 0.f, 0.f, 0.f));
    }
}

__global__ __launch_bounds__(256, 2) void gin_pair_fwd_k(const scgib_pair_fwd_args A) {
    __shared__ Smem sm;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63;
    const int64_t nch0 = n_chunks(A.enc[0].n_cap);
    const int e = static_cast<int64_t>(blockIdx.x) < nch0 ? 0 : 1;
    const scgib_pair_encoder &E = A.enc[e];
    const int64_t c = blockIdx.x - (e ? nch0 : 0);
    const int64_t nch = n_chunks(E.n_cap), ngr = n_groups(E.n_cap);
    const int L = A.n_layers;
    float *ws = ws_of(E.ws);
    const Cnt cnt = cnt_of(E.counters);
    const unsigned tag = __hip_atomic_load(cnt.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const int64_t n = E.dims ? static_cast<int64_t>(E.dims[0]) : E.n_cap;
    const int F = A.n_feat;
    uint64_t *tr = A.trace ? A.trace + static_cast<int64_t>(blockIdx.x) * 64 : nullptr;
    mark(tr, 56);

    // ---- weights of layer 0 (in flight during the chunk search)
    float fw1[16], fw2[16], fwt[4];
    load_frag<32>(E.w1[0], fw1);
    load_frag<64>(E.w2[0], fw2);
    {
        const int cb = wv & 1, g = lane >> 4;
        const float *wr = A.wt + static_cast<int64_t>(16 * cb + (lane & 15)) * F;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int k = 4 * g + t;
            fwt[t] = wr[k < F ? k : 0] * (k < F ? 1.f : 0.f);
        }
    }
    float bias1 = E.b1[0][acc_col16()], bias2 = E.b2[0][acc_col16()];

    // ---- this chunk: components [i0, i1), rows [rb0, rb1)
    int32_t *par = reinterpret_cast<int32_t *>(sm.buf1);  // layer 0 only
    const int64_t nce = comp_count(E.comp_dims, E.n_comp);
    const Chunk ck = load_chunk(E.rowptr, E.col, E.comp_ptr, nce, nch, c, A.sync, sm,
                                E.node_map, par);
    const int64_t i0 = ck.i0, i1 = ck.i1;
    const int rb0 = ck.rb0, nr = ck.nr, nrb = ck.nrb, ncomp = ck.ncomp;
    const int win0 = static_cast<int>(c * kWin), win1 = static_cast<int>(c * kWin + kWin);
    auto nbr = [&](int ei) -> int { return nbr_of(ck, E.col, sm, ei); };
    if (E.chunk_rec) save_chunk(ck, sm, E.chunk_rec + c * kRec);
    mark(tr, 57);
    if (tr && tid == 0)
        tr[61] = static_cast<uint64_t>(nr) | (static_cast<uint64_t>(sm.rp[nr]) << 8) |
                 (static_cast<uint64_t>(ck.lds_col) << 30) | (static_cast<uint64_t>(e) << 31);

    // capacity padding rows this window zeroes (every output, every layer)
    const int64_t z0 = win0 > n ? win0 : n, z1 = win1 < E.n_cap ? win1 : E.n_cap;

    // ---- layer 0: gather the raw features (ope x_v + sum of neighbours)
    const float ope0 = E.one_plus_eps[0];
    {
        // the chunk rows' raw features -> X [kRows][16] in LDS (one round of
        // loads), then the aggregation from LDS as in the later layers
        const int f = tid & 15, rs = tid >> 4;
        float *X = sm.buf1 + 128;  // (after par)
        if (nr > 0) {  // block-uniform
            float xv[kNrb];
#pragma unroll
            for (int k = 0; k < kNrb; ++k) {
                const int v = rs + 16 * k;
                xv[k] = A.x[static_cast<int64_t>(par[v < nr ? v : 0]) * F + (f < F ? f : 0)];
            }
#pragma unroll
            for (int k = 0; k < kNrb; ++k) {
                const int v = rs + 16 * k;
                if (v < nr) X[v * 16 + f] = f < F ? xv[k] : 0.f;
            }
        }
        __syncthreads();
        float acc[kNrb];
        int e0[kNrb], dg[kNrb], md = 0;
#pragma unroll
        for (int k = 0; k < kNrb; ++k) {
            const int v = rs + 16 * k, vv = v < nr ? v : 0;
            e0[k] = sm.rp[vv];
            dg[k] = v < nr ? sm.rp[vv + 1] - e0[k] : 0;
            md = dg[k] > md ? dg[k] : md;
            acc[k] = ope0 * X[vv * 16 + f];
        }
        const int elast = sm.rp[nr] - 1;
        for (int j = 0; j < md; ++j) {
            int u[kNrb];
#pragma unroll
            for (int k = 0; k < kNrb; ++k) u[k] = nbr(j < dg[k] ? e0[k] + j : elast);
#pragma unroll
            for (int k = 0; k < kNrb; ++k) acc[k] = fmaf(X[u[k] * 16 + f], j < dg[k] ? 1.f : 0.f, acc[k]);
        }
#pragma unroll
        for (int k = 0; k < kNrb; ++k) {
            const int v = rs + 16 * k;
            const float a = v < nr ? acc[k] : 0.f;
            if (v < nr) E.aggx[static_cast<int64_t>(rb0 + v) * 16 + f] = a;
            if (v < 16 * nrb) sm.buf0[sidx(v, f)] = a;
        }
        for (int64_t idx = tid; idx < (z1 - z0) * 16; idx += 256) E.aggx[z0 * 16 + idx] = 0.f;
    }
    __syncthreads();
    // agg0 = aggx Wt^T (32 columns): wave w takes column block w & 1, row blocks w >> 1 + 2 k
    {
        const int cb = wv & 1, r16 = lane & 15, g = lane >> 4;
        for (int rb = wv >> 1; rb < nrb; rb += 2) {
            const float4 a = *reinterpret_cast<const float4 *>(sm.buf0 + sidx(16 * rb + r16, 4 * g));
            f32x4 acc{0.f, 0.f, 0.f, 0.f};
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, fwt[0], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, fwt[1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, fwt[2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, fwt[3], acc, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = 16 * rb + 4 * g + i, cc = 16 * cb + r16;
                sm.buf1[sidx(row, cc)] = acc[i];
                if (row < nr) E.agg[0][static_cast<int64_t>(rb0 + row) * 32 + cc] = acc[i];
            }
        }
        zero_rows<32>(E.agg[0], z0, z1);
    }
    __syncthreads();
    mark(tr, 58);

    f32x4 z[kNrb];
    for (int l = 0; l < L; ++l) {
        const int din = l == 0 ? 32 : 64;
        uint64_t *tl = tr ? tr + 8 * l : nullptr;
        mark(tl, 0);
        if (l > 0) {
            // ---- aggregation from LDS: x = relu(scale z2 + shift) of the previous layer
            const int q = tid & 15, rs = tid >> 4;
            const float ope = E.one_plus_eps[l];
            const float4 sc = make_float4(sm.ss[4 * q], sm.ss[4 * q + 1], sm.ss[4 * q + 2], sm.ss[4 * q + 3]);
            const float4 sh = make_float4(sm.ss[64 + 4 * q], sm.ss[65 + 4 * q], sm.ss[66 + 4 * q],
                                          sm.ss[67 + 4 * q]);
            // x = relu(scale z2 + shift) in place, once per row
            for (int v = rs; v < nr; v += 16) {
                float4 *px = reinterpret_cast<float4 *>(sm.buf0 + sidx(v, 4 * q));
                *px = xform4(*px, sc, sh);
            }
            __syncthreads();
            aggregate_rows(ck, E.col, sm, sm.buf0, ope, q, rs, [](float4 x) { return x; },
                           [&](int, int v, float4 a) {
                               if (v < nr) st4(E.agg[l] + static_cast<int64_t>(rb0 + v) * 64 + 4 * q, a);
                               if (v < 16 * nrb) *reinterpret_cast<float4 *>(sm.buf1 + sidx(v, 4 * q)) = a;
                           });
            zero_rows<64>(E.agg[l], z0, z1);
            __syncthreads();
        }
        mark(tl, 1);
        // ---- z1 = agg W1^T; r = relu(z1 + b1) -> buf0 (its previous content is consumed)
        if (din == 32) gemm<32>(sm.buf1, fw1, nrb, z);
        else gemm<64>(sm.buf1, fw1, nrb, z);
#pragma unroll
        for (int rb = 0; rb < kNrb; ++rb)
            if (rb < nrb)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    sm.buf0[sidx(acc_row16(rb, i), acc_col16())] = fmaxf(z[rb][i] + bias1, 0.f);
        __syncthreads();
        lds_to_global<64>(sm.buf0, E.r[l], rb0, nr);
        zero_rows<64>(E.r[l], z0, z1);
        mark(tl, 2);
        // ---- z2 = r W2^T + b2
        gemm<64>(sm.buf0, fw2, nrb, z);
#pragma unroll
        for (int rb = 0; rb < kNrb; ++rb)
#pragma unroll
            for (int i = 0; i < 4; ++i) z[rb][i] += bias2;
        __syncthreads();  // every wave's reads of r done
#pragma unroll
        for (int rb = 0; rb < kNrb; ++rb)
            if (rb < nrb)
#pragma unroll
                for (int i = 0; i < 4; ++i) sm.buf0[sidx(acc_row16(rb, i), acc_col16())] = z[rb][i];
        __syncthreads();
        const Layer Ly{0.f, E.bn_eps[l], E.momentum[l], E.gamma[l], E.beta[l], E.running_mean[l],
                       E.running_var[l], E.stat[l], E.num_batches_tracked[l]};
        mark(tl, 3);
        // the chunk's statistics go out first; the z2 rows and the next
        // layer's weights during the exchange
        bn_exchange(z, nrb, nr, c, nch, ngr, l, ws, cnt, tag, Ly, A.sync, sm, tl, [&]() {
            lds_to_global<64>(sm.buf0, E.z2[l], rb0, nr);
            zero_rows<64>(E.z2[l], z0, z1);
            if (l + 1 < L) {
                load_frag<64>(E.w1[l + 1], fw1);
                load_frag<64>(E.w2[l + 1], fw2);
                bias1 = E.b1[l + 1][acc_col16()];
                bias2 = E.b2[l + 1][acc_col16()];
            }
        });
    }

    // ---- encoder output: out = relu(BN(z2)) -> global and buf1
    {
        const int q = tid & 15, rs = tid >> 4;
        const float4 sc = make_float4(sm.ss[4 * q], sm.ss[4 * q + 1], sm.ss[4 * q + 2], sm.ss[4 * q + 3]);
        const float4 sh = make_float4(sm.ss[64 + 4 * q], sm.ss[65 + 4 * q], sm.ss[66 + 4 * q],
                                      sm.ss[67 + 4 * q]);
        for (int v = rs; v < 16 * nrb; v += 16) {
            float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
            if (v < nr) {
                o = xform4(*reinterpret_cast<const float4 *>(sm.buf0 + sidx(v, 4 * q)), sc, sh);
                st4(E.out + static_cast<int64_t>(rb0 + v) * 64 + 4 * q, o);
            }
            *reinterpret_cast<float4 *>(sm.buf1 + sidx(v, 4 * q)) = o;
        }
        zero_rows<64>(E.out, z0, z1);
    }
    __syncthreads();
    if (E.readout) {
        // per-component sums (dgl.sum_nodes): task = (component k, float4 slot q)
        for (int t = tid; t < ncomp * 16; t += 256) {
            const int k = t >> 4, q = t & 15;
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int v = sm.cs[k]; v < sm.cs[k + 1]; ++v)
                a = add4(a, *reinterpret_cast<const float4 *>(sm.buf1 + sidx(v, 4 * q)));
            st4(E.readout + (i0 + k) * 64 + 4 * q, a);
            if (q == 0)
                for (int v = sm.cs[k]; v < sm.cs[k + 1]; ++v) E.seg[rb0 + v] = static_cast<int32_t>(i0 + k);
        }
        // (the last chunk only) trailing empty components past the LDS table
        for (int64_t k = i0 + ncomp + (tid >> 4); k < i1; k += 16)
            st4(E.readout + k * 64 + 4 * (tid & 15), make_float4(0.f, 0.f, 0.f, 0.f));
        for (int64_t v = z0 + tid; v < z1; v += 256) E.seg[v] = 0;
        // capacity mode: the components past the actual count, round robin
        if (tid < 16)
            for (int64_t k = nce + c; k < E.n_comp; k += nch)
                st4(E.readout + k * 64 + 4 * tid, make_float4(0.f, 0.f, 0.f, 0.f));
    }
    if (E.lin_w) {  // compressor[0] (models.py:596) on the output
        float fw0[16];
        load_frag<64>(E.lin_w, fw0);
        const float b0 = E.lin_b[acc_col16()];
        gemm<64>(sm.buf1, fw0, nrb, z);
#pragma unroll
        for (int rb = 0; rb < kNrb; ++rb)
            if (rb < nrb)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int row = acc_row16(rb, i);
                    if (row < nr) E.lin_out[static_cast<int64_t>(rb0 + row) * 64 + acc_col16()] = z[rb][i] + b0;
                }
        zero_rows<64>(E.lin_out, z0, z1);
    }

    // ---- exit: the last workgroup advances both encoders' epochs (the next
    // launch's tag)
    mark(tr, 60);
    if (arrive(A.sync, sm) == gridDim.x - 1) {
        for (int ee = 0; ee < 2; ++ee) {
            const Cnt k = cnt_of(A.enc[ee].counters);
            if (tid == 64) {
                const unsigned ep = __hip_atomic_load(k.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(k.epoch, ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (tid == 0) __hip_atomic_store(A.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------
// backward (scgib_gin_pair_bwd)
// ---------------------------------------------------------------------------
// Row loads of the saved activations through a buffer resource: 32-bit
// offsets (one VGPR per load instead of a 64-bit address each) and the
// hardware range check returns zeros past the array's rows, so the loads of
// a chunk's padding rows need no clamp.
typedef __amdgpu_buffer_rsrc_t Rsrc;
__device__ __forceinline__ Rsrc rows_rsrc(const float *base, int64_t rows, int width) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(base), 0,
                                             static_cast<int>(rows * width * 4), 0x00020000);
}
// v, or zeros (per component: a select of whole float4 values is lowered
// through scratch memory by hipcc)
__device__ __forceinline__ float4 keep4(bool ok, float4 v) {
    return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}
__device__ __forceinline__ float4 ld_row(Rsrc r, int row, int width, int col) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, (row * width + col) * 4, 0, 0));
}
// acc[jb] += X^T Y over rows [0, 4 ns): output rows = this wave's 16 columns
// of X (16 w + lane & 15), output columns = Y's columns 16 jb + (lane & 15);
// csum += the lane's X values (summed over lane >> 4: X's column sums)
template <int JB>
__device__ __forceinline__ void gemm_tn(const float *X, const float *Y, int ns, f32x4 (&acc)[4],
                                        float &csum) {
    const int l = threadIdx.x & 63, r16 = l & 15, g = l >> 4, w = threadIdx.x >> 6;
    auto step = [&](int s0, int cnt) {  // cnt (1 or 2) row steps, their LDS reads issued together
        float a[2], b[2][JB];
#pragma unroll
        for (int u = 0; u < 2; ++u)
            if (u < cnt) {
                const int row = 4 * (s0 + u) + g;
                a[u] = X[sidx(row, 16 * w + r16)];
#pragma unroll
                for (int jb = 0; jb < JB; ++jb) b[u][jb] = Y[sidx(row, 16 * jb + r16)];
            }
#pragma unroll
        for (int u = 0; u < 2; ++u)
            if (u < cnt) {
                csum += a[u];
#pragma unroll
                for (int jb = 0; jb < JB; ++jb)
                    acc[jb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u][jb], acc[jb], 0, 0, 0);
            }
    };
    int s = 0;
    for (; s + 1 < ns; s += 2) step(s, 2);
    if (s < ns) step(s, 1);
}

// B fragments of the product X W (W [K][N] row-major): column colbase + (lane
// & 15), rows k = 16 j + 4 (lane >> 4) + t -> f[4 j + t] (gemm's convention)
template <int K, int N>
__device__ __forceinline__ void load_frag_col(const float *__restrict__ W, int colbase, float (&f)[16]) {
    const int l = threadIdx.x & 63, c = l & 15, g = l >> 4;
#pragma unroll
    for (int j = 0; j < K / 16; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) f[4 * j + t] = W[(16 * j + 4 * g + t) * N + colbase + c];
}

// for rb = rb0, rb0 + step, ... < nrb: epi(rb, A rows [16 rb, 16 rb + 16) x f)
// (K = 64, b128 reads; one row block's accumulator live at a time)
template <class Epi>
__device__ __forceinline__ void gemm_each(const float *A, const float (&f)[16], int nrb, int rb0,
                                          int step, Epi epi) {
    const int l = threadIdx.x & 63, r16 = l & 15, g = l >> 4;
    for (int rb = rb0; rb < nrb; rb += step) {
        const int row = 16 * rb + r16;
        f32x4 acc{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float4 a = *reinterpret_cast<const float4 *>(A + sidx(row, 16 * j + 4 * g));
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.x, f[4 * j], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.y, f[4 * j + 1], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.z, f[4 * j + 2], acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a.w, f[4 * j + 3], acc, 0, 0, 0);
        }
        epi(rb, acc);
    }
}

// the BatchNorm-backward exchange of layer l, as the forward's: the chunk's
// 128 sums (sum dy, sum dy xhat, already stored at its partial) -> the
// group's last arriver (fp64, fixed order) -> tagged group sums -> every
// chunk adds all groups in order (fp64) and keeps the dz2 coefficients
// tot / N in sm.ss; chunk 0 writes dbeta / dgamma.
__device__ void bwd_exchange(int l, int64_t c, int64_t nch, int64_t ngr, int64_t n, float *ws,
                             const Cnt &cnt, unsigned tag, float *dgamma, float *dbeta, uint32_t *sync, Smem &sm,
                             double *dscr, uint64_t *tr) {
    const int tid = threadIdx.x, ch = tid & 127, p = tid >> 7;  // 128 sums x 2 partitions
    const int64_t grp = c / kGrp, g0 = grp * kGrp;
    const int gsize = static_cast<int>(nch - g0 < kGrp ? nch - g0 : kGrp);
    unsigned *gcnt = cnt.grp + l * kMaxGroups + grp;
    const bool last_in_group = arrive(gcnt, sm) == static_cast<unsigned>(gsize - 1);
    mark(tr, 2);
    if (last_in_group) {
        float v[kGrp / 2];
#pragma unroll
        for (int u = 0; u < kGrp / 2; ++u) {
            const int k = p + 2 * u;
            v[u] = ld_agent(ws + (static_cast<int64_t>(l) * nch + g0 + (k < gsize ? k : 0)) * kPart + ch);
        }
        double a = 0.0;
#pragma unroll
        for (int u = 0; u < kGrp / 2; ++u) a += p + 2 * u < gsize ? static_cast<double>(v[u]) : 0.0;
        dscr[p * 128 + ch] = a;
        __syncthreads();
        uint64_t *gp = cnt.gt + (static_cast<int64_t>(l) * kMaxGroups + grp) * kGT;
        if (p == 0) st_tagged(gp + ch, tag, static_cast<float>(dscr[ch] + dscr[128 + ch]));
        if (tid == 0) {
            st_tagged(gp + 128, tag, 1.f);  // the group's marker word
            __hip_atomic_store(gcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        mark(tr, 3);
    }
    await_groups(cnt, l, ngr, 128, tag, sync, 0x200u + l);
    mark(tr, 4);
    double a = 0.0;
    const uint64_t *base = cnt.gt + static_cast<int64_t>(l) * kMaxGroups * kGT + ch;
    for (int u0 = 0; p + 2 * u0 < ngr; u0 += 8) {  // groups p + 2 u, 8 per batch
        uint64_t w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int64_t g1 = p + 2 * (u0 + u);
            w[u] = __hip_atomic_load(base + (g1 < ngr ? g1 : 0) * kGT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        bool ok = true;
#pragma unroll
        for (int u = 0; u < 8; ++u) ok = ok && (p + 2 * (u0 + u) >= ngr || static_cast<unsigned>(w[u] >> 32) == tag);
        if (!ok)
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (p + 2 * (u0 + u) < ngr)
                    w[u] = __float_as_uint(ld_tagged(base + (p + 2 * (u0 + u)) * kGT, tag, sync, 0x200u + l));
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (p + 2 * (u0 + u) < ngr) a += static_cast<double>(__uint_as_float(static_cast<unsigned>(w[u])));
    }
    __syncthreads();  // (dscr: the group combine above may still read it)
    dscr[p * 128 + ch] = a;
    __syncthreads();
    if (p == 0) {
        const double tot = dscr[ch] + dscr[128 + ch];
        sm.ss[ch] = static_cast<float>(tot / static_cast<double>(n));
        if (c == 0) {
            if (ch < 64) dbeta[ch] = static_cast<float>(tot);
            else dgamma[ch - 64] = static_cast<float>(tot);
        }
    }
    __syncthreads();
    mark(tr, 5);
}

__global__ __launch_bounds__(256, 2) void gin_pair_bwd_k(const scgib_pair_bwd_args A) {
    __shared__ Smem sm;
    const int tid = threadIdx.x, wv = tid >> 6, lane = tid & 63, r16 = lane & 15, g = lane >> 4;
    const int64_t nch0 = n_chunks(A.enc[0].n_cap);
    const int e = static_cast<int64_t>(blockIdx.x) < nch0 ? 0 : 1;
    const scgib_pair_bwd_encoder &E = A.enc[e];
    const int64_t c = blockIdx.x - (e ? nch0 : 0);
    const int64_t nch = n_chunks(E.n_cap), ngr = n_groups(E.n_cap);
    const int L = A.n_layers, F = A.n_feat;
    float *ws = ws_of(E.ws);
    const Cnt cnt = cnt_of(E.counters);
    const unsigned tag = __hip_atomic_load(cnt.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    const int64_t n = E.dims ? static_cast<int64_t>(E.dims[0]) : E.n_cap;
    uint64_t *tr = A.trace ? A.trace + static_cast<int64_t>(blockIdx.x) * 64 : nullptr;
    mark(tr, 56);

    const Chunk ck = E.chunk_rec ? load_chunk_rec(E.chunk_rec + c * kRec, sm)
                                 : load_chunk(E.rowptr, E.col, E.comp_ptr, comp_count(E.comp_dims, E.n_comp),
                                              nch, c, A.sync, sm);
    const int rb0 = ck.rb0, nr = ck.nr, nrb = ck.nrb, ns = (ck.nr + 3) / 4;
    const int q4 = tid & 15, rs = tid >> 4;  // thread-row-wise roles: float4 slot, rows rs + 16 k
    float *P = sm.buf0, *Q = sm.buf1;
    float fw[16];

    // ---- d out of the chunk's rows -> P
    if (E.lin_g) {  // compressor[0] backward first: d out = g_out + g_t W0, dW0 += g_t^T f
        for (int v = rs; v < 16 * nrb; v += 16) {
            const bool ok = v < nr;
            const float4 gt = ld_row(rows_rsrc(E.lin_g, E.n_cap, 64), rb0 + v, 64, 4 * q4);
            const float4 fi = ld_row(rows_rsrc(E.lin_in, E.n_cap, 64), rb0 + v, 64, 4 * q4);
            *reinterpret_cast<float4 *>(Q + sidx(v, 4 * q4)) = keep4(ok, gt);
            *reinterpret_cast<float4 *>(P + sidx(v, 4 * q4)) = keep4(ok, fi);
        }
        load_frag_col<64, 64>(E.lin_w, 16 * wv, fw);
        // g_out rows in flight during the dW0 product
        float4 go[kNrb];
        {
            const Rsrc rg = rows_rsrc(E.g_out, E.g_out ? E.n_cap : 0, 64);
#pragma unroll
            for (int k = 0; k < kNrb; ++k) go[k] = ld_row(rg, rb0 + rs + 16 * k, 64, 4 * q4);
        }
        __syncthreads();
        f32x4 aw[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                       f32x4{0.f, 0.f, 0.f, 0.f}};
        float cs = 0.f;
        gemm_tn<4>(Q, P, ns, aw, cs);          // dW0 = g_t^T f, db0 = sum g_t
        float *sl = E.lin_slab + c * (64 * 64 + 64);
#pragma unroll
        for (int jb = 0; jb < 4; ++jb)
#pragma unroll
            for (int i = 0; i < 4; ++i) sl[(16 * wv + 4 * g + i) * 64 + 16 * jb + r16] = aw[jb][i];
        cs += __shfl_xor(cs, 16, kWave);
        cs += __shfl_xor(cs, 32, kWave);
        if (g == 0) sl[64 * 64 + 16 * wv + r16] = cs;
        __syncthreads();  // every read of P (f) done: g_out -> P, then P += g_t W0
#pragma unroll
        for (int k = 0; k < kNrb; ++k) {
            const int v = rs + 16 * k;
            if (v < 16 * nrb) *reinterpret_cast<float4 *>(P + sidx(v, 4 * q4)) = keep4(v < nr, go[k]);
        }
        __syncthreads();
        gemm_each(Q, fw, nrb, 0, 1, [&](int rb, const f32x4 &d) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int row = acc_row16(rb, i), col = acc_col16();
                float *pp = P + sidx(row, col);
                *pp = row < nr ? d[i] + *pp : 0.f;
            }
        });
    } else {
        for (int v = rs; v < 16 * nrb; v += 16) {
            float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
            if (v < nr && E.g_out) a = ld_row(rows_rsrc(E.g_out, E.n_cap, 64), rb0 + v, 64, 4 * q4);
            *reinterpret_cast<float4 *>(P + sidx(v, 4 * q4)) = a;
        }
        __syncthreads();
        if (E.g_readout)  // the readout's gradient, broadcast to its component's rows
            for (int t = tid; t < ck.ncomp * 16; t += 256) {
                const int k = t >> 4, q = t & 15;
                if (sm.cs[k] < sm.cs[k + 1]) {
                    const float4 gr = ld4(E.g_readout + (ck.i0 + k) * 64 + 4 * q);
                    for (int v = sm.cs[k]; v < sm.cs[k + 1]; ++v) {
                        float4 *d = reinterpret_cast<float4 *>(P + sidx(v, 4 * q));
                        *d = add4(*d, gr);
                    }
                }
            }
    }
    __syncthreads();
    mark(tr, 57);

    for (int l = L - 1; l >= 0; --l) {
        const int din = l == 0 ? 32 : 64;
        uint64_t *tl = tr ? tr + 8 * l : nullptr;
        mark(tl, 0);
        // ---- dy = dh [scale z2 + shift > 0] (in place), xhat, the chunk's sums
        const float *st = E.stat[l];
        const float4 mean = ld4(st + 4 * q4), istd = ld4(st + 64 + 4 * q4);
        const float4 sc = ld4(st + 128 + 4 * q4), sh = ld4(st + 192 + 4 * q4);
        float4 zv[kNrb];
        {
            const Rsrc rz = rows_rsrc(E.z2[l], E.n_cap, 64);
#pragma unroll
            for (int k = 0; k < kNrb; ++k) zv[k] = ld_row(rz, rb0 + rs + 16 * k, 64, 4 * q4);
        }
        // dy -> P (in place of dh), xhat -> Q
        float4 sdy = make_float4(0.f, 0.f, 0.f, 0.f), sdx = sdy;
#pragma unroll
        for (int k = 0; k < kNrb; ++k) {
            const int v = rs + 16 * k;
            if (v < 16 * nrb) {
                const float ok = v < nr ? 1.f : 0.f;
                const float4 zz = zv[k];
                float4 *pd = reinterpret_cast<float4 *>(P + sidx(v, 4 * q4));
                const float4 dh = *pd;
                const float4 dy = make_float4((sc.x * zz.x + sh.x > 0.f ? dh.x : 0.f) * ok,
                                              (sc.y * zz.y + sh.y > 0.f ? dh.y : 0.f) * ok,
                                              (sc.z * zz.z + sh.z > 0.f ? dh.z : 0.f) * ok,
                                              (sc.w * zz.w + sh.w > 0.f ? dh.w : 0.f) * ok);
                const float4 xh = make_float4((zz.x - mean.x) * istd.x, (zz.y - mean.y) * istd.y,
                                              (zz.z - mean.z) * istd.z, (zz.w - mean.w) * istd.w);
                *pd = dy;
                *reinterpret_cast<float4 *>(Q + sidx(v, 4 * q4)) = xh;
                sdy = add4(sdy, dy);
                sdx = add4(sdx, make_float4(dy.x * xh.x, dy.y * xh.y, dy.z * xh.z, dy.w * xh.w));
            }
        }
        {  // the row slots' sums: lane groups by shuffles, the 4 waves through red
#pragma unroll
            for (int off = 16; off <= 32; off <<= 1) {
                sdy = make_float4(sdy.x + __shfl_xor(sdy.x, off, kWave), sdy.y + __shfl_xor(sdy.y, off, kWave),
                                  sdy.z + __shfl_xor(sdy.z, off, kWave), sdy.w + __shfl_xor(sdy.w, off, kWave));
                sdx = make_float4(sdx.x + __shfl_xor(sdx.x, off, kWave), sdx.y + __shfl_xor(sdx.y, off, kWave),
                                  sdx.z + __shfl_xor(sdx.z, off, kWave), sdx.w + __shfl_xor(sdx.w, off, kWave));
            }
            if (lane < 16) {
                *reinterpret_cast<float4 *>(&sm.red[wv][4 * lane]) = sdy;
                *reinterpret_cast<float4 *>(&sm.red[wv][64 + 4 * lane]) = sdx;
            }
            __syncthreads();
            if (tid < 128)
                st_agent(ws + (static_cast<int64_t>(l) * nch + c) * kPart + tid,
                         ((sm.red[0][tid] + sm.red[1][tid]) + sm.red[2][tid]) + sm.red[3][tid]);
        }
        // r rows in flight during the exchange
        float4 rr[kNrb];
        {
            const Rsrc rrs = rows_rsrc(E.r[l], E.n_cap, 64);
#pragma unroll
            for (int k = 0; k < kNrb; ++k) rr[k] = ld_row(rrs, rb0 + rs + 16 * k, 64, 4 * q4);
        }
        mark(tl, 1);
        bwd_exchange(l, c, nch, ngr, n, ws, cnt, tag, E.dgamma[l], E.dbeta[l], A.sync, sm,
                     reinterpret_cast<double *>(&sm.red[0][0]), tl);
        // ---- dz2 = scale (dy - c1 - xhat c2) -> P; r -> Q
        {
            const float4 c1 = make_float4(sm.ss[4 * q4], sm.ss[4 * q4 + 1], sm.ss[4 * q4 + 2], sm.ss[4 * q4 + 3]);
            const float4 c2 = make_float4(sm.ss[64 + 4 * q4], sm.ss[65 + 4 * q4], sm.ss[66 + 4 * q4],
                                          sm.ss[67 + 4 * q4]);
#pragma unroll
            for (int k = 0; k < kNrb; ++k) {
                const int v = rs + 16 * k;
                if (v < 16 * nrb) {
                    const bool ok = v < nr;
                    float4 *pd = reinterpret_cast<float4 *>(P + sidx(v, 4 * q4));
                    float4 *qd = reinterpret_cast<float4 *>(Q + sidx(v, 4 * q4));
                    const float4 dy = *pd, xh = *qd;
                    *pd = keep4(ok, make_float4(sc.x * (dy.x - c1.x - xh.x * c2.x),
                                                sc.y * (dy.y - c1.y - xh.y * c2.y),
                                                sc.z * (dy.z - c1.z - xh.z * c2.z),
                                                sc.w * (dy.w - c1.w - xh.w * c2.w)));
                    *qd = keep4(ok, rr[k]);
                }
            }
        }
        __syncthreads();
        // ---- dW2 += dz2^T r, db2 (slab); dr = dz2 W2, dz1 = dr [r > 0] -> Q (in place of r)
        float *sl = E.slab[l] + c * E.slab_stride[l];
        {
            f32x4 a2[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                           f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            float cs2 = 0.f;
            gemm_tn<4>(P, Q, ns, a2, cs2);
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
#pragma unroll
                for (int i = 0; i < 4; ++i) sl[(16 * wv + 4 * g + i) * 64 + 16 * jb + r16] = a2[jb][i];
            cs2 += __shfl_xor(cs2, 16, kWave);
            cs2 += __shfl_xor(cs2, 32, kWave);
            if (g == 0) sl[64 * 64 + 64 * din + 16 * wv + r16] = cs2;
        }
        load_frag_col<64, 64>(E.w2[l], 16 * wv, fw);
        // agg rows in flight meanwhile (din / 4 float4 slots per row)
        float4 av[kNrb];
        {
            const int aq = q4 < din / 4 ? q4 : 0;
            const Rsrc ra = rows_rsrc(E.agg[l], E.n_cap, din);
#pragma unroll
            for (int k = 0; k < kNrb; ++k) av[k] = ld_row(ra, rb0 + rs + 16 * k, din, 4 * aq);
        }
        __syncthreads();  // every wave's dW2 reads of Q (r) done
        gemm_each(P, fw, nrb, 0, 1, [&](int rb, const f32x4 &d) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float *q = Q + sidx(acc_row16(rb, i), acc_col16());
                *q = *q > 0.f ? d[i] : 0.f;
            }
        });
        mark(tl, 6);
        __syncthreads();  // every read of P (dz2) done: agg -> P
#pragma unroll
        for (int k = 0; k < kNrb; ++k) {
            const int v = rs + 16 * k;
            if (v < 16 * nrb && q4 < din / 4)
                *reinterpret_cast<float4 *>(P + sidx(v, 4 * q4)) = keep4(v < nr, av[k]);
        }
        __syncthreads();
        // ---- dW1 += dz1^T agg, db1 (slab); d(agg) = dz1 W1 -> P (in place of agg)
        {
            f32x4 a1[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                           f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            float cs1 = 0.f;
            if (din == 64) gemm_tn<4>(Q, P, ns, a1, cs1);
            else gemm_tn<2>(Q, P, ns, a1, cs1);
#pragma unroll
            for (int jb = 0; jb < 4; ++jb)
                if (jb < din / 16)
#pragma unroll
                    for (int i = 0; i < 4; ++i) sl[64 * 64 + (16 * wv + 4 * g + i) * din + 16 * jb + r16] = a1[jb][i];
            cs1 += __shfl_xor(cs1, 16, kWave);
            cs1 += __shfl_xor(cs1, 32, kWave);
            if (g == 0) sl[64 * 64 + 64 * din + 64 + 16 * wv + r16] = cs1;
        }
        if (din == 64) load_frag_col<64, 64>(E.w1[l], 16 * wv, fw);
        else load_frag_col<64, 32>(E.w1[l], 16 * (wv & 1), fw);
        __syncthreads();  // every wave's dW1 reads of P (agg) done
        {
            const int ccol = din == 64 ? acc_col16() : 16 * (wv & 1) + r16;
            gemm_each(Q, fw, nrb, din == 64 ? 0 : wv >> 1, din == 64 ? 1 : 2, [&](int rb, const f32x4 &d) {
#pragma unroll
                for (int i = 0; i < 4; ++i) P[sidx(acc_row16(rb, i), ccol)] = d[i];
            });
        }
        __syncthreads();
        if (l > 0) {
            // dh of layer l-1: (1+eps) d(agg)[v] + sum over v's neighbours (P -> Q)
            const float ope = E.one_plus_eps[l];
            aggregate_rows(ck, E.col, sm, P, ope, q4, rs, [](float4 x) { return x; },
                           [&](int, int v, float4 a) {
                               if (v < 16 * nrb) *reinterpret_cast<float4 *>(Q + sidx(v, 4 * q4)) = a;
                           });
            __syncthreads();
            float *t = P;
            P = Q;
            Q = t;
        } else {
            // dWt += d(agg0)^T aggx: aggx rows -> Q (16 columns), waves 0, 1
            for (int v = rs; v < 16 * nrb; v += 16)
                if (q4 < 4)
                    *reinterpret_cast<float4 *>(Q + sidx(v, 4 * q4)) =
                        keep4(v < nr, ld_row(rows_rsrc(E.aggx, E.n_cap, 16), rb0 + v, 16, 4 * q4));
            __syncthreads();
            if (wv < 2) {
                f32x4 at[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                               f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
                float dummy = 0.f;
                gemm_tn<1>(P, Q, ns, at, dummy);
                if (r16 < F)
#pragma unroll
                    for (int i = 0; i < 4; ++i) sl[64 * 64 + 64 * 32 + 128 + (16 * wv + 4 * g + i) * F + r16] = at[0][i];
            }
        }
    }

    // ---- exit: the last workgroup advances both encoders' epochs (the next
    // launch's tag)
    mark(tr, 60);
    if (arrive(A.sync, sm) == gridDim.x - 1) {
        for (int ee = 0; ee < 2; ++ee) {
            const Cnt k = cnt_of(A.enc[ee].counters);
            if (tid == 64) {
                const unsigned ep = __hip_atomic_load(k.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(k.epoch, ep + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if (tid == 0) __hip_atomic_store(A.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

}  // namespace pair
}  // namespace scgib

using namespace scgib;

extern "C" int64_t scgib_gin_pair_args_bytes(void) { return sizeof(scgib_pair_fwd_args); }
extern "C" int32_t scgib_gin_pair_max_component(void) { return pair::kMaxComp; }
extern "C" int64_t scgib_gin_pair_chunks(int64_t n_cap) { return n_cap > 0 ? pair::n_chunks(n_cap) : 0; }
extern "C" int64_t scgib_gin_pair_chunk_rec_ints(void) { return pair::kRec; }
extern "C" int64_t scgib_gin_pair_ws_bytes(int64_t n_cap, int32_t n_layers) {
    return pair::ws_bytes(n_cap, n_layers);
}
extern "C" int64_t scgib_gin_pair_counters(int64_t n_cap, int32_t n_layers) {
    return pair::n_counters(n_cap, n_layers);
}

// co-resident workgroups of gin_pair_fwd_k on the current device (the grid
// must not exceed it: its workgroups wait on each other)
extern "C" int64_t scgib_gin_pair_slots(void) {
    static int64_t slots = -1;
    if (slots < 0) {
        int dev = 0, cus = 0, per = 0, per_b = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, pair::gin_pair_fwd_k, 256, 0) !=
                hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_b, pair::gin_pair_bwd_k, 256, 0) !=
                hipSuccess)
            return 0;
        per = per < per_b ? per : per_b;
        slots = static_cast<int64_t>(cus) * (per < 2 ? per : 2);
    }
    return slots;
}

extern "C" int scgib_gin_pair_fwd(const scgib_pair_fwd_args *args, scgib_stream_t stream) {
    if (!args || !args->x || !args->wt || !args->sync) return SCGIB_EINVAL;
    const scgib_pair_fwd_args &A = *args;
    if (A.n_layers < 1 || A.n_layers > SCGIB_PAIR_MAX_LAYERS || A.n_feat < 1 || A.n_feat > 16)
        return SCGIB_EUNSUPPORTED;
    int64_t grid = 0;
    for (int e = 0; e < 2; ++e) {
        const scgib_pair_encoder &E = A.enc[e];
        if (E.n_cap <= 0 || E.n_comp <= 0 || !E.rowptr || !E.col || !E.comp_ptr || !E.aggx ||
            !E.out || !E.ws || !E.counters || (E.readout && !E.seg) || (E.lin_w && (!E.lin_b || !E.lin_out)))
            return SCGIB_EINVAL;
        if (E.n_cap >= (int64_t(1) << 31) || E.n_comp >= (int64_t(1) << 31) ||
            pair::n_groups(E.n_cap) > pair::kMaxGroups)
            return SCGIB_EUNSUPPORTED;
        for (int l = 0; l < A.n_layers; ++l)
            if (!E.w1[l] || !E.b1[l] || !E.w2[l] || !E.b2[l] || !E.gamma[l] || !E.beta[l] ||
                !E.agg[l] || !E.r[l] || !E.z2[l] || !E.stat[l] ||
                ((E.running_mean[l] == nullptr) != (E.running_var[l] == nullptr)))
                return SCGIB_EINVAL;
        grid += pair::n_chunks(E.n_cap);
    }
    const int64_t slots = scgib_gin_pair_slots();
    if (grid > slots) return SCGIB_EUNSUPPORTED;  // not co-resident: the per-layer path
    pair::gin_pair_fwd_k<<<dim3(static_cast<unsigned>(grid)), 256, 0, as_stream(stream)>>>(A);
    return launch_status();
}

extern "C" int64_t scgib_gin_pair_bwd_args_bytes(void) { return sizeof(scgib_pair_bwd_args); }

extern "C" int scgib_gin_pair_bwd(const scgib_pair_bwd_args *args, scgib_stream_t stream) {
    if (!args || !args->sync) return SCGIB_EINVAL;
    const scgib_pair_bwd_args &A = *args;
    if (A.n_layers < 1 || A.n_layers > SCGIB_PAIR_MAX_LAYERS || A.n_feat < 1 || A.n_feat > 16)
        return SCGIB_EUNSUPPORTED;
    int64_t grid = 0;
    for (int e = 0; e < 2; ++e) {
        const scgib_pair_bwd_encoder &E = A.enc[e];
        if (E.n_cap <= 0 || E.n_comp <= 0 || !E.rowptr || !E.col || !E.comp_ptr || !E.aggx ||
            !E.ws || !E.counters || (E.lin_g && (!E.lin_w || !E.lin_in || !E.lin_slab)))
            return SCGIB_EINVAL;
        if (E.n_cap >= (int64_t(1) << 31) || E.n_comp >= (int64_t(1) << 31) ||
            pair::n_groups(E.n_cap) > pair::kMaxGroups)
            return SCGIB_EUNSUPPORTED;
        for (int l = 0; l < A.n_layers; ++l) {
            const int64_t width = 64 * 64 + 64 * (l == 0 ? 32 : 64) + 128 + (l == 0 ? 32 * A.n_feat : 0);
            if (!E.agg[l] || !E.r[l] || !E.z2[l] || !E.stat[l] || !E.w1[l] || !E.w2[l] ||
                !E.dgamma[l] || !E.dbeta[l] || !E.slab[l] || E.slab_stride[l] < width)
                return SCGIB_EINVAL;
        }
        grid += pair::n_chunks(E.n_cap);
    }
    if (grid > scgib_gin_pair_slots()) return SCGIB_EUNSUPPORTED;
    pair::gin_pair_bwd_k<<<dim3(static_cast<unsigned>(grid)), 256, 0, as_stream(stream)>>>(A);
    return launch_status();
}
