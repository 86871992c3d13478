// Fused k-hop ego-net builder (gfx950): dgl.khop_in_subgraph(g, v, k) for
// every node v of a molecule batch, plus the dgl.batch of all of them, in
// three launches (count + block scan, scan fix-up, fill).
//
// Reference call sites: exp_pretraining.py:269-272 (one libdgl call per
// node, offline) and :308-309 (dgl.batch of the Σ n_i ego-nets every step).
// Semantics restated in oracle/egonet_ref.c; bit-exact parity is tested.
//
// Design: molecules are small, so an ego-net never leaves its molecule and a
// ball fits in a per-thread bitmap over the molecule's local node ids
// (W 64-bit words in registers, n_graph <= 64 W, W in {1,2,4,8}).  One thread
// builds one ego-net:
//   ball = {v}; frontier = {v}; k times: frontier = ∪ in-nbrs(frontier),
//   ball |= frontier                        (DGL: unique(cat(frontiers)))
// The bitmap gives DGL's sorted node order for free (ascending set bits) and
// the relabelling of an induced edge (u, w) is popcount(ball below w), so
// the fill pass writes ego nodes and CSR rows directly in DGL order
// (node_subgraph: rows in ball order, columns in CSR order).
// Integer/pointer-chasing work: no MFMA, all index reads L2-resident.
#include <type_traits>

#include "common.h"

namespace scgib {

template <int W>
__device__ __forceinline__ void bm_set(uint64_t (&b)[W], int32_t idx) {
#pragma unroll
    for (int i = 0; i < W; ++i) b[i] |= (i == (idx >> 6)) ? (1ull << (idx & 63)) : 0ull;
}

template <int W>
__device__ __forceinline__ bool bm_test(const uint64_t (&b)[W], int32_t idx) {
    uint64_t word = 0;
#pragma unroll
    for (int i = 0; i < W; ++i) word = (i == (idx >> 6)) ? b[i] : word;
    return (word >> (idx & 63)) & 1ull;
}

// number of set bits strictly below idx
template <int W>
__device__ __forceinline__ int32_t bm_rank(const uint64_t (&b)[W], int32_t idx) {
    int32_t r = 0;
    const int wi = idx >> 6;
    const uint64_t mask = (1ull << (idx & 63)) - 1ull;
#pragma unroll
    for (int i = 0; i < W; ++i) {
        if (i < wi) r += __popcll(b[i]);
        else if (i == wi) r += __popcll(b[i] & mask);
    }
    return r;
}

__device__ __forceinline__ int64_t graph_of(const int32_t *__restrict__ gptr, int64_t ng,
                                            int64_t v) {
    // largest g with gptr[g] <= v (graphs may be empty)
    int64_t lo = 0, hi = ng - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (gptr[mid] <= v) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

enum : int32_t { kErrEdgeLeavesGraph = 1, kErrGraphTooLarge = 2, kErrCapacity = 4 };

template <int W>
__device__ __forceinline__ void build_ball(int32_t lv, int32_t base, int32_t ng, int k,
                                           const int32_t *__restrict__ rowptr,
                                           const int32_t *__restrict__ col,
                                           uint64_t (&ball)[W], int32_t *err) {
    uint64_t fr[W];
#pragma unroll
    for (int i = 0; i < W; ++i) ball[i] = fr[i] = 0ull;
    bm_set<W>(ball, lv);
    bm_set<W>(fr, lv);
    for (int hop = 0; hop < k; ++hop) {
        uint64_t nx[W];
#pragma unroll
        for (int i = 0; i < W; ++i) nx[i] = 0ull;
#pragma unroll
        for (int wi = 0; wi < W; ++wi) {
            uint64_t m = fr[wi];
            while (m) {
                const int32_t u = wi * 64 + (__ffsll(static_cast<unsigned long long>(m)) - 1);
                m &= m - 1ull;
                const int32_t e1 = rowptr[base + u + 1];
                for (int32_t j = rowptr[base + u]; j < e1; ++j) {
                    const int32_t w = col[j] - base;
                    if (w < 0 || w >= ng) {
                        atomicOr(err, kErrEdgeLeavesGraph);
                        continue;
                    }
                    bm_set<W>(nx, w);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < W; ++i) {
            ball[i] |= nx[i];
            fr[i] = nx[i];
        }
    }
}

// Pool form of the builders (graph.EgoPrefetch): the input batch is the
// resident pool's blob srcs[ctr[0] % n_src] (graph.StaticBatch layout: CSR,
// graph_ptr and dims at byte offsets), resolved when the kernel starts, so a
// replayed step can build the ego-nets of the batch the next step loads.
struct EgoSrc {
    const uint64_t *srcs;  // nullptr: the plain pointers are used
    const unsigned *ctr;
    int64_t o_rowptr, o_col, o_gptr, o_dims;
    int32_t n_src;
};

template <class P, class G>  // (P: the kernels' __restrict__ parameter type)
__device__ __forceinline__ void ego_resolve(const EgoSrc &s, P &rowptr, P &col, G &gptr,
                                            P &dims) {
    if (!s.srcs) return;
    const unsigned c = __hip_atomic_load(s.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const char *base = reinterpret_cast<const char *>(s.srcs[c % static_cast<unsigned>(s.n_src)]);
    rowptr = reinterpret_cast<const int32_t *>(base + s.o_rowptr);
    col = reinterpret_cast<const int32_t *>(base + s.o_col);
    gptr = reinterpret_cast<const int32_t *>(base + s.o_gptr);
    dims = reinterpret_cast<const int32_t *>(base + s.o_dims);
}

template <int W>
__global__ __launch_bounds__(256) void egonet_count_k(
    const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ gptr, int64_t n_graphs, int64_t n, int k,
    int32_t *__restrict__ ego_ptr, int32_t *__restrict__ ego_eptr,
    int32_t *__restrict__ blk_tot, int32_t *err, const int32_t *__restrict__ dims, EgoSrc ps) {
    ego_resolve(ps, rowptr, col, gptr, dims);
    __shared__ int32_t sn[256], se[256];
    const int64_t v = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    int32_t nb = 0, ne = 0;
    if (v < eff_count(dims, 0, n)) {
        const int64_t g = graph_of(gptr, n_graphs, v);
        const int32_t base = gptr[g], ng = gptr[g + 1] - base;
        if (ng > 64 * W) {
            atomicOr(err, kErrGraphTooLarge);
        } else {
            uint64_t ball[W];
            build_ball<W>(static_cast<int32_t>(v - base), base, ng, k, rowptr, col, ball, err);
#pragma unroll
            for (int wi = 0; wi < W; ++wi) {
                uint64_t m = ball[wi];
                nb += __popcll(ball[wi]);
                while (m) {
                    const int32_t u = wi * 64 + (__ffsll(static_cast<unsigned long long>(m)) - 1);
                    m &= m - 1ull;
                    const int32_t e1 = rowptr[base + u + 1];
                    for (int32_t j = rowptr[base + u]; j < e1; ++j) {
                        const int32_t w = col[j] - base;
                        if (w >= 0 && w < ng && bm_test<W>(ball, w)) ++ne;
                    }
                }
            }
        }
    }
    // block-inclusive scan of (nb, ne), Hillis-Steele in LDS
    sn[threadIdx.x] = nb;
    se[threadIdx.x] = ne;
    __syncthreads();
    for (int off = 1; off < 256; off <<= 1) {
        int32_t an = 0, ae = 0;
        if (threadIdx.x >= off) {
            an = sn[threadIdx.x - off];
            ae = se[threadIdx.x - off];
        }
        __syncthreads();
        sn[threadIdx.x] += an;
        se[threadIdx.x] += ae;
        __syncthreads();
    }
    if (v < n) {
        ego_ptr[v + 1] = sn[threadIdx.x];
        ego_eptr[v + 1] = se[threadIdx.x];
    }
    if (threadIdx.x == 255) {
        blk_tot[blockIdx.x] = sn[255];
        blk_tot[gridDim.x + blockIdx.x] = se[255];
    }
}

// Adds the exclusive prefix of the block totals to every element; each block
// sums its predecessors itself (fixed order, no second scan launch).
__global__ __launch_bounds__(256) void egonet_scan_fixup_k(int64_t n, int32_t nblk,
                                                           const int32_t *__restrict__ blk_tot,
                                                           int32_t *__restrict__ ego_ptr,
                                                           int32_t *__restrict__ ego_eptr) {
    __shared__ int32_t rn[256], re[256];
    int32_t an = 0, ae = 0;
    for (int32_t j = threadIdx.x; j < static_cast<int32_t>(blockIdx.x); j += 256) {
        an += blk_tot[j];
        ae += blk_tot[nblk + j];
    }
    rn[threadIdx.x] = an;
    re[threadIdx.x] = ae;
    __syncthreads();
    for (int off = 128; off >= 1; off >>= 1) {
        if (threadIdx.x < off) {
            rn[threadIdx.x] += rn[threadIdx.x + off];
            re[threadIdx.x] += re[threadIdx.x + off];
        }
        __syncthreads();
    }
    const int64_t v = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (v < n) {
        ego_ptr[v + 1] += rn[0];
        ego_eptr[v + 1] += re[0];
    }
    if (v == 0) {
        ego_ptr[0] = 0;
        ego_eptr[0] = 0;
    }
}

template <int W>
__global__ __launch_bounds__(256) void egonet_fill_k(
    const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col,
    const int32_t *__restrict__ gptr, int64_t n_graphs, int64_t n, int k,
    const int32_t *__restrict__ ego_ptr, const int32_t *__restrict__ ego_eptr,
    int32_t *__restrict__ ego_nodes, int32_t *__restrict__ sub_rowptr,
    int32_t *__restrict__ sub_col, int32_t *err, int64_t n_ego_cap,
    const int32_t *__restrict__ dims, int32_t *__restrict__ ego_dims, EgoSrc ps) {
    ego_resolve(ps, rowptr, col, gptr, dims);
    const int64_t v = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (v == 0 && ego_dims) {  // the ego batch's actual [N_s, E_s], device-resident
        ego_dims[0] = ego_ptr[n];
        ego_dims[1] = ego_eptr[n];
    }
    // tail of the ego batch: [N_s, n_ego_cap) gets parent id 0 and empty CSR
    // rows, and sub_rowptr[N_s] = E_s (capacity-sized buffers stay valid)
    {
        const int64_t ns = ego_ptr[n], es = ego_eptr[n];
        for (int64_t i = ns + v; i <= n_ego_cap; i += static_cast<int64_t>(gridDim.x) * 256) {
            sub_rowptr[i] = static_cast<int32_t>(es);
            if (i < n_ego_cap) ego_nodes[i] = 0;
        }
    }
    if (v >= eff_count(dims, 0, n)) return;
    const int64_t g = graph_of(gptr, n_graphs, v);
    const int32_t base = gptr[g], ng = gptr[g + 1] - base;
    if (ng > 64 * W) return;  // flagged by the count pass
    uint64_t ball[W];
    build_ball<W>(static_cast<int32_t>(v - base), base, ng, k, rowptr, col, ball, err);
    const int32_t noff = ego_ptr[v];
    int32_t eo = ego_eptr[v];
    int32_t r = 0;
#pragma unroll
    for (int wi = 0; wi < W; ++wi) {
        uint64_t m = ball[wi];
        while (m) {
            const int32_t u = wi * 64 + (__ffsll(static_cast<unsigned long long>(m)) - 1);
            m &= m - 1ull;
            ego_nodes[noff + r] = base + u;
            sub_rowptr[noff + r] = eo;
            const int32_t e1 = rowptr[base + u + 1];
            for (int32_t j = rowptr[base + u]; j < e1; ++j) {
                const int32_t w = col[j] - base;
                if (w >= 0 && w < ng && bm_test<W>(ball, w)) sub_col[eo++] = noff + bm_rank<W>(ball, w);
            }
            ++r;
        }
    }
}

// ---------------------------------------------------------------------------
// k = 1 fast path (the pretraining configuration): ball(v) = {v} ∪ N(v) —
// DGL's unique(cat(frontiers)) for one hop — as a 128-bit window bitmap
// centred on v (bit 64 + u - v), so neither the molecule's bounds (a binary
// search over graph_ptr) nor a per-molecule bitmap are needed: with every
// molecule <= 64 atoms, |u - v| < 64 inside a molecule.  Ascending bits give
// DGL's sorted order; the relabelled id of a member is a popcount.  Every
// load round is batched: row pointers of v; its <= kK1Deg neighbour ids; the
// row pointers of the ball members; their neighbour ids (members in groups of
// K1G<D>, clamped always-valid addresses, predicates applied to the values).
// Requires in-degree <= kK1Deg, molecules <= 64 atoms and edges inside their
// molecule (host-checked).  Two launches: count + block scan, then fill with
// the cross-block scan fix-up folded in.
// ---------------------------------------------------------------------------
// D = the in-degree bound the launch was built for (6: one member group of
// 7 = |ball|, every molecule set of the benchmarks; 12: two groups)
// members per load group: the whole ball for D <= 8 (one rows round), else 7
template <int D> constexpr int K1G = D <= 8 ? D + 1 : 7;
template <int D> struct K1 {
    static constexpr int kDeg = D, kBall = D + 1;
};

template <int D>
struct K1Win {
    uint64_t w[2];   // bit 64 + (u - v): u in ball(v)
    int32_t v;
    int32_t nb;      // |ball|
    int32_t mem[D + 1];  // members, ascending (entries >= nb repeat the last)
};

template <int D>
__device__ __forceinline__ int32_t k1_index(const K1Win<D> &b, int32_t u) {
    const int32_t i = u - b.v + 64;
    const uint64_t word = i < 64 ? b.w[0] : b.w[1];  // selects: no dynamic indexing
    return (i >= 0 && i < 128 && ((word >> (i & 63)) & 1ull)) ? i : -1;
}

// members strictly below window index i
template <int D>
__device__ __forceinline__ int32_t k1_rank(const K1Win<D> &b, int32_t i) {
    const uint64_t m = (1ull << (i & 63)) - 1ull;
    return i < 64 ? __popcll(b.w[0] & m) : __popcll(b.w[0]) + __popcll(b.w[1] & m);
}

// CSR accessors of the k = 1 builders.  K1Global reads global memory and, for
// the neighbour slots past a row's end (whose values the callers predicate
// away), a clamped always-valid address so every slot is one batched load.
struct K1Global {
    const int32_t *__restrict__ rowptr;
    const int32_t *__restrict__ col;
    __device__ __forceinline__ int32_t rp(int32_t u) const { return rowptr[u]; }
    __device__ __forceinline__ int32_t cl(int32_t e, bool valid, int32_t last) const {
        return col[valid ? e : last];
    }
};

// K1Lds: the block's CSR window staged in LDS by two coalesced rounds —
// rowptr[lo .. lo + win] with lo = P b - 64 for P parents per block, win = P +
// 128 (the parents' rows and every ball member's: |u - v| < 64), then
// col[rowptr[lo] .. rowptr[lo + win]) up to the LDS capacity.  An index
// outside the window (none under the host-checked bounds) reads global
// memory; the slots past a row's end load nothing.
struct K1Lds {
    const int32_t *__restrict__ rowptr;
    const int32_t *__restrict__ col;
    const int32_t *sRp;
    const int32_t *sCol;
    int32_t lo, c0;
    uint32_t ncol, win;  // win: rows in the window (kK1WinRows for 64-parent blocks)
    __device__ __forceinline__ int32_t rp(int32_t u) const {
        const uint32_t i = static_cast<uint32_t>(u - lo);
        return i <= win ? sRp[i] : rowptr[u];
    }
    __device__ __forceinline__ int32_t cl(int32_t e, bool valid, int32_t) const {
        const uint32_t i = static_cast<uint32_t>(e - c0);
        return !valid ? 0 : (i < ncol ? sCol[i] : col[e]);
    }
};

template <int D, class A>
__device__ __forceinline__ void k1_ball(const A &acc, int32_t v, K1Win<D> &b) {
    const int32_t beg = acc.rp(v), end = acc.rp(v + 1);
    const int32_t last = end > beg ? end - 1 : (beg > 0 ? beg - 1 : 0);  // a valid index
    int32_t nbr[D];
#pragma unroll
    for (int j = 0; j < D; ++j) nbr[j] = acc.cl(beg + j, beg + j < end, last);
    b.v = v;
    b.w[0] = 0ull;
    b.w[1] = 1ull;  // v itself: bit 64
#pragma unroll
    for (int j = 0; j < D; ++j) {
        const int32_t i = nbr[j] - v + 64;
        const uint64_t bit = (beg + j < end && i >= 0 && i < 128) ? 1ull << (i & 63) : 0ull;
        b.w[0] |= i < 64 ? bit : 0ull;
        b.w[1] |= i < 64 ? 0ull : bit;
    }
    b.nb = __popcll(b.w[0]) + __popcll(b.w[1]);
    // members in ascending order, statically indexed (registers, no scratch):
    // member q = the lowest remaining bit; past the last, repeat it
    uint64_t m0 = b.w[0], m1 = b.w[1];
    int32_t prev = v;
#pragma unroll
    for (int q = 0; q < D + 1; ++q) {
        const bool lo = m0 != 0ull, hi = m1 != 0ull;
        const int32_t i = lo ? __ffsll(static_cast<unsigned long long>(m0)) - 1
                             : 64 + __ffsll(static_cast<unsigned long long>(m1)) - 1;
        const int32_t u = (lo || hi) ? v - 64 + i : prev;
        b.mem[q] = u;
        prev = u;
        if (lo) m0 &= m0 - 1ull;
        else if (hi) m1 &= m1 - 1ull;
    }
}

// rows of members [g0, g0 + K1G<D>) and their neighbour ids, one batched round each
template <int D>
struct K1Rows {
    int32_t beg[K1G<D>], deg[K1G<D>];
    int32_t w[K1G<D>][D];
};

template <int D, int G0, class A>
__device__ __forceinline__ void k1_rows(const A &acc, const K1Win<D> &b, K1Rows<D> &m) {
    int32_t end[K1G<D>];
#pragma unroll
    for (int r = 0; r < K1G<D>; ++r) {
        const int32_t u = b.mem[G0 + r < D + 1 ? G0 + r : D];
        m.beg[r] = acc.rp(u);
        end[r] = acc.rp(u + 1);
    }
#pragma unroll
    for (int r = 0; r < K1G<D>; ++r) {
        m.deg[r] = end[r] - m.beg[r];
        const int32_t last = end[r] > m.beg[r] ? end[r] - 1 : (m.beg[r] > 0 ? m.beg[r] - 1 : 0);
#pragma unroll
        for (int t = 0; t < D; ++t) m.w[r][t] = acc.cl(m.beg[r] + t, m.beg[r] + t < end[r], last);
    }
}

// inclusive scan of (a, b) over the 64 lanes of a wave (one workgroup)
constexpr int kK1Block = 64;  // 64-thread workgroups: the ego-nets spread over 4x more CUs

__device__ __forceinline__ void wave_scan2(int32_t &a, int32_t &b) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int32_t xa = __shfl_up(a, off, kWave), xb = __shfl_up(b, off, kWave);
        if (lane >= off) {
            a += xa;
            b += xb;
        }
    }
}

template <int D>
__global__ __launch_bounds__(kK1Block) void egonet_k1_count_k(
    const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n,
    int32_t *__restrict__ ego_ptr, int32_t *__restrict__ ego_eptr, int32_t *__restrict__ blk_tot,
    const int32_t *__restrict__ dims) {
    const int64_t v = static_cast<int64_t>(blockIdx.x) * kK1Block + threadIdx.x;
    int32_t nb = 0, ne = 0;
    if (v < eff_count(dims, 0, n)) {
        const K1Global acc{rowptr, col};
        K1Win<D> b;
        k1_ball<D>(acc, static_cast<int32_t>(v), b);
        nb = b.nb;
        auto count = [&](const K1Rows<D> &m, int g0) {
#pragma unroll
            for (int r = 0; r < K1G<D>; ++r)
#pragma unroll
                for (int t = 0; t < D; ++t)
                    ne += (g0 + r < b.nb && t < m.deg[r] && k1_index(b, m.w[r][t]) >= 0) ? 1 : 0;
        };
        {
            K1Rows<D> m;
            k1_rows<D, 0>(acc, b, m);
            count(m, 0);
        }
        if (D + 1 > K1G<D> && b.nb > K1G<D>) {  // balls of more than K1G<D> members: second group
            K1Rows<D> m;
            k1_rows<D, K1G<D>>(acc, b, m);
            count(m, K1G<D>);
        }
    }
    wave_scan2(nb, ne);
    if (v < n) {
        ego_ptr[v + 1] = nb;   // block-local inclusive; the fill adds the block prefix
        ego_eptr[v + 1] = ne;
    }
    if (threadIdx.x == kK1Block - 1) {
        blk_tot[blockIdx.x] = nb;
        blk_tot[gridDim.x + blockIdx.x] = ne;
    }
}

template <int D>
__global__ __launch_bounds__(kK1Block) void egonet_k1_fill_k(
    const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n,
    int32_t *__restrict__ ego_ptr, int32_t *__restrict__ ego_eptr,
    const int32_t *__restrict__ blk_tot, int32_t *__restrict__ ego_nodes,
    int32_t *__restrict__ sub_rowptr, int32_t *__restrict__ sub_col, int64_t n_ego_cap,
    const int32_t *__restrict__ dims, int32_t *__restrict__ ego_dims) {
    const int nblk = gridDim.x;
    const int64_t v = static_cast<int64_t>(blockIdx.x) * kK1Block + threadIdx.x;
    const bool live = v < eff_count(dims, 0, n);
    // the ball's loads go out first; the scan fix-up below overlaps them
    const K1Global acc{rowptr, col};
    K1Win<D> b;
    K1Rows<D> m;
    if (live) {
        k1_ball<D>(acc, static_cast<int32_t>(v), b);
        k1_rows<D, 0>(acc, b, m);
    }
    // block prefix and grand total of (nodes, edges), fixed order (wave sums)
    int32_t pn = 0, pe = 0, tn = 0, te = 0;
    for (int32_t j = threadIdx.x; j < nblk; j += kK1Block) {
        const int32_t a = blk_tot[j], c = blk_tot[nblk + j];
        tn += a;
        te += c;
        if (j < static_cast<int32_t>(blockIdx.x)) {
            pn += a;
            pe += c;
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        pn += __shfl_xor(pn, off, kWave);
        pe += __shfl_xor(pe, off, kWave);
        tn += __shfl_xor(tn, off, kWave);
        te += __shfl_xor(te, off, kWave);
    }
    const int32_t pre_n = pn, pre_e = pe, ns = tn, es = te;
    // this node's exclusive offsets from the count's block-local inclusive scan
    int32_t noff = pre_n, eo = pre_e, incl_n = 0, incl_e = 0;
    if (v < n) {
        incl_n = ego_ptr[v + 1];
        incl_e = ego_eptr[v + 1];
        if (threadIdx.x > 0) {
            noff += ego_ptr[v];
            eo += ego_eptr[v];
        }
    }
    __syncthreads();  // every read of the block-local values precedes the writes (one wave)
    if (v < n) {
        ego_ptr[v + 1] = pre_n + incl_n;
        ego_eptr[v + 1] = pre_e + incl_e;
    }
    if (v == 0) {
        ego_ptr[0] = 0;
        ego_eptr[0] = 0;
        if (ego_dims) {  // the ego batch's actual [N_s, E_s], device-resident
            ego_dims[0] = ns;
            ego_dims[1] = es;
        }
    }
    // tail of the ego batch: [N_s, n_ego_cap) gets parent id 0 and empty CSR rows
    for (int64_t i = ns + v; i <= n_ego_cap; i += static_cast<int64_t>(nblk) * kK1Block) {
        sub_rowptr[i] = es;
        if (i < n_ego_cap) ego_nodes[i] = 0;
    }
    if (!live) return;
    auto fill = [&](const K1Rows<D> &mm, auto g0c) {
        constexpr int G0 = decltype(g0c)::value;
#pragma unroll
        for (int r = 0; r < K1G<D>; ++r) {
            if (G0 + r < b.nb) {
                ego_nodes[noff + G0 + r] = b.mem[G0 + r < D + 1 ? G0 + r : D];
                sub_rowptr[noff + G0 + r] = eo;
#pragma unroll
                for (int t = 0; t < D; ++t) {
                    const int32_t i = k1_index(b, mm.w[r][t]);
                    if (t < mm.deg[r] && i >= 0) sub_col[eo++] = noff + k1_rank(b, i);
                }
            }
        }
    };
    fill(m, std::integral_constant<int, 0>{});
    if constexpr (D + 1 > K1G<D>) {
        if (b.nb > K1G<D>) {
            k1_rows<D, K1G<D>>(acc, b, m);
            fill(m, std::integral_constant<int, K1G<D>>{});
        }
    }
}

// ---------------------------------------------------------------------------
// k = 1 in ONE launch: each 64-parent block computes its balls, publishes its
// (nodes, edges) aggregate and takes its exclusive prefix by a decoupled
// look-back over the preceding blocks' published words, then fills — the
// count kernel's four dependent load rounds are not repeated by a fill
// launch.  state[b] packs (flag:2 | nodes:31 | edges:31) in one 64-bit word
// (flag 1: the block's aggregate, 2: its inclusive prefix); a block waits
// only on lower-numbered blocks.  HIP promises no dispatch order, so when the
// grid may not be co-resident (more than kK1Resident blocks) each block takes
// its logical index from an atomic ticket: every lower index then belongs to
// a block that is already running, and the look-back always progresses.  Each
// block drains its state stores (vmcnt(0)) before it counts itself done; the
// last block to finish zeroes every state word, the ticket and the finish
// counter, so the next launch (graph replay) starts from zeros.  Integer sums:
// exact.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t k1_pack(uint64_t flag, int32_t n, int32_t e) {
    return (flag << 62) | (static_cast<uint64_t>(static_cast<uint32_t>(n)) << 31) |
           static_cast<uint64_t>(static_cast<uint32_t>(e));
}

// The CSR window is staged in LDS and the look-back done by the whole wave
// (the scattered-global-load form with a one-lane look-back measured 2.7 %
// slower in the step, round 2).  kK1Waves: waves (64 parents each) per
// workgroup — 2 and 4 were parity-tested and measured no faster (round 2).
constexpr int kK1Waves = 1;
constexpr int kK1One = 64 * kK1Waves;  // parents per workgroup of the one-pass builder
// grids up to this many blocks are co-resident (64-thread blocks, 256 CUs):
// blockIdx.x serves as the logical index without the ticket's extra round trip
constexpr int kK1Resident = 1024;
template <int D>
__global__ __launch_bounds__(kK1One) void egonet_k1_onepass_k(
    const int32_t *__restrict__ rowptr, const int32_t *__restrict__ col, int64_t n,
    int32_t *__restrict__ ego_ptr, int32_t *__restrict__ ego_eptr, uint64_t *__restrict__ state,
    uint32_t *__restrict__ done, int32_t *__restrict__ ego_nodes,
    int32_t *__restrict__ sub_rowptr, int32_t *__restrict__ sub_col, int64_t n_ego_cap,
    int64_t e_cap, int32_t *__restrict__ err, const int32_t *__restrict__ dims,
    int32_t *__restrict__ ego_dims, EgoSrc ps) {
    const int nblk = gridDim.x, tid = threadIdx.x;
    int blk = blockIdx.x;
    {
        const int32_t *gptr = nullptr;
        ego_resolve(ps, rowptr, col, gptr, dims);
    }
    SCGIB_MARK(0);
    SCGIB_MARK_HWID();
    if (nblk > kK1Resident) {  // block-uniform: the logical index from the ticket
        __shared__ int sTicket;
        if (tid == 0)
            sTicket = static_cast<int>(__hip_atomic_fetch_add(done + 1, 1u, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_AGENT));
        __syncthreads();
        blk = sTicket;
    }
    const int lane = tid & 63, wave = tid >> 6;
    const int64_t v = static_cast<int64_t>(blk) * kK1One + tid;
    const bool live = v < eff_count(dims, 0, n);
    __shared__ int32_t sScan[kK1Waves][2];  // wave totals, then the block's prefix
    __shared__ int32_t sPre[3];
    // the block's CSR window -> LDS (K1Lds): two coalesced rounds instead of
    // four dependent rounds of scattered loads per parent
    constexpr int kWin = kK1One + 128;
    constexpr int kColCap = kWin * D;
    __shared__ int32_t sRp[kWin + 1];
    __shared__ int32_t sCol[kColCap];
    const int32_t lo = blk * kK1One - 64;
    for (int i = tid; i <= kWin; i += kK1One) {
        const int64_t u = lo + i;
        sRp[i] = rowptr[u < 0 ? 0 : (u > n ? n : u)];
    }
    __syncthreads();
    const int32_t c0 = sRp[0], dc = sRp[kWin] - c0;
    const int32_t nc = dc < 0 ? 0 : (dc < kColCap ? dc : kColCap);
    for (int i0 = 0; i0 < nc; i0 += 4 * kK1One) {
        int32_t t[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = i0 + k * kK1One + tid;
            t[k] = i < nc ? col[c0 + i] : 0;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = i0 + k * kK1One + tid;
            if (i < nc) sCol[i] = t[k];
        }
    }
    __syncthreads();
    SCGIB_MARK(1);
    const K1Lds acc{rowptr, col, sRp, sCol, lo, c0, static_cast<uint32_t>(nc),
                    static_cast<uint32_t>(kWin)};
    // with the window in LDS the loops run over the actual members and
    // degrees (not the D-slot predicated batches the global-load form needs)
    K1Win<D> b;
    int32_t nb = 0, ne = 0;
    if (live) {
        const int32_t vv = static_cast<int32_t>(v);
        b.v = vv;
        b.w[0] = 0ull;
        b.w[1] = 1ull;  // v itself: bit 64
        for (int32_t e = acc.rp(vv), e1 = acc.rp(vv + 1); e < e1; ++e) {
            const int32_t i = acc.cl(e, true, 0) - vv + 64;
            if (i >= 0 && i < 128) {
                if (i < 64) b.w[0] |= 1ull << i;
                else b.w[1] |= 1ull << (i - 64);
            }
        }
        nb = b.nb = __popcll(b.w[0]) + __popcll(b.w[1]);
        for (uint64_t m0 = b.w[0], m1 = b.w[1]; m0 | m1;) {  // members, any order
            const int32_t i = m0 ? __ffsll(static_cast<unsigned long long>(m0)) - 1
                                 : 64 + __ffsll(static_cast<unsigned long long>(m1)) - 1;
            if (m0) m0 &= m0 - 1ull;
            else m1 &= m1 - 1ull;
            const int32_t u = vv - 64 + i;
            for (int32_t e = acc.rp(u), e1 = acc.rp(u + 1); e < e1; ++e)
                ne += k1_index(b, acc.cl(e, true, 0)) >= 0 ? 1 : 0;
        }
    }
    SCGIB_MARK(2);
    int32_t in_n = nb, in_e = ne;  // inclusive within the wave, then the block
    wave_scan2(in_n, in_e);
    int32_t agg_n = __shfl(in_n, 63, kWave), agg_e = __shfl(in_e, 63, kWave);
    if constexpr (kK1Waves > 1) {  // waves' totals -> block-inclusive, block aggregate
        if (lane == 63) {
            sScan[wave][0] = agg_n;
            sScan[wave][1] = agg_e;
        }
        __syncthreads();
        int32_t wn = 0, we = 0, tn = 0, te = 0;
#pragma unroll
        for (int q = 0; q < kK1Waves; ++q) {
            wn += q < wave ? sScan[q][0] : 0;
            we += q < wave ? sScan[q][1] : 0;
            tn += sScan[q][0];
            te += sScan[q][1];
        }
        in_n += wn;
        in_e += we;
        agg_n = tn;
        agg_e = te;
    }
    int32_t pre_n = 0, pre_e = 0;
    if (tid == 0) {
        if (blk == 0) {
            __hip_atomic_store(&state[0], k1_pack(2, agg_n, agg_e), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        } else {
            __hip_atomic_store(&state[blk], k1_pack(1, agg_n, agg_e), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    // look-back by the whole wave (wave 0): lane i reads block (base - i)'s
    // word; the nearest inclusive prefix ends it once every nearer block has
    // published
    if (blk > 0 && wave == 0) {
        for (int32_t base = blk - 1;;) {  // wave-uniform control flow (ballots)
            const int32_t j = base - lane;
            const uint64_t w = j >= 0 ? __hip_atomic_load(&state[j], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : k1_pack(2, 0, 0);
            const uint64_t f = w >> 62;
            const uint64_t inc = __ballot(f == 2), unset = __ballot(f == 0);
            const int first = inc ? __ffsll(static_cast<unsigned long long>(inc)) - 1 : 64;
            const uint64_t need = first >= 63 ? ~0ull : ((2ull << first) - 1ull);
            if (unset & need) {
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            int32_t a = lane <= first ? static_cast<int32_t>((w >> 31) & 0x7fffffffull) : 0;
            int32_t e = lane <= first ? static_cast<int32_t>(w & 0x7fffffffull) : 0;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                a += __shfl_xor(a, off, kWave);
                e += __shfl_xor(e, off, kWave);
            }
            pre_n += a;
            pre_e += e;
            if (first < 64) break;
            base -= 64;
        }
        if (lane == 0)
            __hip_atomic_store(&state[blk], k1_pack(2, pre_n + agg_n, pre_e + agg_e),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (kK1Waves > 1) {  // wave 0's prefix to every wave
        if (tid == 0) {
            sPre[0] = pre_n;
            sPre[1] = pre_e;
        }
        __syncthreads();
        pre_n = sPre[0];
        pre_e = sPre[1];
    } else {
        pre_n = __shfl(pre_n, 0, kWave);
        pre_e = __shfl(pre_e, 0, kWave);
    }
    const int32_t noff = pre_n + in_n - nb;
    int32_t eo = pre_e + in_e - ne;
    if (v < n) {
        ego_ptr[v + 1] = pre_n + in_n;
        ego_eptr[v + 1] = pre_e + in_e;
    }
    if (v == 0) {
        ego_ptr[0] = 0;
        ego_eptr[0] = 0;
    }
    if (blk == nblk - 1) {  // the totals: the ego batch's sizes and its tail
        const int32_t ns = pre_n + agg_n, es = pre_e + agg_e;
        if (tid == 0 && ego_dims) {
            ego_dims[0] = ns;
            ego_dims[1] = es;
        }
        for (int64_t i = ns + tid; i <= n_ego_cap; i += kK1One) {
            sub_rowptr[i] = es;
            if (i < n_ego_cap) ego_nodes[i] = 0;
        }
    }
    SCGIB_MARK(3);
    if (live) {  // members ascending (DGL order), each row's columns in CSR order
        // (a ball past the buffers' capacities — a batch larger than the
        // capacity it was sized for — is flagged and its writes dropped)
        if (noff + nb > n_ego_cap || eo + ne > e_cap) {
            if (err) atomicOr(err, kErrCapacity);
        } else {
            int32_t r = 0;
            for (uint64_t m0 = b.w[0], m1 = b.w[1]; m0 | m1; ++r) {
                const int32_t i = m0 ? __ffsll(static_cast<unsigned long long>(m0)) - 1
                                     : 64 + __ffsll(static_cast<unsigned long long>(m1)) - 1;
                if (m0) m0 &= m0 - 1ull;
                else m1 &= m1 - 1ull;
                const int32_t u = b.v - 64 + i;
                ego_nodes[noff + r] = u;
                sub_rowptr[noff + r] = eo;
                for (int32_t e = acc.rp(u), e1 = acc.rp(u + 1); e < e1; ++e) {
                    const int32_t j = k1_index(b, acc.cl(e, true, 0));
                    if (j >= 0) sub_col[eo++] = noff + k1_rank(b, j);
                }
            }
        }
    }
    SCGIB_MARK(4);
    // every look-back of this block is done: count it in; the last one resets
    // (wave 0 only: its look-back is the block's)
    if (wave == 0) {
        if (lane == 0) {
            // this block's state stores are performed before it counts itself
            // done, so the last block's reset cannot be overtaken by one
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t t = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_AGENT);
            pre_n = t == static_cast<uint32_t>(nblk - 1) ? 1 : 0;
        }
        if (__shfl(pre_n, 0, kWave)) {
            for (int j = lane; j < nblk; j += 64)
                __hip_atomic_store(&state[j], uint64_t(0), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 0) {
                __hip_atomic_store(done + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

static int words_for(int32_t max_graph_nodes) {
    if (max_graph_nodes <= 64) return 1;
    if (max_graph_nodes <= 128) return 2;
    if (max_graph_nodes <= 256) return 4;
    if (max_graph_nodes <= 512) return 8;
    return 0;
}

}  // namespace scgib

using namespace scgib;

extern "C" int64_t scgib_egonet_workspace_bytes(int64_t n_nodes) {
    const int64_t nblk = (n_nodes + 63) / 64;  // the k = 1 builder's 64-node blocks
    return 2 * sizeof(int32_t) * (nblk > 0 ? nblk : 1);
}

static int ego_count_launch(const int32_t *rowptr, const int32_t *col, const int32_t *graph_ptr,
                            int64_t n_graphs, int64_t n_nodes, int32_t k, int32_t max_graph_nodes,
                            int32_t *ego_ptr, int32_t *ego_eptr, void *workspace, int32_t *err,
                            const int32_t *dims, EgoSrc ps, scgib_stream_t stream) {
    if (n_nodes < 0 || n_graphs < 0 || k < 0) return SCGIB_EINVAL;
    if (!ego_ptr || !ego_eptr || !err || !workspace) return SCGIB_EINVAL;
    if (n_nodes > 0 && !ps.srcs && (!rowptr || !col || !graph_ptr || n_graphs == 0))
        return SCGIB_EINVAL;
    if (n_nodes >= (int64_t(1) << 31)) return SCGIB_EUNSUPPORTED;
    const int W = words_for(max_graph_nodes);
    if (W == 0) return SCGIB_EUNSUPPORTED;
    hipStream_t st = as_stream(stream);
    if (n_nodes == 0) {
        hipError_t e = hipMemsetAsync(ego_ptr, 0, sizeof(int32_t), st);
        if (e == hipSuccess) e = hipMemsetAsync(ego_eptr, 0, sizeof(int32_t), st);
        return e == hipSuccess ? SCGIB_OK : static_cast<int>(e);
    }
    const int32_t nblk = static_cast<int32_t>((n_nodes + 255) / 256);
    int32_t *blk_tot = static_cast<int32_t *>(workspace);
#define SCGIB_EGO_COUNT(WW)                                                                     \
    egonet_count_k<WW><<<nblk, 256, 0, st>>>(rowptr, col, graph_ptr, n_graphs, n_nodes, k,    \
                                             ego_ptr, ego_eptr, blk_tot, err, dims, ps)
    switch (W) {
        case 1: SCGIB_EGO_COUNT(1); break;
        case 2: SCGIB_EGO_COUNT(2); break;
        case 4: SCGIB_EGO_COUNT(4); break;
        default: SCGIB_EGO_COUNT(8); break;
    }
#undef SCGIB_EGO_COUNT
    egonet_scan_fixup_k<<<nblk, 256, 0, st>>>(n_nodes, nblk, blk_tot, ego_ptr, ego_eptr);
    return launch_status();
}

static bool pool_src_ok(const uint64_t *srcs, int32_t n_src, const uint32_t *ctr,
                        int64_t o_rowptr, int64_t o_col, int64_t o_gptr, int64_t o_dims) {
    return srcs && n_src >= 1 && ctr && o_rowptr >= 0 && o_col >= 0 && o_gptr >= 0 &&
           o_dims >= 0 && (o_rowptr | o_col | o_gptr | o_dims) % 4 == 0;
}

extern "C" int scgib_egonet_count(const int32_t *rowptr, const int32_t *col,
                                  const int32_t *graph_ptr, int64_t n_graphs, int64_t n_nodes,
                                  int32_t k, int32_t max_graph_nodes, int32_t *ego_ptr,
                                  int32_t *ego_eptr, void *workspace, int32_t *err,
                                  const int32_t *dims, scgib_stream_t stream) {
    return ego_count_launch(rowptr, col, graph_ptr, n_graphs, n_nodes, k, max_graph_nodes,
                            ego_ptr, ego_eptr, workspace, err, dims, EgoSrc{}, stream);
}

extern "C" int scgib_egonet_count_pool(const uint64_t *srcs, int32_t n_src, const uint32_t *ctr,
                                       int64_t o_rowptr, int64_t o_col, int64_t o_gptr,
                                       int64_t o_dims, int64_t n_graphs, int64_t n_nodes,
                                       int32_t k, int32_t max_graph_nodes, int32_t *ego_ptr,
                                       int32_t *ego_eptr, void *workspace, int32_t *err,
                                       scgib_stream_t stream) {
    if (!pool_src_ok(srcs, n_src, ctr, o_rowptr, o_col, o_gptr, o_dims) || n_nodes < 1 ||
        n_graphs < 1)
        return SCGIB_EINVAL;
    const EgoSrc ps{srcs, reinterpret_cast<const unsigned *>(ctr), o_rowptr, o_col, o_gptr,
                    o_dims, n_src};
    return ego_count_launch(nullptr, nullptr, nullptr, n_graphs, n_nodes, k, max_graph_nodes,
                            ego_ptr, ego_eptr, workspace, err, nullptr, ps, stream);
}

extern "C" int64_t scgib_egonet_k1_max_degree(void) { return 12; }

extern "C" int64_t scgib_egonet_k1_max_graph_nodes(void) { return 64; }

template <int D>
static void launch_k1(const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                      int32_t *ego_ptr, int32_t *ego_eptr, int32_t *blk_tot, int32_t *ego_nodes,
                      int32_t *sub_rowptr, int32_t *sub_col, int64_t n_ego_cap,
                      const int32_t *dims, int32_t *ego_dims, hipStream_t st) {
    const int32_t nblk = static_cast<int32_t>((n_nodes + kK1Block - 1) / kK1Block);
    egonet_k1_count_k<D><<<nblk, kK1Block, 0, st>>>(rowptr, col, n_nodes, ego_ptr, ego_eptr,
                                                     blk_tot, dims);
    egonet_k1_fill_k<D><<<nblk, kK1Block, 0, st>>>(rowptr, col, n_nodes, ego_ptr, ego_eptr,
                                                    blk_tot, ego_nodes, sub_rowptr, sub_col,
                                                    n_ego_cap, dims, ego_dims);
}

extern "C" int scgib_egonet_k1_build_deg(const int32_t *rowptr, const int32_t *col,
                                         int64_t n_nodes, int32_t max_in_degree,
                                         int32_t *ego_ptr, int32_t *ego_eptr, void *workspace,
                                         int32_t *ego_nodes, int32_t *sub_rowptr,
                                         int32_t *sub_col, int64_t n_ego_cap,
                                         const int32_t *dims, int32_t *ego_dims,
                                         scgib_stream_t stream) {
    if (n_nodes <= 0 || !rowptr || !col || !ego_ptr || !ego_eptr || !workspace || !ego_nodes ||
        !sub_rowptr || !sub_col || max_in_degree < 0)
        return SCGIB_EINVAL;
    if (n_nodes >= (int64_t(1) << 31) || max_in_degree > 12) return SCGIB_EUNSUPPORTED;
    int32_t *blk_tot = static_cast<int32_t *>(workspace);
    hipStream_t st = as_stream(stream);
    if (max_in_degree <= 6)  // one member group, half the neighbour slots
        launch_k1<6>(rowptr, col, n_nodes, ego_ptr, ego_eptr, blk_tot, ego_nodes, sub_rowptr,
                     sub_col, n_ego_cap, dims, ego_dims, st);
    else if (max_in_degree <= 8)  // one member group of 9
        launch_k1<8>(rowptr, col, n_nodes, ego_ptr, ego_eptr, blk_tot, ego_nodes, sub_rowptr,
                     sub_col, n_ego_cap, dims, ego_dims, st);
    else
        launch_k1<12>(rowptr, col, n_nodes, ego_ptr, ego_eptr, blk_tot, ego_nodes, sub_rowptr,
                      sub_col, n_ego_cap, dims, ego_dims, st);
    return launch_status();
}

// one-launch form (egonet_k1_onepass_k): scan_state = scgib_egonet_k1_scan_words(n)
// zeroed uint32 words, left zeroed for the next launch (one launch in flight
// per scan_state)
extern "C" int64_t scgib_egonet_k1_scan_words(int64_t n_nodes) {
    return 2 * ((n_nodes + kK1Block - 1) / kK1Block) + 4;
}

static int k1_onepass_launch(const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                             int32_t max_in_degree, int32_t *ego_ptr, int32_t *ego_eptr,
                             uint32_t *scan_state, int32_t *ego_nodes, int32_t *sub_rowptr,
                             int32_t *sub_col, int64_t n_ego_cap, int64_t e_cap, int32_t *err,
                             const int32_t *dims, int32_t *ego_dims, EgoSrc ps,
                             scgib_stream_t stream) {
    if (n_nodes <= 0 || !ego_ptr || !ego_eptr || !scan_state || !ego_nodes || !sub_rowptr ||
        !sub_col || max_in_degree < 0 || n_ego_cap < 0 || e_cap < 0)
        return SCGIB_EINVAL;
    if (n_nodes >= (int64_t(1) << 31) || max_in_degree > 12) return SCGIB_EUNSUPPORTED;
    if (reinterpret_cast<uintptr_t>(scan_state) % 4) return SCGIB_EINVAL;
    const int32_t nblk = static_cast<int32_t>((n_nodes + kK1One - 1) / kK1One);
    uint32_t *done = scan_state;  // [0]: finished blocks, [1]: ticket
    uint64_t *state = reinterpret_cast<uint64_t *>(
        (reinterpret_cast<uintptr_t>(scan_state) + 2 * sizeof(uint32_t) + 7) & ~uintptr_t(7));
    hipStream_t st = as_stream(stream);
#define SCGIB_K1_ONEPASS(DD)                                                                     \
    egonet_k1_onepass_k<DD><<<nblk, kK1One, 0, st>>>(rowptr, col, n_nodes, ego_ptr, ego_eptr,   \
                                                     state, done, ego_nodes, sub_rowptr, sub_col, \
                                                     n_ego_cap, e_cap, err, dims, ego_dims, ps)
    if (max_in_degree <= 6) SCGIB_K1_ONEPASS(6);
    else if (max_in_degree <= 8) SCGIB_K1_ONEPASS(8);
    else SCGIB_K1_ONEPASS(12);
#undef SCGIB_K1_ONEPASS
    return launch_status();
}

extern "C" int scgib_egonet_k1_build_onepass(const int32_t *rowptr, const int32_t *col,
                                             int64_t n_nodes, int32_t max_in_degree,
                                             int32_t *ego_ptr, int32_t *ego_eptr,
                                             uint32_t *scan_state, int32_t *ego_nodes,
                                             int32_t *sub_rowptr, int32_t *sub_col,
                                             int64_t n_ego_cap, int64_t e_cap, int32_t *err,
                                             const int32_t *dims, int32_t *ego_dims,
                                             scgib_stream_t stream) {
    if (!rowptr || !col) return SCGIB_EINVAL;
    return k1_onepass_launch(rowptr, col, n_nodes, max_in_degree, ego_ptr, ego_eptr, scan_state,
                             ego_nodes, sub_rowptr, sub_col, n_ego_cap, e_cap, err, dims,
                             ego_dims, EgoSrc{}, stream);
}

// The same build over a resident pool's batch srcs[ctr[0] % n_src] (a
// graph.StaticBatch blob: rowptr / col / dims at the given byte offsets),
// resolved on the device at launch: a replayed step builds the ego-nets of the
// batch the next step will load (graph.EgoPrefetch) with no host work.
extern "C" int scgib_egonet_k1_build_onepass_pool(
    const uint64_t *srcs, int32_t n_src, const uint32_t *ctr, int64_t o_rowptr, int64_t o_col,
    int64_t o_dims, int64_t n_nodes, int32_t max_in_degree, int32_t *ego_ptr, int32_t *ego_eptr,
    uint32_t *scan_state, int32_t *ego_nodes, int32_t *sub_rowptr, int32_t *sub_col,
    int64_t n_ego_cap, int64_t e_cap, int32_t *err, int32_t *ego_dims, scgib_stream_t stream) {
    if (!pool_src_ok(srcs, n_src, ctr, o_rowptr, o_col, 0, o_dims)) return SCGIB_EINVAL;
    const EgoSrc ps{srcs, reinterpret_cast<const unsigned *>(ctr), o_rowptr, o_col, 0, o_dims,
                    n_src};
    return k1_onepass_launch(nullptr, nullptr, n_nodes, max_in_degree, ego_ptr, ego_eptr,
                             scan_state, ego_nodes, sub_rowptr, sub_col, n_ego_cap, e_cap, err,
                             nullptr, ego_dims, ps, stream);
}

extern "C" int scgib_egonet_k1_build(const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                                     int32_t *ego_ptr, int32_t *ego_eptr, void *workspace,
                                     int32_t *ego_nodes, int32_t *sub_rowptr, int32_t *sub_col,
                                     int64_t n_ego_cap, const int32_t *dims, int32_t *ego_dims,
                                     scgib_stream_t stream) {
    return scgib_egonet_k1_build_deg(rowptr, col, n_nodes, 12, ego_ptr, ego_eptr, workspace,
                                     ego_nodes, sub_rowptr, sub_col, n_ego_cap, dims, ego_dims,
                                     stream);
}

static int ego_fill_launch(const int32_t *rowptr, const int32_t *col, const int32_t *graph_ptr,
                           int64_t n_graphs, int64_t n_nodes, int32_t k, int32_t max_graph_nodes,
                           const int32_t *ego_ptr, const int32_t *ego_eptr, int32_t *ego_nodes,
                           int32_t *sub_rowptr, int32_t *sub_col, int32_t *err, int64_t n_ego_cap,
                           const int32_t *dims, int32_t *ego_dims, EgoSrc ps,
                           scgib_stream_t stream) {
    if (n_nodes < 0 || n_graphs < 0 || k < 0) return SCGIB_EINVAL;
    if (!ego_ptr || !ego_eptr || !sub_rowptr || !err) return SCGIB_EINVAL;
    if (n_nodes == 0) {
        const hipError_t e = hipMemsetAsync(sub_rowptr, 0, sizeof(int32_t), as_stream(stream));
        return e == hipSuccess ? SCGIB_OK : static_cast<int>(e);
    }
    if ((!ps.srcs && (!rowptr || !col || !graph_ptr)) || !ego_nodes || !sub_col)
        return SCGIB_EINVAL;
    const int W = words_for(max_graph_nodes);
    if (W == 0) return SCGIB_EUNSUPPORTED;
    hipStream_t st = as_stream(stream);
    const int64_t nblk = (n_nodes + 255) / 256;
#define SCGIB_EGO_FILL(WW)                                                                      \
    egonet_fill_k<WW><<<dim3((unsigned)nblk), 256, 0, st>>>(rowptr, col, graph_ptr, n_graphs,  \
                                                            n_nodes, k, ego_ptr, ego_eptr,     \
                                                            ego_nodes, sub_rowptr, sub_col, err, \
                                                            n_ego_cap, dims, ego_dims, ps)
    switch (W) {
        case 1: SCGIB_EGO_FILL(1); break;
        case 2: SCGIB_EGO_FILL(2); break;
        case 4: SCGIB_EGO_FILL(4); break;
        default: SCGIB_EGO_FILL(8); break;
    }
#undef SCGIB_EGO_FILL
    return launch_status();
}

extern "C" int scgib_egonet_fill(const int32_t *rowptr, const int32_t *col,
                                 const int32_t *graph_ptr, int64_t n_graphs, int64_t n_nodes,
                                 int32_t k, int32_t max_graph_nodes, const int32_t *ego_ptr,
                                 const int32_t *ego_eptr, int32_t *ego_nodes,
                                 int32_t *sub_rowptr, int32_t *sub_col, int32_t *err,
                                 int64_t n_ego_cap, const int32_t *dims, int32_t *ego_dims,
                                 scgib_stream_t stream) {
    return ego_fill_launch(rowptr, col, graph_ptr, n_graphs, n_nodes, k, max_graph_nodes, ego_ptr,
                           ego_eptr, ego_nodes, sub_rowptr, sub_col, err, n_ego_cap, dims,
                           ego_dims, EgoSrc{}, stream);
}

extern "C" int scgib_egonet_fill_pool(const uint64_t *srcs, int32_t n_src, const uint32_t *ctr,
                                      int64_t o_rowptr, int64_t o_col, int64_t o_gptr,
                                      int64_t o_dims, int64_t n_graphs, int64_t n_nodes, int32_t k,
                                      int32_t max_graph_nodes, const int32_t *ego_ptr,
                                      const int32_t *ego_eptr, int32_t *ego_nodes,
                                      int32_t *sub_rowptr, int32_t *sub_col, int32_t *err,
                                      int64_t n_ego_cap, int32_t *ego_dims,
                                      scgib_stream_t stream) {
    if (!pool_src_ok(srcs, n_src, ctr, o_rowptr, o_col, o_gptr, o_dims) || n_nodes < 1 ||
        n_graphs < 1)
        return SCGIB_EINVAL;
    const EgoSrc ps{srcs, reinterpret_cast<const unsigned *>(ctr), o_rowptr, o_col, o_gptr,
                    o_dims, n_src};
    return ego_fill_launch(nullptr, nullptr, nullptr, n_graphs, n_nodes, k, max_graph_nodes,
                           ego_ptr, ego_eptr, ego_nodes, sub_rowptr, sub_col, err, n_ego_cap,
                           nullptr, ego_dims, ps, stream);
}

#ifdef SCGIB_TRACE
// debug build only: this translation unit's phase-stamp buffer (common.h)
extern "C" int scgib_trace_set_egonet(void *buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif
