// GIN neighbourhood aggregation and per-segment readouts (gfx950).
//
// Both are HBM/L2-bound gathers of fp32 rows.  A row of `dim` floats is
// split into dim/4 float4 lanes (LPR lanes per row, 16 for dim 64), so one
// wave instruction moves 64 x 16 B = 1 KiB of 4 (dim 64) or 8 (dim 32)
// different rows: every load is a full 16-B-per-lane coalesced access and
// several neighbour rows are in flight per wave.  Neighbour loads are issued
// four at a time before they are consumed (latency hiding, Guideline 7).
// Sums run in CSR order, so results are deterministic.
#include <type_traits>

#include "common.h"

namespace scgib {

__device__ __forceinline__ float4 f4add(float4 a, float4 b) {
    return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

template <int LPR>
__global__ __launch_bounds__(256) void gin_aggregate_k(const float4 *__restrict__ h,
                                                       const int32_t *__restrict__ rowptr,
                                                       const int32_t *__restrict__ col,
                                                       int64_t ncap, float ope,
                                                       float4 *__restrict__ out,
                                                       const int32_t *__restrict__ dims) {
    constexpr int RPB = 256 / LPR;
    const int64_t blk = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t v = blk * RPB + threadIdx.x / LPR;
    const int c = threadIdx.x % LPR;
    if (v >= ncap) return;
    if (v >= eff_count(dims, 0, ncap)) {
        out[v * LPR + c] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    const int32_t beg = rowptr[v], end = rowptr[v + 1];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int32_t j = beg;
    for (; j + 4 <= end; j += 4) {
        const int64_t u0 = col[j], u1 = col[j + 1], u2 = col[j + 2], u3 = col[j + 3];
        const float4 a0 = h[u0 * LPR + c], a1 = h[u1 * LPR + c];
        const float4 a2 = h[u2 * LPR + c], a3 = h[u3 * LPR + c];
        acc = f4add(f4add(f4add(f4add(acc, a0), a1), a2), a3);
    }
    for (; j < end; ++j) acc = f4add(acc, h[static_cast<int64_t>(col[j]) * LPR + c]);
    const float4 self = h[v * LPR + c];
    // DGL GINConv: rst = (1 + eps) * feat_dst + neigh
    out[v * LPR + c] = make_float4(ope * self.x + acc.x, ope * self.y + acc.y,
                                   ope * self.z + acc.z, ope * self.w + acc.w);
}

template <int LPR>
__global__ __launch_bounds__(256) void segment_sum_k(const float4 *__restrict__ x,
                                                     const int32_t *__restrict__ ptr,
                                                     int64_t nseg, float4 *__restrict__ out,
                                                     const int32_t *__restrict__ dims) {
    constexpr int RPB = 256 / LPR;
    const int64_t blk = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t s = blk * RPB + threadIdx.x / LPR;
    const int c = threadIdx.x % LPR;
    if (s >= nseg) return;
    if (s >= eff_count(dims, 0, nseg)) {
        out[s * LPR + c] = make_float4(0.f, 0.f, 0.f, 0.f);
        return;
    }
    const int64_t beg = ptr[s], end = ptr[s + 1];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    int64_t i = beg;
    for (; i + 4 <= end; i += 4) {
        const float4 a0 = x[i * LPR + c], a1 = x[(i + 1) * LPR + c];
        const float4 a2 = x[(i + 2) * LPR + c], a3 = x[(i + 3) * LPR + c];
        acc = f4add(f4add(f4add(f4add(acc, a0), a1), a2), a3);
    }
    for (; i < end; ++i) acc = f4add(acc, x[i * LPR + c]);
    out[s * LPR + c] = acc;
}

template <int LPR>
__global__ __launch_bounds__(256) void segment_broadcast_k(const float4 *__restrict__ g,
                                                           const int32_t *__restrict__ ptr,
                                                           int64_t nseg,
                                                           float4 *__restrict__ out,
                                                           int64_t nrows,
                                                           const int32_t *__restrict__ dims) {
    constexpr int RPB = 256 / LPR;
    const int64_t blk = xcd_remap(blockIdx.x, gridDim.x);
    const int64_t s = blk * RPB + threadIdx.x / LPR;
    const int c = threadIdx.x % LPR;
    const int64_t ns = eff_count(dims, 0, nseg);
    if (dims) {  // zero the rows past the last valid segment (grid-stride)
        const int64_t r0 = ptr[ns];
        const int64_t tot = (nrows - r0) * LPR;
        for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < tot;
             i += static_cast<int64_t>(gridDim.x) * 256)
            out[r0 * LPR + i] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (s >= ns) return;
    const float4 val = g[s * LPR + c];
    for (int64_t i = ptr[s]; i < ptr[s + 1]; ++i) out[i * LPR + c] = val;
}

// Widths that are not a power-of-two multiple of 4 (e.g. the raw 9- or
// 11-wide node features the domain-adaptation Set2Set reads, models.py:114,
// :273): one thread per (segment, column), rows in order — same fixed-order
// sums, scalar loads (off the hot path).
__global__ __launch_bounds__(256) void segment_sum_scalar_k(const float *__restrict__ x,
                                                            const int32_t *__restrict__ ptr,
                                                            int64_t nseg, int32_t dim,
                                                            float *__restrict__ out,
                                                            const int32_t *__restrict__ dims) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (t >= nseg * dim) return;
    const int64_t s = t / dim, c = t % dim;
    if (s >= eff_count(dims, 0, nseg)) {
        out[t] = 0.f;
        return;
    }
    float acc = 0.f;
    for (int64_t i = ptr[s]; i < ptr[s + 1]; ++i) acc += x[i * dim + c];
    out[t] = acc;
}

__global__ __launch_bounds__(256) void segment_broadcast_scalar_k(
    const float *__restrict__ g, const int32_t *__restrict__ ptr, int64_t nseg, int32_t dim,
    float *__restrict__ out, int64_t nrows, const int32_t *__restrict__ dims) {
    const int64_t t = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
    if (t >= nrows * dim) return;
    const int64_t r = t / dim, c = t % dim, ns = eff_count(dims, 0, nseg);
    if (r >= ptr[ns]) {  // capacity-mode padding rows
        out[t] = 0.f;
        return;
    }
    int64_t lo = 0, hi = ns;  // segment of row r: ptr[s] <= r < ptr[s + 1]
    while (hi - lo > 1) {
        const int64_t mid = (lo + hi) / 2;
        if (ptr[mid] <= r) lo = mid;
        else hi = mid;
    }
    out[t] = g[lo * dim + c];
}

#define SCGIB_DISPATCH_LPR(dim, KERNEL, GRID_ROWS, ...)                                    \
    do {                                                                                    \
        const int lpr_ = (dim) / 4;                                                         \
        auto launch_ = [&](auto tag) {                                                      \
            constexpr int L = decltype(tag)::value;                                         \
            const int64_t rpb = 256 / L;                                                    \
            const int64_t grid = ((GRID_ROWS) + rpb - 1) / rpb;                             \
            if (grid > 0) KERNEL<L><<<dim3((unsigned)grid), dim3(256), 0, st>>>(__VA_ARGS__); \
        };                                                                                  \
        switch (lpr_) {                                                                     \
            case 1: launch_(std::integral_constant<int, 1>{}); break;                       \
            case 2: launch_(std::integral_constant<int, 2>{}); break;                       \
            case 4: launch_(std::integral_constant<int, 4>{}); break;                       \
            case 8: launch_(std::integral_constant<int, 8>{}); break;                       \
            case 16: launch_(std::integral_constant<int, 16>{}); break;                     \
            case 32: launch_(std::integral_constant<int, 32>{}); break;                     \
            case 64: launch_(std::integral_constant<int, 64>{}); break;                     \
            default: return SCGIB_EUNSUPPORTED;                                             \
        }                                                                                   \
    } while (0)

// Cross-queue hand-off without a graph edge (ops._GinEncoderPair): a graph
// edge between the step's two chains costs the waiting queue several us even
// when the producer finished long before; a one-wave
// kernel pair does not.  words: [0] signals, [1] waits consumed, [2] wait
// timeouts.  The producer queue's signal kernel runs after its chain (the
// kernel boundary writes that chain's data back); the consumer queue's wait
// kernel returns once a signal it has not consumed is there, so the next
// kernel on its queue (whose start invalidates the caches) reads the data.
__global__ void stream_signal_k(unsigned *w) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void stream_wait_k(unsigned *w, unsigned *fault, unsigned *host_fault) {
    if (threadIdx.x == 0) {
        const unsigned a = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = wall_clock64();
        while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - a - 1u >= 0x80000000u) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - t0 > 20000000) {  // 0.2 s of the 100 MHz clock: counted, not hung
                __hip_atomic_fetch_add(w + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // sticky: the step's loss kernels report NaN while it is set
                if (fault) __hip_atomic_store(fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // and the host's pinned copy, which the host checks without a
                // sync (ops.check_handoff: models' forwards, optim.Adam.step)
                if (host_fault)
                    __hip_atomic_store(host_fault, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
        }
        __hip_atomic_store(w + 1, a + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One batch of a resident pool into a step's static input buffer from inside
// a replayed graph (graph.StaticBatch.load_next): srcs is a device table of
// n_src pointers; the launch copies srcs[ctr[0] % n_src] to dst (n16 16-byte
// words) and, in the same grid, src2 to dst2 (n16b words: the prefetched
// ego-nets, graph.EgoPrefetch), then the last workgroup advances ctr[0] (ctr[1]:
// its arrival counter, left zero), so the replays walk the pool with no host
// work between them.
__global__ void pool_copy_k(const uint64_t *__restrict__ srcs, int32_t n_src, unsigned *ctr,
                            float4 *__restrict__ dst, int64_t n16, const float4 *__restrict__ src2,
                            float4 *__restrict__ dst2, int64_t n16b) {
    __shared__ unsigned s_c;
    if (threadIdx.x == 0) s_c = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned c = s_c;
    const float4 *src = reinterpret_cast<const float4 *>(srcs[c % static_cast<unsigned>(n_src)]);
    const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n16 + n16b;
         i += stride) {
        if (i < n16) dst[i] = src[i];
        else dst2[i - n16] = src2[i - n16];
    }
    if (block_arrive(ctr + 1, gridDim.x) && threadIdx.x == 0) {
        __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ctr, c + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// the hand-off kernels' launch handles, for the two-lane graph split
// (graph_split.hip), which adds them as kernel nodes and recognises the
// encoder pair's in-graph ones by them
void handoff_kernels(const void **signal, const void **wait) {
    *signal = reinterpret_cast<const void *>(&stream_signal_k);
    *wait = reinterpret_cast<const void *>(&stream_wait_k);
}

static bool dim_ok(int32_t dim) {
    return dim >= 4 && dim <= 256 && dim % 4 == 0 && ((dim / 4) & (dim / 4 - 1)) == 0;
}

}  // namespace scgib

using namespace scgib;

extern "C" int scgib_gin_aggregate(const float *h, const int32_t *rowptr, const int32_t *col,
                                   int64_t n_nodes, int32_t dim, float one_plus_eps,
                                   float *out, const int32_t *dims, scgib_stream_t stream) {
    if (n_nodes < 0 || !dim_ok(dim)) return SCGIB_EINVAL;
    if (n_nodes == 0) return SCGIB_OK;
    if (!h || !rowptr || !col || !out) return SCGIB_EINVAL;
    hipStream_t st = as_stream(stream);
    SCGIB_DISPATCH_LPR(dim, gin_aggregate_k, n_nodes, reinterpret_cast<const float4 *>(h),
                       rowptr, col, n_nodes, one_plus_eps, reinterpret_cast<float4 *>(out), dims);
    return launch_status();
}

extern "C" int scgib_segment_sum(const float *x, const int32_t *ptr, int64_t n_seg,
                                 int32_t dim, float *out, const int32_t *dims,
                                 scgib_stream_t stream) {
    if (n_seg < 0 || dim < 1) return SCGIB_EINVAL;
    if (n_seg == 0) return SCGIB_OK;
    if (!x || !ptr || !out) return SCGIB_EINVAL;
    hipStream_t st = as_stream(stream);
    if (!dim_ok(dim)) {
        const int64_t tot = n_seg * dim;
        segment_sum_scalar_k<<<dim3((unsigned)((tot + 255) / 256)), 256, 0, st>>>(
            x, ptr, n_seg, dim, out, dims);
        return launch_status();
    }
    SCGIB_DISPATCH_LPR(dim, segment_sum_k, n_seg, reinterpret_cast<const float4 *>(x), ptr,
                       n_seg, reinterpret_cast<float4 *>(out), dims);
    return launch_status();
}

extern "C" int scgib_segment_broadcast(const float *g, const int32_t *ptr, int64_t n_seg,
                                       int32_t dim, float *out, int64_t n_rows,
                                       const int32_t *dims, scgib_stream_t stream) {
    if (n_seg < 0 || n_rows < 0 || dim < 1) return SCGIB_EINVAL;
    if (n_seg == 0) return SCGIB_OK;
    if (!g || !ptr || !out) return SCGIB_EINVAL;
    hipStream_t st = as_stream(stream);
    if (!dim_ok(dim)) {
        const int64_t tot = n_rows * dim;
        if (tot > 0)
            segment_broadcast_scalar_k<<<dim3((unsigned)((tot + 255) / 256)), 256, 0, st>>>(
                g, ptr, n_seg, dim, out, n_rows, dims);
        return launch_status();
    }
    SCGIB_DISPATCH_LPR(dim, segment_broadcast_k, n_seg, reinterpret_cast<const float4 *>(g),
                       ptr, n_seg, reinterpret_cast<float4 *>(out), n_rows, dims);
    return launch_status();
}

extern "C" int scgib_stream_signal(uint32_t *words, scgib_stream_t stream) {
    if (!words) return SCGIB_EINVAL;
    stream_signal_k<<<1, 64, 0, as_stream(stream)>>>(words);
    return launch_status();
}

// Diagnostics (ops.stamps): the 100 MHz wall clock into buf[slot] when this
// point of the stream is reached — a replayed step's timeline with the
// hand-offs on (a kernel trace turns them off, ops.handoff_rule).
__global__ void stamp_k(uint64_t *buf, int32_t slot) {
    if (threadIdx.x == 0) buf[slot] = wall_clock64();
}

extern "C" int scgib_stamp(uint64_t *buf, int32_t slot, scgib_stream_t stream) {
    if (!buf || slot < 0) return SCGIB_EINVAL;
    stamp_k<<<1, 64, 0, as_stream(stream)>>>(buf, slot);
    return launch_status();
}

extern "C" int scgib_stream_wait(uint32_t *words, uint32_t *fault, uint32_t *host_fault,
                                 scgib_stream_t stream) {
    if (!words) return SCGIB_EINVAL;
    stream_wait_k<<<1, 64, 0, as_stream(stream)>>>(words, fault, host_fault);
    return launch_status();
}

extern "C" int scgib_pool_copy2(const uint64_t *srcs, int32_t n_src, uint32_t *ctr, void *dst,
                                int64_t bytes, const void *src2, void *dst2, int64_t bytes2,
                                scgib_stream_t stream) {
    if (!srcs || n_src < 1 || !ctr || !dst || bytes < 0 || bytes % 16 || bytes2 < 0 ||
        bytes2 % 16 || (bytes2 > 0 && (!src2 || !dst2)))
        return SCGIB_EINVAL;
    const int64_t n16 = bytes / 16, n16b = bytes2 / 16;
    const int64_t grid = std::max<int64_t>(1, std::min<int64_t>((n16 + n16b + 255) / 256, 1024));
    pool_copy_k<<<(unsigned)grid, 256, 0, as_stream(stream)>>>(
        srcs, n_src, reinterpret_cast<unsigned *>(ctr), reinterpret_cast<float4 *>(dst), n16,
        reinterpret_cast<const float4 *>(src2), reinterpret_cast<float4 *>(dst2), n16b);
    return launch_status();
}

extern "C" int scgib_pool_copy(const uint64_t *srcs, int32_t n_src, uint32_t *ctr, void *dst,
                               int64_t bytes, scgib_stream_t stream) {
    return scgib_pool_copy2(srcs, n_src, ctr, dst, bytes, nullptr, nullptr, 0, stream);
}

extern "C" int scgib_abi_version(void) { return 22; }

extern "C" const char *scgib_strerror(int code) {
    if (code == SCGIB_OK) return "ok";
    if (code == SCGIB_EINVAL) return "invalid argument (null pointer, negative size or bad dim)";
    if (code == SCGIB_EUNSUPPORTED) return "shape not supported by the kernels";
    if (code > 0) return hipGetErrorString(static_cast<hipError_t>(code));
    return "unknown scgib error";
}
