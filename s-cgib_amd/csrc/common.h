// Shared device helpers for the gfx950 kernels of libscgib.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/scgib.h"

namespace scgib {

constexpr int kWave = 64;  // CDNA wavefront
constexpr int kHidden = SCGIB_HIDDEN;

inline hipStream_t as_stream(scgib_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Launch status: the launch error of the last kernel, as a positive code.
inline int launch_status() {
    hipError_t e = hipGetLastError();
    return e == hipSuccess ? SCGIB_OK : static_cast<int>(e);
}

// Full-wave sum; every lane receives the total.  Fixed butterfly order, so
// the result is bitwise identical on every lane and every run.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
    return v;
}

// Bijective XCD-aware remap of a 1-D grid (cdna_hip_programming.md §5
// "XCD swizzle must be bijective"): logical tiles t and t+1 land on the same
// XCD, so neighbouring node ranges (same molecules, shared neighbour rows)
// share that XCD's L2.  Speed only: any placement is correct.
__device__ __forceinline__ int64_t xcd_remap(int64_t orig, int64_t nwg) {
    if (nwg <= 8) return orig;
    const int64_t xcd = orig % 8, q = nwg / 8, r = nwg % 8;
    const int64_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + orig / 8;
}

// Cross-workgroup data inside one kernel (last-arriver reductions): each
// XCD has its own L2, and a plain store can sit in the writer's L2 while a
// reader on another XCD misses to memory.  Agent-scope atomic stores/loads are
// coherent across the XCDs without an L2 write-back; an agent-scope release
// fence instead writes back the whole L2 (measured 5-10 us per workgroup).
// Pattern: st_agent the data, block_arrive (vmcnt(0) + barrier + one counter
// atomic), the last arriver ld_agent's it.
__device__ __forceinline__ void st_agent(float *p, float v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte variants (two 8-byte agent-scope accesses; p 16-byte aligned)
__device__ __forceinline__ void st_agent4(float *p, float4 v) {
    uint64_t *q = reinterpret_cast<uint64_t *>(p);
    __hip_atomic_store(q, __builtin_bit_cast(uint64_t, make_float2(v.x, v.y)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 1, __builtin_bit_cast(uint64_t, make_float2(v.z, v.w)), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float4 ld_agent4(const float *p) {
    const uint64_t *q = reinterpret_cast<const uint64_t *>(p);
    const float2 a = __builtin_bit_cast(float2, __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    const float2 b = __builtin_bit_cast(float2, __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    return make_float4(a.x, a.y, b.x, b.y);
}

// Count this workgroup in at `counter` and return whether it is the last of
// `expected` arrivals.  Every wave first waits for its stores to be
// acknowledged (vmcnt(0)); the barrier collects the waves; one thread counts
// the workgroup in.  Data exchanged this way must use st_agent / ld_agent.
__device__ __forceinline__ bool block_arrive(unsigned *counter, unsigned expected,
                                             unsigned count = 1u) {
    __shared__ unsigned s_ticket;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        s_ticket = __hip_atomic_fetch_add(counter, count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return s_ticket + count == expected;  // (count: arrivals this workgroup makes at once)
}

// Batched loads: a load written as `ok ? p[i] : 0` is compiled into its own
// branch with an s_waitcnt inside, which serialises a batch of such loads.
// The kernels instead load unconditionally from a clamped, always-valid index
// and apply the predicate to the value (ld_ok), so a batch stays in flight.
template <class T>
__device__ __forceinline__ T ld_ok(const T *p, int64_t i, int64_t safe, bool ok, T zero) {
    const T v = p[ok ? i : safe];
    return ok ? v : zero;
}

// Capacity mode: when `dims` (device int32) is given, dims[idx] is the actual
// count and `cap` (host) only sizes the grid; rows in [actual, cap) are
// written as zeros so padded buffers stay finite under graph replay.
__device__ __forceinline__ int64_t eff_count(const int32_t *dims, int idx, int64_t cap) {
    return dims ? static_cast<int64_t>(dims[idx]) : cap;
}

// Fixed-order sum of `nslab` per-workgroup slabs of `width` floats into out
// (slab.hip); deterministic.
int launch_slab_reduce(const float *slab, int nslab, int64_t width, float *out, hipStream_t st);

// Fused recon loss, forward finish (recon.hip): Gram reduce over the head
// MLP's tile partials + edge term + last-arriver loss.  wsd: 512 doubles.
// ru (or NULL): the compressor BatchNorm's running update in one more
// workgroup of the same launch.
int launch_recon_fin(const float *gslab, const float *im, const int32_t *rowptr,
                     const int32_t *col, int64_t n_nodes, int64_t n_edges, float *gram,
                     double *wsd, unsigned *cnt, float *loss, const int32_t *dims,
                     const scgib_running_update *ru, const unsigned *fault, hipStream_t st);

// Phase tracing (debug build only, `make trace` -> libscgib_trace.so):
// thread 0 of each workgroup stamps the 100 MHz wall clock at phase marks
// into g_trace[block * 32 + k] and the shader clock (s_memtime) into
// g_trace[block * 32 + 16 + k] (their ratio: the clock the CU held over a
// phase); slot 15 holds (XCC_ID << 32) | HW_ID.
#ifdef SCGIB_TRACE
static __device__ unsigned long long *g_trace;
#define SCGIB_MARK(k)                                                                     \
    do {                                                                                  \
        if (threadIdx.x == 0 && g_trace) {                                                \
            g_trace[static_cast<uint64_t>(blockIdx.x) * 32 + (k)] = wall_clock64();        \
            g_trace[static_cast<uint64_t>(blockIdx.x) * 32 + 16 + (k)] =                   \
                __builtin_amdgcn_s_memtime();                                             \
        }                                                                                 \
    } while (0)
#define SCGIB_MARK_HWID()                                                                 \
    do {                                                                                  \
        if (threadIdx.x == 0 && g_trace)                                                  \
            g_trace[static_cast<uint64_t>(blockIdx.x) * 32 + 15] =                          \
                (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((31 << 11) | 20)) << 32) | \
                static_cast<unsigned>(__builtin_amdgcn_s_getreg((31 << 11) | 4));         \
    } while (0)
#else
#define SCGIB_MARK(k) do {} while (0)
#define SCGIB_MARK_HWID() do {} while (0)
#endif

}  // namespace scgib
