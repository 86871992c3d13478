/* scgib.h — C-ABI of the MI355X-native S-CGIB hot path (libscgib.so).
 *
 * The reference (O-JounLee/S-CGIB) is pure Python on PyTorch + DGL and has no
 * FFI of its own; each entry point below replaces the
 * library kernel the reference reaches through DGL / torch at the cited line.
 * The Python host mirror (s-cgib_amd/ops.py, models.py) binds them with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions (every function):
 *   - all pointers are DEVICE pointers (hipMalloc / torch CUDA tensors),
 *     caller-allocated; indices int32, features fp32 row-major;
 *   - `stream` is a hipStream_t (NULL = legacy default stream); every launch
 *     is asynchronous on it, nothing synchronises, nothing allocates — so a
 *     caller may capture any of them into a HIP graph;
 *   - return 0 (SCGIB_OK), a negative SCGIB_E* argument error, or a positive
 *     hipError_t from the launch; nothing throws across the ABI;
 *   - deterministic: no floating-point atomics; every reduction has a fixed
 *     order for a given shape;
 *   - capacity mode (HIP-graph replay): functions taking `const int32_t *dims`
 *     accept it NULL (the host sizes are exact) or a DEVICE array with the
 *     actual counts, dims[0] = nodes (or segments), dims[1] = edges, each <=
 *     the host size, which then only sizes the launch.  Rows past the actual
 *     count are written as zeros, so capacity-padded buffers stay finite and
 *     one captured graph serves every batch that fits.
 */
#ifndef SCGIB_H
#define SCGIB_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *scgib_stream_t; /* hipStream_t */

/* Deferred BatchNorm finalize (training, fused layers).  A layer launched
 * with defer = 1 leaves its batch statistics as group partials in its bn_ws
 * (at scgib_gin_bn_gpart_offset(n) floats) and does not write `stat` /
 * the running statistics; the NEXT kernel that needs them finishes the
 * combination in every workgroup (workgroup 0 writes the outputs), which
 * takes the serial last-arriver tail off the layer chain.  Layers up to
 * scgib_gin_defer_max_nodes() rows. */
typedef struct {
    const double *gpart;          /* producer's bn_ws + scgib_gin_bn_gpart_offset(n) */
    const float *gamma, *beta;    /* producer layer's BatchNorm affine */
    float *running_mean, *running_var;  /* NULL: untracked */
    int64_t *num_batches_tracked;
    float *stat;                  /* producer's [4][64] record (mean, invstd, scale, shift) */
    float eps, momentum;
} scgib_bn_pending;

typedef struct {
    const double *gpart;          /* bwd-stats bn_ws + scgib_gin_bn_gpart_offset(n) */
    float *dgamma, *dbeta;        /* written by workgroup 0 of the consumer */
    int32_t training;
} scgib_bn_bwd_pending;

enum {
    SCGIB_OK = 0,
    SCGIB_EINVAL = -1,       /* null pointer / negative size / bad dim      */
    SCGIB_EUNSUPPORTED = -2, /* shape outside what the kernels implement    */
};

#define SCGIB_HIDDEN 64     /* S-CGIB hidden width (args.dims, exp_pretraining.py:386) */
#define SCGIB_STATS_STRIDE 260 /* floats per graph in the interaction stats slab */
#define SCGIB_PGRAD_STRIDE 324 /* floats per graph in the parameter-gradient slab */

int scgib_abi_version(void);
/* Cross-queue hand-off without a stream/graph dependency: `words` is four
 * zeroed uint32 shared by one producer/consumer pair.  scgib_stream_signal
 * (producer stream, after the work to hand over) counts one signal;
 * scgib_stream_wait (consumer stream) returns once a signal it has not yet
 * consumed is there, so the consumer stream's later kernels see the
 * producer's data.  Calls must pair up in order (n-th wait <-> n-th signal).
 * A wait that sees no signal for 0.2 s gives up, counts words[2] and sets the
 * sticky *fault word (fault may be NULL): the step's loss kernels
 * (scgib_mlp2_recon_fwd / _contrastive_fwd, given the same word) then
 * report a NaN loss until the caller clears it, since some kernel of that
 * step read data before it was written.  It also sets *host_fault (may be
 * NULL): a host-visible pinned word the host reads without a sync (the
 * Python mirror raises on it at the next model forward / optimizer step,
 * ops.check_handoff — the fine-tune and domain-adaptation heads' losses are
 * torch ops, and NaN scores would trip binary_cross_entropy's range assert).
 * Correctness needs the signal and the wait on queues the device runs
 * concurrently ("Cross-queue hand-offs"). */
/* The next batch of a resident pool into a static input buffer, for a
 * replayed step graph: srcs = device table of n_src device pointers (each
 * `bytes` long, bytes a multiple of 16); copies srcs[ctr[0] % n_src] to dst
 * and advances ctr[0].  ctr: two uint32, ctr[1] zero on entry (left zero). */
int scgib_pool_copy(const uint64_t *srcs, int32_t n_src, uint32_t *ctr, void *dst, int64_t bytes,
                    scgib_stream_t stream);
/* ... and, in the same launch, bytes2 (a multiple of 16) from src2 to dst2
 * (graph.EgoPrefetch: the ego-nets built for this batch during the previous
 * step, staging -> the step's ego buffers). */
int scgib_pool_copy2(const uint64_t *srcs, int32_t n_src, uint32_t *ctr, void *dst, int64_t bytes,
                     const void *src2, void *dst2, int64_t bytes2, scgib_stream_t stream);
int scgib_stream_signal(uint32_t *words, scgib_stream_t stream);
int scgib_stream_wait(uint32_t *words, uint32_t *fault, uint32_t *host_fault,
                      scgib_stream_t stream);
/* Two-lane replay of a captured step graph (ABI 21; DESIGN.md §3, "Host
 * enqueue"): hipGraphLaunch of a graph with parallel branches costs the host
 * ~2.5-3 us per node, a linear graph ~6 us in all.  scgib_graph_split takes a
 * captured hipGraph_t (`graph`; kernel nodes only, else SCGIB_EUNSUPPORTED)
 * whose DAG is at most two chains wide, assigns its nodes to two lanes along
 * the captured chains, and builds one linear graph per lane (the kernel nodes
 * copied; each cross-lane edge becomes a scgib_stream_signal /
 * scgib_stream_wait kernel pair on its own 4-uint32 slot of `words`,
 * n_slots slots, zeroed, alive as long as the split; the last 8 slots are
 * for the queue check below).  `fault` / `host_fault` are the waits' sticky
 * fault words as for scgib_stream_wait.  `stream`: the caller's stream, the
 * one every replay must use — the split's non-blocking side stream is
 * checked at creation to run on another hardware queue than it (a
 * wait / signal pair across the two; up to 8 streams tried, else
 * SCGIB_EUNSUPPORTED).  *out receives an opaque handle; info (8 int32, may be
 * NULL): captured nodes, lane-0 kernels, lane-1 kernels, hand-offs added,
 * lane-0 nodes, lane-1 nodes, nodes serialised beyond two chains, slots used.
 * The captured graph's memory must stay alive while the split is used.
 * scgib_graph_split_launch replays lane 0 on `stream` (the creation stream,
 * else SCGIB_EINVAL) and lane 1 on the side stream, with one launch's stream
 * semantics: ordered after earlier work on `stream`, later work on `stream`
 * ordered after both lanes.  scgib_graph_split_destroy waits for the side
 * lane and frees it. */
int scgib_graph_split(void *graph, uint32_t *words, int32_t n_slots, uint32_t *fault,
                      uint32_t *host_fault, scgib_stream_t stream, void **out, int32_t *info);
int scgib_graph_split_launch(void *split, scgib_stream_t stream);
/* The lane plan scgib_graph_split makes, on the host alone (no device): n
 * nodes, m edges from[k] -> to[k], n_hidden in-graph hand-off pairs
 * (signal node -> wait node).  Per node (n int32 each, may be NULL): lane,
 * position in it, the slot of the wait placed before it and of the signal
 * placed after it (-1: none); info (4 int32): slots, the start hand-off's
 * slot (a signal before lane 0's first node, a wait before lane 1's), the
 * end hand-off's slot (a signal after lane 1's last node, a wait after lane
 * 0's last), nodes serialised beyond two chains (-1: no such hand-off).
 * SCGIB_EUNSUPPORTED where scgib_graph_split refuses the graph. */
int scgib_graph_split_plan(int32_t n, int32_t m, const int32_t *from, const int32_t *to,
                           int32_t n_hidden, const int32_t *hidden_signal,
                           const int32_t *hidden_wait, int32_t *lane, int32_t *pos,
                           int32_t *wait_slot, int32_t *signal_slot, int32_t *info);
int scgib_graph_split_destroy(void *split);
/* Diagnostics: writes the 100 MHz device wall clock (s_memrealtime) to
 * buf[slot] when the stream reaches this point (ops.stamps: the timeline of
 * a replayed step with its hand-offs on; not on the product path). */
int scgib_stamp(uint64_t *buf, int32_t slot, scgib_stream_t stream);
const char *scgib_strerror(int code);

/* ---- A5: GIN neighbourhood aggregation (DGL GINConv, sum aggregator) ------
 * out[v,:] = one_plus_eps * h[v,:] + sum_{j in [rowptr[v], rowptr[v+1])} h[col[j],:]
 * CSR is dst-major (row v lists the SOURCES of v's in-edges).  With the
 * transposed CSR this is also the backward (grad_h from grad_out).
 * Replaces DGL GINConv.forward -> update_all(copy_u, sum) (models.py:69).
 * dim % 4 == 0, 4 <= dim <= 256. */
int scgib_gin_aggregate(const float *h, const int32_t *rowptr, const int32_t *col,
                        int64_t n_nodes, int32_t dim, float one_plus_eps, float *out,
                        const int32_t *dims, scgib_stream_t stream);

/* ---- A5 fused: one GIN layer = GINConv(MLP) + BatchNorm1d + ReLU -----------
 * Replaces, per layer, DGL GINConv + nn.Linear x2 + ReLU + nn.BatchNorm1d +
 * F.relu of GIN.forward (models.py:63-71) and their autograd backward.
 * Tiles of 64 rows; scgib_gin_tiles(n) tiles; tile_stats holds 128 floats per
 * tile.  `stat` is the layer's [4][64] BN record: mean, invstd, scale
 * (= gamma*invstd), shift (= beta - mean*scale).
 *
 * scgib_gin_layer_fwd: agg = (1+eps) x_v + sum_{u->v} x_u with x = h_in, or
 *   x = relu(in_stat.scale * h_in + in_stat.shift) when in_stat != NULL
 *   (the previous layer's BN+ReLU applied on load; d_in must be 64);
 *   r = relu(agg W1^T + b1); z2 = r W2^T + b2; per-tile (sum, centred M2).
 *   d_in in {32, 64}; hidden 64.  Outputs agg [n,d_in], r, z2 [n,64];
 *   r may be NULL (also in scgib_gin_layer_fwd_bn / scgib_gin_layer0_fwd): it
 *   is then not stored and the backward recomputes it (below).
 * scgib_bn_finalize: training: batch mean/var from the tile stats (fp64
 *   Chan combine), running stats updated (momentum, unbiased var,
 *   num_batches_tracked += 1); eval: running stats.  Writes `stat`.
 * scgib_bn_relu_apply: out = relu(stat.scale * z + stat.shift)  [n,64].
 *   in_pending (may be NULL): the last GIN layer's deferred statistics
 *   (scgib_bn_pending below) — finished here, `stat` is then written.
 * scgib_gin_bwd_stats: dy = dh * [stat.scale z2 + stat.shift > 0], dh given,
 *   or, with (rowptr_t, col_t), gathered from the next layer's d(agg):
 *   dh_v = (1+eps) g_v + sum_{u in out(v)} g_u.  Per-tile sum(dy), sum(dy xhat).
 * scgib_bn_bwd_finalize: dgamma, dbeta [64] and coef [2][64] for dz2.
 * scgib_gin_layer_bwd: d(agg) [n,d_in] and wgrad = dW2[64*64] | dW1[64*d_in]
 *   | db2[64] | db1[64] through scgib_gin_layer_bwd_slabs(n, d_in) per-workgroup
 *   slabs of 64*64 + 64*d_in + 128 floats (scgib_gin_slab_floats(n, d_in) in
 *   total; d_in = 64: 32-row sub-tiles, up to two workgroups per CU each
 *   walking its sub-tiles), reduced in a fixed order.  With wgrad NULL the slabs are left for the
 *   caller's scgib_slab_reduce (so the GEMM kernel can be timed alone).
 *   r NULL (d_in = 64, and scgib_gin_layer0_bwd): the forward did not store r
 *   (a third of the forward's HBM writes); the kernel
 *   recomputes r = relu(agg W1^T + b1) from the saved agg with the forward's
 *   own MFMA chain — bitwise the r it would have stored, so every output is
 *   bitwise the stored-r kernel's.  b1 is read only then (may be NULL with r).
 * scgib_gin_hidden: r = relu(agg W1^T + b1) [n,64] with that same chain
 *   (inspection / tests: the hidden ReLU decisions of a step that did not
 *   store r).
 * scgib_slab_reduce: out[w] = sum_s slab[s*width + w], fixed order. */
int64_t scgib_gin_tiles(int64_t n_nodes);
int64_t scgib_gin_slab_floats(int64_t n_nodes, int32_t d_in);
int64_t scgib_gin_bwd_slabs(int64_t n_nodes);  /* layer-0 (transfer_d folded) slabs */
int64_t scgib_gin_layer_bwd_slabs(int64_t n_nodes, int32_t d_in);
/* Up to scgib_slab_reduce_max_jobs() independent scgib_slab_reduce's in one
 * launch (same fixed order per job): out[w] = sum_s slab[s*stride + w] for
 * w < width; stride 0 means width (a column range of wider slabs otherwise,
 * stride >= width). */
typedef struct {
    const float *slab;
    float *out;
    int64_t width;
    int32_t n_slabs;
    int32_t stride;
} scgib_slab_job;
int64_t scgib_slab_reduce_max_jobs(void);
int scgib_slab_reduce_multi(const scgib_slab_job *jobs, int32_t n_jobs, scgib_stream_t stream);
/* The same on at most max_workgroups workgroups (0: no cap; each loops over
 * column blocks) — for a reduce that runs beside another chain's kernels. */
int scgib_slab_reduce_multi_ex(const scgib_slab_job *jobs, int32_t n_jobs,
                               int32_t max_workgroups, scgib_stream_t stream);
int scgib_slab_reduce(const float *slab, int32_t n_slabs, int64_t width, float *out,
                      scgib_stream_t stream);
int scgib_gin_layer_fwd(const float *h_in, int32_t d_in, const float *in_stat,
                        const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                        float one_plus_eps, const float *w1, const float *b1, const float *w2,
                        const float *b2, float *agg, float *r, float *z2, float *tile_stats,
                        const int32_t *dims, scgib_stream_t stream);
int scgib_bn_finalize(const float *tile_stats, int64_t n_nodes, const float *gamma,
                      const float *beta, float eps, float momentum, int32_t training,
                      float *running_mean, float *running_var, int64_t *num_batches_tracked,
                      float *stat, const int32_t *dims, scgib_stream_t stream);
int scgib_bn_relu_apply(const float *z, const float *stat, int64_t n_nodes, float *out,
                        const int32_t *dims, const scgib_bn_pending *in_pending,
                        scgib_stream_t stream);
int scgib_gin_bwd_stats(const float *dh, const int32_t *rowptr_t, const int32_t *col_t,
                        float one_plus_eps, const float *z2, const float *stat, int64_t n_nodes,
                        float *dy, float *tile_stats, const int32_t *dims,
                        scgib_stream_t stream);
int scgib_bn_bwd_finalize(const float *tile_stats, int64_t n_nodes, int32_t training,
                          float *dgamma, float *dbeta, float *coef, const int32_t *dims,
                          scgib_stream_t stream);
/* Training-mode fused variants: the BatchNorm finalize is folded into the
 * tile kernel (hierarchical last-arriver over 16-tile groups, past 64 groups
 * also over 64-group supergroups; fp64, fixed order) — one launch per layer
 * instead of two.  `bn_ws` holds scgib_gin_bn_ws_floats(n) floats (tile
 * statistics + group and supergroup partials);
 * `counters` holds scgib_gin_counters(n) uint32 that are zero on entry and
 * left zero (graph-replay safe; one set per concurrently running encoder).
 * scgib_gin_layer_fwd_bn = scgib_gin_layer_fwd + scgib_bn_finalize(training);
 * running_mean/var/num_batches_tracked may be NULL (track_running_stats off).
 * scgib_gin_bwd_stats_bn = scgib_gin_bwd_stats + scgib_bn_bwd_finalize. */
int64_t scgib_gin_bn_ws_floats(int64_t n_nodes);
int64_t scgib_gin_counters(int64_t n_nodes);

int scgib_gin_layer_fwd_bn(const float *h_in, int32_t d_in, const float *in_stat,
                           const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                           float one_plus_eps, const float *w1, const float *b1, const float *w2,
                           const float *b2, float *agg, float *r, float *z2, const float *gamma,
                           const float *beta, float bn_eps, float momentum, float *running_mean,
                           float *running_var, int64_t *num_batches_tracked, float *stat,
                           float *bn_ws, uint32_t *counters, const int32_t *dims,
                           const scgib_bn_pending *in_pending, int32_t defer,
                           scgib_stream_t stream);
int scgib_gin_bwd_stats_bn(const float *dh, const int32_t *rowptr_t, const int32_t *col_t,
                           float one_plus_eps, const float *z2, const float *stat,
                           int64_t n_nodes, int32_t training, float *dy, float *dgamma,
                           float *dbeta, float *coef, float *bn_ws, uint32_t *counters,
                           const int32_t *dims, int32_t defer, scgib_stream_t stream);
/* scgib_gin_bwd_stats_bn for an encoder output read by a segment-sum readout
 * (dgl.sum_nodes of the ego-net features, models.py:724-726): dh[v] =
 * (dh ? dh[v] : 0) + g_seg[seg[v]] (dh may be NULL), i.e. the readout's
 * backward broadcast is folded in; seg from scgib_bn_relu_segment_sum. */
int scgib_gin_bwd_stats_seg_bn(const float *dh, const float *g_seg, const int32_t *seg,
                               const float *z2, const float *stat, int64_t n_nodes,
                               int32_t training, float *dy, float *dgamma, float *dbeta,
                               float *coef, float *bn_ws, uint32_t *counters,
                               const int32_t *dims, int32_t defer, scgib_stream_t stream);
/* Encoder output and its readout in one pass: out = relu(stat.scale z +
 * stat.shift) [n_rows][64], readout[s] = sum of out rows [ptr[s], ptr[s+1])
 * (same order as scgib_segment_sum), seg[row] = s.  seg_dims (device, may be
 * NULL): actual segment count; rows past the last valid one are zeroed.
 * in_pending / dims (row count, may be NULL): as scgib_bn_relu_apply. */
int scgib_bn_relu_segment_sum(const float *z, const float *stat, const int32_t *ptr,
                              int64_t n_seg, int64_t n_rows, float *out, float *readout,
                              int32_t *seg, const int32_t *seg_dims, const int32_t *dims,
                              const scgib_bn_pending *in_pending, scgib_stream_t stream);
/* Deferred finalize (scgib_bn_pending above): in_pending (NULL: in_stat is
 * used) names the previous layer's pending statistics — this layer finishes
 * them; defer = 1 leaves this layer's own pending (stat / running stats /
 * dgamma, dbeta, coef are then written by the consumer). */
int64_t scgib_gin_bn_gpart_offset(int64_t n_nodes);
int64_t scgib_gin_defer_max_nodes(void);
/* Layer 0 with transfer_d folded in (models.py:668-669 / :1164-1165:
 * h0 = x Wt^T, Wt = transfer_d.weight [32][F], F <= 16): the kernel gathers
 * the raw rows x[node_map[v]] (node_map NULL = identity; ego batches pass
 * the ego -> parent map, so x_subs is never built), aggx = ope x + sum_u x
 * ([n][16] zero-padded, saved) and agg = aggx Wt^T ([n][32], saved), then the
 * usual layer.  counters NULL: BN not fused (bn_ws then holds the tile
 * statistics for scgib_bn_finalize).  Backward: one slab per workgroup of
 * scgib_gin_layer0_slab_width() floats = dW2 | dW1[64*32] | db2 | db1 |
 * dWt[32][n_feat] row-major in the first 32*n_feat floats of a 512-float
 * region (the rest is not written); d(agg0) is not produced. */
int64_t scgib_gin_layer0_slab_width(void);
int scgib_gin_layer0_fwd(const float *x, int32_t n_feat, const int32_t *node_map, const float *wt,
                         const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                         float one_plus_eps, const float *w1, const float *b1, const float *w2,
                         const float *b2, float *agg, float *aggx, float *r, float *z2,
                         const float *gamma, const float *beta, float bn_eps, float momentum,
                         float *running_mean, float *running_var, int64_t *num_batches_tracked,
                         float *stat, float *bn_ws, uint32_t *counters, const int32_t *dims,
                         int32_t defer, scgib_stream_t stream);
/* scgib_gin_bwd_stats_bn with a weight-gradient slab reduce folded in
 * (`fold` NULL: none): extra workgroups past the tile grid compute
 * fold->out[w] = sum_s fold->slab[s*stride + w] (fixed order, as
 * scgib_slab_reduce_multi's job) — the previous layer's reduce runs in the
 * bandwidth the gather-bound statistics tiles leave idle. */
int scgib_gin_bwd_stats_bn_fold(const float *dh, const int32_t *rowptr_t, const int32_t *col_t,
                                float one_plus_eps, const float *z2, const float *stat,
                                int64_t n_nodes, int32_t training, float *dy, float *dgamma,
                                float *dbeta, float *coef, float *bn_ws, uint32_t *counters,
                                const int32_t *dims, int32_t defer, const scgib_slab_job *fold,
                                scgib_stream_t stream);
/* layer backward: `pending` (NULL: coef is read) finishes the deferred
 * scgib_gin_bwd_stats_bn of the same layer (coef may then be NULL). */
/* need_w = 0: the layer's W1 / b1 / W2 / b2 take no gradient (frozen: the
 * fine-tune freezing quirk, models.py:424-434) — only d(agg) (layer 0: dWt)
 * is formed, by the same chains (bitwise the need_w = 1 values); the dW
 * products and slabs are skipped (layer 0: only its dWt slab part is
 * written; agg may then be NULL; r must be given). */
int scgib_gin_layer0_bwd(const float *dy, const float *z2, const float *r, const float *agg,
                         const float *aggx, int32_t n_feat, const float *stat,
                         const float *coef, const float *w1, const float *b1, const float *w2,
                         int64_t n_nodes, float *slab, int32_t need_w, const int32_t *dims,
                         const scgib_bn_bwd_pending *pending, scgib_stream_t stream);
int scgib_gin_layer_bwd(const float *dy, const float *z2, const float *r, const float *agg,
                        int32_t d_in, const float *stat, const float *coef, const float *w1,
                        const float *b1, const float *w2, int64_t n_nodes, float *dagg,
                        float *slab, float *wgrad, int32_t need_w, const int32_t *dims,
                        const scgib_bn_bwd_pending *pending, scgib_stream_t stream);
int scgib_gin_hidden(const float *agg, int32_t d_in, const float *w1, const float *b1,
                     int64_t n_nodes, float *r, scgib_stream_t stream);
/* ---- A5: the agg-free backward of a d_in = 64 layer l >= 1 (ABI 20) ----
 * Replaces the agg half of DGL GINConv's backward (models.py:63-71, the
 * GINConv(MLP) + BatchNorm1d of GIN.forward): for a symmetric molecule graph
 * dW1 = dz1^T agg = g^T h_{l-1} and d h_{l-1} = g W1 with g = (I + A)^T dz1,
 * so the forward stores no agg for such a layer (scgib_gin_layer_fwd[_bn]
 * with agg NULL) and:
 *   scgib_gin_layer_bwd_z   dz2 (BN backward) -> dW2 += dz2^T r, dr = dz2 W2,
 *                           dz1 = dr [r > 0] written to dz1 [n][64]; one slab
 *                           per workgroup: dW2 [64][64] | db2 [64] | db1 [64]
 *                           (scgib_gin_layer_bwd_z_width floats; count
 *                           scgib_gin_layer_bwd_z_slabs); `fold`, `fold2`
 *                           (or NULL): slab jobs reduced in extra workgroups
 *                           (fold: 32 columns x 8 slab partitions each, for
 *                           the previous statistics launch's many dW1
 *                           partials; fold2: as scgib_gin_bwd_stats_bn_fold's);
 *   scgib_gin_bwd_stats_z   layer l-1's statistics from dz1 of layer l:
 *                           g gathered over the transposed CSR (one_plus_eps
 *                           of layer l), dh = g W1 (W1 of layer l), dy = dh
 *                           [scale z2 + shift > 0], BN sums as
 *                           scgib_gin_bwd_stats_bn_fold; dW1 of layer l as
 *                           one [64][64] partial per workgroup in wslab
 *                           (scgib_gin_bwd_stats_z_slabs of them); up to two
 *                           fold jobs reduced in extra workgroups.
 * need_w = 0 (a frozen layer l, resp. l + 1 for the statistics): the same
 * data chains (bitwise the need_w = 1 dz1 / dy), no weight products, no
 * slab (slab / wslab may be NULL).  Results equal the stored-agg path to
 * fp32 rounding (different association of the same sums), deterministic run
 * to run. */
int64_t scgib_gin_layer_bwd_z_slabs(int64_t n_nodes);
int64_t scgib_gin_layer_bwd_z_width(void);
int scgib_gin_layer_bwd_z(const float *dy, const float *z2, const float *r, const float *stat,
                          const float *coef, const float *w2, int64_t n_nodes, float *dz1,
                          float *slab, int32_t need_w, const int32_t *dims,
                          const scgib_bn_bwd_pending *pending, const scgib_slab_job *fold,
                          const scgib_slab_job *fold2, scgib_stream_t stream);
int64_t scgib_gin_bwd_stats_z_slabs(int64_t n_nodes);
int scgib_gin_bwd_stats_z(const float *dz1, const int32_t *rowptr_t, const int32_t *col_t,
                          float one_plus_eps, const float *w1, const float *z2, const float *stat,
                          int64_t n_nodes, int32_t training, float *dy, float *dgamma,
                          float *dbeta, float *coef, float *bn_ws, uint32_t *counters,
                          const int32_t *dims, int32_t defer, float *wslab, int32_t need_w,
                          const scgib_slab_job *fold, int32_t n_fold, scgib_stream_t stream);

/* ---- (f)1/(f)4: Set2Set readout (DGL Set2Set(dim, n_iters, 1), models.py:565) ----
 * The whole readout as Mainmodel_finetuning.forward (models.py:515) and
 * Mainmodel_domainadapt (:271-272) run it, all n_iters rounds in one launch:
 * for graph g (rows [graph_ptr[g], graph_ptr[g+1]) of x [*][dim], dim <= 64),
 * from h = c = 0, q* = 0:
 *   gates = W_ih q* + b_ih + W_hh h + b_hh  (w_ih [4 dim][2 dim], w_hh [4 dim][dim],
 *           PyTorch LSTM gate order i, f, g, o);  c = sig(f) c + sig(i) tanh(g);
 *   h = sig(o) tanh(c);  e_v = <x_v, h>;  alpha = softmax_g(e);  r = sum_v alpha_v x_v;
 *   q* = [h, r];   out [n_graphs][2 dim] = the last q*.
 * save [scgib_set2set_save_floats]: the per-round state the backward reads.
 * Backward: d out -> dx (rows past graph_ptr[n_graphs], up to n_rows:
 * capacity padding, zeroed), dw_ih, dw_hh, db_ih = db_hh; dgates
 * [n_graphs * n_iters * 4 dim] is scratch.  No host sync: graph-capturable.
 * With dw_ih, dw_hh, db_ih and db_hh all NULL, scgib_set2set_bwd writes dx and
 * dgates only, and scgib_set2set_wgrad (the same save / dgates) forms the
 * weight gradients later — the fine-tune step runs it off the critical
 * chain (ops.SlabScope). */
int64_t scgib_set2set_save_floats(int64_t n_graphs, int32_t dim, int32_t n_iters);
int scgib_set2set_fwd(const float *x, const int32_t *graph_ptr, int64_t n_graphs, int32_t dim,
                      int32_t n_iters, const float *w_ih, const float *b_ih, const float *w_hh,
                      const float *b_hh, float *save, float *out, scgib_stream_t stream);
int scgib_set2set_bwd(const float *x, const int32_t *graph_ptr, int64_t n_graphs, int32_t dim,
                      int32_t n_iters, const float *w_ih, const float *w_hh, const float *save,
                      const float *g_out, float *dx, int64_t n_rows, float *dgates,
                      float *dw_ih, float *dw_hh, float *db_ih, float *db_hh,
                      scgib_stream_t stream);
int scgib_set2set_wgrad(const float *save, const float *dgates, int64_t n_graphs, int32_t dim,
                        int32_t n_iters, float *dw_ih, float *dw_hh, float *db_ih, float *db_hh,
                        scgib_stream_t stream);

/* ---- A6: per-segment readouts (dgl.sum_nodes) -------------------------------
 * out[s,:] = sum_{i in [ptr[s], ptr[s+1])} x[i,:]   (models.py:716, 725, 733)
 * segment_broadcast is its adjoint: out[i,:] = g[s,:] for every row i of s.
 * dim: any >= 1 (float4 lanes when dim is 4 x a power of two <= 256, else a
 * scalar kernel, e.g. for raw node features). */
int scgib_segment_sum(const float *x, const int32_t *ptr, int64_t n_seg, int32_t dim,
                      float *out, const int32_t *dims, scgib_stream_t stream);
/* n_rows: rows of `out` (rows past ptr[actual n_seg] are zeroed in capacity mode) */
int scgib_segment_broadcast(const float *g, const int32_t *ptr, int64_t n_seg, int32_t dim,
                            float *out, int64_t n_rows, const int32_t *dims,
                            scgib_stream_t stream);

/* ---- A2: k-hop ego-net builder (dgl.khop_in_subgraph for every node) -------
 * Replaces the per-node Python loop of exp_pretraining.py:269-272 (+ the
 * per-step dgl.batch of the ego-nets, exp_pretraining.py:308-309).
 * Graph: dst-major CSR (rowptr/col) of a batch of graphs whose node ranges are
 * [graph_ptr[g], graph_ptr[g+1]); edges must stay inside their graph, column
 * lists sorted ascending, the graph symmetric (to_bidirected output).
 * max_graph_nodes <= 512.
 *
 * Step 1, scgib_egonet_count: fills ego_ptr[0..n] and ego_eptr[0..n] with the
 * exclusive prefix sums of the ego-net node / edge counts (ego_ptr[n] = N_s,
 * ego_eptr[n] = E_s).  `workspace` holds scgib_egonet_workspace_bytes(n).
 * err (device int32, zeroed by the caller) becomes non-zero if an edge leaves
 * its graph or a graph exceeds max_graph_nodes.
 * Step 2, scgib_egonet_fill: writes, for the batched ego graph (ego j <-> node j,
 * ego nodes sorted ascending, DGL node_subgraph edge order):
 *   ego_nodes[N_s]   parent node id of every ego node (DGL's ndata['_ID'] + offset)
 *   sub_rowptr[N_s+1], sub_col[E_s]  dst-major CSR in ego-batch node ids.
 * n_ego_cap = length of ego_nodes (>= N_s): entries [N_s, n_ego_cap) get
 * parent id 0 and empty CSR rows.  ego_dims (nullable, device int32[2])
 * receives [N_s, E_s] (the ego batch's `dims` in capacity mode). */
int64_t scgib_egonet_workspace_bytes(int64_t n_nodes);
int scgib_egonet_count(const int32_t *rowptr, const int32_t *col, const int32_t *graph_ptr,
                       int64_t n_graphs, int64_t n_nodes, int32_t k, int32_t max_graph_nodes,
                       int32_t *ego_ptr, int32_t *ego_eptr, void *workspace, int32_t *err,
                       const int32_t *dims, scgib_stream_t stream);
/* k = 1 fast path, both passes in two launches: ball(v) = {v} u N(v) as a
 * 128-bit window bitmap centred on v (no molecule bitmap, no graph_ptr
 * search), batched loads; same outputs as scgib_egonet_count +
 * scgib_egonet_fill (ego_ptr, ego_eptr exclusive scans; ego_nodes;
 * sub_rowptr/sub_col in DGL order; ego_dims).  Requires every in-degree <=
 * scgib_egonet_k1_max_degree(), molecules <= scgib_egonet_k1_max_graph_nodes()
 * atoms and edges inside their molecule (the caller checks them on the host).
 * workspace: scgib_egonet_workspace_bytes(n). */
int64_t scgib_egonet_k1_max_degree(void);
int64_t scgib_egonet_k1_max_graph_nodes(void);
int scgib_egonet_k1_build(const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                          int32_t *ego_ptr, int32_t *ego_eptr, void *workspace,
                          int32_t *ego_nodes, int32_t *sub_rowptr, int32_t *sub_col,
                          int64_t n_ego_cap, const int32_t *dims, int32_t *ego_dims,
                          scgib_stream_t stream);
/* The same with the batch's max in-degree (<= scgib_egonet_k1_max_degree()):
 * <= 6 runs the kernels built for balls of <= 7 members (one load group,
 * half the neighbour slots of the general form). */
int scgib_egonet_k1_build_deg(const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                              int32_t max_in_degree, int32_t *ego_ptr, int32_t *ego_eptr,
                              void *workspace, int32_t *ego_nodes, int32_t *sub_rowptr,
                              int32_t *sub_col, int64_t n_ego_cap, const int32_t *dims,
                              int32_t *ego_dims, scgib_stream_t stream);
/* The same in ONE launch: each block of 64 parents takes its offsets by a
 * decoupled look-back over the preceding blocks instead of a second launch.
 * scan_state: scgib_egonet_k1_scan_words(n) ZEROED uint32 words, 4-byte
 * aligned, left zeroed by the launch (reusable by the next one; one launch in
 * flight per scan_state).  Output identical to scgib_egonet_k1_build_deg.
 * e_cap: sub_col's capacity; a ball that would write past n_ego_cap rows or
 * e_cap columns is dropped and ORs the flag value 4 (bit 2; flags 1 and 2
 * as above) into *err (err may be NULL). */
int64_t scgib_egonet_k1_scan_words(int64_t n_nodes);
int scgib_egonet_k1_build_onepass(const int32_t *rowptr, const int32_t *col, int64_t n_nodes,
                                  int32_t max_in_degree, int32_t *ego_ptr, int32_t *ego_eptr,
                                  uint32_t *scan_state, int32_t *ego_nodes, int32_t *sub_rowptr,
                                  int32_t *sub_col, int64_t n_ego_cap, int64_t e_cap,
                                  int32_t *err, const int32_t *dims, int32_t *ego_dims,
                                  scgib_stream_t stream);
/* scgib_egonet_count / scgib_egonet_fill (any k) over the resident pool's
 * batch srcs[ctr[0] % n_src] (rowptr / col / graph_ptr / dims at byte offsets
 * of each graph.StaticBatch blob, capacity mode; n_nodes = the capacity),
 * resolved on the device when each kernel starts (graph.EgoPrefetch, k >= 2). */
int scgib_egonet_count_pool(const uint64_t *srcs, int32_t n_src, const uint32_t *ctr,
                            int64_t o_rowptr, int64_t o_col, int64_t o_gptr, int64_t o_dims,
                            int64_t n_graphs, int64_t n_nodes, int32_t k, int32_t max_graph_nodes,
                            int32_t *ego_ptr, int32_t *ego_eptr, void *workspace, int32_t *err,
                            scgib_stream_t stream);
int scgib_egonet_fill_pool(const uint64_t *srcs, int32_t n_src, const uint32_t *ctr,
                           int64_t o_rowptr, int64_t o_col, int64_t o_gptr, int64_t o_dims,
                           int64_t n_graphs, int64_t n_nodes, int32_t k, int32_t max_graph_nodes,
                           const int32_t *ego_ptr, const int32_t *ego_eptr, int32_t *ego_nodes,
                           int32_t *sub_rowptr, int32_t *sub_col, int32_t *err,
                           int64_t n_ego_cap, int32_t *ego_dims, scgib_stream_t stream);
/* The one-launch k = 1 build over the resident pool's batch srcs[ctr[0] % n_src]
 * (srcs, ctr as in scgib_pool_copy; rowptr / col / dims at byte offsets
 * o_rowptr / o_col / o_dims of each pool blob, capacity mode), resolved on
 * the device when the kernel starts: the ego-nets of the batch the next
 * replayed step loads, built inside the current step (graph.EgoPrefetch;
 * replaces the in-step dgl.khop_in_subgraph pass, exp_pretraining.py:269-272). */
int scgib_egonet_k1_build_onepass_pool(const uint64_t *srcs, int32_t n_src, const uint32_t *ctr,
                                       int64_t o_rowptr, int64_t o_col, int64_t o_dims,
                                       int64_t n_nodes, int32_t max_in_degree, int32_t *ego_ptr,
                                       int32_t *ego_eptr, uint32_t *scan_state,
                                       int32_t *ego_nodes, int32_t *sub_rowptr, int32_t *sub_col,
                                       int64_t n_ego_cap, int64_t e_cap, int32_t *err,
                                       int32_t *ego_dims, scgib_stream_t stream);
int scgib_egonet_fill(const int32_t *rowptr, const int32_t *col, const int32_t *graph_ptr,
                      int64_t n_graphs, int64_t n_nodes, int32_t k, int32_t max_graph_nodes,
                      const int32_t *ego_ptr, const int32_t *ego_eptr, int32_t *ego_nodes,
                      int32_t *sub_rowptr, int32_t *sub_col, int32_t *err, int64_t n_ego_cap,
                      const int32_t *dims, int32_t *ego_dims, scgib_stream_t stream);

/* ---- A6-A8 + A10/A11 inputs: core <-> subgraph interaction, fused ----------
 * One wavefront per molecule.  Restates, per graph i (models.py:595-604,
 * 631-660, 714-749):
 *   z2[i]   = sum_nodes(f)                                  (graph readout)
 *   p       = W2 . relu(BN_i(t)) + b2   with t = f W1^T + b1 given, BN_i the
 *             compressor BatchNorm over graph i's rows (train) or running
 *             stats (eval)
 *   lambda  = sigmoid(log(e) - log(1-e) + p),  e = 0.9999 - 0.9998 * u_gate
 *   (sigma, mu) = std_mean(f_i) (unbiased), noisy = lambda f + (1-lambda) mu
 *             + u_feat (1-lambda) sigma                    -> im[:, 0:64]
 *   z1[i]   = sum_nodes(noisy)
 *   logit_v = w_att[0:64].z1[i] + w_att[64:128].s_v + b_att, alpha = softmax_i
 *   im[:, 64:128] = alpha * s
 *   kl_tensor[2*n_last, 64]: the last graph's KL term, twice (models.py:659)
 * kl_mean (scalar) = mean(kl_tensor); either output may be NULL (not both).
 * pad_rows != 0: n_nodes is a row capacity and rows [graph_ptr[B], n_nodes)
 * of im, lam, logit are zeroed (capacity mode; B stays exact).
 * Saved for backward: lam[N], logit[N] (= w_att[64:128].s_v: the per-graph
 * z-bar term cancels in the softmax, so it is kept out of the saved logits and
 * their max/sum), stats[B, SCGIB_STATS_STRIDE].
 * Scalars b2, b_att are device pointers (no host sync). */
int scgib_interaction_fwd(const float *f, const float *t, const float *s,
                          const float *u_gate, const float *u_feat, const int32_t *graph_ptr,
                          int64_t n_graphs, int64_t n_nodes, const float *bn_gamma,
                          const float *bn_beta, const float *bn_running_mean,
                          const float *bn_running_var, float bn_eps, int32_t training,
                          const float *w2, const float *b2, const float *w_att,
                          const float *b_att, float *im, float *z1, float *z2, float *lam,
                          float *logit, float *stats, float *kl_tensor, float *kl_mean,
                          int32_t pad_rows, scgib_stream_t stream);

/* Device noise for the interaction (replaces the reference's torch.rand gate
 * draw u [n,1], models.py:599, and feature draw u [n,64], :650, when no noise
 * is given): counter-based Philox4x32-10 uniforms in [0, 1) keyed by
 * rng_state[0] (seed) and rng_state[1] (offset; uint64, device) -> u_gate
 * [n_rows], u_feat [n_rows][64], passed to scgib_interaction_fwd as noise.
 * The last workgroup advances rng_state[1] by one, so every launch / graph
 * replay draws fresh noise.  counter: one zeroed uint32, left zero. */
int scgib_noise_uniform(float *u_gate, float *u_feat, int64_t n_rows, uint64_t *rng_state,
                        uint32_t *counter, scgib_stream_t stream);

/* Sequential running-stat update of the per-graph compressor BatchNorm: one
 * nn.BatchNorm1d call per graph in graph order (models.py:642 inside the loop
 * of :639), i.e. B momentum updates with each graph's mean and unbiased var,
 * and num_batches_tracked += B. */
int scgib_bn_running_update(const float *stats, const int32_t *graph_ptr, int64_t n_graphs,
                            float momentum, float *running_mean, float *running_var,
                            int64_t *num_batches_tracked, scgib_stream_t stream);
/* The same update as an argument block, for launches that run it in an
 * extra workgroup beside their own work (scgib_mlp2_recon_contrastive_fwd). */
typedef struct {
    const float *stats;           /* scgib_interaction_fwd's per-graph statistics */
    const int32_t *graph_ptr;
    int64_t n_graphs;
    float momentum;
    float *running_mean, *running_var;
    int64_t *num_batches_tracked;
} scgib_running_update;

/* ---- (f)1: fine-tune prediction head + BCE (models.py:510-523) ------------
 * scgib_head_fwd: hid = relu(x W1^T + b1) [n,64] (saved), out = hid W2^T + b2
 *   [n,C], sigmoid applied when `sigmoid` (the reference's scores unless the
 *   dataset is a regression one, models.py:517-520); x [n,K], K <= 128 and a
 *   multiple of 4, C <= 16; x and w1 16-byte aligned (else SCGIB_EUNSUPPORTED).
 *   ru (may be NULL): the compressor BatchNorm's running update
 *   (scgib_running_update, below), run in one extra workgroup of the launch —
 *   nothing in the fine-tune step reads the running statistics, so it needs no
 *   launch of its own.
 * scgib_head_bwd: from d_out [n,C] (and out = the sigmoid output when
 *   `sigmoid`): dx [n,K], dW1 [64][K], db1 [64], dW2 [C][64], db2 [C]; four
 *   workgroups (dW1 row quarters, dx column quarters), each output summed in a
 *   fixed order.
 * scgib_bce_fwd / _bwd: F.binary_cross_entropy(scores, targets), mean over n
 *   elements (torch's per-element formula and log clamp at -100; fp64 fixed
 *   order sum), and d scores = g (s - t) / max((1 - s) s, 1e-12) / n with g the
 *   device scalar d loss (models.py:522-523). */
int scgib_head_fwd(const float *x, int64_t n_rows, int32_t k_in, const float *w1, const float *b1,
                   const float *w2, const float *b2, int32_t n_out, int32_t sigmoid, float *hid,
                   float *out, const scgib_running_update *ru, scgib_stream_t stream);
int scgib_head_bwd(const float *x, const float *hid, const float *out, const float *d_out,
                   int64_t n_rows, int32_t k_in, const float *w1, const float *w2, int32_t n_out,
                   int32_t sigmoid, float *dx, float *dw1, float *db1, float *dw2, float *db2,
                   scgib_stream_t stream);
int scgib_bce_fwd(const float *scores, const float *targets, int64_t n, float *loss,
                  scgib_stream_t stream);
int scgib_bce_bwd(const float *scores, const float *targets, int64_t n, const float *g_loss,
                  float *d_scores, scgib_stream_t stream);
/* Backward of scgib_interaction_fwd.  The KL gradient is g_kl [2 n_last, 64],
 * or g_klmean (device scalar, gradient of kl_mean), or neither (both NULL);
 * g_z1 / g_z2 may be NULL (readouts that feed no loss: zero gradient).
 * pad_rows: zero rows [graph_ptr[B], n_nodes) of df, dt, ds.
 * Outputs df, dt, ds [N,64] and per-graph parameter-gradient partials
 * pgrad[B, SCGIB_PGRAD_STRIDE] laid out as
 *   [0,64) dW2 | 64 db2 | [65,129) dgamma | [129,193) dbeta |
 *   [193,321) dW_att | 321 db_att
 * If pgrad_total (SCGIB_PGRAD_STRIDE floats) is given, the fixed-order sum
 * over graphs (the parameter gradients) is written there as well. */
int scgib_interaction_bwd(const float *g_im, const float *g_z1, const float *g_z2,
                          const float *g_kl, const float *f, const float *t, const float *s,
                          const float *u_feat, const int32_t *graph_ptr, int64_t n_graphs,
                          int64_t n_nodes, const float *bn_gamma, const float *bn_beta,
                          const float *bn_running_mean, const float *bn_running_var,
                          float bn_eps, int32_t training, const float *w2,
                          const float *w_att, const float *z1, const float *lam,
                          const float *logit, const float *stats, float *df, float *dt,
                          float *ds, float *pgrad, const float *g_klmean, int32_t pad_rows,
                          float *pgrad_total, scgib_stream_t stream);

/* ---- A12: adjacency reconstruction loss, Gram form ------------------------
 * loss = sum_{u,v} (<im_u, im_v> - A_uv)^2 / N
 *      = (||IM^T IM||_F^2 - 2 sum_{(u,v) in E} <im_u, im_v> + |E|) / N
 * exactly (A 0/1, simple graph) — replaces the dense N x N form of
 * loss_recon_adj (models.py:762-768).  Two launches: partial Gram slabs
 * (MFMA f32 32x32x2) + edge dot products, then a fixed-order fp64 finalize.
 * `partials` holds scgib_recon_partials_floats(n) floats.
 * Outputs: gram[64*64] (for backward) and loss[1]. */
int64_t scgib_recon_partials_floats(int64_t n_nodes);
int scgib_recon_fwd(const float *im, const int32_t *rowptr, const int32_t *col,
                    int64_t n_nodes, int64_t n_edges, float *partials, float *gram,
                    float *loss, const int32_t *dims, scgib_stream_t stream);
/* d loss / d im = (g_loss / N) * (4 IM G - 2 (A + A^T) IM); pass the in-CSR and
 * the out-CSR (the same arrays for a symmetric graph).  g_loss is a device
 * scalar. */
int scgib_recon_bwd(const float *im, const float *gram, const int32_t *rowptr_in,
                    const int32_t *col_in, const int32_t *rowptr_out, const int32_t *col_out,
                    int64_t n_nodes, const float *g_loss, float *grad_im,
                    const int32_t *dims, scgib_stream_t stream);

/* ---- A15: logM reconstruction loss (models.py:770-782) --------------------
 * loss = (1/k) sum_g sum_i ||X_g X_g^T - logM_g,i||_F^2 / n_g^2, X_g = the rows
 * of `im` [N][64] of molecule g (graph_ptr).  Targets per molecule, packed at
 * int64 s_offsets[B+1] (n_g^2 floats each): S = sum_i logM_i, and
 * C[g] = sum_i ||logM_i||^2 (fp64).  loss_graphs [B] holds per-molecule terms;
 * loss is a device scalar (fixed-order sum).  Backward: grad_im [N][64] =
 * 2 g_loss (2k X X^T - S - S^T) X / (k n_g^2) per molecule. */
int scgib_recon_logm_fwd(const float *im, const int32_t *graph_ptr, int64_t n_graphs,
                         const float *S, const int64_t *s_offsets, const double *C,
                         int32_t kstep, float *loss_graphs, float *loss, scgib_stream_t stream);
int scgib_recon_logm_bwd(const float *im, const int32_t *graph_ptr, int64_t n_graphs,
                         const float *S, const int64_t *s_offsets, int32_t kstep,
                         const float *g_loss, float *grad_im, scgib_stream_t stream);

/* ---- A11: contrastive loss (batched_semi_loss, tau = 1) --------------------
 * models.py:606-629 (sim :606-609, semi_loss :611-616, batched :618-629;
 * called at models.py:695 with z1 = sum_nodes(noisy), z2 = graph readout).
 * loss = mean_i -log(exp(z1n_i.z2n_i) / (sum_j exp(z1n_i.z1n_j)
 *        + sum_j exp(z1n_i.z2n_j) - exp(z1n_i.z1n_i))),  zn = F.normalize(z).
 * The value is independent of the reference's chunk size.  z1, z2: [B][64].
 * `workspace` holds scgib_contrastive_workspace_floats(B) floats and must be
 * passed unchanged from forward to backward.  `counters` holds
 * scgib_contrastive_counters(B) uint32 that are zero on entry; both launches
 * leave them zero (graph-replay safe).  loss and g_loss are device scalars. */
int64_t scgib_contrastive_workspace_floats(int64_t n_graphs);
int64_t scgib_contrastive_counters(int64_t n_graphs);
int scgib_contrastive_fwd(const float *z1, const float *z2, int64_t n_graphs, float *workspace,
                          float *loss, uint32_t *counters, scgib_stream_t stream);
int scgib_contrastive_bwd(const float *z1, const float *z2, int64_t n_graphs, float *workspace,
                          const float *g_loss, float *dz1, float *dz2, uint32_t *counters,
                          scgib_stream_t stream);

/* ---- A10 head: fused dense layers (exact-f32 MFMA tiles) -----------------
 * mlp2: out = relu(x W1^T + b1) W2^T + b2, x [N][d_in] (d_in 64 or 128),
 * W1 [64][d_in], W2 [64][64] — the interaction-map MLP of Mainmodel /
 * Mainmodel_continue (models.py:569-571 / :1055-1057, applied at :676 /
 * :1174).  Forward saves r = relu(x W1^T + b1) [N][64] for backward.
 * Backward: dx [N][d_in] and wgrad = dW2[64*64] | dW1[64*d_in] | db2 | db1
 * (fixed-order, deterministic); `slab` holds scgib_mlp2_slab_floats(n, d_in)
 * (d_in = 128 on few tiles: two workgroups, two slab rows, per tile — ABI 19);
 * wgrad NULL: the slabs are left for the caller's reduce (a deferred one).
 * linear: out = x W^T (+ b), 64 -> 64 — compressor[0] (models.py:589-592 /
 * :1081-1084, applied at :596 / :1092).  Backward writes dx = add + dy W
 * (`add` may be NULL) and wgrad = dW[64*64] | db[64]; `slab` holds
 * scgib_linear_slab_floats(n).  Capacity mode as above (dims). */
int64_t scgib_mlp2_slab_floats(int64_t n_nodes, int32_t d_in);
int64_t scgib_mlp2_recon_slab_floats(int64_t n_nodes, int32_t d_in);
int scgib_mlp2_fwd(const float *x, int32_t d_in, int64_t n_nodes, const float *w1,
                   const float *b1, const float *w2, const float *b2, float *r, float *out,
                   const int32_t *dims, scgib_stream_t stream);
int scgib_mlp2_bwd(const float *dout, const float *x, const float *r, int32_t d_in,
                   const float *w1, const float *w2, int64_t n_nodes, float *dx, float *slab,
                   float *wgrad, const int32_t *dims, scgib_stream_t stream);
/* mlp2 + recon (fused): the interaction-map MLP followed by loss_recon_adj
 * on its output (models.py:1174 then :1256-1262, i.e. Mainmodel_continue's
 * forward with recons_type 'adj'; replaces scgib_mlp2_fwd + scgib_recon_fwd
 * and their backward).  Forward: out (= IM), r, and loss; `ws` holds
 * scgib_mlp2_recon_ws_floats(n) floats (per-tile Gram partials, G, loss
 * partials) and must be passed unchanged to the backward; `counter` is three
 * zeroed uint32, left zero; `fault` (or NULL) is scgib_stream_wait's sticky
 * hand-off fault word: while it is set, *loss is NaN.  When the launch's workgroups are all co-resident
 * the MLP tiles also finish the loss (no second launch; the same bits either
 * way).  Backward: dx = d loss / d x and wgrad as
 * scgib_mlp2_bwd, for d loss / d recon = *g_loss; rowptr_t/col_t NULL for a
 * symmetric graph (A = A^T).  wgrad NULL: the per-workgroup slabs
 * (scgib_mlp2_recon_slab_floats(n, d_in) floats, width 64*64 + 64*d_in + 128) are
 * left for the caller's scgib_slab_reduce(_multi) — the model path defers
 * them into an encoder chain's final reduce, off the loss section. */
int64_t scgib_mlp2_recon_ws_floats(int64_t n_nodes);
/* Testing hook: 0 = always finish the recon loss in its own launch; returns
 * the previous setting (default 1). */
int scgib_set_recon_fold(int on);
int scgib_mlp2_recon_fwd(const float *x, int32_t d_in, int64_t n_nodes, const float *w1,
                         const float *b1, const float *w2, const float *b2, float *r, float *out,
                         const int32_t *rowptr, const int32_t *col, int64_t n_edges, float *ws,
                         uint32_t *counter, float *loss, const int32_t *dims,
                         const uint32_t *fault, scgib_stream_t stream);
int scgib_mlp2_recon_bwd(const float *x, const float *r, const float *out, const float *ws,
                         int32_t d_in, const float *w1, const float *w2, int64_t n_nodes,
                         const int32_t *rowptr, const int32_t *col, const int32_t *rowptr_t,
                         const int32_t *col_t, const float *g_loss, float *dx, float *slab,
                         float *wgrad, const int32_t *dims, scgib_stream_t stream);
/* The same with the contrastive loss (scgib_contrastive_fwd / _bwd: z1, z2
 * [n_graphs][64], cws / ccounters as documented there) run in extra
 * workgroups of the MLP launches — one launch on the step's critical chain
 * instead of two each way.  d_in must be 128 (the pretraining head).
 * Forward also writes *closs; backward takes d loss / d contrastive =
 * *g_con and writes dz1, dz2.  ru (forward, or NULL): the compressor
 * BatchNorm's running-stat update (scgib_bn_running_update) in one more
 * workgroup of the loss-finishing launch, off the critical path without a
 * second stream. */
int scgib_mlp2_recon_contrastive_fwd(const float *x, int32_t d_in, int64_t n_nodes,
                                     const float *w1, const float *b1, const float *w2,
                                     const float *b2, float *r, float *out,
                                     const int32_t *rowptr, const int32_t *col, int64_t n_edges,
                                     float *ws, uint32_t *counter, float *loss,
                                     const int32_t *dims, const float *z1, const float *z2,
                                     int64_t n_graphs, float *cws, float *closs,
                                     uint32_t *ccounters, const scgib_running_update *ru,
                                     const uint32_t *fault, scgib_stream_t stream);
int scgib_mlp2_recon_contrastive_bwd(const float *x, const float *r, const float *out,
                                     const float *ws, int32_t d_in, const float *w1,
                                     const float *w2, int64_t n_nodes, const int32_t *rowptr,
                                     const int32_t *col, const int32_t *rowptr_t,
                                     const int32_t *col_t, const float *g_loss, float *dx,
                                     float *slab, float *wgrad, const int32_t *dims,
                                     const float *z1, const float *z2, int64_t n_graphs,
                                     float *cws, const float *g_con, float *dz1, float *dz2,
                                     uint32_t *ccounters, scgib_stream_t stream);
int64_t scgib_linear_slab_floats(int64_t n_nodes);
int scgib_linear_fwd(const float *x, int64_t n_nodes, const float *w, const float *b, float *out,
                     const int32_t *dims, scgib_stream_t stream);
/* wgrad NULL: the slabs (scgib_linear_slab_floats(n) floats, width 64*64 + 64)
 * are left for the caller's reduce. */
int scgib_linear_bwd(const float *dy, const float *x, const float *w, int64_t n_nodes,
                     const float *add, float *dx, float *slab, float *wgrad,
                     const int32_t *dims, scgib_stream_t stream);

/* ---- optimizer: one-launch Adam over a tensor list ------------------------
 * torch.optim.Adam(params, lr, betas, eps, weight_decay) as every reference
 * training script builds it (exp_pretraining.py / exp_molhiv.py:53,
 * weight_decay=5e-5; fine-tune :157 1e-5), fused-Adam arithmetic: per
 * tensor t = *step + 1, g += wd p, m = b1 m + (1-b1) g, v = b2 v + (1-b2) g^2,
 * p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps), *step = t (fp32
 * device scalar per tensor, like torch's capturable state['step']); the
 * hyper-parameters are doubles and enter the moment updates in double, as
 * in torch's fused kernel.
 * n_tensors <= scgib_adam_max_tensors(); the table is copied into the kernel
 * arguments (HIP-graph capturable).  `counter`: one uint32, zero on entry,
 * left zero. */
typedef struct {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    float *step;
    int64_t numel;
} scgib_adam_tensor;
int64_t scgib_adam_max_tensors(void);
int scgib_adam_step(const scgib_adam_tensor *tensors, int32_t n_tensors, double lr,
                    double beta1, double beta2, double eps, double weight_decay,
                    uint32_t *counter, scgib_stream_t stream);
/* scgib_slab_reduce_multi(jobs) followed by scgib_adam_step(tensors) in ONE
 * launch, with the same bits: a tensor whose gradient lies inside a job's
 * output is updated by the reduce's workgroups from the value they produce
 * (the replayed pretraining step's last weight-gradient reduce and its Adam
 * step, models.py's training loop exp_pretraining.py:321-323 — no reference
 * counterpart of its own; ABI 22).  n_jobs <= scgib_adam_reduce_max_jobs();
 * a gradient that straddles a job output's edge, or two tensors' gradients
 * overlapping inside one: SCGIB_EINVAL. */
int64_t scgib_adam_reduce_max_jobs(void);
int scgib_adam_step_reduce(const scgib_adam_tensor *tensors, int32_t n_tensors,
                           const scgib_slab_job *jobs, int32_t n_jobs, double lr, double beta1,
                           double beta2, double eps, double weight_decay, uint32_t *counter,
                           scgib_stream_t stream);


/* ---- data parallelism: gradient bucket (dist.GradAllReducer) --------------
 * scgib_grad_pack: flat[offset + i] = data[i] for every slice, one launch;
 * scgib_grad_unpack: data[i] = scale * flat[offset + i] (scale = 1/world after
 * the all-reduce SUM).  n_tensors <= scgib_grad_pack_max_tensors(); the table
 * is copied into the kernel arguments (HIP-graph capturable). */
typedef struct {
    float *data;
    int64_t numel;
    int64_t offset;
} scgib_grad_slice;
int64_t scgib_grad_pack_max_tensors(void);
int scgib_grad_pack(const scgib_grad_slice *tensors, int32_t n_tensors, float *flat,
                    scgib_stream_t stream);
int scgib_grad_unpack(const scgib_grad_slice *tensors, int32_t n_tensors, const float *flat,
                      float scale, scgib_stream_t stream);
#ifdef __cplusplus
}
#endif
#endif /* SCGIB_H */
