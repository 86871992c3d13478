// Two-lane replay of a captured step graph (ops.SplitGraph; DESIGN.md §3,
// "Host enqueue").
//
// hipGraphLaunch of a graph with parallel branches costs the host ~2.5-3 us
// per node (tools/graph_launch_probe.hip: 149 us for 48 nodes over two
// streams), while a LINEAR graph of the same nodes launches in ~6 us whatever
// its length.  The pretraining step is two chains (the encoder pair's ego and
// core chains, ops._GinEncoderPair) joined by a fork and a join edge, so it is
// rebuilt here as two linear graphs — one per chain, every kernel node copied
// with its captured launch parameters — launched on the caller's stream and on
// a side stream of the split's own.  Each cross-lane edge of the captured DAG becomes
// a signal / wait kernel pair (gather.hip: stream_signal_k, stream_wait_k, the
// encoder pair's own hand-off kernels) with its own 4-word counter slot.
//
// Ordering argument: both lanes are sub-sequences of ONE topological order of
// the captured DAG, and a wait is placed before a node only for the latest
// predecessor it has in the other lane (vector-clock pruning), so every wait
// points backwards in that order and the two in-order lanes cannot deadlock
// while both queues run.  Lane 1 always starts with a wait on a lane-0
// signal and lane 0 always ends after a wait on lane 1's last node, so a
// replay is ordered after the caller's earlier work on its stream, the
// caller's later work after the whole replay, and replay i+1 after replay i
// in both lanes — the same stream semantics as one graph launch.
//
// The two lanes must run on hardware queues the device schedules
// concurrently.  The side stream is NON-blocking (tools/lane_probe.hip: a
// blocking side stream — hipExtStreamCreateWithCUMask makes one — waits for
// the null stream's lane 0, which waits for it: every hand-off times out),
// and a new stream is assigned the least-used of the process's
// GPU_MAX_HW_QUEUES queues, which can be the caller's.  So the split checks
// once, at creation, that its side stream does not share the caller's queue:
// a wait kernel on the caller's stream followed by its signal on the side
// stream ends at once on two queues and times out behind each other on one;
// a shared stream is dropped and another one tried (up to 8).  Replays must
// then use that same caller stream (else SCGIB_EINVAL).  A wait that still
// sees no signal gives up after 0.2 s, counted in its slot and in the sticky
// fault words like the encoder pair's hand-offs (ops.xq_timeouts).
//
// Refused (SCGIB_EUNSUPPORTED, the caller replays the captured graph instead):
// non-kernel nodes (memcpy / memset / event / empty), and an in-graph
// hand-off pair (a stream_wait_k and the stream_signal_k on the same words)
// that the lane assignment would put on one lane with the wait first.
#include <algorithm>
#include <cstring>
#include <queue>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace scgib {
void handoff_kernels(const void **signal, const void **wait);  // gather.hip
}

using namespace scgib;

namespace {

struct Split {
    hipGraph_t graph[2] = {nullptr, nullptr};
    hipGraphExec_t exec[2] = {nullptr, nullptr};
    hipStream_t side = nullptr;
    hipStream_t caller = nullptr;
    int32_t info[8] = {};
};

void release(Split *s) {
    if (s->side) (void)hipStreamSynchronize(s->side);
    for (int l = 0; l < 2; ++l) {
        if (s->exec[l]) (void)hipGraphExecDestroy(s->exec[l]);
        if (s->graph[l]) (void)hipGraphDestroy(s->graph[l]);
    }
    if (s->side) (void)hipStreamDestroy(s->side);
    delete s;
}

// one lane under construction: a linear chain of kernel nodes
struct Lane {
    hipGraph_t g = nullptr;
    hipGraphNode_t tail = nullptr;
    int nodes = 0;
    hipError_t add(const hipKernelNodeParams &p) {
        hipGraphNode_t n = nullptr;
        const hipError_t e = hipGraphAddKernelNode(&n, g, tail ? &tail : nullptr, tail ? 1 : 0, &p);
        if (e == hipSuccess) {
            tail = n;
            ++nodes;
        }
        return e;
    }
};

}  // namespace

// The lane plan of a DAG of n nodes (preds[v]: v's predecessors; hidden:
// (signal, wait) node pairs ordered by hand-off words, not by edges): one
// topological order (ties by node index) with the hidden pairs as edges, each
// node on the lane whose tail is its direct predecessor (lane 0 first), and
// the cross-lane waits pruned to the latest predecessor in the other lane,
// plus the start / end hand-offs (header comment).  Host-only: tested on the
// CPU through scgib_graph_split_plan.
struct Plan {
    std::vector<int> lane, pos, wait_slot, signal_slot;
    std::vector<int> seq[2];
    int slots = 0, start_slot = -1, end_slot = -1, loose = 0;
};

static int plan_lanes(int n, const std::vector<std::vector<int>> &preds,
                      const std::vector<std::pair<int, int>> &hidden, Plan &pl) {
    // topological order, ties broken by the runtime's node order (capture order)
    std::priority_queue<int, std::vector<int>, std::greater<int>> ready;
    std::vector<std::vector<int>> after(n);
    std::vector<int> indeg(n, 0);
    for (int v = 0; v < n; ++v)
        for (int u : preds[v]) {
            after[u].push_back(v);
            ++indeg[v];
        }
    for (const auto &h : hidden) {
        after[h.first].push_back(h.second);
        ++indeg[h.second];
    }
    for (int i = 0; i < n; ++i)
        if (indeg[i] == 0) ready.push(i);
    std::vector<int> order;
    order.reserve(n);
    while (!ready.empty()) {
        const int u = ready.top();
        ready.pop();
        order.push_back(u);
        for (int v : after[u])
            if (--indeg[v] == 0) ready.push(v);
    }
    if (static_cast<int>(order.size()) != n) return SCGIB_EUNSUPPORTED;  // a hand-off against the graph's order
    // ancestor bitsets (a step graph has tens to a few hundred nodes)
    const size_t wds = (static_cast<size_t>(n) + 63) / 64;
    std::vector<uint64_t> anc(static_cast<size_t>(n) * wds, 0ull);
    for (int v : order)
        for (int u : preds[v]) {
            for (size_t w = 0; w < wds; ++w) anc[v * wds + w] |= anc[u * wds + w];
            anc[v * wds + u / 64] |= 1ull << (u % 64);
        }
    auto is_anc = [&](int u, int v) { return (anc[v * wds + u / 64] >> (u % 64)) & 1ull; };
    // lanes: follow the captured chains (a node joins the lane whose tail is
    // its direct predecessor), a fork's second child opens the other lane
    std::vector<int> &lane = pl.lane, &pos = pl.pos;
    std::vector<int> *seq = pl.seq;
    lane.assign(n, -1);
    pos.assign(n, -1);
    int &loose = pl.loose;
    loose = 0;
    std::vector<int> nsucc(n, 0);
    for (int v = 0; v < n; ++v)
        for (int u : preds[v]) ++nsucc[u];
    for (int v : order) {
        // both tails direct predecessors (a join, or a mid-capture stream
        // dependency): the tail with the fewer successors is the one whose
        // chain ends in v; the other one's stream continues past it
        int pick = -1;
        for (int l = 0; l < 2; ++l)
            if (!seq[l].empty() &&
                std::find(preds[v].begin(), preds[v].end(), seq[l].back()) != preds[v].end() &&
                (pick < 0 || nsucc[seq[l].back()] < nsucc[seq[pick].back()]))
                pick = l;
        if (pick < 0) {
            if (seq[0].empty()) pick = 0;
            else if (seq[1].empty()) pick = 1;
            else if (is_anc(seq[1].back(), v)) pick = 1;
            else if (is_anc(seq[0].back(), v)) pick = 0;
            else {
                pick = 1;  // a third concurrent chain: serialised behind lane 1
                ++loose;
            }
        }
        lane[v] = pick;
        pos[v] = static_cast<int>(seq[pick].size());
        seq[pick].push_back(v);
    }
    for (const auto &h : hidden)  // (both ends on one lane: in order by construction)
        if (lane[h.first] == lane[h.second] && pos[h.first] > pos[h.second]) return SCGIB_EUNSUPPORTED;
    // cross-lane waits, pruned to the latest predecessor in the other lane
    std::vector<int> &wait_slot = pl.wait_slot, &signal_slot = pl.signal_slot;
    wait_slot.assign(n, -1);
    signal_slot.assign(n, -1);
    int &slots = pl.slots, &start_slot = pl.start_slot, &end_slot = pl.end_slot;
    slots = 0;
    start_slot = end_slot = -1;
    for (int l = 0; l < 2; ++l) {
        int waited = -1;
        for (int v : seq[l]) {
            int need = -1;
            for (int u : preds[v])
                if (lane[u] != l) need = std::max(need, pos[u]);
            if (need > waited) {
                const int src = seq[1 - l][need];
                if (signal_slot[src] >= 0) return SCGIB_EINVAL;  // one wait per source by construction
                signal_slot[src] = wait_slot[v] = slots++;
                waited = need;
            }
        }
        if (l == 0 && !seq[1].empty() && waited < static_cast<int>(seq[1].size()) - 1)
            end_slot = slots++;  // lane 0 ends waiting for lane 1's last node
    }
    if (!seq[1].empty() && wait_slot[seq[1][0]] < 0) start_slot = slots++;
    return SCGIB_OK;
}

// words: n_slots * 4 zeroed uint32 (one slot per added hand-off, the last 8
// for the queue check; kept for the lifetime of the split); fault /
// host_fault: the encoder pair's sticky fault words (ops.handoff_fault_word /
// the pinned host word); stream: the caller's stream, the one every replay
// uses.  info (8 int32, may
// be NULL): captured nodes, lane-0 kernels, lane-1 kernels, hand-offs added,
// lane-0 nodes, lane-1 nodes, nodes placed on a lane whose tail is not among
// their ancestors (0 for a graph of two chains), slots used.
constexpr int kQueueTries = 8;

extern "C" int scgib_graph_split(void *graph, uint32_t *words, int32_t n_slots, uint32_t *fault,
                                 uint32_t *host_fault, scgib_stream_t stream, void **out,
                                 int32_t *info) {
    if (!graph || !words || n_slots < 2 + kQueueTries || !out) return SCGIB_EINVAL;
    *out = nullptr;
    hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
    size_t n = 0;
    hipError_t e = hipGraphGetNodes(g, nullptr, &n);
    if (e != hipSuccess) return static_cast<int>(e);
    if (n == 0) return SCGIB_EUNSUPPORTED;
    std::vector<hipGraphNode_t> nodes(n);
    if ((e = hipGraphGetNodes(g, nodes.data(), &n)) != hipSuccess) return static_cast<int>(e);
    std::unordered_map<hipGraphNode_t, int> index;
    std::vector<hipKernelNodeParams> params(n);
    for (size_t i = 0; i < n; ++i) {
        hipGraphNodeType t;
        if ((e = hipGraphNodeGetType(nodes[i], &t)) != hipSuccess) return static_cast<int>(e);
        if (t != hipGraphNodeTypeKernel) return SCGIB_EUNSUPPORTED;
        if ((e = hipGraphKernelNodeGetParams(nodes[i], &params[i])) != hipSuccess)
            return static_cast<int>(e);
        index[nodes[i]] = static_cast<int>(i);
    }
    size_t m = 0;
    if ((e = hipGraphGetEdges(g, nullptr, nullptr, &m)) != hipSuccess) return static_cast<int>(e);
    std::vector<hipGraphNode_t> from(m), to(m);
    if (m && (e = hipGraphGetEdges(g, from.data(), to.data(), &m)) != hipSuccess)
        return static_cast<int>(e);
    std::vector<std::vector<int>> preds(n);
    for (size_t k = 0; k < m; ++k) preds[index.at(to[k])].push_back(index.at(from[k]));
    // the encoder pair's in-graph hand-offs (a stream_signal_k and the
    // stream_wait_k on the same words): a dependency the graph does not show,
    // added to the topological order below so that it too points backwards
    const void *sig_fn = nullptr, *wait_fn = nullptr;
    handoff_kernels(&sig_fn, &wait_fn);
    std::vector<std::pair<int, int>> hidden;  // (signal, wait)
    {
        std::unordered_map<const void *, std::pair<int, int>> pairs;  // words -> (signal, wait)
        for (size_t i = 0; i < n; ++i) {
            const bool is_s = params[i].func == sig_fn, is_w = params[i].func == wait_fn;
            if (!is_s && !is_w) continue;
            if (!params[i].kernelParams) return SCGIB_EUNSUPPORTED;
            const void *wp = *reinterpret_cast<void *const *>(params[i].kernelParams[0]);
            auto it = pairs.emplace(wp, std::make_pair(-1, -1)).first;
            int &slot = is_s ? it->second.first : it->second.second;
            if (slot >= 0) return SCGIB_EUNSUPPORTED;  // two signals (waits) on one words
            slot = static_cast<int>(i);
        }
        for (const auto &kv : pairs)
            if (kv.second.first >= 0 && kv.second.second >= 0) hidden.push_back(kv.second);
    }
    Plan pl;
    const int prc = plan_lanes(static_cast<int>(n), preds, hidden, pl);
    if (prc != SCGIB_OK) return prc;
    const std::vector<int> &wait_slot = pl.wait_slot, &signal_slot = pl.signal_slot;
    const std::vector<int> *seq = pl.seq;
    const int slots = pl.slots, start_slot = pl.start_slot, end_slot = pl.end_slot, loose = pl.loose;
    if (slots > n_slots - kQueueTries) return SCGIB_EINVAL;
    // the two linear graphs
    auto handoff = [&](bool signal) {
        hipKernelNodeParams p{};
        p.func = const_cast<void *>(signal ? sig_fn : wait_fn);
        p.gridDim = dim3(1, 1, 1);
        p.blockDim = dim3(64, 1, 1);
        p.sharedMemBytes = 0;
        p.extra = nullptr;
        return p;
    };
    Split *s = new Split();
    Lane ln[2];
    auto fail = [&](hipError_t err) {
        for (int l = 0; l < 2; ++l)
            if (ln[l].g && !s->graph[l]) (void)hipGraphDestroy(ln[l].g);
        release(s);
        return static_cast<int>(err);
    };
    for (int l = 0; l < 2; ++l) {
        if (seq[l].empty()) continue;
        if ((e = hipGraphCreate(&ln[l].g, 0)) != hipSuccess) return fail(e);
        auto add_handoff = [&](bool signal, int slot) -> hipError_t {
            uint32_t *w = words + 4 * slot;
            hipKernelNodeParams p = handoff(signal);
            if (signal) {
                void *args[] = {&w};
                p.kernelParams = args;
                return ln[l].add(p);
            }
            void *args[] = {&w, &fault, &host_fault};
            p.kernelParams = args;
            return ln[l].add(p);
        };
        if (l == 0 && start_slot >= 0 && (e = add_handoff(true, start_slot)) != hipSuccess) return fail(e);
        if (l == 1 && start_slot >= 0 && (e = add_handoff(false, start_slot)) != hipSuccess) return fail(e);
        for (int v : seq[l]) {
            if (wait_slot[v] >= 0 && (e = add_handoff(false, wait_slot[v])) != hipSuccess) return fail(e);
            if ((e = ln[l].add(params[v])) != hipSuccess) return fail(e);
            if (signal_slot[v] >= 0 && (e = add_handoff(true, signal_slot[v])) != hipSuccess) return fail(e);
        }
        if (l == 0 && end_slot >= 0 && (e = add_handoff(false, end_slot)) != hipSuccess) return fail(e);
        if (l == 1 && end_slot >= 0 && (e = add_handoff(true, end_slot)) != hipSuccess) return fail(e);
        s->graph[l] = ln[l].g;
        if ((e = hipGraphInstantiate(&s->exec[l], s->graph[l], nullptr, nullptr, 0)) != hipSuccess)
            return fail(e);
    }
    s->caller = as_stream(stream);
    if (s->exec[1]) {
        // a side stream on a queue other than the caller's (header comment)
        std::vector<hipStream_t> shared;
        for (int t = 0; t < kQueueTries && !s->side; ++t) {
            hipStream_t cand = nullptr;
            if ((e = hipStreamCreateWithFlags(&cand, hipStreamNonBlocking)) != hipSuccess) break;
            uint32_t *w = words + 4 * (n_slots - kQueueTries + t);
            uint32_t *nul = nullptr;
            void *wargs[] = {&w, &nul, &nul};
            void *sargs[] = {&w};
            uint32_t late = 1;
            if ((e = hipLaunchKernel(wait_fn, dim3(1), dim3(64), wargs, 0, s->caller)) != hipSuccess ||
                (e = hipLaunchKernel(sig_fn, dim3(1), dim3(64), sargs, 0, cand)) != hipSuccess ||
                (e = hipStreamSynchronize(cand)) != hipSuccess ||
                (e = hipStreamSynchronize(s->caller)) != hipSuccess ||
                (e = hipMemcpy(&late, w + 2, sizeof(late), hipMemcpyDeviceToHost)) != hipSuccess) {
                (void)hipStreamDestroy(cand);
                break;
            }
            if (late == 0) s->side = cand;
            else shared.push_back(cand);  // kept until the search ends: the next stream goes elsewhere
        }
        for (hipStream_t c : shared) (void)hipStreamDestroy(c);
        if (e != hipSuccess) return fail(e);
        if (!s->side) {
            release(s);
            return SCGIB_EUNSUPPORTED;
        }
    }
    s->info[0] = static_cast<int32_t>(n);
    s->info[1] = static_cast<int32_t>(seq[0].size());
    s->info[2] = static_cast<int32_t>(seq[1].size());
    s->info[3] = slots;
    s->info[4] = ln[0].nodes;
    s->info[5] = ln[1].nodes;
    s->info[6] = loose;
    s->info[7] = slots;
    if (info) std::memcpy(info, s->info, sizeof(s->info));
    *out = s;
    return SCGIB_OK;
}

// One replay: lane 0 on `stream`, lane 1 on the split's own side stream.
extern "C" int scgib_graph_split_launch(void *split, scgib_stream_t stream) {
    if (!split) return SCGIB_EINVAL;
    Split *s = reinterpret_cast<Split *>(split);
    if (as_stream(stream) != s->caller) return SCGIB_EINVAL;  // the queue check was against it
    hipError_t e = hipGraphLaunch(s->exec[0], as_stream(stream));
    if (e == hipSuccess && s->exec[1]) e = hipGraphLaunch(s->exec[1], s->side);
    return e == hipSuccess ? SCGIB_OK : static_cast<int>(e);
}

// Waits for the side lane's last replay, then frees both graphs and the stream.
extern "C" int scgib_graph_split_destroy(void *split) {
    if (!split) return SCGIB_EINVAL;
    release(reinterpret_cast<Split *>(split));
    return SCGIB_OK;
}

// The lane plan alone, for tests on the host (no device needed): n nodes,
// m edges from[k] -> to[k], n_hidden signal -> wait pairs.  Outputs (n int32
// each, may be NULL): lane, position in the lane, wait slot before the node
// (-1: none), signal slot after it (-1: none); info (4 int32): slots, the
// start hand-off's slot (a signal before lane 0's first node, a wait before
// lane 1's; -1: none), the end hand-off's slot (a signal after lane 1's last
// node, a wait after lane 0's last; -1: none), nodes serialised beyond two
// chains.  Returns SCGIB_EUNSUPPORTED where scgib_graph_split would.
extern "C" int scgib_graph_split_plan(int32_t n, int32_t m, const int32_t *from, const int32_t *to,
                                      int32_t n_hidden, const int32_t *hidden_signal,
                                      const int32_t *hidden_wait, int32_t *lane, int32_t *pos,
                                      int32_t *wait_slot, int32_t *signal_slot, int32_t *info) {
    if (n < 1 || m < 0 || n_hidden < 0 || (m > 0 && (!from || !to)) ||
        (n_hidden > 0 && (!hidden_signal || !hidden_wait)))
        return SCGIB_EINVAL;
    std::vector<std::vector<int>> preds(n);
    for (int k = 0; k < m; ++k) {
        if (from[k] < 0 || from[k] >= n || to[k] < 0 || to[k] >= n) return SCGIB_EINVAL;
        preds[to[k]].push_back(from[k]);
    }
    std::vector<std::pair<int, int>> hidden;
    for (int k = 0; k < n_hidden; ++k) {
        if (hidden_signal[k] < 0 || hidden_signal[k] >= n || hidden_wait[k] < 0 || hidden_wait[k] >= n)
            return SCGIB_EINVAL;
        hidden.emplace_back(hidden_signal[k], hidden_wait[k]);
    }
    Plan pl;
    const int rc = plan_lanes(n, preds, hidden, pl);
    if (rc != SCGIB_OK) return rc;
    for (int v = 0; v < n; ++v) {
        if (lane) lane[v] = pl.lane[v];
        if (pos) pos[v] = pl.pos[v];
        if (wait_slot) wait_slot[v] = pl.wait_slot[v];
        if (signal_slot) signal_slot[v] = pl.signal_slot[v];
    }
    if (info) {
        info[0] = pl.slots;
        info[1] = pl.start_slot;
        info[2] = pl.end_slot;
        info[3] = pl.loose;
    }
    return SCGIB_OK;
}
