/* CPU restatement of per-node k-hop in-subgraph extraction (DGL 1.1
 * khop_in_subgraph), for every node of a batched graph.
 *
 * TEST INFRASTRUCTURE ONLY: the checker for the HIP ego-net builder.  Loaded
 * by tests/ and bench.py's cpu_baseline leg through ctypes, never by the
 * product path.
 *
 * Follows the reference's call site exp_pretraining.py:269-272
 * (`[dgl.khop_in_subgraph(g, v, k)[0] for v in g.nodes()]`) and DGL 1.1's
 * algorithm, restated (DGL is absent here, see oracle/dgl_semantics.py):
 *   frontier_0 = {v};  frontier_{t+1} = unique(in-neighbours(frontier_t));
 *   ball = unique(frontier_0 ∪ ... ∪ frontier_k)    (sorted ascending);
 *   edges = node_subgraph(ball): out-CSR rows visited in ball order, each
 *           row's columns in CSR order, kept when the column is in the ball,
 *           relabelled to ball positions.
 * The graph is given as CSR with row = node and sorted column lists (for the
 * bidirected simple graphs produced by to_bidirected the in- and out-CSR are
 * identical).  `unique` is restated as a visited stamp + qsort of the ball.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int cmp_i64(const void *a, const void *b) {
    int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return (x > y) - (x < y);
}

/* returns 0 on success; fills counts only when out arrays are NULL */
int egonet_ref(const int64_t *rowptr, const int64_t *col, int64_t n, int k,
               int64_t *ego_sizes, int64_t *ego_ecount,
               int64_t *ego_nodes, int64_t *ego_src, int64_t *ego_dst) {
    int64_t *stamp = (int64_t *)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
    int64_t *pos = (int64_t *)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
    int64_t *front = (int64_t *)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
    int64_t *next = (int64_t *)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
    int64_t *ball = (int64_t *)malloc(sizeof(int64_t) * (n > 0 ? n : 1));
    if (!stamp || !pos || !front || !next || !ball) return -1;
    for (int64_t i = 0; i < n; ++i) { stamp[i] = -1; pos[i] = -1; }
    int64_t node_off = 0, edge_off = 0;
    for (int64_t v = 0; v < n; ++v) {
        /* ball membership via stamp == v */
        int64_t nf = 1, nb = 0;
        front[0] = v;
        stamp[v] = v;
        for (int hop = 0; hop < k; ++hop) {
            /* next frontier = unique in-neighbours of the current frontier
             * (may contain nodes already in the ball: DGL's frontier is not
             * filtered, only the final union is unique'd) */
            int64_t nn = 0;
            for (int64_t f = 0; f < nf; ++f) {
                int64_t u = front[f];
                for (int64_t j = rowptr[u]; j < rowptr[u + 1]; ++j) {
                    int64_t w = col[j];
                    int seen = 0;
                    for (int64_t q = 0; q < nn; ++q) if (next[q] == w) { seen = 1; break; }
                    if (!seen) next[nn++] = w;
                }
            }
            for (int64_t q = 0; q < nn; ++q) {
                front[q] = next[q];
                if (stamp[next[q]] != v) { stamp[next[q]] = v; ball[nb++] = next[q]; }
            }
            nf = nn;
        }
        /* unique(cat(all frontiers)) == the stamped set, sorted ascending */
        ball[nb++] = v;
        qsort(ball, (size_t)nb, sizeof(int64_t), cmp_i64);
        for (int64_t r = 0; r < nb; ++r) pos[ball[r]] = r;
        int64_t ne = 0;
        for (int64_t r = 0; r < nb; ++r) {
            int64_t u = ball[r];
            for (int64_t j = rowptr[u]; j < rowptr[u + 1]; ++j) {
                int64_t w = col[j];
                if (stamp[w] == v) {
                    if (ego_src) {
                        ego_src[edge_off + ne] = r;
                        ego_dst[edge_off + ne] = pos[w];
                    }
                    ++ne;
                }
            }
        }
        if (ego_nodes) memcpy(ego_nodes + node_off, ball, sizeof(int64_t) * nb);
        ego_sizes[v] = nb;
        ego_ecount[v] = ne;
        node_off += nb;
        edge_off += ne;
        /* invalidate this ego-net's stamps so the next v starts clean */
        for (int64_t r = 0; r < nb; ++r) stamp[ball[r]] = -1;
    }
    free(stamp); free(pos); free(front); free(next); free(ball);
    return 0;
}
