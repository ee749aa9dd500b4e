/* gac_axtchain.c -- axtChain's chaining (gac_axt_chain, include/gachain.h).
 *
 * The reference chains the blocks of one (query, strand, target) pair at a
 * time, single-threaded (kent/src/hg/mouseStuff/axtChain/axtChain.c:250-309,
 * 452-470; kent/src/lib/chainBlock.c; kent/src/lib/chainConnect.c).  Here:
 *   1. removeExactOverlaps for every pair (host);
 *   2. every block's axtScoreUngapped in ONE GPU batch (gac_score_blocks);
 *   3. the kd-tree DP of chainBlocks per pair on host threads -- pairs are
 *      independent, so they run concurrently, largest first;
 *   4. chainRemovePartialOverlaps + chainMergeAbutting per chain (host);
 *   5. every chain's chainCalcScore in ONE GPU batch (gac_score_ranges over
 *      whole chains);
 *   6. minScore filter and the final stable score sort.
 *
 * Step 3 is a sequential dynamic programme: each leaf's best predecessor is
 * a branch-and-bound DFS of the kd-tree whose bounds depend on every leaf
 * before it, and whose pruning order decides ties (first in DFS order wins)
 * and -- because the overlap-adjusted connect cost can fall below the
 * gapCost bound -- even which predecessor is found.  Bit-exact output needs
 * that exact search, so the tree, the split rules, the visiting order, the
 * strict/non-strict comparisons and the double arithmetic all follow
 * chainBlock.c line by line (the sums are integral, so double is exact). */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdarg.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "gac_host.h"
#include "gachain.h"

/* ------------------------------------------------------------------ env */
typedef struct ax_env {
    const gac_gapcalc *g;
    int32_t m5[25];    /* [q code * 5 + t code], codes T C A G = 0..3, N = 4 */
    int32_t *gtab;     /* [3][gtab_len] gapCalcCost by kind and distance */
    int gtab_len;
    /* gapCalcCost's linear tail past the last long position, by kind: where
     * most kd-tree bounds of a large pair land (a call into the general
     * function cost the largest C4 pair 10 %) */
    int32_t last_pos[3];
    double last_val[3], last_slope[3];
    /* the exact fast DP (pair_dp_fast): gapCalcCost monotone in each
     * distance (so a subtree's corner bounds every non-overlapping
     * candidate), its linear minorant s*(dq+dt), s = lin_k/1024, and the
     * smallest matrix entry (a lower bound on a crossover's adjustment per
     * overlapping base) */
    int fast;
    int64_t lin_k;
    int32_t min_entry;
} ax_env;

/* chainConnectGapCost = gapCalcCost (chainConnect.c:108-112) */
static inline int gap_cost(const ax_env *e, int dq, int dt) {
    if (dt < 0)
        dt = 0;
    if (dq < 0)
        dq = 0;
    int kind, d;
    if (dt == 0) {
        kind = 0;
        d = dq;
    } else if (dq == 0) {
        kind = 1;
        d = dt;
    } else {
        kind = 2;
        d = dq + dt;
    }
    if (d >= 0 && d < e->gtab_len)
        return e->gtab[kind * e->gtab_len + d];
    if (d >= e->last_pos[kind]) { /* gapCalc.c:307,316,326, same operations (-ffp-contract=off) */
        const double prod = e->last_slope[kind] * (double)(d - e->last_pos[kind]);
        return (int)(e->last_val[kind] + prod);
    }
    return gac_gap_cost(e->g, dq, dt);
}

/* ------------------------------------------------------------------ sequences */
typedef struct ax_seq {
    gac_seq_view v;
    int minus; /* query on '-': coordinates on the reverse complement */
} ax_seq;

/* codes of strand positions [start, start + len) (N = 4) */
static void seq_codes(const ax_seq *s, int32_t start, int32_t len, uint8_t *out) {
    const int32_t size = s->v.size;
    for (int32_t i = 0; i < len; ++i) {
        const int32_t f = s->minus ? size - 1 - (start + i) : start + i;
        const int c = (s->v.packed[f >> 2] >> (6 - 2 * (f & 3))) & 3;
        out[i] = (uint8_t)(s->minus ? c ^ 2 : c);
    }
    if (s->v.n_count == 0 || len <= 0)
        return;
    const int32_t flo = s->minus ? size - (start + len) : start, fhi = flo + len;
    int32_t lo = 0, hi = s->v.n_count; /* first run ending after flo */
    while (lo < hi) {
        const int32_t mid = (lo + hi) / 2;
        if (s->v.n_start[mid] + s->v.n_size[mid] > flo)
            hi = mid;
        else
            lo = mid + 1;
    }
    for (int32_t k = lo; k < s->v.n_count && s->v.n_start[k] < fhi; ++k) {
        const int32_t a = s->v.n_start[k] > flo ? s->v.n_start[k] : flo;
        const int32_t b = s->v.n_start[k] + s->v.n_size[k] < fhi ? s->v.n_start[k] + s->v.n_size[k]
                                                                  : fhi;
        for (int32_t f = a; f < b; ++f)
            out[s->minus ? (size - 1 - f) - start : f - start] = 4;
    }
}

/* ------------------------------------------------------------------ per-thread work */
typedef struct ax_node { /* struct kdBranch (chainBlock.c:17-28), the fixed part */
    int32_t lo, hi, leaf, cut;
    int32_t max_q, max_t;
} ax_node;

/* the part of a node the DP raises (kdBranch.maxScore, and the fast DP's
 * linear bound), apart from the fixed part: a searcher's copy of a node's
 * children and cuts is never invalidated by a bound update */
typedef struct ax_bound {
    double max_score;
    int64_t nw; /* max of 1024 total + k (qEnd + tEnd) */
} ax_bound;

typedef struct ax_out { /* one pair's result */
    int32_t n_chains;
    int32_t *coff;           /* [n_chains + 1] */
    int32_t *bt, *bq, *bs;   /* blocks after overlap removal + merge */
    char *details;
    size_t details_len;
    int err;
    char msg[512];
    double secs; /* wall time of this pair's chaining */
    int64_t *gsc; /* [n_chains]: chainCalcScore of each chain (score_pairs) */
    int scored;
} ax_out;

/* a pair's leaves and kd-tree built on the device (gac_kd_trees) for the
 * host DP: the arrays are adopted by the pair's ax_work */
typedef struct ax_pre {
    int32_t nl;
    int32_t *tord, *qord, *lnode; /* [n] */
    int32_t *nodes;               /* [2 n][6]: ax_node */
} ax_pre;

typedef struct ax_work {
    const ax_env *e;
    ax_seq q, t;
    /* the pair's blocks (after removeExactOverlaps) */
    int32_t n;
    const int32_t *qs, *qe, *ts, *te, *score;
    /* leaves (indexed by block) */
    double *total;
    int32_t *pred; /* best predecessor: node index or -1 */
    uint8_t *hit;
    int32_t *tord, *qord, *tmp;
    int32_t nl;
    ax_node *nodes;
    int32_t nn;
    int32_t *lnode;  /* [block] the leaf's node */
    ax_bound *bnd;   /* [node] the bounds the DP raises */
    int32_t *qpos;   /* [block] the leaf's place in qord */
    int32_t *tpos;   /* [block] the leaf's place in tord */
    int32_t *tbox;   /* [4 leaves] by place in tord: {tStart, tEnd, qStart, qEnd} */
    int32_t *qbox;   /* [4 leaves] by place in qord: {qStart, qEnd, tStart, tEnd} */
    int32_t *qtp;    /* [leaf] by place in qord: its place in tord */
    int32_t cut_t;   /* fast searches see only leaves with tpos < cut_t */
    long long fallbacks;
    int team, team_batch; /* > 1: this pair's DP on that many threads (pair_dp_team) */
    int pred_blk;         /* pred holds blocks, not nodes (gac_chain_dp_blocks' results) */
    ax_pre *pre;          /* this pair's leaves and tree, built on the device (or NULL) */
    /* crossover scratch */
    uint8_t *xs;
    int32_t xcap;
    /* error */
    int err;
    char msg[512];
    size_t cap_n;
    /* gac_chain_blocks: the caller's ConnectCost / GapCost (NULL: built in) */
    gac_connect_fn cb_connect;
    gac_gapcost_fn cb_gap;
    void *cb_user;
} ax_work;

static void w_fail(ax_work *w, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
static void w_fail(ax_work *w, const char *fmt, ...) {
    if (w->err)
        return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(w->msg, sizeof(w->msg), fmt, ap);
    va_end(ap);
    w->err = 1;
}

/* cBlockFindCrossover (chainConnect.c:61-105) on blocks (qs,qe,ts,te) */
static void crossover(ax_work *w, int32_t lqs, int32_t lqe, int32_t lts, int32_t lte,
                      int32_t rqs, int32_t rqe, int32_t rts, int32_t rte, int overlap,
                      int *ret_pos, int *ret_adj) {
    (void)lqs;
    (void)rqe;
    if (overlap > (lte - lts) || overlap > (rte - rts)) {
        w_fail(w, "overlap is %d -- too large for one of these:\nqSize=%d  tSize=%d\n", overlap,
               w->q.v.size, w->t.v.size);
        *ret_pos = 0;
        *ret_adj = 0;
        return;
    }
    if (4 * overlap > w->xcap) {
        w->xcap = 4 * overlap + 1024;
        w->xs = realloc(w->xs, (size_t)w->xcap);
    }
    uint8_t *rq = w->xs, *lq = rq + overlap, *rt = lq + overlap, *lt = rt + overlap;
    seq_codes(&w->q, rqs, overlap, rq);
    seq_codes(&w->q, lqe - overlap, overlap, lq);
    seq_codes(&w->t, rts, overlap, rt);
    seq_codes(&w->t, lte - overlap, overlap, lt);
    const int32_t *m = w->e->m5;
    int64_t r_score = 0, l_score = 0;
    for (int i = 0; i < overlap; ++i) {
        r_score += m[rq[i] * 5 + rt[i]];
        l_score += m[lq[i] * 5 + lt[i]];
    }
    int64_t score = r_score, best = r_score;
    int best_pos = 0;
    for (int i = 0; i < overlap; ++i) {
        score += m[lq[i] * 5 + lt[i]];
        score -= m[rq[i] * 5 + rt[i]];
        if (score > best) {
            best = score;
            best_pos = i + 1;
        }
    }
    *ret_pos = best_pos;
    *ret_adj = (int)(r_score + l_score - best);
}

/* chainConnectCost (chainConnect.c:114-149) of block a then block b; pre:
 * the crossover adjustment of this overlap computed on the device, or NULL */
static int connect_cost_pre(ax_work *w, int32_t a, int32_t b, const int32_t *pre);

static int connect_cost(ax_work *w, int32_t a, int32_t b) { return connect_cost_pre(w, a, b, NULL); }

static int connect_cost_pre(ax_work *w, int32_t a, int32_t b, const int32_t *pre) {
    if (w->cb_connect)
        return w->cb_connect(a, b, w->cb_user);
    int dq = w->qs[b] - w->qe[a];
    int dt = w->ts[b] - w->te[a];
    int adj = 0;
    if (w->qs[a] >= w->qs[b] || w->ts[a] >= w->ts[b]) {
        w_fail(w, "a (%d %d) not strictly before b (%d %d)", w->qs[a], w->ts[a], w->qs[b],
               w->ts[b]);
        return 0;
    }
    if (dq < 0 || dt < 0) {
        const int b_size = w->qe[b] - w->qs[b];
        const int a_size = w->qe[a] - w->qs[a];
        const int overlap = -(dq < dt ? dq : dt);
        if (overlap >= b_size || overlap >= a_size) {
            adj = 100000000;
        } else {
            int cross;
            if (pre)
                adj = *pre;
            else
                crossover(w, w->qs[a], w->qe[a], w->ts[a], w->te[a], w->qs[b], w->qe[b], w->ts[b],
                          w->te[b], overlap, &cross, &adj);
            dq += overlap;
            dt += overlap;
        }
    }
    return adj + gap_cost(w->e, dq, dt);
}

/* stable partition of a[0..n) into hit-first order (splitList, chainBlock.c:92-110) */
static void partition(int32_t *a, int32_t n, const uint8_t *hit, int32_t *tmp) {
    int32_t k = 0;
    for (int32_t i = 0; i < n; ++i)
        if (hit[a[i]])
            tmp[k++] = a[i];
    for (int32_t i = 0; i < n; ++i)
        if (!hit[a[i]])
            tmp[k++] = a[i];
    if (n > 64) {
        memcpy(a, tmp, (size_t)n * sizeof(int32_t));
    } else { /* (most nodes are small: no library call per node) */
        for (int32_t i = 0; i < n; ++i)
            a[i] = tmp[i];
    }
}

/* medianVal + splitList of one node (chainBlock.c:112-122, 92-110): the
 * first half of the list in the cut dimension (D) is the lo side.  Hits are
 * set on D directly (the same leaves as clearHits over Q), and only the other
 * list is partitioned: D's own stable hit-first partition is the identity.
 * Returns the cut. */
static int32_t kd_split(ax_work *w, int32_t *Q, int32_t *T, int32_t n, int dim, int32_t *tmp) {
    const int32_t half = n / 2;
    const int32_t *D = dim == 0 ? Q : T;
    for (int32_t i = 0; i < half; ++i)
        w->hit[D[i]] = 1;
    for (int32_t i = half; i < n; ++i)
        w->hit[D[i]] = 0;
    const int32_t ml = D[half - 1];
    partition(dim == 0 ? T : Q, n, w->hit, tmp);
    return dim == 0 ? w->qs[ml] : w->ts[ml];
}

/* kdBuild (chainBlock.c:124-164): Q in query order, T in target order */
static int32_t kd_build(ax_work *w, int32_t *Q, int32_t *T, int32_t n, int dim) {
    const int32_t id = w->nn++;
    if (n == 1) {
        const int32_t l = Q[0];
        /* leaf node: lo/hi carry the leaf's qStart/tStart */
        w->nodes[id] = (ax_node){w->qs[l], w->ts[l], l, 0, w->qe[l], w->te[l]};
        w->bnd[id] = (ax_bound){0.0, INT64_MIN / 4};
        w->lnode[l] = id;
        return id;
    }
    const int32_t half = n / 2;
    const int32_t cut = kd_split(w, Q, T, n, dim, w->tmp);
    /* hi first: nodes land in the DFS's usual visiting order (pre-order,
     * hi before lo), so a search walks memory forward */
    const int32_t hi = kd_build(w, Q + half, T + half, n - half, 1 - dim);
    const int32_t lo = kd_build(w, Q, T, half, 1 - dim);
    ax_node *nd = &w->nodes[id];
    nd->lo = lo;
    nd->hi = hi;
    nd->leaf = -1;
    nd->cut = cut;
    w->bnd[id] = (ax_bound){0.0, INT64_MIN / 4};
    nd->max_q = w->nodes[lo].max_q > w->nodes[hi].max_q ? w->nodes[lo].max_q : w->nodes[hi].max_q;
    nd->max_t = w->nodes[lo].max_t > w->nodes[hi].max_t ? w->nodes[lo].max_t : w->nodes[hi].max_t;
    return id;
}

enum { kStack = 512 };

#ifdef GAC_DP_STATS /* profiling build only (make cpu-axtchain CPU_EXTRA=-DGAC_DP_STATS) */
static __thread struct {
    long long visits, prune1, prune2, leaves, cands, overlaps, xover_bases, updates, best_wins, ref_visits;
} g_st;
static __thread long long g_wr[8][2]; /* bound writes by depth / 4: max_score, linear */
#define ST(x) (g_st.x++)
#define STN(x, n) (g_st.x += (n))
#else
#define ST(x) ((void)0)
#define STN(x, n) ((void)0)
#endif

/* bestPredecessor (chainBlock.c:207-263), iterative with the same order:
 * the hi subtree (only when the lonely leaf lies past the cut) before lo.
 * ov (the fast DP's fallback, where the nodes' linear bounds are kept): the
 * leaf nodes of the lonely leaf's overlapping candidates, nov of them.  A
 * subtree holding none of them holds only non-overlapping candidates, whose
 * scores its linear bound caps; when that is below the best so far, the
 * reference walks the subtree without taking anything (it takes a strictly
 * greater score only), so skipping it leaves its answer as it was.  Node
 * ranges come from the pre-order layout: node b's subtree is [b, end), its
 * hi child's [b + 1, lo), its lo child's [lo, end). */
static void best_predecessor_at(ax_work *w, int32_t lonely, double *ret_score, int32_t *ret_pred,
                                const int32_t *ov, int nov) {
    const int32_t lq = w->qs[lonely], lt = w->ts[lonely];
    const double lscore = w->score[lonely];
    const int sure = nov >= 0;
    const int64_t kl = sure ? w->e->lin_k * ((int64_t)lq + lt) - 1024 * (int64_t)lscore : 0;
    double best = 0.0;
    int32_t best_node = -1;
    int32_t st_node[kStack], st_end[kStack];
    uint8_t st_dim[kStack];
    int sp = 0;
    st_node[sp] = 0;
    st_end[sp] = w->nn;
    st_dim[sp++] = 0;
    while (sp > 0) {
        --sp;
        const int32_t b = st_node[sp], end = st_end[sp];
        const int dim = st_dim[sp];
        const ax_node *nd = &w->nodes[b];
        ST(visits);
        ST(ref_visits);
        double max_score = w->bnd[b].max_score + lscore;
        if (max_score < best) {
            ST(prune1);
            continue;
        }
        max_score -= w->cb_gap ? w->cb_gap(lq - nd->max_q, lt - nd->max_t, w->cb_user)
                               : gap_cost(w->e, lq - nd->max_q, lt - nd->max_t);
        if (max_score < best) {
            ST(prune2);
            continue;
        }
        if (sure && w->bnd[b].nw - kl < 1024 * (int64_t)best) {
            int held = 0;
            for (int k = 0; k < nov && !held; ++k)
                held = ov[k] >= b && ov[k] < end;
            if (!held)
                continue;
        }
        if (nd->leaf >= 0) {
            const int32_t l = nd->leaf;
            ST(leaves);
            if (nd->lo < lq && nd->hi < lt) {
                ST(cands);
#ifdef GAC_DP_STATS
                if (w->qs[lonely] < w->qe[l] || w->ts[lonely] < w->te[l]) {
                    ST(overlaps);
                    const int dq = w->qs[lonely] - w->qe[l], dt = w->ts[lonely] - w->te[l];
                    STN(xover_bases, -(dq < dt ? dq : dt));
                }
#endif
                const double sc = w->total[l] + lscore - connect_cost(w, l, lonely);
                if (sc > best) {
                    ST(best_wins);
                    best = sc;
                    best_node = b;
                }
            }
            continue;
        }
        if (sp + 2 > kStack) {
            w_fail(w, "kd-tree deeper than %d", kStack / 2);
            break;
        }
        const int32_t coord = dim == 0 ? lq : lt;
        st_node[sp] = nd->lo;
        st_end[sp] = end;
        st_dim[sp++] = (uint8_t)(1 - dim);
        if (coord > nd->cut) {
            st_node[sp] = nd->hi;
            st_end[sp] = nd->lo;
            st_dim[sp++] = (uint8_t)(1 - dim);
        }
    }
    *ret_score = best;
    *ret_pred = best_node;
}

static void best_predecessor(ax_work *w, int32_t lonely, double *ret_score, int32_t *ret_pred) {
    best_predecessor_at(w, lonely, ret_score, ret_pred, NULL, -1);
}

/* updateScoresOnWay (chainBlock.c:265-279): both sides on a tie with the cut */
static void update_scores(ax_work *w, int32_t leaf) {
    const double total = w->total[leaf];
    const int32_t lq = w->qs[leaf], lt = w->ts[leaf];
    int32_t st_node[kStack];
    uint8_t st_dim[kStack];
    int sp = 0;
    st_node[sp] = 0;
    st_dim[sp++] = 0;
    while (sp > 0) {
        --sp;
        const int32_t b = st_node[sp];
        const int dim = st_dim[sp];
        ax_node *nd = &w->nodes[b];
        ST(updates);
        if (w->bnd[b].max_score < total)
            w->bnd[b].max_score = total;
        if (nd->leaf < 0) {
            if (sp + 2 > kStack) {
                w_fail(w, "kd-tree deeper than %d", kStack / 2);
                return;
            }
            const int32_t coord = dim == 0 ? lq : lt;
            if (coord <= nd->cut) {
                st_node[sp] = nd->lo;
                st_dim[sp++] = (uint8_t)(1 - dim);
            }
            if (coord >= nd->cut) {
                st_node[sp] = nd->hi;
                st_dim[sp++] = (uint8_t)(1 - dim);
            }
        }
    }
}

/* ------------------------------------------------------------------ the exact fast DP
 * bestPredecessor returns the first leaf, in its DFS order, of the best
 * score among the candidates it does not prune, and it prunes a subtree when
 * the subtree's bound (max total + the lonely leaf's score - gapCost to the
 * subtree's top corner) is below the best so far.  For a non-overlapping
 * candidate that bound is a true upper bound (gapCalcCost is monotone in
 * each distance: checked per gap setup, ax_env.fast); for an overlapping one
 * it is not when the crossover's adjustment is negative (chainConnect.c:
 * 61-105).  Call a candidate anomalous if its score exceeds
 * the bound at its own leaf node (every ancestor's bound is at least that).
 * If every anomalous candidate scores below the best non-anomalous score M,
 * the reference's search returns the first non-anomalous leaf scoring M:
 * nothing on that leaf's path can be pruned (its bounds are >= M >= best),
 * and nothing before it scores M.  The same holds for any search in the same
 * DFS order that prunes by tighter TRUE bounds.  pair_dp_fast therefore
 *   1. searches with a second bound per subtree, the linear minorant of the
 *      gap cost: max over its leaves of total + s (qEnd + tEnd), minus
 *      s (qStart + tStart) of the lonely leaf -- far high-scoring leaves no
 *      longer keep whole subtrees open;
 *   2. then looks at every overlapping candidate (blocks of earlier leaves
 *      that reach past the lonely leaf's start in q or t, found by scanning
 *      back over the t- and q-ordered leaves by the pair's longest block):
 *      one that could score at least the best found (and > 0) and violates
 *      either bound at its leaf node sends this leaf to the reference search
 *      (best_predecessor), so the result is the reference's in every case. */
static void best_predecessor_fast(ax_work *w, int32_t lonely, double *ret_score, int32_t *ret_pred) {
    const int32_t lq = w->qs[lonely], lt = w->ts[lonely];
    const double lscore = w->score[lonely];
    const int64_t k = w->e->lin_k, kl = k * ((int64_t)lq + lt) - 1024 * (int64_t)lscore;
    double best = 0.0;
    int64_t best1024 = 0;
    int32_t best_node = -1;
    int32_t st_node[kStack];
    uint8_t st_dim[kStack];
    int sp = 0;
    st_node[sp] = 0;
    st_dim[sp++] = 0;
    while (sp > 0) {
        --sp;
        const int32_t b = st_node[sp];
        const int dim = st_dim[sp];
        const ax_node *nd = &w->nodes[b];
        ST(visits);
        double max_score = w->bnd[b].max_score + lscore;
        if (max_score < best) {
            ST(prune1);
            continue;
        }
        if (w->bnd[b].nw - kl < best1024) {
            ST(prune1);
            continue;
        }
        const int dq = lq - nd->max_q, dt = lt - nd->max_t;
        const int gc = gap_cost(w->e, dq, dt);
        max_score -= gc;
        if (max_score < best) {
            ST(prune2);
            continue;
        }
        if (nd->leaf >= 0) {
            /* a leaf node holds its block (lo, hi = qStart, tStart; max_q,
             * max_t = qEnd, tEnd) and its target position (cut, see
             * dp_leaf_positions): a candidate that does not overlap costs
             * the gap just computed, with no look-up of its block */
            const int32_t l = nd->leaf;
            ST(leaves);
            if (nd->lo < lq && nd->hi < lt && nd->cut < w->cut_t) {
                ST(cands);
                const int cost = (dq >= 0 && dt >= 0) ? gc : connect_cost(w, l, lonely);
                const double s = w->total[l] + lscore - cost;
                if (s > best) {
                    ST(best_wins);
                    best = s;
                    best1024 = 1024 * (int64_t)s;
                    best_node = b;
                }
            }
            continue;
        }
        if (sp + 2 > kStack) {
            w_fail(w, "kd-tree deeper than %d", kStack / 2);
            break;
        }
        const int32_t coord = dim == 0 ? lq : lt;
        st_node[sp] = nd->lo;
        st_dim[sp++] = (uint8_t)(1 - dim);
        __builtin_prefetch(&w->nodes[nd->lo]); /* (visited after the hi side) */
        __builtin_prefetch(&w->bnd[nd->lo]);
        if (coord > nd->cut) {
            st_node[sp] = nd->hi;
            st_dim[sp++] = (uint8_t)(1 - dim);
        }
    }
    *ret_score = best;
    *ret_pred = best_node;
}

/* the target position of every leaf, in w->tpos and in its leaf node's
 * (otherwise unused) cut field, where the fast search reads it */
static void dp_leaf_positions(ax_work *w, int32_t *maxsz) {
    int32_t m = 0;
    for (int32_t i = 0; i < w->nl; ++i) {
        const int32_t l = w->tord[i];
        if (w->te[l] - w->ts[l] > m)
            m = w->te[l] - w->ts[l];
        w->qpos[w->qord[i]] = i;
        w->tpos[l] = i;
        w->nodes[w->lnode[l]].cut = i;
        int32_t *b = w->tbox + 4 * (size_t)i;
        b[0] = w->ts[l], b[1] = w->te[l], b[2] = w->qs[l], b[3] = w->qe[l];
    }
    for (int32_t i = 0; i < w->nl; ++i) {
        const int32_t l = w->qord[i];
        int32_t *b = w->qbox + 4 * (size_t)i;
        b[0] = w->qs[l], b[1] = w->qe[l], b[2] = w->ts[l], b[3] = w->te[l];
        w->qtp[i] = w->tpos[l];
    }
    *maxsz = m;
}

/* 1 when an overlapping candidate of `lonely` (the ti-th leaf in t order)
 * could score >= best (and > 0) while violating a bound at its leaf node */
static int dp_anomaly(ax_work *w, int32_t lonely, int32_t ti, double best, int32_t maxsz) {
    const int32_t lq = w->qs[lonely], lt = w->ts[lonely];
    const int32_t lsize = w->qe[lonely] - lq;
    const double lscore = w->score[lonely];
    const double need = best > 0 ? best : 1.0; /* (scores are integral) */
    const int64_t k = w->e->lin_k;
    for (int side = 0; side < 2; ++side) {
        /* the leaves starting within the longest block before the lonely
         * one on this side, read in order from the packed boxes */
        const int32_t *box = side ? w->qbox : w->tbox;
        const int32_t at = side ? w->qpos[lonely] : ti, lo = (side ? lq : lt) - maxsz;
        for (int32_t j = at - 1; j >= 0 && box[4 * (size_t)j] > lo; --j) {
            const int32_t *b = box + 4 * (size_t)j;
            const int32_t cqs = side ? b[0] : b[2], cqe = side ? b[1] : b[3];
            const int32_t cts = side ? b[2] : b[0], cte = side ? b[3] : b[1];
            const int32_t tp = side ? w->qtp[j] : j;
            if (cts >= lt || cqs >= lq || tp >= w->cut_t)
                continue; /* not a candidate (or not yet scored) */
            int dq = lq - cqe, dt = lt - cte;
            if (dq >= 0 && dt >= 0)
                continue; /* no overlap: the bounds hold */
            if (side == 1 && dt < 0)
                continue; /* (the t scan saw it) */
            const int ov = -(dq < dt ? dq : dt);
            if (ov >= lsize || ov >= cqe - cqs)
                continue; /* connect cost 1e8 */
            const int32_t c = side ? w->qord[j] : w->tord[j];
            /* cheap upper bound first: adj >= ov * min_entry */
            const double ub = w->total[c] + lscore - (double)gap_cost(w->e, dq + ov, dt + ov) -
                              (double)ov * w->e->min_entry;
            if (ub < need)
                continue;
            const double sc = w->total[c] + lscore - connect_cost(w, c, lonely);
            if (sc < need)
                continue;
            /* the bounds at c's leaf node are at least those of c alone
             * (its max is >= c's total, its corner is c's end): compared
             * with these, the check holds whatever the node held when the
             * search read it (pair_dp_team reads a tree being updated) */
            const double bc = w->total[c] + lscore - gap_cost(w->e, dq, dt);
            const int64_t bl = 1024 * (int64_t)w->total[c] - k * ((int64_t)dq + dt) + 1024 * (int64_t)lscore;
            if (sc > bc || 1024 * (int64_t)sc > bl)
                return 1;
        }
    }
    return 0;
}

/* the leaf nodes of every overlapping candidate of `lonely` (dp_anomaly's
 * scan, all of them): their count, or -1 past cap */
static int dp_overlaps(ax_work *w, int32_t lonely, int32_t ti, int32_t maxsz, int32_t *out,
                       int cap) {
    const int32_t lq = w->qs[lonely], lt = w->ts[lonely];
    int n = 0;
    for (int side = 0; side < 2; ++side) {
        const int32_t *box = side ? w->qbox : w->tbox;
        const int32_t at = side ? w->qpos[lonely] : ti, lo = (side ? lq : lt) - maxsz;
        for (int32_t j = at - 1; j >= 0 && box[4 * (size_t)j] > lo; --j) {
            const int32_t *b = box + 4 * (size_t)j;
            const int32_t cqs = side ? b[0] : b[2], cqe = side ? b[1] : b[3];
            const int32_t cts = side ? b[2] : b[0], cte = side ? b[3] : b[1];
            const int32_t tp = side ? w->qtp[j] : j;
            if (cts >= lt || cqs >= lq || tp >= w->cut_t)
                continue;
            const int dq = lq - cqe, dt = lt - cte;
            if (dq >= 0 && dt >= 0)
                continue;
            if (side == 1 && dt < 0)
                continue; /* (the t scan saw it) */
            if (n == cap)
                return -1;
            out[n++] = w->lnode[side ? w->qord[j] : w->tord[j]];
        }
    }
    return n;
}

/* the reference-order search, sped up where it provably changes nothing */
static void best_predecessor_fallback(ax_work *w, int32_t lonely, int32_t ti, int32_t maxsz,
                                      double *ret_score, int32_t *ret_pred) {
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("GAC_DP_FALLBACK_PRUNE");
        on = !(e && *e == '0');
    }
    int32_t ov[64];
    const int nov = on ? dp_overlaps(w, lonely, ti, maxsz, ov, 64) : -1;
    best_predecessor_at(w, lonely, ret_score, ret_pred, ov, nov);
}

/* ---- sorts (glibc qsort is a stable merge sort here; ranks make it explicit) */
typedef struct ikey {
    int64_t k;
    int32_t rank, v;
} ikey;

static int ikey_cmp(const void *a, const void *b) {
    const ikey *x = a, *y = b;
    if (x->k != y->k)
        return x->k < y->k ? -1 : 1;
    return (x->rank > y->rank) - (x->rank < y->rank);
}

typedef struct dkey {
    double k;
    int32_t rank, v;
} dkey;
struct dkey;

/* descending by k (kdLeafCmpTotal / chainCmpScore: sign of b - a) */
static int dkey_cmp_desc(const void *a, const void *b) {
    const dkey *x = a, *y = b;
    const double diff = y->k - x->k;
    if (diff < 0)
        return -1;
    if (diff > 0)
        return 1;
    return (x->rank > y->rank) - (x->rank < y->rank);
}

/* ---- chain post-processing on a block list (linked by next[]) ---- */
_Static_assert(sizeof(ikey) == 16 && sizeof(dkey) == 16, "par_sort16 keys");

/* ---- a stable parallel LSD radix sort of 16-byte records by their first 8
 * bytes as an unsigned key.  Where the records go in input (rank) order,
 * stable by key is the (key, rank) order of the comparator sorts.  Per pass
 * every thread counts the digits of its own slice; one prefix over (digit,
 * slice) makes the scatter stable; passes only over the key bits in use. */
enum { kRadixBits = 10, kRadix = 1 << kRadixBits };

typedef struct rsort {
    uint8_t *src, *dst;
    int64_t n;
    int nt, shift;
    int64_t *cnt; /* [nt][kRadix] */
    _Atomic int next;
} rsort;

static inline uint64_t rs_key(const uint8_t *r) {
    uint64_t k;
    memcpy(&k, r, 8);
    return k;
}

static void *rs_count(void *arg) {
    rsort *R = arg;
    for (int c; (c = atomic_fetch_add(&R->next, 1)) < R->nt;) {
        const int64_t lo = R->n * c / R->nt, hi = R->n * (c + 1) / R->nt;
        int64_t *h = R->cnt + (size_t)c * kRadix;
        memset(h, 0, kRadix * sizeof(int64_t));
        for (int64_t i = lo; i < hi; ++i)
            ++h[(rs_key(R->src + 16 * i) >> R->shift) & (kRadix - 1)];
    }
    return NULL;
}

static void *rs_scatter(void *arg) {
    rsort *R = arg;
    for (int c; (c = atomic_fetch_add(&R->next, 1)) < R->nt;) {
        const int64_t lo = R->n * c / R->nt, hi = R->n * (c + 1) / R->nt;
        int64_t *h = R->cnt + (size_t)c * kRadix; /* (the slice's output offsets) */
        for (int64_t i = lo; i < hi; ++i) {
            const uint8_t *r = R->src + 16 * i;
            memcpy(R->dst + 16 * h[(rs_key(r) >> R->shift) & (kRadix - 1)]++, r, 16);
        }
    }
    return NULL;
}

static int radix_sort16_any(void *a, int64_t n, int nt, uint64_t any);

static int radix_sort16(void *a, int64_t n, int nt) { /* -1, unsorted: a key < 0 as int64 */
    uint64_t any = 0;
    for (int64_t i = 0; i < n; ++i)
        any |= rs_key((const uint8_t *)a + 16 * i);
    return radix_sort16_any(a, n, nt, any);
}

/* any: the OR of every key (the bits the passes cover) */
static int radix_sort16_any(void *a, int64_t n, int nt, uint64_t any) {
    if (any >> 63)
        return -1;
    if (n < 2 || any == 0)
        return 0;
    const int bits = 64 - __builtin_clzll(any);
    if (nt < 1 || n < (1 << 16))
        nt = 1;
    rsort R;
    R.src = a;
    R.dst = malloc((size_t)n * 16);
    R.n = n;
    R.nt = nt;
    R.cnt = malloc((size_t)nt * kRadix * sizeof(int64_t));
    uint8_t *const tmp = R.dst;
    for (R.shift = 0; R.shift < bits; R.shift += kRadixBits) {
        atomic_init(&R.next, 0);
        gac_run_threads(nt, rs_count, &R);
        int64_t off = 0;
        for (int d = 0; d < kRadix; ++d)
            for (int c = 0; c < nt; ++c) {
                const int64_t t = R.cnt[(size_t)c * kRadix + d];
                R.cnt[(size_t)c * kRadix + d] = off;
                off += t;
            }
        atomic_init(&R.next, 0);
        gac_run_threads(nt, rs_scatter, &R);
        uint8_t *t = R.src;
        R.src = R.dst;
        R.dst = t;
    }
    if (R.src != (uint8_t *)a)
        memcpy(a, R.src, (size_t)n * 16);
    free(tmp);
    free(R.cnt);
    return 0;
}

/* a stable parallel merge sort of 16-byte keys (ikey, dkey: their
 * comparators end on a rank, so the order is total): runs sorted by qsort
 * on every thread, then merged in rounds */
typedef struct psort16 {
    char *a, *tmp;
    int64_t n;
    int nrun;
    int64_t *cut;
    int64_t width;
    int (*cmp)(const void *, const void *);
    _Atomic int next;
} psort16;

static void *ps16_runs(void *arg) {
    psort16 *J = arg;
    for (;;) {
        const int r = atomic_fetch_add(&J->next, 1);
        if (r >= J->nrun)
            return NULL;
        qsort(J->a + 16 * J->cut[r], (size_t)(J->cut[r + 1] - J->cut[r]), 16, J->cmp);
    }
}

static void *ps16_merge(void *arg) {
    psort16 *J = arg;
    for (;;) {
        const int m = atomic_fetch_add(&J->next, 1);
        const int64_t r0 = (int64_t)m * 2 * J->width;
        if (r0 >= J->nrun)
            return NULL;
        const int64_t r1 = r0 + J->width < J->nrun ? r0 + J->width : J->nrun;
        const int64_t r2 = r0 + 2 * J->width < J->nrun ? r0 + 2 * J->width : J->nrun;
        int64_t i = J->cut[r0], j = J->cut[r1], o = J->cut[r0];
        const int64_t ie = J->cut[r1], je = J->cut[r2];
        while (i < ie && j < je) {
            const int right = J->cmp(J->a + 16 * j, J->a + 16 * i) < 0;
            memcpy(J->tmp + 16 * o++, J->a + 16 * (right ? j++ : i++), 16);
        }
        if (i < ie)
            memcpy(J->tmp + 16 * o, J->a + 16 * i, (size_t)(ie - i) * 16), o += ie - i;
        if (j < je)
            memcpy(J->tmp + 16 * o, J->a + 16 * j, (size_t)(je - j) * 16);
    }
}

static void par_sort16(void *a, int64_t n, int (*cmp)(const void *, const void *), int nt) {
    if (nt <= 1 || n < (1 << 16)) {
        qsort(a, (size_t)n, 16, cmp);
        return;
    }
    psort16 J;
    J.a = a;
    J.n = n;
    J.nrun = nt;
    J.cmp = cmp;
    J.cut = malloc((size_t)(nt + 1) * sizeof(int64_t));
    for (int r = 0; r <= nt; ++r)
        J.cut[r] = n * r / nt;
    atomic_init(&J.next, 0);
    gac_run_threads(nt, ps16_runs, &J);
    J.tmp = malloc((size_t)n * 16);
    for (J.width = 1; J.width < nt; J.width *= 2) {
        atomic_store(&J.next, 0);
        const int64_t merges = (nt + 2 * J.width - 1) / (2 * J.width);
        gac_run_threads(merges < nt ? (int)merges : nt, ps16_merge, &J);
        char *t = J.a;
        J.a = J.tmp;
        J.tmp = t;
    }
    if (J.a != (char *)a) {
        memcpy(a, J.a, (size_t)n * 16);
        J.tmp = J.a;
    }
    free(J.tmp);
    free(J.cut);
}

/* dkey_cmp_desc's order for keys whose ranks are their input positions:
 * scores are integral (sums of integer block scores and gap costs), so
 * (max - k) is an exact unsigned key for radix_sort16 (stable: ties stay in
 * rank order); other keys take the comparator sort */
/* slices [n c / nt, n (c + 1) / nt) of a loop on nt threads (one slice,
 * inline, below 2^18 iterations) */
typedef struct pfor {
    void (*fn)(void *ctx, int c, int64_t a, int64_t b);
    void *ctx;
    int64_t n;
    int nt;
    _Atomic int next;
} pfor;

static void *pfor_thread(void *arg) {
    pfor *P = arg;
    for (int c; (c = atomic_fetch_add(&P->next, 1)) < P->nt;)
        P->fn(P->ctx, c, P->n * c / P->nt, P->n * (c + 1) / P->nt);
    return NULL;
}

static int par_for(int64_t n, int nt, void (*fn)(void *, int, int64_t, int64_t), void *ctx) {
    nt = nt > 256 ? 256 : nt;
    if (nt <= 1 || n < (1 << 18)) {
        fn(ctx, 0, 0, n);
        return 1;
    }
    pfor P = {fn, ctx, n, nt, 0};
    atomic_init(&P.next, 0);
    gac_run_threads(nt, pfor_thread, &P);
    return nt;
}

typedef struct sd16 {
    dkey *k;
    int64_t m;
    double mx[256];
    int bad[256], any[256];
    uint64_t bits[256];
} sd16;

static void sd16_scan(void *arg, int c, int64_t a, int64_t b) {
    sd16 *S = arg;
    double mx = 0;
    S->bad[c] = 0;
    S->any[c] = a < b;
    for (int64_t i = a; i < b; ++i) {
        const double x = S->k[i].k;
        if (!(x > -4.0e15 && x < 4.0e15) || (double)(int64_t)x != x) {
            S->bad[c] = 1;
            return;
        }
        if (i == a || x > mx)
            mx = x;
    }
    S->mx[c] = mx;
}

static void sd16_to_u(void *arg, int c, int64_t a, int64_t b) {
    sd16 *S = arg;
    uint64_t o = 0;
    for (int64_t i = a; i < b; ++i) {
        const uint64_t u = (uint64_t)(S->m - (int64_t)S->k[i].k);
        memcpy(&S->k[i].k, &u, 8);
        o |= u;
    }
    S->bits[c] = o;
}

static void sd16_from_u(void *arg, int c, int64_t a, int64_t b) {
    sd16 *S = arg;
    (void)c;
    for (int64_t i = a; i < b; ++i) {
        uint64_t u;
        memcpy(&u, &S->k[i].k, 8);
        S->k[i].k = (double)(S->m - (int64_t)u);
    }
}

static void sort_desc16(dkey *k, int64_t n, int nt) {
    sd16 *S = malloc(sizeof(sd16));
    S->k = k;
    const int ns = par_for(n, nt, sd16_scan, S);
    int have = 0;
    double mx = 0;
    for (int c = 0; c < ns; ++c) {
        if (S->bad[c]) {
            free(S);
            par_sort16(k, n, dkey_cmp_desc, nt);
            return;
        }
        if (S->any[c] && (!have || S->mx[c] > mx)) {
            mx = S->mx[c];
            have = 1;
        }
    }
    S->m = (int64_t)mx;
    const int nu = par_for(n, nt, sd16_to_u, S);
    uint64_t any = 0;
    for (int c = 0; c < nu; ++c)
        any |= S->bits[c];
    radix_sort16_any(k, n, nt, any);
    par_for(n, nt, sd16_from_u, S);
    free(S);
}

typedef struct ax_cb {
    int32_t qs, qe, ts, te;
    int32_t next;
} ax_cb;

/* crossovers of the chains' adjacent overlapping blocks computed on the
 * device (GAC_AXT_DP=gpu): by chain-block position j (the pair j-1, j), with
 * the inputs they were computed from */
typedef struct ax_xres {
    const int32_t *job;  /* [blocks] job index or -1 */
    const int32_t *pos, *adj;
    const int32_t *lqe, *lte, *rqs, *rts, *ov;
} ax_xres;

static void xover_cb(ax_work *w, const ax_cb *a, const ax_cb *b, int overlap, int *pos, int *adj,
                     const ax_xres *x, int32_t jb) {
    const int32_t k = x ? x->job[jb] : -1;
    if (k >= 0 && x->lqe[k] == a->qe && x->lte[k] == a->te && x->rqs[k] == b->qs &&
        x->rts[k] == b->ts && x->ov[k] == overlap && overlap <= a->te - a->ts &&
        overlap <= b->te - b->ts) {
        *pos = x->pos[k];
        *adj = x->adj[k];
        return;
    }
    crossover(w, a->qs, a->qe, a->ts, a->te, b->qs, b->qe, b->ts, b->te, overlap, pos, adj);
}

/* chainRemovePartialOverlaps (chainConnect.c:255-344) + chainMergeAbutting
 * (:346-368); returns the new head (blocks in cb[], list by next) */
static int32_t remove_partial_overlaps(ax_work *w, ax_cb *cb, int32_t head, const ax_xres *x) {
    for (int32_t a = head, b = cb[a].next; b >= 0; a = b, b = cb[b].next)
        if (cb[a].qs >= cb[b].qs || cb[a].ts >= cb[b].ts) {
            w_fail(w, "a (%d %d) not before b (%d %d) before removePartialOverlaps", cb[a].qs,
                   cb[a].ts, cb[b].qs, cb[b].ts);
            return head;
        }
    for (;;) {
        int trim_a = 0, trim_b = 0;
        int32_t a = head, b = cb[a].next;
        for (;;) {
            if (b < 0)
                break;
            const int dq = cb[b].qs - cb[a].qe, dt = cb[b].ts - cb[a].te;
            if (dq < 0 || dt < 0) {
                const int overlap = -(dq < dt ? dq : dt);
                const int a_size = cb[a].qe - cb[a].qs, b_size = cb[b].qe - cb[b].qs;
                if (overlap >= a_size || overlap >= b_size) {
                    trim_b = 1;
                } else {
                    int cross, adj;
                    xover_cb(w, &cb[a], &cb[b], overlap, &cross, &adj, b == a + 1 ? x : NULL, b);
                    cb[b].qs += cross;
                    cb[b].ts += cross;
                    const int inv = overlap - cross;
                    cb[a].qe -= inv;
                    cb[a].te -= inv;
                    if (cb[b].qe <= cb[b].qs)
                        trim_b = 1;
                    else if (cb[a].qe <= cb[a].qs)
                        trim_a = 1;
                }
            }
            if (trim_a) {
                /* removeNegativeBlocks */
                int32_t nh = -1, tail = -1;
                for (int32_t x = head; x >= 0; x = cb[x].next) {
                    if (cb[x].qs >= cb[x].qe || cb[x].ts >= cb[x].te)
                        continue;
                    if (tail < 0)
                        nh = x;
                    else
                        cb[tail].next = x;
                    tail = x;
                }
                if (tail >= 0)
                    cb[tail].next = -1;
                head = nh;
                break;
            } else if (trim_b) {
                b = cb[b].next;
                cb[a].next = b;
                trim_b = 0;
            } else {
                a = b;
                b = cb[b].next;
            }
        }
        if (!trim_a)
            break;
        if (head < 0)
            break;
    }
    /* checkChainGaps / checkStartBeforeEnd */
    for (int32_t a = head, b = head >= 0 ? cb[head].next : -1; b >= 0; a = b, b = cb[b].next)
        if (cb[a].qe > cb[b].qs || cb[a].te > cb[b].ts) {
            w_fail(w, "Negative gap between (%d %d - %d %d) and (%d %d - %d %d) after removePartialOverlaps",
                   cb[a].qs, cb[a].ts, cb[a].qe, cb[a].te, cb[b].qs, cb[b].ts, cb[b].qe, cb[b].te);
            return head;
        }
    for (int32_t x = head; x >= 0; x = cb[x].next)
        if (cb[x].qs >= cb[x].qe || cb[x].ts >= cb[x].te) {
            w_fail(w, "Start after end in (%d %d) to (%d %d) after removePartialOverlaps",
                   cb[x].qs, cb[x].ts, cb[x].qe, cb[x].te);
            return head;
        }
    /* chainMergeAbutting */
    int32_t last = -1;
    for (int32_t x = head; x >= 0;) {
        const int32_t nx = cb[x].next;
        if (last < 0 || cb[last].qe != cb[x].qs || cb[last].te != cb[x].ts) {
            last = x;
        } else {
            cb[last].qe = cb[x].qe;
            cb[last].te = cb[x].te;
            cb[last].next = nx;
        }
        x = nx;
    }
    return head;
}

/* ------------------------------------------------------------------ one pair */
typedef struct ax_pairinfo {
    const char *tname, *qname;
    int32_t tsize, qsize;
    char strand;
} ax_pairinfo;

/* leaves: slAddHead over the block list (reversed), zero-length blocks
 * skipped, then slSort by tStart (stable); and the query-ordered copy
 * (dlSort by qStart of the target-ordered list).  Returns the leaf count. */
static int32_t pair_leaves(ax_work *w) {
    const int32_t nb = w->n;
    ikey *k = malloc((size_t)(nb ? nb : 1) * sizeof(ikey));
    int32_t nl = 0;
    for (int32_t i = nb - 1; i >= 0; --i) {
        if (w->ts[i] == w->te[i])
            continue;
        k[nl] = (ikey){w->ts[i], nl, i};
        ++nl;
    }
    w->nl = nl;
    if (nl == 0) {
        free(k);
        return 0;
    }
    const int nt = w->team > 1 ? w->team : 1; /* (large pairs: every thread) */
    /* (ranks in input order: stable by key is the (k, rank) order) */
    if (radix_sort16(k, nl, nt) != 0)
        par_sort16(k, nl, ikey_cmp, nt);
    for (int32_t i = 0; i < nl; ++i)
        w->tord[i] = k[i].v;
    for (int32_t i = 0; i < nl; ++i)
        k[i] = (ikey){w->qs[w->tord[i]], i, w->tord[i]};
    if (radix_sort16(k, nl, nt) != 0)
        par_sort16(k, nl, ikey_cmp, nt);
    for (int32_t i = 0; i < nl; ++i)
        w->qord[i] = k[i].v;
    free(k);
    for (int32_t i = 0; i < nb; ++i) {
        w->total[i] = w->score[i];
        w->pred[i] = -1;
    }
    return nl;
}

/* kd_build of a subtree whose node ids are known in advance: a subtree of
 * n leaves has 2n - 1 nodes, laid out hi-first in pre-order from `id`, so
 * disjoint subtrees can be built by different threads (tmp: scratch the
 * size of Q, the same offset as Q into the pair's list) */
static void kd_build_at(ax_work *w, int32_t *Q, int32_t *T, int32_t n, int dim, int32_t id,
                        int32_t *tmp) {
    if (n == 1) {
        const int32_t l = Q[0];
        w->nodes[id] = (ax_node){w->qs[l], w->ts[l], l, 0, w->qe[l], w->te[l]};
        w->bnd[id] = (ax_bound){0.0, INT64_MIN / 4};
        w->lnode[l] = id;
        return;
    }
    const int32_t half = n / 2;
    const int32_t cut = kd_split(w, Q, T, n, dim, tmp);
    const int32_t hi = id + 1, lo = id + 2 * (n - half);
    kd_build_at(w, Q + half, T + half, n - half, 1 - dim, hi, tmp + half);
    kd_build_at(w, Q, T, half, 1 - dim, lo, tmp);
    ax_node *nd = &w->nodes[id];
    nd->lo = lo;
    nd->hi = hi;
    nd->leaf = -1;
    nd->cut = cut;
    w->bnd[id] = (ax_bound){0.0, INT64_MIN / 4};
    nd->max_q = w->nodes[lo].max_q > w->nodes[hi].max_q ? w->nodes[lo].max_q : w->nodes[hi].max_q;
    nd->max_t = w->nodes[lo].max_t > w->nodes[hi].max_t ? w->nodes[lo].max_t : w->nodes[hi].max_t;
}

typedef struct kd_task {
    int32_t *Q, *T, *tmp;
    int32_t n, id;
    int dim;
} kd_task;

typedef struct kd_job {
    ax_work *w;
    kd_task *t;
    int32_t nt;
    _Atomic int32_t next;
} kd_job;

static void *kd_thread(void *arg) {
    kd_job *J = arg;
    for (;;) {
        const int32_t k = atomic_fetch_add(&J->next, 1);
        if (k >= J->nt)
            return NULL;
        const kd_task *t = &J->t[k];
        kd_build_at(J->w, t->Q, t->T, t->n, t->dim, t->id, t->tmp);
    }
}

/* kd_split of a large node on nt threads: the hits set by slices of D, the
 * other list's stable partition by slice counts (hits of earlier slices,
 * then all hits, then the misses of earlier slices) */
typedef struct ksplit {
    ax_work *w;
    const int32_t *D;
    int32_t *O, *tmp;
    int32_t n, half;
    int nt, phase;
    int32_t *nhit; /* [nt + 1]: hits per slice, then their exclusive prefix */
    _Atomic int next;
} ksplit;

static void *ksplit_thread(void *arg) {
    ksplit *K = arg;
    for (int c; (c = atomic_fetch_add(&K->next, 1)) < K->nt;) {
        const int32_t lo = (int32_t)((int64_t)K->n * c / K->nt);
        const int32_t hi = (int32_t)((int64_t)K->n * (c + 1) / K->nt);
        uint8_t *hit = K->w->hit;
        if (K->phase == 0) {
            for (int32_t i = lo; i < hi; ++i)
                hit[K->D[i]] = i < K->half;
        } else if (K->phase == 1) {
            int32_t h = 0;
            for (int32_t i = lo; i < hi; ++i)
                h += hit[K->O[i]];
            K->nhit[c] = h;
        } else if (K->phase == 2) {
            int32_t a = K->nhit[c], b = K->half + (lo - K->nhit[c]);
            for (int32_t i = lo; i < hi; ++i) {
                const int32_t x = K->O[i];
                if (hit[x])
                    K->tmp[a++] = x;
                else
                    K->tmp[b++] = x;
            }
        } else {
            memcpy(K->O + lo, K->tmp + lo, (size_t)(hi - lo) * sizeof(int32_t));
        }
    }
    return NULL;
}

static int32_t kd_split_par(ax_work *w, int32_t *Q, int32_t *T, int32_t n, int dim, int32_t *tmp,
                            int nt) {
    ksplit K;
    K.w = w;
    K.D = dim == 0 ? Q : T;
    K.O = dim == 0 ? T : Q;
    K.tmp = tmp;
    K.n = n;
    K.half = n / 2;
    K.nt = nt;
    K.nhit = malloc((size_t)(nt + 1) * sizeof(int32_t));
    for (K.phase = 0; K.phase < 4; ++K.phase) {
        if (K.phase == 2) { /* exclusive prefix of the hit counts (they sum to half) */
            int32_t run = 0;
            for (int c = 0; c < nt; ++c) {
                const int32_t h = K.nhit[c];
                K.nhit[c] = run;
                run += h;
            }
        }
        atomic_init(&K.next, 0);
        gac_run_threads(nt, ksplit_thread, &K);
    }
    free(K.nhit);
    const int32_t ml = K.D[K.half - 1];
    return dim == 0 ? w->qs[ml] : w->ts[ml];
}

/* the top `depth` levels on this thread (cuts and partitions), the
 * subtrees below them as tasks; *top collects the top nodes' ids */
static void kd_top(ax_work *w, int32_t *Q, int32_t *T, int32_t n, int dim, int32_t id,
                   int32_t *tmp, int depth, kd_task *tasks, int32_t *ntask, int32_t *top,
                   int32_t *ntop, int nt) {
    if (depth == 0 || n < 2) {
        tasks[(*ntask)++] = (kd_task){Q, T, tmp, n, id, dim};
        return;
    }
    const int32_t half = n / 2;
    const int32_t cut = n >= (1 << 18) && nt > 1 ? kd_split_par(w, Q, T, n, dim, tmp, nt)
                                               : kd_split(w, Q, T, n, dim, tmp);
    const int32_t hi = id + 1, lo = id + 2 * (n - half);
    ax_node *nd = &w->nodes[id];
    nd->lo = lo;
    nd->hi = hi;
    nd->leaf = -1;
    nd->cut = cut;
    w->bnd[id] = (ax_bound){0.0, INT64_MIN / 4};
    top[(*ntop)++] = id;
    kd_top(w, Q + half, T + half, n - half, 1 - dim, hi, tmp + half, depth - 1, tasks, ntask, top,
           ntop, nt);
    kd_top(w, Q, T, half, 1 - dim, lo, tmp, depth - 1, tasks, ntask, top, ntop, nt);
}

/* kdTreeMake (chainBlock.c:166-205); the tree is built from copies: kd_build
 * permutes its lists.  Large pairs (pair_dp_team's) build their subtrees
 * below the top levels on every thread: the same tree, node for node. */
static void pair_tree(ax_work *w) {
    const int32_t nl = w->nl;
    int32_t *Q = malloc((size_t)nl * sizeof(int32_t)), *T = malloc((size_t)nl * sizeof(int32_t));
    memcpy(Q, w->qord, (size_t)nl * sizeof(int32_t));
    memcpy(T, w->tord, (size_t)nl * sizeof(int32_t));
    w->nn = 0;
    if (w->team > 1 && nl > (1 << 16)) {
        int depth = 0;
        while ((1 << depth) < 4 * w->team && depth < 12)
            ++depth;
        kd_task *tasks = malloc(sizeof(kd_task) << depth);
        int32_t *top = malloc(sizeof(int32_t) << depth), ntask = 0, ntop = 0;
        kd_top(w, Q, T, nl, 0, 0, w->tmp, depth, tasks, &ntask, top, &ntop, w->team);
        kd_job J = {w, tasks, ntask, 0};
        gac_run_threads(w->team < ntask ? w->team : ntask, kd_thread, &J);
        for (int32_t k = ntop - 1; k >= 0; --k) { /* children before parents */
            ax_node *nd = &w->nodes[top[k]];
            const ax_node *a = &w->nodes[nd->lo], *b = &w->nodes[nd->hi];
            nd->max_q = a->max_q > b->max_q ? a->max_q : b->max_q;
            nd->max_t = a->max_t > b->max_t ? a->max_t : b->max_t;
        }
        w->nn = 2 * nl - 1;
        free(tasks);
        free(top);
    } else {
        kd_build(w, Q, T, nl, 0);
    }
    free(Q);
    free(T);
}

/* findBestPredecessors (chainBlock.c:281-300) on this thread */
static int dp_fast_enabled(const ax_work *w) {
    static int env = -1;
    if (env < 0) {
        const char *v = getenv("GAC_DP_FAST");
        env = !(v && *v == '0');
    }
    return env && w->e && w->e->fast && !w->cb_gap && !w->cb_connect;
}

static void update_both(ax_work *w, int32_t leaf);

static void pair_dp_fast(ax_work *w) {
    int32_t maxsz;
    dp_leaf_positions(w, &maxsz);
    for (int32_t v = 0; v < w->nn; ++v)
        w->bnd[v].nw = INT64_MIN / 4;
    w->fallbacks = 0;
    for (int32_t i = 0; i < w->nl && !w->err; ++i) {
        const int32_t l = w->tord[i];
        double s;
        int32_t p;
        w->cut_t = i;
        best_predecessor_fast(w, l, &s, &p);
        if (dp_anomaly(w, l, i, s, maxsz)) {
            best_predecessor_fallback(w, l, i, maxsz, &s, &p);
            ++w->fallbacks;
        }
        if (s > w->total[l]) {
            w->total[l] = s;
            w->pred[l] = p;
        }
        update_both(w, l);
    }
}

/* ---- the fast DP of a large pair on several threads, exactly.
 * Leaves go in batches of K consecutive leaves (target order).  Phase A, in
 * parallel on the tree as the batch found it: every leaf's fast search and
 * anomaly check.  Phase B, in order on one thread: a leaf keeps its result
 * unless a leaf j before it in the batch -- not yet in the tree during phase
 * A -- is its candidate and scores at least its best with j's final total
 * (then j could be its true best predecessor, and the tree phase A searched
 * lacked j), or its anomaly check failed; such a leaf is searched again
 * there, on the tree with every earlier leaf in it.  A kept result is the
 * reference's by pair_dp_fast's argument: every candidate phase A could not
 * see correctly (the batch's earlier leaves) scores below the best it
 * found.  Then the leaf's total and the subtree bounds are committed. */
/* update_scores and update_nw in one walk (the same path) */
static void update_both(ax_work *w, int32_t leaf) {
    const double total = w->total[leaf];
    const int64_t v = 1024 * (int64_t)total + w->e->lin_k * ((int64_t)w->qe[leaf] + w->te[leaf]);
    const int32_t lq = w->qs[leaf], lt = w->ts[leaf];
    int32_t st_node[kStack];
    uint8_t st_dim[kStack];
#ifdef GAC_DP_STATS
    uint8_t st_dep[kStack];
    st_dep[0] = 0;
#endif
    int sp = 0;
    st_node[sp] = 0;
    st_dim[sp++] = 0;
    while (sp > 0) {
        --sp;
        const int32_t b = st_node[sp];
        const int dim = st_dim[sp];
        ax_node *nd = &w->nodes[b];
#ifdef GAC_DP_STATS
        const int dep = st_dep[sp];
        if (w->bnd[b].max_score < total)
            ++g_wr[dep / 4 < 7 ? dep / 4 : 7][0];
        if (w->bnd[b].nw < v)
            ++g_wr[dep / 4 < 7 ? dep / 4 : 7][1];
        st_dep[sp] = st_dep[sp + 1] = (uint8_t)(dep + 1);
#endif
        if (w->bnd[b].max_score < total)
            __atomic_store(&w->bnd[b].max_score, &total, __ATOMIC_RELAXED);
        if (w->bnd[b].nw < v)
            __atomic_store_n(&w->bnd[b].nw, v, __ATOMIC_RELAXED);
        if (nd->leaf < 0) {
            if (sp + 2 > kStack) {
                w_fail(w, "kd-tree deeper than %d", kStack / 2);
                return;
            }
            const int32_t coord = dim == 0 ? lq : lt;
            if (coord <= nd->cut) {
                st_node[sp] = nd->lo;
                st_dim[sp++] = (uint8_t)(1 - dim);
            }
            if (coord >= nd->cut) {
                st_node[sp] = nd->hi;
                st_dim[sp++] = (uint8_t)(1 - dim);
            }
        }
    }
}

enum { kPath = 96 };

/* the nodes update_both will touch for `leaf` (the path depends only on the
 * coordinates and the cuts): *n = their count, or -1 past kPath */
static void update_path(const ax_work *w, int32_t leaf, int32_t *out, int32_t *n) {
    const int32_t lq = w->qs[leaf], lt = w->ts[leaf];
    int32_t st_node[kStack];
    uint8_t st_dim[kStack];
    int sp = 0, m = 0;
    st_node[sp] = 0;
    st_dim[sp++] = 0;
    while (sp > 0) {
        --sp;
        const int32_t b = st_node[sp];
        const int dim = st_dim[sp];
        if (m == kPath || sp + 2 > kStack) {
            *n = -1;
            return;
        }
        out[m++] = b;
        const ax_node *nd = &w->nodes[b];
        if (nd->leaf < 0) {
            const int32_t coord = dim == 0 ? lq : lt;
            if (coord <= nd->cut) {
                st_node[sp] = nd->lo;
                st_dim[sp++] = (uint8_t)(1 - dim);
            }
            if (coord >= nd->cut) {
                st_node[sp] = nd->hi;
                st_dim[sp++] = (uint8_t)(1 - dim);
            }
        }
    }
    *n = m;
}

static double mono_s(void);

/* ---- the fast DP of a large pair on several threads, exactly.
 * One thread commits leaves in target order; the others search ahead of it
 * (best_predecessor_fast + dp_anomaly + the leaf's update path) on the tree
 * as it stands -- every leaf committed before the search started is in it,
 * later ones are still arriving (their bounds only grow, so the bounds the
 * search reads stay true bounds for every leaf it may take).  A search sees
 * only the leaves committed when it started (cut); the committer weighs the
 * ones committed since (at most kLag) exactly: each that is a candidate is
 * scored with its final total and compared with the search's best by score,
 * then DFS (node) order, the first-in-order argmax rule of pair_dp_fast; if
 * one of them scores at least the best while violating its own bounds (the
 * reference's pruning could hide it), or the search flagged an anomaly, the
 * leaf is searched again in place, on the tree with every earlier leaf in it
 * (best_predecessor_fast, else the reference order).  Then its total and
 * the bounds on its path are committed. */
enum { kLagMax = 64, kRing = 256 }; /* kRing >= lag + searchers */

typedef struct dp_slot {
    /* the committer's line: one cache-to-cache transfer per leaf */
    _Alignas(64) double s; /* search result */
    double score;          /* the leaf's block score */
    int32_t q, t, qe, te;            /* the leaf's block (read once, by its searcher) */
    int32_t p, cut, plen;
    uint8_t flag;
    _Atomic int32_t ready; /* leaf index + 1 once the slot holds its search */
    /* the applier's lines */
    _Alignas(64) int32_t path[kPath];
} dp_slot;
_Static_assert(offsetof(dp_slot, path) == 64, "dp_slot: the committer's fields fill one line");

typedef struct dp_team {
    ax_work *w;
    int32_t maxsz, lag;
    _Atomic int32_t next;      /* next leaf to search */
    _Atomic int32_t committed; /* leaves committed (target order) */
    _Atomic int32_t applied;   /* leaves whose path bounds are in the tree */
    _Atomic int quit;
    int applier;               /* a thread of its own applies the path bounds */
    uint64_t cyc_apply, napply_writes;
    dp_slot *ring;
    int32_t *cq, *ct, *cqe, *cte, *cnode; /* [kRing] committed leaves by tpos % kRing */
    int64_t *cw;
    double *ctot;
    ax_work *tw;
} dp_team;

typedef struct dp_worker {
    dp_team *T;
    int id;
} dp_worker;

static void *team_thread(void *arg) {
    dp_worker *me = arg;
    dp_team *T = me->T;
    ax_work *tw = &T->tw[me->id];
    const int32_t nl = T->w->nl;
    for (;;) {
        const int32_t i = atomic_fetch_add(&T->next, 1);
        if (i >= nl)
            break;
        int32_t cut;
        _Atomic int32_t *const seen = T->applier ? &T->applied : &T->committed;
        while ((cut = atomic_load_explicit(seen, memory_order_acquire)) + T->lag < i)
            if (atomic_load_explicit(&T->quit, memory_order_relaxed))
                return NULL;
            else
                __builtin_ia32_pause();
        dp_slot *sl = &T->ring[i % kRing];
        const int32_t l = T->w->tord[i];
        tw->cut_t = cut;
        best_predecessor_fast(tw, l, &sl->s, &sl->p);
        sl->flag = (uint8_t)dp_anomaly(tw, l, i, sl->s, T->maxsz);
        sl->cut = cut;
        sl->q = T->w->qs[l];
        sl->t = T->w->ts[l];
        sl->qe = T->w->qe[l];
        sl->te = T->w->te[l];
        sl->score = T->w->score[l];
        update_path(tw, l, sl->path, &sl->plen);
        atomic_store_explicit(&sl->ready, i + 1, memory_order_release);
    }
    return NULL;
}

/* the bounds of the committed leaves, in commit order, on a thread of its
 * own: the node writes (lines the searchers share) leave the committer's
 * critical path.  A search sees only leaves < applied, so its tree stays
 * complete for every leaf it takes. */
static void *apply_thread(void *arg) {
    dp_team *T = arg;
    ax_work *w = T->w;
    const int64_t k = w->e->lin_k;
    uint64_t cyc = 0, nwr = 0;
    for (int32_t j = 0; j < w->nl; ++j) {
        int32_t c;
        while ((c = atomic_load_explicit(&T->committed, memory_order_acquire)) <= j)
            if (atomic_load_explicit(&T->quit, memory_order_acquire))
                goto done;
            else
                __builtin_ia32_pause();
        const uint64_t k0 = __builtin_ia32_rdtsc();
        if (j + 4 < c) { /* (committed, so its slot is final: fetch its path early) */
            const dp_slot *nx = &T->ring[(j + 4) % kRing];
            for (int32_t m = 0; m < nx->plen; ++m) {
                __builtin_prefetch(&w->bnd[nx->path[m]], 1);
            }
        }
        const dp_slot *sl = &T->ring[j % kRing];
        const int32_t l = w->tord[j];
        if (sl->plen < 0) {
            update_both(w, l);
        } else {
            const double total = w->total[l];
            const int64_t v = 1024 * (int64_t)total + k * ((int64_t)sl->qe + sl->te);
            for (int32_t m = 0; m < sl->plen; ++m) {
                const int32_t b = sl->path[m];
                if (w->bnd[b].max_score < total) {
                    __atomic_store(&w->bnd[b].max_score, &total, __ATOMIC_RELAXED);
                    ++nwr;
                }
                if (w->bnd[b].nw < v) {
                    __atomic_store_n(&w->bnd[b].nw, v, __ATOMIC_RELAXED);
                    ++nwr;
                }
            }
        }
        atomic_store_explicit(&T->applied, j + 1, memory_order_release);
        cyc += __builtin_ia32_rdtsc() - k0;
    }
done:
    T->cyc_apply = cyc;
    T->napply_writes = nwr;
    return NULL;
}

static void pair_dp_team(ax_work *w, int nt, int k) {
    (void)k;
    int32_t maxsz;
    dp_leaf_positions(w, &maxsz);
    for (int32_t v = 0; v < w->nn; ++v)
        w->bnd[v].nw = INT64_MIN / 4;
    w->fallbacks = 0;
    dp_team T;
    memset(&T, 0, sizeof(T));
    T.w = w;
    T.maxsz = maxsz;
    T.ring = aligned_alloc(64, kRing * sizeof(dp_slot));
    memset(T.ring, 0, kRing * sizeof(dp_slot));
    const char *pv = getenv("GAC_DP_PF"); /* (how far ahead the committer fetches slots) */
    const int pf = pv && atoi(pv) > 0 && atoi(pv) < 64 ? atoi(pv) : 4;
    T.cq = malloc(kRing * sizeof(int32_t));
    T.ct = malloc(kRing * sizeof(int32_t));
    T.cqe = malloc(kRing * sizeof(int32_t));
    T.cte = malloc(kRing * sizeof(int32_t));
    T.cw = malloc(kRing * sizeof(int64_t));
    T.cnode = malloc(kRing * sizeof(int32_t));
    T.ctot = malloc(kRing * sizeof(double));
    const char *lv = getenv("GAC_DP_LAG");
    T.lag = lv && atoi(lv) > 0 ? (atoi(lv) < kLagMax ? atoi(lv) : kLagMax) : 32; /* (<= 64: a mask) */
    const char *av = getenv("GAC_DP_APPLY");
    T.applier = nt >= 4 && av && *av == '1'; /* (measured: in one L3 domain, slower) */
    const int nsw = nt - 1 - T.applier;
    const int ns = nsw > kRing - kLagMax ? kRing - kLagMax : nsw; /* searchers */
    T.tw = calloc((size_t)(ns > 0 ? ns : 1), sizeof(ax_work));
    for (int t = 0; t < ns; ++t) { /* shared tree, own crossover scratch and error */
        T.tw[t] = *w;
        T.tw[t].xs = NULL;
        T.tw[t].xcap = 0;
    }
    pthread_t *th = malloc((size_t)(ns > 0 ? ns : 1) * sizeof(pthread_t));
    dp_worker *wk = malloc((size_t)(ns > 0 ? ns : 1) * sizeof(dp_worker));
    int started = 0;
    pthread_t ath;
    if (T.applier && pthread_create(&ath, NULL, apply_thread, &T) != 0)
        T.applier = 0; /* (no thread: the committer applies) */
    for (int t = 0; t < ns; ++t) {
        wk[t] = (dp_worker){&T, t};
        if (pthread_create(&th[t], NULL, team_thread, &wk[t]) != 0)
            break;
        ++started;
    }
    long long redo = 0, lagsum = 0, nexact = 0, ncand = 0;
    double twait = 0, tredo = 0;
    uint64_t cyc_scan = 0, cyc_commit = 0, cyc_pref = 0, nwrites = 0;
    for (int32_t i = 0; i < w->nl && !w->err; ++i) {
        const int32_t l = w->tord[i];
        dp_slot *sl = &T.ring[i % kRing];
        double s;
        int32_t p, cut, plen;
        int again;
        if (started) {
            if (atomic_load_explicit(&sl->ready, memory_order_acquire) != i + 1) {
                const double t0 = mono_s();
                while (atomic_load_explicit(&sl->ready, memory_order_acquire) != i + 1)
                    __builtin_ia32_pause();
                twait += mono_s() - t0;
            }
            s = sl->s, p = sl->p, cut = sl->cut, plen = sl->plen, again = sl->flag;
        } else { /* (no searcher thread could start: search here) */
            w->cut_t = i;
            best_predecessor_fast(w, l, &s, &p);
            again = dp_anomaly(w, l, i, s, maxsz);
            cut = i;
            plen = -1;
            sl->q = w->qs[l], sl->t = w->ts[l], sl->qe = w->qe[l], sl->te = w->te[l];
            sl->score = w->score[l];
        }
        /* the update paths of the next searched leaves into this core's
         * cache while this one is settled */
        const uint64_t kp = __builtin_ia32_rdtsc();
        if (started && i + pf < w->nl) /* (a searcher wrote it: fetch it early) */
            __builtin_prefetch(&T.ring[(i + pf) % kRing], 0);
        if (started && !T.applier && i + 8 < w->nl) {
            const dp_slot *nx = &T.ring[(i + 8) % kRing];
            if (atomic_load_explicit(&nx->ready, memory_order_acquire) == i + 9)
                for (int32_t m = 0; m < nx->plen; ++m) {
                    __builtin_prefetch(&w->bnd[nx->path[m]], 1);
                }
        }
        if (i + 8 < w->nl) {
            const int32_t ln = w->tord[i + 8];
            __builtin_prefetch(&w->total[ln], 1);
            __builtin_prefetch(&w->pred[ln], 1);
        }
        const uint64_t k0 = __builtin_ia32_rdtsc();
        cyc_pref += k0 - kp;
        /* the leaves committed since the search started: exact, here */
        const int32_t ql = sl->q, tl = sl->t;
        const double lsc = sl->score;
        const int64_t kl = w->e->lin_k * ((int64_t)ql + tl) - 1024 * (int64_t)lsc;
        const int64_t thr = 1024 * (int64_t)(s > 1.0 ? s : 1.0) + kl;
        /* branch-free pre-filter: the candidates among them whose linear
         * bound reaches max(best, 1), or that overlap the leaf */
        uint64_t mask = 0;
        for (int32_t j = cut; j < i; ++j) {
            const int r = j % kRing;
            const int cand = (T.cq[r] < ql) & (T.ct[r] < tl);
            const int keep = (T.cw[r] >= thr) | (T.cqe[r] > ql) | (T.cte[r] > tl);
            mask |= (uint64_t)(cand & keep) << (j - cut);
        }
        for (; mask && !again; mask &= mask - 1) {
            const int32_t j = cut + __builtin_ctzll(mask);
            const int r = j % kRing;
            ++ncand;
            const int32_t c = w->tord[j];
            const double ctot = T.ctot[r];
            const int dq = ql - T.cqe[r], dt = tl - T.cte[r];
            if (dq < 0 || dt < 0) { /* overlap: its own bound */
                const int ov = -(dq < dt ? dq : dt);
                if (ov >= sl->qe - ql || ov >= T.cqe[r] - T.cq[r])
                    continue;
                const double ub = ctot + lsc - (double)gap_cost(w->e, dq + ov, dt + ov) -
                                  (double)ov * w->e->min_entry;
                if (ub < 1.0 || ub < s)
                    continue;
            }
            ++nexact;
            const double sc = ctot + lsc - connect_cost(w, c, l);
            if (sc >= 1.0 && sc >= s) {
                /* hidden by the reference's pruning?  (its bounds at c are
                 * at least c's own) */
                const double bc = ctot + lsc - gap_cost(w->e, dq, dt);
                const int64_t bl = 1024 * (int64_t)ctot - w->e->lin_k * ((int64_t)dq + dt) +
                                   1024 * (int64_t)lsc;
                if (sc > bc || 1024 * (int64_t)sc > bl) {
                    again = 1;
                    break;
                }
            }
            if (sc > 0 && (sc > s || (sc == s && T.cnode[r] < p))) {
                s = sc;
                p = T.cnode[r];
            }
        }
        const uint64_t k1 = __builtin_ia32_rdtsc();
        cyc_scan += k1 - k0;
        lagsum += i - cut;
        if (again) {
            const double t0 = mono_s();
            ++redo;
            if (T.applier) /* (the search needs every earlier leaf's bounds) */
                while (atomic_load_explicit(&T.applied, memory_order_acquire) < i)
                    __builtin_ia32_pause();
            w->cut_t = i;
            best_predecessor_fast(w, l, &s, &p);
            if (dp_anomaly(w, l, i, s, maxsz)) {
                best_predecessor_fallback(w, l, i, maxsz, &s, &p);
                ++w->fallbacks;
            }
            tredo += mono_s() - t0;
        }
        const uint64_t k2 = __builtin_ia32_rdtsc();
        if (s > w->total[l]) {
            w->total[l] = s;
            w->pred[l] = p;
        }
        const double total = w->total[l];
        const int64_t v = 1024 * (int64_t)total + w->e->lin_k * ((int64_t)sl->qe + sl->te);
        if (T.applier) {
            /* (apply_thread writes the bounds) */
        } else if (plen < 0) {
            update_both(w, l);
        } else { /* the recorded path: the same nodes update_both visits */
            for (int32_t m = 0; m < plen; ++m) {
                const int32_t b = sl->path[m];
                if (w->bnd[b].max_score < total) {
                    __atomic_store(&w->bnd[b].max_score, &total, __ATOMIC_RELAXED);
                    ++nwrites;
                }
                if (w->bnd[b].nw < v) {
                    __atomic_store_n(&w->bnd[b].nw, v, __ATOMIC_RELAXED);
                    ++nwrites;
                }
            }
        }
        const int r = i % kRing;
        T.cq[r] = ql;
        T.ct[r] = tl;
        T.cqe[r] = sl->qe;
        T.cte[r] = sl->te;
        T.cw[r] = v;
        T.ctot[r] = total;
        T.cnode[r] = w->lnode[l];
        atomic_store_explicit(&T.committed, i + 1, memory_order_release);
        cyc_commit += __builtin_ia32_rdtsc() - k2;
    }
    atomic_store_explicit(&T.quit, 1, memory_order_release);
    atomic_store(&T.next, w->nl); /* (searchers still waiting leave) */
    for (int t = 0; t < started; ++t)
        pthread_join(th[t], NULL);
    if (T.applier) {
        pthread_join(ath, NULL);
        nwrites = T.napply_writes;
    }
    for (int t = 0; t < ns; ++t) {
        if (T.tw[t].err && !w->err) {
            w->err = 1;
            memcpy(w->msg, T.tw[t].msg, sizeof(w->msg));
        }
        free(T.tw[t].xs);
    }
    if (getenv("GAC_TIMING"))
        fprintf(stderr, "[gac_axt_chain] team DP: %d searchers + 1 committer, %lld of %d leaves "
                "searched again in order (%lld by the reference order, %.3f s); the committer "
                "waited %.3f s; mean lag %.1f, scan %.2f / commit %.2f Gcycles\n", started, redo, w->nl,
                w->fallbacks, tredo, twait, (double)lagsum / (w->nl ? w->nl : 1), cyc_scan * 1e-9,
                cyc_commit * 1e-9);
    if (getenv("GAC_TIMING"))
        fprintf(stderr, "[gac_axt_chain] team DP: %.2f candidates, %.3f exact scores, %.2f node "
                "writes per leaf; prefetch section %.2f Gcycles; applier %s %.2f Gcycles\n",
                (double)ncand / (w->nl ? w->nl : 1), (double)nexact / (w->nl ? w->nl : 1),
                (double)nwrites / (w->nl ? w->nl : 1), cyc_pref * 1e-9,
                T.applier ? "thread" : "off", T.cyc_apply * 1e-9);
    free(T.tw);
    free(th);
    free(wk);
    free(T.ring);
    free(T.cq);
    free(T.ct);
    free(T.cqe);
    free(T.cte);
    free(T.cw);
    free(T.cnode);
    free(T.ctot);
}

static void pair_dp_host(ax_work *w) {
    w->fallbacks = 0;
    if (dp_fast_enabled(w) && w->team > 1) {
        pair_dp_team(w, w->team, w->team_batch);
        return;
    }
    if (dp_fast_enabled(w)) {
        pair_dp_fast(w);
#ifdef GAC_DP_STATS
        fprintf(stderr, "[dp stats] fast DP: %lld of %d leaves searched again by the reference "
                "order (%.1f nodes visited each)\n", w->fallbacks, w->nl,
                (double)g_st.ref_visits / (w->fallbacks ? w->fallbacks : 1));
        const double n = w->nl ? (double)w->nl : 1.0;
        fprintf(stderr, "[dp stats] fast: per leaf visits %.1f prune1 %.1f prune2 %.1f leaves %.2f "
                "cands %.2f wins %.2f\n", g_st.visits / n, g_st.prune1 / n, g_st.prune2 / n,
                g_st.leaves / n, g_st.cands / n, g_st.best_wins / n);
        memset(&g_st, 0, sizeof(g_st));
        for (int d = 0; d < 8; ++d)
            fprintf(stderr, "[dp stats] depth %2d-%2d: %.3f max-score writes, %.3f linear-bound "
                    "writes per leaf\n", 4 * d, 4 * d + 3, g_wr[d][0] / n, g_wr[d][1] / n);
        memset(g_wr, 0, sizeof(g_wr));
#endif
        return;
    }
    for (int32_t i = 0; i < w->nl && !w->err; ++i) {
        const int32_t l = w->tord[i];
        double s;
        int32_t p;
        best_predecessor(w, l, &s, &p);
        if (s > w->total[l]) {
            w->total[l] = s;
            w->pred[l] = p;
        }
        update_scores(w, l);
    }
#ifdef GAC_DP_STATS
    {   /* overlapping candidates per leaf, and how many violate the corner
         * bound of their own leaf node (anomalies: the reference's pruning
         * can hide them) or a linear bound s*(dq+dt) */
        long long ov = 0, neg = 0, big = 0, scans = 0, anom_c = 0, anom_l = 0, leaves_anom = 0;
        int32_t maxsz = 0;
        int32_t *qpos = malloc((size_t)w->n * 4);
        for (int32_t i = 0; i < w->nl; ++i) {
            const int32_t l = w->tord[i];
            if (w->te[l] - w->ts[l] > maxsz) maxsz = w->te[l] - w->ts[l];
            qpos[w->qord[i]] = i;
        }
        const double slope = 0.2;
        for (int32_t i = 0; i < w->nl; ++i) {
            const int32_t L = w->tord[i];
            int any = 0;
            for (int side = 0; side < 2; ++side) {
                const int32_t *ord = side ? w->qord : w->tord;
                const int32_t *st = side ? w->qs : w->ts;
                const int32_t at = side ? qpos[L] : i;
                for (int32_t j = at - 1; j >= 0 && st[ord[j]] > st[L] - maxsz; --j) {
                    const int32_t c = ord[j];
                    ++scans;
                    if (w->ts[c] >= w->ts[L] || w->qs[c] >= w->qs[L])
                        continue;
                    const int dq = w->qs[L] - w->qe[c], dt = w->ts[L] - w->te[c];
                    if (dq >= 0 && dt >= 0)
                        continue;
                    if (side == 1 && dt < 0)
                        continue; /* (counted by the t scan) */
                    ++ov;
                    const int o = -(dq < dt ? dq : dt);
                    if (o >= w->qe[L] - w->qs[L] || o >= w->qe[c] - w->qs[c]) {
                        ++big;
                        continue;
                    }
                    const double S = w->total[c] + w->score[L] - connect_cost(w, c, L);
                    int pos, adj;
                    crossover(w, w->qs[c], w->qe[c], w->ts[c], w->te[c], w->qs[L], w->qe[L],
                              w->ts[L], w->te[L], o, &pos, &adj);
                    neg += adj < 0;
                    const double Bc = w->total[c] + w->score[L] -
                                      gap_cost(w->e, dq < 0 ? 0 : dq, dt < 0 ? 0 : dt);
                    const double Bl = w->total[c] + w->score[L] - slope * (dq + dt);
                    if (S > Bc) { ++anom_c; any = 1; }
                    if (S > Bl) { ++anom_l; any = 1; }
                }
            }
            leaves_anom += any;
        }
        free(qpos);
        fprintf(stderr, "[dp stats] scans %.1f/leaf, overlapping candidates %.2f (%.2f past a block "
                "end), adj<0 %.4f, S > corner bound %.5f, S > linear bound %.5f per leaf; leaves "
                "with an anomaly %.5f; max block %d\n",
                (double)scans / w->nl, (double)ov / w->nl, (double)big / w->nl, (double)neg / w->nl,
                (double)anom_c / w->nl, (double)anom_l / w->nl, (double)leaves_anom / w->nl, maxsz);
    }
    const double n = w->nl ? (double)w->nl : 1.0;
    fprintf(stderr,
            "[dp stats] leaves %d: per leaf visits %.1f prune1 %.1f prune2 %.1f leaves %.2f "
            "cands %.2f overlaps %.2f (%.1f bases each) wins %.2f updates %.1f\n",
            w->nl, g_st.visits / n, g_st.prune1 / n, g_st.prune2 / n, g_st.leaves / n,
            g_st.cands / n, g_st.overlaps / n,
            g_st.overlaps ? (double)g_st.xover_bases / g_st.overlaps : 0.0, g_st.best_wins / n,
            g_st.updates / n);
    memset(&g_st, 0, sizeof(g_st));
#endif
}

/* the chains peelChains (chainBlock.c:311-373) takes off the tree: blocks of
 * chain c are cblk[cstart[c] .. cstart[c+1]), ascending */
typedef struct ax_chains {
    int32_t *cblk, *cstart;
    int32_t nc, nbk;
} ax_chains;

typedef struct peel_keys {
    const ax_work *w;
    dkey *dk;
} peel_keys;

static void peel_keys_fn(void *arg, int c, int64_t a, int64_t b) {
    const peel_keys *K = arg;
    (void)c;
    for (int64_t i = a; i < b; ++i)
        K->dk[i] = (dkey){K->w->total[K->w->tord[i]], (int32_t)i, K->w->tord[i]};
}

static void pair_peel(ax_work *w, const ax_pairinfo *pi, FILE *details, ax_chains *pc) {
    const int32_t nb = w->n, nl = w->nl;
    const int tm = nb > (1 << 20) && getenv("GAC_TIMING");
    const double t0 = tm ? mono_s() : 0;
    /* in totalScore order */
    dkey *dk = malloc((size_t)nl * sizeof(dkey));
    peel_keys K = {w, dk};
    par_for(nl, w->team > 1 ? w->team : 1, peel_keys_fn, &K);
    sort_desc16(dk, nl, w->team > 1 ? w->team : 1);
    const double t1 = tm ? mono_s() : 0;
    for (int32_t i = 0; i < nb; ++i)
        w->hit[i] = 0;
    int32_t *cblk = malloc((size_t)nl * sizeof(int32_t));
    int32_t *cstart = malloc((size_t)(nl + 1) * sizeof(int32_t));
    int32_t nc = 0, nbk = 0;
    for (int32_t i = 0; i < nl; ++i) {
        /* (the chain starts come in score order, at random leaves: their
         * flags, predecessors and the predecessors' nodes prefetched) */
        if (i + 32 < nl) {
            const int32_t f = dk[i + 32].v;
            __builtin_prefetch(&w->hit[f]);
            __builtin_prefetch(&w->pred[f]);
        }
        if (i + 16 < nl) {
            const int32_t f = w->pred[dk[i + 16].v];
            if (f >= 0) {
                if (w->pred_blk)
                    __builtin_prefetch(&w->hit[f]);
                else
                    __builtin_prefetch(&w->nodes[f]);
            }
        }
        const int32_t leaf = dk[i].v;
        if (w->hit[leaf])
            continue;
        if (details)
            fprintf(details, "chain %1.0f %s %d + %d %d %s %d %c %d %d %d\n", w->total[leaf],
                    pi->tname, pi->tsize, 0, w->te[leaf], pi->qname, pi->qsize, pi->strand, 0,
                    w->qe[leaf], -1);
        cstart[nc] = nbk;
        const int32_t first = nbk;
        for (int32_t lf = leaf;;) {
            w->hit[lf] = 1;
            cblk[nbk++] = lf;
            if (details)
                fprintf(details, "%d\t%f\t%d\t%d\t%d\n", w->score[lf], w->total[lf], w->ts[lf],
                        w->qs[lf], w->qe[lf] - w->qs[lf]);
            if (w->pred[lf] < 0)
                break;
            const int32_t pl = w->pred_blk ? w->pred[lf] : w->nodes[w->pred[lf]].leaf;
            if (details)
                fprintf(details, " gap %d\t%d\n", w->ts[lf] - w->te[pl], w->qs[lf] - w->qe[pl]);
            lf = pl;
            if (w->hit[lf])
                break;
        }
        /* slAddHead built the list from the end: reverse to ascending */
        for (int32_t a = first, b = nbk - 1; a < b; ++a, --b) {
            const int32_t x = cblk[a];
            cblk[a] = cblk[b];
            cblk[b] = x;
        }
        ++nc;
    }
    cstart[nc] = nbk;
    free(dk);
    if (tm)
        fprintf(stderr, "[gac_axt_chain] peel of %d leaves: keys + sort %.3f s, walk %.3f s (%d "
                "chains)\n", nl, t1 - t0, mono_s() - t1, nc);
    pc->cblk = cblk;
    pc->cstart = cstart;
    pc->nc = nc;
    pc->nbk = nbk;
}

/* scoreBlocks (chainBlock.c:296-309), slSort(chainCmpScore), then
 * chainRemovePartialOverlaps + chainMergeAbutting per chain, in that order.
 * x: the device's crossovers of the chains' adjacent overlaps, or NULL */
static void pair_finish(ax_work *w, ax_chains *pc, const ax_xres *x, ax_out *out) {
    const int32_t nc = pc->nc, nbk = pc->nbk;
    const int32_t *cblk = pc->cblk, *cstart = pc->cstart;
    dkey *ck = malloc((size_t)(nc ? nc : 1) * sizeof(dkey));
    for (int32_t c = 0; c < nc && !w->err; ++c) {
        double s = 0;
        for (int32_t j = cstart[c]; j < cstart[c + 1]; ++j) {
            s += w->score[cblk[j]];
            if (j > cstart[c]) {
                const int32_t k = x ? x->job[j] : -1;
                s -= connect_cost_pre(w, cblk[j - 1], cblk[j], k >= 0 ? &x->adj[k] : NULL);
            }
        }
        ck[c] = (dkey){s, c, c};
    }
    qsort(ck, (size_t)nc, sizeof(dkey), dkey_cmp_desc);
    ax_cb *cb = malloc((size_t)(nbk ? nbk : 1) * sizeof(ax_cb));
    out->coff = malloc((size_t)(nc + 1) * sizeof(int32_t));
    out->bt = malloc((size_t)(nbk ? nbk : 1) * sizeof(int32_t));
    out->bq = malloc((size_t)(nbk ? nbk : 1) * sizeof(int32_t));
    out->bs = malloc((size_t)(nbk ? nbk : 1) * sizeof(int32_t));
    int32_t no = 0, nob = 0;
    for (int32_t r = 0; r < nc && !w->err; ++r) {
        const int32_t c = ck[r].v, b0 = cstart[c], b1 = cstart[c + 1];
        for (int32_t j = b0; j < b1; ++j) {
            const int32_t b = cblk[j];
            cb[j] = (ax_cb){w->qs[b], w->qe[b], w->ts[b], w->te[b], j + 1 < b1 ? j + 1 : -1};
        }
        const int32_t head = remove_partial_overlaps(w, cb, b0, x);
        out->coff[no] = nob;
        for (int32_t b = head; b >= 0; b = cb[b].next) {
            out->bt[nob] = cb[b].ts;
            out->bq[nob] = cb[b].qs;
            out->bs[nob] = cb[b].qe - cb[b].qs;
            ++nob;
        }
        if (nob > out->coff[no])
            ++no;
    }
    out->coff[no] = nob;
    out->n_chains = no;
    free(ck);
    free(cb);
    free(pc->cblk);
    free(pc->cstart);
    pc->cblk = pc->cstart = NULL;
}

/* pair_finish of a large pair on every thread: scoreBlocks per chain,
 * the sort, overlap removal per chain (each chain's blocks are its own
 * slice of cb), then the surviving blocks gathered in sort order -- the
 * same output; an error is the first failing chain's, as in pair_finish */
typedef struct fin_job {
    ax_work *w;
    ax_work *tw;          /* per-thread copies (crossover scratch, errors) */
    const ax_chains *pc;
    dkey *ck;
    ax_cb *cb;
    int32_t *head, *cnt, *pos;
    ax_out *out;
    int32_t n;
    int phase;
    _Atomic int32_t next, wid;
    pthread_mutex_t mu;
    int32_t err_at;
    char msg[512];
} fin_job;

static void *fin_thread(void *arg) {
    fin_job *F = arg;
    const int id = atomic_fetch_add(&F->wid, 1);
    ax_work *w = &F->tw[id];
    const int32_t *cblk = F->pc->cblk, *cstart = F->pc->cstart;
    for (;;) {
        const int32_t a = atomic_fetch_add(&F->next, 256);
        if (a >= F->n)
            break;
        const int32_t b = a + 256 < F->n ? a + 256 : F->n;
        for (int32_t r = a; r < b; ++r) {
            if (F->phase == 0) { /* scoreBlocks of chain r */
                if (r + 4 < F->n) { /* (the blocks are at random places) */
                    const int32_t k4 = cblk[cstart[r + 4]];
                    __builtin_prefetch(&w->score[k4]);
                    __builtin_prefetch(&w->qs[k4]);
                    __builtin_prefetch(&w->qe[k4]);
                    __builtin_prefetch(&w->ts[k4]);
                    __builtin_prefetch(&w->te[k4]);
                }
                double sc = 0;
                for (int32_t j = cstart[r]; j < cstart[r + 1]; ++j) {
                    sc += w->score[cblk[j]];
                    if (j > cstart[r])
                        sc -= connect_cost(w, cblk[j - 1], cblk[j]);
                }
                F->ck[r] = (dkey){sc, r, r};
            } else if (F->phase == 1) { /* overlap removal of the r-th chain */
                /* (chains in score order, at random places: the chain's
                 * start, first block and its coordinates prefetched) */
                if (r + 8 < F->n)
                    __builtin_prefetch(&cstart[F->ck[r + 8].v]);
                if (r + 4 < F->n)
                    __builtin_prefetch(&cblk[cstart[F->ck[r + 4].v]]);
                if (r + 2 < F->n) {
                    const int32_t j2 = cstart[F->ck[r + 2].v], k2 = cblk[j2];
                    __builtin_prefetch(&w->qs[k2]);
                    __builtin_prefetch(&w->qe[k2]);
                    __builtin_prefetch(&w->ts[k2]);
                    __builtin_prefetch(&w->te[k2]);
                    __builtin_prefetch(&F->cb[j2], 1);
                }
                const int32_t c = F->ck[r].v, b0 = cstart[c], b1 = cstart[c + 1];
                for (int32_t j = b0; j < b1; ++j) {
                    const int32_t k = cblk[j];
                    F->cb[j] = (ax_cb){w->qs[k], w->qe[k], w->ts[k], w->te[k], j + 1 < b1 ? j + 1 : -1};
                }
                const int32_t h = remove_partial_overlaps(w, F->cb, b0, NULL);
                F->head[r] = h;
                int32_t m = 0;
                for (int32_t x = h; x >= 0; x = F->cb[x].next)
                    ++m;
                F->cnt[r] = m;
            } else { /* copy the r-th chain's blocks out */
                if (r + 4 < F->n && F->head[r + 4] >= 0)
                    __builtin_prefetch(&F->cb[F->head[r + 4]]);
                int32_t o = F->pos[r];
                for (int32_t x = F->head[r]; x >= 0; x = F->cb[x].next, ++o) {
                    F->out->bt[o] = F->cb[x].ts;
                    F->out->bq[o] = F->cb[x].qs;
                    F->out->bs[o] = F->cb[x].qe - F->cb[x].qs;
                }
            }
            if (w->err) {
                pthread_mutex_lock(&F->mu);
                if (F->err_at < 0 || r < F->err_at) {
                    F->err_at = r;
                    memcpy(F->msg, w->msg, sizeof(F->msg));
                }
                pthread_mutex_unlock(&F->mu);
                w->err = 0;
            }
        }
    }
    return NULL;
}

static void pair_finish_team(ax_work *w, ax_chains *pc, ax_out *out) {
    const int32_t nc = pc->nc, nbk = pc->nbk, nt = w->team;
    fin_job F;
    memset(&F, 0, sizeof(F));
    F.w = w;
    F.pc = pc;
    F.n = nc;
    F.err_at = -1;
    pthread_mutex_init(&F.mu, NULL);
    F.tw = calloc((size_t)nt, sizeof(ax_work));
    for (int t = 0; t < nt; ++t) {
        F.tw[t] = *w;
        F.tw[t].xs = NULL;
        F.tw[t].xcap = 0;
        F.tw[t].err = 0;
    }
    const int tm = w->n > (1 << 20) && getenv("GAC_TIMING");
    double tf[5] = {tm ? mono_s() : 0, 0, 0, 0, 0};
    F.ck = malloc((size_t)(nc ? nc : 1) * sizeof(dkey));
    F.phase = 0;
    gac_run_threads(nt, fin_thread, &F);
    if (tm) tf[1] = mono_s();
    if (F.err_at < 0) {
        sort_desc16(F.ck, nc, nt);
        if (tm) tf[2] = mono_s();
        F.cb = malloc((size_t)(nbk ? nbk : 1) * sizeof(ax_cb));
        F.head = malloc((size_t)(nc ? nc : 1) * sizeof(int32_t));
        F.cnt = malloc((size_t)(nc ? nc : 1) * sizeof(int32_t));
        F.pos = malloc((size_t)(nc ? nc : 1) * sizeof(int32_t));
        F.phase = 1;
        atomic_store(&F.next, 0);
        atomic_store(&F.wid, 0);
        gac_run_threads(nt, fin_thread, &F);
        if (tm) tf[3] = mono_s();
    }
    if (F.err_at >= 0) {
        w->err = 1;
        memcpy(w->msg, F.msg, sizeof(w->msg));
    } else {
        out->coff = malloc((size_t)(nc + 1) * sizeof(int32_t));
        int32_t no = 0, nob = 0;
        for (int32_t r = 0; r < nc; ++r) {
            F.pos[r] = nob;
            if (F.cnt[r]) {
                out->coff[no++] = nob;
                nob += F.cnt[r];
            }
        }
        out->coff[no] = nob;
        out->n_chains = no;
        out->bt = malloc((size_t)(nob ? nob : 1) * sizeof(int32_t));
        out->bq = malloc((size_t)(nob ? nob : 1) * sizeof(int32_t));
        out->bs = malloc((size_t)(nob ? nob : 1) * sizeof(int32_t));
        F.out = out;
        F.phase = 2;
        atomic_store(&F.next, 0);
        atomic_store(&F.wid, 0);
        gac_run_threads(nt, fin_thread, &F);
        if (tm) {
            tf[4] = mono_s();
            fprintf(stderr, "[gac_axt_chain] finish of %d chains (%d threads): scores %.3f, sort "
                    "%.3f, overlaps %.3f, copy-out %.3f s\n", nc, nt, tf[1] - tf[0],
                    tf[2] - tf[1], tf[3] - tf[2], tf[4] - tf[3]);
        }
    }
    for (int t = 0; t < nt; ++t)
        free(F.tw[t].xs);
    free(F.tw);
    free(F.ck);
    free(F.cb);
    free(F.head);
    free(F.cnt);
    free(F.pos);
    pthread_mutex_destroy(&F.mu);
    free(pc->cblk);
    free(pc->cstart);
    pc->cblk = pc->cstart = NULL;
}

/* pair_leaves + pair_tree from the device's build (gac_kd_trees; the arrays
 * were adopted by run_pair): the totals and the bounds to start from */
static int32_t pair_prebuilt(ax_work *w) {
    w->nl = w->pre->nl;
    for (int32_t i = 0; i < w->n; ++i) {
        w->total[i] = w->score[i];
        w->pred[i] = -1;
    }
    w->nn = w->nl ? 2 * w->nl - 1 : 0;
    for (int32_t v = 0; v < w->nn; ++v)
        w->bnd[v] = (ax_bound){0.0, INT64_MIN / 4};
    return w->nl;
}

static double mono_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void chain_pair(ax_work *w, const ax_pairinfo *pi, FILE *details, ax_out *out) {
    memset(out, 0, sizeof(*out));
    /* GAC_TIMING: the phases of pairs of over a million blocks */
    const int tm = w->n > (1 << 20) && getenv("GAC_TIMING");
    double t0 = tm ? mono_s() : 0, t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    if ((w->pre ? pair_prebuilt(w) : pair_leaves(w)) == 0) {
        out->coff = calloc(1, sizeof(int32_t));
        return;
    }
    if (tm) t1 = mono_s();
    if (!w->pre)
        pair_tree(w);
    if (tm) t2 = mono_s();
    pair_dp_host(w);
    if (w->err)
        return;
    if (tm) t3 = mono_s();
    ax_chains pc;
    pair_peel(w, pi, details, &pc);
    if (tm) t4 = mono_s();
    if (w->team > 1 && !details)
        pair_finish_team(w, &pc, out);
    else
        pair_finish(w, &pc, NULL, out);
    if (tm)
        fprintf(stderr, "[gac_axt_chain] pair %s%c%s, %d leaves: leaves %.3f tree %.3f DP %.3f "
                "(%lld reference-order searches) peel %.3f finish %.3f s\n", pi->qname, pi->strand,
                pi->tname, w->nl, t1 - t0, t2 - t1, t3 - t2, w->fallbacks, t4 - t3, mono_s() - t4);
}

/* ------------------------------------------------------------------ chainBlocks */
static void work_reserve(ax_work *w, int32_t n);

/* kent's chainBlocks (kent/src/lib/chainBlock.c:392-452) with the caller's
 * cost functions: leaves (zero-length blocks skipped), kdTreeMake,
 * findBestPredecessors, peelChains, scoreBlocks with connect(), and the
 * stable chainCmpScore sort -- on the calling thread. */
int gac_chain_blocks(int32_t n, const int32_t *qs, const int32_t *qe, const int32_t *ts,
                     const int32_t *te, const int32_t *score, gac_connect_fn connect,
                     gac_gapcost_fn gap, void *user, const char *qname, int32_t qsize,
                     char qstrand, const char *tname, int32_t tsize, FILE *details,
                     gac_block_chains **out) {
    gac_clear_error();
    if (!out || n < 0 || !connect || !gap || (n && (!qs || !qe || !ts || !te || !score)))
        return gac_fail(GAC_E_ARG, "gac_chain_blocks: bad argument");
    *out = NULL;
    ax_work w;
    memset(&w, 0, sizeof(w));
    w.cb_connect = connect;
    w.cb_gap = gap;
    w.cb_user = user;
    w.n = n;
    w.qs = qs;
    w.qe = qe;
    w.ts = ts;
    w.te = te;
    w.score = score;
    work_reserve(&w, n);
    gac_block_chains *r = calloc(1, sizeof(*r));
    int rc = GAC_OK;
    if (n > 0 && pair_leaves(&w) > 0) {
        pair_tree(&w);
        pair_dp_host(&w);
        if (!w.err) {
            const ax_pairinfo pi = {tname ? tname : "", qname ? qname : "", tsize, qsize, qstrand};
            ax_chains pc;
            pair_peel(&w, &pi, details, &pc);
            dkey *ck = malloc((size_t)(pc.nc ? pc.nc : 1) * sizeof(dkey));
            for (int32_t c = 0; c < pc.nc; ++c) { /* scoreBlocks (chainBlock.c:311-325) */
                double sc = 0;
                for (int32_t j = pc.cstart[c]; j < pc.cstart[c + 1]; ++j) {
                    sc += score[pc.cblk[j]];
                    if (j > pc.cstart[c])
                        sc -= connect(pc.cblk[j - 1], pc.cblk[j], user);
                }
                ck[c] = (dkey){sc, c, c};
            }
            qsort(ck, (size_t)pc.nc, sizeof(dkey), dkey_cmp_desc);
            r->n_chains = pc.nc;
            r->score = malloc((size_t)(pc.nc ? pc.nc : 1) * sizeof(double));
            r->off = malloc((size_t)(pc.nc + 1) * sizeof(int32_t));
            r->blk = malloc((size_t)(pc.nbk ? pc.nbk : 1) * sizeof(int32_t));
            int32_t k = 0;
            for (int32_t i = 0; i < pc.nc; ++i) {
                const int32_t c = ck[i].v;
                r->score[i] = ck[i].k;
                r->off[i] = k;
                for (int32_t j = pc.cstart[c]; j < pc.cstart[c + 1]; ++j)
                    r->blk[k++] = pc.cblk[j];
            }
            r->off[pc.nc] = k;
            free(ck);
            free(pc.cblk);
            free(pc.cstart);
        }
    } else {
        r->off = calloc(1, sizeof(int32_t));
    }
    if (w.err)
        rc = gac_fail(GAC_E_ARG, "%s", w.msg);
    free(w.total);
    free(w.pred);
    free(w.hit);
    free(w.tord);
    free(w.qord);
    free(w.tmp);
    free(w.nodes);
    free(w.lnode);
    free(w.qpos);
    free(w.tpos);
    free(w.tbox);
    free(w.qbox);
    free(w.qtp);
    free(w.bnd);
    free(w.xs);
    if (rc != GAC_OK) {
        gac_block_chains_free(r);
        return rc;
    }
    if (!r->off)
        r->off = calloc(1, sizeof(int32_t));
    *out = r;
    return GAC_OK;
}

void gac_block_chains_free(gac_block_chains *c) {
    if (!c)
        return;
    free(c->score);
    free(c->off);
    free(c->blk);
    free(c);
}

/* ------------------------------------------------------------------ threads */
typedef struct ax_job {
    const ax_env *e;
    gac_ctx *ctx;
    const gac_axt_input *in;
    /* folded blocks per pair: [poff[p], poff[p+1]) */
    const int64_t *poff;
    const int32_t *qs, *qe, *ts, *te, *score;
    const ax_pairinfo *info;
    const int32_t *order; /* pairs, largest first */
    int64_t n_pairs;
    _Atomic int64_t next;
    ax_out *out;
    int want_details;
} ax_job;

static void work_reserve(ax_work *w, int32_t n) {
    if ((size_t)n <= w->cap_n)
        return;
    const size_t c = (size_t)n + 16;
    w->total = realloc(w->total, c * sizeof(double));
    w->pred = realloc(w->pred, c * sizeof(int32_t));
    w->hit = realloc(w->hit, c);
    w->tord = realloc(w->tord, c * sizeof(int32_t));
    w->qord = realloc(w->qord, c * sizeof(int32_t));
    w->tmp = realloc(w->tmp, c * sizeof(int32_t));
    w->nodes = realloc(w->nodes, 2 * c * sizeof(ax_node));
    w->lnode = realloc(w->lnode, c * sizeof(int32_t));
    w->qpos = realloc(w->qpos, c * sizeof(int32_t));
    w->tpos = realloc(w->tpos, c * sizeof(int32_t));
    w->tbox = realloc(w->tbox, 4 * c * sizeof(int32_t));
    w->qbox = realloc(w->qbox, 4 * c * sizeof(int32_t));
    w->qtp = realloc(w->qtp, c * sizeof(int32_t));
    w->bnd = realloc(w->bnd, 2 * c * sizeof(ax_bound));
    w->cap_n = c;
}

/* chain pair p with w (its buffers reused across pairs) */
static void run_pair(ax_job *J, ax_work *w, int32_t p) {
    const int64_t b0 = J->poff[p];
    const int32_t n = (int32_t)(J->poff[p + 1] - b0);
    ax_out *o = &J->out[p];
    w->err = 0;
    w->msg[0] = 0;
    if (gac_genome_view(J->ctx, GAC_Q, J->in->q_seq[p], &w->q.v) != GAC_OK ||
        gac_genome_view(J->ctx, GAC_T, J->in->t_seq[p], &w->t.v) != GAC_OK) {
        memset(o, 0, sizeof(*o));
        o->err = 1;
        snprintf(o->msg, sizeof(o->msg), "pair %d: no host sequence", p);
        return;
    }
    w->q.minus = J->in->q_strand[p] ? 1 : 0;
    w->t.minus = 0;
    w->n = n;
    w->qs = J->qs + b0;
    w->qe = J->qe + b0;
    w->ts = J->ts + b0;
    w->te = J->te + b0;
    w->score = J->score + b0;
    work_reserve(w, n);
    if (w->pre) { /* the device's leaves and tree become this pair's arrays */
        free(w->tord);
        free(w->qord);
        free(w->lnode);
        free(w->nodes);
        w->tord = w->pre->tord;
        w->qord = w->pre->qord;
        w->lnode = w->pre->lnode;
        w->nodes = (ax_node *)w->pre->nodes;
        w->cap_n = 0; /* (not reusable at work_reserve's sizes) */
    }
    char *dbuf = NULL;
    size_t dlen = 0;
    FILE *df = J->want_details ? open_memstream(&dbuf, &dlen) : NULL;
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    chain_pair(w, &J->info[p], df, o);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    o->secs = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
    if (df) {
        fclose(df);
        o->details = dbuf;
        o->details_len = dlen;
    }
    if (w->err) {
        o->err = 1;
        memcpy(o->msg, w->msg, sizeof(o->msg));
    }
}

static void work_free(ax_work *w) {
    free(w->total);
    free(w->pred);
    free(w->hit);
    free(w->tord);
    free(w->qord);
    free(w->tmp);
    free(w->nodes);
    free(w->lnode);
    free(w->qpos);
    free(w->tpos);
    free(w->tbox);
    free(w->qbox);
    free(w->qtp);
    free(w->bnd);
    free(w->xs);
}

typedef struct team_run {
    ax_job *J;
    const ax_env *env;
    ax_pre *pre; /* the pair's leaves and tree built on the device, or NULL */
    int32_t p;
    int team, batch, started, pin;
    _Atomic int done; /* (its pair's chains are in J->out) */
    cpu_set_t cpus; /* (pin) the L3 domain the team runs in */
    pthread_t th;
} team_run;

/* the L3 domains (sysfs cache/index3/shared_cpu_list) of the CPUs this
 * process may run on, in CPU order; 0 when sysfs does not say.  A team's
 * threads pass every committed bound and search slot between them, so they
 * share one L3 (an L3 line moves between cores in tens of ns, a line from
 * another CCD or socket takes several times that) */
typedef struct l3_dom {
    cpu_set_t set;
    int n;
} l3_dom;

static int l3_domains(l3_dom *d, int max) {
    cpu_set_t ok;
    if (sched_getaffinity(0, sizeof(ok), &ok) != 0)
        return 0;
    int nd = 0;
    for (int c = 0; c < CPU_SETSIZE && nd < max; ++c) {
        if (!CPU_ISSET(c, &ok))
            continue;
        int seen = 0;
        for (int k = 0; k < nd && !seen; ++k)
            seen = CPU_ISSET(c, &d[k].set);
        if (seen)
            continue;
        char path[96], buf[1024];
        snprintf(path, sizeof(path), "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", c);
        FILE *f = fopen(path, "r");
        if (!f)
            return 0;
        const int got = fgets(buf, sizeof(buf), f) != NULL;
        fclose(f);
        if (!got)
            return 0;
        CPU_ZERO(&d[nd].set);
        for (char *q = buf; *q && *q != '\n';) { /* "a-b,c,..." */
            char *e;
            const long a = strtol(q, &e, 10);
            long b = a;
            if (e == q)
                return 0;
            if (*e == '-')
                b = strtol(e + 1, &e, 10);
            for (long x = a; x <= b && x < CPU_SETSIZE; ++x)
                if (x >= 0 && CPU_ISSET((int)x, &ok))
                    CPU_SET((int)x, &d[nd].set);
            q = *e == ',' ? e + 1 : e;
        }
        if (!CPU_ISSET(c, &d[nd].set))
            CPU_SET(c, &d[nd].set);
        d[nd].n = CPU_COUNT(&d[nd].set);
        ++nd;
    }
    return nd;
}

static void *team_runner(void *arg) {
    team_run *R = arg;
    if (R->pin) /* (its searchers and applier inherit the mask) */
        pthread_setaffinity_np(pthread_self(), sizeof(R->cpus), &R->cpus);
    ax_work w;
    memset(&w, 0, sizeof(w));
    w.e = R->env;
    w.team = R->team;
    w.team_batch = R->batch;
    w.pre = R->pre;
    run_pair(R->J, &w, R->p);
    work_free(&w);
    atomic_store_explicit(&R->done, 1, memory_order_release);
    return NULL;
}

static void *ax_thread(void *arg) {
    ax_job *J = arg;
    ax_work w;
    memset(&w, 0, sizeof(w));
    w.e = J->e;
    for (;;) {
        const int64_t k = atomic_fetch_add(&J->next, 1);
        if (k >= J->n_pairs)
            break;
        run_pair(J, &w, J->order[k]);
    }
    work_free(&w);
    return NULL;
}

/* ------------------------------------------------------------------ device DP
 * GAC_AXT_DP=gpu: the kd-tree DP of every pair in one gac_chain_dp launch
 * (one wave per pair), and the crossovers of the peeled chains' adjacent
 * overlaps (scoreBlocks, chainRemovePartialOverlaps) in one gac_crossovers
 * batch; tree building, peeling and list surgery stay on host threads.
 * Phases (threads over pairs, largest first): 1 leaves + tree + export,
 * [device DP], 2 import + peel + crossover jobs, [device crossovers],
 * 3 scoreBlocks + sort + overlap removal. */
typedef struct ax_gpair {
    ax_work w;          /* this pair's own buffers (they live across phases) */
    int ok;             /* genome views resolved */
    /* export: tree and leaves */
    int32_t *na, *nb;   /* [nn][4], [nn][2] */
    int32_t *lf, *lsc, *lnode; /* [nl][4], [nl], [nl] */
    int64_t *poff;      /* [nl + 1], local */
    int32_t *path;
    int64_t *ooff;      /* [nl + 1], local: overlapping candidates (fast DP) */
    int32_t *ovl;
    /* peel */
    ax_chains pc;
    int32_t *xjob;      /* [nbk] global crossover job or -1 */
    int32_t nx;         /* this pair's jobs */
    int32_t *xl;        /* [nx][5] lqe, lte, rqs, rts, ov */
    double t0;
} ax_gpair;

typedef struct ax_gjob {
    ax_job *J;
    ax_gpair *G;
    int phase;
    _Atomic int64_t next;
    double t_leaves, t_tree, t_export; /* (phase 1 laps summed over threads; racy, timing only) */
    /* the DP's inputs built on the device (gac_chain_dp_blocks): the pairs'
     * blocks packed at boff[k] (phase 1), the results by packed block */
    int dev_tree;
    const int64_t *boff;
    int32_t *box, *bscore;
    const int32_t *tord;
    const int64_t *btotal;
    const int32_t *bpred;
    /* device results */
    const int64_t *leaf_off, *xoff;
    const int64_t *total;
    const int32_t *pred;
    const int32_t *xpos, *xadj, *xlqe, *xlte, *xrqs, *xrts, *xov;
} ax_gjob;

static double gnow(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

/* the nodes updateScoresOnWay's descent reaches for leaf block l */
static int64_t leaf_path(const ax_work *w, int32_t l, int32_t **path, int64_t *len, int64_t *cap) {
    const int32_t lq = w->qs[l], lt = w->ts[l];
    int32_t st_node[kStack];
    uint8_t st_dim[kStack];
    int sp = 0;
    int64_t n0 = *len;
    st_node[sp] = 0;
    st_dim[sp++] = 0;
    while (sp > 0) {
        --sp;
        const int32_t b = st_node[sp];
        const int dim = st_dim[sp];
        if (*len == *cap) {
            *cap = *cap * 2 + 64;
            *path = realloc(*path, (size_t)*cap * sizeof(int32_t));
        }
        (*path)[(*len)++] = b;
        const ax_node *nd = &w->nodes[b];
        if (nd->leaf < 0) {
            if (sp + 2 > kStack)
                return -1;
            const int32_t coord = dim == 0 ? lq : lt;
            if (coord <= nd->cut) {
                st_node[sp] = nd->lo;
                st_dim[sp++] = (uint8_t)(1 - dim);
            }
            if (coord >= nd->cut) {
                st_node[sp] = nd->hi;
                st_dim[sp++] = (uint8_t)(1 - dim);
            }
        }
    }
    return *len - n0;
}

static void gpair_export(ax_gpair *G) {
    ax_work *w = &G->w;
    const int32_t nn = w->nn, nl = w->nl;
    G->na = malloc((size_t)nn * 4 * sizeof(int32_t));
    G->nb = malloc((size_t)nn * 2 * sizeof(int32_t));
    G->lf = malloc((size_t)nl * 4 * sizeof(int32_t));
    G->lsc = malloc((size_t)nl * sizeof(int32_t));
    G->lnode = malloc((size_t)nl * sizeof(int32_t));
    G->poff = malloc((size_t)(nl + 1) * sizeof(int64_t));
    int32_t *end = malloc((size_t)nn * sizeof(int32_t));
    uint8_t *dim = malloc((size_t)nn);
    int32_t *pos = w->tmp; /* leaf position of each block */
    for (int32_t i = 0; i < nl; ++i)
        pos[w->tord[i]] = i;
    for (int32_t v = nn - 1; v >= 0; --v)
        end[v] = w->nodes[v].leaf >= 0 ? v + 1 : end[w->nodes[v].lo];
    dim[0] = 0;
    for (int32_t v = 0; v < nn; ++v) {
        const ax_node *nd = &w->nodes[v];
        if (nd->leaf >= 0) {
            const int32_t l = nd->leaf;
            G->na[4 * v] = nd->max_q;
            G->na[4 * v + 1] = nd->max_t;
            G->na[4 * v + 2] = w->qs[l];
            G->na[4 * v + 3] = w->ts[l];
            G->nb[2 * v] = v + 1;
            G->nb[2 * v + 1] = ~pos[l];
            G->lnode[pos[l]] = v;
        } else {
            dim[nd->hi] = dim[nd->lo] = (uint8_t)(1 - dim[v]);
            G->na[4 * v] = nd->max_q;
            G->na[4 * v + 1] = nd->max_t;
            G->na[4 * v + 2] = nd->cut;
            G->na[4 * v + 3] = nd->lo;
            G->nb[2 * v] = end[v];
            G->nb[2 * v + 1] = dim[v];
        }
    }
    int64_t len = 0, cap = (int64_t)nl * 24 + 64;
    G->path = malloc((size_t)cap * sizeof(int32_t));
    G->poff[0] = 0;
    for (int32_t i = 0; i < nl && !w->err; ++i) {
        const int32_t l = w->tord[i];
        G->lf[4 * i] = w->qs[l];
        G->lf[4 * i + 1] = w->qe[l];
        G->lf[4 * i + 2] = w->ts[l];
        G->lf[4 * i + 3] = w->te[l];
        G->lsc[i] = w->score[l];
        if (leaf_path(w, l, &G->path, &len, &cap) < 0)
            w_fail(w, "kd-tree deeper than %d", kStack / 2);
        G->poff[i + 1] = len;
    }
    free(end);
    free(dim);
    G->ooff = NULL;
    G->ovl = NULL;
    if (dp_fast_enabled(w)) {
        /* each leaf's overlapping candidates (dp_overlaps: leaf nodes; a
         * single -1 past the cap sends the leaf to the reference search;
         * GAC_DP_OVCAP lowers the cap -- a test hook for that path) */
        enum { kOvCap = 1024 };
        static int ov_cap = -1;
        if (ov_cap < 0) {
            const char *oc = getenv("GAC_DP_OVCAP");
            const int v = oc && *oc ? atoi(oc) : kOvCap;
            ov_cap = v >= 0 && v <= kOvCap ? v : kOvCap;
        }
        int32_t maxsz, buf[kOvCap];
        dp_leaf_positions(w, &maxsz);
        int64_t on = 0, ocap = nl + 64;
        G->ooff = malloc((size_t)(nl + 1) * sizeof(int64_t));
        G->ovl = malloc((size_t)ocap * sizeof(int32_t));
        G->ooff[0] = 0;
        for (int32_t i = 0; i < nl; ++i) {
            w->cut_t = i;
            int k = dp_overlaps(w, w->tord[i], i, maxsz, buf, ov_cap);
            if (k < 0) {
                buf[0] = -1;
                k = 1;
            }
            if (on + k > ocap) {
                ocap = 2 * (on + k) + 64;
                G->ovl = realloc(G->ovl, (size_t)ocap * sizeof(int32_t));
            }
            memcpy(G->ovl + on, buf, (size_t)k * sizeof(int32_t));
            on += k;
            G->ooff[i + 1] = on;
        }
    }
}

static void gpair_free_export(ax_gpair *G) {
    free(G->na);
    free(G->nb);
    free(G->lf);
    free(G->lsc);
    free(G->lnode);
    free(G->poff);
    free(G->path);
    free(G->ooff);
    free(G->ovl);
    G->na = G->nb = G->lf = G->lsc = G->lnode = G->path = G->ovl = NULL;
    G->poff = G->ooff = NULL;
}

static void *gdp_thread(void *arg) {
    ax_gjob *X = arg;
    ax_job *J = X->J;
    for (;;) {
        const int64_t k = atomic_fetch_add(&X->next, 1);
        if (k >= J->n_pairs)
            break;
        const int32_t p = J->order[k];
        ax_gpair *G = &X->G[k]; /* (by place in J->order: the job may be a subset) */
        ax_work *w = &G->w;
        ax_out *o = &J->out[p];
        const double t0 = gnow();
        if (X->phase == 1) {
            memset(o, 0, sizeof(*o));
            w->e = J->e;
            if (gac_genome_view(J->ctx, GAC_Q, J->in->q_seq[p], &w->q.v) != GAC_OK ||
                gac_genome_view(J->ctx, GAC_T, J->in->t_seq[p], &w->t.v) != GAC_OK) {
                o->err = 1;
                snprintf(o->msg, sizeof(o->msg), "pair %d: no host sequence", p);
                continue;
            }
            G->ok = 1;
            w->q.minus = J->in->q_strand[p] ? 1 : 0;
            w->t.minus = 0;
            const int64_t b0 = J->poff[p];
            w->n = (int32_t)(J->poff[p + 1] - b0);
            w->qs = J->qs + b0;
            w->qe = J->qe + b0;
            w->ts = J->ts + b0;
            w->te = J->te + b0;
            w->score = J->score + b0;
            if (X->dev_tree) { /* only what peel and finish use; the blocks packed */
                const size_t c = (size_t)w->n + 16;
                w->total = malloc(c * sizeof(double));
                w->pred = malloc(c * sizeof(int32_t));
                w->hit = malloc(c);
                w->tord = malloc(c * sizeof(int32_t));
                int32_t *bx = X->box + 4 * X->boff[k], *bs = X->bscore + X->boff[k];
                for (int32_t i = 0; i < w->n; ++i) {
                    bx[4 * i] = w->qs[i];
                    bx[4 * i + 1] = w->qe[i];
                    bx[4 * i + 2] = w->ts[i];
                    bx[4 * i + 3] = w->te[i];
                    bs[i] = w->score[i];
                }
                G->t0 += gnow() - t0;
                continue;
            }
            work_reserve(w, w->n);
            const double ta = gnow();
            if (pair_leaves(w) > 0) {
                const double tb = gnow();
                pair_tree(w);
                const double tc = gnow();
                gpair_export(G);
                const double td = gnow();
                X->t_leaves += tb - ta; /* (phase laps, GAC_TIMING; summed over threads) */
                X->t_tree += tc - tb;
                X->t_export += td - tc;
            }
        } else if (X->phase == 2) {
            if (!G->ok || w->err)
                continue;
            if (X->dev_tree) {
                const int64_t lo = X->leaf_off[k], bo = X->boff[k];
                w->nl = (int32_t)(X->leaf_off[k + 1] - lo);
                memcpy(w->tord, X->tord + lo, (size_t)w->nl * sizeof(int32_t));
                for (int32_t i = 0; i < w->n; ++i) {
                    w->total[i] = (double)X->btotal[bo + i];
                    w->pred[i] = X->bpred[bo + i];
                }
                w->pred_blk = 1;
            }
            if (w->nl == 0) {
                o->coff = calloc(1, sizeof(int32_t));
                continue;
            }
            const int64_t lo = X->leaf_off[k];
            for (int32_t i = 0; i < w->nl && !X->dev_tree; ++i) {
                const int32_t l = w->tord[i];
                w->total[l] = (double)X->total[lo + i];
                w->pred[l] = X->pred[lo + i];
            }
            gpair_free_export(G);
            char *dbuf = NULL;
            size_t dlen = 0;
            FILE *df = J->want_details ? open_memstream(&dbuf, &dlen) : NULL;
            pair_peel(w, &J->info[p], df, &G->pc);
            if (df) {
                fclose(df);
                o->details = dbuf;
                o->details_len = dlen;
            }
            /* the chains' adjacent overlapping blocks that take a crossover */
            G->xjob = malloc((size_t)(G->pc.nbk ? G->pc.nbk : 1) * sizeof(int32_t));
            G->xl = NULL;
            G->nx = 0;
            int32_t cap = 0;
            for (int32_t c = 0; c < G->pc.nc; ++c)
                for (int32_t j = G->pc.cstart[c]; j < G->pc.cstart[c + 1]; ++j) {
                    G->xjob[j] = -1;
                    if (j == G->pc.cstart[c])
                        continue;
                    const int32_t a = G->pc.cblk[j - 1], b = G->pc.cblk[j];
                    const int dq = w->qs[b] - w->qe[a], dt = w->ts[b] - w->te[a];
                    if (dq >= 0 && dt >= 0)
                        continue;
                    const int ov = -(dq < dt ? dq : dt);
                    if (ov >= w->qe[b] - w->qs[b] || ov >= w->qe[a] - w->qs[a])
                        continue;
                    if (G->nx == cap) {
                        cap = cap * 2 + 16;
                        G->xl = realloc(G->xl, (size_t)cap * 5 * sizeof(int32_t));
                    }
                    int32_t *x = G->xl + 5 * G->nx;
                    x[0] = w->qe[a];
                    x[1] = w->te[a];
                    x[2] = w->qs[b];
                    x[3] = w->ts[b];
                    x[4] = ov;
                    G->xjob[j] = G->nx++; /* local: made global in phase 3 */
                }
        } else {
            if (!G->ok || w->err || w->nl == 0)
                continue;
            const int64_t x0 = X->xoff[k];
            for (int32_t j = 0; j < G->pc.nbk; ++j)
                if (G->xjob[j] >= 0)
                    G->xjob[j] += (int32_t)x0;
            ax_xres xr = {G->xjob, X->xpos, X->xadj, X->xlqe, X->xlte, X->xrqs, X->xrts, X->xov};
            pair_finish(w, &G->pc, &xr, o);
            free(G->xjob);
            free(G->xl);
            G->xjob = G->xl = NULL;
        }
        G->t0 += gnow() - t0;
        o->secs = G->t0;
        if (w->err) {
            o->err = 1;
            memcpy(o->msg, w->msg, sizeof(o->msg));
        }
    }
    return NULL;
}

static void gdp_phase(ax_gjob *X, int phase, int nt) {
    X->phase = phase;
    atomic_store(&X->next, 0);
    gac_run_threads(nt, gdp_thread, X);
}

/* the peel, the crossovers of the peeled chains (one gac_crossovers batch)
 * and the finish of the device pairs (phases 2 and 3), X->leaf_off and the
 * DP's results set; returns the crossovers' rc.  *nxo: crossover count */
static int gdp_finish(ax_gjob *X, int nt, const int32_t *kt, const int32_t *kq, const uint8_t *ks,
                      int64_t *nxo) {
    ax_job *J = X->J;
    ax_gpair *G = X->G;
    const int64_t np = J->n_pairs;
    gdp_phase(X, 2, nt);
    int64_t *xoff = malloc((size_t)(np + 1) * sizeof(int64_t));
    xoff[0] = 0;
    for (int64_t p = 0; p < np; ++p)
        xoff[p + 1] = xoff[p] + G[p].nx;
    const int64_t nx = xoff[np];
    int32_t *xt = malloc((size_t)(nx ? nx : 1) * 4), *xq = malloc((size_t)(nx ? nx : 1) * 4);
    uint8_t *xs = malloc((size_t)(nx ? nx : 1));
    int32_t *xv[5], *xpos = malloc((size_t)(nx ? nx : 1) * 4), *xadj = malloc((size_t)(nx ? nx : 1) * 4);
    for (int f = 0; f < 5; ++f)
        xv[f] = malloc((size_t)(nx ? nx : 1) * 4);
    for (int64_t p = 0; p < np; ++p) /* (p: place in J->order) */
        for (int32_t k = 0; k < G[p].nx; ++k) {
            const int64_t g = xoff[p] + k;
            xt[g] = kt[p];
            xq[g] = kq[p];
            xs[g] = ks[p] ? 1 : 0;
            for (int f = 0; f < 5; ++f)
                xv[f][g] = G[p].xl[5 * k + f];
        }
    const int rc = gac_crossovers(J->ctx, nx, xt, xq, xs, xv[0], xv[1], xv[2], xv[3], xv[4], xpos, xadj);
    if (rc == GAC_OK) {
        X->xoff = xoff;
        X->xpos = xpos;
        X->xadj = xadj;
        X->xlqe = xv[0];
        X->xlte = xv[1];
        X->xrqs = xv[2];
        X->xrts = xv[3];
        X->xov = xv[4];
        gdp_phase(X, 3, nt);
    }
    free(xt);
    free(xq);
    free(xs);
    free(xpos);
    free(xadj);
    for (int f = 0; f < 5; ++f)
        free(xv[f]);
    free(xoff);
    *nxo = nx;
    return rc;
}

static void gdp_free_pairs(ax_gpair *G, int64_t np) {
    for (int64_t p = 0; p < np; ++p) {
        ax_work *w = &G[p].w;
        gpair_free_export(&G[p]);
        free(G[p].pc.cblk);
        free(G[p].pc.cstart);
        free(G[p].xjob);
        free(G[p].xl);
        free(w->total);
        free(w->pred);
        free(w->hit);
        free(w->tord);
        free(w->qord);
        free(w->tmp);
        free(w->nodes);
        free(w->lnode);
        free(w->qpos);
        free(w->tpos);
        free(w->tbox);
        free(w->qbox);
        free(w->qtp);
        free(w->bnd);
        free(w->xs);
    }
    free(G);
}

/* the device pairs with every input of the DP built on the device
 * (gac_chain_dp_blocks: leaves, kd-trees, update paths, overlap lists): the
 * host packs the pairs' blocks (phase 1) and peels and finishes (phases 2,
 * 3).  GAC_DP_DEVTREE=0: the round-5 path (trees, paths and overlap lists
 * built and exported on host threads, gac_chain_dp_ex) */
static int axt_dp_gpu_devtree(ax_job *J, int nt, ax_gjob *X, int32_t *kt, int32_t *kq, uint8_t *ks) {
    const int64_t np = J->n_pairs;
    ax_gpair *G = X->G;
    const double t = gnow();
    int64_t *boff = malloc((size_t)(np + 1) * sizeof(int64_t));
    boff[0] = 0;
    for (int64_t k = 0; k < np; ++k)
        boff[k + 1] = boff[k] + (J->poff[J->order[k] + 1] - J->poff[J->order[k]]);
    const int64_t nb = boff[np];
    X->dev_tree = 1;
    X->boff = boff;
    X->box = malloc((size_t)(nb ? nb : 1) * 4 * sizeof(int32_t));
    X->bscore = malloc((size_t)(nb ? nb : 1) * sizeof(int32_t));
    gdp_phase(X, 1, nt);
    const double t1 = gnow();
    int rc = GAC_OK;
    for (int64_t k = 0; k < np && rc == GAC_OK; ++k)
        if (!G[k].ok)
            rc = gac_fail(GAC_E_ARG, "pair %d: no host sequence", J->order[k]);
    /* the fast DP when the gap costs allow it (as dp_fast_enabled) */
    const char *fv = getenv("GAC_DP_FAST");
    const int fast = J->e->fast && !(fv && *fv == '0');
    static int ov_cap = -1; /* (GAC_DP_OVCAP: the test hook of gpair_export) */
    if (ov_cap < 0) {
        const char *oc = getenv("GAC_DP_OVCAP");
        const int v = oc && *oc ? atoi(oc) : 1024;
        ov_cap = v >= 0 && v <= 1024 ? v : 1024;
    }
    int64_t *leaf_off = malloc((size_t)(np + 1) * sizeof(int64_t));
    int32_t *tord = malloc((size_t)(nb ? nb : 1) * sizeof(int32_t));
    int64_t *btotal = malloc((size_t)(nb ? nb : 1) * sizeof(int64_t));
    int32_t *bpred = malloc((size_t)(nb ? nb : 1) * sizeof(int32_t));
    if (rc == GAC_OK)
        rc = gac_chain_dp_blocks(J->ctx, np, kt, kq, ks, boff, X->box, X->bscore, fast,
                                 fast ? J->e->lin_k : 0, J->e->min_entry, ov_cap, leaf_off, tord,
                                 btotal, bpred);
    free(X->box);
    free(X->bscore);
    X->box = X->bscore = NULL;
    const double t2 = gnow();
    int64_t nx = 0;
    if (rc == GAC_OK) {
        X->leaf_off = leaf_off;
        X->tord = tord;
        X->btotal = btotal;
        X->bpred = bpred;
        rc = gdp_finish(X, nt, kt, kq, ks, &nx);
    }
    const double t3 = gnow();
    if (getenv("GAC_TIMING"))
        fprintf(stderr, "[gac_axt_chain] device DP (device-built trees): pack %.3f s, "
                        "gac_chain_dp_blocks %.3f s, peel + %lld crossovers + finish %.3f s\n",
                t1 - t, t2 - t1, (long long)nx, t3 - t2);
    free(leaf_off);
    free(tord);
    free(btotal);
    free(bpred);
    free(boff);
    gdp_free_pairs(G, np);
    free(kt);
    free(kq);
    free(ks);
    return rc;
}

/* the pairs J->order[0 .. J->n_pairs) (all of them, or the device's share
 * of a hybrid run); arrays below are by place k in that list */
static int axt_dp_gpu(ax_job *J, int nt) {
    const int64_t np = J->n_pairs;
    ax_gpair *G = calloc((size_t)(np ? np : 1), sizeof(ax_gpair));
    int32_t *kt = malloc((size_t)(np ? np : 1) * sizeof(int32_t));
    int32_t *kq = malloc((size_t)(np ? np : 1) * sizeof(int32_t));
    uint8_t *ks = malloc((size_t)(np ? np : 1));
    for (int64_t k = 0; k < np; ++k) {
        kt[k] = J->in->t_seq[J->order[k]];
        kq[k] = J->in->q_seq[J->order[k]];
        ks[k] = J->in->q_strand[J->order[k]];
    }
    ax_gjob X;
    memset(&X, 0, sizeof(X));
    X.J = J;
    X.G = G;
    atomic_init(&X.next, 0);
    int rc = GAC_OK;
    double t = gnow();
    const char *dtv = getenv("GAC_DP_DEVTREE");
    if (!(dtv && *dtv == '0'))
        return axt_dp_gpu_devtree(J, nt, &X, kt, kq, ks);
    gdp_phase(&X, 1, nt);
    double t1 = gnow();
    /* gather the pairs' trees */
    int64_t *node_off = malloc((size_t)(np + 1) * sizeof(int64_t));
    int64_t *leaf_off = malloc((size_t)(np + 1) * sizeof(int64_t));
    node_off[0] = leaf_off[0] = 0;
    int64_t npath = 0, novl = 0;
    int fast = 1; /* every live pair exported its overlap lists */
    for (int64_t p = 0; p < np; ++p) {
        const int live = G[p].ok && !G[p].w.err && G[p].w.nl > 0;
        node_off[p + 1] = node_off[p] + (live ? G[p].w.nn : 0);
        leaf_off[p + 1] = leaf_off[p] + (live ? G[p].w.nl : 0);
        npath += live ? G[p].poff[G[p].w.nl] : 0;
        if (live && !G[p].ooff)
            fast = 0;
        novl += live && G[p].ooff ? G[p].ooff[G[p].w.nl] : 0;
    }
    const int64_t nn = node_off[np], nl = leaf_off[np];
    int32_t *na = malloc((size_t)(nn ? nn : 1) * 16), *nb = malloc((size_t)(nn ? nn : 1) * 8);
    int32_t *lf = malloc((size_t)(nl ? nl : 1) * 16), *lsc = malloc((size_t)(nl ? nl : 1) * 4);
    int32_t *lnode = malloc((size_t)(nl ? nl : 1) * 4);
    int64_t *poff = malloc((size_t)(nl + 1) * 8);
    int32_t *path = malloc((size_t)(npath ? npath : 1) * 4);
    int64_t *total = malloc((size_t)(nl ? nl : 1) * 8);
    int32_t *pred = malloc((size_t)(nl ? nl : 1) * 4);
    int64_t *ooff = fast ? malloc((size_t)(nl + 1) * 8) : NULL;
    int32_t *ovl = fast ? malloc((size_t)(novl ? novl : 1) * 4) : NULL;
    if (ooff)
        ooff[0] = 0;
    poff[0] = 0;
    for (int64_t p = 0; p < np; ++p) {
        const int64_t n0 = node_off[p], l0 = leaf_off[p], cn = node_off[p + 1] - n0,
                      cl = leaf_off[p + 1] - l0;
        if (!cl)
            continue;
        memcpy(na + 4 * n0, G[p].na, (size_t)cn * 16);
        memcpy(nb + 2 * n0, G[p].nb, (size_t)cn * 8);
        memcpy(lf + 4 * l0, G[p].lf, (size_t)cl * 16);
        memcpy(lsc + l0, G[p].lsc, (size_t)cl * 4);
        memcpy(lnode + l0, G[p].lnode, (size_t)cl * 4);
        const int64_t pb = poff[l0];
        memcpy(path + pb, G[p].path, (size_t)G[p].poff[cl] * 4);
        for (int64_t i = 0; i < cl; ++i)
            poff[l0 + i + 1] = pb + G[p].poff[i + 1];
        if (ooff) {
            const int64_t ob = ooff[l0];
            memcpy(ovl + ob, G[p].ovl, (size_t)G[p].ooff[cl] * 4);
            for (int64_t i = 0; i < cl; ++i)
                ooff[l0 + i + 1] = ob + G[p].ooff[i + 1];
        }
    }
    double t2 = gnow();
    /* the exact fast DP (k_dp_fast) when the gap costs allow it, else the
     * reference search (k_dp) */
    rc = gac_chain_dp_ex(J->ctx, np, kt, kq, ks, node_off, na, nb,
                         leaf_off, lf, lsc, lnode, poff, path, ooff, ovl,
                         ooff ? J->e->lin_k : 0, J->e->min_entry, total, pred);
    free(ooff);
    free(ovl);
    double t3 = gnow();
    free(na);
    free(nb);
    free(lf);
    free(lsc);
    free(lnode);
    free(poff);
    free(path);
    free(node_off);
    if (rc == GAC_OK) {
        X.leaf_off = leaf_off;
        X.total = total;
        X.pred = pred;
        int64_t nx = 0;
        rc = gdp_finish(&X, nt, kt, kq, ks, &nx);
        if (getenv("GAC_TIMING"))
            fprintf(stderr, "[gac_axt_chain] device DP: trees %.3f s (thread-seconds: leaves %.3f, "
                            "tree %.3f, export %.3f), gather %.3f s, gac_chain_dp %.3f s, peel + "
                            "%lld crossovers + finish %.3f s\n",
                    t1 - t, X.t_leaves, X.t_tree, X.t_export, t2 - t1, t3 - t2, (long long)nx,
                    gnow() - t3);
    }
    free(leaf_off);
    free(total);
    free(pred);
    gdp_free_pairs(G, np);
    free(kt);
    free(kq);
    free(ks);
    return rc;
}

/* ---- the hybrid DP (the default): the device takes the smallest pairs
 * (gac_chain_dp_blocks: their leaves, kd-trees, update paths and overlap
 * lists built on the device, then k_dp_spec, 16 waves per pair searching
 * consecutive leaves and committing them in order, every device pair at
 * once) while host threads take the others (teams on the largest).  A
 * device pair must end within the host's critical path, estimated from the
 * largest pair at the team's rate (its device time, leaves x the device's
 * per-leaf time, within 0.7 of it), and is at most 1 M leaves.  C4 at 50 M
 * blocks (r06sp16): the device's 1000 pairs, 23.1 M blocks (46 %), done in
 * 3.7 s inside the largest pair's 7 s on its host team; wall 9.23 / 8.79 s vs
 * host-only 8.97 / 8.91 s -- the wall is that one pair's team, which no
 * device share shortens.  Pairs go to the device from the smallest up.
 * GAC_AXT_DP=host: no device pairs; GAC_DP_GPU_MAX=n: the leaf cap (0:
 * none); GAC_DP_DEV_US / GAC_DP_HOST_US: the per-leaf times of the model.
 * Returns the first device place in `order`. */
static int64_t dp_device_split(const int64_t *psize, const int32_t *order, int64_t np,
                               const ax_env *e) {
    const char *dpm = getenv("GAC_AXT_DP");
    if ((dpm && strcmp(dpm, "host") == 0) || !e->fast || np == 0)
        return np;
    const char *dv = getenv("GAC_DP_DEV_US"), *hv = getenv("GAC_DP_HOST_US");
    const double dev_us = dv && atof(dv) > 0 ? atof(dv) : 4.0;  /* k_dp_spec x 16, r06sp16 */
    const double host_us = hv && atof(hv) > 0 ? atof(hv) : 0.47; /* team, C4 (r04i) */
    const double crit = (double)psize[order[0]] * host_us * 1e-6;
    if (crit < 0.25) /* (small runs: the device's start-up costs more) */
        return np;
    int64_t lmax = (int64_t)(0.7 * crit / (dev_us * 1e-6));
    const char *mx = getenv("GAC_DP_GPU_MAX");
    const int64_t cap = mx && *mx ? atoll(mx) : 1000000;
    if (cap < lmax)
        lmax = cap;
    if (lmax < 1)
        return np;
    int64_t kd = np;
    while (kd > 1 && psize[order[kd - 1]] <= lmax)
        --kd;
    return kd;
}

/* gac_kd_trees for the team pairs order[0 .. big): their blocks packed on
 * nt threads, each pair's arrays allocated here and adopted by its team
 * (run_pair); NULL (and *rc) when the device build fails */
typedef struct tt_pack {
    const ax_job *J;
    const int32_t *order;
    const int64_t *boff; /* [big + 1] */
    int32_t *box;
    int64_t big;
    _Atomic int64_t next; /* slices of 1 M packed blocks */
} tt_pack;

static void *tt_pack_thread(void *arg) {
    tt_pack *T = arg;
    const int64_t nb = T->boff[T->big];
    for (;;) {
        const int64_t c0 = atomic_fetch_add(&T->next, 1) << 20;
        if (c0 >= nb)
            return NULL;
        const int64_t c1 = c0 + (1 << 20) < nb ? c0 + (1 << 20) : nb;
        int64_t k = 0;
        while (T->boff[k + 1] <= c0)
            ++k;
        for (int64_t g = c0; g < c1; ++g) {
            while (T->boff[k + 1] <= g)
                ++k;
            const int64_t b = T->J->poff[T->order[k]] + (g - T->boff[k]);
            int32_t *x = T->box + 4 * g;
            x[0] = T->J->qs[b];
            x[1] = T->J->qe[b];
            x[2] = T->J->ts[b];
            x[3] = T->J->te[b];
        }
    }
}

static ax_pre *team_trees(ax_job *J, const int32_t *order, int64_t big, int nt, int *rc) {
    int64_t *boff = malloc((size_t)(big + 1) * sizeof(int64_t));
    boff[0] = 0;
    for (int64_t k = 0; k < big; ++k)
        boff[k + 1] = boff[k] + (J->poff[order[k] + 1] - J->poff[order[k]]);
    const int64_t nb = boff[big];
    int32_t *box = malloc((size_t)(nb ? nb : 1) * 4 * sizeof(int32_t));
    int32_t *kt = malloc((size_t)big * sizeof(int32_t)), *kq = malloc((size_t)big * sizeof(int32_t));
    uint8_t *ks = malloc((size_t)big);
    ax_pre *pre = calloc((size_t)big, sizeof(ax_pre));
    int32_t **tord = malloc((size_t)big * sizeof(int32_t *)), **qord = malloc((size_t)big * sizeof(int32_t *));
    int32_t **lnode = malloc((size_t)big * sizeof(int32_t *)), **nodes = malloc((size_t)big * sizeof(int32_t *));
    for (int64_t k = 0; k < big; ++k) {
        const int32_t p = order[k];
        const int64_t n = boff[k + 1] - boff[k];
        kt[k] = J->in->t_seq[p];
        kq[k] = J->in->q_seq[p];
        ks[k] = J->in->q_strand[p] ? 1 : 0;
        /* (sized as work_reserve sizes them: + 16) */
        pre[k].tord = tord[k] = malloc((size_t)(n + 16) * sizeof(int32_t));
        pre[k].qord = qord[k] = malloc((size_t)(n + 16) * sizeof(int32_t));
        pre[k].lnode = lnode[k] = malloc((size_t)(n + 16) * sizeof(int32_t));
        pre[k].nodes = nodes[k] = malloc((size_t)(2 * n + 32) * 6 * sizeof(int32_t));
    }
    tt_pack T = {J, order, boff, box, big, 0};
    gac_run_threads(nt, tt_pack_thread, &T);
    int64_t *leaf_off = malloc((size_t)(big + 1) * sizeof(int64_t));
    const int r = gac_kd_trees(J->ctx, big, kt, kq, ks, boff, box, leaf_off, tord, qord, lnode, nodes);
    if (r == GAC_OK) {
        for (int64_t k = 0; k < big; ++k)
            pre[k].nl = (int32_t)(leaf_off[k + 1] - leaf_off[k]);
    } else {
        *rc = r;
        for (int64_t k = 0; k < big; ++k) {
            free(pre[k].tord);
            free(pre[k].qord);
            free(pre[k].lnode);
            free(pre[k].nodes);
        }
        free(pre);
        pre = NULL;
    }
    free(leaf_off);
    free(boff);
    free(box);
    free(kt);
    free(kq);
    free(ks);
    free(tord);
    free(qord);
    free(lnode);
    free(nodes);
    return pre;
}

typedef struct dev_run {
    ax_job J; /* the device's pairs */
    int nt, rc;
    double secs;
} dev_run;

static void *dev_runner(void *arg) {
    dev_run *D = arg;
    const double t0 = gnow();
    D->rc = axt_dp_gpu(&D->J, D->nt);
    D->secs = gnow() - t0;
    return NULL;
}

static int thread_count(int req) {
    if (req > 0)
        return req > 256 ? 256 : req;
    return gac_host_threads();
}

/* ------------------------------------------------------------------ parallel helpers */
#define run_threads gac_run_threads

typedef struct bkey { /* removeExactOverlaps: slSort(cBlockCmpBoth) */
    int32_t qs, ts, rank, qe, te;
} bkey;

static int bkey_cmp(const void *a, const void *b) {
    const bkey *x = a, *y = b;
    if (x->qs != y->qs)
        return x->qs < y->qs ? -1 : 1;
    if (x->ts != y->ts)
        return x->ts < y->ts ? -1 : 1;
    return (x->rank > y->rank) - (x->rank < y->rank);
}

typedef struct fold_job {
    const gac_axt_input *in;
    int32_t *qs, *qe, *ts, *te;
    int64_t *poff; /* poff[p + 1] = folded count of pair p */
    int64_t np;
    int64_t big;   /* pairs above this many blocks were folded beforehand */
    _Atomic int64_t next;
} fold_job;

/* ---- parallel sort of one large pair's keys (ranks make every key unique,
 * so any correct sort is the stable one): runs sorted on threads, then
 * merged pairwise, the merges of a round on threads */
typedef struct psort_job {
    bkey *a, *tmp;
    int64_t n;
    int nrun;
    int64_t *cut; /* [nrun + 1] */
    int64_t width; /* runs merged per output run this round / 2 */
    _Atomic int next;
} psort_job;

static void *psort_runs(void *arg) {
    psort_job *J = arg;
    for (;;) {
        const int r = atomic_fetch_add(&J->next, 1);
        if (r >= J->nrun)
            return NULL;
        qsort(J->a + J->cut[r], (size_t)(J->cut[r + 1] - J->cut[r]), sizeof(bkey), bkey_cmp);
    }
}

static void *psort_merge(void *arg) {
    psort_job *J = arg;
    for (;;) {
        const int m = atomic_fetch_add(&J->next, 1);
        const int64_t r0 = (int64_t)m * 2 * J->width;
        if (r0 >= J->nrun)
            return NULL;
        const int64_t r1 = r0 + J->width < J->nrun ? r0 + J->width : J->nrun;
        const int64_t r2 = r0 + 2 * J->width < J->nrun ? r0 + 2 * J->width : J->nrun;
        int64_t i = J->cut[r0], j = J->cut[r1], o = J->cut[r0];
        const int64_t ie = J->cut[r1], je = J->cut[r2];
        while (i < ie && j < je)
            J->tmp[o++] = bkey_cmp(&J->a[j], &J->a[i]) < 0 ? J->a[j++] : J->a[i++];
        while (i < ie)
            J->tmp[o++] = J->a[i++];
        while (j < je)
            J->tmp[o++] = J->a[j++];
    }
}

static void par_sort_bkey(bkey *a, int64_t n, int nt) {
    psort_job J;
    J.a = a;
    J.n = n;
    J.nrun = nt;
    J.cut = malloc((size_t)(nt + 1) * sizeof(int64_t));
    for (int r = 0; r <= nt; ++r)
        J.cut[r] = n * r / nt;
    atomic_init(&J.next, 0);
    gac_run_threads(nt, psort_runs, &J);
    J.tmp = malloc((size_t)n * sizeof(bkey));
    for (J.width = 1; J.width < nt; J.width *= 2) {
        atomic_store(&J.next, 0);
        const int64_t merges = (nt + 2 * J.width - 1) / (2 * J.width);
        gac_run_threads(merges < nt ? (int)merges : nt, psort_merge, &J);
        bkey *t = J.a;
        J.a = J.tmp;
        J.tmp = t;
    }
    if (J.a != a) { /* an odd number of rounds: the result is in the scratch */
        memcpy(a, J.a, (size_t)n * sizeof(bkey));
        J.tmp = J.a;
    }
    free(J.tmp);
    free(J.cut);
}

/* removeExactOverlaps' 16-byte sort record: (qStart, tStart) as one key,
 * the block's rank and size; NULL when a start is negative (the comparator
 * sort then) */
typedef struct fkey {
    uint64_t k; /* qStart << 32 | tStart */
    int32_t rank, size;
} fkey;
_Static_assert(sizeof(fkey) == 16, "radix_sort16 record");

static fkey *fold_keys(const gac_axt_input *in, int64_t a, int64_t b, fkey *k, int nt) {
    for (int64_t i = a; i < b; ++i) {
        if (in->blk_q[i] < 0 || in->blk_t[i] < 0)
            return NULL;
        k[i - a] = (fkey){(uint64_t)in->blk_q[i] << 32 | (uint32_t)in->blk_t[i], (int32_t)(i - a),
                          in->blk_size[i]};
    }
    radix_sort16(k, b - a, nt);
    return k;
}

/* removeExactOverlaps' fold of one pair's sorted keys into its input slot */
static int64_t fold_sorted(fold_job *F, const bkey *k, int64_t a, int64_t m) {
    int64_t n = a;
    for (int64_t i = 0; i < m; ++i) {
        if (n > a && k[i].qs == F->qs[n - 1] && k[i].ts == F->ts[n - 1]) {
            if (F->qe[n - 1] < k[i].qe)
                F->qe[n - 1] = k[i].qe;
            if (F->te[n - 1] < k[i].te)
                F->te[n - 1] = k[i].te;
            continue;
        }
        F->qs[n] = k[i].qs;
        F->qe[n] = k[i].qe;
        F->ts[n] = k[i].ts;
        F->te[n] = k[i].te;
        ++n;
    }
    return n - a;
}

static int64_t fold_sorted_f(fold_job *F, const fkey *k, int64_t a, int64_t m) {
    int64_t n = a;
    for (int64_t i = 0; i < m; ++i) {
        const int32_t q = (int32_t)(k[i].k >> 32), t = (int32_t)(uint32_t)k[i].k;
        const int32_t qe = q + k[i].size, te = t + k[i].size;
        if (n > a && q == F->qs[n - 1] && t == F->ts[n - 1]) {
            if (F->qe[n - 1] < qe)
                F->qe[n - 1] = qe;
            if (F->te[n - 1] < te)
                F->te[n - 1] = te;
            continue;
        }
        F->qs[n] = q;
        F->qe[n] = qe;
        F->ts[n] = t;
        F->te[n] = te;
        ++n;
    }
    return n - a;
}

/* removeExactOverlaps (axtChain.c:173-197): slSort by (qStart, tStart),
 * stable; blocks with both starts equal fold into the first (max ends) */
static void *fold_thread(void *arg) {
    fold_job *F = arg;
    const gac_axt_input *in = F->in;
    bkey *k = NULL;
    int64_t kcap = 0;
    for (;;) {
        const int64_t p = atomic_fetch_add(&F->next, 1);
        if (p >= F->np)
            break;
        const int64_t a = in->blk_off[p], b = in->blk_off[p + 1];
        if (b - a > F->big)
            continue;
        if (b - a > kcap) {
            kcap = b - a;
            k = realloc(k, (size_t)kcap * sizeof(bkey));
        }
        if (b - a >= 4096) { /* (radix: fkey fits in a bkey's room) */
            const fkey *f = fold_keys(in, a, b, (fkey *)k, 1);
            if (f) {
                F->poff[p + 1] = fold_sorted_f(F, f, a, b - a);
                continue;
            }
        }
        for (int64_t i = a; i < b; ++i)
            k[i - a] = (bkey){in->blk_q[i], in->blk_t[i], (int32_t)(i - a),
                              in->blk_q[i] + in->blk_size[i], in->blk_t[i] + in->blk_size[i]};
        qsort(k, (size_t)(b - a), sizeof(bkey), bkey_cmp);
        F->poff[p + 1] = fold_sorted(F, k, a, b - a);
    }
    free(k);
    return NULL;
}

/* ------------------------------------------------------------------ entry */
/* GAC_TIMING=1: stage wall times on stderr */
static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* free() of n blocks on a detached thread (the caller goes on; the frees
 * unmap GBs at C4 scale) */
typedef struct late_free {
    int n;
    void *p[];
} late_free;

static void *late_free_thread(void *arg) {
    late_free *L = arg;
    for (int i = 0; i < L->n; ++i)
        free(L->p[i]);
    free(L);
    return NULL;
}

static void free_later(void *const *p, int n) {
    late_free *L = malloc(sizeof(late_free) + (size_t)(n > 0 ? n : 1) * sizeof(void *));
    if (!L) {
        for (int i = 0; i < n; ++i)
            free(p[i]);
        return;
    }
    L->n = n;
    memcpy(L->p, p, (size_t)n * sizeof(void *));
    pthread_attr_t at;
    pthread_attr_init(&at);
    pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
    pthread_t th;
    if (pthread_create(&th, &at, late_free_thread, L) != 0)
        late_free_thread(L);
    pthread_attr_destroy(&at);
}

static void stage(const char *what, double *t) {
    static int on = -1;
    if (on < 0) {
        const char *e = getenv("GAC_TIMING");
        on = e && *e && *e != '0';
    }
    const double n = now_s();
    if (on)
        fprintf(stderr, "[gac_axt_chain] %-28s %8.3f s\n", what, n - *t);
    *t = n;
}

static int cmp_i64_desc_pair(const void *a, const void *b, void *arg) {
    const int64_t *sz = arg;
    const int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
    if (sz[x] != sz[y])
        return sz[x] > sz[y] ? -1 : 1;
    return (x > y) - (x < y);
}

/* the pairs' chains gathered into one chain set (parallel over pairs) */
typedef struct gather_job {
    const ax_out *po;
    const gac_axt_input *in;
    int32_t *ct, *cq;
    uint8_t *cs;
    int64_t *coff;
    int32_t *bt, *bq, *bs;
    int64_t *c0, *x0; /* per pair: first chain, first block */
    int64_t np;
    int64_t *task, ntask; /* (pair, first chain, end chain) */
    _Atomic int64_t next;
} gather_job;

static void *gather_thread(void *arg) {
    gather_job *G = arg;
    for (;;) {
        const int64_t t = atomic_fetch_add(&G->next, 1);
        if (t >= G->ntask)
            return NULL;
        /* task t: chains [k0, k1) of pair p (a large pair's chains are
         * several tasks, so one pair does not hold up the copy) */
        const int64_t p = G->task[3 * t];
        const int32_t k0 = (int32_t)G->task[3 * t + 1], k1 = (int32_t)G->task[3 * t + 2];
        const ax_out *o = &G->po[p];
        int64_t c = G->c0[p] + k0, x = G->x0[p] + o->coff[k0];
        /* (the task's chains' blocks are one run of the pair's arrays) */
        const int32_t r0 = o->coff[k0], r1 = o->coff[k1];
        memcpy(G->bt + x, o->bt + r0, (size_t)(r1 - r0) * 4);
        memcpy(G->bq + x, o->bq + r0, (size_t)(r1 - r0) * 4);
        memcpy(G->bs + x, o->bs + r0, (size_t)(r1 - r0) * 4);
        for (int32_t k = k0; k < k1; ++k, ++c) {
            G->ct[c] = G->in->t_seq[p];
            G->cq[c] = G->in->q_seq[p];
            G->cs[c] = G->in->q_strand[p] ? 1 : 0;
            x += o->coff[k + 1] - o->coff[k];
            G->coff[c + 1] = x;
        }
    }
}

/* the kept chains in output order (parallel over chains), copied from each
 * pair's own arrays: chain i of the whole list is chain i - c0[p] of pair
 * p = cpair[i] */
typedef struct out_job {
    gac_axt_chains *R;
    const struct dkey *k;
    const ax_out *po;
    const int64_t *c0, *gsc;
    const int32_t *cpair;
    int64_t nk;
    _Atomic int64_t next;
} out_job;

static void *out_thread(void *arg) {
    out_job *O = arg;
    gac_axt_chains *R = O->R;
    for (;;) {
        const int64_t j0 = atomic_fetch_add(&O->next, 1024);
        if (j0 >= O->nk)
            return NULL;
        const int64_t j1 = j0 + 1024 < O->nk ? j0 + 1024 : O->nk;
        for (int64_t j = j0; j < j1; ++j) {
            const int32_t i = O->k[j].v, p = O->cpair[i];
            const ax_out *po = &O->po[p];
            const int32_t c = (int32_t)(i - O->c0[p]);
            const int64_t b0 = po->coff[c], b1 = po->coff[c + 1], o = R->blk_off[j];
            R->score[j] = (double)O->gsc[i];
            R->pair[j] = p;
            R->t_start[j] = po->bt[b0];
            R->q_start[j] = po->bq[b0];
            R->t_end[j] = po->bt[b1 - 1] + po->bs[b1 - 1];
            R->q_end[j] = po->bq[b1 - 1] + po->bs[b1 - 1];
            memcpy(R->blk_t + o, po->bt + b0, (size_t)(b1 - b0) * 4);
            memcpy(R->blk_q + o, po->bq + b0, (size_t)(b1 - b0) * 4);
            memcpy(R->blk_size + o, po->bs + b0, (size_t)(b1 - b0) * 4);
        }
    }
}

/* chainCalcScore of every chain of the pairs sel[0 .. ns) (axtChain.c:300-305):
 * their chains gathered into one set (pairs in parallel, disjoint slots from
 * prefix sums over the selection), one upload, one GPU batch; each pair's
 * scores to its po[p].gsc.  Called for the pairs that are done while the
 * teams still run (the pool's and the device's), then for the rest, so that
 * only the last pairs' scoring is on the critical path. */
static int score_pairs(gac_ctx *ctx, ax_out *po, const gac_axt_input *in, int64_t np,
                       const int32_t *sel, int64_t ns, int nthreads, double *tclock) {
    int64_t nc = 0, ncb = 0, ntask = 0;
    for (int64_t s = 0; s < ns; ++s) {
        const ax_out *o = &po[sel[s]];
        nc += o->n_chains;
        ncb += o->coff ? o->coff[o->n_chains] : 0;
        ntask += (o->n_chains + 4095) / 4096;
    }
    for (int64_t s = 0; s < ns; ++s) { /* (a pair without chains: nothing to score) */
        ax_out *o = &po[sel[s]];
        o->scored = 1;
        o->gsc = malloc((size_t)(o->n_chains ? o->n_chains : 1) * 8);
    }
    if (nc == 0)
        return GAC_OK;
    int32_t *ct = malloc((size_t)nc * 4), *cq = malloc((size_t)nc * 4);
    uint8_t *cs = malloc((size_t)nc);
    int64_t *coff = malloc((size_t)(nc + 1) * 8);
    int32_t *bt = malloc((size_t)(ncb ? ncb : 1) * 4), *bq = malloc((size_t)(ncb ? ncb : 1) * 4),
            *bs = malloc((size_t)(ncb ? ncb : 1) * 4);
    int64_t *gsc = malloc((size_t)nc * 8);
    int32_t *gali = malloc((size_t)nc * 4);
    gather_job G;
    memset(&G, 0, sizeof(G));
    G.po = po, G.in = in, G.ct = ct, G.cq = cq, G.cs = cs, G.coff = coff;
    G.bt = bt, G.bq = bq, G.bs = bs, G.np = np;
    G.c0 = malloc((size_t)(np + 1) * 8); /* (set for the selected pairs only) */
    G.x0 = malloc((size_t)(np + 1) * 8);
    G.task = malloc((size_t)(ntask ? ntask : 1) * 3 * sizeof(int64_t));
    int64_t c = 0, x = 0;
    for (int64_t s = 0; s < ns; ++s) {
        const int32_t p = sel[s];
        G.c0[p] = c;
        G.x0[p] = x;
        c += po[p].n_chains;
        x += po[p].coff ? po[p].coff[po[p].n_chains] : 0;
        for (int32_t k = 0; k < po[p].n_chains; k += 4096) {
            G.task[3 * G.ntask] = p;
            G.task[3 * G.ntask + 1] = k;
            G.task[3 * G.ntask + 2] = k + 4096 < po[p].n_chains ? k + 4096 : po[p].n_chains;
            ++G.ntask;
        }
    }
    coff[0] = 0;
    atomic_init(&G.next, 0);
    run_threads(nthreads < G.ntask ? nthreads : (int)(G.ntask ? G.ntask : 1), gather_thread, &G);
    free(G.task);
    stage("chains gathered for scoring", tclock);
    gac_chainset_desc d = {nc, ct, cq, cs, coff, ncb, bt, bq, bs};
    gac_chainset *set = NULL;
    int rc = gac_chains_upload(ctx, &d, &set);
    stage("chains to HBM", tclock);
    if (rc == GAC_OK)
        rc = gac_score_chains(ctx, set, 0, gsc, NULL, gali);
    stage("GPU chain scores", tclock);
    gac_chains_free(set);
    if (rc == GAC_OK)
        for (int64_t s = 0; s < ns; ++s) {
            const int32_t p = sel[s];
            memcpy(po[p].gsc, gsc + G.c0[p], (size_t)po[p].n_chains * 8);
        }
    free(G.c0);
    free(G.x0);
    /* (GBs at C4: freed on a detached thread, off the caller's path) */
    void *big[] = {ct, cq, cs, coff, bt, bq, bs, gsc, gali};
    free_later(big, (int)(sizeof(big) / sizeof(big[0])));
    return rc;
}

/* every chain's pair and score in list order (pairs in input order), in
 * slices of the chain list */
typedef struct list_job {
    const ax_out *po;
    const int64_t *c0;
    int64_t np, nc;
    int32_t *cpair;
    int64_t *gsc;
    _Atomic int64_t next;
} list_job;

static void *list_thread(void *arg) {
    list_job *L = arg;
    for (;;) {
        const int64_t a = atomic_fetch_add(&L->next, 1 << 16);
        if (a >= L->nc)
            return NULL;
        const int64_t b = a + (1 << 16) < L->nc ? a + (1 << 16) : L->nc;
        int64_t lo = 0, hi = L->np - 1; /* the pair of chain a: last p with c0[p] <= a */
        while (lo < hi) {
            const int64_t m = (lo + hi + 1) >> 1;
            if (L->c0[m] <= a)
                lo = m;
            else
                hi = m - 1;
        }
        for (int64_t i = a, p = lo; i < b; ++i) {
            while (L->c0[p + 1] <= i)
                ++p;
            L->cpair[i] = (int32_t)p;
            L->gsc[i] = L->po[p].gsc[i - L->c0[p]];
        }
    }
}

/* score_pairs of the pairs not scored yet, unless one of them failed (the
 * caller reports the first pair's error) */
static int score_rest(gac_ctx *ctx, ax_out *po, const gac_axt_input *in, int64_t np,
                      const int32_t *cand, int64_t ncand, int nthreads, double *tclock) {
    int32_t *sel = malloc((size_t)(ncand ? ncand : 1) * 4);
    int64_t ns = 0;
    for (int64_t k = 0; k < ncand; ++k) {
        const int32_t p = cand ? cand[k] : (int32_t)k;
        if (po[p].err) {
            free(sel);
            return GAC_OK;
        }
        if (!po[p].scored)
            sel[ns++] = p;
    }
    const int rc = ns ? score_pairs(ctx, po, in, np, sel, ns, nthreads, tclock) : GAC_OK;
    free(sel);
    return rc;
}

void gac_axt_chains_free(gac_axt_chains *c) {
    if (!c)
        return;
    free(c->score);
    free(c->pair);
    free(c->t_start);
    free(c->t_end);
    free(c->q_start);
    free(c->q_end);
    free(c->blk_off);
    free(c->blk_t);
    free(c->blk_q);
    free(c->blk_size);
    free(c);
}

/* pair_dp_fast's preconditions on the gap costs: with q(d) = cost(d, 0),
 * t(d) = cost(0, d), b(d) = cost(dq, dt) for dq, dt > 0 and dq + dt = d
 * (gapCalc.c:298-331), cost is monotone in each distance iff q, t and b are
 * non-decreasing and b(d + 1) >= q(d), t(d).  Checked up to past the last
 * long position (the linear tails beyond it: slopes >= 0, b's the steepest).
 * lin_k/1024 = the largest s with s d <= every kind's cost at every d >= 1. */
static void dp_fast_setup(ax_env *e) {
    e->fast = 0;
    e->lin_k = 0;
    e->min_entry = 0;
    for (int i = 0; i < 25; ++i)
        if (e->m5[i] < e->min_entry)
            e->min_entry = e->m5[i];
    int32_t dmax = e->gtab_len;
    for (int k = 0; k < 3; ++k)
        if (e->last_pos[k] + 2 > dmax)
            dmax = e->last_pos[k] + 2;
    if (dmax > (1 << 22))
        return;
    for (int k = 0; k < 3; ++k)
        if (!(e->last_slope[k] >= 0))
            return;
    if (e->last_slope[2] < e->last_slope[0] || e->last_slope[2] < e->last_slope[1])
        return;
    double smin = e->last_slope[0];
    for (int k = 1; k < 3; ++k)
        if (e->last_slope[k] < smin)
            smin = e->last_slope[k];
    int pq = gap_cost(e, 0, 0), pt = pq, pb = gap_cost(e, 1, 1);
    if (pq != 0)
        return;
    for (int32_t d = 1; d <= dmax; ++d) {
        const int q = gap_cost(e, d, 0), t = gap_cost(e, 0, d);
        if (q < pq || t < pt)
            return;
        if (d >= 2) {
            const int b = gap_cost(e, 1, d - 1);
            if ((d > 2 && b < pb) || b < pq || b < pt) /* b(d) >= q(d - 1), t(d - 1) */
                return;
            pb = b;
            if (b < smin * d)
                smin = (double)b / d;
        }
        if (q < smin * d)
            smin = (double)q / d;
        if (t < smin * d)
            smin = (double)t / d;
        pq = q;
        pt = t;
    }
    if (smin < 0)
        return;
    e->lin_k = (int64_t)(smin * 1024.0); /* (rounded down: s*d stays below the cost) */
    if (e->lin_k > 0)
        --e->lin_k;
    e->fast = 1;
}

/* host gap-cost table of the last gap setup (gac_axt_chain) */
static pthread_mutex_t g_gtab_mu = PTHREAD_MUTEX_INITIALIZER;
static gac_gapcalc *cached_g = NULL;
static int32_t *cached_tab = NULL;
static int cached_len = 0;

int gac_axt_chain(gac_ctx *ctx, const int32_t mat[16], const gac_gapcalc *g,
                  const gac_axt_input *in, double min_score, int n_threads,
                  const char *details_path, gac_axt_chains **out) {
    gac_clear_error();
    if (!ctx || !mat || !g || !in || !out || in->n_pairs < 0 ||
        (in->n_pairs && (!in->t_seq || !in->q_seq || !in->q_strand || !in->blk_off)))
        return gac_fail(GAC_E_ARG, "gac_axt_chain: bad argument");
    *out = NULL;
    double tclock = now_s();
    int rc = gac_set_scoring(ctx, mat, g);
    if (rc != GAC_OK)
        return rc;
    stage("set scoring", &tclock);
    const int64_t np = in->n_pairs;
    const int64_t nin = np ? in->blk_off[np] : 0;
    /* ---- removeExactOverlaps per pair (axtChain.c:173-197) */
    int64_t *poff = malloc((size_t)(np + 1) * sizeof(int64_t));
    int32_t *qs = malloc((size_t)(nin ? nin : 1) * 4), *qe = malloc((size_t)(nin ? nin : 1) * 4);
    int32_t *ts = malloc((size_t)(nin ? nin : 1) * 4), *te = malloc((size_t)(nin ? nin : 1) * 4);
    int32_t *bsz = malloc((size_t)(nin ? nin : 1) * 4);
    ax_pairinfo *info = calloc((size_t)(np ? np : 1), sizeof(ax_pairinfo));
    for (int64_t p = 0; p < np; ++p) {
        info[p].tname = gac_genome_seq_name(ctx, GAC_T, in->t_seq[p]);
        info[p].qname = gac_genome_seq_name(ctx, GAC_Q, in->q_seq[p]);
        info[p].tsize = gac_genome_seq_size(ctx, GAC_T, in->t_seq[p]);
        info[p].qsize = gac_genome_seq_size(ctx, GAC_Q, in->q_seq[p]);
        info[p].strand = in->q_strand[p] ? '-' : '+';
        if (!info[p].tname || !info[p].qname) {
            rc = gac_fail(GAC_E_ARG, "gac_axt_chain: pair %lld: bad sequence index", (long long)p);
            goto fail;
        }
    }
    const int nthreads = thread_count(n_threads);
    {
        /* every pair folds in parallel into its own input slot, then the
         * slots are compacted in pair order */
        fold_job F = {in, qs, qe, ts, te, poff, np, INT64_MAX, 0};
        /* pairs of more than 1 M blocks (one can hold a third of a
         * whole-genome run) are sorted with every thread first */
        if (nthreads > 1) {
            F.big = 1 << 20;
            for (int64_t p = 0; p < np; ++p) {
                const int64_t a = in->blk_off[p], b = in->blk_off[p + 1];
                if (b - a <= F.big)
                    continue;
                bkey *k = malloc((size_t)(b - a) * sizeof(bkey));
                const fkey *f = fold_keys(in, a, b, (fkey *)k, nthreads);
                if (f) {
                    poff[p + 1] = fold_sorted_f(&F, f, a, b - a);
                    free(k);
                    continue;
                }
                for (int64_t i = a; i < b; ++i)
                    k[i - a] = (bkey){in->blk_q[i], in->blk_t[i], (int32_t)(i - a),
                                      in->blk_q[i] + in->blk_size[i], in->blk_t[i] + in->blk_size[i]};
                par_sort_bkey(k, b - a, nthreads);
                poff[p + 1] = fold_sorted(&F, k, a, b - a);
                free(k);
            }
        }
        atomic_init(&F.next, 0);
        run_threads(nthreads < np ? nthreads : (int)(np ? np : 1), fold_thread, &F);
    }
    int64_t nb = 0;
    for (int64_t p = 0; p < np; ++p) {
        const int64_t a = in->blk_off[p], c = poff[p + 1]; /* c: folded count of pair p */
        memmove(qs + nb, qs + a, (size_t)c * 4);
        memmove(qe + nb, qe + a, (size_t)c * 4);
        memmove(ts + nb, ts + a, (size_t)c * 4);
        memmove(te + nb, te + a, (size_t)c * 4);
        const int64_t first = nb;
        nb += c;
        /* checkBlockRange (axtChain.c:242-248), query then target per block */
        for (int64_t i = first; i < nb; ++i) {
            if (qe[i] > info[p].qsize) {
                rc = gac_fail(GAC_E_ARG, "query %s block %d-%d exceeds sequence length %d",
                              info[p].qname, qs[i], qe[i], info[p].qsize);
                goto fail;
            }
            if (te[i] > info[p].tsize) {
                rc = gac_fail(GAC_E_ARG, "target %s block %d-%d exceeds sequence length %d",
                              info[p].tname, ts[i], te[i], info[p].tsize);
                goto fail;
            }
        }
    }
    poff[0] = 0;
    for (int64_t p = 0; p < np; ++p)
        poff[p + 1] += poff[p];
    stage("removeExactOverlaps", &tclock);
    /* ---- axtScoreUngapped of every block: one GPU batch */
    int32_t *score = malloc((size_t)(nb ? nb : 1) * 4);
    for (int64_t i = 0; i < nb; ++i)
        bsz[i] = qe[i] - qs[i];
    rc = gac_score_blocks(ctx, np, in->t_seq, in->q_seq, in->q_strand, poff, ts, qs, bsz, score);
    if (rc != GAC_OK) {
        free(score);
        goto fail;
    }
    stage("GPU block scores", &tclock);
    /* ---- host gap-cost table + code matrix */
    ax_env env;
    memset(&env, 0, sizeof(env));
    env.g = g;
    {
        static const int acgt_of_code[4] = {3, 1, 0, 2}; /* T C A G -> index in ACGT */
        for (int qc = 0; qc < 5; ++qc)
            for (int tc = 0; tc < 5; ++tc)
                env.m5[qc * 5 + tc] =
                    (qc == 4 || tc == 4) ? 0 : mat[acgt_of_code[qc] * 4 + acgt_of_code[tc]];
        /* kept across calls while the gap table is the same (-jobs
         * batches); held locked until the DP that reads it is done */
        /* 2^15 distances; 2^18 (past the built-in tables' last long
         * position) when a pair is large enough for its DP to pay back the
         * few ms: the interpolation range then never reaches the function */
        int64_t big = 0;
        for (int64_t p = 0; p < np; ++p)
            if (in->blk_off[p + 1] - in->blk_off[p] > big)
                big = in->blk_off[p + 1] - in->blk_off[p];
        const int len = big > 200000 ? 1 << 18 : 1 << 15;
        pthread_mutex_lock(&g_gtab_mu);
        if (!cached_g || !gac_gapcalc_same(cached_g, g) || cached_len < len) {
            int32_t *tab = malloc((size_t)3 * len * sizeof(int32_t));
            for (int d = 0; d < len; ++d) {
                tab[d] = gac_gap_cost(g, d, 0);
                tab[len + d] = gac_gap_cost(g, 0, d);
                tab[2 * len + d] = d >= 2 ? gac_gap_cost(g, 1, d - 1) : gac_gap_cost(g, 0, 0);
            }
            gac_gapcalc_free(cached_g);
            free(cached_tab);
            cached_g = gac_gapcalc_clone(g);
            cached_tab = tab;
            cached_len = len;
        }
        env.gtab_len = cached_len;
        env.gtab = cached_tab;
        env.last_pos[0] = g->q_last_pos;
        env.last_pos[1] = g->t_last_pos;
        env.last_pos[2] = g->b_last_pos;
        env.last_val[0] = g->q_last_val;
        env.last_val[1] = g->t_last_val;
        env.last_val[2] = g->b_last_val;
        env.last_slope[0] = g->q_last_slope;
        env.last_slope[1] = g->t_last_slope;
        env.last_slope[2] = g->b_last_slope;
        dp_fast_setup(&env);
    }
    stage("host gap table", &tclock);
    /* ---- chainBlocks + overlap removal per pair on host threads */
    ax_out *po = calloc((size_t)(np ? np : 1), sizeof(ax_out));
    int32_t *order = malloc((size_t)(np ? np : 1) * sizeof(int32_t));
    int64_t *psize = malloc((size_t)(np ? np : 1) * sizeof(int64_t));
    for (int64_t p = 0; p < np; ++p) {
        order[p] = (int32_t)p;
        psize[p] = poff[p + 1] - poff[p];
    }
    qsort_r(order, (size_t)np, sizeof(int32_t), cmp_i64_desc_pair, psize);
    ax_job J;
    memset(&J, 0, sizeof(J));
    J.e = &env;
    J.ctx = ctx;
    J.in = in;
    J.poff = poff;
    J.qs = qs;
    J.qe = qe;
    J.ts = ts;
    J.te = te;
    J.score = score;
    J.info = info;
    J.order = order;
    J.n_pairs = np;
    atomic_init(&J.next, 0);
    J.out = po;
    J.want_details = details_path != NULL;
    int nt = nthreads;
    if (nt > np)
        nt = np > 0 ? (int)np : 1;
    const char *dpm = getenv("GAC_AXT_DP");
    if (dpm && strcmp(dpm, "gpu") == 0) {
        rc = axt_dp_gpu(&J, nt);
        stage("kd-tree DP (device)", &tclock);
    } else {
        /* the smallest pairs to the device, on a thread of their own (its
         * host phases -- trees, peel, finish -- on 2 threads of its own,
         * beside the host's: taking them from the pool was slower,
         * r05multi hx2) */
        const int64_t kd = dp_device_split(psize, order, np, &env);
        int64_t np_host = np, nb_host = nb; /* the host's pairs and blocks */
        dev_run *D = NULL;
        pthread_t dth;
        int dev_started = 0;
        if (kd < np) {
            D = calloc(1, sizeof(dev_run));
            memcpy(&D->J, &J, sizeof(J));
            D->J.order = order + kd;
            D->J.n_pairs = np - kd;
            atomic_init(&D->J.next, 0);
            const char *dtv = getenv("GAC_DP_DEV_THREADS"); /* (its host phases' threads) */
            D->nt = dtv && atoi(dtv) > 0 ? atoi(dtv) : 2;
            int64_t dl = 0;
            for (int64_t k = kd; k < np; ++k)
                dl += psize[order[k]];
            if (getenv("GAC_TIMING"))
                fprintf(stderr, "[gac_axt_chain] hybrid DP: %lld of %lld pairs (%lld of %lld blocks, "
                        "largest %lld) on the device\n", (long long)(np - kd), (long long)np,
                        (long long)dl, (long long)nb, (long long)psize[order[kd]]);
            nb_host = nb - dl;
            np_host = kd;
        }
        J.n_pairs = np_host;
        if (nt > np_host)
            nt = np_host > 0 ? (int)np_host : 1;
        /* the pairs that would be the critical path on one thread -- over
         * 2^20 blocks and over 1.5x an even share of all blocks (C4: the
         * 11.5 M and 5 M block pairs of 50 M) -- each run as a team
         * (pair_dp_team, parallel sorts / tree / finish) on its share of
         * the threads, beside a pool that takes every other pair, largest
         * first */
        int64_t big = 0;
        const char *tv = getenv("GAC_DP_TEAM");
        const int team_on = !(tv && *tv == '0') && nthreads > 2;
        const char *mv = getenv("GAC_DP_TEAM_MIN"); /* (tests: the size floor of a team pair) */
        const int64_t floor_ = mv && atoll(mv) > 0 ? atoll(mv) : (1 << 20);
        const char *sv = getenv("GAC_DP_SHARE"); /* (a team pair: over this many even shares) */
        const double mult = sv && atof(sv) > 0 ? atof(sv) : 1.5;
        const int64_t even = (int64_t)(mult * (double)(nb_host / nthreads));
        const int64_t share = mv ? floor_ : (even > floor_ ? even : floor_);
        while (team_on && big < np_host && psize[order[big]] > share && big < nthreads / 2)
            ++big;
        /* the team pairs' leaves and kd-trees built on the device first
         * (gac_kd_trees, ~0.1 s for C4's 20 M team blocks, vs ~0.5 s of the
         * largest team's critical path on its threads); then the device
         * takes its own pairs.  GAC_DP_TEAMTREE=0: built on the teams */
        ax_pre *pre = NULL;
        {
            const char *ttv = getenv("GAC_DP_TEAMTREE");
            if (big && !(ttv && *ttv == '0') && !(dpm && strcmp(dpm, "host") == 0)) {
                const double tp0 = now_s();
                pre = team_trees(&J, order, big, nthreads, &rc);
                if (getenv("GAC_TIMING"))
                    fprintf(stderr, "[gac_axt_chain] the %lld team pairs' leaves and kd-trees on the "
                            "device: %.3f s\n", (long long)big, now_s() - tp0);
            }
        }
        if (D) {
            if (pthread_create(&dth, NULL, dev_runner, D) == 0)
                dev_started = 1;
            else
                dev_runner(D);
        }
        team_run *tr = big ? calloc((size_t)big, sizeof(team_run)) : NULL;
        int pool = nt;
        if (big) {
            int64_t sum = 0;
            for (int64_t k = 0; k < big; ++k)
                sum += psize[order[k]];
            const char *pl = getenv("GAC_DP_POOL"); /* (threads beside the teams) */
            pool = pl && atoi(pl) > 0 && atoi(pl) < nthreads
                       ? atoi(pl)
                       : (nthreads / 3 > 1 ? nthreads / 3 : 1);
            /* the device's share relieves the pool: the pool shrinks with
             * its blocks (the threads it gives up run the device's host
             * phases -- pack, peel, finish -- beside it); the teams keep
             * theirs (r06dt3: C4, cap 200 k, pool 5 -> 3: 8.60 / 8.67 s vs
             * host-only 8.62 / 8.86 s; cap 50 k with the pool at 3: 9.39 s) */
            if (D && !(pl && atoi(pl) > 0) && nb - sum > 0) {
                const int64_t all = nb - sum, now = nb_host - sum > 0 ? nb_host - sum : 0;
                int p2 = (int)((pool * now + all - 1) / all);
                p2 = p2 < 2 ? 2 : p2;
                if (p2 < pool)
                    pool = p2;
            }
            if (pool > np_host - big) /* (no pool pairs left, e.g. an -nranks rank holding one big pair) */
                pool = (int)(np_host - big);
            const int tt = nthreads - pool;
            int used = 0;
            /* each team in an L3 domain of its own, from the one this
             * thread runs in (GAC_DP_PIN=0: wherever the scheduler puts it) */
            l3_dom dom[64];
            const char *pv = getenv("GAC_DP_PIN");
            const int nd = pv && *pv == '0' ? 0 : l3_domains(dom, 64);
            int d0 = 0;
            const int here = sched_getcpu();
            for (int d = 0; d < nd; ++d)
                if (here >= 0 && CPU_ISSET(here, &dom[d].set))
                    d0 = d;
            const char *db = getenv("GAC_DP_DOMAIN_BASE"); /* (axtChain -nranks: 2 x rank) */
            if (db && nd > 0)
                d0 = atoi(db) % nd;
            for (int64_t k = 0; k < big; ++k) {
                int t = (int)((double)tt * psize[order[k]] / (double)sum + 0.5);
                const char *t0v = getenv("GAC_DP_TEAM0"); /* (probe: the largest team's threads) */
                if (k == 0 && t0v && atoi(t0v) >= 2 && atoi(t0v) <= tt - 2 * (int)(big - 1))
                    t = atoi(t0v);
                t = t < 2 ? 2 : t;
                if (k == big - 1 || used + t > tt)
                    t = tt - used > 2 ? tt - used : 2;
                used += t;
                tr[k].J = &J;
                tr[k].pre = pre ? &pre[k] : NULL;
                tr[k].p = order[k];
                tr[k].team = t;
                if (nd >= 2 && k < nd && dom[(d0 + k) % nd].n >= t) {
                    tr[k].pin = 1;
                    tr[k].cpus = dom[(d0 + k) % nd].set;
                }
                if (getenv("GAC_TIMING"))
                    fprintf(stderr, "[gac_axt_chain] team %lld: pair %d, %d threads, %s\n", (long long)k,
                            order[k], t, tr[k].pin ? "in one L3 domain" : "unpinned");
                const char *bv = getenv("GAC_DP_BATCH");
                tr[k].batch = bv && atoi(bv) > 0 ? atoi(bv) : 2 * t;
                tr[k].env = &env;
                if (pthread_create(&tr[k].th, NULL, team_runner, &tr[k]) != 0) {
                    /* (no thread: here, unpinned -- a pinned caller would
                     * leave the pool and every later stage in one L3 domain) */
                    tr[k].pin = 0;
                    team_runner(&tr[k]);
                } else
                    tr[k].started = 1;
            }
            atomic_store(&J.next, big);
        }
        if (big == 0 || np_host > big)
            run_threads(pool, ax_thread, &J);
        if (big) {
            /* the pool's and the device's pairs scored while the teams run
             * (GAC_AXT_SCORE_EARLY=0: every pair's chains in one batch after
             * the teams) */
            const char *ev = getenv("GAC_AXT_SCORE_EARLY");
            if (!(ev && *ev == '0')) {
                if (D && dev_started) {
                    pthread_join(dth, NULL);
                    dev_started = 0;
                }
                stage("kd-tree DP (the pool's and the device's pairs)", &tclock);
                /* with the teams that are done by now (the smaller ones) */
                int32_t *cand = malloc((size_t)np * 4);
                int64_t ncand = 0;
                for (int64_t k = 0; k < np; ++k)
                    if (k >= big || atomic_load_explicit(&tr[k].done, memory_order_acquire))
                        cand[ncand++] = order[k];
                if (rc == GAC_OK && (!D || D->rc == GAC_OK))
                    rc = score_rest(ctx, po, in, np, cand, ncand, pool + (D ? D->nt : 0), &tclock);
                free(cand);
            }
        }
        for (int64_t k = 0; k < big; ++k)
            if (tr[k].started)
                pthread_join(tr[k].th, NULL);
        free(tr);
        free(pre); /* (its arrays went to the teams' work) */
        if (big)
            stage("kd-tree DP (teams on the largest pairs, beside the pool)", &tclock);
        else
            stage("kd-tree DP (threads)", &tclock);
        if (D) {
            if (dev_started)
                pthread_join(dth, NULL);
            if (getenv("GAC_TIMING"))
                fprintf(stderr, "[gac_axt_chain] hybrid DP: the device's %lld pairs took %.3f s\n",
                        (long long)D->J.n_pairs, D->secs);
            if (D->rc != GAC_OK && rc == GAC_OK)
                rc = D->rc;
            free(D);
            stage("kd-tree DP (the device's pairs joined)", &tclock);
        }
    }
    if (getenv("GAC_TIMING")) {
        double sum = 0, mx = 0;
        int64_t imx = 0;
        for (int64_t p = 0; p < np; ++p) {
            sum += po[p].secs;
            if (po[p].secs > mx) {
                mx = po[p].secs;
                imx = p;
            }
        }
        fprintf(stderr, "[gac_axt_chain] %d threads, %lld pairs, %lld blocks: sum %.3f s, largest "
                        "pair %lld (%lld blocks) %.3f s\n", nt, (long long)np, (long long)nb, sum,
                (long long)imx, (long long)(poff[imx + 1] - poff[imx]), mx);
    }
    pthread_mutex_unlock(&g_gtab_mu);
    free(score);
    free(order);
    free(psize);
    for (int64_t p = 0; p < np; ++p)
        if (po[p].err) {
            rc = gac_fail(GAC_E_FORMAT, "%s", po[p].msg);
            break;
        }
    if (rc == GAC_OK && details_path) {
        FILE *f = fopen(details_path, "w");
        if (!f) {
            rc = gac_fail(GAC_E_IO, "Can't open %s to write", details_path);
        } else {
            for (int64_t p = 0; p < np; ++p)
                if (po[p].details_len)
                    fwrite(po[p].details, 1, po[p].details_len, f);
            if (fclose(f) != 0)
                rc = gac_fail(GAC_E_IO, "Can't close %s", details_path);
        }
    }
    gac_axt_chains *R = NULL;
    if (rc == GAC_OK) {
        /* ---- chainCalcScore of every chain not scored yet: one GPU batch
         * (score_pairs) */
        rc = score_rest(ctx, po, in, np, NULL, np, nthreads, &tclock);
        int64_t nc = 0;
        int64_t *c0 = malloc((size_t)(np + 1) * 8);
        c0[0] = 0;
        for (int64_t p = 0; p < np; ++p)
            c0[p + 1] = c0[p] + po[p].n_chains;
        nc = c0[np];
        int32_t *cpair = malloc((size_t)(nc ? nc : 1) * 4);
        int64_t *gsc = malloc((size_t)(nc ? nc : 1) * 8);
        if (rc == GAC_OK) {
            list_job L = {po, c0, np, nc, cpair, gsc, 0};
            atomic_init(&L.next, 0);
            run_threads(nthreads, list_thread, &L);
        }
        stage("scores in list order", &tclock);
        if (rc == GAC_OK) {
            /* minScore filter; slAddHead onto the master list (reversed),
             * then slSort(chainCmpScore) -- stable */
            dkey *k = malloc((size_t)(nc ? nc : 1) * sizeof(dkey));
            int64_t nk = 0;
            for (int64_t i = nc - 1; i >= 0; --i)
                if ((double)gsc[i] >= min_score) {
                    k[nk] = (dkey){(double)gsc[i], (int32_t)nk, (int32_t)i};
                    ++nk;
                }
            sort_desc16(k, nk, nthreads); /* (ranks in list order: the stable sort) */
            R = calloc(1, sizeof(*R));
            R->n_chains = nk;
            R->score = malloc((size_t)(nk ? nk : 1) * sizeof(double));
            R->pair = malloc((size_t)(nk ? nk : 1) * 4);
            R->t_start = malloc((size_t)(nk ? nk : 1) * 4);
            R->t_end = malloc((size_t)(nk ? nk : 1) * 4);
            R->q_start = malloc((size_t)(nk ? nk : 1) * 4);
            R->q_end = malloc((size_t)(nk ? nk : 1) * 4);
            R->blk_off = malloc((size_t)(nk + 1) * 8);
            R->blk_off[0] = 0;
            for (int64_t j = 0; j < nk; ++j) {
                const int32_t i = k[j].v, p = cpair[i], c = (int32_t)(i - c0[p]);
                R->blk_off[j + 1] = R->blk_off[j] + (po[p].coff[c + 1] - po[p].coff[c]);
            }
            const int64_t tb = R->blk_off[nk];
            R->n_blocks = tb;
            R->blk_t = malloc((size_t)(tb ? tb : 1) * 4);
            R->blk_q = malloc((size_t)(tb ? tb : 1) * 4);
            R->blk_size = malloc((size_t)(tb ? tb : 1) * 4);
            out_job O = {R, k, po, c0, gsc, cpair, nk, 0};
            atomic_init(&O.next, 0);
            run_threads(nthreads, out_thread, &O);
            free(k);
        }
        void *big[] = {c0, cpair, gsc};
        free_later(big, (int)(sizeof(big) / sizeof(big[0])));
    }
    /* every pair's chains (GBs at C4): freed on a detached thread, off the
     * caller's path */
    {
        void **pp = malloc((size_t)(6 * np + 1) * sizeof(void *));
        int64_t k = 0;
        for (int64_t p = 0; p < np; ++p) {
            pp[k++] = po[p].gsc;
            pp[k++] = po[p].coff;
            pp[k++] = po[p].bt;
            pp[k++] = po[p].bq;
            pp[k++] = po[p].bs;
            pp[k++] = po[p].details;
        }
        pp[k++] = po;
        free_later(pp, (int)k);
        free(pp);
    }
    stage("filter + sort", &tclock);
    if (rc == GAC_OK)
        *out = R;
fail:
    free(poff);
    free(qs);
    free(qe);
    free(ts);
    free(te);
    free(bsz);
    free(info);
    return rc;
}
