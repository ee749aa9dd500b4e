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
typedef struct ax_node { /* struct kdBranch (chainBlock.c:17-28) */
    int32_t lo, hi, leaf, cut;
    double max_score;
    int32_t max_q, max_t;
} ax_node;

typedef struct ax_out { /* one pair's result */
    int32_t n_chains;
    int32_t *coff;           /* [n_chains + 1] */
    int32_t *bt, *bq, *bs;   /* blocks after overlap removal + merge */
    char *details;
    size_t details_len;
    int err;
    char msg[512];
    double secs; /* wall time of this pair's chaining */
} ax_out;

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
    memcpy(a, tmp, (size_t)n * sizeof(int32_t));
}

/* kdBuild (chainBlock.c:124-164): Q in query order, T in target order */
static int32_t kd_build(ax_work *w, int32_t *Q, int32_t *T, int32_t n, int dim) {
    const int32_t id = w->nn++;
    if (n == 1) {
        const int32_t l = Q[0];
        /* leaf node: lo/hi carry the leaf's qStart/tStart */
        w->nodes[id] = (ax_node){w->qs[l], w->ts[l], l, 0, 0.0, w->qe[l], w->te[l]};
        return id;
    }
    const int32_t half = n / 2;
    for (int32_t i = 0; i < n; ++i) /* clearHits(lists[0]) */
        w->hit[Q[i]] = 0;
    const int32_t *D = dim == 0 ? Q : T; /* medianVal: first n/2 marked */
    for (int32_t i = 0; i < half; ++i)
        w->hit[D[i]] = 1;
    const int32_t ml = D[half - 1];
    const int32_t cut = dim == 0 ? w->qs[ml] : w->ts[ml];
    partition(Q, n, w->hit, w->tmp);
    partition(T, n, w->hit, w->tmp);
    /* hi first: nodes land in the DFS's usual visiting order (pre-order,
     * hi before lo), so a search walks memory forward */
    const int32_t hi = kd_build(w, Q + half, T + half, n - half, 1 - dim);
    const int32_t lo = kd_build(w, Q, T, half, 1 - dim);
    ax_node *nd = &w->nodes[id];
    nd->lo = lo;
    nd->hi = hi;
    nd->leaf = -1;
    nd->cut = cut;
    nd->max_score = 0.0;
    nd->max_q = w->nodes[lo].max_q > w->nodes[hi].max_q ? w->nodes[lo].max_q : w->nodes[hi].max_q;
    nd->max_t = w->nodes[lo].max_t > w->nodes[hi].max_t ? w->nodes[lo].max_t : w->nodes[hi].max_t;
    return id;
}

enum { kStack = 512 };

/* bestPredecessor (chainBlock.c:207-263), iterative with the same order:
 * the hi subtree (only when the lonely leaf lies past the cut) before lo */
static void best_predecessor(ax_work *w, int32_t lonely, double *ret_score, int32_t *ret_pred) {
    const int32_t lq = w->qs[lonely], lt = w->ts[lonely];
    const double lscore = w->score[lonely];
    double best = 0.0;
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
        double max_score = nd->max_score + lscore;
        if (max_score < best)
            continue;
        max_score -= w->cb_gap ? w->cb_gap(lq - nd->max_q, lt - nd->max_t, w->cb_user)
                               : gap_cost(w->e, lq - nd->max_q, lt - nd->max_t);
        if (max_score < best)
            continue;
        if (nd->leaf >= 0) {
            const int32_t l = nd->leaf;
            if (nd->lo < lq && nd->hi < lt) {
                const double s = w->total[l] + lscore - connect_cost(w, l, lonely);
                if (s > best) {
                    best = s;
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
        if (coord > nd->cut) {
            st_node[sp] = nd->hi;
            st_dim[sp++] = (uint8_t)(1 - dim);
        }
    }
    *ret_score = best;
    *ret_pred = best_node;
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
        if (nd->max_score < total)
            nd->max_score = total;
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
    qsort(k, (size_t)nl, sizeof(ikey), ikey_cmp);
    for (int32_t i = 0; i < nl; ++i)
        w->tord[i] = k[i].v;
    for (int32_t i = 0; i < nl; ++i)
        k[i] = (ikey){w->qs[w->tord[i]], i, w->tord[i]};
    qsort(k, (size_t)nl, sizeof(ikey), ikey_cmp);
    for (int32_t i = 0; i < nl; ++i)
        w->qord[i] = k[i].v;
    free(k);
    for (int32_t i = 0; i < nb; ++i) {
        w->total[i] = w->score[i];
        w->pred[i] = -1;
    }
    return nl;
}

/* kdTreeMake (chainBlock.c:166-205); the tree is built from copies: kd_build
 * permutes its lists */
static void pair_tree(ax_work *w) {
    const int32_t nl = w->nl;
    int32_t *Q = malloc((size_t)nl * sizeof(int32_t)), *T = malloc((size_t)nl * sizeof(int32_t));
    memcpy(Q, w->qord, (size_t)nl * sizeof(int32_t));
    memcpy(T, w->tord, (size_t)nl * sizeof(int32_t));
    w->nn = 0;
    kd_build(w, Q, T, nl, 0);
    free(Q);
    free(T);
}

/* findBestPredecessors (chainBlock.c:281-300) on this thread */
static void pair_dp_host(ax_work *w) {
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
}

/* the chains peelChains (chainBlock.c:311-373) takes off the tree: blocks of
 * chain c are cblk[cstart[c] .. cstart[c+1]), ascending */
typedef struct ax_chains {
    int32_t *cblk, *cstart;
    int32_t nc, nbk;
} ax_chains;

static void pair_peel(ax_work *w, const ax_pairinfo *pi, FILE *details, ax_chains *pc) {
    const int32_t nb = w->n, nl = w->nl;
    /* in totalScore order */
    dkey *dk = malloc((size_t)nl * sizeof(dkey));
    for (int32_t i = 0; i < nl; ++i)
        dk[i] = (dkey){w->total[w->tord[i]], i, w->tord[i]};
    qsort(dk, (size_t)nl, sizeof(dkey), dkey_cmp_desc);
    for (int32_t i = 0; i < nb; ++i)
        w->hit[i] = 0;
    int32_t *cblk = malloc((size_t)nl * sizeof(int32_t));
    int32_t *cstart = malloc((size_t)(nl + 1) * sizeof(int32_t));
    int32_t nc = 0, nbk = 0;
    for (int32_t i = 0; i < nl; ++i) {
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
            const int32_t pl = w->nodes[w->pred[lf]].leaf;
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

static void chain_pair(ax_work *w, const ax_pairinfo *pi, FILE *details, ax_out *out) {
    memset(out, 0, sizeof(*out));
    if (pair_leaves(w) == 0) {
        out->coff = calloc(1, sizeof(int32_t));
        return;
    }
    pair_tree(w);
    pair_dp_host(w);
    if (w->err)
        return;
    ax_chains pc;
    pair_peel(w, pi, details, &pc);
    pair_finish(w, &pc, NULL, out);
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
    w->cap_n = c;
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
        const int32_t p = J->order[k];
        const int64_t b0 = J->poff[p];
        const int32_t n = (int32_t)(J->poff[p + 1] - b0);
        ax_out *o = &J->out[p];
        w.err = 0;
        w.msg[0] = 0;
        if (gac_genome_view(J->ctx, GAC_Q, J->in->q_seq[p], &w.q.v) != GAC_OK ||
            gac_genome_view(J->ctx, GAC_T, J->in->t_seq[p], &w.t.v) != GAC_OK) {
            memset(o, 0, sizeof(*o));
            o->err = 1;
            snprintf(o->msg, sizeof(o->msg), "pair %d: no host sequence", p);
            continue;
        }
        w.q.minus = J->in->q_strand[p] ? 1 : 0;
        w.t.minus = 0;
        w.n = n;
        w.qs = J->qs + b0;
        w.qe = J->qe + b0;
        w.ts = J->ts + b0;
        w.te = J->te + b0;
        w.score = J->score + b0;
        work_reserve(&w, n);
        char *dbuf = NULL;
        size_t dlen = 0;
        FILE *df = J->want_details ? open_memstream(&dbuf, &dlen) : NULL;
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        chain_pair(&w, &J->info[p], df, o);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        o->secs = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
        if (df) {
            fclose(df);
            o->details = dbuf;
            o->details_len = dlen;
        }
        if (w.err) {
            o->err = 1;
            memcpy(o->msg, w.msg, sizeof(o->msg));
        }
    }
    free(w.total);
    free(w.pred);
    free(w.hit);
    free(w.tord);
    free(w.qord);
    free(w.tmp);
    free(w.nodes);
    free(w.xs);
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
}

static void gpair_free_export(ax_gpair *G) {
    free(G->na);
    free(G->nb);
    free(G->lf);
    free(G->lsc);
    free(G->lnode);
    free(G->poff);
    free(G->path);
    G->na = G->nb = G->lf = G->lsc = G->lnode = G->path = NULL;
    G->poff = NULL;
}

static void *gdp_thread(void *arg) {
    ax_gjob *X = arg;
    ax_job *J = X->J;
    for (;;) {
        const int64_t k = atomic_fetch_add(&X->next, 1);
        if (k >= J->n_pairs)
            break;
        const int32_t p = J->order[k];
        ax_gpair *G = &X->G[p];
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
            work_reserve(w, w->n);
            if (pair_leaves(w) > 0) {
                pair_tree(w);
                gpair_export(G);
            }
        } else if (X->phase == 2) {
            if (!G->ok || w->err)
                continue;
            if (w->nl == 0) {
                o->coff = calloc(1, sizeof(int32_t));
                continue;
            }
            const int64_t lo = X->leaf_off[p];
            for (int32_t i = 0; i < w->nl; ++i) {
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
            const int64_t x0 = X->xoff[p];
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

static int axt_dp_gpu(ax_job *J, int nt) {
    const int64_t np = J->n_pairs;
    ax_gpair *G = calloc((size_t)(np ? np : 1), sizeof(ax_gpair));
    ax_gjob X;
    memset(&X, 0, sizeof(X));
    X.J = J;
    X.G = G;
    atomic_init(&X.next, 0);
    int rc = GAC_OK;
    double t = gnow();
    gdp_phase(&X, 1, nt);
    double t1 = gnow();
    /* gather the pairs' trees */
    int64_t *node_off = malloc((size_t)(np + 1) * sizeof(int64_t));
    int64_t *leaf_off = malloc((size_t)(np + 1) * sizeof(int64_t));
    node_off[0] = leaf_off[0] = 0;
    int64_t npath = 0;
    for (int64_t p = 0; p < np; ++p) {
        const int live = G[p].ok && !G[p].w.err && G[p].w.nl > 0;
        node_off[p + 1] = node_off[p] + (live ? G[p].w.nn : 0);
        leaf_off[p + 1] = leaf_off[p] + (live ? G[p].w.nl : 0);
        npath += live ? G[p].poff[G[p].w.nl] : 0;
    }
    const int64_t nn = node_off[np], nl = leaf_off[np];
    int32_t *na = malloc((size_t)(nn ? nn : 1) * 16), *nb = malloc((size_t)(nn ? nn : 1) * 8);
    int32_t *lf = malloc((size_t)(nl ? nl : 1) * 16), *lsc = malloc((size_t)(nl ? nl : 1) * 4);
    int32_t *lnode = malloc((size_t)(nl ? nl : 1) * 4);
    int64_t *poff = malloc((size_t)(nl + 1) * 8);
    int32_t *path = malloc((size_t)(npath ? npath : 1) * 4);
    int64_t *total = malloc((size_t)(nl ? nl : 1) * 8);
    int32_t *pred = malloc((size_t)(nl ? nl : 1) * 4);
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
    }
    for (int64_t p = 0; p < np; ++p)
        if (leaf_off[p + 1] == leaf_off[p])
            for (int64_t i = leaf_off[p]; i < leaf_off[p + 1]; ++i)
                poff[i + 1] = poff[i];
    double t2 = gnow();
    rc = gac_chain_dp(J->ctx, np, J->in->t_seq, J->in->q_seq, J->in->q_strand, node_off, na, nb,
                      leaf_off, lf, lsc, lnode, poff, path, total, pred);
    double t3 = gnow();
    free(na);
    free(nb);
    free(lf);
    free(lsc);
    free(lnode);
    free(poff);
    free(path);
    free(node_off);
    int64_t *xoff = NULL;
    double t4 = t3, t5 = t3, t6 = t3;
    if (rc == GAC_OK) {
        X.leaf_off = leaf_off;
        X.total = total;
        X.pred = pred;
        gdp_phase(&X, 2, nt);
        t4 = gnow();
        xoff = malloc((size_t)(np + 1) * sizeof(int64_t));
        xoff[0] = 0;
        for (int64_t p = 0; p < np; ++p)
            xoff[p + 1] = xoff[p] + G[p].nx;
        const int64_t nx = xoff[np];
        int32_t *xt = malloc((size_t)(nx ? nx : 1) * 4), *xq = malloc((size_t)(nx ? nx : 1) * 4);
        uint8_t *xs = malloc((size_t)(nx ? nx : 1));
        int32_t *xv[5], *xpos = malloc((size_t)(nx ? nx : 1) * 4), *xadj = malloc((size_t)(nx ? nx : 1) * 4);
        for (int f = 0; f < 5; ++f)
            xv[f] = malloc((size_t)(nx ? nx : 1) * 4);
        for (int64_t p = 0; p < np; ++p)
            for (int32_t k = 0; k < G[p].nx; ++k) {
                const int64_t g = xoff[p] + k;
                xt[g] = J->in->t_seq[p];
                xq[g] = J->in->q_seq[p];
                xs[g] = J->in->q_strand[p] ? 1 : 0;
                for (int f = 0; f < 5; ++f)
                    xv[f][g] = G[p].xl[5 * k + f];
            }
        rc = gac_crossovers(J->ctx, nx, xt, xq, xs, xv[0], xv[1], xv[2], xv[3], xv[4], xpos, xadj);
        t5 = gnow();
        if (rc == GAC_OK) {
            X.xoff = xoff;
            X.xpos = xpos;
            X.xadj = xadj;
            X.xlqe = xv[0];
            X.xlte = xv[1];
            X.xrqs = xv[2];
            X.xrts = xv[3];
            X.xov = xv[4];
            gdp_phase(&X, 3, nt);
        }
        t6 = gnow();
        if (getenv("GAC_TIMING"))
            fprintf(stderr, "[gac_axt_chain] device DP: trees %.3f s, gather %.3f s, gac_chain_dp "
                            "%.3f s, peel %.3f s, %lld crossovers %.3f s, finish %.3f s\n",
                    t1 - t, t2 - t1, t3 - t2, t4 - t3, (long long)nx, t5 - t4, t6 - t5);
        free(xt);
        free(xq);
        free(xs);
        free(xpos);
        free(xadj);
        for (int f = 0; f < 5; ++f)
            free(xv[f]);
    }
    free(xoff);
    free(leaf_off);
    free(total);
    free(pred);
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
        free(w->xs);
    }
    free(G);
    return rc;
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
    int32_t *cpair;
    int64_t *coff;
    int32_t *bt, *bq, *bs;
    int64_t *c0, *x0; /* per pair: first chain, first block */
    int64_t np;
    _Atomic int64_t next;
} gather_job;

static void *gather_thread(void *arg) {
    gather_job *G = arg;
    for (;;) {
        const int64_t p = atomic_fetch_add(&G->next, 1);
        if (p >= G->np)
            return NULL;
        const ax_out *o = &G->po[p];
        int64_t c = G->c0[p], x = G->x0[p];
        for (int32_t k = 0; k < o->n_chains; ++k, ++c) {
            G->ct[c] = G->in->t_seq[p];
            G->cq[c] = G->in->q_seq[p];
            G->cs[c] = G->in->q_strand[p] ? 1 : 0;
            G->cpair[c] = (int32_t)p;
            const int32_t b0 = o->coff[k], b1 = o->coff[k + 1];
            memcpy(G->bt + x, o->bt + b0, (size_t)(b1 - b0) * 4);
            memcpy(G->bq + x, o->bq + b0, (size_t)(b1 - b0) * 4);
            memcpy(G->bs + x, o->bs + b0, (size_t)(b1 - b0) * 4);
            x += b1 - b0;
            G->coff[c + 1] = x;
        }
    }
}

/* the kept chains in output order (parallel over chains) */
typedef struct out_job {
    gac_axt_chains *R;
    const struct dkey *k;
    const int64_t *coff, *gsc;
    const int32_t *cpair, *bt, *bq, *bs;
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
            const int32_t i = O->k[j].v;
            const int64_t b0 = O->coff[i], b1 = O->coff[i + 1], o = R->blk_off[j];
            R->score[j] = (double)O->gsc[i];
            R->pair[j] = O->cpair[i];
            R->t_start[j] = O->bt[b0];
            R->q_start[j] = O->bq[b0];
            R->t_end[j] = O->bt[b1 - 1] + O->bs[b1 - 1];
            R->q_end[j] = O->bq[b1 - 1] + O->bs[b1 - 1];
            memcpy(R->blk_t + o, O->bt + b0, (size_t)(b1 - b0) * 4);
            memcpy(R->blk_q + o, O->bq + b0, (size_t)(b1 - b0) * 4);
            memcpy(R->blk_size + o, O->bs + b0, (size_t)(b1 - b0) * 4);
        }
    }
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
        run_threads(nt, ax_thread, &J);
        stage("kd-tree DP (threads)", &tclock);
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
        /* ---- chainCalcScore of every chain: one GPU batch */
        int64_t nc = 0, ncb = 0;
        for (int64_t p = 0; p < np; ++p) {
            nc += po[p].n_chains;
            ncb += po[p].coff ? po[p].coff[po[p].n_chains] : 0;
        }
        int32_t *ct = malloc((size_t)(nc ? nc : 1) * 4), *cq = malloc((size_t)(nc ? nc : 1) * 4);
        uint8_t *cs = malloc((size_t)(nc ? nc : 1));
        int32_t *cpair = malloc((size_t)(nc ? nc : 1) * 4);
        int64_t *coff = malloc((size_t)(nc + 1) * 8);
        int32_t *bt = malloc((size_t)(ncb ? ncb : 1) * 4), *bq = malloc((size_t)(ncb ? ncb : 1) * 4),
                *bs = malloc((size_t)(ncb ? ncb : 1) * 4);
        int64_t *gsc = malloc((size_t)(nc ? nc : 1) * 8);
        int32_t *gali = malloc((size_t)(nc ? nc : 1) * 4);
        /* every pair's chains into the set, pairs in parallel (disjoint
         * slots from prefix sums over the pairs) */
        gather_job G = {po, in, ct, cq, cs, cpair, coff, bt, bq, bs, NULL, NULL, np, 0};
        G.c0 = malloc((size_t)(np + 1) * 8);
        G.x0 = malloc((size_t)(np + 1) * 8);
        G.c0[0] = G.x0[0] = 0;
        for (int64_t p = 0; p < np; ++p) {
            G.c0[p + 1] = G.c0[p] + po[p].n_chains;
            G.x0[p + 1] = G.x0[p] + (po[p].coff ? po[p].coff[po[p].n_chains] : 0);
        }
        coff[0] = 0;
        atomic_init(&G.next, 0);
        run_threads(nthreads < np ? nthreads : (int)(np ? np : 1), gather_thread, &G);
        free(G.c0);
        free(G.x0);
        gac_chainset_desc d = {nc, ct, cq, cs, coff, ncb, bt, bq, bs};
        gac_chainset *set = NULL;
        if (nc > 0) { /* whole chains: chainCalcScore of each (axtChain.c:300-305) */
            rc = gac_chains_upload(ctx, &d, &set);
            if (rc == GAC_OK)
                rc = gac_score_chains(ctx, set, 0, gsc, NULL, gali);
            gac_chains_free(set);
        }
        stage("GPU chain scores", &tclock);
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
            qsort(k, (size_t)nk, sizeof(dkey), dkey_cmp_desc);
            R = calloc(1, sizeof(*R));
            R->n_chains = nk;
            R->score = malloc((size_t)(nk ? nk : 1) * sizeof(double));
            R->pair = malloc((size_t)(nk ? nk : 1) * 4);
            R->t_start = malloc((size_t)(nk ? nk : 1) * 4);
            R->t_end = malloc((size_t)(nk ? nk : 1) * 4);
            R->q_start = malloc((size_t)(nk ? nk : 1) * 4);
            R->q_end = malloc((size_t)(nk ? nk : 1) * 4);
            R->blk_off = malloc((size_t)(nk + 1) * 8);
            int64_t tb = 0;
            for (int64_t j = 0; j < nk; ++j)
                tb += coff[k[j].v + 1] - coff[k[j].v];
            R->n_blocks = tb;
            R->blk_t = malloc((size_t)(tb ? tb : 1) * 4);
            R->blk_q = malloc((size_t)(tb ? tb : 1) * 4);
            R->blk_size = malloc((size_t)(tb ? tb : 1) * 4);
            R->blk_off[0] = 0;
            for (int64_t j = 0; j < nk; ++j)
                R->blk_off[j + 1] = R->blk_off[j] + (coff[k[j].v + 1] - coff[k[j].v]);
            out_job O = {R, k, coff, gsc, cpair, bt, bq, bs, nk, 0};
            atomic_init(&O.next, 0);
            run_threads(nthreads, out_thread, &O);
            free(k);
        }
        free(ct);
        free(cq);
        free(cs);
        free(cpair);
        free(coff);
        free(bt);
        free(bq);
        free(bs);
        free(gsc);
        free(gali);
    }
    for (int64_t p = 0; p < np; ++p) {
        free(po[p].coff);
        free(po[p].bt);
        free(po[p].bq);
        free(po[p].bs);
        free(po[p].details);
    }
    free(po);
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
