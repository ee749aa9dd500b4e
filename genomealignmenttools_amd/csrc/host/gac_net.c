/* gac_net.c -- host netting engine of chainNet (C11), array-indexed.
 *
 * Same fill/gap trees, same .net text as the reference's
 * src/chainNet/chainNet.c, without its O(fills x blocks) list rescans:
 *   makeChroms / addSpaceForGap / findSpaces   :328-354, :289-300, :527-544
 *       -> per-chromosome B+tree of disjoint spaces, in-order range query;
 *          a filled space is replaced by its remnants and inner gaps at once
 *   addChainT / addChainQ / fillSpace / innerBounds / strictlyInside
 *       :557-679, :487-523, :356-391, :321-325
 *       -> identical decisions; the gap scan stops at the first gap that
 *          ends past the space (gaps are monotone), instead of walking the
 *          rest of the chain for every space
 *   sortNet / rCalcOtherFill / t,qFillOtherRange  :694-723, :393-484
 *       -> fills/gaps sorted once into arrays; other-side ranges by binary
 *          search to the first block of the fill
 *   rOutputFill / rOutputGap / fillOut / subchainInfo / outputNetSide
 *       :747-896 -> same traversal and printf formats; chainBaseCount and
 *          chainBaseCountSubT/SubQ come from per-chain prefix sums
 * Rescored T-side sub-chain scores are supplied by the caller (computed on
 * the GPU through gac_score_ranges); this file never scores bases.
 */
#define _GNU_SOURCE
#include "gac_host.h"

#include <immintrin.h>
#include <sched.h>
#include <stdint.h>
#include <sys/mman.h>
#include <pthread.h>
#include <stdatomic.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <time.h>
#include <stdlib.h>
#include <string.h>

#define BIGNUM 0x3fffffff /* kent common.h:117 */

typedef struct ngap ngap;
typedef struct nfill nfill;

struct ngap {
    int start, end, o_start, o_end;
    nfill *fill_head; /* slAddHead order until sorted */
    nfill **fills;
    int n_fills;
    ngap *next;   /* in parent fill's list */
    nfill *pfill; /* parent fill (NULL: a chromosome's root gap) */
    int32_t pidx; /* index in pfill->gaps; for a root gap, the chromosome */
};

struct nfill {
    int start, end, o_start, o_end;
    int32_t chain;
    int32_t ali;  /* the chain's aligned bases inside [start, end) (chainBaseCountSub*) */
    ngap **gaps; /* ascending (created in block order at fill time) */
    int n_gaps;
    int32_t full; /* the final [start, end) covers the chain's header span on this side */
    nfill *next;
    int64_t ord;  /* pre-order index on its side */
    ngap *pgap;   /* parent gap; index in pgap->fills; fills above this one */
    int32_t pidx, level;
    /* T side: the blocks chainSubsetOnT(chain, start, end) selects
     * (chain.c:481-500: from the first with tEnd > start while tStart < end),
     * chain-local first block and count, known from the netting's own walk */
    int32_t wb0, wn;
};

typedef struct nchrom {
    const char *name;
    int size;
    ngap *root;
    int32_t sroot; /* space index root (a leaf when height == 0) */
    int32_t height;
} nchrom;

/* ------------------------------------------------------------ arena */
typedef struct arena {
    char **blocks;
    size_t *sizes;
    size_t n, cap, used, bsize;
} arena;

/* Arena blocks are 32 MB, 2 MB-aligned anonymous mappings advised for huge
 * pages: a C5 net holds GBs of fills and gaps, and returning that many 4 KB
 * pages to the kernel at exit cost more than writing the nets did. */
#define ARENA_BLOCK ((size_t)32 << 20)
#define ARENA_ALIGN ((size_t)2 << 20)

static char *arena_map(size_t bs) {
    size_t len = bs + ARENA_ALIGN;
    char *m = mmap(NULL, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (m == MAP_FAILED) {
        fprintf(stderr, "gac_net: out of memory mapping %zu bytes\n", bs);
        abort();
    }
    char *p = (char *)(((uintptr_t)m + ARENA_ALIGN - 1) & ~(uintptr_t)(ARENA_ALIGN - 1));
    if (p > m)
        munmap(m, (size_t)(p - m));
    if (p + bs < m + len)
        munmap(p + bs, (size_t)(m + len - (p + bs)));
#ifdef MADV_HUGEPAGE
    madvise(p, bs, MADV_HUGEPAGE);
#endif
    return p;
}

static void *arena_alloc(arena *a, size_t sz) {
    sz = (sz + 15) & ~(size_t)15;
    if (a->n == 0 || a->used + sz > a->bsize) {
        if (a->n == a->cap) {
            a->cap = a->cap ? a->cap * 2 : 64;
            a->blocks = realloc(a->blocks, a->cap * sizeof(char *));
            a->sizes = realloc(a->sizes, a->cap * sizeof(size_t));
        }
        size_t bs = sz > ARENA_BLOCK ? (sz + ARENA_ALIGN - 1) & ~(ARENA_ALIGN - 1) : ARENA_BLOCK;
        a->blocks[a->n] = arena_map(bs);
        a->sizes[a->n++] = bs;
        a->bsize = bs;
        a->used = 0;
    }
    char *p = a->blocks[a->n - 1] + a->used;
    a->used += sz;
    /* the next allocations land just past this one: fetch those lines for
     * writing now (fresh arena memory: every new line is a miss) */
    if (a->used + 512 <= a->bsize)
        __builtin_prefetch(p + sz + 384, 1, 3);
    return p;
}

/* The arenas' pages are dropped by madvise (under the mm's read lock, so the
 * free workers run in parallel) before munmap (write lock: serial, and then
 * cheap): C5 chainNet's nets freed in 0.055 s instead of 0.216 s, one core
 * busy (`profiles/r04free/`).  GAC_FREE_MADV=0: munmap only. */
static int g_free_madv = -1;

static void arena_free(arena *a) {
    for (size_t i = 0; i < a->n && g_free_madv == 1; ++i)
        madvise(a->blocks[i], a->sizes[i], MADV_DONTNEED);
    for (size_t i = 0; i < a->n; ++i)
        munmap(a->blocks[i], a->sizes[i]);
    free(a->blocks);
    free(a->sizes);
    memset(a, 0, sizeof(*a));
}

/* One netting worker: the side trees of the chromosomes it nets live in its
 * own space pool and arena (chromosomes are independent: every chain is
 * added to its target chromosome's tree and to its query chromosome's tree,
 * each in score order, and nothing else is shared). */
typedef struct nwork {
    arena ar;
    /* space index pools (shared by the chromosomes this worker nets) */
    struct sleaf *lf;
    int32_t lf_n, lf_cap, lf_free;
    struct snode *in;
    int32_t in_n, in_cap, in_free;
    /* scratch: findSpaces result, a fill's new spaces, leaf split runs */
    struct sitem *q, *it, *cmb;
    int64_t q_n, q_cap, it_n, it_cap, cmb_cap;
    /* scratch for reversed blocks */
    int32_t *rs, *re, *ros, *roe, *ro; /* ro: each block's other-side start */
    int64_t r_cap;
    /* finishNet scratch: a gap's fill list gathered in one walk */
    struct nfill **sf;
    int64_t sf_cap;
    char pad[64]; /* keep workers' hot fields on separate cache lines */
} nwork;

struct gac_net {
    gac_net_input in;
    gac_net_opts opt;
    int64_t n_netted;
    nchrom *chroms[2]; /* [GAC_T], [GAC_Q] */
    int32_t n_chroms[2];
    nwork *w;          /* [n_w]; w[0] also holds the finishNet arrays */
    int n_w;
    int64_t *chain_ali; /* per chain: aligned bases (chainBaseCount) */
    /* pre-order fill index per side */
    nfill **order[2];
    int64_t n_order[2];
    /* per side, by pre-order position: the parent fill's position (-1 at
     * top level), filled by the first pass that chases the parent links
     * (gac_net_get_fills with flags) and read by the output's "reached" pass */
    int64_t *pord[2];
    int pord_ok[2];          /* (set once, release/acquire: never rebuilt) */
    pthread_mutex_t pord_mu; /* the first build of pord (callers share a const net) */
    /* per side, ascending: the pre-order positions of the top-level fills
     * (where the runs of whole subtrees may start), from finishNet */
    int64_t *top[2];
    int64_t n_top[2];
    int32_t *nlen[2]; /* [GAC_T] / [GAC_Q]: the sequence names' lengths */
    int sides; /* bit 1 << side: side netted */
    atomic_int free_next; /* gac_net_free's worker cursor */
};

/* ------------------------------------------------------------ space index */
/* The open spaces of one chromosome side (chainNet.c's per-chrom rbTree of
 * spaces, :289-300): disjoint [start, end) intervals, each pointing at the
 * gap it lies in.  A B+tree over start with wide nodes, so a chain's range
 * query and the replacement of a filled space by its remnants and inner gaps
 * touch a few cache lines instead of a treap's ~30 dependent nodes.  Leaves
 * are linked in order; inner separators are kept exact (key[i] = smallest
 * start under child i, i >= 1); empty leaves are unlinked. */
#define SP_LF 32    /* spaces per leaf */
#define SP_IF 32    /* children per inner node */
#define SP_FILL 24  /* entries per node after a split */
#define SP_MAXH 24

typedef struct sleaf {
    int32_t n, next, prev, pad;
    int32_t start[SP_LF], end[SP_LF];
    ngap *gap[SP_LF];
} sleaf;

typedef struct snode {
    int32_t n;
    int32_t child[SP_IF];
    int64_t key[SP_IF]; /* spkey of the smallest space under child i (i >= 1) */
} snode;

/* spaces ordered by (start, end): only zero-length spaces (-minSpace=0) share
 * a start */
static inline int64_t spkey(int32_t s, int32_t e) { return ((int64_t)s << 32) | (uint32_t)e; }

typedef struct sitem {
    int32_t start, end;
    ngap *gap;
} sitem;

/* Element moves inside a node or a gap's list: a few entries at a time,
 * tens of millions of times per net -- inline loops, not memmove/memcpy
 * library calls (the loop-to-call rewrite is off for these). */
#define NO_LIBCALL __attribute__((optimize("no-tree-loop-distribute-patterns")))
NO_LIBCALL static inline void move_i32(int32_t *a, int to, int from, int cnt) {
    if (to > from)
        for (int k = cnt - 1; k >= 0; --k)
            a[to + k] = a[from + k];
    else
        for (int k = 0; k < cnt; ++k)
            a[to + k] = a[from + k];
}
NO_LIBCALL static inline void move_gap(ngap **a, int to, int from, int cnt) {
    if (to > from)
        for (int k = cnt - 1; k >= 0; --k)
            a[to + k] = a[from + k];
    else
        for (int k = 0; k < cnt; ++k)
            a[to + k] = a[from + k];
}
NO_LIBCALL static inline void copy_fill(nfill **d, nfill *const *s, int64_t cnt) {
    for (int64_t k = 0; k < cnt; ++k)
        d[k] = s[k];
}

static int32_t sp_new_leaf(nwork *w) {
    int32_t i;
    if (w->lf_free >= 0) {
        i = w->lf_free;
        w->lf_free = w->lf[i].next;
    } else {
        if (w->lf_n == w->lf_cap) {
            w->lf_cap = w->lf_cap ? w->lf_cap * 2 : 1 << 12;
            w->lf = realloc(w->lf, (size_t)w->lf_cap * sizeof(sleaf));
        }
        i = w->lf_n++;
    }
    w->lf[i].n = 0;
    w->lf[i].next = w->lf[i].prev = -1;
    return i;
}

static int32_t sp_new_inner(nwork *w) {
    int32_t i;
    if (w->in_free >= 0) {
        i = w->in_free;
        w->in_free = w->in[i].child[0];
    } else {
        if (w->in_n == w->in_cap) {
            w->in_cap = w->in_cap ? w->in_cap * 2 : 1 << 10;
            w->in = realloc(w->in, (size_t)w->in_cap * sizeof(snode));
        }
        i = w->in_n++;
    }
    w->in[i].n = 0;
    return i;
}

static void sp_init(nwork *w, nchrom *c, int start, int end, ngap *gap) {
    const int32_t l = sp_new_leaf(w);
    w->lf[l].n = 1;
    w->lf[l].start[0] = start;
    w->lf[l].end[0] = end;
    w->lf[l].gap[0] = gap;
    c->sroot = l;
    c->height = 0;
}

/* The node searches as branch-free counts over a whole node (AVX2, 32
 * entries in 4 or 8 compares): a node's entries are sorted, so the entries
 * <= key are a prefix and their count is the position a binary search
 * finds -- without its mispredicted branches (the netting's largest single
 * cost in a line profile).  Lanes past n hold stale entries and are masked. */
static int g_avx2 = -1;
_Static_assert(SP_LF == 32 && SP_IF == 32, "the AVX2 node counts assume 32-entry nodes");

__attribute__((target("avx2"))) static int inner_count_avx2(const snode *s, int64_t key) {
    const __m256i k = _mm256_set1_epi64x(key);
    unsigned le = 0;
    for (int j = 0; j < SP_IF; j += 4) {
        const __m256i v = _mm256_loadu_si256((const __m256i *)(s->key + j));
        const unsigned gt = (unsigned)_mm256_movemask_pd(_mm256_castsi256_pd(_mm256_cmpgt_epi64(v, k)));
        le |= (~gt & 0xfu) << j;
    }
    const unsigned m = (s->n >= 32 ? 0xffffffffu : ((1u << s->n) - 1u)) & ~1u; /* keys [1, n) */
    return __builtin_popcount(le & m);
}

/* entries with spkey(start, end) <= key: start < ks, or start == ks and
 * end <= ke (starts and ends are non-negative int32) */
__attribute__((target("avx2"))) static int leaf_count_avx2(const sleaf *L, int64_t key) {
    const __m256i ks = _mm256_set1_epi32((int32_t)(key >> 32));
    const __m256i ke = _mm256_set1_epi32((int32_t)(uint32_t)key);
    unsigned le = 0;
    for (int j = 0; j < SP_LF; j += 8) {
        const __m256i st = _mm256_loadu_si256((const __m256i *)(L->start + j));
        const __m256i en = _mm256_loadu_si256((const __m256i *)(L->end + j));
        const __m256i lt = _mm256_cmpgt_epi32(ks, st);
        const __m256i eq = _mm256_andnot_si256(_mm256_cmpgt_epi32(en, ke), _mm256_cmpeq_epi32(st, ks));
        le |= (unsigned)_mm256_movemask_ps(_mm256_castsi256_ps(_mm256_or_si256(lt, eq))) << j;
    }
    const unsigned m = L->n >= 32 ? 0xffffffffu : ((1u << L->n) - 1u);
    return __builtin_popcount(le & m);
}

static inline int have_avx2(void) {
    if (g_avx2 < 0)
        g_avx2 = __builtin_cpu_supports("avx2") && !getenv("GAC_NET_NO_AVX2");
    return g_avx2;
}

/* descend to the leaf holding the last space with start <= key; pn/pi = the
 * inner node and child index taken at each depth (root = depth 0) */
static int32_t sp_descend(const nwork *w, const nchrom *c, int64_t key, int32_t *pn, int *pi) {
    int32_t x = c->sroot;
    const int v = have_avx2();
    for (int d = 0; d < c->height; ++d) {
        const snode *s = &w->in[x];
        int lo = 1, hi = s->n; /* first i >= 1 with key[i] > key, minus one */
        if (v) {
            lo = 1 + inner_count_avx2(s, key);
            hi = lo;
        }
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s->key[mid] > key)
                hi = mid;
            else
                lo = mid + 1;
        }
        const int i = lo - 1;
        if (pn) {
            pn[d] = x;
            pi[d] = i;
        }
        x = s->child[i];
    }
    return x;
}

static int sp_leaf_pos(const sleaf *L, int64_t key) {
    if (have_avx2())
        return leaf_count_avx2(L, key) - 1;
    int lo = 0, hi = L->n; /* first i with spkey > key, minus one */
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (spkey(L->start[mid], L->end[mid]) > key)
            hi = mid;
        else
            lo = mid + 1;
    }
    return lo - 1;
}

static void sq_push(nwork *w, int32_t s, int32_t e, ngap *g) {
    if (w->q_n == w->q_cap) {
        w->q_cap = w->q_cap ? w->q_cap * 2 : 1024;
        w->q = realloc(w->q, (size_t)w->q_cap * sizeof(sitem));
    }
    w->q[w->q_n++] = (sitem){s, e, g};
}

/* spaces overlapping [qs, qe) in order (spaceCmp == 0, chainNet.c:277-287)
 * into w->q, leaving out those that overlap none of the chain's blocks
 * s[k], e[k] (sorted, disjoint): innerBounds finds nothing in them, so
 * addChain skips them anyway.  Runs of spaces inside one chain gap are
 * jumped over by a descent instead of a scan. */
static void sp_query(nwork *w, const nchrom *c, int qs, int qe, const int32_t *bs,
                     const int32_t *be, int nb) {
    w->q_n = 0;
    int k = 0; /* first block with end > the current space's start */
    int64_t key = spkey(qs, 0x7fffffff);
    for (;;) {
        int32_t l = sp_descend(w, c, key, NULL, NULL);
        int i = sp_leaf_pos(&w->lf[l], key);
        if (i < 0)
            i = 0;
        int jump = 0;
        while (l >= 0 && !jump) {
            const sleaf *L = &w->lf[l];
            for (; i < L->n; ++i) {
                const int ss = L->start[i], se = L->end[i];
                if (ss >= qe)
                    return;
                if (se <= qs)
                    continue;
                while (k < nb && be[k] <= ss)
                    ++k;
                if (k == nb)
                    return; /* past the last block */
                if (bs[k] < se) {
                    sq_push(w, ss, se, L->gap[i]);
                } else if (L->end[L->n - 1] <= bs[k] && L->next >= 0) {
                    /* the rest of this leaf lies in the gap before block k:
                     * on to the next leaf, or, when that one starts inside
                     * the gap too, a descent to the space holding bs[k]
                     * (which is then past this leaf: progress) */
                    if (w->lf[L->next].start[0] <= bs[k]) {
                        key = spkey(bs[k], 0x7fffffff);
                        jump = 1;
                    }
                    break;
                }
            }
            if (!jump) {
                l = L->next;
                i = 0;
            }
        }
        if (!jump)
            return;
    }
}

/* the smallest start under the child at depth d changed to v: fix the one
 * separator that holds it */
static void sp_fix_sep(nwork *w, const int32_t *pn, const int *pi, int d, int64_t v) {
    for (int k = d - 1; k >= 0; --k)
        if (pi[k] > 0) {
            w->in[pn[k]].key[pi[k]] = v;
            return;
        }
}

/* remove child pi[d] of inner node pn[d] (its subtree is already gone) */
static void sp_inner_remove(nwork *w, nchrom *c, const int32_t *pn, const int *pi, int d) {
    const int32_t x = pn[d];
    snode *s = &w->in[x];
    const int i = pi[d];
    const int64_t first_key = s->n > 1 ? s->key[1] : 0;
    memmove(s->key + i, s->key + i + 1, (size_t)(s->n - i - 1) * 8);
    memmove(s->child + i, s->child + i + 1, (size_t)(s->n - i - 1) * 4);
    --s->n;
    if (s->n == 0) {
        if (d == 0) { /* the whole tree is empty: one empty leaf */
            s->child[0] = w->in_free;
            w->in_free = x;
            c->sroot = sp_new_leaf(w);
            c->height = 0;
            return;
        }
        s->child[0] = w->in_free;
        w->in_free = x;
        sp_inner_remove(w, c, pn, pi, d - 1);
    } else if (i == 0) {
        sp_fix_sep(w, pn, pi, d, first_key); /* old key[1] is the new minimum */
    }
}

/* insert (key, child) pairs after child pi[d] of node pn[d], splitting as
 * needed (a new root when the root splits) */
static void sp_inner_insert(nwork *w, nchrom *c, const int32_t *pn, const int *pi, int d,
                            const int64_t *keys, const int32_t *childs, int cnt) {
    if (d < 0) { /* above the root: a new root over the old one and the new nodes */
        int32_t r = sp_new_inner(w);
        snode *s = &w->in[r];
        s->key[0] = 0;
        s->child[0] = c->sroot;
        s->n = 1;
        int32_t pn2[1] = {r};
        int pi2[1] = {0};
        c->sroot = r;
        c->height += 1;
        sp_inner_insert(w, c, pn2, pi2, 0, keys, childs, cnt);
        return;
    }
    const int32_t x = pn[d];
    const int at = pi[d] + 1, n0 = w->in[x].n, tot = n0 + cnt;
    if (tot <= SP_IF) {
        snode *s = &w->in[x];
        memmove(s->key + at + cnt, s->key + at, (size_t)(n0 - at) * 8);
        memmove(s->child + at + cnt, s->child + at, (size_t)(n0 - at) * 4);
        memcpy(s->key + at, keys, (size_t)cnt * 8);
        memcpy(s->child + at, childs, (size_t)cnt * 4);
        s->n = tot;
        return;
    }
    /* combined sequence, cut into nodes of SP_FILL */
    int64_t *ck = malloc((size_t)tot * 8);
    int32_t *cc = malloc((size_t)tot * 4);
    {
        const snode *s = &w->in[x];
        memcpy(ck, s->key, (size_t)at * 8);
        memcpy(cc, s->child, (size_t)at * 4);
        memcpy(ck + at, keys, (size_t)cnt * 8);
        memcpy(cc + at, childs, (size_t)cnt * 4);
        memcpy(ck + at + cnt, s->key + at, (size_t)(n0 - at) * 8);
        memcpy(cc + at + cnt, s->child + at, (size_t)(n0 - at) * 4);
    }
    const int parts = (tot + SP_FILL - 1) / SP_FILL;
    int64_t *nk = malloc((size_t)parts * 8);
    int32_t *nc = malloc((size_t)parts * 4);
    for (int p = 0; p < parts; ++p) {
        const int lo = (int)((int64_t)tot * p / parts), hi = (int)((int64_t)tot * (p + 1) / parts);
        const int32_t y = p == 0 ? x : sp_new_inner(w);
        snode *s = &w->in[y];
        memcpy(s->key, ck + lo, (size_t)(hi - lo) * 8);
        memcpy(s->child, cc + lo, (size_t)(hi - lo) * 4);
        s->n = hi - lo;
        nk[p] = ck[lo];
        nc[p] = y;
    }
    free(ck);
    free(cc);
    sp_inner_insert(w, c, pn, pi, d - 1, nk + 1, nc + 1, parts - 1);
    free(nk);
    free(nc);
}

/* replace the space [sstart, send) by items[0..m) (sorted, inside it) */
static void sp_replace(nwork *w, nchrom *c, int sstart, int send, const sitem *it, int m) {
    int32_t pn[SP_MAXH];
    int pi[SP_MAXH];
    const int32_t l = sp_descend(w, c, spkey(sstart, send), pn, pi);
    const int idx = sp_leaf_pos(&w->lf[l], spkey(sstart, send));
    if (idx < 0 || w->lf[l].start[idx] != sstart || w->lf[l].end[idx] != send) {
        fprintf(stderr, "gac_net: internal error: space %d-%d not indexed\n", sstart, send);
        abort();
    }
    const int n0 = w->lf[l].n, tot = n0 - 1 + m, H = c->height;
    if (tot == 0) {
        if (H == 0) {
            w->lf[l].n = 0;
            return;
        }
        sleaf *L = &w->lf[l];
        if (L->prev >= 0)
            w->lf[L->prev].next = L->next;
        if (L->next >= 0)
            w->lf[L->next].prev = L->prev;
        L->next = w->lf_free;
        w->lf_free = l;
        sp_inner_remove(w, c, pn, pi, H - 1);
        return;
    }
    if (idx == 0)
        sp_fix_sep(w, pn, pi, H, m > 0 ? spkey(it[0].start, it[0].end)
                                       : spkey(w->lf[l].start[1], w->lf[l].end[1]));
    if (tot <= SP_LF) {
        sleaf *L = &w->lf[l];
        move_i32(L->start, idx + m, idx + 1, n0 - idx - 1);
        move_i32(L->end, idx + m, idx + 1, n0 - idx - 1);
        move_gap(L->gap, idx + m, idx + 1, n0 - idx - 1);
        for (int k = 0; k < m; ++k) {
            L->start[idx + k] = it[k].start;
            L->end[idx + k] = it[k].end;
            L->gap[idx + k] = it[k].gap;
        }
        L->n = tot;
        return;
    }
    /* combined run, cut into leaves of SP_FILL linked after l */
    if (w->cmb_cap < tot) {
        w->cmb_cap = tot * 2;
        w->cmb = realloc(w->cmb, (size_t)w->cmb_cap * sizeof(sitem));
    }
    sitem *cb = w->cmb;
    {
        const sleaf *L = &w->lf[l];
        for (int k = 0; k < idx; ++k)
            cb[k] = (sitem){L->start[k], L->end[k], L->gap[k]};
        memcpy(cb + idx, it, (size_t)m * sizeof(sitem));
        for (int k = idx + 1; k < n0; ++k)
            cb[k - 1 + m] = (sitem){L->start[k], L->end[k], L->gap[k]};
    }
    const int parts = (tot + SP_FILL - 1) / SP_FILL;
    int64_t *nk = malloc((size_t)parts * 8);
    int32_t *nc = malloc((size_t)parts * 4);
    int32_t prev = -1;
    const int32_t after = w->lf[l].next;
    for (int p = 0; p < parts; ++p) {
        const int lo = (int)((int64_t)tot * p / parts), hi = (int)((int64_t)tot * (p + 1) / parts);
        const int32_t y = p == 0 ? l : sp_new_leaf(w);
        sleaf *L = &w->lf[y];
        for (int k = lo; k < hi; ++k) {
            L->start[k - lo] = cb[k].start;
            L->end[k - lo] = cb[k].end;
            L->gap[k - lo] = cb[k].gap;
        }
        L->n = hi - lo;
        if (p > 0) {
            L->prev = prev;
            w->lf[prev].next = y;
        }
        prev = y;
        nk[p] = spkey(cb[lo].start, cb[lo].end);
        nc[p] = y;
    }
    w->lf[prev].next = after;
    if (after >= 0)
        w->lf[after].prev = prev;
    sp_inner_insert(w, c, pn, pi, H - 1, nk + 1, nc + 1, parts - 1);
    free(nk);
    free(nc);
}

static ngap *gap_new(nwork *n, int s, int e, int os, int oe) {
    ngap *g = arena_alloc(&n->ar, sizeof(ngap));
    g->start = s;
    g->end = e;
    g->o_start = os;
    g->o_end = oe;
    return g;
}

/* ------------------------------------------------------------ netting */
static int strictly_inside(const gac_net *n, int min_start, int max_end, int start, int end) {
    return min_start < start && start + n->opt.min_space <= end && end < max_end;
}

static void it_push(nwork *w, int32_t s, int32_t e, ngap *g) {
    if (w->it_n == w->it_cap) {
        w->it_cap = w->it_cap ? w->it_cap * 2 : 1024;
        w->it = realloc(w->it, (size_t)w->it_cap * sizeof(sitem));
    }
    w->it[w->it_n++] = (sitem){s, e, g};
}

/* Generic addChainT/addChainQ on one side.  s[],e[] = this side's block
 * coordinates in list order (+ strand coords), os_gap/oe_gap = other-side
 * gap bounds per block (gap between block b and b+1).  Each filled space is
 * replaced in the index by its remnants and the chain's gaps strictly inside
 * it, in one leaf update (fillSpace + addSpaceForGap, chainNet.c:487-523). */

static void add_chain_side(const gac_net *net, nwork *n, nchrom *c, int32_t chain, int nb,
                           const int32_t *s, const int32_t *e, const int32_t *gos,
                           const int32_t *goe, const int32_t *os, int inv, int oflip, int cstart,
                           int cend, int boff) {
    sp_query(n, c, cstart, cend, s, e, nb);
    const int64_t nsp = n->q_n;
    /* each filled space's gap gets the fill pushed: its line is a cache
     * miss (the gap was made long before), so fetch them all now */
    for (int64_t si = 0; si < nsp; ++si)
        __builtin_prefetch(&n->q[si].gap->fill_head, 1);
    int k = 0;
    for (int64_t si = 0; si < nsp; ++si) {
        const int sstart = n->q[si].start, send = n->q[si].end;
        ngap *sgap = n->q[si].gap;
        while (k + 1 < nb && s[k + 1] <= sstart)
            ++k;
        /* innerBounds (chainNet.c:356-391), and the clipped blocks' bases:
         * the fill's aligned bases, since no block of the chain lies in the
         * space outside [start, end) */
        int start = BIGNUM, end = -BIGNUM, zero = 0;
        int fs = BIGNUM, fe = -BIGNUM, omin = BIGNUM, omax = -BIGNUM; /* (see below) */
        int wfirst = -1, wlast = -2; /* the blocks seen (window when none is zero-size) */
        int64_t ali = 0;
        for (int b = k; b < nb; ++b) {
            const int b0 = s[b], b1 = e[b];
            if (b1 <= sstart)
                continue;
            if (b0 >= send)
                break;
            if (wfirst < 0)
                wfirst = b;
            wlast = b;
            const int cs = b0 < sstart ? sstart : b0, ce = b1 > send ? send : b1;
            if (start > cs)
                start = cs;
            if (end < ce)
                end = ce;
            ali += ce - cs;
            if (ce > cs) {
                const int o0 = inv ? os[b] + (b1 - ce) : os[b] + (cs - b0);
                const int o1 = inv ? os[b] + (b1 - cs) : os[b] + (ce - b0);
                if (fs > cs) fs = cs;
                if (fe < ce) fe = ce;
                if (omin > o0) omin = o0;
                if (omax < o1) omax = o1;
            } else {
                zero = 1;
            }
        }
        if (end < 0 || end - start < net->opt.min_fill)
            continue;
        /* fillSpace (chainNet.c:487-523) */
        nfill *f = arena_alloc(&n->ar, sizeof(nfill));
        f->start = start;
        f->end = end;
        f->chain = chain;
        f->ali = (int32_t)ali;
        /* rCalcOtherFill (chainNet.c:393-484) now, on the same block slice:
         * the blocks clipped to [start, end) give the final own-side bounds
         * (zero-size blocks at the ends dropped; the order of a gap's fills
         * is unchanged, their spaces being disjoint) and the other side's
         * range (inv: the query side of a '-' chain, where the target runs
         * backwards; oflip: the target side of a '-' chain, whose query
         * range is flipped to + strand coordinates); f->full is subchainInfo's
         * whole-chain test (chainNet.c:802-823) */
        /* Every block with bases in the space is inside [start, end), so
         * the loop above already clipped it the same way and saw it; only a
         * zero-size block is treated differently (kept only strictly inside
         * the fill), and then the blocks are walked again */
        if (zero) {
            fs = BIGNUM, fe = -BIGNUM, omin = BIGNUM, omax = -BIGNUM;
            for (int b = k; b < nb; ++b) {
                const int bs = s[b], be = e[b];
                if (be <= start)
                    continue;
                if (bs >= end)
                    break;
                const int cs = bs < start ? start : bs, ce = be > end ? end : be;
                const int o0 = inv ? os[b] + (be - ce) : os[b] + (cs - bs);
                const int o1 = inv ? os[b] + (be - cs) : os[b] + (ce - bs);
                if (fs > cs) fs = cs;
                if (fe < ce) fe = ce;
                if (omin > o0) omin = o0;
                if (omax < o1) omax = o1;
            }
        }
        {
            if (oflip >= 0) {
                const int t = omin;
                omin = oflip - omax;
                omax = oflip - t;
            }
            f->start = fs;
            f->end = fe;
            f->o_start = omin;
            f->o_end = omax;
            f->full = fs <= cstart && fe >= cend;
        }
        if (boff >= 0) {
            /* chainSubsetOnT's window of [fs, fe): every block the walk saw
             * ends after fs (fs is the first clipped start) and starts before
             * fe -- unless a zero-size block sits at a bound, when the rule is
             * applied as written */
            if (zero) {
                wfirst = k;
                while (wfirst < nb && e[wfirst] <= fs)
                    ++wfirst;
                wlast = wfirst - 1;
                while (wlast + 1 < nb && s[wlast + 1] < fe)
                    ++wlast;
            }
            f->wb0 = boff + (wfirst < 0 ? 0 : wfirst);
            f->wn = wfirst < 0 ? 0 : wlast - wfirst + 1;
        }
        /* slAddHead onto the space's gap; region workers of one chromosome
         * side (net_regions) may share the gap, so the push is atomic.  The
         * order does not matter: finishNet sorts a gap's fills by start. */
        nfill *h = __atomic_load_n(&sgap->fill_head, __ATOMIC_RELAXED);
        do
            f->next = h;
        while (!__atomic_compare_exchange_n(&sgap->fill_head, &h, f, 1, __ATOMIC_RELEASE,
                                            __ATOMIC_RELAXED));
        n->it_n = 0;
        if (start - sstart >= net->opt.min_space)
            it_push(n, sstart, start, sgap);
        /* gaps strictly inside the space (all inside [start, end]) */
        const int64_t g0 = n->it_n;
        for (int b = k; b + 1 < nb; ++b) {
            int gs = e[b], ge = s[b + 1];
            if (ge >= send)
                break;
            if (strictly_inside(net, sstart, send, gs, ge))
                it_push(n, gs, ge, gap_new(n, gs, ge, gos[b], goe[b]));
        }
        f->n_gaps = (int)(n->it_n - g0);
        f->gaps = f->n_gaps ? arena_alloc(&n->ar, f->n_gaps * sizeof(ngap *)) : NULL;
        for (int i = 0; i < f->n_gaps; ++i)
            f->gaps[i] = n->it[g0 + i].gap;
        if (send - end >= net->opt.min_space)
            it_push(n, end, send, sgap);
        sp_replace(n, c, sstart, send, n->it, (int)n->it_n);
    }
}

static void ensure_rev(nwork *n, int64_t nb) {
    if (nb > n->r_cap) {
        n->r_cap = nb * 2;
        n->rs = realloc(n->rs, n->r_cap * 4);
        n->re = realloc(n->re, n->r_cap * 4);
        n->ros = realloc(n->ros, n->r_cap * 4);
        n->roe = realloc(n->roe, n->r_cap * 4);
        n->ro = realloc(n->ro, n->r_cap * 4);
    }
}

static int is_haplotype(const char *name) {
    return strstr(name, "_hap") != NULL || strstr(name, "_alt") != NULL;
}

/* Blocks of a chain that can touch spaces inside [A, B) (the whole chain
 * when A/B are INT32_MIN/MAX): those ending after A and starting before B,
 * plus one neighbour on each side, as an index range [*lo, *hi) over the
 * side's + strand block order, whose starts st(i) / ends en(i) ascend.  Every
 * space of a region lies inside [A, B), so innerBounds, the gaps strictly
 * inside a space and findSpaces' skips over chain gaps only ever look at
 * these blocks: a region worker builds just this slice of a long chain. */
#define SLICE(st, en)                                                                      \
    do {                                                                                   \
        int l = 0, h = nb;                                                                 \
        while (l < h) { /* first block ending after A */                                   \
            const int m = (l + h) >> 1;                                                    \
            if ((en(m)) > A) h = m;                                                        \
            else l = m + 1;                                                                \
        }                                                                                  \
        *lo = l > 0 ? l - 1 : 0;                                                           \
        h = nb;                                                                            \
        while (l < h) { /* first block starting at or after B */                           \
            const int m = (l + h) >> 1;                                                    \
            if ((st(m)) >= B) h = m;                                                       \
            else l = m + 1;                                                                \
        }                                                                                  \
        *hi = l < nb ? l + 1 : nb;                                                         \
    } while (0)

/* addChainQ (chainNet.c:610-679) */
static void add_chain_q(const gac_net *net, nwork *n, int64_t c, nchrom *qc, int A, int B) {
    const gac_net_input *in = &net->in;
    const int64_t b0 = in->blk_off[c];
    const int nb = (int)(in->blk_off[c + 1] - b0);
    const int32_t *bt = in->blk_t + b0, *bq = in->blk_q + b0, *bs = in->blk_size + b0;
    const int minus = in->q_strand[c] != 0;
    const int qsize = in->q_sizes[in->q_seq[c]];
    int qs = in->q_start[c], qe = in->q_end[c];
    int l0 = 0, l1 = nb, *lo = &l0, *hi = &l1;
    if (A != INT32_MIN || B != INT32_MAX) {
        if (!minus) {
#define QST(i) bq[i]
#define QEN(i) (bq[i] + bs[i])
            SLICE(QST, QEN);
        } else { /* reversed order: block i of the list is j = nb-1-i */
#define RST(i) (qsize - (bq[nb - 1 - (i)] + bs[nb - 1 - (i)]))
#define REN(i) (qsize - bq[nb - 1 - (i)])
            SLICE(RST, REN);
        }
    }
    const int m = l1 - l0;
    ensure_rev(n, m);
    if (!minus) {
        for (int b = l0; b < l1; ++b) {
            n->rs[b - l0] = bq[b];
            n->re[b - l0] = bq[b] + bs[b];
            n->ro[b - l0] = bt[b];
            if (b + 1 < nb) {
                n->ros[b - l0] = bt[b] + bs[b];
                n->roe[b - l0] = bt[b + 1];
            }
        }
    } else {
        int t = qs;
        qs = qsize - qe;
        qe = qsize - t;
        for (int i = l0; i < l1; ++i) {
            int j = nb - 1 - i; /* original index */
            n->rs[i - l0] = qsize - (bq[j] + bs[j]);
            n->re[i - l0] = qsize - bq[j];
            n->ro[i - l0] = bt[j];
            if (i + 1 < nb) { /* block = j, next = j-1 */
                n->ros[i - l0] = bt[j - 1];
                n->roe[i - l0] = bt[j] + bs[j];
            }
        }
    }
    add_chain_side(net, n, qc, (int32_t)c, m, n->rs, n->re, n->ros, n->roe, n->ro, minus, -1, qs,
                   qe, -1);
}

/* addChainT (chainNet.c:557-608) */
static void add_chain_t(const gac_net *net, nwork *n, int64_t c, nchrom *tc, int A, int B) {
    const gac_net_input *in = &net->in;
    const int64_t b0 = in->blk_off[c];
    const int nb = (int)(in->blk_off[c + 1] - b0);
    const int32_t *bt = in->blk_t + b0, *bq = in->blk_q + b0, *bs = in->blk_size + b0;
    const int minus = in->q_strand[c] != 0;
    const int qsize = in->q_sizes[in->q_seq[c]];
    int l0 = 0, l1 = nb, *lo = &l0, *hi = &l1;
    if (A != INT32_MIN || B != INT32_MAX) {
#define TST(i) bt[i]
#define TEN(i) (bt[i] + bs[i])
        SLICE(TST, TEN);
    }
    const int m = l1 - l0;
    ensure_rev(n, m);
    for (int b = l0; b < l1; ++b) {
        n->rs[b - l0] = bt[b];
        n->re[b - l0] = bt[b] + bs[b];
        n->ro[b - l0] = bq[b];
        if (b + 1 < nb) {
            int qs = bq[b] + bs[b], qe = bq[b + 1];
            if (minus) {
                int t = qs;
                qs = qsize - qe;
                qe = qsize - t;
            }
            n->ros[b - l0] = qs;
            n->roe[b - l0] = qe;
        }
    }
    add_chain_side(net, n, tc, (int32_t)c, m, n->rs, n->re, n->ros, n->roe, n->ro, 0,
                   minus ? qsize : -1, in->t_start[c], in->t_end[c], l0);
}

/* ------------------------------------------------------------ finish */
static int cmp_fill(const void *a, const void *b) {
    const nfill *x = *(nfill *const *)a, *y = *(nfill *const *)b;
    return (x->start > y->start) - (x->start < y->start);
}

/* finishNet per chromosome (sortNet + rCalcOtherFill, chainNet.c:694-723):
 * fills/gaps into sorted arrays, other-side ranges, and the chromosome's
 * fills in pre-order (numbered globally afterwards, in chromosome order) */
typedef struct fin_ctx {
    gac_net *n;
    nwork *w;
    int side;
    nfill **ord;
    int64_t n_ord, cap;
} fin_ctx;

static void finish_gap(fin_ctx *x, ngap *g);

static void finish_fill(fin_ctx *x, nfill *f) {
    if (x->n_ord == x->cap) {
        x->cap = x->cap ? x->cap * 2 : 256;
        x->ord = realloc(x->ord, (size_t)x->cap * sizeof(nfill *));
    }
    x->ord[x->n_ord++] = f;
    for (int i = 0; i < f->n_gaps; ++i) {
        f->gaps[i]->pfill = f;
        f->gaps[i]->pidx = i;
    }
    for (int i = 0; i < f->n_gaps; ++i)
        finish_gap(x, f->gaps[i]);
}

static void sort_gap_fills(nwork *w, ngap *g) {
    if (!g->fill_head) {
        g->n_fills = 0;
        g->fills = NULL;
        return;
    }
    /* one walk of the list (its fills are scattered over the arenas: every
     * link is a miss) into the worker's scratch, then the exact array */
    int cnt = 0;
    for (nfill *f = g->fill_head; f; f = f->next) {
        if (cnt == w->sf_cap) {
            w->sf_cap = w->sf_cap ? 2 * w->sf_cap : 4096;
            w->sf = realloc(w->sf, (size_t)w->sf_cap * sizeof(nfill *));
        }
        w->sf[cnt++] = f;
    }
    g->n_fills = cnt;
    g->fills = arena_alloc(&w->ar, cnt * sizeof(nfill *));
    copy_fill(g->fills, w->sf, cnt);
    const int32_t level = g->pfill ? g->pfill->level + 1 : 0;
    if (cnt <= 16) { /* fills of one gap are disjoint: starts are distinct */
        for (int i = 1; i < cnt; ++i) {
            nfill *v = g->fills[i];
            int j = i - 1;
            while (j >= 0 && g->fills[j]->start > v->start) {
                g->fills[j + 1] = g->fills[j];
                --j;
            }
            g->fills[j + 1] = v;
        }
    } else {
        qsort(g->fills, g->n_fills, sizeof(nfill *), cmp_fill);
    }
    for (int i = 0; i < cnt; ++i) {
        g->fills[i]->pgap = g;
        g->fills[i]->pidx = i;
        g->fills[i]->level = level;
    }
}

static void finish_gap(fin_ctx *x, ngap *g) {
    sort_gap_fills(x->w, g);
    for (int i = 0; i < g->n_fills; ++i)
        finish_fill(x, g->fills[i]);
}

/* ------------------------------------------------------------ API */
/* Workers' pools are released in parallel: unmapping a C5 net is ~0.2 s of
 * page-table teardown on one core. */
static void *free_worker(void *arg) {
    gac_net *n = arg;
    for (;;) {
        int i = atomic_fetch_add(&n->free_next, 1);
        if (i >= n->n_w)
            return NULL;
        nwork *w = &n->w[i];
        arena_free(&w->ar);
        free(w->lf);
        free(w->in);
        free(w->q);
        free(w->it);
        free(w->cmb);
        free(w->rs);
        free(w->re);
        free(w->ros);
        free(w->roe);
        free(w->ro);
        free(w->sf);
    }
}

void gac_net_free(gac_net *n) {
    if (!n)
        return;
    if (n->w) {
        if (g_free_madv < 0) {
            const char *e = getenv("GAC_FREE_MADV");
            g_free_madv = !(e && *e == '0');
        }
        const char *ft = getenv("GAC_FREE_THREADS");
        const int t = ft && atoi(ft) > 0 ? atoi(ft) : 16;
        atomic_store(&n->free_next, 0);
        gac_run_threads(n->n_w < t ? n->n_w : t, free_worker, n);
    }
    free(n->w);
    free(n->chroms[0]);
    free(n->chroms[1]);
    free(n->order[0]);
    free(n->order[1]);
    free(n->pord[0]);
    free(n->pord[1]);
    pthread_mutex_destroy(&n->pord_mu);
    free(n->top[0]);
    free(n->top[1]);
    free(n->nlen[0]);
    free(n->nlen[1]);
    free(n->chain_ali);
    free(n);
}

/* The space index (≈570 MB at C5) and the netting scratch, released on a
 * detached thread once the nets are built, while they are written
 * (GAC_EARLY_FREE=0: by gac_net_free, with the arenas): pages dropped by
 * madvise, then the blocks freed.  C5 chainNet -rescore, alternating on one
 * box: 1652 -> 1615 ms median (`profiles/r05ef/`). */
typedef struct space_drop {
    void *p[16 * 64];
    size_t len[16 * 64];
    int n;
} space_drop;

static void *space_drop_thread(void *arg) {
    space_drop *D = arg;
    const uintptr_t pg = 4096;
    for (int k = 0; k < D->n; ++k) {
        const uintptr_t a = ((uintptr_t)D->p[k] + pg - 1) & ~(pg - 1);
        const uintptr_t b = ((uintptr_t)D->p[k] + D->len[k]) & ~(pg - 1);
        if (b > a)
            madvise((void *)a, b - a, MADV_DONTNEED);
        free(D->p[k]);
    }
    free(D);
    return NULL;
}

static void space_release(gac_net *n) {
    const char *e = getenv("GAC_EARLY_FREE");
    if ((e && *e == '0') || n->n_w > 64)
        return;
    space_drop *D = calloc(1, sizeof(space_drop));
    if (!D)
        return;
#define SDROP(ptr, bytes)                 \
    do {                                  \
        if (ptr) {                        \
            D->p[D->n] = (ptr);           \
            D->len[D->n++] = (bytes);     \
            (ptr) = NULL;                 \
        }                                 \
    } while (0)
    for (int i = 0; i < n->n_w; ++i) {
        nwork *w = &n->w[i];
        SDROP(w->lf, (size_t)w->lf_cap * sizeof(sleaf));
        SDROP(w->in, (size_t)w->in_cap * sizeof(snode));
        SDROP(w->q, (size_t)w->q_cap * sizeof(sitem));
        SDROP(w->it, (size_t)w->it_cap * sizeof(sitem));
        SDROP(w->cmb, (size_t)w->cmb_cap * sizeof(sitem));
        SDROP(w->sf, (size_t)w->sf_cap * sizeof(nfill *));
        w->lf_cap = w->in_cap = 0;
        w->q_cap = w->it_cap = w->cmb_cap = w->sf_cap = 0;
    }
#undef SDROP
    pthread_t th;
    pthread_attr_t at;
    pthread_attr_init(&at);
    pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
    if (pthread_create(&th, &at, space_drop_thread, D) != 0)
        space_drop_thread(D);
    pthread_attr_destroy(&at);
}

/* finishNet in three parallel phases:
 * (A) per chromosome side: the root gap's fills sorted, then the top of the
 *     fill tree (fills of levels 0 and 1, their gaps' fills sorted) walked in
 *     pre-order into a skeleton: FILL items, and GAP items standing for the
 *     whole subtree under a gap of a level-1 fill;
 * (B) the GAP subtrees (independent), in chunks over all threads: sorted
 *     into per-chunk pre-order lists (one long chain's fill can hold most of
 *     a chromosome, so its subtrees are the unit, not the top-level fills);
 * the pre-order index is the skeletons with the subtree lists spliced in;
 * (C) the other-side ranges of every fill, in balanced chunks. */
#define SKEL_DEPTH 0 /* fills of levels 0..SKEL_DEPTH are skeleton FILL items */

typedef struct sk_item {
    nfill *f;    /* a fill in the skeleton, or */
    ngap *g;     /* a gap whose subtree a phase-B chunk orders */
    int64_t cnt; /* (GAP) fills in that subtree */
} sk_item;

typedef struct skel {
    sk_item *it;
    int64_t n, cap;
} skel;

static void sk_push(skel *k, nfill *f, ngap *g) {
    if (k->n == k->cap) {
        k->cap = k->cap ? k->cap * 2 : 256;
        k->it = realloc(k->it, (size_t)k->cap * sizeof(sk_item));
    }
    k->it[k->n++] = (sk_item){f, g, 0};
}

/* finish_fill's pre-order walk down to SKEL_DEPTH */
static void skel_fill(nwork *w, skel *k, nfill *f) {
    sk_push(k, f, NULL);
    for (int i = 0; i < f->n_gaps; ++i) {
        f->gaps[i]->pfill = f;
        f->gaps[i]->pidx = i;
    }
    for (int i = 0; i < f->n_gaps; ++i) {
        ngap *g = f->gaps[i];
        if (f->level < SKEL_DEPTH) {
            sort_gap_fills(w, g);
            for (int j = 0; j < g->n_fills; ++j)
                skel_fill(w, k, g->fills[j]);
        } else if (g->fill_head) {
            sk_push(k, NULL, g);
        } else {
            g->n_fills = 0;
            g->fills = NULL;
        }
    }
}

/* one span of the pre-order index: cnt fills from src, placed at pos */
typedef struct ispan {
    nfill **src;
    int64_t pos, cnt;
    int side;
} ispan;

typedef struct splice_job {
    gac_net *n;
    ispan *sp;
    int64_t nspan;
    _Atomic int64_t next;
} splice_job;

static void *splice_thread(void *arg) {
    splice_job *J = arg;
    for (;;) {
        const int64_t a = atomic_fetch_add(&J->next, 4096);
        if (a >= J->nspan)
            return NULL;
        const int64_t b = a + 4096 < J->nspan ? a + 4096 : J->nspan;
        for (int64_t i = a; i < b; ++i) {
            const ispan *s = &J->sp[i];
            nfill **out = J->n->order[s->side] + s->pos;
            for (int64_t j = 0; j < s->cnt; ++j) {
                nfill *f = s->src[j];
                f->ord = s->pos + j;
                out[j] = f;
            }
        }
    }
}

typedef struct fin_job {
    gac_net *n;
    int phase;
    skel *sk;          /* [n_chroms[T] + n_chroms[Q]]: T chromosomes, then Q */
    sk_item **gi;      /* every GAP item, output order */
    int64_t n_gi, per; /* phase B chunk = per consecutive GAP items */
    fin_ctx *x;        /* [chunks] */
    int64_t ntask;
    _Atomic int64_t next;
    _Atomic int wid;
} fin_job;

static void *fin_thread(void *arg) {
    fin_job *F = arg;
    gac_net *n = F->n;
    nwork *w = &n->w[atomic_fetch_add(&F->wid, 1)];
    if (F->phase == 0) {
        const int64_t nc = n->n_chroms[GAC_T] + (int64_t)n->n_chroms[GAC_Q];
        for (;;) {
            const int64_t k = atomic_fetch_add(&F->next, 1);
            if (k >= nc)
                break;
            const int side = k < n->n_chroms[GAC_T] ? GAC_T : GAC_Q;
            nchrom *c = &n->chroms[side][side == GAC_T ? k : k - n->n_chroms[GAC_T]];
            if (!c->root)
                continue;
            sort_gap_fills(w, c->root);
            for (int j = 0; j < c->root->n_fills; ++j)
                skel_fill(w, &F->sk[k], c->root->fills[j]);
        }
        return NULL;
    }
    for (;;) {
        const int64_t k = atomic_fetch_add(&F->next, 1);
        if (k >= F->ntask)
            break;
        fin_ctx *x = &F->x[k];
        x->n = n;
        x->w = w;
        const int64_t a = k * F->per, b = a + F->per < F->n_gi ? a + F->per : F->n_gi;
        for (int64_t i = a; i < b; ++i) {
            const int64_t before = x->n_ord;
            finish_gap(x, F->gi[i]->g);
            F->gi[i]->cnt = x->n_ord - before;
        }
    }
    return NULL;
}

typedef struct net_task {
    int side;
    int32_t chrom;
    const int64_t *chains;
    int64_t n;
} net_task;

static int net_task_cmp(const void *a, const void *b) {
    const net_task *x = a, *y = b;
    if (x->n != y->n)
        return x->n > y->n ? -1 : 1;
    if (x->side != y->side)
        return x->side - y->side;
    return (x->chrom > y->chrom) - (x->chrom < y->chrom);
}

/* add chain c to side `side` of its sequence, whose space index is ch;
 * [A, B): the region ch covers (INT32_MIN/MAX: the whole sequence) */
static void add_chain(const gac_net *net, nwork *w, int side, int64_t c, nchrom *ch, int A, int B) {
    if (side == GAC_T)
        add_chain_t(net, w, c, ch, A, B);
    else
        add_chain_q(net, w, c, ch, A, B);
}

/* a chain's range on one side (+ strand coordinates) */
static void chain_span(const gac_net *net, int side, int64_t c, int *s, int *e) {
    const gac_net_input *in = &net->in;
    if (side == GAC_T) {
        *s = in->t_start[c];
        *e = in->t_end[c];
    } else if (in->q_strand[c]) {
        const int qsize = in->q_sizes[in->q_seq[c]];
        *s = qsize - in->q_end[c];
        *e = qsize - in->q_start[c];
    } else {
        *s = in->q_start[c];
        *e = in->q_end[c];
    }
}

/* ---- one chromosome side netted by many threads ----
 * The open spaces of a side are disjoint, and every later space lies inside
 * a current one (a filled space is replaced by its remnants and the chain's
 * gaps inside it).  So once no current space contains a point P strictly
 * inside it, no future space will: the chromosome splits at such points into
 * regions whose space sets evolve independently.  A chain only acts on the
 * spaces its range overlaps, space by space (innerBounds, fillSpace and the
 * remnant/gap tests see one space and the chain's own blocks), so netting
 * every region's spaces with the chains overlapping that region, each region
 * in score order, makes exactly the fills and spaces of the sequential
 * chainNet loop (chainNet.c:557-679); fills only meet again in their parent
 * gaps' lists, which finishNet sorts by start.
 *
 * net_regions: the first chains go through sequentially (they are the long,
 * high-scoring ones that cut the chromosome up), the region cuts are then
 * placed at space ends near evenly spaced quantiles of the remaining chains'
 * work, and the regions become tasks for every thread. */
typedef struct region {
    nchrom ch;          /* its own space index (built by the worker that nets it) */
    const sitem *sp;    /* its spaces, in order */
    int64_t n_sp;
    int64_t *chains;    /* remaining chains overlapping it, in order */
    int64_t n_chains;
    int64_t work;
    int side;
    int a, b;           /* [a, b): its part of the sequence */
} region;

typedef struct big_net {
    net_task *t;
    /* per chain of the task, in its order: span on this side and block
     * count, gathered once (the chains of one side lie all over the input's
     * arrays; the cut placement passes over them several times) */
    int32_t *ss, *se;
    int64_t *nbk;
    double t_start, t_gather, t_add, t_cut, t_reg; /* (GAC_TIMING laps of the prefix) */
    int64_t m;          /* chains netted sequentially first */
    sitem *spaces;      /* all spaces after the prefix */
    int64_t *lists;     /* region chain lists, back to back */
    region *reg;
    int32_t n_reg;
} big_net;

/* bulk-load sorted spaces into an empty index of c in w's pools */
static void sp_bulk(nwork *w, nchrom *c, const sitem *it, int64_t n) {
    if (n == 0) {
        c->sroot = sp_new_leaf(w);
        c->height = 0;
        return;
    }
    const int64_t nl = (n + SP_FILL - 1) / SP_FILL;
    int32_t *lvl = malloc((size_t)nl * 4);
    int64_t *key = malloc((size_t)nl * 8);
    int32_t prev = -1;
    for (int64_t j = 0; j < nl; ++j) {
        const int64_t lo = n * j / nl, hi = n * (j + 1) / nl;
        const int32_t l = sp_new_leaf(w);
        sleaf *L = &w->lf[l];
        for (int64_t k = lo; k < hi; ++k) {
            L->start[k - lo] = it[k].start;
            L->end[k - lo] = it[k].end;
            L->gap[k - lo] = it[k].gap;
        }
        L->n = (int32_t)(hi - lo);
        L->prev = prev;
        if (prev >= 0)
            w->lf[prev].next = l;
        prev = l;
        lvl[j] = l;
        key[j] = spkey(it[lo].start, it[lo].end);
    }
    int64_t cnt = nl;
    int h = 0;
    while (cnt > 1) {
        const int64_t np = (cnt + SP_FILL - 1) / SP_FILL;
        for (int64_t j = 0; j < np; ++j) {
            const int64_t lo = cnt * j / np, hi = cnt * (j + 1) / np;
            const int32_t x = sp_new_inner(w);
            snode *s = &w->in[x];
            for (int64_t k = lo; k < hi; ++k) {
                s->child[k - lo] = lvl[k];
                s->key[k - lo] = k == lo ? 0 : key[k];
            }
            s->n = (int32_t)(hi - lo);
            lvl[j] = x;
            key[j] = key[lo];
        }
        cnt = np;
        ++h;
    }
    c->sroot = lvl[0];
    c->height = h;
    free(lvl);
    free(key);
}

/* every space of c in order (leaf chain from the leftmost leaf) */
static sitem *sp_all(const nwork *w, const nchrom *c, int64_t *pn) {
    int32_t l = sp_descend(w, c, INT64_MIN, NULL, NULL);
    int64_t n = 0, cap = 1024;
    sitem *out = malloc((size_t)cap * sizeof(sitem));
    for (; l >= 0; l = w->lf[l].next) {
        const sleaf *L = &w->lf[l];
        for (int i = 0; i < L->n; ++i) {
            if (n == cap) {
                cap *= 2;
                out = realloc(out, (size_t)cap * sizeof(sitem));
            }
            out[n++] = (sitem){L->start[i], L->end[i], L->gap[i]};
        }
    }
    *pn = n;
    return out;
}

static int64_t upper_bound32(const int32_t *a, int64_t n, int32_t v) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (a[mid] <= v)
            lo = mid + 1;
        else
            hi = mid;
    }
    return lo;
}

/* work of a chain (span [cs, ce), nb blocks) inside [a, b): a region
 * builds the block slice there and scans the spaces its blocks reach */
static int64_t chain_work_in(int cs, int ce, int64_t nb, int a, int b) {
    const int64_t lo = cs > a ? cs : a, hi = ce < b ? ce : b;
    if (hi <= lo || ce <= cs)
        return 8;
    return 8 + nb * (hi - lo) / (ce - cs);
}

/* Region cuts for the chains after the first B->m: up to want-1 cut points
 * near equal quantiles of their work along the sequence, each moved to the
 * nearer end of the space holding it (no space may straddle a cut).  Returns
 * the region count; *pmax / *ptot = the largest region's / all work. */
static int32_t place_cuts(const gac_net *net, const big_net *B, const sitem *sp, int64_t nsp,
                          int32_t want, int size, int32_t *cuts, int64_t *pmax, int64_t *ptot) {
    const net_task *t = B->t;
    const int64_t rest = t->n - B->m;
    /* work density: each chain's blocks spread evenly over its span, on a
     * grid of 4096 bins */
    enum { NB = 4096 };
    int64_t *bin = calloc(NB + 1, 8), *dif = calloc(NB + 1, 8), tot = 0;
    const double scale = (double)NB / (size > 0 ? size : 1);
    for (int64_t i = 0; i < rest; ++i) { /* (spread as a difference array) */
        const int cs = B->ss[B->m + i], ce = B->se[B->m + i];
        const int64_t w = 8 + B->nbk[B->m + i];
        int b0 = (int)(cs * scale), b1 = (int)((ce > cs ? ce - 1 : cs) * scale);
        b0 = b0 < 0 ? 0 : (b0 >= NB ? NB - 1 : b0);
        b1 = b1 < b0 ? b0 : (b1 >= NB ? NB - 1 : b1);
        const int64_t per = w / (b1 - b0 + 1);
        dif[b0] += per;
        dif[b1 + 1] -= per;
        bin[b0] += w - per * (b1 - b0 + 1);
        tot += w;
    }
    {
        int64_t run = 0;
        for (int k = 0; k < NB; ++k) {
            run += dif[k];
            bin[k] += run;
        }
    }
    free(dif);
    int32_t nc = 0;
    int64_t acc = 0;
    int k = 0;
    for (int32_t j = 1; j < want && tot > 0; ++j) {
        const int64_t target = tot * j / want;
        while (k < NB && acc + bin[k] <= target)
            acc += bin[k++];
        if (k >= NB)
            break;
        int32_t x = (int32_t)((double)k / scale);
        int64_t lo = 0, hi = nsp; /* last space with start <= x */
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (sp[mid].start <= x)
                lo = mid + 1;
            else
                hi = mid;
        }
        if (lo > 0) {
            const sitem *S = &sp[lo - 1];
            if (S->start < x && x < S->end)
                x = (x - S->start <= S->end - x) ? S->start : S->end;
        }
        if (x <= 0 || x >= size || (nc && x <= cuts[nc - 1]))
            continue;
        cuts[nc++] = x;
    }
    free(bin);
    /* region work */
    int64_t *rw = calloc((size_t)nc + 1, 8), mx = 0;
    for (int64_t i = 0; i < rest; ++i) {
        const int cs = B->ss[B->m + i], ce = B->se[B->m + i];
        const int64_t a = upper_bound32(cuts, nc, cs), b = upper_bound32(cuts, nc, ce > cs ? ce - 1 : cs);
        for (int64_t r = a; r <= b; ++r)
            rw[r] += chain_work_in(cs, ce, B->nbk[B->m + i], r ? cuts[r - 1] : 0,
                                   r < nc ? cuts[r] : size);
    }
    for (int32_t r = 0; r <= nc; ++r)
        mx = rw[r] > mx ? rw[r] : mx;
    free(rw);
    *pmax = mx;
    *ptot = tot;
    return nc + 1;
}

static double mono_s(void);

/* thread 0: the sequential prefix of a big side and its regions */
static void big_prefix(gac_net *n, nwork *w, big_net *B, int nthreads) {
    net_task *t = B->t;
    nchrom *c = &n->chroms[t->side][t->chrom];
    c->root = gap_new(w, 0, c->size, 0, 0);
    c->root->pidx = t->chrom;
    sp_init(w, c, 0, c->size, c->root);
    const int32_t want = 4 * nthreads;
    int32_t *cuts = malloc((size_t)want * 4);
    B->t_start = mono_s();
    B->ss = malloc((size_t)(t->n ? t->n : 1) * 4);
    B->se = malloc((size_t)(t->n ? t->n : 1) * 4);
    B->nbk = malloc((size_t)(t->n ? t->n : 1) * 8);
    for (int64_t i = 0; i < t->n; ++i) {
        const int64_t c = t->chains[i];
        if (i + 8 < t->n) {
            const int64_t d = t->chains[i + 8];
            __builtin_prefetch(&n->in.blk_off[d]);
            __builtin_prefetch(t->side == GAC_T ? &n->in.t_start[d] : &n->in.q_start[d]);
        }
        int cs, ce;
        chain_span(n, t->side, c, &cs, &ce);
        B->ss[i] = cs;
        B->se[i] = ce;
        B->nbk[i] = n->in.blk_off[c + 1] - n->in.blk_off[c];
    }
    /* the prefix doubles from 8 chains until the regions balance: the
     * first chains leave one space over everything they did not reach */
    int64_t m = t->n < 8 ? t->n : 8, done = 0;
    sitem *sp = NULL;
    int64_t nsp = 0;
    int32_t nreg = 1;
    double t_add = 0, t_cut = 0, t0 = mono_s();
    const double t_gather = t0 - B->t_start;
    for (;;) {
        double ta = mono_s();
        for (; done < m; ++done)
            add_chain(n, w, t->side, t->chains[done], c, INT32_MIN, INT32_MAX);
        double tb = mono_s();
        t_add += tb - ta;
        B->m = m;
        free(sp);
        sp = sp_all(w, c, &nsp);
        int64_t mx, tot;
        nreg = place_cuts(n, B, sp, nsp, want, c->size, cuts, &mx, &tot);
        t_cut += mono_s() - tb;
        /* good enough: the largest region at most ~1/threads of the rest */
        if (m >= t->n || mx * nthreads <= tot * 5 / 4 || m >= t->n / 4)
            break;
        m = m * 2 < t->n ? m * 2 : t->n;
    }
    /* regions: spaces and chain lists */
    B->n_reg = nreg;
    B->reg = calloc((size_t)nreg, sizeof(region));
    B->spaces = sp;
    int64_t k = 0;
    for (int32_t r = 0; r < nreg; ++r) {
        region *R = &B->reg[r];
        R->side = t->side;
        R->ch = *c;
        R->a = r ? cuts[r - 1] : INT32_MIN;
        R->b = r < nreg - 1 ? cuts[r] : INT32_MAX;
        R->sp = sp + k;
        while (k < nsp && (r == nreg - 1 || sp[k].start < cuts[r]))
            ++k;
        R->n_sp = sp + k - R->sp;
    }
    const int64_t rest = t->n - m;
    int64_t *cnt = calloc((size_t)nreg + 1, 8);
    int32_t *ra = malloc((size_t)(rest ? rest : 1) * 4), *rb = malloc((size_t)(rest ? rest : 1) * 4);
    for (int64_t i = 0; i < rest; ++i) {
        const int cs = B->ss[m + i], ce = B->se[m + i];
        ra[i] = (int32_t)upper_bound32(cuts, nreg - 1, cs);
        rb[i] = (int32_t)upper_bound32(cuts, nreg - 1, ce > cs ? ce - 1 : cs);
        for (int32_t r = ra[i]; r <= rb[i]; ++r) {
            ++cnt[r];
            B->reg[r].work += chain_work_in(cs, ce, B->nbk[m + i], r ? cuts[r - 1] : 0,
                                            r < nreg - 1 ? cuts[r] : c->size);
        }
    }
    int64_t tot = 0;
    for (int32_t r = 0; r < nreg; ++r)
        tot += cnt[r];
    B->lists = malloc((size_t)(tot ? tot : 1) * 8);
    tot = 0;
    for (int32_t r = 0; r < nreg; ++r) {
        B->reg[r].chains = B->lists + tot;
        tot += cnt[r];
    }
    for (int64_t i = 0; i < rest; ++i)
        for (int32_t r = ra[i]; r <= rb[i]; ++r)
            B->reg[r].chains[B->reg[r].n_chains++] = t->chains[m + i];
    free(cnt);
    free(ra);
    free(rb);
    free(cuts);
    B->t_gather = t_gather;
    B->t_add = t_add;
    B->t_cut = t_cut;
    B->t_reg = mono_s() - t0 - t_add - t_cut;
    free(B->ss);
    free(B->se);
    free(B->nbk);
    B->ss = B->se = NULL;
    B->nbk = NULL;
}

static void net_region(gac_net *n, nwork *w, region *R) {
    sp_bulk(w, &R->ch, R->sp, R->n_sp);
    for (int64_t i = 0; i < R->n_chains; ++i)
        add_chain(n, w, R->side, R->chains[i], &R->ch, R->a, R->b);
}

typedef struct net_job {
    gac_net *n;
    net_task *task;     /* small sides, largest first */
    int64_t ntask;
    big_net *big;       /* big sides (split into regions) */
    int32_t nbig;
    region **rq;        /* the regions, each big side's largest work first, published per side */
    int64_t nrq;        /* (capacity; the published count is rpub) */
    _Atomic int64_t next, rnext, rpub;
    pthread_mutex_t rmu; /* (publishing a side's regions) */
    _Atomic int ready;  /* every prefix is done and every region published */
    _Atomic int wid;
    _Atomic int32_t bnext, bdone; /* big sides whose prefix was taken / is done */
    int nthreads;
    double t0;          /* start of the threads */
    double prefix_s;    /* from the start until every prefix was done */
} net_job;

static int region_cmp(const void *a, const void *b) {
    const region *x = *(region *const *)a, *y = *(region *const *)b;
    return (x->work < y->work) - (x->work > y->work);
}

static void net_small(gac_net *n, nwork *w, const net_task *t) {
    nchrom *c = &n->chroms[t->side][t->chrom];
    /* makeChroms (chainNet.c:328-354): one gap = one space over the whole
     * sequence */
    c->root = gap_new(w, 0, c->size, 0, 0);
    c->root->pidx = t->chrom;
    sp_init(w, c, 0, c->size, c->root);
    for (int64_t i = 0; i < t->n; ++i)
        add_chain(n, w, t->side, t->chains[i], c, INT32_MIN, INT32_MAX);
}

static double mono_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void *net_thread(void *arg) {
    net_job *J = arg;
    const int id = atomic_fetch_add(&J->wid, 1);
    nwork *w = &J->n->w[id];
    /* the big sides' sequential prefixes, one side per thread; the thread
     * finishing the last one publishes every region, largest work first */
    for (;;) {
        const int32_t b = atomic_fetch_add(&J->bnext, 1);
        if (b >= J->nbig)
            break;
        big_prefix(J->n, w, &J->big[b], J->nthreads);
        /* its regions, largest work first, published at once: the other
         * threads take them while the remaining prefixes run (round 4 waited
         * for every prefix; at -nranks=8 that wait was most of the netting) */
        big_net *B = &J->big[b];
        region **tmp = malloc((size_t)(B->n_reg ? B->n_reg : 1) * sizeof(region *));
        for (int32_t r = 0; r < B->n_reg; ++r)
            tmp[r] = &B->reg[r];
        qsort(tmp, (size_t)B->n_reg, sizeof(region *), region_cmp);
        pthread_mutex_lock(&J->rmu);
        const int64_t at = atomic_load(&J->rpub);
        memcpy(J->rq + at, tmp, (size_t)B->n_reg * sizeof(region *));
        atomic_store_explicit(&J->rpub, at + B->n_reg, memory_order_release);
        pthread_mutex_unlock(&J->rmu);
        free(tmp);
        if (atomic_fetch_add(&J->bdone, 1) + 1 < J->nbig)
            continue;
        J->prefix_s = mono_s() - J->t0;
        atomic_store_explicit(&J->ready, 1, memory_order_release);
    }
    for (;;) {
        int64_t k = atomic_load(&J->rnext);
        if (k < atomic_load_explicit(&J->rpub, memory_order_acquire)) {
            if (atomic_compare_exchange_weak(&J->rnext, &k, k + 1))
                net_region(J->n, w, J->rq[k]);
            continue;
        }
        const int64_t t = atomic_fetch_add(&J->next, 1);
        if (t < J->ntask) {
            net_small(J->n, w, &J->task[t]);
            continue;
        }
        if (atomic_load_explicit(&J->ready, memory_order_acquire) &&
            atomic_load(&J->rnext) >= atomic_load(&J->rpub))
            break;
        sched_yield();
    }
    return NULL;
}

typedef struct ca_job {
    const gac_net_input *in;
    int64_t *out;
    _Atomic int64_t next;
} ca_job;

static void *chain_ali_thread(void *arg) {
    ca_job *A = arg;
    for (;;) {
        const int64_t a = atomic_fetch_add(&A->next, 16384);
        if (a >= A->in->n_chains)
            return NULL;
        const int64_t b = a + 16384 < A->in->n_chains ? a + 16384 : A->in->n_chains;
        for (int64_t c = a; c < b; ++c) {
            int64_t t = 0;
            for (int64_t k = A->in->blk_off[c]; k < A->in->blk_off[c + 1]; ++k)
                t += A->in->blk_size[k];
            A->out[c] = t;
        }
    }
}

int gac_net_build(const gac_net_input *in, const gac_net_opts *opt, gac_net **out) {
    return gac_net_build_sides(in, opt, (1 << GAC_T) | (1 << GAC_Q), out);
}

static int net_build(const gac_net_input *in, const gac_net_opts *opt, int sides,
                     const uint8_t *t_keep, const uint8_t *q_keep, gac_net **out);

int gac_net_build_sides(const gac_net_input *in, const gac_net_opts *opt, int sides,
                        gac_net **out) {
    gac_clear_error();
    if (!in || !opt || !out)
        return gac_fail(GAC_E_ARG, "gac_net_build: NULL argument");
    if (sides <= 0 || (sides & ~((1 << GAC_T) | (1 << GAC_Q))))
        return gac_fail(GAC_E_ARG, "gac_net_build_sides: bad side mask %d", sides);
    return net_build(in, opt, sides, NULL, NULL, out);
}

int gac_net_build_subset(const gac_net_input *in, const gac_net_opts *opt, const uint8_t *t_keep,
                         const uint8_t *q_keep, gac_net **out) {
    gac_clear_error();
    if (!in || !opt || !out || !t_keep || !q_keep)
        return gac_fail(GAC_E_ARG, "gac_net_build_subset: NULL argument");
    return net_build(in, opt, (1 << GAC_T) | (1 << GAC_Q), t_keep, q_keep, out);
}

static int net_build(const gac_net_input *in, const gac_net_opts *opt, int sides,
                     const uint8_t *t_keep, const uint8_t *q_keep, gac_net **out) {
    *out = NULL;
    gac_net *n = calloc(1, sizeof(*n));
    if (n)
        pthread_mutex_init(&n->pord_mu, NULL);
    n->in = *in;
    n->opt = *opt;
    n->sides = sides;
    n->n_w = gac_host_threads();
    n->w = calloc((size_t)n->n_w, sizeof(nwork));
    for (int k = 0; k < n->n_w; ++k) {
        n->w[k].lf_free = -1;
        n->w[k].in_free = -1;
    }
    /* chains to net: in order until the first below minScore (must be
     * sorted), haplotype queries skipped unless incl_hap */
    double last = -1;
    int64_t i;
    for (i = 0; i < in->n_chains; ++i) {
        const double sc = in->score[i];
        if (last >= 0 && sc > last) {
            gac_net_free(n);
            return gac_fail(GAC_E_FORMAT, "input must be sorted in order of score");
        }
        last = sc;
        if (sc < opt->min_score)
            break;
        if (in->t_seq[i] < 0 || in->t_seq[i] >= in->n_tseq || in->q_seq[i] < 0 ||
            in->q_seq[i] >= in->n_qseq) {
            gac_net_free(n);
            return gac_fail(GAC_E_ARG, "chain %lld: sequence index out of range", (long long)i);
        }
    }
    const int64_t nn = i;
    /* per (side, chromosome): its chains in order (counting sort) */
    int32_t nt = in->n_tseq, nq = in->n_qseq;
    int64_t *toff = calloc((size_t)nt + 1, 8), *qoff = calloc((size_t)nq + 1, 8);
    int64_t *tl = malloc((size_t)(nn ? nn : 1) * 8), *ql = malloc((size_t)(nn ? nn : 1) * 8);
    int64_t *tfill = malloc((size_t)(nt ? nt : 1) * 8), *qfill = malloc((size_t)(nq ? nq : 1) * 8);
    uint8_t *skip = calloc((size_t)(nq ? nq : 1), 1); /* haplotype queries, by sequence */
    for (int32_t k = 0; k < nq && !opt->incl_hap; ++k)
        skip[k] = (uint8_t)is_haplotype(in->q_names[k]);
    for (int64_t c = 0; c < nn; ++c) {
        if (skip[in->q_seq[c]])
            continue;
        ++toff[in->t_seq[c] + 1];
        ++qoff[in->q_seq[c] + 1];
    }
    for (int32_t k = 0; k < nt; ++k)
        toff[k + 1] += toff[k];
    for (int32_t k = 0; k < nq; ++k)
        qoff[k + 1] += qoff[k];
    memcpy(tfill, toff, (size_t)nt * 8);
    memcpy(qfill, qoff, (size_t)nq * 8);
    for (int64_t c = 0; c < nn; ++c) {
        if (skip[in->q_seq[c]])
            continue;
        tl[tfill[in->t_seq[c]]++] = c;
        ql[qfill[in->q_seq[c]]++] = c;
    }
    free(skip);
    for (int side = 0; side < 2; ++side) {
        int32_t cnt = side == GAC_T ? nt : nq;
        const char *const *names = side == GAC_T ? in->t_names : in->q_names;
        const int32_t *sizes = side == GAC_T ? in->t_sizes : in->q_sizes;
        n->n_chroms[side] = cnt;
        n->chroms[side] = calloc(cnt ? cnt : 1, sizeof(nchrom));
        for (int32_t k = 0; k < cnt; ++k) {
            nchrom *c = &n->chroms[side][k];
            c->name = names[k];
            c->size = sizes[k];
            c->sroot = -1;
        }
    }
    /* tasks, largest first; every task nets one chromosome of one side, the
     * big ones are split into regions (net_regions) */
    net_job J;
    memset(&J, 0, sizeof(J));
    J.n = n;
    J.task = malloc((size_t)(nt + nq ? nt + nq : 1) * sizeof(net_task));
    J.ntask = 0;
    J.nthreads = n->n_w;
    if (sides & (1 << GAC_T))
        for (int32_t k = 0; k < nt; ++k)
            if (!t_keep || t_keep[k])
                J.task[J.ntask++] = (net_task){GAC_T, k, tl + toff[k], toff[k + 1] - toff[k]};
    if (sides & (1 << GAC_Q))
        for (int32_t k = 0; k < nq; ++k)
            if (!q_keep || q_keep[k])
                J.task[J.ntask++] = (net_task){GAC_Q, k, ql + qoff[k], qoff[k + 1] - qoff[k]};
    qsort(J.task, (size_t)J.ntask, sizeof(net_task), net_task_cmp);
    /* big sides: more than a thread's share of all chains (and enough
     * chains to be worth the split); the rest stay whole tasks */
    int64_t all = 0;
    for (int64_t k = 0; k < J.ntask; ++k)
        all += J.task[k].n;
    J.big = calloc((size_t)(J.ntask ? J.ntask : 1), sizeof(big_net));
    const char *split_env = getenv("GAC_NET_SPLIT");
    const int split = n->n_w > 1 && !(split_env && split_env[0] == '0');
    while (split && J.nbig < J.ntask && J.task[J.nbig].n >= 8192 &&
           J.task[J.nbig].n * 2 * n->n_w >= all) {
        J.big[J.nbig].t = &J.task[J.nbig];
        ++J.nbig;
    }
    net_task *small = J.task + J.nbig;
    const int64_t nsmall = J.ntask - J.nbig;
    net_job J2 = J; /* (the small-task view) */
    J2.task = small;
    J2.ntask = nsmall;
    atomic_init(&J2.next, 0);
    atomic_init(&J2.rnext, 0);
    atomic_init(&J2.rpub, 0);
    pthread_mutex_init(&J2.rmu, NULL);
    atomic_init(&J2.ready, J.nbig == 0);
    atomic_init(&J2.wid, 0);
    atomic_init(&J2.bnext, 0);
    atomic_init(&J2.bdone, 0);
    J2.nrq = (int64_t)J.nbig * 4 * n->n_w; /* (place_cuts makes at most 4 x threads regions) */
    J2.rq = malloc((size_t)(J2.nrq ? J2.nrq : 1) * sizeof(region *));
    struct timespec t_add0, t_add1;
    clock_gettime(CLOCK_MONOTONIC, &t_add0);
    J2.t0 = mono_s();
    const int64_t units = nsmall + (J.nbig ? n->n_w : 0);
    gac_run_threads(n->n_w < units ? n->n_w : (units ? (int)units : 1), net_thread, &J2);
    clock_gettime(CLOCK_MONOTONIC, &t_add1);
    if (getenv("GAC_TIMING")) {
        fprintf(stderr, "[gac_net_build] addChainT/Q %.3f s (%d threads, largest task %lld chains; sequential prefixes done after %.3f s)\n",
                (t_add1.tv_sec - t_add0.tv_sec) + 1e-9 * (t_add1.tv_nsec - t_add0.tv_nsec),
                n->n_w, J.ntask ? (long long)J.task[0].n : 0LL, J2.prefix_s);
        for (int32_t b = 0; b < J.nbig; ++b) {
            int64_t mx = 0;
            for (int32_t r = 0; r < J.big[b].n_reg; ++r)
                mx = J.big[b].reg[r].work > mx ? J.big[b].reg[r].work : mx;
            fprintf(stderr, "[gac_net_build] side %d seq %d: %lld chains, %lld sequential, %d regions (largest work %lld); prefix: gather %.3f, chains %.3f, cuts %.3f, regions %.3f s\n",
                    J.big[b].t->side, J.big[b].t->chrom, (long long)J.big[b].t->n,
                    (long long)J.big[b].m, J.big[b].n_reg, (long long)mx, J.big[b].t_gather,
                    J.big[b].t_add, J.big[b].t_cut, J.big[b].t_reg);
        }
    }
    for (int32_t b = 0; b < J.nbig; ++b) {
        free(J.big[b].spaces);
        free(J.big[b].lists);
        free(J.big[b].reg);
    }
    free(J.big);
    free(J2.rq);
    pthread_mutex_destroy(&J2.rmu);
    free(J.task);
    free(toff);
    free(qoff);
    free(tl);
    free(ql);
    free(tfill);
    free(qfill);
    n->n_netted = i;
    struct timespec t_fin0, t_fin1;
    clock_gettime(CLOCK_MONOTONIC, &t_fin0);
    /* finishNet: chromosomes in parallel, then the pre-order index per side
     * in chromosome order */
    {
        fin_job F;
        memset(&F, 0, sizeof(F));
        F.n = n;
        const int64_t nc = n->n_chroms[GAC_T] + (int64_t)n->n_chroms[GAC_Q];
        F.sk = calloc((size_t)(nc ? nc : 1), sizeof(skel));
        atomic_init(&F.next, 0);
        atomic_init(&F.wid, 0);
        gac_run_threads(n->n_w < nc ? n->n_w : (nc ? (int)nc : 1), fin_thread, &F);
        /* phase B: chunks of GAP items, in output order */
        for (int64_t k = 0; k < nc; ++k)
            for (int64_t i = 0; i < F.sk[k].n; ++i)
                F.n_gi += F.sk[k].it[i].g != NULL;
        F.gi = malloc((size_t)(F.n_gi ? F.n_gi : 1) * sizeof(sk_item *));
        F.n_gi = 0;
        for (int64_t k = 0; k < nc; ++k)
            for (int64_t i = 0; i < F.sk[k].n; ++i)
                if (F.sk[k].it[i].g)
                    F.gi[F.n_gi++] = &F.sk[k].it[i];
        F.per = F.n_gi / (16 * (int64_t)n->n_w) + 1;
        F.ntask = (F.n_gi + F.per - 1) / F.per;
        F.x = calloc((size_t)(F.ntask ? F.ntask : 1), sizeof(fin_ctx));
        struct timespec t_a;
        clock_gettime(CLOCK_MONOTONIC, &t_a);
        F.phase = 1;
        atomic_init(&F.next, 0);
        atomic_init(&F.wid, 0);
        gac_run_threads(n->n_w < F.ntask ? n->n_w : (F.ntask ? (int)F.ntask : 1), fin_thread, &F);
        struct timespec t_sp;
        clock_gettime(CLOCK_MONOTONIC, &t_sp);
        /* the pre-order index: skeletons with the subtree lists spliced in */
        int64_t tot[2] = {0, 0};
        for (int64_t k = 0; k < nc; ++k) {
            const int side = k < n->n_chroms[GAC_T] ? GAC_T : GAC_Q;
            for (int64_t i = 0; i < F.sk[k].n; ++i)
                tot[side] += F.sk[k].it[i].g ? F.sk[k].it[i].cnt : 1;
        }
        for (int side = 0; side < 2; ++side) {
            n->order[side] = malloc((size_t)(tot[side] ? tot[side] : 1) * sizeof(nfill *));
            n->n_order[side] = 0;
        }
        /* spans of the index in order (a FILL item: its fill; a GAP item:
         * its run of its chunk's list), placed by a serial pass over the
         * items, then copied -- and every fill's ord set -- on all threads */
        int64_t nspan = 0;
        for (int64_t k = 0; k < nc; ++k)
            nspan += F.sk[k].n;
        splice_job SJ = {n, malloc((size_t)(nspan ? nspan : 1) * sizeof(ispan)), nspan, 0};
        for (int side = 0; side < 2; ++side) {
            n->top[side] = malloc((size_t)(nspan ? nspan : 1) * sizeof(int64_t));
            n->n_top[side] = 0;
        }
        {
            int64_t gidx = 0, used = 0, m = 0; /* GAP item; fills taken from its chunk's list */
            for (int64_t k = 0; k < nc; ++k) {
                const int side = k < n->n_chroms[GAC_T] ? GAC_T : GAC_Q;
                for (int64_t i = 0; i < F.sk[k].n; ++i) {
                    sk_item *it = &F.sk[k].it[i];
                    if (!it->g) {
                        SJ.sp[m++] = (ispan){&it->f, n->n_order[side], 1, side};
                        if (it->f->level == 0)
                            n->top[side][n->n_top[side]++] = n->n_order[side];
                        ++n->n_order[side];
                        continue;
                    }
                    const fin_ctx *x = &F.x[gidx / F.per];
                    if (gidx % F.per == 0)
                        used = 0;
                    SJ.sp[m++] = (ispan){x->ord + used, n->n_order[side], it->cnt, side};
                    n->n_order[side] += it->cnt;
                    used += it->cnt;
                    ++gidx;
                }
            }
        }
        atomic_init(&SJ.next, 0);
        gac_run_threads(n->n_w, splice_thread, &SJ);
        free(SJ.sp);
        for (int64_t k = 0; k < nc; ++k)
            free(F.sk[k].it);
        for (int64_t k = 0; k < F.ntask; ++k)
            free(F.x[k].ord);
        free(F.sk);
        free(F.gi);
        /* (rCalcOtherFill ran as each fill was made: add_chain_side) */
        struct timespec t_b;
        clock_gettime(CLOCK_MONOTONIC, &t_b);
        if (getenv("GAC_TIMING"))
            fprintf(stderr, "[gac_net_build] finishNet skeletons %.3f s, subtrees %.3f s, index %.3f s (%lld gap subtrees in %lld chunks)\n",
                    (t_a.tv_sec - t_fin0.tv_sec) + 1e-9 * (t_a.tv_nsec - t_fin0.tv_nsec),
                    (t_sp.tv_sec - t_a.tv_sec) + 1e-9 * (t_sp.tv_nsec - t_a.tv_nsec),
                    (t_b.tv_sec - t_sp.tv_sec) + 1e-9 * (t_b.tv_nsec - t_sp.tv_nsec), (long long)F.n_gi,
                    (long long)F.ntask);
        free(F.x);
    }
    clock_gettime(CLOCK_MONOTONIC, &t_fin1);
    if (getenv("GAC_TIMING")) {
        size_t sp_bytes = 0, ar_bytes = 0;
        for (int i = 0; i < n->n_w; ++i) {
            sp_bytes += (size_t)n->w[i].lf_cap * sizeof(sleaf) + (size_t)n->w[i].in_cap * sizeof(snode);
            for (size_t k = 0; k < n->w[i].ar.n; ++k)
                ar_bytes += n->w[i].ar.sizes[k];
        }
        fprintf(stderr, "[gac_net_build] finishNet %.3f s (space index %.0f MB, fill/gap arenas %.0f MB)\n",
                (t_fin1.tv_sec - t_fin0.tv_sec) + 1e-9 * (t_fin1.tv_nsec - t_fin0.tv_nsec),
                sp_bytes / 1e6, ar_bytes / 1e6);
    }
    /* the space index is netting-only: released now, on a detached thread */
    space_release(n);
    for (int side = 0; side < 2; ++side) { /* (the writers' line-length check) */
        const int32_t ns = side == GAC_T ? in->n_tseq : in->n_qseq;
        const char *const *nm = side == GAC_T ? in->t_names : in->q_names;
        n->nlen[side] = malloc((size_t)(ns > 0 ? ns : 1) * sizeof(int32_t));
        for (int32_t k = 0; k < ns; ++k)
            n->nlen[side][k] = (int32_t)strlen(nm[k]);
    }
    /* aligned bases per chain (chainBaseCount), in parallel over chains */
    n->chain_ali = malloc((size_t)(in->n_chains ? in->n_chains : 1) * sizeof(int64_t));
    {
        ca_job A = {in, n->chain_ali, 0};
        atomic_init(&A.next, 0);
        gac_run_threads(gac_host_threads(), chain_ali_thread, &A);
    }
    *out = n;
    return GAC_OK;
}

int64_t gac_net_netted(const gac_net *n) { return n ? n->n_netted : -1; }

int64_t gac_net_fill_count(const gac_net *n, int side) {
    if (!n || (side != GAC_T && side != GAC_Q))
        return -1;
    return n->n_order[side];
}

static int full_size(const gac_net *n, int64_t c) { return (int)n->chain_ali[c]; }

/* visibility of each fill: reached by rOutputFill and passing its filters
 * given the score rule; for the T side with rescore the score filter always
 * passes (partial scores are >= 1, netted chains >= minScore = 0).
 * Fills in parallel (contiguous index runs), then one visibility pass in
 * pre-order over the parent links. */
typedef struct gf_job {
    const gac_net *n;
    int side;
    int32_t *chain, *start, *end, *ali;
    uint8_t *flags;
    int64_t per;
    _Atomic int64_t next;
    int32_t *wb0, *wn; /* gac_net_get_fill_windows */
    int64_t *po;       /* the parent positions being built (NULL: built) */
} gf_job;

static void *fills_thread(void *arg) {
    gf_job *J = arg;
    const gac_net *n = J->n;
    const int side = J->side;
    for (;;) {
        const int64_t a = atomic_fetch_add(&J->next, 1) * J->per;
        if (a >= n->n_order[side])
            break;
        const int64_t b = a + J->per < n->n_order[side] ? a + J->per : n->n_order[side];
        for (int64_t i = a; i < b; ++i) {
            const nfill *f = n->order[side][i];
            const int64_t c = f->chain;
            const int full = f->full;
            const int sz = full ? full_size(n, c) : f->ali;
            if (J->chain)
                J->chain[i] = (int32_t)c;
            if (J->start)
                J->start[i] = f->start;
            if (J->end)
                J->end[i] = f->end;
            if (J->ali)
                J->ali[i] = sz;
            if (J->flags)
                J->flags[i] = (uint8_t)(full ? 0 : 1);
            if (J->wb0)
                J->wb0[i] = f->wb0;
            if (J->wn)
                J->wn[i] = f->wn;
        }
    }
    return NULL;
}

static int64_t next_top_level(const gac_net *n, int side, int64_t i) {
    if (n->top[side]) { /* the first top-level position >= i */
        const int64_t *t = n->top[side];
        int64_t lo = 0, hi = n->n_top[side];
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (t[mid] < i)
                lo = mid + 1;
            else
                hi = mid;
        }
        return lo < n->n_top[side] ? t[lo] : n->n_order[side];
    }
    if (__atomic_load_n(&n->pord_ok[side], __ATOMIC_ACQUIRE)) {
        const int64_t *po = n->pord[side];
        while (i < n->n_order[side] && po[i] >= 0)
            ++i;
        return i;
    }
    while (i < n->n_order[side] && n->order[side][i]->pgap->pfill)
        ++i;
    return i;
}

static void *visible_thread(void *arg) {
    gf_job *J = arg;
    const gac_net *n = J->n;
    const int side = J->side;
    const int64_t nf = n->n_order[side];
    for (;;) {
        const int64_t r = atomic_fetch_add(&J->next, 1);
        if (r * J->per >= nf)
            break;
        const int64_t a = next_top_level(n, side, r * J->per);
        const int64_t b = next_top_level(n, side, (r + 1) * J->per < nf ? (r + 1) * J->per : nf);
        int64_t *po = J->po;
        for (int64_t i = a; i < b; ++i) {
            const nfill *pf = n->order[side][i]->pgap->pfill;
            if (po)
                po[i] = pf ? pf->ord : -1;
            const int sz = J->ali ? J->ali[i] : 0;
            if ((!pf || (J->flags[pf->ord] & 2)) && sz >= n->opt.min_fill)
                J->flags[i] |= 2;
        }
    }
    return NULL;
}

int gac_net_get_fills(const gac_net *n, int side, int32_t *chain, int32_t *start, int32_t *end,
                      int32_t *ali, uint8_t *flags) {
    if (!n || (side != GAC_T && side != GAC_Q))
        return gac_fail(GAC_E_ARG, "gac_net_get_fills: bad argument");
    if (!(n->sides & (1 << side)))
        return gac_fail(GAC_E_STATE, "gac_net_get_fills: side %d was not netted", side);
    const int nt = gac_host_threads();
    const int64_t nf = n->n_order[side];
    gf_job J = {n, side, chain, start, end, ali, flags, nf / (8 * (int64_t)nt) + 1, 0, NULL, NULL};
    atomic_init(&J.next, 0);
    const int64_t nrun = (nf + J.per - 1) / J.per;
    gac_mark("get_fills: fills");
    gac_run_threads(nt < nrun ? nt : (int)(nrun ? nrun : 1), fills_thread, &J);
    gac_mark("get_fills: visible");
    /* visibility: a fill is printed when its parent fill is and its own ali
     * >= min_fill -- one pass in pre-order (parents precede children), in
     * parallel over runs that start at top-level fills (whole subtrees) */
    if (flags) {
        /* (the parent positions are kept for the output's pass; the net is
         * const to callers, this is a cache: built once, under pord_mu, and
         * never written again -- a later pass gets po = NULL) */
        gac_net *nm = (gac_net *)n;
        pthread_mutex_lock(&nm->pord_mu);
        const int build = !__atomic_load_n(&nm->pord_ok[side], __ATOMIC_ACQUIRE);
        if (build && !nm->pord[side])
            nm->pord[side] = malloc((size_t)(nf ? nf : 1) * sizeof(int64_t));
        J.po = build ? nm->pord[side] : NULL;
        atomic_store(&J.next, 0);
        gac_run_threads(nt < nrun ? nt : (int)(nrun ? nrun : 1), visible_thread, &J);
        if (build)
            __atomic_store_n(&nm->pord_ok[side], 1, __ATOMIC_RELEASE);
        pthread_mutex_unlock(&nm->pord_mu);
    }
    gac_mark("get_fills: done");
    return GAC_OK;
}

int gac_net_get_fill_windows(const gac_net *n, int side, int32_t *first_block, int32_t *n_blocks) {
    if (!n || side != GAC_T)
        return gac_fail(GAC_E_ARG, "gac_net_get_fill_windows: target side only");
    if (!(n->sides & (1 << side)))
        return gac_fail(GAC_E_STATE, "gac_net_get_fill_windows: side %d was not netted", side);
    const int nt = gac_host_threads();
    const int64_t nf = n->n_order[side];
    gf_job J = {n, side, NULL, NULL, NULL, NULL, NULL, nf / (8 * (int64_t)nt) + 1, 0, first_block,
                n_blocks};
    atomic_init(&J.next, 0);
    const int64_t nrun = (nf + J.per - 1) / J.per;
    gac_run_threads(nt < nrun ? nt : (int)(nrun ? nrun : 1), fills_thread, &J);
    return GAC_OK;
}

/* gac_net_rescore_windows: per run of whole top-level subtrees (as the
 * visibility pass), one read of each fill -- its parent position, its
 * visibility and, when partial and printed, its record into the run's own
 * buffer -- then the runs' buffers placed by a prefix sum and copied. */
typedef struct rw_run {
    gac_window *w;
    int64_t *pos;
    int64_t n, cap;
} rw_run;

typedef struct rw_job {
    const gac_net *n;
    int side;
    uint8_t *vis;
    int64_t *po;
    int64_t per, nrun;
    rw_run *runs;
    gac_window *out;
    int64_t *opos, *off;
    _Atomic int64_t next;
    int phase;
} rw_job;

static void *rw_thread(void *arg) {
    rw_job *J = arg;
    const gac_net *n = J->n;
    const int side = J->side;
    const int64_t nf = n->n_order[side];
    for (;;) {
        const int64_t r = atomic_fetch_add(&J->next, 1);
        if (r >= J->nrun)
            break;
        rw_run *R = &J->runs[r];
        if (J->phase == 1) {
            if (R->n) {
                memcpy(J->out + J->off[r], R->w, (size_t)R->n * sizeof(gac_window));
                memcpy(J->opos + J->off[r], R->pos, (size_t)R->n * sizeof(int64_t));
            }
            free(R->w);
            free(R->pos);
            continue;
        }
        const int64_t a = next_top_level(n, side, r * J->per);
        const int64_t b = next_top_level(n, side, (r + 1) * J->per < nf ? (r + 1) * J->per : nf);
        for (int64_t i = a; i < b; ++i) {
            if (i + 16 < b)
                __builtin_prefetch(n->order[side][i + 16]);
            const nfill *f = n->order[side][i];
            const nfill *pf = f->pgap->pfill;
            if (J->po)
                J->po[i] = pf ? pf->ord : -1;
            const int sz = f->full ? full_size(n, f->chain) : f->ali;
            const uint8_t v = (!pf || J->vis[pf->ord]) && sz >= n->opt.min_fill;
            J->vis[i] = v;
            if (!v || f->full)
                continue;
            if (R->n == R->cap) {
                R->cap = R->cap ? 2 * R->cap : 4096;
                R->w = realloc(R->w, (size_t)R->cap * sizeof(gac_window));
                R->pos = realloc(R->pos, (size_t)R->cap * sizeof(int64_t));
            }
            R->w[R->n] = (gac_window){(int32_t)f->chain, f->start, f->end, f->wb0, f->wn};
            R->pos[R->n++] = i;
        }
    }
    return NULL;
}

int gac_net_rescore_windows(const gac_net *n, int side, gac_window **windows, int64_t **pos,
                            int64_t *count) {
    if (!n || side != GAC_T || !windows || !pos || !count)
        return gac_fail(GAC_E_ARG, "gac_net_rescore_windows: bad argument (target side only)");
    if (!(n->sides & (1 << side)))
        return gac_fail(GAC_E_STATE, "gac_net_rescore_windows: side %d was not netted", side);
    const int nt = gac_host_threads();
    const int64_t nf = n->n_order[side];
    gac_net *nm = (gac_net *)n; /* (the parent positions are a cache, as in get_fills) */
    pthread_mutex_lock(&nm->pord_mu);
    const int build = !__atomic_load_n(&nm->pord_ok[side], __ATOMIC_ACQUIRE);
    if (build && !nm->pord[side])
        nm->pord[side] = malloc((size_t)(nf ? nf : 1) * sizeof(int64_t));
    rw_job J;
    memset(&J, 0, sizeof(J));
    J.n = n;
    J.side = side;
    J.vis = malloc((size_t)(nf ? nf : 1));
    J.po = build ? nm->pord[side] : NULL;
    J.per = nf / (8 * (int64_t)nt) + 1;
    J.nrun = (nf + J.per - 1) / J.per;
    J.runs = calloc((size_t)(J.nrun ? J.nrun : 1), sizeof(rw_run));
    atomic_init(&J.next, 0);
    gac_run_threads(nt < J.nrun ? nt : (int)(J.nrun ? J.nrun : 1), rw_thread, &J);
    if (build)
        __atomic_store_n(&nm->pord_ok[side], 1, __ATOMIC_RELEASE);
    pthread_mutex_unlock(&nm->pord_mu);
    J.off = malloc((size_t)(J.nrun + 1) * sizeof(int64_t));
    J.off[0] = 0;
    for (int64_t r = 0; r < J.nrun; ++r)
        J.off[r + 1] = J.off[r] + J.runs[r].n;
    const int64_t m = J.off[J.nrun];
    J.out = malloc((size_t)(m ? m : 1) * sizeof(gac_window));
    J.opos = malloc((size_t)(m ? m : 1) * sizeof(int64_t));
    J.phase = 1;
    atomic_store(&J.next, 0);
    gac_run_threads(nt < J.nrun ? nt : (int)(J.nrun ? J.nrun : 1), rw_thread, &J);
    free(J.runs);
    free(J.off);
    free(J.vis);
    *windows = J.out;
    *pos = J.opos;
    *count = m;
    return GAC_OK;
}

/* ------------------------------------------------------------ output */
/* deferred scores (gac_net_write_begin): where each rescored fill's score
 * goes in a run's text */
typedef struct wmark {
    int64_t pos, ord;
} wmark;
typedef struct wmarks {
    wmark *m;
    int64_t n, cap;
} wmarks;

typedef struct wctx {
    const gac_net *n;
    gac_obuf *o;
    int side;
    const int64_t *tscore; /* per T fill (pre-order), GPU-rescored partial scores */
    int depth;
    char *buf;
    wmarks *marks; /* deferred: the run's score positions (else NULL) */
} wctx;

/* fill_info's stand-in for the rescored target-fill scores while they are
 * being computed: a rescored score is >= 1 (chainNet.c:244-245), so with
 * minScore <= 1 the fills that print do not depend on it */
static const int64_t k_deferred[1] = {1};

/* line formatting without stdio's format parsing (the .net files hold
 * millions of lines) */
static char *put_int(char *p, int64_t v) {
    static const char dig2[201] = "00010203040506070809101112131415161718192021222324"
                                  "25262728293031323334353637383940414243444546474849"
                                  "50515253545556575859606162636465666768697071727374"
                                  "75767778798081828384858687888990919293949596979899";
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    if (v < 0)
        *p++ = '-';
    /* the digit count first, then the digits straight into place, two per
     * step (no staging copy: a variable-length memcpy is a library call per
     * number, and the nets print ~150 M of them); 32-bit arithmetic when the
     * value fits, as nearly all coordinates do */
    static const uint32_t p10[10] = {0u,      10u,      100u,      1000u,      10000u,
                                     100000u, 1000000u, 10000000u, 100000000u, 1000000000u};
    if (u >> 32) {
        int nd = 1;
        for (uint64_t t = 10; nd < 20 && u >= t; t *= 10)
            ++nd;
        char *const e = p + nd;
        char *q = e;
        while (u >= 100) {
            const unsigned r = (unsigned)(u % 100);
            u /= 100;
            q -= 2;
            memcpy(q, dig2 + 2 * r, 2);
        }
        if (u >= 10) {
            q -= 2;
            memcpy(q, dig2 + 2 * u, 2);
        } else {
            *--q = (char)('0' + u);
        }
        return e;
    }
    uint32_t w = (uint32_t)u;
    int nd = ((32 - __builtin_clz(w | 1)) * 1233) >> 12; /* floor(log10) or one less */
    nd += (nd < 10 && w >= p10[nd]) ? 1 : 0;
    if (nd == 0)
        nd = 1;
    char *const e = p + nd;
    char *q = e;
    while (w >= 100) {
        const uint32_t r = w % 100;
        w /= 100;
        q -= 2;
        memcpy(q, dig2 + 2 * r, 2);
    }
    if (w >= 10) {
        q -= 2;
        memcpy(q, dig2 + 2 * w, 2);
    } else {
        *--q = (char)('0' + w);
    }
    return e;
}

static char *put_str(char *p, const char *s) {
    while (*s)
        *p++ = *s++;
    return p;
}

/* "%1.0f": printf rounds the double's exact value half to even, which is
 * nearbyint in the default rounding mode (and "-0" for negatives that round
 * to zero); beyond 1e15 through printf */
static char *put_score(char *p, double v) {
    if (v > -1e15 && v < 1e15) {
        const double r = nearbyint(v);
        if (r == 0 && signbit(r)) {
            *p++ = '-';
            *p++ = '0';
            return p;
        }
        return put_int(p, (int64_t)r);
    }
    return p + sprintf(p, "%1.0f", v);
}

/* (the callers reserve room past the indentation: whole 16-byte stores) */
static char *put_spaces(char *p, int k) {
    static const char sp[16] = {' ', ' ', ' ', ' ', ' ', ' ', ' ', ' ',
                                ' ', ' ', ' ', ' ', ' ', ' ', ' ', ' '};
    char *const e = p + k;
    for (; p < e; p += 16)
        memcpy(p, sp, 16);
    return e;
}

/* gap line at the given indentation (rOutputGap, chainNet.c:747-761) */
static void put_gap_line(const wctx *w, const nfill *parent, const ngap *g, int depth) {
    const gac_net_input *in = &w->n->in;
    const int64_t c = parent->chain;
    const char *ochrom = w->side == GAC_Q ? in->t_names[in->t_seq[c]] : in->q_names[in->q_seq[c]];
    const int olen = w->side == GAC_Q ? w->n->nlen[GAC_T][in->t_seq[c]] : w->n->nlen[GAC_Q][in->q_seq[c]];
    if (olen > 400 || depth > 400) {
        gac_obuf_printf(w->o, "%*sgap %d %d %s %c %d %d\n", depth, "", g->start, g->end - g->start,
                  ochrom, in->q_strand[c] ? '-' : '+', g->o_start, g->o_end - g->o_start);
        return;
    }
    char *const buf = gac_obuf_reserve(w->o, 512 + 400), *p = buf;
    p = put_spaces(p, depth);
    p = put_str(p, "gap ");
    p = put_int(p, g->start);
    *p++ = ' ';
    p = put_int(p, g->end - g->start);
    *p++ = ' ';
    p = put_str(p, ochrom);
    *p++ = ' ';
    *p++ = in->q_strand[c] ? '-' : '+';
    *p++ = ' ';
    p = put_int(p, g->o_start);
    *p++ = ' ';
    p = put_int(p, g->o_end - g->o_start);
    *p++ = '\n';
    w->o->n += (size_t)(p - buf);
}

/* subchainInfo (chainNet.c:795-843) and rOutputFill's filter (:763-775):
 * the fill's score and aligned bases; 1 = the fill is printed (given that
 * its parent is) */
static int fill_info(const gac_net *n, int side, const int64_t *tscore, const nfill *f,
                     double *score_out, int *sub_out) {
    const gac_net_input *in = &n->in;
    const int64_t c = f->chain;
    int sub;
    double score;
    if (f->full) { /* the whole chain */
        score = in->score[c];
        sub = full_size(n, c);
    } else {
        sub = f->ali;
        if (side == GAC_T && tscore == k_deferred) {
            score = 1; /* placeholder: the fill's text gets the score later */
        } else if (side == GAC_T && tscore) {
            double r = (double)tscore[f->ord];
            score = r <= 0 ? 1 : r; /* chainNet.c:244-245 */
        } else {
            score = in->score[c] * sub / full_size(n, c);
        }
    }
    *score_out = score;
    *sub_out = sub;
    return score >= n->opt.min_score && sub >= n->opt.min_fill;
}

/* fill line (fillOut, chainNet.c:847-856) */
static void put_fill_line(const wctx *w, const nfill *f, int depth, double score, int sub) {
    const gac_net_input *in = &w->n->in;
    const int64_t c = f->chain;
    const char *ochrom = w->side == GAC_Q ? in->t_names[in->t_seq[c]] : in->q_names[in->q_seq[c]];
    const int olen = w->side == GAC_Q ? w->n->nlen[GAC_T][in->t_seq[c]] : w->n->nlen[GAC_Q][in->q_seq[c]];
    const int deferred = w->marks && w->side == GAC_T && !f->full;
    if (olen > 400 || depth > 400 || !(score > -1e300 && score < 1e300)) {
        gac_obuf_printf(w->o, "%*sfill %d %d %s %c %d %d id %d score ", depth, "", f->start,
                  f->end - f->start, ochrom, in->q_strand[c] ? '-' : '+', f->o_start,
                  f->o_end - f->o_start, in->id[c]);
        if (deferred) {
            wmarks *m = w->marks;
            if (m->n == m->cap) {
                m->cap = m->cap ? 2 * m->cap : 256;
                m->m = realloc(m->m, (size_t)m->cap * sizeof(wmark));
            }
            m->m[m->n++] = (wmark){(int64_t)w->o->n, f->ord};
        } else {
            gac_obuf_printf(w->o, "%1.0f", score);
        }
        gac_obuf_printf(w->o, " ali %d\n", sub);
        return;
    }
    char *const buf = gac_obuf_reserve(w->o, 512 + 400 + 400), *p = buf;
    p = put_spaces(p, depth);
    p = put_str(p, "fill ");
    p = put_int(p, f->start);
    *p++ = ' ';
    p = put_int(p, f->end - f->start);
    *p++ = ' ';
    p = put_str(p, ochrom);
    *p++ = ' ';
    *p++ = in->q_strand[c] ? '-' : '+';
    *p++ = ' ';
    p = put_int(p, f->o_start);
    *p++ = ' ';
    p = put_int(p, f->o_end - f->o_start);
    p = put_str(p, " id ");
    p = put_int(p, in->id[c]);
    p = put_str(p, " score ");
    if (deferred) {
        wmarks *m = w->marks; /* a rescored fill: its score is inserted here later */
        if (m->n == m->cap) {
            m->cap = m->cap ? 2 * m->cap : 256;
            m->m = realloc(m->m, (size_t)m->cap * sizeof(wmark));
        }
        m->m[m->n++] = (wmark){(int64_t)w->o->n + (p - buf), f->ord};
    } else {
        p = put_score(p, score);
    }
    p = put_str(p, " ali ");
    p = put_int(p, sub);
    *p++ = '\n';
    w->o->n += (size_t)(p - buf);
}

/* Parallel output.  The .net text of a side is rOutputFill's depth-first
 * walk (chainNet.c:747-776, 858-896).  Cut it at fill lines: the segment of
 * the fill at pre-order index i is its "net" header (a chromosome's first
 * top-level fill), its fill line, and every gap line printed before the next
 * fill line -- its own gaps up to the first one with a printed fill, and,
 * once its subtree is done, the remaining gaps of its ancestors up to the
 * next printed fill.  Segments are independent given the per-fill print
 * flags, so runs of consecutive pre-order fills are formatted on worker
 * threads (balanced by fill count, whatever the nesting) and written in
 * order. */
typedef struct wjob {
    const gac_net *n;
    int side;
    const int64_t *tscore;
    wmarks *marks; /* deferred: per run */
    const nfill *const *ord;
    int64_t nf, per;
    double *score;   /* per fill (pre-order) */
    int32_t *sub;
    uint8_t *show;   /* passes its own filter */
    uint8_t *more;   /* a later sibling in its gap passes its filter */
    uint8_t *reached;/* printed: passes and every ancestor fill is printed */
    uint16_t *lvl;   /* nesting level, for the more and reached passes */
    int32_t *pix;    /* index in its gap's fill list, for the more pass */
    _Atomic int deep; /* a level >= 65535 seen: both passes chase links instead */
    _Atomic int64_t next;
} wjob;

static int gap_prints_fill(const wjob *J, const ngap *g) {
    if (g->n_fills == 0)
        return 0;
    const int64_t o = g->fills[0]->ord;
    return J->show[o] || J->more[o];
}

static void write_segment(const wjob *J, wctx *w, int64_t i) {
    const nfill *f = J->ord[i];
    if (!f->pgap->pfill && f->pidx == 0) { /* first top-level fill: the chromosome header */
        const nchrom *c = &J->n->chroms[J->side][f->pgap->pidx];
        gac_obuf_printf(w->o, "net %s %d\n", c->name, c->size);
    }
    if (!J->reached[i])
        return;
    put_fill_line(w, f, 2 * f->level + 1, J->score[i], J->sub[i]);
    const nfill *cur = f;
    int g0 = 0;
    for (;;) {
        for (int gi = g0; gi < cur->n_gaps; ++gi) {
            const ngap *g = cur->gaps[gi];
            put_gap_line(w, cur, g, 2 * cur->level + 2);
            if (gap_prints_fill(J, g))
                return; /* the next line is that fill's */
        }
        /* cur's subtree is done: its next printed sibling, or up */
        if (J->more[cur->ord])
            return;
        const ngap *pg = cur->pgap;
        if (!pg->pfill)
            return; /* end of the chromosome */
        g0 = pg->pidx + 1;
        cur = pg->pfill;
    }
}

static void write_run(gac_obuf *o, int64_t r, void *arg) {
    wjob *J = arg;
    const int64_t a = r * J->per;
    const int64_t b = a + J->per < J->nf ? a + J->per : J->nf;
    wctx w = {J->n, o, J->side, J->tscore, 0, NULL, J->marks ? &J->marks[r] : NULL};
    const gac_net_input *in = &J->n->in;
    for (int64_t i = a; i < b; ++i) {
        /* the fills are scattered over the netting arenas: fetch ahead */
        if (i + 16 < b)
            __builtin_prefetch(J->ord[i + 16]);
        if (i + 8 < b) {
            const nfill *f = J->ord[i + 8];
            __builtin_prefetch(f->gaps);
            __builtin_prefetch(&in->q_seq[f->chain]);
            __builtin_prefetch(&in->q_strand[f->chain]);
            __builtin_prefetch(&in->id[f->chain]);
            __builtin_prefetch(&in->t_seq[f->chain]);
        }
        if (i + 4 < b) {
            const nfill *f = J->ord[i + 4];
            for (int k = 0; k < f->n_gaps && k < 4; ++k)
                __builtin_prefetch(f->gaps[k]);
        }
        write_segment(J, &w, i);
    }
}

/* per-fill score / print flags (parallel over the pre-order list) */
static void *winfo_thread(void *arg) {
    wjob *J = arg;
    for (;;) {
        const int64_t a = atomic_fetch_add(&J->next, 4096);
        if (a >= J->nf)
            break;
        const int64_t b = a + 4096 < J->nf ? a + 4096 : J->nf;
        for (int64_t i = a; i < b; ++i) {
            if (i + 16 < b)
                __builtin_prefetch(J->ord[i + 16]);
            if (i + 8 < b) {
                const int64_t c = J->ord[i + 8]->chain;
                __builtin_prefetch(&J->n->in.score[c]);
                __builtin_prefetch(&J->n->chain_ali[c]);
            }
            J->show[i] = (uint8_t)fill_info(J->n, J->side, J->tscore, J->ord[i], &J->score[i],
                                            &J->sub[i]);
            const int32_t L = J->ord[i]->level;
            J->lvl[i] = (uint16_t)(L < 65535 ? L : 65535);
            J->pix[i] = J->ord[i]->pidx;
            if (L >= 65535)
                atomic_store(&J->deep, 1);
        }
    }
    return NULL;
}

/* "more" flags: every gap's fills, last to first */
static void mark_more(wjob *J, const ngap *g) {
    uint8_t any = 0;
    for (int k = g->n_fills - 1; k >= 0; --k) {
        const int64_t o = g->fills[k]->ord;
        J->more[o] = any;
        any |= J->show[o];
    }
}

static void *wmore_thread(void *arg) {
    wjob *J = arg;
    for (;;) {
        const int64_t a = atomic_fetch_add(&J->next, 4096);
        if (a >= J->nf)
            break;
        const int64_t b = a + 4096 < J->nf ? a + 4096 : J->nf;
        for (int64_t i = a; i < b; ++i) {
            if (i + 16 < b)
                __builtin_prefetch(J->ord[i + 16]);
            if (i + 8 < b) {
                const nfill *p = J->ord[i + 8];
                for (int k = 0; k < p->n_gaps && k < 4; ++k)
                    __builtin_prefetch(p->gaps[k]);
            }
            const nfill *f = J->ord[i];
            for (int k = 0; k < f->n_gaps; ++k)
                mark_more(J, f->gaps[k]);
        }
    }
    return NULL;
}

static int net_write_f(const gac_net *n, int side, const int64_t *tscores, FILE *f,
                       const char *const *meta, int32_t n_meta);

/* "reached" flags: a fill prints when it passes and every ancestor fill
 * prints; parents precede children in pre-order, so runs that start at
 * top-level fills (whole subtrees) are independent */
/* The same flags from the levels, per run of whole top-level subtrees,
 * scanning backwards: the fills of one gap are the fills of one level seen
 * with their gap indices counting down to 0 (a gap's fills are consecutive at
 * their level in pre-order, their subtrees in between), so a per-level
 * "some later sibling shows" accumulator, reset whenever the index does not
 * continue the count, replaces the walks of every gap's fill list.  Level 0
 * (the root gaps, which span runs) is left to the roots' pass. */
static void *wmore_lvl_thread(void *arg) {
    wjob *J = arg;
    const int64_t per = J->nf / (8 * (int64_t)gac_host_threads()) + 1;
    for (;;) {
        const int64_t r = atomic_fetch_add(&J->next, 1);
        if (r * per >= J->nf)
            return NULL;
        const int64_t a = next_top_level(J->n, J->side, r * per);
        const int64_t b = next_top_level(J->n, J->side, (r + 1) * per < J->nf ? (r + 1) * per : J->nf);
        int32_t pbuf[256], *prev = pbuf;
        uint8_t abuf[256], *acc = abuf;
        int cap = 256;
        for (int k = 0; k < cap; ++k)
            prev[k] = INT32_MIN;
        for (int64_t i = b - 1; i >= a; --i) {
            const int L = J->lvl[i];
            if (L == 0)
                continue;
            if (L >= cap) {
                const int nc = L + 256;
                int32_t *np = malloc((size_t)nc * sizeof(int32_t));
                uint8_t *na = malloc((size_t)nc);
                memcpy(np, prev, (size_t)cap * sizeof(int32_t));
                memcpy(na, acc, (size_t)cap);
                for (int k = cap; k < nc; ++k)
                    np[k] = INT32_MIN;
                if (prev != pbuf) {
                    free(prev);
                    free(acc);
                }
                prev = np;
                acc = na;
                cap = nc;
            }
            const int32_t p = J->pix[i];
            if (prev[L] != INT32_MIN && p == prev[L] - 1) {
                J->more[i] = acc[L];
                acc[L] |= J->show[i];
            } else {
                J->more[i] = 0;
                acc[L] = J->show[i];
            }
            prev[L] = p;
        }
        if (prev != pbuf) {
            free(prev);
            free(acc);
        }
    }
}

static void *wreached_thread(void *arg) {
    wjob *J = arg;
    const int64_t per = J->nf / (8 * (int64_t)gac_host_threads()) + 1;
    for (;;) {
        const int64_t r = atomic_fetch_add(&J->next, 1);
        if (r * per >= J->nf)
            return NULL;
        const int64_t a = next_top_level(J->n, J->side, r * per);
        const int64_t b = next_top_level(J->n, J->side, (r + 1) * per < J->nf ? (r + 1) * per : J->nf);
        const int64_t *po = __atomic_load_n(&J->n->pord_ok[J->side], __ATOMIC_ACQUIRE) ? J->n->pord[J->side] : NULL;
        if (po) {
            for (int64_t i = a; i < b; ++i)
                J->reached[i] = J->show[i] && (po[i] < 0 || J->reached[po[i]]);
            continue;
        }
        if (!atomic_load(&J->deep)) {
            /* pre-order from a top-level fill: a fill's parent is the last
             * fill before it one level up, so a stack of the last position
             * per level replaces the parent links */
            int64_t stk[256], *last = stk;
            int cap = 256;
            for (int64_t i = a; i < b; ++i) {
                const int L = J->lvl[i];
                if (L >= cap) {
                    const int nc = L + 256;
                    int64_t *q = malloc((size_t)nc * sizeof(int64_t));
                    memcpy(q, last, (size_t)cap * sizeof(int64_t));
                    if (last != stk)
                        free(last);
                    last = q;
                    cap = nc;
                }
                last[L] = i;
                J->reached[i] = J->show[i] && (L == 0 || J->reached[last[L - 1]]);
            }
            if (last != stk)
                free(last);
            continue;
        }
        for (int64_t i = a; i < b; ++i) {
            const nfill *pf = J->ord[i]->pgap->pfill;
            J->reached[i] = J->show[i] && (!pf || J->reached[pf->ord]);
        }
    }
}

int gac_net_write(const gac_net *n, int side, const int64_t *tscores, const char *path,
                  const char *const *meta, int32_t n_meta) {
    if (!n || !path || (side != GAC_T && side != GAC_Q))
        return gac_fail(GAC_E_ARG, "gac_net_write: bad argument");
    if (!(n->sides & (1 << side)))
        return gac_fail(GAC_E_STATE, "gac_net_write: side %d was not netted", side);
    FILE *f;
    int close_it = 1;
    if (strcmp(path, "stdout") == 0) {
        f = stdout;
        close_it = 0;
    } else {
        f = gac_open_output(path);
        if (!f)
            return gac_fail(GAC_E_IO, "Can't open %s to write", path);
    }
    int bad = net_write_f(n, side, tscores, f, meta, n_meta) != GAC_OK;
    if (close_it) {
        if (gac_close_output(f) != 0)
            bad = 1;
        gac_mark(side ? "net_write q: closed" : "net_write t: closed");
    } else {
        fflush(f);
    }
    if (bad)
        return gac_fail(GAC_E_IO, "write error on %s", path);
    return GAC_OK;
}

int gac_net_write_file(const gac_net *n, int side, const int64_t *tscores, FILE *f,
                       const char *const *meta, int32_t n_meta) {
    if (!n || !f || (side != GAC_T && side != GAC_Q))
        return gac_fail(GAC_E_ARG, "gac_net_write_file: bad argument");
    if (!(n->sides & (1 << side)))
        return gac_fail(GAC_E_STATE, "gac_net_write_file: side %d was not netted", side);
    if (net_write_f(n, side, tscores, f, meta, n_meta) != GAC_OK || fflush(f) != 0)
        return gac_fail(GAC_E_IO, "write error");
    return GAC_OK;
}

/* per-fill score / print flags of a side and the run split (wjob) */
static void wjob_flags(wjob *J, const gac_net *n, int side, const int64_t *tscore) {
    const int64_t nf = n->n_order[side];
    memset(J, 0, sizeof(*J));
    J->n = n;
    J->side = side;
    J->tscore = side == GAC_T ? tscore : NULL;
    J->ord = (const nfill *const *)n->order[side];
    J->nf = nf;
    const size_t m = (size_t)(nf ? nf : 1);
    J->score = malloc(m * sizeof(double));
    J->sub = malloc(m * sizeof(int32_t));
    J->show = malloc(m);
    J->more = malloc(m);
    J->reached = malloc(m);
    J->lvl = malloc(m * sizeof(uint16_t));
    J->pix = malloc(m * sizeof(int32_t));
    atomic_init(&J->deep, 0);
    const int nt = gac_host_threads();
    atomic_init(&J->next, 0);
    gac_run_threads(nt, winfo_thread, J);
    gac_mark("flags: info done");
    atomic_store(&J->next, 0);
    gac_run_threads(nt, atomic_load(&J->deep) ? wmore_thread : wmore_lvl_thread, J);
    gac_mark("flags: more done");
    for (int32_t k = 0; k < n->n_chroms[side]; ++k) {
        const nchrom *c = &n->chroms[side][k];
        if (c->root && c->root->fill_head)
            mark_more(J, c->root);
    }
    gac_mark("flags: roots done");
    atomic_store(&J->next, 0);
    gac_run_threads(nt, wreached_thread, J);
    gac_mark("flags: reached done");
    /* (runs of 1/64 of a thread's share: capping them at 128 or 1024 fills
     * as for chains made the C5 nets slower, 1.79-1.86 / 1.36 vs 1.31-1.34
     * s; scripts/gpu_net_runs_ab.sh) */
    J->per = nf / (64 * (int64_t)nt) + 1;
}

static void wjob_free_flags(wjob *J) {
    free(J->score);
    free(J->sub);
    free(J->show);
    free(J->more);
    free(J->reached);
    free(J->lvl);
    free(J->pix);
    J->lvl = NULL;
    J->pix = NULL;
    J->score = NULL;
    J->sub = NULL;
    J->show = J->more = J->reached = NULL;
}

static int net_write_f(const gac_net *n, int side, const int64_t *tscores, FILE *f,
                       const char *const *meta, int32_t n_meta) {
    for (int32_t i = 0; i < n_meta; ++i)
        fprintf(f, "%s\n", meta[i]);
    wjob J;
    gac_mark(side ? "net_write q: flags" : "net_write t: flags");
    wjob_flags(&J, n, side, tscores);
    gac_mark(side ? "net_write q: format+write" : "net_write t: format+write");
    const int64_t nr = (J.nf + J.per - 1) / J.per;
    int wbad = gac_par_output_buf(f, nr, write_run, &J);
    wjob_free_flags(&J);
    gac_mark(side ? "net_write q: done" : "net_write t: done");
    return (ferror(f) || wbad) ? GAC_E_IO : GAC_OK;
}

int gac_net_format(const gac_net *n, int side, const int64_t *tscores, const char *const *meta,
                   int32_t n_meta, char ***bufs, size_t **lens, int64_t *nbufs) {
    if (!n || (side != GAC_T && side != GAC_Q) || !bufs || !lens || !nbufs)
        return gac_fail(GAC_E_ARG, "gac_net_format: bad argument");
    if (!(n->sides & (1 << side)))
        return gac_fail(GAC_E_STATE, "gac_net_format: side %d was not netted", side);
    wjob J;
    wjob_flags(&J, n, side, tscores);
    const int64_t nr = (J.nf + J.per - 1) / J.per;
    char **b = NULL;
    size_t *l = NULL;
    const int bad = gac_par_format_buf(nr, write_run, &J, &b, &l);
    wjob_free_flags(&J);
    if (bad) {
        for (int64_t r = 0; r < nr; ++r)
            free(b ? b[r] : NULL);
        free(b);
        free(l);
        return gac_fail(GAC_E_IO, "gac_net_format: out of memory");
    }
    /* the '#' lines in front */
    char **ob = malloc((size_t)(nr + 1) * sizeof(char *));
    size_t *ol = malloc((size_t)(nr + 1) * sizeof(size_t));
    gac_obuf m = {NULL, 0, 0};
    for (int32_t i = 0; i < n_meta; ++i)
        gac_obuf_printf(&m, "%s\n", meta[i]);
    ob[0] = m.p;
    ol[0] = m.n;
    if (nr) {
        memcpy(ob + 1, b, (size_t)nr * sizeof(char *));
        memcpy(ol + 1, l, (size_t)nr * sizeof(size_t));
    }
    free(b);
    free(l);
    *bufs = ob;
    *lens = ol;
    *nbufs = nr + 1;
    return GAC_OK;
}

/* ---- two-phase target net for -rescore (gac_net_write_begin/_end) */
struct gac_net_wpre {
    wjob J;
    int64_t nr;
    char **bufs;
    size_t *lens;
    char **meta;
    int32_t n_meta;
    const int64_t *tscores;
};

int gac_net_write_begin(const gac_net *n, int side, const char *const *meta, int32_t n_meta,
                        gac_net_wpre **out) {
    if (!n || !out || side != GAC_T)
        return gac_fail(GAC_E_ARG, "gac_net_write_begin: bad argument");
    if (!(n->sides & (1 << side)))
        return gac_fail(GAC_E_STATE, "gac_net_write_begin: side %d was not netted", side);
    if (n->opt.min_score > 1)
        return gac_fail(GAC_E_STATE, "gac_net_write_begin: minScore > 1 (which fills print "
                                     "depends on the rescored scores)");
    gac_net_wpre *P = calloc(1, sizeof(*P));
    P->meta = malloc((size_t)(n_meta > 0 ? n_meta : 1) * sizeof(char *));
    for (int32_t i = 0; i < n_meta; ++i)
        P->meta[i] = strdup(meta[i]);
    P->n_meta = n_meta;
    gac_mark("write_begin t: flags");
    wjob_flags(&P->J, n, side, k_deferred);
    gac_mark("write_begin t: format");
    P->nr = (P->J.nf + P->J.per - 1) / P->J.per;
    P->J.marks = calloc((size_t)(P->nr > 0 ? P->nr : 1), sizeof(wmarks));
    const int bad = gac_par_format_buf(P->nr, write_run, &P->J, &P->bufs, &P->lens);
    wjob_free_flags(&P->J);
    gac_mark("write_begin t: done");
    if (bad) {
        gac_net_write_free(P);
        return gac_fail(GAC_E_IO, "gac_net_write_begin: out of memory");
    }
    *out = P;
    return GAC_OK;
}

/* run r of a prepared net with the scores inserted (gac_par_output item) */
static void wpre_run(FILE *f, int64_t r, void *arg) {
    gac_net_wpre *P = arg;
    const char *buf = P->bufs[r];
    const wmarks *m = &P->J.marks[r];
    int64_t last = 0;
    char tmp[64];
    for (int64_t k = 0; k < m->n; ++k) {
        fwrite_unlocked(buf + last, 1, (size_t)(m->m[k].pos - last), f);
        const double v = (double)P->tscores[m->m[k].ord];
        const char *e = put_score(tmp, v <= 0 ? 1 : v); /* chainNet.c:244-245 */
        fwrite_unlocked(tmp, 1, (size_t)(e - tmp), f);
        last = m->m[k].pos;
    }
    fwrite_unlocked(buf + last, 1, P->lens[r] - (size_t)last, f);
}

int gac_net_write_end(gac_net_wpre *P, const int64_t *tscores, FILE *f) {
    if (!P || !tscores || !f)
        return gac_fail(GAC_E_ARG, "gac_net_write_end: bad argument");
    for (int32_t i = 0; i < P->n_meta; ++i)
        fprintf(f, "%s\n", P->meta[i]);
    P->tscores = tscores;
    gac_mark("write_end t: insert+write");
    const int wbad = gac_par_output(f, P->nr, wpre_run, P);
    const int bad = ferror(f) || wbad || fflush(f) != 0;
    gac_mark("write_end t: free");
    gac_net_write_free(P);
    gac_mark("write_end t: done");
    return bad ? gac_fail(GAC_E_IO, "write error") : GAC_OK;
}

void gac_net_write_free(gac_net_wpre *P) {
    if (!P)
        return;
    for (int64_t r = 0; r < P->nr; ++r) {
        free(P->bufs ? P->bufs[r] : NULL);
        free(P->J.marks ? P->J.marks[r].m : NULL);
    }
    free(P->bufs);
    free(P->lens);
    free(P->J.marks);
    for (int32_t i = 0; i < P->n_meta; ++i)
        free(P->meta[i]);
    free(P->meta);
    free(P);
}
