/* gac_kent.c -- kent-signature shims over the libgachain batch ABI
 * (include/gachain_kent.h).  Scoring is gac_score_ranges on the bound
 * context; the subset functions are kent's list surgery on the host. */
#include "gachain_kent.h"

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct gapCalc {
    gac_gapcalc *g;
};

static __thread gac_ctx *t_ctx;

void gac_kent_forget_chains(void);

/* a resident chain set (the chainCalcScore cache) belongs to the context it
 * was scored on: rebinding drops it (gac_chains_free is safe even when that
 * context was closed in between: the set is then only deleted) */
void gac_kent_bind(gac_ctx *ctx) {
    if (ctx != t_ctx)
        gac_kent_forget_chains();
    t_ctx = ctx;
}

static void die(const char *fmt, ...) { /* errAbort */
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    fputc('\n', stderr);
    exit(255);
}

static void need(int rc) {
    if (rc != GAC_OK)
        die("%s", gac_last_error());
}

/* ------------------------------------------------ gapCalc (gapCalc.c:233-331) */
struct gapCalc *gapCalcFromFile(char *fileName) {
    struct gapCalc *c = calloc(1, sizeof(*c));
    need(gac_gapcalc_build(fileName, &c->g));
    return c;
}

struct gapCalc *gapCalcDefault(void) { return gapCalcFromFile("loose"); }

struct gapCalc *gapCalcOriginal(void) { return gapCalcFromFile("medium"); }

void gapCalcFree(struct gapCalc **pGapCalc) {
    if (!pGapCalc || !*pGapCalc)
        return;
    gac_gapcalc_free((*pGapCalc)->g);
    free(*pGapCalc);
    *pGapCalc = NULL;
}

int gapCalcCost(struct gapCalc *gapCalc, int dq, int dt) { return gac_gap_cost(gapCalc->g, dq, dt); }

/* ------------------------------------------------ scoring */
/* the 4x4 of the 256x256 kent matrix, [query][target] in A,C,G,T order */
static void matrix4(const struct axtScoreScheme *ss, int32_t mat[16]) {
    static const char b[4] = {'A', 'C', 'G', 'T'};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            mat[i * 4 + j] = ss->matrix[(unsigned char)b[i]][(unsigned char)b[j]];
}

static int base_ix(int c) {
    switch (c) {
    case 'a': case 'A': return 0;
    case 'c': case 'C': return 1;
    case 'g': case 'G': return 2;
    case 't': case 'T': return 3;
    default: return -1;
    }
}

/* A text entry point's matrix -> the device's 4x4: it must be a kent DNA
 * scheme (nonzero only between a/c/g/t, either case, the same for both
 * cases -- propagateCase, axt.c:402-421).  Checked once per matrix address. */
static void text_matrix(int matrix[256][256], int32_t mat[16]) {
    static __thread const void *ok_addr;
    static __thread int32_t ok_mat[16];
    if (ok_addr == (const void *)matrix) {
        memcpy(mat, ok_mat, sizeof(ok_mat));
        return;
    }
    static const char b[4] = {'A', 'C', 'G', 'T'};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            mat[i * 4 + j] = matrix[(unsigned char)b[i]][(unsigned char)b[j]];
    for (int q = 0; q < 256; ++q)
        for (int t = 0; t < 256; ++t) {
            const int iq = base_ix(q), it = base_ix(t);
            const int want = (iq >= 0 && it >= 0) ? mat[iq * 4 + it] : 0;
            if (matrix[q][t] != want)
                die("gac_kent: matrix[%d][%d] = %d: only a/c/g/t DNA score schemes are "
                    "supported (expected %d)", q, t, matrix[q][t], want);
        }
    ok_addr = matrix;
    memcpy(ok_mat, mat, sizeof(ok_mat));
}

static gac_ctx *bound(void) {
    if (!t_ctx)
        die("gac_kent: no context bound (gac_kent_bind)");
    return t_ctx;
}

void gac_kent_score_blocks(int64_t n, char *const *q, char *const *t, const int *size,
                           int matrix[256][256], double *out) {
    if (n <= 0)
        return;
    int32_t mat[16];
    text_matrix(matrix, mat);
    int64_t *s = malloc((size_t)n * 8);
    int32_t *z = malloc((size_t)n * 4);
    for (int64_t i = 0; i < n; ++i)
        z[i] = size[i] > 0 ? size[i] : 0;
    need(gac_score_text_blocks(bound(), n, (const char *const *)q, (const char *const *)t, z, mat,
                               s));
    for (int64_t i = 0; i < n; ++i)
        out[i] = (double)s[i];
    free(s);
    free(z);
}

double chainScoreBlock(char *q, char *t, int size, int matrix[256][256]) {
    double s;
    gac_kent_score_blocks(1, &q, &t, &size, matrix, &s);
    return s;
}

int axtScoreUngapped(struct axtScoreScheme *ss, char *q, char *t, int size) {
    double s;
    gac_kent_score_blocks(1, &q, &t, &size, ss->matrix, &s);
    return (int)s;
}

void cBlockFindCrossover(struct cBlock *left, struct cBlock *right, struct dnaSeq *qSeq,
                         struct dnaSeq *tSeq, int overlap, int matrix[256][256], int *retPos,
                         int *retScoreAdjustment) {
    if (overlap > (left->tEnd - left->tStart) || overlap > (right->tEnd - right->tStart))
        die("overlap is %d -- too large for one of these:\n"
            "qSize=%d  tSize=%d\n"
            "left: qStart=%d qEnd=%d (%d) tStart=%d tEnd=%d (%d)\n"
            "right: qStart=%d qEnd=%d (%d) tStart=%d tEnd=%d (%d)",
            overlap, qSeq->size, tSeq->size, left->qStart, left->qEnd, left->qEnd - left->qStart,
            left->tStart, left->tEnd, left->tEnd - left->tStart, right->qStart, right->qEnd,
            right->qEnd - right->qStart, right->tStart, right->tEnd, right->tEnd - right->tStart);
    int32_t mat[16];
    text_matrix(matrix, mat);
    const char *lq = qSeq->dna + left->qEnd - overlap, *lt = tSeq->dna + left->tEnd - overlap;
    const char *rq = qSeq->dna + right->qStart, *rt = tSeq->dna + right->tStart;
    const int32_t ov = overlap > 0 ? overlap : 0;
    int32_t pos = 0, adj = 0;
    need(gac_text_crossovers(bound(), 1, &lq, &lt, &rq, &rt, &ov, mat, &pos, &adj));
    *retPos = pos;
    *retScoreAdjustment = adj;
}

int chainConnectGapCost(int dq, int dt, struct chainConnect *cc) {
    return gapCalcCost(cc->gapCalc, dq, dt);
}

int chainConnectCost(struct cBlock *a, struct cBlock *b, struct chainConnect *cc) {
    int dq = b->qStart - a->qEnd, dt = b->tStart - a->tEnd, adj = 0;
    if (a->qStart >= b->qStart || a->tStart >= b->tStart)
        die("a (%d %d) not strictly before b (%d %d)", a->qStart, a->tStart, b->qStart, b->tStart);
    if (dq < 0 || dt < 0) {
        const int bSize = b->qEnd - b->qStart, aSize = a->qEnd - a->qStart;
        const int overlap = -(dq < dt ? dq : dt);
        if (overlap >= bSize || overlap >= aSize) {
            adj = 100000000; /* one block encloses the other on one dimension */
        } else {
            int crossover;
            cBlockFindCrossover(a, b, cc->query, cc->target, overlap, cc->ss->matrix, &crossover,
                                &adj);
            dq += overlap;
            dt += overlap;
        }
    }
    return adj + gapCalcCost(cc->gapCalc, dq, dt);
}

/* ---- chainRemovePartialOverlaps / chainMergeAbutting (chainConnect.c:142-368) */
static void check_increases(struct chain *chain, const char *message) {
    struct cBlock *a = chain->blockList;
    if (!a)
        return;
    for (struct cBlock *b = a->next; b; a = b, b = b->next)
        if (a->qStart >= b->qStart || a->tStart >= b->tStart)
            die("a (%d %d) not before b (%d %d) %s", a->qStart, a->tStart, b->qStart, b->tStart,
                message);
}

static void check_gaps(struct chain *chain, const char *message) {
    struct cBlock *a = chain->blockList;
    if (!a)
        return;
    for (struct cBlock *b = a->next; b; a = b, b = b->next)
        if (a->qEnd > b->qStart || a->tEnd > b->tStart)
            die("Negative gap between (%d %d - %d %d) and (%d %d - %d %d) %s", a->qStart, a->tStart,
                a->qEnd, a->tEnd, b->qStart, b->tStart, b->qEnd, b->tEnd, message);
}

static void check_start_before_end(struct chain *chain, const char *message) {
    for (struct cBlock *b = chain->blockList; b; b = b->next)
        if (b->qStart >= b->qEnd || b->tStart >= b->tEnd)
            die("Start after end in (%d %d) to (%d %d) %s", b->qStart, b->tStart, b->qEnd, b->tEnd,
                message);
}

static void calc_bounds(struct chain *chain) { /* chainCalcBounds */
    struct cBlock *b = chain->blockList;
    if (!b)
        return;
    chain->qStart = b->qStart;
    chain->tStart = b->tStart;
    while (b->next)
        b = b->next;
    chain->qEnd = b->qEnd;
    chain->tEnd = b->tEnd;
}

static void remove_negative_blocks(struct chain *chain) {
    struct cBlock *head = NULL, **tail = &head;
    int got = 0;
    for (struct cBlock *b = chain->blockList, *nx; b; b = nx) {
        nx = b->next;
        if (b->qStart >= b->qEnd || b->tStart >= b->tEnd) {
            got = 1;
            free(b);
        } else {
            *tail = b;
            tail = &b->next;
        }
    }
    *tail = NULL;
    chain->blockList = head;
    if (got)
        calc_bounds(chain);
}

void chainRemovePartialOverlaps(struct chain *chain, struct dnaSeq *qSeq, struct dnaSeq *tSeq,
                                int matrix[256][256]) {
    if (!chain->blockList)
        die("chainRemovePartialOverlaps: empty chain");
    check_increases(chain, "before removePartialOverlaps");
    for (;;) {
        int trimA = 0, trimB = 0;
        struct cBlock *a = chain->blockList, *b = a->next;
        for (;;) {
            if (!b)
                break;
            const int dq = b->qStart - a->qEnd, dt = b->tStart - a->tEnd;
            if (dq < 0 || dt < 0) {
                const int overlap = -(dq < dt ? dq : dt);
                const int aSize = a->qEnd - a->qStart, bSize = b->qEnd - b->qStart;
                if (overlap >= aSize || overlap >= bSize) {
                    trimB = 1;
                } else {
                    int crossover, adj;
                    cBlockFindCrossover(a, b, qSeq, tSeq, overlap, matrix, &crossover, &adj);
                    b->qStart += crossover;
                    b->tStart += crossover;
                    const int inv = overlap - crossover;
                    a->qEnd -= inv;
                    a->tEnd -= inv;
                    if (b->qEnd <= b->qStart)
                        trimB = 1;
                    else if (a->qEnd <= a->qStart)
                        trimA = 1;
                }
            }
            if (trimA) {
                remove_negative_blocks(chain);
                break;
            } else if (trimB) {
                b = b->next;
                free(a->next);
                a->next = b;
                trimB = 0;
            } else {
                a = b;
                b = b->next;
            }
        }
        if (!trimA)
            break;
    }
    calc_bounds(chain); /* setChainBounds */
    check_gaps(chain, "after removePartialOverlaps");
    check_start_before_end(chain, "after removePartialOverlaps");
}

void chainMergeAbutting(struct chain *chain) {
    struct cBlock *head = NULL, **tail = &head, *last = NULL;
    for (struct cBlock *b = chain->blockList, *nx; b; b = nx) {
        nx = b->next;
        if (!last || last->qEnd != b->qStart || last->tEnd != b->tStart) {
            *tail = b;
            tail = &b->next;
            last = b;
        } else {
            last->qEnd = b->qEnd;
            last->tEnd = b->tEnd;
            free(b);
        }
    }
    *tail = NULL;
    chain->blockList = head;
}

/* ---- chainBlocks (chainBlock.c:392-452) over gac_chain_blocks */
typedef struct cb_adapt {
    ConnectCost connect;
    GapCost gap;
    void *data;
    struct cBlock **v;
} cb_adapt;

static int cb_connect(int32_t a, int32_t b, void *u) {
    cb_adapt *x = u;
    return x->connect(x->v[a], x->v[b], x->data);
}

static int cb_gap(int dq, int dt, void *u) {
    cb_adapt *x = u;
    return x->gap(dq, dt, x->data);
}

static char *dup(const char *s);

struct chain *chainBlocks(char *qName, int qSize, char qStrand, char *tName, int tSize,
                          struct cBlock **pBlockList, ConnectCost connectCost, GapCost gapCost,
                          void *gapData, FILE *details) {
    if (!*pBlockList)
        return NULL;
    int32_t n = 0;
    for (struct cBlock *b = *pBlockList; b; b = b->next)
        ++n;
    struct cBlock **v = malloc((size_t)n * sizeof(*v));
    int32_t *qs = malloc((size_t)n * 4), *qe = malloc((size_t)n * 4), *ts = malloc((size_t)n * 4),
            *te = malloc((size_t)n * 4), *sc = malloc((size_t)n * 4);
    int32_t i = 0;
    for (struct cBlock *b = *pBlockList; b; b = b->next, ++i) {
        v[i] = b;
        qs[i] = b->qStart;
        qe[i] = b->qEnd;
        ts[i] = b->tStart;
        te[i] = b->tEnd;
        sc[i] = b->score;
    }
    cb_adapt ad = {connectCost, gapCost, gapData, v};
    gac_block_chains *out = NULL;
    need(gac_chain_blocks(n, qs, qe, ts, te, sc, cb_connect, cb_gap, &ad, qName, qSize, qStrand,
                          tName, tSize, details, &out));
    struct chain *head = NULL, **tail = &head;
    for (int32_t c = 0; c < out->n_chains; ++c) {
        struct chain *ch = calloc(1, sizeof(*ch));
        ch->qName = dup(qName);
        ch->qSize = qSize;
        ch->qStrand = qStrand;
        ch->tName = dup(tName);
        ch->tSize = tSize;
        ch->score = out->score[c];
        struct cBlock **bt = &ch->blockList;
        for (int32_t k = out->off[c]; k < out->off[c + 1]; ++k) {
            struct cBlock *b = v[out->blk[k]];
            *bt = b;
            bt = &b->next;
        }
        *bt = NULL;
        calc_bounds(ch);
        *tail = ch;
        tail = &ch->next;
    }
    gac_block_chains_free(out);
    free(v), free(qs), free(qe), free(ts), free(te), free(sc);
    *pBlockList = NULL;
    return head;
}

/* ---- chainCalcScore: scores of a chain list, resident between calls */
typedef struct kent_cache {
    gac_chainset *cs;
    const void *ss, *gap;
    int64_t n;
    struct chain **ptr;  /* [n] */
    uint64_t *fp;        /* [n] block-list fingerprint at scoring time */
    double *score;       /* [n] */
    int64_t *slot;       /* open-addressing table: chain pointer -> index */
    int64_t nslot;
} kent_cache;

static __thread kent_cache t_cache;

static uint64_t fingerprint(const struct chain *c) {
    uint64_t h = 1469598103934665603ull ^ (uint64_t)(unsigned char)c->qStrand;
    for (const char *p = c->tName; p && *p; ++p)
        h = (h ^ (unsigned char)*p) * 1099511628211ull;
    for (const char *p = c->qName; p && *p; ++p)
        h = (h ^ (unsigned char)*p) * 1099511628211ull;
    for (const struct cBlock *b = c->blockList; b; b = b->next) {
        h = (h ^ (uint32_t)b->tStart) * 1099511628211ull;
        h = (h ^ (uint32_t)b->tEnd) * 1099511628211ull;
        h = (h ^ (uint32_t)b->qStart) * 1099511628211ull;
    }
    return h;
}

static uint64_t hash_ptr(const void *p) {
    uint64_t x = (uint64_t)(uintptr_t)p;
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    return x ^ (x >> 33);
}

static int64_t cache_find(const kent_cache *k, const struct chain *c) {
    if (!k->nslot)
        return -1;
    for (uint64_t h = hash_ptr(c) & (k->nslot - 1);; h = (h + 1) & (k->nslot - 1)) {
        const int64_t i = k->slot[h];
        if (i < 0)
            return -1;
        if (k->ptr[i] == c)
            return i;
    }
}

void gac_kent_forget_chains(void) {
    kent_cache *k = &t_cache;
    if (k->cs)
        gac_chains_free(k->cs);
    free(k->ptr), free(k->fp), free(k->score), free(k->slot);
    memset(k, 0, sizeof(*k));
}

/* upload and score chains[0..n) (one gac_score_chains call); keep them */
static void cache_fill(struct chain *const *chains, int64_t n, struct axtScoreScheme *ss,
                       struct gapCalc *gapCalc) {
    gac_ctx *ctx = bound();
    gac_kent_forget_chains();
    kent_cache *k = &t_cache;
    int32_t mat[16];
    matrix4(ss, mat);
    need(gac_set_scoring(ctx, mat, gapCalc->g)); /* (kept when unchanged) */
    int64_t nb = 0;
    for (int64_t i = 0; i < n; ++i)
        for (const struct cBlock *b = chains[i]->blockList; b; b = b->next)
            ++nb;
    int32_t *ts = malloc((size_t)n * 4), *qs = malloc((size_t)n * 4);
    uint8_t *st = malloc((size_t)n);
    int64_t *off = malloc((size_t)(n + 1) * 8);
    int32_t *bt = malloc((size_t)(nb ? nb : 1) * 4), *bq = malloc((size_t)(nb ? nb : 1) * 4),
            *bs = malloc((size_t)(nb ? nb : 1) * 4);
    off[0] = 0;
    int64_t j = 0;
    for (int64_t i = 0; i < n; ++i) {
        const struct chain *c = chains[i];
        ts[i] = gac_genome_seq_index(ctx, GAC_T, c->tName);
        qs[i] = gac_genome_seq_index(ctx, GAC_Q, c->qName);
        if (ts[i] < 0 || qs[i] < 0)
            die("gac_kent: %s / %s is not loaded on the bound context", c->tName, c->qName);
        st[i] = c->qStrand == '-';
        for (const struct cBlock *b = c->blockList; b; b = b->next, ++j) {
            bt[j] = b->tStart;
            bq[j] = b->qStart;
            bs[j] = b->tEnd - b->tStart;
        }
        off[i + 1] = j;
    }
    gac_chainset_desc d = {n, ts, qs, st, off, nb, bt, bq, bs};
    need(gac_chains_upload(ctx, &d, &k->cs));
    int64_t *g = malloc((size_t)n * 8);
    int32_t *ali = malloc((size_t)n * 4);
    need(gac_score_chains(ctx, k->cs, 0, g, NULL, ali));
    k->n = n;
    k->ss = ss;
    k->gap = gapCalc;
    k->ptr = malloc((size_t)n * sizeof(*k->ptr));
    k->fp = malloc((size_t)n * 8);
    k->score = malloc((size_t)n * 8);
    k->nslot = 16;
    while (k->nslot < 2 * n)
        k->nslot <<= 1;
    k->slot = malloc((size_t)k->nslot * 8);
    memset(k->slot, 0xff, (size_t)k->nslot * 8);
    for (int64_t i = 0; i < n; ++i) {
        k->ptr[i] = chains[i];
        k->fp[i] = fingerprint(chains[i]);
        k->score[i] = (double)g[i];
        if (cache_find(k, chains[i]) >= 0)
            continue; /* the same chain twice: its first index answers */
        uint64_t h = hash_ptr(chains[i]) & (k->nslot - 1);
        while (k->slot[h] >= 0)
            h = (h + 1) & (k->nslot - 1);
        k->slot[h] = i;
    }
    free(ts), free(qs), free(st), free(off), free(bt), free(bq), free(bs), free(g), free(ali);
}

/* the cached score of c, or NAN when c is not (or no longer) cached */
static double cache_score(struct chain *c, struct axtScoreScheme *ss, struct gapCalc *gapCalc) {
    const kent_cache *k = &t_cache;
    /* (a set orphaned by gac_close, or of another context, never answers) */
    if (!k->cs || k->ss != ss || k->gap != gapCalc || !t_ctx || gac_chains_context(k->cs) != t_ctx)
        return NAN;
    const int64_t i = cache_find(k, c);
    if (i < 0 || k->fp[i] != fingerprint(c))
        return NAN;
    return k->score[i];
}

void gac_kent_score_chains(struct chain *const *chains, int64_t n, struct axtScoreScheme *ss,
                           struct gapCalc *gapCalc, double *global) {
    if (n <= 0)
        return;
    int64_t i = 0;
    for (; i < n; ++i)
        if (isnan(global[i] = cache_score(chains[i], ss, gapCalc)))
            break;
    if (i == n)
        return;
    cache_fill(chains, n, ss, gapCalc);
    for (i = 0; i < n; ++i)
        global[i] = t_cache.score[cache_find(&t_cache, chains[i])];
}

/* chainConnect.c:42-59: the chain's blocks scored on caller text that
 * starts at the chain's qStart / tStart (one batched device call), minus
 * the gap costs */
double chainCalcScoreSubChain(struct chain *chain, struct axtScoreScheme *ss,
                              struct gapCalc *gapCalc, struct dnaSeq *query,
                              struct dnaSeq *target) {
    int64_t n = 0;
    for (const struct cBlock *b = chain->blockList; b; b = b->next)
        ++n;
    if (!n)
        return 0;
    char **q = malloc((size_t)n * sizeof(char *)), **t = malloc((size_t)n * sizeof(char *));
    int *z = malloc((size_t)n * sizeof(int));
    double *sc = malloc((size_t)n * sizeof(double));
    int64_t i = 0;
    for (const struct cBlock *b = chain->blockList; b; b = b->next, ++i) {
        q[i] = query->dna + (b->qStart - chain->qStart);
        t[i] = target->dna + (b->tStart - chain->tStart);
        z[i] = b->tEnd - b->tStart;
    }
    gac_kent_score_blocks(n, q, t, z, ss->matrix, sc);
    double score = 0;
    i = 0;
    for (const struct cBlock *b = chain->blockList; b; b = b->next, ++i) {
        score += sc[i];
        if (b->next)
            score -= gapCalcCost(gapCalc, b->next->qStart - b->qEnd, b->next->tStart - b->tEnd);
    }
    free(q), free(t), free(z), free(sc);
    return score;
}

/* the chain can go to the device: its sequences are loaded and its blocks
 * ascend without overlap inside them (what gac_chains_upload accepts) */
static int uploadable(gac_ctx *ctx, const struct chain *c) {
    const int32_t ti = gac_genome_seq_index(ctx, GAC_T, c->tName);
    const int32_t qi = gac_genome_seq_index(ctx, GAC_Q, c->qName);
    if (ti < 0 || qi < 0)
        return 0;
    const int64_t tsize = gac_genome_seq_size(ctx, GAC_T, ti);
    const int64_t qsize = gac_genome_seq_size(ctx, GAC_Q, qi);
    int64_t pt = 0, pq = 0;
    for (const struct cBlock *b = c->blockList; b; b = b->next) {
        const int64_t z = (int64_t)b->tEnd - b->tStart;
        if (z < 0 || b->tStart < pt || b->qStart < pq || b->tEnd > tsize || b->qStart + z > qsize)
            return 0;
        pt = b->tEnd;
        pq = b->qStart + z;
    }
    return 1;
}

double chainCalcScore(struct chain *chain, struct axtScoreScheme *ss, struct gapCalc *gapCalc,
                      struct dnaSeq *query, struct dnaSeq *target) {
    (void)query, (void)target;
    if (!chain->blockList)
        return 0;
    double s = cache_score(chain, ss, gapCalc);
    if (!isnan(s))
        return s;
    /* the chain and the rest of its list in one call: a caller looping
     * chainCalcScore over the list is then served from the resident set */
    int64_t n = 0, cap = 1024;
    struct chain **v = malloc((size_t)cap * sizeof(*v));
    gac_ctx *ctx = bound();
    for (struct chain *c = chain; c; c = c->next) {
        /* the rest of the list only where it can be scored as it stands (a
         * list fresh from chainBlocks still holds overlapping blocks until
         * chainRemovePartialOverlaps reaches each chain); this chain always,
         * so that its problems are reported */
        if (!c->blockList || (c != chain && !uploadable(ctx, c)))
            continue;
        if (n == cap)
            v = realloc(v, (size_t)(cap *= 2) * sizeof(*v));
        v[n++] = c;
    }
    cache_fill(v, n, ss, gapCalc);
    free(v);
    return t_cache.score[cache_find(&t_cache, chain)];
}

/* ------------------------------------------------ chainSubsetOnT (chain.c:471-558) */
static char *dup(const char *s) {
    char *d = malloc(strlen(s) + 1);
    strcpy(d, s);
    return d;
}

void chainFastSubsetOnT(struct chain *chain, struct cBlock *firstBlock, int subStart,
                        int subEnd, struct chain **retSubChain, struct chain **retChainToFree) {
    if (subStart <= chain->tStart && subEnd >= chain->tEnd) { /* the easy case */
        *retSubChain = chain;
        *retChainToFree = NULL;
        return;
    }
    struct cBlock *head = NULL, **tail = &head;
    int qs = 0x3fffffff, qe = -0x3fffffff, tsm = 0x3fffffff, tem = -0x3fffffff;
    for (const struct cBlock *o = firstBlock; o; o = o->next) {
        if (o->tStart >= subEnd)
            break;
        struct cBlock *b = malloc(sizeof(*b));
        *b = *o;
        b->next = NULL;
        if (b->tStart < subStart) {
            b->qStart += subStart - b->tStart;
            b->tStart = subStart;
        }
        if (b->tEnd > subEnd) {
            b->qEnd -= b->tEnd - subEnd;
            b->tEnd = subEnd;
        }
        *tail = b;
        tail = &b->next;
        qs = b->qStart < qs ? b->qStart : qs;
        qe = b->qEnd > qe ? b->qEnd : qe;
        tsm = b->tStart < tsm ? b->tStart : tsm;
        tem = b->tEnd > tem ? b->tEnd : tem;
    }
    struct chain *sub = NULL;
    if (head) {
        sub = calloc(1, sizeof(*sub));
        sub->blockList = head;
        sub->qName = dup(chain->qName);
        sub->qSize = chain->qSize;
        sub->qStrand = chain->qStrand;
        sub->qStart = qs;
        sub->qEnd = qe;
        sub->tName = dup(chain->tName);
        sub->tSize = chain->tSize;
        sub->tStart = tsm;
        sub->tEnd = tem;
        sub->id = chain->id;
        double ratio = sub->tEnd - sub->tStart; /* the "fake new score" */
        ratio /= chain->tEnd - chain->tStart;
        sub->score = ratio * chain->score;
    }
    *retSubChain = *retChainToFree = sub;
}

void chainSubsetOnT(struct chain *chain, int subStart, int subEnd, struct chain **retSubChain,
                    struct chain **retChainToFree) {
    struct cBlock *first = chain->blockList;
    while (first && first->tEnd <= subStart)
        first = first->next;
    chainFastSubsetOnT(chain, first, subStart, subEnd, retSubChain, retChainToFree);
}

void gac_kent_chain_free(struct chain **pChain) {
    struct chain *c = pChain ? *pChain : NULL;
    if (!c)
        return;
    for (struct cBlock *b = c->blockList, *nx; b; b = nx) {
        nx = b->next;
        free(b);
    }
    free(c->tName);
    free(c->qName);
    free(c);
    *pChain = NULL;
}
