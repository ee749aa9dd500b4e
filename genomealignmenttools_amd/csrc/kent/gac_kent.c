/* gac_kent.c -- kent-signature shims over the libgachain batch ABI
 * (include/gachain_kent.h).  Scoring is gac_score_ranges on the bound
 * context; the subset functions are kent's list surgery on the host. */
#include "gachain_kent.h"

#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

struct gapCalc {
    gac_gapcalc *g;
};

static __thread gac_ctx *t_ctx;

void gac_kent_bind(gac_ctx *ctx) { t_ctx = ctx; }

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

void gac_kent_score_chains(struct chain *const *chains, int64_t n, struct axtScoreScheme *ss,
                           struct gapCalc *gapCalc, double *global) {
    gac_ctx *ctx = t_ctx;
    if (!ctx)
        die("gac_kent: no context bound (gac_kent_bind)");
    if (n <= 0)
        return;
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
    gac_range *r = malloc((size_t)n * sizeof(gac_range));
    off[0] = 0;
    int64_t k = 0;
    for (int64_t i = 0; i < n; ++i) {
        const struct chain *c = chains[i];
        ts[i] = gac_genome_seq_index(ctx, GAC_T, c->tName);
        qs[i] = gac_genome_seq_index(ctx, GAC_Q, c->qName);
        if (ts[i] < 0 || qs[i] < 0)
            die("gac_kent: %s / %s is not loaded on the bound context", c->tName, c->qName);
        st[i] = c->qStrand == '-';
        int32_t lo = 0x7fffffff, hi = -0x7fffffff;
        for (const struct cBlock *b = c->blockList; b; b = b->next, ++k) {
            bt[k] = b->tStart;
            bq[k] = b->qStart;
            bs[k] = b->tEnd - b->tStart;
            lo = b->tStart < lo ? b->tStart : lo;
            hi = b->tEnd > hi ? b->tEnd : hi;
        }
        off[i + 1] = k;
        /* a range covering every block: the whole chain */
        r[i] = (gac_range){(int32_t)i, lo <= hi ? lo : 0, lo <= hi ? hi : 0};
    }
    gac_chainset_desc d = {n, ts, qs, st, off, nb, bt, bq, bs};
    gac_chainset *cs = NULL;
    need(gac_chains_upload(ctx, &d, &cs));
    int64_t *g = malloc((size_t)n * 8);
    int32_t *ali = malloc((size_t)n * 4);
    need(gac_score_ranges(ctx, cs, r, n, 0, g, NULL, ali));
    for (int64_t i = 0; i < n; ++i)
        global[i] = (double)g[i];
    gac_chains_free(cs);
    free(ts), free(qs), free(st), free(off), free(bt), free(bq), free(bs), free(r), free(g),
        free(ali);
}

double chainCalcScore(struct chain *chain, struct axtScoreScheme *ss, struct gapCalc *gapCalc,
                      struct dnaSeq *query, struct dnaSeq *target) {
    (void)query, (void)target;
    if (!chain->blockList)
        return 0;
    double s;
    gac_kent_score_chains(&chain, 1, ss, gapCalc, &s);
    return s;
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
