/* chainCleaner -- drop-in for src/chainCleaner/chainCleaner.c: remove
 * chain-breaking alignments ("suspects") from chains that break lower-scoring
 * nested chains in the nets.
 *
 * Same command line, options, output files (out.chain chainSort-ed, out.bed,
 * -newChainIDDict, -suspectDataFile, -debug files) and output order as the
 * reference.  Its output order follows kent hash traversals and its
 * decisions are sequential (a removal changes the breaking chain and the
 * fills of the neighbouring breaks), so the host replays that loop exactly:
 *   - net fills/gaps -> per-chain fill/gap records   (parseFill, :786-866)
 *   - aligning regions merged like genomeRangeTree    (rConvert, :700-784;
 *     isBrokenByAnotherHigherScoringChain, :868-890)
 *   - valid breaks in chainId2Count hash order        (getValidBreaks, :969-1085)
 *   - loopOverBreaks in hashElListHash(breakHash) order (:1452-1631) with
 *     testAndRemoveSuspect's thresholds and break updates (:1191-1398).
 * Every sub-chain score (chainSubsetOnT + chainCalcScore +
 * chainCalcScoreLocal, getChainScore :531-582) comes from libgachain on the
 * GPU.  Scores are cached by sub-chain content: a range of a chain that lost
 * blocks keeps its original key while none of the removed blocks fall in it.
 * The sub-chains of every break (and adjacent pair) are scored in one batch
 * before the loop and again at the start of every later pass over a
 * breaking chain's list; whatever a removal changes mid-pass is scored on
 * demand.  Without -net the chains are netted in-process (chainNet
 * -minScore=0 | NetFilterNonNested.perl -minScore1 3000, :1639-1676), and the
 * final chainSort (:1863) is in-process as well (chainSort.c:41-75). */
#define _GNU_SOURCE
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <string.h>
#include <unistd.h>

#include "gac_netfile.h"
#include "gac_tool.h"
#include "gachain.h"
#include "host/gac_host.h"

static const gt_spec k_opts[] = {
    {"net", GT_STRING},
    {"tSizes", GT_STRING},
    {"qSizes", GT_STRING},
    {"scoreScheme", GT_STRING},
    {"linearGap", GT_STRING},
    {"debug", GT_BOOL},
    {"foldThreshold", GT_DOUBLE},
    {"LRfoldThreshold", GT_DOUBLE},
    {"LRfoldThresholdPairs", GT_DOUBLE},
    {"maxSuspectBases", GT_DOUBLE},
    {"maxSuspectScore", GT_DOUBLE},
    {"minBrokenChainScore", GT_DOUBLE},
    {"minLRGapSize", GT_INT},
    {"doPairs", GT_BOOL},
    {"maxPairDistance", GT_INT},
    {"newChainIDDict", GT_STRING},
    {"suspectDataFile", GT_STRING},
    {"onlyThisChr", GT_STRING},
    {"onlyThisStart", GT_INT},
    {"onlyThisEnd", GT_INT},
    {NULL, 0},
};

/* removal thresholds (chainCleaner.c:99-118) */
static double LRfoldThreshold = 2.5;
static double foldThreshold = 0;
static double maxSuspectBases = INT_MAX;
static double maxSuspectScore = 100000;
static double minBrokenChainScore = 50000;
static int minLRGapSize = 0;
static int doPairs = 0;
static double LRfoldThresholdPairs = 10;
static int maxPairDistance = 10000;
static const char *onlyThisChr = NULL;
static int onlyThisStart = -1, onlyThisEnd = -1;
static int debug = 0;

static void usage(void) {
    gt_abort(
        "chainCleaner - Remove chain-breaking alignments from chains that break nested chains.\n"
        "\n"
        "NOTATION: The \"breaking chain\" contains a local alignment block (called \"chain-breaking alignment\" (CBA) or \"suspect\") that breaks a nested chain (\"broken chain\") into two nets.\n"
        "\n"
        "usage:\n"
        "   chainCleaner in.chain tNibDir qNibDir out.chain out.bed -net=in.net \n"
        " OR \n"
        "   chainCleaner in.chain tNibDir qNibDir out.chain out.bed -tSizes=/dir/to/target/chrom.sizes -qSizes=/dir/to/query/chrom.sizes \n"
        " First option:   you have netted the chains and specify the net file via -net=netFile\n"
        " Second option:  you have not netted the chains. Then chainCleaner will net them (in-process). In this case, you must specify the chrom.sizes file for the target and query with -tSizes/-qSizes\n"
        " tNibDir/qNibDir are the names of .2bit files (nib directories are not supported)\n\n"
        "\n"
        "output:\n"
        "   out.chain      output file in chain format containing the untouched chains, the original broken chain and the modified breaking chains. NOTE: this file is chainSort-ed.\n"
        "   out.bed        output file in bed format containing the coords and information about the removed chain-breaking alignments.\n"
        "\n"
        "Most important options for deciding which chain-breaking alignments (CBA) to remove:\n"
        "   -LRfoldThreshold=N        threshold for removing local alignment blocks if the score of the left and right fill of brokenChain / CBA score is at least this fold threshold. Default %1.1f\n"
        "   -doPairs                  flag: if set, do test if pairs of CBAs can be removed\n"
        "   -LRfoldThresholdPairs=N   threshold for removing local alignment blocks if the score of the left and right fill of brokenChain / CBA score is at least this fold threshold. Default %1.1f\n"
        "   -maxPairDistance=N        only consider pairs of CBAs where the distance between the end of the upstream CBA and the start of the downstream CBA is at most that many bp (Default %d)\n"
        "\n"
        "   -scoreScheme=fileName       Read the scoring matrix from a blastz-format file\n"
        "   -linearGap=<medium|loose|filename> Specify type of linearGap to use.\n"
        "              *Must* specify this argument to one of these choices.\n"
        "              loose is chicken/human linear gap costs.\n"
        "              medium is mouse/human linear gap costs.\n"
        "              Or specify a piecewise linearGap tab delimited file.\n"
        "\n"
        "Other options for deciding which suspects to remove: \n"
        "   -foldThreshold=N          threshold for removing local alignment blocks if the brokenChain score / suspect score is at least this fold threshold. Default %1.1f\n"
        "   -maxSuspectBases=N        threshold for number of target bases in aligning blocks of the suspect subChain. If higher, do not remove suspect. Default %d\n"
        "   -maxSuspectScore=N        threshold for score of suspect subChain. If higher, do not remove suspect. Default %d\n"
        "   -minBrokenChainScore=N    threshold for minimum score of the entire broken chain. If the broken chain scores lower, it is less likely to be a real alignment and we will not remove the suspect. Default %d\n"
        "   -minLRGapSize=N           threshold for min size of left/right gap (how far the suspect is away from other blocks in the breaking chain). If lower, do not remove suspect (suspect to close to left or right part of breaking chain). Default %d\n"
        "\n"
        "Debug and testing options: \n"
        "   -newChainIDDict=fileName  output 'newChainID{tab}breakingChainID' to this file.\n"
        "   -suspectDataFile=fileName output all the data for suspects to this file in bed format. If set, we do not clean any suspect.\n"
        "   -debug                    produces output chain files with the suspect and broken chains, and a bed file with information about all possible suspects.\n",
        LRfoldThreshold, LRfoldThresholdPairs, maxPairDistance, foldThreshold, (int)maxSuspectBases,
        (int)maxSuspectScore, (int)minBrokenChainScore, minLRGapSize);
}

#define GROWV(ptr, cap, n)                                                     \
    do {                                                                       \
        if ((n) >= (cap)) {                                                    \
            (cap) = (cap) ? (cap) * 2 : 256;                                   \
            (ptr) = realloc((ptr), (size_t)(cap) * sizeof(*(ptr)));           \
        }                                                                      \
    } while (0)

/* assert() as in the reference (abort with the expression) */
static void must_assert(int ok, const char *what) {
    if (!ok) {
        fprintf(stderr, "chainCleaner: Assertion `%s' failed.\n", what);
        fflush(stderr);
        abort();
    }
}

/* ================================================================ nets */
enum { kMaxNetDepth = 64 }; /* maxNetDepth */

typedef struct gapinfo { /* depth2gap[depth] */
    int valid;
    int32_t start, end, parent, depth;
} gapinfo;

typedef struct fillgap { /* struct fillGapInfo */
    int32_t depth, chain_id, chrom;
    int32_t fill_start, fill_end;
    int gap_valid;
    int32_t gap_start, gap_end, parent_id, gap_depth;
    int32_t next;
} fillgap;

typedef struct netstate {
    gt_netset ns;
    gt_names chroms;  /* net (target) names */
    gt_khash count;   /* chainId2Count */
    int32_t *cnt, *fg_head, *fg_tail; /* per chainId2Count element */
    int32_t cnt_cap;
    fillgap *fg;
    int64_t nfg, fgcap;
    gapinfo depth2gap[kMaxNetDepth];
    int32_t depth2chain[kMaxNetDepth];
} netstate;

static netstate g_net;

static const char *chrom_name(int32_t chrom) { return g_net.chroms.names[chrom]; }

/* parseFill (chainCleaner.c:786-866) */
static void parse_fill(netstate *st, int32_t f, int depth, int32_t chrom) {
    if (depth >= kMaxNetDepth)
        gt_abort("ERROR: net depth %d exceeds maxNetDepth %d\n", depth, kMaxNetDepth);
    for (; f >= 0; f = st->ns.fills[f].next) {
        const gt_fill *x = &st->ns.fills[f];
        if (x->chain_id) {
            st->depth2chain[depth] = x->chain_id;
            if (depth > 1) {
                int32_t e = gt_khash_find(&st->count, x->chain_id);
                if (e < 0) {
                    e = gt_khash_add(&st->count, x->chain_id);
                    if (e >= st->cnt_cap) {
                        st->cnt_cap = st->cnt_cap ? st->cnt_cap * 2 : 1024;
                        st->cnt = realloc(st->cnt, (size_t)st->cnt_cap * 4);
                        st->fg_head = realloc(st->fg_head, (size_t)st->cnt_cap * 4);
                        st->fg_tail = realloc(st->fg_tail, (size_t)st->cnt_cap * 4);
                    }
                    st->cnt[e] = 0;
                    st->fg_head[e] = st->fg_tail[e] = -1;
                }
                st->cnt[e]++;
                GROWV(st->fg, st->fgcap, st->nfg);
                fillgap *g = &st->fg[st->nfg];
                const gapinfo *gi = &st->depth2gap[depth - 1];
                g->depth = depth;
                g->chain_id = x->chain_id;
                g->chrom = chrom;
                g->fill_start = x->tstart;
                g->fill_end = x->tstart + x->tsize;
                g->gap_valid = gi->valid;
                g->gap_start = gi->start;
                g->gap_end = gi->end;
                g->parent_id = gi->parent;
                g->gap_depth = gi->depth;
                g->next = -1;
                if (st->fg_tail[e] < 0)
                    st->fg_head[e] = (int32_t)st->nfg;
                else
                    st->fg[st->fg_tail[e]].next = (int32_t)st->nfg;
                st->fg_tail[e] = (int32_t)st->nfg;
                ++st->nfg;
            }
        } else {
            gapinfo *gi = &st->depth2gap[depth];
            gi->valid = 1;
            gi->start = x->tstart;
            gi->end = x->tstart + x->tsize;
            gi->parent = st->depth2chain[depth - 1];
            gi->depth = depth;
        }
        if (x->child >= 0)
            parse_fill(st, x->child, depth + 1, chrom);
    }
}

/* ---- aligning regions (rConvert / addAliBlocksToGenomeRangeTree) ---- */
typedef struct arange {
    int32_t start, end, chain_id;
} arange;

typedef struct region { /* one range of the merged range tree */
    int32_t start, end;
    int32_t min1, min2; /* the two smallest distinct chain ids merged in */
} region;

typedef struct chromregions {
    arange *r;
    int64_t n, cap;
    region *c;   /* non-empty unions sorted by start, then empty ranges */
    int64_t nc, nnz;
} chromregions;

static void add_range(chromregions *cr, int32_t s, int32_t e, int32_t id) {
    GROWV(cr->r, cr->cap, cr->n);
    cr->r[cr->n++] = (arange){s, e, id};
}

/* addAliBlocksToGenomeRangeTree with nextGapWithInsert (:700-762) */
static void add_ali_blocks(const gt_netset *ns, int32_t f, chromregions *cr) {
    const gt_fill *x = &ns->fills[f];
    int32_t ts = x->tstart;
    for (int32_t c = x->child;;) {
        while (c >= 0 && ns->fills[c].child < 0)
            c = ns->fills[c].next;
        if (c < 0)
            break;
        add_range(cr, ts, ns->fills[c].tstart, x->chain_id);
        ts = ns->fills[c].tstart + ns->fills[c].tsize;
        c = ns->fills[c].next;
    }
    add_range(cr, ts, x->tstart + x->tsize, x->chain_id);
}

static void r_convert(const gt_netset *ns, int32_t f, chromregions *cr) {
    for (; f >= 0; f = ns->fills[f].next) {
        if (ns->fills[f].chain_id)
            add_ali_blocks(ns, f, cr);
        if (ns->fills[f].child >= 0)
            r_convert(ns, ns->fills[f].child, cr);
    }
}

static int arange_cmp(const void *a, const void *b) {
    const arange *x = a, *y = b;
    if (x->start != y->start)
        return x->start < y->start ? -1 : 1;
    return (x->end > y->end) - (x->end < y->end);
}

static void region_add_id(region *c, int32_t id) {
    if (id == c->min1 || id == c->min2)
        return;
    if (id < c->min1) {
        c->min2 = c->min1;
        c->min1 = id;
    } else if (id < c->min2) {
        c->min2 = id;
    }
}

/* genomeRangeTreeAddValList / rangeTreeAddVal (kent rangeTree.c) merge a new
 * range with every stored range it overlaps under rangeCmp (a.end <= b.start
 * orders a first, b.end <= a.start orders it after, anything else merges),
 * concatenating the value lists.  The final tree therefore holds the unions
 * of the non-empty ranges connected by strict overlap (touching ranges stay
 * apart) -- independent of insertion order -- and an empty range [x,x) is
 * merged into the union that holds x strictly inside, or stays on its own.
 * Each region keeps the two smallest chain ids merged into it, which is all
 * isBrokenByAnotherHigherScoringChain asks of the value list. */
static void build_regions(chromregions *cr) {
    qsort(cr->r, (size_t)cr->n, sizeof(arange), arange_cmp);
    cr->c = malloc((size_t)(cr->n ? cr->n : 1) * sizeof(region));
    cr->nc = 0;
    for (int64_t i = 0; i < cr->n; ++i) {
        const arange a = cr->r[i];
        if (a.start == a.end)
            continue;
        if (cr->nc > 0 && a.start < cr->c[cr->nc - 1].end) {
            region *c = &cr->c[cr->nc - 1];
            if (a.end > c->end)
                c->end = a.end;
            region_add_id(c, a.chain_id);
        } else {
            region *c = &cr->c[cr->nc++];
            *c = (region){a.start, a.end, INT32_MAX, INT32_MAX};
            region_add_id(c, a.chain_id);
        }
    }
    cr->nnz = cr->nc;
    for (int64_t i = 0; i < cr->n; ++i) {
        const arange a = cr->r[i];
        if (a.start != a.end)
            continue;
        const int32_t x = a.start;
        int64_t lo = 0, hi = cr->nnz;
        while (lo < hi) { /* first union with end > x */
            const int64_t mid = (lo + hi) / 2;
            if (cr->c[mid].end > x)
                hi = mid;
            else
                lo = mid + 1;
        }
        if (lo < cr->nnz && cr->c[lo].start < x) {
            region_add_id(&cr->c[lo], a.chain_id);
            continue;
        }
        /* on its own; equal empty ranges are kept as one region holding all
         * their ids (the same answer for the overlap test); sorted input
         * puts equal empty ranges next to each other */
        if (cr->nc > cr->nnz && cr->c[cr->nc - 1].start == x) {
            region_add_id(&cr->c[cr->nc - 1], a.chain_id);
            continue;
        }
        region *c = &cr->c[cr->nc++];
        *c = (region){x, x, INT32_MAX, INT32_MAX};
        region_add_id(c, a.chain_id);
    }
    free(cr->r);
    cr->r = NULL;
    cr->n = cr->cap = 0;
}

/* rangeCmp(region, [s, e)) == 0 */
static int overlaps(int32_t rs, int32_t re, int32_t s, int32_t e) { return !(re <= s) && !(e <= rs); }

static int has_higher(const region *c, int32_t chain_id, int32_t parent) {
    return (c->min1 < chain_id && c->min1 != parent) || (c->min2 < chain_id && c->min2 != parent);
}

/* isBrokenByAnotherHigherScoringChain (:868-890) */
static int broken_by_higher(const chromregions *cr, int32_t s, int32_t e, int32_t chain_id,
                            int32_t parent) {
    int64_t lo = 0, hi = cr->nnz;
    while (lo < hi) {
        const int64_t mid = (lo + hi) / 2;
        if (cr->c[mid].end > s)
            hi = mid;
        else
            lo = mid + 1;
    }
    for (int64_t k = lo; k < cr->nnz && cr->c[k].start <= e; ++k)
        if (overlaps(cr->c[k].start, cr->c[k].end, s, e) && has_higher(&cr->c[k], chain_id, parent))
            return 1;
    for (int64_t k = cr->nnz; k < cr->nc; ++k)
        if (overlaps(cr->c[k].start, cr->c[k].end, s, e) && has_higher(&cr->c[k], chain_id, parent))
            return 1;
    return 0;
}

/* ================================================================ breaks */
typedef struct cbrk { /* struct breakInfo */
    int32_t depth, chain_id, parent_id, chrom;
    int32_t Lfs, Lfe, Rfs, Rfe; /* left / right fill of the broken chain */
    int32_t Lgs, Lge, Rgs, Rge; /* left / right gap of the breaking chain */
    int32_t ss, se;             /* suspect */
    int32_t next, prev;         /* indices into g_brk, -1 = NULL */
} cbrk;

static cbrk *g_brk = NULL;
static int64_t g_nbrk = 0, g_brkcap = 0;

/* newBreak (:913-946) */
static int32_t new_break(int32_t depth, int32_t chain_id, int32_t parent_id, int32_t chrom,
                         int32_t Lfs, int32_t Lfe, int32_t Rfs, int32_t Rfe, int32_t Lgs,
                         int32_t Lge, int32_t Rgs, int32_t Rge) {
    GROWV(g_brk, g_brkcap, g_nbrk);
    cbrk *b = &g_brk[g_nbrk];
    *b = (cbrk){depth, chain_id, parent_id, chrom, Lfs, Lfe, Rfs, Rfe,
                Lgs, Lge, Rgs, Rge, Lge, Rgs, -1, -1};
    must_assert(b->ss < b->se, "breakP->suspectStart < breakP->suspectEnd");
    must_assert(b->Lfs < b->ss, "breakP->LfillStart < breakP->suspectStart");
    must_assert(b->Lfe <= b->ss, "breakP->LfillEnd <= breakP->suspectStart");
    must_assert(b->Rfs >= b->se, "breakP->RfillStart >= breakP->suspectEnd");
    must_assert(b->Rfe > b->se, "breakP->RfillEnd > breakP->suspectEnd");
    return (int32_t)g_nbrk++;
}

/* isValidBreakPair (:1408-1450) */
static int valid_pair(const cbrk *u, const cbrk *d) {
    if (u->parent_id != d->parent_id || u->chain_id != d->chain_id)
        return 0;
    if (u->depth != d->depth)
        return 0;
    if (d->ss - u->se > maxPairDistance)
        return 0;
    return u->Rgs == d->Lgs && u->Rge == d->Lge;
}

/* ================================================================ chains of interest */
typedef struct ichain {
    int64_t ci;       /* index in the input chain file */
    double score;     /* chain->score (getChainScore overwrites it for whole-chain subsets) */
    int32_t *bt, *bq, *bs; /* current blocks */
    int32_t nb;
    int32_t version;  /* bumped by every chainRemoveBlocks */
    int rescore;      /* in chainId2NeedsRescoring */
    /* the blocks removed so far, ascending in t (disjoint: tEnd ascends too):
     * a sub-chain has its original content unless one of them is in it */
    int32_t *rm_s, *rm_e;
    int32_t rm_n, rm_cap;
} ichain;

typedef struct state {
    gt_chains c;
    ichain *ich;
    int32_t nich, ichcap;
    gt_khash id2ich;  /* chainId2chain */
    int32_t *id2ich_val;
    gac_ctx *ctx;
    gac_chainset *cs_base; /* every chain of interest as read (version 0) */
    int32_t *t_seq, *q_seq;
    uint8_t *strand;
} state;

static int32_t ich_of(const state *S, int32_t id) {
    const int32_t e = gt_khash_find(&S->id2ich, id);
    return e < 0 ? -1 : S->id2ich_val[e];
}

/* ---- chainSubsetOnT / chainFastSubsetOnT (kent/src/lib/chain.c:471-558) */
typedef struct subchain {
    int easy;               /* the range covers the chain: the chain itself */
    int32_t b0, nb;         /* selected blocks [b0, b0 + nb) */
    int32_t ts, te, qs, qe; /* bounds of the clipped blocks (not easy) */
} subchain;

static subchain subset_of(const int32_t *bt, const int32_t *bq, const int32_t *bs, int32_t nb,
                          int32_t ctstart, int32_t ctend, int32_t s, int32_t e) {
    subchain r;
    memset(&r, 0, sizeof(r));
    if (s <= ctstart && e >= ctend) {
        r.easy = 1;
        r.nb = nb;
        return r;
    }
    int32_t lo = 0, hi = nb; /* first block with tEnd > s */
    while (lo < hi) {
        const int32_t mid = (lo + hi) / 2;
        if (bt[mid] + bs[mid] > s)
            hi = mid;
        else
            lo = mid + 1;
    }
    r.b0 = lo;
    int32_t l2 = lo;
    hi = nb; /* first block with tStart >= e */
    while (l2 < hi) {
        const int32_t mid = (l2 + hi) / 2;
        if (bt[mid] >= e)
            hi = mid;
        else
            l2 = mid + 1;
    }
    r.nb = l2 - lo;
    if (r.nb > 0) {
        const int32_t f = r.b0, l = r.b0 + r.nb - 1;
        r.ts = bt[f] < s ? s : bt[f];
        r.qs = bq[f] + (bt[f] < s ? s - bt[f] : 0);
        r.te = bt[l] + bs[l] > e ? e : bt[l] + bs[l];
        r.qe = bq[l] + bs[l] - (bt[l] + bs[l] > e ? bt[l] + bs[l] - e : 0);
    }
    return r;
}

static subchain subset(const state *S, int32_t ix, int32_t s, int32_t e) {
    const ichain *x = &S->ich[ix];
    return subset_of(x->bt, x->bq, x->bs, x->nb, S->c.tstart[x->ci], S->c.tend[x->ci], s, e);
}

/* clipped block arrays of a (not easy) sub-chain of [s, e) */
static void clip_blocks(const ichain *x, const subchain *sc, int32_t s, int32_t e, int32_t **pbt,
                        int32_t **pbq, int32_t **pbs) {
    const size_t n = (size_t)(sc->nb ? sc->nb : 1);
    int32_t *bt = malloc(n * 4), *bq = malloc(n * 4), *bs = malloc(n * 4);
    for (int32_t k = 0; k < sc->nb; ++k) {
        const int32_t b = sc->b0 + k;
        int32_t ts = x->bt[b], qs = x->bq[b], te = x->bt[b] + x->bs[b];
        if (ts < s) {
            qs += s - ts;
            ts = s;
        }
        if (te > e)
            te = e;
        bt[k] = ts;
        bq[k] = qs;
        bs[k] = te - ts;
    }
    *pbt = bt;
    *pbq = bq;
    *pbs = bs;
}

static int32_t *dup_i32(const int32_t *p, int32_t n) {
    int32_t *r = malloc((size_t)(n ? n : 1) * 4);
    memcpy(r, p, (size_t)n * 4);
    return r;
}

/* chainWrite of a sub-chain (the chain itself in the easy case) */
static void write_subchain(FILE *f, const state *S, int32_t ix, const subchain *sc, int32_t s,
                           int32_t e, double score, int32_t id) {
    const ichain *x = &S->ich[ix];
    const gt_chains *c = &S->c;
    const int64_t ci = x->ci;
    const char *tn = c->tnames.names[c->tname[ci]], *qn = c->qnames.names[c->qname[ci]];
    if (sc->easy) {
        gt_write_chain_raw(f, score, tn, c->tsize[ci], c->tstart[ci], c->tend[ci], qn,
                           c->qsize[ci], c->qstrand[ci], c->qstart[ci], c->qend[ci], id, x->bt,
                           x->bq, x->bs, x->nb);
        return;
    }
    int32_t *bt, *bq, *bs;
    clip_blocks(x, sc, s, e, &bt, &bq, &bs);
    gt_write_chain_raw(f, score, tn, c->tsize[ci], sc->ts, sc->te, qn, c->qsize[ci],
                       c->qstrand[ci], sc->qs, sc->qe, id, bt, bq, bs, sc->nb);
    free(bt);
    free(bq);
    free(bs);
}

/* ================================================================ GPU scores
 * Cached by (chain, content version, s, e).  A range of a chain that lost
 * blocks selects the original blocks minus the removed ones inside it; the
 * content version is their count (0: the original selection). */
typedef struct sres {
    int64_t g, l;
    int32_t ali;
} sres;

typedef struct qkey {
    int32_t ich, version, s, e;
} qkey;

static qkey *g_ck = NULL;
static sres *g_cv = NULL;
static uint8_t *g_cused = NULL;
static int64_t g_cslots = 0, g_cn = 0;
static int64_t g_gpu_calls = 0, g_gpu_ranges = 0, g_uploads = 0;
static int64_t g_host_chains = 0, g_host_blocks = 0; /* (modified chains' blocks handed over) */
/* GAC_CLEANER_SPEC=0: no speculative keys, no prefetch at a list's first
 * pass (round 5's batching); GAC_CLEANER_LOOKAHEAD=n: n lists per first-pass
 * batch (C3, profiles/r06c3b: 1 list 3208 calls, 8 lists 3672, 32 lists
 * 4141 -- keys of later lists go stale as the lists before them modify
 * chains) */
static int g_spec = 1;
static int g_check_keys = 0;             /* GAC_CLEANER_CHECK_KEYS=1 (tests) */
static int g_lookahead = 1;             /* lists whose keys one first-pass batch holds */
static int64_t g_miss[4][2];            /* test-time misses by key (S F L R) x (original, modified) */
static double g_t_remove = 0, g_t_keys = 0; /* (timing: block removal, key making) */
static int64_t g_calls_site[3];         /* scoring calls: list batches, later passes, tests */
static int g_site = 2;
static double g_gpu_s = 0; /* wall time inside the scoring calls */

static double wall_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static uint64_t key_hash(qkey k) {
    uint64_t h = (uint64_t)(uint32_t)k.ich * 0x9E3779B97F4A7C15ull;
    h ^= (uint64_t)(uint32_t)k.version * 0xC2B2AE3D27D4EB4Full;
    h ^= ((uint64_t)(uint32_t)k.s << 32 | (uint32_t)k.e) * 0x165667B19E3779F9ull;
    return h ^ (h >> 29);
}

static int key_eq(qkey a, qkey b) {
    return a.ich == b.ich && a.version == b.version && a.s == b.s && a.e == b.e;
}

static void cache_put(qkey k, sres v);

static void cache_grow(void) {
    const int64_t old = g_cslots;
    qkey *ok = g_ck;
    sres *ov = g_cv;
    uint8_t *ou = g_cused;
    g_cslots = old ? old * 2 : 4096;
    g_ck = malloc((size_t)g_cslots * sizeof(qkey));
    g_cv = malloc((size_t)g_cslots * sizeof(sres));
    g_cused = calloc((size_t)g_cslots, 1);
    g_cn = 0;
    for (int64_t i = 0; i < old; ++i)
        if (ou[i])
            cache_put(ok[i], ov[i]);
    free(ok);
    free(ov);
    free(ou);
}

static void cache_put(qkey k, sres v) {
    if ((g_cn + 1) * 2 > g_cslots)
        cache_grow();
    uint64_t h = key_hash(k) & (uint64_t)(g_cslots - 1);
    while (g_cused[h] && !key_eq(g_ck[h], k))
        h = (h + 1) & (uint64_t)(g_cslots - 1);
    if (!g_cused[h])
        ++g_cn;
    g_cused[h] = 1;
    g_ck[h] = k;
    g_cv[h] = v;
}

static const sres *cache_get(qkey k) {
    if (!g_cslots)
        return NULL;
    uint64_t h = key_hash(k) & (uint64_t)(g_cslots - 1);
    while (g_cused[h]) {
        if (key_eq(g_ck[h], k))
            return &g_cv[h];
        h = (h + 1) & (uint64_t)(g_cslots - 1);
    }
    return NULL;
}

/* cur: the current subset of [s, e) when the caller has it, else NULL */
static qkey make_key_cur(const state *S, int32_t ix, int32_t s, int32_t e, const subchain *pc) {
    const ichain *x = &S->ich[ix];
    int32_t ver = 0;
    if (x->rm_n) {
        const int64_t ci = x->ci;
        /* the key's version is the number of removed blocks the selection
         * would hold: blocks only ever go, so the current selection is the
         * original one minus those, and equal counts at two times mean the
         * same blocks (a key stays valid across removals elsewhere in the
         * chain).  A whole-chain selection (chainSubsetOnT's easy case, the
         * original bounds) holds every removed block; else those with
         * tEnd > s and tStart < e (the removed list is sorted and disjoint) */
        if (s <= S->c.tstart[ci] && e >= S->c.tend[ci]) {
            ver = x->rm_n;
        } else {
            int32_t lo = 0, hi = x->rm_n; /* first removed block with tEnd > s */
            while (lo < hi) {
                const int32_t m = (lo + hi) >> 1;
                if (x->rm_e[m] > s)
                    hi = m;
                else
                    lo = m + 1;
            }
            int32_t l2 = lo, h2 = x->rm_n; /* first from there with tStart >= e */
            while (l2 < h2) {
                const int32_t m = (l2 + h2) >> 1;
                if (x->rm_s[m] >= e)
                    h2 = m;
                else
                    l2 = m + 1;
            }
            ver = l2 - lo;
        }
        if (g_check_keys) { /* (test hook: the rule as counts of the two selections) */
            const subchain cur = pc ? *pc : subset(S, ix, s, e);
            const int64_t b0 = S->c.blk_off[ci];
            const subchain org = subset_of(S->c.bt + b0, S->c.bq + b0, S->c.bs + b0,
                                           (int32_t)(S->c.blk_off[ci + 1] - b0), S->c.tstart[ci],
                                           S->c.tend[ci], s, e);
            if ((cur.easy ? x->rm_n : org.nb - cur.nb) != ver) {
                for (int32_t k = 0; k < x->rm_n; ++k)
                    if (x->rm_e[k] > s - 1000 && x->rm_s[k] < e + 1000)
                        fprintf(stderr, "removed[%d] = [%d, %d)\n", k, x->rm_s[k], x->rm_e[k]);
                for (int32_t k = 0; k < org.nb; ++k)
                    fprintf(stderr, "org block %d: [%d, %d)\n", org.b0 + k, S->c.bt[b0 + org.b0 + k],
                            S->c.bt[b0 + org.b0 + k] + S->c.bs[b0 + org.b0 + k]);
                fprintf(stderr, "rm_n %d sorted check:", x->rm_n);
                for (int32_t k = 1; k < x->rm_n; ++k)
                    if (x->rm_s[k] < x->rm_e[k - 1]) fprintf(stderr, " bad@%d [%d,%d) [%d,%d)", k, x->rm_s[k-1], x->rm_e[k-1], x->rm_s[k], x->rm_e[k]);
                fprintf(stderr, "\n");
                gt_abort("key version rule: chain %d [%d, %d): counts %d/%d, easy %d, version %d\n",
                         (int)S->c.id[ci], s, e, cur.nb, org.nb, cur.easy, ver);
            }
        }
    }
    return (qkey){ix, ver, s, e};
}

static qkey make_key(const state *S, int32_t ix, int32_t s, int32_t e) {
    return make_key_cur(S, ix, s, e, NULL);
}

static int qkey_cmp(const void *a, const void *b) {
    const qkey *x = a, *y = b;
    if ((x->version != 0) != (y->version != 0))
        return x->version == 0 ? -1 : 1;
    if (x->ich != y->ich)
        return x->ich < y->ich ? -1 : 1;
    if (x->s != y->s)
        return x->s < y->s ? -1 : 1;
    return (x->e > y->e) - (x->e < y->e);
}

/* Score every key not cached yet: original-content keys against the chain
 * set uploaded at start, the rest against one upload of the current block
 * lists of the chains involved.  At most two GPU calls. */
static void score_keys(state *S, const qkey *in, int64_t n) {
    qkey *q = malloc((size_t)(n ? n : 1) * sizeof(qkey));
    int64_t m = 0;
    for (int64_t i = 0; i < n; ++i)
        if (!cache_get(in[i]))
            q[m++] = in[i];
    if (m == 0) {
        free(q);
        return;
    }
    qsort(q, (size_t)m, sizeof(qkey), qkey_cmp);
    int64_t u = 0;
    for (int64_t i = 0; i < m; ++i)
        if (u == 0 || !key_eq(q[u - 1], q[i]))
            q[u++] = q[i];
    m = u;
    gac_range *rb = malloc((size_t)m * sizeof(gac_range));
    int64_t *g = malloc((size_t)m * 8), *l = malloc((size_t)m * 8);
    int32_t *a = malloc((size_t)m * 4);
    int64_t n0 = 0;
    while (n0 < m && q[n0].version == 0) {
        rb[n0] = (gac_range){q[n0].ich, q[n0].s, q[n0].e};
        ++n0;
    }
    const double t0 = wall_s();
    ++g_calls_site[g_site];
    if (n0) {
        gt_check(gac_score_ranges(S->ctx, S->cs_base, rb, n0, GAC_WANT_LOCAL, g, l, a));
        ++g_gpu_calls;
        g_gpu_ranges += n0;
    }
    if (m > n0) {
        /* modified chains (keys sorted by chain): one set of their current blocks */
        int32_t *sel = malloc((size_t)(m - n0) * 4);
        int32_t ns = 0;
        int64_t nbk = 0;
        for (int64_t i = n0; i < m; ++i) {
            must_assert(q[i].version == make_key(S, q[i].ich, q[i].s, q[i].e).version,
                        "key of the current blocks");
            if (ns == 0 || sel[ns - 1] != q[i].ich) {
                sel[ns++] = q[i].ich;
                nbk += S->ich[q[i].ich].nb;
            }
            rb[i] = (gac_range){ns - 1, q[i].s, q[i].e};
        }
        int64_t *off = malloc((size_t)(ns + 1) * 8);
        int32_t *ts = malloc((size_t)ns * 4), *qs = malloc((size_t)ns * 4);
        uint8_t *st = malloc((size_t)ns);
        /* one chain (the usual case: 6.7 k hand-overs of 16 k blocks each on
         * C3): its own block arrays, no copy; several: copied back to back */
        const int one = ns == 1;
        const size_t nbb = (size_t)(nbk && !one ? nbk : 1);
        int32_t *bt = one ? NULL : malloc(nbb * 4), *bq = one ? NULL : malloc(nbb * 4),
                *bs = one ? NULL : malloc(nbb * 4);
        off[0] = 0;
        g_host_chains += ns;
        g_host_blocks += nbk;
        for (int32_t k = 0; k < ns; ++k) {
            const ichain *x = &S->ich[sel[k]];
            ts[k] = S->t_seq[sel[k]];
            qs[k] = S->q_seq[sel[k]];
            st[k] = S->strand[sel[k]];
            if (!one) {
                memcpy(bt + off[k], x->bt, (size_t)x->nb * 4);
                memcpy(bq + off[k], x->bq, (size_t)x->nb * 4);
                memcpy(bs + off[k], x->bs, (size_t)x->nb * 4);
            }
            off[k + 1] = off[k] + x->nb;
        }
        const ichain *x0 = &S->ich[sel[0]];
        gac_chainset_desc d = {ns, ts, qs, st, off, nbk, one ? x0->bt : bt, one ? x0->bq : bq,
                               one ? x0->bs : bs};
        /* the modified chains' current blocks stay on the host: their
         * windows are read by the kernel over the bus (no upload) */
        ++g_uploads;
        gt_check(gac_score_ranges_host(S->ctx, &d, rb + n0, m - n0, GAC_WANT_LOCAL, g + n0,
                                       l + n0, a + n0));
        ++g_gpu_calls;
        g_gpu_ranges += m - n0;
        free(sel);
        free(off);
        free(ts);
        free(qs);
        free(st);
        free(bt);
        free(bq);
        free(bs);
    }
    g_gpu_s += wall_s() - t0;
    for (int64_t i = 0; i < m; ++i)
        cache_put(q[i], (sres){g[i], l[i], a[i]});
    free(rb);
    free(g);
    free(l);
    free(a);
    free(q);
}

/* the four sub-chains testAndRemoveSuspect scores for a break */
static int break_keys(const state *S, const cbrk *b, qkey *out) {
    const int32_t ib = ich_of(S, b->parent_id), ik = ich_of(S, b->chain_id);
    if (ib < 0 || ik < 0)
        return 0;
    out[0] = make_key(S, ib, b->ss, b->se);
    out[1] = make_key(S, ik, b->Lfs, b->Rfe);
    out[2] = make_key(S, ik, b->Lfs, b->se);
    out[3] = make_key(S, ik, b->ss, b->Rfe);
    return 4;
}

/* Speculative keys of break x (prev: its upstream neighbour): when the
 * breaks before it are removed, test_and_remove hands each removed suspect's
 * left fill to its downstream neighbour (d->Lfs = b->Lfs when d's left fill
 * is b's right fill, cascading down a run of such links), so x is then
 * tested with its fill starting at an upstream break's Lfs.  Those keys
 * (the fill and the left fill; the suspect and the right fill keep theirs)
 * for up to kSpecDepth removed predecessors, scored in the pass's batch
 * instead of one call per removal (chainCleaner.c:1191-1398's update of the
 * neighbours, 1452-1631's loop). */
enum { kSpecDepth = 3 };

static int spec_keys(const state *S, int32_t x, qkey *out) {
    int n = 0;
    const cbrk *cur = &g_brk[x];
    const int32_t ik = ich_of(S, cur->chain_id);
    if (ik < 0)
        return 0;
    const int32_t rfe = g_brk[x].Rfe, se = g_brk[x].se;
    for (int32_t p = g_brk[x].prev, k = 0; p >= 0 && k < kSpecDepth; ++k) {
        const cbrk *P = &g_brk[p];
        if (!(P->chain_id == cur->chain_id && P->parent_id == cur->parent_id && cur->Lfs == P->Rfs &&
              cur->Lfe == P->Rfe))
            break;
        out[n++] = make_key(S, ik, P->Lfs, rfe);
        out[n++] = make_key(S, ik, P->Lfs, se);
        cur = P;
        p = P->prev;
    }
    return n;
}

/* keys of every break of a list (singles, with their speculative keys) and
 * of its valid adjacent pairs */
static void list_keys(const state *S, int32_t head, int pairs, int singles, qkey **q, int64_t *n,
                      int64_t *cap) {
    for (int32_t b = head; b >= 0; b = g_brk[b].next) {
        if (*n + 8 + 2 * kSpecDepth > *cap) {
            *cap = *cap ? *cap * 2 : 1024;
            *q = realloc(*q, (size_t)*cap * sizeof(qkey));
        }
        if (singles) {
            *n += break_keys(S, &g_brk[b], *q + *n);
            if (g_spec)
                *n += spec_keys(S, b, *q + *n);
        }
        const int32_t d = g_brk[b].next;
        if (pairs && d >= 0 && valid_pair(&g_brk[b], &g_brk[d])) {
            cbrk p = g_brk[b]; /* newBreakPair without the list / asserts */
            p.Rfs = g_brk[d].Rfs;
            p.Rfe = g_brk[d].Rfe;
            p.Rgs = g_brk[d].Rgs;
            p.Rge = g_brk[d].Rge;
            p.se = g_brk[d].Rgs;
            *n += break_keys(S, &p, *q + *n);
        }
    }
}

static void prefetch_list(state *S, int32_t head, int pairs, int singles) {
    qkey *q = NULL;
    int64_t n = 0, cap = 0;
    list_keys(S, head, pairs, singles, &q, &n, &cap);
    score_keys(S, q, n);
    free(q);
}

/* ================================================================ output chains */
typedef struct outchain {
    double score;
    int64_t from; /* input chain written unchanged, or -1 */
    int32_t tname, tsize, tstart, tend, qname, qsize, qstart, qend, id;
    int qminus;
    int32_t *bt, *bq, *bs;
    int32_t nb;
} outchain;

static outchain *g_out = NULL;
static int64_t g_nout = 0, g_outcap = 0;

static void out_push(const outchain *o) {
    GROWV(g_out, g_outcap, g_nout);
    g_out[g_nout++] = *o;
}

static outchain out_of_ichain(const state *S, const ichain *x, double score, int32_t id) {
    const int64_t ci = x->ci;
    outchain o;
    memset(&o, 0, sizeof(o));
    o.score = score;
    o.from = -1;
    o.tname = S->c.tname[ci];
    o.tsize = S->c.tsize[ci];
    o.tstart = S->c.tstart[ci];
    o.tend = S->c.tend[ci];
    o.qname = S->c.qname[ci];
    o.qsize = S->c.qsize[ci];
    o.qminus = S->c.qstrand[ci];
    o.qstart = S->c.qstart[ci];
    o.qend = S->c.qend[ci];
    o.id = id;
    o.bt = x->bt;
    o.bq = x->bq;
    o.bs = x->bs;
    o.nb = x->nb;
    return o;
}

/* ================================================================ the cleaning loop */
static FILE *g_bed = NULL, *g_dict = NULL, *g_sdata = NULL;
static FILE *g_dbg_susp = NULL, *g_dbg_L = NULL, *g_dbg_R = NULL, *g_dbg_F = NULL,
            *g_dbg_bed = NULL;
static int32_t g_max_chain_id = -1;
static int g_suspect_id = 0;

/* chainRemoveBlocks (:649-686) */
static void remove_blocks(state *S, int32_t ix, int32_t ts, int32_t te) {
    ichain *x = &S->ich[ix];
    const int32_t id = S->c.id[x->ci];
    int32_t first = 0, cur;
    for (cur = 0; cur < x->nb; ++cur) {
        if (x->bt[cur] >= ts)
            break;
        first = cur;
    }
    if (cur == first)
        gt_abort("ERROR in chainRemoveBlocks: boundaries imply that we remove the first block of chain Id %d (tStart %d - tEnd %d)\n",
                 id, ts, te);
    for (cur = first + 1; cur < x->nb; ++cur)
        if (x->bt[cur] >= te)
            break;
    if (cur >= x->nb)
        gt_abort("ERROR in chainRemoveBlocks: boundaries imply that we remove the last block of chain Id %d (tStart %d - tEnd %d)\n",
                 id, ts, te);
    const int32_t last = cur;
    /* the reference frees firstBlock->next up to lastBlock; with no block in
     * between it would run past lastBlock -- the suspect's own blocks
     * (tested non-empty before) rule that out */
    must_assert(last > first + 1, "chainRemoveBlocks: blocks between the boundaries");
    const int32_t gone = last - first - 1, tail = x->nb - last;
    /* the removed run into the sorted removed list */
    if (x->rm_n + gone > x->rm_cap) {
        x->rm_cap = 2 * (x->rm_n + gone) + 16;
        x->rm_s = realloc(x->rm_s, (size_t)x->rm_cap * 4);
        x->rm_e = realloc(x->rm_e, (size_t)x->rm_cap * 4);
    }
    {
        /* merged from the back (the run may straddle blocks removed before:
         * they lay between its blocks in the chain) */
        int32_t i = x->rm_n - 1, j = gone - 1, o = x->rm_n + gone - 1;
        while (j >= 0) {
            const int32_t js = x->bt[first + 1 + j];
            if (i >= 0 && x->rm_s[i] > js) {
                x->rm_s[o] = x->rm_s[i];
                x->rm_e[o--] = x->rm_e[i--];
            } else {
                x->rm_s[o] = js;
                x->rm_e[o--] = js + x->bs[first + 1 + j--];
            }
        }
        x->rm_n += gone;
    }
    memmove(x->bt + first + 1, x->bt + last, (size_t)tail * 4);
    memmove(x->bq + first + 1, x->bq + last, (size_t)tail * 4);
    memmove(x->bs + first + 1, x->bs + last, (size_t)tail * 4);
    x->nb -= gone;
    ++x->version;
}

/* testAndRemoveSuspect (:1191-1398) */
static int test_and_remove(state *S, cbrk *b, int32_t up, int32_t down, int *updated,
                           const char *dbg, int is_pair) {
    *updated = 0;
    const int32_t ib = ich_of(S, b->parent_id);
    if (ib < 0)
        gt_abort("ERROR: cannot get breaking chain with Id %d from chainId2chain hash\n",
                 b->parent_id);
    const double breaking_score = S->ich[ib].score;
    const int32_t ik = ich_of(S, b->chain_id);
    if (ik < 0)
        gt_abort("ERROR: cannot get broken chain with Id %d from chainId2chain hash\n",
                 b->chain_id);
    const double broken_score = S->ich[ik].score;

    const subchain sS = subset(S, ib, b->ss, b->se);
    const subchain sF = subset(S, ik, b->Lfs, b->Rfe);
    const subchain sL = subset(S, ik, b->Lfs, b->se);
    const subchain sR = subset(S, ik, b->ss, b->Rfe);
    if (sS.nb == 0) {
        gt_verbose(3, "\t\tSuspect %d-%d is apparently already deleted as the suspect subChain is NULL\n",
                   b->ss, b->se);
        return 0;
    }
    if (sF.nb == 0 || sL.nb == 0 || sR.nb == 0)
        gt_abort("ERROR: broken chain %d has no block in its fill %d-%d (suspect %d-%d)\n",
                 b->chain_id, b->Lfs, b->Rfe, b->ss, b->se);
    qkey k[4];
    const double tk0 = wall_s();
    /* break_keys with the subsets just taken */
    k[0] = make_key_cur(S, ib, b->ss, b->se, &sS);
    k[1] = make_key_cur(S, ik, b->Lfs, b->Rfe, &sF);
    k[2] = make_key_cur(S, ik, b->Lfs, b->se, &sL);
    k[3] = make_key_cur(S, ik, b->ss, b->Rfe, &sR);
    g_t_keys += wall_s() - tk0;
    for (int j = 0; j < 4; ++j)
        if (!cache_get(k[j]))
            ++g_miss[j][k[j].version != 0];
    score_keys(S, k, 4);
    const sres rS = *cache_get(k[0]), rF = *cache_get(k[1]), rL = *cache_get(k[2]),
               rR = *cache_get(k[3]);
    /* getChainScore sets sub->score = global; a whole-chain subset is the
     * chain, whose score is overwritten (in the reference's call order) */
    const double gS = (double)rS.g, gF = (double)rF.g, gL = (double)rL.g, gR = (double)rR.g;
    if (sS.easy)
        S->ich[ib].score = gS;
    if (sF.easy)
        S->ich[ik].score = gF;
    if (sL.easy)
        S->ich[ik].score = gL;
    if (sR.easy)
        S->ich[ik].score = gR;
    const double localS = (double)rS.l, localF = (double)rF.l, localL = (double)rL.l,
                 localR = (double)rR.l;
    const double ratio = gF / localS, ratioL = gL / localS, ratioR = gR / localS;
    const int suspect_bases = rS.ali;

    gt_verbose(3, "\t\t\tsuspect subChain            %d - %d   gets score %7d   (local score %d, suspect subChain bases %d, left gap size %d, right gap size %d)\n",
               b->ss, b->se, (int)gS, (int)localS, suspect_bases, b->Lge - b->Lgs, b->Rge - b->Rgs);
    gt_verbose(3, "\t\t\tleft-to-right fill subChain %d - %d   gets score %7d   (local %7d)  ratio %1.2f\n",
               b->Lfs, b->Rfe, (int)gF, (int)localF, ratio);
    gt_verbose(3, "\t\t\tleft fill subChain          %d - %d   gets score %7d   (local %7d)  ratio %1.2f\n",
               b->Lfs, b->Lfe, (int)gL, (int)localL, ratioL);
    gt_verbose(3, "\t\t\tright fill subChain         %d - %d   gets score %7d   (local %7d)  ratio %1.2f\n",
               b->Rfs, b->Rfe, (int)gR, (int)localR, ratioR);

    const double lr = is_pair ? LRfoldThresholdPairs : LRfoldThreshold;
    int removed = ratioL >= lr && ratioR >= lr && ratio >= foldThreshold &&
                  localS <= maxSuspectScore && suspect_bases <= maxSuspectBases &&
                  broken_score >= minBrokenChainScore && (b->Lge - b->Lgs) >= minLRGapSize &&
                  (b->Rge - b->Rgs) >= minLRGapSize;

    if (g_sdata) {
        removed = 0;
        ++g_suspect_id;
        fprintf(g_sdata, "%s\t%d\t%d\t%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d,%d\n",
                chrom_name(b->chrom), b->ss, b->se, g_suspect_id, b->parent_id,
                (int)breaking_score, b->chain_id, (int)broken_score, (int)localS, (int)gF, (int)gL,
                (int)gR, suspect_bases, b->Lge - b->Lgs, b->Rge - b->Rgs, (int)localL,
                (int)localR);
    }
    if (debug) {
        const int32_t idb = S->c.id[S->ich[ib].ci], idk = S->c.id[S->ich[ik].ci];
        write_subchain(g_dbg_susp, S, ib, &sS, b->ss, b->se, gS, idb);
        write_subchain(g_dbg_L, S, ik, &sL, b->Lfs, b->se, gL, idk);
        write_subchain(g_dbg_R, S, ik, &sR, b->ss, b->Rfe, gR, idk);
        write_subchain(g_dbg_F, S, ik, &sF, b->Lfs, b->Rfe, gF, idk);
        fprintf(g_dbg_bed,
                "%s\t%d\t%d\t%s%sSuspect__score_%1.0f__Rleft_%1.2f__Rright_%1.2f\t1000\t+\t%d\t%d\t255,0,0\n",
                chrom_name(b->chrom), b->ss, b->se, removed ? "REMOVED_" : "", dbg, localS, ratioL,
                ratioR, b->ss, b->se);
        fprintf(g_dbg_bed, "%s\t%d\t%d\t%sFill__score_%1.0f\t1000\t+\t%d\t%d\t0,0,255\n",
                chrom_name(b->chrom), b->Lfs, b->Rfe, dbg, gF, b->Lfs, b->Rfe);
        fprintf(g_dbg_bed, "%s\t%d\t%d\t%sLfill__score_%1.0f\t1000\t+\t%d\t%d\t0,125,255\n",
                chrom_name(b->chrom), b->Lfs, b->se, dbg, gL, b->Lfs, b->Lfe);
        fprintf(g_dbg_bed, "%s\t%d\t%d\t%sRfill__score_%1.0f\t1000\t+\t%d\t%d\t0,125,255\n",
                chrom_name(b->chrom), b->ss, b->Rfe, dbg, gR, b->Rfs, b->Rfe);
    }
    if (!removed) {
        gt_verbose(3, "\t\t\t===> do not remove suspect from breaking chainID %d\n",
                   S->c.id[S->ich[ib].ci]);
        return 0;
    }
    ichain *x = &S->ich[ib];
    x->rescore = 1;
    gt_verbose(3, "\t\t\t===> REMOVE suspect from breaking chainID %d (this chain will be rescored before writing)\n",
               S->c.id[x->ci]);
    fprintf(g_bed,
            "%s\t%d\t%d\tbreakingChainID_%d_Score_%d_brokenChainID_%d_Score_%d_suspectLocalScore_%d_RatioL_%1.2f_RatioR_%1.2f\t1000\t+\t%d\t%d\t%s\n",
            chrom_name(b->chrom), b->ss, b->se, b->parent_id, (int)breaking_score, b->chain_id,
            (int)broken_score, (int)localS, ratioL, ratioR, b->ss, b->se,
            is_pair ? "0,100,255" : "0,0,153");
    /* the suspect sub-chain (taken before the removal) becomes a new chain */
    outchain o = out_of_ichain(S, x, gS, 0);
    if (sS.easy) {
        o.bt = dup_i32(x->bt, x->nb);
        o.bq = dup_i32(x->bq, x->nb);
        o.bs = dup_i32(x->bs, x->nb);
    } else {
        clip_blocks(x, &sS, b->ss, b->se, &o.bt, &o.bq, &o.bs);
        o.nb = sS.nb;
        o.tstart = sS.ts;
        o.tend = sS.te;
        o.qstart = sS.qs;
        o.qend = sS.qe;
    }
    const double tr0 = wall_s();
    remove_blocks(S, ib, b->ss, b->se);
    g_t_remove += wall_s() - tr0;
    o.id = ++g_max_chain_id;
    if (g_dict)
        fprintf(g_dict, "%d\t%d\n", o.id, S->c.id[x->ci]);
    out_push(&o);
    gt_verbose(4, "\t\t\twrote new chain representing the removed suspect with ID %d\n", o.id);
    if (up >= 0) {
        cbrk *u = &g_brk[up];
        if (b->chain_id == u->chain_id && b->parent_id == u->parent_id && u->Rfs == b->Lfs &&
            u->Rfe == b->Lfe) {
            *updated = 1;
            must_assert(u->Lfe < b->Lfs, "upstreamBreak->LfillEnd < breakP->LfillStart");
            must_assert(u->se < b->ss, "upstreamBreak->suspectEnd < breakP->suspectStart");
            u->Rfe = b->Rfe;
            u->Rge = b->Rge;
        }
    }
    if (down >= 0) {
        cbrk *d = &g_brk[down];
        if (b->chain_id == d->chain_id && b->parent_id == d->parent_id && d->Lfs == b->Rfs &&
            d->Lfe == b->Rfe) {
            *updated = 1;
            must_assert(d->Rfs > b->Rfe, "downstreamBreak->RfillStart > breakP->RfillEnd");
            must_assert(d->ss > b->se, "downstreamBreak->suspectStart > breakP->suspectEnd");
            d->Lfs = b->Lfs;
            d->Lgs = b->Lgs;
        }
    }
    return 1;
}

/* slRemoveEl on a list of break indices */
static void list_remove(int32_t *head, int32_t b) {
    if (*head == b) {
        *head = g_brk[b].next;
        return;
    }
    for (int32_t p = *head; p >= 0; p = g_brk[p].next)
        if (g_brk[p].next == b) {
            g_brk[p].next = g_brk[b].next;
            return;
        }
    gt_abort("ERROR: cannot remove break from the list: suspect %s:%d-%d\n",
             chrom_name(g_brk[b].chrom), g_brk[b].ss, g_brk[b].se);
}

/* loopOverBreaks (:1452-1631), one breaking chain's list */
static void loop_breaks(state *S, int32_t head) {
    int total = 0, first_pass = 1;
    for (;;) {
        for (;;) {
            ++total;
            /* (a list's first pass was batched with every list's before the
             * loop; chains modified by the lists since then change keys: one
             * call for those too) */
            if (!first_pass) {
                g_site = 1;
                prefetch_list(S, head, 0, 1);
                g_site = 2;
            }
            first_pass = 0;
            int any_single = 0;
            for (int32_t b = head; b >= 0;) {
                char dbg[64];
                snprintf(dbg, sizeof(dbg), "SINGLE_%d", total);
                int upd = 0;
                const int rem =
                    test_and_remove(S, &g_brk[b], g_brk[b].prev, g_brk[b].next, &upd, dbg, 0);
                if (upd)
                    any_single = 1;
                const int32_t nx = g_brk[b].next;
                if (rem) {
                    list_remove(&head, b);
                    if (g_brk[b].next >= 0)
                        g_brk[g_brk[b].next].prev = g_brk[b].prev;
                }
                b = nx;
            }
            if (!any_single || head < 0)
                break;
        }
        int any_pair = 0;
        if (doPairs) {
            ++total;
            g_site = 1;
            prefetch_list(S, head, 1, 0);
            g_site = 2;
            for (int32_t b = head; b >= 0 && g_brk[b].next >= 0;) {
                const int32_t u = b, d = g_brk[b].next, after = g_brk[d].next,
                              before = g_brk[b].prev;
                if (!valid_pair(&g_brk[u], &g_brk[d])) {
                    b = d;
                    continue;
                }
                const cbrk U = g_brk[u], D = g_brk[d];
                const int32_t p = new_break(U.depth, U.chain_id, U.parent_id, U.chrom, U.Lfs, U.Lfe,
                                            D.Rfs, D.Rfe, U.Lgs, U.Lge, D.Rgs, D.Rge);
                char dbg[64];
                snprintf(dbg, sizeof(dbg), "PAIR_%d", total);
                int upd = 0;
                const int rem = test_and_remove(S, &g_brk[p], before, after, &upd, dbg, 1);
                if (rem)
                    gt_verbose(3, "\t\t\t===> PAIR REMOVED\n");
                if (upd)
                    any_pair = 1;
                if (rem) {
                    list_remove(&head, u);
                    list_remove(&head, d);
                    if (after >= 0)
                        g_brk[after].prev = before;
                }
                --g_nbrk; /* the pair break is freed (it is the last one made) */
                b = rem ? after : d;
            }
        }
        if (!any_pair || head < 0)
            break;
    }
}

/* chainSort (chainSort.c:41-75): the chains re-read with slAddHead (reversed)
 * and slSort'ed by chainCmpScore, i.e. glibc's stable merge sort on the score
 * as written ("%1.0f"), descending */
typedef struct sortkey {
    double score;
    int64_t rank;
} sortkey;

static int sortkey_cmp(const void *a, const void *b) {
    const sortkey *x = a, *y = b;
    const double diff = y->score - x->score;
    if (diff < 0.0)
        return -1;
    if (diff > 0.0)
        return 1;
    return (x->rank > y->rank) - (x->rank < y->rank);
}

/* chainNet -minScore=0 in.chain tSizes qSizes stdout /dev/null |
 * NetFilterNonNested.perl /dev/stdin -minScore1 3000 (netInputChains) */
static void net_in_process(const char *in_chain, const char *tsizes, const char *qsizes,
                           gt_lines *out) {
    char tmp[] = "tmp.chainCleaner.XXXXXXX.net";
    const int fd = mkstemps(tmp, 4);
    if (fd < 0)
        gt_abort("ERROR: cannot create a tempfile for netting the chain file\n");
    close(fd);
    gt_verbose(1, "\t\ttempfile for netting: %s\n", tmp);
    gt_sizes ts, qs;
    gt_read_sizes(qsizes, &qs);
    gt_read_sizes(tsizes, &ts);
    gt_chains c;
    gt_read_chains(in_chain, &c, 0.0, 1);
    int32_t *tix = malloc((size_t)(c.n ? c.n : 1) * 4), *qix = malloc((size_t)(c.n ? c.n : 1) * 4);
    double last = -1;
    int bad = 0;
    for (int64_t i = 0; i < c.n && !bad; ++i) {
        if (last >= 0 && c.score[i] > last)
            bad = 1; /* chainNet: must be sorted in order of score */
        last = c.score[i];
        tix[i] = gt_names_find(&ts.names, c.tnames.names[c.tname[i]]);
        qix[i] = gt_names_find(&qs.names, c.qnames.names[c.qname[i]]);
        if (tix[i] < 0 || qix[i] < 0 || ts.size[tix[i]] != c.tsize[i] ||
            qs.size[qix[i]] != c.qsize[i])
            bad = 1;
    }
    if (bad) {
        unlink(tmp);
        gt_abort("ERROR: chainNet | NetFilterNonNested.perl failed. Cannot net the chains. Command: set -o pipefail; chainNet -minScore=0 %s %s %s stdout /dev/null | NetFilterNonNested.perl /dev/stdin -minScore1 3000 > %s\n",
                 in_chain, tsizes, qsizes, tmp);
    }
    gac_net_input in;
    memset(&in, 0, sizeof(in));
    in.n_chains = c.n;
    in.score = c.score;
    in.id = c.id;
    in.t_seq = tix;
    in.q_seq = qix;
    in.q_strand = c.qstrand;
    in.t_start = c.tstart;
    in.t_end = c.tend;
    in.q_start = c.qstart;
    in.q_end = c.qend;
    in.blk_off = c.blk_off;
    in.blk_t = c.bt;
    in.blk_q = c.bq;
    in.blk_size = c.bs;
    in.n_tseq = ts.names.n;
    in.t_names = (const char *const *)ts.names.names;
    in.t_sizes = ts.size;
    in.n_qseq = qs.names.n;
    in.q_names = (const char *const *)qs.names.names;
    in.q_sizes = qs.size;
    const gac_net_opts opt = {25, 12, 0.0, 0}; /* chainNet defaults, -minScore=0 */
    gac_net *net = NULL;
    /* only the target net is used (the query net goes to /dev/null) */
    gt_check(gac_net_build_sides(&in, &opt, 1 << GAC_T, &net));
    gt_check(gac_net_write(net, GAC_T, NULL, tmp, (const char *const *)c.meta, c.n_meta));
    gac_net_free(net);
    gt_lines raw;
    gt_lines_read(tmp, &raw);
    unlink(tmp);
    gt_netfilter_nonnested(&raw, "/dev/stdin", 3000, 0, 0, 0, 0, 0, out);
    gt_lines_free(&raw);
    free(tix);
    free(qix);
    gt_chains_free(&c);
    gt_sizes_free(&ts);
    gt_sizes_free(&qs);
}

/* ================================================================ main */
/* chainSort's output, formatted in parallel (gt_par_write keeps the order) */
typedef struct sorted_out {
    const gt_chains *c;
    const sortkey *k;
} sorted_out;

static void write_sorted(FILE *f, int64_t j, void *arg) {
    const sorted_out *so = arg;
    const gt_chains *c = so->c;
    const outchain *o = &g_out[g_nout - 1 - so->k[j].rank];
    if (o->from >= 0)
        gt_write_chain(f, c, o->from, o->score, c->id[o->from]);
    else
        gt_write_chain_raw(f, o->score, c->tnames.names[o->tname], o->tsize, o->tstart, o->tend,
                           c->qnames.names[o->qname], o->qsize, o->qminus, o->qstart, o->qend,
                           o->id, o->bt, o->bq, o->bs, o->nb);
}

int main(int argc, char *argv[]) {
    {
        const char *sv = getenv("GAC_CLEANER_SPEC");
        g_spec = !(sv && *sv == '0');
        const char *ck = getenv("GAC_CLEANER_CHECK_KEYS");
        g_check_keys = ck && *ck == '1';
        const char *lv = getenv("GAC_CLEANER_LOOKAHEAD");
        if (lv && atoi(lv) > 0)
            g_lookahead = atoi(lv);
    }
    gt_stage("");
    gt_options(&argc, argv, k_opts);
    if (argc != 6)
        usage();
    gt_one_device(); /* before the chain reader's threads (setenv) */
    const char *in_chain = argv[1], *tnib = argv[2], *qnib = argv[3];
    const char *out_chain = argv[4], *out_bed = argv[5];
    const char *in_net = gt_opt_str("net", NULL);
    const char *tsizes = gt_opt_str("tSizes", NULL), *qsizes = gt_opt_str("qSizes", NULL);
    const char *gap_name = gt_opt_str("linearGap", NULL);
    const char *scheme = gt_opt_str("scoreScheme", NULL);
    debug = gt_opt_exists("debug");
    foldThreshold = gt_opt_double("foldThreshold", foldThreshold);
    LRfoldThreshold = gt_opt_double("LRfoldThreshold", LRfoldThreshold);
    LRfoldThresholdPairs = gt_opt_double("LRfoldThresholdPairs", LRfoldThresholdPairs);
    maxSuspectBases = gt_opt_double("maxSuspectBases", maxSuspectBases);
    maxSuspectScore = gt_opt_double("maxSuspectScore", maxSuspectScore);
    minBrokenChainScore = gt_opt_double("minBrokenChainScore", minBrokenChainScore);
    minLRGapSize = gt_opt_int("minLRGapSize", minLRGapSize);
    doPairs = gt_opt_exists("doPairs");
    maxPairDistance = gt_opt_int("maxPairDistance", maxPairDistance);
    const char *dict_file = gt_opt_str("newChainIDDict", NULL);
    const char *sdata_file = gt_opt_str("suspectDataFile", NULL);
    onlyThisChr = gt_opt_str("onlyThisChr", NULL);
    onlyThisStart = gt_opt_int("onlyThisStart", -1);
    onlyThisEnd = gt_opt_int("onlyThisEnd", -1);
    if (onlyThisChr)
        gt_verbose(1, "ONLY %s %d %d\n", onlyThisChr, onlyThisStart, onlyThisEnd);
    gt_verbose(1, "Verbosity level: %d\n", gt_verbosity());
    gt_verbose(1, "foldThreshold: %f    LRfoldThreshold: %f   maxSuspectBases: %d  maxSuspectScore: %d  minBrokenChainScore: %d  minLRGapSize: %d",
               foldThreshold, LRfoldThreshold, (int)maxSuspectBases, (int)maxSuspectScore,
               (int)minBrokenChainScore, minLRGapSize);
    if (doPairs)
        gt_verbose(1, " doPairs with LRfoldThreshold: %f   maxPairDistance %d\n",
                   LRfoldThresholdPairs, maxPairDistance);
    else
        gt_verbose(1, "\n");

    int32_t mat[16];
    if (scheme)
        gt_verbose(1, "Reading scoring matrix from %s\n", scheme);
    gt_check(gac_scheme_read(scheme, mat, NULL, NULL, NULL));
    if (gap_name == NULL)
        gt_abort("Must specify linear gap costs.  Use 'loose' or 'medium' for defaults\n");
    gac_gapcalc *gap = NULL;
    gt_check(gac_gapcalc_build(gap_name, &gap));
    if (!gt_file_exists(tnib))
        gt_abort("ERROR: target 2bit file or nib directory %s does not exist\n", tnib);
    if (!gt_file_exists(qnib))
        gt_abort("ERROR: query 2bit file or nib directory %s does not exist\n", qnib);
    if (!gac_is_twobit_file(tnib) || !gac_is_twobit_file(qnib))
        gt_abort("ERROR: only 2bit genome files are supported (got %s, %s)\n", tnib, qnib);
    /* device + genomes come up on a helper thread during steps 0-2 */
    gt_device dev;
    gt_device_start(&dev, tnib, qnib, mat, gap);
    gt_stage("options + setup");

    /* ---- 0. net the chains if no net is given */
    gt_lines net_lines;
    const char *net_what = in_net;
    if (in_net == NULL) {
        if (tsizes == NULL)
            gt_abort("You must specifiy -tSizes /dir/to/target/chrom.sizes if you do not provide a net file with -net in.net\n");
        if (qsizes == NULL)
            gt_abort("You must specifiy -qSizes /dir/to/query/chrom.sizes if you do not provide a net file with -net in.net\n");
        gt_verbose(1, "0. need to net the input chains %s (no net file given) ...\n", in_chain);
        net_in_process(in_chain, tsizes, qsizes, &net_lines);
        net_what = "(in-process nets)";
        gt_verbose(1, "DONE (nets in %s)\n", net_what);
    } else {
        gt_lines_read(in_net, &net_lines);
    }

    gt_stage("0. netting + filter");
    /* ---- 1. fills/gaps and valid breaks (getFillGapAndValidBreaks) */
    gt_verbose(1, "1. parsing fills/gaps from %s and getting valid breaks ...\n", net_what);
    gt_net_parse(&net_lines, net_what, &g_net.ns);
    gt_khash_init(&g_net.count, 0);
    for (int32_t k = 0; k < g_net.ns.n; ++k) {
        const gt_net1 *n = &g_net.ns.nets[k];
        if (onlyThisChr && strcmp(onlyThisChr, n->name) != 0)
            continue;
        const int32_t chrom = gt_names_add(&g_net.chroms, n->name, strlen(n->name));
        parse_fill(&g_net, n->first, 1, chrom);
    }
    chromregions *regions =
        calloc((size_t)(g_net.chroms.n ? g_net.chroms.n : 1), sizeof(chromregions));
    for (int32_t k = 0; k < g_net.ns.n; ++k) {
        const gt_net1 *n = &g_net.ns.nets[k];
        if (onlyThisChr && strcmp(onlyThisChr, n->name) != 0)
            continue;
        r_convert(&g_net.ns, n->first, &regions[gt_names_find(&g_net.chroms, n->name)]);
    }
    for (int32_t k = 0; k < g_net.chroms.n; ++k)
        build_regions(&regions[k]);

    gt_khash interest, breakhash;
    gt_khash_init(&interest, 0);
    gt_khash_init(&breakhash, 0);
    int32_t *bh_head = NULL, *bh_tail = NULL, bh_cap = 0;
    {
        int32_t *order = malloc((size_t)(g_net.count.n ? g_net.count.n : 1) * 4);
        const int32_t no = gt_khash_order(&g_net.count, order);
        for (int32_t oi = 0; oi < no; ++oi) { /* hashTraverseEls(chainId2Count, getValidBreaks) */
            const int32_t e = order[oi];
            if (g_net.cnt[e] == 1)
                continue;
            for (int32_t f = g_net.fg_head[e]; f >= 0; f = g_net.fg[f].next)
                if (!g_net.fg[f].gap_valid) /* chopGapInfo of an empty gap string */
                    gt_abort("chopGapInfo: Expecting 5 tab-separated words in  but can parse only 0\n");
            for (int32_t f = g_net.fg_head[e]; f >= 0; f = g_net.fg[f].next) {
                const fillgap *a = &g_net.fg[f];
                if (a->next < 0)
                    break;
                const fillgap *b = &g_net.fg[a->next];
                if (onlyThisChr && strcmp(onlyThisChr, chrom_name(a->chrom)) != 0)
                    continue;
                if (onlyThisChr && onlyThisStart != a->gap_end)
                    continue;
                if (onlyThisChr && onlyThisEnd != b->gap_start)
                    continue;
                if (a->depth != b->depth)
                    continue;
                if (a->parent_id != b->parent_id)
                    continue;
                if (broken_by_higher(&regions[a->chrom], a->fill_end, b->fill_start, a->chain_id,
                                     a->parent_id))
                    continue;
                if (a->gap_start == b->gap_start && a->gap_end == b->gap_end)
                    continue;
                const int32_t bi = new_break(a->depth, a->chain_id, a->parent_id, a->chrom,
                                             a->fill_start, a->fill_end, b->fill_start,
                                             b->fill_end, a->gap_start, a->gap_end, b->gap_start,
                                             b->gap_end);
                if (gt_khash_find(&interest, a->chain_id) < 0)
                    gt_khash_add(&interest, a->chain_id);
                if (gt_khash_find(&interest, a->parent_id) < 0)
                    gt_khash_add(&interest, a->parent_id);
                int32_t he = gt_khash_find(&breakhash, a->parent_id);
                if (he < 0) {
                    he = gt_khash_add(&breakhash, a->parent_id);
                    if (he >= bh_cap) {
                        bh_cap = bh_cap ? bh_cap * 2 : 1024;
                        bh_head = realloc(bh_head, (size_t)bh_cap * 4);
                        bh_tail = realloc(bh_tail, (size_t)bh_cap * 4);
                    }
                    bh_head[he] = bh_tail[he] = bi;
                } else {
                    g_brk[bi].prev = bh_tail[he];
                    g_brk[bh_tail[he]].next = bi;
                    bh_tail[he] = bi;
                }
            }
        }
        free(order);
    }
    gt_lines_free(&net_lines);
    gt_verbose(1, "DONE (parsing fills/gaps and getting valid breaks)\n\n");
    gt_stage("1. net parse + valid breaks");

    /* ---- 2. read the chains; the others go straight to the output */
    gt_verbose(1, "2. reading breaking and broken chains from %s ...\n", in_chain);
    state S;
    memset(&S, 0, sizeof(S));
    gt_read_chains(in_chain, &S.c, -HUGE_VAL, 1);
    gt_khash_init(&S.id2ich, 0);
    FILE *dbg_interest = debug ? gt_must_open("chainsOfInterest.chain", "w") : NULL;
    for (int64_t i = 0; i < S.c.n; ++i) {
        if (g_max_chain_id < S.c.id[i])
            g_max_chain_id = S.c.id[i];
        if (onlyThisChr && strcmp(onlyThisChr, S.c.tnames.names[S.c.tname[i]]) != 0)
            continue;
        if (gt_khash_find(&interest, S.c.id[i]) < 0) {
            outchain o;
            memset(&o, 0, sizeof(o));
            o.from = i;
            o.score = S.c.score[i];
            out_push(&o);
            continue;
        }
        GROWV(S.ich, S.ichcap, S.nich);
        ichain *x = &S.ich[S.nich];
        memset(x, 0, sizeof(*x));
        x->ci = i;
        x->score = S.c.score[i];
        const int64_t b0 = S.c.blk_off[i];
        x->nb = (int32_t)(S.c.blk_off[i + 1] - b0);
        x->bt = dup_i32(S.c.bt + b0, x->nb);
        x->bq = dup_i32(S.c.bq + b0, x->nb);
        x->bs = dup_i32(S.c.bs + b0, x->nb);
        int32_t e = gt_khash_find(&S.id2ich, S.c.id[i]);
        if (e < 0) {
            e = gt_khash_add(&S.id2ich, S.c.id[i]);
            S.id2ich_val = realloc(S.id2ich_val, (size_t)S.id2ich.cap * 4);
        }
        S.id2ich_val[e] = S.nich; /* hashFindVal finds the last chain added */
        ++S.nich;
        if (dbg_interest)
            gt_write_chain(dbg_interest, &S.c, i, S.c.score[i], S.c.id[i]);
    }
    if (dbg_interest)
        gt_careful_close(dbg_interest, "chainsOfInterest.chain");
    gt_verbose(1, "DONE\n\n");

    /* ---- 3. genomes and the chains of interest to the GPU */
    gt_stage("2. read chains");
    gt_verbose(1, "3. reading target and query DNA sequences for breaking and broken chains ...\n");
    {
        int32_t *order = malloc((size_t)(interest.n ? interest.n : 1) * 4);
        const int32_t no = gt_khash_order(&interest, order);
        for (int32_t oi = 0; oi < no; ++oi) /* loadTandQSeqs */
            if (ich_of(&S, interest.key[order[oi]]) < 0)
                gt_abort("ERROR: cannot get chain with Id %d from chainId2chain hash\n",
                         interest.key[order[oi]]);
        free(order);
    }
    /* the first pass's keys of every list (and its pairs), made while the
     * device may still be opening: host work only */
    int32_t *border = malloc((size_t)(breakhash.n ? breakhash.n : 1) * 4);
    const int32_t nborder = gt_khash_order(&breakhash, border);
    qkey *q0 = NULL;
    int64_t nq0 = 0, capq0 = 0;
    for (int32_t oi = 0; oi < nborder; ++oi)
        list_keys(&S, bh_head[border[oi]], sdata_file ? 0 : doPairs, 1, &q0, &nq0, &capq0);
    S.ctx = gt_device_join(&dev);
    {
        const size_t nn = (size_t)(S.nich ? S.nich : 1);
        S.t_seq = malloc(nn * 4);
        S.q_seq = malloc(nn * 4);
        S.strand = malloc(nn);
        int64_t *off = malloc((nn + 1) * 8);
        off[0] = 0;
        for (int32_t k = 0; k < S.nich; ++k) {
            const int64_t ci = S.ich[k].ci;
            const char *tn = S.c.tnames.names[S.c.tname[ci]], *qn = S.c.qnames.names[S.c.qname[ci]];
            S.t_seq[k] = gac_genome_seq_index(S.ctx, GAC_T, tn);
            S.q_seq[k] = gac_genome_seq_index(S.ctx, GAC_Q, qn);
            if (S.t_seq[k] < 0)
                gt_abort("%s is not in %s\n", tn, tnib);
            if (S.q_seq[k] < 0)
                gt_abort("%s is not in %s\n", qn, qnib);
            S.strand[k] = S.c.qstrand[ci];
            off[k + 1] = off[k] + S.ich[k].nb;
        }
        const size_t nb = (size_t)(off[S.nich] ? off[S.nich] : 1);
        int32_t *bt = malloc(nb * 4), *bq = malloc(nb * 4), *bs = malloc(nb * 4);
        for (int32_t k = 0; k < S.nich; ++k) {
            const ichain *x = &S.ich[k];
            memcpy(bt + off[k], x->bt, (size_t)x->nb * 4);
            memcpy(bq + off[k], x->bq, (size_t)x->nb * 4);
            memcpy(bs + off[k], x->bs, (size_t)x->nb * 4);
        }
        gac_chainset_desc d = {S.nich, S.t_seq, S.q_seq, S.strand, off, off[S.nich], bt, bq, bs};
        gt_check(gac_chains_upload(S.ctx, &d, &S.cs_base));
        free(off);
        free(bt);
        free(bq);
        free(bs);
    }
    gt_verbose(1, "DONE\n\n");

    gt_stage("3. device + chains of interest");
    /* ---- 4. loopOverBreaks */
    gt_verbose(1, "4. loop over all breaks. Remove suspects if they pass our filters and write out deleted suspects to %s ...\n",
               out_bed);
    if (debug) {
        g_dbg_susp = gt_must_open("suspect.chain", "w");
        g_dbg_L = gt_must_open("brokenChainLfill.chain", "w");
        g_dbg_R = gt_must_open("brokenChainRfill.chain", "w");
        g_dbg_F = gt_must_open("brokenChainfill.chain", "w");
        g_dbg_bed = gt_must_open("suspectsAndFills.bed", "w");
    }
    g_bed = gt_must_open(out_bed, "w");
    if (dict_file)
        g_dict = gt_must_open(dict_file, "w");
    if (sdata_file) {
        g_sdata = gt_must_open(sdata_file, "w");
        doPairs = 0;
    }
    {
        int32_t *order = border;
        const int32_t no = nborder;
        /* the first pass over every list (and its pairs) in one batch */
        qkey *q = q0;
        int64_t nq = nq0, capq = capq0;
        g_site = 0;
        score_keys(&S, q, nq);
        g_site = 2;
        gt_verbose(2, "scored %lld sub-chains of %lld breaks in one batch\n",
                   (long long)g_gpu_ranges, (long long)g_nbrk);
        for (int32_t oi = no - 1; oi >= 0; --oi) { /* hashElListHash: traversal reversed */
            /* the next lists' keys as the chains are now (the lists before
             * them modified their breaking chains): one batch for
             * g_lookahead lists; a key a later list changes is scored when
             * it is met */
            if (g_spec && (no - 1 - oi) % g_lookahead == 0) {
                nq = 0;
                for (int32_t oj = oi; oj >= 0 && oj > oi - g_lookahead; --oj)
                    list_keys(&S, bh_head[order[oj]], 0, 1, &q, &nq, &capq);
                g_site = 0;
                score_keys(&S, q, nq);
                g_site = 2;
            }
            loop_breaks(&S, bh_head[order[oi]]);
        }
        free(q);
        free(order);
    }
    gt_careful_close(g_bed, out_bed);
    if (g_dict)
        gt_careful_close(g_dict, dict_file);
    if (g_sdata)
        gt_careful_close(g_sdata, sdata_file);
    if (debug) {
        gt_careful_close(g_dbg_bed, "suspectsAndFills.bed");
        gt_careful_close(g_dbg_susp, "suspect.chain");
        gt_careful_close(g_dbg_L, "brokenChainLfill.chain");
        gt_careful_close(g_dbg_R, "brokenChainRfill.chain");
        gt_careful_close(g_dbg_F, "brokenChainfill.chain");
    }
    gt_verbose(1, "DONE\n\n");

    gt_stage("4. loop over breaks");
    /* ---- 5. the breaking and broken chains (writeAndFreeChainsOfInterest),
     * modified ones rescored -- one batch */
    gt_verbose(1, "5. write the (new) breaking and the broken chains ...\n");
    {
        int32_t *order = malloc((size_t)(interest.n ? interest.n : 1) * 4);
        const int32_t no = gt_khash_order(&interest, order);
        qkey *q = malloc((size_t)(no ? no : 1) * sizeof(qkey));
        int64_t nq = 0;
        for (int32_t oi = 0; oi < no; ++oi) {
            const int32_t ix = ich_of(&S, interest.key[order[oi]]);
            const int64_t ci = S.ich[ix].ci;
            if (S.ich[ix].rescore)
                q[nq++] = make_key(&S, ix, S.c.tstart[ci], S.c.tend[ci]);
        }
        score_keys(&S, q, nq);
        nq = 0;
        for (int32_t oi = 0; oi < no; ++oi) {
            const int32_t ix = ich_of(&S, interest.key[order[oi]]);
            ichain *x = &S.ich[ix];
            if (x->rescore)
                x->score = (double)cache_get(q[nq++])->g;
            const outchain o = out_of_ichain(&S, x, x->score, S.c.id[x->ci]);
            out_push(&o);
        }
        free(q);
        free(order);
    }
    gt_verbose(1, "DONE\n\n");

    /* ---- 6. chainSort */
    gt_stage("5. write chains of interest");
    gt_verbose(1, "6. chainSort %s ...\n", out_chain);
    {
        FILE *f = gt_must_open(out_chain, "w");
        for (int32_t m = 0; m < S.c.n_meta; ++m)
            fprintf(f, "%s\n", S.c.meta[m]);
        sortkey *k = malloc((size_t)(g_nout ? g_nout : 1) * sizeof(sortkey));
        /* the score as written ("%1.0f") and read back: printf rounds the
         * exact binary value to the nearest integer, ties to even, which is
         * nearbyint in the default rounding mode (no string round trip) */
        for (int64_t i = 0; i < g_nout; ++i) {
            k[i].score = nearbyint(g_out[i].score);
            k[i].rank = g_nout - 1 - i;
        }
        qsort(k, (size_t)g_nout, sizeof(sortkey), sortkey_cmp);
        sorted_out so = {&S.c, k};
        gt_par_write(f, g_nout, write_sorted, &so);
        gt_careful_close(f, out_chain);
        free(k);
    }
    gt_verbose(1, "DONE\n\n");
    gt_stage("6. chainSort");
    gt_verbose(1, "GPU: %lld scoring calls, %lld sub-chains, %lld re-uploads, %.3f s in scoring calls\n",
               (long long)g_gpu_calls, (long long)g_gpu_ranges, (long long)g_uploads, g_gpu_s);
    gt_verbose(2, "GPU: modified chains handed over %lld times, %lld blocks\n",
               (long long)g_host_chains, (long long)g_host_blocks);
    gt_verbose(2, "GPU: scoring calls by site: %lld list batches, %lld later passes, %lld tests\n",
               (long long)g_calls_site[0], (long long)g_calls_site[1], (long long)g_calls_site[2]);
    gt_verbose(2, "host: %.3f s removing suspects' blocks, %.3f s making tests' keys\n", g_t_remove,
               g_t_keys);
    gt_verbose(2, "GPU: keys a test missed (original / modified): suspect %lld/%lld fill %lld/%lld "
               "left %lld/%lld right %lld/%lld\n", (long long)g_miss[0][0], (long long)g_miss[0][1],
               (long long)g_miss[1][0], (long long)g_miss[1][1], (long long)g_miss[2][0],
               (long long)g_miss[2][1], (long long)g_miss[3][0], (long long)g_miss[3][1]);
    gt_verbose(1, "\nALL DONE. New chains are in %s. Deleted suspects in %s\n", out_chain, out_bed);
    gac_chains_free(S.cs_base);
    gac_close(S.ctx);
    gt_exit_ok(); /* host state is left to process exit */
}
