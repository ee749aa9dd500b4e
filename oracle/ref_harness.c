/* oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (never part of the product).
 *
 * A thin command-line harness linked against the REFERENCE's own kent
 * objects (built from /root/reference by oracle/ref.mk into
 * oracle/_ref/kentref).  It runs the reference's chainNet -rescore
 * per-fill work exactly as src/chainNet/chainNet.c:795-843 (subchainInfo)
 * does it -- chainBaseCount + chainBaseCountSubT full-list scans,
 * chainSubsetOnT (kent/src/lib/chain.c:471-558) and chainCalcScore
 * (kent/src/lib/chainConnect.c:24-40) on whole-chromosome char sequences with
 * '-' queries reverse-complemented once (chainNet.c:198-224) -- so that
 * bench.py can time the reference CPU path on the same fills as the GPU
 * ("cpu_baseline.kind = reference"), and tests can cross-check the oracle.
 *
 * chainBaseCount / chainBaseCountSubT / score<=0 -> 1 are static helpers in
 * chainNet.c (not in a library), so they are restated here (:763-782, :244-245).
 * scoreChain's chainCalcScoreLocal (src/scoreChain/scoreChain.c:176-198) is
 * likewise restated for the full-chain leg.
 */
#include "common.h"
#include "linefile.h"
#include "hash.h"
#include "dnautil.h"
#include "dnaseq.h"
#include "twoBit.h"
#include "chain.h"
#include "axt.h"
#include "gapCalc.h"
#include "chainConnect.h"
#include "chainBlock.h"
#include <time.h>

#include "kentapi_workload.inc"

struct krHandle {
    struct chain **chains;
    int nChains;
    struct twoBitFile *tbfT, *tbfQ;
    struct hash *tSeq, *qSeq, *qRc;
    struct axtScoreScheme *ss;
    struct gapCalc *gc;
};

static struct dnaSeq *krSeq(struct krHandle *h, char *name, char strand, int isT) {
    struct hash *hh = isT ? h->tSeq : h->qSeq;
    struct dnaSeq *seq = hashFindVal(hh, name);
    if (seq == NULL) {
        seq = twoBitReadSeqFrag(isT ? h->tbfT : h->tbfQ, name, 0, 0);
        hashAdd(hh, name, seq);
    }
    if (strand == '+')
        return seq;
    struct dnaSeq *rc = hashFindVal(h->qRc, name);
    if (rc == NULL) {
        rc = cloneDnaSeq(seq);
        reverseComplement(rc->dna, rc->size);
        hashAdd(h->qRc, name, rc);
    }
    return rc;
}

void *kr_open(char *chainFile, char *t2bit, char *q2bit, char *scoreScheme, char *linearGap) {
    struct krHandle *h;
    AllocVar(h);
    dnaUtilOpen();
    struct lineFile *lf = lineFileOpen(chainFile, TRUE);
    struct chain *chain, *list = NULL;
    int n = 0;
    while ((chain = chainRead(lf)) != NULL) {
        slAddHead(&list, chain);
        ++n;
    }
    lineFileClose(&lf);
    slReverse(&list);
    AllocArray(h->chains, n > 0 ? n : 1);
    h->nChains = n;
    int i = 0;
    for (chain = list; chain != NULL; chain = chain->next)
        h->chains[i++] = chain;
    h->tbfT = twoBitOpen(t2bit);
    h->tbfQ = twoBitOpen(q2bit);
    h->tSeq = newHash(0);
    h->qSeq = newHash(0);
    h->qRc = newHash(0);
    h->ss = (scoreScheme && scoreScheme[0]) ? axtScoreSchemeRead(scoreScheme) : axtScoreSchemeDefault();
    h->gc = gapCalcFromFile(linearGap);
    return h;
}

int kr_chain_count(void *vh) { return ((struct krHandle *)vh)->nChains; }

/* Preload every sequence the chains touch (the reference loads lazily; the
 * baseline times scoring with sequences already decoded, like the GPU leg
 * times scoring with genomes already resident). */
void kr_preload(void *vh) {
    struct krHandle *h = vh;
    int i;
    for (i = 0; i < h->nChains; ++i) {
        krSeq(h, h->chains[i]->tName, '+', 1);
        krSeq(h, h->chains[i]->qName, h->chains[i]->qStrand, 0);
    }
}

static int krBaseCount(struct chain *chain) {
    struct cBlock *b;
    int total = 0;
    for (b = chain->blockList; b != NULL; b = b->next)
        total += b->qEnd - b->qStart;
    return total;
}

static int krBaseCountSubT(struct chain *chain, int tMin, int tMax) {
    struct cBlock *b;
    int total = 0;
    for (b = chain->blockList; b != NULL; b = b->next)
        total += positiveRangeIntersection(b->tStart, b->tEnd, tMin, tMax);
    return total;
}

/* chainNet -rescore T-side subchainInfo for n fills: (chain index, start, end).
 * Writes score (as chainNet would print it) and ali.  Returns 0. */
int kr_rescore_fills(void *vh, int n, const int *chainIx, const int *start, const int *end,
                     double *outScore, int *outAli) {
    struct krHandle *h = vh;
    int i;
    for (i = 0; i < n; ++i) {
        struct chain *chain = h->chains[chainIx[i]];
        int s = start[i], e = end[i];
        int fullSize = krBaseCount(chain);
        if (s <= chain->tStart && e >= chain->tEnd) {
            outScore[i] = chain->score;
            outAli[i] = fullSize;
            continue;
        }
        outAli[i] = krBaseCountSubT(chain, s, e);
        struct chain *sub = NULL, *toFree = NULL;
        chainSubsetOnT(chain, s, e, &sub, &toFree);
        double score = 0;
        if (sub != NULL) {
            struct dnaSeq *q = krSeq(h, sub->qName, sub->qStrand, 0);
            struct dnaSeq *t = krSeq(h, sub->tName, '+', 1);
            score = chainCalcScore(sub, h->ss, h->gc, q, t);
        }
        if (score <= 0)
            score = 1;
        outScore[i] = score;
        chainFree(&toFree);
    }
    return 0;
}

/* Raw sub-chain scores without chainNet's full-chain / <=0 rules:
 * global = chainCalcScore of chainSubsetOnT(chain, s, e); local as
 * scoreChain.c:176-198.  Used to pin the oracle on arbitrary ranges. */
int kr_subchain_scores(void *vh, int n, const int *chainIx, const int *start, const int *end,
                       double *outGlobal, double *outLocal, int *outAli) {
    struct krHandle *h = vh;
    int i;
    for (i = 0; i < n; ++i) {
        struct chain *chain = h->chains[chainIx[i]];
        struct chain *sub = NULL, *toFree = NULL;
        chainSubsetOnT(chain, start[i], end[i], &sub, &toFree);
        outGlobal[i] = outLocal[i] = 0;
        outAli[i] = 0;
        if (sub == NULL)
            continue;
        struct dnaSeq *q = krSeq(h, sub->qName, sub->qStrand, 0);
        struct dnaSeq *t = krSeq(h, sub->tName, '+', 1);
        outGlobal[i] = chainCalcScore(sub, h->ss, h->gc, q, t);
        /* scoreChain.c:176-198 */
        struct cBlock *b1, *b2;
        double score = 0, maxScore = 0;
        int ali = 0;
        for (b1 = sub->blockList; b1 != NULL; b1 = b2) {
            ali += b1->tEnd - b1->tStart;
            score += chainScoreBlock(q->dna + b1->qStart, t->dna + b1->tStart,
                                     b1->tEnd - b1->tStart, h->ss->matrix);
            if (score > maxScore)
                maxScore = score;
            b2 = b1->next;
            if (b2 != NULL) {
                score -= gapCalcCost(h->gc, b2->qStart - b1->qEnd, b2->tStart - b1->tEnd);
                if (score < 0)
                    score = 0;
            }
        }
        outLocal[i] = maxScore;
        outAli[i] = ali;
        chainFree(&toFree);
    }
    return 0;
}

/* gapCalcCost through the reference's own gapCalc.c (KATs / exhaustive pins). */
int kr_gap_costs(char *linearGap, int n, const int *dq, const int *dt, int *out) {
    struct gapCalc *gc = gapCalcFromFile(linearGap);
    int i;
    for (i = 0; i < n; ++i)
        out[i] = gapCalcCost(gc, dq[i], dt[i]);
    gapCalcFree(&gc);
    return 0;
}

/* ------------------------------------------------------------------ main
 * kentref rescore  chain t.2bit q.2bit scheme|- gap ranges.bin out.bin
 * kentref subchain chain t.2bit q.2bit scheme|- gap ranges.bin out.bin
 * kentref gapcost  gap pairs.bin out.bin
 * ranges.bin: int32 (chainIx, start, end) triples; pairs.bin: int32 (dq, dt).
 * out.bin: rescore -> per range double score, int32 ali;
 *          subchain -> double global, double local, int32 ali;
 *          gapcost -> int32.
 * Prints {"seconds": S, "n": N} (scoring loop only, sequences preloaded). */
static void *readAll(char *path, size_t *n) {
    FILE *f = mustOpen(path, "rb");
    fseek(f, 0, SEEK_END);
    *n = ftell(f);
    fseek(f, 0, SEEK_SET);
    void *buf = needLargeMem(*n + 1);
    mustRead(f, buf, *n);
    fclose(f);
    return buf;
}

static double nowSec(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static struct dnaSeq *kaSeq(struct chain *c, int isT, void *u) {
    return krSeq(u, isT ? c->tName : c->qName, isT ? '+' : c->qStrand, isT);
}

int main(int argc, char *argv[]) {
    if (argc == 8 && sameString(argv[1], "kentapi")) {
        /* kentref kentapi chain t.2bit q.2bit scheme|- gap max_chains */
        struct krHandle *h = kr_open(argv[2], argv[3], argv[4],
                                     sameString(argv[5], "-") ? NULL : argv[5], argv[6]);
        int n = atoi(argv[7]);
        if (n > h->nChains)
            n = h->nChains;
        kentapi_run(h->chains, n, kaSeq, h, h->ss, h->gc, stdout);
        return 0;
    }
    if (argc == 5 && sameString(argv[1], "gapcost")) {
        size_t nb;
        int *pairs = readAll(argv[3], &nb);
        int n = nb / 8, i;
        int *dq, *dt, *out;
        AllocArray(dq, n + 1);
        AllocArray(dt, n + 1);
        AllocArray(out, n + 1);
        for (i = 0; i < n; ++i) {
            dq[i] = pairs[2 * i];
            dt[i] = pairs[2 * i + 1];
        }
        double t0 = nowSec();
        kr_gap_costs(argv[2], n, dq, dt, out);
        double t1 = nowSec();
        FILE *f = mustOpen(argv[4], "wb");
        mustWrite(f, out, n * sizeof(int));
        carefulClose(&f);
        printf("{\"seconds\": %.6f, \"n\": %d}\n", t1 - t0, n);
        return 0;
    }
    if (argc != 9)
        errAbort("usage: kentref rescore|subchain chain t.2bit q.2bit scheme|- gap ranges.bin out.bin\n"
                 "       kentref gapcost gap pairs.bin out.bin");
    char *scheme = sameString(argv[5], "-") ? NULL : argv[5];
    void *h = kr_open(argv[2], argv[3], argv[4], scheme, argv[6]);
    size_t nb;
    int *r = readAll(argv[7], &nb);
    int n = nb / 12, i;
    int *c, *s, *e, *ali;
    double *g, *l;
    AllocArray(c, n + 1);
    AllocArray(s, n + 1);
    AllocArray(e, n + 1);
    AllocArray(ali, n + 1);
    AllocArray(g, n + 1);
    AllocArray(l, n + 1);
    for (i = 0; i < n; ++i) {
        c[i] = r[3 * i];
        s[i] = r[3 * i + 1];
        e[i] = r[3 * i + 2];
        if (c[i] < 0 || c[i] >= kr_chain_count(h))
            errAbort("range %d: chain index %d out of range", i, c[i]);
    }
    kr_preload(h);
    double t0 = nowSec();
    if (sameString(argv[1], "rescore"))
        kr_rescore_fills(h, n, c, s, e, g, ali);
    else if (sameString(argv[1], "subchain"))
        kr_subchain_scores(h, n, c, s, e, g, l, ali);
    else
        errAbort("unknown mode %s", argv[1]);
    double t1 = nowSec();
    FILE *f = mustOpen(argv[8], "wb");
    mustWrite(f, g, n * sizeof(double));
    if (sameString(argv[1], "subchain"))
        mustWrite(f, l, n * sizeof(double));
    mustWrite(f, ali, n * sizeof(int));
    carefulClose(&f);
    printf("{\"seconds\": %.6f, \"n\": %d}\n", t1 - t0, n);
    return 0;
}
