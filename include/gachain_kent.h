/* gachain_kent.h -- kent-signature shims over the libgachain batch ABI
 * (libgachain_kent.so).
 *
 * For C callers written against the kent library's chain API (SURVEY.md
 * §8(b)): link libgachain_kent instead of kent's chainConnect.o / gapCalc.o /
 * the subset half of chain.o, keep the calls.  The structs below are
 * layout-compatible with kent's (kent/src/inc/chain.h:17-63,
 * kent/src/inc/axt.h:83-91, kent/src/inc/dnaseq.h:17-25); struct gapCalc is
 * opaque, as in kent/src/inc/gapCalc.h:8.  When the kent headers are already
 * included (CHAIN_H / AXT_H / DNASEQ_H defined) they are used instead.
 *
 * Scoring goes to the GPU: gac_kent_bind() names the context (with both
 * genomes loaded: target and query sequences are looked up by the chain's
 * tName / qName; the '-' query strand is handled on the device, so the
 * dnaSeq arguments are not read).  One chainCalcScore call is one batched
 * call of one chain; gac_kent_score_chains() scores a whole list in one call.
 * Failures end the process with status 255, as kent's errAbort does.
 *
 *   reference                                  shim
 *   gapCalcFromFile / gapCalcDefault /         gac_gapcalc_build ("loose",
 *     gapCalcOriginal / gapCalcFree /            "medium" or a file), gac_gap_cost
 *     gapCalcCost   kent/src/lib/gapCalc.c:233-331
 *   chainCalcScore  kent/src/lib/chainConnect.c:24-40   gac_score_ranges (full chain)
 *   chainSubsetOnT / chainFastSubsetOnT        the same list surgery on the host
 *                   kent/src/lib/chain.c:471-558        (no scoring)
 */
#ifndef GACHAIN_KENT_H
#define GACHAIN_KENT_H

#include <stdint.h>

#include "gachain.h"

#ifdef __cplusplus
extern "C" {
#endif

#if !defined(CHAIN_H)
struct cBlock {
    struct cBlock *next;
    int tStart, tEnd;
    int qStart, qEnd;
    int score;
    void *data;
};

struct chain {
    struct chain *next;
    struct cBlock *blockList;
    double score;
    char *tName;
    int tSize;
    int tStart, tEnd;
    char *qName;
    int qSize;
    char qStrand;
    int qStart, qEnd;
    int id;
};
#endif

#if !defined(AXT_H)
struct axtScoreScheme {
    struct scoreMatrix *next;
    int matrix[256][256];
    int gapOpen;
    int gapExtend;
    char *extra;
};
#endif

#if !defined(DNASEQ_H)
struct dnaSeq {
    struct dnaSeq *next;
    char *name;
    char *dna;
    int size;
    void *mask;
};
#endif

struct gapCalc; /* opaque (wraps a gac_gapcalc) */

/* The context the shims score on, for the calling thread (NULL: unbind). */
void gac_kent_bind(gac_ctx *ctx);

struct gapCalc *gapCalcFromFile(char *fileName);
struct gapCalc *gapCalcDefault(void);
struct gapCalc *gapCalcOriginal(void);
void gapCalcFree(struct gapCalc **pGapCalc);
int gapCalcCost(struct gapCalc *gapCalc, int dq, int dt);

double chainCalcScore(struct chain *chain, struct axtScoreScheme *ss, struct gapCalc *gapCalc,
                      struct dnaSeq *query, struct dnaSeq *target);

void chainSubsetOnT(struct chain *chain, int subStart, int subEnd, struct chain **retSubChain,
                    struct chain **retChainToFree);
void chainFastSubsetOnT(struct chain *chain, struct cBlock *firstBlock, int subStart,
                        int subEnd, struct chain **retSubChain, struct chain **retChainToFree);
/* frees what chainSubsetOnT allocated (malloc/free, like kent's default
 * memory handler) */
void gac_kent_chain_free(struct chain **pChain);

/* chainCalcScore of n chains in one GPU call: global[i] (kent's double) */
void gac_kent_score_chains(struct chain *const *chains, int64_t n, struct axtScoreScheme *ss,
                           struct gapCalc *gapCalc, double *global);

#ifdef __cplusplus
}
#endif
#endif
