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
 *   chainCalcScore  kent/src/lib/chainConnect.c:24-40   gac_score_chains on a chain set
 *                                                        kept resident per chain list
 *                                                        (gac_kent_score_chains)
 *   chainSubsetOnT / chainFastSubsetOnT        the same list surgery on the host
 *                   kent/src/lib/chain.c:471-558        (no scoring)
 *   chainScoreBlock chainConnect.c:14-22       gac_score_text_blocks (device; the
 *   axtScoreUngapped kent/src/lib/axt.c:186-194  caller's text; batch:
 *                                               gac_kent_score_blocks)
 *   cBlockFindCrossover chainConnect.c:61-105  gac_text_crossovers (device)
 *   chainConnectCost / chainConnectGapCost     kent's case analysis on the host, the
 *                   chainConnect.c:108-149      crossover on the device, gapCalcCost
 *   chainRemovePartialOverlaps /               kent's list surgery on the host, each
 *     chainMergeAbutting chainConnect.c:255-368  crossover on the device
 *   chainBlocks     kent/src/lib/chainBlock.c:392-452  gac_chain_blocks (the kd-tree
 *                                               DP with the caller's cost callbacks)
 * The matrix of the text entry points must be a kent DNA scheme: nonzero
 * only between a/c/g/t in either case, the same for both cases
 * (propagateCase, axt.c:402-421); anything else ends the process, as an
 * unsupported input.
 */
#ifndef GACHAIN_KENT_H
#define GACHAIN_KENT_H

#include <stdint.h>
#include <stdio.h>

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

#if !defined(CHAINCONNECT_H)
struct chainConnect { /* kent/src/inc/chainConnect.h:8-15 */
    struct dnaSeq *query;
    struct dnaSeq *target;
    struct axtScoreScheme *ss;
    struct gapCalc *gapCalc;
};
#endif

#if !defined(CHAINBLOCK_H)
typedef int (*GapCost)(int dq, int dt, void *gapData);                         /* chainBlock.h:13 */
typedef int (*ConnectCost)(struct cBlock *a, struct cBlock *b, void *gapData); /* chainBlock.h:17 */
#endif

/* The context the shims score on, for the calling thread (NULL: unbind). */
void gac_kent_bind(gac_ctx *ctx);

struct gapCalc *gapCalcFromFile(char *fileName);
struct gapCalc *gapCalcDefault(void);
struct gapCalc *gapCalcOriginal(void);
void gapCalcFree(struct gapCalc **pGapCalc);
int gapCalcCost(struct gapCalc *gapCalc, int dq, int dt);

double chainCalcScore(struct chain *chain, struct axtScoreScheme *ss, struct gapCalc *gapCalc,
                      struct dnaSeq *query, struct dnaSeq *target);
/* chainConnect.h:41 -- query/target text starts at the chain's qStart/tStart */
double chainCalcScoreSubChain(struct chain *chain, struct axtScoreScheme *ss,
                              struct gapCalc *gapCalc, struct dnaSeq *query,
                              struct dnaSeq *target);

void chainSubsetOnT(struct chain *chain, int subStart, int subEnd, struct chain **retSubChain,
                    struct chain **retChainToFree);
void chainFastSubsetOnT(struct chain *chain, struct cBlock *firstBlock, int subStart,
                        int subEnd, struct chain **retSubChain, struct chain **retChainToFree);
/* frees what chainSubsetOnT allocated (malloc/free, like kent's default
 * memory handler) */
void gac_kent_chain_free(struct chain **pChain);

/* chainCalcScore of n chains in one GPU call: global[i] (kent's double).
 * The uploaded chain set stays resident while the same chains (same
 * pointers, block lists unchanged) are scored again: a caller looping
 * chainCalcScore over a list pays one upload, not one per call. */
void gac_kent_score_chains(struct chain *const *chains, int64_t n, struct axtScoreScheme *ss,
                           struct gapCalc *gapCalc, double *global);
/* drop the resident chain set (e.g. before freeing the chains).  Binding
 * another context drops it too; it stays safe after gac_close of its context. */
void gac_kent_forget_chains(void);

double chainScoreBlock(char *q, char *t, int size, int matrix[256][256]);
int axtScoreUngapped(struct axtScoreScheme *ss, char *q, char *t, int size);
/* chainScoreBlock of n blocks in one GPU call */
void gac_kent_score_blocks(int64_t n, char *const *q, char *const *t, const int *size,
                           int matrix[256][256], double *out);
void cBlockFindCrossover(struct cBlock *left, struct cBlock *right, struct dnaSeq *qSeq,
                         struct dnaSeq *tSeq, int overlap, int matrix[256][256], int *retPos,
                         int *retScoreAdjustment);
int chainConnectCost(struct cBlock *a, struct cBlock *b, struct chainConnect *cc);
int chainConnectGapCost(int dq, int dt, struct chainConnect *cc);
void chainRemovePartialOverlaps(struct chain *chain, struct dnaSeq *qSeq, struct dnaSeq *tSeq,
                                int matrix[256][256]);
void chainMergeAbutting(struct chain *chain);
struct chain *chainBlocks(char *qName, int qSize, char qStrand, char *tName, int tSize,
                          struct cBlock **pBlockList, ConnectCost connectCost, GapCost gapCost,
                          void *gapData, FILE *details);

#ifdef __cplusplus
}
#endif
#endif
