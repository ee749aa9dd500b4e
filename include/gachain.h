/* gachain.h -- C ABI of libgachain, the MI355X-native chain-scoring engine.
 *
 * This is the drop-in boundary for the reference's chain-scoring hot path
 * (hillerlab/GenomeAlignmentTools: scoreChain, chainNet -rescore,
 * chainCleaner suspect rescoring).  The reference is single-threaded C whose
 * tools call the kent library one chain / one sub-chain at a time; this ABI
 * is the batch, struct-of-arrays replacement for those calls.  Plain C types
 * only: no torch, no HIP types in any signature.  Every entry point returns
 * GAC_OK (0) or a negative GAC_E* code; gac_last_error() gives the message.
 * There is NO CPU fallback: if the HIP runtime or an MI355X (gfx950) device
 * is unavailable, gac_open() fails and every call on a NULL context fails.
 *
 * Reference interfaces replaced (paths relative to the reference root):
 *   gac_score_ranges      <- chainSubsetOnT      kent/src/lib/chain.c:471-558
 *   (gac_score_windows: the same, windows known -- chainFastSubsetOnT :489-558)
 *                          + chainCalcScore       kent/src/lib/chainConnect.c:24-40
 *                          + chainScoreBlock      kent/src/lib/chainConnect.c:14-22
 *                          + gapCalcCost          kent/src/lib/gapCalc.c:298-331
 *                          + chainCalcScoreLocal  src/scoreChain/scoreChain.c:176-198
 *                                                 (= src/chainCleaner/chainCleaner.c:531-551)
 *                          + chainBaseCountSubT   src/chainNet/chainNet.c:773-782
 *                          (one call scores a whole batch of (chain, tStart, tEnd)
 *                           sub-chains; a range covering the chain is the full chain)
 *   gac_set_scoring       <- axtScoreSchemeDefault / axtScoreSchemeReadLf
 *                                                 kent/src/lib/axt.c:423-458,692-819
 *                          + gapCalcFromFile      kent/src/lib/gapCalc.c:233-255
 *   gac_genome_load_2bit  <- twoBitOpen + twoBitReadSeqFrag(tbf, name, 0, 0)
 *                                                 kent/src/lib/twoBit.c:482-513,725-888
 *                          + reverseComplement    kent/src/lib/dnautil.c:404-462
 *                          (genomes stay resident 2-bit packed; '-' query strand is
 *                           index arithmetic, not a reverse-complemented copy)
 *   gac_chains_upload     <- chainRead            kent/src/lib/chain.c:256-346
 *                          (the caller hands over parsed chains as SoA arrays)
 */
#ifndef GACHAIN_H
#define GACHAIN_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GAC_ABI_VERSION 1

/* return codes */
#define GAC_OK 0
#define GAC_E_ARG (-1)     /* bad argument / shape */
#define GAC_E_HIP (-2)     /* HIP runtime error (device fault, OOM, no device) */
#define GAC_E_IO (-3)      /* file open/read error */
#define GAC_E_FORMAT (-4)  /* malformed input file */
#define GAC_E_STATE (-5)   /* call out of order (e.g. scoring before set_scoring) */

/* genome sides */
#define GAC_T 0 /* target / reference genome */
#define GAC_Q 1 /* query genome */

/* gac_score_ranges flags */
#define GAC_WANT_LOCAL 1u /* also compute the scoreChain/chainCleaner local score */

typedef struct gac_ctx gac_ctx;
typedef struct gac_chainset gac_chainset;

/* Piecewise-linear gap cost tables exactly as kent's struct gapCalc
 * (kent/src/lib/gapCalc.c:12-37).  small tables have small_size entries,
 * entry 0 unused (0).  Build one with gac_gapcalc_build(). */
typedef struct gac_gapcalc {
    int32_t small_size;
    int32_t long_count;
    int32_t *q_small, *t_small, *b_small; /* [small_size] */
    int32_t *long_pos;                    /* [long_count] */
    double *q_long, *t_long, *b_long;     /* [long_count] */
    int32_t q_last_pos, t_last_pos, b_last_pos;
    double q_last_val, t_last_val, b_last_val;
    double q_last_slope, t_last_slope, b_last_slope;
} gac_gapcalc;

/* One sub-chain query: chain index in the chainset and a half-open target
 * range.  [t_start, t_end) covering the whole chain scores the full chain. */
typedef struct gac_range {
    int32_t chain;
    int32_t t_start;
    int32_t t_end;
} gac_range;

/* A sub-chain whose block window the caller already knows: chain, half-open
 * target range, and the blocks chainSubsetOnT(chain, t_start, t_end) selects
 * (kent/src/lib/chain.c:481-500: from the first block with tEnd > t_start,
 * while tStart < t_end) as a chain-local first block and count.  chainNet's
 * netting walks a fill's blocks when it creates the fill (innerBounds,
 * src/chainNet/chainNet.c:356-391), so its fills come with their windows
 * (gac_net_get_fill_windows) and scoring them needs no block search
 * (subchainInfo's three rescans, chainNet.c:795-843).  A window covering the
 * chain's span scores the whole chain, as a gac_range does. */
typedef struct gac_window {
    int32_t chain;
    int32_t t_start;
    int32_t t_end;
    int32_t first_block; /* chain-local index of the window's first block */
    int32_t n_blocks;    /* blocks in the window (0: scores 0) */
} gac_window;

/* Parsed chains, struct-of-arrays.  Blocks of chain c are
 * blk_*[blk_off[c] .. blk_off[c+1]), in chain order (ascending t and q;
 * q in the chain's strand coordinates, as in the .chain file). */
typedef struct gac_chainset_desc {
    int64_t n_chains;
    const int32_t *t_seq;    /* [n_chains] index into the T genome (gac_genome_seq_index) */
    const int32_t *q_seq;    /* [n_chains] index into the Q genome */
    const uint8_t *q_strand; /* [n_chains] 0 = '+', 1 = '-' */
    const int64_t *blk_off;  /* [n_chains + 1] */
    int64_t n_blocks;
    const int32_t *blk_t;    /* [n_blocks] tStart */
    const int32_t *blk_q;    /* [n_blocks] qStart */
    const int32_t *blk_size; /* [n_blocks] size (tEnd - tStart == qEnd - qStart) */
} gac_chainset_desc;

/* ---- library / context ------------------------------------------------ */
int gac_abi_version(void);
/* Human-readable message of the last error on this thread. */
const char *gac_last_error(void);
/* Open a context on HIP device `device`.  Fails (GAC_E_HIP) if there is no
 * usable gfx950 device: the library never falls back to the CPU. */
int gac_open(int device, gac_ctx **out);
/* Closing a context releases the device memory of every chain set still
 * open on it; such a set is left orphaned (gac_chains_context() is NULL, every
 * call on it fails with GAC_E_ARG) and gac_chains_free() only deletes it. */
void gac_close(gac_ctx *ctx);
/* Name of the device architecture the context runs on (e.g. "gfx950"). */
const char *gac_device_arch(gac_ctx *ctx);

/* ---- scoring scheme (host-side parsing, no device needed) -------------- */
/* Build gap tables from "loose", "medium" or a linearGap file
 * (gapCalcFromFile, kent/src/lib/gapCalc.c:233-255).  Free with gac_gapcalc_free. */
int gac_gapcalc_build(const char *name_or_file, gac_gapcalc **out);
void gac_gapcalc_free(gac_gapcalc *g);
/* gapCalcCost (kent/src/lib/gapCalc.c:298-331) on the host: negative
 * distances clamp to 0, q / t / both tables, interpolation in double with
 * the reference's operation order, truncated to int. */
int gac_gap_cost(const gac_gapcalc *g, int dq, int dt);
/* Read a blastz/lastz matrix file (axtScoreSchemeReadLf, axt.c:692-819), or the
 * blastz default when path is NULL (axtScoreSchemeDefault, axt.c:423-458).
 * mat[i*4+j] = matrix[query base i][target base j], i,j in A,C,G,T order.
 * gap_open/gap_extend/extra may be NULL; extra (malloc'd, caller frees) is the
 * "##blastzParms" text. */
int gac_scheme_read(const char *path, int32_t mat[16], int32_t *gap_open,
                    int32_t *gap_extend, char **extra);
/* Install matrix + gap tables on the device. */
int gac_set_scoring(gac_ctx *ctx, const int32_t mat[16], const gac_gapcalc *g);

/* ---- genomes ------------------------------------------------------------ */
/* Load every sequence of a .2bit file onto the device for side T or Q. */
int gac_genome_load_2bit(gac_ctx *ctx, int side, const char *path);
/* Or add sequences one by one from a raw .2bit payload (2 bits/base, MSB
 * first, T=0 C=1 A=2 G=3) plus N runs, then gac_genome_finalize(). */
int gac_genome_add_seq(gac_ctx *ctx, int side, const char *name, int32_t size,
                       const uint8_t *packed, int32_t n_nblocks,
                       const int32_t *n_starts, const int32_t *n_sizes);
int gac_genome_finalize(gac_ctx *ctx, int side);
int32_t gac_genome_seq_count(gac_ctx *ctx, int side);
/* Sequence index by name, or -1. */
int32_t gac_genome_seq_index(gac_ctx *ctx, int side, const char *name);
int32_t gac_genome_seq_size(gac_ctx *ctx, int side, int32_t index);
const char *gac_genome_seq_name(gac_ctx *ctx, int side, int32_t index);
/* Decode [start, end) of a resident sequence back to 'acgtn' text (test aid:
 * proves the resident layout round-trips; out must hold end-start bytes). */
int gac_genome_decode(gac_ctx *ctx, int side, int32_t index, int32_t start,
                      int32_t end, char *out);

/* ---- chains ------------------------------------------------------------- */
/* At most 2^31 - 17 blocks per chain set (GAC_E_ARG beyond: upload in parts). */
int gac_chains_upload(gac_ctx *ctx, const gac_chainset_desc *d, gac_chainset **out);
/* Replace the contents of an uploaded set with d, reusing its device memory
 * when it is large enough (for callers that score a changing handful of
 * chains many times, e.g. chainCleaner's modified chains: no allocation or
 * free per call). Waits for calls still using the set. */
int gac_chains_reupload(gac_ctx *ctx, const gac_chainset_desc *d, gac_chainset *cs);
void gac_chains_free(gac_chainset *cs);
/* The context a set belongs to; NULL once that context was closed. */
gac_ctx *gac_chains_context(const gac_chainset *cs);
/* gac_score_ranges for chains held in host memory (no upload): each range is
 * planned on the host (its window of blocks found by binary search) and the
 * windows are scored by one kernel launch per 256 ranges reading them from
 * pinned mapped memory, gap costs and N masks on the device.  For callers
 * that score a few sub-chains of chains they keep changing (chainCleaner's
 * modified chains).  Results as gac_score_ranges. */
int gac_score_ranges_host(gac_ctx *ctx, const gac_chainset_desc *d, const gac_range *ranges,
                          int64_t n, uint32_t flags, int64_t *global, int64_t *local,
                          int32_t *ali);
int64_t gac_chains_block_count(const gac_chainset *cs);

/* ---- scoring ------------------------------------------------------------ */
/* Score n sub-chains.  Host buffers; synchronous.  For range r of chain c the
 * sub-chain is chainSubsetOnT(c, r.t_start, r.t_end) and
 *   global[r] = chainCalcScore(sub)            (exact; reference's double is integral)
 *   local[r]  = chainCalcScoreLocal(sub)       (only with GAC_WANT_LOCAL; may be NULL otherwise)
 *   ali[r]    = sum of clipped block sizes     (chainBaseCountSubT)
 * A range selecting no block yields 0, 0, 0. */
int gac_score_ranges(gac_ctx *ctx, const gac_chainset *cs, const gac_range *ranges,
                     int64_t n, uint32_t flags, int64_t *global, int64_t *local,
                     int32_t *ali);
/* Same on device-resident buffers, enqueued on `stream` (a hipStream_t, or
 * NULL for the context's own stream).  Returns as soon as the batch is known
 * to fit the scoring workspace (the first kernels write a status word to
 * pinned host memory; on the rare call that outgrows the workspace it is
 * grown and the batch rerun before returning); the scoring itself completes
 * asynchronously -- synchronise the stream (or gac_synchronize /
 * gac_memcpy_d2h, which are ordered after it) before reading results.
 * d_local may be NULL unless GAC_WANT_LOCAL. */
int gac_score_ranges_device(gac_ctx *ctx, const gac_chainset *cs,
                            const gac_range *d_ranges, int64_t n, uint32_t flags,
                            int64_t *d_global, int64_t *d_local, int32_t *d_ali,
                            void *stream);

/* gac_score_ranges for sub-chains given with their windows (gac_window): the
 * same results as gac_score_ranges on (chain, t_start, t_end) when each window
 * is chainSubsetOnT's; the device reads one chain record per window instead of
 * searching the chain's blocks.  A window outside its chain (first_block < 0,
 * n_blocks < 0, or past the chain's last block; chain out of range) is
 * GAC_E_ARG.  Host buffers, synchronous. */
int gac_score_windows(gac_ctx *ctx, const gac_chainset *cs, const gac_window *windows,
                      int64_t n, uint32_t flags, int64_t *global, int64_t *local,
                      int32_t *ali);
/* The same on device-resident buffers, enqueued on `stream` (NULL: the
 * context's); returns as gac_score_ranges_device does (a bad window is
 * reported by this call, once the planning kernel has run). */
int gac_score_windows_device(gac_ctx *ctx, const gac_chainset *cs, const gac_window *d_windows,
                             int64_t n, uint32_t flags, int64_t *d_global, int64_t *d_local,
                             int32_t *d_ali, void *stream);

/* Every chain of the set, in order -- scoreChain's batch (the per-chain
 * chainCalcScore + chainCalcScoreLocal of src/scoreChain/scoreChain.c:207-220,
 * 301-331): global[c], local[c] (GAC_WANT_LOCAL), ali[c] for c in
 * 0..n_chains-1, equal to gac_score_ranges over ranges covering each whole
 * chain.  The chain set's own scoring plan is built at the first call and
 * kept with the set, so a call is just the scoring kernels. */
int gac_score_chains(gac_ctx *ctx, const gac_chainset *cs, uint32_t flags, int64_t *global,
                     int64_t *local, int32_t *ali);
/* The same into device buffers on `stream` (NULL: the context's); returns once
 * enqueued. */
int gac_score_chains_device(gac_ctx *ctx, const gac_chainset *cs, uint32_t flags,
                            int64_t *d_global, int64_t *d_local, int32_t *d_ali, void *stream);

/* ---- caller text (the kent in-process API's char* entry points) ---------
 * chainScoreBlock / axtScoreUngapped (kent/src/lib/chainConnect.c:14-22,
 * axt.c:186-194) of n blocks of caller-owned text: score[i] = sum over k <
 * size[i] of mat[q][t] (A,C,G,T order as gac_scheme_read; any other
 * character scores 0, either case).  On the device; synchronous. */
int gac_score_text_blocks(gac_ctx *ctx, int64_t n, const char *const *q, const char *const *t,
                          const int32_t *size, const int32_t mat[16], int64_t *score);
/* cBlockFindCrossover (chainConnect.c:61-105) of n overlaps on caller text:
 * lq/lt point at the left block's last overlap[i] bases (qEnd - overlap),
 * rq/rt at the right block's first.  Out: pos (offset of the crossover from
 * the right block's start) and adj (rScore + lScore - bestScore). */
int gac_text_crossovers(gac_ctx *ctx, int64_t n, const char *const *lq, const char *const *lt,
                        const char *const *rq, const char *const *rt, const int32_t *overlap,
                        const int32_t mat[16], int32_t *pos, int32_t *adj);

/* ---- axtChain ------------------------------------------------------------
 * Per-block scores: axtScoreUngapped (kent/src/lib/axt.c:186-194) of every
 * block, the scores chainPair gives the kd-tree (axtChain.c:276-282).  Pairs
 * share a target / query sequence and strand ('-': query coordinates on the
 * reverse strand, as in PSL/axt).  Blocks must lie inside their sequences. */
int gac_score_blocks(gac_ctx *ctx, int64_t n_pairs, const int32_t *t_seq, const int32_t *q_seq,
                     const uint8_t *q_strand, const int64_t *blk_off, const int32_t *blk_t,
                     const int32_t *blk_q, const int32_t *blk_size, int32_t *score);

/* The kd-tree DP of chainBlocks on the device: findBestPredecessors
 * (kent/src/lib/chainBlock.c:281-300) -- bestPredecessor (:207-263) with
 * chainConnectCost / cBlockFindCrossover (chainConnect.c:61-149) as its
 * connect cost, updateScoresOnWay (:265-279) -- for n_pairs seqPairs in one
 * launch, one wave per pair.  The caller builds each pair's tree (kdBuild,
 * :124-164) in pre-order with the hi child first:
 *   node_a[4v..] = {maxQ, maxT, cut, lo child}         internal node
 *                  {qEnd, tEnd, qStart, tStart}        leaf node
 *   node_b[2v..] = {end of v's subtree, dim (0 q, 1 t)} internal node
 *                  {end = v + 1, ~(leaf position)}     leaf node
 * node indices are relative to the pair (nodes [node_off[p], node_off[p+1])).
 * Leaves are in findBestPredecessors' target order, [leaf_off[p],
 * leaf_off[p+1]): leaf[4i..] = {qStart, qEnd, tStart, tEnd}, leaf_score[i]
 * (axtScoreUngapped), leaf_node[i] (its node), and path[path_off[i] ..
 * path_off[i+1]) = the nodes updateScoresOnWay's descent reaches for it
 * (global leaf index i; path_off has total leaves + 1 entries).  Out, per
 * leaf: total[i] = totalScore, pred[i] = best predecessor node or -1.
 * Uses the context's scoring setup (gac_set_scoring) and genomes. */
int gac_chain_dp(gac_ctx *ctx, int64_t n_pairs, const int32_t *t_seq, const int32_t *q_seq,
                 const uint8_t *q_strand, const int64_t *node_off, const int32_t *node_a,
                 const int32_t *node_b, const int64_t *leaf_off, const int32_t *leaf,
                 const int32_t *leaf_score, const int32_t *leaf_node, const int64_t *path_off,
                 const int32_t *path, int64_t *total, int32_t *pred);

/* chainBlocks' kd-tree DP for n_pairs seqPairs straight from their blocks,
 * every input of the DP built on the device:
 *   the leaf list (kent/src/lib/chainBlock.c:400-420: blocks with tStart !=
 *     tEnd, slSort by tStart over the slAddHead-built list) and its query
 *     order (kdTreeMake :166-205),
 *   the kd-trees (kdBuild :124-164, splitList/medianVal :92-122),
 *   the update paths (updateScoresOnWay :265-279) and, for the exact fast
 *     DP, each leaf's overlapping candidates,
 * then findBestPredecessors (:281-300) as in gac_chain_dp.  Blocks of pair p
 * are [blk_off[p], blk_off[p+1]) in the caller's list order (axtChain's order
 * after removeExactOverlaps), box[4g..] = {qStart, qEnd, tStart, tEnd} in
 * the pair's strand coordinates, score[g] = axtScoreUngapped.
 * fast != 0: the exact fast search (k_dp_fast) with the linear gap-cost
 * minorant lin_k / 1024 and the smallest matrix entry min_entry; ov_cap
 * (<= 1024): more overlapping candidates than this send a leaf to the
 * reference search order.  fast == 0: the reference search (k_dp).
 * Out: leaf_off[n_pairs + 1] (the leaves of pair p are [leaf_off[p],
 * leaf_off[p+1])), tord[leaf] = the pair-local block of each leaf in target
 * order, and per block total[g] = totalScore (score for a non-leaf) and
 * pred[g] = the best predecessor as a pair-local block, or -1.  A block
 * outside its sequences is GAC_E_ARG.  Uses the context's scoring setup and
 * genomes. */
/* kdTreeMake (kent/src/lib/chainBlock.c:166-205: the leaf lists and
 * kdBuild :124-164) for n_pairs seqPairs on the device -- the build of
 * gac_chain_dp_blocks -- for a caller that runs the DP itself.  Blocks as in
 * gac_chain_dp_blocks.  Out: leaf_off[n_pairs + 1], and per pair p into the
 * caller's buffers: tord[p][leaf] / qord[p][leaf] = the pair-local blocks of
 * its leaves in target / query order (at most blk_off[p+1] - blk_off[p]
 * each), lnode[p][block] = the leaf node of each block (-1: tStart ==
 * tEnd, not a leaf), nodes[p][6 v ..] = node v of the pair's 2 n - 1 (n =
 * its leaves) in pre-order with the hi child first: {lo, hi, -1, cut, maxQ,
 * maxT} for an internal node, {qStart, tStart, block, 0, qEnd, tEnd} for a
 * leaf node. */
int gac_kd_trees(gac_ctx *ctx, int64_t n_pairs, const int32_t *t_seq, const int32_t *q_seq,
                 const uint8_t *q_strand, const int64_t *blk_off, const int32_t *box,
                 int64_t *leaf_off, int32_t *const *tord, int32_t *const *qord,
                 int32_t *const *lnode, int32_t *const *nodes);

int gac_chain_dp_blocks(gac_ctx *ctx, int64_t n_pairs, const int32_t *t_seq,
                        const int32_t *q_seq, const uint8_t *q_strand, const int64_t *blk_off,
                        const int32_t *box, const int32_t *score, int fast, int64_t lin_k,
                        int32_t min_entry, int32_t ov_cap, int64_t *leaf_off, int32_t *tord,
                        int64_t *total, int32_t *pred);

/* cBlockFindCrossover (kent/src/lib/chainConnect.c:61-105) of n overlapping
 * block pairs on the device (one wave per pair, a prefix-sum / first-maximum
 * scan): left block ending at (lqe, lte), right block starting at (rqs, rts),
 * `overlap` bases, on seqPair (t_seq, q_seq, q_strand) -- strand coordinates.
 * Out: pos (crossover offset from the right block's start) and adj (the
 * score adjustment).  Uses the context's score matrix. */
int gac_crossovers(gac_ctx *ctx, int64_t n, const int32_t *t_seq, const int32_t *q_seq,
                   const uint8_t *q_strand, const int32_t *lqe, const int32_t *lte,
                   const int32_t *rqs, const int32_t *rts, const int32_t *overlap, int32_t *pos,
                   int32_t *adj);

/* axtChain's chaining of every seqPair (axtChain.c:250-309 chainPair and
 * :452-470 the final sort), replacing
 *   removeExactOverlaps          axtChain.c:173-197
 *   axtScoreUngapped per block   axt.c:186-194              (GPU, gac_score_blocks)
 *   chainBlocks                  kent/src/lib/chainBlock.c:400-452: the kd-tree
 *                                (kdBuild :124-164), bestPredecessor (:207-263),
 *                                updateScoresOnWay (:265-279), peelChains
 *                                (:311-373), scoreBlocks (:296-309)
 *   chainConnectCost             kent/src/lib/chainConnect.c:114-149 (+ cBlockFindCrossover :61-105)
 *   chainRemovePartialOverlaps   chainConnect.c:255-344, chainMergeAbutting :346-368
 *   chainCalcScore               chainConnect.c:24-40       (GPU, gac_score_ranges)
 *   minScore filter + slSort(chainCmpScore)
 * Blocks of pair p are [blk_off[p], blk_off[p+1]) in the order axtChain holds
 * them before removeExactOverlaps (input order: the PSL/axt records and their
 * blocks as read).  Pairs are processed in the given order (spList order);
 * the kd-tree DP runs on host threads (n_threads, 0 = all cores), one pair at
 * a time per thread -- or, with GAC_AXT_DP=gpu in the environment, on the
 * device (gac_chain_dp, then the crossovers of scoreBlocks and
 * chainRemovePartialOverlaps through gac_crossovers); the output is the same.
 * Output chains are in chainWrite order; ids are 1..n.
 * details_path (may be NULL): axtChain -details text.  Installs mat/g on
 * the context (gac_set_scoring). */
typedef struct gac_axt_input {
    int64_t n_pairs;
    const int32_t *t_seq;    /* [n_pairs] gac_genome_seq_index(GAC_T) */
    const int32_t *q_seq;    /* [n_pairs] gac_genome_seq_index(GAC_Q) */
    const uint8_t *q_strand; /* [n_pairs] 0 '+', 1 '-' */
    const int64_t *blk_off;  /* [n_pairs + 1] */
    const int32_t *blk_t, *blk_q, *blk_size;
} gac_axt_input;

typedef struct gac_axt_chains {
    int64_t n_chains;
    double *score;           /* chainCalcScore (integral) */
    int32_t *pair;           /* seqPair index of each chain */
    int32_t *t_start, *t_end, *q_start, *q_end;
    int64_t *blk_off;        /* [n_chains + 1] */
    int64_t n_blocks;
    int32_t *blk_t, *blk_q, *blk_size;
} gac_axt_chains;

int gac_axt_chain(gac_ctx *ctx, const int32_t mat[16], const gac_gapcalc *g,
                  const gac_axt_input *in, double min_score, int n_threads,
                  const char *details_path, gac_axt_chains **out);
void gac_axt_chains_free(gac_axt_chains *c);

/* kent's chainBlocks (kent/src/lib/chainBlock.c:392-452) with the caller's
 * cost functions -- the kd-tree DP behind axtChain, for callers that bring
 * their own ConnectCost / GapCost (chainBlock.h:13-19): the DP runs on the
 * calling thread (host: it is a sequential branch-and-bound search by the
 * reference's definition), calling connect(a, b, user) /
 * gap(dq, dt, user) with block indices.  Blocks i: q [qs, qe), t [ts, te),
 * score[i]; zero-length blocks are skipped, as kent does.  Out: chains in
 * chainCmpScore order (stable), chain c = blocks blk[off[c] .. off[c+1])
 * ascending, score[c] = scoreBlocks (block scores minus connect costs).
 * details (may be NULL): peelChains' -details text. */
typedef int (*gac_connect_fn)(int32_t a, int32_t b, void *user);
typedef int (*gac_gapcost_fn)(int dq, int dt, void *user);
typedef struct gac_block_chains {
    int32_t n_chains;
    double *score;
    int32_t *off; /* [n_chains + 1] */
    int32_t *blk;
} gac_block_chains;
int gac_chain_blocks(int32_t n, const int32_t *qs, const int32_t *qe, const int32_t *ts,
                     const int32_t *te, const int32_t *score, gac_connect_fn connect,
                     gac_gapcost_fn gap, void *user, const char *qname, int32_t qsize, char qstrand,
                     const char *tname, int32_t tsize, FILE *details, gac_block_chains **out);
void gac_block_chains_free(gac_block_chains *c);

/* ---- chainNet netting engine (host, no device needed) -------------------
 * Replaces chainNet's netting and output (src/chainNet/chainNet.c:328-896):
 * makeChroms/addChainT/addChainQ/fillSpace/finishNet/rOutputFill/...
 * Same fills, gaps and .net text; no per-fill O(blocks) list rescans.  For
 * -rescore the caller scores the partial T fills with gac_score_ranges and
 * hands the scores to gac_net_write (subchainInfo's rescoring branch,
 * chainNet.c:826-836).  Input arrays are borrowed and must outlive the net. */
typedef struct gac_net gac_net;

typedef struct gac_net_input {
    int64_t n_chains;        /* in file order (chainNet requires descending score) */
    const double *score;     /* header score */
    const int32_t *id;       /* chain id */
    const int32_t *t_seq;    /* index into t_names/t_sizes */
    const int32_t *q_seq;    /* index into q_names/q_sizes */
    const uint8_t *q_strand; /* 0 '+', 1 '-' */
    const int32_t *t_start, *t_end, *q_start, *q_end;
    const int64_t *blk_off;  /* [n_chains + 1] */
    const int32_t *blk_t, *blk_q, *blk_size;
    int32_t n_tseq;          /* target chrom.sizes, file order */
    const char *const *t_names;
    const int32_t *t_sizes;
    int32_t n_qseq;          /* query chrom.sizes, file order */
    const char *const *q_names;
    const int32_t *q_sizes;
} gac_net_input;

typedef struct gac_net_opts {
    int32_t min_space; /* -minSpace, default 25 */
    int32_t min_fill;  /* -minFill, default min_space / 2 */
    double min_score;  /* -minScore, default 2000; 0 with -rescore */
    int32_t incl_hap;  /* -inclHap */
} gac_net_opts;

/* Net chains in order until the first one with score < min_score (error if
 * scores increase).  Chains on *_hap* / *_alt* queries are skipped unless
 * incl_hap. */
int gac_net_build(const gac_net_input *in, const gac_net_opts *opts, gac_net **out);
/* The same for the sides in `sides` only (bit 1 << GAC_T, bit 1 << GAC_Q):
 * the two sides' trees are independent, so a caller that writes only the
 * target net (chainCleaner's `chainNet ... stdout /dev/null`,
 * src/chainCleaner/chainCleaner.c:1660) skips the query side.  Fill queries
 * and writes of a side not built fail with GAC_E_STATE. */
int gac_net_build_sides(const gac_net_input *in, const gac_net_opts *opts, int sides,
                        gac_net **out);
/* The same for a subset of chromosome sides: t_keep[k] / q_keep[k] != 0 =
 * net target / query sequence k (a sequence's side depends only on the
 * chains on it, so ranks of a multi-GPU run each net their own sequences;
 * the unselected ones are written as if they held no chains). */
int gac_net_build_subset(const gac_net_input *in, const gac_net_opts *opts, const uint8_t *t_keep,
                         const uint8_t *q_keep, gac_net **out);
void gac_net_free(gac_net *net);
/* number of input chains consumed (netted or skipped) before stopping */
int64_t gac_net_netted(const gac_net *net);
/* fills of one side, in .net output (pre-order) order */
int64_t gac_net_fill_count(const gac_net *net, int side);
/* Per fill: chain index, start, end (own side, + strand), aligned bases
 * (subchainInfo's subSize) and flags: bit0 = partial (rescored on T with
 * -rescore), bit1 = printed by rOutputFill under -rescore (the fill and all
 * its ancestors have ali >= min_fill).  Any pointer may be NULL. */
int gac_net_get_fills(const gac_net *net, int side, int32_t *chain, int32_t *start,
                      int32_t *end, int32_t *ali, uint8_t *flags);
/* Per target fill, in gac_net_get_fills order: the window of the fill's chain
 * that chainSubsetOnT(chain, start, end) selects (gac_window's first_block /
 * n_blocks), recorded while netting.  side must be GAC_T. */
int gac_net_get_fill_windows(const gac_net *net, int side, int32_t *first_block,
                             int32_t *n_blocks);
/* The -rescore list in one pass: the target fills that are partial and
 * printed (gac_net_get_fills flags == 3), in pre-order, as gac_window
 * records (chain, start, end and their window) with each one's pre-order
 * position in `pos` (for gac_net_write's t_scores).  *windows and *pos are
 * malloc'ed (free them); *n = their count.  side must be GAC_T. */
int gac_net_rescore_windows(const gac_net *net, int side, gac_window **windows, int64_t **pos,
                            int64_t *n);
/* Write one side's .net (outputNetSide) to path ("stdout" allowed) after the
 * n_meta '#' metadata lines.  t_scores (T side only, may be NULL): per fill
 * in gac_net_get_fills order, the rescored global score of partial fills
 * (<= 0 prints as 1); NULL = reference's proportional approximation. */
int gac_net_write(const gac_net *net, int side, const int64_t *t_scores, const char *path,
                  const char *const *meta, int32_t n_meta);
/* The same text written to an open stream (e.g. an open_memstream buffer:
 * chainNet -nranks formats a rank's part in memory, then writes it in place). */
int gac_net_write_file(const gac_net *net, int side, const int64_t *t_scores, FILE *f,
                       const char *const *meta, int32_t n_meta);
/* The same text formatted on all threads and returned as buffers (chainNet
 * -nranks writes a rank's part in place from them, with no staging copy):
 * *bufs[0 .. *nbufs) in order, malloc'ed (free each and the arrays), *lens
 * their lengths; the n_meta '#' lines are the first buffer. */
int gac_net_format(const gac_net *net, int side, const int64_t *t_scores,
                   const char *const *meta, int32_t n_meta, char ***bufs, size_t **lens,
                   int64_t *nbufs);
/* The target net in two phases, for -rescore: _begin formats everything but
 * the rescored partial fills' scores (which fills print does not depend on
 * them when minScore <= 1: a rescored score is >= 1, chainNet.c:244-245),
 * e.g. while the GPU computes them; _end inserts the scores and writes the
 * same text as gac_net_write(..., t_scores, ...).  _free drops a prepared
 * net that is not written. */
typedef struct gac_net_wpre gac_net_wpre;
int gac_net_write_begin(const gac_net *net, int side, const char *const *meta, int32_t n_meta,
                        gac_net_wpre **out);
int gac_net_write_end(gac_net_wpre *w, const int64_t *t_scores, FILE *f);
void gac_net_write_free(gac_net_wpre *w);

/* ---- the -nranks collective (gac_allgather) ---------------
 * One process per GPU of one node.  A communicator joins `nranks` processes
 * through a rendezvous prefix: a path the ranks share and that is unique to
 * the run (the tools use their output path plus the run's GAC_RANK_TOKEN);
 * the host backend keeps its part and barrier files next to it.
 *   GAC_COMM_RCCL  ncclAllGather over xGMI (librccl loaded at run time; the
 *                  unique id passes through the rendezvous files), `device`
 *                  = this rank's GPU; RCCL refuses two ranks on one device.
 *   GAC_COMM_HOST  part files in the node's page cache, no device.
 *   GAC_COMM_AUTO  GAC_COMM=rccl|host if set, else RCCL when device >= 0.
 * A wait gives up after timeout_s seconds (<= 0: 600) or when alive(peer,
 * user) returns 0 (NULL: no check), with GAC_E_STATE.  Every rank must make
 * the same calls in the same order. */
typedef struct gac_comm gac_comm;
#define GAC_COMM_AUTO 0
#define GAC_COMM_HOST 1
#define GAC_COMM_RCCL 2
int gac_comm_open(const char *rendezvous, int nranks, int rank, int device, int backend,
                  double timeout_s, int (*alive)(int rank, void *user), void *user,
                  gac_comm **out);
int gac_comm_backend(const gac_comm *comm); /* GAC_COMM_HOST / GAC_COMM_RCCL */
double gac_comm_init_seconds(const gac_comm *comm); /* RCCL set-up time (0: host) */
/* ncclAllGather: `bytes` from every rank; recv holds nranks * bytes, rank r's
 * part at r * bytes.  Host buffers, synchronous. */
int gac_allgather(gac_comm *comm, const void *send, size_t bytes, void *recv);
/* parts of any size: *recv = malloc'd concatenation in rank order (free()),
 * counts[0 .. nranks) = each rank's bytes */
int gac_allgatherv(gac_comm *comm, const void *send, size_t bytes, void **recv, size_t *counts);
int gac_comm_barrier(gac_comm *comm);
void gac_comm_close(gac_comm *comm);

/* ---- device memory helpers (for callers without their own allocator) ---- */
int gac_dev_alloc(gac_ctx *ctx, size_t bytes, void **dptr);
int gac_dev_free(gac_ctx *ctx, void *dptr);
/* Synchronous copies, ordered after all work enqueued on the context's stream. */
int gac_memcpy_h2d(gac_ctx *ctx, void *dst, const void *src, size_t bytes);
int gac_memcpy_d2h(gac_ctx *ctx, void *dst, const void *src, size_t bytes);
int gac_synchronize(gac_ctx *ctx);

/* ---- kernel timing (HIP events on the launch stream) -------------------- */
#define GAC_K_PLAN 0     /* block-window search + scans + tile map (k_plan, k_tilemap_fused or k_scan_agg + k_tilemap) */
#define GAC_K_TILE 1     /* tile scoring: bases, gaps, per-tile scan (dominant) */
#define GAC_K_COMBINE 2  /* multi-tile range combine */
#define GAC_K_COUNT 3
#define GAC_PROF_ALL ((1 << GAC_K_COUNT) - 1)
/* Event timing of each launch of the kernels in `mask` (bits 1 << GAC_K_*;
 * 0 = off, GAC_PROF_ALL = all).  Each timed kernel adds two event markers
 * to the stream. */
int gac_prof_enable(gac_ctx *ctx, int mask);
/* Synchronise, fold recorded events, and return total ms + launch count of
 * kernel `k` since the last reset. */
int gac_prof_read(gac_ctx *ctx, int k, double *total_ms, int64_t *launches);
int gac_prof_reset(gac_ctx *ctx);

#ifdef __cplusplus
}
#endif
#endif /* GACHAIN_H */
