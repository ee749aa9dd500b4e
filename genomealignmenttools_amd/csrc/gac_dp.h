// gac_dp.h -- device layout of axtChain's chaining kernels (gac_dp.hip):
// the kd-tree DP (k_dp) and the crossover batch (k_xover).  gfx950 only.
//
// Per pair, the kd-tree (kdBuild, kent/src/lib/chainBlock.c:124-164; built
// on the host, or on the device by gac_dptree.hip) in pre-order with the hi
// child first, as structure-of-arrays:
//   nd_a[v] = {maxQ, maxT, cut, lo}        internal node
//             {qEnd, tEnd, qStart, tStart} leaf node
//   nd_b[v] = {end of v's subtree, dim (0 = q, 1 = t) | ~leaf position}
//   nd_ms[v] = maxScore (mutable), nd_tot[v] = a leaf node's totalScore
// and its leaves in target order (findBestPredecessors' order):
//   lf[i] = {qStart, qEnd, tStart, tEnd}, lf_score[i], lf_node[i],
//   path[path_off[i] .. path_off[i+1]) = the nodes updateScoresOnWay visits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gac_kernels.h"

namespace gac {

struct DpPair {
    int64_t node_off;  // first node in nd_*
    int64_t leaf_off;  // first leaf in lf* / path_off
    int64_t tbase;     // global base index of the target sequence start
    int64_t qbase;     // '+': global base index of the query sequence start;
                       // '-': ~(global base index of its start + qSize)
    int32_t n_nodes;
    int32_t n_leaves;
};

struct DpArgs {
    const DpPair *pairs;
    int64_t n_pairs;
    long long *nd_ms;
    long long *nd_tot;
    const int4 *nd_a;
    const int2 *nd_b;
    const int4 *lf;
    const int32_t *lf_score;
    const int32_t *lf_node;
    const int64_t *path_off;  // [leaves + 1] (global)
    const int32_t *path;      // node indices within the pair
    long long *lf_total;      // out: totalScore per leaf
    int32_t *lf_pred;         // out: best predecessor node within the pair, or -1
    const uint2 *t_planes;
    const uint32_t *t_nmask;
    const uint2 *q_planes;
    const uint32_t *q_nmask;
    GapDev gap;
    const int32_t *small_tab;
    const int32_t *gap_tab;
    int32_t gap_len;
    int32_t m16[16];  // score matrix by 2-bit code [q * 4 + t] (T C A G)
    // the exact fast DP (k_dp_fast; see gac_dp.hip): the linear gap-cost
    // minorant s (dq + dt), s = lin_k / 1024, its per-node bound
    // nd_nw[v] = max over the subtree's scored leaves of 1024 total + lin_k
    // (qEnd + tEnd) (mutable), the smallest matrix entry, and per leaf the
    // leaf nodes of its overlapping candidates, ov[ov_off[i] .. ov_off[i+1])
    // (a -1 entry: too many, the leaf takes the reference search)
    long long *nd_nw;
    const int64_t *ov_off;  // [leaves + 1] (global)
    const int32_t *ov;
    long long lin_k;
    int32_t min_entry;
    int32_t pad;
    // GAC_DP_PROF: per-phase cycle counters of k_dp_fast (kDpProf slots,
    // summed over pairs), or null
    unsigned long long *prof;
    // k_dp_spec: set (32) when a wave gave up waiting for its turn (a
    // watchdog: the kernel then ends instead of spinning), or null
    int32_t *err;
};

// k_dp_fast's profile slots (GAC_DP_PROF)
enum DpProf {
    kPfLeaves, kPfWindows, kPfFbWindows, kPfFallbacks, kPfXoverWin, kPfOvChecks,
    kPfCycLoad, kPfCycSeed, kPfCycWalk, kPfCycAnom, kPfCycFb, kPfCycCommit, kPfCycXover,
    kPfNextWin, kPfNextSeq, kDpProf
};

// One overlapping adjacent block pair: left block ends at (lqe, lte), right
// block starts at (rqs, rts), ov bases overlap (strand coordinates).
struct XoverJob {
    int64_t tbase, qbase;  // as DpPair
    int32_t lqe, lte, rqs, rts;
    int32_t ov, pad;
};

// The DP's per-pair inputs built on the device from the pairs' blocks
// (gac_dptree.hip, gac_chain_dp_blocks): P pairs, B packed blocks (pair p's
// [blk_off[p], blk_off[p+1]), box = {qs, qe, ts, te}), L leaves, N nodes.
// The arrays after `tord` come out in the DpArgs layout above.
struct DtTree {
    int64_t P, B, L, N;
    int end_bit;  // radix sort key bits: 31 + bit length of P
    int fast;     // k_dp_fast: overlap lists too
    int32_t ov_cap;
    const int64_t *blk_off;  // [P + 1]
    const int4 *box;         // [B]
    const int32_t *score;    // [B]
    const unsigned long long *keys;  // [B] sorted (pair, tStart) keys
    const int32_t *tord;     // [B] blocks in that order: the first L are the leaves
    const int64_t *leaf_off; // [P + 1]
    const int64_t *node_off; // [P + 1]
    // scratch
    int32_t *pidx, *tpos, *qpos, *posd;  // [L], [B], [B], [B]
    unsigned long long *key2;            // [2L]
    int32_t *val2;                       // [2L]
    int32_t *ql, *tl, *spare;            // [L]
    int32_t *sstart, *slen, *snode;      // [L]
    int32_t *flag, *excl;                // [L]
    int32_t *ndep, *ndl;                 // [N]
    int4 *qbox;                          // [L]
    int32_t *qtp;                        // [L]
    int32_t *msz;                        // [P]
    uint8_t *over;                       // [L]
    long long *pcnt, *ocnt;              // [L + 1]
    int32_t *err;
    void *tmp;
    size_t tmp_bytes;
    // out (DpArgs inputs)
    int4 *na;           // [N]
    int2 *nb;           // [N]
    long long *tot, *ms, *nw;  // [N]
    int4 *lf;           // [L]
    int32_t *lsc, *lnode;      // [L]
    long long *poff, *ooff;    // [L + 1]
};

hipError_t dt_sort_pairs(void *tmp, size_t &tmp_bytes, const unsigned long long *kin,
                         unsigned long long *kout, const int32_t *vin, int32_t *vout, int64_t n,
                         int end_bit, hipStream_t s);
hipError_t dt_scan32(void *tmp, size_t &tmp_bytes, const int32_t *in, int32_t *out, int64_t n,
                     hipStream_t s);
hipError_t dt_scan64(void *tmp, size_t &tmp_bytes, const long long *in, long long *out, int64_t n,
                     hipStream_t s);
hipError_t launch_dt_keys(int64_t P, int64_t B, const int64_t *blk_off, const int2 *sizes,
                          const int4 *box, unsigned long long *keys, int32_t *vals, int32_t *err,
                          hipStream_t s);
hipError_t launch_dt_leaf_off(int64_t P, int64_t B, const unsigned long long *keys,
                              int64_t *leaf_off, hipStream_t s);
// leaves in query order and the tree (levels = splits of the largest pair)
hipError_t launch_dt_build(const DtTree &t, int levels, hipStream_t s);
// launch_dt_build, then path counts and offsets, overlap counts and offsets
// (t.fast)
hipError_t launch_dt_tree(const DtTree &t, int levels, hipStream_t s);
// the built trees in the host DP's layout (6 int32 per node: lo, hi, leaf,
// cut, maxQ, maxT), the target / query orders of the leaves as pair-local
// blocks, each block's leaf node (-1: none)
hipError_t launch_dt_host(const DtTree &t, int32_t *nodes, int32_t *out_t, int32_t *out_q,
                          int32_t *out_lnode, hipStream_t s);
// the paths and overlap lists into arrays of poff[L] / ooff[L] entries
hipError_t launch_dt_lists(const DtTree &t, int32_t *path, int32_t *ov, hipStream_t s);
// per packed block: totalScore, best predecessor (a block of its pair, or
// -1); per leaf: the target order as pair-local blocks
hipError_t launch_dt_out(const DtTree &t, const long long *lf_total, const int32_t *lf_pred,
                         int32_t *out_tord, long long *total, int32_t *pred, hipStream_t s);

hipError_t launch_dp(const DpArgs &a, int grid, hipStream_t s);
hipError_t launch_dp_fast(const DpArgs &a, int grid, hipStream_t s);
// k_dp_fast with `waves` (4, 8, 16) waves per pair searching consecutive
// leaves at once, committed in order (k_dp_spec)
hipError_t launch_dp_spec(const DpArgs &a, int grid, int waves, hipStream_t s);
hipError_t launch_xover(const DpArgs &a, const XoverJob *jobs, int64_t n, int32_t *pos,
                        int32_t *adj, hipStream_t s);

}  // namespace gac
