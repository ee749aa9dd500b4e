// gac_dp.h -- device layout of axtChain's chaining kernels (gac_dp.hip):
// the kd-tree DP (k_dp) and the crossover batch (k_xover).  gfx950 only.
//
// Per pair, the host-built kd-tree (kdBuild, kent/src/lib/chainBlock.c:124-
// 164) in pre-order with the hi child first, as structure-of-arrays:
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

hipError_t launch_dp(const DpArgs &a, int grid, hipStream_t s);
hipError_t launch_dp_fast(const DpArgs &a, int grid, hipStream_t s);
hipError_t launch_xover(const DpArgs &a, const XoverJob *jobs, int64_t n, int32_t *pos,
                        int32_t *adj, hipStream_t s);

}  // namespace gac
