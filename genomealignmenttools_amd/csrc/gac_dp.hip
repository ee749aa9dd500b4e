// gac_dp.hip -- axtChain's chaining on the device:
//
//   k_dp     findBestPredecessors (kent/src/lib/chainBlock.c:207-300): the
//            kd-tree branch-and-bound DP that links ungapped blocks into
//            chains, one wave per (target, query, strand) pair, every pair of
//            a batch in one launch.  chainConnectCost and cBlockFindCrossover
//            (kent/src/lib/chainConnect.c:61-149) are device functions of it.
//   k_xover  cBlockFindCrossover for a batch of overlapping adjacent blocks
//            (chainRemovePartialOverlaps / scoreBlocks, chainConnect.c:255-344,
//            chainBlock.c:296-309): one wave per overlap, the crossover as a
//            wave prefix-sum + first-maximum scan over the overlap's bases.
//
// The DP is exact: the tree (built on the host, nodes in pre-order with the
// hi child first, kd_build in host/gac_axtchain.c) is searched in the
// reference's visiting order.  In that layout the DFS of bestPredecessor is
// a forward walk over node indices: a visited leaf continues at v+1, a pruned
// node at the end of its subtree, an internal node at v+1 (its hi child) when
// the lonely leaf lies past the cut and at its lo child otherwise.  A wave
// loads 64 consecutive nodes at once, evaluates every node's bound (the two
// `maxScore < best` tests) and every leaf's candidate score in parallel, and
// resolves the walk with an exclusive prefix-max of the skip ends: node u is
// visited iff no node before it skips past it.  `best` only changes at a
// visited leaf whose score beats it (strict >, as the reference), so each
// improvement is one more round over the rest of the window.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gac_dp.h"

#pragma clang fp contract(off)

namespace gac {

// ------------------------------------------------------------ gap cost ---
// gapCalcCost (kent/src/lib/gapCalc.c:298-331), the same operation order as
// gac_kernels.hip (k_block_gaps_flat) -- pinned there against the oracle
__device__ __forceinline__ int dp_interp(int x, const GapDev &g, int which) {
    const int n = g.long_count;
    const double *v = g.long_val[which];
    for (int i = 0; i < n; ++i) {
        const int ss = g.long_pos[i];
        if (x == ss) return (int)v[i];
        if (x < ss) {
            const int ds = ss - g.long_pos[i - 1];
            const double dv = v[i] - v[i - 1];
            const double prod = __dmul_rn(dv, (double)(x - g.long_pos[i - 1]));
            return (int)__dadd_rn(v[i - 1], __ddiv_rn(prod, (double)ds));
        }
    }
    const int ds = g.long_pos[n - 1] - g.long_pos[n - 2];
    const double dv = v[n - 1] - v[n - 2];
    const double prod = __dmul_rn(dv, (double)(x - g.long_pos[n - 2]));
    return (int)__dadd_rn(v[n - 2], __ddiv_rn(prod, (double)ds));
}

// chainConnectGapCost (chainConnect.c:108-112) = gapCalcCost(dq, dt)
__device__ __forceinline__ int dp_gap_cost(const DpArgs &a, int dq, int dt) {
    if (dt < 0) dt = 0;
    if (dq < 0) dq = 0;
    int which, d;
    if (dt == 0) {
        which = 0;
        d = dq;
    } else if (dq == 0) {
        which = 1;
        d = dt;
    } else {
        which = 2;
        d = dq + dt;
    }
    if (d < a.gap_len) return a.gap_tab[which * a.gap_len + d];
    const GapDev &g = a.gap;
    if (d < g.small_size) return a.small_tab[which * g.small_size + d];
    if (d >= g.last_pos[which])
        return (int)__dadd_rn(g.last_val[which],
                              __dmul_rn(g.last_slope[which], (double)(d - g.last_pos[which])));
    return dp_interp(d, g, which);
}

// ------------------------------------------------------------ bases ------
// 2-bit code (T C A G = 0..3) of global base g of a genome side, 4 for N
__device__ __forceinline__ int dp_code(const uint2 *planes, const uint32_t *nmask, int64_t g) {
    const int64_t w = g >> 5;
    const int s = (int)(g & 31);
    if ((nmask[w] >> s) & 1u) return 4;
    const uint2 p = planes[w];
    return (int)(((p.x >> s) & 1u) | (((p.y >> s) & 1u) << 1));
}

struct DpSeq {
    int64_t tbase;  // global base index of the target sequence start
    int64_t qbase;  // '+': of the query sequence start; '-': ~(start + qSize)
};

__device__ __forceinline__ int dp_tcode(const DpArgs &a, const DpSeq &s, int x) {
    return dp_code(a.t_planes, a.t_nmask, s.tbase + x);
}

// query base x of the pair's strand ('-': reverse complement, index arithmetic)
__device__ __forceinline__ int dp_qcode(const DpArgs &a, const DpSeq &s, int x) {
    if (s.qbase >= 0) return dp_code(a.q_planes, a.q_nmask, s.qbase + x);
    const int c = dp_code(a.q_planes, a.q_nmask, ~s.qbase - 1 - x);
    return c == 4 ? 4 : c ^ 2;
}

__device__ __forceinline__ int dp_msc(const int *m, int q, int t) {
    return (q == 4 || t == 4) ? 0 : m[q * 4 + t];
}

// cBlockFindCrossover (chainConnect.c:61-105), one lane: left block ends at
// (lqe, lte), right block starts at (rqs, rts), `ov` overlapping bases.
__device__ void dp_crossover(const DpArgs &a, const DpSeq &s, const int *m, int lqe, int lte,
                             int rqs, int rts, int ov, int &pos, int &adj) {
    long long r = 0, l = 0;
    for (int i = 0; i < ov; ++i) {
        r += dp_msc(m, dp_qcode(a, s, rqs + i), dp_tcode(a, s, rts + i));
        l += dp_msc(m, dp_qcode(a, s, lqe - ov + i), dp_tcode(a, s, lte - ov + i));
    }
    long long sc = r, best = r;
    int bp = 0;
    for (int i = 0; i < ov; ++i) {
        sc += dp_msc(m, dp_qcode(a, s, lqe - ov + i), dp_tcode(a, s, lte - ov + i));
        sc -= dp_msc(m, dp_qcode(a, s, rqs + i), dp_tcode(a, s, rts + i));
        if (sc > best) {
            best = sc;
            bp = i + 1;
        }
    }
    pos = bp;
    adj = (int)(r + l - best);
}

// chainConnectCost (chainConnect.c:114-149) of block A then block B; the
// caller guarantees A strictly before B (the reference's errAbort)
__device__ int dp_connect_cost(const DpArgs &a, const DpSeq &s, const int *m, int aqs, int aqe,
                               int ate, int bqs, int bqe, int bts) {
    int dq = bqs - aqe, dt = bts - ate, adj = 0;
    if (dq < 0 || dt < 0) {
        const int bsz = bqe - bqs, asz = aqe - aqs;
        const int ov = -min(dq, dt);
        if (ov >= bsz || ov >= asz) {
            adj = 100000000;
        } else {
            int pos;
            dp_crossover(a, s, m, aqe, ate, bqs, bts, ov, pos, adj);
            dq += ov;
            dt += ov;
        }
    }
    return adj + dp_gap_cost(a, dq, dt);
}

// ------------------------------------------------------------ k_dp -------
// Mutable node state (maxScore, leaf totals) is written and re-read by the
// same wave across leaves: loads of it are agent-scope atomics (no stale L1
// lines) and each leaf's updates are fenced before the next search.
__device__ __forceinline__ long long ld_mut(const long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(kWave) k_dp(DpArgs a) {
    __shared__ int s_m[16];
    const int lane = threadIdx.x;
    if (lane < 16) s_m[lane] = a.m16[lane];
    __syncthreads();
    for (int64_t pi = blockIdx.x; pi < a.n_pairs; pi += gridDim.x) {
        const DpPair P = a.pairs[pi];
        const DpSeq S = {P.tbase, P.qbase};
        long long *ms = a.nd_ms + P.node_off;
        long long *tot = a.nd_tot + P.node_off;
        const int4 *na = a.nd_a + P.node_off;
        const int2 *nb = a.nd_b + P.node_off;
        const int nn = P.n_nodes;
        for (int i = 0; i < P.n_leaves; ++i) {
            const int64_t li = P.leaf_off + i;
            const int4 L = a.lf[li];  // {qs, qe, ts, te}
            const int lq = L.x, lqe = L.y, lt = L.z;
            const long long ls = a.lf_score[li];
            long long best = 0;  // noBest: {NULL, 0}
            int best_node = -1;
            int p0 = 0;
            while (p0 < nn) {
                const int v = p0 + lane;
                const bool in = v < nn;
                long long M = 0, T = 0;
                int4 A = make_int4(0, 0, 0, 0);
                int2 B = make_int2(v + 1, 0);
                if (in) {
                    A = na[v];
                    B = nb[v];
                    M = ld_mut(ms + v);
                    if (B.y < 0) T = ld_mut(tot + v);
                }
                const bool leaf = B.y < 0;
                // bestPredecessor's two bound tests (chainBlock.c:222-232):
                // pruned iff min(M + ls, M + ls - gapCost) < best
                const long long m1 = M + ls;
                const long long m2 = m1 - dp_gap_cost(a, lq - A.x, lt - A.y);
                const long long key = m1 < m2 ? m1 : m2;
                // leaf: candidate score if it lies strictly before the lonely
                // leaf (chainBlock.c:236-246); leaf nodes carry qs/ts in z/w
                bool cand = false;
                long long sc = 0;
                if (in && leaf && A.z < lq && A.w < lt) {
                    cand = true;
                    sc = T + ls - dp_connect_cost(a, S, s_m, A.z, A.x, A.y, lq, lqe, lt);
                }
                // internal: the hi child (v + 1) only when the lonely leaf's
                // coordinate in this node's dimension is past the cut
                int nxt = v + 1;
                if (in && !leaf) {
                    const int coord = B.y == 0 ? lq : lt;
                    nxt = coord > A.z ? v + 1 : A.w;
                }
                int se = v + 1;  // end of what this node skips (frozen once resolved)
                int cur = 0;     // first lane not yet resolved
                for (;;) {
                    if (lane >= cur && in) se = key < best ? B.x : (leaf ? v + 1 : nxt);
                    int incl = se;
#pragma unroll
                    for (int d = 1; d < kWave; d <<= 1) {
                        const int o = __shfl_up(incl, d, kWave);
                        if (lane >= d) incl = max(incl, o);
                    }
                    int excl = __shfl_up(incl, 1, kWave);
                    if (lane == 0) excl = 0;
                    const bool visited = in && excl <= v;
                    const bool imp = visited && lane >= cur && cand && !(key < best) && sc > best;
                    const unsigned long long bal = __ballot(imp);
                    if (!bal) break;
                    const int u = __builtin_ctzll(bal);
                    best = __shfl(sc, u, kWave);
                    best_node = p0 + u;
                    cur = u + 1;
                }
                // the next visited node after the window: past every skip
                // interval that reaches beyond it (they nest)
                int mx = in ? se : 0;
#pragma unroll
                for (int d = 32; d > 0; d >>= 1) mx = max(mx, __shfl_xor(mx, d, kWave));
                p0 = max(p0 + kWave, mx);
            }
            // findBestPredecessors (chainBlock.c:289-297)
            long long total = ls;
            int pred = -1;
            if (best > ls) {
                total = best;
                pred = best_node;
            }
            if (lane == 0) {
                a.lf_total[li] = total;
                a.lf_pred[li] = pred;
                __hip_atomic_store(tot + a.lf_node[li], total, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            }
            // updateScoresOnWay (chainBlock.c:265-279): the nodes its descent
            // reaches (both sides on a tie with the cut), listed by the host
            const int64_t q0 = a.path_off[li], q1 = a.path_off[li + 1];
            for (int64_t k = q0 + lane; k < q1; k += kWave) {
                const int u = a.path[k];
                if (ld_mut(ms + u) < total)
                    __hip_atomic_store(ms + u, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        }
    }
}

hipError_t launch_dp(const DpArgs &a, int grid, hipStream_t s) {
    if (a.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_dp, dim3((unsigned)grid), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------ k_dp_fast --
// The exact fast DP (host: pair_dp_fast, gac_axtchain.c), one wave per pair.
// bestPredecessor's pruned DFS returns the first leaf in DFS order (= node
// order of the pre-order layout) of the best score among the candidates it
// does not prune, and its bounds are true upper bounds for every candidate
// that does not overlap the lonely leaf (gapCalcCost is monotone, checked on
// the host).  So unless an overlapping candidate is anomalous (its score
// exceeds a bound at its own leaf node, chainConnect.c:61-105's negative
// crossover adjustment), the answer is the maximum over all candidates, ties
// to the smallest node -- found here in any order:
//   A. the 64 previous leaves in target order (an LDS ring) that do not
//      overlap the lonely one, scored with the corner gap cost, give a first
//      best (the usual predecessor is a few leaves back);
//   B. the window walk of k_dp, pruning by max score, corner gap and the
//      linear bound of each subtree (all strict, so a subtree that could
//      hold a tie with a smaller node stays open), an improvement being a
//      greater score or an equal one at a smaller node;
//   C. every overlapping candidate of the leaf (listed by the host) that
//      could score at least the best while violating a bound at its leaf
//      sends the leaf to k_dp's reference walk (best from 0, max-score and
//      corner bounds, first strict improvement in DFS order).
// Mutable node state is read and written by this wave only: workgroup-scope
// atomics and fences (no L2 write-back per leaf, as an agent fence costs).
constexpr int kGapLds = 1024;  // gap costs by distance < kGapLds in LDS, per kind

__device__ __forceinline__ long long ld_wg(const long long *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void st_wg(long long *p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// k_dp_fast's LDS: the gap costs of short distances and the long-position
// tables of the interpolation, so a gap cost never waits on memory
struct DpGapLds {
    int gap[3 * kGapLds];
};

// dp_gap_cost with the short distances from LDS (computing the longer ones
// -- the interpolation's division -- measured slower than the L2-resident
// table: 5.2 vs 4.4 s on a 230 k-leaf pair, r05dp2)
__device__ __forceinline__ int dp_gap_lds(const DpArgs &a, const DpGapLds &G, int dq, int dt) {
    if (dt < 0) dt = 0;
    if (dq < 0) dq = 0;
    const int which = dt == 0 ? 0 : (dq == 0 ? 1 : 2);
    const int d = which == 0 ? dq : (which == 1 ? dt : dq + dt);
    if (d < kGapLds) return G.gap[which * kGapLds + d];
    return dp_gap_cost(a, dq, dt);
}

struct DpLeafCtx {
    int lq, lqe, lt, lte;
    long long ls;
};

// One window walk over the pair's nodes for the lonely leaf X.  FAST: the
// linear bound and tie-to-smaller-node improvements (best/best_node come in
// seeded); else the reference: max-score and corner bounds only, strict
// improvements, best from 0.
template <bool FAST>
__device__ void dp_walk(const DpArgs &a, const DpSeq &S, const int *m, const DpGapLds &sg,
                        const DpPair &P, const DpLeafCtx &X, long long kl, long long &best,
                        int &best_node) {
    const int lane = threadIdx.x & (kWave - 1);
    const long long *ms = a.nd_ms + P.node_off;
    const long long *nwp = a.nd_nw + P.node_off;
    const long long *tot = a.nd_tot + P.node_off;
    const int4 *na = a.nd_a + P.node_off;
    const int2 *nb = a.nd_b + P.node_off;
    const int nn = P.n_nodes;
    int p0 = 0;
    while (p0 < nn) {
        const int v = p0 + lane;
        const bool in = v < nn;
        long long M = 0, T = 0, NW = 0;
        int4 A = make_int4(0, 0, 0, 0);
        int2 B = make_int2(v + 1, 0);
        if (in) {
            A = na[v];
            B = nb[v];
            M = ld_wg(ms + v);
            if (FAST) NW = ld_wg(nwp + v);
            if (B.y < 0) T = ld_wg(tot + v);
        }
        const bool leaf = B.y < 0;
        const long long m1 = M + X.ls;
        const int gc = dp_gap_lds(a, sg, X.lq - A.x, X.lt - A.y);
        const long long m2 = m1 - gc;
        const long long key = m1 < m2 ? m1 : m2;
        bool cand = false;
        long long sc = 0;
        if (in && leaf && A.z < X.lq && A.w < X.lt) {
            cand = true;
            // a leaf node's corner is its block's end: a candidate that does
            // not overlap costs the corner gap just computed
            const int dq = X.lq - A.x, dt = X.lt - A.y;
            const int cost = (FAST && dq >= 0 && dt >= 0)
                                 ? gc
                                 : dp_connect_cost(a, S, m, A.z, A.x, A.y, X.lq, X.lqe, X.lt);
            sc = T + X.ls - cost;
        }
        int nxt = v + 1;
        if (in && !leaf) {
            const int coord = B.y == 0 ? X.lq : X.lt;
            nxt = coord > A.z ? v + 1 : A.w;
        }
        int se = v + 1;
        int cur = 0;
        for (;;) {
            const bool pruned = key < best || (FAST && NW - kl < 1024 * best);
            if (lane >= cur && in) se = pruned ? B.x : (leaf ? v + 1 : nxt);
            int incl = se;
#pragma unroll
            for (int d = 1; d < kWave; d <<= 1) {
                const int o = __shfl_up(incl, d, kWave);
                if (lane >= d) incl = max(incl, o);
            }
            int excl = __shfl_up(incl, 1, kWave);
            if (lane == 0) excl = 0;
            const bool visited = in && excl <= v;
            const bool better = sc > best || (FAST && sc == best && v < best_node);
            const bool imp = visited && lane >= cur && cand && !pruned && better;
            const unsigned long long bal = __ballot(imp);
            if (!bal) break;
            const int u = __builtin_ctzll(bal);
            best = __shfl(sc, u, kWave);
            best_node = p0 + u;
            cur = u + 1;
        }
        int mx = in ? se : 0;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) mx = max(mx, __shfl_xor(mx, d, kWave));
        p0 = max(p0 + kWave, mx);
    }
}

__global__ void __launch_bounds__(kWave) k_dp_fast(DpArgs a) {
    __shared__ int s_m[16];
    __shared__ DpGapLds s_gap;
    __shared__ int4 r_box[kWave];  // the previous 64 leaves: {qs, qe, ts, te}
    __shared__ long long r_tot[kWave];
    __shared__ int r_node[kWave];
    const int lane = threadIdx.x;
    if (lane < 16) s_m[lane] = a.m16[lane];
    for (int k = lane; k < 3 * kGapLds; k += kWave) {
        const int which = k / kGapLds, d = k % kGapLds;
        s_gap.gap[k] = which == 0 ? dp_gap_cost(a, d, 0)
                                  : (which == 1 ? dp_gap_cost(a, 0, d)
                                                : (d >= 2 ? dp_gap_cost(a, 1, d - 1) : 0));
    }
    __syncthreads();
    for (int64_t pi = blockIdx.x; pi < a.n_pairs; pi += gridDim.x) {
        const DpPair P = a.pairs[pi];
        const DpSeq S = {P.tbase, P.qbase};
        long long *ms = a.nd_ms + P.node_off;
        long long *nwp = a.nd_nw + P.node_off;
        long long *tot = a.nd_tot + P.node_off;
        const int2 *nb = a.nd_b + P.node_off;
        r_node[lane] = -1;
        __syncthreads();
        for (int i = 0; i < P.n_leaves; ++i) {
            const int64_t li = P.leaf_off + i;
            // every per-leaf record at once (one round trip, not one per stage)
            const int4 L = a.lf[li];  // {qs, qe, ts, te}
            const int node = a.lf_node[li];
            const int64_t q0 = a.path_off[li], q1 = a.path_off[li + 1];
            const int64_t o0 = a.ov_off[li], o1 = a.ov_off[li + 1];
            DpLeafCtx X;
            X.lq = L.x;
            X.lqe = L.y;
            X.lt = L.z;
            X.lte = L.w;
            X.ls = a.lf_score[li];
            const long long kl = a.lin_k * ((long long)X.lq + X.lt) - 1024 * X.ls;
            // ---- A: the ring's non-overlapping candidates
            long long best = 0;
            int best_node = -1;
            {
                const int4 bx = r_box[lane];
                const int nd = r_node[lane];
                long long sc = -1;
                if (nd >= 0 && bx.x < X.lq && bx.z < X.lt) {
                    const int dq = X.lq - bx.y, dt = X.lt - bx.w;
                    if (dq >= 0 && dt >= 0) sc = r_tot[lane] + X.ls - dp_gap_lds(a, s_gap, dq, dt);
                }
                // max score, ties to the smaller node; > 0 only
                long long bs = sc > 0 ? sc : -1;
                int bn = sc > 0 ? nd : 0x7fffffff;
#pragma unroll
                for (int d = 32; d > 0; d >>= 1) {
                    const long long os = __shfl_xor(bs, d, kWave);
                    const int on = __shfl_xor(bn, d, kWave);
                    if (os > bs || (os == bs && on < bn)) {
                        bs = os;
                        bn = on;
                    }
                }
                if (bs > 0) {
                    best = bs;
                    best_node = bn;
                }
            }
            // ---- B: the fast walk
            dp_walk<true>(a, S, s_m, s_gap, P, X, kl, best, best_node);
            // ---- C: anomalies among the overlapping candidates
            bool fb = false;
            {
                const long long need = best > 0 ? best : 1;
                const int lsize = X.lqe - X.lq;
                for (int64_t k = o0 + lane; k < o1; k += kWave) {
                    const int c = a.ov[k];
                    if (c < 0) {
                        fb = true;
                        continue;
                    }
                    const int cpos = ~nb[c].y;
                    const int4 cb = a.lf[P.leaf_off + cpos];  // {qs, qe, ts, te}
                    const int dq = X.lq - cb.y, dt = X.lt - cb.w;
                    const int ov = -(dq < dt ? dq : dt);
                    if (ov >= lsize || ov >= cb.y - cb.x) continue;  // connect cost 1e8
                    const long long tc = ld_wg(tot + c);
                    const long long ub = tc + X.ls - dp_gap_lds(a, s_gap, dq + ov, dt + ov) -
                                         (long long)ov * a.min_entry;
                    if (ub < need) continue;
                    const long long sc =
                        tc + X.ls - dp_connect_cost(a, S, s_m, cb.x, cb.y, cb.w, X.lq, X.lqe, X.lt);
                    if (sc < need) continue;
                    const long long bc = tc + X.ls - dp_gap_lds(a, s_gap, dq, dt);
                    const long long bl = 1024 * tc - a.lin_k * ((long long)dq + dt) + 1024 * X.ls;
                    if (sc > bc || 1024 * sc > bl) fb = true;
                }
            }
            if (__ballot(fb)) {
                best = 0;
                best_node = -1;
                dp_walk<false>(a, S, s_m, s_gap, P, X, 0, best, best_node);
            }
            // ---- D: findBestPredecessors (chainBlock.c:289-297) + updateScoresOnWay
            long long total = X.ls;
            int pred = -1;
            if (best > X.ls) {
                total = best;
                pred = best_node;
            }
            if (lane == 0) {
                a.lf_total[li] = total;
                a.lf_pred[li] = pred;
                st_wg(tot + node, total);
                r_box[i & (kWave - 1)] = L;
                r_tot[i & (kWave - 1)] = total;
                r_node[i & (kWave - 1)] = node;
            }
            const long long nwv = 1024 * total + a.lin_k * ((long long)X.lqe + X.lte);
            for (int64_t k = q0 + lane; k < q1; k += kWave) {
                const int u = a.path[k];
                if (ld_wg(ms + u) < total) st_wg(ms + u, total);
                if (ld_wg(nwp + u) < nwv) st_wg(nwp + u, nwv);
            }
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
            __syncthreads();
        }
        __syncthreads();
    }
}

hipError_t launch_dp_fast(const DpArgs &a, int grid, hipStream_t s) {
    if (a.n_pairs == 0) return hipSuccess;
    hipLaunchKernelGGL(k_dp_fast, dim3((unsigned)grid), dim3(kWave), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------ k_xover ----
// One wave per overlap: lane i scores overlap base k = base + i on both
// blocks, d_k = left - right; the crossover is the first k where the prefix
// sum D_k = d_0 + .. + d_k reaches its maximum, if that maximum is > 0
// (cBlockFindCrossover keeps the first strict improvement over the right
// block's score): pos = k + 1, adj = lScore - max(0, max D).
__global__ void __launch_bounds__(256) k_xover(DpArgs a, const XoverJob *jobs, int64_t n,
                                               int32_t *out_pos, int32_t *out_adj) {
    __shared__ int s_m[16];
    if (threadIdx.x < 16) s_m[threadIdx.x] = a.m16[threadIdx.x];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t wave_id = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t j = wave_id; j < n; j += nwaves) {
        const XoverJob J = jobs[j];
        const DpSeq S = {J.tbase, J.qbase};
        long long carry = 0, lsum = 0, bestv = 0;
        int bestpos = 0;
        for (int base = 0; base < J.ov; base += kWave) {
            const int k = base + lane;
            long long d = 0, l = 0;
            if (k < J.ov) {
                l = dp_msc(s_m, dp_qcode(a, S, J.lqe - J.ov + k), dp_tcode(a, S, J.lte - J.ov + k));
                const long long r = dp_msc(s_m, dp_qcode(a, S, J.rqs + k), dp_tcode(a, S, J.rts + k));
                d = l - r;
            }
            long long incl = d;
#pragma unroll
            for (int s = 1; s < kWave; s <<= 1) {
                const long long o = __shfl_up(incl, s, kWave);
                if (lane >= s) incl += o;
            }
            const long long D = carry + incl;
            // first maximum of D over this segment's valid lanes
            long long mv = k < J.ov ? D : (long long)INT64_MIN;
            int mk = k;
#pragma unroll
            for (int s = 32; s > 0; s >>= 1) {
                const long long ov2 = __shfl_xor(mv, s, kWave);
                const int ok2 = __shfl_xor(mk, s, kWave);
                if (ov2 > mv || (ov2 == mv && ok2 < mk)) {
                    mv = ov2;
                    mk = ok2;
                }
            }
            if (mv > bestv) {  // strict: an earlier segment's equal maximum wins
                bestv = mv;
                bestpos = mk + 1;
            }
            carry = __shfl(incl, kWave - 1, kWave) + carry;
            long long ls = l;
#pragma unroll
            for (int s = 32; s > 0; s >>= 1) ls += __shfl_xor(ls, s, kWave);
            lsum += ls;
        }
        if (lane == 0) {
            out_pos[j] = bestpos;
            out_adj[j] = (int32_t)(lsum - bestv);
        }
    }
}

hipError_t launch_xover(const DpArgs &a, const XoverJob *jobs, int64_t n, int32_t *pos,
                        int32_t *adj, hipStream_t s) {
    if (n == 0) return hipSuccess;
    int64_t nb = (n + 3) / 4;
    if (nb > 8192) nb = 8192;
    hipLaunchKernelGGL(k_xover, dim3((unsigned)nb), dim3(256), 0, s, a, jobs, n, pos, adj);
    return hipGetLastError();
}

}  // namespace gac
