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
    const uint32_t nm = nmask[w];  // (both loads in flight at once)
    const uint2 p = planes[w];
    if ((nm >> s) & 1u) return 4;
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

// ------------------------------------------------------------ wave scans --
// On DPP (row_shr 1/2/4/8 inside each 16-lane row, row_bcast15/31 across
// rows, wave_shr:1 for the exclusive shift): VALU moves, no LDS round trip
// per step as __shfl_up's ds_bpermute costs -- the walk runs a prefix max
// per improvement round and window.
template <int CTRL, int RM>
__device__ __forceinline__ int dp_dpp(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, RM, 0xf, true);
}

// inclusive prefix max over the wave
__device__ __forceinline__ int dp_wave_incl_max(int v, int lane) {
    int o;
    o = dp_dpp<0x111, 0xf>(v);
    if ((lane & 15) >= 1) v = max(v, o);
    o = dp_dpp<0x112, 0xf>(v);
    if ((lane & 15) >= 2) v = max(v, o);
    o = dp_dpp<0x114, 0xf>(v);
    if ((lane & 15) >= 4) v = max(v, o);
    o = dp_dpp<0x118, 0xf>(v);
    if ((lane & 15) >= 8) v = max(v, o);
    o = dp_dpp<0x142, 0xa>(v);  // row_bcast:15 into rows 1 and 3
    if (lane & 16) v = max(v, o);
    o = dp_dpp<0x143, 0xc>(v);  // row_bcast:31 into rows 2 and 3
    if (lane >= 32) v = max(v, o);
    return v;
}

// the wave's maximum (int64) / minimum (int), in every lane: an inclusive
// scan on DPP, then the last lane's value
__device__ __forceinline__ long long dp_dpp64_max_step(long long v, long long o, bool ok) {
    return ok && o > v ? o : v;
}
template <int CTRL, int RM>
__device__ __forceinline__ long long dp_dpp64(long long v) {
    const unsigned long long u = (unsigned long long)v;
    const uint32_t lo = (uint32_t)dp_dpp<CTRL, RM>((int)(uint32_t)u);
    const uint32_t hi = (uint32_t)dp_dpp<CTRL, RM>((int)(uint32_t)(u >> 32));
    return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ long long dp_wave_max64(long long v, int lane) {
    v = dp_dpp64_max_step(v, dp_dpp64<0x111, 0xf>(v), (lane & 15) >= 1);
    v = dp_dpp64_max_step(v, dp_dpp64<0x112, 0xf>(v), (lane & 15) >= 2);
    v = dp_dpp64_max_step(v, dp_dpp64<0x114, 0xf>(v), (lane & 15) >= 4);
    v = dp_dpp64_max_step(v, dp_dpp64<0x118, 0xf>(v), (lane & 15) >= 8);
    v = dp_dpp64_max_step(v, dp_dpp64<0x142, 0xa>(v), (lane & 16) != 0);
    v = dp_dpp64_max_step(v, dp_dpp64<0x143, 0xc>(v), lane >= 32);
    const unsigned long long u = (unsigned long long)v;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, kWave - 1);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), kWave - 1);
    return (long long)(((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ int dp_wave_min32(int v, int lane) {
    return -__builtin_amdgcn_readlane(dp_wave_incl_max(-v, lane), kWave - 1);
}

// lane u's value (u wave-uniform)
__device__ __forceinline__ long long dp_readlane64(long long v, int u) {
    const unsigned long long x = (unsigned long long)v;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), u);
    return (long long)(((unsigned long long)hi << 32) | lo);
}

// the previous lane's value (lane 0: 0)
__device__ __forceinline__ int dp_wave_shr1(int v) { return dp_dpp<0x138, 0xf>(v); }

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
constexpr int kLbOct = 22;     // octaves 2^10 .. 2^31 of the lower-bound grid
constexpr int kLbN = 4 * kLbOct;

// the lower-bound grid: point i = (4 + i % 4) << (i / 4 + 8) (>= kGapLds)
__host__ __device__ inline int64_t dp_lb_point(int i) { return (int64_t)(4 + (i & 3)) << ((i >> 2) + 8); }
// the last grid point <= d (d >= kGapLds)
__device__ __forceinline__ int dp_lb_index(int d) {
    const int e = 31 - __clz(d);               // d in [2^e, 2^(e+1)), e >= 10
    return ((e - 10) << 2) + ((d >> (e - 2)) & 3);
}

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
    int lpos[kMaxLong];
    double lval[3][kMaxLong];
    // gapCalcCost's per-kind scalars (read with a per-lane kind: from the
    // kernel arguments that was a vector load and a wait per gap cost)
    int last_pos[3];
    int small_size, long_count;
    double last_val[3], last_slope[3];
    // k_dp_fast's pruning bound past kGapLds: the cost at the grid point at
    // or below d (4 points per octave, kLbOct octaves from kGapLds) -- a
    // lower bound of gapCalcCost, which k_dp_fast only runs with when it is
    // monotone in each distance (dp_fast_setup, host)
    int lb[3][kLbN];
};

// interpolate (gapCalc.c:82-104) over the LDS copy of the long tables: the
// first long position >= x by binary search (the reference's linear scan
// stops at the same one), then its operation order
__device__ __forceinline__ int dp_interp_lds(const DpGapLds &G, int n, int x, int which) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (G.lpos[mid] < x)
            lo = mid + 1;
        else
            hi = mid;
    }
    const double *v = G.lval[which];
    if (lo < n && G.lpos[lo] == x) return (int)v[lo];
    // past the last position: the last two; (lo == 0, x below every long
    // position, cannot happen: x >= smallSize here)
    const int i = lo == n ? n - 1 : (lo < 1 ? 1 : lo);
    const int p0 = G.lpos[i - 1];
    const int ds = G.lpos[i] - p0;
    const double dv = v[i] - v[i - 1];
    const double prod = __dmul_rn(dv, (double)(x - p0));
    return (int)__dadd_rn(v[i - 1], __ddiv_rn(prod, (double)ds));
}

// dp_gap_cost without a memory round trip: short distances from the LDS
// table, the long ones by gapCalcCost's own branches (gapCalc.c:298-331) on
// the LDS long tables (a table read from L2 was one more dependent round
// trip per search window; r06dp1: 2.6 k cycles per window)
__device__ __forceinline__ int dp_gap_lds(const DpArgs &a, const DpGapLds &G, int dq, int dt) {
    if (dt < 0) dt = 0;
    if (dq < 0) dq = 0;
    const int which = dt == 0 ? 0 : (dq == 0 ? 1 : 2);
    const int d = which == 0 ? dq : (which == 1 ? dt : dq + dt);
    if (d < kGapLds) return G.gap[which * kGapLds + d];
    if (d < G.small_size) return a.small_tab[which * G.small_size + d];
    const int lp = G.last_pos[which];
    if (d >= lp) return (int)__dadd_rn(G.last_val[which], __dmul_rn(G.last_slope[which], (double)(d - lp)));
    return dp_interp_lds(G, G.long_count, d, which);
}

// a lower bound of dp_gap_lds (exact below kGapLds): what pruning needs
__device__ __forceinline__ int dp_gap_lb(const DpGapLds &G, int dq, int dt) {
    if (dt < 0) dt = 0;
    if (dq < 0) dq = 0;
    const int which = dt == 0 ? 0 : (dq == 0 ? 1 : 2);
    const int d = which == 0 ? dq : (which == 1 ? dt : dq + dt);
    if (d < kGapLds) return G.gap[which * kGapLds + d];
    return G.lb[which][dp_lb_index(d)];
}

struct DpLeafCtx {
    int lq, lqe, lt, lte;
    long long ls;
};

// One window walk over the pair's nodes for the lonely leaf X.  FAST: the
// linear bound and tie-to-smaller-node improvements (best/best_node come in
// seeded); else the reference: max-score and corner bounds only, strict
// improvements, best from 0.
// per-wave profile counters (GAC_DP_PROF; wave-uniform)
struct DpPf {
    unsigned long long v[kDpProf];
};

template <bool FAST>
__device__ void dp_walk(const DpArgs &a, const DpSeq &S, const int *m, const DpGapLds &sg,
                        const DpPair &P, const DpLeafCtx &X, long long kl, long long &best,
                        int &best_node, DpPf &pf, bool prof) {
    const int lane = threadIdx.x & (kWave - 1);
    const long long *ms = a.nd_ms + P.node_off;
    const long long *nwp = a.nd_nw + P.node_off;
    const long long *tot = a.nd_tot + P.node_off;
    const int4 *na = a.nd_a + P.node_off;
    const int2 *nb = a.nd_b + P.node_off;
    const int nn = P.n_nodes;
    int p0 = 0;
    while (p0 < nn) {
        unsigned long long c0 = 0;
        if (prof) {
            __builtin_amdgcn_sched_barrier(0);
            c0 = clock64();
            __builtin_amdgcn_sched_barrier(0);
        }
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
            T = ld_wg(tot + v);  // (every node has a slot: no wait on B first)
        }
        const bool leaf = B.y < 0;
        const long long m1 = M + X.ls;
        // FAST: the bound with the gap cost's lower bound (looser, still
        // true); the reference walk needs bestPredecessor's exact one
        const int gc = FAST ? dp_gap_lb(sg, X.lq - A.x, X.lt - A.y) : dp_gap_lds(a, sg, X.lq - A.x, X.lt - A.y);
        const long long m2 = m1 - gc;
        const long long key = m1 < m2 ? m1 : m2;
        bool cand = false;
        long long sc = 0;
        if (prof) {
            // (the bounds of the window's nodes are ready: their loads and
            // gap costs done)
            volatile long long sink = key;
            (void)sink;
            __builtin_amdgcn_sched_barrier(0);
            pf.v[kPfCycXover] += clock64() - c0;
            __builtin_amdgcn_sched_barrier(0);
            ++pf.v[FAST ? kPfWindows : kPfFbWindows];
            if (__ballot(in && leaf && A.z < X.lq && A.w < X.lt && (X.lq < A.x || X.lt < A.y)))
                ++pf.v[kPfXoverWin];
        }
        if (in && leaf && A.z < X.lq && A.w < X.lt) {
            cand = true;
            // a leaf node's corner is its block's end: a candidate that does
            // not overlap costs the corner gap just computed
            const int dq = X.lq - A.x, dt = X.lt - A.y;
            const int cost = (FAST && dq >= 0 && dt >= 0)
                                 ? dp_gap_lds(a, sg, dq, dt)
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
        int incl;
        for (;;) {
            const bool pruned = key < best || (FAST && NW - kl < 1024 * best);
            if (lane >= cur && in) se = pruned ? B.x : (leaf ? v + 1 : nxt);
            incl = dp_wave_incl_max(se, lane);
            const int excl = dp_wave_shr1(incl);
            const bool visited = in && excl <= v;
            const bool better = sc > best || (FAST && sc == best && v < best_node);
            const bool imp = visited && lane >= cur && cand && !pruned && better;
            const unsigned long long bal = __ballot(imp);
            if (!bal) break;
            const int u = __builtin_ctzll(bal);
            best = dp_readlane64(sc, u);
            best_node = p0 + u;
            cur = u + 1;
        }
        // the next visited node after the window: past every skip interval
        // that reaches beyond it (they nest) -- the last lane's prefix max
        // (lanes past the pair's end only push it past the end too)
        const int nx = max(p0 + kWave, __builtin_amdgcn_readlane(incl, kWave - 1));
        if (prof && nx < nn) {  // (the walk goes on: contiguously, or by a jump)
            ++pf.v[kPfNextWin];
            if (nx == p0 + kWave) ++pf.v[kPfNextSeq];
        }
        p0 = nx;
    }
}

// k_dp_fast's step C (the host's dp_anomaly): one of the leaf's overlapping
// candidates ov[o0 .. o1) (leaf nodes; -1: too many listed) could score at
// least `best` while violating a bound at its own leaf -- the leaf then takes
// the reference search order.  Wave-uniform result.
__device__ __forceinline__ bool dp_anomaly_check(const DpArgs &a, const DpSeq &S, const int *m,
                                                 const DpGapLds &sg, const DpPair &P,
                                                 const DpLeafCtx &X, const int2 *nb,
                                                 const long long *tot, int64_t o0, int64_t o1,
                                                 long long best) {
    const int lane = threadIdx.x & (kWave - 1);
    bool fb = false;
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
        const long long ub = tc + X.ls - dp_gap_lds(a, sg, dq + ov, dt + ov) - (long long)ov * a.min_entry;
        if (ub < need) continue;
        const long long sc = tc + X.ls - dp_connect_cost(a, S, m, cb.x, cb.y, cb.w, X.lq, X.lqe, X.lt);
        if (sc < need) continue;
        const long long bc = tc + X.ls - dp_gap_lds(a, sg, dq, dt);
        const long long bl = 1024 * tc - a.lin_k * ((long long)dq + dt) + 1024 * X.ls;
        if (sc > bc || 1024 * sc > bl) fb = true;
    }
    return __ballot(fb) != 0;
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
    if (lane < kMaxLong) {
        s_gap.lpos[lane] = a.gap.long_pos[lane];
        for (int w = 0; w < 3; ++w) s_gap.lval[w][lane] = a.gap.long_val[w][lane];
    }
    for (int k = lane; k < 3 * kLbN; k += kWave) {
        const int which = k / kLbN, i = k % kLbN;
        const int64_t x = dp_lb_point(i);
        const int d = x > 0x7fffffff ? 0x7fffffff : (int)x;
        s_gap.lb[which][i] = which == 0 ? dp_gap_cost(a, d, 0)
                                        : (which == 1 ? dp_gap_cost(a, 0, d) : dp_gap_cost(a, 1, d - 1));
    }
    if (lane < 3) {
        s_gap.last_pos[lane] = a.gap.last_pos[lane];
        s_gap.last_val[lane] = a.gap.last_val[lane];
        s_gap.last_slope[lane] = a.gap.last_slope[lane];
    }
    if (lane == 0) {
        s_gap.small_size = a.gap.small_size;
        s_gap.long_count = a.gap.long_count;
    }
    __syncthreads();
    const bool prof = a.prof != nullptr;
    DpPf pf;
    for (int k = 0; k < kDpProf; ++k) pf.v[k] = 0;
    unsigned long long ck = prof ? clock64() : 0;
    // GAC_DP_PROF: the cycles since the last lap into slot k
#define DP_LAP(k)                        \
    if (prof) {                          \
        const unsigned long long t_ = clock64(); \
        pf.v[k] += t_ - ck;              \
        ck = t_;                         \
    }
    for (int64_t pi = blockIdx.x; pi < a.n_pairs; pi += gridDim.x) {
        const DpPair P = a.pairs[pi];
        const DpSeq S = {P.tbase, P.qbase};
        long long *ms = a.nd_ms + P.node_off;
        long long *nwp = a.nd_nw + P.node_off;
        long long *tot = a.nd_tot + P.node_off;
        const int2 *nb = a.nd_b + P.node_off;
        r_node[lane] = -1;
        __syncthreads();
        // every per-leaf record at once, the next leaf's loaded while this
        // one is searched (software pipelined: no round trip of its own)
        int4 nL = make_int4(0, 0, 0, 0);
        int n_node = 0, n_ls = 0;
        int64_t n_q1 = 0, n_o1 = 0, q1 = 0, o1 = 0;
        if (P.n_leaves > 0) {
            const int64_t l0 = P.leaf_off;
            nL = a.lf[l0];
            n_node = a.lf_node[l0];
            n_ls = a.lf_score[l0];
            q1 = a.path_off[l0];
            o1 = a.ov_off[l0];
            n_q1 = a.path_off[l0 + 1];
            n_o1 = a.ov_off[l0 + 1];
        }
        for (int i = 0; i < P.n_leaves; ++i) {
            const int64_t li = P.leaf_off + i;
            const int4 L = nL;  // {qs, qe, ts, te}
            const int node = n_node;
            const int64_t q0 = q1, o0 = o1;
            q1 = n_q1;
            o1 = n_o1;
            DpLeafCtx X;
            X.lq = L.x;
            X.lqe = L.y;
            X.lt = L.z;
            X.lte = L.w;
            X.ls = n_ls;
            if (i + 1 < P.n_leaves) {
                nL = a.lf[li + 1];
                n_node = a.lf_node[li + 1];
                n_ls = a.lf_score[li + 1];
                n_q1 = a.path_off[li + 2];
                n_o1 = a.ov_off[li + 2];
            }
            const long long kl = a.lin_k * ((long long)X.lq + X.lt) - 1024 * X.ls;
            if (prof) ++pf.v[kPfLeaves];
            DP_LAP(kPfCycLoad)
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
                const long long bs = dp_wave_max64(sc > 0 ? sc : -1, lane);
                if (bs > 0) {
                    best = bs;
                    best_node = dp_wave_min32(sc == bs ? nd : 0x7fffffff, lane);
                }
            }
            DP_LAP(kPfCycSeed)
            // ---- B: the fast walk
            dp_walk<true>(a, S, s_m, s_gap, P, X, kl, best, best_node, pf, prof);
            DP_LAP(kPfCycWalk)
            // ---- C: anomalies among the overlapping candidates
            if (prof) pf.v[kPfOvChecks] += o1 - o0;
            const bool fb = dp_anomaly_check(a, S, s_m, s_gap, P, X, nb, tot, o0, o1, best);
            DP_LAP(kPfCycAnom)
            if (fb) {
                best = 0;
                best_node = -1;
                if (prof) ++pf.v[kPfFallbacks];
                dp_walk<false>(a, S, s_m, s_gap, P, X, 0, best, best_node, pf, prof);
                DP_LAP(kPfCycFb)
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
            DP_LAP(kPfCycCommit)
        }
        __syncthreads();
    }
#undef DP_LAP
    if (prof && lane < kDpProf) {
        unsigned long long v = 0;
        for (int k = 0; k < kDpProf; ++k)
            if (k == lane) v = pf.v[k];
        atomicAdd(a.prof + lane, v);
    }
}

// ------------------------------------------------------------ k_dp_spec --
// k_dp_fast with W waves per pair, searching W consecutive leaves (target
// order) at once and committing them in order -- the device form of the
// host's searcher/committer team (pair_dp_team).  Wave w takes leaves w,
// w + W, ...; leaf i:
//   1. snapshot c0 = the count of committed leaves (every leaf < c0 has its
//      total and its update path's bounds in the tree);
//   2. seed from the ring's leaves in [c0 - 64 + W, c0) (slots no commit in
//      flight can overwrite) and run the fast walk on the tree as it is:
//      its bounds include every leaf < c0, so the walk's best is the exact
//      maximum over the candidates < c0 (ties to the smaller node), joined
//      by at most some of [c0, i) with totals <= their final ones;
//   3. wait for its turn (c = i), then score the leaves [c0, i) exactly from
//      the ring (final totals now) and keep the better of each: the maximum
//      over every candidate < i, as findBestPredecessors' in-order search;
//   4. the anomaly check on final totals (k_dp_fast's step C) and, when it
//      fires, the reference-order walk on the final tree;
//   5. commit (total, update path, ring slot) and release c = i + 1.
// Bounds only grow, so a walk on a tree that lacks some of [c0, i) prunes
// only subtrees whose leaves < c0 cannot reach its best: steps 2-3 give the
// exact result without searching again.
// cBlockFindCrossover's adjustment (chainConnect.c:61-105) with the whole
// wave (arguments wave-uniform): lane k scores overlap base k of both blocks
// (left - right), the best crossover is where the prefix sum peaks (k_xover)
__device__ long long dp_crossover_adj_wave(const DpArgs &a, const DpSeq &S, const int *m, int lqe,
                                           int lte, int rqs, int rts, int ov) {
    const int lane = threadIdx.x & (kWave - 1);
    long long carry = 0, lsum = 0, bestv = 0;
    for (int base = 0; base < ov; base += kWave) {
        const int k = base + lane;
        long long d = 0, l = 0;
        if (k < ov) {
            l = dp_msc(m, dp_qcode(a, S, lqe - ov + k), dp_tcode(a, S, lte - ov + k));
            d = l - dp_msc(m, dp_qcode(a, S, rqs + k), dp_tcode(a, S, rts + k));
        }
        long long incl = d;
#pragma unroll
        for (int sh = 1; sh < kWave; sh <<= 1) {
            const long long o = __shfl_up(incl, sh, kWave);
            if (lane >= sh) incl += o;
        }
        const long long mx = dp_wave_max64(k < ov ? carry + incl : (long long)INT64_MIN, lane);
        bestv = mx > bestv ? mx : bestv;
        carry += dp_readlane64(incl, kWave - 1);
        long long ls = l;
#pragma unroll
        for (int sh = 32; sh > 0; sh >>= 1) ls += __shfl_xor(ls, sh, kWave);
        lsum += ls;
    }
    return lsum - bestv;
}

// k_dp_spec: fold the candidates among committed leaves [j0, j1) (their ring
// slots) into (best, best_node), exactly: a bound first (an overlapping one's
// crossover costs at least ov * min_entry), the exact cost only where the
// bound can reach the best, an overlap's crossover on the whole wave
__device__ void dp_spec_fold(const DpArgs &a, const DpSeq &S, const int *m, const DpGapLds &sg,
                             const DpLeafCtx &X, const int4 *r_box, const long long *r_tot,
                             const int *r_node, int j0, int j1, long long &best, int &best_node) {
    const int lane = threadIdx.x & (kWave - 1);
    for (int jb = j0; jb < j1; jb += kWave) {
        const int j = jb + lane;
        long long sc = -1;
        int nd = 0x7fffffff;
        bool need_x = false;  // an overlap whose bound reaches the best
        int4 bx = make_int4(0, 0, 0, 0);
        long long tj = 0;
        if (j < j1) {
            const int slot = j & (kWave - 1);
            bx = r_box[slot];  // {qs, qe, ts, te}
            if (bx.x < X.lq && bx.z < X.lt) {
                tj = r_tot[slot];
                const int dq = X.lq - bx.y, dt = X.lt - bx.w;
                if (dq >= 0 && dt >= 0) {
                    sc = tj + X.ls - dp_gap_lds(a, sg, dq, dt);
                    nd = r_node[slot];
                } else {
                    const int ov = -(dq < dt ? dq : dt);
                    nd = r_node[slot];
                    if (ov < X.lqe - X.lq && ov < bx.y - bx.x) {
                        const long long ub = tj + X.ls - dp_gap_lds(a, sg, dq + ov, dt + ov) -
                                             (long long)ov * a.min_entry;
                        need_x = ub > 0 && ub >= best;
                    } else {  // (cost 1e8: no crossover)
                        sc = tj + X.ls - dp_connect_cost(a, S, m, bx.x, bx.y, bx.w, X.lq, X.lqe, X.lt);
                    }
                }
            }
        }
        unsigned long long need = __ballot(need_x);
        while (need) {  // (rare: one overlap at a time, on the whole wave)
            const int u = __builtin_ctzll(need);
            need &= need - 1;
            const int uqs = __shfl(bx.x, u), uqe = __shfl(bx.y, u), ute = __shfl(bx.w, u);
            const int dq = X.lq - uqe, dt = X.lt - ute, ov = -(dq < dt ? dq : dt);
            const long long adj = dp_crossover_adj_wave(a, S, m, uqe, ute, X.lq, X.lt, ov);
            const long long s_u = dp_readlane64(tj, u) + X.ls - adj - dp_gap_lds(a, sg, dq + ov, dt + ov);
            (void)uqs;
            if (lane == u) sc = s_u;
        }
        const long long bs = dp_wave_max64(sc, lane);
        if (bs > 0) {
            const int bn = dp_wave_min32(sc == bs ? nd : 0x7fffffff, lane);
            if (bs > best || (bs == best && bn < best_node)) {
                best = bs;
                best_node = bn;
            }
        }
    }
}

// k_dp_spec's in-order turns: wait until *c == i (LDS, polled with a nap);
// false after seconds without progress (err |= 32: the kernel then ends)
__device__ __forceinline__ bool dp_spec_wait(const int *c, int i, int32_t *err) {
    for (unsigned spin = 0; ; ++spin) {
        const int v = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (v == i) return true;
        __builtin_amdgcn_s_sleep(2);
        if (spin > (1u << 26)) {
            if (err && (threadIdx.x & (kWave - 1)) == 0) atomicOr(err, 32);
            return false;
        }
    }
}
// the same, then an acquire of what the publisher released before *c = i
__device__ __forceinline__ bool dp_spec_acquire(const int *c, int i, int32_t *err) {
    if (!dp_spec_wait(c, i, err)) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    return true;
}

template <int W>
__global__ void __launch_bounds__(kWave * W) k_dp_spec(DpArgs a) {
    __shared__ int s_m[16];
    __shared__ DpGapLds s_gap;
    __shared__ int4 r_box[kWave];  // the last 64 committed leaves: {qs, qe, ts, te}
    __shared__ long long r_tot[kWave];
    __shared__ int r_node[kWave];
    __shared__ int r_leaf[kWave];
    __shared__ int s_commit;  // leaves committed (their ring slots written)
    __shared__ int s_vis;     // leaves whose tree updates are visible (<= s_commit)
    const int tid = threadIdx.x, lane = tid & (kWave - 1);
    const int nt = kWave * W;
    if (tid < 16) s_m[tid] = a.m16[tid];
    for (int k = tid; k < 3 * kGapLds; k += nt) {
        const int which = k / kGapLds, d = k % kGapLds;
        s_gap.gap[k] = which == 0 ? dp_gap_cost(a, d, 0)
                                  : (which == 1 ? dp_gap_cost(a, 0, d)
                                                : (d >= 2 ? dp_gap_cost(a, 1, d - 1) : 0));
    }
    if (tid < kMaxLong) {
        s_gap.lpos[tid] = a.gap.long_pos[tid];
        for (int w = 0; w < 3; ++w) s_gap.lval[w][tid] = a.gap.long_val[w][tid];
    }
    for (int k = tid; k < 3 * kLbN; k += nt) {
        const int which = k / kLbN, i = k % kLbN;
        const int64_t x = dp_lb_point(i);
        const int d = x > 0x7fffffff ? 0x7fffffff : (int)x;
        s_gap.lb[which][i] = which == 0 ? dp_gap_cost(a, d, 0)
                                        : (which == 1 ? dp_gap_cost(a, 0, d) : dp_gap_cost(a, 1, d - 1));
    }
    if (tid < 3) {
        s_gap.last_pos[tid] = a.gap.last_pos[tid];
        s_gap.last_val[tid] = a.gap.last_val[tid];
        s_gap.last_slope[tid] = a.gap.last_slope[tid];
    }
    if (tid == 0) {
        s_gap.small_size = a.gap.small_size;
        s_gap.long_count = a.gap.long_count;
    }
    const int wave = tid / kWave;
    const bool prof = a.prof != nullptr;
    DpPf pf;
    for (int k = 0; k < kDpProf; ++k) pf.v[k] = 0;
    for (int64_t pi = blockIdx.x; pi < a.n_pairs; pi += gridDim.x) {
        const DpPair P = a.pairs[pi];
        const DpSeq S = {P.tbase, P.qbase};
        long long *ms = a.nd_ms + P.node_off;
        long long *nwp = a.nd_nw + P.node_off;
        long long *tot = a.nd_tot + P.node_off;
        const int2 *nb = a.nd_b + P.node_off;
        __syncthreads();  // (the previous pair's waves are done with the ring)
        if (tid < kWave) {
            r_node[tid] = -1;
            r_leaf[tid] = -1;
        }
        if (tid == 0) s_commit = s_vis = 0;
        __syncthreads();
        for (int i = wave; i < P.n_leaves; i += W) {
            const int64_t li = P.leaf_off + i;
            const int4 L = a.lf[li];  // {qs, qe, ts, te}
            const int node = a.lf_node[li];
            DpLeafCtx X;
            X.lq = L.x;
            X.lqe = L.y;
            X.lt = L.z;
            X.lte = L.w;
            X.ls = a.lf_score[li];
            const int64_t q0 = a.path_off[li], q1 = a.path_off[li + 1];
            const int64_t o0 = a.ov_off[li], o1 = a.ov_off[li + 1];
            const long long kl = a.lin_k * ((long long)X.lq + X.lt) - 1024 * X.ls;
            // the update path's first 64 nodes now, off the in-order section
            const int pu = q0 + lane < q1 ? a.path[q0 + lane] : -1;
            if (prof) ++pf.v[kPfLeaves];
            // ---- 1-2: snapshot, seed, fast walk
            unsigned long long ck = prof ? clock64() : 0;
            const int c0 = __hip_atomic_load(&s_vis, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            long long best = 0;
            int best_node = -1;
            {
                const int j = r_leaf[lane];
                long long sc = -1;
                int nd = 0x7fffffff;
                if (j >= 0 && j >= c0 - kWave + W && j < c0) {  // (-1: a slot not written yet)
                    const int4 bx = r_box[lane];
                    nd = r_node[lane];
                    if (bx.x < X.lq && bx.z < X.lt) {
                        const int dq = X.lq - bx.y, dt = X.lt - bx.w;
                        if (dq >= 0 && dt >= 0) sc = r_tot[lane] + X.ls - dp_gap_lds(a, s_gap, dq, dt);
                    }
                }
                const long long bs = dp_wave_max64(sc > 0 ? sc : -1, lane);
                if (bs > 0) {
                    best = bs;
                    best_node = dp_wave_min32(sc == bs ? nd : 0x7fffffff, lane);
                }
            }
            dp_walk<true>(a, S, s_m, s_gap, P, X, kl, best, best_node, pf, prof);
            if (prof) {  // (slots: search, wait, in-order section)
                const unsigned long long t_ = clock64();
                pf.v[kPfCycWalk] += t_ - ck;
                ck = t_;
            }
            // ---- 3: in order; the leaves committed since the snapshot
            // ---- 3: until its turn, the leaves committed since the
            // snapshot folded in as they commit (final totals, from the ring)
            {
                int done = c0;
                for (unsigned spin = 0;; ++spin) {
                    const int c = __hip_atomic_load(&s_commit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (c > done) {
                        if (prof) {
                            const unsigned long long t_ = clock64();
                            pf.v[kPfCycLoad] += t_ - ck;
                            ck = t_;
                        }
                        dp_spec_fold(a, S, s_m, s_gap, X, r_box, r_tot, r_node, done, c, best, best_node);
                        if (prof) {
                            const unsigned long long t_ = clock64();
                            pf.v[c == i ? kPfCycSeed : kPfCycLoad] += t_ - ck;
                            ck = t_;
                        }
                        done = c;
                    }
                    if (c == i) break;
                    __builtin_amdgcn_s_sleep(2);
                    if (spin > (1u << 26)) {  // (seconds without a commit: end, reported)
                        if (a.err && lane == 0) atomicOr(a.err, 32);
                        return;
                    }
                }
                if (prof && c0 < i) ++pf.v[kPfXoverWin];
            }
            if (prof) {
                const unsigned long long t_ = clock64();
                pf.v[kPfCycSeed] += t_ - ck;  // (spec: the leaves since the snapshot)
                ck = t_;
            }
            // ---- 4: anomalies on final totals (the earlier leaves' tree
            // updates visible first), the reference walk if one fires
            if (prof) pf.v[kPfOvChecks] += o1 - o0;
            if (o1 > o0 && !dp_spec_acquire(&s_vis, i, a.err)) return;
            if (dp_anomaly_check(a, S, s_m, s_gap, P, X, nb, tot, o0, o1, best)) {
                best = 0;
                best_node = -1;
                if (prof) ++pf.v[kPfFallbacks];
                dp_walk<false>(a, S, s_m, s_gap, P, X, 0, best, best_node, pf, prof);
            }
            if (prof) {
                const unsigned long long t_ = clock64();
                pf.v[kPfCycAnom] += t_ - ck;  // (spec: anomaly check + fallback)
                ck = t_;
            }
            // ---- 5: commit
            long long total = X.ls;
            int pred = -1;
            if (best > X.ls) {
                total = best;
                pred = best_node;
            }
#ifdef GAC_DP_SPEC_CHECK
            if (pred < -1 || pred >= P.n_nodes || node < 0 || node >= P.n_nodes) {
                if (a.err && lane == 0) atomicOr(a.err, pred < -1 || pred >= P.n_nodes ? 64 : 128);
                pred = -1;
                if (node < 0 || node >= P.n_nodes) return;
            }
            for (int64_t k = q0 + lane; k < q1; k += kWave)
                if (a.path[k] < 0 || a.path[k] >= P.n_nodes) {
                    if (a.err) atomicOr(a.err, 256);
                    return;
                }
#endif
            const long long nwv = 1024 * total + a.lin_k * ((long long)X.lqe + X.lte);
            // (GAC_DP_SPEC_LDST: a load and a store, as k_dp_fast; else an
            // atomic max with no return -- no round trip before the fence;
            // the other waves' walks may read either value: bounds only grow)
            for (int64_t k = q0 + lane; k < q1; k += kWave) {
                const int u = k < q0 + kWave ? pu : a.path[k];
#ifdef GAC_DP_SPEC_LDST
                if (ld_wg(ms + u) < total) st_wg(ms + u, total);
                if (ld_wg(nwp + u) < nwv) st_wg(nwp + u, nwv);
#else
                __hip_atomic_fetch_max(ms + u, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_fetch_max(nwp + u, nwv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
            }
            if (lane == 0) {
                a.lf_total[li] = total;
                a.lf_pred[li] = pred;
                st_wg(tot + node, total);
                const int slot = i & (kWave - 1);
                r_box[slot] = L;
                r_tot[slot] = total;
                r_node[slot] = node;
                r_leaf[slot] = i;
                // the next leaf's turn needs the ring only: an LDS-only
                // release (the tree updates are still in flight)
                __asm__ volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __hip_atomic_store(&s_commit, i + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (prof) {
                const unsigned long long t_ = clock64();
                pf.v[kPfCycCommit] += t_ - ck;
                ck = t_;
            }
            // then the tree updates land and are published in order
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (!dp_spec_wait(&s_vis, i, a.err)) return;
            if (lane == 0)
                __hip_atomic_store(&s_vis, i + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (prof) pf.v[kPfCycFb] += clock64() - ck;  // (spec: publishing the tree updates)
        }
    }
    if (prof && lane < kDpProf) {
        unsigned long long v = 0;
        for (int k = 0; k < kDpProf; ++k)
            if (k == lane) v = pf.v[k];
        atomicAdd(a.prof + lane, v);
    }
}

hipError_t launch_dp_spec(const DpArgs &a, int grid, int waves, hipStream_t s) {
    if (a.n_pairs == 0) return hipSuccess;
    switch (waves) {
    case 4: hipLaunchKernelGGL(k_dp_spec<4>, dim3((unsigned)grid), dim3(kWave * 4), 0, s, a); break;
    case 8: hipLaunchKernelGGL(k_dp_spec<8>, dim3((unsigned)grid), dim3(kWave * 8), 0, s, a); break;
    case 16: hipLaunchKernelGGL(k_dp_spec<16>, dim3((unsigned)grid), dim3(kWave * 16), 0, s, a); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
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
