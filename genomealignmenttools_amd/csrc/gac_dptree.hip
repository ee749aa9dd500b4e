// gac_dptree.hip -- the per-pair inputs of axtChain's kd-tree DP built on the
// device (gac_chain_dp_blocks), for every device pair at once:
//
//   leaves   chainBlocks' leaf list (kent/src/lib/chainBlock.c:400-420): the
//            blocks with tStart != tEnd, in target order -- slSort by tStart,
//            stable over the list the reference builds with slAddHead, i.e.
//            reverse input order -- and in query order (kdTreeMake's dlSort by
//            qStart of the target-ordered list, :166-205): two stable radix
//            sorts on (pair, coordinate) keys.
//   kd-tree  kdBuild (:124-164) level-synchronously: at depth d every node of
//            every pair splits at once.  The cut dimension's list is already
//            in order (its first half is the lo child); the other list is
//            partitioned hits-first, stably (splitList :92-110), by ONE global
//            exclusive scan of the hit flags -- a node's hits before position
//            i are excl[i] - excl[segment start].  Node ids follow the host's
//            layout (pre-order, hi child first: a subtree of n leaves is 2n-1
//            consecutive nodes, so every node's id is known from its segment).
//            maxQ/maxT bottom-up, one launch per depth.
//   paths    the nodes updateScoresOnWay (:265-279) descends to for each leaf.
//   overlaps the leaves that overlap each leaf as a candidate (k_dp_fast's
//            anomaly check; dp_overlaps in host/gac_axtchain.c).
// Everything is integer index work, HBM/latency bound: one lane per leaf or
// node, coalesced where the access allows; nothing here is shaped for MFMA.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <stdint.h>

#include "gac_dp.h"

namespace gac {

namespace {

constexpr int kDtThreads = 256;
constexpr int kDtStack = 64;  // > the tree depth (<= 31) + 2: a DFS holds one sibling per level

inline dim3 dt_grid(int64_t n) { return dim3((unsigned)((n + kDtThreads - 1) / kDtThreads)); }

__device__ __forceinline__ int64_t dt_id() {
    return (int64_t)blockIdx.x * kDtThreads + threadIdx.x;
}

// the pair of packed block r: the last p with blk_off[p] <= r
__device__ __forceinline__ int64_t dt_pair_of(const int64_t *blk_off, int64_t P, int64_t r) {
    int64_t lo = 0, hi = P;
    while (hi - lo > 1) {
        const int64_t m = (lo + hi) >> 1;
        if (blk_off[m] <= r)
            lo = m;
        else
            hi = m;
    }
    return lo;
}

__global__ void __launch_bounds__(kDtThreads)
    k_dt_keys(int64_t P, int64_t B, const int64_t *blk_off, const int2 *sizes, const int4 *box,
              unsigned long long *keys, int32_t *vals, int32_t *err) {
    const int64_t r = dt_id();
    if (r >= B) return;
    const int64_t p = dt_pair_of(blk_off, P, r);
    // item r of the pair is its block n-1-r (the reference's list is built
    // by slAddHead), so a stable sort keeps the reference's tie order
    const int64_t g = blk_off[p] + (blk_off[p + 1] - 1 - r);
    const int4 b = box[g];  // {qs, qe, ts, te}
    const int2 sz = sizes[p];  // {tSize, qSize}
    const bool bad = b.x < 0 || b.x > b.y || b.y > sz.y || b.z < 0 || b.z > b.w || b.w > sz.x;
    if (bad) atomicOr(err, 1);
    keys[r] = (!bad && b.z != b.w) ? ((unsigned long long)p << 31) | (unsigned)b.z
                                   : ((unsigned long long)P << 31);
    vals[r] = (int32_t)g;
}

// leaf_off[p] = the first sorted key of pair p (p = P: the leaf count)
__global__ void __launch_bounds__(kDtThreads)
    k_dt_leaf_off(int64_t P, int64_t B, const unsigned long long *keys, int64_t *leaf_off) {
    const int64_t p = dt_id();
    if (p > P) return;
    const unsigned long long k = (unsigned long long)p << 31;
    int64_t lo = 0, hi = B;
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (keys[m] < k)
            lo = m + 1;
        else
            hi = m;
    }
    leaf_off[p] = lo;
}

// per leaf in target order: its pair, records, the query sort's key and the
// root segment of its pair
__global__ void __launch_bounds__(kDtThreads)
    k_dt_tinit(int64_t L, const unsigned long long *keys, const int32_t *tord, const int64_t *leaf_off,
               const int4 *box, const int32_t *score, int32_t *pidx, int32_t *tpos, int4 *lf,
               int32_t *lsc, unsigned long long *key2, int32_t *val2, int32_t *tl, int32_t *sstart,
               int32_t *slen, int32_t *snode) {
    const int64_t i = dt_id();
    if (i >= L) return;
    const int32_t g = tord[i];
    const int32_t p = (int32_t)(keys[i] >> 31);
    const int4 b = box[g];
    pidx[i] = p;
    tpos[g] = (int32_t)i;
    lf[i] = b;
    lsc[i] = score[g];
    key2[i] = ((unsigned long long)p << 31) | (unsigned)b.x;
    val2[i] = g;
    tl[i] = g;
    const int64_t s0 = leaf_off[p];
    sstart[i] = (int32_t)s0;
    slen[i] = (int32_t)(leaf_off[p + 1] - s0);
    snode[i] = 0;
}

__global__ void __launch_bounds__(kDtThreads)
    k_dt_qinit(int64_t L, const int32_t *qord, const int4 *box, const int32_t *tpos, int32_t *ql,
               int32_t *qpos, int4 *qbox, int32_t *qtp) {
    const int64_t k = dt_id();
    if (k >= L) return;
    const int32_t g = qord[k];
    ql[k] = g;
    qpos[g] = (int32_t)k;
    qbox[k] = box[g];
    qtp[k] = tpos[g];
}

// ---- one level of kdBuild: D = the cut dimension's list, O = the other
__global__ void __launch_bounds__(kDtThreads)
    k_dt_posd(int64_t L, int64_t B, const int32_t *D, const int32_t *slen, int32_t *posd) {
    const int64_t i = dt_id();
    if (i >= L || slen[i] < 2) return;
    const int32_t g = D[i];
    if ((uint32_t)g < (uint64_t)B) posd[g] = (int32_t)i;  // (always: a failed split is reported)
}

__global__ void __launch_bounds__(kDtThreads)
    k_dt_flag(int64_t L, int64_t B, const int32_t *O, const int32_t *sstart, const int32_t *slen,
              const int32_t *posd, int32_t *flag) {
    const int64_t i = dt_id();
    if (i >= L) return;
    const int32_t len = slen[i], g = O[i];
    flag[i] = len >= 2 && (uint32_t)g < (uint64_t)B && posd[g] < sstart[i] + (len >> 1);
}

__global__ void __launch_bounds__(kDtThreads)
    k_dt_split(int64_t L, int depth, int dim, const int32_t *D, const int32_t *O, int32_t *O2,
               const int32_t *flag, const int32_t *excl, int32_t *sstart, int32_t *slen,
               int32_t *snode, const int32_t *pidx, const int64_t *node_off, const int4 *box,
               int4 *na, int2 *nb, int32_t *ndep, int32_t *ndl, int32_t *err) {
    const int64_t i = dt_id();
    if (i >= L) return;
    const int32_t s = sstart[i], len = slen[i], e = O[i];
    if (len < 2) {
        O2[i] = e;
        return;
    }
    const int32_t half = len >> 1, hb = excl[i] - excl[s];
    const int32_t np = flag[i] ? s + hb : s + half + ((int32_t)i - s - hb);
    if (np < s || np >= s + len || (flag[i] ? np >= s + half : np < s + half)) {
        atomicOr(err, 8);  // (the hits of a node are exactly its lo half)
        return;
    }
    O2[np] = e;
    const int32_t v = snode[i], lo = v + 2 * (len - half);
    if (i == s) {  // the node itself (medianVal: the last of the lo half)
        const int4 bb = box[D[s + half - 1]];
        const int64_t nv = node_off[pidx[i]] + v;
        na[nv] = make_int4(0, 0, dim ? bb.z : bb.x, lo);
        nb[nv] = make_int2(v + 2 * len - 1, dim);
        ndep[nv] = depth;
        ndl[nv] = lo - v;
    }
    if ((int32_t)i - s < half) {
        slen[i] = half;
        snode[i] = lo;
    } else {
        sstart[i] = s + half;
        slen[i] = len - half;
        snode[i] = v + 1;
    }
}

// every position is a one-leaf segment now: the leaf nodes
__global__ void __launch_bounds__(kDtThreads)
    k_dt_leafnodes(int64_t L, int64_t B, const int32_t *ql, const int32_t *tl, const int32_t *slen,
                   const int32_t *snode, const int32_t *pidx, const int64_t *node_off,
                   const int64_t *leaf_off, const int4 *box, const int32_t *score,
                   const int32_t *tpos, int4 *na, int2 *nb, int32_t *ndep, int32_t *lnode,
                   long long *tot, int32_t *err) {
    const int64_t i = dt_id();
    if (i >= L) return;
    const int32_t g = ql[i];
    if (slen[i] != 1 || tl[i] != g || (uint32_t)g >= (uint64_t)B) {
        atomicOr(err, 2);
        return;
    }
    const int32_t v = snode[i], p = pidx[i];
    const int64_t nv = node_off[p] + v;
    const int4 b = box[g];
    const int32_t tp = tpos[g];
    na[nv] = make_int4(b.y, b.w, b.x, b.z);  // {qEnd, tEnd, qStart, tStart}
    nb[nv] = make_int2(v + 1, ~(int32_t)(tp - leaf_off[p]));
    ndep[nv] = -1;
    lnode[tp] = v;
    tot[nv] = score[g];
}

// maxQ / maxT of the internal nodes at one depth from their children
__global__ void __launch_bounds__(kDtThreads)
    k_dt_max(int64_t N, int depth, const int32_t *ndep, const int32_t *ndl, int4 *na) {
    const int64_t v = dt_id();
    if (v >= N || ndep[v] != depth) return;
    const int4 a = na[v + ndl[v]], b = na[v + 1];
    int4 m = na[v];
    m.x = a.x > b.x ? a.x : b.x;
    m.y = a.y > b.y ? a.y : b.y;
    na[v] = m;
}

__global__ void __launch_bounds__(kDtThreads)
    k_dt_fill64(int64_t n, long long *a, long long v) {
    const int64_t i = dt_id();
    if (i < n) a[i] = v;
}

// the pair's longest block (dp_leaf_positions' maxsz)
__global__ void __launch_bounds__(kDtThreads)
    k_dt_maxsz(int64_t L, const int4 *lf, const int32_t *pidx, int32_t *msz) {
    const int64_t i = dt_id();
    const bool in = i < L;
    const int32_t p = in ? pidx[i] : -1;
    const int32_t v = in ? lf[i].w - lf[i].z : 0;
    const int32_t p0 = __shfl(p, 0);
    const bool same = __all(!in || p == p0);
    if (same) {
        int32_t m = v;
        for (int o = 32; o > 0; o >>= 1) {
            const int32_t x = __shfl_xor(m, o);
            m = x > m ? x : m;
        }
        if ((threadIdx.x & 63) == 0 && p0 >= 0) atomicMax(msz + p0, m);
    } else if (in) {
        atomicMax(msz + p, v);
    }
}

// updateScoresOnWay's descent for leaf i (target order): count, or write
__global__ void __launch_bounds__(kDtThreads)
    k_dt_path(int64_t L, int fill, const int4 *lf, const int32_t *pidx, const int64_t *node_off,
              const int4 *na, const int2 *nb, long long *cnt, const long long *off, int32_t *path,
              int32_t *err) {
    const int64_t i = dt_id();
    if (i >= L) return;
    const int64_t base = node_off[pidx[i]];
    const int4 l = lf[i];
    int32_t st[kDtStack];
    int sp = 0;
    st[sp++] = 0;
    long long n = 0;
    const long long o = fill ? off[i] : 0;
    while (sp > 0) {
        const int32_t v = st[--sp];
        if (fill) path[o + n] = v;
        ++n;
        const int2 b = nb[base + v];
        if (b.y >= 0) {
            if (sp + 2 > kDtStack) {
                atomicOr(err, 4);
                break;
            }
            const int4 a = na[base + v];
            const int32_t coord = b.y == 0 ? l.x : l.z;
            if (coord <= a.z) st[sp++] = a.w;    // lo
            if (coord >= a.z) st[sp++] = v + 1;  // hi (visited first)
        }
    }
    if (!fill) cnt[i] = n;
}

// the overlapping candidates of leaf i (dp_overlaps): count (over the cap:
// one -1 entry), or write their leaf nodes
__global__ void __launch_bounds__(kDtThreads)
    k_dt_ovl(int64_t L, int fill, int32_t cap, const int4 *lf, const int4 *qbox,
             const int32_t *qtp, const int32_t *qpos, const int32_t *tord, const int32_t *pidx,
             const int64_t *leaf_off, const int32_t *msz, const int32_t *lnode, long long *cnt,
             uint8_t *over, const long long *off, int32_t *ov) {
    const int64_t i = dt_id();
    if (i >= L) return;
    const int32_t p = pidx[i];
    const int64_t lo_i = leaf_off[p];
    const int4 me = lf[i];
    const int32_t lq = me.x, lt = me.z, m = msz[p];
    const long long o = fill ? off[i] : 0;
    if (fill && over[i]) {
        ov[o] = -1;
        return;
    }
    int32_t n = 0;
    bool ovf = false;
    // target side: the leaves before it in target order starting within m
    for (int64_t j = i - 1; j >= lo_i; --j) {
        const int4 b = lf[j];
        if (!(b.z > lt - m)) break;
        if (b.z >= lt || b.x >= lq) continue;
        const int32_t dq = lq - b.y, dt = lt - b.w;
        if (dq >= 0 && dt >= 0) continue;
        if (n == cap) {
            ovf = true;
            break;
        }
        if (fill) ov[o + n] = lnode[j];
        ++n;
    }
    // query side (the ones not overlapping in target: the t scan saw those)
    if (!ovf) {
        const int64_t at = qpos[tord[i]];
        for (int64_t j = at - 1; j >= lo_i; --j) {
            const int4 b = qbox[j];  // {qs, qe, ts, te}
            if (!(b.x > lq - m)) break;
            const int32_t tp = qtp[j];
            if (b.z >= lt || b.x >= lq || tp >= i) continue;
            const int32_t dq = lq - b.y, dt = lt - b.w;
            if (dq >= 0 && dt >= 0) continue;
            if (dt < 0) continue;
            if (n == cap) {
                ovf = true;
                break;
            }
            if (fill) ov[o + n] = lnode[tp];
            ++n;
        }
    }
    if (!fill) {
        cnt[i] = ovf ? 1 : n;
        over[i] = ovf ? 1 : 0;
    }
}

__global__ void __launch_bounds__(kDtThreads)
    k_dt_out_init(int64_t B, const int32_t *score, long long *total, int32_t *pred) {
    const int64_t g = dt_id();
    if (g >= B) return;
    total[g] = score[g];
    pred[g] = -1;
}

// per leaf: its block's totalScore and best predecessor as a block of the
// pair, and the target order as pair-local blocks
__global__ void __launch_bounds__(kDtThreads)
    k_dt_out(int64_t L, const int32_t *tord, const int32_t *pidx, const int64_t *blk_off,
             const int64_t *leaf_off, const int64_t *node_off, const int2 *nb,
             const long long *lf_total, const int32_t *lf_pred, int32_t *out_tord,
             long long *total, int32_t *pred, int32_t *err) {
    const int64_t i = dt_id();
    if (i >= L) return;
    const int32_t g = tord[i], p = pidx[i];
    const int64_t b0 = blk_off[p];
    out_tord[i] = (int32_t)(g - b0);
    total[g] = lf_total[i];
    const int32_t pr = lf_pred[i];
    if (pr < 0) {
        pred[g] = -1;
        return;
    }
    const int32_t pl = nb[node_off[p] + pr].y;  // ~(leaf position)
    if (pl >= 0) {
        atomicOr(err, 16);  // (a predecessor is always a leaf)
        pred[g] = -1;
        return;
    }
    pred[g] = (int32_t)(tord[leaf_off[p] + ~pl] - b0);
}

// the tree in the host's node layout (host/gac_axtchain.c ax_node: lo, hi,
// leaf, cut, maxQ, maxT; a leaf node: qStart, tStart, its block, 0, qEnd,
// tEnd), node ids and blocks local to the pair
__global__ void __launch_bounds__(kDtThreads)
    k_dt_host_nodes(int64_t P, int64_t N, const int64_t *node_off, const int64_t *leaf_off,
                    const int64_t *blk_off, const int32_t *tord, const int4 *na, const int2 *nb,
                    const int32_t *ndep, int32_t *out) {
    const int64_t v = dt_id();
    if (v >= N) return;
    const int64_t p = dt_pair_of(node_off, P, v);
    const int32_t vl = (int32_t)(v - node_off[p]);
    const int4 a = na[v];
    const int2 b = nb[v];
    int32_t *o = out + 6 * v;
    if (ndep[v] >= 0) {
        o[0] = a.w;
        o[1] = vl + 1;
        o[2] = -1;
        o[3] = a.z;
    } else {
        o[0] = a.z;
        o[1] = a.w;
        o[2] = (int32_t)(tord[leaf_off[p] + ~b.y] - blk_off[p]);
        o[3] = 0;
    }
    o[4] = a.x;
    o[5] = a.y;
}

// per leaf position: the target and query orders as pair-local blocks; per
// block: its leaf node (-1: not a leaf)
__global__ void __launch_bounds__(kDtThreads)
    k_dt_host_lists(int64_t L, const int32_t *pidx, const int64_t *blk_off, const int32_t *tord,
                    const int32_t *qord, const int32_t *lnode, int32_t *out_t, int32_t *out_q,
                    int32_t *out_lnode) {
    const int64_t i = dt_id();
    if (i >= L) return;
    const int64_t b0 = blk_off[pidx[i]];
    const int32_t g = tord[i];
    out_t[i] = (int32_t)(g - b0);
    out_q[i] = (int32_t)(qord[i] - b0);
    out_lnode[g] = lnode[i];
}

}  // namespace

// ------------------------------------------------------------------ launchers
hipError_t dt_sort_pairs(void *tmp, size_t &tmp_bytes, const unsigned long long *kin,
                         unsigned long long *kout, const int32_t *vin, int32_t *vout, int64_t n,
                         int end_bit, hipStream_t s) {
    return hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, kin, kout, vin, vout, (int)n, 0,
                                              end_bit, s);
}

hipError_t dt_scan32(void *tmp, size_t &tmp_bytes, const int32_t *in, int32_t *out, int64_t n,
                     hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, (int)n, s);
}

hipError_t dt_scan64(void *tmp, size_t &tmp_bytes, const long long *in, long long *out, int64_t n,
                     hipStream_t s) {
    return hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, in, out, (int)n, s);
}

hipError_t launch_dt_keys(int64_t P, int64_t B, const int64_t *blk_off, const int2 *sizes,
                          const int4 *box, unsigned long long *keys, int32_t *vals, int32_t *err,
                          hipStream_t s) {
    if (B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_dt_keys, dt_grid(B), dim3(kDtThreads), 0, s, P, B, blk_off, sizes, box,
                       keys, vals, err);
    return hipGetLastError();
}

hipError_t launch_dt_leaf_off(int64_t P, int64_t B, const unsigned long long *keys,
                              int64_t *leaf_off, hipStream_t s) {
    hipLaunchKernelGGL(k_dt_leaf_off, dt_grid(P + 1), dim3(kDtThreads), 0, s, P, B, keys, leaf_off);
    return hipGetLastError();
}

hipError_t launch_dt_build(const DtTree &t, int levels, hipStream_t s) {
    const int64_t L = t.L, N = t.N;
    if (L == 0) return hipSuccess;
    const dim3 gl = dt_grid(L), bl(kDtThreads);
    hipLaunchKernelGGL(k_dt_tinit, gl, bl, 0, s, L, t.keys, t.tord, t.leaf_off, t.box, t.score,
                       t.pidx, t.tpos, t.lf, t.lsc, t.key2, t.val2, t.tl, t.sstart, t.slen,
                       t.snode);
    size_t b = t.tmp_bytes;
    hipError_t e = dt_sort_pairs(t.tmp, b, t.key2, t.key2 + L, t.val2, t.val2 + L, L, t.end_bit, s);
    if (e != hipSuccess) return e;
    const int32_t *qord = t.val2 + L;
    hipLaunchKernelGGL(k_dt_qinit, gl, bl, 0, s, L, qord, t.box, t.tpos, t.ql, t.qpos, t.qbox,
                       t.qtp);
    // lists: ql (dim 0's), tl (dim 1's) and a spare; the other list of a
    // level is partitioned into the spare, which then takes its place
    int32_t *ql = t.ql, *tl = t.tl, *spare = t.spare;
    if ((e = hipMemsetAsync(t.ndep, 0xff, N * sizeof(int32_t), s)) != hipSuccess) return e;
    for (int d = 0; d < levels; ++d) {
        const int dim = d & 1;
        int32_t *D = dim ? tl : ql, *O = dim ? ql : tl;
        hipLaunchKernelGGL(k_dt_posd, gl, bl, 0, s, L, t.B, D, t.slen, t.posd);
        hipLaunchKernelGGL(k_dt_flag, gl, bl, 0, s, L, t.B, O, t.sstart, t.slen, t.posd, t.flag);
        b = t.tmp_bytes;
        if ((e = dt_scan32(t.tmp, b, t.flag, t.excl, L, s)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_dt_split, gl, bl, 0, s, L, d, dim, D, O, spare, t.flag, t.excl,
                           t.sstart, t.slen, t.snode, t.pidx, t.node_off, t.box, t.na, t.nb,
                           t.ndep, t.ndl, t.err);
        if (dim)
            ql = spare;
        else
            tl = spare;
        spare = O;
    }
    hipLaunchKernelGGL(k_dt_fill64, dt_grid(N), bl, 0, s, N, t.tot, 0LL);
    hipLaunchKernelGGL(k_dt_fill64, dt_grid(N), bl, 0, s, N, t.ms, 0LL);
    hipLaunchKernelGGL(k_dt_fill64, dt_grid(N), bl, 0, s, N, t.nw, (long long)(INT64_MIN / 4));
    hipLaunchKernelGGL(k_dt_leafnodes, gl, bl, 0, s, L, t.B, ql, tl, t.slen, t.snode, t.pidx,
                       t.node_off, t.leaf_off, t.box, t.score, t.tpos, t.na, t.nb, t.ndep, t.lnode,
                       t.tot, t.err);
    for (int d = levels - 1; d >= 0; --d)
        hipLaunchKernelGGL(k_dt_max, dt_grid(N), bl, 0, s, N, d, t.ndep, t.ndl, t.na);
    return hipGetLastError();
}

hipError_t launch_dt_tree(const DtTree &t, int levels, hipStream_t s) {
    hipError_t e = launch_dt_build(t, levels, s);
    const int64_t L = t.L;
    if (e != hipSuccess || L == 0) return e;
    const dim3 gl = dt_grid(L), bl(kDtThreads);
    size_t b;
    hipLaunchKernelGGL(k_dt_path, gl, bl, 0, s, L, 0, t.lf, t.pidx, t.node_off, t.na, t.nb,
                       t.pcnt, nullptr, nullptr, t.err);
    b = t.tmp_bytes;
    if ((e = dt_scan64(t.tmp, b, t.pcnt, t.poff, L + 1, s)) != hipSuccess) return e;
    if (t.fast) {
        hipMemsetAsync(t.msz, 0, t.P * sizeof(int32_t), s);
        hipLaunchKernelGGL(k_dt_maxsz, gl, bl, 0, s, L, t.lf, t.pidx, t.msz);
        hipLaunchKernelGGL(k_dt_ovl, gl, bl, 0, s, L, 0, t.ov_cap, t.lf, t.qbox, t.qtp, t.qpos,
                           t.tord, t.pidx, t.leaf_off, t.msz, t.lnode, t.ocnt, t.over, nullptr,
                           nullptr);
        b = t.tmp_bytes;
        if ((e = dt_scan64(t.tmp, b, t.ocnt, t.ooff, L + 1, s)) != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_dt_lists(const DtTree &t, int32_t *path, int32_t *ov, hipStream_t s) {
    const int64_t L = t.L;
    if (L == 0) return hipSuccess;
    const dim3 gl = dt_grid(L), bl(kDtThreads);
    hipLaunchKernelGGL(k_dt_path, gl, bl, 0, s, L, 1, t.lf, t.pidx, t.node_off, t.na, t.nb,
                       nullptr, t.poff, path, t.err);
    if (t.fast)
        hipLaunchKernelGGL(k_dt_ovl, gl, bl, 0, s, L, 1, t.ov_cap, t.lf, t.qbox, t.qtp, t.qpos,
                           t.tord, t.pidx, t.leaf_off, t.msz, t.lnode, nullptr, t.over, t.ooff,
                           ov);
    return hipGetLastError();
}

hipError_t launch_dt_out(const DtTree &t, const long long *lf_total, const int32_t *lf_pred,
                         int32_t *out_tord, long long *total, int32_t *pred, hipStream_t s) {
    if (t.B == 0) return hipSuccess;
    hipLaunchKernelGGL(k_dt_out_init, dt_grid(t.B), dim3(kDtThreads), 0, s, t.B, t.score, total,
                       pred);
    if (t.L)
        hipLaunchKernelGGL(k_dt_out, dt_grid(t.L), dim3(kDtThreads), 0, s, t.L, t.tord, t.pidx,
                           t.blk_off, t.leaf_off, t.node_off, t.nb, lf_total, lf_pred, out_tord,
                           total, pred, t.err);
    return hipGetLastError();
}

hipError_t launch_dt_host(const DtTree &t, int32_t *nodes, int32_t *out_t, int32_t *out_q,
                          int32_t *out_lnode, hipStream_t s) {
    if (t.B) hipMemsetAsync(out_lnode, 0xff, t.B * sizeof(int32_t), s);
    if (t.N)
        hipLaunchKernelGGL(k_dt_host_nodes, dt_grid(t.N), dim3(kDtThreads), 0, s, t.P, t.N,
                           t.node_off, t.leaf_off, t.blk_off, t.tord, t.na, t.nb, t.ndep, nodes);
    if (t.L)
        hipLaunchKernelGGL(k_dt_host_lists, dt_grid(t.L), dim3(kDtThreads), 0, s, t.L, t.pidx,
                           t.blk_off, t.tord, t.val2 + t.L, t.lnode, out_t, out_q, out_lnode);
    return hipGetLastError();
}

}  // namespace gac
