// gac_kernels.hip -- CDNA4 (gfx950) kernels of libgachain.
//
// The reference hot path (single-threaded C) is, per sub-chain:
//   chainSubsetOnT   kent/src/lib/chain.c:471-558      clip blocks to [s, e)
//   chainCalcScore   kent/src/lib/chainConnect.c:24-40  sum(block) - sum(gap)
//   chainScoreBlock  kent/src/lib/chainConnect.c:14-22  sum matrix[q][t] per base
//   gapCalcCost      kent/src/lib/gapCalc.c:298-331      piecewise-linear gap cost
//   chainCalcScoreLocal src/scoreChain/scoreChain.c:176-198  max-plus local score
// Here one batch of sub-chains ("ranges") is scored by:
//   k_plan    one lane per range: binary-search the block window (replaces
//             the O(blocks) list walks of chainSubsetOnT / chainBaseCountSubT),
//             write a 32-byte range descriptor; workgroup scan of window
//             blocks
//   k_tilemap_fused  one lane per range: each workgroup sums the plan
//             workgroup totals itself (its flat offset, W), then the range's
//             flat offset and the first range of each tile; for > 1 M
//             ranges the same in two launches, k_scan_agg (one-workgroup
//             scan) + k_tilemap
//   k_small   batches of <= 256 ranges: one wave per range, one launch
//   k_tile    one wave per tile of 64 consecutive flat blocks (ranges packed
//             densely, many ranges per tile): lanes score 32-base chunks of
//             2-bit packed T and Q straight from HBM (bit-plane popcounts, the
//             4x4 matrix in SGPRs), LDS atomics fold chunks into blocks, lanes
//             evaluate gapCalcCost in exact f64, and segmented (by range)
//             wave scans fold sums and the max-plus local-score element;
//             ranges complete inside the tile are written directly
//   k_fold_tiles + k_fold_super  ranges spanning > 1 tile: ordered fold of
//             tile segments, parallel over tiles (a segmented wave scan per
//             64 tiles, then one lane per range spanning super-tiles)
// All sums are int64: every addend of the reference's double accumulation is
// an integer, so integer arithmetic is exact and bit-identical.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>
#include <algorithm>
#include <stdint.h>
#include <stdlib.h>

#include "gac_kernels.h"

#pragma clang fp contract(off)

namespace gac {

// ------------------------------------------------------------ gap cost ---
// gapCalcCost (kent/src/lib/gapCalc.c:298-331) with interpolate (:82-104),
// same double operation order, no FMA contraction, truncation to int.
__device__ __forceinline__ int interp_long(int x, const GapDev &g, int which) {
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

// Cost of a gap of kind `which` (0 = query-only, 1 = target-only, 2 = both)
// and length d, the three branches of gapCalcCost.
__device__ __forceinline__ int gap_cost_wd(const GapDev &g, const int32_t *small, int which,
                                           int d) {
    if (d < g.small_size) return small[which * g.small_size + d];
    if (d >= g.last_pos[which])
        return (int)__dadd_rn(g.last_val[which],
                              __dmul_rn(g.last_slope[which], (double)(d - g.last_pos[which])));
    return interp_long(d, g, which);
}

// gapCalcCost's kind/length from (dq, dt)
__device__ __forceinline__ int gap_kind(int dq, int dt, int &d) {
    if (dt < 0) dt = 0;
    if (dq < 0) dq = 0;
    if (dt == 0) {
        d = dq;
        return 0;
    }
    if (dq == 0) {
        d = dt;
        return 1;
    }
    d = dq + dt;
    return 2;
}

// Gap-cost table [3][len] built once per scoring setup from gap_cost_wd (the
// scoring kernel then needs one load per gap; lengths >= len, i.e. beyond the
// last table position, take the slope branch or, past a capped table, the
// interpolation).
__global__ void __launch_bounds__(256) k_gap_table(GapDev g, const int32_t *small, int len,
                                                   int32_t *tab) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 3 * (int64_t)len) return;
    const int which = (int)(i / len), d = (int)(i % len);
    tab[i] = gap_cost_wd(g, small, which, d);
}

// ------------------------------------------------------------ helpers ----
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// The same for LDS handed between the lanes of ONE wave (a wave's LDS
// operations execute in order): wavefront-scope fences order the compiler's
// accesses without the vmcnt(0) a workgroup-scope release implies, so loads
// in flight (the LDS-DMA of k_tile_pipe) stay in flight.
__device__ __forceinline__ void wave_sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t funnel(uint32_t hi, uint32_t lo, int sh) {
    return __builtin_amdgcn_alignbit(hi, lo, (uint32_t)sh);
}

typedef uint32_t u32x4a8 __attribute__((ext_vector_type(4), aligned(8)));
typedef uint32_t u32x2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef int32_t i32x4a8 __attribute__((ext_vector_type(4), aligned(8)));

// 32 bases starting at global base index p: the two code planes (bit i = base
// p+i) with ONE 16-byte load of words w, w+1 ({p0,p1} each; 8-byte aligned).
__device__ __forceinline__ void load_planes(const uint2 *planes, int64_t p, uint32_t &b0,
                                            uint32_t &b1) {
    const int64_t w = p >> 5;
    const int sh = (int)(p & 31);
    const u32x4a8 v = *reinterpret_cast<const u32x4a8 *>(planes + w);
    b0 = funnel(v.z, v.x, sh);
    b1 = funnel(v.w, v.y, sh);
}

__device__ __forceinline__ uint32_t load_nmask(const uint32_t *nmask, int64_t p) {
    const int64_t w = p >> 5;
    const u32x2a4 v = *reinterpret_cast<const u32x2a4 *>(nmask + w);
    return funnel(v.y, v.x, (int)(p & 31));
}

struct Elem {
    long long A, B, C, D;
};

__device__ __forceinline__ long long max2(long long a, long long b) { return a > b ? a : b; }

// x then y
__device__ __forceinline__ Elem compose(const Elem &x, const Elem &y) {
    Elem r;
    r.A = x.A + y.A;
    r.B = max2(x.B + y.A, y.B);
    r.C = max2(x.C, x.A + y.C);
    r.D = max2(max2(x.D, x.B + y.C), y.D);
    return r;
}

__device__ __forceinline__ long long shfl_down64(long long v, int d) {
    return __shfl_down(v, d, kWave);
}

// ordered (non-commutative) wave reduction; lane 0 ends with e_0 . e_1 ... e_63
__device__ __forceinline__ Elem wave_fold(Elem e, int lane) {
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        Elem o;
        o.A = shfl_down64(e.A, d);
        o.B = shfl_down64(e.B, d);
        o.C = shfl_down64(e.C, d);
        o.D = shfl_down64(e.D, d);
        if ((lane & (2 * d - 1)) == 0 && lane + d < kWave) e = compose(e, o);
    }
    return e;
}

__device__ __forceinline__ long long wave_sum(long long v) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, kWave);
    return v;
}

// ---- wave scans on DPP (row_shr 1/2/4/8 inside each 16-lane row, then
// row_bcast15 / row_bcast31 across rows: VALU moves, no LDS).  Step k of
// kScanSteps moves lane src(lane) = the step's source to `lane`; the caller
// combines when src_ok(k, lane) and the source lies in its segment.
// (mov_dpp: lanes whose source is out of the row / rows outside RM get 0 or
// keep garbage -- callers only use lanes where scan_src_ok)
template <int CTRL, int RM>
__device__ __forceinline__ int dpp32(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, RM, 0xf, true);
}
template <int CTRL, int RM>
__device__ __forceinline__ long long dpp64(long long v) {
    const unsigned long long u = (unsigned long long)v;
    const int lo = dpp32<CTRL, RM>((int)(uint32_t)u);
    const int hi = dpp32<CTRL, RM>((int)(uint32_t)(u >> 32));
    return (long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo);
}
// source lane of step K for `lane` (meaningful only where scan_src_ok)
template <int K>
__device__ __forceinline__ int scan_src(int lane) {
    if (K < 4) return lane - (1 << K);
    if (K == 4) return (lane & ~15) - 1;
    return 31;
}
template <int K>
__device__ __forceinline__ bool scan_src_ok(int lane) {
    if (K < 4) return (lane & 15) >= (1 << K);
    if (K == 4) return (lane & 16) != 0;  // rows 1 and 3
    return lane >= 32;                    // rows 2 and 3
}
template <int K>
struct ScanCtl;  // dpp control and row mask of step K
template <> struct ScanCtl<0> { static constexpr int c = 0x111, rm = 0xf; };
template <> struct ScanCtl<1> { static constexpr int c = 0x112, rm = 0xf; };
template <> struct ScanCtl<2> { static constexpr int c = 0x114, rm = 0xf; };
template <> struct ScanCtl<3> { static constexpr int c = 0x118, rm = 0xf; };
template <> struct ScanCtl<4> { static constexpr int c = 0x142, rm = 0xa; };
template <> struct ScanCtl<5> { static constexpr int c = 0x143, rm = 0xc; };

template <int K>
__device__ __forceinline__ int scan_step_add(int v, int lane) {
    const int o = dpp32<ScanCtl<K>::c, ScanCtl<K>::rm>(v);
    return scan_src_ok<K>(lane) ? v + o : v;
}
// plain inclusive prefix sum over the wave (int)
__device__ __forceinline__ int wave_incl_sum(int v, int lane) {
    v = scan_step_add<0>(v, lane);
    v = scan_step_add<1>(v, lane);
    v = scan_step_add<2>(v, lane);
    v = scan_step_add<3>(v, lane);
    v = scan_step_add<4>(v, lane);
    v = scan_step_add<5>(v, lane);
    return v;
}

// ------------------------------------------------------------ N flags ----
// At chain upload: flag blocks whose target / query bases contain an N, so
// the scoring kernel can skip N-mask loads for all other blocks.  Genomes
// hold few N runs (assembly gaps), so a chain is first checked as a whole
// (k_chain_prep: its target and query spans against the sorted global N
// runs); only the blocks of chains whose span meets a run are checked,
// against the same runs (k_build_flat).
// does [lo, hi) meet one of the sorted, disjoint runs [a, b) {start, end}?
__device__ __forceinline__ bool span_meets(const longlong2 *runs, int64_t a, int64_t b, int64_t lo,
                                           int64_t hi) {
    const int64_t n = b;
    while (a < b) {  // first run ending past lo
        const int64_t m = (a + b) >> 1;
        if (runs[m].y > lo) b = m;
        else a = m + 1;
    }
    return a < n && runs[a].x < hi;
}

// the runs of the sorted, disjoint list that meet [lo, hi): [*a, *b), empty
// when none does
__device__ __forceinline__ void runs_in(const longlong2 *runs, int64_t n, int64_t lo, int64_t hi,
                                        int32_t *ra, int32_t *rb) {
    int64_t a = 0, b = n;  // first run ending past lo
    while (a < b) {
        const int64_t m = (a + b) >> 1;
        if (runs[m].y > lo) b = m;
        else a = m + 1;
    }
    int64_t e = a, f = n;  // first run starting at or after hi
    while (e < f) {
        const int64_t m = (e + f) >> 1;
        if (runs[m].x >= hi) f = m;
        else e = m + 1;
    }
    *ra = (int32_t)a;
    *rb = (int32_t)(e > a ? e : a);
}

// ------------------------------------------------------------ flat upload
// The chain-upload kernels one lane per BLOCK (a chain averages ~23 blocks:
// a wave per chain left most lanes idle).  A lane finds its block's chain
// from the chain of its 64-block tile (tile_c0, one binary search per tile)
// and a short binary search of the compact chain offsets coff; empty chains
// share their offset with the next chain, and "last chain starting at or
// before b" picks the non-empty one.
__device__ __forceinline__ int64_t owner_chain(const int32_t *coff, const int32_t *tile_c0,
                                               int64_t ntiles, int64_t b) {
    // (a wave's 64 lanes are one tile: its bounds are wave-uniform loads)
    const int64_t t = __builtin_amdgcn_readfirstlane((int)(b >> 6));
    int64_t lo = tile_c0[t], hi = tile_c0[t + 1 < ntiles ? t + 1 : ntiles];
    while (lo < hi) {  // last c in [lo, hi] with coff[c] <= b
        const int64_t mid = (lo + hi + 1) >> 1;
        if (coff[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// The chains of a workgroup's kUpPer x 256 blocks (4 kUpPer tiles), staged in LDS
// with one coalesced load each: chains tile_c0[t0] .. tile_c0[t0 + 4 kUpPer],
// their compact offsets (and the next chain's), so a lane finds its block's
// chain by a search in LDS instead of dependent global loads.  A workgroup
// over more than kStage chains (a run of empty chains) returns false: its
// lanes take owner_chain's global search.  Each lane takes kUpPer blocks, so
// the staging round trip is paid once per 4 kUpPer tiles.
#ifndef GAC_UP_PER
#define GAC_UP_PER 2  // (A/B probes: make variant VFLAGS=-DGAC_UP_PER=4)
#endif
#ifndef GAC_UP_PROBE
#define GAC_UP_PROBE 0  // (timing probes only: 1 no bucket entries, 2 no N flags, 4 no 12-B records / spans)
#endif
constexpr int kStage = 256, kUpPer = GAC_UP_PER;
struct ChainStage {
    int32_t c0, m;  // (every lane's own copy: workgroup-uniform values)
    int32_t *off;   // [m + 1] in LDS
};

__device__ __forceinline__ bool stage_offsets(const int32_t *coff, const int32_t *tile_c0,
                                              int64_t ntiles, int64_t B0, int32_t *lds_off,
                                              ChainStage &S) {
    const int64_t t0 = B0 >> 6, t1 = t0 + 4 * kUpPer < ntiles ? t0 + 4 * kUpPer : ntiles;
    S.c0 = tile_c0[t0];
    S.m = tile_c0[t1] - S.c0 + 1;
    S.off = lds_off;
    if (S.m > kStage) return false;
    for (int j = threadIdx.x; j <= S.m; j += blockDim.x) lds_off[j] = coff[S.c0 + j];  // (coff[c1 + 1] exists)
    return true;
}

// the staged chain holding block b: last j with off[j] <= b (an empty chain
// shares its offset with the next, which is then the one taken)
__device__ __forceinline__ int staged_chain(const ChainStage &S, int64_t b) {
    int lo = 0, hi = S.m - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (S.off[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// one lane per chain: compact offsets, the bucket terminator, and the N runs
// its target / query span meets (crun: {t first, t end, q first, q end})
__global__ void __launch_bounds__(256) k_chain_prep(const DChain *chains, int64_t n_chains,
                                                    int64_t nb, const int32_t *bq,
                                                    const int32_t *bs, const longlong2 *t_runs,
                                                    int64_t n_trun, const longlong2 *q_runs,
                                                    int64_t n_qrun, const int64_t *q_woff,
                                                    int32_t *coff, int4 *crun,
                                                    uint32_t *bucket) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chains) return;
    const DChain ch = chains[c];
    coff[c] = (int32_t)ch.blk_off;
    if (c == n_chains - 1) coff[n_chains] = (int32_t)nb;
    const int64_t span = (int64_t)ch.tend - ch.tstart;
    const int64_t nbk = span > 0 ? ((span - 1) >> ch.shift) + 1 : 0;
    if (bucket) bucket[ch.idx_off + nbk] = (uint32_t)ch.nblk;  // (null: the index is built later)
    int4 r = make_int4(0, 0, 0, 0);
    if (ch.nblk > 0) {
        if (n_trun) runs_in(t_runs, n_trun, ch.tbase + ch.tstart, ch.tbase + ch.tend, &r.x, &r.y);
        if (n_qrun) {
            const int64_t l = ch.blk_off + ch.nblk - 1;
            const int64_t qs = bq[ch.blk_off], qe = (int64_t)bq[l] + bs[l];
            const int64_t qsize = ch.qinfo & 0x7fffffff, qb = q_woff[ch.q_seq] * 32;
            if (ch.qinfo < 0) runs_in(q_runs, n_qrun, qb + qsize - qe, qb + qsize - qs, &r.z, &r.w);
            else runs_in(q_runs, n_qrun, qb + qs, qb + qe, &r.z, &r.w);
        }
    }
    crun[c] = r;
}

// one lane per chain: its bucket index's terminator (the lazy index build)
__global__ void __launch_bounds__(256) k_bucket_term(const DChain *chains, int64_t n_chains,
                                                     uint32_t *bucket) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chains) return;
    const DChain ch = chains[c];
    const int64_t span = (int64_t)ch.tend - ch.tstart;
    const int64_t nbk = span > 0 ? ((span - 1) >> ch.shift) + 1 : 0;
    bucket[ch.idx_off + nbk] = (uint32_t)ch.nblk;
}

// one lane per 64-block tile: the chain holding its first block
__global__ void __launch_bounds__(256) k_tile_chain(const int32_t *coff, int64_t n_chains,
                                                    int64_t ntiles, int32_t *tile_c0) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles) return;
    if (t == ntiles) {
        tile_c0[t] = (int32_t)(n_chains - 1);
        return;
    }
    const int64_t b = t << 6;
    int64_t lo = 0, hi = n_chains - 1;
    while (lo < hi) {
        const int64_t mid = (lo + hi + 1) >> 1;
        if (coff[mid] <= b) lo = mid;
        else hi = mid - 1;
    }
    tile_c0[t] = (int32_t)lo;
}

// the 12-byte scoring record of a block {t, q, size | N flags} with the gap
// cost to its successor (k_tile reads the 16-byte record of a wide one)
__device__ __forceinline__ Blk12 blk12_of(int t, int q, int zf, int cost) {
    const int z = zf & kSizeMask;
    const bool wide = z >= kB12Wide || cost < 0 || cost >= kB12GapMax;
    Blk12 r;
    r.t = t;
    r.q = q;
    r.w = (wide ? (uint32_t)kB12Wide : ((uint32_t)z | ((uint32_t)cost << 12))) |
          ((uint32_t)(zf & (kTHasN | kQHasN)) << 1);
    return r;
}

// the gap cost between a block and its successor {nt, nq} in the chain
__device__ __forceinline__ int block_gap(const UploadGaps &G, int t, int q, int z, int nt, int nq) {
    int d;
    const int which = gap_kind(nq - (q + z), nt - (t + z), d);
    return d < G.len ? G.tab[which * G.len + d] : gap_cost_wd(G.g, G.small, which, d);
}

// one lane per block: the block record {tStart, qStart, size | N flags, gap},
// its target span, the N flags (blocks of chains whose span meets a run,
// against the same sorted run lists), and the bucket entries it owns (block
// k of a chain is bucket j's first block with tEnd past the bucket start
// for the buckets starting in [tEnd(k-1), tEnd(k))).  GAPS (the scoring is
// set when the chains arrive): the gap costs and the 12-byte records too,
// k_block_gaps_flat's pass folded in; otherwise gap 0 until it runs.
// MODE: 0 everything; 1 the records only (the window-search index -- spans
// and buckets -- is built at the first call that searches windows: chainNet's
// windows and whole chains never do); 2 the index only.
template <bool GAPS, int MODE>
__global__ void __launch_bounds__(256) k_build_flat(const int32_t *bt, const int32_t *bq,
                                                    const int32_t *bs, int64_t nb,
                                                    const DChain *chains, const int32_t *coff,
                                                    const int32_t *tile_c0, int64_t ntiles,
                                                    const int4 *crun, const longlong2 *t_runs,
                                                    int64_t n_trun, const longlong2 *q_runs,
                                                    int64_t n_qrun, const int64_t *q_woff,
                                                    int4 *blk, int2 *tspan, uint32_t *bucket,
                                                    UploadGaps G) {
    __shared__ int32_t s_off[kStage + 1];
    __shared__ int64_t s_tbase[kStage], s_idx[kStage];
    __shared__ int32_t s_ts[kStage], s_te[kStage], s_sh[kStage], s_qseq[kStage], s_qinfo[kStage];
    __shared__ int4 s_run[kStage];
    __shared__ int64_t s_pre[256], s_dst[256];
    __shared__ uint32_t s_val[256];
    const int64_t B0 = (int64_t)blockIdx.x * blockDim.x * kUpPer;
    int t[kUpPer], q[kUpPer], z[kUpPer];
#pragma unroll
    for (int i = 0; i < kUpPer; ++i) {  // (issued before the staging waits)
        const int64_t b = B0 + i * (int64_t)blockDim.x + threadIdx.x;
        t[i] = q[i] = z[i] = 0;
        if (b < nb) t[i] = bt[b], q[i] = bq[b], z[i] = bs[b];
    }
    ChainStage S;
    const bool staged = B0 < nb && stage_offsets(coff, tile_c0, ntiles, B0, s_off, S);
    if (staged) {  // the chain fields the blocks need, one chain per lane
        const int c0 = S.c0;
        for (int j = threadIdx.x; j < S.m; j += blockDim.x) {
            const DChain ch = chains[c0 + j];
            s_tbase[j] = ch.tbase;
            s_idx[j] = ch.idx_off;
            s_ts[j] = ch.tstart;
            s_te[j] = ch.tend;
            s_sh[j] = ch.shift;
            s_qseq[j] = ch.q_seq;
            s_qinfo[j] = ch.qinfo;
            s_run[j] = crun ? crun[c0 + j] : make_int4(0, 0, 0, 0);
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kUpPer; ++i) {
        const int64_t b = B0 + i * (int64_t)blockDim.x + threadIdx.x;
        int64_t cnt = 0, dst = 0;  // this block's bucket entries: cnt from bucket[dst]
        uint32_t val = 0;
        if (b >= nb) {
            if (b < nb + 8) {  // padding: a window search may read 8 past a chain
                if (MODE != 1) tspan[b] = make_int2(0x7fffffff, 0x7fffffff);
                if (MODE != 2) blk[b] = make_int4(0x7fffffff, 0, 0, 0);
            }
        } else {
            int64_t tbase, idx_off, coff_c, coff_n;
            int tstart, tend, shift, q_seq, qinfo;
            int4 rr;
            if (staged) {
                const int j = staged_chain(S, b);
                tbase = s_tbase[j], idx_off = s_idx[j], coff_c = S.off[j], coff_n = S.off[j + 1];
                tstart = s_ts[j], tend = s_te[j], shift = s_sh[j], q_seq = s_qseq[j], qinfo = s_qinfo[j];
                rr = s_run[j];
            } else {
                const int64_t c = owner_chain(coff, tile_c0, ntiles, b);
                const DChain ch = chains[c];
                tbase = ch.tbase, idx_off = ch.idx_off, coff_c = coff[c], coff_n = coff[c + 1];
                tstart = ch.tstart, tend = ch.tend, shift = ch.shift, q_seq = ch.q_seq, qinfo = ch.qinfo;
                rr = crun ? crun[c] : make_int4(0, 0, 0, 0);
            }
            int flags = 0;  // (a block searches only the runs its chain's span meets)
            if (MODE != 2 && !(GAC_UP_PROBE & 2) && z[i] > 0) {
                if (rr.y > rr.x && span_meets(t_runs, rr.x, rr.y, tbase + t[i], tbase + t[i] + z[i]))
                    flags |= kTHasN;
                if (rr.w > rr.z) {
                    const int64_t qb = q_woff[q_seq] * 32;
                    const int64_t qf = qinfo < 0 ? (int64_t)(qinfo & 0x7fffffff) - q[i] - z[i] : q[i];
                    if (span_meets(q_runs, rr.z, rr.w, qb + qf, qb + qf + z[i])) flags |= kQHasN;
                }
            }
            int cost = 0;
            if (GAPS && MODE != 2) {
                if (b + 1 < coff_n) cost = block_gap(G, t[i], q[i], z[i], bt[b + 1], bq[b + 1]);
                if (!(GAC_UP_PROBE & 4)) G.blk12[b] = blk12_of(t[i], q[i], z[i] | flags, cost);
            }
            if (MODE != 2) blk[b] = make_int4(t[i], q[i], z[i] | flags, cost);
            if (MODE != 1 && !(GAC_UP_PROBE & 4)) tspan[b] = make_int2(t[i], t[i] + z[i]);
            const int64_t k = b - coff_c;
            const int64_t span = (int64_t)tend - tstart;
            const int64_t nbk = span > 0 ? ((span - 1) >> shift) + 1 : 0;
            const int64_t round = ((int64_t)1 << shift) - 1;
            const int64_t k0 = k ? ((int64_t)bt[b - 1] + bs[b - 1] - tstart + round) >> shift : 0;
            int64_t k1 = ((int64_t)t[i] + z[i] - tstart + round) >> shift;
            if (k1 > nbk) k1 = nbk;
            if (MODE != 1 && !(GAC_UP_PROBE & 1) && k1 > k0)
                cnt = k1 - k0, dst = idx_off + k0, val = (uint32_t)k;
        }
        if (MODE == 1) continue;  // (no bucket entries: uniform over the workgroup)
        // the wave's bucket entries, lane-strided: a block after a wide gap
        // owns many, and a loop per block left the other lanes idle.  Entry e
        // of the wave belongs to the last lane whose exclusive count is <= e.
        const int lane = threadIdx.x & 63, wb = threadIdx.x & ~63;
        int64_t pre = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(pre, o, 64);
            if (lane >= o) pre += y;
        }
        const int64_t tot = __shfl(pre, 63, 64);
        s_pre[threadIdx.x] = pre - cnt;
        s_dst[threadIdx.x] = dst;
        s_val[threadIdx.x] = val;
        __syncthreads();
        for (int64_t e = lane; e < tot; e += 64) {
            int lo = 0, hi = 63;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_pre[wb + mid] <= e) lo = mid;
                else hi = mid - 1;
            }
            bucket[s_dst[wb + lo] + (e - s_pre[wb + lo])] = s_val[wb + lo];
        }
        __syncthreads();  // (the next round's entries reuse the arrays)
    }
}

// k_block_gaps one lane per block (the chain only says whether the block is
// its last)
__global__ void __launch_bounds__(256) k_block_gaps_flat(const int32_t *coff,
                                                         const int32_t *tile_c0, int64_t ntiles,
                                                         int64_t nb, int4 *blk, Blk12 *blk12,
                                                         UploadGaps G) {
    __shared__ int32_t s_off[kStage + 1];
    const int64_t B0 = (int64_t)blockIdx.x * blockDim.x * kUpPer;
    int4 x[kUpPer];
#pragma unroll
    for (int i = 0; i < kUpPer; ++i) {  // (issued before the staging waits)
        const int64_t b = B0 + i * (int64_t)blockDim.x + threadIdx.x;
        x[i] = b < nb ? blk[b] : make_int4(0, 0, 0, 0);
    }
    ChainStage S;
    const bool staged = stage_offsets(coff, tile_c0, ntiles, B0, s_off, S);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kUpPer; ++i) {
        const int64_t b = B0 + i * (int64_t)blockDim.x + threadIdx.x;
        if (b >= nb) break;
        const int64_t next = staged ? S.off[staged_chain(S, b) + 1]
                                    : coff[owner_chain(coff, tile_c0, ntiles, b) + 1];
        const int z = x[i].z & kSizeMask;
        int cost = 0;
        if (b + 1 < next) {
            const int4 y = blk[b + 1];
            cost = block_gap(G, x[i].x, x[i].y, z, y.x, y.y);
        }
        blk[b] = make_int4(x[i].x, x[i].y, x[i].z, cost);
        blk12[b] = blk12_of(x[i].x, x[i].y, x[i].z, cost);
    }
}

// ------------------------------------------------------------ k_plan -----
// First k in [0, n) with pred(k) true (pred monotone false..true), n if none:
// gallop from guess g, then binary search the bracket.
template <class P>
__device__ __forceinline__ int gallop_first(int n, int g, P pred) {
    if (n <= 0) return 0;
    g = g < 0 ? 0 : (g > n - 1 ? n - 1 : g);
    int lo, hi;
    if (pred(g)) {
        hi = g;
        int x = g - 1, step = 1;
        while (x >= 0 && pred(x)) {
            hi = x;
            x -= step;
            step <<= 1;
        }
        lo = x + 1 > 0 ? x + 1 : 0;
    } else {
        lo = g + 1;
        int x = g + 1, step = 1;
        while (x < n && !pred(x)) {
            lo = x + 1;
            x += step;
            step <<= 1;
        }
        hi = x < n ? x : n;
    }
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (pred(mid)) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// Window of blocks [first, stop) of range r: tEnd > s and tStart < e
// (chainSubsetOnT's first-block walk and stop condition, chain.c:481-500),
// plus the descriptor k_tile needs.  Planning is a chain of dependent random
// accesses, so it is built for few of them: the 64-byte chain record, the
// chain's bucket index (upload-time; bucket k of 2^shift target bases holds
// the first block ending past its start), which brackets the first block,
// then ONE 64-byte load of 8 block spans that settles the window start and,
// for most windows, its end.
__device__ __forceinline__ RangeDesc plan_range(const ScoreArgs &a, const Range r) {
    RangeDesc d;
    d.tbase = 0;
    d.qbase = 0;
    d.b0 = 0;
    d.nblk = 0;
    d.s = r.t_start;
    d.e = r.t_end;
    if (r.chain < 0 || r.chain >= a.n_chains || r.t_start >= r.t_end) return d;
    const DChain c = a.chains[r.chain];
    d.tbase = c.tbase;
    d.qbase = c.qbase;
    const int n = c.nblk;
    if (n == 0) return d;
    const int2 *sp = a.tspan + c.blk_off;
    const int s = r.t_start, e = r.t_end;
    if (s <= c.tstart && e >= c.tend) {
        // chainFastSubsetOnT's easy case (chain.c:499-505): the whole chain,
        // zero-size end blocks included (no clipping inside [s, e) either)
        d.nblk = n;
        d.b0 = (int32_t)c.blk_off;
        return d;
    }
    int lo, hi;  // the first block with tEnd > s is in [lo, hi]
    if (s < c.tstart) {
        lo = hi = 0;
    } else if (s >= c.tend) {
        lo = hi = n;
    } else {
        const int k = (s - c.tstart) >> c.shift;
        const u32x2a4 br = *reinterpret_cast<const u32x2a4 *>(a.bucket + c.idx_off + k);
        lo = (int)br.x;
        hi = (int)br.y;
    }
    // spans of blocks lo .. lo+7 (the span array is padded by 8 entries, so
    // reading past this chain is safe; those entries are masked)
    int2 v[8];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
        const i32x4a8 x = *reinterpret_cast<const i32x4a8 *>(sp + lo + j);
        v[j] = make_int2(x.x, x.y);
        v[j + 1] = make_int2(x.z, x.w);
    }
    int cnt = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) cnt += (lo + j < hi && v[j].y <= s) ? 1 : 0;
    int first = lo + cnt;
    if (cnt == 8 && first < hi) {  // dense bucket: binary search the rest
        int l2 = first, h2 = hi;
        while (l2 < h2) {
            const int mid = (l2 + h2) >> 1;
            if (sp[mid].y > s) h2 = mid;
            else l2 = mid + 1;
        }
        first = l2;
    }
    // first block >= first with tStart >= e (or n)
    int stop = -1;
    if (e > c.tend) {
        stop = n;
    } else {
#pragma unroll
        for (int j = 7; j >= 0; --j) {
            const int bj = lo + j;
            if (bj >= first && (bj >= n || v[j].x >= e)) stop = bj < n ? bj : n;
        }
        if (stop < 0) {  // long window: gallop on
            const int from = max(first, lo + 8);
            stop = from + gallop_first(n - from, 0, [&](int k) { return sp[from + k].x >= e; });
        }
    }
    d.nblk = stop - first;
    d.b0 = (int32_t)(c.blk_off + first);
    return d;
}

// A range whose window the caller knows (gac_score_windows: chainNet's
// netting found each fill's blocks while making it, chainNet.c:557-608):
// only the chain record is read.  A range covering the chain is the whole
// chain, as in plan_range; a window outside its chain sets `bad` and selects
// nothing.
__device__ __forceinline__ RangeDesc plan_window(const ScoreArgs &a, const Window w, bool &bad) {
    RangeDesc d;
    d.tbase = 0;
    d.qbase = 0;
    d.b0 = 0;
    d.nblk = 0;
    d.s = w.t_start;
    d.e = w.t_end;
    if (w.chain < 0 || w.chain >= a.n_chains) {
        bad = true;
        return d;
    }
    const DChain c = a.chains[w.chain];
    d.tbase = c.tbase;
    d.qbase = c.qbase;
    if (w.first < 0 || w.nblk < 0 || (int64_t)w.first + w.nblk > c.nblk) {
        bad = true;
        return d;
    }
    if (c.nblk == 0 || w.t_start >= w.t_end) return d;
    if (w.t_start <= c.tstart && w.t_end >= c.tend) {  // chain.c:499-505
        d.nblk = c.nblk;
        d.b0 = (int32_t)c.blk_off;
        return d;
    }
    d.nblk = w.nblk;
    d.b0 = (int32_t)(c.blk_off + w.first);
    return d;
}

// ------------------------------------------------------------ k_plan -----
// One lane per range: plan, then the workgroup's scan of its window blocks:
// goff[i] = exclusive prefix inside plan workgroup w = i / 256, pb0[i] =
// first window block, agg[w] = the workgroup's total.  Nothing crosses
// workgroups here (an in-kernel hand-off of the totals -- counter fan-in and
// a last-arriver scan -- cost more than the separate one-workgroup
// k_scan_agg launch).
constexpr int kPlanWG = 256;

__device__ __forceinline__ long long wg_exclusive_scan(long long v, long long *s_wsum,
                                                      long long &total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    long long incl = v;
#pragma unroll
    for (int k = 1; k < kWave; k <<= 1) {
        const long long o = __shfl_up(incl, k, kWave);
        if (lane >= k) incl += o;
    }
    if (lane == kWave - 1) s_wsum[wave] = incl;
    __syncthreads();
    long long pre = 0;
    total = 0;
#pragma unroll
    for (int w = 0; w < kPlanWG / kWave; ++w) {
        const long long x = s_wsum[w];
        if (w < wave) pre += x;
        total += x;
    }
    __syncthreads();
    return pre + incl - v;
}

template <bool WIN>
__global__ void __launch_bounds__(kPlanWG, 8) k_plan(ScoreArgs a) {
    __shared__ long long s_wsum[kPlanWG / kWave];
    const int tid = threadIdx.x;
    const int64_t i = (int64_t)blockIdx.x * kPlanWG + tid;
    int nb = 0;
    if (i < a.n) {
        bool bad = false;
        const RangeDesc d = WIN ? plan_window(a, a.wins[i], bad) : plan_range(a, a.ranges[i]);
        if (WIN && bad) atomicOr(&a.status[5], 1);
        a.rdesc[i] = d;
        a.nblk[i] = nb = d.nblk;
        a.pb0[i] = d.b0;
        if (nb == 0) {
            a.out_g[i] = 0;
            a.out_ali[i] = 0;
            if (a.want_local) a.out_l[i] = 0;
        }
    }
    // 64-bit: 256 windows of a huge chain may exceed int32 (saturated; the
    // host reports it)
    long long agg;
    const long long excl = wg_exclusive_scan(nb, s_wsum, agg);
    if (i < a.n) a.goff[i] = (int32_t)(excl < 0x7fffffffLL ? excl : 0x7fffffffLL);
    if (tid == 0) a.agg[blockIdx.x] = (int32_t)(agg < 0x7fffffffLL ? agg : 0x7fffffffLL);
}

// Scan of the plan workgroups' totals by one workgroup (k_scan_agg): flat
// offsets (plan_off).  Thread t owns workgroups [8t, 8t + 8) of each batch of
// 2048, loaded all at once.  Returns W (saturated at INT32_MAX).
__device__ long long scan_totals(const ScoreArgs &a, int G, long long *s_wsum) {
    constexpr int kPer = 8, kBatch = kPer * kPlanWG;
    const int tid = threadIdx.x;
    long long W = 0;
    for (int b0 = 0; b0 < G; b0 += kBatch) {
        int32_t v[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int w = b0 + tid * kPer + k;
            v[k] = w < G ? a.agg[w] : 0;
        }
        long long mine = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) mine += v[k];
        long long bw;
        long long run = W + wg_exclusive_scan(mine, s_wsum, bw);
        W += bw;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int w = b0 + tid * kPer + k;
            if (w < G) a.plan_off[w] = (int32_t)(run < 0x7fffffffLL ? run : 0x7fffffffLL);
            run += v[k];
        }
    }
    return W > 0x7fffffffLL ? 0x7fffffffLL : W;
}

// {W, T, overflow} for the later kernels, and the same, tagged with the
// call's sequence number, straight into the host's pinned status words: the
// host learns whether the workspace sufficed as soon as this kernel ends,
// while k_tilemap / k_tile / the folds still run.
// bad: a window lay outside its chain (k_plan<true> sets status[5], read
// here and cleared for the next call; k_plan_lb carries it in its words)
__device__ __forceinline__ void publish_status(const ScoreArgs &a, long long W, int32_t bad) {
    const long long T = (W + kTileBlocks - 1) / kTileBlocks;
    const bool over = W >= 0x7fffffffLL || T > a.cap_tiles;
    const int32_t st[4] = {(int32_t)W, (int32_t)T, over ? 1 : 0, bad};
    for (int k = 0; k < 4; ++k) {
        a.status[k] = k == 3 ? 0 : st[k];
        __hip_atomic_store(&a.host_status[k], st[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (bad) a.status[5] = 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system scope: values before the tag
    __hip_atomic_store(&a.host_status[4], a.call_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void __launch_bounds__(kPlanWG) k_scan_agg(ScoreArgs a) {
    __shared__ long long s_wsum[kPlanWG / kWave];
    const int G = (int)((a.n + kPlanWG - 1) / kPlanWG);
    const long long W = scan_totals(a, G, s_wsum);
    if (threadIdx.x == 0) publish_status(a, W, a.status[5]);
}

// ------------------------------------------------------------ k_tilemap --
// One lane per range: its flat offset (gflat), and, for every tile whose
// first flat block falls in its window, tile_r0[tile] = the range.  k_tile
// finds the owner of each of a tile's blocks from there with an LDS search
// over the next 64 ranges' offsets (no per-block map in HBM).
__global__ void __launch_bounds__(kPlanWG) k_tilemap(ScoreArgs a) {
    if (a.status[2]) return;  // workspace overflow: the host grows it and reruns
    const int64_t i = (int64_t)blockIdx.x * kPlanWG + threadIdx.x;
    if (i >= a.n) return;
    const int nb = a.nblk[i];
    const int g = a.plan_off[i / kPlanWG] + a.goff[i];
    a.gflat[i] = g;
    if (nb > 0) {
        const int64_t end = (int64_t)g + nb;
        for (int64_t t = ((int64_t)g + kTileBlocks - 1) / kTileBlocks; t * kTileBlocks < end; ++t)
            a.tile_r0[t] = (int32_t)i;
    }
}

// k_tilemap with k_scan_agg folded in, for up to kFusedMapWG plan
// workgroups (1 M ranges): every workgroup sums the plan-workgroup totals
// itself -- all of them for W, those before it for its own offset -- so the
// one-workgroup scan launch disappears.  Workgroup 0 publishes the status
// words; on overflow every workgroup stops before writing the map.
constexpr int kFusedMapWG = 4096;

__global__ void __launch_bounds__(kPlanWG) k_tilemap_fused(ScoreArgs a) {
    __shared__ long long s_part[2][kPlanWG / kWave];
    const int G = (int)((a.n + kPlanWG - 1) / kPlanWG);
    const int w = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    long long tot = 0, pre = 0;
    for (int k = tid; k < G; k += kPlanWG) {
        const long long v = a.agg[k];
        tot += v;
        if (k < w) pre += v;
    }
    tot = wave_sum(tot);
    pre = wave_sum(pre);
    if (lane == 0) {
        s_part[0][wave] = tot;
        s_part[1][wave] = pre;
    }
    __syncthreads();
    tot = pre = 0;
#pragma unroll
    for (int k = 0; k < kPlanWG / kWave; ++k) {
        tot += s_part[0][k];
        pre += s_part[1][k];
    }
    const long long W = tot > 0x7fffffffLL ? 0x7fffffffLL : tot;
    if (w == 0 && tid == 0) publish_status(a, W, a.status[5]);
    const long long T = (W + kTileBlocks - 1) / kTileBlocks;
    if (W >= 0x7fffffffLL || T > a.cap_tiles) return;  // the host grows the workspace, reruns
    if (tid == 0) a.plan_off[w] = (int32_t)pre;
    const int64_t i = (int64_t)w * kPlanWG + tid;
    if (i >= a.n) return;
    const int nb = a.nblk[i];
    const int g = (int)pre + a.goff[i];
    a.gflat[i] = g;
    if (nb > 0) {
        const int64_t end = (int64_t)g + nb;
        for (int64_t t = ((int64_t)g + kTileBlocks - 1) / kTileBlocks; t * kTileBlocks < end; ++t)
            a.tile_r0[t] = (int32_t)i;
    }
}

// ------------------------------------------------------------ k_plan_lb --
// k_plan, k_scan_agg and k_tilemap as ONE pass (a single-pass scan with
// decoupled look-back): a workgroup takes a ticket (tickets follow the order
// the chip started the workgroups, so every workgroup it waits for is already
// running), plans its 256 ranges, publishes its window-block total, adds up
// its predecessors' words back to the first one holding an inclusive prefix,
// publishes its own inclusive prefix, and writes gflat and its tiles'
// tile_r0 straight away.  A word is self-contained -- {state, call tag, bad
// window seen, value} in 64 bits -- so the words need no ordering against
// other memory: relaxed agent-scope atomics (coherent across the XCDs' L2s,
// no L2 write-back or invalidate per workgroup; a release/acquire pair per
// word cost 28 ms per 13 M-window call, r06lb).  The tag makes an earlier
// call's words read as "not yet", so nothing is cleared per call.  The last
// ticket publishes {W, T, overflow, bad} (publish_status) and re-arms the
// ticket counter.  Saves the per-range goff and agg round trip through HBM
// and two launches (C5 fills, 13.2 M windows: k_plan + k_scan_agg +
// k_tilemap = 0.25 + 0.07 + 0.04 ms, r06final).
constexpr unsigned long long kLbAgg = 1ull << 62, kLbInc = 2ull << 62, kLbBad = 1ull << 31;
constexpr unsigned long long kLbTagMask = 0x3fffffffull << 32;

__device__ __forceinline__ unsigned long long lb_word(long long v, int32_t tag, bool bad,
                                                      unsigned long long state) {
    const unsigned long long sv = (unsigned long long)(v < 0x7fffffffLL ? v : 0x7fffffffLL);
    return state | ((unsigned long long)(tag & 0x3fffffff) << 32) | (bad ? kLbBad : 0ull) | sv;
}

// ranges per k_plan_lb workgroup: kLbSlabs slabs of 256 (fewer workgroups,
// so fewer look-back words per range; r06lb3: one slab per workgroup took
// 0.64 ms for the 13.2 M C5 fills against 0.36 ms for the three launches)
constexpr int kLbSlabs = 8;
constexpr int kLbRanges = kLbSlabs * kPlanWG;
int plan_lb_grid(int64_t n) { return (int)((n + kLbRanges - 1) / kLbRanges); }

template <bool WIN>
__global__ void __launch_bounds__(kPlanWG, 8) k_plan_lb(ScoreArgs a) {
    __shared__ long long s_wsum[kPlanWG / kWave];
    __shared__ int s_ticket, s_bad;
    __shared__ long long s_pre;
    const int tid = threadIdx.x;
    if (tid == 0) {
        s_ticket = __hip_atomic_fetch_add(&a.status[8], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_bad = 0;
    }
    __syncthreads();
    const int w = s_ticket;
    const int64_t i0 = (int64_t)w * kLbRanges + tid;
    int nbk[kLbSlabs];
    long long exk[kLbSlabs];
    long long agg = 0;
#pragma unroll
    for (int k = 0; k < kLbSlabs; ++k) {
        const int64_t i = i0 + (int64_t)k * kPlanWG;
        int nb = 0;
        if (i < a.n) {
            bool bad = false;
            const RangeDesc d = WIN ? plan_window(a, a.wins[i], bad) : plan_range(a, a.ranges[i]);
            if (WIN && bad) s_bad = 1;
            a.rdesc[i] = d;
            a.nblk[i] = nb = d.nblk;
            a.pb0[i] = d.b0;
            if (nb == 0) {
                a.out_g[i] = 0;
                a.out_ali[i] = 0;
                if (a.want_local) a.out_l[i] = 0;
            }
        }
        nbk[k] = nb;
    }
#pragma unroll
    for (int k = 0; k < kLbSlabs; ++k) {  // slab by slab: range order
        long long tot;
        exk[k] = agg + wg_exclusive_scan(nbk[k], s_wsum, tot);  // (its barriers order s_bad)
        agg += tot;
    }
    if (tid < kWave) {  // wave 0: the look-back, 64 predecessors' words per load
        unsigned long long *F = a.lbflag;
        const unsigned long long tagbits = (unsigned long long)(a.call_tag & 0x3fffffff) << 32;
        bool bad = s_bad != 0;
        long long pre = 0;
        if (tid == 0)
            __hip_atomic_store(&F[w], lb_word(agg, a.call_tag, bad, w == 0 ? kLbInc : kLbAgg),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (w > 0) {
            for (int j = w - 1;;) {
                // lane k: the word of workgroup j - k (before workgroup 0: an
                // inclusive zero)
                const int q = j - tid;
                const unsigned long long f =
                    q >= 0 ? __hip_atomic_load(&F[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : (kLbInc | tagbits);
                const bool ok = (f & kLbTagMask) == tagbits && (f >> 62) != 0;
                const bool inc = ok && (f >> 62) == 2;
                const unsigned long long incs = __ballot(inc);
                const unsigned long long oks = __ballot(ok);
                // the words up to the nearest inclusive one (all 64 if none)
                const int upto = incs ? __builtin_ctzll(incs) : kWave - 1;
                const unsigned long long need = upto == kWave - 1 ? ~0ull : ((2ull << upto) - 1);
                if ((oks & need) != need) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                const bool mine = tid <= upto;
                pre += wave_sum(mine ? (long long)(f & 0x7fffffffull) : 0ll);
                bad = bad || __ballot(mine && (f & kLbBad)) != 0ull;
                if (incs) break;
                j -= kWave;
            }
            if (pre > 0x7fffffffLL) pre = 0x7fffffffLL;
            if (tid == 0)
                __hip_atomic_store(&F[w], lb_word(pre + agg, a.call_tag, bad, kLbInc),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (tid == 0) {
            s_pre = pre;
            if (w == (int)gridDim.x - 1) {  // every predecessor's word is in: W is known
                const long long W = pre + agg;
                __hip_atomic_store(&a.status[8], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                publish_status(a, W > 0x7fffffffLL ? 0x7fffffffLL : W, bad ? 1 : 0);
            }
        }
    }
    __syncthreads();
    const long long pre = s_pre;
#pragma unroll
    for (int k = 0; k < kLbSlabs; ++k) {
        const int64_t i = i0 + (int64_t)k * kPlanWG;
        if (i >= a.n) break;
        const int nb = nbk[k];
        const long long g = pre + exk[k];
        a.gflat[i] = (int32_t)(g < 0x7fffffffLL ? g : 0x7fffffffLL);
        if (nb > 0 && g + nb < 0x7fffffffLL) {
            // (tiles past the workspace are left out; the last ticket's status
            // words tell k_tile, the folds and the host to grow it and rerun)
            const int64_t end = g + nb, cap = a.cap_tiles;
            for (int64_t t = (g + kTileBlocks - 1) / kTileBlocks; t * kTileBlocks < end && t < cap; ++t)
                a.tile_r0[t] = (int32_t)i;
        }
    }
}

// ------------------------------------------------------------ k_whole_plan
// Whole-chain calls (scoreChain: every chain of a set, in order) need no
// window search: the plan of "range c = chain c" is fixed per chain set, so
// it is built once (first gac_score_chains call) into the same workspace
// shapes k_tile and the folds read -- rdesc, nblk, gflat (= pb0 = the chain's
// first block), tile_r0 -- and a call is k_tile + the fold.  One lane per
// chain.
__global__ void __launch_bounds__(256) k_whole_plan(const DChain *chains, int64_t n,
                                                    RangeDesc *rdesc, int32_t *nblk,
                                                    int32_t *gflat, int32_t *tile_r0) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const DChain ch = chains[c];
    RangeDesc d;
    d.tbase = ch.tbase;
    d.qbase = ch.qbase;
    d.b0 = (int32_t)ch.blk_off;
    d.nblk = ch.nblk;
    d.s = ch.tstart;
    d.e = ch.tend;
    rdesc[c] = d;
    nblk[c] = ch.nblk;
    gflat[c] = (int32_t)ch.blk_off;
    const int64_t g = ch.blk_off, end = g + ch.nblk;
    for (int64_t t = (g + kTileBlocks - 1) / kTileBlocks; t * kTileBlocks < end; ++t)
        tile_r0[t] = (int32_t)c;
}

// The same plan with the chains in target order (position p = chain perm[p]):
// chains that overlap on the target are scored by neighbouring tiles, so an
// XCD's L2 (and the Infinity Cache) serves their shared target-plane lines
// once instead of once per chain.  Flat offsets are the scan of the permuted
// block counts; the results of position p are stored straight to chain
// perm[p] (out_perm).
constexpr int kOrderBits = 36;  // sort key bits: global target base of the chain start

__global__ void __launch_bounds__(256) k_whole_keys(const DChain *chains, int64_t n,
                                                    unsigned long long *key, int32_t *val) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const DChain ch = chains[c];
    key[c] = ch.nblk > 0 ? (unsigned long long)(ch.tbase + ch.tstart)
                         : (1ull << kOrderBits) - 1;  // empty chains last
    val[c] = (int32_t)c;
}

__global__ void __launch_bounds__(256) k_whole_count(const DChain *chains, const int32_t *perm,
                                                     int64_t n, int32_t *nblk) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    nblk[p] = chains[perm[p]].nblk;
}

__global__ void __launch_bounds__(256) k_whole_plan_sorted(const DChain *chains,
                                                           const int32_t *perm, int64_t n,
                                                           const int32_t *gflat, RangeDesc *rdesc,
                                                           int32_t *pb0, int32_t *tile_r0,
                                                           int32_t *inv) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= n) return;
    const int32_t c = perm[p];
    const DChain ch = chains[c];
    RangeDesc d;
    d.tbase = ch.tbase;
    d.qbase = ch.qbase;
    d.b0 = (int32_t)ch.blk_off;
    d.nblk = ch.nblk;
    d.s = ch.tstart;
    d.e = ch.tend;
    rdesc[p] = d;
    pb0[p] = (int32_t)ch.blk_off;
    inv[c] = ch.nblk > 0 ? (int32_t)p : -1;
    const int64_t g = gflat[p], end = g + ch.nblk;
    for (int64_t t = (g + kTileBlocks - 1) / kTileBlocks; t * kTileBlocks < end; ++t)
        tile_r0[t] = (int32_t)p;
}

// Whole-chain tile schedule: key of tile t = global target base of its
// first block (set order: flat block = block index, the tile's first chain
// is tile_r0[t]).
__global__ void __launch_bounds__(256) k_tile_keys(const DChain *chains, const int4 *blk,
                                                   const int32_t *tile_r0, int64_t T,
                                                   unsigned long long *key, int32_t *val) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const DChain c = chains[tile_r0[t]];
    key[t] = (unsigned long long)(c.tbase + blk[t * kTileBlocks].x);
    val[t] = (int32_t)t;
}

// outputs of the ranges in `list` (chains without blocks) := 0
__global__ void __launch_bounds__(256) k_zero_list(const int32_t *list, int64_t n, long long *g,
                                                   long long *l, int32_t *ali) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int32_t r = list[i];
    g[r] = 0;
    ali[r] = 0;
    if (l) l[r] = 0;
}

// ------------------------------------------------------------ k_tile -----
// One wave per tile of 64 consecutive flat blocks (ranges packed densely,
// many per tile).  Per tile: one round trip for the range descriptors and
// blocks (the lane -> (range, block) map was prefetched during the previous
// tile), one for the 2-bit windows (16-byte loads; N masks only for blocks
// flagged at upload), then segmented per-range scans.
struct WaveLds {
    int cg[kTileBlocks];          // flat offsets of the tile's candidate ranges r0 + k
    int cb[kTileBlocks];          // their first window blocks
    int coff[kTileBlocks];        // exclusive chunk prefix per lane-block
    long long tpos[kTileBlocks];  // global base index of the clipped target start
    long long qpos[kTileBlocks];  // '+': global base index of the clipped query start
                                  // '-': global base index of (qSize - clipped qStart)
    int lenq[kTileBlocks];        // clipped length | minus << 31 | qN << 30 | tN << 29
    unsigned long long acc[kTileBlocks];  // block scores (int64: a block may be huge)
};

constexpr int kLenMask = kSizeMask;  // lenq: len | tN (bit 29) | qN (bit 30) | minus (bit 31)

// One 32-base chunk of a tile, split into address preparation, loads and
// evaluation so that the loads of a lane's two chunks are issued together,
// with no branch between them (a branch makes the compiler wait for every
// load in flight).
struct ChunkRef {
    uint32_t tw, qw;  // first plane word of the target / query window
    uint32_t m;       // n (bits 0-5, 0 = no chunk) | target shift (6-10) | query shift
                      // (11-15) | block k (16-21) | minus (22) | tN (23) | qN (24)
};

// (packed: three registers per chunk instead of seven -- k_tile's register
// peak is its two chunks in flight)
__device__ __forceinline__ ChunkRef make_chunk(int64_t tp, int64_t qp, int n, int lq, int k) {
    ChunkRef c;
    c.tw = (uint32_t)(tp >> 5);
    c.qw = (uint32_t)(qp >> 5);
    c.m = (uint32_t)n | ((uint32_t)(tp & 31) << 6) | ((uint32_t)(qp & 31) << 11) |
          ((uint32_t)k << 16) | ((uint32_t)lq >> 31 << 22) |
          ((uint32_t)(lq & (kTHasN | kQHasN)) >> 29 << 23);
    return c;
}
__device__ __forceinline__ int chunk_n(const ChunkRef &c) { return (int)(c.m & 63u); }
__device__ __forceinline__ int chunk_k(const ChunkRef &c) { return (int)((c.m >> 16) & 63u); }

__device__ __forceinline__ ChunkRef chunk_prep(const WaveLds &L, int j);

struct ChunkRaw {
    u32x4a8 t, q;  // plane words w, w+1 ({p0, p1} each)
};

// (non-temporal loads measured slower here: k_tile 1.32 vs 1.13 ms on the
// C5 fills, r03d)
__device__ __forceinline__ ChunkRaw chunk_load(const ScoreArgs &a, const ChunkRef &c) {
    ChunkRaw r;
    r.t = *reinterpret_cast<const u32x4a8 *>(a.t_planes + c.tw);
    r.q = *reinterpret_cast<const u32x4a8 *>(a.q_planes + c.qw);
    return r;
}

__device__ __forceinline__ uint32_t load_nmask_w(const uint32_t *nmask, uint32_t w, int sh) {
    const u32x2a4 v = *reinterpret_cast<const u32x2a4 *>(nmask + w);
    return funnel(v.y, v.x, sh);
}

// sum over the positions in v of the matrix score, in the multilinear basis
// (t1, t0, d1, d0), d = q ^ t (see ScoreArgs::coef): one AND + popcount +
// 24-bit multiply-add per term.  Strand-symmetric matrices (M[comp q][comp t]
// = M[q][t]; comp flips bit 1) have no t1 terms: 8 instead of 16.
template <bool SYM>
__device__ __forceinline__ int score_bits(const ScoreArgs &a, uint32_t v, uint32_t t0,
                                          uint32_t t1, uint32_t d0, uint32_t d1) {
    const uint32_t m2 = v & d1, m1 = v & d0, m4 = v & t0;
    const uint32_t m3 = m2 & d0, m6 = m4 & d1, m5 = m4 & d0, m7 = m6 & d0;
    int sc = __mul24(a.coef[0], (int)__builtin_popcount(v));
    sc += __mul24(a.coef[1], (int)__builtin_popcount(m1));
    sc += __mul24(a.coef[2], (int)__builtin_popcount(m2));
    sc += __mul24(a.coef[3], (int)__builtin_popcount(m3));
    sc += __mul24(a.coef[4], (int)__builtin_popcount(m4));
    sc += __mul24(a.coef[5], (int)__builtin_popcount(m5));
    sc += __mul24(a.coef[6], (int)__builtin_popcount(m6));
    sc += __mul24(a.coef[7], (int)__builtin_popcount(m7));
    if (!SYM) {
        const uint32_t u = v & t1;
        sc += __mul24(a.coef[8], (int)__builtin_popcount(u));
        sc += __mul24(a.coef[9], (int)__builtin_popcount(u & d0));
        sc += __mul24(a.coef[10], (int)__builtin_popcount(u & d1));
        sc += __mul24(a.coef[11], (int)__builtin_popcount(u & d1 & d0));
        sc += __mul24(a.coef[12], (int)__builtin_popcount(u & t0));
        sc += __mul24(a.coef[13], (int)__builtin_popcount(u & t0 & d0));
        sc += __mul24(a.coef[14], (int)__builtin_popcount(u & t0 & d1));
        sc += __mul24(a.coef[15], (int)__builtin_popcount(u & m7));
    }
    return sc;
}

// Score of a chunk: all positions first; N positions (blocks flagged at
// upload only -- rare) are then subtracted, so the common path carries no
// N-mask loads.
template <bool SYM>
__device__ __forceinline__ int chunk_eval(const ScoreArgs &a, const ChunkRef &c,
                                          const ChunkRaw &r) {
    const int n = chunk_n(c);
    const int sht = (int)((c.m >> 6) & 31u), shq = (int)((c.m >> 11) & 31u);
    const uint32_t t0 = funnel(r.t.z, r.t.x, sht), t1 = funnel(r.t.w, r.t.y, sht);
    uint32_t q0 = funnel(r.q.z, r.q.x, shq), q1 = funnel(r.q.w, r.q.y, shq);
    const bool minus = (c.m >> 22) & 1u;
    const int sh = 32 - n;
    if (minus) {
        // '-' strand: rc base j = comp(fwd[qSize-1-(qp+j)]), comp = code ^ 2;
        // the window was read at the forward position of the chunk's end
        q0 = __builtin_bitreverse32(q0) >> sh;
        q1 = ~(__builtin_bitreverse32(q1) >> sh);
    }
    const uint32_t v = n >= 32 ? 0xffffffffu : ((1u << n) - 1u);
    const uint32_t d0 = q0 ^ t0, d1 = q1 ^ t1;
    int sc = score_bits<SYM>(a, v, t0, t1, d0, d1);
    if (c.m & (3u << 23)) {
        uint32_t nm = 0;
        if (c.m & (1u << 23)) nm = load_nmask_w(a.t_nmask, c.tw, sht);
        if (c.m & (1u << 24)) {
            const uint32_t qn = load_nmask_w(a.q_nmask, c.qw, shq);
            nm |= minus ? __builtin_bitreverse32(qn) >> sh : qn;
        }
        sc -= score_bits<SYM>(a, v & nm, t0, t1, d0, d1);
    }
    return sc;
}

// Block owning chunk j: the largest k with coff[k] <= j (coff is
// non-decreasing; blocks without chunks share the next block's offset and
// lanes past the tile's end hold the chunk total, so no bounds are needed).
// 4-ary: three rounds of three independent LDS reads.
__device__ __forceinline__ int find_chunk_block(const WaveLds &L, int j) {
    int k = 0;
#pragma unroll
    for (int step = 16; step > 0; step >>= 2) {
        const int c1 = L.coff[k + step], c2 = L.coff[k + 2 * step], c3 = L.coff[k + 3 * step];
        k += step * ((c1 <= j) + (c2 <= j) + (c3 <= j));
    }
    return k;
}

// Chunk j of the tile: its block, base count and plane positions.  j past
// the tile's chunks yields n <= 0 with in-bounds positions.
__device__ __forceinline__ ChunkRef chunk_prep(const WaveLds &L, int j) {
    const int k = find_chunk_block(L, j);
    const int lq = L.lenq[k];
    int off = (j - L.coff[k]) << 5;
    int n = min(32, (lq & kLenMask) - off);
    if (n <= 0) {
        off = 0;
        n = 0;
    }
    // '-': read the forward window that ends where the chunk starts
    const int64_t qp = lq < 0 ? L.qpos[k] - off - n : L.qpos[k] + off;
    return make_chunk(L.tpos[k] + off, qp, n, lq, k);
}

template <bool LOCAL>
__device__ __forceinline__ void seg_store(const ScoreArgs &a, int ri, long long g, int ali,
                                          const Elem &e) {
    const int o = a.out_perm ? a.out_perm[ri] : ri;
    a.out_g[o] = g;
    a.out_ali[o] = ali;
    if (LOCAL) a.out_l[o] = max2(0, max2(e.C, e.D));
}

// one step of k_tile's segmented (by range) inclusive scan: the source
// lane's (g, ali, local element) folded in front when it lies in my segment
template <int K, bool LOCAL>
__device__ __forceinline__ void seg_scan_step(long long &vg, int &va, Elem &e, int lane, int seg0) {
    constexpr int C = ScanCtl<K>::c, RM = ScanCtl<K>::rm;
    // branch-free: outside my segment the source becomes the identity
    const bool in = scan_src_ok<K>(lane) && scan_src<K>(lane) >= seg0;
    const long long og = dpp64<C, RM>(vg);
    const int oa = dpp32<C, RM>(va);
    vg += in ? og : 0;
    va += in ? oa : 0;
    if (LOCAL) {
        Elem o;
        o.A = dpp64<C, RM>(e.A);
        o.B = dpp64<C, RM>(e.B);
        o.C = dpp64<C, RM>(e.C);
        o.D = dpp64<C, RM>(e.D);
        if (!in) o = {0, kNeg, kNeg, kNeg};
        e = compose(o, e);
    }
}

// The same scan in 32 bits, for tiles whose block scores and gaps are all
// below 2^20 (the common case; the wave picks the path): every tile sum is
// then below 2^27 in magnitude, -inf of the local-score monoid is kNeg32
// and stays below -2^28 however often it is composed inside a tile (it
// drifts by at most the tile's sum of |block - gap|; B + C of two such
// values is still above INT_MIN), so x < kNegThr32 reads as -inf.
struct Elem32 {
    int A, B, C, D;
};
constexpr int kSmallBlk = 1 << 20;
constexpr int kNeg32 = -(1 << 29);
constexpr int kNegThr32 = -(1 << 28);

__device__ __forceinline__ Elem32 compose32(const Elem32 &x, const Elem32 &y) {
    Elem32 r;
    r.A = x.A + y.A;
    r.B = max(x.B + y.A, y.B);
    r.C = max(x.C, x.A + y.C);
    r.D = max(max(x.D, x.B + y.C), y.D);
    return r;
}

__device__ __forceinline__ long long widen_neg(int v) { return v < kNegThr32 ? kNeg : v; }

template <int K, bool LOCAL>
__device__ __forceinline__ void seg_scan_step32(int &vg, int &va, Elem32 &e, int lane, int seg0) {
    constexpr int C = ScanCtl<K>::c, RM = ScanCtl<K>::rm;
    const bool in = scan_src_ok<K>(lane) && scan_src<K>(lane) >= seg0;
    const int og = dpp32<C, RM>(vg);
    const int oa = dpp32<C, RM>(va);
    vg += in ? og : 0;
    va += in ? oa : 0;
    if (LOCAL) {
        Elem32 o;
        o.A = dpp32<C, RM>(e.A);
        o.B = dpp32<C, RM>(e.B);
        o.C = dpp32<C, RM>(e.C);
        o.D = dpp32<C, RM>(e.D);
        if (!in) o = {0, kNeg32, kNeg32, kNeg32};
        e = compose32(o, e);
    }
}

#ifndef GAC_TILE_MINB
#define GAC_TILE_MINB 7  // waves per SIMD the register budget is sized for (r03u: 7 beats 6; 8 spills)
#endif
// Owner of lane-block j of a tile whose candidate ranges rc + k (flat
// offsets L.cg, first window blocks L.cb) are staged: the largest k with
// cg[k] <= j (cg[0] <= the tile's first block), by a 6-step LDS search; past
// 63 range starts in the tile (ranges of one block or empty ones), a binary
// search of the flat offsets beyond.  Returns the range; bi = its block.
__device__ __forceinline__ int tile_owner(const ScoreArgs &a, const WaveLds &L, int j, int rc,
                                          bool active, int n, int &bi) {
    int k = 0;
#pragma unroll
    for (int step = kTileBlocks / 2; step > 0; step >>= 1)
        if (L.cg[k + step] <= j) k += step;
    int ri = rc + k, gr = L.cg[k], b0r = L.cb[k];
    // (keeps these LDS reads: merged with the fallback's global loads they
    // become flat loads, whose vmcnt wait would drain the LDS-DMA in flight)
    asm volatile("" : "+v"(gr), "+v"(b0r));
    if (k == kTileBlocks - 1 && active && ri + 1 < n) {
        int lo = ri, hi = n - 1;  // gflat[lo] <= j
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (a.gflat[mid] <= j) lo = mid;
            else hi = mid - 1;
        }
        ri = lo;
        gr = a.gflat[lo];
        b0r = a.pb0[lo];
    }
    bi = b0r + (j - gr);
    return ri;
}

// Block record bi from the compact copy, as {tStart, qStart, size | N
// flags, gap}; a wide block (rare) reads its 16-B record.
__device__ __forceinline__ int4 load_blk12(const ScoreArgs &a, int bi) {
    if (!a.blk12) return a.blk[bi];  // (A/B probe: GAC_TILE_BLK16=1)
    const Blk12 r = a.blk12[bi];
    const uint32_t sz = r.w & kB12Wide;
    if (sz == (uint32_t)kB12Wide) return a.blk[bi];
    return make_int4(r.t, r.q, (int)(sz | ((r.w >> 1) & (uint32_t)(kTHasN | kQHasN))),
                     (int)((r.w >> 12) & (uint32_t)kB12GapMax));
}

// Per-lane block of the tile: clip to [s, e), gap to the next block, plane
// positions (see WaveLds).
struct LaneBlock {
    int len, g, lenq;
    bool first, last;
    long long tpos, qpos;
};

__device__ __forceinline__ LaneBlock lane_block(const RangeDesc &d, const int4 bk, int bi) {
    LaneBlock r;
    r.first = (bi == d.b0);
    r.last = (bi == d.b0 + d.nblk - 1);
    const int z = bk.z & kSizeMask;
    int cts = bk.x, cqs = bk.y, cte = bk.x + z;
    if (cts < d.s) {
        cqs += d.s - cts;
        cts = d.s;
    }
    if (cte > d.e) cte = d.e;
    r.len = cte - cts;
    r.g = r.last ? 0 : bk.w;
    r.tpos = d.tbase + cts;
    const bool minus = d.qbase < 0;
    r.qpos = minus ? ~d.qbase - cqs : d.qbase + cqs;
    r.lenq = r.len | (minus ? (int)0x80000000 : 0) | (bk.z & (kTHasN | kQHasN));
    return r;
}

// The tile once its lane-blocks are known: 32-base chunks spread over the
// wave (both chunks of a lane loaded together), block sums in LDS, then the
// segmented (by range) scans and the stores / boundary segments.
template <bool LOCAL, bool SYM>
__device__ __forceinline__ void tile_score(const ScoreArgs &a, WaveLds &L, int lane, int tile,
                                           int j, bool active, int W, int ri, const LaneBlock &B,
                                           int /*unused*/) {
    // ---- chunk prefix (32 bases per chunk)
    const int nch = (B.len + 31) >> 5;
    const int incl = wave_incl_sum(nch, lane);
    const int C = __builtin_amdgcn_readlane(incl, kWave - 1);
    L.coff[lane] = incl - nch;
    L.tpos[lane] = B.tpos;
    L.qpos[lane] = B.qpos;
    L.lenq[lane] = B.lenq;
    L.acc[lane] = 0ull;
    wave_sync_lds();

    for (int c0 = 0; c0 < C; c0 += 2 * kWave) {
        const ChunkRef ca = chunk_prep(L, c0 + lane);
        const ChunkRef cb = chunk_prep(L, c0 + kWave + lane);
        const ChunkRaw ra = chunk_load(a, ca);
        const ChunkRaw rb = chunk_load(a, cb);
        const int sa = chunk_eval<SYM>(a, ca, ra);
        const int sb = chunk_eval<SYM>(a, cb, rb);
        if (chunk_n(ca) > 0) atomicAdd(&L.acc[chunk_k(ca)], (unsigned long long)(long long)sa);
        if (chunk_n(cb) > 0) atomicAdd(&L.acc[chunk_k(cb)], (unsigned long long)(long long)sb);
    }
    wave_sync_lds();

    // ---- segmented (by range) inclusive scans over the tile's lanes
    const long long bsc = active ? (long long)L.acc[lane] : 0;
    const bool head = !active || lane == 0 || B.first;
    const unsigned long long heads = __ballot(head);
    // my segment's first lane (lanes <= me: computed here, not held across the tile)
    const int seg0 = 63 - __builtin_clzll(heads & (~0ull >> (63 - lane)));
    int va = active ? B.len : 0;
    long long vg;
    Elem e;
    const bool small = !active || (bsc > -kSmallBlk && bsc < kSmallBlk && B.g < kSmallBlk);
    if (!a.scan64 && __ballot(!small) == 0ull) {  // 32-bit scans
        const int b32 = (int)bsc;
        int v = active ? b32 - B.g : 0;
        Elem32 e32;
        if (LOCAL) {
            if (active) {
                e32.A = B.last ? b32 : b32 - B.g;
                e32.B = B.last ? kNeg32 : 0;
                e32.C = b32;
                e32.D = kNeg32;
            } else {
                e32 = {0, kNeg32, kNeg32, kNeg32};
            }
        }
        seg_scan_step32<0, LOCAL>(v, va, e32, lane, seg0);
        seg_scan_step32<1, LOCAL>(v, va, e32, lane, seg0);
        seg_scan_step32<2, LOCAL>(v, va, e32, lane, seg0);
        seg_scan_step32<3, LOCAL>(v, va, e32, lane, seg0);
        seg_scan_step32<4, LOCAL>(v, va, e32, lane, seg0);
        seg_scan_step32<5, LOCAL>(v, va, e32, lane, seg0);
        vg = v;
        if (LOCAL) {
            e.A = e32.A;
            e.B = widen_neg(e32.B);
            e.C = widen_neg(e32.C);
            e.D = widen_neg(e32.D);
        }
    } else {  // 64-bit scans (a block score or gap of 2^20 or more)
        vg = active ? bsc - B.g : 0;
        if (LOCAL) {
            if (active) {
                e.A = B.last ? bsc : bsc - B.g;
                e.B = B.last ? kNeg : 0;
                e.C = bsc;
                e.D = kNeg;
            } else {
                e = {0, kNeg, kNeg, kNeg};
            }
        }
        seg_scan_step<0, LOCAL>(vg, va, e, lane, seg0);
        seg_scan_step<1, LOCAL>(vg, va, e, lane, seg0);
        seg_scan_step<2, LOCAL>(vg, va, e, lane, seg0);
        seg_scan_step<3, LOCAL>(vg, va, e, lane, seg0);
        seg_scan_step<4, LOCAL>(vg, va, e, lane, seg0);
        seg_scan_step<5, LOCAL>(vg, va, e, lane, seg0);
    }
    const bool seg_end = active && (lane == kWave - 1 || ((heads >> (lane + 1)) & 1ull));
    const bool first0 = __builtin_amdgcn_readfirstlane(B.first ? 1 : 0) != 0;
    if (seg_end) {
        const bool has0 = (seg0 == 0);
        const bool starts = !has0 || first0;
        if (starts && B.last) {
            seg_store<LOCAL>(a, ri, vg, va, e);
        } else {
            SegSum ssum;
            ssum.g = vg;
            ssum.ali = va;
            if (LOCAL) {
                ssum.A = e.A;
                ssum.B = e.B;
                ssum.C = e.C;
                ssum.D = e.D;
            }
            if (has0 && !starts) a.sum_head[tile] = ssum;
            if (!B.last && (lane == kWave - 1 || j + 1 == W)) a.sum_tail[tile] = ssum;
        }
    }
    wave_sync_lds();
}

template <bool LOCAL, bool SYM>
__global__ void __launch_bounds__(256, SYM ? GAC_TILE_MINB : 6) k_tile(ScoreArgs a) {
    __shared__ WaveLds s_w[kWavesPerWG];

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    WaveLds &L = s_w[wave];
    if (a.status[2]) return;  // workspace overflow: the host grows it and reruns
    const int T = a.status[1];
    const int W = a.status[0];

    // XCD-aware logical id: workgroups b and b+8 share an XCD (round-robin
    // dispatch), so give them adjacent tiles (speed only).
    const int G = gridDim.x;
    const int b = blockIdx.x;
    const int L8 = (G % 8 == 0) ? ((b % 8) * (G / 8) + b / 8) : b;
    int stride = G * kWavesPerWG, tend = T;

    // The tile's blocks belong to the ranges r0 .. r1 (r0 = tile_r0[t], r1 =
    // tile_r0[t + 1], the owner of the next tile's first block).  During tile
    // t the wave loads r0, r1 of its next tile t' (at the top; they land
    // with t's descriptors and blocks) and then, once t's blocks are in,
    // the flat offsets / first blocks of exactly t''s candidates r0 .. r1
    // (their lines only, not those of 64 ranges), consumed at the top of t'
    // from LDS by a 6-step owner search.  (Whole-chain plans in set order
    // have pb0 == gflat: one load.)
    // lt: the wave's place in the schedule; the tile it scores is lt itself,
    // or a.tile_perm[lt] (whole chains: tiles in the target order of their
    // first blocks, so the tiles an XCD holds at once read neighbouring
    // target lines -- each tile's partial sums still go to its own slot, and
    // the fold combines them in tile order)
    int lt = L8 * kWavesPerWG + wave;
    if (a.xcd_chunk && G % 8 == 0) {  // (probe) XCD x: tiles [x C, (x + 1) C)
        const int C = (T + 7) / 8;
        lt = (b % 8) * C + (b / 8) * kWavesPerWG + wave;
        stride = (G / 8) * kWavesPerWG;
        tend = T < (b % 8 + 1) * C ? T : (b % 8 + 1) * C;
    }
    const int32_t *perm = a.tile_perm;
    const auto tile_at = [&](int x) { return perm ? perm[x] : x; };
    const int n = (int)a.n;
    const bool same_pb = a.pb0 == a.gflat;
    const auto cand_end = [&](int t) { return t + 1 < T ? a.tile_r0[t + 1] : n - 1; };
    int r0 = 0, gv = 0x7fffffff, bv = 0;
    int tile = lt < tend ? tile_at(lt) : 0;
    if (lt < tend) {
        r0 = a.tile_r0[tile];
        const int r1 = cand_end(tile);
        if (r0 + lane <= r1 && r0 + lane < n) {
            gv = a.gflat[r0 + lane];
            bv = same_pb ? gv : a.pb0[r0 + lane];
        }
    }
    for (; lt < tend; lt += stride) {
        const int j = tile * kTileBlocks + lane;
        const bool active = j < W;
        L.cg[lane] = gv;
        L.cb[lane] = bv;
        const int rc = r0;
        const int ltn = lt + stride;
        const int tn = ltn < tend ? tile_at(ltn) : 0;
        int r0n = 0, r1n = 0;
        if (ltn < tend) {
            r0n = a.tile_r0[tn];
            r1n = cand_end(tn);
        }
        wave_sync_lds();
        int bi;
        const int ri = tile_owner(a, L, j, rc, active, n, bi);
        LaneBlock B = {0, 0, 0, false, false, 0, 0};
        if (active) B = lane_block(a.rdesc[ri], load_blk12(a, bi), bi);
        gv = 0x7fffffff;
        bv = 0;
        if (ltn < tend && r0n + lane <= r1n && r0n + lane < n) {
            gv = a.gflat[r0n + lane];
            bv = same_pb ? gv : a.pb0[r0n + lane];
        }
        r0 = r0n;
        tile_score<LOCAL, SYM>(a, L, lane, tile, j, active, W, ri, B, 0);
        tile = tn;
    }
}

// k_tile with the descriptor/block round trip of tile t + 1 overlapped with
// the plane loads of tile t: the next tile's owners are found while tile t
// is prepared, its RangeDesc halves and block records go to LDS by LDS-DMA
// (global_load_lds, no registers held), issued before t's plane loads, so
// the wave waits for one round trip per tile instead of two.  The candidate
// ranges' offsets are loaded two tiles ahead, tile_r0 three.
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;

struct WaveNext {
    int4 rd_lo[kTileBlocks];  // RangeDesc {tbase, qbase} of each lane's owner, next tile
    int4 rd_hi[kTileBlocks];  // RangeDesc {b0, nblk, s, e}
    int4 bk[kTileBlocks];     // block record
    int ri[kTileBlocks];      // owner range
    int bi[kTileBlocks];      // block index
    int r0;                   // tile_r0 of the tile after next (LDS-DMA, lane 0)
    int pad[3];
};

__device__ __forceinline__ void tile_fetch(const ScoreArgs &a, WaveNext &N, int lane, int ri,
                                           int bi, bool active) {
    // inactive lanes fetch a valid record (range 0, block 0) and ignore it
    const RangeDesc *rd = a.rdesc + (active ? ri : 0);
    const int4 *bk = a.blk + (active ? bi : 0);
    N.ri[lane] = ri;
    N.bi[lane] = bi;
    __builtin_amdgcn_global_load_lds((gbl_void *)rd, (lds_void *)N.rd_lo, 16, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void *)((const char *)rd + 16), (lds_void *)N.rd_hi, 16,
                                     0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void *)bk, (lds_void *)N.bk, 16, 0, 0);
}

template <bool LOCAL, bool SYM>
__global__ void __launch_bounds__(256, GAC_TILE_MINB) k_tile_pipe(ScoreArgs a) {
    __shared__ WaveLds s_w[kWavesPerWG];
    __shared__ WaveNext s_n[kWavesPerWG];

    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    WaveLds &L = s_w[wave];
    WaveNext &N = s_n[wave];
    if (a.status[2]) return;  // workspace overflow: the host grows it and reruns
    const int T = a.status[1];
    const int W = a.status[0];
    const int G = gridDim.x;
    const int b = blockIdx.x;
    const int L8 = (G % 8 == 0) ? ((b % 8) * (G / 8) + b / 8) : b;
    const int stride = G * kWavesPerWG;
    const int n = (int)a.n;

    // wave-uniform tile index (scalar loads of tile_r0: their waits are on
    // lgkmcnt, not on the vmcnt the LDS-DMA counts)
    int tile = __builtin_amdgcn_readfirstlane(L8 * kWavesPerWG + wave);
    if (tile >= T) return;
    // prologue: owners of the first tile, its fetch; offsets of the second
    {
        const int r0 = a.tile_r0[tile];
        L.cg[lane] = r0 + lane < n ? a.gflat[r0 + lane] : 0x7fffffff;
        L.cb[lane] = r0 + lane < n ? a.pb0[r0 + lane] : 0;
        wave_sync_lds();
        const int j = tile * kTileBlocks + lane;
        int bi;
        const int ri = tile_owner(a, L, j, r0, j < W, n, bi);
        tile_fetch(a, N, lane, ri, bi, j < W);
    }
    int r1 = tile + stride < T ? a.tile_r0[tile + stride] : 0;  // range r0 of the next tile
    int gv = 0x7fffffff, bv = 0;  // its candidates' offsets
    if (tile + stride < T && r1 + lane < n) {
        gv = a.gflat[r1 + lane];
        bv = a.pb0[r1 + lane];
    }
    // tile_r0 of the tile after next goes to LDS (N.r0) by LDS-DMA: a
    // register copy of a loaded value would make the compiler wait for every
    // load in flight, the LDS-DMA included
    if (tile + 2 * stride < T && lane == 0)
        __builtin_amdgcn_global_load_lds((gbl_void *)(a.tile_r0 + tile + 2 * stride),
                                         (lds_void *)&N.r0, 4, 0, 0);
    for (; tile < T; tile += stride) {
        const int j = tile * kTileBlocks + lane;
        const bool active = j < W;
        // this tile's descriptors and blocks (fetched during the previous tile)
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the LDS-DMA has landed
        wave_sync_lds();
        const int ri = N.ri[lane];
        LaneBlock B = {0, 0, 0, false, false, 0, 0};
        if (active) {
            const int4 lo = N.rd_lo[lane], hi = N.rd_hi[lane];
            RangeDesc d;
            d.tbase = (long long)(((unsigned long long)(uint32_t)lo.y << 32) | (uint32_t)lo.x);
            d.qbase = (long long)(((unsigned long long)(uint32_t)lo.w << 32) | (uint32_t)lo.z);
            d.b0 = hi.x;
            d.nblk = hi.y;
            d.s = hi.z;
            d.e = hi.w;
            B = lane_block(d, N.bk[lane], N.bi[lane]);
        }
        // owners of the next tile, and its fetch (lands while this tile's
        // planes are read)
        const int tn = tile + stride;
        if (tn < T) {
            L.cg[lane] = gv;
            L.cb[lane] = bv;
            wave_sync_lds();
            const int jn = tn * kTileBlocks + lane;
            int bin;
            const int rin = tile_owner(a, L, jn, r1, jn < W, n, bin);
            r1 = tn + stride < T ? N.r0 : 0;
            __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this tile's LDS reads are done
            tile_fetch(a, N, lane, rin, bin, jn < W);
            gv = 0x7fffffff;
            bv = 0;
            if (tn + stride < T && r1 + lane < n) {
                gv = a.gflat[r1 + lane];
                bv = a.pb0[r1 + lane];
            }
            if (tn + 2 * stride < T && lane == 0)
                __builtin_amdgcn_global_load_lds((gbl_void *)(a.tile_r0 + tn + 2 * stride),
                                                 (lds_void *)&N.r0, 4, 0, 0);
        }
        tile_score<LOCAL, SYM>(a, L, lane, tile, j, active, W, ri, B, 0);
    }
}

// ------------------------------------------------------------ cross-tile fold
// Ranges spanning > 1 tile are folded in tile order: the tail segment of the
// range's first tile (sum_tail), then the head segments of the following
// tiles (sum_head).  The work is spread over tiles, not ranges, so that a
// few very long ranges (score-sorted whole chains put them all at the start)
// do not serialise a wave:
//   k_fold_tiles  one wave per super-tile of 64 tiles, lane = tile: the tile's
//                 head segment keyed by its range, a segmented (by range)
//                 wave scan over the super-tile; the last lane of each run
//                 finishes its range when the run holds all of the range's
//                 heads (prefixed with the first tile's tail), else leaves
//                 the run in sup_head (run starting at lane 0) or the range's
//                 prefix in sup_tail (run reaching lane 63);
//   k_fold_super  one lane per super-tile whose tail range continues: that
//                 prefix, then sup_head of every later super-tile the range
//                 reaches (a 1e5-block chain spans ~25).
struct Seg {
    long long g, ali;
    Elem e;
};

template <bool LOCAL>
__device__ __forceinline__ Seg seg_compose(const Seg &x, const Seg &y) {
    Seg r;
    r.g = x.g + y.g;
    r.ali = x.ali + y.ali;
    if (LOCAL) r.e = compose(x.e, y.e);
    return r;
}

__device__ __forceinline__ Seg seg_load(const SegSum &s) {
    Seg r;
    r.g = s.g;
    r.ali = s.ali;
    r.e.A = s.A;
    r.e.B = s.B;
    r.e.C = s.C;
    r.e.D = s.D;
    return r;
}

__device__ __forceinline__ SegSum seg_pack(const Seg &x) {
    SegSum s;
    s.g = x.g;
    s.ali = x.ali;
    s.A = x.e.A;
    s.B = x.e.B;
    s.C = x.e.C;
    s.D = x.e.D;
    return s;
}

template <bool LOCAL>
__global__ void __launch_bounds__(256) k_fold_tiles(ScoreArgs a) {
    if (a.status[2]) return;  // workspace overflow: the host grows it and reruns
    const int T = a.status[1];
    const int64_t U = ((int64_t)T + kWave - 1) / kWave;
    const int lane = threadIdx.x & 63;
    const unsigned long long lanemask_le = (lane == 63) ? ~0ull : ((2ull << lane) - 1ull);
    const int64_t wave_id = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t u = wave_id; u < U; u += nwaves) {
        const int t = (int)(u * kWave) + lane;
        int key = -1, gr = 0;  // key: the range continuing into tile t (-1: none)
        if (t < T) {
            const int r = a.tile_r0[t];
            gr = a.gflat[r];
            if ((long long)gr < (long long)t * kTileBlocks) key = r;
        }
        Seg v;
        if (key >= 0) {
            v = seg_load(a.sum_head[t]);
        } else {
            v.g = v.ali = 0;
            v.e = {0, kNeg, kNeg, kNeg};
        }
        const int prev = __shfl_up(key, 1, kWave);
        const bool head = lane == 0 || key < 0 || key != prev;
        const unsigned long long heads = __ballot(head);
        const int seg0 = 63 - __builtin_clzll(heads & lanemask_le);
#pragma unroll
        for (int d = 1; d < kWave; d <<= 1) {
            Seg o;
            o.g = __shfl_up(v.g, d, kWave);
            o.ali = __shfl_up(v.ali, d, kWave);
            if (LOCAL) {
                o.e.A = __shfl_up(v.e.A, d, kWave);
                o.e.B = __shfl_up(v.e.B, d, kWave);
                o.e.C = __shfl_up(v.e.C, d, kWave);
                o.e.D = __shfl_up(v.e.D, d, kWave);
            }
            if (lane - d >= seg0) v = seg_compose<LOCAL>(o, v);
        }
        const bool run_end = key >= 0 && (lane == 63 || ((heads >> (lane + 1)) & 1ull));
        int tail_r = -1;
        if (run_end) {
            const int nb = a.nblk[key];
            const int tf = gr / kTileBlocks;
            const int tl = (int)(((long long)gr + nb - 1) / kTileBlocks);
            const int ta = (int)(u * kWave) + seg0;
            if (ta == tf + 1) {  // the run holds the range's first heads
                const Seg full = seg_compose<LOCAL>(seg_load(a.sum_tail[tf]), v);
                if (tl == t) {
                    seg_store<LOCAL>(a, key, full.g, (int)full.ali, full.e);
                } else {  // continues past this super-tile (so t is its last tile)
                    a.sup_tail[u] = seg_pack(full);
                    tail_r = key;
                }
            } else {  // begun in an earlier super-tile: the run starts at lane 0
                a.sup_head[u] = seg_pack(v);
            }
        }
        if (lane == 63) a.sup_tail_r[u] = tail_r;
    }
}

template <bool LOCAL>
__global__ void __launch_bounds__(256) k_fold_super(ScoreArgs a) {
    if (a.status[2]) return;
    const int T = a.status[1];
    const int64_t U = ((int64_t)T + kWave - 1) / kWave;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < U; u += stride) {
        const int r = a.sup_tail_r[u];
        if (r < 0) continue;
        Seg acc = seg_load(a.sup_tail[u]);
        const long long gr = a.gflat[r];
        const int64_t ul = ((gr + a.nblk[r] - 1) / kTileBlocks) / kWave;
        for (int64_t w = u + 1; w <= ul; ++w) acc = seg_compose<LOCAL>(acc, seg_load(a.sup_head[w]));
        seg_store<LOCAL>(a, r, acc.g, (int)acc.ali, acc.e);
    }
}

// ------------------------------------------------------------ k_small ----
// Small batches (chainCleaner's on-demand sub-chains): one launch, one wave
// per range, ranges read from and results written to pinned host memory.
// The wave plans the range like k_plan, then walks its window 64 blocks at a
// time (lane = block, the block's 32-base chunks in turn) and folds global,
// aligned bases and the local-score element in block order.  No workspace,
// no scans across workgroups: a call costs one launch.
// HOST: the ranges of chains held in (mapped, pinned) host memory --
// descriptors already planned by the host (b0 = the window's first record in
// `pool`, records {tStart, qStart, size, 0}); the gaps are computed here from
// the next record and every chunk takes the N-mask path (no upload flags).
template <bool LOCAL, bool SYM, bool HOST>
__device__ __forceinline__ void small_range(const ScoreArgs &a, const Range *rin,
                                            const RangeDesc *hin, const int4 *pool, SmallOut *out,
                                            int64_t w, int lane) {
    const RangeDesc d = HOST ? hin[w] : plan_range(a, rin[w]);
    const bool minus = d.qbase < 0;
    long long gsum = 0, asum = 0;
    Elem acc = {0, kNeg, kNeg, kNeg};
    for (int base = 0; base < d.nblk; base += kWave) {
        const int k = base + lane;
        long long vg = 0;
        int va = 0;
        Elem e = {0, kNeg, kNeg, kNeg};
        if (k < d.nblk) {
            // {tStart, qStart, size | N flags, gap to next}
            int4 bk = HOST ? pool[d.b0 + k] : a.blk[d.b0 + k];
            const bool last = (k == d.nblk - 1);
            const int z = bk.z & kSizeMask;
            if (HOST) {
                bk.w = 0;
                if (!last) {
                    const int4 nx = pool[d.b0 + k + 1];
                    int dd;
                    const int which = gap_kind(nx.y - (bk.y + z), nx.x - (bk.x + z), dd);
                    bk.w = dd < a.gap_len ? a.gap_tab[which * a.gap_len + dd]
                                          : gap_cost_wd(a.gap, a.small_tab, which, dd);
                }
                bk.z = z | kTHasN | kQHasN;
            }
            int cts = bk.x, cqs = bk.y, cte = bk.x + z;
            if (cts < d.s) {
                cqs += d.s - cts;
                cts = d.s;
            }
            if (cte > d.e) cte = d.e;
            const int len = cte - cts;
            const int64_t tpos = d.tbase + cts;
            const int64_t qpos = minus ? ~d.qbase - cqs : d.qbase + cqs;
            const int lq = len | (minus ? (int)0x80000000 : 0) | (bk.z & (kTHasN | kQHasN));
            long long bsc = 0;
            for (int off = 0; off < len; off += 32) {
                const int cn = min(32, len - off);
                const ChunkRef c =
                    make_chunk(tpos + off, minus ? qpos - off - cn : qpos + off, cn, lq, 0);
                bsc += chunk_eval<SYM>(a, c, chunk_load(a, c));
            }
            const int g = last ? 0 : bk.w;
            vg = bsc - g;
            va = len;
            if (LOCAL) {
                e.A = last ? bsc : bsc - g;
                e.B = last ? kNeg : 0;
                e.C = bsc;
            }
        }
        gsum += wave_sum(vg);
        asum += wave_sum(va);
        if (LOCAL) acc = compose(acc, wave_fold(e, lane));  // lane 0 holds the fold
    }
    if (lane == 0) {
        SmallOut o;
        o.g = gsum;
        o.l = LOCAL ? max2(0, max2(acc.C, acc.D)) : 0;
        o.ali = (int32_t)asum;
        o.pad = 0;
        out[w] = o;
    }
}

template <bool LOCAL, bool SYM, bool HOST>
__global__ void __launch_bounds__(256) k_small(ScoreArgs a, const Range *rin, const RangeDesc *hin,
                                               const int4 *pool, SmallOut *out) {
    const int lane = threadIdx.x & 63;
    const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (w >= a.n) return;
    small_range<LOCAL, SYM, HOST>(a, rin, hin, pool, out, w, lane);
}

// ------------------------------------------------------ k_small_server ----
// The small batches of a long run of on-demand calls (chainCleaner's replay
// loop) without a launch per call: a resident grid of kSrvWaves waves takes
// requests from a mailbox in pinned, coherent host memory (SmallMail).  One
// lane of workgroup 0 polls the mailbox's request word (number, kind and
// range count in 32 bits: srv_word; relaxed system-scope loads, s_sleep
// between polls) and copies it to uncached device memory (SmallSync: the
// XCDs' L2s are not coherent with each other, so a cached word could stay
// stale in another XCD's L2); one lane of every other workgroup polls that copy
// (relaxed, then one acquire fence) while its waves wait at a barrier.  Wave
// w scores ranges w, w + kSrvWaves, ... (k_small's body; the kind selects the
// uploaded set's ranges or host-planned descriptors).  A workgroup that wrote
// results makes them visible to the host (one system-scope release) before
// it counts itself in SmallSync.cnt; the last workgroup publishes the
// request word in mail->done.  Measured (GAC_SRV_TRACE, r05lat2/5): every
// workgroup reading the mailbox's kind and count from host memory cost ~38
// us per request, one reader ~1.8 us; polling with acquire loads (a cache
// invalidation per poll) or a cached copy was slower still.  (A 64-bit
// request word hung the grid in r05lat3/4; the 32-bit words are what was
// measured to work.)  Every wave reaches the exit: workgroup
// 0 broadcasts kSrvExit when the host sets mail->stop or no request arrives
// within `idle` ticks of the 100 MHz real-time counter, then marks the
// mailbox exited (state 2); the host re-launches the grid for a request that
// finds it gone.
constexpr uint32_t kSrvExit = 0xffffffffu;

__device__ __forceinline__ uint32_t sys_relaxed(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

template <bool LOCAL, bool SYM>
__global__ void __launch_bounds__(256) k_small_server(ScoreArgs a0, ScoreArgs a1, const Range *rin,
                                                      const RangeDesc *hin, const int4 *pool,
                                                      SmallOut *out, SmallMail *mail,
                                                      SmallSync *sy, uint32_t last_done,
                                                      uint64_t idle, uint32_t trace) {
    __shared__ uint32_t s_req[3];
    const int lane = threadIdx.x & 63;
    const int wave = (int)(blockIdx.x * kWavesPerWG + (threadIdx.x >> 6));
    const int nw = (int)(gridDim.x * kWavesPerWG);
    uint32_t cur = last_done;
    for (;;) {
        if (threadIdx.x == 0) {
            uint32_t s, kind = 0, n = 0;
            if (blockIdx.x == 0) {
                const uint64_t t0 = wall_clock64();
                uint32_t polls = 0;
                for (;;) {
                    ++polls;
                    const uint32_t r = sys_relaxed(&mail->req);
                    if (sys_relaxed(&mail->stop)) {
                        s = kSrvExit;
                        break;
                    }
                    if (r != cur) {
                        s = r;
                        break;
                    }
                    if (wall_clock64() - t0 > (long long)idle) {
                        s = kSrvExit;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                if (trace) {  // (GAC_SRV_TRACE: 10-ns ticks of the request's phases)
                    sy->pad[0] = (uint32_t)wall_clock64();
                    sy->pad[6] = polls;
                }
                __hip_atomic_store(&sy->seq, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
                if (trace) sy->pad[1] = (uint32_t)wall_clock64();
            } else {
                for (;;) {  // (0: the launch's zeroed word, never a request word)
                    s = __hip_atomic_load(&sy->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (s != cur && s != 0) break;
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // (inputs in host memory)
            }
            if (s != kSrvExit) {
                kind = (s >> 29) & 1u;
                n = (s >> 20) & 0x1ffu;
            }
            s_req[0] = s;
            s_req[1] = kind;
            s_req[2] = n;
        }
        __syncthreads();
        const uint32_t s = s_req[0], kind = s_req[1], n = s_req[2];
        if (s == kSrvExit) break;
        if (trace && threadIdx.x == 0)
            atomicMax(&sy->pad[2], (uint32_t)wall_clock64() - sy->pad[0]);
        for (int64_t w = wave; w < (int64_t)n; w += nw) {
            if (kind) small_range<LOCAL, SYM, true>(a1, nullptr, hin, pool, out, w, lane);
            else small_range<LOCAL, SYM, false>(a0, rin, nullptr, nullptr, out, w, lane);
        }
        __syncthreads();  // (the workgroup's results are stored; s_req may be rewritten)
        if (threadIdx.x == 0) {
            if (trace) atomicMax(&sy->pad[4], (uint32_t)wall_clock64() - sy->pad[0]);
            if ((int64_t)blockIdx.x * kWavesPerWG < (int64_t)n)
                __threadfence_system();  // its results, before it is counted
            if (trace) atomicMax(&sy->pad[5], (uint32_t)wall_clock64() - sy->pad[0]);
            const uint32_t old =
                __hip_atomic_fetch_add(&sy->cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == gridDim.x - 1) {  // the last workgroup: reset the count, publish
                __hip_atomic_store(&sy->cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&mail->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (trace) {  // per-request sums of the phase ends, then reset
                    const uint32_t t = (uint32_t)wall_clock64() - sy->pad[0];
                    atomicAdd(&sy->pad[8], sy->pad[1] - sy->pad[0]);
                    atomicAdd(&sy->pad[9], sy->pad[2]);
                    atomicAdd(&sy->pad[11], sy->pad[4]);
                    atomicAdd(&sy->pad[12], sy->pad[5]);
                    atomicAdd(&sy->pad[13], t);
                    atomicAdd(&sy->pad[14], sy->pad[6]);
                    atomicAdd(&sy->pad[15], 1u);
                    sy->pad[2] = sy->pad[4] = sy->pad[5] = 0;
                }
            }
        }
        cur = s;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(&mail->state, 2u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------ genome -----
// Raw .2bit payload (2 bits/base, MSB first in each byte) -> bit planes.
struct SeqDev {
    int64_t byte_off;  // into staging
    int64_t word_off;  // into planes
    int32_t size;
    int32_t pad;
};

// 32 codes of 2 bits, MSB first in each byte (8 payload bytes, loaded as one
// little-endian u64: base 4j + k at bits 8j + 6 - 2k (low bit of the code)
// and 8j + 7 - 2k (high bit)) -> the low-bit and high-bit planes, base i at
// bit i: gather every other bit, then reverse each nibble
__device__ __forceinline__ uint32_t even_bits(uint64_t x) {
    x &= 0x5555555555555555ull;
    x = (x | (x >> 1)) & 0x3333333333333333ull;
    x = (x | (x >> 2)) & 0x0f0f0f0f0f0f0f0full;
    x = (x | (x >> 4)) & 0x00ff00ff00ff00ffull;
    x = (x | (x >> 8)) & 0x0000ffff0000ffffull;
    x = (x | (x >> 16)) & 0x00000000ffffffffull;
    return (uint32_t)x;
}
__device__ __forceinline__ uint32_t rev_nibbles(uint32_t v) {
    v = ((v >> 1) & 0x55555555u) | ((v & 0x55555555u) << 1);
    return ((v >> 2) & 0x33333333u) | ((v & 0x33333333u) << 2);
}

// Two plane words per lane: one 16-byte load of the payload (every sequence
// starts 8-byte aligned in the staging buffer, which is padded past its end),
// one 16-byte plane store and one 8-byte N-mask store (round 4's lane per
// word issued 8-byte accesses).  A workgroup takes kRelPer runs of 512
// words: the sequence search (a chain of dependent scalar loads) is paid once
// per workgroup.  A lane whose two words straddle a sequence start (rare)
// builds each word from its own sequence.
constexpr int kRelPer = 4;
__device__ __forceinline__ int relayout_seq(const SeqDev *seqs, int nseq, int l, int64_t w) {
    while (l + 1 < nseq && seqs[l + 1].word_off <= w) ++l;
    return l;
}

__device__ __forceinline__ void relayout_word(const uint8_t *raw, const SeqDev &s, int64_t w,
                                              uint32_t &p0, uint32_t &p1, uint32_t &pad) {
    const int64_t base0 = (w - s.word_off) * 32;
    const uint64_t x = *reinterpret_cast<const uint64_t *>(raw + s.byte_off + (base0 >> 2));
    const int64_t valid = s.size - base0;  // > 0
    pad = valid >= 32 ? 0u : ~((1u << valid) - 1u);  // padding scores 0 like an N
    p0 = rev_nibbles(even_bits(x)) & ~pad;
    p1 = rev_nibbles(even_bits(x >> 1)) & ~pad;
}

__global__ void __launch_bounds__(256) k_relayout(const uint8_t *raw, const SeqDev *seqs,
                                                  int nseq, int64_t nwords, uint2 *planes,
                                                  uint32_t *nmask) {
    const int64_t W0 = (int64_t)blockIdx.x * blockDim.x * 2 * kRelPer;
    int lo = 0, hi = nseq - 1;
    while (lo < hi) {  // last seq with word_off <= W0
        const int mid = (lo + hi + 1) >> 1;
        if (seqs[mid].word_off <= W0) lo = mid;
        else hi = mid - 1;
    }
    for (int r = 0; r < kRelPer; ++r) {
        const int64_t w0 = W0 + r * 2 * (int64_t)blockDim.x, w = w0 + 2 * threadIdx.x;
        if (w0 >= nwords) return;
        while (lo + 1 < nseq && seqs[lo + 1].word_off <= w0) ++lo;  // (uniform)
        if (w >= nwords) return;
        const int l0 = relayout_seq(seqs, nseq, lo, w);
        const SeqDev s = seqs[l0];
        uint32_t a0, a1, ap, b0 = 0, b1 = 0, bp = 0xffffffffu;
        const bool two = w + 1 < nwords;
        if (two && (l0 + 1 >= nseq || seqs[l0 + 1].word_off > w + 1) &&
            (w + 1 - s.word_off) * 32 < s.size) {  // both words in this sequence
            const int64_t base0 = (w - s.word_off) * 32;
            const u32x4a8 x = *reinterpret_cast<const u32x4a8 *>(raw + s.byte_off + (base0 >> 2));
            const uint64_t x0 = (uint64_t)x.x | ((uint64_t)x.y << 32);
            const uint64_t x1 = (uint64_t)x.z | ((uint64_t)x.w << 32);
            const int64_t valid = s.size - base0 - 32;  // of the second word, > 0
            bp = valid >= 32 ? 0u : ~((1u << valid) - 1u);
            ap = 0;
            a0 = rev_nibbles(even_bits(x0));
            a1 = rev_nibbles(even_bits(x0 >> 1));
            b0 = rev_nibbles(even_bits(x1)) & ~bp;
            b1 = rev_nibbles(even_bits(x1 >> 1)) & ~bp;
        } else {
            relayout_word(raw, s, w, a0, a1, ap);
            if (two) relayout_word(raw, seqs[relayout_seq(seqs, nseq, l0, w + 1)], w + 1, b0, b1, bp);
        }
        if (two) {
            *reinterpret_cast<uint4 *>(planes + w) = make_uint4(a0, a1, b0, b1);
            *reinterpret_cast<uint2 *>(nmask + w) = make_uint2(ap, bp);
        } else {
            planes[w] = make_uint2(a0, a1);
            nmask[w] = ap;
        }
    }
}

// N runs, pre-split on the host into pieces of <= 1024 bases.
struct NPiece {
    int64_t bit0;  // global base index (word_off*32 + start)
    int32_t len;
    int32_t pad;
};

__global__ void __launch_bounds__(256) k_nruns(const NPiece *pieces, int64_t n, uint32_t *nmask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const NPiece p = pieces[i];
    int64_t b = p.bit0;
    const int64_t e = p.bit0 + p.len;
    while (b < e) {
        const int64_t w = b >> 5;
        const int lo = (int)(b & 31);
        const int64_t wend = (w + 1) << 5;
        const int hi = (int)((e < wend ? e : wend) - (w << 5));  // exclusive bit
        const uint32_t m = (hi >= 32 ? 0xffffffffu : ((1u << hi) - 1u)) & ~((1u << lo) - 1u);
        atomicOr(&nmask[w], m);
        b = w * 32 + hi;
    }
}

// ------------------------------------------------------------ text blocks
// The kent in-process API scores caller-owned char text (chainScoreBlock,
// axtScoreUngapped, cBlockFindCrossover: kent/src/lib/chainConnect.c:14-22,
// 61-105, axt.c:186-194).  Text codes: a/A 0, c/C 1, g/G 2, t/T 3, anything
// else 4, scored 0 (the kent matrices are zero outside acgt/ACGT --
// propagateCase, axt.c:402-421; gac_kent checks it).  m25[q * 5 + t].
__device__ __forceinline__ int text_code(uint8_t ch) {
    const int c = ch | 0x20;
    return c == 'a' ? 0 : c == 'c' ? 1 : c == 'g' ? 2 : c == 't' ? 3 : 4;
}

__global__ void __launch_bounds__(256) k_text_blocks(const uint8_t *text, const TextJob *jobs,
                                                     int64_t n, M25 m, long long *out) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_id = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t j = wave_id; j < n; j += nwaves) {
        const TextJob J = jobs[j];
        long long s = 0;
        for (int k = lane; k < J.n; k += kWave)
            s += m.m[text_code(text[J.q + k]) * 5 + text_code(text[J.t + k])];
        s = wave_sum(s);
        if (lane == 0) out[j] = s;
    }
}

// cBlockFindCrossover on text: d_k = left_k - right_k; the crossover is the
// first k where D_k = d_0 + .. + d_k reaches its maximum, if that maximum is
// > 0 (strict improvements over the right block's score): pos = k + 1,
// adj = lScore - max(0, max D).
__global__ void __launch_bounds__(256) k_text_xover(const uint8_t *text, const TextXJob *jobs,
                                                    int64_t n, M25 m, int32_t *out_pos,
                                                    int32_t *out_adj) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_id = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t j = wave_id; j < n; j += nwaves) {
        const TextXJob J = jobs[j];
        long long carry = 0, lsum = 0, bestv = 0;
        int bestpos = 0;
        for (int base = 0; base < J.ov; base += kWave) {
            const int k = base + lane;
            long long d = 0, l = 0;
            if (k < J.ov) {
                l = m.m[text_code(text[J.lq + k]) * 5 + text_code(text[J.lt + k])];
                d = l - m.m[text_code(text[J.rq + k]) * 5 + text_code(text[J.rt + k])];
            }
            long long incl = d;
#pragma unroll
            for (int s = 1; s < kWave; s <<= 1) {
                const long long o = __shfl_up(incl, s, kWave);
                if (lane >= s) incl += o;
            }
            incl += carry;
            long long mx = k < J.ov ? incl : kNeg;
#pragma unroll
            for (int s = 32; s > 0; s >>= 1) mx = max2(mx, __shfl_xor(mx, s, kWave));
            if (mx > bestv) {
                const unsigned long long hit = __ballot(k < J.ov && incl == mx);
                bestv = mx;
                bestpos = base + __builtin_ctzll(hit) + 1;
            }
            carry = __shfl(incl, kWave - 1, kWave);
            lsum += wave_sum(l);
        }
        if (lane == 0) {
            out_pos[j] = bestpos;
            out_adj[j] = (int32_t)(lsum - bestv);
        }
    }
}

}  // namespace gac

// ---------------------------------------------------------------- launch --
namespace gac {

int plan_grid(int64_t n) { return (int)((n + kPlanWG - 1) / kPlanWG); }

hipError_t launch_plan(const ScoreArgs &a, hipStream_t s) {
    if (a.wins)
        hipLaunchKernelGGL(k_plan<true>, dim3((unsigned)plan_grid(a.n)), dim3(kPlanWG), 0, s, a);
    else
        hipLaunchKernelGGL(k_plan<false>, dim3((unsigned)plan_grid(a.n)), dim3(kPlanWG), 0, s, a);
    return hipGetLastError();
}

// GAC_PLAN_LB=1: the single-pass k_plan_lb instead of k_plan + the tile map
// (opt-in: see DESIGN 4.4 for its A/Bs)
// (read per call, like GAC_UNFUSED_MAP: the tests switch paths in one process)
bool plan_lb() {
    const char *e = getenv("GAC_PLAN_LB");
    return e && e[0] == '1';
}

hipError_t launch_plan_lb(const ScoreArgs &a, hipStream_t s) {
    if (a.wins)
        hipLaunchKernelGGL(k_plan_lb<true>, dim3((unsigned)plan_lb_grid(a.n)), dim3(kPlanWG), 0, s, a);
    else
        hipLaunchKernelGGL(k_plan_lb<false>, dim3((unsigned)plan_lb_grid(a.n)), dim3(kPlanWG), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_tilemap(const ScoreArgs &a, hipStream_t s) {
    const int G = plan_grid(a.n);
    if (G <= kFusedMapWG && !getenv("GAC_UNFUSED_MAP")) {
        hipLaunchKernelGGL(k_tilemap_fused, dim3((unsigned)G), dim3(kPlanWG), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_scan_agg, dim3(1), dim3(kPlanWG), 0, s, a);
        hipLaunchKernelGGL(k_tilemap, dim3((unsigned)G), dim3(kPlanWG), 0, s, a);
    }
    return hipGetLastError();
}


// GAC_TILE_PIPE=1: k_tile_pipe (one round trip per tile) instead of k_tile
// (r03n, C5: fills 1.12 vs 1.06 ms, whole chains 2.24 vs 2.25 ms -- opt-in)
static bool tile_pipe() {
    static const bool on = [] {
        const char *e = getenv("GAC_TILE_PIPE");
        return e && e[0] == '1';
    }();
    return on;
}

hipError_t launch_tile(const ScoreArgs &a, int grid, hipStream_t s) {
    if (tile_pipe()) {
        if (a.want_local) {
            if (a.sym) k_tile_pipe<true, true><<<grid, 256, 0, s>>>(a);
            else k_tile_pipe<true, false><<<grid, 256, 0, s>>>(a);
        } else {
            if (a.sym) k_tile_pipe<false, true><<<grid, 256, 0, s>>>(a);
            else k_tile_pipe<false, false><<<grid, 256, 0, s>>>(a);
        }
    } else if (a.want_local) {
        if (a.sym) k_tile<true, true><<<grid, 256, 0, s>>>(a);
        else k_tile<true, false><<<grid, 256, 0, s>>>(a);
    } else {
        if (a.sym) k_tile<false, true><<<grid, 256, 0, s>>>(a);
        else k_tile<false, false><<<grid, 256, 0, s>>>(a);
    }
    return hipGetLastError();
}

// Resident workgroups per CU of the persistent kernels (a grid must not
// exceed what fits at once, or the last workgroups run as a second wave):
// which = 0 k_tile<false, *>, 1 = k_tile<true, *>; sym = the strand-symmetric
// variant (register budgets differ: 7 vs 6 waves per SIMD).
int persistent_blocks_per_cu(int which, int sym) {
    int nb = 0;
    const bool pipe = tile_pipe();
    hipError_t e;
    if (pipe)
        e = which == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_pipe<false, false>, 256, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile_pipe<true, false>, 256, 0);
    else if (sym)
        e = which == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile<false, true>, 256, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile<true, true>, 256, 0);
    else
        e = which == 0 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile<false, false>, 256, 0)
                       : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_tile<true, false>, 256, 0);
    return (e == hipSuccess && nb > 0) ? nb : 4;
}

template <bool HOST>
static void launch_small_t(const ScoreArgs &a, const Range *rin, const RangeDesc *hin,
                           const int4 *pool, SmallOut *out, hipStream_t s) {
    const dim3 g((unsigned)((a.n + kWavesPerWG - 1) / kWavesPerWG)), b(256);
    if (a.want_local) {
        if (a.sym) k_small<true, true, HOST><<<g, b, 0, s>>>(a, rin, hin, pool, out);
        else k_small<true, false, HOST><<<g, b, 0, s>>>(a, rin, hin, pool, out);
    } else {
        if (a.sym) k_small<false, true, HOST><<<g, b, 0, s>>>(a, rin, hin, pool, out);
        else k_small<false, false, HOST><<<g, b, 0, s>>>(a, rin, hin, pool, out);
    }
}

hipError_t launch_small(const ScoreArgs &a, const Range *rin, SmallOut *out, hipStream_t s) {
    launch_small_t<false>(a, rin, nullptr, nullptr, out, s);
    return hipGetLastError();
}

hipError_t launch_small_host(const ScoreArgs &a, const RangeDesc *hin, const int4 *pool,
                             SmallOut *out, hipStream_t s) {
    launch_small_t<true>(a, nullptr, hin, pool, out, s);
    return hipGetLastError();
}

hipError_t launch_small_server(const ScoreArgs &a0, const ScoreArgs &a1, const Range *rin,
                               const RangeDesc *hin, const int4 *pool, SmallOut *out,
                               SmallMail *mail, SmallSync *sy, uint32_t last_done, uint64_t idle,
                               uint32_t trace, int wgs, hipStream_t s) {
    const dim3 g((unsigned)wgs), b(256);
    if (a0.want_local) {
        if (a0.sym) k_small_server<true, true><<<g, b, 0, s>>>(a0, a1, rin, hin, pool, out, mail, sy, last_done, idle, trace);
        else k_small_server<true, false><<<g, b, 0, s>>>(a0, a1, rin, hin, pool, out, mail, sy, last_done, idle, trace);
    } else {
        if (a0.sym) k_small_server<false, true><<<g, b, 0, s>>>(a0, a1, rin, hin, pool, out, mail, sy, last_done, idle, trace);
        else k_small_server<false, false><<<g, b, 0, s>>>(a0, a1, rin, hin, pool, out, mail, sy, last_done, idle, trace);
    }
    return hipGetLastError();
}

hipError_t launch_combine(const ScoreArgs &a, int grid, hipStream_t s) {
    if (a.want_local) {
        hipLaunchKernelGGL(k_fold_tiles<true>, dim3(grid), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_fold_super<true>, dim3(grid / 8 + 1), dim3(256), 0, s, a);
    } else {
        hipLaunchKernelGGL(k_fold_tiles<false>, dim3(grid), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_fold_super<false>, dim3(grid / 8 + 1), dim3(256), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_whole_plan(const DChain *chains, int64_t n, RangeDesc *rdesc, int32_t *nblk,
                             int32_t *gflat, int32_t *tile_r0, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_whole_plan, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, chains, n,
                       rdesc, nblk, gflat, tile_r0);
    return hipGetLastError();
}

// The target-ordered whole-chain plan (see k_whole_keys): radix sort of
// the chains by target start, scan of the permuted block counts, then the
// plan.  `tmp` / `tmp_bytes`: caller-owned scratch, sized by a first call
// with tmp == nullptr (returns the bytes needed in tmp_bytes).
hipError_t launch_whole_plan_sorted(const DChain *chains, int64_t n, int32_t *perm,
                                    unsigned long long *keys, int32_t *vals, RangeDesc *rdesc,
                                    int32_t *nblk, int32_t *gflat, int32_t *pb0,
                                    int32_t *tile_r0, int32_t *inv, void *tmp,
                                    size_t &tmp_bytes, hipStream_t s) {
    unsigned long long *keys_out = keys + n;
    size_t b_sort = 0, b_scan = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b_sort, keys, keys_out, vals, perm,
                                                      (int)n, 0, kOrderBits, s);
    if (e != hipSuccess) return e;
    e = hipcub::DeviceScan::ExclusiveSum(nullptr, b_scan, nblk, gflat, (int)n, s);
    if (e != hipSuccess) return e;
    const size_t need = std::max(b_sort, b_scan);
    if (!tmp) {
        tmp_bytes = need;
        return hipSuccess;
    }
    if (tmp_bytes < need) return hipErrorInvalidValue;
    if (n == 0) return hipSuccess;
    const dim3 grid((unsigned)((n + 255) / 256));
    hipLaunchKernelGGL(k_whole_keys, grid, dim3(256), 0, s, chains, n, keys, vals);
    e = hipcub::DeviceRadixSort::SortPairs(tmp, b_sort, keys, keys_out, vals, perm, (int)n, 0,
                                           kOrderBits, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_whole_count, grid, dim3(256), 0, s, chains, perm, n, nblk);
    e = hipcub::DeviceScan::ExclusiveSum(tmp, b_scan, nblk, gflat, (int)n, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_whole_plan_sorted, grid, dim3(256), 0, s, chains, perm, n, gflat, rdesc,
                       pb0, tile_r0, inv);
    return hipGetLastError();
}

// tiles of a whole-chain plan (set order) sorted by their first block's
// global target base: perm[T]; tmp == nullptr: tmp_bytes := the scratch size
hipError_t launch_tile_order(const DChain *chains, const int4 *blk, const int32_t *tile_r0,
                             int64_t T, unsigned long long *keys, int32_t *vals, int32_t *perm,
                             void *tmp, size_t &tmp_bytes, hipStream_t s) {
    size_t b_sort = 0;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, b_sort, keys, keys + T, vals, perm,
                                                      (int)T, 0, kOrderBits, s);
    if (e != hipSuccess) return e;
    if (!tmp) {
        tmp_bytes = b_sort;
        return hipSuccess;
    }
    if (tmp_bytes < b_sort) return hipErrorInvalidValue;
    if (T == 0) return hipSuccess;
    hipLaunchKernelGGL(k_tile_keys, dim3((unsigned)((T + 255) / 256)), dim3(256), 0, s, chains,
                       blk, tile_r0, T, keys, vals);
    return hipcub::DeviceRadixSort::SortPairs(tmp, b_sort, keys, keys + T, vals, perm, (int)T, 0,
                                              kOrderBits, s);
}

hipError_t launch_zero_list(const int32_t *list, int64_t n, long long *g, long long *l,
                            int32_t *ali, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_zero_list, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, list, n, g,
                       l, ali);
    return hipGetLastError();
}

hipError_t launch_text_blocks(const uint8_t *text, const TextJob *jobs, int64_t n, const M25 &m,
                              long long *out, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t nb = std::min<int64_t>((n + 3) / 4, 16384);
    hipLaunchKernelGGL(k_text_blocks, dim3((unsigned)nb), dim3(256), 0, s, text, jobs, n, m, out);
    return hipGetLastError();
}

hipError_t launch_text_xover(const uint8_t *text, const TextXJob *jobs, int64_t n, const M25 &m,
                             int32_t *pos, int32_t *adj, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t nb = std::min<int64_t>((n + 3) / 4, 16384);
    hipLaunchKernelGGL(k_text_xover, dim3((unsigned)nb), dim3(256), 0, s, text, jobs, n, m, pos,
                       adj);
    return hipGetLastError();
}

hipError_t launch_gap_table(const GapDev &g, const int32_t *small, int len, int32_t *tab,
                            hipStream_t s) {
    const int64_t nb = (3 * (int64_t)len + 255) / 256;
    hipLaunchKernelGGL(k_gap_table, dim3((unsigned)nb), dim3(256), 0, s, g, small, len, tab);
    return hipGetLastError();
}

// index: also the window-search index (spans, bucket entries and
// terminators); without it launch_build_index builds them later
hipError_t launch_build_flat(const int32_t *bt, const int32_t *bq, const int32_t *bs, int64_t nb,
                             const DChain *chains, int64_t n_chains, int32_t *coff,
                             int32_t *tile_c0, int4 *crun, const longlong2 *t_runs,
                             int64_t n_trun, const longlong2 *q_runs, int64_t n_qrun,
                             const int64_t *q_woff, int4 *blk, int2 *tspan, uint32_t *bucket,
                             const UploadGaps &G, bool index, hipStream_t s) {
    const int64_t ntiles = (nb + 63) >> 6;
    if (n_chains > 0) {
        hipLaunchKernelGGL(k_chain_prep, dim3((unsigned)((n_chains + 255) / 256)), dim3(256), 0, s,
                           chains, n_chains, nb, bq, bs, t_runs, n_trun, q_runs, n_qrun, q_woff,
                           coff, crun, index ? bucket : nullptr);
        hipLaunchKernelGGL(k_tile_chain, dim3((unsigned)((ntiles + 1 + 255) / 256)), dim3(256), 0,
                           s, coff, n_chains, ntiles, tile_c0);
    }
    const int64_t g = (nb + 8 + 256 * kUpPer - 1) / (256 * kUpPer);
    int4 *cr = (n_trun || n_qrun) ? crun : nullptr;
#define GAC_BUILD(GP, MD)                                                                         \
    hipLaunchKernelGGL((k_build_flat<GP, MD>), dim3((unsigned)g), dim3(256), 0, s, bt, bq, bs, nb, \
                       chains, coff, tile_c0, ntiles, cr, t_runs, n_trun, q_runs, n_qrun, q_woff,  \
                       blk, tspan, bucket, G)
    if (G.blk12) {
        if (index) GAC_BUILD(true, 0);
        else GAC_BUILD(true, 1);
    } else {
        if (index) GAC_BUILD(false, 0);
        else GAC_BUILD(false, 1);
    }
#undef GAC_BUILD
    return hipGetLastError();
}

// the window-search index of an uploaded set (coff / tile_c0 / chains as the
// upload left them; bt/bq/bs the staged block arrays)
hipError_t launch_build_index(const int32_t *bt, const int32_t *bq, const int32_t *bs, int64_t nb,
                              const DChain *chains, int64_t n_chains, const int32_t *coff,
                              const int32_t *tile_c0, int2 *tspan, uint32_t *bucket,
                              hipStream_t s) {
    const int64_t ntiles = (nb + 63) >> 6;
    if (n_chains > 0)
        hipLaunchKernelGGL(k_bucket_term, dim3((unsigned)((n_chains + 255) / 256)), dim3(256), 0, s,
                           chains, n_chains, bucket);
    const int64_t g = (nb + 8 + 256 * kUpPer - 1) / (256 * kUpPer);
    hipLaunchKernelGGL((k_build_flat<false, 2>), dim3((unsigned)g), dim3(256), 0, s, bt, bq, bs, nb,
                       chains, coff, tile_c0, ntiles, nullptr, nullptr, 0, nullptr, 0, nullptr,
                       nullptr, tspan, bucket, UploadGaps{});
    return hipGetLastError();
}

hipError_t launch_block_gaps_flat(const int32_t *coff, const int32_t *tile_c0, int64_t nb,
                                  int4 *blk, Blk12 *blk12, const UploadGaps &G, hipStream_t s) {
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_block_gaps_flat, dim3((unsigned)((nb + 256 * kUpPer - 1) / (256 * kUpPer))),
                       dim3(256), 0, s, coff,
                       tile_c0, (nb + 63) >> 6, nb, blk, blk12, G);
    return hipGetLastError();
}

hipError_t launch_relayout(const uint8_t *raw, const SeqDev *seqs, int nseq, int64_t nwords,
                           uint2 *planes, uint32_t *nmask, hipStream_t s) {
    const int64_t nb = (nwords + 512 * kRelPer - 1) / (512 * kRelPer);
    if (nb == 0) return hipSuccess;
    hipLaunchKernelGGL(k_relayout, dim3((unsigned)nb), dim3(256), 0, s, raw, seqs, nseq, nwords,
                       planes, nmask);
    return hipGetLastError();
}

// axtScoreUngapped (kent/src/lib/axt.c:186-194) for a batch of ungapped
// blocks -- axtChain's per-block scores (chainPair, axtChain.c:276-282).  One
// lane per block, 32 bases per step through the same plane windows and
// multilinear matrix basis as k_tile; N positions are subtracted with the N
// masks (matrix entries of N are 0).
__global__ void __launch_bounds__(256) k_blocks(ScoreArgs a, const BlockJob *jobs, int64_t n,
                                                int32_t *out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const BlockJob j = jobs[i];
    int sc = 0;
    for (int off = 0; off < j.n; off += 32) {
        const int m = min(32, j.n - off);
        const int64_t tp = j.tp + off;
        const int64_t qp = j.minus ? j.qp - off - m : j.qp + off;
        uint32_t t0, t1, q0, q1;
        load_planes(a.t_planes, tp, t0, t1);
        load_planes(a.q_planes, qp, q0, q1);
        uint32_t qn = load_nmask(a.q_nmask, qp);
        if (j.minus) {
            const int sh = 32 - m;
            q0 = __builtin_bitreverse32(q0) >> sh;
            q1 = ~(__builtin_bitreverse32(q1) >> sh);
            qn = __builtin_bitreverse32(qn) >> sh;
        }
        const uint32_t v = m >= 32 ? 0xffffffffu : ((1u << m) - 1u);
        const uint32_t d0 = q0 ^ t0, d1 = q1 ^ t1;
        sc += score_bits<false>(a, v, t0, t1, d0, d1);
        const uint32_t nm = (load_nmask(a.t_nmask, tp) | qn) & v;
        if (nm) sc -= score_bits<false>(a, nm, t0, t1, d0, d1);
    }
    out[i] = sc;
}

hipError_t launch_blocks(const ScoreArgs &a, const BlockJob *jobs, int64_t n, int32_t *out,
                         hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t nb = (n + 255) / 256;
    hipLaunchKernelGGL(k_blocks, dim3((unsigned)nb), dim3(256), 0, s, a, jobs, n, out);
    return hipGetLastError();
}

// Sparse genome upload: the payload bytes of the uploaded runs arrive packed
// one after another (8-byte aligned); one wave per run copies them to their
// place in the staging layout (the rest of it is never read: no scored range
// reaches outside the runs).
__global__ void __launch_bounds__(256) k_scatter(const SparseRun *runs, int64_t n,
                                                 const uint64_t *compact, uint64_t *raw) {
    const int lane = threadIdx.x & 63;
    const int64_t wave_id = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t r = wave_id; r < n; r += nwaves) {
        const SparseRun R = runs[r];
        const int64_t words = (R.len + 7) >> 3;
        const uint64_t *src = compact + (R.src >> 3);
        uint64_t *dst = raw + (R.dst >> 3);
        for (int64_t u = lane; u < words; u += kWave) dst[u] = src[u];
    }
}

hipError_t launch_scatter(const SparseRun *runs, int64_t n, const uint64_t *compact,
                          uint64_t *raw, hipStream_t s) {
    if (n == 0) return hipSuccess;
    int64_t nb = (n + 3) / 4;
    if (nb > 16384) nb = 16384;
    hipLaunchKernelGGL(k_scatter, dim3((unsigned)nb), dim3(256), 0, s, runs, n, compact, raw);
    return hipGetLastError();
}

hipError_t launch_nruns(const NPiece *p, int64_t n, uint32_t *nmask, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const int64_t nb = (n + 255) / 256;
    hipLaunchKernelGGL(k_nruns, dim3((unsigned)nb), dim3(256), 0, s, p, n, nmask);
    return hipGetLastError();
}

}  // namespace gac
