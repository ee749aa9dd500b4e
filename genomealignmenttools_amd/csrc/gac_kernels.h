// gac_kernels.h -- device data layout shared by the HIP kernels and the
// C-ABI implementation (gac_device.hip).  gfx950 only.
//
// HBM layout (see DESIGN.md "Data layout in HBM"):
//   genome side (T or Q): 32 bases per "word"
//     planes[w] : uint2 {x = bit0 plane, y = bit1 plane} of 2-bit codes
//                 T=0 C=1 A=2 G=3 (the .2bit code; kent dnautil.h:23-28),
//                 base 32w+i at bit i of each plane
//     nmask[w]  : uint32, bit i set = base 32w+i is N (or padding)
//     every sequence starts on a word boundary; word_off[s] = first word
//   chains: DChain[c] + blocks blk[b] = int4 {tStart, qStart, size | flags, gap}
//     flags (bits 29/30 of .z): the block's target/query bases contain an N
//     (precomputed at upload; blocks without N skip the N-mask loads)
//     gap: gapCalcCost to the chain's next block (k_block_gaps_flat, per scoring
//     setup; 0 after the last block)
#pragma once
#include <stdint.h>

namespace gac {

constexpr int kWave = 64;        // CDNA wavefront
constexpr int kTileBlocks = 64;  // blocks per tile (one per lane)
constexpr int kWavesPerWG = 4;   // 256-thread workgroups
constexpr int kMaxLong = 32;     // long gap positions
constexpr long long kNeg = -(1LL << 61);  // -inf of the local-score monoid
constexpr int kSizeMask = (1 << 29) - 1;  // block size field of blk[].z
constexpr int kTHasN = 1 << 29;           // blk[].z: target bases contain an N
constexpr int kQHasN = 1 << 30;           // blk[].z: query bases contain an N

// Compact copy of the block records for k_tile (12 B instead of 16: fewer
// 128-B lines per scored window), written with the gaps per scoring setup:
// {tStart, qStart, w}, w = size (bits 0-11) | gap (bits 12-29) | tN << 30 |
// qN << 31.  A block of kB12Wide or more bases, or a gap costing 2^18 - 1 or
// more, has size field kB12Wide: k_tile reads its 16-B record instead.
struct Blk12 {
    int32_t t, q;
    uint32_t w;
};
static_assert(sizeof(Blk12) == 12, "Blk12 layout");
constexpr int kB12Wide = 0xFFF;
constexpr int kB12GapMax = (1 << 18) - 1;

struct DChain {
    int64_t blk_off;
    int32_t nblk;
    int32_t t_seq;
    int32_t q_seq;
    int32_t qinfo;     // q_seq size (reverse-complement index base) | strand << 31
    int32_t tstart;    // target span of the blocks
    int32_t tend;
    int64_t idx_off;   // this chain's bucket index in ScoreArgs::bucket
    int32_t shift;     // bucket width = 2^shift target bases
    int32_t pad;
    int64_t tbase;     // global base index of the target sequence start (word_off * 32)
    int64_t qbase;     // '+': global base index of the query sequence start;
                       // '-': ~(word_off * 32 + qSize)  (as RangeDesc::qbase)
};
static_assert(sizeof(DChain) == 64, "DChain layout: one 64-byte record");

// Bucket index of a chain (built at upload): the target span [tstart, tend)
// is cut into nb = ((tend - tstart - 1) >> shift) + 1 buckets of 2^shift
// bases (shift chosen so that nb <= 2 * blocks), and
//   bucket[idx_off + k] = first block with tEnd > tstart + (k << shift),
//   bucket[idx_off + nb] = blocks.
// The first block with tEnd > s then lies in [bucket[k], bucket[k + 1]],
// k = (s - tstart) >> shift: one 8-byte load plus a search of that bracket
// (usually one or two blocks) replaces a log2(blocks) binary search.

struct GapDev {
    int32_t small_size;
    int32_t long_count;
    int32_t last_pos[3];  // q, t, both
    int32_t pad;
    double last_val[3];
    double last_slope[3];
    int32_t long_pos[kMaxLong];
    double long_val[3][kMaxLong];
};

// A scoring setup's gap costs for the upload kernels (k_block_gaps_flat, and
// k_build_flat when the setup precedes the chains): blk12 null = none.
struct UploadGaps {
    Blk12 *blk12;
    GapDev g;
    const int32_t *small, *tab;
    int len;
};

// Per-range descriptor written by k_plan (two 16-B loads in k_tile).
struct RangeDesc {
    int64_t tbase;   // global base index of the target sequence start (word_off * 32)
    int64_t qbase;   // '+': global base index of the query sequence start
                     // '-': ~(word_off * 32 + qSize)  (negative)
    int32_t b0;      // first block of the window (global block index)
    int32_t nblk;    // blocks in the window
    int32_t s, e;    // target clip range
};
static_assert(sizeof(RangeDesc) == 32, "RangeDesc layout");

// Partial result of a range segment inside one tile: additive parts + the
// local-score max-plus element  s_out = max(s_in + A, B); m_out = max(m_in, s_in + C, D)
struct SegSum {
    long long g;    // sum(block) - sum(gap)
    long long ali;  // aligned bases
    long long A, B, C, D;
};

struct Range {
    int32_t chain, t_start, t_end;
};

// A range with its window of blocks known to the caller (gac_window):
// chain-local first block and count (chainSubsetOnT's window of
// [t_start, t_end)).
struct Window {
    int32_t chain, t_start, t_end, first, nblk;
};
static_assert(sizeof(Window) == 20, "Window layout (gac_window)");

// Result of one range of a small batch (k_small writes it straight to pinned
// host memory).
struct SmallOut {
    long long g, l;
    int32_t ali, pad;
};

struct ScoreArgs {
    const uint2 *t_planes;
    const uint32_t *t_nmask;
    const int64_t *t_woff;
    const uint2 *q_planes;
    const uint32_t *q_nmask;
    const int64_t *q_woff;
    const DChain *chains;
    int64_t n_chains;
    const int4 *blk;     // [n_blocks + 8] {tStart, qStart, size | N flags, gap to next}
    const Blk12 *blk12;  // [n_blocks] the same, compact (k_tile)
    const int2 *tspan;   // [n_blocks + 8] {tStart, tEnd} (window searches; padded)
    const uint32_t *bucket;  // chain bucket indexes (see DChain)
    const Range *ranges;
    const Window *wins;  // non-null: the ranges come with their windows (k_plan<true>)
    int64_t n;
    // workspace
    RangeDesc *rdesc;    // [n]
    int32_t *nblk;       // [n]   window blocks per range
    int32_t *goff;       // [n]   exclusive scan of nblk inside the plan workgroup
    int32_t *pb0;        // [n]   first window block (compact copy of rdesc.b0)
    int32_t *gflat;      // [n]   flat offset of each range's first window block
    int32_t *tile_r0;    // [T]   range owning each tile's first flat block
    SegSum *sum_head;    // [T]   partial segment containing the tile's first block
    SegSum *sum_tail;    // [T]   partial segment containing the tile's last block
    // cross-tile fold (k_fold_tiles / k_fold_super), per super-tile of 64 tiles
    SegSum *sup_head;    // [U]   fold of the heads, in super-tile u, of a range begun before it
    SegSum *sup_tail;    // [U]   prefix of the range that continues past super-tile u
    int32_t *sup_tail_r; // [U]   that range, or -1
    int32_t *agg;        // [G]   window blocks of each plan workgroup (k_plan; saturated)
    int32_t *plan_off;   // [G+1] flat offset of plan workgroup w
    unsigned long long *lbflag;  // [G] k_plan_lb's look-back words {value, call tag, state}
    int32_t *status;     // [32]  W (flat blocks, saturated), T (tiles), 1 = workspace too
                         //       small; status[5]: a window lay outside its chain (k_plan<true>,
                         //       published to host_status[3] and cleared); status[8]:
                         //       k_plan_lb's workgroup tickets (re-armed by the last one)
    int32_t *host_status;  // pinned host words: status[0..4) + call_tag (k_scan_agg)
    int32_t call_tag;
    int32_t cap_tiles;   // tile_r0 / sum_head / sum_tail capacity
    // outputs
    long long *out_g;
    long long *out_l;
    int32_t *out_ali;
    int32_t want_local;
    int32_t gap_len;           // gap_tab entries per kind
    const int32_t *gap_tab;    // [3][gap_len] gapCalcCost by kind (q, t, both) and length
    const int32_t *small_tab;  // [3][small_size] q, t, both
    int32_t coef[16];          // score matrix in the multilinear basis of the bits
                               // (t1, t0, d1, d0), d = q ^ t: coef[S], S = t1<<3 |
                               // t0<<2 | d1<<1 | d0 (set bits = factors)
    int32_t sym;               // matrix is strand-symmetric: coef[8..15] == 0
    int32_t scan64;            // A/B probe (GAC_TILE_SCAN64=1): k_tile's 64-bit scans only
    int32_t xcd_chunk;         // A/B probe (GAC_TILE_XCD=1): each XCD takes one contiguous
                               // eighth of the tiles (default: per-round XCD blocks)
    GapDev gap;
    const int32_t *out_perm;  // non-null: the results of range (position) p go to
                              // chain out_perm[p] (the whole-chain plan in target order)
    const int32_t *tile_perm; // non-null: k_tile's schedule, tile_perm[k] = the k-th tile
                              // scored (whole chains: target order of the tiles' first blocks)
};

constexpr int kSmallMax = 256;  // ranges per small-batch call

// k_small_server's mailbox, in pinned coherent host memory: the host writes
// kind, n and the inputs, then req; the server writes done, and state = 2
// when it exits (idle or stop)
// k_small_server's mailbox, in pinned coherent host memory: the host writes
// kind, n and the inputs, then req; the server writes done, and state = 2
// when it exits (idle or stop)
struct SmallMail {
    uint32_t req;    // host: the request word (written last, srv_word)
    uint32_t kind;   // (unused)
    uint32_t n;      // (unused)
    uint32_t stop;   // host: 1 = exit now
    uint32_t done;   // server: the last completed request
    uint32_t state;  // server: 2 = exited
    uint32_t pad[26];
};
// its device-side copy for the other workgroups (the request number, kind
// and range count, read from the mailbox by workgroup 0 only) and the
// completion count: uncached device memory, zeroed per launch
struct SmallSync {
    uint32_t seq, kind, n, cnt;
    uint32_t pad[28];  // (GAC_SRV_TRACE's phase words)
};
constexpr int kSrvWaves = 256;  // resident server waves at most (64 workgroups)
// the request word: bits 0-19 the request number (never 0), 20-28 the range
// count (<= kSmallMax), 29 the kind (0: Range batch of the uploaded set; 1:
// host-planned RangeDesc + pool); 0xffffffff (never a request) = exit
__host__ __device__ constexpr uint32_t srv_word(uint32_t seq, uint32_t kind, uint32_t n) {
    return (seq & 0xfffffu) | ((n & 0x1ffu) << 20) | ((kind & 1u) << 29);
}

// One run of a sparse genome upload (bytes): its place in the staging layout
// (8-byte aligned), its offset in the packed upload (8-byte aligned), length.
struct SparseRun {
    int64_t dst, src, len;
};

// One ungapped block for k_blocks (axtScoreUngapped): global plane positions
// of its first target base and, for the query, of its first base ('+') or
// one past its last base on the forward strand ('-').
struct BlockJob {
    int64_t tp, qp;
    int32_t n;
    int32_t minus;
};

// Text jobs of the kent-API shims (k_text_blocks / k_text_xover): offsets
// into one uploaded byte buffer of caller text.
struct TextJob {
    int64_t q, t;  // offsets of the query / target text
    int32_t n;     // bases
    int32_t pad;
};

struct TextXJob {
    int64_t lq, lt, rq, rt;  // left block's last `ov` bases, right block's first
    int32_t ov;
    int32_t pad;
};

struct M25 {  // score by text code, [q * 5 + t]; code 4 (not acgt) scores 0
    int32_t m[25];
};

}  // namespace gac
