// gac_device.hip -- C-ABI implementation of libgachain (include/gachain.h):
// device context, resident genomes, chainsets, batched sub-chain scoring.
// There is deliberately no host fallback: every scoring entry point runs the
// HIP kernels of gac_kernels.hip on a gfx950 device or returns an error.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <time.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <memory>
#include <vector>

#include "gac_dp.h"
#include "gac_kernels.h"
#include "gachain.h"
#include "host/gac_host.h"

namespace gac {
int plan_grid(int64_t n);
int persistent_blocks_per_cu(int which, int sym);
hipError_t launch_plan(const ScoreArgs &a, hipStream_t s);
hipError_t launch_tilemap(const ScoreArgs &a, hipStream_t s);
hipError_t launch_plan_lb(const ScoreArgs &a, hipStream_t s);
bool plan_lb();
hipError_t launch_tile(const ScoreArgs &a, int grid, hipStream_t s);
hipError_t launch_combine(const ScoreArgs &a, int grid, hipStream_t s);
hipError_t launch_small(const ScoreArgs &a, const Range *rin, SmallOut *out, hipStream_t s);
hipError_t launch_small_host(const ScoreArgs &a, const RangeDesc *hin, const int4 *pool,
                             SmallOut *out, hipStream_t s);
hipError_t launch_small_server(const ScoreArgs &a0, const ScoreArgs &a1, const Range *rin,
                               const RangeDesc *hin, const int4 *pool, SmallOut *out,
                               SmallMail *mail, SmallSync *sy, uint32_t last_done, uint64_t idle,
                               uint32_t trace, int wgs, hipStream_t s);
struct SeqDev {
    int64_t byte_off;
    int64_t word_off;
    int32_t size;
    int32_t pad;
};
struct NPiece {
    int64_t bit0;
    int32_t len;
    int32_t pad;
};
hipError_t launch_relayout(const uint8_t *raw, const SeqDev *seqs, int nseq, int64_t nwords,
                           uint2 *planes, uint32_t *nmask, hipStream_t s);
hipError_t launch_gap_table(const GapDev &g, const int32_t *small, int len, int32_t *tab,
                            hipStream_t s);
hipError_t launch_nruns(const NPiece *p, int64_t n, uint32_t *nmask, hipStream_t s);
hipError_t launch_build_index(const int32_t *bt, const int32_t *bq, const int32_t *bs, int64_t nb,
                              const DChain *chains, int64_t n_chains, const int32_t *coff,
                              const int32_t *tile_c0, int2 *tspan, uint32_t *bucket,
                              hipStream_t s);
hipError_t launch_build_flat(const int32_t *bt, const int32_t *bq, const int32_t *bs, int64_t nb,
                             const DChain *chains, int64_t n_chains, int32_t *coff,
                             int32_t *tile_c0, int4 *crun, const longlong2 *t_runs,
                             int64_t n_trun, const longlong2 *q_runs, int64_t n_qrun,
                             const int64_t *q_woff, int4 *blk, int2 *tspan, uint32_t *bucket,
                             const UploadGaps &G, bool index, hipStream_t s);
hipError_t launch_block_gaps_flat(const int32_t *coff, const int32_t *tile_c0, int64_t nb,
                                  int4 *blk, Blk12 *blk12, const UploadGaps &G, hipStream_t s);
hipError_t launch_scatter(const SparseRun *runs, int64_t n, const uint64_t *compact,
                          uint64_t *raw, hipStream_t s);
hipError_t launch_blocks(const ScoreArgs &a, const BlockJob *jobs, int64_t n, int32_t *out,
                         hipStream_t s);
hipError_t launch_whole_plan(const DChain *chains, int64_t n, RangeDesc *rdesc, int32_t *nblk,
                             int32_t *gflat, int32_t *tile_r0, hipStream_t s);
hipError_t launch_zero_list(const int32_t *list, int64_t n, long long *g, long long *l,
                            int32_t *ali, hipStream_t s);
hipError_t launch_tile_order(const DChain *chains, const int4 *blk, const int32_t *tile_r0,
                             int64_t T, unsigned long long *keys, int32_t *vals, int32_t *perm,
                             void *tmp, size_t &tmp_bytes, hipStream_t s);
hipError_t launch_whole_plan_sorted(const DChain *chains, int64_t n, int32_t *perm,
                                    unsigned long long *keys, int32_t *vals, RangeDesc *rdesc,
                                    int32_t *nblk, int32_t *gflat, int32_t *pb0,
                                    int32_t *tile_r0, int32_t *inv, void *tmp,
                                    size_t &tmp_bytes, hipStream_t s);
hipError_t launch_text_blocks(const uint8_t *text, const TextJob *jobs, int64_t n, const M25 &m,
                              long long *out, hipStream_t s);
hipError_t launch_text_xover(const uint8_t *text, const TextXJob *jobs, int64_t n, const M25 &m,
                             int32_t *pos, int32_t *adj, hipStream_t s);
}  // namespace gac

using namespace gac;

#define HIPCHK(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return gac_fail(GAC_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), \
                            __FILE__, __LINE__);                                            \
    } while (0)

namespace {

struct Genome {
    // host-side staging until finalize
    std::vector<std::string> names;
    std::vector<int32_t> sizes;
    std::unordered_map<std::string, int32_t> index;
    std::vector<uint8_t> raw;       // payloads copied by gac_genome_add_seq, 8-B aligned
    std::vector<int64_t> raw_off;   // per seq: offset into raw (-1: payload is ext[i])
    std::vector<const uint8_t *> ext;  // per seq: payload inside the mapped .2bit file
    gac_twobit tb{};                // mapping kept open for ext (gac_genome_load_2bit)
    bool tb_open = false;
    // sparse upload (gac_genome_load_twobit_runs): only these word runs of
    // registered sequence run_seq[k], [run_lo, run_hi) in 32-base words
    bool sparse = false;
    std::vector<int32_t> run_seq, run_lo, run_hi;
    std::vector<NPiece> npieces;    // bit0 relative to the seq start until finalize
    std::vector<int32_t> npiece_seq;
    // host copy kept after finalize (raw stays): merged, sorted N runs per
    // sequence, CSR by nrun_off -- host-side base access (gac_genome_view)
    std::vector<int64_t> nrun_off{0};
    std::vector<int32_t> nrun_start, nrun_size;
    // device
    bool final = false;
    std::vector<int64_t> woff;      // host copy of word offsets
    int64_t n_words = 0;
    uint2 *planes = nullptr;
    uint32_t *nmask = nullptr;
    int64_t *d_woff = nullptr;
    longlong2 *d_nrun = nullptr;    // the N runs as global {start, end} bases, sorted
    int64_t n_nrun = 0;
    const uint8_t *packed(int i) const { return ext[i] ? ext[i] : raw.data() + raw_off[i]; }
};

struct Prof {
    int kernel;
    hipEvent_t a, b;
};

}  // namespace

constexpr size_t kStatusBytes = 128;  // status[0..9) (see ScoreArgs::status)

// held by every entry point that uses a context (see gac_ctx::mu); it also
// parks the small-batch server (k_small_server) first, so that nothing else
// runs beside a resident grid -- only the small-batch paths keep it
#define CTX_LOCK(c) CtxLock ctx_lock_((c), true)
#define CTX_LOCK_SMALL(c) CtxLock ctx_lock_((c), false)

// the resident small-batch server of a context (default; GAC_SMALL_SERVER=0
// launches k_small per batch instead)
struct SmallServer {
    bool on = false;       // enabled for this context
    bool running = false;  // a grid is resident (or exiting: mail->state 2)
    hipStream_t st = nullptr;
    SmallMail *mail = nullptr, *d_mail = nullptr;  // pinned, coherent
    SmallSync *d_sync = nullptr;
    Range *h_in = nullptr, *d_in = nullptr;        // pinned, coherent [kSmallMax]
    RangeDesc *h_hq = nullptr, *d_hq = nullptr;    // pinned, coherent [kSmallMax]
    int4 *h_pool = nullptr, *d_pool = nullptr;     // pinned, coherent, grown while parked
    int64_t pool_cap = 0;
    SmallOut *h_out = nullptr, *d_out = nullptr;   // pinned, coherent [kSmallMax]
    uint32_t seq = 0;                  // the last request made (= completed: calls wait)
    const gac_chainset *cs = nullptr;  // the set of kind-0 requests (nullptr: none)
    uint32_t gap_version = 0;
    int local = -1;
    ScoreArgs a0, a1;                  // the resident grid's arguments
    uint64_t idle = 2000000;           // exit after 20 ms without a request (100 MHz ticks)
    int64_t launches = 0, requests = 0;
    unsigned in_fl = 0;  // hipHostMalloc flags of the inputs
    int wgs = 16;        // workgroups of the grid (GAC_SRV_WGS, 1..kSrvWaves/4)
    bool wedged = false; // a grid did not exit within kParkSecs of its stop:
                         // the server is not used again (no unbounded wait)
};

struct gac_ctx {
    // every entry point that touches the context's state holds this (the
    // ABI is thread-safe per context; calls are serialised)
    std::recursive_mutex mu;
    // the scoring workspace is stream-ordered: ws_ev is recorded on the
    // stream of the last call that used it (ws_last); a call on another
    // stream waits for it on the device, and growing the workspace waits
    // for it on the host
    hipEvent_t ws_ev = nullptr;
    hipStream_t ws_last = nullptr;
    int device = 0;
    char arch[64] = {0};
    hipStream_t stream = nullptr;
    Genome g[2];
    bool scoring = false;
    int32_t coef[16];  // multilinear basis (ScoreArgs::coef)
    uint32_t gap_version = 0;  // bumped by every gac_set_scoring
    int sym = 0;
    GapDev gap;
    int32_t *d_small = nullptr;
    int32_t *d_gap_tab = nullptr;  // [3][gap_len]
    int gap_len = 0;
    // workspace
    int64_t ws_n = 0;
    RangeDesc *rdesc = nullptr;
    int32_t *nblk = nullptr, *goff = nullptr;
    int32_t *pb0 = nullptr;                  // [ws_n]
    int32_t *agg = nullptr;                  // [plan workgroups]
    int32_t *plan_off = nullptr;             // [plan workgroups]
    unsigned long long *lbflag = nullptr;    // [plan workgroups] k_plan_lb's look-back words
    int32_t *gflat = nullptr;                // [ws_n]
    int32_t *status = nullptr;               // [8]
    int64_t ws_tiles = 0;
    int32_t *tile_r0 = nullptr;              // [ws_tiles]
    SegSum *sum_head = nullptr, *sum_tail = nullptr;
    SegSum *sup_head = nullptr, *sup_tail = nullptr;  // [ws_tiles / 64 + 2]
    int32_t *sup_tail_r = nullptr;
    // staging for the host API
    int64_t io_n = 0;
    Range *d_ranges = nullptr;
    long long *d_g = nullptr, *d_l = nullptr;
    int32_t *d_ali = nullptr;
    Range *h_small_in = nullptr;     // pinned, mapped: ranges of a small batch [kSmallMax]
    SmallOut *h_small_out = nullptr; // pinned, mapped, coherent: its results
    Range *d_small_in = nullptr;     // their device addresses
    SmallOut *d_small_out = nullptr;
    int small_max = kSmallMax;       // batches up to this size take k_small (GAC_SMALL_MAX)
    // gac_score_ranges_host: planned ranges and their window records, pinned
    // and mapped (the kernel reads them over the bus), grown on demand
    RangeDesc *h_hq = nullptr, *d_hq = nullptr;  // [kSmallMax]
    int4 *h_pool = nullptr, *d_pool = nullptr;
    int64_t pool_cap = 0;
    int32_t mat[16] = {0};           // the current scoring setup (gac_set_scoring)
    gac_gapcalc *gap_src = nullptr;
    int32_t *h_stat = nullptr;   // pinned, coherent host words written by k_scan_agg [8]
    int32_t *d_h_stat = nullptr; // its device address
    int32_t call_seq = 0;
    // k_tile grids (resident workgroups) by [strand-symmetric matrix][local]
    int tile_grid_sym[2][2] = {{2048, 2048}, {2048, 2048}};
    int combine_grid = 512;
    // pinned staging for genome uploads (two buffers, alternating)
    uint8_t *pin[2] = {nullptr, nullptr};
    hipEvent_t pin_ev[2] = {nullptr, nullptr};
    // profiling
    int prof = 0;  // mask of timed kernels
    std::vector<Prof> prof_pending;
    std::vector<hipEvent_t> prof_free;
    double prof_ms[GAC_K_COUNT] = {0};
    int64_t prof_n[GAC_K_COUNT] = {0};
    // chain sets still open on this context: gac_close releases their
    // device memory and orphans them (ctx = NULL), so a set freed after its
    // context (a kent-shim cache, a garbage-collected binding) is only deleted
    std::vector<gac_chainset *> sets;
    SmallServer srv;
};

static void srv_park(gac_ctx *c);

struct CtxLock {
    std::lock_guard<std::recursive_mutex> g;
    CtxLock(gac_ctx *c, bool park) : g(c->mu) {
        if (park) srv_park(c);
    }
};

struct gac_chainset {
    gac_ctx *ctx;
    int64_t n_chains;
    int64_t n_blocks;
    DChain *chains = nullptr;
    int4 *blk = nullptr;  // {tStart, qStart, size | N flags, gap}, padded by one entry
    Blk12 *blk12 = nullptr;  // compact copy for k_tile (written with the gaps)
    uint32_t gap_version = 0;  // scoring setup the blk[].w gaps were computed for
    int2 *tspan = nullptr;  // {tStart, tEnd}
    uint32_t *bucket = nullptr;  // per-chain bucket indexes
    // whole-chain plan (gac_score_chains; built at its first call): the
    // scoring workspace of the batch "range c = chain c", fixed per set
    bool w_ready = false;
    RangeDesc *w_rdesc = nullptr;  // [n_chains]
    int32_t *w_nblk = nullptr;     // [n_chains]
    int32_t *w_gflat = nullptr;    // [n_chains] first block (= flat offset)
    int32_t *w_tile_r0 = nullptr;  // [tiles] chain owning each tile's first block
    int32_t *w_status = nullptr;   // {W, T, 0, 0}
    int32_t *w_empty = nullptr;    // chains without blocks (their results are 0)
    int64_t w_nempty = 0;
    // target-ordered plan (k_whole_keys): positions p are chains in target
    // order; w_pb0[p] their first blocks, results stored to chain w_perm[p]
    bool w_sorted = false;
    int32_t *w_pb0 = nullptr;
    int32_t *w_perm = nullptr;
    // set-order plan's tile schedule (k_tile's tile_perm): tiles in the
    // target order of their first blocks
    int32_t *w_tile_perm = nullptr;
    // capacities (gac_chains_reupload refills these buffers when they fit)
    size_t cap_chains = 0, cap_blocks = 0, cap_blk12 = 0, cap_tspan = 0, cap_idx = 0;
    int32_t *d_stage = nullptr;  // the caller's block arrays, staged (3 x blocks)
    size_t cap_stage = 0;
    // flat (lane per block) kernels: compact chain offsets [n + 1], the chain
    // of every 64-block tile's first block [tiles + 1], per-chain N-run
    // ranges {t first, t end, q first, q end} (empty: no run in its span)
    int32_t *d_coff = nullptr, *d_tile_c0 = nullptr;
    int4 *d_crun = nullptr;
    size_t cap_coff = 0, cap_tile_c0 = 0, cap_crun = 0;
    // the window-search index (tspan, bucket) is built: at upload
    // (GAC_UP_INDEX=eager) or at the first call that searches windows
    bool idx_ready = false;
    int64_t idx_n = 0;  // bucket entries of the index
};

static void free_whole_plan(gac_chainset *cs) {
    void *w[] = {cs->w_rdesc, cs->w_nblk, cs->w_gflat, cs->w_tile_r0, cs->w_status,
                 cs->w_empty, cs->w_pb0,  cs->w_perm,  cs->w_tile_perm};
    for (void *p : w)
        if (p) hipFree(p);
    cs->w_rdesc = nullptr;
    cs->w_nblk = cs->w_gflat = cs->w_tile_r0 = cs->w_status = cs->w_empty = nullptr;
    cs->w_pb0 = cs->w_perm = cs->w_tile_perm = nullptr;
    cs->w_sorted = false;
    cs->w_nempty = 0;
    cs->w_ready = false;
}

// ----------------------------------------------------------------- context
extern "C" int gac_open(int device, gac_ctx **out) {
    gac_clear_error();
    if (!out) return gac_fail(GAC_E_ARG, "gac_open: NULL out");
    *out = nullptr;
    const bool timing = getenv("GAC_TIMING") != nullptr;
    auto t_now = [] {
        struct timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        return ts.tv_sec + 1e-9 * ts.tv_nsec;
    };
    double t_mark = t_now();
    auto lap = [&](const char *what) {
        if (!timing) return;
        const double t = t_now();
        fprintf(stderr, "[gac_open] %-28s %.3f s\n", what, t - t_mark);
        t_mark = t;
    };
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    lap("hipGetDeviceCount (HIP init)");
    if (e != hipSuccess || n == 0)
        return gac_fail(GAC_E_HIP, "no HIP device available (%s); libgachain has no CPU fallback",
                        hipGetErrorString(e));
    if (device < 0 || device >= n)
        return gac_fail(GAC_E_ARG, "device %d out of range (%d devices)", device, n);
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    lap("hipGetDeviceProperties");
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return gac_fail(GAC_E_HIP, "device %d is %s; libgachain is built for gfx950 only", device,
                        prop.gcnArchName);
    HIPCHK(hipSetDevice(device));
    lap("hipSetDevice");
    gac_ctx *c = new gac_ctx();
    c->device = device;
    snprintf(c->arch, sizeof(c->arch), "%s", prop.gcnArchName);
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return gac_fail(GAC_E_HIP, "hipStreamCreate failed");
    }
    if (hipEventCreateWithFlags(&c->ws_ev, hipEventDisableTiming) != hipSuccess) {
        hipStreamDestroy(c->stream);
        delete c;
        return gac_fail(GAC_E_HIP, "hipEventCreate failed");
    }
    lap("hipStreamCreate");
    c->combine_grid = prop.multiProcessorCount * 8;  // k_fold_tiles: 32 waves per CU
    for (int sym = 0; sym < 2; ++sym)
        for (int l = 0; l < 2; ++l)
            c->tile_grid_sym[sym][l] = prop.multiProcessorCount * persistent_blocks_per_cu(l, sym);
    lap("occupancy (code object)");
    if (hipHostMalloc((void **)&c->h_stat, 64, hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void **)&c->d_h_stat, c->h_stat, 0) != hipSuccess) {
        hipStreamDestroy(c->stream);
        delete c;
        return gac_fail(GAC_E_HIP, "hipHostMalloc failed");
    }
    if (hipHostMalloc((void **)&c->h_small_in, kSmallMax * sizeof(Range), hipHostMallocMapped) !=
            hipSuccess ||
        hipHostMalloc((void **)&c->h_small_out, kSmallMax * sizeof(SmallOut),
                      hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void **)&c->d_small_in, c->h_small_in, 0) != hipSuccess ||
        hipHostGetDevicePointer((void **)&c->d_small_out, c->h_small_out, 0) != hipSuccess) {
        gac_close(c);
        return gac_fail(GAC_E_HIP, "hipHostMalloc failed");
    }
    if (const char *v = getenv("GAC_SMALL_MAX")) {
        const int m = atoi(v);
        c->small_max = m < 0 ? 0 : (m > kSmallMax ? kSmallMax : m);
    }
    c->srv.on = true;  // (GAC_SMALL_SERVER=0: a launch per small batch)
    if (const char *v = getenv("GAC_SMALL_SERVER")) c->srv.on = v[0] != '0';
    if (const char *v = getenv("GAC_SRV_WGS")) {
        const int w = atoi(v);
        if (w >= 1 && w <= kSrvWaves / kWavesPerWG) c->srv.wgs = w;
    }
    if (const char *v = getenv("GAC_SMALL_SERVER_IDLE_US")) {
        const long long us = atoll(v);
        if (us > 0 && us <= 10000000) c->srv.idle = (uint64_t)us * 100;
    }
    lap("hipHostMalloc");
    *out = c;
    return GAC_OK;
}

static void free_genome(Genome &g) {
    if (g.tb_open) gac_twobit_close(&g.tb);
    if (g.planes) hipFree(g.planes);
    if (g.nmask) hipFree(g.nmask);
    if (g.d_woff) hipFree(g.d_woff);
    if (g.d_nrun) hipFree(g.d_nrun);
    g = Genome();
}

static void free_set_memory(gac_chainset *cs);

static void srv_free(gac_ctx *c);

extern "C" void gac_close(gac_ctx *c) {
    if (!c) return;
    hipSetDevice(c->device);
    {
        std::lock_guard<std::recursive_mutex> g(c->mu);
        srv_park(c);
        if (c->srv.launches && getenv("GAC_TIMING"))
            fprintf(stderr, "[gac_close] small-batch server: %lld requests, %lld launches\n",
                    (long long)c->srv.requests, (long long)c->srv.launches);
        if (c->srv.d_sync && getenv("GAC_SRV_TRACE")) {  // (the last grid's phase sums)
            SmallSync t;
            if (hipMemcpy(&t, c->srv.d_sync, sizeof(t), hipMemcpyDeviceToHost) == hipSuccess &&
                t.pad[15])
                fprintf(stderr, "[gac_close] server phases (us after the poll saw the request, "
                                "mean of %u): broadcast %.2f, all saw %.2f, "
                                "work %.2f, fenced %.2f, done %.2f; polls %.1f\n",
                        t.pad[15], 0.01 * t.pad[8] / t.pad[15], 0.01 * t.pad[9] / t.pad[15],
                        0.01 * t.pad[11] / t.pad[15],
                        0.01 * t.pad[12] / t.pad[15], 0.01 * t.pad[13] / t.pad[15],
                        (double)t.pad[14] / t.pad[15]);
        }
        srv_free(c);
    }
    hipStreamSynchronize(c->stream);
    {
        CTX_LOCK(c);
        for (gac_chainset *cs : c->sets) {
            free_set_memory(cs);
            cs->ctx = nullptr;
        }
        c->sets.clear();
    }
    free_genome(c->g[0]);
    free_genome(c->g[1]);
    void *bufs[] = {c->d_small,  c->d_gap_tab, c->rdesc,    c->nblk,     c->goff, c->pb0, c->agg, c->plan_off, c->lbflag, c->gflat,
                    c->status,   c->tile_r0,  c->sum_head, c->sum_tail,
                    c->sup_head, c->sup_tail, c->sup_tail_r,
                    c->d_ranges, c->d_g,      c->d_l,      c->d_ali};
    for (void *p : bufs)
        if (p) hipFree(p);
    for (auto &p : c->prof_pending) {
        hipEventDestroy(p.a);
        hipEventDestroy(p.b);
    }
    for (auto ev : c->prof_free) hipEventDestroy(ev);
    if (c->h_stat) hipHostFree(c->h_stat);
    gac_gapcalc_free(c->gap_src);
    if (c->h_small_in) hipHostFree(c->h_small_in);
    if (c->h_small_out) hipHostFree(c->h_small_out);
    if (c->h_hq) hipHostFree(c->h_hq);
    if (c->h_pool) hipHostFree(c->h_pool);
    for (int k = 0; k < 2; ++k) {
        if (c->pin[k]) hipHostFree(c->pin[k]);
        if (c->pin_ev[k]) hipEventDestroy(c->pin_ev[k]);
    }
    if (c->ws_ev) hipEventDestroy(c->ws_ev);
    hipStreamDestroy(c->stream);
    delete c;
}

extern "C" const char *gac_device_arch(gac_ctx *c) { return c ? c->arch : ""; }

// ----------------------------------------------------------------- scoring
static int acgt_of_code(int code) {  // 2bit code T=0 C=1 A=2 G=3 -> A,C,G,T index
    static const int m[4] = {3, 1, 0, 2};
    return m[code];
}

extern "C" int gac_set_scoring(gac_ctx *c, const int32_t mat[16], const gac_gapcalc *g) {
    gac_clear_error();
    if (!c || !mat || !g) return gac_fail(GAC_E_ARG, "gac_set_scoring: NULL argument");
    CTX_LOCK(c);
    if (g->long_count < 2 || g->long_count > kMaxLong)
        return gac_fail(GAC_E_ARG, "gap table has %d long positions (2..%d supported)",
                        g->long_count, kMaxLong);
    if (g->small_size < 1 || g->small_size != g->long_pos[0])
        return gac_fail(GAC_E_ARG, "inconsistent gap table (smallSize %d)", g->small_size);
    HIPCHK(hipSetDevice(c->device));
    // the same setup again (a batch of jobs): tables, gap version and the
    // chain sets' per-block gaps stay valid
    if (c->scoring && memcmp(c->mat, mat, sizeof(c->mat)) == 0 && gac_gapcalc_same(c->gap_src, g))
        return GAC_OK;
    // the kernel multiplies basis coefficients (|c| <= 16 max|s|) by counts
    // <= 32 in 24 bits (v_mad_i32_i24) and sums 16 terms in int32
    for (int i = 0; i < 16; ++i)
        if (mat[i] <= -(1 << 17) || mat[i] >= (1 << 17))
            return gac_fail(GAC_E_ARG, "score matrix entry %d out of range (|s| < 2^17)", mat[i]);
    // f(S) = M[q][t] at t1,t0,d1,d0 = bits of S (q = t ^ d); Moebius transform
    // to the multilinear coefficients
    int32_t f[16];
    for (int S = 0; S < 16; ++S) {
        const int t = S >> 2, q = t ^ (S & 3);
        f[S] = mat[acgt_of_code(q) * 4 + acgt_of_code(t)];
    }
    for (int S = 0; S < 16; ++S) {
        int32_t cs = 0;
        for (int T = 0; T < 16; ++T)
            if ((T & S) == T) cs += (__builtin_popcount(S ^ T) & 1) ? -f[T] : f[T];
        c->coef[S] = cs;
    }
    c->sym = 1;
    for (int S = 8; S < 16; ++S)
        if (c->coef[S]) c->sym = 0;
    GapDev &d = c->gap;
    memset(&d, 0, sizeof(d));
    d.small_size = g->small_size;
    d.long_count = g->long_count;
    d.last_pos[0] = g->q_last_pos;
    d.last_pos[1] = g->t_last_pos;
    d.last_pos[2] = g->b_last_pos;
    d.last_val[0] = g->q_last_val;
    d.last_val[1] = g->t_last_val;
    d.last_val[2] = g->b_last_val;
    d.last_slope[0] = g->q_last_slope;
    d.last_slope[1] = g->t_last_slope;
    d.last_slope[2] = g->b_last_slope;
    for (int i = 0; i < g->long_count; ++i) {
        d.long_pos[i] = g->long_pos[i];
        d.long_val[0][i] = g->q_long[i];
        d.long_val[1][i] = g->t_long[i];
        d.long_val[2][i] = g->b_long[i];
    }
    std::vector<int32_t> small(3 * (size_t)g->small_size);
    memcpy(small.data(), g->q_small, g->small_size * 4);
    memcpy(small.data() + g->small_size, g->t_small, g->small_size * 4);
    memcpy(small.data() + 2 * g->small_size, g->b_small, g->small_size * 4);
    if (c->d_small) hipFree(c->d_small);
    c->d_small = nullptr;
    HIPCHK(hipMalloc(&c->d_small, small.size() * 4));
    HIPCHK(hipMemcpy(c->d_small, small.data(), small.size() * 4, hipMemcpyHostToDevice));
    // gap-cost table up to the last table position (everything beyond is the
    // slope branch); capped at GAC_GAP_TABLE_MAX entries per kind (default
    // 2^22) -- lengths past a capped table are evaluated in the kernel
    int64_t len = std::max(std::max(g->q_last_pos, g->t_last_pos), g->b_last_pos);
    int64_t cap = 1 << 22;
    if (const char *env = getenv("GAC_GAP_TABLE_MAX")) cap = std::max(1LL, atoll(env));
    len = std::max<int64_t>(g->small_size, std::min(len, cap));
    if (c->d_gap_tab) hipFree(c->d_gap_tab);
    c->d_gap_tab = nullptr;
    HIPCHK(hipMalloc(&c->d_gap_tab, 3 * len * 4));
    HIPCHK(launch_gap_table(d, c->d_small, (int)len, c->d_gap_tab, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    c->gap_len = (int)len;
    ++c->gap_version;
    memcpy(c->mat, mat, sizeof(c->mat));
    gac_gapcalc_free(c->gap_src);
    c->gap_src = gac_gapcalc_clone(g);
    c->scoring = true;
    return GAC_OK;
}

// ----------------------------------------------------------------- genomes
static Genome *side_of(gac_ctx *c, int side) {
    if (!c || (side != GAC_T && side != GAC_Q)) return nullptr;
    return &c->g[side];
}

// copy = false: the payload stays where it is (a mapped .2bit file kept open
// by the genome) and is read straight into pinned staging at finalize.
static int add_seq(gac_ctx *c, int side, const char *name, int32_t size, const uint8_t *packed,
                   bool copy, int32_t n_nblocks, const int32_t *n_starts,
                   const int32_t *n_sizes) {
    Genome *g = side_of(c, side);
    if (!g || !name || size < 0 || (size > 0 && !packed) || n_nblocks < 0)
        return gac_fail(GAC_E_ARG, "gac_genome_add_seq: bad argument");
    if (g->final) return gac_fail(GAC_E_STATE, "genome side %d already finalized", side);
    if (g->index.count(name)) return gac_fail(GAC_E_ARG, "duplicate sequence %s", name);
    int32_t idx = (int32_t)g->names.size();
    g->index[name] = idx;
    g->names.push_back(name);
    g->sizes.push_back(size);
    size_t nbytes = ((size_t)size + 3) / 4;
    if (copy) {
        size_t off = (g->raw.size() + 7) & ~(size_t)7;
        g->raw.resize(off + nbytes);
        if (nbytes) memcpy(g->raw.data() + off, packed, nbytes);
        g->raw_off.push_back((int64_t)off);
        g->ext.push_back(nullptr);
    } else {
        g->raw_off.push_back(-1);
        g->ext.push_back(packed);
    }
    {
        std::vector<std::pair<int32_t, int32_t>> runs;
        for (int32_t i = 0; i < n_nblocks; ++i)
            if (n_sizes[i] > 0) runs.emplace_back(n_starts[i], n_starts[i] + n_sizes[i]);
        std::sort(runs.begin(), runs.end());
        size_t k0 = g->nrun_start.size();
        for (const auto &r : runs) {
            const size_t k = g->nrun_start.size();
            if (k > k0 && r.first <= g->nrun_start[k - 1] + g->nrun_size[k - 1]) {
                const int32_t e = std::max(g->nrun_start[k - 1] + g->nrun_size[k - 1], r.second);
                g->nrun_size[k - 1] = e - g->nrun_start[k - 1];
            } else {
                g->nrun_start.push_back(r.first);
                g->nrun_size.push_back(r.second - r.first);
            }
        }
        g->nrun_off.push_back((int64_t)g->nrun_start.size());
    }
    for (int32_t i = 0; i < n_nblocks; ++i) {
        int64_t s = n_starts[i], len = n_sizes[i];
        if (s < 0 || len < 0 || s + len > size)
            return gac_fail(GAC_E_FORMAT, "N block %d of %s out of range", i, name);
        while (len > 0) {
            int32_t piece = (int32_t)(len < 1024 ? len : 1024);
            g->npieces.push_back(NPiece{s, piece, 0});
            g->npiece_seq.push_back(idx);
            s += piece;
            len -= piece;
        }
    }
    return GAC_OK;
}

extern "C" int gac_genome_add_seq(gac_ctx *c, int side, const char *name, int32_t size,
                                  const uint8_t *packed, int32_t n_nblocks,
                                  const int32_t *n_starts, const int32_t *n_sizes) {
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    return add_seq(c, side, name, size, packed, true, n_nblocks, n_starts, n_sizes);
}

// Staged upload of the packed payloads to d_raw (layout: seqs[i].byte_off,
// 8-byte aligned): host threads copy 32 MB windows into two alternating
// pinned buffers while the previous window's DMA runs.
// (GAC_PIN_MB overrides the window size: measurement knob)
static size_t pin_bytes() {
    static const size_t b = getenv("GAC_PIN_MB") ? (size_t)std::max(1, atoi(getenv("GAC_PIN_MB"))) << 20
                                                  : (size_t)32 << 20;
    return b;
}

struct StageJob {
    const Genome *g;
    const SeqDev *seqs;
    int nseq;
    size_t lo, hi;   // window of the staging layout
    uint8_t *dst;    // pinned buffer (window start)
    int nt;
};

static void *stage_thread_body(StageJob *J, int t) {
    const size_t len = J->hi - J->lo, per = (len + J->nt - 1) / J->nt;
    const size_t a = J->lo + std::min(len, per * t), b = J->lo + std::min(len, per * (t + 1));
    if (a >= b) return nullptr;
    // sequences overlapping [a, b): binary search the first
    int lo = 0, hi = J->nseq;
    while (lo < hi) {
        const int m = (lo + hi) / 2;
        const size_t end = (size_t)J->seqs[m].byte_off + ((size_t)J->seqs[m].size + 3) / 4;
        if (end <= a) lo = m + 1;
        else hi = m;
    }
    size_t pos = a;
    for (int i = lo; i < J->nseq && pos < b; ++i) {
        const size_t s0 = (size_t)J->seqs[i].byte_off;
        const size_t s1 = s0 + ((size_t)J->seqs[i].size + 3) / 4;
        if (s0 > pos) {  // alignment padding
            const size_t z = std::min(s0, b) - pos;
            memset(J->dst + (pos - J->lo), 0, z);
            pos += z;
            if (pos >= b) break;
        }
        const size_t e = std::min(s1, b);
        if (e > pos) {
            memcpy(J->dst + (pos - J->lo), J->g->packed(i) + (pos - s0), e - pos);
            pos = e;
        }
    }
    if (pos < b) memset(J->dst + (pos - J->lo), 0, b - pos);
    return nullptr;
}

struct StageArg {
    StageJob *J;
    std::atomic<int> next;
};

static void *stage_thread(void *p) {
    StageArg *A = (StageArg *)p;
    for (int t; (t = A->next.fetch_add(1)) < A->J->nt;) stage_thread_body(A->J, t);
    return nullptr;
}

static int ensure_pinned(gac_ctx *c) {
    for (int k = 0; k < 2; ++k) {
        if (!c->pin[k]) HIPCHK(hipHostMalloc((void **)&c->pin[k], pin_bytes(), hipHostMallocDefault));
        if (!c->pin_ev[k]) HIPCHK(hipEventCreateWithFlags(&c->pin_ev[k], hipEventDisableTiming));
    }
    return GAC_OK;
}

// Sparse: the runs' bytes packed (compact layout, SparseRun::src), staged the
// same way through the pinned windows.
struct StageRunsJob {
    const Genome *g;
    const SparseRun *runs;
    const int32_t *seq;  // registered sequence of each run
    const SeqDev *seqs;
    int64_t nruns;
    size_t lo, hi;
    uint8_t *dst;
    int nt;
};

static void stage_runs_body(StageRunsJob *J, int t) {
    const size_t len = J->hi - J->lo, per = (len + J->nt - 1) / J->nt;
    const size_t a = J->lo + std::min(len, per * t), b = J->lo + std::min(len, per * (t + 1));
    if (a >= b) return;
    int64_t lo = 0, hi = J->nruns;  // first run ending after a
    while (lo < hi) {
        const int64_t m = (lo + hi) / 2;
        if ((size_t)(J->runs[m].src + ((J->runs[m].len + 7) & ~7LL)) <= a) lo = m + 1;
        else hi = m;
    }
    size_t pos = a;
    for (int64_t r = lo; r < J->nruns && pos < b; ++r) {
        const SparseRun &R = J->runs[r];
        const size_t s0 = (size_t)R.src, s1 = s0 + (size_t)R.len;
        const size_t e0 = s0 + (((size_t)R.len + 7) & ~(size_t)7);  // padded end
        const int k = J->seq[r];
        const uint8_t *from = J->g->packed(k) + (R.dst - J->seqs[k].byte_off);
        if (s1 > pos) {
            const size_t e = std::min(s1, b);
            memcpy(J->dst + (pos - J->lo), from + (pos - s0), e - pos);
            pos = e;
        }
        if (pos < b && e0 > pos) {
            const size_t e = std::min(e0, b);
            memset(J->dst + (pos - J->lo), 0, e - pos);
            pos = e;
        }
    }
    if (pos < b) memset(J->dst + (pos - J->lo), 0, b - pos);
}

struct StageRunsArg {
    StageRunsJob *J;
    std::atomic<int> next;
};

static void *stage_runs_thread(void *p) {
    StageRunsArg *A = (StageRunsArg *)p;
    for (int t; (t = A->next.fetch_add(1)) < A->J->nt;) stage_runs_body(A->J, t);
    return nullptr;
}

static int ensure_pinned(gac_ctx *c);

static int upload_runs(gac_ctx *c, const Genome *g, const SeqDev *seqs, const SparseRun *runs,
                       const int32_t *seq, int64_t nruns, uint8_t *d_compact, size_t bytes) {
    int rc = ensure_pinned(c);
    if (rc != GAC_OK) return rc;
    const int nt = std::max(1, std::min(16, gac_host_threads()));
    int k = 0;
    for (size_t lo = 0; lo < bytes; lo += pin_bytes(), k ^= 1) {
        const size_t hi = std::min(bytes, lo + pin_bytes());
        HIPCHK(hipEventSynchronize(c->pin_ev[k]));
        StageRunsJob J = {g, runs, seq, seqs, nruns, lo, hi, c->pin[k], nt};
        StageRunsArg A;
        A.J = &J;
        A.next = 0;
        gac_run_threads(nt, stage_runs_thread, &A);
        HIPCHK(hipMemcpyAsync(d_compact + lo, c->pin[k], hi - lo, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipEventRecord(c->pin_ev[k], c->stream));
    }
    return GAC_OK;
}

static int upload_payloads(gac_ctx *c, const Genome *g, const SeqDev *seqs, int nseq,
                           uint8_t *d_raw, size_t raw_bytes) {
    int rc = ensure_pinned(c);
    if (rc != GAC_OK) return rc;
    const int nt = std::max(1, std::min(16, gac_host_threads()));
    int k = 0;
    for (size_t lo = 0; lo < raw_bytes; lo += pin_bytes(), k ^= 1) {
        const size_t hi = std::min(raw_bytes, lo + pin_bytes());
        HIPCHK(hipEventSynchronize(c->pin_ev[k]));  // its previous DMA is done
        StageJob J = {g, seqs, nseq, lo, hi, c->pin[k], nt};
        StageArg A;
        A.J = &J;
        A.next = 0;
        gac_run_threads(nt, stage_thread, &A);
        HIPCHK(hipMemcpyAsync(d_raw + lo, c->pin[k], hi - lo, hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipEventRecord(c->pin_ev[k], c->stream));
    }
    return GAC_OK;
}

static double wall_s() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

// GAC_TIMING laps of a genome upload
struct FinLaps {
    bool on = getenv("GAC_TIMING") != nullptr;
    int side;
    double t = wall_s();
    void operator()(const char *what) {
        if (!on) return;
        const double n = wall_s();
        fprintf(stderr, "[gac_genome_finalize %c] %-22s %.3f s\n", side ? 'Q' : 'T', what, n - t);
        t = n;
    }
};

extern "C" int gac_genome_finalize(gac_ctx *c, int side) {
    gac_clear_error();
    Genome *g = side_of(c, side);
    if (!g) return gac_fail(GAC_E_ARG, "gac_genome_finalize: bad side");
    CTX_LOCK(c);
    if (g->final) return gac_fail(GAC_E_STATE, "genome side %d already finalized", side);
    FinLaps lap;
    lap.side = side;
    HIPCHK(hipSetDevice(c->device));
    const int nseq = (int)g->names.size();
    std::vector<SeqDev> seqs(nseq);
    g->woff.resize(nseq);
    int64_t w = 0;
    size_t raw_bytes = 0;  // staging layout: payloads 8-byte aligned, in sequence order
    for (int i = 0; i < nseq; ++i) {
        raw_bytes = (raw_bytes + 7) & ~(size_t)7;
        seqs[i].byte_off = (int64_t)raw_bytes;
        raw_bytes += ((size_t)g->sizes[i] + 3) / 4;
        seqs[i].word_off = w;
        seqs[i].size = g->sizes[i];
        g->woff[i] = w;
        w += ((int64_t)g->sizes[i] + 31) / 32;
    }
    g->n_words = w;
    // the scoring kernels index plane words in 32 bits (2^37 bases per side)
    if (w + 4 > (int64_t)UINT32_MAX)
        return gac_fail(GAC_E_ARG, "genome of %lld words: over the 2^32-word plane limit", (long long)w);
    const int64_t alloc_words = w + 4;  // padding: windows read word w+1
    HIPCHK(hipMalloc(&g->planes, alloc_words * sizeof(uint2)));
    HIPCHK(hipMalloc(&g->nmask, alloc_words * sizeof(uint32_t)));
    HIPCHK(hipMalloc(&g->d_woff, (nseq ? nseq : 1) * sizeof(int64_t)));
    // (k_relayout writes every word of the sequences: only the padding words
    // past them are set here)
    HIPCHK(hipMemsetAsync(g->planes + w, 0, (alloc_words - w) * sizeof(uint2), c->stream));
    HIPCHK(hipMemsetAsync(g->nmask + w, 0xff, (alloc_words - w) * sizeof(uint32_t), c->stream));
    if (nseq) {
        HIPCHK(hipMemcpyAsync(g->d_woff, g->woff.data(), nseq * sizeof(int64_t),
                              hipMemcpyHostToDevice, c->stream));
        uint8_t *d_raw = nullptr;
        SeqDev *d_seqs = nullptr;
        NPiece *d_np = nullptr;
        HIPCHK(hipMalloc(&d_raw, raw_bytes + 16));
        HIPCHK(hipMalloc(&d_seqs, nseq * sizeof(SeqDev)));
        lap("allocations");
        uint8_t *d_compact = nullptr;
        SparseRun *d_runs = nullptr;
        if (g->sparse) {  // only the listed word runs
            std::vector<SparseRun> runs;
            std::vector<int32_t> rseq;
            int64_t compact = 0;
            for (size_t r = 0; r < g->run_seq.size(); ++r) {
                const int k = g->run_seq[r];
                const int64_t pay = ((int64_t)g->sizes[k] + 3) / 4;
                const int64_t b0 = (int64_t)g->run_lo[r] * 8, b1 = std::min<int64_t>((int64_t)g->run_hi[r] * 8, pay);
                if (b1 <= b0) continue;
                runs.push_back(SparseRun{seqs[k].byte_off + b0, compact, b1 - b0});
                rseq.push_back(k);
                compact += ((b1 - b0) + 7) & ~7LL;
            }
            HIPCHK(hipMalloc(&d_compact, (size_t)compact + 16));
            HIPCHK(hipMalloc(&d_runs, std::max<size_t>(runs.size(), 1) * sizeof(SparseRun)));
            int rc = upload_runs(c, g, seqs.data(), runs.data(), rseq.data(), (int64_t)runs.size(),
                                 d_compact, (size_t)compact);
            if (rc != GAC_OK) return rc;
            HIPCHK(hipMemcpyAsync(d_runs, runs.data(), runs.size() * sizeof(SparseRun),
                                  hipMemcpyHostToDevice, c->stream));
            HIPCHK(launch_scatter(d_runs, (int64_t)runs.size(), (const uint64_t *)d_compact,
                                  (uint64_t *)d_raw, c->stream));
            lap("sparse runs queued");
        } else {
            int rc = upload_payloads(c, g, seqs.data(), nseq, d_raw, raw_bytes);
            if (rc != GAC_OK) return rc;
            lap("payload copies queued");
        }
        HIPCHK(hipMemcpyAsync(d_seqs, seqs.data(), nseq * sizeof(SeqDev), hipMemcpyHostToDevice,
                              c->stream));
        HIPCHK(launch_relayout(d_raw, d_seqs, nseq, w, g->planes, g->nmask, c->stream));
        const int64_t np = (int64_t)g->npieces.size();
        if (np) {
            for (int64_t i = 0; i < np; ++i)
                g->npieces[i].bit0 += g->woff[g->npiece_seq[i]] * 32;
            HIPCHK(hipMalloc(&d_np, np * sizeof(NPiece)));
            HIPCHK(hipMemcpyAsync(d_np, g->npieces.data(), np * sizeof(NPiece),
                                  hipMemcpyHostToDevice, c->stream));
            HIPCHK(launch_nruns(d_np, np, g->nmask, c->stream));
        }
        HIPCHK(hipStreamSynchronize(c->stream));
        lap("relayout + N runs done");
        if (d_compact) hipFree(d_compact);
        if (d_runs) hipFree(d_runs);
        hipFree(d_raw);
        hipFree(d_seqs);
        if (d_np) hipFree(d_np);
    } else {
        HIPCHK(hipStreamSynchronize(c->stream));
    }
    std::vector<NPiece>().swap(g->npieces);
    std::vector<int32_t>().swap(g->npiece_seq);
    {  // global N runs (chain-level N test at chain upload)
        std::vector<longlong2> gr(g->nrun_start.size());
        for (int i = 0; i < nseq; ++i)
            for (int64_t k = g->nrun_off[i]; k < g->nrun_off[i + 1]; ++k) {
                gr[k].x = g->woff[i] * 32 + g->nrun_start[k];
                gr[k].y = gr[k].x + g->nrun_size[k];
            }
        g->n_nrun = (int64_t)gr.size();
        HIPCHK(hipMalloc(&g->d_nrun, std::max<size_t>(gr.size(), 1) * sizeof(longlong2)));
        if (!gr.empty())
            HIPCHK(hipMemcpy(g->d_nrun, gr.data(), gr.size() * sizeof(longlong2),
                             hipMemcpyHostToDevice));
    }
    g->final = true;
    return GAC_OK;
}

extern "C" int gac_genome_load_2bit(gac_ctx *c, int side, const char *path) {
    gac_clear_error();
    if (!side_of(c, side) || !path) return gac_fail(GAC_E_ARG, "gac_genome_load_2bit: bad argument");
    gac_twobit tb;
    int rc = gac_twobit_open(path, &tb);
    if (rc != GAC_OK) return rc;
    return gac_genome_load_twobit(c, side, &tb);
}

extern "C" int gac_genome_load_twobit(gac_ctx *c, int side, gac_twobit *tbp) {
    return gac_genome_load_twobit_runs(c, side, tbp, nullptr, nullptr, nullptr, nullptr);
}

extern "C" int gac_genome_load_twobit_keep(gac_ctx *c, int side, gac_twobit *tbp,
                                           const uint8_t *keep) {
    return gac_genome_load_twobit_runs(c, side, tbp, keep, nullptr, nullptr, nullptr);
}

extern "C" int gac_genome_load_twobit_runs(gac_ctx *c, int side, gac_twobit *tbp,
                                           const uint8_t *keep, const int64_t *run_off,
                                           const int32_t *run_lo, const int32_t *run_hi) {
    gac_clear_error();
    if (!side_of(c, side) || !tbp) {
        if (tbp) gac_twobit_close(tbp);
        return gac_fail(GAC_E_ARG, "gac_genome_load_twobit: bad argument");
    }
    CTX_LOCK(c);
    gac_twobit tb = *tbp;
    int rc = GAC_OK;
    std::vector<int32_t> ns, nz;
    for (uint32_t i = 0; i < tb.seq_count && rc == GAC_OK; ++i) {
        if (keep && !keep[i]) continue;  // a sequence this process never scores
        const gac_twobit_seq &s = tb.seqs[i];
        ns.resize(s.n_count);
        nz.resize(s.n_count);
        for (uint32_t k = 0; k < s.n_count; ++k) {
            ns[k] = (int32_t)gac_twobit_u32(&tb, s.n_starts_raw + 4 * k);
            nz[k] = (int32_t)gac_twobit_u32(&tb, s.n_sizes_raw + 4 * k);
        }
        rc = add_seq(c, side, s.name, (int32_t)s.size, s.packed, false, (int32_t)s.n_count,
                     ns.data(), nz.data());
        if (rc == GAC_OK && run_off) {  // this sequence's word runs
            Genome *g = side_of(c, side);
            g->sparse = true;
            const int32_t k = (int32_t)g->names.size() - 1;
            const int64_t nw = ((int64_t)s.size + 31) / 32;
            for (int64_t r = run_off[i]; r < run_off[i + 1]; ++r) {
                const int32_t lo = std::max<int32_t>(0, run_lo[r]);
                const int32_t hi = (int32_t)std::min<int64_t>(nw, run_hi[r]);
                if (hi <= lo) continue;
                g->run_seq.push_back(k);
                g->run_lo.push_back(lo);
                g->run_hi.push_back(hi);
            }
        }
    }
    if (rc != GAC_OK) {  // the side holds pointers into tb: drop it whole
        free_genome(*side_of(c, side));
        gac_twobit_close(&tb);
        return rc;
    }
    // the payloads are read from the mapping at finalize and by gac_genome_view
    Genome *g = side_of(c, side);
    g->tb = tb;
    g->tb_open = true;
    return gac_genome_finalize(c, side);
}

extern "C" int32_t gac_genome_seq_count(gac_ctx *c, int side) {
    Genome *g = side_of(c, side);
    return g ? (int32_t)g->names.size() : -1;
}

extern "C" int32_t gac_genome_seq_index(gac_ctx *c, int side, const char *name) {
    Genome *g = side_of(c, side);
    if (!g || !name) return -1;
    auto it = g->index.find(name);
    return it == g->index.end() ? -1 : it->second;
}

extern "C" int32_t gac_genome_seq_size(gac_ctx *c, int side, int32_t i) {
    Genome *g = side_of(c, side);
    if (!g || i < 0 || i >= (int32_t)g->sizes.size()) return -1;
    return g->sizes[i];
}

extern "C" const char *gac_genome_seq_name(gac_ctx *c, int side, int32_t i) {
    Genome *g = side_of(c, side);
    if (!g || i < 0 || i >= (int32_t)g->names.size()) return nullptr;
    return g->names[i].c_str();
}

extern "C" int gac_genome_decode(gac_ctx *c, int side, int32_t i, int32_t start, int32_t end,
                                 char *out) {
    gac_clear_error();
    Genome *g = side_of(c, side);
    if (!g || !g->final || i < 0 || i >= (int32_t)g->sizes.size() || start < 0 ||
        end > g->sizes[i] || start > end || !out)
        return gac_fail(GAC_E_ARG, "gac_genome_decode: bad argument");
    if (start == end) return GAC_OK;
    HIPCHK(hipSetDevice(c->device));
    const int64_t w0 = g->woff[i] + start / 32, w1 = g->woff[i] + (end - 1) / 32 + 1;
    std::vector<uint2> pl(w1 - w0);
    std::vector<uint32_t> nm(w1 - w0);
    HIPCHK(hipMemcpy(pl.data(), g->planes + w0, pl.size() * sizeof(uint2), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(nm.data(), g->nmask + w0, nm.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    static const char nt[4] = {'t', 'c', 'a', 'g'};
    for (int32_t p = start; p < end; ++p) {
        const int64_t w = g->woff[i] + p / 32 - w0;
        const int b = p & 31;
        if ((nm[w] >> b) & 1u) {
            out[p - start] = 'n';
        } else {
            const int code = (int)(((pl[w].y >> b) & 1u) << 1 | ((pl[w].x >> b) & 1u));
            out[p - start] = nt[code];
        }
    }
    return GAC_OK;
}

extern "C" int gac_genome_view(gac_ctx *c, int side, int32_t i, gac_seq_view *v) {
    Genome *g = side_of(c, side);
    if (!g || !g->final || i < 0 || i >= (int32_t)g->sizes.size() || !v)
        return gac_fail(GAC_E_ARG, "gac_genome_view: bad argument");
    v->packed = g->packed(i);
    v->size = g->sizes[i];
    v->n_start = g->nrun_start.data() + g->nrun_off[i];
    v->n_size = g->nrun_size.data() + g->nrun_off[i];
    v->n_count = (int32_t)(g->nrun_off[i + 1] - g->nrun_off[i]);
    return GAC_OK;
}

// The block jobs of gac_score_blocks, 1 M-block chunks on all threads (one
// pair can hold a quarter of a whole-genome run); the first bad block in
// order is kept for the serial message.
struct BlockFill {
    const int64_t *blk_off;
    int64_t np, n;
    const int32_t *bt, *bq, *bs;
    const int64_t *tw, *qw;  // per pair: global base of the target / query sequence
    const int32_t *tsz, *qsz;
    const uint8_t *minus;
    BlockJob *jobs;
    std::atomic<int64_t> next, err_b;
};

static void *block_fill_thread(void *arg) {
    BlockFill *F = (BlockFill *)arg;
    const int64_t chunk = 1 << 20;
    for (int64_t a; (a = F->next.fetch_add(chunk)) < F->n;) {
        const int64_t e = std::min(F->n, a + chunk);
        int64_t p = std::upper_bound(F->blk_off, F->blk_off + F->np + 1, a) - F->blk_off - 1;
        for (int64_t b = a; b < e; ++b) {
            if (b < F->blk_off[0]) {  // (before the first pair: an empty job, as before)
                F->jobs[b] = BlockJob{0, 0, 0, 0};
                continue;
            }
            if (p < 0) p = 0;
            while (b >= F->blk_off[p + 1]) ++p;  // (past empty pairs too)
            const int32_t bt = F->bt[b], bq = F->bq[b], sz = F->bs[b];
            if (bt < 0 || bq < 0 || sz < 0 || (int64_t)bt + sz > F->tsz[p] ||
                (int64_t)bq + sz > F->qsz[p]) {
                int64_t cur = F->err_b.load();
                while ((cur < 0 || b < cur) && !F->err_b.compare_exchange_weak(cur, b)) {
                }
                break;
            }
            BlockJob &j = F->jobs[b];
            j.tp = F->tw[p] + bt;
            j.minus = F->minus[p];
            j.qp = j.minus ? F->qw[p] + (F->qsz[p] - bq) : F->qw[p] + bq;
            j.n = sz;
        }
    }
    return nullptr;
}

extern "C" int gac_score_blocks(gac_ctx *c, int64_t n_pairs, const int32_t *t_seq,
                                const int32_t *q_seq, const uint8_t *q_strand,
                                const int64_t *blk_off, const int32_t *blk_t,
                                const int32_t *blk_q, const int32_t *blk_size, int32_t *score) {
    gac_clear_error();
    if (!c || n_pairs < 0 || (n_pairs && (!t_seq || !q_seq || !q_strand || !blk_off)))
        return gac_fail(GAC_E_ARG, "gac_score_blocks: bad argument");
    if (!c->scoring) return gac_fail(GAC_E_STATE, "gac_score_blocks before gac_set_scoring");
    CTX_LOCK(c);
    if (!c->g[0].final || !c->g[1].final)
        return gac_fail(GAC_E_STATE, "load both genomes before scoring blocks");
    const int64_t n = n_pairs ? blk_off[n_pairs] : 0;
    if (n == 0) return GAC_OK;
    if (!blk_t || !blk_q || !blk_size || !score)
        return gac_fail(GAC_E_ARG, "gac_score_blocks: NULL block array");
    const Genome &T = c->g[0], &Q = c->g[1];
    std::vector<int64_t> tw(n_pairs), qw(n_pairs);
    std::vector<int32_t> tsz(n_pairs), qsz(n_pairs);
    std::vector<uint8_t> minus(n_pairs);
    for (int64_t p = 0; p < n_pairs; ++p) {
        const int32_t ts = t_seq[p], qs = q_seq[p];
        if (ts < 0 || ts >= (int32_t)T.sizes.size() || qs < 0 || qs >= (int32_t)Q.sizes.size())
            return gac_fail(GAC_E_ARG, "gac_score_blocks: pair %lld: bad sequence index",
                            (long long)p);
        if (blk_off[p + 1] < blk_off[p])
            return gac_fail(GAC_E_ARG, "gac_score_blocks: pair %lld: block offsets descend",
                            (long long)p);
        tw[p] = T.woff[ts] * 32, qw[p] = Q.woff[qs] * 32;
        tsz[p] = T.sizes[ts], qsz[p] = Q.sizes[qs];
        minus[p] = q_strand[p] ? 1 : 0;
    }
    // (not value-initialised: every job is written by a fill thread)
    std::unique_ptr<BlockJob[]> jobs(new BlockJob[n]);
    BlockFill F;
    F.blk_off = blk_off, F.np = n_pairs, F.n = n;
    F.bt = blk_t, F.bq = blk_q, F.bs = blk_size;
    F.tw = tw.data(), F.qw = qw.data(), F.tsz = tsz.data(), F.qsz = qsz.data();
    F.minus = minus.data();
    F.jobs = jobs.get();
    F.next = 0;
    F.err_b = -1;
    const int nt = std::max(1, std::min(16, gac_host_threads()));
    gac_run_threads((int)std::min<int64_t>(nt, (n + (1 << 20) - 1) >> 20), block_fill_thread, &F);
    if (F.err_b.load() >= 0) {  // the first bad block in order, as the serial check reports it
        const int64_t b = F.err_b.load();
        const int64_t p = std::upper_bound(blk_off, blk_off + n_pairs + 1, b) - blk_off - 1;
        return gac_fail(GAC_E_ARG, "block %lld (%d %d %d) outside %s/%s", (long long)b, blk_t[b],
                        blk_q[b], blk_size[b], T.names[t_seq[p]].c_str(), Q.names[q_seq[p]].c_str());
    }
    HIPCHK(hipSetDevice(c->device));
    BlockJob *d_jobs = nullptr;
    int32_t *d_out = nullptr;
    HIPCHK(hipMalloc((void **)&d_jobs, n * sizeof(BlockJob)));
    HIPCHK(hipMalloc((void **)&d_out, n * sizeof(int32_t)));
    HIPCHK(hipMemcpyAsync(d_jobs, jobs.get(), n * sizeof(BlockJob), hipMemcpyHostToDevice,
                          c->stream));
    ScoreArgs a;
    memset(&a, 0, sizeof(a));
    a.t_planes = T.planes;
    a.t_nmask = T.nmask;
    a.q_planes = Q.planes;
    a.q_nmask = Q.nmask;
    memcpy(a.coef, c->coef, sizeof(a.coef));
    a.sym = c->sym;
    HIPCHK(launch_blocks(a, d_jobs, n, d_out, c->stream));
    HIPCHK(hipMemcpyAsync(score, d_out, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    hipFree(d_jobs);
    hipFree(d_out);
    return GAC_OK;
}

// ----------------------------------------------------------------- chaining DP
// DpArgs common part: genomes, matrix by code, gap setup
static void dp_base_args(gac_ctx *c, DpArgs &a) {
    memset(&a, 0, sizeof(a));
    a.t_planes = c->g[0].planes;
    a.t_nmask = c->g[0].nmask;
    a.q_planes = c->g[1].planes;
    a.q_nmask = c->g[1].nmask;
    a.gap = c->gap;
    a.small_tab = c->d_small;
    a.gap_tab = c->d_gap_tab;
    a.gap_len = c->gap_len;
    for (int q = 0; q < 4; ++q)
        for (int t = 0; t < 4; ++t) a.m16[q * 4 + t] = c->mat[acgt_of_code(q) * 4 + acgt_of_code(t)];
}

// global base index of a pair's target start / query start ('-': ~(start + qSize))
static int pair_bases(gac_ctx *c, int32_t ts, int32_t qs, uint8_t minus, int64_t &tb,
                      int64_t &qb) {
    const Genome &T = c->g[0], &Q = c->g[1];
    if (ts < 0 || ts >= (int32_t)T.sizes.size() || qs < 0 || qs >= (int32_t)Q.sizes.size())
        return gac_fail(GAC_E_ARG, "bad sequence index (%d, %d)", ts, qs);
    tb = T.woff[ts] * 32;
    qb = minus ? ~(Q.woff[qs] * 32 + Q.sizes[qs]) : Q.woff[qs] * 32;
    return GAC_OK;
}

template <class T>
static int dev_upload(gac_ctx *c, T **d, const void *h, size_t n) {
    *d = nullptr;
    if (n == 0) return GAC_OK;
    HIPCHK(hipMalloc((void **)d, n * sizeof(T)));
    if (h) HIPCHK(hipMemcpyAsync(*d, h, n * sizeof(T), hipMemcpyHostToDevice, c->stream));
    return GAC_OK;
}

// the fast DP's waves per pair: k_dp_spec with 16 (GAC_DP_WAVES=4/8/16; 1:
// k_dp_fast, one wave per pair -- 7.2x slower on the C4-shaped set, r06spec7)
static int dp_waves() {
    static int waves = -1;
    if (waves < 0) {
        const char *wv = getenv("GAC_DP_WAVES");
        int w = wv && *wv ? atoi(wv) : 16;
        waves = (w == 4 || w == 8 || w == 16) ? w : 1;
    }
    return waves;
}

// k_dp_fast (fast) or k_dp over a.n_pairs pairs; GAC_DP_PROF: k_dp_fast's
// per-phase cycle counters, summed over pairs, to stderr
static hipError_t dp_launch(gac_ctx *c, DpArgs &a, int grid, bool fast) {
    unsigned long long *d_prof = nullptr;
    hipError_t e = hipSuccess;
    const char *dpprof = getenv("GAC_DP_PROF");
    if (fast && dpprof && *dpprof && *dpprof != '0' &&
        (e = hipMalloc(&d_prof, kDpProf * sizeof(unsigned long long))) == hipSuccess)
        e = hipMemsetAsync(d_prof, 0, kDpProf * sizeof(unsigned long long), c->stream);
    a.prof = d_prof;
    const double tk0 = wall_s();
    const int waves = dp_waves();
    // (k_dp_spec's watchdog flag: the caller's, or one of our own)
    int32_t *d_err_own = nullptr;
    if (e == hipSuccess && fast && waves > 1 && !a.err &&
        (e = hipMalloc(&d_err_own, sizeof(int32_t))) == hipSuccess &&
        (e = hipMemsetAsync(d_err_own, 0, sizeof(int32_t), c->stream)) == hipSuccess)
        a.err = d_err_own;
    if (e == hipSuccess)
        e = !fast ? launch_dp(a, grid, c->stream)
                  : (waves > 1 ? launch_dp_spec(a, grid, waves, c->stream) : launch_dp_fast(a, grid, c->stream));
    if (d_err_own) {
        int32_t h = 0;
        if (e == hipSuccess) e = hipMemcpyAsync(&h, d_err_own, sizeof(h), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess && h) e = hipErrorLaunchTimeOut;  // (the in-order commit stalled)
        hipFree(d_err_own);
        a.err = nullptr;
    }
    if (d_prof && e == hipSuccess) {
        unsigned long long pv[kDpProf];
        e = hipMemcpyAsync(pv, d_prof, sizeof(pv), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) {
            const double secs = wall_s() - tk0, L = pv[kPfLeaves] ? (double)pv[kPfLeaves] : 1.0;
            fprintf(stderr,
                    "[gac_chain_dp] %s %.3f s, %llu pairs, %llu leaves, %llu fallbacks; per leaf: "
                    "%.2f windows, %.3f fallback windows, %.3f windows with an overlapping candidate, "
                    "%.2f overlap checks; cycles per leaf: load %.0f seed %.0f walk %.0f "
                    "(node loads + bounds %.0f) anomalies %.0f fallback %.0f commit %.0f; next windows: %.2f per leaf, "
                    "%.3f contiguous\n",
                    waves > 1 ? "k_dp_spec" : "k_dp_fast", secs, (unsigned long long)a.n_pairs,
                    pv[kPfLeaves], pv[kPfFallbacks],
                    pv[kPfWindows] / L, pv[kPfFbWindows] / L, pv[kPfXoverWin] / L, pv[kPfOvChecks] / L,
                    pv[kPfCycLoad] / L, pv[kPfCycSeed] / L, pv[kPfCycWalk] / L, pv[kPfCycXover] / L,
                    pv[kPfCycAnom] / L, pv[kPfCycFb] / L, pv[kPfCycCommit] / L, pv[kPfNextWin] / L,
                    pv[kPfNextWin] ? (double)pv[kPfNextSeq] / pv[kPfNextWin] : 0.0);
            if (waves > 1)
                fprintf(stderr, "[gac_chain_dp] k_dp_spec, %d waves per pair: per leaf %.0f cycles searching, "
                        "%.0f waiting for its turn, in order: %.0f the leaves since the snapshot, %.0f "
                        "anomalies, %.0f commit; then %.0f publishing; %.3f of the leaves "
                        "searched beside earlier ones\n", waves, pv[kPfCycWalk] / L, pv[kPfCycLoad] / L,
                        pv[kPfCycSeed] / L, pv[kPfCycAnom] / L, pv[kPfCycCommit] / L, pv[kPfCycFb] / L,
                        pv[kPfXoverWin] / L);
        }
        hipFree(d_prof);
        a.prof = nullptr;
    }
    return e;
}

extern "C" int gac_chain_dp(gac_ctx *c, int64_t n_pairs, const int32_t *t_seq, const int32_t *q_seq,
                            const uint8_t *q_strand, const int64_t *node_off,
                            const int32_t *node_a, const int32_t *node_b, const int64_t *leaf_off,
                            const int32_t *leaf, const int32_t *leaf_score,
                            const int32_t *leaf_node, const int64_t *path_off,
                            const int32_t *path, int64_t *total, int32_t *pred) {
    return gac_chain_dp_ex(c, n_pairs, t_seq, q_seq, q_strand, node_off, node_a, node_b, leaf_off,
                           leaf, leaf_score, leaf_node, path_off, path, nullptr, nullptr, 0, 0,
                           total, pred);
}

// gac_chain_dp with the exact fast DP (k_dp_fast) when ov_off is given: the
// linear gap-cost minorant lin_k / 1024, the smallest matrix entry, and each
// leaf's overlapping candidates (leaf nodes; -1 = too many to list)
extern "C" int gac_chain_dp_ex(gac_ctx *c, int64_t n_pairs, const int32_t *t_seq,
                               const int32_t *q_seq, const uint8_t *q_strand,
                               const int64_t *node_off, const int32_t *node_a,
                               const int32_t *node_b, const int64_t *leaf_off,
                               const int32_t *leaf, const int32_t *leaf_score,
                               const int32_t *leaf_node, const int64_t *path_off,
                               const int32_t *path, const int64_t *ov_off, const int32_t *ov,
                               int64_t lin_k, int32_t min_entry, int64_t *total, int32_t *pred) {
    gac_clear_error();
    if (!c || n_pairs < 0 ||
        (n_pairs && (!t_seq || !q_seq || !q_strand || !node_off || !leaf_off || !path_off)))
        return gac_fail(GAC_E_ARG, "gac_chain_dp: bad argument");
    if (!c->scoring) return gac_fail(GAC_E_STATE, "gac_chain_dp before gac_set_scoring");
    CTX_LOCK(c);
    if (!c->g[0].final || !c->g[1].final)
        return gac_fail(GAC_E_STATE, "load both genomes before gac_chain_dp");
    if (n_pairs == 0) return GAC_OK;
    const int64_t nn = node_off[n_pairs], nl = leaf_off[n_pairs], np_ = path_off[nl];
    if (nl == 0) return GAC_OK;
    if (!node_a || !node_b || !leaf || !leaf_score || !leaf_node || !path || !total || !pred)
        return gac_fail(GAC_E_ARG, "gac_chain_dp: NULL array");
    std::vector<DpPair> pairs(n_pairs);
    std::vector<long long> tot0(nn, 0);
    for (int64_t p = 0; p < n_pairs; ++p) {
        DpPair &P = pairs[p];
        int rc = pair_bases(c, t_seq[p], q_seq[p], q_strand[p], P.tbase, P.qbase);
        if (rc != GAC_OK) return rc;
        const int64_t n_nodes = node_off[p + 1] - node_off[p], n_leaves = leaf_off[p + 1] - leaf_off[p];
        if (n_nodes < 0 || n_nodes > 0x7fffffff || n_leaves < 0 || (n_leaves > 0 && n_nodes < 1))
            return gac_fail(GAC_E_ARG, "gac_chain_dp: pair %lld: bad tree size", (long long)p);
        P.node_off = node_off[p];
        P.leaf_off = leaf_off[p];
        P.n_nodes = (int32_t)n_nodes;
        P.n_leaves = (int32_t)n_leaves;
        for (int64_t i = leaf_off[p]; i < leaf_off[p + 1]; ++i) {
            const int32_t v = leaf_node[i];
            if (v < 0 || v >= n_nodes || node_b[2 * (node_off[p] + v) + 1] != ~(int32_t)(i - leaf_off[p]))
                return gac_fail(GAC_E_ARG, "gac_chain_dp: leaf %lld: bad node", (long long)i);
            tot0[node_off[p] + v] = leaf_score[i];
        }
    }
    // a kernel reading past its pair would fault: check the structure first
    for (int64_t p = 0; p < n_pairs; ++p) {
        const int64_t o = node_off[p];
        const int32_t n = pairs[p].n_nodes;
        for (int32_t v = 0; v < n; ++v) {
            const int32_t end = node_b[2 * (o + v)], info = node_b[2 * (o + v) + 1];
            const int32_t lo = node_a[4 * (o + v) + 3];
            if (end <= v || end > n || (info >= 0 && (info > 1 || lo <= v + 1 || lo >= end)))
                return gac_fail(GAC_E_ARG, "gac_chain_dp: pair %lld node %d: bad links", (long long)p, v);
        }
    }
    for (int64_t p = 0; p < n_pairs; ++p)
        for (int64_t i = leaf_off[p]; i < leaf_off[p + 1]; ++i)
            for (int64_t k = path_off[i]; k < path_off[i + 1]; ++k)
                if (path[k] < 0 || path[k] >= pairs[p].n_nodes)
                    return gac_fail(GAC_E_ARG, "gac_chain_dp: leaf %lld: bad path node", (long long)i);
    const bool fast = ov_off != nullptr;
    const int64_t nov = fast ? ov_off[nl] : 0;
    if (fast) {
        if (ov_off[0] != 0 || (nov && !ov) || lin_k < 0)
            return gac_fail(GAC_E_ARG, "gac_chain_dp: bad overlap lists");
        for (int64_t p = 0; p < n_pairs; ++p)
            for (int64_t i = leaf_off[p]; i < leaf_off[p + 1]; ++i) {
                if (ov_off[i + 1] < ov_off[i])
                    return gac_fail(GAC_E_ARG, "gac_chain_dp: leaf %lld: bad overlap offsets", (long long)i);
                for (int64_t k = ov_off[i]; k < ov_off[i + 1]; ++k) {
                    const int32_t v = ov[k];
                    if (v != -1 && (v < 0 || v >= pairs[p].n_nodes ||
                                    node_b[2 * (node_off[p] + v) + 1] >= 0))
                        return gac_fail(GAC_E_ARG, "gac_chain_dp: leaf %lld: bad overlap node",
                                        (long long)i);
                }
            }
    }
    HIPCHK(hipSetDevice(c->device));
    DpArgs a;
    dp_base_args(c, a);
    a.n_pairs = n_pairs;
    DpPair *d_pairs = nullptr;
    int4 *d_na = nullptr, *d_lf = nullptr;
    int2 *d_nb = nullptr;
    long long *d_ms = nullptr, *d_tot = nullptr, *d_total = nullptr;
    int32_t *d_score = nullptr, *d_node = nullptr, *d_path = nullptr, *d_pred = nullptr;
    int64_t *d_poff = nullptr;
    long long *d_nw = nullptr;
    int64_t *d_ovoff = nullptr;
    int32_t *d_ov = nullptr;
    int rc = GAC_OK;
    if (fast) {
        std::vector<long long> nw0(nn, INT64_MIN / 4);
        if ((rc = dev_upload(c, &d_nw, nw0.data(), nn)) != GAC_OK ||
            (rc = dev_upload(c, &d_ovoff, ov_off, nl + 1)) != GAC_OK ||
            (rc = dev_upload(c, &d_ov, nov ? ov : nullptr, nov ? nov : 1)) != GAC_OK) {
            hipStreamSynchronize(c->stream);
            hipFree(d_nw);
            hipFree(d_ovoff);
            hipFree(d_ov);
            return rc;
        }
        hipStreamSynchronize(c->stream);  // (nw0 leaves scope)
    }
    if ((rc = dev_upload(c, &d_pairs, pairs.data(), n_pairs)) == GAC_OK &&
        (rc = dev_upload(c, &d_na, node_a, nn)) == GAC_OK &&
        (rc = dev_upload(c, &d_nb, node_b, nn)) == GAC_OK &&
        (rc = dev_upload(c, &d_ms, nullptr, nn)) == GAC_OK &&
        (rc = dev_upload(c, &d_tot, tot0.data(), nn)) == GAC_OK &&
        (rc = dev_upload(c, &d_lf, leaf, nl)) == GAC_OK &&
        (rc = dev_upload(c, &d_score, leaf_score, nl)) == GAC_OK &&
        (rc = dev_upload(c, &d_node, leaf_node, nl)) == GAC_OK &&
        (rc = dev_upload(c, &d_poff, path_off, nl + 1)) == GAC_OK &&
        (rc = dev_upload(c, &d_path, path, np_ ? np_ : 1)) == GAC_OK &&
        (rc = dev_upload(c, &d_total, nullptr, nl)) == GAC_OK &&
        (rc = dev_upload(c, &d_pred, nullptr, nl)) == GAC_OK) {
        hipError_t e = hipMemsetAsync(d_ms, 0, nn * sizeof(long long), c->stream);
        a.pairs = d_pairs;
        a.nd_ms = d_ms;
        a.nd_tot = d_tot;
        a.nd_a = d_na;
        a.nd_b = d_nb;
        a.lf = d_lf;
        a.lf_score = d_score;
        a.lf_node = d_node;
        a.path_off = d_poff;
        a.path = d_path;
        a.lf_total = d_total;
        a.lf_pred = d_pred;
        a.nd_nw = d_nw;
        a.ov_off = d_ovoff;
        a.ov = d_ov;
        a.lin_k = lin_k;
        a.min_entry = min_entry;
        // one wave per pair, every pair resident at once (largest first is
        // the caller's order; the grid covers them all)
        const int grid = (int)std::min<int64_t>(n_pairs, 1 << 20);
        if (e == hipSuccess) e = dp_launch(c, a, grid, fast);
        if (e == hipSuccess)
            e = hipMemcpyAsync(total, d_total, nl * sizeof(long long), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(pred, d_pred, nl * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = gac_fail(GAC_E_HIP, "gac_chain_dp: %s", hipGetErrorString(e));
    }
    hipStreamSynchronize(c->stream);
    hipFree(d_pairs);
    hipFree(d_na);
    hipFree(d_nb);
    hipFree(d_ms);
    hipFree(d_tot);
    hipFree(d_lf);
    hipFree(d_score);
    hipFree(d_node);
    hipFree(d_poff);
    hipFree(d_path);
    hipFree(d_total);
    hipFree(d_pred);
    hipFree(d_nw);
    hipFree(d_ovoff);
    hipFree(d_ov);
    return rc;
}

// device allocations of one call, freed together (after a stream sync)
namespace {
struct DevBufs {
    std::vector<void *> p;
    hipError_t e = hipSuccess;
    template <class T>
    T *take(int64_t n) {
        void *q = nullptr;
        if (e == hipSuccess) e = hipMalloc(&q, (size_t)(n > 0 ? n : 1) * sizeof(T));
        if (q) p.push_back(q);
        return (T *)q;
    }
    ~DevBufs() {
        for (void *q : p) hipFree(q);
    }
};
}  // namespace

// the device build's set-up shared by gac_chain_dp_blocks and gac_kd_trees:
// uploads, leaves in target order and leaf offsets (leaf_off, host), node
// offsets, every array of the build; u.t.L == 0: no leaves (nothing else set)
namespace {
struct DtSetup {
    DtTree t;
    std::vector<DpPair> pairs;
    std::vector<int64_t> node_off;
    int levels = 0;
    int64_t *d_leaf_off = nullptr;
    int32_t *d_err = nullptr;
    long long *d_total = nullptr, *d_lf_total = nullptr;
    int32_t *d_pred = nullptr, *d_lf_pred = nullptr, *d_out_tord = nullptr;
    DpPair *d_pairs = nullptr;
    double t0 = 0, t1 = 0;
};
}  // namespace

static int dt_setup(gac_ctx *c, const char *who, int64_t P, const int32_t *t_seq,
                    const int32_t *q_seq, const uint8_t *q_strand, const int64_t *blk_off,
                    const int32_t *box, const int32_t *score, int fast, int32_t ov_cap,
                    int64_t *leaf_off, DevBufs &M, DtSetup &u) {
    const int64_t B = blk_off[P];
    u.t0 = wall_s();
    const bool timing = getenv("GAC_TIMING") != nullptr;
    (void)timing;
    std::vector<DpPair> &pairs = u.pairs;
    pairs.resize(P);
    std::vector<int2> sizes(P);
    for (int64_t p = 0; p < P; ++p) {
        int rc = pair_bases(c, t_seq[p], q_seq[p], q_strand[p], pairs[p].tbase, pairs[p].qbase);
        if (rc != GAC_OK) return rc;
        sizes[p] = make_int2(c->g[0].sizes[t_seq[p]], c->g[1].sizes[q_seq[p]]);
    }
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    DtTree &t = u.t;
    memset(&t, 0, sizeof(t));
    t.P = P;
    t.B = B;
    t.fast = fast ? 1 : 0;
    t.ov_cap = ov_cap;
    int bits = 0;
    while ((1LL << bits) <= P) ++bits;
    t.end_bit = 31 + bits;
    int64_t *d_blk_off = M.take<int64_t>(P + 1);
    int2 *d_sizes = M.take<int2>(P);
    int4 *d_box = M.take<int4>(B);
    int32_t *d_score = M.take<int32_t>(B);
    unsigned long long *d_keys = M.take<unsigned long long>(2 * B);
    int32_t *d_vals = M.take<int32_t>(2 * B);
    int64_t *d_leaf_off = u.d_leaf_off = M.take<int64_t>(P + 1);
    int32_t *d_err = u.d_err = M.take<int32_t>(1);
    t.tpos = M.take<int32_t>(B);
    t.qpos = M.take<int32_t>(B);
    t.posd = M.take<int32_t>(B);
    u.d_total = M.take<long long>(B);
    u.d_pred = M.take<int32_t>(B);
    if (M.e != hipSuccess)
        return gac_fail(GAC_E_HIP, "%s: hipMalloc: %s", who, hipGetErrorString(M.e));
    size_t b_sort = 0;
    HIPCHK(dt_sort_pairs(nullptr, b_sort, d_keys, d_keys + B, d_vals, d_vals + B, B, t.end_bit, s));
    void *d_tmp = M.take<uint8_t>((int64_t)b_sort);
    HIPCHK(M.e);
    HIPCHK(hipMemcpyAsync(d_blk_off, blk_off, (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_sizes, sizes.data(), P * sizeof(int2), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_box, box, B * sizeof(int4), hipMemcpyHostToDevice, s));
    if (score)
        HIPCHK(hipMemcpyAsync(d_score, score, B * sizeof(int32_t), hipMemcpyHostToDevice, s));
    else
        HIPCHK(hipMemsetAsync(d_score, 0, B * sizeof(int32_t), s));
    HIPCHK(hipMemsetAsync(d_err, 0, sizeof(int32_t), s));
    // ---- leaves in target order, per-pair leaf offsets
    HIPCHK(launch_dt_keys(P, B, d_blk_off, d_sizes, d_box, d_keys, d_vals, d_err, s));
    HIPCHK(dt_sort_pairs(d_tmp, b_sort, d_keys, d_keys + B, d_vals, d_vals + B, B, t.end_bit, s));
    HIPCHK(launch_dt_leaf_off(P, B, d_keys + B, d_leaf_off, s));
    int32_t h_err = 0;
    HIPCHK(hipMemcpyAsync(leaf_off, d_leaf_off, (P + 1) * sizeof(int64_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&h_err, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const double t1 = wall_s();
    (void)t1;
    if (h_err & 1) {  // the first bad block, as a serial check reports it
        for (int64_t p = 0; p < P; ++p)
            for (int64_t g = blk_off[p]; g < blk_off[p + 1]; ++g) {
                const int32_t *b = box + 4 * g;
                if (b[0] < 0 || b[0] > b[1] || b[1] > sizes[p].y || b[2] < 0 || b[2] > b[3] ||
                    b[3] > sizes[p].x)
                    return gac_fail(GAC_E_ARG, "%s: pair %lld block %lld (%d-%d, %d-%d) "
                                    "outside its sequences", who, (long long)p, (long long)(g - blk_off[p]),
                                    b[0], b[1], b[2], b[3]);
            }
        return gac_fail(GAC_E_ARG, "%s: a block outside its sequences", who);
    }
    const int64_t L = leaf_off[P];
    u.t1 = t1;
    if (L == 0) return GAC_OK;
    std::vector<int64_t> &node_off = u.node_off;
    node_off.resize(P + 1);
    int64_t maxnl = 0;
    node_off[0] = 0;
    for (int64_t p = 0; p < P; ++p) {
        const int64_t nl = leaf_off[p + 1] - leaf_off[p];
        maxnl = std::max(maxnl, nl);
        node_off[p + 1] = node_off[p] + (nl ? 2 * nl - 1 : 0);
        pairs[p].node_off = node_off[p];
        pairs[p].leaf_off = leaf_off[p];
        pairs[p].n_nodes = (int32_t)(node_off[p + 1] - node_off[p]);
        pairs[p].n_leaves = (int32_t)nl;
    }
    const int64_t N = node_off[P];
    int &levels = u.levels;
    levels = 0;
    for (int64_t n = maxnl; n > 1; n -= n / 2) ++levels;
    t.L = L;
    t.N = N;
    t.blk_off = d_blk_off;
    t.box = d_box;
    t.score = d_score;
    t.keys = d_keys + B;
    t.tord = d_vals + B;
    t.leaf_off = d_leaf_off;
    int64_t *d_node_off = M.take<int64_t>(P + 1);
    t.node_off = d_node_off;
    t.pidx = M.take<int32_t>(L);
    t.key2 = M.take<unsigned long long>(2 * L);
    t.val2 = M.take<int32_t>(2 * L);
    t.ql = M.take<int32_t>(L);
    t.tl = M.take<int32_t>(L);
    t.spare = M.take<int32_t>(L);
    t.sstart = M.take<int32_t>(L);
    t.slen = M.take<int32_t>(L);
    t.snode = M.take<int32_t>(L);
    t.flag = M.take<int32_t>(L);
    t.excl = M.take<int32_t>(L);
    t.ndep = M.take<int32_t>(N);
    t.ndl = M.take<int32_t>(N);
    t.qbox = M.take<int4>(L);
    t.qtp = M.take<int32_t>(L);
    t.msz = M.take<int32_t>(P);
    t.over = M.take<uint8_t>(L);
    t.pcnt = M.take<long long>(L + 1);
    t.ocnt = M.take<long long>(L + 1);
    t.err = d_err;
    t.na = M.take<int4>(N);
    t.nb = M.take<int2>(N);
    t.tot = M.take<long long>(N);
    t.ms = M.take<long long>(N);
    t.nw = M.take<long long>(N);
    t.lf = M.take<int4>(L);
    t.lsc = M.take<int32_t>(L);
    t.lnode = M.take<int32_t>(L);
    t.poff = M.take<long long>(L + 1);
    t.ooff = M.take<long long>(L + 1);
    u.d_lf_total = M.take<long long>(L);
    u.d_lf_pred = M.take<int32_t>(L);
    u.d_out_tord = M.take<int32_t>(L);
    DpPair *d_pairs = u.d_pairs = M.take<DpPair>(P);
    if (M.e != hipSuccess)
        return gac_fail(GAC_E_HIP, "%s: hipMalloc: %s", who, hipGetErrorString(M.e));
    size_t need = b_sort, b = 0;
    HIPCHK(dt_sort_pairs(nullptr, b, t.key2, t.key2 + L, t.val2, t.val2 + L, L, t.end_bit, s));
    need = std::max(need, b);
    HIPCHK(dt_scan32(nullptr, b, t.flag, t.excl, L, s));
    need = std::max(need, b);
    HIPCHK(dt_scan64(nullptr, b, t.pcnt, t.poff, L + 1, s));
    need = std::max(need, b);
    t.tmp = need > b_sort ? M.take<uint8_t>((int64_t)need) : d_tmp;
    t.tmp_bytes = need;
    HIPCHK(M.e);
    HIPCHK(hipMemcpyAsync(d_node_off, node_off.data(), (P + 1) * sizeof(int64_t),
                          hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_pairs, pairs.data(), P * sizeof(DpPair), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(t.pcnt, 0, (L + 1) * sizeof(long long), s));
    HIPCHK(hipMemsetAsync(t.ocnt, 0, (L + 1) * sizeof(long long), s));
    return GAC_OK;
}

// chainBlocks' DP for n_pairs pairs from their blocks: the leaves, kd-trees,
// update paths and overlap lists built on the device (gac_dptree.hip), then
// k_dp_fast (fast) or k_dp; see include/gachain.h
extern "C" int gac_chain_dp_blocks(gac_ctx *c, int64_t n_pairs, const int32_t *t_seq,
                                   const int32_t *q_seq, const uint8_t *q_strand,
                                   const int64_t *blk_off, const int32_t *box, const int32_t *score,
                                   int fast, int64_t lin_k, int32_t min_entry, int32_t ov_cap,
                                   int64_t *leaf_off, int32_t *tord, int64_t *total, int32_t *pred) {
    gac_clear_error();
    if (!c || n_pairs < 0 || (n_pairs && (!t_seq || !q_seq || !q_strand || !blk_off || !leaf_off)))
        return gac_fail(GAC_E_ARG, "gac_chain_dp_blocks: bad argument");
    if (!c->scoring) return gac_fail(GAC_E_STATE, "gac_chain_dp_blocks before gac_set_scoring");
    CTX_LOCK(c);
    if (!c->g[0].final || !c->g[1].final)
        return gac_fail(GAC_E_STATE, "load both genomes before gac_chain_dp_blocks");
    if (n_pairs == 0) return GAC_OK;
    if (n_pairs >= (1LL << 30)) return gac_fail(GAC_E_ARG, "gac_chain_dp_blocks: too many pairs");
    const int64_t P = n_pairs, B = blk_off[P];
    if (blk_off[0] != 0 || B < 0 || B > 0x7fffffffLL)
        return gac_fail(GAC_E_ARG, "gac_chain_dp_blocks: bad block offsets");
    for (int64_t p = 0; p < P; ++p)
        if (blk_off[p + 1] < blk_off[p])
            return gac_fail(GAC_E_ARG, "gac_chain_dp_blocks: pair %lld: block offsets descend",
                            (long long)p);
    if (B && (!box || !score || !tord || !total || !pred))
        return gac_fail(GAC_E_ARG, "gac_chain_dp_blocks: NULL array");
    if (fast && lin_k < 0) return gac_fail(GAC_E_ARG, "gac_chain_dp_blocks: bad lin_k");
    if (B == 0) {
        for (int64_t p = 0; p <= P; ++p) leaf_off[p] = 0;
        return GAC_OK;
    }
    const bool timing = getenv("GAC_TIMING") != nullptr;
    DevBufs M;
    DtSetup u;
    int rc0 = dt_setup(c, "gac_chain_dp_blocks", P, t_seq, q_seq, q_strand, blk_off, box, score, fast,
                       ov_cap, leaf_off, M, u);
    if (rc0 != GAC_OK) return rc0;
    const double t0 = u.t0, t1 = u.t1;
    if (u.t.L == 0) {
        for (int64_t g = 0; g < B; ++g) {
            total[g] = score[g];
            pred[g] = -1;
        }
        return GAC_OK;
    }
    DtTree &t = u.t;
    hipStream_t s = c->stream;
    const int64_t L = t.L;
    const int levels = u.levels;
    int32_t *d_err = u.d_err;
    long long *d_total = u.d_total, *d_lf_total = u.d_lf_total;
    int32_t *d_pred = u.d_pred, *d_lf_pred = u.d_lf_pred, *d_out_tord = u.d_out_tord;
    DpPair *d_pairs = u.d_pairs;
    int64_t *d_leaf_off = u.d_leaf_off;
    const int64_t N = t.N;
    int32_t h_err = 0;
    // ---- query order, the trees, path and overlap counts
    HIPCHK(launch_dt_tree(t, levels, s));
    long long n_path = 0, n_ov = 0;
    HIPCHK(hipMemcpyAsync(&n_path, t.poff + L, sizeof(long long), hipMemcpyDeviceToHost, s));
    if (fast) HIPCHK(hipMemcpyAsync(&n_ov, t.ooff + L, sizeof(long long), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&h_err, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h_err)
        return gac_fail(GAC_E_HIP, "gac_chain_dp_blocks: device tree build failed (%d)", h_err);
    int32_t *d_path = M.take<int32_t>(n_path);
    int32_t *d_ov = M.take<int32_t>(n_ov);
    if (M.e != hipSuccess)
        return gac_fail(GAC_E_HIP, "gac_chain_dp_blocks: hipMalloc: %s", hipGetErrorString(M.e));
    HIPCHK(launch_dt_lists(t, d_path, d_ov, s));
    HIPCHK(hipMemcpyAsync(&h_err, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h_err)
        return gac_fail(GAC_E_HIP, "gac_chain_dp_blocks: device path build failed (%d)", h_err);
    const double t2 = wall_s();
    // ---- the DP
    DpArgs a;
    dp_base_args(c, a);
    a.n_pairs = P;
    a.pairs = d_pairs;
    a.nd_ms = t.ms;
    a.nd_tot = t.tot;
    a.nd_a = t.na;
    a.nd_b = t.nb;
    a.lf = t.lf;
    a.lf_score = t.lsc;
    a.lf_node = t.lnode;
    a.path_off = (const int64_t *)t.poff;
    a.path = d_path;
    a.lf_total = d_lf_total;
    a.lf_pred = d_lf_pred;
    a.nd_nw = fast ? t.nw : nullptr;
    a.ov_off = fast ? (const int64_t *)t.ooff : nullptr;
    a.ov = fast ? d_ov : nullptr;
    a.lin_k = lin_k;
    a.min_entry = min_entry;
    a.err = d_err;
    const int grid = (int)std::min<int64_t>(P, 1 << 20);
    HIPCHK(dp_launch(c, a, grid, fast != 0));
    {
        // the DP runs for seconds beside the host's own DP threads: wait
        // without spinning a core (hipStreamSynchronize may busy-wait)
        hipEvent_t done;
        HIPCHK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
        hipError_t e = hipEventRecord(done, s);
        while (e == hipSuccess && (e = hipEventQuery(done)) == hipErrorNotReady) {
            const struct timespec nap = {0, 500000};
            nanosleep(&nap, nullptr);
            e = hipSuccess;
        }
        hipEventDestroy(done);
        HIPCHK(e);
    }
    const double t3 = wall_s();
    if (const char *dd = getenv("GAC_DT_DUMP")) {  // (debug: the built arrays, raw)
        auto dump = [&](const char *name, const void *d, size_t bytes) {
            std::vector<char> h(bytes);
            if (hipMemcpy(h.data(), d, bytes, hipMemcpyDeviceToHost) != hipSuccess) return;
            std::string f = std::string(dd) + "/" + name;
            if (FILE *o = fopen(f.c_str(), "wb")) {
                fwrite(h.data(), 1, bytes, o);
                fclose(o);
            }
        };
        dump("leaf_off", d_leaf_off, (P + 1) * 8);
        dump("lf", t.lf, L * 16);
        dump("lnode", t.lnode, L * 4);
        dump("na", t.na, N * 16);
        dump("nb", t.nb, N * 8);
        dump("poff", t.poff, (L + 1) * 8);
        dump("path", d_path, n_path * 4);
        if (fast) dump("ooff", t.ooff, (L + 1) * 8);
        if (fast) dump("ov", d_ov, n_ov * 4);
        dump("lf_total", d_lf_total, L * 8);
        dump("lf_pred", d_lf_pred, L * 4);
    }
    HIPCHK(launch_dt_out(t, d_lf_total, d_lf_pred, d_out_tord, d_total, d_pred, s));
    HIPCHK(hipMemcpyAsync(tord, d_out_tord, L * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(total, d_total, B * sizeof(long long), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(pred, d_pred, B * sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&h_err, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h_err)
        return gac_fail(GAC_E_HIP, "gac_chain_dp_blocks: %s (%d)",
                        (h_err & 32) ? "the DP's in-order commit stalled" : "a predecessor is not a leaf",
                        h_err);
    if (timing)
        fprintf(stderr,
                "[gac_chain_dp_blocks] %lld pairs, %lld blocks, %lld leaves, %d levels, %lld path "
                "nodes, %lld overlap entries: upload + leaves %.3f s, trees + paths + overlaps %.3f s, "
                "%s %.3f s, results %.3f s\n",
                (long long)P, (long long)B, (long long)L, levels, n_path, n_ov, t1 - t0, t2 - t1,
                !fast ? "k_dp" : (dp_waves() > 1 ? "k_dp_spec" : "k_dp_fast"), t3 - t2, wall_s() - t3);
    return GAC_OK;
}

// kdTreeMake for n_pairs pairs on the device (gac_dptree.hip's build), out
// in the host DP's layout, per pair into the caller's buffers; see
// include/gachain.h
extern "C" int gac_kd_trees(gac_ctx *c, int64_t n_pairs, const int32_t *t_seq, const int32_t *q_seq,
                            const uint8_t *q_strand, const int64_t *blk_off, const int32_t *box,
                            int64_t *leaf_off, int32_t *const *tord, int32_t *const *qord,
                            int32_t *const *lnode, int32_t *const *nodes) {
    gac_clear_error();
    if (!c || n_pairs < 0 || (n_pairs && (!t_seq || !q_seq || !q_strand || !blk_off || !leaf_off)))
        return gac_fail(GAC_E_ARG, "gac_kd_trees: bad argument");
    CTX_LOCK(c);
    if (!c->g[0].final || !c->g[1].final)
        return gac_fail(GAC_E_STATE, "load both genomes before gac_kd_trees");
    if (n_pairs == 0) return GAC_OK;
    if (n_pairs >= (1LL << 30)) return gac_fail(GAC_E_ARG, "gac_kd_trees: too many pairs");
    const int64_t P = n_pairs, B = blk_off[P];
    if (blk_off[0] != 0 || B < 0 || B > 0x7fffffffLL)
        return gac_fail(GAC_E_ARG, "gac_kd_trees: bad block offsets");
    for (int64_t p = 0; p < P; ++p)
        if (blk_off[p + 1] < blk_off[p])
            return gac_fail(GAC_E_ARG, "gac_kd_trees: pair %lld: block offsets descend", (long long)p);
    if (B && (!box || !tord || !qord || !lnode || !nodes))
        return gac_fail(GAC_E_ARG, "gac_kd_trees: NULL array");
    if (B == 0) {
        for (int64_t p = 0; p <= P; ++p) leaf_off[p] = 0;
        return GAC_OK;
    }
    const double t0 = wall_s();
    DevBufs M;
    DtSetup u;
    int rc = dt_setup(c, "gac_kd_trees", P, t_seq, q_seq, q_strand, blk_off, box, nullptr, 0, 0,
                      leaf_off, M, u);
    if (rc != GAC_OK) return rc;
    hipStream_t s = c->stream;
    DtTree &t = u.t;
    if (t.L == 0) {
        for (int64_t p = 0; p < P; ++p)
            for (int64_t g = 0; g < blk_off[p + 1] - blk_off[p]; ++g) lnode[p][g] = -1;
        return GAC_OK;
    }
    int32_t *d_nodes = M.take<int32_t>(6 * t.N);
    int32_t *d_qord = M.take<int32_t>(t.L);
    int32_t *d_lnode_blk = M.take<int32_t>(B);
    if (M.e != hipSuccess)
        return gac_fail(GAC_E_HIP, "gac_kd_trees: hipMalloc: %s", hipGetErrorString(M.e));
    HIPCHK(launch_dt_build(t, u.levels, s));
    HIPCHK(launch_dt_host(t, d_nodes, u.d_out_tord, d_qord, d_lnode_blk, s));
    int32_t h_err = 0;
    HIPCHK(hipMemcpyAsync(&h_err, u.d_err, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (h_err) return gac_fail(GAC_E_HIP, "gac_kd_trees: device tree build failed (%d)", h_err);
    const double t1 = wall_s();
    for (int64_t p = 0; p < P; ++p) {
        const int64_t nl = leaf_off[p + 1] - leaf_off[p], nb = blk_off[p + 1] - blk_off[p];
        if (nl) {
            HIPCHK(hipMemcpyAsync(tord[p], u.d_out_tord + leaf_off[p], nl * sizeof(int32_t),
                                  hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(qord[p], d_qord + leaf_off[p], nl * sizeof(int32_t),
                                  hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(nodes[p], d_nodes + 6 * u.node_off[p],
                                  (2 * nl - 1) * 6 * sizeof(int32_t), hipMemcpyDeviceToHost, s));
        }
        if (nb)
            HIPCHK(hipMemcpyAsync(lnode[p], d_lnode_blk + blk_off[p], nb * sizeof(int32_t),
                                  hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    if (getenv("GAC_TIMING"))
        fprintf(stderr, "[gac_kd_trees] %lld pairs, %lld blocks, %lld leaves, %d levels: build %.3f s, "
                        "results %.3f s\n", (long long)P, (long long)B, (long long)t.L, u.levels,
                t1 - t0, wall_s() - t1);
    return GAC_OK;
}

extern "C" int gac_crossovers(gac_ctx *c, int64_t n, const int32_t *t_seq, const int32_t *q_seq,
                              const uint8_t *q_strand, const int32_t *lqe, const int32_t *lte,
                              const int32_t *rqs, const int32_t *rts, const int32_t *overlap,
                              int32_t *pos, int32_t *adj) {
    gac_clear_error();
    if (!c || n < 0 || (n && (!t_seq || !q_seq || !q_strand || !lqe || !lte || !rqs || !rts ||
                              !overlap || !pos || !adj)))
        return gac_fail(GAC_E_ARG, "gac_crossovers: bad argument");
    if (!c->scoring) return gac_fail(GAC_E_STATE, "gac_crossovers before gac_set_scoring");
    CTX_LOCK(c);
    if (!c->g[0].final || !c->g[1].final)
        return gac_fail(GAC_E_STATE, "load both genomes before gac_crossovers");
    if (n == 0) return GAC_OK;
    std::vector<XoverJob> jobs(n);
    const Genome &T = c->g[0], &Q = c->g[1];
    for (int64_t j = 0; j < n; ++j) {
        XoverJob &J = jobs[j];
        int rc = pair_bases(c, t_seq[j], q_seq[j], q_strand[j], J.tbase, J.qbase);
        if (rc != GAC_OK) return rc;
        const int32_t ov = overlap[j];
        if (ov < 0 || lqe[j] - ov < 0 || lte[j] - ov < 0 || rqs[j] < 0 || rts[j] < 0 ||
            lqe[j] > Q.sizes[q_seq[j]] || (int64_t)rqs[j] + ov > Q.sizes[q_seq[j]] ||
            lte[j] > T.sizes[t_seq[j]] || (int64_t)rts[j] + ov > T.sizes[t_seq[j]])
            return gac_fail(GAC_E_ARG, "gac_crossovers: overlap %lld outside its sequences",
                            (long long)j);
        J.lqe = lqe[j];
        J.lte = lte[j];
        J.rqs = rqs[j];
        J.rts = rts[j];
        J.ov = ov;
        J.pad = 0;
    }
    HIPCHK(hipSetDevice(c->device));
    DpArgs a;
    dp_base_args(c, a);
    XoverJob *d_jobs = nullptr;
    int32_t *d_pos = nullptr, *d_adj = nullptr;
    int rc = GAC_OK;
    if ((rc = dev_upload(c, &d_jobs, jobs.data(), n)) == GAC_OK &&
        (rc = dev_upload(c, &d_pos, nullptr, n)) == GAC_OK &&
        (rc = dev_upload(c, &d_adj, nullptr, n)) == GAC_OK) {
        hipError_t e = launch_xover(a, d_jobs, n, d_pos, d_adj, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(pos, d_pos, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess)
            e = hipMemcpyAsync(adj, d_adj, n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = gac_fail(GAC_E_HIP, "gac_crossovers: %s", hipGetErrorString(e));
    }
    hipStreamSynchronize(c->stream);
    hipFree(d_jobs);
    hipFree(d_pos);
    hipFree(d_adj);
    return rc;
}

// ----------------------------------------------------------------- chains
// Host-side build of the device chain set, in parallel over chain ranges
// balanced by blocks: validation + DChain records (pass 1), bucket-index
// offsets (serial prefix), then blocks / spans / bucket indexes (pass 2).
struct UploadJob {
    gac_ctx *c;
    const gac_chainset_desc *d;
    DChain *ch;
    const int64_t *cut;  // chain ranges per task
    std::atomic<int> next;
    int ntask;
    std::atomic<long long> err_chain;  // first failing chain (pass 1), -1 if none
};

static void upload_pass1(UploadJob *J, int64_t i0, int64_t i1) {
    const gac_chainset_desc *d = J->d;
    gac_ctx *c = J->c;
    for (int64_t i = i0; i < i1; ++i) {
        const int32_t ts = d->t_seq[i], qs = d->q_seq[i];
        DChain &x = J->ch[i];
        bool bad = ts < 0 || ts >= (int32_t)c->g[0].sizes.size() || qs < 0 ||
                   qs >= (int32_t)c->g[1].sizes.size();
        const int64_t b0 = d->blk_off[i], b1 = d->blk_off[i + 1];
        bad = bad || b0 < 0 || b1 < b0 || b1 > d->n_blocks || b1 - b0 > INT32_MAX;
        if (!bad) {
            const int32_t tsize = c->g[0].sizes[ts], qsize = c->g[1].sizes[qs];
            int64_t pt = 0, pq = 0;
            for (int64_t b = b0; b < b1 && !bad; ++b) {
                const int64_t t = d->blk_t[b], q = d->blk_q[b], z = d->blk_size[b];
                bad = z < 0 || z >= (1 << 29) || t < 0 || q < 0 || t + z > tsize || q + z > qsize ||
                      (b > b0 && (t < pt || q < pq));
                pt = t + z;
                pq = q + z;
            }
            x.qinfo = qsize | (d->q_strand[i] ? (int32_t)0x80000000 : 0);
        }
        if (bad) {  // reported (with the serial check's message) by the caller
            long long cur = J->err_chain.load();
            while ((cur < 0 || i < cur) && !J->err_chain.compare_exchange_weak(cur, i)) {
            }
            return;
        }
        x.blk_off = b0;
        x.nblk = (int32_t)(b1 - b0);
        x.t_seq = ts;
        x.q_seq = qs;
        x.tstart = b1 > b0 ? d->blk_t[b0] : 0;
        x.tend = b1 > b0 ? d->blk_t[b1 - 1] + d->blk_size[b1 - 1] : 0;
        const int64_t span = (int64_t)x.tend - x.tstart;
        int shift = 0;
        while (span > 0 && (((span - 1) >> shift) + 1) > std::max<int64_t>(2 * x.nblk, 1)) ++shift;
        x.shift = shift;
        x.pad = 0;
        x.idx_off = (span > 0 ? ((span - 1) >> shift) + 1 : 0) + 1;  // count until the prefix
        x.tbase = c->g[0].woff[ts] * 32;
        const int64_t qw = c->g[1].woff[qs] * 32;
        x.qbase = x.qinfo < 0 ? ~(qw + (x.qinfo & 0x7fffffff)) : qw;
    }
}

static void *upload_thread(void *p) {
    UploadJob *J = (UploadJob *)p;
    for (int t; (t = J->next.fetch_add(1)) < J->ntask;) {
        upload_pass1(J, J->cut[t], J->cut[t + 1]);
    }
    return nullptr;
}

// Pageable host array -> device through the context's pinned staging buffers
// (threaded copies into one buffer while the other one's DMA runs).
struct CopyJob {
    const uint8_t *src;
    uint8_t *dst;
    size_t len;
    int nt;
    std::atomic<int> next;
};

static void *copy_thread(void *p) {
    CopyJob *J = (CopyJob *)p;
    const size_t per = (J->len + J->nt - 1) / J->nt;
    for (int t; (t = J->next.fetch_add(1)) < J->nt;) {
        const size_t a = std::min(J->len, per * t), b = std::min(J->len, per * (t + 1));
        if (b > a) memcpy(J->dst + a, J->src + a, b - a);
    }
    return nullptr;
}

static int ensure_pinned(gac_ctx *c);

static int upload_staged(gac_ctx *c, void *d_dst, const void *h_src, size_t bytes) {
    int rc = ensure_pinned(c);
    if (rc != GAC_OK) return rc;
    const int nt = std::max(1, std::min(16, gac_host_threads()));
    int k = 0;
    for (size_t lo = 0; lo < bytes; lo += pin_bytes(), k ^= 1) {
        const size_t hi = std::min(bytes, lo + pin_bytes());
        HIPCHK(hipEventSynchronize(c->pin_ev[k]));
        CopyJob J;
        J.src = (const uint8_t *)h_src + lo;
        J.dst = c->pin[k];
        J.len = hi - lo;
        J.nt = (hi - lo) >= (4u << 20) ? nt : 1;
        J.next = 0;
        gac_run_threads(J.nt, copy_thread, &J);
        HIPCHK(hipMemcpyAsync((uint8_t *)d_dst + lo, c->pin[k], hi - lo, hipMemcpyHostToDevice,
                              c->stream));
        HIPCHK(hipEventRecord(c->pin_ev[k], c->stream));
    }
    return GAC_OK;
}

// device buffer *p of capacity *cap holds at least want elements of sz bytes
// (grown with headroom; the contents are not kept)
static hipError_t ensure_buf(void **p, size_t *cap, size_t want, size_t sz) {
    if (*p && *cap >= want) return hipSuccess;
    if (*p) hipFree(*p);
    *p = nullptr;
    const size_t n = want + want / 4 + 64;
    const hipError_t e = hipMalloc(p, n * sz);
    *cap = e == hipSuccess ? n : 0;
    return e;
}

// the chain set's contents := d (its device buffers reused where they fit)
// the context's scoring setup, as the upload kernels take it
static UploadGaps upload_gaps(const gac_ctx *c, Blk12 *blk12) {
    UploadGaps G;
    G.blk12 = blk12;
    G.g = c->gap;
    G.small = c->d_small;
    G.tab = c->d_gap_tab;
    G.len = c->gap_len;
    return G;
}

static int chains_fill(gac_ctx *c, const gac_chainset_desc *d, gac_chainset *cs) {
    if (!c->g[0].final || !c->g[1].final)
        return gac_fail(GAC_E_STATE, "load both genomes before uploading chains");
    if (d->n_chains < 0 || d->n_blocks < 0 || (d->n_chains && (!d->t_seq || !d->q_seq ||
                                                                !d->q_strand || !d->blk_off)))
        return gac_fail(GAC_E_ARG, "gac_chains_upload: bad descriptor");
    if (d->n_chains && d->blk_off[d->n_chains] != d->n_blocks)
        return gac_fail(GAC_E_ARG, "blk_off[n_chains] != n_blocks");
    // every block belongs to a chain: the flat upload kernels find a block's
    // chain by its offset, so blocks before chain 0 (or with no chain) would
    // be written to negative positions
    if (d->n_chains && d->blk_off[0] != 0)
        return gac_fail(GAC_E_ARG, "blk_off[0] != 0");
    if (!d->n_chains && d->n_blocks)
        return gac_fail(GAC_E_ARG, "blocks without chains (n_chains == 0, n_blocks > 0)");
    // the kernels index blocks of one chain set with int32 (RangeDesc::b0,
    // flat windows): a larger set must be uploaded in parts
    if (d->n_blocks > (int64_t)INT32_MAX - 16)
        return gac_fail(GAC_E_ARG, "chain set of %lld blocks: at most %d per gac_chains_upload "
                        "(upload it in parts)", (long long)d->n_blocks, INT32_MAX - 16);
    const int64_t n = d->n_chains;
    const bool timing = getenv("GAC_TIMING") != nullptr;
    double t_lap = wall_s();
    const double t_fill0 = t_lap;
    auto lap = [&](const char *what) {
        if (!timing) return;
        const double t = wall_s();
        fprintf(stderr, "[gac_chains_upload] %-22s %.3f s\n", what, t - t_lap);
        t_lap = t;
    };
    // (not value-initialised: upload_pass1 writes every field of every good
    // chain on its own thread, so the 64 B/chain are first touched in
    // parallel instead of zeroed on this thread -- 320 MB at C5)
    // (freed on a detached thread when the fill returns: freeing it here
    // waited ~0.11 s at axtChain's C4 chain scoring -- glibc trimming the
    // heap top behind other threads' unmapping, r05c4t4; a private mapping
    // instead was slower still, r05c4t5)
    const size_t n_rec = (size_t)(n ? n : 1);
    struct LateArr {
        DChain *p;
        size_t bytes;
        explicit LateArr(size_t k) : p((DChain *)malloc(k * sizeof(DChain))), bytes(k * sizeof(DChain)) {}
        ~LateArr() {
            DChain *q = p;
            if (!q) return;
            // only the tens-of-MB staging of C4/C5-sized sets goes to a
            // thread: a small set (tests, re-uploads, loops) frees inline
            if (bytes < ((size_t)16 << 20)) {
                free(q);
                return;
            }
            try {
                std::thread([q] { free(q); }).detach();
            } catch (...) {
                free(q);
            }
        }
        DChain *get() const { return p; }
        DChain &operator[](size_t i) const { return p[i]; }
    } ch(n_rec);
    if (!ch.get()) return gac_fail(GAC_E_HIP, "gac_chains_upload: out of host memory");
    if (!n) memset(ch.get(), 0, sizeof(DChain));
    // tasks: contiguous chain ranges of about equal blocks + chains
    const int nt = std::max(1, std::min(64, gac_host_threads()));
    const int ntask = (int)std::min<int64_t>(std::max<int64_t>(n, 1), 8 * nt);
    std::vector<int64_t> cut(ntask + 1, n);
    {
        const int64_t work = d->n_blocks + n;
        int64_t i = 0;
        cut[0] = 0;
        for (int t = 1; t < ntask; ++t) {
            const int64_t target = work * t / ntask;
            while (i < n && d->blk_off[i] + i < target) ++i;
            cut[t] = i;
        }
        cut[ntask] = n;
    }
    UploadJob J;
    J.c = c;
    J.d = d;
    J.ch = ch.get();
    J.cut = cut.data();
    J.ntask = ntask;
    J.next = 0;
    J.err_chain = -1;
    gac_run_threads(std::min(nt, ntask), upload_thread, &J);
    if (J.err_chain.load() >= 0) {  // the first bad chain: the serial checks, for the message
        const int64_t i = J.err_chain.load();
        const int32_t ts = d->t_seq[i], qs = d->q_seq[i];
        if (ts < 0 || ts >= (int32_t)c->g[0].sizes.size() || qs < 0 ||
            qs >= (int32_t)c->g[1].sizes.size())
            return gac_fail(GAC_E_ARG, "chain %lld: sequence index out of range", (long long)i);
        const int64_t b0 = d->blk_off[i], b1 = d->blk_off[i + 1];
        if (b0 < 0 || b1 < b0 || b1 > d->n_blocks || b1 - b0 > INT32_MAX)
            return gac_fail(GAC_E_ARG, "chain %lld: bad block offsets", (long long)i);
        const int32_t tsize = c->g[0].sizes[ts], qsize = c->g[1].sizes[qs];
        int64_t pt = 0, pq = 0;
        for (int64_t b = b0; b < b1; ++b) {
            const int64_t t = d->blk_t[b], q = d->blk_q[b], z = d->blk_size[b];
            if (z < 0 || z >= (1 << 29) || t < 0 || q < 0 || t + z > tsize || q + z > qsize)
                return gac_fail(GAC_E_FORMAT,
                                "chain %lld block %lld [t %lld q %lld size %lld] outside its "
                                "sequences (tSize %d qSize %d)",
                                (long long)i, (long long)(b - b0), (long long)t, (long long)q,
                                (long long)z, tsize, qsize);
            if (b > b0 && (t < pt || q < pq))
                return gac_fail(GAC_E_FORMAT, "chain %lld: blocks not ascending (negative gap)",
                                (long long)i);
            pt = t + z;
            pq = q + z;
        }
        return gac_fail(GAC_E_FORMAT, "chain %lld: invalid", (long long)i);
    }
    lap("chain records + checks");
    int64_t idx_n = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t k = ch[i].idx_off;
        ch[i].idx_off = idx_n;
        idx_n += k;
    }
    HIPCHK(hipSetDevice(c->device));
    cs->ctx = c;
    cs->n_chains = d->n_chains;
    cs->n_blocks = d->n_blocks;
    cs->gap_version = 0;  // block gaps are computed at the next scoring call
    free_whole_plan(cs);
    const size_t nb = (size_t)d->n_blocks;
    // the caller's block arrays, staged; blocks / spans / buckets are built
    // from them on the device (k_build_*)
    hipError_t e = ensure_buf((void **)&cs->chains, &cs->cap_chains, n_rec, sizeof(DChain));
    if (e == hipSuccess) e = ensure_buf((void **)&cs->blk, &cs->cap_blocks, nb + 8, sizeof(int4));
    if (e == hipSuccess) e = ensure_buf((void **)&cs->blk12, &cs->cap_blk12, nb + 8, sizeof(Blk12));
    // (the window-search index -- spans, bucket entries -- is allocated
    // with the index itself: ensure_index, or here when it is built eagerly)
    static const bool eager = [] {
        const char *v = getenv("GAC_UP_INDEX");
        return v && !strcmp(v, "eager");
    }();
    cs->idx_n = idx_n;
    if (e == hipSuccess && eager)
        e = ensure_buf((void **)&cs->tspan, &cs->cap_tspan, nb + 8, sizeof(int2));
    if (e == hipSuccess && eager)
        e = ensure_buf((void **)&cs->bucket, &cs->cap_idx, (size_t)std::max<int64_t>(idx_n, 1), 4);
    if (e == hipSuccess)
        e = ensure_buf((void **)&cs->d_stage, &cs->cap_stage, std::max<size_t>(3 * nb, 1), 4);
    int32_t *d_bt = cs->d_stage;
    int rc = GAC_OK;
    lap("allocations");
    if (e == hipSuccess) rc = upload_staged(c, cs->chains, ch.get(), n_rec * sizeof(DChain));
    if (e == hipSuccess && rc == GAC_OK && nb) rc = upload_staged(c, d_bt, d->blk_t, nb * 4);
    if (e == hipSuccess && rc == GAC_OK && nb) rc = upload_staged(c, d_bt + nb, d->blk_q, nb * 4);
    if (e == hipSuccess && rc == GAC_OK && nb) rc = upload_staged(c, d_bt + 2 * nb, d->blk_size, nb * 4);
    lap("staged copies");
    // blocks, spans, bucket indexes and per-block N flags (scoring skips the
    // N-mask loads of N-free blocks), one lane per block
    const int64_t ntiles = ((int64_t)nb + 63) >> 6;
    if (e == hipSuccess)
        e = ensure_buf((void **)&cs->d_coff, &cs->cap_coff, (size_t)(n + 1), sizeof(int32_t));
    if (e == hipSuccess)
        e = ensure_buf((void **)&cs->d_tile_c0, &cs->cap_tile_c0, (size_t)(ntiles + 1), sizeof(int32_t));
    if (e == hipSuccess)
        e = ensure_buf((void **)&cs->d_crun, &cs->cap_crun, (size_t)(n ? n : 1), sizeof(int4));
    // with the scoring already set, the block gaps and 12-byte records come
    // out of the same pass (GAC_UP_FUSE=0: at the first scoring call, as
    // when the scoring follows the chains)
    static const bool fuse = [] {
        const char *v = getenv("GAC_UP_FUSE");
        return !(v && v[0] == '0');
    }();
    const bool gaps = fuse && c->scoring;
    const UploadGaps G = gaps ? upload_gaps(c, cs->blk12) : UploadGaps{};
    // the window-search index only on demand: chainNet -rescore hands its
    // windows over and whole chains need none (GAC_UP_INDEX=eager: now)
    if (e == hipSuccess && rc == GAC_OK)
        e = launch_build_flat(d_bt, d_bt + nb, d_bt + 2 * nb, (int64_t)nb, cs->chains, n, cs->d_coff,
                              cs->d_tile_c0, cs->d_crun, c->g[0].d_nrun, c->g[0].n_nrun,
                              c->g[1].d_nrun, c->g[1].n_nrun, c->g[1].d_woff, cs->blk, cs->tspan,
                              cs->bucket, G, eager, c->stream);
    cs->idx_ready = eager;
    if (e == hipSuccess && rc == GAC_OK && gaps) cs->gap_version = c->gap_version;
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    lap("device build + sync");
    if (timing)
        fprintf(stderr, "[gac_chains_upload] laps from the fill's start: %.3f s\n", wall_s() - t_fill0);
    if (rc != GAC_OK) return rc;
    if (e != hipSuccess) return gac_fail(GAC_E_HIP, "chain upload failed: %s", hipGetErrorString(e));
    return GAC_OK;
}

extern "C" int gac_chains_upload(gac_ctx *c, const gac_chainset_desc *d, gac_chainset **out) {
    gac_clear_error();
    if (!c || !d || !out) return gac_fail(GAC_E_ARG, "gac_chains_upload: NULL argument");
    const double t_in = wall_s();
    CTX_LOCK(c);
    if (getenv("GAC_TIMING"))
        fprintf(stderr, "[gac_chains_upload] context lock          %.3f s\n", wall_s() - t_in);
    *out = nullptr;
    gac_chainset *cs = new gac_chainset();
    cs->ctx = c;
    c->sets.push_back(cs);
    const double t_f = wall_s();
    const int rc = chains_fill(c, d, cs);
    const double t_r = wall_s();
    if (rc != GAC_OK) {
        gac_chains_free(cs);
        return rc;
    }
    *out = cs;
    if (getenv("GAC_TIMING"))
        fprintf(stderr, "[gac_chains_upload] total                 %.3f s (before the fill %.3f, "
                        "fill %.3f)\n", wall_s() - t_in, t_f - t_in, t_r - t_f);
    return GAC_OK;
}

extern "C" int gac_chains_reupload(gac_ctx *c, const gac_chainset_desc *d, gac_chainset *cs) {
    gac_clear_error();
    if (!c || !d || !cs) return gac_fail(GAC_E_ARG, "gac_chains_reupload: NULL argument");
    if (cs->ctx != c) return gac_fail(GAC_E_ARG, "gac_chains_reupload: a set of another context");
    CTX_LOCK(c);
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipStreamSynchronize(c->stream));  // (calls in flight may still read the set)
    return chains_fill(c, d, cs);
}

static void free_set_memory(gac_chainset *cs) {
    hipSetDevice(cs->ctx->device);  // (hipFree waits for work still using them)
    void *bufs[] = {cs->chains, cs->blk,     cs->blk12,     cs->tspan,  cs->bucket,
                    cs->d_stage, cs->d_coff, cs->d_tile_c0, cs->d_crun};
    for (void *p : bufs)
        if (p) hipFree(p);
    cs->chains = nullptr;
    cs->blk = nullptr;
    cs->blk12 = nullptr;
    cs->tspan = nullptr;
    cs->bucket = nullptr;
    cs->d_stage = nullptr;
    cs->d_coff = cs->d_tile_c0 = nullptr;
    cs->d_crun = nullptr;
    free_whole_plan(cs);
}

extern "C" void gac_chains_free(gac_chainset *cs) {
    if (!cs) return;
    if (gac_ctx *c = cs->ctx) {  // (NULL: its context was closed, the memory went with it)
        CTX_LOCK(c);
        free_set_memory(cs);
        c->sets.erase(std::remove(c->sets.begin(), c->sets.end(), cs), c->sets.end());
        if (c->srv.cs == cs) c->srv.cs = nullptr;
    }
    delete cs;
}

extern "C" gac_ctx *gac_chains_context(const gac_chainset *cs) { return cs ? cs->ctx : nullptr; }

extern "C" int64_t gac_chains_block_count(const gac_chainset *cs) { return cs ? cs->n_blocks : -1; }

// ----------------------------------------------------------------- launch
static int ensure_ws(gac_ctx *c, int64_t n, int64_t max_tiles, hipStream_t s) {
    // buffers may still be in use by calls in flight (on this stream or, for
    // the device-pointer API, on the stream of the previous call)
    if (n > c->ws_n || max_tiles > c->ws_tiles || !c->status) {
        HIPCHK(hipStreamSynchronize(s));
        if (c->ws_last && c->ws_last != s) HIPCHK(hipEventSynchronize(c->ws_ev));
    }
    if (n > c->ws_n) {
        int64_t cap = n + n / 2 + 1024;
        void *bufs[] = {c->rdesc, c->nblk, c->goff, c->pb0, c->agg, c->plan_off, c->lbflag, c->gflat, c->lbflag};
        for (void *p : bufs)
            if (p) hipFree(p);
        c->rdesc = nullptr;
        c->lbflag = nullptr;
        c->nblk = c->goff = c->pb0 = c->plan_off = c->gflat = nullptr;
        c->agg = nullptr;
        const int64_t G = plan_grid(cap) + 2;
        HIPCHK(hipMalloc(&c->rdesc, cap * sizeof(RangeDesc)));
        HIPCHK(hipMalloc(&c->nblk, cap * 4));
        HIPCHK(hipMalloc(&c->goff, cap * 4));
        HIPCHK(hipMalloc(&c->pb0, cap * 4));
        HIPCHK(hipMalloc(&c->gflat, cap * 4));
        HIPCHK(hipMalloc(&c->agg, G * 4));
        HIPCHK(hipMalloc(&c->plan_off, G * 4));
        HIPCHK(hipMalloc(&c->lbflag, G * 8));
        HIPCHK(hipMemsetAsync(c->lbflag, 0, G * 8, s));  // (no tag: "not yet")
        // (this memset returns success but leaves hipErrorInvalidValue as the
        // thread's last error on this runtime, which the next launch check
        // would report as its own: consumed here; r06lbdbg)
        (void)hipGetLastError();
        c->ws_n = cap;
    }
    if (!c->status) {
        HIPCHK(hipMalloc(&c->status, kStatusBytes));
        HIPCHK(hipMemsetAsync(c->status, 0, kStatusBytes, s));
    }
    if (max_tiles > c->ws_tiles) {
        int64_t cap = max_tiles + max_tiles / 4 + 1024;
        void *old[] = {c->sum_head, c->sum_tail, c->tile_r0, c->sup_head, c->sup_tail,
                       c->sup_tail_r};
        for (void *p : old)
            if (p) hipFree(p);
        c->sum_head = c->sum_tail = c->sup_head = c->sup_tail = nullptr;
        c->tile_r0 = c->sup_tail_r = nullptr;
        const int64_t ucap = cap / kWave + 2;
        HIPCHK(hipMalloc(&c->sum_head, cap * sizeof(SegSum)));
        HIPCHK(hipMalloc(&c->sum_tail, cap * sizeof(SegSum)));
        HIPCHK(hipMalloc(&c->tile_r0, cap * 4));
        HIPCHK(hipMalloc(&c->sup_head, ucap * sizeof(SegSum)));
        HIPCHK(hipMalloc(&c->sup_tail, ucap * sizeof(SegSum)));
        HIPCHK(hipMalloc(&c->sup_tail_r, ucap * 4));
        c->ws_tiles = cap;
    }
    return GAC_OK;
}

static hipEvent_t prof_event(gac_ctx *c) {
    if (!c->prof_free.empty()) {
        hipEvent_t e = c->prof_free.back();
        c->prof_free.pop_back();
        return e;
    }
    hipEvent_t e;
    hipEventCreate(&e);
    return e;
}

#define PROF_BEGIN(k)                                   \
    hipEvent_t _pa = nullptr, _pb = nullptr;            \
    if (c->prof & (1 << (k))) {                         \
        _pa = prof_event(c);                            \
        _pb = prof_event(c);                            \
        hipEventRecord(_pa, s);                         \
    }
#define PROF_END(k)                                     \
    if (_pa) {                                          \
        hipEventRecord(_pb, s);                         \
        c->prof_pending.push_back(Prof{(k), _pa, _pb}); \
    }

// Spin on the pinned status words until k_scan_agg of call `tag` has written
// them (checking now and then that the stream is still busy).
static int wait_status(gac_ctx *c, hipStream_t s, int32_t tag, int32_t st[4]) {
    volatile int32_t *h = c->h_stat;
    for (uint64_t spin = 0;; ++spin) {
        if (h[4] == tag) {
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            for (int k = 0; k < 4; ++k) st[k] = h[k];
            return GAC_OK;
        }
        if ((spin & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(s);
            if (q == hipSuccess && h[4] != tag)
                return gac_fail(GAC_E_HIP, "scoring status never arrived (call %d)", tag);
            if (q != hipSuccess && q != hipErrorNotReady)
                return gac_fail(GAC_E_HIP, "scoring failed: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

// the set's window-search index (spans + bucket entries), built at the first
// call that searches windows (stream-ordered before it)
static int ensure_index(gac_ctx *c, const gac_chainset *cs_in, hipStream_t s) {
    gac_chainset *cs = const_cast<gac_chainset *>(cs_in);
    if (cs->idx_ready || (cs->n_blocks == 0 && cs->n_chains == 0)) return GAC_OK;
    const int64_t nb = cs->n_blocks;
    HIPCHK(ensure_buf((void **)&cs->tspan, &cs->cap_tspan, (size_t)nb + 8, sizeof(int2)));
    HIPCHK(ensure_buf((void **)&cs->bucket, &cs->cap_idx, (size_t)std::max<int64_t>(cs->idx_n, 1), 4));
    const int32_t *d_bt = cs->d_stage;
    HIPCHK(launch_build_index(d_bt, d_bt + nb, d_bt + 2 * nb, nb, cs->chains, cs->n_chains,
                              cs->d_coff, cs->d_tile_c0, cs->tspan, cs->bucket, s));
    cs->idx_ready = true;
    return GAC_OK;
}

// One call = k_plan, the tile map (k_tilemap_fused, or k_scan_agg + k_tilemap
// above 1 M ranges), k_tile and the cross-tile fold (k_fold_tiles +
// k_fold_super); the host waits only for the status words (pinned memory),
// not for the scoring itself.  The flat block count W is only known on the
// device (ranges may overlap), so the kernels check the workspace capacity
// themselves; on overflow k_tile and the folds do nothing and the call grows the
// workspace to the reported {W, T} and runs once more (first call or a larger
// batch only).
// Checks shared by both scoring paths, the per-setup block gaps, and the
// kernel arguments that do not depend on the workspace.
static int prepare_args(gac_ctx *c, const gac_chainset *cs, int64_t n, uint32_t flags,
                        const void *d_l, hipStream_t s, ScoreArgs &a) {
    if (!c->scoring) return gac_fail(GAC_E_STATE, "gac_set_scoring() not called");
    if (!cs || cs->ctx != c) return gac_fail(GAC_E_ARG, "chainset does not belong to this context");
    if (n < 0 || n > INT32_MAX / 2) return gac_fail(GAC_E_ARG, "bad range count %lld", (long long)n);
    if ((flags & GAC_WANT_LOCAL) && !d_l) return gac_fail(GAC_E_ARG, "GAC_WANT_LOCAL needs local output");
    if (n == 0) return GAC_OK;
    if (cs->gap_version != c->gap_version) {  // blk[].w for this scoring setup
        HIPCHK(launch_block_gaps_flat(cs->d_coff, cs->d_tile_c0, cs->n_blocks, cs->blk, cs->blk12,
                                      upload_gaps(c, cs->blk12), s));
        const_cast<gac_chainset *>(cs)->gap_version = c->gap_version;
    }
    memset(&a, 0, sizeof(a));
    const Genome &T = c->g[0], &Q = c->g[1];
    a.t_planes = T.planes;
    a.t_nmask = T.nmask;
    a.t_woff = T.d_woff;
    a.q_planes = Q.planes;
    a.q_nmask = Q.nmask;
    a.q_woff = Q.d_woff;
    a.chains = cs->chains;
    a.n_chains = cs->n_chains;
    a.blk = cs->blk;
    static const bool blk16 = [] {
        const char *e = getenv("GAC_TILE_BLK16");
        return e && e[0] == '1';
    }();
    a.blk12 = blk16 ? nullptr : cs->blk12;
    a.tspan = cs->tspan;
    a.bucket = cs->bucket;
    a.n = n;
    a.want_local = (flags & GAC_WANT_LOCAL) ? 1 : 0;
    a.gap_len = c->gap_len;
    a.gap_tab = c->d_gap_tab;
    a.small_tab = c->d_small;
    memcpy(a.coef, c->coef, sizeof(a.coef));
    a.sym = c->sym;
    static const int scan64 = [] {
        const char *e = getenv("GAC_TILE_SCAN64");
        return e && e[0] == '1' ? 1 : 0;
    }();
    a.scan64 = scan64;
    static const int xcd_chunk = [] {
        const char *e = getenv("GAC_TILE_XCD");
        return e && e[0] == '1' ? 1 : 0;
    }();
    a.xcd_chunk = xcd_chunk;
    a.gap = c->gap;
    return GAC_OK;
}

static int score_device_split(gac_ctx *c, const ScoreArgs &a_base, const Range *d_ranges,
                              const Window *d_wins, int64_t n, long long *d_g, long long *d_l,
                              int32_t *d_ali, hipStream_t s);

// ------------------------------------------------ the small-batch server ----
// k_small_server (gac_kernels.hip) keeps a grid resident between the calls of
// a run of small batches (chainCleaner's replay loop), so a call costs a
// mailbox round trip instead of a launch and a stream synchronisation.  Only
// the small-batch entry points keep it running; every other entry point parks
// it first (CTX_LOCK), and the grid exits by itself after `idle` without a
// request.  On by default (GAC_SMALL_SERVER=0: a k_small launch per batch):
// 16.5 vs 23.6 us per 20-range call of an uploaded set, 23.4 vs 30.6 for
// host-held chains, chainCleaner's C3 loop 0.19 vs 0.27 s in its 10 k calls
// (r05lat6).
// (bounded: a grid that has not drained kParkSecs after its stop -- wedged,
// or never scheduled -- is left behind, the server marked unusable, and the
// caller gets an error instead of an unbounded hipStreamSynchronize)
constexpr double kParkSecs = 10.0;

static void srv_park(gac_ctx *c) {
    SmallServer &v = c->srv;
    if (!v.running) return;
    __atomic_store_n(&v.mail->stop, 1u, __ATOMIC_RELEASE);
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t it = 1;; ++it) {
        const hipError_t q = hipStreamQuery(v.st);
        if (q != hipErrorNotReady) break;  // drained (or failed: reported by the next call)
        if ((it & 1023) == 0) {
            clock_gettime(CLOCK_MONOTONIC, &t1);
            if ((t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec) > kParkSecs) {
                v.wedged = true;
                v.on = false;
                v.running = false;
                return;  // (stop stays set: the grid exits whenever it runs)
            }
        }
        __builtin_ia32_pause();
    }
    __atomic_store_n(&v.mail->stop, 0u, __ATOMIC_RELEASE);
    v.running = false;
}

static void srv_free(gac_ctx *c) {
    SmallServer &v = c->srv;
    if (v.wedged) return;  // (a grid may still read these: left allocated)
    void *h[] = {v.mail, v.h_in, v.h_hq, v.h_pool, v.h_out};
    for (void *p : h)
        if (p) hipHostFree(p);
    if (v.d_sync) hipFree(v.d_sync);
    if (v.st) hipStreamDestroy(v.st);
    const bool on = v.on;
    const uint64_t idle = v.idle;
    const int wgs = v.wgs;
    v = SmallServer();
    v.on = on;
    v.idle = idle;
    v.wgs = wgs;
}

static int srv_alloc(gac_ctx *c) {
    SmallServer &v = c->srv;
    if (v.mail) return GAC_OK;
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
    // the inputs: coherent (uncached on the device) or, GAC_SRV_INPUT=nc,
    // cached and invalidated by each workgroup's acquire fence per request
    const char *iv = getenv("GAC_SRV_INPUT");
    const unsigned fin = iv && strcmp(iv, "nc") == 0 ? (unsigned)hipHostMallocMapped : fl;
    v.in_fl = fin;
    HIPCHK(hipStreamCreateWithFlags(&v.st, hipStreamNonBlocking));
    HIPCHK(hipHostMalloc((void **)&v.mail, sizeof(SmallMail), fl));
    memset(v.mail, 0, sizeof(SmallMail));
    HIPCHK(hipHostGetDevicePointer((void **)&v.d_mail, v.mail, 0));
    HIPCHK(hipHostMalloc((void **)&v.h_in, kSmallMax * sizeof(Range), fin));
    HIPCHK(hipHostGetDevicePointer((void **)&v.d_in, v.h_in, 0));
    HIPCHK(hipHostMalloc((void **)&v.h_hq, kSmallMax * sizeof(RangeDesc), fin));
    HIPCHK(hipHostGetDevicePointer((void **)&v.d_hq, v.h_hq, 0));
    HIPCHK(hipHostMalloc((void **)&v.h_out, kSmallMax * sizeof(SmallOut), fl));
    HIPCHK(hipHostGetDevicePointer((void **)&v.d_out, v.h_out, 0));
    // uncached device memory: the broadcast word and the count are polled
    // by workgroups on every XCD, whose L2s are not coherent with each other
    HIPCHK(hipExtMallocWithFlags((void **)&v.d_sync, sizeof(SmallSync), hipDeviceMallocUncached));
    v.seq = 0;
    return GAC_OK;
}

// the pool of host-planned window records: grown (while parked) to `need`
static int srv_pool(gac_ctx *c, int64_t need) {
    SmallServer &v = c->srv;
    if (need <= v.pool_cap) return GAC_OK;
    srv_park(c);
    if (v.h_pool) hipHostFree(v.h_pool);
    v.h_pool = nullptr;
    v.pool_cap = 0;
    const int64_t cap = std::max<int64_t>(need + need / 2, 1 << 16);
    HIPCHK(hipHostMalloc((void **)&v.h_pool, cap * sizeof(int4), v.in_fl));
    HIPCHK(hipHostGetDevicePointer((void **)&v.d_pool, v.h_pool, 0));
    v.pool_cap = cap;
    return GAC_OK;
}

static int srv_launch(gac_ctx *c) {
    SmallServer &v = c->srv;
    HIPCHK(hipMemsetAsync(v.d_sync, 0, sizeof(SmallSync), v.st));
    __atomic_store_n(&v.mail->state, 1u, __ATOMIC_RELEASE);
    __atomic_store_n(&v.mail->done, v.seq, __ATOMIC_RELEASE);
    static const uint32_t trace = getenv("GAC_SRV_TRACE") ? 1u : 0u;
    HIPCHK(launch_small_server(v.a0, v.a1, v.d_in, v.d_hq, v.d_pool, v.d_out, v.d_mail, v.d_sync,
                               v.seq, v.idle, trace, v.wgs, v.st));
    v.running = true;
    ++v.launches;
    return GAC_OK;
}

// a resident grid for requests of this kind: kind 0 scores ranges of `cs`
// (prepared like the k_small path: gaps, window index), kind 1 host-planned
// descriptors (any grid with the same local flag takes them)
static int srv_ensure(gac_ctx *c, const gac_chainset *cs, uint32_t flags) {
    SmallServer &v = c->srv;
    if (v.wedged) return gac_fail(GAC_E_HIP, "small-batch server disabled: an earlier grid did not exit");
    const int local = (flags & GAC_WANT_LOCAL) ? 1 : 0;
    if (v.running && v.local == local && v.gap_version == c->gap_version && (!cs || v.cs == cs))
        return GAC_OK;
    srv_park(c);
    int rc = srv_alloc(c);
    if (rc != GAC_OK) return rc;
    if (!cs) cs = v.cs;  // (a freed set is cleared from v.cs by gac_chains_free)
    ScoreArgs a1;
    memset(&a1, 0, sizeof(a1));
    const Genome &T = c->g[0], &Q = c->g[1];
    a1.t_planes = T.planes;
    a1.t_nmask = T.nmask;
    a1.t_woff = T.d_woff;
    a1.q_planes = Q.planes;
    a1.q_nmask = Q.nmask;
    a1.q_woff = Q.d_woff;
    a1.want_local = local;
    a1.gap_len = c->gap_len;
    a1.gap_tab = c->d_gap_tab;
    a1.small_tab = c->d_small;
    memcpy(a1.coef, c->coef, sizeof(a1.coef));
    a1.sym = c->sym;
    a1.gap = c->gap;
    ScoreArgs a0 = a1;
    if (cs) {
        long long dummy = 0;
        if ((rc = prepare_args(c, cs, 1, flags, &dummy, c->stream, a0)) != GAC_OK) return rc;
        if ((rc = ensure_index(c, cs, c->stream)) != GAC_OK) return rc;
        a0.tspan = cs->tspan;  // (allocated with the index)
        a0.bucket = cs->bucket;
        HIPCHK(hipStreamSynchronize(c->stream));  // (the gaps and the index, before the grid)
    }
    if ((rc = srv_pool(c, 1)) != GAC_OK) return rc;
    v.a0 = a0;
    v.a1 = a1;
    v.cs = cs;
    v.local = local;
    v.gap_version = c->gap_version;
    return srv_launch(c);
}

// one request: inputs already in the mailbox buffers; waits for the results
static int srv_call(gac_ctx *c, uint32_t kind, int64_t n) {
    SmallServer &v = c->srv;
    const uint32_t prev = v.seq;  // (the last request word; 20-bit numbers, never 0)
    uint32_t num = ((prev & 0xfffffu) + 1) & 0xfffffu;
    if (num == 0) num = 1;
    const uint32_t seq = srv_word(num, kind, (uint32_t)n);
    v.seq = seq;
    __atomic_store_n(&v.mail->req, seq, __ATOMIC_RELEASE);
    ++v.requests;
    struct timespec t0;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (uint64_t it = 1;; ++it) {
        if (__atomic_load_n(&v.mail->done, __ATOMIC_ACQUIRE) == seq) return GAC_OK;
        if (__atomic_load_n(&v.mail->state, __ATOMIC_ACQUIRE) == 2u) {
            // the grid left (idle) before it saw this request: once it has
            // drained, a new one takes the request from the mailbox
            HIPCHK(hipStreamSynchronize(v.st));
            v.running = false;
            if (__atomic_load_n(&v.mail->done, __ATOMIC_ACQUIRE) == seq) return GAC_OK;
            v.seq = prev;
            const int rc = srv_launch(c);
            v.seq = seq;
            if (rc != GAC_OK) return rc;
            continue;
        }
        if ((it & 4095) == 0) {
            struct timespec t1;
            clock_gettime(CLOCK_MONOTONIC, &t1);
            if ((t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec) > 10.0) {
                srv_park(c);  // (bounded)
                return gac_fail(GAC_E_HIP, "small-batch server: no answer to request %u in 10 s%s",
                                seq, v.wedged ? " (grid did not exit; server disabled)" : "");
            }
            const hipError_t q = hipStreamQuery(v.st);
            if (q != hipSuccess && q != hipErrorNotReady)
                return gac_fail(GAC_E_HIP, "small-batch server failed: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

static void srv_results(const gac_ctx *c, int64_t n, uint32_t flags, int64_t *global,
                        int64_t *local, int32_t *ali) {
    for (int64_t i = 0; i < n; ++i) {
        const SmallOut o = c->srv.h_out[i];
        global[i] = o.g;
        ali[i] = o.ali;
        if (flags & GAC_WANT_LOCAL) local[i] = o.l;
    }
}

// d_wins non-null: the ranges come with their windows (gac_score_windows*),
// d_ranges is ignored
static int score_device(gac_ctx *c, const gac_chainset *cs, const Range *d_ranges,
                        const Window *d_wins, int64_t n, uint32_t flags, long long *d_g,
                        long long *d_l, int32_t *d_ali, hipStream_t s) {
    ScoreArgs a_base;
    if (c->ws_last && c->ws_last != s) HIPCHK(hipStreamWaitEvent(s, c->ws_ev, 0));
    int rc = prepare_args(c, cs, n, flags, d_l, s, a_base);
    if (rc != GAC_OK || n == 0) return rc;
    if (!d_wins && (rc = ensure_index(c, cs, s)) != GAC_OK) return rc;
    a_base.tspan = cs->tspan;  // (allocated with the index)
    a_base.bucket = cs->bucket;
    rc = score_device_split(c, a_base, d_ranges, d_wins, n, d_g, d_l, d_ali, s);
    if (hipEventRecord(c->ws_ev, s) == hipSuccess) c->ws_last = s;
    return rc;
}

// One batch through the pipeline; a batch whose window blocks overflow int32
// (kernels index flat blocks with 32 bits) is split in halves, recursively.
static int score_device_split(gac_ctx *c, const ScoreArgs &a_base, const Range *d_ranges,
                              const Window *d_wins, int64_t n, long long *d_g, long long *d_l,
                              int32_t *d_ali, hipStream_t s) {
    int rc;
    // first guess for an empty workspace: 8 window blocks per range
    const int64_t guess = c->ws_tiles ? 0 : 8 * n;
    rc = ensure_ws(c, n, guess / kTileBlocks + 1, s);
    if (rc != GAC_OK) return rc;
    ScoreArgs a = a_base;
    a.ranges = d_wins ? nullptr : d_ranges;
    a.wins = d_wins;
    a.out_g = d_g;
    a.out_l = d_l;
    a.out_ali = d_ali;
    for (int pass = 0; pass < 2; ++pass) {
        a.rdesc = c->rdesc;
        a.nblk = c->nblk;
        a.goff = c->goff;
        a.pb0 = c->pb0;
        a.agg = c->agg;
        a.plan_off = c->plan_off;
        a.lbflag = c->lbflag;
        a.gflat = c->gflat;
        a.status = c->status;
        a.tile_r0 = c->tile_r0;
        a.sum_head = c->sum_head;
        a.sum_tail = c->sum_tail;
        a.sup_head = c->sup_head;
        a.sup_tail = c->sup_tail;
        a.sup_tail_r = c->sup_tail_r;
        a.host_status = c->d_h_stat;
        a.call_tag = ++c->call_seq;
        if (a.call_tag <= 0) a.call_tag = c->call_seq = 1;
        a.cap_tiles = (int32_t)(c->ws_tiles < INT32_MAX ? c->ws_tiles : INT32_MAX);
        {
            PROF_BEGIN(GAC_K_PLAN);
            if (plan_lb()) {
                HIPCHK(launch_plan_lb(a, s));
            } else {
                HIPCHK(launch_plan(a, s));
                HIPCHK(launch_tilemap(a, s));
            }
            PROF_END(GAC_K_PLAN);
        }
        {
            PROF_BEGIN(GAC_K_TILE);
            HIPCHK(launch_tile(a, c->tile_grid_sym[a.sym ? 1 : 0][a.want_local ? 1 : 0], s));
            PROF_END(GAC_K_TILE);
        }
        {
            PROF_BEGIN(GAC_K_COMBINE);
            HIPCHK(launch_combine(a, c->combine_grid, s));
            PROF_END(GAC_K_COMBINE);
        }
        // wait for k_scan_agg's status words only; the rest runs on
        int32_t st[4];
        rc = wait_status(c, s, a.call_tag, st);
        if (rc != GAC_OK) return rc;
        if (st[3]) {  // k_plan<true>: a window outside its chain (it selected nothing)
            HIPCHK(hipStreamSynchronize(s));
            return gac_fail(GAC_E_ARG, "a window's blocks lie outside its chain (or its chain "
                            "index is out of range)");
        }
        if (st[0] == INT32_MAX) {  // W >= 2^31: two halves
            HIPCHK(hipStreamSynchronize(s));
            if (n < 2) return gac_fail(GAC_E_ARG, "one range's window exceeds 2^31 blocks");
            const int64_t h = n / 2;
            ScoreArgs b = a_base;
            b.n = h;
            rc = score_device_split(c, b, d_ranges, d_wins, h, d_g, d_l, d_ali, s);
            if (rc != GAC_OK) return rc;
            b.n = n - h;
            return score_device_split(c, b, d_wins ? nullptr : d_ranges + h,
                                      d_wins ? d_wins + h : nullptr, n - h, d_g + h,
                                      d_l ? d_l + h : nullptr, d_ali + h, s);
        }
        if (!st[2]) return GAC_OK;
        rc = ensure_ws(c, n, st[1], s);  // (synchronises before growing)
        if (rc != GAC_OK) return rc;
    }
    return gac_fail(GAC_E_STATE, "scoring workspace still too small after growing it");
}

// ----------------------------------------------------------------- whole chains
// scoreChain's batch: every chain of the set, in order (kent chainCalcScore +
// chainCalcScoreLocal per chain).  The plan is the chain set's own, built
// once; a call is the empty-chain zeroing (if any), k_tile and the fold.
static int ensure_whole(gac_ctx *c, gac_chainset *cs, hipStream_t s) {
    if (cs->w_ready) return GAC_OK;
    const int64_t n = cs->n_chains, nb = cs->n_blocks;
    const int64_t T = (nb + kTileBlocks - 1) / kTileBlocks;
    HIPCHK(hipMalloc(&cs->w_rdesc, std::max<int64_t>(n, 1) * sizeof(RangeDesc)));
    HIPCHK(hipMalloc(&cs->w_nblk, std::max<int64_t>(n, 1) * 4));
    HIPCHK(hipMalloc(&cs->w_gflat, std::max<int64_t>(n, 1) * 4));
    HIPCHK(hipMalloc(&cs->w_tile_r0, std::max<int64_t>(T, 1) * 4));
    HIPCHK(hipMalloc(&cs->w_status, kStatusBytes));
    const int32_t st[8] = {(int32_t)nb, (int32_t)T, 0, 0, 0, 0, 0, 0};
    HIPCHK(hipMemcpyAsync(cs->w_status, st, sizeof(st), hipMemcpyHostToDevice, s));
    // set order by default; GAC_WHOLE_ORDER=target plans the chains in
    // target order (r03k/r03m, C5: k_tile 2.29 vs 2.34 ms, but the scatter
    // back to chain order cost 0.13 ms; r03zb, results stored straight to
    // the chain: k_tile 2.34 vs 2.19 ms in set order, so set order stays)
    const char *ord = getenv("GAC_WHOLE_ORDER");
    const bool sorted = ord && !strcmp(ord, "target");
    if (sorted) {
        HIPCHK(hipMalloc(&cs->w_pb0, n * 4));
        HIPCHK(hipMalloc(&cs->w_perm, n * 4));
        unsigned long long *keys = nullptr;
        int32_t *vals = nullptr, *perm = nullptr, *inv = nullptr;
        void *tmp = nullptr;
        size_t tmp_bytes = 0;
        int rc = GAC_OK;
        hipError_t e = launch_whole_plan_sorted(cs->chains, n, nullptr, nullptr, nullptr, nullptr,
                                                cs->w_nblk, cs->w_gflat, nullptr, nullptr, nullptr,
                                                nullptr, tmp_bytes, s);
        if (e == hipSuccess) e = hipMalloc(&keys, 2 * n * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipMalloc(&vals, 3 * n * 4);
        perm = vals ? vals + n : nullptr;
        inv = vals ? vals + 2 * n : nullptr;
        if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 16));
        if (e == hipSuccess)
            e = launch_whole_plan_sorted(cs->chains, n, perm, keys, vals, cs->w_rdesc, cs->w_nblk,
                                         cs->w_gflat, cs->w_pb0, cs->w_tile_r0, inv, tmp,
                                         tmp_bytes, s);
        if (e == hipSuccess) e = hipMemcpyAsync(cs->w_perm, perm, n * 4, hipMemcpyDeviceToDevice, s);
        std::vector<int32_t> hinv(n);
        if (e == hipSuccess) e = hipMemcpyAsync(hinv.data(), inv, n * 4, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        std::vector<int32_t> empty;  // chains without blocks (inv -1): zeroed by every call
        for (int64_t i = 0; e == hipSuccess && i < n; ++i)
            if (hinv[i] < 0) empty.push_back((int32_t)i);
        cs->w_nempty = (int64_t)empty.size();
        if (e == hipSuccess && !empty.empty()) {
            e = hipMalloc(&cs->w_empty, empty.size() * 4);
            if (e == hipSuccess)
                e = hipMemcpy(cs->w_empty, empty.data(), empty.size() * 4, hipMemcpyHostToDevice);
        }
        if (e != hipSuccess) rc = gac_fail(GAC_E_HIP, "whole-chain plan: %s", hipGetErrorString(e));
        if (keys) hipFree(keys);
        if (vals) hipFree(vals);
        if (tmp) hipFree(tmp);
        if (rc != GAC_OK) return rc;
        cs->w_sorted = true;
        cs->w_ready = true;
        return GAC_OK;
    }
    HIPCHK(launch_whole_plan(cs->chains, n, cs->w_rdesc, cs->w_nblk, cs->w_gflat, cs->w_tile_r0, s));
    // k_tile's schedule: the tiles in the target order of their first
    // blocks (GAC_WHOLE_TILES=set: tile order), so that the tiles an XCD
    // scores at once share target plane lines in its L2 (chains are in score
    // order, so neighbouring tiles of the set are far apart on the target)
    static const bool tiles_set = [] {
        const char *e = getenv("GAC_WHOLE_TILES");
        return e && !strcmp(e, "set");
    }();
    if (!tiles_set && T > 1) {
        unsigned long long *keys = nullptr;
        int32_t *vals = nullptr;
        void *tmp = nullptr;
        size_t tmp_bytes = 0;
        hipError_t e = launch_tile_order(cs->chains, cs->blk, cs->w_tile_r0, T, nullptr, nullptr,
                                         nullptr, nullptr, tmp_bytes, s);
        if (e == hipSuccess) e = hipMalloc(&keys, 2 * T * sizeof(unsigned long long));
        if (e == hipSuccess) e = hipMalloc(&vals, T * 4);
        if (e == hipSuccess) e = hipMalloc(&cs->w_tile_perm, T * 4);
        if (e == hipSuccess) e = hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 16));
        if (e == hipSuccess)
            e = launch_tile_order(cs->chains, cs->blk, cs->w_tile_r0, T, keys, vals,
                                  cs->w_tile_perm, tmp, tmp_bytes, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (keys) hipFree(keys);
        if (vals) hipFree(vals);
        if (tmp) hipFree(tmp);
        if (e != hipSuccess) return gac_fail(GAC_E_HIP, "whole-chain tile order: %s", hipGetErrorString(e));
    }
    // chains without blocks: their results are zeroed by every call
    std::vector<int32_t> nblk(n);
    HIPCHK(hipMemcpyAsync(nblk.data(), cs->w_nblk, n * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<int32_t> empty;
    for (int64_t i = 0; i < n; ++i)
        if (nblk[i] == 0) empty.push_back((int32_t)i);
    cs->w_nempty = (int64_t)empty.size();
    if (!empty.empty()) {
        HIPCHK(hipMalloc(&cs->w_empty, empty.size() * 4));
        HIPCHK(hipMemcpy(cs->w_empty, empty.data(), empty.size() * 4, hipMemcpyHostToDevice));
    }
    cs->w_ready = true;
    return GAC_OK;
}

static int score_whole(gac_ctx *c, const gac_chainset *cs_in, uint32_t flags, long long *d_g,
                       long long *d_l, int32_t *d_ali, hipStream_t s) {
    gac_chainset *cs = const_cast<gac_chainset *>(cs_in);
    ScoreArgs a;
    if (c->ws_last && c->ws_last != s) HIPCHK(hipStreamWaitEvent(s, c->ws_ev, 0));
    int rc = prepare_args(c, cs, cs ? cs->n_chains : 0, flags, d_l, s, a);
    if (rc != GAC_OK || cs->n_chains == 0) return rc;
    if (cs->n_chains > INT32_MAX / 2) return gac_fail(GAC_E_ARG, "too many chains");
    rc = ensure_whole(c, cs, s);
    if (rc != GAC_OK) return rc;
    const int64_t T = (cs->n_blocks + kTileBlocks - 1) / kTileBlocks;
    rc = ensure_ws(c, 0, T, s);
    if (rc != GAC_OK) return rc;
    a.ranges = nullptr;
    a.out_g = d_g;
    a.out_l = d_l;
    a.out_ali = d_ali;
    a.rdesc = cs->w_rdesc;
    a.nblk = cs->w_nblk;
    a.gflat = cs->w_gflat;
    a.pb0 = cs->w_sorted ? cs->w_pb0 : cs->w_gflat;
    a.out_perm = cs->w_sorted ? cs->w_perm : nullptr;
    a.tile_perm = cs->w_sorted ? nullptr : cs->w_tile_perm;
    a.tile_r0 = cs->w_tile_r0;
    a.status = cs->w_status;
    a.sum_head = c->sum_head;
    a.sum_tail = c->sum_tail;
    a.sup_head = c->sup_head;
    a.sup_tail = c->sup_tail;
    a.sup_tail_r = c->sup_tail_r;
    a.cap_tiles = (int32_t)(c->ws_tiles < INT32_MAX ? c->ws_tiles : INT32_MAX);
    HIPCHK(launch_zero_list(cs->w_empty, cs->w_nempty, d_g, a.want_local ? d_l : nullptr, d_ali, s));
    {
        PROF_BEGIN(GAC_K_TILE);
        HIPCHK(launch_tile(a, c->tile_grid_sym[a.sym ? 1 : 0][a.want_local ? 1 : 0], s));
        PROF_END(GAC_K_TILE);
    }
    {
        PROF_BEGIN(GAC_K_COMBINE);
        HIPCHK(launch_combine(a, c->combine_grid, s));
        PROF_END(GAC_K_COMBINE);
    }
    if (hipEventRecord(c->ws_ev, s) == hipSuccess) c->ws_last = s;
    return GAC_OK;
}

extern "C" int gac_score_chains_device(gac_ctx *c, const gac_chainset *cs, uint32_t flags,
                                       int64_t *d_g, int64_t *d_l, int32_t *d_ali, void *stream) {
    gac_clear_error();
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    if (!cs) return gac_fail(GAC_E_ARG, "NULL chainset");
    if (cs->n_chains > 0 && (!d_g || !d_ali)) return gac_fail(GAC_E_ARG, "NULL buffer");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return score_whole(c, cs, flags, (long long *)d_g, (long long *)d_l, d_ali, s);
}

extern "C" int gac_score_chains(gac_ctx *c, const gac_chainset *cs, uint32_t flags, int64_t *global,
                                int64_t *local, int32_t *ali) {
    gac_clear_error();
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    if (!cs) return gac_fail(GAC_E_ARG, "NULL chainset");
    const int64_t n = cs->n_chains;
    if (n == 0) return GAC_OK;
    if (!global || !ali || ((flags & GAC_WANT_LOCAL) && !local)) return gac_fail(GAC_E_ARG, "NULL buffer");
    HIPCHK(hipSetDevice(c->device));
    if (n > c->io_n) {
        int64_t cap = n + n / 2 + 1024;
        if (c->d_ranges) hipFree(c->d_ranges);
        if (c->d_g) hipFree(c->d_g);
        if (c->d_l) hipFree(c->d_l);
        if (c->d_ali) hipFree(c->d_ali);
        c->d_ranges = nullptr;
        c->d_g = c->d_l = nullptr;
        c->d_ali = nullptr;
        HIPCHK(hipMalloc(&c->d_ranges, cap * sizeof(Range)));
        HIPCHK(hipMalloc(&c->d_g, cap * 8));
        HIPCHK(hipMalloc(&c->d_l, cap * 8));
        HIPCHK(hipMalloc(&c->d_ali, cap * 4));
        c->io_n = cap;
    }
    hipStream_t s = c->stream;
    int rc = score_whole(c, cs, flags, c->d_g, c->d_l, c->d_ali, s);
    if (rc != GAC_OK) return rc;
    HIPCHK(hipMemcpyAsync(global, c->d_g, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(ali, c->d_ali, n * 4, hipMemcpyDeviceToHost, s));
    if (flags & GAC_WANT_LOCAL) HIPCHK(hipMemcpyAsync(local, c->d_l, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return GAC_OK;
}

extern "C" int gac_score_ranges_device(gac_ctx *c, const gac_chainset *cs, const gac_range *d_ranges,
                                       int64_t n, uint32_t flags, int64_t *d_g, int64_t *d_l,
                                       int32_t *d_ali, void *stream) {
    gac_clear_error();
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    if (n > 0 && (!d_ranges || !d_g || !d_ali)) return gac_fail(GAC_E_ARG, "NULL buffer");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return score_device(c, cs, (const Range *)d_ranges, nullptr, n, flags, (long long *)d_g,
                        (long long *)d_l, d_ali, s);
}

extern "C" int gac_score_windows_device(gac_ctx *c, const gac_chainset *cs,
                                        const gac_window *d_wins, int64_t n, uint32_t flags,
                                        int64_t *d_g, int64_t *d_l, int32_t *d_ali, void *stream) {
    gac_clear_error();
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    if (n > 0 && (!d_wins || !d_g || !d_ali)) return gac_fail(GAC_E_ARG, "NULL buffer");
    HIPCHK(hipSetDevice(c->device));
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return score_device(c, cs, nullptr, (const Window *)d_wins, n, flags, (long long *)d_g,
                        (long long *)d_l, d_ali, s);
}

// ranges of chains given in host memory: planned here (window by binary
// search over the chain's block starts/ends), scored by k_small<HOST> reading
// the window records from pinned mapped memory, 256 ranges per launch
extern "C" int gac_score_ranges_host(gac_ctx *c, const gac_chainset_desc *d, const gac_range *r,
                                     int64_t n, uint32_t flags, int64_t *global, int64_t *local,
                                     int32_t *ali) {
    gac_clear_error();
    if (!c || !d) return gac_fail(GAC_E_ARG, "gac_score_ranges_host: NULL argument");
    CTX_LOCK_SMALL(c);
    if (!c->srv.on) srv_park(c);
    if (n < 0) return gac_fail(GAC_E_ARG, "negative range count");
    if (n == 0) return GAC_OK;
    if (!r || !global || !ali || ((flags & GAC_WANT_LOCAL) && !local))
        return gac_fail(GAC_E_ARG, "NULL buffer");
    if (!c->scoring) return gac_fail(GAC_E_STATE, "gac_set_scoring() not called");
    if (!c->g[0].final || !c->g[1].final)
        return gac_fail(GAC_E_STATE, "load both genomes before scoring");
    if (d->n_chains < 0 || d->n_blocks < 0 || !d->blk_off || !d->t_seq || !d->q_seq ||
        !d->q_strand || (d->n_blocks && (!d->blk_t || !d->blk_q || !d->blk_size)))
        return gac_fail(GAC_E_ARG, "gac_score_ranges_host: incomplete chain set descriptor");
    if (d->blk_off[0] != 0 || d->blk_off[d->n_chains] != d->n_blocks)
        return gac_fail(GAC_E_ARG, "gac_score_ranges_host: blk_off must run from 0 to n_blocks");
    HIPCHK(hipSetDevice(c->device));
    const bool srv = c->srv.on;  // the resident grid takes the batches
    if (srv) {
        const int rc = srv_ensure(c, nullptr, flags);
        if (rc != GAC_OK) return rc;
    } else if (!c->h_hq) {
        HIPCHK(hipHostMalloc((void **)&c->h_hq, kSmallMax * sizeof(RangeDesc), hipHostMallocMapped));
        HIPCHK(hipHostGetDevicePointer((void **)&c->d_hq, c->h_hq, 0));
    }
    const Genome &T = c->g[0], &Q = c->g[1];
    ScoreArgs a;
    memset(&a, 0, sizeof(a));
    a.t_planes = T.planes;
    a.t_nmask = T.nmask;
    a.t_woff = T.d_woff;
    a.q_planes = Q.planes;
    a.q_nmask = Q.nmask;
    a.q_woff = Q.d_woff;
    a.want_local = (flags & GAC_WANT_LOCAL) ? 1 : 0;
    a.gap_len = c->gap_len;
    a.gap_tab = c->d_gap_tab;
    a.small_tab = c->d_small;
    memcpy(a.coef, c->coef, sizeof(a.coef));
    a.sym = c->sym;
    a.gap = c->gap;
    hipStream_t s = c->stream;
    for (int64_t i0 = 0; i0 < n; i0 += kSmallMax) {
        const int64_t m = std::min<int64_t>(kSmallMax, n - i0);
        // windows (and their checks) first, to size the pool
        int64_t lo[kSmallMax], hi[kSmallMax], tot = 0;
        for (int64_t k = 0; k < m; ++k) {
            const gac_range &q = r[i0 + k];
            if (q.chain < 0 || q.chain >= d->n_chains)
                return gac_fail(GAC_E_ARG, "range %lld: chain %d out of range",
                                (long long)(i0 + k), q.chain);
            const int64_t b0 = d->blk_off[q.chain], b1 = d->blk_off[q.chain + 1];
            if (b0 < 0 || b0 > b1 || b1 > d->n_blocks)
                return gac_fail(GAC_E_ARG, "range %lld: chain %d has blocks [%lld, %lld) outside "
                                "[0, %lld)", (long long)(i0 + k), q.chain, (long long)b0,
                                (long long)b1, (long long)d->n_blocks);
            int64_t a0 = b0, a1 = b1;  // first block ending past s
            while (a0 < a1) {
                const int64_t mid = (a0 + a1) >> 1;
                if ((int64_t)d->blk_t[mid] + d->blk_size[mid] > q.t_start) a1 = mid;
                else a0 = mid + 1;
            }
            int64_t e0 = a0, e1 = b1;  // first block starting at or past e
            while (e0 < e1) {
                const int64_t mid = (e0 + e1) >> 1;
                if (d->blk_t[mid] >= q.t_end) e1 = mid;
                else e0 = mid + 1;
            }
            lo[k] = a0;
            hi[k] = std::max(a0, e0);
            tot += hi[k] - lo[k];
        }
        if (srv) {
            if (tot > c->srv.pool_cap) {  // (parks the grid to grow the pool)
                int rc = srv_pool(c, tot);
                if (rc != GAC_OK || (rc = srv_ensure(c, nullptr, flags)) != GAC_OK) return rc;
            }
        } else if (tot > c->pool_cap) {
            if (c->h_pool) hipHostFree(c->h_pool);
            c->h_pool = nullptr;
            c->pool_cap = 0;
            const int64_t cap = tot + tot / 2 + 1024;
            HIPCHK(hipHostMalloc((void **)&c->h_pool, cap * sizeof(int4), hipHostMallocMapped));
            HIPCHK(hipHostGetDevicePointer((void **)&c->d_pool, c->h_pool, 0));
            c->pool_cap = cap;
        }
        RangeDesc *hq = srv ? c->srv.h_hq : c->h_hq;
        int4 *pool = srv ? c->srv.h_pool : c->h_pool;
        int64_t j = 0;
        for (int64_t k = 0; k < m; ++k) {
            const gac_range &q = r[i0 + k];
            const int32_t ts = d->t_seq[q.chain], qs = d->q_seq[q.chain];
            if (ts < 0 || ts >= (int32_t)T.sizes.size() || qs < 0 || qs >= (int32_t)Q.sizes.size())
                return gac_fail(GAC_E_ARG, "chain %d: sequence index out of range", q.chain);
            const int64_t tsize = T.sizes[ts], qsize = Q.sizes[qs];
            RangeDesc &h = hq[k];
            h.tbase = T.woff[ts] * 32;
            const int64_t qw = Q.woff[qs] * 32;
            h.qbase = d->q_strand[q.chain] ? ~(qw + qsize) : qw;
            h.b0 = (int32_t)j;
            h.nblk = (int32_t)(hi[k] - lo[k]);
            h.s = q.t_start;
            h.e = q.t_end;
            int64_t pt = 0, pq = 0;
            for (int64_t b = lo[k]; b < hi[k]; ++b, ++j) {
                const int64_t t = d->blk_t[b], qq = d->blk_q[b], z = d->blk_size[b];
                if (z < 0 || z >= (1 << 29) || t < 0 || qq < 0 || t + z > tsize || qq + z > qsize ||
                    (b > lo[k] && (t < pt || qq < pq)))
                    return gac_fail(GAC_E_FORMAT, "chain %d: block [t %lld q %lld size %lld] "
                                    "outside its sequences or not ascending", q.chain,
                                    (long long)t, (long long)qq, (long long)z);
                pt = t + z;
                pq = qq + z;
                pool[j] = make_int4((int)t, (int)qq, (int)z, 0);
            }
        }
        if (srv) {
            const int rc = srv_call(c, 1, m);
            if (rc != GAC_OK) return rc;
            srv_results(c, m, flags, global + i0, local ? local + i0 : nullptr, ali + i0);
            continue;
        }
        a.n = m;
        HIPCHK(launch_small_host(a, c->d_hq, c->d_pool, c->d_small_out, s));
        HIPCHK(hipStreamSynchronize(s));
        for (int64_t k = 0; k < m; ++k) {
            const SmallOut o = c->h_small_out[k];
            global[i0 + k] = o.g;
            ali[i0 + k] = o.ali;
            if (flags & GAC_WANT_LOCAL) local[i0 + k] = o.l;
        }
    }
    return GAC_OK;
}

extern "C" int gac_score_ranges(gac_ctx *c, const gac_chainset *cs, const gac_range *ranges,
                                int64_t n, uint32_t flags, int64_t *global, int64_t *local,
                                int32_t *ali) {
    gac_clear_error();
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK_SMALL(c);
    if (n < 0) return gac_fail(GAC_E_ARG, "negative range count");
    if (n == 0) return GAC_OK;
    if (!ranges || !global || !ali || ((flags & GAC_WANT_LOCAL) && !local))
        return gac_fail(GAC_E_ARG, "NULL buffer");
    if (!cs) return gac_fail(GAC_E_ARG, "NULL chainset");
    if (n > c->small_max || !c->srv.on) srv_park(c);
    for (int64_t i = 0; i < n; ++i)
        if (ranges[i].chain < 0 || ranges[i].chain >= cs->n_chains)
            return gac_fail(GAC_E_ARG, "range %lld: chain %d out of range", (long long)i,
                            ranges[i].chain);
    HIPCHK(hipSetDevice(c->device));
    if (n <= c->small_max && c->srv.on) {  // a request to the resident grid
        if (!c->scoring) return gac_fail(GAC_E_STATE, "gac_set_scoring() not called");
        if (cs->ctx != c) return gac_fail(GAC_E_ARG, "chainset does not belong to this context");
        int rc = srv_ensure(c, cs, flags);
        if (rc != GAC_OK) return rc;
        memcpy(c->srv.h_in, ranges, (size_t)n * sizeof(Range));
        if ((rc = srv_call(c, 0, n)) != GAC_OK) return rc;
        srv_results(c, n, flags, global, local, ali);
        return GAC_OK;
    }
    if (n <= c->small_max) {
        // one launch; ranges in and results out through pinned host memory
        hipStream_t s = c->stream;
        ScoreArgs a;
        int rc = prepare_args(c, cs, n, flags, local, s, a);
        if (rc != GAC_OK) return rc;
        if ((rc = ensure_index(c, cs, s)) != GAC_OK) return rc;
        a.tspan = cs->tspan;  // (allocated with the index)
        a.bucket = cs->bucket;
        memcpy(c->h_small_in, ranges, (size_t)n * sizeof(Range));
        HIPCHK(launch_small(a, c->d_small_in, c->d_small_out, s));
        HIPCHK(hipStreamSynchronize(s));
        for (int64_t i = 0; i < n; ++i) {
            const SmallOut o = c->h_small_out[i];
            global[i] = o.g;
            ali[i] = o.ali;
            if (flags & GAC_WANT_LOCAL) local[i] = o.l;
        }
        return GAC_OK;
    }
    if (n > c->io_n) {
        int64_t cap = n + n / 2 + 1024;
        if (c->d_ranges) hipFree(c->d_ranges);
        if (c->d_g) hipFree(c->d_g);
        if (c->d_l) hipFree(c->d_l);
        if (c->d_ali) hipFree(c->d_ali);
        c->d_ranges = nullptr;
        c->d_g = c->d_l = nullptr;
        c->d_ali = nullptr;
        HIPCHK(hipMalloc(&c->d_ranges, cap * sizeof(Range)));
        HIPCHK(hipMalloc(&c->d_g, cap * 8));
        HIPCHK(hipMalloc(&c->d_l, cap * 8));
        HIPCHK(hipMalloc(&c->d_ali, cap * 4));
        c->io_n = cap;
    }
    hipStream_t s = c->stream;
    HIPCHK(hipMemcpyAsync(c->d_ranges, ranges, n * sizeof(Range), hipMemcpyHostToDevice, s));
    int rc = score_device(c, cs, c->d_ranges, nullptr, n, flags, c->d_g, c->d_l, c->d_ali, s);
    if (rc != GAC_OK) return rc;
    HIPCHK(hipMemcpyAsync(global, c->d_g, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(ali, c->d_ali, n * 4, hipMemcpyDeviceToHost, s));
    if (flags & GAC_WANT_LOCAL)
        HIPCHK(hipMemcpyAsync(local, c->d_l, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return GAC_OK;
}

extern "C" int gac_score_windows(gac_ctx *c, const gac_chainset *cs, const gac_window *wins,
                                 int64_t n, uint32_t flags, int64_t *global, int64_t *local,
                                 int32_t *ali) {
    gac_clear_error();
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    if (n < 0) return gac_fail(GAC_E_ARG, "negative window count");
    if (n == 0) return GAC_OK;
    if (!wins || !global || !ali || ((flags & GAC_WANT_LOCAL) && !local))
        return gac_fail(GAC_E_ARG, "NULL buffer");
    if (!cs) return gac_fail(GAC_E_ARG, "NULL chainset");
    HIPCHK(hipSetDevice(c->device));
    // the window records in the range staging buffer (20 B each: sized by
    // the 12-B ranges' capacity + one half)
    const int64_t need = (n * (int64_t)sizeof(Window) + sizeof(Range) - 1) / sizeof(Range);
    if (need > c->io_n) {
        int64_t cap = need + need / 2 + 1024;
        if (c->d_ranges) hipFree(c->d_ranges);
        if (c->d_g) hipFree(c->d_g);
        if (c->d_l) hipFree(c->d_l);
        if (c->d_ali) hipFree(c->d_ali);
        c->d_ranges = nullptr;
        c->d_g = c->d_l = nullptr;
        c->d_ali = nullptr;
        HIPCHK(hipMalloc(&c->d_ranges, cap * sizeof(Range)));
        HIPCHK(hipMalloc(&c->d_g, cap * 8));
        HIPCHK(hipMalloc(&c->d_l, cap * 8));
        HIPCHK(hipMalloc(&c->d_ali, cap * 4));
        c->io_n = cap;
    }
    hipStream_t s = c->stream;
    Window *d_w = reinterpret_cast<Window *>(c->d_ranges);
    HIPCHK(hipMemcpyAsync(d_w, wins, n * sizeof(Window), hipMemcpyHostToDevice, s));
    int rc = score_device(c, cs, nullptr, d_w, n, flags, c->d_g, c->d_l, c->d_ali, s);
    if (rc != GAC_OK) return rc;
    HIPCHK(hipMemcpyAsync(global, c->d_g, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(ali, c->d_ali, n * 4, hipMemcpyDeviceToHost, s));
    if (flags & GAC_WANT_LOCAL)
        HIPCHK(hipMemcpyAsync(local, c->d_l, n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return GAC_OK;
}

// ----------------------------------------------------------------- text (kent API)
// Caller-owned char text scored on the device (the kent in-process API's
// chainScoreBlock / axtScoreUngapped / cBlockFindCrossover take raw text):
// the batch's text is packed into one buffer, uploaded, scored, read back.
static M25 text_matrix(const int32_t mat[16]) {
    M25 m;
    memset(&m, 0, sizeof(m));
    for (int q = 0; q < 4; ++q)
        for (int t = 0; t < 4; ++t) m.m[q * 5 + t] = mat[q * 4 + t];
    return m;
}

template <class J>
static int text_run(gac_ctx *c, const std::vector<uint8_t> &text, const std::vector<J> &jobs,
                    size_t out_bytes, void **d_text, J **d_jobs, void **d_out) {
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMalloc(d_text, std::max<size_t>(text.size(), 1)));
    HIPCHK(hipMalloc((void **)d_jobs, jobs.size() * sizeof(J)));
    HIPCHK(hipMalloc(d_out, out_bytes));
    HIPCHK(hipMemcpyAsync(*d_text, text.data(), text.size(), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyAsync(*d_jobs, jobs.data(), jobs.size() * sizeof(J), hipMemcpyHostToDevice,
                          c->stream));
    return GAC_OK;
}

extern "C" int gac_score_text_blocks(gac_ctx *c, int64_t n, const char *const *q,
                                     const char *const *t, const int32_t *size,
                                     const int32_t mat[16], int64_t *score) {
    gac_clear_error();
    if (!c || n < 0 || (n && (!q || !t || !size || !mat || !score)))
        return gac_fail(GAC_E_ARG, "gac_score_text_blocks: bad argument");
    if (n == 0) return GAC_OK;
    CTX_LOCK(c);
    std::vector<TextJob> jobs(n);
    size_t tot = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (size[i] < 0) return gac_fail(GAC_E_ARG, "block %lld: negative size", (long long)i);
        tot += 2 * (size_t)size[i];
    }
    std::vector<uint8_t> text(tot);
    size_t o = 0;
    for (int64_t i = 0; i < n; ++i) {
        jobs[i] = TextJob{(int64_t)o, (int64_t)(o + size[i]), size[i], 0};
        memcpy(&text[o], q[i], size[i]);
        memcpy(&text[o + size[i]], t[i], size[i]);
        o += 2 * (size_t)size[i];
    }
    void *d_text = nullptr, *d_out = nullptr;
    TextJob *d_jobs = nullptr;
    int rc = text_run(c, text, jobs, n * 8, &d_text, &d_jobs, &d_out);
    if (rc == GAC_OK) {
        hipError_t e = launch_text_blocks((const uint8_t *)d_text, d_jobs, n, text_matrix(mat),
                                          (long long *)d_out, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(score, d_out, n * 8, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = gac_fail(GAC_E_HIP, "gac_score_text_blocks: %s", hipGetErrorString(e));
    }
    hipStreamSynchronize(c->stream);
    hipFree(d_text);
    hipFree(d_jobs);
    hipFree(d_out);
    return rc;
}

extern "C" int gac_text_crossovers(gac_ctx *c, int64_t n, const char *const *lq,
                                   const char *const *lt, const char *const *rq,
                                   const char *const *rt, const int32_t *overlap,
                                   const int32_t mat[16], int32_t *pos, int32_t *adj) {
    gac_clear_error();
    if (!c || n < 0 || (n && (!lq || !lt || !rq || !rt || !overlap || !mat || !pos || !adj)))
        return gac_fail(GAC_E_ARG, "gac_text_crossovers: bad argument");
    if (n == 0) return GAC_OK;
    CTX_LOCK(c);
    std::vector<TextXJob> jobs(n);
    size_t tot = 0;
    for (int64_t i = 0; i < n; ++i) {
        if (overlap[i] < 0) return gac_fail(GAC_E_ARG, "overlap %lld: negative", (long long)i);
        tot += 4 * (size_t)overlap[i];
    }
    std::vector<uint8_t> text(tot);
    size_t o = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t v = overlap[i];
        jobs[i] = TextXJob{(int64_t)o, (int64_t)(o + v), (int64_t)(o + 2 * (size_t)v),
                           (int64_t)(o + 3 * (size_t)v), v, 0};
        memcpy(&text[o], lq[i], v);
        memcpy(&text[o + v], lt[i], v);
        memcpy(&text[o + 2 * (size_t)v], rq[i], v);
        memcpy(&text[o + 3 * (size_t)v], rt[i], v);
        o += 4 * (size_t)v;
    }
    void *d_text = nullptr, *d_out = nullptr;
    TextXJob *d_jobs = nullptr;
    int rc = text_run(c, text, jobs, n * 8, &d_text, &d_jobs, &d_out);
    if (rc == GAC_OK) {
        int32_t *d_pos = (int32_t *)d_out, *d_adj = d_pos + n;
        hipError_t e = launch_text_xover((const uint8_t *)d_text, d_jobs, n, text_matrix(mat), d_pos,
                                         d_adj, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(pos, d_pos, n * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipMemcpyAsync(adj, d_adj, n * 4, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = gac_fail(GAC_E_HIP, "gac_text_crossovers: %s", hipGetErrorString(e));
    }
    hipStreamSynchronize(c->stream);
    hipFree(d_text);
    hipFree(d_jobs);
    hipFree(d_out);
    return rc;
}

// ----------------------------------------------------------------- memory
extern "C" int gac_dev_alloc(gac_ctx *c, size_t bytes, void **p) {
    if (!c || !p) return gac_fail(GAC_E_ARG, "NULL argument");
    HIPCHK(hipSetDevice(c->device));
    HIPCHK(hipMalloc(p, bytes ? bytes : 16));
    return GAC_OK;
}
extern "C" int gac_dev_free(gac_ctx *c, void *p) {
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    if (p) HIPCHK(hipFree(p));
    return GAC_OK;
}
extern "C" int gac_memcpy_h2d(gac_ctx *c, void *dst, const void *src, size_t n) {
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GAC_OK;
}
extern "C" int gac_memcpy_d2h(gac_ctx *c, void *dst, const void *src, size_t n) {
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    HIPCHK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return GAC_OK;
}
extern "C" int gac_synchronize(gac_ctx *c) {
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipDeviceSynchronize());
    return GAC_OK;
}

// ----------------------------------------------------------------- profiling
extern "C" int gac_prof_enable(gac_ctx *c, int on) {
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    c->prof = on & GAC_PROF_ALL;
    return GAC_OK;
}

static int prof_fold(gac_ctx *c) {
    for (auto &p : c->prof_pending) {
        HIPCHK(hipEventSynchronize(p.b));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, p.a, p.b));
        c->prof_ms[p.kernel] += ms;
        c->prof_n[p.kernel] += 1;
        c->prof_free.push_back(p.a);
        c->prof_free.push_back(p.b);
    }
    c->prof_pending.clear();
    return GAC_OK;
}

extern "C" int gac_prof_read(gac_ctx *c, int k, double *ms, int64_t *n) {
    if (!c || k < 0 || k >= GAC_K_COUNT) return gac_fail(GAC_E_ARG, "bad argument");
    CTX_LOCK(c);
    int rc = prof_fold(c);
    if (rc != GAC_OK) return rc;
    if (ms) *ms = c->prof_ms[k];
    if (n) *n = c->prof_n[k];
    return GAC_OK;
}

extern "C" int gac_prof_reset(gac_ctx *c) {
    if (!c) return gac_fail(GAC_E_ARG, "NULL context");
    CTX_LOCK(c);
    int rc = prof_fold(c);
    if (rc != GAC_OK) return rc;
    for (int k = 0; k < GAC_K_COUNT; ++k) {
        c->prof_ms[k] = 0;
        c->prof_n[k] = 0;
    }
    return GAC_OK;
}
