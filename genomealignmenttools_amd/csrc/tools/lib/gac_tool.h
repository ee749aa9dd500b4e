/* gac_tool.h -- shared host code of the drop-in CLI tools (C11):
 * kent-compatible option parsing (kent/src/lib/options.c:121-378),
 * errAbort semantics (message to stderr, exit 255; kent/src/lib/errAbort.c),
 * .chain reading/writing (kent/src/lib/chain.c:200-346) and chrom.sizes. */
#ifndef GAC_TOOL_H
#define GAC_TOOL_H

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>

#include "gachain.h"

#ifdef __cplusplus
extern "C" {
#endif

void gt_abort(const char *fmt, ...) __attribute__((noreturn, format(printf, 1, 2)));
void gt_verbose(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int gt_verbosity(void);
/* worker threads for host stages (GAC_THREADS, else OMP_NUM_THREADS, else
 * all cores; at most 64) */
int gt_threads(void);
/* run fn(args + i * stride) for i in [0, n) on n threads (0 on the caller) */
void gt_parallel(int n, void *(*fn)(void *), void *args, size_t stride);
/* -verbose>=2: wall time since the previous gt_stage call, labelled */
void gt_stage(const char *what);
void gt_check(int rc); /* abort with gac_last_error() unless GAC_OK */
/* fn runs once at the start of gt_abort (e.g. to tell other ranks) */
void gt_on_abort(void (*fn)(void));
/* device index gt_device_start opens (default 0) */
void gt_set_gpu(int gpu);
/* expose only that device to the runtime (ROCR_VISIBLE_DEVICES) unless a
 * visibility list is already set; main thread, before any HIP call (the
 * device start calls it) */
void gt_one_device(void);

/* ---- device bring-up off the critical path ----
 * gt_device_start opens device 0, sets the scoring scheme and uploads both
 * .2bit genomes on a helper thread, so that HIP runtime start-up and the
 * genome upload overlap the host's chain parsing / netting; gt_device_join
 * waits for it and returns the context (aborting with its error, like
 * gt_check).  mat and gap must stay valid until the join. */
struct gt_chains;
struct gt_names;

/* The genome word runs a tool's chains need (chainNet -rescore): the device
 * thread uploads only these (gac_genome_load_twobit_runs) once they are
 * ready.  Per side, CSR by sequence of the .2bit file. */
typedef struct gt_runs {
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int ready, ok;
    int64_t *off[2];
    int32_t *lo[2], *hi[2];
    int64_t words[2]; /* words uploaded (diagnostics) */
    double build_s;
} gt_runs;

typedef struct gt_device {
    const char *t2bit, *q2bit;
    const int32_t *mat;
    const gac_gapcalc *gap;
    gac_ctx *ctx;
    int rc, started, rc_err_set;
    double open_s, load_s, runs_wait_s;
    char err[1024];
    /* bring-up completion: the (detached) device thread sets done under mu
     * and broadcasts cv; any number of threads may wait for it */
    pthread_mutex_t mu;
    pthread_cond_t cv;
    int done;
    unsigned long close_th;
    int closing;
    const struct gt_names *tkeep; /* target sequences to load (NULL: all); -nranks */
    gt_runs *runs;                /* upload only these word runs (NULL: everything) */
} gt_device;
void gt_device_start(gt_device *d, const char *t2bit, const char *q2bit, const int32_t mat[16],
                     const gac_gapcalc *gap);
/* chainNet -rescore: compute the word runs under the blocks of c's chains
 * for the two .2bit files (on a helper thread) and publish them to R; the
 * device thread of a gt_device whose runs == R waits for them */
void gt_runs_init(gt_runs *R);
void gt_runs_build(gt_runs *R, const struct gt_chains *c, const char *t2bit, const char *q2bit);
/* the same, loading only the target sequences named in tkeep */
void gt_device_start_keep(gt_device *d, const char *t2bit, const char *q2bit,
                          const int32_t mat[16], const gac_gapcalc *gap,
                          const struct gt_names *tkeep);
/* the same with the genome uploads restricted to runs (NULL: all): the
 * device thread waits for gt_runs_build to publish them (ok == 0: upload
 * everything; an abort before they are built releases it) */
void gt_device_start_ex(gt_device *d, const char *t2bit, const char *q2bit, const int32_t mat[16],
                        const gac_gapcalc *gap, const struct gt_names *tkeep, gt_runs *runs);
/* main thread only */
gac_ctx *gt_device_join(gt_device *d);
/* the same wait without the abort: NULL if the bring-up failed.  Safe from
 * any thread and any number of times (it only waits for completion). */
gac_ctx *gt_device_wait(gt_device *d);
/* Helper threads that may be inside the HIP runtime: gt_abort/gt_exit_ok
 * join every registered thread (other than the caller) before the process
 * exits.  gt_helper_join joins one and unregisters it (main thread). */
void gt_helper_add(pthread_t th);
void gt_helper_join(pthread_t th);
/* Release a chain set and close the context on a helper thread (the host
 * writes its output meanwhile); gt_device_close_join waits for it. */
void gt_device_close_async(gt_device *d, gac_ctx *ctx, gac_chainset *cs);
void gt_device_close_join(gt_device *d);
/* Successful end of a tool once its outputs are closed and the device context
 * is released: flush stdio and leave without running exit-time destructors
 * (the HIP runtime's teardown of an already closed context, freeing of the
 * host arrays); the kernel reclaims both. */
void gt_exit_ok(void) __attribute__((noreturn));

/* ---- multi-GPU runs: -nranks=N -rank=R (one process per GPU, one node) ----
 * The ranks of a run share GAC_RANK_TOKEN (required with N > 1); every part
 * and marker file carries it.  A rank that fails leaves
 * <key>.gacpart<R>.<token>.failed; each rank also publishes
 * <key>.gacpart<R>.<token>.alive (boot id, pid namespace, pid), so a rank
 * waiting for a peer stops at once when the peer failed or its process is
 * gone, after GAC_RANK_START_TIMEOUT s (300) if the peer never started, and
 * after GAC_RANK_TIMEOUT s (3600) in all.  key = the first output file. */
typedef struct gt_ranks {
    int n, me;
    const char *key;
} gt_ranks;
/* checks n / me and the token, publishes this rank's liveness file and
 * installs the failure-marker hook (every rank) */
void gt_ranks_init(gt_ranks *rk, int n, int me, const char *key);
/* removes this rank's stale part of another output */
void gt_ranks_clear(const gt_ranks *rk, const char *path);
void gt_part_name(char *buf, size_t cap, const char *path, int r, const char *suffix);
/* end of a successful run: liveness files removed, failure hook off */
void gt_ranks_done(const gt_ranks *rk);
/* rank 0: wait until <path>.gacpart<r> exists for every r > 0 */
void gt_ranks_wait(const gt_ranks *rk, const char *path);
/* rank 0: append <path>.gacpart<r>, r = 1..n-1, to f, then remove them */
void gt_ranks_append_parts(const gt_ranks *rk, const char *path, FILE *f);
/* positioned parts: this rank's part of `path` (len bytes) written in place
 * at the sum of the lower ranks' sizes (rank 0 must have truncated `path`
 * before it calls this); rank 0 then waits for all parts (gt_ranks_finish).
 * gt_ranks_clear_markers removes this rank's stale markers at startup. */
void gt_ranks_clear_markers(const gt_ranks *rk, const char *path);
/* GAC_RANK_SOLO=1 (measurement only): ranks run alone, no rank waits for
 * another; a part goes to "<path>.solo<r>" (chainNet) or is dropped
 * (axtChain: rank 0 writes its own chains only) */
int gt_ranks_solo(void);
void gt_ranks_place(const gt_ranks *rk, const char *path, const char *buf, size_t len);
/* the same for a part held as n buffers (the buffers are left to the caller) */
void gt_ranks_place_bufs(const gt_ranks *rk, const char *path, char *const *bufs,
                         const size_t *lens, int64_t n);
void gt_ranks_finish(const gt_ranks *rk, const char *path);

/* ---- options ---- */
enum { GT_BOOL, GT_INT, GT_DOUBLE, GT_STRING };
typedef struct gt_spec {
    const char *name;
    int type;
} gt_spec;
/* Parse and remove options from argv (kent optionInit); "verbose" is always
 * accepted.  Unknown options abort. */
void gt_options(int *argc, char **argv, const gt_spec *spec);
/* optionHash (kent/src/lib/options.c:200-214): the same parsing, but any
 * option name is accepted (axtChain) */
void gt_options_hash(int *argc, char **argv);
/* forget the parsed options (a batch parses one command line per job) */
void gt_options_reset(void);
const char *gt_opt_str(const char *name, const char *def);
int gt_opt_exists(const char *name);
int gt_opt_int(const char *name, int def);
double gt_opt_double(const char *name, double def);

/* ---- kent hash iteration order (kent/src/lib/hash.c) ----
 * Tools whose output order follows a kent hash traversal (hashTraverseEls,
 * hashElListHash) keep the same order by replaying the hash: hashString of
 * the key text (:41-53), head insertion into bucket hashVal & mask
 * (:115-141), doubling when elCount > size (defaultExpansionFactor 1.0) with
 * the bucket lists re-reversed into insertion order (:424-470), default size
 * 2^12 (:355-367).  Keys here are ints printed "%d" (chainCleaner's keys). */
typedef struct gt_khash {
    int pow;
    uint32_t mask;
    int32_t *head;  /* [1 << pow] first element of each bucket, -1 = empty */
    int32_t *next;  /* per element */
    uint32_t *hv;   /* per element: hashString of the key text */
    int32_t *key;   /* per element */
    int32_t n, cap;
} gt_khash;
void gt_khash_init(gt_khash *h, int pow); /* pow 0 = kent's default 12 */
int32_t gt_khash_find(const gt_khash *h, int32_t key); /* element or -1 */
int32_t gt_khash_add(gt_khash *h, int32_t key);        /* new element (no dedupe) */
/* elements in hashTraverseEls order; returns the count */
int32_t gt_khash_order(const gt_khash *h, int32_t *out);
void gt_khash_free(gt_khash *h);

/* ---- string table ---- */
typedef struct gt_names {
    char **names;
    int32_t n, cap;
    int32_t *slots;  /* open addressing, -1 = empty */
    int32_t nslot;
} gt_names;
int32_t gt_names_add(gt_names *t, const char *s, size_t len);
int32_t gt_names_find(const gt_names *t, const char *s);
void gt_names_free(gt_names *t);

/* ---- chains (struct of arrays) ---- */
typedef struct gt_chains {
    int64_t n, cap;
    double *score;
    int32_t *tname, *tsize, *tstart, *tend; /* tname: index into tnames */
    int32_t *qname, *qsize, *qstart, *qend;
    uint8_t *qstrand;
    int32_t *id;
    int64_t *blk_off; /* n + 1 */
    int64_t nb, bcap;
    int32_t *bt, *bq, *bs;
    gt_names tnames, qnames;
    char **meta; /* '#' lines in order */
    int64_t *meta_at; /* the chain whose read consumed meta[k] (n: the read that hit EOF) */
    int32_t n_meta, meta_cap;
} gt_chains;

/* Before exit: drop the pages of a chain set's arrays on several threads
 * (madvise under the mm's read lock; the kernel's exit would free them on
 * one core).  The set must not be used afterwards. */
void gt_chains_drop_pages(gt_chains *c);
/* the block arrays' pages dropped now on a detached thread (the caller no
 * longer reads bt/bq/bs; the arrays stay allocated); GAC_EARLY_FREE=0: not */
void gt_chains_drop_blocks_async(gt_chains *c);
/* large temporary arrays released later, off the critical path: with
 * GAC_LATE_FREE=1 (default) gt_free_late keeps them until gt_free_late_all,
 * which drops their pages on all threads (madvise, read lock) and frees
 * them; otherwise gt_free_late frees at once */
void gt_free_late(void *p, size_t bytes);
void gt_free_late_all(void);

/* stop_below: stop after reading the first chain whose score is < stop_below
 * (that chain is read, like chainNet's loop, but not kept); pass -HUGE_VAL
 * to read everything.  Reads .gz transparently, "stdin" allowed. */
void gt_read_chains(const char *path, gt_chains *c, double stop_below, int keep_meta);
/* Same, but a chain whose target name is not in tkeep and whose query name is
 * not in qkeep keeps its header only (no blocks; its block lines are not
 * parsed): chainNet -nranks, where a rank nets some chromosome sides.  Ids,
 * the minScore stop, '#' lines and header errors are as for every chain. */
void gt_read_chains_keep(const char *path, gt_chains *c, double stop_below, int keep_meta,
                         const gt_names *tkeep, const gt_names *qkeep);
void gt_chains_free(gt_chains *c);
/* chainIdNext (chain.c:180-198): the shared "next id" counter */
int gt_next_chain_id(void);
/* 1: gt_read_chains leaves header ids absent from the text as INT32_MIN, for
 * a caller that consumes chainIdNext in its own read order (chainMergeSort) */
void gt_defer_chain_ids(int on);
/* chainWrite (chain.c:200-227) of chain i with the given score and id */
void gt_write_chain(FILE *f, const gt_chains *c, int64_t i, double score, int32_t id);
/* chainWrite of an explicit header and block list */
void gt_write_chain_raw(FILE *f, double score, const char *tname, int32_t tsize, int32_t tstart,
                        int32_t tend, const char *qname, int32_t qsize, int qminus,
                        int32_t qstart, int32_t qend, int32_t id, const int32_t *bt,
                        const int32_t *bq, const int32_t *bs, int64_t nb);

/* sequence index (gac_genome_seq_index) of every name of a chain file's
 * name table, -1 where absent (malloc'ed) */
int32_t *gt_seq_map(gac_ctx *ctx, int side, const gt_names *names);

/* Ordered parallel output: items [0, n) are cut into contiguous runs, each
 * printed by fn(f, i, arg) into a per-run memory stream on gt_threads()
 * threads, and the runs are written to out in order (the bytes equal a
 * sequential loop's). */
void gt_par_write(FILE *out, int64_t n, void (*fn)(FILE *f, int64_t i, void *arg), void *arg);

/* ---- chrom.sizes ---- */
typedef struct gt_sizes {
    gt_names names;
    int32_t *size;
} gt_sizes;
void gt_read_sizes(const char *path, gt_sizes *s);
void gt_sizes_free(gt_sizes *s);

FILE *gt_must_open(const char *path, const char *mode);
/* whole file (".gz" decompressed, "stdin" allowed) into a NUL-terminated buffer */
char *gt_slurp(const char *path, size_t *len);
void gt_careful_close(FILE *f, const char *path);
int gt_file_exists(const char *path);

#ifdef __cplusplus
}
#endif
#endif
