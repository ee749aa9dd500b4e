/* gac_tool.c -- shared host code of the drop-in CLI tools (see gac_tool.h). */
#define _GNU_SOURCE
#include "gac_tool.h"
#include "host/gac_host.h"

#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <math.h>
#include <stdarg.h>
#include <stdlib.h>
#include <string.h>
#include <signal.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <sys/resource.h>
#include <unistd.h>
#include <sys/syscall.h>
#include <pthread.h>
#include <stdatomic.h>
#include <malloc.h>
#include <sys/mman.h>
#include <time.h>
#include <zlib.h>

/* ------------------------------------------------------------ errors */
static int g_verbose = 1;
static void *g_live_dev; /* gt_device whose helper thread may still run HIP calls */
static void join_live_device(void);

static void (*g_abort_hook)(void);
void gt_on_abort(void (*fn)(void)) { g_abort_hook = fn; }

static int g_gpu; /* device index for gt_device_start */
void gt_set_gpu(int gpu) { g_gpu = gpu; }

/* One thread aborts the process; a helper that aborts too ends itself (so
 * that joins of it return), the main thread waits for the exit. */
static atomic_int g_aborting;

static void abort_second(void) {
    if (syscall(SYS_gettid) == getpid())
        for (;;)
            pause();
    pthread_exit(NULL);
}

void gt_abort(const char *fmt, ...) {
    if (atomic_exchange(&g_aborting, 1))
        abort_second();
    va_list ap;
    void (*hook)(void) = g_abort_hook;
    g_abort_hook = NULL; /* (a failing hook must not recurse) */
    if (hook)
        hook();
    gac_outputs_cut(); /* (no net left holding an earlier run's tail) */
    join_live_device(); /* never exit under a thread that is inside the HIP runtime */
    fflush(stdout);
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
    size_t n = strlen(fmt);
    if (n == 0 || fmt[n - 1] != '\n')
        fputc('\n', stderr);
    exit(255); /* errAbort -> exit(-1) */
}

void gt_verbose(int level, const char *fmt, ...) {
    if (level > g_verbose)
        return;
    va_list ap;
    va_start(ap, fmt);
    vfprintf(stderr, fmt, ap);
    va_end(ap);
}

int gt_verbosity(void) { return g_verbose; }

/* seconds since this process started (/proc/self/stat starttime, clock
 * ticks since boot, against CLOCK_BOOTTIME); -1 if unavailable */
static double since_process_start(void) {
    FILE *f = fopen("/proc/self/stat", "r");
    if (!f)
        return -1;
    char buf[1024];
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = 0;
    const char *p = strrchr(buf, ')'); /* the command name may hold spaces */
    if (!p)
        return -1;
    unsigned long long start = 0;
    /* fields after ")": state is field 3, starttime is field 22 */
    if (sscanf(p + 2, "%*c %*d %*d %*d %*d %*d %*u %*u %*u %*u %*u %*u %*u %*d %*d %*d %*d %*d %*d %llu",
               &start) != 1)
        return -1;
    struct timespec ts;
    clock_gettime(CLOCK_BOOTTIME, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec - (double)start / (double)sysconf(_SC_CLK_TCK);
}

void gt_stage(const char *what) {
    static double last = -1;
    static int env = -1; /* GAC_TIMING prints the stages at any verbosity */
    if (env < 0)
        env = getenv("GAC_TIMING") != NULL;
    const int show = g_verbose >= 2 || env;
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    const double now = ts.tv_sec + 1e-9 * ts.tv_nsec;
    static double startup = -2; /* process start -> first call (main's entry) */
    static double main_rt;      /* CLOCK_REALTIME at main's entry */
    if (startup == -2) {
        startup = since_process_start();
        struct timespec rt;
        clock_gettime(CLOCK_REALTIME, &rt);
        main_rt = rt.tv_sec + 1e-9 * rt.tv_nsec;
    }
    if (last >= 0 && what && show && startup > -2) {
        /* wall-clock anchors: a parent can attribute spawn and exit */
        fprintf(stderr, "[stage-clock] main %.6f process-start %.6f\n", main_rt, main_rt - startup);
        fprintf(stderr, "[stage] %-32s %8.3f s\n", "exec + libraries (approx.)", startup);
        startup = -3;
    }
    /* the process's CPU time over the stage: cpu / wall = the threads it kept
     * busy on average (the headroom a stage leaves in the CPU quota) */
    struct timespec cs;
    clock_gettime(CLOCK_PROCESS_CPUTIME_ID, &cs);
    const double cpu = cs.tv_sec + 1e-9 * cs.tv_nsec;
    static double last_cpu = 0;
    /* and its system time and page faults (first touches of new memory) */
    struct rusage ru;
    getrusage(RUSAGE_SELF, &ru);
    const double sys = ru.ru_stime.tv_sec + 1e-6 * ru.ru_stime.tv_usec;
    static double last_sys = 0;
    static long last_flt = 0;
    if (last >= 0 && what && show)
        fprintf(stderr, "[stage] %-32s %8.3f s  (cpu %.3f s, %.1f busy; sys %.3f s, %ld faults)\n", what,
                now - last, cpu - last_cpu, now > last ? (cpu - last_cpu) / (now - last) : 0.0,
                sys - last_sys, ru.ru_minflt - last_flt);
    last = now;
    last_cpu = cpu;
    last_sys = sys;
    last_flt = ru.ru_minflt;
}

static double now_s(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* the two .2bit files mapped (page tables populated) while the HIP
 * runtime starts on the device thread */
typedef struct twobit_pre {
    const char *path[2];
    gac_twobit tb[2];
    int rc[2];
    char err[2][512];
} twobit_pre;

static void *twobit_pre_thread(void *arg) {
    twobit_pre *P = arg;
    for (int k = 0; k < 2; ++k) {
        P->rc[k] = gac_twobit_open_ex(P->path[k], &P->tb[k], 1);
        if (P->rc[k] != GAC_OK)
            snprintf(P->err[k], sizeof(P->err[k]), "%s", gac_last_error());
    }
    return NULL;
}

static void *device_thread(void *arg) {
    gt_device *d = arg;
    const double t0 = now_s();
    twobit_pre P;
    memset(&P, 0, sizeof(P));
    P.path[0] = d->t2bit;
    P.path[1] = d->q2bit;
    pthread_t pre;
    const int pre_ok = pthread_create(&pre, NULL, twobit_pre_thread, &P) == 0;
    if (!pre_ok)
        twobit_pre_thread(&P);
    int rc = gac_open(g_gpu, &d->ctx);
    d->open_s = now_s() - t0;
    if (rc == GAC_OK && d->mat)
        rc = gac_set_scoring(d->ctx, d->mat, d->gap);
    if (pre_ok)
        pthread_join(pre, NULL);
    for (int k = 0; k < 2; ++k) {
        if (rc == GAC_OK && P.rc[k] != GAC_OK) {
            rc = P.rc[k];
            snprintf(d->err, sizeof(d->err), "%s", P.err[k]);
            d->rc_err_set = 1;
        }
        uint8_t *keep = NULL;
        if (rc == GAC_OK && k == 0 && d->tkeep) {
            keep = malloc(P.tb[k].seq_count + 1);
            for (uint32_t i = 0; i < P.tb[k].seq_count; ++i)
                keep[i] = gt_names_find(d->tkeep, P.tb[k].seqs[i].name) >= 0;
        }
        const gt_runs *R = NULL;
        if (rc == GAC_OK && d->runs) { /* the word runs the chains need */
            const double w0 = now_s();
            pthread_mutex_lock(&d->runs->mu);
            while (!d->runs->ready)
                pthread_cond_wait(&d->runs->cv, &d->runs->mu);
            pthread_mutex_unlock(&d->runs->mu);
            d->runs_wait_s += now_s() - w0;
            if (d->runs->ok < 0) { /* the tool is aborting: skip the upload */
                gac_twobit_close(&P.tb[k]);
                free(keep);
                continue;
            }
            if (d->runs->ok)
                R = d->runs;
        }
        if (rc == GAC_OK)
            rc = gac_genome_load_twobit_runs(d->ctx, k == 0 ? GAC_T : GAC_Q, &P.tb[k], keep,
                                             R ? R->off[k] : NULL, R ? R->lo[k] : NULL,
                                             R ? R->hi[k] : NULL);
        else if (P.rc[k] == GAC_OK)
            gac_twobit_close(&P.tb[k]);
        free(keep);
    }
    d->load_s = now_s() - t0 - d->open_s;
    if (rc != GAC_OK && !d->rc_err_set) /* the error text is thread-local */
        snprintf(d->err, sizeof(d->err), "%s", gac_last_error());
    pthread_mutex_lock(&d->mu);
    d->rc = rc;
    d->done = 1;
    pthread_cond_broadcast(&d->cv);
    pthread_mutex_unlock(&d->mu);
    return NULL;
}

/* ---- genome word runs under the chains' blocks (gt_runs) */
void gt_runs_init(gt_runs *R) {
    memset(R, 0, sizeof(*R));
    pthread_mutex_init(&R->mu, NULL);
    pthread_cond_init(&R->cv, NULL);
}

typedef struct runs_mark {
    const gt_chains *c;
    const int32_t *tmap, *qmap;     /* chain name index -> .2bit sequence */
    const int64_t *twoff, *qwoff;   /* first word of each .2bit sequence (bitmap space) */
    const int32_t *tsize, *qsize;
    _Atomic uint64_t *tbits, *qbits;
    _Atomic int64_t next;
} runs_mark;

/* set bits [w0, w1): one atomic OR per 64-bit bitmap word, skipped when its
 * bits are set already (dense regions are marked by many chains) */
static void mark_words(_Atomic uint64_t *bits, int64_t w0, int64_t w1) {
    for (int64_t i = w0 >> 6; w0 < w1; ++i) {
        const int64_t hi = (i + 1) << 6 < w1 ? (i + 1) << 6 : w1;
        const int lo_b = (int)(w0 & 63), n = (int)(hi - w0);
        const uint64_t m = (n == 64 ? ~0ull : ((1ull << n) - 1ull)) << lo_b;
        if ((atomic_load_explicit(&bits[i], memory_order_relaxed) & m) != m)
            atomic_fetch_or_explicit(&bits[i], m, memory_order_relaxed);
        w0 = hi;
    }
}

/* a chain's word intervals on one side, merged while they touch (the blocks
 * of a chain are co-linear: mostly one interval per run of close blocks) */
typedef struct word_span {
    int64_t a, b; /* pending [a, b), a == b: none */
} word_span;

static void span_add(word_span *p, _Atomic uint64_t *bits, int64_t a, int64_t b) {
    if (p->a < p->b && a <= p->b && b >= p->a) {
        p->a = a < p->a ? a : p->a;
        p->b = b > p->b ? b : p->b;
        return;
    }
    if (p->a < p->b)
        mark_words(bits, p->a, p->b);
    p->a = a;
    p->b = b;
}

static void *runs_mark_thread(void *arg) {
    runs_mark *M = arg;
    const gt_chains *c = M->c;
    for (;;) {
        const int64_t a = atomic_fetch_add(&M->next, 1024);
        if (a >= c->n)
            break;
        const int64_t b = a + 1024 < c->n ? a + 1024 : c->n;
        for (int64_t i = a; i < b; ++i) {
            const int32_t ts = M->tmap[c->tname[i]], qs = M->qmap[c->qname[i]];
            word_span pt = {0, 0}, pq = {0, 0};
            for (int64_t k = c->blk_off[i]; k < c->blk_off[i + 1]; ++k) {
                const int64_t z = c->bs[k];
                if (z <= 0)
                    continue;
                if (ts >= 0) { /* the kernel reads the block's words and the next one */
                    const int64_t t = c->bt[k];
                    const int64_t nw = ((int64_t)M->tsize[ts] + 31) / 32;
                    const int64_t w1 = ((t + z - 1) >> 5) + 2;
                    span_add(&pt, M->tbits, M->twoff[ts] + (t >> 5), M->twoff[ts] + (w1 < nw ? w1 : nw));
                }
                if (qs >= 0) { /* '-': the forward coordinates of the block */
                    const int64_t q = c->bq[k], qz = M->qsize[qs];
                    const int64_t f0 = c->qstrand[i] ? qz - (q + z) : q, f1 = f0 + z;
                    const int64_t nw = (qz + 31) / 32;
                    const int64_t w1 = ((f1 - 1) >> 5) + 2;
                    span_add(&pq, M->qbits, M->qwoff[qs] + (f0 >> 5), M->qwoff[qs] + (w1 < nw ? w1 : nw));
                }
            }
            if (pt.a < pt.b)
                mark_words(M->tbits, pt.a, pt.b);
            if (pq.a < pq.b)
                mark_words(M->qbits, pq.a, pq.b);
        }
    }
    return NULL;
}

/* runs of set bits of each sequence, CSR by sequence; runs less than `gap`
 * words apart are merged (fewer, longer copies: the upload's cost per run
 * outweighs a few KB of extra bases) */
static void bits_to_runs(const _Atomic uint64_t *bits, const int64_t *woff, int32_t nseq,
                         int64_t gap, int64_t **off_out, int32_t **lo_out, int32_t **hi_out,
                         int64_t *words) {
    int64_t *off = malloc((size_t)(nseq + 1) * 8), cap = 1024, n = 0;
    int32_t *lo = malloc((size_t)cap * 4), *hi = malloc((size_t)cap * 4);
    *words = 0;
    for (int32_t s = 0; s < nseq; ++s) {
        off[s] = n;
        int64_t w = woff[s];
        const int64_t end = woff[s + 1];
        while (w < end) {
            const uint64_t x = atomic_load_explicit(&bits[w >> 6], memory_order_relaxed) >> (w & 63);
            if (!x) { /* skip the rest of this 64-bit word */
                w = (w | 63) + 1;
                continue;
            }
            w += __builtin_ctzll(x);
            if (w >= end)
                break;
            const int64_t r0 = w;
            for (;;) { /* to the next clear bit (or the sequence's end) */
                const uint64_t y = ~atomic_load_explicit(&bits[w >> 6], memory_order_relaxed) >> (w & 63);
                if (y) {
                    w += __builtin_ctzll(y);
                    break;
                }
                w = (w | 63) + 1;
                if (w >= end)
                    break;
            }
            if (w > end)
                w = end;
            if (n > off[s] && r0 - (woff[s] + hi[n - 1]) < gap) { /* close to the last run */
                *words += w - (woff[s] + hi[n - 1]);
                hi[n - 1] = (int32_t)(w - woff[s]);
                continue;
            }
            if (n == cap) {
                cap *= 2;
                lo = realloc(lo, (size_t)cap * 4);
                hi = realloc(hi, (size_t)cap * 4);
            }
            lo[n] = (int32_t)(r0 - woff[s]);
            hi[n] = (int32_t)(w - woff[s]);
            *words += w - r0;
            ++n;
        }
    }
    off[nseq] = n;
    *off_out = off;
    *lo_out = lo;
    *hi_out = hi;
}

void gt_runs_build(gt_runs *R, const gt_chains *c, const char *t2bit, const char *q2bit) {
    const double t0 = now_s();
    gac_twobit tb[2];
    int ok = gac_twobit_open_ex(t2bit, &tb[0], 0) == GAC_OK;
    if (ok && gac_twobit_open_ex(q2bit, &tb[1], 0) != GAC_OK) {
        gac_twobit_close(&tb[0]);
        ok = 0;
    }
    if (ok) {
        int64_t *woff[2];
        int32_t *size[2], *map[2];
        _Atomic uint64_t *bits[2];
        const gt_names *cn[2] = {&c->tnames, &c->qnames};
        for (int k = 0; k < 2; ++k) {
            const int32_t ns = (int32_t)tb[k].seq_count;
            gt_names fn;
            memset(&fn, 0, sizeof(fn));
            woff[k] = malloc((size_t)(ns + 1) * 8);
            size[k] = malloc((size_t)(ns ? ns : 1) * 4);
            woff[k][0] = 0;
            for (int32_t i = 0; i < ns; ++i) {
                gt_names_add(&fn, tb[k].seqs[i].name, strlen(tb[k].seqs[i].name));
                size[k][i] = (int32_t)tb[k].seqs[i].size;
                woff[k][i + 1] = woff[k][i] + ((int64_t)tb[k].seqs[i].size + 31) / 32;
            }
            map[k] = malloc((size_t)(cn[k]->n ? cn[k]->n : 1) * 4);
            for (int32_t j = 0; j < cn[k]->n; ++j)
                map[k][j] = gt_names_find(&fn, cn[k]->names[j]);
            gt_names_free(&fn);
            bits[k] = calloc((size_t)(woff[k][ns] / 64 + 2), 8);
        }
        runs_mark M = {c, map[0], map[1], woff[0], woff[1], size[0], size[1], bits[0], bits[1], 0};
        atomic_init(&M.next, 0);
        /* a few threads: this runs beside the netting, off the critical path */
        gac_run_threads(gt_threads() < 4 ? gt_threads() : 4, runs_mark_thread, &M);
        const char *gs = getenv("GAC_RUN_GAP"); /* words (32 bases); default 64 */
        const int64_t gap = gs && *gs ? atoll(gs) : 64;
        for (int k = 0; k < 2; ++k) {
            bits_to_runs(bits[k], woff[k], (int32_t)tb[k].seq_count, gap, &R->off[k], &R->lo[k],
                         &R->hi[k], &R->words[k]);
            free(bits[k]);
            free(woff[k]);
            free(size[k]);
            free(map[k]);
            gac_twobit_close(&tb[k]);
        }
    }
    pthread_mutex_lock(&R->mu);
    R->build_s = now_s() - t0;
    R->ok = ok;
    R->ready = 1;
    pthread_cond_broadcast(&R->cv);
    pthread_mutex_unlock(&R->mu);
}

/* A tool drives one device: unless the caller chose the visible devices,
 * show the runtime only that one, so that its start-up initialises one GPU
 * rather than every GPU of the node.  Before any HIP call and before other
 * threads run (setenv); idempotent. */
void gt_one_device(void) {
    if (getenv("ROCR_VISIBLE_DEVICES") || getenv("HIP_VISIBLE_DEVICES") ||
        getenv("CUDA_VISIBLE_DEVICES") || getenv("GPU_DEVICE_ORDINAL") ||
        getenv("GAC_ALL_DEVICES") || g_gpu < 0)
        return;
    char b[16];
    snprintf(b, sizeof(b), "%d", g_gpu);
    setenv("ROCR_VISIBLE_DEVICES", b, 1);
    g_gpu = 0;
}

void gt_device_start(gt_device *d, const char *t2bit, const char *q2bit, const int32_t mat[16],
                     const gac_gapcalc *gap) {
    gt_device_start_ex(d, t2bit, q2bit, mat, gap, NULL, NULL);
}

void gt_device_start_keep(gt_device *d, const char *t2bit, const char *q2bit,
                          const int32_t mat[16], const gac_gapcalc *gap, const gt_names *tkeep) {
    gt_device_start_ex(d, t2bit, q2bit, mat, gap, tkeep, NULL);
}

void gt_device_start_ex(gt_device *d, const char *t2bit, const char *q2bit, const int32_t mat[16],
                        const gac_gapcalc *gap, const gt_names *tkeep, gt_runs *runs) {
    gt_one_device();
    memset(d, 0, sizeof(*d));
    d->tkeep = tkeep;
    d->runs = runs;
    d->t2bit = t2bit;
    d->q2bit = q2bit;
    d->mat = mat;
    d->gap = gap;
    pthread_mutex_init(&d->mu, NULL);
    pthread_cond_init(&d->cv, NULL);
    pthread_attr_t at;
    pthread_attr_init(&at);
    pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
    pthread_t th;
    if (pthread_create(&th, &at, device_thread, d) != 0)
        gt_abort("can't start the device thread\n");
    pthread_attr_destroy(&at);
    d->started = 1;
    g_live_dev = d;
}

/* wait until the bring-up thread has left the HIP runtime */
static void device_wait_done(gt_device *d) {
    pthread_mutex_lock(&d->mu);
    while (!d->done)
        pthread_cond_wait(&d->cv, &d->mu);
    pthread_mutex_unlock(&d->mu);
}

/* registered helper threads (gt_helper_add); touched by the main thread only */
#define GT_MAX_HELPERS 8
static pthread_t g_helpers[GT_MAX_HELPERS];
static int g_n_helpers;

void gt_helper_add(pthread_t th) {
    if (g_n_helpers == GT_MAX_HELPERS)
        gt_abort("gt_helper_add: too many helper threads\n");
    g_helpers[g_n_helpers++] = th;
}

void gt_helper_join(pthread_t th) {
    for (int i = 0; i < g_n_helpers; ++i)
        if (pthread_equal(g_helpers[i], th)) {
            g_helpers[i] = g_helpers[--g_n_helpers];
            break;
        }
    pthread_join(th, NULL);
}

static void join_live_device(void) {
    /* helpers first: they may be waiting for the device themselves */
    for (int i = 0; i < g_n_helpers; ++i)
        if (!pthread_equal(pthread_self(), g_helpers[i]))
            pthread_join(g_helpers[i], NULL);
    g_n_helpers = 0;
    gt_device *d = g_live_dev;
    if (d && d->closing && !pthread_equal(pthread_self(), (pthread_t)d->close_th)) {
        pthread_join((pthread_t)d->close_th, NULL);
        d->closing = 0;
    }
    if (d && d->started && d->runs) { /* never built (an early abort): let it go */
        pthread_mutex_lock(&d->runs->mu);
        if (!d->runs->ready) {
            d->runs->ready = 1;
            d->runs->ok = -1;
            pthread_cond_broadcast(&d->runs->cv);
        }
        pthread_mutex_unlock(&d->runs->mu);
    }
    if (d && d->started)
        device_wait_done(d);
    g_live_dev = NULL;
}

gac_ctx *gt_device_wait(gt_device *d) {
    if (!d->started)
        return NULL;
    device_wait_done(d);
    return d->rc == GAC_OK ? d->ctx : NULL;
}

gac_ctx *gt_device_join(gt_device *d) {
    if (!d->started)
        gt_abort("gt_device_join: device never started\n");
    device_wait_done(d);
    if (d->rc != GAC_OK)
        gt_abort("%s\n", d->err);
    if (d->runs)
        gt_verbose(2, "[stage] (overlapped) device open %.3f s, 2bit genomes to HBM %.3f s "
                      "(of which waiting for the word runs %.3f s; runs built in %.3f s, %lld + %lld words)\n",
                   d->open_s, d->load_s, d->runs_wait_s, d->runs->build_s,
                   (long long)d->runs->words[0], (long long)d->runs->words[1]);
    else
        gt_verbose(2, "[stage] (overlapped) device open %.3f s, 2bit genomes to HBM %.3f s\n",
                   d->open_s, d->load_s);
    return d->ctx;
}

typedef struct close_job {
    gac_ctx *ctx;
    gac_chainset *cs;
} close_job;

static void *close_thread(void *arg) {
    close_job *j = arg;
    gac_chains_free(j->cs);
    gac_close(j->ctx);
    free(j);
    return NULL;
}

void gt_device_close_async(gt_device *d, gac_ctx *ctx, gac_chainset *cs) {
    close_job *j = malloc(sizeof(*j));
    j->ctx = ctx;
    j->cs = cs;
    pthread_t th;
    if (pthread_create(&th, NULL, close_thread, j) != 0) {
        close_thread(j);
        return;
    }
    d->close_th = (unsigned long)th;
    d->closing = 1;
    g_live_dev = d; /* gt_abort joins it before exiting */
}

void gt_device_close_join(gt_device *d) {
    if (d->closing) {
        pthread_join((pthread_t)d->close_th, NULL);
        d->closing = 0;
    }
    if (g_live_dev == d)
        g_live_dev = NULL;
}

typedef struct drop_job {
    void *p[16];
    size_t len[16];
    int n;
    _Atomic int next;
} drop_job;

static void *drop_thread(void *arg) {
    drop_job *J = arg;
    const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
    for (int k; (k = atomic_fetch_add(&J->next, 1)) < J->n;) {
        const uintptr_t a = ((uintptr_t)J->p[k] + pg - 1) & ~(pg - 1);
        const uintptr_t b = ((uintptr_t)J->p[k] + J->len[k]) & ~(pg - 1);
        if (b > a)
            madvise((void *)a, b - a, MADV_DONTNEED);
    }
    return NULL;
}

static void *drop_detached(void *arg) {
    drop_thread(arg);
    free(arg);
    return NULL;
}

void gt_chains_drop_blocks_async(gt_chains *c) {
    const char *e = getenv("GAC_EARLY_FREE");
    if (e && *e == '0')
        return;
    drop_job *J = calloc(1, sizeof(drop_job));
    if (!J)
        return;
    const size_t nb = (size_t)c->nb;
    J->p[0] = c->bt, J->len[0] = nb * 4;
    J->p[1] = c->bq, J->len[1] = nb * 4;
    J->p[2] = c->bs, J->len[2] = nb * 4;
    J->n = 3;
    atomic_init(&J->next, 0);
    pthread_t th;
    pthread_attr_t at;
    pthread_attr_init(&at);
    pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
    if (pthread_create(&th, &at, drop_detached, J) != 0)
        free(J);
    pthread_attr_destroy(&at);
}

void gt_chains_drop_pages(gt_chains *c) {
    const char *e = getenv("GAC_FREE_MADV");
    if (e && *e == '0')
        return;
    drop_job J;
    memset(&J, 0, sizeof(J));
    const size_t n = (size_t)c->n, nb = (size_t)c->nb;
#define DROP(ptr, bytes) \
    if ((ptr) && J.n < 16) { J.p[J.n] = (void *)(ptr); J.len[J.n++] = (bytes); }
    DROP(c->bt, nb * 4);
    DROP(c->bq, nb * 4);
    DROP(c->bs, nb * 4);
    DROP(c->blk_off, (n + 1) * 8);
    DROP(c->score, n * 8);
    DROP(c->tstart, n * 4);
    DROP(c->tend, n * 4);
    DROP(c->qstart, n * 4);
    DROP(c->qend, n * 4);
    DROP(c->tname, n * 4);
    DROP(c->qname, n * 4);
#undef DROP
    atomic_init(&J.next, 0);
    gac_run_threads(J.n, drop_thread, &J);
}

static drop_job g_late;
static int g_late_on = -1;

void gt_free_late(void *p, size_t bytes) {
    if (!p)
        return;
    if (g_late_on < 0) {
        const char *e = getenv("GAC_LATE_FREE");
        g_late_on = !(e && *e == '0');
    }
    if (!g_late_on || g_late.n == 16) {
        free(p);
        return;
    }
    g_late.p[g_late.n] = p;
    g_late.len[g_late.n++] = bytes;
}

void gt_free_late_all(void) {
    if (!g_late.n)
        return;
    atomic_init(&g_late.next, 0);
    gac_run_threads(g_late.n, drop_thread, &g_late);
    for (int k = 0; k < g_late.n; ++k)
        free(g_late.p[k]);
    g_late.n = 0;
}

void gt_exit_ok(void) {
    join_live_device();
    if (atomic_load(&g_aborting)) /* a helper is aborting: its exit status wins */
        abort_second();
    if (g_verbose >= 2 || getenv("GAC_TIMING")) { /* the last wall-clock anchor */
        struct timespec rt;
        clock_gettime(CLOCK_REALTIME, &rt);
        fprintf(stderr, "[stage-clock] exit %.6f\n", rt.tv_sec + 1e-9 * rt.tv_nsec);
    }
    if (fflush(NULL) != 0)
        gt_abort("write error\n");
    if (getenv("GAC_PROFILE_EXIT")) exit(0); /* gprof builds: write gmon.out */
    _exit(0);
}

void gt_check(int rc) {
    if (rc != GAC_OK)
        gt_abort("%s", gac_last_error());
}

/* ------------------------------------------------------------ ranks */
/* The ranks of one run share a token (GAC_RANK_TOKEN, required with
 * -nranks > 1): every part, marker and liveness file carries it in its name
 * or content, so files a failed earlier run left behind are never read. */
static char g_token[128];

static const char *rank_token(void) { return g_token; }

void gt_part_name(char *buf, size_t cap, const char *path, int r, const char *suffix) {
    snprintf(buf, cap, "%s.gacpart%d.%s%s", path, r, g_token, suffix);
}

static const gt_ranks *g_ranks;

static void rank_failed_hook(void) { /* tell the waiting ranks this one has failed */
    char b[4096];
    gt_part_name(b, sizeof(b), g_ranks->key, g_ranks->me, ".failed");
    const int fd = open(b, O_WRONLY | O_CREAT | O_TRUNC, 0644);
    if (fd >= 0)
        close(fd);
}

/* "<boot id> <pid namespace> <pid>": a waiting rank on the same machine and
 * in the same pid namespace can tell whether a peer process still exists */
static void self_identity(char *b, size_t cap) {
    char boot[64] = "?", ns[64] = "?";
    FILE *f = fopen("/proc/sys/kernel/random/boot_id", "r");
    if (f) {
        if (fscanf(f, "%63s", boot) != 1)
            strcpy(boot, "?");
        fclose(f);
    }
    const ssize_t k = readlink("/proc/self/ns/pid", ns, sizeof(ns) - 1);
    ns[k > 0 ? k : 1] = 0;
    for (char *p = ns; *p; ++p)
        if (*p == ' ')
            *p = '_';
    snprintf(b, cap, "%s %s %ld", boot, ns, (long)getpid());
}

static char g_ident[192];

void gt_ranks_init(gt_ranks *rk, int n, int me, const char *key) {
    rk->n = n;
    rk->me = me;
    rk->key = key;
    if (n < 1 || me < 0 || me >= n)
        gt_abort("-rank=%d is not in 0..%d (-nranks=%d)", me, n - 1, n);
    if (n == 1)
        return;
    const char *t = getenv("GAC_RANK_TOKEN");
    if (!t || !*t)
        gt_abort("-nranks=%d: set GAC_RANK_TOKEN to one per-run value, the same on every rank "
                 "(it tells this run's part files from an earlier run's)", n);
    size_t j = 0;
    for (; t[j] && j + 1 < sizeof(g_token); ++j)
        g_token[j] = (isalnum((unsigned char)t[j]) || t[j] == '-' || t[j] == '_' || t[j] == '.')
                         ? t[j] : '_';
    g_token[j] = 0;
    g_ranks = rk;
    gt_on_abort(rank_failed_hook); /* every rank: the others may wait on any of them */
    /* liveness: "<key>.gacpart<r>.<token>.alive" = this process's identity */
    self_identity(g_ident, sizeof(g_ident));
    char b[4096], tmp[4200];
    gt_part_name(b, sizeof(b), key, me, ".alive");
    snprintf(tmp, sizeof(tmp), "%s.tmp", b);
    FILE *f = fopen(tmp, "w");
    if (!f || fprintf(f, "%s\n", g_ident) < 0 || fclose(f) != 0 || rename(tmp, b) != 0)
        gt_abort("can't write %s: %s", b, strerror(errno));
}

void gt_ranks_clear(const gt_ranks *rk, const char *path) {
    char b[4096];
    gt_part_name(b, sizeof(b), path, rk->me, "");
    unlink(b);
    gt_part_name(b, sizeof(b), path, rk->me, ".tmp");
    unlink(b);
}

/* Waiting for rank r: abort if it has failed (its .failed file), if its
 * process is gone (same machine: its .alive identity names a pid that no
 * longer exists), if it has not started within GAC_RANK_START_TIMEOUT
 * seconds (default 300), or after GAC_RANK_TIMEOUT seconds in all (default
 * 3600, for a live but stuck rank). */
typedef struct rank_wait {
    int r;
    double t0, next_check;
    int seen_alive;
} rank_wait;

static void rank_wait_init(rank_wait *w, int r) {
    w->r = r;
    w->t0 = now_s();
    w->next_check = 0;
    w->seen_alive = 0;
}

static void rank_wait_check(rank_wait *w, const gt_ranks *rk, const char *what) {
    const double now = now_s();
    if (now < w->next_check)
        return;
    w->next_check = now + 0.05;
    char b[4096];
    gt_part_name(b, sizeof(b), rk->key, w->r, ".failed");
    if (access(b, F_OK) == 0)
        gt_abort("%s: rank %d failed", what, w->r);
    if (!w->seen_alive) {
        gt_part_name(b, sizeof(b), rk->key, w->r, ".alive");
        w->seen_alive = access(b, F_OK) == 0;
    }
    const char *st = getenv("GAC_RANK_START_TIMEOUT"), *lim = getenv("GAC_RANK_TIMEOUT");
    const double start_limit = st ? atof(st) : 300.0, limit = lim ? atof(lim) : 3600.0;
    if (!w->seen_alive && now - w->t0 > start_limit)
        gt_abort("%s: rank %d did not start within %.0f s", what, w->r, start_limit);
    if (now - w->t0 > limit)
        gt_abort("%s: timed out waiting for rank %d", what, w->r);
}

/* 1 if rank r's process is known to be gone (same machine) */
static int rank_dead(const gt_ranks *rk, int r) {
    char b[4096];
    gt_part_name(b, sizeof(b), rk->key, r, ".alive");
    FILE *f = fopen(b, "r");
    if (!f)
        return 0;
    char boot[64], ns[64], mine_boot[64], mine_ns[64];
    long pid = 0, mine = 0;
    const int ok = fscanf(f, "%63s %63s %ld", boot, ns, &pid) == 3;
    fclose(f);
    if (!(ok && sscanf(g_ident, "%63s %63s %ld", mine_boot, mine_ns, &mine) == 3 &&
          strcmp(boot, "?") != 0 && strcmp(boot, mine_boot) == 0 && strcmp(ns, mine_ns) == 0 &&
          pid > 0))
        return 0; /* another machine or pid namespace: only the timeouts apply */
    if (kill((pid_t)pid, 0) != 0)
        return errno == ESRCH;
    /* a killed process stays a zombie until its parent reaps it */
    char sp[64], st[512];
    snprintf(sp, sizeof(sp), "/proc/%ld/stat", pid);
    f = fopen(sp, "r");
    if (!f)
        return 0;
    const size_t k = fread(st, 1, sizeof(st) - 1, f);
    fclose(f);
    st[k] = 0;
    const char *q = strrchr(st, ')');
    return q && (q[2] == 'Z' || q[2] == 'X');
}

void gt_ranks_wait(const gt_ranks *rk, const char *path) {
    struct timespec nap = {0, 500000};
    char b[4096];
    for (int r = 1; r < rk->n; ++r) {
        gt_part_name(b, sizeof(b), path, r, "");
        rank_wait w;
        rank_wait_init(&w, r);
        while (access(b, F_OK) != 0) {
            rank_wait_check(&w, rk, path);
            if (rank_dead(rk, r) && access(b, F_OK) != 0)
                gt_abort("%s: rank %d died without its part", path, r);
            nanosleep(&nap, NULL);
        }
    }
}

/* ---- positioned parts (chainNet -nranks): every rank writes its part of
 * an output straight into the final file.  Markers next to the output:
 * "<path>.gacsize<r>" = "<token> <bytes>", published once rank r's part is
 * formatted (rank 0 publishes only after truncating the file at startup),
 * and "<path>.gacdone<r>" once written.  Rank r writes at the sum of the
 * sizes of ranks < r; rank 0 waits for every done marker and removes the
 * markers.  The token inside tells this run's markers from an earlier
 * run's. */
static void marker_name(char *b, size_t cap, const char *path, const char *what, int r) {
    snprintf(b, cap, "%s.gac%s%d", path, what, r);
}

static void put_marker(const char *path, const char *what, int r, long long v) {
    char b[4096], t[4200];
    marker_name(b, sizeof(b), path, what, r);
    snprintf(t, sizeof(t), "%s.tmp", b);
    FILE *f = fopen(t, "w");
    if (!f || fprintf(f, "%s %lld\n", rank_token(), v) < 0 || fclose(f) != 0 || rename(t, b) != 0)
        gt_abort("can't write %s: %s", b, strerror(errno));
}

static int read_marker(const char *b, long long *v) {
    char tok[256];
    FILE *f = fopen(b, "r");
    if (!f)
        return 0;
    const int ok = fscanf(f, "%255s %lld", tok, v) == 2 && strcmp(tok, rank_token()) == 0;
    fclose(f);
    return ok;
}

/* the value of rank r's marker of this run, waiting for it */
static long long get_marker(const gt_ranks *rk, const char *path, const char *what, int r) {
    struct timespec nap = {0, 200000};
    char b[4096];
    marker_name(b, sizeof(b), path, what, r);
    rank_wait w;
    rank_wait_init(&w, r);
    for (;;) {
        long long v;
        if (read_marker(b, &v))
            return v;
        rank_wait_check(&w, rk, path);
        if (rank_dead(rk, r) && !read_marker(b, &v))
            gt_abort("%s: rank %d died before its %s marker", path, r, what);
        nanosleep(&nap, NULL);
    }
}

void gt_ranks_clear_markers(const gt_ranks *rk, const char *path) {
    char b[4096];
    marker_name(b, sizeof(b), path, "size", rk->me);
    unlink(b);
    marker_name(b, sizeof(b), path, "done", rk->me);
    unlink(b);
}

/* GAC_RANK_SOLO=1 (measurement only: DESIGN §6's per-rank table): a rank
 * runs by itself, as on a node where every rank has its own GPU and cores --
 * its part goes to "<path>.solo<r>" and no rank waits for another */
int gt_ranks_solo(void) {
    static int v = -1;
    if (v < 0) {
        const char *e = getenv("GAC_RANK_SOLO");
        v = e && *e == '1';
    }
    return v;
}

void gt_ranks_place(const gt_ranks *rk, const char *path, const char *buf, size_t len) {
    char *b = (char *)buf;
    gt_ranks_place_bufs(rk, path, &b, &len, 1);
}

void gt_ranks_place_bufs(const gt_ranks *rk, const char *path, char *const *bufs,
                         const size_t *lens, int64_t nb) {
    size_t len = 0;
    for (int64_t k = 0; k < nb; ++k)
        len += lens[k];
    char solo[4096];
    const int alone = gt_ranks_solo();
    off_t off = 0;
    if (alone) {
        snprintf(solo, sizeof(solo), "%s.solo%d", path, rk->me);
        path = solo;
    } else {
        put_marker(path, "size", rk->me, (long long)len);
        for (int r = 0; r < rk->me; ++r)
            off += (off_t)get_marker(rk, path, "size", r);
    }
    const int fd = open(path, O_WRONLY | O_CREAT | (alone ? O_TRUNC : 0), 0666);
    if (fd < 0)
        gt_abort("Can't open %s to write: %s", path, strerror(errno));
    for (int64_t k = 0; k < nb; ++k) { /* (pwritev of up to 256 buffers at a time) */
        struct iovec iov[256];
        int m = 0;
        size_t bytes = 0;
        for (; k < nb && m < 256; ++k)
            if (lens[k]) {
                iov[m].iov_base = bufs[k];
                iov[m++].iov_len = lens[k];
                bytes += lens[k];
            }
        --k;
        size_t done = 0;
        while (done < bytes) {
            const ssize_t w = pwritev(fd, iov, m, off);
            if (w <= 0)
                gt_abort("write error on %s: %s", path, strerror(errno));
            done += (size_t)w;
            off += (off_t)w;
            size_t skip = (size_t)w; /* (a short write: drop what went out) */
            int i = 0;
            while (i < m && skip >= iov[i].iov_len)
                skip -= iov[i++].iov_len;
            memmove(iov, iov + i, (size_t)(m - i) * sizeof(struct iovec));
            m -= i;
            if (m) {
                iov[0].iov_base = (char *)iov[0].iov_base + skip;
                iov[0].iov_len -= skip;
            }
        }
    }
    if (close(fd) != 0)
        gt_abort("close failed on %s", path);
    if (!alone)
        put_marker(path, "done", rk->me, 1);
}

void gt_ranks_finish(const gt_ranks *rk, const char *path) {
    if (gt_ranks_solo())
        return;
    off_t total = 0;
    for (int r = 0; r < rk->n; ++r) {
        total += (off_t)get_marker(rk, path, "size", r);
        get_marker(rk, path, "done", r);
    }
    if (truncate(path, total) != 0)
        gt_abort("can't size %s: %s", path, strerror(errno));
    char b[4096];
    for (int r = 0; r < rk->n; ++r) {
        marker_name(b, sizeof(b), path, "size", r);
        unlink(b);
        marker_name(b, sizeof(b), path, "done", r);
        unlink(b);
    }
}

/* the last step of a successful multi-rank run: this rank's liveness file
 * goes (rank 0, once every part is in, also removes the others') */
void gt_ranks_done(const gt_ranks *rk) {
    if (rk->n <= 1)
        return;
    char b[4096];
    for (int r = 0; r < rk->n; ++r)
        if (r == rk->me || rk->me == 0) {
            gt_part_name(b, sizeof(b), rk->key, r, ".alive");
            unlink(b);
        }
    gt_on_abort(NULL);
}

void gt_ranks_append_parts(const gt_ranks *rk, const char *path, FILE *f) {
    char b[4096];
    char *buf = malloc(1 << 22);
    for (int r = 1; r < rk->n; ++r) {
        gt_part_name(b, sizeof(b), path, r, "");
        FILE *p = fopen(b, "r");
        if (!p)
            gt_abort("Can't open %s to read: %s", b, strerror(errno));
        size_t k;
        while ((k = fread(buf, 1, 1 << 22, p)) > 0)
            if (fwrite(buf, 1, k, f) != k)
                gt_abort("write error on %s", path);
        fclose(p);
        unlink(b);
    }
    free(buf);
}

/* ------------------------------------------------------------ options */
typedef struct gt_optval {
    char *name, *val;
} gt_optval;
static gt_optval *g_opts;
static int g_nopts, g_capopts;

static const gt_spec *spec_find(const gt_spec *spec, const char *name) {
    for (; spec && spec->name; ++spec)
        if (strcmp(spec->name, name) == 0)
            return spec;
    return NULL;
}

static int g_any_option = 0; /* optionHash: every option accepted */

static void validate(const gt_spec *spec, const char *name, const char *val) {
    static const gt_spec common[] = {{"verbose", GT_INT}, {NULL, 0}};
    if (g_any_option)
        return;
    const gt_spec *s = spec_find(spec, name);
    if (!s)
        s = spec_find(common, name);
    if (!s)
        gt_abort("-%s is not a valid option", name);
    char *end;
    switch (s->type) {
    case GT_BOOL:
        if (val)
            gt_abort("boolean option -%s must not have value", name);
        break;
    case GT_STRING:
        if (!val)
            gt_abort("string option -%s must have a value", name);
        break;
    case GT_INT:
        if (!val)
            gt_abort("int option -%s must have a value", name);
        (void)strtol(val, &end, 10);
        if (*val == 0 || *end != 0)
            gt_abort("value of -%s is not a valid integer: \"%s\"", name, val);
        break;
    case GT_DOUBLE:
        if (!val)
            gt_abort("double option -%s must have a value", name);
        (void)strtod(val, &end);
        if (*val == 0 || *end != 0)
            gt_abort("value of -%s is not a valid double: \"%s\"", name, val);
        break;
    }
}

/* parseAnOption (kent/src/lib/options.c:121-190) */
static int parse_one(const gt_spec *spec, char *arg) {
    char *eq = strchr(arg, '=');
    if (!(eq || arg[0] == '-'))
        return 0;
    if (arg[0] == '-' && (arg[1] == 0 || isspace((unsigned char)arg[1])))
        return 0;
    if (eq) {
        for (char *s = arg; s < eq; ++s)
            if (*s != '_' && *s != '-' && !isalnum((unsigned char)*s))
                return 0;
    }
    char *name = arg[0] == '-' ? arg + 1 : arg;
    char *val = NULL;
    if (eq) {
        *eq = 0;
        val = eq + 1;
    }
    validate(spec, name, val);
    if (g_nopts == g_capopts) {
        g_capopts = g_capopts ? g_capopts * 2 : 16;
        g_opts = realloc(g_opts, g_capopts * sizeof(gt_optval));
    }
    g_opts[g_nopts].name = strdup(name);
    g_opts[g_nopts].val = strdup(val ? val : "on");
    ++g_nopts;
    if (eq)
        *eq = '=';
    return 1;
}

void gt_options(int *argc, char **argv, const gt_spec *spec) {
    int orig = *argc, n = 1, i;
    char **rd = argv + 1, **wr = argv + 1;
    for (i = 1; i < orig; ++i) {
        if (strcmp(*rd, "--") == 0) {
            rd++;
            i++;
            break;
        }
        if (!parse_one(spec, *rd)) {
            *wr++ = *rd;
            n++;
        }
        rd++;
    }
    for (; i < orig; ++i) {
        *wr++ = *rd++;
        n++;
    }
    *argc = n;
    *wr = NULL;
    g_verbose = gt_opt_int("verbose", 1);
}

void gt_options_reset(void) {
    for (int i = 0; i < g_nopts; ++i) {
        free(g_opts[i].name);
        free(g_opts[i].val);
    }
    g_nopts = 0;
}

void gt_options_hash(int *argc, char **argv) {
    g_any_option = 1;
    gt_options(argc, argv, NULL);
}

const char *gt_opt_str(const char *name, const char *def) {
    for (int i = g_nopts - 1; i >= 0; --i) /* last occurrence wins */
        if (strcmp(g_opts[i].name, name) == 0)
            return g_opts[i].val;
    return def;
}

int gt_opt_exists(const char *name) { return gt_opt_str(name, NULL) != NULL; }

/* optionInt (kent/src/lib/options.c:359-378) */
int gt_opt_int(const char *name, int def) {
    const char *s = gt_opt_str(name, NULL);
    if (!s || strcmp(s, "on") == 0)
        return def;
    char *end;
    long v = strtol(s, &end, 10);
    if (*s == 0 || *end != 0)
        gt_abort("value of -%s is not a valid integer: \"%s\"", name, s);
    return (int)v;
}

/* optionDouble (kent/src/lib/options.c:426-439) */
double gt_opt_double(const char *name, double def) {
    const char *s = gt_opt_str(name, NULL);
    if (!s)
        return def;
    char *end;
    double v = strtod(s, &end);
    if (*s == 0 || *end != 0)
        gt_abort("value of -%s is not a valid double: \"%s\"", name, s);
    return v;
}

/* ------------------------------------------------------------ kent hash order */
static uint32_t kent_hash_string(const char *s) {
    uint32_t r = 0;
    int c;
    while ((c = *s++) != 0)
        r += (r << 3) + (uint32_t)c;
    return r;
}

void gt_khash_init(gt_khash *h, int pow) {
    memset(h, 0, sizeof(*h));
    h->pow = pow ? pow : 12;
    h->mask = (1u << h->pow) - 1;
    h->head = malloc(((size_t)1 << h->pow) * sizeof(int32_t));
    memset(h->head, 0xff, ((size_t)1 << h->pow) * sizeof(int32_t));
}

int32_t gt_khash_find(const gt_khash *h, int32_t key) {
    char buf[16];
    snprintf(buf, sizeof(buf), "%d", key);
    for (int32_t e = h->head[kent_hash_string(buf) & h->mask]; e >= 0; e = h->next[e])
        if (h->key[e] == key)
            return e;
    return -1;
}

static void khash_resize(gt_khash *h, int pow) {
    if (pow > 30)
        pow = 30;
    if (pow == h->pow)
        return;
    const uint32_t old_size = 1u << h->pow;
    int32_t *old = h->head;
    h->pow = pow;
    h->mask = (1u << pow) - 1;
    h->head = malloc(((size_t)1 << pow) * sizeof(int32_t));
    memset(h->head, 0xff, ((size_t)1 << pow) * sizeof(int32_t));
    for (uint32_t i = 0; i < old_size; ++i) {
        int32_t e = old[i];
        while (e >= 0) {
            const int32_t nx = h->next[e];
            const uint32_t b = h->hv[e] & h->mask;
            h->next[e] = h->head[b];
            h->head[b] = e;
            e = nx;
        }
    }
    /* hashReverseAllBucketLists */
    for (uint32_t b = 0; b <= h->mask; ++b) {
        int32_t prev = -1, e = h->head[b];
        while (e >= 0) {
            const int32_t nx = h->next[e];
            h->next[e] = prev;
            prev = e;
            e = nx;
        }
        h->head[b] = prev;
    }
    free(old);
}

int32_t gt_khash_add(gt_khash *h, int32_t key) {
    if (h->n == h->cap) {
        h->cap = h->cap ? h->cap * 2 : 1024;
        h->next = realloc(h->next, (size_t)h->cap * sizeof(int32_t));
        h->hv = realloc(h->hv, (size_t)h->cap * sizeof(uint32_t));
        h->key = realloc(h->key, (size_t)h->cap * sizeof(int32_t));
    }
    char buf[16];
    snprintf(buf, sizeof(buf), "%d", key);
    const int32_t e = h->n++;
    h->key[e] = key;
    h->hv[e] = kent_hash_string(buf);
    const uint32_t b = h->hv[e] & h->mask;
    h->next[e] = h->head[b];
    h->head[b] = e;
    /* autoExpand: elCount > size * 1.0 -> digitsBaseTwo(size) = pow + 1 */
    if ((int64_t)h->n > ((int64_t)1 << h->pow))
        khash_resize(h, h->pow + 1);
    return e;
}

int32_t gt_khash_order(const gt_khash *h, int32_t *out) {
    int32_t k = 0;
    for (uint32_t b = 0; b <= h->mask; ++b)
        for (int32_t e = h->head[b]; e >= 0; e = h->next[e])
            out[k++] = e;
    return k;
}

void gt_khash_free(gt_khash *h) {
    free(h->head);
    free(h->next);
    free(h->hv);
    free(h->key);
    memset(h, 0, sizeof(*h));
}

/* ------------------------------------------------------------ names */
static uint32_t hash_str(const char *s, size_t n) {
    uint32_t h = 2166136261u;
    for (size_t i = 0; i < n; ++i)
        h = (h ^ (uint8_t)s[i]) * 16777619u;
    return h;
}

static void names_rehash(gt_names *t, int32_t nslot) {
    free(t->slots);
    t->nslot = nslot;
    t->slots = malloc(nslot * sizeof(int32_t));
    memset(t->slots, 0xff, nslot * sizeof(int32_t));
    for (int32_t i = 0; i < t->n; ++i) {
        uint32_t h = hash_str(t->names[i], strlen(t->names[i])) & (nslot - 1);
        while (t->slots[h] >= 0)
            h = (h + 1) & (nslot - 1);
        t->slots[h] = i;
    }
}

int32_t gt_names_find(const gt_names *t, const char *s) {
    if (!t->nslot)
        return -1;
    size_t n = strlen(s);
    uint32_t h = hash_str(s, n) & (t->nslot - 1);
    while (t->slots[h] >= 0) {
        if (strcmp(t->names[t->slots[h]], s) == 0)
            return t->slots[h];
        h = (h + 1) & (t->nslot - 1);
    }
    return -1;
}

int32_t gt_names_add(gt_names *t, const char *s, size_t len) {
    if (t->nslot) {
        uint32_t h = hash_str(s, len) & (t->nslot - 1);
        while (t->slots[h] >= 0) {
            const char *x = t->names[t->slots[h]];
            if (strncmp(x, s, len) == 0 && x[len] == 0)
                return t->slots[h];
            h = (h + 1) & (t->nslot - 1);
        }
    }
    if (t->n == t->cap) {
        t->cap = t->cap ? t->cap * 2 : 64;
        t->names = realloc(t->names, t->cap * sizeof(char *));
    }
    t->names[t->n] = strndup(s, len);
    int32_t id = t->n++;
    if (t->n * 2 > t->nslot)
        names_rehash(t, t->nslot ? t->nslot * 2 : 256);
    else {
        uint32_t h = hash_str(s, len) & (t->nslot - 1);
        while (t->slots[h] >= 0)
            h = (h + 1) & (t->nslot - 1);
        t->slots[h] = id;
    }
    return id;
}

void gt_names_free(gt_names *t) {
    for (int32_t i = 0; i < t->n; ++i)
        free(t->names[i]);
    free(t->names);
    free(t->slots);
    memset(t, 0, sizeof(*t));
}

/* ------------------------------------------------------------ files */
FILE *gt_must_open(const char *path, const char *mode) {
    if (strcmp(path, "stdout") == 0)
        return stdout;
    if (strcmp(path, "stdin") == 0)
        return stdin;
    FILE *f = fopen(path, mode);
    if (!f)
        gt_abort("Can't open %s to %s: %s", path, mode[0] == 'w' ? "write" : "read",
                 strerror(errno));
    return f;
}

void gt_careful_close(FILE *f, const char *path) {
    if (f == stdout || f == stdin) {
        if (fflush(f) != 0)
            gt_abort("write error on %s", path);
        return;
    }
    if (fclose(f) != 0)
        gt_abort("close failed on %s", path);
}

int gt_file_exists(const char *path) {
    struct stat st;
    return strcmp(path, "stdin") == 0 || stat(path, &st) == 0;
}

/* parallel pread of [a, b) of a regular file */
typedef struct pr_job {
    int fd;
    char *buf;
    size_t size, per;
    _Atomic size_t next;
    _Atomic int bad;
} pr_job;

static void *pr_thread(void *p) {
    pr_job *J = p;
    for (;;) {
        const size_t a = atomic_fetch_add(&J->next, J->per);
        if (a >= J->size)
            break;
        const size_t b = a + J->per < J->size ? a + J->per : J->size;
        for (size_t o = a; o < b;) {
            const ssize_t r = pread(J->fd, J->buf + o, b - o, (off_t)o);
            if (r <= 0) {
                atomic_store(&J->bad, 1);
                break;
            }
            o += (size_t)r;
        }
    }
    return NULL;
}

/* whole file into a NUL-terminated heap buffer (.gz decompressed); regular
 * files of more than 32 MB are read by several threads at once */
char *gt_slurp(const char *path, size_t *len) {
    size_t n = strlen(path);
    int gz = n > 3 && strcmp(path + n - 3, ".gz") == 0;
    size_t cap = 1 << 20, l = 0;
    char *buf = NULL;
    if (gz) {
        gzFile g = gzopen(path, "rb");
        if (!g)
            gt_abort("Couldn't open %s , %s", path, strerror(errno));
        gzbuffer(g, 1 << 20);
        buf = malloc(cap + 1);
        for (;;) {
            if (l == cap) {
                cap *= 2;
                buf = realloc(buf, cap + 1);
            }
            int r = gzread(g, buf + l, (unsigned)((cap - l) > (1u << 30) ? (1u << 30) : (cap - l)));
            if (r < 0)
                gt_abort("gzip read error on %s", path);
            if (r == 0)
                break;
            l += (size_t)r;
        }
        gzclose(g);
    } else {
        int fd = strcmp(path, "stdin") == 0 ? 0 : open(path, O_RDONLY);
        if (fd < 0)
            gt_abort("Couldn't open %s , %s", path, strerror(errno));
        struct stat st;
        if (fd != 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
            cap = (size_t)st.st_size + 1;
            if (st.st_size > (32 << 20)) {
                const size_t size = (size_t)st.st_size;
                buf = malloc(size + 17);
                memset(buf + size, 0, 17); /* (over-reads of the parsers) */
                pr_job J = {fd, buf, size, 8u << 20, 0, 0};
                atomic_init(&J.next, 0);
                atomic_init(&J.bad, 0);
                int nt = gt_threads();
                if ((size_t)nt > size / J.per + 1)
                    nt = (int)(size / J.per + 1);
                gac_run_threads(nt, pr_thread, &J);
                if (atomic_load(&J.bad))
                    gt_abort("read error on %s", path);
                close(fd);
                buf[size] = 0;
                *len = size;
                return buf;
            }
        }
        buf = malloc(cap + 1);
        for (;;) {
            if (l == cap) {
                cap *= 2;
                buf = realloc(buf, cap + 1);
            }
            ssize_t r = read(fd, buf + l, cap - l);
            if (r < 0)
                gt_abort("read error on %s", path);
            if (r == 0)
                break;
            l += (size_t)r;
        }
        if (fd != 0)
            close(fd);
    }
    buf = realloc(buf, l + 17);
    memset(buf + l, 0, 17); /* (over-reads of the parsers) */
    *len = l;
    return buf;
}

/* ------------------------------------------------------------ chains
 * gt_read_chains parses in parallel: the text is cut into chunks at lines
 * that start with "chain" (only a header can), every chunk is parsed by its
 * own thread with the sequential rules (chainReadChainLine /
 * chainReadBlocks, chain.c:229-335), and the chunks are stitched in order.
 * Everything order-dependent is replayed after the fact: the first error
 * in file order (line numbers from per-chunk newline counts), the first
 * chain scoring below stop_below (the read stops there, as chainNet's loop
 * does, chainNet.c:949-952), chainIdNext ids of id-less headers, and the
 * '#' metadata lines. */
typedef struct lf {
    char *cur, *end;
    const char *path;
    int64_t line;

    gt_chains *meta_to;
    /* first error of the chunk: message, byte position */
    int err;
    char msg[512];
} lf;

static char *lf_next(lf *f) {
    if (f->cur >= f->end)
        return NULL;
    char *line = f->cur;
    char *nl = memchr(line, '\n', f->end - line);
    if (nl) {
        *nl = 0;
        f->cur = nl + 1;
    } else {
        f->cur = f->end;
    }
    ++f->line;
    return line;
}

static void add_meta_at(gt_chains *c, const char *line, int64_t at) {
    if (c->n_meta == c->meta_cap) {
        c->meta_cap = c->meta_cap ? c->meta_cap * 2 : 16;
        c->meta = realloc(c->meta, c->meta_cap * sizeof(char *));
        c->meta_at = realloc(c->meta_at, c->meta_cap * sizeof(int64_t));
    }
    c->meta_at[c->n_meta] = at;
    c->meta[c->n_meta++] = strdup(line);
}

/* a '#' line consumed while reading chain c->n (the next one) */
static void add_meta(gt_chains *c, const char *line) { add_meta_at(c, line, c->n); }

/* lineFileChopNext: next non-blank, non-'#' line chopped into <= max words */
static int lf_chop(lf *f, char **row, int max) {
    char *line;
    while ((line = lf_next(f)) != NULL) {
        if (line[0] == '#') {
            if (f->meta_to)
                add_meta(f->meta_to, line);
            continue;
        }
        int n = gac_chop_white(line, row, max);
        if (n)
            return n;
    }
    return 0;
}

/* messages keep "\001" for the line number and "\002" for the path; both
 * are filled in once the chunk's first line is known */
#define LF_FAIL(f, ...)                                                        \
    do {                                                                       \
        snprintf((f)->msg, sizeof((f)->msg), __VA_ARGS__);                     \
        (f)->err = 1;                                                          \
        return -1;                                                             \
    } while (0)

/* lineFileNeedNum; the message takes the chunk-local line, fixed up later */
static int need_num(lf *f, char **row, int ix, int *out) {
    char c = row[ix][0];
    if (c != '-' && !isdigit((unsigned char)c))
        LF_FAIL(f, "Expecting number field %d line \001 of \002, got %s", ix + 1, row[ix]);
    *out = atoi(row[ix]);
    return 0;
}

static void chains_grow(gt_chains *c, int64_t cap) {
    {
        c->score = realloc(c->score, cap * sizeof(double));
        c->tname = realloc(c->tname, cap * 4);
        c->tsize = realloc(c->tsize, cap * 4);
        c->tstart = realloc(c->tstart, cap * 4);
        c->tend = realloc(c->tend, cap * 4);
        c->qname = realloc(c->qname, cap * 4);
        c->qsize = realloc(c->qsize, cap * 4);
        c->qstart = realloc(c->qstart, cap * 4);
        c->qend = realloc(c->qend, cap * 4);
        c->qstrand = realloc(c->qstrand, cap);
        c->id = realloc(c->id, cap * 4);
        c->blk_off = realloc(c->blk_off, (cap + 1) * 8);
        c->cap = cap;
    }
}

static void chains_reserve(gt_chains *c) {
    if (c->n + 1 >= c->cap)
        chains_grow(c, c->cap ? c->cap * 2 : 4096);
}

/* room for `need` chains (and need + 1 block offsets) */
static void chains_reserve_n(gt_chains *c, int64_t need) {
    if (c->cap < need)
        chains_grow(c, need > 2 * c->cap ? need : 2 * c->cap);
}

static int g_next_id = 1; /* chainIdNext (chain.c:180-198) */
static int g_defer_ids;   /* gt_defer_chain_ids: id-less headers keep INT32_MIN */

typedef struct chunk {
    lf f;
    gt_chains c;       /* local: names local, id -1 = assign later */
    int64_t stop;      /* first chain (local index) scoring below stop_below, or -1 */
    int64_t lines;     /* newlines in the chunk */
    double t0, t1;     /* (GAC_TIMING) when its parse started and ended */
    int64_t err_line;  /* local line of the error */
    double stop_below;
    const gt_names *tkeep, *qkeep; /* gt_read_chains_keep: NULL = keep all */
} chunk;

/* gt_read_chains_keep: the blocks of a chain on neither kept side are
 * skipped to the next "chain" header line of the chunk when only block lines
 * lie between (no '#' line, which is metadata, and a header follows); 1 =
 * skipped, 0 = parse them normally */
/* newlines in [p, p + n), eight bytes at a time */
static int64_t count_nl(const char *p, size_t n) {
    int64_t k = 0;
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        const uint64_t x = w ^ 0x0a0a0a0a0a0a0a0aull; /* zero byte = newline */
        k += __builtin_popcountll((x - 0x0101010101010101ull) & ~x & 0x8080808080808080ull);
    }
    for (; i < n; ++i)
        k += p[i] == '\n';
    return k;
}

static int skip_blocks(lf *f) {
    /* block lines hold only digits, tabs and newlines: the next 'c' is the
     * next header (checked), and a '#' before it is a metadata line (then
     * the lines are parsed normally); both found by memchr */
    const char *s = f->cur, *end = f->end;
    if (s >= end || *s == '#')
        return 0;
    const char *c = memchr(s, 'c', (size_t)(end - s));
    if (!c || c == s || c[-1] != '\n' || end - c < 6 || memcmp(c, "chain", 5) != 0 ||
        (c[5] != ' ' && c[5] != '\t') || memchr(s, '#', (size_t)(c - s)))
        return 0;
    f->line += count_nl(s, (size_t)(c - s));
    f->cur = (char *)c;
    return 1;
}

/* Fast path for the common block line "size[\tdt\tdq]\n" (decimal fields of
 * at most 9 digits, one tab apart): 1 = parsed into v[0..*bw), 0 = anything
 * else (blank or '#' lines, spaces, CR, long numbers, a missing newline,
 * errors), which the general lineFileChopNext + lineFileNeedNum path then
 * reads from the same position. */
static int fast_block_line_scalar(lf *f, int *v, int *bw) {
    const char *p = f->cur, *end = f->end;
    int k = 0;
    for (;;) {
        const int neg = p < end && *p == '-';
        p += neg;
        const char *d0 = p;
        int x = 0;
        while (p < end && (unsigned)(*p - '0') < 10u && p - d0 < 9) {
            x = x * 10 + (*p - '0');
            ++p;
        }
        if (p == d0 || p >= end || (unsigned)(*p - '0') < 10u)
            return 0;
        v[k++] = neg ? -x : x;
        if (*p == '\n')
            break;
        if (*p != '\t' || k == 3)
            return 0;
        ++p;
    }
    if (k == 2)
        return 0;
    f->cur = (char *)p + 1;
    ++f->line;
    *bw = k;
    return 1;
}

/* One decimal field of 1-7 digits starting at p, eight bytes at a time
 * (gt_slurp pads the text, so the load may run past the chunk): the digit
 * count from the first byte that is not '0'..'9', then the digits as one
 * 8-digit number with leading zeros (three multiply-add steps).  0 = not
 * such a field (8+ digits, a sign, the chunk's end): the scalar path. */
static inline int swar_field(const char *p, const char *end, int *val) {
    uint64_t w;
    memcpy(&w, p, 8);
    const uint64_t x = w - 0x3030303030303030ull;
    const uint64_t nd = ((x + 0x7676767676767676ull) | x) & 0x8080808080808080ull;
    if (!nd)
        return 0;
    const int n = __builtin_ctzll(nd) >> 3;
    if (n == 0 || n == 8 || p + n >= end)
        return 0;
    uint64_t d = (x & ((1ull << (8 * n)) - 1)) << (8 * (8 - n));
    d = (d * 10 + (d >> 8)) & 0x00FF00FF00FF00FFull;
    d = (d * 100 + (d >> 16)) & 0x0000FFFF0000FFFFull;
    d = (d * 10000 + (d >> 32)) & 0xFFFFFFFFull;
    *val = (int)d;
    return n;
}

static int fast_block_line(lf *f, int *v, int *bw) {
    const char *p = f->cur, *end = f->end;
    int k = 0;
    for (;;) {
        const int n = swar_field(p, end, &v[k]);
        if (!n)
            return fast_block_line_scalar(f, v, bw);
        p += n;
        ++k;
        if (*p == '\n')
            break;
        if (*p != '\t' || k == 3)
            return fast_block_line_scalar(f, v, bw);
        ++p;
    }
    if (k == 2)
        return 0;
    f->cur = (char *)p + 1;
    ++f->line;
    *bw = k;
    return 1;
}

/* A header line in the form chainWrite prints ("chain" and 11 or 12
 * fields, one space apart, integer score of at most 15 digits, unsigned
 * numbers of at most 9 digits, newline right after the last field) into
 * chain c->n: 1 = parsed and the line consumed; 0 = anything else (the
 * general lf_chop + need_num path reads it, with its messages). */
static inline const char *fh_tok(const char *p, const char *end, const char **t, int *len) {
    const char *q = p;
    while (q < end && (unsigned char)*q > ' ')
        ++q;
    *t = p;
    *len = (int)(q - p);
    return q;
}

static inline const char *fh_num(const char *p, const char *end, int maxd, int64_t *v) {
    int64_t x = 0;
    const char *q = p;
    while (q < end && (unsigned)(*q - '0') < 10u && q - p < maxd) {
        x = x * 10 + (*q - '0');
        ++q;
    }
    if (q == p || q >= end || (unsigned)(*q - '0') < 10u)
        return NULL;
    *v = x;
    return q;
}

static int fast_header(lf *f, gt_chains *c) {
    const char *p = f->cur, *end = f->end;
    /* the empty line chainWrite puts after every chain's blocks (lf_chop
     * skips blank lines the same way, counting them) */
    int64_t blank = 0;
    while (p < end && *p == '\n') {
        ++p;
        ++blank;
    }
    if (end - p < 32 || memcmp(p, "chain ", 6) != 0)
        return 0;
    p += 6;
    int64_t num[13];
    const char *tn = NULL, *qn = NULL;
    int tl = 0, ql = 0, qminus = 0, nf = 1;
    for (; nf < 13; ++nf) {
        if (nf == 2 || nf == 4 || nf == 7 || nf == 9) { /* names and strands */
            const char *t;
            int len;
            p = fh_tok(p, end, &t, &len);
            if (len == 0)
                return 0;
            if (nf == 2)
                tn = t, tl = len;
            else if (nf == 7)
                qn = t, ql = len;
            else if (nf == 9)
                qminus = t[0] == '-';
        } else {
            p = fh_num(p, end, nf == 1 ? 15 : 9, &num[nf]);
            if (!p)
                return 0;
        }
        if (p >= end)
            return 0;
        if (*p == '\n' && nf >= 11)
            break;
        if (*p != ' ')
            return 0;
        ++p;
    }
    if (nf == 13 || *p != '\n')
        return 0;
    const int64_t i = c->n;
    c->score[i] = (double)num[1];
    c->tname[i] = gt_names_add(&c->tnames, tn, (size_t)tl);
    c->tsize[i] = (int)num[3];
    c->id[i] = nf == 12 ? (int)num[12] : INT32_MIN; /* (chainIdNext later) */
    c->tstart[i] = (int)num[5];
    c->tend[i] = (int)num[6];
    c->qname[i] = gt_names_add(&c->qnames, qn, (size_t)ql);
    c->qsize[i] = (int)num[8];
    c->qstrand[i] = (uint8_t)qminus;
    c->qstart[i] = (int)num[10];
    c->qend[i] = (int)num[11];
    f->cur = (char *)p + 1;
    f->line += blank + 1;
    return 1;
}

/* parse one record; 0 = ok, 1 = end of chunk, -1 = error (f->msg) */
static int parse_chain(chunk *k) {
    lf *f = &k->f;
    gt_chains *c = &k->c;
    char *row[13];
    chains_reserve(c);
    int64_t i = c->n;
    if (!fast_header(f, c)) {
        int wc = lf_chop(f, row, 13);
        if (wc == 0)
            return 1;
        if (wc < 12)
            LF_FAIL(f, "Expecting at least 12 words line \001 of \002");
        if (strcmp(row[0], "chain") != 0)
            LF_FAIL(f, "Expecting 'chain' line \001 of \002");
        int v;
        c->score[i] = atof(row[1]);
        c->tname[i] = gt_names_add(&c->tnames, row[2], strlen(row[2]));
        if (need_num(f, row, 3, &v))
            return -1;
        c->tsize[i] = v;
        if (wc >= 13) {
            if (need_num(f, row, 12, &v))
                return -1;
            c->id[i] = v;
        } else {
            c->id[i] = INT32_MIN; /* chainIdNext, assigned in file order later */
        }
        if (need_num(f, row, 5, &c->tstart[i]) || need_num(f, row, 6, &c->tend[i]))
            return -1;
        c->qname[i] = gt_names_add(&c->qnames, row[7], strlen(row[7]));
        if (need_num(f, row, 8, &c->qsize[i]))
            return -1;
        c->qstrand[i] = row[9][0] == '-' ? 1 : 0;
        if (need_num(f, row, 10, &c->qstart[i]) || need_num(f, row, 11, &c->qend[i]))
            return -1;
    }
    if (c->qstart[i] >= c->qend[i] || c->tstart[i] >= c->tend[i])
        LF_FAIL(f, "End before start line \001 of \002");
    if (c->qstart[i] < 0 || c->tstart[i] < 0)
        LF_FAIL(f, "Start before zero line \001 of \002");
    if (c->qend[i] > c->qsize[i] || c->tend[i] > c->tsize[i])
        LF_FAIL(f, "Past end of sequence line \001 of \002");
    if (k->tkeep && gt_names_find(k->tkeep, c->tnames.names[c->tname[i]]) < 0 &&
        gt_names_find(k->qkeep, c->qnames.names[c->qname[i]]) < 0 && skip_blocks(f)) {
        /* on no side this process nets: header only, no blocks */
        c->n++;
        c->blk_off[c->n] = c->nb;
        if (c->score[i] < k->stop_below) {
            k->stop = i;
            return 1;
        }
        return 0;
    }
    /* chainReadBlocks (chain.c:301-335) */
    int q = c->qstart[i], t = c->tstart[i];
    for (;;) {
        int v[3], bw;
        if (!fast_block_line(f, v, &bw)) {
            char *brow[3];
            bw = lf_chop(f, brow, 3);
            if (bw == 0)
                LF_FAIL(f, "Unexpected end of file in \002");
            if (need_num(f, brow, 0, &v[0]))
                return -1;
            if (bw >= 3 && (need_num(f, brow, 1, &v[1]) || need_num(f, brow, 2, &v[2])))
                return -1;
        }
        const int size = v[0];
        if (c->nb + 1 >= c->bcap) {
            c->bcap = c->bcap ? c->bcap * 2 : 1 << 16;
            c->bt = realloc(c->bt, c->bcap * 4);
            c->bq = realloc(c->bq, c->bcap * 4);
            c->bs = realloc(c->bs, c->bcap * 4);
        }
        c->bt[c->nb] = t;
        c->bq[c->nb] = q;
        c->bs[c->nb] = size;
        c->nb++;
        q += size;
        t += size;
        if (bw == 1)
            break;
        if (bw < 3)
            LF_FAIL(f, "Expecting 1 or 3 words line \001 of \002\n");
        t += v[1];
        q += v[2];
    }
    if (q != c->qend[i])
        LF_FAIL(f, "q end mismatch %d vs %d line \001 of \002\n", q, c->qend[i]);
    if (t != c->tend[i])
        LF_FAIL(f, "t end mismatch %d vs %d line \001 of \002\n", t, c->tend[i]);
    c->n++;
    c->blk_off[c->n] = c->nb;
    if (c->score[i] < k->stop_below) { /* read, not kept (chainNet.c:949-952) */
        k->stop = i;
        return 1;
    }
    return 0;
}

static void *parse_chunk(void *arg) {
    chunk *k = arg;
    k->t0 = now_s();
    k->c.blk_off = malloc(8);
    k->c.blk_off[0] = 0;
    if (k->lines > 0) { /* every block is a line: the arrays never grow */
        k->c.bcap = k->lines + 1;
        k->c.bt = malloc((size_t)k->c.bcap * 4);
        k->c.bq = malloc((size_t)k->c.bcap * 4);
        k->c.bs = malloc((size_t)k->c.bcap * 4);
    }
    int r;
    while ((r = parse_chain(k)) == 0)
        ;
    if (r < 0)
        k->err_line = k->f.line;
    /* (f.line now counts the chunk's lines up to where it stopped) */
    k->t1 = now_s();
    return NULL;
}

typedef struct parse_pool {
    chunk *K;
    int nk;
    _Atomic int next;
} parse_pool;

static void *parse_pool_thread(void *arg) {
    parse_pool *P = arg;
    for (int k; (k = atomic_fetch_add(&P->next, 1)) < P->nk;)
        parse_chunk(&P->K[k]);
    return NULL;
}

int gt_threads(void) {
    const char *s = getenv("GAC_THREADS");
    if (!s || !*s)
        s = getenv("OMP_NUM_THREADS");
    int n = s && *s ? atoi(s) : 0;
    if (n <= 0)
        n = gac_host_cpus(); /* (affinity mask and cgroup quota) */
    return n > 64 ? 64 : n;
}

void gt_parallel(int n, void *(*fn)(void *), void *args, size_t stride) {
    pthread_t *th = malloc((size_t)(n > 0 ? n : 1) * sizeof(pthread_t));
    for (int i = 1; i < n; ++i)
        pthread_create(&th[i], NULL, fn, (char *)args + (size_t)i * stride);
    if (n > 0)
        fn(args);
    for (int i = 1; i < n; ++i)
        pthread_join(th[i], NULL);
    free(th);
}

/* copy of the chunks' arrays into the stitched set (disjoint ranges) */
typedef struct stitch_job {
    gt_chains *c;
    chunk *K;
    const int64_t *c0, *b0;
    int32_t **tmaps, **qmaps;
    int nk;
    _Atomic int next;
} stitch_job;

static void *stitch_thread(void *arg) {
    stitch_job *J = arg;
    gt_chains *c = J->c;
    for (;;) {
        const int k = atomic_fetch_add(&J->next, 1);
        if (k >= J->nk)
            break;
        const gt_chains *s = &J->K[k].c;
        const int64_t take = s->n, o = J->c0[k], bo = J->b0[k];
        const int32_t *tmap = J->tmaps[k], *qmap = J->qmaps[k];
        for (int64_t i = 0; i < take; ++i) {
            const int64_t j = o + i;
            c->score[j] = s->score[i];
            c->tname[j] = tmap[s->tname[i]];
            c->tsize[j] = s->tsize[i];
            c->tstart[j] = s->tstart[i];
            c->tend[j] = s->tend[i];
            c->qname[j] = qmap[s->qname[i]];
            c->qsize[j] = s->qsize[i];
            c->qstart[j] = s->qstart[i];
            c->qend[j] = s->qend[i];
            c->qstrand[j] = s->qstrand[i];
            c->id[j] = s->id[i];
            c->blk_off[j + 1] = bo + s->blk_off[i + 1];
        }
        const int64_t nb = J->b0[k + 1] - bo;
        memcpy(c->bt + bo, s->bt, (size_t)nb * 4);
        memcpy(c->bq + bo, s->bq, (size_t)nb * 4);
        memcpy(c->bs + bo, s->bs, (size_t)nb * 4);
    }
    return NULL;
}

static void read_chains(const char *path, gt_chains *c, double stop_below, int keep_meta,
                        const gt_names *tkeep, const gt_names *qkeep);

void gt_read_chains(const char *path, gt_chains *c, double stop_below, int keep_meta) {
    read_chains(path, c, stop_below, keep_meta, NULL, NULL);
}

void gt_read_chains_keep(const char *path, gt_chains *c, double stop_below, int keep_meta,
                         const gt_names *tkeep, const gt_names *qkeep) {
    read_chains(path, c, stop_below, keep_meta, tkeep, qkeep);
}

typedef struct rc_free_job {
    chunk *K;
    int nk;
    void *cut;
    char *buf;
    size_t len;
} rc_free_job;

/* pages of a large heap block dropped first (madvise runs under the mm's
 * read lock; an munmap of populated pages holds the write lock while it
 * frees them, stalling every other thread's page faults -- the netting's
 * and the checks' first touches) */
static void drop_free(void *p, size_t len) {
    if (p && len > malloc_usable_size(p))
        len = malloc_usable_size(p); /* (never past the block) */
    if (p && len >= (1u << 20)) {
        const uintptr_t pg = 4096;
        const uintptr_t a = ((uintptr_t)p + pg - 1) & ~(pg - 1), b = ((uintptr_t)p + len) & ~(pg - 1);
        if (b > a)
            madvise((void *)a, b - a, MADV_DONTNEED);
    }
    free(p);
}

static void *rc_free_thread(void *arg) {
    rc_free_job *F = arg;
    for (int k = 0; k < F->nk; ++k) {
        gt_chains *c = &F->K[k].c;
        drop_free(c->bt, (size_t)c->bcap * 4);
        drop_free(c->bq, (size_t)c->bcap * 4);
        drop_free(c->bs, (size_t)c->bcap * 4);
        c->bt = c->bq = c->bs = NULL;
        gt_chains_free(c);
    }
    free(F->K);
    free(F->cut);
    drop_free(F->buf, F->len + 17);
    free(F);
    return NULL;
}

static void read_chains(const char *path, gt_chains *c, double stop_below, int keep_meta,
                        const gt_names *tkeep, const gt_names *qkeep) {
    memset(c, 0, sizeof(*c));
    const int timing = getenv("GAC_TIMING") != NULL;
    double t_mark = now_s();
#define RC_LAP(what)                                                               \
    do {                                                                           \
        if (timing) {                                                              \
            const double t_ = now_s();                                             \
            fprintf(stderr, "[gt_read_chains] %-16s %.3f s\n", what, t_ - t_mark); \
            t_mark = t_;                                                           \
        }                                                                          \
    } while (0)
    size_t len;
    char *buf = gt_slurp(path, &len);
    RC_LAP("read file");
    /* chunk boundaries at "\nchain": 8 chunks per thread, taken in order by
     * the threads as they finish (chain density varies along a file in score
     * order: equal thirds of the bytes are not equal work) */
    const int nthr = len < (8u << 20) ? 1 : gt_threads();
    const int nt = nthr > 1 ? 8 * nthr : 1;
    char **cut = malloc((size_t)(nt + 1) * sizeof(char *));
    cut[0] = buf;
    int nk = 1;
    for (int k = 1; k < nt; ++k) {
        char *p = buf + len / nt * k;
        if (p < cut[nk - 1])
            p = cut[nk - 1];
        char *h = NULL;
        while (p < buf + len) {
            char *nl = memchr(p, '\n', (size_t)(buf + len - p));
            if (!nl)
                break;
            if ((size_t)(buf + len - (nl + 1)) >= 5 && memcmp(nl + 1, "chain", 5) == 0) {
                h = nl + 1;
                break;
            }
            p = nl + 1;
        }
        if (h && h > cut[nk - 1])
            cut[nk++] = h;
    }
    cut[nk] = buf + len;
    chunk *K = calloc((size_t)nk, sizeof(chunk));
    for (int k = 0; k < nk; ++k) {
        K[k].f = (lf){.cur = cut[k], .end = cut[k + 1], .path = path, .line = 0,
                      .meta_to = keep_meta ? &K[k].c : NULL};
        K[k].lines = (cut[k + 1] - cut[k]) / 8; /* (block-array size hint: a line is ~10 B) */
        K[k].stop = -1;
        K[k].stop_below = stop_below;
        K[k].tkeep = tkeep;
        K[k].qkeep = qkeep;
    }
    RC_LAP("cut");
    {
        parse_pool P = {K, nk, 0};
        atomic_init(&P.next, 0);
        gac_run_threads(nthr < nk ? nthr : nk, parse_pool_thread, &P);
    }
    if (timing) {
        double s0 = 1e30, e0 = 1e30, s1 = 0, e1 = 0, sum = 0;
        for (int k = 0; k < nk; ++k) {
            s0 = K[k].t0 < s0 ? K[k].t0 : s0, s1 = K[k].t0 > s1 ? K[k].t0 : s1;
            e0 = K[k].t1 < e0 ? K[k].t1 : e0, e1 = K[k].t1 > e1 ? K[k].t1 : e1;
            sum += K[k].t1 - K[k].t0;
        }
        fprintf(stderr, "[gt_read_chains] %d chunks: starts within %.3f s, ends within %.3f s, "
                "mean %.3f s\n", nk, s1 - s0, e1 - e0, nk ? sum / nk : 0.0);
    }
    RC_LAP("parse");
    /* stitch in file order up to the first error or stop: a serial pass for
     * everything order-dependent (names, ids, metadata, errors, offsets),
     * then the chunks' arrays are copied in parallel */
    int64_t *c0 = calloc((size_t)nk + 1, 8), *b0 = calloc((size_t)nk + 1, 8);
    int32_t **tmaps = calloc((size_t)nk, sizeof(int32_t *)), **qmaps = calloc((size_t)nk, sizeof(int32_t *));
    int64_t line0 = 0;
    int nuse = 0;
    for (int k = 0; k < nk; ++k) {
        chunk *ch = &K[k];
        const int64_t take = ch->stop >= 0 ? ch->stop : ch->c.n; /* the stop chain is dropped */
        /* metadata: all '#' lines the chunk consumed (a stop drops the rest) */
        for (int32_t m = 0; m < ch->c.n_meta; ++m) {
            add_meta_at(c, ch->c.meta[m], c0[k] + ch->c.meta_at[m]);
        }
        int32_t *tmap = malloc((size_t)(ch->c.tnames.n ? ch->c.tnames.n : 1) * 4);
        int32_t *qmap = malloc((size_t)(ch->c.qnames.n ? ch->c.qnames.n : 1) * 4);
        for (int32_t i = 0; i < ch->c.tnames.n; ++i)
            tmap[i] = gt_names_add(&c->tnames, ch->c.tnames.names[i], strlen(ch->c.tnames.names[i]));
        for (int32_t i = 0; i < ch->c.qnames.n; ++i)
            qmap[i] = gt_names_add(&c->qnames, ch->c.qnames.names[i], strlen(ch->c.qnames.names[i]));
        tmaps[k] = tmap;
        qmaps[k] = qmap;
        /* ids: every header read so far consumes chainIdNext, kept or not */
        const int64_t nread = ch->c.n;
        for (int64_t i = 0; i < nread && !g_defer_ids; ++i)
            if (ch->c.id[i] == INT32_MIN)
                ch->c.id[i] = g_next_id++;
        ch->c.n = take; /* chains to copy */
        c0[k + 1] = c0[k] + take;
        b0[k + 1] = b0[k] + (take > 0 ? ch->c.blk_off[take] : 0);
        nuse = k + 1;
        const int err = ch->f.err && ch->stop < 0;
        if (err) {
            char msg[2048];
            size_t o = 0;
            for (const char *m = ch->f.msg; *m && o + 1 < sizeof(msg); ++m) {
                if (*m == '\001')
                    o += snprintf(msg + o, sizeof(msg) - o, "%lld", (long long)(line0 + ch->err_line));
                else if (*m == '\002')
                    o += snprintf(msg + o, sizeof(msg) - o, "%s", path);
                else
                    msg[o++] = *m;
                if (o >= sizeof(msg))
                    o = sizeof(msg) - 1;
            }
            msg[o] = 0;
            for (int j = 0; j < nk; ++j)
                gt_chains_free(&K[j].c);
            gt_abort("%s", msg);
        }
        line0 += ch->f.line; /* (a chunk that errs or stops is the last one used) */
        if (ch->stop >= 0)
            break;
    }
    chains_reserve_n(c, c0[nuse] + 1);
    c->blk_off[0] = 0;
    c->bcap = b0[nuse] + 1;
    c->bt = malloc((size_t)c->bcap * 4);
    c->bq = malloc((size_t)c->bcap * 4);
    c->bs = malloc((size_t)c->bcap * 4);
    stitch_job SJ = {c, K, c0, b0, tmaps, qmaps, nuse, 0};
    atomic_init(&SJ.next, 0);
    gac_run_threads(nuse < gt_threads() ? nuse : gt_threads(), stitch_thread, &SJ);
    c->n = c0[nuse];
    c->nb = b0[nuse];
    for (int k = 0; k < nuse; ++k) {
        free(tmaps[k]);
        free(qmaps[k]);
    }
    free(tmaps);
    free(qmaps);
    free(c0);
    free(b0);
    RC_LAP("stitch");
    /* the file text and the per-chunk arrays (GBs at whole-genome size:
     * 0.2 s of page freeing on C5 at 5 M chains) are released off the
     * caller's path */
    rc_free_job *F = malloc(sizeof(*F));
    *F = (rc_free_job){K, nk, cut, buf, len};
    pthread_attr_t at;
    pthread_attr_init(&at);
    pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
    pthread_t th;
    if (pthread_create(&th, &at, rc_free_thread, F) != 0)
        rc_free_thread(F);
    pthread_attr_destroy(&at);
    RC_LAP("free");
#undef RC_LAP
}

void gt_chains_free(gt_chains *c) {
    free(c->score);
    free(c->tname);
    free(c->tsize);
    free(c->tstart);
    free(c->tend);
    free(c->qname);
    free(c->qsize);
    free(c->qstart);
    free(c->qend);
    free(c->qstrand);
    free(c->id);
    free(c->blk_off);
    free(c->bt);
    free(c->bq);
    free(c->bs);
    gt_names_free(&c->tnames);
    gt_names_free(&c->qnames);
    for (int32_t i = 0; i < c->n_meta; ++i)
        free(c->meta[i]);
    free(c->meta);
    free(c->meta_at);
    memset(c, 0, sizeof(*c));
}

int gt_next_chain_id(void) { return g_next_id++; }

void gt_defer_chain_ids(int on) { g_defer_ids = on; }

/* decimal text of v at p, returns the end */
static char *put_int(char *p, int64_t v) {
    static const char dig2[201] = "00010203040506070809101112131415161718192021222324"
                                  "25262728293031323334353637383940414243444546474849"
                                  "50515253545556575859606162636465666768697071727374"
                                  "75767778798081828384858687888990919293949596979899";
    uint64_t u = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
    if (v < 0)
        *p++ = '-';
    /* the digit count first, then the digits straight into place, two per
     * step (no staging copy: a variable-length memcpy is a library call per
     * number, and the nets print ~150 M of them); 32-bit arithmetic when the
     * value fits, as nearly all coordinates do */
    static const uint32_t p10[10] = {0u,      10u,      100u,      1000u,      10000u,
                                     100000u, 1000000u, 10000000u, 100000000u, 1000000000u};
    if (u >> 32) {
        int nd = 1;
        for (uint64_t t = 10; nd < 20 && u >= t; t *= 10)
            ++nd;
        char *const e = p + nd;
        char *q = e;
        while (u >= 100) {
            const unsigned r = (unsigned)(u % 100);
            u /= 100;
            q -= 2;
            memcpy(q, dig2 + 2 * r, 2);
        }
        if (u >= 10) {
            q -= 2;
            memcpy(q, dig2 + 2 * u, 2);
        } else {
            *--q = (char)('0' + u);
        }
        return e;
    }
    uint32_t w = (uint32_t)u;
    int nd = ((32 - __builtin_clz(w | 1)) * 1233) >> 12; /* floor(log10) or one less */
    nd += (nd < 10 && w >= p10[nd]) ? 1 : 0;
    if (nd == 0)
        nd = 1;
    char *const e = p + nd;
    char *q = e;
    while (w >= 100) {
        const uint32_t r = w % 100;
        w /= 100;
        q -= 2;
        memcpy(q, dig2 + 2 * r, 2);
    }
    if (w >= 10) {
        q -= 2;
        memcpy(q, dig2 + 2 * w, 2);
    } else {
        *--q = (char)('0' + w);
    }
    return e;
}

/* block lines "size\tdt\tdq" and the last "size", then the blank line
 * (chainWrite, chain.c:214-226), formatted without stdio */
static void write_blocks(FILE *f, const int32_t *bt, const int32_t *bq, const int32_t *bs,
                         int64_t nb) {
    char buf[1 << 14];
    char *p = buf;
    for (int64_t b = 0; b < nb; ++b) {
        if (p - buf > (int)sizeof(buf) - 64) {
            fwrite(buf, 1, (size_t)(p - buf), f);
            p = buf;
        }
        p = put_int(p, bs[b]);
        if (b + 1 < nb) {
            *p++ = '\t';
            p = put_int(p, (int64_t)bt[b + 1] - (bt[b] + bs[b]));
            *p++ = '\t';
            p = put_int(p, (int64_t)bq[b + 1] - (bq[b] + bs[b]));
        }
        *p++ = '\n';
    }
    *p++ = '\n';
    fwrite(buf, 1, (size_t)(p - buf), f);
}

/* "%1.0f" of a score: integral values below 2^53 as integers (the same
 * text), anything else (fractions, -0, huge, NaN) through printf */
static char *put_score(char *p, double x) {
    if (x == (double)(int64_t)x && x > -9007199254740992.0 && x < 9007199254740992.0 &&
        !(x == 0.0 && signbit(x)))
        return put_int(p, (int64_t)x);
    return p + sprintf(p, "%1.0f", x);
}

static char *put_str(char *p, const char *s) {
    const size_t n = strlen(s);
    memcpy(p, s, n);
    return p + n;
}

/* the header line of chainWrite (chain.c:209-213), formatted without stdio */
static void write_header(FILE *f, double score, const char *tname, int32_t tsize, int32_t tstart,
                         int32_t tend, const char *qname, int32_t qsize, int qminus,
                         int32_t qstart, int32_t qend, int32_t id) {
    const size_t need = strlen(tname) + strlen(qname) + 400;
    char small[1024], *buf = need <= sizeof(small) ? small : malloc(need), *p = buf;
    p = put_str(p, "chain ");
    p = put_score(p, score);
    *p++ = ' ';
    p = put_str(p, tname);
    *p++ = ' ';
    p = put_int(p, tsize);
    p = put_str(p, " + ");
    p = put_int(p, tstart);
    *p++ = ' ';
    p = put_int(p, tend);
    *p++ = ' ';
    p = put_str(p, qname);
    *p++ = ' ';
    p = put_int(p, qsize);
    *p++ = ' ';
    *p++ = qminus ? '-' : '+';
    *p++ = ' ';
    p = put_int(p, qstart);
    *p++ = ' ';
    p = put_int(p, qend);
    *p++ = ' ';
    p = put_int(p, id);
    *p++ = '\n';
    fwrite(buf, 1, (size_t)(p - buf), f);
    if (buf != small)
        free(buf);
}

void gt_write_chain(FILE *f, const gt_chains *c, int64_t i, double score, int32_t id) {
    write_header(f, score, c->tnames.names[c->tname[i]], c->tsize[i], c->tstart[i], c->tend[i],
                 c->qnames.names[c->qname[i]], c->qsize[i], c->qstrand[i], c->qstart[i],
                 c->qend[i], id);
    const int64_t b0 = c->blk_off[i];
    write_blocks(f, c->bt + b0, c->bq + b0, c->bs + b0, c->blk_off[i + 1] - b0);
}

void gt_write_chain_raw(FILE *f, double score, const char *tname, int32_t tsize, int32_t tstart,
                        int32_t tend, const char *qname, int32_t qsize, int qminus,
                        int32_t qstart, int32_t qend, int32_t id, const int32_t *bt,
                        const int32_t *bq, const int32_t *bs, int64_t nb) {
    write_header(f, score, tname, tsize, tstart, tend, qname, qsize, qminus, qstart, qend, id);
    write_blocks(f, bt, bq, bs, nb);
}

int32_t *gt_seq_map(gac_ctx *ctx, int side, const gt_names *names) {
    int32_t *m = malloc((size_t)(names->n ? names->n : 1) * 4);
    for (int32_t k = 0; k < names->n; ++k)
        m[k] = gac_genome_seq_index(ctx, side, names->names[k]);
    return m;
}

typedef struct pw_job {
    int64_t n, per;
    void (*fn)(FILE *, int64_t, void *);
    void *arg;
} pw_job;

static void pw_run(FILE *f, int64_t r, void *p) {
    pw_job *J = p;
    const int64_t a = r * J->per, b = a + J->per < J->n ? a + J->per : J->n;
    for (int64_t i = a; i < b; ++i)
        J->fn(f, i, J->arg);
}

void gt_par_write(FILE *out, int64_t n, void (*fn)(FILE *f, int64_t i, void *arg), void *arg) {
    if (n <= 0)
        return;
    /* runs of at most 64 items (≈15 KB of chain text): formatting buffers
     * stay small and are reused (no page faults), the writer batches them
     * into one writev per 256 runs (C2 chains: 54 -> 23 ms to /dev/null
     * with 16 threads, scripts/gpu_write_probe.sh) */
    int64_t per = n / (64 * (int64_t)gt_threads()) + 1;
    if (per > 64)
        per = 64;
    if (getenv("GAC_RUN_ITEMS"))
        per = atoll(getenv("GAC_RUN_ITEMS"));
    pw_job J = {n, per, fn, arg};
    if (gac_par_output(out, (n + per - 1) / per, pw_run, &J) != 0)
        gt_abort("write error\n");
}

/* ------------------------------------------------------------ sizes */
void gt_read_sizes(const char *path, gt_sizes *s) {
    memset(s, 0, sizeof(*s));
    size_t len;
    char *buf = gt_slurp(path, &len);
    lf f = {.cur = buf, .end = buf + len, .path = path, .line = 0};
    int32_t cap = 0;
    char *row[3];
    int wc;
    while ((wc = lf_chop(&f, row, 3)) != 0) {
        if (wc != 2)
            gt_abort("Expecting 2 words line %lld of %s got %d", (long long)f.line, path, wc);
        if (gt_names_find(&s->names, row[0]) >= 0)
            gt_abort("Duplicate %s in %s", row[0], path);
        int32_t id = gt_names_add(&s->names, row[0], strlen(row[0]));
        if (id >= cap) {
            cap = cap ? cap * 2 : 1024;
            s->size = realloc(s->size, (size_t)cap * sizeof(int32_t));
        }
        int v;
        if (need_num(&f, row, 1, &v))
            gt_abort("Expecting number field 2 line %lld of %s, got %s", (long long)f.line, path,
                     row[1]);
        s->size[id] = v;
    }
    free(buf);
}

void gt_sizes_free(gt_sizes *s) {
    gt_names_free(&s->names);
    free(s->size);
    memset(s, 0, sizeof(*s));
}
