/* chainNet -- make alignment nets out of chains (with -rescore on an MI355X).
 *
 * Drop-in for the reference's src/chainNet/chainNet.c (Hiller version with
 * -rescore): same command line, options, defaults, error checks and .net
 * output.  Netting runs on the host (libgachain gac_net_*, array-indexed,
 * no O(fills x blocks) rescans); with -rescore every printed partial
 * target-side fill is rescored in ONE batched GPU call (gac_score_ranges),
 * replacing the per-fill chainSubsetOnT + chainCalcScore of subchainInfo
 * (:795-843). */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <math.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gac_tool.h"
#include "gachain.h"
#include "host/gac_host.h"

static const gt_spec k_opts[] = {
    {"minSpace", GT_INT},      {"minFill", GT_INT},      {"minScore", GT_DOUBLE},
    {"inclHap", GT_BOOL},      {"rescore", GT_BOOL},     {"tNibDir", GT_STRING},
    {"qNibDir", GT_STRING},    {"scoreScheme", GT_STRING}, {"linearGap", GT_STRING},
    {"nranks", GT_INT},        {"rank", GT_INT},         {"gpu", GT_INT},
    {NULL, 0},
};

static void usage(int min_space, double min_score) {
    gt_abort(
        "chainNet - Make alignment nets out of chains (MI355X / libgachain)\n"
        "usage:\n"
        "   chainNet in.chain target.sizes query.sizes target.net query.net\n"
        "where:\n"
        "   in.chain is the chain file sorted by score\n"
        "   target.sizes contains the size of the target sequences\n"
        "   query.sizes contains the size of the query sequences\n"
        "   target.net is the output over the target genome\n"
        "   query.net is the output over the query genome\n"
        "options:\n"
        "   -minSpace=N - minimum gap size to fill, default %d\n"
        "   -minFill=N  - default half of minSpace\n"
        "   -minScore=N - minimum chain score to consider, default %.1lf\n"
        "   -verbose=N - Alter verbosity (default 1)\n"
        "   -inclHap - include query sequences name in the form *_hap*|*_alt*.\n"
        "              Normally these are excluded from nets as being haplotype\n"
        "              pseudochromosomes\n"
        "   -rescore                    compute the real score of the sub-net (on the GPU)\n"
        "   -tNibDir=fileName           target genome file (2bit)\n"
        "   -qNibDir=fileName           query genome file (2bit)\n"
        "   -scoreScheme=fileName       Read the scoring matrix from a blastz-format file\n"
        "   -linearGap=<medium|loose|filename> Specify type of linearGap to use.\n"
        "   -nranks=N -rank=R           multi-GPU run (one process per GPU, same node): rank R\n"
        "                               nets its share of the chromosome sides and writes its\n"
        "                               part of both nets in place; rank 0 waits for all parts\n"
        "   -gpu=D                      device index (default: R with -nranks, else 0)\n",
        min_space, min_score);
}

typedef struct net_out {
    const gac_net *net;
    int side;
    const int64_t *tscores;
    const char *path;
    const gt_chains *c;
    int threaded, rc;
    char err[1024];
    /* -rescore: the target net formatted ahead of its scores (pre_net) */
    gac_net_wpre *pre;
    pthread_t pre_th;
    int pre_started, pre_rc;
} net_out;

static gt_ranks g_rk;

static void *pre_net(void *arg) {
    net_out *w = arg;
    const int m = g_rk.n <= 1 || g_rk.me == 0;
    w->pre_rc = gac_net_write_begin(w->net, w->side, m ? (const char *const *)w->c->meta : NULL,
                                    m ? w->c->n_meta : 0, &w->pre);
    return NULL;
}

/* the prepared target net with its scores */
static int write_pre(net_out *w, FILE *f) {
    const int rc = gac_net_write_end(w->pre, w->tscores, f);
    w->pre = NULL;
    return rc;
}

static void *write_net(void *arg) {
    net_out *w = arg;
    if (w->pre_started) {
        gt_helper_join(w->pre_th);
        w->pre_started = 0;
        if (w->pre_rc != GAC_OK) {
            gac_net_write_free(w->pre);
            w->pre = NULL;
        }
    }
    if (w->pre && g_rk.n <= 1) {
        FILE *f = strcmp(w->path, "stdout") ? gac_open_output(w->path) : stdout;
        w->rc = f ? write_pre(w, f) : GAC_E_IO;
        if (f && f != stdout && gac_close_output(f) != 0 && w->rc == GAC_OK)
            w->rc = GAC_E_IO;
        if (w->rc != GAC_OK)
            snprintf(w->err, sizeof(w->err), "write error on %s", w->path);
        return NULL;
    }
    if (g_rk.n > 1 && !w->pre) {
        /* -nranks: this rank's part formatted on all threads into buffers and
         * written in place from them (rank 0's part carries the '#' lines) */
        const int m = g_rk.me == 0;
        char **bufs = NULL;
        size_t *lens = NULL;
        int64_t nb = 0;
        w->rc = gac_net_format(w->net, w->side, w->tscores,
                               m ? (const char *const *)w->c->meta : NULL, m ? w->c->n_meta : 0,
                               &bufs, &lens, &nb);
        if (w->rc != GAC_OK) {
            snprintf(w->err, sizeof(w->err), "%s", gac_last_error());
            return NULL;
        }
        size_t len = 0;
        for (int64_t k = 0; k < nb; ++k)
            len += lens[k];
        if (getenv("GAC_TIMING")) /* (the per-rank table of DESIGN §6) */
            fprintf(stderr, "[rank %d/%d] %s part: %zu bytes\n", g_rk.me, g_rk.n,
                    w->side == GAC_T ? "target net" : "query net", len);
        gt_ranks_place_bufs(&g_rk, w->path, bufs, lens, nb);
        for (int64_t k = 0; k < nb; ++k)
            free(bufs[k]);
        free(bufs);
        free(lens);
        return NULL;
    }
    if (g_rk.n > 1) {
        /* -nranks with the preformatted target net: formatted in memory and
         * written in place (rank 0's part carries the '#' lines) */
        char *buf = NULL;
        size_t len = 0;
        FILE *mf = open_memstream(&buf, &len);
        const int m = g_rk.me == 0;
        if (w->pre)
            w->rc = mf ? write_pre(w, mf) : GAC_E_IO;
        else
            w->rc = mf ? gac_net_write_file(w->net, w->side, w->tscores, mf,
                                            m ? (const char *const *)w->c->meta : NULL,
                                            m ? w->c->n_meta : 0)
                       : GAC_E_IO;
        if (mf && fclose(mf) != 0 && w->rc == GAC_OK)
            w->rc = GAC_E_IO;
        if (w->rc == GAC_OK) {
            if (getenv("GAC_TIMING")) /* (the per-rank table of DESIGN §6) */
                fprintf(stderr, "[rank %d/%d] %s part: %zu bytes\n", g_rk.me, g_rk.n,
                        w->side == GAC_T ? "target net" : "query net", len);
            gt_ranks_place(&g_rk, w->path, buf, len);
        }
        else
            snprintf(w->err, sizeof(w->err), "write error on %s", w->path);
        free(buf);
        return NULL;
    }
    w->rc = gac_net_write(w->net, w->side, w->tscores, w->path, (const char *const *)w->c->meta,
                          w->c->n_meta);
    if (w->rc != GAC_OK) /* thread-local error text */
        snprintf(w->err, sizeof(w->err), "%s", gac_last_error());
    return NULL;
}

/* block lists of the chains owning a rescored fill, copied in parallel */
typedef struct subset_copy {
    const gt_chains *c;
    const int64_t *src, *goff;
    int32_t *bt, *bq, *bs;
    int64_t n;
    _Atomic int64_t next;
} subset_copy;

static void *subset_copy_thread(void *arg) {
    subset_copy *J = arg;
    for (;;) {
        const int64_t a = atomic_fetch_add(&J->next, 4096);
        if (a >= J->n)
            break;
        const int64_t b = a + 4096 < J->n ? a + 4096 : J->n;
        for (int64_t j = a; j < b; ++j) {
            const int64_t i = J->src[j], b0 = J->c->blk_off[i], nb = J->c->blk_off[i + 1] - b0;
            memcpy(J->bt + J->goff[j], J->c->bt + b0, nb * 4);
            memcpy(J->bq + J->goff[j], J->c->bq + b0, nb * 4);
            memcpy(J->bs + J->goff[j], J->c->bs + b0, nb * 4);
        }
    }
    return NULL;
}

/* -rescore: the genome word runs under the chains' blocks, computed while
 * the chains are netted (the device thread uploads just these) */
typedef struct runs_job {
    gt_runs *R;
    const gt_chains *c;
    const char *t2bit, *q2bit;
} runs_job;

static void *runs_thread(void *arg) {
    runs_job *j = arg;
    gt_runs_build(j->R, j->c, j->t2bit, j->q2bit);
    return NULL;
}

/* With -rescore: the whole chain set goes to HBM on a helper thread while
 * the chains are netted (the usual case: every chain's sequences are in the
 * 2bit files).  If a sequence is missing -- the reference only looks up the
 * chains of rescored fills -- or the upload fails, the main thread uploads
 * just the chains owning a rescored fill, as before. */
typedef struct pre_upload {
    gt_device *dev;
    const gt_chains *c;
    const uint8_t *tkeep; /* -nranks: this rank's target sides (NULL: all) */
    const int32_t *tix;   /* chain -> target sizes index */
    gac_chainset *cs;     /* NULL: use the subset path */
    int32_t *remap;       /* chain -> uploaded index (-1: not uploaded); NULL: identity */
    pthread_t th;
    int started;
} pre_upload;

static void *pre_upload_thread(void *arg) {
    pre_upload *u = arg;
    gac_ctx *ctx = gt_device_wait(u->dev);
    if (!ctx)
        return NULL;
    const gt_chains *c = u->c;
    int32_t *tmap = gt_seq_map(ctx, GAC_T, &c->tnames), *qmap = gt_seq_map(ctx, GAC_Q, &c->qnames);
    int ok = 1;
    for (int32_t k = 0; k < c->qnames.n && ok; ++k)
        ok = qmap[k] >= 0;
    if (!u->tkeep)
        for (int32_t k = 0; k < c->tnames.n && ok; ++k)
            ok = tmap[k] >= 0;
    if (ok && !u->tkeep) { /* the whole set */
        int32_t *ts = malloc((size_t)(c->n ? c->n : 1) * 4), *qs = malloc((size_t)(c->n ? c->n : 1) * 4);
        for (int64_t i = 0; i < c->n; ++i) {
            ts[i] = tmap[c->tname[i]];
            qs[i] = qmap[c->qname[i]];
        }
        gac_chainset_desc d = {c->n, ts, qs, c->qstrand, c->blk_off, c->nb, c->bt, c->bq, c->bs};
        if (gac_chains_upload(ctx, &d, &u->cs) != GAC_OK)
            u->cs = NULL;
        free(ts);
        free(qs);
    } else if (ok) { /* -nranks: the chains on this rank's target sides */
        int32_t *remap = malloc((size_t)(c->n ? c->n : 1) * 4);
        int64_t m = 0, mb = 0;
        for (int64_t i = 0; i < c->n; ++i) {
            remap[i] = -1;
            if (u->tkeep[u->tix[i]] && tmap[c->tname[i]] >= 0) {
                remap[i] = (int32_t)m++;
                mb += c->blk_off[i + 1] - c->blk_off[i];
            }
        }
        int32_t *ts = malloc((size_t)(m ? m : 1) * 4), *qs = malloc((size_t)(m ? m : 1) * 4);
        uint8_t *st = malloc((size_t)(m ? m : 1));
        int64_t *off = malloc((size_t)(m + 1) * 8), *src = malloc((size_t)(m ? m : 1) * 8);
        int32_t *bt = malloc((size_t)(mb ? mb : 1) * 4), *bq = malloc((size_t)(mb ? mb : 1) * 4),
                *bs = malloc((size_t)(mb ? mb : 1) * 4);
        off[0] = 0;
        for (int64_t i = 0; i < c->n; ++i)
            if (remap[i] >= 0) {
                const int64_t j = remap[i];
                src[j] = i;
                ts[j] = tmap[c->tname[i]];
                qs[j] = qmap[c->qname[i]];
                st[j] = c->qstrand[i];
                off[j + 1] = off[j] + (c->blk_off[i + 1] - c->blk_off[i]);
            }
        subset_copy sj = {c, src, off, bt, bq, bs, m, 0};
        atomic_init(&sj.next, 0);
        gac_run_threads(gt_threads(), subset_copy_thread, &sj);
        gac_chainset_desc d = {m, ts, qs, st, off, mb, bt, bq, bs};
        if (gac_chains_upload(ctx, &d, &u->cs) != GAC_OK) {
            u->cs = NULL;
            free(remap);
        } else {
            u->remap = remap;
        }
        free(ts);
        free(qs);
        free(st);
        free(off);
        free(src);
        free(bt);
        free(bq);
        free(bs);
    }
    free(tmap);
    free(qmap);
    return NULL;
}


/* ---------------------------------------------------------------- ranks
 * -nranks=N -rank=R: N processes (one per GPU of one node) run the same
 * command.  A chromosome side's net depends only on the chains on that
 * sequence (chainNet.c:557-679 add each chain to its own target and query
 * trees), so each rank takes a contiguous run of the target and of the
 * query sequences (assign_range); the sequences' sections of a net are in
 * sizes-file order, so rank R's part of each net is one contiguous piece of
 * it: rank R formats it in memory and writes it in place once the lower
 * ranks' sizes are known (gt_ranks_place); rank 0 waits for all parts. */
/* keep[k] for this rank: a contiguous run of the sizes file's sequences,
 * runs balanced by sequence length (the same on every rank and known before
 * the chains are read); kept names go to `kept` */
static int assign_range(const gt_sizes *sz, uint8_t *keep, gt_names *kept) {
    const int32_t n = sz->names.n;
    int64_t total = 0, before = 0;
    for (int32_t k = 0; k < n; ++k)
        total += sz->size[k];
    int any = 0;
    memset(kept, 0, sizeof(*kept));
    for (int32_t k = 0; k < n; ++k) {
        /* the rank whose share of the length holds this sequence's middle */
        int r = total > 0 ? (int)(((2 * before + sz->size[k]) * (int64_t)g_rk.n) / (2 * total)) : 0;
        if (r >= g_rk.n)
            r = g_rk.n - 1;
        keep[k] = r == g_rk.me;
        if (keep[k]) {
            gt_names_add(kept, sz->names.names[k], strlen(sz->names.names[k]));
            any = 1;
        }
        before += sz->size[k];
    }
    return any;
}

/* chainNet's per-chain checks (score order, names in the sizes files, sizes
 * agree): q/t sequence indices of every chain, the first failing chain */
typedef struct check_job {
    const gt_chains *c;
    const gt_sizes *ts, *qs;
    int32_t *tix, *qix;
    const int32_t *tmap, *qmap; /* the chain set's distinct names -> sizes rows */
    int64_t n;
    _Atomic int64_t next, first_bad;
} check_job;

static void *check_thread(void *arg) {
    check_job *J = arg;
    const gt_chains *c = J->c;
    for (;;) {
        const int64_t a = atomic_fetch_add(&J->next, 65536);
        if (a >= J->n)
            return NULL;
        const int64_t b = a + 65536 < J->n ? a + 65536 : J->n;
        for (int64_t i = a; i < b; ++i) {
            int ok = i == 0 || c->score[i - 1] < 0 || c->score[i] <= c->score[i - 1];
            J->qix[i] = J->qmap[c->qname[i]];
            J->tix[i] = J->tmap[c->tname[i]];
            ok = ok && J->qix[i] >= 0 && J->qs->size[J->qix[i]] == c->qsize[i] && J->tix[i] >= 0 &&
                 J->ts->size[J->tix[i]] == c->tsize[i];
            if (!ok) {
                int64_t cur = atomic_load(&J->first_bad);
                while (i < cur && !atomic_compare_exchange_weak(&J->first_bad, &cur, i)) {
                }
                break; /* later chains of this run cannot come first */
            }
        }
    }
}


/* chainNet -rescore's rescoring list: the target fills that are partial
 * (flag 1) and printed (flag 2), in fill order */
int main(int argc, char *argv[]) {
    gt_stage("");
    int min_space = 25;
    double min_score = 2000;
    gt_options(&argc, argv, k_opts);
    if (argc != 6)
        usage(min_space, min_score);
    min_space = gt_opt_int("minSpace", min_space);
    const int min_fill = gt_opt_int("minFill", min_space / 2);
    min_score = gt_opt_int("minScore", (int)min_score); /* optionInt, chainNet.c:1015 */
    const int incl_hap = gt_opt_exists("inclHap");
    const int rescore = gt_opt_exists("rescore");
    const char *tnib = NULL, *qnib = NULL;
    int32_t mat[16];
    gac_gapcalc *gap = NULL;
    if (rescore) {
        min_score = 0;
        tnib = gt_opt_str("tNibDir", NULL);
        qnib = gt_opt_str("qNibDir", NULL);
        if (tnib == NULL)
            gt_abort("With -rescore you must specify the target genome file (parameter -tNibDir)\n");
        if (qnib == NULL)
            gt_abort("With -rescore you must specify the query genome file (parameter -qNibDir)\n");
        const char *gap_name = gt_opt_str("linearGap", NULL);
        const char *scheme = gt_opt_str("scoreScheme", NULL);
        if (scheme)
            gt_verbose(1, "Reading scoring matrix from %s\n", scheme);
        gt_check(gac_scheme_read(scheme, mat, NULL, NULL, NULL));
        if (gap_name == NULL)
            gt_abort("Must specify linear gap costs.  Use 'loose' or 'medium' for defaults\n");
        gt_check(gac_gapcalc_build(gap_name, &gap));
        gt_verbose(1, "-rescore is set: read target/query genome from %s and %s. scoreSchemeName %s. gap costs %s.\n",
                   tnib, qnib, scheme ? scheme : "default", gap_name);
        if (!gac_is_twobit_file(tnib) || !gac_is_twobit_file(qnib))
            gt_abort("ERROR: only 2bit genome files are supported (got %s, %s)\n", tnib, qnib);
    }
    const char *chain_file = argv[1], *tsizes_file = argv[2], *qsizes_file = argv[3];
    const char *tnet = argv[4], *qnet = argv[5];
    gt_ranks_init(&g_rk, gt_opt_int("nranks", 1), gt_opt_int("rank", 0), tnet);
    const int multi = g_rk.n > 1;
    gt_set_gpu(gt_opt_int("gpu", multi ? g_rk.me : 0));
    if (multi) {
        if (!strcmp(tnet, "stdout") || !strcmp(qnet, "stdout"))
            gt_abort("-nranks needs file names for both nets (not stdout)");
        gt_ranks_clear_markers(&g_rk, tnet);
        gt_ranks_clear_markers(&g_rk, qnet);
    }

    /* with -rescore the device and both genomes come up on a helper thread
     * while the chains are read and netted (with -nranks once this rank knows
     * it rescores target fills) */
    gt_device dev;
    memset(&dev, 0, sizeof(dev));
    /* GAC_NET_SPARSE=1: upload only the genome words under the chains'
     * blocks (a tenth of a whole-genome query; for genomes that crowd HBM):
     * the device thread opens the context and maps the .2bit files while the
     * chains are read, then waits for the word runs.  Off by default: the
     * whole upload overlaps HIP start-up anyway, and building the runs costs
     * host time (C2: 274 vs 288 ms median single-GPU, 860-879 vs 871-927 ms
     * with 4 ranks on one GPU; profiles/r02h_sparse) */
    const char *sp = getenv("GAC_NET_SPARSE");
    const int sparse = rescore && sp && *sp == '1';
    gt_runs runs;
    gt_runs_init(&runs);
    if (rescore && !multi)
        gt_device_start_ex(&dev, tnib, qnib, mat, gap, NULL, sparse ? &runs : NULL);

    gt_sizes qs, ts;
    gt_stage("options + setup");
    gt_read_sizes(qsizes_file, &qs);
    gt_read_sizes(tsizes_file, &ts);
    gt_verbose(1, "Got %d chroms in %s, %d in %s\n", ts.names.n, tsizes_file, qs.names.n,
               qsizes_file);
    /* open outputs like mustOpen before reading (with -nranks only rank 0
     * truncates them: the other ranks write their parts in place later) */
    if (!multi || g_rk.me == 0) {
        FILE *tf = gt_must_open(tnet, "w");
        FILE *qf = gt_must_open(qnet, "w");
        if (tf != stdout)
            fclose(tf);
        if (qf != stdout)
            fclose(qf);
    } else {
        for (int k = 0; k < 2; ++k) {
            const char *o = k ? qnet : tnet;
            const int fd = open(o, O_WRONLY | O_CREAT, 0666);
            if (fd < 0)
                gt_abort("Can't open %s to write: %s", o, strerror(errno));
            close(fd);
        }
    }

    /* -nranks: this rank's chromosome sides (from the sizes files), the
     * device with just its target sequences, and only the chains on its
     * sides parsed in full */
    uint8_t *tkeep = NULL, *qkeep = NULL;
    gt_names tkept, qkept;
    if (multi) {
        tkeep = malloc((size_t)ts.names.n + 1);
        qkeep = malloc((size_t)qs.names.n + 1);
        const int own_t = assign_range(&ts, tkeep, &tkept);
        assign_range(&qs, qkeep, &qkept);
        if (rescore && own_t)
            gt_device_start_ex(&dev, tnib, qnib, mat, gap, &tkept, sparse ? &runs : NULL);
        gt_stage("rank sides");
    }
    gt_chains c;
    if (multi)
        gt_read_chains_keep(chain_file, &c, min_score, 1, &tkept, &qkept);
    else
        gt_read_chains(chain_file, &c, min_score, 1);
    gt_stage("read chains");
    int32_t *tix = malloc((c.n ? c.n : 1) * 4), *qix = malloc((c.n ? c.n : 1) * 4);
    {
        /* in parallel; the first failing chain in file order is re-checked
         * serially for its message */
        /* (each distinct name looked up once, not once per chain) */
        int32_t *tmap = malloc((size_t)(c.tnames.n ? c.tnames.n : 1) * 4);
        int32_t *qmap = malloc((size_t)(c.qnames.n ? c.qnames.n : 1) * 4);
        for (int32_t k = 0; k < c.tnames.n; ++k)
            tmap[k] = gt_names_find(&ts.names, c.tnames.names[k]);
        for (int32_t k = 0; k < c.qnames.n; ++k)
            qmap[k] = gt_names_find(&qs.names, c.qnames.names[k]);
        check_job cj = {&c, &ts, &qs, tix, qix, tmap, qmap, c.n, 0};
        atomic_init(&cj.next, 0);
        atomic_init(&cj.first_bad, c.n);
        gac_run_threads(gt_threads(), check_thread, &cj);
        const int64_t bad = atomic_load(&cj.first_bad);
        if (bad < c.n) {
            const int64_t i = bad;
            if (i > 0 && c.score[i - 1] >= 0 && c.score[i] > c.score[i - 1])
                gt_abort("%s must be sorted in order of score", chain_file);
            const char *qn = c.qnames.names[c.qname[i]], *tn = c.tnames.names[c.tname[i]];
            if (qix[i] < 0)
                gt_abort("hashMustFindVal: '%s' not found", qn);
            if (qs.size[qix[i]] != c.qsize[i])
                gt_abort("%s is %d in %s but %d in %s", qn, c.qsize[i], chain_file,
                         qs.size[qix[i]], qsizes_file);
            if (tix[i] < 0)
                gt_abort("hashMustFindVal: '%s' not found", tn);
            gt_abort("%s is %d in %s but %d in %s", tn, c.tsize[i], chain_file, ts.size[tix[i]],
                     tsizes_file);
        }
        free(tmap);
        free(qmap);
    }
    gt_stage("chain checks");
    runs_job rj = {&runs, &c, tnib, qnib};
    if (dev.started && dev.runs) {
        pthread_t rth;
        if (pthread_create(&rth, NULL, runs_thread, &rj) == 0)
            gt_helper_add(rth); /* gt_abort joins it before exiting */
        else
            runs_thread(&rj);
    }
    pre_upload pu;
    memset(&pu, 0, sizeof(pu));
    if (rescore && dev.started) {
        pu.dev = &dev;
        pu.c = &c;
        pu.tkeep = tkeep;
        pu.tix = tix;
        pu.started = pthread_create(&pu.th, NULL, pre_upload_thread, &pu) == 0;
        if (pu.started) /* gt_abort joins it before exiting */
            gt_helper_add(pu.th);
    }
    gac_net_input in;
    memset(&in, 0, sizeof(in));
    in.n_chains = c.n;
    in.score = c.score;
    in.id = c.id;
    in.t_seq = tix;
    in.q_seq = qix;
    in.q_strand = c.qstrand;
    in.t_start = c.tstart;
    in.t_end = c.tend;
    in.q_start = c.qstart;
    in.q_end = c.qend;
    in.blk_off = c.blk_off;
    in.blk_t = c.bt;
    in.blk_q = c.bq;
    in.blk_size = c.bs;
    in.n_tseq = ts.names.n;
    in.t_names = (const char *const *)ts.names.names;
    in.t_sizes = ts.size;
    in.n_qseq = qs.names.n;
    in.q_names = (const char *const *)qs.names.names;
    in.q_sizes = qs.size;
    gac_net_opts opt = {min_space, min_fill, min_score, incl_hap};
    gac_net *net = NULL;
    if (multi)
        gt_check(gac_net_build_subset(&in, &opt, tkeep, qkeep, &net));
    else
        gt_check(gac_net_build(&in, &opt, &net));
    gt_stage("netting");
    if (multi && getenv("GAC_TIMING")) { /* this rank's work (DESIGN §6's per-rank table) */
        int64_t tb = 0, qb = 0;
        for (int32_t k = 0; k < ts.names.n; ++k)
            tb += tkeep[k] ? ts.size[k] : 0;
        for (int32_t k = 0; k < qs.names.n; ++k)
            qb += qkeep[k] ? qs.size[k] : 0;
        fprintf(stderr, "[rank %d/%d] sides: %d target seqs (%lld bases), %d query seqs (%lld "
                        "bases); %lld chain headers, %lld blocks parsed; fills: %lld target, %lld query\n",
                g_rk.me, g_rk.n, tkept.n, (long long)tb, qkept.n, (long long)qb, (long long)c.n,
                (long long)c.blk_off[c.n], (long long)gac_net_fill_count(net, GAC_T),
                (long long)gac_net_fill_count(net, GAC_Q));
    }
    gt_verbose(1, "Finishing nets\n");

    /* the two nets are independent files, written concurrently; the query
     * net needs no rescoring, so it is written while the target fills are
     * rescored (with -nranks: this rank's parts, renamed into place when
     * complete) */
    gt_verbose(1, "writing %s\n", tnet);
    gt_verbose(1, "writing %s\n", qnet);
    net_out wo[2] = {{net, GAC_T, NULL, tnet, &c, 0, 0}, {net, GAC_Q, NULL, qnet, &c, 0, 0}};
    /* GAC_NET_PREFORMAT=1 (measurement knob): the target net's text is
     * formatted while the GPU rescores and the scores inserted afterwards.
     * Off by default: the rescoring takes ~25 ms at C5, and holding the
     * whole preformatted net to insert the scores cost more (1.16 s from the
     * flags to the written net vs ~0.5 s streaming, r03e) */
    const char *pf = getenv("GAC_NET_PREFORMAT");
    if (rescore && pf && *pf == '1') {
        wo[0].pre_started = pthread_create(&wo[0].pre_th, NULL, pre_net, &wo[0]) == 0;
        if (wo[0].pre_started)
            gt_helper_add(wo[0].pre_th);
    }
    pthread_t qth;
    if (pthread_create(&qth, NULL, write_net, &wo[1]) != 0) {
        write_net(&wo[1]);
    } else {
        wo[1].threaded = 1;
        gt_helper_add(qth); /* gt_abort joins it before exiting */
    }

    int64_t *tscores = NULL;
    if (rescore) {
        const int64_t nf = gac_net_fill_count(net, GAC_T);
        /* the partial, printed target fills in pre-order with the window of
         * blocks the netting found for each (the device reads it instead of
         * searching the chain), in one pass over the fills */
        gac_window *r = NULL;
        int64_t *rix = NULL, nr = 0;
        gt_check(gac_net_rescore_windows(net, GAC_T, &r, &rix, &nr));
        gac_mark("fill list: ranges");
        tscores = calloc(nf ? nf : 1, 8);
        /* GAC_DUMP_RANGES=FILE (measurement hook, one process only): the
         * rescored fills as gac_window records (int32 chain index in file
         * order, tStart, tEnd, first block, block count), in submission order
         * -- bench.py replays them in its kernel leg */
        const char *dump = multi ? NULL : getenv("GAC_DUMP_RANGES");
        if (dump && *dump) {
            FILE *df = fopen(dump, "wb");
            if (!df || (nr && fwrite(r, sizeof(gac_window), nr, df) != (size_t)nr) || fclose(df) != 0)
                gt_abort("can't write %s", dump);
        }
        gac_mark("fill list: join upload");
        if (pu.started)
            gt_helper_join(pu.th);
        gac_mark("fill list: joined");
        if (pu.cs && pu.remap) { /* -nranks: the uploaded subset's indices */
            int ok = 1;
            for (int64_t k = 0; k < nr && ok; ++k)
                ok = pu.remap[r[k].chain] >= 0;
            if (ok) {
                for (int64_t k = 0; k < nr; ++k)
                    r[k].chain = pu.remap[r[k].chain];
            } else { /* (cannot happen: every fill's chain is on a kept side) */
                gac_chains_free(pu.cs);
                pu.cs = NULL;
            }
        }
        if (nr && pu.cs) { /* the chain set is on the device */
            gt_stage("fill list");
            gac_ctx *ctx = gt_device_join(&dev);
            gt_stage("device open + 2bit genomes + chains to HBM (rest)");
            int64_t *g = malloc(nr * 8);
            int32_t *ali = malloc(nr * 4);
            gt_check(gac_score_windows(ctx, pu.cs, r, nr, 0, g, NULL, ali));
            gt_stage("GPU fill rescoring");
            for (int64_t k = 0; k < nr; ++k)
                tscores[rix[k]] = g[k];
            gac_mark("scores placed");
            gt_free_late(g, (size_t)nr * 8);
            gt_free_late(ali, (size_t)nr * 4);
            gt_device_close_async(&dev, ctx, pu.cs); /* overlaps writing the nets */
            gac_mark("device close queued");
            pu.cs = NULL;
        } else if (nr) {
            if (pu.cs) {
                gac_chains_free(pu.cs);
                pu.cs = NULL;
            }
            gt_stage("fill list");
            gac_ctx *ctx = gt_device_join(&dev);
            gt_stage("device open + 2bit genomes (rest)");
            /* upload only the chains owning a rescored fill (their sequences
             * must be in the 2bit files; others are never looked up) */
            int32_t *remap = malloc(c.n * 4);
            for (int64_t i = 0; i < c.n; ++i)
                remap[i] = -1;
            int64_t nsub = 0, nbsub = 0;
            for (int64_t k = 0; k < nr; ++k)
                if (remap[r[k].chain] < 0) {
                    remap[r[k].chain] = (int32_t)nsub++;
                    nbsub += c.blk_off[r[k].chain + 1] - c.blk_off[r[k].chain];
                }
            int32_t *gts = malloc(nsub * 4), *gqs = malloc(nsub * 4);
            uint8_t *gst = malloc(nsub);
            int64_t *goff = malloc((nsub + 1) * 8);
            int32_t *gbt = malloc((nbsub ? nbsub : 1) * 4), *gbq = malloc((nbsub ? nbsub : 1) * 4),
                    *gbs = malloc((nbsub ? nbsub : 1) * 4);
            int64_t *src = malloc(nsub * 8);
            for (int64_t i = 0; i < c.n; ++i)
                if (remap[i] >= 0)
                    src[remap[i]] = i;
            goff[0] = 0;
            int32_t *tmap = gt_seq_map(ctx, GAC_T, &c.tnames), *qmap = gt_seq_map(ctx, GAC_Q, &c.qnames);
            for (int64_t j = 0; j < nsub; ++j) {
                const int64_t i = src[j];
                const char *tn = c.tnames.names[c.tname[i]], *qn = c.qnames.names[c.qname[i]];
                gts[j] = tmap[c.tname[i]];
                if (gts[j] < 0)
                    gt_abort("%s is not in %s", tn, tnib);
                gqs[j] = qmap[c.qname[i]];
                if (gqs[j] < 0)
                    gt_abort("%s is not in %s", qn, qnib);
                gst[j] = c.qstrand[i];
                goff[j + 1] = goff[j] + (c.blk_off[i + 1] - c.blk_off[i]);
            }
            free(tmap);
            free(qmap);
            subset_copy sj = {&c, src, goff, gbt, gbq, gbs, nsub, 0};
            atomic_init(&sj.next, 0);
            gac_run_threads(gt_threads(), subset_copy_thread, &sj);
            for (int64_t k = 0; k < nr; ++k)
                r[k].chain = remap[r[k].chain];
            gac_chainset_desc d = {nsub, gts, gqs, gst, goff, nbsub, gbt, gbq, gbs};
            gac_chainset *cs = NULL;
            gt_check(gac_chains_upload(ctx, &d, &cs));
            gt_stage("chains to HBM");
            int64_t *g = malloc(nr * 8);
            int32_t *ali = malloc(nr * 4);
            gt_check(gac_score_windows(ctx, cs, r, nr, 0, g, NULL, ali));
            gt_stage("GPU fill rescoring");
            for (int64_t k = 0; k < nr; ++k)
                tscores[rix[k]] = g[k];
            free(g);
            free(ali);
            free(gts);
            free(gqs);
            free(gst);
            free(goff);
            free(gbt);
            free(gbq);
            free(gbs);
            free(src);
            free(remap);
            gt_device_close_async(&dev, ctx, cs); /* overlaps writing the nets */
        }
        if (!nr) { /* nothing to rescore: the genomes were never needed */
            if (pu.cs)
                gac_chains_free(pu.cs);
            gac_ctx *ctx = gt_device_wait(&dev);
            if (ctx)
                gac_close(ctx);
        }
        /* (13 M-entry arrays: unmapping them here cost the target net's
         * start tens of ms; their pages go after the nets are written) */
        const size_t nrb = (size_t)(nr ? nr : 1);
        gt_free_late(r, nrb * sizeof(gac_window));
        gt_free_late(rix, nrb * 8);
        gac_mark("fill arrays released");
        /* the block coordinates are read by nothing after the rescoring */
        if (!multi)
            gt_chains_drop_blocks_async(&c);
    }
    wo[0].tscores = tscores;
    write_net(&wo[0]);
    gac_mark("target net written");
    if (wo[1].threaded)
        gt_helper_join(qth);
    gac_mark("query net joined");
    for (int k = 0; k < 2; ++k)
        if (wo[k].rc != GAC_OK)
            gt_abort("%s\n", wo[k].err);
    gt_stage("write nets");
    if (multi && g_rk.me == 0) {
        gt_ranks_finish(&g_rk, tnet);
        gt_ranks_finish(&g_rk, qnet);
        gt_stage("wait for ranks");
    }
    gt_device_close_join(&dev);
    gt_stage("device close (rest)");
    gac_gapcalc_free(gap);
    gt_ranks_done(&g_rk);
    /* The net's pools are unmapped on 8 threads: left to process teardown
     * they are freed on one core after the output is complete. */
    gac_net_free(net);
    gt_chains_drop_pages(&c);
    gt_free_late_all();
    gt_stage("free nets and chains");
    gt_exit_ok();
}
