/* axtChain -- drop-in for kent/src/hg/mouseStuff/axtChain/axtChain.c: chain
 * together axt (or -psl) alignments.
 *
 * Same command line (kent optionHash: any option is accepted), same output
 * text.  Input parsing, seqPair grouping and output follow the reference
 * (readPslBlocks :345-377, readAxtBlocks :311-343, axtChain :379-470):
 *   - pairs keyed by qName + strand + tName; PSL pairs stay in reverse
 *     first-seen order (slAddHead), axt pairs are sorted by seqPairCmp;
 *   - blocks of a pair in input order (slAddHead per block, then
 *     slReverse);
 *   - output: the ##matrix / ##gapPenalties / ##blastzParms header
 *     (axtScoreSchemeDnaWrite, axt.c:836-872), the input's '#' lines
 *     (unique), then the chains in chainCmpScore order with ids 1..n.
 * The chaining itself -- removeExactOverlaps, block scores, chainBlocks'
 * kd-tree DP, overlap removal, chainCalcScore, the minScore filter and the
 * final sort -- is one libgachain call, gac_axt_chain (GPU block and chain
 * scoring, host-threaded DP).  Genomes must be .2bit files (-faQ/-faT fasta
 * inputs are read and uploaded as sequences). */
#define _GNU_SOURCE
#include <ctype.h>
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdatomic.h>
#include <time.h>
#include <unistd.h>

#include "gac_tool.h"
#include "gachain.h"
#include "host/gac_host.h"

static void usage(int min_score) {
    gt_abort(
        "axtChain - Chain together axt alignments.\n"
        "usage:\n"
        "   axtChain [options] -linearGap=loose in.axt tNibDir qNibDir out.chain\n"
        "Where tNibDir/qNibDir are either directories full of nib files, the name\n"
        "of a .2bit file, or a single fasta file with additional -faQ or -faT options.\n"
        "options:\n"
        "   -psl Use psl instead of axt format for input\n"
        "   -faQ The specified qNibDir is a fasta file with multiple sequences for query\n"
        "   -faT The specified tNibDir is a fasta file with multiple sequences for target\n"
        "                NOTE: will not work with gzipped fasta files\n"
        "   -minScore=N  Minimum score for chain, default %d\n"
        "   -details=fileName Output some additional chain details\n"
        "   -scoreScheme=fileName Read the scoring matrix from a blastz-format file\n"
        "   -linearGap=<medium|loose|filename> Specify type of linearGap to use.\n"
        "              *Must* specify this argument to one of these choices.\n"
        "              loose is chicken/human linear gap costs.\n"
        "              medium is mouse/human linear gap costs.\n"
        "              Or specify a piecewise linearGap tab delimited file.\n"
        "   (this build reads .2bit genomes, or fasta with -faQ/-faT; not nib directories)\n"
        "batch (this build): axtChain -jobs=FILE runs every line of FILE as one axtChain\n"
        "   command line (arguments only) in one process and one GPU context\n"
        "multi-GPU (this build): -nranks=N -rank=R [-gpu=D], one process per GPU on one node\n"
        "   (GAC_RANK_TOKEN shared by the ranks): seqPairs dealt out by block count, rank 0\n"
        "   merges every rank's chains and writes the file\n",
        min_score);
}

/* ------------------------------------------------------------ kent lineFile */
typedef struct rd {
    char *buf, *cur, *end;
    const char *path;
    int line;
    FILE *meta;       /* lineFileSetMetaDataOutput */
    gt_names seen;    /* lineFileSetUniqueMetaData */
    char *last;       /* last line returned (for lineFileReuse) */
    int reuse;
} rd;

static void rd_open(rd *r, const char *path, FILE *meta) {
    memset(r, 0, sizeof(*r));
    size_t len;
    r->buf = gt_slurp(path, &len);
    r->cur = r->buf;
    r->end = r->buf + len;
    r->path = path;
    r->meta = meta;
}

static void rd_meta(rd *r, const char *line) {
    if (!r->meta || line[0] != '#')
        return;
    if (gt_names_find(&r->seen, line) >= 0)
        return;
    gt_names_add(&r->seen, line, strlen(line));
    fprintf(r->meta, "%s\n", line);
}

/* lineFileNext */
static char *rd_next(rd *r) {
    if (r->reuse) {
        r->reuse = 0;
        rd_meta(r, r->last);
        return r->last;
    }
    if (r->cur >= r->end)
        return NULL;
    char *line = r->cur;
    char *nl = memchr(line, '\n', (size_t)(r->end - line));
    if (nl) {
        *nl = 0;
        r->cur = nl + 1;
    } else {
        r->cur = r->end;
    }
    ++r->line;
    r->last = line;
    rd_meta(r, line);
    return line;
}

/* kent chopByWhite into at most max words (modifies s) */
static int chop(char *s, char **w, int max) {
    return gac_chop_white(s, w, max);
}

/* ------------------------------------------------------------ seqPairs */
typedef struct pair {
    char *qname, *tname;
    char strand;
    int64_t nb, cap;
    int64_t deferred; /* of nb, the blocks still in PSL chunk runs (pairs.defer) */
    int32_t *bt, *bq, *bs;
} pair;

typedef struct merge_task {
    int32_t g;                 /* the global pair */
    int64_t off, nb;           /* where a chunk's run goes among the pair's blocks */
    int32_t *bt, *bq, *bs;     /* the run (the chunk's arrays) */
    char *qname, *tname;       /* the chunk pair's names, freed with the run */
} merge_task;

typedef struct pairs {
    gt_names keys;   /* "qName<strand>tName" -> index (hashAddSaveName) */
    pair *p;
    int32_t n, cap;
    /* PSL input: each pair's blocks past its own arrays stay as chunk runs
     * until they are copied once, straight into the chaining input */
    merge_task *defer;
    int64_t ndefer;
} pairs;

static pair *pair_get(pairs *P, const char *qname, const char *strand, const char *tname) {
    char key[4096];
    snprintf(key, sizeof(key), "%s%s%s", qname, strand, tname);
    int32_t i = gt_names_find(&P->keys, key);
    if (i < 0) {
        i = gt_names_add(&P->keys, key, strlen(key));
        if (P->n == P->cap) {
            P->cap = P->cap ? P->cap * 2 : 64;
            P->p = realloc(P->p, (size_t)P->cap * sizeof(pair));
        }
        pair *p = &P->p[P->n++];
        memset(p, 0, sizeof(*p));
        p->qname = strdup(qname);
        p->tname = strdup(tname);
        p->strand = strand[0];
    }
    return &P->p[i];
}

static void pair_add(pair *p, int32_t t, int32_t q, int32_t size) {
    if (p->nb == p->cap) {
        p->cap = p->cap ? p->cap * 2 : 256;
        p->bt = realloc(p->bt, (size_t)p->cap * 4);
        p->bq = realloc(p->bq, (size_t)p->cap * 4);
        p->bs = realloc(p->bs, (size_t)p->cap * 4);
    }
    p->bt[p->nb] = t;
    p->bq[p->nb] = q;
    p->bs[p->nb] = size;
    ++p->nb;
}

/* sqlUnsigned without aborting: 0 = ok */
/* sqlUnsignedOrError (kent/src/lib/sqlNum.c:14-46): digits to the end,
 * accumulated in unsigned arithmetic (wrapping as the reference does) */
static int sql_unsigned_ok(const char *s, unsigned *v, char *err) {
    unsigned res = 0;
    const char *p = s;
    while (*p >= '0' && *p <= '9')
        res = res * 10u + (unsigned)(*p++ - '0');
    if (*p != 0 || p == s) {
        snprintf(err, 600, "invalid unsigned integer: \"%.400s\"", s);
        return -1;
    }
    *v = res;
    return 0;
}

/* sqlUnsignedDynamicArray into a reusable buffer: 0 = ok */
static int sql_uarray_ok(char *s, int32_t **a, int *cap, int *count, char *err) {
    int n = 0;
    while (*s) { /* (sqlUnsignedInList per item, kent/src/lib/sqlNum.c:56-85) */
        unsigned res = 0;
        char *q = s;
        while (*q >= '0' && *q <= '9')
            res = res * 10u + (unsigned)(*q++ - '0');
        if ((*q != ',' && *q != 0) || q == s) {
            char *c = strchr(s, ',');
            if (c)
                *c = 0;
            snprintf(err, 600, "invalid unsigned integer: \"%.400s\"", s);
            return -1;
        }
        if (n == *cap) {
            *cap = *cap ? *cap * 2 : 64;
            *a = realloc(*a, (size_t)*cap * sizeof(int32_t));
        }
        (*a)[n++] = (int32_t)res;
        if (*q == 0)
            break;
        s = q + 1;
    }
    *count = n;
    return 0;
}

/* One pslLoad line (psl.c pslLoad + readPslBlocks :345-377) into P.
 * 0 = ok; else the reference's error: PSL_E_WORDS (word count in *wc_out),
 * PSL_E_COUNT (block count mismatch) -- both name the file line, which the
 * caller knows -- or PSL_E_MSG with the whole message in err. */
enum { PSL_E_WORDS = 1, PSL_E_COUNT = 2, PSL_E_MSG = 3 };

static void psl_error(int kind, int wc, const char *msg, int64_t lineno, const char *path) {
    if (kind == PSL_E_WORDS)
        gt_abort("Bad line %lld of %s wordCount is %d instead of 21 or 23\n", (long long)lineno,
                 path, wc);
    if (kind == PSL_E_COUNT)
        gt_abort("Assertion `sizeOne == ret->blockCount' failed (line %lld of %s)",
                 (long long)lineno, path);
    gt_abort("%s", msg);
}

static int psl_line(char *line, pairs *P, char *err, int *wc_out) {
    static __thread int32_t *sz, *qs, *ts;
    static __thread int csz, cqs, cts;
    char *w[32];
    const int wc = chop(line, w, 32);
    if (wc != 21 && wc != 23) {
        *wc_out = wc;
        return PSL_E_WORDS;
    }
    unsigned block_count, v;
    if (sql_unsigned_ok(w[17], &block_count, err) != 0)
        return PSL_E_MSG;
    for (int i = 0; i < 8; ++i)
        if (sql_unsigned_ok(w[i][0] == '-' ? w[i] + 1 : w[i], &v, err) != 0)
            return PSL_E_MSG;
    const char *strand = w[8];
    if (sql_unsigned_ok(w[10], &v, err) != 0 || sql_unsigned_ok(w[14], &v, err) != 0)
        return PSL_E_MSG;
    int n1, n2, n3;
    if (sql_uarray_ok(w[18], &sz, &csz, &n1, err) != 0 || sql_uarray_ok(w[19], &qs, &cqs, &n2, err) != 0 ||
        sql_uarray_ok(w[20], &ts, &cts, &n3, err) != 0)
        return PSL_E_MSG;
    if ((unsigned)n1 != block_count || (unsigned)n2 != block_count || (unsigned)n3 != block_count)
        return PSL_E_COUNT;
    if (strand[1] != '\0') {
        snprintf(err, 600, "requires PSLs to have implicit positive strand, found `%.400s'", strand);
        return PSL_E_MSG;
    }
    /* (consecutive records mostly share their pair: the last one is kept,
     * by index, and its names compared before any key is built) */
    static __thread const pairs *last_P;
    static __thread int32_t last_i = -1;
    pair *p;
    if (last_P == P && last_i >= 0 && last_i < P->n && P->p[last_i].strand == strand[0] &&
        strcmp(P->p[last_i].qname, w[9]) == 0 && strcmp(P->p[last_i].tname, w[13]) == 0) {
        p = &P->p[last_i];
    } else {
        p = pair_get(P, w[9], strand, w[13]);
        last_P = P;
        last_i = (int32_t)(p - P->p);
    }
    for (unsigned i = 0; i < block_count; ++i)
        pair_add(p, ts[i], qs[i], sz[i]);
    return 0;
}

/* A line-aligned piece of the PSL body, parsed on its own thread into local
 * seqPairs (first-seen order, blocks in file order), its '#' lines and its
 * first error; the pieces are merged in file order, so pair order, block
 * order, metadata output and the reported error match a sequential read. */
typedef struct psl_chunk {
    char *a, *b;
    const char *path;
    int64_t lines; /* newlines parsed (up to the error) */
    pairs P;
    char **meta;
    int32_t n_meta, meta_cap;
    int err, err_wc;  /* PSL_E_* of the first bad line, its word count */
    int64_t err_line; /* within the chunk, 1-based */
    char msg[600];
} psl_chunk;

typedef struct psl_job {
    psl_chunk *k;
    int nk;
    _Atomic int next;
} psl_job;

static void *psl_chunk_thread(void *arg) {
    psl_job *J = arg;
    for (;;) {
        const int i = atomic_fetch_add(&J->next, 1);
        if (i >= J->nk)
            break;
        psl_chunk *k = &J->k[i];
        for (char *p = k->a; p < k->b;) {
            char *nl = memchr(p, '\n', (size_t)(k->b - p));
            char *line = p;
            if (nl) {
                *nl = 0;
                p = nl + 1;
            } else {
                p = k->b;
            }
            ++k->lines;
            if (line[0] == '#') { /* lineFileSetUniqueMetaData: in order, de-duplicated later */
                if (k->n_meta == k->meta_cap) {
                    k->meta_cap = k->meta_cap ? 2 * k->meta_cap : 16;
                    k->meta = realloc(k->meta, (size_t)k->meta_cap * sizeof(char *));
                }
                k->meta[k->n_meta++] = line;
            }
            const char *s = line; /* lineFileNextReal */
            while (isspace((unsigned char)*s))
                ++s;
            if (*s == 0 || *s == '#')
                continue;
            const int e = psl_line(line, &k->P, k->msg, &k->err_wc);
            if (e) {
                k->err = e;
                k->err_line = k->lines;
                break;
            }
        }
    }
    return NULL;
}

static double wall(void);

/* the chaining input's block columns filled from the pairs: each deferred
 * chunk run copied once, on all threads, to its pair's slice (pairs not on
 * this rank only freed) */
typedef struct merge_job {
    const merge_task *t;
    int64_t n;
    const int32_t *pos;   /* global pair -> its index in the input, or -1 */
    const int64_t *moff;  /* input index -> first block */
    int32_t *bt, *bq, *bs;
    int release; /* free the runs as they are copied (batch jobs; a single
                  * run leaves them to process exit, as its other arrays) */
    _Atomic int64_t next;
} merge_job;

static void *merge_thread(void *arg) {
    merge_job *M = arg;
    for (int64_t i; (i = atomic_fetch_add(&M->next, 1)) < M->n;) {
        const merge_task *t = &M->t[i];
        const int32_t k = M->pos[t->g];
        if (k >= 0) {
            const int64_t o = M->moff[k] + t->off;
            memcpy(M->bt + o, t->bt, (size_t)t->nb * 4);
            memcpy(M->bq + o, t->bq, (size_t)t->nb * 4);
            memcpy(M->bs + o, t->bs, (size_t)t->nb * 4);
        }
        if (!M->release)
            continue;
        free(t->bt);
        free(t->bq);
        free(t->bs);
        free(t->qname);
        free(t->tname);
    }
    return NULL;
}

static void read_psl_chunks(rd *r, pairs *P) {
    char *a = r->cur, *end = r->end;
    const size_t len = (size_t)(end - a);
    int nk = len < (4u << 20) ? 1 : gt_threads() * 4;
    psl_chunk *K = calloc((size_t)nk, sizeof(psl_chunk));
    int n = 0;
    char *prev = a;
    for (int i = 1; i <= nk && prev < end; ++i) {
        char *cut = i == nk ? end : a + len / nk * i;
        if (cut < prev)
            cut = prev;
        if (cut < end) {
            char *nl = memchr(cut, '\n', (size_t)(end - cut));
            cut = nl ? nl + 1 : end;
        }
        if (cut > prev) {
            K[n].a = prev;
            K[n].b = cut;
            K[n].path = r->path;
            ++n;
            prev = cut;
        }
    }
    psl_job J = {K, n, 0};
    atomic_init(&J.next, 0);
    const double tp = wall();
    gac_run_threads(gt_threads() < n ? gt_threads() : (n ? n : 1), psl_chunk_thread, &J);
    const double tpe = wall();
    gt_verbose(2, "[read_psl] %d chunks parsed in %.3f s\n", n, tpe - tp);
    /* merge in file order: the metadata and the first error as a sequential
     * read meets them; every chunk's pairs placed at their offsets in the
     * global pairs (serial: pair order is first-seen order); the block runs
     * stay where the parse left them (copied once, into the chaining input) */
    int64_t line0 = r->line, ntask = 0;
    for (int i = 0; i < n; ++i) {
        psl_chunk *k = &K[i];
        for (int32_t m = 0; m < k->n_meta; ++m)
            rd_meta(r, k->meta[m]);
        if (k->err)
            psl_error(k->err, k->err_wc, k->msg, line0 + k->err_line, r->path);
        line0 += k->lines;
        ntask += k->P.n;
    }
    r->line = (int)line0;
    merge_task *T = realloc(P->defer, (size_t)(P->ndefer + ntask + 1) * sizeof(merge_task));
    int64_t nt = P->ndefer;
    for (int i = 0; i < n; ++i) {
        psl_chunk *k = &K[i];
        for (int32_t j = 0; j < k->P.n; ++j) {
            pair *lp = &k->P.p[j];
            const char strand[2] = {lp->strand, 0};
            pair *gp = pair_get(P, lp->qname, strand, lp->tname);
            T[nt++] = (merge_task){(int32_t)(gp - P->p), gp->nb, lp->nb, lp->bt, lp->bq, lp->bs,
                                   lp->qname, lp->tname};
            gp->nb += lp->nb;
            gp->deferred += lp->nb;
        }
    }
    P->defer = T;
    P->ndefer = nt;
    gt_verbose(2, "[read_psl] %lld chunk pairs placed %.3f s after the parse\n", (long long)ntask,
               wall() - tpe);
    for (int i = 0; i < n; ++i) {
        psl_chunk *k = &K[i];
        free(k->P.p);
        gt_names_free(&k->P.keys);
        free(k->meta);
    }
    free(K);
}

static void *free_text(void *p) {
    free(p);
    return NULL;
}

/* readPslBlocks (:345-377) with pslxFileOpenWithUniqueMeta (psl.c:547-612) */
static void read_psl(const char *path, pairs *P, FILE *out) {
    rd r;
    const double t0 = wall();
    rd_open(&r, path, out);
    gt_verbose(2, "[read_psl] file in memory after %.3f s\n", wall() - t0);
    char *line = rd_next(&r);
    if (!line) {
        fprintf(stderr, "%s is empty\n", path);
    } else if (strncmp(line, "psLayout version", 16) == 0) {
        char *copy = strdup(line), *w[32];
        const int wc = chop(copy, w, 32);
        if (wc < 3)
            gt_abort("%s is not a psLayout file", path);
        if (strcmp(w[2], "3") != 0 && strcmp(w[2], "4") != 0)
            gt_abort("%s is version %s of psLayout, this program can only handle through version 4",
                     path, w[2]);
        free(copy);
        for (int i = 0; i < 4; ++i)
            if (!rd_next(&r))
                gt_abort("%s severely truncated", path);
    } else {
        int eof = 0;
        while (line[0] == '#' && !eof) {
            char *nx = rd_next(&r);
            if (!nx)
                eof = 1;
            else
                line = nx;
        }
        char *copy = strdup(line), *w[32];
        const int wc = chop(copy, w, 32);
        if ((wc < 21 || wc > 23 || (w[8][0] != '+' && w[8][0] != '-')) && !eof)
            gt_abort("%s is not a psLayout file", path);
        else if (!eof)
            r.reuse = 1;
        free(copy);
    }
    /* the first data line was read for the format check: parse it here,
     * then the rest of the file in parallel chunks */
    char err[600];
    int wc = 0;
    if (r.reuse) {
        r.reuse = 0;
        const int e = psl_line(r.last, P, err, &wc);
        if (e)
            psl_error(e, wc, err, r.line, path);
    }
    read_psl_chunks(&r, P);
    gt_names_free(&r.seen);
    /* the text (GBs at C4) is released off the caller's path: unmapping 2.6 GB
     * takes a core ~0.3 s */
    pthread_t th;
    pthread_attr_t at;
    pthread_attr_init(&at);
    pthread_attr_setdetachstate(&at, PTHREAD_CREATE_DETACHED);
    if (pthread_create(&th, &at, free_text, r.buf) != 0)
        free(r.buf);
    pthread_attr_destroy(&at);
}

static int need_num(rd *r, char **w, int i) {
    char *end;
    const char *s = w[i];
    long v = strtol(s, &end, 10);
    if (*s == 0 || *end != 0 || !(isdigit((unsigned char)s[0]) || s[0] == '-'))
        gt_abort("Expecting number field %d line %d of %s, got %s", i + 1, r->line, r->path, s);
    return (int)v;
}

/* readAxtBlocks (:311-343): axtRead (axt.c:52-92) + axtAddBlocksToBoxInList
 * (axt.c:929-970) */
static void read_axt(const char *path, pairs *P, FILE *out) {
    rd r;
    rd_open(&r, path, out);
    for (;;) {
        char *w[10];
        int wc = 0;
        char *line;
        while ((line = rd_next(&r)) != NULL) { /* lineFileChopNext */
            if (line[0] == '#')
                continue;
            wc = chop(line, w, 10);
            if (wc != 0)
                break;
        }
        if (!line || wc <= 0)
            break;
        if (wc < 8)
            gt_abort("Expecting at least 8 words line %d of %s got %d\n", r.line, path, wc);
        const int qstart = need_num(&r, w, 5) - 1, qend = need_num(&r, w, 6);
        const int tstart = need_num(&r, w, 2) - 1, tend = need_num(&r, w, 3);
        (void)qend;
        (void)tend;
        if (wc > 8)
            (void)need_num(&r, w, 8);
        char strand[2] = {w[7][0], 0};
        char *qname = w[4], *tname = w[1];
        char *tsym = rd_next(&r);
        if (!tsym)
            gt_abort("Premature end of file in %s", path);
        char *qsym = rd_next(&r);
        if (!qsym)
            gt_abort("Premature end of file in %s", path);
        const size_t sym = strlen(tsym);
        if (strlen(qsym) != sym)
            gt_abort("Symbol count %d != %d inconsistent between sequences line %d and prev line of %s",
                     (int)sym, (int)strlen(qsym), r.line, path);
        rd_next(&r); /* blank line */
        pair *p = pair_get(P, qname, strand, tname);
        int q_pos = qstart, t_pos = tstart, qs = 0, ts = 0, last_in = 0;
        for (size_t i = 0; i <= sym; ++i) {
            const int aq = isalpha((unsigned char)qsym[i]) ? 1 : 0;
            const int at = isalpha((unsigned char)tsym[i]) ? 1 : 0;
            const int this_in = aq && at;
            if (this_in) {
                if (!last_in) {
                    qs = q_pos;
                    ts = t_pos;
                }
            } else if (last_in) {
                const int size = q_pos - qs;
                if (size > 0)
                    pair_add(p, ts, qs, size);
            }
            last_in = this_in;
            q_pos += aq;
            t_pos += at;
        }
    }
    gt_names_free(&r.seen);
    free(r.buf);
}

/* seqPairCmp (:71-83) */
static int pair_cmp(const void *a, const void *b) {
    const pair *x = *(pair *const *)a, *y = *(pair *const *)b;
    int d = strcmp(x->tname, y->tname);
    if (d == 0)
        d = strcmp(x->qname, y->qname);
    if (d == 0)
        d = (int)x->strand - (int)y->strand;
    return d;
}

/* ------------------------------------------------------------ fasta (-faQ/-faT) */
static void load_fasta(gac_ctx *ctx, int side, const char *path) {
    size_t len;
    char *buf = gt_slurp(path, &len);
    char *p = buf, *end = buf + len;
    int nseq = 0;
    while (p < end) {
        if (*p != '>') {
            char *nl = memchr(p, '\n', (size_t)(end - p));
            p = nl ? nl + 1 : end;
            continue;
        }
        char *nl = memchr(p, '\n', (size_t)(end - p));
        char *hdr_end = nl ? nl : end;
        char *name = p + 1;
        while (name < hdr_end && isspace((unsigned char)*name))
            ++name;
        char *ne = name;
        while (ne < hdr_end && !isspace((unsigned char)*ne))
            ++ne;
        char saved = *ne;
        *ne = 0;
        char *seqname = strdup(name);
        *ne = saved;
        p = nl ? nl + 1 : end;
        /* sequence lines until the next '>' */
        size_t cap = 1 << 16, n = 0;
        uint8_t *codes = malloc(cap);
        while (p < end && *p != '>') {
            const char c = *p++;
            if (isspace((unsigned char)c))
                continue;
            if (n == cap) {
                cap *= 2;
                codes = realloc(codes, cap);
            }
            switch (c) {
            case 't': case 'T': codes[n++] = 0; break;
            case 'c': case 'C': codes[n++] = 1; break;
            case 'a': case 'A': codes[n++] = 2; break;
            case 'g': case 'G': codes[n++] = 3; break;
            default: codes[n++] = 4; break;
            }
        }
        uint8_t *packed = calloc((n + 3) / 4 + 1, 1);
        int32_t *ns = malloc((n + 1) * sizeof(int32_t)), *nz = malloc((n + 1) * sizeof(int32_t));
        int32_t nn = 0;
        for (size_t i = 0; i < n; ++i) {
            const int c = codes[i] == 4 ? 0 : codes[i];
            packed[i >> 2] |= (uint8_t)(c << (6 - 2 * (i & 3)));
            if (codes[i] == 4) {
                if (nn > 0 && (size_t)(ns[nn - 1] + nz[nn - 1]) == i)
                    ++nz[nn - 1];
                else {
                    ns[nn] = (int32_t)i;
                    nz[nn] = 1;
                    ++nn;
                }
            }
        }
        gt_check(gac_genome_add_seq(ctx, side, seqname, (int32_t)n, packed, nn, ns, nz));
        gt_verbose(2, "read %s: %zu bases from %s\n", seqname, n, path);
        free(seqname);
        free(codes);
        free(packed);
        free(ns);
        free(nz);
        ++nseq;
    }
    free(buf);
    gt_check(gac_genome_finalize(ctx, side));
}

static double wall(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ------------------------------------------------------------ main */
/* -jobs=FILE: many chaining jobs in one process (SURVEY §8(f) item 4:
 * RepeatFiller's thousands of small axtChain runs) -- one device context,
 * genomes kept loaded while consecutive jobs name the same files */
typedef struct ax_batch {
    int on;
    gac_ctx *ctx;
    char *tpath, *qpath; /* genomes loaded in ctx */
    int tfa, qfa;
} ax_batch;

static void batch_genomes(ax_batch *B, const char *tnib, const char *qnib, int fa_t, int fa_q) {
    if (B->ctx && B->tpath && B->qpath && strcmp(B->tpath, tnib) == 0 && strcmp(B->qpath, qnib) == 0 &&
        B->tfa == fa_t && B->qfa == fa_q)
        return;
    if (B->ctx) /* other genomes: a fresh context (the runtime stays initialised) */
        gac_close(B->ctx);
    B->ctx = NULL;
    free(B->tpath);
    free(B->qpath);
    B->tpath = B->qpath = NULL;
    gt_check(gac_open(0, &B->ctx));
    if (fa_t) {
        load_fasta(B->ctx, GAC_T, tnib);
    } else {
        if (!gac_is_twobit_file(tnib))
            gt_abort("given tNibDir argument: '%s' is not a 2bit file (nib directories are not supported)\n",
                     tnib);
        gt_check(gac_genome_load_2bit(B->ctx, GAC_T, tnib));
    }
    if (fa_q) {
        load_fasta(B->ctx, GAC_Q, qnib);
    } else {
        if (!gac_is_twobit_file(qnib))
            gt_abort("given qNibDir argument: '%s' is not a 2bit file (nib directories are not supported)\n",
                     qnib);
        gt_check(gac_genome_load_2bit(B->ctx, GAC_Q, qnib));
    }
    B->tpath = strdup(tnib);
    B->qpath = strdup(qnib);
    B->tfa = fa_t;
    B->qfa = fa_q;
}

/* ------------------------------------------------------------ -nranks
 * seqPairs are independent up to the final sort (axtChain.c:379-470:
 * chainPair per pair, then one slSort(chainCmpScore) of the whole list), so
 * rank R chains the pairs the LPT deal gives it -- largest block count first,
 * each to the least loaded rank -- in spList order, and rank 0 merges.  The
 * reference's list is built by slAddHead pair after pair, so its stable sort
 * orders equal scores by pair index descending, then by the pair's own order;
 * every rank's gac_axt_chain output is already sorted that way on its subset
 * of pairs, so a merge by (score descending, global pair descending) that
 * takes equal keys from one rank in that rank's order (one pair lives on one
 * rank) is the reference's order, and ids 1..n follow it (chain.c:203-204). */
typedef struct ax_part {
    int64_t n, nb;
    double *score;
    int32_t *pair, *ts, *te, *qs, *qe;
    int64_t *off;
    int32_t *bt, *bq, *bs;
} ax_part;

/* rank 0's output: chain j of the merged order is chain[j] of part[j],
 * written with id j + 1 (chainWrite order) */
typedef struct ax_out {
    const ax_part *parts;
    int32_t *part;
    int64_t *chain;
    pair *const *ord;
    const uint8_t *strand;
    int32_t *tsize, *qsize; /* per pair */
} ax_out;

static void out_chain(FILE *f, int64_t j, void *arg) {
    const ax_out *O = arg;
    const ax_part *P = &O->parts[O->part[j]];
    const int64_t c = O->chain[j];
    const int32_t p = P->pair[c];
    const int64_t b0 = P->off[c];
    gt_write_chain_raw(f, P->score[c], O->ord[p]->tname, O->tsize[p], P->ts[c], P->te[c],
                       O->ord[p]->qname, O->qsize[p], O->strand[p], P->qs[c], P->qe[c],
                       (int32_t)(j + 1), P->bt + b0, P->bq + b0, P->bs + b0, P->off[c + 1] - b0);
}

static void lpt_deal(const int64_t *boff, int64_t np, int nranks, int32_t *owner) {
    int64_t *ix = malloc((size_t)(np ? np : 1) * 8), *load = calloc((size_t)nranks, 8);
    for (int64_t i = 0; i < np; ++i)
        ix[i] = i;
    /* by block count descending, then pair index (insertion into runs of a
     * merge sort would do; pairs number in the thousands) */
    for (int64_t w = 1; w < np; w *= 2) {
        int64_t *tmp = malloc((size_t)np * 8);
        for (int64_t lo = 0; lo < np; lo += 2 * w) {
            int64_t a = lo, am = lo + w < np ? lo + w : np, b = am, bm = lo + 2 * w < np ? lo + 2 * w : np,
                    k = lo;
            while (a < am && b < bm) {
                const int64_t na = boff[ix[a] + 1] - boff[ix[a]], nb = boff[ix[b] + 1] - boff[ix[b]];
                tmp[k++] = (nb > na) ? ix[b++] : ix[a++];
            }
            while (a < am)
                tmp[k++] = ix[a++];
            while (b < bm)
                tmp[k++] = ix[b++];
        }
        memcpy(ix, tmp, (size_t)np * 8);
        free(tmp);
    }
    for (int64_t k = 0; k < np; ++k) {
        int best = 0;
        for (int r = 1; r < nranks; ++r)
            if (load[r] < load[best])
                best = r;
        owner[ix[k]] = best;
        load[best] += boff[ix[k] + 1] - boff[ix[k]];
    }
    free(ix);
    free(load);
}

static void part_write(const char *path, const gac_axt_chains *ch, const int32_t *gpair) {
    FILE *f = fopen(path, "wb");
    if (!f)
        gt_abort("Can't open %s to write: %s", path, strerror(errno));
    const int64_t n = ch->n_chains, nb = ch->n_blocks;
    int ok = fwrite("GACAXP01", 1, 8, f) == 8 && fwrite(&n, 8, 1, f) == 1 && fwrite(&nb, 8, 1, f) == 1;
    int32_t *gp = malloc((size_t)(n ? n : 1) * 4);
    for (int64_t c = 0; c < n; ++c)
        gp[c] = gpair[ch->pair[c]];
    ok = ok && fwrite(ch->score, 8, (size_t)n, f) == (size_t)n && fwrite(ch->blk_off, 8, (size_t)n + 1, f) == (size_t)n + 1;
    const int32_t *cols[5] = {gp, ch->t_start, ch->t_end, ch->q_start, ch->q_end};
    for (int k = 0; k < 5; ++k)
        ok = ok && fwrite(cols[k], 4, (size_t)n, f) == (size_t)n;
    const int32_t *bcols[3] = {ch->blk_t, ch->blk_q, ch->blk_size};
    for (int k = 0; k < 3; ++k)
        ok = ok && fwrite(bcols[k], 4, (size_t)nb, f) == (size_t)nb;
    free(gp);
    if (fclose(f) != 0 || !ok)
        gt_abort("write error on %s", path);
}

static void part_read(const char *path, ax_part *P) {
    FILE *f = fopen(path, "rb");
    if (!f)
        gt_abort("Can't open %s to read: %s", path, strerror(errno));
    char mg[8];
    if (fread(mg, 1, 8, f) != 8 || memcmp(mg, "GACAXP01", 8) != 0 || fread(&P->n, 8, 1, f) != 1 ||
        fread(&P->nb, 8, 1, f) != 1 || P->n < 0 || P->nb < 0)
        gt_abort("%s: not an axtChain rank part", path);
    const size_t n = (size_t)P->n, nb = (size_t)P->nb;
    P->score = malloc((n ? n : 1) * 8);
    P->off = malloc((n + 1) * 8);
    int32_t **cols[5] = {&P->pair, &P->ts, &P->te, &P->qs, &P->qe};
    int ok = fread(P->score, 8, n, f) == n && fread(P->off, 8, n + 1, f) == n + 1;
    for (int k = 0; k < 5; ++k) {
        *cols[k] = malloc((n ? n : 1) * 4);
        ok = ok && fread(*cols[k], 4, n, f) == n;
    }
    int32_t **bcols[3] = {&P->bt, &P->bq, &P->bs};
    for (int k = 0; k < 3; ++k) {
        *bcols[k] = malloc((nb ? nb : 1) * 4);
        ok = ok && fread(*bcols[k], 4, nb, f) == nb;
    }
    fclose(f);
    if (!ok || P->off[0] != 0 || P->off[n] != P->nb)
        gt_abort("%s: truncated axtChain rank part", path);
}

static void run_job(int argc, char *argv[], ax_batch *B) {
    gt_options_hash(&argc, argv);
    int min_score = gt_opt_int("minScore", 1000);
    const char *details = gt_opt_str("details", NULL);
    const char *gap_name = gt_opt_str("linearGap", NULL);
    const char *scheme = gt_opt_str("scoreScheme", NULL);
    if (argc != 5)
        usage(min_score);
    const char *in = argv[1], *tnib = argv[2], *qnib = argv[3], *out_path = argv[4];
    int32_t mat[16], gap_open = 0, gap_extend = 0;
    char *extra = NULL;
    if (scheme)
        gt_verbose(1, "Reading scoring matrix from %s\n", scheme);
    gt_check(gac_scheme_read(scheme, mat, &gap_open, &gap_extend, &extra));
    if (gap_name == NULL)
        gt_abort("Must specify linear gap costs.  Use 'loose' or 'medium' for defaults\n");
    gac_gapcalc *gap = NULL;
    gt_check(gac_gapcalc_build(gap_name, &gap));
    const int fa_q = gt_opt_exists("faQ"), fa_t = gt_opt_exists("faT");

    gt_ranks rk;
    memset(&rk, 0, sizeof(rk));
    rk.n = 1;
    if (gt_opt_int("nranks", 1) > 1) {
        if (B->on)
            gt_abort("-nranks does not go with -jobs\n");
        if (details)
            gt_abort("-details is not supported with -nranks\n");
        if (!strcmp(out_path, "stdout"))
            gt_abort("-nranks needs an output file name (not stdout)");
        gt_ranks_init(&rk, gt_opt_int("nranks", 1), gt_opt_int("rank", 0), out_path);
    }
    const int multi = rk.n > 1;
    /* ranks > 0 write a binary part; the text (headers, '#' lines, chains)
     * is rank 0's */
    FILE *f = multi && rk.me > 0 ? fopen("/dev/null", "w") : gt_must_open(out_path, "w");
    if (!f)
        gt_abort("Can't open /dev/null");
    /* axtScoreSchemeDnaWrite (axt.c:836-872): matrix in ACGT x ACGT order */
    fprintf(f, "##matrix=axtChain 16");
    for (int i = 0; i < 16; ++i)
        fprintf(f, "%c%d", i ? ',' : ' ', mat[i]);
    fprintf(f, "\n##gapPenalties=axtChain O=%d E=%d\n", gap_open, gap_extend);
    if (extra) {
        char *w = extra;
        for (char *r = extra; *r; ++r)
            if (*r != ' ' && *r != '"')
                *w++ = *r;
        *w = 0;
        fprintf(f, "##blastzParms=%s\n", extra);
    }
    if (details) {
        FILE *d = gt_must_open(details, "w");
        fclose(d);
    }
    /* 2bit genomes: device + genomes come up on a helper thread while the
     * alignments are read (scoring is set later, by gac_axt_chain) */
    gt_device dev;
    memset(&dev, 0, sizeof(dev));
    const int early_dev =
        !B->on && !fa_t && !fa_q && gac_is_twobit_file(tnib) && gac_is_twobit_file(qnib);
    if (early_dev)
        gt_device_start(&dev, tnib, qnib, NULL, NULL);
    double t0 = wall();
    pairs P;
    memset(&P, 0, sizeof(P));
    const int psl = gt_opt_exists("psl");
    if (psl)
        read_psl(in, &P, f);
    else
        read_axt(in, &P, f);
    /* pair order: PSL slAddHead (reverse first-seen); axt also sorted */
    pair **ord = malloc((size_t)(P.n ? P.n : 1) * sizeof(pair *));
    for (int32_t i = 0; i < P.n; ++i)
        ord[i] = &P.p[P.n - 1 - i];
    if (!psl)
        qsort(ord, (size_t)P.n, sizeof(pair *), pair_cmp); /* keys are distinct */

    gt_verbose(2, "read %d pairs from %s in %.3f s\n", P.n, in, wall() - t0);
    t0 = wall();
    gac_ctx *ctx = NULL;
    if (B->on) {
        batch_genomes(B, tnib, qnib, fa_t, fa_q);
        ctx = B->ctx;
    } else if (early_dev) {
        ctx = gt_device_join(&dev);
    } else {
        gt_check(gac_open(0, &ctx));
        if (fa_t) {
            load_fasta(ctx, GAC_T, tnib);
        } else {
            if (!gac_is_twobit_file(tnib))
                gt_abort("given tNibDir argument: '%s' is not a 2bit file (nib directories are not supported)\n",
                         tnib);
            gt_check(gac_genome_load_2bit(ctx, GAC_T, tnib));
        }
        if (fa_q) {
            load_fasta(ctx, GAC_Q, qnib);
        } else {
            if (!gac_is_twobit_file(qnib))
                gt_abort("given qNibDir argument: '%s' is not a 2bit file (nib directories are not supported)\n",
                         qnib);
            gt_check(gac_genome_load_2bit(ctx, GAC_Q, qnib));
        }
    }
    /* sequences in the order the reference loads them (q, then t, per pair) */
    const int64_t np = P.n;
    int32_t *tseq = malloc((size_t)(np ? np : 1) * 4), *qseq = malloc((size_t)(np ? np : 1) * 4);
    uint8_t *strand = malloc((size_t)(np ? np : 1));
    int64_t *boff = malloc((size_t)(np + 1) * 8);
    boff[0] = 0;
    for (int64_t i = 0; i < np; ++i) {
        const pair *p = ord[i];
        qseq[i] = gac_genome_seq_index(ctx, GAC_Q, p->qname);
        if (qseq[i] < 0) {
            if (fa_q)
                gt_abort("ERROR: can not find sequence name '%s' from fasta file '%s'\n", p->qname, qnib);
            gt_abort("%s is not in %s", p->qname, qnib);
        }
        tseq[i] = gac_genome_seq_index(ctx, GAC_T, p->tname);
        if (tseq[i] < 0) {
            if (fa_t)
                gt_abort("ERROR: can not find sequence name '%s' from fasta file '%s'\n", p->tname, tnib);
            gt_abort("%s is not in %s", p->tname, tnib);
        }
        strand[i] = p->strand == '-' ? 1 : 0;
        boff[i + 1] = boff[i] + p->nb;
    }
    /* this rank's pairs (all of them without -nranks), in spList order */
    int32_t *mine = malloc((size_t)(np ? np : 1) * 4);
    int64_t nm = 0;
    if (multi) {
        int32_t *owner = malloc((size_t)(np ? np : 1) * 4);
        lpt_deal(boff, np, rk.n, owner);
        for (int64_t i = 0; i < np; ++i)
            if (owner[i] == rk.me)
                mine[nm++] = (int32_t)i;
        free(owner);
    } else {
        for (int64_t i = 0; i < np; ++i)
            mine[nm++] = (int32_t)i;
    }
    int32_t *mt = malloc((size_t)(nm ? nm : 1) * 4), *mq = malloc((size_t)(nm ? nm : 1) * 4);
    uint8_t *ms = malloc((size_t)(nm ? nm : 1));
    int64_t *moff = malloc((size_t)(nm + 1) * 8);
    moff[0] = 0;
    for (int64_t k = 0; k < nm; ++k) {
        mt[k] = tseq[mine[k]];
        mq[k] = qseq[mine[k]];
        ms[k] = strand[mine[k]];
        moff[k + 1] = moff[k] + ord[mine[k]]->nb;
    }
    const int64_t nb = moff[nm];
    int32_t *bt = malloc((size_t)(nb ? nb : 1) * 4), *bq = malloc((size_t)(nb ? nb : 1) * 4),
            *bs = malloc((size_t)(nb ? nb : 1) * 4);
    {
        /* each pair's own blocks first (all of them from an axt file, the
         * first line's from a PSL), then the PSL chunk runs at their offsets */
        int32_t *pos = malloc((size_t)(np ? np : 1) * 4);
        for (int64_t i = 0; i < np; ++i)
            pos[i] = -1;
        for (int64_t k = 0; k < nm; ++k) {
            const pair *p = ord[mine[k]];
            const int64_t own = p->nb - p->deferred;
            pos[p - P.p] = (int32_t)k;
            memcpy(bt + moff[k], p->bt, (size_t)own * 4);
            memcpy(bq + moff[k], p->bq, (size_t)own * 4);
            memcpy(bs + moff[k], p->bs, (size_t)own * 4);
        }
        merge_job M = {P.defer, P.ndefer, pos, moff, bt, bq, bs, B->on};
        atomic_init(&M.next, 0);
        const double tm = wall();
        const int nth = gt_threads() < M.n ? gt_threads() : (M.n ? (int)M.n : 1);
        gac_run_threads(nth, merge_thread, &M);
        gt_verbose(2, "[input] %lld blocks gathered from %lld chunk runs in %.3f s\n", (long long)nb,
                   (long long)M.n, wall() - tm);
        free(P.defer);
        P.defer = NULL;
        P.ndefer = 0;
        free(pos);
    }
    gt_verbose(2, "device + genomes in %.3f s\n", wall() - t0);
    t0 = wall();
    gac_axt_input ai = {nm, mt, mq, ms, moff, bt, bq, bs};
    gac_axt_chains *ch = NULL;
    gt_check(gac_axt_chain(ctx, mat, gap, &ai, (double)min_score, 0, details, &ch));
    if (multi && getenv("GAC_TIMING")) /* (DESIGN §6's per-rank table) */
        fprintf(stderr, "[rank %d/%d] %lld pairs, %lld blocks, %lld chains: chained in %.3f s\n",
                rk.me, rk.n, (long long)nm, (long long)nb, (long long)ch->n_chains, wall() - t0);
    if (multi && rk.me > 0) { /* this rank's chains, sorted, to rank 0 */
        char part[4096], tmp[4096];
        gt_part_name(part, sizeof(part), out_path, rk.me, "");
        gt_part_name(tmp, sizeof(tmp), out_path, rk.me, ".tmp");
        part_write(tmp, ch, mine);
        if (rename(tmp, part) != 0)
            gt_abort("can't rename %s", tmp);
        fclose(f);
        gt_verbose(2, "rank %d: %lld pairs, %lld blocks, %lld chains in %.3f s\n", rk.me,
                   (long long)nm, (long long)nb, (long long)ch->n_chains, wall() - t0);
        gac_close(ctx);
        gt_ranks_done(&rk);
        gt_exit_ok();
    }
    /* rank 0 (or the only rank): its own chains as part 0, the others' read
     * back, merged into chainWrite order */
    ax_part *parts = calloc((size_t)rk.n, sizeof(ax_part));
    {
        ax_part *P0 = &parts[0];
        P0->n = ch->n_chains;
        P0->nb = ch->n_blocks;
        P0->score = ch->score;
        P0->pair = malloc((size_t)(P0->n ? P0->n : 1) * 4);
        for (int64_t c = 0; c < P0->n; ++c)
            P0->pair[c] = mine[ch->pair[c]];
        P0->ts = ch->t_start, P0->te = ch->t_end, P0->qs = ch->q_start, P0->qe = ch->q_end;
        P0->off = ch->blk_off;
        P0->bt = ch->blk_t, P0->bq = ch->blk_q, P0->bs = ch->blk_size;
    }
    if (multi && !gt_ranks_solo()) {
        gt_ranks_wait(&rk, out_path);
        for (int r = 1; r < rk.n; ++r) {
            char part[4096];
            gt_part_name(part, sizeof(part), out_path, r, "");
            part_read(part, &parts[r]);
            unlink(part);
        }
    }
    /* the merged order first (part, chain), then the text formatted on all
     * threads in runs and written in order (ids = output positions) */
    int64_t n_out = 0;
    for (int r = 0; r < rk.n; ++r)
        n_out += parts[r].n;
    ax_out O = {parts, malloc((size_t)(n_out ? n_out : 1) * 4), malloc((size_t)(n_out ? n_out : 1) * 8),
                ord, strand, NULL, NULL};
    O.tsize = malloc((size_t)(np ? np : 1) * 4);
    O.qsize = malloc((size_t)(np ? np : 1) * 4);
    for (int64_t p = 0; p < np; ++p) {
        O.tsize[p] = gac_genome_seq_size(ctx, GAC_T, tseq[p]);
        O.qsize[p] = gac_genome_seq_size(ctx, GAC_Q, qseq[p]);
    }
    int64_t *head = calloc((size_t)rk.n, 8);
    for (int64_t j = 0;; ++j) {
        int best = -1;
        for (int r = 0; r < rk.n; ++r) {
            if (head[r] >= parts[r].n)
                continue;
            if (best < 0) {
                best = r;
                continue;
            }
            const double a = parts[r].score[head[r]], b = parts[best].score[head[best]];
            if (a > b || (a == b && parts[r].pair[head[r]] > parts[best].pair[head[best]]))
                best = r;
        }
        if (best < 0)
            break;
        O.part[j] = best;
        O.chain[j] = head[best]++;
    }
    free(head);
    fflush(f);
    gt_par_write(f, n_out, out_chain, &O);
    free(O.part);
    free(O.chain);
    free(O.tsize);
    free(O.qsize);
    gt_careful_close(f, out_path);
    gt_ranks_done(&rk);
    gt_verbose(2, "chaining + writing in %.3f s\n", wall() - t0);
    gt_verbose(2, "%lld pairs, %lld blocks, %lld chains\n", (long long)np, (long long)nb,
               (long long)ch->n_chains);
    if (!B->on) {
        gac_close(ctx); /* host arrays are left to process exit */
        gt_exit_ok();
    }
    /* batch: this job's arrays go now */
    gac_axt_chains_free(ch);
    for (int32_t i = 0; i < P.n; ++i) {
        free(P.p[i].bt);
        free(P.p[i].bq);
        free(P.p[i].bs);
        free(P.p[i].qname);
        free(P.p[i].tname);
    }
    free(P.p);
    gt_names_free(&P.keys);
    free(ord);
    free(tseq);
    free(qseq);
    free(strand);
    free(boff);
    free(mine);
    free(mt);
    free(mq);
    free(ms);
    free(moff);
    free(parts[0].pair);
    free(parts);
    free(bt);
    free(bq);
    free(bs);
    gac_gapcalc_free(gap);
    free(extra);
}

int main(int argc, char *argv[]) {
    const char *jobs = NULL;
    for (int i = 1; i < argc; ++i)
        if (strncmp(argv[i], "-jobs=", 6) == 0)
            jobs = argv[i] + 6;
    ax_batch B;
    memset(&B, 0, sizeof(B));
    /* the device: -gpu=D, else the rank with -nranks, else 0 -- exposed alone
     * to the runtime before any thread or HIP call */
    int gpu = -1, rank = 0, nranks = 1;
    for (int i = 1; i < argc; ++i) {
        if (!strncmp(argv[i], "-gpu=", 5))
            gpu = atoi(argv[i] + 5);
        else if (!strncmp(argv[i], "-rank=", 6))
            rank = atoi(argv[i] + 6);
        else if (!strncmp(argv[i], "-nranks=", 8))
            nranks = atoi(argv[i] + 8);
    }
    gt_set_gpu(gpu >= 0 ? gpu : (nranks > 1 ? rank : 0));
    gt_one_device();
    if (nranks > 1 && !getenv("GAC_DP_DOMAIN_BASE")) { /* ranks' DP teams in L3 domains of their own */
        char b[16];
        snprintf(b, sizeof(b), "%d", 2 * rank);
        setenv("GAC_DP_DOMAIN_BASE", b, 0);
    }
    if (!jobs) {
        run_job(argc, argv, &B); /* exits */
        return 0;
    }
    /* one job per line: the arguments of one axtChain run (whitespace
     * separated, no quoting); blank and '#' lines are skipped; the first
     * failing job stops the batch with that job's error and exit status */
    gt_options_hash(&argc, argv);
    if (argc != 1)
        gt_abort("axtChain -jobs=FILE takes no other arguments (put them in FILE, one run per line)\n");
    B.on = 1;
    size_t len;
    char *text = gt_slurp(jobs, &len);
    int64_t njobs = 0;
    for (char *line = text, *nl; line && *line; line = nl ? nl + 1 : NULL) {
        nl = strchr(line, '\n');
        if (nl)
            *nl = 0;
        char *w[256];
        const int wc = gac_chop_white(line, w, 255);
        if (wc == 0 || w[0][0] == '#')
            continue;
        char *jargv[257];
        jargv[0] = argv[0];
        for (int i = 0; i < wc; ++i)
            jargv[i + 1] = w[i];
        jargv[wc + 1] = NULL;
        gt_options_reset();
        run_job(wc + 1, jargv, &B);
        ++njobs;
    }
    gt_verbose(2, "%lld jobs in one device context\n", (long long)njobs);
    if (B.ctx)
        gac_close(B.ctx);
    gt_exit_ok();
}
