/* chainMergeSort -- combine score-sorted chain files into one sorted stream
 * (drop-in for kent/src/hg/mouseStuff/chainMergeSort/chainMergeSort.c).
 *
 * Same command line and standard-output bytes as the reference:
 *   - each input is read with chainRead (kent/src/lib/chain.c:256-346), its
 *     '#' lines echoed to the output at the moment the reference's line file
 *     would read them (lineFileSetMetaDataOutput, linefile.c:66-104: the
 *     lines consumed while reading a file's k-th chain, or its end);
 *   - the merge is the reference's quickHeap (kent/src/lib/quickHeap.c)
 *     keyed by cmpChainScores (chainMergeSort.c:71-87), replayed exactly --
 *     including the order in which equal scores leave the heap;
 *   - ids are renumbered 1..n unless -saveId (:107-108);
 *   - more than 400 files, or -inputList, go through hierSort (:127-197):
 *     groups of 400 inputs merged into intermediate streams, level by level;
 *     an intermediate stream holds what the reference writes to its temp
 *     files (scores as printed by %1.0f and re-read, ids as written, '#'
 *     lines), so ties resolve as they do there.
 * The inputs are parsed on all threads (gt_read_chains) instead of streamed;
 * the merge order is computed first and the text formatted in parallel. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gac_tool.h"

#define MAXFILES 400 /* chainMergeSort.c:16 */

static const gt_spec k_opts[] = {
    {"saveId", GT_BOOL},
    {"inputList", GT_STRING},
    {"tempDir", GT_STRING},
    {NULL, 0},
};

static void usage(void) {
    gt_abort("chainMergeSort - Combine sorted files into larger sorted file\n"
             "usage:\n"
             "   chainMergeSort file(s)\n"
             "Output goes to standard output\n"
             "options:\n"
             "   -saveId - keep the existing chain ids.\n"
             "   -inputList=somefile - somefile contains list of input chain files.\n"
             "   -tempDir=somedir/ - somedir has space for temporary sorting data, default ./\n");
}

/* A stream item: a chain (file, index; score and id as this stream holds
 * them) or a '#' line. */
typedef struct item {
    const char *meta; /* non-NULL: a '#' line */
    int32_t file;
    int64_t idx;
    double score;
    int32_t id;
} item;

typedef struct stream {
    item *it;
    int64_t n, cap;
} stream;

static void push(stream *s, item x) {
    if (s->n == s->cap) {
        s->cap = s->cap ? s->cap * 2 : 1024;
        s->it = realloc(s->it, (size_t)s->cap * sizeof(item));
    }
    s->it[s->n++] = x;
}

/* a cursor over a stream: chainRead consumes '#' items up to the next chain */
typedef struct cursor {
    const stream *s;
    int64_t pos;
    const item *chain; /* current chain, NULL at EOF */
} cursor;

static void cursor_read(cursor *c, stream *out) {
    c->chain = NULL;
    while (c->pos < c->s->n) {
        item *x = &c->s->it[c->pos++];
        if (x->meta) {
            push(out, *x); /* echoed to the merge's output as it is read */
            continue;
        }
        /* a header without an id takes chainIdNext when chainRead reads it:
         * files interleave in the merge's order (chainMergeSort.c:35-67) */
        if (x->id == INT32_MIN)
            x->id = gt_next_chain_id();
        c->chain = x;
        return;
    }
}

/* cmpChainScores */
static int cmp_cur(const cursor *a, const cursor *b) {
    const double diff = a->chain->score - b->chain->score;
    return diff > 0.0 ? 1 : diff < 0.0 ? -1 : 0;
}

/* quickHeap (kent/src/lib/quickHeap.c) over cursor pointers */
typedef struct qheap {
    cursor **h;
    int n;
} qheap;

static void heap_add(qheap *q, cursor *e) {
    int n = q->n;
    q->h[q->n++] = e;
    int p = (n - 1) / 2;
    while (n > 0 && cmp_cur(q->h[p], q->h[n]) < 0) {
        cursor *t = q->h[p];
        q->h[p] = q->h[n];
        q->h[n] = t;
        n = p;
        p = (n - 1) / 2;
    }
}

static void heap_balance(qheap *q, int n) {
    const int hc = q->n;
    int c1 = 2 * n + 1, c2 = 2 * n + 2;
    for (;;) {
        int best = n;
        if (c1 < hc && cmp_cur(q->h[c1], q->h[best]) > 0)
            best = c1;
        if (c2 < hc && cmp_cur(q->h[c2], q->h[best]) > 0)
            best = c2;
        if (best == n)
            break;
        cursor *t = q->h[best];
        q->h[best] = q->h[n];
        q->h[n] = t;
        n = best;
        c1 = 2 * n + 1;
        c2 = 2 * n + 2;
    }
}

static void heap_remove(qheap *q, cursor *e) { /* removeFromQuickHeapByElem */
    int n = 0;
    while (n < q->n && q->h[n] != e)
        ++n;
    if (n == q->n)
        gt_abort("unexpected error: chainFile not found on heap");
    q->h[n] = q->h[--q->n];
    if (n < q->n)
        heap_balance(q, n);
}

/* the %1.0f text of a score, re-read with atof (a temp file round trip):
 * printf rounds the exact value to the nearest integer, ties to even --
 * nearbyint in the default rounding mode, at any magnitude */
static double printed(double s) {
    return nearbyint(s);
}

/* chainMergeSort(fileCount, files, out, level): intermediate outputs keep
 * what their temp file would hold */
static void merge(stream *const *in, int nin, stream *out, int save_id, int intermediate) {
    cursor *cur = calloc((size_t)(nin ? nin : 1), sizeof(cursor));
    qheap q = {malloc((size_t)(nin ? nin : 1) * sizeof(cursor *)), 0};
    int32_t id = 0;
    for (int i = 0; i < nin; ++i) {
        cur[i].s = in[i];
        cursor_read(&cur[i], out);
        if (cur[i].chain)
            heap_add(&q, &cur[i]);
    }
    while (q.n > 0) {
        cursor *c = q.h[0];
        item x = *c->chain;
        if (!save_id)
            x.id = ++id;
        if (intermediate)
            x.score = printed(x.score);
        push(out, x);
        cursor_read(c, out);
        if (c->chain)
            heap_balance(&q, 0);
        else
            heap_remove(&q, c);
    }
    free(cur);
    free(q.h);
}

typedef struct write_ctx {
    const stream *s;
    const gt_chains *files;
} write_ctx;

static void write_item(FILE *f, int64_t k, void *arg) {
    const write_ctx *w = arg;
    const item *x = &w->s->it[k];
    if (x->meta) {
        fprintf(f, "%s\n", x->meta);
        return;
    }
    gt_write_chain(f, &w->files[x->file], x->idx, x->score, x->id);
}

int main(int argc, char *argv[]) {
    gt_options(&argc, argv, k_opts);
    const int save_id = gt_opt_exists("saveId");
    const char *input_list = gt_opt_str("inputList", NULL);
    if ((argc < 2 && !input_list) || (argc > 1 && input_list))
        usage();
    /* input names */
    char **names = NULL;
    int nf = 0, cap = 0;
    if (input_list) {
        size_t len;
        char *buf = gt_slurp(input_list, &len);
        for (char *p = buf, *e; p < buf + len; p = e + 1) {
            e = memchr(p, '\n', (size_t)(buf + len - p));
            if (!e)
                e = buf + len;
            *e = 0;
            if (nf == cap)
                names = realloc(names, (size_t)(cap = cap ? cap * 2 : 64) * sizeof(char *));
            names[nf++] = strdup(p);
        }
        free(buf);
    } else {
        nf = argc - 1;
        names = malloc((size_t)(nf ? nf : 1) * sizeof(char *));
        for (int i = 0; i < nf; ++i)
            names[i] = argv[i + 1];
    }
    /* every input parsed; its stream: chain k after the '#' lines read with it */
    gt_chains *files = calloc((size_t)(nf ? nf : 1), sizeof(gt_chains));
    stream *level = calloc((size_t)(nf ? nf : 1), sizeof(stream));
    gt_defer_chain_ids(1); /* ids in read order: cursor_read */
    for (int i = 0; i < nf; ++i) {
        gt_read_chains(names[i], &files[i], -HUGE_VAL, 1);
        const gt_chains *c = &files[i];
        int32_t m = 0;
        for (int64_t k = 0; k <= c->n; ++k) {
            while (m < c->n_meta && c->meta_at[m] <= k)
                push(&level[i], (item){c->meta[m++], i, 0, 0, 0});
            if (k < c->n)
                push(&level[i], (item){NULL, i, k, c->score[k], c->id[k]});
        }
    }
    /* chainWriteHead gives a header id of 0 the next chainIdNext (-saveId) */
    /* hierSort: groups of MAXFILES, level by level, until one merge remains */
    stream out = {0};
    int n = nf;
    stream *cur = level;
    for (;;) {
        const int ngroups = (n + MAXFILES - 1) / MAXFILES;
        if (ngroups <= 1) {
            stream **in = malloc((size_t)(n ? n : 1) * sizeof(stream *));
            for (int i = 0; i < n; ++i)
                in[i] = &cur[i];
            merge(in, n, &out, save_id, 0);
            free(in);
            break;
        }
        stream *next = calloc((size_t)ngroups, sizeof(stream));
        for (int g = 0; g < ngroups; ++g) {
            const int a = g * MAXFILES, b = a + MAXFILES < n ? a + MAXFILES : n;
            stream **in = malloc((size_t)(b - a) * sizeof(stream *));
            for (int i = a; i < b; ++i)
                in[i - a] = &cur[i];
            merge(in, b - a, &next[g], save_id, 1);
            free(in);
        }
        for (int i = 0; i < n; ++i)
            free(cur[i].it);
        if (cur != level)
            free(cur);
        cur = next;
        n = ngroups;
    }
    for (int64_t k = 0; k < out.n; ++k)
        if (!out.it[k].meta && out.it[k].id == 0)
            out.it[k].id = gt_next_chain_id();
    write_ctx w = {&out, files};
    gt_par_write(stdout, out.n, write_item, &w);
    gt_careful_close(stdout, "stdout");
    gt_exit_ok();
}
