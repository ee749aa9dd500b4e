/* chainSort -- sort chains (drop-in for kent/src/hg/mouseStuff/chainSort).
 *
 * Same command line, options and output bytes as the reference
 * (chainSort.c:41-116): every chain is read (chainRead, kent/src/lib/
 * chain.c:256-346; '#' lines echoed first, as lineFileSetMetaDataOutput
 * does while reading), the list is reversed by slAddHead (:65) and
 * slSort'ed -- glibc's stable merge sort -- with chainCmpScore (descending
 * score), chainCmpTarget (tName, tStart) or chainCmpQuery (qName, qStart)
 * (chain.c:132-178), then written with chainWrite (chain.c:200-227).
 * -index=file writes "<hex output offset>\t<key>" whenever the key changes.
 * Here the file is parsed on all threads (gt_read_chains) and the sorted
 * text is formatted on all threads (gt_par_write). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gac_tool.h"

static const gt_spec k_opts[] = {
    {"target", GT_BOOL},
    {"query", GT_BOOL},
    {"index", GT_STRING},
    {NULL, 0},
};

static void usage(void) {
    gt_abort("chainSort - Sort chains.  By default sorts by score.\n"
             "Note this loads all chains into memory, so it is not\n"
             "suitable for large sets.  Instead, run chainSort on\n"
             "multiple small files, followed by chainMergeSort.\n"
             "usage:\n"
             "   chainSort inFile outFile\n"
             "Note that inFile and outFile can be the same\n"
             "options:\n"
             "   -target sort on target start rather than score\n"
             "   -query sort on query start rather than score\n"
             "   -index=out.tab build simple two column index file\n"
             "                    <out file position>  <value>\n"
             "                  where <value> is score, target, or query \n"
             "                  depending on the sort.\n");
}

enum { BY_SCORE, BY_TARGET, BY_QUERY };

typedef struct sort_ctx {
    const gt_chains *c;
    int mode;
    int32_t *id; /* ids as written (chainWriteHead assigns one to id 0) */
} sort_ctx;

static const sort_ctx *g_sc;

/* chainCmpScore / chainCmpTarget / chainCmpQuery, then the list position
 * (slSort is stable) */
static int cmp_chain(const void *va, const void *vb) {
    const int64_t a = *(const int64_t *)va, b = *(const int64_t *)vb;
    const gt_chains *c = g_sc->c;
    int d = 0;
    if (g_sc->mode == BY_SCORE) {
        const double diff = c->score[b] - c->score[a];
        d = diff < 0.0 ? -1 : diff > 0.0 ? 1 : 0;
    } else if (g_sc->mode == BY_TARGET) {
        d = strcmp(c->tnames.names[c->tname[a]], c->tnames.names[c->tname[b]]);
        if (d == 0)
            d = c->tstart[a] - c->tstart[b];
    } else {
        d = strcmp(c->qnames.names[c->qname[a]], c->qnames.names[c->qname[b]]);
        if (d == 0)
            d = c->qstart[a] - c->qstart[b];
    }
    if (d)
        return d;
    return (a < b) - (a > b); /* slAddHead: later chains come first */
}

typedef struct write_ctx {
    const gt_chains *c;
    const int64_t *ord;
    const int32_t *id;
} write_ctx;

static void write_one(FILE *f, int64_t k, void *arg) {
    const write_ctx *w = arg;
    const int64_t i = w->ord[k];
    gt_write_chain(f, w->c, i, w->c->score[i], w->id[i]);
}

int main(int argc, char *argv[]) {
    gt_options(&argc, argv, k_opts);
    if (argc != 3)
        usage();
    const char *in = argv[1], *out = argv[2];
    const int mode = gt_opt_exists("target") ? BY_TARGET : gt_opt_exists("query") ? BY_QUERY
                                                                                   : BY_SCORE;
    const char *index_name = gt_opt_str("index", NULL);
    gt_chains c;
    gt_read_chains(in, &c, -HUGE_VAL, 1);
    FILE *f = gt_must_open(out, "w");
    FILE *index = index_name ? gt_must_open(index_name, "w") : NULL;
    gt_verbose(2, "indexName %s, index %p\n", index_name ? index_name : "(null)", (void *)index);
    for (int32_t m = 0; m < c.n_meta; ++m)
        fprintf(f, "%s\n", c.meta[m]);
    int64_t *ord = malloc((size_t)(c.n ? c.n : 1) * 8);
    for (int64_t k = 0; k < c.n; ++k)
        ord[k] = k;
    sort_ctx sc = {&c, mode, NULL};
    g_sc = &sc;
    qsort(ord, (size_t)c.n, 8, cmp_chain);
    /* chainWriteHead: a header id of 0 gets chainIdNext, in output order */
    int32_t *id = malloc((size_t)(c.n ? c.n : 1) * 4);
    memcpy(id, c.id, (size_t)c.n * 4);
    for (int64_t k = 0; k < c.n; ++k)
        if (id[ord[k]] == 0)
            id[ord[k]] = gt_next_chain_id();
    write_ctx w = {&c, ord, id};
    if (!index) {
        gt_par_write(f, c.n, write_one, &w);
    } else {
        double last_score = -1;
        const char *last_name = "";
        for (int64_t k = 0; k < c.n; ++k) {
            const int64_t i = ord[k];
            if (mode == BY_TARGET || mode == BY_QUERY) {
                const char *nm = mode == BY_TARGET ? c.tnames.names[c.tname[i]]
                                                   : c.qnames.names[c.qname[i]];
                if (strcmp(nm, last_name) != 0) {
                    last_name = nm;
                    fprintf(index, "%lx\t", ftell(f));
                    fprintf(index, "%s\n", nm);
                }
            } else if (c.score[i] != last_score) {
                last_score = c.score[i];
                fprintf(index, "%lx\t", ftell(f));
                fprintf(index, "%1.0f\n", c.score[i]);
            }
            write_one(f, k, &w);
        }
        gt_careful_close(index, index_name);
    }
    gt_careful_close(f, out);
    gt_exit_ok();
}
