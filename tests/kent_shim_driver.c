/* Test infrastructure: a kent-style caller of the libgachain_kent shims
 * (include/gachain_kent.h).  It reads a .chain file into kent struct chain
 * lists itself, binds a context with both .2bit genomes, and for every
 * "chain_index start end" line of the ranges file prints
 *   chainCalcScore(chainSubsetOnT(chain, start, end))   (0 if empty)
 * exactly as src/chainNet/chainNet.c:230-248 / subchainInfo compose them.
 * usage: kent_shim_driver in.chain t.2bit q.2bit ranges.txt gap [batch|rebind]
 * ("rebind": after the scores, close the context while its chainCalcScore
 * cache is resident, open and bind a second one, score the same sub-chains
 * again and print "rebind mismatches=K")
 *        kent_shim_driver in.chain t.2bit q.2bit kentapi gap max_chains
 * The second form runs oracle/kentapi_workload.inc (the rest of the kent
 * chain API: chainScoreBlock, axtScoreUngapped, chainConnectCost,
 * cBlockFindCrossover, chainBlocks, chainRemovePartialOverlaps,
 * chainMergeAbutting, chainCalcScore) through the shims; oracle/_ref/kentref
 * runs the same workload on the reference's objects. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gachain_kent.h"

#include "kentapi_workload.inc"

/* the text of a chain's sequence (decoded from the bound context's resident
 * genome; the '-' query reverse-complemented, as axtChain loads it) */
typedef struct seq_cache {
    gac_ctx *ctx;
    char *name[2][4096];
    int strand[2][4096];
    struct dnaSeq *seq[2][4096];
    int n[2];
} seq_cache;

static struct dnaSeq *drv_seq(struct chain *c, int is_t, void *u) {
    seq_cache *sc = u;
    const int side = is_t ? 0 : 1;
    const char *nm = is_t ? c->tName : c->qName;
    const int minus = !is_t && c->qStrand == '-';
    for (int i = 0; i < sc->n[side]; ++i)
        if (!strcmp(sc->name[side][i], nm) && sc->strand[side][i] == minus)
            return sc->seq[side][i];
    const int32_t ix = gac_genome_seq_index(sc->ctx, side, nm);
    const int32_t size = gac_genome_seq_size(sc->ctx, side, ix);
    struct dnaSeq *d = calloc(1, sizeof(*d));
    d->name = strdup(nm);
    d->size = size;
    d->dna = malloc(size + 1);
    if (gac_genome_decode(sc->ctx, side, ix, 0, size, d->dna) != GAC_OK) {
        fprintf(stderr, "%s\n", gac_last_error());
        exit(1);
    }
    d->dna[size] = 0;
    if (minus) { /* reverseComplement (kent/src/lib/dnautil.c:404-462) */
        for (int i = 0, j = size - 1; i < j; ++i, --j) {
            const char x = d->dna[i];
            d->dna[i] = d->dna[j];
            d->dna[j] = x;
        }
        for (int i = 0; i < size; ++i) {
            const char x = d->dna[i];
            d->dna[i] = x == 'a' ? 't' : x == 't' ? 'a' : x == 'c' ? 'g' : x == 'g' ? 'c' : x;
        }
    }
    const int k = sc->n[side]++;
    sc->name[side][k] = strdup(nm);
    sc->strand[side][k] = minus;
    sc->seq[side][k] = d;
    return d;
}

static struct chain **read_chains(const char *path, int *pn) {
    FILE *f = fopen(path, "r");
    if (!f) {
        perror(path);
        exit(1);
    }
    char line[1 << 16];
    int n = 0, cap = 1024;
    struct chain **v = malloc(cap * sizeof(*v));
    struct chain *c = NULL;
    struct cBlock **tail = NULL;
    int t = 0, q = 0;
    while (fgets(line, sizeof(line), f)) {
        if (line[0] == '#' || line[0] == '\n')
            continue;
        if (!strncmp(line, "chain ", 6)) {
            c = calloc(1, sizeof(*c));
            char tn[256], qn[256], qs;
            sscanf(line, "chain %lf %255s %d + %d %d %255s %d %c %d %d %d", &c->score, tn, &c->tSize,
                   &c->tStart, &c->tEnd, qn, &c->qSize, &qs, &c->qStart, &c->qEnd, &c->id);
            c->tName = strdup(tn);
            c->qName = strdup(qn);
            c->qStrand = qs;
            tail = &c->blockList;
            t = c->tStart;
            q = c->qStart;
            if (n == cap)
                v = realloc(v, (cap *= 2) * sizeof(*v));
            v[n++] = c;
            continue;
        }
        int size, dt = 0, dq = 0;
        const int k = sscanf(line, "%d %d %d", &size, &dt, &dq);
        struct cBlock *b = calloc(1, sizeof(*b));
        b->tStart = t;
        b->qStart = q;
        b->tEnd = t + size;
        b->qEnd = q + size;
        *tail = b;
        tail = &b->next;
        t += size + (k == 3 ? dt : 0);
        q += size + (k == 3 ? dq : 0);
    }
    fclose(f);
    *pn = n;
    return v;
}

int main(int argc, char **argv) {
    if (argc < 6)
        return 2;
    int n;
    struct chain **ch = read_chains(argv[1], &n);
    gac_ctx *ctx;
    if (gac_open(0, &ctx) != GAC_OK || gac_genome_load_2bit(ctx, GAC_T, argv[2]) != GAC_OK ||
        gac_genome_load_2bit(ctx, GAC_Q, argv[3]) != GAC_OK) {
        fprintf(stderr, "%s\n", gac_last_error());
        return 1;
    }
    gac_kent_bind(ctx);
    struct axtScoreScheme *ss = calloc(1, sizeof(*ss)); /* blastz default */
    const char *b = "ACGT";
    const int m[4][4] = {{91, -114, -31, -123}, {-114, 100, -125, -31},
                         {-31, -125, 100, -114}, {-123, -31, -114, 91}};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            for (int ci = 0; ci < 2; ++ci)
                for (int cj = 0; cj < 2; ++cj)
                    ss->matrix[(unsigned char)(ci ? b[i] + 32 : b[i])]
                              [(unsigned char)(cj ? b[j] + 32 : b[j])] = m[i][j];
    struct gapCalc *gc = gapCalcFromFile(argv[5]);
    if (!strcmp(argv[4], "kentapi")) {
        seq_cache *sc = calloc(1, sizeof(*sc));
        sc->ctx = ctx;
        const int m = argc > 6 ? atoi(argv[6]) : n;
        kentapi_run(ch, m < n ? m : n, drv_seq, sc, ss, gc, stdout);
        fflush(stdout);
        gac_kent_forget_chains();
        gac_close(ctx);
        return 0;
    }
    FILE *rf = fopen(argv[4], "r");
    int ci, s, e, cnt = 0;
    struct chain **sub = malloc(sizeof(*sub) * 100000), **fr = malloc(sizeof(*fr) * 100000);
    while (fscanf(rf, "%d %d %d", &ci, &s, &e) == 3 && cnt < 100000) {
        chainSubsetOnT(ch[ci], s, e, &sub[cnt], &fr[cnt]);
        ++cnt;
    }
    fclose(rf);
    const int rebind = argc > 6 && !strcmp(argv[6], "rebind");
    double *first = malloc(sizeof(double) * (cnt + 1));
    if (argc > 6 && !rebind) { /* one batched call for every non-empty subset */
        struct chain **list = malloc(sizeof(*list) * cnt);
        double *g = malloc(sizeof(double) * cnt);
        int k = 0;
        for (int i = 0; i < cnt; ++i)
            if (sub[i])
                list[k++] = sub[i];
        gac_kent_score_chains(list, k, ss, gc, g);
        k = 0;
        for (int i = 0; i < cnt; ++i)
            printf("%.0f\n", sub[i] ? g[k++] : 0.0);
    } else {
        for (int i = 0; i < cnt; ++i)
            printf("%.0f\n", first[i] = sub[i] ? chainCalcScore(sub[i], ss, gc, NULL, NULL) : 0.0);
    }
    if (rebind) { /* bind A, score, close A, bind B, score (the cache must not answer) */
        gac_close(ctx);
        if (gac_open(0, &ctx) != GAC_OK || gac_genome_load_2bit(ctx, GAC_T, argv[2]) != GAC_OK ||
            gac_genome_load_2bit(ctx, GAC_Q, argv[3]) != GAC_OK) {
            fprintf(stderr, "%s\n", gac_last_error());
            return 1;
        }
        gac_kent_bind(ctx);
        int bad = 0;
        for (int i = 0; i < cnt; ++i)
            bad += (sub[i] ? chainCalcScore(sub[i], ss, gc, NULL, NULL) : 0.0) != first[i];
        printf("rebind mismatches=%d\n", bad);
        gac_kent_forget_chains();
    }
    for (int i = 0; i < cnt; ++i)
        gac_kent_chain_free(&fr[i]);
    printf("gapCalcCost(110,0)=%d\n", gapCalcCost(gc, 110, 0));
    gapCalcFree(&gc);
    gac_close(ctx);
    return 0;
}
