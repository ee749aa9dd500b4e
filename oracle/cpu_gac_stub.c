/* cpu_gac_stub.c -- TEST INFRASTRUCTURE ONLY (never linked into libgachain
 * or any shipped tool).
 *
 * A CPU stand-in for the device half of the libgachain ABI, so that the
 * host-side axtChain DP (csrc/host/gac_axtchain.c) and the tool front end
 * (csrc/tools/axtChain.c) can be profiled and checked against the reference
 * in this GPU-less container: `make -f oracle/ref.mk` does not build it;
 * `make cpu-axtchain` links oracle/_build/axtChain_cpu from the product
 * sources plus this file.  Scoring here is the plain reference arithmetic
 * (axtScoreUngapped, chainCalcScore: kent/src/lib/axt.c:186-194,
 * chainConnect.c:24-40); the parity evidence for the product remains the
 * GPU tests. */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gachain.h"
#include "host/gac_host.h"

typedef struct side {
    gac_twobit tb;
    int loaded;
    int32_t n;
    char **names;
    int32_t *sizes;
    const uint8_t **packed;
    int32_t **ns, **nz, *nn;
} side;

struct gac_ctx {
    side s[2];
    int32_t mat[16];
    const gac_gapcalc *g;
};

struct gac_chainset {
    int64_t n;
    int32_t *tseq, *qseq;
    uint8_t *strand;
    int64_t *off;
    int32_t *bt, *bq, *bs;
};

int gac_open(int device, gac_ctx **out) {
    (void)device;
    *out = calloc(1, sizeof(gac_ctx));
    return GAC_OK;
}
void gac_close(gac_ctx *c) { free(c); }

int gac_set_scoring(gac_ctx *c, const int32_t mat[16], const gac_gapcalc *g) {
    memcpy(c->mat, mat, sizeof(c->mat));
    c->g = g;
    return GAC_OK;
}

int gac_genome_load_2bit(gac_ctx *c, int which, const char *path) {
    side *s = &c->s[which];
    int rc = gac_twobit_open(path, &s->tb);
    if (rc != GAC_OK)
        return rc;
    s->n = (int32_t)s->tb.seq_count;
    s->names = calloc(s->n, sizeof(char *));
    s->sizes = calloc(s->n, 4);
    s->packed = calloc(s->n, sizeof(uint8_t *));
    s->ns = calloc(s->n, sizeof(int32_t *));
    s->nz = calloc(s->n, sizeof(int32_t *));
    s->nn = calloc(s->n, 4);
    for (int32_t i = 0; i < s->n; ++i) {
        const gac_twobit_seq *q = &s->tb.seqs[i];
        s->names[i] = q->name;
        s->sizes[i] = (int32_t)q->size;
        s->packed[i] = q->packed;
        s->nn[i] = (int32_t)q->n_count;
        s->ns[i] = malloc((q->n_count + 1) * 4);
        s->nz[i] = malloc((q->n_count + 1) * 4);
        for (uint32_t k = 0; k < q->n_count; ++k) {
            s->ns[i][k] = (int32_t)gac_twobit_u32(&s->tb, q->n_starts_raw + 4 * k);
            s->nz[i][k] = (int32_t)gac_twobit_u32(&s->tb, q->n_sizes_raw + 4 * k);
        }
    }
    s->loaded = 1;
    return GAC_OK;
}

int gac_genome_add_seq(gac_ctx *c, int which, const char *name, int32_t size,
                       const uint8_t *packed, int32_t n_nblocks, const int32_t *n_starts,
                       const int32_t *n_sizes) {
    side *s = &c->s[which];
    s->names = realloc(s->names, (s->n + 1) * sizeof(char *));
    s->sizes = realloc(s->sizes, (s->n + 1) * 4);
    s->packed = realloc(s->packed, (s->n + 1) * sizeof(uint8_t *));
    s->ns = realloc(s->ns, (s->n + 1) * sizeof(int32_t *));
    s->nz = realloc(s->nz, (s->n + 1) * sizeof(int32_t *));
    s->nn = realloc(s->nn, (s->n + 1) * 4);
    s->names[s->n] = strdup(name);
    s->sizes[s->n] = size;
    uint8_t *p = malloc((size_t)(size + 3) / 4 + 1);
    memcpy(p, packed, (size_t)(size + 3) / 4);
    s->packed[s->n] = p;
    s->ns[s->n] = malloc((n_nblocks + 1) * 4);
    s->nz[s->n] = malloc((n_nblocks + 1) * 4);
    memcpy(s->ns[s->n], n_starts, n_nblocks * 4);
    memcpy(s->nz[s->n], n_sizes, n_nblocks * 4);
    s->nn[s->n] = n_nblocks;
    ++s->n;
    return GAC_OK;
}

int gac_genome_finalize(gac_ctx *c, int which) {
    c->s[which].loaded = 1;
    return GAC_OK;
}

int32_t gac_genome_seq_index(gac_ctx *c, int which, const char *name) {
    for (int32_t i = 0; i < c->s[which].n; ++i)
        if (strcmp(c->s[which].names[i], name) == 0)
            return i;
    return -1;
}
int32_t gac_genome_seq_size(gac_ctx *c, int which, int32_t i) { return c->s[which].sizes[i]; }
const char *gac_genome_seq_name(gac_ctx *c, int which, int32_t i) { return c->s[which].names[i]; }

int gac_genome_view(gac_ctx *c, int which, int32_t i, gac_seq_view *v) {
    side *s = &c->s[which];
    v->packed = s->packed[i];
    v->size = s->sizes[i];
    v->n_start = s->ns[i];
    v->n_size = s->nz[i];
    v->n_count = s->nn[i];
    return GAC_OK;
}

static int base(const side *s, int32_t i, int minus, int32_t j) {
    const int32_t size = s->sizes[i];
    const int32_t f = minus ? size - 1 - j : j;
    for (int32_t k = 0; k < s->nn[i]; ++k)
        if (f >= s->ns[i][k] && f < s->ns[i][k] + s->nz[i][k])
            return 4;
    const int c = (s->packed[i][f >> 2] >> (6 - 2 * (f & 3))) & 3;
    return minus ? c ^ 2 : c;
}

static int block_score(gac_ctx *c, int32_t ts, int32_t qs, int minus, int32_t t, int32_t q,
                       int32_t n) {
    static const int acgt[4] = {3, 1, 0, 2};
    int s = 0;
    for (int32_t i = 0; i < n; ++i) {
        const int tc = base(&c->s[0], ts, 0, t + i), qc = base(&c->s[1], qs, minus, q + i);
        if (tc < 4 && qc < 4)
            s += c->mat[acgt[qc] * 4 + acgt[tc]];
    }
    return s;
}

int gac_score_blocks(gac_ctx *c, int64_t np, const int32_t *ts, const int32_t *qs,
                     const uint8_t *st, const int64_t *off, const int32_t *bt, const int32_t *bq,
                     const int32_t *bs, int32_t *out) {
    for (int64_t p = 0; p < np; ++p)
        for (int64_t b = off[p]; b < off[p + 1]; ++b)
            out[b] = block_score(c, ts[p], qs[p], st[p], bt[b], bq[b], bs[b]);
    return GAC_OK;
}

int gac_chains_upload(gac_ctx *c, const gac_chainset_desc *d, gac_chainset **out) {
    (void)c;
    gac_chainset *s = calloc(1, sizeof(*s));
    s->n = d->n_chains;
    s->tseq = malloc(d->n_chains * 4 + 4);
    s->qseq = malloc(d->n_chains * 4 + 4);
    s->strand = malloc(d->n_chains + 1);
    s->off = malloc((d->n_chains + 1) * 8);
    s->bt = malloc(d->n_blocks * 4 + 4);
    s->bq = malloc(d->n_blocks * 4 + 4);
    s->bs = malloc(d->n_blocks * 4 + 4);
    memcpy(s->tseq, d->t_seq, d->n_chains * 4);
    memcpy(s->qseq, d->q_seq, d->n_chains * 4);
    memcpy(s->strand, d->q_strand, d->n_chains);
    memcpy(s->off, d->blk_off, (d->n_chains + 1) * 8);
    memcpy(s->bt, d->blk_t, d->n_blocks * 4);
    memcpy(s->bq, d->blk_q, d->n_blocks * 4);
    memcpy(s->bs, d->blk_size, d->n_blocks * 4);
    *out = s;
    return GAC_OK;
}

void gac_chains_free(gac_chainset *s) {
    if (!s)
        return;
    free(s->tseq);
    free(s->qseq);
    free(s->strand);
    free(s->off);
    free(s->bt);
    free(s->bq);
    free(s->bs);
    free(s);
}

/* whole-chain ranges only (what gac_axt_chain asks for) */
int gac_score_ranges(gac_ctx *c, const gac_chainset *s, const gac_range *r, int64_t n,
                     uint32_t flags, int64_t *g, int64_t *l, int32_t *ali) {
    (void)flags;
    (void)l;
    for (int64_t i = 0; i < n; ++i) {
        const int32_t k = r[i].chain;
        int64_t sc = 0;
        int32_t a = 0;
        for (int64_t b = s->off[k]; b < s->off[k + 1]; ++b) {
            sc += block_score(c, s->tseq[k], s->qseq[k], s->strand[k], s->bt[b], s->bq[b], s->bs[b]);
            a += s->bs[b];
            if (b + 1 < s->off[k + 1])
                sc -= gac_gap_cost(c->g, s->bq[b + 1] - (s->bq[b] + s->bs[b]),
                                   s->bt[b + 1] - (s->bt[b] + s->bs[b]));
        }
        g[i] = sc;
        ali[i] = a;
    }
    return GAC_OK;
}
