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

int gac_genome_load_twobit(gac_ctx *c, int which, gac_twobit *tb);

int gac_genome_load_2bit(gac_ctx *c, int which, const char *path) {
    gac_twobit tb;
    int rc = gac_twobit_open(path, &tb);
    if (rc != GAC_OK)
        return rc;
    return gac_genome_load_twobit(c, which, &tb);
}

int gac_genome_load_twobit_runs(gac_ctx *c, int which, gac_twobit *tb, const uint8_t *keep,
                                const int64_t *run_off, const int32_t *run_lo, const int32_t *run_hi) {
    (void)keep; /* the host stand-in keeps every sequence */
    int rc = gac_genome_load_twobit(c, which, tb);
    if (rc != GAC_OK || !run_off)
        return rc;
    /* words outside the runs are poisoned (a different base pattern), so a
     * run set that misses a word the scoring reads changes the scores */
    side *s = &c->s[which];
    const int all = getenv("GAC_STUB_POISON_ALL") != NULL; /* tests the check itself */
    for (int32_t i = 0; i < s->n; ++i) {
        const size_t nb = ((size_t)s->sizes[i] + 3) / 4;
        uint8_t *p = malloc(nb + 8);
        memset(p, 0x9c, nb + 8);
        for (int64_t r = run_off[i]; r < run_off[i + 1] && !all; ++r) {
            const size_t b0 = (size_t)run_lo[r] * 8, b1 = (size_t)run_hi[r] * 8;
            memcpy(p + b0, s->packed[i] + b0, (b1 < nb ? b1 : nb) - b0);
        }
        s->packed[i] = p;
    }
    return GAC_OK;
}

int gac_genome_load_twobit_keep(gac_ctx *c, int which, gac_twobit *tb, const uint8_t *keep) {
    (void)keep; /* the axtChain front end loads whole files */
    return gac_genome_load_twobit(c, which, tb);
}

/* the file is already open (the tools map it while the device starts) */
int gac_genome_load_twobit(gac_ctx *c, int which, gac_twobit *tb) {
    side *s = &c->s[which];
    s->tb = *tb;
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
    int32_t lo = 0, hi = s->nn[i]; /* first N run ending past f (runs sorted, disjoint) */
    while (lo < hi) {
        const int32_t mid = (lo + hi) / 2;
        if (s->ns[i][mid] + s->nz[i][mid] > f)
            hi = mid;
        else
            lo = mid + 1;
    }
    if (lo < s->nn[i] && s->ns[i][lo] <= f)
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

/* the chain's blocks clipped to [t_start, t_end) on the target, scored with
 * the linear gap costs between consecutive clipped blocks (whole chains for
 * gac_axt_chain; chainNet's partial fills) */
int gac_score_ranges(gac_ctx *c, const gac_chainset *s, const gac_range *r, int64_t n,
                     uint32_t flags, int64_t *g, int64_t *l, int32_t *ali) {
    for (int64_t i = 0; i < n; ++i) {
        const int32_t k = r[i].chain, lo = r[i].t_start, hi = r[i].t_end;
        int64_t sc = 0, ls = 0, lm = 0; /* (local: chainCalcScoreLocal's running score, max) */
        int32_t a = 0, have = 0, pq = 0, pt = 0;
        for (int64_t b = s->off[k]; b < s->off[k + 1]; ++b) {
            const int32_t t0 = s->bt[b] > lo ? s->bt[b] : lo;
            const int32_t t1 = s->bt[b] + s->bs[b] < hi ? s->bt[b] + s->bs[b] : hi;
            if (t1 <= t0)
                continue;
            const int32_t q0 = s->bq[b] + (t0 - s->bt[b]);
            if (have) {
                const int gc = gac_gap_cost(c->g, q0 - pq, t0 - pt);
                sc -= gc;
                ls = ls - gc > 0 ? ls - gc : 0;
            }
            const int bsc = block_score(c, s->tseq[k], s->qseq[k], s->strand[k], t0, q0, t1 - t0);
            sc += bsc;
            ls += bsc;
            if (ls > lm)
                lm = ls;
            a += t1 - t0;
            pq = q0 + (t1 - t0);
            pt = t1;
            have = 1;
        }
        g[i] = sc;
        ali[i] = a;
        if ((flags & GAC_WANT_LOCAL) && l)
            l[i] = lm;
    }
    return GAC_OK;
}

/* chains in host memory: a temporary set */
int gac_score_ranges_host(gac_ctx *c, const gac_chainset_desc *d, const gac_range *r, int64_t n,
                          uint32_t flags, int64_t *g, int64_t *l, int32_t *ali) {
    gac_chainset *s = NULL;
    gac_chains_upload(c, d, &s);
    const int rc = gac_score_ranges(c, s, r, n, flags, g, l, ali);
    gac_chains_free(s);
    return rc;
}

/* windows: each one checked against chainSubsetOnT's walk (kent/src/lib/
 * chain.c:481-500: first block with tEnd > tStart, then while tStart < tEnd)
 * -- the netting's recorded windows must be exactly those -- then scored as
 * its range */
int gac_score_windows(gac_ctx *c, const gac_chainset *s, const gac_window *w, int64_t n,
                      uint32_t flags, int64_t *g, int64_t *l, int32_t *ali) {
    gac_range *r = malloc((size_t)(n ? n : 1) * sizeof(gac_range));
    for (int64_t i = 0; i < n; ++i) {
        const int32_t k = w[i].chain;
        if (k < 0 || k >= s->n) {
            free(r);
            return gac_fail(GAC_E_ARG, "window %lld: chain %d out of range", (long long)i, k);
        }
        const int64_t b0 = s->off[k], b1 = s->off[k + 1];
        const int32_t ts = b1 > b0 ? s->bt[b0] : 0, te = b1 > b0 ? s->bt[b1 - 1] + s->bs[b1 - 1] : 0;
        if (!(w[i].t_start <= ts && w[i].t_end >= te) && w[i].t_start < w[i].t_end) {
            int64_t f = b0, e;
            while (f < b1 && s->bt[f] + s->bs[f] <= w[i].t_start)
                ++f;
            for (e = f; e < b1 && s->bt[e] < w[i].t_end; ++e)
                ;
            if (w[i].first_block != f - b0 || w[i].n_blocks != e - f) {
                fprintf(stderr, "cpu stub: window %lld of chain %d [%d, %d): got blocks %d + %d, "
                                "chainSubsetOnT selects %lld + %lld\n", (long long)i, k,
                        w[i].t_start, w[i].t_end, w[i].first_block, w[i].n_blocks,
                        (long long)(f - b0), (long long)(e - f));
                free(r);
                return gac_fail(GAC_E_ARG, "window mismatch");
            }
        }
        r[i].chain = k;
        r[i].t_start = w[i].t_start;
        r[i].t_end = w[i].t_end;
    }
    const int rc = gac_score_ranges(c, s, r, n, flags, g, l, ali);
    free(r);
    return rc;
}

/* ---- gac_chain_dp / gac_crossovers: a lane-by-lane CPU emulation of the
 * device algorithm of k_dp / k_xover (csrc/gac_dp.hip) -- windows of 64
 * pre-order nodes resolved by prefix-max rounds, crossovers by prefix sum
 * and first maximum -- so that the algorithm and the host's GAC_AXT_DP=gpu
 * phases can be checked against the reference here. */
static int emu_gap(gac_ctx *c, int dq, int dt) {
    if (dq < 0)
        dq = 0;
    if (dt < 0)
        dt = 0;
    return gac_gap_cost(c->g, dq, dt);
}

static int emu_msc(gac_ctx *c, int q, int t) {
    static const int acgt[4] = {3, 1, 0, 2};
    return (q == 4 || t == 4) ? 0 : c->mat[acgt[q] * 4 + acgt[t]];
}

static void emu_xover(gac_ctx *c, int32_t ts, int32_t qs, int minus, int lqe, int lte, int rqs,
                      int rts, int ov, int *pos, int *adj) {
    long long carry = 0, lsum = 0, bestv = 0;
    int bestpos = 0;
    for (int base0 = 0; base0 < ov; base0 += 64) {
        long long incl[64], l[64];
        long long run = 0;
        for (int lane = 0; lane < 64; ++lane) {
            const int k = base0 + lane;
            long long d = 0;
            l[lane] = 0;
            if (k < ov) {
                l[lane] = emu_msc(c, base(&c->s[1], qs, minus, lqe - ov + k), base(&c->s[0], ts, 0, lte - ov + k));
                d = l[lane] - emu_msc(c, base(&c->s[1], qs, minus, rqs + k), base(&c->s[0], ts, 0, rts + k));
            }
            run += d;
            incl[lane] = run;
        }
        long long mv = INT64_MIN;
        int mk = 0;
        for (int lane = 0; lane < 64; ++lane)
            if (base0 + lane < ov && carry + incl[lane] > mv) {
                mv = carry + incl[lane];
                mk = base0 + lane;
            }
        if (mv > bestv) {
            bestv = mv;
            bestpos = mk + 1;
        }
        carry += incl[63];
        for (int lane = 0; lane < 64; ++lane)
            lsum += l[lane];
    }
    *pos = bestpos;
    *adj = (int)(lsum - bestv);
}

/* whole chains: the ranges API over every chain's full target span */
int gac_score_chains(gac_ctx *c, const gac_chainset *s, uint32_t flags, int64_t *g, int64_t *l,
                     int32_t *ali) {
    gac_range *r = malloc((size_t)(s->n ? s->n : 1) * sizeof(gac_range));
    for (int64_t k = 0; k < s->n; ++k) {
        const int64_t b0 = s->off[k], b1 = s->off[k + 1];
        r[k].chain = (int32_t)k;
        r[k].t_start = b1 > b0 ? s->bt[b0] : 0;
        r[k].t_end = b1 > b0 ? s->bt[b1 - 1] + s->bs[b1 - 1] : 0;
    }
    const int rc = gac_score_ranges(c, s, r, s->n, flags, g, l, ali);
    free(r);
    return rc;
}

int gac_crossovers(gac_ctx *c, int64_t n, const int32_t *t_seq, const int32_t *q_seq,
                   const uint8_t *q_strand, const int32_t *lqe, const int32_t *lte,
                   const int32_t *rqs, const int32_t *rts, const int32_t *overlap, int32_t *pos,
                   int32_t *adj) {
    for (int64_t j = 0; j < n; ++j)
        emu_xover(c, t_seq[j], q_seq[j], q_strand[j], lqe[j], lte[j], rqs[j], rts[j], overlap[j],
                  &pos[j], &adj[j]);
    return GAC_OK;
}

static int emu_connect(gac_ctx *c, int32_t ts, int32_t qs, int minus, int aqs, int aqe, int ate,
                       int bqs, int bqe, int bts) {
    int dq = bqs - aqe, dt = bts - ate, adj = 0;
    if (dq < 0 || dt < 0) {
        const int bsz = bqe - bqs, asz = aqe - aqs, ov = -(dq < dt ? dq : dt);
        if (ov >= bsz || ov >= asz) {
            adj = 100000000;
        } else {
            int p;
            emu_xover(c, ts, qs, minus, aqe, ate, bqs, bts, ov, &p, &adj);
            dq += ov;
            dt += ov;
        }
    }
    return adj + emu_gap(c, dq, dt);
}

/* one window walk of k_dp / k_dp_fast (csrc/gac_dp.hip dp_walk), lane by
 * lane: fast = the linear bound and ties to the smaller node (best seeded) */
typedef struct emu_pair {
    gac_ctx *c;
    int32_t ts, qs;
    uint8_t minus;
    const int32_t *na, *nb;
    long long *ms, *nw, *tot;
    int nn;
} emu_pair;

static long long g_emu_windows[2], g_emu_walks[2];
static void emu_walk(const emu_pair *E, int fast, int lq, int lqe, int lt, long long ls,
                     long long kl, long long *best_io, int *node_io) {
    long long best = *best_io;
    int best_node = *node_io, p0 = 0;
    const int nn = E->nn;
    ++g_emu_walks[fast];
    while (p0 < nn) {
        ++g_emu_windows[fast];
        long long key[64], sc[64], NW[64];
        int cand[64], se[64], nxt[64], in[64], lf[64], end[64];
        for (int lane = 0; lane < 64; ++lane) {
            const int v = p0 + lane;
            in[lane] = v < nn;
            se[lane] = v + 1;
            cand[lane] = 0;
            lf[lane] = 0;
            key[lane] = 0;
            sc[lane] = 0;
            NW[lane] = 0;
            nxt[lane] = v + 1;
            end[lane] = v + 1;
            if (!in[lane])
                continue;
            const int32_t *A = E->na + 4 * v, *B = E->nb + 2 * v;
            const long long m1 = E->ms[v] + ls;
            const int gc = emu_gap(E->c, lq - A[0], lt - A[1]);
            const long long m2 = m1 - gc;
            key[lane] = m1 < m2 ? m1 : m2;
            NW[lane] = fast ? E->nw[v] : 0;
            lf[lane] = B[1] < 0;
            end[lane] = B[0];
            if (lf[lane] && A[2] < lq && A[3] < lt) {
                cand[lane] = 1;
                const int dq = lq - A[0], dt = lt - A[1];
                const int cost = (fast && dq >= 0 && dt >= 0)
                                     ? gc
                                     : emu_connect(E->c, E->ts, E->qs, E->minus, A[2], A[0], A[1],
                                                   lq, lqe, lt);
                sc[lane] = E->tot[v] + ls - cost;
            }
            if (!lf[lane])
                nxt[lane] = (B[1] == 0 ? lq : lt) > A[2] ? v + 1 : A[3];
        }
        int cur = 0;
        for (;;) {
            int pr[64];
            for (int lane = 0; lane < 64; ++lane) {
                pr[lane] = key[lane] < best || (fast && NW[lane] - kl < 1024 * best);
                if (lane >= cur && in[lane])
                    se[lane] = pr[lane] ? end[lane] : (lf[lane] ? p0 + lane + 1 : nxt[lane]);
            }
            int u = -1, pm = 0;
            for (int lane = 0; lane < 64; ++lane) {
                const int visited = in[lane] && pm <= p0 + lane;
                const int better = sc[lane] > best || (fast && sc[lane] == best && p0 + lane < best_node);
                if (u < 0 && visited && lane >= cur && cand[lane] && !pr[lane] && better)
                    u = lane;
                if (se[lane] > pm)
                    pm = se[lane];
            }
            if (u < 0)
                break;
            best = sc[u];
            best_node = p0 + u;
            cur = u + 1;
        }
        int mx = 0;
        for (int lane = 0; lane < 64; ++lane)
            if (in[lane] && se[lane] > mx)
                mx = se[lane];
        p0 = p0 + 64 > mx ? p0 + 64 : mx;
    }
    *best_io = best;
    *node_io = best_node;
}

int gac_chain_dp_ex(gac_ctx *c, int64_t n_pairs, const int32_t *t_seq, const int32_t *q_seq,
                    const uint8_t *q_strand, const int64_t *node_off, const int32_t *node_a,
                    const int32_t *node_b, const int64_t *leaf_off, const int32_t *leaf,
                    const int32_t *leaf_score, const int32_t *leaf_node, const int64_t *path_off,
                    const int32_t *path, const int64_t *ov_off, const int32_t *ov, int64_t lin_k,
                    int32_t min_entry, int64_t *total, int32_t *pred) {
    const int64_t NN = node_off[n_pairs];
    const int fast = ov_off != NULL;
    long long *ms = calloc((size_t)(NN ? NN : 1), 8), *tot = calloc((size_t)(NN ? NN : 1), 8);
    long long *nw = malloc((size_t)(NN ? NN : 1) * 8);
    for (int64_t v = 0; v < NN; ++v)
        nw[v] = INT64_MIN / 4;
    for (int64_t p = 0; p < n_pairs; ++p)
        for (int64_t i = leaf_off[p]; i < leaf_off[p + 1]; ++i)
            tot[node_off[p] + leaf_node[i]] = leaf_score[i];
    for (int64_t p = 0; p < n_pairs; ++p) {
        const int64_t o = node_off[p];
        emu_pair E = {c, t_seq[p], q_seq[p], q_strand[p], node_a + 4 * o, node_b + 2 * o,
                      ms + o, nw + o, tot + o, (int)(node_off[p + 1] - o)};
        /* k_dp_fast's ring: the previous 64 leaves */
        int rbox[64][4], rnode[64];
        long long rtot[64];
        for (int k = 0; k < 64; ++k)
            rnode[k] = -1;
        for (int64_t li = leaf_off[p]; li < leaf_off[p + 1]; ++li) {
            const int i = (int)(li - leaf_off[p]);
            const int lq = leaf[4 * li], lqe = leaf[4 * li + 1], lt = leaf[4 * li + 2],
                      lte = leaf[4 * li + 3];
            const long long ls = leaf_score[li];
            const long long kl = fast ? lin_k * ((long long)lq + lt) - 1024 * ls : 0;
            long long best = 0;
            int best_node = -1;
            if (fast) {
                /* A: the ring's non-overlapping candidates, max score, ties
                 * to the smaller node, > 0 only */
                for (int k = 0; k < 64; ++k) {
                    if (rnode[k] < 0 || !(rbox[k][0] < lq && rbox[k][2] < lt))
                        continue;
                    const int dq = lq - rbox[k][1], dt = lt - rbox[k][3];
                    if (dq < 0 || dt < 0)
                        continue;
                    const long long sc = rtot[k] + ls - emu_gap(c, dq, dt);
                    if (sc > 0 && (sc > best || (sc == best && rnode[k] < best_node))) {
                        best = sc;
                        best_node = rnode[k];
                    }
                }
                /* B */
                emu_walk(&E, 1, lq, lqe, lt, ls, kl, &best, &best_node);
                /* C */
                int fb = 0;
                const long long need = best > 0 ? best : 1;
                for (int64_t k = ov_off[li]; k < ov_off[li + 1] && !fb; ++k) {
                    const int cn = ov[k];
                    if (cn < 0) {
                        fb = 1;
                        break;
                    }
                    const int cpos = ~E.nb[2 * cn + 1];
                    const int32_t *cb = leaf + 4 * (leaf_off[p] + cpos);
                    const int dq = lq - cb[1], dt = lt - cb[3];
                    const int ovl = -(dq < dt ? dq : dt);
                    if (ovl >= lqe - lq || ovl >= cb[1] - cb[0])
                        continue;
                    const long long tc = tot[o + cn];
                    const long long ub = tc + ls - emu_gap(c, dq + ovl, dt + ovl) - (long long)ovl * min_entry;
                    if (ub < need)
                        continue;
                    const long long sc = tc + ls - emu_connect(c, t_seq[p], q_seq[p], q_strand[p], cb[0],
                                                                cb[1], cb[3], lq, lqe, lt);
                    if (sc < need)
                        continue;
                    const long long bc = tc + ls - emu_gap(c, dq, dt);
                    const long long bl = 1024 * tc - lin_k * ((long long)dq + dt) + 1024 * ls;
                    if (sc > bc || 1024 * sc > bl)
                        fb = 1;
                }
                if (fb) {
                    best = 0;
                    best_node = -1;
                    emu_walk(&E, 0, lq, lqe, lt, ls, 0, &best, &best_node);
                }
            } else {
                emu_walk(&E, 0, lq, lqe, lt, ls, 0, &best, &best_node);
            }
            long long t = ls;
            int pr = -1;
            if (best > ls) {
                t = best;
                pr = best_node;
            }
            total[li] = t;
            pred[li] = pr;
            tot[o + leaf_node[li]] = t;
            const long long nwv = 1024 * t + lin_k * ((long long)lqe + lte);
            for (int64_t k = path_off[li]; k < path_off[li + 1]; ++k) {
                if (ms[o + path[k]] < t)
                    ms[o + path[k]] = t;
                if (nw[o + path[k]] < nwv)
                    nw[o + path[k]] = nwv;
            }
            rbox[i & 63][0] = lq;
            rbox[i & 63][1] = lqe;
            rbox[i & 63][2] = lt;
            rbox[i & 63][3] = lte;
            rtot[i & 63] = t;
            rnode[i & 63] = leaf_node[li];
        }
    }
    free(ms);
    free(tot);
    free(nw);
    if (getenv("GAC_EMU_STATS"))
        fprintf(stderr, "[emu dp] fast walks %lld, %.2f windows each; reference walks %lld, %.2f windows each\n",
                g_emu_walks[1], (double)g_emu_windows[1] / (g_emu_walks[1] ? g_emu_walks[1] : 1),
                g_emu_walks[0], (double)g_emu_windows[0] / (g_emu_walks[0] ? g_emu_walks[0] : 1));
    return GAC_OK;
}

int gac_chain_dp(gac_ctx *c, int64_t n_pairs, const int32_t *t_seq, const int32_t *q_seq,
                 const uint8_t *q_strand, const int64_t *node_off, const int32_t *node_a,
                 const int32_t *node_b, const int64_t *leaf_off, const int32_t *leaf,
                 const int32_t *leaf_score, const int32_t *leaf_node, const int64_t *path_off,
                 const int32_t *path, int64_t *total, int32_t *pred) {
    return gac_chain_dp_ex(c, n_pairs, t_seq, q_seq, q_strand, node_off, node_a, node_b, leaf_off,
                           leaf, leaf_score, leaf_node, path_off, path, NULL, NULL, 0, 0, total,
                           pred);
}

/* gac_chain_dp_blocks: the device build of gac_dptree.hip restated kernel by
 * kernel as sequential loops (every kernel is a per-element map or scatter,
 * so a loop in any order gives the device's result), then the emulated DP
 * above -- the level-synchronous kd-tree build is checked here, on CPU,
 * against the reference's chains by the axtChain_cpu tests */
typedef struct dt_key {
    unsigned long long k;
    int64_t r;
    int32_t v;
} dt_key;

static int dt_key_cmp(const void *a, const void *b) {
    const dt_key *x = a, *y = b;
    if (x->k != y->k)
        return x->k < y->k ? -1 : 1;
    return (x->r > y->r) - (x->r < y->r);
}

int gac_chain_dp_blocks(gac_ctx *c, int64_t P, const int32_t *t_seq, const int32_t *q_seq,
                        const uint8_t *q_strand, const int64_t *blk_off, const int32_t *box,
                        const int32_t *score, int fast, int64_t lin_k, int32_t min_entry,
                        int32_t ov_cap, int64_t *leaf_off, int32_t *tord_out, int64_t *total,
                        int32_t *pred) {
    const int64_t B = blk_off[P];
    dt_key *k1 = malloc((size_t)(B ? B : 1) * sizeof(dt_key));
    for (int64_t p = 0, r = 0; p < P; ++p)
        for (int64_t j = blk_off[p]; j < blk_off[p + 1]; ++j, ++r) {
            const int64_t g = blk_off[p] + (blk_off[p + 1] - 1 - r); /* (k_dt_keys) */
            const int32_t *b = box + 4 * g;
            if (b[0] < 0 || b[0] > b[1] || b[1] > c->s[1].sizes[q_seq[p]] || b[2] < 0 ||
                b[2] > b[3] || b[3] > c->s[0].sizes[t_seq[p]]) {
                fprintf(stderr, "stub: bad block p %lld g %lld: %d %d %d %d sizes t %d q %d\n", (long long)p, (long long)g, b[0], b[1], b[2], b[3], c->s[0].sizes[t_seq[p]], c->s[1].sizes[q_seq[p]]);
                free(k1);
                return GAC_E_ARG;
            }
            k1[r] = (dt_key){b[2] != b[3] ? ((unsigned long long)p << 31) | (unsigned)b[2]
                                          : ((unsigned long long)P << 31), r, (int32_t)g};
        }
    qsort(k1, (size_t)B, sizeof(dt_key), dt_key_cmp);
    for (int64_t p = 0, r = 0; p <= P; ++p) {
        while (r < B && k1[r].k < ((unsigned long long)p << 31))
            ++r;
        leaf_off[p] = r;
    }
    const int64_t L = leaf_off[P];
    int64_t *node_off = malloc((size_t)(P + 1) * 8), maxnl = 0;
    node_off[0] = 0;
    for (int64_t p = 0; p < P; ++p) {
        const int64_t nl = leaf_off[p + 1] - leaf_off[p];
        maxnl = nl > maxnl ? nl : maxnl;
        node_off[p + 1] = node_off[p] + (nl ? 2 * nl - 1 : 0);
    }
    const int64_t N = node_off[P];
    int32_t *tord = malloc((size_t)(L + 1) * 4), *pidx = malloc((size_t)(L + 1) * 4);
    int32_t *tpos = malloc((size_t)(B + 1) * 4), *qpos = malloc((size_t)(B + 1) * 4),
            *posd = malloc((size_t)(B + 1) * 4);
    int32_t *lf = malloc((size_t)(L + 1) * 16), *lsc = malloc((size_t)(L + 1) * 4);
    int32_t *ql = malloc((size_t)(L + 1) * 4), *tl = malloc((size_t)(L + 1) * 4),
            *spare = malloc((size_t)(L + 1) * 4);
    int32_t *ss = malloc((size_t)(L + 1) * 4), *sl = malloc((size_t)(L + 1) * 4),
            *sn = malloc((size_t)(L + 1) * 4), *flag = malloc((size_t)(L + 1) * 4),
            *excl = malloc((size_t)(L + 1) * 4);
    int32_t *qbox = malloc((size_t)(L + 1) * 16), *qtp = malloc((size_t)(L + 1) * 4),
            *lnode = malloc((size_t)(L + 1) * 4);
    int32_t *na = calloc((size_t)(N + 1), 16), *nb = calloc((size_t)(N + 1), 8),
            *ndep = malloc((size_t)(N + 1) * 4), *ndl = malloc((size_t)(N + 1) * 4);
    dt_key *k2 = malloc((size_t)(L + 1) * sizeof(dt_key));
    for (int64_t i = 0; i < L; ++i) { /* k_dt_tinit */
        const int32_t g = k1[i].v, p = (int32_t)(k1[i].k >> 31);
        tord[i] = g;
        pidx[i] = p;
        tpos[g] = (int32_t)i;
        memcpy(lf + 4 * i, box + 4 * (int64_t)g, 16);
        lsc[i] = score[g];
        k2[i] = (dt_key){((unsigned long long)p << 31) | (unsigned)box[4 * (int64_t)g], i, g};
        tl[i] = g;
        ss[i] = (int32_t)leaf_off[p];
        sl[i] = (int32_t)(leaf_off[p + 1] - leaf_off[p]);
        sn[i] = 0;
    }
    qsort(k2, (size_t)L, sizeof(dt_key), dt_key_cmp);
    for (int64_t k = 0; k < L; ++k) { /* k_dt_qinit */
        const int32_t g = k2[k].v;
        ql[k] = g;
        qpos[g] = (int32_t)k;
        memcpy(qbox + 4 * k, box + 4 * (int64_t)g, 16);
        qtp[k] = tpos[g];
    }
    int levels = 0;
    for (int64_t n = maxnl; n > 1; n -= n / 2)
        ++levels;
    for (int d = 0; d < levels; ++d) {
        const int dim = d & 1;
        int32_t *D = dim ? tl : ql, *O = dim ? ql : tl;
        for (int64_t i = 0; i < L; ++i)
            if (sl[i] >= 2)
                posd[D[i]] = (int32_t)i;
        for (int64_t i = 0; i < L; ++i)
            flag[i] = sl[i] >= 2 && posd[O[i]] < ss[i] + (sl[i] >> 1);
        for (int64_t i = 0, run = 0; i < L; ++i) {
            excl[i] = (int32_t)run;
            run += flag[i];
        }
        for (int64_t i = 0; i < L; ++i) { /* k_dt_split */
            const int32_t s = ss[i], len = sl[i], e = O[i];
            if (len < 2) {
                spare[i] = e;
                continue;
            }
            const int32_t half = len >> 1, hb = excl[i] - excl[s];
            spare[flag[i] ? s + hb : s + half + ((int32_t)i - s - hb)] = e;
            const int32_t v = sn[i], lo = v + 2 * (len - half);
            if (i == s) {
                const int32_t *bb = box + 4 * (int64_t)D[s + half - 1];
                const int64_t nv = node_off[pidx[i]] + v;
                na[4 * nv + 2] = dim ? bb[2] : bb[0];
                na[4 * nv + 3] = lo;
                nb[2 * nv] = v + 2 * len - 1;
                nb[2 * nv + 1] = dim;
                ndep[nv] = d;
                ndl[nv] = lo - v;
            }
            if ((int32_t)i - s < half) {
                sl[i] = half;
                sn[i] = lo;
            } else {
                ss[i] = s + half;
                sl[i] = len - half;
                sn[i] = v + 1;
            }
        }
        if (dim)
            ql = spare;
        else
            tl = spare;
        spare = O;
    }
    for (int64_t i = 0; i < L; ++i) { /* k_dt_leafnodes */
        const int32_t g = ql[i];
        if (sl[i] != 1 || tl[i] != g) {
            fprintf(stderr, "gac_chain_dp_blocks (CPU stand-in): bad leaf segment at %lld\n", (long long)i);
            abort();
        }
        const int64_t nv = node_off[pidx[i]] + sn[i];
        const int32_t *b = box + 4 * (int64_t)g;
        na[4 * nv] = b[1];
        na[4 * nv + 1] = b[3];
        na[4 * nv + 2] = b[0];
        na[4 * nv + 3] = b[2];
        nb[2 * nv] = sn[i] + 1;
        nb[2 * nv + 1] = ~(int32_t)(tpos[g] - leaf_off[pidx[i]]);
        ndep[nv] = -1;
        lnode[tpos[g]] = sn[i];
    }
    for (int d = levels - 1; d >= 0; --d) /* k_dt_max */
        for (int64_t v = 0; v < N; ++v)
            if (ndep[v] == d) {
                const int32_t *a = na + 4 * (v + ndl[v]), *b = na + 4 * (v + 1);
                na[4 * v] = a[0] > b[0] ? a[0] : b[0];
                na[4 * v + 1] = a[1] > b[1] ? a[1] : b[1];
            }
    /* k_dt_path */
    int64_t *poff = malloc((size_t)(L + 1) * 8), pcap = L * 24 + 64, np_ = 0;
    int32_t *path = malloc((size_t)pcap * 4);
    for (int64_t i = 0; i < L; ++i) {
        poff[i] = np_;
        const int64_t base = node_off[pidx[i]];
        int32_t st[64];
        int sp = 0;
        st[sp++] = 0;
        while (sp > 0) {
            const int32_t v = st[--sp];
            if (np_ == pcap) {
                pcap *= 2;
                path = realloc(path, (size_t)pcap * 4);
            }
            path[np_++] = v;
            if (nb[2 * (base + v) + 1] >= 0) {
                const int32_t coord = nb[2 * (base + v) + 1] == 0 ? lf[4 * i] : lf[4 * i + 2];
                const int32_t cut = na[4 * (base + v) + 2];
                if (sp + 2 > 64)
                    abort();
                if (coord <= cut)
                    st[sp++] = na[4 * (base + v) + 3];
                if (coord >= cut)
                    st[sp++] = v + 1;
            }
        }
    }
    poff[L] = np_;
    /* k_dt_maxsz + k_dt_ovl */
    int64_t *ooff = NULL;
    int32_t *ov = NULL;
    if (fast) {
        int32_t *msz = calloc((size_t)(P + 1), 4);
        for (int64_t i = 0; i < L; ++i)
            if (lf[4 * i + 3] - lf[4 * i + 2] > msz[pidx[i]])
                msz[pidx[i]] = lf[4 * i + 3] - lf[4 * i + 2];
        int64_t ocap = L + 64, no = 0;
        ooff = malloc((size_t)(L + 1) * 8);
        ov = malloc((size_t)ocap * 4);
        int32_t *buf = malloc(1025 * 4);
        for (int64_t i = 0; i < L; ++i) {
            ooff[i] = no;
            const int32_t p = pidx[i], lq = lf[4 * i], lt = lf[4 * i + 2], m = msz[p];
            const int64_t lo_i = leaf_off[p];
            int n = 0, ovf = 0;
            for (int64_t j = i - 1; j >= lo_i && !ovf; --j) {
                const int32_t *b = lf + 4 * j;
                if (!(b[2] > lt - m))
                    break;
                if (b[2] >= lt || b[0] >= lq)
                    continue;
                if (lq - b[1] >= 0 && lt - b[3] >= 0)
                    continue;
                if (n == ov_cap)
                    ovf = 1;
                else
                    buf[n++] = lnode[j];
            }
            for (int64_t j = (int64_t)qpos[tord[i]] - 1; j >= lo_i && !ovf; --j) {
                const int32_t *b = qbox + 4 * j;
                if (!(b[0] > lq - m))
                    break;
                if (b[2] >= lt || b[0] >= lq || qtp[j] >= i)
                    continue;
                const int32_t dq = lq - b[1], dt = lt - b[3];
                if ((dq >= 0 && dt >= 0) || dt < 0)
                    continue;
                if (n == ov_cap)
                    ovf = 1;
                else
                    buf[n++] = lnode[qtp[j]];
            }
            if (ovf) {
                buf[0] = -1;
                n = 1;
            }
            if (no + n > ocap) {
                ocap = 2 * (no + n) + 64;
                ov = realloc(ov, (size_t)ocap * 4);
            }
            memcpy(ov + no, buf, (size_t)n * 4);
            no += n;
        }
        ooff[L] = no;
        free(buf);
        free(msz);
    }
    int64_t *lt_ = malloc((size_t)(L + 1) * 8);
    int32_t *lp = malloc((size_t)(L + 1) * 4);
    const int rc = gac_chain_dp_ex(c, P, t_seq, q_seq, q_strand, node_off, na, nb, leaf_off, lf, lsc,
                                   lnode, poff, path, ooff, ov, fast ? lin_k : 0, min_entry, lt_, lp);
    if (getenv("GAC_DT_DUMP")) { /* (debug: as the device's dump) */
        const char *dd = getenv("GAC_DT_DUMP");
        const struct { const char *n; const void *p; size_t b; } F[] = {
            {"leaf_off", leaf_off, (size_t)(P + 1) * 8}, {"lf", lf, (size_t)L * 16},
            {"lnode", lnode, (size_t)L * 4}, {"na", na, (size_t)N * 16}, {"nb", nb, (size_t)N * 8},
            {"poff", poff, (size_t)(L + 1) * 8}, {"path", path, (size_t)poff[L] * 4},
            {"ooff", ooff, fast ? (size_t)(L + 1) * 8 : 0}, {"ov", ov, fast ? (size_t)ooff[L] * 4 : 0},
            {"lf_total", lt_, (size_t)L * 8}, {"lf_pred", lp, (size_t)L * 4}};
        for (size_t k = 0; k < sizeof(F) / sizeof(F[0]); ++k) {
            char fn[4096];
            snprintf(fn, sizeof(fn), "%s/%s", dd, F[k].n);
            FILE *o = fopen(fn, "wb");
            if (o) {
                fwrite(F[k].p, 1, F[k].b, o);
                fclose(o);
            }
        }
    }
    for (int64_t g = 0; g < B; ++g) { /* k_dt_out_init + k_dt_out */
        total[g] = score[g];
        pred[g] = -1;
    }
    for (int64_t i = 0; i < L; ++i) {
        const int32_t g = tord[i], p = pidx[i];
        tord_out[i] = (int32_t)(g - blk_off[p]);
        total[g] = lt_[i];
        pred[g] = lp[i] < 0 ? -1
                            : (int32_t)(tord[leaf_off[p] + ~nb[2 * (node_off[p] + lp[i]) + 1]] - blk_off[p]);
    }
    free(k1);
    free(k2);
    free(node_off);
    free(tord);
    free(pidx);
    free(tpos);
    free(qpos);
    free(posd);
    free(lf);
    free(lsc);
    free(ql);
    free(tl);
    free(spare);
    free(ss);
    free(sl);
    free(sn);
    free(flag);
    free(excl);
    free(qbox);
    free(qtp);
    free(lnode);
    free(na);
    free(nb);
    free(ndep);
    free(ndl);
    free(poff);
    free(path);
    free(ooff);
    free(ov);
    free(lt_);
    free(lp);
    return rc;
}

/* gac_kd_trees: kdTreeMake (chainBlock.c:166-205) restated recursively --
 * the leaf sorts of gac_chain_dp_blocks' stand-in above, then kdBuild
 * (:124-164) in pre-order with the hi child first -- into the host layout */
typedef struct stub_kd {
    const int32_t *box; /* the pair's blocks */
    int32_t *nodes, *lnode, *hit, *tmp;
    int32_t nn;
} stub_kd;

static int32_t stub_kd_build(stub_kd *K, int32_t *Q, int32_t *T, int32_t n, int dim) {
    const int32_t id = K->nn++;
    int32_t *nd = K->nodes + 6 * id;
    if (n == 1) {
        const int32_t l = Q[0];
        const int32_t *b = K->box + 4 * l;
        nd[0] = b[0], nd[1] = b[2], nd[2] = l, nd[3] = 0, nd[4] = b[1], nd[5] = b[3];
        K->lnode[l] = id;
        return id;
    }
    const int32_t half = n / 2;
    int32_t *D = dim == 0 ? Q : T, *O = dim == 0 ? T : Q;
    for (int32_t i = 0; i < n; ++i)
        K->hit[D[i]] = i < half;
    int32_t k = 0;
    for (int32_t i = 0; i < n; ++i)
        if (K->hit[O[i]])
            K->tmp[k++] = O[i];
    for (int32_t i = 0; i < n; ++i)
        if (!K->hit[O[i]])
            K->tmp[k++] = O[i];
    memcpy(O, K->tmp, (size_t)n * 4);
    const int32_t *mb = K->box + 4 * D[half - 1];
    const int32_t cut = dim == 0 ? mb[0] : mb[2];
    const int32_t hi = stub_kd_build(K, Q + half, T + half, n - half, 1 - dim);
    const int32_t lo = stub_kd_build(K, Q, T, half, 1 - dim);
    nd = K->nodes + 6 * id;
    const int32_t *a = K->nodes + 6 * lo, *b = K->nodes + 6 * hi;
    nd[0] = lo, nd[1] = hi, nd[2] = -1, nd[3] = cut;
    nd[4] = a[4] > b[4] ? a[4] : b[4];
    nd[5] = a[5] > b[5] ? a[5] : b[5];
    return id;
}

int gac_kd_trees(gac_ctx *c, int64_t P, const int32_t *t_seq, const int32_t *q_seq,
                 const uint8_t *q_strand, const int64_t *blk_off, const int32_t *box,
                 int64_t *leaf_off, int32_t *const *tord, int32_t *const *qord,
                 int32_t *const *lnode, int32_t *const *nodes) {
    (void)c, (void)t_seq, (void)q_seq, (void)q_strand;
    leaf_off[0] = 0;
    for (int64_t p = 0; p < P; ++p) {
        const int64_t b0 = blk_off[p];
        const int32_t nb = (int32_t)(blk_off[p + 1] - b0);
        const int32_t *bx = box + 4 * b0;
        dt_key *k = malloc((size_t)(nb ? nb : 1) * sizeof(dt_key));
        int32_t nl = 0;
        for (int32_t r = 0; r < nb; ++r) { /* reverse input order (slAddHead) */
            const int32_t g = nb - 1 - r;
            lnode[p][g] = -1;
            if (bx[4 * g + 2] != bx[4 * g + 3])
                k[nl++] = (dt_key){(unsigned long long)(uint32_t)bx[4 * g + 2], r, g};
        }
        qsort(k, (size_t)nl, sizeof(dt_key), dt_key_cmp);
        for (int32_t i = 0; i < nl; ++i)
            tord[p][i] = k[i].v;
        for (int32_t i = 0; i < nl; ++i)
            k[i] = (dt_key){(unsigned long long)(uint32_t)bx[4 * tord[p][i]], i, tord[p][i]};
        qsort(k, (size_t)nl, sizeof(dt_key), dt_key_cmp);
        for (int32_t i = 0; i < nl; ++i)
            qord[p][i] = k[i].v;
        free(k);
        leaf_off[p + 1] = leaf_off[p] + nl;
        if (!nl)
            continue;
        stub_kd K = {bx, nodes[p], lnode[p], calloc((size_t)nb, 4), malloc((size_t)nl * 4), 0};
        int32_t *Q = malloc((size_t)nl * 4), *T = malloc((size_t)nl * 4);
        memcpy(Q, qord[p], (size_t)nl * 4);
        memcpy(T, tord[p], (size_t)nl * 4);
        stub_kd_build(&K, Q, T, nl, 0);
        free(Q);
        free(T);
        free(K.hit);
        free(K.tmp);
    }
    return GAC_OK;
}
