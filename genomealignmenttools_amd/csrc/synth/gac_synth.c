/* gac_synth.c -- seeded whole-genome synthetic chain sets (SURVEY.md §8(d)
 * config C5) for bench.py and the full-length GPU parity tests.  Test and
 * bench infrastructure: no product code calls it.
 *
 *   gac_synth c5 OUTDIR [-seed=S] [-chains=N] [-scale=X] [-minSize=M]
 *                [-sizesDir=D] [-threads=T]
 *
 * Writes OUTDIR/{t,q}.2bit, {t,q}.sizes, in.chain (score-sorted, ids 1..n),
 * chains.bin (the same chains as arrays, for bench.py's kernel legs) and
 * info.json.  The model is synth.py's C2/C5 chain model (make_chains):
 *   - target = every hg38 sequence, query = every mm10 sequence (sizes from
 *     D/hg38.chrom.sizes, D/mm10.chrom.sizes), scaled by X (not below M);
 *   - uniform random bases, 0.5 % N in runs of mean 20 kb (stored as T, as
 *     in .2bit files);
 *   - chains per target sequence in proportion to its length; per chain
 *     20 % spurious (1-5 blocks), else power-law blocks (alpha 1.8, up to
 *     1e5); query sequence by length; 50 % '-' strand; geometric blocks
 *     (mean 40); gaps 70 % < 30 bp, 28 % 30 bp-10 kb, 2 % 10 kb-1 Mb, on the
 *     target, the query or both; a chain keeps the prefix of its blocks that
 *     spans at most half of each sequence;
 *   - query bases under every block := the target's with 12 % substitutions
 *     (transitions 2/3), reverse-complemented for '-' chains;
 *   - header score = blastz-matrix block scores minus approximate loose gap
 *     costs (rounded; only the sort order and the netting stop depend on it).
 * Every random draw comes from a stream seeded by (seed, purpose, index), so
 * the output does not depend on the thread count. */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

static void die(const char *fmt, const char *a) {
    fprintf(stderr, "gac_synth: ");
    fprintf(stderr, fmt, a);
    fputc('\n', stderr);
    exit(1);
}

/* ---------------------------------------------------------------- RNG */
typedef struct { uint64_t s[4]; } rng_t;

static uint64_t splitmix(uint64_t *x) {
    uint64_t z = (*x += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static void rng_seed(rng_t *r, uint64_t seed, uint64_t purpose, uint64_t index) {
    uint64_t x = seed * 0x2545f4914f6cdd1dull ^ (purpose << 48) ^ index;
    for (int i = 0; i < 4; ++i)
        r->s[i] = splitmix(&x);
}

static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

static inline uint64_t next64(rng_t *r) { /* xoshiro256** */
    uint64_t *s = r->s;
    const uint64_t out = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return out;
}

static inline double unif(rng_t *r) { return (double)(next64(r) >> 11) * 0x1.0p-53; }

static inline int64_t geometric(rng_t *r, double p) { /* trials until success, >= 1 */
    const double u = 1.0 - unif(r);                   /* (0, 1] */
    return (int64_t)floor(log(u) / log1p(-p)) + 1;
}

static inline int64_t uniform_int(rng_t *r, int64_t lo, int64_t hi) { /* [lo, hi) */
    return lo + (int64_t)(unif(r) * (double)(hi - lo));
}

enum { P_GENOME = 1, P_NRUNS, P_CHAIN, P_MUTATE };

/* ---------------------------------------------------------------- threads */
static int g_threads = 16;

static void run_threads(void *(*fn)(void *), void *arg) {
    pthread_t th[256];
    int n = g_threads > 256 ? 256 : g_threads;
    for (int i = 0; i < n; ++i)
        if (pthread_create(&th[i], NULL, fn, arg) != 0)
            die("%s", "pthread_create failed");
    for (int i = 0; i < n; ++i)
        pthread_join(th[i], NULL);
}

/* ---------------------------------------------------------------- genomes */
typedef struct {
    char **names;
    int64_t *size;
    int n;
    uint8_t **packed; /* .2bit payload per sequence (2 bits/base, MSB first) */
    int64_t **nstart, **nlen;
    int *nn;
} genome_t;

static void read_sizes(const char *path, double scale, int64_t min_size, genome_t *g) {
    FILE *f = fopen(path, "r");
    if (!f)
        die("can't open %s", path);
    char name[1024];
    long long v;
    int cap = 1024;
    memset(g, 0, sizeof(*g));
    g->names = malloc(cap * sizeof(char *));
    g->size = malloc(cap * 8);
    while (fscanf(f, "%1023s %lld", name, &v) == 2) {
        if (g->n == cap) {
            cap *= 2;
            g->names = realloc(g->names, cap * sizeof(char *));
            g->size = realloc(g->size, cap * 8);
        }
        int64_t s = v;
        if (scale != 1.0) {
            s = (int64_t)((double)v * scale);
            if (s < min_size)
                s = min_size;
        }
        g->names[g->n] = strdup(name);
        g->size[g->n++] = s;
    }
    fclose(f);
    if (!g->n)
        die("no sequences in %s", path);
}

typedef struct {
    genome_t *g;
    uint64_t seed, side;
    _Atomic int64_t next; /* (sequence, 1 MB chunk) work items */
    int64_t *chunk_off;   /* first work item of each sequence */
} gen_job;

static void *gen_thread(void *arg) {
    gen_job *J = arg;
    genome_t *g = J->g;
    const int64_t total = J->chunk_off[g->n];
    for (;;) {
        const int64_t w = atomic_fetch_add(&J->next, 1);
        if (w >= total)
            break;
        int lo = 0, hi = g->n - 1;
        while (lo < hi) {
            const int mid = (lo + hi + 1) / 2;
            if (J->chunk_off[mid] <= w) lo = mid;
            else hi = mid - 1;
        }
        const int64_t c = w - J->chunk_off[lo], nbytes = (g->size[lo] + 3) / 4;
        const int64_t a = c << 20, b = (a + (1 << 20)) < nbytes ? a + (1 << 20) : nbytes;
        rng_t r;
        rng_seed(&r, J->seed, P_GENOME, (J->side << 40) ^ ((uint64_t)lo << 24) ^ (uint64_t)c);
        uint8_t *p = g->packed[lo];
        for (int64_t i = a; i < b; i += 8) {
            uint64_t x = next64(&r);
            for (int k = 0; k < 8 && i + k < b; ++k, x >>= 8)
                p[i + k] = (uint8_t)x;
        }
    }
    return NULL;
}

static inline int get_code(const uint8_t *p, int64_t i) { return (p[i >> 2] >> (6 - 2 * (i & 3))) & 3; }

static inline void set_code(uint8_t *p, int64_t i, int c) {
    const int sh = 6 - 2 * (int)(i & 3);
    p[i >> 2] = (uint8_t)((p[i >> 2] & ~(3 << sh)) | (c << sh));
}

static int cmp_i64(const void *a, const void *b) {
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    return x < y ? -1 : x > y;
}

static void make_genome(genome_t *g, uint64_t seed, uint64_t side) {
    g->packed = malloc(g->n * sizeof(uint8_t *));
    g->nstart = malloc(g->n * sizeof(int64_t *));
    g->nlen = malloc(g->n * sizeof(int64_t *));
    g->nn = malloc(g->n * sizeof(int));
    gen_job J = {g, seed, side, 0, malloc((g->n + 1) * 8)};
    J.chunk_off[0] = 0;
    for (int i = 0; i < g->n; ++i) {
        const int64_t nbytes = (g->size[i] + 3) / 4;
        g->packed[i] = malloc(nbytes + 8);
        J.chunk_off[i + 1] = J.chunk_off[i] + ((nbytes + (1 << 20) - 1) >> 20);
    }
    atomic_init(&J.next, 0);
    run_threads(gen_thread, &J);
    free(J.chunk_off);
    /* N runs: 0.5 % of the bases in runs of mean 20 kb, merged, stored as T */
    for (int i = 0; i < g->n; ++i) {
        const int64_t size = g->size[i];
        rng_t r;
        rng_seed(&r, seed, P_NRUNS, (side << 32) ^ (uint64_t)i);
        int64_t k = (int64_t)((double)size * 0.005 / 20000.0);
        if (k < 1)
            k = 1;
        int64_t *st = malloc(k * 8), *en = malloc(k * 8);
        for (int64_t j = 0; j < k; ++j)
            st[j] = uniform_int(&r, 0, size);
        qsort(st, k, 8, cmp_i64);
        int64_t m = 0;
        for (int64_t j = 0; j < k; ++j) {
            int64_t e = st[j] + geometric(&r, 1.0 / 20000.0);
            if (e > size)
                e = size;
            if (m && st[j] <= en[m - 1]) {
                if (e > en[m - 1])
                    en[m - 1] = e;
            } else {
                st[m] = st[j];
                en[m++] = e;
            }
        }
        g->nn[i] = (int)m;
        g->nstart[i] = st;
        g->nlen[i] = en;
        for (int64_t j = 0; j < m; ++j) {
            for (int64_t b = st[j]; b < en[j]; ++b)
                set_code(g->packed[i], b, 0);
            en[j] -= st[j]; /* lengths from here on */
        }
    }
}

static void write_u32(FILE *f, uint32_t v) { fwrite(&v, 4, 1, f); }

static void write_2bit(const genome_t *g, const char *path) {
    FILE *f = fopen(path, "wb");
    if (!f)
        die("can't write %s", path);
    write_u32(f, 0x1A412743);
    write_u32(f, 0);
    write_u32(f, (uint32_t)g->n);
    write_u32(f, 0);
    uint64_t off = 16;
    for (int i = 0; i < g->n; ++i)
        off += 1 + strlen(g->names[i]) + 4;
    for (int i = 0; i < g->n; ++i) {
        const uint8_t nl = (uint8_t)strlen(g->names[i]);
        fwrite(&nl, 1, 1, f);
        fwrite(g->names[i], 1, nl, f);
        if (off >= (1ull << 32))
            die("%s: version-0 .2bit limited to 4 GB", path);
        write_u32(f, (uint32_t)off);
        off += 4 + 4 + 8ull * g->nn[i] + 4 + 4 + (g->size[i] + 3) / 4;
    }
    for (int i = 0; i < g->n; ++i) {
        write_u32(f, (uint32_t)g->size[i]);
        write_u32(f, (uint32_t)g->nn[i]);
        for (int j = 0; j < g->nn[i]; ++j)
            write_u32(f, (uint32_t)g->nstart[i][j]);
        for (int j = 0; j < g->nn[i]; ++j)
            write_u32(f, (uint32_t)g->nlen[i][j]);
        write_u32(f, 0); /* mask blocks */
        write_u32(f, 0); /* reserved */
        fwrite(g->packed[i], 1, (g->size[i] + 3) / 4, f);
    }
    if (fclose(f) != 0)
        die("write error on %s", path);
}

static void write_sizes(const genome_t *g, const char *path) {
    FILE *f = fopen(path, "w");
    if (!f)
        die("can't write %s", path);
    for (int i = 0; i < g->n; ++i)
        fprintf(f, "%s\t%lld\n", g->names[i], (long long)g->size[i]);
    if (fclose(f) != 0)
        die("write error on %s", path);
}

/* ---------------------------------------------------------------- chains */
typedef struct {
    int64_t n, nb;
    int32_t *tseq, *qseq, *tstart, *tend, *qstart, *qend;
    uint8_t *strand;
    int64_t *off; /* [n + 1] */
    int32_t *bt, *bq, *bs;
    double *score;
} chains_t;

static const genome_t *G_T, *G_Q;
static uint64_t g_seed;
static double *g_qcum; /* cumulative query sizes (query choice by length) */

static int64_t gap_mixture(rng_t *r) {
    const double u = unif(r);
    if (u < 0.70)
        return uniform_int(r, 1, 30);
    if (u < 0.98)
        return (int64_t)exp(log(30.0) + unif(r) * (log(10000.0) - log(30.0)));
    return (int64_t)exp(log(10000.0) + unif(r) * (log(1e6) - log(10000.0)));
}

/* one chain: blocks into (bt, bq, bs) if non-NULL; returns the block count.
 * Target sequence ts_i is given; everything else is drawn from the chain's
 * stream. */
static int64_t make_chain(int64_t ci, int ts_i, int32_t *qseq, uint8_t *strand, int32_t *bt,
                          int32_t *bq, int32_t *bs, int32_t *tspan, int32_t *qspan) {
    rng_t r;
    rng_seed(&r, g_seed, P_CHAIN, (uint64_t)ci);
    const int64_t tsize = G_T->size[ts_i];
    int64_t nb;
    const int spur = unif(&r) < 0.2;
    if (spur) {
        nb = uniform_int(&r, 1, 6);
    } else {
        const double a1 = 1.0 - 1.8, u = unif(&r);
        nb = (int64_t)floor(pow(1.0 + u * (pow(100000.0, a1) - 1.0), 1.0 / a1));
        if (nb < 1)
            nb = 1;
        if (nb > 100000)
            nb = 100000;
    }
    const double x = unif(&r) * g_qcum[G_Q->n];
    int lo = 0, hi = G_Q->n - 1;
    while (lo < hi) {
        const int mid = (lo + hi) / 2;
        if (g_qcum[mid + 1] > x) hi = mid;
        else lo = mid + 1;
    }
    const int qs_i = lo;
    const int64_t qsize = G_Q->size[qs_i];
    const int minus = unif(&r) < 0.5;
    const double tlim = 0.5 * (double)tsize, qlim = 0.5 * (double)qsize;
    int64_t ct = 0, cq = 0, kept = 0, prev_dt = 0, prev_dq = 0;
    for (int64_t b = 0; b < nb; ++b) {
        const int64_t size = geometric(&r, 1.0 / 40.0);
        const int64_t g1 = gap_mixture(&r), g2 = gap_mixture(&r);
        const int mode = (int)uniform_int(&r, 0, 3);
        const int64_t dt = mode == 1 ? 0 : g1, dq = mode == 0 ? 0 : (mode == 1 ? g1 : g2);
        const int64_t nt = ct + prev_dt + size, nq = cq + prev_dq + size;
        if (b > 0 && ((double)nt > tlim || (double)nq > qlim))
            break;
        if (bs) {
            bt[kept] = (int32_t)(ct + prev_dt);
            bq[kept] = (int32_t)(cq + prev_dq);
            bs[kept] = (int32_t)size;
        }
        ct = nt;
        cq = nq;
        prev_dt = dt;
        prev_dq = dq;
        ++kept;
    }
    if (bs) { /* place the chain: uniform start in what is left of each sequence */
        int64_t t0 = (int64_t)(unif(&r) * (double)(tsize - ct > 0 ? tsize - ct : 0));
        int64_t q0 = (int64_t)(unif(&r) * (double)(qsize - cq > 0 ? qsize - cq : 0));
        for (int64_t k = 0; k < kept; ++k) {
            bt[k] += (int32_t)t0;
            bq[k] += (int32_t)q0;
        }
        *qseq = qs_i;
        *strand = (uint8_t)minus;
        tspan[0] = (int32_t)t0;
        tspan[1] = (int32_t)(t0 + ct);
        qspan[0] = (int32_t)q0;
        qspan[1] = (int32_t)(q0 + cq);
    }
    return kept;
}

typedef struct {
    chains_t *C;
    const int32_t *tseq;
    _Atomic int64_t next;
    int pass;
} chain_job;

static void *chain_thread(void *arg) {
    chain_job *J = arg;
    chains_t *C = J->C;
    for (;;) {
        const int64_t a = atomic_fetch_add(&J->next, 4096);
        if (a >= C->n)
            break;
        const int64_t b = a + 4096 < C->n ? a + 4096 : C->n;
        for (int64_t i = a; i < b; ++i) {
            if (J->pass == 0) {
                C->off[i + 1] = make_chain(i, J->tseq[i], NULL, NULL, NULL, NULL, NULL, NULL, NULL);
            } else {
                int32_t tsp[2], qsp[2];
                const int64_t o = C->off[i];
                make_chain(i, J->tseq[i], &C->qseq[i], &C->strand[i], C->bt + o, C->bq + o,
                           C->bs + o, tsp, qsp);
                C->tstart[i] = tsp[0];
                C->tend[i] = tsp[1];
                C->qstart[i] = qsp[0];
                C->qend[i] = qsp[1];
            }
        }
    }
    return NULL;
}

/* blastz default matrix in 2bit code order (T, C, A, G), [q][t] */
static const int k_mat[4][4] = {
    {91, -114, -31, -123}, {-114, 100, -125, -31}, {-31, -125, 100, -114}, {-123, -31, -114, 91}};

/* kent loose gap table (gapCalc.c:51-57): approximate header scores only */
static const double k_pos[11] = {1, 2, 3, 11, 111, 2111, 12111, 32111, 72111, 152111, 252111};
static const double k_q[11] = {325, 360, 400, 450, 600, 1100, 3600, 7600, 15600, 31600, 56600};
static const double k_b[11] = {625, 660, 700, 750, 900, 1400, 4000, 8000, 16000, 32000, 57000};

static double interp(const double *v, double d, double last) {
    if (d >= k_pos[10])
        return last + 0.25 * (d - k_pos[10]);
    if (d <= k_pos[0])
        return v[0];
    int i = 1;
    while (k_pos[i] < d)
        ++i;
    return v[i - 1] + (v[i] - v[i - 1]) * (d - k_pos[i - 1]) / (k_pos[i] - k_pos[i - 1]);
}

static double approx_gap(int64_t dq, int64_t dt) {
    if (dq > 0 && dt > 0)
        return interp(k_b, (double)(dq + dt), 57000);
    return interp(k_q, (double)(dq > dt ? dq : dt), 56600);
}

typedef struct {
    chains_t *C;
    const int64_t *qoff, *qlist; /* chains per query sequence, in chain order */
    const int *qorder;           /* queries, largest first */
    _Atomic int next;
} mut_job;

static uint8_t g_xor[256];

static void *mutate_thread(void *arg) {
    mut_job *J = arg;
    chains_t *C = J->C;
    for (;;) {
        const int w = atomic_fetch_add(&J->next, 1);
        if (w >= G_Q->n)
            break;
        const int qi = J->qorder[w];
        uint8_t *qp = G_Q->packed[qi];
        const int64_t qsize = G_Q->size[qi];
        for (int64_t k = J->qoff[qi]; k < J->qoff[qi + 1]; ++k) {
            const int64_t c = J->qlist[k];
            rng_t r;
            rng_seed(&r, g_seed, P_MUTATE, (uint64_t)c);
            const uint8_t *tp = G_T->packed[C->tseq[c]];
            const int minus = C->strand[c];
            double score = 0;
            uint64_t bits = 0;
            int left = 0;
            for (int64_t b = C->off[c]; b < C->off[c + 1]; ++b) {
                int64_t bsc = 0;
                const int64_t t0 = C->bt[b], q0 = C->bq[b], n = C->bs[b];
                for (int64_t j = 0; j < n; ++j) {
                    if (!left) {
                        bits = next64(&r);
                        left = 8;
                    }
                    const int tc = get_code(tp, t0 + j);
                    const int q = tc ^ g_xor[bits & 255];
                    bits >>= 8;
                    --left;
                    const int64_t rp = q0 + j;
                    if (minus)
                        set_code(qp, qsize - 1 - rp, q ^ 2);
                    else
                        set_code(qp, rp, q);
                    bsc += k_mat[q][tc];
                }
                score += (double)bsc;
                if (b + 1 < C->off[c + 1])
                    score -= approx_gap(C->bq[b + 1] - (q0 + n), C->bt[b + 1] - (t0 + n));
            }
            C->score[c] = nearbyint(score);
        }
    }
    return NULL;
}

/* stable descending sort by score */
static const double *g_sort_score;
static int cmp_score(const void *a, const void *b) {
    const int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
    const double sx = g_sort_score[x], sy = g_sort_score[y];
    if (sx != sy)
        return sx < sy ? 1 : -1;
    return x < y ? -1 : x > y;
}

/* ---------------------------------------------------------------- output */
typedef struct {
    const chains_t *C;
    const int64_t *order;
    char **buf;
    size_t *len;
    int64_t nchunks, per;
    _Atomic int64_t next;
} fmt_job;

static char *put_i64(char *p, int64_t v) {
    char t[24];
    int n = 0;
    const int neg = v < 0;
    uint64_t u = neg ? (uint64_t)(-v) : (uint64_t)v;
    do {
        t[n++] = (char)('0' + u % 10);
        u /= 10;
    } while (u);
    if (neg)
        *p++ = '-';
    while (n)
        *p++ = t[--n];
    return p;
}

static void *fmt_thread(void *arg) {
    fmt_job *J = arg;
    const chains_t *C = J->C;
    for (;;) {
        const int64_t k = atomic_fetch_add(&J->next, 1);
        if (k >= J->nchunks)
            break;
        const int64_t a = k * J->per, b = a + J->per < C->n ? a + J->per : C->n;
        size_t cap = 0;
        for (int64_t s = a; s < b; ++s) {
            const int64_t i = J->order[s];
            cap += 200 + 36 * (size_t)(C->off[i + 1] - C->off[i]);
        }
        char *buf = malloc(cap), *p = buf;
        for (int64_t s = a; s < b; ++s) {
            const int64_t i = J->order[s];
            p += sprintf(p, "chain %1.0f %s %lld + %d %d %s %lld %c %d %d %lld\n", C->score[i],
                         G_T->names[C->tseq[i]], (long long)G_T->size[C->tseq[i]], C->tstart[i],
                         C->tend[i], G_Q->names[C->qseq[i]], (long long)G_Q->size[C->qseq[i]],
                         C->strand[i] ? '-' : '+', C->qstart[i], C->qend[i], (long long)(s + 1));
            for (int64_t bk = C->off[i]; bk < C->off[i + 1]; ++bk) {
                p = put_i64(p, C->bs[bk]);
                if (bk + 1 < C->off[i + 1]) {
                    *p++ = '\t';
                    p = put_i64(p, (int64_t)C->bt[bk + 1] - (C->bt[bk] + C->bs[bk]));
                    *p++ = '\t';
                    p = put_i64(p, (int64_t)C->bq[bk + 1] - (C->bq[bk] + C->bs[bk]));
                    *p++ = '\n';
                } else {
                    *p++ = '\n';
                    *p++ = '\n';
                }
            }
        }
        J->buf[k] = buf;
        J->len[k] = (size_t)(p - buf);
    }
    return NULL;
}

static void fwrite_all(FILE *f, const void *p, size_t n, const char *path) {
    if (n && fwrite(p, 1, n, f) != n)
        die("write error on %s", path);
}

static char *path_in(const char *dir, const char *name) {
    char *p = malloc(strlen(dir) + strlen(name) + 2);
    sprintf(p, "%s/%s", dir, name);
    return p;
}

/* ---------------------------------------------------------------- C4 (PSL) */
/* n_blocks PSL blocks over nt x nq chromosome pairs x 2
 * strands, blocks per pair by a power law (alpha 1.2 over a seeded
 * permutation of the pairs, at least 50), 80 % of each pair's blocks on
 * planted collinear paths of ~200 blocks (geometric sizes of mean 50 capped
 * at 500; gaps 80 % 1-59 bp, 20 % 60-4999 bp on the target, the query or
 * both, query gaps jittered by -20..19), the query bases under them := the
 * target's with 12 % substitutions (reverse-complemented on '-'), and 20 %
 * random blocks (20-299 bp anywhere).  Records: a path's blocks in runs of 5,
 * one record per random block, all records in a seeded random order (as
 * lastz job outputs are concatenated).  The same statistical model as
 * synth.py's psl_c4, drawn from per-pair streams (any thread count gives the
 * same bytes). */
enum { P_C4PAIRS = 9, P_C4PAIR, P_C4MUT, P_C4ORDER };

typedef struct {
    int ti, qi, strand;
    int64_t nb, ncol;      /* requested blocks, collinear share */
    int64_t n;             /* blocks kept: collinear (after the bounds filter) + random */
    int64_t nc;            /* collinear blocks kept (first nc of the arrays) */
    int32_t *bt, *bq, *bs; /* n blocks; collinear first, in path order */
    int32_t *path;         /* path of each collinear block */
    int64_t nrec, rec0;    /* records of this pair, first global record */
    int64_t *rec_first;    /* [nrec + 1]: first block of each record */
} c4pair;

typedef struct {
    c4pair *P;
    int np;
    int64_t tsize, qsize;
    _Atomic int next;
    const int *qorder_pairs; /* pairs grouped by query sequence (mutation pass) */
    const int *qoff;
} c4job;

static void *c4_pair_thread(void *arg) {
    c4job *J = arg;
    for (;;) {
        const int w = atomic_fetch_add(&J->next, 1);
        if (w >= J->np)
            break;
        c4pair *p = &J->P[w];
        rng_t r;
        rng_seed(&r, g_seed, P_C4PAIR, (uint64_t)w);
        const int64_t ncol = p->ncol, nr = p->nb - ncol;
        int64_t npath = ncol / 200;
        if (npath < 1)
            npath = 1;
        p->bt = malloc((size_t)(p->nb + 1) * 4);
        p->bq = malloc((size_t)(p->nb + 1) * 4);
        p->bs = malloc((size_t)(p->nb + 1) * 4);
        p->path = malloc((size_t)(ncol + 1) * 4);
        int64_t *lt = malloc((size_t)(ncol + 1) * 8), *lq = malloc((size_t)(ncol + 1) * 8);
        int32_t *sz = malloc((size_t)(ncol + 1) * 4);
        /* path k holds blocks [k*ncol/npath, (k+1)*ncol/npath): local offsets */
        int64_t k0 = 0;
        for (int64_t k = 0; k < npath; ++k) {
            const int64_t a = k0, b = (k + 1) * ncol / npath;
            int64_t ct = 0, cq = 0, pdt = 0, pdq = 0;
            for (int64_t i = a; i < b; ++i) {
                int64_t s = geometric(&r, 1.0 / 50.0);
                if (s > 500)
                    s = 500;
                const int mode = (int)uniform_int(&r, 0, 3);
                const int64_t g = unif(&r) < 0.8 ? uniform_int(&r, 1, 60) : uniform_int(&r, 60, 5000);
                int64_t dq = g + uniform_int(&r, -20, 20);
                if (dq < 1)
                    dq = 1;
                if (i > a) {
                    ct += pdt;
                    cq += pdq;
                }
                lt[i] = ct;
                lq[i] = cq;
                sz[i] = (int32_t)s;
                ct += s;
                cq += s;
                pdt = mode == 1 ? 0 : g;
                pdq = mode == 0 ? 0 : dq;
            }
            /* origin: uniform where the path fits */
            const int64_t rt = J->tsize - ct - 1 > 1 ? J->tsize - ct - 1 : 1;
            const int64_t rq = J->qsize - cq - 1 > 1 ? J->qsize - cq - 1 : 1;
            const int64_t t0 = (int64_t)(unif(&r) * (double)rt), q0 = (int64_t)(unif(&r) * (double)rq);
            for (int64_t i = a; i < b; ++i) {
                const int64_t bt = t0 + lt[i], bq = q0 + lq[i];
                if (bt + sz[i] < J->tsize && bq + sz[i] < J->qsize) {
                    p->bt[p->nc] = (int32_t)bt;
                    p->bq[p->nc] = (int32_t)bq;
                    p->bs[p->nc] = sz[i];
                    p->path[p->nc++] = (int32_t)k;
                }
            }
            k0 = b;
        }
        free(lt);
        free(lq);
        free(sz);
        p->n = p->nc;
        for (int64_t i = 0; i < nr; ++i, ++p->n) {
            p->bs[p->n] = (int32_t)uniform_int(&r, 20, 300);
            p->bt[p->n] = (int32_t)uniform_int(&r, 0, J->tsize - 400);
            p->bq[p->n] = (int32_t)uniform_int(&r, 0, J->qsize - 400);
        }
        /* records: collinear runs of 5 (cut at path changes), random singles */
        p->rec_first = malloc((size_t)(p->nc + nr + 2) * 8);
        p->nrec = 0;
        for (int64_t i = 0; i < p->nc; ++i)
            if (i == 0 || i % 5 == 0 || p->path[i] != p->path[i - 1])
                p->rec_first[p->nrec++] = i;
        for (int64_t i = p->nc; i < p->n; ++i)
            p->rec_first[p->nrec++] = i;
        p->rec_first[p->nrec] = p->n;
    }
    return NULL;
}

static const genome_t *C4T, *C4Q;

/* plant the collinear blocks' homology, one query sequence per work item
 * (its pairs in pair order), from per-pair mutation streams */
static void *c4_mut_thread(void *arg) {
    c4job *J = arg;
    for (;;) {
        const int w = atomic_fetch_add(&J->next, 1);
        if (w >= C4Q->n)
            break;
        uint8_t *qp = C4Q->packed[w];
        for (int k = J->qoff[w]; k < J->qoff[w + 1]; ++k) {
            const int pi = J->qorder_pairs[k];
            const c4pair *p = &J->P[pi];
            const uint8_t *tp = C4T->packed[p->ti];
            rng_t r;
            rng_seed(&r, g_seed, P_C4MUT, (uint64_t)pi);
            uint64_t bits = 0;
            int left = 0;
            for (int64_t b = 0; b < p->nc; ++b)
                for (int64_t j = 0; j < p->bs[b]; ++j) {
                    if (!left) {
                        bits = next64(&r);
                        left = 8;
                    }
                    const int q = get_code(tp, p->bt[b] + j) ^ g_xor[bits & 255];
                    bits >>= 8;
                    --left;
                    const int64_t rp = p->bq[b] + j;
                    if (p->strand)
                        set_code(qp, J->qsize - 1 - rp, q ^ 2);
                    else
                        set_code(qp, rp, q);
                }
        }
    }
    return NULL;
}

typedef struct {
    const c4pair *P;
    int np;
    const int64_t *perm; /* output position -> global record */
    int64_t nrec, per, nchunks;
    int64_t tsize, qsize;
    char **buf;
    size_t *len;
    _Atomic int64_t next;
} c4fmt;

static void *c4_fmt_thread(void *arg) {
    c4fmt *J = arg;
    for (;;) {
        const int64_t k = atomic_fetch_add(&J->next, 1);
        if (k >= J->nchunks)
            break;
        const int64_t a = k * J->per, b = a + J->per < J->nrec ? a + J->per : J->nrec;
        size_t cap = 0;
        int *pidx = malloc((size_t)(b - a + 1) * sizeof(int));
        for (int64_t s = a; s < b; ++s) {
            const int64_t g = J->perm[s];
            int lo = 0, hi = J->np - 1; /* the pair owning global record g */
            while (lo < hi) {
                const int mid = (lo + hi + 1) / 2;
                if (J->P[mid].rec0 <= g) lo = mid;
                else hi = mid - 1;
            }
            pidx[s - a] = lo;
            const c4pair *p = &J->P[lo];
            const int64_t r = g - p->rec0;
            cap += 160 + 36 * (size_t)(p->rec_first[r + 1] - p->rec_first[r]);
        }
        char *buf = malloc(cap), *o = buf;
        for (int64_t s = a; s < b; ++s) {
            const c4pair *p = &J->P[pidx[s - a]];
            const int64_t r = J->perm[s] - p->rec0, b0 = p->rec_first[r], b1 = p->rec_first[r + 1];
            int64_t qs = INT64_MAX, qe = 0, te = 0;
            for (int64_t i = b0; i < b1; ++i) {
                if (p->bq[i] < qs) qs = p->bq[i];
                if (p->bq[i] + p->bs[i] > qe) qe = p->bq[i] + p->bs[i];
                if (p->bt[i] + p->bs[i] > te) te = p->bt[i] + p->bs[i];
            }
            if (p->strand) {
                const int64_t x = J->qsize - qe;
                qe = J->qsize - qs;
                qs = x;
            }
            o += sprintf(o, "0\t0\t0\t0\t0\t0\t0\t0\t%c\t%s\t%lld\t%lld\t%lld\t%s\t%lld\t%d\t%lld\t%lld\t",
                         p->strand ? '-' : '+', C4Q->names[p->qi], (long long)J->qsize,
                         (long long)qs, (long long)qe, C4T->names[p->ti], (long long)J->tsize,
                         p->bt[b0], (long long)te, (long long)(b1 - b0));
            const int32_t *cols[3] = {p->bs, p->bq, p->bt};
            for (int c = 0; c < 3; ++c) {
                for (int64_t i = b0; i < b1; ++i) {
                    o = put_i64(o, cols[c][i]);
                    *o++ = ',';
                }
                *o++ = c < 2 ? '\t' : '\n';
            }
        }
        free(pidx);
        J->buf[k] = buf;
        J->len[k] = (size_t)(o - buf);
    }
    return NULL;
}

static int c4_main(int argc, char **argv) {
    const char *out = argv[2];
    uint64_t seed = 7;
    int64_t nblocks = 50000000, tsize = 60000000, qsize = 50000000;
    int nt = 24, nq = 21;
    double alpha = 1.2, collinear = 0.8;
    for (int i = 3; i < argc; ++i) {
        const char *a = argv[i];
        if (!strncmp(a, "-seed=", 6)) seed = strtoull(a + 6, NULL, 10);
        else if (!strncmp(a, "-blocks=", 8)) nblocks = atoll(a + 8);
        else if (!strncmp(a, "-nt=", 4)) nt = atoi(a + 4);
        else if (!strncmp(a, "-nq=", 4)) nq = atoi(a + 4);
        else if (!strncmp(a, "-tsize=", 7)) tsize = atoll(a + 7);
        else if (!strncmp(a, "-qsize=", 7)) qsize = atoll(a + 7);
        else if (!strncmp(a, "-threads=", 9)) g_threads = atoi(a + 9);
        else die("unknown option %s", a);
    }
    if (g_threads < 1)
        g_threads = 1;
    if (nt < 1 || nq < 1 || tsize < 1000 || qsize < 1000 || tsize >= (1ll << 31) ||
        qsize >= (1ll << 31))
        die("%s", "bad C4 shape");
    mkdir(out, 0777);
    g_seed = seed;
    {
        const int k = (int)lround(0.12 * 256), a = (int)lround(k * 2.0 / 3), b = (int)lround(k * 5.0 / 6);
        for (int i = 0; i < 256; ++i)
            g_xor[i] = i < a ? 1 : i < b ? 2 : i < k ? 3 : 0;
    }
    genome_t T, Q;
    memset(&T, 0, sizeof(T));
    memset(&Q, 0, sizeof(Q));
    T.n = nt;
    Q.n = nq;
    T.names = malloc(nt * sizeof(char *));
    T.size = malloc(nt * 8);
    Q.names = malloc(nq * sizeof(char *));
    Q.size = malloc(nq * 8);
    char nm[64];
    for (int i = 0; i < nt; ++i) {
        snprintf(nm, sizeof(nm), "chr%d", i + 1);
        T.names[i] = strdup(nm);
        T.size[i] = tsize;
    }
    for (int i = 0; i < nq; ++i) {
        snprintf(nm, sizeof(nm), "chrQ%d", i + 1);
        Q.names[i] = strdup(nm);
        Q.size[i] = qsize;
    }
    make_genome(&T, seed, 0);
    make_genome(&Q, seed + 1, 1);
    C4T = &T;
    C4Q = &Q;

    /* pairs (target, query, strand) and their block counts */
    const int np = nt * nq * 2;
    c4pair *P = calloc(np, sizeof(c4pair));
    double *w = malloc(np * sizeof(double)), wsum = 0;
    int *perm = malloc(np * sizeof(int));
    rng_t r;
    rng_seed(&r, seed, P_C4PAIRS, 0);
    for (int i = 0; i < np; ++i)
        perm[i] = i;
    for (int i = np - 1; i > 0; --i) {
        const int j = (int)uniform_int(&r, 0, i + 1), t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
    }
    for (int i = 0; i < np; ++i) {
        w[i] = 1.0 / pow((double)(perm[i] + 1), alpha);
        wsum += w[i];
    }
    int64_t total = 0;
    for (int i = 0, k = 0; i < nt; ++i)
        for (int j = 0; j < nq; ++j)
            for (int s = 0; s < 2; ++s, ++k) {
                P[k].ti = i;
                P[k].qi = j;
                P[k].strand = s;
                P[k].nb = (int64_t)(w[k] / wsum * (double)nblocks);
                if (P[k].nb < 50)
                    P[k].nb = 50;
                P[k].ncol = (int64_t)((double)P[k].nb * collinear);
                total += P[k].nb;
            }
    c4job J = {P, np, tsize, qsize, 0, NULL, NULL};
    atomic_init(&J.next, 0);
    run_threads(c4_pair_thread, &J);
    /* mutation pass: pairs grouped by query sequence, pair order inside */
    int *qoff = calloc(nq + 1, sizeof(int)), *qp = malloc(np * sizeof(int));
    for (int k = 0; k < np; ++k)
        qoff[P[k].qi + 1]++;
    for (int j = 0; j < nq; ++j)
        qoff[j + 1] += qoff[j];
    {
        int *fill = malloc((nq + 1) * sizeof(int));
        memcpy(fill, qoff, (nq + 1) * sizeof(int));
        for (int k = 0; k < np; ++k)
            qp[fill[P[k].qi]++] = k;
        free(fill);
    }
    J.qorder_pairs = qp;
    J.qoff = qoff;
    atomic_store(&J.next, 0);
    run_threads(c4_mut_thread, &J);

    int64_t nrec = 0, nb = 0, largest = 0;
    for (int k = 0; k < np; ++k) {
        P[k].rec0 = nrec;
        nrec += P[k].nrec;
        nb += P[k].n;
        if (P[k].n > largest)
            largest = P[k].n;
    }
    int64_t *order = malloc((size_t)(nrec + 1) * 8);
    for (int64_t i = 0; i < nrec; ++i)
        order[i] = i;
    rng_seed(&r, seed, P_C4ORDER, 0);
    for (int64_t i = nrec - 1; i > 0; --i) {
        const int64_t j = uniform_int(&r, 0, i + 1), t = order[i];
        order[i] = order[j];
        order[j] = t;
    }
    char *p;
    write_2bit(&T, p = path_in(out, "t.2bit"));
    write_2bit(&Q, p = path_in(out, "q.2bit"));
    write_sizes(&T, p = path_in(out, "t.sizes"));
    write_sizes(&Q, p = path_in(out, "q.sizes"));
    c4fmt F;
    memset(&F, 0, sizeof(F));
    F.P = P;
    F.np = np;
    F.perm = order;
    F.nrec = nrec;
    F.per = 65536;
    F.nchunks = (nrec + F.per - 1) / F.per;
    F.tsize = tsize;
    F.qsize = qsize;
    F.buf = calloc(F.nchunks + 1, sizeof(char *));
    F.len = calloc(F.nchunks + 1, sizeof(size_t));
    atomic_init(&F.next, 0);
    run_threads(c4_fmt_thread, &F);
    char *tp = path_in(out, "in.psl.tmp");
    FILE *f = fopen(tp, "wb");
    if (!f)
        die("can't write %s", tp);
    for (int64_t k = 0; k < F.nchunks; ++k) {
        fwrite_all(f, F.buf[k], F.len[k], tp);
        free(F.buf[k]);
    }
    if (fclose(f) != 0)
        die("write error on %s", tp);
    if (rename(tp, p = path_in(out, "in.psl")) != 0)
        die("can't rename %s", tp);
    f = fopen(p = path_in(out, "info.json.tmp"), "w");
    fprintf(f,
            "{\"generator\": \"gac_synth c4\", \"seed\": %llu, \"t_seqs\": %d, \"q_seqs\": %d, "
            "\"tsize\": %lld, \"qsize\": %lld, \"pairs\": %d, \"blocks\": %lld, \"records\": %lld, "
            "\"largest_pair_blocks\": %lld}\n",
            (unsigned long long)seed, nt, nq, (long long)tsize, (long long)qsize, np, (long long)nb,
            (long long)nrec, (long long)largest);
    fclose(f);
    if (rename(p, path_in(out, "info.json")) != 0)
        die("%s", "can't write info.json");
    (void)total;
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 3 && strcmp(argv[1], "c4") == 0)
        return c4_main(argc, argv);
    if (argc < 3 || strcmp(argv[1], "c5") != 0) {
        fprintf(stderr, "usage: gac_synth c5 OUTDIR [-seed=S] [-chains=N] [-scale=X] "
                        "[-minSize=M] [-sizesDir=D] [-threads=T]\n"
                        "       gac_synth c4 OUTDIR [-seed=S] [-blocks=N] [-nt=24] [-nq=21] "
                        "[-tsize=60000000] [-qsize=50000000] [-threads=T]\n");
        return 1;
    }
    const char *out = argv[2];
    uint64_t seed = 1234;
    int64_t nchains = 5000000, min_size = 20000;
    double scale = 1.0;
    const char *sizes_dir = NULL;
    for (int i = 3; i < argc; ++i) {
        const char *a = argv[i];
        if (!strncmp(a, "-seed=", 6)) seed = strtoull(a + 6, NULL, 10);
        else if (!strncmp(a, "-chains=", 8)) nchains = atoll(a + 8);
        else if (!strncmp(a, "-scale=", 7)) scale = atof(a + 7);
        else if (!strncmp(a, "-minSize=", 9)) min_size = atoll(a + 9);
        else if (!strncmp(a, "-sizesDir=", 10)) sizes_dir = a + 10;
        else if (!strncmp(a, "-threads=", 9)) g_threads = atoi(a + 9);
        else die("unknown option %s", a);
    }
    if (g_threads < 1)
        g_threads = 1;
    if (!sizes_dir)
        die("%s", "-sizesDir is required");
    mkdir(out, 0777);
    g_seed = seed;
    /* substitution table: 12 % of the bytes, transitions 2/3 */
    {
        const int k = (int)lround(0.12 * 256), a = (int)lround(k * 2.0 / 3), b = (int)lround(k * 5.0 / 6);
        for (int i = 0; i < 256; ++i)
            g_xor[i] = i < a ? 1 : i < b ? 2 : i < k ? 3 : 0;
    }
    genome_t T, Q;
    char *hp = path_in(sizes_dir, "hg38.chrom.sizes"), *mp = path_in(sizes_dir, "mm10.chrom.sizes");
    read_sizes(hp, scale, min_size, &T);
    read_sizes(mp, scale, min_size, &Q);
    G_T = &T;
    G_Q = &Q;
    make_genome(&T, seed, 0);
    make_genome(&Q, seed + 1, 1);
    g_qcum = malloc((Q.n + 1) * sizeof(double));
    g_qcum[0] = 0;
    for (int i = 0; i < Q.n; ++i)
        g_qcum[i + 1] = g_qcum[i] + (double)Q.size[i];

    /* chains per target sequence in proportion to its length */
    double total = 0;
    for (int i = 0; i < T.n; ++i)
        total += (double)T.size[i];
    int64_t n = 0;
    int64_t *per = malloc(T.n * 8);
    for (int i = 0; i < T.n; ++i) {
        per[i] = (int64_t)nearbyint((double)nchains * (double)T.size[i] / total);
        n += per[i];
    }
    chains_t C;
    memset(&C, 0, sizeof(C));
    C.n = n;
    int32_t *tseq = malloc((n ? n : 1) * 4);
    for (int i = 0, k = 0; i < T.n; ++i)
        for (int64_t j = 0; j < per[i]; ++j)
            tseq[k++] = i;
    C.tseq = tseq;
    C.off = calloc(n + 1, 8);
    chain_job cj = {&C, tseq, 0, 0};
    atomic_init(&cj.next, 0);
    run_threads(chain_thread, &cj);
    for (int64_t i = 0; i < n; ++i)
        C.off[i + 1] += C.off[i];
    C.nb = C.off[n];
    C.bt = malloc(C.nb * 4);
    C.bq = malloc(C.nb * 4);
    C.bs = malloc(C.nb * 4);
    C.qseq = malloc(n * 4);
    C.strand = malloc(n);
    C.tstart = malloc(n * 4);
    C.tend = malloc(n * 4);
    C.qstart = malloc(n * 4);
    C.qend = malloc(n * 4);
    C.score = malloc(n * 8);
    cj.pass = 1;
    atomic_store(&cj.next, 0);
    run_threads(chain_thread, &cj);

    /* plant homology, query sequence by query sequence (chain order within) */
    int64_t *qoff = calloc(Q.n + 1, 8), *qlist = malloc(n * 8);
    for (int64_t i = 0; i < n; ++i)
        qoff[C.qseq[i] + 1]++;
    for (int i = 0; i < Q.n; ++i)
        qoff[i + 1] += qoff[i];
    int64_t *fill = malloc((size_t)Q.n * 8 + 8);
    memcpy(fill, qoff, Q.n * 8);
    for (int64_t i = 0; i < n; ++i)
        qlist[fill[C.qseq[i]]++] = i;
    int *qorder = malloc(Q.n * sizeof(int));
    for (int i = 0; i < Q.n; ++i)
        qorder[i] = i;
    for (int i = 1; i < Q.n; ++i) /* by bases to mutate, largest first (insertion sort) */
        for (int j = i; j > 0 && qoff[qorder[j] + 1] - qoff[qorder[j]] >
                                     qoff[qorder[j - 1] + 1] - qoff[qorder[j - 1]]; --j) {
            const int t = qorder[j];
            qorder[j] = qorder[j - 1];
            qorder[j - 1] = t;
        }
    mut_job mj = {&C, qoff, qlist, qorder, 0};
    atomic_init(&mj.next, 0);
    run_threads(mutate_thread, &mj);

    int64_t *order = malloc(n * 8);
    for (int64_t i = 0; i < n; ++i)
        order[i] = i;
    g_sort_score = C.score;
    qsort(order, n, 8, cmp_score);

    /* outputs */
    char *p;
    write_2bit(&T, p = path_in(out, "t.2bit"));
    write_2bit(&Q, p = path_in(out, "q.2bit"));
    write_sizes(&T, p = path_in(out, "t.sizes"));
    write_sizes(&Q, p = path_in(out, "q.sizes"));
    fmt_job fj;
    memset(&fj, 0, sizeof(fj));
    fj.C = &C;
    fj.order = order;
    fj.per = 8192;
    fj.nchunks = (n + fj.per - 1) / fj.per;
    fj.buf = calloc(fj.nchunks + 1, sizeof(char *));
    fj.len = calloc(fj.nchunks + 1, sizeof(size_t));
    atomic_init(&fj.next, 0);
    run_threads(fmt_thread, &fj);
    char *cp = path_in(out, "in.chain.tmp");
    FILE *f = fopen(cp, "wb");
    if (!f)
        die("can't write %s", cp);
    for (int64_t k = 0; k < fj.nchunks; ++k) {
        fwrite_all(f, fj.buf[k], fj.len[k], cp);
        free(fj.buf[k]);
    }
    if (fclose(f) != 0)
        die("write error on %s", cp);
    if (rename(cp, p = path_in(out, "in.chain")) != 0)
        die("can't rename %s", cp);

    /* chains.bin: the sorted set as arrays (little endian):
     * "GACSYN01", int64 n, int64 nb, then f64 score[n], i32 tseq[n], qseq[n],
     * tstart[n], tend[n], qstart[n], qend[n], u8 strand[n] (padded to 8),
     * i64 off[n+1], i32 bt[nb], bq[nb], bs[nb] */
    char *bp = path_in(out, "chains.bin.tmp");
    f = fopen(bp, "wb");
    if (!f)
        die("can't write %s", bp);
    fwrite_all(f, "GACSYN01", 8, bp);
    fwrite_all(f, &n, 8, bp);
    fwrite_all(f, &C.nb, 8, bp);
    {
        double *sd = malloc(n * 8 + 8);
        int32_t *v = malloc(n * 4 + 8);
        for (int64_t s = 0; s < n; ++s)
            sd[s] = C.score[order[s]];
        fwrite_all(f, sd, n * 8, bp);
        const int32_t *cols[6] = {C.tseq, C.qseq, C.tstart, C.tend, C.qstart, C.qend};
        for (int k = 0; k < 6; ++k) {
            for (int64_t s = 0; s < n; ++s)
                v[s] = cols[k][order[s]];
            fwrite_all(f, v, n * 4, bp);
        }
        uint8_t *st = calloc(n + 8, 1);
        for (int64_t s = 0; s < n; ++s)
            st[s] = C.strand[order[s]];
        fwrite_all(f, st, (n + 7) / 8 * 8, bp);
        int64_t *o2 = malloc((n + 1) * 8);
        o2[0] = 0;
        for (int64_t s = 0; s < n; ++s)
            o2[s + 1] = o2[s] + (C.off[order[s] + 1] - C.off[order[s]]);
        fwrite_all(f, o2, (n + 1) * 8, bp);
        int32_t *bv = malloc(C.nb * 4 + 8);
        const int32_t *bcols[3] = {C.bt, C.bq, C.bs};
        for (int k = 0; k < 3; ++k) {
            for (int64_t s = 0; s < n; ++s) {
                const int64_t i = order[s];
                memcpy(bv + o2[s], bcols[k] + C.off[i], (C.off[i + 1] - C.off[i]) * 4);
            }
            fwrite_all(f, bv, C.nb * 4, bp);
        }
        free(sd);
        free(v);
        free(st);
        free(o2);
        free(bv);
    }
    if (fclose(f) != 0)
        die("write error on %s", bp);
    if (rename(bp, p = path_in(out, "chains.bin")) != 0)
        die("can't rename %s", bp);

    /* info.json: the netting loop of chainNet -rescore stops at the first
     * chain scoring below 0 (chainNet.c:949-952,1022) */
    int64_t aligned = 0, stop = n, netted = 0;
    for (int64_t s = 0; s < n; ++s)
        if (C.score[order[s]] < 0) {
            stop = s;
            break;
        }
    for (int64_t s = 0; s < n; ++s) {
        const int64_t i = order[s];
        int64_t a = 0;
        for (int64_t b = C.off[i]; b < C.off[i + 1]; ++b)
            a += C.bs[b];
        aligned += a;
        if (s < stop)
            netted += a;
    }
    f = fopen(p = path_in(out, "info.json.tmp"), "w");
    fprintf(f,
            "{\"generator\": \"gac_synth c5\", \"seed\": %llu, \"scale\": %g, \"t_seqs\": %d, "
            "\"q_seqs\": %d, \"chains\": %lld, \"blocks\": %lld, \"input_aligned_bases\": %lld, "
            "\"netted_chains\": %lld, \"netted_aligned_bases\": %lld}\n",
            (unsigned long long)seed, scale, T.n, Q.n, (long long)n, (long long)C.nb,
            (long long)aligned, (long long)stop, (long long)netted);
    fclose(f);
    if (rename(p, path_in(out, "info.json")) != 0)
        die("%s", "can't write info.json");
    return 0;
}
