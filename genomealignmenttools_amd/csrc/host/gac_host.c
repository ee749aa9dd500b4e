/* gac_host.c -- host-side parsing for libgachain (C11).
 *
 * Restates, with the same observable results, the kent routines the scoring
 * path needs before any device work:
 *   gapCalcRead / gapCalcFromFile / interpolate / calcSlope
 *       kent/src/lib/gapCalc.c:82-255   (gap tables; built-in loose/medium :40-73)
 *   axtScoreSchemeReadLf / axtScoreSchemeDefault
 *       kent/src/lib/axt.c:423-458,692-819
 *   twoBitOpen / readTwoBitSeqHeader (index only; decoding is on the device)
 *       kent/src/lib/twoBit.c:420-635
 */
#define _GNU_SOURCE
#include "gac_host.h"
#include <stdatomic.h>

#include <pthread.h>
#include <sched.h>
#include <unistd.h>

#include <ctype.h>
#include <errno.h>
#include <fcntl.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <time.h>
#include <unistd.h>

/* ------------------------------------------------------------------ errors */
static __thread char g_err[1024];

int gac_fail(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

void gac_clear_error(void) { g_err[0] = 0; }

const char *gac_last_error(void) { return g_err; }

int gac_abi_version(void) { return GAC_ABI_VERSION; }

/* ------------------------------------------------------------- file mapping */
static int map_file(const char *path, gac_map *m, int populate);
int gac_map_file(const char *path, gac_map *m) { return map_file(path, m, 0); }

static int map_file(const char *path, gac_map *m, int populate) {
    memset(m, 0, sizeof(*m));
    m->fd = -1;
    int fd = (strcmp(path, "stdin") == 0) ? 0 : open(path, O_RDONLY);
    if (fd < 0)
        return gac_fail(GAC_E_IO, "can't open %s: %s", path, strerror(errno));
    struct stat st;
    if (fd != 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode)) {
        m->size = (size_t)st.st_size;
        if (m->size == 0) {
            m->data = (const uint8_t *)"";
            m->fd = fd;
            m->mapped = 0;
            close(fd);
            m->fd = -1;
            return GAC_OK;
        }
        void *p = mmap(NULL, m->size, PROT_READ, MAP_PRIVATE | (populate ? MAP_POPULATE : 0), fd, 0);
        if (p == MAP_FAILED) {
            close(fd);
            return gac_fail(GAC_E_IO, "can't mmap %s: %s", path, strerror(errno));
        }
        madvise(p, m->size, MADV_SEQUENTIAL);
        m->data = p;
        m->fd = fd;
        m->mapped = 1;
        return GAC_OK;
    }
    /* pipe / stdin: slurp */
    size_t cap = 1 << 20, len = 0;
    uint8_t *buf = malloc(cap);
    if (!buf)
        return gac_fail(GAC_E_IO, "out of memory reading %s", path);
    for (;;) {
        if (len == cap) {
            cap *= 2;
            uint8_t *nb = realloc(buf, cap);
            if (!nb) {
                free(buf);
                return gac_fail(GAC_E_IO, "out of memory reading %s", path);
            }
            buf = nb;
        }
        ssize_t r = read(fd, buf + len, cap - len);
        if (r < 0) {
            free(buf);
            return gac_fail(GAC_E_IO, "read error on %s", path);
        }
        if (r == 0)
            break;
        len += (size_t)r;
    }
    if (fd != 0)
        close(fd);
    m->data = buf;
    m->size = len;
    m->mapped = 0;
    m->fd = -2; /* heap-owned */
    return GAC_OK;
}

void gac_unmap_file(gac_map *m) {
    if (m->mapped) {
        munmap((void *)m->data, m->size);
        close(m->fd);
    } else if (m->fd == -2) {
        free((void *)m->data);
    }
    memset(m, 0, sizeof(*m));
}

/* ------------------------------------------------------------ word helpers */
int gac_chop_white(char *s, char **words, int max) {
    int n = 0;
    while (n < max) {
        while (*s && isspace((unsigned char)*s))
            ++s;
        if (*s == 0)
            break;
        words[n++] = s;
        while (*s && !isspace((unsigned char)*s))
            ++s;
        if (*s == 0)
            break;
        *s++ = 0;
    }
    return n;
}

int gac_same_word(const char *a, const char *b) { return strcasecmp(a, b) == 0; }

/* ------------------------------------------------------------------ gapCalc */
/* Built-in tables, same numbers as kent/src/lib/gapCalc.c:40-73. */
static const char *k_gap_loose =
    "tablesize 11\n"
    "smallSize 111\n"
    "position 1 2 3 11 111 2111 12111 32111 72111 152111 252111\n"
    "qGap 325 360 400 450 600 1100 3600 7600 15600 31600 56600\n"
    "tGap 325 360 400 450 600 1100 3600 7600 15600 31600 56600\n"
    "bothGap 625 660 700 750 900 1400 4000 8000 16000 32000 57000\n";
static const char *k_gap_medium =
    "tableSize 11\n"
    "smallSize 111\n"
    "position 1 2 3 11 111 2111 12111 32111 72111 152111 252111\n"
    "qGap 350 425 450 600 900 2900 22900 57900 117900 217900 317900\n"
    "tGap 350 425 450 600 900 2900 22900 57900 117900 217900 317900\n"
    "bothGap 750 825 850 1000 1300 3300 23300 58300 118300 218300 318300\n";

/* kent interpolate(): linear interpolation between table points, evaluated in
 * double with the reference's operation order, truncated to int on return. */
static int gc_interp(int x, const int *s, const double *v, int n) {
    for (int i = 0; i < n; ++i) {
        if (x == s[i])
            return (int)v[i];
        if (x < s[i]) {
            int ds = s[i] - s[i - 1];
            double dv = v[i] - v[i - 1];
            volatile double prod = dv * (x - s[i - 1]); /* no contraction */
            return (int)(v[i - 1] + prod / ds);
        }
    }
    int ds = s[n - 1] - s[n - 2];
    double dv = v[n - 1] - v[n - 2];
    volatile double prod = dv * (x - s[n - 2]);
    return (int)(v[n - 2] + prod / ds);
}

typedef struct gc_text {
    char *buf;
    char *cur;
    const char *name;
    int line;
} gc_text;

/* Next line that is not blank and not a comment (kent lineFileNextReal). */
static char *gc_next_real(gc_text *t) {
    while (t->cur && *t->cur) {
        char *line = t->cur;
        char *nl = strchr(line, '\n');
        if (nl) {
            *nl = 0;
            t->cur = nl + 1;
        } else {
            t->cur = line + strlen(line);
        }
        ++t->line;
        char *p = line;
        while (*p && isspace((unsigned char)*p))
            ++p;
        if (*p != 0 && *p != '#')
            return line;
    }
    return NULL;
}

/* kent readTaggedNumLine (gapCalc.c:112-144). */
static int gc_tagged(gc_text *t, const char *tag, int count, int *iout, double *fout) {
    char *line = gc_next_real(t);
    if (!line)
        return gac_fail(GAC_E_FORMAT, "Unexpected end of file in %s", t->name);
    char *w[512];
    int nw = gac_chop_white(line, w, 512);
    if (nw == 0 || !gac_same_word(tag, w[0]))
        return gac_fail(GAC_E_FORMAT, "Expecting %s got %s line %d of %s", tag,
                        nw ? w[0] : "", t->line, t->name);
    if (nw - 1 < count)
        return gac_fail(GAC_E_FORMAT, "Not enough numbers line %d of %s", t->line, t->name);
    if (nw - 1 > count)
        return gac_fail(GAC_E_FORMAT, "Too many numbers line %d of %s", t->line, t->name);
    for (int i = 0; i < count; ++i) {
        const char *word = w[i + 1];
        if (!isdigit((unsigned char)word[0]))
            return gac_fail(GAC_E_FORMAT, "Expecting number got %s line %d of %s", word,
                            t->line, t->name);
        if (iout)
            iout[i] = atoi(word);
        if (fout)
            fout[i] = atof(word);
    }
    return GAC_OK;
}

/* interpolate() over the long positions (gapCalc.c:82-104) */
static int gc_long(const gac_gapcalc *g, const double *v, int x) {
    return gc_interp(x, g->long_pos, v, g->long_count);
}

int gac_gap_cost(const gac_gapcalc *g, int dq, int dt) {
    if (dt < 0)
        dt = 0;
    if (dq < 0)
        dq = 0;
    if (dt == 0) {
        if (dq < g->small_size)
            return g->q_small[dq];
        if (dq >= g->q_last_pos) {
            volatile double prod = g->q_last_slope * (dq - g->q_last_pos);
            return (int)(g->q_last_val + prod);
        }
        return gc_long(g, g->q_long, dq);
    }
    if (dq == 0) {
        if (dt < g->small_size)
            return g->t_small[dt];
        if (dt >= g->t_last_pos) {
            volatile double prod = g->t_last_slope * (dt - g->t_last_pos);
            return (int)(g->t_last_val + prod);
        }
        return gc_long(g, g->t_long, dt);
    }
    const int both = dq + dt;
    if (both < g->small_size)
        return g->b_small[both];
    if (both >= g->b_last_pos) {
        volatile double prod = g->b_last_slope * (both - g->b_last_pos);
        return (int)(g->b_last_val + prod);
    }
    return gc_long(g, g->b_long, both);
}

void gac_gapcalc_free(gac_gapcalc *g) {
    if (!g)
        return;
    free(g->q_small);
    free(g->t_small);
    free(g->b_small);
    free(g->long_pos);
    free(g->q_long);
    free(g->t_long);
    free(g->b_long);
    free(g);
}

int gac_gapcalc_same(const gac_gapcalc *a, const gac_gapcalc *b) {
    if (a == b)
        return 1;
    if (!a || !b || a->small_size != b->small_size || a->long_count != b->long_count ||
        a->q_last_pos != b->q_last_pos || a->t_last_pos != b->t_last_pos ||
        a->b_last_pos != b->b_last_pos || a->q_last_val != b->q_last_val ||
        a->t_last_val != b->t_last_val || a->b_last_val != b->b_last_val ||
        a->q_last_slope != b->q_last_slope || a->t_last_slope != b->t_last_slope ||
        a->b_last_slope != b->b_last_slope)
        return 0;
    const size_t ns = (size_t)a->small_size * 4, nl = (size_t)a->long_count;
    return memcmp(a->q_small, b->q_small, ns) == 0 && memcmp(a->t_small, b->t_small, ns) == 0 &&
           memcmp(a->b_small, b->b_small, ns) == 0 &&
           memcmp(a->long_pos, b->long_pos, nl * 4) == 0 &&
           memcmp(a->q_long, b->q_long, nl * 8) == 0 && memcmp(a->t_long, b->t_long, nl * 8) == 0 &&
           memcmp(a->b_long, b->b_long, nl * 8) == 0;
}

static void *dup_mem(const void *p, size_t n) {
    void *q = malloc(n ? n : 1);
    if (n)
        memcpy(q, p, n);
    return q;
}

gac_gapcalc *gac_gapcalc_clone(const gac_gapcalc *g) {
    gac_gapcalc *c = malloc(sizeof(*c));
    *c = *g;
    const size_t ns = (size_t)g->small_size * 4, nl = (size_t)g->long_count;
    c->q_small = dup_mem(g->q_small, ns);
    c->t_small = dup_mem(g->t_small, ns);
    c->b_small = dup_mem(g->b_small, ns);
    c->long_pos = dup_mem(g->long_pos, nl * 4);
    c->q_long = dup_mem(g->q_long, nl * 8);
    c->t_long = dup_mem(g->t_long, nl * 8);
    c->b_long = dup_mem(g->b_long, nl * 8);
    return c;
}

static int gc_parse(char *text, const char *name, gac_gapcalc **out) {
    gc_text t = {text, text, name, 0};
    int table_size = 0, small_size = 0, rc;
    if ((rc = gc_tagged(&t, "tableSize", 1, &table_size, NULL)) != GAC_OK)
        return rc;
    if ((rc = gc_tagged(&t, "smallSize", 1, &small_size, NULL)) != GAC_OK)
        return rc;
    if (table_size < 2 || table_size > 4096 || small_size < 1)
        return gac_fail(GAC_E_FORMAT, "bad tableSize/smallSize in %s", name);
    int *pos = calloc(table_size, sizeof(int));
    double *qg = calloc(table_size, sizeof(double));
    double *tg = calloc(table_size, sizeof(double));
    double *bg = calloc(table_size, sizeof(double));
    gac_gapcalc *g = calloc(1, sizeof(*g));
    if (!pos || !qg || !tg || !bg || !g) {
        rc = gac_fail(GAC_E_ARG, "out of memory");
        goto done;
    }
    if ((rc = gc_tagged(&t, "position", table_size, pos, NULL)) != GAC_OK ||
        (rc = gc_tagged(&t, "qGap", table_size, NULL, qg)) != GAC_OK ||
        (rc = gc_tagged(&t, "tGap", table_size, NULL, tg)) != GAC_OK ||
        (rc = gc_tagged(&t, "bothGap", table_size, NULL, bg)) != GAC_OK)
        goto done;
    g->small_size = small_size;
    g->q_small = calloc(small_size, sizeof(int32_t));
    g->t_small = calloc(small_size, sizeof(int32_t));
    g->b_small = calloc(small_size, sizeof(int32_t));
    /* small tables for 1..smallSize-1; index 0 stays 0 (gapCalc.c:174-182) */
    for (int i = 1; i < small_size; ++i) {
        g->q_small[i] = gc_interp(i, pos, qg, table_size);
        g->t_small[i] = gc_interp(i, pos, tg, table_size);
        g->b_small[i] = gc_interp(i, pos, bg, table_size);
    }
    int start_long = -1;
    for (int i = 0; i < table_size; ++i)
        if (pos[i] == small_size) {
            start_long = i;
            break;
        }
    if (start_long < 0) {
        rc = gac_fail(GAC_E_FORMAT, "No position %d in gapCalcRead()", small_size);
        goto done;
    }
    int lc = table_size - start_long;
    if (lc < 2) {
        rc = gac_fail(GAC_E_FORMAT, "need >= 2 long positions in %s", name);
        goto done;
    }
    g->long_count = lc;
    g->long_pos = malloc(lc * sizeof(int32_t));
    g->q_long = malloc(lc * sizeof(double));
    g->t_long = malloc(lc * sizeof(double));
    g->b_long = malloc(lc * sizeof(double));
    for (int i = 0; i < lc; ++i) {
        g->long_pos[i] = pos[start_long + i];
        g->q_long[i] = qg[start_long + i];
        g->t_long[i] = tg[start_long + i];
        g->b_long[i] = bg[start_long + i];
    }
    g->q_last_pos = g->t_last_pos = g->b_last_pos = g->long_pos[lc - 1];
    g->q_last_val = g->q_long[lc - 1];
    g->t_last_val = g->t_long[lc - 1];
    g->b_last_val = g->b_long[lc - 1];
    /* calcSlope (gapCalc.c:106-110): (y2-y1)/(x2-x1) in double */
    double dx = (double)g->long_pos[lc - 1] - (double)g->long_pos[lc - 2];
    g->q_last_slope = (g->q_last_val - g->q_long[lc - 2]) / dx;
    g->t_last_slope = (g->t_last_val - g->t_long[lc - 2]) / dx;
    g->b_last_slope = (g->b_last_val - g->b_long[lc - 2]) / dx;
    *out = g;
    g = NULL;
    rc = GAC_OK;
done:
    free(pos);
    free(qg);
    free(tg);
    free(bg);
    gac_gapcalc_free(g);
    return rc;
}

int gac_gapcalc_build(const char *name, gac_gapcalc **out) {
    if (!name || !out)
        return gac_fail(GAC_E_ARG, "gac_gapcalc_build: NULL argument");
    *out = NULL;
    char *text = NULL;
    int rc;
    if (strcmp(name, "loose") == 0)
        text = strdup(k_gap_loose);
    else if (strcmp(name, "medium") == 0)
        text = strdup(k_gap_medium);
    else {
        gac_map m;
        if ((rc = gac_map_file(name, &m)) != GAC_OK)
            return rc;
        text = malloc(m.size + 1);
        memcpy(text, m.data, m.size);
        text[m.size] = 0;
        gac_unmap_file(&m);
    }
    rc = gc_parse(text, name, out);
    free(text);
    return rc;
}

/* --------------------------------------------------------- score matrix */
/* blastz default (axt.c:423-458), A,C,G,T order, [query][target] */
static const int32_t k_blastz[16] = {91, -114, -31, -123, -114, 100, -125, -31,
                                     -31, -125, 100, -114, -123, -31, -114, 91};

typedef struct sc_lines {
    char *cur;
    int line;
} sc_lines;

/* raw next line (kent lineFileNext) */
static char *sc_next(sc_lines *l) {
    if (!l->cur || !*l->cur)
        return NULL;
    char *line = l->cur;
    char *nl = strchr(line, '\n');
    if (nl) {
        *nl = 0;
        l->cur = nl + 1;
    } else {
        l->cur = line + strlen(line);
    }
    ++l->line;
    return line;
}

/* kent lineFileChopNext: skip lines starting with '#' and blank lines */
static int sc_chop_next(sc_lines *l, char **row, int max) {
    char *line;
    while ((line = sc_next(l)) != NULL) {
        if (line[0] == '#')
            continue;
        int n = gac_chop_white(line, row, max);
        if (n)
            return n;
    }
    return 0;
}

static void sc_append(char **buf, size_t *len, size_t *cap, const char *s) {
    size_t n = strlen(s);
    if (*len + n + 1 > *cap) {
        *cap = (*len + n + 1) * 2;
        *buf = realloc(*buf, *cap);
    }
    memcpy(*buf + *len, s, n + 1);
    *len += n;
}

/* split on any char of seps, dropping empty fields (kent chopString) */
static int sc_chop_string(char *s, const char *seps, char **parts, int max) {
    int n = 0;
    while (*s && n < max) {
        while (*s && strchr(seps, *s))
            ++s;
        if (!*s)
            break;
        parts[n++] = s;
        while (*s && !strchr(seps, *s))
            ++s;
        if (*s)
            *s++ = 0;
    }
    return n;
}

int gac_scheme_read(const char *path, int32_t mat[16], int32_t *gap_open,
                    int32_t *gap_extend, char **extra) {
    if (extra)
        *extra = NULL;
    if (!path) {
        memcpy(mat, k_blastz, sizeof(k_blastz));
        if (gap_open)
            *gap_open = 400;
        if (gap_extend)
            *gap_extend = 30;
        return GAC_OK;
    }
    gac_map m;
    int rc = gac_map_file(path, &m);
    if (rc != GAC_OK)
        return rc;
    char *text = malloc(m.size + 1);
    memcpy(text, m.data, m.size);
    text[m.size] = 0;
    gac_unmap_file(&m);

    sc_lines l = {text, 0};
    char *row[6];
    char *ex = calloc(1, 64);
    size_t exlen = 0, excap = 64;
    int go = 400, ge = 30;
    int wc = sc_chop_next(&l, row, 6);
    if (!wc) {
        rc = gac_fail(GAC_E_FORMAT, "Scoring matrix file %s too short", path);
        goto out;
    }
    for (;;) {
        if (strchr(row[0], '=') || (wc > 1 && strchr(row[1], '='))) {
            char joined[4096];
            joined[0] = 0;
            for (int i = 0; i < wc; ++i)
                strncat(joined, row[i], sizeof(joined) - strlen(joined) - 1);
            char *hash = strchr(joined, '#');
            if (hash)
                *hash = 0;
            char *parts[32];
            int np = sc_chop_string(joined, "=", parts, 32);
            if (np >= 2 && !(strcmp(parts[0], "O") == 0 || strcmp(parts[0], "E") == 0)) {
                sc_append(&ex, &exlen, &excap, parts[0]);
                sc_append(&ex, &exlen, &excap, "=");
                sc_append(&ex, &exlen, &excap, parts[1]);
                sc_append(&ex, &exlen, &excap, ",");
            }
            wc = sc_chop_next(&l, row, 6);
            if (!wc) {
                rc = gac_fail(GAC_E_FORMAT, "Scoring matrix file %s too short", path);
                goto out;
            }
            continue;
        }
        if (wc < 4 || row[0][0] != 'A' || row[1][0] != 'C' || row[2][0] != 'G' ||
            row[3][0] != 'T') {
            rc = gac_fail(GAC_E_FORMAT, "%s doesn't seem to be a score matrix file", path);
            goto out;
        }
        for (int i = 0; i < 4; ++i) {
            wc = sc_chop_next(&l, row, 6);
            if (!wc) {
                rc = gac_fail(GAC_E_FORMAT, "Scoring matrix file %s too short", path);
                goto out;
            }
            int c0 = (wc == 5) ? 1 : 0;
            if (wc < c0 + 4) {
                rc = gac_fail(GAC_E_FORMAT, "short matrix row line %d of %s", l.line, path);
                goto out;
            }
            for (int j = 0; j < 4; ++j) {
                char *end;
                const char *w = row[c0 + j];
                long v = strtol(w, &end, 10);
                if (end == w || *end != 0) {
                    rc = gac_fail(GAC_E_FORMAT, "Expecting number got %s line %d of %s", w,
                                  l.line, path);
                    goto out;
                }
                mat[i * 4 + j] = (int32_t)v;
            }
        }
        char *line = sc_next(&l);
        if (line) {
            sc_append(&ex, &exlen, &excap, line);
            sc_append(&ex, &exlen, &excap, ",");
            char *parts[32];
            int np = sc_chop_string(line, " =,\t", parts, 32);
            int got_o = 0, got_e = 0;
            for (int i = 0; i < np - 1; i += 2) {
                if (strcmp(parts[i], "O") == 0) {
                    got_o = 1;
                    go = atoi(parts[i + 1]);
                }
                if (strcmp(parts[i], "E") == 0) {
                    got_e = 1;
                    ge = atoi(parts[i + 1]);
                }
            }
            if (!got_o || !got_e) {
                rc = gac_fail(GAC_E_FORMAT, "Expecting O = and E = in last line of %s", path);
                goto out;
            }
            if (go <= 0 || ge <= 0) {
                rc = gac_fail(GAC_E_FORMAT, "Must have positive gap scores");
                goto out;
            }
        }
        break;
    }
    if (exlen && ex[exlen - 1] == ',')
        ex[--exlen] = 0;
    if (gap_open)
        *gap_open = go;
    if (gap_extend)
        *gap_extend = ge;
    if (extra) {
        *extra = ex;
        ex = NULL;
    }
    rc = GAC_OK;
out:
    free(ex);
    free(text);
    return rc;
}

/* ------------------------------------------------------------------- 2bit */
#define TWOBIT_SIG 0x1A412743u
#define TWOBIT_SIG_SWAP 0x4327411Au

uint32_t gac_twobit_u32(const gac_twobit *tb, const uint8_t *p) {
    uint32_t v;
    memcpy(&v, p, 4);
    return tb->swapped ? __builtin_bswap32(v) : v;
}

static uint64_t tb_u64(const gac_twobit *tb, const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return tb->swapped ? __builtin_bswap64(v) : v;
}

int gac_is_twobit_file(const char *path) {
    size_t n = strlen(path);
    return n >= 5 && strcmp(path + n - 5, ".2bit") == 0;
}

void gac_twobit_close(gac_twobit *tb) {
    if (tb->seqs) {
        for (uint32_t i = 0; i < tb->seq_count; ++i)
            free(tb->seqs[i].name);
        free(tb->seqs);
    }
    gac_unmap_file(&tb->map);
    memset(tb, 0, sizeof(*tb));
}

int gac_twobit_open(const char *path, gac_twobit *tb) { return gac_twobit_open_ex(path, tb, 0); }

int gac_twobit_open_ex(const char *path, gac_twobit *tb, int populate) {
    memset(tb, 0, sizeof(*tb));
    int rc = map_file(path, &tb->map, populate);
    if (rc != GAC_OK)
        return rc;
    const uint8_t *d = tb->map.data;
    size_t sz = tb->map.size;
    if (sz < 16) {
        gac_twobit_close(tb);
        return gac_fail(GAC_E_FORMAT, "%s doesn't have a valid twoBitSig", path);
    }
    uint32_t sig;
    memcpy(&sig, d, 4);
    if (sig == TWOBIT_SIG_SWAP)
        tb->swapped = 1;
    else if (sig != TWOBIT_SIG) {
        gac_twobit_close(tb);
        return gac_fail(GAC_E_FORMAT, "%s doesn't have a valid twoBitSig", path);
    }
    tb->version = gac_twobit_u32(tb, d + 4);
    if (tb->version != 0 && tb->version != 1) {
        gac_twobit_close(tb);
        return gac_fail(GAC_E_FORMAT,
                        "Can only handle version 0 or version 1 of this file. This is version %u",
                        tb->version);
    }
    tb->seq_count = gac_twobit_u32(tb, d + 8);
    tb->seqs = calloc(tb->seq_count ? tb->seq_count : 1, sizeof(gac_twobit_seq));
    size_t off = 16;
    for (uint32_t i = 0; i < tb->seq_count; ++i) {
        if (off + 1 > sz)
            goto trunc;
        uint32_t nl = d[off++];
        if (off + nl + (tb->version == 1 ? 8 : 4) > sz)
            goto trunc;
        tb->seqs[i].name = strndup((const char *)d + off, nl);
        off += nl;
        uint64_t so;
        if (tb->version == 1) {
            so = tb_u64(tb, d + off);
            off += 8;
        } else {
            so = gac_twobit_u32(tb, d + off);
            off += 4;
        }
        /* sequence record */
        size_t p = (size_t)so;
        if (p + 8 > sz)
            goto trunc;
        gac_twobit_seq *s = &tb->seqs[i];
        s->size = gac_twobit_u32(tb, d + p);
        p += 4;
        s->n_count = gac_twobit_u32(tb, d + p);
        p += 4;
        if (p + 8ull * s->n_count + 4 > sz)
            goto trunc;
        s->n_starts_raw = d + p;
        p += 4ull * s->n_count;
        s->n_sizes_raw = d + p;
        p += 4ull * s->n_count;
        uint32_t mc = gac_twobit_u32(tb, d + p);
        p += 4 + 8ull * mc;
        p += 4; /* reserved */
        if (p + ((size_t)s->size + 3) / 4 > sz)
            goto trunc;
        s->packed = d + p;
    }
    return GAC_OK;
trunc:
    gac_twobit_close(tb);
    return gac_fail(GAC_E_FORMAT, "%s is truncated", path);
}

/* ------------------------------------------------------------------- threads */
/* CPUs of a cgroup CPU quota, rounded up: cgroup v2 "cpu.max" ("max 100000"
 * or "<quota> <period>") or v1 cpu.cfs_quota_us / cpu.cfs_period_us.  0 = no
 * quota (or none readable). */
static int cgroup_quota_cpus(const char *v2_path) {
    long long q = -1, p = 0;
    FILE *f = fopen(v2_path, "r");
    if (f) {
        char a[32] = {0};
        if (fscanf(f, "%31s %lld", a, &p) == 2 && strcmp(a, "max") != 0)
            q = atoll(a);
        fclose(f);
    } else if ((f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r"))) {
        if (fscanf(f, "%lld", &q) != 1)
            q = -1;
        fclose(f);
        if ((f = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r"))) {
            if (fscanf(f, "%lld", &p) != 1)
                p = 0;
            fclose(f);
        }
    }
    if (q <= 0 || p <= 0)
        return 0;
    const long long n = (q + p - 1) / p;
    return n > 0 && n < 1 << 20 ? (int)n : 0;
}

/* The CPUs this process may use: the online CPUs, narrowed by its affinity
 * mask and by its cgroup's CPU quota (a container with a 16-CPU quota on a
 * 256-CPU host gets 16 threads, not 64 time-sliced ones). */
int gac_host_cpus(void) {
    static _Atomic int cached;
    const char *cg = getenv("GAC_CGROUP_CPU_MAX"); /* (tests: another cpu.max file) */
    int n = cg ? 0 : atomic_load(&cached);
    if (n > 0)
        return n;
    const long c = sysconf(_SC_NPROCESSORS_ONLN);
    n = c > 0 ? (int)c : 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) {
        const int a = CPU_COUNT(&set);
        if (a > 0 && a < n)
            n = a;
    }
    const int q = cgroup_quota_cpus(cg ? cg : "/sys/fs/cgroup/cpu.max");
    if (q > 0 && q < n)
        n = q;
    if (!cg)
        atomic_store(&cached, n);
    return n;
}

int gac_host_threads(void) {
    const char *s = getenv("GAC_THREADS");
    if (!s || !*s)
        s = getenv("OMP_NUM_THREADS");
    int n = s && *s ? atoi(s) : 0;
    if (n <= 0)
        n = gac_host_cpus();
    return n > 64 ? 64 : n;
}

void gac_mark(const char *what) {
    static int on = -1;
    static double t0;
    if (on < 0) {
        on = getenv("GAC_TIMING") != NULL;
        struct timespec ts;
        clock_gettime(CLOCK_MONOTONIC, &ts);
        t0 = ts.tv_sec + 1e-9 * ts.tv_nsec;
    }
    if (!on)
        return;
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    fprintf(stderr, "[mark] %8.3f %lx %s\n", ts.tv_sec + 1e-9 * ts.tv_nsec - t0,
            (unsigned long)pthread_self() & 0xffff, what);
}

void gac_run_threads(int n, void *(*fn)(void *), void *arg) {
    if (n < 1)
        n = 1;
    pthread_t *th = malloc((size_t)n * sizeof(pthread_t));
    int started = 1; /* (callers claim work from a shared counter, so fewer threads still finish it) */
    for (int i = 1; i < n && th; ++i, ++started)
        if (pthread_create(&th[i], NULL, fn, arg) != 0)
            break;
    fn(arg);
    for (int i = 1; i < started; ++i)
        pthread_join(th[i], NULL);
    free(th);
}

/* ------------------------------------------------------------ output */
/* outputs opened by gac_open_output and not yet closed: an abort cuts each
 * to the bytes this run wrote (gac_outputs_cut), so no file is left holding
 * new text followed by an earlier run's tail */
#define GAC_MAX_OUTPUTS 32
static pthread_mutex_t g_out_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_out_fd[GAC_MAX_OUTPUTS];
static int g_out_n;

static void out_register(int fd, int add) {
    pthread_mutex_lock(&g_out_mu);
    if (add) {
        if (g_out_n < GAC_MAX_OUTPUTS)
            g_out_fd[g_out_n++] = fd;
    } else {
        for (int i = 0; i < g_out_n; ++i)
            if (g_out_fd[i] == fd) {
                g_out_fd[i] = g_out_fd[--g_out_n];
                break;
            }
    }
    pthread_mutex_unlock(&g_out_mu);
}

/* cut a regular file to `end` bytes when it is longer */
static int cut_to(int fd, off_t end) {
    struct stat st;
    if (end >= 0 && fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > end)
        return ftruncate(fd, end);
    return 0;
}

void gac_outputs_cut(void) {
    /* (no lock: the abort path may run while another thread holds it; the
     * table is only read, and a stale fd at worst fails the fstat) */
    for (int i = 0; i < g_out_n; ++i)
        (void)cut_to(g_out_fd[i], lseek(g_out_fd[i], 0, SEEK_CUR));
}

FILE *gac_open_output(const char *path) {
    const int fd = open(path, O_WRONLY | O_CREAT | O_CLOEXEC, 0666);
    if (fd < 0)
        return NULL;
    FILE *f = fdopen(fd, "w");
    if (!f) {
        close(fd);
        return NULL;
    }
    out_register(fd, 1);
    return f;
}

/* The file is opened without O_TRUNC (re-truncating a file the tool created
 * at start makes ext4 flush it on close): it is cut to the bytes written
 * here instead -- on a failed flush to the bytes that reached the file, so a
 * failed write leaves a short file (as the reference's), never an earlier
 * run's tail after the new text. */
int gac_close_output(FILE *f) {
    const int fd = fileno(f);
    int bad = fflush(f) != 0;
    const off_t end = bad ? lseek(fd, 0, SEEK_CUR) : ftello(f);
    if (cut_to(fd, end) != 0)
        bad = 1;
    out_register(fd, 0);
    return (fclose(f) != 0 || bad) ? EOF : 0;
}

char *gac_obuf_reserve(gac_obuf *o, size_t k) {
    if (o->n + k > o->cap) {
        size_t c = o->cap ? 2 * o->cap : (size_t)1 << 16;
        while (c < o->n + k)
            c *= 2;
        char *q = realloc(o->p, c);
        if (!q) {
            fprintf(stderr, "out of memory formatting output\n");
            abort();
        }
        o->p = q;
        o->cap = c;
    }
    return o->p + o->n;
}

void gac_obuf_printf(gac_obuf *o, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    const int k = vsnprintf(NULL, 0, fmt, ap);
    va_end(ap);
    if (k <= 0)
        return;
    char *p = gac_obuf_reserve(o, (size_t)k + 1);
    va_start(ap, fmt);
    vsnprintf(p, (size_t)k + 1, fmt, ap);
    va_end(ap);
    o->n += (size_t)k;
}

typedef struct po_job {
    int64_t nr;
    void (*fn)(FILE *, int64_t, void *);
    void (*fn_buf)(gac_obuf *, int64_t, void *);
    void *arg;
    char **buf;
    size_t *len;
    _Atomic int *ready;
    _Atomic int64_t next;
    _Atomic int64_t done; /* runs formatted (GAC_TIMING: a mark when all are) */
    _Atomic int oom;
} po_job;

static void *po_thread(void *p) {
    po_job *J = p;
    for (;;) {
        const int64_t r = atomic_fetch_add(&J->next, 1);
        if (r >= J->nr)
            break;
        if (J->fn_buf) {
            gac_obuf o = {NULL, 0, 0};
            J->fn_buf(&o, r, J->arg);
            J->buf[r] = o.p;
            J->len[r] = o.n;
            atomic_store_explicit(&J->ready[r], 1, memory_order_release);
            if (atomic_fetch_add(&J->done, 1) + 1 == J->nr)
                gac_mark("output: every run formatted");
            continue;
        }
        FILE *f = open_memstream(&J->buf[r], &J->len[r]);
        if (!f) {
            atomic_store(&J->oom, 1);
        } else {
            J->fn(f, r, J->arg);
            fclose(f);
        }
        atomic_store_explicit(&J->ready[r], 1, memory_order_release);
    }
    return NULL;
}

/* the same runs formatted in parallel but kept: bufs[r] / lens[r] (malloc'd) */
static int par_format(int64_t nr, void (*fn)(FILE *f, int64_t r, void *arg),
                      void (*fn_buf)(gac_obuf *o, int64_t r, void *arg), void *arg, char ***bufs,
                      size_t **lens) {
    po_job J;
    J.nr = nr;
    J.fn = fn;
    J.fn_buf = fn_buf;
    J.arg = arg;
    J.buf = calloc((size_t)(nr > 0 ? nr : 1), sizeof(char *));
    J.len = calloc((size_t)(nr > 0 ? nr : 1), sizeof(size_t));
    J.ready = calloc((size_t)(nr > 0 ? nr : 1), sizeof(_Atomic int));
    atomic_init(&J.next, 0);
    atomic_init(&J.done, 0);
    atomic_init(&J.oom, 0);
    int nt = gac_host_threads();
    if (nt > nr)
        nt = (int)(nr > 0 ? nr : 1);
    if (nr > 0)
        gac_run_threads(nt, po_thread, &J);
    free((void *)J.ready);
    *bufs = J.buf;
    *lens = J.len;
    return atomic_load(&J.oom) ? -1 : 0;
}

/* Large outputs into a regular file, opt-in: every run formatted first,
 * then copied into a shared mapping of the reserved file range by all
 * threads (buffered write() calls into one file serialise on its inode lock;
 * page faults on a mapping do not).  GAC_OUTPUT_MMAP_MIN = the size from
 * which it is used (bytes; 0 = always; unset or negative = never).  Off by
 * default: on the GPU box's overlay filesystem the copy itself is fast (330
 * MB in 0.14-0.18 s) but losing the overlap of formatting and writing made
 * chainNet's two nets slower (write stage 0.40 vs 0.22 s on C5 at 1 M
 * chains) and scoreChain no faster (0.26 vs 0.29 s); scripts/gpu_output_ab.sh. */
static long long output_mmap_min(void) {
    const char *s = getenv("GAC_OUTPUT_MMAP_MIN");
    return s && *s ? atoll(s) : -1;
}

typedef struct mcopy_job {
    char *dst;
    char **buf;
    const size_t *len, *pre;
    int64_t nr;
    size_t total, chunk;
    _Atomic size_t next;
} mcopy_job;

static void *mcopy_thread(void *p) {
    mcopy_job *M = p;
    for (;;) {
        size_t a = atomic_fetch_add(&M->next, M->chunk);
        if (a >= M->total)
            break;
        const size_t b = a + M->chunk < M->total ? a + M->chunk : M->total;
        int64_t lo = 0, hi = M->nr - 1; /* last run starting at or before a */
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) / 2;
            if (M->pre[mid] <= a)
                lo = mid;
            else
                hi = mid - 1;
        }
        for (int64_t r = lo; a < b && r < M->nr; ++r) {
            const size_t s0 = M->pre[r], s1 = s0 + M->len[r];
            if (s1 <= a)
                continue;
            const size_t e = s1 < b ? s1 : b;
            memcpy(M->dst + a, M->buf[r] + (a - s0), e - a);
            a = e;
        }
    }
    return NULL;
}

/* 1: written; 0: not possible here (the caller writes with fwrite); -1: error */
static int par_output_mapped(FILE *out, char **buf, const size_t *len, int64_t nr, size_t total) {
    const int fd = fileno(out);
    if (fflush(out) != 0)
        return -1;
    const off_t off0 = ftello(out);
    if (off0 < 0 || posix_fallocate(fd, off0, (off_t)total) != 0)
        return 0; /* (no space: the fwrite path reports it) */
    char path[64];
    snprintf(path, sizeof(path), "/proc/self/fd/%d", fd);
    const int rw = open(path, O_RDWR); /* a shared writable mapping needs read access too */
    if (rw < 0)
        return 0;
    const long pg = sysconf(_SC_PAGESIZE);
    const off_t pa = off0 & ~(off_t)(pg - 1);
    const size_t mlen = (size_t)(off0 - pa) + total;
    char *m = mmap(NULL, mlen, PROT_READ | PROT_WRITE, MAP_SHARED, rw, pa);
    close(rw);
    if (m == MAP_FAILED)
        return 0;
    size_t *pre = malloc((size_t)nr * sizeof(size_t));
    size_t acc = 0;
    for (int64_t r = 0; r < nr; ++r) {
        pre[r] = acc;
        acc += len[r];
    }
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    mcopy_job M = {m + (off0 - pa), buf, len, pre, nr, total, 4u << 20, 0};
    atomic_init(&M.next, 0);
    gac_run_threads(gac_host_threads(), mcopy_thread, &M);
    free(pre);
    const int bad = munmap(m, mlen) != 0;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    if (getenv("GAC_TIMING"))
        fprintf(stderr, "[gac_par_output] %zu bytes copied through a mapping in %.3f s\n", total,
                (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec));
    if (fseeko(out, off0 + (off_t)total, SEEK_SET) != 0 || bad)
        return -1;
    return 1;
}

/* writev() until every byte is out (short writes, EINTR); 0 or -1 */
static int writev_all(int fd, struct iovec *iov, int n) {
    while (n > 0) {
        const ssize_t w = writev(fd, iov, n);
        if (w < 0) {
            if (errno == EINTR)
                continue;
            return -1;
        }
        size_t left = (size_t)w;
        while (n > 0 && left >= iov->iov_len) {
            left -= iov->iov_len;
            ++iov;
            --n;
        }
        if (n > 0) {
            iov->iov_base = (char *)iov->iov_base + left;
            iov->iov_len -= left;
        }
    }
    return 0;
}

/* The writer waits for run r: spin (a run is usually a few µs away) before
 * sleeping -- a usleep() per run costs the timer slack (≈50 µs), which over
 * ~1000 runs was the whole output stage (C2 chain text: 54 ms with 16
 * threads, formatting alone 7). */
static void wait_ready(_Atomic int *flag) {
    if (atomic_load_explicit(flag, memory_order_acquire))
        return;
    struct timespec t0, t;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (unsigned spin = 1;; ++spin) {
        if (atomic_load_explicit(flag, memory_order_acquire))
            return;
        __builtin_ia32_pause();
        if ((spin & 1023) == 0) {
            clock_gettime(CLOCK_MONOTONIC, &t);
            if ((t.tv_sec - t0.tv_sec) * 1000000000L + (t.tv_nsec - t0.tv_nsec) > 2000000L)
                break; /* a long wait: sleep instead */
        }
    }
    while (!atomic_load_explicit(flag, memory_order_acquire))
        usleep(20);
}

int gac_par_format(int64_t nr, void (*fn)(FILE *f, int64_t r, void *arg), void *arg, char ***bufs,
                   size_t **lens) {
    return par_format(nr, fn, NULL, arg, bufs, lens);
}

int gac_par_format_buf(int64_t nr, void (*fn)(gac_obuf *o, int64_t r, void *arg), void *arg,
                       char ***bufs, size_t **lens) {
    return par_format(nr, NULL, fn, arg, bufs, lens);
}

/* GAC_OUT_WRITERS=K (K > 1): the in-order loop below places each batch at
 * its file offset and K threads write the batches with pwritev, so a file's
 * writes are not one thread's copy into the page cache (the formatters can
 * finish well before a single writer does).  Default 1: one writev loop. */
typedef struct wbatch {
    struct iovec iov[256];
    int n;
    off_t off;
    char *owned[256]; /* run buffers to free once written */
    int n_owned;
} wbatch;

typedef struct wpool {
    int fd;
    wbatch *q; /* ring */
    int cap, head, tail, count, closing;
    pthread_mutex_t mu;
    pthread_cond_t can_put, can_take;
    _Atomic int bad;
} wpool;

static int pwritev_all(int fd, struct iovec *iov, int n, off_t off) {
    while (n > 0) {
        const ssize_t w = pwritev(fd, iov, n, off);
        if (w < 0) {
            if (errno == EINTR)
                continue;
            return -1;
        }
        if (w == 0) { /* (no progress with bytes left: an error, not a spin) */
            errno = EIO;
            return -1;
        }
        off += w;
        size_t left = (size_t)w;
        while (n > 0 && left >= iov->iov_len) {
            left -= iov->iov_len;
            ++iov;
            --n;
        }
        if (n > 0) {
            iov->iov_base = (char *)iov->iov_base + left;
            iov->iov_len -= left;
        }
    }
    return 0;
}

static void *wpool_thread(void *arg) {
    wpool *P = arg;
    wbatch b;
    for (;;) {
        pthread_mutex_lock(&P->mu);
        while (P->count == 0 && !P->closing)
            pthread_cond_wait(&P->can_take, &P->mu);
        if (P->count == 0) {
            pthread_mutex_unlock(&P->mu);
            return NULL;
        }
        b = P->q[P->head];
        P->head = (P->head + 1) % P->cap;
        --P->count;
        pthread_cond_signal(&P->can_put);
        pthread_mutex_unlock(&P->mu);
        if (!atomic_load(&P->bad) && pwritev_all(P->fd, b.iov, b.n, b.off) != 0)
            atomic_store(&P->bad, 1);
        for (int k = 0; k < b.n_owned; ++k)
            free(b.owned[k]);
    }
}

static void wpool_put(wpool *P, const wbatch *b) {
    pthread_mutex_lock(&P->mu);
    while (P->count == P->cap)
        pthread_cond_wait(&P->can_put, &P->mu);
    P->q[P->tail] = *b;
    P->tail = (P->tail + 1) % P->cap;
    ++P->count;
    pthread_cond_signal(&P->can_take);
    pthread_mutex_unlock(&P->mu);
}

static int out_writers(void) {
    const char *e = getenv("GAC_OUT_WRITERS");
    const int k = e && *e ? atoi(e) : 1;
    return k < 1 ? 1 : (k > 8 ? 8 : k);
}

static int par_output(FILE *out, int64_t nr, void (*fn)(FILE *f, int64_t r, void *arg),
                      void (*fn_buf)(gac_obuf *o, int64_t r, void *arg), void *arg) {
    if (nr <= 0)
        return 0;
    po_job J;
    J.nr = nr;
    J.fn = fn;
    J.fn_buf = fn_buf;
    J.arg = arg;
    J.buf = calloc((size_t)nr, sizeof(char *));
    J.len = calloc((size_t)nr, sizeof(size_t));
    J.ready = calloc((size_t)nr, sizeof(_Atomic int));
    atomic_init(&J.next, 0);
    atomic_init(&J.done, 0);
    atomic_init(&J.oom, 0);
    int nt = gac_host_threads() - 1;
    if (nt < 1)
        nt = 1;
    if (nt > nr)
        nt = (int)nr;
    pthread_t *th = malloc((size_t)nt * sizeof(pthread_t));
    for (int i = 0; i < nt; ++i)
        pthread_create(&th[i], NULL, po_thread, &J);
    int bad = 0;
    int64_t r = 0;
    /* a regular file and a large output (estimated from the first runs):
     * format everything, then copy through a mapping */
    const long long mmin = output_mmap_min();
    struct stat st;
    if (mmin >= 0 && fstat(fileno(out), &st) == 0 && S_ISREG(st.st_mode)) {
        const int64_t probe = nr < 2 * (int64_t)nt ? nr : 2 * (int64_t)nt;
        size_t got = 0;
        for (int64_t k = 0; k < probe; ++k) {
            wait_ready(&J.ready[k]);
            got += J.len[k];
        }
        if ((double)got / (double)probe * (double)nr >= (double)mmin) {
            size_t total = got;
            for (int64_t k = probe; k < nr; ++k) {
                wait_ready(&J.ready[k]);
                total += J.len[k];
            }
            for (int i = 0; i < nt; ++i)
                pthread_join(th[i], NULL);
            nt = 0;
            const int rc = atomic_load(&J.oom) ? 0 : par_output_mapped(out, J.buf, J.len, nr, total);
            if (rc != 0) {
                bad = rc < 0;
                for (int64_t k = 0; k < nr; ++k)
                    free(J.buf[k]);
                r = nr;
            }
        }
    }
    /* the finished runs in order, gathered into one writev() per batch (up
     * to 256 runs / 8 MB): many small runs keep the formatters' buffers
     * small and reused, one syscall per batch keeps the file write at
     * memory speed; stdio only for streams without a descriptor */
    const int fd = r < nr ? fileno(out) : -1;
    const int use_fd = fd >= 0 && fflush(out) == 0;
    const int nw = use_fd ? out_writers() : 1;
    if (nw > 1 && r < nr) {
        off_t off = lseek(fd, 0, SEEK_CUR);
        wpool P;
        memset(&P, 0, sizeof(P));
        P.fd = fd;
        P.cap = 4 * nw;
        P.q = malloc((size_t)P.cap * sizeof(wbatch));
        pthread_mutex_init(&P.mu, NULL);
        pthread_cond_init(&P.can_put, NULL);
        pthread_cond_init(&P.can_take, NULL);
        atomic_init(&P.bad, 0);
        pthread_t wt[8];
        int started = 0;
        for (int i = 0; i < nw; ++i)
            if (pthread_create(&wt[i], NULL, wpool_thread, &P) == 0)
                ++started;
        wbatch *b = malloc(sizeof(wbatch));
        while (r < nr && off >= 0 && started > 0) {
            wait_ready(&J.ready[r]);
            b->n = b->n_owned = 0;
            b->off = off;
            size_t bytes = 0;
            const int64_t r0 = r;
            while (r < nr && b->n_owned < 256 && bytes < (8u << 20) &&
                   (r == r0 || atomic_load_explicit(&J.ready[r], memory_order_acquire))) {
                if (J.len[r]) {
                    b->iov[b->n].iov_base = J.buf[r];
                    b->iov[b->n].iov_len = J.len[r];
                    bytes += J.len[r];
                    ++b->n;
                }
                b->owned[b->n_owned++] = J.buf[r];
                ++r;
            }
            off += (off_t)bytes;
            wpool_put(&P, b);
        }
        pthread_mutex_lock(&P.mu);
        P.closing = 1;
        pthread_cond_broadcast(&P.can_take);
        pthread_mutex_unlock(&P.mu);
        for (int i = 0; i < started; ++i)
            pthread_join(wt[i], NULL);
        if (atomic_load(&P.bad) || off < 0 || started == 0 || lseek(fd, off, SEEK_SET) < 0)
            bad = 1;
        for (; r < nr; ++r) { /* (only after a failure above) */
            wait_ready(&J.ready[r]);
            free(J.buf[r]);
        }
        free(b);
        free(P.q);
        pthread_mutex_destroy(&P.mu);
        pthread_cond_destroy(&P.can_put);
        pthread_cond_destroy(&P.can_take);
    }
    while (r < nr) {
        wait_ready(&J.ready[r]);
        if (!use_fd) {
            if (J.len[r] && fwrite(J.buf[r], 1, J.len[r], out) != J.len[r])
                bad = 1;
            free(J.buf[r]);
            ++r;
            continue;
        }
        struct iovec iov[256];
        int k = 0;
        size_t bytes = 0;
        const int64_t r0 = r;
        while (r < nr && k < 256 && bytes < (8u << 20) &&
               (r == r0 || atomic_load_explicit(&J.ready[r], memory_order_acquire))) {
            if (J.len[r]) {
                iov[k].iov_base = J.buf[r];
                iov[k].iov_len = J.len[r];
                bytes += J.len[r];
                ++k;
            }
            ++r;
        }
        if (!bad && writev_all(fd, iov, k) != 0)
            bad = 1;
        for (int64_t x = r0; x < r; ++x)
            free(J.buf[x]);
    }
    for (int i = 0; i < nt; ++i)
        pthread_join(th[i], NULL);
    free(th);
    free(J.buf);
    free(J.len);
    free((void *)J.ready);
    return (bad || atomic_load(&J.oom)) ? -1 : 0;
}

int gac_par_output(FILE *out, int64_t nr, void (*fn)(FILE *f, int64_t r, void *arg), void *arg) {
    return par_output(out, nr, fn, NULL, arg);
}

int gac_par_output_buf(FILE *out, int64_t nr, void (*fn)(gac_obuf *o, int64_t r, void *arg),
                       void *arg) {
    return par_output(out, nr, NULL, fn, arg);
}
