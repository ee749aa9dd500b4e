/* gac_netfile.c -- .net text: kent net reader tree and NetFilterNonNested
 * (see gac_netfile.h for the reference semantics restated here). */
#define _GNU_SOURCE
#include "gac_netfile.h"

#include <ctype.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdatomic.h>
#include <string.h>

#include "gac_tool.h"
#include "host/gac_host.h"

/* ------------------------------------------------------------ lines */
void gt_lines_push(gt_lines *l, char *s) {
    if (l->n == l->cap) {
        l->cap = l->cap ? l->cap * 2 : 1024;
        l->line = realloc(l->line, (size_t)l->cap * sizeof(char *));
    }
    l->line[l->n++] = s;
}

void gt_lines_read(const char *path, gt_lines *l) {
    memset(l, 0, sizeof(*l));
    FILE *f = gt_must_open(path, "r");
    size_t cap = 1 << 20, len = 0;
    char *buf = malloc(cap + 1);
    size_t r;
    while ((r = fread(buf + len, 1, cap - len, f)) > 0) {
        len += r;
        if (len == cap) {
            cap *= 2;
            buf = realloc(buf, cap + 1);
        }
    }
    if (f != stdin)
        fclose(f);
    buf[len] = 0;
    l->buf = buf;
    char *p = buf, *end = buf + len;
    while (p < end) {
        char *nl = memchr(p, '\n', end - p);
        if (nl)
            *nl = 0;
        if (l->n == l->cap) {
            l->cap = l->cap ? l->cap * 2 : 1024;
            l->line = realloc(l->line, (size_t)l->cap * sizeof(char *));
        }
        l->line[l->n++] = p;
        p = nl ? nl + 1 : end;
    }
}

void gt_lines_free(gt_lines *l) {
    if (!l->buf)
        for (int64_t i = 0; i < l->n; ++i)
            free(l->line[i]);
    free(l->line);
    free(l->buf);
    memset(l, 0, sizeof(*l));
}

/* ------------------------------------------------------------ net tree */
/* Every line is classified and parsed as a fill/gap line on all threads
 * first (pre_line); the tree is then built by the reference's recursion in
 * one serial pass that only reads those records.  A line the fast parse
 * cannot settle (or an error) goes through fill_from_line as before, which
 * aborts with the reference's message at the same point of the serial
 * pass. */
typedef struct pre_line {
    int32_t lead;    /* leading spaces */
    uint8_t real;    /* lineFileNextReal keeps it */
    uint8_t ok;      /* fill record parsed (else: fill_from_line decides) */
    gt_fill f;
} pre_line;

typedef struct reader {
    const gt_lines *l;
    int64_t pos;
    const char *what;
    gt_netset *ns;
    const pre_line *pre; /* NULL: parse lines as they come */
} reader;

/* lineFileNextReal: skip blank lines and lines whose first non-blank is '#' */
static char *next_real(reader *r) {
    while (r->pos < r->l->n) {
        if (r->pre) {
            const int64_t i = r->pos++;
            if (r->pre[i].real)
                return r->l->line[i];
            continue;
        }
        char *s = r->l->line[r->pos++];
        const char *p = s;
        while (isspace((unsigned char)*p))
            ++p;
        if (*p != 0 && *p != '#')
            return s;
    }
    return NULL;
}

static int32_t need_num(reader *r, char **w, int i) {
    char *end;
    long v = strtol(w[i], &end, 10);
    if (*w[i] == 0 || *end != 0)
        gt_abort("Expecting number field %d line %lld of %s, got %s", i + 1, (long long)r->pos,
                 r->what, w[i]);
    return (int32_t)v;
}

/* cnFillFromLine (chainNet.c:86-150): the fields chainCleaner uses */
static int32_t fill_from_line(reader *r, char *line) {
    if (r->pre && r->pre[r->pos - 1].ok) { /* (parsed on the threads) */
        gt_netset *ns = r->ns;
        if (ns->nf == ns->fcap) {
            ns->fcap = ns->fcap ? ns->fcap * 2 : 4096;
            ns->fills = realloc(ns->fills, (size_t)ns->fcap * sizeof(gt_fill));
        }
        ns->fills[ns->nf] = r->pre[r->pos - 1].f;
        return (int32_t)ns->nf++;
    }
    char *w[64];
    char *copy = strdup(line);
    int wc = gac_chop_white(copy, w, 64);
    if (wc < 7)
        gt_abort("Expecting 7 words line %lld of %s got %d", (long long)r->pos, r->what, wc);
    gt_netset *ns = r->ns;
    if (ns->nf == ns->fcap) {
        ns->fcap = ns->fcap ? ns->fcap * 2 : 4096;
        ns->fills = realloc(ns->fills, (size_t)ns->fcap * sizeof(gt_fill));
    }
    gt_fill *f = &ns->fills[ns->nf];
    memset(f, 0, sizeof(*f));
    f->child = f->next = -1;
    f->tstart = need_num(r, w, 1);
    f->tsize = need_num(r, w, 2);
    need_num(r, w, 5);
    need_num(r, w, 6);
    for (int i = 7; i < wc; i += 2) {
        if (i + 1 >= wc)
            break;
        if (strcmp(w[i], "score") == 0)
            f->score = atof(w[i + 1]);
        else if (strcmp(w[i], "type") == 0)
            ;
        else {
            int32_t v = need_num(r, w, i + 1);
            if (strcmp(w[i], "id") == 0)
                f->chain_id = v;
        }
    }
    free(copy);
    return (int32_t)ns->nf++;
}

static int lead_spaces(const char *s) {
    int d = 0;
    while (s[d] == ' ')
        ++d;
    return d;
}

/* need_num's test on a token: the whole token is a decimal long (strtol) */
static int tok_num(const char *t, int len, int32_t *v) {
    char b[64];
    if (len <= 0 || len >= (int)sizeof(b))
        return 0;
    memcpy(b, t, (size_t)len);
    b[len] = 0;
    char *end;
    const long x = strtol(b, &end, 10);
    if (*end != 0)
        return 0;
    *v = (int32_t)x;
    return 1;
}

/* fill_from_line's fields without the copy: 1 = parsed exactly as it
 * would; 0 = let fill_from_line handle it (errors, odd tokens) */
static int fast_fill(const char *line, gt_fill *f) {
    const char *w[64];
    int wl[64], wc = 0;
    const char *p = line;
    while (wc < 64) { /* gac_chop_white */
        while (*p && isspace((unsigned char)*p))
            ++p;
        if (*p == 0)
            break;
        w[wc] = p;
        while (*p && !isspace((unsigned char)*p))
            ++p;
        wl[wc] = (int)(p - w[wc]);
        ++wc;
    }
    if (wc < 7)
        return 0;
    memset(f, 0, sizeof(*f));
    f->child = f->next = -1;
    int32_t v;
    if (!tok_num(w[1], wl[1], &f->tstart) || !tok_num(w[2], wl[2], &f->tsize) ||
        !tok_num(w[5], wl[5], &v) || !tok_num(w[6], wl[6], &v))
        return 0;
    for (int i = 7; i < wc; i += 2) {
        if (i + 1 >= wc)
            break;
        if (wl[i] == 5 && memcmp(w[i], "score", 5) == 0) {
            char b[64];
            if (wl[i + 1] >= (int)sizeof(b))
                return 0;
            memcpy(b, w[i + 1], (size_t)wl[i + 1]);
            b[wl[i + 1]] = 0;
            f->score = atof(b);
        } else if (wl[i] == 4 && memcmp(w[i], "type", 4) == 0) {
        } else {
            if (!tok_num(w[i + 1], wl[i + 1], &v))
                return 0;
            if (wl[i] == 2 && memcmp(w[i], "id", 2) == 0)
                f->chain_id = v;
        }
    }
    return 1;
}

typedef struct pre_job {
    const gt_lines *l;
    pre_line *pre;
    int64_t per;
    _Atomic int64_t next;
} pre_job;

static void *pre_thread(void *arg) {
    pre_job *J = arg;
    for (;;) {
        const int64_t a = atomic_fetch_add(&J->next, 1) * J->per;
        if (a >= J->l->n)
            return NULL;
        const int64_t b = a + J->per < J->l->n ? a + J->per : J->l->n;
        for (int64_t i = a; i < b; ++i) {
            const char *s = J->l->line[i];
            pre_line *x = &J->pre[i];
            const char *q = s;
            while (isspace((unsigned char)*q))
                ++q;
            x->real = *q != 0 && *q != '#';
            x->lead = lead_spaces(s);
            x->ok = x->real && x->lead > 0 && fast_fill(s, &x->f);
        }
    }
}

/* cnFillRead (chainNet.c:152-178) */
static int32_t read_list(reader *r) {
    int depth = 0;
    int32_t head = -1, tail = -1, fill = -1;
    for (;;) {
        char *line = next_real(r);
        if (!line)
            break;
        const int d = r->pre ? r->pre[r->pos - 1].lead : lead_spaces(line);
        if (fill < 0)
            depth = d;
        if (d < depth) {
            --r->pos; /* lineFileReuse */
            break;
        }
        if (d > depth) {
            --r->pos;
            const int32_t c = read_list(r);
            r->ns->fills[fill].child = c;
        } else {
            fill = fill_from_line(r, line);
            if (tail < 0)
                head = fill;
            else
                r->ns->fills[tail].next = fill;
            tail = fill;
        }
    }
    return head;
}

void gt_net_parse(const gt_lines *l, const char *what, gt_netset *ns) {
    memset(ns, 0, sizeof(*ns));
    reader r = {l, 0, what, ns, NULL};
    pre_line *pre = NULL;
    if (l->n >= 65536 && !getenv("GAC_NET_PARSE_SERIAL")) {
        pre = malloc((size_t)l->n * sizeof(pre_line));
        pre_job J = {l, pre, 8192, 0};
        atomic_init(&J.next, 0);
        gac_run_threads(gt_threads(), pre_thread, &J);
        r.pre = pre;
    }
    char *line;
    while ((line = next_real(&r)) != NULL) {
        if (strncmp(line, "net ", 4) != 0)
            gt_abort("Expecting 'net' first word of line %lld of %s", (long long)r.pos, what);
        char *w[3];
        char *copy = strdup(line);
        int wc = gac_chop_white(copy, w, 3);
        if (wc < 3)
            gt_abort("Expecting 3 words line %lld of %s got %d", (long long)r.pos, what, wc);
        if (ns->n == ns->cap) {
            ns->cap = ns->cap ? ns->cap * 2 : 64;
            ns->nets = realloc(ns->nets, (size_t)ns->cap * sizeof(gt_net1));
        }
        gt_net1 *n = &ns->nets[ns->n++];
        n->name = strdup(w[1]);
        n->size = need_num(&r, w, 2);
        free(copy);
        n->first = read_list(&r);
    }
    free(pre);
}

void gt_netset_free(gt_netset *ns) {
    for (int32_t i = 0; i < ns->n; ++i)
        free(ns->nets[i].name);
    free(ns->nets);
    free(ns->fills);
    memset(ns, 0, sizeof(*ns));
}

/* ------------------------------------------------------------ NetFilterNonNested */
/* the script's fill/gap pattern /^([ ]+)([fill|gap].*)/: spaces, then one of
 * the characters f i l | g a p; returns the space count or -1 */
static int level_of(const char *s) {
    int d = lead_spaces(s);
    if (d == 0 || !strchr("fil|gap", s[d]) || s[d] == 0)
        return -1;
    return d;
}

/* Perl's numeric value of a decimal field (as used by the script's >=) */
static double field_num(const char *s) { return atof(s); }

void gt_netfilter_nonnested(const gt_lines *in, const char *what, double s1, double t1,
                            double q1, double s2, double t2, double q2, gt_lines *out) {
    /* mode "12": an unset set 2 (all zero) -> INT_MAX; an unset set 1 -> INT_MAX */
    if (s2 == 0 && t2 == 0 && q2 == 0)
        s2 = t2 = q2 = INT_MAX;
    if (s1 == 0 && t1 == 0 && q1 == 0)
        s1 = t1 = q1 = INT_MAX;
    const double sc[2] = {s1, s2}, ts[2] = {t1, t2}, qs[2] = {q1, q2};
    gt_netfilter_sets(in, what, 2, sc, ts, qs, out);
}

void gt_netfilter_sets(const gt_lines *in, const char *what, int nsets, const double *set_score,
                       const double *set_t, const double *set_q, gt_lines *out) {
    gt_netfilter_opts o = {nsets, set_score, set_t, set_q, 0, 0, 0, INT_MAX, INT_MAX};
    gt_netfilter(in, what, &o, out);
}

/* first match of /<key>(X+) / in s (X: \w or \d) -- or, with at_end, of
 * /<key>(X+)$/; the value as a string in buf */
static int find_field(const char *s, const char *key, int word, int at_end, char *buf,
                      size_t cap) {
    const size_t kl = strlen(key);
    for (const char *p = strstr(s, key); p; p = strstr(p + 1, key)) {
        const char *v = p + kl, *q = v;
        while (*q && (word ? (isalnum((unsigned char)*q) || *q == '_') : isdigit((unsigned char)*q)))
            ++q;
        if (q == v || (at_end ? *q != 0 : *q != ' '))
            continue;
        snprintf(buf, cap, "%.*s", (int)(q - v), v);
        return 1;
    }
    return 0;
}

/* Level2IsSkipped (a perl hash: absent = 0) */
typedef struct lvmap {
    char *v;
    int n;
} lvmap;

static int lv_get(const lvmap *m, int k) { return k >= 0 && k < m->n ? m->v[k] : 0; }

static void lv_set(lvmap *m, int k, int x) {
    if (k < 0)
        return;
    if (k >= m->n) {
        const int n2 = k + 64;
        m->v = realloc(m->v, (size_t)n2);
        memset(m->v + m->n, 0, (size_t)(n2 - m->n));
        m->n = n2;
    }
    m->v[k] = (char)x;
}

/* testInvSynNet (:330-361) */
static int inv_syn_ok(const gt_netfilter_opts *o, const lvmap *skipped, double score,
                      const char *type, int level) {
    if (lv_get(skipped, level - 2) != 0)
        return 0;
    if (strcmp(type, "inv") == 0)
        return score >= o->keep_inv;
    if (strcmp(type, "syn") == 0)
        return score >= o->keep_syn;
    return 0;
}

/* passesFilter (:365-396) with UCSCsynFilter_nonRecursive (:268-302) and
 * scoreFilter_nonRecursive (:305-327) */
static int passes(const gt_netfilter_opts *o, const lvmap *skipped, double score, double tsz,
                  double qsz, const char *type, double ali, double qfar, int level) {
    if (o->ucsc) {
        if (!*type)
            gt_abort("No type field, please run input net through netSyntenic");
        if (score >= 200000 && tsz >= 20000 && ali >= 10000) /* minSynScore/Size/Ali */
            return 1;
        if (strcmp(type, "top") == 0)
            return score >= 300000; /* minTopScore */
        if (strcmp(type, "nonSyn") == 0)
            return 0;
        if (qfar > 200000) /* maxFar */
            return 0;
        return inv_syn_ok(o, skipped, score, type, level);
    }
    if (o->score_filter) {
        if (!*type)
            gt_abort("No type field, please run input net through netSyntenic");
        if (score >= o->min_score1)
            return 1;
        if (strcmp(type, "top") == 0 || strcmp(type, "nonSyn") == 0)
            return 0;
        return inv_syn_ok(o, skipped, score, type, level);
    }
    if (strcmp(type, "syn") == 0 && score >= o->keep_syn)
        return 1;
    if (strcmp(type, "inv") == 0 && score >= o->keep_inv)
        return 1;
    if (o->nsets == 0)
        gt_abort("ERROR: unknown value for filterMode \n");
    for (int k = 0; k < o->nsets; ++k)
        if (score >= o->set_score[k] && tsz >= o->set_t[k] && qsz >= o->set_q[k])
            return 1;
    return 0;
}

void gt_netfilter(const gt_lines *in, const char *what, const gt_netfilter_opts *o,
                  gt_lines *out) {
    memset(out, 0, sizeof(*out));
    const int64_t n = in->n;
    char *skip = calloc(n ? n : 1, 1);
    int *minus = calloc(n ? n : 1, sizeof(int));
    const int want_type = o->keep_syn < INT_MAX || o->keep_inv < INT_MAX || o->ucsc;
    lvmap skipped = {NULL, 0};
    int max_level = 1;
    /* the script keys its per-net counter by the net line's text */
    gt_names netkey;
    memset(&netkey, 0, sizeof(netkey));
    int64_t *kept = calloc(n ? n : 1, sizeof(int64_t)); /* per distinct net line */
    int64_t i = 0;
    for (; i < n; ++i) {
        if (in->line[i][0] == '#')
            continue;
        if (strncmp(in->line[i], "net ", 4) != 0)
            gt_abort("ERROR: expect file to start with net, but got this line instead: %s\n",
                     in->line[i]);
        break;
    }
    int64_t cur = 0;
    if (i < n) {
        cur = gt_names_add(&netkey, in->line[i], strlen(in->line[i]));
        kept[cur] = 0;
    }
    for (int64_t k = i + 1; k < n; ++k) {
        const char *line = in->line[k];
        if (strstr(line, " gap "))
            continue;
        if (strncmp(line, "net ", 4) == 0) {
            cur = gt_names_add(&netkey, line, strlen(line));
            kept[cur] = 0;
            continue;
        }
        const int level = level_of(line);
        if (level < 0)
            gt_abort("ERROR: expect fill or gap in %s\n", line);
        if (!strstr(line, " fill "))
            continue;
        const char *rest = line + level;
        const char *sc = strstr(rest, "score ");
        /* /score (\d+) /: digits followed by a space */
        double score = -1;
        while (sc) {
            const char *p = sc + 6;
            const char *q = p;
            while (isdigit((unsigned char)*q))
                ++q;
            if (q > p && *q == ' ') {
                score = atof(p);
                break;
            }
            sc = strstr(sc + 1, "score ");
        }
        if (score < 0)
            gt_abort("ERROR: no score field is given in this fill line: %s\n", rest);
        /* split / / of the rest: f[2] = tSize, f[6] = qSize */
        char *copy = strdup(rest);
        char *f[8] = {0};
        int nf = 0;
        for (char *tok = copy;;) {
            char *sp = strchr(tok, ' ');
            if (nf < 8)
                f[nf] = tok;
            ++nf;
            if (!sp)
                break;
            *sp = 0;
            tok = sp + 1;
        }
        const double tsz = nf > 2 ? field_num(f[2]) : 0, qsz = nf > 6 ? field_num(f[6]) : 0;
        free(copy);
        char type[64] = "", num[64];
        if (want_type && !find_field(rest, "type ", 1, 0, type, sizeof(type)) &&
            !find_field(rest, "type ", 1, 1, type, sizeof(type)))
            gt_abort("ERROR: parameter -keepSynNetsWithScore/-keepInvNetsWithScore-doUCSCSynFilter is given, but I cannot parse the net type from this fill line: %s\n",
                     rest);
        double ali = 0, qfar = 0;
        if (o->ucsc) {
            if (!find_field(rest, "ali ", 0, 0, num, sizeof(num)))
                gt_abort("ERROR: parameter -doUCSCSynFilter is given, but I cannot parse the ali filed from this fill line: %s\n",
                         rest);
            ali = atof(num);
            if (strcmp(type, "inv") == 0 || strcmp(type, "syn") == 0) {
                if (!find_field(rest, "qFar ", 0, 0, num, sizeof(num)))
                    gt_abort("ERROR: parameter -doUCSCSynFilter is given, but I cannot parse the qFar filed from this syn/inv fill line: %s\n",
                             rest);
                qfar = atof(num);
            }
        }
        if (max_level < level)
            max_level = level;
        if (passes(o, &skipped, score, tsz, qsz, type, ali, qfar, level)) {
            kept[cur]++;
            for (int l = level; l <= max_level; ++l) /* resetLevel2IsSkipped */
                lv_set(&skipped, l, 0);
        } else {
            lv_set(&skipped, level, 1);
            skip[k] = 1;
            /* eraseGapsMarkSkip(k + 1, level) */
            for (int64_t j = k + 1; j < n; ++j) {
                const char *lj = in->line[j];
                if (strncmp(lj, "net ", 4) == 0)
                    break;
                const int cl = level_of(lj);
                if (cl < 0)
                    gt_abort("ERROR: expect fill or gap in %s\n", lj);
                if (cl <= level)
                    break;
                if (cl == level + 1)
                    skip[j] = 1;
                else
                    minus[j] += 2;
            }
        }
    }
    (void)what;
    /* output(): net lines if a fill of theirs is kept, then kept fill/gap
     * lines re-indented */
    for (int64_t k = 0; k < n; ++k) {
        const char *line = in->line[k];
        if (strncmp(line, "net ", 4) == 0) {
            const int32_t key = gt_names_find(&netkey, line);
            if (key >= 0 && kept[key] > 0)
                gt_lines_push(out, strdup(line));
        }
        if (!skip[k]) {
            const int level = level_of(line);
            if (level >= 0) {
                const int cl = level - minus[k];
                const char *rest = line + level;
                const size_t rl = strlen(rest);
                char *s = malloc((size_t)(cl > 0 ? cl : 0) + rl + 1);
                int p = 0;
                for (; p < cl; ++p)
                    s[p] = ' ';
                memcpy(s + p, rest, rl + 1);
                gt_lines_push(out, s);
            }
        }
    }
    free(skip);
    free(minus);
    free(kept);
    free(skipped.v);
    gt_names_free(&netkey);
}
