/* NetFilterNonNested.perl -- native drop-in for src/NetFilterNonNested.perl
 * (the binary keeps the script's name, so callers that run it through $PATH,
 * like chainCleaner's self-netting at src/chainCleaner/chainCleaner.c:1661,
 * pick it up unchanged).
 *
 * Non-nested net filtering: a fill that fails the filter is removed together
 * with its gaps, and everything nested below it moves up two levels
 * (eraseGapsMarkSkip, :425-459); a net line is printed if any of its fills is
 * kept (output, :397-419).  Modes:
 *   "12"    -minScore1 -minSizeT1 -minSizeQ1 [-minScore2 -minSizeT2 -minSizeQ2]
 *           (:93-109; an unset set is INT_MAX)
 *   batch   -minScore a,b,.. -minSizeT .. -minSizeQ .. (:110-120)
 *   UCSC    -doUCSCSynFilter [-keepSynNetsWithScore n -keepInvNetsWithScore n]
 *           (UCSCsynFilter_nonRecursive, :268-302)
 *   score   -doScoreFilter -minScore1 n [-keepSyn.. -keepInv..] (:305-327)
 * plus -keepSynNetsWithScore / -keepInvNetsWithScore in the other modes
 * (:368-374); the type, ali and qFar fields come from netSyntenic.  -v (the
 * script's debug trace, printed into its output) is rejected.  Options
 * follow Getopt::Long: "-opt value", "-opt=value" or "--opt". */
#define _GNU_SOURCE
#include <ctype.h>
#include <limits.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>

#include "gac_netfile.h"
#include "gac_tool.h"

static void usage(void) {
    fprintf(stderr,
            "non-nested net filtering\n"
            "netFilter from the kent source removes all nested nets if the top level net does not pass the filters.\n"
            "NetFilterNonNested.perl keeps nested nets that pass the filters, even if higher level nets are excluded. The level of the nets is adjusted.\n"
            "\n"
            "Output goes to stdout\n"
            "\n"
            "NetFilterNonNested.perl input.net[.gz] [other parameters depending on filter mode]\n"
            "\tEITHER [-doUCSCSynFilter -keepSynNetsWithScore int -keepInvNetsWithScore int]\n"
            "\t    OR [-doScoreFilter -minScore1 int -keepSynNetsWithScore int -keepInvNetsWithScore int]\n"
            "\t    OR [-minScore comma-separated-string -minSizeT comma-separated-string -minSizeQ comma-separated-string]\n"
            "\t    OR [-minScore1 int -minSizeT1 int -minSizeQ1 int  -minScore2 int -minSizeT2 int -minSizeQ2 int]\n"
            "(this native build does not implement -v)\n\n");
    exit(255);
}

static int parse_int(const char *name, const char *v) {
    char *end;
    if (!v || !*v)
        usage();
    long x = strtol(v, &end, 10);
    if (*end != 0) {
        fprintf(stderr, "Value \"%s\" invalid for option %s (number expected)\n", v, name);
        usage();
    }
    return (int)x;
}

/* split "a,b,c" into doubles (perl split /,/ then numeric compare) */
static int split_nums(const char *s, double **out) {
    int n = 0, cap = 8;
    double *a = malloc(cap * sizeof(double));
    const char *p = s;
    while (*p) {
        const char *c = strchr(p, ',');
        const size_t len = c ? (size_t)(c - p) : strlen(p);
        char buf[64];
        snprintf(buf, sizeof(buf), "%.*s", (int)(len < 63 ? len : 63), p);
        if (n == cap) {
            cap *= 2;
            a = realloc(a, cap * sizeof(double));
        }
        a[n++] = atof(buf);
        if (!c)
            break;
        p = c + 1;
    }
    *out = a;
    return n;
}

int main(int argc, char *argv[]) {
    int s1 = 0, t1 = 0, q1 = 0, s2 = 0, t2 = 0, q2 = 0;
    int ucsc = 0, score_filter = 0, keep_syn = INT_MAX, keep_inv = INT_MAX;
    const char *ms = "", *mt = "", *mq = "";
    const char *input = NULL;
    static const char *unsupported[] = {"v", "verbose", NULL};
    for (int i = 1; i < argc; ++i) {
        const char *a = argv[i];
        if (a[0] != '-' || a[1] == 0) {
            if (!input)
                input = a;
            continue;
        }
        const char *name = a + 1;
        if (*name == '-')
            ++name;
        char key[64];
        const char *eq = strchr(name, '=');
        const size_t klen = eq ? (size_t)(eq - name) : strlen(name);
        snprintf(key, sizeof(key), "%.*s", (int)(klen < 63 ? klen : 63), name);
        for (int k = 0; unsupported[k]; ++k)
            if (strcasecmp(key, unsupported[k]) == 0)
                gt_abort("NetFilterNonNested: option -%s is not supported by this native build", key);
        if (strcasecmp(key, "doUCSCSynFilter") == 0 || strcasecmp(key, "doScoreFilter") == 0) {
            if (eq) { /* a boolean takes no value */
                fprintf(stderr, "Option %s does not take an argument\n", key);
                usage();
            }
            *(strcasecmp(key, "doUCSCSynFilter") == 0 ? &ucsc : &score_filter) = 1;
            continue;
        }
        const char *val = eq ? eq + 1 : (i + 1 < argc ? argv[++i] : NULL);
        if (strcasecmp(key, "keepSynNetsWithScore") == 0)
            keep_syn = parse_int(key, val);
        else if (strcasecmp(key, "keepInvNetsWithScore") == 0)
            keep_inv = parse_int(key, val);
        else if (strcasecmp(key, "minScore1") == 0)
            s1 = parse_int(key, val);
        else if (strcasecmp(key, "minSizeT1") == 0)
            t1 = parse_int(key, val);
        else if (strcasecmp(key, "minSizeQ1") == 0)
            q1 = parse_int(key, val);
        else if (strcasecmp(key, "minScore2") == 0)
            s2 = parse_int(key, val);
        else if (strcasecmp(key, "minSizeT2") == 0)
            t2 = parse_int(key, val);
        else if (strcasecmp(key, "minSizeQ2") == 0)
            q2 = parse_int(key, val);
        else if (strcasecmp(key, "minScore") == 0 && val)
            ms = val;
        else if (strcasecmp(key, "minSizeT") == 0 && val)
            mt = val;
        else if (strcasecmp(key, "minSizeQ") == 0 && val)
            mq = val;
        else {
            fprintf(stderr, "Unknown option: %s\n", key);
            usage();
        }
    }
    if (!input)
        usage();
    if (score_filter && s1 == 0)
        gt_abort("ERROR: you have to set -minScore1 with -doScoreFilter");
    int mode12 = s1 || t1 || q1 || s2 || t2 || q2;
    int batch = *ms || *mt || *mq;
    if (batch && mode12)
        gt_abort("ERROR: you have used BOTH batch filtering (minScore/minSizeT/minSizeQ) AND individual filtering (minScore1/minSizeT1/minSizeQ1 etc)\n\n"
                 "\t\t     USE Either batch or individual");
    gt_lines in, out;
    gt_lines_read(input, &in);
    gt_netfilter_opts o = {0, NULL, NULL, NULL, ucsc, score_filter, s1, keep_syn, keep_inv};
    double sc[2], ts[2], qs[2], *a = NULL, *b = NULL, *c = NULL;
    if (mode12) { /* an unset set is INT_MAX (:96-108) */
        if (s2 == 0 && t2 == 0 && q2 == 0)
            s2 = t2 = q2 = INT_MAX;
        if (s1 == 0 && t1 == 0 && q1 == 0)
            s1 = t1 = q1 = INT_MAX;
        sc[0] = s1, ts[0] = t1, qs[0] = q1, sc[1] = s2, ts[1] = t2, qs[1] = q2;
        o.nsets = 2;
        o.set_score = sc, o.set_t = ts, o.set_q = qs;
    } else if (batch) {
        const int na = split_nums(ms, &a), nb = split_nums(mt, &b), nc = split_nums(mq, &c);
        if (na != nb)
            gt_abort("ERROR: number of minScores differ from minTsizes");
        if (na != nc)
            gt_abort("ERROR: number of minScores differ from minQsizes");
        o.nsets = na;
        o.set_score = a, o.set_t = b, o.set_q = c;
    }
    gt_netfilter(&in, input, &o, &out);
    free(a);
    free(b);
    free(c);
    for (int64_t i = 0; i < out.n; ++i) {
        fputs(out.line[i], stdout);
        fputc('\n', stdout);
    }
    if (fflush(stdout) != 0)
        gt_abort("write error on stdout");
    return 0;
}
