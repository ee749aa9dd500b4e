/* gac_netfile.h -- .net text for the drop-in tools (C11):
 *  - the kent net reader's tree (chainNetRead / cnFillRead,
 *    kent/src/hg/lib/chainNet.c:152-265): nesting by leading-space count,
 *    a line is a fill if it carries a non-zero "id", a gap otherwise;
 *  - NetFilterNonNested.perl's two-set score/size filter ("12" mode,
 *    src/NetFilterNonNested.perl:93-172,330-459), which chainCleaner runs on
 *    its own chainNet output (src/chainCleaner/chainCleaner.c:1656-1660). */
#ifndef GAC_NETFILE_H
#define GAC_NETFILE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* text lines of a file (newline-terminated lines, '\n' stripped) */
typedef struct gt_lines {
    char **line;
    int64_t n, cap;
    char *buf; /* owns the text when read from a file */
} gt_lines;
void gt_lines_read(const char *path, gt_lines *l);
void gt_lines_push(gt_lines *l, char *s); /* takes ownership of malloc'd s */
void gt_lines_free(gt_lines *l);

/* One fill or gap; children / next are indices into gt_netset.fills (-1 = none). */
typedef struct gt_fill {
    int32_t tstart, tsize;
    int32_t chain_id; /* 0 = gap */
    double score;
    int32_t child, next;
} gt_fill;

typedef struct gt_net1 {
    char *name;
    int32_t size;
    int32_t first; /* first top-level fill */
} gt_net1;

typedef struct gt_netset {
    gt_net1 *nets;
    int32_t n, cap;
    gt_fill *fills;
    int64_t nf, fcap;
} gt_netset;

/* Parse nets from text lines (blank and '#' lines skipped, like
 * lineFileNextReal).  `what` names the source in error messages. */
void gt_net_parse(const gt_lines *l, const char *what, gt_netset *ns);
void gt_netset_free(gt_netset *ns);

/* NetFilterNonNested.perl "12" mode: keep a fill if (score >= s1 && tSize >=
 * t1 && qSize >= q1) || (score >= s2 && tSize >= t2 && qSize >= q2); the gaps
 * of a removed fill go with it and everything nested below it moves up two
 * levels; a net line is printed only if one of its fills is kept.  Set 2
 * defaults to INT_MAX when not given (as the script does).  Returns the
 * filtered lines (new strings). */
void gt_netfilter_nonnested(const gt_lines *in, const char *what, double s1, double t1,
                            double q1, double s2, double t2, double q2, gt_lines *out);
/* the same filter with any number of (score, tSize, qSize) sets: a fill is
 * kept if it passes all three thresholds of at least one set ("batch" mode,
 * NetFilterNonNested.perl:368-374; "12" mode is two sets) */
void gt_netfilter_sets(const gt_lines *in, const char *what, int nsets, const double *set_score,
                       const double *set_t, const double *set_q, gt_lines *out);

/* All of NetFilterNonNested.perl's filter modes (:87-120, :268-396):
 *   ucsc          -doUCSCSynFilter: UCSC netFilter -syn thresholds, non-nested
 *   score_filter  -doScoreFilter: keep score >= min_score1, plus syn/inv nets
 *   keep_syn/inv  -keepSynNetsWithScore / -keepInvNetsWithScore (INT_MAX: off)
 *   sets          the "12" / batch (score, tSize, qSize) sets (nsets 0: none;
 *                 a fill then reaching that test is an error, as in the script)
 * The type / ali / qFar fields come from netSyntenic's fill lines. */
typedef struct gt_netfilter_opts {
    int nsets;
    const double *set_score, *set_t, *set_q;
    int ucsc, score_filter;
    double min_score1, keep_syn, keep_inv;
} gt_netfilter_opts;
void gt_netfilter(const gt_lines *in, const char *what, const gt_netfilter_opts *o, gt_lines *out);

#ifdef __cplusplus
}
#endif
#endif
