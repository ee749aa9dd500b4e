/* scoreChain -- (re)score existing chains on an MI355X.
 *
 * Drop-in for the reference's src/scoreChain/scoreChain.c: same command
 * line, options and output formats (chain, -returnOnlyScore,
 * -returnOnlyScoreAndCoords; :42-79, :301-331).  Genomes are loaded once,
 * resident 2-bit packed on the GPU; every chain's global score
 * (chainCalcScore), local score (chainCalcScoreLocal, :176-198) and aligned
 * bases are computed in one batched GPU call (gac_score_ranges). */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "gac_tool.h"
#include "gachain.h"
#include "host/gac_host.h"

static const gt_spec k_opts[] = {
    {"scoreScheme", GT_STRING},
    {"linearGap", GT_STRING},
    {"doLocalScore", GT_BOOL},
    {"forceLocalScore", GT_BOOL},
    {"returnOnlyScore", GT_BOOL},
    {"returnOnlyScoreAndCoords", GT_BOOL},
    {NULL, 0},
};

static void usage(void) {
    gt_abort(
        "scoreChain - (re)score existing chains (MI355X / libgachain)\n"
        "usage:\n"
        "   scoreChain in.chainFile reference.2bit query.2bit out.chain  -linearGap=loose|medium|filename\n"
        "Where reference.2bit and query.2bit are the names of a .2bit files for the reference and query\n"
        "options:\n"
        " Local score = we set score = 0 if score < 0 and return the max of the score that we reach for a chain\n"
        "   -returnOnlyScore             default=FALSE. Just return chain ID{tab}globalScore{tab}localScore{tab}totalAligningBases, not the entire chain\n"
        "   -returnOnlyScoreAndCoords    default=FALSE. Just return chain ID{tab}chainStartInRef{tab}chainEndInRef{tab}localScore{tab}totalAligningBases, not the entire chain\n"
        "   -doLocalScore                default=FALSE. Only if the global score of a chain is negative, compute and output the local score in the chain file.\n"
        "   -forceLocalScore             default=FALSE. Always output the local score in the chain file.\n"
        "   -scoreScheme=fileName        Read the scoring matrix from a blastz-format file\n"
        "   -linearGap=<medium|loose|filename>    Specify type of linearGap to use.\n"
        "              *Must* specify this argument to one of these choices.\n");
}

typedef struct sc_out {
    const gt_chains *c;
    const int64_t *glob, *loc;
    const int32_t *ali, *id;
    int do_local, force_local, only_score, only_coords;
} sc_out;

/* one output record (scoreChain.c:301-331) */
static void write_one(FILE *out, int64_t i, void *arg) {
    const sc_out *o = arg;
    const gt_chains *c = o->c;
    const double g = (double)o->glob[i], l = (double)o->loc[i];
    double score;
    if (o->force_local) {
        score = l;
    } else {
        score = g;
        if (score <= 0 && o->do_local)
            score = l;
    }
    if (o->only_score)
        fprintf(out, "%d\t%1.0f\t%1.0f\t%d\n", o->id[i], g, l, o->ali[i]);
    else if (o->only_coords)
        fprintf(out, "%d\t%d\t%d\t%1.0f\t%1.0f\t%d\n", o->id[i], c->tstart[i], c->tend[i], g, l,
                o->ali[i]);
    else
        gt_write_chain(out, c, i, score, o->id[i]);
}

int main(int argc, char *argv[]) {
    gt_stage("");
    gt_options(&argc, argv, k_opts);
    const char *gap_name = gt_opt_str("linearGap", NULL);
    const char *scheme_name = gt_opt_str("scoreScheme", NULL);
    const int do_local = gt_opt_exists("doLocalScore");
    const int force_local = gt_opt_exists("forceLocalScore");
    const int only_score = gt_opt_exists("returnOnlyScore");
    const int only_coords = gt_opt_exists("returnOnlyScoreAndCoords");
    if (argc != 5)
        usage();
    if (only_score && only_coords)
        gt_abort("ERROR: You cannot specify both returnOnlyScore and returnOnlyScoreAndCoords\n");

    int32_t mat[16];
    gt_check(gac_scheme_read(scheme_name, mat, NULL, NULL, NULL));
    if (gap_name == NULL)
        gt_abort("Must specify linear gap costs.  Use 'loose' or 'medium' for defaults\n");
    gac_gapcalc *gap = NULL;
    gt_check(gac_gapcalc_build(gap_name, &gap));

    const char *t2bit = argv[2], *q2bit = argv[3];
    if (!gt_file_exists(t2bit))
        gt_abort("ERROR: target 2bit file or nib directory %s does not exist\n", t2bit);
    if (!gt_file_exists(q2bit))
        gt_abort("ERROR: query 2bit file or nib directory %s does not exist\n", q2bit);
    if (!gac_is_twobit_file(t2bit))
        gt_abort("ERROR: only 2bit files are supported, not %s\n", t2bit);
    if (!gac_is_twobit_file(q2bit))
        gt_abort("ERROR: only 2bit files are supported, not %s\n", q2bit);

    /* device open + genome upload run on a helper thread beside the parse */
    gt_device dev;
    gt_stage("options + setup");
    gt_device_start(&dev, t2bit, q2bit, mat, gap);

    FILE *out = gt_must_open(argv[4], "w");
    gt_chains c;
    gt_read_chains(argv[1], &c, -HUGE_VAL, 0);
    gt_stage("read chains");
    gac_ctx *ctx = gt_device_join(&dev);
    gt_stage("device open + 2bit genomes (rest)");

    /* resolve sequence names (twoBitReadSeqFrag aborts on unknown names) */
    int32_t *tseq = malloc((c.n ? c.n : 1) * 4), *qseq = malloc((c.n ? c.n : 1) * 4);
    int32_t *tmap = gt_seq_map(ctx, GAC_T, &c.tnames), *qmap = gt_seq_map(ctx, GAC_Q, &c.qnames);
    for (int64_t i = 0; i < c.n; ++i) {
        tseq[i] = tmap[c.tname[i]];
        if (tseq[i] < 0)
            gt_abort("%s is not in %s", c.tnames.names[c.tname[i]], t2bit);
        qseq[i] = qmap[c.qname[i]];
        if (qseq[i] < 0)
            gt_abort("%s is not in %s", c.qnames.names[c.qname[i]], q2bit);
    }
    free(tmap);
    free(qmap);
    gac_chainset_desc d = {c.n, tseq, qseq, c.qstrand, c.blk_off, c.nb, c.bt, c.bq, c.bs};
    gac_chainset *cs = NULL;
    gt_check(gac_chains_upload(ctx, &d, &cs));
    gt_stage("chains to HBM");
    gac_range *r = malloc((c.n ? c.n : 1) * sizeof(gac_range));
    for (int64_t i = 0; i < c.n; ++i) {
        r[i].chain = (int32_t)i;
        r[i].t_start = c.tstart[i];
        r[i].t_end = c.tend[i];
    }
    int64_t *glob = malloc((c.n ? c.n : 1) * 8), *loc = malloc((c.n ? c.n : 1) * 8);
    int32_t *ali = malloc((c.n ? c.n : 1) * 4);
    gt_check(gac_score_ranges(ctx, cs, r, c.n, GAC_WANT_LOCAL, glob, loc, ali));
    gt_stage("GPU scoring");
    gt_device_close_async(&dev, ctx, cs); /* overlaps writing the output */

    /* chainWriteHead assigns ids to id-less chains in output order
     * (chain.c:203-204): fix them before the parallel formatting */
    int32_t *ids = malloc((c.n ? c.n : 1) * 4);
    for (int64_t i = 0; i < c.n; ++i)
        ids[i] = (c.id[i] == 0 && !only_score && !only_coords) ? gt_next_chain_id() : c.id[i];
    sc_out so = {&c, glob, loc, ali, ids, do_local, force_local, only_score, only_coords};
    gt_par_write(out, c.n, write_one, &so);
    free(ids);
    gt_careful_close(out, argv[4]);
    gt_stage("write output");
    /* host arrays are left to process exit */
    gt_device_close_join(&dev);
    gt_stage("device close (rest)");
    gt_exit_ok();
}
