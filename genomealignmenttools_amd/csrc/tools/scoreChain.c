/* scoreChain -- (re)score existing chains on an MI355X.
 *
 * Drop-in for the reference's src/scoreChain/scoreChain.c: same command
 * line, options and output formats (chain, -returnOnlyScore,
 * -returnOnlyScoreAndCoords; :42-79, :301-331).  Genomes are loaded once,
 * resident 2-bit packed on the GPU; every chain's global score
 * (chainCalcScore), local score (chainCalcScoreLocal, :176-198) and aligned
 * bases are computed in one batched GPU call (gac_score_chains).
 *
 * -nranks=N -rank=R: chains are independent, so N processes (one per GPU)
 * each parse the file, score a contiguous run of chains balanced by blocks
 * and format it into a part; rank 0 appends the parts to its own run in
 * order (no collective: the output is the exchange). */
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
    {"nranks", GT_INT},
    {"rank", GT_INT},
    {"gpu", GT_INT},
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
        "              *Must* specify this argument to one of these choices.\n"
        "   -nranks=N -rank=R            multi-GPU run (one process per GPU, same node): rank R scores\n"
        "                                its contiguous share of the chains; rank 0 writes the output\n"
        "   -gpu=D                       device index (default: R with -nranks, else 0)\n");
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

    gt_ranks rk;
    gt_ranks_init(&rk, gt_opt_int("nranks", 1), gt_opt_int("rank", 0), argv[4]);
    const int multi = rk.n > 1;
    if (multi && !strcmp(argv[4], "stdout"))
        gt_abort("-nranks needs an output file name (not stdout)");
    gt_set_gpu(gt_opt_int("gpu", multi ? rk.me : 0));
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

    char part[4096], part_tmp[4096];
    gt_part_name(part, sizeof(part), argv[4], rk.me, "");
    gt_part_name(part_tmp, sizeof(part_tmp), argv[4], rk.me, ".tmp");
    FILE *out = gt_must_open(multi && rk.me > 0 ? part_tmp : argv[4], "w");
    gt_chains c;
    gt_read_chains(argv[1], &c, -HUGE_VAL, 0);
    gt_stage("read chains");
    /* this rank's chains: [c0, c1), runs of about equal block counts */
    int64_t c0 = 0, c1 = c.n;
    if (multi) {
        const int64_t nb = c.blk_off[c.n];
        int64_t lo = 0, hi = c.n;
        while (lo < hi) { /* first chain whose blocks start at or past me/n */
            const int64_t m = (lo + hi) >> 1;
            if (c.blk_off[m] * rk.n < nb * rk.me) lo = m + 1;
            else hi = m;
        }
        c0 = lo;
        lo = c0, hi = c.n;
        while (lo < hi) {
            const int64_t m = (lo + hi) >> 1;
            if (c.blk_off[m] * rk.n < nb * (rk.me + 1)) lo = m + 1;
            else hi = m;
        }
        c1 = rk.me == rk.n - 1 ? c.n : lo;
    }
    const int64_t nc = c1 - c0, bo = c.blk_off[c0];
    gac_ctx *ctx = gt_device_join(&dev);
    gt_stage("device open + 2bit genomes (rest)");

    /* resolve sequence names (twoBitReadSeqFrag aborts on unknown names) */
    int32_t *tseq = malloc((nc ? nc : 1) * 4), *qseq = malloc((nc ? nc : 1) * 4);
    int32_t *tmap = gt_seq_map(ctx, GAC_T, &c.tnames), *qmap = gt_seq_map(ctx, GAC_Q, &c.qnames);
    for (int64_t i = c0; i < c1; ++i) {
        tseq[i - c0] = tmap[c.tname[i]];
        if (tseq[i - c0] < 0)
            gt_abort("%s is not in %s", c.tnames.names[c.tname[i]], t2bit);
        qseq[i - c0] = qmap[c.qname[i]];
        if (qseq[i - c0] < 0)
            gt_abort("%s is not in %s", c.qnames.names[c.qname[i]], q2bit);
    }
    free(tmap);
    free(qmap);
    int64_t *boff = c.blk_off + c0; /* rebased offsets of this rank's run */
    if (c0) {
        boff = malloc((size_t)(nc + 1) * 8);
        for (int64_t i = 0; i <= nc; ++i)
            boff[i] = c.blk_off[c0 + i] - bo;
    }
    gac_chainset_desc d = {nc, tseq, qseq, c.qstrand + c0, boff, c.blk_off[c1] - bo,
                           c.bt + bo, c.bq + bo, c.bs + bo};
    gac_chainset *cs = NULL;
    gt_check(gac_chains_upload(ctx, &d, &cs));
    gt_stage("chains to HBM");
    /* results indexed like the chains (this rank's run filled): every chain
     * of the uploaded set, whole (gac_score_chains) */
    int64_t *glob = malloc((c.n ? c.n : 1) * 8), *loc = malloc((c.n ? c.n : 1) * 8);
    int32_t *ali = malloc((c.n ? c.n : 1) * 4);
    gt_check(gac_score_chains(ctx, cs, GAC_WANT_LOCAL, glob + c0, loc + c0, ali + c0));
    gt_stage("GPU scoring");
    gt_device_close_async(&dev, ctx, cs); /* overlaps writing the output */

    /* chainWriteHead assigns ids to id-less chains in output order
     * (chain.c:203-204): fix them before the parallel formatting */
    int32_t *ids = malloc((c.n ? c.n : 1) * 4);
    for (int64_t i = 0; i < c.n; ++i)
        ids[i] = (c.id[i] == 0 && !only_score && !only_coords) ? gt_next_chain_id() : c.id[i];
    sc_out so = {&c, glob + c0, loc + c0, ali + c0, ids + c0, do_local, force_local, only_score,
                 only_coords};
    sc_out *sp = &so;
    gt_chains cv = c; /* chain fields seen from c0 */
    if (c0) {
        cv.score += c0, cv.tname += c0, cv.tsize += c0, cv.tstart += c0, cv.tend += c0;
        cv.qname += c0, cv.qsize += c0, cv.qstart += c0, cv.qend += c0, cv.qstrand += c0;
        cv.id += c0, cv.blk_off += c0;
        so.c = &cv;
    }
    gt_par_write(out, nc, write_one, sp);
    free(ids);
    if (multi && rk.me > 0) {
        gt_careful_close(out, part_tmp);
        if (rename(part_tmp, part) != 0)
            gt_abort("can't rename %s", part_tmp);
    } else {
        if (multi) {
            gt_ranks_wait(&rk, argv[4]);
            gt_stage("wait for ranks");
            gt_ranks_append_parts(&rk, argv[4], out);
        }
        gt_careful_close(out, argv[4]);
    }
    gt_stage("write output");
    gt_chains_drop_pages(&c); /* (the rest of the host arrays is left to process exit) */
    gt_device_close_join(&dev);
    gt_stage("device close (rest)");
    gt_ranks_done(&rk);
    gt_exit_ok();
}
