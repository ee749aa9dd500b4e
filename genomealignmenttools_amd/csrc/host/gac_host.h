/* gac_host.h -- internal host-side (C11) helpers of libgachain: error state,
 * file mapping, word splitting, 2bit index, gap-table and score-matrix
 * parsing.  Not part of the public ABI (see include/gachain.h). */
#ifndef GAC_HOST_H
#define GAC_HOST_H

#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include "gachain.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ---- errors: thread-local last message ---- */
int gac_fail(int code, const char *fmt, ...)
#ifdef __GNUC__
    __attribute__((format(printf, 2, 3)))
#endif
    ;
void gac_clear_error(void);

/* ---- read-only whole-file mapping ---- */
typedef struct gac_map {
    const uint8_t *data;
    size_t size;
    int fd;
    int mapped; /* 1 = mmap, 0 = heap (pipes / stdin) */
} gac_map;
int gac_map_file(const char *path, gac_map *m);
void gac_unmap_file(gac_map *m);

/* ---- line / word helpers (kent chopByWhite semantics) ---- */
/* Split s (modified in place) on whitespace into at most max words. */
int gac_chop_white(char *s, char **words, int max);
/* Case-insensitive string equality (kent sameWord). */
int gac_same_word(const char *a, const char *b);

/* ---- 2bit index (kent/src/lib/twoBit.c:420-635) ---- */
typedef struct gac_twobit_seq {
    char *name;
    uint32_t size;
    uint32_t n_count;
    const uint8_t *n_starts_raw, *n_sizes_raw; /* file order, maybe byte-swapped */
    const uint8_t *packed;                     /* (size+3)/4 bytes */
} gac_twobit_seq;

typedef struct gac_twobit {
    gac_map map;
    int swapped;
    uint32_t version;
    uint32_t seq_count;
    gac_twobit_seq *seqs;
} gac_twobit;

int gac_twobit_open(const char *path, gac_twobit *tb);
/* the same; populate != 0 maps the file with MAP_POPULATE (page tables
 * filled up front: the tools open the .2bit files this way on a helper
 * thread while the HIP runtime starts) */
int gac_twobit_open_ex(const char *path, gac_twobit *tb, int populate);
/* gac_genome_load_2bit of an already opened file; the genome side takes
 * over tb (closed on error as well) */
int gac_genome_load_twobit(gac_ctx *c, int side, gac_twobit *tb);
/* the same with only the sequences i of the file where keep[i] != 0 (keep
 * may be NULL: all) */
int gac_genome_load_twobit_keep(gac_ctx *c, int side, gac_twobit *tb, const uint8_t *keep);
/* the same uploading only word runs (32-base words) of each sequence i of
 * the file: [run_lo[r], run_hi[r]) for r in [run_off[i], run_off[i+1]);
 * bases outside them are undefined on the device -- the caller scores no
 * range that reaches outside them (chainNet: the words under its chains'
 * blocks, plus one).  run_off NULL: every base. */
int gac_genome_load_twobit_runs(gac_ctx *c, int side, gac_twobit *tb, const uint8_t *keep,
                                const int64_t *run_off, const int32_t *run_lo,
                                const int32_t *run_hi);
void gac_twobit_close(gac_twobit *tb);
uint32_t gac_twobit_u32(const gac_twobit *tb, const uint8_t *p);
int gac_is_twobit_file(const char *path);

/* ---- host threads: GAC_THREADS, else OMP_NUM_THREADS, else gac_host_cpus() (<= 64) */
/* gac_chain_dp (include/gachain.h) with the exact fast DP when ov_off is
 * given: lin_k / 1024 = the linear minorant of the gap cost (0 <= s), the
 * smallest matrix entry, and per leaf (global index) the leaf nodes of its
 * overlapping candidates ov[ov_off[i] .. ov_off[i+1]) (-1: too many, the
 * reference search).  Internal to libgachain (gac_axt_chain). */
int gac_chain_dp_ex(gac_ctx *c, int64_t n_pairs, const int32_t *t_seq, const int32_t *q_seq,
                    const uint8_t *q_strand, const int64_t *node_off, const int32_t *node_a,
                    const int32_t *node_b, const int64_t *leaf_off, const int32_t *leaf,
                    const int32_t *leaf_score, const int32_t *leaf_node, const int64_t *path_off,
                    const int32_t *path, const int64_t *ov_off, const int32_t *ov, int64_t lin_k,
                    int32_t min_entry, int64_t *total, int32_t *pred);
/* CPUs usable by this process: online CPUs narrowed by the affinity mask and
 * the cgroup CPU quota (cpu.max) */
int gac_host_cpus(void);
int gac_host_threads(void);
/* GAC_TIMING: "[mark] <seconds since the first mark> <thread> <what>" on
 * stderr (timelines of overlapped phases; no-op otherwise) */
void gac_mark(const char *what);
/* gap tables with the same content (as gapCalcCost sees them) */
int gac_gapcalc_same(const gac_gapcalc *a, const gac_gapcalc *b);
/* deep copy, freed with gac_gapcalc_free */
gac_gapcalc *gac_gapcalc_clone(const gac_gapcalc *g);
/* fn(arg) on n threads (one of them the caller); fn pulls work itself */
void gac_run_threads(int n, void *(*fn)(void *), void *arg);
/* Ordered parallel output with formatting and writing overlapped: fn(f, r,
 * arg) prints run r into a memory stream on worker threads (runs taken in
 * increasing order), while the calling thread writes the finished runs to
 * out in order.  0 on success. */
int gac_par_output(FILE *out, int64_t nr, void (*fn)(FILE *f, int64_t r, void *arg), void *arg);
/* An output file opened for writing from offset 0 WITHOUT O_TRUNC, and
 * closed after cutting it to the bytes written: the same contents as
 * fopen(path, "w"), but truncating a file to zero at open makes ext4 flush
 * its whole delayed allocation on close (auto_da_alloc: 0.25 s for a 770 MB
 * net). */
FILE *gac_open_output(const char *path);
int gac_close_output(FILE *f); /* 0 or EOF, as fclose */
/* Abort path: cut every output still open (gac_open_output) to the bytes
 * written so far (the tools' gt_abort calls it before exiting). */
void gac_outputs_cut(void);
/* A growable text buffer (formatting without stdio): the *_buf variants hand
 * each run an empty one and take its bytes as the run's text (no copy). */
typedef struct gac_obuf {
    char *p;
    size_t n, cap;
} gac_obuf;
/* room for k more bytes at o->p + o->n (the caller advances o->n) */
char *gac_obuf_reserve(gac_obuf *o, size_t k);
void gac_obuf_printf(gac_obuf *o, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int gac_par_output_buf(FILE *out, int64_t nr, void (*fn)(gac_obuf *o, int64_t r, void *arg),
                       void *arg);
int gac_par_format_buf(int64_t nr, void (*fn)(gac_obuf *o, int64_t r, void *arg), void *arg,
                       char ***bufs, size_t **lens);
/* the same runs formatted on worker threads and returned, not written */
int gac_par_format(int64_t nr, void (*fn)(FILE *f, int64_t r, void *arg), void *arg, char ***bufs,
                   size_t **lens);

/* ---- host view of a resident sequence (kept after gac_genome_finalize) ----
 * packed: 2 bits/base MSB-first (T=0 C=1 A=2 G=3); N runs merged and sorted. */
typedef struct gac_seq_view {
    const uint8_t *packed;
    int32_t size;
    const int32_t *n_start, *n_size;
    int32_t n_count;
} gac_seq_view;
int gac_genome_view(gac_ctx *ctx, int side, int32_t index, gac_seq_view *v);

#ifdef __cplusplus
}
#endif
#endif
