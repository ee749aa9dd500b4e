/* Probe (measurement only): what process exit costs after libgachain work.
 *   exit_probe open            gac_open, gac_close, _exit
 *   exit_probe alloc GB        ... plus GB of device memory allocated and freed
 *   exit_probe keep GB         ... allocated and left for the exit
 *   exit_probe host GB         GB of host memory touched, then _exit (no device)
 * Prints "[stage-clock] exit <realtime>" just before _exit; the caller
 * measures when its wait returns. */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "gachain.h"

static double rt(void) {
    struct timespec t;
    clock_gettime(CLOCK_REALTIME, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "open";
    const double gb = argc > 2 ? atof(argv[2]) : 0;
    if (!strcmp(mode, "host")) {
        size_t n = (size_t)(gb * (1 << 30));
        char *p = malloc(n);
        memset(p, 1, n);
        fprintf(stderr, "[stage-clock] exit %.6f\n", rt());
        _exit(p[n / 2] == 7);
    }
    gac_ctx *c;
    if (gac_open(0, &c) != GAC_OK) {
        fprintf(stderr, "%s\n", gac_last_error());
        return 1;
    }
    void *d = NULL;
    if (gb > 0 && gac_dev_alloc(c, (size_t)(gb * (1 << 30)), &d) != GAC_OK) return 1;
    if (d && !strcmp(mode, "alloc")) gac_dev_free(c, d);
    if (strcmp(mode, "keep")) gac_close(c);
    fprintf(stderr, "[stage-clock] exit %.6f\n", rt());
    _exit(0);
}
