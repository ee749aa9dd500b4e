// Probe (analysis only): per-XCD set-associative LRU model of the 4 MiB L2s
// for scripts/archive/traffic_sim/sim.py.  Input: uint64 pairs {xcd, line} in issue
// order; line >> 40 tags the region.  Prints the misses per region.
// per-XCD set-associative LRU L2 simulator: input = uint64 keys sorted by (xcd, time);
// each record: uint32 xcd, uint64 line. Reports misses per region (line>>40).
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
int main(int argc, char **argv) {
    FILE *f = fopen(argv[1], "rb");
    long ways = argc > 2 ? atol(argv[2]) : 16, mb = argc > 3 ? atol(argv[3]) : 4;
    long nsets = mb * 1024 * 1024 / 128 / ways;
    fseek(f, 0, SEEK_END); long n = ftell(f) / 16; fseek(f, 0, SEEK_SET);
    uint64_t *r = malloc(n * 16);
    if (fread(r, 16, n, f) != (size_t)n) return 1;
    fclose(f);
    uint64_t *tag = malloc(8 * nsets * ways * 8); uint32_t *age = calloc(8 * nsets * ways, 4);
    memset(tag, 0xff, 8 * nsets * ways * 8);
    long miss[8] = {0}, acc[8] = {0}; uint32_t clk = 0;
    for (long i = 0; i < n; ++i) {
        uint64_t x = r[2 * i], line = r[2 * i + 1];
        int reg = (int)(line >> 40) & 7;
        uint64_t h = line * 0x9E3779B97F4A7C15ull;
        long set = (long)((h >> 20) % nsets);
        uint64_t *t = tag + (x * nsets + set) * ways; uint32_t *a = age + (x * nsets + set) * ways;
        ++acc[reg]; ++clk; int hit = -1, lru = 0;
        for (int w = 0; w < ways; ++w) { if (t[w] == line) { hit = w; break; } if (a[w] < a[lru]) lru = w; }
        if (hit >= 0) a[hit] = clk; else { ++miss[reg]; t[lru] = line; a[lru] = clk; }
    }
    long tm = 0;
    for (int k = 0; k < 8; ++k) if (acc[k]) { printf("region %d: access %ld miss %ld (%.2f GB)\n", k, acc[k], miss[k], miss[k] * 128e-9); tm += miss[k]; }
    printf("total miss %.3f GB\n", tm * 128e-9);
}
