/* Buffered write throughput of one output file on this host's TMPDIR: one
 * writer (writev of 8 MB batches) vs k threads each pwrite()-ing its own
 * contiguous part, and a shared-mapping copy -- what chainNet's net writer
 * could gain from splitting a file.  usage: write_probe DIR MB */
#define _GNU_SOURCE
#include <fcntl.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/vfs.h>
#include <time.h>
#include <unistd.h>

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef struct job {
    int fd;
    char *src, *map;
    size_t off, len;
} job;

static void *pw(void *a) {
    job *j = a;
    for (size_t d = 0; d < j->len;) {
        size_t n = j->len - d < (8u << 20) ? j->len - d : (8u << 20);
        ssize_t k = pwrite(j->fd, j->src + j->off + d, n, (off_t)(j->off + d));
        if (k <= 0) { perror("pwrite"); exit(1); }
        d += (size_t)k;
    }
    return NULL;
}

static void *mc(void *a) {
    job *j = a;
    memcpy(j->map + j->off, j->src + j->off, j->len);
    return NULL;
}

int main(int argc, char **argv) {
    const char *dir = argc > 1 ? argv[1] : "/tmp";
    const size_t size = (size_t)(argc > 2 ? atol(argv[2]) : 1300) << 20;
    char path[4096];
    snprintf(path, sizeof path, "%s/write_probe.out", dir);
    char *src = malloc(size);
    for (size_t i = 0; i < size; ++i) src[i] = (char)('0' + i % 10);
    struct statfs sf;
    if (statfs(dir, &sf) == 0) printf("fs magic 0x%lx\n", (long)sf.f_type);
    for (int rep = 0; rep < 2; ++rep) {
        for (int k = 1; k <= 8; k *= 2) {
            unlink(path);
            int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0644);
            double t0 = now();
            pthread_t th[8];
            job J[8];
            for (int i = 0; i < k; ++i) {
                J[i] = (job){fd, src, NULL, size / k * i, i == k - 1 ? size - size / k * i : size / k};
                pthread_create(&th[i], NULL, pw, &J[i]);
            }
            for (int i = 0; i < k; ++i) pthread_join(th[i], NULL);
            close(fd);
            double t1 = now();
            printf("pwrite %d threads: %.3f s (%.2f GB/s)\n", k, t1 - t0, size / (t1 - t0) / 1e9);
        }
        for (int k = 1; k <= 8; k *= 4) {
            unlink(path);
            int fd = open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
            double t0 = now();
            if (ftruncate(fd, (off_t)size) != 0) { perror("ftruncate"); return 1; }
            char *m = mmap(NULL, size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            pthread_t th[8];
            job J[8];
            for (int i = 0; i < k; ++i) {
                J[i] = (job){fd, src, m, size / k * i, i == k - 1 ? size - size / k * i : size / k};
                pthread_create(&th[i], NULL, mc, &J[i]);
            }
            for (int i = 0; i < k; ++i) pthread_join(th[i], NULL);
            munmap(m, size);
            close(fd);
            double t1 = now();
            printf("mmap copy %d threads: %.3f s (%.2f GB/s)\n", k, t1 - t0, size / (t1 - t0) / 1e9);
        }
    }
    unlink(path);
    return 0;
}
