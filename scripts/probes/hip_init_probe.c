/* hip_init_probe.c -- times the HIP runtime bring-up steps a tool pays before
 * its first kernel (dlopen of libamdhip64, hipInit, device properties, stream
 * creation, a 1 GB hipMalloc, a 256 MB pinned host buffer + H2D copy).
 * Build: gcc -O2 hip_init_probe.c -o hip_init_probe -ldl */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

typedef int (*f_init)(unsigned);
typedef int (*f_count)(int *);
typedef int (*f_set)(int);
typedef int (*f_stream)(void **);
typedef int (*f_malloc)(void **, size_t);
typedef int (*f_hmalloc)(void **, size_t, unsigned);
typedef int (*f_memcpy)(void *, const void *, size_t, int);
typedef int (*f_sync)(void);

int main(void) {
    double t = now(), t0 = t;
    void *h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 1;
    }
    double t1 = now();
    f_init hipInit = (f_init)dlsym(h, "hipInit");
    f_count hipGetDeviceCount = (f_count)dlsym(h, "hipGetDeviceCount");
    f_set hipSetDevice = (f_set)dlsym(h, "hipSetDevice");
    f_stream hipStreamCreate = (f_stream)dlsym(h, "hipStreamCreate");
    f_malloc hipMalloc = (f_malloc)dlsym(h, "hipMalloc");
    f_hmalloc hipHostMalloc = (f_hmalloc)dlsym(h, "hipHostMalloc");
    f_memcpy hipMemcpy = (f_memcpy)dlsym(h, "hipMemcpy");
    f_sync hipDeviceSynchronize = (f_sync)dlsym(h, "hipDeviceSynchronize");
    int n = 0;
    hipInit(0);
    double t2 = now();
    hipGetDeviceCount(&n);
    hipSetDevice(0);
    double t3 = now();
    void *s = NULL;
    hipStreamCreate(&s);
    double t4 = now();
    void *d = NULL;
    hipMalloc(&d, 1ull << 30);
    double t5 = now();
    void *p = NULL;
    hipHostMalloc(&p, 256u << 20, 0);
    memset(p, 1, 256u << 20);
    double t6 = now();
    hipMemcpy(d, p, 256u << 20, 1);
    hipDeviceSynchronize();
    double t7 = now();
    printf("devices %d dlopen %.1f ms hipInit %.1f ms setDevice %.1f ms stream %.1f ms malloc1G %.1f ms "
           "hostMalloc256M+touch %.1f ms H2D256M %.1f ms (%.1f GB/s) total %.1f ms\n",
           n, 1e3 * (t1 - t0), 1e3 * (t2 - t1), 1e3 * (t3 - t2), 1e3 * (t4 - t3), 1e3 * (t5 - t4),
           1e3 * (t6 - t5), 1e3 * (t7 - t6), 0.256 / (t7 - t6) * 1.048576, 1e3 * (t7 - t0));
    fflush(stdout);
    _exit(0);
}
