// gather_ceiling.hip -- measurement infrastructure (bench.py runs the built
// binary, genomealignmenttools_amd/libexec/gac_gather_ceiling): the rate at
// which an MI355X serves RANDOM 128-B LINES out of HBM, the access pattern
// of k_tile (a chain's blocks sit at random genome positions, and every
// random 8- or 16-B load fetches a whole 128-B line on gfx950,
// scripts/probes/ld_granularity.hip).  The ceiling bench.py reports
// k_tile's measured HBM traffic against (frac_of_gather_ceiling).
//
// Buffer of F bytes (default 2 GiB: about the resident hg38 + mm10 planes
// and N masks), never cached between passes at this size.  Shapes:
//   isolated   -- each lane loads 16 B of its own random line (k_tile's
//                 plane and record loads);
//   line       -- 8 lanes load the 8 x 16 B of one random line (a whole
//                 line per 8 lanes: the best case for a line fetch);
// each with K independent loads in flight per lane (K = 1, 2, 4, 8) and
// 8 or 16 waves per CU.  Output: one JSON line, bytes = lines x 128.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

template <int K, bool LINE>
__global__ void __launch_bounds__(256) k_gather(const uint8_t *__restrict__ buf, uint64_t nlines,
                                                int iters, uint32_t *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint64_t who = LINE ? tid >> 3 : tid;
    const uint32_t piece = LINE ? (threadIdx.x & 7) : 0;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint64_t h = mix(who * 0x9e3779b97f4a7c15ull + (uint64_t)(it * K + k));
            const uint64_t line = h % nlines;
            const uint32_t pc = LINE ? piece : (uint32_t)(h >> 60) & 7;
            v[k] = *reinterpret_cast<const u32x4 *>(buf + line * 128 + pc * 16);
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            acc += v[k].x ^ v[k].y ^ v[k].z ^ v[k].w;
    }
    if (acc == 0x9e3779b9u) out[0] = acc;  // (keeps the loads; never true in practice)
}

template <int K, bool LINE>
static double run(const uint8_t *buf, uint64_t nlines, int blocks, int iters, uint32_t *out) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    double best = 1e30;
    for (int rep = 0; rep < 4; ++rep) {
        hipEventRecord(a, 0);
        hipLaunchKernelGGL((k_gather<K, LINE>), dim3(blocks), dim3(256), 0, 0, buf, nlines, iters, out);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (rep && ms < best) best = ms;  // (rep 0 warms up)
    }
    hipEventDestroy(a);
    hipEventDestroy(b);
    const double lines = (double)blocks * 256 * iters * K / (LINE ? 8 : 1);
    return lines * 128 / (best * 1e-3) / 1e9;  // GB/s of 128-B lines
}

int main(int argc, char **argv) {
    const size_t bytes = (argc > 1 ? strtoull(argv[1], NULL, 10) : 2048ull) << 20;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    uint8_t *buf;
    uint32_t *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    hipDeviceSynchronize();
    const uint64_t nlines = bytes / 128;
    const int cus = prop.multiProcessorCount;
    printf("{\"probe\": \"random 128-B line gathers\", \"footprint_bytes\": %zu, \"cus\": %d, "
           "\"arch\": \"%s\", \"configs\": [", bytes, cus, prop.gcnArchName);
    double best = 0;
    const char *bname = "";
    int first = 1;
    for (int wpc = 8; wpc <= 16; wpc *= 2) {
        const int blocks = cus * wpc / 4;  // 256 threads = 4 waves
        struct {
            const char *name;
            double gbs;
        } r[8] = {
            {"isolated K=1", run<1, false>(buf, nlines, blocks, 64, out)},
            {"isolated K=2", run<2, false>(buf, nlines, blocks, 32, out)},
            {"isolated K=4", run<4, false>(buf, nlines, blocks, 16, out)},
            {"isolated K=8", run<8, false>(buf, nlines, blocks, 8, out)},
            {"line K=1", run<1, true>(buf, nlines, blocks, 512, out)},
            {"line K=2", run<2, true>(buf, nlines, blocks, 256, out)},
            {"line K=4", run<4, true>(buf, nlines, blocks, 128, out)},
            {"line K=8", run<8, true>(buf, nlines, blocks, 64, out)},
        };
        for (int i = 0; i < 8; ++i) {
            printf("%s{\"shape\": \"%s\", \"waves_per_cu\": %d, \"GBps\": %.1f}", first ? "" : ", ",
                   r[i].name, wpc, r[i].gbs);
            first = 0;
            if (i < 4 && r[i].gbs > best) {  // the isolated shape is k_tile's
                best = r[i].gbs;
                bname = r[i].name;
            }
        }
    }
    printf("], \"ceiling_isolated_GBps\": %.1f, \"ceiling_shape\": \"%s\"}\n", best, bname);
    hipFree(buf);
    hipFree(out);
    return 0;
}
