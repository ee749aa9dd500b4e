// Probe (measurement only): throughput of the vector memory pipeline
// (TA -> TCP -> TD) for k_tile-shaped loads on gfx950.  k_tile's counters
// (r03s) show TD busy 96-99 % of the time at ~62 TD cycles per vector load
// instruction, i.e. about one lane per cycle; this probe asks what a wave
// load instruction costs as a function of
//   BYTES  bytes per lane (4, 8, 16),
//   ACT    active lanes (64, 32, 16: the rest masked off by EXEC),
//   GRP    lanes reading one 128-B line together (1 = every lane its own
//          random line, 8 = groups of 8 lanes sweep one line),
// with 4 independent loads in flight per wave per round (k_tile's plane
// loads), over a 2 GiB buffer (beyond the Infinity Cache).
// Prints, per variant: ms, wave-instructions/s, active lane-loads/s, lines/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(16)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2), aligned(8)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

template <int BYTES>
__device__ __forceinline__ uint32_t ld(const uint8_t *p) {
    if (BYTES == 16) {
        const u32x4 v = *reinterpret_cast<const u32x4 *>(p);
        return v.x ^ v.y ^ v.z ^ v.w;
    } else if (BYTES == 8) {
        const u32x2 v = *reinterpret_cast<const u32x2 *>(p);
        return v.x ^ v.y;
    }
    return *reinterpret_cast<const uint32_t *>(p);
}

template <int BYTES, int ACT, int GRP>
__global__ void __launch_bounds__(256) k_rate(const uint8_t *buf, uint64_t lines, int rounds,
                                              uint32_t *out) {
    const int lane = threadIdx.x & 63;
    const uint64_t wid = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    uint32_t acc = 0;
    if (lane < ACT) {
        const int g = lane / GRP, sub = lane % GRP;  // lanes of a group share a line
        for (int r = 0; r < rounds; ++r) {
            const uint64_t b = (wid * 1315423911ull + (uint64_t)r * 4) * 64 + g;
            const uint64_t l0 = mix(b) % lines, l1 = mix(b + 64) % lines;
            const uint64_t l2 = mix(b + 128) % lines, l3 = mix(b + 192) % lines;
            const int off = (sub * BYTES) & 127;
            const uint32_t v0 = ld<BYTES>(buf + l0 * 128 + off);
            const uint32_t v1 = ld<BYTES>(buf + l1 * 128 + off);
            const uint32_t v2 = ld<BYTES>(buf + l2 * 128 + off);
            const uint32_t v3 = ld<BYTES>(buf + l3 * 128 + off);
            acc += v0 ^ v1 ^ v2 ^ v3;
        }
    }
    if (acc == 0x12345678u) out[wid] = acc;  // (keeps the loads)
}

template <int BYTES, int ACT, int GRP>
static void run(const uint8_t *buf, uint64_t lines, uint32_t *out, int grid, int rounds) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    k_rate<BYTES, ACT, GRP><<<grid, 256>>>(buf, lines, rounds, out);  // warm-up
    hipEventRecord(a);
    const int reps = 3;
    for (int i = 0; i < reps; ++i) k_rate<BYTES, ACT, GRP><<<grid, 256>>>(buf, lines, rounds, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    const double waves = grid * 4.0, instr = waves * rounds * 4;
    const double lane_loads = instr * ACT, line_reqs = instr * ((ACT + GRP - 1) / GRP);
    printf("{\"bytes\": %d, \"active\": %d, \"group\": %d, \"ms\": %.4f, \"winstr_per_s\": %.4g, "
           "\"lane_loads_per_s\": %.4g, \"lines_per_s\": %.4g, \"line_GBps\": %.1f}\n",
           BYTES, ACT, GRP, ms, instr / ms * 1e3, lane_loads / ms * 1e3, line_reqs / ms * 1e3,
           line_reqs * 128 / ms * 1e-6);
    hipEventDestroy(a);
    hipEventDestroy(b);
}

int main(int argc, char **argv) {
    const uint64_t bytes = 2ull << 30, lines = bytes / 128;
    uint8_t *buf;
    uint32_t *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 1 << 24) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    const int grid = 256 * 6;  // 24 waves per CU, as k_tile
    const int rounds = argc > 1 ? atoi(argv[1]) : 64;
    run<16, 64, 1>(buf, lines, out, grid, rounds);
    run<8, 64, 1>(buf, lines, out, grid, rounds);
    run<4, 64, 1>(buf, lines, out, grid, rounds);
    run<16, 32, 1>(buf, lines, out, grid, rounds);
    run<16, 16, 1>(buf, lines, out, grid, rounds);
    run<16, 64, 2>(buf, lines, out, grid, rounds);
    run<16, 64, 4>(buf, lines, out, grid, rounds);
    run<16, 64, 8>(buf, lines, out, grid, rounds);
    run<4, 64, 8>(buf, lines, out, grid, rounds);
    run<4, 64, 32>(buf, lines, out, grid, rounds);
    hipDeviceSynchronize();
    hipFree(buf);
    hipFree(out);
    return 0;
}
