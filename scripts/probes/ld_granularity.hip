// Probe (measurement only): how many bytes leave L2 per random 16-B / 8-B
// load on gfx950, with the default cache policy vs non-temporal loads --
// k_tile's plane and block reads are random 8-16 B pieces of 128-B lines.
// Each lane reads `per` random 16-B (or 8-B) pieces of a 4 GiB buffer.
// Run under rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum
// TCC_EA0_RDREQ_128B_sum to see the request sizes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    return x ^ (x >> 33);
}

template <int MODE>  // 0: 16-B default, 1: 16-B nontemporal, 2: 8-B default, 3: 8-B nontemporal
__global__ void __launch_bounds__(256) k_probe(const uint8_t *buf, uint64_t words16, int per,
                                               uint32_t *out) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (int k = 0; k < per; ++k) {
        const uint64_t w = mix(tid * 1315423911ull + k) % words16;
        if (MODE == 0) {
            const u32x4 v = *reinterpret_cast<const u32x4 *>(buf + 16 * w);
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if (MODE == 1) {
            const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(buf + 16 * w));
            acc += v.x ^ v.y ^ v.z ^ v.w;
        } else if (MODE == 2) {
            const u32x2 v = *reinterpret_cast<const u32x2 *>(buf + 16 * w);
            acc += v.x ^ v.y;
        } else {
            const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2 *>(buf + 16 * w));
            acc += v.x ^ v.y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = 4ull << 30;
    uint8_t *buf;
    uint32_t *out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    const int per = 16, blocks = 256 * 64;
    const char *names[4] = {"16B default", "16B nontemporal", "8B default", "8B nontemporal"};
    for (int rep = 0; rep < 3; ++rep)
        for (int m = 0; m < 4; ++m) {
            hipEvent_t a, b;
            hipEventCreate(&a);
            hipEventCreate(&b);
            hipEventRecord(a, 0);
            if (m == 0) hipLaunchKernelGGL(k_probe<0>, dim3(blocks), dim3(256), 0, 0, buf, bytes / 16, per, out);
            if (m == 1) hipLaunchKernelGGL(k_probe<1>, dim3(blocks), dim3(256), 0, 0, buf, bytes / 16, per, out);
            if (m == 2) hipLaunchKernelGGL(k_probe<2>, dim3(blocks), dim3(256), 0, 0, buf, bytes / 16, per, out);
            if (m == 3) hipLaunchKernelGGL(k_probe<3>, dim3(blocks), dim3(256), 0, 0, buf, bytes / 16, per, out);
            hipEventRecord(b, 0);
            hipEventSynchronize(b);
            float ms = 0;
            hipEventElapsedTime(&ms, a, b);
            const double loads = (double)blocks * 256 * per;
            if (rep == 2)
                printf("%-16s %8.3f ms  %.2f G loads/s  %.1f GB/s of 128-B lines\n", names[m], ms,
                       loads / ms / 1e6, loads * 128 / ms / 1e6);
        }
    return 0;
}
