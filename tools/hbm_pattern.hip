// hbm_pattern.hip — does the order in which waves walk HBM matter?
// Each wave owns consecutive regions of R bytes (region r -> wave r % W) and
// streams each region front to back in 1 KiB wave-loads, 4 in flight.
// R = 1 KiB reproduces a plain grid-stride stream; R = 96 KiB is the rx
// kernel's "64 frames of 1536 B per wave" order.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void walk(const uint4 *__restrict__ p, uint64_t nbytes,
                                            uint32_t region, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint64_t nw = (uint64_t)gridDim.x * 4;
    const uint64_t nreg = nbytes / region;
    uint32_t acc = 0;
    for (uint64_t r = wave; r < nreg; r += nw) {
        const uint4 *base = p + r * (region / 16);
        const uint32_t nwin = region / 1024;
        for (uint32_t w = 0; w < nwin; w += 4) {
            uint4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u)
                v[u] = (w + u < nwin) ? base[(w + u) * 64 + lane] : make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                acc = __builtin_amdgcn_sad_u16(v[u].x, 0u, acc);
                acc = __builtin_amdgcn_sad_u16(v[u].y, 0u, acc);
                acc = __builtin_amdgcn_sad_u16(v[u].z, 0u, acc);
                acc = __builtin_amdgcn_sad_u16(v[u].w, 0u, acc);
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const uint64_t bytes = 1610612736ull;   // 1 M x 1536 B
    uint4 *p;
    uint32_t *out;
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(p, 0x5a, bytes);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    const uint32_t regions[] = {1024, 4096, 6144, 24576, 98304, 99328, 393216};
    for (int blocks : {512, 1024, 2048}) {
        for (uint32_t R : regions) {
            for (int i = 0; i < 2; ++i) walk<<<blocks, 256>>>(p, bytes, R, out);
            (void)hipEventRecord(a);
            for (int i = 0; i < 10; ++i) walk<<<blocks, 256>>>(p, bytes, R, out);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            const uint64_t used = bytes / R * R;
            printf("{\"blocks\": %d, \"region\": %u, \"GBs\": %.1f}\n", blocks, R, used / (ms / 10) / 1e6);
        }
    }
    return 0;
}
