// hbm_ceiling.hip — measured read-only streaming ceiling of the box's HBM
// ("also report against a measured read-only streaming ceiling").
// A grid-stride dwordx4 read + v_sad_u16 sum over a buffer far larger than
// the 256 MiB Infinity Cache; one u32 per workgroup written.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

template <int UNROLL>
__global__ __launch_bounds__(256) void stream_read(const uint4 *__restrict__ p, uint64_t n16,
                                                   uint32_t *out) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * UNROLL;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * UNROLL + threadIdx.x; i < n16; i += stride) {
        uint4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u)
            v[u] = (i + u * 256 < n16) ? p[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            acc = __builtin_amdgcn_sad_u16(v[u].x, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].y, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].z, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].w, 0u, acc);
        }
    }
    if (acc == 0x12345678u) out[blockIdx.x] = acc;   // keep the loads live
}

template <int UNROLL>
float run(const uint4 *p, uint64_t n16, uint32_t *out, int blocks, int reps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    for (int i = 0; i < 3; ++i) stream_read<UNROLL><<<blocks, 256>>>(p, n16, out);
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) stream_read<UNROLL><<<blocks, 256>>>(p, n16, out);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main(int argc, char **argv) {
    const uint64_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : (1572864000ull);
    uint4 *p;
    uint32_t *out;
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
    hipMemset(p, 0x5a, bytes);
    const uint64_t n16 = bytes / 16;
    for (int blocks : {1024, 2048, 4096, 8192}) {
        float m1 = run<1>(p, n16, out, blocks, 20);
        float m4 = run<4>(p, n16, out, blocks, 20);
        float m8 = run<8>(p, n16, out, blocks, 20);
        printf("{\"blocks\": %d, \"bytes\": %llu, \"unroll1_GBs\": %.1f, \"unroll4_GBs\": %.1f, \"unroll8_GBs\": %.1f}\n",
               blocks, (unsigned long long)bytes, bytes / m1 / 1e6, bytes / m4 / 1e6, bytes / m8 / 1e6);
    }
    return 0;
}
