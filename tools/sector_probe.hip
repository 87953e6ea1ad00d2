// sector_probe.hip — HBM fetch granularity (profiling tool, not product
// code).  A 1500 B frame in a 1536 B PSIO slot leaves the slot's last 32 B
// unread, inside the frame's last 64 B line; the rx kernel's PMC traffic is
// the whole slot.  Does any read shape fetch 32 B sectors instead?
//   blocks: every 64 B block read whole (4 lanes x 16 B), or only its first
//           32 B (2 lanes x 16 B), plain and non-temporal loads;
//   slots:  1 M x 1536 B slots, 16 lanes per slot, chunks 0..93 (the 1504 B a
//           1500 B frame covers) or 0..95 (the whole slot).
// HIP events over back-to-back launches, median of rounds.
// usage: tools/sector_probe [rounds]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdint.h>

#include <algorithm>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ v4u ld(const v4u *p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}

// LPB lanes per 64 B block (4: whole, 2: first 32 B); 4 loads in flight
template <int LPB, bool NT>
__global__ __launch_bounds__(256) void blocks(const v4u *__restrict__ p, uint64_t nblk, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 4;
    constexpr uint32_t BPW = 64 / LPB;               // blocks per wave-load
    uint32_t acc = 0;
    for (uint64_t b0 = wave * BPW * 4; b0 < nblk; b0 += nw * BPW * 4) {
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            uint64_t b = b0 + u * BPW + lane / LPB;
            b = b < nblk ? b : nblk - 1;
            v[u] = ld<NT>(p + b * 4 + (lane % LPB));
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_sad_u16(v[u].x ^ v[u].y ^ v[u].z ^ v[u].w, 0u, acc);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// a 16-lane row per slot, 6 loads per lane in flight (the rx kernel's trip shape)
template <int NCH, bool NT>
__global__ __launch_bounds__(256) void slots(const v4u *__restrict__ p, uint32_t nslot, uint32_t *out) {
    const uint32_t lane = threadIdx.x & 63, row = lane >> 4, rl = lane & 15;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    uint32_t acc = 0;
    for (uint32_t s0 = wave * 4; s0 < nslot; s0 += nw * 4) {
        const uint32_t s = s0 + row < nslot ? s0 + row : nslot - 1;
        const v4u *f = p + (uint64_t)s * 96;
        v4u v[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) {
            uint32_t c = u * 16 + rl;
            c = c < NCH ? c : NCH - 1;
            v[u] = ld<NT>(f + c);
        }
#pragma unroll
        for (int u = 0; u < 6; ++u) acc = __builtin_amdgcn_sad_u16(v[u].x ^ v[u].y ^ v[u].z ^ v[u].w, 0u, acc);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main(int argc, char **argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 5;
    const uint32_t nslot = 1u << 20;
    const uint64_t bytes = (uint64_t)nslot * 1536;
    v4u *p;
    uint32_t *out;
    if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(p, 0x5a, bytes);
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int grid = prop.multiProcessorCount * 8;
    const uint64_t nblk = bytes / 64;
    struct V { const char *name; void (*launch)(); };
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    auto timeit = [&](auto fn) {
        std::vector<float> t;
        for (int r = 0; r < rounds; ++r) {
            fn();
            (void)hipEventRecord(a);
            for (int i = 0; i < 20; ++i) fn();
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            t.push_back(ms * 1e3f / 20);
        }
        std::sort(t.begin(), t.end());
        return t[t.size() / 2];
    };
    const float b4 = timeit([&] { hipLaunchKernelGGL((blocks<4, false>), dim3(grid), dim3(256), 0, 0, p, nblk, out); });
    const float b2 = timeit([&] { hipLaunchKernelGGL((blocks<2, false>), dim3(grid), dim3(256), 0, 0, p, nblk, out); });
    const float b4n = timeit([&] { hipLaunchKernelGGL((blocks<4, true>), dim3(grid), dim3(256), 0, 0, p, nblk, out); });
    const float b2n = timeit([&] { hipLaunchKernelGGL((blocks<2, true>), dim3(grid), dim3(256), 0, 0, p, nblk, out); });
    const float s96 = timeit([&] { hipLaunchKernelGGL((slots<96, true>), dim3(grid), dim3(256), 0, 0, p, nslot, out); });
    const float s94 = timeit([&] { hipLaunchKernelGGL((slots<94, true>), dim3(grid), dim3(256), 0, 0, p, nslot, out); });
    const float s92 = timeit([&] { hipLaunchKernelGGL((slots<92, true>), dim3(grid), dim3(256), 0, 0, p, nslot, out); });
    printf("{\"probe\": \"sector\", \"bytes\": %llu, \"blocks64_us\": %.2f, \"blocks32_us\": %.2f, "
           "\"blocks64_nt_us\": %.2f, \"blocks32_nt_us\": %.2f, \"slots96_nt_us\": %.2f, "
           "\"slots94_nt_us\": %.2f, \"slots92_nt_us\": %.2f}\n",
           (unsigned long long)bytes, b4, b2, b4n, b2n, s96, s94, s92);
    return 0;
}
