// occ_probe.hip — rx_kernel occupancy probe (profiling tool, not product
// code): the compact-record (CMP) instantiations need fewer registers (C3's
// sorted RSS schedule 195 VGPRs instead of 252), so a third 256-thread
// workgroup per CU fits if the kernel is allocated for three waves per SIMD
// (WPE 3: <= 168 VGPRs).  Same frames, same process, HIP events over
// back-to-back launches, median of rounds; the records of every variant are
// compared byte for byte with the dispatched one's.
// usage: tools/occ_probe CONFIG [rounds]     CONFIG: c2 | c3 | c5
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../include/mtcp_gpu.h"
#include "../include/mtcp_gpu_pktgen.h"
#include "../mtcp_amd/csrc/rx_kernels.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef void (*kfn)(mg::KParams);

// util/rss.c:13-105 key cache -> the kernel's 24 nibble tables (as mtcp_gpu.hip does)
static void rss_tables(uint32_t *tables) {
    uint8_t key[40];
    memset(key, 5, sizeof(key));
    uint32_t cache[96];
    uint32_t result = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) | ((uint32_t)key[2] << 8) | key[3];
    uint32_t idx = 32;
    for (int i = 0; i < 96; i++, idx++) {
        cache[i] = result;
        const uint32_t bit = ((key[idx / 8] << (idx % 8)) & 0x80) ? 1u : 0u;
        result = (result << 1) | bit;
    }
    for (int t = 0; t < 24; ++t)
        for (int v = 0; v < 16; ++v) {
            uint32_t h = 0;
            for (int m = 0; m < 4; ++m)
                if (v & (0x8 >> m)) h ^= cache[4 * t + m];
            tables[t * 16 + v] = h;
        }
}

static uint32_t bimodal_len(uint64_t i, uint64_t seed) {   // mtcp_amd/pktgen.py lengths
    uint64_t z = i * 0x9E3779B97F4A7C15ull + seed * 0xD6E8FEB86659FD93ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (z & 1) ? 1500 : 64;
}

int main(int argc, char **argv) {
    const char *cfg = argc > 1 ? argv[1] : "c3";
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const bool c3 = !strcmp(cfg, "c3"), c5 = !strcmp(cfg, "c5");
    const uint32_t n = c5 ? (1u << 19) : (1u << 20);
    const uint64_t seed = c3 ? 3 : c5 ? 5 : 2;
    std::vector<mtcp_gpu_desc> desc(n);
    uint64_t off = 0, sum_l = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t L = c3 ? bimodal_len(i, seed) : c5 ? 9000 : 1500;
        desc[i].offset = (uint32_t)(off >> 6);
        desc[i].len = (uint16_t)L;
        desc[i].flags = desc[i].rsvd = 0;
        off += (L + 63) & ~63u;
        sum_l += L;
    }
    uint8_t *d_buf;
    mtcp_gpu_desc *d_desc;
    uint8_t *d_out;
    uint32_t *d_tab;
    uint32_t tab[mg::kRssTableWords];
    rss_tables(tab);
    CK(hipMalloc(&d_buf, off));
    CK(hipMalloc(&d_desc, n * sizeof(mtcp_gpu_desc)));
    CK(hipMalloc(&d_out, (size_t)n * 40));
    CK(hipMalloc(&d_tab, sizeof(tab)));
    CK(hipMemcpy(d_tab, tab, sizeof(tab), hipMemcpyHostToDevice));
    CK(hipMemcpy(d_desc, desc.data(), n * sizeof(mtcp_gpu_desc), hipMemcpyHostToDevice));
    if (mtcp_gpu_pktgen_dev(d_buf, off, d_desc, n, 6, seed, 0, nullptr) != 0) return 1;
    CK(hipDeviceSynchronize());
    int ncu = 256;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    ncu = prop.multiProcessorCount;
    mg::KParams kp{};
    kp.buf = d_buf;
    kp.buf_len = off;
    kp.desc = d_desc;
    kp.n = n;
    kp.off_shift = 6;
    kp.out = reinterpret_cast<mtcp_gpu_result *>(d_out);
    kp.rss_tables = d_tab;
    kp.rss_nq = 8;
    kp.rss_endian = 1;
    kp.compact = 1;
    struct V { const char *name; kfn fn; uint32_t per_cu; };
    // the dispatched schedule for the config (mtcp_gpu.hip launch_sched), WPE 2 and 3
    std::vector<V> vs;
    if (c3) {
        vs = {{"cmp_wpe2_2wg", mg::rx_kernel<0, true, mg::kSchedSorted, false, 0, 8, 8, true, 6, false, false, 0, 4, 0, true, 2>, 2},
              {"cmp_wpe3_2wg", mg::rx_kernel<0, true, mg::kSchedSorted, false, 0, 8, 8, true, 6, false, false, 0, 4, 0, true, 3>, 2},
              {"cmp_wpe3_3wg", mg::rx_kernel<0, true, mg::kSchedSorted, false, 0, 8, 8, true, 6, false, false, 0, 4, 0, true, 3>, 3}};
    } else if (c5) {
        vs = {{"cmp_wpe2_2wg", mg::rx_kernel<0, false, mg::kSchedUnrolled, true, 0, 8, 8, true, 6, true, false, 0, 4, 0, true, 2>, 2},
              {"cmp_wpe3_2wg", mg::rx_kernel<0, false, mg::kSchedUnrolled, true, 0, 8, 8, true, 6, true, false, 0, 4, 0, true, 3>, 2},
              {"cmp_wpe3_3wg", mg::rx_kernel<0, false, mg::kSchedUnrolled, true, 0, 8, 8, true, 6, true, false, 0, 4, 0, true, 3>, 3}};
    } else {
        vs = {{"cmp_wpe2_2wg", mg::rx_kernel<0, false, mg::kSchedUnrolled, false, 0, 8, 8, true, 6, false, false, 5, 4, 0, true, 2>, 2},
              {"cmp_wpe3_2wg", mg::rx_kernel<0, false, mg::kSchedUnrolled, false, 0, 8, 8, true, 6, false, false, 5, 4, 0, true, 3>, 2},
              {"cmp_wpe3_3wg", mg::rx_kernel<0, false, mg::kSchedUnrolled, false, 0, 8, 8, true, 6, false, false, 5, 4, 0, true, 3>, 3}};
    }
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<uint8_t> ref((size_t)n * 16), got((size_t)n * 16);
    printf("{\"config\": \"%s\", \"n\": %u, \"frame_bytes\": %llu", cfg, n, (unsigned long long)sum_l);
    for (size_t vi = 0; vi < vs.size(); ++vi) {
        const V &v = vs[vi];
        // one launch holds 8 passes per wave: grid = per_cu x CUs, and the
        // batch splits into launches of grid x 4 x 64 x 8 packets, as mtcp_gpu.hip launch()
        const uint32_t grid = std::min<uint32_t>((n + 255) / 256, ncu * v.per_cu);
        const uint32_t cap = grid * 4 * 64 * 8;
        std::vector<float> t;
        for (int r = 0; r < rounds; ++r) {
            auto run = [&]() {
                for (uint32_t first = 0; first < n; first += cap) {
                    mg::KParams sub = kp;
                    sub.n = std::min(n - first, cap);
                    sub.desc = kp.desc + first;
                    sub.out = reinterpret_cast<mtcp_gpu_result *>(d_out + (size_t)first * 16);
                    hipLaunchKernelGGL(v.fn, dim3(grid), dim3(256), 0, st, sub);
                }
            };
            for (int i = 0; i < 3; ++i) run();
            CK(hipEventRecord(a, st));
            const int reps = 50;
            for (int i = 0; i < reps; ++i) run();
            CK(hipEventRecord(b, st));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            t.push_back(ms * 1e3f / reps);
        }
        std::sort(t.begin(), t.end());
        printf(", \"%s_us\": %.2f, \"%s_min_us\": %.2f", v.name, t[t.size() / 2], v.name, t[0]);
        CK(hipMemcpy(got.data(), d_out, got.size(), hipMemcpyDeviceToHost));
        if (vi == 0) ref = got;
        else if (memcmp(ref.data(), got.data(), ref.size()) != 0) {
            fprintf(stderr, "%s records differ\n", v.name);
            return 2;
        }
    }
    printf("}\n");
    return 0;
}
