// wave_probe.hip — where the wave-per-packet kernel's time goes on small
// batches (profiling tool, not product code).  Same frames, same process,
// back-to-back launches timed with HIP events:
//   empty      a kernel of the same grid that only writes lane 0's index
//   desc       rx_wave_kernel ABL 2: descriptor load only
//   phase1     ABL 1: + the frame stream and the chunk sum
//   full       the dispatched kernel (phase 2 and the record)
//   rows       rx_kernel (the schedule mtcp_gpu.hip picks for big batches)
// usage: tools/wave_probe [size] [n...]      size: bytes (64 .. 9000) | imix | bimodal
//   imix: 64 / 576 / 1500 B frames in the ratio 7 : 4 : 1, in a hashed order
//   bimodal: 64 / 1500 B, p = 0.5 each (C3's mix, hashed order)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../include/mtcp_gpu.h"
#include "../include/mtcp_gpu_pktgen.h"
#include "../mtcp_amd/csrc/rx_span.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

template <int WPB>
__global__ __launch_bounds__(64 * WPB) void empty_kernel(mg::KParams kp) {
    const uint32_t k = blockIdx.x * WPB + (threadIdx.x >> 6);
    if (k < kp.n && (threadIdx.x & 63) == 0) kp.out[k].saddr = k;
}

typedef void (*kfn)(mg::KParams);

int main(int argc, char **argv) {
    const bool imix = argc > 1 && !strcmp(argv[1], "imix");
    const bool bimodal = argc > 1 && !strcmp(argv[1], "bimodal");
    const uint32_t L = imix || bimodal ? 0u : argc > 1 ? (uint32_t)atoi(argv[1]) : 1500;
    auto len_of = [&](uint32_t i) -> uint32_t {
        const uint32_t h = (i * 2654435761u) >> 16;
        if (bimodal) return (h ^ (h >> 7)) & 1 ? 1500u : 64u;
        if (!imix) return L;
        const uint32_t r = h % 12;
        return r < 7 ? 64u : r < 11 ? 576u : 1500u;
    };
    std::vector<uint32_t> ns;
    for (int i = 2; i < argc; ++i) ns.push_back((uint32_t)atoi(argv[i]));
    if (ns.empty()) ns = {64, 1024, 4096, 16384};
    hipStream_t st;
    CK(hipStreamCreate(&st));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    // threads per block and packets per block of each variant
    // ppb: packets per workgroup (0: a persistent grid, `persist` workgroups
    // per CU, at most one 64-frame tile per wave; rx_kernel's grid when 0)
    struct V { const char *name; kfn fn; uint32_t threads, ppb, persist = 0; };
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const V vs[] = {
        {"empty", empty_kernel<4>, 256, 4},
        {"empty16", empty_kernel<16>, 1024, 16},
        {"w8nl2", mg::rx_wave_kernel<mg::kRxChunk, false, 0, 1, 2, 8>, 512, 8},
        {"w16nl2", mg::rx_wave_kernel<mg::kRxChunk, false, 0, 1, 2, 16>, 1024, 16},
        {"desc", mg::rx_wave_kernel<mg::kRxChunk, false, 2>, 256, 4},
        {"phase1", mg::rx_wave_kernel<mg::kRxChunk, false, 1>, 256, 4},
        {"full", mg::rx_wave_kernel<mg::kRxChunk, false, 0>, 256, 4},
        {"seg0", mg::rx_wave_kernel<mg::kRxChunk, false, 0, 0>, 256, 4},
        {"nl2", mg::rx_wave_kernel<mg::kRxChunk, false, 0, 1, 2>, 256, 4},
        {"nl4", mg::rx_wave_kernel<mg::kRxChunk, false, 0, 1, 4>, 256, 4},
        {"head", mg::rx_wave_kernel<mg::kRxChunk, false, 3, 1, 2>, 256, 4},
        {"segsum", mg::rx_wave_kernel<mg::kRxChunk, false, 4, 1, 2>, 256, 4},
        {"p1nl2", mg::rx_wave_kernel<mg::kRxChunk, false, 1, 1, 2>, 256, 4},
        {"g64_p1", mg::rx_group_kernel<mg::kRxChunk, false, 64, 1>, 1024, 16},
        {"g64", mg::rx_group_kernel<mg::kRxChunk, false, 64>, 1024, 16},
        {"g16_p1", mg::rx_group_kernel<mg::kRxChunk, false, 16, 1>, 1024, 64},
        {"g16", mg::rx_group_kernel<mg::kRxChunk, false, 16>, 1024, 64},
        {"g4", mg::rx_group_kernel<mg::kRxChunk, false, 4>, 1024, 256},
        {"g4noal", mg::rx_group_kernel<mg::kRxChunk, false, 4, 0, 0>, 1024, 256},
        {"g16noal", mg::rx_group_kernel<mg::kRxChunk, false, 16, 0, 0>, 1024, 64},
        // workgroup size (P = 64 packets: one full phase-2 wave) and 8-lane groups
        {"g4b256", mg::rx_group_kernel<mg::kRxChunk, false, 4, 0, 1, 256>, 256, 64},
        {"g4b512", mg::rx_group_kernel<mg::kRxChunk, false, 4, 0, 1, 512>, 512, 128},
        {"g8b256", mg::rx_group_kernel<mg::kRxChunk, false, 8, 0, 1, 256>, 256, 32},
        {"g8b512", mg::rx_group_kernel<mg::kRxChunk, false, 8, 0, 1, 512>, 512, 64},
        {"g8", mg::rx_group_kernel<mg::kRxChunk, false, 8>, 1024, 128},
        {"g8u2b512", mg::rx_group_kernel<mg::kRxChunk, false, 8, 0, 1, 512, 2>, 512, 64},
        {"g16b256", mg::rx_group_kernel<mg::kRxChunk, false, 16, 0, 1, 256>, 256, 16},
        {"g16b512", mg::rx_group_kernel<mg::kRxChunk, false, 16, 0, 1, 512>, 512, 32},
        {"g16u2", mg::rx_group_kernel<mg::kRxChunk, false, 16, 0, 1, 1024, 2>, 1024, 64},
        {"g4b128", mg::rx_group_kernel<mg::kRxChunk, false, 4, 0, 1, 128>, 128, 32},
        {"g4b64", mg::rx_group_kernel<mg::kRxChunk, false, 4, 0, 1, 64>, 64, 16},
        {"g8b128", mg::rx_group_kernel<mg::kRxChunk, false, 8, 0, 1, 128>, 128, 16},
        {"g8u2b256", mg::rx_group_kernel<mg::kRxChunk, false, 8, 0, 1, 256, 2>, 256, 32},
        {"g8u6b256", mg::rx_group_kernel<mg::kRxChunk, false, 8, 0, 1, 256, 6>, 256, 32},
        {"g16b128", mg::rx_group_kernel<mg::kRxChunk, false, 16, 0, 1, 128>, 128, 8},
        {"span2", mg::rx_span_kernel<mg::kRxChunk, false, 2>, 256, 64},
        {"span4", mg::rx_span_kernel<mg::kRxChunk, false, 4>, 256, 64},
        {"span8", mg::rx_span_kernel<mg::kRxChunk, false, 8>, 256, 64},
        {"span4_p1", mg::rx_span_kernel<mg::kRxChunk, false, 4, 1>, 256, 64},
        {"span4_desc", mg::rx_span_kernel<mg::kRxChunk, false, 4, 2>, 256, 64},
        {"rows", mg::rx_kernel<mg::kRxChunk, false, mg::kSchedSorted>, 256, 0},
    };
    for (uint32_t n : ns) {
        std::vector<mtcp_gpu_desc> desc(n);
        uint64_t off = 0;
        for (uint32_t i = 0; i < n; ++i) {
            desc[i].offset = (uint32_t)(off >> 6);
            desc[i].len = (uint16_t)len_of(i);
            desc[i].flags = desc[i].rsvd = 0;
            off += (len_of(i) + 63) & ~63u;
        }
        uint8_t *d_buf;
        mtcp_gpu_desc *d_desc;
        mtcp_gpu_result *d_out;
        CK(hipMalloc(&d_buf, off));
        CK(hipMalloc(&d_desc, n * sizeof(mtcp_gpu_desc)));
        CK(hipMalloc(&d_out, n * sizeof(mtcp_gpu_result)));
        CK(hipMemcpy(d_desc, desc.data(), n * sizeof(mtcp_gpu_desc), hipMemcpyHostToDevice));
        if (mtcp_gpu_pktgen_dev(d_buf, off, d_desc, n, 6, 7, 0, nullptr) != 0) return 1;
        CK(hipDeviceSynchronize());
        mg::KParams kp{};
        kp.buf = d_buf;
        kp.buf_len = off;
        kp.desc = d_desc;
        kp.n = n;
        kp.off_shift = 6;
        kp.out = d_out;
        kp.rss_nq = 1;
        printf("{\"L\": %u, \"n\": %u", L, n);
        const char *only = getenv("WP_ONLY");             // e.g. "full,phase1" (PMC runs)
        const int rounds = getenv("WP_ROUNDS") ? atoi(getenv("WP_ROUNDS")) : 5;
        // WP_SYNC=1: wait for each launch before issuing the next, so that a
        // rocprofv3 kernel trace sees every dispatch on an idle GPU (its
        // begin->end is then the kernel's own, with no queueing behind the
        // previous launch); the event figure then includes the host round trip
        const bool sync_each = getenv("WP_SYNC") && atoi(getenv("WP_SYNC"));
        for (const V &v : vs) {
            if (only && !strstr(only, v.name)) continue;
            const uint32_t blocks = v.ppb ? (n + v.ppb - 1) / v.ppb
                                    : v.persist ? std::min<uint32_t>((n + 255) / 256, (uint32_t)cus * v.persist)
                                                : std::min<uint32_t>((n + 255) / 256, 512);
            std::vector<float> t;
            for (int r = 0; r < rounds; ++r) {
                for (int i = 0; i < 5; ++i) hipLaunchKernelGGL(v.fn, dim3(blocks), dim3(v.threads), 0, st, kp);
                CK(hipEventRecord(a, st));
                const int reps = rounds < 5 ? 2 : 100;
                for (int i = 0; i < reps; ++i) {
                    hipLaunchKernelGGL(v.fn, dim3(blocks), dim3(v.threads), 0, st, kp);
                    if (sync_each) CK(hipStreamSynchronize(st));
                }
                CK(hipEventRecord(b, st));
                CK(hipEventSynchronize(b));
                float ms;
                CK(hipEventElapsedTime(&ms, a, b));
                t.push_back(ms * 1e3f / reps);
            }
            std::sort(t.begin(), t.end());
            printf(", \"%s_us\": %.2f", v.name, t[t.size() / 2]);
            // every full variant's records must equal the wave kernel's
            static std::vector<mtcp_gpu_result> ref;
            const bool full = !strchr(v.name, '_') && strncmp(v.name, "empty", 5) && strcmp(v.name, "desc") &&
                              strcmp(v.name, "phase1") && strcmp(v.name, "head") && strcmp(v.name, "segsum") &&
                              strcmp(v.name, "p1nl2");
            if (full) {
                std::vector<mtcp_gpu_result> got(n);
                CK(hipMemcpy(got.data(), d_out, n * sizeof(mtcp_gpu_result), hipMemcpyDeviceToHost));
                if (!strcmp(v.name, "full")) ref = got;
                else if (ref.size() == n && memcmp(ref.data(), got.data(), n * sizeof(mtcp_gpu_result)) != 0) {
                    fprintf(stderr, "%s records differ from the wave kernel's (n %u)\n", v.name, n);
                    return 2;
                }
            }
        }
        printf("}\n");
        CK(hipFree(d_buf));
        CK(hipFree(d_desc));
        CK(hipFree(d_out));
    }
    return 0;
}
