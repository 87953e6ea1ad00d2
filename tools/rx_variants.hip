// rx_variants.hip — in-process A/B timing of rx-kernel variants on one GPU
// (guide §5.4 rule 24: interleaved rounds in ONE process).  Frames come from
// libmtcp_gpu.so's generator; every variant's results must be byte-identical.
//   usage: rx_variants [config: c2|c3|c5] [rounds]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../include/mtcp_gpu_pktgen.h"
#include "../mtcp_amd/csrc/rx_kernels.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef void (*kfn)(mg::KParams);

__global__ __launch_bounds__(256) void plain_stream_nt(mg::KParams kp) {
    const uint64_t base = (uint64_t)(uintptr_t)kp.buf;
    const uint64_t n16 = kp.buf_len / 16;
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
        mg::v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = mg::gload_nt(base + 16 * ((i + u * 256 < n16) ? i + u * 256 : i));
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = mg::halves4(v[u], acc);
    }
    if (acc == 0x12345678u) kp.out[0].saddr = acc;
}

// Pure read-only stream over the same frame buffer (the measured ceiling on
// THIS data): grid-stride dwordx4 + v_sad_u16, 4 loads in flight per lane.
__global__ __launch_bounds__(256) void plain_stream(mg::KParams kp) {
    const uint4 *p = reinterpret_cast<const uint4 *>(kp.buf);
    const uint64_t n16 = kp.buf_len / 16;
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < n16; i += stride) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = (i + u * 256 < n16) ? p[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            acc = __builtin_amdgcn_sad_u16(v[u].x, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].y, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].z, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].w, 0u, acc);
        }
    }
    if (acc == 0x12345678u) kp.out[0].saddr = acc;
}

struct Variant { const char *name; kfn fn; uint32_t blocks_per_cu; };

static uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int main(int argc, char **argv) {
    const char *cfg = argc > 1 ? argv[1] : "c2";
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const bool single = argc > 3 && !strcmp(argv[3], "single");   // profiling: variant 0 only
    uint32_t n = 1u << 20, L = 1500;
    int bimodal = 0, rss = 0;
    uint64_t seed = 2;
    if (!strcmp(cfg, "c3")) { bimodal = 1; rss = 1; seed = 3; }
    if (!strcmp(cfg, "c5")) { n = 1u << 19; L = 9000; seed = 5; }

    std::vector<mtcp_gpu_desc> desc(n);
    uint64_t off = 0, frame_bytes = 0;
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t len = L;
        if (bimodal) {
            uint64_t z = mix((uint64_t)i * 0x9E3779B97F4A7C15ull + seed * 0xD6E8FEB86659FD93ull);
            len = (z & 1) ? 1500 : 64;
        }
        desc[i].offset = (uint32_t)(off >> 6);
        desc[i].len = (uint16_t)len;
        desc[i].flags = desc[i].rsvd = 0;
        off += (len + 63) & ~63u;
        frame_bytes += len;
    }
    uint8_t *d_buf;
    mtcp_gpu_desc *d_desc;
    mtcp_gpu_result *d_out, *d_ref;
    uint32_t *d_tab;
    CK(hipMalloc(&d_buf, off));
    CK(hipMalloc(&d_desc, n * sizeof(mtcp_gpu_desc)));
    CK(hipMalloc(&d_out, n * sizeof(mtcp_gpu_result)));
    CK(hipMalloc(&d_ref, n * sizeof(mtcp_gpu_result)));
    CK(hipMalloc(&d_tab, mg::kRssTableWords * 4));
    CK(hipMemset(d_tab, 0x5A, mg::kRssTableWords * 4));
    CK(hipMemcpy(d_desc, desc.data(), n * sizeof(mtcp_gpu_desc), hipMemcpyHostToDevice));
    if (mtcp_gpu_pktgen_dev(d_buf, off, d_desc, n, 6, seed, 0, nullptr) != 0) return 1;
    CK(hipDeviceSynchronize());

    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const uint32_t cus = prop.multiProcessorCount;

    mg::KParams kp{};
    kp.buf = d_buf;
    kp.buf_len = off;
    kp.desc = d_desc;
    kp.n = n;
    kp.off_shift = 6;
    kp.rss_tables = d_tab;
    kp.rss_nq = 8;
    kp.rss_endian = 1;

    std::vector<Variant> vs;
    using namespace mg;
    if (rss) {
        vs.push_back({"rss_U6_cu4", rx_kernel<kRxChunk, true, 0, 8, true, 6, false>, 4});
    } else {
        vs.push_back({"U6_cu2", rx_kernel<kRxChunk, false, 0, 8, true, 6, false>, 2});
        vs.push_back({"abl1_p1only", rx_kernel<kRxChunk, false, 1, 8, true, 6, false>, 2});
        vs.push_back({"abl2_nolds", rx_kernel<kRxChunk, false, 2, 8, true, 6, false>, 2});
        vs.push_back({"abl3_nomask", rx_kernel<kRxChunk, false, 3, 8, true, 6, false>, 2});
        vs.push_back({"abl3_nomask_cu3", rx_kernel<kRxChunk, false, 3, 8, true, 6, false>, 3});
        vs.push_back({"plain_stream_nt_cu2", plain_stream_nt, 2});
    }
    if (single) vs.resize(1);
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> ms(vs.size());
    const int reps = 20;
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            const uint32_t groups = (n + 63) / 64;
            uint32_t blocks = strstr(vs[v].name, "plain") ? 1u << 20 : (groups + 3) / 4;
            if (blocks > cus * vs[v].blocks_per_cu) blocks = cus * vs[v].blocks_per_cu;
            kp.out = v == 0 ? d_ref : d_out;
            CK(hipMemset(kp.out, 0, n * sizeof(mtcp_gpu_result)));
            hipLaunchKernelGGL(vs[v].fn, dim3(blocks), dim3(256), 0, 0, kp);
            CK(hipEventRecord(a));
            for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(vs[v].fn, dim3(blocks), dim3(256), 0, 0, kp);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float t;
            CK(hipEventElapsedTime(&t, a, b));
            ms[v].push_back(t / reps);
            if (v > 0 && r == 0 && !strstr(vs[v].name, "abl") && !strstr(vs[v].name, "plain")) {
                std::vector<mtcp_gpu_result> x(n), y(n);
                CK(hipMemcpy(x.data(), d_ref, n * sizeof(mtcp_gpu_result), hipMemcpyDeviceToHost));
                CK(hipMemcpy(y.data(), d_out, n * sizeof(mtcp_gpu_result), hipMemcpyDeviceToHost));
                if (memcmp(x.data(), y.data(), n * sizeof(mtcp_gpu_result)) != 0) {
                    fprintf(stderr, "variant %s differs from %s\n", vs[v].name, vs[0].name);
                    return 2;
                }
            }
        }
    }
    for (size_t v = 0; v < vs.size(); ++v) {
        std::vector<float> m = ms[v];
        std::sort(m.begin(), m.end());
        const float med = m[m.size() / 2];
        printf("{\"config\": \"%s\", \"variant\": \"%s\", \"median_us\": %.2f, \"min_us\": %.2f, "
               "\"GBs_median\": %.1f, \"GBs_best\": %.1f, \"frac_of_8TBs\": %.4f}\n",
               cfg, vs[v].name, med * 1e3, m[0] * 1e3, frame_bytes / (med * 1e6),
               frame_bytes / (m[0] * 1e6), frame_bytes / (m[0] * 1e6) / 8000.0);
    }
    return 0;
}
