// pcie_probe.hip — host -> device copy ceiling of the box's PCIe link, to
// judge mtcp_gpu_rx_chunk's PCIe-inclusive rate: pinned source, 1.5 GB in
// pieces of S MiB spread round-robin over K streams (K concurrent DMA
// copies), wall clock.
//   usage: pcie_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

int main() {
    const size_t total = 1536ull << 20;
    void *h, *d;
    CK(hipHostMalloc(&h, total, hipHostMallocDefault));
    CK(hipMalloc(&d, total));
    for (size_t i = 0; i < total; i += 4096) static_cast<char *>(h)[i] = (char)i;
    std::vector<hipStream_t> st(8);
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int k : {1, 2, 3, 4, 8}) {
        for (size_t mib : {16, 64, 256}) {
            const size_t piece = mib << 20;
            double best = 0;
            for (int rep = 0; rep < 4; ++rep) {
                CK(hipDeviceSynchronize());
                const auto t0 = std::chrono::steady_clock::now();
                size_t i = 0;
                for (size_t off = 0; off < total; off += piece, ++i) {
                    const size_t len = off + piece <= total ? piece : total - off;
                    CK(hipMemcpyAsync(static_cast<char *>(d) + off, static_cast<char *>(h) + off, len,
                                      hipMemcpyHostToDevice, st[i % k]));
                }
                for (int s = 0; s < k; ++s) CK(hipStreamSynchronize(st[s]));
                const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
                if (rep > 0 && total / sec / 1e9 > best) best = total / sec / 1e9;
            }
            printf("{\"probe\": \"h2d\", \"streams\": %d, \"piece_MiB\": %zu, \"GBs\": %.1f}\n", k, mib, best);
        }
    }
    return 0;
}
