// asan_host.hip — TEST HARNESS: the C ABI's host code (mtcp_gpu.hip,
// rxq.hip: staging, bounce buffers, gathers, parking, bounded waits) built
// with AddressSanitizer on the HOST side only (-Xarch_host -fsanitize=address;
// the kernels are not instrumented: this pool has no GPU ASan), driven through
// every host entry point, with and without a wait limit, healthy and behind a
// stall that makes each bounded call give up.  Run on the GPU box by
// tests/test_gpu_bounded.py::test_host_code_under_asan_on_the_gpu.
//   asan_host RX_BUF RX_DESC   -> one JSON line; ASan reports go to stderr
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../include/mtcp_gpu.h"
#include "../../include/mtcp_gpu_rxq.h"

namespace {

__global__ __launch_bounds__(64) void stall_kernel(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

void stall(mtcp_gpu_ctx *ctx, uint32_t us) {
    hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(mtcp_gpu_stream(ctx)),
                       (uint64_t)us * 100);
}

std::vector<uint8_t> slurp(const char *path) {
    std::vector<uint8_t> v;
    FILE *f = fopen(path, "rb");
    if (!f) return v;
    fseek(f, 0, SEEK_END);
    v.resize((size_t)ftell(f));
    fseek(f, 0, SEEK_SET);
    if (fread(v.data(), 1, v.size(), f) != v.size()) v.clear();
    fclose(f);
    return v;
}

int fails = 0;
#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) {                                                        \
            fprintf(stderr, "asan_host: check failed at line %d: %s\n", __LINE__, #c); \
            ++fails;                                                       \
        }                                                                  \
    } while (0)

struct Outputs {
    std::vector<uint8_t> rx, rx_unsorted, ptrs, tx, tx_ptrs, rxq;
    std::vector<uint32_t> bins;
    std::vector<mtcp_gpu_addr_entry> pool;
    uint32_t n_filled = 0, n_found = 0;
};

// every host entry point once on a context with wait limit `limit_us`;
// returns what they wrote (compared across limits by the caller)
Outputs run_all(const std::vector<uint8_t> &buf, const std::vector<mtcp_gpu_desc> &desc, uint32_t limit_us) {
    Outputs o;
    const uint32_t n = (uint32_t)desc.size();
    mtcp_gpu_ctx *ctx = nullptr;
    CHECK(mtcp_gpu_open(&ctx, 0, nullptr, 8, MTCP_GPU_F_RSS | MTCP_GPU_F_RSS_ENDIAN) == MTCP_GPU_OK);
    if (!ctx) return o;
    CHECK(mtcp_gpu_set_wait_limit(ctx, limit_us) == MTCP_GPU_OK);
    o.rx.assign((size_t)n * 40, 0xA5);
    CHECK(mtcp_gpu_rx_chunk(ctx, buf.data(), buf.size(), desc.data(), n, 0,
                            reinterpret_cast<mtcp_gpu_result *>(o.rx.data())) == MTCP_GPU_OK);
    std::vector<mtcp_gpu_desc> rev(desc.rbegin(), desc.rend());
    o.rx_unsorted.assign((size_t)n * 40, 0xA5);
    CHECK(mtcp_gpu_rx_chunk(ctx, buf.data(), buf.size(), rev.data(), n, 0,
                            reinterpret_cast<mtcp_gpu_result *>(o.rx_unsorted.data())) == MTCP_GPU_OK);
    const uint32_t np = n < 500 ? n : 500;
    std::vector<const uint8_t *> ptrs(np);
    std::vector<uint16_t> lens(np);
    for (uint32_t i = 0; i < np; ++i) ptrs[i] = buf.data() + desc[i].offset, lens[i] = desc[i].len;
    o.ptrs.assign((size_t)np * 40, 0xA5);
    CHECK(mtcp_gpu_rx_ptrs(ctx, ptrs.data(), lens.data(), np,
                           reinterpret_cast<mtcp_gpu_result *>(o.ptrs.data())) == MTCP_GPU_OK);
    o.tx = buf;
    CHECK(mtcp_gpu_tx_fill(ctx, o.tx.data(), o.tx.size(), desc.data(), n, 0, &o.n_filled) == MTCP_GPU_OK);
    o.tx_ptrs = buf;
    std::vector<uint8_t *> wptrs(64);
    std::vector<uint16_t> wlens(64);
    for (uint32_t i = 0; i < 64 && i < n; ++i) wptrs[i] = o.tx_ptrs.data() + desc[i].offset, wlens[i] = desc[i].len;
    CHECK(mtcp_gpu_tx_fill_ptrs(ctx, wptrs.data(), wlens.data(), n < 64 ? n : 64, nullptr) == MTCP_GPU_OK);
    o.bins.assign(n, 0xA5A5A5A5u);
    CHECK(mtcp_gpu_flow_hash(ctx, reinterpret_cast<const mtcp_gpu_result *>(o.rx.data()), n, o.bins.data()) ==
          MTCP_GPU_OK);
    o.pool.resize(4 * 64511);
    CHECK(mtcp_gpu_addr_pool_search(ctx, 1, 4, 0x0A00000Au, 4, 0x0B00000Au, 0x5000, 1, o.pool.data(),
                                    (uint32_t)o.pool.size(), &o.n_found) == MTCP_GPU_OK);
    mtcp_gpu_rxq *q = nullptr;
    CHECK(mtcp_gpu_rxq_create(&q, ctx, 256, 256 * 20000) == MTCP_GPU_OK);
    if (q) {
        for (uint32_t i = 0; i < 256 && i < n; ++i) CHECK(mtcp_gpu_rxq_push(q, buf.data() + desc[i].offset, desc[i].len) == MTCP_GPU_OK);
        uint32_t done = 0;
        CHECK(mtcp_gpu_rxq_flush(q, &done) == MTCP_GPU_OK);
        for (uint32_t i = 0; i < done; ++i) {
            const mtcp_gpu_result *r = nullptr;
            uint16_t len = 0;
            (void)mtcp_gpu_rxq_get(q, i, &len, &r);
            if (r) o.rxq.insert(o.rxq.end(), reinterpret_cast<const uint8_t *>(r), reinterpret_cast<const uint8_t *>(r) + 40);
        }
        mtcp_gpu_rxq_destroy(q);
    }
    CHECK(mtcp_gpu_sync(ctx) == MTCP_GPU_OK);
    mtcp_gpu_close(ctx);
    return o;
}

// each bounded call behind a stall: ETIMEDOUT, and the caller's buffer
// untouched once the device is idle again
int timeouts(const std::vector<uint8_t> &buf, const std::vector<mtcp_gpu_desc> &desc) {
    const uint32_t n = (uint32_t)desc.size();
    int seen = 0;
    for (int call = 0; call < 7; ++call) {
        mtcp_gpu_ctx *ctx = nullptr;
        if (mtcp_gpu_open(&ctx, 0, nullptr, 8, MTCP_GPU_F_RSS) != MTCP_GPU_OK) {
            ++fails;
            continue;
        }
        std::vector<uint8_t> out((size_t)n * 40, 0xA5), host = buf;
        std::vector<uint32_t> bins(n, 0xA5A5A5A5u);
        // warm: stages sized without a limit
        CHECK(mtcp_gpu_rx_chunk(ctx, buf.data(), buf.size(), desc.data(), n, 0,
                                reinterpret_cast<mtcp_gpu_result *>(out.data())) == MTCP_GPU_OK);
        std::vector<uint8_t> warm_out = out;
        out.assign(out.size(), 0xA5);
        mtcp_gpu_set_wait_limit(ctx, 30000);
        stall(ctx, 300000);
        int rc = 0;
        uint32_t cnt = 0;
        std::vector<const uint8_t *> ptrs(64);
        std::vector<uint8_t *> wptrs(64);
        std::vector<uint16_t> lens(64);
        for (uint32_t i = 0; i < 64 && i < n; ++i)
            ptrs[i] = buf.data() + desc[i].offset, wptrs[i] = host.data() + desc[i].offset, lens[i] = desc[i].len;
        std::vector<mtcp_gpu_addr_entry> pool(4 * 64511);
        uint32_t found = 0;
        switch (call) {
            case 0: rc = mtcp_gpu_rx_chunk(ctx, buf.data(), buf.size(), desc.data(), n, 0,
                                           reinterpret_cast<mtcp_gpu_result *>(out.data())); break;
            case 1: rc = mtcp_gpu_rx_ptrs(ctx, ptrs.data(), lens.data(), 64,
                                          reinterpret_cast<mtcp_gpu_result *>(out.data())); break;
            case 2: rc = mtcp_gpu_tx_fill(ctx, host.data(), host.size(), desc.data(), n, 0, &cnt); break;
            case 3: rc = mtcp_gpu_tx_fill_ptrs(ctx, wptrs.data(), lens.data(), 64, &cnt); break;
            case 4: rc = mtcp_gpu_flow_hash(ctx, reinterpret_cast<const mtcp_gpu_result *>(warm_out.data()), n,
                                            bins.data()); break;
            case 5: rc = mtcp_gpu_addr_pool_search(ctx, 1, 4, 0x0A00000Au, 4, 0x0B00000Au, 0x5000, 1, pool.data(),
                                                   (uint32_t)pool.size(), &found); break;
            default: rc = mtcp_gpu_reserve(ctx, 256u << 20, 1u << 20); break;
        }
        CHECK(rc == MTCP_GPU_ETIMEDOUT);
        seen += rc == MTCP_GPU_ETIMEDOUT;
        const hipStream_t st = reinterpret_cast<hipStream_t>(mtcp_gpu_stream(ctx));
        mtcp_gpu_close(ctx);                       // abandoned: host state only
        CHECK(hipStreamSynchronize(st) == hipSuccess);   // the stall and the work behind it end
        for (size_t i = 0; i < out.size(); ++i)
            if (out[i] != 0xA5) { CHECK(!"rx records written after the call gave up"); break; }
        CHECK(memcmp(host.data(), buf.data(), buf.size()) == 0);
        for (uint32_t b : bins)
            if (b != 0xA5A5A5A5u) { CHECK(!"flow bins written after the call gave up"); break; }
    }
    return seen;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: asan_host RX_BUF RX_DESC\n");
        return 2;
    }
    std::vector<uint8_t> buf = slurp(argv[1]);
    std::vector<uint8_t> draw = slurp(argv[2]);
    if (buf.empty() || draw.empty()) return 2;
    buf.resize((buf.size() + 63) & ~size_t(63), 0);
    std::vector<mtcp_gpu_desc> desc(draw.size() / sizeof(mtcp_gpu_desc));
    memcpy(desc.data(), draw.data(), desc.size() * sizeof(mtcp_gpu_desc));

    // golden frames: unbounded and bounded calls write the same bytes
    const Outputs a = run_all(buf, desc, 0), b = run_all(buf, desc, 5000000);
    int same = a.rx == b.rx && a.rx_unsorted == b.rx_unsorted && a.ptrs == b.ptrs && a.tx == b.tx &&
               a.tx_ptrs == b.tx_ptrs && a.bins == b.bins && a.rxq == b.rxq && a.n_filled == b.n_filled &&
               a.n_found == b.n_found &&
               memcmp(a.pool.data(), b.pool.data(), a.pool.size() * sizeof(mtcp_gpu_addr_entry)) == 0;
    CHECK(same);
    // a chunk over several 64 MiB stages (random bytes: the bounce and
    // collect logic across stages, not the verdicts)
    const uint32_t big_n = 150000;
    std::vector<uint8_t> big((size_t)big_n * 1536);
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < big.size(); i += 8) {
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        memcpy(&big[i], &x, 8);
    }
    std::vector<mtcp_gpu_desc> bdesc(big_n);
    for (uint32_t i = 0; i < big_n; ++i) bdesc[i] = {i * 1536u, (uint16_t)(64 + (i * 37u) % 1437u), 0, 0};
    std::vector<uint8_t> r0((size_t)big_n * 40), r1((size_t)big_n * 40, 0xA5);
    mtcp_gpu_ctx *ctx = nullptr;
    CHECK(mtcp_gpu_open(&ctx, 0, nullptr, 1, 0) == MTCP_GPU_OK);
    if (ctx) {
        CHECK(mtcp_gpu_rx_chunk(ctx, big.data(), big.size(), bdesc.data(), big_n, 0,
                                reinterpret_cast<mtcp_gpu_result *>(r0.data())) == MTCP_GPU_OK);
        mtcp_gpu_set_wait_limit(ctx, 10000000);
        CHECK(mtcp_gpu_rx_chunk(ctx, big.data(), big.size(), bdesc.data(), big_n, 0,
                                reinterpret_cast<mtcp_gpu_result *>(r1.data())) == MTCP_GPU_OK);
        CHECK(r0 == r1);
        mtcp_gpu_close(ctx);
    }
    const int seen = timeouts(buf, desc);
    CHECK(hipDeviceSynchronize() == hipSuccess);
    printf("{\"ok\": %d, \"fails\": %d, \"bounded_equals_unbounded\": %d, \"timeouts\": %d, \"frames\": %zu}\n",
           fails == 0, fails, same, seen, desc.size());
    return fails ? 1 : 0;
}
