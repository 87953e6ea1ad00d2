// pktgen.hip — synthetic traffic on the GPU (spec: include/mtcp_gpu_pktgen.h).
// Payload fill is one wave per frame writing 16 B per lane; headers one lane
// per frame; checksums by the product's tx-fill kernel; then corruption.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtcp_gpu_pktgen.h"
#include "rx_kernels.hpp"

namespace {

constexpr uint64_t kGamma = 0x9E3779B97F4A7C15ull;

__device__ __forceinline__ uint64_t mix(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ uint64_t state(uint64_t seed, uint64_t i) {
    return mix(seed ^ (i * 0xD1342543DE82EF95ull + 0x632BE59BD9B4E019ull));
}
__device__ __forceinline__ uint64_t rk(uint64_t s, uint64_t k) { return mix(s + (k + 1) * kGamma); }

struct GenParams {
    uint8_t *buf;
    uint64_t buf_len;
    const mtcp_gpu_desc *desc;
    uint32_t n, off_shift;
    uint64_t seed, first;
};

__device__ __forceinline__ bool frame_of(const GenParams &gp, uint32_t i, uint8_t *&p, uint32_t &L) {
    const mtcp_gpu_desc d = gp.desc[i];
    const uint64_t pos = (uint64_t)d.offset << gp.off_shift;
    L = d.len;
    const uint32_t padded = (L + 63u) & ~63u;
    p = gp.buf + pos;
    return (pos & 63) == 0 && pos + padded <= gp.buf_len;
}

__global__ __launch_bounds__(256) void gen_fill(GenParams gp) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    for (uint32_t i = wave; i < gp.n; i += gridDim.x * 4) {
        uint8_t *p;
        uint32_t L;
        if (!frame_of(gp, i, p, L)) continue;
        const uint64_t s = state(gp.seed, gp.first + i);
        const uint32_t nchunk = ((L + 63u) & ~63u) >> 4;
        for (uint32_t c = lane; c < nchunk; c += 64) {
            const uint32_t pb = c * 16;
            uint64_t w0 = rk(s, 16 + (pb >> 3)), w1 = rk(s, 17 + (pb >> 3));
            if (pb + 16 > L) {   // zero bytes >= L
                const int k0 = (int)L - (int)pb;           // bytes to keep
                const int k1 = k0 - 8;
                w0 = k0 <= 0 ? 0 : k0 >= 8 ? w0 : (w0 & ((1ull << (8 * k0)) - 1));
                w1 = k1 <= 0 ? 0 : k1 >= 8 ? w1 : (w1 & ((1ull << (8 * k1)) - 1));
            }
            *reinterpret_cast<uint4 *>(p + pb) =
                make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
        }
    }
}

__global__ __launch_bounds__(256) void gen_headers(GenParams gp) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= gp.n) return;
    uint8_t *p;
    uint32_t L;
    if (!frame_of(gp, i, p, L) || L < 54) return;
    const uint64_t s = state(gp.seed, gp.first + i);
    const uint64_t r0 = rk(s, 0), r1 = rk(s, 1), r2 = rk(s, 2), r3 = rk(s, 3), r4 = rk(s, 4),
                   r5 = rk(s, 5);
    const uint32_t doff = (L >= 66 && ((r4 >> 32) & 1)) ? 8 : 5;
    const uint32_t ip_len = L - 14;
    for (int b = 0; b < 6; ++b) {
        p[b] = (uint8_t)(r0 >> (8 * b));
        p[6 + b] = (uint8_t)(r1 >> (8 * b));
    }
    p[12] = 0x08; p[13] = 0x00; p[14] = 0x45; p[15] = 0x00;
    p[16] = (uint8_t)(ip_len >> 8); p[17] = (uint8_t)ip_len;
    p[18] = (uint8_t)(r0 >> 48); p[19] = (uint8_t)(r0 >> 56);
    p[20] = 0x40; p[21] = 0x00; p[22] = 64; p[23] = 6; p[24] = 0; p[25] = 0;
    for (int b = 0; b < 8; ++b) p[26 + b] = (uint8_t)(r2 >> (8 * b));
    for (int b = 0; b < 8; ++b) p[34 + b] = (uint8_t)(r3 >> (8 * b));
    for (int b = 0; b < 4; ++b) p[42 + b] = (uint8_t)(r4 >> (8 * b));
    p[46] = (uint8_t)(doff << 4);
    p[47] = (uint8_t)(0x10 | (((r4 >> 33) & 1) ? 0x08 : 0));
    p[48] = (uint8_t)(r4 >> 40); p[49] = (uint8_t)(r4 >> 48);
    p[50] = 0; p[51] = 0; p[52] = 0; p[53] = 0;
    if (doff == 8) {
        p[54] = 0x01; p[55] = 0x01; p[56] = 0x08; p[57] = 0x0A;
        for (int b = 0; b < 8; ++b) p[58 + b] = (uint8_t)(r5 >> (8 * b));
    }
}

__global__ __launch_bounds__(256) void gen_corrupt(GenParams gp) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= gp.n) return;
    uint8_t *p;
    uint32_t L;
    if (!frame_of(gp, i, p, L) || L < 54) return;
    const uint64_t s = state(gp.seed, gp.first + i);
    const uint64_t c = rk(s, 6);
    const uint32_t doff = p[46] >> 4;
    const uint32_t T = 34, pay = T + 4 * doff;
    if ((c & 1023) == 0) {
        const uint32_t lo = pay < L ? pay : T;
        const uint32_t b = (uint32_t)((c >> 10) % (8ull * (L - lo)));
        p[lo + (b >> 3)] ^= (uint8_t)(1u << (b & 7));
    }
    if (((c >> 32) & 4095) == 0) {
        const uint32_t b = (uint32_t)((c >> 44) % 160);
        p[14 + (b >> 3)] ^= (uint8_t)(1u << (b & 7));
    }
}

}  // namespace

extern "C" int mtcp_gpu_pktgen_dev(void *d_buf, uint64_t buf_len, const mtcp_gpu_desc *d_desc,
                                   uint32_t n, uint32_t off_shift, uint64_t seed,
                                   uint64_t first_index, void *stream) {
    if (!d_buf || (!d_desc && n) || off_shift > 16) return MTCP_GPU_EINVAL;
    if (n == 0) return MTCP_GPU_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    GenParams gp{static_cast<uint8_t *>(d_buf), buf_len, d_desc, n, off_shift, seed, first_index};
    const uint32_t wave_blocks = (n + 3) / 4 < 8192 ? (n + 3) / 4 : 8192;
    const uint32_t lane_blocks = (n + 255) / 256;
    hipLaunchKernelGGL(gen_fill, dim3(wave_blocks), dim3(256), 0, st, gp);
    hipLaunchKernelGGL(gen_headers, dim3(lane_blocks), dim3(256), 0, st, gp);
    mg::KParams kp{};
    kp.buf = static_cast<const uint8_t *>(d_buf);
    kp.buf_len = buf_len & ~15ull;
    kp.desc = d_desc;
    kp.n = n;
    kp.off_shift = off_shift;
    const uint32_t groups = (n + 63) / 64;
    const uint32_t fill_blocks = (groups + 3) / 4 < 2048 ? (groups + 3) / 4 : 2048;
    hipLaunchKernelGGL((mg::rx_kernel<mg::kTxChunk, false, mg::kSchedUnrolled, true>), dim3(fill_blocks), dim3(256), 0, st, kp);
    hipLaunchKernelGGL(gen_corrupt, dim3(lane_blocks), dim3(256), 0, st, gp);
    return hipGetLastError() == hipSuccess ? MTCP_GPU_OK : MTCP_GPU_EIO;
}
