// frame_pattern.hip — read-only access-pattern study on a 1 M x 1536 B frame
// buffer: does splitting a wave-load over R frames (R rows of 64/R lanes, one
// frame each) or the number of frames a wave walks cost HBM bandwidth?
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
template <int R, int NLOAD, bool NT>
__global__ __launch_bounds__(256) void walk(const uint4 *__restrict__ p, uint32_t nframes,
                                            uint32_t *out) {
    constexpr int LPR = 64 / R;                      // lanes per row
    const uint32_t lane = threadIdx.x & 63, row = lane / LPR, rl = lane % LPR;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t nw = gridDim.x * 4;
    uint32_t acc = 0;
    for (uint32_t g = wave; g * 64 < nframes; g += nw) {           // 64 frames per wave
        for (uint32_t f0 = 0; f0 < 64; f0 += R) {
            const uint4 *fr = p + (uint64_t)(g * 64 + f0 + row) * 96;  // 1536 B = 96 chunks
            uint4 v[NLOAD];
#pragma unroll
            for (int u = 0; u < NLOAD; ++u) {
                uint32_t c = u * LPR + rl;
                c = c < 94 ? c : 93;
                if (NT) {
                    const v4u w = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(fr + c));
                    v[u] = make_uint4(w.x, w.y, w.z, w.w);
                } else {
                    v[u] = fr[c];
                }
            }
#pragma unroll
            for (int u = 0; u < NLOAD; ++u) {
                acc = __builtin_amdgcn_sad_u16(v[u].x, 0u, acc);
                acc = __builtin_amdgcn_sad_u16(v[u].y, 0u, acc);
                acc = __builtin_amdgcn_sad_u16(v[u].z, 0u, acc);
                acc = __builtin_amdgcn_sad_u16(v[u].w, 0u, acc);
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int R, int NLOAD, bool NT>
void run(const char *name, const uint4 *p, uint32_t nframes, uint32_t *out, int blocks) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 2; ++i) walk<R, NLOAD, NT><<<blocks, 256>>>(p, nframes, out);
    (void)hipEventRecord(a);
    for (int i = 0; i < 10; ++i) walk<R, NLOAD, NT><<<blocks, 256>>>(p, nframes, out);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    printf("{\"pattern\": \"%s\", \"blocks\": %d, \"us\": %.1f, \"GBs_1500\": %.1f}\n", name, blocks,
           ms * 100, nframes * 1500.0 / (ms / 10) / 1e6);
}

int main() {
    const uint32_t nframes = 1u << 20;
    uint4 *p;
    uint32_t *out;
    if (hipMalloc(&p, (size_t)nframes * 1536) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(p, 0x5a, (size_t)nframes * 1536);
    for (int blocks : {512, 768}) {
        run<1, 2, false>("1 frame x 1KiB/instr", p, nframes, out, blocks);
        run<4, 6, false>("4 frames x 256B", p, nframes, out, blocks);
        run<1, 2, true>("NT 1 frame x 1KiB/instr", p, nframes, out, blocks);
        run<2, 3, true>("NT 2 frames x 512B", p, nframes, out, blocks);
        run<4, 6, true>("NT 4 frames x 256B", p, nframes, out, blocks);
        run<8, 12, true>("NT 8 frames x 128B", p, nframes, out, blocks);
    }
    return 0;
}
