// stream_ceiling.hip — the box's read-only streaming ceiling, measured on the
// bench's own frame buffer in the same run ("also report
// against a measured read-only streaming ceiling on the box").  Measurement
// infrastructure: bench.py loads tools/libstream_ceiling.so for this one leg;
// nothing here is part of libmtcp_gpu.so or of the timed rx launches.
//
// A grid-stride walk over the whole buffer: each lane keeps U non-temporal
// 16 B loads in flight (global_load_dwordx4 nt, as the rx kernels' frame
// stream), v_sad_u16 folds them so the loads stay live, one word per
// workgroup is written only if an impossible sum shows up.  Eight shapes (U
// 3, 4, 6 or 8, 2 or 4 workgroups of 256 lanes per CU) are timed and the
// fastest is the ceiling (on C2's buffer U 3 at 2 per CU: 24 KB in flight per
// CU); every byte of the buffer, slot padding included, is read once.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void stream_read(const v4u *__restrict__ p, uint64_t n16, uint32_t *sink) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            v[u] = __builtin_nontemporal_load(p + (j < n16 ? j : n16 - 1));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            acc = __builtin_amdgcn_sad_u16(v[u].x, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].y, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].z, 0u, acc);
            acc = __builtin_amdgcn_sad_u16(v[u].w, 0u, acc);
        }
    }
    if (acc == 0x9E3779B9u) sink[blockIdx.x] = acc;
}

// The tx fill's memory pattern without its arithmetic (f1):
// a 16-lane row reads a frame's 16 B chunks (U loads per lane in flight),
// then lane 1 and lane 3 of the row write the u16 at frame bytes 24..25 and
// 50..51 (iph->check, and tcph->check for ihl 5: ip_out.c:164,
// tcp_out.c:329) — the value already there, xor a sum-dependent 0, so the
// buffer keeps its bytes while the store cannot be elided.  Frames come from
// the descriptors (offset << off_shift, len), as the fill reads them.
template <int U>
__global__ __launch_bounds__(256) void patch_walk(uint8_t *__restrict__ buf, const uint2 *__restrict__ desc,
                                                  uint32_t n, uint32_t off_shift) {
    const uint32_t lane = threadIdx.x & 63, row = lane >> 4, rl = lane & 15;
    uint32_t acc = 0;
    // rows walk their frames independently (no cross-lane step in the loop)
    for (uint32_t f = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + row; f < n; f += gridDim.x * 16) {
        const uint2 d = desc[f];
        const uint64_t base = (uint64_t)d.x << off_shift;
        const uint32_t len = d.y & 0xFFFFu;
        const uint32_t nch = (len + 15) >> 4;
        const v4u *p = reinterpret_cast<const v4u *>(buf + base);
        v4u first = {0, 0, 0, 0};
        for (uint32_t c0 = 0; c0 < nch; c0 += 16 * U) {
            v4u v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = c0 + u * 16 + rl;
                v[u] = __builtin_nontemporal_load(p + (c < nch ? c : nch - 1));
            }
            if (c0 == 0) first = v[0];
#pragma unroll
            for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_sad_u16(v[u].x ^ v[u].y, v[u].z ^ v[u].w, acc);
        }
        const uint16_t z = acc == 0x9E3779B9u ? 1 : 0;
        uint16_t *q = reinterpret_cast<uint16_t *>(buf + base);
        if (len >= 52 && rl == 1) q[12] = (uint16_t)(first.z & 0xFFFFu) ^ z;   // bytes 24..25
        if (len >= 52 && rl == 3) q[25] = (uint16_t)(first.x >> 16) ^ z;       // bytes 50..51
    }
}

}  // namespace

extern "C" {

// The f1 row's ceiling on the bench's own frames (patch_walk above): the
// fastest of four shapes (U 6 or 8 loads per lane, 2 or 4 workgroups per
// CU), `reps` launches each after 3 untimed, HIP events on `stream`.
// *shape = U * 10 + workgroups per CU.  The frames' bytes are unchanged.
int patch_ceiling_us(void *buf, const void *desc, uint32_t n, uint32_t off_shift, int reps, void *stream,
                     float *best_us, int *shape) {
    if (!buf || !desc || !n || reps <= 0 || !best_us || !shape) return -1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return -1;
    hipEvent_t a = nullptr, b = nullptr;
    int rc = 0;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) rc = -1;
    uint8_t *p = reinterpret_cast<uint8_t *>(buf);
    const uint2 *dsc = reinterpret_cast<const uint2 *>(desc);
    *best_us = 0.0f;
    *shape = 0;
    for (int u : {6, 8}) {
        for (int per_cu : {2, 4}) {
            if (rc) break;
            const dim3 grid((unsigned)(per_cu * cus)), block(256);
            auto launch = [&] {
                if (u == 6) hipLaunchKernelGGL(patch_walk<6>, grid, block, 0, st, p, dsc, n, off_shift);
                else hipLaunchKernelGGL(patch_walk<8>, grid, block, 0, st, p, dsc, n, off_shift);
            };
            for (int i = 0; i < 3; ++i) launch();
            if (hipEventRecord(a, st) != hipSuccess) { rc = -1; break; }
            for (int i = 0; i < reps; ++i) launch();
            float ms = 0.0f;
            if (hipEventRecord(b, st) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
                hipEventElapsedTime(&ms, a, b) != hipSuccess || hipGetLastError() != hipSuccess) {
                rc = -1;
                break;
            }
            const float us = ms * 1e3f / reps;
            if (*best_us == 0.0f || us < *best_us) {
                *best_us = us;
                *shape = u * 10 + per_cu;
            }
        }
    }
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    (void)hipStreamSynchronize(st);
    return rc;
}

// Times `reps` back-to-back launches of each shape over [buf, buf + bytes) on
// `stream` (HIP events, after 3 untimed launches) and returns the fastest
// shape's average launch time in *best_us and the shape in *shape
// (U * 10 + workgroups per CU).  0 on success, -1 on a HIP error or bad
// arguments.
int stream_ceiling_us(const void *buf, uint64_t bytes, int reps, void *stream, float *best_us, int *shape) {
    if (!buf || bytes < 16 || reps <= 0 || !best_us || !shape) return -1;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        return -1;
    uint32_t *sink = nullptr;
    if (hipMalloc(&sink, (size_t)4 * cus * sizeof(uint32_t)) != hipSuccess) return -1;
    hipEvent_t a = nullptr, b = nullptr;
    int rc = 0;
    if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) rc = -1;
    const v4u *p = reinterpret_cast<const v4u *>(buf);
    const uint64_t n16 = bytes / 16;
    *best_us = 0.0f;
    *shape = 0;
    for (int u : {3, 4, 6, 8}) {
        for (int per_cu : {2, 4}) {
            if (rc) break;
            const dim3 grid((unsigned)(per_cu * cus)), block(256);
            auto launch = [&] {
                switch (u) {
                case 3: hipLaunchKernelGGL(stream_read<3>, grid, block, 0, st, p, n16, sink); break;
                case 4: hipLaunchKernelGGL(stream_read<4>, grid, block, 0, st, p, n16, sink); break;
                case 6: hipLaunchKernelGGL(stream_read<6>, grid, block, 0, st, p, n16, sink); break;
                default: hipLaunchKernelGGL(stream_read<8>, grid, block, 0, st, p, n16, sink); break;
                }
            };
            for (int i = 0; i < 3; ++i) launch();
            if (hipEventRecord(a, st) != hipSuccess) { rc = -1; break; }
            for (int i = 0; i < reps; ++i) launch();
            float ms = 0.0f;
            if (hipEventRecord(b, st) != hipSuccess || hipEventSynchronize(b) != hipSuccess ||
                hipEventElapsedTime(&ms, a, b) != hipSuccess || hipGetLastError() != hipSuccess) {
                rc = -1;
                break;
            }
            const float us = ms * 1e3f / reps;
            if (*best_us == 0.0f || us < *best_us) {
                *best_us = us;
                *shape = u * 10 + per_cu;
            }
        }
    }
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    (void)hipStreamSynchronize(st);
    (void)hipFree(sink);
    return rc;
}

}  // extern "C"
