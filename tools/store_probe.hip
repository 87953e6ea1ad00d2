// store_probe.hip — what does writing the rx records cost by itself?
// Pure write streams (dwordx4 per lane, grid-stride, 2 workgroups per CU like
// the rx kernel) of the C2/C3 record volume (1 M x 40 B) and of 10x that,
// plain and non-temporal, and a read stream followed by a write burst in the
// same kernel (the shape of the rx kernel's deferred stores).
//   usage: store_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(256) void wstream(v4u *out, uint64_t n16, uint32_t salt) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
        const v4u v = {(uint32_t)i ^ salt, (uint32_t)i, salt, 7u};
        if (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}

// read `rbytes` (grid-stride, 4 loads in flight per lane), then write `n16`
// pieces of 16 B: the deferred-store shape
template <bool NT>
__global__ __launch_bounds__(256) void read_then_write(const v4u *in, uint64_t r16, v4u *out,
                                                       uint64_t n16) {
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 1024;
    for (uint64_t i = (uint64_t)blockIdx.x * 1024 + threadIdx.x; i < r16; i += stride) {
        v4u v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = __builtin_nontemporal_load(in + ((i + u * 256 < r16) ? i + u * 256 : i));
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_sad_u16(v[u].x ^ v[u].y ^ v[u].z ^ v[u].w, 0u, acc);
    }
    const uint64_t ws = (uint64_t)gridDim.x * 256;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += ws) {
        const v4u v = {acc, (uint32_t)i, 1u, 2u};
        if (NT) __builtin_nontemporal_store(v, out + i);
        else out[i] = v;
    }
}

__global__ void fill_random(uint32_t *p, uint64_t n4) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t z = i * 0x9E3779B97F4A7C15ull;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        p[i] = (uint32_t)(z ^ (z >> 31));
    }
}

template <class F>
float timeit(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) f();
    CK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;   // us
}

int main() {
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const uint32_t blocks = prop.multiProcessorCount * 2;
    const uint64_t rec = (1ull << 20) * 40;           // 41.9 MB
    const uint64_t big = rec * 10;
    const uint64_t rbytes = 1572864000ull;
    v4u *out, *in;
    CK(hipMalloc(&out, big));
    CK(hipMalloc(&in, rbytes));
    CK(hipMemset(in, 0x5a, rbytes));
    for (uint64_t bytes : {rec, big}) {
        const uint64_t n16 = bytes / 16;
        const float t0 = timeit([&] { wstream<false><<<blocks, 256>>>(out, n16, 1); }, 20);
        const float t1 = timeit([&] { wstream<true><<<blocks, 256>>>(out, n16, 1); }, 20);
        printf("{\"probe\": \"write_stream\", \"bytes\": %llu, \"plain_us\": %.2f, \"plain_GBs\": %.0f, "
               "\"nt_us\": %.2f, \"nt_GBs\": %.0f}\n", (unsigned long long)bytes, t0, bytes / t0 / 1e3,
               t1, bytes / t1 / 1e3);
    }
    const float r0 = timeit([&] { read_then_write<false><<<blocks, 256>>>(in, rbytes / 16, out, 0); }, 20);
    const float r1 = timeit([&] { read_then_write<false><<<blocks, 256>>>(in, rbytes / 16, out, rec / 16); }, 20);
    const float r2 = timeit([&] { read_then_write<true><<<blocks, 256>>>(in, rbytes / 16, out, rec / 16); }, 20);
    printf("{\"probe\": \"read_then_write\", \"read_bytes\": %llu, \"write_bytes\": %llu, \"read_only_us\": %.2f, "
           "\"plus_write_us\": %.2f, \"plus_write_nt_us\": %.2f}\n", (unsigned long long)rbytes,
           (unsigned long long)rec, r0, r1, r2);
    // the same read stream over constant and over random bytes
    const float c0 = timeit([&] { read_then_write<false><<<blocks, 256>>>(in, rbytes / 16, out, 0); }, 20);
    fill_random<<<4096, 256>>>(reinterpret_cast<uint32_t *>(in), rbytes / 4);
    CK(hipDeviceSynchronize());
    const float c1 = timeit([&] { read_then_write<false><<<blocks, 256>>>(in, rbytes / 16, out, 0); }, 20);
    const float c2 = timeit([&] { read_then_write<false><<<blocks, 256>>>(in, rbytes / 16, out, rec / 16); }, 20);
    printf("{\"probe\": \"data_dependence\", \"read_bytes\": %llu, \"const_us\": %.2f, \"const_GBs\": %.0f, "
           "\"random_us\": %.2f, \"random_GBs\": %.0f, \"random_plus_write_us\": %.2f}\n",
           (unsigned long long)rbytes, c0, rbytes / c0 / 1e3, c1, rbytes / c1 / 1e3, c2);
    // write streams of random-looking vs constant data
    const float w0 = timeit([&] { wstream<false><<<blocks, 256>>>(out, big / 16, 0); }, 20);
    printf("{\"probe\": \"write_stream_salt0\", \"bytes\": %llu, \"us\": %.2f}\n", (unsigned long long)big, w0);
    return 0;
}
