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

// tx-fill shape: a 16-lane row reads one 1536 B slot (6 x 16 B per lane),
// then PATCH 0: no write; 1: two 2-byte stores (iph->check at 24, tcph->check
// at 50); 2: the two 32 B sectors holding them rewritten whole (lanes 0..3,
// 16 B each); 3: 2-byte stores, but all of a wave's at the end (deferred).
template <int PATCH>
__global__ __launch_bounds__(256) void slot_patch(uint8_t *buf, uint32_t nslots) {
    const uint32_t lane = threadIdx.x & 63, row = lane >> 4, rl = lane & 15;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    uint32_t acc = 0;
    uint32_t held[16];
    uint32_t nh = 0;
    for (uint32_t s0 = wave * 4; s0 < nslots; s0 += nw * 4) {
        const uint32_t slot = s0 + row;
        const bool live = slot < nslots;
        const v4u *b = reinterpret_cast<const v4u *>(buf + (uint64_t)(live ? slot : 0) * 1536);
        v4u v[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) v[u] = b[rl + 16 * u];
#pragma unroll
        for (int u = 0; u < 6; ++u) acc = __builtin_amdgcn_sad_u16(v[u].x ^ v[u].y, v[u].z ^ v[u].w, acc);
        const uint32_t chk = acc & 0xFFFF;
        uint8_t *f = buf + (uint64_t)slot * 1536;
        if (PATCH == 1 && live && rl == 0) {
            reinterpret_cast<uint16_t *>(f)[12] = (uint16_t)chk;
            reinterpret_cast<uint16_t *>(f)[25] = (uint16_t)(chk >> 1);
        }
        if (PATCH == 2 && live && rl < 4) {
            v4u w = v[0];                                 // chunk rl of the slot
            if (rl == 1) w.z = (w.z & 0xFFFF0000u) | chk;                      // bytes 24..25
            if (rl == 3) w.x = (w.x & 0x0000FFFFu) | (chk << 16);              // bytes 50..51
            reinterpret_cast<v4u *>(f)[rl] = w;
        }
        if (PATCH == 7 && live && rl < 8) {                // the whole first 128 B line
            v4u w = rl < 4 ? v[0] : v[0] ^ v[1];
            if (rl == 1) w.z = (w.z & 0xFFFF0000u) | chk;
            if (rl == 3) w.x = (w.x & 0x0000FFFFu) | (chk << 16);
            reinterpret_cast<v4u *>(f)[rl] = w;
        }
        if ((PATCH == 8 || PATCH == 9) && live && rl < (PATCH == 8 ? 4u : 8u)) {   // non-temporal, whole
            v4u w = v[0];                                                        // 64 B / 128 B
            if (rl == 1) w.z = (w.z & 0xFFFF0000u) | chk;
            if (rl == 3) w.x = (w.x & 0x0000FFFFu) | (chk << 16);
            __builtin_nontemporal_store(w, reinterpret_cast<v4u *>(f) + rl);
        }
        if (PATCH == 6 && live && rl == 0) {
            __builtin_nontemporal_store((uint16_t)chk, reinterpret_cast<uint16_t *>(f) + 12);
            __builtin_nontemporal_store((uint16_t)(chk >> 1), reinterpret_cast<uint16_t *>(f) + 25);
        }
        if (PATCH == 3) {
            if (nh == 16) {                               // a burst of the held stores
#pragma unroll
                for (int i = 0; i < 16; ++i)
                    if (held[i] != 0xFFFFFFFFu) {
                        uint8_t *g = buf + (uint64_t)held[i] * 1536;
                        reinterpret_cast<uint16_t *>(g)[12] = (uint16_t)acc;
                        reinterpret_cast<uint16_t *>(g)[25] = (uint16_t)(acc >> 1);
                    }
                nh = 0;
            }
#pragma unroll
            for (int i = 15; i > 0; --i) held[i] = held[i - 1];
            held[0] = live && rl == 0 ? slot : 0xFFFFFFFFu;
            ++nh;
        }
    }
    if (PATCH == 3) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
            if ((uint32_t)i < nh && held[i] != 0xFFFFFFFFu) {
                uint8_t *f = buf + (uint64_t)held[i] * 1536;
                reinterpret_cast<uint16_t *>(f)[12] = (uint16_t)acc;
                reinterpret_cast<uint16_t *>(f)[25] = (uint16_t)(acc >> 1);
            }
    }
    if (acc == 0x12345678u) buf[0] = 1;
}

// the check writes alone, after a read-only pass: lane per slot, two 2-byte
// stores (WIDE 0) or the two 32 B sectors holding them (WIDE 1, 4 x 16 B)
template <int WIDE>
__global__ __launch_bounds__(256) void slot_scatter(uint8_t *buf, uint32_t nslots, uint32_t salt) {
    for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < nslots; s += gridDim.x * 256) {
        uint8_t *f = buf + (uint64_t)s * 1536;
        if (WIDE == 0) {
            reinterpret_cast<uint16_t *>(f)[12] = (uint16_t)(s ^ salt);
            reinterpret_cast<uint16_t *>(f)[25] = (uint16_t)(s + salt);
        } else if (WIDE == 3) {                      // read the 64 B, patch, write it whole
            v4u w[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) w[c] = reinterpret_cast<const v4u *>(f)[c];
            w[1].z = (w[1].z & 0xFFFF0000u) | (s & 0xFFFFu);
            w[3].x = (w[3].x & 0x0000FFFFu) | (salt << 16);
#pragma unroll
            for (int c = 0; c < 4; ++c) reinterpret_cast<v4u *>(f)[c] = w[c];
        } else {
            const v4u w = {s, salt, s ^ salt, 5u};
#pragma unroll
            for (int c = 0; c < 4 * WIDE; ++c) reinterpret_cast<v4u *>(f)[c] = w;
        }
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
    // tx-fill shape over 1 536 B slots (the f1 row's layout)
    {
        const uint32_t ns = (uint32_t)(rbytes / 1536);   // inside the 1.57 GB buffer
        uint8_t *sb = reinterpret_cast<uint8_t *>(in);
        const float p0 = timeit([&] { slot_patch<0><<<blocks, 256>>>(sb, ns); }, 20);
        const float p1 = timeit([&] { slot_patch<1><<<blocks, 256>>>(sb, ns); }, 20);
        const float p2 = timeit([&] { slot_patch<2><<<blocks, 256>>>(sb, ns); }, 20);
        const float p3 = timeit([&] { slot_patch<3><<<blocks, 256>>>(sb, ns); }, 20);
        const float p6 = timeit([&] { slot_patch<6><<<blocks, 256>>>(sb, ns); }, 20);
        const float q0 = timeit([&] { slot_scatter<0><<<(ns + 255) / 256, 256>>>(sb, ns, 3); }, 20);
        const float q1 = timeit([&] { slot_scatter<1><<<(ns + 255) / 256, 256>>>(sb, ns, 3); }, 20);
        const float q2 = timeit([&] { slot_patch<0><<<blocks, 256>>>(sb, ns);
                                      slot_scatter<0><<<(ns + 255) / 256, 256>>>(sb, ns, 3); }, 20);
        const float q3 = timeit([&] { slot_patch<0><<<blocks, 256>>>(sb, ns);
                                      slot_scatter<2><<<(ns + 255) / 256, 256>>>(sb, ns, 3); }, 20);
        const float q4 = timeit([&] { slot_patch<0><<<blocks, 256>>>(sb, ns);
                                      slot_scatter<1><<<(ns + 255) / 256, 256>>>(sb, ns, 3); }, 20);
        const float q5 = timeit([&] { slot_patch<0><<<blocks, 256>>>(sb, ns);
                                      slot_scatter<3><<<(ns + 255) / 256, 256>>>(sb, ns, 3); }, 20);
        const float q6 = timeit([&] { slot_scatter<3><<<(ns + 255) / 256, 256>>>(sb, ns, 3); }, 20);
        printf("{\"probe\": \"slot_rmw\", \"read_then_scatter_rmw64_us\": %.2f, \"scatter_rmw64_alone_us\": %.2f}\n",
               q5, q6);
        const float p7 = timeit([&] { slot_patch<7><<<blocks, 256>>>(sb, ns); }, 20);
        const float p8 = timeit([&] { slot_patch<8><<<blocks, 256>>>(sb, ns); }, 20);
        const float p9 = timeit([&] { slot_patch<9><<<blocks, 256>>>(sb, ns); }, 20);
        printf("{\"probe\": \"slot_line_nt\", \"nt64_in_pass_us\": %.2f, \"nt128_in_pass_us\": %.2f}\n", p8, p9);
        printf("{\"probe\": \"slot_line\", \"line128_in_pass_us\": %.2f, \"read_then_scatter_line128_us\": %.2f, "
               "\"read_then_scatter_64B_us\": %.2f}\n", p7, q3, q4);
        printf("{\"probe\": \"slot_patch\", \"slots\": %u, \"read_only_us\": %.2f, \"u16_pair_us\": %.2f, "
               "\"sector32_us\": %.2f, \"u16_pair_deferred_us\": %.2f, \"u16_pair_nt_us\": %.2f, "
               "\"scatter_u16_alone_us\": %.2f, \"scatter_sector_alone_us\": %.2f, "
               "\"read_then_scatter_kernel_us\": %.2f}\n", ns, p0, p1, p2, p3, p6, q0, q1, q2);
    }
    // write streams of random-looking vs constant data
    const float w0 = timeit([&] { wstream<false><<<blocks, 256>>>(out, big / 16, 0); }, 20);
    printf("{\"probe\": \"write_stream_salt0\", \"bytes\": %llu, \"us\": %.2f}\n", (unsigned long long)big, w0);
    return 0;
}
