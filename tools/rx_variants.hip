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

// bench.py's read-ceiling stream (tools/stream_ceiling.hip) on the same
// buffer: a generic pointer and __builtin_nontemporal_load on it, U loads
// per lane in flight
template <int U>
__global__ __launch_bounds__(256) void plain_ceil(mg::KParams kp) {
    const mg::v4u *p = reinterpret_cast<const mg::v4u *>(kp.buf);
    const uint64_t n16 = kp.buf_len / 16;
    uint32_t acc = 0;
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
        mg::v4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint64_t j = i + (uint64_t)u * 256;
            v[u] = __builtin_nontemporal_load(p + (j < n16 ? j : n16 - 1));
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc = mg::halves4(v[u], acc);
    }
    if (acc == 0x9E3779B9u) kp.out[blockIdx.x].saddr = acc;
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


// Ladder from frame_pattern's walk to the rx kernel's phase 1 (C2 layout:
// frames at a 1536 B stride), one feature at a time.
//   B     packet<->lane interleave (64 = each wave walks 64 consecutive frames)
//   DESC  addresses from the descriptors (load, bpermute, row broadcast);
//         2: the workgroup loads its 8 x 256 B of descriptors per pass
//         together (contiguous pieces, through LDS) instead of 8 x 64 B per wave
//   SUMS  0: per-lane accumulator; 1: row sums -> LDS (lane 15, branch)
//   ST    per-pass stores: 0 none; 1 one dword per 40 B record; 2 one dword
//         per packet into a dense array; 3 whole 40 B records (8 B pieces)
//   DBUF  explicit double buffering of the rounds
template <int B, int DESC, int SUMS, int ST, bool DBUF>
__global__ __launch_bounds__(256) void ladder(mg::KParams kp) {
    using namespace mg;
    __shared__ uint32_t sums[4][64];
    __shared__ uint32_t held[ST == 7 ? 4 : 1][ST == 7 ? 32 : 1][64];
    __shared__ uint32_t rec[ST >= 9 ? 4 : 1][ST == 10 ? 4 * 640 : (ST >= 9 ? 640 : 1)];
    uint32_t pass_i = 0;
    uint32_t keep[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const uint32_t lane = threadIdx.x & 63, row = lane >> 4, rl = lane & 15;
    const uint32_t wib = threadIdx.x >> 6;
    const uint32_t wave = blockIdx.x * 4 + wib, nw = gridDim.x * 4;
    const uint64_t base = (uint64_t)(uintptr_t)kp.buf;
    auto map = [&](uint32_t l) -> uint32_t {
        return B == 64 ? wave * 64 + l : (l / B) * (nw * B) + wave * B + (l % B);
    };
    uint32_t acc = 0;
    for (uint32_t g0 = 0; g0 < kp.n; g0 += nw * 64) {
        uint32_t r_lo = 0, r_hi = 0, r_n = 0;
        const uint32_t k = g0 + map(lane);
        if constexpr (DESC) {
            uint64_t p = base;
            uint32_t nch = 0;
            uint64_t raw = 0;
            if constexpr (DESC == 2 && B == 8) {
                __shared__ uint64_t dsc[4][64];
                const uint32_t j = 2 * wib + (lane >> 5), idx = lane & 31;
                const uint32_t kk = g0 + j * 8 * nw + 32 * blockIdx.x + idx;
                const uint64_t v = kk < kp.n ? *reinterpret_cast<const uint64_t *>(kp.desc + kk) : 0ull;
                __syncthreads();
                dsc[idx >> 3][j * 8 + (idx & 7)] = v;
                __syncthreads();
                raw = dsc[wib][lane];
            } else if (k < kp.n) {
                raw = *reinterpret_cast<const uint64_t *>(kp.desc + k);
            }
            if (k < kp.n) {
                p = base + ((uint64_t)(uint32_t)raw << kp.off_shift);
                const uint32_t L = (uint32_t)(raw >> 32) & 0xFFFFu;
                nch = (uint32_t)((((p + L + 15) & ~15ull) - (p & ~15ull)) >> 4);
            }
            const int src = 4 * (int)rl + (int)row;
            r_n = shfl32(nch, src);
            r_lo = shfl32((uint32_t)p, src);
            r_hi = shfl32((uint32_t)(p >> 32), src);
        }
        auto trip = [&](int i, uint64_t &fb, uint32_t &nj) {
            if constexpr (DESC) {
                nj = row_bcast(r_n, i);
                fb = ((uint64_t)row_bcast(r_hi, i) << 32) | row_bcast(r_lo, i);
            } else {
                const uint32_t f = g0 + map(4 * i + row);
                nj = f < kp.n ? 94 : 0;
                fb = base + (uint64_t)(f < kp.n ? f : 0) * 1536;
            }
        };
        auto issue6 = [&](uint64_t fb, uint32_t nj, v4u (&x)[6]) {
#pragma unroll
            for (int u = 0; u < 6; ++u) {
                const uint32_t c = u * 16 + rl;
                const uint32_t cc = c < nj ? c : (nj ? nj - 1 : 0u);
                x[u] = gload_nt(fb + 16ull * cc);
            }
        };
        auto finish = [&](int i, uint32_t nj, const v4u (&x)[6]) {
            uint32_t a = 0;
#pragma unroll
            for (int u = 0; u < 6; ++u) {
                const uint32_t s4 = halves4(x[u], 0u);
                a += (u * 16 + rl < nj) ? s4 : 0u;
            }
            if constexpr (SUMS == 1) {
                a = row_sum(a);
                if (rl == 15) sums[wib][4 * i + row] = a;
            } else {
                acc += a;
            }
        };
        if constexpr (DBUF) {
            v4u X[6], Y[6];
            uint64_t fb;
            uint32_t nj;
            trip(0, fb, nj);
            issue6(fb, nj, X);
            static_for<0, 16>([&](auto I) {
                constexpr int i = decltype(I)::value;
                v4u(&cb)[6] = (i & 1) ? Y : X;
                v4u(&nb)[6] = (i & 1) ? X : Y;
                uint64_t cfb, nfb;
                uint32_t cnj, nnj;
                trip(i, cfb, cnj);
                if constexpr (i + 1 < 16) {
                    trip(i + 1, nfb, nnj);
                    issue6(nfb, nnj, nb);
                }
                finish(i, cnj, cb);
            });
        } else {
            static_for<0, 16>([&](auto I) {
                constexpr int i = decltype(I)::value;
                uint64_t fb;
                uint32_t nj;
                trip(i, fb, nj);
                v4u x[6];
                issue6(fb, nj, x);
                finish(i, nj, x);
            });
        }
        const uint32_t v = SUMS == 1 ? sums[wib][lane] : acc;
        if (k < kp.n) {
            if constexpr (ST == 1) kp.out[k].saddr = v;
            if constexpr (ST == 2) reinterpret_cast<uint32_t *>(kp.out)[k] = v;
            if constexpr (ST == 3) {
                uint64_t *o = reinterpret_cast<uint64_t *>(kp.out + k);
#pragma unroll
                for (int q = 0; q < 5; ++q) o[q] = (uint64_t)v * (q + 1);
            }
            if constexpr (ST == 4) {      // non-temporal stores
                uint64_t *o = reinterpret_cast<uint64_t *>(kp.out + k);
#pragma unroll
                for (int q = 0; q < 5; ++q) __builtin_nontemporal_store((uint64_t)v * (q + 1), o + q);
            }
            if constexpr (ST == 5) {      // system-scope relaxed stores (sc0 sc1)
                uint64_t *o = reinterpret_cast<uint64_t *>(kp.out + k);
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    __hip_atomic_store(o + q, (uint64_t)v * (q + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            if constexpr (ST == 8) {      // whole records into a per-wave private, L2-resident slot
                uint64_t *o = reinterpret_cast<uint64_t *>(kp.out + (size_t)wave * 64 + lane);
#pragma unroll
                for (int q = 0; q < 5; ++q) o[q] = (uint64_t)v * (q + 1);
            }
            if constexpr (ST == 9 || ST == 10 || ST == 11) {   // record -> LDS (SoA-free: AoS)
                uint32_t *r = &rec[wib][(ST == 10 ? (pass_i & 3) * 640 : 0) + lane * 10];
#pragma unroll
                for (int q = 0; q < 10; ++q) r[q] = v + q;
            }
            if constexpr (ST >= 12) {     // keep the pass's value in a register shift array
#pragma unroll
                for (int q = 7; q > 0; --q) keep[q] = keep[q - 1];
                keep[0] = v;
            }
            if constexpr (ST == 7) {      // keep the dword in LDS; written at kernel end
                held[wib][(g0 / (nw * 64)) & 31][lane] = v;
            }
            if constexpr (ST == 6) {      // agent-scope relaxed stores
                uint64_t *o = reinterpret_cast<uint64_t *>(kp.out + k);
#pragma unroll
                for (int q = 0; q < 5; ++q)
                    __hip_atomic_store(o + q, (uint64_t)v * (q + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
        if constexpr (ST == 9 || ST == 11 || ST == 10) {
            // coalesced flush of the wave's records: runs of B consecutive packets
            const bool flush = ST != 10 || (pass_i & 3) == 3 || g0 + nw * 64 >= kp.n;
            if (flush) {
                const uint32_t npass = ST == 10 ? (pass_i & 3) + 1 : 1;
                for (uint32_t pp = 0; pp < npass; ++pp) {
                    const uint32_t gp = g0 - (npass - 1 - pp) * nw * 64;
                    const uint32_t *r = &rec[wib][(ST == 10 ? pp * 640 : 0)];
                    if constexpr (ST == 11) {
                        // 16 B pieces: 160 per wave-pass, 20 per run of 8 packets
                        for (uint32_t q = lane; q < 160; q += 64) {
                            const uint32_t run = q / 20, w = q % 20;
                            const uint32_t pk = gp + run * (nw * 8) + wave * 8;
                            uint4 val = make_uint4(r[run * 80 + 4 * w], r[run * 80 + 4 * w + 1],
                                                   r[run * 80 + 4 * w + 2], r[run * 80 + 4 * w + 3]);
                            if (pk < kp.n) reinterpret_cast<uint4 *>(kp.out + pk)[w] = val;
                        }
                    } else {
                        for (uint32_t q = lane; q < 320; q += 64) {
                            const uint32_t run = q / 40, w = q % 40;
                            const uint32_t pk = gp + run * (nw * 8) + wave * 8;
                            const uint64_t val = (uint64_t)r[run * 80 + 2 * w] |
                                                 ((uint64_t)r[run * 80 + 2 * w + 1] << 32);
                            if (pk < kp.n) reinterpret_cast<uint64_t *>(kp.out + pk)[w] = val;
                        }
                    }
                }
            }
        }
        ++pass_i;
    }
    if constexpr (ST == 12 || ST == 14) {
        // pass p's value sits in keep[npass - 1 - p]; whole 40 B records
        const uint32_t npass = pass_i < 8 ? pass_i : 8;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if ((uint32_t)q < npass) {
                const uint32_t p = npass - 1 - q;
                const uint32_t k = p * nw * 64 + map(lane);
                if (k < kp.n) {
                    uint64_t *o = reinterpret_cast<uint64_t *>(kp.out + k);
#pragma unroll
                    for (int r = 0; r < 5; ++r) {
                        if constexpr (ST == 14)
                            __builtin_nontemporal_store((uint64_t)keep[q] * (r + 1), o + r);
                        else
                            o[r] = (uint64_t)keep[q] * (r + 1);
                    }
                }
            }
        }
    }
    if constexpr (ST == 13 || ST == 15) {
        // coalesced: the wave's records of one pass through LDS, runs of 8 packets
        const uint32_t npass = pass_i < 8 ? pass_i : 8;
        uint32_t *r = rec[wib];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if ((uint32_t)q < npass) {
                const uint32_t gp = (npass - 1 - q) * nw * 64;
#pragma unroll
                for (int d = 0; d < 10; ++d) r[lane * 10 + d] = keep[q] + d;
                if constexpr (ST == 13) {
                    for (uint32_t qq = lane; qq < 320; qq += 64) {
                        const uint32_t run = qq / 40, w = qq % 40;
                        const uint32_t pk = gp + run * (nw * 8) + wave * 8;
                        const uint64_t val = (uint64_t)r[run * 80 + 2 * w] |
                                             ((uint64_t)r[run * 80 + 2 * w + 1] << 32);
                        if (pk < kp.n) reinterpret_cast<uint64_t *>(kp.out + pk)[w] = val;
                    }
                } else {
                    for (uint32_t qq = lane; qq < 160; qq += 64) {
                        const uint32_t run = qq / 20, w = qq % 20;
                        const uint32_t pk = gp + run * (nw * 8) + wave * 8;
                        const uint4 val = make_uint4(r[run * 80 + 4 * w], r[run * 80 + 4 * w + 1],
                                                     r[run * 80 + 4 * w + 2], r[run * 80 + 4 * w + 3]);
                        if (pk < kp.n) reinterpret_cast<uint4 *>(kp.out + pk)[w] = val;
                    }
                }
            }
        }
    }
    if constexpr (ST == 7) {
        uint32_t pass = 0;
        for (uint32_t g0 = 0; g0 < kp.n && pass < 32; g0 += nw * 64, ++pass) {
            const uint32_t k = g0 + map(lane);
            if (k < kp.n) kp.out[k].saddr = held[wib][pass][lane];
        }
    }
    if (ST == 0 && acc == 0x12345678u) kp.out[0].saddr = acc;
}


// The north star's literal shape (BASELINE.json): one wavefront per packet.
// The wave's 64 lanes stream the frame on the 16 B chunk grid, two loads per
// lane in flight (2 KiB per wave-instruction pair: a 1500 B frame is one
// trip), v_sad_u16 halves, a DPP row reduction and a cross-row readlane
// reduction, then lanes 0..9 store a 40 B record {chunk sum, 0...}: the same
// records as rx_kernel's ABL 1 (phase 1 alone, chunk sums stored), against
// which it is compared byte for byte.  PERSIST: waves loop over packets with
// a capped grid; otherwise one packet per wave and the hardware dispatcher
// fills the GPU (uncapped grid of n/4 workgroups).
template <bool PERSIST>
__global__ __launch_bounds__(256) void wave_per_packet(mg::KParams kp) {
    using namespace mg;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t step = PERSIST ? gridDim.x * 4 : kp.n;
    const uint64_t base = (uint64_t)(uintptr_t)kp.buf;
    for (uint32_t k = wave; k < kp.n; k += step) {
        const uint64_t raw = *reinterpret_cast<const uint64_t *>(kp.desc + k);
        const uint64_t p = base + ((uint64_t)(uint32_t)raw << kp.off_shift);
        const uint32_t L = (uint32_t)(raw >> 32) & 0xFFFFu;
        const uint64_t p16 = p & ~15ull;
        const uint32_t nch = (uint32_t)((((p + L + 15) & ~15ull) - p16) >> 4);
        uint32_t acc = 0;
        for (uint32_t c0 = 0; c0 < nch; c0 += 128) {
            const uint32_t ca = c0 + lane, cb = c0 + 64 + lane;
            const v4u xa = gload_nt(p16 + 16ull * (ca < nch ? ca : nch - 1));
            const v4u xb = gload_nt(p16 + 16ull * (cb < nch ? cb : nch - 1));
            const uint32_t sa = halves4(xa, 0u), sb = halves4(xb, 0u);
            acc += (ca < nch ? sa : 0u) + (cb < nch ? sb : 0u);
        }
        acc = row_sum(acc);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)acc, 15) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 31) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 47) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 63);
        if (lane < 10) reinterpret_cast<uint32_t *>(kp.out + k)[lane] = lane == 0 ? tot : 0u;
    }
}

// Read-only probe of an address-ordered phase 1: per pass, the wave streams
// each of its 8 runs (B = 8 consecutive frames, contiguous in a PSIO chunk)
// as ONE byte range with all 64 lanes (1 KiB per wave-load, U loads in
// flight per lane), in run order, so the grid reads one compact window at a
// time and every 128 B line of a run, small frames' included, exactly once,
// in order.  No per-frame attribution: a ceiling for that schedule.
template <int U, bool SKIP = false>
__global__ __launch_bounds__(256) void run_stream(mg::KParams kp) {
    using namespace mg;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = blockIdx.x * 4 + (threadIdx.x >> 6), nw = gridDim.x * 4;
    const uint64_t base = (uint64_t)(uintptr_t)kp.buf;
    uint32_t acc = 0;
    for (uint32_t g0 = 0; g0 < kp.n; g0 += nw * 64) {
        const uint32_t k = g0 + (lane / 8) * (nw * 8) + wave * 8 + (lane % 8);
        uint64_t lo = 0, hi = 0;
        if (k < kp.n) {
            const uint64_t raw = *reinterpret_cast<const uint64_t *>(kp.desc + k);
            const uint64_t p = base + ((uint64_t)(uint32_t)raw << kp.off_shift);
            const uint32_t L = (uint32_t)(raw >> 32) & 0xFFFFu;
            lo = p & ~15ull;
            hi = (p + L + 15) & ~15ull;
        }
#pragma unroll 1
        for (int j = 0; j < 8; ++j) {
            const uint64_t rlo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(lo >> 32), 8 * j) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lo, 8 * j);
            const uint64_t rhi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(hi >> 32), 8 * j + 7) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hi, 8 * j + 7);
            if (rlo == 0 || rhi <= rlo) continue;
            const uint32_t nc = (uint32_t)((rhi - rlo) >> 4);
            for (uint32_t c0 = 0; c0 < nc; c0 += 64 * U) {
                v4u x[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const uint32_t c = c0 + u * 64 + lane;
                    // SKIP: no load instruction for a window wholly past the run
                    if (!SKIP || c0 + u * 64 < nc) x[u] = gload_nt(rlo + 16ull * (c < nc ? c : nc - 1));
                    else x[u] = v4u{0, 0, 0, 0};
                }
#pragma unroll
                for (int u = 0; u < U; ++u) acc += (c0 + u * 64 + lane < nc) ? halves4(x[u], 0u) : 0u;
            }
        }
    }
    if (acc == 0x12345678u) kp.out[0].saddr = acc;
}

namespace mg {
// Probe (round 4): run_stream's linear walk of each run of 8 consecutive
// frames, staged through an LDS image of the run (unconditional clamped
// loads, so the 12 loads of a run stay in flight), then the per-frame sums
// read back from LDS by 16-lane rows (frames of <= 96 chunks: C2, C3); the
// loads of run j + 1 are in flight while run j is summed.  Timing only: sums
// to out[k].saddr, no parse, no records (compare with abl1_*_nostore).
template <int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void lds_run_walk(mg::KParams kp) {
    __shared__ mg::v4u img[4][U * 64];
    const uint32_t lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const uint32_t row = lane >> 4, rlane = lane & 15;
    const uint32_t wave = blockIdx.x * 4 + wib, nw = gridDim.x * 4;
    const uint64_t base = (uint64_t)(uintptr_t)kp.buf;
    v4u *im = img[wib];
    for (uint32_t g0 = 0; g0 < kp.n; g0 += nw * 64) {
        const uint32_t k = g0 + (lane / 8) * (nw * 8) + wave * 8 + (lane % 8);
        uint64_t lo = 0, hi = 0;
        uint32_t nch = 0;
        if (k < kp.n) {
            const uint64_t raw = *reinterpret_cast<const uint64_t *>(kp.desc + k);
            const uint64_t p = base + ((uint64_t)(uint32_t)raw << kp.off_shift);
            const uint32_t L = (uint32_t)(raw >> 32) & 0xFFFFu;
            lo = p & ~15ull;
            hi = (p + L + 15) & ~15ull;
            nch = L ? (uint32_t)((hi - lo) >> 4) : 0u;
        }
        auto run_lo = [&](int j) -> uint64_t {
            return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(lo >> 32), 8 * j) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lo, 8 * j);
        };
        auto run_nc = [&](int j) -> uint32_t {
            const uint64_t rlo = run_lo(j);
            const uint64_t rhi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(hi >> 32), 8 * j + 7) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hi, 8 * j + 7);
            return rlo == 0 || rhi <= rlo ? 0u : (uint32_t)((rhi - rlo) >> 4);
        };
        v4u x[U];
        auto issue = [&](int j) {
            const uint64_t rlo = run_lo(j);
            const uint32_t nc = run_nc(j);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = u * 64 + lane;
                x[u] = gload_nt(rlo + 16ull * (c < nc ? c : (nc ? nc - 1 : 0u)));   // clamp: no exec mask
            }
        };
        issue(0);
#pragma unroll 1
        for (int j = 0; j < 8; ++j) {
            const uint32_t nc = run_nc(j);
            const uint64_t rlo = run_lo(j);
#pragma unroll
            for (int u = 0; u < U; ++u)
                im[u * 64 + lane] = x[u];
            __builtin_amdgcn_wave_barrier();
            if (j + 1 < 8) issue(j + 1);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int src = 8 * j + 4 * h + (int)row;
                const uint32_t f_n = shfl32(nch, src);
                const uint32_t f_lo = shfl32((uint32_t)lo, src);
                const uint32_t s = (f_lo - (uint32_t)rlo) >> 4;
                uint32_t acc = 0;
                v4u y[6];
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    const uint32_t c = u * 16 + rlane;
                    y[u] = im[(s + (c < f_n ? c : 0u)) & (U * 64 - 1 > 0 ? 0xFFFFFFFFu : 0u)];
                }
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    const uint32_t c = u * 16 + rlane;
                    const uint32_t v = halves4(y[u], 0u);
                    acc += c < f_n ? v : 0u;
                }
                acc = row_sum(acc);
                const uint32_t kk = g0 + j * (nw * 8) + wave * 8 + 4 * h + row;
                if (rlane == 15 && kk < kp.n) kp.out[kk].saddr = acc;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}
// Probe (round 4): the same run walk with the run image filled by LDS-DMA
// (global_load_lds_dwordx4: each wave-instruction lands 1 KiB straight in
// LDS, no VGPR -> LDS write pass), then per-frame sums from LDS.  Timing
// only, like lds_run_walk.
template <int U>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void lds_dma_walk(mg::KParams kp) {
    __shared__ v4u img[4][U * 64];
    const uint32_t lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const uint32_t row = lane >> 4, rlane = lane & 15;
    const uint32_t wave = blockIdx.x * 4 + wib, nw = gridDim.x * 4;
    const uint64_t base = (uint64_t)(uintptr_t)kp.buf;
    v4u *im = img[wib];
    for (uint32_t g0 = 0; g0 < kp.n; g0 += nw * 64) {
        const uint32_t k = g0 + (lane / 8) * (nw * 8) + wave * 8 + (lane % 8);
        uint64_t lo = 0, hi = 0;
        uint32_t nch = 0;
        if (k < kp.n) {
            const uint64_t raw = *reinterpret_cast<const uint64_t *>(kp.desc + k);
            const uint64_t p = base + ((uint64_t)(uint32_t)raw << kp.off_shift);
            const uint32_t L = (uint32_t)(raw >> 32) & 0xFFFFu;
            lo = p & ~15ull;
            hi = (p + L + 15) & ~15ull;
            nch = L ? (uint32_t)((hi - lo) >> 4) : 0u;
        }
#pragma unroll 1
        for (int j = 0; j < 8; ++j) {
            const uint64_t rlo = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(lo >> 32), 8 * j) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)lo, 8 * j);
            const uint64_t rhi = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(hi >> 32), 8 * j + 7) << 32) |
                                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)hi, 8 * j + 7);
            const uint32_t nc = rlo == 0 || rhi <= rlo ? 0u : (uint32_t)((rhi - rlo) >> 4);
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const uint32_t c = u * 64 + lane;
                const uint32_t cc = c < nc ? c : (nc ? nc - 1 : 0u);
                __builtin_amdgcn_global_load_lds(reinterpret_cast<const void *>(rlo + 16ull * cc),
                                                 (__attribute__((address_space(3))) void *)(im + u * 64),
                                                 16, 0, 0);
            }
            __builtin_amdgcn_s_waitcnt(0);   // (coarse: every counter)
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int src = 8 * j + 4 * h + (int)row;
                const uint32_t f_n = shfl32(nch, src);
                const uint32_t f_lo = shfl32((uint32_t)lo, src);
                const uint32_t s = (f_lo - (uint32_t)rlo) >> 4;
                uint32_t acc = 0;
                v4u y[6];
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    const uint32_t c = u * 16 + rlane;
                    y[u] = im[s + (c < f_n ? c : 0u)];
                }
#pragma unroll
                for (int u = 0; u < 6; ++u) {
                    const uint32_t c = u * 16 + rlane;
                    const uint32_t v = halves4(y[u], 0u);
                    acc += c < f_n ? v : 0u;
                }
                acc = row_sum(acc);
                const uint32_t kk = g0 + j * (nw * 8) + wave * 8 + 4 * h + row;
                if (rlane == 15 && kk < kp.n) kp.out[kk].saddr = acc;
            }
            __builtin_amdgcn_s_waitcnt(0);
            __builtin_amdgcn_wave_barrier();
        }
    }
}
}  // namespace mg

struct Variant { const char *name; kfn fn; uint32_t blocks_per_cu; uint32_t wpb = 4; };

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
    if (getenv("RXV_N")) n = (uint32_t)atoi(getenv("RXV_N"));   // e.g. one io_module aggregate (4096)

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
    // the same frames as a pointer burst (DPDK-style): ptrs[i] = buf + offset
    {
        std::vector<uint64_t> hp(n);
        std::vector<uint16_t> hl(n);
        for (uint32_t i = 0; i < n; ++i) {
            hp[i] = (uint64_t)(uintptr_t)d_buf + ((uint64_t)desc[i].offset << 6);
            hl[i] = desc[i].len;
        }
        uint64_t *dp;
        uint16_t *dl;
        CK(hipMalloc(&dp, n * 8));
        CK(hipMalloc(&dl, n * 2));
        CK(hipMemcpy(dp, hp.data(), n * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dl, hl.data(), n * 2, hipMemcpyHostToDevice));
        kp.ptrs = reinterpret_cast<const uint8_t *const *>(dp);
        kp.lens = dl;
    }

    if (argc > 3 && !strcmp(argv[3], "stampsab")) {
        // The end-time classes (old / young workgroup on a CU, XCC) of several
        // phase-1 layouts of the C2 kernel, and their launch times, one process.
        using namespace mg;
        struct SV { const char *name; kfn fn; };
        const SV svs_c2[] = {
            {"B8", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, true>},
            {"B8_prio1half", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, true, 5>},
        };
        const SV svs_c3[] = {
            {"sorted6", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, true>},
            {"sorted6_prio1half", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, true, 5>},
            {"sorted6_prio2half", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, true, 6>},
        };
        const SV svs_c5[] = {
            {"lalign_rev", rx_kernel<kRxChunk, false, 3, true, 0, 8, 8, true, 6, true, true>},
            {"lalign_rev_prio1half", rx_kernel<kRxChunk, false, 3, true, 0, 8, 8, true, 6, true, true, 5>},
        };
        const SV *svs = rss ? svs_c3 : !strcmp(cfg, "c5") ? svs_c5 : svs_c2;
        const size_t nsv = rss ? 3 : 2;
        const uint32_t groups = (n + 63) / 64;
        const uint32_t blocks = std::min<uint32_t>((groups + 3) / 4, cus * 2), waves = blocks * 4;
        uint32_t *d_st;
        CK(hipMalloc(&d_st, waves * 16));
        kp.stamps = d_st;
        kp.out = d_out;
        std::vector<uint32_t> st(waves * 4);
        std::vector<mtcp_gpu_result> ref(n), got(n);
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int r = 0; r < rounds; ++r) {
            for (size_t v = 0; v < nsv; ++v) {
                for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(svs[v].fn, dim3(blocks), dim3(256), 0, 0, kp);
                CK(hipEventRecord(e0));
                for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(svs[v].fn, dim3(blocks), dim3(256), 0, 0, kp);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                CK(hipMemcpy(st.data(), d_st, waves * 16, hipMemcpyDeviceToHost));
                CK(hipMemcpy(got.data(), d_out, n * sizeof(mtcp_gpu_result), hipMemcpyDeviceToHost));
                if (v == 0) ref = got;
                else if (memcmp(ref.data(), got.data(), n * sizeof(mtcp_gpu_result))) {
                    fprintf(stderr, "%s records differ from %s's\n", svs[v].name, svs[0].name);
                    return 2;
                }
                uint32_t t0 = 0xFFFFFFFFu;
                for (uint32_t w = 0; w < waves; ++w) t0 = std::min(t0, st[4 * w]);
                double cls[2][8] = {{0}}; int cn[2][8] = {{0}}; double mx = 0, sum = 0;
                for (uint32_t w = 0; w < waves; ++w) {
                    const double e = (st[4 * w + 1] - t0) * 0.01;
                    const int y = (w / 4) >= blocks / 2, x = st[4 * w + 2] & 7;
                    cls[y][x] += e; cn[y][x]++; mx = std::max(mx, e); sum += e;
                }
                printf("{\"round\": %d, \"variant\": \"%s\", \"launch_us\": %.2f, \"end_mean\": %.2f, \"end_max\": %.2f, \"old_by_xcc\": [",
                       r, svs[v].name, ms * 1e3 / 20, sum / waves, mx);
                for (int x = 0; x < 8; ++x) printf("%s%.1f", x ? ", " : "", cn[0][x] ? cls[0][x] / cn[0][x] : 0.0);
                printf("], \"young_by_xcc\": [");
                for (int x = 0; x < 8; ++x) printf("%s%.1f", x ? ", " : "", cn[1][x] ? cls[1][x] / cn[1][x] : 0.0);
                printf("]}\n");
            }
        }
        return 0;
    }
    if (argc > 3 && !strcmp(argv[3], "stamps")) {
        // Per-wave start/end of the dispatched kernel (rx_kernel STAMP): is the
        // end-time spread systematic (by XCD, SE, CU, wave slot) or random?
        using namespace mg;
        const int prio = argc > 4 ? atoi(argv[4]) : 0;
        kfn fn = rss ? (prio ? (kfn)rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, true, 1>
                             : (kfn)rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, true>)
                     : !strcmp(cfg, "c5") ? (kfn)rx_kernel<kRxChunk, false, 3, true, 0, 8, 8, true, 6, true, true>
                     : prio ? (kfn)rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, true, 1>
                            : (kfn)rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, true>;
        const uint32_t groups = (n + 63) / 64;
        uint32_t blocks = std::min<uint32_t>((groups + 3) / 4, cus * 2);
        const uint32_t waves = blocks * 4;
        uint32_t *d_st;
        CK(hipMalloc(&d_st, waves * 16));
        kp.stamps = d_st;
        kp.out = d_out;
        std::vector<uint32_t> st(waves * 4);
        for (int r = 0; r < rounds; ++r) {
            for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(fn, dim3(blocks), dim3(256), 0, 0, kp);
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(st.data(), d_st, waves * 16, hipMemcpyDeviceToHost));
            uint32_t t0 = 0xFFFFFFFFu;
            for (uint32_t w = 0; w < waves; ++w) t0 = std::min(t0, st[4 * w]);
            // one line per wave of the last round only; a summary per round
            std::vector<double> ends(waves);
            double xe[16] = {0}; int xn[16] = {0};
            for (uint32_t w = 0; w < waves; ++w) {
                ends[w] = (st[4 * w + 1] - t0) * 0.01;    // us (100 MHz)
                const uint32_t x = st[4 * w + 2] & 15;
                xe[x] += ends[w]; xn[x]++;
                if (r == rounds - 1)
                    printf("{\"wave\": %u, \"start_us\": %.2f, \"end_us\": %.2f, \"xcc\": %u, \"hw_id\": %u}\n",
                           w, (st[4 * w] - t0) * 0.01, ends[w], x, st[4 * w + 3]);
            }
            std::vector<double> e = ends;
            std::sort(e.begin(), e.end());
            printf("{\"round\": %d, \"end_p0\": %.2f, \"end_p10\": %.2f, \"end_p50\": %.2f, \"end_p90\": %.2f, \"end_p100\": %.2f, \"xcc_mean_end\": [",
                   r, e[0], e[waves / 10], e[waves / 2], e[waves * 9 / 10], e[waves - 1]);
            for (int x = 0; x < 8; ++x) printf("%s%.2f", x ? ", " : "", xn[x] ? xe[x] / xn[x] : 0.0);
            printf("]}\n");
        }
        return 0;
    }
    std::vector<Variant> vs;
    using namespace mg;
    if (rss) {
        // variant 0 = what mtcp_gpu.hip dispatches for C3 (sorted, runs of 16);
        // every other variant's records must equal its records byte for byte
        vs.push_back({"b16_rss_sorted6_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 16>, 2});
        // the read ceiling's shapes on this buffer (tools/stream_ceiling.hip)
        vs.push_back({"plain_ceil3_cu2", plain_ceil<3>, 2});
        vs.push_back({"plain_ceil4_cu2", plain_ceil<4>, 2});
        vs.push_back({"plain_ceil6_cu2", plain_ceil<6>, 2});
        vs.push_back({"plain_ceil8_cu4", plain_ceil<8>, 4});
        // the ladder of the shipped schedule: phase 1 alone, + records
        vs.push_back({"abl1_b16_rss_sorted6_nostore_cu2", rx_kernel<kRxChunk, true, 6, false, 1, 0, 16>, 2});
        vs.push_back({"abl1_b16_rss_sorted6_cu2", rx_kernel<kRxChunk, true, 6, false, 1, 8, 16>, 2});
        // round 5: phase 1 without its LDS header / tail copies (every
        // bank-conflicting ds_write of the size-sorted rounds): the most those
        // copies, and so their conflicts, can cost (records wrong)
        vs.push_back({"abl2_b16_rss_sorted6_nostore_cu2", rx_kernel<kRxChunk, true, 6, false, 2, 0, 16>, 2});
        vs.push_back({"abl3_b16_rss_sorted6_nostore_cu2", rx_kernel<kRxChunk, true, 6, false, 3, 0, 16>, 2});
        vs.push_back({"rss_sorted6_cu2", rx_kernel<kRxChunk, true, 6>, 2});
        vs.push_back({"b16_rss_sorted6_cmp_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 16, true, 6, false, false, 0, 4, 0, true>, 2});
        vs.push_back({"ldsrun12_cu2", lds_run_walk<12>, 2});
        vs.push_back({"ldsdma12_cu2", lds_dma_walk<12>, 2});
        vs.push_back({"rss_sorted6_wpb8_cu1", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, false, 0, 8>, 1, 8});
        vs.push_back({"rss_sorted6_wpb2_cu4", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, false, 0, 2>, 4, 2});
        vs.push_back({"rss_sorted6_prio1half_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, false, 5>, 2});
        vs.push_back({"rss_sorted6_prio2half_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, false, 6>, 2});
        vs.push_back({"rss_sorted6_prio1_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, false, 1>, 2});
        vs.push_back({"rss_sorted6_prio2_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, false, 2>, 2});
        vs.push_back({"rss_sorted6_prio3_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 6, false, false, 3>, 2});
        vs.push_back({"rss_sorted6_fullgrid", rx_kernel<kRxChunk, true, 6>, 1u << 20});
        vs.push_back({"rss_sorted6_cu4", rx_kernel<kRxChunk, true, 6>, 4});
        vs.push_back({"rss_sorted6_cu8", rx_kernel<kRxChunk, true, 6>, 8});
        vs.push_back({"ptrs_rss_unrolled_lalign_cu2", rx_kernel<kRxPtrs, true, 3, true>, 2});
        vs.push_back({"ptrs_rss_sorted6_lalign_cu2", rx_kernel<kRxPtrs, true, 6, true>, 2});
        vs.push_back({"rss_rolled_cu2", rx_kernel<kRxChunk, true, 0>, 2});
        vs.push_back({"rss_unrolled_cu2", rx_kernel<kRxChunk, true, 3>, 2});
        vs.push_back({"rss_sorted_cu2", rx_kernel<kRxChunk, true, 4>, 2});
        vs.push_back({"rss_sorted5_cu2", rx_kernel<kRxChunk, true, 5>, 2});
        vs.push_back({"rss_sorted6_cu3", rx_kernel<kRxChunk, true, 6>, 3});
        vs.push_back({"rss_sorted6_defer0_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 0>, 2});
        vs.push_back({"rss_sorted6_defer1_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 1>, 2});
        vs.push_back({"rss_sorted6_defer2_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 2>, 2});
        vs.push_back({"rss_sorted6_defer4_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 4>, 2});
        vs.push_back({"abl1_rss_sorted6_cu2", rx_kernel<kRxChunk, true, 6, false, 1>, 2});
        vs.push_back({"abl2_rss_sorted6_cu2", rx_kernel<kRxChunk, true, 6, false, 2>, 2});
        vs.push_back({"abl1_rss_sorted6_nostore_cu2", rx_kernel<kRxChunk, true, 6, false, 1, 0>, 2});
        vs.push_back({"wpp_fullgrid", wave_per_packet<false>, 1u << 20});
        vs.push_back({"wpp_persist_cu2", wave_per_packet<true>, 2});
        vs.push_back({"wpp_persist_cu8", wave_per_packet<true>, 8});
        vs.push_back({"norss_sorted6_cu2", rx_kernel<kRxChunk, false, 6>, 2});
        vs.push_back({"plain_stream_nt_cu2", plain_stream_nt, 2});
        vs.push_back({"runstream4_cu2", run_stream<4>, 2});
        vs.push_back({"runstream8_cu2", run_stream<8>, 2});
        vs.push_back({"runstream12_cu2", run_stream<12>, 2});
        vs.push_back({"runstream16_cu2", run_stream<16>, 2});
        vs.push_back({"runstream12skip_cu2", run_stream<12, true>, 2});
        vs.push_back({"runstream16skip_cu2", run_stream<16, true>, 2});
        vs.push_back({"runstream24skip_cu2", run_stream<24, true>, 2});

        vs.push_back({"b32_rss_sorted6_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 32>, 2});
        vs.push_back({"abl1_rss_sorted6_nostore_u8_cu2", rx_kernel<kRxChunk, true, 6, false, 1, 0, 8, true, 8>, 2});
        vs.push_back({"rss_sorted6_u8_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 8, 8, true, 8>, 2});
        vs.push_back({"rss_sorted6_u8_defer4_cu2", rx_kernel<kRxChunk, true, 6, false, 0, 4, 8, true, 8>, 2});
    } else {
        // variant 0 = what mtcp_gpu.hip dispatches for C2 (C5 adds LALIGN)
        vs.push_back({"unrolled_cu2", rx_kernel<kRxChunk, false, 3>, 2});
        vs.push_back({"unrolled_wpb8_cu1", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 0, 8>, 1, 8});
        vs.push_back({"unrolled_wpb2_cu4", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 0, 2>, 4, 2});
        vs.push_back({"unrolled_lalign_rev_wpb8_cu1", rx_kernel<kRxChunk, false, 3, true, 0, 8, 8, true, 6, true, false, 0, 8>, 1, 8});
        vs.push_back({"unrolled_prio1half_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 5>, 2});
        // XCD balance probe (records wrong: compared with nothing): odd / even
        // XCD waves leave their last 8 / 16 / 24 frames of the last pass unread
        vs.push_back({"abl_xskip_odd8_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 5, 4, 8>, 2});
        vs.push_back({"abl_xskip_odd16_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 5, 4, 16>, 2});
        vs.push_back({"abl_xskip_odd24_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 5, 4, 24>, 2});
        vs.push_back({"abl_xskip_even16_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 5, 4, -16>, 2});
        vs.push_back({"unrolled_prio2half_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 6>, 2});
        vs.push_back({"unrolled_lalign_rev_prio1half_cu2", rx_kernel<kRxChunk, false, 3, true, 0, 8, 8, true, 6, true, false, 5>, 2});
        vs.push_back({"unrolled_prio1_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 1>, 2});
        vs.push_back({"unrolled_prio2_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 2>, 2});
        vs.push_back({"unrolled_prio3_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 3>, 2});
        vs.push_back({"unrolled_lalign_rev_prio1_cu2", rx_kernel<kRxChunk, false, 3, true, 0, 8, 8, true, 6, true, false, 1>, 2});
        vs.push_back({"unrolled_fullgrid", rx_kernel<kRxChunk, false, 3>, 1u << 20});
        vs.push_back({"unrolled_cu4", rx_kernel<kRxChunk, false, 3>, 4});
        vs.push_back({"unrolled_cu8", rx_kernel<kRxChunk, false, 3>, 8});
        vs.push_back({"unrolled_lalign_rev_fullgrid", rx_kernel<kRxChunk, false, 3, true, 0, 8, 8, true, 6, true>, 1u << 20});
        vs.push_back({"unrolled_lalign_cu2", rx_kernel<kRxChunk, false, 3, true>, 2});
        vs.push_back({"unrolled_lalign_rev_cu2", rx_kernel<kRxChunk, false, 3, true, 0, 8, 8, true, 6, true>, 2});
        vs.push_back({"ptrs_unrolled_lalign_cu2", rx_kernel<kRxPtrs, false, 3, true>, 2});
        vs.push_back({"ptrs_sorted6_lalign_cu2", rx_kernel<kRxPtrs, false, 6, true>, 2});
        vs.push_back({"rolled_cu2", rx_kernel<kRxChunk, false, 0>, 2});
        vs.push_back({"rolled_lalign_cu2", rx_kernel<kRxChunk, false, 0, true>, 2});
        vs.push_back({"unrolled_cu3", rx_kernel<kRxChunk, false, 3>, 3});
        vs.push_back({"unrolled_defer0_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 0>, 2});
        vs.push_back({"unrolled_defer4_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 4>, 2});
        vs.push_back({"sorted_cu2", rx_kernel<kRxChunk, false, 4>, 2});
        vs.push_back({"sorted6_cu2", rx_kernel<kRxChunk, false, 6>, 2});
        vs.push_back({"abl1_unrolled_nostore_cu2", rx_kernel<kRxChunk, false, 3, false, 1, 0>, 2});
        vs.push_back({"abl1_unrolled_cu2", rx_kernel<kRxChunk, false, 3, false, 1>, 2});
        vs.push_back({"abl2_unrolled_cu2", rx_kernel<kRxChunk, false, 3, false, 2>, 2});
        vs.push_back({"abl3_unrolled_cu2", rx_kernel<kRxChunk, false, 3, false, 3>, 2});
        vs.push_back({"wpp_fullgrid", wave_per_packet<false>, 1u << 20});
        vs.push_back({"wpp_persist_cu2", wave_per_packet<true>, 2});
        vs.push_back({"wpp_persist_cu8", wave_per_packet<true>, 8});
        if (strcmp(cfg, "c2") == 0) {
            vs.push_back({"lad_B8_desc", ladder<8, true, 0, 0, false>, 2});
            vs.push_back({"lad_B8_nodesc", ladder<8, false, 0, 0, false>, 2});
            vs.push_back({"lad_B8_descwg", ladder<8, 2, 0, 0, false>, 2});
            vs.push_back({"lad_B8_descwg_sums", ladder<8, 2, 1, 0, false>, 2});
            vs.push_back({"lad_B8_nodesc_dbuf", ladder<8, false, 0, 0, true>, 2});
            vs.push_back({"lad_B8_desc_dbuf", ladder<8, true, 0, 0, true>, 2});
            vs.push_back({"lad_B64_nodesc", ladder<64, false, 0, 0, false>, 2});
            vs.push_back({"lad_B8_nodesc_cu1", ladder<8, false, 0, 0, false>, 1});
            vs.push_back({"lad_B8_nodesc_cu3", ladder<8, false, 0, 0, false>, 3});
            vs.push_back({"lad_B8_desc_st2", ladder<8, true, 0, 2, false>, 2});
            vs.push_back({"lad_B8_desc_st3", ladder<8, true, 0, 3, false>, 2});
            vs.push_back({"lad_B8_desc_st4_nt", ladder<8, true, 0, 4, false>, 2});
            vs.push_back({"lad_B8_desc_st5_sys", ladder<8, true, 0, 5, false>, 2});
            vs.push_back({"lad_B8_desc_st11_coal16_perpass", ladder<8, true, 0, 11, false>, 2});
            vs.push_back({"lad_B8_desc_st12_regs_atend", ladder<8, true, 0, 12, false>, 2});
            vs.push_back({"lad_B8_desc_st15_regs_coal16", ladder<8, true, 0, 15, false>, 2});
        }
        vs.push_back({"plain_stream_nt_cu2", plain_stream_nt, 2});
        vs.push_back({"plain_ceil4_cu2", plain_ceil<4>, 2});
        vs.push_back({"plain_ceil8_cu2", plain_ceil<8>, 2});
        vs.push_back({"plain_ceil4_cu4", plain_ceil<4>, 4});
        vs.push_back({"plain_ceil2_cu2", plain_ceil<2>, 2});
        vs.push_back({"plain_ceil3_cu2", plain_ceil<3>, 2});
        vs.push_back({"plain_ceil6_cu2", plain_ceil<6>, 2});
        vs.push_back({"plain_ceil4_cu1", plain_ceil<4>, 1});
        vs.push_back({"plain_ceil6_cu1", plain_ceil<6>, 1});
        vs.push_back({"plain_ceil8_cu1", plain_ceil<8>, 1});
        vs.push_back({"plain_ceil4_cu3", plain_ceil<4>, 3});
        vs.push_back({"plain_ceil2_cu4", plain_ceil<2>, 4});
        // waves per CU for the shipped C2 schedule: 6 (3 x 2, 2 x 3) and 4 (2 x 2)
        vs.push_back({"wv_unrolled_wpb3_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 0, 3>, 2, 3});
        vs.push_back({"wv_unrolled_wpb2_cu3", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 0, 2>, 3, 2});
        vs.push_back({"wv_unrolled_wpb2_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 0, 2>, 2, 2});
        vs.push_back({"wv_abl1_nostore_wpb3_cu2", rx_kernel<kRxChunk, false, 3, false, 1, 0, 8, true, 6, false, false, 0, 3>, 2, 3});
        vs.push_back({"nocoop_unrolled_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 6, false, false, 0, 4, 0, false, 2, false>, 2});
        vs.push_back({"b16_unrolled_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 16>, 2});
        vs.push_back({"b32_unrolled_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 32>, 2});
        vs.push_back({"abl2_nostore_cu2", rx_kernel<kRxChunk, false, 3, false, 2, 0>, 2});
        vs.push_back({"abl3_nostore_cu2", rx_kernel<kRxChunk, false, 3, false, 3, 0>, 2});
        vs.push_back({"nocoop_abl1_nostore_cu2", rx_kernel<kRxChunk, false, 3, false, 1, 0, 8, true, 6, false, false, 0, 4, 0, false, 2, false>, 2});
        vs.push_back({"u3_unrolled_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 3>, 2});
        vs.push_back({"u4_unrolled_cu2", rx_kernel<kRxChunk, false, 3, false, 0, 8, 8, true, 4>, 2});
        vs.push_back({"u3_abl1_nostore_cu2", rx_kernel<kRxChunk, false, 3, false, 1, 0, 8, true, 3>, 2});
        vs.push_back({"u4_abl1_nostore_cu2", rx_kernel<kRxChunk, false, 3, false, 1, 0, 8, true, 4>, 2});
        vs.push_back({"wv_abl1_nostore_wpb2_cu2", rx_kernel<kRxChunk, false, 3, false, 1, 0, 8, true, 6, false, false, 0, 2>, 2, 2});
        vs.push_back({"runstream4_cu2", run_stream<4>, 2});
        vs.push_back({"runstream8_cu2", run_stream<8>, 2});
        vs.push_back({"runstream12_cu2", run_stream<12>, 2});
        vs.push_back({"ldsrun12_cu2", lds_run_walk<12>, 2});
        vs.push_back({"ldsdma12_cu2", lds_dma_walk<12>, 2});
        // tx fill last: it repairs the corrupted frames the rx variants compare on
        vs.push_back({"tx_unrolled_cu2", rx_kernel<kTxChunk, false, 3>, 2});
        vs.push_back({"tx_unrolled_nodefer_cu2", rx_kernel<kTxChunk, false, 3, false, 0, 0>, 2});
        vs.push_back({"tx_unrolled_nodefer_temporal_cu2", rx_kernel<kTxChunk, false, 3, false, 0, 0, 8, false>, 2});
        vs.push_back({"tx_unrolled_temporal_cu2", rx_kernel<kTxChunk, false, 3, false, 0, 8, 8, false>, 2});
    }
    if (single) vs.resize(1);
    if (const char *only = getenv("RXV_ONLY")) {     // variant 0 and the named ones
        std::vector<Variant> keep{vs[0]};
        for (size_t v = 1; v < vs.size(); ++v)
            if (strstr(only, vs[v].name)) keep.push_back(vs[v]);
        vs = keep;
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    std::vector<std::vector<float>> ms(vs.size());
    // the ABL 1 records (chunk sums), which the one-wave-per-packet variants must equal
    std::vector<mtcp_gpu_result> abl1_rec;
    std::vector<uint8_t> cmp_rec;                   // the first compact variant's 16 B records
    const int reps = 20;
    for (int r = 0; r < rounds; ++r) {
        for (size_t v = 0; v < vs.size(); ++v) {
            const uint32_t groups = (n + 63) / 64, wpb = vs[v].wpb;
            uint32_t blocks = strstr(vs[v].name, "plain") ? 1u << 20
                              : strstr(vs[v].name, "wpp") ? (n + 3) / 4 : (groups + wpb - 1) / wpb;
            if (blocks > cus * vs[v].blocks_per_cu) blocks = cus * vs[v].blocks_per_cu;
            kp.out = v == 0 ? d_ref : d_out;
            CK(hipMemset(kp.out, 0, n * sizeof(mtcp_gpu_result)));
            const uint32_t threads = 64 * wpb;
            hipLaunchKernelGGL(vs[v].fn, dim3(blocks), dim3(threads), 0, 0, kp);
            CK(hipEventRecord(a));
            for (int i = 0; i < reps; ++i)
                hipLaunchKernelGGL(vs[v].fn, dim3(blocks), dim3(threads), 0, 0, kp);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float t;
            CK(hipEventElapsedTime(&t, a, b));
            ms[v].push_back(t / reps);
            if (r == 0 && (!strcmp(vs[v].name, "abl1_unrolled_cu2") || !strcmp(vs[v].name, "abl1_rss_sorted6_cu2"))) {
                abl1_rec.resize(n);
                CK(hipMemcpy(abl1_rec.data(), d_out, n * sizeof(mtcp_gpu_result), hipMemcpyDeviceToHost));
            }
            if (r == 0 && strstr(vs[v].name, "wpp")) {
                std::vector<mtcp_gpu_result> y(n);
                CK(hipMemcpy(y.data(), d_out, n * sizeof(mtcp_gpu_result), hipMemcpyDeviceToHost));
                if (abl1_rec.size() != n || memcmp(abl1_rec.data(), y.data(), n * sizeof(mtcp_gpu_result)) != 0) {
                    fprintf(stderr, "variant %s differs from the ABL 1 chunk sums\n", vs[v].name);
                    return 2;
                }
            }
            // compact-record (CMP) variants: 16 B records, compared among themselves
            if (r == 0 && strstr(vs[v].name, "_cmp")) {
                std::vector<uint8_t> y(n * 16);
                CK(hipMemcpy(y.data(), d_out, n * 16, hipMemcpyDeviceToHost));
                if (cmp_rec.empty()) cmp_rec = y;
                else if (memcmp(cmp_rec.data(), y.data(), n * 16) != 0) {
                    fprintf(stderr, "variant %s differs from the first compact variant\n", vs[v].name);
                    return 2;
                }
            }
            if (v > 0 && r == 0 && !strstr(vs[v].name, "abl") && !strstr(vs[v].name, "wpp") && !strstr(vs[v].name, "norss") && strncmp(vs[v].name, "tx_", 3) != 0 && !strstr(vs[v].name, "plain") && !strstr(vs[v].name, "lad") && !strstr(vs[v].name, "runstream") && !strstr(vs[v].name, "ldsrun") && !strstr(vs[v].name, "ldsdma") && !strstr(vs[v].name, "_cmp")) {
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
