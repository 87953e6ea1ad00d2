// flow_kernels.hpp — gfx950 kernels for the two rows SURVEY §8(f) puts next
// to the rx path:
//
//   f3  HashFlow (mtcp/src/tcp_stream.c:56-90) of the stream key every TCP_OK
//       packet is looked up with (mtcp/src/tcp_in.c:1180-1186);
//   f4  the RSS-friendly source-address search of CreateAddressPoolPerCore
//       (mtcp/src/addr_pool.c:103-180): GetRSSCPUCore (mtcp/src/rss.c:90-103)
//       over every (address, port) candidate, then an order-preserving
//       compaction of the candidates that land on one core's queue.
//
// Both are small integer kernels: flow_hash reads 16 B of each 40 B result
// record and writes 4 B (HBM-bound, like rx); the pool search is a Toeplitz
// hash per candidate through the same LDS nibble tables as rx, then a
// count / scan / emit compaction that keeps the reference's order.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtcp_gpu.h"
#include "rx_kernels.hpp"

namespace mg {

constexpr uint32_t kPorts = MTCP_GPU_MAX_PORT - MTCP_GPU_MIN_PORT;   // 64511
constexpr int kPoolPerThread = 16;                                   // candidates per lane
constexpr int kPoolTile = kBlock * kPoolPerThread;                   // per workgroup

// One lane per result record: saddr @0, daddr @4, sport|dport @8, verdict @36.
__global__ __launch_bounds__(kBlock) void flow_hash_kernel(const mtcp_gpu_result *__restrict__ res,
                                                           uint32_t n, uint32_t *__restrict__ bins) {
    const uint32_t stride = gridDim.x * kBlock;
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
        const uint32_t *r = reinterpret_cast<const uint32_t *>(res + i);
        const uint32_t saddr = r[0], daddr = r[1], ports = r[2];
        bins[i] = flow_bin(saddr, daddr, ports, r[9] & 0xFFu);   // rx_kernels.hpp
    }
}

// GetRSSHash (mtcp/src/rss.c:44-82) of host-order (sip, dip, sp, dp) through
// the 24 nibble tables: nibble t of the 96-bit input sip|dip|sp|dp, most
// significant first, selects tables[t][nibble].
__device__ __forceinline__ uint32_t toeplitz96(const uint32_t *tab, uint32_t sip, uint32_t dip,
                                               uint32_t ports) {
    uint32_t h = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        h ^= tab[(t << 4) | ((sip >> (28 - 4 * t)) & 15u)];
        h ^= tab[((8 + t) << 4) | ((dip >> (28 - 4 * t)) & 15u)];
        h ^= tab[((16 + t) << 4) | ((ports >> (28 - 4 * t)) & 15u)];
    }
    return h;
}

struct PoolParams {
    const uint32_t *rss_tables;
    uint32_t saddr_base_h;   // candidate i's address: saddr_base_h + i
    uint32_t daddr_h;
    uint32_t dport_h;
    uint32_t nq;
    uint32_t endian;
    uint64_t total;          // num_addr * kPorts candidates
};

// queue[g] for candidate g = i * kPorts + (port - MIN_PORT).  The reference
// calls GetRSSCPUCore(daddr_h, saddr_h, dport_h, sport_h, ...)
// (addr_pool.c:164): the peer's side comes first, as the incoming packets
// of the connection will carry it.
//
// The Toeplitz hash is linear over GF(2) (each input bit XORs a fixed
// 32-bit window of the key into the hash, rss.c:63-79), so for the 96-bit
// input daddr | saddr_i | dport | sport it splits into a part fixed per
// address, C(i) (20 nibble tables), and a part of the port alone: the high
// byte's two nibble tables (20, 21) and the low byte's (22, 23) merged into
// two 256-entry byte tables.  And GetRSSCPUCore reads only the hash's low 7
// bits ((h & 0x7F) [^ 3] % nq, rss.c:90-103), so every table holds just
// those, and the queue of all 128 values is one more table.  A candidate then
// costs three LDS byte reads (C(i) sits in a register) instead of 24 dword
// reads and a division: bit-identical, by linearity.
//
// A workgroup maps one tile of kQmapTile consecutive candidates (at most two
// addresses: kPorts > kQmapTile); each pass of its 256 lanes covers 1024
// consecutive candidates, a lane four of them, so every dword store of a
// wave is 256 contiguous bytes.
constexpr uint32_t kQmapTile = 4 * 4 * kBlock;     // 4096 candidates per workgroup
// rss_queue_map_kernel fills its 256-entry nibble tables one entry per lane
// and walks a tile in passes of 4 x 256 candidates (1024u * k below)
static_assert(kBlock == 256, "rss_queue_map_kernel's table fill and pass stride assume 256 lanes");

__device__ __forceinline__ uint32_t toeplitz_fixed7(const uint32_t *tab, uint32_t sip, uint32_t dip,
                                                    uint32_t dport) {
    uint32_t h = 0;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
        h ^= tab[(t << 4) | ((sip >> (28 - 4 * t)) & 15u)];
        h ^= tab[((8 + t) << 4) | ((dip >> (28 - 4 * t)) & 15u)];
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) h ^= tab[((16 + t) << 4) | ((dport >> (12 - 4 * t)) & 15u)];
    return h & 0x7Fu;
}

__global__ __launch_bounds__(kBlock) void rss_queue_map_kernel(PoolParams pp,
                                                               uint8_t *__restrict__ queue) {
    __shared__ uint8_t t_hi[256], t_lo[256], q_of[128];
    __shared__ uint32_t c_addr[2];
    const uint32_t tid = threadIdx.x;
    const uint32_t *tab = pp.rss_tables;
    // tiles of kQmapTile candidates, grid-stride (any num_addr: a grid of
    // one workgroup per tile would pass 2^31 tiles at ~140 K addresses)
    const uint64_t ntiles = (pp.total + kQmapTile - 1) / kQmapTile;
    uint64_t tile = blockIdx.x;
    uint64_t first = tile * kQmapTile;
    uint32_t i0 = (uint32_t)(first / kPorts);
    {
        const uint32_t b = tid;                                    // kBlock == 256
        t_hi[b] = (uint8_t)((tab[(20 << 4) | (b >> 4)] ^ tab[(21 << 4) | (b & 15u)]) & 0x7Fu);
        t_lo[b] = (uint8_t)((tab[(22 << 4) | (b >> 4)] ^ tab[(23 << 4) | (b & 15u)]) & 0x7Fu);
        if (b < 128) q_of[b] = (uint8_t)rss_core(b, pp.nq, pp.endian);
        if (b < 2) c_addr[b] = toeplitz_fixed7(tab, pp.daddr_h, pp.saddr_base_h + i0 + b, pp.dport_h);
    }
    __syncthreads();
    for (;;) {
    const uint64_t edge = (uint64_t)(i0 + 1) * kPorts;             // first candidate of address i0 + 1
    const uint32_t c0 = c_addr[0], c1 = c_addr[1];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint64_t g0 = first + 1024u * k + 4u * tid;
        if (g0 >= pp.total) break;
        uint32_t word = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint64_t g = g0 + b;
            const bool second = g >= edge;
            const uint32_t port = MTCP_GPU_MIN_PORT + (uint32_t)(g - (second ? edge : edge - kPorts));
            const uint32_t m = (second ? c1 : c0) ^ t_hi[port >> 8] ^ t_lo[port & 0xFFu];
            word |= (uint32_t)q_of[m] << (8 * b);
        }
        if (g0 + 3 < pp.total) {
            reinterpret_cast<uint32_t *>(queue)[g0 / 4] = word;
        } else {
            for (int b = 0; g0 + b < pp.total; ++b) queue[g0 + b] = (uint8_t)(word >> (8 * b));
        }
    }
    tile += gridDim.x;                                             // the next tile, if any
    if (tile >= ntiles) break;
    first = tile * kQmapTile;
    i0 = (uint32_t)(first / kPorts);
    __syncthreads();                                               // this tile's c_addr is read
    if (tid < 2) c_addr[tid] = toeplitz_fixed7(tab, pp.daddr_h, pp.saddr_base_h + i0 + tid, pp.dport_h);
    __syncthreads();
    }
}

// Matches of lane `t` of tile `blk`: candidates [blk*kPoolTile + 16t, +16).
__device__ __forceinline__ uint32_t pool_lane_mask(const uint8_t *queue, uint64_t total,
                                                   uint32_t core, uint64_t first) {
    uint32_t m = 0;
#pragma unroll
    for (int k = 0; k < kPoolPerThread; ++k)
        if (first + k < total && queue[first + k] == core) m |= 1u << k;
    return m;
}

// Exclusive prefix of v over the workgroup (4 waves); returns the total.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t &excl) {
    __shared__ uint32_t wsum[kWavesPerBlock];
    const uint32_t lane = threadIdx.x & (kWave - 1), wib = threadIdx.x / kWave;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, kWave);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == kWave - 1) wsum[wib] = x;
    __syncthreads();
    uint32_t before = 0, total = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) {
        if (w < (int)wib) before += wsum[w];
        total += wsum[w];
    }
    excl = before + x - v;
    __syncthreads();
    return total;
}

__global__ __launch_bounds__(kBlock) void pool_count_kernel(const uint8_t *__restrict__ queue,
                                                            uint64_t total, uint32_t core,
                                                            uint32_t *__restrict__ counts) {
    const uint64_t first = (uint64_t)blockIdx.x * kPoolTile + (uint64_t)threadIdx.x * kPoolPerThread;
    const uint32_t c = __popc(pool_lane_mask(queue, total, core, first));
    uint32_t excl;
    const uint32_t tot = block_exclusive_scan(c, excl);
    if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

// In place exclusive scan of counts[0..nb) by one workgroup; counts[nb] = sum.
__global__ __launch_bounds__(kBlock) void pool_scan_kernel(uint32_t *counts, uint32_t nb) {
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += kBlock) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < nb ? counts[i] : 0u;
        uint32_t excl;
        const uint32_t tot = block_exclusive_scan(v, excl);
        if (i < nb) counts[i] = carry + excl;
        carry += tot;
    }
    if (threadIdx.x == 0) counts[nb] = carry;
}

// Writes entry r (global rank among matches) for r < limit.
__global__ __launch_bounds__(kBlock) void pool_emit_kernel(const uint8_t *__restrict__ queue,
                                                           uint64_t total, uint32_t core,
                                                           const uint32_t *__restrict__ offsets,
                                                           uint32_t saddr_base_h, uint32_t limit,
                                                           mtcp_gpu_addr_entry *__restrict__ out) {
    const uint64_t first = (uint64_t)blockIdx.x * kPoolTile + (uint64_t)threadIdx.x * kPoolPerThread;
    uint32_t m = pool_lane_mask(queue, total, core, first);
    uint32_t excl;
    (void)block_exclusive_scan(__popc(m), excl);
    uint32_t r = offsets[blockIdx.x] + excl;
    while (m && r < limit) {
        const int k = __ffs(m) - 1;
        m &= m - 1;
        const uint64_t g = first + k;
        const uint32_t i = (uint32_t)(g / kPorts);
        const uint32_t port = MTCP_GPU_MIN_PORT + (uint32_t)(g - (uint64_t)i * kPorts);
        mtcp_gpu_addr_entry e;
        e.saddr = __builtin_bswap32(saddr_base_h + i);                  // htonl (addr_pool.c:158)
        e.sport = (uint16_t)(((port & 0xFFu) << 8) | (port >> 8));      // htons (addr_pool.c:168)
        e.rsvd = 0;
        out[r++] = e;
    }
}

}  // namespace mg
