// rx_span.hpp — chunk-parallel rx: a workgroup's lanes stream the 16 B chunks
// of its 64 frames back to back, whatever their sizes.
//
// rx_kernel (rx_kernels.hpp) gives each frame a 16-lane row for a round and
// the small-batch kernels (rx_wave.hpp) G lanes for the frame's whole life;
// either way a lane idles wherever its frame is shorter than the row or
// group.  Mid-size frames (128-640 B) and mixes of sizes (IMIX) are where
// that costs: rx_kernel's rounds for 128 B frames load 256 B rows that are
// half empty, and a group kernel's wave waits on its longest frame.  Here the
// workgroup (4 waves, 64 frames) numbers the chunks of its frames 0 .. C-1 in
// packet order (an exclusive scan of the chunk counts) and wave w takes
// windows w, w+4, ... of 64 consecutive chunks, U windows in flight:
//   chunk -> frame  lane i's chunk j belongs to the last frame whose first
//                   chunk is <= j: a 6-step binary search over the 64 starts,
//                   each step a ds_bpermute of the lane that holds them (a
//                   frame with no chunks shares its start with the next one,
//                   and the search takes the larger index, so it is skipped);
//                   a tile whose 64 frames have one chunk count divides instead
//   sums            v_sad_u16 over the chunk, an inclusive scan over the
//                   wave; the last lane of each frame's run in the window
//                   adds the run's sum (scan minus the scan before the run)
//                   to the wave's LDS sum of that frame — one lane per frame
//                   per window, so the adds never collide; the add is an
//                   LDS atomic only because that is one ds_add_u32 with no
//                   return (a plain += is a ds_read, a wait and a ds_write).
//                   Headroom: a 65 535 B frame is 4 097 chunks of at most
//                   8 x 0xFFFF, 2.15e9 < 2^32 (tests/test_gpu_wave.py
//                   test_max_length_frames_every_schedule)
//   headers         chunks 0..6 and the last chunk of every frame go to LDS
//                   packet-minor, as in rx_kernel, for parse_finish
// After one barrier wave 0 runs phase 2 with one lane per frame (the code
// every other kernel runs) and stores the records.  Loads stay fully
// coalesced for contiguous chunks (PSIO / io_module aggregates) and every
// loaded chunk is a chunk of a frame: no idle lanes, no partial rows.
// HBM traffic: the frames' chunks once, descriptors, records.
#pragma once

#include "rx_wave.hpp"

namespace mg {

constexpr int kSpanBlock = 256;                  // 4 waves
constexpr int kSpanWaves = kSpanBlock / kWave;
constexpr int kSpanP = kWave;                    // frames per workgroup: phase 2 on one wave

// Inclusive prefix sum over the wave: the row scans (DPP row_shr), then the
// totals of the rows below each row (readlanes of lanes 15, 31, 47).
__device__ __forceinline__ uint32_t wave_scan(uint32_t v, uint32_t lane) {
    v = row_sum(v);
    const uint32_t r0 = (uint32_t)__builtin_amdgcn_readlane((int)v, 15);
    const uint32_t r1 = r0 + (uint32_t)__builtin_amdgcn_readlane((int)v, 31);
    const uint32_t r2 = r1 + (uint32_t)__builtin_amdgcn_readlane((int)v, 47);
    const uint32_t row = lane >> 4;
    return v + (row == 0 ? 0u : row == 1 ? r0 : row == 2 ? r1 : r2);
}

// The frame of chunk j: the largest q with start[q] <= j (start[0] = 0 <= j),
// start[q] held by lane q.  *s = start[q].
__device__ __forceinline__ uint32_t span_find(uint32_t start, uint32_t j, uint32_t *s) {
    uint32_t lo = 0, slo = 0;
#pragma unroll
    for (int step = 32; step >= 1; step >>= 1) {
        const uint32_t m = lo + (uint32_t)step;
        const uint32_t v = shfl32(start, (int)m);
        const bool le = v <= j;
        lo = le ? m : lo;
        slo = le ? v : slo;
    }
    *s = slo;
    return lo;
}

// U: windows (64-chunk loads) in flight per wave.
// ABL (profiling only, tools/wave_probe.hip): 1 = phase 2 stores the sum
// only; 2 = descriptors and the scan only (stores the chunk count).
template <int MODE, bool RSS, int U = 4, int ABL = 0>
__global__ __launch_bounds__(kSpanBlock) void rx_span_kernel(KParams kp) {
    static_assert(MODE == kRxChunk || MODE == kRxPtrs, "rx modes only");
#ifndef MTCP_GPU_TESTING
    static_assert(ABL == 0, "the ABL (profiling) variants need a -DMTCP_GPU_TESTING build (tools/)");
#endif
    constexpr int P = kSpanP, S = P + 1;
    constexpr uint32_t kStride = kSpanWaves * kWave;          // chunks between a wave's windows
    __shared__ uint32_t rss_lds[RSS ? kRssTableWords : 1];
    __shared__ uint32_t hd[kHdRows * S];                        // dword i of frame q at hd[i * S + q]
    __shared__ uint32_t psum[kSpanWaves][P];                    // per wave: its runs' sums per frame
    __shared__ uint4 info[P];                                   // {p lo, p hi, L | ok << 16, nch}
    if constexpr (RSS) {
        for (int i = threadIdx.x; i < kRssTableWords; i += kSpanBlock) rss_lds[i] = kp.rss_tables[i];
    }
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr bool kPtrs = MODE == kRxPtrs;
    const uint64_t safe = (uint64_t)(uintptr_t)(kPtrs ? (const void *)kp.lens : (const void *)kp.buf);

    // ---- descriptors: lane q of every wave holds frame q of the tile (the
    //      same 512 B for the four waves: cache hits after the first) ---------
    const uint32_t k = blockIdx.x * P + lane;
    uint64_t p = safe;
    uint32_t L = 0;
    bool ok = false;
    if (k < kp.n) {
        if constexpr (kPtrs) {
            const uint64_t a = (uint64_t)(uintptr_t)kp.ptrs[k];
            L = kp.lens[k];
            ok = a != 0 && (a & 1) == 0;                       // any even start
            if (ok) p = a;
        } else {
            const uint64_t raw = *reinterpret_cast<const uint64_t *>(kp.desc + k);
            L = (uint32_t)(raw >> 32) & 0xFFFFu;
            const int64_t pos = (int64_t)((uint64_t)(uint32_t)raw << kp.off_shift) - kp.base_sub;
            ok = pos >= 0 && (pos & 1) == 0 && (uint64_t)pos + L <= kp.buf_len;
            if (ok) p = safe + (uint64_t)pos;
        }
    }
    const uint64_t p16 = p & ~15ull;
    const uint32_t nch = ok && L ? (uint32_t)((((p + L + 15) & ~15ull) - p16) >> 4) : 0u;
    const uint32_t inc = wave_scan(nch, lane);
    const uint32_t start = inc - nch;                           // first chunk of frame `lane`
    const uint32_t C = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    const uint32_t p16lo = (uint32_t)p16, p16hi = (uint32_t)(p16 >> 32);
    uint32_t *ps = psum[wib];
    ps[lane] = 0;
    if (wib == 0) info[lane] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), L | ((uint32_t)ok << 16), nch);
    __builtin_amdgcn_wave_barrier();
    if constexpr (ABL == 2) {
        if (wib == 0 && k < kp.n) kp.out[k].saddr = nch;
        return;
    }

    // ---- the chunk stream ----------------------------------------------------------
    // A tile of 64 frames of one chunk count (fixed-size traffic) needs no
    // search: frame j / nch, chunk j % nch.
    const uint32_t nch0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)nch);
    const bool uniform = nch0 != 0 && __ballot(nch != nch0) == 0;
    for (uint32_t base = wib * kWave; base < C; base += kStride * U) {      // wave-uniform
        v4u x[U];
        uint32_t qv[U], cv[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j0 = base + u * kStride;
            if (j0 < C) {
                const uint32_t j = min(j0 + lane, C - 1);               // past the end: a valid chunk, unused
                uint32_t s, q;
                if (uniform) {
                    q = j / nch0;
                    s = q * nch0;
                } else {
                    q = span_find(start, j, &s);
                }
                qv[u] = q;
                cv[u] = j - s;
                const uint64_t fq = ((uint64_t)shfl32(p16hi, (int)q) << 32) | shfl32(p16lo, (int)q);
                x[u] = gload_nt(fq + 16ull * (j - s));
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j0 = base + u * kStride;
            if (j0 < C) {
                const uint32_t j = j0 + lane;
                const bool valid = j < C;
                const uint32_t q = qv[u], c = cv[u];
                const uint32_t nq = shfl32(nch, (int)q);
                const uint32_t sc = wave_scan(valid ? halves4(x[u], 0u) : 0u, lane);
                // the run of frame q in this window starts at lane `first`
                const uint32_t sq = j - c;
                const uint32_t first = sq > j0 ? sq - j0 : 0u;
                const uint32_t before = shfl32(sc, (int)(first ? first - 1 : 0u));
                if (valid && (c == nq - 1 || lane == kWave - 1)) atomicAdd(&ps[q], sc - (first ? before : 0u));
                if (valid) {
                    if (c < kSlotChunks - 1) {                          // raw chunks 0..6
                        uint32_t *d = hd + 4 * c * S + q;
                        d[0] = x[u].x; d[S] = x[u].y; d[2 * S] = x[u].z; d[3 * S] = x[u].w;
                    }
                    if (c == nq - 1) {                                  // last chunk
                        uint32_t *d = hd + 4 * (kSlotChunks - 1) * S + q;
                        d[0] = x[u].x; d[S] = x[u].y; d[2 * S] = x[u].z; d[3 * S] = x[u].w;
                    }
                }
            }
        }
    }
    __syncthreads();

    // ---- phase 2: wave 0, one lane per frame -------------------------------------------
    if (wib != 0) return;
    const uint32_t q = lane;
    if (k >= kp.n) return;
    const uint4 inf = info[q];
    const uint64_t pq = ((uint64_t)inf.y << 32) | inf.x;
    uint32_t sum = 0;
#pragma unroll
    for (int w = 0; w < kSpanWaves; ++w) sum += psum[w][q];
    if constexpr (ABL == 1) {
        kp.out[k].saddr = sum;
        return;
    }
    Pkt pk;
    if (__ballot((pq & 3) != 0) == 0)
        pk = parse_finish<MODE, S, true, true>(hd + q, sum, pq, inf.z & 0xFFFFu, inf.w, (inf.z >> 16) & 1u);
    else
        pk = parse_finish<MODE, S, true, false>(hd + q, sum, pq, inf.z & 0xFFFFu, inf.w, (inf.z >> 16) & 1u);
    uint32_t rss_hash = 0, rss_queue = 0;
    if constexpr (RSS) {
        if (pk.tcp_entry) {
            rss_hash = toeplitz_tables(rss_lds, pk.saddr, pk.daddr, pk.ports);
            rss_queue = rss_core(rss_hash, kp.rss_nq, kp.rss_endian);
        }
    }
    store_record(kp, k, pk, rss_hash, rss_queue);
    if (kp.bins) kp.bins[k] = flow_bin(pk.saddr, pk.daddr, pk.ports, pk.verdict);
}

}  // namespace mg
