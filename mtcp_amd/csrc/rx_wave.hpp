// rx_wave.hpp — one wavefront per packet: the shape BASELINE.json's north
// star names, dispatched for small batches (mtcp_gpu.hip pick_sched).
//
// rx_kernel (rx_kernels.hpp) gives a wave 64 packets and streams them four
// at a time through 16-lane rows; on 1 M-packet batches that keeps every
// lane busy and runs at the HBM read ceiling.  A batch of a few thousand
// frames — one io_module aggregate is 4 096, mTCP's own bursts are <= 64
// (MAX_PKT_BURST dpdk_module.c:71, PS_CHUNK_SIZE psio_module.c:15) — then
// occupies only n/64 waves of a GPU that holds 2 048 and runs as a chain of
// dependent round trips.  Here every packet gets its own wave, so a small
// batch puts n waves in flight at once:
//   phase 1  the wave's 64 lanes stream the frame on the absolute 16 B chunk
//            grid, up to kWaveLoads loads per lane issued before any is
//            consumed (8 KiB per trip: an MTU frame is one round trip, a
//            9000 B frame two); v_sad_u16 adds the 16-bit halves, a DPP row
//            reduction and four readlanes give the frame's chunk sum in an
//            SGPR.  Chunks 0..6 (the headers) and the last chunk go to the
//            wave's 128 B of LDS.
//   phase 2  parse_head_wave / finish_seg (rx_kernels.hpp: the common frame
//            on one straight path, parse_head's chain for every other one)
//            on the whole wave with wave-uniform operands: one
//            instruction stream per packet, mostly scalar.  The CU's one
//            scalar unit serves its 16 waves of a 4 096-packet batch, so the
//            SALU count per packet sets phase 2's time (PMC, 4 096 x 1500 B:
//            ~190 SALU of phase 2 per wave ~ 1.3 us); the segment sum is
//            therefore the plain chunk total (taken as the loads land) minus
//            the header and tail bytes, branch-free in the lanes.  RSS is the
//            Toeplitz sum spread over the lanes — lane i owns input bits i and
//            64 + i, the key window of each bit comes straight from the key
//            words (BuildKeyCache, util/rss.c:13-105, without the table), an
//            XOR reduction finishes it — so no table is staged per workgroup.
//   stores   lanes 0..4 write the 40 B record as five 8 B pieces (lanes 0..1
//            the 16 B compact record, MTCP_GPU_F_COMPACT); the tx fill
//            writes its two 16-bit check fields from lane 0.
#pragma once

#include "rx_kernels.hpp"

namespace mg {

constexpr int kWaveLoads = 10;  // 16 B loads per lane per trip: 10 KiB of frame (a 9000 B frame in one)

// XOR over the 64 lanes (DPP row_shr steps, then the four row results).
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 15) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 31) ^
           (uint32_t)__builtin_amdgcn_readlane((int)v, 47) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

// GetRSSHash (util/rss.c:107-145) over the wave.  The 96 input bits are
// sip | dip | sp | dp in host order, most significant first: the wire bytes
// of saddr, daddr, sport, dport, i.e. bswap32 of the record's memory-order
// words.  Input bit i selects key_cache[i] = key bits [i, i + 32)
// (BuildKeyCache); kw[] are key bytes 0..15 as big-endian words.
__device__ __forceinline__ uint32_t toeplitz_wave(const uint32_t (&kw)[4], uint32_t saddr,
                                                  uint32_t daddr, uint32_t ports, uint32_t lane) {
    const uint32_t b = lane & 31;
    const uint32_t in = lane < 32 ? bswap32(saddr) : bswap32(daddr);
    const uint64_t lo = lane < 32 ? (((uint64_t)kw[0] << 32) | kw[1]) : (((uint64_t)kw[1] << 32) | kw[2]);
    uint32_t v = ((in >> (31 - b)) & 1u) ? (uint32_t)(lo >> (32 - b)) : 0u;   // bit lane
    const uint64_t hi = ((uint64_t)kw[2] << 32) | kw[3];
    if (lane < 32 && ((bswap32(ports) >> (31 - b)) & 1u)) v ^= (uint32_t)(hi >> (32 - b));   // bit 64 + lane
    return wave_xor(v);
}

// ABL (profiling only, tools/wave_probe.hip): 1 = the frame stream and its
// plain chunk sum only (lane 0 stores it); 2 = descriptor only (stores L);
// 3 = stop after the header parse (stores the verdict); 4 = after the
// segment sum (stores the TCP checksum).
// SEG, the segment sum [T, 14 + ip_len): 1 = the plain sum of every chunk
// minus the bytes outside the segment (the header bytes from LDS, the tail of
// the last chunk from LDS), one lane per dword and one reduction, when the
// segment runs to the frame's last chunk and the frame fits one trip; any
// other frame, and SEG 0 always, masks each chunk against the segment.
// NL: 16 B loads per lane per trip (a trip covers 1 KiB * NL of frame):
// 2 for MTU-sized batches, kWaveLoads for jumbo ones (mtcp_gpu.hip picks by
// the batch's average slot); fewer unrolled loads, fewer instructions.
// WPB: waves (= packets) per workgroup.
template <int MODE, bool RSS, int ABL = 0, int SEG = 1, int NL = kWaveLoads, int WPB = kWavesPerBlock>
__global__ __launch_bounds__(kWave * WPB) void rx_wave_kernel(KParams kp) {
#ifndef MTCP_GPU_TESTING
    static_assert(ABL == 0, "the ABL (profiling) variants need a -DMTCP_GPU_TESTING build (tools/)");
#endif
    __shared__ uint4 lds[WPB][kSlotChunks];                // the frame's chunks 0..6
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t k = blockIdx.x * WPB + wib;             // this wave's packet
    if (k >= kp.n) return;
    uint4 *hd4 = lds[wib];
    const uint32_t *hd = reinterpret_cast<const uint32_t *>(hd4);

    // ---- descriptor (wave-uniform, scalar loads) ------------------------------------
    uint64_t p = 0;
    uint32_t L;
    bool ok;
    if constexpr (MODE == kRxPtrs || MODE == kTxPtrs) {
        const uint64_t a = (uint64_t)(uintptr_t)kp.ptrs[k];
        L = kp.lens[k];
        ok = a != 0 && (a & 1) == 0;                       // any even start
        if (ok) p = a;
    } else {
        const uint64_t raw = *reinterpret_cast<const uint64_t *>(kp.desc + k);
        L = (uint32_t)(raw >> 32) & 0xFFFFu;
        const int64_t pos = (int64_t)((uint64_t)(uint32_t)raw << kp.off_shift) - kp.base_sub;
        ok = pos >= 0 && (pos & 1) == 0 && (uint64_t)pos + L <= kp.buf_len;
        if (ok) p = (uint64_t)(uintptr_t)kp.buf + (uint64_t)pos;
    }
    const uint64_t p16 = p & ~15ull;
    const uint32_t nch = ok && L ? (uint32_t)((((p + L + 15) & ~15ull) - p16) >> 4) : 0u;
    if constexpr (ABL == 2) {
        if (lane == 0) kp.out[k].saddr = L;
        return;
    }

    // ---- phase 1: the wave issues the frame's first trip (10 KiB) --------------------
    constexpr uint32_t kTrip = kWave * NL;
    v4u x[NL];
    auto issue = [&](uint32_t c0) {
#pragma unroll
        for (int u = 0; u < NL; ++u) {
            if (c0 + u * kWave < nch) {                    // wave-uniform
                const uint32_t c = c0 + u * kWave + lane;
                x[u] = gload_nt(p16 + 16ull * (c < nch ? c : nch - 1));
            }
        }
    };
    issue(0);
    if constexpr (ABL == 1) {
        uint32_t acc = 0;
        for (uint32_t c0 = 0; c0 < nch; c0 += kTrip) {
            if (c0) issue(c0);
#pragma unroll
            for (int u = 0; u < NL; ++u)
                if (c0 + u * kWave < nch && c0 + u * kWave + lane < nch) acc = halves4(x[u], acc);
        }
        acc = row_sum(acc);
        const uint32_t sum = (uint32_t)__builtin_amdgcn_readlane((int)acc, 15) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 31) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 47) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 63);
        if (lane == 0) kp.out[k].saddr = sum;
        return;
    }

    // ---- phase 2a: the header, as soon as chunks 0..6 arrive (lanes 0..6 of
    //      the first load).  Lane i then holds packet dword i (i < 25, funneled
    //      for 2-byte-aligned starts); the fields are readlanes of it, the IP
    //      header sum a 32-lane reduction, the verdict chain scalar code. ----------
    if (nch && lane < kSlotChunks - 1) hd4[lane] = make_uint4(x[0].x, x[0].y, x[0].z, x[0].w);
    // SEG 1: the plain sum of every chunk of a one-trip frame, taken now so
    // that the loads' registers are free during the parse, and the load that
    // holds the last chunk (lane (nch - 1) % 64 of load (nch - 1) / 64)
    uint32_t total = 0;
    v4u last = {0u, 0u, 0u, 0u};
    if constexpr (SEG == 1) {
        if (nch <= kTrip) {
            const uint32_t ul = (nch - 1) / kWave;
#pragma unroll
            for (int u = 0; u < NL; ++u) {
                const uint32_t c = u * kWave + lane;
                if ((uint32_t)u * kWave < nch) {
                    if (c < nch) total = halves4(x[u], total);
                    if (ul == (uint32_t)u) last = x[u];
                }
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t sh = (uint32_t)(p & 15);
    const uint32_t a = sh >> 2, fb = 8 * (sh & 3);
    const uint32_t li = lane < 25 ? lane : 24u;
    const uint32_t pdw = __builtin_amdgcn_alignbit(hd[a + li + 1], hd[a + li], fb);
    auto pd = [&](uint32_t i) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)pdw, (int)i); };
    auto ipsum = [&](uint32_t ihl) -> uint32_t {
        // words of bytes [14, 14 + 4*ihl): the high half of dword 3, dwords
        // 4 .. 2 + ihl, the low half of dword 3 + ihl
        // (as lane masks, not branches: the scalar unit is this kernel's bound)
        const uint32_t hi = pdw >> 16, lo = pdw & 0xFFFFu;
        const uint32_t m3 = 0u - (uint32_t)(lane == 3);
        const uint32_t mm = 0u - (uint32_t)(lane > 3 && lane < 3 + ihl);
        const uint32_t ml = 0u - (uint32_t)(lane == 3 + ihl);
        const uint32_t w = (hi & (m3 | mm)) + (lo & (mm | ml));
        const uint32_t r = row_sum(w);
        return (uint32_t)__builtin_amdgcn_readlane((int)r, 15) + (uint32_t)__builtin_amdgcn_readlane((int)r, 31);
    };
    // bytes 4i+2..4i+5 in lane i (lane i + 1's dword through DPP wave_shl:1)
    const uint32_t nxt = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)pdw, 0x130, 0xF, 0xF, false);
    const uint32_t swv = __builtin_amdgcn_alignbit(nxt, pdw, 16), swbv = bswap32(swv);
    auto sw = [&](uint32_t i) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)swv, (int)i); };
    auto swb = [&](uint32_t i) -> uint32_t { return (uint32_t)__builtin_amdgcn_readlane((int)swbv, (int)i); };
    Pkt pk = parse_head_wave<MODE>(pd, ipsum, sw, swb, L, ok);
    if constexpr (ABL == 3) {
        if (lane == 0) kp.out[k].saddr = pk.verdict;
        return;
    }

    // ---- phase 2b: the segment [T, 14 + ip_len), summed by the lanes holding it --------
    // SEG 1: the segment runs to the last chunk ([E, end of the chunk grid)
    // lies inside it) and the frame is one trip
    const uint32_t e_rel = sh + 14 + pk.ip_len;                      // byte E on the grid
    const bool seg_fast = SEG == 1 && nch <= kTrip && ((e_rel + 15) >> 4) == nch;
    if (pk.need_sum && seg_fast) {
        uint32_t acc = total;
        // bytes to remove, without branches: [0, sh + T) from the header
        // dwords (lanes 0..22; the low half of dword `whole` when sh + T ends
        // mid-dword) and [E, 16 * nch) from the last chunk, by its lane
        const uint32_t nb = sh + pk.T, whole = nb >> 2, te = e_rel & 15;
        const uint32_t v = hd[lane < 23 ? lane : 0u];
        const uint32_t mw = 0u - (uint32_t)(lane < whole);
        const uint32_t mh = 0u - (uint32_t)(lane == whole && (nb & 2));
        uint32_t w = halves(v & mw, 0u) + (v & 0xFFFFu & mh);
        const uint32_t d[4] = {last.x, last.y, last.z, last.w};
        uint32_t t = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            // bytes of dword j at or past E: all when E lies before it, none
            // when after it, else its bytes from E - 4j on
            const int sft = min(max(8 * ((int)te - 4 * j), 0), 32);
            t = halves(d[j] & (uint32_t)(0xFFFFFFFFull << sft), t);
        }
        w += t & (0u - (uint32_t)(te && lane == (nch - 1) % kWave));
        acc -= w;
        acc = row_sum(acc);
        const uint32_t seg = (uint32_t)__builtin_amdgcn_readlane((int)acc, 15) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 31) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 47) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 63);
        finish_seg<MODE>(pk, seg);
    } else if (pk.need_sum) {
        const uint32_t lo = sh + pk.T, span = 14 + pk.ip_len - pk.T;   // bytes [lo, lo + span) of the grid
        uint32_t acc = 0;
        auto take = [&](const v4u &v, uint32_t c) {
            const uint32_t cb = 16 * c - lo;                // chunk start relative to the segment
            if (cb <= span - 16 && span >= 16) {            // whole chunk inside
                acc = halves4(v, acc);
            } else if (16 * c < lo + span && 16 * c + 16 > lo) {
                // a boundary chunk: keep its bytes inside the segment (an odd
                // span ends on the low byte of a word: tcp_util.c:176)
                const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const uint32_t o = cb + 4 * j;          // wraps below the segment
                    const uint32_t m = (o < span ? 0xFFu : 0u) | (o + 1 < span ? 0xFF00u : 0u) |
                                       (o + 2 < span ? 0xFF0000u : 0u) | (o + 3 < span ? 0xFF000000u : 0u);
                    acc = halves(d[j] & m, acc);
                }
            }
        };
        for (uint32_t c0 = 0; c0 < nch; c0 += kTrip) {
            if (c0 || SEG == 1) issue(c0);                  // jumbo frames: later trips (SEG 1: all)
#pragma unroll
            for (int u = 0; u < NL; ++u) {
                const uint32_t c = c0 + u * kWave + lane;
                if (c0 + u * kWave < nch && c < nch) take(x[u], c);
            }
        }
        acc = row_sum(acc);
        const uint32_t seg = (uint32_t)__builtin_amdgcn_readlane((int)acc, 15) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 31) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 47) +
                             (uint32_t)__builtin_amdgcn_readlane((int)acc, 63);
        finish_seg<MODE>(pk, seg);
    }

    if constexpr (ABL == 4) {
        if (lane == 0) kp.out[k].saddr = pk.tcp_csum;
        return;
    }
    if constexpr (is_tx(MODE)) {
        if (lane == 0) {
            const uint32_t checks = fold_csum(pk.s_ip - pk.ip_check) | (pk.tcp_csum << 16);
            if (kp.tx_report) {
                // report mode (mtcp_gpu_tx_fill_ptrs): the host writes the
                // two fields into its own frames; T = 0: not filled
                kp.tx_report[k] = make_uint2(pk.need_sum ? checks : 0u, pk.need_sum ? pk.T : 0u);
            } else if (pk.need_sum) {
                uint16_t *q16 = reinterpret_cast<uint16_t *>(p);
                q16[12] = (uint16_t)checks;                            // iph->check (ip_out.c:145,164)
                q16[(pk.T + 16) >> 1] = (uint16_t)(checks >> 16);      // tcph->check (tcp_out.c:329)
            }
            if (pk.need_sum && kp.fill_count) atomicAdd(kp.fill_count, 1u);
        }
    } else {
        uint32_t rss_hash = 0, rss_queue = 0;
        if constexpr (RSS) {
            if (pk.tcp_entry) {
                rss_hash = toeplitz_wave(kp.rss_key, pk.saddr, pk.daddr, pk.ports, lane);
                rss_queue = rss_core(rss_hash, kp.rss_nq, kp.rss_endian);
            }
        }
        if (kp.compact) {
            uint32_t c[4];
            pack_compact(pk, rss_hash, rss_queue, c);
            if (lane < 2)
                reinterpret_cast<uint2 *>(kp.out)[2 * k + lane] = lane ? make_uint2(c[2], c[3])
                                                                      : make_uint2(c[0], c[1]);
        } else {
            uint32_t r[10];
            pack_record(pk, rss_hash, rss_queue, r);
            if (lane < 5) {
                uint32_t xx = r[0], yy = r[1];
#pragma unroll
                for (int i = 1; i < 5; ++i)
                    if (lane == (uint32_t)i) xx = r[2 * i], yy = r[2 * i + 1];
                reinterpret_cast<uint2 *>(kp.out + k)[lane] = make_uint2(xx, yy);
            }
        }
        if (kp.bins && lane == 0) kp.bins[k] = flow_bin(pk.saddr, pk.daddr, pk.ports, pk.verdict);
    }
}

// ---------------------------------------------------------------------------
// The small-batch kernel as dispatched: phase 1 with G lanes per packet (a
// whole wave per packet for G = 64, the north star's shape; a 16-lane row or
// a 4-lane quad for smaller frames), phase 2 with ONE LANE per packet.
//
// rx_wave_kernel above runs phase 2 on the whole wave with wave-uniform
// operands, i.e. ~400 wave-instructions per packet, scalar-unit bound when
// many waves share a CU (tools/wave_probe.hip: phase 1 over 4 096 x 1500 B is
// at the 2.3-2.6 us launch floor, the whole kernel 3.8 us).  Here a
// 16-wave workgroup streams P = 1024 / G packets, leaves each packet's chunk
// sum, header chunks, last chunk and descriptor in LDS (packet-minor, as in
// rx_kernel), meets at one barrier, and then P lanes parse P packets in one
// instruction stream (parse_finish, the code rx_kernel runs), so phase 2
// costs 1/P of the wave-uniform version's issue slots.
constexpr int kGroupBlock = 1024;              // 16 waves
// Quads run in 256-thread workgroups (P = 64: one full phase-2 wave, and
// four times the workgroups in flight): 1 M x 64 B 24.9 vs 31.5 us in
// 1024-thread ones, 4 096 x 64 B 2.76 vs 3.23 (tools/wave_probe g4b256 / g4,
// profiles/r4/group_span_probe.jsonl).  Rows keep 1024: at 2-4 K MTU frames
// the 256-thread rows lose (5.9 vs 4.2 us).
constexpr int kQuadBlock = 256;
// 8-lane groups (mid-size batches of MTU-class frames): 512 threads, P = 64
constexpr int kOctBlock = 512;

// BLK: threads per workgroup (P = BLK / G packets).  U: 16 B loads per lane
// per trip (0: by G).
template <int G, int BLK = kGroupBlock, int U_ = 0>
struct GroupShape {
    static_assert(G == 4 || G == 8 || G == 16 || G == 64, "lanes per packet: a quad, 8 lanes, a row or the wave");
    static_assert(BLK % kWave == 0 && BLK >= G && BLK <= 1024, "whole waves, at most 1024 threads");
    static constexpr int P = BLK / G;                           // packets per workgroup
    static constexpr int U = U_ ? U_ : G == 64 ? 8 : G == 16 ? 6 : G == 8 ? 4 : 2;   // loads per lane per trip
    static constexpr int R = G >= 16 ? G / 16 : 1;              // partial sums per packet
    static constexpr int S = P + 1;                             // LDS stride (odd: no conflicts)
    static constexpr int W2 = (P + kWave - 1) / kWave;          // waves that run phase 2
};

// ABL (profiling only, tools/wave_probe.hip): 1 = phase 2 stores the sum only.
// AL: phase 2 takes parse_finish's ALIGNED form when every frame of the wave
// starts on a 4-byte boundary (AL 0: never; an A/B baseline).
template <int MODE, bool RSS, int G, int ABL = 0, int AL = 1, int BLK = kGroupBlock, int U_ = 0>
__global__ __launch_bounds__(BLK) void rx_group_kernel(KParams kp) {
#ifndef MTCP_GPU_TESTING
    static_assert(ABL == 0, "the ABL (profiling) variants need a -DMTCP_GPU_TESTING build (tools/)");
#endif
    using Sh = GroupShape<G, BLK, U_>;
    constexpr int P = Sh::P, U = Sh::U, R = Sh::R, S = Sh::S;
    __shared__ uint32_t rss_lds[RSS ? kRssTableWords : 1];
    __shared__ uint32_t hd[kHdRows * S];       // dword i of packet q at hd[i * S + q]
    __shared__ uint32_t psum[P * R];
    __shared__ uint4 info[P];                  // {p lo, p hi, L | ok << 16, nch}
    if constexpr (RSS) {
        for (int i = threadIdx.x; i < kRssTableWords; i += BLK) rss_lds[i] = kp.rss_tables[i];
    }
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wib = threadIdx.x >> 6;
    const uint32_t gl = lane % G;
    const uint32_t pkt = wib * (kWave / G) + lane / G;     // packet within the workgroup
    const uint32_t k = blockIdx.x * P + pkt;
    constexpr bool kPtrs = MODE == kRxPtrs || MODE == kTxPtrs;
    const uint64_t safe = (uint64_t)(uintptr_t)(kPtrs ? (const void *)kp.lens : (const void *)kp.buf);

    // ---- descriptor -----------------------------------------------------------
    uint64_t p = safe;
    uint32_t L = 0;
    bool ok = false;
    if (k < kp.n) {
        if constexpr (kPtrs) {
            const uint64_t a = (uint64_t)(uintptr_t)kp.ptrs[k];
            L = kp.lens[k];
            ok = a != 0 && (a & 1) == 0;                   // any even start
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

    // ---- phase 1: G lanes stream each frame -------------------------------------
    uint32_t acc = 0;
    for (uint32_t c0 = 0; __ballot(c0 < nch); c0 += U * G) {
        v4u x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (__ballot(c0 + u * G < nch)) {              // some frame of the wave needs load u
                const uint32_t c = c0 + u * G + gl;
                const uint32_t cc = c < nch ? c : (nch ? nch - 1 : 0u);   // clamp: no exec mask
                x[u] = gload_nt(p16 + 16ull * cc);
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (__ballot(c0 + u * G < nch)) {
                const uint32_t c = c0 + u * G + gl;
                if (c < nch) {
                    acc = halves4(x[u], acc);
                    if (c < kSlotChunks - 1) {                      // raw chunks 0..6
                        uint32_t *d = hd + 4 * c * S + pkt;
                        d[0] = x[u].x; d[S] = x[u].y; d[2 * S] = x[u].z; d[3 * S] = x[u].w;
                    }
                    if (c == nch - 1) {                             // last chunk
                        uint32_t *d = hd + 4 * (kSlotChunks - 1) * S + pkt;
                        d[0] = x[u].x; d[S] = x[u].y; d[2 * S] = x[u].z; d[3 * S] = x[u].w;
                    }
                }
            }
        }
    }
    if constexpr (G <= 8) {
        acc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)acc, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
        acc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)acc, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
        if constexpr (G == 8)
            acc += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)acc, 0x141, 0xF, 0xF, false);  // row_half_mirror
        if (gl == 0) psum[pkt] = acc;
    } else {
        acc = row_sum(acc);
        if ((lane & (kRow - 1)) == kRow - 1) psum[pkt * R + gl / kRow] = acc;
    }
    if (gl == 0) info[pkt] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), L | ((uint32_t)ok << 16), nch);
    __syncthreads();

    // ---- phase 2: one lane per packet --------------------------------------------
    if (wib >= (uint32_t)Sh::W2) return;
    const uint32_t q = wib * kWave + lane;
    const uint32_t kk = blockIdx.x * P + q;
    if (q >= (uint32_t)P || kk >= kp.n) return;
    const uint4 inf = info[q];
    const uint64_t pq = ((uint64_t)inf.y << 32) | inf.x;
    uint32_t sum = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) sum += psum[q * R + r];
    if constexpr (ABL == 1) {
        kp.out[kk].saddr = sum;
        return;
    }
    Pkt pk;
    if (AL && __ballot((pq & 3) != 0) == 0)
        pk = parse_finish<MODE, S, true, true>(hd + q, sum, pq, inf.z & 0xFFFFu, inf.w, (inf.z >> 16) & 1u);
    else
        pk = parse_finish<MODE, S, true, false>(hd + q, sum, pq, inf.z & 0xFFFFu, inf.w, (inf.z >> 16) & 1u);
    if constexpr (is_tx(MODE)) {
        const uint32_t checks = fold_csum(pk.s_ip - pk.ip_check) | (pk.tcp_csum << 16);
        if (kp.tx_report) {
            // report mode (mtcp_gpu_tx_fill_ptrs): the host writes the two
            // fields into its own frames; T = 0: not filled
            kp.tx_report[kk] = make_uint2(pk.need_sum ? checks : 0u, pk.need_sum ? pk.T : 0u);
        } else if (pk.need_sum) {
            uint16_t *q16 = reinterpret_cast<uint16_t *>(pq);
            q16[12] = (uint16_t)checks;                            // iph->check (ip_out.c:145,164)
            q16[(pk.T + 16) >> 1] = (uint16_t)(checks >> 16);      // tcph->check (tcp_out.c:329)
        }
        if (pk.need_sum && kp.fill_count) atomicAdd(kp.fill_count, 1u);
    } else {
        uint32_t rss_hash = 0, rss_queue = 0;
        if constexpr (RSS) {
            if (pk.tcp_entry) {
                rss_hash = toeplitz_tables(rss_lds, pk.saddr, pk.daddr, pk.ports);
                rss_queue = rss_core(rss_hash, kp.rss_nq, kp.rss_endian);
            }
        }
        store_record(kp, kk, pk, rss_hash, rss_queue);
        if (kp.bins) kp.bins[kk] = flow_bin(pk.saddr, pk.daddr, pk.ports, pk.verdict);
    }
}

}  // namespace mg
