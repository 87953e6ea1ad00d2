// rx_kernels.hpp — gfx950 (CDNA4) kernels for mTCP's software per-packet path:
// the rx chain ProcessPacket -> ProcessIPv4Packet -> head of ProcessTCPPacket
// (mtcp/src/eth_in.c:9-56, ip_in.c:15-62, tcp_in.c:1138-1175) with its
// ip_fast_csum (io_engine/include/ps.h:66-95) and TCPCalcChecksum
// (mtcp/src/tcp_util.c:157-190), the Toeplitz RSS hash (util/rss.c:107-165),
// and the tx checksum fill (ip_out.c:94,164; tcp_out.c:211,329).
//
// Work decomposition: one 64-lane wave per group of 64 packets (interleaved
// over the grid in runs of B = 8); lane k owns packet k of the group.  The
// phase-1 round order depends on the schedule (SCHED, below): the 16 rounds
// in frame order for large frames, size-sorted rounds (large frames four
// per round, small ones sixteen per round) for mixed or small ones.
//   phase 0  lane k loads its descriptor (one coalesced 8-byte load); no
//            header is read yet.
//   phase 1  the four 16-lane DPP rows of the wave stream four frames at a
//            time (round i: row r takes frame 4i + r), each row 256 B per
//            wave-instruction on the absolute 16 B chunk grid, six loads
//            (6 KiB per wave) issued before any is consumed — a 1500 B frame
//            is one round trip.  v_sad_u16 adds the 16-bit halves; a row
//            reduction (4 DPP row_shr adds) leaves each frame's chunk sum in
//            LDS.  While a frame is in registers its first seven chunks (the
//            headers) and its last chunk are copied to the owner's LDS slot.
//   phase 2  lane k parses its headers from LDS (verdict chain, fields, IP
//            checksum), subtracts from the chunk sum the bytes outside the
//            TCP segment [T, E) (E = 14 + tot_len), adds the pseudo header,
//            folds, hashes the 4-tuple through 24 nibble tables in LDS and
//            holds its 40 B record (16 B with CMP) in registers; the held records of up to
//            8 passes are stored at the end (through LDS, as 16 B pieces of
//            contiguous runs) — stores interleaved with the frame stream
//            cost several times their bytes.
// HBM traffic is one pass over the frames plus descriptors and results.
// Exactness: the reference sums little-endian u16 words into a u32 (no
// overflow for any u16 length).  Every packet starts at an even address, so
// its words are exactly the 16-bit halves of the aligned dwords that hold
// it; all partial sums here are exact integers below 2^31 and the final fold
// is the reference's own two-step fold.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/mtcp_gpu.h"

namespace mg {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kRssTableWords = 24 * 16;  // nibble tables
constexpr int kSlotChunks = 8;           // chunks 0..6 raw (headers), 7 = last chunk
constexpr int kRow = 16;                 // lanes per DPP row = lanes per frame
constexpr int kUnroll = 6;               // loads in flight per row (96 chunks = 1536 B)

// kTxPtrs (tx fill of a pointer burst) and the tx report run in the small
// kernels only (rx_wave_kernel, rx_group_kernel: mtcp_gpu.hip pick_sched).
enum Mode : int { kRxChunk = 0, kRxPtrs = 1, kTxChunk = 2, kTxPtrs = 3 };
constexpr bool is_tx(int m) { return m == kTxChunk || m == kTxPtrs; }
// Phase-1 schedules (rx_kernel's SCHED; see its comment).  Dispatched:
// kSchedUnrolled and kSchedSorted; the others are A/B baselines.
enum Sched : int {
    kSchedRolled = 0,        // rolled trip loop
    kSchedUnrolled = 3,      // 16 rounds unrolled, single-buffered
    kSchedSortedBase = 4,    // size-sorted rounds
    kSchedSortedEarly = 5,   // + first small rounds with the first large round
    kSchedSorted = 6,        // + issued with the previous pass's pre-issue
};

struct KParams {
    const uint8_t *buf;            // chunk base (chunk modes), 16 B aligned
    uint64_t buf_len;              // descriptor bound: bytes valid from buf
    int64_t base_sub;              // subtracted from every descriptor byte offset
    const mtcp_gpu_desc *desc;
    const uint8_t *const *ptrs;    // pointer mode
    const uint16_t *lens;
    uint32_t n;
    uint32_t off_shift;
    mtcp_gpu_result *out;
    const uint32_t *rss_tables;    // 24 x 16 Toeplitz nibble tables
    uint32_t rss_nq;
    uint32_t rss_endian;
    uint32_t *fill_count;          // tx fill: frames written (may be null)
    uint32_t *bins;                // rx: HashFlow bin per packet (may be null)
    uint2 *tx_report;              // tx (wave kernel): {checks, T} per frame instead of writing them
    uint32_t *stamps;              // profiling builds only (rx_kernel STAMP): 4 dwords per wave
    uint32_t rss_key[4];           // key bytes 0..15, big-endian words (wave kernel's Toeplitz)
    uint32_t compact;              // rx: 16 B mtcp_gpu_result16 records (MTCP_GPU_F_COMPACT)
};

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// Loads through address-space-1 (global) pointers: a generic pointer built
// from shuffled lane values would compile to flat_load, whose out-of-order
// completion forces s_waitcnt vmcnt(0) lgkmcnt(0) before every use.
typedef __attribute__((address_space(1))) const v4u gv4u;
__device__ __forceinline__ v4u gload(uint64_t addr) { return *reinterpret_cast<gv4u *>(addr); }
// Streaming (once-read) frame data: non-temporal global load.
__device__ __forceinline__ v4u gload_nt(uint64_t addr) {
    return __builtin_nontemporal_load(reinterpret_cast<gv4u *>(addr));
}
__device__ __forceinline__ uint4 gload4(uint64_t addr) {
    const v4u v = gload(addr);
    return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t bswap16(uint32_t v) {
    return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// acc + lo16(d) + hi16(d) in one v_sad_u16
__device__ __forceinline__ uint32_t halves(uint32_t d, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(d, 0u, acc);
}
__device__ __forceinline__ uint32_t halves4(const v4u &v, uint32_t acc) {
    return halves(v.w, halves(v.z, halves(v.y, halves(v.x, acc))));
}

// The reference's fold (tcp_util.c:184-188), also ip_fast_csum's result for
// ihl >= 5 (ps.h:66-95; SURVEY §8 a2').
__device__ __forceinline__ uint32_t fold_csum(uint32_t s) {
    s = (s >> 16) + (s & 0xFFFFu);
    s += s >> 16;
    return (~s) & 0xFFFFu;
}

// Sum over each 16-lane row; the row total lands in the row's lane 15.
__device__ __forceinline__ uint32_t row_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    return v;
}

__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

// Lane i of each 16-lane row, broadcast to the row (DPP row_newbcast:i).
__device__ __forceinline__ uint32_t row_bcast(uint32_t v, int i) {
#define MG_NB(n) case n: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x150 + n, 0xF, 0xF, false)
    switch (i) {
        MG_NB(0); MG_NB(1); MG_NB(2); MG_NB(3); MG_NB(4); MG_NB(5); MG_NB(6); MG_NB(7);
        MG_NB(8); MG_NB(9); MG_NB(10); MG_NB(11); MG_NB(12); MG_NB(13); MG_NB(14);
        default: return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x15F, 0xF, 0xF, false);
    }
#undef MG_NB
}

// Jenkins one-at-a-time over the 12 key bytes, each read as a signed char
// (tcp_stream.c:77-87 `char *key`; x86 char is signed).  The bytes of w are
// key bytes 4q..4q+3 in memory order.
__device__ __forceinline__ uint32_t hash_flow(const uint32_t (&w)[3]) {
    uint32_t h = 0;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        h += (uint32_t)(int32_t)(int8_t)(uint8_t)(w[i >> 2] >> (8 * (i & 3)));
        h += h << 10;
        h ^= h >> 6;
    }
    h += h << 3;
    h ^= h >> 11;
    h += h << 15;
    return h & (MTCP_GPU_NUM_BINS_FLOWS - 1);
}

// The flow-table bin of one rx record (f3): HashFlow of the key
// ProcessTCPPacket hands to StreamHTSearch (tcp_in.c:1180-1186: saddr =
// iph->daddr, daddr = iph->saddr, sport = tcph->dest, dport = tcph->source),
// FLOW_NONE for packets that never get there.
__device__ __forceinline__ uint32_t flow_bin(uint32_t saddr, uint32_t daddr, uint32_t ports,
                                             uint32_t verdict) {
    const uint32_t w[3] = {daddr, saddr, (ports >> 16) | (ports << 16)};
    return verdict == MTCP_GPU_V_TCP_OK ? hash_flow(w) : MTCP_GPU_FLOW_NONE;
}

// Compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N).
template <int I0, int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    if constexpr (I0 < N) {
        f(std::integral_constant<int, I0>{});
        static_for<I0 + 1, N>(f);
    }
}

// Per-wave LDS, packet-minor ("structure of arrays") so that phase 2, where
// lane k reads dword i of its own packet, hits 64 distinct banks: dword i of
// packet k lives at hd[i * kHdStride + k].  Rows 0..27 hold raw chunks 0..6
// of the frame on the 16 B grid (the headers), rows 28..31 its last chunk.
// The odd stride also keeps phase 1's writes (7 chunks of 4 packets at once)
// conflict-free.  sum[k] is packet k's chunk sum.
constexpr int kHdRows = 4 * kSlotChunks;   // 32
constexpr int kHdStride = kWave + 1;       // 65 dwords
struct WaveLds {
    uint32_t hd[kHdRows * kHdStride];
    uint32_t sum[kWave + 1];       // [kWave]: scratch for rows without a frame
    uint4 info[kWave];             // size-sorted schedule: {p16 lo, p16 hi, nch, owner}
};

// What phase 2 derives for one packet: the record's fields, and for the tx
// fill the TCP header offset, the IP header's word sum and its check field.
struct Pkt {
    uint32_t verdict = MTCP_GPU_V_BAD_DESC;
    uint32_t eth_type = 0, ip_len = 0, ihl_doff = 0, ip_csum = 0, tcp_csum = 0;
    uint32_t saddr = 0, daddr = 0, ports = 0, seq = 0, ack = 0, window = 0, flags = 0;
    uint32_t payload_len = 0;
    uint32_t T = 0, s_ip = 0, ip_check = 0;
    uint32_t seg_len = 0;     // bytes of the summed segment [T, 14 + ip_len) (pseudo header length)
    uint32_t tcheck = 0;      // tcph->check as received (tx: the sum is taken with it zeroed)
    bool tcp_entry = false;   // reached the TCP header: the 4-tuple is valid (RSS)
    bool need_sum = false;    // the segment sum is needed (tx: fill this frame)
    bool icmp = false;        // the segment is an ICMP message (no pseudo header)
};

// The reference's rx chain in its order (eth_in.c:9-56, ip_in.c:15-62, head
// of tcp_in.c:1138-1175) up to the segment sum: verdict, fields, ip_fast_csum
// from the header words, and whether and over which bytes the TCP (or ICMP)
// checksum is taken.  pd(i) = packet dword i (bytes 4i..4i+3), read only for
// the bytes each step has checked to lie inside the frame (L bytes);
// ipsum(ihl) = the sum of the 16-bit words of the IP header, bytes
// [14, 14 + 4*ihl), for 5 <= ihl <= 15 (ip_fast_csum's adc chain, exact:
// SURVEY §8 a2'); sw(i) = bytes 4i+2..4i+5 (the funnel of dwords i and i+1
// by 16 bits: every 4-byte field past the Ethernet header sits there) and
// swb(i) = its byte swap — a wave parsing one packet computes both in all
// lanes at once and reads them out, instead of two shifts and an or per field.
template <int MODE, class PD, class IPSUM, class SW, class SWB>
__device__ __forceinline__ Pkt parse_head(PD pd, IPSUM ipsum, SW sw, SWB swb, uint32_t L,
                                          bool desc_ok) {
    Pkt k;
    uint32_t h[7];
#pragma unroll
    for (int i = 3; i < 7; ++i) h[i] = pd(i);
    const uint32_t d0 = h[3];                 // bytes 12..15
    if (!desc_ok) return k;
    k.verdict = MTCP_GPU_V_TRUNCATED;
    if (L < 14) return k;
    k.eth_type = bswap16(d0 & 0xFFFFu);                                    // eth_in.c:13
    if (k.eth_type != 0x0800u) {
        k.verdict = k.eth_type == 0x0806u ? MTCP_GPU_V_ARP : MTCP_GPU_V_ETH_OTHER;
        return k;
    }
    if (L < 18) return k;
    k.ip_len = bswap16(h[4] & 0xFFFFu);                                    // ip_in.c:21
    const uint32_t ihl = (d0 >> 16) & 0xFu;
    k.ihl_doff = ihl;
    const uint32_t ver = (d0 >> 20) & 0xFu;
    if (!is_tx(MODE) && k.ip_len < 20) {
        k.verdict = MTCP_GPU_V_IP_SHORT;                                   // ip_in.c:25-26
        return k;
    }
    if (L < 14 + 4 * (ihl > 4 ? ihl : 1)) return k;   // ps.h:68-70: ihl <= 4 reads one dword
    // ip_fast_csum: ihl <= 4 returns dword 0 as is (ps.h:72-73)
    if (ihl >= 5) k.s_ip = ipsum(ihl);
    k.ip_check = h[6] & 0xFFFFu;
    k.ip_csum = ihl <= 4 ? (d0 >> 16) : fold_csum(k.s_ip);
    const uint32_t proto = h[5] >> 24;                                     // ip_in.c:52
    k.T = 14 + 4 * ihl;
    bool tcp_entry = false;
    if (is_tx(MODE)) {
        tcp_entry = ver == 4 && ihl >= 5 && proto == 6 && L >= k.T + 20;
        k.verdict = MTCP_GPU_V_ETH_OTHER;
    } else if (k.ip_csum != 0) {
        k.verdict = MTCP_GPU_V_IP_CSUM_BAD;                                // ip_in.c:35-36
    } else if (ver != 4) {
        k.verdict = MTCP_GPU_V_IP_VERSION;                                 // ip_in.c:47-50
    } else if (proto == 1) {
        k.verdict = MTCP_GPU_V_ICMP;
        // ICMPChecksum(icmph, ip_len - 4*ihl) (icmp.c:18-42), the echo-request
        // check of icmp.c:94, when the datagram lies inside the frame; a
        // negative length skips the loop: ~0
        if (14 + k.ip_len <= L) {
            if (k.ip_len >= 4 * ihl) {
                k.icmp = k.need_sum = true;
                k.seg_len = k.payload_len = k.ip_len - 4 * ihl;
            } else {
                k.tcp_csum = 0xFFFFu;
            }
        }
    } else if (proto != 6) {
        k.verdict = MTCP_GPU_V_IP_PROTO_OTHER;                             // ip_in.c:57-59
    } else if (L >= k.T + 16) {
        tcp_entry = true;
    }
    if (tcp_entry) {
        // tcp_in.c:1142-1149: tcph = iph + 4*ihl
        const uint32_t tw = (k.T - 2) >> 2;                                // T = 4 tw + 2
        const uint32_t e3 = pd(tw + 3), e4 = pd(tw + 4);
        const uint32_t doff = (e3 >> 20) & 0xFu;
        k.tcp_entry = true;
        k.saddr = sw(6);                                                   // bytes 26..29
        k.daddr = sw(7);                                                   // bytes 30..33
        k.ports = sw(tw);                                                  // sport | dport << 16
        k.seq = swb(tw + 1);
        k.ack = swb(tw + 2);
        k.window = bswap16(e4 & 0xFFFFu);
        k.flags = e3 >> 24;
        k.tcheck = e4 >> 16;
        k.ihl_doff = ihl | (doff << 4);
        if (is_tx(MODE)) {
            if (doff >= 5 && k.ip_len >= 4 * (ihl + doff) && 14 + k.ip_len <= L) {
                k.need_sum = true;
                k.seg_len = k.ip_len - 4 * ihl;
            }
        } else if (k.ip_len < ((ihl + doff) << 2)) {
            k.verdict = MTCP_GPU_V_TCP_LEN_BAD;                            // tcp_in.c:1155-1156
        } else {
            k.payload_len = k.ip_len - ((ihl + doff) << 2);                // tcp_in.c:1144
            if (14 + k.ip_len <= L) {
                k.need_sum = true;
                k.seg_len = k.ip_len - 4 * ihl;                            // tcp_in.c:1166
            }
        }
    }
    return k;
}

// The common rx frame — Ethernet IPv4 (version 4, ihl 5) carrying TCP,
// tot_len >= 20, its headers inside the frame, the IP checksum good — parsed
// on one straight path with one exit; false (k untouched) for every other
// frame, which parse_head's chain then decides.  Same results: the checks
// are the chain's own for ihl = 5 (ip_in.c:25-60, tcp_in.c:1142-1156).
// The chain's early returns cost a zeroing of every record field per exit
// edge (scalar moves in the wave kernel, divergent blocks per lane).
template <int MODE, class PD, class IPSUM, class SW, class SWB>
__device__ __forceinline__ bool parse_common(PD pd, IPSUM ipsum, SW sw, SWB swb, uint32_t L,
                                             bool desc_ok, Pkt &k) {
    if constexpr (is_tx(MODE)) {
        return false;
    } else {
        const uint32_t d0 = pd(3), h4 = pd(4), h5 = pd(5);              // bytes 12..23
        const uint32_t ipl = bswap16(h4 & 0xFFFFu);
        // bytes 12..14 = 08 00 45: ethertype IPv4, version 4, ihl 5; protocol 6;
        // L >= T + 16 with T = 34
        if (!(desc_ok && L >= 50 && (d0 & 0xFFFFFFu) == 0x450008u && (h5 >> 24) == 6u && ipl >= 20u))
            return false;
        const uint32_t s_ip = ipsum(5u);
        if (fold_csum(s_ip) != 0) return false;
        const uint32_t e3 = pd(11), e4 = pd(12);                          // tcph bytes 12..19
        const uint32_t doff = (e3 >> 20) & 0xFu, hlen = (5 + doff) << 2;
        const bool len_bad = ipl < hlen;
        k.verdict = len_bad ? MTCP_GPU_V_TCP_LEN_BAD : MTCP_GPU_V_TRUNCATED;
        k.eth_type = 0x0800u;
        k.ip_len = ipl;
        k.ihl_doff = 5u | (doff << 4);
        k.ip_csum = 0;
        k.s_ip = s_ip;
        k.ip_check = pd(6) & 0xFFFFu;
        k.T = 34;
        k.tcp_entry = true;
        k.saddr = sw(6);
        k.daddr = sw(7);
        k.ports = sw(8);
        k.seq = swb(9);
        k.ack = swb(10);
        k.window = bswap16(e4 & 0xFFFFu);
        k.flags = e3 >> 24;
        k.tcheck = e4 >> 16;
        k.payload_len = len_bad ? 0u : ipl - hlen;
        k.need_sum = !len_bad && 14 + ipl <= L;
        k.seg_len = k.need_sum ? ipl - 20 : 0u;
        k.icmp = false;
        k.tcp_csum = 0;
        return true;
    }
}

// parse_head_wave: a wave parsing one packet (rx_wave_kernel): the common
// frame on the straight path, the chain for the rest (interleaved A/B:
// 4 096 x 1500 B 3.91 -> 3.76 us).
template <int MODE, class PD, class IPSUM, class SW, class SWB>
__device__ __forceinline__ Pkt parse_head_wave(PD pd, IPSUM ipsum, SW sw, SWB swb, uint32_t L,
                                               bool desc_ok) {
    Pkt k;
    if (parse_common<MODE>(pd, ipsum, sw, swb, L, desc_ok, k)) return k;
    return parse_head<MODE>(pd, ipsum, sw, swb, L, desc_ok);
}

// parse_head_sel: the per-lane form (rx_kernel and the grouped kernels,
// through parse_finish), with the same results as parse_head above, for
// callers whose pd(i) is readable for every i <= 22 (a staged copy, past the
// frame's end too) and whose ipsum(ihl) takes any ihl.  Single exit: every candidate field is computed from the header dwords and kept
// only where the reference's chain reaches it (the step's length check
// passed); the verdict is a select chain in the reference's check order.  The
// early-return form costs a divergent branch, an exec-mask save and a
// re-zeroing of every record field per check when lanes parse different
// packets (quad kernel phase 2: 1071 -> 907 instructions, 64 K x 64 B
// 5.1 -> 4.8 us).  A wave parsing ONE packet (rx_wave_kernel) keeps the
// early-return form: its branches are scalar and nearly free, while the
// selects cost scalar-unit issue slots, its bound (4 096 x 1500 B 3.9 ->
// 4.4 us with this form).
template <int MODE, class PD, class IPSUM, class SW, class SWB>
__device__ __forceinline__ Pkt parse_head_sel(PD pd, IPSUM ipsum, SW sw, SWB swb, uint32_t L,
                                          bool desc_ok) {
    constexpr bool tx = is_tx(MODE);
    const uint32_t d0 = pd(3), h4 = pd(4), h5 = pd(5), h6 = pd(6);     // bytes 12..27
    const uint32_t eth = bswap16(d0 & 0xFFFFu);                           // eth_in.c:13
    const uint32_t ipl = bswap16(h4 & 0xFFFFu);                           // ip_in.c:21
    const uint32_t ihl = (d0 >> 16) & 0xFu, ver = (d0 >> 20) & 0xFu;
    const uint32_t proto = h5 >> 24;                                      // ip_in.c:52
    const uint32_t T = 14 + 4 * ihl;
    // how far the chain gets: the frame holds the Ethernet header, it is
    // IPv4, tot_len is readable, passes ip_len >= 20 (rx), and the IP header
    // lies inside the frame (ip_fast_csum reads 4*ihl bytes for ihl >= 5, one
    // dword for ihl <= 4: ps.h:68-70, pinned by oracle/ref/ub_probe.c)
    const bool ok14 = desc_ok && L >= 14;
    const bool isip = ok14 && eth == 0x0800u;
    const bool ok18 = isip && L >= 18;
    const bool shrt = !tx && ipl < 20;                                    // ip_in.c:25-26
    const bool okhdr = ok18 && !shrt && L >= 14 + 4 * (ihl > 4 ? ihl : 1);
    // ip_fast_csum: ihl <= 4 returns dword 0 as is (ps.h:72-73)
    const uint32_t s_ip = ipsum(ihl);
    const uint32_t ip_csum = ihl <= 4 ? (d0 >> 16) : fold_csum(s_ip);
    const bool ip_good = okhdr && ip_csum == 0 && ver == 4;              // ip_in.c:35-50
    // tcp_in.c:1142-1149: tcph = iph + 4*ihl (T = 4 tw + 2)
    const uint32_t tw = (T - 2) >> 2;
    const uint32_t e3 = pd(tw + 3), e4 = pd(tw + 4);
    const uint32_t doff = (e3 >> 20) & 0xFu;
    const bool tcp_entry = tx ? okhdr && ver == 4 && ihl >= 5 && proto == 6 && L >= T + 20
                              : ip_good && proto == 6 && L >= T + 16;
    const uint32_t hlen = (ihl + doff) << 2;
    const bool in_frame = 14 + ipl <= L;                                  // the datagram is readable
    const bool len_bad = !tx && tcp_entry && ipl < hlen;                  // tcp_in.c:1155-1156
    // ICMPChecksum(icmph, ip_len - 4*ihl) (icmp.c:18-42), the echo-request
    // check of icmp.c:94, when the datagram lies inside the frame; a negative
    // length skips the loop: ~0
    const bool icmp_in = !tx && ip_good && proto == 1 && in_frame;
    const bool icmp = icmp_in && ipl >= 4 * ihl;
    const bool tcp_sum = tx ? tcp_entry && doff >= 5 && ipl >= hlen && in_frame
                            : tcp_entry && !len_bad && in_frame;          // tcp_in.c:1166

    uint32_t v = MTCP_GPU_V_TRUNCATED;                  // no check failed, the TCP sum pending
    if (!tx) {
        v = len_bad ? MTCP_GPU_V_TCP_LEN_BAD : v;
        v = ip_good && proto != 6 ? MTCP_GPU_V_IP_PROTO_OTHER : v;        // ip_in.c:57-59
        v = ip_good && proto == 1 ? MTCP_GPU_V_ICMP : v;
        v = okhdr && ip_csum == 0 && ver != 4 ? MTCP_GPU_V_IP_VERSION : v; // ip_in.c:47-50
        v = okhdr && ip_csum != 0 ? MTCP_GPU_V_IP_CSUM_BAD : v;           // ip_in.c:35-36
        v = ok18 && shrt ? MTCP_GPU_V_IP_SHORT : v;
    } else {
        v = okhdr ? MTCP_GPU_V_ETH_OTHER : v;
    }
    v = ok14 && !isip ? (eth == 0x0806u ? MTCP_GPU_V_ARP : MTCP_GPU_V_ETH_OTHER) : v;
    v = desc_ok ? v : MTCP_GPU_V_BAD_DESC;

    Pkt k;
    k.verdict = v;
    k.eth_type = ok14 ? eth : 0u;
    k.ip_len = ok18 ? ipl : 0u;
    k.ihl_doff = ok18 ? ihl | (tcp_entry ? doff << 4 : 0u) : 0u;
    k.s_ip = okhdr && ihl >= 5 ? s_ip : 0u;
    k.ip_check = okhdr ? h6 & 0xFFFFu : 0u;
    k.ip_csum = okhdr ? ip_csum : 0u;
    k.T = okhdr ? T : 0u;
    k.tcp_entry = tcp_entry;
    k.saddr = tcp_entry ? sw(6) : 0u;                                     // bytes 26..29
    k.daddr = tcp_entry ? sw(7) : 0u;                                     // bytes 30..33
    k.ports = tcp_entry ? sw(tw) : 0u;                                    // sport | dport << 16
    k.seq = tcp_entry ? swb(tw + 1) : 0u;
    k.ack = tcp_entry ? swb(tw + 2) : 0u;
    k.window = tcp_entry ? bswap16(e4 & 0xFFFFu) : 0u;
    k.flags = tcp_entry ? e3 >> 24 : 0u;
    k.tcheck = tcp_entry ? e4 >> 16 : 0u;
    k.icmp = icmp;
    k.need_sum = tcp_sum || icmp;
    k.seg_len = k.need_sum ? ipl - 4 * ihl : 0u;
    k.payload_len = icmp ? ipl - 4 * ihl                                  // icmp.c:94's length
                  : !tx && tcp_entry && !len_bad ? ipl - hlen : 0u;       // tcp_in.c:1144
    k.tcp_csum = icmp_in && !icmp ? 0xFFFFu : 0u;
    return k;
}

// The checksum from the exact word sum of the segment [T, 14 + ip_len):
// TCPCalcChecksum's pseudo header and two-step fold (tcp_util.c:157-190),
// or ICMPChecksum's fold (icmp.c:36-38); the rx verdict (tcp_in.c:1167-1173).
template <int MODE>
__device__ __forceinline__ void finish_seg(Pkt &k, uint32_t seg) {
    uint32_t s = seg;
    if (is_tx(MODE)) s -= k.tcheck;                            // computed with check = 0
    if (!k.icmp) {
        s += (k.saddr & 0xFFFFu) + (k.saddr >> 16);            // tcp_util.c:179-182
        s += (k.daddr & 0xFFFFu) + (k.daddr >> 16);
        s += bswap16(k.seg_len);
        s += 0x0600u;                                          // htons(IPPROTO_TCP)
    }
    k.tcp_csum = fold_csum(s);
    if (!is_tx(MODE) && !k.icmp)
        k.verdict = k.tcp_csum ? MTCP_GPU_V_TCP_CSUM_BAD : MTCP_GPU_V_TCP_OK;
}

// Phase 2 of one packet from the LDS copy of its header chunks and its
// chunk sum (rx_kernel's per-lane phase 2):
//   raw[i * S], i < 28: dword i of the frame's first seven 16 B chunks on the
//                       absolute grid (chunk 0 holds the frame's first byte);
//   raw[(28 + j) * S]:  dword j of its last chunk;
//   sum:                the sum of the 16-bit halves over all its chunks.
// The frame starts at any even address p (sh = p & 15 bytes into chunk 0):
// packet dword i is the funnel of raw dwords a+i and a+i+1 (a = sh / 4) by
// 8 * (sh & 3) bits, and each 16-bit word of the packet is still a whole
// half of one aligned dword, which keeps the sum exact.  The segment sum is
// the chunk sum minus the bytes outside [T, 14 + ip_len).
// COMMON: the common frame on parse_common's straight path first (the
// grouped kernels; rx_kernel's RSS instantiations have no registers left for
// both paths).
// ALIGNED: the caller knows the frame starts on a 4-byte boundary (p & 3 == 0,
// every frame of a PSIO chunk): packet dword i is raw dword a + i, no funnel
// shift and one LDS read per dword.
template <int MODE, int S, bool COMMON = false, bool ALIGNED = false>
__device__ __forceinline__ Pkt parse_finish(const uint32_t *raw, uint32_t sum, uint64_t p,
                                            uint32_t L, uint32_t nch, bool desc_ok) {
    const uint32_t sh = (uint32_t)(p & 15);
    const uint32_t a = sh >> 2, fb = 8 * (sh & 3);
    auto pd = [&](uint32_t i) -> uint32_t {      // packet dword i (bytes 4i..4i+3)
        if constexpr (ALIGNED) return raw[(a + i) * S];
        return __builtin_amdgcn_alignbit(raw[(a + i + 1) * S], raw[(a + i) * S], fb);
    };
    auto ipsum = [&](uint32_t ihl) -> uint32_t {  // words [14, 14 + 4*ihl): dwords 3..3+ihl
        // every dword read, the ones past the header masked: no per-dword
        // branch (the staged rows reach pd(18))
        uint32_t s_ip = pd(3) >> 16, lo_last = 0;
#pragma unroll
        for (int j = 1; j < 16; ++j) {
            const uint32_t w = pd(3 + j);
            s_ip = halves(j < (int)ihl ? w : 0u, s_ip);
            lo_last = j == (int)ihl ? w & 0xFFFFu : lo_last;
        }
        return s_ip + lo_last;
    };
    auto sw = [&](uint32_t i) -> uint32_t { return __builtin_amdgcn_alignbit(pd(i + 1), pd(i), 16); };
    auto swb = [&](uint32_t i) -> uint32_t { return bswap32(sw(i)); };
    Pkt k;
    if (!COMMON || !parse_common<MODE>(pd, ipsum, sw, swb, L, desc_ok, k))
        k = parse_head_sel<MODE>(pd, ipsum, sw, swb, L, desc_ok);
    if (k.need_sum) {
        // The chunk sum covers [p16, p16 + 16*nch).  Remove the bytes before
        // the frame, the header bytes [0, T), and everything at or past
        // E = 14 + ip_len.
        // (a) bytes [p16, p + T): the bytes of chunk 0 before the frame (raw
        //     dwords 0..a-1, and the low half of dword a when sh & 2), the
        //     Ethernet header (frame words 0..6: packet dwords 0..2 and the
        //     low half of dword 3) and the IP header [14, T), whose exact
        //     word sum s_ip the IP checksum already took (a segment is summed
        //     only past an IP header that passed, so ihl >= 5)
        uint32_t s_out = k.s_ip + (pd(3) & 0xFFFFu);
        s_out = halves(pd(2), halves(pd(1), halves(pd(0), s_out)));
#pragma unroll
        for (uint32_t i = 0; i < 3; ++i)
            if (i < a) s_out = halves(raw[i * S], s_out);
        if (!ALIGNED && (sh & 2)) s_out += raw[a * S] & 0xFFFFu;
        // (b) bytes [p + E, p16 + 16*nch)
        const uint64_t p16 = p & ~15ull;
        const uint64_t e_abs = p + 14 + k.ip_len;
        const uint64_t end = p16 + 16ull * nch;
        const uint32_t te = (uint32_t)(e_abs & 15);
        uint64_t cstart = e_abs & ~15ull;                          // chunk holding byte E
        if (te) {
            // partial chunk: the last chunk when E and the frame end share it
            uint4 w;
            if (cstart + 16 == end) {
                const uint32_t *t = raw + 4 * (kSlotChunks - 1) * S;
                w = make_uint4(t[0], t[S], t[2 * S], t[3 * S]);
            } else {
                w = gload4(cstart);                                // rare: E well before len
            }
            const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int drop = (int)te - 4 * i;   // low bytes inside the segment
                const uint32_t m = drop <= 0 ? 0xFFFFFFFFu : drop >= 4 ? 0u : (0xFFFFFFFFu << (8 * drop));
                s_out = halves(wv[i] & m, s_out);
            }
            cstart += 16;
        }
        for (; cstart < end; cstart += 16) {                       // rare: whole chunks past E
            const uint4 w = gload4(cstart);
            s_out = halves(w.w, halves(w.z, halves(w.y, halves(w.x, s_out))));
        }
        finish_seg<MODE>(k, sum - s_out);                          // exact segment sum
    }
    return k;
}

// The 40 B record (include/mtcp_gpu.h mtcp_gpu_result) as ten dwords.
__device__ __forceinline__ void pack_record(const Pkt &k, uint32_t rss_hash, uint32_t rss_queue,
                                            uint32_t (&r)[10]) {
    r[0] = k.saddr;
    r[1] = k.daddr;
    r[2] = k.ports;
    r[3] = k.seq;
    r[4] = k.ack;
    r[5] = k.window | (k.ip_len << 16);
    r[6] = k.ip_csum | (k.tcp_csum << 16);
    r[7] = rss_hash;
    r[8] = k.payload_len | (k.ihl_doff << 16) | (k.flags << 24);
    r[9] = k.verdict | (rss_queue << 8) | (k.eth_type << 16);
}

// The 16 B record (mtcp_gpu_result16, MTCP_GPU_F_COMPACT) as four dwords:
// the same fields as pack_record's, for callers that need the verdict only.
__device__ __forceinline__ void pack_compact(const Pkt &k, uint32_t rss_hash, uint32_t rss_queue,
                                             uint32_t (&r)[4]) {
    r[0] = rss_hash;
    r[1] = k.ip_csum | (k.tcp_csum << 16);
    r[2] = k.payload_len | (k.ip_len << 16);
    r[3] = k.ihl_doff | (k.flags << 8) | (k.verdict << 16) | (rss_queue << 24);
}

// Store one packet's record from one lane (the small kernels' per-lane phase
// 2): 40 B as five 8 B pieces, or 16 B as one piece.
__device__ __forceinline__ void store_record(const KParams &kp, uint32_t rec, const Pkt &k,
                                             uint32_t rss_hash, uint32_t rss_queue) {
    if (kp.compact) {
        uint32_t c[4];
        pack_compact(k, rss_hash, rss_queue, c);
        reinterpret_cast<uint4 *>(kp.out)[rec] = make_uint4(c[0], c[1], c[2], c[3]);
    } else {
        uint32_t r[10];
        pack_record(k, rss_hash, rss_queue, r);
        uint2 *o = reinterpret_cast<uint2 *>(kp.out + rec);
#pragma unroll
        for (int i = 0; i < 5; ++i) o[i] = make_uint2(r[2 * i], r[2 * i + 1]);
    }
}

// util/rss.c:107-145 as 24 nibble tables (built on the host from the key
// cache of BuildKeyCache, util/rss.c:13-105): the input bytes (sip, dip, sp,
// dp host order, MSB first) are saddr / daddr / ports in memory order.
__device__ __forceinline__ uint32_t toeplitz_tables(const uint32_t *tab, uint32_t saddr,
                                                    uint32_t daddr, uint32_t ports) {
    uint32_t hh = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const uint32_t sb = (saddr >> (8 * b)) & 0xFFu;
        const uint32_t db = (daddr >> (8 * b)) & 0xFFu;
        const uint32_t pb = (ports >> (8 * b)) & 0xFFu;
        hh ^= tab[((2 * b) << 4) | (sb >> 4)] ^ tab[((2 * b + 1) << 4) | (sb & 15)];
        hh ^= tab[((8 + 2 * b) << 4) | (db >> 4)] ^ tab[((9 + 2 * b) << 4) | (db & 15)];
        hh ^= tab[((16 + 2 * b) << 4) | (pb >> 4)] ^ tab[((17 + 2 * b) << 4) | (pb & 15)];
    }
    return hh;
}

// util/rss.c:153-165 / mtcp/src/rss.c:90-103: off[m & 3] = {3,1,-1,-3} == m ^ 3
__device__ __forceinline__ uint32_t rss_core(uint32_t hh, uint32_t nq, uint32_t endian) {
    uint32_t m = hh & 0x7Fu;
    if (endian) m ^= 3u;
    return m % nq;
}

// A lane's frame: address, length, descriptor validity, and its chunk range
// [p16, p16 + 16*nch) on the absolute 16 B grid.
struct Frame {
    uint64_t p;
    uint32_t L;
    bool ok, live;
    uint64_t p16;
    uint32_t nch;
    // the frame row `row` streams in round `rlane`, i.e. frame 4*rlane + row,
    // gathered once per pass so that a round only needs a row broadcast
    uint32_t r_nch, r_lo, r_hi;
};

// One row-step of phase 1: kUnroll loads of 256 B per row, round i (rows take
// frames 4i..4i+3), chunks [c0, c0 + kUnroll*16) of the row's frame.
struct Trip {
    int i;
    uint32_t c0, nj;
    uint64_t base;
    uint32_t col;     // the frame's owner lane = its column in WaveLds (kWave: scratch)
    uint32_t skip = 0;  // LALIGN: chunks before the frame at the start of the first trip
    uint32_t k = 0, ntrip = 0;   // REV: trip step and the frame's trip count
};

// Packet <-> lane mapping, in passes of 64*W packets (W = waves in the grid):
// lane k of wave w owns packet pass*64W + (k/B)*(W*B) + w*B + k%B.  B = 64:
// each wave owns 64 consecutive packets; smaller B interleaves the waves so
// that, round by round, the whole grid streams one compact window of frames.
// ABL (profiling only): 1 = stop after phase 1 (store the chunk sums);
// 2 = also no LDS header/tail copies; 3 = also no per-chunk range mask.
// With DEFER 0, ABL >= 1 stores nothing (phase 1 alone).
// DEFER (rx modes): results of up to DEFER passes wait in registers and are
// stored together when the buffer is full and at the end, instead of after
// every pass.  Stores interleaved with the frame stream cost far more HBM
// time than their bytes (tools/rx_variants ladder: 40 B/packet written per
// pass +45 us on C2, written at the end +18 us); DEFER 0 stores per pass.
// SCHED, the phase-1 schedule: 0 = rolled trip loop (row broadcasts through
// a switch); 3 = the 16 rounds unrolled, single-buffered (constant DPP
// broadcasts); 4 = size-sorted rounds; 5 = sorted, the first two small rounds
// issued with the first large round through L2; 6 = as 5, issued with the
// pre-issued first large round at the end of the previous pass.  Dispatched:
// 3 (large frames) and 6 (small-slot chunks); the others are A/B baselines
// for tools/rx_variants.hip (earlier variants — double-buffered unrolled
// rounds, round pairs, software-pipelined trips, per-pass stores interleaved
// with the next pass's loads — lost on every config and were removed).
// LALIGN: multi-trip frames stream from the start of their first 128 B line.
// STAMP (profiling builds, tools/rx_variants.hip): lane 0 of each wave writes
// {start, end} of s_memrealtime (100 MHz), HW_REG_XCC_ID and HW_REG_HW_ID to
// kp.stamps[4 * wave ...].
// WPB: waves per workgroup (the grid then holds 8 / WPB workgroups per CU).
// XSKIP (timing probe only, tools/rx_variants "abl_xskip*": its records are
// wrong): in the last pass, the waves on odd XCDs (XSKIP > 0) or on even
// ones (XSKIP < 0) leave their last |XSKIP| frames unread — how much a
// launch would gain if work moved between the XCD groups.
// PRIO: the second workgroup on each CU (blockIdx >= gridDim / 2; the
// dispatcher fills every CU once before the second round) runs at
// s_setprio(PRIO & 3): the older wave of a SIMD otherwise wins its issue
// arbitration and finishes first; PRIO & 4: only for the first half of its
// passes.
// CMP: write 16 B mtcp_gpu_result16 records (MTCP_GPU_F_COMPACT) — four dwords
// held per pass instead of ten, plus the flow bin when one is asked for (the
// compact record has no 4-tuple to hash at the flush).
// WPE: waves per SIMD the register allocation must allow (2: up to 256
// VGPRs; 3: 168, a third workgroup per CU; tools/occ_probe.hip).
// COOP: the workgroup loads its descriptors together (phase 0 below; the
// unrolled schedule of the chunk modes); false: each lane its own (A/B).
template <int MODE, bool RSS, int SCHED, bool LALIGN = false, int ABL = 0, int DEFER = 8, int B = 8,
          bool NT = true, int U = 6, bool REV = false, bool STAMP = false, int PRIO = 0,
          int WPB = kWavesPerBlock, int XSKIP = 0, bool CMP = false, int WPE = 2, bool COOP = true>
__global__ __launch_bounds__(kWave * WPB) __attribute__((amdgpu_waves_per_eu(WPE))) void rx_kernel(KParams kp) {
#ifndef MTCP_GPU_TESTING
    // the product library instantiates no profiling or timing-probe variant
    // (XSKIP's records are wrong by design): those exist for tools/ only
    static_assert(ABL == 0 && !STAMP && XSKIP == 0,
                  "rx_kernel's ABL / STAMP / XSKIP variants need a -DMTCP_GPU_TESTING build (tools/)");
#endif
    uint64_t t_start = 0;
    if constexpr (STAMP) t_start = __builtin_amdgcn_s_memrealtime();
    if constexpr ((PRIO & 3) > 0) {
        if (blockIdx.x >= gridDim.x / 2) __builtin_amdgcn_s_setprio(PRIO & 3);
    }
    __shared__ uint32_t rss_lds[RSS ? kRssTableWords : 1];
    __shared__ WaveLds lds[WPB];
    if constexpr (RSS) {
        for (int i = threadIdx.x; i < kRssTableWords; i += kWave * WPB) rss_lds[i] = kp.rss_tables[i];
        __syncthreads();
    }

    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t row = lane >> 4, rlane = lane & (kRow - 1);
    const uint32_t wib = threadIdx.x >> 6;
    const uint32_t wave = blockIdx.x * WPB + wib;
    const uint32_t nwaves = gridDim.x * WPB;
    WaveLds &wl = lds[wib];
    const uint32_t pass_pkts = nwaves * kWave;
    // packet index of lane l relative to the pass base
    auto map = [&](uint32_t l) -> uint32_t {
        return B == kWave ? wave * kWave + l : (l / B) * (nwaves * B) + wave * B + (l % B);
    };
    const uint32_t lane_off = map(lane);
    bool xskip_wave = false;
    if constexpr (XSKIP != 0) {
        const uint32_t xcc = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 1u;  // HW_REG_XCC_ID[0]
        xskip_wave = XSKIP > 0 ? xcc == 1u : xcc == 0u;
    }
    const uint64_t safe = (uint64_t)(uintptr_t)(MODE == kRxPtrs ? (const void *)kp.out
                                                               : (const void *)kp.buf);
    // the packet of this lane in pass g0, and whether the batch has it
    auto lane_pkt = [&](uint32_t g0, bool &live) -> uint32_t {
        live = g0 + lane_off < kp.n;
        return g0 + lane_off;
    };

    // ---------------- phase 0: descriptors (of the NEXT pass, prefetched) ---
    // The raw descriptor fields are loaded one pass ahead so that their
    // latency hides under the current pass's streaming.
    // COOP (B == 8, the unrolled chunk schedule: C2, C4, C5 and the tx fill):
    // the workgroup loads its descriptors together.  A lane's
    // own descriptors lie 8 x 8 B per wave-run at a stride of 8 * nwaves
    // packets, i.e. eight scattered 64 B pieces per wave and pass; the WPB
    // waves of a workgroup own adjacent runs, so for each of the eight runs
    // the workgroup's descriptors are one contiguous 8 * WPB-packet piece
    // (256 B at WPB 4).  Each lane loads one entry of those pieces (one
    // coalesced load per wave), and `exchange` hands every entry to the lane
    // that owns its packet through LDS.  Scattered 64 B pieces cost the frame
    // stream ~7 us of C2's 1.6 GB (tools/rx_variants lad_B8_desc 228.3 vs
    // lad_B8_descwg 220.6 us, the arithmetic-address walk 221.8): each one
    // opens a DRAM row for 64 B; the kernel gains 1.7-2.6 us.  Not for the
    // size-sorted schedule (2.7-2.8 us slower: the barrier holds back its
    // desynchronised waves; it takes runs of 16 instead, mtcp_gpu.hip), nor
    // for pointer bursts (the RSS pointer schedule would spill).
    constexpr bool kCoop = B == 8 && MODE != kRxPtrs && SCHED == 3 && COOP;
    __shared__ uint64_t coop_a[kCoop ? 2 : 1][kCoop ? WPB * kWave : 1];   // double-buffered by pass
    uint32_t coop_buf = 0;

    // entry (run cj, packet cidx of the workgroup's piece) is this lane's to
    // load; it belongs to lane cj * 8 + cidx % 8 of wave cidx / 8
    const uint32_t cq = wib * kWave + lane, cj = cq / (8 * WPB), cidx = cq % (8 * WPB);
    const uint32_t coop_off = cj * (nwaves * 8) + blockIdx.x * (8 * WPB) + cidx;   // from the pass base
    const uint32_t coop_slot = (cidx / 8) * kWave + cj * 8 + (cidx % 8);
    uint64_t raw_a = 0;     // chunk mode: the 8-byte descriptor; ptrs mode: the pointer
    uint32_t raw_b = 0;     // ptrs mode: the length
    uint64_t cv_a = 0;      // COOP: the entry this lane loaded for the workgroup
    auto fetch = [&](uint32_t g0) {
        if constexpr (kCoop) {
            const uint32_t kk = g0 + coop_off;
            if (kk < kp.n) cv_a = *reinterpret_cast<const uint64_t *>(kp.desc + kk);
            return;
        }
        bool live;
        const uint32_t k = lane_pkt(g0, live);
        if (live) {
            if constexpr (MODE == kRxPtrs) {
                raw_a = (uint64_t)(uintptr_t)kp.ptrs[k];
                raw_b = kp.lens[k];
            } else {
                raw_a = *reinterpret_cast<const uint64_t *>(kp.desc + k);
            }
        }
    };
    // COOP: the fetched entries to their owners (raw_a), once per
    // pass before its first decode.  Every wave of the workgroup calls it the
    // same number of times: before the pass loop, and where a next pass
    // exists (has_next is the same for the whole grid).
    // Two buffers, alternating: the entries of exchange k are read before
    // the barrier of exchange k + 1, so buffer k & 1 is free again at
    // exchange k + 2 and one barrier per pass suffices.
    auto exchange = [&]() {
        if constexpr (kCoop) {
            coop_a[coop_buf][coop_slot] = cv_a;
            __syncthreads();
            raw_a = coop_a[coop_buf][wib * kWave + lane];
            coop_buf ^= 1u;
        }
    };
    auto decode = [&](uint32_t g0) -> Frame {
        Frame f;
        bool live;
        (void)lane_pkt(g0, live);
        f.live = live;
        if constexpr (XSKIP != 0) {
            if (xskip_wave && g0 + pass_pkts >= kp.n && lane >= (uint32_t)(kWave - (XSKIP > 0 ? XSKIP : -XSKIP)))
                f.live = false;
        }
        f.p = safe;
        f.L = 0;
        f.ok = false;
        if (f.live) {
            if constexpr (MODE == kRxPtrs) {
                f.L = raw_b;
                f.ok = raw_a != 0 && (raw_a & 1) == 0;      // any even start
                // rows with nothing to read still issue (clamped) loads: keep
                // their address on always-mapped memory
                if (f.ok) f.p = raw_a;
            } else {
                const uint32_t off = (uint32_t)raw_a;
                f.L = (uint32_t)(raw_a >> 32) & 0xFFFFu;
                const int64_t pos = (int64_t)((uint64_t)off << kp.off_shift) - kp.base_sub;
                f.ok = pos >= 0 && (pos & 1) == 0 && (uint64_t)pos + f.L <= kp.buf_len;
                if (f.ok) f.p = safe + (uint64_t)pos;
            }
        }
        f.p16 = f.p & ~15ull;
        f.nch = f.ok && f.L ? (uint32_t)((((f.p + f.L + 15) & ~15ull) - f.p16) >> 4) : 0u;
        const int src = 4 * (int)rlane + (int)row;
        f.r_nch = shfl32(f.nch, src);
        f.r_lo = shfl32((uint32_t)f.p16, src);
        f.r_hi = shfl32((uint32_t)(f.p16 >> 32), src);
        return f;
    };

    // ---------------- phase 1 building blocks -----------------------------
    // LALIGN: a frame that needs more than one trip is streamed from the
    // start of its first 128 B line: the trip's base moves back by the
    // `skip` = (p16 & 127) / 16 chunks before the frame (same line, same page;
    // masked out of the sum), so that every later trip starts on a line.  A
    // trip boundary inside a line would fetch that line twice, once per trip
    // (C5: 9024 B slots put every other frame off the line grid).
    auto line_align = [&](Trip &t) {
        t.skip = 0;
        if constexpr (LALIGN) {
            if (t.nj > (uint32_t)(U * kRow)) {
                t.skip = (uint32_t)((t.base & 127) >> 4);
                t.base -= 16ull * t.skip;
                t.nj += t.skip;
            }
        }
    };
    auto enter_round = [&](const Frame &f, Trip &t, int ii) {
        t.i = ii;
        t.col = 4 * (uint32_t)ii + row;
        t.nj = row_bcast(f.r_nch, ii);
        t.base = ((uint64_t)row_bcast(f.r_hi, ii) << 32) | row_bcast(f.r_lo, ii);
        t.c0 = 0;
        line_align(t);
        if constexpr (REV) {
            // odd rows walk their frame's trips last to first, so that the
            // line a frame shares with its neighbour in the next row is read
            // by both rows in the same step (3 of every 4 frame boundaries)
            t.k = 0;
            t.ntrip = (t.nj + U * kRow - 1) / (U * kRow);
            if ((row & 1) && t.ntrip > 1) t.c0 = (t.ntrip - 1) * (U * kRow);
        }
    };
    auto rev_step = [&](Trip &t) {     // REV: the next trip of each row
        ++t.k;
        t.c0 = t.k >= t.ntrip ? t.nj                           // done: every lane masked
               : (row & 1) ? (t.ntrip - 1 - t.k) * (U * kRow) : t.k * (U * kRow);
    };
    // next trip with work; false (nj = 0, base kept valid) when the pass is done
    auto advance = [&](const Frame &f, Trip &t) -> bool {
        if (__ballot(t.c0 + U * kRow < t.nj)) {
            t.c0 += U * kRow;
            return true;
        }
        for (int ii = t.i + 1; ii < kWave / 4; ++ii) {
            enter_round(f, t, ii);
            if (__ballot(t.nj != 0)) return true;
        }
        t.nj = 0;
        return false;
    };
    auto first_trip = [&](const Frame &f, Trip &t) -> bool {
        enter_round(f, t, 0);
        return __ballot(t.nj != 0) || advance(f, t);
    };
    auto issue = [&](const Trip &t, v4u (&x)[U]) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = t.c0 + u * kRow + rlane;
            const uint32_t cc = c < t.nj ? c : (t.nj ? t.nj - 1 : 0u);   // clamp: no exec mask
            x[u] = NT ? gload_nt(t.base + 16ull * cc) : gload(t.base + 16ull * cc);
        }
    };
    auto consume = [&](const Trip &t, const v4u (&x)[U], uint32_t &acc) {
        const uint32_t j = t.col;
        const uint32_t c_hd = rlane - t.skip;                        // frame chunk of x[0]
        if (ABL < 2 && t.c0 == 0 && c_hd < kSlotChunks - 1) {        // first trip: raw chunks 0..6
            uint32_t *d = wl.hd + 4 * c_hd * kHdStride + j;
            d[0] = x[0].x; d[kHdStride] = x[0].y;
            d[2 * kHdStride] = x[0].z; d[3 * kHdStride] = x[0].w;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t c = t.c0 + u * kRow + rlane;
            const uint32_t s = halves4(x[u], 0u);
            acc += (ABL >= 3 || c - t.skip < t.nj - t.skip) ? s : 0u;   // skip <= c < nj
            if (ABL < 2 && c == t.nj - 1) {                            // last chunk
                uint32_t *d = wl.hd + 4 * (kSlotChunks - 1) * kHdStride + j;
                d[0] = x[u].x; d[kHdStride] = x[u].y;
                d[2 * kHdStride] = x[u].z; d[3 * kHdStride] = x[u].w;
            }
        }
    };

    // ---- size-sorted schedule (SCHED == 4) ---------------------------------
    constexpr uint32_t kSmallChunks = 4;        // <= 64 B on the 16 B grid
    constexpr uint32_t kQuads = kWave / 4;      // small frames per round
    uint32_t pre_nL = 0, pre_nS = 0;            // class counts of the pre-issued pass
    // rank the wave's frames by class and publish {base, chunks, owner}
    auto prepare = [&](const Frame &fr, uint32_t &nL, uint32_t &nS) {
        const bool big = fr.nch > kSmallChunks, sml = fr.nch != 0 && !big;
        const uint64_t mb = __ballot(big), ms = __ballot(sml);
        nL = (uint32_t)__popcll(mb);
        nS = (uint32_t)__popcll(ms);
        const uint64_t below = (1ull << lane) - 1;
        const uint4 e = make_uint4((uint32_t)fr.p16, (uint32_t)(fr.p16 >> 32), fr.nch, lane);
        if (big) wl.info[__popcll(mb & below)] = e;
        if (sml) wl.info[kWave - 1 - __popcll(ms & below)] = e;
    };
    auto big_trip = [&](uint32_t nL, uint32_t ii, Trip &t) {
        const uint32_t r = 4 * ii + row;
        t.i = (int)ii;
        t.c0 = 0;
        t.skip = 0;
        t.nj = 0;
        t.base = safe;
        t.col = kWave;                            // scratch column
        if (r < nL) {
            const uint4 e = wl.info[r];
            t.base = ((uint64_t)e.y << 32) | e.x;
            t.nj = e.z;
            t.col = e.w;
            line_align(t);
        }
    };
    auto small_trip = [&](uint32_t nS, uint32_t ii, Trip &t) {
        const uint32_t r = kQuads * ii + (lane >> 2);
        t.i = (int)ii;
        t.c0 = 0;
        t.skip = 0;
        t.nj = 0;
        t.base = safe;
        t.col = kWave;
        if (r < nS) {
            const uint4 e = wl.info[kWave - 1 - r];
            t.base = ((uint64_t)e.y << 32) | e.x;
            t.nj = e.z;
            t.col = e.w;
        }
    };
    auto small_load = [&](const Trip &t) -> v4u {
        const uint32_t q = lane & 3;
        const uint32_t cc = q < t.nj ? q : (t.nj ? t.nj - 1 : 0u);
        // SCHED 5: small frames load through L2 normally (their 128 B line is
        // shared with a neighbour's edge, streamed in another round)
        return NT && SCHED < 5 ? gload_nt(t.base + 16ull * cc) : gload(t.base + 16ull * cc);
    };
    auto small_finish = [&](const Trip &t, const v4u &v) {
        const uint32_t q = lane & 3;
        uint32_t s4 = q < t.nj ? halves4(v, 0u) : 0u;
        s4 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s4, 0xB1, 0xF, 0xF, false);  // quad_perm 1,0,3,2
        s4 += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)s4, 0x4E, 0xF, 0xF, false);  // quad_perm 2,3,0,1
        if (q == 0) wl.sum[t.col] = s4;
        if (q < t.nj) {                                              // raw chunk q
            uint32_t *d = wl.hd + 4 * q * kHdStride + t.col;
            d[0] = v.x; d[kHdStride] = v.y; d[2 * kHdStride] = v.z; d[3 * kHdStride] = v.w;
        }
        if (q + 1 == t.nj) {                                         // last chunk
            uint32_t *d = wl.hd + 4 * (kSlotChunks - 1) * kHdStride + t.col;
            d[0] = v.x; d[kHdStride] = v.y; d[2 * kHdStride] = v.z; d[3 * kHdStride] = v.w;
        }
    };

    constexpr int kDefer = MODE == kTxChunk ? 0 : DEFER;
    // record dwords stored per packet (RW) and held per packet (HW: the
    // compact record also holds its flow bin)
    constexpr int RW = CMP ? 4 : 10, HW = CMP ? 5 : 10;
    uint32_t keep[kDefer > 0 ? kDefer : 1][HW];   // keep[q]: the record of q passes ago
    uint32_t held = 0;                            // passes in keep[] (wave-uniform)
    uint32_t last_g0 = 0;                         // pass base of keep[0]
    uint8_t *const out_b = reinterpret_cast<uint8_t *>(kp.out);
    // Store the held records (lane k's record of pass last_g0 - q*pass_pkts).
    // Each pass's 64 records go through this wave's LDS so that the stores
    // are 16 B pieces of the contiguous runs of B packets (B*RW*4 bytes each):
    // measured 8 us faster on C2 than every lane storing its own 40 B.
    auto flush = [&]() {
        if constexpr (kDefer > 0) {
            static_assert(B % 2 == 0, "16 B pieces need runs of an even number of records");
            constexpr uint32_t kRunDw = B * RW, kRunPieces = kRunDw / 4;
            uint32_t *stg = reinterpret_cast<uint32_t *>(&wl.hd[0]);
#pragma unroll
            for (int q = 0; q < kDefer; ++q) {
                if ((uint32_t)q < held) {
                    const uint32_t gq = last_g0 - (uint32_t)q * pass_pkts;
                    uint2 *st = reinterpret_cast<uint2 *>(stg) + lane * (RW / 2);
#pragma unroll
                    for (int i = 0; i < RW / 2; ++i) st[i] = make_uint2(keep[q][2 * i], keep[q][2 * i + 1]);
#pragma unroll
                    for (uint32_t pc = lane; pc < kWave * RW / 4; pc += kWave) {
                        const uint32_t run = pc / kRunPieces, w = pc % kRunPieces;
                        const uint32_t first = gq + map(run * B);      // runs: B consecutive packets
                        const uint32_t r0 = first + (4 * w) / RW, r1 = first + (4 * w + 2) / RW;
                        const uint4 v = *reinterpret_cast<const uint4 *>(stg + run * kRunDw + 4 * w);
                        uint8_t *dst = out_b + (uint64_t)first * (4 * RW) + 16 * w;
                        if (r1 < kp.n) {
                            *reinterpret_cast<uint4 *>(dst) = v;
                        } else if (r0 < kp.n) {                        // tail: half a piece
                            *reinterpret_cast<uint2 *>(dst) = make_uint2(v.x, v.y);
                        }
                    }
                    // f3 fused: the flow-table bin of each held record (40 B:
                    // computed from the record itself, no register held for
                    // it; 16 B: held beside it), stored in runs of B packets
                    if (kp.bins) {
                        bool live;
                        const uint32_t rec = lane_pkt(gq, live);
                        if (live)
                            kp.bins[rec] = CMP ? keep[q][HW - 1]
                                               : flow_bin(keep[q][0], keep[q][1], keep[q][2], keep[q][9] & 0xFFu);
                    }
                }
            }
            held = 0;
        }
    };

    // hold this pass's record (flushing first when the buffer is full)
    auto push = [&](const uint32_t (&r)[HW], uint32_t g0) {
        if constexpr (kDefer > 0) {
            if (held == (uint32_t)kDefer) flush();
#pragma unroll
            for (int q = kDefer - 1; q > 0; --q)
#pragma unroll
                for (int i = 0; i < HW; ++i) keep[q][i] = keep[q - 1][i];
#pragma unroll
            for (int i = 0; i < HW; ++i) keep[0][i] = r[i];
            last_g0 = g0;
            ++held;
        }
    };

    // tx fill: the two check fields of each frame (iph->check at byte 24,
    // tcph->check at T + 16) are held for up to kTxDefer passes and written
    // together at the end: sub-dword stores into the frames interleaved with
    // the read stream cost like the rx records' per-pass stores.
    constexpr int kTxDefer = MODE == kTxChunk && DEFER > 0 ? DEFER : 0;
    uint32_t tkeep[kTxDefer > 0 ? kTxDefer : 1][4];
    uint32_t tx_held = 0;                         // wave-uniform
    auto tx_write = [&](const uint32_t (&w)[4]) {
        if (w[3]) {
            uint16_t *q16 = reinterpret_cast<uint16_t *>(((uint64_t)w[1] << 32) | w[0]);
            q16[12] = (uint16_t)w[2];                                // iph->check (byte 24)
            q16[(w[3] + 16) >> 1] = (uint16_t)(w[2] >> 16);          // tcph->check (tcp_out.c:329)
        }
    };
    auto tx_flush = [&]() {
        if constexpr (kTxDefer > 0) {
#pragma unroll
            for (int q = 0; q < kTxDefer; ++q)
                if ((uint32_t)q < tx_held) tx_write(tkeep[q]);
            tx_held = 0;
        }
    };
    auto tx_push = [&](const uint32_t (&w)[4]) {
        if constexpr (kTxDefer > 0) {
            if (tx_held == (uint32_t)kTxDefer) tx_flush();
#pragma unroll
            for (int q = kTxDefer - 1; q > 0; --q)
#pragma unroll
                for (int i = 0; i < 4; ++i) tkeep[q][i] = tkeep[q - 1][i];
#pragma unroll
            for (int i = 0; i < 4; ++i) tkeep[0][i] = w[i];
            ++tx_held;
        }
    };

    fetch(0);
    exchange();
    v4u X[U], Y[U];
    Trip pre;                    // next pass's first trip, already issued into X
    bool have_pre = false;
    Trip sa, sb;                 // SCHED >= 5: the first two small rounds
    v4u va, vb;
    bool have_pre_small = false; // SCHED 6: already issued into va, vb
    for (uint32_t g0 = 0; g0 < kp.n; g0 += pass_pkts) {
        if constexpr ((PRIO & 4) != 0) {
            if (g0 == 4 * pass_pkts) __builtin_amdgcn_s_setprio(0);
        }
        const Frame f = decode(g0);
        if (!__ballot(f.live)) break;
        fetch(g0 + pass_pkts);                                     // next pass's descriptors
        const uint32_t k = g0 + lane_off;
        const bool live = f.live, desc_ok = f.ok;
        const uint64_t p = f.p;
        const uint32_t L = f.L, nch = f.nch;
        const bool has_next = g0 + pass_pkts < kp.n;

        // ---------------- phase 1: four frames per wave-instruction ---------
        if constexpr (SCHED >= 4) {
            // Size-sorted rounds.  The wave's frames are ranked by class:
            // large (> kSmallChunks chunks) frames stream four per round as
            // above (a 16-lane row each, U loads per lane), small ones
            // sixteen per round (a 4-lane quad each, one load per lane);
            // empty ones are skipped.  A mix of 64 B and 1500 B frames then
            // needs ~10 round trips per pass instead of 16, and no round
            // waits on a large frame with mostly small ones.  The rank ->
            // frame table (base, chunk count, owner lane) lives in LDS; each
            // lane reads its row's / quad's entry (LDS broadcast).  Large
            // rounds are double-buffered (X/Y).
            uint32_t nL, nS;
            if (!have_pre) prepare(f, nL, nS);
            else nL = pre_nL, nS = pre_nS;
            const uint32_t RL = (nL + 3) / 4, RS = (nS + kQuads - 1) / kQuads;
            uint32_t acc = 0;
            auto finish_big = [&](Trip &t, const v4u (&cb)[U]) {
                consume(t, cb, acc);
                while (__ballot(t.c0 + U * kRow < t.nj)) {
                    t.c0 += U * kRow;
                    v4u Z[U];
                    issue(t, Z);
                    consume(t, Z, acc);
                }
                acc = row_sum(acc);
                if (rlane == kRow - 1) wl.sum[t.col] = acc;
                acc = 0;
            };
            // SCHED 5: the first two small rounds go out with the first large
            // round, before the large frames around them stream.  SCHED 6:
            // they go out even earlier, with the pre-issued first large round
            // at the end of the previous pass (below).
            if constexpr (SCHED >= 5) {
                if (have_pre_small) {
                    // issued at the end of the previous pass
                } else if (RL > 0 && !have_pre) {
                    Trip t0;
                    big_trip(nL, 0, t0);
                    issue(t0, X);
                    pre = t0;
                    have_pre = true;
                }
                if (!have_pre_small) {
                    small_trip(nS, 0, sa);
                    small_trip(nS, 1, sb);
                    va = small_load(sa);
                    vb = small_load(sb);
                }
                have_pre_small = false;
            }
            if (RL > 0) {
                Trip cur, nxt;
                if (have_pre) {
                    cur = pre;
                } else {
                    big_trip(nL, 0, cur);
                    issue(cur, X);
                }
                for (uint32_t i = 0; i < RL; i += 2) {
                    if (i + 1 < RL) {                 // round i+1 goes out into Y
                        big_trip(nL, i + 1, nxt);
                        issue(nxt, Y);
                    }
                    finish_big(cur, X);
                    if (i + 1 >= RL) break;
                    if (i + 2 < RL) {                 // round i+2 into X
                        big_trip(nL, i + 2, cur);
                        issue(cur, X);
                    }
                    finish_big(nxt, Y);
                }
            }
            have_pre = false;
            uint32_t s0 = 0;
            if constexpr (SCHED >= 5) {
                if (RS > 0) {
                    small_finish(sa, va);
                    small_finish(sb, vb);
                }
                s0 = 2;
            }
            // small rounds, two at a time (two loads in flight per lane)
            for (uint32_t i = s0; i < RS; i += 2) {
                Trip a, b;
                small_trip(nS, i, a);
                small_trip(nS, i + 1, b);
                const v4u va = small_load(a), vb = small_load(b);
                small_finish(a, va);
                small_finish(b, vb);
            }
            if (has_next) {                           // the next pass's first large round
                exchange();
                const Frame fn = decode(g0 + pass_pkts);
                prepare(fn, pre_nL, pre_nS);
                if constexpr (SCHED == 6) {
                    small_trip(pre_nS, 0, sa);
                    small_trip(pre_nS, 1, sb);
                    va = small_load(sa);
                    vb = small_load(sb);
                    have_pre_small = true;
                }
                if (pre_nL) {
                    big_trip(pre_nL, 0, pre);
                    issue(pre, X);
                    have_pre = true;
                }
            }
        } else if constexpr (SCHED == 3) {
            // The 16 rounds unrolled (constant DPP broadcasts) but single-
            // buffered: each round's loads are issued, then consumed, like
            // the read-only walk of tools/rx_variants (lad_B8_desc); only the
            // next pass's first trip is issued before phase 2.
            uint32_t acc = 0;
            static_for<0, kWave / 4>([&](auto I) {
                constexpr int i = decltype(I)::value;
                Trip t;
                enter_round(f, t, i);
                if (i > 0 || !have_pre) issue(t, X);
                consume(t, X, acc);
                if constexpr (REV) {
                    while (__ballot(t.k + 1 < t.ntrip)) {
                        rev_step(t);
                        issue(t, X);
                        consume(t, X, acc);
                    }
                } else {
                    while (__ballot(t.c0 + U * kRow < t.nj)) {
                        t.c0 += U * kRow;
                        issue(t, X);
                        consume(t, X, acc);
                    }
                }
                acc = row_sum(acc);
                if (rlane == kRow - 1) wl.sum[4 * i + (int)row] = acc;
                acc = 0;
            });
            have_pre = false;
            if (has_next) {
                exchange();
                const Frame fn = decode(g0 + pass_pkts);
                Trip n;
                enter_round(fn, n, 0);
                issue(n, X);
                have_pre = true;
            }
        } else {
            // SCHED 0, rolled: one trip at a time through the pass's rounds;
            // only the next pass's first trip is issued early (before this
            // pass's phase 2).
            Trip cur;
            bool have;
            if (have_pre) {
                cur = pre;
                have = true;
            } else {
                have = first_trip(f, cur);
                issue(cur, X);
            }
            have_pre = false;
            uint32_t acc = 0;
            while (have) {
                Trip n = cur;
                const bool more = advance(f, n);
                consume(cur, X, acc);
                if (!more || n.i != cur.i) {                        // frame sums -> LDS
                    acc = row_sum(acc);
                    if (rlane == kRow - 1) wl.sum[4 * cur.i + (int)row] = acc;
                    acc = 0;
                }
                if (!more) break;
                issue(n, X);
                cur = n;
            }
            if (has_next) {
                Trip n;
                exchange();
                const Frame fn = decode(g0 + pass_pkts);
                if (__ballot(fn.live) && first_trip(fn, n)) {
                    issue(n, X);
                    pre = n;
                    have_pre = true;
                }
            }
        }

        if constexpr (ABL >= 1) {
            if constexpr (kDefer > 0) {
                uint32_t r[HW] = {};
                r[0] = wl.sum[lane];
                push(r, g0);
            } else if (live && wl.sum[lane] == 0x12345678u) {   // profiling: no stores
                kp.out[k].saddr = wl.sum[lane];
            }
            continue;
        }
        // ---------------- phase 2: per-lane parse and finish ---------------
        const Pkt pk = parse_finish<MODE, kHdStride>(wl.hd + lane, wl.sum[lane], p, L, nch, desc_ok);
        uint32_t rss_hash = 0, rss_queue = 0;
        if constexpr (RSS) {
            if (pk.tcp_entry) {
                rss_hash = toeplitz_tables(rss_lds, pk.saddr, pk.daddr, pk.ports);
                rss_queue = rss_core(rss_hash, kp.rss_nq, kp.rss_endian);
            }
        }

        if constexpr (MODE == kTxChunk) {
            uint32_t fill[4] = {0, 0, 0, 0};                        // {p lo, p hi, checks, T}
            if (live && pk.need_sum) {
                const uint32_t ipc = fold_csum(pk.s_ip - pk.ip_check);   // ip_out.c:145,164
                fill[0] = (uint32_t)p;
                fill[1] = (uint32_t)(p >> 32);
                fill[2] = ipc | (pk.tcp_csum << 16);
                fill[3] = pk.T;
                if (kp.fill_count) atomicAdd(kp.fill_count, 1u);
            }
            if constexpr (kTxDefer > 0) {
                tx_push(fill);
            } else {
                tx_write(fill);
            }
        } else {
            uint32_t r[HW];
            if constexpr (CMP) {
                uint32_t c[4];
                pack_compact(pk, rss_hash, rss_queue, c);
#pragma unroll
                for (int i = 0; i < 4; ++i) r[i] = c[i];
                r[4] = kp.bins ? flow_bin(pk.saddr, pk.daddr, pk.ports, pk.verdict) : 0u;
            } else {
                pack_record(pk, rss_hash, rss_queue, r);
            }
            if constexpr (kDefer > 0) {
                push(r, g0);
            } else {
                // stage the 64 records (64 x RW dwords) in this wave's LDS,
                // then store them as 8-byte pieces: lanes of one run of B
                // packets write one contiguous span of the output
                uint2 *st = reinterpret_cast<uint2 *>(wl.hd) + lane * (RW / 2);
#pragma unroll
                for (int i = 0; i < RW / 2; ++i) st[i] = make_uint2(r[2 * i], r[2 * i + 1]);
                const uint2 *src = reinterpret_cast<const uint2 *>(wl.hd);
#pragma unroll
                for (uint32_t i = 0; i < RW / 2; ++i) {
                    const uint32_t q = i * kWave + lane;      // 8-byte piece of record q / (RW / 2)
                    const uint32_t rec = g0 + map(q / (RW / 2));
                    if (rec < kp.n)
                        reinterpret_cast<uint2 *>(out_b + (uint64_t)rec * (4 * RW))[q % (RW / 2)] = src[q];
                }
                if (kp.bins && live)
                    kp.bins[k] = CMP ? r[HW - 1] : flow_bin(r[0], r[1], r[2], r[9] & 0xFFu);
            }
        }
    }
    flush();
    tx_flush();
    if constexpr (STAMP) {
        __builtin_amdgcn_s_waitcnt(0);                 // the wave's stores have left
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) {
            uint32_t *st = kp.stamps + 4 * wave;
            st[0] = (uint32_t)t_start;
            st[1] = (uint32_t)t_end;
            st[2] = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20);   // HW_REG_XCC_ID[3:0]
            st[3] = (uint32_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
        }
    }
}

}  // namespace mg
