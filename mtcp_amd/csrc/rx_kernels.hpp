// rx_kernels.hpp — gfx950 (CDNA4) kernels for mTCP's software per-packet path:
// the rx chain ProcessPacket -> ProcessIPv4Packet -> head of ProcessTCPPacket
// (mtcp/src/eth_in.c:9-56, ip_in.c:15-62, tcp_in.c:1138-1175) with its
// ip_fast_csum (io_engine/include/ps.h:66-95) and TCPCalcChecksum
// (mtcp/src/tcp_util.c:157-190), the Toeplitz RSS hash (util/rss.c:107-165),
// and the tx checksum fill (ip_out.c:94,164; tcp_out.c:211,329).
//
// Work decomposition (one 64-lane wave per group of 64 packets):
//   phase 0  lane k parses packet k of the group: descriptor, the header
//            dwords it needs (L1/L2-resident gathers), verdict up to the TCP
//            checksum, and the TCP segment [T, 14+tot_len) as a range of
//            16-byte aligned chunks.
//   phase 1  the WHOLE wave streams each packet's chunks in turn, 1 KiB per
//            wave-instruction (global_load_dwordx4, lane l -> chunk l), adds
//            the 16-bit halves with v_sad_u16 and reduces across the wave
//            with DPP; two packets are in flight at once.
//   phase 2  lane k removes the bytes the aligned chunks over-cover (the
//            <= 14 header bytes before T and the <= 15 bytes after the
//            segment), adds the pseudo header, folds, finishes the verdict,
//            hashes the 4-tuple through 12 byte tables in LDS, and stores its
//            40-byte record.
// Exactness: the reference sums little-endian u16 words of the segment into
// a u32 (no overflow for any u16 length).  The segment starts at an even
// address, so its words are exactly the 16-bit halves of the aligned dwords
// that hold it; every partial sum here is an exact integer below 2^31 and
// the final fold is the reference's own two-step fold.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mtcp_gpu.h"

namespace mg {

constexpr int kWave = 64;
constexpr int kBlock = 256;
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr int kRssTableWords = 12 * 256;

enum Mode : int { kRxChunk = 0, kRxPtrs = 1, kTxChunk = 2 };

struct KParams {
    const uint8_t *buf;            // chunk base (chunk modes)
    uint64_t buf_len;              // readable bytes from buf (multiple of 16)
    int64_t base_sub;              // subtracted from every descriptor byte offset
    const mtcp_gpu_desc *desc;
    const uint8_t *const *ptrs;    // pointer mode
    const uint16_t *lens;
    uint32_t n;
    uint32_t off_shift;
    mtcp_gpu_result *out;
    const uint32_t *rss_tables;    // 12 x 256 Toeplitz byte tables
    uint32_t rss_nq;
    uint32_t rss_endian;
    uint32_t *fill_count;          // tx fill: frames written (may be null)
};

__device__ __forceinline__ uint32_t bswap16(uint32_t v) {
    return ((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

// acc + lo16(d) + hi16(d) in one v_sad_u16
__device__ __forceinline__ uint32_t halves(uint32_t d, uint32_t acc) {
    return __builtin_amdgcn_sad_u16(d, 0u, acc);
}
__device__ __forceinline__ uint32_t halves4(const uint4 &v, uint32_t acc) {
    return halves(v.w, halves(v.z, halves(v.y, halves(v.x, acc))));
}

// The reference's fold (tcp_util.c:184-188), also ip_fast_csum's result for
// ihl >= 5 (ps.h:66-95; SURVEY §8 a2').
__device__ __forceinline__ uint32_t fold_csum(uint32_t s) {
    s = (s >> 16) + (s & 0xFFFFu);
    s += s >> 16;
    return (~s) & 0xFFFFu;
}

// Wave-wide u32 sum via DPP; the total is returned in every lane (SGPR).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, true);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false); // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false); // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
    uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
    uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// Sum of the halves of chunk windows [w0, ...) of one packet (jumbo tail).
__device__ __forceinline__ uint32_t sum_rest(const uint4 *base, uint32_t nch, uint32_t lane) {
    uint32_t acc = 0;
    for (uint32_t c0 = 2 * kWave; c0 < nch; c0 += 4 * kWave) {
        uint4 v0 = make_uint4(0, 0, 0, 0), v1 = v0, v2 = v0, v3 = v0;
        uint32_t c = c0 + lane;
        if (c < nch) v0 = base[c];
        if (c + kWave < nch) v1 = base[c + kWave];
        if (c + 2 * kWave < nch) v2 = base[c + 2 * kWave];
        if (c + 3 * kWave < nch) v3 = base[c + 3 * kWave];
        acc = halves4(v0, acc);
        acc = halves4(v1, acc);
        acc = halves4(v2, acc);
        acc = halves4(v3, acc);
    }
    return acc;
}

template <int MODE, bool RSS>
__global__ __launch_bounds__(kBlock) void rx_kernel(KParams kp) {
    __shared__ uint32_t rss_lds[RSS ? kRssTableWords : 1];
    if constexpr (RSS) {
        for (int i = threadIdx.x; i < kRssTableWords; i += kBlock) rss_lds[i] = kp.rss_tables[i];
        __syncthreads();
    }

    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wave = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const uint32_t nwaves = gridDim.x * kWavesPerBlock;
    const uint32_t ngroups = (kp.n + kWave - 1) / kWave;

    for (uint32_t g = wave; g < ngroups; g += nwaves) {
        const uint32_t k = g * kWave + lane;
        const bool live = k < kp.n;

        // ---------------- phase 0: per-lane parse -------------------------
        const uint8_t *pkt = nullptr;
        uint32_t L = 0;
        bool desc_ok = false;
        if (live) {
            if constexpr (MODE == kRxPtrs) {
                pkt = kp.ptrs[k];
                L = kp.lens[k];
                desc_ok = pkt != nullptr && (((uintptr_t)pkt) & 3) == 0;
            } else {
                const mtcp_gpu_desc d = kp.desc[k];
                const int64_t pos = (int64_t)((uint64_t)d.offset << kp.off_shift) - kp.base_sub;
                L = d.len;
                desc_ok = pos >= 0 && (pos & 3) == 0 && (uint64_t)pos + L <= kp.buf_len;
                pkt = kp.buf + (desc_ok ? pos : 0);
            }
        }
        const uint32_t *pw = reinterpret_cast<const uint32_t *>(pkt);
        // header dword at byte offset o (o % 4 == 0): only bytes < L are read
        auto ldw = [&](uint32_t o) -> uint32_t { return (desc_ok && o < L) ? pw[o >> 2] : 0u; };

        uint32_t verdict = MTCP_GPU_V_BAD_DESC;
        uint32_t eth_type = 0, ip_len = 0, ihl = 0, ihl_doff = 0, ip_csum = 0;
        uint32_t saddr = 0, daddr = 0, ports = 0, seq = 0, ack = 0, window = 0, flags = 0;
        uint32_t payload_len = 0, rss_hash = 0, rss_queue = 0;
        bool need_sum = false;   // TCP segment checksum pending
        uint32_t tcp_len = 0, T = 0, s_ip = 0, d0 = 0, d3 = 0, s_head = 0, tcheck = 0;

        uint32_t d[16];
#pragma unroll
        for (int j = 0; j < 6; ++j) d[j] = ldw(12 + 4 * j);
        d0 = d[0];
        d3 = d[3];
        if (desc_ok) {
            verdict = MTCP_GPU_V_TRUNCATED;
            if (L >= 14) {
                eth_type = bswap16(d0 & 0xFFFFu);                          // eth_in.c:13
                if (eth_type != 0x0800u) {
                    verdict = eth_type == 0x0806u ? MTCP_GPU_V_ARP : MTCP_GPU_V_ETH_OTHER;
                } else if (L >= 18) {
                    ip_len = bswap16(d[1] & 0xFFFFu);                      // ip_in.c:21
                    ihl = (d0 >> 16) & 0xFu;
                    ihl_doff = ihl;
                    const uint32_t ver = (d0 >> 20) & 0xFu;
                    if (MODE != kTxChunk && ip_len < 20) {
                        verdict = MTCP_GPU_V_IP_SHORT;                     // ip_in.c:25-26
                    } else if (L >= 14 + 4 * (ihl > 1 ? ihl : 1)) {
#pragma unroll
                        for (int j = 6; j < 16; ++j) d[j] = (j <= (int)ihl) ? ldw(12 + 4 * j) : 0u;
                        // ip_fast_csum: ihl <= 4 returns dword 0 as is (ps.h:72-73)
                        s_ip = d0 >> 16;
                        uint32_t lo_last = 0;
#pragma unroll
                        for (int j = 1; j < 16; ++j) {
                            if (j < (int)ihl) s_ip = halves(d[j], s_ip);
                            if (j == (int)ihl) lo_last = d[j] & 0xFFFFu;
                        }
                        s_ip += lo_last;
                        ip_csum = ihl <= 4 ? (d0 >> 16) : fold_csum(s_ip);
                        const uint32_t proto = d[2] >> 24;                 // ip_in.c:52
                        T = 14 + 4 * ihl;
                        bool tcp_entry = false;
                        if (MODE == kTxChunk) {
                            tcp_entry = ver == 4 && ihl >= 5 && proto == 6 && L >= T + 20;
                            verdict = MTCP_GPU_V_ETH_OTHER;
                        } else if (ip_csum != 0) {
                            verdict = MTCP_GPU_V_IP_CSUM_BAD;              // ip_in.c:35-36
                        } else if (ver != 4) {
                            verdict = MTCP_GPU_V_IP_VERSION;               // ip_in.c:47-50
                        } else if (proto == 1) {
                            verdict = MTCP_GPU_V_ICMP;
                        } else if (proto != 6) {
                            verdict = MTCP_GPU_V_IP_PROTO_OTHER;           // ip_in.c:57-59
                        } else if (L >= T + 16) {
                            tcp_entry = true;
                        }
                        if (tcp_entry) {
                            // tcp_in.c:1142-1149: tcph = iph + 4*ihl
                            const uint32_t e0 = ldw(T - 2), e1 = ldw(T + 2), e2 = ldw(T + 6);
                            const uint32_t e3 = ldw(T + 10), e4 = ldw(T + 14);
                            const uint32_t doff = (e3 >> 20) & 0xFu;
                            saddr = (d[3] >> 16) | (d[4] << 16);
                            daddr = (d[4] >> 16) | (d[5] << 16);
                            ports = (e0 >> 16) | (e1 << 16);               // sport | dport << 16
                            seq = bswap32((e1 >> 16) | (e2 << 16));
                            ack = bswap32((e2 >> 16) | (e3 << 16));
                            window = bswap16(e4 & 0xFFFFu);
                            flags = e3 >> 24;
                            tcheck = e4 >> 16;
                            ihl_doff = ihl | (doff << 4);
                            if constexpr (RSS) {
                                // util/rss.c:107-145 as 12 byte tables: the input
                                // bytes (sip, dip, sp, dp host order, MSB first)
                                // are saddr/daddr/ports in memory order.
                                uint32_t h = 0;
#pragma unroll
                                for (int b = 0; b < 4; ++b) {
                                    h ^= rss_lds[(b << 8) | ((saddr >> (8 * b)) & 0xFFu)];
                                    h ^= rss_lds[((4 + b) << 8) | ((daddr >> (8 * b)) & 0xFFu)];
                                    h ^= rss_lds[((8 + b) << 8) | ((ports >> (8 * b)) & 0xFFu)];
                                }
                                rss_hash = h;
                                // util/rss.c:153-165: off[m & 3] = {3,1,-1,-3} == m ^ 3
                                uint32_t m = h & 0x7Fu;
                                if (kp.rss_endian) m ^= 3u;
                                rss_queue = m % kp.rss_nq;
                            }
                            if (MODE == kTxChunk) {
                                if (doff >= 5 && ip_len >= 4 * (ihl + doff) && 14 + ip_len <= L) {
                                    need_sum = true;
                                    tcp_len = ip_len - 4 * ihl;
                                }
                            } else if (ip_len < ((ihl + doff) << 2)) {
                                verdict = MTCP_GPU_V_TCP_LEN_BAD;          // tcp_in.c:1155-1156
                            } else {
                                payload_len = ip_len - ((ihl + doff) << 2);   // tcp_in.c:1144
                                if (14 + ip_len <= L) {
                                    need_sum = true;
                                    tcp_len = ip_len - 4 * ihl;              // tcp_in.c:1166
                                }
                            }
                            if (need_sum) {
                                // header bytes [s16, pkt+T) the first chunk over-covers
                                const uint32_t hs = (uint32_t)(((uintptr_t)pkt + T) & 15u);
                                const uint32_t hstart = T - hs;
                                uint32_t sh = 0, lo2 = 0;
#pragma unroll
                                for (int j = 1; j < 16; ++j) {
                                    if (j < (int)ihl && 12 + 4 * j >= (int)hstart) sh = halves(d[j], sh);
                                    if (j == (int)ihl) lo2 = d[j] & 0xFFFFu;
                                }
                                s_head = sh + lo2;
                            }
                        }
                    }
                }
            }
        }

        // chunk range of the TCP segment [pkt+T, pkt+14+ip_len)
        uint64_t s16 = 0;
        uint32_t nch = 0;
        if (need_sum) {
            const uint64_t s = (uint64_t)(uintptr_t)pkt + T;
            const uint64_t e = (uint64_t)(uintptr_t)pkt + 14 + ip_len;
            s16 = s & ~15ull;
            nch = (uint32_t)((((e + 15) & ~15ull) - s16) >> 4);
        }

        // ---------------- phase 1: wave-wide segment sums -----------------
        uint32_t s_chunks = 0;
        const uint64_t any = __ballot(nch != 0);
        if (any) {
            for (int j = 0; j < kWave; j += 2) {
                if (((any >> j) & 3ull) == 0) continue;
                const uint4 *ba = reinterpret_cast<const uint4 *>(readlane64(s16, j));
                const uint4 *bb = reinterpret_cast<const uint4 *>(readlane64(s16, j + 1));
                const uint32_t na = (uint32_t)__builtin_amdgcn_readlane((int)nch, j);
                const uint32_t nb = (uint32_t)__builtin_amdgcn_readlane((int)nch, j + 1);
                uint4 a0 = make_uint4(0, 0, 0, 0), a1 = a0, b0 = a0, b1 = a0;
                if (lane < na) a0 = ba[lane];
                if (lane + kWave < na) a1 = ba[lane + kWave];
                if (lane < nb) b0 = bb[lane];
                if (lane + kWave < nb) b1 = bb[lane + kWave];
                uint32_t acc_a = halves4(a1, halves4(a0, 0u));
                uint32_t acc_b = halves4(b1, halves4(b0, 0u));
                if (na > 2 * kWave) acc_a += sum_rest(ba, na, lane);
                if (nb > 2 * kWave) acc_b += sum_rest(bb, nb, lane);
                const uint32_t ta = wave_sum(acc_a);
                const uint32_t tb = wave_sum(acc_b);
                if (lane == (uint32_t)j) s_chunks = ta;
                if (lane == (uint32_t)j + 1) s_chunks = tb;
            }
        }

        // ---------------- phase 2: finish per lane ------------------------
        uint32_t tcp_csum = 0;
        if (need_sum) {
            // bytes after the segment inside its last aligned chunk
            const uint64_t e = (uint64_t)(uintptr_t)pkt + 14 + ip_len;
            const uint32_t te = (uint32_t)(e & 15u);
            uint32_t s_tail = 0;
            if (te) {
                const uint4 w = *reinterpret_cast<const uint4 *>(e & ~15ull);
                const uint32_t wv[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int drop = (int)te - 4 * i;   // low bytes inside the segment
                    const uint32_t m = drop <= 0 ? 0xFFFFFFFFu : drop >= 4 ? 0u : (0xFFFFFFFFu << (8 * drop));
                    s_tail = halves(wv[i] & m, s_tail);
                }
            }
            uint32_t s = s_chunks - s_head - s_tail;               // exact segment sum
            if (MODE == kTxChunk) s -= tcheck;                     // computed with check = 0
            s += (saddr & 0xFFFFu) + (saddr >> 16);                // tcp_util.c:179-182
            s += (daddr & 0xFFFFu) + (daddr >> 16);
            s += bswap16(tcp_len);
            s += 0x0600u;                                          // htons(IPPROTO_TCP)
            tcp_csum = fold_csum(s);
            if (MODE != kTxChunk)
                verdict = tcp_csum ? MTCP_GPU_V_TCP_CSUM_BAD : MTCP_GPU_V_TCP_OK;   // tcp_in.c:1167-1173
        }

        if (!live) continue;
        if constexpr (MODE == kTxChunk) {
            if (need_sum) {
                const uint32_t ipc = fold_csum(s_ip - (d3 & 0xFFFFu));   // ip_out.c:145,164
                uint16_t *p16 = reinterpret_cast<uint16_t *>(const_cast<uint8_t *>(pkt));
                p16[12] = (uint16_t)ipc;                              // iph->check (byte 24)
                p16[(T + 16) >> 1] = (uint16_t)tcp_csum;              // tcph->check (tcp_out.c:329)
                if (kp.fill_count) atomicAdd(kp.fill_count, 1u);
            }
        } else {
            uint2 *o = reinterpret_cast<uint2 *>(kp.out + k);
            o[0] = make_uint2(saddr, daddr);
            o[1] = make_uint2(ports, seq);
            o[2] = make_uint2(ack, window | (ip_len << 16));
            o[3] = make_uint2(ip_csum | (tcp_csum << 16), rss_hash);
            o[4] = make_uint2(payload_len | (ihl_doff << 16) | (flags << 24),
                              verdict | (rss_queue << 8) | (eth_type << 16));
        }
    }
}

}  // namespace mg
