// rx_wave.hpp — one wavefront per packet: the shape BASELINE.json's north
// star names, dispatched for small batches (mtcp_gpu.hip kWaveUpToPkts).
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
//   phase 2  parse_finish (rx_kernels.hpp, the same code rx_kernel runs per
//            lane) on the whole wave with wave-uniform operands: one
//            instruction stream per packet, LDS reads broadcast.  RSS is the
//            Toeplitz sum spread over the lanes — lane i owns input bits i and
//            64 + i, the key window of each bit comes straight from the key
//            words (BuildKeyCache, util/rss.c:13-105, without the table), an
//            XOR reduction finishes it — so no table is staged per workgroup.
//   stores   lanes 0..4 write the 40 B record as five 8 B pieces; the tx fill
//            writes its two 16-bit check fields from lane 0.
#pragma once

#include "rx_kernels.hpp"

namespace mg {

constexpr int kWaveLoads = 8;   // 16 B loads per lane per trip: 8 KiB of frame

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

template <int MODE, bool RSS>
__global__ __launch_bounds__(kBlock) void rx_wave_kernel(KParams kp) {
    __shared__ uint4 lds[kWavesPerBlock][kSlotChunks];     // chunks 0..6, then the last chunk
    const uint32_t lane = threadIdx.x & (kWave - 1);
    const uint32_t wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t k = blockIdx.x * kWavesPerBlock + wib;  // this wave's packet
    if (k >= kp.n) return;
    uint4 *hd = lds[wib];

    // ---- descriptor (wave-uniform) ------------------------------------------
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

    // ---- phase 1: the whole wave streams the frame ----------------------------
    uint32_t acc = 0;
    for (uint32_t c0 = 0; c0 < nch; c0 += kWave * kWaveLoads) {
        v4u x[kWaveLoads];
#pragma unroll
        for (int u = 0; u < kWaveLoads; ++u) {
            if (c0 + u * kWave < nch) {                    // wave-uniform
                const uint32_t c = c0 + u * kWave + lane;
                x[u] = gload_nt(p16 + 16ull * (c < nch ? c : nch - 1));
            }
        }
#pragma unroll
        for (int u = 0; u < kWaveLoads; ++u) {
            if (c0 + u * kWave < nch) {
                const uint32_t c = c0 + u * kWave + lane;
                if (c < nch) acc = halves4(x[u], acc);
                const uint4 v = make_uint4(x[u].x, x[u].y, x[u].z, x[u].w);
                if (u == 0 && c < kSlotChunks - 1) hd[c] = v;          // raw chunks 0..6
                if (c == nch - 1) hd[kSlotChunks - 1] = v;             // last chunk
            }
        }
    }
    acc = row_sum(acc);
    const uint32_t sum = (uint32_t)__builtin_amdgcn_readlane((int)acc, 15) +
                         (uint32_t)__builtin_amdgcn_readlane((int)acc, 31) +
                         (uint32_t)__builtin_amdgcn_readlane((int)acc, 47) +
                         (uint32_t)__builtin_amdgcn_readlane((int)acc, 63);
    __builtin_amdgcn_wave_barrier();

    // ---- phase 2: parse and finish, wave-uniform -------------------------------
    const Pkt pk = parse_finish<MODE, 1, true>(reinterpret_cast<const uint32_t *>(hd), sum, p, L, nch, ok);

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
        uint32_t r[10];
        pack_record(pk, rss_hash, rss_queue, r);
        if (lane < 5) {
            uint32_t x = r[0], y = r[1];
#pragma unroll
            for (int i = 1; i < 5; ++i)
                if (lane == (uint32_t)i) x = r[2 * i], y = r[2 * i + 1];
            reinterpret_cast<uint2 *>(kp.out + k)[lane] = make_uint2(x, y);
        }
        if (kp.bins && lane == 0) kp.bins[k] = flow_bin(r[0], r[1], r[2], r[9] & 0xFFu);
    }
}

}  // namespace mg
