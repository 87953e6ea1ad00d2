/*
 * mtcp_gpu_pktgen.h — synthetic traffic source on the GPU, for benchmarks
 * and tests (the role io_engine/samples/packet_generator/packet_generator.c
 * plays for PacketShader: build_packet :248-301, 64 B-aligned layout
 * :404-417).  Not part of the rx/tx offload itself.
 *
 * Frame i of a batch is a pure function of (seed, first_index + i, len), so
 * shards generated on different GPUs are byte-identical slices of one global
 * stream.  Spec (host mirror: oracle_pktgen in oracle/mtcp_oracle.c):
 *
 *   mix(z)     = splitmix64 finaliser
 *   s_i        = mix(seed ^ (i * 0xD1342543DE82EF95 + 0x632BE59BD9B4E019))
 *   r_i(k)     = mix(s_i + (k + 1) * 0x9E3779B97F4A7C15)
 *   byte p < L = byte (p & 7) of r_i(16 + p / 8); bytes [L, ALIGN(L, 64)) = 0
 *   if L >= 54, the headers are then written:
 *     Eth  dst = r0[0..5], src = r1[0..5], type 0x0800
 *     IPv4 45 00, tot_len = L - 14, id = r0[6..7], frag 0x4000 (DF, ip_out.c:140),
 *          ttl 64, proto 6, saddr = r2[0..3], daddr = r2[4..7]
 *     TCP  sport = r3[0..1], dport = r3[2..3], seq = r3[4..7], ack = r4[0..3],
 *          doff = 8 if L >= 66 and bit 32 of r4 (NOP NOP TS, tsval/tsecr = r5,
 *          mTCP's own option shape tcp_out.c:185-192) else 5,
 *          flags ACK (+PSH if bit 33 of r4), window = r4[5..6], urg 0
 *   checksums filled by the tx fill (mtcp_gpu_tx_fill semantics), then with
 *   c = r_i(6): if (c & 1023) == 0 one bit of the payload (or of the TCP
 *   segment when the payload is empty) is flipped, bit (c >> 10) mod its bits;
 *   if ((c >> 32) & 4095) == 0 one bit of bytes 14..33 is flipped,
 *   bit (c >> 44) mod 160.
 *
 * Descriptor offsets must be 64 B aligned (off_shift 6 gives that by
 * construction); frames whose padded extent leaves the buffer are skipped.
 */
#ifndef MTCP_GPU_PKTGEN_H
#define MTCP_GPU_PKTGEN_H

#include <stdint.h>
#include "mtcp_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

int mtcp_gpu_pktgen_dev(void *d_buf, uint64_t buf_len, const mtcp_gpu_desc *d_desc,
                        uint32_t n, uint32_t off_shift, uint64_t seed,
                        uint64_t first_index, void *stream);

#ifdef __cplusplus
}
#endif
#endif
