/*
 * mtcp_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement, in plain C, of mTCP's software (--disable-hwcsum)
 * per-packet rx/tx path.  It is the parity checker for the HIP kernels and
 * the "port" CPU baseline of bench.py.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product
 * (mtcp_amd/, libmtcp_gpu.so) never links or calls it.
 *
 * Parity of this restatement is pinned against golden vectors produced by
 * the reference's own code compiled from /root/reference
 * (oracle/ref/golden_gen.c, fixtures in tests/golden/) and against the
 * Microsoft Toeplitz known-answer vectors of util/rss.c:185-189.
 */
#ifndef MTCP_ORACLE_H
#define MTCP_ORACLE_H

#include <stdint.h>
#include "../include/mtcp_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* io_engine/include/ps.h:66-95 (x86 asm ip_fast_csum, restated). */
uint16_t oracle_ip_fast_csum(const void *iph, unsigned int ihl);

/* mtcp/src/tcp_util.c:157-190 (TCPCalcChecksum). */
uint16_t oracle_tcp_calc_checksum(const uint16_t *buf, uint16_t len,
                                  uint32_t saddr, uint32_t daddr);

/* mtcp/src/icmp.c:18-42 (ICMPChecksum; odd len: high byte taken as 0). */
uint16_t oracle_icmp_checksum(const uint8_t *icmph, int len);

/* util/rss.c:13-105 BuildKeyCache with the key as a parameter. */
void oracle_build_key_cache(const uint8_t key[40], uint32_t *cache, int cache_len);

/* util/rss.c:107-145 GetRSSHash over a prebuilt 96-entry key cache. */
uint32_t oracle_get_rss_hash(const uint32_t cache[96], uint32_t sip, uint32_t dip,
                             uint16_t sp, uint16_t dp);

/* util/rss.c:153-165 (endian_check = 1) / mtcp/src/rss.c:90-103. */
int oracle_get_rss_cpu_core(const uint32_t cache[96], uint32_t sip, uint32_t dip,
                            uint16_t sp, uint16_t dp, int num_queues,
                            int endian_check);

/* The key the reference ships active: 0x05 x 40 (util/rss.c:84-90). */
extern const uint8_t oracle_rss_key_0x05[40];
/* The Microsoft key (util/rss.c:73-82, #if 0 in the reference). */
extern const uint8_t oracle_rss_key_microsoft[40];

typedef struct oracle_rss_cfg {
    uint32_t cache[96];
    int num_queues;
    int endian_check;
} oracle_rss_cfg;

void oracle_rss_cfg_init(oracle_rss_cfg *cfg, const uint8_t key[40],
                         int num_queues, int endian_check);

/*
 * One frame through ProcessPacket (eth_in.c:9-56) -> ProcessIPv4Packet
 * (ip_in.c:15-62) -> head of ProcessTCPPacket (tcp_in.c:1138-1175).
 * rss may be NULL.  Returns the verdict (also stored in out->verdict).
 */
int oracle_rx_packet(const uint8_t *pkt, uint32_t len, const oracle_rss_cfg *rss,
                     mtcp_gpu_result *out);

/* A PSIO-style chunk (same descriptor rules as mtcp_gpu_rx_chunk). */
void oracle_rx_chunk(const uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc,
                     uint32_t n, uint32_t off_shift, const oracle_rss_cfg *rss,
                     mtcp_gpu_result *out);

/* tx fill (ip_out.c:94,164; tcp_out.c:211,329); returns frames written. */
uint32_t oracle_tx_fill(uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc,
                        uint32_t n, uint32_t off_shift);

/* Host mirror of the synthetic traffic generator (mtcp_gpu_pktgen.h). */
void oracle_pktgen(uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc,
                   uint32_t n, uint32_t off_shift, uint64_t seed,
                   uint64_t first_index);

/*
 * CPU baseline: the rx chain over a chunk on `nthreads` pthreads, each pinned
 * to one core (mtcp/src/core.c:1057, mtcp_core_affinitize) and owning a
 * contiguous shard of the packets (mTCP's share-nothing model).  Runs the
 * whole chunk `reps` times and returns the best wall time in seconds.
 */
double oracle_bench_rx(const uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc,
                       uint32_t n, uint32_t off_shift, const oracle_rss_cfg *rss,
                       mtcp_gpu_result *out, int nthreads, int reps);

/*
 * mtcp/src/tcp_stream.c:56-90 HashFlow (the #else branch: Jenkins
 * one-at-a-time over the 12 bytes saddr|daddr|sport|dport of a tcp_stream,
 * tcp_stream.h:163-166, read as x86 signed char), masked to NUM_BINS_FLOWS
 * (fhash.h:7).
 */
uint32_t oracle_hash_flow(const uint8_t key[12]);

/* The flow-table bin of each rx result: HashFlow of the stream key
 * ProcessTCPPacket looks up (tcp_in.c:1180-1186: saddr = iph->daddr,
 * sport = tcph->dest, daddr = iph->saddr, dport = tcph->source) for TCP_OK
 * packets, MTCP_GPU_FLOW_NONE for the rest. */
void oracle_flow_bins(const mtcp_gpu_result *res, uint32_t n, uint32_t *bins);

/*
 * mtcp/src/addr_pool.c:103-180 CreateAddressPoolPerCore's search: in
 * (address, port) order, the (saddr, sport) pairs, network order, whose
 * GetRSSCPUCore(daddr_h, saddr_h, dport_h, sport_h, nq, endian)
 * (mtcp/src/rss.c:90-103) is `core`; at most
 * num_addr * (MAX_PORT - MIN_PORT) / num_queues of them (addr_pool.c:129).
 * Writes up to max_out entries; returns the number the reference keeps.
 */
uint32_t oracle_addr_pool_search(const uint8_t key[40], int core, int num_queues,
                                 uint32_t saddr_base, int num_addr, uint32_t daddr,
                                 uint16_t dport, int endian_check,
                                 mtcp_gpu_addr_entry *out, uint32_t max_out);

#ifdef __cplusplus
}
#endif
#endif
