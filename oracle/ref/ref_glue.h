/*
 * ref_glue.h — TEST INFRASTRUCTURE ONLY: entry points of the oracle/_ref
 * build (the reference's own rx code compiled from /root/reference).
 */
#ifndef REF_GLUE_H
#define REF_GLUE_H
#include <stdint.h>

enum {
    REF_BR_TCP_OK = 0, REF_BR_ETH_OTHER = 1, REF_BR_ARP = 2, REF_BR_IP_SHORT = 3,
    REF_BR_IP_CSUM_BAD = 4, REF_BR_IP_VERSION = 5, REF_BR_ICMP = 6,
    REF_BR_IP_PROTO_OTHER = 7, REF_BR_TCP_LEN_BAD = 8, REF_BR_TCP_CSUM_BAD = 9,
    REF_BR_UNKNOWN = 255
};

typedef struct { uint32_t offset; uint16_t len; uint8_t flags, rsvd; } ref_desc_t;

int      ref_rx_packet(unsigned char *pkt, int len, int *ret_out, uint16_t *tcp_csum);
/* the stream key StreamHTSearch received for the last TCP_OK ref_rx_packet */
void     ref_last_flow_key(uint8_t key[12]);
uint16_t ref_ip_fast_csum(const void *iph, unsigned int ihl);
uint16_t ref_tcp_calc_checksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr);

/* mtcp/src/icmp.c:18-42 ICMPChecksum (static; reached via ref_icmp.c) */
uint16_t ref_icmp_checksum(const uint8_t *icmph, int len);

/* util/rss.c (key 0x05, compiled as shipped) */
uint32_t ref_util_rss_hash(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp);
int      ref_util_rss_core(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp, int nq);
/* mtcp/src/rss.c (key 0x05) */
int      ref_mtcp_rss_core(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp, int nq,
                           uint8_t endian_check);
/* GetRSSHash over the 4-tuple of a well-formed IPv4/TCP frame (host order) */
uint32_t ref_rss_hash_pkt(const unsigned char *pkt);

double   ref_bench_rx(unsigned char *buf, const ref_desc_t *desc, uint32_t n,
                      uint32_t off_shift, int rss, int nthreads, int reps);
#endif
