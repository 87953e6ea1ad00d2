/*
 * mtcp_oracle.c — TEST INFRASTRUCTURE ONLY (see mtcp_oracle.h).
 *
 * Plain-C restatement of mTCP's --disable-hwcsum rx/tx per-packet path.
 * Every function cites the reference lines it restates (paths relative to
 * the mTCP tree).  Loop shapes follow the reference so that, compiled with
 * gcc -O3 -m64 like mtcp/src/Makefile.in:20-31, it is also a representative
 * CPU baseline.
 */
#define _GNU_SOURCE
#include "mtcp_oracle.h"

#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

static inline uint32_t ld32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint16_t ld16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline uint16_t bswap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }
static inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

/*
 * io_engine/include/ps.h:66-95.  The x86 asm, instruction by instruction:
 *   movl (%1),%0 ; subl $4,%2 ; jbe 2f        -> ihl <= 4 returns dword 0 as is
 *   addl 4(%1) ; adcl 8(%1) ; adcl 12(%1)     -> words 1..3, carry chained
 *   1: adcl 16(%1) ; lea 4(%1) ; decl ; jne   -> words 4..ihl-1 (lea/decl keep CF)
 *   adcl $0                                   -> end-around carry (its carry-out is lost)
 *   movl %0,%2 ; shrl $16,%0 ; addw %w2,%w0 ; adcl $0,%0 ; notl %0
 */
uint16_t oracle_ip_fast_csum(const void *iph, unsigned int ihl)
{
    const uint8_t *p = (const uint8_t *)iph;
    uint32_t sum = ld32(p);
    uint64_t t;
    uint32_t cf = 0, i, hi, lo;

    if (ihl <= 4)                       /* subl $4, %2 ; jbe 2f */
        return (uint16_t)sum;
    for (i = 1; i < ihl; i++) {         /* addl / adcl chain */
        t = (uint64_t)sum + ld32(p + 4 * i) + cf;
        sum = (uint32_t)t;
        cf = (uint32_t)(t >> 32);
    }
    sum = sum + cf;                     /* adcl $0, %0 (carry-out dropped) */
    hi = sum >> 16;                     /* movl %0,%2 ; shrl $16,%0 */
    lo = sum & 0xFFFF;
    t = (uint64_t)(hi & 0xFFFF) + lo;   /* addw %w2, %w0 */
    sum = (hi & 0xFFFF0000u) | (uint32_t)(t & 0xFFFF);
    sum += (uint32_t)(t >> 16);         /* adcl $0, %0 */
    sum = ~sum;                         /* notl %0 */
    return (uint16_t)sum;
}

/* mtcp/src/tcp_util.c:157-190 */
uint16_t oracle_tcp_calc_checksum(const uint16_t *buf, uint16_t len,
                                  uint32_t saddr, uint32_t daddr)
{
    uint32_t sum = 0;
    const uint8_t *w = (const uint8_t *)buf;
    int nleft = len;

    while (nleft > 1) {                 /* tcp_util.c:168-172 */
        sum += ld16(w);
        w += 2;
        nleft -= 2;
    }
    if (nleft)                          /* tcp_util.c:175-176: *w & ntohs(0xFF00) */
        sum += w[0];                    /* the low byte of a little-endian u16 */

    sum += (saddr & 0x0000FFFF) + (saddr >> 16);   /* :179-182 pseudo header */
    sum += (daddr & 0x0000FFFF) + (daddr >> 16);
    sum += bswap16(len);
    sum += bswap16(6);                  /* htons(IPPROTO_TCP) */

    sum = (sum >> 16) + (sum & 0xFFFF); /* :184-185 */
    sum += (sum >> 16);
    sum = ~sum;
    return (uint16_t)sum;
}

const uint8_t oracle_rss_key_0x05[40] = {
    0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05,
    0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05,
    0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05,
    0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05, 0x05 };

const uint8_t oracle_rss_key_microsoft[40] = {
    0x6d, 0x5a, 0x56, 0xda, 0x25, 0x5b, 0x0e, 0xc2,
    0x41, 0x67, 0x25, 0x3d, 0x43, 0xa3, 0x8f, 0xb0,
    0xd0, 0xca, 0x2b, 0xcb, 0xae, 0x7b, 0x30, 0xb4,
    0x77, 0xcb, 0x2d, 0xa3, 0x80, 0x30, 0xf2, 0x0c,
    0x6a, 0x42, 0xb7, 0x3b, 0xbe, 0xac, 0x01, 0xfa };

/* util/rss.c:13-105 (BuildKeyCache): cache[i] = 32-bit key window at bit i. */
void oracle_build_key_cache(const uint8_t key[40], uint32_t *cache, int cache_len)
{
    uint32_t result = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) |
                      ((uint32_t)key[2] << 8) | (uint32_t)key[3];
    uint32_t idx = 32;
    int i;

    for (i = 0; i < cache_len; i++, idx++) {
        uint8_t shift = (uint8_t)(idx % 8);
        uint32_t bit;

        cache[i] = result;
        bit = ((key[idx / 8] << shift) & 0x80) ? 1 : 0;
        result = ((result << 1) | bit);
    }
}

/* util/rss.c:107-145 (GetRSSHash), inputs in host order. */
uint32_t oracle_get_rss_hash(const uint32_t cache[96], uint32_t sip, uint32_t dip,
                             uint16_t sp, uint16_t dp)
{
    uint32_t res = 0;
    int i;

    for (i = 0; i < 32; i++) {
        if (sip & 0x80000000u)
            res ^= cache[i];
        sip <<= 1;
    }
    for (i = 0; i < 32; i++) {
        if (dip & 0x80000000u)
            res ^= cache[32 + i];
        dip <<= 1;
    }
    for (i = 0; i < 16; i++) {
        if (sp & 0x8000)
            res ^= cache[64 + i];
        sp = (uint16_t)(sp << 1);
    }
    for (i = 0; i < 16; i++) {
        if (dp & 0x8000)
            res ^= cache[80 + i];
        dp = (uint16_t)(dp << 1);
    }
    return res;
}

/* util/rss.c:153-165 (always endian fix) / mtcp/src/rss.c:90-103. */
static int rss_queue_of(uint32_t hash, int num_queues, int endian_check)
{
    static const uint32_t off[4] = {3, 1, (uint32_t)-1, (uint32_t)-3};
    uint32_t masked = hash & 0x0000007F;

    if (endian_check)
        masked += off[masked & 0x3];
    return (int)(masked % (uint32_t)num_queues);
}

int oracle_get_rss_cpu_core(const uint32_t cache[96], uint32_t sip, uint32_t dip,
                            uint16_t sp, uint16_t dp, int num_queues, int endian_check)
{
    return rss_queue_of(oracle_get_rss_hash(cache, sip, dip, sp, dp), num_queues,
                        endian_check);
}

void oracle_rss_cfg_init(oracle_rss_cfg *cfg, const uint8_t key[40], int num_queues,
                         int endian_check)
{
    oracle_build_key_cache(key ? key : oracle_rss_key_0x05, cfg->cache, 96);
    cfg->num_queues = num_queues;
    cfg->endian_check = endian_check;
}

/*
 * ProcessPacket (eth_in.c:9-56) -> ProcessIPv4Packet (ip_in.c:15-62) -> head
 * of ProcessTCPPacket (tcp_in.c:1138-1175).  Before each step reads a header
 * byte it checks that the byte lies inside the frame; where the reference
 * would read past `len` (undefined behaviour) the verdict is TRUNCATED.
 */
/* mtcp/src/icmp.c:18-42 ICMPChecksum.  A negative len skips the loop (the
 * assert is compiled out): ~0.  An odd len reads the last byte into the low
 * half of an uninitialised u16 (icmp.c:31-33, undefined); the high half is
 * taken as 0 here. */
uint16_t oracle_icmp_checksum(const uint8_t *icmph, int len)
{
    uint32_t sum = 0;
    while (len > 1) {
        sum += ld16(icmph);
        icmph += 2;
        len -= 2;
    }
    if (len == 1)
        sum += *icmph;
    sum = (sum >> 16) + (sum & 0xffff);
    sum += (sum >> 16);
    return (uint16_t)~sum;
}

int oracle_rx_packet(const uint8_t *pkt, uint32_t len, const oracle_rss_cfg *rss,
                     mtcp_gpu_result *r)
{
    uint32_t ip_len, ihl, version, proto, T, doff;
    uint16_t tcp_len;

    memset(r, 0, sizeof(*r));
#define VERDICT(v) do { r->verdict = (uint8_t)(v); return (v); } while (0)
#define NEED(nbytes) do { if ((uint32_t)(nbytes) > len) VERDICT(MTCP_GPU_V_TRUNCATED); } while (0)

    NEED(14);                                        /* struct ethhdr */
    r->eth_type = bswap16(ld16(pkt + 12));           /* eth_in.c:13 */
    if (r->eth_type != 0x0800) {
        if (r->eth_type == 0x0806)                   /* eth_in.c:39-41 */
            VERDICT(MTCP_GPU_V_ARP);
        VERDICT(MTCP_GPU_V_ETH_OTHER);               /* eth_in.c:43-46 */
    }
    NEED(18);
    ip_len = bswap16(ld16(pkt + 16));                /* ip_in.c:21 */
    ihl = pkt[14] & 0x0F;
    r->ip_len = (uint16_t)ip_len;
    r->ihl_doff = (uint8_t)ihl;
    if (ip_len < 20)                                 /* ip_in.c:25-26 */
        VERDICT(MTCP_GPU_V_IP_SHORT);
    NEED(14 + 4 * (ihl > 4 ? ihl : 1));              /* ps.h:68-70: ihl <= 4 reads one dword */
    r->ip_csum = oracle_ip_fast_csum(pkt + 14, ihl); /* ip_in.c:35 */
    if (r->ip_csum)
        VERDICT(MTCP_GPU_V_IP_CSUM_BAD);
    version = pkt[14] >> 4;
    if (version != 4)                                /* ip_in.c:47-50 */
        VERDICT(MTCP_GPU_V_IP_VERSION);
    NEED(24);
    proto = pkt[23];                                 /* ip_in.c:52 */
    if (proto == 1) {
        /* ProcessICMPECHORequest's check (icmp.c:94): ICMPChecksum over
         * ip_len - 4*ihl bytes from iph + 4*ihl, when they lie in the frame */
        if (14 + ip_len <= len) {
            int ilen = (int)ip_len - (int)(ihl << 2);
            r->tcp_csum = oracle_icmp_checksum(pkt + 14 + 4 * ihl, ilen);
            r->payload_len = (uint16_t)(ilen > 0 ? ilen : 0);
        }
        VERDICT(MTCP_GPU_V_ICMP);
    }
    if (proto != 6)
        VERDICT(MTCP_GPU_V_IP_PROTO_OTHER);

    /* ProcessTCPPacket: tcph = iph + 4*ihl (tcp_in.c:1142); the declarations
     * read seq/ack_seq/window (:1147-1149) and doff before the length check. */
    T = 14 + 4 * ihl;
    NEED(T + 16);
    doff = pkt[T + 12] >> 4;
    r->saddr = ld32(pkt + 26);
    r->daddr = ld32(pkt + 30);
    r->sport = ld16(pkt + T);
    r->dport = ld16(pkt + T + 2);
    r->seq = bswap32(ld32(pkt + T + 4));
    r->ack_seq = bswap32(ld32(pkt + T + 8));
    r->window = bswap16(ld16(pkt + T + 14));
    r->tcp_flags = pkt[T + 13];
    r->ihl_doff = (uint8_t)(ihl | (doff << 4));
    if (rss) {
        r->rss_hash = oracle_get_rss_hash(rss->cache, bswap32(r->saddr), bswap32(r->daddr),
                                          bswap16(r->sport), bswap16(r->dport));
        r->rss_queue = (uint8_t)rss_queue_of(r->rss_hash, rss->num_queues,
                                             rss->endian_check);
    }
    if (ip_len < ((ihl + doff) << 2))                /* tcp_in.c:1155-1156 */
        VERDICT(MTCP_GPU_V_TCP_LEN_BAD);
    r->payload_len = (uint16_t)(ip_len - ((ihl + doff) << 2));   /* tcp_in.c:1144 */
    tcp_len = (uint16_t)((doff << 2) + r->payload_len);          /* tcp_in.c:1166 */
    NEED(14 + ip_len);
    r->tcp_csum = oracle_tcp_calc_checksum((const uint16_t *)(pkt + T), tcp_len,
                                           r->saddr, r->daddr);  /* tcp_in.c:1165 */
    if (r->tcp_csum)                                 /* tcp_in.c:1167-1173 */
        VERDICT(MTCP_GPU_V_TCP_CSUM_BAD);
    VERDICT(MTCP_GPU_V_TCP_OK);
#undef NEED
#undef VERDICT
}

static int desc_bad(uint64_t buf_len, const mtcp_gpu_desc *d, uint32_t off_shift,
                    uint64_t *pos)
{
    uint64_t p = (uint64_t)d->offset << off_shift;
    *pos = p;
    return (p & 1) != 0 || p + d->len > buf_len;      /* any even start (include/mtcp_gpu.h) */
}

void oracle_rx_chunk(const uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc,
                     uint32_t n, uint32_t off_shift, const oracle_rss_cfg *rss,
                     mtcp_gpu_result *out)
{
    uint32_t i;
    uint64_t p;

    for (i = 0; i < n; i++) {
        if (desc_bad(buf_len, &desc[i], off_shift, &p)) {
            memset(&out[i], 0, sizeof(out[i]));
            out[i].verdict = MTCP_GPU_V_BAD_DESC;
            continue;
        }
        oracle_rx_packet(buf + p, desc[i].len, rss, &out[i]);
    }
}

/*
 * tx checksum fill: IPOutput's iph->check = 0 ... ip_fast_csum (ip_out.c:145,164)
 * and SendTCPPacket's memset-zeroed check ... TCPCalcChecksum
 * (tcp_out.c:241,327-329), for frames that are well-formed IPv4/TCP.
 */
uint32_t oracle_tx_fill(uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc,
                        uint32_t n, uint32_t off_shift)
{
    uint32_t i, filled = 0;

    for (i = 0; i < n; i++) {
        uint64_t p;
        uint8_t *pkt;
        uint32_t len = desc[i].len, ip_len, ihl, doff, T;
        uint16_t c;

        if (desc_bad(buf_len, &desc[i], off_shift, &p))
            continue;
        pkt = buf + p;
        if (len < 34 || bswap16(ld16(pkt + 12)) != 0x0800)
            continue;
        ihl = pkt[14] & 0x0F;
        ip_len = bswap16(ld16(pkt + 16));
        if ((pkt[14] >> 4) != 4 || ihl < 5 || pkt[23] != 6)
            continue;
        T = 14 + 4 * ihl;
        if (T + 20 > len)
            continue;
        doff = pkt[T + 12] >> 4;
        if (doff < 5 || ip_len < 4 * (ihl + doff) || 14 + ip_len > len)
            continue;
        pkt[24] = pkt[25] = 0;
        c = oracle_ip_fast_csum(pkt + 14, ihl);
        memcpy(pkt + 24, &c, 2);
        pkt[T + 16] = pkt[T + 17] = 0;
        c = oracle_tcp_calc_checksum((const uint16_t *)(pkt + T), (uint16_t)(ip_len - 4 * ihl),
                                     ld32(pkt + 26), ld32(pkt + 30));
        memcpy(pkt + T + 16, &c, 2);
        filled++;
    }
    return filled;
}

/*
 * Synthetic traffic (host mirror of mtcp_amd/csrc/pktgen.hip; spec in
 * include/mtcp_gpu_pktgen.h).
 */
#define PG_GAMMA 0x9E3779B97F4A7C15ull
static inline uint64_t pg_mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static inline uint64_t pg_state(uint64_t seed, uint64_t i)
{
    return pg_mix(seed ^ (i * 0xD1342543DE82EF95ull + 0x632BE59BD9B4E019ull));
}
static inline uint64_t pg_r(uint64_t s, uint64_t k) { return pg_mix(s + (k + 1) * PG_GAMMA); }

static void pg_one(uint8_t *pkt, uint32_t L, uint64_t seed, uint64_t gi)
{
    uint64_t s = pg_state(seed, gi);
    uint64_t r0 = pg_r(s, 0), r1 = pg_r(s, 1), r2 = pg_r(s, 2), r3 = pg_r(s, 3);
    uint64_t r4 = pg_r(s, 4), r5 = pg_r(s, 5), c = pg_r(s, 6);
    uint32_t p, doff, T = 34, ip_len = L - 14, pay, nbits;
    uint32_t padded = (L + 63) & ~63u;

    for (p = 0; p < padded; p++) {
        uint64_t w = pg_r(s, 16 + (p >> 3));
        pkt[p] = p < L ? (uint8_t)(w >> (8 * (p & 7))) : 0;
    }
    if (L < 54)
        return;
    doff = (L >= 66 && ((r4 >> 32) & 1)) ? 8 : 5;
    for (p = 0; p < 6; p++) {
        pkt[p] = (uint8_t)(r0 >> (8 * p));
        pkt[6 + p] = (uint8_t)(r1 >> (8 * p));
    }
    pkt[12] = 0x08; pkt[13] = 0x00;
    pkt[14] = 0x45; pkt[15] = 0x00;
    pkt[16] = (uint8_t)(ip_len >> 8); pkt[17] = (uint8_t)ip_len;
    pkt[18] = (uint8_t)(r0 >> 48); pkt[19] = (uint8_t)(r0 >> 56);
    pkt[20] = 0x40; pkt[21] = 0x00; pkt[22] = 64; pkt[23] = 6;
    pkt[24] = 0; pkt[25] = 0;
    for (p = 0; p < 8; p++) pkt[26 + p] = (uint8_t)(r2 >> (8 * p));
    for (p = 0; p < 8; p++) pkt[34 + p] = (uint8_t)(r3 >> (8 * p));
    for (p = 0; p < 4; p++) pkt[42 + p] = (uint8_t)(r4 >> (8 * p));
    pkt[46] = (uint8_t)(doff << 4);
    pkt[47] = (uint8_t)(0x10 | (((r4 >> 33) & 1) ? 0x08 : 0));
    pkt[48] = (uint8_t)(r4 >> 40); pkt[49] = (uint8_t)(r4 >> 48);
    pkt[50] = 0; pkt[51] = 0; pkt[52] = 0; pkt[53] = 0;
    if (doff == 8) {
        pkt[54] = 0x01; pkt[55] = 0x01; pkt[56] = 0x08; pkt[57] = 0x0A;
        for (p = 0; p < 8; p++) pkt[58 + p] = (uint8_t)(r5 >> (8 * p));
    }
    {   /* checksums, as the tx fill would write them */
        uint16_t v = oracle_ip_fast_csum(pkt + 14, 5);
        memcpy(pkt + 24, &v, 2);
        v = oracle_tcp_calc_checksum((const uint16_t *)(pkt + T), (uint16_t)(ip_len - 20),
                                     ld32(pkt + 26), ld32(pkt + 30));
        memcpy(pkt + T + 16, &v, 2);
    }
    /* corruption: 1/1024 a TCP bit, 1/4096 an IP header bit */
    pay = T + 4 * doff;
    if ((c & 1023) == 0) {
        uint32_t lo = pay < L ? pay : T;
        nbits = 8 * (L - lo);
        p = (uint32_t)((c >> 10) % nbits);
        pkt[lo + (p >> 3)] ^= (uint8_t)(1u << (p & 7));
    }
    if (((c >> 32) & 4095) == 0) {
        p = (uint32_t)((c >> 44) % 160);
        pkt[14 + (p >> 3)] ^= (uint8_t)(1u << (p & 7));
    }
}

void oracle_pktgen(uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc, uint32_t n,
                   uint32_t off_shift, uint64_t seed, uint64_t first_index)
{
    uint32_t i;
    for (i = 0; i < n; i++) {
        uint64_t p = (uint64_t)desc[i].offset << off_shift;
        uint32_t padded = ((uint32_t)desc[i].len + 63) & ~63u;
        if ((p & 63) || p + padded > buf_len)
            continue;
        pg_one(buf + p, desc[i].len, seed, first_index + i);
    }
}

/* ---- multi-core CPU baseline --------------------------------------------- */
typedef struct {
    const uint8_t *buf; uint64_t buf_len; const mtcp_gpu_desc *desc;
    uint32_t lo, hi, off_shift; const oracle_rss_cfg *rss; mtcp_gpu_result *out;
    int cpu, reps; pthread_barrier_t *bar; double *best;
} bench_arg;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void *bench_thread(void *vp)
{
    bench_arg *a = (bench_arg *)vp;
    cpu_set_t set;
    int r;

    CPU_ZERO(&set);
    CPU_SET(a->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);  /* core.c:1057 */
    for (r = 0; r < a->reps + 1; r++) {              /* rep 0 = warm-up */
        double t0;
        pthread_barrier_wait(a->bar);
        t0 = now_s();
        oracle_rx_chunk(a->buf, a->buf_len, a->desc + a->lo, a->hi - a->lo, a->off_shift,
                        a->rss, a->out + a->lo);
        pthread_barrier_wait(a->bar);
        if (a->lo == 0 && r > 0) {                   /* thread 0 times the slowest shard */
            double dt = now_s() - t0;
            if (*a->best < 0 || dt < *a->best)
                *a->best = dt;
        }
    }
    return NULL;
}

double oracle_bench_rx(const uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc,
                       uint32_t n, uint32_t off_shift, const oracle_rss_cfg *rss,
                       mtcp_gpu_result *out, int nthreads, int reps)
{
    pthread_t *th;
    bench_arg *args;
    pthread_barrier_t bar;
    double best = -1.0;
    int t;
    cpu_set_t allowed;
    int cpus[1024], ncpu = 0, c;

    if (nthreads < 1)
        nthreads = 1;
    sched_getaffinity(0, sizeof(allowed), &allowed);
    for (c = 0; c < CPU_SETSIZE && ncpu < 1024; c++)
        if (CPU_ISSET(c, &allowed))
            cpus[ncpu++] = c;
    th = (pthread_t *)calloc((size_t)nthreads, sizeof(*th));
    args = (bench_arg *)calloc((size_t)nthreads, sizeof(*args));
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    for (t = 0; t < nthreads; t++) {
        bench_arg *a = &args[t];
        a->buf = buf; a->buf_len = buf_len; a->desc = desc; a->off_shift = off_shift;
        a->lo = (uint32_t)((uint64_t)n * t / nthreads);
        a->hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        a->rss = rss; a->out = out; a->cpu = ncpu ? cpus[t % ncpu] : 0;
        a->reps = reps; a->bar = &bar; a->best = &best;
        pthread_create(&th[t], NULL, bench_thread, a);
    }
    for (t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    pthread_barrier_destroy(&bar);
    free(th);
    free(args);
    return best;
}

/* ---- flow-table hash ------------------------------------ */
/* mtcp/src/tcp_stream.c:77-87: hash += key[i] with key a (signed) char
 * pointer, so bytes >= 0x80 add a sign-extended negative value. */
uint32_t oracle_hash_flow(const uint8_t key[12])
{
    uint32_t hash = 0;
    for (int i = 0; i < 12; ++i) {
        hash += (uint32_t)(int32_t)(int8_t)key[i];
        hash += hash << 10;
        hash ^= hash >> 6;
    }
    hash += hash << 3;
    hash ^= hash >> 11;
    hash += hash << 15;
    return hash & (MTCP_GPU_NUM_BINS_FLOWS - 1);
}

void oracle_flow_bins(const mtcp_gpu_result *res, uint32_t n, uint32_t *bins)
{
    for (uint32_t i = 0; i < n; ++i) {
        if (res[i].verdict != MTCP_GPU_V_TCP_OK) {
            bins[i] = MTCP_GPU_FLOW_NONE;
            continue;
        }
        /* tcp_in.c:1180-1183: the local side first */
        uint8_t key[12];
        memcpy(key, &res[i].daddr, 4);
        memcpy(key + 4, &res[i].saddr, 4);
        memcpy(key + 8, &res[i].dport, 2);
        memcpy(key + 10, &res[i].sport, 2);
        bins[i] = oracle_hash_flow(key);
    }
}

/* ---- RSS-friendly address pool --------------------------- */
uint32_t oracle_addr_pool_search(const uint8_t key[40], int core, int num_queues,
                                 uint32_t saddr_base, int num_addr, uint32_t daddr,
                                 uint16_t dport, int endian_check,
                                 mtcp_gpu_addr_entry *out, uint32_t max_out)
{
    uint32_t cache[96];
    oracle_build_key_cache(key ? key : oracle_rss_key_0x05, cache, 96);
    const uint32_t nports = MTCP_GPU_MAX_PORT - MTCP_GPU_MIN_PORT;
    /* addr_pool.c:129: int arithmetic, as the reference */
    const int num_entry = (num_addr * (int)nports) / num_queues;
    const uint32_t base_h = bswap32(saddr_base), daddr_h = bswap32(daddr);
    const uint16_t dport_h = bswap16(dport);
    uint32_t cnt = 0;
    for (int i = 0; i < num_addr; ++i) {
        const uint32_t saddr_h = base_h + (uint32_t)i;
        for (uint32_t j = MTCP_GPU_MIN_PORT; j < MTCP_GPU_MAX_PORT; ++j) {
            if ((int)cnt >= num_entry) break;                  /* addr_pool.c:160-161 */
            const int q = oracle_get_rss_cpu_core(cache, daddr_h, saddr_h, dport_h,
                                                  (uint16_t)j, num_queues, endian_check);
            if (q != core) continue;
            if (cnt < max_out) {
                out[cnt].saddr = bswap32(saddr_h);
                out[cnt].sport = bswap16((uint16_t)j);
                out[cnt].rsvd = 0;
            }
            cnt++;
        }
    }
    return cnt;
}
