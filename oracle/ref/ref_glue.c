/*
 * ref_glue.c — TEST INFRASTRUCTURE ONLY (oracle/_ref build, this container
 * and, as a prebuilt CPU baseline, the GPU box).
 *
 * Drives the REFERENCE's own rx chain, compiled from /root/reference:
 * ProcessPacket (mtcp/src/eth_in.c:9) -> ProcessIPv4Packet (ip_in.c:16) ->
 * ProcessTCPPacket (tcp_in.c:1139) -> TCPCalcChecksum (tcp_util.c:158).
 * A packet whose checksums pass reaches StreamHTSearch (tcp_in.c:1186); the
 * stub below longjmps back here, so the stateful rest of mTCP never runs.
 * Branch identification uses only observable effects of the reference code:
 * its return value, which of release_pkt / ProcessARPPacket /
 * ProcessICMPPacket / ProcessTCPPacket / TCPCalcChecksum it called, the
 * TCPCalcChecksum return, and the nstat.rx_errors counter.
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <setjmp.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mtcp.h"
#include "eth_in.h"
#include "io_module.h"
#include "ps.h"
#include "tcp_stream.h"

#include "ref_glue.h"

struct mtcp_config CONFIG;           /* referenced by tcp_in.o, never read here */

typedef struct {
    jmp_buf env;
    int released, arp, icmp, tcp_reached, csum_called;
    uint16_t csum_value;
    uint8_t flow_key[12];            /* s_stream.saddr..dport at StreamHTSearch */
} probe_t;

static __thread probe_t *g_probe;

/* ---- stubs with the reference's prototypes ------------------------------ */
void *StreamHTSearch(struct hashtable *ht, const void *key)
{
    /* tcp_in.c:1180-1186: the tcp_stream key HashFlow will hash
     * (fields saddr, daddr, sport, dport: tcp_stream.h:163-166) */
    const tcp_stream *s = (const tcp_stream *)key;
    (void)ht;
    memcpy(g_probe->flow_key, &s->saddr, 4);
    memcpy(g_probe->flow_key + 4, &s->daddr, 4);
    memcpy(g_probe->flow_key + 8, &s->sport, 2);
    memcpy(g_probe->flow_key + 10, &s->dport, 2);
    longjmp(g_probe->env, 1);        /* tcp_in.c:1186: checksum path passed */
}

int ProcessARPPacket(mtcp_manager_t mtcp, uint32_t cur_ts, const int ifidx,
                     unsigned char *pkt_data, int len)
{
    (void)mtcp; (void)cur_ts; (void)ifidx; (void)pkt_data; (void)len;
    g_probe->arp = 1;
    return TRUE;
}

int ProcessICMPPacket(mtcp_manager_t mtcp, struct iphdr *iph, int len)
{
    (void)mtcp; (void)iph; (void)len;
    g_probe->icmp = 1;
    return TRUE;
}

/* linker --wrap: observe the reference's calls without changing them */
int __real_ProcessTCPPacket(mtcp_manager_t, uint32_t, const int, const struct iphdr *, int);
int __wrap_ProcessTCPPacket(mtcp_manager_t mtcp, uint32_t cur_ts, const int ifidx,
                            const struct iphdr *iph, int ip_len)
{
    g_probe->tcp_reached = 1;
    return __real_ProcessTCPPacket(mtcp, cur_ts, ifidx, iph, ip_len);
}

uint16_t __real_TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr);
uint16_t __wrap_TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr)
{
    uint16_t v = __real_TCPCalcChecksum(buf, len, saddr, daddr);
    g_probe->csum_called = 1;
    g_probe->csum_value = v;
    return v;
}

static void fake_release_pkt(struct mtcp_thread_context *ctx, int ifidx,
                             unsigned char *pkt_data, int len)
{
    (void)ctx; (void)ifidx; (void)pkt_data; (void)len;
    g_probe->released = 1;
}

static struct io_module_func g_fake_iom;   /* only release_pkt is used */

typedef struct {
    struct mtcp_manager mgr;
    probe_t probe;
} ref_ctx_t;

static void ref_ctx_init(ref_ctx_t *c)
{
    memset(c, 0, sizeof(*c));
    g_fake_iom.release_pkt = fake_release_pkt;
    c->mgr.iom = &g_fake_iom;
}

/* Run one frame through the reference; returns the branch taken. */
static int ref_run(ref_ctx_t *c, unsigned char *pkt, int len, int *ret_out,
                   uint16_t *tcp_csum)
{
    volatile int ret = 0;
    probe_t *p = &c->probe;
    uint64_t err0 = c->mgr.nstat.rx_errors[0];

    memset(p, 0, sizeof(*p));
    g_probe = p;
    if (setjmp(p->env) == 0) {
        ret = ProcessPacket(&c->mgr, 0, 0, pkt, len);
    } else {
        *ret_out = 2;   /* not a reference return value: reached flow lookup */
        *tcp_csum = p->csum_value;
        return REF_BR_TCP_OK;
    }
    *ret_out = ret;
    *tcp_csum = p->csum_value;
    if (p->arp)
        return REF_BR_ARP;
    if (p->icmp)
        return REF_BR_ICMP;
    if (p->released)
        return ret == TRUE ? REF_BR_ETH_OTHER : REF_BR_IP_VERSION;
    if (ret == FALSE)
        return REF_BR_IP_PROTO_OTHER;
    if (ret == ERROR) {
        if (c->mgr.nstat.rx_errors[0] != err0 + 1)
            return REF_BR_UNKNOWN;
        if (p->csum_called)
            return p->csum_value ? REF_BR_TCP_CSUM_BAD : REF_BR_UNKNOWN;
        if (p->tcp_reached)
            return REF_BR_TCP_LEN_BAD;
        /* ip_in.c:25-26 vs :35-36, distinguished by the first test's input */
        return ((pkt[16] << 8) | pkt[17]) < 20 ? REF_BR_IP_SHORT : REF_BR_IP_CSUM_BAD;
    }
    return REF_BR_UNKNOWN;
}

static __thread ref_ctx_t *g_ctx1;

int ref_rx_packet(unsigned char *pkt, int len, int *ret_out, uint16_t *tcp_csum)
{
    if (!g_ctx1) {
        g_ctx1 = (ref_ctx_t *)malloc(sizeof(*g_ctx1));
        ref_ctx_init(g_ctx1);
    }
    return ref_run(g_ctx1, pkt, len, ret_out, tcp_csum);
}

void ref_last_flow_key(uint8_t key[12])
{
    if (g_ctx1)
        memcpy(key, g_ctx1->probe.flow_key, 12);
    else
        memset(key, 0, 12);
}

uint16_t ref_ip_fast_csum(const void *iph, unsigned int ihl)
{
    return ip_fast_csum(iph, ihl);   /* io_engine/include/ps.h:66-95 */
}

uint16_t ref_tcp_calc_checksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr)
{
    return __real_TCPCalcChecksum(buf, len, saddr, daddr);
}

/* ---- CPU baseline on the reference's own code --------------------------- */
typedef struct {
    unsigned char *buf; const ref_desc_t *desc; uint32_t lo, hi, off_shift;
    int rss, cpu, reps; pthread_barrier_t *bar; double *best; uint64_t sink;
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
    ref_ctx_t *c = (ref_ctx_t *)malloc(sizeof(*c));
    cpu_set_t set;
    int r;
    uint32_t i;

    ref_ctx_init(c);
    CPU_ZERO(&set);
    CPU_SET(a->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);   /* core.c:1057 */
    for (r = 0; r < a->reps + 1; r++) {
        double t0;
        pthread_barrier_wait(a->bar);
        t0 = now_s();
        for (i = a->lo; i < a->hi; i++) {      /* core.c:768-776 */
            unsigned char *pkt = a->buf + ((uint64_t)a->desc[i].offset << a->off_shift);
            int len = a->desc[i].len, ret;
            uint16_t cs;
            int br = ref_run(c, pkt, len, &ret, &cs);
            a->sink += (uint64_t)br + cs;
            if (a->rss && br == REF_BR_TCP_OK)
                a->sink += ref_rss_hash_pkt(pkt);
        }
        pthread_barrier_wait(a->bar);
        if (a->lo == 0 && r > 0) {
            double dt = now_s() - t0;
            if (*a->best < 0 || dt < *a->best)
                *a->best = dt;
        }
    }
    free(c);
    return NULL;
}

double ref_bench_rx(unsigned char *buf, const ref_desc_t *desc, uint32_t n,
                    uint32_t off_shift, int rss, int nthreads, int reps)
{
    pthread_t th[1024];
    bench_arg args[1024];
    pthread_barrier_t bar;
    double best = -1.0;
    cpu_set_t allowed;
    int cpus[1024], ncpu = 0, cc, t;

    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    if (rss)
        ref_rss_hash_pkt(buf + ((uint64_t)desc[0].offset << off_shift));  /* lazy key cache */
    sched_getaffinity(0, sizeof(allowed), &allowed);
    for (cc = 0; cc < CPU_SETSIZE && ncpu < 1024; cc++)
        if (CPU_ISSET(cc, &allowed))
            cpus[ncpu++] = cc;
    pthread_barrier_init(&bar, NULL, (unsigned)nthreads);
    for (t = 0; t < nthreads; t++) {
        bench_arg *a = &args[t];
        memset(a, 0, sizeof(*a));
        a->buf = buf; a->desc = desc; a->off_shift = off_shift; a->rss = rss;
        a->lo = (uint32_t)((uint64_t)n * t / nthreads);
        a->hi = (uint32_t)((uint64_t)n * (t + 1) / nthreads);
        a->cpu = ncpu ? cpus[t % ncpu] : 0; a->reps = reps; a->bar = &bar; a->best = &best;
        pthread_create(&th[t], NULL, bench_thread, a);
    }
    for (t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
    pthread_barrier_destroy(&bar);
    return best;
}
