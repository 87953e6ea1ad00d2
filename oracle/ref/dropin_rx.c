/*
 * dropin_rx.c — TEST HARNESS (oracle/_ref build: needs /root/reference to
 * build; the binary then runs on the GPU box like the other oracle/_ref
 * files).
 *
 * The drop-in proof at the reference's REAL call sites:
 * mTCP's own rx chain — ProcessPacket (mtcp/src/eth_in.c:9-56) ->
 * ProcessIPv4Packet (ip_in.c:15-62) -> ProcessTCPPacket (tcp_in.c:1138-1175)
 * -> TCPCalcChecksum (tcp_util.c:157-190) — compiled from /root/reference
 * WITHOUT -DDISABLE_HWCSUM, so that ip_in.c:28-31 and tcp_in.c:1159-1164 ask
 * `mtcp->iom->dev_ioctl(mtcp->ctx, ifidx, PKT_RX_IP_CSUM / PKT_RX_TCP_CSUM,
 * ...)` first and skip their own checksum on a 0.  mtcp->iom is
 * &gpu_module_func: mtcp_amd/io_module/gpu_module.c compiled against mTCP's
 * real headers (mtcp.h, io_module.h, tcp_util.h, with mTCP's flags), wrapping
 * a PSIO-like backend (below) that serves a chunk file in bursts of <= 64
 * frames from ONE receive buffer it overwrites on every recv_pkts (the
 * recycling psio_module.c:244-246 / dpdk_module.c:395-398 do).  The loop is
 * the rx section of RunMainLoop, core.c:763-777, over the real
 * struct mtcp_manager / mtcp_thread_context.
 *
 * Observation only (nothing on the path is replaced): StreamHTSearch
 * (tcp_in.c:1186, reached only after both checksum steps) records the stream
 * key and longjmps back (the stateful rest of mTCP never runs);
 * ProcessARPPacket / ProcessICMPPacket record that they were reached;
 * `--wrap=TCPCalcChecksum` counts the reference's software TCP checksums;
 * with mode "observe" mtcp->iom is a copy of gpu_module_func whose dev_ioctl
 * records each answer of gpu_module_func.dev_ioctl (mode "plain": mtcp->iom
 * = &gpu_module_func itself).  Every other symbol the reference objects name
 * is ref_stubs.c's aborting stub.
 *
 *   dropin_rx CHUNK DESC OUT [observe|plain [stop]]
 *     CHUNK, DESC  tests/golden/rx_buf.bin, rx_desc.bin (byte offsets)
 *     OUT          one dropin_rec per frame (below)
 *     stop         mTCP stops as soon as the backend has run dry: the
 *                  pipelined module's last aggregate is still on the GPU
 *                  when destroy_handle runs (its frames are never served)
 *   prints one JSON line: counters, nstat.rx_errors[0] / rx_packets[0]
 */
#define _GNU_SOURCE
#include <setjmp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <time.h>

#include "mtcp.h"
#include "eth_in.h"
#include "io_module.h"
#include "ps.h"
#include "tcp_stream.h"
#include "tcp_in.h"             /* TIMEVAL_TO_TS (core.c:760) */
#include "ref_glue.h"          /* REF_BR_* branch codes, ref_desc_t */

struct mtcp_config CONFIG;     /* eths_num = 1 (mtcp.conf's one port) */
extern io_module_func gpu_module_func;
extern io_module_func *gpu_inner_module;

/* per frame, in arrival order */
typedef struct {
    uint8_t served;            /* get_rptr returned a frame                 */
    uint8_t branch;            /* REF_BR_* of the reference's chain, 254: NULL */
    int8_t ret;                /* ProcessPacket's return (2: reached flow lookup) */
    int8_t ioctl_ip;           /* dev_ioctl(PKT_RX_IP_CSUM) answer, -2 not asked */
    int8_t ioctl_tcp;          /* dev_ioctl(PKT_RX_TCP_CSUM) answer, -2 not asked */
    uint8_t csum_called;       /* the reference ran TCPCalcChecksum          */
    uint8_t same;              /* served bytes == the original frame's       */
    uint8_t pad;
    uint8_t key[12];           /* stream key StreamHTSearch received          */
} dropin_rec;

typedef struct {
    jmp_buf env;
    int arp, icmp, released, tcp_reached, csum_called;
    uint16_t csum_value;
    int ioctl_ip, ioctl_tcp;
    uint8_t key[12];
} probe_t;
static probe_t g_probe;
static uint64_t g_csum_calls;

/* ---- observation points with the reference's prototypes ------------------ */
void *StreamHTSearch(struct hashtable *ht, const void *key)
{
    const tcp_stream *s = (const tcp_stream *)key;
    (void)ht;
    memcpy(g_probe.key, &s->saddr, 4);
    memcpy(g_probe.key + 4, &s->daddr, 4);
    memcpy(g_probe.key + 8, &s->sport, 2);
    memcpy(g_probe.key + 10, &s->dport, 2);
    longjmp(g_probe.env, 1);
}

int ProcessARPPacket(mtcp_manager_t mtcp, uint32_t cur_ts, const int ifidx,
                     unsigned char *pkt_data, int len)
{
    (void)mtcp; (void)cur_ts; (void)ifidx; (void)pkt_data; (void)len;
    g_probe.arp = 1;
    return TRUE;
}

int ProcessICMPPacket(mtcp_manager_t mtcp, struct iphdr *iph, int len)
{
    (void)mtcp; (void)iph; (void)len;
    g_probe.icmp = 1;
    return TRUE;
}

int __real_ProcessTCPPacket(mtcp_manager_t, uint32_t, const int, const struct iphdr *, int);
int __wrap_ProcessTCPPacket(mtcp_manager_t mtcp, uint32_t cur_ts, const int ifidx,
                            const struct iphdr *iph, int ip_len)
{
    g_probe.tcp_reached = 1;
    return __real_ProcessTCPPacket(mtcp, cur_ts, ifidx, iph, ip_len);
}

uint16_t __real_TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr);
uint16_t __wrap_TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr)
{
    uint16_t v = __real_TCPCalcChecksum(buf, len, saddr, daddr);
    g_probe.csum_called = 1;
    g_probe.csum_value = v;
    g_csum_calls++;
    return v;
}

static io_module_func g_observed;          /* mode observe: gpu_module_func, dev_ioctl logged */
static int32_t observe_ioctl(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp)
{
    int32_t r = gpu_module_func.dev_ioctl(ctx, nif, cmd, argp);
    if (cmd == PKT_RX_IP_CSUM) g_probe.ioctl_ip = r;
    if (cmd == PKT_RX_TCP_CSUM) g_probe.ioctl_tcp = r;
    return r;
}

/* ---- the wrapped backend: PSIO-like bursts from one recycled buffer ------- */
struct fake_nic {
    const uint8_t *chunk;
    const ref_desc_t *desc;
    uint32_t n, next, base, cnt;
    uint8_t *rx;                            /* the receive buffer, reused per burst */
    uint32_t off[64];
    int recv_calls, released;
};
static struct fake_nic g_nic;
#define RX_TAIL (1u << 17)                  /* a frame's tot_len may point 64 KiB past it */

static void nic_load(void) {}
static void nic_init(struct mtcp_thread_context *ctx) { ctx->io_private_context = &g_nic; }
static int32_t nic_link(struct mtcp_thread_context *ctx) { (void)ctx; return 0; }
static void nic_release(struct mtcp_thread_context *ctx, int ifidx, unsigned char *p, int len)
{
    struct fake_nic *f = ctx->io_private_context;
    (void)ifidx; (void)p; (void)len;
    if (f != &g_nic) { fprintf(stderr, "context swap broken\n"); exit(3); }
    f->released++;
    g_probe.released = 1;
}
static uint8_t *nic_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
    (void)ctx; (void)ifidx; (void)len;
    return NULL;
}
static int32_t nic_send(struct mtcp_thread_context *ctx, int nif) { (void)ctx; (void)nif; return 0; }
static int32_t nic_recv(struct mtcp_thread_context *ctx, int ifidx)
{
    struct fake_nic *f = ctx->io_private_context;
    uint32_t i, o = 0;
    (void)ifidx;
    if (f != &g_nic) { fprintf(stderr, "context swap broken\n"); exit(3); }
    f->recv_calls++;
    f->base = f->next;
    f->cnt = f->n - f->next < 64 ? f->n - f->next : 64;
    f->next += f->cnt;
    /* the NIC overwrites the same buffer: the previous burst's frames are gone */
    memset(f->rx, 0xA5, 64 * 16384 + RX_TAIL);
    for (i = 0; i < f->cnt; i++) {
        const ref_desc_t *d = &f->desc[f->base + i];
        f->off[i] = o;
        memcpy(f->rx + o, f->chunk + d->offset, d->len);
        o += ((uint32_t)d->len + 63) & ~63u;
    }
    return (int32_t)f->cnt;
}
static uint8_t *nic_rptr(struct mtcp_thread_context *ctx, int ifidx, int index, uint16_t *len)
{
    struct fake_nic *f = ctx->io_private_context;
    (void)ifidx;
    *len = f->desc[f->base + (uint32_t)index].len;
    return f->rx + f->off[index];
}
static int32_t nic_select(struct mtcp_thread_context *ctx) { (void)ctx; return 0; }
static void nic_destroy(struct mtcp_thread_context *ctx) { ctx->io_private_context = NULL; }

static io_module_func nic_module = {
    .load_module = nic_load, .init_handle = nic_init, .link_devices = nic_link,
    .release_pkt = nic_release, .get_wptr = nic_wptr, .send_pkts = nic_send,
    .get_rptr = nic_rptr, .recv_pkts = nic_recv, .select = nic_select,
    .destroy_handle = nic_destroy, .dev_ioctl = NULL,
};

/* ---- one frame through the reference's ProcessPacket (eth_in.c:9) -------- */
static void process(mtcp_manager_t mtcp, uint32_t ts, uint8_t *pkt, uint16_t len,
                    const uint8_t *orig, dropin_rec *rec)
{
    volatile int ret = 0, flow = 0;
    uint64_t err0 = mtcp->nstat.rx_errors[0];

    memset(&g_probe, 0, sizeof(g_probe));
    g_probe.ioctl_ip = g_probe.ioctl_tcp = -2;
    rec->served = 1;
    rec->same = memcmp(pkt, orig, len) == 0;
    if (setjmp(g_probe.env) == 0)
        ret = ProcessPacket(mtcp, 0, ts, pkt, len);       /* core.c:773 */
    else
        flow = 1;
    rec->ret = (int8_t)(flow ? 2 : ret);
    rec->ioctl_ip = (int8_t)g_probe.ioctl_ip;
    rec->ioctl_tcp = (int8_t)g_probe.ioctl_tcp;
    rec->csum_called = (uint8_t)g_probe.csum_called;
    if (flow) {
        rec->branch = REF_BR_TCP_OK;
        memcpy(rec->key, g_probe.key, 12);
    } else if (g_probe.arp) {
        rec->branch = REF_BR_ARP;
    } else if (g_probe.icmp) {
        rec->branch = REF_BR_ICMP;
    } else if (g_probe.released) {
        rec->branch = ret == TRUE ? REF_BR_ETH_OTHER : REF_BR_IP_VERSION;
    } else if (ret == FALSE) {
        rec->branch = REF_BR_IP_PROTO_OTHER;
    } else if (ret == ERROR && mtcp->nstat.rx_errors[0] == err0 + 1) {
        if (g_probe.csum_called)
            rec->branch = g_probe.csum_value ? REF_BR_TCP_CSUM_BAD : REF_BR_UNKNOWN;
        else if (g_probe.tcp_reached)
            rec->branch = REF_BR_TCP_LEN_BAD;
        else
            rec->branch = ((pkt[16] << 8) | pkt[17]) < 20 ? REF_BR_IP_SHORT : REF_BR_IP_CSUM_BAD;
    } else {
        rec->branch = REF_BR_UNKNOWN;
    }
}

static void *slurp(const char *path, size_t *size)
{
    FILE *f = fopen(path, "rb");
    void *p;
    long n;
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    n = ftell(f);
    fseek(f, 0, SEEK_SET);
    p = malloc((size_t)n + RX_TAIL);
    if (fread(p, 1, (size_t)n, f) != (size_t)n) { perror(path); exit(1); }
    memset((uint8_t *)p + n, 0, RX_TAIL);
    fclose(f);
    *size = (size_t)n;
    return p;
}

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

int main(int argc, char **argv)
{
    size_t nb, nd;
    const uint8_t *chunk;
    const ref_desc_t *desc;
    uint32_t n, seen = 0, served = 0, nulls = 0, changed = 0;
    int observe, stop, rounds = 0, idle = 0;
    double destroy_s;
    dropin_rec *recs;
    struct mtcp_thread_context ctx;
    mtcp_manager_t mtcp;
    struct timeval tv;
    FILE *out;

    if (argc < 4) {
        fprintf(stderr, "usage: dropin_rx CHUNK DESC OUT [observe|plain [stop]]\n");
        return 1;
    }
    observe = !(argc > 4 && strcmp(argv[4], "plain") == 0);
    stop = argc > 5 && strcmp(argv[5], "stop") == 0;
    chunk = slurp(argv[1], &nb);
    desc = slurp(argv[2], &nd);
    n = (uint32_t)(nd / sizeof(ref_desc_t));
    recs = calloc(n + 1, sizeof(*recs));
    g_nic.chunk = chunk;
    g_nic.desc = desc;
    g_nic.n = n;
    g_nic.rx = malloc(64 * 16384 + RX_TAIL);

    CONFIG.eths_num = 1;
    memset(&ctx, 0, sizeof(ctx));
    mtcp = calloc(1, sizeof(*mtcp));
    ctx.cpu = 0;
    ctx.mtcp_manager = mtcp;
    mtcp->ctx = &ctx;
    if (observe) {
        g_observed = gpu_module_func;
        g_observed.dev_ioctl = observe_ioctl;
        mtcp->iom = &g_observed;
    } else {
        mtcp->iom = &gpu_module_func;
    }
    gpu_inner_module = &nic_module;
    mtcp->iom->load_module();
    mtcp->iom->init_handle(&ctx);
    mtcp->iom->link_devices(&ctx);

    /* RunMainLoop's rx section, core.c:763-777 (one interface) */
    while (1) {
        int32_t recv_cnt, i;
        gettimeofday(&tv, NULL);
        mtcp->cur_ts = TIMEVAL_TO_TS(&tv);
        recv_cnt = mtcp->iom->recv_pkts(&ctx, 0);
        if (recv_cnt <= 0) {
            /* the pipelined module returns 0 while it fills and its last
             * aggregate one call after the backend ran dry */
            if (g_nic.next == g_nic.n && ++idle >= 2)
                break;
            continue;
        }
        idle = 0;
        rounds++;
        for (i = 0; i < recv_cnt; i++) {
            uint16_t len;
            uint8_t *pktbuf = mtcp->iom->get_rptr(mtcp->ctx, 0, i, &len);
            dropin_rec *r = &recs[seen + (uint32_t)i];
            if (seen + (uint32_t)i >= n) { fprintf(stderr, "more frames than sent\n"); return 2; }
            if (pktbuf != NULL) {
                process(mtcp, mtcp->cur_ts, pktbuf, len, chunk + desc[seen + i].offset, r);
                served++;
                changed += !r->same;
            } else {
                r->branch = 254;
                r->ioctl_ip = r->ioctl_tcp = -2;             /* ProcessPacket never ran */
                mtcp->nstat.rx_errors[0]++;
                nulls++;
            }
        }
        seen += (uint32_t)recv_cnt;
        if (stop && g_nic.next == g_nic.n)
            break;                                   /* shut down with frames in flight */
    }
    {
        double t0 = now_s();
        mtcp->iom->destroy_handle(&ctx);
        destroy_s = now_s() - t0;
    }

    out = fopen(argv[3], "wb");
    if (!out || fwrite(recs, sizeof(*recs), n, out) != n) { perror(argv[3]); return 1; }
    fclose(out);
    printf("{\"frames\": %u, \"seen\": %u, \"served\": %u, \"null\": %u, \"changed\": %u, "
           "\"rx_errors\": %llu, \"rx_packets\": %llu, \"rx_bytes\": %llu, \"tcp_csum_calls\": %llu, "
           "\"rounds\": %d, \"recv_calls\": %d, \"released\": %d, \"observe\": %d, "
           "\"destroy_s\": %.6f}\n",
           n, seen, served, nulls, changed, (unsigned long long)mtcp->nstat.rx_errors[0],
           (unsigned long long)mtcp->nstat.rx_packets[0], (unsigned long long)mtcp->nstat.rx_bytes[0],
           (unsigned long long)g_csum_calls,
           rounds, g_nic.recv_calls, g_nic.released, observe, destroy_s);
    free(recs);
    free(mtcp);
    return 0;
}
