/*
 * rxloop.c — TEST HARNESS for mtcp_amd/io_module/gpu_module.c.
 *
 * Runs the rx section of mTCP's RunMainLoop (mtcp/src/core.c:763-777)
 * against gpu_module_func wrapping a fake PSIO-like backend that serves a
 * chunk file in bursts of <= 64 frames (PS_CHUNK_SIZE, psio_module.c:15) and
 * keeps its own io_private_context (to exercise the context swap).  For every
 * frame it records whether get_rptr returned NULL (core.c:774-775 counts
 * those as rx_errors) and whether a served frame is byte-identical to the
 * original; dev_ioctl(PKT_RX_IP_CSUM / PKT_RX_TCP_CSUM) answers are logged.
 *
 *   rxloop CHUNK DESC OUT [timing|verify|tx] [THREADS]
 *     CHUNK  frame bytes; DESC mtcp_gpu_desc records (byte offsets)
 *     OUT    one byte per frame: 0 NULL, 1 served intact, 2 served but changed
 *     timing served frames are not compared (only their first 64 B are read,
 *            as ProcessPacket's parse would): the loop's rate without the
 *            harness's own byte-for-byte check
 *     tx     the transmit side instead: every frame of the chunk goes out
 *            through get_wptr (copied in as mTCP's EthernetOutput would
 *            write it), dev_ioctl(PKT_TX_TCPIP_CSUM_PEEK) decides who fills
 *            the checksums (-1: the harness fills them, as mTCP's software
 *            path, ip_out.c:164 / tcp_out.c:327-329), send_pkts every 64
 *            frames (MAX_PKT_BURST); OUT = the sent frames, laid out as CHUNK
 *     THREADS  mTCP threads (default 1), one per core as core.c:1057 runs
 *            them: each has its own mtcp_thread_context (cpu = thread index),
 *            so its own gpu_module context, GPU ctx and staging, and its own
 *            backend over a contiguous shard of the frames (share-nothing);
 *            the wall time runs from a common start barrier to the last
 *            thread's end; thread t is pinned to the t-th CPU the process
 *            may run on, as mtcp_core_affinitize (cpu.c) pins each mTCP
 *            thread to its core (RXLOOP_CPUS=a,b,..: thread t on the t-th
 *            CPU of that list; RXLOOP_PIN=0: unpinned)
 *   RXLOOP_CTX_CPU=1 the thread's mtcp_thread_context.cpu is the cpu it is
 *            pinned to (mTCP's ctx->cpu is the core, core.c:1057), not its
 *            index: gpu_module.c then picks the GPU on that cpu's node
 *   RXLOOP_PASSES=p  (timing modes) each thread's backend serves its shard p
 *            times over, so that a run lasts long enough to time many threads
 *   RXLOOP_REF=lib   (timing modes) the software checks of a thread the module
 *            does not offload (dev_ioctl -1) are the REFERENCE's own
 *            ProcessPacket chain (oracle/_ref/libref_rx.so, ref_rx_packet:
 *            eth_in / ip_in / tcp_in / tcp_util compiled from /root/reference),
 *            not the oracle's restatement
 * Prints one JSON line with the counters and the wall time of the rx loop
 * (tools/io_path_bench.py turns that into the io_module path's rate).  Built with the test doubles in
 * tests/c/mtcp_double (two fields of mtcp_thread_context, io_module_func).
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mtcp.h"
#include "io_module.h"
#include "mtcp_gpu.h"
#include "tcp_util.h"
#include "../../oracle/mtcp_oracle.h"

/* mTCP's checksum functions, which gpu_module.c calls for frames the GPU
 * could not fill (ps.h:66-95, tcp_util.c:157-190): the oracle's restatement */
uint16_t ip_fast_csum(const void *iph, unsigned int ihl) { return oracle_ip_fast_csum(iph, ihl); }
uint16_t TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr)
{
    return oracle_tcp_calc_checksum(buf, len, saddr, daddr);
}

extern io_module_func gpu_module_func;
int gpu_module_thread_device(struct mtcp_thread_context *ctx);   /* test build of gpu_module.c */
struct mtcp_config CONFIG = {1, 1};                /* one interface (mtcp.conf's port list); num_cores set below */
extern io_module_func *gpu_inner_module;

/* RXLOOP_REF: the reference's rx chain (ref_glue.h's ref_rx_packet) */
typedef int (*ref_rx_fn)(unsigned char *pkt, int len, int *ret_out, uint16_t *tcp_csum);
static ref_rx_fn g_ref_rx;
enum { REF_BR_IP_CSUM_BAD = 4, REF_BR_TCP_CSUM_BAD = 9 };   /* oracle/ref/ref_glue.h */

struct fake_psio {
    const uint8_t *buf;
    const mtcp_gpu_desc *desc;
    uint32_t n, next, base, cnt;
    uint32_t passes_left;            /* RXLOOP_PASSES - 1: serve the shard again */
    int recv_calls;
    uint8_t *tx_buf;                 /* tx: frame i is written at desc[i].offset */
    uint32_t tx_next, tx_queued, tx_sent;
    int send_calls;
};
static __thread struct fake_psio *tl_fake;         /* this thread's backend */

static void fake_load(void) {}
static void fake_init(struct mtcp_thread_context *ctx) { ctx->io_private_context = tl_fake; }
static int32_t fake_link(struct mtcp_thread_context *ctx) { (void)ctx; return 0; }
static void fake_release(struct mtcp_thread_context *ctx, int ifidx, unsigned char *p, int len)
{
    (void)ctx; (void)ifidx; (void)p; (void)len;
}
static uint8_t *fake_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
    struct fake_psio *f = ctx->io_private_context;
    (void)ifidx;
    if (f != tl_fake) { fprintf(stderr, "context swap broken\n"); exit(3); }
    if (!f->tx_buf || f->tx_next >= f->n || len != f->desc[f->tx_next].len)
        return NULL;
    f->tx_queued++;
    return f->tx_buf + f->desc[f->tx_next++].offset;
}
static int32_t fake_send(struct mtcp_thread_context *ctx, int nif)
{
    struct fake_psio *f = ctx->io_private_context;
    (void)nif;
    if (f != tl_fake) { fprintf(stderr, "context swap broken\n"); exit(3); }
    f->send_calls++;
    f->tx_sent += f->tx_queued;        /* the frames already sit in tx_buf */
    f->tx_queued = 0;
    return 0;
}
static int32_t fake_recv(struct mtcp_thread_context *ctx, int ifidx)
{
    struct fake_psio *f = ctx->io_private_context;    /* must be the inner's */
    (void)ifidx;
    if (f != tl_fake) { fprintf(stderr, "context swap broken\n"); exit(3); }
    f->recv_calls++;
    if (f->next == f->n && f->passes_left) {
        f->passes_left--;
        f->next = 0;
    }
    f->base = f->next;
    f->cnt = f->n - f->next < 64 ? f->n - f->next : 64;
    f->next += f->cnt;
    return (int32_t)f->cnt;
}
static uint8_t *fake_rptr(struct mtcp_thread_context *ctx, int ifidx, int index, uint16_t *len)
{
    struct fake_psio *f = ctx->io_private_context;
    const mtcp_gpu_desc *d = &f->desc[f->base + (uint32_t)index];
    (void)ifidx;
    *len = d->len;
    return (uint8_t *)(f->buf + d->offset);
}
static int32_t fake_select(struct mtcp_thread_context *ctx) { (void)ctx; return 0; }
static void fake_destroy(struct mtcp_thread_context *ctx) { ctx->io_private_context = NULL; }

/* RXLOOP_AS_NETMAP=1: the fake backend is registered as netmap_module_func
 * (gpu_module.c refuses the tx offload over netmap) */
io_module_func netmap_module_func;

static io_module_func fake_module = {
    .load_module = fake_load, .init_handle = fake_init, .link_devices = fake_link,
    .release_pkt = fake_release, .get_wptr = fake_wptr, .send_pkts = fake_send,
    .get_rptr = fake_rptr, .recv_pkts = fake_recv, .select = fake_select,
    .destroy_handle = fake_destroy, .dev_ioctl = NULL,
};

static void *slurp(const char *path, size_t *size)
{
    FILE *f = fopen(path, "rb");
    void *p;
    long n;
    if (!f) { perror(path); exit(1); }
    fseek(f, 0, SEEK_END);
    n = ftell(f);
    fseek(f, 0, SEEK_SET);
    p = malloc((size_t)n + 64);
    if (fread(p, 1, (size_t)n, f) != (size_t)n) { perror(path); exit(1); }
    fclose(f);
    *size = (size_t)n;
    return p;
}

struct worker {
    pthread_t tid;
    int cpu, pin_cpu, timing, tx;
    struct fake_psio fake;                 /* frames [first, first + fake.n) */
    uint32_t first;
    uint8_t *status;                       /* status + first */
    uint64_t rx_packets, rx_errors, changed, hdr_sum;
    int rounds, ioctl_ip, ioctl_tcp, ioctl_tx, sw_filled;
    uint32_t seen;
    int device;                            /* gpu_module_thread_device after init */
    struct timespec t1;
};
static pthread_barrier_t g_start;
static struct timespec g_t0;

/* The transmit side of RunMainLoop: EthernetOutput's get_wptr, IPOutput /
 * SendTCPPacket's dev_ioctl and software fills, then send_pkts per burst. */
static void tx_main(struct worker *w, struct mtcp_thread_context *ctx)
{
    const struct fake_psio *f = &w->fake;
    uint32_t i;
    for (i = 0; i < f->n; i++) {
        const mtcp_gpu_desc *d = &f->desc[i];
        uint8_t *p = gpu_module_func.get_wptr(ctx, 0, d->len);
        if (!p) { fprintf(stderr, "get_wptr refused frame %u\n", i); exit(4); }
        memcpy(p, f->buf + d->offset, d->len);
        w->ioctl_tx = gpu_module_func.dev_ioctl(ctx, 0, PKT_TX_TCPIP_CSUM_PEEK, p + 14);
        if (w->ioctl_tx == -1) {                         /* mTCP fills them itself */
            mtcp_gpu_desc one = {0, d->len, 0, 0};
            w->sw_filled += (int)oracle_tx_fill(p, d->len, &one, 1, 0);
        }
        if ((i + 1) % 64 == 0 || i + 1 == f->n)
            gpu_module_func.send_pkts(ctx, 0);
    }
}

/* The t-th CPU of the process's affinity mask (wraps), or -1. */
static int nth_allowed_cpu(int t)
{
    cpu_set_t set;
    int c, k = 0, count;
    if (sched_getaffinity(0, sizeof(set), &set) != 0 || (count = CPU_COUNT(&set)) == 0)
        return -1;
    t %= count;
    for (c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &set) && k++ == t)
            return c;
    return -1;
}

static void *worker_main(void *arg)
{
    struct worker *w = arg;
    struct mtcp_thread_context ctx = {w->cpu, NULL};
    const struct fake_psio *f = &w->fake;

    if (w->pin_cpu >= 0) {                           /* before init_handle's allocations */
        cpu_set_t one;
        CPU_ZERO(&one);
        CPU_SET(w->pin_cpu, &one);
        pthread_setaffinity_np(pthread_self(), sizeof(one), &one);
    }
    tl_fake = &w->fake;
    w->ioctl_ip = w->ioctl_tcp = -2;
    gpu_module_func.init_handle(&ctx);
    gpu_module_func.link_devices(&ctx);
    w->device = gpu_module_thread_device(&ctx);
    if (pthread_barrier_wait(&g_start) == PTHREAD_BARRIER_SERIAL_THREAD)
        clock_gettime(CLOCK_MONOTONIC, &g_t0);
    pthread_barrier_wait(&g_start);                  /* g_t0 set before anyone runs */
    if (w->tx) {
        tx_main(w, &ctx);
        clock_gettime(CLOCK_MONOTONIC, &w->t1);
        gpu_module_func.destroy_handle(&ctx);
        return NULL;
    }
    for (int idle = 0;;) {                            /* core.c:763-777 */
        int32_t recv_cnt = gpu_module_func.recv_pkts(&ctx, 0), i;
        if (recv_cnt <= 0) {
            /* mTCP polls on; the harness stops once its backend is drained
             * and the module has returned nothing twice (a pipelined module
             * returns 0 while it fills, and its last aggregate one call
             * after the backend ran dry) */
            if (f->next == f->n && !f->passes_left && ++idle >= 2)
                break;
            continue;
        }
        idle = 0;
        w->rounds++;
        /* timing modes: where the module answers -1 (a thread it does not
         * offload, MTCP_GPU_THREADS), ProcessPacket runs mTCP's own checks
         * (ip_in.c:35-36, tcp_in.c:1165-1173): the harness pays for them
         * with the restated chain and drops what they drop */
        const int sw = w->timing && gpu_module_func.dev_ioctl(&ctx, 0, PKT_RX_TCP_CSUM, NULL) == -1;
        for (i = 0; i < recv_cnt; i++) {
            uint16_t len = 0;
            uint8_t *pktbuf = gpu_module_func.get_rptr(&ctx, 0, i, &len);
            const uint32_t at = (w->seen + (uint32_t)i) % f->n;   /* RXLOOP_PASSES wraps */
            const mtcp_gpu_desc *d = &f->desc[at];
            if (pktbuf != NULL && sw && g_ref_rx) {
                int ret;
                uint16_t csum;
                const int br = g_ref_rx(pktbuf, len, &ret, &csum);
                if (br == REF_BR_IP_CSUM_BAD || br == REF_BR_TCP_CSUM_BAD)
                    pktbuf = NULL;                     /* ERROR: counted in rx_errors */
                else
                    w->hdr_sum += csum;
            } else if (pktbuf != NULL && sw) {
                mtcp_gpu_result r;
                const int v = oracle_rx_packet(pktbuf, len, NULL, &r);
                if (v == MTCP_GPU_V_IP_CSUM_BAD || v == MTCP_GPU_V_TCP_CSUM_BAD || v == MTCP_GPU_V_TRUNCATED)
                    pktbuf = NULL;                     /* ERROR: counted in rx_errors */
                else
                    w->hdr_sum += r.ip_csum + r.tcp_csum;
            }
            if (pktbuf != NULL) {
                /* ProcessPacket(mtcp, rx_inf, ts, pktbuf, len) would run here */
                if (w->timing == 1) {
                    /* timing mode: touch the headers as ProcessPacket's parse
                     * would (first 64 B), no byte-for-byte check */
                    uint32_t k;
                    for (k = 0; k < 64 && k < len; k += 8) w->hdr_sum += pktbuf[k];
                    w->status[at] = 1;
                } else if (w->timing == 2) {
                    /* payload mode: read every byte once, as the payload's copy
                     * into the stream's receive buffer would (tcp_in.c ->
                     * RBPut), no byte-for-byte check */
                    uint64_t acc = 0;
                    uint32_t k;
                    for (k = 0; k + 8 <= len; k += 8) {
                        uint64_t v;
                        memcpy(&v, pktbuf + k, 8);
                        acc += v;
                    }
                    w->hdr_sum += acc;
                    w->status[at] = 1;
                } else {
                    int same = len == d->len && memcmp(pktbuf, f->buf + d->offset, len) == 0;
                    w->status[at] = same ? 1 : 2;
                    w->changed += !same;
                }
                w->rx_packets++;
            } else {
                w->rx_errors++;                        /* nstat.rx_errors[rx_inf]++ */
            }
        }
        if (w->ioctl_ip == -2) {
            w->ioctl_ip = gpu_module_func.dev_ioctl(&ctx, 0, PKT_RX_IP_CSUM, NULL);
            w->ioctl_tcp = gpu_module_func.dev_ioctl(&ctx, 0, PKT_RX_TCP_CSUM, NULL);
        }
        w->seen += (uint32_t)recv_cnt;
    }
    clock_gettime(CLOCK_MONOTONIC, &w->t1);
    gpu_module_func.destroy_handle(&ctx);
    return NULL;
}

int main(int argc, char **argv)
{
    size_t nb, nd;
    uint8_t *status;
    const uint8_t *buf;
    const mtcp_gpu_desc *desc;
    uint32_t n, seen = 0;
    uint64_t rx_packets = 0, rx_errors = 0, changed = 0, hdr_sum = 0, frame_bytes = 0;
    int offloading = 0;                               /* threads whose dev_ioctl answered 0 */
    int rounds = 0, recv_calls = 0, timing, threads, t;
    struct timespec t1;
    struct worker *ws;
    double secs;
    FILE *out;

    if (argc < 4) {
        fprintf(stderr, "usage: rxloop CHUNK DESC OUT [timing|payload|verify|tx] [THREADS]\n");
        return 1;
    }
    timing = argc > 4 && strcmp(argv[4], "timing") == 0 ? 1
             : argc > 4 && strcmp(argv[4], "payload") == 0 ? 2 : 0;
    int tx = argc > 4 && strcmp(argv[4], "tx") == 0;
    uint8_t *tx_buf = NULL;
    threads = argc > 5 ? atoi(argv[5]) : 1;
    if (threads < 1 || threads > 64) { fprintf(stderr, "THREADS: 1..64\n"); return 1; }
    CONFIG.num_cores = threads;                     /* mtcp.conf's num_cores: one mTCP thread each */
    buf = slurp(argv[1], &nb);
    desc = slurp(argv[2], &nd);
    n = (uint32_t)(nd / sizeof(mtcp_gpu_desc));
    status = calloc(n + 1, 1);
    if (tx) tx_buf = calloc(nb + 64, 1);
    ws = calloc((size_t)threads, sizeof(*ws));
    const char *pin_env = getenv("RXLOOP_PIN");
    const int pin = !(pin_env && strcmp(pin_env, "0") == 0);
    int pin_cpu[64];
    for (t = 0; t < threads; t++) pin_cpu[t] = pin ? nth_allowed_cpu(t) : -1;
    const char *cpus_env = getenv("RXLOOP_CPUS");     /* "a,b,c": thread t -> t-th entry (wraps) */
    if (pin && cpus_env && *cpus_env) {
        int list[64], cnt = 0;
        for (const char *c = cpus_env; *c && cnt < 64;) {
            char *end;
            long v = strtol(c, &end, 10);
            if (end == c) break;
            list[cnt++] = (int)v;
            c = *end == ',' ? end + 1 : end;
        }
        for (t = 0; t < threads && cnt; t++) pin_cpu[t] = list[t % cnt];
    }

    const char *passes_env = getenv("RXLOOP_PASSES");
    const uint32_t passes = passes_env && atoi(passes_env) > 1 && timing ? (uint32_t)atoi(passes_env) : 1;
    const char *ref_env = getenv("RXLOOP_REF");
    if (ref_env && *ref_env) {
        void *h = dlopen(ref_env, RTLD_NOW | RTLD_LOCAL);
        g_ref_rx = h ? (ref_rx_fn)dlsym(h, "ref_rx_packet") : NULL;
        if (!g_ref_rx) { fprintf(stderr, "RXLOOP_REF: %s\n", dlerror()); return 1; }
    }
    gpu_inner_module = &fake_module;
    if (getenv("RXLOOP_AS_NETMAP") && strcmp(getenv("RXLOOP_AS_NETMAP"), "1") == 0) {
        netmap_module_func = fake_module;
        gpu_inner_module = &netmap_module_func;
    }
    gpu_module_func.load_module();
    pthread_barrier_init(&g_start, NULL, (unsigned)threads);
    for (t = 0; t < threads; t++) {                   /* contiguous shards */
        struct worker *w = &ws[t];
        const uint32_t lo = (uint32_t)((uint64_t)n * t / threads);
        const uint32_t hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
        w->cpu = t;
        w->pin_cpu = pin_cpu[t];
        if (getenv("RXLOOP_CTX_CPU") && strcmp(getenv("RXLOOP_CTX_CPU"), "1") == 0 && pin_cpu[t] >= 0)
            w->cpu = pin_cpu[t];
        w->timing = timing;
        w->tx = tx;
        w->fake.tx_buf = tx_buf;
        w->first = lo;
        w->status = status + lo;
        w->fake.buf = buf;
        w->fake.desc = desc + lo;
        w->fake.n = hi - lo;
        w->fake.passes_left = passes - 1;
        if (pthread_create(&w->tid, NULL, worker_main, w) != 0) { perror("pthread_create"); return 1; }
    }
    t1 = g_t0;
    for (t = 0; t < threads; t++) {
        struct worker *w = &ws[t];
        pthread_join(w->tid, NULL);
        rx_packets += w->rx_packets;
        rx_errors += w->rx_errors;
        changed += w->changed;
        hdr_sum += w->hdr_sum;
        rounds += w->rounds;
        offloading += w->ioctl_tcp == 0;
        recv_calls += w->fake.recv_calls;
        seen += w->seen;
        if (t == 0 || w->t1.tv_sec > t1.tv_sec ||
            (w->t1.tv_sec == t1.tv_sec && w->t1.tv_nsec > t1.tv_nsec))
            t1 = w->t1;
    }
    for (uint32_t k = 0; k < n; k++) frame_bytes += desc[k].len;

    out = fopen(argv[3], "wb");
    if (tx) {
        int sw = 0, sends = 0;
        uint32_t sent = 0;
        for (t = 0; t < threads; t++) {
            sw += ws[t].sw_filled;
            sends += ws[t].fake.send_calls;
            sent += ws[t].fake.tx_sent;
        }
        if (!out || fwrite(tx_buf, 1, nb, out) != nb) { perror(argv[3]); return 1; }
        fclose(out);
        secs = (double)(t1.tv_sec - g_t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - g_t0.tv_nsec);
        printf("{\"frames\": %u, \"sent\": %u, \"send_calls\": %d, \"ioctl_tx\": %d, "
               "\"sw_filled\": %d, \"seconds\": %.6f, \"frame_bytes\": %llu, \"threads\": %d}\n",
               n, sent, sends, ws[0].ioctl_tx, sw, secs, (unsigned long long)frame_bytes, threads);
        free(tx_buf);
        free(ws);
        free(status);
        free((void *)buf);
        free((void *)desc);
        return 0;
    }
    if (!out || fwrite(status, 1, n, out) != n) { perror(argv[3]); return 1; }
    fclose(out);
    char devs[64 * 12] = "", *dp = devs;
    char tsec[64 * 24] = "", *tp = tsec;
    for (t = 0; t < threads; t++) {
        dp += sprintf(dp, "%s[%d, %d]", t ? ", " : "", ws[t].cpu, ws[t].device);
        /* each thread's own time from the common start, and whether it offloaded */
        tp += sprintf(tp, "%s[%.6f, %d]", t ? ", " : "",
                      (double)(ws[t].t1.tv_sec - g_t0.tv_sec) + 1e-9 * (double)(ws[t].t1.tv_nsec - g_t0.tv_nsec),
                      ws[t].ioctl_tcp == 0);
    }
    secs = (double)(t1.tv_sec - g_t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - g_t0.tv_nsec);
    printf("{\"frames\": %u, \"seen\": %u, \"rounds\": %d, \"inner_bursts\": %d, "
           "\"rx_packets\": %llu, \"rx_errors\": %llu, \"changed\": %llu, "
           "\"ioctl_rx_ip\": %d, \"ioctl_rx_tcp\": %d, \"seconds\": %.6f, "
           "\"frame_bytes\": %llu, \"timing_mode\": %d, \"hdr_sum\": %llu, \"threads\": %d, "
           "\"offloading_threads\": %d, \"passes\": %u, \"sw_checks\": \"%s\", "
           "\"cpu_device\": [%s], \"thread_seconds_offload\": [%s]}\n",
           n, seen, rounds, recv_calls, (unsigned long long)rx_packets,
           (unsigned long long)rx_errors, (unsigned long long)changed, ws[0].ioctl_ip,
           ws[0].ioctl_tcp, secs, (unsigned long long)frame_bytes, timing,
           (unsigned long long)hdr_sum, threads, offloading, passes, g_ref_rx ? "reference" : "oracle", devs, tsec);
    free(ws);
    free(status);
    free((void *)buf);
    free((void *)desc);
    return 0;
}
