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
 *   rxloop CHUNK DESC OUT [timing]
 *     CHUNK  frame bytes; DESC mtcp_gpu_desc records (byte offsets)
 *     OUT    one byte per frame: 0 NULL, 1 served intact, 2 served but changed
 *     timing served frames are not compared (only their first 64 B are read,
 *            as ProcessPacket's parse would): the loop's rate without the
 *            harness's own byte-for-byte check
 * Prints one JSON line with the counters and the wall time of the rx loop
 * (tools/io_path_bench.py turns that into the io_module path's rate).  Built with the test doubles in
 * tests/c/mtcp_double (two fields of mtcp_thread_context, io_module_func).
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mtcp.h"
#include "io_module.h"
#include "mtcp_gpu.h"

extern io_module_func gpu_module_func;
extern io_module_func *gpu_inner_module;

struct fake_psio {
    const uint8_t *buf;
    const mtcp_gpu_desc *desc;
    uint32_t n, next, base, cnt;
    int recv_calls;
};
static struct fake_psio g_fake;

static void fake_load(void) {}
static void fake_init(struct mtcp_thread_context *ctx) { ctx->io_private_context = &g_fake; }
static int32_t fake_link(struct mtcp_thread_context *ctx) { (void)ctx; return 0; }
static void fake_release(struct mtcp_thread_context *ctx, int ifidx, unsigned char *p, int len)
{
    (void)ctx; (void)ifidx; (void)p; (void)len;
}
static uint8_t *fake_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
    (void)ctx; (void)ifidx; (void)len;
    return NULL;
}
static int32_t fake_send(struct mtcp_thread_context *ctx, int nif) { (void)ctx; (void)nif; return 0; }
static int32_t fake_recv(struct mtcp_thread_context *ctx, int ifidx)
{
    struct fake_psio *f = ctx->io_private_context;    /* must be the inner's */
    (void)ifidx;
    if (f != &g_fake) { fprintf(stderr, "context swap broken\n"); exit(3); }
    f->recv_calls++;
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

int main(int argc, char **argv)
{
    struct mtcp_thread_context ctx = {0, NULL};
    size_t nb, nd;
    uint8_t *status;
    uint64_t rx_packets = 0, rx_errors = 0, changed = 0;
    int rounds = 0, ioctl_ip = -2, ioctl_tcp = -2;
    uint32_t seen = 0;
    uint64_t frame_bytes = 0, hdr_sum = 0;
    int timing;
    struct timespec t0, t1;
    double secs;
    FILE *out;

    if (argc < 4) { fprintf(stderr, "usage: rxloop CHUNK DESC OUT [timing]\n"); return 1; }
    timing = argc > 4 && strcmp(argv[4], "timing") == 0;
    g_fake.buf = slurp(argv[1], &nb);
    g_fake.desc = slurp(argv[2], &nd);
    g_fake.n = (uint32_t)(nd / sizeof(mtcp_gpu_desc));
    status = calloc(g_fake.n + 1, 1);

    gpu_inner_module = &fake_module;
    gpu_module_func.load_module();
    gpu_module_func.init_handle(&ctx);
    gpu_module_func.link_devices(&ctx);
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (;;) {                                        /* core.c:763-777 */
        int32_t recv_cnt = gpu_module_func.recv_pkts(&ctx, 0), i;
        if (recv_cnt <= 0)
            break;
        rounds++;
        for (i = 0; i < recv_cnt; i++) {
            uint16_t len = 0;
            uint8_t *pktbuf = gpu_module_func.get_rptr(&ctx, 0, i, &len);
            const mtcp_gpu_desc *d = &g_fake.desc[seen + (uint32_t)i];
            if (pktbuf != NULL) {
                /* ProcessPacket(mtcp, rx_inf, ts, pktbuf, len) would run here */
                if (timing) {
                    /* timing mode: touch the headers as ProcessPacket's parse
                     * would (first 64 B), no byte-for-byte check */
                    uint32_t k;
                    for (k = 0; k < 64 && k < len; k += 8) hdr_sum += pktbuf[k];
                    status[seen + i] = 1;
                } else {
                    int same = len == d->len && memcmp(pktbuf, g_fake.buf + d->offset, len) == 0;
                    status[seen + i] = same ? 1 : 2;
                    changed += !same;
                }
                rx_packets++;
            } else {
                rx_errors++;                           /* nstat.rx_errors[rx_inf]++ */
            }
        }
        if (ioctl_ip == -2) {
            ioctl_ip = gpu_module_func.dev_ioctl(&ctx, 0, PKT_RX_IP_CSUM, NULL);
            ioctl_tcp = gpu_module_func.dev_ioctl(&ctx, 0, PKT_RX_TCP_CSUM, NULL);
        }
        seen += (uint32_t)recv_cnt;
    }
    clock_gettime(CLOCK_MONOTONIC, &t1);
    gpu_module_func.destroy_handle(&ctx);
    for (uint32_t k = 0; k < g_fake.n; k++) frame_bytes += g_fake.desc[k].len;

    out = fopen(argv[3], "wb");
    if (!out || fwrite(status, 1, g_fake.n, out) != g_fake.n) { perror(argv[3]); return 1; }
    fclose(out);
    secs = (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
    printf("{\"frames\": %u, \"seen\": %u, \"rounds\": %d, \"inner_bursts\": %d, "
           "\"rx_packets\": %llu, \"rx_errors\": %llu, \"changed\": %llu, "
           "\"ioctl_rx_ip\": %d, \"ioctl_rx_tcp\": %d, \"seconds\": %.6f, "
           "\"frame_bytes\": %llu, \"timing_mode\": %d, \"hdr_sum\": %llu}\n",
           g_fake.n, seen, rounds, g_fake.recv_calls, (unsigned long long)rx_packets,
           (unsigned long long)rx_errors, (unsigned long long)changed, ioctl_ip, ioctl_tcp, secs,
           (unsigned long long)frame_bytes, timing, (unsigned long long)hdr_sum);
    return 0;
}
