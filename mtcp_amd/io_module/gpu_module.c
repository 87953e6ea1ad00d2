/*
 * gpu_module.c — the "gpu" I/O module for mTCP: an
 * io_module_func backend (mtcp/src/include/io_module.h:56-68) that wraps the
 * real driver backend (psio or dpdk), aggregates its receive bursts, checks
 * them on the MI355X in one launch and answers mTCP's checksum offload hook.
 *
 * Built inside the mTCP tree, against its headers (mtcp.h, io_module.h) and
 * include/mtcp_gpu.h + include/mtcp_gpu_rxq.h; link -lmtcp_gpu.  Wiring, as
 * for the other backends (io_module.h:93-112, config.c:569-570):
 *
 *     extern io_module_func gpu_module_func;
 *     AssignIOModule: else if (!strcmp(m, "gpu")) current_iomodule_func = &gpu_module_func;
 *     mtcp.conf:      io = gpu   (+ the wrapped backend in gpu_inner_module)
 *
 * mTCP must be built WITHOUT --disable-hwcsum so that ProcessIPv4Packet and
 * ProcessTCPPacket ask dev_ioctl first (ip_in.c:28-31, tcp_in.c:1159-1164).
 *
 * Receive (RunMainLoop, core.c:763-777): recv_pkts pulls up to
 * GPU_AGG_BURSTS bursts from the wrapped backend, copying each frame into
 * the rxq's pinned staging (the backend recycles its buffers on the next
 * receive: psio_module.c:244-246, dpdk_module.c:395-398), runs the rx
 * kernel once over the aggregate and returns the total count; get_rptr then
 * serves the staged frames and returns NULL for the frames whose IP or TCP
 * checksum fails — the packets mTCP's software path drops with ERROR
 * (ip_in.c:35-36, tcp_in.c:1167-1173) — which core.c:774-775 counts as
 * rx_errors, the pattern dpdk_get_rptr uses for NIC-verified checksums
 * (dpdk_module.c:473-479).  dev_ioctl(PKT_RX_IP_CSUM / PKT_RX_TCP_CSUM)
 * answers 0 while the GPU path is healthy and -1 after any GPU error, so
 * mTCP falls back to its own checksums exactly as with a NIC that lacks the
 * offload (dpdk_dev_ioctl, dpdk_module.c:809-816).
 *
 * Transmit is passed through and checksummed by mTCP (dev_ioctl answers -1
 * for the tx commands): the wrapped backend owns the tx chunk layout.  A
 * psio-specific build can call mtcp_gpu_tx_fill on ppc->w_chunk_buf before
 * psio_send_pkts and answer 0 for PKT_TX_IP_CSUM / PKT_TX_TCPIP_CSUM.
 */
#include <stdlib.h>
#include <string.h>

#include "mtcp.h"
#include "io_module.h"
#include "debug.h"

#include "mtcp_gpu.h"
#include "mtcp_gpu_rxq.h"

#define GPU_AGG_BURSTS 64                 /* bursts per GPU launch           */
#define GPU_BURST      64                 /* PS_CHUNK_SIZE / MAX_PKT_BURST   */
#define GPU_RXQ_PKTS   (GPU_AGG_BURSTS * GPU_BURST)
#define GPU_FRAME_MAX  2048ull            /* MAX_PACKET_SIZE (ps.h:173)      */

/* the backend being wrapped (e.g. &ps_module_func or &dpdk_module_func) */
io_module_func *gpu_inner_module;

struct gpu_private_context {
    void *inner;                          /* the wrapped backend's context   */
    mtcp_gpu_ctx *gpu;                    /* NULL: software checksums        */
    mtcp_gpu_rxq *rxq[MAX_DEVICES];       /* one per rx interface            */
    int passthrough;                      /* no GPU at init: the inner backend */
    uint8_t dropped[MAX_DEVICES][GPU_RXQ_PKTS];   /* inner get_rptr gave NULL */
    int served_raw[MAX_DEVICES];          /* this aggregate has no verdicts  */
};

/* Call into the wrapped backend with its own io_private_context in place. */
#define INNER_CALL(ctx, expr)                                                  \
    ({                                                                         \
        struct gpu_private_context *g_ = (ctx)->io_private_context;           \
        (ctx)->io_private_context = g_->inner;                                 \
        __typeof__(expr) r_ = (expr);                                          \
        g_->inner = (ctx)->io_private_context;                                 \
        (ctx)->io_private_context = g_;                                        \
        r_;                                                                    \
    })
#define INNER_VOID(ctx, stmt)                                                  \
    do {                                                                       \
        struct gpu_private_context *g_ = (ctx)->io_private_context;           \
        (ctx)->io_private_context = g_->inner;                                 \
        stmt;                                                                  \
        g_->inner = (ctx)->io_private_context;                                 \
        (ctx)->io_private_context = g_;                                        \
    } while (0)

static void gpu_load_module(void)
{
    gpu_inner_module->load_module();
}

static void gpu_init_handle(struct mtcp_thread_context *ctx)
{
    struct gpu_private_context *g = calloc(1, sizeof(*g));
    int i, ndev;

    if (!g) {
        TRACE_ERROR("gpu_module: out of memory\n");
        exit(EXIT_FAILURE);
    }
    gpu_inner_module->init_handle(ctx);       /* sets ctx->io_private_context */
    g->inner = ctx->io_private_context;
    ctx->io_private_context = g;

    ndev = mtcp_gpu_device_count();
    if (ndev <= 0 || mtcp_gpu_open(&g->gpu, ctx->cpu % ndev, NULL, 1, 0) != MTCP_GPU_OK) {
        g->gpu = NULL;
        g->passthrough = 1;                  /* behave exactly like the inner */
        return;
    }
    for (i = 0; i < MAX_DEVICES; i++)
        if (mtcp_gpu_rxq_create(&g->rxq[i], g->gpu, GPU_RXQ_PKTS,
                                GPU_RXQ_PKTS * GPU_FRAME_MAX) != MTCP_GPU_OK) {
            TRACE_ERROR("gpu_module: no pinned staging\n");
            exit(EXIT_FAILURE);
        }
}

static int32_t gpu_link_devices(struct mtcp_thread_context *ctx)
{
    return INNER_CALL(ctx, gpu_inner_module->link_devices(ctx));
}

static void gpu_release_pkt(struct mtcp_thread_context *ctx, int ifidx,
                            unsigned char *pkt_data, int len)
{
    struct gpu_private_context *g = ctx->io_private_context;
    /* staged copies need no release; the originals went back at recv time */
    if (g->passthrough)
        INNER_VOID(ctx, gpu_inner_module->release_pkt(ctx, ifidx, pkt_data, len));
}

static uint8_t *gpu_get_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
    return INNER_CALL(ctx, gpu_inner_module->get_wptr(ctx, ifidx, len));
}

static int32_t gpu_send_pkts(struct mtcp_thread_context *ctx, int nif)
{
    return INNER_CALL(ctx, gpu_inner_module->send_pkts(ctx, nif));
}

static int32_t gpu_recv_pkts(struct mtcp_thread_context *ctx, int ifidx)
{
    struct gpu_private_context *g = ctx->io_private_context;
    mtcp_gpu_rxq *q = g->rxq[ifidx];
    uint32_t total = 0, n_done = 0;
    int b, i;

    if (g->passthrough)
        return INNER_CALL(ctx, gpu_inner_module->recv_pkts(ctx, ifidx));
    mtcp_gpu_rxq_reset(q);
    for (b = 0; b < GPU_AGG_BURSTS; b++) {
        int32_t n = INNER_CALL(ctx, gpu_inner_module->recv_pkts(ctx, ifidx));
        if (n <= 0)
            break;
        for (i = 0; i < n && total < GPU_RXQ_PKTS; i++) {
            uint16_t len = 0;
            uint8_t *p = INNER_CALL(ctx, gpu_inner_module->get_rptr(ctx, ifidx, i, &len));
            g->dropped[ifidx][total] = (p == NULL);
            if (mtcp_gpu_rxq_push(q, p, p ? len : 0) != MTCP_GPU_OK)
                break;
            total++;
        }
        if (n < GPU_BURST || total + GPU_BURST > GPU_RXQ_PKTS)
            break;                                   /* nothing more waiting */
    }
    g->served_raw[ifidx] = 1;
    if (total && g->gpu) {
        if (mtcp_gpu_rxq_flush(q, &n_done) == MTCP_GPU_OK && n_done == total)
            g->served_raw[ifidx] = 0;
        else {
            TRACE_ERROR("gpu_module: GPU rx failed; software checksums from now on\n");
            mtcp_gpu_close(g->gpu);
            g->gpu = NULL;
        }
    }
    return (int32_t)total;
}

static uint8_t *gpu_get_rptr(struct mtcp_thread_context *ctx, int ifidx, int index,
                             uint16_t *len)
{
    struct gpu_private_context *g = ctx->io_private_context;
    if (g->passthrough)
        return INNER_CALL(ctx, gpu_inner_module->get_rptr(ctx, ifidx, index, len));
    if (g->dropped[ifidx][index])
        return NULL;
    if (g->served_raw[ifidx])
        return mtcp_gpu_rxq_frame(g->rxq[ifidx], (uint32_t)index, len);
    return mtcp_gpu_rxq_get(g->rxq[ifidx], (uint32_t)index, len, NULL);
}

static int32_t gpu_select(struct mtcp_thread_context *ctx)
{
    return INNER_CALL(ctx, gpu_inner_module->select(ctx));
}

static void gpu_destroy_handle(struct mtcp_thread_context *ctx)
{
    struct gpu_private_context *g = ctx->io_private_context;
    int i;

    for (i = 0; i < MAX_DEVICES; i++)
        mtcp_gpu_rxq_destroy(g->rxq[i]);           /* NULL-safe */
    if (g->gpu)
        mtcp_gpu_close(g->gpu);
    INNER_VOID(ctx, gpu_inner_module->destroy_handle(ctx));
    ctx->io_private_context = g->inner;
    free(g);
}

static int32_t gpu_dev_ioctl(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp)
{
    struct gpu_private_context *g = ctx->io_private_context;

    switch (cmd) {
    case PKT_RX_IP_CSUM:
    case PKT_RX_TCP_CSUM:
        /* verified on the GPU at recv time: bad frames never reach mTCP */
        if (g->passthrough)
            break;
        return (g->gpu && !g->served_raw[nif]) ? 0 : -1;
    default:
        if (!g->passthrough && (cmd == PKT_TX_IP_CSUM || cmd == PKT_TX_TCP_CSUM ||
                                cmd == PKT_TX_TCPIP_CSUM || cmd == PKT_TX_TCPIP_CSUM_PEEK))
            return -1;                        /* tx: mTCP computes (see above) */
        break;
    }
    if (gpu_inner_module->dev_ioctl == NULL)
        return -1;
    return INNER_CALL(ctx, gpu_inner_module->dev_ioctl(ctx, nif, cmd, argp));
}

io_module_func gpu_module_func = {
    .load_module    = gpu_load_module,
    .init_handle    = gpu_init_handle,
    .link_devices   = gpu_link_devices,
    .release_pkt    = gpu_release_pkt,
    .get_wptr       = gpu_get_wptr,
    .send_pkts      = gpu_send_pkts,
    .get_rptr       = gpu_get_rptr,
    .recv_pkts      = gpu_recv_pkts,
    .select         = gpu_select,
    .destroy_handle = gpu_destroy_handle,
    .dev_ioctl      = gpu_dev_ioctl,
};
