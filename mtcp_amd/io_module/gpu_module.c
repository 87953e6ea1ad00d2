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
 * an rxq's pinned staging (the backend recycles its buffers on the next
 * receive: psio_module.c:244-246, dpdk_module.c:395-398), and runs the rx
 * kernel once over the aggregate.  Pipelined (the default): each interface
 * has two rxqs; recv_pkts starts the GPU on the aggregate it just gathered
 * and returns the PREVIOUS aggregate, checked meanwhile, so that the GPU's
 * copies and kernel overlap the gathering and mTCP's processing (one
 * aggregate of added latency; the first call of a burst returns 0, which
 * RunMainLoop's poll loop simply repeats; an aggregate is returned by the
 * next call even when nothing new arrives).  MTCP_GPU_PIPELINE=0 in the
 * environment: gather, check and return the same aggregate in one call.
 * get_rptr then serves the staged frames and returns NULL for the frames
 * whose IP or TCP
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
    int passthrough;                      /* no GPU at init: the inner backend */
    int pipeline;                         /* serve aggregate k while k+1 is checked */
    /* per rx interface, two aggregates (pipelined; synchronous uses [0]) */
    mtcp_gpu_rxq *rxq[MAX_DEVICES][2];
    uint8_t dropped[MAX_DEVICES][2][GPU_RXQ_PKTS];   /* inner get_rptr gave NULL */
    uint32_t count[MAX_DEVICES][2];       /* frames gathered                 */
    int launched[MAX_DEVICES][2];         /* on the GPU (flush_async went out) */
    int served_raw[MAX_DEVICES][2];       /* no verdicts: serve raw, ioctl -1 */
    int pending[MAX_DEVICES];             /* aggregate the next recv returns, -1 none */
    int serving[MAX_DEVICES];             /* aggregate get_rptr answers from */
};

/* After any GPU error: let the queued work finish, then software checksums
 * from now on (dev_ioctl answers -1). */
static void gpu_fail(struct gpu_private_context *g)
{
    int i, b;
    TRACE_ERROR("gpu_module: GPU rx failed; software checksums from now on\n");
    for (i = 0; i < MAX_DEVICES; i++)
        for (b = 0; b < 2; b++)
            if (g->rxq[i][b])
                (void)mtcp_gpu_rxq_wait(g->rxq[i][b], NULL);
    if (g->gpu)
        mtcp_gpu_close(g->gpu);
    g->gpu = NULL;
}

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
    const char *pl = getenv("MTCP_GPU_PIPELINE");
    int i, b, ndev;

    if (!g) {
        TRACE_ERROR("gpu_module: out of memory\n");
        exit(EXIT_FAILURE);
    }
    gpu_inner_module->init_handle(ctx);       /* sets ctx->io_private_context */
    g->inner = ctx->io_private_context;
    ctx->io_private_context = g;
    g->pipeline = !(pl && strcmp(pl, "0") == 0);
    for (i = 0; i < MAX_DEVICES; i++)
        g->pending[i] = g->serving[i] = -1;

    ndev = mtcp_gpu_device_count();
    if (ndev <= 0 || mtcp_gpu_open(&g->gpu, ctx->cpu % ndev, NULL, 1, 0) != MTCP_GPU_OK) {
        g->gpu = NULL;
        g->passthrough = 1;                  /* behave exactly like the inner */
        return;
    }
    for (i = 0; i < MAX_DEVICES; i++)
        for (b = 0; b < (g->pipeline ? 2 : 1); b++)
            if (mtcp_gpu_rxq_create(&g->rxq[i][b], g->gpu, GPU_RXQ_PKTS,
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

/* Pull up to GPU_AGG_BURSTS bursts from the wrapped backend into aggregate
 * a of interface ifidx and start the GPU on it; returns the frame count. */
static uint32_t gather(struct mtcp_thread_context *ctx, int ifidx, int a)
{
    struct gpu_private_context *g = ctx->io_private_context;
    mtcp_gpu_rxq *q = g->rxq[ifidx][a];
    uint32_t total = 0;
    int b, i;

    mtcp_gpu_rxq_reset(q);
    for (b = 0; b < GPU_AGG_BURSTS; b++) {
        int32_t n = INNER_CALL(ctx, gpu_inner_module->recv_pkts(ctx, ifidx));
        if (n <= 0)
            break;
        for (i = 0; i < n && total < GPU_RXQ_PKTS; i++) {
            uint16_t len = 0;
            uint8_t *p = INNER_CALL(ctx, gpu_inner_module->get_rptr(ctx, ifidx, i, &len));
            g->dropped[ifidx][a][total] = (p == NULL);
            if (mtcp_gpu_rxq_push(q, p, p ? len : 0) != MTCP_GPU_OK)
                break;
            total++;
        }
        if (n < GPU_BURST || total + GPU_BURST > GPU_RXQ_PKTS)
            break;                                   /* nothing more waiting */
    }
    g->count[ifidx][a] = total;
    g->launched[ifidx][a] = 0;
    if (total && g->gpu) {
        if (mtcp_gpu_rxq_flush_async(q) == MTCP_GPU_OK)
            g->launched[ifidx][a] = 1;
        else
            gpu_fail(g);
    }
    return total;
}

/* Wait for aggregate a's verdicts (served raw if it has none). */
static void finish(struct gpu_private_context *g, int ifidx, int a)
{
    uint32_t n_done = 0;
    g->served_raw[ifidx][a] = 1;
    if (!g->launched[ifidx][a])
        return;
    if (mtcp_gpu_rxq_wait(g->rxq[ifidx][a], &n_done) == MTCP_GPU_OK &&
        n_done == g->count[ifidx][a] && g->gpu)
        g->served_raw[ifidx][a] = 0;
    else
        gpu_fail(g);
}

static int32_t gpu_recv_pkts(struct mtcp_thread_context *ctx, int ifidx)
{
    struct gpu_private_context *g = ctx->io_private_context;
    int a, p;
    uint32_t total;

    if (g->passthrough)
        return INNER_CALL(ctx, gpu_inner_module->recv_pkts(ctx, ifidx));
    if (!g->pipeline) {
        total = gather(ctx, ifidx, 0);
        finish(g, ifidx, 0);
        g->serving[ifidx] = 0;
        return (int32_t)total;
    }
    /* mTCP is done with the aggregate served last time: gather into the
     * one not on the GPU, start it, then return the one that is */
    p = g->pending[ifidx];
    a = p >= 0 ? 1 - p : 0;
    total = gather(ctx, ifidx, a);
    g->pending[ifidx] = total ? a : -1;
    g->serving[ifidx] = p;
    if (p < 0)
        return 0;                                    /* filling the pipeline */
    finish(g, ifidx, p);
    return (int32_t)g->count[ifidx][p];
}

static uint8_t *gpu_get_rptr(struct mtcp_thread_context *ctx, int ifidx, int index,
                             uint16_t *len)
{
    struct gpu_private_context *g = ctx->io_private_context;
    int a;
    if (g->passthrough)
        return INNER_CALL(ctx, gpu_inner_module->get_rptr(ctx, ifidx, index, len));
    a = g->serving[ifidx];
    if (a < 0 || g->dropped[ifidx][a][index])
        return NULL;
    if (g->served_raw[ifidx][a])
        return mtcp_gpu_rxq_frame(g->rxq[ifidx][a], (uint32_t)index, len);
    return mtcp_gpu_rxq_get(g->rxq[ifidx][a], (uint32_t)index, len, NULL);
}

static int32_t gpu_select(struct mtcp_thread_context *ctx)
{
    return INNER_CALL(ctx, gpu_inner_module->select(ctx));
}

static void gpu_destroy_handle(struct mtcp_thread_context *ctx)
{
    struct gpu_private_context *g = ctx->io_private_context;
    int i;

    for (i = 0; i < MAX_DEVICES; i++) {
        mtcp_gpu_rxq_destroy(g->rxq[i][0]);        /* NULL-safe; waits for its stream */
        mtcp_gpu_rxq_destroy(g->rxq[i][1]);
    }
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
        return (g->gpu && g->serving[nif] >= 0 && !g->served_raw[nif][g->serving[nif]]) ? 0 : -1;
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
