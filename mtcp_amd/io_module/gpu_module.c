/*
 * gpu_module.c — the "gpu" I/O module for mTCP: an
 * io_module_func backend (mtcp/src/include/io_module.h:56-68) that wraps the
 * real driver backend (psio or dpdk), checks received frames on the MI355X
 * in aggregated launches, fills transmitted frames' checksums on it, and
 * answers mTCP's checksum offload hooks.
 *
 * Built inside the mTCP tree, against its headers (mtcp.h, io_module.h,
 * tcp_util.h) and include/mtcp_gpu.h + include/mtcp_gpu_rxq.h; link
 * -lmtcp_gpu.  Wiring, as for the other backends (io_module.h:93-112,
 * config.c:569-570):
 *
 *     extern io_module_func gpu_module_func;
 *     AssignIOModule: else if (!strcmp(m, "gpu")) current_iomodule_func = &gpu_module_func;
 *     mtcp.conf:      io = gpu   (+ the wrapped backend in gpu_inner_module)
 *
 * mTCP must be built WITHOUT --disable-hwcsum so that it asks dev_ioctl
 * first (ip_in.c:28-31, tcp_in.c:1159-1164, ip_out.c:147-161,
 * tcp_out.c:320-324).
 *
 * Receive (RunMainLoop, core.c:763-777): recv_pkts pulls up to
 * GPU_AGG_BURSTS bursts from the wrapped backend, copying each frame into
 * an rxq's pinned staging (the backend recycles its buffers on the next
 * receive: psio_module.c:244-246, dpdk_module.c:395-398), and runs the rx
 * kernel once over the aggregate.  Pipelined (the default): each interface
 * has two rxqs; recv_pkts starts the GPU on the aggregate it just gathered
 * and returns the PREVIOUS aggregate, checked meanwhile (one aggregate of
 * added latency; the first call of a burst returns 0, which RunMainLoop's
 * poll loop simply repeats; an aggregate is returned by the next call even
 * when nothing new arrives).  MTCP_GPU_PIPELINE=0 in the environment:
 * gather, check and return the same aggregate in one call.  get_rptr then
 * serves the staged frames and returns NULL for the frames whose IP or TCP
 * checksum fails — the packets mTCP's software path drops with ERROR
 * (ip_in.c:35-36, tcp_in.c:1167-1173) — and for the frames whose headers
 * claim more bytes than the frame holds (the reference would read past the
 * frame there); core.c:774-775 counts them as rx_errors, the pattern
 * dpdk_get_rptr uses for NIC-verified checksums (dpdk_module.c:473-479).
 * dev_ioctl(PKT_RX_IP_CSUM / PKT_RX_TCP_CSUM) answers 0 while the GPU path
 * of that interface is healthy and -1 otherwise, so mTCP falls back to its
 * own checksums exactly as with a NIC that lacks the offload
 * (dpdk_dev_ioctl, dpdk_module.c:809-816).  Every wait on the GPU — receive,
 * transmit, init_handle's and destroy_handle's — is bounded
 * (MTCP_GPU_WAIT_TIMEOUT_MS, default 2000, 0: none; clamped to 4294967; set
 * on the thread's context with mtcp_gpu_set_wait_limit): a GPU that stops
 * answering is abandoned, never waited on again, and mTCP checks and fills
 * every frame from then on.
 * NETSTAT: a frame dropped here never reaches ProcessPacket, so get_rptr
 * counts it in rx_packets / rx_bytes as ProcessPacket would have
 * (eth_in.c:20-23) and core.c:774-775 counts the NULL in rx_errors: the three
 * counters equal the --disable-hwcsum path's (tests/test_dropin.py).
 *
 * Transmit, with MTCP_GPU_TX=1 in the environment (psio or dpdk underneath;
 * refused over netmap, whose get_wptr sends the previous frame): dev_ioctl
 * (PKT_TX_TCPIP_CSUM_PEEK / PKT_TX_TCPIP_CSUM) answers 0, so mTCP leaves
 * iph->check and tcph->check for the device; get_wptr records every frame
 * it hands out, and send_pkts fills the recorded frames' checksums on the
 * GPU (mtcp_gpu_tx_fill_ptrs: only the two check fields are written) before
 * the wrapped backend sends them.  ICMP's IP checksum (PKT_TX_IP_CSUM) stays
 * with mTCP.  The fill waits at most MTCP_GPU_WAIT_TIMEOUT_MS
 * (mtcp_gpu_tx_fill_ptrs_for), as mTCP's own fill never waits on a device
 * (tcp_out.c:320-329, ip_out.c:147-165, core.c:818-824).  If the GPU fails
 * or does not answer in time at send time (or at destroy_handle's last
 * flush), the recorded frames are filled with mTCP's own ip_fast_csum /
 * TCPCalcChecksum, the GPU is abandoned and every later answer is -1.
 * Off by default: send_pkts is synchronous and mTCP calls it every loop
 * with at most a burst (64 frames on DPDK, MAX_PKT_BURST), so each send pays
 * a GPU round trip (gather, H2D, kernel, D2H) that costs more than the CPU's
 * own fill of 64 frames (measured: DESIGN.md §7).
 *
 * Device: the thread's GPU context opens a device on its core's NUMA node,
 * dealt round-robin among that node's devices (gpu_topo.h; mTCP binds each
 * thread's memory to its core's node, mtcp/src/cpu.c:54-79, and DPDK puts
 * each port's queues on the NIC's socket, dpdk_module.c:660-663);
 * MTCP_GPU_DEVICE=d forces one.  Admission: at most GPU_THREADS_DEFAULT
 * (2) mTCP threads per GPU offload; the others pass through and mTCP checks
 * their frames itself (dev_ioctl -1), as dpdk_module.c claims an offload
 * only where the device has it (dpdk_module.c:809-816): past two threads a
 * GPU's PCIe link is full and an offloading thread waits on it while its
 * core could check the frames; where 4 or more mTCP threads
 * share a GPU (mtcp.conf's num_cores over the GPUs) none offloads by
 * default.  MTCP_GPU_THREADS=k sets another limit, MTCP_GPU_THREADS=all
 * admits every thread.
 *
 * Fault injection (MTCP_GPU_FAIL_AFTER, MTCP_GPU_STALL_AFTER /
 * MTCP_GPU_TX_STALL_AFTER / MTCP_GPU_STALL_US) exists only in test builds (-DMTCP_GPU_TESTING, linked
 * with tests/c/libmtcp_gpu_testing.so); a production build ignores those
 * variables.
 *
 * Resources per mTCP thread: one GPU context with one HIP stream, which
 * carries the thread's rx aggregates and its tx fills alike (with the
 * default two offloading threads a GPU's streams take two of the
 * GPU_MAX_HW_QUEUES hardware queues, 4 by default, so one thread's stalled
 * GPU work never delays the other's; an admission past the queue count is
 * logged with TRACE_CONFIG), and, for each
 * of the CONFIG.eths_num interfaces (mtcp.h:138), two rxqs (pinned staging
 * of GPU_AGG_BURSTS x GPU_BURST frames of up to GPU_FRAME_MAX bytes each,
 * plus a device copy), created at init_handle, off the data path (a pinned
 * allocation and a stream's first copies take milliseconds); an interface
 * whose rxqs cannot be created runs on the wrapped backend alone.  Nothing
 * here calls exit().
 */
#include <stdlib.h>
#include <string.h>

#include "mtcp.h"
#include "io_module.h"
#include "debug.h"            /* brings tcp_in.h: struct iphdr / tcphdr, ntohs */
#include "tcp_util.h"

#include "mtcp_gpu.h"
#include "mtcp_gpu_rxq.h"
#include "gpu_topo.h"
#ifdef MTCP_GPU_TESTING
#include "mtcp_gpu_testing.h"     /* mtcp_gpu_debug_stall (tests/c) */
#endif

#define GPU_AGG_BURSTS 64                 /* bursts per GPU launch           */
#define GPU_BURST      64                 /* PS_CHUNK_SIZE / MAX_PKT_BURST   */
#define GPU_RXQ_PKTS   (GPU_AGG_BURSTS * GPU_BURST)
#define GPU_FRAME_MAX  2048ull            /* MAX_PACKET_SIZE (ps.h:173)      */
#define GPU_FRAME_JUMBO 9216ull           /* the largest frame a burst is expected to bring */
#define GPU_TX_MAX     4096               /* frames recorded between two send_pkts */
#define GPU_THREADS_DEFAULT 2             /* offloading threads per GPU */
#define GPU_CROWDED_THREADS 4             /* mTCP threads per GPU from which, by default,
                                             none offloads */
#define GPU_STREAMS_PER_THREAD 1          /* a thread's GPU context runs its rx aggregates and
                                             tx fills on its one stream (include/mtcp_gpu.h) */

/* the backend being wrapped (e.g. &ps_module_func or &dpdk_module_func) */
io_module_func *gpu_inner_module;

/* netmap's get_wptr transmits the PREVIOUS frame and hands out one reused
 * buffer (netmap_get_wptr, netmap_module.c:139-151): a frame has left before
 * send_pkts, where the tx fill runs.  The tx offload is refused over it.
 * Weak: harnesses that link no netmap module leave it NULL. */
extern io_module_func netmap_module_func __attribute__((weak));

/* The wrapped backend hands out separate tx buffers and transmits them only
 * in send_pkts (psio: psio_module.c:154-245, dpdk: dpdk_module.c:282-370). */
static int gpu_tx_capable(const io_module_func *inner)
{
    return inner != NULL && inner != &netmap_module_func;
}

/* One receiving interface: two aggregates (pipelined; synchronous uses [0]). */
struct gpu_ifq {
    mtcp_gpu_rxq *rxq[2];
    uint8_t dropped[2][GPU_RXQ_PKTS];     /* inner get_rptr gave NULL */
    uint32_t count[2];                    /* frames gathered          */
    int launched[2];                      /* on the GPU (flush_async went out) */
    int served_raw[2];                    /* no verdicts: serve raw, ioctl -1 */
    int pending;                          /* aggregate the next recv returns, -1 none */
    int serving;                          /* aggregate get_rptr answers from */
};

/* Frames handed out by get_wptr since the last send_pkts of an interface. */
struct gpu_txq {
    uint8_t *pkt[GPU_TX_MAX];
    uint16_t len[GPU_TX_MAX];
    uint32_t n;
};

struct gpu_private_context {
    void *inner;                          /* the wrapped backend's context   */
    mtcp_gpu_ctx *gpu;                    /* NULL: software checksums        */
    int passthrough;                      /* no GPU at init: the inner backend */
    int pipeline;                         /* serve aggregate k while k+1 is checked */
    int tx;                               /* tx checksums filled here        */
#ifdef MTCP_GPU_TESTING
    long fail_after;                      /* MTCP_GPU_FAIL_AFTER: fault injection, -1 off */
    long stall_after;                     /* MTCP_GPU_STALL_AFTER: fault injection, -1 off */
    long tx_stall_after;                  /* MTCP_GPU_TX_STALL_AFTER: fault injection, -1 off */
    uint32_t stall_us;                    /* MTCP_GPU_STALL_US                */
#endif
    uint32_t wait_us;                     /* MTCP_GPU_WAIT_TIMEOUT_MS, 0: no limit */
    int slot_dev;                         /* device whose admission slot this thread holds, -1 */
    mtcp_gpu_ctx *hung;                   /* abandoned after a timed-out wait: never waited on */
    long launches;                        /* aggregates sent to the GPU       */
    long tx_fills;                        /* tx flushes sent to the GPU       */
    struct gpu_ifq *ifq[MAX_DEVICES];     /* created at init (or first recv_pkts) */
    int ifq_failed[MAX_DEVICES];          /* no staging: this interface passes through */
    struct gpu_txq *txq[MAX_DEVICES];
};

/* a context for threads whose own allocation failed: passthrough only */
static __thread struct gpu_private_context gpu_fallback_ctx;

/* A wait ran past MTCP_GPU_WAIT_TIMEOUT_MS: the GPU is not answering.
 * Software checksums from now on, without waiting for it again: every
 * aggregate still on it is abandoned (its frames are served unchecked and
 * mTCP checks them), and its context and staging are never freed (freeing
 * would wait for the device). */
static void gpu_abandon(struct gpu_private_context *g)
{
    int i, b;
    TRACE_ERROR("gpu_module: GPU did not answer within the wait limit; software checksums from now on\n");
    g->hung = g->gpu;
    g->gpu = NULL;
    for (i = 0; i < MAX_DEVICES; i++)
        if (g->ifq[i])
            for (b = 0; b < 2; b++)
                if (g->ifq[i]->rxq[b] && g->ifq[i]->launched[b]) {
                    (void)mtcp_gpu_rxq_wait_for(g->ifq[i]->rxq[b], NULL, 1);
                    g->ifq[i]->launched[b] = 0;
                }
}

/* After any GPU error: let the queued work finish (each wait bounded by
 * MTCP_GPU_WAIT_TIMEOUT_MS: a device that does not finish it is abandoned
 * instead), then software checksums from now on (dev_ioctl answers -1). */
static void gpu_fail(struct gpu_private_context *g)
{
    int i, b;
    TRACE_ERROR("gpu_module: GPU path failed; software checksums from now on\n");
    for (i = 0; i < MAX_DEVICES; i++)
        if (g->ifq[i])
            for (b = 0; b < 2; b++)
                if (g->ifq[i]->rxq[b] &&
                    mtcp_gpu_rxq_wait_for(g->ifq[i]->rxq[b], NULL, g->wait_us) == MTCP_GPU_ETIMEDOUT &&
                    g->gpu) {
                    gpu_abandon(g);              /* never waited on (or closed) again */
                    return;
                }
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

/* The rx state of interface ifidx (created at init for CONFIG.eths_num
 * interfaces, on first use for any other); NULL: the interface runs on the
 * wrapped backend alone. */
static struct gpu_ifq *gpu_ifq_get(struct gpu_private_context *g, int ifidx)
{
    struct gpu_ifq *f = g->ifq[ifidx];
    int b;

    if (f || g->ifq_failed[ifidx] || !g->gpu)
        return f;
    f = calloc(1, sizeof(*f));
    for (b = 0; f && b < (g->pipeline ? 2 : 1); b++)
        if (mtcp_gpu_rxq_create(&f->rxq[b], g->gpu, GPU_RXQ_PKTS,
                                GPU_RXQ_PKTS * GPU_FRAME_MAX) != MTCP_GPU_OK) {
            TRACE_ERROR("gpu_module: no staging for interface %d; it runs on the wrapped backend\n",
                        ifidx);
            mtcp_gpu_rxq_destroy(f->rxq[0]);
            free(f);
            f = NULL;
        }
    if (!f) {
        g->ifq_failed[ifidx] = 1;
        return NULL;
    }
    f->pending = f->serving = -1;
    g->ifq[ifidx] = f;
    return f;
}

/* The device of the mTCP thread on `cpu`: one on the core's NUMA node
 * (gpu_topo.h); MTCP_GPU_DEVICE=d in the environment forces device d. */
static int gpu_pick_device(int cpu, int ndev)
{
    const char *forced = getenv("MTCP_GPU_DEVICE");
    const char *sysfs = gpu_topo_sysfs();
    int dev_node[GPU_TOPO_MAX_DEVS], d, rank = 0, node;

    if (forced && *forced) {
        d = atoi(forced);
        return d >= 0 && d < ndev ? d : -1;
    }
    if (ndev > GPU_TOPO_MAX_DEVS)
        ndev = GPU_TOPO_MAX_DEVS;
    for (d = 0; d < ndev; d++) {
        char bdf[64];
        dev_node[d] = mtcp_gpu_device_pci_bus_id(d, bdf, (int)sizeof(bdf)) == MTCP_GPU_OK
                          ? gpu_topo_pci_node(sysfs, bdf) : -1;
    }
    node = gpu_topo_cpu_node(sysfs, cpu, &rank);
    return gpu_topo_pick(cpu, node, rank, ndev, dev_node);
}

/* Admission: at most k mTCP threads per GPU offload; the others run on the
 * wrapped backend alone (dev_ioctl -1: mTCP's own checksums).  One GPU's
 * PCIe link carries the frames of about two threads, so
 * threads beyond that would wait on the link while their cores could check
 * frames themselves.  k = GPU_THREADS_DEFAULT, except where a GPU is shared
 * by GPU_CROWDED_THREADS (4) or more mTCP threads (CONFIG.num_cores,
 * mtcp.h:147, over the GPUs): there an offloading thread runs no faster than
 * a thread checking its own frames (from 4 threads on, offloading and
 * software threads at the same per-thread rate and the default at 0.92-1.00
 * of no offload in three rounds of paired runs) and its
 * frames cost the host two more passes over memory (the copy into pinned
 * staging and the DMA read) and more CPU per frame, so by default none
 * offloads; at 1-3 threads per GPU two offload (1.6-1.9x at 1-2 threads).  MTCP_GPU_THREADS=k sets the limit
 * ("all": no limit).  A thread holds its slot from a successful open until
 * destroy_handle (gpu_thread_release). */
static int gpu_thread_count[GPU_TOPO_MAX_DEVS];

/* mTCP threads per GPU in this process (0: unknown) */
static int gpu_threads_per_gpu(int ndev)
{
    return ndev > 0 && CONFIG.num_cores > 0 ? (CONFIG.num_cores + ndev - 1) / ndev : 0;
}

static int gpu_thread_limit(int per_gpu)
{
    const char *lim = getenv("MTCP_GPU_THREADS");
    if (!lim || !*lim)
        return per_gpu >= GPU_CROWDED_THREADS ? 0 : GPU_THREADS_DEFAULT;
    if (strcmp(lim, "all") == 0)
        return -1;
    return atoi(lim) < 0 ? 0 : atoi(lim);
}

/* Returns the thread's place among the device's offloading threads (1, 2,
 * ...), or 0 when it is refused. */
static int gpu_thread_admit(int dev, int per_gpu)
{
    const int lim = gpu_thread_limit(per_gpu);  /* -1: no limit (still counted) */
    int n;
    if (dev < 0 || dev >= GPU_TOPO_MAX_DEVS)
        return 1;
    n = __sync_add_and_fetch(&gpu_thread_count[dev], 1);
    if (n <= lim || lim < 0)
        return n;
    __sync_sub_and_fetch(&gpu_thread_count[dev], 1);
    return 0;
}

/* HIP maps a process's streams on a device onto GPU_MAX_HW_QUEUES hardware
 * queues (4 unless the environment sets it).  Up to that many streams never
 * share one, so a thread whose GPU work stalls holds up no other thread's;
 * past it two threads' streams can share a queue and one's stall delays the
 * other's aggregates.  True when the n-th offloading thread on a device is
 * past that point. */
static int gpu_hw_queues(void)
{
    const char *e = getenv("GPU_MAX_HW_QUEUES");
    int q = e && *e ? atoi(e) : 4;
    return q > 0 ? q : 4;
}

static int gpu_queues_shared(int n)
{
    return n * GPU_STREAMS_PER_THREAD > gpu_hw_queues();
}

static void gpu_thread_release(struct gpu_private_context *g)
{
    if (g->slot_dev >= 0 && g->slot_dev < GPU_TOPO_MAX_DEVS)
        __sync_sub_and_fetch(&gpu_thread_count[g->slot_dev], 1);
    g->slot_dev = -1;
}

/* MTCP_GPU_WAIT_TIMEOUT_MS in microseconds: default 2000 ms; negative or 0:
 * no limit; at most 4294967 ms (the limit is a 32-bit count of us) */
static uint32_t gpu_wait_us(void)
{
    const char *e = getenv("MTCP_GPU_WAIT_TIMEOUT_MS");
    long long ms = e && *e ? strtoll(e, NULL, 10) : 2000;
    if (ms <= 0)
        return 0;
    if (ms > 4294967ll)
        ms = 4294967ll;
    return (uint32_t)(ms * 1000);
}

static void gpu_init_handle(struct mtcp_thread_context *ctx)
{
    struct gpu_private_context *g = calloc(1, sizeof(*g));
    const char *pl = getenv("MTCP_GPU_PIPELINE");
    const char *tx = getenv("MTCP_GPU_TX");
    int ndev, dev, place, per_gpu, i;

    gpu_inner_module->init_handle(ctx);       /* sets ctx->io_private_context */
    if (!g) {
        TRACE_ERROR("gpu_module: out of memory; running on the wrapped backend\n");
        g = &gpu_fallback_ctx;
        memset(g, 0, sizeof(*g));
        g->passthrough = 1;
    }
    g->slot_dev = -1;
    g->inner = ctx->io_private_context;
    ctx->io_private_context = g;
    if (g->passthrough)
        return;
    g->pipeline = !(pl && strcmp(pl, "0") == 0);
    g->tx = tx && strcmp(tx, "1") == 0;
#ifdef MTCP_GPU_TESTING
    /* MTCP_GPU_FAIL_AFTER=k: the (k+1)-th aggregate's launch fails as a GPU
     * error would, so the fallback to mTCP's own checksums is exercised on a
     * healthy GPU (tests/test_dropin.py) */
    g->fail_after = getenv("MTCP_GPU_FAIL_AFTER") ? atol(getenv("MTCP_GPU_FAIL_AFTER")) : -1;
    /* MTCP_GPU_STALL_AFTER=k, MTCP_GPU_STALL_US=u: the (k+1)-th aggregate
     * waits u us on the GPU behind mtcp_gpu_debug_stall, so that the wait
     * limit (MTCP_GPU_WAIT_TIMEOUT_MS) and the fallback after it are
     * exercised on a healthy GPU */
    g->stall_after = getenv("MTCP_GPU_STALL_AFTER") ? atol(getenv("MTCP_GPU_STALL_AFTER")) : -1;
    g->stall_us = getenv("MTCP_GPU_STALL_US") ? (uint32_t)atol(getenv("MTCP_GPU_STALL_US")) : 0;
    /* MTCP_GPU_TX_STALL_AFTER=k: the (k+1)-th tx fill waits MTCP_GPU_STALL_US
     * behind mtcp_gpu_debug_stall (the bounded send_pkts) */
    g->tx_stall_after = getenv("MTCP_GPU_TX_STALL_AFTER") ? atol(getenv("MTCP_GPU_TX_STALL_AFTER")) : -1;
#endif
    g->wait_us = gpu_wait_us();
    if (g->tx && !gpu_tx_capable(gpu_inner_module)) {
        TRACE_ERROR("gpu_module: MTCP_GPU_TX=1 refused: the wrapped backend sends from get_wptr\n");
        g->tx = 0;
    }

    ndev = mtcp_gpu_device_count();
    dev = ndev > 0 ? gpu_pick_device(ctx->cpu, ndev) : -1;
    per_gpu = gpu_threads_per_gpu(ndev);
    place = dev >= 0 ? gpu_thread_admit(dev, per_gpu) : 0;
    if (dev >= 0 && !place) {
        /* said once per refused thread, at init: a deployment with more
         * threads than the limit per GPU sees where its offload went */
        if (gpu_thread_limit(per_gpu) == 0 && !getenv("MTCP_GPU_THREADS"))
            TRACE_CONFIG("gpu_module: core %d: %d mTCP threads share each GPU (>= %d): by default "
                         "none offloads and this thread checks its own frames "
                         "(MTCP_GPU_THREADS=k offloads k threads per GPU)\n",
                         ctx->cpu, per_gpu, GPU_CROWDED_THREADS);
        else
            TRACE_CONFIG("gpu_module: core %d: GPU %d already serves %d mTCP threads "
                         "(MTCP_GPU_THREADS, default %d); this thread checks its own frames "
                         "(MTCP_GPU_THREADS=all offloads every thread)\n",
                         ctx->cpu, dev, gpu_thread_limit(per_gpu), GPU_THREADS_DEFAULT);
        g->passthrough = 1;                  /* mTCP's own checksums on this core */
        return;
    }
    if (dev >= 0 && gpu_queues_shared(place))
        TRACE_CONFIG("gpu_module: core %d: offloading thread %d on GPU %d needs more than the "
                     "%d hardware queues of GPU_MAX_HW_QUEUES: its stream shares a queue with "
                     "another thread's, whose stalled GPU work can then delay it\n",
                     ctx->cpu, place, dev, gpu_hw_queues());
    g->slot_dev = dev;
    /* compact 16 B records: the rxqs read the verdict only (40 -> 16 B of D2H per frame);
     * every wait of the context (and of its rxqs) bounded by MTCP_GPU_WAIT_TIMEOUT_MS */
    if (dev < 0 || mtcp_gpu_open(&g->gpu, dev, NULL, 1, MTCP_GPU_F_COMPACT) != MTCP_GPU_OK ||
        mtcp_gpu_set_wait_limit(g->gpu, g->wait_us) != MTCP_GPU_OK ||
        mtcp_gpu_reserve(g->gpu, 0, 0) != MTCP_GPU_OK) {     /* load the kernels now */
        if (g->gpu)
            mtcp_gpu_close(g->gpu);
        g->gpu = NULL;
        g->passthrough = 1;                  /* behave exactly like the inner */
        gpu_thread_release(g);               /* the slot goes to a thread that opens */
        return;
    }
    for (i = 0; i < CONFIG.eths_num && i < MAX_DEVICES; i++)
        (void)gpu_ifq_get(g, i);
}

static int32_t gpu_link_devices(struct mtcp_thread_context *ctx)
{
    return INNER_CALL(ctx, gpu_inner_module->link_devices(ctx));
}

static void gpu_release_pkt(struct mtcp_thread_context *ctx, int ifidx,
                            unsigned char *pkt_data, int len)
{
    /* always the wrapped backend's: psio hands the frame to the host stack
     * (psio_release_pkt, psio_module.c:122-132, copies from pkt_data, here
     * the staged copy); dpdk's is a no-op */
    if (gpu_inner_module->release_pkt)
        INNER_VOID(ctx, gpu_inner_module->release_pkt(ctx, ifidx, pkt_data, len));
}

/* ---- transmit --------------------------------------------------------------- */

/* mTCP's own fills (ip_out.c:164, tcp_out.c:327-329) for the frames the GPU
 * did not fill; the same rule as mtcp_gpu_tx_fill (include/mtcp_gpu.h). */
static void gpu_tx_fill_sw(uint8_t *pkt, uint16_t len)
{
    struct iphdr *iph = (struct iphdr *)(pkt + 14);
    uint16_t proto = (uint16_t)((pkt[12] << 8) | pkt[13]);
    unsigned int ihl, doff, tot_len;
    struct tcphdr *tcph;

    if (len < 34 || proto != 0x0800)
        return;
    ihl = iph->ihl;
    tot_len = ntohs(iph->tot_len);
    if (iph->version != 4 || ihl < 5 || iph->protocol != 6 || len < 14 + 4 * ihl + 20)
        return;
    tcph = (struct tcphdr *)(pkt + 14 + 4 * ihl);
    doff = tcph->doff;
    if (doff < 5 || tot_len < 4 * (ihl + doff) || 14 + tot_len > len)
        return;
    iph->check = 0;
    iph->check = ip_fast_csum(iph, ihl);
    tcph->check = 0;
    tcph->check = TCPCalcChecksum((uint16_t *)tcph, (uint16_t)(tot_len - 4 * ihl),
                                  iph->saddr, iph->daddr);
}

/* Fill the checksums of the frames recorded for interface nif: on the GPU,
 * waiting at most MTCP_GPU_WAIT_TIMEOUT_MS; a GPU that does not report in
 * time is abandoned (nothing of it was written into the frames) and the
 * frames are filled here, as after any other GPU error. */
static void gpu_tx_flush(struct gpu_private_context *g, int nif)
{
    struct gpu_txq *t = g->txq[nif];
    uint32_t i;
    int rc;

    if (!t || !t->n)
        return;
    if (g->gpu) {
#ifdef MTCP_GPU_TESTING
        if (g->tx_fills == g->tx_stall_after)
            (void)mtcp_gpu_debug_stall(g->gpu, g->stall_us);
#endif
        g->tx_fills++;
        rc = mtcp_gpu_tx_fill_ptrs_for(g->gpu, t->pkt, t->len, t->n, NULL, g->wait_us);
        if (rc == MTCP_GPU_ETIMEDOUT)
            gpu_abandon(g);                   /* never waited on (or closed) again */
        else if (rc != MTCP_GPU_OK)
            gpu_fail(g);
    }
    if (!g->gpu)                              /* mTCP skipped these: fill them here */
        for (i = 0; i < t->n; i++)
            gpu_tx_fill_sw(t->pkt[i], t->len[i]);
    t->n = 0;
}

static uint8_t *gpu_get_wptr(struct mtcp_thread_context *ctx, int ifidx, uint16_t len)
{
    struct gpu_private_context *g = ctx->io_private_context;
    uint8_t *p = INNER_CALL(ctx, gpu_inner_module->get_wptr(ctx, ifidx, len));
    struct gpu_txq *t;

    if (!p || g->passthrough || !g->tx)
        return p;
    t = g->txq[ifidx];
    if (!t) {
        t = g->txq[ifidx] = calloc(1, sizeof(*t));
        if (!t) {
            /* nowhere to record it, and mTCP has been told the device fills
             * it: from now on mTCP computes tx checksums */
            g->tx = 0;
            return p;
        }
    }
    if (t->n == GPU_TX_MAX)
        gpu_tx_flush(g, ifidx);
    if (!g->gpu)
        return p;     /* abandoned: dev_ioctl answers -1, mTCP fills this frame itself */
    t->pkt[t->n] = p;
    t->len[t->n] = len;
    t->n++;
    return p;
}

static int32_t gpu_send_pkts(struct mtcp_thread_context *ctx, int nif)
{
    struct gpu_private_context *g = ctx->io_private_context;
    if (!g->passthrough)
        gpu_tx_flush(g, nif);
    return INNER_CALL(ctx, gpu_inner_module->send_pkts(ctx, nif));
}

/* ---- receive ---------------------------------------------------------------- */

/* Pull up to GPU_AGG_BURSTS bursts from the wrapped backend into aggregate
 * a of interface ifidx and start the GPU on it; returns the frame count. */
static uint32_t gather(struct mtcp_thread_context *ctx, struct gpu_ifq *f, int ifidx, int a)
{
    struct gpu_private_context *g = ctx->io_private_context;
    mtcp_gpu_rxq *q = f->rxq[a];
    uint32_t total = 0;
    uint64_t bytes = 0;                              /* staging used (64 B slots) */
    int b, i;

    mtcp_gpu_rxq_reset(q);
    for (b = 0; b < GPU_AGG_BURSTS; b++) {
        int32_t n;
        /* a burst is only pulled when the staging holds it even if every
         * frame is jumbo: a received burst cannot be left half staged (the
         * backend recycles its buffers on the next receive) */
        if (bytes + GPU_BURST * GPU_FRAME_JUMBO > GPU_RXQ_PKTS * GPU_FRAME_MAX)
            break;
        n = INNER_CALL(ctx, gpu_inner_module->recv_pkts(ctx, ifidx));
        if (n <= 0)
            break;
        for (i = 0; i < n && total < GPU_RXQ_PKTS; i++) {
            uint16_t len = 0;
            uint8_t *p = INNER_CALL(ctx, gpu_inner_module->get_rptr(ctx, ifidx, i, &len));
            f->dropped[a][total] = (p == NULL);
            if (mtcp_gpu_rxq_push(q, p, p ? len : 0) == MTCP_GPU_OK) {
                bytes += p ? ((uint64_t)len + 63) & ~63ull : 0;
            } else {
                /* larger than the room left (a frame above GPU_FRAME_JUMBO):
                 * served as NULL, counted in rx_errors (core.c:772-775) */
                f->dropped[a][total] = 1;
                if (mtcp_gpu_rxq_push(q, NULL, 0) != MTCP_GPU_OK)
                    break;                           /* cannot happen: total < GPU_RXQ_PKTS */
            }
            total++;
        }
        if (n < GPU_BURST || total + GPU_BURST > GPU_RXQ_PKTS)
            break;                                   /* nothing more waiting */
    }
    f->count[a] = total;
    f->launched[a] = 0;
    if (total && g->gpu) {
        int inject_fail = 0;
#ifdef MTCP_GPU_TESTING
        if (g->launches == g->stall_after)
            (void)mtcp_gpu_debug_stall(g->gpu, g->stall_us);
        inject_fail = g->fail_after >= 0 && g->launches >= g->fail_after;
#endif
        if (!inject_fail && mtcp_gpu_rxq_flush_async(q) == MTCP_GPU_OK) {
            f->launched[a] = 1;
            g->launches++;
        } else {
            gpu_fail(g);
        }
    }
    return total;
}

/* Wait for aggregate a's verdicts (served raw if it has none).  An aggregate
 * launched before a GPU failure keeps its verdicts: gpu_fail waited for it,
 * and the wait here then only reads the rxq's host-side state. */
static void finish(struct gpu_private_context *g, struct gpu_ifq *f, int a)
{
    uint32_t n_done = 0;
    int rc;
    f->served_raw[a] = 1;
    if (!f->launched[a])
        return;
    f->launched[a] = 0;
    rc = mtcp_gpu_rxq_wait_for(f->rxq[a], &n_done, g->wait_us);
    if (rc == MTCP_GPU_OK && n_done == f->count[a])
        f->served_raw[a] = 0;
    else if (rc == MTCP_GPU_ETIMEDOUT && g->gpu)
        gpu_abandon(g);
    else if (g->gpu)
        gpu_fail(g);
}

static int32_t gpu_recv_pkts(struct mtcp_thread_context *ctx, int ifidx)
{
    struct gpu_private_context *g = ctx->io_private_context;
    struct gpu_ifq *f = g->passthrough ? NULL : gpu_ifq_get(g, ifidx);
    int a, p;
    uint32_t total;

    if (!f)
        return INNER_CALL(ctx, gpu_inner_module->recv_pkts(ctx, ifidx));
    if (!g->pipeline) {
        total = gather(ctx, f, ifidx, 0);
        finish(g, f, 0);
        f->serving = 0;
        return (int32_t)total;
    }
    /* mTCP is done with the aggregate served last time: gather into the
     * one not on the GPU, start it, then return the one that is */
    p = f->pending;
    a = p >= 0 ? 1 - p : 0;
    total = gather(ctx, f, ifidx, a);
    f->pending = total ? a : -1;
    f->serving = p;
    if (p < 0)
        return 0;                                    /* filling the pipeline */
    finish(g, f, p);
    return (int32_t)f->count[p];
}

static uint8_t *gpu_get_rptr(struct mtcp_thread_context *ctx, int ifidx, int index,
                             uint16_t *len)
{
    struct gpu_private_context *g = ctx->io_private_context;
    struct gpu_ifq *f = g->passthrough ? NULL : g->ifq[ifidx];
    uint8_t *p;
    int a;
    if (!f)
        return INNER_CALL(ctx, gpu_inner_module->get_rptr(ctx, ifidx, index, len));
    a = f->serving;
    if (a < 0 || index < 0 || (uint32_t)index >= f->count[a])
        return NULL;                  /* not a frame of the burst recv_pkts returned */
    if (f->dropped[a][index])
        return NULL;                  /* the wrapped backend's own NULL */
    if (f->served_raw[a])
        return mtcp_gpu_rxq_frame(f->rxq[a], (uint32_t)index, len);
    p = mtcp_gpu_rxq_get(f->rxq[a], (uint32_t)index, len, NULL);
#ifdef NETSTAT
    if (!p && ctx->mtcp_manager) {
        /* a frame dropped on its GPU verdict never reaches ProcessPacket,
         * which counts every frame it is handed, checksum drops included
         * (eth_in.c:20-23): count it here, so that rx_packets / rx_bytes /
         * rx_errors (core.c:774-775) equal the software path's */
        struct mtcp_manager *m = ctx->mtcp_manager;
        m->nstat.rx_packets[ifidx]++;
        m->nstat.rx_bytes[ifidx] += *len + 24;
    }
#endif
    return p;
}

static int32_t gpu_select(struct mtcp_thread_context *ctx)
{
    return INNER_CALL(ctx, gpu_inner_module->select(ctx));
}

static void gpu_destroy_handle(struct mtcp_thread_context *ctx)
{
    struct gpu_private_context *g = ctx->io_private_context;
    int i, b;

    /* an aggregate still on the GPU (the pipeline's last one, when mTCP
     * stops with frames in flight): the same bounded wait as recv_pkts'; a
     * GPU that does not finish it is abandoned and its staging stays below */
    for (i = 0; i < MAX_DEVICES && g->gpu; i++)
        for (b = 0; b < 2 && g->gpu && g->ifq[i]; b++)
            if (g->ifq[i]->rxq[b] && g->ifq[i]->launched[b]) {
                if (mtcp_gpu_rxq_wait_for(g->ifq[i]->rxq[b], NULL, g->wait_us) == MTCP_GPU_ETIMEDOUT)
                    gpu_abandon(g);
                else
                    g->ifq[i]->launched[b] = 0;
            }
    for (i = 0; i < MAX_DEVICES; i++) {
        gpu_tx_flush(g, i);                          /* frames still recorded */
        free(g->txq[i]);
        if (g->ifq[i]) {
            if (!g->hung) {                          /* a hung GPU's staging stays */
                mtcp_gpu_rxq_destroy(g->ifq[i]->rxq[0]);   /* NULL-safe; nothing in flight */
                mtcp_gpu_rxq_destroy(g->ifq[i]->rxq[1]);
            }
            free(g->ifq[i]);
        }
    }
    if (g->gpu)
        mtcp_gpu_close(g->gpu);
    gpu_thread_release(g);
    INNER_VOID(ctx, gpu_inner_module->destroy_handle(ctx));
    ctx->io_private_context = g->inner;
    if (g != &gpu_fallback_ctx)
        free(g);
}

static int32_t gpu_dev_ioctl(struct mtcp_thread_context *ctx, int nif, int cmd, void *argp)
{
    struct gpu_private_context *g = ctx->io_private_context;
    struct gpu_ifq *f;

    if (!g->passthrough && nif >= 0 && nif < MAX_DEVICES) {
        switch (cmd) {
        case PKT_RX_IP_CSUM:
        case PKT_RX_TCP_CSUM:
            /* verified on the GPU at recv time: bad frames never reach mTCP */
            f = g->ifq[nif];
            if (f)      /* the frames being served carry GPU verdicts */
                return (f->serving >= 0 && !f->served_raw[f->serving]) ? 0 : -1;
            break;                                   /* a passthrough interface */
        case PKT_TX_TCPIP_CSUM_PEEK:
        case PKT_TX_TCPIP_CSUM:
            /* filled on the GPU at send_pkts (ICMP's PKT_TX_IP_CSUM stays with mTCP) */
            return g->gpu && g->tx ? 0 : -1;
        case PKT_TX_IP_CSUM:
        case PKT_TX_TCP_CSUM:
            return -1;
        default:
            break;
        }
    }
    if (gpu_inner_module->dev_ioctl == NULL)
        return -1;
    return INNER_CALL(ctx, gpu_inner_module->dev_ioctl(ctx, nif, cmd, argp));
}

#ifdef MTCP_GPU_TESTING
/* Test builds: the device a thread's context runs on, -1 when it passes
 * through (the multi-device test checks the NUMA choice with it). */
int gpu_module_thread_device(struct mtcp_thread_context *ctx)
{
    struct gpu_private_context *g = ctx->io_private_context;
    return g && g->gpu ? g->slot_dev : -1;
}
#endif

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
