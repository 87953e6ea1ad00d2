/*
 * mtcp_gpu.h — C ABI of the MI355X (gfx950) rx/tx checksum, parse and RSS
 * offload for mTCP's software (--disable-hwcsum) per-packet path.
 *
 * Plain C, no HIP or C++ types: a libmtcp built with
 * `gcc -O3 -fgnu89-inline -Werror` (mtcp/src/Makefile.in:20-31) includes this
 * header and links libmtcp_gpu.so.  Every entry point returns 0 or a negative
 * errno-style code (MTCP_GPU_E*); nothing here calls exit() or throws.
 *
 * What each entry point replaces in the reference (paths relative to the
 * mTCP tree):
 *
 *   mtcp_gpu_rx_chunk / _rx_chunk_dev
 *       the per-packet loop of RunMainLoop (mtcp/src/core.c:768-776), i.e.
 *       get_rptr (mtcp/src/include/io_module.h:62) + ProcessPacket
 *       (mtcp/src/eth_in.c:9-56) → ProcessIPv4Packet (mtcp/src/ip_in.c:15-62)
 *       → the head of ProcessTCPPacket (mtcp/src/tcp_in.c:1138-1175), run for
 *       a whole PSIO-style chunk (io_engine/include/ps.h:181-200) at once.
 *       Inside, ip_fast_csum (io_engine/include/ps.h:66-95) and
 *       TCPCalcChecksum (mtcp/src/tcp_util.c:157-190) are evaluated for every
 *       packet, and optionally GetRSSHash / GetRSSCPUCore
 *       (util/rss.c:107-165, mtcp/src/rss.c:44-103).
 *   mtcp_gpu_rx_ptrs / _rx_ptrs_dev
 *       the same for a DPDK/netmap style burst of (pointer, len) pairs
 *       (dpdk_get_rptr mtcp/src/dpdk_module.c:454-485,
 *        netmap_get_rptr mtcp/src/netmap_module.c:193-200).
 *   mtcp_gpu_tx_fill / _tx_fill_dev
 *       the DISABLE_HWCSUM checksum fills of the tx path:
 *       iph->check = ip_fast_csum(iph, iph->ihl)   (mtcp/src/ip_out.c:94,164)
 *       tcph->check = TCPCalcChecksum(...)          (mtcp/src/tcp_out.c:211,329)
 *   mtcp_gpu_tx_fill_ptrs / _tx_fill_ptrs_dev
 *       the same fills for a DPDK-style burst of frame pointers, the batch
 *       send_pkts hands to the NIC (wmbufs[ifidx].m_table,
 *       mtcp/src/dpdk_module.c:282-338, filled by get_wptr :341-370); what a
 *       NIC does after dev_ioctl(PKT_TX_TCPIP_CSUM[_PEEK]) answered 0
 *       (ip_out.c:147-161, tcp_out.c:320-324).
 *   mtcp_gpu_rx_chunk_flow_dev / _rx_ptrs_flow_dev
 *       rx as above plus HashFlow (mtcp/src/tcp_stream.c:56-90) of every
 *       TCP_OK packet's flow-table key in the same pass (no second launch
 *       over the records).
 *   mtcp_gpu_flow_hash / _flow_hash_dev
 *       HashFlow (mtcp/src/tcp_stream.c:56-90) of the flow-table lookup key
 *       (mtcp/src/tcp_in.c:1180-1186), the step after the checksums.
 *   mtcp_gpu_addr_pool_search / _rss_queue_map_dev
 *       the RSS-friendly address search of CreateAddressPoolPerCore
 *       (mtcp/src/addr_pool.c:155-178) over GetRSSCPUCore (mtcp/src/rss.c:90-103).
 *   mtcp_gpu_dev_ioctl
 *       io_module_func.dev_ioctl (mtcp/src/include/io_module.h:67) for the
 *       checksum commands PKT_RX_IP_CSUM / PKT_RX_TCP_CSUM / PKT_TX_IP_CSUM /
 *       PKT_TX_TCPIP_CSUM (io_module.h:80-87): 0 = "the device does it",
 *       -1 = "do it in software", the contract of dpdk_dev_ioctl
 *       (mtcp/src/dpdk_module.c:809-816).
 *
 * Ownership: packet memory belongs to the caller (the I/O module) and is
 * never retained past a call; rx never writes packets (the reference's
 * `tcph->check = 0` on a bad TCP checksum, tcp_in.c:1171, is reported through
 * the verdict only); results belong to the caller.
 *
 * Threading: one context per mTCP thread (mtcp/src/core.c:1057 pins one
 * thread per core); a context owns one HIP stream (mtcp_gpu_stream) and its
 * staging buffers and is not re-entrant.  Distinct contexts may be used
 * concurrently.  Everything a context does runs on that one stream — its
 * device-resident launches with stream NULL, its host-memory calls, its
 * rxqs' flushes (mtcp_gpu_rxq.h) — except a host-memory rx call over more
 * than 64 MiB, which pipelines through two more streams of its own.  HIP
 * maps a process's streams onto GPU_MAX_HW_QUEUES hardware queues per device
 * (4 by default): up to that many contexts on one device never share a
 * queue, so one context's stalled work cannot hold up another's.
 *
 * Waits: mtcp_gpu_set_wait_limit bounds every wait of every synchronous call
 * on a context (see there).  Without a limit the synchronous calls block
 * until the GPU is done, as hipStreamSynchronize does.
 */
#ifndef MTCP_GPU_H
#define MTCP_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MTCP_GPU_ABI_VERSION 5   /* 2: MTCP_GPU_F_COMPACT, mtcp_gpu_result16;
                                    3: mtcp_gpu_rxq_get16, mtcp_gpu_debug_stall moved to the test library;
                                    4: mtcp_gpu_tx_fill_ptrs_for, mtcp_gpu_host_stream,
                                       mtcp_gpu_size_hint, mtcp_gpu_rx_chunk_hint_dev;
                                    5: mtcp_gpu_set_wait_limit, mtcp_gpu_wait_limit (every
                                       synchronous call bounded); mtcp_gpu_host_stream removed
                                       (host calls run on mtcp_gpu_stream) */

/* ---- error codes (negative returns) ----------------------------------- */
#define MTCP_GPU_OK        0
#define MTCP_GPU_EINVAL   (-22)  /* bad argument (NULL, misaligned, too big) */
#define MTCP_GPU_ENOMEM   (-12)  /* device or pinned host allocation failed  */
#define MTCP_GPU_ENODEV   (-19)  /* no such HIP device / no GPU              */
#define MTCP_GPU_EIO       (-5)  /* HIP runtime error during the call        */
#define MTCP_GPU_ETIMEDOUT (-110) /* the GPU did not finish within the limit the caller set */

/* ---- dev_ioctl commands: same values as mtcp/src/include/io_module.h:80-87 */
#define MTCP_GPU_PKT_TX_IP_CSUM          0x01
#define MTCP_GPU_PKT_TX_TCP_CSUM         0x02
#define MTCP_GPU_PKT_RX_TCP_LROSEG       0x03
#define MTCP_GPU_PKT_TX_TCPIP_CSUM       0x04
#define MTCP_GPU_PKT_RX_IP_CSUM          0x05
#define MTCP_GPU_PKT_RX_TCP_CSUM         0x06
#define MTCP_GPU_PKT_TX_TCPIP_CSUM_PEEK  0x07
#define MTCP_GPU_DRV_NAME                0x08

/* ---- open flags -------------------------------------------------------- */
#define MTCP_GPU_F_RSS           0x1u  /* compute rss_hash / rss_queue per packet */
#define MTCP_GPU_F_RSS_ENDIAN    0x2u  /* GetRSSCPUCore endian fix (util/rss.c:161-162;
                                          mtcp/src/rss.c:96-99 endian_check) */
#define MTCP_GPU_F_COMPACT       0x4u  /* rx writes 16 B mtcp_gpu_result16 records (below)
                                          instead of the 40 B mtcp_gpu_result */

/*
 * Packet descriptor of a contiguous chunk.  Layout-compatible with PSIO's
 * struct ps_pkt_info {uint32_t offset; uint16_t len; uint8_t checksum_rx;}
 * (io_engine/include/ps.h:181-185), so a ps_chunk's info[] array can be
 * passed as is with off_shift = 0.  With off_shift = 6 the offset counts 64 B
 * units (PSIO aligns packets to 64 B, io_engine/lib/pslib.c:146), which
 * reaches 256 GiB chunks.  Byte offset = offset << off_shift; it must be
 * even (2-byte aligned frame starts, e.g. NET_IP_ALIGN buffers, are fine)
 * and offset + len must lie inside the chunk, otherwise the packet gets
 * MTCP_GPU_V_BAD_DESC and is not read.
 * len = frame length as get_rptr's *len (Ethernet header through the end of
 * the frame, CRC stripped; mtcp/src/dpdk_module.c:467).
 */
typedef struct mtcp_gpu_desc {
    uint32_t offset;
    uint16_t len;
    uint8_t  flags;      /* ignored (ps_pkt_info.checksum_rx) */
    uint8_t  rsvd;
} mtcp_gpu_desc;

/* Per-packet verdict: one value per exit of the reference's rx chain. */
enum mtcp_gpu_verdict {
    MTCP_GPU_V_TCP_OK         = 0,  /* checksums good, reached StreamHTSearch (tcp_in.c:1186) */
    MTCP_GPU_V_ETH_OTHER      = 1,  /* not IPv4/ARP: release, TRUE        (eth_in.c:43-46) */
    MTCP_GPU_V_ARP            = 2,  /* h_proto 0x0806                     (eth_in.c:39-41) */
    MTCP_GPU_V_IP_SHORT       = 3,  /* tot_len < 20, ERROR                (ip_in.c:25-26)  */
    MTCP_GPU_V_IP_CSUM_BAD    = 4,  /* ip_fast_csum != 0, ERROR           (ip_in.c:35-36)  */
    MTCP_GPU_V_IP_VERSION     = 5,  /* version != 4, release, FALSE       (ip_in.c:47-50)  */
    MTCP_GPU_V_ICMP           = 6,  /* protocol 1 -> ProcessICMPPacket    (ip_in.c:55-56)  */
    MTCP_GPU_V_IP_PROTO_OTHER = 7,  /* other protocol, FALSE              (ip_in.c:57-59)  */
    MTCP_GPU_V_TCP_LEN_BAD    = 8,  /* tot_len < 4*(ihl+doff), ERROR      (tcp_in.c:1155-1156) */
    MTCP_GPU_V_TCP_CSUM_BAD   = 9,  /* TCPCalcChecksum != 0, ERROR; the reference also
                                       sets tcph->check = 0               (tcp_in.c:1167-1173) */
    MTCP_GPU_V_TRUNCATED      = 10, /* the reference would read past len here (undefined) */
    MTCP_GPU_V_BAD_DESC       = 11  /* descriptor outside the chunk or misaligned */
};

/* ProcessPacket's `ret < 0` (eth_in.c:49-53): the verdicts counted in
 * nstat.rx_errors. */
#define MTCP_GPU_VERDICT_IS_RX_ERROR(v) \
    ((v) == MTCP_GPU_V_IP_SHORT || (v) == MTCP_GPU_V_IP_CSUM_BAD || \
     (v) == MTCP_GPU_V_TCP_LEN_BAD || (v) == MTCP_GPU_V_TCP_CSUM_BAD)

/*
 * Per-packet result, 40 B.  A field is written only once the reference's
 * rx chain has read it; everything else is 0.  Byte orders follow the
 * reference's own variables.
 */
typedef struct mtcp_gpu_result {
    uint32_t saddr;       /*  0 iph->saddr, as in memory (network order)       */
    uint32_t daddr;       /*  4 iph->daddr, as in memory                       */
    uint16_t sport;       /*  8 tcph->source, as in memory                     */
    uint16_t dport;       /* 10 tcph->dest, as in memory                       */
    uint32_t seq;         /* 12 ntohl(tcph->seq)        tcp_in.c:1147          */
    uint32_t ack_seq;     /* 16 ntohl(tcph->ack_seq)    tcp_in.c:1148          */
    uint16_t window;      /* 20 ntohs(tcph->window)     tcp_in.c:1149          */
    uint16_t ip_len;      /* 22 ntohs(iph->tot_len)     ip_in.c:21             */
    uint16_t ip_csum;     /* 24 ip_fast_csum(iph, ihl)  ip_in.c:35 (0 = good)  */
    uint16_t tcp_csum;    /* 26 TCPCalcChecksum(...)    tcp_in.c:1165 (0 = good);
                                 verdict ICMP: ICMPChecksum(iph + 4*ihl, ip_len - 4*ihl)
                                 (icmp.c:18-42, checked at icmp.c:94) when the datagram
                                 lies inside the frame, else 0; an odd ICMP length makes
                                 the reference read an uninitialised byte (icmp.c:31-33):
                                 the missing high byte is taken as 0 here       */
    uint32_t rss_hash;    /* 28 GetRSSHash(ntohl(saddr), ntohl(daddr),
                                           ntohs(sport), ntohs(dport))         */
    uint16_t payload_len; /* 32 ip_len - 4*(ihl+doff)   tcp_in.c:1144
                                 (ICMP: the ICMP length ip_len - 4*ihl, >= 0)     */
    uint8_t  ihl_doff;    /* 34 ihl | doff << 4                                */
    uint8_t  tcp_flags;   /* 35 FIN 0x01 SYN 0x02 RST 0x04 PSH 0x08 ACK 0x10 URG 0x20 */
    uint8_t  verdict;     /* 36 enum mtcp_gpu_verdict                          */
    uint8_t  rss_queue;   /* 37 GetRSSCPUCore(...) queue                       */
    uint16_t eth_type;    /* 38 ntohs(ethh->h_proto)    eth_in.c:13            */
} mtcp_gpu_result;

/*
 * Compact per-packet result, 16 B, for callers that act on the verdict (and
 * the checksums / RSS queue) only — an io_module that answers get_rptr with
 * the frame or NULL, as dpdk_get_rptr does on the NIC's one checksum bit
 * (mtcp/src/dpdk_module.c:473-479).  Written instead of mtcp_gpu_result by a
 * context opened with MTCP_GPU_F_COMPACT: the rx entry points' `out` /
 * `d_out` then point to mtcp_gpu_result16[n] (cast to mtcp_gpu_result *).
 * Every field equals the same-named field of the 40 B record.
 */
typedef struct mtcp_gpu_result16 {
    uint32_t rss_hash;    /*  0 */
    uint16_t ip_csum;     /*  4 */
    uint16_t tcp_csum;    /*  6 */
    uint16_t payload_len; /*  8 */
    uint16_t ip_len;      /* 10 */
    uint8_t  ihl_doff;    /* 12 */
    uint8_t  tcp_flags;   /* 13 */
    uint8_t  verdict;     /* 14 */
    uint8_t  rss_queue;   /* 15 */
} mtcp_gpu_result16;

typedef struct mtcp_gpu_ctx mtcp_gpu_ctx;

/* Library / device introspection. */
int         mtcp_gpu_abi_version(void);
const char *mtcp_gpu_strerror(int err);
int         mtcp_gpu_device_count(void);
/* PCI address "dddd:bb:dd.f" of HIP device `device` (hipDeviceGetPCIBusId),
 * for NUMA placement: an mTCP thread opens the device on its core's node, as
 * mTCP binds a thread's memory to that node (mtcp/src/cpu.c:54-79). */
int         mtcp_gpu_device_pci_bus_id(int device, char *buf, int len);

/*
 * Open a context on HIP device `device`.
 *   rss_key        40-byte Toeplitz key (util/rss.c:84-90 layout); NULL selects
 *                  the reference's active key, 0x05 x 40 (util/rss.c:84-90).
 *   rss_num_queues queue count for rss_queue (>= 1; ignored without F_RSS).
 *   flags          MTCP_GPU_F_*.
 */
int  mtcp_gpu_open(mtcp_gpu_ctx **out, int device, const uint8_t *rss_key,
                   int rss_num_queues, uint32_t flags);

/* Bound of mtcp_gpu_open's one wait (the first context with a given RSS key
 * on a device uploads the key's tables on its new stream): past it open
 * answers MTCP_GPU_ETIMEDOUT and returns no context. */
#define MTCP_GPU_OPEN_WAIT_US 2000000u

/*
 * Close: the context's own work finishes first (within its wait limit, if
 * set; past it the context is abandoned as below and close returns without
 * waiting more).  Work the CALLER queued on its own streams through the
 * *_dev entry points is not waited for: the device-side RSS tables such a
 * launch reads are shared by every context with the same key and never
 * freed, so the launch computes with its own key whatever contexts are
 * opened or closed meanwhile; every other buffer of it is the caller's, who
 * must keep it alive until that stream is done.
 */
void mtcp_gpu_close(mtcp_gpu_ctx *ctx);

/*
 * Bound every wait of the context's synchronous calls to timeout_us
 * (0: no bound, the default).  Each call computes one deadline when it
 * starts and polls the GPU until then instead of blocking; the calls are
 * mtcp_gpu_rx_chunk, _rx_ptrs, _tx_fill, _tx_fill_ptrs (whose
 * _tx_fill_ptrs_for argument, when non-zero, overrides the limit),
 * _flow_hash, _addr_pool_search, _reserve, _sync and _close, and the calls
 * of the context's rxqs (mtcp_gpu_rxq.h: create, flush, wait, destroy; an
 * rxq takes the limit its context has when it is created).
 *
 * A call whose GPU work is not done by the deadline answers
 * MTCP_GPU_ETIMEDOUT and ABANDONS the context: that work may still run, so
 * every later call on the context answers MTCP_GPU_EIO without touching the
 * device, and mtcp_gpu_close frees only its host-side state (its streams and
 * buffers stay allocated, never used again).  Nothing is written into the
 * caller's memory after such a return, and nothing of it is read: with a
 * limit, the host calls copy the caller's input into pinned staging first
 * and the GPU's output back out of pinned staging only once it is complete
 * (one more host copy of the input, the price of the bound).  The caller
 * then does the work itself, as mTCP does when dev_ioctl answers -1
 * (mtcp/src/ip_in.c:29-31, tcp_in.c:1160-1164, ip_out.c:147-165,
 * tcp_out.c:320-329).  mtcp_gpu_sync alone does not abandon: it answers
 * MTCP_GPU_ETIMEDOUT and the context stays usable (what it waits for is the
 * caller's own device work).
 */
int      mtcp_gpu_set_wait_limit(mtcp_gpu_ctx *ctx, uint32_t timeout_us);
uint32_t mtcp_gpu_wait_limit(const mtcp_gpu_ctx *ctx);

/*
 * Optional, at init time (an io_module's init_handle): allocate the device
 * staging that host-buffer calls (mtcp_gpu_rx_chunk, _rx_ptrs, _tx_fill) of
 * up to `max_bytes` chunk bytes and `max_pkts` frames use, and load the
 * kernels, so that the first call on the data path pays for neither
 * (otherwise both happen lazily on the first call, and a HIP stream's first
 * large copy alone took 7.8 ms).  max_bytes = max_pkts = 0: load the kernels
 * only.  MTCP_GPU_ENOMEM if the device memory is not there.
 */
int  mtcp_gpu_reserve(mtcp_gpu_ctx *ctx, uint64_t max_bytes, uint32_t max_pkts);

/* dev_ioctl-compatible capability answer (0 = offloaded, -1 = software). */
int  mtcp_gpu_dev_ioctl(mtcp_gpu_ctx *ctx, int nif, int cmd, void *argp);

/* The HIP stream the context runs on (a hipStream_t, as void*): its
 * device-resident launches with stream NULL, its host-memory calls and its
 * rxqs.  A caller may order its own work after the context's on it; work it
 * queues there runs before the context's next calls and counts against their
 * wait limit. */
void *mtcp_gpu_stream(mtcp_gpu_ctx *ctx);

/* Bytes per rx result record this context writes: 40, or 16 with
 * MTCP_GPU_F_COMPACT; 0 for a NULL context. */
uint32_t mtcp_gpu_record_size(const mtcp_gpu_ctx *ctx);

/* Name of the kernel the context's last rx / tx launch dispatched (the
 * schedule chosen by batch size and average slot), for profiles and bench
 * lines; "" before the first launch. */
const char *mtcp_gpu_last_kernel(const mtcp_gpu_ctx *ctx);

/*
 * Device-resident rx: chunk, descriptors and results are device (or
 * device-mapped) memory.  Asynchronous on `stream` (a hipStream_t; NULL =
 * the context's stream).  buf_len must be a multiple of 16.
 */
int mtcp_gpu_rx_chunk_dev(mtcp_gpu_ctx *ctx, const void *d_buf, uint64_t buf_len,
                          const mtcp_gpu_desc *d_desc, uint32_t n,
                          uint32_t off_shift, mtcp_gpu_result *d_out,
                          void *stream);

/*
 * Device-resident rx over a pointer burst.  d_pkts[i] is a device-accessible
 * address (device memory, or host memory registered with
 * mtcp_gpu_host_register: the kernel then reads it over PCIe, zero copy) at
 * any even address (a NULL or odd pointer gives MTCP_GPU_V_BAD_DESC);
 * d_lens[i] its frame length.
 */
int mtcp_gpu_rx_ptrs_dev(mtcp_gpu_ctx *ctx, const uint8_t *const *d_pkts,
                         const uint16_t *d_lens, uint32_t n,
                         mtcp_gpu_result *d_out, void *stream);

/*
 * The two device-resident rx calls with the flow-table step fused in:
 * d_bins[i] = the HashFlow bin of packet i (as mtcp_gpu_flow_hash_dev would
 * give for d_out[i]: MTCP_GPU_FLOW_NONE unless TCP_OK), computed in the same
 * kernel from the record it writes.  d_bins may be NULL (then exactly the
 * calls above).
 */
int mtcp_gpu_rx_chunk_flow_dev(mtcp_gpu_ctx *ctx, const void *d_buf, uint64_t buf_len,
                               const mtcp_gpu_desc *d_desc, uint32_t n,
                               uint32_t off_shift, mtcp_gpu_result *d_out,
                               uint32_t *d_bins, void *stream);
int mtcp_gpu_rx_ptrs_flow_dev(mtcp_gpu_ctx *ctx, const uint8_t *const *d_pkts,
                              const uint16_t *d_lens, uint32_t n,
                              mtcp_gpu_result *d_out, uint32_t *d_bins, void *stream);

/*
 * What the caller knows of a batch's frame lengths, for the choice of kernel:
 * the smallest and the largest non-zero frame length in it.  The device
 * entry points above cannot see the lengths (the descriptors are in device
 * memory) and choose by the batch's average slot (buf_len / n) alone, which
 * cannot tell a uniform batch of 768 B frames from a 64 / 1500 B mix of the
 * same average.  An io_module sees every length as it stages a frame
 * (mtcp_gpu_rxq_push, as RunMainLoop's get_rptr hands it over, core.c:771):
 * with the hint, a batch whose 64 B slots all lie within 2x of each other
 * takes the kernel measured fastest for uniform batches of that size.  The
 * records are the same with or without a hint, and for any hint; the host
 * rx calls (mtcp_gpu_rx_chunk, _rx_ptrs) and the rxqs derive it themselves.
 */
typedef struct mtcp_gpu_size_hint {
    uint16_t min_len;
    uint16_t max_len;
} mtcp_gpu_size_hint;

/* mtcp_gpu_rx_chunk_flow_dev with a size hint (NULL: exactly that call). */
int mtcp_gpu_rx_chunk_hint_dev(mtcp_gpu_ctx *ctx, const void *d_buf, uint64_t buf_len,
                               const mtcp_gpu_desc *d_desc, uint32_t n,
                               uint32_t off_shift, mtcp_gpu_result *d_out,
                               uint32_t *d_bins, const mtcp_gpu_size_hint *hint, void *stream);

/*
 * Host-memory rx (the drop-in for the rx loop): chunk and descriptors in host
 * memory, results written to host memory; synchronous, bounded by the
 * context's wait limit.  Large chunks are streamed H2D -> kernel -> D2H in
 * 64 MiB stages on up to three streams; register the chunk with
 * mtcp_gpu_host_register for full PCIe rate (without a wait limit the DMA
 * reads it in place).  Descriptor offsets must be non-decreasing for the
 * streamed path (PSIO chunks are); otherwise the chunk is staged whole.
 */
int mtcp_gpu_rx_chunk(mtcp_gpu_ctx *ctx, const uint8_t *buf, uint64_t buf_len,
                      const mtcp_gpu_desc *desc, uint32_t n, uint32_t off_shift,
                      mtcp_gpu_result *out);

/* Host-memory rx of a pointer burst (gathered into pinned staging). */
int mtcp_gpu_rx_ptrs(mtcp_gpu_ctx *ctx, const uint8_t *const *pkts,
                     const uint16_t *lens, uint32_t n, mtcp_gpu_result *out);

/*
 * tx checksum fill, in place: for every well-formed IPv4/TCP frame
 * (eth 0x0800, version 4, ihl >= 5, protocol 6, doff >= 5,
 * 4*(ihl+doff) <= tot_len, 14 + tot_len <= len) write
 *   iph->check  = ip_fast_csum(iph, ihl)      computed with check = 0
 *   tcph->check = TCPCalcChecksum(tcph, tot_len - 4*ihl, saddr, daddr)
 *                                             computed with check = 0
 * Other frames are left untouched.  *n_filled (may be NULL) receives the
 * number of frames written (host variant only).  The host variant sends the
 * chunk to the GPU once and gets back 8 B per frame (the two check values):
 * only the check fields of the chunk are written, by the calling thread.
 */
int mtcp_gpu_tx_fill_dev(mtcp_gpu_ctx *ctx, void *d_buf, uint64_t buf_len,
                         const mtcp_gpu_desc *d_desc, uint32_t n,
                         uint32_t off_shift, void *stream);
int mtcp_gpu_tx_fill(mtcp_gpu_ctx *ctx, uint8_t *buf, uint64_t buf_len,
                     const mtcp_gpu_desc *desc, uint32_t n, uint32_t off_shift,
                     uint32_t *n_filled);

/*
 * tx checksum fill of a pointer burst, same rule as mtcp_gpu_tx_fill.
 *   _dev: d_pkts[i] device-accessible (device memory or registered host
 *         memory, written in place over PCIe), asynchronous on `stream`.
 *   host: pkts[i] in host memory; the frames are staged to the GPU, the
 *         check values come back, and only the two check fields of each
 *         filled frame are written (by the calling thread); synchronous.
 *         *n_filled (may be NULL) receives the number of frames filled.
 */
int mtcp_gpu_tx_fill_ptrs_dev(mtcp_gpu_ctx *ctx, uint8_t *const *d_pkts,
                              const uint16_t *d_lens, uint32_t n, void *stream);
int mtcp_gpu_tx_fill_ptrs(mtcp_gpu_ctx *ctx, uint8_t *const *pkts, const uint16_t *lens,
                          uint32_t n, uint32_t *n_filled);

/*
 * mtcp_gpu_tx_fill_ptrs with its own bound on the wait (timeout_us 0: the
 * context's wait limit, i.e. exactly mtcp_gpu_tx_fill_ptrs).  If the GPU has
 * not reported within the bound, nothing has been written into the caller's
 * frames, MTCP_GPU_ETIMEDOUT is returned and the context is ABANDONED
 * (mtcp_gpu_set_wait_limit).  The caller fills the frames itself, as mTCP
 * does when dev_ioctl answers -1 (tcp_out.c:320-329, ip_out.c:147-165): an
 * io_module's send_pkts (core.c:818-824) never blocks on a GPU that stopped
 * answering.
 */
int mtcp_gpu_tx_fill_ptrs_for(mtcp_gpu_ctx *ctx, uint8_t *const *pkts, const uint16_t *lens,
                              uint32_t n, uint32_t *n_filled, uint32_t timeout_us);

/* ---- flow-table hash (HashFlow) --------------------------------------- */
#define MTCP_GPU_NUM_BINS_FLOWS  131072u      /* mtcp/src/include/fhash.h:7 */
#define MTCP_GPU_FLOW_NONE       0xFFFFFFFFu  /* packet never reaches the flow table */

/*
 * (Both flow_hash entry points read 40 B records: a MTCP_GPU_F_COMPACT
 * context answers MTCP_GPU_EINVAL; use the fused rx_*_flow_dev calls.)
 * Flow-table bin of every rx result: HashFlow (mtcp/src/tcp_stream.c:56-90,
 * Jenkins one-at-a-time over signed chars, masked to NUM_BINS_FLOWS - 1) of
 * the stream key ProcessTCPPacket hands to StreamHTSearch
 * (mtcp/src/tcp_in.c:1180-1186): saddr = iph->daddr, daddr = iph->saddr,
 * sport = tcph->dest, dport = tcph->source.  Results whose verdict is not
 * MTCP_GPU_V_TCP_OK get MTCP_GPU_FLOW_NONE.  This is the step right after the
 * checksum; CreateHashtable(HashFlow, ...) at mtcp/src/core.c:899.
 */
int mtcp_gpu_flow_hash_dev(mtcp_gpu_ctx *ctx, const mtcp_gpu_result *d_res, uint32_t n,
                           uint32_t *d_bins, void *stream);
int mtcp_gpu_flow_hash(mtcp_gpu_ctx *ctx, const mtcp_gpu_result *res, uint32_t n,
                       uint32_t *bins);

/* ---- RSS-friendly source address pool --------------------------------- */
#define MTCP_GPU_MIN_PORT 1025u               /* mtcp/src/include/addr_pool.h:7 */
#define MTCP_GPU_MAX_PORT 65536u              /* mtcp/src/include/addr_pool.h:8 */

/* One pool entry: sockaddr_in's address and port, network order. */
typedef struct mtcp_gpu_addr_entry {
    uint32_t saddr;
    uint16_t sport;
    uint16_t rsvd;
} mtcp_gpu_addr_entry;

/*
 * RSS queue of every candidate (source address, source port) of an active
 * opener: d_queue[i * (MAX_PORT - MIN_PORT) + (port - MIN_PORT)] =
 * GetRSSCPUCore(daddr_h, saddr_base_h + i, dport_h, port, num_queues,
 * endian_check) (mtcp/src/rss.c:90-103) with the context's Toeplitz key, for
 * i < num_addr and MIN_PORT <= port < MAX_PORT.  Host-order arguments.
 */
int mtcp_gpu_rss_queue_map_dev(mtcp_gpu_ctx *ctx, uint32_t saddr_base_h, uint32_t num_addr,
                               uint32_t daddr_h, uint16_t dport_h, int num_queues,
                               int endian_check, uint8_t *d_queue, void *stream);

/*
 * The search of CreateAddressPoolPerCore (mtcp/src/addr_pool.c:103-180): the
 * candidates whose RSS queue is `core`, in (address, port) order, at most
 * num_addr * (MAX_PORT - MIN_PORT) / num_queues of them (addr_pool.c:129).
 * saddr_base, daddr and dport are network order, as the reference's
 * arguments.  Writes min(count, max_out) entries to host memory `out` and the
 * count the reference keeps to *n_found.  Synchronous.
 */
int mtcp_gpu_addr_pool_search(mtcp_gpu_ctx *ctx, int core, int num_queues,
                              uint32_t saddr_base, int num_addr, uint32_t daddr,
                              uint16_t dport, int endian_check,
                              mtcp_gpu_addr_entry *out, uint32_t max_out,
                              uint32_t *n_found);

/* Pin / unpin host memory for DMA and zero-copy device access
 * (hipHostRegister; the pattern SURVEY §7 names for DPDK mempools).
 * Unregistering waits for the work of every stream on the device, other
 * threads' included (hipHostUnregister; profiles/r5/free_sync.jsonl):
 * unpin at shutdown, after every context on the device is closed, not on a
 * thread's own way out.  The library's own buffers are never freed that way
 * (mtcp_amd/csrc/park.hpp). */
int mtcp_gpu_host_register(void *ptr, uint64_t len);
int mtcp_gpu_host_unregister(void *ptr);

/* Synchronise the context's stream (within its wait limit, if set:
 * MTCP_GPU_ETIMEDOUT past it, the context still usable). */
int mtcp_gpu_sync(mtcp_gpu_ctx *ctx);

/* (The fault-injection entry point the hang tests use, mtcp_gpu_debug_stall,
 * is not part of this library: tests/c/mtcp_gpu_testing.h.) */

#ifdef __cplusplus
}
#endif

#endif /* MTCP_GPU_H */
