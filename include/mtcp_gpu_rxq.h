/*
 * mtcp_gpu_rxq.h — burst aggregation for a GPU-offload io_module backend
 * (SURVEY §8 f2).  Plain C ABI, part of libmtcp_gpu.so.
 *
 * mTCP's rx loop (RunMainLoop, mtcp/src/core.c:763-777) asks the I/O module
 * for a burst (recv_pkts, io_module.h:63), then for each packet's pointer
 * (get_rptr, io_module.h:62), and counts a NULL pointer as rx_errors
 * (core.c:771-775).  Real bursts are <= 64 packets (PS_CHUNK_SIZE
 * psio_module.c:15, MAX_PKT_BURST dpdk_module.c:71), too small for one GPU
 * launch each, and the wrapped backend recycles its buffers on the next
 * receive (psio_module.c:244-246, dpdk_module.c:395-398).  An rxq therefore
 * copies the frames of several bursts into pinned staging laid out like a
 * PSIO chunk (64 B aligned, io_engine/lib/pslib.c:146), runs the rx kernel
 * over the aggregate once (mtcp_gpu_rx_chunk_dev), and then answers get_rptr
 * from the staging copy:
 *
 *   - MTCP_GPU_V_IP_CSUM_BAD, MTCP_GPU_V_TCP_CSUM_BAD -> NULL, exactly the
 *     packets the reference's software checksums drop with ERROR
 *     (ip_in.c:35-36, tcp_in.c:1167-1173), the dpdk_get_rptr pattern for
 *     NIC-verified checksums (dpdk_module.c:473-479);
 *   - MTCP_GPU_V_TRUNCATED -> NULL: a header claims bytes past the frame, so
 *     the reference's checks would read past len (undefined) and no checksum
 *     was computed that dev_ioctl's 0 could vouch for;
 *   - every other verdict -> the frame, and mTCP's own code takes its usual
 *     branch (the checks before and around the checksums stay in mTCP), with
 *     dev_ioctl(PKT_RX_IP_CSUM / PKT_RX_TCP_CSUM) answering 0
 *     (ip_in.c:29-31, tcp_in.c:1160-1164) so the checksum is not recomputed.
 *
 * An rxq's copies and kernel run on its context's stream (mtcp_gpu_stream),
 * with its own completion event; one context per mTCP thread, its rxqs used
 * by that thread only (not re-entrant).  Every wait of an rxq (create's,
 * flush's, wait's, destroy's) is bounded by the wait limit its context had
 * when the rxq was created (mtcp_gpu_set_wait_limit; none by default).
 */
#ifndef MTCP_GPU_RXQ_H
#define MTCP_GPU_RXQ_H

#include <stdint.h>

#include "mtcp_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MTCP_GPU_ENOSPC (-28)   /* the staging area is full: flush first */

typedef struct mtcp_gpu_rxq mtcp_gpu_rxq;

/* Staging for up to max_pkts frames / max_bytes (64 B aligned) bytes. */
int  mtcp_gpu_rxq_create(mtcp_gpu_rxq **out, mtcp_gpu_ctx *ctx, uint32_t max_pkts,
                         uint64_t max_bytes);

/* Free the rxq (before mtcp_gpu_close of its context).  A flush still in
 * flight is waited for (within the wait limit; past it the buffers are left
 * allocated, as below).  After
 * mtcp_gpu_rxq_wait_for gave up on a flush (MTCP_GPU_ETIMEDOUT), that flush
 * may still copy into the staging and results: destroy then waits for it at
 * most MTCP_GPU_RXQ_DESTROY_WAIT_US more, and if it still has not finished,
 * the rxq's pinned and device buffers are left allocated (leaked, never
 * touched again) instead of freed under the DMA, and destroy returns without
 * blocking on the device.  Safe to call straight after ETIMEDOUT. */
#define MTCP_GPU_RXQ_DESTROY_WAIT_US 100000u
void mtcp_gpu_rxq_destroy(mtcp_gpu_rxq *q);

/* Copy one received frame (get_rptr's pointer and *len) into staging. */
int  mtcp_gpu_rxq_push(mtcp_gpu_rxq *q, const uint8_t *frame, uint16_t len);

/* Copy a whole PSIO chunk: frame i at buf + (info[i].offset << off_shift),
 * length info[i].len (struct ps_chunk, io_engine/include/ps.h:187-200). */
int  mtcp_gpu_rxq_push_chunk(mtcp_gpu_rxq *q, const uint8_t *buf, const mtcp_gpu_desc *info,
                             uint32_t cnt, uint32_t off_shift);

/* Frames staged and not yet flushed. */
uint32_t mtcp_gpu_rxq_pending(const mtcp_gpu_rxq *q);

/* Run the rx kernel over everything staged since the last reset; *n = the
 * number of frames now served by mtcp_gpu_rxq_get (synchronous). */
int  mtcp_gpu_rxq_flush(mtcp_gpu_rxq *q, uint32_t *n);

/* The same in two halves, so that a backend can overlap the GPU with its
 * own work (gpu_module.c serves aggregate k while k+1 is checked):
 * flush_async starts the rx kernel over the frames staged since the last
 * flush (one H2D of frames + descriptors, the kernel, one D2H of results, on
 * the rxq's own stream) and returns; until rxq_wait the rxq takes no pushes,
 * flushes or resets (MTCP_GPU_EINVAL).  rxq_wait blocks until the results
 * are in and then behaves like the end of rxq_flush. */
int  mtcp_gpu_rxq_flush_async(mtcp_gpu_rxq *q);
int  mtcp_gpu_rxq_wait(mtcp_gpu_rxq *q, uint32_t *n);

/* rxq_wait with a limit (timeout_us 0: the context's wait limit,
 * mtcp_gpu_set_wait_limit, i.e. exactly rxq_wait).  If the results are not in
 * after timeout_us, the flush is abandoned and MTCP_GPU_ETIMEDOUT returned:
 * its frames stay staged (served by rxq_frame, without verdicts), the rxq
 * takes resets and pushes again, but no further flush (MTCP_GPU_EIO: the
 * abandoned flush may still write its results). */
int  mtcp_gpu_rxq_wait_for(mtcp_gpu_rxq *q, uint32_t *n, uint32_t timeout_us);

/* get_rptr for flushed frame i: the staged frame and its length, or NULL for
 * the verdicts listed above.  *res (may be NULL) receives the frame's 40 B
 * result record; on an rxq of a MTCP_GPU_F_COMPACT context (16 B records,
 * mtcp_gpu_record_size 16) *res is set to NULL — use mtcp_gpu_rxq_get16.
 * A compact context moves 16 B per frame back instead of 40 (gpu_module.c's
 * rxqs read the verdict only). */
uint8_t *mtcp_gpu_rxq_get(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len,
                          const mtcp_gpu_result **res);

/* mtcp_gpu_rxq_get for the rxq of a compact context: *res16 (may be NULL)
 * receives the frame's mtcp_gpu_result16; on a 40 B context *res16 is set
 * to NULL (use mtcp_gpu_rxq_get).  The frame pointer is rxq_get's. */
uint8_t *mtcp_gpu_rxq_get16(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len,
                            const mtcp_gpu_result16 **res16);

/* The staged copy of frame i (flushed or not), without a verdict: what a
 * backend serves when the GPU is unavailable and dev_ioctl answers -1. */
uint8_t *mtcp_gpu_rxq_frame(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len);

/* Drop all staged and flushed frames (the next burst reuses the staging). */
void mtcp_gpu_rxq_reset(mtcp_gpu_rxq *q);

#ifdef __cplusplus
}
#endif
#endif
