// rxq.hip — burst aggregation of include/mtcp_gpu_rxq.h: pinned PSIO-style
// staging (64 B aligned frames, io_engine/lib/pslib.c:146) filled by the
// io_module backend, one mtcp_gpu_rx_chunk over the aggregate, get_rptr
// answered from the staging copy.  Host code only; the checksums run in
// the rx kernel behind mtcp_gpu_rx_chunk.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <new>

#include "../../include/mtcp_gpu.h"
#include "../../include/mtcp_gpu_rxq.h"
#include "host_copy.hpp"

struct mtcp_gpu_rxq {
    mtcp_gpu_ctx *ctx = nullptr;
    uint8_t *buf = nullptr;              // pinned staging chunk
    mtcp_gpu_desc *desc = nullptr;       // pinned
    mtcp_gpu_result *res = nullptr;      // pinned
    uint32_t max_pkts = 0;
    uint64_t max_bytes = 0;
    uint32_t n = 0;                      // frames staged
    uint32_t done = 0;                   // frames with results
    uint64_t used = 0;                   // staging bytes in use
};

extern "C" {

int mtcp_gpu_rxq_create(mtcp_gpu_rxq **out, mtcp_gpu_ctx *ctx, uint32_t max_pkts,
                        uint64_t max_bytes) {
    if (!out || !ctx || !max_pkts || max_bytes < 64) return MTCP_GPU_EINVAL;
    *out = nullptr;
    mtcp_gpu_rxq *q = new (std::nothrow) mtcp_gpu_rxq;
    if (!q) return MTCP_GPU_ENOMEM;
    q->ctx = ctx;
    q->max_pkts = max_pkts;
    q->max_bytes = (max_bytes + 63) & ~63ull;
    if (hipHostMalloc(&q->buf, q->max_bytes, hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(&q->desc, (size_t)max_pkts * sizeof(mtcp_gpu_desc), hipHostMallocDefault) !=
            hipSuccess ||
        hipHostMalloc(&q->res, (size_t)max_pkts * sizeof(mtcp_gpu_result), hipHostMallocDefault) !=
            hipSuccess) {
        mtcp_gpu_rxq_destroy(q);
        return MTCP_GPU_ENOMEM;
    }
    *out = q;
    return MTCP_GPU_OK;
}

void mtcp_gpu_rxq_destroy(mtcp_gpu_rxq *q) {
    if (!q) return;
    if (q->buf) (void)hipHostFree(q->buf);
    if (q->desc) (void)hipHostFree(q->desc);
    if (q->res) (void)hipHostFree(q->res);
    delete q;
}

int mtcp_gpu_rxq_push(mtcp_gpu_rxq *q, const uint8_t *frame, uint16_t len) {
    if (!q || (!frame && len)) return MTCP_GPU_EINVAL;
    const uint64_t slot = ((uint64_t)len + 63) & ~63ull;
    if (q->n == q->max_pkts || q->used + slot > q->max_bytes) return MTCP_GPU_ENOSPC;
    if (q->done) return MTCP_GPU_EINVAL;           // flushed frames not yet reset
    mtcp_gpu_desc &d = q->desc[q->n];
    d.offset = (uint32_t)(q->used >> 6);           // 64 B units (off_shift 6)
    d.len = len;
    d.flags = d.rsvd = 0;
    if (len) stage_copy(q->buf + q->used, frame, len);
    q->used += slot;
    q->n++;
    return MTCP_GPU_OK;
}

int mtcp_gpu_rxq_push_chunk(mtcp_gpu_rxq *q, const uint8_t *buf, const mtcp_gpu_desc *info,
                            uint32_t cnt, uint32_t off_shift) {
    if (!q || (cnt && (!buf || !info)) || off_shift > 16) return MTCP_GPU_EINVAL;
    for (uint32_t i = 0; i < cnt; ++i) {
        const int rc = mtcp_gpu_rxq_push(q, buf + ((uint64_t)info[i].offset << off_shift),
                                         info[i].len);
        if (rc != MTCP_GPU_OK) return rc;
    }
    return MTCP_GPU_OK;
}

uint32_t mtcp_gpu_rxq_pending(const mtcp_gpu_rxq *q) { return q ? q->n - q->done : 0; }

int mtcp_gpu_rxq_flush(mtcp_gpu_rxq *q, uint32_t *n) {
    if (!q) return MTCP_GPU_EINVAL;
    int rc = MTCP_GPU_OK;
    if (q->n > q->done) {
        stage_fence();                    // the streaming stores of rxq_push are visible to the DMA
        // frames staged after the last flush: their descriptors are relative
        // to the staging base, so the whole chunk prefix is handed over
        rc = mtcp_gpu_rx_chunk(q->ctx, q->buf, q->used, q->desc + q->done, q->n - q->done, 6,
                               q->res + q->done);
        if (rc == MTCP_GPU_OK) q->done = q->n;
    }
    if (n) *n = q->done;
    return rc;
}

uint8_t *mtcp_gpu_rxq_get(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len,
                          const mtcp_gpu_result **res) {
    if (!q || i >= q->done) return nullptr;
    const mtcp_gpu_result &r = q->res[i];
    if (len) *len = q->desc[i].len;
    if (res) *res = &r;
    if (r.verdict == MTCP_GPU_V_IP_CSUM_BAD || r.verdict == MTCP_GPU_V_TCP_CSUM_BAD)
        return nullptr;                            // core.c:774-775: rx_errors++
    return q->buf + ((uint64_t)q->desc[i].offset << 6);
}

uint8_t *mtcp_gpu_rxq_frame(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len) {
    if (!q || i >= q->n) return nullptr;
    if (len) *len = q->desc[i].len;
    return q->buf + ((uint64_t)q->desc[i].offset << 6);
}

void mtcp_gpu_rxq_reset(mtcp_gpu_rxq *q) {
    if (!q) return;
    q->n = q->done = 0;
    q->used = 0;
}

}  // extern "C"
