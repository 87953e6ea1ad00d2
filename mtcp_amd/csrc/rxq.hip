// rxq.hip — burst aggregation of include/mtcp_gpu_rxq.h: pinned PSIO-style
// staging (64 B aligned frames, io_engine/lib/pslib.c:146) filled by the
// io_module backend, one rx kernel launch over the aggregate, get_rptr
// answered from the staging copy.  Host code only; the checksums run in the
// rx kernel behind mtcp_gpu_rx_chunk_dev.
//
// Each rxq owns a device copy of its staging and a completion event; its
// work goes on its context's stream (one stream per mTCP thread, however
// many interfaces and aggregates it stages): a flush is one H2D of [first
// frame, end of the descriptors) — the descriptors are copied right behind
// the frames in the pinned buffer so that frames and descriptors travel in
// one transfer — the kernel, and one D2H of the results, then the event, so
// that flush_async / wait can overlap the GPU with the backend's own work and
// a wait does not wait for a later aggregate queued behind it.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#include <chrono>
#include <new>
#include <thread>

#include "../../include/mtcp_gpu.h"
#include "../../include/mtcp_gpu_rxq.h"
#include "ctx_internal.hpp"
#include "host_copy.hpp"
#include "park.hpp"
#include "wait.hpp"

using mtcp_wait::Deadline;

// get_rptr serves frame i; the header of frame i + kServeAhead is fetched
// meanwhile (the staged frames were written with streaming stores, so each
// header is a DRAM read, at a 1.5 KiB stride for MTU frames)
constexpr uint32_t kServeAhead = 16;

struct mtcp_gpu_rxq {
    mtcp_gpu_ctx *ctx = nullptr;
    int device = 0;
    hipStream_t stream = nullptr;        // the context's (not owned)
    hipEvent_t evt = nullptr;            // recorded after a flush's D2H
    uint8_t *buf = nullptr;              // pinned staging: frames, then room for descriptors
    mtcp_gpu_desc *desc = nullptr;       // pinned
    uint8_t *res = nullptr;              // pinned result records (rec bytes each)
    uint8_t *d_buf = nullptr;            // device copy of buf
    uint8_t *d_out = nullptr;
    uint32_t rec = 40;                   // record bytes: 40, or 16 for a compact context
    uint32_t max_pkts = 0;
    uint64_t max_bytes = 0;
    uint64_t staging = 0;                // bytes of buf and d_buf
    uint32_t n = 0;                      // frames staged
    uint32_t done_n = 0;                 // frames with results
    uint32_t inflight = 0;               // frames of an unfinished flush_async (0: none)
    bool abandoned = false;              // a flush timed out in rxq_wait_for: no more flushes
    uint32_t wait_us = 0;                // the context's wait limit at create (0: none)
    uint64_t used = 0;                   // staging bytes in use
    // the frames staged since the last flush: smallest and largest non-zero
    // length, the size hint of their launch (mtcp_gpu_size_hint)
    uint16_t size_min = 0xFFFF, size_max = 0;
    // A/B knobs (environment at create): MTCP_GPU_STAGE=plain copies frames
    // with memcpy (cached stores) instead of streaming stores;
    // MTCP_GPU_SERVE_AHEAD=k prefetches frame i + k's header and result when
    // frame i is served (0: off)
    bool plain = false;
    uint32_t ahead = kServeAhead;
    uint32_t hint = 3;                   // MTCP_GPU_SERVE_HINT: prefetch locality 0..3
};

namespace {
inline void serve_prefetch(const void *p, uint32_t hint) {
    switch (hint) {
    case 0: __builtin_prefetch(p, 0, 0); break;
    case 1: __builtin_prefetch(p, 0, 1); break;
    case 2: __builtin_prefetch(p, 0, 2); break;
    default: __builtin_prefetch(p, 0, 3); break;
    }
}
}  // namespace

namespace {

// the rxq's device is current for one call; the caller's is restored
struct RxqDevice {
    int prev = -1;
    bool ok = false;
    explicit RxqDevice(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = prev == device || hipSetDevice(device) == hipSuccess;
    }
    ~RxqDevice() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

extern "C" {

int mtcp_gpu_rxq_create(mtcp_gpu_rxq **out, mtcp_gpu_ctx *ctx, uint32_t max_pkts,
                        uint64_t max_bytes) {
    if (!out || !ctx || !max_pkts || max_bytes < 64) return MTCP_GPU_EINVAL;
    *out = nullptr;
    if (mg_ctx_abandoned(ctx)) return MTCP_GPU_EIO;   // its stream may never finish
    hipDevice_t dev = 0;
    if (hipStreamGetDevice(reinterpret_cast<hipStream_t>(mtcp_gpu_stream(ctx)), &dev) != hipSuccess)
        return MTCP_GPU_ENODEV;
    RxqDevice dg(dev);
    if (!dg.ok) return MTCP_GPU_ENODEV;
    mtcp_gpu_rxq *q = new (std::nothrow) mtcp_gpu_rxq;
    if (!q) return MTCP_GPU_ENOMEM;
    q->ctx = ctx;
    q->device = dev;
    q->max_pkts = max_pkts;
    q->max_bytes = (max_bytes + 63) & ~63ull;
    q->stream = reinterpret_cast<hipStream_t>(mtcp_gpu_stream(ctx));
    q->rec = mtcp_gpu_record_size(ctx);
    q->wait_us = mtcp_gpu_wait_limit(ctx);
    if (const char *e = getenv("MTCP_GPU_STAGE")) q->plain = strcmp(e, "plain") == 0;
    if (const char *e = getenv("MTCP_GPU_SERVE_AHEAD")) q->ahead = (uint32_t)atoi(e);
    if (const char *e = getenv("MTCP_GPU_SERVE_HINT")) q->hint = (uint32_t)atoi(e);
    const uint64_t staging = q->max_bytes + (uint64_t)max_pkts * sizeof(mtcp_gpu_desc);
    q->staging = staging;
    // park.hpp: a destroy never waits for other threads' work on the device
    using mtcp_park::kDevice;
    using mtcp_park::kHost;
    if (hipEventCreateWithFlags(&q->evt, hipEventDisableTiming) != hipSuccess ||
        mtcp_park::alloc(&q->buf, staging, kHost) != hipSuccess ||
        mtcp_park::alloc(&q->desc, (size_t)max_pkts * sizeof(mtcp_gpu_desc), kHost) != hipSuccess ||
        mtcp_park::alloc(&q->res, (size_t)max_pkts * q->rec, kHost) != hipSuccess ||
        mtcp_park::alloc(&q->d_buf, staging, kDevice) != hipSuccess ||
        mtcp_park::alloc(&q->d_out, (size_t)max_pkts * q->rec, kDevice) != hipSuccess) {
        mtcp_gpu_rxq_destroy(q);
        return MTCP_GPU_ENOMEM;
    }
    // load the kernels and bring up the stream's copy queues (created on
    // first use: the first H2D of a stream took 7.8 ms) now, not on the
    // first flush of the data path
    // (copies the size of a flush's: small ones take another path)
    int rc = mtcp_gpu_reserve(ctx, 0, 0);
    const uint64_t h2d = staging < (1ull << 20) ? staging : (1ull << 20);
    const uint64_t d2h = (uint64_t)max_pkts * q->rec;
    memset(q->buf, 0, h2d);
    const bool queued = rc == MTCP_GPU_OK;
    if (queued &&
        (hipMemcpyAsync(q->d_buf, q->buf, h2d, hipMemcpyHostToDevice, q->stream) != hipSuccess ||
         hipMemcpyAsync(q->res, q->d_out, d2h, hipMemcpyDeviceToHost, q->stream) != hipSuccess))
        rc = MTCP_GPU_EIO;
    if (queued) {
        // (a failed enqueue drains too: a copy already queued uses the staging)
        const int w = mtcp_wait::drain(q->stream, Deadline(q->wait_us));
        if (w == MTCP_GPU_ETIMEDOUT) {
            delete q;                            // the copies may still run: the buffers stay
            return w;
        }
        if (rc == MTCP_GPU_OK) rc = w;
    }
    if (rc != MTCP_GPU_OK) {
        mtcp_gpu_rxq_destroy(q);
        return rc;
    }
    *out = q;
    return MTCP_GPU_OK;
}

void mtcp_gpu_rxq_destroy(mtcp_gpu_rxq *q) {
    if (!q) return;
    RxqDevice dg(q->device);
    if (q->evt && (q->abandoned || (q->inflight && mg_ctx_abandoned(q->ctx)))) {
        // a flush rxq_wait_for gave up on may still copy into buf / res /
        // d_out: wait for it a bounded time; if the device still has not
        // finished it, leave every buffer and the event allocated (never
        // touched again) rather than free memory under its DMA, or block in
        // a free that synchronises with a hung device
        const auto deadline = std::chrono::steady_clock::now() +
                              std::chrono::microseconds(MTCP_GPU_RXQ_DESTROY_WAIT_US);
        hipError_t e;
        while ((e = hipEventQuery(q->evt)) == hipErrorNotReady &&
               std::chrono::steady_clock::now() < deadline)
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (e == hipErrorNotReady) {
            delete q;
            return;
        }
    }
    if (q->evt) {
        // a flush still in flight finishes first (within the context's wait
        // limit; past it the buffers stay, as after a timeout above)
        if (q->inflight && mtcp_wait::wait_event(q->evt, Deadline(q->wait_us)) == MTCP_GPU_ETIMEDOUT) {
            delete q;
            return;
        }
        (void)hipEventDestroy(q->evt);
    }
    // parked, not freed (park.hpp): hipFree / hipHostFree would wait for
    // every stream on the device, other threads' hung work included
    // (with a wait limit not even a buffer too large to park is freed)
    const bool may_free = q->wait_us == 0;
    mtcp_park::release(q->buf, q->staging, mtcp_park::kHost, may_free);
    mtcp_park::release(q->desc, (size_t)q->max_pkts * sizeof(mtcp_gpu_desc), mtcp_park::kHost, may_free);
    mtcp_park::release(q->res, (size_t)q->max_pkts * q->rec, mtcp_park::kHost, may_free);
    mtcp_park::release(q->d_buf, q->staging, mtcp_park::kDevice, may_free);
    mtcp_park::release(q->d_out, (size_t)q->max_pkts * q->rec, mtcp_park::kDevice, may_free);
    delete q;
}

int mtcp_gpu_rxq_push(mtcp_gpu_rxq *q, const uint8_t *frame, uint16_t len) {
    if (!q || (!frame && len)) return MTCP_GPU_EINVAL;
    const uint64_t slot = ((uint64_t)len + 63) & ~63ull;
    if (q->inflight) return MTCP_GPU_EINVAL;       // staging is being read by the GPU
    if (q->n == q->max_pkts || q->used + slot > q->max_bytes) return MTCP_GPU_ENOSPC;
    if (q->done_n) return MTCP_GPU_EINVAL;           // flushed frames not yet reset
    mtcp_gpu_desc &d = q->desc[q->n];
    d.offset = (uint32_t)(q->used >> 6);           // 64 B units (off_shift 6)
    d.len = len;
    d.flags = d.rsvd = 0;
    if (len) {
        if (q->plain) memcpy(q->buf + q->used, frame, len);
        else stage_copy(q->buf + q->used, frame, len);
    }
    q->used += slot;
    q->n++;
    if (len) {
        q->size_min = len < q->size_min ? len : q->size_min;
        q->size_max = len > q->size_max ? len : q->size_max;
    }
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

uint32_t mtcp_gpu_rxq_pending(const mtcp_gpu_rxq *q) { return q ? q->n - q->done_n : 0; }

int mtcp_gpu_rxq_flush_async(mtcp_gpu_rxq *q) {
    if (!q || q->inflight) return MTCP_GPU_EINVAL;
    if (q->abandoned || mg_ctx_abandoned(q->ctx)) return MTCP_GPU_EIO;
    if (q->n == q->done_n) return MTCP_GPU_OK;
    RxqDevice dg(q->device);
    if (!dg.ok) return MTCP_GPU_ENODEV;
    const uint32_t first = q->done_n, cnt = q->n - q->done_n;
    // frames staged since the last flush: their descriptors are relative to
    // the staging base; the descriptors go right behind the frames
    const uint64_t lo = (uint64_t)q->desc[first].offset << 6;
    const uint64_t dbytes = (uint64_t)cnt * sizeof(mtcp_gpu_desc);
    memcpy(q->buf + q->used, q->desc + first, dbytes);
    stage_fence();                        // rxq_push's streaming stores are visible to the DMA
    if (hipMemcpyAsync(q->d_buf + lo, q->buf + lo, q->used - lo + dbytes, hipMemcpyHostToDevice,
                       q->stream) != hipSuccess)
        return MTCP_GPU_EIO;
    // every length was seen at push: the launch gets the batch's size class
    const mtcp_gpu_size_hint hint = {q->size_max ? q->size_min : (uint16_t)0, q->size_max};
    int rc = mtcp_gpu_rx_chunk_hint_dev(q->ctx, q->d_buf, q->used,
                                        reinterpret_cast<const mtcp_gpu_desc *>(q->d_buf + q->used), cnt,
                                        6, reinterpret_cast<mtcp_gpu_result *>(q->d_out), nullptr, &hint,
                                        q->stream);
    if (rc == MTCP_GPU_OK &&
        (hipMemcpyAsync(q->res + (size_t)first * q->rec, q->d_out, (size_t)cnt * q->rec,
                        hipMemcpyDeviceToHost, q->stream) != hipSuccess ||
         hipEventRecord(q->evt, q->stream) != hipSuccess))
        rc = MTCP_GPU_EIO;
    if (rc != MTCP_GPU_OK) {
        // the copies already queued finish before the staging is touched again
        if (mtcp_wait::drain(q->stream, Deadline(q->wait_us)) == MTCP_GPU_ETIMEDOUT) q->abandoned = true;
        return rc;
    }
    q->inflight = cnt;
    q->size_min = 0xFFFF;
    q->size_max = 0;
    return MTCP_GPU_OK;
}

int mtcp_gpu_rxq_wait(mtcp_gpu_rxq *q, uint32_t *n) {
    if (!q) return MTCP_GPU_EINVAL;
    return mtcp_gpu_rxq_wait_for(q, n, 0);
}

int mtcp_gpu_rxq_wait_for(mtcp_gpu_rxq *q, uint32_t *n, uint32_t timeout_us) {
    if (!q) return MTCP_GPU_EINVAL;
    int rc = MTCP_GPU_OK;
    if (q->inflight) {
        RxqDevice dg(q->device);
        // (a context abandoned meanwhile, e.g. by a tx fill that timed out on
        // the same stream, is not waited on: one look at the event)
        uint32_t lim = timeout_us ? timeout_us : q->wait_us;
        if (!lim && mg_ctx_abandoned(q->ctx)) lim = 1;
        rc = mtcp_wait::wait_event(q->evt, Deadline(lim));
        if (rc == MTCP_GPU_OK)
            q->done_n += q->inflight;
        else if (rc == MTCP_GPU_ETIMEDOUT)
            q->abandoned = true;              // its results may still arrive: never read them
        q->inflight = 0;
    }
    if (n) *n = q->done_n;
    return rc;
}

int mtcp_gpu_rxq_flush(mtcp_gpu_rxq *q, uint32_t *n) {
    if (!q) return MTCP_GPU_EINVAL;
    const int rc = mtcp_gpu_rxq_flush_async(q);
    if (rc != MTCP_GPU_OK) {
        if (n) *n = q->done_n;
        return rc;
    }
    return mtcp_gpu_rxq_wait(q, n);
}

namespace {
// rxq_get / rxq_get16: frame i's record (rec bytes) through `rec_out`
uint8_t *rxq_serve(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len, const uint8_t **rec_out) {
    if (rec_out) *rec_out = nullptr;
    if (!q || i >= q->done_n) return nullptr;
    if (q->ahead && i + q->ahead < q->done_n) {
        serve_prefetch(q->buf + ((uint64_t)q->desc[i + q->ahead].offset << 6), q->hint);
        serve_prefetch(q->res + (size_t)(i + q->ahead) * q->rec, q->hint);
    }
    const uint8_t *r = q->res + (size_t)i * q->rec;
    // the verdict byte: mtcp_gpu_result.verdict (36) or mtcp_gpu_result16.verdict (14)
    const uint8_t verdict = r[q->rec == 16 ? offsetof(mtcp_gpu_result16, verdict)
                                           : offsetof(mtcp_gpu_result, verdict)];
    if (len) *len = q->desc[i].len;
    if (rec_out) *rec_out = r;
    // core.c:774-775 counts NULL as rx_errors: the checksum failures, and the
    // frames whose headers claim bytes past the frame (the reference would
    // read past len there; the GPU computed no checksum to vouch for them)
    if (verdict == MTCP_GPU_V_IP_CSUM_BAD || verdict == MTCP_GPU_V_TCP_CSUM_BAD ||
        verdict == MTCP_GPU_V_TRUNCATED)
        return nullptr;
    return q->buf + ((uint64_t)q->desc[i].offset << 6);
}
}  // namespace

uint8_t *mtcp_gpu_rxq_get(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len,
                          const mtcp_gpu_result **res) {
    const uint8_t *r = nullptr;
    uint8_t *p = rxq_serve(q, i, len, res ? &r : nullptr);
    // a 16 B record is not a mtcp_gpu_result: never hand it out as one
    if (res) *res = q && q->rec == sizeof(mtcp_gpu_result) ? reinterpret_cast<const mtcp_gpu_result *>(r) : nullptr;
    return p;
}

uint8_t *mtcp_gpu_rxq_get16(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len,
                            const mtcp_gpu_result16 **res16) {
    const uint8_t *r = nullptr;
    uint8_t *p = rxq_serve(q, i, len, res16 ? &r : nullptr);
    if (res16)
        *res16 = q && q->rec == sizeof(mtcp_gpu_result16) ? reinterpret_cast<const mtcp_gpu_result16 *>(r)
                                                          : nullptr;
    return p;
}

uint8_t *mtcp_gpu_rxq_frame(mtcp_gpu_rxq *q, uint32_t i, uint16_t *len) {
    if (!q || i >= q->n) return nullptr;
    if (q->ahead && i + q->ahead < q->n)
        serve_prefetch(q->buf + ((uint64_t)q->desc[i + q->ahead].offset << 6), q->hint);
    if (len) *len = q->desc[i].len;
    return q->buf + ((uint64_t)q->desc[i].offset << 6);
}

void mtcp_gpu_rxq_reset(mtcp_gpu_rxq *q) {
    if (!q || q->inflight) return;                 // a flush_async is reading the staging
    q->n = q->done_n = 0;
    q->used = 0;
    q->size_min = 0xFFFF;
    q->size_max = 0;
}

}  // extern "C"
