// mtcp_gpu.hip — the C ABI of include/mtcp_gpu.h: contexts, launches and the
// host-memory pipelines around the gfx950 kernels of rx_kernels.hpp.
//
// Product code only: there is no CPU fallback here.  When no GPU is usable
// every entry point returns an error code, and the caller (mTCP) keeps its
// software path exactly as dev_ioctl returning -1 would make it
// (mtcp/src/ip_in.c:29-31, tcp_in.c:1160-1164).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/mtcp_gpu.h"
#include "ctx_internal.hpp"
#include "dispatch.hpp"
#include "flow_kernels.hpp"
#include "host_copy.hpp"
#include "park.hpp"
#include "rx_kernels.hpp"
#include "rx_span.hpp"
#include "wait.hpp"

namespace {

constexpr int kStages = 3;                       // H2D | kernel | D2H overlap
constexpr uint64_t kStageBytes = 64ull << 20;    // chunk bytes per pipeline stage
constexpr uint32_t kStagePkts = 1u << 16;        // descriptors per pipeline stage

// One pipeline stage of the host-memory calls.  Stage 0 runs on the
// context's own stream (one stream per mTCP thread: an io_module's rxqs, its
// tx fills and every host call of a batch that fits one stage share it);
// stages 1 and 2 get streams of their own only when a call spans more than
// one stage (a chunk above kStageBytes), to overlap H2D, kernel and D2H.
struct Stage {
    uint8_t *d_buf = nullptr;
    mtcp_gpu_desc *d_desc = nullptr;
    mtcp_gpu_result *d_out = nullptr;
    uint64_t buf_cap = 0;
    uint32_t pkt_cap = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    // bounded calls (a context wait limit): pinned bounce buffers, so that
    // no copy the call gives up on can read or write the caller's memory
    uint8_t *h_in = nullptr;                    // caller data -> H2D
    uint64_t h_in_cap = 0;
    uint8_t *h_out = nullptr;                   // D2H -> caller data
    uint64_t h_out_cap = 0;
    uint32_t pend_first = 0, pend_cnt = 0;      // records of this stage's batch not yet copied out
};

using mtcp_wait::Deadline;
using mtcp_wait::drain;

}  // namespace

struct mtcp_gpu_ctx {
    int device = 0;
    int num_cu = 256;
    uint32_t flags = 0;
    uint32_t rss_nq = 1;
    uint32_t rss_endian = 0;
    uint32_t rss_key_w[4] = {0, 0, 0, 0};        // key bytes 0..15, big-endian words
    int sched = 0;                               // Sched: kSchedAuto unless MTCP_GPU_SCHED forces one
    hipStream_t stream = nullptr;
    const uint32_t *d_rss_tables = nullptr;      // shared, immutable (rss_tables_for)
    uint32_t wait_us = 0;                        // mtcp_gpu_set_wait_limit (0: no limit)
    Stage stage[kStages];
    uint8_t *h_gather = nullptr;                 // pinned, for rx_ptrs
    uint64_t h_gather_cap = 0;
    mtcp_gpu_desc *h_gather_desc = nullptr;
    uint32_t h_gather_desc_cap = 0;
    const char *last_kernel = "";                // mtcp_gpu_last_kernel
    // a host call's bounded wait gave up: work of that call may still read
    // or write the staging, so nothing is issued, staged or freed on this
    // context again (every call answers EIO)
    bool abandoned = false;
};

namespace {

// MTCP_GPU_DEBUG=1 in the environment: report every failing HIP call.
bool hip_ok(hipError_t e, const char *what) {
    if (e == hipSuccess) return true;
    static const bool debug = getenv("MTCP_GPU_DEBUG") != nullptr;
    if (debug) fprintf(stderr, "mtcp_gpu: %s -> %s\n", what, hipGetErrorString(e));
    return false;
}
#define HIP_OK(x) hip_ok((x), #x)

// Makes `device` current for one ABI call and restores the caller's device
// on return: an mTCP thread (or a torch process) keeps the device it chose.
struct DeviceGuard {
    int prev = -1;
    bool ok = false, switched = false;
    explicit DeviceGuard(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev == device) {
            ok = true;
        } else {
            ok = HIP_OK(hipSetDevice(device));
            switched = ok && prev >= 0;
        }
    }
    ~DeviceGuard() {
        if (switched) (void)hipSetDevice(prev);
    }
    DeviceGuard(const DeviceGuard &) = delete;
    DeviceGuard &operator=(const DeviceGuard &) = delete;
};

// util/rss.c:13-105 (BuildKeyCache), then the 24 nibble tables the kernel
// XORs: table[t][v] = XOR of cache[4t + m] over the bits of nibble v, MSB
// first (nibble t of the 96-bit input sip|dip|sp|dp, most significant first).
void build_rss_tables(const uint8_t key[40], uint32_t *tables) {
    uint32_t cache[96];
    uint32_t result = ((uint32_t)key[0] << 24) | ((uint32_t)key[1] << 16) |
                      ((uint32_t)key[2] << 8) | (uint32_t)key[3];
    uint32_t idx = 32;
    for (int i = 0; i < 96; i++, idx++) {
        cache[i] = result;
        const uint32_t bit = ((key[idx / 8] << (idx % 8)) & 0x80) ? 1u : 0u;
        result = (result << 1) | bit;
    }
    for (int t = 0; t < 24; ++t)
        for (int v = 0; v < 16; ++v) {
            uint32_t h = 0;
            for (int m = 0; m < 4; ++m)
                if (v & (0x8 >> m)) h ^= cache[4 * t + m];
            tables[t * 16 + v] = h;
        }
}

// Two 256-thread workgroups per CU (8 waves): measured fastest on MI355X for
// this streaming kernel (fewer concurrent streams keep HBM efficiency up;
// tools/rx_variants.hip sweeps 1..4 per CU).  Each wave walks its passes.
uint32_t grid_for(const mtcp_gpu_ctx *ctx, uint32_t n) {
    const uint32_t groups = (n + mg::kWave - 1) / mg::kWave;
    const uint32_t blocks = (groups + mg::kWavesPerBlock - 1) / mg::kWavesPerBlock;
    const uint32_t cap = (uint32_t)ctx->num_cu * 2;
    return std::max(1u, std::min(blocks, cap));
}

// Two workgroups share each CU, and the first one dispatched wins the memory
// arbitration: per-wave s_memrealtime stamps of C2 (tools/rx_variants
// stampsab) show the second workgroup ending ~7 us after the first, with
// the CU half-occupied meanwhile.  The second workgroup runs at s_setprio(1)
// for its first four passes (rx_kernel PRIO 5), which evens the two (C2:
// 242.9-245.8 -> 239.7-240.8 us in the same process); the other schedules
// showed no change and keep the default.
template <int SCHED, bool LALIGN>
constexpr int prio_for() { return SCHED == mg::kSchedUnrolled && !LALIGN ? 5 : 0; }

template <int MODE, bool RSS, int SCHED, bool LALIGN, bool CMP>
void launch_one(dim3 grid, dim3 block, hipStream_t st, const mg::KParams &kp) {
    // tx fill streams its frames through L2 normally (NT off): its check-field
    // writes at the end then find part of the last passes' lines resident
    // (f1: 324 -> 317 us on 1 M x 1500 B; rx keeps the non-temporal stream)
    constexpr bool kNT = MODE != mg::kTxChunk;
    // multi-trip frames in the unrolled schedule: odd rows walk their trips
    // backwards so neighbouring frames' shared lines are read in one step
    // (C5: 4.768 -> 4.737 GB per launch = chunk + descriptors, no line twice)
    constexpr bool kRev = LALIGN && SCHED == mg::kSchedUnrolled;
    // runs of 16 packets for the size-sorted chunk schedule (C3-shaped
    // batches): its per-lane descriptors come in 128 B pieces instead of 64 B
    // (tools/rx_variants c3: 133.8 vs 134.9 us, records identical); the
    // unrolled schedule keeps 8 and loads them per workgroup (rx_kernel COOP)
    constexpr int kB = SCHED == mg::kSchedSorted && !LALIGN && MODE == mg::kRxChunk ? 16 : 8;
    hipLaunchKernelGGL((mg::rx_kernel<MODE, RSS, SCHED, LALIGN, 0, 8, kB, kNT, 6, kRev, false,
                                      prio_for<SCHED, LALIGN>(), mg::kWavesPerBlock, 0, CMP>),
                       grid, block, 0, st, kp);
}

template <int MODE, bool RSS, bool CMP>
const char *launch_sched(dim3 grid, dim3 block, hipStream_t st, const mg::KParams &kp, uint64_t slot,
                         uint32_t batch_n) {
    // the schedule (dispatch.hpp big_schedule) is chosen once per batch
    // (batch_n: the whole batch, not this launch's share of it)
    const int b = big_schedule(MODE == mg::kRxPtrs, slot, batch_n);
    if constexpr (MODE == mg::kRxPtrs) {
        launch_one<MODE, RSS, mg::kSchedSorted, true, CMP>(grid, block, st, kp);
    } else if (b == kBigSorted) {
        launch_one<MODE, RSS, mg::kSchedSorted, false, CMP>(grid, block, st, kp);
    } else if (b == kBigUnrolledLineAligned) {
        launch_one<MODE, RSS, mg::kSchedUnrolled, true, CMP>(grid, block, st, kp);
    } else {
        launch_one<MODE, RSS, mg::kSchedUnrolled, false, CMP>(grid, block, st, kp);
    }
    return kernel_name(kSchedBig, b, slot);
}

// A wave holds its results for up to kHeldPasses passes and stores them in
// one burst at the end (rx_kernel DEFER); a batch needing more passes would
// flush mid-stream, which costs more than a second launch (C4's 2 M x 1500 B
// per GPU: one launch 511 us, two launches of 1 M ~486 us).  So a batch is
// cut into launches of at most grid x 4 waves x 64 x kHeldPasses packets.
constexpr uint32_t kHeldPasses = 8;

// The kernel choice (batch size, average slot, size hint) is dispatch.hpp's
// pick_sched / big_schedule, shared with the CPU test of its rules.

template <int MODE, bool RSS>
const char *launch_small(int sched, uint32_t n, uint64_t slot, hipStream_t st, const mg::KParams &kp) {
    if (sched == kSchedWave) {
        const dim3 grid((n + mg::kWavesPerBlock - 1) / mg::kWavesPerBlock);
        if (slot <= kWaveShortUpToSlot) {
            hipLaunchKernelGGL((mg::rx_wave_kernel<MODE, RSS, 0, 1, 2>), grid, dim3(mg::kBlock), 0, st, kp);
            return "rx_wave_kernel<2 loads>";
        }
        hipLaunchKernelGGL((mg::rx_wave_kernel<MODE, RSS>), grid, dim3(mg::kBlock), 0, st, kp);
        return "rx_wave_kernel<10 loads>";
    } else if (sched == kSchedQuad) {
        constexpr int kBlk = mg::kQuadBlock;
        constexpr uint32_t P = mg::GroupShape<4, kBlk>::P;
        hipLaunchKernelGGL((mg::rx_group_kernel<MODE, RSS, 4, 0, 1, kBlk>), dim3((n + P - 1) / P), dim3(kBlk), 0,
                           st, kp);
        return "rx_group_kernel<quad>";
    } else if (sched == kSchedOct) {
        constexpr int kBlk = mg::kOctBlock;
        constexpr uint32_t P = mg::GroupShape<8, kBlk>::P;
        hipLaunchKernelGGL((mg::rx_group_kernel<MODE, RSS, 8, 0, 1, kBlk>), dim3((n + P - 1) / P), dim3(kBlk), 0,
                           st, kp);
        return "rx_group_kernel<oct>";
    } else if (sched == kSchedSpan) {
        if constexpr (!mg::is_tx(MODE)) {
            hipLaunchKernelGGL((mg::rx_span_kernel<MODE, RSS>), dim3((n + mg::kSpanP - 1) / mg::kSpanP),
                               dim3(mg::kSpanBlock), 0, st, kp);
            return "rx_span_kernel";
        }
    }
    constexpr uint32_t P = mg::GroupShape<16>::P;
    hipLaunchKernelGGL((mg::rx_group_kernel<MODE, RSS, 16>), dim3((n + P - 1) / P), dim3(mg::kGroupBlock), 0,
                       st, kp);
    return "rx_group_kernel<row>";
}

// bytes per rx record: 40 (mtcp_gpu_result) or 16 (mtcp_gpu_result16)
uint64_t record_size(const mg::KParams &kp) { return kp.compact ? 16 : 40; }
uint64_t record_size(const mtcp_gpu_ctx *ctx) { return (ctx->flags & MTCP_GPU_F_COMPACT) ? 16 : 40; }

template <int MODE>
int launch(mtcp_gpu_ctx *ctx, const mg::KParams &kp, hipStream_t st, const mtcp_gpu_size_hint *hint = nullptr) {
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (kp.n == 0) return MTCP_GPU_OK;
    const bool rss = !mg::is_tx(MODE) && (ctx->flags & MTCP_GPU_F_RSS);
    const bool ptrs = MODE == mg::kRxPtrs || MODE == mg::kTxPtrs;
    const uint64_t avg_slot = ptrs ? 1024 : kp.buf_len / kp.n;
    const int sched = pick_sched(ctx->sched, kp.n, avg_slot, MODE == mg::kTxPtrs || kp.tx_report != nullptr,
                                 !mg::is_tx(MODE), !ptrs && narrow_batch(hint));
    if (sched != kSchedBig) {
        ctx->last_kernel = rss ? launch_small<MODE, true>(sched, kp.n, avg_slot, st, kp)
                               : launch_small<MODE, false>(sched, kp.n, avg_slot, st, kp);
        return HIP_OK(hipGetLastError()) ? MTCP_GPU_OK : MTCP_GPU_EIO;
    }
    if constexpr (MODE != mg::kTxPtrs) {
    const dim3 grid(grid_for(ctx, kp.n)), block(mg::kBlock);
    const uint64_t slot = kp.n ? kp.buf_len / kp.n : 0;       // the whole batch's average slot
    const uint32_t cap = grid.x * mg::kWavesPerBlock * mg::kWave * kHeldPasses;
    for (uint32_t first = 0; first < kp.n; first += cap) {
        mg::KParams sub = kp;
        sub.n = std::min(kp.n - first, cap);
        if (MODE == mg::kRxPtrs) {
            sub.ptrs = kp.ptrs + first;
            sub.lens = kp.lens + first;
        } else {
            sub.desc = kp.desc + first;
        }
        if (MODE != mg::kTxChunk)
            sub.out = reinterpret_cast<mtcp_gpu_result *>(reinterpret_cast<uint8_t *>(kp.out) +
                                                          (uint64_t)first * record_size(kp));
        if (kp.bins) sub.bins = kp.bins + first;
        if constexpr (mg::is_tx(MODE)) {
            ctx->last_kernel = launch_sched<MODE, false, false>(grid, block, st, sub, slot, kp.n);
        } else if (kp.compact) {
            ctx->last_kernel = rss ? launch_sched<MODE, true, true>(grid, block, st, sub, slot, kp.n)
                                   : launch_sched<MODE, false, true>(grid, block, st, sub, slot, kp.n);
        } else {
            ctx->last_kernel = rss ? launch_sched<MODE, true, false>(grid, block, st, sub, slot, kp.n)
                                   : launch_sched<MODE, false, false>(grid, block, st, sub, slot, kp.n);
        }
    }
    }
    return HIP_OK(hipGetLastError()) ? MTCP_GPU_OK : MTCP_GPU_EIO;
}

mg::KParams base_params(mtcp_gpu_ctx *ctx) {
    mg::KParams kp{};
    kp.rss_tables = ctx->d_rss_tables;
    kp.rss_nq = ctx->rss_nq;
    kp.rss_endian = ctx->rss_endian;
    for (int i = 0; i < 4; ++i) kp.rss_key[i] = ctx->rss_key_w[i];
    kp.compact = (ctx->flags & MTCP_GPU_F_COMPACT) ? 1u : 0u;
    return kp;
}

// results of the device entry points: 8 B aligned (40 B records, stored in
// 8 and 16 B pieces), 16 B aligned for the compact records (one 16 B store)
uintptr_t out_align(const mtcp_gpu_ctx *ctx) { return (ctx->flags & MTCP_GPU_F_COMPACT) ? 15 : 7; }

hipStream_t pick(mtcp_gpu_ctx *ctx, void *stream) {
    return stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
}

// a stage's buffers back to park.hpp (its stream has no work on them);
// may_free = false inside a bounded call: nothing may wait on the device
void stage_release_buf(Stage &s, bool may_free) {
    mtcp_park::release(s.d_buf, s.buf_cap, mtcp_park::kDevice, may_free);
    s.d_buf = nullptr;
    s.buf_cap = 0;
}
void stage_release_pkts(Stage &s, bool may_free) {
    mtcp_park::release(s.d_desc, (size_t)s.pkt_cap * sizeof(mtcp_gpu_desc), mtcp_park::kDevice, may_free);
    mtcp_park::release(s.d_out, (size_t)s.pkt_cap * sizeof(mtcp_gpu_result), mtcp_park::kDevice, may_free);
    s.d_desc = nullptr;
    s.d_out = nullptr;
    s.pkt_cap = 0;
}
void stage_release_host(Stage &s, bool may_free) {
    mtcp_park::release(s.h_in, s.h_in_cap, mtcp_park::kHost, may_free);
    mtcp_park::release(s.h_out, s.h_out_cap, mtcp_park::kHost, may_free);
    s.h_in = s.h_out = nullptr;
    s.h_in_cap = s.h_out_cap = 0;
}

// A wait of a host call ended: past the deadline the context is abandoned
// (the work it gave up on may still use the staging), and the call answers
// MTCP_GPU_ETIMEDOUT.
int waited(mtcp_gpu_ctx *ctx, int rc) {
    if (rc == MTCP_GPU_ETIMEDOUT) ctx->abandoned = true;
    return rc;
}

// The stage's stream: stage 0 is the context's own; the others are created
// on the first call that spans more than one stage.
int stage_stream(mtcp_gpu_ctx *ctx, Stage &s) {
    if (s.stream) return MTCP_GPU_OK;
    if (&s == &ctx->stage[0]) {
        s.stream = ctx->stream;
        return MTCP_GPU_OK;
    }
    if (!HIP_OK(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking))) return MTCP_GPU_EIO;
    s.own_stream = true;
    return MTCP_GPU_OK;
}

int stage_reserve(mtcp_gpu_ctx *ctx, Stage &s, uint64_t bytes, uint32_t pkts, const Deadline &dl) {
    if (ctx->abandoned) return MTCP_GPU_EIO;
    int rc = stage_stream(ctx, s);
    if (rc != MTCP_GPU_OK) return rc;
    // growing releases buffers that the stage's previous batch may still
    // use: drain that batch first (park.hpp releases without any device wait)
    if ((bytes > s.buf_cap || pkts > s.pkt_cap) && (rc = waited(ctx, drain(s.stream, dl))) != MTCP_GPU_OK)
        return rc;
    if (bytes > s.buf_cap) {
        stage_release_buf(s, !dl.bounded);
        const uint64_t cap = (bytes + 4095) & ~4095ull;
        if (!HIP_OK(mtcp_park::alloc(&s.d_buf, cap, mtcp_park::kDevice))) return MTCP_GPU_ENOMEM;
        s.buf_cap = cap;
    }
    if (pkts > s.pkt_cap) {
        stage_release_pkts(s, !dl.bounded);
        if (!HIP_OK(mtcp_park::alloc(&s.d_desc, (size_t)pkts * sizeof(mtcp_gpu_desc), mtcp_park::kDevice)))
            return MTCP_GPU_ENOMEM;
        if (!HIP_OK(mtcp_park::alloc(&s.d_out, (size_t)pkts * sizeof(mtcp_gpu_result), mtcp_park::kDevice))) {
            mtcp_park::release(s.d_desc, (size_t)pkts * sizeof(mtcp_gpu_desc), mtcp_park::kDevice, !dl.bounded);
            s.d_desc = nullptr;
            return MTCP_GPU_ENOMEM;
        }
        s.pkt_cap = pkts;
    }
    return MTCP_GPU_OK;
}

// Pinned host buffers of a stage: in_bytes of bounce for the caller's input
// (a bounded call copies it there first), out_bytes for what comes back.
// The stage's stream has no work on them (a grown buffer is released).
int stage_host(mtcp_gpu_ctx *ctx, Stage &s, uint64_t in_bytes, uint64_t out_bytes, const Deadline &dl) {
    int rc = MTCP_GPU_OK;
    if ((in_bytes > s.h_in_cap || out_bytes > s.h_out_cap) && s.stream &&
        (rc = waited(ctx, drain(s.stream, dl))) != MTCP_GPU_OK)
        return rc;
    if (in_bytes > s.h_in_cap) {
        mtcp_park::release(s.h_in, s.h_in_cap, mtcp_park::kHost, !dl.bounded);
        s.h_in = nullptr;
        s.h_in_cap = 0;
        const uint64_t cap = (in_bytes + 4095) & ~4095ull;
        if (!HIP_OK(mtcp_park::alloc(&s.h_in, cap, mtcp_park::kHost))) return MTCP_GPU_ENOMEM;
        s.h_in_cap = cap;
    }
    if (out_bytes > s.h_out_cap) {
        mtcp_park::release(s.h_out, s.h_out_cap, mtcp_park::kHost, !dl.bounded);
        s.h_out = nullptr;
        s.h_out_cap = 0;
        const uint64_t cap = (out_bytes + 4095) & ~4095ull;
        if (!HIP_OK(mtcp_park::alloc(&s.h_out, cap, mtcp_park::kHost))) return MTCP_GPU_ENOMEM;
        s.h_out_cap = cap;
    }
    return MTCP_GPU_OK;
}

// A bounded call's copy of caller memory into a bounce buffer (16 B aligned
// destination; streaming stores: the DMA engine reads it next, not a core)
void bounce_in(uint8_t *dst, const void *src, uint64_t len) {
    const uint8_t *p = static_cast<const uint8_t *>(src);
    constexpr uint64_t kPiece = 1u << 30;
    for (uint64_t o = 0; o < len; o += kPiece)
        stage_copy(dst + o, p + o, (uint32_t)std::min(kPiece, len - o));
    stage_fence();
}

// The end of a host call that used stages [0, nstages): every stage's
// stream drained within the call's deadline, the records of a bounded
// call's batches still in the stages' bounce buffers copied out to `out_b`
// (rec bytes each).  Returns the call's result: rc if every drain
// succeeded, MTCP_GPU_ETIMEDOUT (the context abandoned, nothing more copied
// out) past the deadline.
int finish_call(mtcp_gpu_ctx *ctx, int rc, const Deadline &dl, int nstages, uint8_t *out_b = nullptr,
                size_t rec = 0) {
    for (int i = 0; i < nstages; ++i) {
        Stage &s = ctx->stage[i];
        if (!s.stream) continue;
        const int r = drain(s.stream, dl);
        if (r == MTCP_GPU_ETIMEDOUT) {
            for (auto &t : ctx->stage) t.pend_cnt = 0;
            return waited(ctx, r);
        }
        if (r != MTCP_GPU_OK && rc == MTCP_GPU_OK) rc = r;
    }
    for (int i = 0; i < nstages; ++i) {
        Stage &s = ctx->stage[i];
        if (rc == MTCP_GPU_OK && s.pend_cnt && out_b)
            memcpy(out_b + (size_t)s.pend_first * rec, s.h_out, (size_t)s.pend_cnt * rec);
        s.pend_cnt = 0;
    }
    return rc;
}

// A bounded call reuses stage s for its next batch: the batch it holds
// finishes (within the deadline) and its records are copied out.
int stage_collect(mtcp_gpu_ctx *ctx, Stage &s, uint8_t *out_b, size_t rec, const Deadline &dl) {
    if (!s.pend_cnt) return MTCP_GPU_OK;
    const int rc = waited(ctx, drain(s.stream, dl));
    if (rc != MTCP_GPU_OK) return rc;
    memcpy(out_b + (size_t)s.pend_first * rec, s.h_out, (size_t)s.pend_cnt * rec);
    s.pend_cnt = 0;
    return MTCP_GPU_OK;
}

// The Toeplitz tables of one RSS key on one device (build_rss_tables):
// built and uploaded by the first context opened with that key, then shared
// by every later one, never written again and never freed.  So a kernel
// still reading them — a *_dev launch on a caller's stream that has not
// finished when its context is closed — reads the key it was launched with,
// whatever contexts open or close meanwhile.  At most one set of 1.5 KiB
// per distinct key and device.
struct RssTables {
    int device;
    uint8_t key[40];
    uint32_t host[mg::kRssTableWords];           // the upload's source, kept with the tables
    uint32_t *d;
};

std::mutex &rss_mutex() {
    static std::mutex *m = new std::mutex;
    return *m;
}
std::vector<RssTables *> &rss_cache() {
    static std::vector<RssTables *> *v = new std::vector<RssTables *>;
    return *v;
}

// Bound of the one wait at mtcp_gpu_open (a new key's table upload on the
// new context's stream), before any limit can be set on the context.
constexpr uint32_t kOpenWaitUs = 2000000;

int rss_tables_for(int device, const uint8_t key[40], hipStream_t st, const uint32_t **out) {
    {
        std::lock_guard<std::mutex> lk(rss_mutex());
        for (const RssTables *t : rss_cache())
            if (t->device == device && memcmp(t->key, key, 40) == 0) {
                *out = t->d;
                return MTCP_GPU_OK;
            }
    }
    RssTables *t = new (std::nothrow) RssTables;
    if (!t) return MTCP_GPU_ENOMEM;
    t->device = device;
    memcpy(t->key, key, 40);
    build_rss_tables(key, t->host);
    if (!HIP_OK(hipMalloc(&t->d, sizeof(t->host)))) {
        delete t;
        return MTCP_GPU_ENOMEM;
    }
    int rc = HIP_OK(hipMemcpyAsync(t->d, t->host, sizeof(t->host), hipMemcpyHostToDevice, st))
                 ? drain(st, Deadline(kOpenWaitUs)) : MTCP_GPU_EIO;
    if (rc != MTCP_GPU_OK) return rc;            // t and its buffer stay (the copy may still run)
    std::lock_guard<std::mutex> lk(rss_mutex());
    rss_cache().push_back(t);
    *out = t->d;
    return MTCP_GPU_OK;
}

// The size hint of a host-side batch: its smallest and largest non-zero
// frame length ({0, 0} when every length is 0).
mtcp_gpu_size_hint size_hint(const mtcp_gpu_desc *desc, uint32_t n) {
    mtcp_gpu_size_hint h = {0xFFFF, 0};
    for (uint32_t i = 0; i < n; ++i)
        if (desc[i].len) h.min_len = std::min(h.min_len, desc[i].len), h.max_len = std::max(h.max_len, desc[i].len);
    if (!h.max_len) h.min_len = 0;
    return h;
}

bool offsets_sorted(const mtcp_gpu_desc *desc, uint32_t n) {
    for (uint32_t i = 1; i < n; ++i)
        if (desc[i].offset < desc[i - 1].offset) return false;
    return true;
}

}  // namespace

extern "C" {

int mtcp_gpu_abi_version(void) { return MTCP_GPU_ABI_VERSION; }

const char *mtcp_gpu_strerror(int err) {
    switch (err) {
        case MTCP_GPU_OK: return "success";
        case MTCP_GPU_EINVAL: return "invalid argument";
        case MTCP_GPU_ENOMEM: return "out of device or pinned host memory";
        case MTCP_GPU_ENODEV: return "no usable HIP device";
        case MTCP_GPU_EIO: return "HIP runtime error";
        case MTCP_GPU_ETIMEDOUT: return "GPU work not finished within the caller's limit";
        default: return "unknown error";
    }
}

int mtcp_gpu_device_count(void) {
    int n = 0;
    if (!HIP_OK(hipGetDeviceCount(&n))) return 0;
    return n;
}

int mtcp_gpu_device_pci_bus_id(int device, char *buf, int len) {
    if (!buf || len < 13) return MTCP_GPU_EINVAL;
    int ndev = 0;
    if (!HIP_OK(hipGetDeviceCount(&ndev)) || device < 0 || device >= ndev) return MTCP_GPU_ENODEV;
    return HIP_OK(hipDeviceGetPCIBusId(buf, len, device)) ? MTCP_GPU_OK : MTCP_GPU_EIO;
}

int mtcp_gpu_open(mtcp_gpu_ctx **out, int device, const uint8_t *rss_key, int rss_num_queues,
                  uint32_t flags) {
    static const uint8_t key05[40] = {
        5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5,
        5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5};
    if (!out) return MTCP_GPU_EINVAL;
    *out = nullptr;
    if ((flags & MTCP_GPU_F_RSS) && rss_num_queues < 1) return MTCP_GPU_EINVAL;
    int ndev = 0;
    if (!HIP_OK(hipGetDeviceCount(&ndev)) || device < 0 || device >= ndev) return MTCP_GPU_ENODEV;
    DeviceGuard dg(device);
    if (!dg.ok) return MTCP_GPU_ENODEV;

    mtcp_gpu_ctx *ctx = new (std::nothrow) mtcp_gpu_ctx();
    if (!ctx) return MTCP_GPU_ENOMEM;
    ctx->device = device;
    ctx->flags = flags;
    ctx->rss_nq = (uint32_t)std::max(1, rss_num_queues);
    ctx->rss_endian = (flags & MTCP_GPU_F_RSS_ENDIAN) ? 1u : 0u;
    hipDeviceProp_t prop;
    if (HIP_OK(hipGetDeviceProperties(&prop, device)) && prop.multiProcessorCount > 0)
        ctx->num_cu = prop.multiProcessorCount;

    const uint8_t *key = rss_key ? rss_key : key05;
    for (int i = 0; i < 4; ++i)
        ctx->rss_key_w[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
                            ((uint32_t)key[4 * i + 2] << 8) | (uint32_t)key[4 * i + 3];
    ctx->sched = sched_from_env();
    // one stream per context: its device-resident launches, the host calls
    // that fit one stage and its rxqs all go on it (the context's tables are
    // uploaded on it too, never through the null stream)
    int rc = HIP_OK(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking)) ? MTCP_GPU_OK : MTCP_GPU_ENOMEM;
    if (rc == MTCP_GPU_OK) rc = rss_tables_for(device, key, ctx->stream, &ctx->d_rss_tables);
    if (rc == MTCP_GPU_ETIMEDOUT) {
        ctx->abandoned = true;                   // the upload may still run: leave the stream
        delete ctx;
        return rc;
    }
    if (rc != MTCP_GPU_OK) {
        mtcp_gpu_close(ctx);
        return rc;
    }
    ctx->stage[0].stream = ctx->stream;
    *out = ctx;
    return MTCP_GPU_OK;
}

void mtcp_gpu_close(mtcp_gpu_ctx *ctx) {
    if (!ctx) return;
    DeviceGuard dg(ctx->device);
    if (!ctx->abandoned) {
        // the context's own work finishes first (within its wait limit, if
        // it has one: a device that does not finish it gets the context
        // abandoned instead).  Work the caller queued on its own streams is
        // not waited for: the RSS tables it may read are never freed
        // (rss_tables_for), every other buffer of such a launch is the caller's.
        const Deadline dl(ctx->wait_us);
        for (auto &s : ctx->stage)
            if (s.own_stream && drain(s.stream, dl) == MTCP_GPU_ETIMEDOUT) ctx->abandoned = true;
        if (ctx->stream && drain(ctx->stream, dl) == MTCP_GPU_ETIMEDOUT) ctx->abandoned = true;
    }
    if (ctx->abandoned) {
        // work a timed-out wait gave up on may still copy into the staging:
        // leave every stream and buffer allocated (never touched again)
        // rather than block on a device that stopped answering or free
        // memory under its DMA; only the host-side struct goes
        delete ctx;
        return;
    }
    // every buffer goes back to park.hpp: a free here would wait for the
    // other contexts' work on the device (with a wait limit not even a
    // buffer too large to park is freed)
    const bool may_free = ctx->wait_us == 0;
    for (auto &s : ctx->stage) {
        if (s.own_stream) (void)hipStreamDestroy(s.stream);
        stage_release_buf(s, may_free);
        stage_release_pkts(s, may_free);
        stage_release_host(s, may_free);
    }
    mtcp_park::release(ctx->h_gather, ctx->h_gather_cap, mtcp_park::kHost, may_free);
    mtcp_park::release(ctx->h_gather_desc, (size_t)ctx->h_gather_desc_cap * sizeof(mtcp_gpu_desc),
                       mtcp_park::kHost, may_free);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

int mtcp_gpu_set_wait_limit(mtcp_gpu_ctx *ctx, uint32_t timeout_us) {
    if (!ctx) return MTCP_GPU_EINVAL;
    ctx->wait_us = timeout_us;
    return MTCP_GPU_OK;
}

uint32_t mtcp_gpu_wait_limit(const mtcp_gpu_ctx *ctx) { return ctx ? ctx->wait_us : 0u; }

bool mg_ctx_abandoned(const mtcp_gpu_ctx *ctx) { return ctx && ctx->abandoned; }

int mtcp_gpu_reserve(mtcp_gpu_ctx *ctx, uint64_t max_bytes, uint32_t max_pkts) {
    if (!ctx) return MTCP_GPU_EINVAL;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    DeviceGuard dg(ctx->device);
    if (!dg.ok) return MTCP_GPU_ENODEV;
    const Deadline dl(ctx->wait_us);
    // a host call's batches span at most kStageBytes / kStagePkts and start
    // at stage 0; later stages are used only by calls larger than one stage
    const uint64_t bytes = std::min(max_bytes, kStageBytes);
    const uint32_t pkts = std::min(max_pkts, kStagePkts);
    const int stages = max_bytes == 0 && max_pkts == 0                  ? 0   // kernels only
                       : max_bytes > kStageBytes || max_pkts > kStagePkts ? kStages
                                                                          : 1;
    for (int i = 0; i < stages; ++i) {
        const int rc = stage_reserve(ctx, ctx->stage[i], ((bytes + 15) & ~15ull) + 16, std::max(pkts, 1u), dl);
        if (rc != MTCP_GPU_OK) return rc;
    }
    // a stream sets up its copy queues on its first large copy (7.8 ms
    // measured): do that here for the stages the host calls use, with the
    // pinned buffers a bounded context's calls go through
    const size_t warm = stages ? (size_t)std::min<uint64_t>(ctx->stage[0].buf_cap, 1ull << 20) : 0;
    int rc = MTCP_GPU_OK;
    for (int i = 0; i < stages && rc == MTCP_GPU_OK; ++i) {
        Stage &st = ctx->stage[i];
        rc = stage_host(ctx, st, warm, warm, dl);
        if (rc == MTCP_GPU_OK) {
            memset(st.h_in, 0, warm);
            if (!HIP_OK(hipMemcpyAsync(st.d_buf, st.h_in, warm, hipMemcpyHostToDevice, st.stream)) ||
                !HIP_OK(hipMemcpyAsync(st.h_out, st.d_buf, warm, hipMemcpyDeviceToHost, st.stream)))
                rc = MTCP_GPU_EIO;
        }
    }
    rc = finish_call(ctx, rc, dl, stages);
    if (rc != MTCP_GPU_OK) return rc;
    // the code object loads on the first launch of any of its kernels
    hipFuncAttributes attr;
    if (!HIP_OK(hipFuncGetAttributes(
            &attr, reinterpret_cast<const void *>(
                       &mg::rx_kernel<mg::kRxChunk, false, mg::kSchedSorted, false, 0, 8, 8, true, 6, false>))))
        return MTCP_GPU_EIO;
    return MTCP_GPU_OK;
}

int mtcp_gpu_dev_ioctl(mtcp_gpu_ctx *ctx, int nif, int cmd, void *argp) {
    (void)nif;
    (void)argp;
    if (!ctx) return -1;
    switch (cmd) {   // the commands this device computes (dpdk_module.c:809-816 contract)
        case MTCP_GPU_PKT_RX_IP_CSUM:
        case MTCP_GPU_PKT_RX_TCP_CSUM:
        case MTCP_GPU_PKT_TX_IP_CSUM:
        case MTCP_GPU_PKT_TX_TCPIP_CSUM:
            return 0;
        default:
            return -1;
    }
}

void *mtcp_gpu_stream(mtcp_gpu_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

uint32_t mtcp_gpu_record_size(const mtcp_gpu_ctx *ctx) { return ctx ? (uint32_t)record_size(ctx) : 0u; }

const char *mtcp_gpu_last_kernel(const mtcp_gpu_ctx *ctx) { return ctx ? ctx->last_kernel : ""; }

int mtcp_gpu_sync(mtcp_gpu_ctx *ctx) {
    if (!ctx) return MTCP_GPU_EINVAL;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    DeviceGuard dg(ctx->device);
    // with a wait limit: MTCP_GPU_ETIMEDOUT past it, and the context stays
    // usable (what is still running is the caller's own device work)
    return drain(ctx->stream, Deadline(ctx->wait_us));
}

int mtcp_gpu_rx_chunk_flow_dev(mtcp_gpu_ctx *ctx, const void *d_buf, uint64_t buf_len,
                               const mtcp_gpu_desc *d_desc, uint32_t n, uint32_t off_shift,
                               mtcp_gpu_result *d_out, uint32_t *d_bins, void *stream) {
    return mtcp_gpu_rx_chunk_hint_dev(ctx, d_buf, buf_len, d_desc, n, off_shift, d_out, d_bins, nullptr, stream);
}

int mtcp_gpu_rx_chunk_hint_dev(mtcp_gpu_ctx *ctx, const void *d_buf, uint64_t buf_len,
                               const mtcp_gpu_desc *d_desc, uint32_t n, uint32_t off_shift,
                               mtcp_gpu_result *d_out, uint32_t *d_bins, const mtcp_gpu_size_hint *hint,
                               void *stream) {
    if (!ctx || (n && (!d_buf || !d_desc || !d_out)) || off_shift > 16 || (buf_len & 15) ||
        ((uintptr_t)d_buf & 15) || ((uintptr_t)d_out & out_align(ctx)) || ((uintptr_t)d_desc & 7) ||
        ((uintptr_t)d_bins & 3))
        return MTCP_GPU_EINVAL;
    DeviceGuard dg(ctx->device);
    mg::KParams kp = base_params(ctx);
    kp.buf = static_cast<const uint8_t *>(d_buf);
    kp.buf_len = buf_len;
    kp.desc = d_desc;
    kp.n = n;
    kp.off_shift = off_shift;
    kp.out = d_out;
    kp.bins = d_bins;
    return launch<mg::kRxChunk>(ctx, kp, pick(ctx, stream), hint);
}

int mtcp_gpu_rx_chunk_dev(mtcp_gpu_ctx *ctx, const void *d_buf, uint64_t buf_len,
                          const mtcp_gpu_desc *d_desc, uint32_t n, uint32_t off_shift,
                          mtcp_gpu_result *d_out, void *stream) {
    return mtcp_gpu_rx_chunk_flow_dev(ctx, d_buf, buf_len, d_desc, n, off_shift, d_out, nullptr, stream);
}

int mtcp_gpu_rx_ptrs_flow_dev(mtcp_gpu_ctx *ctx, const uint8_t *const *d_pkts, const uint16_t *d_lens,
                              uint32_t n, mtcp_gpu_result *d_out, uint32_t *d_bins, void *stream) {
    if (!ctx || (n && (!d_pkts || !d_lens || !d_out)) || ((uintptr_t)d_out & out_align(ctx)) ||
        ((uintptr_t)d_bins & 3))
        return MTCP_GPU_EINVAL;
    DeviceGuard dg(ctx->device);
    mg::KParams kp = base_params(ctx);
    kp.ptrs = d_pkts;
    kp.lens = d_lens;
    kp.n = n;
    kp.out = d_out;
    kp.bins = d_bins;
    return launch<mg::kRxPtrs>(ctx, kp, pick(ctx, stream));
}

int mtcp_gpu_rx_ptrs_dev(mtcp_gpu_ctx *ctx, const uint8_t *const *d_pkts, const uint16_t *d_lens,
                         uint32_t n, mtcp_gpu_result *d_out, void *stream) {
    return mtcp_gpu_rx_ptrs_flow_dev(ctx, d_pkts, d_lens, n, d_out, nullptr, stream);
}

int mtcp_gpu_tx_fill_ptrs_dev(mtcp_gpu_ctx *ctx, uint8_t *const *d_pkts, const uint16_t *d_lens,
                              uint32_t n, void *stream) {
    if (!ctx || (n && (!d_pkts || !d_lens))) return MTCP_GPU_EINVAL;
    DeviceGuard dg(ctx->device);
    mg::KParams kp = base_params(ctx);
    kp.ptrs = reinterpret_cast<const uint8_t *const *>(d_pkts);
    kp.lens = d_lens;
    kp.n = n;
    return launch<mg::kTxPtrs>(ctx, kp, pick(ctx, stream));
}

int mtcp_gpu_tx_fill_dev(mtcp_gpu_ctx *ctx, void *d_buf, uint64_t buf_len,
                         const mtcp_gpu_desc *d_desc, uint32_t n, uint32_t off_shift,
                         void *stream) {
    if (!ctx || (n && (!d_buf || !d_desc)) || off_shift > 16 || (buf_len & 15) ||
        ((uintptr_t)d_buf & 15) || ((uintptr_t)d_desc & 7))
        return MTCP_GPU_EINVAL;
    DeviceGuard dg(ctx->device);
    mg::KParams kp = base_params(ctx);
    kp.buf = static_cast<const uint8_t *>(d_buf);
    kp.buf_len = buf_len;
    kp.desc = d_desc;
    kp.n = n;
    kp.off_shift = off_shift;
    return launch<mg::kTxChunk>(ctx, kp, pick(ctx, stream));
}

}  // extern "C"

namespace {

// Host-memory rx (mtcp_gpu_rx_chunk, _rx_ptrs): batches of packets stream
// through kStages stages — stage 0 on the context's stream, 1 and 2 on their
// own — so that the H2D of batch b+1 overlaps the kernel of b and the D2H of
// b-1.  Each batch copies only the byte span its packets occupy and the
// kernel rebases descriptor offsets by that span's start.  Unbounded (the
// context has no wait limit): the copies read the caller's chunk and write
// its records directly.  Bounded: every byte passes through the stages'
// pinned bounce buffers (`owned`: buf / desc already are the context's own
// pinned gather and are not copied again), so that no copy the call gives up
// on at its deadline can touch the caller's memory afterwards.
int rx_host(mtcp_gpu_ctx *ctx, const uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc, uint32_t n,
            uint32_t off_shift, mtcp_gpu_result *out, bool owned, const Deadline &dl) {
    int rc = MTCP_GPU_OK;
    uint8_t *const out_b = reinterpret_cast<uint8_t *>(out);
    const size_t rec = (size_t)record_size(ctx);
    const bool bounce = dl.bounded;
    const uint64_t out_bytes = (uint64_t)kStagePkts * rec;
    if (!offsets_sorted(desc, n)) {
        // arbitrary order: stage the whole chunk once, then batches of descriptors
        Stage &s = ctx->stage[0];
        const uint64_t padded = (buf_len + 15) & ~15ull;
        rc = stage_reserve(ctx, s, padded + 16, kStagePkts, dl);
        if (rc == MTCP_GPU_OK && bounce)
            rc = stage_host(ctx, s, owned ? 0 : padded + (uint64_t)kStagePkts * sizeof(mtcp_gpu_desc), out_bytes, dl);
        const uint8_t *src = buf;
        if (rc == MTCP_GPU_OK && bounce && !owned) {
            bounce_in(s.h_in, buf, buf_len);
            src = s.h_in;
        }
        if (rc == MTCP_GPU_OK && !HIP_OK(hipMemcpyAsync(s.d_buf, src, buf_len, hipMemcpyHostToDevice, s.stream)))
            rc = MTCP_GPU_EIO;
        for (uint32_t first = 0; first < n && rc == MTCP_GPU_OK; first += kStagePkts) {
            const uint32_t cnt = std::min(n - first, kStagePkts);
            if ((rc = stage_collect(ctx, s, out_b, rec, dl)) != MTCP_GPU_OK) break;   // the previous batch
            const mtcp_gpu_desc *dsrc = desc + first;
            if (bounce && !owned) {
                mtcp_gpu_desc *d = reinterpret_cast<mtcp_gpu_desc *>(s.h_in + padded);
                memcpy(d, desc + first, (size_t)cnt * sizeof(mtcp_gpu_desc));
                dsrc = d;
            }
            const mtcp_gpu_size_hint hint = size_hint(desc + first, cnt);
            mg::KParams kp = base_params(ctx);
            kp.buf = s.d_buf;
            kp.buf_len = buf_len;
            kp.desc = s.d_desc;
            kp.n = cnt;
            kp.off_shift = off_shift;
            kp.out = s.d_out;
            if (!HIP_OK(hipMemcpyAsync(s.d_desc, dsrc, (size_t)cnt * sizeof(mtcp_gpu_desc),
                                       hipMemcpyHostToDevice, s.stream)))
                rc = MTCP_GPU_EIO;
            if (rc == MTCP_GPU_OK) rc = launch<mg::kRxChunk>(ctx, kp, s.stream, &hint);
            if (rc == MTCP_GPU_OK &&
                !HIP_OK(hipMemcpyAsync(bounce ? s.h_out : out_b + first * rec, s.d_out, cnt * rec,
                                       hipMemcpyDeviceToHost, s.stream)))
                rc = MTCP_GPU_EIO;
            if (rc == MTCP_GPU_OK && bounce) s.pend_first = first, s.pend_cnt = cnt;
        }
    } else {
        uint32_t first = 0;
        for (int b = 0; first < n && rc == MTCP_GPU_OK; ++b) {
            // grow the batch while its byte span fits one stage
            const uint64_t lo = std::min(((uint64_t)desc[first].offset << off_shift) & ~15ull,
                                         buf_len & ~15ull);
            uint64_t hi = lo;
            uint32_t cnt = 0;
            mtcp_gpu_size_hint hint = {0xFFFF, 0};
            while (first + cnt < n && cnt < kStagePkts) {
                const uint64_t p = (uint64_t)desc[first + cnt].offset << off_shift;
                const uint16_t len = desc[first + cnt].len;
                const uint64_t end = std::max(std::min(p + len, buf_len), lo);
                if (cnt > 0 && std::max(hi, end) - lo > kStageBytes) break;
                hi = std::max(hi, end);
                if (len) hint.min_len = std::min(hint.min_len, len), hint.max_len = std::max(hint.max_len, len);
                ++cnt;
            }
            if (!hint.max_len) hint.min_len = 0;
            Stage &s = ctx->stage[b % kStages];
            const uint64_t span = hi - lo, padded = (span + 15) & ~15ull;
            if ((rc = stage_collect(ctx, s, out_b, rec, dl)) != MTCP_GPU_OK) break;   // its batch b - kStages
            rc = stage_reserve(ctx, s, padded + 16, kStagePkts, dl);
            if (rc == MTCP_GPU_OK && bounce)
                rc = stage_host(ctx, s, owned ? 0 : padded + (uint64_t)cnt * sizeof(mtcp_gpu_desc), out_bytes, dl);
            if (rc != MTCP_GPU_OK) break;
            const uint8_t *src = buf + lo;
            const mtcp_gpu_desc *dsrc = desc + first;
            if (bounce && !owned) {
                bounce_in(s.h_in, buf + lo, span);
                memcpy(s.h_in + padded, desc + first, (size_t)cnt * sizeof(mtcp_gpu_desc));
                src = s.h_in;
                dsrc = reinterpret_cast<const mtcp_gpu_desc *>(s.h_in + padded);
            }
            mg::KParams kp = base_params(ctx);
            kp.buf = s.d_buf;
            kp.buf_len = span;           // descriptors are bounded by the caller's buf_len
            kp.base_sub = (int64_t)lo;
            kp.desc = s.d_desc;
            kp.n = cnt;
            kp.off_shift = off_shift;
            kp.out = s.d_out;
            if ((span && !HIP_OK(hipMemcpyAsync(s.d_buf, src, span, hipMemcpyHostToDevice, s.stream))) ||
                !HIP_OK(hipMemcpyAsync(s.d_desc, dsrc, (size_t)cnt * sizeof(mtcp_gpu_desc),
                                       hipMemcpyHostToDevice, s.stream)))
                rc = MTCP_GPU_EIO;
            if (rc == MTCP_GPU_OK) rc = launch<mg::kRxChunk>(ctx, kp, s.stream, &hint);
            if (rc == MTCP_GPU_OK &&
                !HIP_OK(hipMemcpyAsync(bounce ? s.h_out : out_b + first * rec, s.d_out, cnt * rec,
                                       hipMemcpyDeviceToHost, s.stream)))
                rc = MTCP_GPU_EIO;
            if (rc == MTCP_GPU_OK && bounce) s.pend_first = first, s.pend_cnt = cnt;
            first += cnt;
        }
    }
    // a stage_collect that timed out has abandoned the context already: no
    // more waits, and no stage's records are copied out
    if (rc == MTCP_GPU_ETIMEDOUT) {
        for (auto &t : ctx->stage) t.pend_cnt = 0;
        return rc;
    }
    return finish_call(ctx, rc, dl, kStages, out_b, rec);
}

// Gather a pointer burst into the context's pinned PSIO-style chunk (64 B
// aligned slots, pslib.c:146) with its descriptors; *total = chunk bytes.
int gather_burst(mtcp_gpu_ctx *ctx, const uint8_t *const *pkts, const uint16_t *lens, uint32_t n,
                 uint64_t *total_out, const Deadline &dl) {
    if (ctx->abandoned) return MTCP_GPU_EIO;     // its staging may still be under DMA
    const bool may_free = !dl.bounded;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) total += ((uint64_t)lens[i] + 63) & ~63ull;
    if (total > ctx->h_gather_cap) {
        mtcp_park::release(ctx->h_gather, ctx->h_gather_cap, mtcp_park::kHost, may_free);
        ctx->h_gather = nullptr;
        ctx->h_gather_cap = 0;
        if (!HIP_OK(mtcp_park::alloc(&ctx->h_gather, total, mtcp_park::kHost))) return MTCP_GPU_ENOMEM;
        ctx->h_gather_cap = total;
    }
    if (n > ctx->h_gather_desc_cap) {
        mtcp_park::release(ctx->h_gather_desc, (size_t)ctx->h_gather_desc_cap * sizeof(mtcp_gpu_desc),
                           mtcp_park::kHost, may_free);
        ctx->h_gather_desc = nullptr;
        ctx->h_gather_desc_cap = 0;
        if (!HIP_OK(mtcp_park::alloc(&ctx->h_gather_desc, (size_t)n * sizeof(mtcp_gpu_desc), mtcp_park::kHost)))
            return MTCP_GPU_ENOMEM;
        ctx->h_gather_desc_cap = n;
    }
    uint64_t off = 0;
    for (uint32_t i = 0; i < n; ++i) {
        mtcp_gpu_desc &d = ctx->h_gather_desc[i];
        d.offset = (uint32_t)(off >> 6);
        d.len = lens[i];
        d.flags = d.rsvd = 0;
        if (pkts[i]) stage_copy(ctx->h_gather + off, pkts[i], lens[i]);
        else d.len = 0xFFFF, d.offset = 0xFFFFFFFFu;   // -> BAD_DESC
        off += ((uint64_t)lens[i] + 63) & ~63ull;
    }
    stage_fence();
    *total_out = total;
    return MTCP_GPU_OK;
}

// The two check fields of a filled frame (the tx kernels' report: {ip check
// | tcp check << 16, T}, T the TCP header's offset, 0 = not filled), written
// by the calling thread: iph->check (ip_out.c:164), tcph->check (tcp_out.c:329)
inline void write_checks(uint8_t *frame, uint2 r) {
    const uint16_t ipc = (uint16_t)r.x, tcpc = (uint16_t)(r.x >> 16);
    memcpy(frame + 24, &ipc, 2);
    memcpy(frame + r.y + 16, &tcpc, 2);
}

}  // namespace

extern "C" {

int mtcp_gpu_rx_chunk(mtcp_gpu_ctx *ctx, const uint8_t *buf, uint64_t buf_len,
                      const mtcp_gpu_desc *desc, uint32_t n, uint32_t off_shift,
                      mtcp_gpu_result *out) {
    if (!ctx || (n && (!buf || !desc || !out)) || off_shift > 16) return MTCP_GPU_EINVAL;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (n == 0) return MTCP_GPU_OK;
    DeviceGuard dg(ctx->device);
    return rx_host(ctx, buf, buf_len, desc, n, off_shift, out, false, Deadline(ctx->wait_us));
}

int mtcp_gpu_rx_ptrs(mtcp_gpu_ctx *ctx, const uint8_t *const *pkts, const uint16_t *lens,
                     uint32_t n, mtcp_gpu_result *out) {
    if (!ctx || (n && (!pkts || !lens || !out))) return MTCP_GPU_EINVAL;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (n == 0) return MTCP_GPU_OK;
    DeviceGuard dg(ctx->device);
    const Deadline dl(ctx->wait_us);
    uint64_t total = 0;
    const int rc = gather_burst(ctx, pkts, lens, n, &total, dl);
    if (rc != MTCP_GPU_OK) return rc;
    return rx_host(ctx, ctx->h_gather, total, ctx->h_gather_desc, n, 6, out, true, dl);
}

// tx fill of a host pointer burst (a DPDK wmbufs[].m_table, dpdk_module.c:341-370):
// the frames are gathered into pinned staging and checked on the GPU, which
// reports {checks, T} per frame (the tx kernels' report mode); only the two
// check fields are written back into the caller's frames, here on the host,
// once the report is in.  With a limit (timeout_us, else the context's wait
// limit) the wait polls the device: past the limit nothing has been written
// into the caller's frames, the call answers MTCP_GPU_ETIMEDOUT and the
// context is abandoned (the copies may still run into its staging).  mTCP's
// own tx fill never waits on a device (tcp_out.c:320-329, ip_out.c:147-165,
// run from RunMainLoop core.c:818-824): the caller fills the frames itself.
int mtcp_gpu_tx_fill_ptrs_for(mtcp_gpu_ctx *ctx, uint8_t *const *pkts, const uint16_t *lens, uint32_t n,
                              uint32_t *n_filled, uint32_t timeout_us) {
    if (!ctx || (n && (!pkts || !lens))) return MTCP_GPU_EINVAL;
    if (n_filled) *n_filled = 0;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (n == 0) return MTCP_GPU_OK;
    DeviceGuard dg(ctx->device);
    const Deadline dl(timeout_us ? timeout_us : ctx->wait_us);
    uint64_t total = 0;
    int rc = gather_burst(ctx, pkts, lens, n, &total, dl);
    if (rc != MTCP_GPU_OK) return rc;
    Stage &s = ctx->stage[0];
    rc = stage_reserve(ctx, s, ((total + 15) & ~15ull) + 16, n, dl);
    if (rc != MTCP_GPU_OK) return rc;
    uint2 *report = reinterpret_cast<uint2 *>(ctx->h_gather_desc);    // reused once the H2D is done
    static_assert(sizeof(uint2) == sizeof(mtcp_gpu_desc), "report reuses the descriptor staging");
    if (!HIP_OK(hipMemcpyAsync(s.d_buf, ctx->h_gather, total, hipMemcpyHostToDevice, s.stream)) ||
        !HIP_OK(hipMemcpyAsync(s.d_desc, ctx->h_gather_desc, (size_t)n * sizeof(mtcp_gpu_desc),
                               hipMemcpyHostToDevice, s.stream)))
        rc = MTCP_GPU_EIO;
    mg::KParams kp = base_params(ctx);
    kp.buf = s.d_buf;
    kp.buf_len = total;
    kp.desc = s.d_desc;
    kp.n = n;
    kp.off_shift = 6;
    kp.tx_report = reinterpret_cast<uint2 *>(s.d_out);                // n x 8 B <= n x 40 B
    if (rc == MTCP_GPU_OK) rc = launch<mg::kTxChunk>(ctx, kp, s.stream);
    if (rc == MTCP_GPU_OK && !HIP_OK(hipMemcpyAsync(report, s.d_out, (size_t)n * sizeof(uint2),
                                                    hipMemcpyDeviceToHost, s.stream)))
        rc = MTCP_GPU_EIO;
    // every path drains the stream within the deadline, a failed enqueue's
    // too: an H2D already queued may be reading the staging
    rc = finish_call(ctx, rc, dl, 1);
    if (rc != MTCP_GPU_OK) return rc;
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < n; ++i) {
        if (!report[i].y) continue;
        write_checks(pkts[i], report[i]);
        ++cnt;
    }
    if (n_filled) *n_filled = cnt;
    return MTCP_GPU_OK;
}

int mtcp_gpu_tx_fill_ptrs(mtcp_gpu_ctx *ctx, uint8_t *const *pkts, const uint16_t *lens, uint32_t n,
                          uint32_t *n_filled) {
    return mtcp_gpu_tx_fill_ptrs_for(ctx, pkts, lens, n, n_filled, 0);
}

// tx fill of a host chunk, in place: the chunk goes to the GPU once, the
// kernel reports {checks, T} per frame (n x 8 B back instead of the whole
// chunk) and the calling thread writes the two check fields of each filled
// frame.  Bounded (a context wait limit): the chunk and the descriptors are
// copied into pinned bounce buffers first, so that no copy given up on at
// the deadline reads the caller's memory later, and nothing is written into
// the chunk unless the report came in time.
int mtcp_gpu_tx_fill(mtcp_gpu_ctx *ctx, uint8_t *buf, uint64_t buf_len, const mtcp_gpu_desc *desc,
                     uint32_t n, uint32_t off_shift, uint32_t *n_filled) {
    if (!ctx || (n && (!buf || !desc)) || off_shift > 16) return MTCP_GPU_EINVAL;
    if (n_filled) *n_filled = 0;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (n == 0) return MTCP_GPU_OK;
    DeviceGuard dg(ctx->device);
    const Deadline dl(ctx->wait_us);
    const bool bounce = dl.bounded;
    Stage &s = ctx->stage[0];
    const uint64_t padded = (buf_len + 15) & ~15ull;
    const uint64_t dbytes = (uint64_t)n * sizeof(mtcp_gpu_desc);
    int rc = stage_reserve(ctx, s, padded + 16, n, dl);
    if (rc == MTCP_GPU_OK) rc = stage_host(ctx, s, bounce ? padded + dbytes : 0, (uint64_t)n * sizeof(uint2), dl);
    if (rc != MTCP_GPU_OK) return rc;
    const uint8_t *src = buf;
    const mtcp_gpu_desc *dsrc = desc;
    if (bounce) {
        bounce_in(s.h_in, buf, buf_len);
        memcpy(s.h_in + padded, desc, dbytes);
        src = s.h_in;
        dsrc = reinterpret_cast<const mtcp_gpu_desc *>(s.h_in + padded);
    }
    // the 16 B past the chunk (the kernels' last vector load of a frame
    // ending there) read as zeros
    if (!HIP_OK(hipMemsetAsync(s.d_buf + (buf_len & ~15ull), 0, 16, s.stream)) ||
        !HIP_OK(hipMemcpyAsync(s.d_buf, src, buf_len, hipMemcpyHostToDevice, s.stream)) ||
        !HIP_OK(hipMemcpyAsync(s.d_desc, dsrc, dbytes, hipMemcpyHostToDevice, s.stream)))
        rc = MTCP_GPU_EIO;
    mg::KParams kp = base_params(ctx);
    kp.buf = s.d_buf;
    kp.buf_len = buf_len;   // descriptor bound: the caller's length
    kp.desc = s.d_desc;
    kp.n = n;
    kp.off_shift = off_shift;
    kp.tx_report = reinterpret_cast<uint2 *>(s.d_out);                // n x 8 B <= n x 40 B
    uint2 *report = reinterpret_cast<uint2 *>(s.h_out);
    if (rc == MTCP_GPU_OK) rc = launch<mg::kTxChunk>(ctx, kp, s.stream);
    if (rc == MTCP_GPU_OK && !HIP_OK(hipMemcpyAsync(report, s.d_out, (size_t)n * sizeof(uint2),
                                                    hipMemcpyDeviceToHost, s.stream)))
        rc = MTCP_GPU_EIO;
    rc = finish_call(ctx, rc, dl, 1);
    if (rc != MTCP_GPU_OK) return rc;
    uint32_t cnt = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t off = (uint64_t)desc[i].offset << off_shift;
        // the kernel reports only frames inside the chunk (checked again here)
        if (!report[i].y || off + report[i].y + 18 > buf_len) continue;
        write_checks(buf + off, report[i]);
        ++cnt;
    }
    if (n_filled) *n_filled = cnt;
    return MTCP_GPU_OK;
}

// ---- flow-table hash --------------------------------------
int mtcp_gpu_flow_hash_dev(mtcp_gpu_ctx *ctx, const mtcp_gpu_result *d_res, uint32_t n,
                           uint32_t *d_bins, void *stream) {
    if (!ctx || (n && (!d_res || !d_bins)) || ((uintptr_t)d_res & 7) || ((uintptr_t)d_bins & 3) ||
        (ctx->flags & MTCP_GPU_F_COMPACT))          // reads 40 B records (the 4-tuple)
        return MTCP_GPU_EINVAL;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (n == 0) return MTCP_GPU_OK;
    DeviceGuard dg(ctx->device);
    const uint32_t blocks = std::min<uint32_t>((n + mg::kBlock - 1) / mg::kBlock,
                                               (uint32_t)ctx->num_cu * 8);
    hipLaunchKernelGGL(mg::flow_hash_kernel, dim3(blocks), dim3(mg::kBlock), 0, pick(ctx, stream),
                       d_res, n, d_bins);
    return HIP_OK(hipGetLastError()) ? MTCP_GPU_OK : MTCP_GPU_EIO;
}

int mtcp_gpu_flow_hash(mtcp_gpu_ctx *ctx, const mtcp_gpu_result *res, uint32_t n,
                       uint32_t *bins) {
    if (!ctx || (n && (!res || !bins)) || (ctx->flags & MTCP_GPU_F_COMPACT)) return MTCP_GPU_EINVAL;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (n == 0) return MTCP_GPU_OK;
    DeviceGuard dg(ctx->device);
    const Deadline dl(ctx->wait_us);
    const bool bounce = dl.bounded;
    const uint64_t rbytes = (uint64_t)n * sizeof(mtcp_gpu_result), bbytes = (uint64_t)n * sizeof(uint32_t);
    Stage &s = ctx->stage[0];
    int rc = stage_reserve(ctx, s, bbytes, n, dl);
    if (rc == MTCP_GPU_OK && bounce) rc = stage_host(ctx, s, rbytes, bbytes, dl);
    if (rc != MTCP_GPU_OK) return rc;
    const void *src = res;
    if (bounce) {
        memcpy(s.h_in, res, rbytes);
        src = s.h_in;
    }
    uint32_t *d_bins = reinterpret_cast<uint32_t *>(s.d_buf);
    if (!HIP_OK(hipMemcpyAsync(s.d_out, src, rbytes, hipMemcpyHostToDevice, s.stream)))
        rc = MTCP_GPU_EIO;
    if (rc == MTCP_GPU_OK) rc = mtcp_gpu_flow_hash_dev(ctx, s.d_out, n, d_bins, s.stream);
    if (rc == MTCP_GPU_OK && !HIP_OK(hipMemcpyAsync(bounce ? (void *)s.h_out : (void *)bins, d_bins, bbytes,
                                                    hipMemcpyDeviceToHost, s.stream)))
        rc = MTCP_GPU_EIO;
    rc = finish_call(ctx, rc, dl, 1);
    if (rc == MTCP_GPU_OK && bounce) memcpy(bins, s.h_out, bbytes);
    return rc;
}

// ---- RSS-friendly address pool -----------------------------
int mtcp_gpu_rss_queue_map_dev(mtcp_gpu_ctx *ctx, uint32_t saddr_base_h, uint32_t num_addr,
                               uint32_t daddr_h, uint16_t dport_h, int num_queues,
                               int endian_check, uint8_t *d_queue, void *stream) {
    if (!ctx || num_queues < 1 || (num_addr && !d_queue) || ((uintptr_t)d_queue & 3))
        return MTCP_GPU_EINVAL;
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (num_addr == 0) return MTCP_GPU_OK;
    DeviceGuard dg(ctx->device);
    mg::PoolParams pp{};
    pp.rss_tables = ctx->d_rss_tables;
    pp.saddr_base_h = saddr_base_h;
    pp.daddr_h = daddr_h;
    pp.dport_h = dport_h;
    pp.nq = (uint32_t)num_queues;
    pp.endian = endian_check ? 1u : 0u;
    pp.total = (uint64_t)num_addr * mg::kPorts;
    // one tile of kQmapTile candidates per workgroup, up to 8 workgroups per
    // CU (the kernel walks further tiles grid-stride)
    const uint64_t tiles = (pp.total + mg::kQmapTile - 1) / mg::kQmapTile;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(tiles, (uint64_t)ctx->num_cu * 8);
    hipLaunchKernelGGL(mg::rss_queue_map_kernel, dim3(blocks), dim3(mg::kBlock), 0,
                       pick(ctx, stream), pp, d_queue);
    return HIP_OK(hipGetLastError()) ? MTCP_GPU_OK : MTCP_GPU_EIO;
}

int mtcp_gpu_addr_pool_search(mtcp_gpu_ctx *ctx, int core, int num_queues, uint32_t saddr_base,
                              int num_addr, uint32_t daddr, uint16_t dport, int endian_check,
                              mtcp_gpu_addr_entry *out, uint32_t max_out, uint32_t *n_found) {
    if (!ctx || num_queues < 1 || num_addr < 0 || !n_found || (max_out && !out))
        return MTCP_GPU_EINVAL;
    *n_found = 0;
    // addr_pool.c:129 computes num_entry in int: keep the product in range
    const uint64_t total = (uint64_t)num_addr * mg::kPorts;
    if (total > (uint64_t)INT32_MAX) return MTCP_GPU_EINVAL;
    const uint32_t num_entry = (uint32_t)((int)total / num_queues);
    if (ctx->abandoned) return MTCP_GPU_EIO;
    if (num_addr == 0 || core < 0 || core >= num_queues) return MTCP_GPU_OK;
    DeviceGuard dg(ctx->device);
    const uint32_t nb = (uint32_t)((total + mg::kPoolTile - 1) / mg::kPoolTile);
    const uint32_t limit = std::min(num_entry, max_out);
    const uint64_t qbytes = (total + 15) & ~15ull;
    uint8_t *d_mem = nullptr;
    const uint64_t out_off = (qbytes + 4ull * (nb + 1) + 7) & ~7ull;     // 8 B aligned entries
    const uint64_t bytes = out_off + 8ull * std::max(limit, 1u);
    if (!HIP_OK(mtcp_park::alloc(&d_mem, bytes, mtcp_park::kDevice))) return MTCP_GPU_ENOMEM;
    uint8_t *d_queue = d_mem;
    uint32_t *d_counts = reinterpret_cast<uint32_t *>(d_mem + qbytes);
    mtcp_gpu_addr_entry *d_out = reinterpret_cast<mtcp_gpu_addr_entry *>(d_mem + out_off);
    hipStream_t st = ctx->stream;
    const Deadline dl(ctx->wait_us);
    Stage &s0 = ctx->stage[0];                                             // its stream is st
    const uint32_t saddr_base_h = __builtin_bswap32(saddr_base);           // addr_pool.c:150
    int rc = mtcp_gpu_rss_queue_map_dev(ctx, saddr_base_h, (uint32_t)num_addr,
                                        __builtin_bswap32(daddr),
                                        (uint16_t)((dport >> 8) | (dport << 8)), num_queues,
                                        endian_check, d_queue, st);
    // what comes back lands in the stage's pinned buffer first (the count,
    // then the entries), copied out once its copy has finished
    if (rc == MTCP_GPU_OK) rc = stage_host(ctx, s0, 0, 8ull * std::max(limit, 1u), dl);
    if (rc == MTCP_GPU_OK) {
        hipLaunchKernelGGL(mg::pool_count_kernel, dim3(nb), dim3(mg::kBlock), 0, st, d_queue, total,
                           (uint32_t)core, d_counts);
        hipLaunchKernelGGL(mg::pool_scan_kernel, dim3(1), dim3(mg::kBlock), 0, st, d_counts, nb);
        if (limit)
            hipLaunchKernelGGL(mg::pool_emit_kernel, dim3(nb), dim3(mg::kBlock), 0, st, d_queue,
                               total, (uint32_t)core, d_counts, saddr_base_h, limit, d_out);
        if (!HIP_OK(hipGetLastError()) ||
            !HIP_OK(hipMemcpyAsync(s0.h_out, d_counts + nb, sizeof(uint32_t), hipMemcpyDeviceToHost, st)))
            rc = MTCP_GPU_EIO;
        rc = finish_call(ctx, rc, dl, 1);
    }
    if (rc == MTCP_GPU_OK) {
        uint32_t count;
        memcpy(&count, s0.h_out, sizeof(count));
        const uint32_t kept = std::min(count, num_entry);
        const uint32_t copy = std::min(kept, max_out);
        if (copy && !HIP_OK(hipMemcpyAsync(s0.h_out, d_out, (size_t)copy * sizeof(mtcp_gpu_addr_entry),
                                           hipMemcpyDeviceToHost, st)))
            rc = MTCP_GPU_EIO;
        rc = finish_call(ctx, rc, dl, 1);
        if (rc == MTCP_GPU_OK) {
            memcpy(out, s0.h_out, (size_t)copy * sizeof(mtcp_gpu_addr_entry));
            *n_found = kept;
        }
    }
    if (rc == MTCP_GPU_ETIMEDOUT) return rc;                 // abandoned: d_mem stays allocated
    if (rc != MTCP_GPU_OK) (void)finish_call(ctx, rc, dl, 1);
    if (!ctx->abandoned) mtcp_park::release(d_mem, bytes, mtcp_park::kDevice, !dl.bounded);
    return rc;
}

int mtcp_gpu_host_register(void *ptr, uint64_t len) {
    if (!ptr || !len) return MTCP_GPU_EINVAL;
    return HIP_OK(hipHostRegister(ptr, len, hipHostRegisterMapped)) ? MTCP_GPU_OK : MTCP_GPU_EIO;
}

int mtcp_gpu_host_unregister(void *ptr) {
    if (!ptr) return MTCP_GPU_EINVAL;
    return HIP_OK(hipHostUnregister(ptr)) ? MTCP_GPU_OK : MTCP_GPU_EIO;
}

}  // extern "C"
