// dispatch.hpp — which kernel a batch runs on (host logic only: plain C++,
// no HIP), shared by mtcp_gpu.hip and the CPU test of the rules
// (tests/c/dispatch_test.cpp, tests/test_dispatch_rules.py).  The kernels
// themselves are rx_kernels.hpp (rx_kernel, 64 packets per wave),
// rx_wave.hpp (a wave, a 16-lane row, 8 lanes or a 4-lane quad per packet)
// and rx_span.hpp (a workgroup's chunks back to back).
#pragma once

#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/mtcp_gpu.h"

namespace {

// Small batches (rx_wave.hpp).  rx_kernel gives a wave 64 packets, so a
// batch of n packets runs on n/64 waves and its phase 1 is a chain of round
// trips; the small-batch kernels put a wave (or a 16-lane row, or a 4-lane
// quad) on every packet.  The choice by batch size and average slot, from
// tools/wave_probe.hip and tools/small_batch_probe.py (same frames, same
// process):
//   slot < 256 B:   n <= 2 048  wave;  n <= 128 K a quad per packet (64 per workgroup)
//   slot >= 4 KiB:  n <= 64 K   wave (a jumbo frame in one trip; 4 KiB slots
//                   since round 4: 16 K / 32 K / 64 K frames 11.8 / 21.1 / 40.4 us
//                   against the row kernel's 16.1 / 27.6 and rx_kernel's 51.6,
//                   profiles/r4/dispatch_map.jsonl)
//   otherwise:      n <= 8 192  wave;  n <= 32 K  a row per packet (64 per workgroup)
//   larger batches: slot <= 64 B a quad per packet; slot <= 640 B rx_span_kernel
//                   (rx_span.hpp: the workgroup's chunks back to back, whatever
//                   the sizes); up to 64 K frames of <= 2 KiB slots 8 lanes per
//                   packet; above, rx_kernel (64 packets per wave)
// (since the select-form per-lane phase 2: 4 096 x 64 B quad 3.55 vs wave
// 3.86 us, 2 048 x 64 B 3.53 vs 3.21; 8 192 x 1500 B wave 6.05 vs row 7.32,
// 16 K 9.31 vs 7.35: profiles/r2/wave_probe_dispatch.jsonl; 128 K x 64 B quad 5.37
// vs rx_kernel 6.05 us through the Python ABI: profiles/r2/small_batch_sched.jsonl.
// Round 4, profiles/r4/group_span_probe.jsonl: quads in 256-thread workgroups
// beat the 1024-thread ones at every n (1 M x 64 B 24.9 vs 31.5 us, rx_kernel
// 32.3); on 1 M frames of 128 / 256 / 512 B rx_span_kernel takes 39.7 / 60.3 /
// 101.9 us where rx_kernel's rows take 122.6 / 126.5 / 136.1, and on an IMIX
// (64 / 576 / 1500 B, 7 : 4 : 1) 77.8 vs 86.1 us; from 768 B slots on
// rx_kernel is ahead again, 142.4 vs 146.4 us.)
// Pointer bursts carry no size the host can see: they count as mid-size.
// MTCP_GPU_SCHED=wave|row|quad|oct|span|big at context open forces one kernel for
// every batch (A/B runs, and the parity tests of each); the tx fill of
// pointer bursts and the tx report exist only in the small kernels, and the
// span kernel is rx only (a forced span runs tx on rx_kernel).
enum Sched : int { kSchedAuto = 0, kSchedWave, kSchedRow, kSchedQuad, kSchedBig, kSchedSpan, kSchedOct };

constexpr uint64_t kQuadOnlyUpToSlot = 64;
constexpr uint64_t kSpanUpToSlot = 640;
// 32 K < n <= 64 K frames of 640 B < slot <= 2 KiB: 8-lane groups.  rx_kernel
// fills half the GPU's wave slots at 64 K frames (1 024 waves of 64); through
// the ABI, same frames and process, records identical (profiles/r4/oct_sweep.jsonl):
// 64 K x 768 / 1024 / 1500 / 2048 B 8.8 / 11.8 / 17.3 / 21.3 us against
// 16.9 / 17.3 / 19.8 / 32.4 (bimodal equal, 14.3 vs 14.2; 4 KiB slots and
// 128 K frames of 1500 B keep rx_kernel).
constexpr uint32_t kOctUpToPkts = 1u << 16;
constexpr uint64_t kOctUpToSlot = 2048;

inline int sched_from_env() {
    const char *e = getenv("MTCP_GPU_SCHED");
    if (!e) return kSchedAuto;
    if (!strcmp(e, "wave")) return kSchedWave;
    if (!strcmp(e, "row")) return kSchedRow;
    if (!strcmp(e, "quad")) return kSchedQuad;
    if (!strcmp(e, "span")) return kSchedSpan;
    if (!strcmp(e, "oct")) return kSchedOct;
    if (!strcmp(e, "big")) return kSchedBig;
    return kSchedAuto;
}

// A batch known to be of one size class (mtcp_gpu_size_hint: every 64 B
// slot within 2x of the smallest) takes the kernels measured fastest on
// uniform batches where those differ from the choice for mixes of the same
// average slot (profiles/r4/dispatch_map_final.jsonl, same process, records
// identical): 64 K frames of 256 / 512 B 8 lanes per packet, 5.27 / 7.17 us
// against the span kernel's 6.16 / 8.75; 256 K / 1 M frames of 768 B the span
// kernel, 37.2 / 151.6 us against rx_kernel's sorted rounds 41.5 / 167.8
// (which a 64 / 1500 B mix of 800 B average slots needs: 141.7 against 183.1
// at 1 M); 1 M frames of 4 KiB the wave kernel, 620.6 against 655.4 us
// (256 K: rx_kernel 165.7 against 171.4; 9000 B frames stay on rx_kernel).
constexpr uint64_t kSpanNarrowUpToSlot = 896;
constexpr uint64_t kWaveNarrowUpToSlot = 4096;
constexpr uint32_t kWaveNarrowFromPkts = 1u << 20;

// Is the hinted batch of one size class: every slot within 2x of the
// smallest (a zero length is a NULL / empty entry and costs nothing)?
inline bool narrow_batch(const mtcp_gpu_size_hint *h) {
    if (!h || h->min_len == 0 || h->max_len < h->min_len) return false;
    const uint32_t lo = ((uint32_t)h->min_len + 63) & ~63u, hi = ((uint32_t)h->max_len + 63) & ~63u;
    return hi <= 2 * lo;
}

// forced: the context's MTCP_GPU_SCHED (kSchedAuto: choose); n: the batch's
// packets; slot: its average slot (buf_len / n; 1 KiB for pointer bursts);
// small_only: only the small kernels implement the launch (tx of pointer
// bursts, the tx report); rx: an rx launch (the span kernel exists for rx
// only); narrow: a hint says the batch is of one size class (narrow_batch)
inline int pick_sched(int forced, uint32_t n, uint64_t slot, bool small_only, bool rx, bool narrow = false) {
    int s = forced;
    if (s == kSchedAuto) {
        int big = slot <= kQuadOnlyUpToSlot ? kSchedQuad
                  : slot <= kSpanUpToSlot   ? kSchedSpan
                  : (n <= kOctUpToPkts && slot <= kOctUpToSlot) ? kSchedOct : kSchedBig;
        if (narrow && slot > kQuadOnlyUpToSlot && slot <= kSpanUpToSlot && n <= kOctUpToPkts)
            big = kSchedOct;
        else if (narrow && slot > kSpanUpToSlot && slot <= kSpanNarrowUpToSlot && n > kOctUpToPkts)
            big = kSchedSpan;
        if (slot < 256) {
            s = n <= 2048 ? kSchedWave : n <= (1u << 17) ? kSchedQuad : big;
        } else if (narrow && slot <= kSpanUpToSlot && n > 2048 && n <= kOctUpToPkts) {
            // one size class of 256-640 B slots: 8 lanes per packet from 4 K
            // frames on (4 K x 256 / 512 B 3.34 / 3.61 us against the wave
            // kernel's 3.96 / 3.98, 32 K x 256 B 4.20 against the row
            // kernel's 4.82; an IMIX of 4 K frames keeps the wave kernel,
            // 3.86 against 5.06: profiles/r5/dispatch_map.jsonl)
            s = kSchedOct;
        } else if (narrow && slot <= 320 && n > 2048 && n <= (1u << 17)) {
            // 128 K frames of 256 B: quads, 8.55 against the span kernel's 9.27 us
            // (a hinted batch of <= 2 048 frames keeps the wave kernel, as an
            // unhinted one: the map has no measured quad cell below 4 K frames)
            s = kSchedQuad;
        } else if (slot >= 4096) {
            s = n <= (1u << 16) || (narrow && slot <= kWaveNarrowUpToSlot && n >= kWaveNarrowFromPkts)
                    ? kSchedWave : kSchedBig;
        } else {
            // 16 K frames of 2 KiB slots: the wave kernel, 8.64 against the
            // row kernel's 9.09 us (1500 B frames keep the rows: 7.28 / 8.27)
            s = n <= 8192 || (slot >= 2048 && n <= 16384) ? kSchedWave
                : n <= (1u << 15)                          ? kSchedRow : big;
        }
    }
    if (s == kSchedSpan && !rx) s = kSchedBig;
    if (s == kSchedBig && small_only) s = kSchedRow;
    return s;
}

// The wave kernel's loads per lane per trip: two (2 KiB, an MTU frame in one
// trip) when the batch's average slot is at most 2 KiB, ten (10 KiB, a 9000 B
// frame in one trip) otherwise; a longer frame takes more trips either way.
// Pointer bursts count as 1 KiB slots: a DPDK mbuf's default data room is
// 2 KiB (RTE_MBUF_DEFAULT_DATAROOM), so their frames fit the short trip.
constexpr uint64_t kWaveShortUpToSlot = 2048;

// rx_kernel's phase-1 schedule (kSchedBig) by the chunk's average slot size:
// with mostly large frames (C2 1500 B, C5 9000 B) the 16 rounds unrolled and
// single-buffered (SCHED 3) stream best; with many small frames (C3: half
// 64 B) the size-sorted rounds win — large frames four per round,
// double-buffered, small ones sixteen per round (tools/rx_variants, in-process
// A/B, four boxes: C2 unrolled 240.9-243.1 / rolled 244.2-246.0 / sorted
// 248-250 us; C5 unrolled and rolled equal, 683-686 us; C3 rolled 164,
// unrolled 145, sorted 141 us).  The sorted schedule issues the first two
// small rounds together with the pre-issued first large round, through L2
// (SCHED 6): a 64 B frame shares its 128 B line with a neighbour's edge that
// another round streams, and the early temporal load lets that round hit it
// (C3 140.7 -> 134.3 us).  Frames longer than one trip (1536 B) are streamed
// from the start of their first 128 B line (rx_kernel LALIGN) so that no trip
// boundary splits a line: C5's 9024 B slots put every other frame off the
// line grid, and without it 2.4 % of the chunk is fetched twice (PMC
// FETCH_SIZE 4.887 -> 4.768 GB per launch; 688.6 vs 690.7 us).  Chunks of
// <= 1536 B slots skip the bookkeeping.
constexpr uint64_t kUnrollBelowSlotBytes = 1024;
constexpr uint64_t kLineAlignAboveSlotBytes = 1536;
// Small batches (one io_module aggregate is 4096 frames) give each wave one
// pass, so phase 1 is latency-bound: the sorted rounds, double-buffered, beat
// the single-buffered unrolled ones there also for MTU frames (tools/rx_variants
// RXV_N, 1500 B frames: 4096 -> 13.6 vs 15.0 us, 65536 -> 19.4 vs 22.4 us;
// 1 M -> 248 vs 243 us, so large batches keep the unrolled rounds).  Jumbo
// frames keep the unrolled, line-aligned rounds at every size.
constexpr uint32_t kSortedUpToPkts = 1u << 16;

enum BigSched : int { kBigSorted = 0, kBigUnrolled, kBigUnrolledLineAligned, kBigSortedLineAligned };

// ptrs: a pointer burst — no size the host can see (the lengths are in
// device memory): the size-sorted, line-aligned rounds are the robust choice
// (C3-shaped bursts 135.5 vs 162.1 us unrolled, C2-shaped 250.5 vs 245.3,
// C5-shaped 687.7 vs 685.2; tools/rx_variants ptrs_*).  The schedule is
// chosen once per batch (batch_n: the whole batch, not one launch's share).
inline int big_schedule(bool ptrs, uint64_t slot, uint32_t batch_n) {
    if (ptrs) return kBigSortedLineAligned;
    if (slot < kUnrollBelowSlotBytes || (batch_n <= kSortedUpToPkts && slot <= kLineAlignAboveSlotBytes))
        return kBigSorted;
    return slot > kLineAlignAboveSlotBytes ? kBigUnrolledLineAligned : kBigUnrolled;
}

// The name mtcp_gpu_last_kernel reports for a choice.
inline const char *kernel_name(int sched, int big, uint64_t slot) {
    switch (sched) {
        case kSchedWave: return slot <= kWaveShortUpToSlot ? "rx_wave_kernel<2 loads>" : "rx_wave_kernel<10 loads>";
        case kSchedQuad: return "rx_group_kernel<quad>";
        case kSchedOct: return "rx_group_kernel<oct>";
        case kSchedSpan: return "rx_span_kernel";
        case kSchedRow: return "rx_group_kernel<row>";
        default: break;
    }
    switch (big) {
        case kBigSorted: return "rx_kernel<sorted>";
        case kBigUnrolled: return "rx_kernel<unrolled>";
        case kBigUnrolledLineAligned: return "rx_kernel<unrolled,line-aligned>";
        default: return "rx_kernel<sorted,line-aligned>";
    }
}

}  // namespace
