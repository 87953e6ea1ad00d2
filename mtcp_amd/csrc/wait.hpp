// wait.hpp — the library's waits on the GPU, bounded or not.  Host-side C++.
//
// A context's wait limit (mtcp_gpu_set_wait_limit) bounds every wait of a
// synchronous call: the call computes one deadline when it starts, and each
// of its waits polls the device (hipStreamQuery / hipEventQuery, neither of
// which blocks) until that deadline instead of blocking in
// hipStreamSynchronize.  mTCP's own loop never waits on a device
// (mtcp/src/core.c:763-777); a device without the offload answers dev_ioctl
// with -1 (dpdk_module.c:809-816), which is where a caller goes when a wait
// here gives up.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <chrono>
#include <thread>

#include "../../include/mtcp_gpu.h"

namespace mtcp_wait {

struct Deadline {
    bool bounded = false;
    std::chrono::steady_clock::time_point end{};
    explicit Deadline(uint32_t timeout_us)
        : bounded(timeout_us != 0),
          end(std::chrono::steady_clock::now() + std::chrono::microseconds(timeout_us)) {}
    bool passed() const { return bounded && std::chrono::steady_clock::now() >= end; }
};

// Poll until query() is no longer hipErrorNotReady or the deadline passes:
// MTCP_GPU_OK, MTCP_GPU_EIO (the runtime reported an error) or
// MTCP_GPU_ETIMEDOUT.  The first few polls spin (a batch of frames finishes
// in microseconds); later ones yield the core.
template <typename Q>
inline int poll(Q query, const Deadline &dl) {
    for (uint32_t i = 0;; ++i) {
        const hipError_t e = query();
        if (e == hipSuccess) return MTCP_GPU_OK;
        if (e != hipErrorNotReady) return MTCP_GPU_EIO;
        if (dl.passed()) return MTCP_GPU_ETIMEDOUT;
        if (i >= 64) std::this_thread::yield();
    }
}

// Everything queued on `st` so far has finished.  Unbounded: one
// hipStreamSynchronize.  Bounded: hipStreamQuery until the deadline.
inline int drain(hipStream_t st, const Deadline &dl) {
    if (!dl.bounded) return hipStreamSynchronize(st) == hipSuccess ? MTCP_GPU_OK : MTCP_GPU_EIO;
    return poll([st] { return hipStreamQuery(st); }, dl);
}

// The work recorded by `evt` has finished (later work on its stream need not).
inline int wait_event(hipEvent_t evt, const Deadline &dl) {
    if (!dl.bounded) return hipEventSynchronize(evt) == hipSuccess ? MTCP_GPU_OK : MTCP_GPU_EIO;
    return poll([evt] { return hipEventQuery(evt); }, dl);
}

}  // namespace mtcp_wait
