// park.hpp — the library's pinned host and device buffers are parked when
// released, not freed, and handed out again to the next allocation of the
// same size on the same device.  Host-side C++ only.
//
// Why: hipFree, hipHostFree and hipHostUnregister wait for the work of every
// stream on the device, not only the caller's (tools/free_sync_probe.py on
// the MI355X: each took the 0.29 s of a stall another context had queued;
// hipMalloc / hipHostMalloc / hipStreamDestroy / hipEventDestroy did not
// wait).  One mTCP thread's shutdown (mtcp_gpu_rxq_destroy, mtcp_gpu_close)
// or its software fallback (gpu_module.c gpu_fail) would then wait for the
// other threads' GPU work on the same device — without limit if their GPU
// stopped answering, which is the case the io_module's bounded waits exist
// for.  Parking keeps every release free of device-wide waits; the io
// module's buffers are the same sizes on every thread, so a parked buffer is
// the next thread's (or the next context's) buffer.
//
// Bounds: buffers above kParkMaxBytes (a bench-sized reserve) are freed as
// before, and at most kParkDeviceBytes of each kind (pinned host, device)
// are parked per device (past that a release frees) — except for a release
// that must not wait (a call bounded by a context wait limit), which parks
// whatever the size.  A parked buffer is
// handed to the smallest request it covers up to twice over (best fit), so
// that a process whose sizes vary (a sweep of rxq sizes, the tests) reuses
// what it parked instead of filling the park with sizes that never match
// again.  The caller has made the buffer's device current and has finished
// its own work on the buffer (its streams are synchronised).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include <mutex>
#include <vector>

namespace mtcp_park {

constexpr size_t kParkMaxBytes = 80ull << 20;       // a 64 MiB pipeline stage and its rounding
constexpr size_t kParkDeviceBytes = 1ull << 30;
constexpr int kParkDevices = 64;

enum Kind { kDevice = 0, kHost = 1 };

struct Parked {
    int device;
    Kind kind;
    size_t bytes;
    void *p;
};

struct Pool {
    std::mutex m;
    std::vector<Parked> bufs;        // parked
    std::vector<Parked> lent;        // handed out larger than asked: their real size
    size_t parked[kParkDevices][2] = {};
};

// never destroyed: a release from an atexit handler or a late thread finds it
inline Pool &pool() {
    static Pool *p = new Pool;
    return *p;
}

inline int current_device() {
    int d = -1;
    return hipGetDevice(&d) == hipSuccess ? d : -1;
}

// hipMalloc / hipHostMalloc(hipHostMallocDefault) of `bytes`, or the
// smallest parked buffer of `bytes` to 2 x `bytes` on the current device
inline hipError_t alloc(void **out, size_t bytes, Kind kind) {
    *out = nullptr;
    const int dev = current_device();
    if (dev >= 0 && dev < kParkDevices) {
        Pool &pl = pool();
        std::lock_guard<std::mutex> lk(pl.m);
        size_t best = pl.bufs.size();
        for (size_t i = 0; i < pl.bufs.size(); ++i) {
            const Parked &b = pl.bufs[i];
            if (b.device == dev && b.kind == kind && b.bytes >= bytes && b.bytes / 2 <= bytes &&
                (best == pl.bufs.size() || b.bytes < pl.bufs[best].bytes))
                best = i;
        }
        if (best < pl.bufs.size()) {
            const Parked b = pl.bufs[best];
            *out = b.p;
            pl.parked[dev][kind] -= b.bytes;
            pl.bufs[best] = pl.bufs.back();
            pl.bufs.pop_back();
            if (b.bytes != bytes) pl.lent.push_back(b);
            return hipSuccess;
        }
    }
    return kind == kHost ? hipHostMalloc(out, bytes, hipHostMallocDefault) : hipMalloc(out, bytes);
}

template <typename T>
inline hipError_t alloc(T **out, size_t bytes, Kind kind) {
    void *p = nullptr;
    const hipError_t e = alloc(&p, bytes, kind);
    *out = static_cast<T *>(p);
    return e;
}

// give back a buffer alloc() returned (with the size it was asked for).
// may_free = false: the caller must not wait on the device (a call bounded
// by a context wait limit), so the buffer is parked whatever its size and
// the caps — a free here would wait for every stream on the device.
inline void release(void *p, size_t bytes, Kind kind, bool may_free = true) {
    if (!p) return;
    const int dev = current_device();
    Pool &pl = pool();
    {
        std::lock_guard<std::mutex> lk(pl.m);
        for (size_t i = 0; i < pl.lent.size(); ++i)
            if (pl.lent[i].p == p) {
                bytes = pl.lent[i].bytes;            // the buffer's real size
                pl.lent[i] = pl.lent.back();
                pl.lent.pop_back();
                break;
            }
        if (dev >= 0 && dev < kParkDevices &&
            (!may_free || (bytes <= kParkMaxBytes && pl.parked[dev][kind] + bytes <= kParkDeviceBytes))) {
            pl.bufs.push_back({dev, kind, bytes, p});
            pl.parked[dev][kind] += bytes;
            return;
        }
    }
    if (kind == kHost)
        (void)hipHostFree(p);
    else
        (void)hipFree(p);
}

}  // namespace mtcp_park
