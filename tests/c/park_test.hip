// park_test.hip — TEST HARNESS for mtcp_amd/csrc/park.hpp on the GPU box
// (tests/test_gpu_bounded.py::test_park_best_fit): parked buffers are handed
// to the smallest request they cover up to twice over, a buffer handed out
// larger than asked goes back with its real size, and the per-device cap
// frees instead of parking.  Prints one JSON line.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../../mtcp_amd/csrc/park.hpp"

using mtcp_park::alloc;
using mtcp_park::kDevice;
using mtcp_park::kHost;
using mtcp_park::release;

static size_t parked(int dev, mtcp_park::Kind k) { return mtcp_park::pool().parked[dev][k]; }

int main() {
    if (hipSetDevice(0) != hipSuccess) return 2;
    const size_t MiB = 1u << 20;
    void *a = nullptr, *b = nullptr, *c = nullptr, *d = nullptr, *e = nullptr;
    int ok = 1;
    // a 1 MiB device buffer parked, then a 700 KiB request: the same buffer
    ok &= alloc(&a, MiB, kDevice) == hipSuccess;
    release(a, MiB, kDevice);
    const size_t p0 = parked(0, kDevice);
    ok &= alloc(&b, 700 * 1024, kDevice) == hipSuccess;
    const int best_fit_reused = b == a;
    const size_t p1 = parked(0, kDevice);
    // a 400 KiB request: the 1 MiB buffer is more than twice that -> new
    ok &= alloc(&c, 400 * 1024, kDevice) == hipSuccess;
    const int small_not_reused = c != a && c != nullptr;
    // b goes back with its real size (1 MiB): a 1 MiB request gets it again
    release(b, 700 * 1024, kDevice);
    const size_t p2 = parked(0, kDevice);
    ok &= alloc(&d, MiB, kDevice) == hipSuccess;
    const int real_size_kept = d == a;
    release(d, MiB, kDevice);
    release(c, 400 * 1024, kDevice);
    // the smallest covering buffer wins: parked 1 MiB and 400 KiB, ask 390 KiB
    ok &= alloc(&e, 390 * 1024, kDevice) == hipSuccess;
    const int smallest_wins = e == c;
    release(e, 390 * 1024, kDevice);
    // pinned host memory is parked apart from device memory
    void *h = nullptr, *h2 = nullptr;
    ok &= alloc(&h, MiB, kHost) == hipSuccess;
    release(h, MiB, kHost);
    ok &= alloc(&h2, MiB, kDevice) == hipSuccess;
    const int kinds_apart = h2 != h;
    release(h2, MiB, kDevice);
    // the cap: buffers above kParkMaxBytes are freed, not parked
    void *big = nullptr;
    const size_t before_big = parked(0, kDevice);
    ok &= alloc(&big, mtcp_park::kParkMaxBytes + MiB, kDevice) == hipSuccess;
    release(big, mtcp_park::kParkMaxBytes + MiB, kDevice);
    const int big_freed = parked(0, kDevice) == before_big;
    // ... unless the release must not wait (a bounded call): parked anyway,
    // and the next request of that size gets it back
    void *big2 = nullptr, *big3 = nullptr;
    const size_t bigsz = mtcp_park::kParkMaxBytes + MiB;
    ok &= alloc(&big2, bigsz, kDevice) == hipSuccess;
    release(big2, bigsz, kDevice, /*may_free=*/false);
    const int big_parked_when_bounded = parked(0, kDevice) == before_big + bigsz;
    ok &= alloc(&big3, bigsz, kDevice) == hipSuccess;
    const int big_reused = big3 == big2;
    release(big3, bigsz, kDevice);
    printf("{\"ok\": %d, \"best_fit_reused\": %d, \"small_not_reused\": %d, \"real_size_kept\": %d, "
           "\"smallest_wins\": %d, \"kinds_apart\": %d, \"big_freed\": %d, \"big_parked_when_bounded\": %d, "
           "\"big_reused\": %d, \"parked_after_release\": %zu, "
           "\"parked_after_reuse\": %zu, \"parked_after_lent_release\": %zu}\n",
           ok, best_fit_reused, small_not_reused, real_size_kept, smallest_wins, kinds_apart, big_freed,
           big_parked_when_bounded, big_reused, p0, p1, p2);
    return 0;
}
