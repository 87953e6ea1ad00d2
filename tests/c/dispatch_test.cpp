// dispatch_test.cpp — the kernel choice of mtcp_amd/csrc/dispatch.hpp on the
// CPU (no GPU, no HIP): reads "n slot min_len max_len rx small_only forced
// ptrs" lines on stdin (min_len = max_len = 0: no size hint) and prints, for
// each, the kernel name mtcp_gpu_last_kernel would report.
// Built and driven by tests/test_dispatch_rules.py.
#include <stdio.h>

#include "../../mtcp_amd/csrc/dispatch.hpp"

int main() {
    unsigned long long n, slot;
    unsigned mn, mx;
    int rx, small_only, forced, ptrs;
    while (scanf("%llu %llu %u %u %d %d %d %d", &n, &slot, &mn, &mx, &rx, &small_only, &forced, &ptrs) == 8) {
        const mtcp_gpu_size_hint h = {(uint16_t)mn, (uint16_t)mx};
        const bool hinted = mn || mx;
        const int s = pick_sched(forced, (uint32_t)n, slot, small_only != 0, rx != 0,
                                 !ptrs && hinted && narrow_batch(&h));
        printf("%s\n", kernel_name(s, big_schedule(ptrs != 0, slot, (uint32_t)n), slot));
    }
    return 0;
}
