/*
 * mtcp_gpu_testing.h — TEST-ONLY entry points (tests/c/libmtcp_gpu_testing.so),
 * kept out of the product library libmtcp_gpu.so and its public headers.
 * The test builds of gpu_module.c (-DMTCP_GPU_TESTING: rxloop, the drop-in
 * harnesses) and tests/test_gpu_rxq.py use them.
 */
#ifndef MTCP_GPU_TESTING_H
#define MTCP_GPU_TESTING_H

#include <stdint.h>

#include "mtcp_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fault injection for tests of a caller's hang handling: queue a kernel on
 * the context's stream (mtcp_gpu_stream: its host calls, tx fills and rxqs
 * all run there) that keeps it busy for `us` microseconds (at most 10 s), so
 * that work queued behind it completes that much later.  MTCP_GPU_EINVAL for
 * a NULL context or a longer stall. */
int mtcp_gpu_debug_stall(mtcp_gpu_ctx *ctx, uint32_t us);

/* The same on any stream of the caller's (a hipStream_t, as void*; not
 * NULL): the close test stalls a caller stream with a launch queued behind. */
int mtcp_gpu_debug_stall_stream(void *stream, uint32_t us);

#ifdef __cplusplus
}
#endif
#endif
