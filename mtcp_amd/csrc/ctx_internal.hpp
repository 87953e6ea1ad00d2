// ctx_internal.hpp — library-internal view of a context for rxq.hip (not
// part of the C ABI, not exported from libmtcp_gpu.so).
#pragma once

struct mtcp_gpu_ctx;

// The context gave up on GPU work at a deadline (mtcp_gpu_set_wait_limit):
// nothing may be issued on it or waited for without a bound again.
extern "C" __attribute__((visibility("hidden"))) bool mg_ctx_abandoned(const mtcp_gpu_ctx *ctx);
