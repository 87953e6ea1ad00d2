// gpu_testing.hip — TEST-ONLY library (tests/c/libmtcp_gpu_testing.so): the
// fault injection the hang tests use (tests/c/mtcp_gpu_testing.h), built on
// the product's public ABI only (mtcp_gpu_stream), so that the product
// library exports no debug entry point.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mtcp_gpu.h"
#include "mtcp_gpu_testing.h"

namespace {
// one wave that returns `ticks` of the 100 MHz s_memrealtime clock after it
// started (it reads the clock, writes nothing)
__global__ __launch_bounds__(64) void stall_kernel(uint64_t ticks) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
}  // namespace

namespace {
int stall_on(hipStream_t st, uint32_t us) {
    if (!st || us > 10u * 1000 * 1000) return MTCP_GPU_EINVAL;
    hipDevice_t dev = 0;
    int prev = -1;
    if (hipStreamGetDevice(st, &dev) != hipSuccess || hipGetDevice(&prev) != hipSuccess) return MTCP_GPU_ENODEV;
    if (prev != dev && hipSetDevice(dev) != hipSuccess) return MTCP_GPU_ENODEV;
    hipLaunchKernelGGL(stall_kernel, dim3(1), dim3(64), 0, st, (uint64_t)us * 100);
    const bool ok = hipGetLastError() == hipSuccess;
    if (prev != dev) (void)hipSetDevice(prev);
    return ok ? MTCP_GPU_OK : MTCP_GPU_EIO;
}
}  // namespace

extern "C" int mtcp_gpu_debug_stall(mtcp_gpu_ctx *ctx, uint32_t us) {
    if (!ctx) return MTCP_GPU_EINVAL;
    return stall_on(reinterpret_cast<hipStream_t>(mtcp_gpu_stream(ctx)), us);
}

extern "C" int mtcp_gpu_debug_stall_stream(void *stream, uint32_t us) {
    return stall_on(reinterpret_cast<hipStream_t>(stream), us);
}
