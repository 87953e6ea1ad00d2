"""Which HIP free/unregister calls wait for OTHER streams' work on the
device?  For each call: queue a 300 ms mtcp_gpu_debug_stall on context A,
then time the call on memory A's work never touches.  ~0.3 s = the call
synchronises the device; ~0 = it does not.  One JSON line per call."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    assert torch.cuda.is_available()
    from mtcp_amd import gpu
    from mtcp_amd._lib import lib
    L = lib()
    T = ctypes.CDLL(os.path.join(ROOT, "tests", "c", "libmtcp_gpu_testing.so"))
    T.mtcp_gpu_debug_stall.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    H = ctypes.CDLL("libamdhip64.so")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    H.hipMalloc.argtypes = [ctypes.POINTER(vp), sz]
    H.hipFree.argtypes = [vp]
    H.hipHostMalloc.argtypes = [ctypes.POINTER(vp), sz, ctypes.c_uint]
    H.hipHostFree.argtypes = [vp]
    H.hipMallocAsync.argtypes = [ctypes.POINTER(vp), sz, vp]
    H.hipFreeAsync.argtypes = [vp, vp]
    H.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    H.hipStreamSynchronize.argtypes = [vp]
    H.hipStreamDestroy.argtypes = [vp]
    H.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
    H.hipHostUnregister.argtypes = [vp]
    H.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
    H.hipEventDestroy.argtypes = [vp]
    a = gpu.Context(0)
    s = vp()
    assert H.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0       # non-blocking
    n = 8 << 20

    def timed(name, prep, call):
        obj = prep()
        assert L.mtcp_gpu_sync(a._h) == 0
        assert T.mtcp_gpu_debug_stall(a._h, 300_000) == 0
        time.sleep(0.01)
        t0 = time.monotonic()
        rc = call(obj)
        dt = time.monotonic() - t0
        assert L.mtcp_gpu_sync(a._h) == 0
        print(json.dumps({"call": name, "rc": rc, "s": round(dt, 4)}), flush=True)

    def dmalloc():
        p = vp(); assert H.hipMalloc(ctypes.byref(p), n) == 0; return p

    def hmalloc():
        p = vp(); assert H.hipHostMalloc(ctypes.byref(p), n, 0) == 0; return p

    def amalloc():
        p = vp(); assert H.hipMallocAsync(ctypes.byref(p), n, s) == 0
        assert H.hipStreamSynchronize(s) == 0; return p

    keep = []

    def registered():
        b = ctypes.create_string_buffer(n); keep.append(b)
        assert H.hipHostRegister(ctypes.cast(b, vp), n, 0) == 0; return ctypes.cast(b, vp)

    def stream():
        t = vp(); assert H.hipStreamCreateWithFlags(ctypes.byref(t), 1) == 0; return t

    def event():
        e = vp(); assert H.hipEventCreateWithFlags(ctypes.byref(e), 2) == 0; return e

    timed("hipFree", dmalloc, lambda p: H.hipFree(p))
    timed("hipHostFree", hmalloc, lambda p: H.hipHostFree(p))
    timed("hipFreeAsync(hipMalloc)", dmalloc, lambda p: H.hipFreeAsync(p, s))
    timed("hipFreeAsync(hipMallocAsync)", amalloc, lambda p: H.hipFreeAsync(p, s))
    timed("hipFreeAsync(hipMallocAsync)+own stream sync", amalloc,
          lambda p: H.hipFreeAsync(p, s) or H.hipStreamSynchronize(s))
    timed("hipHostUnregister", registered, lambda p: H.hipHostUnregister(p))
    timed("hipStreamDestroy", stream, lambda t: H.hipStreamDestroy(t))
    timed("hipEventDestroy", event, lambda e: H.hipEventDestroy(e))
    H.hipMemcpy.argtypes = [vp, vp, sz, ctypes.c_int]
    H.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    H.hipGetDeviceProperties = getattr(H, "hipGetDevicePropertiesR0600", H.hipGetDeviceProperties)
    H.hipGetDeviceProperties.argtypes = [vp, ctypes.c_int]
    small = ctypes.create_string_buffer(4096)
    timed("hipStreamCreateWithFlags", lambda: None, lambda _: H.hipStreamCreateWithFlags(ctypes.byref(vp()), 1))
    timed("hipEventCreateWithFlags", lambda: None, lambda _: H.hipEventCreateWithFlags(ctypes.byref(vp()), 2))
    timed("hipGetDeviceProperties", lambda: None,
          lambda _: H.hipGetDeviceProperties(ctypes.cast(ctypes.create_string_buffer(8192), vp), 0))
    timed("hipMemcpy H2D 4 KiB pageable (null stream)", dmalloc,
          lambda p: H.hipMemcpy(p, ctypes.cast(small, vp), 4096, 1))
    timed("hipMemcpyAsync H2D 4 KiB + own stream sync", dmalloc,
          lambda p: H.hipMemcpyAsync(p, ctypes.cast(small, vp), 4096, 1, s) or H.hipStreamSynchronize(s))
    from mtcp_amd import gpu as _g
    timed("mtcp_gpu_open", lambda: None, lambda _: _g.Context(0) and 0)
    def ctx_prep():
        return _g.Context(0)
    timed("mtcp_gpu_reserve(1 MiB, 1024)", ctx_prep, lambda c: c.reserve(1 << 20, 1024) or 0)
    def rxq_make(c):
        q = vp()
        return L.mtcp_gpu_rxq_create(ctypes.byref(q), c._h, 256, 256 * 2048)
    timed("mtcp_gpu_rxq_create(256, 512 KiB)", ctx_prep, rxq_make)
    timed("hipMalloc", lambda: None, lambda _: H.hipMalloc(ctypes.byref(vp()), n))
    timed("hipHostMalloc", lambda: None, lambda _: H.hipHostMalloc(ctypes.byref(vp()), n, 0))
    a.close()


if __name__ == "__main__":
    main()
