// host_copy.hpp — host-side frame copies into pinned staging (rxq.hip,
// mtcp_gpu.hip's pointer gather).  Host code only.
#pragma once

#include <emmintrin.h>
#include <stdint.h>
#include <string.h>

// Copy a frame into its 64 B-aligned staging slot with streaming stores:
// the slot is read next by the DMA engine, not by this core, so the stores
// skip the read-for-ownership of a normal memcpy.  The slot's tail up to the
// next 16 B is written too (it belongs to the slot's padding).
static inline void stage_copy(uint8_t *dst, const uint8_t *src, uint32_t len) {
    uint32_t i = 0;
    for (; i + 64 <= len; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 48), d);
    }
    for (; i + 16 <= len; i += 16)
        _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i),
                         _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + i)));
    if (i < len) {                        // last partial 16 B: through a bounce buffer
        alignas(16) uint8_t t[16] = {0};
        memcpy(t, src + i, len - i);
        _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), _mm_load_si128(reinterpret_cast<const __m128i *>(t)));
    }
}

// Make the streaming stores of stage_copy visible before a DMA reads them.
static inline void stage_fence() { _mm_sfence(); }
