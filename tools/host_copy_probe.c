// host_copy_probe.c — the io_module staging copy (rxq.hip stage_copy) on one
// core: 1 M x 1500 B frames from a 1.6 GB source into an 8 MiB staging ring,
// with 16 / 32 / 64 B streaming stores and memcpy, beside a read-only pass
// over the same frames (the reference check reads each byte once).
//   gcc -O2 -o tools/host_copy_probe tools/host_copy_probe.c
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
static double now(void){struct timespec t;clock_gettime(CLOCK_MONOTONIC,&t);return t.tv_sec+t.tv_nsec*1e-9;}
static void cp_sse(uint8_t *d,const uint8_t *s,uint32_t n){uint32_t i=0;for(;i+64<=n;i+=64){__m128i a=_mm_loadu_si128((const __m128i*)(s+i)),b=_mm_loadu_si128((const __m128i*)(s+i+16)),c=_mm_loadu_si128((const __m128i*)(s+i+32)),e=_mm_loadu_si128((const __m128i*)(s+i+48));_mm_stream_si128((__m128i*)(d+i),a);_mm_stream_si128((__m128i*)(d+i+16),b);_mm_stream_si128((__m128i*)(d+i+32),c);_mm_stream_si128((__m128i*)(d+i+48),e);}for(;i<n;i+=16)_mm_stream_si128((__m128i*)(d+i),_mm_loadu_si128((const __m128i*)(s+i)));}
__attribute__((target("avx2"))) static void cp_avx2(uint8_t *d,const uint8_t *s,uint32_t n){uint32_t i=0;for(;i+128<=n;i+=128){__m256i a=_mm256_loadu_si256((const __m256i*)(s+i)),b=_mm256_loadu_si256((const __m256i*)(s+i+32)),c=_mm256_loadu_si256((const __m256i*)(s+i+64)),e=_mm256_loadu_si256((const __m256i*)(s+i+96));_mm256_stream_si256((__m256i*)(d+i),a);_mm256_stream_si256((__m256i*)(d+i+32),b);_mm256_stream_si256((__m256i*)(d+i+64),c);_mm256_stream_si256((__m256i*)(d+i+96),e);}for(;i<n;i+=16)_mm_stream_si128((__m128i*)(d+i),_mm_loadu_si128((const __m128i*)(s+i)));}
__attribute__((target("avx512f"))) static void cp_avx512(uint8_t *d,const uint8_t *s,uint32_t n){uint32_t i=0;for(;i+256<=n;i+=256){__m512i a=_mm512_loadu_si512(s+i),b=_mm512_loadu_si512(s+i+64),c=_mm512_loadu_si512(s+i+128),e=_mm512_loadu_si512(s+i+192);_mm512_stream_si512((void*)(d+i),a);_mm512_stream_si512((void*)(d+i+64),b);_mm512_stream_si512((void*)(d+i+128),c);_mm512_stream_si512((void*)(d+i+192),e);}for(;i+64<=n;i+=64)_mm512_stream_si512((void*)(d+i),_mm512_loadu_si512(s+i));for(;i<n;i+=16)_mm_stream_si128((__m128i*)(d+i),_mm_loadu_si128((const __m128i*)(s+i)));}
static void cp_mem(uint8_t *d,const uint8_t *s,uint32_t n){memcpy(d,s,n);}
static uint64_t rd(const uint8_t *s,uint32_t n){uint64_t a=0;for(uint32_t i=0;i<n;i+=8)a+=*(const uint64_t*)(s+i);return a;}
int main(int argc,char**argv){
  const uint32_t N=1u<<20, L=1500, SLOT=1536; const uint64_t src_bytes=(uint64_t)N*SLOT;
  const uint64_t ring=8u<<20;
  uint8_t *src=aligned_alloc(64,src_bytes), *dst=aligned_alloc(64,ring);
  memset(src,1,src_bytes); memset(dst,0,ring);
  const char *names[]={"sse2_nt","avx2_nt","avx512_nt","memcpy"};
  void (*fns[])(uint8_t*,const uint8_t*,uint32_t)={cp_sse,cp_avx2,cp_avx512,cp_mem};
  int have512=__builtin_cpu_supports("avx512f");
  for(int r=0;r<3;r++){
   for(int f=0;f<4;f++){ if(f==2&&!have512)continue;
    double t0=now(); uint64_t o=0;
    for(uint32_t i=0;i<N;i++){ if(o+SLOT>ring)o=0; fns[f](dst+o,src+(uint64_t)i*SLOT,L); o+=SLOT; }
    _mm_sfence(); double t=now()-t0;
    printf("{\"copy\":\"%s\",\"round\":%d,\"GBs\":%.1f,\"Mpkts\":%.1f}\n",names[f],r,(double)N*L/t/1e9,N/t/1e6);
   }
   double t0=now(); uint64_t a=0; for(uint32_t i=0;i<N;i++) a+=rd(src+(uint64_t)i*SLOT,L); double t=now()-t0;
   printf("{\"copy\":\"read_only\",\"round\":%d,\"GBs\":%.1f,\"Mpkts\":%.1f,\"x\":%llu}\n",r,(double)N*L/t/1e9,N/t/1e6,(unsigned long long)(a&1));
  }
  return 0;}
