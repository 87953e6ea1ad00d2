/*
 * ref_rss_util.c — TEST INFRASTRUCTURE ONLY.  Compiles the reference's
 * util/rss.c as shipped (key 0x05 x 40, util/rss.c:84-90) by #including it
 * from /root/reference (path given by the Makefile), so that its static
 * GetRSSHash (util/rss.c:107-145) is reachable.  Nothing is copied.
 */
#include <stdint.h>
#include <string.h>
#define GetRSSCPUCore ref_util_GetRSSCPUCore_impl
#include REF_UTIL_RSS_C
#undef GetRSSCPUCore

uint32_t ref_util_rss_hash(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp)
{
    return GetRSSHash(sip, dip, sp, dp);
}

int ref_util_rss_core(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp, int nq)
{
    return ref_util_GetRSSCPUCore_impl(sip, dip, sp, dp, nq);
}

uint32_t ref_rss_hash_pkt(const unsigned char *pkt)
{
    uint32_t s, d;
    uint16_t sp, dp;
    unsigned t = 14 + 4 * (pkt[14] & 0x0F);
    memcpy(&s, pkt + 26, 4);
    memcpy(&d, pkt + 30, 4);
    memcpy(&sp, pkt + t, 2);
    memcpy(&dp, pkt + t + 2, 2);
    return GetRSSHash(__builtin_bswap32(s), __builtin_bswap32(d),
                      (uint16_t)((sp >> 8) | (sp << 8)), (uint16_t)((dp >> 8) | (dp << 8)));
}
