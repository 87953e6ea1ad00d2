/*
 * ref_rss_mtcp.c — TEST INFRASTRUCTURE ONLY.  Compiles the reference's
 * mtcp/src/rss.c (6-argument GetRSSCPUCore with endian_check,
 * mtcp/src/rss.c:90-103) by #including it from /root/reference.
 */
#include <stdint.h>
#define GetRSSCPUCore ref_mtcp_GetRSSCPUCore_impl
#include REF_MTCP_RSS_C
#undef GetRSSCPUCore

int ref_mtcp_rss_core(uint32_t sip, uint32_t dip, uint16_t sp, uint16_t dp, int nq,
                      uint8_t endian_check)
{
    return ref_mtcp_GetRSSCPUCore_impl(sip, dip, sp, dp, nq, endian_check);
}
