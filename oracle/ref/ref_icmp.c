/*
 * ref_icmp.c — TEST INFRASTRUCTURE ONLY.  Compiles the reference's
 * mtcp/src/icmp.c by #including it from /root/reference so that its static
 * ICMPChecksum (icmp.c:18-42) is reachable; the file's other functions are
 * renamed out of the way.
 */
#include <stdint.h>
#define ProcessICMPPacket ref_icmp_ProcessICMPPacket_unused
#define RequestICMP ref_icmp_RequestICMP_unused
#define DumpICMPPacket ref_icmp_DumpICMPPacket_unused
#include REF_ICMP_C
#undef ProcessICMPPacket
#undef RequestICMP
#undef DumpICMPPacket

uint16_t ref_icmp_checksum(const uint8_t *icmph, int len)
{
    return ICMPChecksum((uint16_t *)icmph, len);
}
