/*
 * tx_stubs.c — TEST INFRASTRUCTURE ONLY (oracle/_ref build, this container).
 *
 * The reference's tcp_out.o (compiled from /root/reference by oracle/Makefile)
 * names these for its stateful sender (SendTCPPacket, the RTO list); the
 * standalone builder dropin_tx.c drives (SendTCPPacketStandalone,
 * tcp_out.c:135-218) never reaches them.  Each aborts, so reaching one would
 * be loud.  Compiled without the reference headers (names only), as
 * ref_stubs.c (which cannot be linked here: it stubs the tx builders
 * themselves).
 */
#include <stdlib.h>

#define STUB(name) void name(void) { abort(); }
STUB(AddtoRTOList)
STUB(TCPStateToString)
STUB(DestroyTCPStream)
STUB(UpdateTimeoutList)
