/*
 * ref_stubs.c — TEST INFRASTRUCTURE ONLY (oracle/_ref build, this container).
 *
 * The reference's rx objects (eth_in.o, ip_in.o, tcp_in.o, tcp_util.o,
 * compiled from /root/reference by oracle/Makefile) refer to the stateful
 * rest of mTCP.  None of these is reached by the checksum/parse head of the
 * rx chain: ref_glue.c stops every packet at StreamHTSearch
 * (tcp_in.c:1186).  Each stub aborts, so reaching one would be loud.
 * Deliberately compiled without the reference headers (names only).
 */
#include <stdlib.h>

#define STUB(name) void name(void) { abort(); }
STUB(AddEpollEvent)
STUB(AddtoControlList)
STUB(AddtoSendList)
STUB(AddtoTimeoutList)
STUB(AddtoTimewaitList)
STUB(CreateTCPStream)
STUB(DestroyTCPStream)
STUB(EnqueueACK)
STUB(IPOutputStandalone)
STUB(ListenerHTSearch)
STUB(RBInit)
STUB(RBPut)
STUB(RBRemove)
STUB(RaiseCloseEvent)
STUB(RaiseErrorEvent)
STUB(RaiseReadEvent)
STUB(RaiseWriteEvent)
STUB(RemoveFromRTOList)
STUB(RemoveFromSendList)
STUB(RemoveFromTimewaitList)
STUB(SBRemove)
STUB(SendTCPPacketStandalone)
STUB(StreamEnqueue)
STUB(UpdateRetransmissionTimer)
STUB(UpdateTimeoutList)
