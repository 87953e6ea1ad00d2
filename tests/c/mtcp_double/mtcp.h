/*
 * Test double (not the reference's header): the two fields of
 * struct mtcp_thread_context (mtcp/src/include/mtcp.h:274-284) and the two
 * of CONFIG that mtcp_amd/io_module/gpu_module.c touches, so the module can be unit-tested
 * on a box without the mTCP tree.  The real build compiles gpu_module.c
 * against mTCP's own headers (tests/test_io_module.py checks that too).
 */
#ifndef TEST_DOUBLE_MTCP_H
#define TEST_DOUBLE_MTCP_H
#include <arpa/inet.h>
#include <netinet/ip.h>
#include <linux/tcp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

/* ip_fast_csum of io_engine/include/ps.h:66-95, which mtcp.h includes
 * (defined by the harness, tests/c/rxloop.c, over the oracle's restatement) */
uint16_t ip_fast_csum(const void *iph, unsigned int ihl);

/* the fields of struct mtcp_config (mtcp.h:136-176) gpu_module.c reads:
 * eths_num (mtcp.h:138) and num_cores (mtcp.h:147) */
struct mtcp_config {
    int eths_num;
    int num_cores;
};
extern struct mtcp_config CONFIG;

struct mtcp_thread_context {
    int cpu;
    void *io_private_context;
};
#endif
