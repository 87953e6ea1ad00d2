/*
 * Test double (not the reference's header): the two fields of
 * struct mtcp_thread_context (mtcp/src/include/mtcp.h:274-284) that
 * mtcp_amd/io_module/gpu_module.c touches, so the module can be unit-tested
 * on a box without the mTCP tree.  The real build compiles gpu_module.c
 * against mTCP's own headers (tests/test_io_module.py checks that too).
 */
#ifndef TEST_DOUBLE_MTCP_H
#define TEST_DOUBLE_MTCP_H
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

struct mtcp_thread_context {
    int cpu;
    void *io_private_context;
};
#endif
