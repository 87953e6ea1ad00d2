/* Test double: TCPCalcChecksum of mtcp/src/include/tcp_util.h:27 (defined by
 * the harness, tests/c/rxloop.c, over the oracle's restatement). */
#ifndef TEST_DOUBLE_TCP_UTIL_H
#define TEST_DOUBLE_TCP_UTIL_H
#include <stdint.h>
uint16_t TCPCalcChecksum(uint16_t *buf, uint16_t len, uint32_t saddr, uint32_t daddr);
#endif
