/* Test double: TRACE_ERROR / TRACE_CONFIG of mtcp/src/include/debug.h. */
#ifndef TEST_DOUBLE_DEBUG_H
#define TEST_DOUBLE_DEBUG_H
#include <stdio.h>
#define TRACE_ERROR(f, ...) fprintf(stderr, "[gpu_module] " f, ##__VA_ARGS__)
#define TRACE_CONFIG(f, ...) fprintf(stderr, f, ##__VA_ARGS__)
#endif
