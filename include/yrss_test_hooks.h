/* yrss_test_hooks.h — test-only entry points of libyrss_test.so.
 *
 * libyrss_test.so is the same sources as libyrss.so compiled with
 * -DYRSS_TEST_HOOKS (__graft_entry__.build()).  The shipping libyrss.so
 * exports none of these and contains none of the paths they drive
 * (tests/test_abi.py checks that).  The reference has no equivalent: these
 * exist to drive this engine's own fault guards from the GPU tests.
 */
#ifndef YRSS_TEST_HOOKS_H
#define YRSS_TEST_HOOKS_H

#include <stdint.h>

#include "yrss.h"

#ifdef __cplusplus
extern "C" {
#endif

/* The persistent worker's burst with this ticket fires a list guard
 * (YRSS_FAULT_LIST_RANGE, value 0xdead) at the next worker launch: the
 * per-burst fault path of yrss_worker_poll.  0 disables. */
int yrss_debug_worker_inject(yrss_ctx *ctx, uint64_t ticket);

/* Force the line scatter's instantiation: 2 or 4 yrss_scatter_lines<kG>
 * (8-packet groups a thread), 0 = the built-in choice (kG = 2 up to 128
 * buckets, 4 past that).  A pairing whose per-bucket arrays cannot
 * hold nb_queues + 1 buckets makes yrss_dispatch_dev return -EINVAL before
 * anything is launched; with skip_host_check = 1 it is launched anyway, and
 * the kernel's entry check must report YRSS_FAULT_LINE_CAPACITY and leave. */
int yrss_debug_line_groups(yrss_ctx *ctx, uint32_t groups, int skip_host_check);

/* 1: the partial list lines of a workgroup's range (its first and last line
 * of each bucket, the other part written by the neighbouring range) leave as
 * plain stores, so the two parts can meet in L2 and be written back once;
 * 0: streaming stores like every other line (results unchanged). */
int yrss_debug_partial_merge(yrss_ctx *ctx, int on);

#ifdef __cplusplus
}
#endif
#endif /* YRSS_TEST_HOOKS_H */
