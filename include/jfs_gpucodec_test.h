/*
 * jfs_gpucodec_test.h -- test hooks exported by libjfsgpu.so for its own test
 * suite (tests/test_capi.py).  NOT part of the drop-in ABI of jfs_gpucodec.h:
 * the Go adapter never binds these.
 */
#ifndef JFS_GPUCODEC_TEST_H
#define JFS_GPUCODEC_TEST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Host only, no GPU: runs the coalescer's burst-spreading lane acquisition
 * (own lane blocking, other devices' lanes try-locked) on ndev fake devices,
 * NLANE concurrent workers each, iters bursts per worker.  Returns the number
 * of bursts that took at least one foreign lane, or -1 if the workers did not
 * finish within timeout_ms (a deadlock: the stuck workers and their fake
 * devices are then left behind for the rest of the process), -2 on bad
 * arguments. */
int64_t jfs_test_spread_locking(int ndev, int iters, int timeout_ms);

#ifdef __cplusplus
}
#endif
#endif /* JFS_GPUCODEC_TEST_H */
