/* mrnnt_devtools.h -- libmrnnt_devtools.so, bench / test helpers (not part of the product ABI).
 * Return 0 on success, 2 on invalid arguments, 3 on a launch failure. */
#ifndef MONOTONIC_RNNT_DEVTOOLS_H
#define MONOTONIC_RNNT_DEVTOOLS_H

#include <stddef.h>
#include <stdint.h>

typedef struct ihipStream_t *hipStream_t;

#ifdef __cplusplus
extern "C" {
#endif

/* out[0..count) = element (begin + i) of the counter-based generator: N(0,1)-like (normal=1) or U[0,1). */
int mrnnt_synth_acts(float *out, int64_t begin, int64_t count, uint64_t seed, int normal, hipStream_t stream);

/* Nontemporal device copy of `bytes` (multiple of 16, 16-byte aligned pointers) in the gradient pass's
 * access pattern (contiguous slabs per workgroup). */
int mrnnt_copy_probe(void *dst, const void *src, size_t bytes, hipStream_t stream);

/* Nontemporal read of `bytes` (multiple of 16, 16-byte aligned) in the same slab walk (the log-softmax pass's load
 * stream); `sink` is 4 bytes of device memory the kernel may write. */
int mrnnt_read_probe(const void *src, size_t bytes, void *sink, hipStream_t stream);

/* Nontemporal zero fill of `bytes` (multiple of 16, 16-byte aligned) in the same slab walk: the write half of
 * the copy probe alone. */
int mrnnt_write_probe(void *dst, size_t bytes, hipStream_t stream);

/* out[2 * slot] = the dispatch id the launch sees (the AQL packet index of its queue), out[2 * slot + 1] = its queue
 * address: what makes the chase launch's ready tags unique per launch, including HIP-graph replays. */
int mrnnt_dispatch_probe(uint64_t *out, int slot, hipStream_t stream);

/* Occupies every workgroup slot it gets (blocks_per_cu 256-thread workgroups per CU) for `us` microseconds of the
 * constant 100 MHz clock, then exits: a co-running kernel that holds the CUs, for scheduling tests. */
int mrnnt_occupy(int us, int blocks_per_cu, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif
