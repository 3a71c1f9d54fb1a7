/*
 * chunkfs_amd_debug.h -- diagnostic entry points (not part of the drop-in
 * boundary).  They expose intermediate arrays of the LAST FastCDC batch of a
 * handle, so the scan's candidate records can be checked stage by stage on a
 * GPU (tests/test_gpu_resolve_paths.py).
 */
#ifndef CHUNKFS_AMD_DEBUG_H
#define CHUNKFS_AMD_DEBUG_H

#include "chunkfs_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* FastCDC pipeline of the handle: 3 (fastcdc.hip: scan + resolve), the only one. */
int cdc_debug_pipeline(const cdc_handle_t *h);
/* Candidate-record capacity per span (records are stored `cap` per span). */
uint32_t cdc_debug_record_cap(const cdc_handle_t *h);
/* Copy array `what` of the last batch to host memory `out` (at most
 * max_bytes): 0 = per-span candidate counts (u32; > cap means overflowed),
 * 1 = candidate records (u32, cap per span: offset in span (bits 0-23) |
 * truncated-region result of a chunk starting there (bits 24-29; 63 none, 62
 * not precomputed) | bit30 mask_l hit | bit31 mask_s hit).  Returns the bytes copied or a negative CDC_E*
 * code (CDC_EINVAL for any other `what`). */
int64_t cdc_debug_copy(cdc_handle_t *h, int what, void *out, size_t max_bytes);
/* Host-path statistics into v[0..n): cdc_chunk_data calls, their upload
 * seconds (CPU copy into the pinned ring + queueing the H2D), their total
 * seconds, then the chunking seconds and segment count of the current or
 * last streaming write (cdc_write_*), then the FastCDC batches taken by the
 * one-launch small-stream kernel (small.hip) and how many of them fell back
 * to the regular pipeline (a record / start budget exceeded). */
int cdc_debug_host_stats(const cdc_handle_t *h, double *v, size_t n);
/* Kernel times of the FastCDC batch `back` calls before the last one (0 = the
 * last; up to 63 back): scan_ms, resolve_ms, total_ms of t (the other fields
 * are the last batch's).  Each batch records its HIP events in its own slot of
 * a 64-entry ring, so a caller timing many back-to-back batches reads them
 * after the loop instead of waiting on each batch's events inside it.
 * Synchronous batches always record events; batches of
 * cdc_chunk_batch_device_async record them one in four
 * (CHUNKFS_AMD_EVENT_EVERY=k: one in k), the others report 0 ms.
 * CDC_EINVAL when that batch is not in the ring. */
int cdc_debug_timing_back(cdc_handle_t *h, uint32_t back, cdc_timing_t *t, size_t t_size);
/* Measured-achievable HBM read rate on the handle's device: a read-only
 * reduction kernel (16-byte coalesced loads, every byte once) over the DEVICE
 * buffer d_buf[len], `reps` timed launches after one warm-up; *ms = the
 * average launch time (HIP events).  The denominator of the bench line's
 * roofline.frac_of_achievable. */
int cdc_debug_read_bw(cdc_handle_t *h, const uint8_t *d_buf, size_t len, int reps, double *ms);

/* Host placement of the boundary as a JSON object written into buf (cap bytes,
 * NUL-terminated, truncated if short): the device's PCI address, NUMA node
 * ("gpu_node", -1 unknown) and PCIe link (current and max), whether the pinned
 * ring / chunk list / staging were allocated on that node and the copy helpers
 * bound to its CPUs ("numa_placement"; CHUNKFS_AMD_COPY_NUMA=0 turns it off),
 * the node the ring and chunk list actually landed on, the CPUs this process
 * may use and how many of the helpers were pinned.  Allocates the ring if the
 * handle has none yet.  Returns the JSON length or a negative CDC_E* code. */
int64_t cdc_debug_host_placement(cdc_handle_t *h, char *buf, size_t cap);

#ifdef __cplusplus
}
#endif

#endif /* CHUNKFS_AMD_DEBUG_H */
