// smax_internal.h -- internal interfaces between the kernels file
// (smax_kernels.hip) and the host runtime (smax_runtime.cpp).  Not part of
// the C-ABI.
#ifndef GT_SMAX_INTERNAL_H
#define GT_SMAX_INTERNAL_H

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include "gt_smax_hip.h"

// Offset of the library's own LCP/BWT tables past a 128-byte line: K1's
// window of tile l0 reads LCP[l0-16 .. l0+2064), 2080 bytes, which fit in 17
// lines when l0-16 starts 16 bytes into one and take 18 when the table is
// line-aligned (C3 step -0.5 %, 3/8 shard -0.7 %, profiles/s5/lcp_align_ab_*)
#define SMAX_TABLE_SHIFT 32

// Per-device caching allocator of the host runtime: plan buffers and staged
// tables come from it, so back-to-back calls in one process reuse device
// memory instead of hipMalloc/hipFree of multi-GB buffers per call.
// Blocks are stream-ordered: smax_dev_free returns a block whose work the
// caller has already synchronised (a blocking copy, a stream or event wait)
// to the cache at once; smax_dev_free_fenced returns one that work on some
// streams may still use, with a fence (events recorded on those streams) that
// the next smax_dev_alloc handing the block out waits for -- no call waits on
// the whole device.  With caching off (GT_SMAX_NO_CACHE=1) a block is freed.
// gt_smax_release_cache() frees everything cached.
hipError_t smax_dev_alloc(void **ptr, size_t bytes);   // on the current device
void smax_dev_free(void *ptr);                          // any device; NULL ok
struct SmaxFence;
// events on `streams` of the current device now (nstreams < 0: the whole
// device, for callers that lost track of their streams); released with the
// last block that holds it
SmaxFence *smax_fence_create(const hipStream_t *streams, int nstreams);
// a fence over events the caller already recorded (it takes ownership and
// destroys them); whole_device: also wait for the whole device
SmaxFence *smax_fence_adopt(const hipEvent_t *events, int nevents, bool whole_device);
void smax_dev_free_fenced(void *ptr, SmaxFence *fence);  // NULL ptr ok
void smax_fence_release(SmaxFence *fence);               // the creator's reference

// The streams a device-resident plan (F2 / F3) enqueued work on, each with
// an event recorded behind its last work there: waits and the delete-time
// fence of the plan's buffers use the events only (never a caller's stream
// handle, which may be destroyed first) and never the whole device unless
// more than SMAX_MARK_STREAMS streams were used.
#define SMAX_MARK_STREAMS 4
struct SmaxStreamMarks {
  hipStream_t s[SMAX_MARK_STREAMS];
  hipEvent_t ev[SMAX_MARK_STREAMS];
  int n;
  bool overflow;
};
void smax_marks_init(SmaxStreamMarks *m);
// after enqueueing on stream s (current device): the mark now stands behind it
void smax_marks_record(SmaxStreamMarks *m, hipStream_t s);
// waits for everything marked (host side)
hipError_t smax_marks_sync(SmaxStreamMarks *m);
// makes stream s wait for everything marked (device side)
hipError_t smax_marks_wait(SmaxStreamMarks *m, hipStream_t s);
// a fence over the marks (ownership of the events moves to it; m is reset)
SmaxFence *smax_marks_fence(SmaxStreamMarks *m);

// Device records of a plan -> host (lcp, lb, rb) triples through the
// device's pinned ring (the plan's work must be complete).
hipError_t smax_d2h_triples(uint64_t *dst, const GtSmaxRecord *dev, uint64_t cnt, void *stream);

// Host <-> device copies through the current device's pinned staging ring
// (threaded fill / copy-out overlapping the DMA; the host side stays
// pageable), for the F2/F3 host-table entry points.  Synchronous.
hipError_t smax_stage_upload(void *dst_dev, const void *src_host, uint64_t bytes);
hipError_t smax_stage_download(void *dst_host, const void *src_dev, uint64_t bytes);

// The calling thread's device on entry, restored when the guard goes out of
// scope (the host-table entry points work on it and leave it as found).
struct SmaxDeviceGuard {
  int dev = -1;
  SmaxDeviceGuard() { if (hipGetDevice(&dev) != hipSuccess) dev = -1; }
  ~SmaxDeviceGuard() { if (dev >= 0) (void) hipSetDevice(dev); }
  SmaxDeviceGuard(const SmaxDeviceGuard &) = delete;
  SmaxDeviceGuard &operator=(const SmaxDeviceGuard &) = delete;
};

// Packed BWT groups (GT_SMAX_PK_GROUPS layout) on the device from their code
// planes (the low 32 bits of each group) and the groups holding a special
// row, given as (group << 16 | special mask); enqueued on `stream`.
hipError_t smax_groups_from_planes(uint64_t *groups, const uint32_t *planes, uint64_t ngroups,
                                   const uint64_t *spec, uint64_t nspec, hipStream_t stream);

// Allocates and frees (into the cache) every buffer a plan over `shard`
// will take and loads the scan kernels' code object: run ahead of
// gt_smax_plan_create (e.g. beside the tables' upload) it takes the cold
// allocations off the plan's path.  Current device.
hipError_t smax_plan_reserve(const GtSmaxDevShard *shard, uint64_t capacity);

// GT_SMAX_TIMING=1: phase times of the host-table entry points on stderr.
double smax_phase_clock();
void smax_phase_mark(const char *what, double *t);

#endif
