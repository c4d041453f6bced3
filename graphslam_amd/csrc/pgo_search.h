// Loop-closure candidate search kernels (internal; see pgo_search.hip).
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

namespace pgo {

// partial-result slots needed by launch_closest_scan for `limit` candidates
int closest_scan_blocks(int limit);
// closest of pose[0 .. limit) to (qx, qy): *out_d distance, *out_i index
// (part_*: closest_scan_blocks(limit) slots); start/stop optional dispatch events
hipError_t launch_closest_scan(const double4* pose, int limit, double qx, double qy, double* part_d, int* part_i,
                               double* out_d, int* out_i, hipStream_t s, hipEvent_t start = nullptr,
                               hipEvent_t stop = nullptr);
// candidate chunks of the batched search when no query has more than max_limit
int closest_batch_chunks(int max_limit);
// query q: pose index qv[q], candidates pose[0 .. qv[q] + 1 - skip); out_i = -1
// when none.  part_*: nq * closest_batch_chunks(max_limit) slots.  start/stop
// bracket both launches (search + merge)
hipError_t launch_closest_batch(const double4* pose, const int* qv, int nq, int skip, int max_limit,
                                double* part_d, int* part_i, double* out_d, int* out_i, hipStream_t s,
                                hipEvent_t start = nullptr, hipEvent_t stop = nullptr);

}  // namespace pgo
