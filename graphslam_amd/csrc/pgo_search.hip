// Loop-closure candidate search: the graph node's
// closest_keyframe service, /root/reference/src/graph/src/graph.cpp:146-178.
//
// The reference walks keyframes[0 .. size - skip - 1] (skip =
// keyframes_to_skip_in_loop_closing, graph.cpp:15), computes
// sqrt(pow(x2 - x1, 2) + pow(y2 - y1, 2)) to the request's pose_opti (:153-158)
// and keeps the first index with the smallest distance (strict <, :161-166).
// Here the keyframe positions are the handle's current values (pose, HBM,
// insertion order) -- the reference's pose_opti after its solve() write-back.
//
// Exactness: distances are formed with round-to-nearest multiplies and adds
// (no FMA contraction, like the reference's x86-64 build) and a correctly
// rounded sqrt.  A scan keeps (d, index) and takes the square root only when
// the squared distance drops below the best one's (sqrt is monotone, so
// s >= s_best cannot give d < d_best); partial results merge by the
// lexicographic minimum of (d, index), which is the reference's "first index
// among the smallest distances" whatever the merge order.
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

#include "pgo_device.h"
#include "pgo_search.h"

namespace pgo {
namespace {

constexpr int kScanThreads = 256;
constexpr int kBatchTile = 512;   // candidate positions staged in LDS per tile (8 KB)
constexpr int kBatchChunk = 4096; // candidates per workgroup of the batched search

// (px - qx)^2 + (py - qy)^2 with every operation rounded on its own: HIP
// compiles with -ffp-contract=fast, which would fuse this into an FMA
__device__ __forceinline__ double sq_dist(double px, double py, double qx, double qy) {
#pragma clang fp contract(off)
  const double dx = px - qx, dy = py - qy;
  return dx * dx + dy * dy;
}

// consider candidate j (scanned in increasing j) against the running best
__device__ __forceinline__ void consider(double s, int j, double& sb, double& db, int& ib) {
  if (s < sb) {
    const double d = __builtin_sqrt(s);   // llvm.sqrt.f64: correctly rounded on gfx950
    sb = s;
    if (d < db) {
      db = d;
      ib = j;
    }
  }
}

__device__ __forceinline__ bool lex_less(double d, int i, double db, int ib) {
  return d < db || (d == db && i < ib);
}

// lexicographic (d, index) minimum over the workgroup; result in lane 0 of wave 0
__device__ __forceinline__ void block_argmin(double& d, int& i, double* lds_d, int* lds_i) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double d2 = __shfl_xor(d, o, 64);
    const int i2 = __shfl_xor(i, o, 64);
    if (lex_less(d2, i2, d, i)) {
      d = d2;
      i = i2;
    }
  }
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    lds_d[w] = d;
    lds_i[w] = i;
  }
  __syncthreads();
  if (threadIdx.x == 0)
    for (int k = 1; k < nw; k++)
      if (lex_less(lds_d[k], lds_i[k], d, i)) {
        d = lds_d[k];
        i = lds_i[k];
      }
}

// One query over candidates [0, limit): grid-stride scan, one partial per workgroup.
__global__ __launch_bounds__(kScanThreads) void k_closest_scan(const double4* __restrict__ pose, int limit, double qx,
                                                               double qy, double* __restrict__ pd,
                                                               int* __restrict__ pi) {
  __shared__ double lds_d[kScanThreads / 64];
  __shared__ int lds_i[kScanThreads / 64];
  double sb = INFINITY, db = INFINITY;
  int ib = 0x7fffffff;
  const double2* p2 = reinterpret_cast<const double2*>(pose);   // (x, y) halves of the double4 values
  for (int j = blockIdx.x * kScanThreads + threadIdx.x; j < limit; j += gridDim.x * kScanThreads) {
    const double2 p = p2[2 * j];
    consider(sq_dist(p.x, p.y, qx, qy), j, sb, db, ib);
  }
  block_argmin(db, ib, lds_d, lds_i);
  if (threadIdx.x == 0) {
    pd[blockIdx.x] = db;
    pi[blockIdx.x] = ib;
  }
}

__global__ __launch_bounds__(kScanThreads) void k_closest_final(const double* __restrict__ pd,
                                                                const int* __restrict__ pi, int nb,
                                                                double* __restrict__ out_d, int* __restrict__ out_i) {
  __shared__ double lds_d[kScanThreads / 64];
  __shared__ int lds_i[kScanThreads / 64];
  double db = INFINITY;
  int ib = 0x7fffffff;
  for (int k = threadIdx.x; k < nb; k += kScanThreads)
    if (lex_less(pd[k], pi[k], db, ib)) {
      db = pd[k];
      ib = pi[k];
    }
  block_argmin(db, ib, lds_d, lds_i);
  if (threadIdx.x == 0) {
    *out_d = db;
    *out_i = ib;
  }
}

// Many queries: thread t of workgroup (bx, by) owns query q = bx * 256 + t
// (pose index qv[q], candidates [0, qv[q] + 1 - skip)) and scans candidate
// chunk by = [by * kBatchChunk, (by + 1) * kBatchChunk) of it; the workgroup
// streams the chunk's positions through LDS in tiles of kBatchTile, every lane
// reading the same LDS word (broadcast) per candidate, two candidates per
// step.  The 2-D grid keeps >> 256 workgroups in flight; partials go to
// part[by * nq + q] and k_closest_merge folds them in chunk order.
__global__ __launch_bounds__(kScanThreads) void k_closest_batch(const double4* __restrict__ pose,
                                                                const int* __restrict__ qv, int nq, int skip,
                                                                double* __restrict__ part_d,
                                                                int* __restrict__ part_i) {
  __shared__ double2 tile[kBatchTile];
  __shared__ int lim_max;
  const int q = blockIdx.x * kScanThreads + threadIdx.x;
  const double2* p2 = reinterpret_cast<const double2*>(pose);
  const int c0 = blockIdx.y * kBatchChunk;
  int lim = 0;
  double qx = 0.0, qy = 0.0;
  if (q < nq) {
    const int v = qv[q];
    lim = min(max(v + 1 - skip, 0) - c0, kBatchChunk);   // candidates of this chunk (may be <= 0)
    const double2 p = p2[2 * v];
    qx = p.x;
    qy = p.y;
  }
  if (threadIdx.x == 0) lim_max = 0;
  __syncthreads();
  atomicMax(&lim_max, lim);
  __syncthreads();
  const int L = lim_max;
  double sb = INFINITY, db = INFINITY;
  int ib = -1;
  for (int t0 = 0; t0 < L; t0 += kBatchTile) {
    const int nt = min(kBatchTile, L - t0);
    for (int k = threadIdx.x; k < nt; k += kScanThreads) tile[k] = p2[2 * (c0 + t0 + k)];
    __syncthreads();
    const int m = min(nt, lim - t0);
    int k = 0;
    for (; k + 1 < m; k += 2) {
      const double2 a = tile[k], b = tile[k + 1];
      const double sa = sq_dist(a.x, a.y, qx, qy), sbb = sq_dist(b.x, b.y, qx, qy);
      consider(sa, c0 + t0 + k, sb, db, ib);
      consider(sbb, c0 + t0 + k + 1, sb, db, ib);
    }
    if (k < m) consider(sq_dist(tile[k].x, tile[k].y, qx, qy), c0 + t0 + k, sb, db, ib);
    __syncthreads();
  }
  if (q < nq && lim > 0) {
    part_d[(size_t)blockIdx.y * nq + q] = db;
    part_i[(size_t)blockIdx.y * nq + q] = ib;
  }
}

// fold the chunk partials of every query in chunk order (lexicographic (d, i))
__global__ __launch_bounds__(kScanThreads) void k_closest_merge(const int* __restrict__ qv, int nq, int skip,
                                                                const double* __restrict__ part_d,
                                                                const int* __restrict__ part_i,
                                                                double* __restrict__ out_d, int* __restrict__ out_i) {
  const int q = blockIdx.x * kScanThreads + threadIdx.x;
  if (q >= nq) return;
  const int lim = max(qv[q] + 1 - skip, 0);
  const int nc = (lim + kBatchChunk - 1) / kBatchChunk;
  double db = INFINITY;
  int ib = -1;
  for (int c = 0; c < nc; c++) {
    const double d = part_d[(size_t)c * nq + q];
    const int i = part_i[(size_t)c * nq + q];
    if (i >= 0 && (ib < 0 || lex_less(d, i, db, ib))) {
      db = d;
      ib = i;
    }
  }
  out_d[q] = db;
  out_i[q] = ib;
}

}  // namespace

int closest_scan_blocks(int limit) {
  const int nb = (limit + kScanThreads - 1) / kScanThreads;
  return nb < 1 ? 1 : (nb > kMaxBlocks ? kMaxBlocks : nb);
}

hipError_t launch_closest_scan(const double4* pose, int limit, double qx, double qy, double* part_d, int* part_i,
                               double* out_d, int* out_i, hipStream_t s, hipEvent_t start, hipEvent_t stop) {
  const int nb = closest_scan_blocks(limit);
  hipExtLaunchKernelGGL(k_closest_scan, dim3(nb), dim3(kScanThreads), 0, s, start, stop, 0, pose, limit, qx, qy,
                        part_d, part_i);
  k_closest_final<<<1, kScanThreads, 0, s>>>(part_d, part_i, nb, out_d, out_i);
  return hipGetLastError();
}

int closest_batch_chunks(int max_limit) { return std::max(1, (max_limit + kBatchChunk - 1) / kBatchChunk); }

hipError_t launch_closest_batch(const double4* pose, const int* qv, int nq, int skip, int max_limit,
                                double* part_d, int* part_i, double* out_d, int* out_i, hipStream_t s,
                                hipEvent_t start, hipEvent_t stop) {
  if (nq <= 0) return hipSuccess;
  const int nb = (nq + kScanThreads - 1) / kScanThreads;
  const int nc = closest_batch_chunks(max_limit);
  hipExtLaunchKernelGGL(k_closest_batch, dim3(nb, nc), dim3(kScanThreads), 0, s, start, nullptr, 0, pose, qv, nq,
                        skip, part_d, part_i);
  hipExtLaunchKernelGGL(k_closest_merge, dim3(nb), dim3(kScanThreads), 0, s, nullptr, stop, 0, qv, nq, skip, part_d,
                        part_i, out_d, out_i);
  return hipGetLastError();
}

}  // namespace pgo
