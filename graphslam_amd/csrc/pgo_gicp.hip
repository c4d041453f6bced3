// Batched Generalized-ICP scan registration on the GPU.
//
// Replaces the scanner node's registration (/root/reference/src/scanner/src/
// scanner.cpp:35-74: pcl::GeneralizedIterativeClosestPoint<PointXYZ, PointXYZ>
// with PCL's defaults, gicp.align(), hasConverged(), getFitnessScore(),
// getFinalTransformation(), then make_Delta / compute_covariance of
// scanner.hpp).  PCL is not vendored (third-party, version unpinned, ROS-era
// 1.7 / 1.8); its published GICP algorithm (pcl/registration/impl/gicp.hpp) is
// restated:
//   * per point, a plane-regularised covariance from its k nearest neighbours in
//     its own cloud (the point included): C = U diag(1, 1, eps) U^T with U the
//     eigenvectors of the neighbours' covariance, largest first;
//   * outer iterations: every source point transformed by T, its nearest
//     target point, kept when the squared distance < max_correspondence_distance^2;
//     M_i = (R C_src,i R^T + C_tgt,j)^-1 fixed for the iteration; T minimising
//     (1/n) sum d_i^T M_i d_i, d_i = T p_i - q_j; converged when no element of
//     T moved by more than rotation_epsilon (rotation part) / transformation_
//     epsilon (translation column) -- or at max_iterations, which PCL also
//     reports as converged;
//   * fitness = mean squared nearest-neighbour distance of the transformed source.
// Deviation: PCL minimises each iteration's objective with BFGS; here with
// Gauss-Newton on a left perturbation of T (the same objective, the same
// minimiser).  Ties in the nearest-neighbour searches go to the
// lowest index (PCL's kd-tree leaves them unspecified).
//
// MI355X layout: one workgroup per registration (a batch of B pairs is one
// launch), the target cloud staged in LDS for the brute-force nearest-neighbour
// scans, Gauss-Newton normal equations reduced in fixed order (bitwise
// reproducible), covariances one thread per point (register top-k).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "pgo.h"

namespace pgo {

constexpr int kGicpMaxK = 32;
constexpr int kGicpMaxPoints = 4096;   // per cloud (LDS: 4096 float4 = 64 KB)
constexpr int kGicpThreads = 256;

__device__ __forceinline__ float dist2(float dx, float dy, float dz);

// ---- plane-regularised covariances: one thread per point of any cloud
// cov[6 * p ..] = upper (00 01 02 11 12 22), double
__device__ void sym_eigen3(double a[3][3], double v[3][3]) {   // cyclic Jacobi; a -> diagonal, v columns = eigenvectors
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) v[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; sweep++) {
    const double off = fabs(a[0][1]) + fabs(a[0][2]) + fabs(a[1][2]);
    if (off < 1e-300) break;
#pragma unroll
    for (int pq = 0; pq < 3; pq++) {
      const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
      if (fabs(a[p][q]) < 1e-300) continue;
      const double theta = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
      const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
      const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
      for (int k = 0; k < 3; k++) {   // A <- J^T A J
        const double akp = a[k][p], akq = a[k][q];
        a[k][p] = c * akp - s * akq;
        a[k][q] = s * akp + c * akq;
      }
      for (int k = 0; k < 3; k++) {
        const double apk = a[p][k], aqk = a[q][k];
        a[p][k] = c * apk - s * aqk;
        a[q][k] = s * apk + c * aqk;
      }
      for (int k = 0; k < 3; k++) {
        const double vkp = v[k][p], vkq = v[k][q];
        v[k][p] = c * vkp - s * vkq;
        v[k][q] = s * vkp + c * vkq;
      }
    }
  }
}

// One workgroup per cloud, the cloud staged in LDS.  Each thread keeps the k
// nearest (distance, index) pairs of its point sorted by (distance, index) --
// the order the restatement's ascending scan with strict comparisons gives --
// through a branch-free compare-exchange network, so the scan may start at the
// point's index neighbours (scan order: i - 16, i - 15, ... wrapping): laser
// clouds come in beam order, the threshold tightens within the first few dozen
// candidates and the network rarely runs after that.  K: compile-time list
// length (20, PCL's default, or 32 for any k <= 32; slots >= k hold -inf and
// never take an entry).
template <int K>
__global__ __launch_bounds__(128) void k_gicp_cov(const float4* __restrict__ pts, const int2* __restrict__ clouds, int k,
                                                  double eps, double* __restrict__ cov) {
  extern __shared__ float4 cl[];
  const int2 c = clouds[blockIdx.x];   // (first point, count)
  const int n = c.y;
  for (int j = threadIdx.x; j < n; j += 128) cl[j] = pts[c.x + j];
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 128) {
    float bd[K];
    int bi[K];
#pragma unroll
    for (int t = 0; t < K; t++) {
      bd[t] = t < k ? INFINITY : -INFINITY;
      bi[t] = 0x7fffffff;
    }
    const float4 q = cl[i];
    int j = (i - 16) % n;
    if (j < 0) j += n;
    for (int u = 0; u < n; u++) {
      const float4 r = cl[j];
      const float d = dist2(r.x - q.x, r.y - q.y, r.z - q.z);
      if (K != 20 || d < bd[K - 1] || (d == bd[K - 1] && j < bi[K - 1])) {
        float v = d;
        int vi = j;
#pragma unroll
        for (int t = 0; t < K; t++) {
          const bool sw = v < bd[t] || (v == bd[t] && vi < bi[t]);
          const float nb = sw ? v : bd[t];
          const int ni = sw ? vi : bi[t];
          v = sw ? bd[t] : v;
          vi = sw ? bi[t] : vi;
          bd[t] = nb;
          bi[t] = ni;
        }
      }
      j = j + 1 == n ? 0 : j + 1;
    }
    double m[3] = {0, 0, 0}, s[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    int cnt = 0;
#pragma unroll
    for (int t = 0; t < K; t++) {
      if (t >= k || bi[t] == 0x7fffffff) continue;
      const float4 r = cl[bi[t]];
      const double x[3] = {r.x, r.y, r.z};
      for (int a = 0; a < 3; a++) {
        m[a] += x[a];
        for (int b = 0; b < 3; b++) s[a][b] += x[a] * x[b];
      }
      cnt++;
    }
    double a3[3][3], v[3][3];
    for (int a = 0; a < 3; a++) m[a] /= cnt;
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) a3[a][b] = s[a][b] / cnt - m[a] * m[b];
    sym_eigen3(a3, v);
    // eigenvalues descending: the same bubble order as the restatement, by
    // compare-exchange of whole columns (register indices stay static)
    double e[3] = {a3[0][0], a3[1][1], a3[2][2]};
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
      for (int y = 0; y < 2 - x; y++) {
        const bool sw = e[y] < e[y + 1];
        const double t = e[y];
        e[y] = sw ? e[y + 1] : e[y];
        e[y + 1] = sw ? t : e[y + 1];
#pragma unroll
        for (int r = 0; r < 3; r++) {
          const double tv = v[r][y];
          v[r][y] = sw ? v[r][y + 1] : v[r][y];
          v[r][y + 1] = sw ? tv : v[r][y + 1];
        }
      }
    double cc[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll
    for (int kk = 0; kk < 3; kk++) {
      const double w = kk == 2 ? eps : 1.0;
#pragma unroll
      for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = 0; b < 3; b++) cc[a][b] += w * v[a][kk] * v[b][kk];
    }
    double* out = cov + 6 * (size_t)(c.x + i);
    out[0] = cc[0][0]; out[1] = cc[0][1]; out[2] = cc[0][2]; out[3] = cc[1][1]; out[4] = cc[1][2]; out[5] = cc[2][2];
  }
}

__device__ __forceinline__ void inv3(const double a[3][3], double r[3][3]) {
  const double c00 = a[1][1] * a[2][2] - a[1][2] * a[2][1], c01 = a[1][2] * a[2][0] - a[1][0] * a[2][2],
               c02 = a[1][0] * a[2][1] - a[1][1] * a[2][0];
  const double det = a[0][0] * c00 + a[0][1] * c01 + a[0][2] * c02, id = 1.0 / det;
  r[0][0] = c00 * id;
  r[1][0] = c01 * id;
  r[2][0] = c02 * id;
  r[0][1] = (a[0][2] * a[2][1] - a[0][1] * a[2][2]) * id;
  r[1][1] = (a[0][0] * a[2][2] - a[0][2] * a[2][0]) * id;
  r[2][1] = (a[0][1] * a[2][0] - a[0][0] * a[2][1]) * id;
  r[0][2] = (a[0][1] * a[1][2] - a[0][2] * a[1][1]) * id;
  r[1][2] = (a[0][2] * a[1][0] - a[0][0] * a[1][2]) * id;
  r[2][2] = (a[0][0] * a[1][1] - a[0][1] * a[1][0]) * id;
}

// fixed-order workgroup sum of n doubles per thread into out[0..n) (thread 0)
template <int N>
__device__ __forceinline__ void wg_sum(double* v, double* red, double* out) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#pragma unroll
  for (int q = 0; q < N; q++) {
    double x = v[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
    if (lane == 0) red[q * 4 + wv] = x;
  }
  __syncthreads();
  if (tid < N) out[tid] = (red[tid * 4] + red[tid * 4 + 1]) + (red[tid * 4 + 2] + red[tid * 4 + 3]);
  __syncthreads();
}

// Squared distance, one fixed evaluation order (the restatement's too):
// fma(dz, dz, fma(dy, dy, dx * dx)).
__device__ __forceinline__ float dist2(float dx, float dy, float dz) { return fmaf(dz, dz, fmaf(dy, dy, dx * dx)); }

typedef float f2 __attribute__((ext_vector_type(2)));

// Nearest target point of two queries at once: one LDS read serves both, the
// queries' coordinates packed in float2 (v_pk_* with the target broadcast by
// op_sel), ties to the lower index; a query at +inf matches nothing.
__device__ __forceinline__ void nn2(const float4* __restrict__ tgt, int nt, float ax, float ay, float az, float bx,
                                    float by, float bz, float& da, int& ia, float& db, int& ib) {
  const f2 qx = {ax, bx}, qy = {ay, by}, qz = {az, bz};
  da = db = INFINITY;
  ia = ib = -1;
#pragma unroll 4
  for (int j = 0; j < nt; j++) {
    const float4 r = tgt[j];
    const f2 dx = (f2){r.x, r.x} - qx, dy = (f2){r.y, r.y} - qy, dz = (f2){r.z, r.z} - qz;
    const f2 d = __builtin_elementwise_fma(dz, dz, __builtin_elementwise_fma(dy, dy, dx * dx));
    if (d.x < da) {
      da = d.x;
      ia = j;
    }
    if (d.y < db) {
      db = d.y;
      ib = j;
    }
  }
}

// Workgroup sum of 28 doubles per thread (fixed order, bitwise reproducible):
// a reduce-scatter butterfly inside each wave (offsets 32 .. 2 halve the
// vector, so lane l ends with element (l >> 1) & 31 summed over its wave: 32
// shuffles instead of 28 x 6), then the 4 waves' partials through LDS.
__device__ __forceinline__ void wg_sum28(const double* v, double* red, double* out) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  double a[32];
#pragma unroll
  for (int q = 0; q < 32; q++) a[q] = q < 28 ? v[q] : 0.0;
#pragma unroll
  for (int o = 32, L = 32; o >= 2; o >>= 1, L >>= 1) {
    const bool up = lane & o;
#pragma unroll
    for (int i = 0; i < L / 2; i++) {
      const double keep = up ? a[L / 2 + i] : a[i];
      const double send = up ? a[i] : a[L / 2 + i];
      a[i] = keep + __shfl_xor(send, o);
    }
  }
  a[0] += __shfl_xor(a[0], 1);
  if (!(lane & 1) && (lane >> 1) < 28) red[(lane >> 1) * 4 + wv] = a[0];
  __syncthreads();
  if (tid < 28) out[tid] = (red[tid * 4] + red[tid * 4 + 1]) + (red[tid * 4 + 2] + red[tid * 4 + 3]);
  __syncthreads();
}

struct GicpArgs {
  const float4* pts;
  const double* cov;
  const int4* pairs;   // (source first, source count, target first, target count)
  const double* guess; // 16 per pair, row-major
  int max_it, max_inner;
  double thr2, rot_eps, trans_eps;
  int* nn;             // scratch: per point
  double* M;           // scratch: 6 per point
  double* out;         // per pair: T[16], iterations, converged, fitness, correspondences
};

// One correspondence's contribution to the Gauss-Newton normal equations of
// d^T M d, d = T p - q, at the current T = (R, t): acc[0..21) J'MJ (upper,
// row-major 6x6), acc[21..27) J'Md, acc[27] the count.
__device__ __forceinline__ void gn_point(const double (&R)[3][3], const double (&t)[3], float4 p, float4 qt,
                                         const double* mi, double (&acc)[28]) {
  const double w0 = R[0][0] * p.x + R[0][1] * p.y + R[0][2] * p.z + t[0];
  const double w1 = R[1][0] * p.x + R[1][1] * p.y + R[1][2] * p.z + t[1];
  const double w2 = R[2][0] * p.x + R[2][1] * p.y + R[2][2] * p.z + t[2];
  const double d[3] = {w0 - qt.x, w1 - qt.y, w2 - qt.z};
  const double M[3][3] = {{mi[0], mi[1], mi[2]}, {mi[1], mi[3], mi[4]}, {mi[2], mi[4], mi[5]}};
  // J = [A | I], A = -[w]x: J'MJ = [[A'MA, A'M], [MA, M]], J'Md = [A'Md; Md]
  // with A' = [w]x, so A'v = w x v, N := A'M (rows: w x M's columns),
  // A'MA = N A = -N [w]x, whose rows are w x (N's rows) -- closed forms
  // instead of the 3 x 6 products (fewer live registers)
  const double w[3] = {w0, w1, w2};
  auto cross = [&](const double* v, double* o) {
    o[0] = w[1] * v[2] - w[2] * v[1];
    o[1] = w[2] * v[0] - w[0] * v[2];
    o[2] = w[0] * v[1] - w[1] * v[0];
  };
  double Md[3], wMd[3], N[3][3], NT[3][3], UL[3][3];
#pragma unroll
  for (int x = 0; x < 3; x++) Md[x] = M[x][0] * d[0] + M[x][1] * d[1] + M[x][2] * d[2];
  cross(Md, wMd);
#pragma unroll
  for (int c = 0; c < 3; c++) cross(M[c], NT[c]);   // NT[c] = N's column c
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) N[r][c] = NT[c][r];
#pragma unroll
  for (int r = 0; r < 3; r++) cross(N[r], UL[r]);   // UL[r] = w x N_r = row r of N [w]x ^T
  int q = 0;
#pragma unroll
  for (int x = 0; x < 6; x++)
#pragma unroll
    for (int y = x; y < 6; y++)
      acc[q++] += x < 3 ? (y < 3 ? UL[x][y] : N[x][y - 3]) : M[x - 3][y - 3];
#pragma unroll
  for (int x = 0; x < 3; x++) {
    acc[21 + x] += wMd[x];
    acc[24 + x] += Md[x];
  }
  acc[27] += 1.0;
}

// One registration per workgroup.  kReg: the source cloud has <= 2 x 256
// points, every thread keeps its two points' correspondence, Mahalanobis
// matrix and coordinates in registers across the optimiser steps (otherwise
// they live in an L2-resident scratch).
template <bool kReg>
__global__ __launch_bounds__(kGicpThreads) void k_gicp(GicpArgs a) {
  extern __shared__ float4 tgt[];   // the target cloud (dynamic: max target count of the batch)
  __shared__ double red[28 * 4];
  __shared__ double sums[28];
  __shared__ double T[12];          // R (row-major 3x3) | t
  __shared__ int done;
  const int4 pr = a.pairs[blockIdx.x];
  const int tid = threadIdx.x;
  for (int j = tid; j < pr.w; j += kGicpThreads) tgt[j] = a.pts[pr.z + j];
  if (tid < 3) T[9 + tid] = a.guess[16 * blockIdx.x + tid * 4 + 3];
  if (tid < 9) T[tid] = a.guess[16 * blockIdx.x + (tid / 3) * 4 + tid % 3];
  __syncthreads();
  int* nnv = a.nn + pr.x;            // per source point: its correspondence (-1: none)
  double* Mv = a.M + 6 * (size_t)pr.x;   // and its Mahalanobis matrix (upper), L2-resident scratch
  int nnr[2] = {-1, -1};                 // kReg: the same in registers
  double Mr[2][6];
  float4 Pr[2];
  int it = 0, inner_total = 0;
  bool conv = false;
  while (!conv) {
    // correspondences at the current T; Mahalanobis M_i = (R C_s R^T + C_t)^-1
    double R[3][3], t[3];
    for (int x = 0; x < 3; x++) {
      for (int y = 0; y < 3; y++) R[x][y] = T[3 * x + y];
      t[x] = T[9 + x];
    }
    for (int i0 = tid; i0 < pr.y; i0 += 2 * kGicpThreads) {
      float q[2][3];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int i = i0 + h * kGicpThreads;
        if (i < pr.y) {
          const float4 p = a.pts[pr.x + i];
          for (int x = 0; x < 3; x++) q[h][x] = (float)(R[x][0] * p.x + R[x][1] * p.y + R[x][2] * p.z + t[x]);
        } else {
          q[h][0] = q[h][1] = q[h][2] = INFINITY;
        }
      }
      float bd[2];
      int bj[2];
      nn2(tgt, pr.w, q[0][0], q[0][1], q[0][2], q[1][0], q[1][1], q[1][2], bd[0], bj[0], bd[1], bj[1]);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int i = i0 + h * kGicpThreads;
        if (i >= pr.y) continue;
        const bool ok = bj[h] >= 0 && (double)bd[h] < a.thr2;
        if constexpr (kReg) {
          nnr[h] = ok ? bj[h] : -1;
          Pr[h] = a.pts[pr.x + i];
        } else {
          nnv[i] = ok ? bj[h] : -1;
        }
        if (!ok) continue;
        const double* cs = a.cov + 6 * (size_t)(pr.x + i);
        const double* ct = a.cov + 6 * (size_t)(pr.z + bj[h]);
        const double C[3][3] = {{cs[0], cs[1], cs[2]}, {cs[1], cs[3], cs[4]}, {cs[2], cs[4], cs[5]}};
        double RC[3][3], S[3][3], Minv[3][3];
        for (int x = 0; x < 3; x++)
          for (int y = 0; y < 3; y++) RC[x][y] = R[x][0] * C[0][y] + R[x][1] * C[1][y] + R[x][2] * C[2][y];
        const double Ct[3][3] = {{ct[0], ct[1], ct[2]}, {ct[1], ct[3], ct[4]}, {ct[2], ct[4], ct[5]}};
        for (int x = 0; x < 3; x++)
          for (int y = 0; y < 3; y++)
            S[x][y] = RC[x][0] * R[y][0] + RC[x][1] * R[y][1] + RC[x][2] * R[y][2] + Ct[x][y];
        inv3(S, Minv);
        double* mo = kReg ? Mr[h] : Mv + 6 * (size_t)i;
        mo[0] = Minv[0][0]; mo[1] = Minv[0][1]; mo[2] = Minv[0][2];
        mo[3] = Minv[1][1]; mo[4] = Minv[1][2]; mo[5] = Minv[2][2];
      }
    }
    double Tprev[12];
    for (int q = 0; q < 12; q++) Tprev[q] = T[q];
    // Gauss-Newton on (1/n) sum d^T M d, left perturbation T <- exp(dw, dt) T
    for (int inner = 0; inner < a.max_inner; inner++) {
      inner_total++;
      double acc[28];   // 21 JtMJ (upper, row-major 6x6) + 6 JtMd + count
#pragma unroll
      for (int q = 0; q < 28; q++) acc[q] = 0.0;
      for (int x = 0; x < 3; x++) {
        for (int y = 0; y < 3; y++) R[x][y] = T[3 * x + y];
        t[x] = T[9 + x];
      }
      if constexpr (kReg) {
#pragma unroll
        for (int h = 0; h < 2; h++)
          if (nnr[h] >= 0) gn_point(R, t, Pr[h], tgt[nnr[h]], Mr[h], acc);
      } else {
#pragma unroll 1
        for (int i = tid; i < pr.y; i += kGicpThreads) {
          const int j = nnv[i];
          if (j >= 0) gn_point(R, t, a.pts[pr.x + i], tgt[j], Mv + 6 * (size_t)i, acc);
        }
      }
      wg_sum28(acc, red, sums);
      if (tid == 0) {
        // 6x6 Cholesky solve, fully unrolled (the 1/n of the objective cancels)
        double A[6][6], x[6];
        int q = 0;
#pragma unroll
        for (int r = 0; r < 6; r++)
#pragma unroll
          for (int c = r; c < 6; c++) A[r][c] = A[c][r] = sums[q++];
        bool ok = sums[27] >= 3;
        double inv[6];   // reciprocal pivots: 6 divisions instead of 33
#pragma unroll
        for (int k = 0; k < 6; k++) {
          double d = A[k][k];
#pragma unroll
          for (int j = 0; j < k; j++) d -= A[k][j] * A[k][j];
          ok = ok && d > 0;
          inv[k] = 1.0 / sqrt(ok ? d : 1.0);
#pragma unroll
          for (int i = k + 1; i < 6; i++) {
            double v = A[i][k];
#pragma unroll
            for (int j = 0; j < k; j++) v -= A[i][j] * A[k][j];
            A[i][k] = v * inv[k];
          }
        }
#pragma unroll
        for (int i = 0; i < 6; i++) {
          double v = -sums[21 + i];
#pragma unroll
          for (int j = 0; j < i; j++) v -= A[i][j] * x[j];
          x[i] = v * inv[i];
        }
#pragma unroll
        for (int i = 5; i >= 0; i--) {
          double v = x[i];
#pragma unroll
          for (int j = i + 1; j < 6; j++) v -= A[j][i] * x[j];
          x[i] = v * inv[i];
        }
        int stop = 1;
        if (ok) {
          // exp of the rotation part (Rodrigues), applied on the left
          const double th = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
          double E[3][3];
          if (th < 1e-12) {
            E[0][0] = 1; E[0][1] = -x[2]; E[0][2] = x[1];
            E[1][0] = x[2]; E[1][1] = 1; E[1][2] = -x[0];
            E[2][0] = -x[1]; E[2][1] = x[0]; E[2][2] = 1;
          } else {
            const double ith = 1.0 / th, k0 = x[0] * ith, k1 = x[1] * ith, k2 = x[2] * ith;
            double sn, c;
            sincos(th, &sn, &c);
            const double v = 1 - c;
            E[0][0] = c + k0 * k0 * v; E[0][1] = k0 * k1 * v - k2 * sn; E[0][2] = k0 * k2 * v + k1 * sn;
            E[1][0] = k1 * k0 * v + k2 * sn; E[1][1] = c + k1 * k1 * v; E[1][2] = k1 * k2 * v - k0 * sn;
            E[2][0] = k2 * k0 * v - k1 * sn; E[2][1] = k2 * k1 * v + k0 * sn; E[2][2] = c + k2 * k2 * v;
          }
          double Tn[12];
#pragma unroll
          for (int r = 0; r < 3; r++) {
#pragma unroll
            for (int cc = 0; cc < 3; cc++) Tn[3 * r + cc] = E[r][0] * T[cc] + E[r][1] * T[3 + cc] + E[r][2] * T[6 + cc];
            Tn[9 + r] = E[r][0] * T[9] + E[r][1] * T[10] + E[r][2] * T[11] + x[3 + r];
          }
#pragma unroll
          for (int r = 0; r < 12; r++) T[r] = Tn[r];
          double step = 0;
#pragma unroll
          for (int i = 0; i < 6; i++) step = fmax(step, fabs(x[i]));
          stop = step < 1e-12;
        }
        done = stop;
      }
      __syncthreads();
      if (done) break;
    }
    it++;
    // PCL's convergence test on the change of T's elements
    double delta = 0;
    for (int q = 0; q < 12; q++) {
      const double ratio = q < 9 ? 1.0 / a.rot_eps : 1.0 / a.trans_eps;
      delta = fmax(delta, ratio * fabs(Tprev[q] - T[q]));
    }
    conv = it >= a.max_it || delta < 1.0;
  }
  // fitness: mean squared nearest-target distance of the transformed source
  double R[3][3], t[3];
  for (int x = 0; x < 3; x++) {
    for (int y = 0; y < 3; y++) R[x][y] = T[3 * x + y];
    t[x] = T[9 + x];
  }
  double fit[2] = {0, 0};
  for (int i0 = tid; i0 < pr.y; i0 += 2 * kGicpThreads) {
    float q[2][3];
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int i = i0 + h * kGicpThreads;
      if (i < pr.y) {
        const float4 p = a.pts[pr.x + i];
        for (int x = 0; x < 3; x++) q[h][x] = (float)(R[x][0] * p.x + R[x][1] * p.y + R[x][2] * p.z + t[x]);
      } else {
        q[h][0] = q[h][1] = q[h][2] = INFINITY;
      }
    }
    float bd[2];
    int bj[2];
    nn2(tgt, pr.w, q[0][0], q[0][1], q[0][2], q[1][0], q[1][1], q[1][2], bd[0], bj[0], bd[1], bj[1]);
    fit[0] += bd[0];
    fit[1] += 1.0;
    if (i0 + kGicpThreads < pr.y) {
      fit[0] += bd[1];
      fit[1] += 1.0;
    }
  }
  wg_sum<2>(fit, red, sums);
  if (tid == 0) {
    double* o = a.out + 20 * (size_t)blockIdx.x;
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) o[4 * r + c] = T[3 * r + c];
      o[4 * r + 3] = T[9 + r];
    }
    o[12] = o[13] = o[14] = 0.0;
    o[15] = 1.0;
    o[16] = it;
    o[17] = 1.0;   // PCL: converged_ is set at max_iterations too
    o[18] = sums[1] > 0 ? sums[0] / sums[1] : INFINITY;
    o[19] = inner_total;
  }
}

}  // namespace pgo

// ============================================================== C-ABI
struct pgo_gicp {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string last_error;
  double ms_last = 0.0;
  hipEvent_t ev[2] = {};
  void* host = nullptr;   // pinned staging (inputs, then results)
  size_t host_cap = 0;
  void *d_in = nullptr, *d_work = nullptr;   // grow-only device buffers
  size_t in_cap = 0, work_cap = 0;
};

namespace {
int gfail(pgo_gicp* h, int code, const std::string& m) {
  if (h) h->last_error = m;
  return code;
}
}  // namespace

extern "C" {

void pgo_gicp_default_params(pgo_gicp_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->max_iterations = 200;
  p->k_correspondences = 20;
  p->gicp_epsilon = 1e-3;
  p->max_correspondence_distance = 5.0;
  p->transformation_epsilon = 5e-4;
  p->rotation_epsilon = 2e-3;
  p->max_inner_iterations = 20;
}

pgo_gicp* pgo_gicp_create(int device) {
  pgo_gicp* h = new (std::nothrow) pgo_gicp();
  if (!h) return nullptr;
  h->device = device;
  return h;
}

void pgo_gicp_destroy(pgo_gicp* h) {
  if (!h) return;
  if (h->stream) {
    (void)hipSetDevice(h->device);
    (void)hipStreamSynchronize(h->stream);
    (void)hipStreamDestroy(h->stream);
    for (auto e : h->ev) (void)hipEventDestroy(e);
    if (h->d_in) (void)hipFree(h->d_in);
    if (h->d_work) (void)hipFree(h->d_work);
    if (h->host) (void)hipHostFree(h->host);
  }
  delete h;
}

const char* pgo_gicp_last_error(const pgo_gicp* h) { return h ? h->last_error.c_str() : "null handle"; }

int pgo_gicp_align_batch(pgo_gicp* h, int B, const float* src, const int* src_n, const float* tgt, const int* tgt_n,
                         const double* guess, const pgo_gicp_params* params, pgo_gicp_result* out) {
  if (!h || B < 0 || (B > 0 && (!src || !src_n || !tgt || !tgt_n || !out))) return PGO_E_ARG;
  if (B == 0) return PGO_OK;
  pgo_gicp_params p;
  if (params) p = *params;
  else pgo_gicp_default_params(&p);
  if (p.k_correspondences < 1 || p.k_correspondences > pgo::kGicpMaxK || p.max_iterations < 1 ||
      p.max_inner_iterations < 1 || !(p.gicp_epsilon > 0))
    return gfail(h, PGO_E_ARG, "gicp: k_correspondences in [1, 32], iterations >= 1, epsilon > 0");
  for (int b = 0; b < B; b++)
    if (src_n[b] < 1 || tgt_n[b] < 1 || src_n[b] > pgo::kGicpMaxPoints || tgt_n[b] > pgo::kGicpMaxPoints)
      return gfail(h, PGO_E_ARG, "gicp: clouds must hold 1 .. 4096 points");
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= h->device) return gfail(h, PGO_E_NO_DEVICE, "no HIP device");
  if (hipSetDevice(h->device) != hipSuccess) return gfail(h, PGO_E_NO_DEVICE, "hipSetDevice");
  if (!h->stream) {
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&h->ev[0]) != hipSuccess || hipEventCreate(&h->ev[1]) != hipSuccess)
      return gfail(h, PGO_E_HIP, "gicp stream");
  }
  // one staging block, one copy: points of all clouds (pair b's source then its
  // target, float4 x y z 0) | clouds (first, count) |
  // pairs (source first, count, target first, count) | guesses (16 doubles)
  long long npts_ll = 0;
  int max_t = 1;
  for (int b = 0; b < B; b++) {
    npts_ll += (long long)src_n[b] + tgt_n[b];
    max_t = std::max(max_t, tgt_n[b]);
  }
  if (npts_ll >= (1LL << 31) / 8) return gfail(h, PGO_E_ARG, "gicp: batch too large");
  const int npts = (int)npts_ll, ncl = 2 * B;
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_cl = al(sizeof(float4) * npts),
               o_pairs = o_cl + al(sizeof(int2) * ncl), o_guess = o_pairs + al(sizeof(int4) * B),
               in_bytes = o_guess + al(sizeof(double) * 16 * B);
  const size_t o_M = al(sizeof(double) * 6 * npts), o_nn = o_M + al(sizeof(double) * 6 * npts),
               o_out = o_nn + al(sizeof(int) * npts), work_bytes = o_out + al(sizeof(double) * 20 * B);
  if (h->host_cap < std::max(in_bytes, sizeof(double) * 20 * B)) {
    if (h->host) (void)hipHostFree(h->host);
    h->host = nullptr;
    h->host_cap = 0;
    const size_t want = std::max(in_bytes, sizeof(double) * 20 * B) * 3 / 2;
    if (hipHostMalloc(&h->host, want) != hipSuccess) return gfail(h, PGO_E_NOMEM, "gicp: pinned staging");
    h->host_cap = want;
  }
  char* hb = (char*)h->host;
  float4* pts = (float4*)hb;
  int2* clouds = (int2*)(hb + o_cl);
  int4* pairs = (int4*)(hb + o_pairs);
  double* g = (double*)(hb + o_guess);
  long long so = 0, to = 0;
  int k = 0;
  for (int b = 0; b < B; b++) {
    const int s0 = k;
    for (int i = 0; i < src_n[b]; i++, k++) {
      const float* q = src + 3 * (so + i);
      if (!std::isfinite(q[0]) || !std::isfinite(q[1]) || !std::isfinite(q[2]))
        return gfail(h, PGO_E_NONFINITE, "gicp: non-finite point");
      pts[k] = make_float4(q[0], q[1], q[2], 0.f);
    }
    const int t0 = k;
    for (int i = 0; i < tgt_n[b]; i++, k++) {
      const float* q = tgt + 3 * (to + i);
      if (!std::isfinite(q[0]) || !std::isfinite(q[1]) || !std::isfinite(q[2]))
        return gfail(h, PGO_E_NONFINITE, "gicp: non-finite point");
      pts[k] = make_float4(q[0], q[1], q[2], 0.f);
    }
    clouds[2 * b] = make_int2(s0, src_n[b]);
    clouds[2 * b + 1] = make_int2(t0, tgt_n[b]);
    pairs[b] = make_int4(s0, src_n[b], t0, tgt_n[b]);
    so += src_n[b];
    to += tgt_n[b];
    for (int q = 0; q < 16; q++) g[16 * b + q] = guess ? guess[16 * b + q] : (q % 5 == 0 ? 1.0 : 0.0);
  }
  hipError_t e = hipSuccess;
  auto grow = [&](void** p, size_t& cap, size_t need) {
    if (e != hipSuccess || cap >= need) return;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    e = hipMalloc(p, need * 3 / 2);
    if (e == hipSuccess) cap = need * 3 / 2;
  };
  hipStream_t s = h->stream;
  e = hipStreamSynchronize(s);   // the previous batch is done with the buffers
  grow(&h->d_in, h->in_cap, in_bytes);
  grow(&h->d_work, h->work_cap, work_bytes);
  if (e == hipSuccess) e = hipMemcpyAsync(h->d_in, hb, in_bytes, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    char* di = (char*)h->d_in;
    char* dw = (char*)h->d_work;
    (void)hipEventRecord(h->ev[0], s);
    int max_c = 1;
    for (int b = 0; b < B; b++) max_c = std::max({max_c, src_n[b], tgt_n[b]});
    if (p.k_correspondences == 20)
      pgo::k_gicp_cov<20><<<ncl, 128, sizeof(float4) * max_c, s>>>((const float4*)di, (const int2*)(di + o_cl), 20,
                                                                   p.gicp_epsilon, (double*)dw);
    else
      pgo::k_gicp_cov<pgo::kGicpMaxK><<<ncl, 128, sizeof(float4) * max_c, s>>>(
          (const float4*)di, (const int2*)(di + o_cl), p.k_correspondences, p.gicp_epsilon, (double*)dw);
    pgo::GicpArgs a;
    a.pts = (const float4*)di;
    a.cov = (const double*)dw;
    a.pairs = (const int4*)(di + o_pairs);
    a.guess = (const double*)(di + o_guess);
    a.max_it = p.max_iterations;
    a.max_inner = p.max_inner_iterations;
    a.thr2 = p.max_correspondence_distance * p.max_correspondence_distance;
    a.rot_eps = p.rotation_epsilon;
    a.trans_eps = p.transformation_epsilon;
    a.M = (double*)(dw + o_M);
    a.nn = (int*)(dw + o_nn);
    a.out = (double*)(dw + o_out);
    int max_s = 1;
    for (int b = 0; b < B; b++) max_s = std::max(max_s, src_n[b]);
    if (max_s <= 2 * pgo::kGicpThreads)
      pgo::k_gicp<true><<<B, pgo::kGicpThreads, sizeof(float4) * max_t, s>>>(a);
    else
      pgo::k_gicp<false><<<B, pgo::kGicpThreads, sizeof(float4) * max_t, s>>>(a);
    (void)hipEventRecord(h->ev[1], s);
    e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(h->host, dw + o_out, sizeof(double) * 20 * B, hipMemcpyDeviceToHost, s);
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  float ms = 0.f;
  if (e == hipSuccess && hipEventElapsedTime(&ms, h->ev[0], h->ev[1]) == hipSuccess) h->ms_last = ms;
  const double* o = (const double*)h->host;
  if (e != hipSuccess) return gfail(h, PGO_E_HIP, std::string("gicp: ") + hipGetErrorString(e));
  for (int b = 0; b < B; b++) {
    const double* r = &o[20 * (size_t)b];
    pgo_gicp_result& res = out[b];
    std::memcpy(res.T, r, 16 * sizeof(double));
    res.iterations = (int)r[16];
    res.converged = r[17] != 0.0;
    res.fitness = r[18];
    res.inner_iterations = (int)r[19];
    // make_Delta (scanner.hpp): x = T(0,3), y = T(1,3), theta = atan(T(1,0) / T(0,0)); the
    // reference reads the float transform (getFinalTransformation() is Matrix4f)
    const float T00 = (float)r[0], T10 = (float)r[4];
    res.delta[0] = (float)r[3];
    res.delta[1] = (float)r[7];
    res.delta[2] = std::atan((double)(T10 / T00));
    // compute_covariance(0.1, 0.1, 0.1, Delta) (scanner.hpp), row-major
    const double Dl = std::sqrt(std::pow(res.delta[0], 2) + std::pow(res.delta[1], 2));
    const double sxy = 0.1 * Dl, sth = 0.1 * Dl + 0.1 * res.delta[2];
    for (int q = 0; q < 9; q++) res.cov[q] = 0.0;
    res.cov[0] = sxy;
    res.cov[4] = sxy;
    res.cov[8] = sth;
    // scanner.cpp:55-58: a keyframe when converged and fitness > 0.1
    res.keyframe = res.converged && res.fitness > 0.1;
  }
  return PGO_OK;
}

int pgo_gicp_debug_ms(const pgo_gicp* h, double* ms) {
  if (!h || !ms) return PGO_E_ARG;
  *ms = h->ms_last;
  return PGO_OK;
}

}  // extern "C"
