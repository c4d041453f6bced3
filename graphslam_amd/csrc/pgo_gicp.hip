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

#include <cstring>
#include <string>
#include <vector>

#include "pgo.h"

namespace pgo {

constexpr int kGicpMaxK = 32;
constexpr int kGicpMaxPoints = 4096;   // per cloud (LDS: 4096 float4 = 64 KB)
constexpr int kGicpThreads = 256;

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

__global__ __launch_bounds__(kGicpThreads) void k_gicp_cov(const float4* __restrict__ pts, const int* __restrict__ cloud_of,
                                                          const int2* __restrict__ clouds, int npts, int k, double eps,
                                                          double* __restrict__ cov) {
  const int p = blockIdx.x * kGicpThreads + threadIdx.x;
  if (p >= npts) return;
  const int2 cl = clouds[cloud_of[p]];   // (first point, count)
  const float4 q = pts[p];
  float bd[kGicpMaxK];
  int bi[kGicpMaxK];
  for (int t = 0; t < k; t++) {
    bd[t] = INFINITY;
    bi[t] = -1;
  }
  for (int j = 0; j < cl.y; j++) {   // k nearest (the point itself included), ties to the lower index
    const float4 r = pts[cl.x + j];
    const float dx = r.x - q.x, dy = r.y - q.y, dz = r.z - q.z;
    const float d = dx * dx + dy * dy + dz * dz;
    if (!(d < bd[k - 1])) continue;
    int t = k - 1;
    while (t > 0 && d < bd[t - 1]) {
      bd[t] = bd[t - 1];
      bi[t] = bi[t - 1];
      t--;
    }
    bd[t] = d;
    bi[t] = j;
  }
  double m[3] = {0, 0, 0}, s[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  int cnt = 0;
  for (int t = 0; t < k; t++) {
    if (bi[t] < 0) continue;
    const float4 r = pts[cl.x + bi[t]];
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
  int o[3] = {0, 1, 2};   // eigenvalues descending
  for (int x = 0; x < 2; x++)
    for (int y = 0; y < 2 - x; y++)
      if (a3[o[y]][o[y]] < a3[o[y + 1]][o[y + 1]]) {
        const int t = o[y];
        o[y] = o[y + 1];
        o[y + 1] = t;
      }
  double c[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  for (int kk = 0; kk < 3; kk++) {
    const double w = kk == 2 ? eps : 1.0;
    const int col = o[kk];
    for (int a = 0; a < 3; a++)
      for (int b = 0; b < 3; b++) c[a][b] += w * v[a][col] * v[b][col];
  }
  double* out = cov + 6 * (size_t)p;
  out[0] = c[0][0]; out[1] = c[0][1]; out[2] = c[0][2]; out[3] = c[1][1]; out[4] = c[1][2]; out[5] = c[2][2];
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

// One registration per workgroup.
__global__ __launch_bounds__(kGicpThreads) void k_gicp(GicpArgs a) {
  __shared__ float4 tgt[kGicpMaxPoints];
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
  int it = 0;
  bool conv = false;
  while (!conv) {
    // correspondences at the current T; Mahalanobis M_i = (R C_s R^T + C_t)^-1
    double R[3][3], t[3];
    for (int x = 0; x < 3; x++) {
      for (int y = 0; y < 3; y++) R[x][y] = T[3 * x + y];
      t[x] = T[9 + x];
    }
    for (int i = tid; i < pr.y; i += kGicpThreads) {
      nnv[i] = -1;
      const float4 p = a.pts[pr.x + i];
      const double q0 = R[0][0] * p.x + R[0][1] * p.y + R[0][2] * p.z + t[0];
      const double q1 = R[1][0] * p.x + R[1][1] * p.y + R[1][2] * p.z + t[1];
      const double q2 = R[2][0] * p.x + R[2][1] * p.y + R[2][2] * p.z + t[2];
      const float qf0 = (float)q0, qf1 = (float)q1, qf2 = (float)q2;
      float best = INFINITY;
      int bj = -1;
      for (int j = 0; j < pr.w; j++) {
        const float4 r = tgt[j];
        const float dx = r.x - qf0, dy = r.y - qf1, dz = r.z - qf2;
        const float d = dx * dx + dy * dy + dz * dz;
        if (d < best) {
          best = d;
          bj = j;
        }
      }
      if (!(bj >= 0 && (double)best < a.thr2)) continue;
      nnv[i] = bj;
      const double* cs = a.cov + 6 * (size_t)(pr.x + i);
      const double* ct = a.cov + 6 * (size_t)(pr.z + bj);
      const double C[3][3] = {{cs[0], cs[1], cs[2]}, {cs[1], cs[3], cs[4]}, {cs[2], cs[4], cs[5]}};
      double RC[3][3], S[3][3], Minv[3][3];
      for (int x = 0; x < 3; x++)
        for (int y = 0; y < 3; y++) RC[x][y] = R[x][0] * C[0][y] + R[x][1] * C[1][y] + R[x][2] * C[2][y];
      const double Ct[3][3] = {{ct[0], ct[1], ct[2]}, {ct[1], ct[3], ct[4]}, {ct[2], ct[4], ct[5]}};
      for (int x = 0; x < 3; x++)
        for (int y = 0; y < 3; y++) S[x][y] = RC[x][0] * R[y][0] + RC[x][1] * R[y][1] + RC[x][2] * R[y][2] + Ct[x][y];
      inv3(S, Minv);
      double* mo = Mv + 6 * (size_t)i;
      mo[0] = Minv[0][0]; mo[1] = Minv[0][1]; mo[2] = Minv[0][2];
      mo[3] = Minv[1][1]; mo[4] = Minv[1][2]; mo[5] = Minv[2][2];
    }
    double Tprev[12];
    for (int q = 0; q < 12; q++) Tprev[q] = T[q];
    // Gauss-Newton on (1/n) sum d^T M d, left perturbation T <- exp(dw, dt) T
    for (int inner = 0; inner < a.max_inner; inner++) {
      double acc[28];   // 21 JtMJ (upper, row-major 6x6) + 6 JtMd + count
#pragma unroll
      for (int q = 0; q < 28; q++) acc[q] = 0.0;
      for (int x = 0; x < 3; x++) {
        for (int y = 0; y < 3; y++) R[x][y] = T[3 * x + y];
        t[x] = T[9 + x];
      }
      for (int i = tid; i < pr.y; i += kGicpThreads) {
        const int j = nnv[i];
        if (j < 0) continue;
        const float4 p = a.pts[pr.x + i];
        const float4 qt = tgt[j];
        const double* mi = Mv + 6 * (size_t)i;
        const double w0 = R[0][0] * p.x + R[0][1] * p.y + R[0][2] * p.z + t[0];
        const double w1 = R[1][0] * p.x + R[1][1] * p.y + R[1][2] * p.z + t[1];
        const double w2 = R[2][0] * p.x + R[2][1] * p.y + R[2][2] * p.z + t[2];
        const double d[3] = {w0 - qt.x, w1 - qt.y, w2 - qt.z};
        const double M[3][3] = {{mi[0], mi[1], mi[2]}, {mi[1], mi[3], mi[4]}, {mi[2], mi[4], mi[5]}};
        // J = [ -[w]x | I ]  (3 x 6)
        const double J[3][6] = {{0, w2, -w1, 1, 0, 0}, {-w2, 0, w0, 0, 1, 0}, {w1, -w0, 0, 0, 0, 1}};
        double MJ[3][6], Md[3];
        for (int x = 0; x < 3; x++) {
          Md[x] = M[x][0] * d[0] + M[x][1] * d[1] + M[x][2] * d[2];
          for (int y = 0; y < 6; y++) MJ[x][y] = M[x][0] * J[0][y] + M[x][1] * J[1][y] + M[x][2] * J[2][y];
        }
        int q = 0;
        for (int x = 0; x < 6; x++)
          for (int y = x; y < 6; y++) acc[q++] += J[0][x] * MJ[0][y] + J[1][x] * MJ[1][y] + J[2][x] * MJ[2][y];
        for (int x = 0; x < 6; x++) acc[21 + x] += J[0][x] * Md[0] + J[1][x] * Md[1] + J[2][x] * Md[2];
        acc[27] += 1.0;
      }
      wg_sum<28>(acc, red, sums);
      if (tid == 0) {
        done = 0;
        double A[6][6], b[6];
        int q = 0;
        for (int x = 0; x < 6; x++)
          for (int y = x; y < 6; y++) A[x][y] = A[y][x] = sums[q++];
        for (int x = 0; x < 6; x++) b[x] = -sums[21 + x];
        bool ok = sums[27] >= 3;
        for (int k = 0; k < 6 && ok; k++) {   // Cholesky solve (the 1/n of the objective cancels)
          double s = A[k][k];
          for (int j = 0; j < k; j++) s -= A[k][j] * A[k][j];
          if (!(s > 0)) {
            ok = false;
            break;
          }
          A[k][k] = sqrt(s);
          for (int i = k + 1; i < 6; i++) {
            double v = A[i][k];
            for (int j = 0; j < k; j++) v -= A[i][j] * A[k][j];
            A[i][k] = v / A[k][k];
          }
        }
        double x[6] = {0, 0, 0, 0, 0, 0};
        if (ok) {
          for (int i = 0; i < 6; i++) {
            double v = b[i];
            for (int j = 0; j < i; j++) v -= A[i][j] * x[j];
            x[i] = v / A[i][i];
          }
          for (int i = 5; i >= 0; i--) {
            double v = x[i];
            for (int j = i + 1; j < 6; j++) v -= A[j][i] * x[j];
            x[i] = v / A[i][i];
          }
          // exp of the rotation part (Rodrigues), applied on the left
          const double th = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
          double E[3][3];
          if (th < 1e-12) {
            E[0][0] = 1; E[0][1] = -x[2]; E[0][2] = x[1];
            E[1][0] = x[2]; E[1][1] = 1; E[1][2] = -x[0];
            E[2][0] = -x[1]; E[2][1] = x[0]; E[2][2] = 1;
          } else {
            const double k0 = x[0] / th, k1 = x[1] / th, k2 = x[2] / th, c = cos(th), s = sin(th), v = 1 - c;
            E[0][0] = c + k0 * k0 * v; E[0][1] = k0 * k1 * v - k2 * s; E[0][2] = k0 * k2 * v + k1 * s;
            E[1][0] = k1 * k0 * v + k2 * s; E[1][1] = c + k1 * k1 * v; E[1][2] = k1 * k2 * v - k0 * s;
            E[2][0] = k2 * k0 * v - k1 * s; E[2][1] = k2 * k1 * v + k0 * s; E[2][2] = c + k2 * k2 * v;
          }
          double Rn[3][3], tn[3];
          for (int r = 0; r < 3; r++) {
            for (int cc = 0; cc < 3; cc++) Rn[r][cc] = E[r][0] * T[cc] + E[r][1] * T[3 + cc] + E[r][2] * T[6 + cc];
            tn[r] = E[r][0] * T[9] + E[r][1] * T[10] + E[r][2] * T[11] + x[3 + r];
          }
          for (int r = 0; r < 3; r++) {
            for (int cc = 0; cc < 3; cc++) T[3 * r + cc] = Rn[r][cc];
            T[9 + r] = tn[r];
          }
          double step = 0;
          for (int i = 0; i < 6; i++) step = fmax(step, fabs(x[i]));
          if (step < 1e-12) done = 1;
        } else {
          done = 1;
        }
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
  for (int i = tid; i < pr.y; i += kGicpThreads) {
    const float4 p = a.pts[pr.x + i];
    const float q0 = (float)(R[0][0] * p.x + R[0][1] * p.y + R[0][2] * p.z + t[0]);
    const float q1 = (float)(R[1][0] * p.x + R[1][1] * p.y + R[1][2] * p.z + t[1]);
    const float q2 = (float)(R[2][0] * p.x + R[2][1] * p.y + R[2][2] * p.z + t[2]);
    float best = INFINITY;
    for (int j = 0; j < pr.w; j++) {
      const float4 r = tgt[j];
      const float dx = r.x - q0, dy = r.y - q1, dz = r.z - q2;
      best = fminf(best, dx * dx + dy * dy + dz * dz);
    }
    fit[0] += best;
    fit[1] += 1.0;
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
    o[19] = 0;
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
  // points of all clouds: pair b's source then its target, float4 (x, y, z, 0)
  std::vector<float4> pts;
  std::vector<int> cloud_of;
  std::vector<int2> clouds;
  std::vector<int4> pairs(B);
  long long so = 0, to = 0;
  for (int b = 0; b < B; b++) {
    const int s0 = (int)pts.size();
    for (int i = 0; i < src_n[b]; i++) {
      const float* q = src + 3 * (so + i);
      if (!std::isfinite(q[0]) || !std::isfinite(q[1]) || !std::isfinite(q[2]))
        return gfail(h, PGO_E_NONFINITE, "gicp: non-finite point");
      pts.push_back(make_float4(q[0], q[1], q[2], 0.f));
      cloud_of.push_back((int)clouds.size());
    }
    clouds.push_back(make_int2(s0, src_n[b]));
    const int t0 = (int)pts.size();
    for (int i = 0; i < tgt_n[b]; i++) {
      const float* q = tgt + 3 * (to + i);
      if (!std::isfinite(q[0]) || !std::isfinite(q[1]) || !std::isfinite(q[2]))
        return gfail(h, PGO_E_NONFINITE, "gicp: non-finite point");
      pts.push_back(make_float4(q[0], q[1], q[2], 0.f));
      cloud_of.push_back((int)clouds.size());
    }
    clouds.push_back(make_int2(t0, tgt_n[b]));
    pairs[b] = make_int4(s0, src_n[b], t0, tgt_n[b]);
    so += src_n[b];
    to += tgt_n[b];
  }
  std::vector<double> g(16 * (size_t)B, 0.0);
  for (int b = 0; b < B; b++)
    for (int q = 0; q < 16; q++) g[16 * b + q] = guess ? guess[16 * b + q] : (q % 5 == 0 ? 1.0 : 0.0);
  const int npts = (int)pts.size();
  float4* d_pts = nullptr;
  int *d_cof = nullptr;
  int2* d_cl = nullptr;
  int4* d_pairs = nullptr;
  double *d_cov = nullptr, *d_guess = nullptr, *d_out = nullptr;
  hipError_t e = hipMalloc((void**)&d_pts, sizeof(float4) * npts);
  if (e == hipSuccess) e = hipMalloc((void**)&d_cof, sizeof(int) * npts);
  if (e == hipSuccess) e = hipMalloc((void**)&d_cl, sizeof(int2) * clouds.size());
  if (e == hipSuccess) e = hipMalloc((void**)&d_pairs, sizeof(int4) * B);
  if (e == hipSuccess) e = hipMalloc((void**)&d_cov, sizeof(double) * 6 * npts);
  if (e == hipSuccess) e = hipMalloc((void**)&d_guess, sizeof(double) * 16 * B);
  if (e == hipSuccess) e = hipMalloc((void**)&d_out, sizeof(double) * 20 * B);
  int* d_nn = nullptr;
  double* d_M = nullptr;
  if (e == hipSuccess) e = hipMalloc((void**)&d_nn, sizeof(int) * npts);
  if (e == hipSuccess) e = hipMalloc((void**)&d_M, sizeof(double) * 6 * npts);
  hipStream_t s = h->stream;
  if (e == hipSuccess) e = hipMemcpyAsync(d_pts, pts.data(), sizeof(float4) * npts, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_cof, cloud_of.data(), sizeof(int) * npts, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_cl, clouds.data(), sizeof(int2) * clouds.size(), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_pairs, pairs.data(), sizeof(int4) * B, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(d_guess, g.data(), sizeof(double) * 16 * B, hipMemcpyHostToDevice, s);
  std::vector<double> o(20 * (size_t)B);
  if (e == hipSuccess) {
    (void)hipEventRecord(h->ev[0], s);
    pgo::k_gicp_cov<<<(npts + pgo::kGicpThreads - 1) / pgo::kGicpThreads, pgo::kGicpThreads, 0, s>>>(
        d_pts, d_cof, d_cl, npts, p.k_correspondences, p.gicp_epsilon, d_cov);
    pgo::GicpArgs a;
    a.pts = d_pts;
    a.cov = d_cov;
    a.pairs = d_pairs;
    a.guess = d_guess;
    a.max_it = p.max_iterations;
    a.max_inner = p.max_inner_iterations;
    a.thr2 = p.max_correspondence_distance * p.max_correspondence_distance;
    a.rot_eps = p.rotation_epsilon;
    a.trans_eps = p.transformation_epsilon;
    a.nn = d_nn;
    a.M = d_M;
    a.out = d_out;
    pgo::k_gicp<<<B, pgo::kGicpThreads, 0, s>>>(a);
    (void)hipEventRecord(h->ev[1], s);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(o.data(), d_out, sizeof(double) * 20 * B, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  float ms = 0.f;
  if (e == hipSuccess && hipEventElapsedTime(&ms, h->ev[0], h->ev[1]) == hipSuccess) h->ms_last = ms;
  for (void* q : {(void*)d_pts, (void*)d_cof, (void*)d_cl, (void*)d_pairs, (void*)d_cov, (void*)d_guess, (void*)d_out, (void*)d_nn, (void*)d_M})
    if (q) (void)hipFree(q);
  if (e != hipSuccess) return gfail(h, PGO_E_HIP, std::string("gicp: ") + hipGetErrorString(e));
  for (int b = 0; b < B; b++) {
    const double* r = &o[20 * (size_t)b];
    pgo_gicp_result& res = out[b];
    std::memcpy(res.T, r, 16 * sizeof(double));
    res.iterations = (int)r[16];
    res.converged = r[17] != 0.0;
    res.fitness = r[18];
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
