/* ORACLE (test infrastructure only -- never the product path): CPU restatement
 * of the scanner node's scan registration for the parity tests of
 * pgo_gicp_align_batch (graphslam_amd/csrc/pgo_gicp.hip).
 *
 * Reference call site: /root/reference/src/scanner/src/scanner.cpp:35-74 (gicp():
 * pcl::GeneralizedIterativeClosestPoint<PointXYZ, PointXYZ>, default parameters,
 * align, hasConverged, getFitnessScore, getFinalTransformation) and
 * scanner.hpp (make_Delta, compute_covariance).  PCL itself is a third-party
 * dependency absent from /root/reference (ROS-era PCL 1.7 / 1.8, version not
 * pinned by the reference); its published GICP (Segal, Haehnel, Thrun 2009, as
 * implemented in pcl/registration/impl/gicp.hpp) is restated:
 *   computeCovariances  -> gicp_covariances
 *   computeTransformation -> the outer loop of orc_gicp_align
 *   getFitnessScore     -> gicp_fitness
 * with Gauss-Newton where PCL's estimateRigidTransformationBFGS runs BFGS (the
 * same per-iteration objective).  Brute-force neighbour searches, ties to the
 * lowest index.  PARITY UNPINNED against PCL: the reference holds no GICP
 * fixtures or outputs; the tests pin this restatement by known-motion recovery
 * on synthetic scans and compare the GPU with it.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define GICP_MAXK 32

/* squared distance in one fixed evaluation order (the GPU's too) */
static inline float dist2(float dx, float dy, float dz) { return fmaf(dz, dz, fmaf(dy, dy, dx * dx)); }

/* cyclic Jacobi on a symmetric 3x3: a -> diagonal, v columns = eigenvectors */
static void sym_eigen3(double a[3][3], double v[3][3]) {
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) v[i][j] = i == j ? 1.0 : 0.0;
  for (int sweep = 0; sweep < 12; sweep++) {
    const double off = fabs(a[0][1]) + fabs(a[0][2]) + fabs(a[1][2]);
    if (off < 1e-300) break;
    for (int pq = 0; pq < 3; pq++) {
      const int p = pq == 2 ? 1 : 0, q = pq == 0 ? 1 : 2;
      if (fabs(a[p][q]) < 1e-300) continue;
      const double theta = (a[q][q] - a[p][p]) / (2.0 * a[p][q]);
      const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
      const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
      for (int k = 0; k < 3; k++) {
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

/* computeCovariances: k nearest neighbours in the same cloud (the point itself
 * included), their covariance (1/k sum p p^T - mean mean^T), eigenvalues
 * replaced by (1, 1, eps) largest first.  cov: 6 per point (00 01 02 11 12 22). */
static void gicp_covariances(const float* P, int n, int k, double eps, double* cov) {
  for (int p = 0; p < n; p++) {
    const float* q = P + 3 * p;
    float bd[GICP_MAXK];
    int bi[GICP_MAXK];
    for (int t = 0; t < k; t++) {
      bd[t] = INFINITY;
      bi[t] = -1;
    }
    for (int j = 0; j < n; j++) {
      const float* r = P + 3 * j;
      const float d = dist2(r[0] - q[0], r[1] - q[1], r[2] - q[2]);
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
      const float* r = P + 3 * bi[t];
      const double x[3] = {r[0], r[1], r[2]};
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
    int o[3] = {0, 1, 2};
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
      for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) c[a][b] += w * v[a][o[kk]] * v[b][o[kk]];
    }
    double* out = cov + 6 * (size_t)p;
    out[0] = c[0][0]; out[1] = c[0][1]; out[2] = c[0][2]; out[3] = c[1][1]; out[4] = c[1][2]; out[5] = c[2][2];
  }
}

static void inv3(const double a[3][3], double r[3][3]) {
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

/* nearest target point of q (float distances, ties to the lowest index) */
static int nearest(const float* Q, int nq, const double w[3], float* best_out) {
  const float q0 = (float)w[0], q1 = (float)w[1], q2 = (float)w[2];
  float best = INFINITY;
  int bj = -1;
  for (int j = 0; j < nq; j++) {
    const float d = dist2(Q[3 * j] - q0, Q[3 * j + 1] - q1, Q[3 * j + 2] - q2);
    if (d < best) {
      best = d;
      bj = j;
    }
  }
  *best_out = best;
  return bj;
}

static void apply(const double T[12], const float* p, double w[3]) {
  for (int r = 0; r < 3; r++) w[r] = T[3 * r] * p[0] + T[3 * r + 1] * p[1] + T[3 * r + 2] * p[2] + T[9 + r];
}

/* One registration.  T (12: R row-major | t) holds the guess on entry and the
 * result on return; out[0] iterations, out[1] converged, out[2] fitness, out[3]
 * optimiser steps in total. */
int orc_gicp_align(const float* S, int ns, const float* Q, int nq, int k, double eps, int max_it, int max_inner,
                   double max_dist, double trans_eps, double rot_eps, double* T, double* out) {
  if (ns < 1 || nq < 1 || k < 1 || k > GICP_MAXK) return -1;
  double* cs = malloc(sizeof(double) * 6 * ns);
  double* ct = malloc(sizeof(double) * 6 * nq);
  double* M = malloc(sizeof(double) * 6 * ns);
  int* nn = malloc(sizeof(int) * ns);
  if (!cs || !ct || !M || !nn) {
    free(cs); free(ct); free(M); free(nn);
    return -2;
  }
  gicp_covariances(S, ns, k, eps, cs);
  gicp_covariances(Q, nq, k, eps, ct);
  const double thr2 = max_dist * max_dist;
  int it = 0, conv = 0, inner_total = 0;
  while (!conv) {
    /* correspondences and Mahalanobis matrices at the current T */
    for (int i = 0; i < ns; i++) {
      double w[3];
      float best;
      apply(T, S + 3 * i, w);
      const int j = nearest(Q, nq, w, &best);
      nn[i] = -1;
      if (!(j >= 0 && (double)best < thr2)) continue;
      nn[i] = j;
      const double* a = cs + 6 * i;
      const double* b = ct + 6 * j;
      const double C[3][3] = {{a[0], a[1], a[2]}, {a[1], a[3], a[4]}, {a[2], a[4], a[5]}};
      const double Ct[3][3] = {{b[0], b[1], b[2]}, {b[1], b[3], b[4]}, {b[2], b[4], b[5]}};
      double RC[3][3], Sm[3][3], Mi[3][3];
      for (int x = 0; x < 3; x++)
        for (int y = 0; y < 3; y++) RC[x][y] = T[3 * x] * C[0][y] + T[3 * x + 1] * C[1][y] + T[3 * x + 2] * C[2][y];
      for (int x = 0; x < 3; x++)
        for (int y = 0; y < 3; y++)
          Sm[x][y] = RC[x][0] * T[3 * y] + RC[x][1] * T[3 * y + 1] + RC[x][2] * T[3 * y + 2] + Ct[x][y];
      inv3(Sm, Mi);
      double* mo = M + 6 * i;
      mo[0] = Mi[0][0]; mo[1] = Mi[0][1]; mo[2] = Mi[0][2]; mo[3] = Mi[1][1]; mo[4] = Mi[1][2]; mo[5] = Mi[2][2];
    }
    double Tprev[12];
    memcpy(Tprev, T, sizeof(Tprev));
    /* minimise (1/n) sum d^T M d: Gauss-Newton, left perturbation T <- exp(dw, dt) T */
    for (int inner = 0; inner < max_inner; inner++) {
      inner_total++;
      double acc[28] = {0};
      for (int i = 0; i < ns; i++) {
        if (nn[i] < 0) continue;
        double w[3];
        apply(T, S + 3 * i, w);
        const float* qt = Q + 3 * nn[i];
        const double d[3] = {w[0] - qt[0], w[1] - qt[1], w[2] - qt[2]};
        const double* mi = M + 6 * i;
        const double Mm[3][3] = {{mi[0], mi[1], mi[2]}, {mi[1], mi[3], mi[4]}, {mi[2], mi[4], mi[5]}};
        const double J[3][6] = {{0, w[2], -w[1], 1, 0, 0}, {-w[2], 0, w[0], 0, 1, 0}, {w[1], -w[0], 0, 0, 0, 1}};
        double MJ[3][6], Md[3];
        for (int x = 0; x < 3; x++) {
          Md[x] = Mm[x][0] * d[0] + Mm[x][1] * d[1] + Mm[x][2] * d[2];
          for (int y = 0; y < 6; y++) MJ[x][y] = Mm[x][0] * J[0][y] + Mm[x][1] * J[1][y] + Mm[x][2] * J[2][y];
        }
        int q = 0;
        for (int x = 0; x < 6; x++)
          for (int y = x; y < 6; y++) acc[q++] += J[0][x] * MJ[0][y] + J[1][x] * MJ[1][y] + J[2][x] * MJ[2][y];
        for (int x = 0; x < 6; x++) acc[21 + x] += J[0][x] * Md[0] + J[1][x] * Md[1] + J[2][x] * Md[2];
        acc[27] += 1.0;
      }
      double A[6][6], b[6], x[6] = {0, 0, 0, 0, 0, 0};
      int q = 0, ok = acc[27] >= 3;
      for (int r = 0; r < 6; r++)
        for (int c = r; c < 6; c++) A[r][c] = A[c][r] = acc[q++];
      for (int r = 0; r < 6; r++) b[r] = -acc[21 + r];
      double inv[6];   /* reciprocal pivots (the GPU's arithmetic) */
      for (int kk = 0; kk < 6; kk++) {
        double s = A[kk][kk];
        for (int j = 0; j < kk; j++) s -= A[kk][j] * A[kk][j];
        ok = ok && s > 0;
        inv[kk] = 1.0 / sqrt(ok ? s : 1.0);
        for (int i = kk + 1; i < 6; i++) {
          double v = A[i][kk];
          for (int j = 0; j < kk; j++) v -= A[i][j] * A[kk][j];
          A[i][kk] = v * inv[kk];
        }
      }
      if (!ok) break;
      for (int i = 0; i < 6; i++) {
        double v = b[i];
        for (int j = 0; j < i; j++) v -= A[i][j] * x[j];
        x[i] = v * inv[i];
      }
      for (int i = 5; i >= 0; i--) {
        double v = x[i];
        for (int j = i + 1; j < 6; j++) v -= A[j][i] * x[j];
        x[i] = v * inv[i];
      }
      const double th = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
      double E[3][3];
      if (th < 1e-12) {
        E[0][0] = 1; E[0][1] = -x[2]; E[0][2] = x[1];
        E[1][0] = x[2]; E[1][1] = 1; E[1][2] = -x[0];
        E[2][0] = -x[1]; E[2][1] = x[0]; E[2][2] = 1;
      } else {
        const double ith = 1.0 / th, k0 = x[0] * ith, k1 = x[1] * ith, k2 = x[2] * ith, c = cos(th), s = sin(th),
                     v = 1 - c;
        E[0][0] = c + k0 * k0 * v; E[0][1] = k0 * k1 * v - k2 * s; E[0][2] = k0 * k2 * v + k1 * s;
        E[1][0] = k1 * k0 * v + k2 * s; E[1][1] = c + k1 * k1 * v; E[1][2] = k1 * k2 * v - k0 * s;
        E[2][0] = k2 * k0 * v - k1 * s; E[2][1] = k2 * k1 * v + k0 * s; E[2][2] = c + k2 * k2 * v;
      }
      double Tn[12];
      for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) Tn[3 * r + c] = E[r][0] * T[c] + E[r][1] * T[3 + c] + E[r][2] * T[6 + c];
        Tn[9 + r] = E[r][0] * T[9] + E[r][1] * T[10] + E[r][2] * T[11] + x[3 + r];
      }
      memcpy(T, Tn, sizeof(Tn));
      double step = 0;
      for (int i = 0; i < 6; i++) step = fmax(step, fabs(x[i]));
      if (step < 1e-12) break;
    }
    it++;
    /* PCL's test: the largest element change of T, rotation entries scaled by
     * 1/rotation_epsilon, translation by 1/transformation_epsilon, below 1 */
    double delta = 0;
    for (int q = 0; q < 12; q++) delta = fmax(delta, (q < 9 ? 1.0 / rot_eps : 1.0 / trans_eps) * fabs(Tprev[q] - T[q]));
    conv = it >= max_it || delta < 1.0;
  }
  /* getFitnessScore(): mean squared nearest-target distance of the transformed source */
  double fit = 0;
  for (int i = 0; i < ns; i++) {
    double w[3];
    float best;
    apply(T, S + 3 * i, w);
    (void)nearest(Q, nq, w, &best);
    fit += best;
  }
  out[0] = it;
  out[1] = 1.0;
  out[2] = fit / ns;
  out[3] = inner_total;
  free(cs); free(ct); free(M); free(nn);
  return 0;
}

/* the covariances alone (tests of computeCovariances) */
int orc_gicp_covariances(const float* P, int n, int k, double eps, double* cov) {
  if (n < 1 || k < 1 || k > GICP_MAXK) return -1;
  gicp_covariances(P, n, k, eps, cov);
  return 0;
}
