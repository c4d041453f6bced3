/* ORACLE self-test (test infrastructure only): drives every entry point of the
 * C restatement on small synthetic inputs so that a host AddressSanitizer /
 * UndefinedBehaviorSanitizer build (`make -C oracle sanitize`)
 * exercises its memory accesses: LM / GN optimisation (AMD and caller
 * ordering), linearisation, damped solve, error, supernodes, the information
 * matrix check, closest_keyframe and the scan registration.  Exit 0 when every
 * result is sane. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pgo_oracle.h"

static unsigned long long lcg = 88172645463325252ULL;
static double urand(void) {
  lcg = lcg * 6364136223846793005ULL + 1442695040888963407ULL;
  return (double)(lcg >> 11) / 9007199254740992.0;
}
static double nrand(void) { return sqrt(-2.0 * log(urand() + 1e-300)) * cos(6.283185307179586 * urand()); }

#define CHECK(c, msg)                              \
  do {                                             \
    if (!(c)) {                                    \
      fprintf(stderr, "selftest: %s\n", msg);      \
      return 1;                                    \
    }                                              \
  } while (0)

static int graph_checks(void) {
  enum { N = 400, LC = 80 };
  const int ne = (N - 1) + LC;
  int32_t *ei = malloc(sizeof(int32_t) * ne), *ej = malloc(sizeof(int32_t) * ne), pi[1] = {0};
  double *ez = malloc(sizeof(double) * 3 * ne), *ecov = malloc(sizeof(double) * 9 * ne);
  double *gt = malloc(sizeof(double) * 3 * N), *init = malloc(sizeof(double) * 3 * N), *out = malloc(sizeof(double) * 3 * N);
  double pz[3] = {0, 0, 0}, pcov[9] = {0.01, 0, 0, 0, 0.01, 0, 0, 0, 0.01};
  for (int i = 0; i < N; i++) {   /* a spiral walk */
    gt[3 * i] = 10 * cos(0.05 * i) * (1 + 0.002 * i);
    gt[3 * i + 1] = 10 * sin(0.05 * i) * (1 + 0.002 * i);
    gt[3 * i + 2] = atan2(sin(0.05 * i + 1.5707963), cos(0.05 * i + 1.5707963));
  }
  for (int e = 0; e < ne; e++) {
    const int a = e < N - 1 ? e : (int)(urand() * (N - 20)) + 15, b = e < N - 1 ? e + 1 : a - 10 - (int)(urand() * 5);
    ei[e] = a;
    ej[e] = b;
    const double c = cos(gt[3 * a + 2]), s = sin(gt[3 * a + 2]), dx = gt[3 * b] - gt[3 * a], dy = gt[3 * b + 1] - gt[3 * a + 1];
    ez[3 * e] = c * dx + s * dy + 0.02 * nrand();
    ez[3 * e + 1] = -s * dx + c * dy + 0.02 * nrand();
    ez[3 * e + 2] = atan2(sin(gt[3 * b + 2] - gt[3 * a + 2]), cos(gt[3 * b + 2] - gt[3 * a + 2])) + 0.005 * nrand();
    const double cv[9] = {4e-4, 1e-5, 0, 1e-5, 4e-4, 0, 0, 0, 2.5e-5};
    memcpy(ecov + 9 * e, cv, sizeof(cv));
  }
  for (int i = 0; i < 3 * N; i++) init[i] = gt[i] + 0.3 * nrand();
  int st = 0;
  void *h = orc_create(N, ne, ei, ej, ez, ecov, 1, pi, pz, pcov, &st);
  CHECK(h && st == ORC_OK, "orc_create");
  orc_params p;
  orc_default_params(&p);
  orc_stats s;
  double trace[7 * 256];
  int tl = 0;
  CHECK(orc_optimize(h, init, &p, out, &s, trace, 256, &tl) >= 0, "orc_optimize");
  CHECK(s.final_error < s.initial_error && tl > 0, "LM did not decrease the error");
  p.algorithm = 1;
  p.max_outer = 3;
  CHECK(orc_optimize(h, init, &p, out, &s, NULL, 0, NULL) >= 0, "GN");
  double *hd = malloc(sizeof(double) * 9 * N), *ho = malloc(sizeof(double) * 9 * ne), *g = malloc(sizeof(double) * 3 * N);
  double err = 0;
  CHECK(orc_linearize(h, init, hd, ho, g, &err) == ORC_OK && err > 0, "orc_linearize");
  CHECK(fabs(orc_error(h, init) - err) <= 1e-9 * err, "orc_error");
  double *delta = malloc(sizeof(double) * 3 * N);
  CHECK(orc_solve(h, init, 1e-3, delta) == ORC_OK, "orc_solve");
  int *m = malloc(sizeof(int) * 3 * N), *w = malloc(sizeof(int) * 3 * N), *par = malloc(sizeof(int) * 3 * N);
  CHECK(orc_supernodes(h, m, w, par) > 0, "orc_supernodes");
  orc_destroy(h);
  int32_t *order = malloc(sizeof(int32_t) * N);
  for (int i = 0; i < N; i++) order[i] = N - 1 - i;
  h = orc_create_ordered(N, ne, ei, ej, ez, ecov, 1, pi, pz, pcov, order, &st);
  CHECK(h && st == ORC_OK, "orc_create_ordered");
  orc_default_params(&p);
  p.max_outer = 2;
  CHECK(orc_optimize(h, init, &p, out, &s, NULL, 0, NULL) >= 0, "ordered optimize");
  orc_destroy(h);
  double om[9], bad[9] = {1, 2, 0, 2, 1, 0, 0, 0, 1};
  CHECK(orc_information(pcov, om) == ORC_OK && fabs(om[0] - 100) < 1e-9, "information");
  CHECK(orc_information(bad, om) == ORC_E_BAD_COV, "non-PD covariance accepted");
  double *xy = malloc(sizeof(double) * 2 * N), dist = 0;
  for (int i = 0; i < N; i++) {
    xy[2 * i] = gt[3 * i];
    xy[2 * i + 1] = gt[3 * i + 1];
  }
  CHECK(orc_closest_keyframe(N, xy, xy[0], xy[1], 10, &dist) == 0 && dist == 0, "closest_keyframe");
  CHECK(orc_closest_keyframe(5, xy, 0, 0, 10, &dist) == -1, "closest_keyframe skip");
  free(ei); free(ej); free(ez); free(ecov); free(gt); free(init); free(out); free(hd); free(ho); free(g);
  free(delta); free(m); free(w); free(par); free(order); free(xy);
  return 0;
}

static int gicp_checks(void) {
  enum { NP = 300 };
  float *S = malloc(sizeof(float) * 3 * NP), *Q = malloc(sizeof(float) * 3 * NP);
  for (int i = 0; i < NP; i++) {   /* scattered points (no sliding directions) */
    S[3 * i] = (float)(5 * urand());
    S[3 * i + 1] = (float)(5 * urand());
    S[3 * i + 2] = 0.f;
  }
  const double a = 0.05, c = cos(a), s = sin(a), tx = 0.2, ty = -0.1;
  for (int i = 0; i < NP; i++) {
    Q[3 * i] = (float)(c * S[3 * i] - s * S[3 * i + 1] + tx);
    Q[3 * i + 1] = (float)(s * S[3 * i] + c * S[3 * i + 1] + ty);
    Q[3 * i + 2] = 0.f;
  }
  double T[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0}, out[4];
  CHECK(orc_gicp_align(S, NP, Q, NP, 20, 1e-3, 200, 20, 5.0, 5e-4, 2e-3, T, out) == 0, "gicp");
  if (!(fabs(T[9] - tx) < 1e-5 && fabs(T[10] - ty) < 1e-5 && fabs(T[3] - s) < 1e-5))
    fprintf(stderr, "T %g %g %g it %g fit %g\n", T[9], T[10], T[3], out[0], out[2]);
  CHECK(fabs(T[9] - tx) < 1e-5 && fabs(T[10] - ty) < 1e-5 && fabs(T[3] - s) < 1e-5, "gicp motion");
  double *cov = malloc(sizeof(double) * 6 * NP);
  CHECK(orc_gicp_covariances(S, 7, 20, 1e-3, cov) == 0, "gicp covariances (k > n)");
  CHECK(orc_gicp_align(S, 1, Q, 1, 20, 1e-3, 5, 5, 5.0, 5e-4, 2e-3, T, out) == 0, "gicp single point");
  free(S); free(Q); free(cov);
  return 0;
}

int main(void) {
  orc_set_threads(2);
  if (graph_checks() || gicp_checks()) return 1;
  printf("selftest ok\n");
  return 0;
}
