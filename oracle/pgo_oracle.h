/*
 * ORACLE -- test infrastructure only (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  Never linked into or called by the product library.
 *
 * C restatement of the reference's optimiser call
 *   gtsam::LevenbergMarquardtOptimizer(graph, initial).optimize()
 *   (/root/reference/src/graph/src/graph.cpp:119)
 * on the Pose2 prior + between factor graph built by graph.cpp:27-113.
 * GTSAM is not vendored, not installed and not version-pinned
 * (src/graph/CMakeLists.txt:9), so the GTSAM 4.0.x semantics are restated from
 * its published algorithm (see pgo_oracle.c and oracle/pgo_numpy.py headers).
 * Parity status vs GTSAM itself: UNPINNED (no reference fixtures exist); pinned
 * by known-answer graphs, finite-difference Jacobians and agreement with the
 * independent numpy/scipy twin oracle/pgo_numpy.py.
 */
#ifndef PGO_ORACLE_H
#define PGO_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_OK 0
#define ORC_E_ARG (-1)
#define ORC_E_BAD_COV (-3)
#define ORC_E_INDETERMINANT (-5)
#define ORC_E_NONFINITE (-6)
#define ORC_E_NOMEM (-9)

typedef struct {
  int max_iterations;          /* 100   */
  double relative_error_tol;   /* 1e-5  */
  double absolute_error_tol;   /* 1e-5  */
  double error_tol;            /* 0     */
  double lambda_initial;       /* 1e-5  */
  double lambda_factor;        /* 10    */
  double lambda_upper_bound;   /* 1e5   */
  double lambda_lower_bound;   /* 0     */
  double min_model_fidelity;   /* 1e-3  */
  int use_fixed_lambda_factor; /* 1     */
  int algorithm;               /* 0 = Levenberg-Marquardt, 1 = Gauss-Newton */
  int max_outer;               /* >0: stop after this many linearisations (bounded CPU sample) */
} orc_params;

typedef struct {
  int status;
  int iterations;        /* accepted steps (GTSAM's iterations()) */
  int inner_iterations;  /* lambda tries / GN steps */
  int linearizations;
  double initial_error;
  double final_error;
  double t_total, t_linearize, t_factor, t_solve, t_error; /* seconds */
  double factor_flops;   /* flops of one numeric factorisation */
  double nnz_l;          /* scalar nonzeros of L */
  int nsuper;
  double t_symbolic;
} orc_stats;

/* edges: 0-based pose indices; z/prior poses as (x, y, theta); covariances
 * row-major 3x3 (Pose2DWithCovariance.covariance, graph.hpp:45-58). */
void *orc_create(int n, int ne, const int32_t *ei, const int32_t *ej, const double *ez,
                 const double *ecov, int np, const int32_t *pi, const double *pz,
                 const double *pcov, int *status);
/* the same with a caller-supplied fill-reducing ordering (order[k] = old
 * index of the k-th eliminated pose) instead of AMD; NULL: AMD */
void *orc_create_ordered(int n, int ne, const int32_t *ei, const int32_t *ej, const double *ez,
                         const double *ecov, int np, const int32_t *pi, const double *pz,
                         const double *pcov, const int32_t *order, int *status);
void orc_destroy(void *h);
void orc_default_params(orc_params *p);
/* OpenMP threads used by later calls (bench.py: 1 and all host cores) */
void orc_set_threads(int t);

/* Full optimisation from init (x,y,theta)[n]; writes out (x,y,theta)[n].
 * trace (optional): 7 doubles per lambda try / GN step:
 *   outer iteration, lambda, solved, linear cost change, new error, fidelity, accepted */
int orc_optimize(void *h, const double *init, const orc_params *p, double *out,
                 orc_stats *st, double *trace, int trace_cap, int *trace_len);

/* One linearisation at poses (x,y,theta): per-pose 3x3 diagonal block of H
 * (row-major, 9 doubles), per-edge off-diagonal block H_{ei,ej} = J1^T Omega
 * (row-major), gradient g = J^T Omega e (3 per pose), error = 0.5 sum e^T Omega e. */
int orc_linearize(void *h, const double *poses, double *hdiag, double *hoff, double *g,
                  double *err);

/* Solve (H + lambda I) delta = -g at poses with the sparse Cholesky. */
int orc_solve(void *h, const double *poses, double lambda, double *delta);

/* Supernode front sizes (scalar rows m, columns w) and supernodal parents; returns count. */
int orc_supernodes(void *h, int *m, int *w, int *parent);

/* 0.5 sum e^T Omega e at poses. */
double orc_error(void *h, const double *poses);

/* Omega for noiseModel::Gaussian::Covariance(cov) (GTSAM smart check).  0 / ORC_E_BAD_COV. */
int orc_information(const double *cov, double *omega);

/* closest_keyframe service, graph.cpp:146-178 (xy: n x 2 keyframe positions in
 * insertion order); index of the closest of the first n - skip, -1 if n <= skip */
int orc_closest_keyframe(int n, const double *xy, double qx, double qy, int skip, double *dist);

/* Scan registration (gicp_oracle.c; scanner.cpp:35-74): GICP of source S (ns
 * float xyz) to target Q (nq).  T: 12 doubles (R row-major | t), the guess on
 * entry and the result on return; out: iterations, converged, fitness,
 * optimiser steps.  0 / negative on bad arguments. */
int orc_gicp_align(const float *S, int ns, const float *Q, int nq, int k, double eps, int max_it, int max_inner,
                   double max_dist, double trans_eps, double rot_eps, double *T, double *out);
/* plane-regularised covariances (6 per point: 00 01 02 11 12 22) */
int orc_gicp_covariances(const float *P, int n, int k, double eps, double *cov);

#ifdef __cplusplus
}
#endif
#endif
