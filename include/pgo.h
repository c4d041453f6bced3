/*
 * pgo.h -- C-ABI of the MI355X-native SE(2) pose-graph optimisation backend.
 *
 * Drop-in boundary for the one hot path of Sergimech/GraphSLAM: the src/graph
 * node's Levenberg-Marquardt solve over Pose2 prior + between factors, which
 * the reference performs in-process through GTSAM (/root/reference paths):
 *
 *   graph.cpp:58,86      initial.insert(Key, Pose2)             -> pgo_add_vertex
 *   graph.cpp:57         graph.add(PriorFactor<Pose2>(...))      -> pgo_add_prior
 *   graph.cpp:87-92,     graph.add(BetweenFactor<Pose2>(...))    -> pgo_add_edge
 *            106-111
 *   graph.cpp:45,83,103  noiseModel::Gaussian::Covariance(Q)     -> the cov[9] argument
 *   graph.hpp:45-58      covariance_to_eigen: row-major float64[9] -> same layout
 *   graph.cpp:119        LevenbergMarquardtOptimizer(graph, initial).optimize()
 *                                                                -> pgo_optimize
 *   graph.cpp:123-125    poses_opti.at<Pose2>(id).x()/y()/theta() -> pgo_get_pose(s)
 *   graph.cpp:130        initial = poses_opti (warm start)       -> in-place update
 *   graph.cpp:60,94,112  graph.nrFactors()                       -> pgo_num_factors
 *
 * Plain C types only: no exceptions, no torch types, caller buffers are
 * borrowed for the duration of a call.  Keys are 64-bit like gtsam::Key
 * (the reference's int8 ids, Factor.msg:1-2, wrap after 127).
 * A handle is single-threaded (like the reference's one ROS spinner,
 * graph.cpp:214); distinct handles are independent; each owns one HIP stream.
 */
#ifndef PGO_H
#define PGO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGO_ABI_VERSION 6   /* 6: pgo_stats.handoff_retries / transport / part_transport
                                 (round 6); 5: the hybrid mode's partition-group
                                 communicator, pgo_debug_poison_fronts */

/* ---- status codes (GTSAM exception each one replaces) -------------------- */
#define PGO_OK 0
#define PGO_E_ARG (-1)           /* null handle / bad size                          */
#define PGO_E_DUP_KEY (-2)       /* gtsam::ValuesKeyAlreadyExists  (Values::insert) */
#define PGO_E_NO_KEY (-3)        /* gtsam::ValuesKeyDoesNotExist   (Values::at, or a
                                    factor on a key never inserted, at optimize)    */
#define PGO_E_BAD_COV (-4)       /* covariance not positive definite (LLT failure)   */
#define PGO_E_INDETERMINANT (-5) /* gtsam::IndeterminantLinearSystemException (GN)  */
#define PGO_E_NONFINITE (-6)     /* non-finite input or error                       */
#define PGO_E_HIP (-7)           /* HIP runtime failure (pgo_last_error has text)   */
#define PGO_E_NO_DEVICE (-8)     /* no usable MI355X / HIP device                   */
#define PGO_E_NOMEM (-9)
#define PGO_E_BAD_EDGE (-10)     /* between factor with key1 == key2                */
#define PGO_E_COMM (-11)         /* inter-rank exchange failed (RCCL / host callback) */
#define PGO_E_NOT_ENOUGH (-12)   /* closest_keyframe: no more keyframes than `skip`
                                    (the service returns false, graph.cpp:170-171) */
#define PGO_NO_KEY UINT64_MAX    /* batched search: the query has no candidate      */
#define PGO_W_MAXITER 1          /* informational: stopped at max_iterations        */

/* ---- algorithms / solvers ------------------------------------------------ */
#define PGO_ALG_LM 0             /* gtsam::LevenbergMarquardtOptimizer (graph.cpp:119) */
#define PGO_ALG_GN 1             /* gtsam::GaussNewtonOptimizer                      */
#define PGO_SOLVER_PCG 0         /* block-Jacobi preconditioned CG on the 3x3 BSR H  */
#define PGO_SOLVER_CHOLESKY 1    /* supernodal multifrontal Cholesky on the GPU (exact,
                                    like GTSAM's multifrontal elimination)          */

typedef struct pgo_graph pgo_graph;

#define PGO_ORDERING_ND 0        /* multilevel nested dissection of the pose graph
                                    (default: balanced elimination tree, C3 half
                                    the flops of minimum degree)                   */
#define PGO_ORDERING_AMD 1       /* approximate minimum degree                       */

typedef struct {
  int device;        /* HIP device ordinal (default 0) */
  int ordering;      /* fill-reducing ordering of the Cholesky solver, computed once
                        per graph structure (GTSAM: COLAMD every solve) [PGO_ORDERING_ND] */
  int reserved[6];
} pgo_opts;

typedef struct {
  /* gtsam::NonlinearOptimizerParams (defaults in brackets) */
  int max_iterations;           /* [100]  */
  double relative_error_tol;    /* [1e-5] */
  double absolute_error_tol;    /* [1e-5] */
  double error_tol;             /* [0]    */
  /* gtsam::LevenbergMarquardtParams */
  double lambda_initial;        /* [1e-5] */
  double lambda_factor;         /* [10]   */
  double lambda_upper_bound;    /* [1e5]  */
  double lambda_lower_bound;    /* [0]    */
  double min_model_fidelity;    /* [1e-3] */
  int use_fixed_lambda_factor;  /* [1]    */
  int algorithm;                /* [PGO_ALG_LM] */
  /* linear solver (the GPU replacement for GTSAM's multifrontal Cholesky) */
  int linear_solver;            /* [PGO_SOLVER_CHOLESKY] */
  double pcg_relative_tol;      /* stop when r'M^-1 r <= tol^2 * r0'M^-1 r0 [1e-10] */
  int pcg_max_iterations;       /* [20000] */
  int pcg_check_interval;       /* iterations enqueued between convergence reads [32] */
  int max_outer;                /* >0: stop after this many linearisations [0] */
  int profile_every;            /* >0: time every k-th PCG SpMV launch and every
                                   linearisation with HIP events on the handle's
                                   stream (pgo_stats.kernel_*) [0] */
  int use_graphs;               /* replay the captured factor+solve hipGraph [1] */
  int lambda_lanes;             /* Cholesky LM: consecutive lambda tries solved in
                                   one batched factor + solve on this GPU (the plan
                                   holds a numeric workspace per lane; every launch
                                   carries the lanes as grid dimension y, so the
                                   latency-bound top of the elimination tree costs
                                   about one pass for all lanes).  Speculative
                                   lambda search (see pgo_comm_*): results are
                                   those of 1 lane bit for bit [1] */
  int multi_gpu;                /* with a communicator of size > 1 (pgo_comm_*):
                                   PGO_MULTI_SPECULATIVE -- every rank solves
                                   different lambda tries of GTSAM's sequence;
                                   PGO_MULTI_PARTITION -- every try's
                                   factorisation is split: each rank factors
                                   its subtrees of the elimination tree, the
                                   subtree roots' Schur complements are
                                   all-gathered (the boundary reduction) and
                                   the top separators' columns are dealt to
                                   the ranks (each factored panel broadcast by
                                   its rank); composes with lambda_lanes;
                                   PGO_MULTI_HYBRID -- both: the ranks form
                                   groups, each group splits every
                                   factorisation over its partition-group
                                   communicator (pgo_comm_init_*_part) and the
                                   groups run the speculative search over the
                                   main communicator (one rank of every group
                                   each) [PGO_MULTI_SPECULATIVE] */
} pgo_params;

#define PGO_MULTI_SPECULATIVE 0
#define PGO_MULTI_PARTITION 1
#define PGO_MULTI_HYBRID 2

typedef struct {
  int status;                   /* PGO_OK / PGO_W_MAXITER / error                 */
  int iterations;               /* accepted steps (gtsam iterations())            */
  int inner_iterations;         /* lambda tries (LM) / steps (GN)                 */
  int linearizations;
  double initial_error;         /* graph.error(initial) = 0.5 chi^2               */
  double final_error;
  long long pcg_iterations;     /* summed over all solves                          */
  double ms_total;              /* wall time inside pgo_optimize                   */
  double ms_upload;             /* host->device graph upload (0 when resident)     */
  double ms_linearize;          /* device time of linearisation kernels            */
  double ms_solve;              /* device time of PCG                              */
  double ms_update;             /* retract + error + model-decrease kernels        */
  double kernel_spmv_ms;        /* summed device time of the timed SpMV launches   */
  long long kernel_spmv_count;  /* number of timed SpMV launches                   */
  double kernel_linearize_ms;   /* summed device time of the linearisation kernel  */
  long long kernel_linearize_count;
  double kernel_syrk_ms;        /* summed device time of Schur-update (MFMA) launches
                                   of the profiled factorisations                  */
  long long kernel_syrk_count;  /* profiled factorisations                         */
  double syrk_flops;            /* Schur-update flops of one factorisation         */
  double factor_flops;          /* flops of one numeric factorisation              */
  long long kernel_syrk_launches; /* timed Schur-update launches (all profiled
                                   factorisations)                                  */
  /* multi-GPU speculative lambda search (pgo_comm_*; zero / 1 on one rank) */
  int lambda_rounds;            /* lambda rounds: one parallel try on every rank    */
  int ranks;                    /* ranks that took part                             */
  long long solves;             /* linear solves this rank performed (incl. the
                                   speculative tries GTSAM's sequence never reached) */
  double ms_comm;               /* wall time in the all-gathers and broadcasts      */
  /* profiled factorisations (profile_every > 0, eager launches): device time from
     the first to the last launch of chol_factor / of the triangular solves,
     summed; per-kernel detail in pgo_get_kernel_profile */
  double ms_factor_profiled;
  double ms_solve_profiled;
  int stop_reason;              /* PGO_STOP_* : why the outer loop ended          */
  /* graph-replayed factorisations (use_graphs, every unprofiled one): summed
     device time of the factorisation graphs and the algorithmic flops they
     performed (lanes x one factorisation's flops) */
  double ms_factor_graph;
  double factor_graph_flops;
  /* the solver's plan on this call (the per-registration re-solve): 0 reused,
     1 same fronts / new H assembly (appended factors inside the existing fill),
     2 re-planned on the previous ordering with the appended poses inserted,
     3 full analysis (first call, or too much appended), 4 appended poses
     added to the plan incrementally (eliminated last, rows added along their
     fill paths to the root; PGO_NO_PLAN_APPEND=1 disables); ms_plan its
     host+upload ms */
  int plan_update;
  double ms_plan;
  /* how the device graph was brought up to date on this call: 0 resident, 1
     full upload, 2 appended in place (new keyframes / factors after the
     previous ones: the live re-solve); its host+upload time is ms_upload */
  int upload_kind;
  /* factorisations re-run because an in-launch hand-off timed out (a workgroup
     starved on a time-sliced GPU: the poll gives up after
     PGO_HANDOFF_TIMEOUT_MS and the try is run once more before the optimize
     fails with PGO_E_HIP).  0 in a healthy run; the parity tests assert it. */
  int handoff_retries;
  /* the transport of the handle's communicators on this call: PGO_TRANSPORT_*
     (main communicator; part_transport: the hybrid's partition group) */
  int transport;
  int part_transport;
} pgo_stats;

#define PGO_TRANSPORT_NONE 0     /* no communicator (one rank)                     */
#define PGO_TRANSPORT_RCCL 1     /* RCCL over xGMI                                 */
#define PGO_TRANSPORT_HOST 2     /* the caller's host callbacks (gloo in tests)    */

/* pgo_stats.stop_reason.  GTSAM reports every one of these as convergence
   (an LM that gives up leaves the values unchanged, so checkConvergence sees a
   zero decrease); the library tells them apart. */
#define PGO_STOP_CONVERGED 0     /* checkConvergence: relative / absolute decrease, error tol */
#define PGO_STOP_LAMBDA_BOUND 1  /* LM gave up: lambda reached lambda_upper_bound, no step accepted */
#define PGO_STOP_MAX_ITER 2      /* max_iterations accepted steps                   */
#define PGO_STOP_MAX_OUTER 3     /* pgo_params.max_outer linearisations              */
#define PGO_STOP_SMALL_CHANGE 4  /* tryLambda: |cost change| < relative_error_tol * error */
#define PGO_STOP_ERROR 5         /* error status (singular GN system, HIP, comm)    */

/* ---- lifetime ------------------------------------------------------------ */
pgo_graph *pgo_create(const pgo_opts *opts);        /* NULL opts: device 0 */
void pgo_destroy(pgo_graph *g);
const char *pgo_last_error(const pgo_graph *g);
const char *pgo_status_string(int status);
int pgo_abi_version(void);
void pgo_default_params(pgo_params *p);

/* ---- graph construction (graph.cpp:27-113) ------------------------------- */
/* Values::insert(key, Pose2(x, y, theta)); duplicate key -> PGO_E_DUP_KEY */
int pgo_add_vertex(pgo_graph *g, uint64_t key, double x, double y, double theta);
int pgo_add_vertices(pgo_graph *g, size_t n, const uint64_t *keys, const double *xyt);
/* graph.add(PriorFactor<Pose2>(key, pose, Covariance(cov))), cov row-major 3x3 */
int pgo_add_prior(pgo_graph *g, uint64_t key, const double pose[3], const double cov[9]);
/* graph.add(BetweenFactor<Pose2>(k1, k2, z, Covariance(cov))) */
int pgo_add_edge(pgo_graph *g, uint64_t k1, uint64_t k2, const double z[3], const double cov[9]);
/* bulk form; cov_stride 9 = one covariance per edge, 0 = one shared covariance */
int pgo_add_edges(pgo_graph *g, size_t n, const uint64_t *k1, const uint64_t *k2,
                  const double *z, const double *cov, int cov_stride);

/* ---- optimisation (graph.cpp:119, write-back :122-130) ------------------- */
/* Runs the optimiser from the handle's current values and replaces them with
 * the result (the reference's `initial = poses_opti`).  NULL params: defaults. */
int pgo_optimize(pgo_graph *g, const pgo_params *params, pgo_stats *stats);

/* Per-iteration record of the last pgo_optimize: one row of 8
 * doubles per lambda try GTSAM's sequence reached (LM) or per step (GN):
 *   accepted steps so far (LM: before this try; GN: after the step), lambda,
 *   solved (1/0), linear model decrease -(g'd + d'H d / 2) (NaN: not solved /
 *   GN), error at the candidate (+inf: not evaluated), model fidelity,
 *   accepted (1/0), wall ms since pgo_optimize entry when the outcome was known.
 * The columns match the oracle's trace (oracle/pgo_oracle.h) plus the ms.
 * Returns the row count (rows beyond cap are not written). */
int pgo_get_trace(const pgo_graph *g, double *out, int cap);

/* Profiled factorisations of the last pgo_optimize (pgo_params.profile_every
 * > 0): per kernel family f (0 <= f < returned count, name from
 * pgo_kernel_family_name) out[5 f ..] = launches, summed device ms (dispatch
 * events), algorithmic flops, algorithmic HBM bytes, 0. */
int pgo_get_kernel_profile(const pgo_graph *g, double *out, int cap);
const char *pgo_kernel_family_name(int f);

/* ---- values access ------------------------------------------------------- */
int pgo_get_pose(pgo_graph *g, uint64_t key, double out[3]);           /* Values::at */
/* keys NULL: all poses in insertion order (out holds 3*n doubles) */
int pgo_get_poses(pgo_graph *g, size_t n, const uint64_t *keys, double *out);
/* Values::update: overwrite current values (keys NULL: insertion order) */
int pgo_set_poses(pgo_graph *g, size_t n, const uint64_t *keys, const double *xyt);
/* Device-side copy of the current values into a snapshot slot / back (no PCIe
 * traffic): re-run a solve from the same initial values (graph.cpp:130 keeps
 * `initial` around the same way). */
int pgo_save_values(pgo_graph *g);
int pgo_restore_values(pgo_graph *g);
size_t pgo_num_factors(const pgo_graph *g);   /* graph.nrFactors() */
size_t pgo_num_vertices(const pgo_graph *g);  /* initial.size()    */
/* graph.error(values) = 0.5 sum e^T Omega e at the current values (device). */
int pgo_error(pgo_graph *g, double *err);

/* ---- marginals ------------------------------------------
   gtsam::Marginals(graph, values).marginalCovariance(key) (graph.cpp:120,
   126-127, commented out in the reference; eigen_to_covariance graph.hpp:60-68):
   the 3x3 covariance of each pose in its tangent space (x, y, theta), i.e. the
   pose's block of H^-1 with H = J'Omega J linearised at the current values (no
   damping).  out: n x 9 doubles, row-major.  A singular H (a component without
   prior) returns PGO_E_INDETERMINANT, as GTSAM's Cholesky throws. */
int pgo_marginal_covariances(pgo_graph *g, size_t n, const uint64_t *keys, double *out);

/* ---- loop-closure candidate search -----------------------
   The closest_keyframe service (graph.cpp:146-178): among the vertices in
   insertion order except the last `skip` (keyframes_to_skip_in_loop_closing,
   graph.cpp:15, = 10), the one whose current (x, y) is nearest to (x, y):
   distance sqrt((x2-x1)^2 + (y2-y1)^2) as the reference forms it, ties to the
   earliest inserted.  Fewer than skip + 1 vertices -> PGO_E_NOT_ENOUGH. */
int pgo_closest_keyframe(pgo_graph *g, double x, double y, int skip, uint64_t *key, double *dist);
/* Batched: for every query key (vertex i in insertion order) the service's
   answer when that key was keyframes.back(): query = its current (x, y),
   candidates = the vertices inserted before it except the last skip - 1 of
   them (indices [0, i + 1 - skip)).  No candidate: key PGO_NO_KEY, dist +inf. */
int pgo_closest_keyframes(pgo_graph *g, size_t q, const uint64_t *query_keys, int skip, uint64_t *keys_out,
                          double *dist_out);
/* device time (ms) of the last scan / batch search kernel launch */
int pgo_debug_search_ms(pgo_graph *g, double *scan_ms, double *batch_ms);

/* ---- scan registration: Generalized-ICP -----------------
   The scanner node's gicp() (scanner/src/scanner.cpp:35-74):
   pcl::GeneralizedIterativeClosestPoint<PointXYZ, PointXYZ> with PCL's default
   parameters, setInputSource(current scan) / setInputTarget(keyframe scan),
   align(), hasConverged(), getFitnessScore(), getFinalTransformation(), then
   make_Delta and compute_covariance (scanner.hpp) and the keyframe rule
   (converged && fitness > converged_fitness_threshold = 0.1).  A batch of B
   independent registrations (pair b: source cloud b -> target cloud b) runs as
   one launch, one workgroup per registration.  Clouds are float xyz triplets,
   concatenated (src: sum(src_n) x 3, tgt: sum(tgt_n) x 3), 1 .. 4096 points
   each; guess: B x 16 row-major initial transforms (NULL = identity, as
   align(output) without a guess).  The optimiser restates PCL's GICP with
   Gauss-Newton where PCL runs BFGS (DESIGN.md "Scan registration"). */
typedef struct pgo_gicp pgo_gicp;
typedef struct {
  int max_iterations;                 /* 200   (GICP's max_iterations_) */
  int k_correspondences;              /* 20    neighbours per covariance, <= 32 */
  double gicp_epsilon;                /* 1e-3  smallest covariance eigenvalue */
  double max_correspondence_distance; /* 5     (squared: 25) */
  double transformation_epsilon;      /* 5e-4  translation-column change to stop */
  double rotation_epsilon;            /* 2e-3  rotation-element change to stop */
  int max_inner_iterations;           /* 20    optimiser steps per correspondence set */
} pgo_gicp_params;
typedef struct {
  double T[16];      /* getFinalTransformation(), row-major, source -> target frame */
  int converged;     /* hasConverged() (PCL sets it at max_iterations too) */
  int iterations;    /* correspondence rounds */
  double fitness;    /* getFitnessScore(): mean squared nearest-target distance */
  double delta[3];   /* make_Delta: T(0,3), T(1,3), atan(T(1,0) / T(0,0)) */
  double cov[9];     /* compute_covariance(0.1, 0.1, 0.1, delta), row-major */
  int keyframe;      /* converged && fitness > 0.1 (scanner.cpp:55-58) */
  int inner_iterations; /* optimiser steps over all rounds */
} pgo_gicp_result;
void pgo_gicp_default_params(pgo_gicp_params *p);
pgo_gicp *pgo_gicp_create(int device);
void pgo_gicp_destroy(pgo_gicp *h);
const char *pgo_gicp_last_error(const pgo_gicp *h);
int pgo_gicp_align_batch(pgo_gicp *h, int B, const float *src, const int *src_n, const float *tgt,
                         const int *tgt_n, const double *guess, const pgo_gicp_params *params,
                         pgo_gicp_result *out);
/* device time (ms) of the last batch (covariance + registration kernels) */
int pgo_gicp_debug_ms(const pgo_gicp *h, double *ms);

/* ---- multi-GPU: speculative lambda search ---------------------
   One process per GPU, every rank holding the same graph and values.  Where
   GTSAM's LM (graph.cpp:119) tries lambda, lambda*f, lambda*f^2, ... one after
   another until a try is accepted, the ranks of a communicator solve the next
   `size` tries of that sequence at once (rank r: the r-th), all-gather the
   outcomes (error, model decrease), apply GTSAM's accept rule in sequence order
   and take the first accepted candidate from the rank that computed it
   (broadcast of N poses).  Accepted steps, lambdas and values are bitwise those
   of the one-GPU run; the wall time of a linearisation drops from its number of
   lambda tries to ceil(tries / size) factorisations.
   Transports: RCCL over xGMI (pgo_comm_init_rccl; rank 0 makes the id with
   pgo_comm_unique_id and the caller distributes its bytes), or the caller's
   own host transport (pgo_comm_init_host).  Every rank must call pgo_optimize
   with the same params. */
typedef struct {
  void *ctx;
  int rank, size;
  /* out[size * bytes] = every rank's in[bytes], rank order; 0 on success */
  int (*allgather)(void *ctx, const void *in, void *out, size_t bytes);
  /* buf[bytes] of rank `root` to every rank, in place; 0 on success */
  int (*broadcast)(void *ctx, void *buf, size_t bytes, int root);
} pgo_host_comm;

/* ncclGetUniqueId; returns the id size in bytes (128) or < 0 */
int pgo_comm_unique_id(void *out, size_t cap);
/* ncclCommInitRank on the handle's device (collective: all ranks call it) */
int pgo_comm_init_rccl(pgo_graph *g, const void *unique_id, size_t id_bytes, int rank, int size);
int pgo_comm_init_host(pgo_graph *g, const pgo_host_comm *comm);
int pgo_comm_free(pgo_graph *g);
/* rank / size of the handle's communicator (0 / 1 without one) */
int pgo_comm_rank(const pgo_graph *g, int *rank, int *size);
/* PGO_MULTI_HYBRID: the partition group's communicator (the ranks that split
   one factorisation; collective over the group), RCCL or host transport; the
   main communicator then holds one rank of every group (the same position in
   each).  Set it up BEFORE the main communicator: a main init binds the
   group set up since the previous main init and frees an older one, so a
   main communicator replaced without pgo_comm_free never runs with a stale
   group.  A bound group of one rank makes PGO_MULTI_HYBRID the speculative
   search alone; none bound with a main communicator of > 1 rank ->
   PGO_E_ARG.  pgo_comm_free frees both. */
int pgo_comm_init_rccl_part(pgo_graph *g, const void *unique_id, size_t id_bytes, int rank, int size);
int pgo_comm_init_host_part(pgo_graph *g, const pgo_host_comm *comm);
int pgo_comm_part_rank(const pgo_graph *g, int *rank, int *size);
/* exchange check (no solve): all-gather of (rank, size, rank^2, 1) and a
   broadcast from rank size-1; PGO_OK when every rank saw the right data.  The
   host transport needs no GPU. */
int pgo_comm_selftest(pgo_graph *g);

/* ---- diagnostics (parity tests; device results at the current values) ---- */
/* H diagonal blocks (9 doubles row-major per vertex, insertion order), the
 * off-diagonal block H_{k1,k2} = J1^T Omega of every between factor (9 per
 * factor, insertion order), gradient g = J^T Omega e (3 per vertex), error. */
int pgo_debug_linearize(pgo_graph *g, double *hdiag, double *hoff, double *grad, double *err);
/* The same four outputs from the Cholesky-mode linearisation (owner blocks in
 * factor order, the path pgo_optimize takes with PGO_SOLVER_CHOLESKY). */
int pgo_debug_linearize_cholesky(pgo_graph *g, double *hdiag, double *hoff, double *grad, double *err);
/* y = (H + lambda I) x at the current linearisation (x, y: 3 per vertex) */
int pgo_debug_spmv(pgo_graph *g, double lambda, const double *x, double *y);
/* Diagnostics: device time of one replay of the captured factorisation graph
 * of `lanes` lambda lanes (lambda_l = 1e-5 10^l) at the current linearisation,
 * averaged over `reps` back-to-back replays (HIP events on the handle's
 * stream); PGO_ABLATE (families to leave out) applies at capture. */
int pgo_debug_factor_time(pgo_graph *g, int lanes, int reps, double *ms);
/* Diagnostics (tests): NaN into every element of the Cholesky workspace
 * (all lambda lanes) that a factorisation must write before it reads it --
 * the fronts' lower trapezoids, the frontal vectors, the diagonal inverses --
 * so a later optimize equals a clean run bit for bit only if no stale element
 * is ever read.  Needs the workspace (an optimize with the Cholesky solver). */
int pgo_debug_poison_fronts(pgo_graph *g);
/* delta = PCG solve of (H + lambda I) delta = -g at the current values */
int pgo_debug_solve(pgo_graph *g, double lambda, const pgo_params *params, double *delta,
                    int *pcg_iterations);
/* Host-only symbolic analysis of the current graph (no device needed):
 * out[0..11] = supernodes, levels, nnz(L), factor flops, Schur-update flops,
 * front doubles, launches per factorisation, launches per solve, max front,
 * trsm tasks, syrk tiles, small fronts; from out[16], 6 per level (leaves first):
 * fronts, max m, max 64-blocks, panel steps, small fronts, syrk tiles. */
int pgo_debug_plan(pgo_graph *g, double *out, int cap);
/* Host-only: the subtree partition the PGO_MULTI_PARTITION factorisation
 * uses over `size` ranks: owner[s] per supernode (rank, -1 = top front;
 * returns the supernode count, arrays filled up to cap) and out[0..size+1] =
 * per-rank subtree flops, then the top's flops; then (as cap allows)
 * out[size+1 .. 2 size+1] = per-rank flops with the distributed top (subtrees
 * + the rank's top columns + the top work every rank repeats) and
 * out[2 size+1] = that repeated work, out[2 size+2] = the exchange points
 * (panel broadcast rounds) per factorisation and out[2 size+3] = the doubles
 * they broadcast per lambda lane. */
int pgo_debug_partition(pgo_graph *g, int size, int *owner, double *out, int cap);
/* Host-only: the supernodal elimination tree (parent per supernode, -1 root);
 * returns the supernode count. */
int pgo_debug_parents(pgo_graph *g, int *parent, int cap);
/* Host-only: the Cholesky solver's fill-reducing ordering of the poses
 * (perm[k] = insertion index of the k-th eliminated pose), n = vertex count.
 * bench.py hands it to the CPU restatement so both factor the same fill. */
int pgo_debug_ordering(pgo_graph *g, int32_t *perm, size_t n);
/* per supernode of the same host-only plan: pivot columns w, rows m, level
   (height in the elimination tree); returns the supernode count (arrays are
   filled up to cap entries) or a negative status */
int pgo_debug_fronts(pgo_graph *g, int *w, int *m, int *level, int cap);

#ifdef __cplusplus
}
#endif
#endif /* PGO_H */
