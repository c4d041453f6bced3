// libpgo.so: host side of the C-ABI in include/pgo.h.
//
// Mirrors, call for call, what /root/reference/src/graph/src/graph.cpp does
// through GTSAM (insert / add / optimize / at / nrFactors), keeps the graph and
// its values resident in HBM between calls, and drives the device kernels of
// pgo_kernels.hip with GTSAM's Levenberg-Marquardt control logic
// (tryLambda / decreaseLambda / increaseLambda / checkConvergence, GTSAM 4.0
// defaults) running on host scalars read back once per lambda try.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <unordered_map>
#include <thread>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "pgo.h"
#include "pgo_chol.h"
#include "pgo_comm.h"
#include "pgo_search.h"
#include "pgo_device.h"

using pgo::DevGraph;

// Lambda lane l >= 1 of a batched factorisation (lane 0 is the handle's own
// buffers): the Cholesky plan holds a numeric workspace per lane and every
// launch of the factor + solve carries the lanes as grid dimension y, so L
// consecutive lambda tries cost one pass over the (mostly latency-bound)
// schedule.  Per lane: candidate values, reduction partials and scalars of its
// try; the linearisation (D, V, g) and the current values are shared.
struct Lane {
  double4* pose_cand = nullptr;
  double* part = nullptr;
  double* scal = nullptr;
};

struct Staging {
  char* buf = nullptr;
  size_t cap = 0, used = 0;
  hipEvent_t done = nullptr;                // recorded after a batch's copies (stage_end)
};

struct HostStructure {
  std::vector<int2> eij;           // device order
  std::vector<int> dorder;         // device factor -> user factor index
  std::vector<int> pv, row_ptr, slot_edge, slot_col, prior_ptr, porder;
  std::vector<int> uf;             // union-find parents over the vertices (gauge check)
  std::vector<int> erow, s1_ptr, s1pos;   // the Cholesky-mode sweep structure (upload_structure)
  std::vector<int> spare_rp, spare_sc, spare_se;   // the previous block-CSR arrays, reused by the next append
  bool gauge_free = false;
};

struct pgo_graph {
  int device = 0;
  std::string last_error;
  // ---- host copy of the factor graph (insertion order) ----
  std::unordered_map<uint64_t, int32_t> index;
  std::vector<uint64_t> keys;
  std::vector<double> xyt;                  // current values (x, y, theta)
  std::vector<uint64_t> ek1, ek2;
  std::vector<double> ez;                   // 3 per between factor
  std::vector<double> eom;                  // 6 per factor: O00 O01 O02 O11 O12 O22
  std::vector<uint64_t> pk;
  std::vector<double> pz, pom;
  // ---- device state ----
  bool hip_ready = false;
  bool dev_structure = false;               // device graph matches host graph
  bool dev_values = false;                  // device pose == host xyt
  bool host_values = true;                  // host xyt == device pose
  DevGraph d;
  std::vector<int> edge_slot0;              // side-0 slot of every between factor (user order)
  std::vector<int> h_slot_edge;             // host copy of slot_edge (owner bits)
  // the device slot_edge carries the Cholesky plan's owner bits (bind_plan);
  // after an in-place append its rows from the first changed one carry the
  // pre-plan codes instead (side 0 owns), so the two halves disagree until the
  // next bind_plan -- the PCG path (k_model_decrease counts `se & 2` slots)
  // re-uploads the whole array first (slot_codes_mixed)
  bool slot_codes_plan = false;
  bool slot_codes_mixed = false;
  // rows from bind_row0 on need their owner bits (re)computed by the next
  // bind_plan (in-place appends: the plan keeps the old poses' order, so the
  // earlier rows' bits and their factors' owner sides stand); h_eside the
  // owner side of every factor, as uploaded
  int bind_row0 = 0;
  std::vector<unsigned char> h_eside;
  // mirror_bound: h_slot_edge (and the device copy) carries the plan's owner
  // bits on every slot but new_slots (an append's, pre-plan codes): the next
  // bind_plan on the same order sets only those
  bool mirror_bound = false;
  std::vector<int> new_slots;
  bool gauge_free = false;                 // some connected component has no prior
  double* h_scal = nullptr;                 // pinned
  int* h_ctrl = nullptr;                    // pinned
  hipEvent_t ev[6] = {};
  static constexpr int kProfPairs = 64;     // sampled SpMV timings per read-back
  hipEvent_t pev[2 * kProfPairs] = {};
  int pk_iter[kProfPairs] = {};
  // ---- supernodal Cholesky (built on first use; structure-dependent) ----
  std::vector<int> h_row_ptr, h_slot_col;   // block-CSR pattern (old indices)
  pgo::CholPlan chol;
  int ordering = pgo::kOrderNd;             // fill-reducing ordering (pgo_opts.ordering)
  int part_size = 1;                        // subtree partition the plan must have (PGO_MULTI_PARTITION)
  bool plan_stale = false;                  // the graph changed since the plan was built (kept, see ensure_chol)
  size_t plan_edges = 0;                    // between factors (user order) the plan holds: later ones are new
  int plan_update = 0;                      // how the last ensure_chol refreshed it (pgo_stats.plan_update)
  double plan_ms = 0.0;
  pgo::ExchangeHook hook;                   // the partitioned factorisation's all-gathers (comm)
  bool chol_ready = false;
  bool handoff_timeout = false;             // the last factorisation's in-launch hand-off gave up (retried once)
  // profiled factorisations (pgo_params.profile_every): every launch timed
  std::vector<hipEvent_t> sev;              // event pairs, one per launch
  std::vector<int> sev_fam;
  std::vector<double> sev_flops, sev_bytes;
  std::vector<int> sev_grid, sev_tag;
  hipEvent_t fev[4] = {};                   // factor start / end, solve end (profiled factorisation)
  double fam_ms[pgo::kFamCount] = {}, fam_flops[pgo::kFamCount] = {}, fam_bytes[pgo::kFamCount] = {};
  long long fam_launches[pgo::kFamCount] = {};
  std::vector<double> trace;                // per lambda try / GN step of the last optimize (kTraceCols each)
  long long factorizations = 0;
  hipGraphExec_t fac_exec[9] = {};          // captured factorisation, per lane count (1: d.x path)
  hipGraphExec_t sol_exec[9] = {};          // captured triangular solves, per lane count
  // graphs of a plan an incremental update replaced: destroyed only at the next
  // capture or with the device state (a destruction costs ~10 ms, on the first
  // live registration after a full optimize otherwise; on this thread only --
  // destroying them on a helper thread raced with the workspace re-allocation)
  std::vector<hipGraphExec_t> stale_exec;
  int graph_eager[9] = {};                  // eager factorisations of this plan before the capture
  int eager_first = 0;                      // ... how many (8 after an incremental plan update, else 0)
  double* h_lam = nullptr;                  // pinned lambda staging
  Staging stage;                            // pinned upload staging (append_structure)
  // ---- multi-GPU speculative lambda search (pgo_comm_*) ----
  pgo::Comm comm;
  // the partition group's communicator of the hybrid mode (pgo_comm_init_*_part:
  // the ranks that split one factorisation; comm then links one rank of every
  // group for the speculative search), and the communicator the partitioned
  // factorisation exchanges over (set per optimize: pcomm in the hybrid mode,
  // else comm)
  pgo::Comm pcomm;
  pgo::Comm* part_comm = &comm;
  // pcomm belongs to the main communicator set up right after it (the order
  // multi_gpu.attach_hybrid uses): pcomm_fresh = set since the last main init;
  // a main init binds a fresh pcomm and frees a stale one (round 6: a main
  // communicator replaced without pgo_comm_free no longer keeps the old group's)
  bool pcomm_fresh = false, pcomm_bound = false;
  std::vector<Lane> lanes;                  // lanes 1..L-1 (speculative tries on this GPU)
  double* xb = nullptr;                     // [L x 3n] solutions of a batched factor + solve
  size_t xb_n = 0;                          // ... allocated for this many vertices (capacity)
  double* h_lanes = nullptr;                // pinned [48]: 4 scalars per lane, lambdas at 32, flags at 40
  hipEvent_t lin_done = nullptr;            // linearisation complete
  int lane_cap = 8;                         // 1 after a lane allocation failed (reset per plan)
  // ---- incremental appends (append_structure, the live re-solve) ----
  HostStructure hs;                         // the structure the device holds (host side)
  std::vector<double> h_Dc;                 // its per-row sums of side-1 Omega
  size_t cap_n = 0, cap_ne = 0;             // device capacities in vertices / factors
  bool dev_complete = false;                // the device holds hs exactly (appendable)
  int last_upload = 0;                      // 1 full upload, 2 append (diagnostics)
  bool saved_valid = false;                 // d.pose_saved holds a snapshot of this structure (pgo_save_values)
  // ---- closest-keyframe search scratch ----
  double* s_d = nullptr;                    // [kMaxBlocks + 1] partial / final distances
  int* s_i = nullptr;                       // [kMaxBlocks + 1] partial / final indices
  double* sb_d = nullptr;                   // batched: per-query distance, index, query pose index
  int* sb_i = nullptr;
  int* sb_q = nullptr;
  double* sbp_d = nullptr;                  // batched: per (chunk, query) partials
  int* sbp_i = nullptr;
  size_t sb_cap = 0, sbp_cap = 0;
  hipEvent_t sev_scan[2] = {}, sev_batch[2] = {};
  bool scan_timed = false, batch_timed = false;
};

namespace {
// roctx range over a host scope (rocprofv3 --marker-trace shows the LM
// structure: optimize > plan / linearisation > lambda rounds; a no-op without
// a profiler attached)
struct RoctxRange {
  explicit RoctxRange(const char* m) { roctxRangePush(m); }
  ~RoctxRange() { roctxRangePop(); }
  RoctxRange(const RoctxRange&) = delete;
  RoctxRange& operator=(const RoctxRange&) = delete;
};
}  // namespace

namespace {

constexpr int kProfLaunches = 4096;   // timed launches per profiled factorisation + solve
constexpr int kTraceCols = 8;         // pgo_get_trace row

int fail(pgo_graph* g, int code, const std::string& msg) {
  if (g) g->last_error = msg;
  return code;
}

#define HIP_TRY(g, expr)                                                                       \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess)                                                                      \
      return fail(g, PGO_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));            \
  } while (0)

// noiseModel::Gaussian::Covariance(Q) (graph.cpp:45,83,103) -> Omega upper 6.
// GTSAM's smart check: all |off-diagonal| <= 1e-9 -> Diagonal::Variances;
// otherwise Information(Q^-1) with R = LLT(Q^-1).matrixU(): the lower triangle
// of Q^-1 is what counts, mirrored.
int information(const double* q, double* om6) {
  for (int i = 0; i < 9; i++)
    if (!std::isfinite(q[i])) return PGO_E_BAD_COV;
  bool full = false;
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++)
      if (i != j && std::fabs(q[3 * i + j]) > 1e-9) full = true;
  if (!full) {
    for (int i = 0; i < 3; i++)
      if (!(q[4 * i] > 0.0)) return PGO_E_BAD_COV;
    om6[0] = 1.0 / q[0]; om6[1] = 0; om6[2] = 0;
    om6[3] = 1.0 / q[4]; om6[4] = 0;
    om6[5] = 1.0 / q[8];
    return PGO_OK;
  }
  const double a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5], g = q[6], h = q[7], k = q[8];
  const double A = e * k - f * h, B = -(d * k - f * g), C = d * h - e * g;
  const double det = a * A + b * B + c * C;
  if (!(std::fabs(det) > 0.0) || !std::isfinite(det)) return PGO_E_BAD_COV;
  // lower triangle of the inverse: (1,0)=B/det, (2,0)=C/det, (2,1)=-(a h - b g)/det
  const double l00 = A / det, l10 = B / det, l20 = C / det;
  const double l11 = (a * k - c * g) / det, l21 = -(a * h - b * g) / det, l22 = (a * e - b * d) / det;
  // LLT must succeed
  if (!(l00 > 0)) return PGO_E_BAD_COV;
  const double r00 = std::sqrt(l00), r10 = l10 / r00, r20 = l20 / r00;
  const double s11 = l11 - r10 * r10;
  if (!(s11 > 0)) return PGO_E_BAD_COV;
  const double r11 = std::sqrt(s11), r21 = (l21 - r20 * r10) / r11;
  if (!(l22 - r20 * r20 - r21 * r21 > 0)) return PGO_E_BAD_COV;
  om6[0] = l00; om6[1] = l10; om6[2] = l20; om6[3] = l11; om6[4] = l21; om6[5] = l22;
  return PGO_OK;
}


// The captured graphs are destroyed here, before the caller frees or
// re-allocates the memory they point to (destroying them on a helper thread
// while the workspaces were freed and re-allocated raced: an intermittent host
// segfault on rapid lane-count changes).  The callers have drained the stream.
void destroy_stale_graphs(pgo_graph* g) {
  for (hipGraphExec_t e : g->stale_exec) (void)hipGraphExecDestroy(e);
  g->stale_exec.clear();
}

// defer: keep the execs for destroy_stale_graphs (they are never launched again)
void drop_graphs(pgo_graph* g, bool defer = false) {
  for (int l = 0; l < 9; l++) {
    for (hipGraphExec_t* e : {&g->fac_exec[l], &g->sol_exec[l]}) {
      if (*e) {
        if (defer) g->stale_exec.push_back(*e);
        else (void)hipGraphExecDestroy(*e);
      }
      *e = nullptr;
    }
    g->graph_eager[l] = 0;
  }
  if (!defer) destroy_stale_graphs(g);
}

void free_lanes(pgo_graph* g) {
  if (g->d.stream) (void)hipStreamSynchronize(g->d.stream);
  for (Lane& ln : g->lanes) {
    void* ptrs[] = {ln.pose_cand, ln.part, ln.scal};
    for (void* q : ptrs)
      if (q) (void)hipFree(q);
  }
  g->lanes.clear();
  if (g->xb) (void)hipFree(g->xb);
  g->xb = nullptr;
  for (int l = 2; l < 9; l++)   // the batched graphs hold xb
    for (hipGraphExec_t* e : {&g->fac_exec[l], &g->sol_exec[l]}) {
      if (*e) (void)hipGraphExecDestroy(*e);
      *e = nullptr;
    }
}

void free_device(pgo_graph* g, bool keep_plan = false) {
  g->dev_complete = false;
  free_lanes(g);
  g->lane_cap = 8;
  DevGraph& d = g->d;
  void* ptrs[] = {d.eij, d.ez, d.eom, d.prior_ptr, d.prior_vtx, d.pz, d.pom, d.row_ptr, d.slot_edge, d.slot_col, d.V,
                  d.erow, d.brow, d.s1_ptr, d.s1pos, d.eside, d.Dc, d.W, d.D, d.g, d.pose, d.pose_cand, d.pose_saved, d.x, d.r, d.z, d.p, d.q, d.Minv, d.part, d.scal, d.ctrl};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  hipStream_t s = d.stream;
  d = DevGraph();
  d.stream = s;
  g->dev_structure = false;
  g->dev_values = false;
  drop_graphs(g);
  if (keep_plan && g->chol_ready) {   // the structure changed: ensure_chol decides what to keep
    g->plan_stale = true;
    return;
  }
  if (g->chol_ready) pgo::chol_free(g->chol);
  g->chol_ready = false;
}

int ensure_hip(pgo_graph* g) {
  if (g->hip_ready) return PGO_OK;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
    return fail(g, PGO_E_NO_DEVICE, "no HIP device available");
  if (g->device < 0 || g->device >= count) return fail(g, PGO_E_NO_DEVICE, "device ordinal out of range");
  HIP_TRY(g, hipSetDevice(g->device));
  HIP_TRY(g, hipStreamCreateWithFlags(&g->d.stream, hipStreamNonBlocking));
  HIP_TRY(g, hipHostMalloc((void**)&g->h_scal, 16 * sizeof(double), hipHostMallocDefault));
  HIP_TRY(g, hipHostMalloc((void**)&g->h_ctrl, 4 * sizeof(int), hipHostMallocDefault));
  HIP_TRY(g, hipHostMalloc((void**)&g->h_lam, sizeof(double), hipHostMallocDefault));
  HIP_TRY(g, hipHostMalloc((void**)&g->h_lanes, 48 * sizeof(double), hipHostMallocDefault));
  for (auto& e : g->ev) HIP_TRY(g, hipEventCreate(&e));
  for (auto& e : g->pev) HIP_TRY(g, hipEventCreate(&e));
  HIP_TRY(g, hipEventCreateWithFlags(&g->lin_done, hipEventDisableTiming));
  g->sev.resize(2 * kProfLaunches);
  g->sev_fam.resize(kProfLaunches);
  g->sev_flops.resize(kProfLaunches);
  g->sev_bytes.resize(kProfLaunches);
  g->sev_grid.resize(kProfLaunches);
  g->sev_tag.resize(kProfLaunches);
  for (auto& e : g->sev) HIP_TRY(g, hipEventCreate(&e));
  for (auto& e : g->fev) HIP_TRY(g, hipEventCreate(&e));
  g->hip_ready = true;
  return PGO_OK;
}

template <class T>
int dev_alloc(pgo_graph* g, T** p, size_t count) {
  HIP_TRY(g, hipMalloc((void**)p, std::max<size_t>(count, 1) * sizeof(T)));
  return PGO_OK;
}

template <class T>
int h2d(pgo_graph* g, T* dst, const T* src, size_t count) {
  if (count == 0) return PGO_OK;
  HIP_TRY(g, hipMemcpyAsync(dst, src, count * sizeof(T), hipMemcpyHostToDevice, g->d.stream));
  return PGO_OK;
}

// Host -> device through the handle's pinned staging buffer (a bump region per
// batch of copies; stage_reset after the stream has drained): the live
// re-solve's per-registration uploads at pinned speed
// a batch of staged copies: wait until the previous batch's copies have read
// the buffer, then refill it from the start; stage_end marks the batch
int stage_begin(pgo_graph* g, Staging& st) {
  if (st.done) HIP_TRY(g, hipEventSynchronize(st.done));
  else HIP_TRY(g, hipEventCreateWithFlags(&st.done, hipEventDisableTiming));
  st.used = 0;
  return PGO_OK;
}
int stage_end(pgo_graph* g, Staging& st) {
  HIP_TRY(g, hipEventRecord(st.done, g->d.stream));
  return PGO_OK;
}

template <class T>
int staged_h2d(pgo_graph* g, Staging& st, T* dst, const T* src, size_t count) {
  if (count == 0) return PGO_OK;
  const size_t bytes = count * sizeof(T), off = (st.used + 255) / 256 * 256;
  if (off + bytes > st.cap) return h2d(g, dst, src, count);   // (full: a pageable copy)
  std::memcpy(st.buf + off, src, bytes);
  st.used = off + bytes;
  HIP_TRY(g, hipMemcpyAsync(dst, st.buf + off, bytes, hipMemcpyHostToDevice, g->d.stream));
  return PGO_OK;
}

#define RC_TRY(expr)          \
  do {                        \
    int rc_ = (expr);         \
    if (rc_ != PGO_OK) return rc_; \
  } while (0)

// Host values -> device pose (Pose2(x, y, theta): Rot2::fromAngle), vertices
// [first, n) (the ones before stay as they are on the device)
int upload_values(pgo_graph* g, size_t first = 0) {
  const size_t n = g->keys.size();
  std::vector<double4> h(n > first ? n - first : 0);
  for (size_t i = first; i < n; i++) {
    const double th = g->xyt[3 * i + 2];
    h[i - first] = make_double4(g->xyt[3 * i], g->xyt[3 * i + 1], std::cos(th), std::sin(th));
  }
  RC_TRY(h2d(g, g->d.pose + first, h.data(), n - std::min(n, first)));
  HIP_TRY(g, hipStreamSynchronize(g->d.stream));
  g->dev_values = true;
  return PGO_OK;
}

// Device pose -> host values (Values::at<Pose2>(k).x()/y()/theta(), graph.cpp:123-125)
int download_values(pgo_graph* g) {
  if (g->host_values) return PGO_OK;
  // the device-resident vertices (vertices appended since keep their host values)
  const size_t n = std::min(g->keys.size(), (size_t)g->d.n);
  std::vector<double4> h(n);
  if (n) {
    HIP_TRY(g, hipMemcpyAsync(h.data(), g->d.pose, n * sizeof(double4), hipMemcpyDeviceToHost, g->d.stream));
    HIP_TRY(g, hipStreamSynchronize(g->d.stream));
  }
  for (size_t i = 0; i < n; i++) {
    g->xyt[3 * i] = h[i].x;
    g->xyt[3 * i + 1] = h[i].y;
    g->xyt[3 * i + 2] = std::atan2(h[i].w, h[i].z);
  }
  g->host_values = true;
  return PGO_OK;
}

// Build the device graph: resolve keys (GTSAM raises ValuesKeyDoesNotExist at
// optimize time for a factor on an unknown key), block-CSR slots, priors.
// Host-side structure of the graph (no HIP): resolved factor endpoints,
// block-CSR slots, priors by vertex, gauge freedom.

int build_structure(pgo_graph* g, HostStructure& H) {
  const int n = (int)g->keys.size();
  const int ne = (int)g->ek1.size();
  const int np = (int)g->pk.size();
  std::vector<int2> eij(ne);
  for (int e = 0; e < ne; e++) {
    auto a = g->index.find(g->ek1[e]), b = g->index.find(g->ek2[e]);
    if (a == g->index.end() || b == g->index.end()) {
      const uint64_t k = a == g->index.end() ? g->ek1[e] : g->ek2[e];
      return fail(g, PGO_E_NO_KEY, "between factor " + std::to_string(e) + " references key " +
                                       std::to_string(k) + " with no inserted value");
    }
    eij[e] = make_int2(a->second, b->second);
  }
  std::vector<int> pv(np);
  for (int q = 0; q < np; q++) {
    auto a = g->index.find(g->pk[q]);
    if (a == g->index.end())
      return fail(g, PGO_E_NO_KEY, "prior factor on key " + std::to_string(g->pk[q]) + " with no inserted value");
    pv[q] = a->second;
  }
  // device order of the factors: sorted by (ei, ej), so that the side-0 slots
  // of a row read consecutive factors (coalesced factor loads in k_linearize)
  std::vector<int> dorder(ne);
  for (int e = 0; e < ne; e++) dorder[e] = e;
  std::stable_sort(dorder.begin(), dorder.end(), [&](int a, int b) {
    return eij[a].x != eij[b].x ? eij[a].x < eij[b].x : eij[a].y < eij[b].y;
  });
  {
    std::vector<int2> t(ne);
    for (int e = 0; e < ne; e++) t[e] = eij[dorder[e]];
    eij.swap(t);
  }
  // block-CSR rows: every factor owns a slot in row ei (side 0) and row ej (side 1)
  const int ns = 2 * ne;
  std::vector<int> row_ptr(n + 1, 0);
  for (int e = 0; e < ne; e++) {
    row_ptr[eij[e].x + 1]++;
    row_ptr[eij[e].y + 1]++;
  }
  for (int i = 0; i < n; i++) row_ptr[i + 1] += row_ptr[i];
  std::vector<int> fillp(row_ptr.begin(), row_ptr.end() - 1);
  std::vector<int> slot_edge(ns), slot_col(ns);
  for (int e = 0; e < ne; e++) {   // owner: side 0 until a Cholesky plan re-assigns it
    int s0 = fillp[eij[e].x]++;
    slot_edge[s0] = (e << 2) | 2;
    slot_col[s0] = eij[e].y;
    int s1 = fillp[eij[e].y]++;
    slot_edge[s1] = (e << 2) | 1;
    slot_col[s1] = eij[e].x;
  }
  // order each row by column (locality of the x gathers)
  std::vector<std::pair<int, int>> tmp;
  for (int i = 0; i < n; i++) {
    const int b = row_ptr[i], en = row_ptr[i + 1];
    if (en - b < 2) continue;
    tmp.clear();
    for (int k = b; k < en; k++) tmp.emplace_back(slot_col[k], slot_edge[k]);
    std::sort(tmp.begin(), tmp.end());
    for (int k = b; k < en; k++) {
      slot_col[k] = tmp[k - b].first;
      slot_edge[k] = tmp[k - b].second;
    }
  }
  // connected components without a prior leave H singular (3-dof gauge):
  // GTSAM's Cholesky throws IndeterminantLinearSystemException there (GN);
  // LM's damping keeps it solvable.
  {
    std::vector<int>& uf = H.uf;
    uf.resize(n);
    for (int i = 0; i < n; i++) uf[i] = i;
    auto find = [&](int x) {
      while (uf[x] != x) x = uf[x] = uf[uf[x]];
      return x;
    };
    for (int e = 0; e < ne; e++) {
      const int a = find(eij[e].x), b = find(eij[e].y);
      if (a != b) uf[a] = b;
    }
    std::vector<char> anchored(n, 0);
    for (int q = 0; q < np; q++) anchored[find(pv[q])] = 1;
    g->gauge_free = false;
    for (int i = 0; i < n; i++)
      if (!anchored[find(i)]) g->gauge_free = true;
  }
  // priors CSR by vertex
  std::vector<int> prior_ptr(n + 1, 0);
  for (int q = 0; q < np; q++) prior_ptr[pv[q] + 1]++;
  for (int i = 0; i < n; i++) prior_ptr[i + 1] += prior_ptr[i];
  std::vector<int> porder(np);
  {
    std::vector<int> f(prior_ptr.begin(), prior_ptr.end() - 1);
    for (int q = 0; q < np; q++) porder[f[pv[q]]++] = q;
  }
  H.gauge_free = g->gauge_free;
  H.dorder = std::move(dorder);
  H.eij = std::move(eij);
  H.pv = std::move(pv);
  H.row_ptr = std::move(row_ptr);
  H.slot_edge = std::move(slot_edge);
  H.slot_col = std::move(slot_col);
  H.prior_ptr = std::move(prior_ptr);
  H.porder = std::move(porder);
  return PGO_OK;
}

int upload_structure(pgo_graph* g) {
  RC_TRY(ensure_hip(g));
  RC_TRY(download_values(g));
  HostStructure H;
  RC_TRY(build_structure(g, H));
  const int n = (int)g->keys.size();
  const int ne = (int)g->ek1.size();
  const int np = (int)g->pk.size();
  const int ns = 2 * ne;
  const auto& eij = H.eij;
  const auto& pv = H.pv;
  const auto& row_ptr = H.row_ptr;
  const auto& slot_edge = H.slot_edge;
  const auto& slot_col = H.slot_col;
  const auto& prior_ptr = H.prior_ptr;
  const auto& porder = H.porder;
  g->h_row_ptr = row_ptr;
  g->h_slot_col = slot_col;
  g->h_slot_edge = slot_edge;
  g->edge_slot0.assign(ne, -1);   // user factor -> its side-0 slot
  for (int k = 0; k < ns; k++)
    if ((slot_edge[k] & 1) == 0) g->edge_slot0[H.dorder[slot_edge[k] >> 2]] = k;
  std::vector<double4> hz(ne), hpz(np);
  std::vector<double2> hom(3 * (size_t)ne), hpom(3 * (size_t)np);
  for (int de = 0; de < ne; de++) {
    const int e = H.dorder[de];
    const double th = g->ez[3 * e + 2];
    hz[de] = make_double4(g->ez[3 * e], g->ez[3 * e + 1], std::cos(th), std::sin(th));
    const double* o = &g->eom[6 * (size_t)e];
    hom[3 * de] = make_double2(o[0], o[1]);
    hom[3 * de + 1] = make_double2(o[2], o[3]);
    hom[3 * de + 2] = make_double2(o[4], o[5]);
  }
  for (int t = 0; t < np; t++) {
    const int q = porder[t];
    const double th = g->pz[3 * q + 2];
    hpz[t] = make_double4(g->pz[3 * q], g->pz[3 * q + 1], std::cos(th), std::sin(th));
    const double* o = &g->pom[6 * (size_t)q];
    hpom[3 * t] = make_double2(o[0], o[1]);
    hpom[3 * t + 1] = make_double2(o[2], o[3]);
    hpom[3 * t + 2] = make_double2(o[4], o[5]);
  }
  // the values already resident stay bit for bit (no host atan2 -> cos / sin
  // round trip): vertices are append-only, so the first n_old keep their index
  // (freed on every exit path: an early error return below must not leak it)
  struct HipFree {
    void operator()(double4* p) const { (void)hipFree(p); }
  };
  std::unique_ptr<double4, HipFree> keep;
  const int n_old = g->dev_values && g->d.pose ? std::min(g->d.n, n) : 0;
  if (n_old > 0) {
    double4* k = nullptr;
    HIP_TRY(g, hipMalloc((void**)&k, sizeof(double4) * n_old));
    keep.reset(k);
    HIP_TRY(g, hipMemcpyAsync(keep.get(), g->d.pose, sizeof(double4) * n_old, hipMemcpyDeviceToDevice, g->d.stream));
  }
  free_device(g, true);
  DevGraph& d = g->d;
  d.n = n;
  d.ne = ne;
  d.np = np;
  d.nslots = ns;
  // room for appended vertices / factors (the live re-solve appends one
  // keyframe and a few factors per registration: append_structure)
  const size_t cn = (size_t)n + std::max<size_t>(1024, n / 8);
  const size_t ce = (size_t)ne + std::max<size_t>(4096, ne / 8), cs = 2 * ce;
  g->cap_n = cn;
  g->cap_ne = ce;
  {   // the appends' pinned staging (append_structure / bind_plan), sized for the
      // largest per-registration upload of this graph, allocated with the graph
    const size_t want = 8 * cs + 8 * ce + 80 * cn + ((size_t)1 << 20);
    if (g->stage.cap < want) {
      if (g->stage.done) HIP_TRY(g, hipEventSynchronize(g->stage.done));
      if (g->stage.buf) (void)hipHostFree(g->stage.buf);
      g->stage.buf = nullptr;
      g->stage.cap = 0;
      HIP_TRY(g, hipHostMalloc((void**)&g->stage.buf, want, hipHostMallocDefault));
      g->stage.cap = want;
    }
  }
  // lanes per row: smallest power of two >= mean degree, in [4, 32]
  const double mean_deg = n ? (double)ns / n : 0.0;
  d.G = 4;
  while (d.G < 32 && d.G < mean_deg) d.G *= 2;
  d.G1 = 4;
  while (d.G1 < 32 && d.G1 < (n ? (double)ne / n : 0.0)) d.G1 *= 2;
  // Cholesky-mode sweep structure: factors are sorted by (ei, ej), so the
  // side-0 factors of row i are the contiguous range [erow[i], erow[i+1]);
  // side-1 factors of row j take positions s1_ptr[j].. in device order (s1pos).  Dc[j] is
  // the (iteration-invariant) sum of Omega over row j's side-1 factors.
  std::vector<int> erow(n + 1, 0), s1_ptr(n + 1, 0), s1pos(ne);
  std::vector<double> Dc(6 * (size_t)n, 0.0);
  for (int e = 0; e < ne; e++) {
    erow[eij[e].x + 1]++;
    s1_ptr[eij[e].y + 1]++;
  }
  for (int i = 0; i < n; i++) {
    erow[i + 1] += erow[i];
    s1_ptr[i + 1] += s1_ptr[i];
  }
  {
    std::vector<int> f(s1_ptr.begin(), s1_ptr.end() - 1);
    for (int e = 0; e < ne; e++) {
      const int j = eij[e].y;
      s1pos[e] = f[j]++;
      const double* o = &g->eom[6 * (size_t)H.dorder[e]];
      for (int q = 0; q < 6; q++) Dc[6 * (size_t)j + q] += o[q];
    }
  }
  // k_linearize_own blocks: whole rows, greedily packed to <= kThreads side-0
  // factors and <= kThreads rows (a row with more factors is a block alone)
  std::vector<int> brow(1, 0);
  for (int r = 0; r < n;) {
    int r1 = r + 1;
    while (r1 < n && r1 - r < pgo::kThreads && erow[r1 + 1] - erow[r] <= pgo::kThreads) r1++;
    brow.push_back(r1);
    r = r1;
  }
  d.nlb = (int)brow.size() - 1;
  RC_TRY(dev_alloc(g, &d.brow, cn + 1));
  RC_TRY(h2d(g, d.brow, brow.data(), brow.size()));
  RC_TRY(dev_alloc(g, &d.erow, cn + 1));
  RC_TRY(dev_alloc(g, &d.s1_ptr, cn + 1));
  RC_TRY(dev_alloc(g, &d.s1pos, ce));
  RC_TRY(dev_alloc(g, &d.Dc, 6 * cn));
  RC_TRY(dev_alloc(g, &d.W, ce));
  RC_TRY(h2d(g, d.erow, erow.data(), n + 1));
  RC_TRY(h2d(g, d.s1_ptr, s1_ptr.data(), n + 1));
  RC_TRY(h2d(g, d.s1pos, s1pos.data(), ne));
  RC_TRY(h2d(g, d.Dc, Dc.data(), 6 * (size_t)n));
  RC_TRY(dev_alloc(g, &d.eij, ce));
  RC_TRY(dev_alloc(g, &d.ez, ce));
  RC_TRY(dev_alloc(g, &d.eom, 3 * ce));
  RC_TRY(dev_alloc(g, &d.prior_ptr, cn + 1));
  RC_TRY(dev_alloc(g, &d.prior_vtx, np));
  RC_TRY(dev_alloc(g, &d.pz, np));
  RC_TRY(dev_alloc(g, &d.pom, 3 * (size_t)np));
  RC_TRY(dev_alloc(g, &d.row_ptr, cn + 1));
  RC_TRY(dev_alloc(g, &d.slot_edge, cs));
  RC_TRY(dev_alloc(g, &d.slot_col, cs));
  RC_TRY(dev_alloc(g, &d.V, 9 * cs));
  RC_TRY(dev_alloc(g, &d.D, 6 * cn));
  RC_TRY(dev_alloc(g, &d.g, 3 * cn));
  RC_TRY(dev_alloc(g, &d.pose, cn));
  RC_TRY(dev_alloc(g, &d.pose_cand, cn));
  RC_TRY(dev_alloc(g, &d.x, 3 * cn));
  RC_TRY(dev_alloc(g, &d.r, 3 * cn));
  RC_TRY(dev_alloc(g, &d.z, 3 * cn));
  RC_TRY(dev_alloc(g, &d.p, 3 * cn));
  RC_TRY(dev_alloc(g, &d.q, 3 * cn));
  RC_TRY(dev_alloc(g, &d.Minv, 6 * cn));
  RC_TRY(dev_alloc(g, &d.part, (size_t)pgo::kMaxBlocks * pgo::kPartSlices));
  RC_TRY(dev_alloc(g, &d.scal, 16));
  RC_TRY(dev_alloc(g, &d.ctrl, 4));
  std::vector<int> pvs(np);
  for (int t = 0; t < np; t++) pvs[t] = pv[porder[t]];
  RC_TRY(h2d(g, d.eij, eij.data(), ne));
  RC_TRY(h2d(g, d.ez, hz.data(), ne));
  RC_TRY(h2d(g, d.eom, hom.data(), 3 * (size_t)ne));
  RC_TRY(h2d(g, d.prior_ptr, prior_ptr.data(), n + 1));
  RC_TRY(h2d(g, d.prior_vtx, pvs.data(), np));
  RC_TRY(h2d(g, d.pz, hpz.data(), np));
  RC_TRY(h2d(g, d.pom, hpom.data(), 3 * (size_t)np));
  RC_TRY(h2d(g, d.row_ptr, row_ptr.data(), n + 1));
  RC_TRY(h2d(g, d.slot_edge, slot_edge.data(), ns));
  g->slot_codes_plan = g->slot_codes_mixed = false;   // pre-plan codes throughout
  g->bind_row0 = 0;
  g->mirror_bound = false;
  g->new_slots.clear();
  g->chol.asm_bound = false;   // (a new device factor order: the plan's bound sources are void)
  RC_TRY(h2d(g, d.slot_col, slot_col.data(), ns));
  HIP_TRY(g, hipMemsetAsync(d.part, 0, sizeof(double) * pgo::kMaxBlocks * pgo::kPartSlices, d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  g->dev_structure = true;
  g->h_Dc = std::move(Dc);
  H.erow = std::move(erow);
  H.s1_ptr = std::move(s1_ptr);
  H.s1pos = std::move(s1pos);
  {   // room for in-place appends (append_structure), as the device arrays have
    const size_t rn = g->cap_n + 1, re = g->cap_ne, rs = 2 * g->cap_ne;
    H.eij.reserve(re);
    H.dorder.reserve(re);
    H.erow.reserve(rn);
    H.s1_ptr.reserve(rn);
    H.s1pos.reserve(re);
    H.prior_ptr.reserve(rn);
    H.uf.reserve(rn);
    g->edge_slot0.reserve(re);
    g->h_row_ptr.reserve(rn);
    g->h_slot_col.reserve(rs);
    g->h_slot_edge.reserve(rs);
    g->h_Dc.reserve(6 * rn);
  }
  g->hs = std::move(H);
  g->dev_complete = true;
  g->last_upload = 1;
  if (n_old > 0) {
    HIP_TRY(g, hipMemcpyAsync(d.pose, keep.get(), sizeof(double4) * n_old, hipMemcpyDeviceToDevice, d.stream));
    HIP_TRY(g, hipStreamSynchronize(d.stream));
  }
  return upload_values(g, n_old);
}

// Appended vertices and between factors (pgo_add_vertex / pgo_add_edge after
// an upload -- the live re-solve, graph.cpp:180-200) extend the device graph in
// place when the device holds the previous structure, no prior was added,
// capacities suffice and the new factors sort after the old ones in device
// order ((ei, ej): a new keyframe's odometry and loop closures do).  The host
// structure is updated in step (block-CSR rows merged, side-1 lists, row
// blocks); only the new factors, the per-row arrays and the slot arrays are
// uploaded.  Returns 1 when the full upload must run instead.
// fn(begin, end) over contiguous chunks of [0, n) on the planner's host threads
// (the live re-solve's per-registration host work; chunk results independent)
template <class F>
void host_parallel(int n, F&& fn) {
  static const int hw = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  const int nth = std::max(1, std::min(hw, n / 16384));
  pgo::plan_parallel(nth, [&](int t) { fn((int)((long long)n * t / nth), (int)((long long)n * (t + 1) / nth)); });
}

// PGO_PLAN_TIMING: phase times of the plan / append paths on stderr
struct PhaseTimer {
  const char* who;
  bool on = getenv("PGO_PLAN_TIMING") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  explicit PhaseTimer(const char* w) : who(w) {}
  void operator()(const char* what) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "%s %-14s %8.2f ms\n", who, what, std::chrono::duration<double, std::milli>(now - t).count());
    t = now;
  }
};

int append_structure(pgo_graph* g) {
  PhaseTimer phase("append_structure");
  DevGraph& d = g->d;
  HostStructure& H = g->hs;
  const int n_old = d.n, ne_old = d.ne;
  const int n = (int)g->keys.size(), ne = (int)g->ek1.size(), np = (int)g->pk.size();
  if (!g->dev_complete || !g->hip_ready || np != d.np || n < n_old || ne < ne_old || (n == n_old && ne == ne_old) ||
      (size_t)n > g->cap_n || (size_t)ne > g->cap_ne || (int)H.eij.size() != ne_old ||
      (int)H.erow.size() != n_old + 1 || (int)H.s1pos.size() != ne_old || getenv("PGO_NO_APPEND"))
    return 1;
  // the new factors, resolved and in device order
  std::vector<int> nd(ne - ne_old);
  std::vector<int2> nij(ne - ne_old);
  for (int e = ne_old; e < ne; e++) {
    auto a = g->index.find(g->ek1[e]), b = g->index.find(g->ek2[e]);
    if (a == g->index.end() || b == g->index.end()) return 1;   // the full path reports it
    nij[e - ne_old] = make_int2(a->second, b->second);
    nd[e - ne_old] = e;
  }
  {
    std::vector<int> o(nd.size());
    for (size_t q = 0; q < o.size(); q++) o[q] = (int)q;
    std::stable_sort(o.begin(), o.end(), [&](int a, int b) {
      return nij[a].x != nij[b].x ? nij[a].x < nij[b].x : nij[a].y < nij[b].y;
    });
    std::vector<int> nd2(nd.size());
    std::vector<int2> nij2(nij.size());
    for (size_t q = 0; q < o.size(); q++) {
      nd2[q] = nd[o[q]];
      nij2[q] = nij[o[q]];
    }
    nd.swap(nd2);
    nij.swap(nij2);
  }
  if (!nij.empty() && ne_old > 0) {
    const int2 last = H.eij.back(), f = nij.front();
    if (f.x < last.x || (f.x == last.x && f.y < last.y)) return 1;   // not an append in device order
  }
  phase("resolve");
  // host structure: device order, block-CSR rows (every row sorted by (column,
  // code) as build_structure sorts them, codes in their pre-plan form)
  H.eij.insert(H.eij.end(), nij.begin(), nij.end());
  H.dorder.insert(H.dorder.end(), nd.begin(), nd.end());
  std::vector<int> add(n, 0);
  for (const int2& ij : nij) {
    add[ij.x]++;
    add[ij.y]++;
  }
  const int ns = 2 * ne;
  // (into the previous append's arrays: their pages are mapped already;
  // every element is written below)
  std::vector<int>& rp = H.spare_rp;
  std::vector<int>& sc = H.spare_sc;
  std::vector<int>& se = H.spare_se;
  rp.resize(n + 1);
  sc.resize(ns);
  se.resize(ns);
  rp[0] = 0;
  for (int i = 0; i < n; i++) rp[i + 1] = rp[i] + (i < n_old ? H.row_ptr[i + 1] - H.row_ptr[i] : 0) + add[i];
  // the new slots (row, column, code), by row then (column, code): merged
  // into the old rows (sorted by (column, code), as build_structure sorts them)
  std::vector<int3> extra;
  extra.reserve(2 * nij.size());
  for (size_t q = 0; q < nij.size(); q++) {
    const int de = ne_old + (int)q;
    extra.push_back(make_int3(nij[q].x, nij[q].y, (de << 2) | 2));
    extra.push_back(make_int3(nij[q].y, nij[q].x, (de << 2) | 1));
  }
  std::sort(extra.begin(), extra.end(), [](const int3& a, const int3& b) {
    return a.x != b.x ? a.x < b.x : a.y != b.y ? a.y < b.y : a.z < b.z;
  });
  int prev = 0;   // rows [prev, r) copied whole (H.slot_edge holds pre-plan codes)
  auto copy_rows = [&](int r) {
    if (prev >= n_old) return;
    const int b = H.row_ptr[prev], e0 = H.row_ptr[std::min(r, n_old)];
    if (e0 > b) {
      std::copy(H.slot_col.begin() + b, H.slot_col.begin() + e0, sc.begin() + rp[prev]);
      std::copy(H.slot_edge.begin() + b, H.slot_edge.begin() + e0, se.begin() + rp[prev]);
    }
  };
  for (size_t q = 0; q < extra.size();) {
    const int i = extra[q].x;
    size_t q1 = q;
    while (q1 < extra.size() && extra[q1].x == i) q1++;
    copy_rows(i);
    const int b = i < n_old ? H.row_ptr[i] : 0, e0 = i < n_old ? H.row_ptr[i + 1] : 0;
    int o = rp[i], k = b;
    for (size_t t = q; t < q1; t++) {   // merge: old slots before an equal (column, code) stay first
      while (k < e0 && (H.slot_col[k] < extra[t].y || (H.slot_col[k] == extra[t].y && H.slot_edge[k] <= extra[t].z))) {
        sc[o] = H.slot_col[k];
        se[o++] = H.slot_edge[k++];
      }
      sc[o] = extra[t].y;
      se[o++] = extra[t].z;
    }
    for (; k < e0; k++) {
      sc[o] = H.slot_col[k];
      se[o++] = H.slot_edge[k];
    }
    prev = i + 1;
    q = q1;
  }
  copy_rows(n);
  H.row_ptr.swap(rp);
  H.slot_col.swap(sc);
  H.slot_edge.swap(se);
  // gauge: the new factors join components; anchored roots from the priors
  H.uf.resize(n);
  for (int i = n_old; i < n; i++) H.uf[i] = i;
  auto find = [&](int x) {
    while (H.uf[x] != x) x = H.uf[x] = H.uf[H.uf[x]];
    return x;
  };
  for (const int2& ij : nij) {
    const int a = find(ij.x), b = find(ij.y);
    if (a != b) H.uf[a] = b;
  }
  {
    std::vector<char> anchored(n, 0);
    for (int q = 0; q < np; q++) anchored[find(H.pv[q])] = 1;
    g->gauge_free = false;
    for (int i = 0; i < n; i++)
      if (!anchored[find(i)]) g->gauge_free = true;
    H.gauge_free = g->gauge_free;
  }
  H.prior_ptr.resize(n + 1, H.prior_ptr.empty() ? 0 : H.prior_ptr.back());
  phase("rows");
  // rows before r0 (the first with a new slot) and their slots are unchanged:
  // the host mirrors, the factor -> side-0 slot map and the sweep structure
  // are updated from there on (h_slot_edge keeps the plan's bits before r0,
  // as the device copy does)
  const int r0 = extra.empty() ? n_old : std::min(extra.front().x, n_old);
  const int k0 = H.row_ptr[r0];
  g->h_row_ptr.resize(n + 1);
  std::copy(H.row_ptr.begin() + r0, H.row_ptr.end(), g->h_row_ptr.begin() + r0);
  g->h_slot_col.resize(ns);
  std::copy(H.slot_col.begin() + k0, H.slot_col.end(), g->h_slot_col.begin() + k0);
  if (!g->new_slots.empty()) g->mirror_bound = false;   // (an earlier append not bound yet: its list is stale now)
  if (g->mirror_bound && (int)g->h_slot_edge.size() >= k0) {
    // the old slots keep their bound codes (the merge keeps their order), the
    // new ones get pre-plan codes and are listed for bind_plan
    std::vector<int> tail_old(g->h_slot_edge.begin() + k0, g->h_slot_edge.end());
    g->h_slot_edge.resize(ns);
    size_t kk = 0;
    for (int o = k0; o < ns; o++) {
      const int code = H.slot_edge[o];
      if ((code >> 2) >= ne_old) {
        g->h_slot_edge[o] = code;
        g->new_slots.push_back(o);
      } else {
        g->h_slot_edge[o] = kk < tail_old.size() ? tail_old[kk] : code;
        kk++;
      }
    }
    if (kk != tail_old.size()) {   // (cannot happen: the merge keeps every old slot, in order)
      std::copy(H.slot_edge.begin() + k0, H.slot_edge.end(), g->h_slot_edge.begin() + k0);
      g->mirror_bound = false;
      g->new_slots.clear();
    }
  } else {
    g->h_slot_edge.resize(ns);
    std::copy(H.slot_edge.begin() + k0, H.slot_edge.end(), g->h_slot_edge.begin() + k0);
    g->mirror_bound = false;
    g->new_slots.clear();
  }
  g->edge_slot0.resize(ne, -1);
  for (int k = k0; k < ns; k++)
    if ((H.slot_edge[k] & 1) == 0) g->edge_slot0[H.dorder[H.slot_edge[k] >> 2]] = k;
  // Cholesky-mode sweep structure (see upload_structure): the new factors come
  // last in device order, so an old factor keeps its rank among its row's
  // side-1 factors and moves by its row's shift of s1_ptr
  int x0 = n_old, y0 = n_old;   // first rows of erow / s1_ptr that change (the new rows always)
  for (const int2& ij : nij) {
    x0 = std::min(x0, ij.x);
    y0 = std::min(y0, ij.y);
  }
  std::vector<int>& erow = H.erow;
  std::vector<int>& s1_ptr = H.s1_ptr;
  std::vector<int>& s1pos = H.s1pos;
  {
    std::vector<int> ecnt(n, 0), scnt(n, 0);   // new factors per row, by side
    for (const int2& ij : nij) {
      ecnt[ij.x]++;
      scnt[ij.y]++;
    }
    erow.resize(n + 1, erow.back());
    s1_ptr.resize(n + 1, s1_ptr.back());
    for (int i = x0, c = 0; i < n; i++) erow[i + 1] += (c += ecnt[i]);
    std::vector<int> dy(n + 1, 0);   // new side-1 factors in rows < j
    for (int j = y0, c = 0; j < n; j++) {
      dy[j] = c;
      s1_ptr[j + 1] += (c += scnt[j]);
    }
    for (int e = 0; e < ne_old; e++) {
      const int y = H.eij[e].y;
      if (y > y0) s1pos[e] += dy[y];
    }
    s1pos.resize(ne);
    std::vector<int> f(n, 0);   // the new factors after the old ones of their row
    for (size_t q = 0; q < nij.size(); q++) {
      const int y = nij[q].y;
      s1pos[ne_old + q] = s1_ptr[y + 1] - scnt[y] + f[y]++;
    }
  }
  g->h_Dc.resize(6 * (size_t)n, 0.0);
  for (size_t q = 0; q < nij.size(); q++) {   // new side-1 terms, in device order after the old ones
    const double* o = &g->eom[6 * (size_t)nd[q]];
    for (int c = 0; c < 6; c++) g->h_Dc[6 * (size_t)nij[q].y + c] += o[c];
  }
  std::vector<int> brow(1, 0);
  for (int r = 0; r < n;) {
    int r1 = r + 1;
    while (r1 < n && r1 - r < pgo::kThreads && erow[r1 + 1] - erow[r] <= pgo::kThreads) r1++;
    brow.push_back(r1);
    r = r1;
  }
  phase("per-row");
  // the device: new factors, per-row arrays, slots
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  phase("sync");
  if (g->xb && (size_t)n > g->xb_n) free_lanes(g);   // (else the lanes hold the grown graph too)
  drop_graphs(g, true);
  phase("drop graphs");
  g->saved_valid = false;   // (the snapshot holds the old structure's values; its buffer, sized
                            // for the capacity, is kept: a hipFree would wait for the device)
  phase("free");
  std::vector<double4> hz(nij.size());
  std::vector<double2> hom(3 * nij.size());
  for (size_t q = 0; q < nij.size(); q++) {
    const int e = nd[q];
    const double th = g->ez[3 * e + 2];
    hz[q] = make_double4(g->ez[3 * e], g->ez[3 * e + 1], std::cos(th), std::sin(th));
    const double* o = &g->eom[6 * (size_t)e];
    hom[3 * q] = make_double2(o[0], o[1]);
    hom[3 * q + 1] = make_double2(o[2], o[3]);
    hom[3 * q + 2] = make_double2(o[4], o[5]);
  }
  // only what changed: the new factors; the row / slot arrays from the first
  // row with a new slot (earlier rows and their slots are unchanged); the
  // side-1 sums of the rows that gained side-1 terms; whole for the rest
  Staging& sg = g->stage;   // (allocated by upload_structure; staged_h2d falls back to pageable copies)
  RC_TRY(stage_begin(g, sg));
  RC_TRY(staged_h2d(g, sg, d.eij + ne_old, nij.data(), nij.size()));
  RC_TRY(staged_h2d(g, sg, d.ez + ne_old, hz.data(), hz.size()));
  RC_TRY(staged_h2d(g, sg, d.eom + 3 * (size_t)ne_old, hom.data(), hom.size()));
  RC_TRY(staged_h2d(g, sg, d.prior_ptr + n_old + 1, H.prior_ptr.data() + n_old + 1, n - n_old));
  RC_TRY(staged_h2d(g, sg, d.row_ptr + r0 + 1, H.row_ptr.data() + r0 + 1, n - r0));
  RC_TRY(staged_h2d(g, sg, d.slot_edge + H.row_ptr[r0], g->h_slot_edge.data() + H.row_ptr[r0], ns - H.row_ptr[r0]));
  RC_TRY(staged_h2d(g, sg, d.slot_col + H.row_ptr[r0], H.slot_col.data() + H.row_ptr[r0], ns - H.row_ptr[r0]));
  RC_TRY(staged_h2d(g, sg, d.erow + x0 + 1, erow.data() + x0 + 1, n - x0));
  RC_TRY(staged_h2d(g, sg, d.s1_ptr + y0 + 1, s1_ptr.data() + y0 + 1, n - y0));
  RC_TRY(staged_h2d(g, sg, d.s1pos, s1pos.data(), ne));
  {
    std::vector<int> ys;
    for (const int2& ij : nij)
      if (ij.y < n_old) ys.push_back(ij.y);
    std::sort(ys.begin(), ys.end());
    ys.erase(std::unique(ys.begin(), ys.end()), ys.end());
    for (int y : ys) RC_TRY(staged_h2d(g, sg, d.Dc + 6 * (size_t)y, g->h_Dc.data() + 6 * (size_t)y, 6));
    RC_TRY(staged_h2d(g, sg, d.Dc + 6 * (size_t)n_old, g->h_Dc.data() + 6 * (size_t)n_old, 6 * (size_t)(n - n_old)));
  }
  RC_TRY(staged_h2d(g, sg, d.brow, brow.data(), brow.size()));
  RC_TRY(stage_end(g, sg));
  d.n = n;
  d.ne = ne;
  d.nslots = ns;
  d.nlb = (int)brow.size() - 1;
  const double mean_deg = n ? (double)ns / n : 0.0;
  d.G = 4;
  while (d.G < 32 && d.G < mean_deg) d.G *= 2;
  d.G1 = 4;
  while (d.G1 < 32 && d.G1 < (n ? (double)ne / n : 0.0)) d.G1 *= 2;
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  g->dev_structure = true;
  g->last_upload = 2;
  if (g->slot_codes_plan && H.row_ptr[r0] > 0) g->slot_codes_mixed = true;   // rows < r0 keep the plan's bits
  g->bind_row0 = std::min(g->bind_row0, r0);
  if (g->chol_ready) g->plan_stale = true;   // ensure_chol decides what to keep
  phase("upload");
  // the new vertices' values (the resident ones stay bit for bit, unless the
  // caller set values since: then all of them)
  return upload_values(g, g->dev_values ? n_old : 0);
}

int ensure_device(pgo_graph* g) {
  if (!g->dev_structure) {
    const int rc = append_structure(g);
    if (rc == 1) RC_TRY(upload_structure(g));
    else if (rc != PGO_OK) return rc;
  }
  else if (!g->dev_values) RC_TRY(upload_values(g));
  return PGO_OK;
}

int sync_scalars(pgo_graph* g, int count) {
  HIP_TRY(g, hipMemcpyAsync(g->h_scal, g->d.scal, count * sizeof(double), hipMemcpyDeviceToHost, g->d.stream));
  HIP_TRY(g, hipStreamSynchronize(g->d.stream));
  return PGO_OK;
}

int device_error(pgo_graph* g, const double4* pose, double* err) {
  HIP_TRY(g, pgo::launch_error(g->d, pose, g->d.scal));
  RC_TRY(sync_scalars(g, 1));
  *err = g->h_scal[0];
  return PGO_OK;
}

struct PcgResult {
  int flag = pgo::kRunning;
  int iterations = 0;
};

double ms_between(hipEvent_t a, hipEvent_t b);

int exchange_allgather(void* ctx, const void* send, void* recv, size_t bytes, hipStream_t s) {
  pgo_graph* g = static_cast<pgo_graph*>(ctx);
  std::string why;
  const int rc = pgo::comm_allgather_device(g->part_comm, send, recv, bytes, s, &why);
  if (rc != PGO_OK) g->last_error = "partition exchange: " + why;
  return rc == PGO_OK ? 0 : -1;
}

int exchange_broadcast(void* ctx, void* buf, size_t bytes, int root, hipStream_t s) {
  pgo_graph* g = static_cast<pgo_graph*>(ctx);
  std::string why;
  const int rc = pgo::comm_broadcast_device_async(g->part_comm, buf, bytes, root, s, &why);
  if (rc != PGO_OK) g->last_error = "panel exchange: " + why;
  return rc == PGO_OK ? 0 : -1;
}

int exchange_group(void* ctx, int begin) {
  pgo_graph* g = static_cast<pgo_graph*>(ctx);
  std::string why;
  const int rc = pgo::comm_group(g->part_comm, begin, &why);
  if (rc != PGO_OK) g->last_error = "panel exchange group: " + why;
  return rc == PGO_OK ? 0 : -1;
}

int bind_plan(pgo_graph* g, bool full);

// Before a PCG linearisation: an in-place append after a Cholesky plan left
// the device owner bits (and the host mirror h_slot_edge) half the plan's, half
// pre-plan; upload the pre-plan codes whole so every factor has exactly one
// `se & 2` slot.
int unmix_slot_codes(pgo_graph* g) {
  if (!g->slot_codes_mixed) return PGO_OK;
  g->h_slot_edge = g->hs.slot_edge;
  g->mirror_bound = false;
  g->new_slots.clear();
  RC_TRY(h2d(g, g->d.slot_edge, g->h_slot_edge.data(), g->h_slot_edge.size()));
  HIP_TRY(g, hipStreamSynchronize(g->d.stream));
  g->slot_codes_plan = g->slot_codes_mixed = false;
  g->bind_row0 = 0;
  return PGO_OK;
}

int ensure_chol(pgo_graph* g) {
  const int psz = g->part_size > 1 ? g->part_comm->size : 1, prk = psz > 1 ? g->part_comm->rank : 0;
  if (g->chol_ready && (g->chol.part_size != psz || g->chol.part_rank != prk)) {   // other partition: re-plan
    (void)hipStreamSynchronize(g->d.stream);
    free_lanes(g);
    drop_graphs(g);
    pgo::chol_free(g->chol);
    g->chol_ready = false;
    g->lane_cap = 8;
  }
  const auto t0 = std::chrono::steady_clock::now();
  auto timed = [&](int kind) {
    g->plan_update = kind;
    g->plan_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  g->plan_update = 0;
  g->plan_ms = 0.0;
  std::vector<int> order_in;
  if (g->chol_ready && g->plan_stale) {
    // the graph grew since the plan (pgo_add_edge / pgo_add_vertex after an
    // optimize: the live per-registration re-solve, graph.cpp:180-200).  Factors
    // whose blocks fit the plan's fronts (a loop closure inside existing fill):
    // keep the plan, rebuild only the H assembly lists.  New vertices / fill:
    // re-plan on the previous ordering with the new poses inserted in front of
    // their earliest-eliminated neighbour (no new nested dissection) while the
    // appended part is small; otherwise a full analysis.
    pgo::CholPlan& P = g->chol;
    const int n = g->d.n;
    std::vector<int2> pairs;   // the factors added since the plan (vertex indices)
    for (size_t e = g->plan_edges; e < g->ek1.size(); e++)
      pairs.push_back(make_int2(g->index.at(g->ek1[e]), g->index.at(g->ek2[e])));
    if (n == P.n && pgo::chol_covers(P, pairs)) {
      pgo::chol_assembly(P, g->h_row_ptr, g->h_slot_col);
      RC_TRY(bind_plan(g, false));
      g->plan_stale = false;
      g->plan_edges = g->ek1.size();
      g->eager_first = 8;
      timed(1);
      return PGO_OK;
    }
    // appended poses: into the plan incrementally while the tail is short and
    // the factor has not grown much (then a re-plan below)
    constexpr int kMaxTail = 64;
    PhaseTimer phase("ensure_chol");
    if (!getenv("PGO_NO_PLAN_APPEND") && pgo::chol_append(P, n, g->h_row_ptr, g->h_slot_col, pairs, kMaxTail, 1.05)) {
      phase("chol_append");
      if (P.schedule_error) return fail(g, PGO_E_HIP, "internal: inconsistent panel schedule");
      drop_graphs(g, true);
      RC_TRY(bind_plan(g, true));
      g->plan_stale = false;
      g->plan_edges = g->ek1.size();
      g->eager_first = 8;
      timed(4);
      return PGO_OK;
    }
    if (n >= P.n && n - P.n <= std::max(256, P.n / 10)) {
      // (base, order): old pose k -> (iperm[k], 0); a new pose -> (min base of its
      // already-placed neighbours, -(index)), so it is eliminated just before that
      // neighbour, later new poses before earlier ones (leaves of the chain first)
      const int n0 = P.n;
      std::vector<long long> key(n);
      for (int k = 0; k < n0; k++) key[k] = (long long)P.iperm[k] << 32;
      for (int v = n0; v < n; v++) {
        long long base = n;
        for (int q = g->h_row_ptr[v]; q < g->h_row_ptr[v + 1]; q++) {
          const int u = g->h_slot_col[q];
          if (u < v) base = std::min(base, key[u] >> 32);
        }
        key[v] = (base << 32) | (0x7fffffffLL - (v - n0 + 1));   // below the old pose's 0x7fffffff
      }
      for (int k = 0; k < n0; k++) key[k] |= 0x7fffffffLL;
      order_in.resize(n);
      for (int k = 0; k < n; k++) order_in[k] = k;
      std::stable_sort(order_in.begin(), order_in.end(), [&](int a, int b) { return key[a] < key[b]; });
    }
    (void)hipStreamSynchronize(g->d.stream);
    free_lanes(g);
    drop_graphs(g);
    pgo::chol_free(P);
    g->chol_ready = false;
    g->lane_cap = 8;
  }
  g->plan_stale = false;
  if (g->chol_ready) return PGO_OK;
  g->chol.ordering = g->ordering;
  g->chol.part_size = psz;
  g->chol.part_rank = prk;
  g->chol.order_in = order_in;
  g->hook.ctx = g;
  g->hook.allgather = exchange_allgather;
  g->hook.broadcast = exchange_broadcast;
  g->hook.group = exchange_group;
  pgo::chol_analyze(g->chol, g->d.n, g->h_row_ptr, g->h_slot_col);
  g->bind_row0 = 0;   // (a new order: every owner bit)
  if (g->chol.schedule_error) return fail(g, PGO_E_HIP, "internal: inconsistent panel schedule");
  const auto tb = std::chrono::steady_clock::now();
  RC_TRY(bind_plan(g, true));
  if (getenv("PGO_PLAN_TIMING"))
    fprintf(stderr, "ensure_chol bind_plan %8.2f ms\n",
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb).count());
  g->chol_ready = true;
  g->plan_edges = g->ek1.size();
  g->eager_first = 0;
  timed(order_in.empty() ? 3 : 2);
  return PGO_OK;
}

// Bind the plan to the device graph: owner slot of every factor := its block
// in the lower triangle of the permuted matrix (the one the assembly reads;
// with write_all = 0 the linearisation writes only these), the assembly's
// sources remapped slot -> factor, and the plan (full) or its assembly lists
// uploaded.
int bind_plan(pgo_graph* g, bool full) {
  PhaseTimer phase("bind_plan");
  {
    const int n = g->d.n, ne = g->d.ne;
    const int r0 = std::min(std::max(g->bind_row0, 0), n), k0 = g->h_row_ptr[r0];
    std::vector<int>& slot_edge = g->h_slot_edge;
    std::vector<unsigned char>& eside = g->h_eside;
    if (eside.capacity() < (size_t)ne) eside.reserve(std::max<size_t>(g->cap_ne, ne));
    eside.resize(ne, 0);
    // Cholesky-mode linearisation writes each factor's owner block at its
    // device factor index (one 72-byte record per factor), so the assembly reads V[9 e + q]
    auto own_bit = [&](int r, int k) {
      const bool own = g->chol.iperm[r] > g->chol.iperm[g->h_slot_col[k]];
      slot_edge[k] = (slot_edge[k] & ~2) | (own ? 2 : 0);
      if (own) eside[slot_edge[k] >> 2] = (unsigned char)(slot_edge[k] & 1);   // one owner slot per factor
    };
    if (r0 > 0 && g->mirror_bound) {   // the order kept and every other slot bound: the new slots only
      for (int k : g->new_slots) {
        const int r = (int)(std::upper_bound(g->h_row_ptr.begin(), g->h_row_ptr.begin() + n + 1, k) - g->h_row_ptr.begin()) - 1;
        own_bit(r, k);
      }
    } else {
      host_parallel(n - r0, [&](int a, int b) {
        for (int r = r0 + a; r < r0 + b; r++)
          for (int k = g->h_row_ptr[r]; k < g->h_row_ptr[r + 1]; k++) own_bit(r, k);
      });
    }
    std::vector<int>& src = g->chol.asm_src;
    host_parallel((int)src.size(), [&](int q0, int q1) {
      for (int q = q0; q < q1; q++)   // (~slot: not yet bound; kept ones are factor indices already)
        if (src[q] < 0) src[q] = slot_edge[~src[q]] >> 2;
    });
    g->chol.asm_bound = true;
    phase("owners");
    const hipError_t e = full ? pgo::chol_upload(g->chol, g->d.stream) : pgo::chol_upload_assembly(g->chol, g->d.stream);
    if (e != hipSuccess) {
      pgo::chol_free(g->chol);
      return fail(g, e == hipErrorOutOfMemory ? PGO_E_NOMEM : PGO_E_HIP,
                  std::string("Cholesky plan upload: ") + hipGetErrorString(e));
    }
    phase("chol_upload");
    if (!g->d.eside) RC_TRY(dev_alloc(g, &g->d.eside, std::max<size_t>(g->cap_ne, g->d.ne)));
    if (g->stage.buf) {   // pinned staging: the copies (and the fronts' zeroing) run on unsynchronised
      RC_TRY(stage_begin(g, g->stage));
      RC_TRY(staged_h2d(g, g->stage, g->d.eside, eside.data(), eside.size()));
      RC_TRY(staged_h2d(g, g->stage, g->d.slot_edge + k0, slot_edge.data() + k0, slot_edge.size() - k0));
      RC_TRY(stage_end(g, g->stage));
    } else {
      RC_TRY(h2d(g, g->d.eside, eside.data(), eside.size()));
      RC_TRY(h2d(g, g->d.slot_edge + k0, slot_edge.data() + k0, slot_edge.size() - k0));
      HIP_TRY(g, hipStreamSynchronize(g->d.stream));
    }
    g->slot_codes_plan = true;
    g->slot_codes_mixed = false;
    g->bind_row0 = n;
    g->mirror_bound = true;
    g->new_slots.clear();
    phase("slots");
  }
  return PGO_OK;
}

// PCG solve of (H + lambda I) x = -g at the current linearisation.  With
// profile_every = k > 0, every k-th SpMV launch is bracketed by HIP events on
// the handle's stream; launches that ran after convergence (early-exit no-ops)
// are not counted.
int pcg_solve(pgo_graph* g, const pgo_params& p, double lam, PcgResult* out, pgo_stats* st) {
  const DevGraph& d = g->d;
  HIP_TRY(g, pgo::launch_pcg_init(d, lam));
  const double tol2 = p.pcg_relative_tol * p.pcg_relative_tol;
  const int chk = std::max(1, p.pcg_check_interval);
  const int prof = st ? p.profile_every : 0;
  int k = 0;
  out->flag = pgo::kRunning;
  while (k < p.pcg_max_iterations) {
    const int stop = std::min(p.pcg_max_iterations, k + chk);
    int npairs = 0;
    for (; k < stop; k++) {
      const bool timed = prof > 0 && (k % prof) == 0 && npairs < pgo_graph::kProfPairs;
      if (timed) {
        HIP_TRY(g, pgo::launch_pcg_spmv(d, lam, g->pev[2 * npairs], g->pev[2 * npairs + 1]));
        g->pk_iter[npairs++] = k;
      } else {
        HIP_TRY(g, pgo::launch_pcg_spmv(d, lam));
      }
      HIP_TRY(g, pgo::launch_pcg_vec(d, k, tol2));
    }
    HIP_TRY(g, hipMemcpyAsync(g->h_ctrl, d.ctrl, 2 * sizeof(int), hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(g, hipStreamSynchronize(d.stream));
    for (int t = 0; t < npairs; t++)
      if (g->pk_iter[t] < g->h_ctrl[1] || (g->h_ctrl[0] == pgo::kRunning)) {
        st->kernel_spmv_ms += ms_between(g->pev[2 * t], g->pev[2 * t + 1]);
        st->kernel_spmv_count++;
      }
    if (g->h_ctrl[0] != pgo::kRunning) break;
  }
  out->flag = g->h_ctrl[0];
  out->iterations = g->h_ctrl[1];
  return PGO_OK;
}

// (H + lambda I) x = -g.  PCG runs to completion here (its convergence reads
// sync); the Cholesky path is only enqueued and its pivot flag is read back with
// the next scalars (*known = false).
struct SolveState {
  bool known = true, solved = true;
  bool profiled = false;
  bool graph = false;                       // factor / solve replayed from graphs (ev[5] between them)
  pgo::LaunchProfile prof;
};

// Replay of the captured factorisation and solve graphs for nb lanes (captured
// on first use; one graph launch each instead of ~1e3 kernel launches), with
// ev[5] recorded between them: the factorisation's device time is ev[2]..ev[5].
int graph_factor_solve(pgo_graph* g, int nb, double* x, long long xstride, bool capture_now) {
  DevGraph& d = g->d;
  // after an incremental plan update the first factorisations per lane count
  // run eagerly: capturing ~1e3 launches costs ~14 ms on C3 and destroying the
  // graphs ~10 ms, more than a few replays gain -- the live re-solve refreshes
  // the plan every registration and factors it ~4 times (eager_first)
  if (!capture_now && !g->fac_exec[nb] && g->graph_eager[nb] < g->eager_first) {
    g->graph_eager[nb]++;
    HIP_TRY(g, pgo::chol_factor(g->chol, d.D, d.V, d.g, -1.0, d.stream, nullptr, nb));
    HIP_TRY(g, hipEventRecord(g->ev[5], d.stream));
    HIP_TRY(g, pgo::chol_solve(g->chol, x, d.stream, nb, xstride));
    return PGO_OK;
  }
  auto capture = [&](hipGraphExec_t* exec, bool factor) -> int {
    if (*exec) return PGO_OK;
    PhaseTimer phase("graph_capture");
    destroy_stale_graphs(g);
    hipGraph_t graph = nullptr;
    HIP_TRY(g, hipStreamBeginCapture(d.stream, hipStreamCaptureModeThreadLocal));
    const hipError_t e1 = factor ? pgo::chol_factor(g->chol, d.D, d.V, d.g, -1.0, d.stream, nullptr, nb)
                                 : pgo::chol_solve(g->chol, x, d.stream, nb, xstride);
    HIP_TRY(g, hipStreamEndCapture(d.stream, &graph));
    HIP_TRY(g, e1);
    HIP_TRY(g, hipGraphInstantiate(exec, graph, nullptr, nullptr, 0));
    HIP_TRY(g, hipGraphDestroy(graph));
    phase(factor ? "factor" : "solve");
    return PGO_OK;
  };
  RC_TRY(capture(&g->fac_exec[nb], true));
  RC_TRY(capture(&g->sol_exec[nb], false));
  HIP_TRY(g, hipGraphLaunch(g->fac_exec[nb], d.stream));
  HIP_TRY(g, hipEventRecord(g->ev[5], d.stream));
  HIP_TRY(g, hipGraphLaunch(g->sol_exec[nb], d.stream));
  return PGO_OK;
}

int linear_solve(pgo_graph* g, const pgo_params& p, double lam, pgo_stats* st, SolveState* ss) {
  if (p.linear_solver == PGO_SOLVER_PCG) {
    PcgResult pr;
    RC_TRY(pcg_solve(g, p, lam, &pr, st));
    if (st) st->pcg_iterations += pr.iterations;
    ss->known = true;
    ss->solved = pr.flag != pgo::kBreakdown;
    return PGO_OK;
  }
  RC_TRY(ensure_chol(g));
  const DevGraph& d = g->d;
  ss->profiled = st && p.profile_every > 0 && (g->factorizations % p.profile_every) == 0;
  g->factorizations++;
  pgo::LaunchProfile* prof = nullptr;
  if (ss->profiled) {
    ss->prof.ev = g->sev.data();
    ss->prof.cap = kProfLaunches;
    ss->prof.used = 0;
    ss->prof.fam = g->sev_fam.data();
    ss->prof.flops = g->sev_flops.data();
    ss->prof.bytes = g->sev_bytes.data();
    ss->prof.grid = g->sev_grid.data();
    ss->prof.tag = g->sev_tag.data();
    prof = &ss->prof;
  }
  *g->h_lam = lam;
  HIP_TRY(g, hipMemcpyAsync(g->chol.d_lambda, g->h_lam, sizeof(double), hipMemcpyHostToDevice, d.stream));
  const bool part = g->chol.part_size > 1;
  if (prof || !p.use_graphs || part) {  // eager: a profiled factorisation times every launch; the
                                        // partitioned one runs its exchanges between the phases
    pgo::ExchangeHook* hook = part ? &g->hook : nullptr;
    g->hook.failed = false;
    if (prof) HIP_TRY(g, hipEventRecord(g->fev[0], d.stream));
    const hipError_t ef = pgo::chol_factor(g->chol, d.D, d.V, d.g, -1.0, d.stream, prof, 1, hook);
    if (g->hook.failed) return fail(g, PGO_E_COMM, g->last_error);
    HIP_TRY(g, ef);
    if (prof) HIP_TRY(g, hipEventRecord(g->fev[1], d.stream));
    const hipError_t es = pgo::chol_solve(g->chol, d.x, d.stream, 1, 0, prof, hook);
    if (g->hook.failed) return fail(g, PGO_E_COMM, g->last_error);
    HIP_TRY(g, es);
    if (prof) HIP_TRY(g, hipEventRecord(g->fev[2], d.stream));
  } else {
    RC_TRY(graph_factor_solve(g, 1, d.x, 0, false));
    ss->graph = true;
  }
  ss->known = false;
  return PGO_OK;
}

// after the stream has drained: pivot flag and profile of an enqueued Cholesky solve
int finish_solve(pgo_graph* g, pgo_stats* st, SolveState* ss) {
  if (ss->known) return PGO_OK;
  if (ss->graph && st) {
    st->ms_factor_graph += ms_between(g->ev[2], g->ev[5]);
    st->factor_graph_flops += g->chol.flops;
  }
  int flag = 0;
  HIP_TRY(g, hipMemcpy(&flag, g->chol.d_flag, sizeof(int), hipMemcpyDeviceToHost));
  if (flag & 2) {
    g->handoff_timeout = true;
    return fail(g, PGO_E_HIP, "factorisation: an in-launch hand-off timed out");
  }
  ss->solved = flag == 0;
  ss->known = true;
  if (st) st->factor_flops = g->chol.flops;
  if (ss->profiled && st) {
    for (int u = 0; u < ss->prof.used; u++) {
      const int f = ss->prof.fam[u];
      const double ms = ms_between(ss->prof.ev[2 * u], ss->prof.ev[2 * u + 1]);
      g->fam_ms[f] += ms;
      g->fam_flops[f] += ss->prof.flops[u];
      g->fam_bytes[f] += ss->prof.bytes[u];
      g->fam_launches[f]++;
      if (f == pgo::kFamPanelSyrk || f == pgo::kFamPanelSyrk128) {
        st->kernel_syrk_ms += ms;
        st->kernel_syrk_launches++;
      }
    }
    st->kernel_syrk_count++;
    st->syrk_flops = g->chol.syrk_flops;
    if (getenv("PGO_STEP_STAMPS") && getenv("PGO_PROFILE_DUMP")) {   // top level's k_step stamps
      std::vector<unsigned long long> stp(10 * pgo::kMaxStampSlots);
      if (pgo::chol_step_stamps(stp.data(), pgo::kMaxStampSlots) == hipSuccess)
        if (FILE* f = fopen(getenv("PGO_PROFILE_DUMP"), "a")) {
          for (int q = 0; q < pgo::kMaxStampSlots; q++) {
            const unsigned long long* t = &stp[10 * q];
            if (!t[0] || !t[5]) continue;
            fprintf(f, "# stamp step %d:", q);
            for (int k = 1; k < 9; k++) fprintf(f, " %.2f", (double)((long long)(t[k] - t[0])) * 0.01);
            fprintf(f, "\n");
          }
          fclose(f);
        }
    }
    // PGO_PROFILE_DUMP=path: append the launch timeline of this factorisation
    // (family, level, panel step, workgroups, start and duration in ms from the
    // factorisation's first event, algorithmic flops, bytes)
    if (const char* path = getenv("PGO_PROFILE_DUMP")) {
      if (FILE* f = fopen(path, "a")) {
        fprintf(f, "# factorisation %lld\n", g->factorizations - 1);
        for (int u = 0; u < ss->prof.used; u++)
          fprintf(f, "%s %d %d %d %.4f %.4f %.4g %.4g\n", pgo::kernel_family_name(ss->prof.fam[u]),
                  ss->prof.tag[u] >> 16, ss->prof.tag[u] & 0xffff, ss->prof.grid[u],
                  ms_between(g->fev[0], ss->prof.ev[2 * u]), ms_between(ss->prof.ev[2 * u], ss->prof.ev[2 * u + 1]),
                  ss->prof.flops[u], ss->prof.bytes[u]);
        fclose(f);
      }
    }
    st->ms_factor_profiled += ms_between(g->fev[0], g->fev[1]);
    st->ms_solve_profiled += ms_between(g->fev[1], g->fev[2]);
  }
  return PGO_OK;
}

// Lanes 1..want-1 over the current Cholesky plan (numeric workspaces for want
// lanes); returns the lane count available (fewer when HBM runs out: each lane
// holds a full set of fronts).
int ensure_lanes(pgo_graph* g, int want) {
  want = std::max(1, std::min({want, 8, g->lane_cap}));
  if ((int)g->lanes.size() == want - 1 && g->chol.batch >= want) return want;
  free_lanes(g);
  const DevGraph& d = g->d;
  if (g->chol.batch != want) {
    // the captured graphs hold the old workspace pointers
    drop_graphs(g);
    if (pgo::chol_set_batch(g->chol, want, d.stream) != hipSuccess) {
      (void)hipGetLastError();
      g->lane_cap = 1;
      return 1;
    }
  }
  g->xb_n = std::max<size_t>({g->cap_n, (size_t)d.n, 1});   // appended vertices keep the lanes
  bool ok = hipMalloc((void**)&g->xb, sizeof(double) * 3 * g->xb_n * want) == hipSuccess;
  for (int l = 1; l < want && ok; l++) {
    g->lanes.emplace_back();
    Lane& ln = g->lanes.back();
    // (capacity, not n: an accepted lane's buffer becomes the handle's pose
    // array, which appended vertices extend in place)
    ok = hipMalloc((void**)&ln.pose_cand, sizeof(double4) * std::max<size_t>({g->cap_n, (size_t)d.n, 1})) ==
             hipSuccess &&
         hipMalloc((void**)&ln.part, sizeof(double) * pgo::kMaxBlocks * pgo::kPartSlices) == hipSuccess &&
         hipMalloc((void**)&ln.scal, sizeof(double) * 16) == hipSuccess &&
         hipMemsetAsync(ln.part, 0, sizeof(double) * pgo::kMaxBlocks * pgo::kPartSlices, d.stream) == hipSuccess;
  }
  if (ok) ok = hipStreamSynchronize(d.stream) == hipSuccess;
  if (!ok) {  // out of memory (or similar): one lane, and do not try again for this plan
    (void)hipGetLastError();
    free_lanes(g);
    drop_graphs(g);
    (void)pgo::chol_set_batch(g->chol, 1, d.stream);
    g->lane_cap = 1;
    return 1;
  }
  return want;
}

// The device view of lane l's try (lane 0: the handle's own buffers), solution in xb
DevGraph lane_view(const pgo_graph* g, int l) {
  DevGraph v = g->d;
  v.x = g->xb + (size_t)l * 3 * g->d.n;
  if (l == 0) return v;
  const Lane& ln = g->lanes[l - 1];
  v.pose_cand = ln.pose_cand;
  v.part = ln.part;
  v.scal = ln.scal;
  return v;
}

// nb >= 2 consecutive lambda tries in one batched factor + solve (captured
// graph per lane count), then per lane: model decrease, retract, error; one
// read-back.  out[4 l ..] = {solved, new error, delta'H delta, g'delta}.
int run_lanes(pgo_graph* g, const pgo_params& p, int nb, const double* lams, double* out, pgo_stats* st) {
  DevGraph& d = g->d;
  hipEvent_t* ev = g->ev;
  g->factorizations++;
  for (int l = 0; l < nb; l++) g->h_lanes[4 * 8 + l] = lams[l];
  HIP_TRY(g, hipEventRecord(ev[2], d.stream));
  HIP_TRY(g, hipMemcpyAsync(g->chol.d_lambda, g->h_lanes + 4 * 8, nb * sizeof(double), hipMemcpyHostToDevice,
                            d.stream));
  const bool part = g->chol.part_size > 1;
  if (!p.use_graphs || part) {   // (partitioned: eager, the exchanges run between the phases)
    pgo::ExchangeHook* hook = part ? &g->hook : nullptr;
    g->hook.failed = false;
    const hipError_t ef = pgo::chol_factor(g->chol, d.D, d.V, d.g, -1.0, d.stream, nullptr, nb, hook);
    if (g->hook.failed) return fail(g, PGO_E_COMM, g->last_error);
    HIP_TRY(g, ef);
    const hipError_t es = pgo::chol_solve(g->chol, g->xb, d.stream, nb, 3LL * d.n, nullptr, hook);
    if (g->hook.failed) return fail(g, PGO_E_COMM, g->last_error);
    HIP_TRY(g, es);
  } else {
    RC_TRY(graph_factor_solve(g, nb, g->xb, 3LL * d.n, false));
  }
  HIP_TRY(g, hipEventRecord(ev[3], d.stream));
  for (int l = 0; l < nb; l++) {
    const DevGraph v = lane_view(g, l);
    HIP_TRY(g, pgo::launch_model_decrease(v, v.x, v.scal + 1));
    HIP_TRY(g, pgo::launch_retract(v, v.x));
    HIP_TRY(g, pgo::launch_error(v, v.pose_cand, v.scal));
    HIP_TRY(g, hipMemcpyAsync(g->h_lanes + 4 * l, v.scal, 3 * sizeof(double), hipMemcpyDeviceToHost, d.stream));
  }
  HIP_TRY(g, hipMemcpyAsync(g->h_lanes + 4 * 8 + 8, g->chol.d_flag, nb * sizeof(int), hipMemcpyDeviceToHost,
                            d.stream));
  HIP_TRY(g, hipEventRecord(ev[4], d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  int flags[8];
  std::memcpy(flags, g->h_lanes + 4 * 8 + 8, nb * sizeof(int));
  for (int l = 0; l < nb; l++)
    if (flags[l] & 2) {
      g->handoff_timeout = true;
      return fail(g, PGO_E_HIP, "factorisation: an in-launch hand-off timed out");
    }
  for (int l = 0; l < nb; l++) {
    out[4 * l] = flags[l] == 0 ? 1.0 : 0.0;
    out[4 * l + 1] = g->h_lanes[4 * l];
    out[4 * l + 2] = g->h_lanes[4 * l + 1];
    out[4 * l + 3] = g->h_lanes[4 * l + 2];
  }
  if (st) {
    st->ms_solve += ms_between(ev[2], ev[3]);
    st->ms_update += ms_between(ev[3], ev[4]);
    st->factor_flops = g->chol.flops;
    if (p.use_graphs && !part) {   // (ev[5] is recorded by the graph replay only)
      st->ms_factor_graph += ms_between(ev[2], ev[5]);
      st->factor_graph_flops += nb * g->chol.flops;
    }
  }
  return PGO_OK;
}

// scratch + timing events of the closest-keyframe search (first use)
int ensure_search(pgo_graph* g) {
  if (g->s_d) return PGO_OK;
  HIP_TRY(g, hipMalloc((void**)&g->s_i, sizeof(int) * (pgo::kMaxBlocks + 1)));
  for (hipEvent_t* e : {&g->sev_scan[0], &g->sev_scan[1], &g->sev_batch[0], &g->sev_batch[1]})
    HIP_TRY(g, hipEventCreate(e));
  HIP_TRY(g, hipMalloc((void**)&g->s_d, sizeof(double) * (pgo::kMaxBlocks + 1)));
  return PGO_OK;
}

double ms_between(hipEvent_t a, hipEvent_t b) {
  float ms = 0.f;
  if (hipEventElapsedTime(&ms, a, b) != hipSuccess) {
    (void)hipGetLastError();   // (an unrecorded event must not surface as the next launch's error)
    return 0.0;
  }
  return ms;
}

bool check_convergence(const pgo_params& p, double cur, double nw) {  // NonlinearOptimizer.cpp
  if (nw <= p.error_tol) return true;
  const double absd = cur - nw;
  const double reld = absd / cur;
  return (p.relative_error_tol != 0.0 && reld <= p.relative_error_tol) || absd <= p.absolute_error_tol;
}

}  // namespace

// ============================================================== C-ABI
extern "C" {

int pgo_abi_version(void) { return PGO_ABI_VERSION; }

const char* pgo_status_string(int s) {
  switch (s) {
    case PGO_OK: return "ok";
    case PGO_E_ARG: return "invalid argument";
    case PGO_E_DUP_KEY: return "ValuesKeyAlreadyExists: key already inserted";
    case PGO_E_NO_KEY: return "ValuesKeyDoesNotExist: key has no value";
    case PGO_E_BAD_COV: return "covariance is not symmetric positive definite";
    case PGO_E_INDETERMINANT: return "IndeterminantLinearSystemException: linear system is singular";
    case PGO_E_NONFINITE: return "non-finite value";
    case PGO_E_HIP: return "HIP runtime error";
    case PGO_E_NO_DEVICE: return "no HIP device";
    case PGO_E_NOMEM: return "out of memory";
    case PGO_E_BAD_EDGE: return "between factor connects a key to itself";
    case PGO_E_COMM: return "inter-rank exchange failed";
    case PGO_E_NOT_ENOUGH: return "not enough keyframes";
    case PGO_W_MAXITER: return "stopped at max_iterations";
    default: return "unknown status";
  }
}

void pgo_default_params(pgo_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->max_iterations = 100;
  p->relative_error_tol = 1e-5;
  p->absolute_error_tol = 1e-5;
  p->error_tol = 0.0;
  p->lambda_initial = 1e-5;
  p->lambda_factor = 10.0;
  p->lambda_upper_bound = 1e5;
  p->lambda_lower_bound = 0.0;
  p->min_model_fidelity = 1e-3;
  p->use_fixed_lambda_factor = 1;
  p->algorithm = PGO_ALG_LM;
  p->linear_solver = PGO_SOLVER_CHOLESKY;
  p->pcg_relative_tol = 1e-10;
  p->pcg_max_iterations = 20000;
  p->pcg_check_interval = 32;
  p->max_outer = 0;
  p->profile_every = 0;
  p->use_graphs = 1;
  p->lambda_lanes = 1;
  p->multi_gpu = PGO_MULTI_SPECULATIVE;
}

pgo_graph* pgo_create(const pgo_opts* opts) {
  pgo_graph* g = new (std::nothrow) pgo_graph();
  if (!g) return nullptr;
  if (opts) {
    if (opts->ordering != PGO_ORDERING_ND && opts->ordering != PGO_ORDERING_AMD) {
      delete g;
      return nullptr;
    }
    g->device = opts->device;
    g->ordering = opts->ordering == PGO_ORDERING_AMD ? pgo::kOrderAmd : pgo::kOrderNd;
  }
  return g;
}

void pgo_destroy(pgo_graph* g) {
  if (!g) return;
  if (g->comm.nccl || g->comm.d_gather || g->pcomm.nccl || g->pcomm.d_gather) (void)hipSetDevice(g->device);
  pgo::comm_free(&g->comm);
  pgo::comm_free(&g->pcomm);
  if (g->hip_ready) {
    (void)hipSetDevice(g->device);
    (void)hipStreamSynchronize(g->d.stream);
    free_device(g);
    for (auto& e : g->ev)
      if (e) (void)hipEventDestroy(e);
    if (g->h_scal) (void)hipHostFree(g->h_scal);
    if (g->h_ctrl) (void)hipHostFree(g->h_ctrl);
    if (g->h_lam) (void)hipHostFree(g->h_lam);
    if (g->stage.buf) (void)hipHostFree(g->stage.buf);
    if (g->stage.done) (void)hipEventDestroy(g->stage.done);
    if (g->h_lanes) (void)hipHostFree(g->h_lanes);
    for (auto& e : g->pev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : g->sev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : g->fev)
      if (e) (void)hipEventDestroy(e);
    if (g->lin_done) (void)hipEventDestroy(g->lin_done);
    void* sp[] = {g->s_d, g->s_i, g->sb_d, g->sb_i, g->sb_q, g->sbp_d, g->sbp_i};
    for (void* q : sp)
      if (q) (void)hipFree(q);
    for (hipEvent_t e : {g->sev_scan[0], g->sev_scan[1], g->sev_batch[0], g->sev_batch[1]})
      if (e) (void)hipEventDestroy(e);
    if (g->d.stream) (void)hipStreamDestroy(g->d.stream);
  }
  delete g;
}

const char* pgo_last_error(const pgo_graph* g) { return g ? g->last_error.c_str() : "null handle"; }

int pgo_add_vertex(pgo_graph* g, uint64_t key, double x, double y, double theta) {
  if (!g) return PGO_E_ARG;
  if (!std::isfinite(x) || !std::isfinite(y) || !std::isfinite(theta))
    return fail(g, PGO_E_NONFINITE, "non-finite initial value for key " + std::to_string(key));
  if (g->index.count(key)) return fail(g, PGO_E_DUP_KEY, "key " + std::to_string(key) + " already inserted");
  // (no download: the resident values stay on the device, the new one is host-side
  // until the next upload -- download_values reads back the resident ones only)
  g->index.emplace(key, (int32_t)g->keys.size());
  g->keys.push_back(key);
  g->xyt.insert(g->xyt.end(), {x, y, theta});
  g->dev_structure = false;
  return PGO_OK;
}

// Bulk adds leave 1/8 room in the host arrays (and the key index), as the device
// arrays have: the live node's first single appends after a bulk load then do
// not copy the whole graph (a 500k-factor graph: ~46 MB, ~9 ms).
static size_t with_room(size_t n) { return n + n / 8 + 64; }

int pgo_add_vertices(pgo_graph* g, size_t n, const uint64_t* keys, const double* xyt) {
  if (!g || (n && (!keys || !xyt))) return PGO_E_ARG;
  const size_t nv = with_room(g->keys.size() + n);
  if (g->keys.capacity() < g->keys.size() + n) {
    g->keys.reserve(nv);
    g->xyt.reserve(3 * nv);
    g->index.reserve(nv);
  }
  for (size_t i = 0; i < n; i++) RC_TRY(pgo_add_vertex(g, keys[i], xyt[3 * i], xyt[3 * i + 1], xyt[3 * i + 2]));
  return PGO_OK;
}

int pgo_add_prior(pgo_graph* g, uint64_t key, const double pose[3], const double cov[9]) {
  if (!g || !pose || !cov) return PGO_E_ARG;
  for (int a = 0; a < 3; a++)
    if (!std::isfinite(pose[a])) return fail(g, PGO_E_NONFINITE, "non-finite prior pose");
  double om[6];
  if (information(cov, om) != PGO_OK) return fail(g, PGO_E_BAD_COV, "prior covariance not positive definite");
  g->pk.push_back(key);
  g->pz.insert(g->pz.end(), pose, pose + 3);
  g->pom.insert(g->pom.end(), om, om + 6);
  g->dev_structure = false;
  return PGO_OK;
}

int pgo_add_edge(pgo_graph* g, uint64_t k1, uint64_t k2, const double z[3], const double cov[9]) {
  if (!g || !z || !cov) return PGO_E_ARG;
  if (k1 == k2) return fail(g, PGO_E_BAD_EDGE, "between factor on key " + std::to_string(k1) + " and itself");
  for (int a = 0; a < 3; a++)
    if (!std::isfinite(z[a])) return fail(g, PGO_E_NONFINITE, "non-finite measurement");
  double om[6];
  if (information(cov, om) != PGO_OK)
    return fail(g, PGO_E_BAD_COV, "between factor covariance not positive definite");
  if (g->ek1.size() >= (size_t)(1 << 30)) return fail(g, PGO_E_NOMEM, "too many factors");
  g->ek1.push_back(k1);
  g->ek2.push_back(k2);
  g->ez.insert(g->ez.end(), z, z + 3);
  g->eom.insert(g->eom.end(), om, om + 6);
  g->dev_structure = false;
  return PGO_OK;
}

int pgo_add_edges(pgo_graph* g, size_t n, const uint64_t* k1, const uint64_t* k2, const double* z,
                  const double* cov, int cov_stride) {
  if (!g || (n && (!k1 || !k2 || !z || !cov)) || (cov_stride != 0 && cov_stride != 9)) return PGO_E_ARG;
  if (g->ek1.capacity() < g->ek1.size() + n) {
    const size_t ne = with_room(g->ek1.size() + n);
    g->ek1.reserve(ne);
    g->ek2.reserve(ne);
    g->ez.reserve(3 * ne);
    g->eom.reserve(6 * ne);
  }
  for (size_t i = 0; i < n; i++) RC_TRY(pgo_add_edge(g, k1[i], k2[i], z + 3 * i, cov + (size_t)cov_stride * i));
  return PGO_OK;
}

size_t pgo_num_factors(const pgo_graph* g) { return g ? g->ek1.size() + g->pk.size() : 0; }
size_t pgo_num_vertices(const pgo_graph* g) { return g ? g->keys.size() : 0; }

int pgo_get_pose(pgo_graph* g, uint64_t key, double out[3]) {
  if (!g || !out) return PGO_E_ARG;
  auto it = g->index.find(key);
  if (it == g->index.end()) return fail(g, PGO_E_NO_KEY, "key " + std::to_string(key) + " has no value");
  RC_TRY(download_values(g));
  std::memcpy(out, &g->xyt[3 * (size_t)it->second], 3 * sizeof(double));
  return PGO_OK;
}

int pgo_get_poses(pgo_graph* g, size_t n, const uint64_t* keys, double* out) {
  if (!g || (n && !out)) return PGO_E_ARG;
  RC_TRY(download_values(g));
  if (!keys) {
    if (n != g->keys.size()) return fail(g, PGO_E_ARG, "n must equal the number of vertices when keys is NULL");
    if (n) std::memcpy(out, g->xyt.data(), 3 * n * sizeof(double));
    return PGO_OK;
  }
  for (size_t i = 0; i < n; i++) {
    auto it = g->index.find(keys[i]);
    if (it == g->index.end()) return fail(g, PGO_E_NO_KEY, "key " + std::to_string(keys[i]) + " has no value");
    std::memcpy(out + 3 * i, &g->xyt[3 * (size_t)it->second], 3 * sizeof(double));
  }
  return PGO_OK;
}

int pgo_set_poses(pgo_graph* g, size_t n, const uint64_t* keys, const double* xyt) {
  if (!g || (n && !xyt)) return PGO_E_ARG;
  RC_TRY(download_values(g));
  for (size_t i = 0; i < 3 * n; i++)
    if (!std::isfinite(xyt[i])) return fail(g, PGO_E_NONFINITE, "non-finite value");
  if (!keys) {
    if (n != g->keys.size()) return fail(g, PGO_E_ARG, "n must equal the number of vertices when keys is NULL");
    if (n) std::memcpy(g->xyt.data(), xyt, 3 * n * sizeof(double));
  } else {
    for (size_t i = 0; i < n; i++) {
      auto it = g->index.find(keys[i]);
      if (it == g->index.end()) return fail(g, PGO_E_NO_KEY, "key " + std::to_string(keys[i]) + " has no value");
      std::memcpy(&g->xyt[3 * (size_t)it->second], xyt + 3 * i, 3 * sizeof(double));
    }
  }
  g->dev_values = false;
  return PGO_OK;
}

int pgo_save_values(pgo_graph* g) {
  if (!g) return PGO_E_ARG;
  RC_TRY(ensure_device(g));
  DevGraph& d = g->d;
  if (!d.pose_saved) RC_TRY(dev_alloc(g, &d.pose_saved, std::max<size_t>(g->cap_n, d.n)));
  if (d.n)
    HIP_TRY(g, hipMemcpyAsync(d.pose_saved, d.pose, d.n * sizeof(double4), hipMemcpyDeviceToDevice, d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  g->saved_valid = true;
  return PGO_OK;
}

int pgo_restore_values(pgo_graph* g) {
  if (!g) return PGO_E_ARG;
  DevGraph& d = g->d;
  if (!g->dev_structure || !d.pose_saved || !g->saved_valid)
    return fail(g, PGO_E_ARG, "no saved values (graph changed or never saved)");
  if (d.n)
    HIP_TRY(g, hipMemcpyAsync(d.pose, d.pose_saved, d.n * sizeof(double4), hipMemcpyDeviceToDevice, d.stream));
  g->dev_values = true;
  g->host_values = false;
  return PGO_OK;
}

int pgo_marginal_covariances(pgo_graph* g, size_t n, const uint64_t* keys, double* out) {
  if (!g || (n && (!keys || !out))) return PGO_E_ARG;
  if (n == 0) return PGO_OK;
  std::vector<int> poses(n);
  for (size_t i = 0; i < n; i++) {
    auto it = g->index.find(keys[i]);
    if (it == g->index.end()) return fail(g, PGO_E_NO_KEY, "marginal of key " + std::to_string(keys[i]) + " with no inserted value");
    poses[i] = it->second;
  }
  RC_TRY(ensure_device(g));
  HIP_TRY(g, hipSetDevice(g->device));
  g->part_size = 1;   // the path solves walk every front: a one-rank plan
  RC_TRY(ensure_chol(g));
  DevGraph& d = g->d;
  d.write_all = 0;
  HIP_TRY(g, pgo::launch_linearize(d));
  *g->h_lam = 0.0;
  HIP_TRY(g, hipMemcpyAsync(g->chol.d_lambda, g->h_lam, sizeof(double), hipMemcpyHostToDevice, d.stream));
  HIP_TRY(g, pgo::chol_factor(g->chol, d.D, d.V, d.g, 0.0, d.stream, nullptr));
  int flag = 0;
  HIP_TRY(g, hipMemcpyAsync(&flag, g->chol.d_flag, sizeof(int), hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  if (flag) return fail(g, PGO_E_INDETERMINANT, "marginals: the linearised system is not positive definite");
  // batches bound the per-workgroup scratch (6 x max front rows doubles each)
  const size_t B = 256;
  for (size_t b0 = 0; b0 < n; b0 += B) {
    const int nb = (int)std::min(B, n - b0);
    HIP_TRY(g, pgo::chol_marginals(g->chol, poses.data() + b0, nb, out + 9 * b0, d.stream));
  }
  return PGO_OK;
}

int pgo_error(pgo_graph* g, double* err) {
  if (!g || !err) return PGO_E_ARG;
  RC_TRY(ensure_device(g));
  return device_error(g, g->d.pose, err);
}

int pgo_optimize(pgo_graph* g, const pgo_params* params, pgo_stats* stats) {
  RoctxRange range_opt("pgo_optimize");
  if (!g) return PGO_E_ARG;
  pgo_params p;
  if (params) p = *params;
  else pgo_default_params(&p);
  pgo_stats st;
  std::memset(&st, 0, sizeof(st));
  const auto T0 = std::chrono::steady_clock::now();
  auto upload0 = std::chrono::steady_clock::now();
  g->trace.clear();
  for (int f = 0; f < pgo::kFamCount; f++) {
    g->fam_ms[f] = g->fam_flops[f] = g->fam_bytes[f] = 0.0;
    g->fam_launches[f] = 0;
  }
  auto since_T0 = [&]() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count();
  };
  // per-iteration record (pgo_get_trace): the oracle's trace columns + wall ms
  auto trace_row = [&](double it, double lam_t, double solved, double lin_change, double new_e, double fid,
                       double acc) {
    const double row[kTraceCols] = {it, lam_t, solved, lin_change, new_e, fid, acc, since_T0()};
    g->trace.insert(g->trace.end(), row, row + kTraceCols);
  };
  g->last_upload = 0;
  int rc = ensure_device(g);
  if (rc != PGO_OK) return rc;
  st.ms_upload = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - upload0).count();
  st.upload_kind = g->last_upload;
  DevGraph& d = g->d;
  HIP_TRY(g, hipSetDevice(g->device));
  double err = 0.0;
  RC_TRY(device_error(g, d.pose, &err));
  st.initial_error = err;
  if (!std::isfinite(err)) {
    st.status = PGO_E_NONFINITE;
    if (stats) *stats = st;
    return fail(g, PGO_E_NONFINITE, "initial error is not finite");
  }
  double lam = p.lambda_initial, factor = p.lambda_factor;
  int iters = 0, inner = 0;
  int status = PGO_OK;
  if (p.algorithm == PGO_ALG_GN && g->gauge_free && d.n > 0 && !(err <= p.error_tol)) {
    st.status = PGO_E_INDETERMINANT;
    if (stats) *stats = st;
    return fail(g, PGO_E_INDETERMINANT,
                "Gauss-Newton: a connected component has no prior, the linear system is singular");
  }
  hipEvent_t* ev = g->ev;
  // PGO_MULTI_PARTITION with ranks: every try's factorisation is split over
  // the ranks (each rank then walks the same, replicated LM control).
  // PGO_MULTI_HYBRID: split over the partition group (pcomm), and the groups
  // run the speculative search over comm (one rank of every group each)
  const bool chol_lm = p.linear_solver != PGO_SOLVER_PCG && p.algorithm != PGO_ALG_GN;
  // (a bound partition group of one rank is the speculative search alone)
  const bool hybrid = p.multi_gpu == PGO_MULTI_HYBRID && g->pcomm_bound && g->pcomm.size > 1 && chol_lm;
  if (p.multi_gpu == PGO_MULTI_HYBRID && !g->pcomm_bound && g->comm.size > 1 && chol_lm)
    return fail(g, PGO_E_ARG, "PGO_MULTI_HYBRID needs a partition-group communicator (pgo_comm_init_*_part, "
                              "set up before the main communicator)");
  g->part_comm = hybrid ? &g->pcomm : &g->comm;
  const bool partition = (hybrid || (p.multi_gpu == PGO_MULTI_PARTITION && g->comm.size > 1)) && chol_lm;
  g->part_size = partition ? g->part_comm->size : 1;
  // Cholesky: the plan (and the owner bits it assigns) first, then the
  // linearisation writes only the blocks the assembly reads
  if (p.linear_solver != PGO_SOLVER_PCG && d.n > 0) {
    RoctxRange range_plan("plan");
    RC_TRY(ensure_chol(g));
    st.plan_update = g->plan_update;
    st.ms_plan = g->plan_ms;
  }
  if (p.linear_solver == PGO_SOLVER_PCG) RC_TRY(unmix_slot_codes(g));
  d.write_all = p.linear_solver == PGO_SOLVER_PCG ? 1 : 0;
  // One lambda try (GTSAM tryLambda): solve (H + lam I) delta = -g, retract into
  // pose_cand, error there and the linear model decrease; one read-back.
  // out = {solved, new error, delta'H delta, g'delta}.
  bool first_try = true;
  auto account_linearize = [&]() {   // after the first try of a linearisation has synchronised
    if (!first_try) return;
    const double lin_ms = ms_between(ev[0], ev[1]);
    st.ms_linearize += lin_ms;
    if (p.profile_every > 0) {
      st.kernel_linearize_ms += lin_ms;
      st.kernel_linearize_count++;
    }
    first_try = false;
  };
  auto run_try_once = [&](double lam_try, double* out) -> int {
    SolveState ss;
    HIP_TRY(g, hipEventRecord(ev[2], d.stream));
    RC_TRY(linear_solve(g, p, lam_try, &st, &ss));
    st.solves++;
    HIP_TRY(g, hipEventRecord(ev[3], d.stream));
    if (!ss.known || ss.solved) {
      if (p.algorithm != PGO_ALG_GN) HIP_TRY(g, pgo::launch_model_decrease(d, d.x, d.scal + 1));
      HIP_TRY(g, pgo::launch_retract(d, d.x));
      HIP_TRY(g, pgo::launch_error(d, d.pose_cand, d.scal));
    }
    HIP_TRY(g, hipEventRecord(ev[4], d.stream));
    RC_TRY(sync_scalars(g, 3));
    RC_TRY(finish_solve(g, &st, &ss));
    account_linearize();
    st.ms_solve += ms_between(ev[2], ev[3]);
    st.ms_update += ms_between(ev[3], ev[4]);
    out[0] = ss.solved ? 1.0 : 0.0;
    out[1] = g->h_scal[0];
    out[2] = g->h_scal[1];
    out[3] = g->h_scal[2];
    return PGO_OK;
  };
  // a try whose in-launch hand-off timed out (a workgroup starved on a shared
  // GPU) runs once more before the optimize fails (every rank of a partitioned
  // run sees the same flags, so all retry together)
  auto retried = [&](auto&& body) -> int {
    g->handoff_timeout = false;
    int rc = body();
    if (rc == PGO_E_HIP && g->handoff_timeout) {
      g->handoff_timeout = false;
      st.handoff_retries++;   // visible in pgo_stats / the bench's per_step (round 6)
      rc = body();
    }
    return rc;
  };
  auto run_try = [&](double lam_try, double* out) -> int {
    return retried([&] { return run_try_once(lam_try, out); });
  };
  pgo::Comm& cm = g->comm;
  // the speculative search's ranks (a partitioned run is one search: P = 1
  // here; the hybrid's search runs over the groups, one rank of each in cm)
  const bool spec = !partition || hybrid;
  const int P = spec ? cm.size : 1, me = spec ? cm.rank : 0;
  const bool exchange = spec && (P > 1 || pgo::force_collectives(&cm));   // forced: 1-rank RCCL too
  st.ranks = hybrid ? cm.size * g->pcomm.size : cm.size;
  auto transport_of = [](const pgo::Comm& c) {
    return c.size <= 1 && !c.nccl ? PGO_TRANSPORT_NONE : (c.host ? PGO_TRANSPORT_HOST : PGO_TRANSPORT_RCCL);
  };
  st.transport = transport_of(cm);
  st.part_transport = hybrid ? transport_of(g->pcomm) : PGO_TRANSPORT_NONE;
  // lanes: concurrent tries on this GPU (Cholesky LM only)
  int L = 1;
  if (p.algorithm != PGO_ALG_GN && p.linear_solver != PGO_SOLVER_PCG && p.lambda_lanes > 1 && d.n > 0)
    L = ensure_lanes(g, p.lambda_lanes);
  // every rank must agree on the lanes per rank (a lane allocation may fail on
  // one); a partitioned run's ranks factor the same lanes together (the
  // hybrid: the minimum over the group, then over the groups)
  auto agree_lanes = [&](pgo::Comm& c) -> int {
    std::vector<double> all(c.size);
    const double mineL = L;
    std::string why;
    const int rc = pgo::comm_allgather(&c, &mineL, 1, all.data(), d.stream, &why);
    if (rc != PGO_OK) return fail(g, rc, "lane count all-gather: " + why);
    for (double v : all) L = std::min(L, (int)v);
    return PGO_OK;
  };
  if (partition && g->part_comm->size > 1) RC_TRY(agree_lanes(*g->part_comm));
  if (exchange && (!partition || hybrid)) RC_TRY(agree_lanes(cm));
  const int T = P * L;                       // tries per round
  std::vector<double> lam_k(T), fac_k(T), outs(4 * T);
  int last_outcome = PGO_STOP_CONVERGED;     // how the last linearisation's tries ended
  std::vector<char> valid(T);
  // Lanes sized to the tries expected, so the round that should reach the
  // accepted try runs only the lanes up to it (a one-lane round is cheaper than
  // a batched one); all lanes again if that try fails.  The expectation follows
  // GTSAM's lambda dynamics: after a first-try acceptance lambda keeps falling
  // and the next linearisation is expected to accept at once (1 try); after an
  // acceptance that needed k >= 2 tries the next linearisation starts one decade
  // below the accepted lambda, which just failed, so 2 tries are expected
  // rather than k (C3: 13 rounds either way, two of them 2-lane instead of
  // 3-lane).  The first linearisation of an optimize() expects 1: GTSAM starts
  // at lambda = 1e-5, a nearly undamped step, which from odometry-initialised
  // or warm-started values is accepted.  The tries and their order are
  // unchanged (PGO_LANES_ADAPT=0: every round runs all lanes; 2: the previous
  // linearisation's count, all lanes first; 3: this rule, all lanes first).
  static const int adapt_mode = getenv("PGO_LANES_ADAPT") ? atoi(getenv("PGO_LANES_ADAPT")) : 1;
  static const bool adapt_lanes = adapt_mode != 0;
  int prev_walked = 0;   // tries the previous linearisation walked (0: none yet)
  if (!(err <= p.error_tol) && iters < p.max_iterations && d.n > 0) {
    double new_err = err;
    for (;;) {
      const double cur_err = new_err;
      RoctxRange range_lin("linearisation");
      HIP_TRY(g, pgo::launch_linearize(d, ev[0], ev[1]));
      HIP_TRY(g, hipEventRecord(g->lin_done, d.stream));
      st.linearizations++;
      first_try = true;
      if (p.algorithm == PGO_ALG_GN) {  // one plain step; every rank computes the same one
        double o[4];
        RC_TRY(run_try(0.0, o));
        if (o[0] == 0.0) {
          status = PGO_E_INDETERMINANT;
          break;
        }
        std::swap(d.pose, d.pose_cand);
        err = o[1];
        iters++;
        inner++;
        trace_row(iters, 0.0, 1.0, NAN, err, 0.0, 1.0);
      } else {
        // Lambda rounds.  GTSAM tries lam_0 = lam, lam_{k+1} = lam_k * f_k (f_k
        // doubling when the factor is not fixed) until one is accepted, the cost
        // change is negligible, or lam_{k+1} reaches the upper bound.  Try k of a
        // round runs on rank k / L, lane k % L; the outcomes are walked in
        // sequence order with GTSAM's rules, so the accepted step is the
        // sequential one.
        int walked = 0;   // tries of this linearisation walked so far
        for (;;) {
          RoctxRange range_round("lambda_round");
          lam_k[0] = lam;
          fac_k[0] = factor;
          valid[0] = 1;
          for (int k = 1; k < T; k++) {
            lam_k[k] = lam_k[k - 1] * fac_k[k - 1];
            fac_k[k] = p.use_fixed_lambda_factor ? fac_k[k - 1] : 2.0 * fac_k[k - 1];
            valid[k] = valid[k - 1] && lam_k[k] < p.lambda_upper_bound;
          }
          // a profiled factorisation (lane 0, eager, timed launches) runs alone
          const bool prof_next = p.profile_every > 0 && (g->factorizations % p.profile_every) == 0;
          int Lr = prof_next ? 1 : L;
          const int expect = adapt_mode == 2 ? prev_walked : prev_walked == 0 ? (adapt_mode == 3 ? 0 : 1)
                                                                              : std::min(prev_walked, 2);
          if (adapt_lanes && !exchange && expect > walked) Lr = std::min(Lr, expect - walked);
          std::vector<double> mine(4 * L, 0.0);
          for (int l = 0; l < L; l++) mine[4 * l] = -1.0;  // -1: no try (past the bound / lane idle)
          int nb = 0;   // this rank's valid tries (a prefix of its lanes)
          while (nb < Lr && valid[me * L + nb]) nb++;
          if (nb == 1) {
            RC_TRY(run_try(lam_k[me * L], &mine[0]));
          } else if (nb > 1) {
            RC_TRY(retried([&] { return run_lanes(g, p, nb, &lam_k[me * L], mine.data(), &st); }));
            st.solves += nb;
            account_linearize();
          }
          st.lambda_rounds++;
          if (exchange) {
            const auto c0 = std::chrono::steady_clock::now();
            std::string why;
            const int rc = pgo::comm_allgather(&cm, mine.data(), 4 * L, outs.data(), d.stream, &why);
            if (rc != PGO_OK) return fail(g, rc, "lambda round all-gather: " + why);
            st.ms_comm += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
          } else {
            std::copy(mine.begin(), mine.end(), outs.begin());
          }
          // a lane that sat out a profiled round: its tries count as not made,
          // the walk stops there and the next round resumes from it
          for (int k = 0; k < T; k++)
            if (outs[4 * k] == -1.0) {
              for (int j = k; j < T; j++) valid[j] = 0;
              break;
            }
          int winner = -1;
          bool done = false;
          double new_e = INFINITY;
          for (int k = 0; k < T && valid[k]; k++) {
            const double* o = &outs[4 * k];
            double fidelity = 0.0, lin_change = NAN, try_e = INFINITY;
            bool success = false, stop = false;
            if (o[0] == 1.0) {
              const double xhx = o[2], gx = o[3];
              lin_change = -(gx + 0.5 * xhx);
              if (lin_change >= 0) {
                new_e = try_e = o[1];
                const double cost_change = err - new_e;
                if (lin_change > 2.220446049250313e-16 * err) {
                  fidelity = cost_change / lin_change;
                  success = fidelity > p.min_model_fidelity;
                }
                if (std::fabs(cost_change) < p.relative_error_tol * err) stop = true;
              }
            }
            trace_row(iters, lam_k[k], o[0], lin_change, try_e, fidelity, success ? 1.0 : 0.0);
            walked++;
            lam = lam_k[k];
            factor = fac_k[k];
            if (success) last_outcome = PGO_STOP_CONVERGED;
            else if (stop) last_outcome = PGO_STOP_SMALL_CHANGE;
            if (success) {  // decreaseLambda
              if (p.use_fixed_lambda_factor) {
                lam /= p.lambda_factor;
              } else {
                const double q = 2.0 * fidelity - 1.0;
                lam *= std::max(1.0 / 3.0, 1.0 - q * q * q);
                factor *= 2.0;
              }
              lam = std::max(p.lambda_lower_bound, lam);
              winner = k;
              done = true;
              break;
            }
            if (stop) {
              done = true;
              break;
            }
            lam *= factor;  // increaseLambda
            inner++;
            if (!p.use_fixed_lambda_factor) factor *= 2.0;
            if (lam >= p.lambda_upper_bound) {
              last_outcome = PGO_STOP_LAMBDA_BOUND;
              done = true;
              break;
            }
          }
          if (winner >= 0) {
            const int wr = winner / L, wl = winner % L;
            // the accepted candidate values: lane wl's buffer on rank wr
            double4** cand = wr == me && wl > 0 ? &g->lanes[wl - 1].pose_cand : &d.pose_cand;
            if (exchange) {
              const auto c0 = std::chrono::steady_clock::now();
              std::string why;
              const int rc = pgo::comm_broadcast_device(&cm, *cand, sizeof(double4) * (size_t)d.n, wr, d.stream, &why);
              if (rc != PGO_OK) return fail(g, rc, "accepted values broadcast: " + why);
              st.ms_comm += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c0).count();
            }
            std::swap(d.pose, *cand);
            err = new_e;
            iters++;
            inner++;
          }
          if (done) break;
        }
        prev_walked = walked;
      }
      if (status != PGO_OK) break;
      new_err = err;
      if (p.max_outer > 0 && st.linearizations >= p.max_outer) {
        last_outcome = PGO_STOP_MAX_OUTER;
        break;
      }
      if (!(iters < p.max_iterations && !check_convergence(p, cur_err, new_err) && std::isfinite(cur_err))) break;
    }
  }
  if (status == PGO_OK && iters >= p.max_iterations && p.max_iterations > 0) status = PGO_W_MAXITER;
  st.stop_reason = status < 0 ? PGO_STOP_ERROR
                   : (status == PGO_W_MAXITER && last_outcome != PGO_STOP_MAX_OUTER ? PGO_STOP_MAX_ITER : last_outcome);
  g->host_values = false;
  st.status = status;
  st.iterations = iters;
  st.inner_iterations = inner;
  st.final_error = err;
  st.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - T0).count();
  if (stats) *stats = st;
  if (status < 0) return fail(g, status, pgo_status_string(status));
  return status;
}

int pgo_closest_keyframe(pgo_graph* g, double x, double y, int skip, uint64_t* key, double* dist) {
  if (!g || !key || !dist || skip < 0 || !std::isfinite(x) || !std::isfinite(y)) return PGO_E_ARG;
  const size_t n = g->keys.size();
  if (n <= (size_t)skip)
    return fail(g, PGO_E_NOT_ENOUGH, "closest_keyframe: not enough keyframes (" + std::to_string(n) + " <= skip " +
                                         std::to_string(skip) + ")");
  RC_TRY(ensure_device(g));
  HIP_TRY(g, hipSetDevice(g->device));
  const DevGraph& d = g->d;
  RC_TRY(ensure_search(g));
  const int limit = (int)(n - skip);
  HIP_TRY(g, pgo::launch_closest_scan(d.pose, limit, x, y, g->s_d, g->s_i, g->s_d + pgo::kMaxBlocks,
                                      g->s_i + pgo::kMaxBlocks, d.stream, g->sev_scan[0], g->sev_scan[1]));
  g->scan_timed = true;
  HIP_TRY(g, hipMemcpyAsync(g->h_scal, g->s_d + pgo::kMaxBlocks, sizeof(double), hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipMemcpyAsync(g->h_ctrl, g->s_i + pgo::kMaxBlocks, sizeof(int), hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  const int idx = g->h_ctrl[0];
  if (idx < 0 || idx >= limit) return fail(g, PGO_E_NONFINITE, "closest_keyframe: no finite distance");
  *key = g->keys[idx];
  *dist = g->h_scal[0];
  return PGO_OK;
}

int pgo_closest_keyframes(pgo_graph* g, size_t q, const uint64_t* query_keys, int skip, uint64_t* keys_out,
                          double* dist_out) {
  if (!g || skip < 0 || (q && (!query_keys || !keys_out || !dist_out)) || q > (size_t)INT32_MAX) return PGO_E_ARG;
  if (q == 0) return PGO_OK;
  // queries sorted by vertex index: a workgroup's candidate ranges are then alike
  std::vector<std::pair<int, int>> order(q);
  for (size_t k = 0; k < q; k++) {
    auto it = g->index.find(query_keys[k]);
    if (it == g->index.end()) return fail(g, PGO_E_NO_KEY, "closest_keyframes: key " + std::to_string(query_keys[k]) + " has no value");
    order[k] = {it->second, (int)k};
  }
  std::stable_sort(order.begin(), order.end());
  std::vector<int> qv(q);
  for (size_t k = 0; k < q; k++) qv[k] = order[k].first;
  RC_TRY(ensure_device(g));
  HIP_TRY(g, hipSetDevice(g->device));
  const DevGraph& d = g->d;
  RC_TRY(ensure_search(g));
  const int max_limit = std::max(qv.back() + 1 - skip, 0);
  const size_t parts = q * (size_t)pgo::closest_batch_chunks(max_limit);
  if (g->sb_cap < q || g->sbp_cap < parts) {
    for (void* p : {(void*)g->sb_d, (void*)g->sb_i, (void*)g->sb_q, (void*)g->sbp_d, (void*)g->sbp_i})
      if (p) (void)hipFree(p);
    g->sb_d = g->sbp_d = nullptr;
    g->sb_i = g->sb_q = g->sbp_i = nullptr;
    g->sb_cap = g->sbp_cap = 0;
    HIP_TRY(g, hipMalloc((void**)&g->sb_d, sizeof(double) * q));
    HIP_TRY(g, hipMalloc((void**)&g->sb_i, sizeof(int) * q));
    HIP_TRY(g, hipMalloc((void**)&g->sb_q, sizeof(int) * q));
    HIP_TRY(g, hipMalloc((void**)&g->sbp_d, sizeof(double) * parts));
    HIP_TRY(g, hipMalloc((void**)&g->sbp_i, sizeof(int) * parts));
    g->sb_cap = q;
    g->sbp_cap = parts;
  }
  HIP_TRY(g, hipMemcpyAsync(g->sb_q, qv.data(), sizeof(int) * q, hipMemcpyHostToDevice, d.stream));
  HIP_TRY(g, pgo::launch_closest_batch(d.pose, g->sb_q, (int)q, skip, max_limit, g->sbp_d, g->sbp_i, g->sb_d,
                                       g->sb_i, d.stream, g->sev_batch[0], g->sev_batch[1]));
  g->batch_timed = true;
  std::vector<double> hd(q);
  std::vector<int> hi(q);
  HIP_TRY(g, hipMemcpyAsync(hd.data(), g->sb_d, sizeof(double) * q, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipMemcpyAsync(hi.data(), g->sb_i, sizeof(int) * q, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  for (size_t k = 0; k < q; k++) {
    const int o = order[k].second;
    keys_out[o] = hi[k] >= 0 ? g->keys[hi[k]] : PGO_NO_KEY;
    dist_out[o] = hi[k] >= 0 ? hd[k] : INFINITY;
  }
  return PGO_OK;
}

int pgo_debug_search_ms(pgo_graph* g, double* scan_ms, double* batch_ms) {
  if (!g || !scan_ms || !batch_ms) return PGO_E_ARG;
  *scan_ms = g->scan_timed ? ms_between(g->sev_scan[0], g->sev_scan[1]) : 0.0;
  *batch_ms = g->batch_timed ? ms_between(g->sev_batch[0], g->sev_batch[1]) : 0.0;
  return PGO_OK;
}

int pgo_comm_unique_id(void* out, size_t cap) {
  std::string why;
  return pgo::comm_unique_id(out, cap, &why);
}

// a main communicator (re)initialised: the partition group's communicator set
// up since the previous main init is bound to it, an older one is freed
static void bind_part_comm(pgo_graph* g) {
  if (!g->pcomm_fresh) {
    if (g->pcomm.nccl) (void)hipSetDevice(g->device);
    pgo::comm_free(&g->pcomm);
  }
  g->pcomm_bound = g->pcomm_fresh;
  g->pcomm_fresh = false;
}

int pgo_comm_init_rccl(pgo_graph* g, const void* unique_id, size_t id_bytes, int rank, int size) {
  if (!g) return PGO_E_ARG;
  RC_TRY(ensure_hip(g));
  HIP_TRY(g, hipSetDevice(g->device));
  std::string why;
  const int rc = pgo::comm_init_rccl(&g->comm, unique_id, id_bytes, rank, size, &why);
  bind_part_comm(g);
  return rc == PGO_OK ? rc : fail(g, rc, why);
}

int pgo_comm_init_host(pgo_graph* g, const pgo_host_comm* comm) {
  if (!g) return PGO_E_ARG;
  if (g->comm.nccl) (void)hipSetDevice(g->device);
  std::string why;
  const int rc = pgo::comm_init_host(&g->comm, comm, &why);
  bind_part_comm(g);
  return rc == PGO_OK ? rc : fail(g, rc, why);
}

int pgo_comm_free(pgo_graph* g) {
  if (!g) return PGO_E_ARG;
  if (g->comm.nccl || g->pcomm.nccl) (void)hipSetDevice(g->device);
  pgo::comm_free(&g->comm);
  pgo::comm_free(&g->pcomm);
  g->part_comm = &g->comm;
  g->pcomm_fresh = g->pcomm_bound = false;
  return PGO_OK;
}

int pgo_comm_init_rccl_part(pgo_graph* g, const void* unique_id, size_t id_bytes, int rank, int size) {
  if (!g) return PGO_E_ARG;
  RC_TRY(ensure_hip(g));
  HIP_TRY(g, hipSetDevice(g->device));
  std::string why;
  const int rc = pgo::comm_init_rccl(&g->pcomm, unique_id, id_bytes, rank, size, &why);
  g->pcomm_fresh = rc == PGO_OK;
  g->pcomm_bound = false;
  return rc == PGO_OK ? rc : fail(g, rc, why);
}

int pgo_comm_init_host_part(pgo_graph* g, const pgo_host_comm* comm) {
  if (!g) return PGO_E_ARG;
  if (g->pcomm.nccl) (void)hipSetDevice(g->device);
  std::string why;
  const int rc = pgo::comm_init_host(&g->pcomm, comm, &why);
  g->pcomm_fresh = rc == PGO_OK;
  g->pcomm_bound = false;
  return rc == PGO_OK ? rc : fail(g, rc, why);
}

int pgo_comm_part_rank(const pgo_graph* g, int* rank, int* size) {
  if (!g || !rank || !size) return PGO_E_ARG;
  *rank = g->pcomm.rank;
  *size = g->pcomm.size;
  return PGO_OK;
}

int pgo_comm_rank(const pgo_graph* g, int* rank, int* size) {
  if (!g || !rank || !size) return PGO_E_ARG;
  *rank = g->comm.rank;
  *size = g->comm.size;
  return PGO_OK;
}

int pgo_comm_selftest(pgo_graph* g) {
  if (!g) return PGO_E_ARG;
  pgo::Comm& c = g->comm;
  hipStream_t s = nullptr;
  if (!c.host) {
    RC_TRY(ensure_hip(g));
    HIP_TRY(g, hipSetDevice(g->device));
    s = g->d.stream;
  }
  const double mine[4] = {(double)c.rank, (double)c.size, (double)c.rank * c.rank, 1.0};
  std::vector<double> all(4 * (size_t)c.size);
  std::string why;
  int rc = pgo::comm_allgather(&c, mine, 4, all.data(), s, &why);
  if (rc != PGO_OK) return fail(g, rc, why);
  for (int r = 0; r < c.size; r++)
    if (all[4 * r] != r || all[4 * r + 1] != c.size || all[4 * r + 2] != (double)r * r || all[4 * r + 3] != 1.0)
      return fail(g, PGO_E_COMM, "all-gather returned wrong data for rank " + std::to_string(r));
  // broadcast from the last rank: 1000 doubles root * 1e6 + i
  const int root = c.size - 1, nb = 1000;
  std::vector<double> h(nb);
  for (int i = 0; i < nb; i++) h[i] = c.rank == root ? root * 1e6 + i : -1.0;
  if (c.host) {  // host transport: exercise the callback directly on host memory
    if (c.hc.broadcast(c.hc.ctx, h.data(), sizeof(double) * nb, root) != 0)
      return fail(g, PGO_E_COMM, "host broadcast callback failed");
  } else {
    double* dbuf = nullptr;
    HIP_TRY(g, hipMalloc((void**)&dbuf, sizeof(double) * nb));
    HIP_TRY(g, hipMemcpy(dbuf, h.data(), sizeof(double) * nb, hipMemcpyHostToDevice));
    rc = pgo::comm_broadcast_device(&c, dbuf, sizeof(double) * nb, root, s, &why);
    if (rc == PGO_OK) (void)hipMemcpy(h.data(), dbuf, sizeof(double) * nb, hipMemcpyDeviceToHost);
    (void)hipFree(dbuf);
    if (rc != PGO_OK) return fail(g, rc, why);
  }
  for (int i = 0; i < nb; i++)
    if (h[i] != root * 1e6 + i) return fail(g, PGO_E_COMM, "broadcast returned wrong data");
  return PGO_OK;
}

int pgo_get_trace(const pgo_graph* g, double* out, int cap) {
  if (!g || cap < 0 || (cap > 0 && !out)) return PGO_E_ARG;
  const int rows = (int)(g->trace.size() / kTraceCols);
  if (cap > 0 && rows > 0) std::memcpy(out, g->trace.data(), sizeof(double) * kTraceCols * std::min(rows, cap));
  return rows;
}

const char* pgo_kernel_family_name(int f) { return pgo::kernel_family_name(f); }

int pgo_get_kernel_profile(const pgo_graph* g, double* out, int cap) {
  if (!g || cap < 0 || (cap > 0 && !out)) return PGO_E_ARG;
  for (int f = 0; f < pgo::kFamCount && f < cap; f++) {
    double* o = out + 5 * (size_t)f;
    o[0] = (double)g->fam_launches[f];
    o[1] = g->fam_ms[f];
    o[2] = g->fam_flops[f];
    o[3] = g->fam_bytes[f];
    o[4] = 0.0;
  }
  return pgo::kFamCount;
}

int pgo_debug_parents(pgo_graph* g, int* parent, int cap) {
  if (!g || cap < 0 || (cap > 0 && !parent)) return PGO_E_ARG;
  RC_TRY(download_values(g));
  HostStructure H;
  RC_TRY(build_structure(g, H));
  pgo::CholPlan P;
  P.ordering = g->ordering;
  pgo::chol_analyze(P, (int)g->keys.size(), H.row_ptr, H.slot_col);
  for (int s = 0; s < P.ns && s < cap; s++) parent[s] = P.parent[s];
  return P.ns;
}

int pgo_debug_partition(pgo_graph* g, int size, int* owner, double* out, int cap) {
  if (!g || size < 1 || cap < 0 || (cap > 0 && (!owner || !out))) return PGO_E_ARG;
  RC_TRY(download_values(g));
  HostStructure H;
  RC_TRY(build_structure(g, H));
  pgo::CholPlan P;
  P.ordering = g->ordering;
  pgo::chol_analyze(P, (int)g->keys.size(), H.row_ptr, H.slot_col);
  std::vector<double> rf;
  double top = 0;
  const std::vector<int> own = pgo::partition_subtrees(P, size, &rf, &top);
  for (int s = 0; s < P.ns && s < cap; s++) owner[s] = own[s];
  for (int r = 0; r < size && r < cap; r++) out[r] = rf[r];
  if (size < cap) out[size] = top;
  if (cap >= 2 * size + 2) {
    double rep = 0;
    const std::vector<double> df = pgo::distributed_rank_flops(P, size, &rep);
    for (int r = 0; r < size; r++) out[size + 1 + r] = df[r];
    out[2 * size + 1] = rep;
  }
  if (cap >= 2 * size + 4 && size > 1) {   // the exchanges of the distributed top (rank 0's plan: all ranks share them)
    pgo::CholPlan Q;
    Q.ordering = g->ordering;
    Q.part_size = size;
    Q.part_rank = 0;
    pgo::chol_analyze(Q, (int)g->keys.size(), H.row_ptr, H.slot_col);
    double pts = 0, dbl = 0;
    for (const pgo::XExchange& x : Q.xchg) {
      pts++;
      for (long long v : x.size) dbl += (double)v;
    }
    out[2 * size + 2] = pts;
    out[2 * size + 3] = dbl;
  }
  return P.ns;
}

int pgo_debug_ordering(pgo_graph* g, int32_t* perm, size_t n) {
  if (!g || (n && !perm) || n != g->keys.size()) return PGO_E_ARG;
  RC_TRY(download_values(g));
  if (g->chol_ready) {
    if (n) std::memcpy(perm, g->chol.perm.data(), n * sizeof(int32_t));
    return PGO_OK;
  }
  HostStructure H;
  RC_TRY(build_structure(g, H));
  pgo::CholPlan P;
  P.ordering = g->ordering;
  pgo::chol_analyze(P, (int)n, H.row_ptr, H.slot_col);
  if (n) std::memcpy(perm, P.perm.data(), n * sizeof(int32_t));
  return PGO_OK;
}

int pgo_debug_fronts(pgo_graph* g, int* w, int* m, int* level, int cap) {
  if (!g || cap < 0 || (cap > 0 && (!w || !m || !level))) return PGO_E_ARG;
  RC_TRY(download_values(g));
  HostStructure H;
  RC_TRY(build_structure(g, H));
  pgo::CholPlan P;
  P.ordering = g->ordering;
  pgo::chol_analyze(P, (int)g->keys.size(), H.row_ptr, H.slot_col);
  for (int s = 0; s < P.ns && s < cap; s++) {
    w[s] = P.w[s];
    m[s] = P.m[s];
    level[s] = P.height[s];
  }
  return P.ns;
}

int pgo_debug_plan(pgo_graph* g, double* out, int cap) {
  if (!g || !out || cap < 16) return PGO_E_ARG;
  RC_TRY(download_values(g));
  HostStructure H;
  RC_TRY(build_structure(g, H));
  pgo::CholPlan P;
  P.ordering = g->ordering;
  pgo::chol_analyze(P, (int)g->keys.size(), H.row_ptr, H.slot_col);
  if (P.schedule_error) return fail(g, PGO_E_HIP, "internal: inconsistent panel schedule");
  // launches: factor = memsets, assembly, rhs permutation, per level extend-add
  // ranks + vector assembly + small classes + per panel diag/trsm/Schur (+look-ahead);
  // solve (backward only) = per level partials + init + steps, perm out
  long long lf = 5, ls = 1, trsm = 0, syrk = 0;
  int maxm = 0;
  for (int s = 0; s < P.ns; s++) maxm = std::max(maxm, P.m[s]);
  for (const auto& lv : P.levels) {
    lf += (long long)lv.ea_off.size() + 1 + lv.small.size();
    for (const auto& ps : lv.panels)
      lf += (ps.potrf_cnt > 0) + (ps.sdiag_cnt + ps.col_cnt + ps.prep_cnt + (ps.syrk_inline ? ps.syrk_cnt : 0) > 0) +
            (ps.syrk_cnt > 0 && !ps.syrk_inline) + (ps.far_cnt > 0);
    ls += (lv.bwd_part.cnt > 0) + (long long)lv.bwd.size();
    for (const auto& ps : lv.panels) {
      trsm += ps.fcol_cnt + ps.col_cnt;
      syrk += ps.syrk_cnt;
    }
  }
  for (int i = 0; i < cap; i++) out[i] = 0.0;
  out[0] = P.ns;
  out[1] = (double)P.levels.size();
  out[2] = P.nnzl;
  out[3] = P.flops;
  out[4] = P.syrk_flops;
  out[5] = (double)P.ftotal;
  out[6] = (double)lf;
  out[7] = (double)ls;
  out[8] = maxm;
  out[9] = (double)trsm;
  out[10] = (double)syrk;
  out[11] = (double)P.small_list.size();
  int o = 16;
  for (const auto& lv : P.levels) {   // per level: fronts, max m, max blocks, panels, small fronts, syrk tiles
    if (o + 6 > cap) break;
    long long tiles = 0;
    int small = 0;
    for (const auto& ps : lv.panels) tiles += ps.syrk_cnt;
    for (const auto& sc : lv.small) small += sc.cnt;
    out[o++] = lv.front_cnt;
    out[o++] = lv.maxm;
    out[o++] = lv.maxblk;
    out[o++] = (double)lv.panels.size();
    out[o++] = small;
    out[o++] = (double)tiles;
  }
  return PGO_OK;
}

int pgo_debug_linearize(pgo_graph* g, double* hdiag, double* hoff, double* grad, double* err) {
  if (!g) return PGO_E_ARG;
  RC_TRY(ensure_device(g));
  DevGraph& d = g->d;
  d.write_all = 1;   // diagnostics read every block
  HIP_TRY(g, pgo::launch_linearize(d));
  HIP_TRY(g, pgo::launch_error(d, d.pose, d.scal));  // overwrites partial slice A
  std::vector<double> V(9 * (size_t)d.nslots), D(6 * (size_t)d.n), G(3 * (size_t)d.n);
  if (d.nslots) HIP_TRY(g, hipMemcpyAsync(V.data(), d.V, V.size() * 8, hipMemcpyDeviceToHost, d.stream));
  if (d.n) {
    HIP_TRY(g, hipMemcpyAsync(D.data(), d.D, D.size() * 8, hipMemcpyDeviceToHost, d.stream));
    HIP_TRY(g, hipMemcpyAsync(G.data(), d.g, G.size() * 8, hipMemcpyDeviceToHost, d.stream));
  }
  RC_TRY(sync_scalars(g, 1));
  if (err) *err = g->h_scal[0];
  if (hdiag)
    for (int i = 0; i < d.n; i++) {
      const double* s = &D[6 * (size_t)i];
      double* o = hdiag + 9 * (size_t)i;
      o[0] = s[0]; o[1] = s[1]; o[2] = s[2];
      o[3] = s[1]; o[4] = s[3]; o[5] = s[4];
      o[6] = s[2]; o[7] = s[4]; o[8] = s[5];
    }
  if (hoff)
    for (int e = 0; e < d.ne; e++)
      for (int q = 0; q < 9; q++) hoff[9 * (size_t)e + q] = V[q * (size_t)d.nslots + g->edge_slot0[e]];
  if (grad && !G.empty()) std::memcpy(grad, G.data(), G.size() * 8);
  return PGO_OK;
}

// Same outputs from the Cholesky-mode linearisation (k_linearize_own +
// k_linearize_side1): owner blocks in factor order, transposed back to
// H_{k1,k2} where the owner is the factor's side-1 block.
int pgo_debug_linearize_cholesky(pgo_graph* g, double* hdiag, double* hoff, double* grad, double* err) {
  if (!g) return PGO_E_ARG;
  RC_TRY(ensure_device(g));
  DevGraph& d = g->d;
  if (d.n == 0) return PGO_OK;
  RC_TRY(ensure_chol(g));
  d.write_all = 0;
  HIP_TRY(g, pgo::launch_linearize(d));
  HIP_TRY(g, pgo::launch_error(d, d.pose, d.scal));
  std::vector<double> V(9 * (size_t)d.nslots), D(6 * (size_t)d.n), G(3 * (size_t)d.n);
  if (d.nslots) HIP_TRY(g, hipMemcpyAsync(V.data(), d.V, V.size() * 8, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipMemcpyAsync(D.data(), d.D, D.size() * 8, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipMemcpyAsync(G.data(), d.g, G.size() * 8, hipMemcpyDeviceToHost, d.stream));
  RC_TRY(sync_scalars(g, 1));
  if (err) *err = g->h_scal[0];
  if (hdiag)
    for (int i = 0; i < d.n; i++) {
      const double* s = &D[6 * (size_t)i];
      double* o = hdiag + 9 * (size_t)i;
      o[0] = s[0]; o[1] = s[1]; o[2] = s[2];
      o[3] = s[1]; o[4] = s[3]; o[5] = s[4];
      o[6] = s[2]; o[7] = s[4]; o[8] = s[5];
    }
  if (hoff)
    for (int e = 0; e < d.ne; e++) {
      const int se = g->h_slot_edge[g->edge_slot0[e]];
      const size_t de = (size_t)(se >> 2);
      const bool side0_owner = (se & 2) != 0;
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++)
          hoff[9 * (size_t)e + 3 * r + c] = V[9 * de + (side0_owner ? 3 * r + c : 3 * c + r)];
    }
  if (grad && !G.empty()) std::memcpy(grad, G.data(), G.size() * 8);
  return PGO_OK;
}

int pgo_debug_spmv(pgo_graph* g, double lambda, const double* x, double* y) {
  if (!g || !x || !y) return PGO_E_ARG;
  RC_TRY(ensure_device(g));
  DevGraph& d = g->d;
  d.write_all = 1;   // diagnostics read every block
  HIP_TRY(g, pgo::launch_linearize(d));
  RC_TRY(h2d(g, d.p, x, 3 * (size_t)d.n));
  HIP_TRY(g, pgo::launch_spmv(d, lambda, d.p, d.q));
  if (d.n) HIP_TRY(g, hipMemcpyAsync(y, d.q, 3 * (size_t)d.n * 8, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  return PGO_OK;
}

int pgo_debug_factor_time(pgo_graph* g, int lanes, int reps, double* ms) {
  if (!g || lanes < 1 || lanes > 8 || reps < 1 || !ms) return PGO_E_ARG;
  RC_TRY(ensure_device(g));
  HIP_TRY(g, hipSetDevice(g->device));
  DevGraph& d = g->d;
  if (d.n == 0) return fail(g, PGO_E_ARG, "empty graph");
  g->part_size = 1;
  RC_TRY(ensure_chol(g));
  d.write_all = 0;
  HIP_TRY(g, pgo::launch_linearize(d));
  const int L = lanes > 1 ? ensure_lanes(g, lanes) : 1;
  if (L < lanes) return fail(g, PGO_E_NOMEM, "not enough memory for the lambda lanes");
  for (int l = 0; l < L; l++) g->h_lanes[4 * 8 + l] = 1e-5 * std::pow(10.0, l);
  HIP_TRY(g, hipMemcpyAsync(g->chol.d_lambda, g->h_lanes + 4 * 8, L * sizeof(double), hipMemcpyHostToDevice,
                            d.stream));
  RC_TRY(graph_factor_solve(g, L, L > 1 ? g->xb : d.x, L > 1 ? 3LL * d.n : 0, true));   // capture + warm
  HIP_TRY(g, hipEventRecord(g->ev[0], d.stream));
  for (int r = 0; r < reps; r++) HIP_TRY(g, hipGraphLaunch(g->fac_exec[L], d.stream));
  HIP_TRY(g, hipEventRecord(g->ev[1], d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  *ms = ms_between(g->ev[0], g->ev[1]) / reps;
  return PGO_OK;
}

int pgo_debug_poison_fronts(pgo_graph* g) {
  if (!g) return PGO_E_ARG;
  if (!g->chol_ready || !g->chol.F) return fail(g, PGO_E_ARG, "no Cholesky workspace yet (optimize first)");
  HIP_TRY(g, hipSetDevice(g->device));
  HIP_TRY(g, pgo::chol_debug_poison(g->chol, g->d.stream));
  return PGO_OK;
}

int pgo_debug_solve(pgo_graph* g, double lambda, const pgo_params* params, double* delta, int* pcg_iterations) {
  if (!g || !delta) return PGO_E_ARG;
  pgo_params p;
  if (params) p = *params;
  else pgo_default_params(&p);
  RC_TRY(ensure_device(g));
  DevGraph& d = g->d;
  // the Cholesky assembly reads the owner blocks in factor order (k_linearize_own)
  g->part_size = 1;
  if (p.linear_solver != PGO_SOLVER_PCG && d.n > 0) RC_TRY(ensure_chol(g));
  if (p.linear_solver == PGO_SOLVER_PCG) RC_TRY(unmix_slot_codes(g));
  d.write_all = p.linear_solver == PGO_SOLVER_PCG ? 1 : 0;
  HIP_TRY(g, pgo::launch_linearize(d));
  pgo_stats st;
  std::memset(&st, 0, sizeof(st));
  SolveState ss;
  RC_TRY(linear_solve(g, p, lambda, &st, &ss));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  RC_TRY(finish_solve(g, nullptr, &ss));
  if (d.n) HIP_TRY(g, hipMemcpyAsync(delta, d.x, 3 * (size_t)d.n * 8, hipMemcpyDeviceToHost, d.stream));
  HIP_TRY(g, hipStreamSynchronize(d.stream));
  if (pcg_iterations) *pcg_iterations = (int)st.pcg_iterations;
  if (!ss.solved) return fail(g, PGO_E_INDETERMINANT, "linear system not positive definite");
  return PGO_OK;
}

}  // extern "C"
