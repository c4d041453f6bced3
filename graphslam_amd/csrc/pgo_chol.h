// Supernodal multifrontal Cholesky of H + lambda I on the GPU (internal).
//
// Replaces GTSAM's per-solve COLAMD ordering + multifrontal Cholesky
// (GaussianFactorGraph::optimize inside LevenbergMarquardtOptimizer, graph.cpp:119)
// with: a symbolic analysis done once per graph structure on the host
// (approximate-minimum-degree ordering of the pose graph, elimination tree,
// relaxed supernodes, front row structures, level schedule, task lists), and a
// numeric factorisation + triangular solves on the device, level by level
// (leaves first), every front of a level in flight at once.
//
// Fronts: supernode s has w_s = 3 * (its poses) pivot columns and
// m_s = w_s + 3 * (its below-diagonal pose rows) rows; its frontal matrix (the
// lower trapezoid by 64-column blocks, or m_s x m_s for a small front:
// front_packed) lives at F + foff[s] for the whole factorisation, so the
// L panel (first w_s columns) stays in place for the solves and the update
// matrix (trailing block) stays in place until the parent pulls it.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

namespace pgo {

constexpr int kSmallFront = 128;   // m <= this: whole front factorised in LDS by one workgroup
constexpr int kWaveW = 32;         // ... and w <= this: by one wavefront (panel in LDS, Schur update streamed)
constexpr int kNB = 64;            // panel width of the blocked path
constexpr int kTile = 64;          // Schur-update output tile
constexpr int kBigTile = 128;      // Schur-update output tile of the LDS-pipelined kernel
constexpr int kKB = 256;         // Schur updates deferred per kKB-column block (inner steps update the block only)
constexpr int kInlineTiles = 512;
constexpr int kLookaheadM = 512;   // fronts this tall skip the next step's column block in their plain tiles
                                   // (2048 until round 4: 512 measured 0.1 ms faster per replay at 1 and 3
                                   // lanes, profiles/r04k_ab_lookahead_threshold.txt)
constexpr int kMaxStampSlots = 256;  // PGO_STEP_STAMPS diagnostics // syrk tiles per step that ride inside k_step
constexpr int kBwdRows = 512;      // rows per partial product of the backward solve
// Schur-update tile tasks (front, row0 | clip << kClipShift, col0, k0): clip > 0
// limits the tile to columns [col0, col0 + clip) (a distributed top front's
// tile split where the column owner changes)
constexpr int kClipShift = 20;
constexpr int kRowMask = (1 << kClipShift) - 1;

// Front storage.  A front on the blocked path (front_packed: more than
// kSmallFront rows or more than kWaveW pivot columns) keeps only its lower
// trapezoid, in 64-column blocks: block b (columns [64 b, 64 b + 64)) holds
// rows [64 b, m) column-major with leading dimension fpad(m) - 64 b, the blocks
// back to back from fblock_off(fpad(m), b) -- about half the m x m square.  The small
// fronts (one wavefront / workgroup each, m <= kSmallFront) stay m x m
// column-major.  front_elems: the doubles a front occupies.
// Round 5: a packed front is stored for the height fpad(m) = m rounded up to 16
// rows (the rows past m are never touched), so every leading dimension and
// block start is a multiple of 16 doubles and, with 128-byte aligned fronts, a
// 64-row tile column is exactly four 128-byte lines instead of straddling five.
__host__ __device__ inline bool front_packed(int m, int w) { return m > kSmallFront || w > kWaveW; }
__host__ __device__ inline int fpad(int m) { return (m + 15) & ~15; }
__host__ __device__ inline long long fblock_off(int mp, long long b) { return 64 * b * mp - 2048 * b * (b - 1); }
__host__ __device__ inline long long front_elems(int m, int w) {
  if (!front_packed(m, w)) return (long long)m * m;
  const int mp = fpad(m);
  const long long nb = (m + 63) / 64, r = m - 64 * (nb - 1);
  return fblock_off(mp, nb - 1) + (mp - 64 * (nb - 1)) * r;
}

struct PanelStep {                 // one 64-column panel kb of every big front of a level
  int kb;
  int potrf_off, potrf_cnt;        // first panel: fronts whose diagonal tile k_panel_first factors (potrf_list)
  int col_off, fcol_cnt, col_cnt;  // col_tasks [col_off, +fcol_cnt): first panel's trsm row tiles (front, r0, 0, -1);
                                   // then col_cnt (front, r0, kn, kb): next panel's column block below its
                                   // diagonal tile, updated with panel kb then solved (k_step); then
  int prep_cnt = 0;                // prep tiles (front, r0, kn + 64, k0): the block after next brought up
                                   // to panel kb (k_step workgroups, look-ahead fronts)
  int sdiag_off, sdiag_cnt;        // next panel's diagonal tiles (front, kn, kn, kb) updated + factored (k_step)
  int syrk_off, syrk_cnt;          // the other Schur-update tiles (front, row0, col0, kb)
  int syrk_tile;                   // kTile or kBigTile
  int syrk_inline;                 // 1: the (64-)tiles are k_step workgroups, 0: a concurrent launch
  double syrk_flops;               // algorithmic flops of the whole Schur update of the step
  double plain_flops;              // ... of the syrk tiles alone
  double first_flops;              // algorithmic flops of k_panel_first (factor, inverse, trsm)
  double step_flops;               // ... of k_step (updates, factor, inverse, trsm, inline tiles)
  int plain_lag = 0;               // apart plain tiles: joined before step +1 or (look-ahead skip) +2
  int xfirst = -1, xstep = -1;     // distributed top: exchanges after k_panel_first / k_step (index in xchg)
  // deferred far updates: the last far_cnt of the syrk tiles (an apart step at a
  // kKB block end: the columns past the next block) go to launches of their own
  // on a fourth stream, one per piece (a kKB column block of every front, the
  // update-matrix columns one piece: CholLevel::far_pieces [far_p0, +far_np)),
  // each joined before the first step that touches it
  int far_cnt = 0, far_p0 = 0, far_np = 0;
  double far_flops = 0;            // ... their share of plain_flops
  // k_step's flops by role (sdiag; col + prep updates; col solves): a step with
  // many diagonal tiles runs them as three launches instead (chol_factor)
  double diag_flops = 0, colupd_flops = 0, trsm_flops = 0;
};

// Distributed top (part_size > 1): one exchange point -- the panels (or tails)
// xp_tasks[off, off + cnt) go from their owners to every rank, one broadcast per
// rank with a payload (size[r] doubles per lane, rank r's region of d_xprecv).
struct XExchange {
  int off = 0, cnt = 0;
  std::vector<long long> size;
};

struct SolveStep {                 // one launch of the blocked triangular solves
  int off, cnt;                    // int4 tasks (front, begin, end, owner-block or -1)
};

struct SmallClass {                // small fronts of one level with m <= mmax
  int off, cnt, mmax;
  int wave;                        // > 0: one wavefront per front (k_front_wave), panel width W (8, 16, kWaveW >= w)
  double flops = 0;                // algorithmic flops (factor + diagonal-block inverses)
};

struct CholLevel {
  std::vector<SmallClass> small;   // fronts in small_list, by size class
  std::vector<PanelStep> panels;   // blocked path
  std::vector<int> ea_off, ea_cnt; // [0]: extend-add tile tasks in ea_tasks (parents in this level)
  int front_off, front_cnt;        // all fronts of the level in level_fronts (solves)
  int small_maxm = 0, maxm = 0;    // LDS sizing
  int maxblk = 0;                  // max 64-column blocks of a front's pivot columns
  std::vector<SolveStep> bwd;      // backward: [0] = init (all columns), then steps b = maxblk-1 .. 1
  SolveStep bwd_part{0, 0};        // partial products feeding the init tasks
  SolveStep bwdc{0, 0};            // the backward steps as one chained launch (k_bwd_chain)
  int xtail = -1;                  // distributed top: the fronts' tail columns to every rank at the level's end
  mutable double at_bytes = -1;    // algorithmic HBM bytes of the level's k_assemble_tile (-1: not yet, level_at_bytes)
  double bwd_part_flops = 0;       // ... flops of its k_bwd_part
  // algorithmic HBM bytes of the level's k_vec_assemble, k_bwd_part,
  // k_bwd_init and k_bwd_chain (k_bwd_step: the same reads, split by step)
  double vec_bytes = 0, bwd_part_bytes = 0, bwd_init_bytes = 0, bwd_chain_bytes = 0;
  // far pieces (PanelStep::far_*): (step, first tile relative to its syrk_off,
  // tiles, join step or -1 = the level's end) and their flops
  std::vector<int4> far_pieces;
  std::vector<double> far_piece_flops;
};

enum { kOrderNd = 0, kOrderAmd = 1 };

struct NumericCap {                // element counts of the numeric workspaces (all lanes)
  long long F = 0, T = 0, v = 0, x = 0, sf = 0, part = 0;
};

struct CholPlan {
  int ordering = kOrderNd;         // fill-reducing ordering of the pose graph (input of chol_analyze)
  int part_size = 1, part_rank = 0; // subtree partition over ranks (input of chol_analyze)
  bool schedule_error = false;     // the panel schedule's update bookkeeping failed (a bug: the plan is unusable)
  std::vector<int> order_in;       // optional given ordering (new -> old) instead of ND / AMD (input)
  int batch = 1;                   // lambda lanes with a numeric workspace (input of chol_upload)
  // ---- host symbolic result ----
  int n = 0, ns = 0;
  int n_analyzed = 0;              // poses at the last full analysis (chol_append's tail starts there)
  double flops_analyzed = 0;       // ... and its factorisation flops
  long long nslots = 0;            // block-CSR slots of the analysed pattern (stride of V)
  std::vector<int> perm, iperm;    // pose level: new -> old, old -> new
  std::vector<int> sfirst;         // [ns+1] first pose (new index) of each supernode
  std::vector<int> m, w;           // scalar front rows / pivot columns
  std::vector<long long> foff;     // [ns+1] front offsets (doubles)
  std::vector<long long> toff;     // [ns+1] offsets of the inverted 64x64 diagonal blocks (doubles)
  std::vector<int> voff;           // [ns+1] frontal-vector offsets (doubles)
  std::vector<int> rptr, rows;     // front row poses (new index): own poses, then below rows
  std::vector<int> parent, height;
  std::vector<int> cptr, children; // children of each supernode, increasing order
  std::vector<int> ea_rel;         // per supernode: local pose index in the parent of each below row
  std::vector<int> ea_ptr;         // [ns+1] into ea_rel
  // assembly of H: target blocks (front, local row pose, local col pose) and their
  // sources: ~slot as chol_assembly writes them, the factor's device index once
  // the host binds the plan (asm_bound: every source bound)
  std::vector<int> asm_front, asm_li, asm_lj, asm_ptr, asm_src;
  bool asm_bound = false;
  // chol_append -> chol_assembly: the columns whose entries the append changed
  // (the rest of the bound lists are spliced, not rebuilt); asm_splice false: rebuild
  std::vector<int> asm_dirty;
  bool asm_splice = false;
  std::vector<int> dg_front, dg_loc;   // per new pose: front and local index (diagonal block)
  // schedules
  std::vector<CholLevel> levels;
  std::vector<int> small_list, level_fronts, potrf_list;
  std::vector<int4> syrk_tasks, sdiag_tasks, col_tasks;
  std::vector<int4> bwd_tasks;
  std::vector<int4> bwdc_tasks;    // (front, c0, c1, block): k_bwd_chain, per level
  std::vector<int2> bwd_pref;      // per bwd task: first partial, partial count (init tasks)
  std::vector<int4> bwd_part_tasks;  // (front, c0, r0, partial slot)
  int npart = 0;
  std::vector<int4> ea_tasks;      // (front, tile row << 16 | tile col, first pair, pairs): every 64x64
                                   // lower tile of every front, per level (k_assemble_tile)
  std::vector<int2> at_iptr;       // per tile task: (first, count) of its H entries in at_items
  std::vector<int> at_items;       // H entries: asm target t >= 0, or ~pose (diagonal block + lambda)
  std::vector<int4> ea_pairs;      // (child, first row a0, first column b0, rows | columns << 8):
                                   // a child's rectangle of one tile, children in order
  // ---- subtree partition (part_size > 1): levels [0, split) are this rank's
  // subtree fronts, [split, end) the replicated top; between them every rank's
  // subtree roots' update matrices + vectors are all-gathered (xroot*), after
  // the backward solve every rank's subtree solution range (xsol_ranges)
  std::vector<int> owner;          // per front: rank of its subtree, -1 top
  std::vector<int> subtree_cnt;    // fronts in the subtree of each front (postorder range)
  int split = 0;
  std::vector<int> xroot, xroot_rank;   // subtree roots (all ranks) and their ranks
  std::vector<long long> xroot_off;     // payload offset (doubles) in its rank's buffer
  std::vector<long long> xsize, xsol_size;
  long long xmax = 0, xsol_max = 0;     // largest per-rank payload (all-gather slot)
  std::vector<int4> xsol_ranges;        // (rank, first, end, offset): solution entries (xv) of each subtree
  // distributed top: column owners of the top fronts (cown[cown_off[s] + col]:
  // rank, -1 every rank; cown_off -1 for subtree fronts) and the exchanges
  std::vector<int> cown_off, cown;
  std::vector<XExchange> xchg;
  std::vector<int4> xp_tasks;           // (front, kn, nb | kind << 16, owner): kind 0 panel, 1 tail columns
  std::vector<long long> xp_loff;       // offset of the item in its owner's payload (doubles)
  std::vector<long long> xp_lstride;    // its owner's payload per lane at that exchange (doubles)
  long long xp_rslot = 0;               // largest payload per rank and lane
  double flops = 0, nnzl = 0, syrk_flops = 0;
  long long ftotal = 0, ttotal = 0;
  int vtotal = 0;
  // chol_schedule's per-level scratch lists, kept with the plan from one
  // schedule to the next (a live refresh reuses their storage) and released by
  // chol_free; not copied with the plan (a copy starts without scratch)
  struct Scratch {
    std::shared_ptr<void> p;
    Scratch() = default;
    Scratch(const Scratch&) {}
    Scratch& operator=(const Scratch&) { return *this; }
  } sched_scratch;

  // ---- device copies ----
  void* d_blob = nullptr;          // every index array below (d_m ... d_ea_pairs) in one allocation
  size_t blob_cap = 0;
  void* h_blob = nullptr;          // its pinned staging copy
  size_t h_blob_cap = 0;
  NumericCap num_cap;              // allocated workspaces (room for appended poses)
  double* F = nullptr;             // fronts
  double* Tinv = nullptr;          // inverses of the diagonal 64-blocks, column-major 64x64 each
  double* fv = nullptr;            // frontal vectors (solve)
  double* xv = nullptr;            // permuted rhs / solution, 3n
  int *d_m = nullptr, *d_w = nullptr, *d_voff = nullptr, *d_rptr = nullptr, *d_rows = nullptr;
  long long* d_foff = nullptr;
  long long* d_toff = nullptr;
  int *d_cptr = nullptr, *d_children = nullptr, *d_ea_rel = nullptr, *d_ea_ptr = nullptr, *d_parent = nullptr;
  int *d_asm_front = nullptr, *d_asm_li = nullptr, *d_asm_lj = nullptr, *d_asm_ptr = nullptr, *d_asm_src = nullptr;
  int *d_dg_front = nullptr, *d_dg_loc = nullptr, *d_perm = nullptr;
  int *d_small = nullptr, *d_level_fronts = nullptr, *d_potrf = nullptr;
  int4 *d_syrk = nullptr, *d_sdiag = nullptr, *d_col = nullptr;
  int2* d_at_iptr = nullptr;
  int* d_at_items = nullptr;
  int4 *d_xown = nullptr, *d_xforeign = nullptr, *d_xsol_own = nullptr, *d_xsol_foreign = nullptr;
  int n_xown = 0, n_xforeign = 0, n_xsol_own = 0, n_xsol_foreign = 0;
  double *d_xsend = nullptr, *d_xrecv = nullptr;   // exchange buffers (xmax / size x xmax doubles, x lanes)
  int4* d_xp = nullptr;            // xp_tasks
  long long* d_xp_off = nullptr;   // (xp_loff, xp_lstride) pairs
  double* d_xprecv = nullptr;      // panel exchange: size regions of xp_rslot x batch doubles
  int* d_stepflag = nullptr;       // [batch][ns]: last panel (kb / 64 + 1) whose diagonal inverse is published
  hipStream_t side = nullptr;      // look-ahead diagonal tiles
  hipStream_t side2 = nullptr;     // small fronts beside the blocked path
  hipStream_t side3 = nullptr;     // the second wavefront class of small fronts, beside side2
  hipStream_t side4 = nullptr;     // deferred far Schur updates (PanelStep::far_cnt)
  hipStream_t side5 = nullptr;     // a split step's column-block updates beside its diagonal tiles
  hipStream_t side6 = nullptr;     // the m > 64 small-front classes narrower than kWaveW (PGO_WAVE_STREAMS)
  hipEvent_t ev6 = nullptr;        // ... joined at the level's end
  hipEvent_t fev[8] = {};          // their join events (ring)
  hipEvent_t evs[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  int4 *d_bwd = nullptr, *d_bwd_part = nullptr, *d_bwdc = nullptr;
  int2* d_bwd_pref = nullptr;
  double* d_partial = nullptr;
  int4* d_ea_tasks = nullptr;
  int4* d_ea_pairs = nullptr;
  int* d_flag = nullptr;           // non-positive pivot seen
  double* d_lambda = nullptr;      // damping read by the assembly (graph-replay friendly)
};

// host: XCD-aware order of Schur-update tile tasks (front, row0, col0, k0): tiles
// are grouped into 8x8-tile blocks, blocks dealt round-robin to the 8 XCDs
// (workgroup i runs on XCD i mod 8), so each XCD's L2 holds the panel rows and
// columns of the blocks it works on
void xcd_order(std::vector<int4>& tasks, int tile);

// host: fill-reducing orderings of a pose graph (adjacency without self loops
// allowed); both return new -> old.  pgo_order.cpp / pgo_symbolic.cpp
std::vector<int> order_amd(int n, const std::vector<int>& xadj, const std::vector<int>& adj);
std::vector<int> order_nd(int n, const std::vector<int>& xadj, const std::vector<int>& adj);

// host: subtree partition of the supernodal tree over `size` ranks (owner per
// front, -1 = replicated top); per-rank subtree flops and the top's flops
std::vector<int> partition_subtrees(const CholPlan& P, int size, std::vector<double>* rank_flops = nullptr,
                                    double* top_flops = nullptr);

// host: per-rank flops of the partitioned factorisation with the distributed
// top (subtrees + the rank's top columns + the top work every rank repeats,
// returned in *replicated)
std::vector<double> distributed_rank_flops(const CholPlan& P, int size, double* replicated = nullptr);

// host: fn(t) for t in [0, ntask) on the planner's thread pool (the caller
// takes part; PGO_PLAN_THREADS threads, default the hardware's, at most 16)
void plan_parallel(int ntask, const std::function<void(int)>& fn);

// host: symbolic analysis from the block-CSR pattern (old pose indices)
void chol_analyze(CholPlan& P, int n, const std::vector<int>& row_ptr, const std::vector<int>& slot_col);
// host: (re)build the plan's H assembly lists for a pattern its fronts hold
void chol_assembly(CholPlan& P, const std::vector<int>& row_ptr, const std::vector<int>& slot_col);
double level_at_bytes(const CholPlan& P, int L);
// host: does the plan's factor structure hold every block of this pattern?
bool chol_covers(const CholPlan& P, int n, const std::vector<int>& row_ptr, const std::vector<int>& slot_col);
// ... every given block (old pose index pairs)?
bool chol_covers(const CholPlan& P, const std::vector<int2>& pairs);
// host: incremental symbolic update for poses P.n .. n-1 appended to the pattern
// (eliminated last, rows added along their fill paths); false = not applicable,
// plan unchanged (pgo_symbolic.cpp)
bool chol_append(CholPlan& P, int n, const std::vector<int>& row_ptr, const std::vector<int>& slot_col,
                 const std::vector<int2>& new_pairs, int max_tail, double max_growth);
hipError_t chol_upload(CholPlan& P, hipStream_t s);
// device: re-upload the assembly lists after chol_assembly (same fronts)
hipError_t chol_upload_assembly(CholPlan& P, hipStream_t s);
void chol_free(CholPlan& P);
// numeric workspaces for nb lambda lanes (P.batch); on failure one lane is kept
// and the allocation error returned
hipError_t chol_set_batch(CholPlan& P, int nb, hipStream_t s);

// Exchange of the partitioned factorisation (part_size > 1): all-gather of
// `bytes` per rank from send into recv (size x bytes, rank order), device
// buffers, enqueued on / completed with respect to stream s.  Returns 0 on
// success; a failure is remembered in `failed`.
struct ExchangeHook {
  void* ctx = nullptr;
  int (*allgather)(void* ctx, const void* send, void* recv, size_t bytes, hipStream_t s) = nullptr;
  // distributed top: `bytes` at buf from rank root to every rank (in place),
  // enqueued on stream s; several in a row form one group (group(ctx, 1) ...
  // group(ctx, 0) around them, optional)
  int (*broadcast)(void* ctx, void* buf, size_t bytes, int root, hipStream_t s) = nullptr;
  int (*group)(void* ctx, int begin) = nullptr;
  bool failed = false;
};

// device: factor H + lambda I (D: 6 doubles/pose upper, V: the Cholesky-mode
// linearisation's owner blocks, V[9 f + q] = element q of device factor f; only
// the factors in asm_src are read)
// prof (optional): every launch of the factorisation / solve timed with
// dispatch events (hipExtLaunchKernelGGL start/stop on the launch's stream),
// with its kernel family and algorithmic flops / HBM bytes: pairs of events,
// capacity cap, *used pairs recorded.
enum KernelFamily {
  kFamAssemble = 0, kFamUnused1, kFamPerm, kFamUnused3, kFamVecAssemble, kFamFrontWave, kFamFrontSmall,
  kFamPanelFirst, kFamStep, kFamPanelSyrk, kFamPanelSyrk128,
  kFamBwdPart, kFamBwdInit, kFamBwdStep, kFamStepDiag, kFamColTrsm, kFamCount
};
const char* kernel_family_name(int f);
struct LaunchProfile {
  hipEvent_t* ev = nullptr;
  int cap = 0, used = 0;
  int* fam = nullptr;
  double* flops = nullptr;
  double* bytes = nullptr;
  int* grid = nullptr;             // workgroups (x) of each launch
  int* tag = nullptr;              // level << 16 | panel step of each launch (timeline dumps)
  int cur_tag = 0;
};
// lambda is read from P.d_lambda (set it with a stream-ordered copy first).  The
// right-hand side scale_b * b (old pose indexing) is carried through the
// factorisation as an extra column: on return the frontal vectors hold y = L^-1 b.
// nb <= P.batch lanes at once: lane y factors H + lambda[y] I (lambda = P.d_lambda[y])
// in its own workspace, grid dimension y of every launch (bitwise equal to a
// one-lane factorisation)
// With a partitioned plan, hook performs the subtree roots' exchange between
// the phases (nb must be 1).
hipError_t chol_factor(const CholPlan& P, const double* D, const double* V, const double* b, double scale_b,
                       hipStream_t s, LaunchProfile* prof = nullptr, int nb = 1, ExchangeHook* hook = nullptr);
// after chol_factor: 3x3 blocks of (L L^T)^{-1} at the given poses (old index),
// row-major 9 doubles each into host memory out (synchronises the stream)
// diagnostics: the step stamps of the last factorisation run with PGO_STEP_STAMPS
// set (top level's steps, 10 wall-clock ticks of 10 ns each per step)
hipError_t chol_step_stamps(unsigned long long* out, int slots);
// diagnostics (tests): NaN into everything a factorisation writes before it
// reads it (fronts' lower trapezoids, frontal vectors, diagonal inverses), every lane
hipError_t chol_debug_poison(const CholPlan& P, hipStream_t s);
hipError_t chol_marginals(const CholPlan& P, const int* poses, int n, double* out, hipStream_t s);
// after chol_factor: x = L^-T y = (L L^T)^{-1} scale_b b, indexed by old pose
// lane y's solution to x + y * xstride
hipError_t chol_solve(const CholPlan& P, double* x, hipStream_t s, int nb = 1, long long xstride = 0,
                      LaunchProfile* prof = nullptr, ExchangeHook* hook = nullptr);

}  // namespace pgo
