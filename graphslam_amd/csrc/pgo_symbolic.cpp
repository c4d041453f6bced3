// Host-side symbolic analysis for the GPU supernodal Cholesky (pgo_chol.h).
// Runs once per graph structure (GTSAM recomputes COLAMD every solve).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <chrono>
#include <thread>
#include <tuple>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "pgo_chol.h"

namespace pgo {

// Approximate minimum degree on the quotient graph (Amestoy, Davis & Duff):
// eliminated pivots become elements that absorb their adjacent elements;
// external degrees are bounded by |A_i| + |L_p \ i| + sum_e |L_e \ L_p|,
// with |L_e \ L_p| from the w(e) counters; aggressive element absorption.
std::vector<int> order_amd(int n, const std::vector<int>& xadj, const std::vector<int>& adj) {
  std::vector<std::vector<int>> var(n), elem(n), members(n);
  std::vector<char> state(n, 0);  // 0 variable, 1 element, 2 absorbed
  std::vector<int> deg(n), w(n, 0), wstamp(n, -1), mark(n, -1);
  std::vector<int> head(n + 1, -1), nxt(n, -1), prv(n, -1);
  auto unlink = [&](int i) {
    if (prv[i] >= 0) nxt[prv[i]] = nxt[i];
    else head[deg[i]] = nxt[i];
    if (nxt[i] >= 0) prv[nxt[i]] = prv[i];
  };
  auto link = [&](int i) {
    nxt[i] = head[deg[i]];
    prv[i] = -1;
    if (head[deg[i]] >= 0) prv[head[deg[i]]] = i;
    head[deg[i]] = i;
  };
  for (int i = 0; i < n; i++) {
    for (int k = xadj[i]; k < xadj[i + 1]; k++)
      if (adj[k] != i) var[i].push_back(adj[k]);
    deg[i] = (int)var[i].size();
  }
  for (int i = n - 1; i >= 0; i--) link(i);
  std::vector<int> order(n);
  int mindeg = 0;
  for (int k = 0; k < n; k++) {
    while (head[mindeg] < 0) mindeg++;
    const int p = head[mindeg];
    unlink(p);
    order[k] = p;
    std::vector<int> Lp;
    mark[p] = k;
    for (int j : var[p])
      if (state[j] == 0 && mark[j] != k) {
        mark[j] = k;
        Lp.push_back(j);
      }
    for (int e : elem[p]) {
      if (state[e] != 1) continue;
      for (int j : members[e])
        if (state[j] == 0 && mark[j] != k) {
          mark[j] = k;
          Lp.push_back(j);
        }
      state[e] = 2;
      std::vector<int>().swap(members[e]);
    }
    state[p] = 1;
    std::vector<int>().swap(var[p]);
    std::vector<int>().swap(elem[p]);
    for (int i : Lp) unlink(i);
    for (int i : Lp)
      for (int e : elem[i]) {
        if (state[e] != 1) continue;
        if (wstamp[e] != k) {
          wstamp[e] = k;
          w[e] = (int)members[e].size();
        }
        w[e]--;
      }
    const int left = n - k - 1;
    const int lp = (int)Lp.size();
    for (int i : Lp) {
      long ext = 0;
      auto& ei = elem[i];
      size_t m = 0;
      for (int e : ei) {
        if (state[e] != 1) continue;
        if (w[e] == 0) {  // aggressive absorption: L_e inside L_p
          state[e] = 2;
          std::vector<int>().swap(members[e]);
          continue;
        }
        ei[m++] = e;
        ext += w[e];
      }
      ei.resize(m);
      ei.push_back(p);
      auto& vi = var[i];
      m = 0;
      for (int j : vi)
        if (state[j] == 0 && mark[j] != k) vi[m++] = j;
      vi.resize(m);
      long d = (long)vi.size() + (lp - 1) + ext;
      d = std::min<long>(d, (long)deg[i] + lp - 1);
      d = std::min<long>(d, left - 1);
      deg[i] = (int)std::max<long>(d, 0);
      link(i);
      mindeg = std::min(mindeg, deg[i]);
    }
    members[p] = std::move(Lp);
  }
  return order;
}

void xcd_order(std::vector<int4>& tasks, int tile) {
  constexpr int kXcd = 8, kBlk = 8;
  if ((int)tasks.size() < 4 * kXcd * kBlk) return;   // small launches: keep the natural order
  const int span = tile * kBlk;
  // (front, column block, row block) packed in the high bits, the task index in
  // the low 32: a plain sort of the keys is the stable sort by block
  // (block indices below 2^16: rows and columns below 2^20, span >= 512)
  using u128 = unsigned __int128;
  std::vector<u128> key(tasks.size());
  for (size_t i = 0; i < tasks.size(); i++) {
    const int4& t = tasks[i];
    const unsigned long long blk = (unsigned long long)(unsigned)t.x << 32 | (unsigned long long)(t.z / span) << 16 |
                                   (unsigned)((t.y & kRowMask) / span);
    key[i] = (u128)blk << 32 | i;
  }
  std::sort(key.begin(), key.end());
  std::vector<std::vector<int4>> q(kXcd);
  for (auto& v : q) v.reserve(tasks.size() / kXcd + 1);
  int blk = -1;
  unsigned long long prev = ~0ull;
  for (const u128 k : key) {
    if ((unsigned long long)(k >> 32) != prev) {
      blk++;
      prev = (unsigned long long)(k >> 32);
    }
    q[blk % kXcd].push_back(tasks[(size_t)(k & 0xffffffffu)]);
  }
  std::vector<int4> out;
  out.reserve(tasks.size());
  std::vector<size_t> pos(kXcd, 0);
  for (size_t left = tasks.size(); left;)
    for (int x = 0; x < kXcd; x++)
      if (pos[x] < q[x].size()) {
        out.push_back(q[x][pos[x]++]);
        left--;
      }
  tasks.swap(out);
}

// XCD-aware order of a level's tile-assembly tasks [off, end): a child's
// update-matrix column lands on a parent column as one run of child rows that
// crosses the parent's row tiles, so vertically adjacent tiles read the same
// 128-byte lines at their run boundaries.  Blocks of kCols x kRows tiles of a
// front, column-major inside, are dealt round-robin to the 8 XCDs (blockIdx
// b -> XCD b % 8 as observed: speed only, each tile is computed alike
// wherever and whenever it runs).  PGO_ASM_XCD=0 keeps the natural order;
// 2 orders every level, however few its tiles (host self-test).
static void ea_xcd_order(std::vector<int4>& tasks, size_t off) {
  constexpr int kXcd = 8, kCols = 4, kRows = 16;
  static const int mode = getenv("PGO_ASM_XCD") ? atoi(getenv("PGO_ASM_XCD")) : 1;
  const size_t n = tasks.size() - off;
  if (mode == 0 || (mode == 1 && n < (size_t)4 * kXcd * kCols * kRows)) return;
  // key: (block of the front in order of first appearance, column, row), task index
  using u128 = unsigned __int128;
  std::vector<u128> key(n);
  int blk = -1, fprev = -1;
  std::vector<int> bid;   // the front's blocks: (tj / kCols, ti / kRows) -> block number
  int nbr = 0;
  for (size_t i = 0; i < n; i++) {
    const int4& t = tasks[off + i];
    const int ti = t.y >> 16, tj = t.y & 0xffff;
    if (t.x != fprev) {   // a front's tasks are contiguous (row-major lower triangle)
      fprev = t.x;
      int nt = 0;
      for (size_t k = i; k < n && tasks[off + k].x == t.x; k++) nt = std::max(nt, (tasks[off + k].y >> 16) + 1);
      nbr = (nt + kRows - 1) / kRows;
      bid.assign((size_t)((nt + kCols - 1) / kCols) * nbr, -1);
    }
    int& b = bid[(size_t)(tj / kCols) * nbr + ti / kRows];
    if (b < 0) b = ++blk;
    key[i] = (u128)((unsigned long long)b << 32 | (unsigned)tj << 16 | (unsigned)ti) << 32 | i;
  }
  std::sort(key.begin(), key.end());
  std::vector<std::vector<int4>> q(kXcd);
  for (const u128 k : key) q[(int)(k >> 64) % kXcd].push_back(tasks[off + (size_t)(k & 0xffffffffu)]);
  std::vector<size_t> pos(kXcd, 0);
  size_t o = off;
  for (size_t left = n; left;)
    for (int x = 0; x < kXcd; x++)
      if (pos[x] < q[x].size()) {
        tasks[o++] = q[x][pos[x]++];
        left--;
      }
}

// dense Cholesky flops of the w pivot columns of an m-row front, plus the
// inverses of its diagonal blocks (what the small-front kernels form)
static double front_flops(int m, int w) {
  double f = (double)w * w * w / 3.0;
  for (int k = 0; k < w; k++) {
    const double r = m - k - 1;
    f += 1 + r + r * (r + 1);
  }
  return f;
}

// blocked path (64-column panels) vs one workgroup / wavefront per front
// Fronts of 128 < m <= 256 rows and w <= kWaveW pivots: one four-wave
// workgroup each (k_front_wave4) instead of the blocked path, though stored
// packed -- opt-in, PGO_WAVE4=1: measured on C3 8.86 / 16.75 ms against 8.44 /
// 16.92 ms replays at 1 / 3 lanes, 44.0 against 44.5 it/s
// (profiles/r04m_ab_wave4.txt: one workgroup per front is a longer latency
// than the blocked path's tiles spread over the chip)
static bool wave4_front(int m, int w) {
  static const bool on = getenv("PGO_WAVE4") && atoi(getenv("PGO_WAVE4")) == 1;
  return on && m > kSmallFront && m <= 2 * kSmallFront && w <= kWaveW;
}
static bool is_blocked(const CholPlan& P, int s) { return front_packed(P.m[s], P.w[s]) && !wave4_front(P.m[s], P.w[s]); }

// Column owners of the distributed top (see chol_analyze): per top front s
// (owner[s] < 0) its m columns at cown[off[s] ..]: rank, or -1 (every rank).
static void column_owners(const CholPlan& P, const std::vector<int>& owner, int psz, std::vector<int>& off,
                          std::vector<int>& cown) {
  const int ns = P.ns;
  off.assign(ns, -1);
  cown.clear();
  int rr = 0;   // round-robin position over the panels of the top fronts
  for (int s = ns - 1; s >= 0; s--) {   // parents before children
    if (owner[s] >= 0) continue;
    const int m = P.m[s], w = P.w[s], p = P.parent[s];
    off[s] = (int)cown.size();
    cown.resize(cown.size() + m, -1);
    int* own = cown.data() + off[s];
    const bool blk = is_blocked(P, s);
    const int wr = blk ? std::min(m, (w + kNB - 1) / kNB * kNB) : 0;
    for (int col = 0; col < wr; col += kNB, rr++)
      for (int j = col; j < std::min(col + kNB, wr); j++) own[j] = rr % psz;
    for (int col = std::max(wr, w); col < m; col++) {
      const int t = col - w;
      own[col] = p >= 0 ? cown[off[p] + 3 * P.ea_rel[P.ea_ptr[s] + t / 3] + t % 3] : -1;
    }
    if (!blk)
      for (int j = 0; j < m; j++) own[j] = -1;
  }
}

std::vector<double> distributed_rank_flops(const CholPlan& P, int size, double* replicated) {
  std::vector<double> rf;
  double top = 0;
  const std::vector<int> owner = partition_subtrees(P, size, &rf, &top);
  std::vector<int> off, cown;
  column_owners(P, owner, size, off, cown);
  double rep = 0;
  for (int s = 0; s < P.ns; s++) {
    if (owner[s] >= 0) continue;
    const int m = P.m[s], w = P.w[s];
    for (int j = 0; j < m; j++) {
      // column j: its scaling as a pivot, its update by every earlier pivot
      const double f = 2.0 * std::min(j, w) * (m - j) + (j < w ? (double)(m - j) : 0.0);
      const int o = cown[off[s] + j];
      if (o < 0) rep += f;
      else rf[o] += f;
    }
  }
  for (double& v : rf) v += rep;
  if (replicated) *replicated = rep;
  return rf;
}

// Front storage offsets (F, Tinv, frontal vectors) and the factor's flops /
// nonzeros from the fronts' sizes m, w.
static void size_fronts(CholPlan& P) {
  const int ns = P.ns;
  P.foff.assign(ns + 1, 0);
  P.toff.assign(ns + 1, 0);
  P.voff.assign(ns + 1, 0);
  P.flops = 0;
  P.nnzl = 0;
  for (int s = 0; s < ns; s++) {
    P.foff[s + 1] = P.foff[s] + ((front_elems(P.m[s], P.w[s]) + 15) / 16) * 16;   // 128-byte aligned fronts
    P.voff[s + 1] = P.voff[s] + ((P.m[s] + 7) / 8) * 8;
    P.toff[s + 1] = P.toff[s] + (long long)((P.w[s] + 63) / 64) * 4096;
    for (int k = 0; k < P.w[s]; k++) {
      const double r = P.m[s] - k - 1;
      P.flops += 1 + r + r * (r + 1);
      P.nnzl += r + 1;
    }
  }
  P.ftotal = P.foff[ns];
  P.ttotal = P.toff[ns];
  P.vtotal = P.voff[ns];
}

// Threads of the host planning (PGO_PLAN_THREADS, default: the hardware's, at
// most 16), kept in a pool for the process (a plan refresh runs ~10 parallel
// passes: spawning threads per pass cost more than some passes).
static int plan_threads() {
  static const int t = [] {
    if (const char* e = getenv("PGO_PLAN_THREADS")) return std::max(1, atoi(e));
    return (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  }();
  return t;
}

namespace {
class PlanPool {
 public:
  explicit PlanPool(int workers) {
    for (int i = 0; i < workers; i++) th_.emplace_back([this] { work(); });
  }
  ~PlanPool() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // fn(t) for t in [0, ntask), on the workers and the caller; one job at a time
  void run(int ntask, const std::function<void(int)>& fn) {
    if (ntask <= 1 || th_.empty()) {
      for (int t = 0; t < ntask; t++) fn(t);
      return;
    }
    std::lock_guard<std::mutex> job(job_m_);
    {
      std::lock_guard<std::mutex> lk(m_);
      fn_ = &fn;
      ntask_ = ntask;
      next_ = 0;
      busy_ = (int)th_.size();
      gen_++;
    }
    cv_.notify_all();
    for (int t; (t = next_.fetch_add(1)) < ntask;) fn(t);
    std::unique_lock<std::mutex> lk(m_);
    done_.wait(lk, [&] { return busy_ == 0; });
  }

 private:
  void work() {
    unsigned long seen = 0;
    for (;;) {
      std::unique_lock<std::mutex> lk(m_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void(int)>* fn = fn_;
      const int n = ntask_;
      lk.unlock();
      for (int t; (t = next_.fetch_add(1)) < n;) (*fn)(t);
      lk.lock();
      if (--busy_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex m_, job_m_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  int ntask_ = 0, busy_ = 0;
  std::atomic<int> next_{0};
  unsigned long gen_ = 0;
  bool stop_ = false;
};

PlanPool& plan_pool() {
  static PlanPool pool(plan_threads() - 1);
  return pool;
}
}  // namespace

void plan_parallel(int ntask, const std::function<void(int)>& fn) { plan_pool().run(ntask, fn); }

// v.resize(n) leaving room when it has to grow (the live path's plan refreshes
// then resize within capacity: no reallocation and copy of the whole list)
template <class V>
static void resize_room(V& v, size_t n) {
  if (v.capacity() < n) v.reserve(n + n / 16 + 1024);
  v.resize(n);
}

// fn(t, begin, end) on nth contiguous chunks of [0, n), chunk t by index (the
// results are independent of which thread runs it and of nth)
template <class F>
static void parallel_chunks(int n, int nth, F&& fn) {
  nth = std::max(1, std::min(nth, n));
  plan_parallel(nth, [&](int t) { fn(t, (int)((long long)n * t / nth), (int)((long long)n * (t + 1) / nth)); });
}

// One level's share of the schedule lists (chol_schedule builds the levels
// concurrently, then appends them to the plan's lists in level order).
struct LevelLists {
  std::vector<int> small_list, level_fronts, potrf_list;
  std::vector<int4> syrk_tasks, sdiag_tasks, col_tasks, bwd_tasks, bwdc_tasks, bwd_part_tasks, ea_tasks, ea_pairs;
  std::vector<int2> bwd_pref;
  std::vector<XExchange> xchg;
  std::vector<int4> xp_tasks;
  std::vector<long long> xp_loff, xp_lstride;
  long long xp_rslot = 0;
  int npart = 0;
  bool schedule_error = false;
  // empty again, capacity kept
  void reset() {
    for (auto* v : {&small_list, &level_fronts, &potrf_list}) v->clear();
    for (auto* v : {&syrk_tasks, &sdiag_tasks, &col_tasks, &bwd_tasks, &bwdc_tasks, &bwd_part_tasks, &ea_tasks, &ea_pairs,
                    &xp_tasks})
      v->clear();
    bwd_pref.clear();
    xchg.clear();
    xp_loff.clear();
    xp_lstride.clear();
    xp_rslot = 0;
    npart = 0;
    schedule_error = false;
  }
};

// The plan's schedules from its fronts (chol_analyze's second half; the
// incremental append re-runs it on the updated fronts): the subtree partition,
// the level schedules and task lists, then the H assembly lists.
static void chol_schedule(CholPlan& P, const std::vector<int>& row_ptr, const std::vector<int>& slot_col) {
  static const bool timing = getenv("PGO_PLAN_TIMING") != nullptr;
  auto tlast = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "chol_schedule %-12s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - tlast).count());
    tlast = t;
  };
  const int ns = P.ns;
  P.schedule_error = false;
  // ---- multi-GPU subtree partition (part_size > 1, DESIGN.md "Multi-GPU"):
  // rank part_rank factorises the fronts of its subtrees (phase 1), then every
  // rank the replicated top fronts (phase 2), after the subtree roots' update
  // matrices / vectors have been exchanged.  Storage only for the fronts this
  // rank touches: its own, the top, and the other ranks' subtree roots (their
  // update matrices arrive in the exchange).  One rank: everything is phase 1.
  const int psz = std::max(P.part_size, 1), prk = P.part_rank;
  P.owner = partition_subtrees(P, psz);
  P.subtree_cnt.assign(ns, 1);
  for (int s = 0; s < ns; s++)
    if (P.parent[s] >= 0) P.subtree_cnt[P.parent[s]] += P.subtree_cnt[s];
  std::vector<char> need(ns, 0);
  P.xroot.clear();
  P.xroot_rank.clear();
  for (int s = 0; s < ns; s++) {
    const bool root = P.owner[s] >= 0 && (P.parent[s] < 0 || P.owner[P.parent[s]] < 0);
    if (root) {
      P.xroot.push_back(s);
      P.xroot_rank.push_back(P.owner[s]);
    }
    need[s] = P.owner[s] == prk || P.owner[s] < 0 || (root && P.parent[s] >= 0);
  }
  if (psz > 1) {   // offsets over the needed fronts only
    for (int s = 0; s < ns; s++) {
      P.foff[s + 1] = P.foff[s] + (need[s] ? ((front_elems(P.m[s], P.w[s]) + 15) / 16) * 16 : 0);
      P.voff[s + 1] = P.voff[s] + (need[s] ? ((P.m[s] + 7) / 8) * 8 : 0);
      P.toff[s + 1] = P.toff[s] + (need[s] ? (long long)((P.w[s] + 63) / 64) * 4096 : 0);
    }
    P.ftotal = P.foff[ns];
    P.ttotal = P.toff[ns];
    P.vtotal = P.voff[ns];
  }
  // exchange layout: per rank its roots' payloads (packed lower update matrix,
  // then the update vector) back to back; the solve's: its subtrees' poses
  P.xroot_off.assign(P.xroot.size(), 0);
  P.xsize.assign(psz, 0);
  P.xsol_size.assign(psz, 0);
  P.xsol_ranges.clear();
  for (size_t q = 0; q < P.xroot.size(); q++) {
    const int sr = P.xroot[q], r = P.xroot_rank[q];
    const long long u = P.m[sr] - P.w[sr];
    P.xroot_off[q] = P.xsize[r];
    P.xsize[r] += u * (u + 1) / 2 + u;
    const int first = sr - P.subtree_cnt[sr] + 1;   // the subtree: postorder fronts [first, sr]
    P.xsol_ranges.push_back(make_int4(r, 3 * P.sfirst[first], 3 * P.sfirst[sr + 1], (int)P.xsol_size[r]));
    P.xsol_size[r] += 3LL * (P.sfirst[sr + 1] - P.sfirst[first]);
  }
  P.xmax = *std::max_element(P.xsize.begin(), P.xsize.end());
  P.xsol_max = *std::max_element(P.xsol_size.begin(), P.xsol_size.end());
  phase("partition");
  // ---- level schedules: phase 1 (this rank's subtree fronts) then phase 2 (top)
  std::vector<std::vector<int>> bylevel;
  for (int phase = 0; phase < 2; phase++) {
    int hmax = -1;
    for (int s = 0; s < ns; s++)
      if ((phase == 0 ? P.owner[s] == prk : P.owner[s] < 0)) hmax = std::max(hmax, P.height[s]);
    const size_t base = bylevel.size();
    bylevel.resize(base + hmax + 1);
    for (int s = 0; s < ns; s++)
      if ((phase == 0 ? P.owner[s] == prk : P.owner[s] < 0)) bylevel[base + P.height[s]].push_back(s);
    if (phase == 0) P.split = (int)bylevel.size();
  }
  {   // drop empty levels (a height with no front of this rank), keeping the split
    std::vector<std::vector<int>> kept;
    int split = 0;
    for (size_t L = 0; L < bylevel.size(); L++)
      if (!bylevel[L].empty()) {
        kept.push_back(std::move(bylevel[L]));
        if ((int)L < P.split) split++;
      }
    bylevel.swap(kept);
    P.split = split;
  }
  auto blocked = [&](int s) { return is_blocked(P, s); };
  // ---- distributed top (part_size > 1): the top fronts' columns are dealt to
  // the ranks instead of every rank factoring every top front.  A blocked top
  // front's pivot columns go by 64-column panel, round robin (continuing over
  // the fronts); its columns past the last whole panel (the update matrix) take
  // the rank of the parent column they extend-add into, so a rank's share of a
  // parent's columns is assembled from its own shares of the children's update
  // matrices (no exchange of update matrices between top fronts).  Small top
  // fronts (one workgroup / wavefront each) are computed by every rank (-1),
  // and so are the update columns of their children.  Each column's updates
  // are applied by its rank only, with the same tasks (same depths, same
  // order) as the one-rank plan: bitwise the one-rank factor.  A rank receives
  // every panel (broadcast by its owner right after it is factored) for its own
  // columns' updates and the replicated backward solve.
  // (PGO_DIST_TOP=0: the top fronts replicated on every rank instead -- the
  // previous scheme, kept as a reference for the host self-test)
  const bool dtop = psz > 1 && !(getenv("PGO_DIST_TOP") && atoi(getenv("PGO_DIST_TOP")) == 0);
  P.cown_off.assign(ns, -1);
  P.cown.clear();
  if (dtop) column_owners(P, P.owner, psz, P.cown_off, P.cown);
  P.xchg.clear();
  P.xp_tasks.clear();
  P.xp_loff.clear();
  P.xp_lstride.clear();
  P.xp_rslot = 0;
  // an exchange point: every panel / tail in `items` (front, kn, nb | kind << 16,
  // owner) goes from its owner to every rank (one broadcast per sending rank)
  auto add_exchange = [&](LevelLists& S, const std::vector<int4>& items) -> int {
    if (items.empty()) return -1;
    XExchange x;
    x.off = (int)S.xp_tasks.size();
    x.cnt = (int)items.size();
    x.size.assign(psz, 0);
    for (const int4& t : items) {
      const int s = t.x, kn = t.y, nb = t.z & 0xffff, kind = t.z >> 16, m = P.m[s];
      // kind 0: the L below the diagonal tile (the tile's own L is never stored),
      // the inverse, the frontal vector; kind 1: the tail columns whole
      const long long sz = kind == 0 ? (long long)(m - kn - nb) * nb + 4096 + (m - kn) : (long long)(m - kn) * nb;
      S.xp_tasks.push_back(t);
      S.xp_loff.push_back(x.size[t.w]);
      x.size[t.w] += sz;
    }
    for (int q = x.off; q < x.off + x.cnt; q++) S.xp_lstride.push_back(x.size[S.xp_tasks[q].w]);
    for (long long v : x.size) S.xp_rslot = std::max(S.xp_rslot, v);
    S.xchg.push_back(x);
    return (int)S.xchg.size() - 1;
  };
  const int nl = (int)bylevel.size();
  P.levels.assign(nl, CholLevel());
  // one level's schedule into its own lists (offsets level-relative; merged
  // below in level order, so the plan is the same for any thread count)
  auto schedule_level = [&](int L, LevelLists& S, int part) {
    CholLevel& lv = P.levels[L];
    // distributed top level: this rank generates only the tasks of its columns
    const bool dist = dtop && L >= P.split;
    auto mine = [&](int s, int col) {
      if (!dist) return true;
      const int o = P.cown[P.cown_off[s] + col];
      return o < 0 || o == prk;
    };
    auto cowner = [&](int s, int col) { return dist ? P.cown[P.cown_off[s] + col] : -1; };
    // part 0: the front list, the backward-solve and assembly lists (members of
    // S and lv disjoint from part 1's: the two parts of a level run concurrently)
    if (part == 0) {
      lv.front_off = (int)S.level_fronts.size();
      lv.front_cnt = (int)bylevel[L].size();
      for (int s : bylevel[L]) {
        S.level_fronts.push_back(s);
        lv.maxm = std::max(lv.maxm, P.m[s]);
        if (P.m[s] <= kSmallFront) lv.small_maxm = std::max(lv.small_maxm, P.m[s]);
      }
      // blocked backward solve (64-column blocks of each front's pivot columns);
      // the forward substitution is carried by the factorisation
      for (int s : bylevel[L]) lv.maxblk = std::max(lv.maxblk, (P.w[s] + 63) / 64);
      {                                            // backward init: all columns vs the rows below w
        // partial products L21[r0:r0+kBwdRows, block]' x_below, one task each,
        // reduced in fixed order by the init task of the block
        SolveStep sp{(int)S.bwd_part_tasks.size(), 0};
        SolveStep st{(int)S.bwd_tasks.size(), 0};
        for (int s : bylevel[L]) {
          const int w = P.w[s], m = P.m[s], nblk = (w + 63) / 64;
          for (int b = 0; b < nblk; b++) {
            const int p0 = S.npart;
            for (int r0 = w; r0 < m; r0 += kBwdRows) S.bwd_part_tasks.push_back(make_int4(s, b * 64, r0, S.npart++));
            S.bwd_tasks.push_back(make_int4(s, b * 64, std::min(b * 64 + 64, w), b == nblk - 1 ? b : -1));
            S.bwd_pref.push_back(make_int2(p0, S.npart - p0));
          }
        }
        sp.cnt = (int)S.bwd_part_tasks.size() - sp.off;
        for (int q = sp.off; q < sp.off + sp.cnt; q++) {
          const int4 t = S.bwd_part_tasks[q];
          const double ncol = std::min(64, P.w[t.x] - t.y), rows = std::min(kBwdRows, P.m[t.x] - t.z);
          lv.bwd_part_flops += 2.0 * ncol * rows;
          // L rows x columns, x gathered per row (+ its pose index per 3 rows), the 64 partial sums out
          lv.bwd_part_bytes += 8.0 * ncol * rows + rows * (8.0 + 4.0 / 3.0) + 8.0 * 64;
        }
        st.cnt = (int)S.bwd_tasks.size() - st.off;
        for (int q = st.off; q < st.off + st.cnt; q++) {   // init: partials + y in, X_jj' z for the last block, x out
          const int4 t = S.bwd_tasks[q];
          const double n2 = t.z - t.y, np = S.bwd_pref[q].y;
          lv.bwd_init_bytes += 8.0 * n2 * (np + 2.0) + (t.w >= 0 ? 8.0 * n2 * (64.0 + 1.0) + 4.0 * n2 / 3.0 : 0.0);
        }
        // frontal vectors: own rows gathered from the permuted rhs, the children's
        // update vectors with their row maps, the vector written
        for (int s : bylevel[L]) {
          lv.vec_bytes += 8.0 * P.m[s] + (8.0 + 4.0 / 3.0) * P.w[s];
          for (int q = P.cptr[s]; q < P.cptr[s + 1]; q++) lv.vec_bytes += (8.0 + 4.0 / 3.0) * (P.m[P.children[q]] - P.w[P.children[q]]);
        }
        lv.bwd_part = sp;
        lv.bwd.push_back(st);
      }
      {   // the same steps as one chained launch (k_bwd_chain): block j of a front
          // after the blocks above it, tasks ordered by distance from the last
          // block so that every workgroup waits only on earlier-dispatched ones
        lv.bwdc.off = (int)S.bwdc_tasks.size();
        for (int d = 1; d < lv.maxblk; d++)
          for (int s : bylevel[L]) {
            const int w = P.w[s], nblk = (w + 63) / 64;
            if (d >= nblk) continue;
            const int j = nblk - 1 - d;
            S.bwdc_tasks.push_back(make_int4(s, j * 64, j * 64 + 64, j));
            // L[block b, block j] for every block b below j and its x_b, X_jj, z in, x out
            const double n2 = std::min(64, w - 64 * j);
            lv.bwd_chain_bytes += 8.0 * (w - 64.0 * (j + 1)) * (n2 + 1.0) + 8.0 * n2 * (64.0 + 3.0) + 4.0 * n2 / 3.0;
          }
        lv.bwdc.cnt = (int)S.bwdc_tasks.size() - lv.bwdc.off;
      }
      for (int b = lv.maxblk - 1; b >= 1; b--) {   // backward step b: columns left of block b
        SolveStep st{(int)S.bwd_tasks.size(), 0};
        for (int s : bylevel[L]) {
          const int w = P.w[s], nblk = (w + 63) / 64;
          if (b >= nblk) continue;
          for (int c = 0; c < b; c++)
          {
            S.bwd_tasks.push_back(make_int4(s, c * 64, c * 64 + 64, c == b - 1 ? c : -1));
            S.bwd_pref.push_back(make_int2(0, 0));
          }
        }
        st.cnt = (int)S.bwd_tasks.size() - st.off;
        lv.bwd.push_back(st);
      }
      // assembly: one task per 64x64 tile of every front's lower triangle, which
      // it writes whole: its H entries (+ lambda on the diagonal), then the
      // update-matrix elements of the front's children in order (fixed
      // summation order, no atomics), each child contributing a rectangle of its
      // update matrix (child rows [a0, a0+nr) x columns [b0, b0+nc), the rows /
      // columns whose parent index falls in the tile).  No front is zeroed.
      lv.ea_off.push_back((int)S.ea_tasks.size());
      std::vector<int> tcnt, tpos;
      std::vector<int4> runs;   // (child, tile, first child row, rows) of every child, children in order
      for (int sp : bylevel[L]) {
        const int nt = (P.m[sp] + 63) / 64;
        tcnt.assign((size_t)nt * (nt + 1) / 2, 0);
        runs.clear();
        std::vector<int> cr(1, 0);   // runs of child q: [cr[q], cr[q + 1])
        for (int q = P.cptr[sp]; q < P.cptr[sp + 1]; q++) {
          const int c = P.children[q];
          const int u = P.m[c] - P.w[c];
          const size_t r0 = runs.size();
          const int* rel = P.ea_rel.data() + P.ea_ptr[c];
          auto add = [&](int t, int a, int nr) {
            if (runs.size() == r0 || runs.back().y != t) runs.push_back(make_int4(c, t, a, 0));
            runs.back().w += nr;
          };
          // (row a of the update matrix: parent row 3 rel[a / 3] + a % 3; a pose's
          // three rows in one tile go as one)
          for (int a = 0; a < u; a += 3) {
            const int r = 3 * rel[a / 3];
            if ((r >> 6) == ((r + 2) >> 6) && a + 3 <= u) {
              add(r >> 6, a, 3);
            } else {
              for (int k = 0; k < 3 && a + k < u; k++) add((r + k) >> 6, a + k, 1);
            }
          }
          for (size_t i = r0; i < runs.size(); i++)   // a child's runs are in increasing tiles: one pair per tile
            for (size_t j = r0; j <= i; j++) tcnt[(size_t)runs[i].y * (runs[i].y + 1) / 2 + runs[j].y]++;
          cr.push_back((int)runs.size());
        }
        const int base = (int)S.ea_pairs.size();
        tpos.assign(tcnt.size(), 0);
        for (size_t k = 1; k < tcnt.size(); k++) tpos[k] = tpos[k - 1] + tcnt[k - 1];
        for (int ti = 0; ti < nt; ti++)
          for (int tj = 0; tj <= ti; tj++) {
            const size_t k = (size_t)ti * (ti + 1) / 2 + tj;
            S.ea_tasks.push_back(make_int4(sp, (ti << 16) | tj, base + tpos[k], tcnt[k]));
          }
        S.ea_pairs.resize(base + (tcnt.empty() ? 0 : tpos.back() + tcnt.back()));
        for (size_t q = 0; q + 1 < cr.size(); q++)   // children in order: their pairs in order within every tile
          for (int i = cr[q]; i < cr[q + 1]; i++)
            for (int j = cr[q]; j <= i; j++) {
              const size_t k = (size_t)runs[i].y * (runs[i].y + 1) / 2 + runs[j].y;
              S.ea_pairs[base + tpos[k]++] = make_int4(runs[i].x, runs[i].z, runs[j].z, runs[i].w | (runs[j].w << 8));
            }
      }
      ea_xcd_order(S.ea_tasks, (size_t)lv.ea_off.back());
      lv.ea_cnt.push_back((int)S.ea_tasks.size() - lv.ea_off.back());
      return;
    }
    // part 1: the factorisation lists (small-front classes, blocked panel steps)
    // small fronts (m <= kSmallFront): with w <= kWaveW one wavefront each (the
    // m x w panel in LDS, the rank-w Schur update streamed), largest first;
    // else one workgroup each with the whole front in LDS, launched per size
    // class so the LDS request (m^2 doubles) does not cap the occupancy
    std::vector<int> big;
    {
      const int classes[4] = {32, 64, 96, kSmallFront};
      std::vector<int> bucket[4], wave;
      for (int s : bylevel[L]) {
        // w > kWaveW: the blocked path (64-column panels, every front of the
        // level in the same launches) -- a whole-front-in-LDS workgroup runs
        // its w pivots one after the other at ~2 us each
        if (blocked(s)) {
          big.push_back(s);
          continue;
        }
        if (P.w[s] <= kWaveW) {
          wave.push_back(s);
          continue;
        }
        int q = 0;
        while (P.m[s] > classes[q]) q++;
        bucket[q].push_back(s);
      }
      // m <= 64 (one row per lane) | 64 < m <= 128 | 128 < m <= 256 (four waves)  x  w <= 8 | 16 | 32
      // (the four-wave class has no W = 8 form: its w <= 8 fronts go with W = 16)
      for (int cls = 0; cls < 9; cls++) {
        const int rc = cls / 3, W = cls % 3 == 0 ? 8 : cls % 3 == 1 ? 16 : kWaveW;
        const int Wlo = cls % 3 == 0 ? 0 : (rc == 2 && W == 16 ? 0 : W / 2);
        if (rc == 2 && W == 8) continue;
        std::vector<int> part;
        for (int s : wave) {
          const int mc = P.m[s] <= 64 ? 0 : P.m[s] <= kSmallFront ? 1 : 2;
          if (mc == rc && P.w[s] > Wlo && P.w[s] <= W) part.push_back(s);
        }
        if (part.empty()) continue;
        std::stable_sort(part.begin(), part.end(), [&](int a, int b) {
          const double wa = (double)P.m[a] * P.m[a] * P.w[a], wb = (double)P.m[b] * P.m[b] * P.w[b];
          return wa > wb;
        });
        SmallClass sc{(int)S.small_list.size(), (int)part.size(), 0, W};
        for (int s : part) {
          S.small_list.push_back(s);
          sc.mmax = std::max(sc.mmax, P.m[s]);
          sc.flops += front_flops(P.m[s], P.w[s]);
        }
        lv.small.push_back(sc);
      }
      for (int q = 0; q < 4; q++) {
        if (bucket[q].empty()) continue;
        SmallClass sc{(int)S.small_list.size(), (int)bucket[q].size(), 0, 0};
        for (int s : bucket[q]) {
          S.small_list.push_back(s);
          sc.mmax = std::max(sc.mmax, P.m[s]);
          sc.flops += front_flops(P.m[s], P.w[s]);
        }
        lv.small.push_back(sc);
      }
    }
    int maxw = 0;
    for (int s : big) maxw = std::max(maxw, P.w[s]);
    // Blocked path, one step per 64-column panel kb of every big front of the
    // level (right-looking, look-ahead 1, Schur updates of depth 64):
    //   first step  k_panel_first: the front's first diagonal tile factored +
    //               inverted, the rows below it solved (trsm) by workgroups that
    //               wait for that inverse (in-launch hand-off)
    //   each step   k_step: the next panel's diagonal tile updated with panel kb,
    //               factored and inverted (sdiag); the tiles below it in the
    //               next panel's column block updated, then solved against that
    //               inverse (col); the other trailing tiles updated (syrk:
    //               inline, or a concurrent k_panel_syrk_lds / 128 launch)
    // Look-ahead bookkeeping: applied[i][j] = the first panel column whose
    // Schur update column j of big front i has not received yet (every task
    // updates whole columns: rows from the column down).  A step's tasks must
    // find their columns uniform; a violation drops the step's skip (below) or
    // marks the plan invalid (schedule_error).
    std::vector<std::vector<int>> applied(big.size());
    for (size_t i = 0; i < big.size(); i++) applied[i].assign(P.m[big[i]], 0);
    auto uniform = [&](size_t i, int c0, int c1, int k0) {
      for (int j = c0; j < c1; j++)
        if (applied[i][j] != k0) return false;
      return true;
    };
    bool apart_chain = false;   // once a step's plain tiles go to their own launch, the later ones do too
    // deferred far updates (apart steps at a kKB block end): per step and big
    // front, the largest column its k_step tasks and near plain tiles touch
    // (touch), and the first column of its far plain tiles (far0, m = none)
    // far0[step][piece][front]: the far pieces are the far range cut at the kKB
    // blocks (the update-matrix columns past w one piece), each joined on its own
    std::vector<std::vector<int>> touch;
    std::vector<std::vector<std::vector<int>>> far0;
    for (int kb = 0; kb < maxw; kb += kNB) {
      touch.emplace_back(big.size(), 0);
      far0.emplace_back();
      PanelStep ps;
      ps.kb = kb;
      ps.syrk_flops = ps.plain_flops = ps.step_flops = ps.first_flops = 0;
      ps.col_off = (int)S.col_tasks.size();
      ps.syrk_off = (int)S.syrk_tasks.size();
      ps.potrf_off = (int)S.potrf_list.size();
      ps.sdiag_off = (int)S.sdiag_tasks.size();
      // first panel of a front: k_panel_first (diagonal + trsm waiters)
      std::vector<int4> xfirst, xstep;   // distributed top: panels factored by the first / the step launch
      for (int s : big) {
        if (kb != 0 || P.w[s] <= 0) continue;
        const int nb = std::min(kNB, P.w[s]), m = P.m[s];
        if (dist) xfirst.push_back(make_int4(s, 0, nb, cowner(s, 0)));
        if (!mine(s, 0)) continue;
        S.potrf_list.push_back(s);
        ps.first_flops += 2.0 * nb * nb * (double)nb / 3.0 + (double)std::max(0, m - nb) * nb * nb;
      }
      ps.potrf_cnt = (int)S.potrf_list.size() - ps.potrf_off;
      for (int s : big)
        if (kb == 0 && P.w[s] > 0 && mine(s, 0))
          for (int r0 = kNB; r0 < P.m[s]; r0 += kNB) S.col_tasks.push_back(make_int4(s, r0, 0, -1));
      ps.fcol_cnt = (int)S.col_tasks.size() - ps.col_off;
      ps.xfirst = add_exchange(S, xfirst);
      // this panel's Schur update, deferred by kKB-column blocks: inside a block
      // only the block's remaining columns [kn, be) are updated ("inner", bit 31
      // of k0: tasks clip columns at the block end); after the block's last
      // panel the trailing columns [be, m) get the whole block's update.
      // With the plain tiles in their own launch (apart) the column block the
      // next step prepares, [kn + 64, kn + 128), is skipped: the next step's
      // diagonal / column tasks apply this panel's update with their own
      // (depth 2 panels, or the deferred block + 1 panel), so the next step
      // does not wait for this step's plain tiles (joined one step later).
      // The skip is a property of the front alone (its size), never of the
      // level it sits in: the update grouping -- hence the rounding -- of a
      // front is the same in every plan (the partitioned plans' fronts are bit
      // for bit the one-rank plan's).
      const bool lookahead = !getenv("PGO_NO_LOOKAHEAD");
      const bool far_on = getenv("PGO_FAR") && atoi(getenv("PGO_FAR")) == 1;
      // (PGO_LOOKAHEAD_M: the front height threshold, a test knob)
      const int la_m = getenv("PGO_LOOKAHEAD_M") ? atoi(getenv("PGO_LOOKAHEAD_M")) : kLookaheadM;
      auto front_skip = [&](int s) { return lookahead && P.m[s] >= la_m; };
      // Prep (look-ahead fronts): the step also brings the column block after
      // the next one, [kn + 64, kn + 128), up to date with the panels before kn
      // (k_step workgroups beside the diagonal chain), so the next step's
      // diagonal and column tasks apply one panel only; the plain tiles skip
      // that block too.  Only for whole 64-column pivot blocks.
      auto has_prep = [&](int s, int kn_) { return front_skip(s) && kn_ + 2 * kNB <= P.w[s]; };
      auto plain_range = [&](int s, bool skip, int& cstart, int& cend) {
        const int w = P.w[s], m = P.m[s], nb = std::min(kNB, w - kb), kn = kb + nb;
        const int bs = kb & ~(kKB - 1), be = std::min(bs + kKB, w);
        const bool inner = kn < be;
        cend = inner ? be : m;
        cstart = kn < w ? kn + kNB : kn;
        if (skip && kn + kNB < w) {   // the next step prepares [kn2, kn2 + 64): only when it covers all of it
          const int kn2 = kn + kNB, bs2 = kn & ~(kKB - 1), be2 = std::min(bs2 + kKB, w);
          const int colend2 = kn2 < be2 ? be2 : m;
          if (std::min(kn2 + kNB, colend2) == kn2 + kNB && cstart + kNB <= cend) {
            cstart += kNB;
            if (has_prep(s, kn2)) cstart += kNB;   // the next step's prep block
          }
        }
      };
      auto ntiles = [&](int T) {
        long long cnt = 0;
        for (int s : big) {
          if (P.w[s] <= kb) continue;
          int c0, c1;
          plain_range(s, front_skip(s), c0, c1);
          for (int cc = c0; cc < c1; cc += T) cnt += (P.m[s] - cc + T - 1) / T;
        }
        return cnt;
      };
      // plain tiles: 128x128 (LDS-pipelined kernel) when there are many rounds of
      // them (measured: at <= ~500 tiles the 64x64 kernel's finer granularity
      // wins, scripts/ubench_syrk.hip), else 64x64; few 64-tiles ride in k_step,
      // many go to a concurrent launch (k_step's LDS request, sized for the
      // diagonal workgroups, halves their occupancy)
      // (PGO_BIGTILE_MIN: the 128-tile threshold, a tuning knob)
      static const long long big_min = getenv("PGO_BIGTILE_MIN") ? atoll(getenv("PGO_BIGTILE_MIN")) : 4096;
      const int tile0 = ntiles(kBigTile) >= big_min ? kBigTile : kTile;
      const bool apart = apart_chain || !(tile0 == kTile && ntiles(kTile) <= kInlineTiles);
      std::vector<int4> plain;   // (front, first column, end column, k0): rows from the column down
      // ... the far part of an apart step's plain range (a kKB block end: the
      // columns past the next block, [be + kKB, m)): its own launch on a fourth
      // stream, joined only before the first later step that touches them
      std::vector<std::vector<int4>> plain_far;   // [piece]: the ranges of every front's piece g
      std::vector<double> far_pflops;
      std::vector<int4> prep;    // prep tiles (front, r0, c0, k0), whole 64x64 tiles
      bool conflict = false;   // a front's next step reads this step's plain tiles
      for (size_t i = 0; i < big.size(); i++) {
        const int s = big[i];
        if (P.w[s] <= kb) continue;
        const int w = P.w[s], m = P.m[s];
        const int nb = std::min(kNB, w - kb), kn = kb + nb;
        const int bs = kb & ~(kKB - 1), be = std::min(bs + kKB, w);
        const bool inner = kn < be;
        const int colend = inner ? be : m;   // the device's column clip
        if (kn < w) {   // next panel: its diagonal tile and the tiles below it
          const int nb2 = std::min(kNB, w - kn), c1 = std::min(kn + kNB, colend);
          const int k0 = applied[i][kn];
          if (!uniform(i, kn, c1, k0)) {
            if (getenv("PGO_SCHED_DEBUG") && !S.schedule_error)
              fprintf(stderr, "sched: sdiag front %d w %d m %d kb %d cols [%d,%d) k0 %d\n", s, w, m, kb, kn, c1, k0);
            S.schedule_error = true;
          }
          for (int j = kn; j < c1; j++) applied[i][j] = kn;
          touch.back()[i] = std::max(touch.back()[i], c1);
          const int depth = kn - k0, kw = inner ? (k0 | (int)0x80000000) : k0;
          if (dist) xstep.push_back(make_int4(s, kn, nb2, cowner(s, kn)));
          const bool own = mine(s, kn);
          if (own) S.sdiag_tasks.push_back(make_int4(s, kn, kn, kw));
          const double fd = (double)depth * kNB * (kNB + 1) + 2.0 * nb2 * nb2 * (double)nb2 / 3.0 +
                            (double)std::min(kNB - nb2, m - kn - nb2) * nb2 * nb2;
          ps.step_flops += fd;
          ps.diag_flops += fd;
          for (int r0 = kn + kNB; r0 < m; r0 += kNB) {
            if (own) S.col_tasks.push_back(make_int4(s, r0, kn, kw));
            const int rows = std::min(kNB, m - r0);
            ps.step_flops += 2.0 * depth * rows * (c1 - kn) + (double)rows * nb2 * nb2;
            ps.colupd_flops += 2.0 * depth * rows * (c1 - kn);
            ps.trsm_flops += (double)rows * nb2 * nb2;
          }
          ps.syrk_flops += (double)depth * (c1 - kn) * (2.0 * m - kn - c1 + 1.0);
        }
        if (has_prep(s, kn)) {
          const int b0 = kn + kNB, b1 = b0 + kNB, k0 = applied[i][b0];
          if (!uniform(i, b0, b1, k0) || k0 > kb) {
            if (getenv("PGO_SCHED_DEBUG") && !S.schedule_error)
              fprintf(stderr, "sched: prep front %d w %d m %d kb %d cols [%d,%d) k0 %d\n", s, w, m, kb, b0, b1, k0);
            S.schedule_error = true;
          }
          for (int j = b0; j < b1; j++) applied[i][j] = kn;
          touch.back()[i] = std::max(touch.back()[i], b1);
          if (mine(s, b0))
            for (int r0 = b0; r0 < m; r0 += kNB) prep.push_back(make_int4(s, r0, b0, k0));
          const double f = (double)(kn - k0) * kNB * (2.0 * m - b0 - b1 + 1.0);
          ps.step_flops += f;
          ps.colupd_flops += f;
          ps.syrk_flops += f;
        }
        int cstart, cend;
        plain_range(s, front_skip(s), cstart, cend);
        // far split at a block end: columns past the next kKB block (the next
        // steps touch none of them until that block ends)
        // (PGO_FAR=1: measured within the replay noise on C3 -- 8.70 / 17.50 ms
        // at 1 / 3 lanes with and without, profiles/r04c_ab_far.txt -- while
        // the concurrent far tiles slow the k_step launches they overlap; off)
        const int nend = (!inner && cstart < cend && far_on) ? std::max(cstart, std::min(cend, std::min(be + kKB, w)))
                                                             : cend;
        if (kn + kNB < w && cstart < nend) {   // the next step prepares [kn2, c2) of this front
          const int kn2 = kn + kNB, bs2 = kn & ~(kKB - 1), be2 = std::min(bs2 + kKB, w);
          const int c2 = std::min(kn2 + kNB, kn2 < be2 ? be2 : m);
          if (cstart < c2 && kn2 < nend) conflict = true;   // this step's plain tiles feed it: lag 1
        }
        if (cstart < cend) {
          int k0 = applied[i][cstart];
          if (!uniform(i, cstart, cend, k0)) {
            if (getenv("PGO_SCHED_DEBUG") && !S.schedule_error) {
              fprintf(stderr, "sched: plain front %d w %d m %d kb %d cols [%d,%d) k0 %d:", s, w, m, kb, cstart, cend, k0);
              for (int j = cstart; j < cend; j += 16) fprintf(stderr, " %d", applied[i][j]);
              fprintf(stderr, "\n");
            }
            S.schedule_error = true;
            k0 = kb;
          }
          for (int j = cstart; j < cend; j++) applied[i][j] = kn;
          const int depth = kn - k0, kw = inner ? (k0 | (int)0x80000000) : k0;
          for (int cc = cstart; cc < cend; cc++) ps.plain_flops += 2.0 * depth * (m - cc);
          if (cstart < nend) plain.push_back(make_int4(s, cstart, nend, kw));
          touch.back()[i] = std::max(touch.back()[i], nend);
          for (int c0 = nend, g = 0; c0 < cend; g++) {   // far pieces: a kKB block each, [w, m) one
            const int c1 = c0 < w ? std::min(std::min(cend, w), (c0 / kKB + 1) * kKB) : cend;
            if ((int)plain_far.size() <= g) {
              plain_far.emplace_back();
              far_pflops.push_back(0.0);
              far0.back().emplace_back(big.size(), 0);
              for (size_t i2 = 0; i2 < big.size(); i2++) far0.back()[g][i2] = P.m[big[i2]];
            }
            plain_far[g].push_back(make_int4(s, c0, c1, kw));
            far0.back()[g][i] = c0;
            for (int cc = c0; cc < c1; cc++) far_pflops[g] += 2.0 * depth * (m - cc);
            c0 = c1;
          }
        }
      }
      ps.syrk_flops += ps.plain_flops;
      ps.sdiag_cnt = (int)S.sdiag_tasks.size() - ps.sdiag_off;
      ps.col_cnt = (int)S.col_tasks.size() - ps.col_off - ps.fcol_cnt;
      S.col_tasks.insert(S.col_tasks.end(), prep.begin(), prep.end());
      ps.prep_cnt = (int)prep.size();
      long long cnt128 = 0;
      for (const int4& u : plain)
        for (int c0 = u.y; c0 < u.z; c0 += kBigTile) cnt128 += (P.m[u.x] - c0 + kBigTile - 1) / kBigTile;
      for (const auto& pl : plain_far)
        for (const int4& u : pl)
          for (int c0 = u.y; c0 < u.z; c0 += kBigTile) cnt128 += (P.m[u.x] - c0 + kBigTile - 1) / kBigTile;
      // (distributed top: 64-wide tiles, split where the column owner changes;
      // a tile's elements are computed alike in either kernel, so this is
      // bitwise the 128-tile update)
      ps.syrk_tile = cnt128 >= big_min && !dist ? kBigTile : kTile;
      // A tile's columns stay inside one 64-column block of the packed front
      // (pgo_chol.h front_packed): a range starting inside a block (the update
      // matrix starts at w) opens with a narrow tile up to the block's end,
      // clipped; a tile's elements are computed alike whatever its shape
      auto gen_tiles = [&](const std::vector<int4>& ranges) {
      for (const int4& u : ranges)
        for (int c0 = u.y; c0 < u.z;) {
          const int T = ps.syrk_tile;
          const int ce = (c0 & 63) ? std::min(u.z, (c0 + 63) & ~63) : std::min(u.z, c0 + T);
          // a tile narrower than T carries its width (the kernels clip its columns
          // there): a block's end inside the range, or the range's end -- which
          // is not the kernels' own column end where a step's range is split
          // into near and far parts
          const bool narrow = ce - c0 < T;
          if (!dist) {
            const int clip = narrow ? ce - c0 : 0;
            for (int r0 = c0; r0 < P.m[u.x]; r0 += T) S.syrk_tasks.push_back(make_int4(u.x, r0 | (clip << kClipShift), c0, u.w));
          } else {
            for (int a = c0; a < ce;) {   // runs of one column owner: (a, b)
              int b = a + 1;
              while (b < ce && cowner(u.x, b) == cowner(u.x, a)) b++;
              if (mine(u.x, a)) {
                const int clip = (a == c0 && b == ce && !narrow) ? 0 : b - a;
                for (int r0 = c0; r0 < P.m[u.x]; r0 += kTile)
                  S.syrk_tasks.push_back(make_int4(u.x, r0 | (clip << kClipShift), a, u.w));
              }
              a = b;
            }
          }
          c0 = ce;
        }
      };
      gen_tiles(plain);
      const int near_end = (int)S.syrk_tasks.size();
      std::vector<int> piece_end;
      for (const auto& pl : plain_far) {
        gen_tiles(pl);
        piece_end.push_back((int)S.syrk_tasks.size());
      }
      ps.syrk_cnt = (int)S.syrk_tasks.size() - ps.syrk_off;
      ps.syrk_inline = !apart && ps.syrk_tile == kTile && ps.syrk_cnt <= kInlineTiles;
      ps.far_cnt = ps.syrk_inline ? 0 : (int)S.syrk_tasks.size() - near_end;
      auto xcd = [&](int b, int e) {   // XCD-aware order of a launch's Schur-update tiles
        std::vector<int4> mine(S.syrk_tasks.begin() + b, S.syrk_tasks.begin() + e);
        xcd_order(mine, ps.syrk_tile);
        std::copy(mine.begin(), mine.end(), S.syrk_tasks.begin() + b);
      };
      if (ps.far_cnt == 0) {   // (inline, or nothing far: the far ranges' columns are this step's)
        for (const auto& pl : plain_far)
          for (const int4& u : pl)
            for (size_t i = 0; i < big.size(); i++)
              if (big[i] == u.x) touch.back()[i] = std::max(touch.back()[i], u.z);
        far0.back().clear();
        xcd(ps.syrk_off, ps.syrk_off + ps.syrk_cnt);
      } else {
        xcd(ps.syrk_off, near_end);
        ps.far_p0 = (int)lv.far_pieces.size();
        int b = near_end;
        for (size_t g = 0; g < plain_far.size(); g++) {   // (piece: first tile relative to syrk_off, count)
          xcd(b, piece_end[g]);
          lv.far_pieces.push_back(make_int4((int)lv.panels.size(), b - ps.syrk_off, piece_end[g] - b, -1));
          lv.far_piece_flops.push_back(far_pflops[g]);   // (a piece may hold no tile of this rank)
          ps.far_flops += far_pflops[g];
          b = piece_end[g];
        }
        ps.far_np = (int)lv.far_pieces.size() - ps.far_p0;
      }
      // an apart launch no front's next step reads is joined before the step after next
      ps.plain_lag = ps.syrk_cnt > 0 && !ps.syrk_inline ? (conflict ? 1 : 2) : 0;
      // (an inline plain after a lag-2 apart one could touch its tiles at once)
      apart_chain = apart_chain || (ps.plain_lag == 2);
      if (ps.syrk_inline) ps.step_flops += ps.plain_flops;
      ps.xstep = add_exchange(S, xstep);
      lv.panels.push_back(ps);
    }
    // a far piece is joined before the first later step whose k_step tasks or
    // near plain tiles touch one of its columns (-1: at the level's end)
    for (size_t q = 0; q < lv.far_pieces.size(); q++) {
      int4& fp = lv.far_pieces[q];
      const int j = fp.x, g = (int)q - lv.panels[j].far_p0;
      const std::vector<int>& f0 = far0[j][g];
      fp.w = -1;
      for (size_t j2 = j + 1; j2 < lv.panels.size() && fp.w < 0; j2++)
        for (size_t i = 0; i < big.size(); i++)
          if (touch[j2][i] > f0[i]) {
            fp.w = (int)j2;
            break;
          }
    }
    if (dist) {   // update columns past a front's last whole panel, factored with it: to every rank
      std::vector<int4> tails;
      for (int s : big) {
        const int w = P.w[s], wr = std::min(P.m[s], (w + kNB - 1) / kNB * kNB);
        if (wr > w) tails.push_back(make_int4(s, w, (wr - w) | (1 << 16), cowner(s, w)));
      }
      lv.xtail = add_exchange(S, tails);
    }
    // every column has its updates: pivot columns up to their panel, the
    // trailing ones from every panel
    for (size_t i = 0; i < big.size(); i++) {
      const int s = big[i], w = P.w[s];
      for (int j = 0; j < P.m[s]; j++)
        if (applied[i][j] != (j < w ? (j / kNB) * kNB : w)) {
          if (getenv("PGO_SCHED_DEBUG") && !S.schedule_error)
            fprintf(stderr, "sched: end front %d w %d m %d col %d applied %d\n", s, w, P.m[s], j, applied[i][j]);
          S.schedule_error = true;
        }
    }
  };
  // the level lists keep their storage from one schedule to the next in the
  // plan (a live plan refresh rebuilds them all: fresh allocations cost it the
  // page faults of ~tens of MB); chol_free releases them with the plan
  if (!P.sched_scratch.p) P.sched_scratch.p = std::make_shared<std::vector<LevelLists>>();
  std::vector<LevelLists>& out = *static_cast<std::vector<LevelLists>*>(P.sched_scratch.p.get());
  if ((int)out.size() < nl) out.resize(nl);
  for (int L = 0; L < nl; L++) out[L].reset();
  std::vector<double> lms(2 * nl, 0.0);
  plan_parallel(2 * nl, [&](int t) {
    const auto t0 = std::chrono::steady_clock::now();
    schedule_level(t >> 1, out[t >> 1], t & 1);
    lms[t] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  });
  if (timing) {
    for (int L = 0; L < nl; L++)
      fprintf(stderr, "  level %d: %.2f + %.2f ms (%zu fronts)\n", L, lms[2 * L], lms[2 * L + 1], bylevel[L].size());
    phase("levels");
  }
  // merge: level-relative offsets and indices made absolute; the level lists
  // copied into place level by level on the pool (offsets from a serial pass)
  struct Base {
    size_t small_list, level_fronts, potrf_list, syrk_tasks, sdiag_tasks, col_tasks, bwd_tasks, bwdc_tasks, bwd_pref,
        bwd_part_tasks, ea_tasks, ea_pairs, xchg, xp_tasks, xp_loff, xp_lstride;
    int npart;
  };
  std::vector<Base> base(nl + 1);
  {
    Base z{};
    for (int L = 0; L < nl; L++) {
      const LevelLists& S = out[L];
      base[L] = z;
      z.small_list += S.small_list.size();
      z.level_fronts += S.level_fronts.size();
      z.potrf_list += S.potrf_list.size();
      z.syrk_tasks += S.syrk_tasks.size();
      z.sdiag_tasks += S.sdiag_tasks.size();
      z.col_tasks += S.col_tasks.size();
      z.bwd_tasks += S.bwd_tasks.size();
      z.bwdc_tasks += S.bwdc_tasks.size();
      z.bwd_pref += S.bwd_pref.size();
      z.bwd_part_tasks += S.bwd_part_tasks.size();
      z.ea_tasks += S.ea_tasks.size();
      z.ea_pairs += S.ea_pairs.size();
      z.xchg += S.xchg.size();
      z.xp_tasks += S.xp_tasks.size();
      z.xp_loff += S.xp_loff.size();
      z.xp_lstride += S.xp_lstride.size();
      z.npart += S.npart;
    }
    base[nl] = z;
  }
  const Base& tot = base[nl];
  resize_room(P.small_list, tot.small_list);
  resize_room(P.level_fronts, tot.level_fronts);
  resize_room(P.potrf_list, tot.potrf_list);
  resize_room(P.syrk_tasks, tot.syrk_tasks);
  resize_room(P.sdiag_tasks, tot.sdiag_tasks);
  resize_room(P.col_tasks, tot.col_tasks);
  resize_room(P.bwd_tasks, tot.bwd_tasks);
  resize_room(P.bwdc_tasks, tot.bwdc_tasks);
  resize_room(P.bwd_pref, tot.bwd_pref);
  resize_room(P.bwd_part_tasks, tot.bwd_part_tasks);
  resize_room(P.ea_tasks, tot.ea_tasks);
  resize_room(P.ea_pairs, tot.ea_pairs);
  P.xchg.resize(tot.xchg);
  resize_room(P.xp_tasks, tot.xp_tasks);
  resize_room(P.xp_loff, tot.xp_loff);
  resize_room(P.xp_lstride, tot.xp_lstride);
  P.npart = tot.npart;
  plan_parallel(nl, [&](int L) {
    LevelLists& S = out[L];
    CholLevel& lv = P.levels[L];
    const Base& b = base[L];
    const int bx = (int)b.xchg, npart0 = b.npart;
    lv.front_off += (int)b.level_fronts;
    lv.bwd_part.off += (int)b.bwd_part_tasks;
    for (int4& t : S.bwd_part_tasks) t.w += npart0;
    for (int q = lv.bwd[0].off; q < lv.bwd[0].off + lv.bwd[0].cnt; q++) S.bwd_pref[q].x += npart0;   // init tasks
    for (SolveStep& st : lv.bwd) st.off += (int)b.bwd_tasks;
    lv.bwdc.off += (int)b.bwdc_tasks;
    for (int& o : lv.ea_off) o += (int)b.ea_tasks;
    for (int4& t : S.ea_tasks) t.z += (int)b.ea_pairs;
    for (SmallClass& sc : lv.small) sc.off += (int)b.small_list;
    for (PanelStep& ps : lv.panels) {
      ps.potrf_off += (int)b.potrf_list;
      ps.col_off += (int)b.col_tasks;
      ps.syrk_off += (int)b.syrk_tasks;
      ps.sdiag_off += (int)b.sdiag_tasks;
      if (ps.xfirst >= 0) ps.xfirst += bx;
      if (ps.xstep >= 0) ps.xstep += bx;
    }
    if (lv.xtail >= 0) lv.xtail += bx;
    for (XExchange& x : S.xchg) x.off += (int)b.xp_tasks;
    auto put = [](auto& dst, size_t at, const auto& src) { std::copy(src.begin(), src.end(), dst.begin() + at); };
    put(P.small_list, b.small_list, S.small_list);
    put(P.level_fronts, b.level_fronts, S.level_fronts);
    put(P.potrf_list, b.potrf_list, S.potrf_list);
    put(P.syrk_tasks, b.syrk_tasks, S.syrk_tasks);
    put(P.sdiag_tasks, b.sdiag_tasks, S.sdiag_tasks);
    put(P.col_tasks, b.col_tasks, S.col_tasks);
    put(P.bwd_tasks, b.bwd_tasks, S.bwd_tasks);
    put(P.bwdc_tasks, b.bwdc_tasks, S.bwdc_tasks);
    put(P.bwd_pref, b.bwd_pref, S.bwd_pref);
    put(P.bwd_part_tasks, b.bwd_part_tasks, S.bwd_part_tasks);
    put(P.ea_tasks, b.ea_tasks, S.ea_tasks);
    put(P.ea_pairs, b.ea_pairs, S.ea_pairs);
    put(P.xchg, b.xchg, S.xchg);
    put(P.xp_tasks, b.xp_tasks, S.xp_tasks);
    put(P.xp_loff, b.xp_loff, S.xp_loff);
    put(P.xp_lstride, b.xp_lstride, S.xp_lstride);
  });
  P.syrk_flops = 0;
  for (int L = 0; L < nl; L++) {
    for (const PanelStep& ps : P.levels[L].panels) P.syrk_flops += ps.plain_flops;
    P.xp_rslot = std::max(P.xp_rslot, out[L].xp_rslot);
    P.schedule_error = P.schedule_error || out[L].schedule_error;
  }
  phase("schedule");
  chol_assembly(P, row_ptr, slot_col);
  phase("assembly");
}

void chol_analyze(CholPlan& P, int n, const std::vector<int>& row_ptr, const std::vector<int>& slot_col) {
  // PGO_PLAN_TIMING: phase times of the analysis on stderr (diagnostics)
  static const bool timing = getenv("PGO_PLAN_TIMING") != nullptr;
  auto tlast = std::chrono::steady_clock::now();
  auto phase = [&](const char* what) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "chol_analyze %-12s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - tlast).count());
    tlast = t;
  };
  P.nslots = (long long)slot_col.size();
  P.n = n;
  // ---- pose adjacency (old index), unique, no self loops
  std::vector<int> xadj(n + 1, 0), adj;
  adj.reserve(slot_col.size());
  {
    std::vector<int> stamp(n, -1);
    for (int i = 0; i < n; i++) {
      stamp[i] = i;
      for (int k = row_ptr[i]; k < row_ptr[i + 1]; k++) {
        const int j = slot_col[k];
        if (stamp[j] != i) {
          stamp[j] = i;
          adj.push_back(j);
        }
      }
      xadj[i + 1] = (int)adj.size();
    }
  }
  // a caller-given ordering (the incremental re-plan: the previous ordering
  // with the appended poses inserted) skips the fill-reducing ordering
  const std::vector<int> order0 = (int)P.order_in.size() == n ? P.order_in
                                  : P.ordering == kOrderAmd ? order_amd(n, xadj, adj) : order_nd(n, xadj, adj);
  std::vector<int> ip0(n);
  for (int k = 0; k < n; k++) ip0[order0[k]] = k;
  phase("ordering");
  // ---- elimination tree of the permuted pattern (Liu, path compression)
  std::vector<int> et(n, -1), anc(n, -1);
  for (int j = 0; j < n; j++) {
    const int oj = order0[j];
    for (int k = xadj[oj]; k < xadj[oj + 1]; k++) {
      int r = ip0[adj[k]];
      if (r >= j) continue;
      while (anc[r] != -1 && anc[r] != j) {
        const int t = anc[r];
        anc[r] = j;
        r = t;
      }
      if (anc[r] == -1) {
        anc[r] = j;
        et[r] = j;
      }
    }
  }
  phase("etree");
  // ---- postorder (children in increasing order)
  std::vector<int> chead(n, -1), cnext(n, -1), post;
  post.reserve(n);
  for (int j = n - 1; j >= 0; j--)
    if (et[j] >= 0) {
      cnext[j] = chead[et[j]];
      chead[et[j]] = j;
    }
  {
    std::vector<int> stack;
    for (int r = 0; r < n; r++) {
      if (et[r] != -1) continue;
      stack.push_back(r);
      while (!stack.empty()) {
        const int j = stack.back();
        const int c = chead[j];
        if (c == -1) {
          stack.pop_back();
          post.push_back(j);
        } else {
          chead[j] = cnext[c];
          stack.push_back(c);
        }
      }
    }
  }
  P.perm.resize(n);
  P.iperm.resize(n);
  std::vector<int> pos(n), par(n);
  for (int k = 0; k < n; k++) {
    P.perm[k] = order0[post[k]];
    pos[post[k]] = k;
  }
  for (int k = 0; k < n; k++) P.iperm[P.perm[k]] = k;
  for (int k = 0; k < n; k++) par[k] = et[post[k]] >= 0 ? pos[et[post[k]]] : -1;
  phase("postorder");
  // ---- column counts (off-diagonal pose rows) via row subtrees
  std::vector<int> cc(n, 0), mark(n, -1), nch(n, 0);
  for (int i = 0; i < n; i++) {
    mark[i] = i;
    const int oi = P.perm[i];
    for (int k = xadj[oi]; k < xadj[oi + 1]; k++) {
      int j = P.iperm[adj[k]];
      if (j >= i) continue;
      while (mark[j] != i) {
        cc[j]++;
        mark[j] = i;
        j = par[j];
      }
    }
  }
  for (int j = 0; j < n; j++)
    if (par[j] >= 0) nch[par[j]]++;
  phase("colcounts");
  // ---- fundamental supernodes, then relaxed amalgamation of a child that
  // immediately precedes its parent when it adds few explicit zeros
  std::vector<int> fs;
  for (int j = 0; j < n; j++) {
    if (j > 0 && par[j - 1] == j && nch[j] == 1 && cc[j - 1] == cc[j] + 1) continue;
    fs.push_back(j);
  }
  fs.push_back(n);
  std::vector<int> of, ol;
  std::vector<double> onz;
  // merge rule: a chain of W poses is kept together when W <= r[0], or
  // W <= r[1] with explicit-zero share z < r[2], W <= r[3] with z < r[4], or
  // z < r[5] (PGO_RELAX="r0,r1,r2,r3,r4,r5": a tuning knob)
  double rx[6] = {4, 8, 0.8, 24, 0.2, 0.05};   // (measured: C3 replays -4 % at 1 lane, -2 % at 3 lanes against {2, 6, 0.8, 16, 0.1, 0.05})
  if (const char* e = getenv("PGO_RELAX"))   // (separated by ',' or ';')
    for (int q = 0; q < 6 && *e; q++) {
      char* end = nullptr;
      rx[q] = strtod(e, &end);
      if (end == e) break;
      e = *end ? end + 1 : end;
    }
  for (size_t s = 0; s + 1 < fs.size(); s++) {
    int f = fs[s];
    const int l = fs[s + 1];
    const int wd = l - f, nb = cc[l - 1];
    double nz = 0.5 * wd * (wd + 1.0) + (double)wd * nb;
    while (!of.empty()) {
      const size_t t = of.size() - 1;
      if (ol[t] != f) break;
      const int lastc = ol[t] - 1;
      if (par[lastc] < f || par[lastc] >= l) break;
      const int W = l - of[t];
      const double tot = 0.5 * W * (W + 1.0) + (double)W * nb;
      const double tnz = nz + onz[t];
      const double z = (tot - tnz) / tot;
      const bool ok = (W <= rx[0]) || (W <= rx[1] && z < rx[2]) || (W <= rx[3] && z < rx[4]) || (z < rx[5]);
      if (!ok) break;
      f = of[t];
      nz = tnz;
      of.pop_back();
      ol.pop_back();
      onz.pop_back();
    }
    of.push_back(f);
    ol.push_back(l);
    onz.push_back(nz);
  }
  const int ns = (int)of.size();
  P.ns = ns;
  P.sfirst.assign(of.begin(), of.end());
  P.sfirst.push_back(n);
  std::vector<int> snode(n);
  for (int s = 0; s < ns; s++)
    for (int j = P.sfirst[s]; j < P.sfirst[s + 1]; j++) snode[j] = s;
  P.parent.assign(ns, -1);
  for (int s = 0; s < ns; s++) {
    const int lc = P.sfirst[s + 1] - 1;
    P.parent[s] = par[lc] >= 0 ? snode[par[lc]] : -1;
  }
  P.cptr.assign(ns + 1, 0);
  for (int s = 0; s < ns; s++)
    if (P.parent[s] >= 0) P.cptr[P.parent[s] + 1]++;
  for (int s = 0; s < ns; s++) P.cptr[s + 1] += P.cptr[s];
  P.children.assign(P.cptr[ns], 0);
  {
    std::vector<int> f(P.cptr.begin(), P.cptr.end() - 1);
    for (int s = 0; s < ns; s++)
      if (P.parent[s] >= 0) P.children[f[P.parent[s]]++] = s;
  }
  phase("supernodes");
  // ---- front rows: own poses then sorted below rows (A's pattern + children's rows)
  std::vector<std::vector<int>> below(ns);
  std::fill(mark.begin(), mark.end(), -1);
  for (int s = 0; s < ns; s++) {
    const int f = P.sfirst[s], l = P.sfirst[s + 1];
    auto& b = below[s];
    for (int j = f; j < l; j++) {
      const int oj = P.perm[j];
      for (int k = xadj[oj]; k < xadj[oj + 1]; k++) {
        const int i = P.iperm[adj[k]];
        if (i >= l && mark[i] != s) {
          mark[i] = s;
          b.push_back(i);
        }
      }
    }
    for (int q = P.cptr[s]; q < P.cptr[s + 1]; q++)
      for (int i : below[P.children[q]])
        if (i >= l && mark[i] != s) {
          mark[i] = s;
          b.push_back(i);
        }
    std::sort(b.begin(), b.end());
  }
  P.rptr.assign(ns + 1, 0);
  P.m.resize(ns);
  P.w.resize(ns);
  for (int s = 0; s < ns; s++) {
    const int wp = P.sfirst[s + 1] - P.sfirst[s];
    P.w[s] = 3 * wp;
    P.m[s] = 3 * (wp + (int)below[s].size());
    P.rptr[s + 1] = P.rptr[s] + wp + (int)below[s].size();
  }
  size_fronts(P);
  P.rows.resize(P.rptr[ns]);
  for (int s = 0; s < ns; s++) {
    int q = P.rptr[s];
    for (int j = P.sfirst[s]; j < P.sfirst[s + 1]; j++) P.rows[q++] = j;
    for (int i : below[s]) P.rows[q++] = i;
  }
  auto local_of = [&](int s, int i) {  // local pose index of new pose i in front s
    const int f = P.sfirst[s], l = P.sfirst[s + 1];
    if (i < l) return i - f;
    const auto& b = below[s];
    return (l - f) + (int)(std::lower_bound(b.begin(), b.end(), i) - b.begin());
  };
  phase("frontrows");
  // ---- extend-add maps: each below row of s -> local pose index in parent's front
  P.ea_ptr.assign(ns + 1, 0);
  for (int s = 0; s < ns; s++) P.ea_ptr[s + 1] = P.ea_ptr[s] + (int)below[s].size();
  P.ea_rel.resize(P.ea_ptr[ns]);
  for (int s = 0; s < ns; s++) {
    const int p = P.parent[s];
    for (size_t t = 0; t < below[s].size(); t++)
      P.ea_rel[P.ea_ptr[s] + t] = p >= 0 ? local_of(p, below[s][t]) : -1;
  }
  // ---- heights (leaves 0)
  P.height.assign(ns, 0);
  for (int s = 0; s < ns; s++)  // children precede parents (postorder)
    if (P.parent[s] >= 0) P.height[P.parent[s]] = std::max(P.height[P.parent[s]], P.height[s] + 1);
  P.dg_front.resize(n);
  P.dg_loc.resize(n);
  for (int j = 0; j < n; j++) {
    P.dg_front[j] = snode[j];
    P.dg_loc[j] = j - P.sfirst[snode[j]];
  }
  P.n_analyzed = n;
  P.flops_analyzed = P.flops;
  chol_schedule(P, row_ptr, slot_col);
}

// The targets after an append (chol_append): the columns in P.asm_dirty (the
// append's factors' columns and the new poses') get their entry lists rebuilt
// from the pattern, as chol_assembly builds every column; the other columns'
// targets and bound sources are kept (an append adds rows at the end of its
// fronts' row lists, so their local indices stand) and moved past the rebuilt
// ones.  Same lists as a rebuild once bound (host_selftest: check_append).
static void assembly_splice(CholPlan& P, const std::vector<int>& row_ptr, const std::vector<int>& slot_col) {
  std::vector<int>& dc = P.asm_dirty;
  std::sort(dc.begin(), dc.end());
  dc.erase(std::unique(dc.begin(), dc.end()), dc.end());
  const int ntg0 = (int)P.asm_front.size(), ne0 = P.asm_ptr[ntg0];
  auto colof = [&](int g) { return P.sfirst[P.asm_front[g]] + P.asm_lj[g]; };
  // old target range of each dirty column (targets are by column)
  std::vector<int> glo(dc.size()), ghi(dc.size());
  for (size_t d = 0; d < dc.size(); d++) {
    int lo = 0, hi = ntg0;
    while (lo < hi) {   // first g with colof(g) >= dc[d]
      const int mid = (lo + hi) / 2;
      if (colof(mid) < dc[d]) lo = mid + 1; else hi = mid;
    }
    glo[d] = lo;
    int g = lo;
    while (g < ntg0 && colof(g) == dc[d]) g++;
    ghi[d] = g;
  }
  // the dirty columns' new lists
  struct Col { std::vector<int> front, li, lj, cnt, src; };
  std::vector<Col> nc(dc.size());
  for (size_t d = 0; d < dc.size(); d++) {
    const int j = dc[d], r = P.perm[j];
    std::vector<int2> eik;
    for (int k = row_ptr[r]; k < row_ptr[r + 1]; k++) {
      const int i = P.iperm[slot_col[k]];
      if (i > j) eik.push_back(make_int2(i, k));
    }
    std::sort(eik.begin(), eik.end(), [](const int2& x, const int2& y) { return x.x != y.x ? x.x < y.x : x.y < y.y; });
    const int s = P.dg_front[j], f = P.sfirst[s], l = P.sfirst[s + 1];
    const int* b0 = P.rows.data() + P.rptr[s] + (l - f);
    const int* b1 = P.rows.data() + P.rptr[s + 1];
    const int* cur = b0;
    Col& c = nc[d];
    for (size_t q = 0; q < eik.size(); q++) {
      const int i = eik[q].x;
      if (q == 0 || i != eik[q - 1].x) {
        int li;
        if (i < l) {
          li = i - f;
        } else {
          cur = std::lower_bound(cur, b1, i);
          li = (l - f) + (int)(cur - b0);
        }
        c.front.push_back(s);
        c.li.push_back(li);
        c.lj.push_back(j - f);
        c.cnt.push_back(0);
      }
      c.cnt.back()++;
      c.src.push_back(~eik[q].y);
    }
  }
  // splice in place: the kept segments between the dirty columns' old ranges
  // move up by the targets / entries the dirty columns before them gained (an
  // append only adds to the pattern: shifts >= 0), last segment first, then the
  // dirty columns' new lists are written into the gaps
  const int D = (int)dc.size();
  std::vector<long long> tshift(D + 1, 0), eshift(D + 1, 0);   // shift of kept segment d (after dirty d - 1)
  std::vector<int> plo(D), phi(D);                             // old entry pointers at glo / ghi
  for (int d = 0; d < D; d++) {
    plo[d] = P.asm_ptr[glo[d]];
    phi[d] = P.asm_ptr[ghi[d]];
    tshift[d + 1] = tshift[d] + (long long)nc[d].front.size() - (ghi[d] - glo[d]);
    eshift[d + 1] = eshift[d] + (long long)nc[d].src.size() - (phi[d] - plo[d]);
  }
  bool grows = true;
  for (int d = 0; d <= D; d++) grows = grows && tshift[d] >= 0 && eshift[d] >= 0;
  if (!grows) {   // (not an append: the caller's rebuild)
    dc.clear();
    P.asm_bound = false;
    return;
  }
  const long long ntg = ntg0 + tshift[D], ne = ne0 + eshift[D];
  auto grow = [](auto& v, long long n) {   // (room for the next appends too)
    if ((long long)v.capacity() < n) v.reserve(n + n / 16 + 1024);
    v.resize(n);
  };
  grow(P.asm_front, ntg);
  grow(P.asm_li, ntg);
  grow(P.asm_lj, ntg);
  grow(P.asm_ptr, ntg + 1);
  grow(P.asm_src, ne);
  for (int d = D; d >= 1; d--) {   // kept segment d: old targets [ghi[d-1], glo[d] or ntg0)
    const int a0 = ghi[d - 1], a1 = d < D ? glo[d] : ntg0;
    const int e0 = phi[d - 1], e1 = d < D ? plo[d] : ne0;
    const long long ts = tshift[d], es = eshift[d];
    if (ts == 0 && es == 0) continue;
    std::copy_backward(P.asm_src.begin() + e0, P.asm_src.begin() + e1, P.asm_src.begin() + e1 + es);
    std::copy_backward(P.asm_front.begin() + a0, P.asm_front.begin() + a1, P.asm_front.begin() + a1 + ts);
    std::copy_backward(P.asm_li.begin() + a0, P.asm_li.begin() + a1, P.asm_li.begin() + a1 + ts);
    std::copy_backward(P.asm_lj.begin() + a0, P.asm_lj.begin() + a1, P.asm_lj.begin() + a1 + ts);
    for (int g = a1 - 1; g >= a0; g--) P.asm_ptr[g + ts] = P.asm_ptr[g] + (int)es;
  }
  for (int d = 0; d < D; d++) {   // dirty column d's list: targets from glo[d] + tshift[d], entries from plo[d] + eshift[d]
    const Col& c = nc[d];
    const long long g0 = glo[d] + tshift[d];
    long long e = plo[d] + eshift[d];
    std::copy(c.src.begin(), c.src.end(), P.asm_src.begin() + e);
    for (size_t t = 0; t < c.front.size(); t++) {
      P.asm_front[g0 + t] = c.front[t];
      P.asm_li[g0 + t] = c.li[t];
      P.asm_lj[g0 + t] = c.lj[t];
      P.asm_ptr[g0 + t] = (int)e;
      e += c.cnt[t];
    }
  }
  P.asm_ptr[ntg] = (int)ne;
  dc.clear();
}

// Assembly of H into the plan's fronts (k_assemble_tile's H entries): the
// targets (lower 3x3 blocks H_{i,j}, i > j, of the permuted pattern: front,
// local row, local column, and their block-CSR slots -- parallel factors summed
// in slot order) and, per tile task, the targets and diagonal blocks with an
// element in the tile.  Depends on the pattern and the plan's fronts only: the
// incremental path re-runs it alone when appended factors fit the fronts.
void chol_assembly(CholPlan& P, const std::vector<int>& row_ptr, const std::vector<int>& slot_col) {
  const int n = P.n, ns = P.ns;
  const int nth = std::max(1, std::min(plan_threads(), n));   // (the chunks over the n poses: one per thread)
  static const bool timing = getenv("PGO_PLAN_TIMING") != nullptr;
  auto tl = std::chrono::steady_clock::now();
  auto lap = [&](const char* what) {
    if (!timing) return;
    const auto t = std::chrono::steady_clock::now();
    fprintf(stderr, "chol_assembly %-12s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - tl).count());
    tl = t;
  };
  P.nslots = (long long)slot_col.size();
  const bool splice = P.asm_splice && P.asm_bound && !P.asm_ptr.empty();
  P.asm_splice = false;
  if (splice) {
    assembly_splice(P, row_ptr, slot_col);
    lap("splice");
  } else {
  // entries (j, i, k) of the permuted lower triangle (new indices i > j), by
  // (j, i, k).  Column j's entries are read from row perm[j]: its slots whose
  // column comes later, i.e. the mirror slot of each block (i, j).  Both slots
  // of a factor carry its device index, the only thing bind_plan keeps of k,
  // and a row's slots to one column are in the factors' device order whichever
  // end the row is: the same sources in the same order as from row perm[i].
  // Each column's few entries then sorted by (i, k) and its targets (distinct
  // (j, i)) counted per chunk of columns, then written.
  std::vector<int> jcnt(n + 1, 0);
  parallel_chunks(n, nth, [&](int, int r0, int r1) {   // (rows in their order: streamed)
    for (int r = r0; r < r1; r++) {
      const int j = P.iperm[r];
      int c = 0;
      for (int k = row_ptr[r]; k < row_ptr[r + 1]; k++) c += P.iperm[slot_col[k]] > j;
      jcnt[j + 1] = c;
    }
  });
  for (int j = 0; j < n; j++) jcnt[j + 1] += jcnt[j];
  lap("count");
  std::vector<int2> eik(jcnt[n]);   // (i, k) per entry, bucketed by j
  parallel_chunks(n, 8 * nth, [&](int, int r0, int r1) {
    for (int r = r0; r < r1; r++) {
      const int j = P.iperm[r];
      int q = jcnt[j];
      for (int k = row_ptr[r]; k < row_ptr[r + 1]; k++) {
        const int i = P.iperm[slot_col[k]];
        if (i > j) eik[q++] = make_int2(i, k);
      }
    }
  });
  lap("bucket");
  // (column chunks: 8 per thread, dealt dynamically -- the columns' work varies)
  const int nck = std::max(1, std::min(n, 8 * nth));
  std::vector<int> tstart(nck + 1, 0);
  parallel_chunks(n, nck, [&](int t, int j0, int j1) {
    int cnt = 0;
    for (int j = j0; j < j1; j++) {
      std::sort(eik.begin() + jcnt[j], eik.begin() + jcnt[j + 1],
                [](const int2& x, const int2& y) { return x.x != y.x ? x.x < y.x : x.y < y.y; });
      for (int q = jcnt[j]; q < jcnt[j + 1]; q++) cnt += (q == jcnt[j] || eik[q].x != eik[q - 1].x);
    }
    tstart[t + 1] = cnt;
  });
  lap("sort");
  for (int t = 0; t < nck; t++) tstart[t + 1] += tstart[t];
  const int ntg = tstart[nck];
  {   // (room for the live path's spliced appends: no regrowth on the first one)
    const size_t rt = ntg + ntg / 16 + 1024, re = eik.size() + eik.size() / 16 + 1024;
    P.asm_front.reserve(rt);
    P.asm_li.reserve(rt);
    P.asm_lj.reserve(rt);
    P.asm_ptr.reserve(rt + 1);
    P.asm_src.reserve(re);
  }
  P.asm_front.resize(ntg);
  P.asm_li.resize(ntg);
  P.asm_lj.resize(ntg);
  P.asm_ptr.resize(ntg + 1);
  P.asm_src.resize(eik.size());
  parallel_chunks(n, nck, [&](int t, int j0, int j1) {
    int g = tstart[t];
    for (int j = j0; j < j1; j++) {
      const int s = P.dg_front[j], f = P.sfirst[s], l = P.sfirst[s + 1];
      const int* b0 = P.rows.data() + P.rptr[s] + (l - f);
      const int* b1 = P.rows.data() + P.rptr[s + 1];
      const int* cur = b0;   // the bucket's rows come in increasing order: a forward scan finds them
      for (int q = jcnt[j]; q < jcnt[j + 1]; q++) {
        const int i = eik[q].x;
        if (q == jcnt[j] || i != eik[q - 1].x) {
          P.asm_ptr[g] = q;
          P.asm_front[g] = s;
          P.asm_lj[g] = j - f;
          int li;
          if (i < l) {
            li = i - f;
          } else {
            cur = std::lower_bound(cur, b1, i);
            li = (l - f) + (int)(cur - b0);
          }
          P.asm_li[g++] = li;
        }
        P.asm_src[q] = ~eik[q].y;
      }
    }
  });
  P.asm_bound = false;
  lap("targets");
  P.asm_ptr[ntg] = (int)eik.size();
  if (ntg == 0) P.asm_ptr.assign(1, 0);
  }
  const int ntg = (int)P.asm_front.size();
  // H entries by front tile: every 64x64 lower tile of a front lists the 3x3
  // blocks of H (off-diagonal targets t >= 0, diagonal blocks ~pose) with an
  // element in it (a block can straddle tile boundaries); items of a tile in
  // the order they are added (off-diagonal targets, then diagonal blocks).
  // Per front (its targets are contiguous: columns sorted), tiles in key order
  // ti (ti + 1) / 2 + tj -- the order of the front's tile tasks in ea_tasks.
  // targets of front s: [fg[s], fg[s + 1]) -- asm_front is nondecreasing (targets
  // by column, a front's columns contiguous and in front order): binary searches
  std::vector<int> fg(ns + 1, 0);
  parallel_chunks(ns + 1, nth, [&](int, int s0, int s1) {
    for (int s = s0; s < s1; s++)
      fg[s] = (int)(std::lower_bound(P.asm_front.begin(), P.asm_front.begin() + ntg, s) - P.asm_front.begin());
  });
  auto for_item = [](int r0, int c0, auto&& fn) {
    for (int ti = r0 / 64; ti <= (r0 + 2) / 64; ti++)
      for (int tj = c0 / 64; tj <= (c0 + 2) / 64; tj++)
        if (ti >= tj) fn(ti * (ti + 1) / 2 + tj);
  };
  std::vector<long long> fitems(ns + 1, 0);   // items of front s (counted, then its offset)
  // per front: item count per tile key, then its start (flat: front s at kbase[s], nt (nt + 1) / 2 + 1 keys)
  std::vector<long long> kbase(ns + 1, 0);
  for (int s = 0; s < ns; s++) {
    const long long nt = (P.m[s] + 63) / 64;
    kbase[s + 1] = kbase[s] + nt * (nt + 1) / 2 + 1;
  }
  std::vector<int> fcnt(kbase[ns], 0);
  parallel_chunks(ns, 8 * nth, [&](int, int s0, int s1) {
    for (int s = s0; s < s1; s++) {
      int* c = fcnt.data() + kbase[s];
      const long long nk = kbase[s + 1] - kbase[s];
      for (int g = fg[s]; g < fg[s + 1]; g++) for_item(3 * P.asm_li[g], 3 * P.asm_lj[g], [&](int key) { c[key + 1]++; });
      for (int j = P.sfirst[s]; j < P.sfirst[s + 1]; j++)
        for_item(3 * P.dg_loc[j], 3 * P.dg_loc[j], [&](int key) { c[key + 1]++; });
      for (long long k = 0; k + 1 < nk; k++) c[k + 1] += c[k];
      fitems[s + 1] = c[nk - 1];
    }
  });
  lap("tile count");
  // front blocks of at_items in the order of the fronts' tile tasks (level order)
  std::vector<long long> fbase(ns, -1);   // (-1: a front this rank does not assemble)
  {
    long long pos = 0;
    for (size_t q = 0; q < P.ea_tasks.size(); q++) {
      const int s = P.ea_tasks[q].x;
      if (P.ea_tasks[q].y == 0) {   // the front's first tile (0, 0)
        fbase[s] = pos;
        pos += fitems[s + 1];
      }
    }
    resize_room(P.at_items, pos);
  }
  parallel_chunks(ns, 8 * nth, [&](int, int s0, int s1) {
    std::vector<int> fill;   // (reused across the chunk's fronts)
    for (int s = s0; s < s1; s++) {
      if (fbase[s] < 0) continue;
      fill.assign(fcnt.begin() + kbase[s], fcnt.begin() + kbase[s + 1] - 1);
      int* out = P.at_items.data() + fbase[s];
      for (int g = fg[s]; g < fg[s + 1]; g++)
        for_item(3 * P.asm_li[g], 3 * P.asm_lj[g], [&](int key) { out[fill[key]++] = g; });
      for (int j = P.sfirst[s]; j < P.sfirst[s + 1]; j++)
        for_item(3 * P.dg_loc[j], 3 * P.dg_loc[j], [&](int key) { out[fill[key]++] = ~j; });
    }
  });
  lap("tile items");
  resize_room(P.at_iptr, P.ea_tasks.size());
  parallel_chunks((int)P.ea_tasks.size(), nth, [&](int, int q0, int q1) {
    for (int q = q0; q < q1; q++) {
      const int4 t = P.ea_tasks[q];
      const int ti = t.y >> 16, tj = t.y & 0xffff, key = ti * (ti + 1) / 2 + tj;
      const int* c = fcnt.data() + kbase[t.x];
      P.at_iptr[q] = make_int2((int)(fbase[t.x] + c[key]), c[key + 1] - c[key]);
    }
  });
  lap("tile ptrs");
  // (the levels' k_assemble_tile bytes: on first use, level_at_bytes)
  for (CholLevel& lv : P.levels) lv.at_bytes = -1.0;
}

// Does the plan's factor structure hold every block of the pattern (old pose
// indices)?  Block (r, c) with new indices i < j must have row j in the front of
// column i (its own poses or its below rows).
// Is block (a, b) (old pose indices < P.n) inside the plan's factor structure?
static bool covered(const CholPlan& P, int a, int b) {
  int i = P.iperm[a], j = P.iperm[b];
  if (i == j) return true;
  if (i > j) std::swap(i, j);
  const int s = P.dg_front[i];
  if (j < P.sfirst[s + 1]) return true;
  const int* b0 = P.rows.data() + P.rptr[s] + (P.sfirst[s + 1] - P.sfirst[s]);
  const int* b1 = P.rows.data() + P.rptr[s + 1];
  return std::binary_search(b0, b1, j);
}

bool chol_covers(const CholPlan& P, const std::vector<int2>& pairs) {
  for (const int2& e : pairs)
    if (e.x >= P.n || e.y >= P.n || !covered(P, e.x, e.y)) return false;
  return true;
}

// Incremental symbolic update for appended poses (the live re-solve,
// graph.cpp:180-200): poses P.n .. n-1 are eliminated last, as extra pivot
// columns of the root front (the last supernode), so no existing row moves.
// A new pose v coupled to an old pose a fills L(v, .) along the elimination
// tree path from a's front to the root: every front on it gains row v at the
// end of its row list (old rows keep their local indices, so the children's
// extend-add maps stay valid; v's own map entry points at the parent's new last
// rows); a root other than the last supernode reached this way becomes its
// child.  Only the fronts on these paths change size.  The schedules and
// assembly lists are then rebuilt from the fronts (chol_schedule).
// new_pairs: every factor added since the plan (old pose indices); factors
// between old poses must lie in the existing structure.  Returns false (plan
// untouched) when the update does not apply: a partitioned plan, an old-old
// factor outside the fill, a tail past max_tail poses since the last full
// analysis, or a factor past max_growth x the analysed one's flops.
bool chol_append(CholPlan& P, int n, const std::vector<int>& row_ptr, const std::vector<int>& slot_col,
                 const std::vector<int2>& new_pairs, int max_tail, double max_growth) {
  const int n0 = P.n, ns = P.ns;
  if (n <= n0 || ns == 0 || P.part_size > 1 || P.parent[ns - 1] != -1 || n - P.n_analyzed > max_tail ||
      P.flops > max_growth * P.flops_analyzed)
    return false;
  for (const int2& e : new_pairs)
    if (e.x < n0 && e.y < n0 && !covered(P, e.x, e.y)) return false;
  const int T = ns - 1;
  // 1. the fill paths: (front, new pose) in increasing pose order per front
  std::vector<int> stamp(ns, -1), added(ns, 0), reparent;
  std::vector<int2> adds;
  for (int v = n0; v < n; v++)
    for (int q = row_ptr[v]; q < row_ptr[v + 1]; q++) {
      const int a = slot_col[q];
      if (a >= n0) continue;
      int s = P.dg_front[P.iperm[a]];
      while (s != T && stamp[s] != v) {
        stamp[s] = v;
        adds.push_back(make_int2(s, v));
        added[s]++;
        if (P.parent[s] < 0) {
          reparent.push_back(s);
          break;
        }
        s = P.parent[s];
      }
    }
  // the growth limit on the plan after this append (the fronts on the fill
  // paths gain 3 rows per new pose, the root its new poses), before anything
  // of the plan is changed
  {
    auto pf = [](double m, double w) {   // size_fronts' flops of one front, closed form
      // sum_{k<w} 1 + r + r (r + 1), r = m - 1 - k
      const double s1 = w * (m - 1) - w * (w - 1) / 2;                       // sum r
      auto sq = [](double a) { return a * (a + 1) * (2 * a + 1) / 6; };      // sum_{r=0..a} r^2
      return w + 2 * s1 + (sq(m - 1) - sq(m - 1 - w));
    };
    double est = P.flops;
    for (int s = 0; s < ns; s++)
      if (added[s]) est += pf(P.m[s] + 3.0 * added[s], P.w[s]) - pf(P.m[s], P.w[s]);
    const double wt = 3.0 * (n - P.sfirst[T]);
    est += pf(wt, wt) - pf(P.m[T], P.w[T]);
    if (est > max_growth * P.flops_analyzed) return false;
  }
  // 2. row lists: old segment, then the new rows; the root front's own poses extended
  std::vector<int> rptr(ns + 1, 0);
  for (int s = 0; s < ns; s++) rptr[s + 1] = rptr[s] + (P.rptr[s + 1] - P.rptr[s]) + added[s] + (s == T ? n - n0 : 0);
  std::vector<int> rows(rptr[ns]);
  std::vector<int> fillp(ns);
  for (int s = 0; s < ns; s++) {
    std::copy(P.rows.begin() + P.rptr[s], P.rows.begin() + P.rptr[s + 1], rows.begin() + rptr[s]);
    fillp[s] = rptr[s] + (P.rptr[s + 1] - P.rptr[s]);
  }
  for (int v = n0; v < n; v++) rows[fillp[T]++] = v;
  std::stable_sort(adds.begin(), adds.end(), [](const int2& x, const int2& y) { return x.x < y.x; });
  for (const int2& t : adds) rows[fillp[t.x]++] = t.y;
  // 3. extend-add maps: old entries kept, the new rows' local index in the parent
  for (int s : reparent) P.parent[s] = T;
  std::vector<int> ea_ptr(ns + 1, 0);
  for (int s = 0; s < ns; s++) ea_ptr[s + 1] = ea_ptr[s] + (P.ea_ptr[s + 1] - P.ea_ptr[s]) + added[s];
  std::vector<int> ea_rel(ea_ptr[ns]);
  P.sfirst[ns] = n;
  for (int s = 0; s < ns; s++) {
    const int old = P.ea_ptr[s + 1] - P.ea_ptr[s];
    std::copy(P.ea_rel.begin() + P.ea_ptr[s], P.ea_rel.begin() + P.ea_ptr[s + 1], ea_rel.begin() + ea_ptr[s]);
    if (!added[s]) continue;
    const int p = P.parent[s];
    const int* b0 = rows.data() + rptr[p];
    const int* b1 = rows.data() + rptr[p + 1];
    const int* nr = rows.data() + rptr[s + 1] - added[s];
    for (int t = 0; t < added[s]; t++) {
      const int v = nr[t];
      // in the root front v is an own pose; elsewhere one of the parent's new rows
      const int li = p == T ? v - P.sfirst[T] : (int)(std::lower_bound(b1 - added[p], b1, v) - b0);
      ea_rel[ea_ptr[s] + old + t] = li;
    }
  }
  // 4. the rest of the plan's per-front / per-pose arrays
  P.rows.swap(rows);
  P.rptr.swap(rptr);
  P.ea_rel.swap(ea_rel);
  P.ea_ptr.swap(ea_ptr);
  for (int s = 0; s < ns; s++) P.m[s] += 3 * added[s];
  P.w[T] = 3 * (n - P.sfirst[T]);
  P.m[T] = P.w[T];
  P.perm.resize(n);
  P.iperm.resize(n);
  P.dg_front.resize(n);
  P.dg_loc.resize(n);
  for (int v = n0; v < n; v++) {
    P.perm[v] = P.iperm[v] = v;
    P.dg_front[v] = T;
    P.dg_loc[v] = v - P.sfirst[T];
  }
  if (!reparent.empty()) {
    P.cptr.assign(ns + 1, 0);
    for (int s = 0; s < ns; s++)
      if (P.parent[s] >= 0) P.cptr[P.parent[s] + 1]++;
    for (int s = 0; s < ns; s++) P.cptr[s + 1] += P.cptr[s];
    P.children.assign(P.cptr[ns], 0);
    std::vector<int> f(P.cptr.begin(), P.cptr.end() - 1);
    for (int s = 0; s < ns; s++)
      if (P.parent[s] >= 0) P.children[f[P.parent[s]]++] = s;
    P.height.assign(ns, 0);
    for (int s = 0; s < ns; s++)
      if (P.parent[s] >= 0) P.height[P.parent[s]] = std::max(P.height[P.parent[s]], P.height[s] + 1);
  }
  P.n = n;
  size_fronts(P);
  // the assembly targets: spliced (the columns of the new factors and poses rebuilt)
  P.asm_dirty.clear();
  for (const int2& e : new_pairs) P.asm_dirty.push_back(std::min(P.iperm[e.x], P.iperm[e.y]));
  for (int v = n0; v < n; v++) P.asm_dirty.push_back(v);
  P.asm_splice = !getenv("PGO_NO_ASM_SPLICE");
  chol_schedule(P, row_ptr, slot_col);
  return true;
}

bool chol_covers(const CholPlan& P, int n, const std::vector<int>& row_ptr, const std::vector<int>& slot_col) {
  if (n != P.n) return false;
  for (int r = 0; r < n; r++)
    for (int k = row_ptr[r]; k < row_ptr[r + 1]; k++) {
      int i = P.iperm[r], j = P.iperm[slot_col[k]];
      if (i == j) continue;
      if (i > j) std::swap(i, j);
      const int s = P.dg_front[i];
      if (j < P.sfirst[s + 1]) continue;
      const int* b0 = P.rows.data() + P.rptr[s] + (P.sfirst[s + 1] - P.sfirst[s]);
      const int* b1 = P.rows.data() + P.rptr[s + 1];
      if (!std::binary_search(b0, b1, j)) return false;
    }
  return true;
}

}  // namespace pgo

namespace pgo {

// Subtree partition of the supernodal tree over `size` ranks (the partitioned
// multi-GPU factorisation): starting from the tree roots, the heaviest
// candidate subtree (by factorisation flops) is split -- its root joins the
// replicated "top" and its children become candidates -- until every
// candidate holds at most 1/(2 size) of the candidates' flops (or cannot be
// split); the candidates are then dealt to ranks largest first, each to the
// least-loaded rank.  owner[s] = rank of front s's subtree, -1 for top fronts.
// Deterministic: every rank computes the same partition from the same plan.
std::vector<int> partition_subtrees(const CholPlan& P, int size, std::vector<double>* rank_flops,
                                    double* top_flops) {
  const int ns = P.ns;
  std::vector<double> f(ns, 0.0), sub(ns, 0.0);
  for (int s = 0; s < ns; s++) {
    for (int k = 0; k < P.w[s]; k++) {
      const double r = P.m[s] - k - 1;
      f[s] += 1 + r + r * (r + 1);
    }
    sub[s] += f[s];
    if (P.parent[s] >= 0) sub[P.parent[s]] += sub[s];   // children precede parents (postorder)
  }
  std::vector<int> owner(ns, -1), cand;
  for (int s = 0; s < ns; s++)
    if (P.parent[s] < 0) cand.push_back(s);
  if (size > 1) {
    for (;;) {
      double tot = 0;
      int best = -1;
      for (int c : cand) {
        tot += sub[c];
        if (best < 0 || sub[c] > sub[best]) best = c;
      }
      if (best < 0 || sub[best] <= tot / (2.0 * size) || P.cptr[best] == P.cptr[best + 1]) break;
      cand.erase(std::find(cand.begin(), cand.end(), best));
      for (int q = P.cptr[best]; q < P.cptr[best + 1]; q++) cand.push_back(P.children[q]);
    }
  }
  std::stable_sort(cand.begin(), cand.end(), [&](int a, int b) { return sub[a] > sub[b]; });
  std::vector<double> load(size, 0.0);
  std::vector<int> root_rank(ns, -1);
  for (int c : cand) {
    const int r = (int)(std::min_element(load.begin(), load.end()) - load.begin());
    load[r] += sub[c];
    root_rank[c] = r;
  }
  for (int s = ns - 1; s >= 0; s--) {   // parents before children: inherit the subtree's rank
    if (root_rank[s] >= 0) owner[s] = root_rank[s];
    else if (P.parent[s] >= 0 && owner[P.parent[s]] >= 0) owner[s] = owner[P.parent[s]];
  }
  if (rank_flops) *rank_flops = load;
  if (top_flops) {
    *top_flops = 0;
    for (int s = 0; s < ns; s++)
      if (owner[s] < 0) *top_flops += f[s];
  }
  return owner;
}

}  // namespace pgo
