// Host self-test of the solver's planning code (test infrastructure, not part
// of libpgo.so): drives the symbolic analysis on synthetic pose graphs so a host
// AddressSanitizer / UndefinedBehaviorSanitizer build (`make -C
// graphslam_amd/csrc asan-host`) exercises its memory accesses --
// nested-dissection and AMD orderings, supernodes, level schedule, panel steps,
// the assembly lists, the subtree partition for 2 and 4 ranks, the incremental
// paths (chol_covers / chol_assembly, a caller-given ordering).  No GPU calls.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <tuple>
#include <random>
#include <vector>

#include "pgo_chol.h"

namespace {

struct Pattern {
  int n = 0;
  std::vector<int> row_ptr, col;
};

// block pattern of H for a chain of n poses with `lc` random loop closures;
// `dups` of the loop closures (every lc / dups-th) repeated as a parallel
// factor: the same block listed twice in both rows, as the library's block-CSR
// lists parallel factors (one slot each, in device order)
Pattern make_pattern(int n, int lc, unsigned seed, const std::vector<std::pair<int, int>>& extra = {}, int dups = 0) {
  std::mt19937 rng(seed);
  std::vector<std::pair<int, int>> e;
  for (int i = 0; i + 1 < n; i++) e.emplace_back(i, i + 1);
  for (int q = 0; q < lc; q++) {
    const int a = 20 + (int)(rng() % (unsigned)(n - 20));
    e.emplace_back(a, (int)(rng() % (unsigned)(a - 10)));
  }
  e.insert(e.end(), extra.begin(), extra.end());
  Pattern P;
  P.n = n;
  std::vector<std::vector<int>> adj(n);
  for (auto& [a, b] : e) {
    adj[a].push_back(b);
    adj[b].push_back(a);
  }
  for (int i = 0; i < n; i++) {
    adj[i].push_back(i);
    std::sort(adj[i].begin(), adj[i].end());
    adj[i].erase(std::unique(adj[i].begin(), adj[i].end()), adj[i].end());
  }
  for (int q = 0; dups > 0 && q < lc; q += std::max(1, lc / dups)) {
    const auto [a, b] = e[n - 1 + q];
    if (a == b) continue;
    adj[a].push_back(b);
    adj[b].push_back(a);
  }
  P.row_ptr.assign(1, 0);
  for (int i = 0; i < n; i++) {
    std::sort(adj[i].begin(), adj[i].end());
    P.col.insert(P.col.end(), adj[i].begin(), adj[i].end());
    P.row_ptr.push_back((int)P.col.size());
  }
  return P;
}

constexpr int kDupIds = 8;   // parallel factors per pose pair the emulated bind tells apart

int fail(const char* m) {
  std::fprintf(stderr, "host_selftest: %s\n", m);
  return 1;
}

// Task coverage of one top level / panel step: (kind, front, row tile, column,
// depth) -> how often.  Plain tiles count per (64-row tile, column) they
// update (128-tiles split), clipped as the kernels clip them.
using Key = std::tuple<int, int, int, int, int>;
void step_keys(const pgo::CholPlan& P, const pgo::PanelStep& ps, std::map<Key, int>& out) {
  for (int q = ps.syrk_off; q < ps.syrk_off + ps.syrk_cnt; q++) {
    const int4 t = P.syrk_tasks[q];
    const int s = t.x, row0 = t.y & pgo::kRowMask, clip = t.y >> pgo::kClipShift, c0 = t.z, m = P.m[s], w = P.w[s];
    const int T = ps.syrk_tile;
    int colend = t.w < 0 ? std::min((ps.kb & ~(pgo::kKB - 1)) + pgo::kKB, w) : m;
    const int cend = std::min({colend, c0 + (clip ? clip : T), m});
    for (int r0 = row0; r0 < std::min(row0 + T, m); r0 += 64)
      for (int col = c0; col < cend; col++)
        if (col <= r0 + 63) out[Key(0, s, r0, col, t.w)]++;
  }
  for (int q = ps.sdiag_off; q < ps.sdiag_off + ps.sdiag_cnt; q++) {
    const int4 t = P.sdiag_tasks[q];
    out[Key(1, t.x, t.y, t.z, t.w)]++;
  }
  for (int q = ps.col_off; q < ps.col_off + ps.fcol_cnt + ps.col_cnt + ps.prep_cnt; q++) {
    const int4 t = P.col_tasks[q];
    out[Key(2, t.x, t.y, t.z, t.w)]++;
  }
  for (int q = ps.potrf_off; q < ps.potrf_off + ps.potrf_cnt; q++) out[Key(3, P.potrf_list[q], 0, 0, 0)]++;
}

// The distributed top (part_size > 1): every rank's top tasks together are the
// replicated plan's (PGO_DIST_TOP=0), each task on its column's rank (every
// rank for the replicated columns); every factored panel is exchanged.
int check_distributed(const Pattern& G, int ordering, int size) {
  std::vector<pgo::CholPlan> D(size), R(size);
  for (int r = 0; r < size; r++) {
    for (int dist : {1, 0}) {
      pgo::CholPlan& Q = dist ? D[r] : R[r];
      if (!dist) setenv("PGO_DIST_TOP", "0", 1);
      Q.ordering = ordering;
      Q.part_size = size;
      Q.part_rank = r;
      pgo::chol_analyze(Q, G.n, G.row_ptr, G.col);
      unsetenv("PGO_DIST_TOP");
      if (Q.schedule_error) return fail("distributed: schedule");
    }
  }
  const pgo::CholPlan& A = R[0];
  long long tasks = 0, exch = 0;
  for (size_t L = A.split; L < A.levels.size(); L++)
    for (size_t j = 0; j < A.levels[L].panels.size(); j++) {
      std::map<Key, int> full;
      step_keys(A, A.levels[L].panels[j], full);
      std::vector<std::map<Key, int>> got(size);
      for (int r = 0; r < size; r++) {
        const pgo::CholPlan& Q = D[r];
        const size_t LQ = Q.split + (L - A.split);
        if (LQ >= Q.levels.size() || Q.levels[LQ].panels.size() != A.levels[L].panels.size())
          return fail("distributed: top levels differ");
        step_keys(Q, Q.levels[LQ].panels[j], got[r]);
        const pgo::PanelStep& ps = Q.levels[LQ].panels[j];
        for (int xi : {ps.xfirst, ps.xstep})
          if (xi >= 0) exch += Q.xchg[xi].cnt;
      }
      for (const auto& [k, cnt] : full) {
        const int kind = std::get<0>(k), s = std::get<1>(k);
        const int col = kind == 0 ? std::get<3>(k) : kind == 1 ? std::get<2>(k) : kind == 2 ? std::get<3>(k) : 0;
        const int o = D[0].cown[D[0].cown_off[s] + col];
        for (int r = 0; r < size; r++) {
          const auto it = got[r].find(k);
          const int want = (o < 0 || o == r) ? cnt : 0;
          if ((it == got[r].end() ? 0 : it->second) != want) {
            std::fprintf(stderr, "kind %d front %d row %d col %d depth %d: rank %d has %d, owner %d\n", kind, s,
                         std::get<2>(k), std::get<3>(k), std::get<4>(k), r, it == got[r].end() ? 0 : it->second, o);
            return fail("distributed: task coverage");
          }
          if (it != got[r].end()) got[r].erase(it);
        }
        tasks++;
      }
      for (int r = 0; r < size; r++)
        if (!got[r].empty()) return fail("distributed: a rank has a task the replicated plan lacks");
    }
  std::printf("distributed top, %d ranks: %lld task keys checked, %lld panels exchanged\n", size, tasks, exch);
  return 0;
}

// The tile lists of the H assembly (at_iptr / at_items): every tile task of
// every front this rank assembles lists exactly the front's off-diagonal
// targets, then its diagonal blocks, with an element in the tile, in order.
int check_assembly(const pgo::CholPlan& P) {
  std::vector<std::vector<int>> tg(P.ns);
  for (size_t g = 0; g < P.asm_front.size(); g++) tg[P.asm_front[g]].push_back((int)g);
  auto touches = [](int r0, int c0, int ti, int tj) {
    return r0 / 64 <= ti && ti <= (r0 + 2) / 64 && c0 / 64 <= tj && tj <= (c0 + 2) / 64;
  };
  for (size_t q = 0; q < P.ea_tasks.size(); q++) {
    const int4 t = P.ea_tasks[q];
    const int s = t.x, ti = t.y >> 16, tj = t.y & 0xffff;
    std::vector<int> want;
    for (int g : tg[s])
      if (touches(3 * P.asm_li[g], 3 * P.asm_lj[g], ti, tj)) want.push_back(g);
    for (int j = P.sfirst[s]; j < P.sfirst[s + 1]; j++)
      if (touches(3 * P.dg_loc[j], 3 * P.dg_loc[j], ti, tj)) want.push_back(~j);
    const int2 it = P.at_iptr[q];
    if (it.y != (int)want.size() || !std::equal(want.begin(), want.end(), P.at_items.begin() + it.x))
      return fail("assembly: a tile's H entries");
  }
  // every front's lower tiles exactly once, whatever the order (the tasks of
  // a level are dealt to the XCDs in blocks, ea_xcd_order)
  std::vector<std::vector<char>> seen(P.ns);
  for (const int4& t : P.ea_tasks) {
    const int s = t.x, ti = t.y >> 16, tj = t.y & 0xffff, nt = (P.m[s] + 63) / 64;
    if (ti >= nt || tj > ti) return fail("assembly: a tile outside its front's lower triangle");
    if (seen[s].empty()) seen[s].assign((size_t)nt * (nt + 1) / 2, 0);
    char& k = seen[s][(size_t)ti * (ti + 1) / 2 + tj];
    if (k) return fail("assembly: a tile listed twice");
    k = 1;
  }
  for (int s = 0; s < P.ns; s++)
    for (char k : seen[s])
      if (!k) return fail("assembly: a front's tile missing");
  return 0;
}

// The assembly's targets and sources against the pattern: every target (j, i)
// of the permuted lower triangle (i > j) lists exactly the slots of one end of
// the block -- as many as row perm[i] holds to column perm[j] -- and every
// slot of the lower triangle is listed once.
// (sources: ~slot unbound; bound ones -- bind emulated by emulate_bind, ids
// (a * idn + b) * kDupIds + k of the k-th parallel factor of the pose pair
// a < b -- checked against the block's poses, and a target's parallel
// factors in their slot order, the summation order)
int check_sources(const pgo::CholPlan& P, const std::vector<int>& row_ptr, const std::vector<int>& col, int idn = 0) {
  long long total = 0, want = 0;
  for (size_t g = 0; g < P.asm_front.size(); g++) {
    const int s = P.asm_front[g], j = P.sfirst[s] + P.asm_lj[g], i = P.rows[P.rptr[s] + P.asm_li[g]];
    if (i <= j) return fail("assembly: a target above the diagonal");
    const int a = P.perm[i], b = P.perm[j];
    int cnt = 0;
    for (int k = row_ptr[a]; k < row_ptr[a + 1]; k++) cnt += col[k] == b;
    if (P.asm_ptr[g + 1] - P.asm_ptr[g] != cnt) return fail("assembly: a target's source count");
    for (int q = P.asm_ptr[g]; q < P.asm_ptr[g + 1]; q++) {
      if (P.asm_src[q] >= 0) {   // bound: the factor id
        if (!idn || P.asm_src[q] / kDupIds != std::min(a, b) * idn + std::max(a, b))
          return fail("assembly: a bound source off its block");
        if (P.asm_src[q] % kDupIds != q - P.asm_ptr[g]) return fail("assembly: parallel factors out of slot order");
        continue;
      }
      const int k = ~P.asm_src[q];
      const int r = (int)(std::upper_bound(row_ptr.begin(), row_ptr.end(), k) - row_ptr.begin()) - 1;
      if (!((r == a && col[k] == b) || (r == b && col[k] == a))) return fail("assembly: a source off its block");
    }
    total += cnt;
  }
  for (int r = 0; r + 1 < (int)row_ptr.size(); r++)
    for (int k = row_ptr[r]; k < row_ptr[r + 1]; k++) want += P.iperm[r] > P.iperm[col[k]];
  if (total != want || P.asm_ptr.back() != want) return fail("assembly: sources of the lower triangle");
  return 0;
}

// Packed fronts: no Schur tile's columns straddle a 64-column block (the
// kernels address a tile's columns from one block base).
int check_tiles(const pgo::CholPlan& P) {
  for (const auto& lv : P.levels)
    for (const auto& ps : lv.panels)
      for (int q = ps.syrk_off; q < ps.syrk_off + ps.syrk_cnt; q++) {
        const int4 t = P.syrk_tasks[q];
        const int clip = t.y >> pgo::kClipShift, c0 = t.z, T = ps.syrk_tile;
        const int c1 = std::min(c0 + (clip ? clip : T), P.m[t.x]);
        if (T == pgo::kTile && (c0 >> 6) != ((c1 - 1) >> 6)) return fail("a 64-tile straddles two column blocks");
        if (T == pgo::kBigTile && (c0 & 63) && (c0 >> 6) != ((c1 - 1) >> 6))
          return fail("an unaligned 128-tile straddles two column blocks");
      }
  return 0;
}

// the pattern restricted to poses [0, n)
Pattern restrict_pattern(const Pattern& G, int n) {
  Pattern R;
  R.n = n;
  R.row_ptr.assign(1, 0);
  for (int i = 0; i < n; i++) {
    for (int k = G.row_ptr[i]; k < G.row_ptr[i + 1]; k++)
      if (G.col[k] < n) R.col.push_back(G.col[k]);
    R.row_ptr.push_back((int)R.col.size());
  }
  return R;
}

// The host's bind (pgo_api.cpp bind_plan) emulated: every unbound source ~k
// becomes a factor id, (a * idn + b) * kDupIds + j for the j-th slot of row r
// to column c (pose pair a < b of {r, c}) -- a factor index in the library:
// equal for both slots of a factor (a row lists a pair's parallel factors in
// device order from either end), distinct between parallel factors, so a
// splice that reorders them inside a target shows.
void emulate_bind(pgo::CholPlan& P, const std::vector<int>& row_ptr, const std::vector<int>& col, int idn) {
  for (int& x : P.asm_src)
    if (x < 0) {
      const int k = ~x;
      const int r = (int)(std::upper_bound(row_ptr.begin(), row_ptr.end(), k) - row_ptr.begin()) - 1;
      int j = 0;
      for (int q = row_ptr[r]; q < k; q++) j += col[q] == col[k];
      x = (std::min(r, col[k]) * idn + std::max(r, col[k])) * kDupIds + j;
    }
  P.asm_bound = true;
}

// The spliced assembly targets of an append equal a rebuild of the same plan,
// once both are bound.
int check_splice(const pgo::CholPlan& P, const std::vector<int>& row_ptr, const std::vector<int>& col, int idn) {
  pgo::CholPlan R = P;
  R.asm_splice = false;
  pgo::chol_assembly(R, row_ptr, col);
  emulate_bind(R, row_ptr, col, idn);
  pgo::CholPlan Q = P;
  emulate_bind(Q, row_ptr, col, idn);
  if (Q.asm_front != R.asm_front || Q.asm_li != R.asm_li || Q.asm_lj != R.asm_lj || Q.asm_ptr != R.asm_ptr ||
      Q.asm_src != R.asm_src || Q.at_items != R.at_items || Q.at_iptr.size() != R.at_iptr.size())
    return fail("append: spliced assembly lists differ from a rebuild");
  for (size_t q = 0; q < Q.at_iptr.size(); q++)
    if (Q.at_iptr[q].x != R.at_iptr[q].x || Q.at_iptr[q].y != R.at_iptr[q].y) return fail("append: spliced tile items");
  return 0;
}

// The incremental symbolic update (chol_append): poses appended one at a time
// to a plan of the first n0 poses.  After each: the schedule is consistent,
// every front's below rows sit in its parent at the extend-add map's index, the
// sizes match the row lists, and the structure holds the exact fill of the
// plan's own ordering (a fresh analysis on P.perm) and the whole pattern.
int check_append(const Pattern& G, int n0, int ordering) {
  pgo::CholPlan P;
  P.ordering = ordering;
  const Pattern B = restrict_pattern(G, n0);
  pgo::chol_analyze(P, n0, B.row_ptr, B.col);
  emulate_bind(P, B.row_ptr, B.col, G.n);
  {   // the growth limit applies to the plan after the append: no headroom refuses the first one
    pgo::CholPlan Q;
    Q.ordering = ordering;
    pgo::chol_analyze(Q, n0, B.row_ptr, B.col);
    const Pattern G1 = restrict_pattern(G, n0 + 1);
    std::vector<int2> pairs;
    for (int k = G1.row_ptr[n0]; k < G1.row_ptr[n0 + 1]; k++) pairs.push_back(make_int2(n0, G1.col[k]));
    if (pgo::chol_append(Q, n0 + 1, G1.row_ptr, G1.col, pairs, 1 << 30, 1.0)) return fail("append: growth limit not applied");
    if (Q.n != n0) return fail("append: a refused append changed the plan");
  }
  for (int n = n0 + 1; n <= G.n; n++) {
    const Pattern Gn = restrict_pattern(G, n);
    std::vector<int2> pairs;
    for (int k = Gn.row_ptr[n - 1]; k < Gn.row_ptr[n]; k++) pairs.push_back(make_int2(n - 1, Gn.col[k]));
    if (!pgo::chol_append(P, n, Gn.row_ptr, Gn.col, pairs, 1 << 30, 1e30)) return fail("append: refused");
    if (P.schedule_error) return fail("append: panel schedule bookkeeping");
    if (check_assembly(P) || check_sources(P, Gn.row_ptr, Gn.col, G.n) || check_splice(P, Gn.row_ptr, Gn.col, G.n)) return 1;
    emulate_bind(P, Gn.row_ptr, Gn.col, G.n);   // (the next append splices)
    if (P.n != n || !pgo::chol_covers(P, n, Gn.row_ptr, Gn.col)) return fail("append: pattern not covered");
    for (int s = 0; s < P.ns; s++) {
      const int wp = P.sfirst[s + 1] - P.sfirst[s], nr = P.rptr[s + 1] - P.rptr[s];
      if (P.m[s] != 3 * nr || P.w[s] != 3 * wp || P.ea_ptr[s + 1] - P.ea_ptr[s] != nr - wp)
        return fail("append: front sizes");
      const int p = P.parent[s];
      for (int t = 0; t < nr - wp; t++) {
        const int r = P.rows[P.rptr[s] + wp + t];
        if (t > 0 && r <= P.rows[P.rptr[s] + wp + t - 1]) return fail("append: rows unsorted");
        if (p < 0 || P.rows[P.rptr[p] + P.ea_rel[P.ea_ptr[s] + t]] != r) return fail("append: extend-add map");
      }
    }
    pgo::CholPlan Q;
    Q.order_in = P.perm;
    pgo::chol_analyze(Q, n, Gn.row_ptr, Gn.col);
    for (int q = 0; q < Q.ns; q++)
      for (int a = Q.rptr[q]; a < Q.rptr[q + 1]; a++)
        for (int j = Q.sfirst[q]; j < Q.sfirst[q + 1]; j++) {
          const int i = Q.rows[a];
          if (i > j) {
            std::vector<int2> one{make_int2(Q.perm[i], Q.perm[j])};
            if (!pgo::chol_covers(P, one)) return fail("append: fill of the ordering not covered");
          }
        }
  }
  std::printf("append: %d poses onto %d, %d fronts, flops %.3g\n", G.n - n0, n0, P.ns, P.flops);
  return 0;
}

}  // namespace

int main() {
  for (int n : {1, 2, 5}) {   // graphs smaller than the planner's thread count
    const Pattern G = restrict_pattern(make_pattern(40, 0, 3), n);
    pgo::CholPlan P;
    pgo::chol_analyze(P, G.n, G.row_ptr, G.col);
    if (P.schedule_error || !pgo::chol_covers(P, G.n, G.row_ptr, G.col)) return fail("tiny graph");
  }
  // every front a look-ahead front (the skip and prep bookkeeping on small ones too), then the default
  // (PGO_SELFTEST_QUICK=1: the default only -- a second pass under another planner knob)
  const bool quick = getenv("PGO_SELFTEST_QUICK") && atoi(getenv("PGO_SELFTEST_QUICK")) == 1;
  for (const char* la : {"64", "1000000000", ""}) {
  if (quick && *la) continue;
  if (*la) setenv("PGO_LOOKAHEAD_M", la, 1);
  else unsetenv("PGO_LOOKAHEAD_M");
  for (int ordering : {pgo::kOrderNd, pgo::kOrderAmd}) {
    const Pattern G = make_pattern(3000, 400, 7);
    pgo::CholPlan P;
    P.ordering = ordering;
    pgo::chol_analyze(P, G.n, G.row_ptr, G.col);
    if (P.ns <= 0 || P.flops <= 0) return fail("analysis");
    if (P.schedule_error) return fail("panel schedule bookkeeping");
    if (!pgo::chol_covers(P, G.n, G.row_ptr, G.col)) return fail("plan does not cover its own pattern");
    if (check_assembly(P) || check_tiles(P) || check_sources(P, G.row_ptr, G.col)) return 1;
    for (int size : {2, 4}) {
      std::vector<double> rf;
      double top = 0;
      const auto own = pgo::partition_subtrees(P, size, &rf, &top);
      if ((int)own.size() != P.ns) return fail("partition size");
      for (int r = 0; r < size; r++) {
        pgo::CholPlan Q;
        Q.ordering = ordering;
        Q.part_size = size;
        Q.part_rank = r;
        pgo::chol_analyze(Q, G.n, G.row_ptr, G.col);
        if (Q.ns != P.ns || Q.schedule_error) return fail("partitioned plan");
        if (check_assembly(Q) || check_tiles(Q)) return 1;
      }
    }
    // a loop closure inside the existing fill: same fronts, new assembly lists
    const Pattern G2 = make_pattern(3000, 400, 7, {{2, 0}});
    if (pgo::chol_covers(P, G2.n, G2.row_ptr, G2.col)) pgo::chol_assembly(P, G2.row_ptr, G2.col);
    // appended poses re-planned on a given ordering
    const Pattern G3 = make_pattern(3010, 400, 7, {{3009, 5}});
    pgo::CholPlan R;
    R.ordering = ordering;
    R.order_in.resize(G3.n);
    for (int k = 0; k < G3.n; k++) R.order_in[k] = G3.n - 1 - k;
    pgo::chol_analyze(R, G3.n, G3.row_ptr, G3.col);
    if (!pgo::chol_covers(R, G3.n, G3.row_ptr, G3.col) || R.schedule_error) return fail("given ordering");
    // appended poses: the incremental symbolic update
    if (check_append(make_pattern(1500, 200, 9, {}, 40), 1490, ordering)) return 1;
  }
  {   // a 2-D grid of poses: nested dissection gives big separator fronts (many
      // panels, kKB block boundaries, partial last panels) -- the look-ahead
      // schedule's bookkeeping is checked on them
    const int side = 60, n = side * side;
    std::vector<std::pair<int, int>> e;
    for (int y = 0; y < side; y++)
      for (int x = 0; x < side; x++) {
        if (x + 1 < side) e.emplace_back(y * side + x, y * side + x + 1);
        if (y + 1 < side) e.emplace_back(y * side + x, (y + 1) * side + x);
      }
    std::vector<std::vector<int>> adj(n);
    for (auto& [a, b] : e) {
      adj[a].push_back(b);
      adj[b].push_back(a);
    }
    Pattern G;
    G.n = n;
    G.row_ptr.assign(1, 0);
    for (int i = 0; i < n; i++) {
      adj[i].push_back(i);
      std::sort(adj[i].begin(), adj[i].end());
      G.col.insert(G.col.end(), adj[i].begin(), adj[i].end());
      G.row_ptr.push_back((int)G.col.size());
    }
    pgo::CholPlan P;
    pgo::chol_analyze(P, G.n, G.row_ptr, G.col);
    if (check_tiles(P)) return 1;
    for (int size : {2, 3, 4, 8})
      if (check_distributed(G, pgo::kOrderNd, size)) return 1;
    int maxw = 0;
    for (int s2 = 0; s2 < P.ns; s2++) maxw = std::max(maxw, P.w[s2]);
    if (P.schedule_error) return fail("grid: panel schedule bookkeeping");
    std::printf("grid plan (look-ahead threshold %s): %d fronts, widest %d pivot columns\n", *la ? la : "default",
                P.ns, maxw);
  }
  }
  std::printf("host selftest ok\n");
  return 0;
}
