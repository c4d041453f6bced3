// Fill-reducing orderings of the pose graph for the supernodal Cholesky
// (pgo_chol.h).  GTSAM orders with COLAMD on every solve (inside
// LevenbergMarquardtOptimizer::optimize, graph.cpp:119); this library orders
// once per graph structure, and for the GPU factorisation the shape of the
// elimination tree matters as much as the fill: the levels of the tree run one
// after the other, so a deep chain of small fronts at the top is a serial
// critical path.  Nested dissection gives a balanced tree (every level of the
// recursion is one level of independent fronts) and, on the 2-D Manhattan
// graphs of BASELINE.json, fewer flops than minimum degree.
//
// order_nd: multilevel nested dissection.  Each bisection coarsens the graph by
// heavy-edge matching down to ~100 vertices, bisects the coarsest graph by
// greedy region growing (best of several seeds), and projects back with
// Fiduccia-Mattheyses refinement of the edge cut at every level; the vertex
// separator is a minimum vertex cover of the cut edges (Hopcroft-Karp matching
// + Koenig).  Sides are ordered first (recursively), separator last; subgraphs
// of at most kLeaf (64) vertices are ordered by exact minimum degree.  Deterministic
// (fixed-seed generator), so the plan and the results are reproducible.
#include <algorithm>
#include <cstdlib>
#include <cstdint>
#include <numeric>
#include <queue>
#include <thread>
#include <utility>
#include <vector>

#include "pgo_chol.h"

namespace pgo {
namespace {

constexpr int kLeaf = 64;         // subgraphs this small: minimum degree
constexpr int kCoarsest = 96;     // stop coarsening below this many vertices
constexpr int kInitTries = 8;     // region-growing seeds on the coarsest graph
constexpr double kMaxSide = 0.55; // heaviest side <= this fraction of the weight
constexpr int kTopTries = 24;     // bisection tries at the root of the dissection (half that below it)
constexpr int kTriedDepth = 8;    // ... down to this depth

struct Graph {
  int n = 0;
  std::vector<int> xadj{0}, adj, ew, vw;
  long long tw = 0;
};

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint32_t next() {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    return (uint32_t)(s >> 33);
  }
  int below(int n) { return (int)(next() % (uint32_t)n); }
};

// heavy-edge matching; returns false when the graph hardly shrinks
bool coarsen(const Graph& g, Graph& c, std::vector<int>& cmap, Rng& rng) {
  std::vector<int> perm(g.n);
  std::iota(perm.begin(), perm.end(), 0);
  for (int i = g.n - 1; i > 0; i--) std::swap(perm[i], perm[rng.below(i + 1)]);
  const long long maxvw = std::max<long long>(1, (long long)(1.5 * g.tw / kCoarsest));
  std::vector<int> match(g.n, -1), rep;
  cmap.assign(g.n, -1);
  rep.reserve(g.n);
  for (int v : perm) {
    if (match[v] >= 0) continue;
    int best = -1, bw = -1;
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++) {
      const int u = g.adj[k];
      if (match[u] >= 0 || u == v || g.vw[v] + g.vw[u] > maxvw) continue;
      if (g.ew[k] > bw || (g.ew[k] == bw && g.vw[u] < g.vw[best])) {
        best = u;
        bw = g.ew[k];
      }
    }
    const int id = (int)rep.size();
    rep.push_back(v);
    cmap[v] = id;
    match[v] = best < 0 ? v : best;
    if (best >= 0) {
      match[best] = v;
      cmap[best] = id;
    }
  }
  const int nc = (int)rep.size();
  if (nc > 0.93 * g.n) return false;
  c.n = nc;
  c.tw = g.tw;
  c.vw.assign(nc, 0);
  c.xadj.assign(nc + 1, 0);
  c.adj.clear();
  c.ew.clear();
  std::vector<int> mark(nc, -1), pos(nc, 0);
  for (int id = 0; id < nc; id++) {
    const int v = rep[id], u = match[v];
    c.vw[id] = g.vw[v] + (u != v ? g.vw[u] : 0);
    for (int x : {v, u}) {
      for (int k = g.xadj[x]; k < g.xadj[x + 1]; k++) {
        const int t = cmap[g.adj[k]];
        if (t == id) continue;
        if (mark[t] != id) {
          mark[t] = id;
          pos[t] = (int)c.adj.size();
          c.adj.push_back(t);
          c.ew.push_back(g.ew[k]);
        } else {
          c.ew[pos[t]] += g.ew[k];
        }
      }
      if (u == v) break;
    }
    c.xadj[id + 1] = (int)c.adj.size();
  }
  return true;
}

long long cut_of(const Graph& g, const std::vector<char>& part) {
  long long cut = 0;
  for (int v = 0; v < g.n; v++)
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++)
      if (part[g.adj[k]] != part[v]) cut += g.ew[k];
  return cut / 2;
}

// Fiduccia-Mattheyses passes on the edge cut under the balance bound; a state
// is better when it violates the bound less, then when it cuts less.
void refine(const Graph& g, std::vector<char>& part, int passes) {
  const long long maxw = std::max<long long>((long long)(kMaxSide * g.tw + 0.5), (g.tw + 1) / 2);
  std::vector<int> id(g.n, 0), ed(g.n, 0);
  long long pw[2] = {0, 0};
  long long cut = 0;
  for (int v = 0; v < g.n; v++) {
    pw[(int)part[v]] += g.vw[v];
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++) (part[g.adj[k]] == part[v] ? id[v] : ed[v]) += g.ew[k];
    cut += ed[v];
  }
  cut /= 2;
  auto viol = [&]() { return std::max<long long>(0, std::max(pw[0], pw[1]) - maxw); };
  std::vector<char> locked(g.n, 0);
  std::vector<int> moves;
  const int limit = std::max(64, g.n / 50);
  for (int pass = 0; pass < passes; pass++) {
    std::priority_queue<std::pair<int, int>> heap;
    for (int v = 0; v < g.n; v++)
      if (ed[v] > 0 || viol() > 0) heap.push({ed[v] - id[v], v});
    std::fill(locked.begin(), locked.end(), 0);
    moves.clear();
    long long best_cut = cut, best_viol = viol();
    size_t best_at = 0;
    auto move = [&](int v) {
      const int from = part[v], to = 1 - from;
      part[v] = (char)to;
      pw[from] -= g.vw[v];
      pw[to] += g.vw[v];
      cut -= ed[v] - id[v];
      std::swap(id[v], ed[v]);
      for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++) {
        const int u = g.adj[k];
        if (part[u] == to) {
          id[u] += g.ew[k];
          ed[u] -= g.ew[k];
        } else {
          id[u] -= g.ew[k];
          ed[u] += g.ew[k];
        }
      }
    };
    while (!heap.empty()) {
      const auto [gain, v] = heap.top();
      heap.pop();
      if (locked[v] || gain != ed[v] - id[v]) continue;
      const int from = part[v], to = 1 - from;
      const long long vb = viol();
      // moves must not make the balance worse than the bound (or the current violation)
      if (pw[to] + g.vw[v] > std::max(maxw, vb > 0 ? pw[from] - 1 : maxw)) continue;
      if (vb > 0 && pw[to] >= pw[from]) continue;
      move(v);
      locked[v] = 1;
      moves.push_back(v);
      for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++) {
        const int u = g.adj[k];
        if (!locked[u] && ed[u] > 0) heap.push({ed[u] - id[u], u});
      }
      const long long cv = viol();
      if (cv < best_viol || (cv == best_viol && cut < best_cut)) {
        best_viol = cv;
        best_cut = cut;
        best_at = moves.size();
      } else if (moves.size() - best_at > (size_t)limit) {
        break;
      }
    }
    for (size_t q = moves.size(); q > best_at; q--) move(moves[q - 1]);
    if (best_at == 0) break;
  }
}

// greedy region growing from a seed: add the frontier vertex that adds the
// least cut until the grown side holds half the weight
std::vector<char> grow(const Graph& g, int seed, Rng& rng) {
  std::vector<char> part(g.n, 1);
  std::vector<int> conn(g.n, 0);   // edge weight into the grown side
  long long w0 = 0;
  const long long half = g.tw / 2;
  std::vector<char> inq(g.n, 0);
  int v = seed;
  while (w0 < half) {
    part[v] = 0;
    w0 += g.vw[v];
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++) {
      conn[g.adj[k]] += g.ew[k];
      inq[g.adj[k]] = 1;
    }
    if (w0 >= half) break;
    int best = -1;
    long long bg = 0;
    for (int u = 0; u < g.n; u++) {
      if (part[u] == 0 || !inq[u]) continue;
      long long tot = 0;
      for (int k = g.xadj[u]; k < g.xadj[u + 1]; k++) tot += g.ew[k];
      const long long gain = 2LL * conn[u] - tot;
      if (best < 0 || gain > bg) {
        best = u;
        bg = gain;
      }
    }
    if (best < 0) {   // frontier empty (disconnected): any vertex still outside
      std::vector<int> rest;
      for (int u = 0; u < g.n; u++)
        if (part[u] == 1) rest.push_back(u);
      if (rest.empty()) break;
      best = rest[rng.below((int)rest.size())];
    }
    v = best;
  }
  return part;
}

std::vector<char> bisect(const Graph& g0, Rng& rng) {
  std::vector<Graph> gs;
  std::vector<std::vector<int>> maps;
  gs.push_back(g0);
  while (gs.back().n > kCoarsest) {
    Graph c;
    std::vector<int> cmap;
    if (!coarsen(gs.back(), c, cmap, rng)) break;
    gs.push_back(std::move(c));
    maps.push_back(std::move(cmap));
  }
  const Graph& top = gs.back();
  std::vector<char> best;
  long long best_cut = -1;
  for (int t = 0; t < kInitTries && top.n > 0; t++) {
    std::vector<char> p = grow(top, rng.below(top.n), rng);
    refine(top, p, 8);
    const long long c = cut_of(top, p);
    if (best_cut < 0 || c < best_cut) {
      best_cut = c;
      best.swap(p);
    }
  }
  for (int l = (int)gs.size() - 2; l >= 0; l--) {
    std::vector<char> p(gs[l].n);
    for (int v = 0; v < gs[l].n; v++) p[v] = best[maps[l][v]];
    best.swap(p);
    refine(gs[l], best, 6);
  }
  return best;
}

// minimum vertex cover of the cut edges (Hopcroft-Karp + Koenig); in[v] = 1 for covered
std::vector<char> cut_cover(const Graph& g, const std::vector<char>& part) {
  std::vector<int> L, R, lid(g.n, -1), rid(g.n, -1);
  for (int v = 0; v < g.n; v++)
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++)
      if (part[g.adj[k]] != part[v]) {
        if (part[v] == 0) {
          lid[v] = (int)L.size();
          L.push_back(v);
        } else {
          rid[v] = (int)R.size();
          R.push_back(v);
        }
        break;
      }
  const int nl = (int)L.size(), nr = (int)R.size();
  std::vector<int> ml(nl, -1), mr(nr, -1), dist(nl);
  auto nbrs = [&](int l, auto&& f) {
    const int v = L[l];
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++)
      if (rid[g.adj[k]] >= 0) f(rid[g.adj[k]]);
  };
  const int INF = 1 << 30;
  for (;;) {   // Hopcroft-Karp phases
    std::queue<int> q;
    for (int l = 0; l < nl; l++) {
      dist[l] = ml[l] < 0 ? 0 : INF;
      if (ml[l] < 0) q.push(l);
    }
    bool found = false;
    while (!q.empty()) {
      const int l = q.front();
      q.pop();
      nbrs(l, [&](int r) {
        const int l2 = mr[r];
        if (l2 < 0) found = true;
        else if (dist[l2] == INF) {
          dist[l2] = dist[l] + 1;
          q.push(l2);
        }
      });
    }
    if (!found) break;
    // iterative DFS along the layered graph
    std::vector<int> it(nl, 0);
    for (int s = 0; s < nl; s++) {
      if (ml[s] >= 0) continue;
      std::vector<int> stk{s};
      std::vector<int> via;   // right vertex taken from each stacked left vertex
      while (!stk.empty()) {
        const int l = stk.back();
        const int v = L[l];
        bool advanced = false;
        while (g.xadj[v] + it[l] < g.xadj[v + 1]) {
          const int u = g.adj[g.xadj[v] + it[l]++];
          const int r = rid[u];
          if (r < 0) continue;
          const int l2 = mr[r];
          if (l2 < 0) {   // augment along the stack
            via.push_back(r);
            for (size_t d = 0; d < stk.size(); d++) {
              ml[stk[d]] = via[d];
              mr[via[d]] = stk[d];
            }
            stk.clear();
            advanced = true;
            break;
          }
          if (dist[l2] == dist[l] + 1) {
            via.push_back(r);
            stk.push_back(l2);
            advanced = true;
            break;
          }
        }
        if (!advanced) {
          dist[l] = INF;
          stk.pop_back();
          if (!via.empty()) via.pop_back();
        }
      }
    }
  }
  // Koenig: Z = vertices reachable from unmatched left ones by alternating paths;
  // cover = (L \ Z) u (R n Z)
  std::vector<char> zl(nl, 0), zr(nr, 0);
  std::vector<int> stk;
  for (int l = 0; l < nl; l++)
    if (ml[l] < 0) {
      zl[l] = 1;
      stk.push_back(l);
    }
  while (!stk.empty()) {
    const int l = stk.back();
    stk.pop_back();
    nbrs(l, [&](int r) {
      if (zr[r]) return;
      zr[r] = 1;
      const int l2 = mr[r];
      if (l2 >= 0 && !zl[l2]) {
        zl[l2] = 1;
        stk.push_back(l2);
      }
    });
  }
  std::vector<char> in(g.n, 0);
  for (int l = 0; l < nl; l++)
    if (!zl[l]) in[L[l]] = 1;
  for (int r = 0; r < nr; r++)
    if (zr[r]) in[R[r]] = 1;
  return in;
}

Graph induced(const Graph& g, const std::vector<int>& verts, std::vector<int>& local) {
  Graph s;
  s.n = (int)verts.size();
  for (int i = 0; i < s.n; i++) local[verts[i]] = i;
  s.xadj.assign(s.n + 1, 0);
  s.vw.assign(s.n, 1);
  s.tw = s.n;
  for (int i = 0; i < s.n; i++) {
    const int v = verts[i];
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++) {
      const int u = local[g.adj[k]];
      if (u >= 0) {
        s.adj.push_back(u);
        s.ew.push_back(1);
      }
    }
    s.xadj[i + 1] = (int)s.adj.size();
  }
  for (int v : verts) local[v] = -1;
  return s;
}

// exact minimum degree on a graph of at most 64 vertices (adjacency bitmasks)
void leaf_order(const Graph& g, const std::vector<int>& gid, std::vector<int>& order) {
  uint64_t nb[64], alive = g.n == 64 ? ~0ULL : ((1ULL << g.n) - 1);
  for (int v = 0; v < g.n; v++) {
    nb[v] = 0;
    for (int k = g.xadj[v]; k < g.xadj[v + 1]; k++) nb[v] |= 1ULL << g.adj[k];
  }
  for (int step = 0; step < g.n; step++) {
    int p = -1, pd = 1 << 30;
    for (uint64_t a = alive; a; a &= a - 1) {
      const int v = __builtin_ctzll(a);
      const int d = __builtin_popcountll(nb[v] & alive);
      if (d < pd) {
        pd = d;
        p = v;
      }
    }
    alive &= ~(1ULL << p);
    const uint64_t clique = nb[p] & alive;
    for (uint64_t a = clique; a; a &= a - 1) {
      const int u = __builtin_ctzll(a);
      nb[u] |= clique & ~(1ULL << u);
    }
    order.push_back(gid[p]);
  }
}

// g: unit-weight subgraph, gid: its vertices' global ids; returns its ordering
// (global ids).  Large halves recurse on their own thread (each subtree has its
// own generator, so the result does not depend on the scheduling).
std::vector<int> nd(const Graph& g, const std::vector<int>& gid, uint64_t seed, int depth) {
  std::vector<int> order;
  order.reserve(g.n);
  if (g.n <= kLeaf) {
    leaf_order(g, gid, order);
    return order;
  }
  // near the root of the dissection the separators become the largest fronts
  // and the longest panel chains: there the bisection is tried from several
  // seeds (concurrently) and the smallest separator kept (ties: the first try)
  static const int top = getenv("PGO_ND_TRIES") ? std::max(1, atoi(getenv("PGO_ND_TRIES"))) : kTopTries;   // (A/B knob)
  const int tries = depth == 0 ? top : depth < kTriedDepth ? std::max(1, top / 2) : 1;
  std::vector<std::vector<char>> parts(tries), seps(tries);
  auto attempt = [&](int t) {
    Rng rng(seed + 0x632be59bd9b4e019ULL * (uint64_t)t);
    parts[t] = bisect(g, rng);
    seps[t] = cut_cover(g, parts[t]);
  };
  if (tries > 1 && g.n > 4096) {
    std::vector<std::thread> th;
    for (int t = 1; t < tries; t++) th.emplace_back(attempt, t);
    attempt(0);
    for (auto& x : th) x.join();
  } else {
    for (int t = 0; t < tries; t++) attempt(t);
  }
  int pick = 0;
  long long best = -1;
  for (int t = 0; t < tries; t++) {
    long long ns = 0;
    for (char v : seps[t]) ns += v;
    if (best < 0 || ns < best) {
      best = ns;
      pick = t;
    }
  }
  const std::vector<char>& part = parts[pick];
  const std::vector<char>& sep = seps[pick];
  std::vector<int> side[2], sv;
  for (int v = 0; v < g.n; v++) (sep[v] ? sv : side[(int)part[v]]).push_back(v);
  if (side[0].empty() || side[1].empty()) {   // no useful split
    for (int v : order_amd(g.n, g.xadj, g.adj)) order.push_back(gid[v]);
    return order;
  }
  Graph sg[2];
  std::vector<int> sgid[2];
  {
    std::vector<int> scratch(g.n, -1);
    for (int h = 0; h < 2; h++) {
      sg[h] = induced(g, side[h], scratch);
      sgid[h].resize(side[h].size());
      for (size_t i = 0; i < side[h].size(); i++) sgid[h][i] = gid[side[h][i]];
    }
  }
  std::vector<int> sub[2];
  const uint64_t s0 = seed * 0x9e3779b97f4a7c15ULL + 1, s1 = seed * 0xbf58476d1ce4e5b9ULL + 2;
  if (depth < 3 && sg[0].n > 4096 && sg[1].n > 4096) {
    std::thread t([&] { sub[0] = nd(sg[0], sgid[0], s0, depth + 1); });
    sub[1] = nd(sg[1], sgid[1], s1, depth + 1);
    t.join();
  } else {
    sub[0] = nd(sg[0], sgid[0], s0, depth + 1);
    sub[1] = nd(sg[1], sgid[1], s1, depth + 1);
  }
  for (int h = 0; h < 2; h++) order.insert(order.end(), sub[h].begin(), sub[h].end());
  for (int v : sv) order.push_back(gid[v]);
  return order;
}

}  // namespace

std::vector<int> order_nd(int n, const std::vector<int>& xadj, const std::vector<int>& adj) {
  Graph g;
  g.n = n;
  g.xadj = xadj;
  g.adj.reserve(adj.size());
  for (int v = 0; v < n; v++) {
    for (int k = xadj[v]; k < xadj[v + 1]; k++)
      if (adj[k] != v) g.adj.push_back(adj[k]);
    g.xadj[v + 1] = (int)g.adj.size();
  }
  g.ew.assign(g.adj.size(), 1);
  g.vw.assign(n, 1);
  g.tw = n;
  std::vector<int> gid(n);
  std::iota(gid.begin(), gid.end(), 0);
  uint64_t seed = 0x2545f4914f6cdd1dULL;
  if (const char* e = getenv("PGO_ND_SEED")) seed += strtoull(e, nullptr, 10);
  return nd(g, gid, seed, 0);
}

}  // namespace pgo
