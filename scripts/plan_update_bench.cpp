// Host timing of the live re-solve's plan update (chol_append, the incremental
// symbolic update) against a full analysis, on an edge list (int32 pairs):
// registrations of one pose each (odometry to the previous pose + one loop
// closure to a random earlier pose), as bench.py's live_resolve.
//   hipcc -O2 -std=c++17 scripts/plan_update_bench.cpp graphslam_amd/csrc/pgo_symbolic.cpp \
//     graphslam_amd/csrc/pgo_order.cpp -o /tmp/plan_update_bench
//   PGO_PLAN_TIMING=1 /tmp/plan_update_bench edges.bin n [registrations]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../graphslam_amd/csrc/pgo_chol.h"

static void pattern(int n, const std::vector<int>& e, std::vector<int>& row_ptr, std::vector<int>& col) {
  std::vector<std::vector<int>> adj(n);
  for (size_t q = 0; q + 1 < e.size(); q += 2) {
    adj[e[q]].push_back(e[q + 1]);
    adj[e[q + 1]].push_back(e[q]);
  }
  row_ptr.assign(1, 0);
  col.clear();
  for (int i = 0; i < n; i++) {
    adj[i].push_back(i);
    std::sort(adj[i].begin(), adj[i].end());
    adj[i].erase(std::unique(adj[i].begin(), adj[i].end()), adj[i].end());
    col.insert(col.end(), adj[i].begin(), adj[i].end());
    row_ptr.push_back((int)col.size());
  }
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  int n = atoi(argv[2]);
  const int regs = argc > 3 ? atoi(argv[3]) : 5;
  std::vector<int> e;
  int buf[2];
  while (fread(buf, 4, 2, f) == 2) e.insert(e.end(), buf, buf + 2);
  fclose(f);
  std::vector<int> row_ptr, col;
  pattern(n, e, row_ptr, col);
  pgo::CholPlan P;
  auto t0 = std::chrono::steady_clock::now();
  pgo::chol_analyze(P, n, row_ptr, col);
  auto ms = [](auto a) { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count(); };
  printf("full analysis %.1f ms, %d fronts, flops %.4g, F %.3g doubles\n", ms(t0), P.ns, P.flops, (double)P.ftotal);
  std::mt19937 rng(7);
  for (int r = 0; r < regs; r++) {
    const int v = n;
    const int j = (int)(rng() % (unsigned)(v - 20));
    e.insert(e.end(), {v - 1, v, v, j});
    n++;
    pattern(n, e, row_ptr, col);
    std::vector<int2> pairs{make_int2(v - 1, v), make_int2(v, j)};
    t0 = std::chrono::steady_clock::now();
    const bool ok = pgo::chol_append(P, n, row_ptr, col, pairs, 1 << 30, 1e30);
    printf("registration %d: append %s %.1f ms, %d fronts, flops %.4g, F %.3g\n", r, ok ? "ok" : "REFUSED", ms(t0),
           P.ns, P.flops, (double)P.ftotal);
  }
  return 0;
}
