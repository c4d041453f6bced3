// Host-only timing of the live re-solve's plan update (chol_append): the plan
// of an edge list's graph, then R registrations of one pose each (odometry to
// the previous pose + one loop closure to an old pose), as bench.py's live line.
//   hipcc -O2 -std=c++17 -I include scripts/live_plan_bench.cpp graphslam_amd/csrc/pgo_symbolic.cpp \
//     graphslam_amd/csrc/pgo_order.cpp -o /tmp/live_plan_bench
//   PGO_PLAN_TIMING=1 /tmp/live_plan_bench edges.bin n [R]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../graphslam_amd/csrc/pgo_chol.h"

static void pattern(int n, const std::vector<int>& e, std::vector<int>& row_ptr, std::vector<int>& col) {
  const int ne = (int)e.size() / 2;
  row_ptr.assign(n + 1, 0);
  for (int q = 0; q < ne; q++) {
    row_ptr[e[2 * q] + 1]++;
    row_ptr[e[2 * q + 1] + 1]++;
  }
  for (int i = 0; i < n; i++) row_ptr[i + 1] += row_ptr[i];
  std::vector<int> fill(row_ptr.begin(), row_ptr.end() - 1);
  col.assign(row_ptr[n], 0);
  for (int q = 0; q < ne; q++) {
    col[fill[e[2 * q]]++] = e[2 * q + 1];
    col[fill[e[2 * q + 1]]++] = e[2 * q];
  }
  for (int i = 0; i < n; i++) std::sort(col.begin() + row_ptr[i], col.begin() + row_ptr[i + 1]);
}

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  int n = atoi(argv[2]);
  const int R = argc > 3 ? atoi(argv[3]) : 5;
  std::vector<int> e;
  int buf[2];
  while (fread(buf, 4, 2, f) == 2) {
    e.push_back(buf[0]);
    e.push_back(buf[1]);
  }
  fclose(f);
  std::vector<int> row_ptr, col;
  pattern(n, e, row_ptr, col);
  pgo::CholPlan P;
  auto t0 = std::chrono::steady_clock::now();
  pgo::chol_analyze(P, n, row_ptr, col);
  printf("analysis %.3f s, %d fronts\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(),
         P.ns);
  // the library binds the plan after every update (sources -> factor indices,
  // pgo_api.cpp bind_plan), which lets the next append splice the assembly
  // targets; emulated (timing only: any bound value)
  auto bind = [&] {
    for (int& x : P.asm_src)
      if (x < 0) x = 0;
    P.asm_bound = true;
  };
  if (!getenv("NO_BIND")) bind();
  std::mt19937 rng(7);
  std::vector<double> ms;
  for (int r = 0; r < R; r++) {
    const int v = n, a = (int)(rng() % (unsigned)(n - 1));
    e.push_back(v - 1);
    e.push_back(v);
    e.push_back(a);
    e.push_back(v);
    n++;
    pattern(n, e, row_ptr, col);
    std::vector<int2> pairs{make_int2(v - 1, v), make_int2(a, v)};
    t0 = std::chrono::steady_clock::now();
    const bool ok = pgo::chol_append(P, n, row_ptr, col, pairs, 64, 1.05);
    ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    if (!ok) return 1;
    if (!getenv("NO_BIND")) bind();
  }
  std::sort(ms.begin() + 1, ms.end());
  printf("chol_append: first %.2f ms, then min %.2f median %.2f ms over %d\n", ms[0], ms[1], ms[1 + (R - 1) / 2],
         R - 1);
  return 0;
}
