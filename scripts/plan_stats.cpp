// Host-only statistics of the supernodal plan for an edge list (int32 pairs):
// per level the fronts, panel steps and extend-add volume.
//   hipcc -O2 -std=c++17 -I include scripts/plan_stats.cpp graphslam_amd/csrc/pgo_symbolic.cpp -o /tmp/plan_stats
//   /tmp/plan_stats edges.bin n [nd|amd]
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <string>
#include <chrono>
#include <algorithm>

#include "../graphslam_amd/csrc/pgo_chol.h"

int main(int argc, char** argv) {
  if (argc < 3) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  const int n = atoi(argv[2]);
  std::vector<int> e;
  int buf[2];
  while (fread(buf, 4, 2, f) == 2) {
    e.push_back(buf[0]);
    e.push_back(buf[1]);
  }
  fclose(f);
  const int ne = (int)e.size() / 2;
  std::vector<int> row_ptr(n + 1, 0);
  for (int q = 0; q < ne; q++) {
    row_ptr[e[2 * q] + 1]++;
    row_ptr[e[2 * q + 1] + 1]++;
  }
  for (int i = 0; i < n; i++) row_ptr[i + 1] += row_ptr[i];
  std::vector<int> fill(row_ptr.begin(), row_ptr.end() - 1), col(row_ptr[n]);
  for (int q = 0; q < ne; q++) {
    col[fill[e[2 * q]]++] = e[2 * q + 1];
    col[fill[e[2 * q + 1]]++] = e[2 * q];
  }
  for (int i = 0; i < n; i++) std::sort(col.begin() + row_ptr[i], col.begin() + row_ptr[i + 1]);   // as build_structure
  pgo::CholPlan P;
  if (argc > 3 && std::string(argv[3]) == "amd") P.ordering = pgo::kOrderAmd;
  const auto t0 = std::chrono::steady_clock::now();
  pgo::chol_analyze(P, n, row_ptr, col);
  printf("analysis %.3f s\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  double tri = 0, ftot = 0;
  for (int s = 0; s < P.ns; s++) {
    tri += 0.5 * P.m[s] * (P.m[s] + 1.0);
    ftot += (double)pgo::front_elems(P.m[s], P.w[s]);
  }
  printf("fronts %d, F %.0fM doubles, lower triangles %.0fM, flops %.3g, syrk_flops %.3g\n", P.ns, ftot / 1e6, tri / 1e6,
         P.flops, P.syrk_flops);
  double inv = 0, uel = 0;
  for (int s2 = 0; s2 < P.ns; s2++)
    if (P.parent[s2] >= 0) {
      inv += P.m[P.parent[s2]];
      const double u = P.m[s2] - P.w[s2];
      uel += 0.5 * u * (u + 1);
    }
  printf("inverse maps %.1fM ints, update-matrix elements %.1fM\n", inv / 1e6, uel / 1e6);
  int li = 0;
  for (const auto& lv : P.levels) {
    int nsmall = 0;
    for (const auto& sc : lv.small) nsmall += sc.cnt;
    double ea = 0;   // update matrices extended into this level (lower triangles, doubles)
    for (int q = 0; q < lv.ea_cnt[0]; q++) {
      const int4 t = P.ea_tasks[lv.ea_off[0] + q];
      for (int k = 0; k < t.w; k++) {
        const int4 pr = P.ea_pairs[t.z + k];
        ea += (pr.w & 0xff) * (pr.w >> 8);
      }
    }
    int nfused = 0, ntr = 0, nsy = 0, npotrf = 0, nfar = 0;
    std::string joins;
    for (const auto& ps : lv.panels) {
      for (int q = ps.far_p0; q < ps.far_p0 + ps.far_np; q++)
        joins += " " + std::to_string(&ps - lv.panels.data()) + "->" + std::to_string(lv.far_pieces[q].w) + "(" +
                 std::to_string(lv.far_pieces[q].z) + ")";
      nfar += ps.far_cnt;
      nfused += ps.syrk_inline;
      ntr += ps.fcol_cnt + ps.col_cnt;
      nsy += ps.syrk_cnt;
      npotrf += ps.potrf_cnt;
    }
    printf("level %2d: fronts %6d (small %6d) maxm %5d tiles %6d ea %6.1fM dbl, steps %3zu (inline %3d) potrf %5d trsm %6d syrk %7d\n",
           li++, lv.front_cnt, nsmall, lv.maxm, lv.ea_cnt[0], ea / 1e6, lv.panels.size(), nfused, npotrf, ntr, nsy);
    if (nfar) printf("          far tiles %d, far launches (step->join):%s\n", nfar, joins.c_str());
    {   // assembly: pairs (child rectangles) and H items per tile task
      int hist[6] = {0, 0, 0, 0, 0, 0};
      double items = 0;
      for (int q = 0; q < lv.ea_cnt[0]; q++) {
        const int4 t = P.ea_tasks[lv.ea_off[0] + q];
        hist[std::min(t.w, 5)]++;
        items += P.at_iptr[lv.ea_off[0] + q].y;
      }
      printf("          assembly tiles by child pairs 0/1/2/3/4/5+: %d %d %d %d %d %d, H items per tile %.1f\n", hist[0],
             hist[1], hist[2], hist[3], hist[4], hist[5], lv.ea_cnt[0] ? items / lv.ea_cnt[0] : 0.0);
    }
  }
  for (int size : {2, 4, 8}) {
    std::vector<double> rf;
    double top = 0;
    const auto own = pgo::partition_subtrees(P, size, &rf, &top);
    double mx = 0, sm = 0;
    for (double v : rf) {
      mx = std::max(mx, v);
      sm += v;
    }
    printf("partition %d: top %.1f GFLOP (%.0f%%), subtrees %.1f GFLOP, max rank %.1f GFLOP -> bound %.2fx\n", size,
           top / 1e9, 100 * top / P.flops, sm / 1e9, mx / 1e9, P.flops / (top + mx));
  }
  return 0;
}
