// Microbenchmark of the one-wavefront small-front kernel (k_front_wave) on
// synthetic SPD fronts of one shape; per-phase clocks of front 0.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_wave.hip -o graphslam_amd/build/ubench_wave
//   ./graphslam_amd/build/ubench_wave [fronts] [m] [w]
#ifndef UB_NO_CLOCKS   // (-DUB_NO_CLOCKS: no fenced phase stamps -- the launch times without their fences)
#define PGO_DIAG_CLOCKS 1
#endif
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

using namespace pgo;

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 4096;
  const int M = argc > 2 ? atoi(argv[2]) : 80;
  const int W = argc > 3 ? atoi(argv[3]) : 15;
  if (W > kWaveW || M > kSmallFront || W > M) return 1;
  hipStream_t st;
  hipStreamCreate(&st);
  std::vector<double> h((size_t)N * M * M, 0.0);
  srand(5);
  for (int s = 0; s < N; s++)
    for (int j = 0; j < M; j++)
      for (int i = j; i < M; i++)
        h[(size_t)s * M * M + i + (size_t)j * M] = i == j ? 64.0 : ((rand() % 2001) - 1000) / 4000.0;
  const size_t bytes = h.size() * 8;
  double *F, *F0, *T, *fv;
  hipMalloc(&F, bytes);
  hipMalloc(&F0, bytes);
  hipMalloc(&T, (size_t)N * 4096 * 8);
  hipMalloc(&fv, (size_t)N * M * 8);
  {
    std::vector<double> hv((size_t)N * M);
    for (size_t q = 0; q < hv.size(); q++) hv[q] = ((int)(q * 2654435761u % 2001) - 1000) / 1000.0;
    hipMemcpy(fv, hv.data(), hv.size() * 8, hipMemcpyHostToDevice);
  }
  hipMemset(T, 0, (size_t)N * 4096 * 8);
  hipMemcpy(F0, h.data(), bytes, hipMemcpyHostToDevice);
  std::vector<int> hm(N, M), hw(N, W), list(N), voff(N + 1);
  std::vector<long long> foff(N + 1), toff(N + 1);
  for (int s = 0; s <= N; s++) {
    foff[s] = (long long)s * M * M;
    toff[s] = (long long)s * 4096;
    voff[s] = s * M;
    if (s < N) list[s] = s;
  }
  auto up = [](auto* hv, size_t n) {
    void* d;
    hipMalloc(&d, n);
    hipMemcpy(d, hv, n, hipMemcpyHostToDevice);
    return d;
  };
  CholDev c{};
  c.F = F;
  c.Tinv = T;
  c.fv = fv;
  c.m = (int*)up(hm.data(), N * 4);
  c.w = (int*)up(hw.data(), N * 4);
  c.voff = (int*)up(voff.data(), (N + 1) * 4);
  c.foff = (long long*)up(foff.data(), (N + 1) * 8);
  c.toff = (long long*)up(toff.data(), (N + 1) * 8);
  int* flag;
  hipMalloc(&flag, 4);
  hipMemset(flag, 0, 4);
  c.flag = flag;
  int* dl = (int*)up(list.data(), N * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    hipMemcpyAsync(F, F0, bytes, hipMemcpyDeviceToDevice, st);
    hipEventRecord(a, st);
    const int WC = W <= 8 ? 8 : W <= 16 ? 16 : kWaveW;   // the plan's panel-width classes
    const size_t lds = (size_t)(M * (WC + 1) + 130 + WC) * 8;
    static const bool wave2 = getenv("UB_WAVE2") != nullptr;   // the two-wave kernel (m > 64, W 16 / 32)
    if (M > 64 && WC >= 16 && wave2) {
      if (WC == 16) k_front_wave2<16><<<N, 128, lds, st>>>(c, dl);
      else k_front_wave2<kWaveW><<<N, 128, lds, st>>>(c, dl);
    } else if (M > 64) {
      if (WC == 8) k_front_wave<8, true><<<N, 64, lds, st>>>(c, dl);
      else if (WC == 16) k_front_wave<16, true><<<N, 64, lds, st>>>(c, dl);
      else k_front_wave<kWaveW, true><<<N, 64, lds, st>>>(c, dl);
    } else {
      if (WC == 8) k_front_wave<8, false><<<N, 64, lds, st>>>(c, dl);
      else if (WC == 16) k_front_wave<16, false><<<N, 64, lds, st>>>(c, dl);
      else k_front_wave<kWaveW, false><<<N, 64, lds, st>>>(c, dl);
    }
    hipEventRecord(b, st);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    best = ms < best ? ms : best;
  }
  // check: the lower triangle of fronts 0, N/2, N-1 against a host partial
  // Cholesky (w pivots, then the trailing update)
  std::vector<double> out(h.size());
  hipMemcpy(out.data(), F, bytes, hipMemcpyDeviceToHost);
  double maxd = 0;
  for (int s : {0, N / 2, N - 1}) {
    std::vector<double> A(h.begin() + (size_t)s * M * M, h.begin() + (size_t)(s + 1) * M * M);
    for (int k = 0; k < W; k++) {
      const double p = std::sqrt(A[k + k * M]);
      A[k + k * M] = p;
      for (int i = k + 1; i < M; i++) A[i + k * M] /= p;
      for (int j = k + 1; j < M; j++)
        for (int i = j; i < M; i++) A[i + j * M] -= A[i + k * M] * A[j + k * M];
    }
    for (int j = 0; j < M; j++)
      for (int i = j; i < M; i++) {
        const double d = std::fabs(A[i + j * M] - out[(size_t)s * M * M + i + (size_t)j * M]);
        maxd = d > maxd ? d : maxd;
      }
  }
  printf("  max |F - host| over 3 fronts: %.3g\n", maxd);
  {   // bitwise fingerprint of every output (F, frontal vectors, inverses): old / new builds compare equal
    std::vector<double> vv((size_t)N * M), tt((size_t)N * 4096);
    hipMemcpy(vv.data(), fv, vv.size() * 8, hipMemcpyDeviceToHost);
    hipMemcpy(tt.data(), T, tt.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long hsh = 1469598103934665603ULL;
    auto mix = [&](const std::vector<double>& a) {
      for (double x : a) {
        unsigned long long u;
        memcpy(&u, &x, 8);
        hsh = (hsh ^ u) * 1099511628211ULL;
      }
    };
    mix(out);
    mix(vv);
    mix(tt);
    printf("  output fingerprint %016llx\n", hsh);
  }
#ifndef UB_NO_CLOCKS
  long long clk[32];
  hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_diag_clk), sizeof(clk));
#endif
  int fl = 0;
  hipMemcpy(&fl, flag, 4, hipMemcpyDeviceToHost);
  printf("fronts %d m %d w %d: %.1f us per launch (%.3f us per front), flag %d\n", N, M, W, best * 1e3,
         best * 1e3 / N, fl);
#ifndef UB_NO_CLOCKS
  // (k_front_wave: stamps 27 / 28 close the inverse / the trailing update; k_front_wave2: the reverse)
  printf("  front 0 clocks: start->loads %lld factor %lld store %lld then %lld, %lld\n", clk[24] - clk[23],
         clk[25] - clk[24], clk[26] - clk[25], clk[27] - clk[26], clk[28] - clk[27]);
#endif
  return 0;
}
