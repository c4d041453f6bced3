// Microbenchmark of the Schur-update kernels (k_panel_syrk 64x64 tiles,
// k_panel_syrk128 128x128 tiles) on one front: the outer update of depth 256
// after the first kKB block, the largest launches of a C3 factorisation.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_syrk.hip -o graphslam_amd/build/ubench_syrk
//   ./graphslam_amd/build/ubench_syrk [m] [w]
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace pgo;

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096;
  const int W = argc > 2 ? atoi(argv[2]) : 512;
  hipStream_t st;
  hipStreamCreate(&st);
  const size_t n = (size_t)M * M;
  std::vector<double> h(n);
  srand(3);
  for (size_t i = 0; i < n; i++) h[i] = ((rand() % 2001) - 1000) / 1000.0;
  double *F, *F0;
  hipMalloc(&F, n * 8);
  hipMalloc(&F0, n * 8);
  hipMemcpy(F0, h.data(), n * 8, hipMemcpyHostToDevice);
  int hm = M, hw = W;
  long long hf[2] = {0, (long long)n};
  int *dm, *dw;
  long long* dfo;
  hipMalloc(&dm, 4);
  hipMalloc(&dw, 4);
  hipMalloc(&dfo, 16);
  hipMemcpy(dm, &hm, 4, hipMemcpyHostToDevice);
  hipMemcpy(dw, &hw, 4, hipMemcpyHostToDevice);
  hipMemcpy(dfo, hf, 16, hipMemcpyHostToDevice);
  CholDev c{};
  c.F = F;
  c.m = dm;
  c.w = dw;
  c.foff = dfo;
  // outer update after panel kb = 192 (block 0 = columns 0..255): trailing [256, M), k0 = 0
  const int kb = 192, be = 256;
  const double flops = 256.0 * (M - be) * (M - be + 1.0);
  for (int T : {64, 128}) {
    std::vector<int4> tasks;
    for (int c0 = be; c0 < M; c0 += T)
      for (int r0 = c0; r0 < M; r0 += T) tasks.push_back(make_int4(0, r0, c0, 0));
    int4* dt;
    hipMalloc(&dt, tasks.size() * sizeof(int4));
    hipMemcpy(dt, tasks.data(), tasks.size() * sizeof(int4), hipMemcpyHostToDevice);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int reps = 10;
    float best = 1e30f;
    for (int r = 0; r < reps; r++) {
      hipMemcpyAsync(F, F0, n * 8, hipMemcpyDeviceToDevice, st);
      hipEventRecord(a, st);
      if (T == 64) k_panel_syrk<<<(int)tasks.size(), 256, 0, st>>>(c, dt, kb);
      else k_panel_syrk128<<<(int)tasks.size(), 256, 0, st>>>(c, dt, kb);
      hipEventRecord(b, st);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      best = ms < best ? ms : best;
    }
    // checksum of the trailing lower triangle
    std::vector<double> out(n);
    hipMemcpy(out.data(), F, n * 8, hipMemcpyDeviceToHost);
    double cs = 0;
    for (int j = be; j < M; j += 7)
      for (int i = j; i < M; i += 5) cs += out[i + (size_t)j * M];
    printf("m %d tile %3d: %6zu tasks  %8.1f us  %6.2f TFLOP/s  checksum %.10e\n", M, T, tasks.size(), best * 1e3,
           flops / (best * 1e-3) / 1e12, cs);
    hipFree(dt);
  }
  return 0;
}
