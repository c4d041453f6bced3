// Microbenchmark of the panel-step chain (k_panel_trsm -> k_syrk_diag ->
// k_panel_trsm ...) on one front: per-launch cost of each kernel alone,
// of an empty kernel, and of the alternating chain, eager and in a hipGraph.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_chain.hip -o graphslam_amd/build/ubench_chain
//   ./graphslam_amd/build/ubench_chain [m]
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

using namespace pgo;

__global__ void u_empty(int* p) {
  if (threadIdx.x == 1023) p[0] = 1;
}

static float timeit(hipStream_t st, int reps, const std::function<void()>& body, bool graph) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipGraphExec_t ge = nullptr;
  if (graph) {
    hipGraph_t g;
    hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
    for (int r = 0; r < reps; r++) body();
    hipStreamEndCapture(st, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, st);
  } else {
    for (int r = 0; r < 5; r++) body();
  }
  hipStreamSynchronize(st);
  hipEventRecord(a, st);
  if (graph) hipGraphLaunch(ge, st);
  else
    for (int r = 0; r < reps; r++) body();
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return 1e3f * ms / reps;
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 1024;
  const int W = 256;
  hipStream_t st;
  hipStreamCreate(&st);
  const size_t n = (size_t)M * M;
  std::vector<double> h(n, 0.0);
  srand(5);
  for (int j = 0; j < M; j++)
    for (int i = j; i < M; i++) h[i + (size_t)j * M] = i == j ? 4.0 * M : ((rand() % 2001) - 1000) / 1000.0;
  double *F, *T, *fv;
  hipMalloc(&F, n * 8);
  hipMalloc(&T, (size_t)(W / 64) * 4096 * 8);
  hipMalloc(&fv, M * 8);
  hipMemcpy(F, h.data(), n * 8, hipMemcpyHostToDevice);
  hipMemset(T, 0, (size_t)(W / 64) * 4096 * 8);
  hipMemset(fv, 0, M * 8);
  int hm = M, hw = W, hv = 0;
  long long hf[2] = {0, (long long)n}, ht[2] = {0, (long long)(W / 64) * 4096};
  int *dm, *dw, *dv, *flag, *dump;
  long long *dfo, *dto;
  hipMalloc(&dm, 4);
  hipMalloc(&dw, 4);
  hipMalloc(&dv, 8);
  hipMalloc(&flag, 4);
  hipMalloc(&dump, 4);
  hipMalloc(&dfo, 16);
  hipMalloc(&dto, 16);
  hipMemcpy(dm, &hm, 4, hipMemcpyHostToDevice);
  hipMemcpy(dw, &hw, 4, hipMemcpyHostToDevice);
  hipMemcpy(dv, &hv, 4, hipMemcpyHostToDevice);
  hipMemcpy(dfo, hf, 16, hipMemcpyHostToDevice);
  hipMemcpy(dto, ht, 16, hipMemcpyHostToDevice);
  hipMemset(flag, 0, 4);
  CholDev c{};
  c.F = F;
  c.m = dm;
  c.w = dw;
  c.foff = dfo;
  c.Tinv = T;
  c.toff = dto;
  c.fv = fv;
  c.voff = dv;
  c.flag = flag;
  // panel kb = 64 (inside the first 256-block): trsm chunks of rows [128, M),
  // look-ahead diagonal tile of panel 128 with depth from 0
  const int kb = 64;
  std::vector<int2> tt;
  for (int ch = 0; ch * 64 < M - kb - 64; ch++) tt.push_back(make_int2(0, ch));
  int4 sd = make_int4(0, kb + 64, kb + 64, (int)0x80000000);
  int list0 = 0;
  int2* dtt;
  int4* dsd;
  int* dl;
  hipMalloc(&dtt, tt.size() * sizeof(int2));
  hipMalloc(&dsd, sizeof(int4));
  hipMalloc(&dl, 4);
  hipMemcpy(dtt, tt.data(), tt.size() * sizeof(int2), hipMemcpyHostToDevice);
  hipMemcpy(dsd, &sd, sizeof(int4), hipMemcpyHostToDevice);
  hipMemcpy(dl, &list0, 4, hipMemcpyHostToDevice);
  const int nt = (int)tt.size();
  printf("m %d: trsm %d workgroups\n", M, nt);
  const int reps = 200;
  for (int g = 0; g < 2; g++) {
    const char* mode = g ? "graph" : "eager";
    printf("%s: empty 1 WG            %7.2f us\n", mode,
           timeit(st, reps, [&] { u_empty<<<1, 64, 0, st>>>(dump); }, g));
    printf("%s: empty 256 WG          %7.2f us\n", mode,
           timeit(st, reps, [&] { u_empty<<<256, 256, 0, st>>>(dump); }, g));
    printf("%s: k_panel_trsm          %7.2f us\n", mode,
           timeit(st, reps, [&] { k_panel_trsm<<<nt, 256, 0, st>>>(c, dtt, kb); }, g));
    printf("%s: k_panel_trsm 1 WG     %7.2f us\n", mode,
           timeit(st, reps, [&] { k_panel_trsm<<<1, 256, 0, st>>>(c, dtt, kb); }, g));
    printf("%s: k_panel_diag          %7.2f us\n", mode,
           timeit(st, reps, [&] { k_panel_diag<<<1, 256, 0, st>>>(c, dl, kb + 64); }, g));
    printf("%s: k_syrk_diag           %7.2f us\n", mode,
           timeit(st, reps, [&] { k_syrk_diag<<<1, 256, 0, st>>>(c, dsd, kb); }, g));
    printf("%s: trsm + syrk_diag      %7.2f us\n", mode, timeit(st, reps, [&] {
             k_panel_trsm<<<nt, 256, 0, st>>>(c, dtt, kb);
             k_syrk_diag<<<1, 256, 0, st>>>(c, dsd, kb);
           }, g));
    printf("%s: empty + empty         %7.2f us\n", mode, timeit(st, reps, [&] {
             u_empty<<<nt, 256, 0, st>>>(dump);
             u_empty<<<1, 256, 0, st>>>(dump);
           }, g));
  }
  int fl = 0;
  hipMemcpy(&fl, flag, 4, hipMemcpyDeviceToHost);
  printf("flag %d (values are not meaningful: repeated in-place updates)\n", fl);
  return 0;
}
