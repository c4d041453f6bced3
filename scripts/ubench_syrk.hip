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

// 32 panel columns per chunk (69.6 KB of LDS: 2 workgroups per CU instead of
// 4; bitwise the 16-column form) -- round 5's A/B, not kept
__global__ __launch_bounds__(256) void k_panel_syrk_lds32(CholDev c, const int4* __restrict__ tasks, int kb) {
  lane_offset(c);
  __shared__ __attribute__((aligned(16))) double smem[4 * 32 * 68];
  syrk_lds_body<false, 32>(c, tasks[blockIdx.x], kb, smem);
}

__device__ long long g_mclk[4];
template <int NC>
__global__ __launch_bounds__(256) void u_mfma4_peak(double* out, int iters) {
  double a[NC];
#pragma unroll
  for (int q = 0; q < NC; q++) a[q] = 0.0;
  double x = threadIdx.x * 1e-3, y = 1.0 - x;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int q = 0; q < NC; q++) a[q] = __builtin_amdgcn_mfma_f64_4x4x4f64(q & 1 ? x : y, q & 2 ? y : x, a[q], 0, 0, 0);
  }
  double acc = 0;
#pragma unroll
  for (int q = 0; q < NC; q++) acc += a[q];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}
template <int NC>
__global__ __launch_bounds__(256) void u_mfma_peak(double* out, int iters) {
  d4 a[NC];
#pragma unroll
  for (int q = 0; q < NC; q++) a[q] = d4{0, 0, 0, 0};
  double x = threadIdx.x * 1e-3, y = 1.0 - x;
  const long long t0 = clock64(), w0 = wall_clock64();
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int q = 0; q < NC; q++) a[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(q & 1 ? x : y, q & 2 ? y : x, a[q], 0, 0, 0);
  }
  const long long t1 = clock64(), w1 = wall_clock64();
  double acc = 0;
#pragma unroll
  for (int q = 0; q < NC; q++) acc += a[q][q & 3];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    g_mclk[0] = t1 - t0;
    g_mclk[1] = w1 - w0;
  }
}

int main(int argc, char** argv) {
  for (int wpc : {32}) {
    double* o;
    const int nb = 256 * (wpc / 4), iters = 8192;
    hipMalloc(&o, (size_t)nb * 256 * 8);
    u_mfma4_peak<16><<<nb, 256>>>(o, 16);
    hipDeviceSynchronize();
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipEventRecord(a);
    u_mfma4_peak<16><<<nb, 256>>>(o, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double flops = (double)nb * 4 * iters * 16 * 512.0;
    printf("mfma f64 4x4x4_4b: 16 chains/wave, %d waves/CU: %.1f TFLOP/s\n", wpc, flops / (ms * 1e-3) / 1e12);
    hipFree(o);
  }
  for (int NC : {8}) {
    for (int wpc : {32}) {   // waves per CU requested (WGs of 4 waves)
      double* o;
      const int nb = 256 * (wpc / 4), iters = 2048;
      hipMalloc(&o, (size_t)nb * 256 * 8);
      auto run = [&](int it) {
        if (NC == 4) u_mfma_peak<4><<<nb, 256>>>(o, it);
        else if (NC == 8) u_mfma_peak<8><<<nb, 256>>>(o, it);
        else u_mfma_peak<16><<<nb, 256>>>(o, it);
      };
      run(16);
      hipDeviceSynchronize();
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      hipEventRecord(a);
      run(iters);
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      long long mc[4];
      hipMemcpyFromSymbol(mc, HIP_SYMBOL(g_mclk), sizeof(mc));
      const double flops = (double)nb * 4 * iters * NC * 2048.0;
      printf("mfma f64 16x16x4: %2d chains/wave, %d waves/CU: %.1f TFLOP/s, %.1f cycles per MFMA per wave, %.2f GHz\n",
             NC, wpc, flops / (ms * 1e-3) / 1e12, (double)mc[0] / ((double)NC * iters), mc[0] / (mc[1] * 10.0));
      hipFree(o);
    }
  }
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
  // outer update after panel kb = 192 (block 0 = columns 0..255): trailing [256, M), k0 = 0, depth 256;
  // then the same tiles at depth 64 (kb = 0: one panel, the inner steps' depth)
  for (const int kb : {192, 0}) {
  const int be = 256, depth = kb + 64;
  const double flops = (double)depth * (M - be) * (M - be + 1.0);
  for (int T : {64, 65, 66, 67, 128}) {   // 65: the LDS-staged 64x64 kernel; 66: the same with the C tile prefetched; 67: 32-column chunks
    const int TT = (T >= 65 && T <= 67) ? 64 : T;
    std::vector<int4> tasks;
    for (int c0 = be; c0 < M; c0 += TT)
      for (int r0 = c0; r0 < M; r0 += TT) tasks.push_back(make_int4(0, r0, c0, 0));
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
      else if (T == 65) k_panel_syrk_lds<<<(int)tasks.size(), 256, 0, st>>>(c, dt, kb);
      else if (T == 66) k_panel_syrk_lds_pc<<<(int)tasks.size(), 256, 0, st>>>(c, dt, kb);
      else if (T == 67) k_panel_syrk_lds32<<<(int)tasks.size(), 256, 0, st>>>(c, dt, kb);
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
    printf("m %d depth %3d tile %3d: %6zu tasks  %8.1f us  %6.2f TFLOP/s  checksum %.10e\n", M, depth, T, tasks.size(),
           best * 1e3, flops / (best * 1e-3) / 1e12, cs);
    hipFree(dt);
  }
  }
  return 0;
}
