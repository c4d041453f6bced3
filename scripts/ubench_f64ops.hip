// fp64 VALU issue and latency on one wave (gfx950), for the diagonal-block
// chain (lane-redundant 8x8 factor / inverse): cycles per instruction of
//   indep  : 8 independent v_fma_f64 chains interleaved (issue cost)
//   dep    : one dependent v_fma_f64 chain (latency)
//   rsq    : dependent v_rsq_f64 chain;  rsqnr: rsq + two Newton steps (the pivot)
//   mul    : dependent v_mul_f64 chain
// with 1 wave per SIMD and with 4 waves of the workgroup on 4 SIMDs.
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_f64ops.hip -o graphslam_amd/build/ubench_f64ops
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 1024;

template <int kMode>
__global__ __launch_bounds__(256) void u_ops(double* out, long long* clk, double seed) {
  double a[8];
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = seed + threadIdx.x * 1e-3 + i;
  const double m = 1.0000001, b = 1e-9;
  const long long t0 = clock64();
  if (kMode == 0) {   // 8 independent chains
    for (int it = 0; it < N / 8; it++)
#pragma unroll
      for (int i = 0; i < 8; i++) a[i] = fma(a[i], m, b);
  } else if (kMode == 1) {   // one dependent chain
    for (int it = 0; it < N; it++) a[0] = fma(a[0], m, b);
  } else if (kMode == 2) {   // dependent rsq chain
    for (int it = 0; it < N; it++) a[0] = __builtin_amdgcn_rsq(a[0]) + 1.0;
  } else if (kMode == 3) {   // pivot: rsq + two Newton steps (rsqrt_nr), dependent
    for (int it = 0; it < N / 8; it++) {
      const double d = a[0];
      double y = __builtin_amdgcn_rsq(d);
      y = y * fma(-0.5 * d * y, y, 1.5);
      y = y * fma(-0.5 * d * y, y, 1.5);
      a[0] = y + 1.0;
    }
  } else {   // dependent mul chain
    for (int it = 0; it < N; it++) a[0] = a[0] * m;
  }
  const long long t1 = clock64();
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += a[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int kMode>
static void run(const char* name, int threads, int per, double* d, long long* dc) {
  u_ops<kMode><<<1, threads>>>(d, dc, 1.5);
  hipDeviceSynchronize();
  u_ops<kMode><<<1, threads>>>(d, dc, 1.5);
  long long c = 0;
  hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-6s %3d threads: %lld cycles for %d ops = %.2f cycles/op\n", name, threads, c, per, (double)c / per);
}

int main() {
  double* d;
  long long* dc;
  hipMalloc(&d, sizeof(double) * 256);
  hipMalloc(&dc, sizeof(long long) * 4);
  for (int th : {64, 256}) {
    run<0>("indep", th, N, d, dc);
    run<1>("dep", th, N, d, dc);
    run<2>("rsq", th, 2 * N, d, dc);
    run<3>("rsqnr", th, N / 8, d, dc);
    run<4>("mul", th, N, d, dc);
  }
  return 0;
}
