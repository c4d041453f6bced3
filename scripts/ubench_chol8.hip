// Cycles of the lane-redundant 8x8 pieces of the diagonal-block chain
// (chol8_lane, inv8_lane of pgo_chol.hip) on one wave, back to back with a
// data dependence between calls, and of a 16x16 lane-redundant factor +
// inverse in registers (chol16 / inv16 below: 136 values per lane), to price
// the diagonal block's alternatives.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_chol8.hip -o graphslam_amd/build/ubench_chol8
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>

using namespace pgo;

#define P16(i, j) ((i) * ((i) + 1) / 2 + (j))

__device__ __forceinline__ bool chol16_lane(double (&a)[136], double (&iv)[16]) {
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 16; j++) {
    double d = a[P16(j, j)];
    if (!(d > 0.0) || !isfinite(d)) {
      bad = true;
      d = 1.0;
    }
    const double inv = rsqrt_nr(d);
    iv[j] = inv;
    a[P16(j, j)] = d * inv;
#pragma unroll
    for (int i = j + 1; i < 16; i++) a[P16(i, j)] *= inv;
#pragma unroll
    for (int i = j + 1; i < 16; i++)
#pragma unroll
      for (int k = j + 1; k <= i; k++) a[P16(i, k)] = fma(-a[P16(i, j)], a[P16(k, j)], a[P16(i, k)]);
  }
  return bad;
}

template <int kMode>   // 0: chol8, 1: chol8 + inv8, 2: chol16, 3: 2x(chol8+inv8) (the diag16 scalar part)
__global__ __launch_bounds__(64) void u_chol(const double* A, double* out, long long* clk, int reps) {
  const int l = threadIdx.x;
  double a8[36], iv8[8], a16[136], iv16[16];
#pragma unroll
  for (int i = 0; i < 36; i++) a8[i] = A[i];
#pragma unroll
  for (int i = 0; i < 136; i++) a16[i] = A[i];
  double acc = 0;
  const long long t0 = clock64();
  for (int r = 0; r < reps; r++) {
    if (kMode == 0 || kMode == 1 || kMode == 3) {
      double b[36];
#pragma unroll
      for (int i = 0; i < 36; i++) b[i] = a8[i] + acc * 1e-300;
      acc += chol8_lane(b, iv8) ? 1.0 : 0.0;
      if (kMode >= 1) inv8_lane(b, iv8);
      if (kMode == 3) {
        double c[36];
#pragma unroll
        for (int i = 0; i < 36; i++) c[i] = a8[i] + b[i] * 1e-300;
        acc += chol8_lane(c, iv8) ? 1.0 : 0.0;
        inv8_lane(c, iv8);
        acc += c[35] * 1e-300;
      }
      acc += b[35] * 1e-300;
    } else {
      double b[136];
#pragma unroll
      for (int i = 0; i < 136; i++) b[i] = a16[i] + acc * 1e-300;
      acc += chol16_lane(b, iv16) ? 1.0 : 0.0;
      acc += b[135] * 1e-300;
    }
  }
  const long long t1 = clock64();
  out[l] = acc;
  if (l == 0) clk[0] = t1 - t0;
}

template <int kMode>
static void run(const char* name, const double* dA, double* dO, long long* dc) {
  u_chol<kMode><<<1, 64>>>(dA, dO, dc, 4);
  hipDeviceSynchronize();
  u_chol<kMode><<<1, 64>>>(dA, dO, dc, 64);
  long long c = 0;
  hipMemcpy(&c, dc, sizeof(c), hipMemcpyDeviceToHost);
  printf("%-22s %.0f cycles per call\n", name, (double)c / 64);
}

int main() {
  double h[136];
  for (int i = 0; i < 16; i++)
    for (int j = 0; j <= i; j++) h[P16(i, j)] = (i == j ? 40.0 : 0.0) + 1.0 / (1.0 + i + j);
  double h8[36];
  for (int i = 0; i < 8; i++)
    for (int j = 0; j <= i; j++) h8[P8(i, j)] = h[P16(i, j)];
  double *dA, *dA8, *dO;
  long long* dc;
  hipMalloc(&dA, sizeof(h));
  hipMalloc(&dA8, sizeof(double) * 136);
  hipMalloc(&dO, 64 * sizeof(double));
  hipMalloc(&dc, 8 * sizeof(long long));
  hipMemcpy(dA, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemcpy(dA8, h8, sizeof(h8), hipMemcpyHostToDevice);
  run<0>("chol8_lane", dA8, dO, dc);
  run<1>("chol8_lane + inv8_lane", dA8, dO, dc);
  run<3>("2 x (chol8 + inv8)", dA8, dO, dc);
  run<2>("chol16_lane", dA, dO, dc);
  return 0;
}
