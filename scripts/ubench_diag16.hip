// Phase breakdown of diag16_lane (the 16x16 diagonal block of the 64x64
// factor + inverse): one wave, the block in LDS, fenced clock stamps
// (s_waitcnt + sched_barrier around s_memtime, so no instruction moves across a
// stamp) after each phase of a copy of its body.  Stamps serialise the phases:
// the sum is an upper bound of the unstamped time (printed too).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_diag16.hip -o graphslam_amd/build/ubench_diag16
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>

using namespace pgo;

#define ST(q)                                                                    \
  do {                                                                           \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                  \
    __builtin_amdgcn_sched_barrier(0);                                           \
    t[q] = clock64();                                                            \
    __builtin_amdgcn_sched_barrier(0);                                           \
  } while (0)

__device__ bool diag16_stamped(double* TJ, double* WJ, double* sc, long long* t) {
  const int l = threadIdx.x & 63, r = l >> 3, c = l & 7;
  double a[36], iv[8];
  ST(0);
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) a[P8(i, j)] = TJ[i + j * 65];
  WJ[r + (8 + c) * 65] = 0.0;
  if (c > r) {
    WJ[r + c * 65] = 0.0;
    WJ[(8 + r) + (8 + c) * 65] = 0.0;
  }
  ST(1);
  bool bad = chol8_lane(a, iv);
  ST(2);
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) TJ[i + j * 65] = a[P8(i, j)];
  }
  ST(3);
  inv8_lane(a, iv);
  ST(4);
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) WJ[i + j * 65] = a[P8(i, j)];
  }
  __builtin_amdgcn_wave_barrier();
  ST(5);
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) s = fma(TJ[(8 + r) + k * 65], WJ[c + k * 65], s);
  __builtin_amdgcn_wave_barrier();
  TJ[(8 + r) + c * 65] = s;
  __builtin_amdgcn_wave_barrier();
  ST(6);
  double tt = TJ[(8 + r) + (8 + c) * 65];
#pragma unroll
  for (int k = 0; k < 8; k++) tt = fma(-TJ[(8 + r) + k * 65], TJ[(8 + c) + k * 65], tt);
  double y = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) y = fma(TJ[(8 + r) + k * 65], WJ[k + c * 65], y);
  __builtin_amdgcn_wave_barrier();
  if (c <= r) TJ[(8 + r) + (8 + c) * 65] = tt;
  sc[r * 8 + c] = y;
  __builtin_amdgcn_wave_barrier();
  ST(7);
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) a[P8(i, j)] = TJ[(8 + i) + (8 + j) * 65];
  ST(8);
  bad = chol8_lane(a, iv) || bad;
  ST(9);
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) TJ[(8 + i) + (8 + j) * 65] = a[P8(i, j)];
  }
  ST(10);
  inv8_lane(a, iv);
  ST(11);
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) WJ[(8 + i) + (8 + j) * 65] = a[P8(i, j)];
  }
  __builtin_amdgcn_wave_barrier();
  ST(12);
  double z = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) z = fma(WJ[(8 + r) + (8 + k) * 65], sc[k * 8 + c], z);
  WJ[(8 + r) + c * 65] = -z;
  ST(13);
  return bad;
}

__global__ __launch_bounds__(64) void u_d16(const double* A, double* out, long long* clk, int mode) {
  __shared__ double T[16 * 65], W[16 * 65], sc[64];
  long long t[14];
  long long t0 = 0, t1 = 0;
  for (int rep = 0; rep < 4; rep++) {
    for (int i = threadIdx.x; i < 16 * 65; i += 64) {
      T[i] = (i % 65) < 16 ? A[(i % 65) + 16 * (i / 65)] : 0.0;
      W[i] = 0.0;
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    t0 = clock64();
    bool bad = mode ? diag16_stamped(T, W, sc, t) : diag16_lane(T, W, sc);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    t1 = clock64();
    if (threadIdx.x == 0) out[0] += T[15 + 15 * 65] + W[15 + 15 * 65] + bad;
  }
  if (threadIdx.x == 0) {
    clk[0] = t1 - t0;
    if (mode)
      for (int q = 0; q < 14; q++) clk[1 + q] = t[q];
  }
}

int main() {
  double h[256];
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) h[i + 16 * j] = (i == j ? 40.0 : 0.0) + 1.0 / (1.0 + i + j);
  double *dA, *dO;
  long long* dc;
  hipMalloc(&dA, sizeof(h));
  hipMalloc(&dO, 64 * sizeof(double));
  hipMalloc(&dc, 32 * sizeof(long long));
  hipMemcpy(dA, h, sizeof(h), hipMemcpyHostToDevice);
  long long c[32];
  u_d16<<<1, 64>>>(dA, dO, dc, 0);
  hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
  printf("diag16_lane unstamped: %lld cycles\n", c[0]);
  u_d16<<<1, 64>>>(dA, dO, dc, 1);
  hipMemcpy(c, dc, sizeof(c), hipMemcpyDeviceToHost);
  const char* nm[] = {"load A11 + zero W", "chol8 A11", "store L11 (lane 0)", "inv8 L11", "store X11 (lane 0)",
                      "L21 = A21 X11'", "A22 -= L21 L21', Y", "load A22", "chol8 A22", "store L22 (lane 0)",
                      "inv8 L22", "store X22 (lane 0)", "X21 = -X22 Y"};
  printf("stamped total: %lld cycles\n", c[0]);
  for (int q = 0; q < 13; q++) printf("  %-22s %6lld\n", nm[q], c[2 + q] - c[1 + q]);
  return 0;
}
