// Probe of v_mfma_f64_4x4x4f64 (4 blocks of 4x4x4 per wave): operand / result
// lane layouts, and whether its arithmetic matches v_mfma_f64_16x16x4f64 bit
// for bit on the same dot products (the Schur-update kernels' choice).
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_mfma4.hip -o graphslam_amd/build/ubench_mfma4
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

__global__ void probe(double* out, int t) {
  const int l = threadIdx.x;
  const double a = 1.0 + l;                 // distinct A per lane
  const double b = (l == t) ? 1.0 : 0.0;    // one-hot B
  double d = 0.0;
  d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, d, 0, 0, 0);
  out[l] = d;
}

typedef double d4 __attribute__((ext_vector_type(4)));
// Same 4-term dot products on both instructions: D = acc + A(16x4) B(4x16),
// 16x16x4 (lane l: A[l & 15][l >> 4], B[l >> 4][l & 15], D reg r -> row
// (l >> 4) + 4 r, col l & 15) and 4x4x4 rows 0..3 (lane 16 k + 4 g + i: A[i][k];
// lane 16 k + 4 g + j: B[k][4 g + j]; D lane 16 i + 4 g + j -> (i, 4 g + j)).
__global__ void compare(const double* A, const double* B, const double* C0, double* o4, double* o16) {
  const int l = threadIdx.x;
  d4 acc;
  for (int r = 0; r < 4; r++) acc[r] = C0[((l >> 4) + 4 * r) * 16 + (l & 15)];
  acc = __builtin_amdgcn_mfma_f64_16x16x4f64(A[(l & 15) * 4 + (l >> 4)], B[(l >> 4) * 16 + (l & 15)], acc, 0, 0, 0);
  for (int r = 0; r < 4; r++) o16[((l >> 4) + 4 * r) * 16 + (l & 15)] = acc[r];
  const int k = l >> 4, g = (l >> 2) & 3, ij = l & 3;
  double d = C0[(l >> 4) * 16 + (l & 15)];
  d = __builtin_amdgcn_mfma_f64_4x4x4f64(A[ij * 4 + k], B[k * 16 + 4 * g + ij], d, 0, 0, 0);
  o4[(l >> 4) * 16 + (l & 15)] = d;
}

int main() {
  double* o;
  hipMalloc(&o, 64 * 8);
  double h[64];
  for (int t = 0; t < 64; t += 21) {
    probe<<<1, 64>>>(o, t);
    hipMemcpy(h, o, 64 * 8, hipMemcpyDeviceToHost);
    printf("B one-hot lane %2d:", t);
    for (int l = 0; l < 64; l++)
      if (h[l] != 0.0) printf(" D[%d]=A[%d]", l, (int)h[l] - 1);
    printf("\n");
  }
  {
    double hA[64], hB[64], hC[256], r4[64], r16[256];
    srand(7);
    int same = 0, diff = 0;
    double *dA, *dB, *dC, *d4o, *d16;
    hipMalloc(&dA, 512); hipMalloc(&dB, 512); hipMalloc(&dC, 2048); hipMalloc(&d4o, 512); hipMalloc(&d16, 2048);
    for (int trial = 0; trial < 200; trial++) {
      for (int i = 0; i < 64; i++) {
        hA[i] = (rand() / (double)RAND_MAX - 0.5) * pow(10.0, rand() % 7 - 3);
        hB[i] = (rand() / (double)RAND_MAX - 0.5) * pow(10.0, rand() % 7 - 3);
      }
      for (int i = 0; i < 256; i++) hC[i] = (rand() / (double)RAND_MAX - 0.5) * pow(10.0, rand() % 7 - 3);
      hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice);
      hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
      hipMemcpy(dC, hC, 2048, hipMemcpyHostToDevice);
      compare<<<1, 64>>>(dA, dB, dC, d4o, d16);
      hipMemcpy(r4, d4o, 512, hipMemcpyDeviceToHost);
      hipMemcpy(r16, d16, 2048, hipMemcpyDeviceToHost);
      for (int i = 0; i < 64; i++) (r4[i] == r16[i] ? same : diff)++;
    }
    printf("4x4x4 vs 16x16x4 on the same dot products: %d equal, %d different\n", same, diff);
  }
  return 0;
}
