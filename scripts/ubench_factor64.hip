// Microbenchmark of diag_factor_invert (the 64x64 factor + inverse on the
// panel chain): one workgroup, a random SPD tile, clock64 stamps at its phases
// (PGO_DIAG_CLOCKS): per 16-column block J the wave-0 diagonal block (A, beside
// the previous block's trailing updates C) and the panel / inverse-row products (B).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_factor64.hip -o graphslam_amd/build/ubench_factor64
#define PGO_DIAG_CLOCKS 1
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>
#include <vector>
#include <cmath>
#include <algorithm>

using namespace pgo;

__global__ __launch_bounds__(256) void u_factor(const double* A, double* out, int reps, double* LX = nullptr) {
  __shared__ double T[64 * 65], W[64 * 65], bc[64];
  for (int rep = 0; rep < reps; rep++) {
    for (int i = threadIdx.x; i < 64 * 65; i += 256) {
      const int r = i % 65, cc = i / 65;
      T[i] = r < 64 ? A[r + 64 * cc] : 0.0;
      W[i] = 0.0;
    }
    __syncthreads();
    const bool bad = diag_factor_invert(T, W, bc);
    __syncthreads();
    if (threadIdx.x == 0) out[0] += T[63 + 63 * 65] + W[63 + 63 * 65] + (bad ? 1 : 0);
  }
  if (LX)
    for (int i = threadIdx.x; i < 4096; i += 256) {
      LX[i] = T[(i & 63) + (i >> 6) * 65];
      LX[4096 + i] = W[(i & 63) + (i >> 6) * 65];
    }
}

int main() {
  std::vector<double> A(64 * 64);
  for (int i = 0; i < 64; i++)
    for (int j = 0; j < 64; j++) A[i + 64 * j] = (i == j ? 70.0 : 0.0) + 1.0 / (1.0 + i + j);
  double *dA, *dO;
  hipMalloc(&dA, sizeof(double) * 4096);
  hipMalloc(&dO, sizeof(double));
  hipMemcpy(dA, A.data(), sizeof(double) * 4096, hipMemcpyHostToDevice);
  hipMemset(dO, 0, sizeof(double));
  double* dLX;
  hipMalloc(&dLX, sizeof(double) * 8192);
  u_factor<<<1, 256>>>(dA, dO, 3, dLX);
  hipDeviceSynchronize();
  {  // check: X A X^T = I with X = L^-1 (the diagonal tile's L itself is not kept since round 5)
    std::vector<double> LX(8192);
    hipMemcpy(LX.data(), dLX, sizeof(double) * 8192, hipMemcpyDeviceToHost);
    const double* X = LX.data() + 4096;
    std::vector<double> XA(4096, 0.0);
    for (int i = 0; i < 64; i++)
      for (int j = 0; j < 64; j++) {
        double s = 0;
        for (int k = 0; k <= i; k++) s += X[i + 64 * k] * A[k + 64 * j];
        XA[i + 64 * j] = s;
      }
    double e1 = 0;
    for (int i = 0; i < 64; i++)
      for (int j = 0; j <= i; j++) {
        double s = 0;
        for (int k = 0; k <= j; k++) s += XA[i + 64 * k] * X[j + 64 * k];
        e1 = std::max(e1, std::fabs(s - (i == j ? 1.0 : 0.0)));
      }
    double up = 0;
    for (int i = 0; i < 64; i++)
      for (int j = i + 1; j < 64; j++) up = std::max(up, std::fabs(X[i + 64 * j]));
    printf("max |X A X^T - I| %.3g  max |X upper| %.3g\n", e1, up);
  }
  long long clk[32];
  hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_diag_clk), sizeof(clk));
  printf("total %lld cycles\n", clk[12] - clk[0]);
  long long prev = clk[0];
  for (int J = 0; J < 4; J++) {   // A: wave 0's diagonal block (with phase C of J-1 beside it), B: panel products
    const long long b = J < 3 ? clk[2 + 3 * J] : clk[12];
    printf("J%d A(+C) %lld  B %lld\n", J, clk[1 + 3 * J] - prev, b - clk[1 + 3 * J]);
    prev = b;
  }
  printf("diag16_lane (last J), cycles: chol8 %lld, inv8 %lld, L21/A22/Y %lld, chol8 %lld, inv8 %lld, X21 %lld\n",
         clk[14] - clk[13], clk[15] - clk[14], clk[16] - clk[15], clk[17] - clk[16], clk[18] - clk[17], clk[19] - clk[18]);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  u_factor<<<1, 256>>>(dA, dO, 100);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  printf("per factor+inverse (incl. LDS load): %.2f us\n", 1e3 * ms / 100);
  return 0;
}
