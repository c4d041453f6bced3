// Microbenchmark of diag_factor_invert (the 64x64 factor + inverse on the
// panel chain): one workgroup, a random SPD tile, clock64 stamps at its phases
// (PGO_DIAG_CLOCKS): per 16-column block J the wave-0 pivot chain (A), the
// panel / inverse-row products (B) and the trailing updates (C).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_factor64.hip -o graphslam_amd/build/ubench_factor64
#define PGO_DIAG_CLOCKS 1
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>
#include <vector>

using namespace pgo;

__global__ __launch_bounds__(256) void u_factor(const double* A, double* out, int reps) {
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
  u_factor<<<1, 256>>>(dA, dO, 3);
  hipDeviceSynchronize();
  long long clk[32];
  hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_diag_clk), sizeof(clk));
  printf("total %lld cycles\n", clk[12] - clk[0]);
  long long prev = clk[0];
  for (int J = 0; J < 4; J++) {
    const int a = 1 + 3 * J, b = 2 + 3 * J, cq = 3 + 3 * J;
    if (J < 3) {
      printf("J%d chain %lld  B %lld  C %lld\n", J, clk[a] - prev, clk[b] - clk[a], clk[cq] - clk[b]);
      prev = clk[cq];
    } else {
      printf("J%d chain %lld  B+end %lld\n", J, clk[a] - prev, clk[12] - clk[a]);
    }
  }
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
