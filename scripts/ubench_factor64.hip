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

template <int kAlg>   // 0: diag_factor_invert (16-column blocks, round 4), 1: diag_factor_invert8 (round 5)
__global__ __launch_bounds__(256) void u_factor(const double* A, double* out, int reps, int nbl, double* LX = nullptr) {
  __shared__ double T[64 * 65], W[64 * 65], bc[64];
  for (int rep = 0; rep < reps; rep++) {
    for (int i = threadIdx.x; i < 64 * 65; i += 256) {
      const int r = i % 65, cc = i / 65;
      T[i] = r < 64 ? ((r < nbl && cc < nbl) ? A[r + 64 * cc] : (r == cc ? 1.0 : 0.0)) : 0.0;
      W[i] = 0.0;
    }
    __syncthreads();
    const bool bad = kAlg == 0 ? diag_factor_invert(T, W, bc, nbl) : diag_factor_invert8(T, W, bc, nbl);
    __syncthreads();
    if (threadIdx.x == 0) out[0] += T[63 + 63 * 65] + W[63 + 63 * 65] + (bad ? 1 : 0);
  }
  if (LX)
    for (int i = threadIdx.x; i < 4096; i += 256) {
      LX[i] = T[(i & 63) + (i >> 6) * 65];
      LX[4096 + i] = W[(i & 63) + (i >> 6) * 65];
    }
}

static void run(int alg, int nbl, const std::vector<double>& A, double* dA, double* dO, double* dLX, std::vector<double>& LX) {
  hipMemset(dLX, 0, sizeof(double) * 8192);
  if (alg == 0) u_factor<0><<<1, 256>>>(dA, dO, 3, nbl, dLX);
  else u_factor<1><<<1, 256>>>(dA, dO, 3, nbl, dLX);
  hipDeviceSynchronize();
  LX.assign(8192, 0.0);
  hipMemcpy(LX.data(), dLX, sizeof(double) * 8192, hipMemcpyDeviceToHost);
  double e1 = 0, e2 = 0, up = 0;   // live part: L L^T = A, X L = I, X upper 0
  for (int i = 0; i < nbl; i++)
    for (int j = 0; j <= i; j++) {
      double s = 0, t = 0;
      for (int k = 0; k <= j; k++) s += LX[i + 64 * k] * LX[j + 64 * k];
      for (int k = j; k <= i; k++) t += LX[4096 + i + 64 * k] * LX[k + 64 * j];
      e1 = std::max(e1, std::fabs(s - A[i + 64 * j]));
      e2 = std::max(e2, std::fabs(t - (i == j ? 1.0 : 0.0)));
    }
  for (int i = 0; i < nbl; i++)
    for (int j = i + 1; j < nbl; j++) up = std::max(up, std::fabs(LX[4096 + i + 64 * j]));
  long long clk[32];
  hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_diag_clk), sizeof(clk));
  hipEvent_t t0, t1;
  hipEventCreate(&t0);
  hipEventCreate(&t1);
  hipEventRecord(t0);
  if (alg == 0) u_factor<0><<<1, 256>>>(dA, dO, 100, nbl);
  else u_factor<1><<<1, 256>>>(dA, dO, 100, nbl);
  hipEventRecord(t1);
  hipEventSynchronize(t1);
  float ms = 0;
  hipEventElapsedTime(&ms, t0, t1);
  printf("%s nbl %2d: max |LL'-A| %.3g  |XL-I| %.3g  |X upper| %.3g  cycles %lld  per factor+inverse (incl. LDS load) %.2f us\n",
         alg ? "8-blocks (r05)" : "16-blocks (r04)", nbl, e1, e2, up, clk[12] - clk[0], 1e3 * ms / 100);
}

int main() {
  std::vector<double> A(64 * 64);
  for (int i = 0; i < 64; i++)
    for (int j = 0; j < 64; j++) A[i + 64 * j] = (i == j ? 70.0 : 0.0) + 1.0 / (1.0 + i + j);
  double *dA, *dO, *dLX;
  hipMalloc(&dA, sizeof(double) * 4096);
  hipMalloc(&dO, sizeof(double));
  hipMalloc(&dLX, sizeof(double) * 8192);
  hipMemcpy(dA, A.data(), sizeof(double) * 4096, hipMemcpyHostToDevice);
  hipMemset(dO, 0, sizeof(double));
  for (int nbl : {64, 63, 48, 45, 24, 9, 3}) {
    std::vector<double> L0, L1;
    run(0, nbl, A, dA, dO, dLX, L0);
    run(1, nbl, A, dA, dO, dLX, L1);
    double dl = 0, dx = 0;
    for (int i = 0; i < nbl; i++)
      for (int j = 0; j <= i; j++) {
        dl = std::max(dl, std::fabs(L0[i + 64 * j] - L1[i + 64 * j]));
        dx = std::max(dx, std::fabs(L0[4096 + i + 64 * j] - L1[4096 + i + 64 * j]));
      }
    printf("   nbl %2d: max |L_r04 - L_r05| %.3g  |X_r04 - X_r05| %.3g\n", nbl, dl, dx);
  }
  return 0;
}
