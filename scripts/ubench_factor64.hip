// Microbenchmark of the diagonal tile's factor + inverse on the panel chain:
// one workgroup, an SPD tile, clock64 stamps (PGO_DIAG_CLOCKS).  Mode 0:
// diag_factor_invert (16-column blocks, wave 0's lane-redundant 16x16 blocks);
// mode 1: diag_factor_invert8 (round 6: 8-column steps, the chain on wave 0, the
// trailing updates and the inverse on waves 1-3 beside it).  Checks X A X^T = I
// for live sizes 64 and 37 and the two modes against each other.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_factor64.hip -o graphslam_amd/build/ubench_factor64
#define PGO_DIAG_CLOCKS 1
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>
#include <vector>
#include <cmath>
#include <algorithm>

using namespace pgo;

__global__ __launch_bounds__(256) void u_factor(const double* A, double* out, int reps, int mode, int nbl,
                                                double* LX = nullptr) {
  __shared__ __attribute__((aligned(16))) double T[64 * 65], W[64 * 65], bc[64];
  for (int rep = 0; rep < reps; rep++) {
    for (int i = threadIdx.x; i < 64 * 65; i += 256) {
      const int r = i % 65, cc = i / 65;
      T[i] = r < 64 ? ((r < nbl && cc < nbl) ? A[r + 64 * cc] : (r == cc ? 1.0 : 0.0)) : 0.0;
      W[i] = 0.0;
    }
    __syncthreads();
    int bad;
    if (mode == 0) bad = diag_factor_invert<false>(T, W, bc, nbl) ? 1 : 0;
    else if (mode == 2) bad = diag_factor_invert<true>(T, W, bc, nbl) ? 1 : 0;
    else bad = diag_factor_invert8(T, W, bc, nbl);
    __syncthreads();
    if (threadIdx.x == 0) out[0] += W[63 + 63 * 65] + bad;
    if (threadIdx.x == 0 && bad) out[1] += bad;
  }
  if (LX)
    for (int i = threadIdx.x; i < 4096; i += 256) LX[i] = W[(i & 63) + (i >> 6) * 65];
}

static double check(const std::vector<double>& A, const double* X, int n) {
  std::vector<double> XA(4096, 0.0);
  for (int i = 0; i < n; i++)
    for (int j = 0; j < n; j++) {
      double s = 0;
      for (int k = 0; k <= i; k++) s += X[i + 64 * k] * A[k + 64 * j];
      XA[i + 64 * j] = s;
    }
  double e1 = 0;
  for (int i = 0; i < n; i++)
    for (int j = 0; j <= i; j++) {
      double s = 0;
      for (int k = 0; k <= j; k++) s += XA[i + 64 * k] * X[j + 64 * k];
      e1 = std::max(e1, std::fabs(s - (i == j ? 1.0 : 0.0)));
    }
  double up = 0;
  for (int i = 0; i < 64; i++)
    for (int j = i + 1; j < 64; j++) up = std::max(up, std::fabs(X[i + 64 * j]));
  printf("  max |X A X^T - I| %.3g  max |X upper| %.3g\n", e1, up);
  return e1;
}

int main() {
  std::vector<double> A(64 * 64);
  unsigned s = 12345;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return (s >> 8) * (1.0 / 16777216.0) - 0.5; };
  std::vector<double> B(64 * 64);
  for (auto& v : B) v = rnd();
  for (int i = 0; i < 64; i++)   // A = B B^T + 2 I + the old ubench's Hilbert-like part
    for (int j = 0; j < 64; j++) {
      double t = 0;
      for (int k = 0; k < 64; k++) t += B[i + 64 * k] * B[j + 64 * k];
      A[i + 64 * j] = t + (i == j ? 2.0 : 0.0) + 1.0 / (1.0 + i + j);
    }
  double *dA, *dO, *dLX;
  hipMalloc(&dA, sizeof(double) * 4096);
  hipMalloc(&dO, 2 * sizeof(double));
  hipMalloc(&dLX, sizeof(double) * 4096 * 3);
  hipMemcpy(dA, A.data(), sizeof(double) * 4096, hipMemcpyHostToDevice);
  int fail = 0;
  for (int nbl : {64, 37, 8, 1}) {
    std::vector<double> X0(4096), X1(4096), X2(4096);
    for (int mode = 0; mode < 3; mode++) {
      hipMemset(dO, 0, 2 * sizeof(double));
      u_factor<<<1, 256>>>(dA, dO, 1, mode, nbl, dLX + 4096 * mode);
      if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 1; }
      double o[2];
      hipMemcpy(o, dO, 2 * sizeof(double), hipMemcpyDeviceToHost);
      std::vector<double>& X = mode == 2 ? X2 : mode ? X1 : X0;
      hipMemcpy(X.data(), dLX + 4096 * mode, sizeof(double) * 4096, hipMemcpyDeviceToHost);
      printf("nbl %d mode %d bad/err %.0f\n", nbl, mode, o[1]);
      if (check(A, X.data(), nbl) > 1e-9 || o[1] != 0) fail = 1;
    }
    double d = 0, d2 = 0, mx = 0;   // (the live part: the callers read nothing past nbl)
    for (int i = 0; i < 4096; i++)
      if ((i & 63) < nbl && (i >> 6) < nbl) {
        d = std::max(d, std::fabs(X0[i] - X1[i]));
        d2 = std::max(d2, std::fabs(X0[i] - X2[i]));
        mx = std::max(mx, std::fabs(X0[i]));
      }
    printf("  nbl %d: max |X_mode1 - X_mode0| %.3g, max |X_mode2 - X_mode0| %.3g (max |X| %.3g)\n", nbl, d, d2, mx);
    if (d > 1e-10 * mx || d2 > 1e-10 * mx) fail = 1;
  }
  for (int dbg : {0, 8, 1, 1 | 8, 2 | 4, 2 | 4 | 1}) {   // diagnostics: which waves' work the chain waits on
    hipMemcpyToSymbol(HIP_SYMBOL(g_d8_dbg), &dbg, sizeof(int));
    u_factor<<<1, 256>>>(dA, dO, 3, 1, 64);
    hipDeviceSynchronize();
    long long clk[32], d8[4][8][8];
    hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_diag_clk), sizeof(clk));
    hipMemcpyFromSymbol(d8, HIP_SYMBOL(g_d8_clk), sizeof(d8));
    printf("dbg %d (1 = X waves idle, 2 = no waits, 4 = trailing wave idle, 8 = trailing on wave 2): total %lld, wave 0 done %lld; wave 0 per step:", dbg,
           clk[12] - clk[0], clk[1] - clk[0]);
    for (int k = 0; k < 7; k++) printf(" [%lld %lld %lld %lld %lld]", d8[0][k][1] - d8[0][k][0], d8[0][k][2] - d8[0][k][1],
                                       d8[0][k][3] - d8[0][k][2], d8[0][k][4] - d8[0][k][3], d8[0][k][5] - d8[0][k][4]);
    printf("\n");
  }
  { int z = 0; hipMemcpyToSymbol(HIP_SYMBOL(g_d8_dbg), &z, sizeof(int)); }
  for (int mode = 0; mode < 3; mode++) {
    u_factor<<<1, 256>>>(dA, dO, 3, mode, 64);
    hipDeviceSynchronize();
    long long clk[32];
    hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_diag_clk), sizeof(clk));
    printf("mode %d: total %lld cycles", mode, clk[12] - clk[0]);
    if (mode == 1) {
      printf(" (wave 0 chain done at %lld)\n", clk[1] - clk[0]);
      long long d8[4][8][8];
      hipMemcpyFromSymbol(d8, HIP_SYMBOL(g_d8_clk), sizeof(d8));
      const long long t0 = clk[0];
      const char* names[4] = {"wave0 chain: a+chol8 | chol8 done | T1A seen | d done | T1B seen | e+signal",
                              "wave1 trail: start | U1 done | U2 col done | rest done",
                              "wave2 inv:   start | inverse | XDONE seen | U done | M done",
                              "wave3 inv:   start | inverse | XDONE seen | U done | M done"};
      const int nq[4] = {6, 4, 5, 5};
      for (int w = 0; w < 4; w++) {
        printf("%s\n", names[w]);
        for (int k = 0; k < 8; k++) {
          printf("  k%d:", k);
          for (int q = 0; q < nq[w]; q++) printf(" %6lld", d8[w][k][q] ? d8[w][k][q] - t0 : -1);
          printf("\n");
        }
      }
    } else {
      printf("\n");
      long long prev = clk[0];
      for (int J = 0; J < 4; J++) {   // A: wave 0's diagonal block (+ the update before it), B: the panel / inverse-row products
        const long long b = J < 3 ? clk[2 + 3 * J] : clk[12];
        printf("  J%d A %lld  B %lld\n", J, clk[1 + 3 * J] - prev, b - clk[1 + 3 * J]);
        prev = b;
      }
      if (mode == 2)
        printf("  diag16_fs (J3, fenced): chol8 %lld, fwd+store %lld, A22/Y+load %lld, chol8 %lld, fwd+store %lld\n",
               clk[21] - clk[20], clk[22] - clk[21], clk[23] - clk[22], clk[24] - clk[23], clk[25] - clk[24]);
    }
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    u_factor<<<1, 256>>>(dA, dO, 100, mode, 64);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("mode %d: per factor+inverse (incl. LDS load): %.2f us\n", mode, 1e3 * ms / 100);
  }
  printf(fail ? "FAIL\n" : "PASS\n");
  return fail;
}
