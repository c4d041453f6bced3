// Pieces of diag_factor_invert8 timed alone (round 6): wave 1's batched
// trailing tiles (d8_trail3, 3 tiles), and a chol8 + inv8, each on one wave of
// a one-workgroup launch, the other waves idle at the end barrier or running
// the same piece (concurrency of 1 / 4 waves), to see what a phase costs on
// its own.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I include scripts/ubench_d8parts.hip -o graphslam_amd/build/ubench_d8parts
#include "../graphslam_amd/csrc/pgo_chol.hip"

#include <cstdio>
#include <vector>

using namespace pgo;

__device__ long long g_t[4][4];

template <int PIECE>
__global__ __launch_bounds__(256) void u_piece(double* out, int reps, int nwaves) {
  __shared__ double T[64 * 65];
  for (int i = threadIdx.x; i < 64 * 65; i += 256) T[i] = 1.0 / (1.0 + (i % 97));
  __syncthreads();
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  double acc = 0;
  if (wv < nwaves) {
    const long long t0 = clock64();
    for (int rep = 0; rep < reps; rep++) {
      if (PIECE == 0) {
        const int R[3] = {16, 32, 48}, C[3] = {16, 16, 16};
        d8_trail3(T, 0, R, C, 3, 64, 64, true);
      } else if (PIECE == 1) {
        double a[36], iv[8];
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
          for (int j = 0; j <= i; j++) a[P8(i, j)] = T[(8 * (rep & 7) + i) + 65 * (8 * (rep & 7) + j)] + (i == j ? 8.0 : 0.0);
        chol8_lane(a, iv);
        inv8_lane(a, iv);
        acc += a[35] + a[0];
      } else {   // 8 strided loads + 36 fma + 8 stores (the M phase)
        double sv[8];
        const int sb = 8 * (rep & 7);
#pragma unroll
        for (int q = 0; q < 8; q++) sv[q] = T[(sb + q) + 65 * l];
#pragma unroll
        for (int r = 0; r < 8; r++) {
          double o = 0.0;
#pragma unroll
          for (int q = 0; q <= r; q++) o = fma(0.5 + 0.01 * (r + q), sv[q], o);
          T[(sb + r) + 65 * l] = -o;
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const long long t1 = clock64();
    if (l == 0) g_t[wv][0] = t1 - t0;
  }
  __syncthreads();
  if (threadIdx.x == 0) out[0] += T[5] + acc;
}

int main() {
  double* dO;
  hipMalloc(&dO, sizeof(double));
  const char* names[3] = {"d8_trail3 (3 tiles)", "chol8+inv8 (lane-redundant)", "M phase (8 ld, 36 fma, 8 st)"};
  for (int piece = 0; piece < 3; piece++)
    for (int nw : {1, 4}) {
      const int reps = 64;
      if (piece == 0) u_piece<0><<<1, 256>>>(dO, reps, nw);
      else if (piece == 1) u_piece<1><<<1, 256>>>(dO, reps, nw);
      else u_piece<2><<<1, 256>>>(dO, reps, nw);
      hipDeviceSynchronize();
      long long t[4][4];
      hipMemcpyFromSymbol(t, HIP_SYMBOL(g_t), sizeof(t));
      printf("%-32s waves %d: %.0f cycles per call (wave 0)\n", names[piece], nw, (double)t[0][0] / reps);
    }
  return 0;
}
