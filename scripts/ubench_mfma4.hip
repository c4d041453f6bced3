// Probe of the v_mfma_f64_4x4x4_4b_f64 operand / result lane layout (one-hot
// operands; 64 waves with A one-hot, 64 with B one-hot; then the same A probes
// with the block broadcast cbsz = 2, abid = 1).
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_mfma4.hip -o graphslam_amd/build/ubench_mfma4
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void probe(double* out) {
  const int p = blockIdx.x, l = threadIdx.x;
  double a, b, d;
  if (p < 64) {
    a = l == p ? 1.0 : 0.0;
    b = 1.0;
    d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  } else if (p < 128) {
    a = 1.0;
    b = l == p - 64 ? 1.0 : 0.0;
    d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
  } else {
    a = l == p - 128 ? 1.0 : 0.0;
    b = 1.0;
    d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 2, 1, 0);
  }
  out[p * 64 + l] = d;
}

int main() {
  double* o;
  hipMalloc(&o, 192 * 64 * 8);
  probe<<<192, 64>>>(o);
  std::vector<double> h(192 * 64);
  hipMemcpy(h.data(), o, h.size() * 8, hipMemcpyDeviceToHost);
  const char* name[3] = {"A", "B", "A(cbsz2,abid1)"};
  for (int set = 0; set < 3; set++)
    for (int L = 0; L < 64; L++) {
      printf("%s lane %2d ->", name[set], L);
      for (int q = 0; q < 64; q++)
        if (h[(set * 64 + L) * 64 + q] != 0.0) printf(" %d", q);
      printf("\n");
    }
  return 0;
}
