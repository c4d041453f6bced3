// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// widths and patterns of this repo's kernels (MI355X_MICROARCH.md §HBM: "other
// access widths are uncalibrated: calibrate on a known byte count in your own
// access pattern").  Each kernel moves a known number of bytes of a 1 GiB
// buffer (4x the Infinity Cache, so nothing is absorbed on-die):
//   rd16     16 B per lane, coalesced              (the guide's calibrated case)
//   rd8      8 B per lane, coalesced                (double loads: most kernels)
//   rd32     32 B per lane (double4), coalesced     (poses, z)
//   gath8    8 B per lane, random 8-B gathers      (1/16 of the buffer's lines touched once: 8 B used per line)
//   gath32   32 B per lane, random 32-B gathers
//   wr8      8 B per lane, coalesced stores
//   wr32     32 B per lane, coalesced stores
//   scat32   32 B per lane, random 32-B scattered stores
// Run under rocprofv3 --pmc FETCH_SIZE (one pass) and --pmc WRITE_SIZE (another);
// scripts/pmc_calib.py divides the counters by the bytes each kernel moved.
//   hipcc -O3 --offload-arch=gfx950 scripts/ubench_pmc_calib.hip -o graphslam_amd/build/ubench_pmc_calib
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t kBytes = 1ull << 30;

__global__ void rd16(const double2* __restrict__ a, double* out, size_t n) {
  double s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i].x + a[i].y;
  if (s == 12345.0) out[0] = s;
}
__global__ void rd8(const double* __restrict__ a, double* out, size_t n) {
  double s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  if (s == 12345.0) out[0] = s;
}
__global__ void rd32(const double4* __restrict__ a, double* out, size_t n) {
  double s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const double4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.0) out[0] = s;
}
__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  return x;
}
// random distinct lines: line L = (i * odd) mod nlines, one access per line
__global__ void gath8(const double* __restrict__ a, double* out, size_t nlines, size_t cnt) {
  double s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < cnt; i += (size_t)gridDim.x * 256) {
    const size_t line = (i * 0x9E3779B97F4A7C15ull) & (nlines - 1);
    s += a[line * 16 + (mix(i) & 15)];
  }
  if (s == 12345.0) out[0] = s;
}
__global__ void gath32(const double4* __restrict__ a, double* out, size_t nlines, size_t cnt) {
  double s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < cnt; i += (size_t)gridDim.x * 256) {
    const size_t line = (i * 0x9E3779B97F4A7C15ull) & (nlines - 1);
    const double4 v = a[line * 4 + (mix(i) & 3)];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.0) out[0] = s;
}
__global__ void wr8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = (double)i;
}
__global__ void wr32(double4* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    a[i] = make_double4((double)i, 1.0, 2.0, 3.0);
}
__global__ void scat32(double4* __restrict__ a, size_t nlines, size_t cnt) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < cnt; i += (size_t)gridDim.x * 256) {
    const size_t line = (i * 0x9E3779B97F4A7C15ull) & (nlines - 1);
    a[line * 4 + (mix(i) & 3)] = make_double4((double)i, 1.0, 2.0, 3.0);
  }
}

int main() {
  char* buf;
  double* out;
  if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, kBytes);
  (void)hipDeviceSynchronize();
  const dim3 g(4096), b(256);
  const size_t nlines = kBytes / 128;        // 128-byte lines
  const size_t cnt = nlines / 16;            // one access in 16 lines' worth: every touched line distinct
  // each kernel twice (the second launch is the one to read)
  for (int r = 0; r < 2; r++) {
    rd16<<<g, b>>>((const double2*)buf, out, kBytes / 16);
    rd8<<<g, b>>>((const double*)buf, out, kBytes / 8);
    rd32<<<g, b>>>((const double4*)buf, out, kBytes / 32);
    gath8<<<g, b>>>((const double*)buf, out, nlines, cnt);
    gath32<<<g, b>>>((const double4*)buf, out, nlines, cnt);
    wr8<<<g, b>>>((double*)buf, kBytes / 8);
    wr32<<<g, b>>>((double4*)buf, kBytes / 32);
    scat32<<<g, b>>>((double4*)buf, nlines, cnt);
  }
  (void)hipDeviceSynchronize();
  printf("bytes moved: rd16/rd8/rd32/wr8/wr32 %zu each; gath8 %zu (useful), lines %zu; gath32/scat32 %zu (useful)\n",
         kBytes, cnt * 8, cnt, cnt * 32);
  return 0;
}
