// HIP kernels of the Gauss-Newton / Levenberg-Marquardt hot path (gfx950).
//
// Replaces, inside gtsam::LevenbergMarquardtOptimizer::optimize()
// (/root/reference/src/graph/src/graph.cpp:119):
//   NonlinearFactorGraph::linearize   -> k_linearize  (residual + Jacobian sweep,
//                                        block-CSR H and b built in one pass)
//   GaussianFactorGraph::optimize     -> k_pcg_*      (block-Jacobi PCG on H + lambda I)
//   GaussianFactorGraph::error(delta) -> k_model_decrease
//   Values::retract                   -> k_retract
//   NonlinearFactorGraph::error       -> k_error
//
// Every reduction is a fixed-order tree (xor butterflies inside a wave, LDS
// across waves, fixed-order partial sums across blocks): results are bitwise
// reproducible run to run; no floating-point atomics anywhere.
#include <hip/hip_ext.h>
#include <math.h>

#include "pgo_device.h"

namespace pgo {

// ------------------------------------------------------------ Pose2 helpers
// GTSAM Rot2::normalize: rescale only when |c^2+s^2-1| > 1e-10.
__device__ __forceinline__ void rot_normalize(double& c, double& s) {
  const double scale = c * c + s * s;
  if (fabs(scale - 1.0) > 1e-10) {
    const double f = 1.0 / sqrt(scale);   // pow(scale, -0.5) up to rounding; taken only off the unit circle
    c *= f;
    s *= f;
  }
}

// ------------------------------------------------------------ reductions
template <int G>
__device__ __forceinline__ double sg_sum(double v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, G);
  return v;  // bit-identical in every lane of the sub-group
}

__device__ __forceinline__ double block_sum(double v, double* lds) {
  v = sg_sum<64>(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) lds[w] = v;
  __syncthreads();
  double s = 0.0;
#pragma unroll
  for (int i = 0; i < kThreads / 64; i++) s += lds[i];
  __syncthreads();
  return s;
}

// Sum of nb block partials; every block obtains the bit-identical value.
__device__ __forceinline__ double sum_partials(const double* __restrict__ part, int nb, double* lds) {
  double v = 0.0;
  for (int i = threadIdx.x; i < nb; i += kThreads) v += part[i];
  return block_sum(v, lds);
}

// ------------------------------------------------------------ linearize
// One sub-group of G lanes per vertex row; one lane per slot.  Each slot
// recomputes its factor's residual and J1 (both endpoints need them) and writes
// its 3x3 block coalesced in row order; the row's diagonal block, gradient and
// (side-0 slots only) 0.5 e'Omega e are summed across the sub-group.
template <int G>
__global__ __launch_bounds__(kThreads) void k_linearize(DevGraph d) {
  const int lane = threadIdx.x & (G - 1);
  const int nsg = gridDim.x * (kThreads / G);
  for (int row = (blockIdx.x * kThreads + threadIdx.x) / G; row < d.n; row += nsg) {
    double a00 = 0, a01 = 0, a02 = 0, a11 = 0, a12 = 0, a22 = 0, g0 = 0, g1 = 0, g2 = 0;
    const int beg = d.row_ptr[row], end = d.row_ptr[row + 1];
#pragma unroll 1
    for (int k = beg + lane; k < end; k += G) {
      const int se = d.slot_edge[k];
      const bool put = d.write_all || (se & 2);   // owner blocks only for the Cholesky assembly
      const int2 ij = d.eij[se >> 2];
      const double4 p1 = d.pose[ij.x], p2 = d.pose[ij.y], z = d.ez[se >> 2];
      const double2 oA = d.eom[3 * (se >> 2)], oB = d.eom[3 * (se >> 2) + 1], oC = d.eom[3 * (se >> 2) + 2];
      const double o00 = oA.x, o01 = oA.y, o02 = oB.x, o11 = oB.y, o12 = oC.x, o22 = oC.y;
      // hx = between(p1, p2)                                 [GTSAM Pose2::between]
      double hc = p1.z * p2.z + p1.w * p2.w, hs = -p1.w * p2.z + p1.z * p2.w;
      rot_normalize(hc, hs);
      const double dx = p2.x - p1.x, dy = p2.y - p1.y;
      const double hx = p1.z * dx + p1.w * dy, hy = -p1.w * dx + p1.z * dy;
      // e = Local(z, hx) = (between(z, hx).t, theta)        [GTSAM BetweenFactor]
      double ec = z.z * hc + z.w * hs, es = -z.w * hc + z.z * hs;
      rot_normalize(ec, es);
      const double tx = hx - z.x, ty = hy - z.y;
      const double e0 = z.z * tx + z.w * ty, e1 = -z.w * tx + z.z * ty, e2 = atan2(es, ec);
      // J1 = [[-hc,-hs,dt1],[hs,-hc,dt2],[0,0,-1]], J2 = I
      const double dt1 = -p2.w * dx + p2.z * dy, dt2 = -p2.z * dx - p2.w * dy;
      // M = Omega J1
      const double m00 = -hc * o00 + hs * o01, m01 = -hs * o00 - hc * o01, m02 = dt1 * o00 + dt2 * o01 - o02;
      const double m10 = -hc * o01 + hs * o11, m11 = -hs * o01 - hc * o11, m12 = dt1 * o01 + dt2 * o11 - o12;
      const double m20 = -hc * o02 + hs * o12, m21 = -hs * o02 - hc * o12, m22 = dt1 * o02 + dt2 * o12 - o22;
      const double w0 = o00 * e0 + o01 * e1 + o02 * e2;
      const double w1 = o01 * e0 + o11 * e1 + o12 * e2;
      const double w2 = o02 * e0 + o12 * e1 + o22 * e2;
      double* v = d.V + k;
      const size_t S = d.nslots;
      if ((se & 1) == 0) {  // row ei: H_ij = J1'Omega = M', H_ii += J1'M, g_i += J1'w
        if (put) {
          v[0] = m00; v[S] = m10; v[2 * S] = m20;
          v[3 * S] = m01; v[4 * S] = m11; v[5 * S] = m21;
          v[6 * S] = m02; v[7 * S] = m12; v[8 * S] = m22;
        }
        a00 += -hc * m00 + hs * m10;
        a01 += -hc * m01 + hs * m11;
        a02 += -hc * m02 + hs * m12;
        a11 += -hs * m01 - hc * m11;
        a12 += -hs * m02 - hc * m12;
        a22 += dt1 * m02 + dt2 * m12 - m22;
        g0 += -hc * w0 + hs * w1;
        g1 += -hs * w0 - hc * w1;
        g2 += dt1 * w0 + dt2 * w1 - w2;
      } else {              // row ej: H_ji = Omega J1 = M, H_jj += Omega, g_j += w
        if (put) {
          v[0] = m00; v[S] = m01; v[2 * S] = m02;
          v[3 * S] = m10; v[4 * S] = m11; v[5 * S] = m12;
          v[6 * S] = m20; v[7 * S] = m21; v[8 * S] = m22;
        }
        a00 += o00; a01 += o01; a02 += o02; a11 += o11; a12 += o12; a22 += o22;
        g0 += w0; g1 += w1; g2 += w2;
      }
    }
    if (lane == 0) {  // PriorFactor<Pose2>: e = -Local(x, prior), H = I   [GTSAM PriorFactor]
      for (int q = d.prior_ptr[row]; q < d.prior_ptr[row + 1]; q++) {
        const double4 x = d.pose[row], pz = d.pz[q];
        double c = x.z * pz.z + x.w * pz.w, s = -x.w * pz.z + x.z * pz.w;
        rot_normalize(c, s);
        const double dx = pz.x - x.x, dy = pz.y - x.y;
        const double e0 = -(x.z * dx + x.w * dy), e1 = -(-x.w * dx + x.z * dy), e2 = -atan2(s, c);
        const double2 oA = d.pom[3 * q], oB = d.pom[3 * q + 1], oC = d.pom[3 * q + 2];
        const double o00 = oA.x, o01 = oA.y, o02 = oB.x, o11 = oB.y, o12 = oC.x, o22 = oC.y;
        const double w0 = o00 * e0 + o01 * e1 + o02 * e2;
        const double w1 = o01 * e0 + o11 * e1 + o12 * e2;
        const double w2 = o02 * e0 + o12 * e1 + o22 * e2;
        a00 += o00; a01 += o01; a02 += o02; a11 += o11; a12 += o12; a22 += o22;
        g0 += w0; g1 += w1; g2 += w2;
      }
    }
    a00 = sg_sum<G>(a00); a01 = sg_sum<G>(a01); a02 = sg_sum<G>(a02);
    a11 = sg_sum<G>(a11); a12 = sg_sum<G>(a12); a22 = sg_sum<G>(a22);
    g0 = sg_sum<G>(g0); g1 = sg_sum<G>(g1); g2 = sg_sum<G>(g2);
    if (lane == 0) {
      double* D = d.D + 6 * (size_t)row;
      D[0] = a00; D[1] = a01; D[2] = a02; D[3] = a11; D[4] = a12; D[5] = a22;
      double* g = d.g + 3 * (size_t)row;
      g[0] = g0; g[1] = g1; g[2] = g2;
    }
  }
}

// Cholesky-mode linearisation (write_all = 0 with a plan), one thread per
// between factor.  Factors are sorted by (ei, ej); block b owns the whole rows
// [brow[b], brow[b+1]) (at most kThreads rows, their side-0 factors in chunks
// of kThreads), so a wave streams eij / z / Omega once each, coalesced, with
// every lane busy and no erow -> factor load chain.  Each factor's owner block
// goes to V[9 e + q] in factor order (the assembly's source index: a factor's
// block is one 72-byte record, so the assembly's gathers read one or two lines
// per block instead of nine), staged through LDS so a chunk's records leave as
// contiguous 16-byte stores; its Omega e to W[s1pos[e]] (row ej's side-1 list)
// for k_linearize_side1; the factor's side-0 terms (J1' Omega J1, J1' Omega e)
// go through LDS to one thread per row, which sums them in factor order and
// adds Dc[i] (sum of Omega over the row's side-1 factors) and the row's
// priors.  No error partials: the error is k_error's.
__global__ __launch_bounds__(kThreads, 4) void k_linearize_own(DevGraph d) {
  __shared__ double sm[9][kThreads];
  const int t = threadIdx.x;
  const int r0 = d.brow[blockIdx.x], r1 = d.brow[blockIdx.x + 1];
  const int e0 = d.erow[r0], e1 = d.erow[r1];
  const int row = r0 + t;
  const bool rowt = row < r1;
  const int rb = rowt ? d.erow[row] : 0, re = rowt ? d.erow[row + 1] : 0;
  double a00 = 0, a01 = 0, a02 = 0, a11 = 0, a12 = 0, a22 = 0, g0 = 0, g1 = 0, g2 = 0;
  for (int c0 = e0; c0 < e1; c0 += kThreads) {
    const int e = c0 + t;
    double s0 = 0, s1 = 0, s2 = 0, s3 = 0, s4 = 0, s5 = 0, s6 = 0, s7 = 0, s8 = 0;
    if (e < e1) {
      const int2 ij = d.eij[e];
      const double4 p1 = d.pose[ij.x], p2 = d.pose[ij.y], z = d.ez[e];
      const double2 oA = d.eom[3 * e], oB = d.eom[3 * e + 1], oC = d.eom[3 * e + 2];
      const double o00 = oA.x, o01 = oA.y, o02 = oB.x, o11 = oB.y, o12 = oC.x, o22 = oC.y;
      double hc = p1.z * p2.z + p1.w * p2.w, hs = -p1.w * p2.z + p1.z * p2.w;
      rot_normalize(hc, hs);
      const double dx = p2.x - p1.x, dy = p2.y - p1.y;
      const double hx = p1.z * dx + p1.w * dy, hy = -p1.w * dx + p1.z * dy;
      double ec = z.z * hc + z.w * hs, es = -z.w * hc + z.z * hs;
      rot_normalize(ec, es);
      const double tx = hx - z.x, ty = hy - z.y;
      const double r0e = z.z * tx + z.w * ty, r1e = -z.w * tx + z.z * ty, r2e = atan2(es, ec);
      const double dt1 = -p2.w * dx + p2.z * dy, dt2 = -p2.z * dx - p2.w * dy;
      const double m00 = -hc * o00 + hs * o01, m01 = -hs * o00 - hc * o01, m02 = dt1 * o00 + dt2 * o01 - o02;
      const double m10 = -hc * o01 + hs * o11, m11 = -hs * o01 - hc * o11, m12 = dt1 * o01 + dt2 * o11 - o12;
      const double m20 = -hc * o02 + hs * o12, m21 = -hs * o02 - hc * o12, m22 = dt1 * o02 + dt2 * o12 - o22;
      const double w0 = o00 * r0e + o01 * r1e + o02 * r2e;
      const double w1 = o01 * r0e + o11 * r1e + o12 * r2e;
      const double w2 = o02 * r0e + o12 * r1e + o22 * r2e;
      double* v = &sm[0][0] + 9 * t;   // this factor's record, staged
      if (d.eside[e] == 0) {   // owner block H_ij = M'
        v[0] = m00; v[1] = m10; v[2] = m20;
        v[3] = m01; v[4] = m11; v[5] = m21;
        v[6] = m02; v[7] = m12; v[8] = m22;
      } else {                 // owner block H_ji = M
        v[0] = m00; v[1] = m01; v[2] = m02;
        v[3] = m10; v[4] = m11; v[5] = m12;
        v[6] = m20; v[7] = m21; v[8] = m22;
      }
      d.W[d.s1pos[e]] = make_double4(w0, w1, w2, 0.0);   // row ej's side-1 list order
      s0 = -hc * m00 + hs * m10;
      s1 = -hc * m01 + hs * m11;
      s2 = -hc * m02 + hs * m12;
      s3 = -hs * m01 - hc * m11;
      s4 = -hs * m02 - hc * m12;
      s5 = dt1 * m02 + dt2 * m12 - m22;
      s6 = -hc * w0 + hs * w1;
      s7 = -hs * w0 - hc * w1;
      s8 = dt1 * w0 + dt2 * w1 - w2;
    }
    __syncthreads();
    {   // the chunk's records [9 c0, 9 c0 + nv): 16-byte stores from an even element on
      const double* sv = &sm[0][0];
      const int nv = 9 * min(kThreads, e1 - c0), head = c0 & 1;   // (9 c0 odd <=> c0 odd)
      double* dst = d.V + 9 * (size_t)c0;
      if (head && t == 0) dst[0] = sv[0];
      for (int k = t; 2 * k + 1 < nv - head; k += kThreads)
        *reinterpret_cast<double2*>(dst + head + 2 * k) = make_double2(sv[head + 2 * k], sv[head + 2 * k + 1]);
      if (((nv - head) & 1) && t == 0) dst[nv - 1] = sv[nv - 1];
    }
    __syncthreads();
    if (e < e1) {
      sm[0][t] = s0; sm[1][t] = s1; sm[2][t] = s2; sm[3][t] = s3; sm[4][t] = s4;
      sm[5][t] = s5; sm[6][t] = s6; sm[7][t] = s7; sm[8][t] = s8;
    }
    __syncthreads();
    if (rowt) {
      const int kb = rb > c0 ? rb : c0, ke = re < c0 + kThreads ? re : c0 + kThreads;
      for (int k = kb - c0; k < ke - c0; k++) {
        a00 += sm[0][k]; a01 += sm[1][k]; a02 += sm[2][k]; a11 += sm[3][k]; a12 += sm[4][k];
        a22 += sm[5][k]; g0 += sm[6][k]; g1 += sm[7][k]; g2 += sm[8][k];
      }
    }
    __syncthreads();
  }
  if (rowt) {
    const double* dc = d.Dc + 6 * (size_t)row;
    a00 += dc[0]; a01 += dc[1]; a02 += dc[2]; a11 += dc[3]; a12 += dc[4]; a22 += dc[5];
    for (int q = d.prior_ptr[row]; q < d.prior_ptr[row + 1]; q++) {   // PriorFactor<Pose2>
      const double4 p1 = d.pose[row], pz = d.pz[q];
      double c = p1.z * pz.z + p1.w * pz.w, s = -p1.w * pz.z + p1.z * pz.w;
      rot_normalize(c, s);
      const double dx = pz.x - p1.x, dy = pz.y - p1.y;
      const double e0 = -(p1.z * dx + p1.w * dy), e1 = -(-p1.w * dx + p1.z * dy), e2 = -atan2(s, c);
      const double2 oA = d.pom[3 * q], oB = d.pom[3 * q + 1], oC = d.pom[3 * q + 2];
      const double o00 = oA.x, o01 = oA.y, o02 = oB.x, o11 = oB.y, o12 = oC.x, o22 = oC.y;
      const double w0 = o00 * e0 + o01 * e1 + o02 * e2;
      const double w1 = o01 * e0 + o11 * e1 + o12 * e2;
      const double w2 = o02 * e0 + o12 * e1 + o22 * e2;
      a00 += o00; a01 += o01; a02 += o02; a11 += o11; a12 += o12; a22 += o22;
      g0 += w0; g1 += w1; g2 += w2;
    }
    double* D = d.D + 6 * (size_t)row;
    D[0] = a00; D[1] = a01; D[2] = a02; D[3] = a11; D[4] = a12; D[5] = a22;
    double* g = d.g + 3 * (size_t)row;
    g[0] = g0; g[1] = g1; g[2] = g2;
  }
}

// Row j's side-1 gradient terms: g_j += sum of Omega e over the factors with
// ej = j (fixed order: device factor order), after k_linearize_own.  W is in
// side-1 list order, so a row's terms are contiguous (no index gather).
template <int G>
__global__ __launch_bounds__(kThreads) void k_linearize_side1(DevGraph d) {
  const int lane = threadIdx.x & (G - 1);
  const int nsg = gridDim.x * (kThreads / G);
  for (int row = (blockIdx.x * kThreads + threadIdx.x) / G; row < d.n; row += nsg) {
    double s0 = 0, s1 = 0, s2 = 0;
    for (int t = d.s1_ptr[row] + lane; t < d.s1_ptr[row + 1]; t += G) {
      const double4 w = d.W[t];
      s0 += w.x; s1 += w.y; s2 += w.z;
    }
    s0 = sg_sum<G>(s0); s1 = sg_sum<G>(s1); s2 = sg_sum<G>(s2);
    if (lane == 0) {
      double* g = d.g + 3 * (size_t)row;
      g[0] += s0; g[1] += s1; g[2] += s2;
    }
  }
}

// ------------------------------------------------------------ error / retract
// 0.5 e'Omega e per factor (NonlinearFactorGraph::error), block partials.
__global__ __launch_bounds__(kThreads) void k_error(DevGraph d, const double4* __restrict__ pose) {
  __shared__ double lds[kThreads / 64];
  double acc = 0.0;
  const int total = d.ne + d.np;
  for (int t = blockIdx.x * kThreads + threadIdx.x; t < total; t += gridDim.x * kThreads) {
    double e0, e1, e2;
    double2 oA, oB, oC;
    if (t < d.ne) {
      const int2 ij = d.eij[t];
      const double4 p1 = pose[ij.x], p2 = pose[ij.y], z = d.ez[t];
      double hc = p1.z * p2.z + p1.w * p2.w, hs = -p1.w * p2.z + p1.z * p2.w;
      rot_normalize(hc, hs);
      const double dx = p2.x - p1.x, dy = p2.y - p1.y;
      const double hx = p1.z * dx + p1.w * dy, hy = -p1.w * dx + p1.z * dy;
      double ec = z.z * hc + z.w * hs, es = -z.w * hc + z.z * hs;
      rot_normalize(ec, es);
      const double tx = hx - z.x, ty = hy - z.y;
      e0 = z.z * tx + z.w * ty;
      e1 = -z.w * tx + z.z * ty;
      e2 = atan2(es, ec);
      oA = d.eom[3 * t]; oB = d.eom[3 * t + 1]; oC = d.eom[3 * t + 2];
    } else {
      const int q = t - d.ne;
      const double4 x = pose[d.prior_vtx[q]], pz = d.pz[q];
      double c = x.z * pz.z + x.w * pz.w, s = -x.w * pz.z + x.z * pz.w;
      rot_normalize(c, s);
      const double dx = pz.x - x.x, dy = pz.y - x.y;
      e0 = -(x.z * dx + x.w * dy);
      e1 = -(-x.w * dx + x.z * dy);
      e2 = -atan2(s, c);
      oA = d.pom[3 * q]; oB = d.pom[3 * q + 1]; oC = d.pom[3 * q + 2];
    }
    const double w0 = oA.x * e0 + oA.y * e1 + oB.x * e2;
    const double w1 = oA.y * e0 + oB.y * e1 + oC.x * e2;
    const double w2 = oB.x * e0 + oC.x * e1 + oC.y * e2;
    acc += 0.5 * (e0 * w0 + e1 * w1 + e2 * w2);
  }
  acc = block_sum(acc, lds);
  if (threadIdx.x == 0) d.part[kPartA * kMaxBlocks + blockIdx.x] = acc;
}

// Single block: out[v] = sum of nb partials of slice (first + v), v < nv.
__global__ __launch_bounds__(kThreads) void k_reduce(const double* __restrict__ part, int first, int nv,
                                                    int nb, double* __restrict__ out) {
  __shared__ double lds[kThreads / 64];
  for (int v = 0; v < nv; v++) {
    const double s = sum_partials(part + (size_t)(first + v) * kMaxBlocks, nb, lds);
    if (threadIdx.x == 0) out[v] = s;
  }
}

// Values::retract: pose_cand = pose * Pose2(delta)  (default Pose2 chart)
__global__ __launch_bounds__(kThreads) void k_retract(DevGraph d, const double* __restrict__ delta) {
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < d.n; i += gridDim.x * kThreads) {
    const double4 p = d.pose[i];
    const double d0 = delta[3 * i], d1 = delta[3 * i + 1], d2 = delta[3 * i + 2];
    double sd, cd;
    sincos(d2, &sd, &cd);
    double c = p.z * cd - p.w * sd, s = p.w * cd + p.z * sd;
    rot_normalize(c, s);
    d.pose_cand[i] = make_double4(p.x + p.z * d0 - p.w * d1, p.y + p.w * d0 + p.z * d1, c, s);
  }
}

// ------------------------------------------------------------ PCG
// (H + lambda I) delta = -g, block-Jacobi preconditioner M = blockdiag(H_ii + lambda I).
__global__ __launch_bounds__(kThreads) void k_pcg_init(DevGraph d, double lam) {
  __shared__ double lds[kThreads / 64];
  double rz = 0.0;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < d.n; i += gridDim.x * kThreads) {
    const double* D = d.D + 6 * (size_t)i;
    const double a00 = D[0] + lam, a01 = D[1], a02 = D[2], a11 = D[3] + lam, a12 = D[4], a22 = D[5] + lam;
    const double c00 = a11 * a22 - a12 * a12, c01 = a02 * a12 - a01 * a22, c02 = a01 * a12 - a02 * a11;
    const double c11 = a00 * a22 - a02 * a02, c12 = a01 * a02 - a00 * a12, c22 = a00 * a11 - a01 * a01;
    const double det = a00 * c00 + a01 * c01 + a02 * c02;
    if (!(det > 0.0) || !isfinite(det)) d.ctrl[0] = kBreakdown;
    const double inv = 1.0 / det;
    double* M = d.Minv + 6 * (size_t)i;
    M[0] = c00 * inv; M[1] = c01 * inv; M[2] = c02 * inv; M[3] = c11 * inv; M[4] = c12 * inv; M[5] = c22 * inv;
    const double r0 = -d.g[3 * i], r1 = -d.g[3 * i + 1], r2 = -d.g[3 * i + 2];
    const double z0 = M[0] * r0 + M[1] * r1 + M[2] * r2;
    const double z1 = M[1] * r0 + M[3] * r1 + M[4] * r2;
    const double z2 = M[2] * r0 + M[4] * r1 + M[5] * r2;
    d.r[3 * i] = r0; d.r[3 * i + 1] = r1; d.r[3 * i + 2] = r2;
    d.z[3 * i] = z0; d.z[3 * i + 1] = z1; d.z[3 * i + 2] = z2;
    d.p[3 * i] = z0; d.p[3 * i + 1] = z1; d.p[3 * i + 2] = z2;
    d.x[3 * i] = 0.0; d.x[3 * i + 1] = 0.0; d.x[3 * i + 2] = 0.0;
    rz += r0 * z0 + r1 * z1 + r2 * z2;
  }
  rz = block_sum(rz, lds);
  if (threadIdx.x == 0) d.part[kPartRZ0 * kMaxBlocks + blockIdx.x] = rz;
}

// q = (H + lambda I) p, partial p.q
template <int G>
__global__ __launch_bounds__(kThreads) void k_pcg_spmv(DevGraph d, double lam) {
  if (d.ctrl[0] != kRunning) return;
  __shared__ double lds[kThreads / 64];
  const int lane = threadIdx.x & (G - 1);
  const int nsg = gridDim.x * (kThreads / G);
  const double* __restrict__ P = d.p;
  double pq = 0.0;
  for (int row = (blockIdx.x * kThreads + threadIdx.x) / G; row < d.n; row += nsg) {
    double y0 = 0, y1 = 0, y2 = 0;
    const int beg = d.row_ptr[row], end = d.row_ptr[row + 1];
    for (int k = beg + lane; k < end; k += G) {
      const int c = d.slot_col[k];
      const double* v = d.V + k;
      const size_t S = d.nslots;
      const double x0 = P[3 * c], x1 = P[3 * c + 1], x2 = P[3 * c + 2];
      y0 += v[0] * x0 + v[S] * x1 + v[2 * S] * x2;
      y1 += v[3 * S] * x0 + v[4 * S] * x1 + v[5 * S] * x2;
      y2 += v[6 * S] * x0 + v[7 * S] * x1 + v[8 * S] * x2;
    }
    y0 = sg_sum<G>(y0);
    y1 = sg_sum<G>(y1);
    y2 = sg_sum<G>(y2);
    if (lane == 0) {
      const double* D = d.D + 6 * (size_t)row;
      const double x0 = P[3 * row], x1 = P[3 * row + 1], x2 = P[3 * row + 2];
      y0 += (D[0] + lam) * x0 + D[1] * x1 + D[2] * x2;
      y1 += D[1] * x0 + (D[3] + lam) * x1 + D[4] * x2;
      y2 += D[2] * x0 + D[4] * x1 + (D[5] + lam) * x2;
      d.q[3 * row] = y0; d.q[3 * row + 1] = y1; d.q[3 * row + 2] = y2;
      pq += x0 * y0 + x1 * y1 + x2 * y2;
    }
  }
  pq = block_sum(pq, lds);
  if (threadIdx.x == 0) d.part[kPartPQ * kMaxBlocks + blockIdx.x] = pq;
}

// alpha = r.z / p.q ; x += alpha p ; r -= alpha q ; z = M^-1 r ; partial r.z
__global__ __launch_bounds__(kThreads) void k_pcg_update(DevGraph d, int nb_spmv, int nb_vec,
                                                        int old_slice, int new_slice) {
  if (d.ctrl[0] != kRunning) return;
  __shared__ double lds[kThreads / 64];
  const double pq = sum_partials(d.part + kPartPQ * kMaxBlocks, nb_spmv, lds);
  const double rzo = sum_partials(d.part + (size_t)old_slice * kMaxBlocks, nb_vec, lds);
  if (rzo == 0.0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) d.ctrl[0] = kConverged;
    return;
  }
  if (!(pq > 0.0) || !isfinite(pq)) {
    if (blockIdx.x == 0 && threadIdx.x == 0) d.ctrl[0] = kBreakdown;
    return;
  }
  const double alpha = rzo / pq;
  double rz = 0.0;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < d.n; i += gridDim.x * kThreads) {
    double r[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
      d.x[3 * i + a] += alpha * d.p[3 * i + a];
      r[a] = d.r[3 * i + a] - alpha * d.q[3 * i + a];
      d.r[3 * i + a] = r[a];
    }
    const double* M = d.Minv + 6 * (size_t)i;
    const double z0 = M[0] * r[0] + M[1] * r[1] + M[2] * r[2];
    const double z1 = M[1] * r[0] + M[3] * r[1] + M[4] * r[2];
    const double z2 = M[2] * r[0] + M[4] * r[1] + M[5] * r[2];
    d.z[3 * i] = z0; d.z[3 * i + 1] = z1; d.z[3 * i + 2] = z2;
    rz += r[0] * z0 + r[1] * z1 + r[2] * z2;
  }
  rz = block_sum(rz, lds);
  if (threadIdx.x == 0) d.part[(size_t)new_slice * kMaxBlocks + blockIdx.x] = rz;
}

// beta = r.z(new) / r.z(old) ; p = z + beta p ; convergence test in block 0
__global__ __launch_bounds__(kThreads) void k_pcg_dir(DevGraph d, int nb_vec, int old_slice, int new_slice,
                                                     double tol2) {
  if (d.ctrl[0] != kRunning) return;
  __shared__ double lds[kThreads / 64];
  const double rzo = sum_partials(d.part + (size_t)old_slice * kMaxBlocks, nb_vec, lds);
  const double rzn = sum_partials(d.part + (size_t)new_slice * kMaxBlocks, nb_vec, lds);
  const double beta = rzn / rzo;
  for (int i = blockIdx.x * kThreads + threadIdx.x; i < d.n; i += gridDim.x * kThreads) {
#pragma unroll
    for (int a = 0; a < 3; a++) d.p[3 * i + a] = d.z[3 * i + a] + beta * d.p[3 * i + a];
  }
  if (blockIdx.x == 0) {
    const double rz0 = sum_partials(d.part + kPartRZ0 * kMaxBlocks, nb_vec, lds);
    if (threadIdx.x == 0) {
      d.ctrl[1] += 1;
      if (!isfinite(rzn)) d.ctrl[0] = kBreakdown;
      else if (rzn <= tol2 * rz0) d.ctrl[0] = kConverged;
    }
  }
}

// Partials delta'H delta (slice A) and g'delta (slice A+1), H undamped:
// delta'H delta = sum_i d_i'H_ii d_i + 2 sum over owner slots d_row'H_{row,col} d_col,
// so it needs only the owner blocks (what the Cholesky-mode linearisation writes).
template <int G>
__global__ __launch_bounds__(kThreads) void k_model_decrease(DevGraph d, const double* __restrict__ X) {
  __shared__ double lds[kThreads / 64];
  const int lane = threadIdx.x & (G - 1);
  const int nsg = gridDim.x * (kThreads / G);
  const size_t S = d.nslots;
  double xhx = 0.0, gx = 0.0;
  const bool own_at_edge = !d.write_all && d.eside;   // k_linearize_own layout
  for (int row = (blockIdx.x * kThreads + threadIdx.x) / G; row < d.n; row += nsg) {
    const double r0 = X[3 * row], r1 = X[3 * row + 1], r2 = X[3 * row + 2];
    double t = 0.0;
    const int beg = d.row_ptr[row], end = d.row_ptr[row + 1];
    for (int k = beg + lane; k < end; k += G) {
      const int se = d.slot_edge[k];
      if (!(se & 2)) continue;
      const int c = d.slot_col[k];
      const double* v = d.V + (own_at_edge ? 9 * (size_t)(se >> 2) : k);
      const size_t st = own_at_edge ? 1 : S;   // (k_linearize_own: a factor's 9 elements together)
      const double x0 = X[3 * c], x1 = X[3 * c + 1], x2 = X[3 * c + 2];
      const double y0 = v[0] * x0 + v[st] * x1 + v[2 * st] * x2;
      const double y1 = v[3 * st] * x0 + v[4 * st] * x1 + v[5 * st] * x2;
      const double y2 = v[6 * st] * x0 + v[7 * st] * x1 + v[8 * st] * x2;
      t += r0 * y0 + r1 * y1 + r2 * y2;
    }
    t = sg_sum<G>(t);
    if (lane == 0) {
      const double* D = d.D + 6 * (size_t)row;
      const double y0 = D[0] * r0 + D[1] * r1 + D[2] * r2;
      const double y1 = D[1] * r0 + D[3] * r1 + D[4] * r2;
      const double y2 = D[2] * r0 + D[4] * r1 + D[5] * r2;
      xhx += 2.0 * t + (r0 * y0 + r1 * y1 + r2 * y2);
      gx += d.g[3 * row] * r0 + d.g[3 * row + 1] * r1 + d.g[3 * row + 2] * r2;
    }
  }
  xhx = block_sum(xhx, lds);
  gx = block_sum(gx, lds);
  if (threadIdx.x == 0) {
    d.part[kPartA * kMaxBlocks + blockIdx.x] = xhx;
    d.part[(kPartA + 1) * kMaxBlocks + blockIdx.x] = gx;
  }
}

// y = (H + lambda I) x  (diagnostics)
template <int G>
__global__ __launch_bounds__(kThreads) void k_spmv(DevGraph d, double lam, const double* __restrict__ X,
                                                  double* __restrict__ Y) {
  const int lane = threadIdx.x & (G - 1);
  const int nsg = gridDim.x * (kThreads / G);
  for (int row = (blockIdx.x * kThreads + threadIdx.x) / G; row < d.n; row += nsg) {
    double y0 = 0, y1 = 0, y2 = 0;
    const int beg = d.row_ptr[row], end = d.row_ptr[row + 1];
    for (int k = beg + lane; k < end; k += G) {
      const int c = d.slot_col[k];
      const double* v = d.V + k;
      const size_t S = d.nslots;
      const double x0 = X[3 * c], x1 = X[3 * c + 1], x2 = X[3 * c + 2];
      y0 += v[0] * x0 + v[S] * x1 + v[2 * S] * x2;
      y1 += v[3 * S] * x0 + v[4 * S] * x1 + v[5 * S] * x2;
      y2 += v[6 * S] * x0 + v[7 * S] * x1 + v[8 * S] * x2;
    }
    y0 = sg_sum<G>(y0);
    y1 = sg_sum<G>(y1);
    y2 = sg_sum<G>(y2);
    if (lane == 0) {
      const double* D = d.D + 6 * (size_t)row;
      const double x0 = X[3 * row], x1 = X[3 * row + 1], x2 = X[3 * row + 2];
      Y[3 * row] = y0 + (D[0] + lam) * x0 + D[1] * x1 + D[2] * x2;
      Y[3 * row + 1] = y1 + D[1] * x0 + (D[3] + lam) * x1 + D[4] * x2;
      Y[3 * row + 2] = y2 + D[2] * x0 + D[4] * x1 + (D[5] + lam) * x2;
    }
  }
}

// ------------------------------------------------------------ launchers
int grid_for(int work) {
  int b = (work + kThreads - 1) / kThreads;
  if (b < 1) b = 1;
  return b > kMaxBlocks ? kMaxBlocks : b;
}

int grid_rows(const DevGraph& d) {
  const long long threads = (long long)d.n * d.G;
  long long b = (threads + kThreads - 1) / kThreads;
  if (b < 1) b = 1;
  return (int)(b > kMaxBlocks ? kMaxBlocks : b);
}

#define PGO_DISPATCH_G(G_, KERNEL, ...)                                           \
  switch (G_) {                                                                   \
    case 4: KERNEL<4><<<grid_rows(d), kThreads, 0, d.stream>>>(__VA_ARGS__); break;   \
    case 8: KERNEL<8><<<grid_rows(d), kThreads, 0, d.stream>>>(__VA_ARGS__); break;   \
    case 16: KERNEL<16><<<grid_rows(d), kThreads, 0, d.stream>>>(__VA_ARGS__); break; \
    default: KERNEL<32><<<grid_rows(d), kThreads, 0, d.stream>>>(__VA_ARGS__); break; \
  }

hipError_t launch_linearize(const DevGraph& d, hipEvent_t start, hipEvent_t stop) {
  if (d.n == 0) return hipSuccess;
  const dim3 block(kThreads);
  if (!d.write_all && d.eside) {   // Cholesky mode: owner blocks in factor order
    const dim3 grid1((unsigned)(((long long)d.n * d.G1 + kThreads - 1) / kThreads));
    hipExtLaunchKernelGGL(k_linearize_own, dim3(d.nlb), block, 0, d.stream, start, nullptr, 0, d);
    switch (d.G1) {
      case 4: hipExtLaunchKernelGGL(k_linearize_side1<4>, grid1, block, 0, d.stream, nullptr, stop, 0, d); break;
      case 8: hipExtLaunchKernelGGL(k_linearize_side1<8>, grid1, block, 0, d.stream, nullptr, stop, 0, d); break;
      case 16: hipExtLaunchKernelGGL(k_linearize_side1<16>, grid1, block, 0, d.stream, nullptr, stop, 0, d); break;
      default: hipExtLaunchKernelGGL(k_linearize_side1<32>, grid1, block, 0, d.stream, nullptr, stop, 0, d); break;
    }
    return hipGetLastError();
  }
  const dim3 grid((unsigned)(((long long)d.n * d.G + kThreads - 1) / kThreads));   // one sub-group per row
  switch (d.G) {
    case 4: hipExtLaunchKernelGGL(k_linearize<4>, grid, block, 0, d.stream, start, stop, 0, d); break;
    case 8: hipExtLaunchKernelGGL(k_linearize<8>, grid, block, 0, d.stream, start, stop, 0, d); break;
    case 16: hipExtLaunchKernelGGL(k_linearize<16>, grid, block, 0, d.stream, start, stop, 0, d); break;
    default: hipExtLaunchKernelGGL(k_linearize<32>, grid, block, 0, d.stream, start, stop, 0, d); break;
  }
  return hipGetLastError();
}

hipError_t launch_error(const DevGraph& d, const double4* pose, double* out_scalar) {
  const int nb = grid_for(d.ne + d.np);
  k_error<<<nb, kThreads, 0, d.stream>>>(d, pose);
  k_reduce<<<1, kThreads, 0, d.stream>>>(d.part, kPartA, 1, nb, out_scalar);
  return hipGetLastError();
}

hipError_t launch_retract(const DevGraph& d, const double* delta) {
  if (d.n == 0) return hipSuccess;
  k_retract<<<grid_for(d.n), kThreads, 0, d.stream>>>(d, delta);
  return hipGetLastError();
}

hipError_t launch_pcg_init(const DevGraph& d, double lambda) {
  hipError_t e = hipMemsetAsync(d.ctrl, 0, 4 * sizeof(int), d.stream);
  if (e != hipSuccess) return e;
  k_pcg_init<<<grid_for(d.n), kThreads, 0, d.stream>>>(d, lambda);
  return hipGetLastError();
}

// start/stop (optional): events written by the dispatch itself
// (hipExtLaunchKernelGGL), i.e. the kernel's own begin/end like rocprofv3's
// kernel trace -- no extra marker packets around the launch.
hipError_t launch_pcg_spmv(const DevGraph& d, double lambda, hipEvent_t start, hipEvent_t stop) {
  const dim3 grid(grid_rows(d)), block(kThreads);
  switch (d.G) {
    case 4: hipExtLaunchKernelGGL(k_pcg_spmv<4>, grid, block, 0, d.stream, start, stop, 0, d, lambda); break;
    case 8: hipExtLaunchKernelGGL(k_pcg_spmv<8>, grid, block, 0, d.stream, start, stop, 0, d, lambda); break;
    case 16: hipExtLaunchKernelGGL(k_pcg_spmv<16>, grid, block, 0, d.stream, start, stop, 0, d, lambda); break;
    default: hipExtLaunchKernelGGL(k_pcg_spmv<32>, grid, block, 0, d.stream, start, stop, 0, d, lambda); break;
  }
  return hipGetLastError();
}

// iteration k: rz ping-pong slices (k == 0 reads the initial slice)
hipError_t launch_pcg_vec(const DevGraph& d, int k, double tol2) {
  const int old_slice = k == 0 ? kPartRZ0 : kPartRZ0 + 1 + ((k - 1) & 1);
  const int new_slice = kPartRZ0 + 1 + (k & 1);
  const int nbv = grid_for(d.n);
  k_pcg_update<<<nbv, kThreads, 0, d.stream>>>(d, grid_rows(d), nbv, old_slice, new_slice);
  k_pcg_dir<<<nbv, kThreads, 0, d.stream>>>(d, nbv, old_slice, new_slice, tol2);
  return hipGetLastError();
}

hipError_t launch_model_decrease(const DevGraph& d, const double* delta, double* out2) {
  PGO_DISPATCH_G(d.G, k_model_decrease, d, delta);
  k_reduce<<<1, kThreads, 0, d.stream>>>(d.part, kPartA, 2, grid_rows(d), out2);
  return hipGetLastError();
}

hipError_t launch_spmv(const DevGraph& d, double lambda, const double* x, double* y) {
  if (d.n == 0) return hipSuccess;
  PGO_DISPATCH_G(d.G, k_spmv, d, lambda, x, y);
  return hipGetLastError();
}

}  // namespace pgo
