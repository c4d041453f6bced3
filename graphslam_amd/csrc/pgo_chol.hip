// GPU supernodal multifrontal Cholesky of H + lambda I and its triangular
// solves (gfx950).  Host plan: pgo_symbolic.cpp; layout: pgo_chol.h.
//
// Factorisation, per level of the supernodal tree (leaves first):
//   k_assemble_tile every front of the level, one workgroup per 64x64 lower
//                  tile, written whole: H entries (+ lambda), then the
//                  children's update matrices in order (no atomics, fixed
//                  order, bitwise reproducible; no front is ever zeroed)
//   k_front_wave   fronts with m <= 128, w <= 32: one wavefront each
//   k_panel_first  blocked path, first 64-column panel: diagonal tile factored
//                  and inverted in LDS, the rows below solved as MFMA GEMMs with
//                  the inverse by workgroups that wait for it in the same launch
//   k_step         each further panel: the next diagonal tile updated, factored
//                  and inverted (look-ahead), the tiles below it updated then
//                  solved (in-launch hand-off), the other trailing tiles updated
//                  (v_mfma_f64_16x16x4_f64); big updates in k_panel_syrk_lds /
//                  k_panel_syrk128 beside it
// Solves: the forward substitution rides in the factorisation (the right-hand
// side is an extra column), backward top-down per level.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>

#include "pgo_chol.h"

namespace pgo {

struct CholDev {
  double* F;
  double* Tinv;
  const long long* toff;
  double* fv;
  double* xv;
  const int *m, *w, *voff, *rptr, *rows;
  const long long* foff;
  const int *cptr, *children, *ea_rel, *ea_ptr, *parent;
  const int *asm_front, *asm_li, *asm_lj, *asm_ptr, *asm_src;
  const int *dg_front, *dg_loc, *perm;
  int* flag;
  int* stepflag;                   // [lane][ns] in-launch hand-off of the diagonal inverses
  int ns;
  // lambda lanes: lane y = blockIdx.y works on its own numeric workspace
  long long fst, tst;              // F, Tinv doubles per lane
  long long tfo;                   // Tinv + tfo: the inverses again, in the trsm's MFMA operand order
  int vst, xst, pst;               // fv, xv, backward partials per lane
  unsigned long long poll_ticks;   // in-launch hand-off: give up after this many 10 ns ticks
  int diag_full;                   // PGO_DIAG_FULL=1 (A/B): diagonal tiles factored over all four 16-column blocks
};

// this workgroup's lane (blockIdx.y): every lane factors H + lambda_y I with
// the same schedule, so lanes are bitwise equal to one-lane runs
__device__ __forceinline__ void lane_offset(CholDev& c) {
  const int y = blockIdx.y;
  c.F += y * c.fst;
  c.Tinv += y * c.tst;
  c.fv += y * c.vst;
  c.xv += y * c.xst;
  c.flag += y;
  c.stepflag += (long long)y * c.ns;
}

static CholDev dev_view(const CholPlan& P) {
  CholDev c;
  c.F = P.F; c.fv = P.fv; c.xv = P.xv; c.Tinv = P.Tinv; c.toff = P.d_toff;
  c.m = P.d_m; c.w = P.d_w; c.voff = P.d_voff; c.rptr = P.d_rptr; c.rows = P.d_rows; c.foff = P.d_foff;
  c.cptr = P.d_cptr; c.children = P.d_children; c.ea_rel = P.d_ea_rel; c.ea_ptr = P.d_ea_ptr;
  c.parent = P.d_parent;
  c.asm_front = P.d_asm_front; c.asm_li = P.d_asm_li; c.asm_lj = P.d_asm_lj; c.asm_ptr = P.d_asm_ptr;
  c.asm_src = P.d_asm_src; c.dg_front = P.d_dg_front; c.dg_loc = P.d_dg_loc; c.perm = P.d_perm;
  c.flag = P.d_flag;
  c.stepflag = P.d_stepflag;
  c.ns = P.ns;
  static const int diag_full = getenv("PGO_DIAG_FULL") && atoi(getenv("PGO_DIAG_FULL")) == 1;
  c.diag_full = diag_full;
  c.fst = P.ftotal;
  c.tst = 2 * P.ttotal;
  c.tfo = P.ttotal;
  c.vst = P.vtotal;
  c.xst = 3 * P.n;
  c.pst = std::max(P.npart, 1) * 64;
  // PGO_HANDOFF_TIMEOUT_MS (default 2000): a hand-off wait that long means a
  // lost workgroup (a time-sliced queue on a shared GPU waits far less)
  static const double tmo_ms = getenv("PGO_HANDOFF_TIMEOUT_MS") ? atof(getenv("PGO_HANDOFF_TIMEOUT_MS")) : 2000.0;
  c.poll_ticks = (unsigned long long)(std::max(tmo_ms, 1.0) * 1e5);
  return c;
}

typedef double d4 __attribute__((ext_vector_type(4)));

// Front storage (pgo_chol.h front_packed / front_elems): element (i, j) of the
// front at Fs is fcol(Fs, m, pk, j)[i] -- for a packed front (the blocked
// path) column block b = j / 64 holds rows [64 b, m) with leading dimension
// fld(m, pk, j) = fpad(m) - 64 b, so i >= 64 b; an unpacked one is m x m.
__device__ __forceinline__ long long fcol_off(int m, bool pk, int j) {
  if (!pk) return (long long)j * m;
  const int mp = fpad(m);
  const long long b = j >> 6, c0 = b << 6;
  return fblock_off(mp, b) + (j - c0) * (long long)(mp - c0) - c0;
}
template <class T>
__device__ __forceinline__ T* fcol(T* Fs, int m, bool pk, int j) {
  return Fs + fcol_off(m, pk, j);
}
__device__ __forceinline__ int fld(int m, bool pk, int j) { return pk ? fpad(m) - (j & ~63) : m; }


// Step timing stamps (diagnostics, PGO_STEP_STAMPS): k_step launches given a
// slot >= 0 record wall-clock stamps of their first diagonal workgroup and first
// waiting workgroup; read back with chol_step_stamps.  Written only here and
// read only by the host.
__device__ unsigned long long g_stamps[kMaxStampSlots][10];
#define STAMP(slot, q)                                                        \
  do {                                                                        \
    if ((slot) >= 0 && threadIdx.x == 0) g_stamps[(slot)][(q)] = wall_clock64(); \
  } while (0)

#ifdef PGO_DIAG_CLOCKS
__device__ long long g_diag_clk[32];
__device__ long long g_d8_clk[4][8][8];   // diag_factor_invert8: [wave][step][phase]
__device__ int g_d8_dbg;   // diagnostics: 1 = waves 2-3 idle, 2 = no waits on wave 1, 4 = wave 1 idle
#define D8_DBG(bit) (g_d8_dbg & (bit))
#define DIAG_CLKF(q)                                                                   \
  do {                                                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    if (threadIdx.x == 0 && blockIdx.x == 0) g_diag_clk[q] = clock64();                \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#define DIAG_CLK(q) if (threadIdx.x == 0 && blockIdx.x == 0) g_diag_clk[q] = clock64()
#define D8_CLK(k, q)                                                                 \
  do {                                                                               \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                              \
    __builtin_amdgcn_sched_barrier(0);                                               \
    if ((threadIdx.x & 63) == 0 && blockIdx.x == 0) g_d8_clk[threadIdx.x >> 6][k][q] = clock64(); \
    __builtin_amdgcn_sched_barrier(0);                                               \
  } while (0)
#else
#define DIAG_CLK(q)
#define DIAG_CLKF(q)
#define D8_CLK(k, q)
#define D8_DBG(bit) 0
#endif


// ------------------------------------------------------------ assembly
// One 64x64 lower tile (ti, tj) of a front per workgroup, written whole (so no
// front is ever zeroed), gathered element by element: thread (i = tid & 63,
// columns j = tid / 64 + 4u) owns 16 elements of the tile and forms each as
// its H entry -- an off-diagonal block H_{a,b} summed over its slots (V,
// structure of arrays) or a diagonal block H_jj + lambda I, lower part -- plus
// the front's children's update-matrix elements that land on it, in child
// order (fixed summation order, bitwise reproducible, no atomics, no LDS
// read-modify-write).  What an element needs is looked up in LDS maps built
// once per tile: the H item of each 3x3 pose block the tile spans, and per
// child rectangle the child row of each tile row and the child column (and
// its column offset) of each tile column.  Two barriers per tile (per 16 child
// rectangles), and every element's loads are in flight together.
constexpr int kAsmPairs = 16;
#ifndef PGO_ASM_GE
#define PGO_ASM_GE 8
#endif
constexpr int kAsmGE = PGO_ASM_GE;   // a thread's 16 elements in 16 / kAsmGE groups: kAsmGE loads in flight per child
constexpr int kAsmNone = (int)0x80000000;

// Frontal vector of front s before its factorisation: own rows from the
// permuted right-hand side, below rows zero, plus the children's update
// vectors in child order (the factorisation then carries it as an extra
// column: forward substitution fused into the panels).  Built in LDS (v:
// kVecChunk doubles) a row range at a time -- each element sees the same adds
// in the same order whatever the chunking.
constexpr int kVecChunk = 1024;
__device__ __forceinline__ void vec_assemble_body(const CholDev& c, int s, double* v) {
  const int m = c.m[s], w = c.w[s];
  const int* rows = c.rows + c.rptr[s];
  double* fv = c.fv + c.voff[s];
  const int tid = threadIdx.x;
  for (int c0 = 0; c0 < m; c0 += kVecChunk) {
    const int c1 = min(m, c0 + kVecChunk);
    if (c0) __syncthreads();   // the previous range's reads of v are done
    for (int r = c0 + tid; r < c1; r += 256) v[r - c0] = r < w ? c.xv[3 * rows[r / 3] + r % 3] : 0.0;
    __syncthreads();
    for (int q = c.cptr[s]; q < c.cptr[s + 1]; q++) {
      const int ch = c.children[q];
      const int uc = c.m[ch] - c.w[ch];
      const double* uv = c.fv + c.voff[ch] + c.w[ch];
      const int* rel = c.ea_rel + c.ea_ptr[ch];
      for (int t = tid; t < uc; t += 256) {
        const int r = 3 * rel[t / 3] + t % 3;
        if (r >= c0 && r < c1) v[r - c0] += uv[t];
      }
      __syncthreads();
    }
    for (int r = c0 + tid; r < c1; r += 256) fv[r] = v[r - c0];
  }
}

// The level's tile assembly and, in workgroups [ntile, ntile + nvec) of the
// same launch, its frontal vectors (vec_assemble_body on the tile role's LDS
// maps, fronts vfronts[b - ntile]): disjoint data (F / fv), one launch and no
// side-stream fork and join per level
template <int kUnroll>
__global__ __launch_bounds__(256, 4) void k_assemble_tile(CholDev c, const int4* __restrict__ tasks,
                                                       const int2* __restrict__ iptr, const int* __restrict__ items,
                                                       const int4* __restrict__ pairs, const double* __restrict__ V,
                                                       const double* __restrict__ D,
                                                       const double* __restrict__ lam_p, int ntile = 1 << 30,
                                                       const int* __restrict__ vfronts = nullptr) {
  lane_offset(c);
  __shared__ int bcode[22 * 22];   // H item of pose block (bi, bj): asm target >= 0, ~pose (diagonal), or none
  __shared__ int bsrc[22 * 22];    // ... its first slot's factor (off-diagonal) or its pose's old index (diagonal)
  __shared__ int bcnt[22 * 22];    // ... its slot count
  __shared__ int rmap[kAsmPairs][64];            // child row landing on tile row i (-1: none)
  __shared__ int cmap[kAsmPairs][64];            // child column landing on tile column j (-1: none)
  __shared__ long long coff[kAsmPairs][64];      // ... its offset in the child front (row wc)
  __shared__ long long pbase[kAsmPairs];         // the child front's base
  static_assert(sizeof(coff) >= kVecChunk * sizeof(double), "frontal-vector range in coff");
  if ((int)blockIdx.x >= ntile) {   // (workgroup-uniform)
    vec_assemble_body(c, vfronts[blockIdx.x - ntile], reinterpret_cast<double*>(&coff[0][0]));
    return;
  }
  const int4 t = tasks[blockIdx.x];
  const int p = t.x, mp = c.m[p];
  const int R0 = 64 * (t.y >> 16), C0 = 64 * (t.y & 0xffff);
  const int P0 = R0 / 3, Q0 = C0 / 3;   // first pose block row / column the tile touches
  const int tid = threadIdx.x, i = tid & 63, cg = tid >> 6;
  const double lam = lam_p[blockIdx.y];
  const int2 it = iptr[blockIdx.x];
  for (int q = tid; q < 22 * 22; q += 256) bcode[q] = kAsmNone;
  for (int q = tid; q < kAsmPairs * 64; q += 256) {
    rmap[q >> 6][q & 63] = -1;
    cmap[q >> 6][q & 63] = -1;
  }
  __syncthreads();
  for (int q = tid; q < it.y; q += 256) {   // H items -> their pose blocks
    const int code = items[it.x + q];
    int li, lj, src, cnt;
    if (code >= 0) {
      li = c.asm_li[code];
      lj = c.asm_lj[code];
      const int k0 = c.asm_ptr[code];
      cnt = c.asm_ptr[code + 1] - k0;
      src = c.asm_src[k0];
    } else {
      li = lj = c.dg_loc[~code];
      src = c.perm[~code];
      cnt = 0;
    }
    const int bq = (li - P0) * 22 + (lj - Q0);
    bcode[bq] = code;
    bsrc[bq] = src;
    bcnt[bq] = cnt;
  }
  // this thread's 16 elements: (R0 + i, C0 + cg + 4u), in two groups of 8
  const int row = R0 + i;
  const int a3 = row - 3 * (row / 3), bi = row / 3 - P0;
  const bool pkp = front_packed(mp, c.w[p]);
  double* __restrict__ Fp = fcol(c.F + c.foff[p], mp, pkp, C0);   // the tile's columns: one column block
  const int ldp = fld(mp, pkp, C0);
  for (int pass = 0; pass * kAsmPairs < t.w || pass == 0; pass++) {
    const int k0 = pass * kAsmPairs, np = min(kAsmPairs, t.w - k0);
    if (pass > 0) {   // the previous pass's maps are read: reset them
      __syncthreads();
      for (int q = tid; q < kAsmPairs * 64; q += 256) {
        rmap[q >> 6][q & 63] = -1;
        cmap[q >> 6][q & 63] = -1;
      }
      __syncthreads();
    }
    for (int q = tid; q < np * 128; q += 256) {   // child rectangles -> row / column maps
      const int kk = q >> 7, h = q & 127;
      const int4 pr = pairs[t.z + k0 + kk];
      const int ch = pr.x, nr = pr.w & 0xff, nc = pr.w >> 8;
      const int* __restrict__ rel = c.ea_rel + c.ea_ptr[ch];
      if (h < 64) {
        if (h < nr) {
          const int a = pr.y + h;
          rmap[kk][3 * rel[a / 3] + a % 3 - R0] = a;
        }
        if (h == 0) pbase[kk] = c.foff[ch];
      } else if (h - 64 < nc) {
        const int b = pr.z + h - 64, mc = c.m[ch], wc = c.w[ch];
        const int pc = 3 * rel[b / 3] + b % 3 - C0;
        cmap[kk][pc] = b;
        coff[kk][pc] = fcol_off(mc, front_packed(mc, wc), wc + b) + wc;
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int g = 0; g < 16 / kAsmGE; g++) {
      double val[kAsmGE];
      if (pass == 0) {   // the H entries
#pragma unroll
        for (int u = 0; u < kAsmGE; u++) {
          const int col = C0 + cg + 4 * (kAsmGE * g + u);
          const int bq = bi * 22 + (col / 3 - Q0), b3 = col - 3 * (col / 3);
          const int code = bcode[bq];
          double v = 0.0;
          if (code >= 0) {
            const int e = 3 * a3 + b3;
            v += V[9 * (size_t)bsrc[bq] + e];   // (0 + first slot: the sum's order and zero signs as before)
            for (int k = 1; k < bcnt[bq]; k++) v += V[9 * (size_t)c.asm_src[c.asm_ptr[code] + k] + e];   // (repeated factors)
          } else if (code != kAsmNone && a3 >= b3) {
            const double* d = D + 6 * (size_t)bsrc[bq];
            const int e = a3 == 0 ? 0 : (a3 == 1 ? (b3 == 0 ? 1 : 3) : (b3 == 0 ? 2 : (b3 == 1 ? 4 : 5)));
            v = d[e] + (a3 == b3 ? lam : 0.0);
          }
          val[u] = v;
        }
      } else {           // a later pass (more than 16 child rectangles): this thread's partial sums so far
#pragma unroll
        for (int u = 0; u < kAsmGE; u++) {
          const int j = cg + 4 * (kAsmGE * g + u), col = C0 + j;
          val[u] = (row < mp && col < mp && row >= col) ? Fp[row + (size_t)j * ldp] : 0.0;
        }
      }
      // the children's elements, in child order; kUnroll children's loads in
      // flight together (the adds stay in child order: the same sums)
      for (int k1 = 0; k1 < np; k1 += kUnroll) {
        double add[kUnroll][kAsmGE];
        bool in[kUnroll][kAsmGE];
#pragma unroll
        for (int x = 0; x < kUnroll; x++) {
          const int kk = k1 + x;
          const int a = kk < np ? rmap[kk][i] : -1;
          const double* __restrict__ Fch = c.F + (kk < np ? pbase[kk] : 0) + a;
#pragma unroll
          for (int u = 0; u < kAsmGE; u++) {
            const int b = a >= 0 ? cmap[kk][cg + 4 * (kAsmGE * g + u)] : -1;
            in[x][u] = b >= 0 && b <= a;
            add[x][u] = in[x][u] ? Fch[coff[kk][cg + 4 * (kAsmGE * g + u)]] : 0.0;
          }
        }
#pragma unroll
        for (int x = 0; x < kUnroll; x++)
#pragma unroll
          for (int u = 0; u < kAsmGE; u++)
            if (in[x][u]) val[u] += add[x][u];
      }
#pragma unroll
      for (int u = 0; u < kAsmGE; u++) {
        const int j = cg + 4 * (kAsmGE * g + u), col = C0 + j;
        if (row < mp && col < mp && row >= col) Fp[row + (size_t)j * ldp] = val[u];
      }
    }
  }
}

// The previous form of the same assembly (scatter into an LDS tile, two barriers
// per child rectangle), bitwise the same tile: PGO_ASM_PUSH=1 selects it (A/B)
__global__ __launch_bounds__(256) void k_assemble_tile_push(CholDev c, const int4* __restrict__ tasks,
                                                       const int2* __restrict__ iptr, const int* __restrict__ items,
                                                       const int4* __restrict__ pairs, const double* __restrict__ V,
                                                       const double* __restrict__ D,
                                                       const double* __restrict__ lam_p) {
  lane_offset(c);
  __shared__ double T[64 * 65];
  __shared__ int prow[64], pcol[64];
  __shared__ long long ucol[64];   // the child's update-matrix columns: offset of (wc, wc + b0 + q) in its front
  const int4 t = tasks[blockIdx.x];
  const int p = t.x, mp = c.m[p];
  const int R0 = 64 * (t.y >> 16), C0 = 64 * (t.y & 0xffff);
  const int tid = threadIdx.x, r = tid & 63, cg = tid >> 6;
  const double lam = lam_p[blockIdx.y];
#pragma unroll
  for (int u = 0; u < 16; u++) T[(tid & 63) + ((tid >> 6) + 4 * u) * 65] = 0.0;
  __syncthreads();
  const int2 it = iptr[blockIdx.x];
  for (int q = tid; q < it.y; q += 256) {
    const int code = items[it.x + q];
    if (code >= 0) {
      double acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
      for (int k = c.asm_ptr[code]; k < c.asm_ptr[code + 1]; k++) {
        const double* v = V + 9 * (size_t)c.asm_src[k];   // element e at v[e]
#pragma unroll
        for (int e = 0; e < 9; e++) acc[e] += v[e];
      }
      const int i0 = 3 * c.asm_li[code] - R0, j0 = 3 * c.asm_lj[code] - C0;
#pragma unroll
      for (int a = 0; a < 3; a++)
#pragma unroll
        for (int b = 0; b < 3; b++)
          if (i0 + a >= 0 && i0 + a < 64 && j0 + b >= 0 && j0 + b < 64) T[(i0 + a) + (j0 + b) * 65] = acc[3 * a + b];
    } else {
      const int j = ~code;
      const double* d = D + 6 * (size_t)c.perm[j];
      const int o = 3 * c.dg_loc[j];
      const double dv[6] = {d[0] + lam, d[1], d[2], d[3] + lam, d[4], d[5] + lam};   // (0,0) (1,0) (2,0) (1,1) (2,1) (2,2)
      const int ia[6] = {0, 1, 2, 1, 2, 2}, ib[6] = {0, 0, 0, 1, 1, 2};
#pragma unroll
      for (int e = 0; e < 6; e++) {
        const int i = o + ia[e] - R0, jj = o + ib[e] - C0;
        if (i >= 0 && i < 64 && jj >= 0 && jj < 64) T[i + jj * 65] = dv[e];
      }
    }
  }
  for (int k = 0; k < t.w; k++) {
    const int4 q = pairs[t.z + k];
    const int ch = q.x, a0 = q.y, b0 = q.z, nr = q.w & 0xff, nc = q.w >> 8;
    const int mc = c.m[ch], wc = c.w[ch];
    const int* __restrict__ rel = c.ea_rel + c.ea_ptr[ch];
    __syncthreads();   // the H entries / the previous child's adds are done, prow / pcol reusable
    if (tid < nr) {
      const int a = a0 + tid;
      prow[tid] = 3 * rel[a / 3] + a % 3 - R0;
    } else if (tid >= 64 && tid - 64 < nc) {
      const int b = b0 + tid - 64;
      pcol[tid - 64] = (3 * rel[b / 3] + b % 3 - C0) * 65;
    } else if (tid >= 128 && tid - 128 < nc) {
      ucol[tid - 128] = fcol_off(mc, front_packed(mc, wc), wc + b0 + tid - 128) + wc;
    }
    __syncthreads();
    if (r >= nr) continue;
    const int a = a0 + r;
    const double* __restrict__ Fch = c.F + c.foff[ch] + a;
    constexpr int R = 16;
    double v[R];
#pragma unroll
    for (int j = 0; j < R; j++) {
      const int bb = cg + 4 * j;
      v[j] = (bb < nc && b0 + bb <= a) ? Fch[ucol[bb]] : 0.0;
    }
    const int pr = prow[r];
#pragma unroll
    for (int j = 0; j < R; j++) {
      const int bb = cg + 4 * j;
      if (bb < nc && b0 + bb <= a) T[pr + pcol[bb]] += v[j];
    }
  }
  __syncthreads();
  const bool pkp = front_packed(mp, c.w[p]);
  double* __restrict__ Fp = fcol(c.F + c.foff[p], mp, pkp, C0);   // the tile's columns: one column block
  const int ldp = fld(mp, pkp, C0);
#pragma unroll
  for (int u = 0; u < 16; u++) {
    const int i = tid & 63, j = (tid >> 6) + 4 * u, row = R0 + i, col = C0 + j;
    if (row < mp && col < mp && row >= col) Fp[row + (size_t)j * ldp] = T[i + j * 65];
  }
}

// ------------------------------------------------------------ triangular inverse
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, lane);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ double rsqrt_nr(double d) {   // 1/sqrt(d), two Newton steps from v_rsq_f64
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d * y, y, 1.5);
  y = y * fma(-0.5 * d * y, y, 1.5);
  return y;
}

// X = L^-1 of an LDS-resident lower-triangular nbk x nbk block (element (r,c) at
// L[r + c*ld]), by the 4 waves of a workgroup: wave wv owns columns 16wv..16wv+15,
// lane i row i; column-oriented substitution, row k broadcast with v_readlane
// (no LDS round trip on the dependency chain).  dinv: LDS scratch of 64.
// Written row-major to M (M[a*64 + b] = X[a][b]), zero outside nbk x nbk.
__device__ __forceinline__ void tri_inverse_wg(const double* L, int ld, int nbk, double* __restrict__ M,
                                               double* dinv) {
  const int tid = threadIdx.x;
  if (tid < 64) dinv[tid] = tid < nbk ? 1.0 / L[tid + tid * ld] : 1.0;
  __syncthreads();
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6), i = tid & 63;
  const int j0 = 16 * wv;
  double xr[16];
#pragma unroll
  for (int q = 0; q < 16; q++) xr[q] = (i == j0 + q) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < 64; k++) {
    if (k < j0 || k >= nbk) continue;     // wave-uniform
    const double dk = dinv[k];
    const double lik = (i > k && i < nbk) ? L[i + k * ld] : 0.0;
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const double b = readlane_f64(xr[q], k) * dk;
      xr[q] = (i == k) ? b : fma(-lik, b, xr[q]);
    }
  }
#pragma unroll
  for (int q = 0; q < 16; q++) M[i * 64 + j0 + q] = (i < nbk && j0 + q < nbk) ? xr[q] : 0.0;
  __syncthreads();  // dinv reusable
}

// dst[0..n) = src[0..n) with 8 loads per thread in flight (a plain copy loop
// would wait on every global load before its LDS store)
__device__ __forceinline__ void copy_in(double* __restrict__ dst, const double* __restrict__ src, int n, int t,
                                        int nt) {
  for (int base = t; base < n; base += 8 * nt) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int idx = base + q * nt;
      v[q] = idx < n ? src[idx] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int idx = base + q * nt;
      if (idx < n) dst[idx] = v[q];
    }
  }
}

// 8x8 lower triangle packed row by row
#define P8(i, j) ((i) * ((i) + 1) / 2 + (j))

// Cholesky factor of an 8x8 SPD block held whole, the same values, in every
// lane: the pivot chain (rsqrt, scale, rank-1 update of the next diagonal) runs
// in registers with no cross-lane traffic.  a: lower, packed; iv[j] = 1 / L_jj.
__device__ __forceinline__ bool chol8_lane(double (&a)[36], double (&iv)[8]) {
  bool bad = false;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    double d = a[P8(j, j)];
    if (!(d > 0.0) || !isfinite(d)) {
      bad = true;
      d = 1.0;
    }
    const double inv = rsqrt_nr(d);
    iv[j] = inv;
    a[P8(j, j)] = d * inv;
#pragma unroll
    for (int i = j + 1; i < 8; i++) a[P8(i, j)] *= inv;
#pragma unroll
    for (int i = j + 1; i < 8; i++)
#pragma unroll
      for (int k = j + 1; k <= i; k++) a[P8(i, k)] = fma(-a[P8(i, j)], a[P8(k, j)], a[P8(i, k)]);
  }
  return bad;
}

// ------------------------------------------------------------ small fronts (LDS)
// m <= 128: the whole front in LDS; right-looking, two threads per row (the
// row's columns split even/odd) so LDS accesses of a wave are consecutive rows.
__global__ __launch_bounds__(256) void k_front_small(CholDev c, const int* __restrict__ list) {
  lane_offset(c);
  extern __shared__ __attribute__((aligned(16))) double A[];   // m*m front, 64 scratch, m frontal vector
  const int s = list[blockIdx.x];
  const int m = c.m[s], w = c.w[s];
  double* Fs = c.F + c.foff[s];
  double* fv = c.fv + c.voff[s];
  double* v = A + m * m + 64;
  const int tid = threadIdx.x;
  copy_in(A, Fs, m * m, tid, 256);   // (the upper triangle comes along; never read)
  copy_in(v, fv, m, tid, 256);
  __syncthreads();
  // the frontal vector is carried as an extra column: forward substitution
  // L y = v for the pivot rows and v_below -= L21 y, in the same sweep
  const int half = tid >> 7, rsub = tid & 127;
  for (int k = 0; k < w; k++) {
    double d = A[k + k * m];
    if (!(d > 0.0) || !isfinite(d)) {
      *c.flag = 1;
      d = 1.0;
    }
    const double piv = sqrt(d);
    __syncthreads();  // every thread has read the pivot before it is overwritten
    const double inv = 1.0 / piv;
    if (tid == 0) {
      A[k + k * m] = piv;
      v[k] *= inv;
    }
    for (int i = k + 1 + tid; i < m; i += 256) A[i + k * m] *= inv;
    __syncthreads();
    const double vk = v[k];
    for (int i = k + 1 + rsub; i < m; i += 128) {
      const double lik = A[i + k * m];
      if (half == 0) v[i] -= lik * vk;
      for (int j = k + 1 + half; j <= i; j += 2) A[i + j * m] -= lik * A[j + k * m];
    }
    __syncthreads();
  }
  for (int j = 0; j < m; j++)
    for (int i = j + tid; i < m; i += 256) Fs[i + (size_t)j * m] = A[i + j * m];
  for (int i = tid; i < m; i += 256) fv[i] = v[i];
  // inverses of the 64-column diagonal blocks (used by the backward solve)
  double* scratch = A + m * m;
  for (int jb = 0; jb < w; jb += 64)
    tri_inverse_wg(A + jb + jb * m, m, min(64, w - jb), c.Tinv + c.toff[s] + (jb / 64) * 4096, scratch);
}

// Small front with w <= kWaveW pivot columns (and m <= 128), one wavefront:
// lane l owns rows l and l + 64 of the m x w panel in registers; per pivot k the
// panel's column k is published through LDS (one store per lane, broadcast
// reads, no read-modify-write of LDS), so the pivot chain costs one LDS round
// trip and one rsqrt.  The frontal vector rides along (forward substitution).
// Then the rank-w Schur update of the trailing block is streamed through global
// memory (rows of L from registers, columns broadcast from an LDS copy), and
// the w x w inverse for the backward solve is formed lane = column.
// W: the compile-time panel width (8, 16 or kWaveW >= w): the pivot loop, the
// per-pivot column updates and the trailing update's inner products run over W,
// so narrow fronts (most leaves) do a quarter of the wide ones' work.
#ifndef PGO_WAVE_PERPIVOT_W
#define PGO_WAVE_PERPIVOT_W 16   // widest class factored one pivot at a time (scripts/ubench_wave.hip A/B)
#endif
template <int W, bool kTwoRows>   // m > 64: lane also owns row l + 64
__device__ __forceinline__ void front_wave_body(const CholDev& c, int s, double* S) {
  constexpr int LDP = W + 1;   // odd row stride: conflict-free per-lane rows
  const int m = c.m[s], w = c.w[s];
  double* PR = S;                 // m x W row-major copy of L (after the factorisation)
  double* cb = S + m * LDP;       // 128 + 2: column k of the panel, then v[k]; then 1/L(k,k)
  double* Fs = c.F + c.foff[s];
  double* fv = c.fv + c.voff[s];
  const int l = threadIdx.x, lb = l + 64;
  const bool ra = l < m, rb = kTwoRows && lb < m;
  DIAG_CLK(23);
  double* invs = cb + 130;        // [W] 1 / L(k,k)
  double pa[W], pb[W];
#pragma unroll
  for (int k = 0; k < W; k++) {
    pa[k] = (ra && k < w && k <= l) ? Fs[l + (size_t)k * m] : 0.0;
    pb[k] = (rb && k < w) ? Fs[lb + (size_t)k * m] : 0.0;
  }
  double va = ra ? fv[l] : 0.0, vb = rb ? fv[lb] : 0.0;
  bool bad = false;
  DIAG_CLK(24);
  if constexpr (W <= PGO_WAVE_PERPIVOT_W) {
    // (the narrow classes, most leaves: one pivot at a time.  The blocked form
    // below needs ~210 VGPRs at W = 16 -- 2 waves per SIMD instead of 4 -- and
    // measured 33-38 % slower on 4096 fronts of m = 64, w = 12 / 16, 9 % on
    // m = 90, w = 12; it pays at W = 32: m = 100, w = 24 9 % faster;
    // profiles/r04c_front_wave_ubench_blocked.txt)
    // pivot k: column k of the panel is lane j's pa[k] (rows j < W <= 64), read
    // with v_readlane (no LDS round trip on the pivot chain)
  #pragma unroll
    for (int k = 0; k < W; k++) {
      if (k < w) {                              // uniform
        double d = readlane_f64(pa[k], k);
        const double vk = readlane_f64(va, k);
        if (!(d > 0.0) || !isfinite(d)) {
          bad = true;
          d = 1.0;
        }
        const double r = rsqrt_nr(d);
        const double yk = vk * r;
        const double la = l > k ? pa[k] * r : (l == k ? d * r : pa[k]);
        const double lbv = pb[k] * r;
        // columns j >= w (the class width W past the front's w) are updated
        // with a zero multiplier -- fma(x, 0, y) == y exactly, so they stay zero
        // -- instead of a branch per column: the per-(k, j) branches compiled to
        // ~500 out-of-line blocks, a 16k-line kernel thrashing the instruction
        // cache on the pivot chain
        const double rj = r;
  #pragma unroll
        for (int j = k + 1; j < W; j++) {
          const double lj = readlane_f64(pa[k], j) * (j < w ? rj : 0.0);
          pa[j] = fma(l >= j ? -la : 0.0, lj, pa[j]);
          pb[j] = fma(-lbv, lj, pb[j]);
        }
        pa[k] = la;
        pb[k] = lbv;
        va = l == k ? yk : (l > k ? fma(-la, yk, va) : va);
        vb = fma(-lbv, yk, vb);
        if (l == 0) invs[k] = r;
      }
    }
  } else {
    // pivots in blocks of 8 columns kb .. kb + 7 (right-looking): the block's
    // diagonal 8x8 (rows kb .. kb + 7, lanes kb ..) and their v go through LDS
    // once, every lane factors it in registers (chol8_lane: no cross-lane
    // traffic on the pivot chain) and forms y; each lane then solves its own
    // rows' L(row, kb ..) against it; the panel columns right of the block get
    // the block's rank-8 update with the block's L rows read back from LDS as
    // broadcasts.  Every element sees the same fma's in the same order as the
    // one-pivot-at-a-time sweep (fma(-L(row, k), L(col, k), a) per pivot k in
    // increasing k; L(row, k) = a * 1/L(k, k); y likewise): bitwise its result.
    double* db = cb;                // 8 x 9: the diagonal block's rows and their v
    double* lrb = PR;               // (W - 8) x 8: L rows of the columns right of the block
    // (no data-dependent loop exits: pivots past w are identity pivots on zero
    // columns -- fma(-0, x, a) == a, the zero columns stay zero -- so every loop
    // unrolls with static register indices; only whole 8-blocks past w are skipped)
  #pragma unroll
    for (int kb = 0; kb < W; kb += 8) {
      if (kb < w) {                 // uniform
        const int nb8 = min(8, w - kb);
        if (l >= kb && l < kb + nb8) {
  #pragma unroll
          for (int q = 0; q < 8; q++) db[(l - kb) * 9 + q] = pa[kb + q];
          db[(l - kb) * 9 + 8] = va;
        }
        __builtin_amdgcn_wave_barrier();
        double a[36], iv[8], y[8];
  #pragma unroll
        for (int i = 0; i < 8; i++) {
  #pragma unroll
          for (int j = 0; j <= i; j++) a[P8(i, j)] = i < nb8 ? db[i * 9 + j] : (i == j ? 1.0 : 0.0);
          y[i] = i < nb8 ? db[i * 9 + 8] : 0.0;
        }
        __builtin_amdgcn_wave_barrier();   // (db is rewritten by the next block)
        bad = chol8_lane(a, iv) || bad;    // (padded pivots: 1, so L = I there)
  #pragma unroll
        for (int q = 0; q < 8; q++) {
          y[q] *= iv[q];
  #pragma unroll
          for (int i = q + 1; i < 8; i++) y[i] = fma(-a[P8(i, q)], y[q], y[i]);
        }
        if (l == 0)
  #pragma unroll
          for (int q = 0; q < 8; q++) invs[kb + q] = iv[q];   // (past w: never read)
        const bool own = l >= kb && l < kb + nb8, below = l >= kb + nb8;
        if (own) {                       // the block's own rows: L and y (static register indices)
  #pragma unroll
          for (int i = 0; i < 8; i++)
            if (i == l - kb) {
  #pragma unroll
              for (int q = 0; q <= i; q++) pa[kb + q] = a[P8(i, q)];
              va = y[i];
            }
        }
  #pragma unroll
        for (int q = 0; q < 8; q++) {    // rows below: L(row, kb + q) against the block, then v
  #pragma unroll
          for (int t = 0; t < q; t++) {
            if (below) pa[kb + q] = fma(-pa[kb + t], a[P8(q, t)], pa[kb + q]);
            pb[kb + q] = fma(-pb[kb + t], a[P8(q, t)], pb[kb + q]);   // (rows l + 64: always below)
          }
          if (below) pa[kb + q] *= iv[q];
          pb[kb + q] *= iv[q];
        }
  #pragma unroll
        for (int q = 0; q < 8; q++) {
          if (below) va = fma(-pa[kb + q], y[q], va);
          vb = fma(-pb[kb + q], y[q], vb);
        }
        // columns right of the block: rank-8 update with L(col, kb ..) from the
        // lanes holding those rows (rows past w: zero)
        if (kb + 8 < W && kb + 8 < w) {  // uniform
          if (l >= kb + 8 && l < W)
  #pragma unroll
            for (int q = 0; q < 8; q++) lrb[(l - kb - 8) * 8 + q] = l < w ? pa[kb + q] : 0.0;
          __builtin_amdgcn_wave_barrier();
  #pragma unroll
          for (int j = kb + 8; j < W; j++) {
            const double2* lj2 = reinterpret_cast<const double2*>(lrb + (j - kb - 8) * 8);
  #pragma unroll
            for (int q2 = 0; q2 < 4; q2++) {
              const double2 t2 = lj2[q2];
              pa[j] = fma(l >= j ? -pa[kb + 2 * q2] : 0.0, t2.x, pa[j]);
              pb[j] = fma(-pb[kb + 2 * q2], t2.x, pb[j]);
              pa[j] = fma(l >= j ? -pa[kb + 2 * q2 + 1] : 0.0, t2.y, pa[j]);
              pb[j] = fma(-pb[kb + 2 * q2 + 1], t2.y, pb[j]);
            }
          }
          __builtin_amdgcn_wave_barrier();   // (lrb is rewritten by the next block)
        }
      }
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (bad && l == 0) *c.flag = 1;
  DIAG_CLK(25);
  if constexpr (kTwoRows) {
    // m > 64 (up to 8 column blocks of the trailing update below): the first
    // block's C loads issued before the panel's stores and the inverse, each
    // next block's before this one's products (the blocks touch disjoint
    // columns, none of the panel's): latency per front 12-16 % lower on 1 - 256
    // fronts of m = 100, w = 8 / 16, bitwise the same fronts
    // (profiles/r05u_front_wave_ahead.txt)
    constexpr int NT = 8;   // tiles per column block (m <= 128)
    const int u = m - w, nt = (u + 15) >> 4, li = l & 15, lk = l >> 4;
    auto load_c = [&](int tj, double (&cv)[NT][4]) {
      const int j0 = w + 16 * tj;
#pragma unroll
      for (int q = 0; q < NT; q++) {
        const int i = w + 16 * (tj + q) + li;
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int j = j0 + lk + 4 * r;
          cv[q][r] = (tj + q < nt && i < m && j <= i) ? Fs[i + (size_t)j * m] : 0.0;
        }
      }
    };
    auto update = [&](int tj, const double (&cv)[NT][4]) {   // as the m <= 64 branch's
      const int j0 = w + 16 * tj;
      const double* Aj = PR + min(j0 + li, m - 1) * LDP + lk;
      double a[W / 4];
#pragma unroll
      for (int kc = 0; kc < W / 4; kc++) a[kc] = Aj[4 * kc];
#pragma unroll
      for (int q = 0; q < NT; q++) {
        if (tj + q >= nt) break;   // uniform
        const int i = w + 16 * (tj + q) + li;
        const double* Bi = PR + min(i, m - 1) * LDP + lk;
        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kc = 0; kc < W / 4; kc++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kc], Bi[4 * kc], acc, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; r++) {
          const int j = j0 + lk + 4 * r;
          if (i < m && j <= i) Fs[i + (size_t)j * m] = cv[q][r] - acc[r];
        }
      }
    };
    double c0[NT][4], c1[NT][4];
    if (nt > 0) load_c(0, c0);
    // L back to the front (and a row-major LDS copy), y to the frontal vector
#pragma unroll
    for (int k = 0; k < W; k++) {
      if (k < w) {
        if (ra && k <= l) Fs[l + (size_t)k * m] = pa[k];
        if (rb) Fs[lb + (size_t)k * m] = pb[k];
      }
      if (ra) PR[l * LDP + k] = k <= l ? pa[k] : 0.0;
      if (rb) PR[lb * LDP + k] = pb[k];
    }
    if (ra) fv[l] = va;
    if (rb) fv[lb] = vb;
    __builtin_amdgcn_wave_barrier();
    DIAG_CLK(26);
    // X = L11^-1 (w x w), lane = column: forward substitution of e_l
    if (l < w) {
      double x[W];
#pragma unroll
      for (int r = 0; r < W; r++) {
        double acc = r == l ? 1.0 : 0.0;
#pragma unroll
        for (int t = 0; t < r; t++) acc = fma(-PR[min(r, m - 1) * LDP + t], x[t], acc);
        x[r] = r < w ? acc * invs[r] : 0.0;
      }
      double* M = c.Tinv + c.toff[s];   // row-major, live w x w
#pragma unroll
      for (int r = 0; r < W; r++)
        if (r < w) M[r * 64 + l] = r >= l ? x[r] : 0.0;
    }
    DIAG_CLK(27);
    for (int tj = 0; tj < nt; tj += 2) {   // (the trailing update: see the m <= 64 branch)
      if (tj + 1 < nt) load_c(tj + 1, c1);
      update(tj, c0);
      if (tj + 1 >= nt) break;
      if (tj + 2 < nt) load_c(tj + 2, c0);
      update(tj + 1, c1);
    }
  } else {
    // m <= 64 (<= 4 blocks; the one-block-ahead form cost the leaves'
    // 12288-front launch 4-5 % and saved < 0.5 us of latency)
    // L back to the front (and a row-major LDS copy), y to the frontal vector
#pragma unroll
    for (int k = 0; k < W; k++) {   // (columns k >= w of the LDS copy are zero)
      if (k < w) {
        if (ra && k <= l) Fs[l + (size_t)k * m] = pa[k];
        if (rb) Fs[lb + (size_t)k * m] = pb[k];
      }
      if (ra) PR[l * LDP + k] = k <= l ? pa[k] : 0.0;
      if (rb) PR[lb * LDP + k] = pb[k];
    }
    if (ra) fv[l] = va;
    if (rb) fv[lb] = vb;
    __builtin_amdgcn_wave_barrier();
    DIAG_CLK(26);
    // trailing update C[i][j] -= L[i,:] L[j,:]', w <= j <= i < m, on
    // v_mfma_f64_16x16x4f64: per 16 x 16 lower tile D(jj, ii) = sum_k L[j0 + jj][k]
    // L[i0 + ii][k] with both operands from the row-major LDS copy (zero beyond
    // w); lane l holds rows i0 + (l & 15) of columns j0 + (l >> 4) + 4 r, so each
    // column's 16 rows are one coalesced segment of the front.  A 16-column block
    // at a time: all its tiles' loads in flight together (m <= 128: <= 8 tiles).
    {
      constexpr int NT = kTwoRows ? 8 : 4;   // tiles per column block (m <= 128 | 64)
      const int u = m - w, nt = (u + 15) >> 4, li = l & 15, lk = l >> 4;
      for (int tj = 0; tj < nt; tj++) {
        const int j0 = w + 16 * tj;
        const double* Aj = PR + min(j0 + li, m - 1) * LDP + lk;
        double a[W / 4];
#pragma unroll
        for (int kc = 0; kc < W / 4; kc++) a[kc] = Aj[4 * kc];
        double cv[NT][4];
#pragma unroll
        for (int q = 0; q < NT; q++) {
          const int i = w + 16 * (tj + q) + li;
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int j = j0 + lk + 4 * r;
            cv[q][r] = (tj + q < nt && i < m && j <= i) ? Fs[i + (size_t)j * m] : 0.0;
          }
        }
#pragma unroll
        for (int q = 0; q < NT; q++) {
          if (tj + q >= nt) break;   // uniform
          const int i = w + 16 * (tj + q) + li;
          const double* Bi = PR + min(i, m - 1) * LDP + lk;
          d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kc = 0; kc < W / 4; kc++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kc], Bi[4 * kc], acc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int j = j0 + lk + 4 * r;
            if (i < m && j <= i) Fs[i + (size_t)j * m] = cv[q][r] - acc[r];
          }
        }
      }
    }
    DIAG_CLK(27);
    // X = L11^-1 (w x w), lane = column: forward substitution of e_l
    if (l < w) {
      double x[W];
#pragma unroll
      for (int r = 0; r < W; r++) {
        double acc = r == l ? 1.0 : 0.0;
#pragma unroll
        for (int t = 0; t < r; t++) acc = fma(-PR[min(r, m - 1) * LDP + t], x[t], acc);
        x[r] = r < w ? acc * invs[r] : 0.0;
      }
      double* M = c.Tinv + c.toff[s];   // row-major, live w x w
#pragma unroll
      for (int r = 0; r < W; r++)
        if (r < w) M[r * 64 + l] = r >= l ? x[r] : 0.0;
    }
  }
  DIAG_CLK(28);
}

// Small front with 64 < m <= 64 NW rows and w <= W (16 or 32) pivot columns,
// by NW wavefronts: wave q holds rows [64 q, 64 q + 64) of the m x w panel in
// registers (thread t: row t) -- half the registers of one wave holding two
// rows per lane -- and the trailing update's 16-column blocks are dealt to the
// waves.  The pivot steps are front_wave_body's blocked form, with workgroup
// barriers where its LDS hand-offs cross the waves; every element sees the
// same fma's in the same order: bitwise front_wave_body's front.  NW = 4
// (round 4): 128 < m <= 256, fronts stored packed (pgo_chol.h front_packed:
// the panel's columns lie in the first 64-column block, the trailing columns
// are addressed by their block), which the blocked path took before.
template <int W, int NW = 2>
__device__ __forceinline__ void front_wave2_body(const CholDev& c, int s, double* S) {
  constexpr int LDP = W + 1;
  const int m = c.m[s], w = c.w[s];
  const bool pk = front_packed(m, w);
  const int ld0 = fld(m, pk, 0);  // the panel's columns (the first column block when packed)
  double* PR = S;                 // m x W row-major copy of L (after the factorisation)
  double* cb = S + m * LDP;       // the diagonal block's rows and v (8 x 9)
  double* invs = cb + 130;        // [W] 1 / L(k,k)
  double* Fs = c.F + c.foff[s];
  double* fv = c.fv + c.voff[s];
  const int row = threadIdx.x, l = row & 63, wq = row >> 6;
  const bool ra = row < m;
  DIAG_CLK(23);
  double pa[W];
#pragma unroll
  for (int k = 0; k < W; k++) pa[k] = (ra && k < w && k <= row) ? Fs[row + (size_t)k * ld0] : 0.0;
  double va = ra ? fv[row] : 0.0;
  bool bad = false;
  DIAG_CLK(24);
  double* db = cb;
  double* lrb = PR;               // (W - 8) x 8: L rows of the columns right of the block
#pragma unroll
  for (int kb = 0; kb < W; kb += 8) {
    if (kb < w) {                 // uniform
      const int nb8 = min(8, w - kb);
      if (row >= kb && row < kb + nb8) {
#pragma unroll
        for (int q = 0; q < 8; q++) db[(row - kb) * 9 + q] = pa[kb + q];
        db[(row - kb) * 9 + 8] = va;
      }
      __syncthreads();
      double a[36], iv[8], y[8];
#pragma unroll
      for (int i = 0; i < 8; i++) {
#pragma unroll
        for (int j = 0; j <= i; j++) a[P8(i, j)] = i < nb8 ? db[i * 9 + j] : (i == j ? 1.0 : 0.0);
        y[i] = i < nb8 ? db[i * 9 + 8] : 0.0;
      }
      bad = chol8_lane(a, iv) || bad;
#pragma unroll
      for (int q = 0; q < 8; q++) {
        y[q] *= iv[q];
#pragma unroll
        for (int i = q + 1; i < 8; i++) y[i] = fma(-a[P8(i, q)], y[q], y[i]);
      }
      if (row == 0)
#pragma unroll
        for (int q = 0; q < 8; q++) invs[kb + q] = iv[q];
      const bool own = row >= kb && row < kb + nb8, below = row >= kb + nb8;
      if (own) {
#pragma unroll
        for (int i = 0; i < 8; i++)
          if (i == row - kb) {
#pragma unroll
            for (int q = 0; q <= i; q++) pa[kb + q] = a[P8(i, q)];
            va = y[i];
          }
      }
#pragma unroll
      for (int q = 0; q < 8; q++) {
#pragma unroll
        for (int t = 0; t < q; t++)
          if (below) pa[kb + q] = fma(-pa[kb + t], a[P8(q, t)], pa[kb + q]);
        if (below) pa[kb + q] *= iv[q];
      }
#pragma unroll
      for (int q = 0; q < 8; q++)
        if (below) va = fma(-pa[kb + q], y[q], va);
      const bool right = kb + 8 < W && kb + 8 < w;   // uniform
      if (right && row >= kb + 8 && row < W)
#pragma unroll
        for (int q = 0; q < 8; q++) lrb[(row - kb - 8) * 8 + q] = row < w ? pa[kb + q] : 0.0;
      __syncthreads();            // lrb written; every db read done before the next block's
      if (right) {
#pragma unroll
        for (int j = kb + 8; j < W; j++) {
          const double2* lj2 = reinterpret_cast<const double2*>(lrb + (j - kb - 8) * 8);
#pragma unroll
          for (int q2 = 0; q2 < 4; q2++) {
            const double2 t2 = lj2[q2];
            pa[j] = fma(row >= j ? -pa[kb + 2 * q2] : 0.0, t2.x, pa[j]);
            pa[j] = fma(row >= j ? -pa[kb + 2 * q2 + 1] : 0.0, t2.y, pa[j]);
          }
        }
      }
      __syncthreads();            // lrb read before the next block rewrites it (or PR below)
    }
  }
  if (bad && row == 0) *c.flag = 1;
  DIAG_CLK(25);
  // L back to the front (and the row-major LDS copy), y to the frontal vector
#pragma unroll
  for (int k = 0; k < W; k++) {
    if (ra && k < w && k <= row) Fs[row + (size_t)k * ld0] = pa[k];
    if (ra) PR[row * LDP + k] = k <= row ? pa[k] : 0.0;
  }
  if (ra) fv[row] = va;
  __syncthreads();
  DIAG_CLK(26);
  // X = L11^-1 (w x w), lane = column, by the last wave ahead of its share of
  // the trailing update (blocks tj = wq, wq + NW, ..: the last wave's share is
  // the smallest); wave 0 did it after its larger share before
  if (wq == NW - 1 && l < w) {
    double x[W];
#pragma unroll
    for (int r = 0; r < W; r++) {
      double acc = r == l ? 1.0 : 0.0;
#pragma unroll
      for (int t = 0; t < r; t++) acc = fma(-PR[min(r, m - 1) * LDP + t], x[t], acc);
      x[r] = r < w ? acc * invs[r] : 0.0;
    }
    double* M = c.Tinv + c.toff[s];   // row-major, live w x w
#pragma unroll
    for (int r = 0; r < W; r++)
      if (r < w) M[r * 64 + l] = r >= l ? x[r] : 0.0;
  }
  DIAG_CLK(27);
  {   // trailing update C[i][j] -= L[i,:] L[j,:]' as front_wave_body's, 16-column blocks dealt to the
      // waves, their row tiles 8 at a time
    const int u = m - w, nt = (u + 15) >> 4, li = l & 15, lk = l >> 4;
    for (int tj = wq; tj < nt; tj += NW) {
      const int j0 = w + 16 * tj;
      const double* Aj = PR + min(j0 + li, m - 1) * LDP + lk;
      double a[W / 4];
#pragma unroll
      for (int kc = 0; kc < W / 4; kc++) a[kc] = Aj[4 * kc];
      double* colp[4];   // this lane's 4 columns (packed fronts: each in its own 64-column block)
#pragma unroll
      for (int r = 0; r < 4; r++) colp[r] = Fs + fcol_off(m, pk, min(j0 + lk + 4 * r, m - 1));
      for (int qb = 0; tj + qb < nt; qb += 8) {
        double cv[8][4];
#pragma unroll
        for (int q = 0; q < 8; q++) {
          const int i = w + 16 * (tj + qb + q) + li;
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int j = j0 + lk + 4 * r;
            cv[q][r] = (tj + qb + q < nt && i < m && j <= i) ? colp[r][i] : 0.0;
          }
        }
#pragma unroll
        for (int q = 0; q < 8; q++) {
          if (tj + qb + q >= nt) break;   // uniform
          const int i = w + 16 * (tj + qb + q) + li;
          const double* Bi = PR + min(i, m - 1) * LDP + lk;
          d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kc = 0; kc < W / 4; kc++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kc], Bi[4 * kc], acc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const int j = j0 + lk + 4 * r;
            if (i < m && j <= i) colp[r][i] = cv[q][r] - acc[r];
          }
        }
      }
    }
  }
  DIAG_CLK(28);
}

template <int W>
__global__ __launch_bounds__(128) void k_front_wave2(CholDev c, const int* __restrict__ list) {
  lane_offset(c);
  extern __shared__ __attribute__((aligned(16))) double S[];
  front_wave2_body<W, 2>(c, list[blockIdx.x], S);
}
template <int W>
__global__ __launch_bounds__(256) void k_front_wave4(CholDev c, const int* __restrict__ list) {
  lane_offset(c);
  extern __shared__ __attribute__((aligned(16))) double S[];
  front_wave2_body<W, 4>(c, list[blockIdx.x], S);
}

template <int W, bool kTwoRows>
__global__ __launch_bounds__(64) void k_front_wave(CholDev c, const int* __restrict__ list) {
  lane_offset(c);
  extern __shared__ __attribute__((aligned(16))) double S[];
  front_wave_body<W, kTwoRows>(c, list[blockIdx.x], S);
}

// ------------------------------------------------------------ blocked path
// ------------------------------------------------------------ diagonal tile

// 16x16x16 product on one wave from LDS: D(i,j) = sum_k A(i,k) B(k,j),
// A(i,k) = A[i*ars + k*acs], B(k,j) = B[k*brs + j*bcs]; D in the f64 MFMA
// layout (lane l, reg r -> row (l>>4)+4r, col l&15).
__device__ __forceinline__ d4 mm16(const double* A, int ars, int acs, const double* B, int brs, int bcs) {
  const int l = threadIdx.x & 63, i = l & 15, kq = l >> 4;
  double a[4], b[4];
#pragma unroll
  for (int t = 0; t < 4; t++) {
    a[t] = A[i * ars + (4 * t + kq) * acs];
    b[t] = B[(4 * t + kq) * brs + i * bcs];
  }
  d4 acc = {0, 0, 0, 0};
#pragma unroll
  for (int t = 0; t < 4; t++) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t], b[t], acc, 0, 0, 0);
  return acc;
}

// C(16x16, ld 65) op= D
__device__ __forceinline__ void st16(double* C, d4 v, bool sub) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 4; r++) {
    double* p = C + ((l >> 4) + 4 * r) + (l & 15) * 65;
    *p = sub ? *p - v[r] : v[r];
  }
}

// In place L -> L^-1 (8x8 lower, packed), columns right to left:
// X_ij = -(1 / L_jj) sum_{k=j+1..i} X_ik L_kj.
__device__ __forceinline__ void inv8_lane(double (&a)[36], const double (&iv)[8]) {
#pragma unroll
  for (int j = 7; j >= 0; j--) {
#pragma unroll
    for (int i = 7; i > j; i--) {
      double s = 0.0;
#pragma unroll
      for (int k = i; k > j; k--) s = fma(a[P8(i, k)], a[P8(k, j)], s);   // X_i,j+1 (newest) last
      a[P8(i, j)] = -iv[j] * s;
    }
    a[P8(j, j)] = iv[j];
  }
}

// Factor and inverse of the 16x16 diagonal block TJ (LDS, ld 65, lower valid)
// by one wave, as 2x2 blocks of 8: A11 = L11 L11^T and X11 = L11^-1 lane-local
// (chol8_lane, inv8_lane, every lane the same values), L21 = A21 X11^T and
// A22 - L21 L21^T one element per lane, A22' lane-local again, then
// X21 = -X22 (L21 X11).  Writes L21 to TJ (the 8x8 diagonal blocks of L are
// not stored: round 5, nothing reads a diagonal tile's L) and X to WJ (ld 65,
// lower, zeros above); sc: LDS scratch of 64.  Same wave only: LDS accesses of one
// wave complete in order, so no barrier between a lane's store and another's
// load.  (Solving rows of L21 against a lane-held L11 instead, with A22' formed
// in registers, measured slower: 34.4 k against 33.0 k cycles per 64x64.)
__device__ __forceinline__ bool diag16_lane(double* TJ, double* WJ, double* sc) {
  const int l = threadIdx.x & 63, r = l >> 3, c = l & 7;
  double a[36], iv[8];
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) a[P8(i, j)] = TJ[i + j * 65];
  // zeros above the diagonal of X (blocks (0,0), (1,1) upper, (0,1))
  WJ[r + (8 + c) * 65] = 0.0;
  if (c > r) {
    WJ[r + c * 65] = 0.0;
    WJ[(8 + r) + (8 + c) * 65] = 0.0;
  }
  DIAG_CLK(13);
  bool bad = chol8_lane(a, iv);
  DIAG_CLK(14);
  inv8_lane(a, iv);   // (L11 itself is not stored: nothing reads a diagonal block's L, see store_factor)
  DIAG_CLK(15);
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) WJ[i + j * 65] = a[P8(i, j)];
  }
  __builtin_amdgcn_wave_barrier();
  // L21 (r, c) = sum_k A21(r, k) X11(c, k)   (X11 upper is zero)
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) s = fma(TJ[(8 + r) + k * 65], WJ[c + k * 65], s);
  __builtin_amdgcn_wave_barrier();
  TJ[(8 + r) + c * 65] = s;
  __builtin_amdgcn_wave_barrier();
  // A22 (r, c) -= sum_k L21(r, k) L21(c, k), lower part
  double t = TJ[(8 + r) + (8 + c) * 65];
#pragma unroll
  for (int k = 0; k < 8; k++) t = fma(-TJ[(8 + r) + k * 65], TJ[(8 + c) + k * 65], t);
  // Y = L21 X11 (X11 (k, c) zero for k < c)
  double y = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) y = fma(TJ[(8 + r) + k * 65], WJ[k + c * 65], y);
  __builtin_amdgcn_wave_barrier();
  if (c <= r) TJ[(8 + r) + (8 + c) * 65] = t;
  sc[r * 8 + c] = y;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) a[P8(i, j)] = TJ[(8 + i) + (8 + j) * 65];
  DIAG_CLK(16);
  bad = chol8_lane(a, iv) || bad;
  DIAG_CLK(17);
  inv8_lane(a, iv);   // (nor L22)
  if (l == 0) {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j <= i; j++) WJ[(8 + i) + (8 + j) * 65] = a[P8(i, j)];
  }
  __builtin_amdgcn_wave_barrier();
  DIAG_CLK(18);
  // X21 (r, c) = -sum_k X22 (r, k) Y (k, c)   (X22 upper is zero)
  double z = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) z = fma(WJ[(8 + r) + (8 + k) * 65], sc[k * 8 + c], z);
  WJ[(8 + r) + c * 65] = -z;
  DIAG_CLK(19);
  return bad;
}

// x = L^-1 x in place, L an 8x8 lower block held whole in every lane (packed,
// iv[k] = 1 / L_kk): the forward substitution of one right-hand side per lane
__device__ __forceinline__ void fwd8_lane(const double (&a)[36], const double (&iv)[8], double (&x)[8]) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    double s = x[k];
#pragma unroll
    for (int t = 0; t < k; t++) s = fma(-a[P8(k, t)], x[t], s);
    x[k] = s * iv[k];
  }
}

// diag16_lane's factor and inverse with the lane-redundant work cut to the two
// 8x8 factors (round 6).  Every other piece is one forward substitution per
// lane against the lane-held L11 / L22 -- lanes 0-7 one right-hand side e_c
// each (a column of X11 / X22), lanes 8-15 a row of A21 (-> a row of L21) /
// a column of -Y (-> a column of X21 = -X22 Y, Y = L21 X11) -- in the same
// instructions, instead of inv8_lane's lane-redundant inverse and its lane-0
// stores (36 each) and the L21 / X21 products through LDS.  Same outputs as
// diag16_lane (L21 in TJ, X lower in WJ with zeros above); a different
// operation order, so not bitwise its result (the oracle tolerances hold).
__device__ __forceinline__ bool diag16_fs(double* TJ, double* WJ, double* sc) {
  const int l = threadIdx.x & 63, r = l >> 3, c = l & 7;
  double a[36], iv[8], x[8];
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) a[P8(i, j)] = TJ[i + j * 65];
  const bool xl = l < 8, rl = l >= 8 && l < 16;
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = xl ? (k == l ? 1.0 : 0.0) : (rl ? TJ[l + k * 65] : 0.0);   // e_l / row l-8 of A21
  WJ[r + (8 + c) * 65] = 0.0;   // block (0, 1) of X
  DIAG_CLKF(20);
  bool bad = chol8_lane(a, iv);
  DIAG_CLKF(21);
  fwd8_lane(a, iv, x);          // lanes 0-7: column l of X11; lanes 8-15: row l-8 of L21
  if (xl || rl) {
#pragma unroll
    for (int k = 0; k < 8; k++) (xl ? WJ[k + l * 65] : TJ[l + k * 65]) = x[k];
  }
  __builtin_amdgcn_wave_barrier();
  DIAG_CLKF(22);
  // A22 -= L21 L21^T (lower), Y = L21 X11 (X11 (k, c) zero for k < c)
  double t = TJ[(8 + r) + (8 + c) * 65], y = 0.0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const double lrk = TJ[(8 + r) + k * 65];
    t = fma(-lrk, TJ[(8 + c) + k * 65], t);
    y = fma(lrk, WJ[k + c * 65], y);
  }
  __builtin_amdgcn_wave_barrier();
  if (c <= r) TJ[(8 + r) + (8 + c) * 65] = t;
  sc[r * 8 + c] = y;
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int j = 0; j <= i; j++) a[P8(i, j)] = TJ[(8 + i) + (8 + j) * 65];
#pragma unroll
  for (int k = 0; k < 8; k++) x[k] = xl ? (k == l ? 1.0 : 0.0) : (rl ? -sc[k * 8 + (l - 8)] : 0.0);   // e_l / -Y column
  DIAG_CLKF(23);
  bad = chol8_lane(a, iv) || bad;
  DIAG_CLKF(24);
  fwd8_lane(a, iv, x);          // lanes 0-7: column l of X22; lanes 8-15: column l-8 of X21
  if (xl || rl) {
#pragma unroll
    for (int k = 0; k < 8; k++) (xl ? WJ[(8 + k) + (8 + l) * 65] : WJ[(8 + k) + (l - 8) * 65]) = x[k];
  }
  DIAG_CLKF(25);
  return bad;
}

// Cholesky factor L and inverse X = L^-1 of the 64x64 SPD tile T (LDS,
// column-major, ld 65, lower part valid, identity beyond the live size), by the
// 4 waves of the workgroup: right-looking over 16-column blocks J; the 16x16
// diagonal block is factored and inverted by wave 0 (diag16_lane), the rest
// are 16x16x16 MFMA products:
//   L_IJ = A_IJ X_JJ^T,  X_JK = X_JJ W_JK (K < J),
//   A_IK -= L_IJ L_KJ^T (K > J),  W_IK -= L_IJ X_JK (K <= J)
// where W (LDS, ld 65) must hold zeros below the diagonal blocks on entry
// (the diagonal blocks are written here) and ends as X.  Look-ahead: of the
// trailing updates of step J, wave 0 takes only the next diagonal block's and
// goes straight on to factor it while waves 1-3 finish the others (they touch
// neither that block nor its W block).
// nbl (round 4): the live size; the 16-column blocks past it (identity in T,
// zeros in W) are skipped, which leaves them as they came in -- every live
// element sees the same operations as with all four blocks, the callers read
// only the live part of L and X.
// Returns (wave 0) whether a pivot was not positive and finite.
template <bool kFS = true>   // kFS: diag16_fs (round 6), else diag16_lane
__device__ __forceinline__ bool diag_factor_invert(double* T, double* W, double* bc, int nbl = 64) {
  const int tid = threadIdx.x, wv = tid >> 6;
  const int Jn = (nbl + 15) >> 4;   // live 16-column blocks (1..4)
  DIAG_CLK(0);
  bool bad = false;
  for (int J = 0; J < Jn; J++) {
    const int o = 16 * J;
    double* TJ = T + o + o * 65;
    if (wv == 0) {
      if (J > 0) {   // A_JJ -= L_J,J-1 L_J,J-1^T, the update left to this wave
        const d4 v = mm16(T + o + (o - 16) * 65, 1, 65, T + o + (o - 16) * 65, 65, 1);
        st16(TJ, v, true);
        __builtin_amdgcn_wave_barrier();
      }
      bad = (kFS ? diag16_fs(TJ, W + o + o * 65, bc) : diag16_lane(TJ, W + o + o * 65, bc)) || bad;
    }
    __syncthreads();
    DIAG_CLK(1 + 3 * J);
    // phase B: Jn - 1 independent products (Jn-1-J panel blocks, J blocks of X's row J)
    if (wv < Jn - 1) {
      if (wv < Jn - 1 - J) {
        const int oi = o + 16 * (wv + 1);
        const d4 v = mm16(T + oi + o * 65, 1, 65, W + o + o * 65, 65, 1);
        st16(T + oi + o * 65, v, false);
      } else {
        const int ok = 16 * (wv - (Jn - 1 - J));
        const d4 v = mm16(W + o + o * 65, 1, 65, W + o + ok * 65, 1, 65);
        st16(W + o + ok * 65, v, false);
      }
    }
    if (J == Jn - 1) break;
    __syncthreads();
    DIAG_CLK(2 + 3 * J);
    // phase C on waves 1-3: trailing updates of T and W but the next diagonal
    // block (pair 0).  A wave's (up to 3) products read only block column / row
    // J and write blocks outside it: all products' loads and MFMAs first, then
    // the read-modify-write stores, so their latencies overlap
    if (wv == 0) continue;
    const int nA = (Jn - 1 - J) * (Jn - J) / 2, nW = (Jn - 1 - J) * (J + 1);
    d4 acc[3];
    double* dst[3];
#pragma unroll
    for (int u = 0; u < 3; u++) {
      const int t = wv + 3 * u;
      dst[u] = nullptr;
      if (t >= nA + nW) continue;               // wave-uniform
      if (t < nA) {
        int I = J + 1, q = t;                 // t-th pair J < K <= I
        while (q >= I - J) {
          q -= I - J;
          I++;
        }
        const int K = J + 1 + q;
        const int oi = 16 * I, ok = 16 * K;
        acc[u] = mm16(T + oi + o * 65, 1, 65, T + ok + o * 65, 65, 1);
        dst[u] = T + oi + ok * 65;
      } else {
        const int q = t - nA, I = J + 1 + q / (J + 1), K = q % (J + 1);
        const int oi = 16 * I, ok = 16 * K;
        acc[u] = mm16(T + oi + o * 65, 1, 65, W + o + ok * 65, 1, 65);
        dst[u] = W + oi + ok * 65;
      }
    }
#pragma unroll
    for (int u = 0; u < 3; u++)
      if (dst[u]) st16(dst[u], acc[u], true);
  }
  __syncthreads();
  DIAG_CLK(12);
  return bad;
}

// ---- diagonal tile in 8-column steps on four concurrent waves (round 6) ----
// The same output as diag_factor_invert -- X = L^-1 of the 64x64 SPD tile T
// (LDS, ld 65, lower valid, identity past the live size nbl) into W (ld 65,
// zeros on entry, lower X, zeros above) -- with the pivot chain cut to what
// one wave must do in sequence: eight lane-redundant 8x8 factors (chol8_lane)
// and, between them, two short element-parallel phases.  Everything else runs
// beside the chain on the other waves, synchronised by LDS flags (workgroup
// scope release / acquire, no s_barrier per step):
//   wave 0 (the chain), step k (kb = 8k): A_kk (final) -> chol8_lane -> each
//     lane i >= kb+8 solves its row of block column k against the lane-held
//     L_kk (x_i = a_i L_kk^-T; stored transposed in T's strict upper part, at
//     T[(kb + q) + 65 i], where row i's eight values are contiguous) -> the
//     next diagonal block A_{k+1,k+1} -= L_{k+1,k} L_{k+1,k}^T one element per
//     lane -> flag PANEL = k + 1;
//   wave 1 (trailing updates, v_mfma_f64_16x16x4f64 tiles): after PANEL > k,
//     panel k onto block column k+1 below its diagonal block (flag T1A), then
//     onto the tile column from block k+2 (flag T1B: blocks k+2, k+3, what the
//     chain's next two steps read), then the rest;
//   waves 2 and 3 (the inverse, by 8-row blocks of parity p): X_ss =
//     inv8(chol8(A_ss)) in registers for s = p mod 2, S_i += L_{i,s-1} X_{s-1}
//     (MFMA, into W) for the wave's row blocks i >= s once row block s-1 of X
//     is final (flag XDONE), then row block s of X = -X_ss [S_s | -I] (flag
//     XDONE = s + 1).
// Every element of T and W has one writer per update and sees its updates in
// panel order (the flags order the writers), every sum has a fixed order: the
// result does not depend on the waves' timing.  A flag wait gives up after a
// bounded spin (never expected) and reports it as bit 2 of the return value,
// which the callers OR into the pivot flag (the host's hand-off timeout path).
namespace d8f {
constexpr int PANEL = 0, T1A = 1, T1B = 2, XDONE = 3, ERR = 4;
}
// signal: this wave's LDS writes have completed (lgkmcnt(0); the LDS is
// coherent across the CU), then the flag store.  wait: poll the flag (the
// loads after it are issued only once it is seen); no global-memory fence --
// the flags order LDS traffic only.
__device__ __forceinline__ void lds_signal(int* fl, int which, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  *reinterpret_cast<volatile int*>(fl + which) = v;
}
__device__ __forceinline__ void lds_wait(int* fl, int which, int v) {
  int n = 0;
  while (*reinterpret_cast<volatile int*>(fl + which) < v) {
    if (++n > (1 << 21)) {   // ~0.1 s: a lost signal must never hang the GPU
      *reinterpret_cast<volatile int*>(fl + d8f::ERR) = 1;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
}

// D(16x16) = sum_{q < 8} A(row, q) B(q, col) on one wave, operands read from
// LDS by row: A(row, q) = Ar[row][q0 + q], B(q, col) = Bc[col][q0 + q] with
// rows at pa(row), pb(col) (ld 65 "transposed" storage: element q of row r at
// base[q + 65 r]); D in the f64 MFMA layout (lane l, reg r -> row (l >> 4) + 4r,
// col l & 15); acc holds the initial values
__device__ __forceinline__ d4 mm16x8(const double* A, const double* B, int q0, int ra, int rb, d4 acc) {
  const int l = threadIdx.x & 63, kq = l >> 4;
#pragma unroll
  for (int u = 0; u < 2; u++) {
    const double a = A[(q0 + 4 * u + kq) + 65 * ra];
    const double b = B[(q0 + 4 * u + kq) + 65 * rb];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
  return acc;
}

// trailing tiles on wave 1, up to 3 per call: T[R + row][C + col] -= sum_q
// L[R + row][kb + q] L[C + col][kb + q] for row + R < nbl, col + C < cend and
// (lower) R + row >= C + col.  Every tile's LDS loads (operands and C) are
// issued first, then the MFMAs, then the stores: one LDS latency per call
// instead of three per tile.
__device__ __forceinline__ void d8_trail3(double* T, int kb, const int (&R)[3], const int (&C)[3], int nt, int nbl,
                                          int cend, bool lower) {
  // Branch-free: an element outside the region reads and writes the lane's own
  // slot in T's padding row (T[64 + 65 l]: ld 65, rows 0..63 used), so no load
  // or store needs an EXEC mask of its own (measured: the per-element masks cost
  // more than the MFMAs, profiles/r06*_ubench_factor64.txt)
  const int l = threadIdx.x & 63, kq = l >> 4, li = l & 15;
  double a[3][2], b[3][2], cv[3][4];
  int ad[3][4];
#pragma unroll
  for (int t = 0; t < 3; t++) {
    if (t >= nt) break;   // (wave-uniform)
    const int ra = min(R[t] + li, 63), rb = min(C[t] + li, 63);
#pragma unroll
    for (int u = 0; u < 2; u++) {
      a[t][u] = T[(kb + 4 * u + kq) + 65 * ra];
      b[t][u] = T[(kb + 4 * u + kq) + 65 * rb];
    }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = R[t] + kq + 4 * r, j = C[t] + li;
      ad[t][r] = (i < nbl && j < cend && (!lower || i >= j)) ? i + 65 * j : 64 + 65 * l;
      cv[t][r] = T[ad[t][r]];
    }
  }
#pragma unroll
  for (int t = 0; t < 3; t++) {
    if (t >= nt) break;
    d4 acc = {0, 0, 0, 0};
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t][0], b[t][0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[t][1], b[t][1], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; r++) T[ad[t][r]] = cv[t][r] - acc[r];
  }
}

__device__ __forceinline__ int diag_factor_invert8(double* T, double* W, double* bc, int nbl = 64) {
  const int tid = threadIdx.x, l = tid & 63;
  // roles by wave: 0 the chain, 1 the trailing updates, 2-3 the inverse
  // (diagnostics bit 8: the trailing updates on wave 2, the inverse on waves 1, 3)
  const int wv = D8_DBG(8) ? ((tid >> 6) == 1 ? 2 : (tid >> 6) == 2 ? 1 : (tid >> 6)) : tid >> 6;
  int* fl = reinterpret_cast<int*>(bc);
  const int K = (nbl + 7) >> 3;   // live 8-column steps
  if (tid < 8) fl[tid] = 0;
  __syncthreads();
  DIAG_CLK(0);
  int ret = 0;
  if (wv == 0) {   // ---------------- the pivot chain
    for (int k = 0; k < K; k++) {
      const int kb = 8 * k;
      double a[36], iv[8];
#pragma unroll
      for (int i = 0; i < 8; i++)
#pragma unroll
        for (int j = 0; j <= i; j++) a[P8(i, j)] = T[(kb + i) + 65 * (kb + j)];
      D8_CLK(k, 0);
      if (chol8_lane(a, iv)) ret |= 1;
      D8_CLK(k, 1);
      if (k == K - 1) break;
      if (!D8_DBG(2)) lds_wait(fl, d8f::T1A, k);   // block column k through panel k-1 (wave 1)
      D8_CLK(k, 2);
      const int i = l;
      if (i >= kb + 8 && i < nbl) {   // row i of block column k: x = a L_kk^-T
        double x[8];
#pragma unroll
        for (int c = 0; c < 8; c++) x[c] = T[i + 65 * (kb + c)];
#pragma unroll
        for (int c = 0; c < 8; c++) {
          double s = x[c];
#pragma unroll
          for (int t = 0; t < c; t++) s = fma(-a[P8(c, t)], x[t], s);
          x[c] = s * iv[c];
        }
#pragma unroll
        for (int c = 0; c < 8; c++) T[(kb + c) + 65 * i] = x[c];
      }
      __builtin_amdgcn_wave_barrier();
      D8_CLK(k, 3);
      if (!D8_DBG(2)) lds_wait(fl, d8f::T1B, k);   // the next diagonal block through panel k-1 (wave 1)
      D8_CLK(k, 4);
      {   // A_{k+1,k+1} -= L_{k+1,k} L_{k+1,k}^T, lane (r, c), r >= c
        const int r = l >> 3, c = l & 7, ii = kb + 8 + r, jj = kb + 8 + c;
        if (c <= r && ii < nbl) {
          double t = T[ii + 65 * jj];
#pragma unroll
          for (int q = 0; q < 8; q++) t = fma(-T[(kb + q) + 65 * ii], T[(kb + q) + 65 * jj], t);
          T[ii + 65 * jj] = t;
        }
      }
      __builtin_amdgcn_wave_barrier();
      lds_signal(fl, d8f::PANEL, k + 1);
      D8_CLK(k, 5);
    }
    DIAG_CLK(1);
  } else if (wv == 1) {   // ---------------- trailing updates
    for (int k = 0; k + 1 < K && !D8_DBG(4); k++) {
      const int kb = 8 * k;
      lds_wait(fl, d8f::PANEL, k + 1);
      D8_CLK(k, 0);
      const int nt = (nbl - kb - 16 + 15) >> 4;   // 16-row tiles below the next diagonal block (<= 3)
      {
        const int R[3] = {kb + 16, kb + 32, kb + 48}, C[3] = {kb + 8, kb + 8, kb + 8};
        d8_trail3(T, kb, R, C, nt, nbl, min(kb + 16, nbl), false);
      }
      lds_signal(fl, d8f::T1A, k + 1);
      D8_CLK(k, 1);
      {
        const int R[3] = {kb + 16, kb + 32, kb + 48}, C[3] = {kb + 16, kb + 16, kb + 16};
        d8_trail3(T, kb, R, C, nt, nbl, nbl, true);
      }
      lds_signal(fl, d8f::T1B, k + 1);
      D8_CLK(k, 2);
      {   // the rest: tile columns from kb + 32 (<= 3 tiles)
        int R[3] = {0, 0, 0}, C[3] = {0, 0, 0}, n = 0;
        for (int c0 = kb + 32; c0 < nbl; c0 += 16)
          for (int r0 = c0; r0 < nbl; r0 += 16)
            if (n < 3) {
              R[n] = r0;
              C[n] = c0;
              n++;
            }
        d8_trail3(T, kb, R, C, n, nbl, nbl, true);
      }
      D8_CLK(k, 3);
    }
  } else {   // ---------------- the inverse, row blocks of parity p
    const int p = wv - 2;
    for (int s = 0; s < K && !D8_DBG(1); s++) {
      const int sb = 8 * s;
      lds_wait(fl, d8f::PANEL, s);   // A_ss final, panels < s written
      D8_CLK(s, 0);
      double xs[36], iv[8];
      const bool mine = (s & 1) == p;
      if (mine) {   // X_ss = L_ss^-1, lane-redundant (the chain's own factor of the same A_ss)
#pragma unroll
        for (int i = 0; i < 8; i++)
#pragma unroll
          for (int j = 0; j <= i; j++) xs[P8(i, j)] = T[(sb + i) + 65 * (sb + j)];
        chol8_lane(xs, iv);
        inv8_lane(xs, iv);
      }
      D8_CLK(s, 1);
      if (s >= 1) {   // S_i += L_{i,s-1} X_{s-1} for my row blocks i >= s
        lds_wait(fl, d8f::XDONE, s);
        D8_CLK(s, 2);
        const int tb = sb - 8;                       // X_{s-1}: rows tb.., columns < sb
        const int i0 = s + (((s & 1) == p) ? 0 : 1);  // my first row block >= s
        const int nr = i0 < K ? 8 * ((K - i0 + 1) >> 1) : 0;   // stacked rows (8 per block)
        // tiles (stacked 16-row tile, 16-column tile), up to 8, four per batch:
        // every load of a batch first, then its MFMAs, then its stores
        const int nrt = (nr + 15) >> 4, nct = (sb + 15) >> 4, ntile = nrt * nct;
        const int kq = l >> 4, li = l & 15;
        for (int t0 = 0; t0 < ntile; t0 += 4) {
          double av[4][2], bv[4][2];
          d4 acc[4];
          int wad[4][4];
#pragma unroll
          for (int t = 0; t < 4; t++) {
            if (t0 + t >= ntile) break;   // (wave-uniform)
            const int R = 16 * ((t0 + t) / nct), C = 16 * ((t0 + t) % nct);
            const int rr = R + li;                                                   // A operand's stacked row
            const int ra = min(8 * (i0 + 2 * (rr >> 3)) + (rr & 7), 63);
            const int cb = min(C + li, 63);                                          // B operand's column
            // A(row, q) = L[ra][tb + q] = T[(tb + q) + 65 ra]; B(q, col) = X[tb + q][cb] = W[(tb + q) + 65 cb]
#pragma unroll
            for (int u = 0; u < 2; u++) {
              av[t][u] = T[(tb + 4 * u + kq) + 65 * ra];
              bv[t][u] = W[(tb + 4 * u + kq) + 65 * cb];
            }
#pragma unroll
            for (int r = 0; r < 4; r++) {   // S so far (zeros before the first update); outside: the padding slot
              const int ro = R + kq + 4 * r, blk = i0 + 2 * (ro >> 3), row = 8 * blk + (ro & 7), col = C + li;
              wad[t][r] = (ro < nr && blk < K && col < sb && row < nbl) ? row + 65 * col : 64 + 65 * l;
              acc[t][r] = W[wad[t][r]];
            }
          }
#pragma unroll
          for (int t = 0; t < 4; t++) {
            if (t0 + t >= ntile) break;
#pragma unroll
            for (int u = 0; u < 2; u++) acc[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[t][u], bv[t][u], acc[t], 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; r++) W[wad[t][r]] = acc[t][r];
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      D8_CLK(s, 3);
      if (mine) {   // row block s of X: -X_ss [S_s | -I], lane = column
        const int col = l;
        if (col < sb + 8) {
          double sv[8];
#pragma unroll
          for (int q = 0; q < 8; q++) sv[q] = col < sb ? W[(sb + q) + 65 * col] : (q == col - sb ? -1.0 : 0.0);
#pragma unroll
          for (int r = 0; r < 8; r++) {
            double o = 0.0;
#pragma unroll
            for (int q = 0; q <= r; q++) o = fma(xs[P8(r, q)], sv[q], o);
            W[sb + r < nbl ? (sb + r) + 65 * col : 64 + 65 * l] = -o;   // (outside: the padding slot)
          }
        }
        __builtin_amdgcn_wave_barrier();
        lds_signal(fl, d8f::XDONE, s + 1);
        D8_CLK(s, 4);
      }
    }
  }
  __syncthreads();
  DIAG_CLK(12);
  if (fl[d8f::ERR]) ret |= 2;
  return ret;
}

// The diagonal tiles' factor + inverse, chosen at build time (one form per
// library keeps k_step's code and registers to that form; A/B builds:
// `make -C graphslam_amd/csrc ab-forms` -> graphslam_amd/build/libpgo_form<N>.so,
// loaded with PGO_LIB_PATH): 1 diag_factor_invert over diag16_fs (default,
// round 6), 0 over diag16_lane (round 5), 2 diag_factor_invert8 (8-column steps
// on four concurrent waves; measured slower, profiles/r06*_ubench_factor64.txt)
#ifndef PGO_DIAG_FORM
#define PGO_DIAG_FORM 1
#endif
// the diagonal tile's factor + inverse by the configured form; a pivot that is
// not positive and finite (bit 1) or a lost LDS flag (bit 2: the host's
// hand-off timeout path) goes to the lane's pivot flag
__device__ __forceinline__ void factor_invert_tile(const CholDev& c, double* Ts, double* Ws, double* bc, int nb) {
  const int nbl = c.diag_full ? 64 : nb;
#if PGO_DIAG_FORM == 2
  const int r = diag_factor_invert8(Ts, Ws, bc, nbl);
#else
  const int r = diag_factor_invert<PGO_DIAG_FORM != 0>(Ts, Ws, bc, nbl) ? 1 : 0;
#endif
  if (r) __hip_atomic_fetch_or(c.flag, r, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- in-launch hand-off of a diagonal tile's inverse (MI355X_MICROARCH.md,
// inter-workgroup visibility, the "sc1 stores / sc1 flag / sc1 loads" row): the
// diagonal workgroup stores the inverse (trsm operand order) and the panel's y
// with sc1 (write-through) stores, every wave waits for its stores, a barrier,
// then one lane stores the step flag sc1; a waiting workgroup polls the flag
// with sc1 loads (one lane, s_sleep, bounded), joins a barrier, and reads the
// handed-off bytes with sc1 loads only.  The flags are zeroed at the start of
// every factorisation; a step publishes kn / 64 + 1 for its panel kn.
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte forms (MI355X_MICROARCH.md: 8-byte accesses run at 0.54-0.70x the
// 16-byte rate): buffer loads / stores with aux 16 = sc1, through a
// wave-uniform descriptor of the payload
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wave_rsrc(const void* p, unsigned bytes) {
  const unsigned long long a = (unsigned long long)p;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)a), hi = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((unsigned long long)hi << 32) | lo), 0, bytes, 0x00020000);
}
__device__ __forceinline__ void st2_sc1(__amdgpu_buffer_rsrc_t r, int elem, double x, double y) {
  const double2 v = make_double2(x, y);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), r, elem * 8, 0, 16);
}
__device__ __forceinline__ double2 ld2_sc1(__amdgpu_buffer_rsrc_t r, int elem) {
  return __builtin_bit_cast(double2, __builtin_amdgcn_raw_buffer_load_b128(r, elem * 8, 0, 16));
}
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void publish_step(int* flag, int val) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(flag, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Waits (one lane polls, the workgroup joins a barrier) until *flag >= val;
// gives up after c.poll_ticks (PGO_HANDOFF_TIMEOUT_MS, default 2 s) with bit 2
// of the pivot flag set (the host retries the try once, then reports a HIP
// failure), so a lost hand-off can never hang the GPU.
__device__ __forceinline__ void wait_step(const CholDev& c, const int* flag, int val) {
  if (threadIdx.x == 0) {
    const unsigned long long t0 = wall_clock64();   // 100 MHz
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < val) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > c.poll_ticks) {
        __hip_atomic_fetch_or(c.flag, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// Forward substitution of the panel's rows of the frontal vector: y = X v with
// X = L_bb^-1 (LDS, ld 65), published sc1 (the rows below get v -= L y in the
// trsm); y is also left in ys (LDS).
// (4 waves: wave q sums k in [16q, 16q + 16), then a fixed-order sum of the 4)
__device__ __forceinline__ void panel_rhs(double* v, const double* X, int nb, double* buf, double* ys) {
  __shared__ double part[4][64];
  const int tid = threadIdx.x, r = tid & 63, q = tid >> 6;
  if (tid < 64) buf[tid] = tid < nb ? v[tid] : 0.0;
  __syncthreads();
  double acc = 0.0;
#pragma unroll
  for (int k = 16 * q; k < 16 * q + 16; k++) acc = fma(k <= r ? X[r + k * 65] : 0.0, buf[k], acc);
  part[q][r] = acc;
  __syncthreads();
  if (tid < 64) {
    const double y = tid < nb ? ((part[0][tid] + part[1][tid]) + part[2][tid]) + part[3][tid] : 0.0;
    ys[tid] = y;
    if (tid < nb) st_sc1(v + tid, y);
  }
}

// X = L^-1 (LDS Ws, ld 65), stored sc1 in the trsm's operand order to Mf:
// Mf[(4 ks + ct) * 64 + l] = X[16 ct + (l & 15)][4 ks + (l >> 4)] (what the
// trsm's lane l needs for k-step ks, column tile ct) -- the hand-off payload.
// X is lower triangular, so fragment (ks, ct) is all zeros when 4 ks > 16 ct +
// 15, i.e. ct < ks / 4: 24 of the 64 (round 6) -- neither stored nor loaded,
// and their MFMAs (products with zero) skipped by the readers (inv_frag_zero)
__device__ __forceinline__ constexpr bool inv_frag_zero(int ks, int ct) { return ct < (ks >> 2); }
__device__ __forceinline__ void publish_inverse(double* __restrict__ Mf, const double* Ws, int nb) {
  const int tid = threadIdx.x;
  const __amdgpu_buffer_rsrc_t r = wave_rsrc(Mf, 4096 * 8);
#pragma unroll
  for (int u = 0; u < 8; u++) {   // element pairs (idx, idx + 1): rows fa, fa + 1 of one column fb
    const int idx = 2 * (tid + 256 * u);
    const int l = idx & 63, ct = (idx >> 6) & 3, ks = idx >> 8;
    if (inv_frag_zero(ks, ct)) continue;   // (a zero fragment: never read)
    const int fa = 16 * ct + (l & 15), fb = 4 * ks + (l >> 4);
    const double x0 = (fa < nb && fb < nb && fa >= fb) ? Ws[fa + fb * 65] : 0.0;
    const double x1 = (fa + 1 < nb && fb < nb && fa + 1 >= fb) ? Ws[fa + 1 + fb * 65] : 0.0;
    st2_sc1(r, idx, x0, x1);
  }
}

// After the hand-off: X row-major to M (the backward solve's copy).  The
// tile's own L_bb is not written back to the front (round 5): every later
// reader of a diagonal tile uses its inverse (the column solves' operand copy,
// the backward solve and the marginals M, the panel exchange) and reads L
// only below the tile, so those stores and the diagonal blocks' lane-0 stores
// in diag16_lane were dead (the front keeps the assembled values there).
__device__ __forceinline__ void store_factor(double* __restrict__ M, const double* Ws, int nb) {
  const int tid = threadIdx.x;
  for (int idx = tid; idx < 4096; idx += 256) {
    const int a = idx >> 6, b = idx & 63;
    M[idx] = (a < nb && b < nb && a >= b) ? Ws[a + b * 65] : 0.0;
  }
}

// The rows of a diagonal tile below its live nb x nb block (nb < 64: a front's
// last panel) were kept in `keep` (the thread's 16 elements, idx = tid + 256 u,
// columns < nb) while the block was factored; solved here: L = A X^T (X = Ws),
// written to the front (columns < nb) and v -= L y for those rows (rows with
// r0 + i >= m, i >= rrem, skipped).  Ts is scratch (the live block is stored).
__device__ __forceinline__ void diag_own_rows(double* Fs, int ld, int rrem, double* v, const double* keep, double* Ts,
                                              const double* Ws, const double* ys, int nb) {
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
#pragma unroll
  for (int u = 0; u < 16; u++) {
    const int idx = tid + 256 * u, i = idx & 63, j = idx >> 6;
    Ts[i + j * 65] = (i >= nb && j < nb) ? keep[u] : 0.0;
  }
  __syncthreads();
  const int J = wv;   // wave wv: column block J = wv, all row blocks
  d4 acc[4];
#pragma unroll
  for (int I = 0; I < 4; I++) {
    acc[I] = d4{0, 0, 0, 0};
    if (16 * I + 15 < nb || 16 * J >= nb) continue;   // wave-uniform: no row >= nb / no column < nb
#pragma unroll
    for (int K = 0; K < 4; K++) {
      const d4 p = mm16(Ts + 16 * I + 16 * K * 65, 1, 65, Ws + 16 * J + 16 * K * 65, 65, 1);
#pragma unroll
      for (int r = 0; r < 4; r++) acc[I][r] += p[r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int I = 0; I < 4; I++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = 16 * I + (l >> 4) + 4 * r, j = 16 * J + (l & 15);
      Ts[i + j * 65] = (i >= nb && j < nb) ? acc[I][r] : 0.0;
    }
  __syncthreads();
  if (tid >= nb && tid < 64 && tid < rrem) {
    double t = 0.0;
    for (int j = 0; j < nb; j++) {
      const double lij = Ts[tid + j * 65];
      Fs[tid + (size_t)j * ld] = lij;
      t = fma(lij, ys[j], t);
    }
    v[tid] -= t;
  }
}

// Rows r0 .. r0+63 of front s below panel kn (nb columns): L = A X^T with the
// published inverse (operand-order copy Mf, sc1 loads) as a GEMM on
// v_mfma_f64_16x16x4_f64 (16 rows per wave), L written to the front and the
// frontal vector's rows updated with v -= L y.  A(i, k) = A[i * ars + k * acs]
// (an LDS tile or the front itself).
__device__ __forceinline__ void trsm_rows(const CholDev& c, int s, int r0, int kn, int nb, const double* A, int ars,
                                          int acs, double* xs) {
  const int m = c.m[s];
  const double* Mf = c.Tinv + c.tfo + c.toff[s] + (kn / 64) * 4096;
  double* fv = c.fv + c.voff[s];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  {   // the inverse once per workgroup into LDS (xs: 4096 doubles), 8 coalesced 16-byte sc1 loads per thread in flight
    const __amdgpu_buffer_rsrc_t r = wave_rsrc(Mf, 4096 * 8);
    double2 t[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {   // (fragment ks = idx >> 8, ct = (idx >> 6) & 3 of idx = 2 (tid + 256 u))
      const int idx = 2 * (tid + 256 * u);
      t[u] = inv_frag_zero(idx >> 8, (idx >> 6) & 3) ? make_double2(0.0, 0.0) : ld2_sc1(r, idx);
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = 2 * (tid + 256 * u);
      if (inv_frag_zero(idx >> 8, (idx >> 6) & 3)) continue;
      xs[idx] = t[u].x;
      xs[idx + 1] = t[u].y;
    }
  }
  // the panel's y (handed off, sc1) and this lane's right-hand-side rows, in
  // flight with the inverse's loads (one memory latency, not three)
  const int rw = r0 + wv * 16, kl = l >> 4;
  double yc[4], fvr[4];
#pragma unroll
  for (int ct = 0; ct < 4; ct++) {
    const int col = 16 * ct + (l & 15);
    yc[ct] = col < nb ? ld_sc1(fv + kn + col) : 0.0;
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int row = rw + kl + 4 * r;
    fvr[r] = ((l & 15) == 0 && row < m) ? fv[row] : 0.0;
  }
  __syncthreads();
  if (rw >= m) return;                                // (no barriers below)
  double* Fc = fcol(c.F + c.foff[s], m, true, kn);   // the panel's column block (blocked fronts are packed)
  const int ldc = fld(m, true, kn);
  const int il = wv * 16 + (l & 15), arow = r0 + il;
  double a[16], tb[16][4];   // A fragments, inverse fragments
#pragma unroll
  for (int ks = 0; ks < 16; ks++) {
    const int k = 4 * ks + kl;
    a[ks] = (arow < m && k < nb) ? A[il * ars + k * acs] : 0.0;
  }
#pragma unroll
  for (int ks = 0; ks < 16; ks++)
#pragma unroll
    for (int ct = 0; ct < 4; ct++) tb[ks][ct] = inv_frag_zero(ks, ct) ? 0.0 : xs[(4 * ks + ct) * 64 + l];
  d4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0}, acc3 = {0, 0, 0, 0};
#pragma unroll
  for (int ks = 0; ks < 16; ks++) {   // (zero fragments: no product -- column tile ct takes k-steps ks < 4 ct + 4)
    if (!inv_frag_zero(ks, 0)) acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], tb[ks][0], acc0, 0, 0, 0);
    if (!inv_frag_zero(ks, 1)) acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], tb[ks][1], acc1, 0, 0, 0);
    if (!inv_frag_zero(ks, 2)) acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], tb[ks][2], acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], tb[ks][3], acc3, 0, 0, 0);
  }
  double part[4] = {0, 0, 0, 0};   // L[row, panel] y for the lane's 4 rows
#pragma unroll
  for (int ct = 0; ct < 4; ct++) {
    const d4 v = ct == 0 ? acc0 : (ct == 1 ? acc1 : (ct == 2 ? acc2 : acc3));
    const int col = 16 * ct + (l & 15);
#pragma unroll
    for (int r = 0; r < 4; r++) part[r] = fma(v[r], yc[ct], part[r]);
    if (col >= nb) continue;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = rw + kl + 4 * r;
      if (row < m) Fc[row + (size_t)col * ldc] = v[r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {   // sum over the 16 lanes of the row group
    double t = part[r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) t += __shfl_xor(t, o);
    const int row = rw + kl + 4 * r;
    if ((l & 15) == 0 && row < m) fv[row] = fvr[r] - t;
  }
}

// Schur update of one 64x64 lower tile: C[r0:r0+64, c0:c0+64] -= P_r P_c^T with
// P = F[:, k0:kend), kend = end of the current panel (depth <= kKB).  Each wave
// owns 32x32 of the tile as 2x2 v_mfma_f64_16x16x4_f64 blocks, operands straight
// from global (the panel columns are L2-resident); the product is formed
// transposed (A = column-side rows) so each store covers 16 consecutive rows.
// Inner tasks (bit 31 of k0) clip columns at the end of the current kKB block.
template <bool kToLds>
__device__ __forceinline__ void syrk_tile64(const CholDev& c, const int4 t, int kb, double* Ts) {
  const int s = t.x, row0 = t.y, col0 = t.z;
  const bool inner = t.w < 0;
  const int k0 = t.w & 0x7fffffff;
  const int m = c.m[s], w = c.w[s];
  const int kend = min(kb + kNB, w);
  const int colend = inner ? min((kb & ~(kKB - 1)) + kKB, w) : m;
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int qi = 32 * (wv >> 1), qj = 32 * (wv & 1);
  if (row0 == col0 && qi < qj) return;       // strictly upper quarter of a diagonal tile (caller syncs)
  const int li = l & 15, lk = l >> 4;
  double* Fs = c.F + c.foff[s];
  double* Cb = fcol(Fs, m, true, col0);   // the tile's columns: one column block (col0 = kn)
  const int ldc = fld(m, true, col0);
  const int rA = row0 + qi + li, rB = rA + 16;          // C rows (B operand rows)
  const int cA = col0 + qj + li, cB = cA + 16;          // C columns (A operand rows)
  // C prefetch (output layout: lane l, reg r -> column col0+qj+16mj+lk+4r, row row0+qi+16mi+li)
  double cold[2][2][4];
#pragma unroll
  for (int mi = 0; mi < 2; mi++)
#pragma unroll
    for (int mj = 0; mj < 2; mj++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = row0 + qi + 16 * mi + li, col = col0 + qj + 16 * mj + lk + 4 * r;
        cold[mi][mj][r] = (row < m && col < colend && row >= col) ? Cb[row + (size_t)(col - col0) * ldc] : 0.0;
      }
  const bool vrA = rA < m, vrB = rB < m, vcA = cA < m, vcB = cB < m;
  d4 acc00 = {0, 0, 0, 0}, acc01 = {0, 0, 0, 0}, acc10 = {0, 0, 0, 0}, acc11 = {0, 0, 0, 0};
  const int K = kend - k0;
  for (int kk = 0; kk < K; kk += 16) {       // 16 operand loads in flight, then 16 MFMAs
    double ra[4], rb[4], ca[4], cb[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const bool kin = kk + 4 * u + lk < K;   // (16 panel columns from k0 + kk: one column block)
      const double* pk = fcol(Fs, m, true, k0 + kk) + (size_t)(4 * u + lk) * fld(m, true, k0 + kk);
      ra[u] = (kin && vrA) ? pk[rA] : 0.0;
      rb[u] = (kin && vrB) ? pk[rB] : 0.0;
      ca[u] = (kin && vcA) ? pk[cA] : 0.0;
      cb[u] = (kin && vcB) ? pk[cB] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      acc00 = __builtin_amdgcn_mfma_f64_16x16x4f64(ca[u], ra[u], acc00, 0, 0, 0);  // [mj=0][mi=0]
      acc01 = __builtin_amdgcn_mfma_f64_16x16x4f64(ca[u], rb[u], acc01, 0, 0, 0);  // [mj=0][mi=1]
      acc10 = __builtin_amdgcn_mfma_f64_16x16x4f64(cb[u], ra[u], acc10, 0, 0, 0);  // [mj=1][mi=0]
      acc11 = __builtin_amdgcn_mfma_f64_16x16x4f64(cb[u], rb[u], acc11, 0, 0, 0);  // [mj=1][mi=1]
    }
  }
#pragma unroll
  for (int mi = 0; mi < 2; mi++)
#pragma unroll
    for (int mj = 0; mj < 2; mj++) {
      const d4 a = mj == 0 ? (mi == 0 ? acc00 : acc01) : (mi == 0 ? acc10 : acc11);
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = row0 + qi + 16 * mi + li, col = col0 + qj + 16 * mj + lk + 4 * r;
        if (row < m && col < colend && row >= col) {
          const double v = cold[mi][mj][r] - a[r];
          Cb[row + (size_t)(col - col0) * ldc] = v;
          if (kToLds) Ts[(row - row0) + (col - col0) * 65] = v;
        }
      }
    }
}

// register-fragment variant (kept for the microbenchmark; k_panel_syrk_lds is launched)
__global__ __launch_bounds__(256) void k_panel_syrk(CholDev c, const int4* __restrict__ tasks, int kb) {
  lane_offset(c);
  syrk_tile64<false>(c, tasks[blockIdx.x], kb, nullptr);
}

// Same tile and semantics as k_panel_syrk, with the panel rows and columns of
// the tile staged through LDS in chunks of 16 k (double-buffered, every operand
// loaded once per workgroup instead of once per wave pair; 8 loads per thread
// per chunk, issued one chunk ahead of the MFMAs).  Low register count, so
// several workgroups per CU hide the load latency.
// smem: 4 * 16 * 68 doubles (Sr[2], Sc[2])
// KC: panel columns staged per chunk (16; 32 halves the round trips with the
// same 4-deep MFMA steps in the same k order -- bitwise the same tile -- but
// measured no faster, profiles/r05n_syrk_ubench.txt)
template <bool kPrefC = false, int KC = 16>   // kPrefC: the C tile's loads issued before the k loop
__device__ __forceinline__ void syrk_lds_body(const CholDev& c, const int4 t, int kb, double* smem) {
  constexpr int LD = 64 + 4, NQ = KC / 4;
  double(*Sr)[KC * LD] = reinterpret_cast<double(*)[KC * LD]>(smem);
  double(*Sc)[KC * LD] = reinterpret_cast<double(*)[KC * LD]>(smem + 2 * KC * LD);
  const int s = t.x, row0 = t.y & kRowMask, col0 = t.z, clip = t.y >> kClipShift;
  const bool inner = t.w < 0;
  const int k0 = t.w & 0x7fffffff;
  const int m = c.m[s], w = c.w[s];
  const int kend = min(kb + kNB, w);
  int colend = inner ? min((kb & ~(kKB - 1)) + kKB, w) : m;
  if (clip) colend = min(colend, col0 + clip);   // a split tile: its columns only
  const int K = kend - k0, nch = (K + KC - 1) / KC;
  double* Fs = c.F + c.foff[s];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int qi = 32 * (wv >> 1), qj = 32 * (wv & 1);
  const bool active = !(row0 == col0 && qi < qj);
  const int lk = l >> 4;
  // staging map: thread -> (k = idx >> 6, r = idx & 63), idx = tid + 256 q, q < NQ
  double st[2 * NQ];
  auto load = [&](int ch) {
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      // the chunk's KC panel columns sit in one column block (k0: a panel start)
      const int idx = tid + 256 * q, k = KC * ch + (idx >> 6), r = idx & 63;
      const double* pk = fcol(Fs, m, true, k0 + KC * ch) + (size_t)(idx >> 6) * fld(m, true, k0 + KC * ch);
      st[q] = (k < K && row0 + r < m) ? pk[row0 + r] : 0.0;
      st[NQ + q] = (k < K && col0 + r < m) ? pk[col0 + r] : 0.0;
    }
  };
  auto stash = [&](int b) {
#pragma unroll
    for (int q = 0; q < NQ; q++) {
      const int idx = tid + 256 * q;
      Sr[b][(idx >> 6) * LD + (idx & 63)] = st[q];
      Sc[b][(idx >> 6) * LD + (idx & 63)] = st[NQ + q];
    }
  };
  // v_mfma_f64_4x4x4f64 (4 blocks of 4x4x4): the wave's 32x32 quadrant as 8
  // column groups of 4 (p) x 2 row groups of 16 (h), 16 independent
  // accumulators.  Block g of an instruction: A(i, k) at lane 16k + 4g + i,
  // B(k, j) at lane 16k + 4g + j, D(i, j) at lane 16i + 4g + j (probed,
  // scripts/ubench_mfma4.hip); here A = the column side (i: column 4p + i),
  // B = the row side (g, j: row 16h + 4g + j), so lane l holds row 16h + (l & 15),
  // column 4p + (l >> 4).  Each element is the same 4-term MFMA dot product in
  // the same k order as with v_mfma_f64_16x16x4f64 (bitwise the same result,
  // probed), at up to 69 instead of 48 TFLOP/s (independent chains).
  double acc[8][2];
#pragma unroll
  for (int p = 0; p < 8; p++) acc[p][0] = acc[p][1] = 0.0;
  // C read-modify-write: lane l holds (row row0 + qi + 16h + (l & 15), column col0 + qj + 4p + (l >> 4));
  // the tile's columns lie in col0's column block (the planner never lets a tile straddle two)
  double* Cb = fcol(Fs, m, true, col0);
  const int ldc = fld(m, true, col0);
  double cold[8][2];
  auto load_c = [&] {
#pragma unroll
    for (int p = 0; p < 8; p++)
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const int row = row0 + qi + 16 * h + (l & 15), col = col0 + qj + 4 * p + lk;
        cold[p][h] = (active && row < m && col < colend && row >= col) ? Cb[row + (size_t)(col - col0) * ldc] : 0.0;
      }
  };
  if (kPrefC) load_c();
  load(0);
  stash(0);
  __syncthreads();
  for (int ch = 0; ch < nch; ch++) {
    const int b = ch & 1;
    if (ch + 1 < nch) load(ch + 1);
    if (active) {
#pragma unroll
      for (int u = 0; u < KC / 4; u++) {
        const double* sr = Sr[b] + (4 * u + lk) * LD + qi + (l & 15);
        const double* sc = Sc[b] + (4 * u + lk) * LD + qj + (l & 3);
        const double r0v = sr[0], r1v = sr[16];
        double cv[8];
#pragma unroll
        for (int p = 0; p < 8; p++) cv[p] = sc[4 * p];
#pragma unroll
        for (int p = 0; p < 8; p++) {
          acc[p][0] = __builtin_amdgcn_mfma_f64_4x4x4f64(cv[p], r0v, acc[p][0], 0, 0, 0);
          acc[p][1] = __builtin_amdgcn_mfma_f64_4x4x4f64(cv[p], r1v, acc[p][1], 0, 0, 0);
        }
      }
    }
    if (ch + 1 < nch) stash(b ^ 1);
    __syncthreads();
  }
  if (!active) return;
  if (!kPrefC) load_c();
#pragma unroll
  for (int p = 0; p < 8; p++)
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const int row = row0 + qi + 16 * h + (l & 15), col = col0 + qj + 4 * p + lk;
      if (row < m && col < colend && row >= col) Cb[row + (size_t)(col - col0) * ldc] = cold[p][h] - acc[p][h];
    }
}

__global__ __launch_bounds__(256) void k_panel_syrk_lds(CholDev c, const int4* __restrict__ tasks, int kb) {
  lane_offset(c);
  __shared__ __attribute__((aligned(16))) double smem[4 * 16 * 68];
  syrk_lds_body(c, tasks[blockIdx.x], kb, smem);
}
// (the C-prefetch form, for the microbenchmark A/B: scripts/ubench_syrk.hip)
__global__ __launch_bounds__(256) void k_panel_syrk_lds_pc(CholDev c, const int4* __restrict__ tasks, int kb) {
  lane_offset(c);
  __shared__ __attribute__((aligned(16))) double smem[4 * 16 * 68];
  syrk_lds_body<true>(c, tasks[blockIdx.x], kb, smem);
}

// Schur update of a diagonal 64x64 tile into LDS: Ts (ld 65, lower) = C - P P^T,
// P = F[r0:r0+64, k0:kend).  C and the first 64-deep chunk of P are loaded
// together (one memory latency for the usual inner depth of 64); P goes
// through Sp (LDS, [k][row], ld 68) chunk by chunk, the next chunk's loads in
// flight during the MFMAs; the 10 lower 16x16 blocks are dealt 3/3/2/2 to the
// waves.  Elements outside the live nb x nb block (nb < 64 at a front's last
// panel) are written back to F here; the caller factors the live block.
__device__ __forceinline__ void diag_tile_update(const CholDev& c, const int4 t, int kb, double* Ts, double* Sp) {
  constexpr int LD = 68;
  const int s = t.x, r0 = t.y;
  const bool inner = t.w < 0;
  const int k0 = t.w & 0x7fffffff;
  const int m = c.m[s], w = c.w[s];
  const int kend = min(kb + kNB, w);
  const int colend = inner ? min((kb & ~(kKB - 1)) + kKB, w) : m;
  const int K = kend - k0, nch = (K + 63) >> 6;
  const int nb = min(kNB, w - r0);
  double* Fs = c.F + c.foff[s];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int li = l & 15, lk = l >> 4;
  double st[16];
  auto load = [&](int ch) {   // chunk ch: panel columns k0 + 64 ch ..: one column block
    const double* Pb = fcol(Fs, m, true, k0 + 64 * ch);
    const int ldp = fld(m, true, k0 + 64 * ch);
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int idx = tid + 256 * q, i = idx & 63, k = 64 * ch + (idx >> 6);
      st[q] = (k < K && r0 + i < m) ? Pb[(r0 + i) + (size_t)(idx >> 6) * ldp] : 0.0;
    }
  };
  double* Db = fcol(Fs, m, true, r0) + r0;   // the diagonal tile
  const int ldd = fld(m, true, r0);
  double cv[16];   // C, lower part of the updated region: its loads and the first chunk's in flight together
#pragma unroll
  for (int q = 0; q < 16; q++) {
    const int idx = tid + 256 * q, i = idx & 63, j = idx >> 6;
    cv[q] = (i >= j && r0 + i < m && r0 + j < colend) ? Db[i + (size_t)j * ldd] : 0.0;
  }
  load(0);
#pragma unroll
  for (int q = 0; q < 16; q++) {
    const int idx = tid + 256 * q;
    Ts[(idx & 63) + (idx >> 6) * 65] = cv[q];
  }
  // lower 16x16 blocks (I, J) of this wave
  const int nblk = wv < 2 ? 3 : 2;
  const int bI0 = wv == 0 ? 0 : (wv == 1 ? 3 : 3), bJ0 = wv == 0 ? 0 : (wv == 1 ? 0 : (wv == 2 ? 1 : 2));
  const int bI1 = wv == 0 ? 1 : (wv == 1 ? 1 : (wv == 2 ? 2 : 3)), bJ1 = wv == 0 ? 0 : (wv == 1 ? 1 : (wv == 2 ? 2 : 3));
  const int bI2 = wv == 0 ? 2 : 2, bJ2 = wv == 0 ? 0 : 1;
  d4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0};
  for (int ch = 0; ch < nch; ch++) {
    if (ch) __syncthreads();   // previous chunk's MFMAs are done with Sp
#pragma unroll
    for (int q = 0; q < 16; q++) {
      const int idx = tid + 256 * q;
      Sp[(idx >> 6) * LD + (idx & 63)] = st[q];
    }
    __syncthreads();
    if (ch + 1 < nch) load(ch + 1);
#pragma unroll
    for (int u = 0; u < 16; u++) {
      const double* sk = Sp + (4 * u + lk) * LD + li;
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(sk[16 * bJ0], sk[16 * bI0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(sk[16 * bJ1], sk[16 * bI1], acc1, 0, 0, 0);
      if (nblk == 3) acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(sk[16 * bJ2], sk[16 * bI2], acc2, 0, 0, 0);
    }
  }
  // lane l, reg r of block (I, J): row 16I + li, column 16J + lk + 4r
#pragma unroll
  for (int b = 0; b < 3; b++) {
    if (b == 2 && nblk < 3) break;
    const d4 a = b == 0 ? acc0 : (b == 1 ? acc1 : acc2);
    const int I = b == 0 ? bI0 : (b == 1 ? bI1 : bI2), J = b == 0 ? bJ0 : (b == 1 ? bJ1 : bJ2);
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int i = 16 * I + li, j = 16 * J + lk + 4 * r;
      if (i >= j && r0 + i < m && r0 + j < colend) {
        const double v = Ts[i + j * 65] - a[r];
        Ts[i + j * 65] = v;
        if (!(i < nb && j < nb)) Db[i + (size_t)j * ldd] = v;
      }
    }
  }
}

// The next panel's diagonal tile (row0 = col0 = kn < w): updated with panel kb
// (diag_tile_update), factored and inverted in LDS, L and the inverses stored,
// y of the panel formed; at a front's last panel (nb < 64) the tile's rows
// below the live block are solved here too; then the inverse is published for
// the workgroups solving the rows below the tile.
// smem: kDiagSmem = 64*65 + 64*68 + 2*64 doubles.
constexpr int kDiagSmem = 64 * 65 + 64 * 68 + 2 * 64;

__device__ __forceinline__ void syrk_diag_body(const CholDev& c, const int4 t, int kb, double* smem, int slot = -1) {
  double* Ts = smem;
  double* Ws = smem + 64 * 65;
  double* bc = Ws + 64 * 68;
  double* ys = bc + 64;
  const int s = t.x, kn = t.y;
  const int m = c.m[s], w = c.w[s];
  const int nb = min(kNB, w - kn);
  const int tid = threadIdx.x;
  STAMP(slot, 0);
  diag_tile_update(c, t, kb, Ts, Ws);
  __syncthreads();
  STAMP(slot, 1);
  double keep[16];
#pragma unroll
  for (int u = 0; u < 16; u++) {   // same element set as the loop below: no hazard
    const int idx = tid + 256 * u, i = idx & 63, j = idx >> 6;
    keep[u] = (i >= nb && j < nb) ? Ts[i + j * 65] : 0.0;
    if (!(i < nb && j < nb)) Ts[i + j * 65] = i == j ? 1.0 : 0.0;
    Ws[i + j * 65] = 0.0;
  }
  __syncthreads();
  factor_invert_tile(c, Ts, Ws, bc, nb);
  STAMP(slot, 2);
  double* Fs = fcol(c.F + c.foff[s], m, true, kn) + kn;   // the diagonal tile, ld fld(m, true, kn)
  double* M = c.Tinv + c.toff[s] + (kn / 64) * 4096;   // row-major L^-1 of the tile
  double* v = c.fv + c.voff[s] + kn;
  publish_inverse(M + c.tfo, Ws, nb);
  panel_rhs(v, Ws, nb, bc, ys);
  STAMP(slot, 3);
  publish_step(c.stepflag + s, kn / 64 + 1);
  STAMP(slot, 4);
  store_factor(M, Ws, nb);
  if (nb < kNB) {
    __syncthreads();
    diag_own_rows(Fs, fld(m, true, kn), m - kn, v, keep, Ts, Ws, ys, nb);
  }
}

// First panel of a front: its assembled diagonal tile factored and inverted,
// the rest as syrk_diag_body.
__device__ __forceinline__ void first_diag_body(const CholDev& c, int s, double* smem) {
  double* Ts = smem;
  double* Ws = smem + 64 * 65;
  double* bc = Ws + 64 * 68;
  double* ys = bc + 64;
  const int m = c.m[s], w = c.w[s];
  const int nb = min(kNB, w);
  double* Fs = c.F + c.foff[s];
  const int ld0 = fld(m, true, 0);   // (blocked fronts are packed)
  const int tid = threadIdx.x;
  double tv[16], keep[16];
#pragma unroll
  for (int u = 0; u < 16; u++) {   // all loads in flight
    const int idx = tid + 256 * u, i = idx & 63, j = idx >> 6;
    tv[u] = (i < nb && j < nb) ? (i >= j ? Fs[i + (size_t)j * ld0] : 0.0) : (i == j ? 1.0 : 0.0);
    keep[u] = (i >= nb && i < m && j < nb) ? Fs[i + (size_t)j * ld0] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < 16; u++) {
    const int idx = tid + 256 * u, i = idx & 63, j = idx >> 6;
    Ts[i + j * 65] = tv[u];
    Ws[i + j * 65] = 0.0;
  }
  __syncthreads();
  factor_invert_tile(c, Ts, Ws, bc, nb);
  double* M = c.Tinv + c.toff[s];
  double* v = c.fv + c.voff[s];
  publish_inverse(M + c.tfo, Ws, nb);
  panel_rhs(v, Ws, nb, bc, ys);
  publish_step(c.stepflag + s, 1);
  store_factor(M, Ws, nb);
  if (nb < kNB) {
    __syncthreads();
    diag_own_rows(Fs, ld0, m, v, keep, Ts, Ws, ys, nb);
  }
}

// First panel of every big front of a level: workgroups [0, np) factor the
// fronts' first diagonal tiles (list), the others solve 64-row tiles below
// them (col: (front, r0, 0, -1)) once the tile's inverse is published.
__global__ __launch_bounds__(256, 2) void k_panel_first(CholDev c, const int* __restrict__ list, int np,
                                                     const int4* __restrict__ col) {
  lane_offset(c);
  __shared__ __attribute__((aligned(16))) double smem[kDiagSmem];
  const int b = blockIdx.x;
  if (b < np) {
    first_diag_body(c, list[b], smem);
    return;
  }
  const int4 t = col[b - np];
  const int s = t.x, m = c.m[s], nb = min(kNB, c.w[s]);
  wait_step(c, c.stepflag + s, 1);
  trsm_rows(c, s, t.y, 0, nb, c.F + c.foff[s] + t.y, 1, fld(m, true, 0), smem);
}

// The same first panel in two launches, for levels with many big fronts (the
// lower levels: hundreds of fronts x lanes): k_first_diag factors and inverts
// the first diagonal tiles (first_diag_body, one workgroup each), then
// k_first_trsm solves the 64-row tiles below them against the inverses of the
// previous launch -- a workgroup of ~64 VGPRs per lane and 32 KB of LDS, so
// 4-5 fit a CU instead of k_panel_first's 2 (the in-launch waiters hold
// k_step's LDS and registers).  Same arithmetic in the same order as
// trsm_rows: bitwise k_panel_first's result.
__global__ __launch_bounds__(256, 2) void k_first_diag(CholDev c, const int* __restrict__ list) {
  lane_offset(c);
  __shared__ __attribute__((aligned(16))) double smem[kDiagSmem];
  first_diag_body(c, list[blockIdx.x], smem);
}

// (k_col_trsm: the same for the tiles below panel kn = task.z of a split step
// (k_step's column workgroups, after k_step_diag published the inverse and
// k_panel_syrk_lds updated the tiles): same arithmetic as trsm_rows)
__global__ __launch_bounds__(256) void k_first_trsm(CholDev c, const int4* __restrict__ col) {
  lane_offset(c);
  __shared__ __attribute__((aligned(16))) double xs[4096];
  const int4 t = col[blockIdx.x];
  const int s = t.x, m = c.m[s], r0 = t.y, kn = max(t.z, 0), nb = min(kNB, c.w[s] - kn);
  const int ld = fld(m, true, kn);                            // (blocked fronts are packed)
  const double* Mf = c.Tinv + c.tfo + c.toff[s] + (kn / 64) * 4096;
  double* fv = c.fv + c.voff[s];
  const double* A = fcol(c.F + c.foff[s], m, true, kn) + r0;  // A(i, k) = A[i + k ld]
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  {
    double2 tq[8];
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = 2 * (tid + 256 * u);
      tq[u] = inv_frag_zero(idx >> 8, (idx >> 6) & 3) ? make_double2(0.0, 0.0)
                                                      : reinterpret_cast<const double2*>(Mf)[tid + 256 * u];
    }
#pragma unroll
    for (int u = 0; u < 8; u++) {
      const int idx = 2 * (tid + 256 * u);
      if (inv_frag_zero(idx >> 8, (idx >> 6) & 3)) continue;
      xs[idx] = tq[u].x;
      xs[idx + 1] = tq[u].y;
    }
  }
  const int rw = r0 + wv * 16, kl = l >> 4;
  double yc[4], fvr[4];
#pragma unroll
  for (int ct = 0; ct < 4; ct++) {
    const int col = 16 * ct + (l & 15);
    yc[ct] = col < nb ? fv[kn + col] : 0.0;
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    const int row = rw + kl + 4 * r;
    fvr[r] = ((l & 15) == 0 && row < m) ? fv[row] : 0.0;
  }
  const int il = wv * 16 + (l & 15), arow = r0 + il;
  double a[16];
#pragma unroll
  for (int ks = 0; ks < 16; ks++) {
    const int k = 4 * ks + kl;
    a[ks] = (arow < m && k < nb) ? A[il + (size_t)k * ld] : 0.0;
  }
  __syncthreads();
  if (rw >= m) return;
  double* Fc = fcol(c.F + c.foff[s], m, true, kn);
  d4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0}, acc2 = {0, 0, 0, 0}, acc3 = {0, 0, 0, 0};
#pragma unroll
  for (int ks = 0; ks < 16; ks++) {   // (zero fragments of the inverse: no product, as trsm_rows)
    const double* x = xs + 4 * ks * 64 + l;
    if (!inv_frag_zero(ks, 0)) acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], x[0], acc0, 0, 0, 0);
    if (!inv_frag_zero(ks, 1)) acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], x[64], acc1, 0, 0, 0);
    if (!inv_frag_zero(ks, 2)) acc2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], x[128], acc2, 0, 0, 0);
    acc3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[ks], x[192], acc3, 0, 0, 0);
  }
  double part[4] = {0, 0, 0, 0};
#pragma unroll
  for (int ct = 0; ct < 4; ct++) {
    const d4 v = ct == 0 ? acc0 : (ct == 1 ? acc1 : (ct == 2 ? acc2 : acc3));
    const int col = 16 * ct + (l & 15);
#pragma unroll
    for (int r = 0; r < 4; r++) part[r] = fma(v[r], yc[ct], part[r]);
    if (col >= nb) continue;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const int row = rw + kl + 4 * r;
      if (row < m) Fc[row + (size_t)col * ld] = v[r];
    }
  }
#pragma unroll
  for (int r = 0; r < 4; r++) {
    double t2 = part[r];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) t2 += __shfl_xor(t2, o);
    const int row = rw + kl + 4 * r;
    if ((l & 15) == 0 && row < m) fv[row] = fvr[r] - t2;
  }
}

// One panel step kb of every big front of a level in one launch:
//   [0, nsd)            the next panel's diagonal tiles (syrk_diag_body)
//   [nsd, nsd + ncol)   64-row tiles of the next panel's column block below
//                       its diagonal tile: Schur update with panel kb (kept in
//                       LDS), then, once the diagonal inverse is published,
//                       solved against it (trsm_rows)
//   the rest            the other Schur-update tiles (syrk_lds_body)
// The diagonal workgroups come first in dispatch order, so every waiting
// workgroup waits on a workgroup dispatched before it.
__global__ __launch_bounds__(256, 2) void k_step(CholDev c, const int4* __restrict__ sdiag, int nsd,
                                              const int4* __restrict__ col, int ncol, int nprep,
                                              const int4* __restrict__ tiles, int kb, int slot) {
  lane_offset(c);
  __shared__ __attribute__((aligned(16))) double smem[kDiagSmem];
  const int b = blockIdx.x;
  if (b < nsd) {
    syrk_diag_body(c, sdiag[b], kb, smem, b == 0 && blockIdx.y == 0 ? slot : -1);
    return;
  }
  if (b < nsd + ncol) {
    const int sl = b == nsd && blockIdx.y == 0 ? slot : -1;
    STAMP(sl, 5);
    const int4 t = col[b - nsd];   // (front, r0, kn, kb)
    syrk_tile64<true>(c, t, kb, smem);
    __syncthreads();
    STAMP(sl, 6);
    const int s = t.x, kn = t.z, nb = min(kNB, c.w[s] - kn);
    wait_step(c, c.stepflag + s, kn / 64 + 1);
    STAMP(sl, 7);
    trsm_rows(c, s, t.y, kn, nb, smem, 1, 65, smem + 64 * 65);
    STAMP(sl, 8);
    return;
  }
  if (b < nsd + ncol + nprep) {   // prep tiles follow the column tasks in col
    syrk_lds_body(c, col[b - nsd], kb, smem);
    return;
  }
  syrk_lds_body(c, tiles[b - nsd - ncol - nprep], kb, smem);
}

// A split step's diagonal tiles (k_step's [0, nsd) role alone): updated,
// factored, inverted, stored; the tiles below them are updated by a concurrent
// k_panel_syrk_lds and solved by k_first_trsm after both (chol_factor)
__global__ __launch_bounds__(256, 2) void k_step_diag(CholDev c, const int4* __restrict__ sdiag, int kb) {
  lane_offset(c);
  __shared__ __attribute__((aligned(16))) double smem[kDiagSmem];
  syrk_diag_body(c, sdiag[blockIdx.x], kb, smem);
}

// Schur update of one 128x128 lower tile (same task format and semantics as
// k_panel_syrk).  The panel rows/columns are staged through LDS in chunks of
// 16 k (double-buffered: the global loads of chunk c+1 are in flight while the
// MFMAs of chunk c run); each wave owns 64x64 of the tile as 4x4
// v_mfma_f64_16x16x4_f64 blocks.
__global__ __launch_bounds__(256) void k_panel_syrk128(CholDev c, const int4* __restrict__ tasks, int kb) {
  lane_offset(c);
  constexpr int LD = 144;   // [k][row] rows of 128 + pad
  __shared__ __attribute__((aligned(16))) double Sr[2][16 * LD];
  __shared__ __attribute__((aligned(16))) double Sc[2][16 * LD];
  const int4 t = tasks[blockIdx.x];
  const int s = t.x, row0 = t.y & kRowMask, col0 = t.z, clip = t.y >> kClipShift;
  const bool inner = t.w < 0;
  const int k0 = t.w & 0x7fffffff;
  const int m = c.m[s], w = c.w[s];
  const int kend = min(kb + kNB, w);
  int colend = inner ? min((kb & ~(kKB - 1)) + kKB, w) : m;
  if (clip) colend = min(colend, col0 + clip);   // a narrow tile (up to its column block's end)
  const int K = kend - k0, nchunk = (K + 15) >> 4;
  double* Fs = c.F + c.foff[s];
  const int tid = threadIdx.x, wv = tid >> 6, l = tid & 63;
  const int wi = wv >> 1, wj = wv & 1;
  const bool active = !(row0 == col0 && wi < wj) && row0 + 64 * wi < m && col0 + 64 * wj < colend;
  // staging: thread covers (k = idx >> 7, r = idx & 127), idx = tid + 256 q, q < 8
  double st[16];
  auto load = [&](int ch) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int idx = tid + 256 * q, k = 16 * ch + (idx >> 7), r = idx & 127;
      const bool kin = k < K;
      const double* pk = fcol(Fs, m, true, k0 + 16 * ch) + (size_t)(idx >> 7) * fld(m, true, k0 + 16 * ch);
      st[q] = (kin && row0 + r < m) ? pk[row0 + r] : 0.0;
      st[8 + q] = (kin && col0 + r < m) ? pk[col0 + r] : 0.0;
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; q++) {
      const int idx = tid + 256 * q, k = idx >> 7, r = idx & 127;
      Sr[buf][k * LD + r] = st[q];
      Sc[buf][k * LD + r] = st[8 + q];
    }
  };
  // v_mfma_f64_4x4x4f64, as syrk_lds_body: the wave's 64x64 quarter as 16
  // column groups of 4 (p) x 4 row groups of 16 (h), 64 accumulators; lane l
  // holds (row 64wi + 16h + (l & 15), column 64wj + 4p + (l >> 4))
  double acc[16][4];
#pragma unroll
  for (int p = 0; p < 16; p++)
#pragma unroll
    for (int h = 0; h < 4; h++) acc[p][h] = 0.0;
  load(0);
  stash(0);
  __syncthreads();
  for (int ch = 0; ch < nchunk; ch++) {
    const int buf = ch & 1;
    if (ch + 1 < nchunk) load(ch + 1);
    if (active) {
      const double* sr = Sr[buf] + 64 * wi + (l & 15);
      const double* sc = Sc[buf] + 64 * wj + (l & 3);
#pragma unroll
      for (int kk = 0; kk < 4; kk++) {
        const int ko = (4 * kk + (l >> 4)) * LD;
        double rv[4];
#pragma unroll
        for (int h = 0; h < 4; h++) rv[h] = sr[ko + 16 * h];
#pragma unroll
        for (int p = 0; p < 16; p++) {
          const double cv = sc[ko + 4 * p];
#pragma unroll
          for (int h = 0; h < 4; h++) acc[p][h] = __builtin_amdgcn_mfma_f64_4x4x4f64(cv, rv[h], acc[p][h], 0, 0, 0);
        }
      }
    }
    if (ch + 1 < nchunk) stash(buf ^ 1);
    __syncthreads();
  }
  if (!active) return;
  double* Cb = fcol(Fs, m, true, col0 + 64 * wj);   // the wave's columns: one column block
  const int ldc = fld(m, true, col0 + 64 * wj);
#pragma unroll
  for (int p = 0; p < 16; p++) {
    double cold[4];
    const int col = col0 + 64 * wj + 4 * p + (l >> 4);
#pragma unroll
    for (int h = 0; h < 4; h++) {
      const int row = row0 + 64 * wi + 16 * h + (l & 15);
      cold[h] = (row < m && col < colend && row >= col) ? Cb[row + (size_t)(col - col0 - 64 * wj) * ldc] : 0.0;
    }
#pragma unroll
    for (int h = 0; h < 4; h++) {
      const int row = row0 + 64 * wi + 16 * h + (l & 15);
      if (row < m && col < colend && row >= col) Cb[row + (size_t)(col - col0 - 64 * wj) * ldc] = cold[h] - acc[p][h];
    }
  }
}

// ------------------------------------------------------------ partition exchange
// Subtree roots' payloads (partitioned factorisation): the lower triangle of
// the update matrix U (u x u, column-major inside the front at (w, w)), packed
// column by column (column j: rows j..u-1 at j u - j (j - 1) / 2), then the
// update vector fv[w..m).  One workgroup per root, a wave per column.
// tasks: (front, payload offset in buf, u, 0); unpack reverses it.
// tasks: (front, payload offset, u, rank); lane y (grid y) at rank * rstride +
// y * slot in buf (pack: rank 0, rstride 0 -- this rank's send buffer)
template <bool kPack>
__global__ __launch_bounds__(256) void k_xroots(CholDev c, const int4* __restrict__ tasks, double* __restrict__ buf,
                                                long long slot, long long rstride) {
  lane_offset(c);
  const int4 t = tasks[blockIdx.x];
  const int s = t.x, u = t.z, m = c.m[s], w = c.w[s];
  double* Fs = c.F + c.foff[s];
  const bool pk = front_packed(m, w);
  double* v = c.fv + c.voff[s] + w;
  double* b = buf + t.w * rstride + blockIdx.y * slot + t.y;
  const int wv = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (int j = wv; j < u; j += 4) {
    double* col = b + (size_t)j * u - (size_t)j * (j - 1) / 2;
    double* U = fcol(Fs, m, pk, w + j) + w;   // U(i, j) = U[i]
    for (int i = j + l; i < u; i += 64) {
      if (kPack) col[i - j] = U[i];
      else U[i] = col[i - j];
    }
  }
  double* bv = b + (size_t)u * (u + 1) / 2;
  for (int i = threadIdx.x; i < u; i += 256) {
    if (kPack) bv[i] = v[i];
    else v[i] = bv[i];
  }
}

// Solution ranges of the subtrees: (rank, first, end, offset), lane z: pack:
// buf[z * slot + off + k] = xv[first + k]; unpack: xv[first + k] = buf[rank *
// rstride + z * slot + off + k]
template <bool kPack>
__global__ __launch_bounds__(256) void k_xsol(CholDev c, const int4* __restrict__ ranges, double* __restrict__ buf,
                                              long long slot, long long rstride) {
  const int4 r = ranges[blockIdx.y];
  const int n = r.z - r.y;
  double* xv = c.xv + blockIdx.z * c.xst;
  const double* b = buf + (kPack ? 0 : r.x * rstride) + blockIdx.z * slot + r.w;
  for (int k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
    if (kPack) buf[blockIdx.z * slot + r.w + k] = xv[r.y + k];
    else xv[r.y + k] = b[k];
  }
}

// Pivot flags through the solution exchange (every rank must take the same LM
// decision: a bad pivot can be seen by one rank only): pack puts lane y's flag
// at buf[y * slot + at]; reduce ORs every rank's into the flag.
__global__ void k_xflag(CholDev c, double* __restrict__ buf, long long slot, long long at, long long rstride,
                        int ranks, int pack) {
  const int y = threadIdx.x;
  if (pack) {
    buf[y * slot + at] = (double)c.flag[y];
    return;
  }
  int f = 0;
  for (int r = 0; r < ranks; r++) f |= (int)buf[r * rstride + y * slot + at];
  c.flag[y] = f;
}

// diagnostics (PGO_DEBUG_BAD_PIVOT=rank:count): a bad pivot reported by one rank
__global__ void k_set_flag(int* flag, int v) { flag[threadIdx.x] |= v; }

// Distributed top: panels / tail columns between ranks.  Task (front, kn, nb |
// kind << 16, owner); its payload sits in the owner's region of buf (owner *
// rstride), lane y at y * lstride, + loff.  kind 0 (a factored panel): F rows
// [kn + nb, m) x columns [kn, kn + nb) -- the L below the diagonal tile; the
// tile's own L is never stored (store_factor: every reader uses its inverse),
// so its region is not sent (round 6) -- the panel's row-major
// inverse (backward solve), the frontal vector [kn, m) (y and the rows below,
// forward substitution so far); kind 1 (tail): F rows [kn, m) x columns
// [kn, kn + nb).
// Pack: this rank's items (owner == me); unpack: the others'.
template <bool kPack>
__global__ __launch_bounds__(256) void k_xpanel(CholDev c, const int4* __restrict__ tasks,
                                                const long long* __restrict__ offs, double* __restrict__ buf,
                                                long long rstride, int me) {
  lane_offset(c);
  const int4 t = tasks[blockIdx.x];
  if (kPack != (t.w == me)) return;
  const int s = t.x, kn = t.y, nb = t.z & 0xffff, kind = t.z >> 16, m = c.m[s];
  double* b = buf + t.w * rstride + blockIdx.y * offs[2 * blockIdx.x + 1] + offs[2 * blockIdx.x];
  double* Fs = c.F + c.foff[s];
  const int r0 = kind == 0 ? nb : 0, rows = m - kn - r0, tid = threadIdx.x;
  for (int cc = 0; cc < nb; cc++) {
    double* col = fcol(Fs, m, true, kn + cc) + kn + r0;   // (a top front on the blocked path)
    double* bc = b + (size_t)cc * rows;
    for (int r = tid; r < rows; r += 256) {
      if (kPack) bc[r] = col[r];
      else col[r] = bc[r];
    }
  }
  if (kind != 0) return;
  b += (size_t)rows * nb;
  const int vrows = m - kn;
  double* M = c.Tinv + c.toff[s] + (kn / 64) * 4096;
  for (int i = tid; i < 4096; i += 256) {
    if (kPack) b[i] = M[i];
    else M[i] = b[i];
  }
  b += 4096;
  double* v = c.fv + c.voff[s] + kn;
  for (int r = tid; r < vrows; r += 256) {
    if (kPack) b[r] = v[r];
    else v[r] = b[r];
  }
}

// ------------------------------------------------------------ solves
__global__ __launch_bounds__(256) void k_perm_in(CholDev c, const double* __restrict__ b, double scale, int n) {
  lane_offset(c);
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const int o = c.perm[j];
#pragma unroll
  for (int a = 0; a < 3; a++) c.xv[3 * j + a] = scale * b[3 * o + a];
}

__global__ __launch_bounds__(256) void k_perm_out(CholDev c, double* __restrict__ x, int n, long long xstride) {
  lane_offset(c);
  x += blockIdx.y * xstride;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  const int o = c.perm[j];
#pragma unroll
  for (int a = 0; a < 3; a++) x[3 * o + a] = c.xv[3 * j + a];
}

// Diagonal-block solves with the inverted blocks: wave 0, lane i <-> row i.
// y = X v (forward, X = L_bb^-1) and x = X' z (backward); v / z in LDS.

// Backward diagonal step: x = X' z for the owner block (X = L_bb^-1, row-major
// in global memory: lane i reads column i of X' = X[k][i], coalesced over i).
struct TinvCol {
  double m[64];
};
__device__ __forceinline__ void tinv_col_load(TinvCol& t, const double* __restrict__ M, int n) {
  const int i = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 64; k++) t.m[k] = k < n ? M[k * 64 + i] : 0.0;
}
__device__ __forceinline__ double tinv_col_dot(const TinvCol& t, const double* z, int n) {
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 64; k++)
    if (k < n) acc = fma(t.m[k], z[k], acc);
  return acc;
}

// Frontal vectors of a level before its factorisation: own rows from the
// permuted right-hand side, below rows zero, plus the children's update
// vectors (fixed order).  The factorisation then carries them as an extra
// column (forward substitution fused into the panels).
__global__ __launch_bounds__(256) void k_vec_assemble(CholDev c, const int* __restrict__ list) {
  lane_offset(c);
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* v = sm;                  // m
  const int s = list[blockIdx.x];
  const int m = c.m[s], w = c.w[s];
  const int* rows = c.rows + c.rptr[s];
  const int tid = threadIdx.x;
  for (int r = tid; r < m; r += 256) v[r] = r < w ? c.xv[3 * rows[r / 3] + r % 3] : 0.0;
  __syncthreads();
  for (int q = c.cptr[s]; q < c.cptr[s + 1]; q++) {
    const int ch = c.children[q];
    const int uc = c.m[ch] - c.w[ch];
    const double* uv = c.fv + c.voff[ch] + c.w[ch];
    const int* rel = c.ea_rel + c.ea_ptr[ch];
    for (int t = tid; t < uc; t += 256) v[3 * rel[t / 3] + t % 3] += uv[t];
    __syncthreads();
  }
  double* fv = c.fv + c.voff[s];
  for (int r = tid; r < m; r += 256) fv[r] = v[r];
}

// acc[0..N) of each lane -> acc[0..N/2): lanes with bit N/2 set keep the upper
// half, the other half goes to the partner lane (recursive halving).  After
// halve<64> ... halve<2>, acc[0] of lane q is the wave sum of column q.
template <int N>
__device__ __forceinline__ void halve(double* acc, int lane) {
  const bool up = lane & (N / 2);
#pragma unroll
  for (int i = 0; i < N / 2; i++) {
    const double send = up ? acc[i] : acc[i + N / 2];
    const double keep = up ? acc[i + N / 2] : acc[i];
    acc[i] = keep + __shfl_xor(send, N / 2);
  }
}

// One wave's share of a backward partial product: lane = row (r, r + 256, ...
// below r1), NC column accumulators, summed over the wave; lane q < NC returns
// column q's sum.  Every column load is issued unconditionally (columns past
// ncol re-read the last one and are not accumulated): a predicated load per
// column made the compiler branch around each one and wait on it, NC serial
// memory latencies.  NC = 16 serves the narrow fronts near the leaves with a
// quarter of the reduction.
template <int NC, int STRIDE = 256>
__device__ __forceinline__ double bwd_part_wave(const CholDev& c, const double* L, const int* rows, int ld,
                                                int ncol, int rbeg, int r1, int lane) {
  double acc[NC];
#pragma unroll
  for (int q = 0; q < NC; q++) acc[q] = 0.0;
  for (int r = rbeg; r < r1; r += STRIDE) {
    const double xr = c.xv[3 * rows[r / 3] + r % 3];
    const double* Lr = L + r;
    double lv[NC];
#pragma unroll
    for (int q = 0; q < NC; q++) lv[q] = Lr[(size_t)min(q, ncol - 1) * ld];
#pragma unroll
    for (int q = 0; q < NC; q++)
      if (q < ncol) acc[q] += lv[q] * xr;
  }
  if constexpr (NC == 64) {
    halve<64>(acc, lane);
    halve<32>(acc, lane);
  }
  halve<16>(acc, lane);
  halve<8>(acc, lane);
  halve<4>(acc, lane);
  halve<2>(acc, lane);
  double v = acc[0];
  if constexpr (NC == 16) {   // lane l: column l & 15 over its 16-lane group; add the 4 groups
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    v = lane < 16 ? v : 0.0;
  }
  return v;
}

// Backward partial product: part[slot][j] = sum over rows [r0, r0+kBwdRows) of
// L[r, c0+j] x_r (rows below the pivot columns; x gathered from xv).
__global__ __launch_bounds__(256) void k_bwd_part(CholDev c, const int4* __restrict__ tasks,
                                                  double* __restrict__ part) {
  lane_offset(c);
  part += blockIdx.y * c.pst;
  __shared__ double red[4][64];
  const int4 t = tasks[blockIdx.x];
  const int s = t.x, c0 = t.y, r0 = t.z, slot = t.w;
  const int m = c.m[s], w = c.w[s];
  const int ncol = min(64, w - c0), r1 = min(r0 + kBwdRows, m);
  const bool pk = front_packed(m, w);
  const double* L = fcol(c.F + c.foff[s], m, pk, c0);   // columns c0 .. c0 + 63: one column block
  const int ld = fld(m, pk, c0);
  const int* rows = c.rows + c.rptr[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (ncol > 16) {
    // wave wv: columns [16 wv, 16 wv + 16) over all the task's rows (lane =
    // row, stride 64): 16 accumulators per lane reduced over the wave -- a
    // quarter of the shuffles of 64 per lane, and no cross-wave sum
    const int nw = min(16, ncol - 16 * wv);
    if (nw <= 0) {
      if (lane < 16) part[(size_t)slot * 64 + 16 * wv + lane] = 0.0;
      return;
    }
    const double v = bwd_part_wave<16, 64>(c, L + (size_t)(16 * wv) * ld, rows, ld, nw, r0 + lane, r1, lane);
    if (lane < 16) part[(size_t)slot * 64 + 16 * wv + lane] = v;
    return;
  }
  if (r0 + 64 * wv >= r1)
    red[wv][lane] = 0.0;   // no rows for this wave (small fronts): skip the reduction
  else
    red[wv][lane] = bwd_part_wave<16>(c, L, rows, ld, ncol, r0 + tid, r1, lane);
  __syncthreads();
  if (tid < 64) part[(size_t)slot * 64 + tid] = (red[0][tid] + red[1][tid]) + (red[2][tid] + red[3][tid]);
}

// Backward init of a level: z_j = y_j - sum of the block's partials (fixed
// order); the owner of the last block then solves it.
__global__ __launch_bounds__(256) void k_bwd_init(CholDev c, const int4* __restrict__ tasks,
                                                  const int2* __restrict__ pref, const double* __restrict__ part) {
  lane_offset(c);
  part += blockIdx.y * c.pst;
  __shared__ double z[64];
  const int4 t = tasks[blockIdx.x];
  const int s = t.x, c0 = t.y, c1 = t.z, owner = t.w;
  const int n2 = c1 - c0;
  const int2 pr = pref[blockIdx.x];
  double* fv = c.fv + c.voff[s];
  const int* rows = c.rows + c.rptr[s];
  const int tid = threadIdx.x;
  TinvCol tc;
  if (owner >= 0 && tid < 64) tinv_col_load(tc, c.Tinv + c.toff[s] + owner * 4096, n2);   // in flight
  if (tid < n2) {
    double acc = 0.0;
    for (int p = 0; p < pr.y; p++) acc += part[(size_t)(pr.x + p) * 64 + tid];
    z[tid] = fv[c0 + tid] - acc;
  }
  __syncthreads();
  if (owner < 0) {
    if (tid < n2) fv[c0 + tid] = z[tid];
    return;
  }
  if (tid < 64) {
    const double x = tinv_col_dot(tc, z, n2);
    if (tid < n2) {
      fv[c0 + tid] = x;
      c.xv[3 * rows[(c0 + tid) / 3] + (c0 + tid) % 3] = x;
    }
  }
}

// Backward step b: z_j -= L[block b, j]' x_b for the task's columns (< 64 b);
// the owner of block b-1 then solves it.
__global__ __launch_bounds__(256) void k_bwd_step(CholDev c, const int4* __restrict__ tasks, int b) {
  lane_offset(c);
  __shared__ double xbk[64];
  __shared__ double z[64];
  const int4 t = tasks[blockIdx.x];
  const int s = t.x, c0 = t.y, c1 = t.z, owner = t.w;
  const int n2 = c1 - c0;
  const int m = c.m[s], w = c.w[s];
  const double* L = c.F + c.foff[s];
  double* fv = c.fv + c.voff[s];
  const int* rows = c.rows + c.rptr[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int jb = b * 64, nbk = min(64, w - jb);
  TinvCol tc;
  if (owner >= 0 && tid < 64) tinv_col_load(tc, c.Tinv + c.toff[s] + owner * 4096, n2);   // in flight
  // wave wv: columns c0 + 16 wv + q (q < 16), lane = row jb + lane of block b
  double acc[16];
  const bool rin = lane < nbk;
  const bool pk = front_packed(m, w);
  const double* Lr = fcol(L, m, pk, c0 + 16 * wv) + (jb + lane);   // (c0: a column block's start)
  const int ld = fld(m, pk, c0);
#pragma unroll
  for (int q = 0; q < 16; q++) acc[q] = (rin && c0 + 16 * wv + q < c1) ? Lr[(size_t)q * ld] : 0.0;
  if (tid < 64) xbk[tid] = tid < nbk ? fv[jb + tid] : 0.0;
  __syncthreads();
  const double xl = xbk[lane];
#pragma unroll
  for (int q = 0; q < 16; q++) acc[q] *= xl;
  halve<16>(acc, lane);   // lane l: column (l & 15), summed over its 16-lane group
  halve<8>(acc, lane);
  halve<4>(acc, lane);
  halve<2>(acc, lane);
  double tsum = acc[0];
  tsum += __shfl_xor(tsum, 16);
  tsum += __shfl_xor(tsum, 32);
  const int j = c0 + 16 * wv + lane;
  if (lane < 16 && j < c1) z[j - c0] = fv[j] - tsum;
  __syncthreads();
  if (owner < 0) {
    if (tid < n2) fv[c0 + tid] = z[tid];
    return;
  }
  if (tid < 64) {
    const double x = tinv_col_dot(tc, z, n2);
    if (tid < n2) {
      fv[c0 + tid] = x;
      c.xv[3 * rows[(c0 + tid) / 3] + (c0 + tid) % 3] = x;
    }
  }
}

// All backward steps of a level in one launch (replacing one k_bwd_step launch
// per block): the workgroup of block j of a front takes z_j from k_bwd_init,
// then for b = nblk-1 down to j+1 -- as soon as block b's x is published by its
// workgroup (in-launch hand-off: sc1 stores, flag, sc1 loads; the flags are the
// factorisation's stepflag, zeroed per solve) -- z_j -= L[block b, j]' x_b with
// k_bwd_step's arithmetic, then solves x_j = X_jj' z_j and publishes it.  The
// same operations in the same order as the step launches: bitwise their result.
// Tasks are ordered by distance from the front's last block, so a workgroup
// waits only on workgroups dispatched before it; the waits are bounded.
__global__ __launch_bounds__(256) void k_bwd_chain(CholDev c, const int4* __restrict__ tasks) {
  lane_offset(c);
  __shared__ double xbk[64];
  __shared__ double z[64];
  const int4 t = tasks[blockIdx.x];
  const int s = t.x, c0 = t.y, c1 = t.z, jblk = t.w;
  const int n2 = c1 - c0;
  const int m = c.m[s], w = c.w[s], nblk = (w + 63) / 64;
  const double* L = c.F + c.foff[s];
  double* fv = c.fv + c.voff[s];
  const int* rows = c.rows + c.rptr[s];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  TinvCol tc;
  if (tid < 64) {
    tinv_col_load(tc, c.Tinv + c.toff[s] + jblk * 4096, n2);   // in flight
    z[tid] = tid < n2 ? fv[c0 + tid] : 0.0;                    // k_bwd_init's z (earlier launch)
  }
  for (int b = nblk - 1; b > jblk; b--) {
    const int jb = b * 64, nbk = min(64, w - jb);
    double acc[16];
    const bool rin = lane < nbk;
    const bool pk = front_packed(m, w);
    const double* Lr = fcol(L, m, pk, c0 + 16 * wv) + (jb + lane);   // (c0: a column block's start)
    const int ld = fld(m, pk, c0);
#pragma unroll
    for (int q = 0; q < 16; q++) acc[q] = (rin && c0 + 16 * wv + q < c1) ? Lr[(size_t)q * ld] : 0.0;
    if (b < nblk - 1) wait_step(c, c.stepflag + s, nblk - 1 - b);   // x_b from its chain workgroup
    if (tid < 64) xbk[tid] = tid < nbk ? ld_sc1(fv + jb + tid) : 0.0;
    __syncthreads();
    const double xl = xbk[lane];
#pragma unroll
    for (int q = 0; q < 16; q++) acc[q] *= xl;
    halve<16>(acc, lane);
    halve<8>(acc, lane);
    halve<4>(acc, lane);
    halve<2>(acc, lane);
    double tsum = acc[0];
    tsum += __shfl_xor(tsum, 16);
    tsum += __shfl_xor(tsum, 32);
    const int j = c0 + 16 * wv + lane;
    if (lane < 16 && j < c1) z[j - c0] = z[j - c0] - tsum;
    __syncthreads();
  }
  if (tid < 64) {
    const double x = tinv_col_dot(tc, z, n2);
    if (tid < n2) {
      st_sc1(fv + c0 + tid, x);
      c.xv[3 * rows[(c0 + tid) / 3] + (c0 + tid) % 3] = x;
    }
  }
  publish_step(c.stepflag + s, nblk - 1 - jblk);
}

// ------------------------------------------------------------ marginals
// Marginal covariance of one pose (GTSAM Marginals::marginalCovariance): with
// H_perm = L L', the 3x3 block of H^-1 at the pose is Y'Y, Y = L^-1 [e_a e_b e_c]
// for the pose's three (permuted) columns.  Y is nonzero only on the fronts
// from the pose's supernode up to the root, so one workgroup per pose walks
// that path: per 64-column block y_b = X_bb v_b (X = inverted diagonal block),
// the rows below get v -= L y_b, the Gram of the y blocks accumulates, and the
// update vector moves to the parent front (extend-add of a single child).
// v lives in a per-workgroup global scratch (two buffers of 3 x maxm).
__global__ __launch_bounds__(256) void k_marginals(CholDev c, const int2* __restrict__ start, int maxm,
                                                   double* __restrict__ scratch, double* __restrict__ out) {
  lane_offset(c);
  __shared__ double ys[3][64];
  __shared__ double red[6][4];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int2 st = start[blockIdx.x];   // (supernode, local row of the pose's first column)
  double* va = scratch + (size_t)blockIdx.x * 6 * maxm;
  double* vb = va + 3 * (size_t)maxm;
  int s = st.x;
  {
    const int m = c.m[s];
    for (int r = 0; r < 3; r++)
      for (int i = tid; i < m; i += 256) va[r * maxm + i] = i == st.y + r ? 1.0 : 0.0;
  }
  double g[6] = {0, 0, 0, 0, 0, 0};    // (aa, ab, ac, bb, bc, cc)
  __syncthreads();
  while (s >= 0) {
    const int m = c.m[s], w = c.w[s];
    const double* L = c.F + c.foff[s];
    for (int c0 = 0; c0 < w; c0 += 64) {
      const int n2 = min(64, w - c0);
      if (tid < 64) {
        const double* M = c.Tinv + c.toff[s] + (c0 / 64) * 4096;   // row-major X_bb
        double y0 = 0, y1 = 0, y2 = 0;
        if (tid < n2)
          for (int k = 0; k <= tid; k++) {
            const double x = M[tid * 64 + k];
            y0 = fma(x, va[c0 + k], y0);
            y1 = fma(x, va[maxm + c0 + k], y1);
            y2 = fma(x, va[2 * maxm + c0 + k], y2);
          }
        ys[0][tid] = y0;
        ys[1][tid] = y1;
        ys[2][tid] = y2;
        g[0] += y0 * y0;
        g[1] += y0 * y1;
        g[2] += y0 * y2;
        g[3] += y1 * y1;
        g[4] += y1 * y2;
        g[5] += y2 * y2;
      }
      __syncthreads();
      const bool pk = front_packed(m, w);
      const double* Lb = fcol(L, m, pk, c0);   // columns c0 .. c0 + n2: one column block
      const int ld = fld(m, pk, c0);
      for (int r = c0 + n2 + tid; r < m; r += 256) {
        double a0 = 0, a1 = 0, a2 = 0;
        for (int k = 0; k < n2; k++) {
          const double l = Lb[r + (size_t)k * ld];
          a0 = fma(l, ys[0][k], a0);
          a1 = fma(l, ys[1][k], a1);
          a2 = fma(l, ys[2][k], a2);
        }
        va[r] -= a0;
        va[maxm + r] -= a1;
        va[2 * maxm + r] -= a2;
      }
      __syncthreads();
    }
    const int p = c.parent[s];
    if (p >= 0) {
      const int mp = c.m[p];
      for (int r = 0; r < 3; r++)
        for (int i = tid; i < mp; i += 256) vb[r * maxm + i] = 0.0;
      __syncthreads();
      const int* rel = c.ea_rel + c.ea_ptr[s];
      for (int t = tid; t < m - w; t += 256) {
        const int q = 3 * rel[t / 3] + t % 3;
        for (int r = 0; r < 3; r++) vb[r * maxm + q] = va[r * maxm + w + t];
      }
      __syncthreads();
      double* tmp = va;
      va = vb;
      vb = tmp;
    }
    s = p;
  }
  // Gram reduction (wave butterflies, then the 4 waves)
#pragma unroll
  for (int q = 0; q < 6; q++) {
    double v = g[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if (lane == 0) red[q][wv] = v;
  }
  __syncthreads();
  if (tid < 9) {
    const int i = tid / 3, j = tid % 3;
    const int a = i <= j ? i : j, b = i <= j ? j : i;
    const int q = a == 0 ? b : (a == 1 ? 2 + b : 5);
    out[(size_t)blockIdx.x * 9 + tid] = (red[q][0] + red[q][1]) + (red[q][2] + red[q][3]);
  }
}

// ------------------------------------------------------------ host drivers
#define CH_TRY(x)                       \
  do {                                  \
    hipError_t e_ = (x);                \
    if (e_ != hipSuccess) return e_;    \
  } while (0)

// numeric workspaces of nb lanes (fronts zeroed: the upper triangles stay zero)
static void free_numeric(CholPlan& P) {
  void* ptrs[] = {P.F, P.Tinv, P.fv, P.xv, P.d_flag, P.d_lambda, P.d_partial, P.d_stepflag, P.d_xsend, P.d_xrecv,
                  P.d_xprecv};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  P.F = P.Tinv = P.fv = P.xv = P.d_lambda = P.d_partial = nullptr;
  P.d_xsend = P.d_xrecv = P.d_xprecv = nullptr;
  P.d_flag = P.d_stepflag = nullptr;
  P.batch = 0;
  P.num_cap = NumericCap();
}

// partition exchange slots per lane (doubles): the subtree roots' payloads, the
// solution ranges + the pivot flag (xsol_max), the largest of the two
static long long xroot_slot(const CholPlan& P) { return std::max(P.xmax, 1LL); }
static long long xsol_slot(const CholPlan& P) { return P.xsol_max + 1; }

// The workspaces' element counts for nb lanes of the plan as it is
static NumericCap numeric_need(const CholPlan& P, int nb) {
  NumericCap c;
  c.F = nb * std::max<long long>(P.ftotal, 1);
  c.T = nb * std::max<long long>(2 * P.ttotal, 1);
  c.v = (long long)nb * std::max(P.vtotal, 1);
  c.x = (long long)nb * std::max(3 * P.n, 1);
  c.sf = (long long)nb * std::max(P.ns, 1);
  c.part = (long long)nb * std::max(P.npart, 1) * 64;
  return c;
}

// With room_for_growth (the appendable one-rank plan, chol_append), every
// workspace gets 1/32 more than it needs, so the next appended poses reuse it.
static hipError_t alloc_numeric(CholPlan& P, int nb, hipStream_t s) {
  NumericCap need = numeric_need(P, nb), cap = need;
  if (P.part_size <= 1) {
    for (long long* v : {&cap.F, &cap.T, &cap.v, &cap.x, &cap.sf, &cap.part}) *v += *v / 32 + 4096;
  }
  CH_TRY(hipMalloc((void**)&P.F, cap.F * sizeof(double)));
  CH_TRY(hipMalloc((void**)&P.Tinv, cap.T * sizeof(double)));
  CH_TRY(hipMalloc((void**)&P.fv, cap.v * sizeof(double)));
  CH_TRY(hipMalloc((void**)&P.xv, cap.x * sizeof(double)));
  CH_TRY(hipMalloc((void**)&P.d_flag, nb * sizeof(int)));
  CH_TRY(hipMalloc((void**)&P.d_stepflag, cap.sf * sizeof(int)));
  CH_TRY(hipMalloc((void**)&P.d_lambda, nb * sizeof(double)));
  CH_TRY(hipMalloc((void**)&P.d_partial, cap.part * sizeof(double)));
  CH_TRY(hipMemsetAsync(P.F, 0, need.F * sizeof(double), s));
  {   // partition exchange buffers, nb lanes per rank
    const long long xs = P.part_size > 1 ? std::max(xroot_slot(P), xsol_slot(P)) : 1;
    CH_TRY(hipMalloc((void**)&P.d_xsend, sizeof(double) * xs * nb));
    CH_TRY(hipMalloc((void**)&P.d_xrecv, sizeof(double) * xs * nb * std::max(P.part_size, 1)));
    const long long xp = P.part_size > 1 ? std::max(P.xp_rslot, 1LL) : 1;
    CH_TRY(hipMalloc((void**)&P.d_xprecv, sizeof(double) * xp * nb * std::max(P.part_size, 1)));
  }
  P.batch = nb;
  P.num_cap = cap;
  return hipStreamSynchronize(s);
}

// The plan changed shape (chol_append): keep the workspaces when they hold it
// (the fronts zeroed again: their layout moved), else allocate anew.
static hipError_t refresh_numeric(CholPlan& P, int nb, hipStream_t s) {
  const NumericCap need = numeric_need(P, nb), &cap = P.num_cap;
  if (P.F && P.part_size <= 1 && nb <= P.batch && need.F <= cap.F && need.T <= cap.T && need.v <= cap.v &&
      need.x <= cap.x && need.sf <= cap.sf && need.part <= cap.part) {
    CH_TRY(hipMemsetAsync(P.F, 0, need.F * sizeof(double), s));
    P.batch = nb;
    return hipSuccess;
  }
  CH_TRY(hipStreamSynchronize(s));
  free_numeric(P);
  return alloc_numeric(P, nb, s);
}

hipError_t chol_set_batch(CholPlan& P, int nb, hipStream_t s) {
  if (nb == P.batch) return hipSuccess;
  CH_TRY(hipStreamSynchronize(s));
  free_numeric(P);
  const hipError_t e = alloc_numeric(P, nb, s);
  if (e != hipSuccess) {   // keep one lane
    (void)hipGetLastError();
    free_numeric(P);
    CH_TRY(alloc_numeric(P, 1, s));
    return e;
  }
  return hipSuccess;
}

// The plan's index arrays live in one device allocation, filled by one copy
// from a pinned staging buffer (a plan refresh is one upload, not ~45
// allocations and pageable copies).
namespace {
struct BlobItem {
  void** dptr;
  const void* src;
  size_t bytes, off;
};
template <class T>
void blob_add(std::vector<BlobItem>& items, T** dptr, const std::vector<T>& h) {
  items.push_back({(void**)dptr, h.data(), h.size() * sizeof(T), 0});
}
}  // namespace

// (pgo_symbolic.cpp's thread pool in the library; this serial stand-in only
// for the microbenchmarks that compile this file alone)
__attribute__((weak)) void plan_parallel(int ntask, const std::function<void(int)>& fn) {
  for (int t = 0; t < ntask; t++) fn(t);
}

static hipError_t upload_index(CholPlan& P, hipStream_t s) {
  std::vector<int4> own, foreign, sown, sforeign;   // partition exchange lists (this rank's roots / the others')
  std::vector<long long> xo(2 * P.xp_tasks.size());
  if (P.part_size > 1 && (long long)P.part_size * std::max(P.xmax, P.xsol_max) >= (1LL << 31))
    return hipErrorInvalidValue;   // int offsets
  for (size_t q = 0; q < P.xroot.size(); q++) {
    const int sr = P.xroot[q], r = P.xroot_rank[q], u = P.m[sr] - P.w[sr];
    if (u == 0) continue;
    if (r == P.part_rank) own.push_back(make_int4(sr, (int)P.xroot_off[q], u, 0));
    else if (P.parent[sr] >= 0) foreign.push_back(make_int4(sr, (int)P.xroot_off[q], u, r));
  }
  for (const int4& rg : P.xsol_ranges) (rg.x == P.part_rank ? sown : sforeign).push_back(rg);
  P.n_xown = (int)own.size();
  P.n_xforeign = (int)foreign.size();
  P.n_xsol_own = (int)sown.size();
  P.n_xsol_foreign = (int)sforeign.size();
  for (size_t q = 0; q < P.xp_tasks.size(); q++) {
    xo[2 * q] = P.xp_loff[q];
    xo[2 * q + 1] = P.xp_lstride[q];
  }
  std::vector<BlobItem> it;
  blob_add(it, &P.d_toff, P.toff);
  blob_add(it, &P.d_m, P.m);
  blob_add(it, &P.d_w, P.w);
  blob_add(it, &P.d_voff, P.voff);
  blob_add(it, &P.d_rptr, P.rptr);
  blob_add(it, &P.d_rows, P.rows);
  blob_add(it, &P.d_foff, P.foff);
  blob_add(it, &P.d_cptr, P.cptr);
  blob_add(it, &P.d_children, P.children);
  blob_add(it, &P.d_ea_rel, P.ea_rel);
  blob_add(it, &P.d_ea_ptr, P.ea_ptr);
  blob_add(it, &P.d_parent, P.parent);
  blob_add(it, &P.d_asm_front, P.asm_front);
  blob_add(it, &P.d_asm_li, P.asm_li);
  blob_add(it, &P.d_asm_lj, P.asm_lj);
  blob_add(it, &P.d_asm_ptr, P.asm_ptr);
  blob_add(it, &P.d_asm_src, P.asm_src);
  blob_add(it, &P.d_dg_front, P.dg_front);
  blob_add(it, &P.d_dg_loc, P.dg_loc);
  blob_add(it, &P.d_perm, P.perm);
  blob_add(it, &P.d_small, P.small_list);
  blob_add(it, &P.d_level_fronts, P.level_fronts);
  blob_add(it, &P.d_potrf, P.potrf_list);
  blob_add(it, &P.d_bwd, P.bwd_tasks);
  blob_add(it, &P.d_bwdc, P.bwdc_tasks);
  blob_add(it, &P.d_bwd_pref, P.bwd_pref);
  blob_add(it, &P.d_bwd_part, P.bwd_part_tasks);
  blob_add(it, &P.d_syrk, P.syrk_tasks);
  blob_add(it, &P.d_sdiag, P.sdiag_tasks);
  blob_add(it, &P.d_col, P.col_tasks);
  blob_add(it, &P.d_xown, own);
  blob_add(it, &P.d_xforeign, foreign);
  blob_add(it, &P.d_xsol_own, sown);
  blob_add(it, &P.d_xsol_foreign, sforeign);
  blob_add(it, &P.d_xp, P.xp_tasks);
  blob_add(it, &P.d_xp_off, xo);
  blob_add(it, &P.d_at_iptr, P.at_iptr);
  blob_add(it, &P.d_at_items, P.at_items);
  blob_add(it, &P.d_ea_tasks, P.ea_tasks);
  blob_add(it, &P.d_ea_pairs, P.ea_pairs);
  size_t total = 0;
  for (BlobItem& b : it) {
    b.off = total;
    total += (std::max<size_t>(b.bytes, 1) + 255) / 256 * 256;
  }
  CH_TRY(hipStreamSynchronize(s));   // the staging buffer and the old blob are idle
  if (total > P.blob_cap) {
    if (P.d_blob) (void)hipFree(P.d_blob);
    P.d_blob = nullptr;
    P.blob_cap = 0;
    const size_t cap = total + total / 8;
    CH_TRY(hipMalloc(&P.d_blob, cap));
    P.blob_cap = cap;
  }
  if (total > P.h_blob_cap) {
    if (P.h_blob) (void)hipHostFree(P.h_blob);
    P.h_blob = nullptr;
    P.h_blob_cap = 0;
    const size_t cap = total + total / 8;
    CH_TRY(hipHostMalloc(&P.h_blob, cap, hipHostMallocDefault));
    P.h_blob_cap = cap;
  }
  char* h = static_cast<char*>(P.h_blob);
  char* d = static_cast<char*>(P.d_blob);
  // the host copies into the pinned staging on the plan's thread pool, in
  // pieces of <= 1 MiB (the plan refresh of the live path uploads ~25 MB)
  std::vector<std::pair<size_t, size_t>> piece;   // (item, byte offset)
  for (size_t q = 0; q < it.size(); q++) {
    *it[q].dptr = d + it[q].off;
    for (size_t o = 0; o < it[q].bytes; o += (1u << 20)) piece.emplace_back(q, o);
  }
  plan_parallel((int)piece.size(), [&](int t) {
    const BlobItem& b = it[piece[t].first];
    const size_t o = piece[t].second, n = std::min<size_t>(1u << 20, b.bytes - o);
    memcpy(h + b.off + o, static_cast<const char*>(b.src) + o, n);
  });
  CH_TRY(hipMemcpyAsync(d, h, total, hipMemcpyHostToDevice, s));
  return hipSuccess;
}

hipError_t chol_upload_assembly(CholPlan& P, hipStream_t s) {
  CH_TRY(upload_index(P, s));
  return hipStreamSynchronize(s);
}

// an opt-in environment knob set to 1
static bool knob_on(const char* name) {
  const char* v = getenv(name);
  return v && atoi(v) == 1;
}

// PGO_STEP_SPLIT: diagonal tiles x lanes from which a panel step runs as three
// launches (k_step_diag, k_panel_syrk_lds on P.side5, k_first_trsm) instead of
// one k_step; 0 = never, the default since round 5: bitwise the same factor
// (final error and pose hash equal at 0 / 64 / 1 on C2 and C3), and the
// replays measured slower with it (C3 8.39 / 17.00 ms at 1 / 3 lanes against
// 8.34 / 16.81 without, profiles/r05a_ab_split.txt; round 4's r04e A/B: within
// noise)
static int step_split_threshold() {
  static const int v = getenv("PGO_STEP_SPLIT") ? atoi(getenv("PGO_STEP_SPLIT")) : 0;
  return v;
}

hipError_t chol_upload(CholPlan& P, hipStream_t s) {
  CH_TRY(upload_index(P, s));
  CH_TRY(P.F ? refresh_numeric(P, std::max(P.batch, 1), s) : alloc_numeric(P, std::max(P.batch, 1), s));
  if (!P.side) {   // PGO_SIDE_PRIORITY=1: the plain Schur tiles' stream at the lowest dispatch
                   // priority (measured on C3: 22.0 vs 26.0 it/s -- the starved tiles hold
                   // the level ends back more than the panel chain gains -- so off)
    int least = 0, greatest = 0;
    const char* pr = getenv("PGO_SIDE_PRIORITY");
    // PGO_SIDE_CUMASK=r (A/B): the plain Schur tiles' stream kept off r of every
    // 32 CUs (PGO_SIDE_CUMASK_MODE=1: off CUs i with (i / 8) % 32 < r), so the
    // panel chain's workgroups always find CUs free of them.  Measured on C3:
    // 13.8 / 20.3 ms against 8.5 / 17.0 ms replays at 1 / 3 lanes
    // (profiles/r04j_ab_queues_cumask_lookahead.txt), so off
    const int cum = getenv("PGO_SIDE_CUMASK") ? atoi(getenv("PGO_SIDE_CUMASK")) : 0;
    if (cum > 0) {
      const int mode = getenv("PGO_SIDE_CUMASK_MODE") ? atoi(getenv("PGO_SIDE_CUMASK_MODE")) : 0;
      int dev = 0, ncu = 0;
      CH_TRY(hipGetDevice(&dev));
      CH_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
      std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
      for (int i = 0; i < ncu; i++) {
        const bool off_cu = mode == 1 ? (i / 8) % 32 < cum : i % 32 < cum;
        if (!off_cu) mask[i / 32] |= 1u << (i % 32);
      }
      CH_TRY(hipExtStreamCreateWithCUMask(&P.side, (uint32_t)mask.size(), mask.data()));
    } else if (pr && pr[0] == '1' && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      CH_TRY(hipStreamCreateWithPriority(&P.side, hipStreamNonBlocking, least));
    else
      CH_TRY(hipStreamCreateWithFlags(&P.side, hipStreamNonBlocking));
    CH_TRY(hipStreamCreateWithFlags(&P.side2, hipStreamNonBlocking));
    CH_TRY(hipStreamCreateWithFlags(&P.side3, hipStreamNonBlocking));
    // the streams of opt-in knobs exist only with their knob (with
    // GPU_MAX_HW_QUEUES=4 every idle stream still takes a slot in the
    // round-robin mapping of streams to hardware queues)
    if (step_split_threshold() > 0) CH_TRY(hipStreamCreateWithFlags(&P.side5, hipStreamNonBlocking));
    if (knob_on("PGO_WAVE_STREAMS")) {
      CH_TRY(hipStreamCreateWithFlags(&P.side6, hipStreamNonBlocking));
      CH_TRY(hipEventCreateWithFlags(&P.ev6, hipEventDisableTiming));
    }
    // the deferred far updates fill the CUs the panel chain leaves idle: their
    // stream at the lowest dispatch priority (PGO_FAR_PRIORITY=0: default)
    const char* fp = getenv("PGO_FAR_PRIORITY");
    if (!knob_on("PGO_FAR"))
      ;
    else if (!(fp && fp[0] == '0') && hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      CH_TRY(hipStreamCreateWithPriority(&P.side4, hipStreamNonBlocking, least));
    else
      CH_TRY(hipStreamCreateWithFlags(&P.side4, hipStreamNonBlocking));
    for (auto& e : P.evs) CH_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (auto& e : P.fev) CH_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    // the four-wave small fronts ask for up to 256 x 33 doubles of LDS (> 64 KiB;
    // 160 KiB per CU on gfx950)
    (void)hipFuncSetAttribute((const void*)k_front_wave4<16>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    (void)hipFuncSetAttribute((const void*)k_front_wave4<kWaveW>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  }
  return hipSuccess;   // (the fronts' zeroing runs on, stream-ordered before any use)
}

void chol_free(CholPlan& P) {
  free_numeric(P);
  if (P.d_blob) (void)hipFree(P.d_blob);
  if (P.h_blob) (void)hipHostFree(P.h_blob);
  for (hipEvent_t e : P.evs)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : P.fev)
    if (e) (void)hipEventDestroy(e);
  if (P.side) (void)hipStreamDestroy(P.side);
  if (P.side2) (void)hipStreamDestroy(P.side2);
  if (P.side3) (void)hipStreamDestroy(P.side3);
  if (P.side4) (void)hipStreamDestroy(P.side4);
  if (P.side5) (void)hipStreamDestroy(P.side5);
  if (P.side6) (void)hipStreamDestroy(P.side6);
  if (P.ev6) (void)hipEventDestroy(P.ev6);
  P.sched_scratch.p.reset();   // (not touched by the assignment below)
  P = CholPlan();
}

const char* kernel_family_name(int f) {
  static const char* const names[kFamCount] = {
      "k_assemble_tile", "(unused)", "k_perm_in+k_perm_out", "(unused)", "k_vec_assemble",
      "k_front_wave", "k_front_small", "k_panel_first", "k_step", "k_panel_syrk_lds", "k_panel_syrk128",
      "k_bwd_part", "k_bwd_init", "k_bwd_step", "k_step_diag", "k_col_trsm"};
  return f >= 0 && f < kFamCount ? names[f] : "?";
}

// Launch through the profile: with prof, the launch is bracketed by dispatch
// events on its stream and recorded with its family and algorithmic work
// (cost(): {flops, bytes}, evaluated only for profiled launches).
template <typename Cost, typename K, typename... Args>
static void launch(LaunchProfile* prof, int fam, Cost cost, K kern, dim3 grid, dim3 block, size_t smem,
                   hipStream_t s, Args... args) {
  if (grid.x == 0 || grid.y == 0 || grid.z == 0) return;   // an empty task list: no dispatch at all
  if (prof && prof->used < prof->cap) {
    const int u = prof->used++;
    const double2 fb = cost();
    prof->fam[u] = fam;
    prof->flops[u] = fb.x;
    prof->bytes[u] = fb.y;
    if (prof->grid) prof->grid[u] = (int)grid.x;
    if (prof->tag) prof->tag[u] = prof->cur_tag;
    hipExtLaunchKernelGGL(kern, grid, block, smem, s, prof->ev[2 * u], prof->ev[2 * u + 1], 0, args...);
  } else {
    hipLaunchKernelGGL(kern, grid, block, smem, s, args...);
  }
}

// Algorithmic HBM bytes of level L's k_assemble_tile (the profiles' family
// table): children's elements read + tile elements written, 8 B each, plus the
// H slots read.  Computed on first use (profiled runs only), cached in the level.
double level_at_bytes(const CholPlan& P, int L) {
  const CholLevel& lv = P.levels[L];
  if (lv.at_bytes >= 0) return lv.at_bytes;
  // sum_{t=A..B} clamp(t, 0, c) in closed form (G(x) = sum_{t=1..x} min(t, c))
  auto G = [](long long x, long long c) -> long long {
    if (x <= 0) return 0;
    return x <= c ? x * (x + 1) / 2 : c * (c + 1) / 2 + (x - c) * c;
  };
  double bytes = 0;
  for (int q = lv.ea_off[0]; q < lv.ea_off[0] + lv.ea_cnt[0]; q++) {
    const int4 t = P.ea_tasks[q];
    double e = 0, h = 0;   // children's elements read + tile elements written; H slots read
    for (int k = 0; k < t.w; k++) {   // rows r < nr of a child rectangle: min(max(a0 + r - b0 + 1, 0), nc) columns
      const int4 pr = P.ea_pairs[t.z + k];
      const long long nr = pr.w & 0xff, ncl = pr.w >> 8, d = pr.y - pr.z + 1;
      e += (double)(G(d + nr - 1, ncl) - G(d - 1, ncl));
    }
    const int2 it = P.at_iptr[q];
    for (int k = 0; k < it.y; k++) {
      const int code = P.at_items[it.x + k];
      h += code >= 0 ? 72.0 * (P.asm_ptr[code + 1] - P.asm_ptr[code]) : 48.0;
    }
    const long long mp = P.m[t.x], R0 = 64 * (t.y >> 16), C0 = 64 * (t.y & 0xffff);
    const long long R1 = std::min(R0 + 64, mp), C1 = std::min(C0 + 64, mp);
    // tile elements: columns j in [C0, C1), rows [max(R0, j), R1)
    const long long jd = std::min(std::max(R0, C0), C1);   // columns below jd see all R1 - R0 rows
    e += (double)((jd - C0) * std::max(0LL, R1 - R0));
    for (long long a = std::max(jd, C0); a < C1; a++) e += (double)std::max(0LL, R1 - a);
    bytes += 8.0 * e + h;
  }
  return lv.at_bytes = bytes;
}

hipError_t chol_factor(const CholPlan& P, const double* D, const double* V, const double* b, double scale_b,
                       hipStream_t s, LaunchProfile* prof, int nb, ExchangeHook* hook) {
  if (P.n == 0) return hipSuccess;
  if (nb < 1 || nb > P.batch) return hipErrorInvalidValue;
  const CholDev c = dev_view(P);
  const dim3 B256(256);
  static const bool stamps = getenv("PGO_STEP_STAMPS") != nullptr;
  launch(prof, kFamPerm, [&] { return make_double2(0, 48.0 * P.n * nb); }, k_perm_in, dim3((P.n + 255) / 256, nb),
         B256, 0, s, c, b, scale_b, P.n);
  CH_TRY(hipMemsetAsync(P.d_flag, 0, sizeof(int) * nb, s));
  CH_TRY(hipMemsetAsync(P.d_stepflag, 0, sizeof(int) * std::max(P.ns, 1) * nb, s));
  const bool part = P.part_size > 1;
  if (part && (!hook || !hook->allgather || (!P.xchg.empty() && !hook->broadcast))) return hipErrorInvalidValue;
  auto exchange = [&]() -> hipError_t {   // subtree roots -> every rank
    const long long slot = xroot_slot(P);
    if (P.n_xown) k_xroots<true><<<dim3(P.n_xown, nb), 256, 0, s>>>(c, P.d_xown, P.d_xsend, slot, 0);
    CH_TRY(hipGetLastError());
    if (hook->allgather(hook->ctx, P.d_xsend, P.d_xrecv, sizeof(double) * slot * nb, s) != 0) {
      hook->failed = true;
      return hipErrorUnknown;
    }
    if (P.n_xforeign) k_xroots<false><<<dim3(P.n_xforeign, nb), 256, 0, s>>>(c, P.d_xforeign, P.d_xrecv, slot, slot * nb);
    return hipGetLastError();
  };
  // distributed top: the panels (tails) of exchange point xi from their owners
  // to every rank -- pack, one broadcast per sending rank, unpack
  auto xpanels = [&](int xi) -> hipError_t {
    if (!part || xi < 0) return hipSuccess;
    const XExchange& X = P.xchg[xi];
    const long long rstride = std::max(P.xp_rslot, 1LL) * nb;
    k_xpanel<true><<<dim3(X.cnt, nb), 256, 0, s>>>(c, P.d_xp + X.off, P.d_xp_off + 2 * X.off, P.d_xprecv, rstride,
                                                   P.part_rank);
    CH_TRY(hipGetLastError());
    if (hook->group) hook->group(hook->ctx, 1);
    bool bad = false;
    for (int r = 0; r < P.part_size && !bad; r++)
      if (X.size[r] > 0)
        bad = hook->broadcast(hook->ctx, P.d_xprecv + r * rstride, sizeof(double) * X.size[r] * nb, r, s) != 0;
    if (hook->group && hook->group(hook->ctx, 0) != 0) bad = true;
    if (bad) {
      hook->failed = true;
      return hipErrorUnknown;
    }
    k_xpanel<false><<<dim3(X.cnt, nb), 256, 0, s>>>(c, P.d_xp + X.off, P.d_xp_off + 2 * X.off, P.d_xprecv, rstride,
                                                    P.part_rank);
    return hipGetLastError();
  };
  // PGO_ABLATE (diagnostics only -- the factor is wrong): skip the named launch
  // families (small, plain, assemble, vec, first, step) to time what the rest of
  // the schedule costs in graph mode
  static const char* ablate = getenv("PGO_ABLATE");
  auto off = [&](const char* fam) { return ablate && strstr(ablate, fam); };
  for (size_t li = 0; li < P.levels.size(); li++) {
    const CholLevel& lv = P.levels[li];
    if (prof) prof->cur_tag = (int)li << 16;
    if (part && (int)li == P.split) CH_TRY(exchange());
    // frontal vectors (fv) on the second side stream beside the tile assembly
    // (F): disjoint data, both need only the previous levels; joined before the
    // level's first factor launch
    static const bool asm_push = getenv("PGO_ASM_PUSH") && atoi(getenv("PGO_ASM_PUSH")) == 1;
    // (PGO_VEC_FUSE=0, A/B: the frontal vectors in their own launch on the
    // second side stream, as before round 5)
    static const bool vec_fuse = !(getenv("PGO_VEC_FUSE") && atoi(getenv("PGO_VEC_FUSE")) == 0) && !asm_push;
    const bool vec = !off("vec") && !vec_fuse;
    const int nvec = !off("vec") && vec_fuse ? lv.front_cnt : 0;
    if (vec) {
      CH_TRY(hipEventRecord(P.evs[0], s));
      CH_TRY(hipStreamWaitEvent(P.side2, P.evs[0], 0));
      launch(prof, kFamVecAssemble, [&] { return make_double2(0, lv.vec_bytes * nb); }, k_vec_assemble, dim3(lv.front_cnt, nb), B256,
             (size_t)lv.maxm * sizeof(double), P.side2, c, (const int*)(P.d_level_fronts + lv.front_off));
      CH_TRY(hipEventRecord(P.evs[1], P.side2));
    }
    // (PGO_ASM_UNROLL: children whose loads are in flight together, 1 or 2)
    static const int asm_unroll = getenv("PGO_ASM_UNROLL") ? atoi(getenv("PGO_ASM_UNROLL")) : 1;
    const int ntile = lv.ea_cnt[0] && !off("assemble") ? lv.ea_cnt[0] : 0;
    if (asm_push && ntile)
      launch(prof, kFamAssemble, [&] { return make_double2(0, level_at_bytes(P, (int)li) * nb); },
             k_assemble_tile_push, dim3(ntile, nb), B256, 0, s, c,
             (const int4*)(P.d_ea_tasks + lv.ea_off[0]), (const int2*)(P.d_at_iptr + lv.ea_off[0]),
             (const int*)P.d_at_items, (const int4*)P.d_ea_pairs, V, D,
             (const double*)P.d_lambda);
    else if (ntile + nvec > 0)   // (the tile tasks' arrays are read only by workgroups < ntile)
      launch(prof, kFamAssemble,
             [&] { return make_double2(0, (level_at_bytes(P, (int)li) * (ntile > 0) + lv.vec_bytes * (nvec > 0)) * nb); },
             asm_unroll == 2 ? k_assemble_tile<2> : k_assemble_tile<1>, dim3(ntile + nvec, nb), B256, 0, s, c,
             (const int4*)(P.d_ea_tasks + lv.ea_off[0]), (const int2*)(P.d_at_iptr + lv.ea_off[0]),
             (const int*)P.d_at_items, (const int4*)P.d_ea_pairs, V, D,
             (const double*)P.d_lambda, ntile, (const int*)(P.d_level_fronts + lv.front_off));
    if (vec) CH_TRY(hipStreamWaitEvent(s, P.evs[1], 0));
    // small fronts on the second side stream, beside the blocked path of the
    // same level (disjoint fronts); joined before the next level
    // (the two wavefront classes -- m <= 64, m > 64 -- on two side streams,
    // concurrently: each is a grid of independent latency-bound waves)
    const bool fork_small = !lv.small.empty() && !lv.panels.empty();
    bool lo = false, hi = false;   // wavefront classes with m <= 64 / m > 64
    for (const SmallClass& sc : lv.small)
      if (sc.wave) (sc.mmax > 64 ? hi : lo) = true;
    const bool fork_wave = lo && hi;
    // PGO_WAVE_STREAMS=1 (A/B): the m > 64 classes narrower than kWaveW (few
    // fronts, latency-bound) on a fourth side stream instead of ahead of the
    // kWaveW class on the third
    static const bool wave_streams = knob_on("PGO_WAVE_STREAMS");
    hipStream_t ss = s;
    if (fork_small || fork_wave) {
      CH_TRY(hipEventRecord(P.evs[0], s));
      CH_TRY(hipStreamWaitEvent(P.side2, P.evs[0], 0));
      if (fork_wave) CH_TRY(hipStreamWaitEvent(P.side3, P.evs[0], 0));
      if (fork_wave && wave_streams) CH_TRY(hipStreamWaitEvent(P.side6, P.evs[0], 0));
      ss = P.side2;
    }
    for (const SmallClass& sc : lv.small) {
      if (off("small")) break;
      auto small_cost = [&] { return make_double2(sc.flops * nb, 0); };
      const int* list = P.d_small + sc.off;
      if (sc.wave) {
        // classes by (m <= 64 | m > 64) x panel width W in {8, 16, 32}; the
        // m > 64 ones on the third stream
        const hipStream_t st = fork_wave && sc.mmax > 64 ? (wave_streams && sc.wave < kWaveW ? P.side6 : P.side3) : ss;
        const size_t lds = (size_t)(sc.mmax * (sc.wave + 1) + 130 + sc.wave) * sizeof(double);
        const dim3 g(sc.cnt, nb), b(64);
        // (m > 64 with W = 32: two waves per front, k_front_wave2, 15-24 % faster
        // per 4096 fronts (profiles/r04e_front_wave_ubench.txt); PGO_WAVE2=0: one
        // wave holding two rows per lane -- bitwise the same fronts.  W = 16
        // stays one wave of per-pivot steps: 102 us against 124 for the two-wave
        // blocked form on m = 90, w = 12; PGO_WAVE2=2 forces the two waves there)
        static const int wave2_mode = getenv("PGO_WAVE2") ? atoi(getenv("PGO_WAVE2")) : 1;
        const bool wave2 = wave2_mode != 0;
        const dim3 b2(128);
        if (sc.mmax > kSmallFront) {   // 128 < m <= 256: four waves (k_front_wave4), W 16 or 32
          if (sc.wave == 16) launch(prof, kFamFrontWave, small_cost, k_front_wave4<16>, g, dim3(256), lds, st, c, list);
          else launch(prof, kFamFrontWave, small_cost, k_front_wave4<kWaveW>, g, dim3(256), lds, st, c, list);
        } else if (sc.mmax > 64) {
          if (sc.wave == 8) launch(prof, kFamFrontWave, small_cost, k_front_wave<8, true>, g, b, lds, st, c, list);
          else if (sc.wave == 16 && wave2_mode == 2) launch(prof, kFamFrontWave, small_cost, k_front_wave2<16>, g, b2, lds, st, c, list);
          else if (sc.wave == 16) launch(prof, kFamFrontWave, small_cost, k_front_wave<16, true>, g, b, lds, st, c, list);
          else if (wave2) launch(prof, kFamFrontWave, small_cost, k_front_wave2<kWaveW>, g, b2, lds, st, c, list);
          else launch(prof, kFamFrontWave, small_cost, k_front_wave<kWaveW, true>, g, b, lds, st, c, list);
        } else {
          if (sc.wave == 8) launch(prof, kFamFrontWave, small_cost, k_front_wave<8, false>, g, b, lds, st, c, list);
          else if (sc.wave == 16) launch(prof, kFamFrontWave, small_cost, k_front_wave<16, false>, g, b, lds, st, c, list);
          else launch(prof, kFamFrontWave, small_cost, k_front_wave<kWaveW, false>, g, b, lds, st, c, list);
        }
      } else {
        launch(prof, kFamFrontSmall, small_cost, k_front_small, dim3(sc.cnt, nb), B256,
               (size_t)(sc.mmax * sc.mmax + 64 + sc.mmax) * sizeof(double), ss, c, list);
      }
    }
    // apart plain tiles run on P.side (in order, so two of them never touch a
    // tile at once); plain(j) is joined before step j + plain_lag (1, or 2 when
    // the look-ahead skip left the next step independent of it), and at the
    // level's end.  Ring of two join events (evs[3], evs[5]).
    bool side_pending = false;
    std::vector<char> on_side(lv.panels.size(), 0);   // plain(j) went to P.side and recorded its event
    // deferred far updates on P.side4: (join step, event slot) of the pending ones
    std::vector<int2> far_pending;
    int fslot = 0;
    auto join_far = [&](int step) -> hipError_t {   // step -1: all of them
      for (size_t q = 0; q < far_pending.size();) {
        if (step < 0 || far_pending[q].x == step) {
          CH_TRY(hipStreamWaitEvent(s, P.fev[far_pending[q].y], 0));
          far_pending.erase(far_pending.begin() + q);
        } else {
          q++;
        }
      }
      return hipSuccess;
    };
    for (size_t j = 0; j < lv.panels.size(); j++) {
      const PanelStep& ps = lv.panels[j];
      CH_TRY(join_far((int)j));
      for (size_t back = 1; back <= 2 && back <= j; back++) {
        const PanelStep& pp = lv.panels[j - back];
        if (on_side[j - back] && pp.plain_lag == (int)back)
          CH_TRY(hipStreamWaitEvent(s, P.evs[(j - back) & 1 ? 5 : 3], 0));
      }
      if (prof) prof->cur_tag = ((int)li << 16) | (ps.kb / kNB + 1);
      const int4* cols = (const int4*)(P.d_col + ps.col_off);
      // many first panels (x lanes): diagonal tiles, then the tiles below in a
      // second launch of higher occupancy; few: one launch with in-launch
      // hand-offs (PGO_FIRST_SPLIT: the fronts x lanes from which to split)
      static const int first_split = getenv("PGO_FIRST_SPLIT") ? atoi(getenv("PGO_FIRST_SPLIT")) : 64;
      if (ps.potrf_cnt && !off("first")) {
        if (ps.potrf_cnt * nb >= first_split && ps.fcol_cnt > 0) {
          launch(prof, kFamPanelFirst, [&] { return make_double2(ps.first_flops * nb, 0); }, k_first_diag,
                 dim3(ps.potrf_cnt, nb), B256, 0, s, c, (const int*)(P.d_potrf + ps.potrf_off));
          launch(prof, kFamPanelFirst, [&] { return make_double2(0, 0); }, k_first_trsm, dim3(ps.fcol_cnt, nb), B256,
                 0, s, c, cols);
        } else {
          launch(prof, kFamPanelFirst, [&] { return make_double2(ps.first_flops * nb, 0); }, k_panel_first,
                 dim3(ps.potrf_cnt + ps.fcol_cnt, nb), B256, 0, s, c, (const int*)(P.d_potrf + ps.potrf_off),
                 ps.potrf_cnt, cols);
        }
      }
      CH_TRY(xpanels(ps.xfirst));
      const int4* tiles = (const int4*)(P.d_syrk + ps.syrk_off);
      const int nin = ps.syrk_inline && !off("plain") ? ps.syrk_cnt : 0;
      const bool apart = ps.syrk_cnt > 0 && !ps.syrk_inline && !off("plain");   // plain tiles in their own launch
      const bool step = ps.sdiag_cnt + ps.col_cnt + ps.prep_cnt + nin > 0 && !off("step");
      auto plain = [&](hipStream_t st, int first, int cnt, double flops) {
        const bool big = ps.syrk_tile == kBigTile;
        launch(prof, big ? kFamPanelSyrk128 : kFamPanelSyrk, [&] { return make_double2(flops * nb, 0); },
               big ? k_panel_syrk128 : k_panel_syrk_lds, dim3(cnt, nb), B256, 0, st, c, tiles + first, ps.kb);
      };
      if (apart) {   // on the side stream (beside k_step, behind the earlier plains)
        CH_TRY(hipEventRecord(P.evs[2], s));
        CH_TRY(hipStreamWaitEvent(P.side, P.evs[2], 0));
      }
      // many diagonal tiles (x lanes): the step as three launches -- the
      // diagonal tiles (k_step_diag: 2 workgroups per CU) beside the column
      // block's, prep and inline tile updates (k_panel_syrk_lds on P.side5:
      // 4 per CU), then the column block's solves (k_first_trsm) -- instead of
      // one k_step whose column workgroups hold a diagonal workgroup's LDS and
      // registers while they wait; same arithmetic (the tile kernels compute a
      // tile's elements alike), bitwise k_step's factor
      const int step_split = step_split_threshold();
      const bool split = step && step_split > 0 && ps.sdiag_cnt * nb >= step_split && ps.col_cnt > 0;
      if (split) {
        const int4* cupd = cols + ps.fcol_cnt;   // col then prep tasks: 64x64 tile updates
        CH_TRY(hipEventRecord(P.evs[0], s));
        CH_TRY(hipStreamWaitEvent(P.side5, P.evs[0], 0));
        launch(prof, kFamPanelSyrk, [&] { return make_double2(ps.colupd_flops * nb, 0); }, k_panel_syrk_lds,
               dim3(ps.col_cnt + ps.prep_cnt, nb), B256, 0, P.side5, c, cupd, ps.kb);
        if (nin)
          launch(prof, kFamPanelSyrk, [&] { return make_double2(ps.plain_flops * nb, 0); }, k_panel_syrk_lds,
                 dim3(nin, nb), B256, 0, P.side5, c, tiles, ps.kb);
        CH_TRY(hipEventRecord(P.evs[1], P.side5));
        launch(prof, kFamStepDiag, [&] { return make_double2(ps.diag_flops * nb, 0); }, k_step_diag,
               dim3(ps.sdiag_cnt, nb), B256, 0, s, c, (const int4*)(P.d_sdiag + ps.sdiag_off), ps.kb);
        CH_TRY(hipStreamWaitEvent(s, P.evs[1], 0));
        launch(prof, kFamColTrsm, [&] { return make_double2(ps.trsm_flops * nb, 0); }, k_first_trsm,
               dim3(ps.col_cnt, nb), B256, 0, s, c, cupd);
      } else if (step)
        launch(prof, kFamStep, [&] { return make_double2(ps.step_flops * nb, 0); }, k_step,
               dim3(ps.sdiag_cnt + ps.col_cnt + ps.prep_cnt + nin, nb), B256, 0, s, c,
               (const int4*)(P.d_sdiag + ps.sdiag_off), ps.sdiag_cnt, cols + ps.fcol_cnt, ps.col_cnt, ps.prep_cnt,
               tiles, ps.kb,
               stamps && li + 1 == P.levels.size() && ps.kb / kNB < kMaxStampSlots ? ps.kb / kNB : -1);
      if (apart) {   // (never on the main stream: an earlier plain may still run on P.side)
        const int nnear = ps.syrk_cnt - ps.far_cnt;
        plain(P.side, 0, nnear, ps.plain_flops - ps.far_flops);
        CH_TRY(hipEventRecord(P.evs[j & 1 ? 5 : 3], P.side));
        side_pending = true;
        on_side[j] = 1;
        if (ps.far_cnt > 0) {   // the far pieces: on P.side4 (behind the earlier far launches), each joined late
          CH_TRY(hipStreamWaitEvent(P.side4, P.evs[2], 0));
          for (int q = ps.far_p0; q < ps.far_p0 + ps.far_np; q++) {
            const int4 fp = lv.far_pieces[q];
            if (fp.z == 0) continue;
            int busy = -2;   // (a ring slot still pending: joined now)
            for (const int2& pend : far_pending)
              if (pend.y == fslot) busy = pend.x;
            if (busy != -2) CH_TRY(join_far(busy));
            plain(P.side4, fp.y, fp.z, lv.far_piece_flops[q]);
            CH_TRY(hipEventRecord(P.fev[fslot], P.side4));
            far_pending.push_back(make_int2(fp.w, fslot));
            fslot = (fslot + 1) % 8;
          }
        }
      }
      // the panel this step factored, to every rank (the apart plain tiles
      // beside it neither read nor write its columns)
      CH_TRY(xpanels(ps.xstep));
    }
    if (side_pending) {   // every apart plain of the level done before the next level
      CH_TRY(hipEventRecord(P.evs[2], P.side));
      CH_TRY(hipStreamWaitEvent(s, P.evs[2], 0));
    }
    CH_TRY(join_far(-1));
    if (fork_small || fork_wave) {
      CH_TRY(hipEventRecord(P.evs[1], P.side2));
      CH_TRY(hipStreamWaitEvent(s, P.evs[1], 0));
      if (fork_wave) {
        CH_TRY(hipEventRecord(P.evs[4], P.side3));
        CH_TRY(hipStreamWaitEvent(s, P.evs[4], 0));
        if (wave_streams) {
          CH_TRY(hipEventRecord(P.ev6, P.side6));
          CH_TRY(hipStreamWaitEvent(s, P.ev6, 0));
        }
      }
    }
    CH_TRY(xpanels(lv.xtail));
  }
  if (part && P.split >= (int)P.levels.size()) CH_TRY(exchange());
  // PGO_DEBUG_BAD_PIVOT=r:k (tests): rank r's first k factorisations report a
  // non-positive pivot that only it has seen -- the partitioned solve must
  // still take the same decision on every rank
  static const char* bad = getenv("PGO_DEBUG_BAD_PIVOT");
  static int bad_left = bad && strchr(bad, ':') ? atoi(strchr(bad, ':') + 1) : 0;
  if (bad && bad_left > 0 && atoi(bad) == P.part_rank) {
    bad_left--;
    k_set_flag<<<1, nb, 0, s>>>(P.d_flag, 1);
  }
  return hipGetLastError();
}

// Diagnostics (tests): every element a factorisation must write before it
// reads it -- the lower trapezoid of every front, the frontal vectors, the
// diagonal inverses in both orders -- set to NaN in every lane's workspace.  A
// factorisation that read one of them before writing it would carry the NaN
// into its factor (the class of round 4's r04b failure: an element the tile
// assembly did not write, read stale).  The small fronts' upper triangles stay
// as allocated (zero): no kernel writes them.
__global__ __launch_bounds__(256) void k_poison(CholDev c) {
  lane_offset(c);
  const int s = blockIdx.x;
  const long long f0 = c.foff[s];
  if (c.foff[s + 1] == f0) return;   // (a partitioned plan: no storage for another rank's front)
  const int m = c.m[s];
  const bool pk = front_packed(m, c.w[s]);
  const double nan = __builtin_nan("");
  for (int j = 0; j < m; j++) {
    double* col = fcol(c.F + f0, m, pk, j);
    for (int i = j + (int)threadIdx.x; i < m; i += 256) col[i] = nan;
  }
  for (int i = threadIdx.x; i < m; i += 256) c.fv[c.voff[s] + i] = nan;
  for (long long q = c.toff[s] + threadIdx.x; q < c.toff[s + 1]; q += 256) {
    c.Tinv[q] = nan;
    c.Tinv[c.tfo + q] = nan;
  }
}

hipError_t chol_debug_poison(const CholPlan& P, hipStream_t s) {
  if (!P.F || P.ns == 0) return hipSuccess;
  k_poison<<<dim3(P.ns, std::max(P.batch, 1)), 256, 0, s>>>(dev_view(P));
  CH_TRY(hipGetLastError());
  return hipStreamSynchronize(s);
}

hipError_t chol_step_stamps(unsigned long long* out, int slots) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 10 * std::min(slots, kMaxStampSlots));
}

hipError_t chol_marginals(const CholPlan& P, const int* poses, int n, double* out, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  int maxm = 1;
  for (int q = 0; q < P.ns; q++) maxm = std::max(maxm, P.m[q]);
  std::vector<int2> st(n);
  for (int i = 0; i < n; i++) {
    const int j = P.iperm[poses[i]];
    st[i] = make_int2(P.dg_front[j], 3 * P.dg_loc[j]);
  }
  int2* d_st = nullptr;
  double *d_scr = nullptr, *d_out = nullptr;
  hipError_t e = hipMalloc((void**)&d_st, n * sizeof(int2));
  if (e == hipSuccess) e = hipMalloc((void**)&d_scr, (size_t)n * 6 * maxm * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&d_out, (size_t)n * 9 * sizeof(double));
  if (e == hipSuccess) e = hipMemcpyAsync(d_st, st.data(), n * sizeof(int2), hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    k_marginals<<<n, 256, 0, s>>>(dev_view(P), d_st, maxm, d_scr, d_out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipMemcpyAsync(out, d_out, (size_t)n * 9 * sizeof(double), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (d_st) (void)hipFree(d_st);
  if (d_scr) (void)hipFree(d_scr);
  if (d_out) (void)hipFree(d_out);
  return e;
}

hipError_t chol_solve(const CholPlan& P, double* x, hipStream_t s, int nb, long long xstride, LaunchProfile* prof,
                      ExchangeHook* hook) {
  if (P.n == 0) return hipSuccess;
  if (nb < 1 || nb > P.batch) return hipErrorInvalidValue;
  const CholDev c = dev_view(P);
  const int g = (P.n + 255) / 256;
  const dim3 B256(256);
  // backward steps chained in one launch per level (PGO_BWD_STEPS=1: one launch per step)
  static const bool chain = !getenv("PGO_BWD_STEPS");
  if (chain) CH_TRY(hipMemsetAsync(P.d_stepflag, 0, sizeof(int) * std::max(P.ns, 1) * nb, s));
  for (auto it = P.levels.rbegin(); it != P.levels.rend(); ++it) {
    const CholLevel& lv = *it;
    if (prof) prof->cur_tag = (int)(&lv - P.levels.data()) << 16;
    if (lv.bwd_part.cnt)
      launch(prof, kFamBwdPart, [&] { return make_double2(lv.bwd_part_flops * nb, lv.bwd_part_bytes * nb); },
             k_bwd_part, dim3(lv.bwd_part.cnt, nb), B256, 0, s, c, (const int4*)(P.d_bwd_part + lv.bwd_part.off),
             P.d_partial);
    launch(prof, kFamBwdInit, [&] { return make_double2(0, lv.bwd_init_bytes * nb); }, k_bwd_init, dim3(lv.bwd[0].cnt, nb), B256, 0, s, c,
           (const int4*)(P.d_bwd + lv.bwd[0].off), (const int2*)(P.d_bwd_pref + lv.bwd[0].off),
           (const double*)P.d_partial);
    if (chain) {
      if (lv.bwdc.cnt)
        launch(prof, kFamBwdStep, [&] { return make_double2(0, lv.bwd_chain_bytes * nb); }, k_bwd_chain, dim3(lv.bwdc.cnt, nb), B256, 0,
               s, c, (const int4*)(P.d_bwdc + lv.bwdc.off));
    } else {
      for (size_t q = 1; q < lv.bwd.size(); q++) {
        const int bb = lv.maxblk - (int)q;   // step b = maxblk-1 .. 1
        if (lv.bwd[q].cnt)
          launch(prof, kFamBwdStep, [&] { return make_double2(0, 0); }, k_bwd_step, dim3(lv.bwd[q].cnt, nb), B256,
                 0, s, c, (const int4*)(P.d_bwd + lv.bwd[q].off), bb);
      }
    }
  }
  if (P.part_size > 1) {   // every rank's subtree solutions (and pivot flags) -> every rank
    if (!hook) return hipErrorInvalidValue;
    const long long slot = xsol_slot(P), rstride = slot * nb;
    if (P.n_xsol_own) k_xsol<true><<<dim3(16, P.n_xsol_own, nb), 256, 0, s>>>(c, P.d_xsol_own, P.d_xsend, slot, 0);
    k_xflag<<<1, nb, 0, s>>>(c, P.d_xsend, slot, P.xsol_max, 0, 1, 1);
    CH_TRY(hipGetLastError());
    if (hook->allgather(hook->ctx, P.d_xsend, P.d_xrecv, sizeof(double) * rstride, s) != 0) {
      hook->failed = true;
      return hipErrorUnknown;
    }
    if (P.n_xsol_foreign)
      k_xsol<false><<<dim3(16, P.n_xsol_foreign, nb), 256, 0, s>>>(c, P.d_xsol_foreign, P.d_xrecv, slot, rstride);
    k_xflag<<<1, nb, 0, s>>>(c, P.d_xrecv, slot, P.xsol_max, rstride, P.part_size, 0);
    CH_TRY(hipGetLastError());
  }
  launch(prof, kFamPerm, [&] { return make_double2(0, 48.0 * P.n * nb); }, k_perm_out, dim3(g, nb), B256, 0, s, c, x,
         P.n, xstride);
  return hipGetLastError();
}

}  // namespace pgo
