// Device-resident pose graph and the kernel launchers (internal to libpgo.so).
//
// HBM layout (N vertices, E between factors, S = 2E slots, P priors):
//   per vertex : pose/pose_cand double4 (x, y, c, s) -- Pose2 stores Rot2(c, s),
//                row_ptr int, prior_ptr int, D 6 doubles (upper of H_ii),
//                g 3, Minv 6, PCG x/r/z/p/q 3 each
//   per factor : eij int2, ez double4 (x, y, c, s), eom 3 x double2
//                (O00,O01)(O02,O11)(O12,O22) -- Omega upper triangle.  Factors
//                are stored in device order, sorted by (ei, ej), so the side-0
//                slots of a row read consecutive factors.
//   per slot   : V 9 doubles, structure of arrays (write_all = 1: PCG and
//                diagnostics): V[q * S + k] = element q (row-major) of the 3x3
//                block H_{row,col} of slot k (coalesced in slot order); the
//                Cholesky mode keeps one record per factor instead, V[9 e + q];
//                slot_edge int (factor << 2 | owner << 1 | side), slot_col int.
//                Slots of a row are contiguous (block-CSR over vertices, full
//                symmetric storage), each between factor owns two
//                slots: side 0 in row ei holds H_{ei,ej} = J1^T Omega, side 1 in
//                row ej holds H_{ej,ei} = Omega J1.  One of the two is the
//                factor's owner slot (side 0, or with the Cholesky plan the
//                block in the lower triangle of the permuted matrix).
#pragma once
#include <hip/hip_runtime.h>

namespace pgo {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 1024;   // partial-sum arrays are sized for this

struct DevGraph {
  int n = 0, ne = 0, np = 0, nslots = 0;
  int G = 8;                      // lanes per row (sub-group) for row kernels
  // factors
  int2* eij = nullptr;
  double4* ez = nullptr;
  double2* eom = nullptr;
  int* prior_ptr = nullptr;       // [n+1] priors grouped by vertex
  int* prior_vtx = nullptr;       // [P]   vertex of each (grouped) prior
  double4* pz = nullptr;
  double2* pom = nullptr;
  // block-CSR rows
  int* row_ptr = nullptr;
  int* slot_edge = nullptr;        // (device edge << 2) | (owner << 1) | side
  int write_all = 1;                // 1: both blocks of every edge in V (PCG, diagnostics);
                                    // 0: owner blocks only (the Cholesky assembly reads no others)
  int* slot_col = nullptr;
  // Cholesky-mode linearisation (write_all = 0 with a plan: owner blocks in
  // device factor order, V[9 e + q]: a factor's 9 elements together; see k_linearize_own)
  int G1 = 8;                       // lanes per row for the side-0 / side-1 sweeps
  int* erow = nullptr;              // [n+1] side-0 factors of row i: [erow[i], erow[i+1])
  int nlb = 0;                      // k_linearize_own blocks
  int* brow = nullptr;              // [nlb+1] whole rows of each block (<= kThreads rows,
                                    // side-0 factors <= kThreads unless a single row)
  int* s1_ptr = nullptr;            // [n+1] side-1 factors of row j: W[s1_ptr[j] .. s1_ptr[j+1])
  int* s1pos = nullptr;             // [E] position of factor e in the side-1 lists
  unsigned char* eside = nullptr;   // [E] side of the factor's owner block (set with the plan)
  double* Dc = nullptr;             // [6n] sum of Omega over the side-1 factors of each row
  double4* W = nullptr;             // [E] Omega e of each factor, side-1 list order (gradient hand-off)
  double* V = nullptr;
  double* D = nullptr;
  double* g = nullptr;
  // values
  double4* pose = nullptr;
  double4* pose_cand = nullptr;
  double4* pose_saved = nullptr;  // pgo_save_values snapshot (allocated on first use)
  // PCG
  double *x = nullptr, *r = nullptr, *z = nullptr, *p = nullptr, *q = nullptr, *Minv = nullptr;
  double* part = nullptr;         // [kMaxBlocks * 8] partial sums
  double* scal = nullptr;         // [16] device scalars
  int* ctrl = nullptr;            // [4]: done flag, PCG iterations
  hipStream_t stream = nullptr;
};

// partial-sum buffer slices
constexpr int kPartPQ = 0;          // p.q
constexpr int kPartRZ0 = 1;         // r.z of the three ping-pong buffers 1..3
constexpr int kPartA = 4;           // generic 2-value reductions use 4,5
constexpr int kPartSlices = 8;

// PCG control flags
constexpr int kRunning = 0, kConverged = 1, kBreakdown = 2;

int grid_rows(const DevGraph& d);
int grid_for(int work);

hipError_t launch_linearize(const DevGraph& d, hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
hipError_t launch_error(const DevGraph& d, const double4* pose, double* out_scalar);
hipError_t launch_retract(const DevGraph& d, const double* delta);
hipError_t launch_pcg_init(const DevGraph& d, double lambda);
hipError_t launch_pcg_spmv(const DevGraph& d, double lambda, hipEvent_t start = nullptr, hipEvent_t stop = nullptr);
hipError_t launch_pcg_vec(const DevGraph& d, int k, double tol2);
hipError_t launch_model_decrease(const DevGraph& d, const double* delta, double* out2);
hipError_t launch_spmv(const DevGraph& d, double lambda, const double* x, double* y);

}  // namespace pgo
