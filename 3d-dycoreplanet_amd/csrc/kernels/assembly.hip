// Cell-local finite-element assembly kernels for CDNA4 (gfx950), FP64.
//
// Replaces the WorkStream worker/copier pairs of the reference
// (include/core/boussinesq_model.tpp):
//   local_assemble_nse_system + copy_local_to_global_nse_system   :550-687
//   local_assemble_nse_preconditioner (diagonal only) + Jacobi     :421-542
//   local_assemble_temperature_matrix + copy                       :748-817
//   local_assemble_temperature_rhs + copy (matrix_for_bc lift)     :873-964
//
// One 256-thread workgroup owns one cell. The MappingQ(3) geometry of the
// reference (boussinesq_model.tpp:20) is recomputed from the cell's 64
// support points (1536 B per cell instead of 2160 B of stored J^-1/JxW),
// shape tables and per-quadrature physical gradients are staged in LDS, and the
// 27x27 node-pair Gram sums run as 1x3 register tiles (243 threads). The
// condensed (AffineConstraints) 3x3 node blocks are added into the block-CSR
// matrices with plain read-modify-write: the launch processes one colour of a
// cell colouring, so no two workgroups touch the same node and the result is
// deterministic (no atomics).
#include <hip/hip_runtime.h>

#include <stdexcept>

#include <cstddef>
#include <cstdlib>

#include "../device.h"
#include "../fe_tables.h"


namespace dcp {
namespace {

// 1D Lagrange bases at the 3 Gauss points: [basis][point]
__constant__ double cL2[3][3] = {
    {2 * (kGaussX[0] - 0.5) * (kGaussX[0] - 1), 2 * (kGaussX[1] - 0.5) * (kGaussX[1] - 1),
     2 * (kGaussX[2] - 0.5) * (kGaussX[2] - 1)},
    {-4 * kGaussX[0] * (kGaussX[0] - 1), -4 * kGaussX[1] * (kGaussX[1] - 1),
     -4 * kGaussX[2] * (kGaussX[2] - 1)},
    {2 * kGaussX[0] * (kGaussX[0] - 0.5), 2 * kGaussX[1] * (kGaussX[1] - 0.5),
     2 * kGaussX[2] * (kGaussX[2] - 0.5)}};
__constant__ double cdL2[3][3] = {{4 * kGaussX[0] - 3, 4 * kGaussX[1] - 3, 4 * kGaussX[2] - 3},
                                  {-8 * kGaussX[0] + 4, -8 * kGaussX[1] + 4, -8 * kGaussX[2] + 4},
                                  {4 * kGaussX[0] - 1, 4 * kGaussX[1] - 1, 4 * kGaussX[2] - 1}};
__constant__ double cL1[2][3] = {{1 - kGaussX[0], 1 - kGaussX[1], 1 - kGaussX[2]},
                                 {kGaussX[0], kGaussX[1], kGaussX[2]}};
__constant__ double cW[3] = {kGaussW[0], kGaussW[1], kGaussW[2]};
// MappingQ(3) 1D basis (Gauss-Lobatto support points) at the 3 Gauss points: [basis][point]
__constant__ double cL3[4][3] = {
    {map_lag(0, kGaussX[0]), map_lag(0, kGaussX[1]), map_lag(0, kGaussX[2])},
    {map_lag(1, kGaussX[0]), map_lag(1, kGaussX[1]), map_lag(1, kGaussX[2])},
    {map_lag(2, kGaussX[0]), map_lag(2, kGaussX[1]), map_lag(2, kGaussX[2])},
    {map_lag(3, kGaussX[0]), map_lag(3, kGaussX[1]), map_lag(3, kGaussX[2])}};
__constant__ double cdL3[4][3] = {
    {map_dlag(0, kGaussX[0]), map_dlag(0, kGaussX[1]), map_dlag(0, kGaussX[2])},
    {map_dlag(1, kGaussX[0]), map_dlag(1, kGaussX[1]), map_dlag(1, kGaussX[2])},
    {map_dlag(2, kGaussX[0]), map_dlag(2, kGaussX[1]), map_dlag(2, kGaussX[2])},
    {map_dlag(3, kGaussX[0]), map_dlag(3, kGaussX[1]), map_dlag(3, kGaussX[2])}};

// Row i of the MappingQ(3) Jacobian and x_i at Gauss point q from the 64
// support points X (lexicographic): J[i][e] = sum_n X_n,i dN_n/dxi_e.
__device__ inline void map_row(const double* X, int q, int i, double& x, double& J0, double& J1,
                               double& J2) {
  const int qa = q % 3, qb = (q / 3) % 3, qc = q / 9;
  x = J0 = J1 = J2 = 0;
#pragma unroll 1
  for (int c = 0; c < 4; ++c) {
    const double lc = cL3[c][qc], dc = cdL3[c][qc];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const double lb = cL3[b][qb], db = cdL3[b][qb];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const double Xi = X[3 * (a + 4 * b + 16 * c) + i];
        const double la = cL3[a][qa];
        x += Xi * la * lb * lc;
        J0 += Xi * cdL3[a][qa] * lb * lc;
        J1 += Xi * la * db * lc;
        J2 += Xi * la * lb * dc;
      }
    }
  }
}

// Lexicographic Q2 node -> hierarchic FE_Q(2) index (inverse of kQ2HierToLex).
__constant__ int cLexToHier[27] = {0, 10, 1, 8, 24, 9, 2, 11, 3, 16, 22, 17, 20, 26,
                                   21, 18, 23, 19, 4, 14, 5, 12, 25, 13, 6, 15, 7};

__device__ inline int fesys_velocity(int lex, int c) {
  const int h = cLexToHier[lex];
  return h < 8 ? 4 * h + c : 32 + 3 * (h - 8) + c;
}

// Shared per-cell geometry: J^-1 (as dxi_e/dx_d, [q][e][d]), JxW, x_q.
struct Geo {
  double Ji[27 * 9];
  double JxW[27];
  double xq[27 * 3];
};

// Radially separable mesh (cd.sep_col != null): J^-1, JxW and x at Gauss point
// q from the column / layer tables, the products the matrix-free kernel forms
// (J^-1 rows m0 / R, m1 / R, m2 / R'; JxW = R^2 R' D2 w; x = R phi).
__device__ inline void sep_geometry(const CellData& cd, int cell, Geo& g, int q) {
  const int q0 = q % 3, q1 = (q / 3) % 3, q2 = q / 9;
  const int col = cd.sep_col[cell], lay = cd.sep_layer[cell];
  const double* m = cd.sep_colgeo + 90 * size_t(col) + 10 * (q0 + 3 * q1);
  const double* lg = cd.sep_laygeo + 9 * size_t(lay) + 3 * q2;
  const double* ph = cd.sep_colphi + 27 * size_t(col) + 3 * (q0 + 3 * q1);
  const double iR = lg[0], iRp = lg[1], R = cd.sep_layR[3 * size_t(lay) + q2];
  double* Ji = &g.Ji[9 * q];
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    Ji[d] = m[d] * iR;
    Ji[3 + d] = m[3 + d] * iR;
    Ji[6 + d] = m[6 + d] * iRp;
    g.xq[3 * q + d] = R * ph[d];
  }
  g.JxW[q] = lg[2] * m[9] * (cW[q0] * cW[q1] * cW[q2]);
}

// 27 threads: the MappingQ(3) map at the QGauss(3) points (X: 64 support points).
__device__ inline void cell_geometry(const double* X, Geo& g, int q) {
  double J[3][3];
  double x[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) map_row(X, q, i, x[i], J[i][0], J[i][1], J[i][2]);
  const int qa = q % 3, qb = (q / 3) % 3, qc = q / 9;
  const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
  const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
  const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
  const double det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
  const double id = 1.0 / det;
  double* Ji = &g.Ji[9 * q];
  Ji[0] = c00 * id;
  Ji[1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * id;
  Ji[2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * id;
  Ji[3] = c01 * id;
  Ji[4] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * id;
  Ji[5] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * id;
  Ji[6] = c02 * id;
  Ji[7] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * id;
  Ji[8] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * id;
  g.JxW[q] = det * cW[qa] * cW[qb] * cW[qc];
  g.xq[3 * q + 0] = x[0];
  g.xq[3 * q + 1] = x[1];
  g.xq[3 * q + 2] = x[2];
}

// Physical gradient of the Q2 shape n at point q: grad_d = sum_e dN/dxi_e Ji[e][d]
__device__ inline void q2_grad(const Geo& g, int q, int n, double* out) {
  const int qa = q % 3, qb = (q / 3) % 3, qc = q / 9;
  const int na = n % 3, nb = (n / 3) % 3, nc = n / 9;
  const double la = cL2[na][qa], lb = cL2[nb][qb], lc = cL2[nc][qc];
  const double r0 = cdL2[na][qa] * lb * lc, r1 = la * cdL2[nb][qb] * lc, r2 = la * lb * cdL2[nc][qc];
  const double* Ji = &g.Ji[9 * q];
#pragma unroll
  for (int d = 0; d < 3; ++d) out[d] = r0 * Ji[d] + r1 * Ji[3 + d] + r2 * Ji[6 + d];
}

__device__ inline void q1_grad(const Geo& g, int q, int v, double* out) {
  const int qa = q % 3, qb = (q / 3) % 3, qc = q / 9;
  const int va = v & 1, vb = (v >> 1) & 1, vc = v >> 2;
  const double la = cL1[va][qa], lb = cL1[vb][qb], lc = cL1[vc][qc];
  const double da = va ? 1.0 : -1.0, db = vb ? 1.0 : -1.0, dc = vc ? 1.0 : -1.0;
  const double r0 = da * lb * lc, r1 = la * db * lc, r2 = la * lb * dc;
  const double* Ji = &g.Ji[9 * q];
#pragma unroll
  for (int d = 0; d < 3; ++d) out[d] = r0 * Ji[d] + r1 * Ji[3 + d] + r2 * Ji[6 + d];
}

__device__ inline double q1_value(int q, int v) {
  return cL1[v & 1][q % 3] * cL1[(v >> 1) & 1][(q / 3) % 3] * cL1[v >> 2][q / 9];
}
__device__ inline double q2_value(int q, int n) {
  return cL2[n % 3][q % 3] * cL2[(n / 3) % 3][(q / 3) % 3] * cL2[n / 9][q / 9];
}

// Local condensation matrix of a velocity node: full = C * reduced.
__device__ inline void condensation(const NodeConstraint& nc, double C[3][3]) {
#pragma unroll
  for (int i = 0; i < 3; ++i)
#pragma unroll
    for (int j = 0; j < 3; ++j) C[i][j] = 0.0;
  if (nc.type == 0) {
    C[0][0] = C[1][1] = C[2][2] = 1.0;
  } else if (nc.type == 2) {
#pragma unroll
    for (int d = 0; d < 3; ++d)
      if (d != nc.k) {
        C[d][d] = 1.0;
        C[nc.k][d] = nc.w[d];
      }
  }
}

// ---------------------------------------------------------------------------
// Cell-independent reference tables at the QGauss(3) points, evaluated at
// compile time with the same products the per-point helpers above use.
struct RefTables {
  double S2[27 * 27];      // [q][n] Q2 values
  double G2[27 * 27 * 3];  // [q][n][e] Q2 reference gradients
  double S1[27 * 8];       // [q][v] Q1 values
};
constexpr double ce_l2(int i, double x) {
  return i == 0 ? 2 * (x - 0.5) * (x - 1) : i == 1 ? -4 * x * (x - 1) : 2 * x * (x - 0.5);
}
constexpr double ce_dl2(int i, double x) {
  return i == 0 ? 4 * x - 3 : i == 1 ? -8 * x + 4 : 4 * x - 1;
}
constexpr double ce_l1(int i, double x) { return i == 0 ? 1 - x : x; }
constexpr RefTables make_ref_tables() {
  RefTables t{};
  for (int q = 0; q < 27; ++q) {
    const double xa = kGaussX[q % 3], xb = kGaussX[(q / 3) % 3], xc = kGaussX[q / 9];
    for (int n = 0; n < 27; ++n) {
      const int na = n % 3, nb = (n / 3) % 3, nc = n / 9;
      const double la = ce_l2(na, xa), lb = ce_l2(nb, xb), lc = ce_l2(nc, xc);
      t.S2[27 * q + n] = la * lb * lc;
      t.G2[3 * (27 * q + n) + 0] = ce_dl2(na, xa) * lb * lc;
      t.G2[3 * (27 * q + n) + 1] = la * ce_dl2(nb, xb) * lc;
      t.G2[3 * (27 * q + n) + 2] = la * lb * ce_dl2(nc, xc);
    }
    for (int v = 0; v < 8; ++v)
      t.S1[8 * q + v] = ce_l1(v & 1, xa) * ce_l1((v >> 1) & 1, xb) * ce_l1(v >> 2, xc);
  }
  return t;
}
__constant__ RefTables cRef = make_ref_tables();
__device__ inline double sel_gauss(int i) {
  return i == 0 ? kGaussX[0] : (i == 1 ? kGaussX[1] : kGaussX[2]);
}

// Node-group pairs (A <= B) of the 9 groups of 3 lexicographic nodes.
constexpr int kGroupPairs = 45;
__constant__ unsigned char cPairA[kGroupPairs] = {
    0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2,
    2, 3, 3, 3, 3, 3, 3, 4, 4, 4, 4, 4, 5, 5, 5, 5, 6, 6, 6, 7, 7, 8};
__constant__ unsigned char cPairB[kGroupPairs] = {
    0, 1, 2, 3, 4, 5, 6, 7, 8, 1, 2, 3, 4, 5, 6, 7, 8, 2, 3, 4, 5, 6, 7,
    8, 3, 4, 5, 6, 7, 8, 4, 5, 6, 7, 8, 5, 6, 7, 8, 6, 7, 8, 7, 8, 8};

// ---------------------------------------------------------------------------
// NSE system: local_assemble_nse_system (:550-673) + distribute_local_to_global.
// MODE 0 = scatter into block-CSR (colour launch), MODE 1 = dense element output.
//
// 256 threads (4 waves) per cell, 38.4 KB LDS and 110 VGPRs: four workgroups
// per CU. The velocity-velocity block is symmetric node-pair-wise
// (K_(b,.),(a,.) = K_(a,.),(b,.)^T), so only the 45 node-group pairs A <= B are
// summed: 135 1x3 tiles on waves 0-2. Wave 3 sums the 216 divergence blocks; 27
// otherwise idle lanes of wave 2 the rhs nodes. The average-diagonal value of
// the |K_ii| rule is computed up front from the 27 node-diagonal blocks.
//
// Writes are the bound (729 scattered 72-byte blocks per cell): the tile lanes
// park their blocks in LDS (over the dead geometry/gradient tables; the
// AffineConstraints condensation is applied there, only for blocks with a
// constrained node), then all four waves write the whole element matrix back
// with consecutive lanes on consecutive doubles of a block, 16
// read-modify-write loads in flight per lane; the (b, a) transposes are read
// from the staged (a, b) blocks (cSlot). Scatter positions (this cell's posA /
// posBt / posB, loaded into LDS up front) carry a first-touch mark (~pos): the
// first cell in launch order that touches a block stores instead of adding, so
// the matrices need no zero fill.
constexpr int kNseThreads = 256;
constexpr int kNseTiles = 3 * kGroupPairs;   // 135
constexpr int kRhsLane0 = 160;               // wave 2 lanes 32..58: rhs nodes

// Write staging (after the tile phase, over the dead X..F tables): the 405
// condensed A blocks of the tiles (slot 3 tile + tt, 9 doubles) then the 216
// condensed B^T rows (3 doubles).
constexpr int kStageA = 405 * 9;
constexpr int kStageDoubles = kStageA + 216 * 3;
struct NseSmem {
  double X[3 * kMapPts], U[81], T[27];  // T: 8 vertex (FE_Q(1)) or 27 lexicographic (FE_Q(2)) values
  Geo geo;
  double D[27 * 27 * 3];   // [q][n][d] reference, then physical gradients
  double S[27 * 27];       // [q][n] shape values
  double W1[27 * 8];       // [q][v] JxW * Q1 value
  double F[27 * 3];        // JxW * rhs integrand (velocity part) per q
  double stage_pad[448];   // write staging: X..stage_pad (dead by then)
  double diag[27];         // sum_c |K_(a,c),(a,c)| per node (average-diagonal rule)
  int node[27];
  int orig[27];            // original node (!= node: a periodic image of node)
  int pdof[8];
  int pos[729 + 216 + 216];  // this cell's posA, posBt, posB
};
static_assert(offsetof(NseSmem, diag) - offsetof(NseSmem, X) >= sizeof(double) * kStageDoubles,
              "NSE write staging overlaps live LDS");
static_assert(sizeof(NseSmem) <= 40960, "NSE LDS above 40 KB (four workgroups per CU)");

// Element-matrix block (a, b) -> staging slot: A blocks of group pairs
// grp(a) <= grp(b) are stored (tile lane a % 3, tt = b % 3), the others are
// the transposes of (b, a). Bit 15: transposed.
constexpr int ce_pair_index(int A, int B) {
  int i = 0;
  for (int x = 0; x < A; ++x) i += 9 - x;
  return i + (B - A);
}
struct SlotTable {
  unsigned short s[729];
};
constexpr SlotTable make_slot_table() {
  SlotTable t{};
  for (int a = 0; a < 27; ++a)
    for (int b = 0; b < 27; ++b) {
      const int A = a / 3, B = b / 3;
      if (A <= B) {
        const int tile = 3 * ce_pair_index(A, B) + a % 3;
        t.s[27 * a + b] = static_cast<unsigned short>(3 * tile + b % 3);
      } else {
        const int tile = 3 * ce_pair_index(B, A) + b % 3;
        t.s[27 * a + b] = static_cast<unsigned short>((3 * tile + a % 3) | 0x8000);
      }
    }
  return t;
}
__constant__ SlotTable cSlot = make_slot_table();

// All-wave scatter of the staged element matrix: element e of
// [0, kScatterElems) is component e % 9 of the A block e / 9 (posA order),
// then the B^T rows, then the B rows (3 doubles each), so consecutive lanes
// write consecutive doubles of a block. pos >= 0: add, ~pos: first touch
// (store). A lane keeps kScatterBatch read-modify-write loads in flight (the
// destinations of one cell are distinct).
constexpr int kScatterElems = 729 * 9 + 2 * 216 * 3;
#ifndef DCP_SCATTER_BATCH
#define DCP_SCATTER_BATCH 16
#endif
constexpr int kScatterBatch = DCP_SCATTER_BATCH;
__device__ inline double* scatter_target(const NseSmem& sh, const NseOut& out, int e, bool& add,
                                         double& v) {
  const double* st = sh.X;  // staging base
  int p;
  double* dst;
  if (e < 729 * 9) {
    const int pr = e / 9, comp = e - 9 * pr;
    const int sl = cSlot.s[pr];
    const int k = sl & 0x7fff;
    const int i = comp / 3, j = comp - 3 * i;
    v = st[9 * k + ((sl & 0x8000) ? 3 * j + i : comp)];
    p = sh.pos[pr];
    add = p >= 0;
    dst = out.A + 9 * size_t(add ? p : ~p) + comp;
  } else if (e < 729 * 9 + 648) {
    const int r = (e - 729 * 9) / 3, c = e - 729 * 9 - 3 * r;
    v = st[kStageA + 3 * r + c];
    p = sh.pos[729 + r];
    add = p >= 0;
    dst = out.Bt + 3 * size_t(add ? p : ~p) + c;
  } else {
    const int r = (e - 729 * 9 - 648) / 3, c = e - 729 * 9 - 648 - 3 * r;
    const int pv = r / 27, an = r - 27 * pv;  // B row (pv, an) = B^T row (an, pv)
    v = st[kStageA + 3 * (8 * an + pv) + c];
    p = sh.pos[945 + r];
    add = p >= 0;
    dst = out.B + 3 * size_t(add ? p : ~p) + c;
  }
  return dst;
}

// Sum of the velocity-velocity 3x3 blocks (a, b0..b0+2) over the 27 points:
// K_(a,c),(b,c') = delta_cc' (M + dt/Re L) + dt/Re Q_{c'c}   (2 eps:eps / 2)
__device__ inline void nse_tile(const NseSmem& sh, const PhysicsDev& ph, int a, int b0,
                                double blk[3][9]) {
  double m[3] = {0, 0, 0}, Q[3][9];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < 9; ++i) Q[t][i] = 0;
#pragma unroll 1
  for (int q = 0; q < 27; ++q) {
    const double w = sh.geo.JxW[q];
    const double* Da = &sh.D[3 * (27 * q + a)];
    const double da0 = w * Da[0], da1 = w * Da[1], da2 = w * Da[2];
    const double sa = w * sh.S[27 * q + a];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const double* Db = &sh.D[3 * (27 * q + b0 + t)];
      const double db0 = Db[0], db1 = Db[1], db2 = Db[2];
      m[t] += sa * sh.S[27 * q + b0 + t];
      Q[t][0] += da0 * db0; Q[t][1] += da0 * db1; Q[t][2] += da0 * db2;
      Q[t][3] += da1 * db0; Q[t][4] += da1 * db1; Q[t][5] += da1 * db2;
      Q[t][6] += da2 * db0; Q[t][7] += da2 * db1; Q[t][8] += da2 * db2;
    }
  }
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    const double L = Q[t][0] + Q[t][4] + Q[t][8];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int cp = 0; cp < 3; ++cp)
        blk[t][3 * c + cp] = (c == cp ? m[t] + ph.nu_sys * L : 0.0) + ph.nu_sys * Q[t][3 * cp + c];
  }
}

// B^T block of velocity node an and pressure vertex v: -sum_q JxW phi_p div phi_u
__device__ inline void nse_div(const NseSmem& sh, int an, int v, double bt[3]) {
  bt[0] = bt[1] = bt[2] = 0;
#pragma unroll 1
  for (int q = 0; q < 27; ++q) {
    const double wp = sh.W1[8 * q + v];
    const double* Da = &sh.D[3 * (27 * q + an)];
    bt[0] -= Da[0] * wp; bt[1] -= Da[1] * wp; bt[2] -= Da[2] * wp;
  }
}

__device__ inline void nse_rhs_node(const NseSmem& sh, int an, double fa[3]) {
  fa[0] = fa[1] = fa[2] = 0;
#pragma unroll 1
  for (int q = 0; q < 27; ++q) {
    const double s = sh.S[27 * q + an];
    fa[0] += s * sh.F[3 * q]; fa[1] += s * sh.F[3 * q + 1]; fa[2] += s * sh.F[3 * q + 2];
  }
}

// ---------------------------------------------------------------------------
// The velocity-velocity Gram sums on the matrix cores (DCP_OPT_ELEMENT_MFMA):
// G = D^T W D over the 81 (node, direction) physical gradients -- D is [q][n][d]
// in LDS, so column r = 3n + d of the 27 x 81 matrix is D[81 q + r] -- and the
// mass M = S^T W S over the 27 shape values, both as v_mfma_f64_16x16x4_f64
// tiles with K = 27 points padded to 28 (7 steps): the 21 upper tiles of the
// 96 x 96 padded G and the 3 upper tiles of the 32 x 32 padded M, six per wave.
// Lane l feeds A[l & 15][k = l >> 4] = w_q D[q][16 I + (l & 15)] and
// B[k][l & 15] = D[q][16 J + (l & 15)]; result register i holds
// G[16 I + (l >> 4) + 4 i][16 J + (l & 15)] (the f64 C/D map).
// The element block then is K_(a,c),(b,c') = nu Q_c'c + delta_cc' (m + nu L),
// Q_de = G[3a + d][3b + e], L = trace Q (nse_tile's formula, summed in MFMA order).
typedef double f64x4_t __attribute__((ext_vector_type(4)));
constexpr int kGramQTiles = 21;
constexpr int kGramTilesPerWave = 6;  // 21 G + 3 M = 24 tiles over 4 waves
__constant__ unsigned char cGramI[24] = {0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 4, 4, 5,
                                         0, 0, 1};
__constant__ unsigned char cGramJ[24] = {0, 1, 2, 3, 4, 5, 1, 2, 3, 4, 5, 2, 3, 4, 5, 3, 4, 5, 4, 5, 5,
                                         0, 1, 1};

__device__ inline void gram_tiles(const NseSmem& sh, int wave, int lane,
                                  f64x4_t acc[kGramTilesPerWave]) {
  const int li = lane & 15, lk = lane >> 4;
  {
#pragma unroll
    for (int t = 0; t < kGramTilesPerWave; ++t) {
      const int tile = wave + 4 * t;
      const bool mass = tile >= kGramQTiles;
      const int ra = 16 * cGramI[tile] + li, cb = 16 * cGramJ[tile] + li;
      const int nmax = mass ? 27 : 81;
      const double* tab = mass ? sh.S : sh.D;
      const int ld = mass ? 27 : 81;
      f64x4_t c = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < 7; ++s) {
        const int q = 4 * s + lk;
        double a = 0.0, b = 0.0;
        if (q < 27) {
          if (ra < nmax) a = sh.geo.JxW[q] * tab[ld * q + ra];
          if (cb < nmax) b = tab[ld * q + cb];
        }
        c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
      }
      acc[t] = c;
    }
  }
}

// Staging slot of the element block (a, b), grp(a) <= grp(b) (stored untransposed).
__device__ inline double* gram_slot(double* st, int a, int b) {
  return st + 9 * (cSlot.s[27 * a + b] & 0x7fff);
}

// Phase 1: nu G into the staged blocks (entry [3 e + d] of block (a, b) for
// G[3a + d][3b + e]); every (row, col) with grp(row / 3) <= grp(col / 3) is
// written exactly once: directly from its upper tile, or, for a same-group
// pair below a tile boundary, as the transpose of its mirror.
__device__ inline void gram_stage_q(double* st, int wave, int lane,
                                    const f64x4_t acc[kGramTilesPerWave], double nu) {
#pragma unroll
  for (int t = 0; t < kGramTilesPerWave; ++t) {
    const int tile = wave + 4 * t;
    if (tile >= kGramQTiles) continue;
    const int I = cGramI[tile], J = cGramJ[tile];
    const int col = 16 * J + (lane & 15);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = 16 * I + (lane >> 4) + 4 * i;
      if (row >= 81 || col >= 81) continue;
      const double v = nu * acc[t][i];
      if (row / 9 <= col / 9) gram_slot(st, row / 3, col / 3)[3 * (col % 3) + row % 3] = v;
      if (I < J && row / 9 == col / 9) gram_slot(st, col / 3, row / 3)[3 * (row % 3) + col % 3] = v;
    }
  }
}

// Phase 2 (after phase 1 is visible): the diagonal m + nu L of every staged block.
__device__ inline void gram_stage_m(double* st, int wave, int lane,
                                    const f64x4_t acc[kGramTilesPerWave]) {
  const int tile = wave + 4 * (kGramTilesPerWave - 1);
  if (tile < kGramQTiles) return;
  const int I = cGramI[tile], J = cGramJ[tile];
  const int b = 16 * J + (lane & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int a = 16 * I + (lane >> 4) + 4 * i;
    if (a >= 27 || b >= 27) continue;
    const double m = acc[kGramTilesPerWave - 1][i];
    if (a / 3 <= b / 3) {
      double* s = gram_slot(st, a, b);
      const double d = m + (s[0] + s[4] + s[8]);
      s[0] += d; s[4] += d; s[8] += d;
    }
    if (I < J && a / 3 == b / 3) {
      double* s = gram_slot(st, b, a);
      const double d = m + (s[0] + s[4] + s[8]);
      s[0] += d; s[4] += d; s[8] += d;
    }
  }
}

// MODE 0: full distribute_local_to_global into block-CSR A, B^T, B (+ rhs);
// MODE 1: dense element output; MODE 2: the operator form of nse_matrix that
// the solve reads (B^T, B, rhs and the diagonal of the constrained velocity
// rows), with the velocity-velocity block left to the matrix-free apply
// (kernels/matfree.hip) and materialised only on request (MODE 0).
template <int MODE, bool GM>
__global__ __launch_bounds__(kNseThreads) void k_nse_system(CellData cd, ScatterMaps sm,
                                                            const int32_t* __restrict__ cells,
                                                            int first,
                                                            const double* __restrict__ u_old,
                                                            const double* __restrict__ T_old,
                                                            PhysicsDev ph, NseOut out) {
  __shared__ NseSmem sh;
  const int tid = threadIdx.x;
#ifndef DCP_ASM_XCD
#define DCP_ASM_XCD 0
#endif
  // DCP_ASM_XCD: each XCD takes one contiguous (tree-ordered) run of the colour class
  const int cell = MODE != 1 ? cells[DCP_ASM_XCD ? xcd_block(blockIdx.x, gridDim.x) : int(blockIdx.x)]
                             : first + blockIdx.x;
  const bool want_matrix = MODE == 1 || (MODE == 0 && out.A != nullptr);
  const bool want_B = want_matrix || (MODE == 2 && out.Bt != nullptr);
  const bool want_rhs = MODE == 1 || out.rhs != nullptr;
  const bool want_cdiag = MODE != 1 && out.cdiag != nullptr;

  const bool sep = cd.sep_col != nullptr;
  if (!sep && tid < 3 * kMapPts) sh.X[tid] = cd.geo[3 * kMapPts * size_t(cell) + tid];
  if (tid < 27) {
    const int n = cd.cell_q2[27 * size_t(cell) + tid];
    sh.node[tid] = n;
    const int o = cd.cell_q2o ? cd.cell_q2o[27 * size_t(cell) + tid] : n;
    sh.orig[tid] = o;
    // the old solutions at the cell's own dofs (cell->get_dof_values; for a
    // periodic image its own entry, not its partner's)
#pragma unroll
    for (int d = 0; d < 3; ++d) sh.U[3 * tid + d] = u_old[3 * size_t(o) + d];
  } else if (tid >= 64 && tid < 72) {
    const int v = tid - 64;
    sh.pdof[v] = cd.cell_p[8 * size_t(cell) + v];
    if (cd.tdpc == 8) sh.T[v] = T_old[(cd.cell_To ? cd.cell_To : cd.cell_T)[8 * size_t(cell) + v]];
  } else if (cd.tdpc == 27 && tid >= 96 && tid < 123) {
    sh.T[tid - 96] = T_old[cd.cell_T[27 * size_t(cell) + tid - 96]];
  }
  if (MODE == 0 && want_matrix)
    for (int i = tid; i < 729; i += kNseThreads) sh.pos[i] = sm.posA[729 * size_t(cell) + i];
  // MODE 2 with out.B == null: B^T only (B is its transpose, copied afterwards)
  const bool scatter_B = MODE != 2 || out.B != nullptr;
  if (MODE != 1 && want_B) {
    for (int i = tid; i < 216; i += kNseThreads) {
      sh.pos[729 + i] = sm.posBt[216 * size_t(cell) + i];
      if (scatter_B) sh.pos[945 + i] = sm.posB[216 * size_t(cell) + i];
    }
  }
  // reference shape values / gradients at the Gauss points, formed from the 1D
  // bases (a 23 KB table copy per cell would stream through L2 for every cell)
  for (int i = tid; i < 729; i += kNseThreads) {
    const int q = i / 27, n = i - 27 * q;
    const double xa = sel_gauss(q % 3), xb = sel_gauss((q / 3) % 3), xc = sel_gauss(q / 9);
    const int na = n % 3, nb = (n / 3) % 3, nc = n / 9;
    const double la = ce_l2(na, xa), lb = ce_l2(nb, xb), lc = ce_l2(nc, xc);
    sh.S[i] = la * lb * lc;
    sh.D[3 * i + 0] = ce_dl2(na, xa) * lb * lc;
    sh.D[3 * i + 1] = la * ce_dl2(nb, xb) * lc;
    sh.D[3 * i + 2] = la * lb * ce_dl2(nc, xc);
  }
  __syncthreads();

  // MappingQ(3): J[i][e] = sum_n X_n,i dN_n/dxi_e over the 64 support points, thread (q, i)
  // (timing probe only: DCP_OP_NOGEO skips the map and the gradient transform)
#ifndef DCP_OP_NOGEO
#define DCP_OP_NOGEO 0
#endif
#ifndef DCP_OP_NOMAP
#define DCP_OP_NOMAP 0  // timing probe: skips the map only (wrong results)
#endif
  if (sep) {
    if (tid < 27) sep_geometry(cd, cell, sh.geo, tid);
  } else {
  if (tid < 81 && !DCP_OP_NOGEO && !DCP_OP_NOMAP) {
    const int q = tid / 3, i = tid % 3;
    double J0, J1, J2, x;
    map_row(sh.X, q, i, x, J0, J1, J2);
    sh.geo.Ji[9 * q + 3 * i + 0] = J0;
    sh.geo.Ji[9 * q + 3 * i + 1] = J1;
    sh.geo.Ji[9 * q + 3 * i + 2] = J2;
    sh.geo.xq[3 * q + i] = x;
  }
  __syncthreads();
  double Jinv[9], jxw = 0;
  if (tid < 27) {
    const int q = tid;
    double J[3][3];
#pragma unroll
    for (int k = 0; k < 9; ++k) J[k / 3][k % 3] = sh.geo.Ji[9 * q + k];
    const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
    const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
    const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
    const double det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
    const double id = 1.0 / det;
    Jinv[0] = c00 * id;
    Jinv[1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * id;
    Jinv[2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * id;
    Jinv[3] = c01 * id;
    Jinv[4] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * id;
    Jinv[5] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * id;
    Jinv[6] = c02 * id;
    Jinv[7] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * id;
    Jinv[8] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * id;
    jxw = det * cW[q % 3] * cW[(q / 3) % 3] * cW[q / 9];
  }
  __syncthreads();   // all J reads done before Ji overwrites them
  if (tid < 27) {
#pragma unroll
    for (int k = 0; k < 9; ++k) sh.geo.Ji[9 * tid + k] = Jinv[k];
    sh.geo.JxW[tid] = jxw;
  }
  }
  __syncthreads();
  // physical gradients in place: grad_d = sum_e dN/dxi_e Ji[e][d]
  for (int i = tid; i < (DCP_OP_NOGEO ? 0 : 729); i += kNseThreads) {
    const double* Ji = &sh.geo.Ji[9 * (i / 27)];
    double* g = &sh.D[3 * i];
    const double r0 = g[0], r1 = g[1], r2 = g[2];
#pragma unroll
    for (int d = 0; d < 3; ++d) g[d] = r0 * Ji[d] + r1 * Ji[3 + d] + r2 * Ji[6 + d];
  }
  for (int i = tid; i < 216; i += kNseThreads) sh.W1[i] = sh.geo.JxW[i / 8] * cRef.S1[i];
  __syncthreads();

  if (want_rhs && tid < 27) {
    // Right-hand-side integrand per quadrature point (:593-650, 655-669).
    const int q = tid;
    double u[3] = {0, 0, 0}, G[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll 1
    for (int n = 0; n < 27; ++n) {
      const double s = sh.S[27 * q + n];
      const double* Dn = &sh.D[3 * (27 * q + n)];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const double un = sh.U[3 * n + c];
        u[c] += un * s;
        G[c][0] += un * Dn[0];
        G[c][1] += un * Dn[1];
        G[c][2] += un * Dn[2];
      }
    }
    double T = 0;
    if (cd.tdpc == 8) {
#pragma unroll
      for (int v = 0; v < 8; ++v) T += sh.T[v] * cRef.S1[8 * q + v];
    } else {
      // FE_Q(2) temperature: the Q2 basis of the velocity at the same points
      for (int n = 0; n < 27; ++n) T += sh.T[n] * sh.S[27 * q + n];
    }
    const double rho = 1 - ph.beta * (T - ph.T_ref);            // density_scaling
    double grav[3];
    if (ph.cuboid) {
      grav[0] = grav[1] = 0;
      grav[2] = -ph.g;                                            // vertical_gravity_vector
    } else {                                                      // gravity_vector (Q4)
      const double* x = &sh.geo.xq[3 * q];
      const double r = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
      const double den = r > 1 ? r : sqrt(r);
#pragma unroll
      for (int d = 0; d < 3; ++d) grav[d] = -ph.g * x[d] / den;
    }
    // (u . grad) u ; Coriolis 2 (Omega x u) with Omega = (0,0,coriolis_z) (Q2)
    const double cxu[3] = {-ph.coriolis_z * u[1], ph.coriolis_z * u[0], 0.0};
    const double w = sh.geo.JxW[q];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double adv = u[0] * G[c][0] + u[1] * G[c][1] + u[2] * G[c][2];
      sh.F[3 * q + c] = (u[c] + ph.dt * rho * (ph.grav_scale * grav[c]) - ph.dt * adv -
                         ph.dt * (2 * cxu[c])) * w;
    }
  }
  double kii_d[3] = {0, 0, 0};  // diag lanes: K_(a,c),(a,c) of node a
  if (((MODE == 0 && want_matrix) || want_cdiag) && tid >= 64 && tid < 91) {
    // node-diagonal blocks for the |K_ii| / average-diagonal rule
    const int a = tid - 64;
    double msum = 0, g2[3] = {0, 0, 0};
#pragma unroll 1
    for (int q = 0; q < 27; ++q) {
      const double w = sh.geo.JxW[q];
      const double* Da = &sh.D[3 * (27 * q + a)];
      const double sa = sh.S[27 * q + a];
      msum += w * sa * sa;
      g2[0] += w * Da[0] * Da[0];
      g2[1] += w * Da[1] * Da[1];
      g2[2] += w * Da[2] * Da[2];
    }
    const double L = g2[0] + g2[1] + g2[2];
#pragma unroll
    for (int c = 0; c < 3; ++c) kii_d[c] = msum + ph.nu_sys * L + ph.nu_sys * g2[c];
    sh.diag[a] = fabs(kii_d[0]) + fabs(kii_d[1]) + fabs(kii_d[2]);
  }
  __syncthreads();
  if (want_cdiag && tid >= 64 && tid < 91) {
    // diagonal of the constrained rows of nse_matrix: AffineConstraints puts
    // |K_ii| of every cell (the average diagonal if 0) on a constrained local
    // dof -- the original one for a periodic image (type 3, all components)
    const int n = sh.orig[tid - 64];
    const int ci = out.cidx[n];
    if (ci >= 0) {
      const NodeConstraint nc = cd.vcon[n];
      double avg = 0;
      for (int m = 0; m < 27; ++m) avg += sh.diag[m];
      avg /= 89.0;  // pressure diagonals of the local matrix are 0
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (nc.type == 1 || nc.type == 3 || c == nc.k) {
          const double d = fabs(kii_d[c]);
          out.cdiag[3 * size_t(ci) + c] += d != 0.0 ? d : avg;
        }
    }
  } else if (want_cdiag && cd.cell_po && tid >= 96 && tid < 104) {
    // identified pressure dofs: their local diagonal is 0, so the average
    const int po = cd.cell_po[8 * size_t(cell) + tid - 96];
    const int pci = out.pcidx[po];
    if (pci >= 0) {
      double avg = 0;
      for (int m = 0; m < 27; ++m) avg += sh.diag[m];
      out.pcdiag[pci] += avg / 89.0;
    }
  }

  constexpr int kAux = kNseThreads - kNseTiles;  // threads for B^T/B and rhs in MODE 1
  if (MODE == 1 && GM) {
    double* K = out.elemK + size_t(blockIdx.x) * 89 * 89;
    double* f = out.elemF + size_t(blockIdx.x) * 89;
    const int wave = tid >> 6, lane = tid & 63;
    f64x4_t acc[kGramTilesPerWave];
    gram_tiles(sh, wave, lane, acc);
    // B^T / B entries, rhs, the pressure rows (the tables are still live)
    for (int t = tid; t < 216 + 27 + 8; t += kNseThreads) {
      if (t < 216) {
        const int an = t / 8, v = t % 8;
        double bt[3];
        nse_div(sh, an, v, bt);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          K[89 * fesys_velocity(an, c) + 4 * v + 3] = bt[c];
          K[89 * (4 * v + 3) + fesys_velocity(an, c)] = bt[c];
        }
      } else if (t < 243) {
        const int an = t - 216;
        double fa[3];
        nse_rhs_node(sh, an, fa);
#pragma unroll
        for (int c = 0; c < 3; ++c) f[fesys_velocity(an, c)] = fa[c];
      } else {
        const int v = t - 243;
        f[4 * v + 3] = 0.0;
        for (int w = 0; w < 8; ++w) K[89 * (4 * v + 3) + 4 * w + 3] = 0.0;
      }
    }
    __syncthreads();  // tables dead: stage the velocity blocks over them
    double* stage = sh.X;
    gram_stage_q(stage, wave, lane, acc, ph.nu_sys);
    __syncthreads();
    gram_stage_m(stage, wave, lane, acc);
    __syncthreads();
    for (int e = tid; e < 729 * 9; e += kNseThreads) {
      const int pr = e / 9, comp = e - 9 * pr;
      const int a = pr / 27, b = pr - 27 * a;
      const int sl = cSlot.s[pr];
      const int i = comp / 3, j = comp - 3 * i;
      const double v = stage[9 * (sl & 0x7fff) + ((sl & 0x8000) ? 3 * j + i : comp)];
      K[89 * fesys_velocity(a, i) + fesys_velocity(b, j)] = v;
    }
    return;
  }
  if (MODE == 1) {
    double* K = out.elemK + size_t(blockIdx.x) * 89 * 89;
    double* f = out.elemF + size_t(blockIdx.x) * 89;
    if (tid < kNseTiles) {
      const int A = cPairA[tid / 3], B = cPairB[tid / 3];
      const int a = 3 * A + tid % 3, b0 = 3 * B;
      double blk[3][9];
      nse_tile(sh, ph, a, b0, blk);
#pragma unroll
      for (int tt = 0; tt < 3; ++tt)
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int cp = 0; cp < 3; ++cp) {
            const int ia = fesys_velocity(a, c), ib = fesys_velocity(b0 + tt, cp);
            K[89 * ia + ib] = blk[tt][3 * c + cp];
            if (A != B) K[89 * ib + ia] = blk[tt][3 * c + cp];
          }
    } else {
      for (int t = tid - kNseTiles; t < 216 + 27 + 8; t += kAux) {
        if (t < 216) {
          const int an = t / 8, v = t % 8;
          double bt[3];
          nse_div(sh, an, v, bt);
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            K[89 * fesys_velocity(an, c) + 4 * v + 3] = bt[c];
            K[89 * (4 * v + 3) + fesys_velocity(an, c)] = bt[c];
          }
        } else if (t < 243) {
          const int an = t - 216;
          double fa[3];
          nse_rhs_node(sh, an, fa);
#pragma unroll
          for (int c = 0; c < 3; ++c) f[fesys_velocity(an, c)] = fa[c];
        } else {
          const int v = t - 243;  // pressure rows of f and the empty p-p block
          f[4 * v + 3] = 0.0;
          for (int w = 0; w < 8; ++w) K[89 * (4 * v + 3) + 4 * w + 3] = 0.0;
        }
      }
    }
    return;
  }

  if (MODE == 2) {
    // B^T rows (an, v): one per thread, condensed C_a^T b; rhs nodes on 27 more
    // (timing probes only: DCP_OP_NOBT skips the rows, DCP_OP_NOSCATTER the
    // matrix writes; both give wrong matrices)
#ifndef DCP_OP_NOBT
#define DCP_OP_NOBT 0
#endif
#ifndef DCP_OP_NOSCATTER
#define DCP_OP_NOSCATTER 0
#endif
    double bt[3] = {0, 0, 0};
    if (want_B && tid < 216 && !DCP_OP_NOBT) {
      nse_div(sh, tid / 8, tid % 8, bt);
      double Ca[3][3];
      condensation(cd.vcon[sh.node[tid / 8]], Ca);
      const double b0 = bt[0], b1 = bt[1], b2 = bt[2];
#pragma unroll
      for (int j = 0; j < 3; ++j) bt[j] = Ca[0][j] * b0 + Ca[1][j] * b1 + Ca[2][j] * b2;
    } else if (want_rhs && tid >= 216 && tid < 216 + 27) {
      const int an = tid - 216;
      double fa[3];
      nse_rhs_node(sh, an, fa);
      double Ca[3][3];
      condensation(cd.vcon[sh.node[an]], Ca);
      double* dst = out.rhs + 3 * size_t(sh.node[an]);
#pragma unroll
      for (int j = 0; j < 3; ++j) dst[j] += Ca[0][j] * fa[0] + Ca[1][j] * fa[1] + Ca[2][j] * fa[2];
    }
    if (!want_B || DCP_OP_NOSCATTER) return;
    __syncthreads();  // gradient tables dead: stage the rows for the all-wave scatter
    double* stage = sh.X;
    if (tid < 216) {
#pragma unroll
      for (int j = 0; j < 3; ++j) stage[kStageA + 3 * tid + j] = bt[j];
    }
    __syncthreads();
    // B^T then B rows: elements [729 * 9, kScatterElems) of the MODE 0 order
    // (B^T rows only: [729 * 9, 729 * 9 + 648))
    constexpr int kOpBatch = (2 * 648 + kNseThreads - 1) / kNseThreads;  // 6
    const int e_end = scatter_B ? kScatterElems : 729 * 9 + 648;
    double old[kOpBatch];
#pragma unroll
    for (int j = 0; j < kOpBatch; ++j) {
      const int e = 729 * 9 + tid + j * kNseThreads;
      old[j] = 0.0;
      if (e < e_end) {
        bool add;
        double v;
        const double* dst = scatter_target(sh, out, e, add, v);
        if (add) old[j] = *dst;
      }
    }
#pragma unroll
    for (int j = 0; j < kOpBatch; ++j) {
      const int e = 729 * 9 + tid + j * kNseThreads;
      if (e < e_end) {
        bool add;
        double v;
        double* dst = scatter_target(sh, out, e, add, v);
        *dst = old[j] + v;
      }
    }
    return;
  }

  // ---- MODE 0: condensation + colour-exclusive scatter ----------------------
  const int wave = tid >> 6, lane = tid & 63;
  double blk[3][9];   // tile lanes: element blocks (a, b0+tt); wave 3: B^T rows
  double fa[3] = {0, 0, 0};
  const bool tile_lane = want_matrix && tid < kNseTiles;
  const bool rhs_lane = want_rhs && tid >= kRhsLane0 && tid < kRhsLane0 + 27;
  f64x4_t acc[kGramTilesPerWave];
  if (GM && want_matrix) gram_tiles(sh, wave, lane, acc);  // block-uniform branch
  if (tile_lane && !GM) {
    const int A = cPairA[tid / 3], B = cPairB[tid / 3];
    nse_tile(sh, ph, 3 * A + tid % 3, 3 * B, blk);
  } else if (rhs_lane) {
    nse_rhs_node(sh, tid - kRhsLane0, fa);
  } else if (want_matrix && wave == 3) {
    // B^T rows (an, v), 4 rounds of 64
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = lane + 64 * k;
      if (t < 216) nse_div(sh, t / 8, t % 8, &blk[0][0] + 3 * k);
    }
  }
  __syncthreads();   // geometry and gradient tables dead: reuse them as the write staging area
  double* stage = sh.X;
  if (GM && want_matrix) {
    gram_stage_q(stage, wave, lane, acc, ph.nu_sys);
    __syncthreads();
    gram_stage_m(stage, wave, lane, acc);
    __syncthreads();
  }
  if (tile_lane) {
    const int A = cPairA[tid / 3], B = cPairB[tid / 3];
    const int a = 3 * A + tid % 3, b0 = 3 * B;
    double* slot = stage + 27 * tid;   // slots 3 tid + tt
    if (!GM) {
#pragma unroll
      for (int i = 0; i < 27; ++i) slot[i] = blk[i / 9][i % 9];
    }
    // condensation C_a^T K C_b in place, only where a constraint is involved
    const NodeConstraint ca = cd.vcon[sh.node[a]];
#pragma unroll 1
    for (int tt = 0; tt < 3; ++tt) {
      const int b = b0 + tt;
      const NodeConstraint cb = cd.vcon[sh.node[b]];
      if (ca.type == 0 && cb.type == 0) continue;
      double* K = slot + 9 * tt;
      double Ca[3][3], Cb[3][3], KC[3][3];
      condensation(ca, Ca);
      condensation(cb, Cb);
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          KC[i][j] = K[3 * i] * Cb[0][j] + K[3 * i + 1] * Cb[1][j] + K[3 * i + 2] * Cb[2][j];
      double kii[3] = {K[0], K[4], K[8]};
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          K[3 * i + j] = Ca[0][i] * KC[0][j] + Ca[1][i] * KC[1][j] + Ca[2][i] * KC[2][j];
      if (b == a && ca.type != 0 && sh.orig[a] == sh.node[a]) {
        // constrained local dofs: global diagonal += |K_ii| (average if 0)
        double avg = 0;
        for (int n = 0; n < 27; ++n) avg += sh.diag[n];
        avg /= 89.0;  // pressure diagonals of the local matrix are 0
#pragma unroll
        for (int c = 0; c < 3; ++c)
          if (ca.type == 1 || c == ca.k) {
            const double d = fabs(kii[c]);
            K[4 * c] += d != 0.0 ? d : avg;
          }
      }
    }
  } else if (rhs_lane) {
    const int an = tid - kRhsLane0;
    double Ca[3][3];
    condensation(cd.vcon[sh.node[an]], Ca);
    double* dst = out.rhs + 3 * size_t(sh.node[an]);
#pragma unroll
    for (int j = 0; j < 3; ++j) dst[j] += Ca[0][j] * fa[0] + Ca[1][j] * fa[1] + Ca[2][j] * fa[2];
  } else if (want_matrix && wave == 3) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = lane + 64 * k;
      if (t < 216) {
        const double* bt = &blk[0][0] + 3 * k;
        double Ca[3][3];
        condensation(cd.vcon[sh.node[t / 8]], Ca);
#pragma unroll
        for (int j = 0; j < 3; ++j)
          stage[kStageA + 3 * t + j] = Ca[0][j] * bt[0] + Ca[1][j] * bt[1] + Ca[2][j] * bt[2];
      }
    }
  }
  if (!want_matrix) return;
  __syncthreads();
  // all four waves: read-modify-write / first-touch store of the 7857 doubles
  // (timing probes only: DCP_ASM_STOREONLY drops the reads, DCP_ASM_NOWRITE
  // all but the first block's writes; both give wrong matrices)
#ifndef DCP_ASM_STOREONLY
#define DCP_ASM_STOREONLY 0
#endif
#ifndef DCP_ASM_NOWRITE
#define DCP_ASM_NOWRITE 0
#endif
  constexpr int kElems = DCP_ASM_NOWRITE ? 9 : kScatterElems;
  for (int e0 = tid; e0 < kElems; e0 += kNseThreads * kScatterBatch) {
    double old[kScatterBatch];
#pragma unroll
    for (int j = 0; j < kScatterBatch; ++j) {
      const int e = e0 + j * kNseThreads;
      old[j] = 0.0;
      if (e < kElems) {
        bool add;
        double v;
        const double* dst = scatter_target(sh, out, e, add, v);
        if (add && !DCP_ASM_STOREONLY) old[j] = *dst;
      }
    }
#pragma unroll
    for (int j = 0; j < kScatterBatch; ++j) {
      const int e = e0 + j * kNseThreads;
      if (e < kElems) {
        bool add;
        double v;
        double* dst = scatter_target(sh, out, e, add, v);
        *dst = old[j] + v;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Preconditioner diagonals: the velocity block of local_assemble_nse_preconditioner
// couples only equal components, P_(a,c),(a,c) = M_aa + dt/Re |grad s_a|^2,
// so diag(C^T P C) is (1 + w_d^2) p for the free components of a
// no-normal-flux node, p for constrained components (the |K_ii| rule).
__global__ __launch_bounds__(64) void k_nse_precond_diag(CellData cd, const int32_t* __restrict__ cells,
                                                         PhysicsDev ph, double* A_diag,
                                                         double* Mp_diag) {
  __shared__ double X[3 * kMapPts];
  __shared__ Geo geo;
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  if (!cd.sep_col)
    for (int i = tid; i < 3 * kMapPts; i += 64) X[i] = cd.geo[3 * kMapPts * size_t(cell) + i];
  __syncthreads();
  if (tid < 27) {
    if (cd.sep_col) sep_geometry(cd, cell, geo, tid);
    else cell_geometry(X, geo, tid);
  }
  __syncthreads();
  if (tid < 27) {
    const int a = tid;
    double p = 0;
    for (int q = 0; q < 27; ++q) {
      double g[3];
      q2_grad(geo, q, a, g);
      const double s = q2_value(q, a);
      p += (s * s + ph.nu_pre * (g[0] * g[0] + g[1] * g[1] + g[2] * g[2])) * geo.JxW[q];
    }
    const int n = cd.cell_q2[27 * size_t(cell) + a];
    const int o = cd.cell_q2o ? cd.cell_q2o[27 * size_t(cell) + a] : n;
    const NodeConstraint nc = cd.vcon[n];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const bool con = nc.type == 1 || (nc.type == 2 && d == nc.k);
      double f = 1.0;
      if (nc.type == 2 && d != nc.k) f = 1.0 + nc.w[d] * nc.w[d];
      // a periodic image: condensed onto its partner, |P_ii| onto itself
      if (o == n || !con) A_diag[3 * size_t(n) + d] += f * p;
      if (o != n) A_diag[3 * size_t(o) + d] += p;
    }
  } else if (tid >= 32 && tid < 40) {
    const int v = tid - 32;
    double p = 0;
    for (int q = 0; q < 27; ++q) {
      const double s = q1_value(q, v);
      p += s * s * geo.JxW[q];
    }
    const int pi = cd.cell_p[8 * size_t(cell) + v];
    Mp_diag[pi] += p;
    if (cd.cell_po && cd.cell_po[8 * size_t(cell) + v] != pi) Mp_diag[cd.cell_po[8 * size_t(cell) + v]] += p;
  }
}

// ---------------------------------------------------------------------------
// Temperature mass / stiffness (Q1, QGauss(3)) with Dirichlet condensation.
__global__ __launch_bounds__(64) void k_T_matrix(CellData cd, ScatterMaps sm,
                                                 const int32_t* __restrict__ cells, PhysicsDev ph,
                                                 double* Tmass, double* Tstiff,
                                                 const int32_t* __restrict__ posTs) {
  __shared__ double X[3 * kMapPts];
  __shared__ Geo geo;
  __shared__ double G1[27 * 8 * 3];
  __shared__ int dof[8];
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  if (!cd.sep_col)
    for (int i = tid; i < 3 * kMapPts; i += 64) X[i] = cd.geo[3 * kMapPts * size_t(cell) + i];
  if (tid >= 32 && tid < 40) dof[tid - 32] = cd.cell_T[8 * size_t(cell) + tid - 32];
  __syncthreads();
  if (tid < 27) {
    if (cd.sep_col) sep_geometry(cd, cell, geo, tid);
    else cell_geometry(X, geo, tid);
  }
  __syncthreads();
  for (int i = tid; i < 216; i += 64) q1_grad(geo, i / 8, i % 8, &G1[3 * i]);
  __syncthreads();
  const int i = tid / 8, j = tid % 8;
  double M = 0, K = 0;
  for (int q = 0; q < 27; ++q) {
    const double w = geo.JxW[q];
    M += q1_value(q, i) * q1_value(q, j) * w;
    const double* gi = &G1[3 * (8 * q + i)];
    const double* gj = &G1[3 * (8 * q + j)];
    K += (gi[0] * gj[0] + gi[1] * gj[1] + gi[2] * gj[2]) * ph.one_over_peclet * w;
  }
  const bool fi = cd.T_fixed[dof[i]], fj = cd.T_fixed[dof[j]];
  const size_t pos = size_t(sm.posT[64 * size_t(cell) + tid]);
  if (!fi && !fj) {
    Tmass[pos] += M;
    Tstiff[pos] += K;
  } else if (i == j) {
    Tmass[pos] += fabs(M);
    Tstiff[pos] += fabs(K);
  }
  if (posTs && i == j) {
    // a periodic image: its own (constrained) diagonal entry
    const int ps = posTs[8 * size_t(cell) + i];
    if (ps >= 0) {
      Tmass[ps] += fabs(M);
      Tstiff[ps] += fabs(K);
    }
  }
}

__global__ void k_image_diag(int n, const int32_t* __restrict__ node, const int64_t* __restrict__ blk,
                             const int32_t* __restrict__ cidx, const double* __restrict__ cdiag,
                             double* __restrict__ A) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const double* d = cdiag + 3 * size_t(cidx[node[k]]);
  double* b = A + 9 * size_t(blk[k]);
#pragma unroll
  for (int e = 0; e < 9; ++e) b[e] = (e % 4 == 0) ? d[e / 4] : 0.0;
}

// Temperature rhs with the matrix_for_bc lift of inhomogeneous Dirichlet dofs.
__global__ __launch_bounds__(64) void k_T_rhs(CellData cd, const int32_t* __restrict__ cells,
                                              const double* __restrict__ T_old,
                                              const double* __restrict__ u_cur, PhysicsDev ph,
                                              double* rhs) {
  __shared__ double X[3 * kMapPts], U[81];
  __shared__ Geo geo;
  __shared__ double G1[27 * 8 * 3];
  __shared__ double Tq[27], Fq[27];
  __shared__ double Tn[8];
  __shared__ int dof[8];
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  if (!cd.sep_col)
    for (int i = tid; i < 3 * kMapPts; i += 64) X[i] = cd.geo[3 * kMapPts * size_t(cell) + i];
  if (tid < 27) {
    const int n = (cd.cell_q2o ? cd.cell_q2o : cd.cell_q2)[27 * size_t(cell) + tid];
#pragma unroll
    for (int d = 0; d < 3; ++d) U[3 * tid + d] = u_cur[3 * size_t(n) + d];
  } else if (tid >= 32 && tid < 40) {
    const int d = cd.cell_T[8 * size_t(cell) + tid - 32];
    dof[tid - 32] = d;
    Tn[tid - 32] = T_old[(cd.cell_To ? cd.cell_To : cd.cell_T)[8 * size_t(cell) + tid - 32]];
  }
  __syncthreads();
  if (tid < 27) {
    if (cd.sep_col) sep_geometry(cd, cell, geo, tid);
    else cell_geometry(X, geo, tid);
  }
  __syncthreads();
  for (int i = tid; i < 216; i += 64) q1_grad(geo, i / 8, i % 8, &G1[3 * i]);
  __syncthreads();
  if (tid < 27) {
    const int q = tid;
    double T = 0, gT[3] = {0, 0, 0}, u[3] = {0, 0, 0};
    for (int v = 0; v < 8; ++v) {
      T += Tn[v] * q1_value(q, v);
      const double* g = &G1[3 * (8 * q + v)];
      gT[0] += Tn[v] * g[0]; gT[1] += Tn[v] * g[1]; gT[2] += Tn[v] * g[2];
    }
    for (int n = 0; n < 27; ++n) {
      const double s = q2_value(q, n);
      u[0] += U[3 * n] * s; u[1] += U[3 * n + 1] * s; u[2] += U[3 * n + 2] * s;
    }
    const double w = geo.JxW[q];
    Tq[q] = T * w;
    Fq[q] = ph.dt_T * (u[0] * gT[0] + u[1] * gT[1] + u[2] * gT[2]) * w;
  }
  __syncthreads();
  if (tid < 8) {
    const int j = tid;
    if (cd.T_fixed[dof[j]]) return;  // constrained rows receive nothing
    double f = 0;
    for (int q = 0; q < 27; ++q) f += q1_value(q, j) * (Tq[q] - Fq[q]);
    // lift: - sum_{i inhomogeneous} g_i (M + dt_T K)_ji
    for (int i = 0; i < 8; ++i) {
      if (!cd.T_fixed[dof[i]]) continue;
      const double g = cd.T_bc[dof[i]];
      if (g == 0.0) continue;
      double mb = 0;
      for (int q = 0; q < 27; ++q) {
        const double* gi = &G1[3 * (8 * q + i)];
        const double* gj = &G1[3 * (8 * q + j)];
        mb += (q1_value(q, i) * q1_value(q, j) +
               ph.dt_T * ph.one_over_peclet * (gi[0] * gj[0] + gi[1] * gj[1] + gi[2] * gj[2])) *
              geo.JxW[q];
      }
      f -= g * mb;
    }
    rhs[dof[j]] += f;
  }
}

// ---------------------------------------------------------------------------
__device__ inline int find_sorted(const int32_t* __restrict__ col, int b, int e, int key) {
  while (b < e) {
    const int m = (b + e) >> 1;
    if (col[m] < key) b = m + 1; else e = m;
  }
  return b;
}

__global__ void k_scatter_maps(CellData cd, const int32_t* A_ptr, const int32_t* A_col,
                               const int32_t* Bt_ptr, const int32_t* Bt_col, const int32_t* B_ptr,
                               const int32_t* B_col, const int32_t* T_ptr, const int32_t* T_col,
                               int32_t* posA, int32_t* posBt, int32_t* posB, int32_t* posT) {
  const int cell = blockIdx.x;
  const int32_t* nodes = cd.cell_q2 + 27 * size_t(cell);
  const int32_t* pd = cd.cell_p + 8 * size_t(cell);
  const int tp = cd.tdpc;
  const int32_t* td = cd.cell_T + tp * size_t(cell);
  for (int i = threadIdx.x; i < 729; i += blockDim.x) {
    const int ra = nodes[i / 27], cb = nodes[i % 27];
    posA[729 * size_t(cell) + i] = find_sorted(A_col, A_ptr[ra], A_ptr[ra + 1], cb);
  }
  for (int i = threadIdx.x; i < 216; i += blockDim.x) {
    const int ra = nodes[i / 8], v = pd[i % 8];
    posBt[216 * size_t(cell) + i] = find_sorted(Bt_col, Bt_ptr[ra], Bt_ptr[ra + 1], v);
    const int rv = pd[i / 27], cn = nodes[i % 27];
    posB[216 * size_t(cell) + i] = find_sorted(B_col, B_ptr[rv], B_ptr[rv + 1], cn);
  }
  for (int i = threadIdx.x; i < tp * tp; i += blockDim.x) {
    const int r = td[i / tp], c = td[i % tp];
    posT[size_t(tp) * tp * cell + i] = find_sorted(T_col, T_ptr[r], T_ptr[r + 1], c);
  }
}

// First-touch marks for one colour: an entry whose block no earlier colour
// touched is re-encoded as ~pos. Within a colour no two cells share a node, so
// every block is touched at most once per launch.
__global__ __launch_bounds__(256) void k_first_touch(const int32_t* __restrict__ cells, int per_cell,
                                                     int32_t* __restrict__ pos,
                                                     uint8_t* __restrict__ touched,
                                                     unsigned long long* __restrict__ count) {
  __shared__ unsigned int n_first;
  if (threadIdx.x == 0) n_first = 0;
  __syncthreads();
  int32_t* pc = pos + size_t(per_cell) * cells[blockIdx.x];
  unsigned int mine = 0;
  for (int i = threadIdx.x; i < per_cell; i += blockDim.x) {
    const int32_t p = pc[i];
    if (p >= 0 && !touched[p]) {
      touched[p] = 1;
      pc[i] = ~p;
      ++mine;
    }
  }
  if (mine) atomicAdd(&n_first, mine);
  __syncthreads();
  if (threadIdx.x == 0 && n_first) atomicAdd(count, (unsigned long long)n_first);
}

__global__ void k_clear_first_touch(size_t n, int32_t* __restrict__ pos) {
  for (size_t i = blockIdx.x * size_t(blockDim.x) + threadIdx.x; i < n; i += size_t(gridDim.x) * blockDim.x)
    if (pos[i] < 0) pos[i] = ~pos[i];
}

// S_pq = sum_n sum_c B[p][n][c] d[3n+c] B^T[n][q][c]; one wave per pressure
// row. The row's nodes (n, the weights B[p][n][c] d[3n+c], the B^T row range)
// are staged in LDS first, all lanes at once; then the node loop runs in node
// order, 2 kSchurU nodes per iteration (one per half-wave) with their B^T
// loads and column searches issued together, each lane one entry q of a
// node's B^T row (distinct q per node: the adds into the row's accumulators
// keep node order, and one wave needs no barrier between nodes). Every entry
// is summed in the same (node) order as before.
constexpr int kSchurU = 4;
__global__ __launch_bounds__(64) void k_schur_form(int n_p, const int32_t* __restrict__ B_ptr,
                                                   const int32_t* __restrict__ B_col,
                                                   const double* __restrict__ B_val,
                                                   const int32_t* __restrict__ tperm,
                                                   const int32_t* __restrict__ Bt_ptr,
                                                   const int32_t* __restrict__ Bt_col,
                                                   const double* __restrict__ Bt_val,
                                                   const double* __restrict__ d,
                                                   const int32_t* __restrict__ S_ptr,
                                                   const int32_t* __restrict__ S_col,
                                                   const int32_t* __restrict__ pmap,
                                                   double* __restrict__ S_val, int max_row) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int p = blockIdx.x, lane = threadIdx.x;
  const int s0 = S_ptr[p], len = S_ptr[p + 1] - s0;
  const int k0 = B_ptr[p], nb = B_ptr[p + 1] - k0;
  double* acc = reinterpret_cast<double*>(smem);
  double* wv = acc + max_row;                                   // [nb][3]
  int* cols = reinterpret_cast<int*>(wv + 3 * size_t(max_row)); // [len]
  int* rb = cols + max_row;                                     // [nb] B^T row begin
  int* rn = rb + max_row;                                       // [nb] B^T row length
  for (int j = lane; j < len; j += 64) {
    acc[j] = 0.0;
    cols[j] = S_col[s0 + j];
  }
  for (int i = lane; i < nb; i += 64) {
    const int k = k0 + i;
    const size_t n = size_t(B_col[k]);
    // B[p][n] = B^T[n][p] (tperm: B not materialised)
    const double* bk = tperm ? Bt_val + 3 * size_t(tperm[k]) : B_val + 3 * size_t(k);
    wv[3 * i] = bk[0] * d[3 * n];
    wv[3 * i + 1] = bk[1] * d[3 * n + 1];
    wv[3 * i + 2] = bk[2] * d[3 * n + 2];
    const int b = Bt_ptr[n];
    rb[i] = b;
    rn[i] = Bt_ptr[n + 1] - b;
  }
  __syncthreads();
  auto find = [&](int q) {
    int lo = 0, hi = len;
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (cols[m] < q) lo = m + 1; else hi = m;
    }
    return lo;
  };
  // half-waves: nodes i0 + 2u (lanes 0-31) and i0 + 2u + 1 (lanes 32-63), one
  // lane per B^T row entry (<= 32); the two halves' adds run one after the
  // other, so node order is kept
  const int half = lane >> 5, hl = lane & 31;
  for (int i0 = 0; i0 < nb; i0 += 2 * kSchurU) {
    int q[kSchurU], pos[kSchurU];
    double val[kSchurU];
#pragma unroll
    for (int u = 0; u < kSchurU; ++u) {
      const int i = i0 + 2 * u + half;
      const bool on = i < nb && hl < rn[i < nb ? i : 0];
      const int j = on ? rb[i] + hl : 0;
      q[u] = on ? Bt_col[j] : -1;
      const double b0 = on ? Bt_val[3 * size_t(j)] : 0.0;
      const double b1 = on ? Bt_val[3 * size_t(j) + 1] : 0.0;
      const double b2 = on ? Bt_val[3 * size_t(j) + 2] : 0.0;
      val[u] = on ? wv[3 * i] * b0 + wv[3 * i + 1] * b1 + wv[3 * i + 2] * b2 : 0.0;
    }
#pragma unroll
    for (int u = 0; u < kSchurU; ++u) pos[u] = q[u] >= 0 ? find(q[u]) : 0;
    // node 2u (half 0) before node 2u + 1 (half 1): two masked read-modify-
    // writes kept apart (a merged one would lose an update where both halves
    // hit the same column)
#pragma unroll
    for (int u = 0; u < kSchurU; ++u) {
      if (half == 0 && q[u] >= 0) acc[pos[u]] += val[u];
      __builtin_amdgcn_wave_barrier();
      if (half == 1 && q[u] >= 0) acc[pos[u]] += val[u];
      __builtin_amdgcn_wave_barrier();
    }
  }
  __syncthreads();
  if (pmap) {
    for (int j = lane; j < len; j += 64) S_val[pmap[s0 + j]] = acc[j];
  } else {
    for (int j = lane; j < len; j += 64) S_val[s0 + j] = acc[j];
  }
}

}  // namespace

void form_schur_complement(int n_p, const int32_t* B_ptr, const int32_t* B_col, const double* B_val,
                           const int32_t* tperm, const int32_t* Bt_ptr, const int32_t* Bt_col,
                           const double* Bt_val,
                           const double* d, const int32_t* S_ptr, const int32_t* S_col,
                           const int32_t* pmap, double* S_val, int max_row, hipStream_t s) {
  if (n_p <= 0) return;
  // max_row bounds both the S row and the B row (nodes) lengths
  const size_t lds = size_t(max_row) * (4 * sizeof(double) + 3 * sizeof(int)) + 16;
  hipLaunchKernelGGL(k_schur_form, dim3(n_p), dim3(64), lds, s, n_p, B_ptr, B_col, B_val, tperm, Bt_ptr,
                     Bt_col, Bt_val, d, S_ptr, S_col, pmap, S_val, max_row);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_nse_system(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                       const double* u_old, const double* T_old, const PhysicsDev& ph,
                       const NseOut& out, hipStream_t s, bool mfma) {
  if (n <= 0) return;
  if (mfma)
    hipLaunchKernelGGL((k_nse_system<0, true>), dim3(n), dim3(kNseThreads), 0, s, cd, sm, cells, 0,
                       u_old, T_old, ph, out);
  else
    hipLaunchKernelGGL((k_nse_system<0, false>), dim3(n), dim3(kNseThreads), 0, s, cd, sm, cells, 0,
                       u_old, T_old, ph, out);
  DCP_HIP_CHECK(hipGetLastError());
}

namespace {

// ---------------------------------------------------------------------------
// Operator form on the radially separable shell, one wave per cell
// (k_nse_system<2> keeps one 256-thread workgroup per cell for every other
// mesh). The 256-thread form spends most of its 3.4 ms at r=5 in
// workgroup-barrier phases with 27-81 active lanes; here a 64-lane wave owns a
// cell, lanes hold Gauss points (rhs integrand) or (node, 4 vertices) pairs
// (B^T rows), reference shape values and gradients are formed in registers,
// and the only synchronisation is the wave's own (no __syncthreads). Every
// product and sum runs in k_nse_system's order (the q loops, the condensation,
// the staged scatter), so the result is bitwise that of k_nse_system<2> / <0>
// where they overlap.
struct OpWaveSmem {
  union {
    struct {
      double U[81], T[27];
      Geo geo;
      double F[81];
      double diag[27];
    } a;
    double stage[648];  // condensed B^T rows (8 an + v), after the phases above
  };
  int node[27];
  int pos[432];  // posBt, then posB (scatter_B)
};
#ifndef DCP_OPW_WAVES
#define DCP_OPW_WAVES 4
#endif
constexpr int kOpWaves = DCP_OPW_WAVES;  // waves (cells) per workgroup
// colour classes below this many cells take the workgroup-per-cell kernel
constexpr int kOpSmallColour = 1024;
// timing probes only (wrong results): DCP_OPW_NOSCATTER skips the B^T / B
// scatter, DCP_OPW_NORHS the rhs integrand, DCP_OPW_NOBT the B^T rows
#ifndef DCP_OPW_NOSCATTER
#define DCP_OPW_NOSCATTER 0
#endif
#ifndef DCP_OPW_NORHS
#define DCP_OPW_NORHS 0
#endif
#ifndef DCP_OPW_NOBT
#define DCP_OPW_NOBT 0
#endif
#ifndef DCP_OPW_BATCH
#define DCP_OPW_BATCH 14
#endif

__device__ inline double sel3v(int i, const double (&v)[3]) {
  return i == 0 ? v[0] : (i == 1 ? v[1] : v[2]);
}

// wave-level LDS hand-off (a cell never spans waves)
__device__ inline void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


__global__ __launch_bounds__(64 * kOpWaves) void k_nse_operator_wave(
    CellData cd, ScatterMaps sm, const int32_t* __restrict__ cells, int n_cells,
    const double* __restrict__ u_old, const double* __restrict__ T_old, PhysicsDev ph, NseOut out) {
  __shared__ OpWaveSmem smem[kOpWaves];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int k = int(blockIdx.x) * kOpWaves + wave;
  if (k >= n_cells) return;
  OpWaveSmem& sh = smem[wave];
  const int cell = cells[k];
  const bool want_B = out.Bt != nullptr;
  const bool scatter_B = out.B != nullptr;
  const bool want_rhs = out.rhs != nullptr;
  const bool want_cdiag = out.cdiag != nullptr;
  // ---- state, scatter positions, geometry
  if (lane < 27) {
    const int nd = cd.cell_q2[27 * size_t(cell) + lane];
    sh.node[lane] = nd;
#pragma unroll
    for (int d = 0; d < 3; ++d) sh.a.U[3 * lane + d] = u_old[3 * size_t(nd) + d];
    if (cd.tdpc == 27) sh.a.T[lane] = T_old[cd.cell_T[27 * size_t(cell) + lane]];
    sep_geometry(cd, cell, sh.a.geo, lane);
  } else if (lane >= 32 && lane < 40 && cd.tdpc == 8) {
    sh.a.T[lane - 32] = T_old[cd.cell_T[8 * size_t(cell) + lane - 32]];
  }
  if (want_B)
    for (int i = lane; i < 216; i += 64) {
      sh.pos[i] = sm.posBt[216 * size_t(cell) + i];
      if (scatter_B) sh.pos[216 + i] = sm.posB[216 * size_t(cell) + i];
    }
  wsync();
  // ---- rhs integrand per Gauss point (lanes 0-26), k_nse_system's formulas
  if (want_rhs && lane < 27 && !DCP_OPW_NORHS) {
    const int q = lane;
    const double xa = sel_gauss(q % 3), xb = sel_gauss((q / 3) % 3), xc = sel_gauss(q / 9);
    const double* Ji = &sh.a.geo.Ji[9 * q];
    // the 1D factors at this lane's point; the node loop indexes them at
    // compile time (same values and products as the table k_nse_system builds)
    double LA[3], DA[3], LB[3], DB[3], LC[3], DC[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      LA[i] = ce_l2(i, xa);
      DA[i] = ce_dl2(i, xa);
      LB[i] = ce_l2(i, xb);
      DB[i] = ce_dl2(i, xb);
      LC[i] = ce_l2(i, xc);
      DC[i] = ce_dl2(i, xc);
    }
    double u[3] = {0, 0, 0}, G[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    // nodes n = na + 3 nb + 9 nc in order; na unrolled (register factors),
    // the nb / nc factors picked once per row of three
#pragma unroll 1
    for (int nc = 0; nc < 3; ++nc) {
      const double lc = sel3v(nc, LC), dc = sel3v(nc, DC);
#pragma unroll 1
      for (int nb = 0; nb < 3; ++nb) {
        const double lb = sel3v(nb, LB), db = sel3v(nb, DB);
#pragma unroll
        for (int na = 0; na < 3; ++na) {
          const int n = na + 3 * nb + 9 * nc;
          const double s = LA[na] * lb * lc;
          const double r0 = DA[na] * lb * lc;
          const double r1 = LA[na] * db * lc;
          const double r2 = LA[na] * lb * dc;
          double Dn[3];
#pragma unroll
          for (int d = 0; d < 3; ++d) Dn[d] = r0 * Ji[d] + r1 * Ji[3 + d] + r2 * Ji[6 + d];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const double un = sh.a.U[3 * n + c];
            u[c] += un * s;
            G[c][0] += un * Dn[0];
            G[c][1] += un * Dn[1];
            G[c][2] += un * Dn[2];
          }
        }
      }
    }
    double T = 0;
    if (cd.tdpc == 8) {
#pragma unroll
      for (int v = 0; v < 8; ++v) T += sh.a.T[v] * cRef.S1[8 * q + v];
    } else {
      for (int n = 0; n < 27; ++n)
        T += sh.a.T[n] * (sel3v(n % 3, LA) * sel3v((n / 3) % 3, LB) * sel3v(n / 9, LC));
    }
    const double rho = 1 - ph.beta * (T - ph.T_ref);
    double grav[3];
    if (ph.cuboid) {
      grav[0] = grav[1] = 0;
      grav[2] = -ph.g;
    } else {
      const double* x = &sh.a.geo.xq[3 * q];
      const double r = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
      const double den = r > 1 ? r : sqrt(r);
#pragma unroll
      for (int d = 0; d < 3; ++d) grav[d] = -ph.g * x[d] / den;
    }
    const double cxu[3] = {-ph.coriolis_z * u[1], ph.coriolis_z * u[0], 0.0};
    const double w = sh.a.geo.JxW[q];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double adv = u[0] * G[c][0] + u[1] * G[c][1] + u[2] * G[c][2];
      sh.a.F[3 * q + c] = (u[c] + ph.dt * rho * (ph.grav_scale * grav[c]) - ph.dt * adv -
                           ph.dt * (2 * cxu[c])) * w;
    }
  }
  wsync();
  // ---- B^T rows (an, v) for v in [4 h, 4 h + 4) on lanes an + 32 h; lanes
  // 0-26 also the node-diagonal sums (|K_ii| rule), lanes 32-58 the rhs node
  const int an = lane & 31, h = lane >> 5;
  const bool row_lane = an < 27;
  double bt[4][3];
  double kii[3] = {0, 0, 0};
  double fa[3] = {0, 0, 0};
  // the constrained-row diagonal (|K_ii| or the cell average) only matters on
  // cells with a constrained node (boundary layers): skip the sums elsewhere
  const bool cell_con =
      want_cdiag && __any(lane < 27 && out.cidx[sh.node[lane < 27 ? lane : 0]] >= 0);
  const bool do_diag = cell_con && h == 0;
  if (row_lane) {
#pragma unroll
    for (int vv = 0; vv < 4; ++vv) bt[vv][0] = bt[vv][1] = bt[vv][2] = 0;
    double msum = 0, g2[3] = {0, 0, 0};
    // this lane's node: its 1D factors at the 3 Gauss points per direction; the
    // point loop indexes them at compile time
    const int na = an % 3, nb = (an / 3) % 3, nc = an / 9;
    double La[3], Da1[3], Lb[3], Db1[3], Lc[3], Dc1[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double x = sel_gauss(i);
      La[i] = ce_l2(na, x);
      Da1[i] = ce_dl2(na, x);
      Lb[i] = ce_l2(nb, x);
      Db1[i] = ce_dl2(nb, x);
      Lc[i] = ce_l2(nc, x);
      Dc1[i] = ce_dl2(nc, x);
    }
#pragma unroll 1
    for (int q2 = 0; q2 < 3; ++q2) {
      const double lc = sel3v(q2, Lc), dc = sel3v(q2, Dc1);
#pragma unroll 1
      for (int q1 = 0; q1 < 3; ++q1) {
        const double lb = sel3v(q1, Lb), db = sel3v(q1, Db1);
#pragma unroll
        for (int q0 = 0; q0 < 3; ++q0) {
          const int q = q0 + 3 * q1 + 9 * q2;
          const double s = La[q0] * lb * lc;
          const double r0 = Da1[q0] * lb * lc;
          const double r1 = La[q0] * db * lc;
          const double r2 = La[q0] * lb * dc;
          const double* Ji = &sh.a.geo.Ji[9 * q];
          double Da[3];
#pragma unroll
          for (int d = 0; d < 3; ++d) Da[d] = r0 * Ji[d] + r1 * Ji[3 + d] + r2 * Ji[6 + d];
          const double w = sh.a.geo.JxW[q];
          if (want_B) {
#pragma unroll
            for (int vv = 0; vv < 4; ++vv) {
              const double wp = w * cRef.S1[8 * q + 4 * h + vv];
              bt[vv][0] -= Da[0] * wp;
              bt[vv][1] -= Da[1] * wp;
              bt[vv][2] -= Da[2] * wp;
            }
          }
          if (do_diag) {
            msum += w * s * s;
            g2[0] += w * Da[0] * Da[0];
            g2[1] += w * Da[1] * Da[1];
            g2[2] += w * Da[2] * Da[2];
          }
          if (want_rhs && h == 1) {
            fa[0] += s * sh.a.F[3 * q];
            fa[1] += s * sh.a.F[3 * q + 1];
            fa[2] += s * sh.a.F[3 * q + 2];
          }
        }
      }
    }
    if (do_diag) {
      const double L = g2[0] + g2[1] + g2[2];
#pragma unroll
      for (int c = 0; c < 3; ++c) kii[c] = msum + ph.nu_sys * L + ph.nu_sys * g2[c];
      sh.a.diag[an] = fabs(kii[0]) + fabs(kii[1]) + fabs(kii[2]);
    }
    const int nd = sh.node[an];
    double Ca[3][3];
    condensation(cd.vcon[nd], Ca);
    if (want_B) {
#pragma unroll
      for (int vv = 0; vv < 4; ++vv) {
        const double b0 = bt[vv][0], b1 = bt[vv][1], b2 = bt[vv][2];
#pragma unroll
        for (int j = 0; j < 3; ++j) bt[vv][j] = Ca[0][j] * b0 + Ca[1][j] * b1 + Ca[2][j] * b2;
      }
    }
    if (want_rhs && h == 1) {
      double* dst = out.rhs + 3 * size_t(nd);
#pragma unroll
      for (int j = 0; j < 3; ++j) dst[j] += Ca[0][j] * fa[0] + Ca[1][j] * fa[1] + Ca[2][j] * fa[2];
    }
  }
  wsync();
  if (do_diag && row_lane) {
    const int nd = sh.node[an];
    const int ci = out.cidx[nd];
    if (ci >= 0) {
      const NodeConstraint nc = cd.vcon[nd];
      double avg = 0;
      for (int m = 0; m < 27; ++m) avg += sh.a.diag[m];
      avg /= 89.0;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        if (nc.type == 1 || nc.type == 3 || c == nc.k) {
          const double d = fabs(kii[c]);
          out.cdiag[3 * size_t(ci) + c] += d != 0.0 ? d : avg;
        }
    }
  }
  if (!want_B || DCP_OPW_NOSCATTER) return;
  wsync();  // every lane is past its reads of the phase tables: stage over them
  if (row_lane) {
#pragma unroll
    for (int vv = 0; vv < 4; ++vv)
#pragma unroll
      for (int j = 0; j < 3; ++j) sh.stage[3 * (8 * an + 4 * h + vv) + j] = bt[vv][j];
  }
  wsync();
  // ---- the staged rows into B^T (and B): first touch stores, else add;
  // DCP_OPW_BATCH (14) read-modify-writes in flight per lane: the B^T rows of
  // one GPU in one round (r=5: 7 per lane 2.49 ms, 14 per lane and 4 waves
  // per workgroup 2.21 ms; profiles/r03y_*)
  constexpr int kB = DCP_OPW_BATCH, kRounds = (2 * 648 + 64 * kB - 1) / (64 * kB);
  const int e_end = scatter_B ? 2 * 648 : 648;
#pragma unroll 1
  for (int rd = 0; rd < kRounds; ++rd) {
    double old[kB], val[kB];
    double* dst[kB];
#pragma unroll
    for (int j = 0; j < kB; ++j) {
      const int e = lane + 64 * (kB * rd + j);
      old[j] = 0.0;
      val[j] = 0.0;
      dst[j] = nullptr;
      if (e < e_end) {
        int p;
        if (e < 648) {
          const int r = e / 3, c = e - 3 * r;
          val[j] = sh.stage[3 * r + c];
          p = sh.pos[r];
          dst[j] = out.Bt + 3 * size_t(p >= 0 ? p : ~p) + c;
        } else {
          const int r = (e - 648) / 3, c = e - 648 - 3 * r;
          const int pv = r / 27, a = r - 27 * pv;  // B row (pv, a) = B^T row (a, pv)
          val[j] = sh.stage[3 * (8 * a + pv) + c];
          p = sh.pos[216 + r];
          dst[j] = out.B + 3 * size_t(p >= 0 ? p : ~p) + c;
        }
        if (p >= 0) old[j] = *dst[j];
      }
    }
#pragma unroll
    for (int j = 0; j < kB; ++j)
      if (dst[j]) *dst[j] = old[j] + val[j];
  }
}

// ---------------------------------------------------------------------------
// The operator form without B^T (B^T by row tasks, k_bt_tasks): what stays per
// cell is the rhs (local_assemble_nse_system's f_i, boussinesq_model.tpp:
// 655-669, condensed and added into nse_rhs) and the constrained-row diagonal.
// Half a wave per cell, two cells per wave (the rhs phases use 27 lanes):
// lanes 0-26 of the half hold Gauss points (state, geometry, integrand), then
// nodes (test-function sums, on cells with a constrained node also the
// |K_ii| sums of k_nse_operator_wave). Every sum in k_nse_operator_wave's
// order: the rhs and the diagonal are bitwise that kernel's.
struct RhsCellSmem {
  double U[81], T[27];
  Geo geo;
  double F[81];
  double diag[27];
  int node[27];
};
constexpr int kRhsCellsPerGroup = 8;  // 4 waves x 2 cells

__global__ __launch_bounds__(256) void k_nse_rhs_halfwave(
    CellData cd, const int32_t* __restrict__ cells, int n_cells, const double* __restrict__ u_old,
    const double* __restrict__ T_old, PhysicsDev ph, NseOut out) {
  __shared__ RhsCellSmem smem[kRhsCellsPerGroup];
  const int half = threadIdx.x >> 5, hl = threadIdx.x & 31;
  const int k = int(blockIdx.x) * kRhsCellsPerGroup + half;
  const bool live = k < n_cells;
  RhsCellSmem& sh = smem[half];
  const int cell = live ? cells[k] : 0;
  const bool want_cdiag = out.cdiag != nullptr;
  // ---- state and geometry (lanes 0-26: nodes / points)
  bool con = false;
  // without the rhs (the constrained diagonals only) the state is not read
  const bool want_rhs = out.rhs != nullptr;
  if (live && hl < 27) {
    const int nd = cd.cell_q2[27 * size_t(cell) + hl];
    sh.node[hl] = nd;
    if (want_rhs) {
#pragma unroll
      for (int d = 0; d < 3; ++d) sh.U[3 * hl + d] = u_old[3 * size_t(nd) + d];
      if (cd.tdpc == 27) sh.T[hl] = T_old[cd.cell_T[27 * size_t(cell) + hl]];
    }
    sep_geometry(cd, cell, sh.geo, hl);
    con = want_cdiag && out.cidx[nd] >= 0;
  }
  if (want_rhs && live && cd.tdpc == 8 && hl < 8) sh.T[hl] = T_old[cd.cell_T[8 * size_t(cell) + hl]];
  // this half's cell has a constrained node
  const unsigned long long bal = __ballot(con);
  const bool cell_con = ((bal >> (32 * ((threadIdx.x >> 5) & 1))) & 0xffffffffull) != 0;
  wsync();
  // ---- rhs integrand per Gauss point (k_nse_operator_wave's formulas)
  if (want_rhs && live && hl < 27) {
    const int q = hl;
    const double xa = sel_gauss(q % 3), xb = sel_gauss((q / 3) % 3), xc = sel_gauss(q / 9);
    const double* Ji = &sh.geo.Ji[9 * q];
    double LA[3], DA[3], LB[3], DB[3], LC[3], DC[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      LA[i] = ce_l2(i, xa);
      DA[i] = ce_dl2(i, xa);
      LB[i] = ce_l2(i, xb);
      DB[i] = ce_dl2(i, xb);
      LC[i] = ce_l2(i, xc);
      DC[i] = ce_dl2(i, xc);
    }
    double u[3] = {0, 0, 0}, G[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
#pragma unroll 1
    for (int nc = 0; nc < 3; ++nc) {
      const double lc = sel3v(nc, LC), dc = sel3v(nc, DC);
#pragma unroll 1
      for (int nb = 0; nb < 3; ++nb) {
        const double lb = sel3v(nb, LB), db = sel3v(nb, DB);
#pragma unroll
        for (int na = 0; na < 3; ++na) {
          const int n = na + 3 * nb + 9 * nc;
          const double s = LA[na] * lb * lc;
          const double r0 = DA[na] * lb * lc;
          const double r1 = LA[na] * db * lc;
          const double r2 = LA[na] * lb * dc;
          double Dn[3];
#pragma unroll
          for (int d = 0; d < 3; ++d) Dn[d] = r0 * Ji[d] + r1 * Ji[3 + d] + r2 * Ji[6 + d];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const double un = sh.U[3 * n + c];
            u[c] += un * s;
            G[c][0] += un * Dn[0];
            G[c][1] += un * Dn[1];
            G[c][2] += un * Dn[2];
          }
        }
      }
    }
    double T = 0;
    if (cd.tdpc == 8) {
#pragma unroll
      for (int v = 0; v < 8; ++v) T += sh.T[v] * cRef.S1[8 * q + v];
    } else {
      for (int n = 0; n < 27; ++n)
        T += sh.T[n] * (sel3v(n % 3, LA) * sel3v((n / 3) % 3, LB) * sel3v(n / 9, LC));
    }
    const double rho = 1 - ph.beta * (T - ph.T_ref);
    double grav[3];
    if (ph.cuboid) {
      grav[0] = grav[1] = 0;
      grav[2] = -ph.g;
    } else {
      const double* x = &sh.geo.xq[3 * q];
      const double r = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
      const double den = r > 1 ? r : sqrt(r);
#pragma unroll
      for (int d = 0; d < 3; ++d) grav[d] = -ph.g * x[d] / den;
    }
    const double cxu[3] = {-ph.coriolis_z * u[1], ph.coriolis_z * u[0], 0.0};
    const double w = sh.geo.JxW[q];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double adv = u[0] * G[c][0] + u[1] * G[c][1] + u[2] * G[c][2];
      sh.F[3 * q + c] = (u[c] + ph.dt * rho * (ph.grav_scale * grav[c]) - ph.dt * adv -
                         ph.dt * (2 * cxu[c])) * w;
    }
  }
  wsync();
  // ---- per node: the rhs test-function sums (and on constrained cells the
  // node-diagonal sums of the |K_ii| rule)
  const int an = hl;
  double kii[3] = {0, 0, 0};
  if (live && an < 27) {
    double fa[3] = {0, 0, 0};
    double msum = 0, g2[3] = {0, 0, 0};
    const int na = an % 3, nb = (an / 3) % 3, nc = an / 9;
    double La[3], Da1[3], Lb[3], Db1[3], Lc[3], Dc1[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double x = sel_gauss(i);
      La[i] = ce_l2(na, x);
      Da1[i] = ce_dl2(na, x);
      Lb[i] = ce_l2(nb, x);
      Db1[i] = ce_dl2(nb, x);
      Lc[i] = ce_l2(nc, x);
      Dc1[i] = ce_dl2(nc, x);
    }
#pragma unroll 1
    for (int q2 = 0; q2 < 3; ++q2) {
      const double lc = sel3v(q2, Lc), dc = sel3v(q2, Dc1);
#pragma unroll 1
      for (int q1 = 0; q1 < 3; ++q1) {
        const double lb = sel3v(q1, Lb), db = sel3v(q1, Db1);
#pragma unroll
        for (int q0 = 0; q0 < 3; ++q0) {
          const int q = q0 + 3 * q1 + 9 * q2;
          const double s = La[q0] * lb * lc;
          if (want_rhs) {
            fa[0] += s * sh.F[3 * q];
            fa[1] += s * sh.F[3 * q + 1];
            fa[2] += s * sh.F[3 * q + 2];
          }
          if (cell_con) {
            const double r0 = Da1[q0] * lb * lc;
            const double r1 = La[q0] * db * lc;
            const double r2 = La[q0] * lb * dc;
            const double* Ji = &sh.geo.Ji[9 * q];
            double Da[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) Da[d] = r0 * Ji[d] + r1 * Ji[3 + d] + r2 * Ji[6 + d];
            const double w = sh.geo.JxW[q];
            msum += w * s * s;
            g2[0] += w * Da[0] * Da[0];
            g2[1] += w * Da[1] * Da[1];
            g2[2] += w * Da[2] * Da[2];
          }
        }
      }
    }
    if (cell_con) {
      const double L = g2[0] + g2[1] + g2[2];
#pragma unroll
      for (int c = 0; c < 3; ++c) kii[c] = msum + ph.nu_sys * L + ph.nu_sys * g2[c];
      sh.diag[an] = fabs(kii[0]) + fabs(kii[1]) + fabs(kii[2]);
    }
    const int nd = sh.node[an];
    double Ca[3][3];
    condensation(cd.vcon[nd], Ca);
    if (out.rhs) {
      double* dst = out.rhs + 3 * size_t(nd);
#pragma unroll
      for (int j = 0; j < 3; ++j) dst[j] += Ca[0][j] * fa[0] + Ca[1][j] * fa[1] + Ca[2][j] * fa[2];
    }
  }
  if (!cell_con) return;
  wsync();
  if (live && an < 27) {
    const int nd = sh.node[an];
    const int ci = out.cidx[nd];
    if (ci >= 0) {
      const NodeConstraint nc = cd.vcon[nd];
      double avg = 0;
      for (int m = 0; m < 27; ++m) avg += sh.diag[m];
      avg /= 89.0;
      double* slot = out.cbuf ? out.cbuf + 3 * size_t(out.cslot[27 * size_t(k) + an]) : nullptr;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const bool on = nc.type == 1 || nc.type == 3 || c == nc.k;
        const double d = fabs(kii[c]);
        if (slot)
          slot[c] = on ? (d != 0.0 ? d : avg) : 0.0;
        else if (on)
          out.cdiag[3 * size_t(ci) + c] += d != 0.0 ? d : avg;
      }
    }
  }
}

// the constrained-row diagonals from their per-cell slots, in slot (= the
// cells' colour) order: the sums the per-colour additions formed
__global__ void k_con_gather(int n_con, const int32_t* __restrict__ cptr,
                             const double* __restrict__ cbuf, double* __restrict__ cdiag) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_con) return;
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int k = cptr[i]; k < cptr[i + 1]; ++k) {
    s0 += cbuf[3 * size_t(k)];
    s1 += cbuf[3 * size_t(k) + 1];
    s2 += cbuf[3 * size_t(k) + 2];
  }
  cdiag[3 * size_t(i)] = s0;
  cdiag[3 * size_t(i) + 1] = s1;
  cdiag[3 * size_t(i) + 2] = s2;
}

// ---------------------------------------------------------------------------
// B^T by rows on the radially separable shell (copy_local_to_global_nse_system
// of the B^T block, boussinesq_model.tpp:626-637 / 677-687, restated as a
// gather). The entry of velocity node n = (a, b, c) of cell K and vertex
// p = (i, j, k) of K is -sum_q JxW psi_p d_d phi_n, and with the separable map
// (J^-1 rows m0 / R, m1 / R, m2 / R', JxW = R^2 R' D2 w; sep_geometry) the
// 27-point sum factors into a 9-point column sum and a 3-point layer sum:
//   B^T = -(P01[a b i j][d] Q01[c][k] + P2[a b i j][d] Q2[c][k])
//   P01 = sum_xy w w psi_i psi_j D2 (m0[d] l'_a l_b + m1[d] l_a l'_b)
//   P2  = sum_xy w w psi_i psi_j D2 m2[d] l_a l_b
//   Q01 = sum_z w R^2 R' / R l_c psi_k,   Q2 = sum_z w R^2 R' / R' l'_c psi_k.
// k_bt_coltab forms P per column (216 values) from the column table once at
// upload (mesh geometry). k_bt_tasks then writes B^T by tasks: a task is a run of consecutive
// velocity node rows with at most 8 (row, cell) slots and 64 row entries in
// all, so the task's entries are one contiguous piece of the B^T values. Lane
// (slot k, vertex v) evaluates that cell's contribution and knows (from the
// slot record built at upload) which task entry it belongs to; lane j sums
// entry j over its contributions in slot order (the row's cells in colour
// order), condenses it with its row's constraint (C_a^T b: linear, so the same
// as condensing each cell's part) and stores it -- every entry written once,
// the task's piece coalesced, no read-modify-write, no zero fill, no colouring.
#ifndef DCP_BT_WAVES
#define DCP_BT_WAVES 4
#endif
constexpr int kBtRowWaves = DCP_BT_WAVES;
// B^T entry stores: 0 plain, 1 / 2 through LDS in 512-byte runs (2:
// nontemporal), 3 nontemporal from the entry lanes (default: B^T is 584 MB at
// r=5, larger than the Infinity Cache, and is next read by the S formation;
// 0.553 -> 0.525 ms per assembly, bitwise, profiles/r04y_bt_store_variants.json)
#ifndef DCP_BT_STORE
#define DCP_BT_STORE 3
#endif
constexpr int kBtColEntries = 216;  // [P01 | P2][a][b][i][j][d]
// DCP_BT_NTLOAD (default on): the task headers and slot records (read once
// per assembly) as nontemporal loads, keeping the caches for the tables
#ifndef DCP_BT_NTLOAD
#define DCP_BT_NTLOAD 1
#endif
__device__ __forceinline__ int4 bt_ld4(const int4* p) {
#if DCP_BT_NTLOAD
  typedef int v4i __attribute__((ext_vector_type(4)));
  const v4i x = __builtin_nontemporal_load(reinterpret_cast<const v4i*>(p));
  return make_int4(x.x, x.y, x.z, x.w);
#else
  return *p;
#endif
}

__global__ __launch_bounds__(kBtColEntries) void k_bt_coltab(const double* __restrict__ colgeo,
                                                             double* __restrict__ P) {
  const int col = blockIdx.x, t = threadIdx.x;
  const int which = t / 108, r = t % 108;
  const int a = r / 36, b = (r / 12) % 3, i = (r / 6) % 2, j = (r / 3) % 2, d = r % 3;
  double s = 0.0;
#pragma unroll
  for (int q1 = 0; q1 < 3; ++q1)
#pragma unroll
    for (int q0 = 0; q0 < 3; ++q0) {
      const double* m = colgeo + 90 * size_t(col) + 10 * (q0 + 3 * q1);
      const double w = cW[q0] * cW[q1] * m[9] * cL1[i][q0] * cL1[j][q1];
      if (which == 0)
        s += w * (m[d] * cdL2[a][q0] * cL2[b][q1] + m[3 + d] * cL2[a][q0] * cdL2[b][q1]);
      else
        s += w * (m[6 + d] * cL2[a][q0] * cL2[b][q1]);
    }
  P[kBtColEntries * size_t(col) + t] = s;
}

// the layer factors Q01, Q2 of (node layer c, vertex layer k) for layer lay:
// [lay][c][k][Q01 | Q2], formed once at upload (k_bt_laytab)
constexpr int kBtLayEntries = 12;
__device__ inline double bt_layer_factor(const double* __restrict__ lg, int c, int k, bool d2) {
  double q = 0.0;
#pragma unroll
  for (int z = 0; z < 3; ++z) {
    const double wz = cW[z] * lg[3 * z + 2] * cL1[k][z];
    q += d2 ? wz * lg[3 * z + 1] * cdL2[c][z] : wz * lg[3 * z] * cL2[c][z];
  }
  return q;
}
__global__ __launch_bounds__(kBtLayEntries) void k_bt_laytab(const double* __restrict__ laygeo,
                                                             double* __restrict__ Q) {
  const int lay = blockIdx.x, t = threadIdx.x;
  Q[kBtLayEntries * size_t(lay) + t] =
      bt_layer_factor(laygeo + 9 * size_t(lay), t / 4, (t / 2) % 2, t % 2 == 1);
}

// the (node lex, vertex v) contribution of a cell in column-table entry col
// and layer lay, components d = 0..2
__device__ inline void bt_entry(const double* __restrict__ P, const double* __restrict__ Q, int col,
                                int lay, int lex, int v, double out[3]) {
  const int a = lex % 3, b = (lex / 3) % 3, c = lex / 9;
  const int i = v & 1, j = (v >> 1) & 1, k = v >> 2;
  const double* qq = Q + kBtLayEntries * size_t(lay) + 4 * c + 2 * k;
  const double q01 = qq[0], q2 = qq[1];
  const double* pp = P + kBtColEntries * size_t(col) + 6 * (2 * (3 * a + b) + i) + 3 * j;
#pragma unroll
  for (int d = 0; d < 3; ++d) out[d] = -(pp[d] * q01 + pp[108 + d] * q2);
}

// task header: {first B^T entry, first row, slots | entries << 8, first slot
// record (= SL task)}; slot record: {column-table entry, layer << 16 | lex <<
// 8 | row in task, the 8 vertices' task entries as 6-bit fields (lo, hi
// words)}. SL slots per task (8 or 16, DCP_BT_SLOTS at upload), at most 64
// entries: lane (k, v) evaluates slot k (and k + 8) for vertex v, so a task of
// 16 slots fills the 64 entry lanes (~32 entries per 8-slot task at r=5) and
// one wave's chain of dependent loads (header / record -> tables -> row
// constraint) serves twice the entries. Several tasks per wave one after the
// other (the next header / record prefetched) measured 10 / 17 % slower for 2
// / 4 (profiles/r04l_bt_tpw_variants.json); loading the row constraints in
// phase 1 into LDS with a packed destination scan, 20 % slower (r04m).
// DCP_BT_PROBE (timing probes only, wrong B^T): 1 no entry stores, 2 the
// column / layer tables replaced by register values, 3 no row-constraint
// loads, 4 = 2 + 3
#ifndef DCP_BT_PROBE
#define DCP_BT_PROBE 0
#endif
// mode (DCP_BT_MODE, default 3): bit 0: the doubles of the task's first and
// last 128-byte line stored plainly (the rest nontemporal), so the two tasks
// sharing a line meet in one L2 instead of each writing the partial line to
// HBM; bit 1: each XCD a contiguous range of workgroups (neighbouring tasks,
// hence the shared lines, on the same XCD)
template <int SL, int EL>
__global__ __launch_bounds__(64 * kBtRowWaves) void k_bt_tasks(
    CellData cd, int n_tasks, const int4* __restrict__ hdr, const int4* __restrict__ rec,
    const double* __restrict__ P, const double* __restrict__ Q, double* __restrict__ Bt,
    int mode) {
  constexpr int R = SL / 8;             // slot records per lane
  constexpr int NE = 64 * EL;           // task entries (EL per lane)
  constexpr int FB = EL == 1 ? 6 : 7;   // bits per destination field of a record
  __shared__ double vals[kBtRowWaves][R * 64 * 3];
  // per (slot, task entry) the slot's vertex contributing to that entry, or
  // 0xff: the entry lanes read their contributions slot by slot (no scan over
  // every (slot, vertex) pair)
  __shared__ uint8_t vof[kBtRowWaves][SL][NE];
  __shared__ int rowl[kBtRowWaves][SL];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int blk = (mode & 2) ? xcd_block(int(blockIdx.x), int(gridDim.x)) : int(blockIdx.x);
  const int task = blk * kBtRowWaves + wave;
  if (task >= n_tasks) return;
  const int k = lane >> 3, v = lane & 7;
  // records at SL task + slot (unused slots zero): header and record loads
  // issue together
  const int4 h = bt_ld4(hdr + task);
  int4 r[R];
#pragma unroll
  for (int i = 0; i < R; ++i) r[i] = bt_ld4(rec + SL * size_t(task) + 8 * i + k);
  const int ns = h.z & 255, ne = h.z >> 8;
#if DCP_BT_STORE && DCP_BT_STORE != 3
  double out[EL][3];
#endif
  unsigned long long* vw = reinterpret_cast<unsigned long long*>(&vof[wave][0][0]);
#pragma unroll
  for (int i = 0; i < SL * NE / 8 / 64; ++i) vw[64 * i + lane] = ~0ull;
  wsync();
#ifndef DCP_BT_UNCOND
#define DCP_BT_UNCOND 1
#endif
  // DCP_BT_UNCOND (default): every slot's table loads issued up front, without
  // the per-slot branch (an unused slot's zero record reads column 0 / layer
  // 0), so the R slots' table latencies overlap: k_bt_tasks<16,1> 313.6 ->
  // 306.0 us under the tracer, bitwise (profiles/r05/r05ad_bt_uncond_variants.log)
  double evu[R][3];
  if (DCP_BT_UNCOND && !(DCP_BT_PROBE == 2 || DCP_BT_PROBE == 4)) {
#pragma unroll
    for (int i = 0; i < R; ++i) bt_entry(P, Q, r[i].x, r[i].y >> 16, (r[i].y >> 8) & 31, v, evu[i]);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int sl = 8 * i + k, e = 64 * i + lane;  // e = 8 slot + v
    if (sl < ns) {
      const unsigned long long dm =
          (unsigned long long)(unsigned)r[i].z | ((unsigned long long)(unsigned)r[i].w << 32);
      vof[wave][sl][int((dm >> (FB * v)) & (NE - 1))] = uint8_t(v);
      double ev[3];
      if (DCP_BT_PROBE == 2 || DCP_BT_PROBE == 4) {
        ev[0] = 1e-3 * r[i].x;
        ev[1] = 1e-3 * (r[i].y >> 16);
        ev[2] = 1e-3 * v;
      } else if (DCP_BT_UNCOND) {
        ev[0] = evu[i][0];
        ev[1] = evu[i][1];
        ev[2] = evu[i][2];
      } else {
        bt_entry(P, Q, r[i].x, r[i].y >> 16, (r[i].y >> 8) & 31, v, ev);
      }
      vals[wave][3 * e] = ev[0];
      vals[wave][3 * e + 1] = ev[1];
      vals[wave][3 * e + 2] = ev[2];
      if (v == 0) rowl[wave][sl] = r[i].y & 0x80ff;  // row in task | constrained flag
    }
  }
  wsync();
#pragma unroll
  for (int q = 0; q < EL; ++q) {
    const int j = lane + 64 * q;
    if (j >= ne) break;
    // entry j: its contributions in slot order (the row's cells in colour
    // order), the same order as a scan over (slot, vertex)
    double acc[3] = {0.0, 0.0, 0.0};
    int rl = 0;
    for (int sl = 0; sl < ns; ++sl) {
      const int vv = vof[wave][sl][j];
      if (vv != 0xff) {
        const int e = 8 * sl + vv;
        acc[0] += vals[wave][3 * e];
        acc[1] += vals[wave][3 * e + 1];
        acc[2] += vals[wave][3 * e + 2];
        rl = rowl[wave][sl];
      }
    }
    double Ca[3][3];
    // unconstrained rows: identity (the same products as condensation() forms)
    const NodeConstraint nc = ((rl & 0x8000) && DCP_BT_PROBE != 3 && DCP_BT_PROBE != 4)
                                  ? cd.vcon[h.y + (rl & 255)]
                                  : NodeConstraint{{0.0, 0.0, 0.0}, 0, 0};
    condensation(nc, Ca);
#if DCP_BT_STORE == 3
    double* dst = Bt + 3 * size_t(h.x + j);
    if (DCP_BT_PROBE == 1) {
      if (acc[0] == 12345.0) dst[0] = Ca[0][0];  // keeps the work alive
      continue;
    }
    if (mode & 1) {
      // the task's piece spans doubles [3 h.x, 3 (h.x + ne)); its first and
      // last 128-byte lines may be shared with the neighbouring tasks
      const size_t first_line = (3 * size_t(h.x)) >> 4;
      const size_t last_line = (3 * size_t(h.x + ne) - 1) >> 4;
#pragma unroll
      for (int jj = 0; jj < 3; ++jj) {
        const double val = Ca[0][jj] * acc[0] + Ca[1][jj] * acc[1] + Ca[2][jj] * acc[2];
        const size_t line = (3 * size_t(h.x + j) + jj) >> 4;
        if (line == first_line || line == last_line) dst[jj] = val;
        else __builtin_nontemporal_store(val, dst + jj);
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < 3; ++jj)
        __builtin_nontemporal_store(Ca[0][jj] * acc[0] + Ca[1][jj] * acc[1] + Ca[2][jj] * acc[2],
                                    dst + jj);
    }
#elif DCP_BT_STORE
    out[q][0] = Ca[0][0] * acc[0] + Ca[1][0] * acc[1] + Ca[2][0] * acc[2];
    out[q][1] = Ca[0][1] * acc[0] + Ca[1][1] * acc[1] + Ca[2][1] * acc[2];
    out[q][2] = Ca[0][2] * acc[0] + Ca[1][2] * acc[1] + Ca[2][2] * acc[2];
#else
    double* dst = Bt + 3 * size_t(h.x + j);
#pragma unroll
    for (int jj = 0; jj < 3; ++jj)
      dst[jj] = Ca[0][jj] * acc[0] + Ca[1][jj] * acc[1] + Ca[2][jj] * acc[2];
#endif
  }
#if DCP_BT_STORE && DCP_BT_STORE != 3
  // the task's piece through LDS (over vals, every lane past its reads): each
  // store instruction then covers 512 consecutive bytes instead of every
  // third double of 1536
  wsync();
#pragma unroll
  for (int q = 0; q < EL; ++q) {
    const int j = lane + 64 * q;
    if (j < ne) {
      vals[wave][3 * j] = out[q][0];
      vals[wave][3 * j + 1] = out[q][1];
      vals[wave][3 * j + 2] = out[q][2];
    }
  }
  wsync();
  double* dst = Bt + 3 * size_t(h.x);
#pragma unroll
  for (int q = 0; q < 3 * EL; ++q) {
    const int idx = 64 * q + lane;
    if (idx < 3 * ne) {
#if DCP_BT_STORE == 2
      __builtin_nontemporal_store(vals[wave][idx], dst + idx);
#else
      dst[idx] = vals[wave][idx];
#endif
    }
  }
#endif
}

// ---------------------------------------------------------------------------
// The constrained-row diagonals in Kronecker form (one GPU, layered shell).
// A constrained node's diagonal sums, over the cells holding it, the cell's
// |K_ii| per component (local_assemble_nse_system :626-637 restricted to the
// diagonal, the value AffineConstraints puts on a constrained row):
//   K_ii[d] = M + nu (g[0] + g[1] + g[2]) + nu g[d],  nu = dt / Re,
//   M = sum_q JxW phi^2,  g[d] = sum_q JxW (d_d phi)^2.
// With J^-1 rows m0 / R, m1 / R, m2 / R', JxW = R^2 R' D2 w and phi =
// psi_ab(x, y) chi_c(z), d_d phi = (A_d chi_c) / R + (B_d chi'_c) / R' with
// A_d = psi'_a psi_b m0[d] + psi_a psi'_b m1[d], B_d = psi_a psi_b m2[d], so
// every term is a lateral 9-point sum times a radial 3-point sum:
//   M = LM RM,  g[d] = L1[d] R1 + L2[d] R2 + L3[d] R3.
// k_cdk_lateral / k_cdk_radial form the tables at upload (mesh geometry, like
// the B^T column / layer factors); per assembly k_cdk_diag sums a node's cells
// in the slot order of k_nse_rhs_halfwave + k_con_gather, which it replaces.
// K_ii > 0 (the mass term), so the |.| and the zero-diagonal average rule of
// the cell kernel never change a value here.
__global__ void k_cdk_lateral(const double* __restrict__ colgeo, int n_cols, double* __restrict__ L) {
  const int i = int(blockIdx.x) * blockDim.x + int(threadIdx.x);
  if (i >= 9 * n_cols) return;
  const int col = i / 9, ab = i - 9 * col, na = ab % 3, nb = ab / 3;
  double lm = 0, l1[3] = {0, 0, 0}, l2[3] = {0, 0, 0}, l3[3] = {0, 0, 0};
  for (int q1 = 0; q1 < 3; ++q1)
    for (int q0 = 0; q0 < 3; ++q0) {
      const double* m = colgeo + 90 * size_t(col) + 10 * (q0 + 3 * q1);
      const double xa = sel_gauss(q0), xb = sel_gauss(q1);
      const double la = ce_l2(na, xa), lb = ce_l2(nb, xb), da = ce_dl2(na, xa), db = ce_dl2(nb, xb);
      const double w = cW[q0] * cW[q1] * m[9];
      lm += w * (la * lb) * (la * lb);
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const double A = da * lb * m[d] + la * db * m[3 + d], B = la * lb * m[6 + d];
        l1[d] += w * A * A;
        l2[d] += 2 * w * A * B;
        l3[d] += w * B * B;
      }
    }
  double* o = L + 10 * size_t(i);
  o[0] = lm;
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    o[1 + d] = l1[d];
    o[4 + d] = l2[d];
    o[7 + d] = l3[d];
  }
}

__global__ void k_cdk_radial(const double* __restrict__ laygeo, int n_layers, double* __restrict__ R) {
  const int i = int(blockIdx.x) * blockDim.x + int(threadIdx.x);
  if (i >= 3 * n_layers) return;
  const int lay = i / 3, c = i - 3 * lay;
  double rm = 0, r1 = 0, r2 = 0, r3 = 0;
  for (int q2 = 0; q2 < 3; ++q2) {
    const double* lg = laygeo + 9 * size_t(lay) + 3 * q2;
    const double x = sel_gauss(q2), lc = ce_l2(c, x), dc = ce_dl2(c, x);
    const double W = cW[q2] * lg[2], iR = lg[0], iRp = lg[1];
    rm += W * lc * lc;
    r1 += W * (iR * lc) * (iR * lc);
    r2 += W * (iR * lc) * (iRp * dc);
    r3 += W * (iRp * dc) * (iRp * dc);
  }
  double* o = R + 4 * size_t(i);
  o[0] = rm;
  o[1] = r1;
  o[2] = r2;
  o[3] = r3;
}

__global__ void k_cdk_diag(int n_con, const int32_t* __restrict__ cptr, const int2* __restrict__ rec,
                           const int32_t* __restrict__ mask, const double* __restrict__ L,
                           const double* __restrict__ R, double nu, double* __restrict__ cdiag) {
  const int ci = int(blockIdx.x) * blockDim.x + int(threadIdx.x);
  if (ci >= n_con) return;
  double s[3] = {0, 0, 0};
  auto add = [&](int2 r, bool on) {  // r: lateral table (column id 9 + ab), radial (layer 3 + c)
    const double* l = L + 10 * size_t(r.x);
    const double* rr = R + 4 * size_t(r.y);
    double g[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) g[d] = l[1 + d] * rr[1] + l[4 + d] * rr[2] + l[7 + d] * rr[3];
    const double M = l[0] * rr[0], G = g[0] + g[1] + g[2];
#pragma unroll
    for (int d = 0; d < 3; ++d) s[d] += on ? fabs(M + nu * G + nu * g[d]) : 0.0;
  };
  // a surface node lies in at most 4 cells of its layer: those records loaded
  // together (clamped, unpredicated), a longer list (none on the shell) after
  const int k0 = cptr[ci], n = cptr[ci + 1] - k0;
  int2 r4[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) r4[j] = rec[k0 + min(j, n - 1)];
#pragma unroll
  for (int j = 0; j < 4; ++j) add(r4[j], j < n);
  for (int k = k0 + 4; k < k0 + n; ++k) add(rec[k], true);
  const int on = mask[ci];  // the row's constrained components (condensation)
#pragma unroll
  for (int d = 0; d < 3; ++d) cdiag[3 * size_t(ci) + d] = (on >> d) & 1 ? s[d] : 0.0;
}

}  // namespace

void cdk_tables(const double* colgeo, int n_cols, const double* laygeo, int n_layers, double* L,
                double* R, hipStream_t s) {
  hipLaunchKernelGGL(k_cdk_lateral, dim3((9 * n_cols + 255) / 256), dim3(256), 0, s, colgeo, n_cols, L);
  hipLaunchKernelGGL(k_cdk_radial, dim3((3 * n_layers + 255) / 256), dim3(256), 0, s, laygeo,
                     n_layers, R);
  DCP_HIP_CHECK(hipGetLastError());
}

void cdk_diag(int n_con, const int32_t* cptr, const int32_t* rec, const int32_t* mask,
              const double* L, const double* R, double nu, double* cdiag, hipStream_t s) {
  if (n_con <= 0) return;
  hipLaunchKernelGGL(k_cdk_diag, dim3((n_con + 255) / 256), dim3(256), 0, s, n_con, cptr,
                     reinterpret_cast<const int2*>(rec), mask, L, R, nu, cdiag);
  DCP_HIP_CHECK(hipGetLastError());
}

void con_gather(int n_con, const int32_t* cptr, const double* cbuf, double* cdiag, hipStream_t s) {
  if (n_con <= 0) return;
  hipLaunchKernelGGL(k_con_gather, dim3((n_con + 255) / 256), dim3(256), 0, s, n_con, cptr, cbuf,
                     cdiag);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_nse_operator(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                         const double* u_old, const double* T_old, const PhysicsDev& ph,
                         const NseOut& out, hipStream_t s) {
  if (n <= 0) return;
  // the wave-per-cell form on the separable shell (no periodic images there);
  // DCP_ASM_CELL_BLOCK=1 keeps the workgroup-per-cell kernel (timing comparisons)
  static const bool cell_block = [] {
    const char* e = std::getenv("DCP_ASM_CELL_BLOCK");
    return e && *e == '1';
  }();
  // small colour classes (the greedy colouring's tail: 6 of 14 classes hold
  // 2.3 % of the cells at refine 5) are latency-bound: there the
  // workgroup-per-cell kernel (4 waves on one cell) finishes sooner; both
  // kernels give bitwise the same matrix (DCP_ASM_SMALL_COLOUR: the threshold)
  static const int small_colour = [] {
    const char* e = std::getenv("DCP_ASM_SMALL_COLOUR");
    return e ? std::atoi(e) : kOpSmallColour;
  }();
  // without B^T / B (written by row tasks): the rhs-only half-wave kernel
  // (DCP_ASM_RHS_HALFWAVE=0 keeps the wave kernel, for comparisons)
  static const bool halfwave = [] {
    const char* e = std::getenv("DCP_ASM_RHS_HALFWAVE");
    return !(e && *e == '0');
  }();
  // The one-launch constrained-diagonal pass (out.cbuf: every (cell, node) into
  // its own slot, summed per node in colour order by con_gather) runs over the
  // cells of ALL colours at once; only the half-wave kernel writes slots, the
  // others add straight into con_diag and would race across colours. So that
  // pass always takes the half-wave kernel, whatever the timing switches say.
  if (out.cbuf) {
    if (!(cd.sep_col && !cd.cell_q2o && !cd.cell_po) || out.Bt || out.B || out.A)
      throw std::runtime_error("constrained-diagonal slots need the separable-shell rhs kernel");
    hipLaunchKernelGGL(k_nse_rhs_halfwave, dim3((n + kRhsCellsPerGroup - 1) / kRhsCellsPerGroup),
                       dim3(256), 0, s, cd, cells, n, u_old, T_old, ph, out);
    DCP_HIP_CHECK(hipGetLastError());
    return;
  }
  const bool sep = cd.sep_col && !cd.cell_q2o && !cd.cell_po && !cell_block;
  if (sep && halfwave && !out.Bt && !out.B && !out.A) {
    hipLaunchKernelGGL(k_nse_rhs_halfwave, dim3((n + kRhsCellsPerGroup - 1) / kRhsCellsPerGroup),
                       dim3(256), 0, s, cd, cells, n, u_old, T_old, ph, out);
  } else if (sep && n >= small_colour) {
    hipLaunchKernelGGL(k_nse_operator_wave, dim3((n + kOpWaves - 1) / kOpWaves), dim3(64 * kOpWaves),
                       0, s, cd, sm, cells, n, u_old, T_old, ph, out);
  } else {
    hipLaunchKernelGGL((k_nse_system<2, false>), dim3(n), dim3(kNseThreads), 0, s, cd, sm, cells, 0,
                       u_old, T_old, ph, out);
  }
  DCP_HIP_CHECK(hipGetLastError());
}

// B = (B^T)^T: block k of B is block tperm[k] of B^T (bitwise: both are summed
// over the same cells in the same colour order, and the local B and B^T
// entries are the same products)
__global__ void k_transpose_blocks3(long n, const int32_t* __restrict__ tperm,
                                    const double* __restrict__ src, double* __restrict__ dst) {
  const long i = blockIdx.x * long(blockDim.x) + threadIdx.x;  // one double of dst
  if (i >= 3 * n) return;
  const long k = i / 3;
  dst[i] = src[3 * long(tperm[k]) + (i - 3 * k)];
}

void transpose_blocks3(long n, const int32_t* tperm, const double* src, double* dst,
                       hipStream_t s) {
  if (n <= 0) return;
  const long threads = 3 * n;
  hipLaunchKernelGGL(k_transpose_blocks3, dim3(unsigned((threads + 255) / 256)), dim3(256), 0, s,
                     n, tperm, src, dst);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_nse_system_elements(const CellData& cd, int first, int n, const double* u_old,
                                const double* T_old, const PhysicsDev& ph, double* K, double* f,
                                hipStream_t s, bool mfma) {
  if (n <= 0) return;
  NseOut out{};
  out.elemK = K;
  out.elemF = f;
  if (mfma)
    hipLaunchKernelGGL((k_nse_system<1, true>), dim3(n), dim3(kNseThreads), 0, s, cd, ScatterMaps{},
                       nullptr, first, u_old, T_old, ph, out);
  else
    hipLaunchKernelGGL((k_nse_system<1, false>), dim3(n), dim3(kNseThreads), 0, s, cd, ScatterMaps{},
                       nullptr, first, u_old, T_old, ph, out);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_nse_precond_diag(const CellData& cd, const int32_t* cells, int n, const PhysicsDev& ph,
                             double* A_diag, double* Mp_diag, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_nse_precond_diag, dim3(n), dim3(64), 0, s, cd, cells, ph, A_diag, Mp_diag);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_T_matrix(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                     const PhysicsDev& ph, double* Tmass, double* Tstiff, const int32_t* posTs,
                     hipStream_t s) {
  if (n <= 0) return;
  if (cd.tdpc == 27) return launch_T2_matrix(cd, sm, cells, n, ph, Tmass, Tstiff, s);
  hipLaunchKernelGGL(k_T_matrix, dim3(n), dim3(64), 0, s, cd, sm, cells, ph, Tmass, Tstiff, posTs);
  DCP_HIP_CHECK(hipGetLastError());
}

void image_diagonal_blocks(int n, const int32_t* node, const int64_t* blk, const int32_t* cidx,
                           const double* cdiag, double* A_val, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_image_diag, dim3((n + 255) / 256), dim3(256), 0, s, n, node, blk, cidx,
                     cdiag, A_val);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_T_rhs(const CellData& cd, const int32_t* cells, int n, const double* T_old,
                  const double* u_cur, const PhysicsDev& ph, double* rhs, hipStream_t s) {
  if (n <= 0) return;
  if (cd.tdpc == 27) return launch_T2_rhs(cd, cells, n, T_old, u_cur, ph, rhs, s);
  hipLaunchKernelGGL(k_T_rhs, dim3(n), dim3(64), 0, s, cd, cells, T_old, u_cur, ph, rhs);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_build_scatter_maps(const CellData& cd, const int32_t* A_ptr, const int32_t* A_col,
                               const int32_t* Bt_ptr, const int32_t* Bt_col, const int32_t* B_ptr,
                               const int32_t* B_col, const int32_t* T_ptr, const int32_t* T_col,
                               int32_t* posA, int32_t* posBt, int32_t* posB, int32_t* posT,
                               hipStream_t s) {
  if (cd.n_cells <= 0) return;
  hipLaunchKernelGGL(k_scatter_maps, dim3(cd.n_cells), dim3(256), 0, s, cd, A_ptr, A_col, Bt_ptr,
                     Bt_col, B_ptr, B_col, T_ptr, T_col, posA, posBt, posB, posT);
  DCP_HIP_CHECK(hipGetLastError());
}

bool mark_first_touch(const int32_t* color_cells, const std::vector<int>& color_ptr, int per_cell,
                      int32_t* pos, size_t n_cells, size_t nnz, hipStream_t s,
                      unsigned long long* touched_out) {
  uint8_t* touched = nullptr;
  unsigned long long* count = nullptr;
  DCP_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&touched), nnz, s));
  DCP_HIP_CHECK(hipMallocAsync(reinterpret_cast<void**>(&count), sizeof(unsigned long long), s));
  DCP_HIP_CHECK(hipMemsetAsync(touched, 0, nnz, s));
  DCP_HIP_CHECK(hipMemsetAsync(count, 0, sizeof(unsigned long long), s));
  for (size_t k = 0; k + 1 < color_ptr.size(); ++k) {
    const int n = color_ptr[k + 1] - color_ptr[k];
    if (n <= 0) continue;
    hipLaunchKernelGGL(k_first_touch, dim3(n), dim3(256), 0, s, color_cells + color_ptr[k],
                       per_cell, pos, touched, count);
    DCP_HIP_CHECK(hipGetLastError());
  }
  unsigned long long h = 0;
  DCP_HIP_CHECK(hipMemcpyAsync(&h, count, sizeof(h), hipMemcpyDeviceToHost, s));
  DCP_HIP_CHECK(hipStreamSynchronize(s));
  DCP_HIP_CHECK(hipFree(touched));
  DCP_HIP_CHECK(hipFree(count));
  if (touched_out) *touched_out = h;
  if (h == nnz) return true;
  // some block is never touched by a cell: keep plain positions (zero fill needed)
  hipLaunchKernelGGL(k_clear_first_touch, dim3(1024), dim3(256), 0, s, size_t(per_cell) * n_cells, pos);
  DCP_HIP_CHECK(hipGetLastError());
  return false;
}

void launch_bt_rows(const CellData& cd, int n_cols, int n_layers, double* P, double* Q,
                    int n_tasks, int slots, const int32_t* task_hdr, const int32_t* slot_rec,
                    double* Bt, hipStream_t s) {
  if (n_cols > 0) {
    hipLaunchKernelGGL(k_bt_coltab, dim3(n_cols), dim3(kBtColEntries), 0, s, cd.sep_colgeo, P);
    DCP_HIP_CHECK(hipGetLastError());
  }
  if (n_layers > 0) {
    hipLaunchKernelGGL(k_bt_laytab, dim3(n_layers), dim3(kBtLayEntries), 0, s, cd.sep_laygeo, Q);
    DCP_HIP_CHECK(hipGetLastError());
  }
  if (n_tasks > 0) {
    const char* env = std::getenv("DCP_BT_MODE");
    const int mode = env ? std::atoi(env) : 3;
    hipLaunchKernelGGL((slots == 32 ? k_bt_tasks<32, 2> : slots == 16 ? k_bt_tasks<16, 1> : k_bt_tasks<8, 1>),
                       dim3((n_tasks + kBtRowWaves - 1) / kBtRowWaves), dim3(64 * kBtRowWaves), 0,
                       s, cd, n_tasks, reinterpret_cast<const int4*>(task_hdr),
                       reinterpret_cast<const int4*>(slot_rec), P, Q, Bt, mode);
    DCP_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace dcp
