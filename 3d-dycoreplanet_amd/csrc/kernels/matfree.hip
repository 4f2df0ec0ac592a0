// Matrix-free Stokes operator of the classic Q2^3/Q1 system for CDNA4 (gfx950), FP64.
//
// Applies the operator that assemble_nse_system + distribute_local_to_global
// build (boussinesq_model.tpp:550-687; its matrix part :626-637) without the
// matrix:
//   [A B^T; B 0] x = sum_cells C^T K_cell C x  (+ the constrained diagonal)
// with, per quadrature point (w = JxW, nu = dt/Re, u / grad u / p of C x):
//   velocity test a, component c:  w [ phi_a u_c + sum_d d_d phi_a F_cd ],
//       F_cd = nu (d_d u_c + d_c u_d) - p delta_cd        (2 nu eps:eps, -p div)
//   pressure test v:              -w psi_v div u.
// C is the per-node AffineConstraints condensation of the assembly kernel
// (no-normal-flux / no-slip velocity constraints; pressure unconstrained). The
// rows and columns of constrained velocity dofs of C^T K C vanish; their
// entries are the |K_ii| diagonal the assembly adds, applied by a small fix-up
// pass from the assembled diagonal (k_mf_constrained).
//
// Layout: 27 lanes per cell (lexicographic node / quadrature index, x
// fastest), two cells per wave, four per 128-thread workgroup; the per-cell
// arrays (node map, pressure dofs, first-touch bits, geometry) are stored in
// colour order, so a colour class is a contiguous range streamed without an
// indirection. Values and
// reference gradients at the 27 Gauss points come from sum factorisation over
// the 3x3 1D tables (3 passes forward, 3 back, 27 FMAs per component and pass
// set), exchanged through a 12-field LDS slab per cell with wave-level
// synchronisation only. J^-1 and JxW per point are precomputed once per mesh
// (k_mf_geometry; the mesh does not move) and streamed: 2160 B per cell, the
// dominant HBM traffic (SURVEY §8d's matrix-free byte count). The cell loop
// runs over the colour classes of the assembly, so no two workgroups of a
// launch touch the same dof: plain read-modify-write, deterministic, and the
// first cell touching a dof (colour order) stores instead of adding, so dst
// needs no zero fill.
#include <hip/hip_runtime.h>

#include <utility>

#include "../device.h"
#include "../fe_tables.h"

namespace dcp {
namespace {

constexpr double l2c(int i, double x) {
  return i == 0 ? 2 * (x - 0.5) * (x - 1) : i == 1 ? -4 * x * (x - 1) : 2 * x * (x - 0.5);
}
constexpr double dl2c(int i, double x) { return i == 0 ? 4 * x - 3 : i == 1 ? -8 * x + 4 : 4 * x - 1; }
constexpr double l1c(int i, double x) { return i == 0 ? 1 - x : x; }

// 1D Q2 basis n at Gauss point q: value / derivative (geometry precompute)
__constant__ double mW[3] = {kGaussW[0], kGaussW[1], kGaussW[2]};

// The apply kernel picks its 1D coefficients by lane index with selects
// between compile-time constants (no lane-divergent constant-memory loads).
__device__ inline double sel3(int x, double a, double b, double c) {
  return x == 0 ? a : (x == 1 ? b : c);
}
// L[n][q] / D[n][q] with n compile-time, q per lane
template <int N>
__device__ inline double Lq(int q) {
  return sel3(q, l2c(N, kGaussX[0]), l2c(N, kGaussX[1]), l2c(N, kGaussX[2]));
}
template <int N>
__device__ inline double Dq(int q) {
  return sel3(q, dl2c(N, kGaussX[0]), dl2c(N, kGaussX[1]), dl2c(N, kGaussX[2]));
}
// L[n][q] / D[n][q] with q compile-time, n per lane
template <int Q>
__device__ inline double Ln(int n) {
  return sel3(n, l2c(0, kGaussX[Q]), l2c(1, kGaussX[Q]), l2c(2, kGaussX[Q]));
}
template <int Q>
__device__ inline double Dn(int n) {
  return sel3(n, dl2c(0, kGaussX[Q]), dl2c(1, kGaussX[Q]), dl2c(2, kGaussX[Q]));
}
// Q1 vertex function v (per lane) at Gauss point Q (compile-time)
template <int Q>
__device__ inline double psi_v(int v) {
  constexpr double x0 = kGaussX[Q % 3], x1 = kGaussX[(Q / 3) % 3], x2 = kGaussX[Q / 9];
  return ((v & 1) ? l1c(1, x0) : l1c(0, x0)) * (((v >> 1) & 1) ? l1c(1, x1) : l1c(0, x1)) *
         ((v >> 2) ? l1c(1, x2) : l1c(0, x2));
}
template <int... Q>
__device__ inline double psi_dot(int v, const double* s, std::integer_sequence<int, Q...>) {
  double r = 0.0;
  ((r += psi_v<Q>(v) * s[Q]), ...);
  return r;
}

constexpr int kMfCells = 4;    // cells per 128-thread workgroup (two per wave)
constexpr int kGeoCells = 8;            // k_mf_geometry: cells per 256-thread workgroup
constexpr int kMfFields = 13;   // LDS fields of 27 doubles per cell

// wave-level LDS hand-off (a cell never spans waves)
__device__ inline void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// full = C reduced (no-normal-flux: component k eliminated; no-slip: 0)
__device__ inline void expand(const NodeConstraint& nc, const double r[3], double f[3]) {
  if (nc.type == 0) {
    f[0] = r[0]; f[1] = r[1]; f[2] = r[2];
  } else if (nc.type == 1) {
    f[0] = f[1] = f[2] = 0.0;
  } else {
    double s = 0.0;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      f[d] = r[d];
      if (d != nc.k) s += nc.w[d] * r[d];
    }
    f[nc.k] = s;
  }
}
// reduced = C^T full
__device__ inline void condense(const NodeConstraint& nc, double f[3]) {
  if (nc.type == 1 || nc.type == 3) {
    f[0] = f[1] = f[2] = 0.0;
  } else if (nc.type == 2) {
    const double fk = f[nc.k];
#pragma unroll
    for (int d = 0; d < 3; ++d) f[d] = d == nc.k ? 0.0 : f[d] + nc.w[d] * fk;
  }
}

// J^-1 (dxi_e/dx_d as [e][d]) and JxW of the cell's MappingQ(3) at every
// Gauss point, stored [cell][k][q] (k < 9: J^-1, k = 9: JxW). Same formulas as
// the assembly kernel (kernels/assembly.hip, cell_geometry).
// Position e of the output belongs to cell order[e] (colour order; null =
// identity). 8 cells per 256-thread block, thread t < 27 of a 32-lane slot
// owns Gauss point t; the cell's 64 support points are staged in LDS.
__constant__ double mL3[4][3] = {
    {map_lag(0, kGaussX[0]), map_lag(0, kGaussX[1]), map_lag(0, kGaussX[2])},
    {map_lag(1, kGaussX[0]), map_lag(1, kGaussX[1]), map_lag(1, kGaussX[2])},
    {map_lag(2, kGaussX[0]), map_lag(2, kGaussX[1]), map_lag(2, kGaussX[2])},
    {map_lag(3, kGaussX[0]), map_lag(3, kGaussX[1]), map_lag(3, kGaussX[2])}};
__constant__ double mD3[4][3] = {
    {map_dlag(0, kGaussX[0]), map_dlag(0, kGaussX[1]), map_dlag(0, kGaussX[2])},
    {map_dlag(1, kGaussX[0]), map_dlag(1, kGaussX[1]), map_dlag(1, kGaussX[2])},
    {map_dlag(2, kGaussX[0]), map_dlag(2, kGaussX[1]), map_dlag(2, kGaussX[2])},
    {map_dlag(3, kGaussX[0]), map_dlag(3, kGaussX[1]), map_dlag(3, kGaussX[2])}};
__global__ __launch_bounds__(256) void k_mf_geometry(CellData cd, const int32_t* __restrict__ order,
                                                     double* __restrict__ geo) {
  __shared__ double X[kGeoCells][3 * kMapPts];
  const int slot = threadIdx.x >> 5, t = threadIdx.x & 31;
  const int pos = blockIdx.x * kGeoCells + slot;
  const bool live = pos < cd.n_cells;
  const int cell = live ? (order ? order[pos] : pos) : 0;
  if (live)
    for (int i = t; i < 3 * kMapPts; i += 32) X[slot][i] = cd.geo[3 * kMapPts * size_t(cell) + i];
  __syncthreads();
  if (!live || t >= 27) return;
  const int q0 = t % 3, q1 = (t / 3) % 3, q2 = t / 9;
  double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  for (int n = 0; n < kMapPts; ++n) {
    const int a = n % 4, b = (n / 4) % 4, c = n / 16;
    const double la = mL3[a][q0], lb = mL3[b][q1], lc = mL3[c][q2];
    const double g0 = mD3[a][q0] * lb * lc, g1 = la * mD3[b][q1] * lc, g2 = la * lb * mD3[c][q2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double Xi = X[slot][3 * n + i];
      J[i][0] += Xi * g0;
      J[i][1] += Xi * g1;
      J[i][2] += Xi * g2;
    }
  }
  const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
  const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
  const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
  const double det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
  const double id = 1.0 / det;
  double Ji[9];
  Ji[0] = c00 * id;
  Ji[1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * id;
  Ji[2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * id;
  Ji[3] = c01 * id;
  Ji[4] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * id;
  Ji[5] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * id;
  Ji[6] = c02 * id;
  Ji[7] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * id;
  Ji[8] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * id;
  double* g = geo + 270 * size_t(pos);
#pragma unroll
  for (int k = 0; k < 9; ++k) g[27 * k + t] = Ji[k];
  g[243 + t] = det * mW[q0] * mW[q1] * mW[q2];
}

// One colour class of the matrix-free apply: positions [base, base + n) of the
// colour-ordered cell arrays. STOKES: [A B^T; B 0] on the [u | p] vector (p at
// offset n_u); else the velocity block A alone.
template <bool STOKES>
__global__ __launch_bounds__(32 * kMfCells) void k_mf_stokes(MfData md, int base, int n, double nu,
                                                   const double* __restrict__ src,
                                                   double* __restrict__ dst) {
  __shared__ double slab[kMfCells][kMfFields][27];
  const int slot = threadIdx.x >> 5, t = threadIdx.x & 31;
  const int ci = blockIdx.x * kMfCells + slot;
  const bool active = t < 27 && ci < n;
  double(*B)[27] = slab[slot];
  const int i = t % 3, j = (t / 3) % 3, k = t / 9;
  const size_t e = size_t(base) + (active ? ci : 0);
  int node = 0, pdof = 0;
  NodeConstraint nc{};
  uint64_t first = 0;
  double Ji[9], w = 0.0;
  if (active) {
    // independent streamed loads first: node map, geometry, first-touch bits
    node = md.cell_q2[27 * e + t];
    const double* g = md.geo + 270 * e + t;
#pragma unroll
    for (int q = 0; q < 9; ++q) Ji[q] = g[27 * q];
    w = g[243];
    first = md.first[e];
    if (STOKES && t < 8) pdof = md.cell_p[8 * e + t];
    nc = md.vcon[node];
    const double r[3] = {src[3 * size_t(node)], src[3 * size_t(node) + 1],
                         src[3 * size_t(node) + 2]};
    double f[3];
    expand(nc, r, f);
    B[0][t] = f[0];
    B[1][t] = f[1];
    B[2][t] = f[2];
    if (STOKES && t < 8) B[3][t] = src[md.n_u + pdof];
  }
  wsync();
  // ---- values and reference gradients at the Gauss points
  double o[9];
  double pq = 0.0;
  if (active) {
    const double l0 = Lq<0>(i), l1 = Lq<1>(i), l2 = Lq<2>(i);
    const double d0 = Dq<0>(i), d1 = Dq<1>(i), d2 = Dq<2>(i);
#pragma unroll
    for (int c = 0; c < 3; ++c) {  // pass x: (n0 -> q0 = i)
      const double* x = &B[c][3 * j + 9 * k];
      o[c] = l0 * x[0] + l1 * x[1] + l2 * x[2];
      o[3 + c] = d0 * x[0] + d1 * x[1] + d2 * x[2];
    }
    if (STOKES) {
      // p at q = t from the 8 vertex values
      const double a0 = 1.0 - sel3(i, kGaussX[0], kGaussX[1], kGaussX[2]);
      const double b0 = 1.0 - sel3(j, kGaussX[0], kGaussX[1], kGaussX[2]);
      const double c0 = 1.0 - sel3(k, kGaussX[0], kGaussX[1], kGaussX[2]);
      const double a1 = 1.0 - a0, b1 = 1.0 - b0, c1 = 1.0 - c0;
      const double* p = B[3];
      pq = c0 * (b0 * (a0 * p[0] + a1 * p[1]) + b1 * (a0 * p[2] + a1 * p[3])) +
           c1 * (b0 * (a0 * p[4] + a1 * p[5]) + b1 * (a0 * p[6] + a1 * p[7]));
    }
  }
  wsync();
  if (active) {
#pragma unroll
    for (int f = 0; f < 6; ++f) B[f][t] = o[f];
  }
  wsync();
  if (active) {
    const double l0 = Lq<0>(j), l1 = Lq<1>(j), l2 = Lq<2>(j);
    const double d0 = Dq<0>(j), d1 = Dq<1>(j), d2 = Dq<2>(j);
#pragma unroll
    for (int c = 0; c < 3; ++c) {  // pass y: (n1 -> q1 = j)
      const double* v = &B[c][i + 9 * k];
      const double* dx = &B[3 + c][i + 9 * k];
      o[c] = l0 * v[0] + l1 * v[3] + l2 * v[6];
      o[3 + c] = l0 * dx[0] + l1 * dx[3] + l2 * dx[6];
      o[6 + c] = d0 * v[0] + d1 * v[3] + d2 * v[6];
    }
  }
  wsync();
  if (active) {
#pragma unroll
    for (int f = 0; f < 9; ++f) B[f][t] = o[f];
  }
  wsync();
  double sq = 0.0;
  if (active) {
    const double l0 = Lq<0>(k), l1 = Lq<1>(k), l2 = Lq<2>(k);
    const double d0 = Dq<0>(k), d1 = Dq<1>(k), d2 = Dq<2>(k);
    double u[3], Gh[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {  // pass z: (n2 -> q2 = k)
      const double* v = &B[c][i + 3 * j];
      const double* dx = &B[3 + c][i + 3 * j];
      const double* dy = &B[6 + c][i + 3 * j];
      u[c] = l0 * v[0] + l1 * v[9] + l2 * v[18];
      Gh[c][0] = l0 * dx[0] + l1 * dx[9] + l2 * dx[18];
      Gh[c][1] = l0 * dy[0] + l1 * dy[9] + l2 * dy[18];
      Gh[c][2] = d0 * v[0] + d1 * v[9] + d2 * v[18];
    }
    // quadrature point q = t: physical gradient, flux, back to reference
    double G[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int d = 0; d < 3; ++d)
        G[c][d] = Gh[c][0] * Ji[d] + Gh[c][1] * Ji[3 + d] + Gh[c][2] * Ji[6 + d];
    double F[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int d = 0; d < 3; ++d) F[c][d] = nu * (G[c][d] + G[d][c]);
    if (STOKES) {
      F[0][0] -= pq;
      F[1][1] -= pq;
      F[2][2] -= pq;
      sq = -w * (G[0][0] + G[1][1] + G[2][2]);
    }
    // every lane has read its pass-z inputs before any lane overwrites them
    wsync();
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      B[c][t] = w * u[c];
#pragma unroll
      for (int e2 = 0; e2 < 3; ++e2)
        B[3 + 3 * e2 + c][t] =
            w * (Ji[3 * e2] * F[c][0] + Ji[3 * e2 + 1] * F[c][1] + Ji[3 * e2 + 2] * F[c][2]);
    }
    if (STOKES) B[12][t] = sq;
  } else {
    wsync();
  }
  wsync();
  // ---- test functions: transposed passes (fields: V 0-2, Fx 3-5, Fy 6-8, Fz 9-11)
  double yp = 0.0;
  if (active) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {  // back z: (q2 -> n2 = k)
      const double* v = &B[c][i + 3 * j];
      const double* fx = &B[3 + c][i + 3 * j];
      const double* fy = &B[6 + c][i + 3 * j];
      const double* fz = &B[9 + c][i + 3 * j];
      o[c] = Ln<0>(k) * v[0] + Ln<1>(k) * v[9] + Ln<2>(k) * v[18] + Dn<0>(k) * fz[0] +
             Dn<1>(k) * fz[9] + Dn<2>(k) * fz[18];
      o[3 + c] = Ln<0>(k) * fx[0] + Ln<1>(k) * fx[9] + Ln<2>(k) * fx[18];
      o[6 + c] = Ln<0>(k) * fy[0] + Ln<1>(k) * fy[9] + Ln<2>(k) * fy[18];
    }
    if (STOKES && t < 8) yp = psi_dot(t, B[12], std::make_integer_sequence<int, 27>{});
  }
  wsync();
  if (active) {
#pragma unroll
    for (int f = 0; f < 9; ++f) B[f][t] = o[f];
  }
  wsync();
  if (active) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {  // back y: (q1 -> n1 = j)
      const double* v = &B[c][i + 9 * k];
      const double* fx = &B[3 + c][i + 9 * k];
      const double* fy = &B[6 + c][i + 9 * k];
      o[c] = Ln<0>(j) * v[0] + Ln<1>(j) * v[3] + Ln<2>(j) * v[6] + Dn<0>(j) * fy[0] +
             Dn<1>(j) * fy[3] + Dn<2>(j) * fy[6];
      o[3 + c] = Ln<0>(j) * fx[0] + Ln<1>(j) * fx[3] + Ln<2>(j) * fx[6];
    }
  }
  wsync();
  if (active) {
#pragma unroll
    for (int f = 0; f < 6; ++f) B[f][t] = o[f];
  }
  wsync();
  if (!active) return;
  double y[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {  // back x: (q0 -> n0 = i)
    const double* v = &B[c][3 * j + 9 * k];
    const double* fx = &B[3 + c][3 * j + 9 * k];
    y[c] = Ln<0>(i) * v[0] + Ln<1>(i) * v[1] + Ln<2>(i) * v[2] + Dn<0>(i) * fx[0] +
           Dn<1>(i) * fx[1] + Dn<2>(i) * fx[2];
  }
  condense(nc, y);
  double* d = dst + 3 * size_t(node);
  if ((first >> t) & 1) {
    d[0] = y[0];
    d[1] = y[1];
    d[2] = y[2];
  } else {
    d[0] += y[0];
    d[1] += y[1];
    d[2] += y[2];
  }
  if (STOKES && t < 8) {
    double* dp = dst + md.n_u + pdof;
    *dp = ((first >> (32 + t)) & 1) ? yp : *dp + yp;
  }
}

// ---- cell-order pencil kernel -----------------------------------------------
//
// Nine lanes per cell, seven cells per wave (lane 63 works a dummy slot). Each
// lane owns a "pencil" of three nodes / points along one axis, so every 1D
// contraction of the sum factorisation runs in registers with compile-time
// coefficients; the LDS only transposes between the x-, y- and z-pencil
// layouts (x-pencil p = b + 3c, y-pencil p = a + 3c, z-pencil p = a + 3b over
// lexicographic (a, b, c)). The MappingQ(3) geometry (J^-1, JxW at the 27
// Gauss points) comes from the radially separable tables (a per-column 2D
// table and per-layer radii, L2-resident) or, for other meshes, the streamed
// per-cell table of k_mf_geometry. The seven cells of a wave are consecutive in
// tree order and share nodes: their velocity results are summed per node in
// LDS (one partial per node and wave, chained occurrences, host-built) before
// the store, 35 % fewer records than one per (cell, node) at r=5; src is
// gathered through the caches.
#ifndef DCP_MF_CELLS
#define DCP_MF_CELLS 7
#endif
constexpr int kPenCells = DCP_MF_CELLS;  // cells per wave
constexpr int kPenWaves = DCP_MF_WAVES;  // waves per workgroup (device.h)
static_assert(kPenCells * kPenWaves == kMfGroupCells,
              "the host groups the velocity partial sums per workgroup");
#ifndef DCP_MF_SLOTS
#define DCP_MF_SLOTS DCP_MF_CELLS
#endif
// LDS cell slots per wave: 7 (lane 63, the dummy cell, stores nothing) or 8
constexpr int kPenSlots = DCP_MF_SLOTS;
// LDS: 9 fields of 27 doubles per cell slot, field-major ([field][slot][27]):
// fewer bank conflicts for the three pencil patterns than cell-major slots;
// then per slot the 8 vertex pressures and the 18 pressure-test partials.
#ifndef DCP_MF_FIELD_MAJOR
#define DCP_MF_FIELD_MAJOR 1
#endif
constexpr int kFS = DCP_MF_FIELD_MAJOR ? kPenSlots * 27 : 27;   // field stride (doubles)
constexpr int kPenFields = 9 * kPenSlots * 27;           // per wave
// DCP_MF_LDS_ALIAS: the vertex pressures, the pressure-test partials and the
// chain links live in field slabs that are dead at the time (see the kernel),
// so a wave needs only the 9 fields: 13.6 instead of 15.3 KB, 12 instead of
// 10 waves per CU (the 166 VGPRs allow 3 per SIMD)
#ifndef DCP_MF_LDS_ALIAS
#define DCP_MF_LDS_ALIAS 1
#endif
#if !DCP_MF_LDS_ALIAS
constexpr int kPenAux = 8 + 18 + 1;  // per slot
#endif
#ifndef DCP_MF_BATCHES
#define DCP_MF_BATCHES 1
#endif
constexpr int kMfBatches = DCP_MF_BATCHES;  // cell batches per workgroup (pipelined)
__host__ __device__ constexpr int kMfBatchTotal(int n_cells) {
  return (n_cells + kPenCells * kPenWaves - 1) / (kPenCells * kPenWaves);
}

struct Tab3 {
  double v[3][3];
};
constexpr Tab3 make_tab(bool deriv) {
  Tab3 t{};
  for (int n = 0; n < 3; ++n)
    for (int q = 0; q < 3; ++q) t.v[n][q] = deriv ? dl2c(n, kGaussX[q]) : l2c(n, kGaussX[q]);
  return t;
}
constexpr Tab3 kTL = make_tab(false);  // [node][point] value
constexpr Tab3 kTD = make_tab(true);   // [node][point] derivative

// out[q] = sum_n T[n][q] in[n]
__device__ inline void fwd(const Tab3& T, const double in[3], double out[3]) {
#pragma unroll
  for (int q = 0; q < 3; ++q) out[q] = T.v[0][q] * in[0] + T.v[1][q] * in[1] + T.v[2][q] * in[2];
}
// out[n] = sum_q T[n][q] in[q]
__device__ inline void bwd(const Tab3& T, const double in[3], double out[3]) {
#pragma unroll
  for (int n = 0; n < 3; ++n) out[n] = T.v[n][0] * in[0] + T.v[n][1] * in[1] + T.v[n][2] * in[2];
}

// the NSE rhs flux of one Gauss point (k_mf_pencil<.., RHS>): value u,
// reference gradients Gh[c][e], J^-1 ji (rows e), JxW wq, temperature Tq,
// position R Phi (separable shell; cuboid: constant gravity), added to the
// z-pencil's test sums V[c][k] with the values of the point's 1D functions
__device__ __forceinline__ void rhs_flux(const PhysicsDev& ph, const double u[3],
                                         const double Gh[3][3], const double ji[9], double wq,
                                         double Tq, double gs, const double rphi[3], int q,
                                         double V[3][3]) {
  double G[3][3];
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int d = 0; d < 3; ++d) G[c][d] = Gh[c][0] * ji[d] + Gh[c][1] * ji[3 + d] + Gh[c][2] * ji[6 + d];
  const double rho = 1 - ph.beta * (Tq - ph.T_ref);
  double grav[3];
  if (ph.cuboid) {
    grav[0] = grav[1] = 0;
    grav[2] = -ph.g;
  } else {
    // -g x / den(|x|) with x = R Phi: gs = -g R / den(R |Phi|) (MfCells::colphin)
    grav[0] = gs * rphi[0];
    grav[1] = gs * rphi[1];
    grav[2] = gs * rphi[2];
  }
  const double cxu[3] = {-ph.coriolis_z * u[1], ph.coriolis_z * u[0], 0.0};
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const double adv = u[0] * G[c][0] + u[1] * G[c][1] + u[2] * G[c][2];
    const double F =
        (u[c] + ph.dt * rho * (ph.grav_scale * grav[c]) - ph.dt * adv - ph.dt * (2 * cxu[c])) * wq;
#pragma unroll
    for (int k = 0; k < 3; ++k) V[c][k] += kTL.v[k][q] * F;
  }
}

#ifndef DCP_MF_WAVES_PER_EU
#define DCP_MF_WAVES_PER_EU 2
#endif
// RHS: the NSE rhs instead of an operator apply (mf_rhs): src = the old
// velocity (a full vector: no constraint expansion), T_old its temperature
// (FE_Q(1), interpolated like the pressure), and per Gauss point the flux
// F = (u + dt rho g' - dt (u.grad) u - 2 dt Omega x u) JxW of
// local_assemble_nse_system (boussinesq_model.tpp:655-669) against the test
// function values only
// record stores of the fused apply (k_mf_fused): agent-scope (sc1) stores, so a
// gather task on any XCD reads them after the batch's done flag
// timing switches: DCP_MF_FUSED_SC1=0 plain record stores / loads in the fused
// kernel (wrong across XCDs: probes only); DCP_MF_REC_SC1=1 agent-coherent
// record stores in the two-launch kernel too (the cost of write-through alone)
#ifndef DCP_MF_FUSED_SC1
#define DCP_MF_FUSED_SC1 1
#endif
#ifndef DCP_MF_REC_SC1
#define DCP_MF_REC_SC1 0
#endif
__device__ __forceinline__ void rec_store(double* p, double v, bool fused) {
  if ((fused && DCP_MF_FUSED_SC1) || DCP_MF_REC_SC1)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p),
                       (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  else
    *p = v;
}
__device__ __forceinline__ double rec_load(const double* p, bool fused) {
  if (fused && DCP_MF_FUSED_SC1)
    return __longlong_as_double((long long)__hip_atomic_load(
        reinterpret_cast<const unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  return *p;
}

// The pencil kernel's work for cell batch `blk` (k_mf_pencil: the block's
// XCD-contiguous batch; k_mf_fused: the batch of its schedule entry). FUSED:
// records stored agent-coherent and, once they are complete, the batch's done
// flag (done[blk] = seq) for the gather tasks waiting on it.
template <bool STOKES, bool SEP, bool RHS, bool FUSED>
__device__ __forceinline__ void pencil_body(const MfCells& mc, int blk, int c0, int c1, double nu,
                                            const double* __restrict__ src,
                                            double* __restrict__ buf, double* __restrict__ dst,
                                            const double* __restrict__ T_old,
                                            const PhysicsDev& ph, double (*lds)[kPenFields],
                                            unsigned* done, unsigned seq) {
  static_assert(!(RHS && STOKES), "the rhs pass has no pressure");
#if !DCP_MF_LDS_ALIAS
  __shared__ double aux[kPenWaves][kPenSlots][kPenAux];
  __shared__ MfLink nxt_own[kPenWaves * kPenCells * 27];  // chain links of the group partial sums
#endif
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  // lane 63 shadows lane 54 (slot 6, pencil 0) with 7 LDS slots: it computes
  // and stores the same LDS values and skips the global store; with 8 slots it
  // works a dummy slot of its own
  // (with 6 cells per wave, lanes 54..62 shadow lanes 45..53 the same way)
  const bool dummy = lane >= 9 * kPenCells;
#ifndef DCP_MF_SHADOW
#define DCP_MF_SHADOW (kPenSlots == kPenCells)
#endif
  const int cs = DCP_MF_SHADOW && dummy ? kPenCells - 1 : lane / 9;
  const int p = DCP_MF_SHADOW && dummy ? (lane - 9 * (lane / 9)) % 9 : lane - 9 * cs;
  const int pa = p % 3, pb = p / 3;
  double* S = lds[wave] + (DCP_MF_FIELD_MAJOR ? 27 * cs : 243 * cs);
#if DCP_MF_LDS_ALIAS
  // P (vertex values): field 8 of the slot, read before the forward y pass
  // writes it; SP (pressure-test partials): field 6, written after the back y
  // pass has read it; the chain links: bytes of fields 3.. of the wave, written
  // after the back x pass has read them
  double* P = S + 8 * kFS;
  double* SP = S + 6 * kFS;
  MfLink* nxt0 = reinterpret_cast<MfLink*>(&lds[0][3 * kFS]);
  auto nxt = [&](int k) -> MfLink& {
    const int wk = k / (27 * kPenCells);
    return nxt0[wk * int(sizeof(double)) * kPenFields + (k - 27 * kPenCells * wk)];
  };
#else
  double* P = aux[wave][cs];
  double* SP = P + 8;
  auto nxt = [&](int k) -> MfLink& { return nxt_own[k]; };
#endif
  // LDS reads through a volatile view: keeps them single ds_read_b64 (256 B/clk)
  // instead of merged ds_read2_b64 pairs (128 B/clk on gfx950)
#ifndef DCP_MF_VOLATILE_READS
#define DCP_MF_VOLATILE_READS 1
#endif
#if DCP_MF_VOLATILE_READS
  typedef __attribute__((address_space(3))) const volatile double lds_vdouble;
  lds_vdouble* SR = (lds_vdouble*)S;
#else
  const double* SR = S;
#endif
  // Slot layout of node / point (a, b, c): 3a + b + 9c (DCP_MF_SWAP_AB, default)
  // or lexicographic a + 3b + 9c. With 7 cells of 9 lanes per wave the swapped
  // form makes the y-pencil accesses (15 of the 30 per batch) conflict-free and
  // leaves x and z at 2-way, against 2-way y and z for the lexicographic one.
#ifndef DCP_MF_SWAP_AB
#define DCP_MF_SWAP_AB 1
#endif
  constexpr int xs = DCP_MF_SWAP_AB ? 3 : 1, ys = DCP_MF_SWAP_AB ? 1 : 3;
  const int xo = DCP_MF_SWAP_AB ? pa + 9 * pb : 3 * p;       // x-pencil (b, c) = (pa, pb)
  const int yo = DCP_MF_SWAP_AB ? 3 * pa + 9 * pb : pa + 9 * pb;  // y-pencil (a, c)
  const int zo = DCP_MF_SWAP_AB ? 3 * pa + pb : p;            // z-pencil (a, b)
  const double wab = sel3(pa, kGaussW[0], kGaussW[1], kGaussW[2]) *
                     sel3(pb, kGaussW[0], kGaussW[1], kGaussW[2]);

  // Software pipeline over the workgroup's kMfBatches batches of cells: the
  // node ids of batch j + 2 and the node data of batch j + 1 are in flight
  // while batch j computes.
  auto cell_of = [&](int j) {
    return c0 + ((blk * kMfBatches + j) * kPenWaves + wave) * kPenCells + cs;
  };
  struct Ids {
    int nd[3], slot[3], next[3];
    int pdof, pslot;
    uint32_t mask;
  };
  struct Nodes {
    double U[3][3];
    double pv;
  };
  // DCP_MF_NTIDX (default on): the per-cell index streams (read once per
  // apply) as nontemporal loads, keeping the caches for the gathered src
#ifndef DCP_MF_NTIDX
#define DCP_MF_NTIDX 1
#endif
  auto ldi = [](const auto* q) {
    if (DCP_MF_NTIDX) return __builtin_nontemporal_load(q);
    return *q;
  };
  auto load_ids = [&](int j, Ids& I) {
    const int cell = cell_of(j);
    const size_t e = (cs < kPenCells && cell < c1) ? size_t(cell) : 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      I.nd[a] = ldi(mc.cell_q2 + 27 * e + 3 * p + a);
      I.slot[a] = ldi(mc.vslot + 27 * e + 3 * p + a);
      I.next[a] = ldi(mc.vnext + 27 * e + 3 * p + a);
    }
    I.mask = ldi(mc.cmask + e);
    I.pdof = (STOKES && p < 8) ? ldi(mc.cell_p + 8 * e + p) : (RHS && p < 8) ? ldi(mc.cell_T + 8 * e + p) : 0;
    I.pslot = (STOKES && p < 8) ? ldi(mc.pslot + 8 * e + p) : 0;
  };
  auto load_nodes = [&](const Ids& I, Nodes& N) {
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        N.U[a][d] = src[3 * size_t(I.nd[a]) + d];
      }
    N.pv = (STOKES && p < 8) ? src[mc.n_u + I.pdof] : (RHS && p < 8) ? T_old[I.pdof] : 0.0;
  };
#ifndef DCP_MF_PREFETCH_NODES
#define DCP_MF_PREFETCH_NODES 1
#endif
  Ids Ic, In;
  Nodes Nc;
  load_ids(0, Ic);
  if (DCP_MF_PREFETCH_NODES) load_nodes(Ic, Nc);
  if (kMfBatches > 1) load_ids(1, In);
  for (int j = 0; j < kMfBatches; ++j) {
  if (blk * kMfBatches + j >= kMfBatchTotal(c1 - c0)) break;  // uniform per workgroup
  Nodes Nn;
  Ids Inn;
  if (!DCP_MF_PREFETCH_NODES) load_nodes(Ic, Nc);
  if (DCP_MF_PREFETCH_NODES && j + 1 < kMfBatches) load_nodes(In, Nn);
  if (j + 2 < kMfBatches) load_ids(j + 2, Inn);
  const int cell = cell_of(j);
  const bool live = !dummy && cell < c1;
  // loads index the cell (the shadow lane must see exactly its twin's data)
  const size_t e = (cs < kPenCells && cell < c1) ? size_t(cell) : 0;
  const int* nd = Ic.nd;
  const uint32_t mask = Ic.mask;
  double(&U)[3][3] = Nc.U;
  const int colc = SEP ? mc.col[e] : 0;
  const int layc = SEP ? mc.layer[e] : 0;
  if ((STOKES || RHS) && p < 8) P[p] = Nc.pv;  // pressure / temperature at the vertices
  if (mask && !RHS) {
#pragma unroll
    for (int a = 0; a < 3; ++a)
      if ((mask >> (3 * p + a)) & 1) {
        const NodeConstraint nc = mc.vcon[nd[a]];
        double f[3];
        expand(nc, U[a], f);
        U[a][0] = f[0];
        U[a][1] = f[1];
        U[a][2] = f[2];
      }
  }

  // ---- geometry: J^-1 and JxW at the z-pencil's three points
  double Ji[3][9], w[3];
  if (!SEP) {
    // general MappingQ(3) geometry: J^-1 / JxW of the z-pencil's three points
    // streamed from the per-cell table k_mf_geometry builds at upload
    const double* g = mc.geo + 270 * e;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
#pragma unroll
      for (int i = 0; i < 9; ++i) Ji[q][i] = g[27 * i + p + 9 * q];
      w[q] = g[243 + p + 9 * q];
    }
  }
  // ---- velocity: values and reference gradients
#pragma unroll
  for (int c = 0; c < 3; ++c) {  // x
    const double in[3] = {U[0][c], U[1][c], U[2][c]};
    double v[3], g[3];
    fwd(kTL, in, v);
    fwd(kTD, in, g);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      S[c * kFS + xo + xs * q] = v[q];
      S[(3 + c) * kFS + xo + xs * q] = g[q];
    }
  }
  wsync();
  // the pressure (temperature) at the z-pencil's two end levels, read before
  // the forward y pass reuses P's slab (DCP_MF_LDS_ALIAS)
  double Plo = 0.0, Phi = 0.0;
  if (STOKES || RHS) {
    const double xa = sel3(pa, kGaussX[0], kGaussX[1], kGaussX[2]);
    const double xb = sel3(pb, kGaussX[0], kGaussX[1], kGaussX[2]);
    Plo = (1.0 - xb) * ((1.0 - xa) * P[0] + xa * P[1]) + xb * ((1.0 - xa) * P[2] + xa * P[3]);
    Phi = (1.0 - xb) * ((1.0 - xa) * P[4] + xa * P[5]) + xb * ((1.0 - xa) * P[6] + xa * P[7]);
  }
  {
    double A[3][3], B[3][3], C[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {  // y: A = value, B = d/dxi1, C = d/dxi0
      double v[3], g[3];
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        v[b] = SR[c * kFS + yo + ys * b];
        g[b] = SR[(3 + c) * kFS + yo + ys * b];
      }
      fwd(kTL, v, A[c]);
      fwd(kTD, v, B[c]);
      fwd(kTL, g, C[c]);
    }
    wsync();
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        S[c * kFS + yo + ys * q] = A[c][q];
        S[(3 + c) * kFS + yo + ys * q] = B[c][q];
        S[(6 + c) * kFS + yo + ys * q] = C[c][q];
      }
  }
  wsync();

  // separable geometry: the z-pencil's 2D table entry and the cell's radii
  // (small, L2-resident tables)
  double m[10], lg[9];
  if (SEP) {
    const double* cg = mc.colgeo + 90 * size_t(colc) + 10 * p;
#pragma unroll
    for (int i = 0; i < 10; ++i) m[i] = cg[i];
    const double* lp = mc.laygeo + 9 * size_t(layc);
#pragma unroll
    for (int i = 0; i < 9; ++i) lg[i] = lp[i];
  }
  // ---- z-pencil: per point flux, accumulated straight into the back z pass
  double V[3][3], FX[3][3], FY[3][3];  // [c][node along z]
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int k = 0; k < 3; ++k) V[c][k] = FX[c][k] = FY[c][k] = 0.0;
  double slo = 0.0, shi = 0.0;
  // RHS: Phi of the lane's column point, the gravity factor per point
  double rphi[3] = {0, 0, 0}, rR[3] = {0, 0, 0};
  if (RHS && SEP && !ph.cuboid) {
#pragma unroll
    for (int d = 0; d < 3; ++d) rphi[d] = mc.colphi[27 * size_t(colc) + 3 * p + d];
    // -g R / den(R |Phi|): -g / |Phi| where R |Phi| > 1, else -g sqrt(R) / sqrt|Phi|
    const double* pn = mc.colphin + 27 * size_t(colc) + 3 * p;
    const double am = pn[0], ai = pn[1], asi = pn[2];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const double R = mc.layR[3 * size_t(layc) + q];
      rR[q] = R * am > 1 ? -ph.g * ai : -ph.g * mc.layRs[3 * size_t(layc) + q] * asi;
    }
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    double u[3], Gh[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double A[3], B[3], C[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        // re-read per point (volatile view): holding the 27 values across
        // the point loop costs an occupancy step (194 VGPRs), 154 -> 160 us
        A[k] = SR[c * kFS + zo + 9 * k];
        B[k] = SR[(3 + c) * kFS + zo + 9 * k];
        C[k] = SR[(6 + c) * kFS + zo + 9 * k];
      }
      u[c] = kTL.v[0][q] * A[0] + kTL.v[1][q] * A[1] + kTL.v[2][q] * A[2];
      Gh[c][0] = kTL.v[0][q] * C[0] + kTL.v[1][q] * C[1] + kTL.v[2][q] * C[2];
      Gh[c][1] = kTL.v[0][q] * B[0] + kTL.v[1][q] * B[1] + kTL.v[2][q] * B[2];
      Gh[c][2] = kTD.v[0][q] * A[0] + kTD.v[1][q] * A[1] + kTD.v[2][q] * A[2];
    }
    double ji[9], wq;
    if (SEP) {  // rows m0 / R, m1 / R, m2 / R'; JxW = R^2 R' D2 w
      const double iR = lg[3 * q], iRp = lg[3 * q + 1];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        ji[d] = m[d] * iR;
        ji[3 + d] = m[3 + d] * iR;
        ji[6 + d] = m[6 + d] * iRp;
      }
      wq = lg[3 * q + 2] * m[9] * (wab * kGaussW[q]);
    } else {
#pragma unroll
      for (int i = 0; i < 9; ++i) ji[i] = Ji[q][i];
      wq = w[q];
    }
    if (RHS) {
      rhs_flux(ph, u, Gh, ji, wq, (1.0 - kGaussX[q]) * Plo + kGaussX[q] * Phi, rR[q], rphi, q, V);
      continue;
    }
#ifndef DCP_MF_NOZMATH
#define DCP_MF_NOZMATH 0
#endif
    if (DCP_MF_NOZMATH) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          V[c][k] += u[c] * wq;
          FX[c][k] += Gh[c][0];
          FY[c][k] += Gh[c][1] + Gh[c][2] * ji[k];
        }
      continue;
    }
    double G[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int d = 0; d < 3; ++d)
        G[c][d] = Gh[c][0] * ji[d] + Gh[c][1] * ji[3 + d] + Gh[c][2] * ji[6 + d];
    double F[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int d = 0; d < 3; ++d) F[c][d] = nu * (G[c][d] + G[d][c]);
    if (STOKES) {
      const double pq = (1.0 - kGaussX[q]) * Plo + kGaussX[q] * Phi;
      F[0][0] -= pq;
      F[1][1] -= pq;
      F[2][2] -= pq;
      const double sq = -wq * (G[0][0] + G[1][1] + G[2][2]);
      slo += (1.0 - kGaussX[q]) * sq;
      shi += kGaussX[q] * sq;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const double r0 = wq * (ji[0] * F[c][0] + ji[1] * F[c][1] + ji[2] * F[c][2]);
      const double r1 = wq * (ji[3] * F[c][0] + ji[4] * F[c][1] + ji[5] * F[c][2]);
      const double r2 = wq * (ji[6] * F[c][0] + ji[7] * F[c][1] + ji[8] * F[c][2]);
      const double wu = wq * u[c];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        V[c][k] += kTL.v[k][q] * wu + kTD.v[k][q] * r2;
        FX[c][k] += kTL.v[k][q] * r0;
        FY[c][k] += kTL.v[k][q] * r1;
      }
    }
  }
  wsync();
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      S[c * kFS + zo + 9 * k] = V[c][k];
      if (!RHS) {
        S[(3 + c) * kFS + zo + 9 * k] = FX[c][k];
        S[(6 + c) * kFS + zo + 9 * k] = FY[c][k];
      }
    }
  if (STOKES && !DCP_MF_LDS_ALIAS) {
    SP[p] = slo;
    SP[9 + p] = shi;
  }
  wsync();

  // ---- back y (y-pencil), the pressure test functions
  double yp = 0.0;
  auto pressure_test = [&] {
    if (STOKES && p < 8) {
      const int v0 = p & 1, v1 = (p >> 1) & 1, v2 = p >> 2;
      const double* s = SP + 9 * v2;
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const double pb1 = v1 ? kGaussX[b] : 1.0 - kGaussX[b];
        double r = 0.0;
#pragma unroll
        for (int a = 0; a < 3; ++a) r += (v0 ? kGaussX[a] : 1.0 - kGaussX[a]) * s[a + 3 * b];
        yp += pb1 * r;
      }
    }
  };
  {
    double V1[3][3], FX1[3][3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      double v[3], fx[3], fy[3], t[3];
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        v[b] = SR[c * kFS + yo + ys * b];
        fx[b] = RHS ? 0.0 : SR[(3 + c) * kFS + yo + ys * b];
        fy[b] = RHS ? 0.0 : SR[(6 + c) * kFS + yo + ys * b];
      }
      bwd(kTL, v, V1[c]);
      if (!RHS) {
        bwd(kTD, fy, t);
#pragma unroll
        for (int n = 0; n < 3; ++n) V1[c][n] += t[n];
        bwd(kTL, fx, FX1[c]);
      }
    }
    if (!DCP_MF_LDS_ALIAS) pressure_test();
    wsync();
    if (STOKES && DCP_MF_LDS_ALIAS) {  // field 6 is dead now (FY read above)
      SP[p] = slo;
      SP[9 + p] = shi;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
      for (int n = 0; n < 3; ++n) {
        S[c * kFS + yo + ys * n] = V1[c][n];
        if (!RHS) S[(3 + c) * kFS + yo + ys * n] = FX1[c][n];
      }
  }
  wsync();
  if (DCP_MF_LDS_ALIAS) pressure_test();

  // ---- back x (x-pencil) and the cell record
  double y[3][3];  // [node a][c]
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    double v[3], fx[3], t0[3], t1[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      v[q] = SR[c * kFS + xo + xs * q];
      fx[q] = RHS ? 0.0 : SR[(3 + c) * kFS + xo + xs * q];
    }
    bwd(kTL, v, t0);
    if (RHS) {
#pragma unroll
      for (int n = 0; n < 3; ++n) y[n][c] = t0[n];
    } else {
      bwd(kTD, fx, t1);
#pragma unroll
      for (int n = 0; n < 3; ++n) y[n][c] = t0[n] + t1[n];
    }
  }
  // (timing probes only, wrong results: DCP_MF_NOSTORE skips the cell
  // records, DCP_MF_NOZMATH the per-point flux of the z-pencil)
#ifndef DCP_MF_NOSTORE
#define DCP_MF_NOSTORE 0
#endif
  // group partial sums: every occurrence parks its triple (fields 0-2) and its
  // chain link; the owner (first occurrence of the node in the group) adds the
  // chained ones in (cell, t) order and stores one triple per node and group
  wsync();  // every lane has read its back-x inputs
#pragma unroll
  for (int n = 0; n < 3; ++n) {
#pragma unroll
    for (int c = 0; c < 3; ++c) S[c * kFS + xo + xs * n] = y[n][c];
    if (cs < kPenCells) nxt(27 * (kPenCells * wave + cs) + 3 * p + n) = MfLink(Ic.next[n]);
  }
  // the group spans the workgroup's waves: their records are read across waves
  if (kPenWaves > 1)
    __syncthreads();
  else
    wsync();
  if (live && !DCP_MF_NOSTORE) {
#pragma unroll
    for (int n = 0; n < 3; ++n) {
      if (Ic.slot[n] < 0) continue;  // not the node's first occurrence in the group
      double s0 = y[n][0], s1 = y[n][1], s2 = y[n][2];
      // links point forward inside the group (at most kMfGroupCells - 1 hops)
      int k = Ic.next[n];
      for (int hop = 0; k != kMfLinkEnd && hop < kMfGroupCells; ++hop, k = nxt(k)) {
        const int ck = k / 27, tk = k - 27 * ck;
        const int wk = ck / kPenCells, sk = ck - kPenCells * wk;  // wave and cell slot
        const int ak = tk % 3, bk = (tk / 3) % 3, zk = tk / 9;
        const int idx = (DCP_MF_FIELD_MAJOR ? 27 : 243) * sk +
                        (DCP_MF_SWAP_AB ? 3 * ak + bk + 9 * zk : tk);
        const double* Sw = lds[wk];
        s0 += Sw[idx];
        s1 += Sw[kFS + idx];
        s2 += Sw[2 * kFS + idx];
      }
      double* out = buf + Ic.slot[n];
      rec_store(out, s0, FUSED);
      rec_store(out + 1, s1, FUSED);
      rec_store(out + 2, s2, FUSED);
    }
    if (STOKES && p < 8) rec_store(buf + Ic.pslot, yp, FUSED);
  }
  // the next batch overwrites the slabs this one just read
  if (kPenWaves > 1)
    __syncthreads();
  else
    wsync();
  Ic = In;
  In = Inn;
  if (DCP_MF_PREFETCH_NODES) Nc = Nn;
  }
  if (FUSED) {
    // every record store of the batch acknowledged, then its flag
    // (release: the record stores are ordered before the flag by the memory
    // model, not only by this wait)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (kPenWaves > 1) __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(done + blk, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

#ifndef DCP_MF_XCD
#define DCP_MF_XCD 1
#endif
template <bool STOKES, bool SEP, bool RHS = false>
__global__ __launch_bounds__(64 * kPenWaves, DCP_MF_WAVES_PER_EU)
void k_mf_pencil(MfCells mc, int c0, int c1, double nu, const double* __restrict__ src,
                 double* __restrict__ buf, double* __restrict__ dst,
                 const double* __restrict__ T_old, PhysicsDev ph) {
  __shared__ double lds[kPenWaves][kPenFields];
  const int blk = DCP_MF_XCD ? xcd_block(blockIdx.x, gridDim.x) : int(blockIdx.x);
  pencil_body<STOKES, SEP, RHS, false>(mc, blk, c0, c1, nu, src, buf, dst, T_old, ph, lds, nullptr,
                                       0);
}

// Every dof sums its contiguous run of slots in slot (= ascending cell) order,
// then C^T and the constrained diagonal. One wave per 64 consecutive dofs: the
// runs of those dofs form one contiguous span, which the wave loads
// cooperatively (coalesced) into LDS; each lane then adds its own run.
#ifndef DCP_MF_GWAVES
#define DCP_MF_GWAVES 4
#endif
constexpr int kGatherWaves = DCP_MF_GWAVES;
#ifndef DCP_MF_GSPAN
#define DCP_MF_GSPAN 512  // 64 nodes x ~2.1 wave partials x 3 (r=5: 768 -> 512, 34.8 -> 32.0 us)
#endif
constexpr int kGvSpan = DCP_MF_GSPAN;  // doubles per wave window (longer spans: direct reads)
// Gather wave w (velocity windows first, then pressure windows); W: the
// wave's LDS window (kGvSpan doubles). FUSED: records read agent-coherent.
// the wave's record window into LDS: DCP_MF_WIN_UNROLL (default) issues all of
// a lane's window loads (kGvSpan / 64 of them, clamped to the window) before
// the LDS writes, instead of one load-wait-write per loop trip (r=5 Stokes
// apply 156.6-160.9 -> 152.8-153.0 us in tools/mf_probe.py, bitwise;
// profiles/r05/r05af_mf_window_variants.log)
#ifndef DCP_MF_WIN_UNROLL
#define DCP_MF_WIN_UNROLL 1
#endif
template <bool FUSED>
__device__ __forceinline__ void load_window(const double* __restrict__ b, int len, double* W,
                                            int lane) {
  if (DCP_MF_WIN_UNROLL) {
    if (len <= 0) return;
    constexpr int U = kGvSpan / 64;
    double t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = rec_load(b + min(lane + 64 * u, len - 1), FUSED);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (lane + 64 * u < len) W[lane + 64 * u] = t[u];
  } else {
    for (int i = lane; i < len; i += 64) W[i] = rec_load(b + i, FUSED);
  }
}

template <bool STOKES, bool FUSED>
__device__ __forceinline__ void gather_body(const MfGather& g, int w, int v0, int v1, int p0,
                                            int p1, const double* __restrict__ buf,
                                            const double* __restrict__ src,
                                            double* __restrict__ dst, double* W) {
  const int lane = threadIdx.x & 63;
  const int nvw = (v1 - v0 + 63) >> 6;
  if (w < nvw) {
    const int n0 = v0 + 64 * w, n1 = min(n0 + 64, v1);  // gather positions
    const int s0 = g.vptr[n0];
    const int len = 3 * (g.vptr[n1] - s0);
    const double* b = buf + 3 * size_t(s0);
    const bool fits = len <= kGvSpan;
    if (fits) load_window<FUSED>(b, len, W, lane);
    wsync();
    const int pos = n0 + lane;
    if (pos >= n1) return;
    const int i = g.vorder ? g.vorder[pos] : pos;
    const int k0 = g.vptr[pos] - s0, k1 = g.vptr[pos + 1] - s0;
    double s[3] = {0.0, 0.0, 0.0};
    if (fits) {
      for (int k = k0; k < k1; ++k) {
        s[0] += W[3 * k];
        s[1] += W[3 * k + 1];
        s[2] += W[3 * k + 2];
      }
    } else {
      for (int k = k0; k < k1; ++k) {
        s[0] += rec_load(b + 3 * k, FUSED);
        s[1] += rec_load(b + 3 * k + 1, FUSED);
        s[2] += rec_load(b + 3 * k + 2, FUSED);
      }
    }
    // the cidx lookup only where the wave's positions hold a constrained node
    const bool maybe = !g.wcon || g.wcon[n0 >> 6] || g.wcon[(n1 - 1) >> 6];
    const int ci = maybe ? g.cidx[i] : -1;
    if (ci >= 0) {
      const NodeConstraint nc = g.vcon[i];
      condense(nc, s);
      if (g.cdiag) {  // operator rows (null: the rhs, condensation only)
        const double* dg = g.cdiag + 3 * size_t(ci);
#pragma unroll
        for (int comp = 0; comp < 3; ++comp)
          if (nc.type == 1 || nc.type == 3 || comp == nc.k)
            s[comp] = dg[comp] * src[3 * size_t(i) + comp];
      }
    }
    double* d = dst + 3 * size_t(i);
    d[0] = s[0];
    d[1] = s[1];
    d[2] = s[2];
  } else if (STOKES) {
    const int j0 = p0 + 64 * (w - nvw);
    if (j0 >= p1) return;
    const int j1 = min(j0 + 64, p1);
    const int s0 = g.pptr[j0];
    const int len = g.pptr[j1] - s0;
    const double* b = buf + g.pbase + s0;
    const bool fits = len <= kGvSpan;
    if (fits) load_window<FUSED>(b, len, W, lane);
    wsync();
    const int pos = j0 + lane;
    if (pos >= j1) return;
    const int j = g.porder ? g.porder[pos] : pos;
    const int k0 = g.pptr[pos] - s0, k1 = g.pptr[pos + 1] - s0;
    double s = 0.0;
    if (fits)
      for (int k = k0; k < k1; ++k) s += W[k];
    else
      for (int k = k0; k < k1; ++k) s += rec_load(b + k, FUSED);
    if (g.pcidx && g.pcidx[j] >= 0) s = g.pcdiag[g.pcidx[j]] * src[g.n_u + j];  // periodic image
    dst[g.n_u + j] = s;
  }
}

template <bool STOKES>
__global__ __launch_bounds__(64 * kGatherWaves) void k_mf_gather(MfGather g, int v0, int v1,
                                                                  int p0, int p1,
                                                                  const double* __restrict__ buf,
                                                                  const double* __restrict__ src,
                                                                  double* __restrict__ dst) {
  __shared__ double win[kGatherWaves][kGvSpan];
  const int wave = threadIdx.x >> 6;
  gather_body<STOKES, false>(g, int(blockIdx.x) * kGatherWaves + wave, v0, v1, p0, p1, buf, src,
                             dst, win[wave]);
}

// One launch for the whole apply (DCP_MF_FUSED): pencil batches and gather
// windows in one grid, in the order of the schedule built at upload
// (api.cpp): every gather window after all the batches that write its
// records. A gather task polls those batches' done flags (agent-coherent,
// tag = this apply's seq) before it reads. It waits only on tasks of lower
// workgroup ids, and an XCD dispatches its workgroups in id order, so the
// lowest unfinished task always has its inputs: no deadlock whatever the
// residency. A poll that exceeds the spin bound raises f.err (host-mapped)
// and reads anyway; the host then refuses the result. The same sums in the
// same order as the two launches: bitwise their result.
static_assert(kPenWaves == 1 && kMfBatches == 1, "k_mf_fused: one-wave pencil batches");
static_assert(kGvSpan <= kPenFields, "the gather window aliases the pencil slab");
template <bool STOKES, bool SEP, bool RHS>
__global__ __launch_bounds__(64, DCP_MF_WAVES_PER_EU) void k_mf_fused(
    MfCells mc, MfGather g, MfFused f, double nu, const double* __restrict__ src,
    double* __restrict__ buf, double* __restrict__ dst, unsigned seq,
    const double* __restrict__ T_old, PhysicsDev ph) {
  __shared__ double lds[1][kPenFields];
  const int task = f.sched[blockIdx.x];
  const int kind = (task >> 30) & 3, idx = task & 0x3fffffff;
  if (kind == 0) {
    pencil_body<STOKES, SEP, RHS, true>(mc, idx, 0, mc.n_cells, nu, src, buf, dst, T_old, ph,
                                        lds, f.done, seq);
    return;
  }
  // padding; pressure windows of a velocity-only pass (A x, the rhs)
  if (kind == 3 || (kind == 2 && !STOKES)) return;
  const int lane = threadIdx.x & 63;
  const int win = kind == 1 ? idx : f.n_vwin + idx;
  const int d0 = f.dep_ptr[win], d1 = f.dep_ptr[win + 1];
  bool late = false;
  for (int i = d0 + lane; i < d1; i += 64) {
    const unsigned* flag = f.done + f.dep[i];
    long spins = 0;
    while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != seq) {
      if (++spins > f.spin_limit) {
        late = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // acquire for the whole wave: every lane's polled flags happen-before the
  // window reads of gather_body, whichever lane observed them
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (__any(late) && lane == 0) *f.err = 1.0;
  gather_body<STOKES, true>(g, kind == 1 ? idx : ((g.n_vnodes + 63) >> 6) + idx, 0, g.n_vnodes, 0,
                            g.n_p, buf, src, dst, lds[0]);
}

// constrained velocity dofs: dst = (assembled diagonal) * src
__global__ void k_mf_constrained(int n, const int32_t* __restrict__ dof,
                                 const int64_t* __restrict__ diag_pos,
                                 const double* __restrict__ cdiag, const double* __restrict__ src,
                                 double* __restrict__ dst) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < n) dst[dof[e]] = cdiag[diag_pos[e]] * src[dof[e]];
}

}  // namespace

void mf_geometry(const CellData& cd, const int32_t* order, double* geo, hipStream_t s) {
  if (cd.n_cells <= 0) return;
  hipLaunchKernelGGL(k_mf_geometry, dim3((cd.n_cells + kGeoCells - 1) / kGeoCells), dim3(256), 0, s,
                     cd, order, geo);
  DCP_HIP_CHECK(hipGetLastError());
}

void mf_apply_colour(const MfData& md, int base, int n, double nu, bool stokes,
                     const double* src, double* dst, hipStream_t s) {
  if (n <= 0) return;
  const dim3 grid((n + kMfCells - 1) / kMfCells);
  if (stokes)
    hipLaunchKernelGGL(k_mf_stokes<true>, grid, dim3(32 * kMfCells), 0, s, md, base, n, nu, src,
                       dst);
  else
    hipLaunchKernelGGL(k_mf_stokes<false>, grid, dim3(32 * kMfCells), 0, s, md, base, n, nu, src,
                       dst);
  DCP_HIP_CHECK(hipGetLastError());
}

void mf_cells(const MfCells& mc, int c0, int c1, double nu, bool stokes, const double* src,
              double* buf, double* dst, hipStream_t s) {
  if (c1 <= c0) return;
  const dim3 grid((kMfBatchTotal(c1 - c0) + kMfBatches - 1) / kMfBatches);
#ifndef DCP_MF_SEP
#define DCP_MF_SEP 1
#endif
  const bool sep = DCP_MF_SEP && mc.col != nullptr;
  auto k = stokes ? (sep ? k_mf_pencil<true, true> : k_mf_pencil<true, false>)
                  : (sep ? k_mf_pencil<false, true> : k_mf_pencil<false, false>);
  hipLaunchKernelGGL(k, grid, dim3(64 * kPenWaves), 0, s, mc, c0, c1, nu, src, buf, dst, nullptr,
                     PhysicsDev{});
  DCP_HIP_CHECK(hipGetLastError());
}

void mf_rhs_cells(const MfCells& mc, int c0, int c1, const double* u_old, const double* T_old,
                  const PhysicsDev& ph, double* buf, double* rhs, hipStream_t s) {
  if (c1 <= c0) return;
  const dim3 grid((kMfBatchTotal(c1 - c0) + kMfBatches - 1) / kMfBatches);
  const bool sep = DCP_MF_SEP && mc.col != nullptr;
  auto k = sep ? k_mf_pencil<false, true, true> : k_mf_pencil<false, false, true>;
  hipLaunchKernelGGL(k, grid, dim3(64 * kPenWaves), 0, s, mc, c0, c1, 0.0, u_old, buf, rhs, T_old,
                     ph);
  DCP_HIP_CHECK(hipGetLastError());
}

void mf_gather(const MfGather& mg, int v0, int v1, int p0, int p1, bool stokes, const double* buf,
               const double* src, double* dst, hipStream_t s) {
  const int waves = (v1 - v0 + 63) / 64 + (stokes ? (p1 - p0 + 63) / 64 : 0);
  if (waves <= 0) return;
  const dim3 grid((waves + kGatherWaves - 1) / kGatherWaves), block(64 * kGatherWaves);
  if (stokes)
    hipLaunchKernelGGL(k_mf_gather<true>, grid, block, 0, s, mg, v0, v1, p0, p1, buf, src, dst);
  else
    hipLaunchKernelGGL(k_mf_gather<false>, grid, block, 0, s, mg, v0, v1, p0, p1, buf, src, dst);
  DCP_HIP_CHECK(hipGetLastError());
}

void mf_fused(const MfCells& mc, const MfGather& mg, const MfFused& f, int n_tasks, double nu,
              bool stokes, const double* src, double* buf, double* dst, unsigned seq,
              hipStream_t s) {
  if (n_tasks <= 0) return;
  const bool sep = DCP_MF_SEP && mc.col != nullptr;
  auto k = stokes ? (sep ? k_mf_fused<true, true, false> : k_mf_fused<true, false, false>)
                  : (sep ? k_mf_fused<false, true, false> : k_mf_fused<false, false, false>);
  hipLaunchKernelGGL(k, dim3(n_tasks), dim3(64), 0, s, mc, mg, f, nu, src, buf, dst, seq, nullptr,
                     PhysicsDev{});
  DCP_HIP_CHECK(hipGetLastError());
}

void mf_rhs_fused(const MfCells& mc, const MfGather& mg, const MfFused& f, int n_tasks,
                  const double* u_old, const double* T_old, const PhysicsDev& ph, double* buf,
                  double* rhs, unsigned seq, hipStream_t s) {
  if (n_tasks <= 0) return;
  const bool sep = DCP_MF_SEP && mc.col != nullptr;
  auto k = sep ? k_mf_fused<false, true, true> : k_mf_fused<false, false, true>;
  hipLaunchKernelGGL(k, dim3(n_tasks), dim3(64), 0, s, mc, mg, f, 0.0, u_old, buf, rhs, seq, T_old,
                     ph);
  DCP_HIP_CHECK(hipGetLastError());
}

void mf_constrained(int n, const int32_t* dof, const int64_t* diag_pos, const double* cdiag,
                    const double* src, double* dst, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_mf_constrained, dim3((n + 255) / 256), dim3(256), 0, s, n, dof, diag_pos,
                     cdiag, src, dst);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
