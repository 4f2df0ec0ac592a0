// Two-dimensional model, Standard::BoussinesqModel<2> (boussinesq_model.inst.cc:8,
// data/aqua_planet_test_2d.prm), hand-written HIP for gfx950, FP64.
//
//   k2d_nse_system     local_assemble_nse_system at dim = 2 (boussinesq_model.tpp:
//                      550-673, QGauss(3), the 2D Coriolis term -2 phi . cross_product_2d(u))
//                      + copy_local_to_global_nse_system (:677-687)
//   k2d_precond_diag   local_assemble_nse_preconditioner (:421-464), condensed diagonal
//   k2d_T_matrix       local_assemble_temperature_matrix (:748-800), QGauss(deg + 2)
//   k2d_T_rhs          local_assemble_temperature_rhs (:873-952) with the matrix_for_bc lift
//   k2d_vel_stats      get_maximal_velocity / get_cfl_number (:1023-1101)
//   k2d_distribute     AffineConstraints::distribute of the NSE lines
//
// One 64-lane wavefront per cell (colour launches: no two cells of a launch
// share a support point, so the scatter needs no atomics). Lanes 0..Q-1
// evaluate the MappingQ(3) map and the physical Q2 / Q1 shape functions at one
// quadrature point each into LDS; every lane then sums ~8 of the 22 x 22
// local entries over the points. Local dofs: FESystem(FE_Q(2)^2, FE_Q(1)):
// 3 per vertex (u_x u_y p), 2 per line, 2 interior.
//
// Constraints are node-local (no-slip: both components fixed; no-normal-flux:
// u_k = w u_other at the same support point), so the condensation C^T K C of
// AffineConstraints::distribute_local_to_global stays inside the cell: local
// dof a receives the row / column of at most one constrained local dof
// src[a] with weight srcw[a] (model2d.cpp builds the table).
#include <hip/hip_runtime.h>

#include "../device.h"

namespace dcp {
namespace {

__constant__ double cGX3[3] = {0.11270166537925831148, 0.5, 0.88729833462074168852};
__constant__ double cGW3[3] = {0.27777777777777777778, 0.44444444444444444444,
                               0.27777777777777777778};
__constant__ double cGX4[4] = {0.069431844202973712388, 0.33000947820757186760,
                               0.66999052179242813240, 0.93056815579702628761};
__constant__ double cGW4[4] = {0.17392742256872692869, 0.32607257743127307131,
                               0.32607257743127307131, 0.17392742256872692869};
__constant__ double cGL[4] = {0.0, 0.27639320225002103036, 0.72360679774997896964, 1.0};
// FE_Q(2) hierarchic -> lexicographic (a + 3 b)
__constant__ int cH2L[9] = {0, 2, 6, 8, 3, 5, 1, 7, 4};

__device__ inline double lag1(int i, double x) { return i ? x : 1.0 - x; }
__device__ inline double dlag1(int i) { return i ? 1.0 : -1.0; }
__device__ inline double lag2(int i, double x) {
  return i == 0 ? 2.0 * (x - 0.5) * (x - 1.0) : i == 1 ? -4.0 * x * (x - 1.0) : 2.0 * x * (x - 0.5);
}
__device__ inline double dlag2(int i, double x) {
  return i == 0 ? 4.0 * x - 3.0 : i == 1 ? -8.0 * x + 4.0 : 4.0 * x - 1.0;
}
__device__ inline double lag3(int i, double x) {
  double v = 1.0;
  for (int j = 0; j < 4; ++j)
    if (j != i) v *= (x - cGL[j]) / (cGL[i] - cGL[j]);
  return v;
}
__device__ inline double dlag3(int i, double x) {
  double s = 0.0;
  for (int k = 0; k < 4; ++k) {
    if (k == i) continue;
    double v = 1.0 / (cGL[i] - cGL[k]);
    for (int j = 0; j < 4; ++j)
      if (j != i && j != k) v *= (x - cGL[j]) / (cGL[i] - cGL[j]);
    s += v;
  }
  return s;
}

// local dof -> component (0, 1 velocity, 2 pressure) and lexicographic point / vertex
__device__ inline void sysdof2d(int i, int& comp, int& idx) {
  if (i < 12) {
    comp = i % 3;
    idx = comp == 2 ? i / 3 : cH2L[i / 3];
  } else if (i < 20) {
    comp = (i - 12) % 2;
    idx = cH2L[4 + (i - 12) / 2];
  } else {
    comp = i - 20;
    idx = 4;
  }
}

// MappingQ(3) at xi: position, inverse Jacobian, determinant
__device__ inline void map2d(const double* X, const double xi[2], double x[2], double Ji[2][2],
                             double& det) {
  double J[2][2] = {{0, 0}, {0, 0}};
  x[0] = x[1] = 0;
  double l0[4], l1[4], d0[4], d1[4];
  for (int a = 0; a < 4; ++a) {
    l0[a] = lag3(a, xi[0]);
    l1[a] = lag3(a, xi[1]);
    d0[a] = dlag3(a, xi[0]);
    d1[a] = dlag3(a, xi[1]);
  }
  for (int t = 0; t < 16; ++t) {
    const int a = t & 3, b = t >> 2;
    const double s = l0[a] * l1[b], g0 = d0[a] * l1[b], g1 = l0[a] * d1[b];
    for (int i = 0; i < 2; ++i) {
      const double Xi = X[2 * t + i];
      x[i] += Xi * s;
      J[i][0] += Xi * g0;
      J[i][1] += Xi * g1;
    }
  }
  det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
  const double id = 1.0 / det;
  Ji[0][0] = J[1][1] * id;
  Ji[0][1] = -J[0][1] * id;
  Ji[1][0] = -J[1][0] * id;
  Ji[1][1] = J[0][0] * id;
}

struct Smem2D {
  double X[32];
  double uloc[22];
  double Tloc[9];
  double v2[9][9], g2[9][9][2], v1[9][4];  // [q][node]
  double JxW[9];
  double F[9][2];     // rhs integrand (times JxW) at q: f_i = phi_i . F_q
  double K[22][22];
  double f[22];
  double diag[22];
  int dof[22];
  int src[22];
  double srcw[22];
  int fixed[22];
};

__device__ inline double nse_entry(const Smem2D& sh, int i, int j, double nu_dt) {
  int ci, ai, cj, aj;
  sysdof2d(i, ci, ai);
  sysdof2d(j, cj, aj);
  double s = 0;
  if (ci < 2 && cj < 2) {
    for (int q = 0; q < 9; ++q) {
      const double* ga = sh.g2[q][ai];
      const double* gb = sh.g2[q][aj];
      double v = 0.5 * (ga[cj] * gb[ci]);
      double mass = 0;
      if (ci == cj) {
        v += 0.5 * (ga[0] * gb[0] + ga[1] * gb[1]);
        mass = sh.v2[q][ai] * sh.v2[q][aj];
      }
      s += (mass + nu_dt * 2.0 * v) * sh.JxW[q];
    }
  } else if (ci < 2 && cj == 2) {
    for (int q = 0; q < 9; ++q) s -= sh.g2[q][ai][ci] * sh.v1[q][aj] * sh.JxW[q];
  } else if (ci == 2 && cj < 2) {
    for (int q = 0; q < 9; ++q) s -= sh.v1[q][ai] * sh.g2[q][aj][cj] * sh.JxW[q];
  }
  return s;
}

__device__ inline double pre_entry(const Smem2D& sh, int i, int j, double nu_dt) {
  int ci, ai, cj, aj;
  sysdof2d(i, ci, ai);
  sysdof2d(j, cj, aj);
  double s = 0;
  if (ci < 2 && ci == cj) {
    for (int q = 0; q < 9; ++q) {
      const double* ga = sh.g2[q][ai];
      const double* gb = sh.g2[q][aj];
      s += (sh.v2[q][ai] * sh.v2[q][aj] + nu_dt * (ga[0] * gb[0] + ga[1] * gb[1])) * sh.JxW[q];
    }
  } else if (ci == 2 && cj == 2) {
    for (int q = 0; q < 9; ++q) s += sh.v1[q][ai] * sh.v1[q][aj] * sh.JxW[q];
  }
  return s;
}

__device__ inline void load_cell(Smem2D& sh, const Mesh2DDev& m, int cell, const double* old_nse,
                                 const double* old_T, int tid) {
  if (tid < 32) sh.X[tid] = m.X[32 * size_t(cell) + tid];
  if (tid < 22) {
    const int d = m.dofs[22 * size_t(cell) + tid];
    sh.dof[tid] = d;
    sh.uloc[tid] = old_nse ? old_nse[d] : 0.0;
    sh.src[tid] = m.src[22 * size_t(cell) + tid];
    sh.srcw[tid] = m.srcw[22 * size_t(cell) + tid];
    sh.fixed[tid] = m.fixed[22 * size_t(cell) + tid];
  }
  if (tid >= 32 && tid < 32 + m.tdpc)
    sh.Tloc[tid - 32] = old_T ? old_T[m.tdofs[size_t(m.tdpc) * cell + tid - 32]] : 0.0;
}

// shape functions at QGauss(3) point q (+ the rhs integrand)
__device__ inline void eval_point(Smem2D& sh, const Mesh2DDev& m, const PhysicsDev& ph, int q,
                                  bool rhs) {
  const double xi[2] = {cGX3[q % 3], cGX3[q / 3]};
  double x[2], Ji[2][2], det;
  map2d(sh.X, xi, x, Ji, det);
  const double jxw = det * cGW3[q % 3] * cGW3[q / 3];
  sh.JxW[q] = jxw;
  for (int n = 0; n < 9; ++n) {
    const int a = n % 3, b = n / 3;
    sh.v2[q][n] = lag2(a, xi[0]) * lag2(b, xi[1]);
    const double r0 = dlag2(a, xi[0]) * lag2(b, xi[1]), r1 = lag2(a, xi[0]) * dlag2(b, xi[1]);
    sh.g2[q][n][0] = r0 * Ji[0][0] + r1 * Ji[1][0];
    sh.g2[q][n][1] = r0 * Ji[0][1] + r1 * Ji[1][1];
  }
  for (int n = 0; n < 4; ++n) sh.v1[q][n] = lag1(n & 1, xi[0]) * lag1(n >> 1, xi[1]);
  if (!rhs) return;
  // old velocity, its gradient and the old temperature (dof-order sums)
  double u[2] = {0, 0}, G[2][2] = {{0, 0}, {0, 0}};
  for (int k = 0; k < 22; ++k) {
    int c, a;
    sysdof2d(k, c, a);
    if (c == 2) continue;
    u[c] += sh.uloc[k] * sh.v2[q][a];
    G[c][0] += sh.uloc[k] * sh.g2[q][a][0];
    G[c][1] += sh.uloc[k] * sh.g2[q][a][1];
  }
  double T = 0;
  if (m.tdpc == 4) {
    for (int k = 0; k < 4; ++k) T += sh.Tloc[k] * sh.v1[q][k];
  } else {
    for (int k = 0; k < 9; ++k) T += sh.Tloc[k] * sh.v2[q][cH2L[k]];
  }
  const double rho = 1 - ph.beta * (T - ph.T_ref);
  double adv[2];
  for (int j = 0; j < 2; ++j) adv[j] = u[0] * G[j][0] + u[1] * G[j][1];
  double grav[2];
  if (ph.cuboid) {
    grav[0] = 0;
    grav[1] = -ph.g;
  } else {
    const double r = sqrt(x[0] * x[0] + x[1] * x[1]);
    const double den = r > 1 ? r : sqrt(r);
    grav[0] = -ph.g * x[0] / den;
    grav[1] = -ph.g * x[1] / den;
  }
  // -dt * (-2 phi . cross_product_2d(u)), cross_product_2d(u) = (u_y, -u_x)
  const double cu[2] = {u[1], -u[0]};
  for (int d = 0; d < 2; ++d)
    sh.F[q][d] = (u[d] + ph.dt * rho * ph.grav_scale * grav[d] - ph.dt * adv[d] +
                  ph.dt * 2.0 * cu[d]) *
                 jxw;
}

// MODE 0: condensed scatter into the CSR + rhs (colour launch);
// MODE 1: dense element output K[22][22], f[22] of cells [first, first + n).
template <int MODE>
__global__ __launch_bounds__(64) void k2d_nse_system(Mesh2DDev m, const int32_t* __restrict__ cells,
                                                     int first, const double* __restrict__ old_nse,
                                                     const double* __restrict__ old_T,
                                                     PhysicsDev ph, double* __restrict__ A,
                                                     double* __restrict__ rhs,
                                                     double* __restrict__ elemK,
                                                     double* __restrict__ elemF) {
  __shared__ Smem2D sh;
  const int tid = threadIdx.x;
  const int cell = MODE == 0 ? cells[blockIdx.x] : first + blockIdx.x;
  load_cell(sh, m, cell, old_nse, old_T, tid);
  __syncthreads();
  if (tid < 9) eval_point(sh, m, ph, tid, true);
  __syncthreads();
  for (int e = tid; e < 484; e += 64) {
    const int i = e / 22, j = e % 22;
    const double k = nse_entry(sh, i, j, ph.nu_sys);
    sh.K[i][j] = k;
    if (MODE == 1) elemK[484 * size_t(blockIdx.x) + e] = k;
  }
  if (tid < 22) {
    int c, a;
    sysdof2d(tid, c, a);
    double f = 0;
    if (c < 2)
      for (int q = 0; q < 9; ++q) f += sh.v2[q][a] * sh.F[q][c];
    sh.f[tid] = f;
    if (MODE == 1) elemF[22 * size_t(blockIdx.x) + tid] = f;
  }
  if (MODE == 1) return;
  __syncthreads();
  if (tid < 22) sh.diag[tid] = fabs(sh.K[tid][tid]);
  __syncthreads();
  double avg = 0;
  for (int k = 0; k < 22; ++k) avg += sh.diag[k];
  avg /= 22.0;
  for (int e = tid; A && e < 484; e += 64) {
    const int a = e / 22, b = e % 22;
    const int p = m.pos[484 * size_t(cell) + e];
    if (sh.fixed[a] || sh.fixed[b]) {
      // constrained row / column: only the diagonal, |K_aa| or the mean (:677-687)
      if (a == b && p >= 0) A[p] += sh.diag[a] != 0.0 ? sh.diag[a] : avg;
      continue;
    }
    if (p < 0) continue;
    const int sa = sh.src[a], sb = sh.src[b];
    double k = sh.K[a][b];
    if (sa >= 0) k += sh.srcw[a] * sh.K[sa][b];
    if (sb >= 0) k += sh.srcw[b] * sh.K[a][sb];
    if (sa >= 0 && sb >= 0) k += sh.srcw[a] * sh.srcw[b] * sh.K[sa][sb];
    A[p] += k;
  }
  if (tid < 22 && rhs && !sh.fixed[tid]) {
    double f = sh.f[tid];
    if (sh.src[tid] >= 0) f += sh.srcw[tid] * sh.f[sh.src[tid]];
    rhs[sh.dof[tid]] += f;
  }
}

// condensed diagonals of the preconditioner blocks (point Jacobi of P(0,0), P(1,1))
__global__ __launch_bounds__(64) void k2d_precond_diag(Mesh2DDev m, const int32_t* __restrict__ cells,
                                                       PhysicsDev ph, double* __restrict__ Ad,
                                                       double* __restrict__ Mpd) {
  __shared__ Smem2D sh;
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  load_cell(sh, m, cell, nullptr, nullptr, tid);
  __syncthreads();
  if (tid < 9) eval_point(sh, m, ph, tid, false);
  __syncthreads();
  if (tid < 22) sh.diag[tid] = pre_entry(sh, tid, tid, ph.nu_pre);
  __syncthreads();
  if (tid >= 22) return;
  const int a = tid;
  const int d = sh.dof[a];
  double v;
  if (sh.fixed[a]) {
    double avg = 0;
    for (int k = 0; k < 22; ++k) avg += fabs(sh.diag[k]);
    avg /= 22.0;
    v = sh.diag[a] != 0.0 ? fabs(sh.diag[a]) : avg;
  } else {
    v = sh.diag[a];
    const int s = sh.src[a];
    if (s >= 0) {
      const double w = sh.srcw[a];
      v += 2.0 * w * pre_entry(sh, s, a, ph.nu_pre) + w * w * sh.diag[s];
    }
  }
  if (d < m.n_u) Ad[d] += v;
  else Mpd[d - m.n_u] += v;
}

// temperature shape function k (FE_Q local order) at point q of an n1 x n1 rule
struct TShape {
  double v[9], g[9][2];
};
__device__ inline void t_shapes(int tdpc, const double xi[2], const double Ji[2][2], TShape& s) {
  if (tdpc == 4) {
    for (int k = 0; k < 4; ++k) {
      const int a = k & 1, b = k >> 1;
      s.v[k] = lag1(a, xi[0]) * lag1(b, xi[1]);
      const double r0 = dlag1(a) * lag1(b, xi[1]), r1 = lag1(a, xi[0]) * dlag1(b);
      s.g[k][0] = r0 * Ji[0][0] + r1 * Ji[1][0];
      s.g[k][1] = r0 * Ji[0][1] + r1 * Ji[1][1];
    }
  } else {
    for (int k = 0; k < 9; ++k) {
      const int n = cH2L[k], a = n % 3, b = n / 3;
      s.v[k] = lag2(a, xi[0]) * lag2(b, xi[1]);
      const double r0 = dlag2(a, xi[0]) * lag2(b, xi[1]), r1 = lag2(a, xi[0]) * dlag2(b, xi[1]);
      s.g[k][0] = r0 * Ji[0][0] + r1 * Ji[1][0];
      s.g[k][1] = r0 * Ji[0][1] + r1 * Ji[1][1];
    }
  }
}

struct SmemT {
  double X[32];
  double Tloc[9];
  double uloc[22];
  double v[16][9], g[16][9][2], JxW[16];
  double Tq[16], Fq[16];
  double dM[9], dK[9];
  int tdof[9];
  int fixed[9];
};

__device__ inline void t_points(SmemT& sh, const Mesh2DDev& m, int q, int n1) {
  const double* gx = n1 == 3 ? cGX3 : cGX4;
  const double* gw = n1 == 3 ? cGW3 : cGW4;
  const double xi[2] = {gx[q % n1], gx[q / n1]};
  double x[2], Ji[2][2], det;
  map2d(sh.X, xi, x, Ji, det);
  sh.JxW[q] = det * gw[q % n1] * gw[q / n1];
  TShape s;
  t_shapes(m.tdpc, xi, Ji, s);
  for (int k = 0; k < m.tdpc; ++k) {
    sh.v[q][k] = s.v[k];
    sh.g[q][k][0] = s.g[k][0];
    sh.g[q][k][1] = s.g[k][1];
  }
}

// mass + stiffness (1/Pe) matrices, QGauss(deg + 2), scattered with the
// constrained-diagonal rule of distribute_local_to_global (separately per matrix)
__global__ __launch_bounds__(64) void k2d_T_matrix(Mesh2DDev m, const int32_t* __restrict__ cells,
                                                   PhysicsDev ph, double* __restrict__ Mg,
                                                   double* __restrict__ Kg) {
  __shared__ SmemT sh;
  const int tid = threadIdx.x, n = m.tdpc, n1 = n == 4 ? 3 : 4, nq = n1 * n1;
  const int cell = cells[blockIdx.x];
  if (tid < 32) sh.X[tid] = m.X[32 * size_t(cell) + tid];
  if (tid >= 32 && tid < 32 + n) {
    const int d = m.tdofs[size_t(n) * cell + tid - 32];
    sh.tdof[tid - 32] = d;
    sh.fixed[tid - 32] = m.T_fixed[d];
  }
  __syncthreads();
  if (tid < nq) t_points(sh, m, tid, n1);
  __syncthreads();
  auto entry = [&](int i, int j, double& mm, double& kk) {
    mm = kk = 0;
    for (int q = 0; q < nq; ++q) {
      mm += sh.v[q][i] * sh.v[q][j] * sh.JxW[q];
      kk += (sh.g[q][i][0] * sh.g[q][j][0] + sh.g[q][i][1] * sh.g[q][j][1]) * ph.one_over_peclet *
            sh.JxW[q];
    }
  };
  if (tid < n) {
    double mm, kk;
    entry(tid, tid, mm, kk);
    sh.dM[tid] = fabs(mm);
    sh.dK[tid] = fabs(kk);
  }
  __syncthreads();
  double aM = 0, aK = 0;
  for (int k = 0; k < n; ++k) {
    aM += sh.dM[k];
    aK += sh.dK[k];
  }
  aM /= n;
  aK /= n;
  for (int e = tid; e < n * n; e += 64) {
    const int i = e / n, j = e % n;
    const int p = m.posT[size_t(n) * n * cell + e];
    if (sh.fixed[i] || sh.fixed[j]) {
      if (i == j && p >= 0) {
        Mg[p] += sh.dM[i] != 0.0 ? sh.dM[i] : aM;
        Kg[p] += sh.dK[i] != 0.0 ? sh.dK[i] : aK;
      }
      continue;
    }
    if (p < 0) continue;
    double mm, kk;
    entry(i, j, mm, kk);
    Mg[p] += mm;
    Kg[p] += kk;
  }
}

// temperature rhs: (phi T - dt_T phi u . grad T) JxW on unconstrained dofs, minus
// the matrix_for_bc columns of the Dirichlet dofs (distribute_local_to_global
// with the local matrix, :1003-1012)
__global__ __launch_bounds__(64) void k2d_T_rhs(Mesh2DDev m, const int32_t* __restrict__ cells,
                                                const double* __restrict__ T_old,
                                                const double* __restrict__ nse, PhysicsDev ph,
                                                double* __restrict__ rhs) {
  __shared__ SmemT sh;
  const int tid = threadIdx.x, n = m.tdpc, n1 = n == 4 ? 3 : 4, nq = n1 * n1;
  const int cell = cells[blockIdx.x];
  if (tid < 32) sh.X[tid] = m.X[32 * size_t(cell) + tid];
  if (tid >= 32 && tid < 32 + n) {
    const int d = m.tdofs[size_t(n) * cell + tid - 32];
    sh.tdof[tid - 32] = d;
    sh.fixed[tid - 32] = m.T_fixed[d];
    sh.Tloc[tid - 32] = T_old[d];
  }
  if (tid >= 42 && tid < 64) sh.uloc[tid - 42] = nse[m.dofs[22 * size_t(cell) + tid - 42]];
  __syncthreads();
  if (tid < nq) {
    const int q = tid;
    t_points(sh, m, q, n1);
    // velocity from the Q2 nodal values at this point
    const double* gx = n1 == 3 ? cGX3 : cGX4;
    const double xi[2] = {gx[q % n1], gx[q / n1]};
    double u[2] = {0, 0};
    for (int k = 0; k < 22; ++k) {
      int c, a;
      sysdof2d(k, c, a);
      if (c == 2) continue;
      u[c] += sh.uloc[k] * lag2(a % 3, xi[0]) * lag2(a / 3, xi[1]);
    }
    double T = 0, gT[2] = {0, 0};
    for (int k = 0; k < n; ++k) {
      T += sh.Tloc[k] * sh.v[q][k];
      gT[0] += sh.Tloc[k] * sh.g[q][k][0];
      gT[1] += sh.Tloc[k] * sh.g[q][k][1];
    }
    sh.Tq[q] = T * sh.JxW[q];
    sh.Fq[q] = ph.dt_T * (u[0] * gT[0] + u[1] * gT[1]) * sh.JxW[q];
  }
  __syncthreads();
  if (tid >= n) return;
  const int j = tid;
  if (sh.fixed[j]) return;
  double f = 0;
  for (int q = 0; q < nq; ++q) f += sh.v[q][j] * (sh.Tq[q] - sh.Fq[q]);
  for (int i = 0; i < n; ++i) {
    if (!sh.fixed[i]) continue;
    const double g = m.T_bc[sh.tdof[i]];
    if (g == 0.0) continue;
    double mb = 0;
    for (int q = 0; q < nq; ++q)
      mb += (sh.v[q][i] * sh.v[q][j] +
             ph.dt_T * ph.one_over_peclet *
                 (sh.g[q][i][0] * sh.g[q][j][0] + sh.g[q][i][1] * sh.g[q][j][1])) *
            sh.JxW[q];
    f -= g * mb;
  }
  rhs[sh.tdof[j]] += f;
}

__device__ inline void atomic_max_nonneg(double* addr, double v) {
  atomicMax(reinterpret_cast<unsigned long long*>(addr), __double_as_longlong(v));
}

// max |u| and max over cells of max(1e-10, max |u|) / diameter on the 9 Q2
// support points (QIterated<QTrapez>(2))
__global__ __launch_bounds__(256) void k2d_vel_stats(Mesh2DDev m, const double* __restrict__ nse,
                                                     double* out2) {
  const long cell = long(blockIdx.x) * 256 + threadIdx.x;
  double mx = 0, cfl = 0;
  if (cell < m.n_cells) {
    const int32_t* d = m.dofs + 22 * cell;
    double cm = 1e-10;
    for (int t = 0; t < 9; ++t) {
      const int k = t < 4 ? 3 * t : 12 + 2 * (t - 4);
      const double ux = nse[d[k]], uy = nse[d[k + 1]];
      const double s = sqrt(ux * ux + uy * uy);
      mx = fmax(mx, s);
      cm = fmax(cm, s);
    }
    cfl = cm / m.diameter[cell];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mx = fmax(mx, __shfl_xor(mx, off, 64));
    cfl = fmax(cfl, __shfl_xor(cfl, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomic_max_nonneg(&out2[0], mx);
    atomic_max_nonneg(&out2[1], cfl);
  }
}

// x_i = sum_k w_k x_t(k) + g_i for every constrained line (targets unconstrained)
__global__ void k2d_distribute(int n_lines, const int32_t* __restrict__ line_dof,
                               const int32_t* __restrict__ ptr, const int32_t* __restrict__ ent,
                               const double* __restrict__ w, const double* __restrict__ inhom,
                               double* x) {
  const int l = blockIdx.x * 256 + threadIdx.x;
  if (l >= n_lines) return;
  double v = inhom[l];
  for (int k = ptr[l]; k < ptr[l + 1]; ++k) v += w[k] * x[ent[k]];
  x[line_dof[l]] = v;
}

// scatter positions of the local entries into a sorted CSR (-1: absent)
__global__ void k2d_positions(int n_cells, int dpc, const int32_t* __restrict__ dofs,
                              const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
                              int32_t* __restrict__ pos) {
  const long t = long(blockIdx.x) * 256 + threadIdx.x;
  const long per = long(dpc) * dpc;
  if (t >= long(n_cells) * per) return;
  const long cell = t / per;
  const int e = int(t % per), i = e / dpc, j = e % dpc;
  const int r = dofs[dpc * cell + i], c = dofs[dpc * cell + j];
  int b = ptr[r], en = ptr[r + 1];
  while (b < en) {
    const int mid = (b + en) >> 1;
    if (col[mid] < c) b = mid + 1;
    else en = mid;
  }
  pos[t] = (b < ptr[r + 1] && col[b] == c) ? b : -1;
}

}  // namespace

void launch2d_nse_system(const Mesh2DDev& m, const int32_t* cells, int n, const double* old_nse,
                         const double* old_T, const PhysicsDev& ph, double* A, double* rhs,
                         hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL((k2d_nse_system<0>), dim3(n), dim3(64), 0, s, m, cells, 0, old_nse, old_T, ph, A,
                     rhs, nullptr, nullptr);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch2d_nse_elements(const Mesh2DDev& m, int first, int n, const double* old_nse,
                           const double* old_T, const PhysicsDev& ph, double* K, double* f,
                           hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL((k2d_nse_system<1>), dim3(n), dim3(64), 0, s, m, nullptr, first, old_nse, old_T,
                     ph, nullptr, nullptr, K, f);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch2d_precond_diag(const Mesh2DDev& m, const int32_t* cells, int n, const PhysicsDev& ph,
                           double* Ad, double* Mpd, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k2d_precond_diag, dim3(n), dim3(64), 0, s, m, cells, ph, Ad, Mpd);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch2d_T_matrix(const Mesh2DDev& m, const int32_t* cells, int n, const PhysicsDev& ph,
                       double* M, double* K, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k2d_T_matrix, dim3(n), dim3(64), 0, s, m, cells, ph, M, K);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch2d_T_rhs(const Mesh2DDev& m, const int32_t* cells, int n, const double* T_old,
                    const double* nse, const PhysicsDev& ph, double* rhs, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k2d_T_rhs, dim3(n), dim3(64), 0, s, m, cells, T_old, nse, ph, rhs);
  DCP_HIP_CHECK(hipGetLastError());
}

void velocity_stats_2d(const Mesh2DDev& m, const double* nse, double* out2, hipStream_t s) {
  DCP_HIP_CHECK(hipMemsetAsync(out2, 0, 2 * sizeof(double), s));
  if (m.n_cells <= 0) return;
  hipLaunchKernelGGL(k2d_vel_stats, dim3((m.n_cells + 255) / 256), dim3(256), 0, s, m, nse, out2);
  DCP_HIP_CHECK(hipGetLastError());
}

void distribute_2d(int n_lines, const int32_t* line_dof, const int32_t* ptr, const int32_t* ent,
                   const double* w, const double* inhom, double* x, hipStream_t s) {
  if (n_lines <= 0) return;
  hipLaunchKernelGGL(k2d_distribute, dim3((n_lines + 255) / 256), dim3(256), 0, s, n_lines, line_dof,
                     ptr, ent, w, inhom, x);
  DCP_HIP_CHECK(hipGetLastError());
}

void positions_2d(int n_cells, int dpc, const int32_t* dofs, const int32_t* ptr, const int32_t* col,
                  int32_t* pos, hipStream_t s) {
  const long t = long(n_cells) * dpc * dpc;
  if (t <= 0) return;
  hipLaunchKernelGGL(k2d_positions, dim3((t + 255) / 256), dim3(256), 0, s, n_cells, dpc, dofs, ptr,
                     col, pos);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
