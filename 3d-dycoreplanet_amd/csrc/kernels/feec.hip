// FEEC variant of the assembly (ExteriorCalculus::BoussinesqModel<3>, config 4),
// hand-written HIP for gfx950, FP64.
//
//   k_feec_system      local_assemble_nse_system   boussineq_model_FEEC.tpp:669-808
//                      + distribute_local_to_global :812-820
//   k_feec_precond     local_assemble_nse_preconditioner :509-572 (Q14 integrand)
//   k_feec_T_rhs       local_assemble_temperature_rhs (velocity from the RT field)
//   k_feec_vel_stats   get_maximal_velocity / get_cfl_number on QIterated(QTrapez, 2)
//
// One 64-lane wavefront per cell: lanes 0..Q-1 evaluate the mapping (MappingQ1,
// as the FEEC scratch has no mapping argument: boussineq_model_assembly_FEEC.tpp:67)
// and the 19 physical shape functions at one quadrature point each into LDS,
// then every lane sums ~6 of the 19x19 local entries over the points.
// Local DoFs: 0..11 Nedelec (edges, deal.II line order), 12..17 Raviart-
// Thomas (faces), 18 DGQ0. Covariant Piola for Nedelec (phi = J^-T N,
// curl phi = J curl N / det J), contravariant for RT (phi = J R / det J,
// div phi = div R / det J).
#include <hip/hip_runtime.h>

#include "../feec.h"

namespace dcp {
namespace {

constexpr double kG2[2] = {0.21132486540518711775, 0.78867513459481288225};  // QGauss(2)

__device__ inline double lin(int s, double t) { return s ? t : 1.0 - t; }
__device__ inline double dlin(int s) { return s ? 1.0 : -1.0; }

// line -> (axis, transverse b, transverse c, side on b, side on c)
__constant__ int cLine[12][5] = {{1, 0, 2, 0, 0}, {1, 0, 2, 1, 0}, {0, 1, 2, 0, 0}, {0, 1, 2, 1, 0},
                                 {1, 0, 2, 0, 1}, {1, 0, 2, 1, 1}, {0, 1, 2, 0, 1}, {0, 1, 2, 1, 1},
                                 {2, 0, 1, 0, 0}, {2, 0, 1, 1, 0}, {2, 0, 1, 0, 1}, {2, 0, 1, 1, 1}};

// MappingQ1 at xi: position, Jacobian, its inverse and determinant
__device__ inline void q1_map(const double* X, const double xi[3], double x[3], double J[3][3],
                              double Ji[3][3], double& det) {
  for (int i = 0; i < 3; ++i) {
    x[i] = 0;
    J[i][0] = J[i][1] = J[i][2] = 0;
  }
  for (int v = 0; v < 8; ++v) {
    const int a = v & 1, b = (v >> 1) & 1, c = v >> 2;
    const double la = lin(a, xi[0]), lb = lin(b, xi[1]), lc = lin(c, xi[2]);
    const double N = la * lb * lc;
    const double d0 = dlin(a) * lb * lc, d1 = la * dlin(b) * lc, d2 = la * lb * dlin(c);
    for (int i = 0; i < 3; ++i) {
      const double Xi = X[3 * v + i];
      x[i] += Xi * N;
      J[i][0] += Xi * d0;
      J[i][1] += Xi * d1;
      J[i][2] += Xi * d2;
    }
  }
  const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
  const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
  const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
  det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
  const double id = 1.0 / det;
  Ji[0][0] = c00 * id;
  Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * id;
  Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * id;
  Ji[1][0] = c01 * id;
  Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * id;
  Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * id;
  Ji[2][0] = c02 * id;
  Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * id;
  Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * id;
}

// physical Nedelec value/curl of line l (sign applied)
__device__ inline void nedelec(int l, double sg, const double xi[3], const double J[3][3],
                               const double Ji[3][3], double det, double v[3], double c[3]) {
  const int a = cLine[l][0], b = cLine[l][1], cc = cLine[l][2], sb = cLine[l][3], sc = cLine[l][4];
  const double g = lin(sb, xi[b]) * lin(sc, xi[cc]);
  double gg[3] = {0, 0, 0};  // reference gradient of g
  gg[b] = dlin(sb) * lin(sc, xi[cc]);
  gg[cc] = lin(sb, xi[b]) * dlin(sc);
  // reference value N = g e_a, reference curl = grad g x e_a
  double rc[3];
  rc[0] = gg[1] * (a == 2) - gg[2] * (a == 1);
  rc[1] = gg[2] * (a == 0) - gg[0] * (a == 2);
  rc[2] = gg[0] * (a == 1) - gg[1] * (a == 0);
  for (int i = 0; i < 3; ++i) {
    v[i] = sg * Ji[a][i] * g;  // (J^-T N)_i = sum_j Ji[j][i] N_j
    c[i] = sg * (J[i][0] * rc[0] + J[i][1] * rc[1] + J[i][2] * rc[2]) / det;
  }
}

// physical RT value/divergence of face f (sign applied)
__device__ inline void raviart_thomas(int f, double sg, const double xi[3], const double J[3][3],
                                      double det, double v[3], double& dv) {
  const int a = f / 2, s = f % 2;
  const double r = lin(s, xi[a]);
  for (int i = 0; i < 3; ++i) v[i] = sg * J[i][a] * r / det;
  dv = sg * dlin(s) / det;
}

__device__ inline double dot3(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

struct FeecSmem {
  double X[24];
  double sg[19];
  double dofv[19];     // old w/u coefficients
  double Tn[8];
  double PW[27][12][3], CW[27][12][3], PU[27][6][3], DU[27][6];
  double JxW[27];
  double F[27][3], G[27];   // rhs: phi_u . F_q + div phi_u G_q
  double diag[19];
  int dof[19];
  int fixed[19];
};

// local matrix entry (i, j) of local_assemble_nse_system (FEEC.tpp:753-769)
__device__ inline double feec_entry(const FeecSmem& sh, int nq, int i, int j, double nu_dt) {
  const int ti = i < 12 ? 0 : i < 18 ? 1 : 2, tj = j < 12 ? 0 : j < 18 ? 1 : 2;
  double s = 0;
  for (int q = 0; q < nq; ++q) {
    double v = 0;
    if (ti == 0 && tj == 0) v = dot3(sh.PW[q][i], sh.PW[q][j]);                        // mass_w
    else if (ti == 0 && tj == 1) v = -dot3(sh.CW[q][i], sh.PU[q][j - 12]);             // -curl w . u
    else if (ti == 1 && tj == 1) v = dot3(sh.PU[q][i - 12], sh.PU[q][j - 12]);         // mass_u
    else if (ti == 1 && tj == 0) v = nu_dt * dot3(sh.PU[q][i - 12], sh.CW[q][j]);      // dt/Re u . curl w
    else if (ti == 1 && tj == 2) v = -sh.DU[q][i - 12];                                 // -div u p
    else if (ti == 2 && tj == 1) v = -sh.DU[q][j - 12];                                 // -q div u
    s += v * sh.JxW[q];
  }
  return s;
}

// Q14 indicator: +-1 by the sign of v when |v| > 1e-9, else 0
__device__ inline double ind(double v) {
  return fabs(v) > 1.0e-9 ? -2 * ((signbit(v) ? 1.0 : 0.0) - 0.5) : 0.0;
}

// preconditioner entry (FEEC.tpp:550-569): only phi_p phi_p carries JxW
__device__ inline double feec_pre_entry(const FeecSmem& sh, int nq, int i, int j, double nu_dt) {
  const int ti = i < 12 ? 0 : i < 18 ? 1 : 2, tj = j < 12 ? 0 : j < 18 ? 1 : 2;
  double s = 0;
  for (int q = 0; q < nq; ++q) {
    double v = 0;
    if (ti == 0 && tj == 0) v += nu_dt * dot3(sh.CW[q][i], sh.CW[q][j]);
    if (ti == 1 && tj == 0) v += ind(dot3(sh.PU[q][i - 12], sh.PW[q][j]));
    if (ti == 0 && tj == 1) v += ind(dot3(sh.PW[q][i], sh.PU[q][j - 12]));
    if (ti == 2 && tj == 2) v += sh.JxW[q];
    s += v;
  }
  return s;
}

// lanes < nq: shape functions + rhs integrand at point q
template <int NQ1>
__device__ inline void eval_point(FeecSmem& sh, const FeecCellData& cd, const PhysicsDev& ph,
                                  int q, bool rhs) {
  const double* g1 = NQ1 == 3 ? kGaussX : kG2;
  const double* w1 = NQ1 == 3 ? kGaussW : nullptr;
  const int qa = q % NQ1, qb = (q / NQ1) % NQ1, qc = q / (NQ1 * NQ1);
  const double xi[3] = {g1[qa], g1[qb], g1[qc]};
  const double wq = NQ1 == 3 ? w1[qa] * w1[qb] * w1[qc] : 0.125;
  double x[3], J[3][3], Ji[3][3], det;
  q1_map(sh.X, xi, x, J, Ji, det);
  sh.JxW[q] = det * wq;
  for (int l = 0; l < 12; ++l) nedelec(l, sh.sg[l], xi, J, Ji, det, sh.PW[q][l], sh.CW[q][l]);
  for (int f = 0; f < 6; ++f) raviart_thomas(f, sh.sg[12 + f], xi, J, det, sh.PU[q][f], sh.DU[q][f]);
  if (!rhs) return;
  double u[3] = {0, 0, 0}, w[3] = {0, 0, 0};
  for (int l = 0; l < 12; ++l)
    for (int i = 0; i < 3; ++i) w[i] += sh.dofv[l] * sh.PW[q][l][i];
  for (int f = 0; f < 6; ++f)
    for (int i = 0; i < 3; ++i) u[i] += sh.dofv[12 + f] * sh.PU[q][f][i];
  double T = 0;
  for (int v = 0; v < 8; ++v)
    T += sh.Tn[v] * lin(v & 1, xi[0]) * lin((v >> 1) & 1, xi[1]) * lin(v >> 2, xi[2]);
  const double rho = 1 - ph.beta * (T - ph.T_ref);  // density_scaling
  double grav[3];
  if (ph.cuboid) {
    grav[0] = grav[1] = 0;
    grav[2] = -ph.g;
  } else {
    const double r = sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
    const double den = r > 1 ? r : sqrt(r);
    for (int d = 0; d < 3; ++d) grav[d] = -ph.g * x[d] / den;
  }
  const double wxu[3] = {w[1] * u[2] - w[2] * u[1], w[2] * u[0] - w[0] * u[2],
                         w[0] * u[1] - w[1] * u[0]};
  const double cxu[3] = {-ph.coriolis_z * u[1], ph.coriolis_z * u[0], 0.0};  // Omega x u (Q2)
  for (int d = 0; d < 3; ++d)
    sh.F[q][d] = (u[d] + ph.dt * rho * ph.grav_scale * grav[d] - ph.dt * wxu[d] -
                  ph.dt * 2 * cxu[d]) * sh.JxW[q];
  sh.G[q] = -ph.dt * 0.5 * dot3(u, u) * sh.JxW[q];
}

__device__ inline void load_cell(FeecSmem& sh, const FeecCellData& cd, int cell,
                                 const double* __restrict__ old_nse, const double* __restrict__ T_old,
                                 int tid) {
  if (tid < 24) sh.X[tid] = cd.X[24 * size_t(cell) + tid];
  if (tid < 19) {
    const int d = cd.cell_dofs[19 * size_t(cell) + tid];
    sh.dof[tid] = d;
    sh.sg[tid] = cd.sign[19 * size_t(cell) + tid];
    sh.fixed[tid] = cd.fixed[d];
    sh.dofv[tid] = old_nse ? old_nse[d] : 0.0;
  }
  if (tid >= 32 && tid < 40 && T_old) sh.Tn[tid - 32] = T_old[cd.cell_T[8 * size_t(cell) + tid - 32]];
}

// MODE 0: condensed scatter into the CSR (colour launch, no atomics);
// MODE 1: dense element output K[19][19], f[19] of cells [first, first+n).
template <int MODE>
__global__ __launch_bounds__(64) void k_feec_system(FeecCellData cd, const int32_t* __restrict__ cells,
                                                    int first, const int32_t* __restrict__ pos,
                                                    const double* __restrict__ old_nse,
                                                    const double* __restrict__ T_old, PhysicsDev ph,
                                                    double* __restrict__ A, double* __restrict__ rhs,
                                                    double* __restrict__ elemK,
                                                    double* __restrict__ elemF) {
  __shared__ FeecSmem sh;
  const int tid = threadIdx.x;
  const int cell = MODE == 0 ? cells[blockIdx.x] : first + blockIdx.x;
  load_cell(sh, cd, cell, old_nse, T_old, tid);
  __syncthreads();
  if (tid < 27) eval_point<3>(sh, cd, ph, tid, true);
  __syncthreads();
  if (tid < 19) sh.diag[tid] = fabs(feec_entry(sh, 27, tid, tid, ph.nu_sys));
  __syncthreads();
  double avg = 0;
  for (int k = 0; k < 19; ++k) avg += sh.diag[k];
  avg /= 19.0;
  for (int e = tid; e < 361; e += 64) {
    const int i = e / 19, j = e % 19;
    double k = feec_entry(sh, 27, i, j, ph.nu_sys);
    if (MODE == 1) {
      elemK[361 * size_t(blockIdx.x) + e] = k;
      continue;
    }
    if (sh.fixed[i] || sh.fixed[j]) {
      if (i != j) continue;
      k = sh.diag[i] != 0.0 ? sh.diag[i] : avg;  // constrained diagonal: |K_ii| or the mean
    }
    const int p = pos[361 * size_t(cell) + e];
    if (p >= 0) A[p] += k;
  }
  if (tid < 19) {
    double f = 0;
    if (tid >= 12 && tid < 18)
      for (int q = 0; q < 27; ++q) f += dot3(sh.PU[q][tid - 12], sh.F[q]) + sh.DU[q][tid - 12] * sh.G[q];
    if (MODE == 1) elemF[19 * size_t(blockIdx.x) + tid] = f;
    else if (rhs && !sh.fixed[tid]) rhs[sh.dof[tid]] += f;
  }
}

// preconditioner matrix (QGauss(deg+1) = QGauss(2), FEEC.tpp:611)
__global__ __launch_bounds__(64) void k_feec_precond(FeecCellData cd, const int32_t* __restrict__ cells,
                                                     const int32_t* __restrict__ pos, PhysicsDev ph,
                                                     double* __restrict__ P) {
  __shared__ FeecSmem sh;
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  load_cell(sh, cd, cell, nullptr, nullptr, tid);
  __syncthreads();
  if (tid < 8) eval_point<2>(sh, cd, ph, tid, false);
  __syncthreads();
  if (tid < 19) sh.diag[tid] = fabs(feec_pre_entry(sh, 8, tid, tid, ph.nu_sys));
  __syncthreads();
  double avg = 0;
  for (int k = 0; k < 19; ++k) avg += sh.diag[k];
  avg /= 19.0;
  for (int e = tid; e < 361; e += 64) {
    const int i = e / 19, j = e % 19;
    double k = feec_pre_entry(sh, 8, i, j, ph.nu_sys);
    if (sh.fixed[i] || sh.fixed[j]) {
      if (i != j) continue;
      k = sh.diag[i] != 0.0 ? sh.diag[i] : avg;
    }
    const int p = pos[361 * size_t(cell) + e];
    if (p >= 0) P[p] += k;
  }
}

// temperature rhs with the RT velocity of nse_solution (Q5) and the
// matrix_for_bc lift; MappingQ1, QGauss(T_degree + 2) = QGauss(3)
__global__ __launch_bounds__(64) void k_feec_T_rhs(FeecCellData cd, const int32_t* __restrict__ cells,
                                                   const double* __restrict__ T_old,
                                                   const double* __restrict__ nse, PhysicsDev ph,
                                                   const uint8_t* __restrict__ T_fixed,
                                                   const double* __restrict__ T_bc, double* rhs) {
  __shared__ FeecSmem sh;
  __shared__ double GT[27][8][3], ST[27][8];
  __shared__ double Tq[27], Fq[27];
  __shared__ int tdof[8];
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  load_cell(sh, cd, cell, nse, T_old, tid);
  if (tid >= 40 && tid < 48) tdof[tid - 40] = cd.cell_T[8 * size_t(cell) + tid - 40];
  __syncthreads();
  if (tid < 27) {
    const int q = tid;
    const double xi[3] = {kGaussX[q % 3], kGaussX[(q / 3) % 3], kGaussX[q / 9]};
    double x[3], J[3][3], Ji[3][3], det;
    q1_map(sh.X, xi, x, J, Ji, det);
    const double jxw = det * kGaussW[q % 3] * kGaussW[(q / 3) % 3] * kGaussW[q / 9];
    double u[3] = {0, 0, 0};
    for (int f = 0; f < 6; ++f) {
      double v[3], dv;
      raviart_thomas(f, sh.sg[12 + f], xi, J, det, v, dv);
      for (int i = 0; i < 3; ++i) u[i] += sh.dofv[12 + f] * v[i];
    }
    double T = 0, gT[3] = {0, 0, 0};
    for (int v = 0; v < 8; ++v) {
      const int a = v & 1, b = (v >> 1) & 1, c = v >> 2;
      const double la = lin(a, xi[0]), lb = lin(b, xi[1]), lc = lin(c, xi[2]);
      const double r[3] = {dlin(a) * lb * lc, la * dlin(b) * lc, la * lb * dlin(c)};
      ST[q][v] = la * lb * lc;
      for (int i = 0; i < 3; ++i) GT[q][v][i] = Ji[0][i] * r[0] + Ji[1][i] * r[1] + Ji[2][i] * r[2];
      T += sh.Tn[v] * ST[q][v];
      for (int i = 0; i < 3; ++i) gT[i] += sh.Tn[v] * GT[q][v][i];
    }
    sh.JxW[q] = jxw;
    Tq[q] = T * jxw;
    Fq[q] = ph.dt_T * dot3(u, gT) * jxw;
  }
  __syncthreads();
  if (tid < 8) {
    const int j = tid;
    if (T_fixed[tdof[j]]) return;
    double f = 0;
    for (int q = 0; q < 27; ++q) f += ST[q][j] * (Tq[q] - Fq[q]);
    for (int i = 0; i < 8; ++i) {
      if (!T_fixed[tdof[i]]) continue;
      const double g = T_bc[tdof[i]];
      if (g == 0.0) continue;
      double mb = 0;
      for (int q = 0; q < 27; ++q)
        mb += (ST[q][i] * ST[q][j] + ph.dt_T * ph.one_over_peclet * dot3(GT[q][i], GT[q][j])) *
              sh.JxW[q];
      f -= g * mb;
    }
    rhs[tdof[j]] += f;
  }
}

// max |u| and max over cells of max(1e-10, max |u|) / diameter on the 27 points
// of QIterated(QTrapez, nse_velocity_degree + 1) = {0, 1/2, 1}^3 (FEEC.tpp:1134-1180)
__device__ inline void atomic_max_nonneg(double* addr, double v) {
  atomicMax(reinterpret_cast<unsigned long long*>(addr), __double_as_longlong(v));
}

__global__ __launch_bounds__(256) void k_feec_vel_stats(FeecCellData cd, int n_cells,
                                                        const double* __restrict__ nse,
                                                        double* out2) {
  const long cell = long(blockIdx.x) * 256 + threadIdx.x;
  double mx = 0, cfl = 0;
  if (cell < n_cells) {
    const double* X = cd.X + 24 * size_t(cell);
    double uf[6], sg[6];
    for (int f = 0; f < 6; ++f) {
      uf[f] = nse[cd.cell_dofs[19 * size_t(cell) + 12 + f]];
      sg[f] = cd.sign[19 * size_t(cell) + 12 + f];
    }
    double cm = 1e-10;
    for (int q = 0; q < 27; ++q) {
      const double xi[3] = {0.5 * (q % 3), 0.5 * ((q / 3) % 3), 0.5 * (q / 9)};
      double x[3], J[3][3], Ji[3][3], det;
      q1_map(X, xi, x, J, Ji, det);
      double u[3] = {0, 0, 0};
      for (int f = 0; f < 6; ++f) {
        double v[3], dv;
        raviart_thomas(f, sg[f], xi, J, det, v, dv);
        for (int i = 0; i < 3; ++i) u[i] += uf[f] * v[i];
      }
      const double n = sqrt(dot3(u, u));
      mx = fmax(mx, n);
      cm = fmax(cm, n);
    }
    cfl = cm / cd.diameter[cell];
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

// per-cell weight of compute_mean_value(QGauss(1)) on MappingQ1: det J at the centre
// per cell the JxW sum of compute_mean_value's quadrature on the MappingQ1
// cell: QGauss(1) (npt = 1: det J at the centre, the nested Schur correction) or
// QGauss(2) (npt = 2: the exact volume, PreconditionerBlockIdentity)
__global__ void k_feec_cell_weights(FeecCellData cd, int n_cells, double* w, int npt) {
  const long cell = long(blockIdx.x) * 256 + threadIdx.x;
  if (cell >= n_cells) return;
  double x[3], J[3][3], Ji[3][3], det;
  if (npt == 1) {
    const double xi[3] = {0.5, 0.5, 0.5};
    q1_map(cd.X + 24 * size_t(cell), xi, x, J, Ji, det);
    w[cell] = det;
    return;
  }
  const double g[2] = {0.5 - 0.5 / sqrt(3.0), 0.5 + 0.5 / sqrt(3.0)};
  double s = 0.0;
  for (int q = 0; q < 8; ++q) {
    const double xi[3] = {g[q & 1], g[(q >> 1) & 1], g[q >> 2]};
    q1_map(cd.X + 24 * size_t(cell), xi, x, J, Ji, det);
    s += det * 0.125;
  }
  w[cell] = s;
}

// scatter positions of the 19x19 local entries into a sorted CSR (-1: absent)
__global__ void k_feec_positions(FeecCellData cd, int n_cells, const int32_t* __restrict__ ptr,
                                 const int32_t* __restrict__ col, int32_t* __restrict__ pos) {
  const long t = long(blockIdx.x) * 256 + threadIdx.x;
  if (t >= long(n_cells) * 361) return;
  const long cell = t / 361;
  const int e = int(t % 361), i = e / 19, j = e % 19;
  const int r = cd.cell_dofs[19 * cell + i], c = cd.cell_dofs[19 * cell + j];
  int b = ptr[r], en = ptr[r + 1];
  while (b < en) {
    const int m = (b + en) >> 1;
    if (col[m] < c) b = m + 1; else en = m;
  }
  pos[t] = (b < ptr[r + 1] && col[b] == c) ? b : -1;
}

}  // namespace

void launch_feec_system(const FeecCellData& cd, const int32_t* cells, int n, const int32_t* pos,
                        const double* old_nse, const double* T_old, const PhysicsDev& ph, double* A,
                        double* rhs, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL((k_feec_system<0>), dim3(n), dim3(64), 0, s, cd, cells, 0, pos, old_nse, T_old,
                     ph, A, rhs, nullptr, nullptr);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_feec_elements(const FeecCellData& cd, int first, int n, const double* old_nse,
                          const double* T_old, const PhysicsDev& ph, double* K, double* f,
                          hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL((k_feec_system<1>), dim3(n), dim3(64), 0, s, cd, nullptr, first, nullptr,
                     old_nse, T_old, ph, nullptr, nullptr, K, f);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_feec_precond(const FeecCellData& cd, const int32_t* cells, int n, const int32_t* pos,
                         const PhysicsDev& ph, double* P, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_feec_precond, dim3(n), dim3(64), 0, s, cd, cells, pos, ph, P);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_feec_T_rhs(const FeecCellData& cd, const int32_t* cells, int n, const double* T_old,
                       const double* nse, const PhysicsDev& ph, const uint8_t* T_fixed,
                       const double* T_bc, double* rhs, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_feec_T_rhs, dim3(n), dim3(64), 0, s, cd, cells, T_old, nse, ph, T_fixed,
                     T_bc, rhs);
  DCP_HIP_CHECK(hipGetLastError());
}

void feec_velocity_stats(const FeecCellData& cd, int n_cells, const double* nse, double* out2,
                         hipStream_t s) {
  DCP_HIP_CHECK(hipMemsetAsync(out2, 0, 2 * sizeof(double), s));
  if (n_cells <= 0) return;
  hipLaunchKernelGGL(k_feec_vel_stats, dim3((n_cells + 255) / 256), dim3(256), 0, s, cd, n_cells,
                     nse, out2);
  DCP_HIP_CHECK(hipGetLastError());
}

void feec_cell_weights(const FeecCellData& cd, int n_cells, double* w, hipStream_t s, int npt) {
  if (n_cells <= 0) return;
  hipLaunchKernelGGL(k_feec_cell_weights, dim3((n_cells + 255) / 256), dim3(256), 0, s, cd, n_cells,
                     w, npt);
  DCP_HIP_CHECK(hipGetLastError());
}

void feec_positions(const FeecCellData& cd, int n_cells, const int32_t* ptr, const int32_t* col,
                    int32_t* pos, hipStream_t s) {
  const long t = long(n_cells) * 361;
  if (t <= 0) return;
  hipLaunchKernelGGL(k_feec_positions, dim3((t + 255) / 256), dim3(256), 0, s, cd, n_cells, ptr, col,
                     pos);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
