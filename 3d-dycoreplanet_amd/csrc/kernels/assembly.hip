// Cell-local finite-element assembly kernels for CDNA4 (gfx950), FP64.
//
// Replaces the WorkStream worker/copier pairs of the reference
// (include/core/boussinesq_model.tpp):
//   local_assemble_nse_system + copy_local_to_global_nse_system   :550-687
//   local_assemble_nse_preconditioner (diagonal only) + Jacobi     :421-542
//   local_assemble_temperature_matrix + copy                       :748-817
//   local_assemble_temperature_rhs + copy (matrix_for_bc lift)     :873-964
//
// One 256-thread workgroup owns one cell. The Q2 isoparametric geometry is
// recomputed from the 27 node coordinates (gathered through the cell's node
// map, 648 B of unique-per-cell traffic instead of 2160 B of stored J^-1/JxW),
// shape tables and per-quadrature physical gradients are staged in LDS, and the
// 27x27 node-pair Gram sums run as 1x3 register tiles (243 threads). The
// condensed (AffineConstraints) 3x3 node blocks are added into the block-CSR
// matrices with plain read-modify-write: the launch processes one colour of a
// cell colouring, so no two workgroups touch the same node and the result is
// deterministic (no atomics).
#include <hip/hip_runtime.h>

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

// 27 threads: Q2 isoparametric mapping at the QGauss(3) points.
__device__ inline void cell_geometry(const double* X, Geo& g, int q) {
  const int qa = q % 3, qb = (q / 3) % 3, qc = q / 9;
  double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  double x[3] = {0, 0, 0};
#pragma unroll 1
  for (int n = 0; n < 27; ++n) {
    const int na = n % 3, nb = (n / 3) % 3, nc = n / 9;
    const double la = cL2[na][qa], lb = cL2[nb][qb], lc = cL2[nc][qc];
    const double gx = cdL2[na][qa] * lb * lc, gy = la * cdL2[nb][qb] * lc,
                 gz = la * lb * cdL2[nc][qc], s = la * lb * lc;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double Xi = X[3 * n + i];
      x[i] += Xi * s;
      J[i][0] += Xi * gx;
      J[i][1] += Xi * gy;
      J[i][2] += Xi * gz;
    }
  }
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
// NSE system: local_assemble_nse_system (:550-673) + distribute_local_to_global.
// MODE 0 = scatter into block-CSR (colour launch), MODE 1 = dense element output.
struct NseSmem {
  double X[81], U[81], T[8];
  Geo geo;
  double D[27 * 27 * 3];   // [q][n][d] physical gradients
  double S[27 * 27];       // [q][n] shape values
  double F[27 * 3];        // JxW * rhs integrand (velocity part) per q
  double diag[27];         // sum_c |K_(a,c),(a,c)| per node (average-diagonal rule)
  int node[27];
  int pdof[8];
};

template <int MODE>
__global__ __launch_bounds__(256) void k_nse_system(CellData cd, ScatterMaps sm,
                                                    const int32_t* __restrict__ cells, int first,
                                                    const double* __restrict__ u_old,
                                                    const double* __restrict__ T_old,
                                                    PhysicsDev ph, NseOut out) {
  __shared__ NseSmem sh;
  const int tid = threadIdx.x;
  const int cell = MODE == 0 ? cells[blockIdx.x] : first + blockIdx.x;
  const bool want_matrix = MODE == 1 || out.A != nullptr;
  const bool want_rhs = MODE == 1 || out.rhs != nullptr;

  if (tid < 27) {
    const int n = cd.cell_q2[27 * size_t(cell) + tid];
    sh.node[tid] = n;
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      sh.X[3 * tid + d] = cd.xyz[3 * size_t(n) + d];
      sh.U[3 * tid + d] = u_old[3 * size_t(n) + d];
    }
  } else if (tid >= 32 && tid < 40) {
    const int v = tid - 32;
    sh.pdof[v] = cd.cell_p[8 * size_t(cell) + v];
    sh.T[v] = T_old[cd.cell_T[8 * size_t(cell) + v]];
  }
  for (int i = tid; i < 729; i += 256) sh.S[i] = q2_value(i / 27, i % 27);
  __syncthreads();
  if (tid < 27) cell_geometry(sh.X, sh.geo, tid);
  __syncthreads();
  for (int i = tid; i < 729; i += 256) q2_grad(sh.geo, i / 27, i % 27, &sh.D[3 * i]);
  __syncthreads();

  // Right-hand-side integrand per quadrature point (:593-650, 655-669).
  if (want_rhs && tid < 27) {
    const int q = tid;
    double u[3] = {0, 0, 0}, G[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
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
#pragma unroll
    for (int v = 0; v < 8; ++v) T += sh.T[v] * q1_value(q, v);
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

  // Velocity-velocity node blocks: 1x3 register tiles over (a, b0..b0+2).
  double blk[3][9];
  int a = 0, b0 = 0;
  if (want_matrix && tid < 243) {
    a = tid / 9;
    b0 = 3 * (tid % 9);
    double m[3] = {0, 0, 0}, Q[3][9];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
      for (int i = 0; i < 9; ++i) Q[t][i] = 0;
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
    // K_(a,c),(b,c') = delta_cc' (M + dt/Re L) + dt/Re Q_{c'c}   (2 eps:eps / 2)
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const double L = Q[t][0] + Q[t][4] + Q[t][8];
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int cp = 0; cp < 3; ++cp)
          blk[t][3 * c + cp] = (c == cp ? m[t] + ph.nu_sys * L : 0.0) + ph.nu_sys * Q[t][3 * cp + c];
      if (b0 + t == a) sh.diag[a] = fabs(blk[t][0]) + fabs(blk[t][4]) + fabs(blk[t][8]);
    }
  }
  __syncthreads();

  if (MODE == 1) {
    double* K = out.elemK + size_t(blockIdx.x) * 89 * 89;
    double* f = out.elemF + size_t(blockIdx.x) * 89;
    if (tid < 243) {
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
          for (int cp = 0; cp < 3; ++cp)
            K[89 * fesys_velocity(a, c) + fesys_velocity(b0 + t, cp)] = blk[t][3 * c + cp];
    }
    if (tid < 216) {
      const int an = tid / 8, v = tid % 8;
      double bt[3] = {0, 0, 0};
      for (int q = 0; q < 27; ++q) {
        const double wp = sh.geo.JxW[q] * q1_value(q, v);
        const double* Da = &sh.D[3 * (27 * q + an)];
        bt[0] -= Da[0] * wp; bt[1] -= Da[1] * wp; bt[2] -= Da[2] * wp;
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        K[89 * fesys_velocity(an, c) + 4 * v + 3] = bt[c];
        K[89 * (4 * v + 3) + fesys_velocity(an, c)] = bt[c];
      }
    } else if (tid < 243) {
      const int an = tid - 216;
      double fa[3] = {0, 0, 0};
      for (int q = 0; q < 27; ++q) {
        const double s = sh.S[27 * q + an];
        fa[0] += s * sh.F[3 * q]; fa[1] += s * sh.F[3 * q + 1]; fa[2] += s * sh.F[3 * q + 2];
      }
#pragma unroll
      for (int c = 0; c < 3; ++c) f[fesys_velocity(an, c)] = fa[c];
    } else if (tid < 251) {
      const int v = tid - 243;  // pressure rows of f and the empty p-p block
      f[4 * v + 3] = 0.0;
      for (int w = 0; w < 8; ++w) K[89 * (4 * v + 3) + 4 * w + 3] = 0.0;
    }
    return;
  }

  // ---- MODE 0: condensation + colour-exclusive read-modify-write -----------
  double avg = 0;
  if (want_matrix) {
    for (int n = 0; n < 27; ++n) avg += sh.diag[n];
    avg /= 89.0;  // pressure diagonals of the local matrix are 0
  }
  if (want_matrix && tid < 243) {
    const NodeConstraint ca = cd.vcon[sh.node[a]];
    double Ca[3][3];
    condensation(ca, Ca);
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      const int b = b0 + t;
      const NodeConstraint cb = cd.vcon[sh.node[b]];
      double Cb[3][3];
      condensation(cb, Cb);
      double KC[3][3], R[9];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          KC[i][j] = blk[t][3 * i] * Cb[0][j] + blk[t][3 * i + 1] * Cb[1][j] + blk[t][3 * i + 2] * Cb[2][j];
#pragma unroll
      for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j)
          R[3 * i + j] = Ca[0][i] * KC[0][j] + Ca[1][i] * KC[1][j] + Ca[2][i] * KC[2][j];
      if (b == a && ca.type != 0) {
        // constrained local dofs: global diagonal += |K_ii| (average if 0)
#pragma unroll
        for (int c = 0; c < 3; ++c)
          if (ca.type == 1 || c == ca.k) {
            const double kii = fabs(blk[t][4 * c]);
            R[4 * c] += kii != 0.0 ? kii : avg;
          }
      }
      double* dst = out.A + 9 * size_t(sm.posA[729 * size_t(cell) + 27 * a + b]);
#pragma unroll
      for (int i = 0; i < 9; ++i) dst[i] += R[i];
    }
  }
  if (want_matrix && tid < 216) {
    const int an = tid / 8, v = tid % 8;
    double bt[3] = {0, 0, 0};
    for (int q = 0; q < 27; ++q) {
      const double wp = sh.geo.JxW[q] * q1_value(q, v);
      const double* Da = &sh.D[3 * (27 * q + an)];
      bt[0] -= Da[0] * wp; bt[1] -= Da[1] * wp; bt[2] -= Da[2] * wp;
    }
    double Ca[3][3];
    condensation(cd.vcon[sh.node[an]], Ca);
    double r[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) r[j] = Ca[0][j] * bt[0] + Ca[1][j] * bt[1] + Ca[2][j] * bt[2];
    double* dbt = out.Bt + 3 * size_t(sm.posBt[216 * size_t(cell) + 8 * an + v]);
    double* db = out.B + 3 * size_t(sm.posB[216 * size_t(cell) + 27 * v + an]);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      dbt[j] += r[j];
      db[j] += r[j];
    }
  }
  if (want_rhs && tid >= 216 && tid < 243) {
    const int an = tid - 216;
    double fa[3] = {0, 0, 0};
    for (int q = 0; q < 27; ++q) {
      const double s = sh.S[27 * q + an];
      fa[0] += s * sh.F[3 * q]; fa[1] += s * sh.F[3 * q + 1]; fa[2] += s * sh.F[3 * q + 2];
    }
    double Ca[3][3];
    condensation(cd.vcon[sh.node[an]], Ca);
    double* dst = out.rhs + 3 * size_t(sh.node[an]);
#pragma unroll
    for (int j = 0; j < 3; ++j) dst[j] += Ca[0][j] * fa[0] + Ca[1][j] * fa[1] + Ca[2][j] * fa[2];
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
  __shared__ double X[81];
  __shared__ Geo geo;
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  if (tid < 27) {
    const int n = cd.cell_q2[27 * size_t(cell) + tid];
#pragma unroll
    for (int d = 0; d < 3; ++d) X[3 * tid + d] = cd.xyz[3 * size_t(n) + d];
  }
  __syncthreads();
  if (tid < 27) cell_geometry(X, geo, tid);
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
    const NodeConstraint nc = cd.vcon[n];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      double f = 1.0;
      if (nc.type == 2 && d != nc.k) f = 1.0 + nc.w[d] * nc.w[d];
      A_diag[3 * size_t(n) + d] += f * p;
    }
  } else if (tid >= 32 && tid < 40) {
    const int v = tid - 32;
    double p = 0;
    for (int q = 0; q < 27; ++q) {
      const double s = q1_value(q, v);
      p += s * s * geo.JxW[q];
    }
    Mp_diag[cd.cell_p[8 * size_t(cell) + v]] += p;
  }
}

// ---------------------------------------------------------------------------
// Temperature mass / stiffness (Q1, QGauss(3)) with Dirichlet condensation.
__global__ __launch_bounds__(64) void k_T_matrix(CellData cd, ScatterMaps sm,
                                                 const int32_t* __restrict__ cells, PhysicsDev ph,
                                                 double* Tmass, double* Tstiff) {
  __shared__ double X[81];
  __shared__ Geo geo;
  __shared__ double G1[27 * 8 * 3];
  __shared__ int dof[8];
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  if (tid < 27) {
    const int n = cd.cell_q2[27 * size_t(cell) + tid];
#pragma unroll
    for (int d = 0; d < 3; ++d) X[3 * tid + d] = cd.xyz[3 * size_t(n) + d];
  } else if (tid >= 32 && tid < 40) {
    dof[tid - 32] = cd.cell_T[8 * size_t(cell) + tid - 32];
  }
  __syncthreads();
  if (tid < 27) cell_geometry(X, geo, tid);
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
}

// Temperature rhs with the matrix_for_bc lift of inhomogeneous Dirichlet dofs.
__global__ __launch_bounds__(64) void k_T_rhs(CellData cd, const int32_t* __restrict__ cells,
                                              const double* __restrict__ T_old,
                                              const double* __restrict__ u_cur, PhysicsDev ph,
                                              double* rhs) {
  __shared__ double X[81], U[81];
  __shared__ Geo geo;
  __shared__ double G1[27 * 8 * 3];
  __shared__ double Tq[27], Fq[27];
  __shared__ double Tn[8];
  __shared__ int dof[8];
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  if (tid < 27) {
    const int n = cd.cell_q2[27 * size_t(cell) + tid];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      X[3 * tid + d] = cd.xyz[3 * size_t(n) + d];
      U[3 * tid + d] = u_cur[3 * size_t(n) + d];
    }
  } else if (tid >= 32 && tid < 40) {
    const int d = cd.cell_T[8 * size_t(cell) + tid - 32];
    dof[tid - 32] = d;
    Tn[tid - 32] = T_old[d];
  }
  __syncthreads();
  if (tid < 27) cell_geometry(X, geo, tid);
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
  const int32_t* td = cd.cell_T + 8 * size_t(cell);
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
  for (int i = threadIdx.x; i < 64; i += blockDim.x) {
    const int r = td[i / 8], c = td[i % 8];
    posT[64 * size_t(cell) + i] = find_sorted(T_col, T_ptr[r], T_ptr[r + 1], c);
  }
}

// S_pq = sum_n sum_c B[p][n][c] d[3n+c] B^T[n][q][c]; one 64-lane workgroup
// per pressure row. The node loop is sequential and the lanes of one node
// write distinct q, so every entry is summed in the same (node) order.
__global__ __launch_bounds__(64) void k_schur_form(int n_p, const int32_t* __restrict__ B_ptr,
                                                   const int32_t* __restrict__ B_col,
                                                   const double* __restrict__ B_val,
                                                   const int32_t* __restrict__ Bt_ptr,
                                                   const int32_t* __restrict__ Bt_col,
                                                   const double* __restrict__ Bt_val,
                                                   const double* __restrict__ d,
                                                   const int32_t* __restrict__ S_ptr,
                                                   const int32_t* __restrict__ S_col,
                                                   double* __restrict__ S_val) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int p = blockIdx.x;
  const int s0 = S_ptr[p], len = S_ptr[p + 1] - s0;
  double* acc = reinterpret_cast<double*>(smem);
  int* cols = reinterpret_cast<int*>(acc + len);
  for (int j = threadIdx.x; j < len; j += 64) {
    acc[j] = 0.0;
    cols[j] = S_col[s0 + j];
  }
  __syncthreads();
  for (int k = B_ptr[p]; k < B_ptr[p + 1]; ++k) {
    const size_t n = size_t(B_col[k]);
    const double w0 = B_val[3 * size_t(k)] * d[3 * n];
    const double w1 = B_val[3 * size_t(k) + 1] * d[3 * n + 1];
    const double w2 = B_val[3 * size_t(k) + 2] * d[3 * n + 2];
    const int b = Bt_ptr[n], e = Bt_ptr[n + 1];
    for (int j = b + int(threadIdx.x); j < e; j += 64) {
      const int q = Bt_col[j];
      const double v = w0 * Bt_val[3 * size_t(j)] + w1 * Bt_val[3 * size_t(j) + 1] +
                       w2 * Bt_val[3 * size_t(j) + 2];
      int lo = 0, hi = len;
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (cols[m] < q) lo = m + 1; else hi = m;
      }
      acc[lo] += v;
    }
    __syncthreads();
  }
  for (int j = threadIdx.x; j < len; j += 64) S_val[s0 + j] = acc[j];
}

}  // namespace

void form_schur_complement(int n_p, const int32_t* B_ptr, const int32_t* B_col, const double* B_val,
                           const int32_t* Bt_ptr, const int32_t* Bt_col, const double* Bt_val,
                           const double* d, const int32_t* S_ptr, const int32_t* S_col,
                           double* S_val, int max_row, hipStream_t s) {
  if (n_p <= 0) return;
  const size_t lds = size_t(max_row) * (sizeof(double) + sizeof(int)) + 16;
  hipLaunchKernelGGL(k_schur_form, dim3(n_p), dim3(64), lds, s, n_p, B_ptr, B_col, B_val, Bt_ptr,
                     Bt_col, Bt_val, d, S_ptr, S_col, S_val);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_nse_system(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                       const double* u_old, const double* T_old, const PhysicsDev& ph,
                       const NseOut& out, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_nse_system<0>, dim3(n), dim3(256), 0, s, cd, sm, cells, 0, u_old, T_old, ph,
                     out);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_nse_system_elements(const CellData& cd, int first, int n, const double* u_old,
                                const double* T_old, const PhysicsDev& ph, double* K, double* f,
                                hipStream_t s) {
  if (n <= 0) return;
  NseOut out{};
  out.elemK = K;
  out.elemF = f;
  hipLaunchKernelGGL(k_nse_system<1>, dim3(n), dim3(256), 0, s, cd, ScatterMaps{}, nullptr, first,
                     u_old, T_old, ph, out);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_nse_precond_diag(const CellData& cd, const int32_t* cells, int n, const PhysicsDev& ph,
                             double* A_diag, double* Mp_diag, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_nse_precond_diag, dim3(n), dim3(64), 0, s, cd, cells, ph, A_diag, Mp_diag);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_T_matrix(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                     const PhysicsDev& ph, double* Tmass, double* Tstiff, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_T_matrix, dim3(n), dim3(64), 0, s, cd, sm, cells, ph, Tmass, Tstiff);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_T_rhs(const CellData& cd, const int32_t* cells, int n, const double* T_old,
                  const double* u_cur, const PhysicsDev& ph, double* rhs, hipStream_t s) {
  if (n <= 0) return;
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

}  // namespace dcp
