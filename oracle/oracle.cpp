// ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h). CPU restatement of the
// reference hot path. Reference paths are relative to konsim83/3D-DyCorePlanet.
#include "oracle.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// Reference element (deal.II FE_Q / FESystem / QGauss conventions).

// FE_Q(2) hierarchic -> lexicographic (vertices, lines 0..11, faces 0..5, interior).
const int kHier2Lex[27] = {0, 2, 6, 8, 18, 20, 24, 26, 3, 5, 1, 7, 21, 23,
                           19, 25, 9, 11, 15, 17, 12, 14, 10, 16, 4, 22, 13};
const int kVertexLex[8] = {0, 2, 6, 8, 18, 20, 24, 26};

double lag2(int a, double x) {
  return a == 0 ? 2 * (x - 0.5) * (x - 1) : a == 1 ? -4 * x * (x - 1) : 2 * x * (x - 0.5);
}
double dlag2(int a, double x) { return a == 0 ? 4 * x - 3 : a == 1 ? -8 * x + 4 : 4 * x - 1; }
double lag1(int a, double x) { return a == 0 ? 1 - x : x; }
double dlag1(int a, double) { return a == 0 ? -1.0 : 1.0; }

// QGauss(n) on [0,1], n = 1..4.
void gauss1d(int n, double* x, double* w) {
  if (n == 1) {
    x[0] = 0.5; w[0] = 1.0;
  } else if (n == 2) {
    const double d = 0.5 / std::sqrt(3.0);
    x[0] = 0.5 - d; x[1] = 0.5 + d; w[0] = w[1] = 0.5;
  } else if (n == 3) {
    const double d = 0.5 * std::sqrt(0.6);
    x[0] = 0.5 - d; x[1] = 0.5; x[2] = 0.5 + d;
    w[0] = w[2] = 5.0 / 18.0; w[1] = 8.0 / 18.0;
  } else if (n == 4) {
    const double a = std::sqrt(3.0 / 7.0 - 2.0 / 7.0 * std::sqrt(6.0 / 5.0));
    const double b = std::sqrt(3.0 / 7.0 + 2.0 / 7.0 * std::sqrt(6.0 / 5.0));
    const double wa = (18.0 + std::sqrt(30.0)) / 36.0, wb = (18.0 - std::sqrt(30.0)) / 36.0;
    x[0] = 0.5 - 0.5 * b; x[1] = 0.5 - 0.5 * a; x[2] = 0.5 + 0.5 * a; x[3] = 0.5 + 0.5 * b;
    w[0] = w[3] = 0.5 * wb; w[1] = w[2] = 0.5 * wa;
  } else {
    throw std::invalid_argument("QGauss n");
  }
}

struct Vec3 {
  double v[3] = {0, 0, 0};
  double& operator[](int i) { return v[i]; }
  double operator[](int i) const { return v[i]; }
};
double dot(const Vec3& a, const Vec3& b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// MappingQ(3) (boussinesq_model.tpp:20; deal.II MappingQGeneric(3)): tensor-
// product Lagrange polynomials on the 4 Gauss-Lobatto points of [0,1]
// (0, (1-1/sqrt5)/2, (1+1/sqrt5)/2, 1), 64 support points per cell in
// lexicographic order. Restated here independently of the product's tables.
const double kGL[4] = {0.0, 0.5 - 0.5 / std::sqrt(5.0), 0.5 + 0.5 / std::sqrt(5.0), 1.0};
double lag3(int i, double x) {
  double v = 1.0;
  for (int j = 0; j < 4; ++j)
    if (j != i) v *= (x - kGL[j]) / (kGL[i] - kGL[j]);
  return v;
}
double dlag3(int i, double x) {
  double s = 0.0;
  for (int k = 0; k < 4; ++k) {
    if (k == i) continue;
    double v = 1.0 / (kGL[i] - kGL[k]);
    for (int j = 0; j < 4; ++j)
      if (j != i && j != k) v *= (x - kGL[j]) / (kGL[i] - kGL[j]);
    s += v;
  }
  return s;
}

// FEValues for one cell: the cell's MappingQ(3) from its 64 support points;
// Q2 and Q1 scalar shapes with physical gradients.
struct CellValues {
  int nq = 0;
  std::vector<double> JxW;
  std::vector<Vec3> xq;
  std::vector<double> v2, v1;   // [q][27], [q][8]   (lexicographic / vertex order)
  std::vector<Vec3> g2, g1;     // physical gradients

  void reinit(const double* geom, int n1d) {
    double qx[4], qw[4];
    gauss1d(n1d, qx, qw);
    nq = n1d * n1d * n1d;
    JxW.assign(nq, 0);
    xq.assign(nq, Vec3());
    v2.assign(size_t(nq) * 27, 0);
    v1.assign(size_t(nq) * 8, 0);
    g2.assign(size_t(nq) * 27, Vec3());
    g1.assign(size_t(nq) * 8, Vec3());
    for (int q = 0; q < nq; ++q) {
      const double p[3] = {qx[q % n1d], qx[(q / n1d) % n1d], qx[q / (n1d * n1d)]};
      const double w = qw[q % n1d] * qw[(q / n1d) % n1d] * qw[q / (n1d * n1d)];
      double rv2[27], rg2[27][3], rv1[8], rg1[8][3];
      for (int n = 0; n < 27; ++n) {
        const int a = n % 3, b = (n / 3) % 3, c = n / 9;
        rv2[n] = lag2(a, p[0]) * lag2(b, p[1]) * lag2(c, p[2]);
        rg2[n][0] = dlag2(a, p[0]) * lag2(b, p[1]) * lag2(c, p[2]);
        rg2[n][1] = lag2(a, p[0]) * dlag2(b, p[1]) * lag2(c, p[2]);
        rg2[n][2] = lag2(a, p[0]) * lag2(b, p[1]) * dlag2(c, p[2]);
      }
      for (int n = 0; n < 8; ++n) {
        const int a = n & 1, b = (n >> 1) & 1, c = n >> 2;
        rv1[n] = lag1(a, p[0]) * lag1(b, p[1]) * lag1(c, p[2]);
        rg1[n][0] = dlag1(a, p[0]) * lag1(b, p[1]) * lag1(c, p[2]);
        rg1[n][1] = lag1(a, p[0]) * dlag1(b, p[1]) * lag1(c, p[2]);
        rg1[n][2] = lag1(a, p[0]) * lag1(b, p[1]) * dlag1(c, p[2]);
      }
      // Jacobian J[i][j] = d x_i / d xi_j of the cubic map
      double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
      Vec3 x;
      for (int n = 0; n < 64; ++n) {
        const int a = n % 4, b = (n / 4) % 4, c = n / 16;
        const double s = lag3(a, p[0]) * lag3(b, p[1]) * lag3(c, p[2]);
        const double g[3] = {dlag3(a, p[0]) * lag3(b, p[1]) * lag3(c, p[2]),
                             lag3(a, p[0]) * dlag3(b, p[1]) * lag3(c, p[2]),
                             lag3(a, p[0]) * lag3(b, p[1]) * dlag3(c, p[2])};
        for (int i = 0; i < 3; ++i) {
          x[i] += geom[3 * n + i] * s;
          for (int j = 0; j < 3; ++j) J[i][j] += geom[3 * n + i] * g[j];
        }
      }
      const double det = J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
                         J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
                         J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
      if (!(det > 0)) throw std::runtime_error("oracle: non-positive Jacobian");
      double Ji[3][3];  // inverse
      Ji[0][0] = (J[1][1] * J[2][2] - J[1][2] * J[2][1]) / det;
      Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / det;
      Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / det;
      Ji[1][0] = (J[1][2] * J[2][0] - J[1][0] * J[2][2]) / det;
      Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / det;
      Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / det;
      Ji[2][0] = (J[1][0] * J[2][1] - J[1][1] * J[2][0]) / det;
      Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / det;
      Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / det;
      JxW[q] = det * w;
      xq[q] = x;
      // physical gradient: grad_i = sum_j dN/dxi_j * Ji[j][i]
      for (int n = 0; n < 27; ++n) {
        v2[27 * q + n] = rv2[n];
        for (int i = 0; i < 3; ++i)
          g2[27 * q + n][i] = rg2[n][0] * Ji[0][i] + rg2[n][1] * Ji[1][i] + rg2[n][2] * Ji[2][i];
      }
      for (int n = 0; n < 8; ++n) {
        v1[8 * q + n] = rv1[n];
        for (int i = 0; i < 3; ++i)
          g1[8 * q + n][i] = rg1[n][0] * Ji[0][i] + rg1[n][1] * Ji[1][i] + rg1[n][2] * Ji[2][i];
      }
    }
  }
};

// FESystem(FE_Q(2)^3, FE_Q(1)) local dof i -> (component, scalar shape index).
// Scalar index: lexicographic Q2 node for velocity, vertex for pressure.
struct SysDof {
  int comp, idx;
};
SysDof sysdof(int i) {
  if (i < 32) return {i % 4, i % 4 == 3 ? i / 4 : kHier2Lex[i / 4]};
  return {(i - 32) % 3, kHier2Lex[8 + (i - 32) / 3]};
}

// Temperature FE_Q(k) hierarchic local dof -> value/grad accessors.
double T_value(const CellValues& cv, int deg, int q, int k) {
  return deg == 1 ? cv.v1[8 * q + k] : cv.v2[27 * q + kHier2Lex[k]];
}
const Vec3& T_grad(const CellValues& cv, int deg, int q, int k) {
  return deg == 1 ? cv.g1[8 * q + k] : cv.g2[27 * q + kHier2Lex[k]];
}
int T_dofs_per_cell(int deg) { return deg == 1 ? 8 : 27; }

// Per-q views of the NSE system shape functions (FEValuesViews::Vector /
// Scalar): value, gradient (row = component), symmetric gradient, divergence.
struct NseShapes {
  Vec3 phi_u[89];
  double grad[89][3][3];
  double eps[89][3][3];
  double div[89];
  double phi_p[89];
  void at(const CellValues& cv, int q) {
    for (int k = 0; k < 89; ++k) {
      const SysDof s = sysdof(k);
      phi_u[k] = Vec3();
      std::memset(grad[k], 0, sizeof(grad[k]));
      std::memset(eps[k], 0, sizeof(eps[k]));
      div[k] = 0;
      phi_p[k] = 0;
      if (s.comp < 3) {
        const double v = cv.v2[27 * q + s.idx];
        const Vec3& g = cv.g2[27 * q + s.idx];
        phi_u[k][s.comp] = v;
        for (int d = 0; d < 3; ++d) grad[k][s.comp][d] = g[d];
        for (int a = 0; a < 3; ++a)
          for (int b = 0; b < 3; ++b) eps[k][a][b] = 0.5 * (grad[k][a][b] + grad[k][b][a]);
        div[k] = g[s.comp];
      } else {
        phi_p[k] = cv.v1[8 * q + s.idx];
      }
    }
  }
};

double ddot(const double a[3][3], const double b[3][3]) {
  double s = 0;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) s += a[i][j] * b[i][j];
  return s;
}

// CoreModelData::gravity_vector (core_model_data.tpp:97-106, Q4)
Vec3 gravity_vector(const Vec3& p, double g) {
  const double r = std::sqrt(dot(p, p));
  Vec3 out;
  for (int d = 0; d < 3; ++d) out[d] = (r > 1) ? -g * p[d] / r : -g * p[d] / std::sqrt(r);
  return out;
}

Vec3 cross(const Vec3& a, const Vec3& b) {
  Vec3 c;
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
  return c;
}

}  // namespace

// ===========================================================================
// Element level

namespace {
// The (a, b) entries, in ddot's lexicographic order, where the symmetric
// gradients of a component-ci and a component-cj velocity shape can both be
// non-zero (eps of component c lives in row c and column c). Every other term
// of ddot(eps_i, eps_j) has an exactly-zero factor.
int eps_common(int ci, int cj, int* ab) {
  int n = 0;
  for (int a = 0; a < 3; ++a)
    for (int b = 0; b < 3; ++b)
      if ((a == ci || b == ci) && (a == cj || b == cj)) ab[n++] = 3 * a + b;
  return n;
}
}  // namespace

// The element matrix loops below skip the structural zeros of the FESystem
// (a velocity shape has one non-zero component; phi_p vanishes on velocity
// shapes and vice versa) and sum every other term in the literal loop's order,
// so each entry is bitwise the one of the literal loop of
// boussinesq_model.tpp:626-637 (orc_cell_nse_system_literal; only the sign of
// an exact zero may differ). tests/test_oracle_kat.py checks this on every
// cell of a mesh. They exist to make the refine-5 oracle affordable.
// Local dofs grouped by component (27 per velocity component, 8 pressure);
// Kb accumulates the element matrix in that grouped order (entry (i, j) at
// Kb[89 * pos(i) + pos(j)]) and is permuted into K after the point loop.
struct CompBlocks {
  int idx[4][27], cnt[4], pos[89];
  int ab[3][3][9], nab[3][3];
  CompBlocks() {
    for (int c = 0; c < 4; ++c) cnt[c] = 0;
    int p = 0;
    for (int c = 0; c < 4; ++c)
      for (int k = 0; k < 89; ++k)
        if (sysdof(k).comp == c) {
          idx[c][cnt[c]++] = k;
          pos[k] = p++;
        }
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) nab[a][b] = eps_common(a, b, ab[a][b]);
  }
};
const CompBlocks& comp_blocks() {
  static const CompBlocks cb;
  return cb;
}

static void nse_K_q(const NseShapes& sh, double dt, double R2, double JxW, double* Kb) {
  const CompBlocks& cb = comp_blocks();
  double V[3][27], E[3][9][27], D[3][27], Pp[8];
  for (int c = 0; c < 3; ++c)
    for (int n = 0; n < 27; ++n) {
      const int k = cb.idx[c][n];
      V[c][n] = sh.phi_u[k][c];
      D[c][n] = sh.div[k];
      for (int e = 0; e < 9; ++e) E[c][e][n] = (&sh.eps[k][0][0])[e];
    }
  for (int n = 0; n < 8; ++n) Pp[n] = sh.phi_p[cb.idx[3][n]];
  for (int ci = 0; ci < 3; ++ci)
    for (int ii = 0; ii < 27; ++ii) {
      double* row = Kb + 89 * (27 * ci + ii);
      for (int cj = 0; cj < 3; ++cj) {
        const int na = cb.nab[ci][cj];
        const int* ab = cb.ab[ci][cj];
        double* r = row + 27 * cj;
        if (ci == cj) {  // na == 5
          const double vi = V[ci][ii];
          const double a0 = E[ci][ab[0]][ii], a1 = E[ci][ab[1]][ii], a2 = E[ci][ab[2]][ii],
                       a3 = E[ci][ab[3]][ii], a4 = E[ci][ab[4]][ii];
          const double *b0 = E[cj][ab[0]], *b1 = E[cj][ab[1]], *b2 = E[cj][ab[2]],
                       *b3 = E[cj][ab[3]], *b4 = E[cj][ab[4]];
          for (int jj = 0; jj < 27; ++jj) {
            const double a = vi * V[cj][jj];
            double s = 0;
            s += a0 * b0[jj];
            s += a1 * b1[jj];
            s += a2 * b2[jj];
            s += a3 * b3[jj];
            s += a4 * b4[jj];
            r[jj] += (a + dt * (R2 * s)) * JxW;
          }
        } else {  // na == 2
          const double a0 = E[ci][ab[0]][ii], a1 = E[ci][ab[1]][ii];
          const double *b0 = E[cj][ab[0]], *b1 = E[cj][ab[1]];
          for (int jj = 0; jj < 27; ++jj) {
            double s = 0;
            s += a0 * b0[jj];
            s += a1 * b1[jj];
            r[jj] += (dt * (R2 * s)) * JxW;
          }
        }
        (void)na;
      }
      for (int jp = 0; jp < 8; ++jp) row[81 + jp] += (-(D[ci][ii] * Pp[jp])) * JxW;
    }
  for (int ip = 0; ip < 8; ++ip) {
    double* row = Kb + 89 * (81 + ip);
    for (int cj = 0; cj < 3; ++cj)
      for (int jj = 0; jj < 27; ++jj) row[27 * cj + jj] += (-(Pp[ip] * D[cj][jj])) * JxW;
  }
}

extern "C" void orc_cell_nse_system_literal(const orc_physics* ph, const double* geom64,
                                            const double* u_local, const double* T_local,
                                            double* K, double* f);

extern "C" void orc_cell_nse_system(const orc_physics* ph, const double* geom64,
                                    const double* u_local, const double* T_local, double* K,
                                    double* f) {
  // boussinesq_model.tpp:550-673; QGauss(nse_velocity_degree + 1) = 3 (:708)
  CellValues cv;
  cv.reinit(geom64, 3);
  const int tdeg = ph->temperature_degree, ntd = T_dofs_per_cell(tdeg);
  std::fill(K, K + 89 * 89, 0.0);
  std::fill(f, f + 89, 0.0);
  static thread_local NseShapes sh;
  static thread_local std::vector<double> Kb(89 * 89);
  std::fill(Kb.begin(), Kb.end(), 0.0);
  for (int q = 0; q < cv.nq; ++q) {
    sh.at(cv, q);
    double old_temperature = 0;
    for (int k = 0; k < ntd; ++k) old_temperature += T_local[k] * T_value(cv, tdeg, q, k);
    Vec3 old_velocity;
    double G[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int k = 0; k < 89; ++k) {
      const SysDof s = sysdof(k);
      if (s.comp == 3) continue;
      old_velocity[s.comp] += u_local[k] * sh.phi_u[k][s.comp];
      for (int d = 0; d < 3; ++d) G[s.comp][d] += u_local[k] * sh.grad[k][s.comp][d];
    }
    const double density_scaling =
        1 - ph->expansion_coefficient * (old_temperature - ph->temperature_ref);
    Vec3 advection;
    for (int j = 0; j < 3; ++j)
      for (int i = 0; i < 3; ++i) advection[j] += old_velocity[i] * G[j][i];
    Vec3 coriolis;
    if (ph->cuboid) coriolis[2] = ph->coriolis_scale * ph->omega;
    const double JxW = cv.JxW[q];
    const double dt = ph->time_step;
    nse_K_q(sh, dt, ph->one_over_reynolds * 2, JxW, Kb.data());
    Vec3 gravity;
    if (ph->cuboid) {
      gravity[2] = -ph->gravity_constant;
    } else {
      gravity = gravity_vector(cv.xq[q], ph->gravity_constant);
    }
    for (int d = 0; d < 3; ++d) gravity[d] *= ph->gravity_scale;
    const Vec3 cor_x_u = cross(coriolis, old_velocity);
    for (int i = 0; i < 89; ++i)
      f[i] += (dot(sh.phi_u[i], old_velocity) + dt * density_scaling * dot(gravity, sh.phi_u[i]) -
               dt * dot(sh.phi_u[i], advection) - dt * (2 * dot(sh.phi_u[i], cor_x_u))) *
              JxW;
  }
  const CompBlocks& cb = comp_blocks();
  for (int i = 0; i < 89; ++i)
    for (int j = 0; j < 89; ++j) K[89 * i + j] = Kb[89 * cb.pos[i] + cb.pos[j]];
}

// The literal restatement of local_assemble_nse_system (every 89 x 89 term);
// the checker of the structural-zero loop above (tests/test_oracle_kat.py).
extern "C" void orc_cell_nse_system_literal(const orc_physics* ph, const double* geom64,
                                            const double* u_local, const double* T_local,
                                            double* K, double* f) {
  // boussinesq_model.tpp:550-673; QGauss(nse_velocity_degree + 1) = 3 (:708)
  CellValues cv;
  cv.reinit(geom64, 3);
  const int tdeg = ph->temperature_degree, ntd = T_dofs_per_cell(tdeg);
  std::fill(K, K + 89 * 89, 0.0);
  std::fill(f, f + 89, 0.0);
  static thread_local NseShapes sh;
  for (int q = 0; q < cv.nq; ++q) {
    sh.at(cv, q);
    // get_function_values / get_function_gradients (dof-order sums)
    double old_temperature = 0;
    for (int k = 0; k < ntd; ++k) old_temperature += T_local[k] * T_value(cv, tdeg, q, k);
    Vec3 old_velocity;
    double G[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int k = 0; k < 89; ++k) {
      const SysDof s = sysdof(k);
      if (s.comp == 3) continue;
      old_velocity[s.comp] += u_local[k] * sh.phi_u[k][s.comp];
      for (int d = 0; d < 3; ++d) G[s.comp][d] += u_local[k] * sh.grad[k][s.comp][d];
    }
    // :594-597 density_scaling = 1 - beta (T - T_ref)   (core_model_data.cc:88-94)
    const double density_scaling =
        1 - ph->expansion_coefficient * (old_temperature - ph->temperature_ref);
    // :599-600 transpose(grad u); advection (u . grad) u = u * transpose(grad u)
    Vec3 advection;
    for (int j = 0; j < 3; ++j)
      for (int i = 0; i < 3; ++i) advection[j] += old_velocity[i] * G[j][i];
    // :615-621 Coriolis only on the cuboid (Q2)
    Vec3 coriolis;
    if (ph->cuboid) coriolis[2] = ph->coriolis_scale * ph->omega;
    const double JxW = cv.JxW[q];
    const double dt = ph->time_step;
    // :626-637
    for (int i = 0; i < 89; ++i)
      for (int j = 0; j < 89; ++j)
        K[89 * i + j] += (dot(sh.phi_u[i], sh.phi_u[j]) +
                          dt * (ph->one_over_reynolds * 2 * ddot(sh.eps[i], sh.eps[j])) -
                          (sh.div[i] * sh.phi_p[j]) - (sh.phi_p[i] * sh.div[j])) *
                         JxW;
    // :640-650
    Vec3 gravity;
    if (ph->cuboid) {
      gravity[2] = -ph->gravity_constant;  // vertical_gravity_vector (core_model_data.tpp:86-95)
    } else {
      gravity = gravity_vector(cv.xq[q], ph->gravity_constant);
    }
    for (int d = 0; d < 3; ++d) gravity[d] *= ph->gravity_scale;
    const Vec3 cor_x_u = cross(coriolis, old_velocity);
    // :655-669 (3D branch)
    for (int i = 0; i < 89; ++i)
      f[i] += (dot(sh.phi_u[i], old_velocity) + dt * density_scaling * dot(gravity, sh.phi_u[i]) -
               dt * dot(sh.phi_u[i], advection) - dt * (2 * dot(sh.phi_u[i], cor_x_u))) *
              JxW;
  }
}

extern "C" void orc_cell_nse_preconditioner(const orc_physics* ph, const double* geom64,
                                            double* P) {
  // boussinesq_model.tpp:421-464, structural zeros skipped as in nse_K_q:
  // velocity pairs of one component (dot + (dt/Re) grad:grad over that
  // component's gradient row) and pressure pairs (phi_p phi_p); bitwise the
  // literal loop (orc_cell_nse_preconditioner_literal)
  CellValues cv;
  cv.reinit(geom64, 3);
  std::fill(P, P + 89 * 89, 0.0);
  static thread_local NseShapes sh;
  const CompBlocks& cb = comp_blocks();
  const double dtr = ph->time_step * ph->one_over_reynolds;
  for (int q = 0; q < cv.nq; ++q) {
    sh.at(cv, q);
    const double JxW = cv.JxW[q];
    for (int c = 0; c < 3; ++c) {
      double V[27], G[3][27];
      for (int n = 0; n < 27; ++n) {
        const int k = cb.idx[c][n];
        V[n] = sh.phi_u[k][c];
        for (int b = 0; b < 3; ++b) G[b][n] = sh.grad[k][c][b];
      }
      for (int ii = 0; ii < 27; ++ii) {
        double* Pi = P + 89 * cb.idx[c][ii];
        const double vi = V[ii], g0 = G[0][ii], g1 = G[1][ii], g2 = G[2][ii];
        for (int jj = 0; jj < 27; ++jj) {
          const double a = vi * V[jj];
          double s = 0;
          s += g0 * G[0][jj];
          s += g1 * G[1][jj];
          s += g2 * G[2][jj];
          Pi[cb.idx[c][jj]] += (a + dtr * s) * JxW;
        }
      }
    }
    for (int ii = 0; ii < 8; ++ii)
      for (int jj = 0; jj < 8; ++jj)
        P[89 * cb.idx[3][ii] + cb.idx[3][jj]] += (sh.phi_p[cb.idx[3][ii]] * sh.phi_p[cb.idx[3][jj]]) * JxW;
  }
}

extern "C" void orc_cell_nse_preconditioner_literal(const orc_physics* ph, const double* geom64,
                                                    double* P) {
  // boussinesq_model.tpp:421-464
  CellValues cv;
  cv.reinit(geom64, 3);
  std::fill(P, P + 89 * 89, 0.0);
  static thread_local NseShapes sh;
  for (int q = 0; q < cv.nq; ++q) {
    sh.at(cv, q);
    const double JxW = cv.JxW[q];
    for (int i = 0; i < 89; ++i)
      for (int j = 0; j < 89; ++j)
        P[89 * i + j] += (dot(sh.phi_u[i], sh.phi_u[j]) +
                          ph->time_step * ph->one_over_reynolds * ddot(sh.grad[i], sh.grad[j]) +
                          sh.phi_p[i] * sh.phi_p[j]) *
                         JxW;
  }
}

extern "C" void orc_cell_temperature_matrix(const orc_physics* ph, const double* geom64,
                                            double* M, double* Kt) {
  // boussinesq_model.tpp:748-800, QGauss(temperature_degree + 2) (:834)
  const int tdeg = ph->temperature_degree, n = T_dofs_per_cell(tdeg);
  CellValues cv;
  cv.reinit(geom64, tdeg + 2);
  std::fill(M, M + n * n, 0.0);
  std::fill(Kt, Kt + n * n, 0.0);
  for (int q = 0; q < cv.nq; ++q) {
    const double JxW = cv.JxW[q];
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        M[n * i + j] += T_value(cv, tdeg, q, i) * T_value(cv, tdeg, q, j) * JxW;
        Kt[n * i + j] +=
            dot(T_grad(cv, tdeg, q, i), T_grad(cv, tdeg, q, j)) * ph->one_over_peclet * JxW;
      }
  }
}

extern "C" void orc_cell_temperature_rhs(const orc_physics* ph, const double* geom64,
                                         const double* T_local, const double* u_local,
                                         const int* inhom_mask, double* rhs, double* mfbc) {
  // boussinesq_model.tpp:873-952, QGauss(temperature_degree + 2) (:990)
  const int tdeg = ph->temperature_degree, n = T_dofs_per_cell(tdeg);
  CellValues cv;
  cv.reinit(geom64, tdeg + 2);
  std::fill(rhs, rhs + n, 0.0);
  std::fill(mfbc, mfbc + n * n, 0.0);
  const double dt_eff = ph->time_step / ph->nse_solver_interval;  // Q8
  const double gamma = 0;                                          // Q6
  for (int q = 0; q < cv.nq; ++q) {
    double old_T = 0;
    Vec3 old_grad_T, old_u;
    for (int k = 0; k < n; ++k) {
      old_T += T_local[k] * T_value(cv, tdeg, q, k);
      const Vec3& g = T_grad(cv, tdeg, q, k);
      for (int d = 0; d < 3; ++d) old_grad_T[d] += T_local[k] * g[d];
    }
    for (int k = 0; k < 89; ++k) {
      const SysDof s = sysdof(k);
      if (s.comp < 3) old_u[s.comp] += u_local[k] * cv.v2[27 * q + s.idx];
    }
    const double JxW = cv.JxW[q];
    for (int i = 0; i < n; ++i) {
      const double phi_i = T_value(cv, tdeg, q, i);
      rhs[i] += (phi_i * old_T - dt_eff * phi_i * dot(old_u, old_grad_T) - dt_eff * gamma * phi_i) * JxW;
      if (inhom_mask[i])
        for (int j = 0; j < n; ++j)
          mfbc[n * j + i] += (phi_i * T_value(cv, tdeg, q, j) +
                              dt_eff * ph->one_over_peclet *
                                  dot(T_grad(cv, tdeg, q, i), T_grad(cv, tdeg, q, j))) *
                             JxW;
    }
  }
}

// ===========================================================================
// Global objects

namespace {

struct Cons {
  std::vector<int> line_of;
  std::vector<std::vector<std::pair<int, double>>> entries;
  std::vector<double> inhom;
  void init(int n, const orc_constraints* c) {
    line_of.assign(n, -1);
    entries.clear();
    inhom.clear();
    if (!c) return;
    for (int l = 0; l < c->n_lines; ++l) {
      line_of[c->line_dof[l]] = l;
      std::vector<std::pair<int, double>> e;
      for (int k = c->entry_ptr[l]; k < c->entry_ptr[l + 1]; ++k)
        e.push_back({c->entry_dof[k], c->entry_w[k]});
      entries.push_back(e);
      inhom.push_back(c->inhomogeneity[l]);
    }
  }
  bool constrained(int d) const { return line_of[d] >= 0; }
  // distribute(): x_i = sum w x_t + g for every constrained i
  void distribute(double* x) const {
    for (size_t d = 0; d < line_of.size(); ++d) {
      const int l = line_of[d];
      if (l < 0) continue;
      double v = inhom[l];
      for (const auto& e : entries[l]) v += e.second * x[e.first];
      x[d] = v;
    }
  }
};

// threads of the row-parallel operator applies (orc_set_threads; default 1)
int g_threads = 1;

struct Csr {
  int n = 0;
  std::vector<int> rowptr, cols;
  std::vector<double> vals;
  // sorted pattern from row sets
  void build(const std::vector<std::vector<int>>& rows) {
    n = int(rows.size());
    rowptr.assign(n + 1, 0);
    for (int r = 0; r < n; ++r) rowptr[r + 1] = rowptr[r] + int(rows[r].size());
    cols.resize(rowptr[n]);
    for (int r = 0; r < n; ++r) std::copy(rows[r].begin(), rows[r].end(), cols.begin() + rowptr[r]);
    vals.assign(cols.size(), 0.0);
  }
  double& at(int r, int c) {
    auto b = cols.begin() + rowptr[r], e = cols.begin() + rowptr[r + 1];
    auto it = std::lower_bound(b, e, c);
    if (it == e || *it != c) throw std::runtime_error("oracle: entry not in sparsity pattern");
    return vals[it - cols.begin()];
  }
  void zero() { std::fill(vals.begin(), vals.end(), 0.0); }
  // per row, the first entry with column >= c (the pattern never changes
  // after build, so the table is built once per boundary)
  mutable std::vector<int> split;
  mutable int split_col = -1;
  const int* split_at(int c) const {
    if (split_col != c || int(split.size()) != n) {
      split.resize(n);
      for (int r = 0; r < n; ++r)
        split[r] = int(std::lower_bound(cols.begin() + rowptr[r], cols.begin() + rowptr[r + 1], c) -
                       cols.begin());
      split_col = c;
    }
    return split.data();
  }
};

void add_sorted_unique(std::vector<int>& v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}

// Row split of [0, n) into T ranges of about equal pattern entries.
std::vector<int> row_split(const std::vector<int>& rowptr, int n, int T) {
  std::vector<int> s(T + 1, n);
  s[0] = 0;
  const long nnz = rowptr.empty() ? n : rowptr[n];
  int r = 0;
  for (int t = 1; t < T; ++t) {
    const long goal = nnz * t / T;
    while (r < n && (rowptr.empty() ? r : rowptr[r]) < goal) ++r;
    s[t] = r;
  }
  return s;
}

// Expansion of a local dof under the constraints: unconstrained -> itself,
// constrained -> its targets with weights (AffineConstraints condensation).
void expand(const Cons& c, int dof, std::vector<std::pair<int, double>>& out) {
  out.clear();
  const int l = c.line_of[dof];
  if (l < 0) {
    out.push_back({dof, 1.0});
  } else {
    for (const auto& e : c.entries[l]) out.push_back(e);
  }
}

// make_sparsity_pattern(dof_handler, coupling, sp, constraints, false)
// coupling(ci, cj) decides local pairs; constrained rows keep only their diagonal.
template <class Coupling>
void make_pattern(Csr& A, int n, int n_cells, int dpc, const int* cell_dofs, const Cons& cons,
                  Coupling coupling) {
  // rows split over g_threads threads by range (the sorted unique rows do
  // not depend on the insertion order)
  std::vector<std::vector<int>> rows(n);
  const std::vector<int> split = row_split({}, n, g_threads);
#pragma omp parallel for num_threads(g_threads) schedule(static, 1) if (g_threads > 1)
  for (int t = 0; t < g_threads; ++t) {
    const int r0 = split[t], r1 = split[t + 1];
    std::vector<std::pair<int, double>> ei, ej;
    for (int c = 0; c < n_cells; ++c) {
      const int* d = cell_dofs + size_t(c) * dpc;
      for (int i = 0; i < dpc; ++i) {
        expand(cons, d[i], ei);
        bool any_own = false;
        for (const auto& a : ei) any_own |= a.first >= r0 && a.first < r1;
        if (!any_own) continue;
        for (int j = 0; j < dpc; ++j) {
          if (!coupling(i, j)) continue;
          expand(cons, d[j], ej);
          for (const auto& a : ei)
            if (a.first >= r0 && a.first < r1)
              for (const auto& b : ej) rows[a.first].push_back(b.first);
        }
      }
    }
    for (int r = r0; r < r1; ++r) {
      if (cons.constrained(r)) rows[r].push_back(r);
      add_sorted_unique(rows[r]);
    }
  }
  A.build(rows);
}

// AffineConstraints::distribute_local_to_global(local_matrix, [local_vector],
// dofs, global_matrix, [global_vector]) with use_inhomogeneities_for_rhs =
// false: condensed entries C^T K C, constrained diagonals += |K_ii| (or the
// mean |K_jj| when K_ii == 0), rhs_t += w f_i, inhomogeneities lifted into
// unconstrained rows: rhs_r -= K_rj g_j.
//
// [r0, r1): only the global rows in this range are written (every entry of
// such a row gets its contributions in the same order as with the full range).
// Threads that own disjoint row ranges and each walk all cells in cell order
// therefore produce bitwise the serial copier's result (assemble_ordered).
void distribute_local_to_global(const Cons& cons, int dpc, const int* dofs, const double* K,
                                const double* f, Csr* A, double* rhs, int r0 = 0,
                                int r1 = INT32_MAX) {
  std::vector<std::pair<int, double>> ei, ej;
  bool any_constrained = false;
  for (int i = 0; i < dpc; ++i) any_constrained |= cons.constrained(dofs[i]);
  auto own = [&](int r) { return r >= r0 && r < r1; };
  for (int i = 0; i < dpc; ++i) {
    expand(cons, dofs[i], ei);
    bool any_own = false;
    for (const auto& a : ei) any_own |= own(a.first);
    if (!any_own) continue;
    if (A)
      for (int j = 0; j < dpc; ++j) {
        const double k = K[dpc * i + j];
        if (k == 0.0) continue;
        expand(cons, dofs[j], ej);
        for (const auto& a : ei)
          if (own(a.first))
            for (const auto& b : ej) A->at(a.first, b.first) += a.second * b.second * k;
      }
    if (rhs && f) {
      for (const auto& a : ei)
        if (own(a.first)) rhs[a.first] += a.second * f[i];
      // inhomogeneity of constrained columns j into the rows of i
      for (int j = 0; j < dpc; ++j) {
        const int l = cons.line_of[dofs[j]];
        if (l < 0 || cons.inhom[l] == 0.0) continue;
        for (const auto& a : ei)
          if (own(a.first)) rhs[a.first] -= a.second * K[dpc * i + j] * cons.inhom[l];
      }
    }
  }
  if (A && any_constrained) {
    double avg = 0;
    for (int i = 0; i < dpc; ++i) avg += std::fabs(K[dpc * i + i]);
    avg /= dpc;
    for (int i = 0; i < dpc; ++i)
      if (cons.constrained(dofs[i]) && own(dofs[i])) {
        const double kii = std::fabs(K[dpc * i + i]);
        A->at(dofs[i], dofs[i]) += (kii != 0.0 ? kii : avg);
      }
  }
}

// Cell loop of an assembly with WorkStream's result (boussinesq_model.tpp:712-734):
// element work `compute(c, K, f)` on g_threads threads in chunks of cells, then
// the copier `scatter(c, K, f, r0, r1)` by the row ranges of `split`, each thread walking the
// chunk in cell order -- bitwise the serial cell-order copier.
template <class Compute, class Scatter>
void assemble_ordered(int n_cells, size_t kmat, size_t kvec, const std::vector<int>& split,
                      Compute compute, Scatter scatter) {
  const int T = int(split.size()) - 1, W = g_threads;
  const int chunk = 128 * std::max(W, 1);
  std::vector<double> K(size_t(chunk) * kmat), f(size_t(chunk) * kvec);
  for (int c0 = 0; c0 < n_cells; c0 += chunk) {
    const int c1 = std::min(n_cells, c0 + chunk);
#pragma omp parallel for num_threads(W) schedule(dynamic, 2) if (W > 1)
    for (int c = c0; c < c1; ++c) compute(c, &K[size_t(c - c0) * kmat], &f[size_t(c - c0) * kvec]);
#pragma omp parallel for num_threads(T) schedule(static, 1) if (T > 1)
    for (int t = 0; t < T; ++t)
      for (int c = c0; c < c1; ++c)
        scatter(c, &K[size_t(c - c0) * kmat], &f[size_t(c - c0) * kvec], split[t], split[t + 1]);
  }
}

// distribute_local_to_global(local_vector, dofs, global_vector, local_matrix)
// (the matrix_for_bc variant used by assemble_temperature_rhs).
void distribute_rhs_with_bc(const Cons& cons, int dpc, const int* dofs, const double* f,
                            const double* Mbc, double* rhs) {
  for (int i = 0; i < dpc; ++i) {
    const int l = cons.line_of[dofs[i]];
    if (l < 0) {
      rhs[dofs[i]] += f[i];
      continue;
    }
    const double val = cons.inhom[l];
    if (val != 0.0)
      for (int j = 0; j < dpc; ++j) {
        const int lj = cons.line_of[dofs[j]];
        if (lj < 0) {
          rhs[dofs[j]] -= val * Mbc[dpc * j + i];
        } else {
          const double me = Mbc[dpc * j + i];
          if (me == 0.0) continue;
          for (const auto& e : cons.entries[lj]) rhs[e.first] -= val * e.second * me;
        }
      }
    for (const auto& e : cons.entries[l]) rhs[e.first] += f[i] * e.second;
  }
}

double norm2(const std::vector<double>& v, size_t b, size_t e) {
  double s = 0;
  for (size_t i = b; i < e; ++i) s += v[i] * v[i];
  return std::sqrt(s);
}

// SolverControl::check (success is tested before failure)
enum State { kIterate, kSuccess, kFailure };
struct Control {
  unsigned max_steps;
  double tol;
  unsigned last_step = 0;
  double last_value = 0;
  State check(unsigned step, double value) {
    last_step = step;
    last_value = value;
    if (value <= tol) return kSuccess;
    if (step >= max_steps || std::isnan(value)) return kFailure;
    return kIterate;
  }
};

struct NoConvergence {};

}  // namespace

struct orc_model {
  orc_physics ph;
  int n_cells, n_u, n_p, n_T, tdeg, tdpc;
  int dim = 3;  // 2: Standard::BoussinesqModel<2> (orc2d_create)
  std::vector<int> cell_nse, cell_T;
  std::vector<double> geom;
  Cons cnse, cT;
  Csr nse;  // full nse_matrix (blocks by index range)
  std::vector<double> nse_rhs;
  std::vector<double> A_diag, Mp_diag, A_inv, Mp_inv;
  Csr Tmass, Tstiff, Tmat;
  std::vector<double> T_rhs, T_inv;
  // scratch of the Schur complement (schur_complement.hpp:113)
  mutable std::vector<double> tmp1, tmp2;
  int inner_iterations = 0;
  long a_solve_iterations = 0;  // AztecOO A-GMRES iterations of the last solve (do_solve_A)
  int inner_max_steps = 5000;   // SolverControl(5000) of the inner Schur GMRES (timing hook)
  int schur_fixed_inner = 0;    // parity hook: the Schur solver's inner CGs run exactly k steps
  // the Schur solver's ILU on P MPI ranks: Trilinos' ILU with zero overlap
  // factors each rank's owned diagonal block (block Jacobi); empty: one rank
  std::vector<int> ilu_block;   // [n_u] rank owning each velocity dof
  int block_fixed_inner = 0;    // parity hook: the block preconditioner's inner GMRES runs exactly k steps
};

extern "C" orc_model* orc_create(const orc_physics* ph, int n_cells, const int* cell_nse_dofs,
                                 const int* cell_T_dofs, const double* cell_geom, int n_u, int n_p,
                                 int n_T, const orc_constraints* nse_c, const orc_constraints* T_c) {
  auto m = new orc_model();
  m->ph = *ph;
  m->n_cells = n_cells;
  m->n_u = n_u;
  m->n_p = n_p;
  m->n_T = n_T;
  m->tdeg = ph->temperature_degree;
  m->tdpc = T_dofs_per_cell(m->tdeg);
  m->cell_nse.assign(cell_nse_dofs, cell_nse_dofs + size_t(n_cells) * 89);
  m->cell_T.assign(cell_T_dofs, cell_T_dofs + size_t(n_cells) * m->tdpc);
  m->geom.assign(cell_geom, cell_geom + size_t(n_cells) * 192);
  m->cnse.init(n_u + n_p, nse_c);
  m->cT.init(n_T, T_c);
  // setup_nse_matrices (boussinesq_model.tpp:79-112): couple everything but p-p
  make_pattern(m->nse, n_u + n_p, n_cells, 89, m->cell_nse.data(), m->cnse,
               [](int i, int j) { return !(sysdof(i).comp == 3 && sysdof(j).comp == 3); });
  m->nse_rhs.assign(n_u + n_p, 0.0);
  // setup_temperature_matrices (:153-180): full coupling
  make_pattern(m->Tmass, n_T, n_cells, m->tdpc, m->cell_T.data(), m->cT,
               [](int, int) { return true; });
  m->Tstiff = m->Tmass;
  m->Tmat = m->Tmass;
  m->T_rhs.assign(n_T, 0.0);
  m->tmp1.assign(n_u, 0.0);
  m->tmp2.assign(n_u, 0.0);
  return m;
}

extern "C" void orc_destroy(orc_model* m) { delete m; }
extern "C" void orc_set_time_step(orc_model* m, double dt) { m->ph.time_step = dt; }

namespace {
void gather(const std::vector<int>& cd, size_t c, int dpc, const double* src, double* out) {
  for (int i = 0; i < dpc; ++i) out[i] = src[cd[c * dpc + i]];
}
}  // namespace

void orc2d_assemble_nse_system(orc_model* m, const double* old_nse, const double* old_T);
extern "C" void orc2d_cell_nse_preconditioner(const orc_physics* ph, const double* geom16, double* P);
void orc2d_assemble_temperature_matrix(orc_model* m);
void orc2d_assemble_temperature_rhs(orc_model* m, const double* old_T, const double* nse_solution);

extern "C" void orc_assemble_nse_system(orc_model* m, const double* old_nse, const double* old_T) {
  // assemble_nse_system (:691-740); the four unused block matrices of :700-704 (Q22) are not kept.
  // WorkStream (:712-734): local_assemble_nse_system per cell, copy_local_to_global_nse_system
  // (:677-687) in cell order; on g_threads threads bitwise the serial loop (assemble_ordered).
  if (m->dim == 2) return orc2d_assemble_nse_system(m, old_nse, old_T);
  m->nse.zero();
  std::fill(m->nse_rhs.begin(), m->nse_rhs.end(), 0.0);
  assemble_ordered(
      m->n_cells, 89 * 89, 89, row_split(m->nse.rowptr, m->nse.n, g_threads),
      [&](int c, double* K, double* f) {
        double ul[89], Tl[27];
        gather(m->cell_nse, c, 89, old_nse, ul);
        gather(m->cell_T, c, m->tdpc, old_T, Tl);
        orc_cell_nse_system(&m->ph, &m->geom[192 * size_t(c)], ul, Tl, K, f);
      },
      [&](int c, const double* K, const double* f, int r0, int r1) {
        distribute_local_to_global(m->cnse, 89, &m->cell_nse[89 * size_t(c)], K, f, &m->nse,
                                   m->nse_rhs.data(), r0, r1);
      });
}

extern "C" void orc_assemble_nse_system_threads(orc_model* m, const double* old_nse,
                                                const double* old_T, int threads) {
  // orc_assemble_nse_system on `threads` threads (bench.py's cpu_baseline legs)
  const int keep = g_threads;
  g_threads = threads > 1 ? threads : 1;
  orc_assemble_nse_system(m, old_nse, old_T);
  g_threads = keep;
}

extern "C" void orc_set_inner_max_steps(orc_model* m, int n) { m->inner_max_steps = n; }
extern "C" void orc_set_schur_fixed_inner(orc_model* m, int k) { m->schur_fixed_inner = k; }
extern "C" void orc_set_ilu_blocks(orc_model* m, const int* owner) {
  if (owner) m->ilu_block.assign(owner, owner + m->n_u);
  else m->ilu_block.clear();
}
extern "C" void orc_set_block_fixed_inner(orc_model* m, int k) { m->block_fixed_inner = k; }

extern "C" void orc_build_nse_preconditioner(orc_model* m) {
  // assemble_nse_preconditioner (:479-514) + build_nse_preconditioner (:518-542).
  // Only the diagonals of block(0,0) / block(1,1) are consumed (Ifpack point
  // Jacobi), so the condensed diagonal is accumulated directly. A pair of
  // unconstrained local dofs i != j never lands on a diagonal, so only the
  // other pairs are walked (the same additions in the same order).
  m->A_diag.assign(m->n_u, 0.0);
  m->Mp_diag.assign(m->n_p, 0.0);
  const int npc = m->dim == 2 ? 22 : 89, ngeom = m->dim == 2 ? 32 : 192;
  std::vector<std::pair<int, double>> ei, ej;
  assemble_ordered(
      m->n_cells, size_t(npc) * npc, 0, {0, m->n_u + m->n_p},
      [&](int c, double* P, double*) {
        if (m->dim == 2)
          orc2d_cell_nse_preconditioner(&m->ph, &m->geom[ngeom * size_t(c)], P);
        else
          orc_cell_nse_preconditioner(&m->ph, &m->geom[ngeom * size_t(c)], P);
      },
      [&](int c, const double* P, const double*, int, int) {
        const int* d = &m->cell_nse[npc * size_t(c)];
        bool any = false;
        for (int i = 0; i < npc; ++i) any |= m->cnse.constrained(d[i]);
        for (int i = 0; i < npc; ++i) {
          const bool ci = m->cnse.constrained(d[i]);
          for (int j = 0; j < npc; ++j) {
            const double k = P[npc * i + j];
            if (k == 0.0) continue;
            if (!ci && !m->cnse.constrained(d[j]) && d[i] != d[j]) continue;
            expand(m->cnse, d[i], ei);
            expand(m->cnse, d[j], ej);
            for (const auto& a : ei)
              for (const auto& b : ej)
                if (a.first == b.first) {
                  if (a.first < m->n_u)
                    m->A_diag[a.first] += a.second * b.second * k;
                  else
                    m->Mp_diag[a.first - m->n_u] += a.second * b.second * k;
                }
          }
        }
        if (any) {
          double avg = 0;
          for (int i = 0; i < npc; ++i) avg += std::fabs(P[npc * i + i]);
          avg /= npc;
          for (int i = 0; i < npc; ++i)
            if (m->cnse.constrained(d[i])) {
              const double kii = std::fabs(P[npc * i + i]);
              const double v = kii != 0.0 ? kii : avg;
              if (d[i] < m->n_u) m->A_diag[d[i]] += v; else m->Mp_diag[d[i] - m->n_u] += v;
            }
        }
      });
  m->A_inv.resize(m->n_u);
  m->Mp_inv.resize(m->n_p);
  for (int i = 0; i < m->n_u; ++i) m->A_inv[i] = 1.0 / m->A_diag[i];
  for (int i = 0; i < m->n_p; ++i) m->Mp_inv[i] = 1.0 / m->Mp_diag[i];
}

extern "C" void orc_assemble_temperature_matrix(orc_model* m) {
  // :821-864
  if (m->dim == 2) return orc2d_assemble_temperature_matrix(m);
  m->Tmass.zero();
  m->Tstiff.zero();
  const int n = m->tdpc;
  assemble_ordered(
      m->n_cells, size_t(2 * n * n), 0, row_split(m->Tmass.rowptr, m->n_T, g_threads),
      [&](int c, double* MK, double*) {
        orc_cell_temperature_matrix(&m->ph, &m->geom[192 * size_t(c)], MK, MK + n * n);
      },
      [&](int c, const double* MK, const double*, int r0, int r1) {
        const int* d = &m->cell_T[size_t(n) * c];
        distribute_local_to_global(m->cT, n, d, MK, nullptr, &m->Tmass, nullptr, r0, r1);
        distribute_local_to_global(m->cT, n, d, MK + n * n, nullptr, &m->Tstiff, nullptr, r0, r1);
      });
}

extern "C" void orc_assemble_temperature_rhs(orc_model* m, const double* old_T,
                                             const double* nse_solution) {
  // :966-1020: T_matrix = M + dt/interval K, Jacobi rebuilt (:975-986)
  const double dt_eff = m->ph.time_step / m->ph.nse_solver_interval;
  for (size_t k = 0; k < m->Tmat.vals.size(); ++k)
    m->Tmat.vals[k] = m->Tmass.vals[k] + dt_eff * m->Tstiff.vals[k];
  m->T_inv.assign(m->n_T, 0.0);
  for (int r = 0; r < m->n_T; ++r) m->T_inv[r] = 1.0 / m->Tmat.at(r, r);
  std::fill(m->T_rhs.begin(), m->T_rhs.end(), 0.0);
  if (m->dim == 2) return orc2d_assemble_temperature_rhs(m, old_T, nse_solution);
  const int n = m->tdpc;
  assemble_ordered(
      m->n_cells, size_t(n * n), size_t(n), {0, m->n_T},
      [&](int c, double* mfbc, double* rhs) {
        const int* d = &m->cell_T[size_t(n) * c];
        double Tl[27], ul[89];
        int mask[27];
        gather(m->cell_T, c, n, old_T, Tl);
        gather(m->cell_nse, c, 89, nse_solution, ul);
        for (int i = 0; i < n; ++i)
          mask[i] = m->cT.constrained(d[i]) && m->cT.inhom[m->cT.line_of[d[i]]] != 0.0;
        orc_cell_temperature_rhs(&m->ph, &m->geom[192 * size_t(c)], Tl, ul, mask, rhs, mfbc);
      },
      [&](int c, const double* mfbc, const double* rhs, int, int) {
        distribute_rhs_with_bc(m->cT, n, &m->cell_T[size_t(n) * c], rhs, mfbc, m->T_rhs.data());
      });
}

extern "C" long orc_nse_matrix_nnz(const orc_model* m) { return long(m->nse.cols.size()); }
extern "C" void orc_nse_matrix_csr(const orc_model* m, int* rowptr, int* cols, double* vals) {
  std::copy(m->nse.rowptr.begin(), m->nse.rowptr.end(), rowptr);
  std::copy(m->nse.cols.begin(), m->nse.cols.end(), cols);
  std::copy(m->nse.vals.begin(), m->nse.vals.end(), vals);
}
// One block of nse_matrix (which: 0 = (0,0) A, 1 = (0,1) B^T, 2 = (1,0) B) as
// CSR with block-local columns; rowptr NULL: return the block's nnz only.
extern "C" long orc_nse_block_csr(const orc_model* m, int which, int* rowptr, int* cols,
                                  double* vals) {
  const int nu = m->n_u, n = m->nse.n;
  const int r0 = which == 2 ? nu : 0, r1 = which == 2 ? n : nu;
  const int c0 = which == 1 ? nu : 0, c1 = which == 1 ? n : nu;
  long k = 0;
  if (rowptr) rowptr[0] = 0;
  for (int r = r0; r < r1; ++r) {
    for (int e = m->nse.rowptr[r]; e < m->nse.rowptr[r + 1]; ++e) {
      const int c = m->nse.cols[e];
      if (c < c0 || c >= c1) continue;
      if (rowptr) {
        cols[k] = c - c0;
        vals[k] = m->nse.vals[e];
      }
      ++k;
    }
    if (rowptr) rowptr[r - r0 + 1] = int(k);
  }
  return k;
}
extern "C" void orc_nse_rhs(const orc_model* m, double* out) {
  std::copy(m->nse_rhs.begin(), m->nse_rhs.end(), out);
}
extern "C" void orc_precond_diagonals(const orc_model* m, double* A, double* Mp) {
  std::copy(m->A_diag.begin(), m->A_diag.end(), A);
  std::copy(m->Mp_diag.begin(), m->Mp_diag.end(), Mp);
}
extern "C" long orc_T_matrix_nnz(const orc_model* m) { return long(m->Tmat.cols.size()); }
extern "C" void orc_T_matrix_csr(const orc_model* m, int* rowptr, int* cols, double* vals) {
  std::copy(m->Tmat.rowptr.begin(), m->Tmat.rowptr.end(), rowptr);
  std::copy(m->Tmat.cols.begin(), m->Tmat.cols.end(), cols);
  std::copy(m->Tmat.vals.begin(), m->Tmat.vals.end(), vals);
}
extern "C" void orc_T_rhs(const orc_model* m, double* out) {
  std::copy(m->T_rhs.begin(), m->T_rhs.end(), out);
}

// ===========================================================================
// Operators

namespace {

// Block SpMV pieces of the NSE matrix (TrilinosWrappers::BlockSparseMatrix):
// each block sums its row in column order; blocks are added afterwards.
// A row's entries inside [col0, col1): the NSE blocks split every row at
// column n_u (Csr::split, the first entry >= n_u, cached per boundary), so a
// block visits only its own entries, as a separately stored Trilinos block
// does. Rows are independent: g_threads > 1 splits them across threads with
// bitwise the same sums (the CPU baseline's multi-core leg).
void block_vmult(const Csr& A, int row0, int row1, int col0, int col1, const double* src,
                 double* dst, bool add) {
  const int* sp = nullptr;
  bool lo = false;
  if (col0 > 0 && col1 >= A.n) {
    sp = A.split_at(col0);
    lo = false;  // [split, end)
  } else if (col0 == 0 && col1 < A.n) {
    sp = A.split_at(col1);
    lo = true;   // [begin, split)
  }
#pragma omp parallel for num_threads(g_threads) schedule(static) if (g_threads > 1)
  for (int r = row0; r < row1; ++r) {
    int k0 = A.rowptr[r], k1 = A.rowptr[r + 1];
    if (sp) {
      if (lo) k1 = sp[r]; else k0 = sp[r];
    } else {
      const int* b = A.cols.data() + k0;
      const int* e = A.cols.data() + k1;
      k0 = int(std::lower_bound(b, e, col0) - A.cols.data());
      k1 = int(std::lower_bound(b, e, col1) - A.cols.data());
    }
    double s = 0;
    for (int k = k0; k < k1; ++k) s += A.vals[k] * src[A.cols[k] - col0];
    if (add) dst[r - row0] += s; else dst[r - row0] = s;
  }
}

void nse_vmult(const orc_model* m, const double* src, double* dst) {
  // BlockSparseMatrix::vmult: block(0,0) then vmult_add block(0,1); block(1,0)
  // then vmult_add block(1,1) (empty but for the constrained pressure dofs'
  // diagonal, e.g. the cuboid's periodic images)
  const int nu = m->n_u, np = m->n_p;
  block_vmult(m->nse, 0, nu, 0, nu, src, dst, false);
  block_vmult(m->nse, 0, nu, nu, nu + np, src + nu, dst, true);
  block_vmult(m->nse, nu, nu + np, 0, nu, src, dst + nu, false);
  block_vmult(m->nse, nu, nu + np, nu, nu + np, src + nu, dst + nu, true);
}

void schur_vmult(const orc_model* m, const double* src, double* dst) {
  // SchurComplement::vmult (schur_complement.hpp:143-150) with the A-Jacobi (Q9)
  const int nu = m->n_u, np = m->n_p;
  block_vmult(m->nse, 0, nu, nu, nu + np, src, m->tmp1.data(), false);   // block_01
  for (int i = 0; i < nu; ++i) m->tmp2[i] = m->tmp1[i] * m->A_inv[i];    // Jacobi
  block_vmult(m->nse, nu, nu + np, 0, nu, m->tmp2.data(), dst, false);   // block_10
}

double dotv(const double* a, const double* b, int n) {
  double s = 0;
  for (int i = 0; i < n; ++i) s += a[i] * b[i];
  return s;
}

// Givens rotation of deal.II SolverGMRES::givens_rotation
void givens_rotation(std::vector<double>& h, std::vector<double>& b, std::vector<double>& ci,
                     std::vector<double>& si, int col) {
  for (int i = 0; i < col; i++) {
    const double s = si[i], c = ci[i], dummy = h[i];
    h[i] = c * dummy + s * h[i + 1];
    h[i + 1] = -s * dummy + c * h[i + 1];
  }
  const double r = 1. / std::sqrt(h[col] * h[col] + h[col + 1] * h[col + 1]);
  si[col] = h[col + 1] * r;
  ci[col] = h[col] * r;
  h[col] = ci[col] * h[col] + si[col] * h[col + 1];
  b[col + 1] = -si[col] * b[col];
  b[col] *= ci[col];
}

// deal.II SolverGMRES (left preconditioning, use_default_residual, 30 tmp
// vectors -> restart 28, modified Gram-Schmidt with add_and_dot and the
// every-5th-step re-orthogonalisation test). Throws NoConvergence.
template <class OpA, class OpP>
void gmres(int n, OpA A, OpP P, double* x, const double* b, Control& ctl, int& iters_out,
           int n_tmp = 30) {
  std::vector<std::vector<double>> tv(n_tmp, std::vector<double>(n, 0.0));
  std::vector<double>& v = tv[0];
  std::vector<double>& p = tv[n_tmp - 1];
  std::vector<std::vector<double>> H(n_tmp, std::vector<double>(n_tmp - 1, 0.0));
  std::vector<double> gamma(n_tmp, 0.0), ci(n_tmp - 1, 0.0), si(n_tmp - 1, 0.0), h(n_tmp - 1, 0.0);
  unsigned accumulated = 0;
  int dim = 0;
  State state = kIterate;
  bool re_orthogonalize = false;
  do {
    std::fill(h.begin(), h.end(), 0.0);
    A(x, p.data());
    for (int i = 0; i < n; ++i) p[i] = -1. * p[i] + 1. * b[i];
    P(p.data(), v.data());
    double rho = std::sqrt(dotv(v.data(), v.data(), n));
    state = ctl.check(accumulated, rho);
    if (state != kIterate) break;
    gamma[0] = rho;
    for (int i = 0; i < n; ++i) v[i] *= 1. / rho;
    for (int inner = 0; inner < n_tmp - 2 && state == kIterate; ++inner) {
      ++accumulated;
      std::vector<double>& vv = tv[inner + 1];
      A(tv[inner].data(), p.data());
      P(p.data(), vv.data());
      dim = inner + 1;
      // modified_gram_schmidt
      double norm_vv_start = 0;
      const bool consider_reorth = (!re_orthogonalize) && (inner % 5 == 4);
      if (consider_reorth) norm_vv_start = std::sqrt(dotv(vv.data(), vv.data(), n));
      h[0] = dotv(vv.data(), tv[0].data(), n);
      for (int i = 1; i < dim; ++i) {
        // add_and_dot(-h(i-1), v[i-1], v[i])
        double s = 0;
        const double a = -h[i - 1];
        for (int k = 0; k < n; ++k) {
          vv[k] += a * tv[i - 1][k];
          s += vv[k] * tv[i][k];
        }
        h[i] = s;
      }
      double nn = 0;
      {
        const double a = -h[dim - 1];
        for (int k = 0; k < n; ++k) {
          vv[k] += a * tv[dim - 1][k];
          nn += vv[k] * vv[k];
        }
      }
      double norm_vv = std::sqrt(nn);
      bool do_second = false;
      if (consider_reorth) {
        if (norm_vv > 10. * norm_vv_start * std::sqrt(2.220446049250313e-16)) {
          // keep
        } else {
          re_orthogonalize = true;
          do_second = true;
        }
      } else if (re_orthogonalize) {
        do_second = true;
      }
      if (do_second) {
        // second pass: classical correction, as in deal.II
        double htmp = dotv(vv.data(), tv[0].data(), n);
        h[0] += htmp;
        for (int i = 1; i < dim; ++i) {
          double s = 0;
          const double a = -htmp;
          for (int k = 0; k < n; ++k) {
            vv[k] += a * tv[i - 1][k];
            s += vv[k] * tv[i][k];
          }
          htmp = s;
          h[i] += htmp;
        }
        nn = 0;
        const double a = -htmp;
        for (int k = 0; k < n; ++k) {
          vv[k] += a * tv[dim - 1][k];
          nn += vv[k] * vv[k];
        }
        norm_vv = std::sqrt(nn);
      }
      const double s = norm_vv;
      h[inner + 1] = s;
      if (s != 0)
        for (int k = 0; k < n; ++k) vv[k] *= 1. / s;
      givens_rotation(h, gamma, ci, si, inner);
      for (int i = 0; i < dim; ++i) H[i][inner] = h[i];
      rho = std::fabs(gamma[dim]);
      state = ctl.check(accumulated, rho);
    }
    // H1.backward(h, gamma)
    std::vector<double> y(dim, 0.0);
    for (int i = dim - 1; i >= 0; --i) {
      double s = gamma[i];
      for (int j = i + 1; j < dim; ++j) s -= y[j] * H[i][j];
      y[i] = s / H[i][i];
    }
    for (int i = 0; i < dim; ++i)
      for (int k = 0; k < n; ++k) x[k] += y[i] * tv[i][k];
  } while (state == kIterate);
  iters_out = int(ctl.last_step);
  if (state != kSuccess) throw NoConvergence();
}

// TrilinosWrappers::SolverGMRES (block_schur_preconditioner.hpp:59-67; LA =
// TrilinosWrappers, base/config.h:20-28) -> AztecOO's AZ_gmres, restated from
// the published AztecOO algorithm (Trilinos az_gmres.c) with the options
// deal.II's SolverBase::do_solve sets: AZ_kspace = restart parameter (default
// 30), AZ_conv = AZ_noscaled (absolute |r|_2), AZ_orthog = AZ_classic
// (classical Gram-Schmidt with one re-orthogonalisation pass), the
// preconditioner applied from the RIGHT (v_{i+1} = A M^-1 v_i, x += M^-1 V y).
// The recursive residual ends an Arnoldi cycle; convergence is then confirmed
// on the true residual b - A x (a cycle whose true residual misses the
// tolerance continues, AztecOO's loss-of-precision path). deal.II finally
// checks the true residual: SolverControl::check(NumIters, TrueResidual),
// NoConvergence when it exceeds the tolerance.
template <class OpA, class OpP>
void aztec_gmres(int n, OpA A, OpP Minv, double* x, const double* b, double tol, int max_it,
                 int kspace, int& iters_out) {
  std::vector<std::vector<double>> v(kspace + 1, std::vector<double>(n, 0.0));
  std::vector<double> r(n), z(n), w(n);
  std::vector<std::vector<double>> H(kspace + 1, std::vector<double>(kspace, 0.0));
  std::vector<double> rs(kspace + 1, 0.0), cs(kspace, 0.0), sn(kspace, 0.0), h(kspace + 1, 0.0);
  auto residual = [&]() {
    A(x, r.data());
    for (int k = 0; k < n; ++k) r[k] = b[k] - r[k];
    return std::sqrt(dotv(r.data(), r.data(), n));
  };
  double rnorm = residual();
  // <= as SolverControl: a zero rhs (tol 0) with a zero residual is converged
  bool converged = rnorm <= tol;
  int iter = 0;
  while (!converged && iter < max_it) {
    for (int k = 0; k < n; ++k) v[0][k] = r[k] / rnorm;
    rs[0] = rnorm;
    int i = 0;
    bool cycle_converged = false;
    while (i < kspace && !cycle_converged && iter < max_it) {
      ++iter;
      Minv(v[i].data(), z.data());
      A(z.data(), w.data());
      for (int pass = 0; pass < 2; ++pass) {  // classical Gram-Schmidt, twice
        std::vector<double> c(i + 1);
        for (int k = 0; k <= i; ++k) c[k] = dotv(v[k].data(), w.data(), n);
        for (int k = 0; k <= i; ++k)
          for (int q = 0; q < n; ++q) w[q] -= c[k] * v[k][q];
        for (int k = 0; k <= i; ++k) h[k] = pass ? h[k] + c[k] : c[k];
      }
      const double hn = std::sqrt(dotv(w.data(), w.data(), n));
      h[i + 1] = hn;
      if (hn != 0)
        for (int q = 0; q < n; ++q) v[i + 1][q] = w[q] / hn;
      for (int k = 0; k < i; ++k) {  // previous plane rotations
        const double t = h[k];
        h[k] = cs[k] * t + sn[k] * h[k + 1];
        h[k + 1] = cs[k] * h[k + 1] - sn[k] * t;
      }
      const double d = std::sqrt(h[i] * h[i] + h[i + 1] * h[i + 1]);
      cs[i] = d != 0 ? h[i] / d : 1.0;  // d = 0: an exact breakdown, no rotation
      sn[i] = d != 0 ? h[i + 1] / d : 0.0;
      rs[i + 1] = -sn[i] * rs[i];
      rs[i] = cs[i] * rs[i];
      h[i] = cs[i] * h[i] + sn[i] * h[i + 1];
      for (int k = 0; k <= i; ++k) H[k][i] = h[k];
      cycle_converged = std::fabs(rs[i + 1]) <= tol;
      ++i;
    }
    // y = H^-1 rs (upper triangular), x += M^-1 (V y)
    std::vector<double> y(i, 0.0);
    for (int k = i - 1; k >= 0; --k) {
      double t = rs[k];
      for (int j = k + 1; j < i; ++j) t -= H[k][j] * y[j];
      y[k] = t / H[k][k];
    }
    std::fill(w.begin(), w.end(), 0.0);
    for (int k = 0; k < i; ++k)
      for (int q = 0; q < n; ++q) w[q] += y[k] * v[k][q];
    Minv(w.data(), z.data());
    for (int q = 0; q < n; ++q) x[q] += z[q];
    rnorm = residual();
    converged = cycle_converged && rnorm <= tol;
  }
  iters_out = iter;
  if (!(rnorm <= tol)) throw NoConvergence();
}

// deal.II Householder<double> (initialize + least_squares).
double householder_least_squares(std::vector<std::vector<double>> S, int m, int n,
                                 std::vector<double>& dst, const std::vector<double>& src) {
  std::vector<double> diagonal(m, 0.0);
  for (int j = 0; j < n; ++j) {
    double sigma = 0;
    for (int i = j; i < m; ++i) sigma += S[i][j] * S[i][j];
    if (std::fabs(sigma) < 1.e-15) break;
    const double s = (S[j][j] < 0) ? std::sqrt(sigma) : -std::sqrt(sigma);
    const double beta = std::sqrt(1. / (sigma - s * S[j][j]));
    diagonal[j] = beta * (S[j][j] - s);
    S[j][j] = s;
    for (int i = j + 1; i < m; ++i) S[i][j] *= beta;
    for (int k = j + 1; k < n; ++k) {
      double sum = diagonal[j] * S[j][k];
      for (int i = j + 1; i < m; ++i) sum += S[i][j] * S[i][k];
      S[j][k] -= sum * diagonal[j];
      for (int i = j + 1; i < m; ++i) S[i][k] -= sum * S[i][j];
    }
  }
  std::vector<double> aux = src;
  for (int j = 0; j < n; ++j) {
    double sum = diagonal[j] * aux[j];
    for (int i = j + 1; i < m; ++i) sum += S[i][j] * aux[i];
    aux[j] -= sum * diagonal[j];
    for (int i = j + 1; i < m; ++i) aux[i] -= sum * S[i][j];
  }
  double sum = 0;
  for (int i = n; i < m; ++i) sum += aux[i] * aux[i];
  dst.assign(n, 0.0);
  for (int i = n - 1; i >= 0; --i) {
    double s = aux[i];
    for (int j = i + 1; j < n; ++j) s -= dst[j] * S[i][j];
    dst[i] = s / S[i][i];
  }
  return std::sqrt(sum);
}

// BlockSchurPreconditioner::vmult (block_schur_preconditioner.hpp:42-70)
void block_prec_vmult(orc_model* m, const double* src, double* dst, bool do_solve_A, int& inner) {
  const int nu = m->n_u, np = m->n_p;
  std::vector<double> utmp(src, src + nu);
  {
    // parity hook (block_fixed_inner = k, the device's DCP_OPT_BLOCK_FIXED_INNER):
    // exactly k steps, no tolerance test, the k-step iterate used as is
    const int fk = m->block_fixed_inner;
    Control ctl = fk > 0 ? Control{unsigned(fk), 0.0}
                         : Control{unsigned(m->inner_max_steps),
                                   1e-6 * norm2(std::vector<double>(src + nu, src + nu + np), 0, np)};
    int it = 0;
    try {
      gmres(
          np, [&](const double* x, double* y) { schur_vmult(m, x, y); },
          [&](const double* x, double* y) { std::copy(x, x + np, y); }, dst + nu, src + nu, ctl,
          it);
    } catch (const NoConvergence&) {
      inner += it;  // count the failed solve's iterations too (as the device path does)
      if (fk <= 0) throw;
      it = 0;
    }
    inner += it;
    for (int i = 0; i < np; ++i) dst[nu + i] *= -1.0;
  }
  {
    block_vmult(m->nse, 0, nu, nu, nu + np, dst + nu, utmp.data(), false);
    for (int i = 0; i < nu; ++i) utmp[i] *= -1.0;
    for (int i = 0; i < nu; ++i) utmp[i] += src[i];
  }
  if (do_solve_A) {
    // LA::SolverGMRES = AztecOO GMRES(30) with the A-Jacobi (Ifpack point
    // Jacobi) from the right, absolute tol 1e-2 ||utmp||, <= 5000 (:59-67);
    // initial guess: what dst's velocity block holds.
    int it = 0;
    aztec_gmres(
        nu, [&](const double* x, double* y) { block_vmult(m->nse, 0, nu, 0, nu, x, y, false); },
        [&](const double* x, double* y) { for (int i = 0; i < nu; ++i) y[i] = x[i] * m->A_inv[i]; },
        dst, utmp.data(), norm2(utmp, 0, nu) * 1e-2, 5000, 30, it);
    m->a_solve_iterations += it;
  } else {
    for (int i = 0; i < nu; ++i) dst[i] = utmp[i] * m->A_inv[i];
  }
}

// deal.II SolverFGMRES (restated; Householder least squares every step from
// j = 1, solution update with the first y.size() z vectors; z vectors persist
// across restarts within one solve and are zero on first use).
State fgmres(orc_model* m, double* x, const double* b, int basis_size, unsigned max_steps,
             double tol, bool do_solve_A, int& accumulated_out, int& inner) {
  const int n = m->n_u + m->n_p;
  Control ctl{max_steps, tol};
  std::vector<std::vector<double>> v(basis_size), z(basis_size);
  std::vector<double> aux(n);
  unsigned accumulated = 0;
  State state = kIterate;
  std::vector<std::vector<double>> H;
  std::vector<double> y;
  double res = 0;
  do {
    nse_vmult(m, x, aux.data());
    for (int i = 0; i < n; ++i) aux[i] = -1. * aux[i] + 1. * b[i];
    const double beta = std::sqrt(dotv(aux.data(), aux.data(), n));
    res = beta;
    state = ctl.check(accumulated, res);
    if (state == kSuccess) break;
    H.assign(basis_size + 1, std::vector<double>(basis_size, 0.0));
    double a = beta;
    y.clear();
    for (int j = 0; j < basis_size; ++j) {
      if (v[j].empty()) v[j].assign(n, 0.0);
      if (z[j].empty()) z[j].assign(n, 0.0);
      if (a != 0)
        for (int i = 0; i < n; ++i) v[j][i] = 1. / a * aux[i];
      else
        std::fill(v[j].begin(), v[j].end(), 0.0);
      block_prec_vmult(m, v[j].data(), z[j].data(), do_solve_A, inner);
      nse_vmult(m, z[j].data(), aux.data());
      H[0][j] = dotv(aux.data(), v[0].data(), n);
      for (int i = 1; i <= j; ++i) {
        double s = 0;
        const double c = -H[i - 1][j];
        for (int k = 0; k < n; ++k) {
          aux[k] += c * v[i - 1][k];
          s += aux[k] * v[i][k];
        }
        H[i][j] = s;
      }
      {
        double s = 0;
        const double c = -H[j][j];
        for (int k = 0; k < n; ++k) {
          aux[k] += c * v[j][k];
          s += aux[k] * aux[k];
        }
        H[j + 1][j] = a = std::sqrt(s);
      }
      if (j > 0) {
        std::vector<std::vector<double>> H1(j + 1, std::vector<double>(j, 0.0));
        for (int r = 0; r <= j; ++r)
          for (int c = 0; c < j; ++c) H1[r][c] = H[r][c];
        std::vector<double> prhs(j + 1, 0.0);
        prhs[0] = beta;
        res = householder_least_squares(H1, j + 1, j, y, prhs);
        state = ctl.check(++accumulated, res);
        if (state != kIterate) break;
      }
    }
    for (size_t j = 0; j < y.size(); ++j)
      for (int k = 0; k < n; ++k) x[k] += y[j] * z[j][k];
  } while (state == kIterate);
  accumulated_out = int(ctl.last_step);
  return state;
}

}  // namespace

extern "C" void orc_set_threads(int n) { g_threads = n > 1 ? n : 1; }

extern "C" void orc_nse_vmult(const orc_model* m, const double* src, double* dst) {
  nse_vmult(m, src, dst);
}
extern "C" void orc_schur_vmult(const orc_model* m, const double* src, double* dst) {
  schur_vmult(m, src, dst);
}
extern "C" void orc_block_preconditioner_vmult(orc_model* m, const double* src, double* dst,
                                               int do_solve_A, int* inner_iterations) {
  int inner = 0;
  try {
    block_prec_vmult(m, src, dst, do_solve_A != 0, inner);
  } catch (const NoConvergence&) {
    inner = -1;
  }
  if (inner_iterations) *inner_iterations = inner;
}

extern "C" int orc_solve_nse(orc_model* m, double* sol, int* outer_it, int* inner_it,
                             int max_outer) {
  // solve_NSE_block_preconditioned (boussinesq_model.tpp:1131-1245)
  const int nu = m->n_u, np = m->n_p, n = nu + np;
  if (int(m->A_inv.size()) != nu || int(m->Mp_inv.size()) != np) return -4;  // no preconditioner yet
  const double dt = m->ph.time_step;
  std::vector<double> x(sol, sol + n);
  for (int i = nu; i < n; ++i) x[i] *= dt;                         // :1151
  for (int i = nu; i < n; ++i) if (m->cnse.constrained(i)) x[i] = 0;  // :1153-1161
  const double tol = 1e-8 * norm2(m->nse_rhs, 0, n);               // :1165
  for (int i = nu; i < n; ++i) x[i] *= dt;                         // :1177 (Q1)
  int inner = 0, acc1 = 0, acc2 = 0;
  int status = 0;
  m->a_solve_iterations = 0;
  try {
    State s = fgmres(m, x.data(), m->nse_rhs.data(), 30, unsigned(max_outer), tol, false, acc1, inner);
    if (s != kSuccess) throw NoConvergence();
  } catch (const NoConvergence&) {
    // :1203-1232 fallback (Q10): do_solve_A, FGMRES(50), max_it = n
    try {
      State s = fgmres(m, x.data(), m->nse_rhs.data(), 50, unsigned(n), tol, true, acc2, inner);
      if (s != kSuccess) status = 1;
    } catch (const NoConvergence&) {
      status = 1;
    }
  }
  m->cnse.distribute(x.data());                                     // :1233
  for (int i = nu; i < n; ++i) x[i] /= dt;                         // :1239
  std::copy(x.begin(), x.end(), sol);
  if (outer_it) *outer_it = acc1 + acc2;
  if (inner_it) *inner_it = inner;
  m->inner_iterations = inner;
  return status;
}

// Timing hook (bench cpu_baseline): the first FGMRES(30) of
// solve_NSE_block_preconditioned cut at k outer iterations (SolverControl(k)),
// no fallback; the initial guess as the solve sets it up. Returns the
// iterations done, inner Schur GMRES iterations to *inner_it.
// CPU baseline sample of the inner Schur GMRES at any size, on given coupling
// blocks: deal.II's SolverGMRES (modified Gram-Schmidt, restart 28) on
// S = B (D_A^-1 (B^T p)) (schur_complement.hpp:143-150 with the A-Jacobi, Q9),
// held at exactly k steps; the CSR products row-parallel on g_threads threads
// (Epetra's row-distributed SpMV). Bt: n_u x n_p, B: n_p x n_u (block-local
// columns), A_inv: n_u. Returns the wall seconds of the k steps; dst_p gets the
// iterate.
extern "C" double orc_schur_gmres_sample(int n_u, int n_p, const int* bt_ptr, const int* bt_col,
                                         const double* bt_val, const int* b_ptr, const int* b_col,
                                         const double* b_val, const double* A_inv,
                                         const double* src_p, double* dst_p, int k) {
  std::vector<double> t1(n_u), t2(n_u);
  auto csr = [](int rows, const int* rp, const int* cl, const double* v, const double* x,
                double* y) {
#pragma omp parallel for num_threads(g_threads) schedule(static) if (g_threads > 1)
    for (int r = 0; r < rows; ++r) {
      double s = 0;
      for (int e = rp[r]; e < rp[r + 1]; ++e) s += v[e] * x[cl[e]];
      y[r] = s;
    }
  };
  std::fill(dst_p, dst_p + n_p, 0.0);
  Control ctl{unsigned(k), 0.0};
  int it = 0;
  const auto t0 = std::chrono::steady_clock::now();
  try {
    gmres(
        n_p,
        [&](const double* x, double* y) {
          csr(n_u, bt_ptr, bt_col, bt_val, x, t1.data());
          for (int i = 0; i < n_u; ++i) t2[i] = t1[i] * A_inv[i];
          csr(n_p, b_ptr, b_col, b_val, t2.data(), y);
        },
        [&](const double* x, double* y) { std::copy(x, x + n_p, y); }, dst_p, src_p, ctl, it);
  } catch (const NoConvergence&) {
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

extern "C" int orc_fgmres_outer(orc_model* m, const double* sol, int k, int* inner_it) {
  const int nu = m->n_u, np = m->n_p, n = nu + np;
  const double dt = m->ph.time_step;
  std::vector<double> x(sol, sol + n);
  for (int i = nu; i < n; ++i) x[i] *= dt * dt;  // :1151, :1177 (Q1)
  const double tol = 1e-8 * norm2(m->nse_rhs, 0, n);
  int inner = 0, acc = 0;
  try {
    (void)fgmres(m, x.data(), m->nse_rhs.data(), 30, unsigned(k), tol, false, acc, inner);
  } catch (const NoConvergence&) {
  }
  if (inner_it) *inner_it = inner;
  return acc;
}

extern "C" long orc_a_solve_iterations(const orc_model* m) { return m->a_solve_iterations; }

namespace {
// y = block (rows [r0, r1), cols [c0, c1)) of A times x (x indexed from c0)
void csr_block(const Csr& A, int r0, int r1, int c0, int c1, const double* x, double* y, bool add) {
  for (int r = r0; r < r1; ++r) {
    double acc = 0;
    for (int k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k)
      if (A.cols[k] >= c0 && A.cols[k] < c1) acc += A.vals[k] * x[A.cols[k] - c0];
    y[r - r0] = add ? y[r - r0] + acc : acc;
  }
}

// LA::PreconditionILU (linear_algebra/preconditioner.h:40) =
// TrilinosWrappers::PreconditionILU with its default AdditionalData
// (ilu_fill 0, ilu_atol 0, ilu_rtol 1, overlap 0): ILU(0) of
// nse_matrix.block(0,0) on its own pattern. Restated as the row-wise IKJ
// elimination (l_ik = a_ik / u_kk in column order k, then a_ij -= l_ik u_kj on
// the pattern of row i); apply: unit-lower forward, upper backward (division
// by u_ii), a row summed as 64 lane-strided partial sums combined by an xor
// butterfly (the device's wave-per-row order). Ifpack's CrsRiluk is not in
// this image, so the operation order against Trilinos is unpinned.
double row_sum64(const std::vector<double>& val, const std::vector<int>& col, int b, int e,
                 const double* x) {
  double v[64];
  for (int l = 0; l < 64; ++l) {
    v[l] = 0.0;
    for (int p = b + l; p < e; p += 64) v[l] += val[p] * x[col[p]];
  }
  for (int o = 32; o > 0; o >>= 1) {
    double w[64];
    for (int l = 0; l < 64; ++l) w[l] = v[l] + v[l ^ o];
    for (int l = 0; l < 64; ++l) v[l] = w[l];
  }
  return v[0];
}

struct Ilu0 {
  int n = 0;
  std::vector<int> ptr, col, diag;
  std::vector<double> val;
  // block: optional [rows] block id; entries between blocks are dropped (the
  // factor of each diagonal block, TrilinosWrappers::PreconditionILU with
  // overlap 0 on several ranks)
  void factor(const Csr& A, int rows, const std::vector<int>* block = nullptr) {
    n = rows;
    ptr.assign(n + 1, 0);
    col.clear();
    val.clear();
    for (int r = 0; r < n; ++r) {
      for (int k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k)
        if (A.cols[k] < n && (!block || (*block)[A.cols[k]] == (*block)[r])) {
          col.push_back(A.cols[k]);
          val.push_back(A.vals[k]);
        }
      ptr[r + 1] = int(col.size());
    }
    diag.assign(n, -1);
    for (int r = 0; r < n; ++r)
      for (int k = ptr[r]; k < ptr[r + 1]; ++k)
        if (col[k] == r) diag[r] = k;
    for (int i = 0; i < n; ++i) {
      for (int p = ptr[i]; p < ptr[i + 1] && col[p] < i; ++p) {
        const int k = col[p];
        val[p] /= val[diag[k]];
        const double lik = val[p];
        int r = p + 1;
        for (int q = diag[k] + 1; q < ptr[k + 1]; ++q) {
          while (r < ptr[i + 1] && col[r] < col[q]) ++r;
          if (r == ptr[i + 1]) break;
          if (col[r] == col[q]) val[r] -= lik * val[q];
        }
      }
    }
  }
  void apply(const double* b, double* x) const {
    for (int i = 0; i < n; ++i) x[i] = b[i] - row_sum64(val, col, ptr[i], diag[i], x);
    for (int i = n - 1; i >= 0; --i)
      x[i] = (x[i] - row_sum64(val, col, diag[i] + 1, ptr[i + 1], x)) / val[diag[i]];
  }
};

// deal.II SolverCG with a preconditioner; throws NoConvergence
template <class OpA, class OpP>
void pcg(int n, OpA A, OpP P, double* x, const double* b, Control& ctl) {
  std::vector<double> g(n), d(n), h(n);
  bool all_zero = true;
  for (int i = 0; i < n; ++i) all_zero &= (x[i] == 0.0);
  if (!all_zero) {
    A(x, g.data());
    for (int i = 0; i < n; ++i) g[i] += -1. * b[i];
  } else {
    for (int i = 0; i < n; ++i) g[i] = -1. * b[i];
  }
  double res = std::sqrt(dotv(g.data(), g.data(), n));
  State conv = ctl.check(0, res);
  if (conv == kIterate) {
    P(g.data(), h.data());
    for (int i = 0; i < n; ++i) d[i] = -1. * h[i];
    double gh = dotv(g.data(), h.data(), n);
    int it = 0;
    while (conv == kIterate) {
      it++;
      A(d.data(), h.data());
      double alpha = dotv(d.data(), h.data(), n);
      alpha = gh / alpha;
      for (int i = 0; i < n; ++i) x[i] += alpha * d[i];
      double gg = 0;
      for (int i = 0; i < n; ++i) {
        g[i] += alpha * h[i];
        gg += g[i] * g[i];
      }
      res = std::sqrt(std::fabs(gg));
      conv = ctl.check(it, res);
      if (conv != kIterate) break;
      P(g.data(), h.data());
      double beta = gh;
      gh = dotv(g.data(), h.data(), n);
      beta = gh / beta;
      for (int i = 0; i < n; ++i) d[i] = beta * d[i] - h[i];
    }
  }
  if (conv != kSuccess) throw NoConvergence();
}
}  // namespace

extern "C" int orc_solve_nse_schur(orc_model* m, double* sol, int* schur_iterations,
                                   int* a_solves) {
  // solve_NSE_Schur_complement (boussinesq_model.tpp:1248-1414)
  const int nu = m->n_u, np = m->n_p, n = nu + np;
  const double dt = m->ph.time_step;
  const Csr& M = m->nse;
  Ilu0 ilu;
  // inner_schur_preconditioner->initialize(block(0,0))
  ilu.factor(M, nu, m->ilu_block.empty() ? nullptr : &m->ilu_block);
  auto A = [&](const double* x, double* y) { csr_block(M, 0, nu, 0, nu, x, y, false); };
  auto P = [&](const double* x, double* y) { ilu.apply(x, y); };
  int n_inv = 0;
  // InverseMatrix<A, ILU>::vmult (inverse_matrix.hpp:93-120): CG, tol 1e-6 |src|,
  // max(n, 1000) steps, dst = 0, NoConvergence swallowed
  const int fk = m->schur_fixed_inner;  // > 0: both inner CGs run exactly fk steps (tol 0)
  auto inverse = [&](const double* src, double* dst) {
    Control ctl = fk > 0 ? Control{unsigned(fk), 0.0}
                         : Control{unsigned(std::max(nu, 1000)), 1e-6 * std::sqrt(dotv(src, src, nu))};
    std::fill(dst, dst + nu, 0.0);
    ++n_inv;
    try {
      pcg(nu, A, P, dst, src, ctl);
    } catch (const NoConvergence&) {
    }
  };
  std::vector<double> x(sol, sol + n), tmp(nu), t1(nu), t2(nu), srhs(np);
  for (int i = nu; i < n; ++i) x[i] *= dt;                                  // :1283
  for (int i = nu; i < n; ++i) if (m->cnse.constrained(i)) x[i] = 0;       // :1290-1292
  // schur_rhs = B A^-1 f - g (:1319-1321)
  inverse(m->nse_rhs.data(), tmp.data());
  csr_block(M, nu, n, 0, nu, tmp.data(), srhs.data(), false);
  for (int i = 0; i < np; ++i) srhs[i] -= m->nse_rhs[nu + i];
  // SchurComplement::vmult (schur_complement.hpp:143-150): B A^-1 B^T
  auto S = [&](const double* s, double* d) {
    csr_block(M, 0, nu, nu, n, s, t1.data(), false);
    inverse(t1.data(), t2.data());
    csr_block(M, nu, n, 0, nu, t2.data(), d, false);
  };
  // ApproximateSchurComplement::vmult (approximate_schur_complement.hpp:131-139): B ILU^-1 B^T
  auto Sa = [&](const double* s, double* d) {
    csr_block(M, 0, nu, nu, n, s, t1.data(), false);
    ilu.apply(t1.data(), t2.data());
    csr_block(M, nu, n, 0, nu, t2.data(), d, false);
  };
  auto identity = [&](const double* s, double* d) { std::copy(s, s + np, d); };
  // ApproximateInverseMatrix<S~, identity>(n_iter = invalid): CG, tol 1e-6 |src|
  auto precond = [&](const double* s, double* d) {
    Control ctl = fk > 0 ? Control{unsigned(fk), 0.0} : Control{~0u, 1e-6 * std::sqrt(dotv(s, s, np))};
    std::fill(d, d + np, 0.0);
    try {
      pcg(np, Sa, identity, d, s, ctl);
    } catch (const NoConvergence&) {
    }
  };
  // SolverGMRES (30 tmp vectors), SolverControl(nse_matrix.m(), 1e-6 |schur_rhs|)
  Control ctl{unsigned(n), 1e-6 * std::sqrt(dotv(srhs.data(), srhs.data(), np))};
  int its = 0, rc = 0;
  try {
    gmres(np, S, precond, x.data() + nu, srhs.data(), ctl, its);
  } catch (const NoConvergence&) {
    rc = 1;
  }
  m->cnse.distribute(x.data());                                             // :1353
  // u = A^-1 (f - B^T p) (:1366-1372)
  csr_block(M, 0, nu, nu, n, x.data() + nu, tmp.data(), false);
  for (int i = 0; i < nu; ++i) tmp[i] = -1. * tmp[i] + m->nse_rhs[i];
  inverse(tmp.data(), x.data());
  m->cnse.distribute(x.data());                                             // :1378
  for (int i = nu; i < n; ++i) x[i] /= dt;                                 // :1384
  std::copy(x.begin(), x.end(), sol);
  if (schur_iterations) *schur_iterations = int(ctl.last_step);
  if (a_solves) *a_solves = n_inv;
  return rc;
}

extern "C" int orc_solve_temperature(orc_model* m, double* T, int* iterations) {
  // solve_temperature (:1417-1476): SolverCG + Jacobi, tol 1e-12 ||rhs||, max n_T
  const int n = m->n_T;
  Control ctl{unsigned(n), 1e-12 * norm2(m->T_rhs, 0, n)};
  std::vector<double> x(T, T + n), g(n), d(n), h(n);
  const Csr& A = m->Tmat;
  auto Av = [&](const std::vector<double>& s, std::vector<double>& o) {
    for (int r = 0; r < n; ++r) {
      double acc = 0;
      for (int k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k) acc += A.vals[k] * s[A.cols[k]];
      o[r] = acc;
    }
  };
  bool all_zero = true;
  for (double v : x) all_zero &= (v == 0.0);
  if (!all_zero) {
    Av(x, g);
    for (int i = 0; i < n; ++i) g[i] += -1. * m->T_rhs[i];
  } else {
    for (int i = 0; i < n; ++i) g[i] = -1. * m->T_rhs[i];
  }
  double res = norm2(g, 0, n);
  State conv = ctl.check(0, res);
  int it = 0;
  if (conv == kIterate) {
    for (int i = 0; i < n; ++i) h[i] = g[i] * m->T_inv[i];
    for (int i = 0; i < n; ++i) d[i] = -1. * h[i];
    double gh = dotv(g.data(), h.data(), n);
    while (conv == kIterate) {
      it++;
      Av(d, h);
      double alpha = dotv(d.data(), h.data(), n);
      alpha = gh / alpha;
      for (int i = 0; i < n; ++i) x[i] += alpha * d[i];
      double gg = 0;
      for (int i = 0; i < n; ++i) {
        g[i] += alpha * h[i];
        gg += g[i] * g[i];
      }
      res = std::sqrt(std::fabs(gg));
      conv = ctl.check(it, res);
      if (conv != kIterate) break;
      for (int i = 0; i < n; ++i) h[i] = g[i] * m->T_inv[i];
      double beta = gh;
      gh = dotv(g.data(), h.data(), n);
      beta = gh / beta;
      for (int i = 0; i < n; ++i) d[i] = beta * d[i] - h[i];
    }
  }
  m->cT.distribute(x.data());
  std::copy(x.begin(), x.end(), T);
  if (iterations) *iterations = int(ctl.last_step);
  return conv == kSuccess ? 0 : 1;
}

double orc2d_max_velocity(const orc_model* m, const double* sol, const double* diam);

extern "C" double orc_max_velocity(const orc_model* m, const double* sol) {
  // get_maximal_velocity (:1023-1061) on QIterated<QTrapez>(2) = the Q2 nodes
  if (m->dim == 2) return orc2d_max_velocity(m, sol, nullptr);
  double mx = 0;
  for (int c = 0; c < m->n_cells; ++c)
    for (int n = 0; n < 27; ++n) {
      const int b = m->cell_nse[89 * size_t(c) + (n < 8 ? 4 * n : 32 + 3 * (n - 8))];
      const double u0 = sol[b], u1 = sol[b + 1], u2 = sol[b + 2];
      mx = std::max(mx, std::sqrt(u0 * u0 + u1 * u1 + u2 * u2));
    }
  return mx;
}

extern "C" double orc_cfl(const orc_model* m, const double* sol, const double* diam) {
  // get_cfl_number (:1064-1101)
  if (m->dim == 2) return orc2d_max_velocity(m, sol, diam);
  double cfl = 0;
  for (int c = 0; c < m->n_cells; ++c) {
    double mx = 1e-10;
    for (int n = 0; n < 27; ++n) {
      const int b = m->cell_nse[89 * size_t(c) + (n < 8 ? 4 * n : 32 + 3 * (n - 8))];
      const double u0 = sol[b], u1 = sol[b + 1], u2 = sol[b + 2];
      mx = std::max(mx, std::sqrt(u0 * u0 + u1 * u1 + u2 * u2));
    }
    cfl = std::max(cfl, mx / diam[c]);
  }
  return cfl;
}

// ===========================================================================
// FEEC variant: ExteriorCalculus::BoussinesqModel<3> (boussineq_model_FEEC.tpp)
// FESystem(FE_Nedelec(0), FE_RaviartThomas(0), FE_DGQ(0)) with MappingQ1; local
// dofs 0..11 edges (deal.II line order), 12..17 faces, 18 cell. Orientation
// signs (one per local dof) stand for deal.II's line orientation (Nedelec) and
// for the RT face-sign fix of utilities.cc:20-45.

namespace {

const int kLineVtx[12][2] = {{0, 2}, {1, 3}, {0, 1}, {2, 3}, {4, 6}, {5, 7},
                             {4, 5}, {6, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};

// reference coordinate d of vertex v (lexicographic)
int vbit(int v, int d) { return (v >> d) & 1; }

// MappingQ1 (trilinear) at xi: J (dx_i/dxi_j) and x
void map_q1(const double* X, const double* xi, double J[3][3], Vec3& x) {
  for (int i = 0; i < 3; ++i) {
    x[i] = 0;
    for (int j = 0; j < 3; ++j) J[i][j] = 0;
  }
  for (int v = 0; v < 8; ++v) {
    double s = 1, g[3] = {1, 1, 1};
    for (int d = 0; d < 3; ++d) {
      const double l = lag1(vbit(v, d), xi[d]), dl = dlag1(vbit(v, d), xi[d]);
      s *= l;
      for (int e = 0; e < 3; ++e) g[e] *= (e == d ? dl : l);
    }
    for (int i = 0; i < 3; ++i) {
      x[i] += X[3 * v + i] * s;
      for (int j = 0; j < 3; ++j) J[i][j] += X[3 * v + i] * g[j];
    }
  }
}

double det3(const double J[3][3]) {
  return J[0][0] * (J[1][1] * J[2][2] - J[1][2] * J[2][1]) -
         J[0][1] * (J[1][0] * J[2][2] - J[1][2] * J[2][0]) +
         J[0][2] * (J[1][0] * J[2][1] - J[1][1] * J[2][0]);
}

void inv3(const double J[3][3], double I[3][3]) {
  const double d = det3(J);
  I[0][0] = (J[1][1] * J[2][2] - J[1][2] * J[2][1]) / d;
  I[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) / d;
  I[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) / d;
  I[1][0] = (J[1][2] * J[2][0] - J[1][0] * J[2][2]) / d;
  I[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) / d;
  I[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) / d;
  I[2][0] = (J[1][0] * J[2][1] - J[1][1] * J[2][0]) / d;
  I[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) / d;
  I[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) / d;
}

// FEValues of the FEEC system element at tensor points (n1d Gauss points, or
// the given 1D point set with weights)
struct FeecValues {
  int nq = 0;
  std::vector<double> JxW;
  std::vector<Vec3> xq;
  std::vector<Vec3> w, cw, u;   // [q][12], [q][12], [q][6]
  std::vector<double> du;       // [q][6]
  void reinit(const double* X, const signed char* sgn, int n1, const double* px,
              const double* pw) {
    nq = n1 * n1 * n1;
    JxW.assign(nq, 0);
    xq.assign(nq, Vec3());
    w.assign(size_t(nq) * 12, Vec3());
    cw.assign(size_t(nq) * 12, Vec3());
    u.assign(size_t(nq) * 6, Vec3());
    du.assign(size_t(nq) * 6, 0);
    for (int q = 0; q < nq; ++q) {
      const int ia = q % n1, ib = (q / n1) % n1, ic = q / (n1 * n1);
      const double xi[3] = {px[ia], px[ib], px[ic]};
      double J[3][3], Ji[3][3];
      map_q1(X, xi, J, xq[q]);
      const double det = det3(J);
      inv3(J, Ji);
      JxW[q] = det * (pw ? pw[ia] * pw[ib] * pw[ic] : 1.0);
      // Nedelec: N = prod_{transverse c} l_{s_c}(xi_c) e_axis (unit tangential
      // moment along the edge), covariant Piola
      for (int l = 0; l < 12; ++l) {
        const int a = kLineVtx[l][0], b = kLineVtx[l][1];
        int axis = 0;
        for (int d = 0; d < 3; ++d)
          if (vbit(a, d) != vbit(b, d)) axis = d;
        double g = 1, grad[3] = {1, 1, 1};
        for (int d = 0; d < 3; ++d) {
          if (d == axis) {
            grad[d] = 0;
            continue;
          }
          const double lv = lag1(vbit(a, d), xi[d]), dl = dlag1(vbit(a, d), xi[d]);
          g *= lv;
          for (int e = 0; e < 3; ++e)
            if (e != axis) grad[e] *= (e == d ? dl : lv);
        }
        Vec3 N, curlN;
        N[axis] = g;
        // curl (g e_axis) = grad g x e_axis
        Vec3 gg, ea;
        for (int d = 0; d < 3; ++d) gg[d] = grad[d];
        ea[axis] = 1;
        curlN = cross(gg, ea);
        const double s = sgn[l];
        for (int i = 0; i < 3; ++i) {
          double v = 0, c = 0;
          for (int j = 0; j < 3; ++j) {
            v += Ji[j][i] * N[j];
            c += J[i][j] * curlN[j];
          }
          w[12 * q + l][i] = s * v;
          cw[12 * q + l][i] = s * c / det;
        }
      }
      // Raviart-Thomas: R = l_side(xi_axis) e_axis (unit flux), contravariant Piola
      for (int f = 0; f < 6; ++f) {
        const int axis = f / 2, side = f % 2;
        const double r = lag1(side, xi[axis]);
        const double s = sgn[12 + f];
        for (int i = 0; i < 3; ++i) u[6 * q + f][i] = s * J[i][axis] * r / det;
        du[6 * q + f] = s * dlag1(side, 0.0) / det;
      }
    }
  }
};

// component views of local dof k (zero outside its own block)
Vec3 phi_w(const FeecValues& fv, int q, int k) { return k < 12 ? fv.w[12 * q + k] : Vec3(); }
Vec3 curl_w(const FeecValues& fv, int q, int k) { return k < 12 ? fv.cw[12 * q + k] : Vec3(); }
Vec3 phi_u(const FeecValues& fv, int q, int k) {
  return (k >= 12 && k < 18) ? fv.u[6 * q + k - 12] : Vec3();
}
double div_u(const FeecValues& fv, int q, int k) {
  return (k >= 12 && k < 18) ? fv.du[6 * q + k - 12] : 0.0;
}
double phi_p(int k) { return k == 18 ? 1.0 : 0.0; }

int feec_block(int k) { return k < 12 ? 0 : k < 18 ? 1 : 2; }

}  // namespace

extern "C" void orc_feec_cell_system(const orc_physics* ph, const double* X, const signed char* sgn,
                                     const double* dofv, const double* T_local, double* K,
                                     double* f) {
  // local_assemble_nse_system (boussineq_model_FEEC.tpp:669-808), QGauss(deg+2)
  double gx[4], gw[4];
  gauss1d(3, gx, gw);
  FeecValues fv;
  fv.reinit(X, sgn, 3, gx, gw);
  const double one_over_re = ph->one_over_reynolds, dt = ph->time_step;
  std::fill(K, K + 361, 0.0);
  std::fill(f, f + 19, 0.0);
  for (int q = 0; q < fv.nq; ++q) {
    // old T (Q1, MappingQ1): trilinear value at the point
    const int ia = q % 3, ib = (q / 3) % 3, ic = q / 9;
    const double xi[3] = {gx[ia], gx[ib], gx[ic]};
    double T = 0;
    for (int v = 0; v < 8; ++v)
      T += T_local[v] * lag1(vbit(v, 0), xi[0]) * lag1(vbit(v, 1), xi[1]) * lag1(vbit(v, 2), xi[2]);
    const double rho = 1 - ph->expansion_coefficient * (T - ph->temperature_ref);
    Vec3 old_w, old_u;
    for (int k = 0; k < 19; ++k) {
      const Vec3 a = phi_w(fv, q, k), b = phi_u(fv, q, k);
      for (int d = 0; d < 3; ++d) {
        old_w[d] += dofv[k] * a[d];
        old_u[d] += dofv[k] * b[d];
      }
    }
    Vec3 coriolis;
    if (ph->cuboid) coriolis[2] = ph->coriolis_scale * ph->omega;
    for (int i = 0; i < 19; ++i)
      for (int j = 0; j < 19; ++j)
        K[19 * i + j] += (dot(phi_w(fv, q, i), phi_w(fv, q, j)) -
                          dot(curl_w(fv, q, i), phi_u(fv, q, j)) +
                          dot(phi_u(fv, q, i), phi_u(fv, q, j)) +
                          dt * one_over_re * dot(phi_u(fv, q, i), curl_w(fv, q, j)) -
                          div_u(fv, q, i) * phi_p(j) - phi_p(i) * div_u(fv, q, j)) *
                         fv.JxW[q];
    Vec3 grav;
    if (ph->cuboid) {
      grav[2] = -ph->gravity_constant;
    } else {
      grav = gravity_vector(fv.xq[q], ph->gravity_constant);
    }
    for (int d = 0; d < 3; ++d) grav[d] *= ph->gravity_scale;
    const Vec3 wxu = cross(old_w, old_u), cxu = cross(coriolis, old_u);
    for (int i = 0; i < 19; ++i)
      f[i] += (dot(phi_u(fv, q, i), old_u) + dt * rho * dot(grav, phi_u(fv, q, i)) -
               dt * (div_u(fv, q, i) * 0.5 * dot(old_u, old_u) + dot(phi_u(fv, q, i), wxu)) -
               dt * 2 * dot(phi_u(fv, q, i), cxu)) *
              fv.JxW[q];
  }
}

extern "C" void orc_feec_cell_preconditioner(const orc_physics* ph, const double* X,
                                             const signed char* sgn, double* P) {
  // local_assemble_nse_preconditioner (FEEC.tpp:509-572), QGauss(deg+1); only
  // phi_p phi_p carries JxW (Q14)
  double gx[4], gw[4];
  gauss1d(2, gx, gw);
  FeecValues fv;
  fv.reinit(X, sgn, 2, gx, gw);
  const double c = ph->time_step * ph->one_over_reynolds;
  std::fill(P, P + 361, 0.0);
  auto ind = [](double v) { return std::fabs(v) > 1.0e-9 ? -2 * (std::signbit(v) - 0.5) : 0.0; };
  for (int q = 0; q < fv.nq; ++q)
    for (int i = 0; i < 19; ++i)
      for (int j = 0; j < 19; ++j)
        P[19 * i + j] += c * dot(curl_w(fv, q, i), curl_w(fv, q, j)) +
                         ind(dot(phi_u(fv, q, i), phi_w(fv, q, j))) +
                         ind(dot(phi_w(fv, q, i), phi_u(fv, q, j))) +
                         phi_p(i) * phi_p(j) * fv.JxW[q];
}

struct orc_feec {
  orc_physics ph;
  int n_cells, n_w, n_u, n_p, n, n_T;
  std::vector<int> dofs, cell_T;
  std::vector<signed char> sgn;
  std::vector<double> X, geom64, diam;
  Cons cons, cT;
  Csr nse, pre, Tmass, Tstiff, Tmat;
  std::vector<double> rhs, T_rhs, T_inv;
  bool zero_mean = true;
  int fixed_inner = 0;  // test hook: both inner GMRES run exactly this many steps
  bool block_prec = true;  // parameters.use_block_preconditioner_feec
};

extern "C" orc_feec* orc_feec_create(const orc_physics* ph, int n_cells, const int* cell_dofs19,
                                     const signed char* sign19, const double* X24,
                                     const unsigned char* fixed, int n_w, int n_u, int n_p,
                                     const int* cell_T, int n_T, const orc_constraints* T_c,
                                     const double* diameter) {
  auto m = new orc_feec();
  m->ph = *ph;
  m->n_cells = n_cells;
  m->n_w = n_w;
  m->n_u = n_u;
  m->n_p = n_p;
  m->n = n_w + n_u + n_p;
  m->n_T = n_T;
  m->dofs.assign(cell_dofs19, cell_dofs19 + 19 * size_t(n_cells));
  m->sgn.assign(sign19, sign19 + 19 * size_t(n_cells));
  m->X.assign(X24, X24 + 24 * size_t(n_cells));
  m->cell_T.assign(cell_T, cell_T + 8 * size_t(n_cells));
  m->diam.assign(diameter, diameter + n_cells);
  // homogeneous boundary constraints (project_boundary_values_* of zero, FEEC.tpp:311-350)
  std::vector<int> line, ptr(1, 0);
  std::vector<double> inh;
  for (int d = 0; d < m->n; ++d)
    if (fixed[d]) {
      line.push_back(d);
      ptr.push_back(0);
      inh.push_back(0.0);
    }
  const orc_constraints oc{int(line.size()), line.data(), ptr.data(), nullptr, nullptr, inh.data()};
  m->cons.init(m->n, &oc);
  m->cT.init(n_T, T_c);
  // coupling tables of setup_nse_matrices (FEEC.tpp:82-130) / setup_nse_preconditioner (:146-185)
  make_pattern(m->nse, m->n, n_cells, 19, m->dofs.data(), m->cons, [](int i, int j) {
    const int a = feec_block(i), b = feec_block(j);
    return a == 0 ? b < 2 : a == 1 ? true : b == 1;
  });
  make_pattern(m->pre, m->n, n_cells, 19, m->dofs.data(), m->cons, [](int i, int j) {
    const int a = feec_block(i), b = feec_block(j);
    return a < 2 ? b < 2 : b != 1;
  });
  make_pattern(m->Tmass, n_T, n_cells, 8, m->cell_T.data(), m->cT, [](int, int) { return true; });
  m->Tstiff = m->Tmass;
  m->Tmat = m->Tmass;
  // Q1 temperature mapping (temperature_mapping(1), FEEC.tpp:20) as the cubic
  // map's support points at the trilinear interpolants
  m->geom64.resize(192 * size_t(n_cells));
  for (int c = 0; c < n_cells; ++c)
    for (int k = 0; k < 64; ++k) {
      const double t[3] = {kGL[k % 4], kGL[(k / 4) % 4], kGL[k / 16]};
      for (int d = 0; d < 3; ++d) {
        double x = 0;
        for (int v = 0; v < 8; ++v)
          x += lag1(vbit(v, 0), t[0]) * lag1(vbit(v, 1), t[1]) * lag1(vbit(v, 2), t[2]) *
               m->X[24 * size_t(c) + 3 * v + d];
        m->geom64[192 * size_t(c) + 3 * k + d] = x;
      }
    }
  m->rhs.assign(m->n, 0.0);
  m->T_rhs.assign(n_T, 0.0);
  return m;
}

extern "C" void orc_feec_destroy(orc_feec* m) { delete m; }
extern "C" void orc_feec_set_zero_mean(orc_feec* m, int on) { m->zero_mean = on != 0; }
extern "C" void orc_feec_set_fixed_inner(orc_feec* m, int k) { m->fixed_inner = k; }

extern "C" void orc_feec_assemble_nse_system(orc_feec* m, const double* old_nse, const double* old_T) {
  m->nse.zero();
  std::fill(m->rhs.begin(), m->rhs.end(), 0.0);
  std::vector<double> K(361), f(19), dv(19), Tl(8);
  for (int c = 0; c < m->n_cells; ++c) {
    for (int i = 0; i < 19; ++i) dv[i] = old_nse[m->dofs[19 * size_t(c) + i]];
    for (int v = 0; v < 8; ++v) Tl[v] = old_T[m->cell_T[8 * size_t(c) + v]];
    orc_feec_cell_system(&m->ph, &m->X[24 * size_t(c)], &m->sgn[19 * size_t(c)], dv.data(),
                         Tl.data(), K.data(), f.data());
    distribute_local_to_global(m->cons, 19, &m->dofs[19 * size_t(c)], K.data(), f.data(), &m->nse,
                               m->rhs.data());
  }
}

extern "C" void orc_feec_assemble_preconditioner(orc_feec* m) {
  m->pre.zero();
  std::vector<double> P(361);
  for (int c = 0; c < m->n_cells; ++c) {
    orc_feec_cell_preconditioner(&m->ph, &m->X[24 * size_t(c)], &m->sgn[19 * size_t(c)], P.data());
    distribute_local_to_global(m->cons, 19, &m->dofs[19 * size_t(c)], P.data(), nullptr, &m->pre,
                               nullptr);
  }
}

extern "C" long orc_feec_matrix_nnz(const orc_feec* m, int which) {
  return long((which == 0 ? m->nse : m->pre).cols.size());
}
extern "C" void orc_feec_matrix_csr(const orc_feec* m, int which, int* rowptr, int* cols,
                                    double* vals) {
  const Csr& A = which == 0 ? m->nse : m->pre;
  std::copy(A.rowptr.begin(), A.rowptr.end(), rowptr);
  std::copy(A.cols.begin(), A.cols.end(), cols);
  std::copy(A.vals.begin(), A.vals.end(), vals);
}
extern "C" void orc_feec_rhs(const orc_feec* m, double* out) {
  std::copy(m->rhs.begin(), m->rhs.end(), out);
}

extern "C" void orc_feec_assemble_temperature(orc_feec* m, const double* old_T,
                                              const double* nse_solution) {
  // assemble_temperature_matrix (FEEC.tpp:882-960) + _rhs (:966-1100), MappingQ1,
  // QGauss(T_degree + 2); u from the RT field of nse_solution (Q5)
  m->Tmass.zero();
  m->Tstiff.zero();
  std::vector<double> M(64), K(64);
  for (int c = 0; c < m->n_cells; ++c) {
    orc_cell_temperature_matrix(&m->ph, &m->geom64[192 * size_t(c)], M.data(), K.data());
    const int* d = &m->cell_T[8 * size_t(c)];
    distribute_local_to_global(m->cT, 8, d, M.data(), nullptr, &m->Tmass, nullptr);
    distribute_local_to_global(m->cT, 8, d, K.data(), nullptr, &m->Tstiff, nullptr);
  }
  const double dt_eff = m->ph.time_step / m->ph.nse_solver_interval;
  for (size_t k = 0; k < m->Tmat.vals.size(); ++k)
    m->Tmat.vals[k] = m->Tmass.vals[k] + dt_eff * m->Tstiff.vals[k];
  m->T_inv.assign(m->n_T, 0.0);
  for (int r = 0; r < m->n_T; ++r) m->T_inv[r] = 1.0 / m->Tmat.at(r, r);
  std::fill(m->T_rhs.begin(), m->T_rhs.end(), 0.0);
  double gx[4], gw[4];
  gauss1d(3, gx, gw);
  std::vector<double> rhs(8), mfbc(64);
  CellValues cv;
  FeecValues fv;
  for (int c = 0; c < m->n_cells; ++c) {
    const int* d = &m->cell_T[8 * size_t(c)];
    cv.reinit(&m->geom64[192 * size_t(c)], 3);
    fv.reinit(&m->X[24 * size_t(c)], &m->sgn[19 * size_t(c)], 3, gx, gw);
    std::fill(rhs.begin(), rhs.end(), 0.0);
    std::fill(mfbc.begin(), mfbc.end(), 0.0);
    for (int q = 0; q < 27; ++q) {
      double T = 0;
      Vec3 gT, u;
      for (int v = 0; v < 8; ++v) {
        T += old_T[d[v]] * cv.v1[8 * q + v];
        for (int k = 0; k < 3; ++k) gT[k] += old_T[d[v]] * cv.g1[8 * q + v][k];
      }
      for (int f = 0; f < 6; ++f)
        for (int k = 0; k < 3; ++k)
          u[k] += nse_solution[m->dofs[19 * size_t(c) + 12 + f]] * fv.u[6 * q + f][k];
      for (int i = 0; i < 8; ++i) {
        rhs[i] += (cv.v1[8 * q + i] * T - dt_eff * cv.v1[8 * q + i] * dot(u, gT)) * cv.JxW[q];
        if (m->cT.constrained(d[i]) && m->cT.inhom[m->cT.line_of[d[i]]] != 0.0)
          for (int j = 0; j < 8; ++j)
            mfbc[8 * j + i] += (cv.v1[8 * q + i] * cv.v1[8 * q + j] +
                                dt_eff * m->ph.one_over_peclet *
                                    dot(cv.g1[8 * q + i], cv.g1[8 * q + j])) *
                               cv.JxW[q];
      }
    }
    distribute_rhs_with_bc(m->cT, 8, d, rhs.data(), mfbc.data(), m->T_rhs.data());
  }
}

extern "C" void orc_feec_T_rhs(const orc_feec* m, double* out) {
  std::copy(m->T_rhs.begin(), m->T_rhs.end(), out);
}


extern "C" int orc_feec_solve_nse(orc_feec* m, double* sol, int* iterations) {
  // solve_NSE_block_preconditioned (FEEC.tpp:1268-1477), block preconditioner on
  const int nw = m->n_w, nu = m->n_u, np = m->n_p, n = m->n, ou = nw, op = nw + nu;
  const double dt = m->ph.time_step;
  const Csr& A = m->nse;
  // Mw / Mu: Ifpack Jacobi of nse_matrix.block(0,0) / block(1,1) (:1288-1303)
  std::vector<double> dinv(nw + nu);
  for (int r = 0; r < nw + nu; ++r) dinv[r] = 1.0 / const_cast<Csr&>(A).at(r, r);
  std::vector<double> cellw(np);
  double wsum = 0;
  for (int c = 0; c < m->n_cells; ++c) {
    const double xi[3] = {0.5, 0.5, 0.5};
    double J[3][3];
    Vec3 x;
    map_q1(&m->X[24 * size_t(c)], xi, J, x);
    cellw[c] = det3(J);  // QGauss(1) JxW of compute_mean_value
    wsum += cellw[c];
  }
  std::vector<double> t1(nu), t2(np), s1(std::max(nw, nu)), s2(std::max(nw, nu));
  // ShiftedSchurComplement::vmult (shifted_schur_complement.hpp:155-171)
  auto shifted = [&](const double* x, double* y) {
    csr_block(A, ou, op, ou, op, x, y, false);
    csr_block(A, 0, nw, ou, op, x, s1.data(), false);
    for (int i = 0; i < nw; ++i) s2[i] = s1[i] * dinv[i];
    for (int i = 0; i < nw; ++i) s2[i] *= -1;
    csr_block(A, ou, op, 0, nw, s2.data(), y, true);
  };
  auto mu_jacobi = [&](const double* x, double* y) {
    for (int i = 0; i < nu; ++i) y[i] = x[i] * dinv[nw + i];
  };
  // SchurComplementLowerBlock::vmult, do_full_solve = false (schur_complement.hpp:256-276)
  auto lower = [&](const double* x, double* y) {
    csr_block(A, ou, op, op, n, x, s1.data(), false);
    for (int i = 0; i < nu; ++i) s2[i] = s1[i] * dinv[nw + i];
    csr_block(A, op, n, ou, op, s2.data(), y, false);
  };
  auto identity = [&](const double* x, double* y) { std::copy(x, x + np, y); };
  // BlockSchurPreconditionerFEEC::vmult (block_schur_preconditioner.hpp:115-147)
  auto precondition = [&](const double* src, double* dst) {
    for (int i = 0; i < nw; ++i) dst[i] = src[i] * dinv[i];  // Mw Jacobi (Q16)
    csr_block(A, ou, op, 0, nw, dst, t1.data(), false);
    for (int i = 0; i < nu; ++i) t1[i] = -1.0 * t1[i] + src[ou + i];
    {
      // ApproxShiftedSchurComplementInverse (shifted_schur_complement.hpp:271-298)
      const int k = m->fixed_inner;
      Control ctl = k > 0 ? Control{unsigned(std::min(k, 30)), 0.0} : Control{30, 1e-6 * norm2(t1, 0, nu)};
      int it = 0;
      try {
        gmres(nu, shifted, mu_jacobi, dst + ou, t1.data(), ctl, it);
      } catch (const NoConvergence&) {
      }
    }
    for (int i = 0; i < np; ++i) t2[i] = -1.0 * (src[op + i] + src[op + i]);  // Q15
    csr_block(A, op, n, ou, op, dst + ou, t2.data(), true);
    {
      // ApproxNestedSchurComplementInverse (nested_schur_complement.hpp:287-322)
      const int k = m->fixed_inner;
      Control ctl = k > 0 ? Control{unsigned(k), 0.0} : Control{100, 1e-6 * norm2(t2, 0, np)};
      int it = 0;
      try {
        gmres(np, lower, identity, dst + op, t2.data(), ctl, it);
      } catch (const NoConvergence&) {
      }
    }
    if (m->zero_mean) {
      double s = 0;
      for (int i = 0; i < np; ++i) s += cellw[i] * dst[op + i];
      const double mean = s / wsum;
      for (int i = 0; i < np; ++i) dst[op + i] += -mean;
    }
  };
  // PreconditionerBlockIdentity::vmult (preconditioner_block_identity.hpp:31-53):
  // dst = src; with correct_pressure_mean_value the pressure block minus
  // VectorTools::compute_mean_value(dof_handler, QGauss<3>(2), dst, 6): per
  // cell, per point, mean += p_K JxW, area += JxW (the DGQ0 value is p_K)
  auto identity_block = [&](const double* src, double* dst) {
    std::copy(src, src + n, dst);
    if (!m->zero_mean) return;
    const double g[2] = {0.5 - 0.5 / std::sqrt(3.0), 0.5 + 0.5 / std::sqrt(3.0)};
    double mean = 0, area = 0;
    for (int c = 0; c < m->n_cells; ++c)
      for (int q = 0; q < 8; ++q) {
        const double xi[3] = {g[q & 1], g[(q >> 1) & 1], g[q >> 2]};
        double J[3][3];
        Vec3 xq;
        map_q1(&m->X[24 * size_t(c)], xi, J, xq);
        const double JxW = det3(J) * 0.125;
        mean += dst[op + c] * JxW;
        area += JxW;
      }
    mean /= area;
    for (int i = 0; i < np; ++i) dst[op + i] += -mean;
  };
  auto Aop = [&](const double* x, double* y) { csr_block(A, 0, n, 0, n, x, y, false); };
  std::vector<double> x(sol, sol + n);
  for (int i = op; i < n; ++i) x[i] *= dt;  // :1345
  // n_max_iter 500 with the block preconditioner, 15000 without (:1386-1391)
  Control ctl{m->block_prec ? 500u : 15000u, 1e-8 * norm2(m->rhs, 0, n)};
  int its = 0, rc = 0;
  try {
    if (m->block_prec)
      gmres(n, Aop, precondition, x.data(), m->rhs.data(), ctl, its, 100);
    else
      gmres(n, Aop, identity_block, x.data(), m->rhs.data(), ctl, its, 100);  // :1420-1431
  } catch (const NoConvergence&) {
    rc = 1;
  }
  m->cons.distribute(x.data());
  for (int i = op; i < n; ++i) x[i] /= dt;
  std::copy(x.begin(), x.end(), sol);
  if (iterations) *iterations = int(ctl.last_step);
  return rc;
}

extern "C" void orc_feec_set_block_preconditioner(orc_feec* m, int on) { m->block_prec = on != 0; }

extern "C" int orc_feec_solve_temperature(orc_feec* m, double* T, int* iterations) {
  // solve_temperature: same CG + Jacobi as the classic model (:1417-1476)
  const int n = m->n_T;
  Control ctl{unsigned(n), 1e-12 * norm2(m->T_rhs, 0, n)};
  std::vector<double> x(T, T + n), g(n), d(n), h(n);
  const Csr& A = m->Tmat;
  auto Av = [&](const std::vector<double>& s, std::vector<double>& o) {
    for (int r = 0; r < n; ++r) {
      double acc = 0;
      for (int k = A.rowptr[r]; k < A.rowptr[r + 1]; ++k) acc += A.vals[k] * s[A.cols[k]];
      o[r] = acc;
    }
  };
  bool all_zero = true;
  for (double v : x) all_zero &= (v == 0.0);
  if (!all_zero) {
    Av(x, g);
    for (int i = 0; i < n; ++i) g[i] += -1. * m->T_rhs[i];
  } else {
    for (int i = 0; i < n; ++i) g[i] = -1. * m->T_rhs[i];
  }
  double res = norm2(g, 0, n);
  State conv = ctl.check(0, res);
  int it = 0;
  if (conv == kIterate) {
    for (int i = 0; i < n; ++i) h[i] = g[i] * m->T_inv[i];
    for (int i = 0; i < n; ++i) d[i] = -1. * h[i];
    double gh = dotv(g.data(), h.data(), n);
    while (conv == kIterate) {
      it++;
      Av(d, h);
      double alpha = dotv(d.data(), h.data(), n);
      alpha = gh / alpha;
      for (int i = 0; i < n; ++i) x[i] += alpha * d[i];
      double gg = 0;
      for (int i = 0; i < n; ++i) {
        g[i] += alpha * h[i];
        gg += g[i] * g[i];
      }
      res = std::sqrt(std::fabs(gg));
      conv = ctl.check(it, res);
      if (conv != kIterate) break;
      for (int i = 0; i < n; ++i) h[i] = g[i] * m->T_inv[i];
      double beta = gh;
      gh = dotv(g.data(), h.data(), n);
      beta = gh / beta;
      for (int i = 0; i < n; ++i) d[i] = beta * d[i] - h[i];
    }
  }
  m->cT.distribute(x.data());
  std::copy(x.begin(), x.end(), T);
  if (iterations) *iterations = int(ctl.last_step);
  return conv == kSuccess ? 0 : 1;
}

extern "C" void orc_feec_velocity_stats(const orc_feec* m, const double* sol, double* out2) {
  // get_maximal_velocity / get_cfl_number (FEEC.tpp:1134-1230) on
  // QIterated(QTrapez, 2): points {0, 1/2, 1}^3
  const double px[3] = {0.0, 0.5, 1.0};
  FeecValues fv;
  double mx = 0, cfl = 0;
  for (int c = 0; c < m->n_cells; ++c) {
    fv.reinit(&m->X[24 * size_t(c)], &m->sgn[19 * size_t(c)], 3, px, nullptr);
    double cm = 1e-10;
    for (int q = 0; q < 27; ++q) {
      Vec3 u;
      for (int f = 0; f < 6; ++f)
        for (int k = 0; k < 3; ++k) u[k] += sol[m->dofs[19 * size_t(c) + 12 + f]] * fv.u[6 * q + f][k];
      const double nu = std::sqrt(dot(u, u));
      mx = std::max(mx, nu);
      cm = std::max(cm, nu);
    }
    cfl = std::max(cfl, cm / m->diam[c]);
  }
  out2[0] = mx;
  out2[1] = cfl;
}

// ===========================================================================
// Two-dimensional model: Standard::BoussinesqModel<2>
// (boussinesq_model.inst.cc:8; data/aqua_planet_test_2d.prm, BASELINE C1).
// FESystem(FE_Q(2)^2, FE_Q(1)): 22 local dofs (per vertex u_x u_y p, per line
// u_x u_y, interior u_x u_y); temperature FE_Q(deg); MappingQ(3) from 16
// support points; the 2D branches of local_assemble_nse_system (Q3: the
// Coriolis term is -2 phi . cross_product_2d(u) without omega, :663-664).

namespace {

const int kHier2Lex2D[9] = {0, 2, 6, 8, 3, 5, 1, 7, 4};

struct Vec2 {
  double v[2] = {0, 0};
  double& operator[](int i) { return v[i]; }
  double operator[](int i) const { return v[i]; }
};
double dot2(const Vec2& a, const Vec2& b) { return a[0] * b[0] + a[1] * b[1]; }

struct CellValues2D {
  int nq = 0;
  std::vector<double> JxW;
  std::vector<Vec2> xq;
  std::vector<double> v2, v1;  // [q][9], [q][4]
  std::vector<Vec2> g2, g1;
  void reinit(const double* geom16, int n1d) {
    double qx[4], qw[4];
    gauss1d(n1d, qx, qw);
    nq = n1d * n1d;
    JxW.assign(nq, 0);
    xq.assign(nq, Vec2());
    v2.assign(size_t(nq) * 9, 0);
    v1.assign(size_t(nq) * 4, 0);
    g2.assign(size_t(nq) * 9, Vec2());
    g1.assign(size_t(nq) * 4, Vec2());
    for (int q = 0; q < nq; ++q) {
      const double p[2] = {qx[q % n1d], qx[q / n1d]};
      const double w = qw[q % n1d] * qw[q / n1d];
      double J[2][2] = {{0, 0}, {0, 0}};
      Vec2 x;
      for (int n = 0; n < 16; ++n) {
        const int a = n % 4, b = n / 4;
        const double s = lag3(a, p[0]) * lag3(b, p[1]);
        const double g[2] = {dlag3(a, p[0]) * lag3(b, p[1]), lag3(a, p[0]) * dlag3(b, p[1])};
        for (int i = 0; i < 2; ++i) {
          x[i] += geom16[2 * n + i] * s;
          for (int j = 0; j < 2; ++j) J[i][j] += geom16[2 * n + i] * g[j];
        }
      }
      const double det = J[0][0] * J[1][1] - J[0][1] * J[1][0];
      if (!(det > 0)) throw std::runtime_error("oracle 2D: non-positive Jacobian");
      const double Ji[2][2] = {{J[1][1] / det, -J[0][1] / det}, {-J[1][0] / det, J[0][0] / det}};
      JxW[q] = det * w;
      xq[q] = x;
      for (int n = 0; n < 9; ++n) {
        const int a = n % 3, b = n / 3;
        v2[9 * q + n] = lag2(a, p[0]) * lag2(b, p[1]);
        const double r0 = dlag2(a, p[0]) * lag2(b, p[1]), r1 = lag2(a, p[0]) * dlag2(b, p[1]);
        for (int i = 0; i < 2; ++i) g2[9 * q + n][i] = r0 * Ji[0][i] + r1 * Ji[1][i];
      }
      for (int n = 0; n < 4; ++n) {
        const int a = n & 1, b = n >> 1;
        v1[4 * q + n] = lag1(a, p[0]) * lag1(b, p[1]);
        const double r0 = dlag1(a, p[0]) * lag1(b, p[1]), r1 = lag1(a, p[0]) * dlag1(b, p[1]);
        for (int i = 0; i < 2; ++i) g1[4 * q + n][i] = r0 * Ji[0][i] + r1 * Ji[1][i];
      }
    }
  }
};

// local dof -> (component 0, 1 velocity / 2 pressure, lexicographic point or vertex)
SysDof sysdof2d(int i) {
  if (i < 12) return {i % 3, i % 3 == 2 ? i / 3 : kHier2Lex2D[i / 3]};
  if (i < 20) return {(i - 12) % 2, kHier2Lex2D[4 + (i - 12) / 2]};
  return {i - 20, 4};
}

double T2_value(const CellValues2D& cv, int deg, int q, int k) {
  return deg == 1 ? cv.v1[4 * q + k] : cv.v2[9 * q + kHier2Lex2D[k]];
}
const Vec2& T2_grad(const CellValues2D& cv, int deg, int q, int k) {
  return deg == 1 ? cv.g1[4 * q + k] : cv.g2[9 * q + kHier2Lex2D[k]];
}
int T2_dofs_per_cell(int deg) { return deg == 1 ? 4 : 9; }

}  // namespace

extern "C" void orc2d_cell_nse_system(const orc_physics* ph, const double* geom16,
                                      const double* u_local, const double* T_local, double* K,
                                      double* f) {
  // boussinesq_model.tpp:550-673 at dim = 2; QGauss(3)
  CellValues2D cv;
  cv.reinit(geom16, 3);
  const int tdeg = ph->temperature_degree, ntd = T2_dofs_per_cell(tdeg);
  std::fill(K, K + 22 * 22, 0.0);
  std::fill(f, f + 22, 0.0);
  Vec2 phi_u[22];
  double grad[22][2][2], eps[22][2][2], div[22], phi_p[22];
  for (int q = 0; q < cv.nq; ++q) {
    for (int k = 0; k < 22; ++k) {
      const SysDof s = sysdof2d(k);
      phi_u[k] = Vec2();
      std::memset(grad[k], 0, sizeof(grad[k]));
      div[k] = phi_p[k] = 0;
      if (s.comp < 2) {
        const Vec2& g = cv.g2[9 * q + s.idx];
        phi_u[k][s.comp] = cv.v2[9 * q + s.idx];
        for (int d = 0; d < 2; ++d) grad[k][s.comp][d] = g[d];
        div[k] = g[s.comp];
      } else {
        phi_p[k] = cv.v1[4 * q + s.idx];
      }
      for (int a = 0; a < 2; ++a)
        for (int b = 0; b < 2; ++b) eps[k][a][b] = 0.5 * (grad[k][a][b] + grad[k][b][a]);
    }
    double old_T = 0;
    for (int k = 0; k < ntd; ++k) old_T += T_local[k] * T2_value(cv, tdeg, q, k);
    Vec2 u;
    double G[2][2] = {{0, 0}, {0, 0}};
    for (int k = 0; k < 22; ++k) {
      const SysDof s = sysdof2d(k);
      if (s.comp == 2) continue;
      u[s.comp] += u_local[k] * phi_u[k][s.comp];
      for (int d = 0; d < 2; ++d) G[s.comp][d] += u_local[k] * grad[k][s.comp][d];
    }
    const double rho = 1 - ph->expansion_coefficient * (old_T - ph->temperature_ref);
    Vec2 adv;  // (u . grad) u
    for (int j = 0; j < 2; ++j)
      for (int i = 0; i < 2; ++i) adv[j] += u[i] * G[j][i];
    const double JxW = cv.JxW[q], dt = ph->time_step;
    for (int i = 0; i < 22; ++i)
      for (int j = 0; j < 22; ++j) {
        double ee = 0;
        for (int a = 0; a < 2; ++a)
          for (int b = 0; b < 2; ++b) ee += eps[i][a][b] * eps[j][a][b];
        K[22 * i + j] += (dot2(phi_u[i], phi_u[j]) + dt * (ph->one_over_reynolds * 2 * ee) -
                          div[i] * phi_p[j] - phi_p[i] * div[j]) *
                         JxW;
      }
    // gravity: vertical on the cuboid, gravity_vector (Q4) on the shell
    Vec2 grav;
    const Vec2& x = cv.xq[q];
    if (ph->cuboid) {
      grav[1] = -ph->gravity_constant;
    } else {
      const double r = std::sqrt(dot2(x, x));
      for (int d = 0; d < 2; ++d)
        grav[d] = (r > 1) ? -ph->gravity_constant * x[d] / r : -ph->gravity_constant * x[d] / std::sqrt(r);
    }
    for (int d = 0; d < 2; ++d) grav[d] *= ph->gravity_scale;
    // cross_product_2d(u) = (u_y, -u_x); the 2D Coriolis term (Q3)
    Vec2 cu;
    cu[0] = u[1];
    cu[1] = -u[0];
    for (int i = 0; i < 22; ++i)
      f[i] += (dot2(phi_u[i], u) + dt * rho * dot2(grav, phi_u[i]) - dt * dot2(phi_u[i], adv) -
               dt * (-2 * dot2(phi_u[i], cu))) *
              JxW;
  }
}

extern "C" void orc2d_cell_nse_preconditioner(const orc_physics* ph, const double* geom16,
                                              double* P) {
  // boussinesq_model.tpp:421-464 at dim = 2
  CellValues2D cv;
  cv.reinit(geom16, 3);
  std::fill(P, P + 22 * 22, 0.0);
  for (int q = 0; q < cv.nq; ++q) {
    Vec2 phi_u[22];
    double grad[22][2][2] = {}, phi_p[22] = {};
    for (int k = 0; k < 22; ++k) {
      const SysDof s = sysdof2d(k);
      if (s.comp < 2) {
        phi_u[k][s.comp] = cv.v2[9 * q + s.idx];
        for (int d = 0; d < 2; ++d) grad[k][s.comp][d] = cv.g2[9 * q + s.idx][d];
      } else {
        phi_p[k] = cv.v1[4 * q + s.idx];
      }
    }
    for (int i = 0; i < 22; ++i)
      for (int j = 0; j < 22; ++j) {
        double gg = 0;
        for (int a = 0; a < 2; ++a)
          for (int b = 0; b < 2; ++b) gg += grad[i][a][b] * grad[j][a][b];
        P[22 * i + j] += (dot2(phi_u[i], phi_u[j]) + ph->time_step * ph->one_over_reynolds * gg +
                          phi_p[i] * phi_p[j]) *
                         cv.JxW[q];
      }
  }
}

extern "C" void orc2d_cell_temperature_matrix(const orc_physics* ph, const double* geom16,
                                              double* M, double* Kt) {
  const int tdeg = ph->temperature_degree, n = T2_dofs_per_cell(tdeg);
  CellValues2D cv;
  cv.reinit(geom16, tdeg + 2);
  std::fill(M, M + n * n, 0.0);
  std::fill(Kt, Kt + n * n, 0.0);
  for (int q = 0; q < cv.nq; ++q)
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < n; ++j) {
        M[n * i + j] += T2_value(cv, tdeg, q, i) * T2_value(cv, tdeg, q, j) * cv.JxW[q];
        Kt[n * i + j] += dot2(T2_grad(cv, tdeg, q, i), T2_grad(cv, tdeg, q, j)) *
                         ph->one_over_peclet * cv.JxW[q];
      }
}

extern "C" void orc2d_cell_temperature_rhs(const orc_physics* ph, const double* geom16,
                                           const double* T_local, const double* u_local,
                                           const int* inhom_mask, double* rhs, double* mfbc) {
  const int tdeg = ph->temperature_degree, n = T2_dofs_per_cell(tdeg);
  CellValues2D cv;
  cv.reinit(geom16, tdeg + 2);
  std::fill(rhs, rhs + n, 0.0);
  std::fill(mfbc, mfbc + n * n, 0.0);
  const double dt_eff = ph->time_step / ph->nse_solver_interval;
  for (int q = 0; q < cv.nq; ++q) {
    double T = 0;
    Vec2 gT, u;
    for (int k = 0; k < n; ++k) {
      T += T_local[k] * T2_value(cv, tdeg, q, k);
      const Vec2& g = T2_grad(cv, tdeg, q, k);
      for (int d = 0; d < 2; ++d) gT[d] += T_local[k] * g[d];
    }
    for (int k = 0; k < 22; ++k) {
      const SysDof s = sysdof2d(k);
      if (s.comp < 2) u[s.comp] += u_local[k] * cv.v2[9 * q + s.idx];
    }
    const double JxW = cv.JxW[q];
    for (int i = 0; i < n; ++i) {
      const double phi_i = T2_value(cv, tdeg, q, i);
      rhs[i] += (phi_i * T - dt_eff * phi_i * dot2(u, gT)) * JxW;
      if (inhom_mask[i])
        for (int j = 0; j < n; ++j)
          mfbc[n * j + i] += (phi_i * T2_value(cv, tdeg, q, j) +
                              dt_eff * ph->one_over_peclet *
                                  dot2(T2_grad(cv, tdeg, q, i), T2_grad(cv, tdeg, q, j))) *
                             JxW;
    }
  }
}

extern "C" orc_model* orc2d_create(const orc_physics* ph, int n_cells, const int* cell_nse_dofs,
                                   const int* cell_T_dofs, const double* cell_geom, int n_u,
                                   int n_p, int n_T, const orc_constraints* nse_c,
                                   const orc_constraints* T_c) {
  auto m = new orc_model();
  m->dim = 2;
  m->ph = *ph;
  m->n_cells = n_cells;
  m->n_u = n_u;
  m->n_p = n_p;
  m->n_T = n_T;
  m->tdeg = ph->temperature_degree;
  m->tdpc = T2_dofs_per_cell(m->tdeg);
  m->cell_nse.assign(cell_nse_dofs, cell_nse_dofs + size_t(n_cells) * 22);
  m->cell_T.assign(cell_T_dofs, cell_T_dofs + size_t(n_cells) * m->tdpc);
  m->geom.assign(cell_geom, cell_geom + size_t(n_cells) * 32);
  m->cnse.init(n_u + n_p, nse_c);
  m->cT.init(n_T, T_c);
  make_pattern(m->nse, n_u + n_p, n_cells, 22, m->cell_nse.data(), m->cnse,
               [](int i, int j) { return !(sysdof2d(i).comp == 2 && sysdof2d(j).comp == 2); });
  m->nse_rhs.assign(n_u + n_p, 0.0);
  make_pattern(m->Tmass, n_T, n_cells, m->tdpc, m->cell_T.data(), m->cT, [](int, int) { return true; });
  m->Tstiff = m->Tmass;
  m->Tmat = m->Tmass;
  m->T_rhs.assign(n_T, 0.0);
  m->tmp1.assign(n_u, 0.0);
  m->tmp2.assign(n_u, 0.0);
  return m;
}

void orc2d_assemble_nse_system(orc_model* m, const double* old_nse, const double* old_T) {
  m->nse.zero();
  std::fill(m->nse_rhs.begin(), m->nse_rhs.end(), 0.0);
  std::vector<double> K(22 * 22), f(22), ul(22), Tl(9);
  for (int c = 0; c < m->n_cells; ++c) {
    gather(m->cell_nse, c, 22, old_nse, ul.data());
    gather(m->cell_T, c, m->tdpc, old_T, Tl.data());
    orc2d_cell_nse_system(&m->ph, &m->geom[32 * size_t(c)], ul.data(), Tl.data(), K.data(), f.data());
    distribute_local_to_global(m->cnse, 22, &m->cell_nse[22 * size_t(c)], K.data(), f.data(),
                               &m->nse, m->nse_rhs.data());
  }
}

void orc2d_assemble_temperature_matrix(orc_model* m) {
  m->Tmass.zero();
  m->Tstiff.zero();
  const int n = m->tdpc;
  std::vector<double> M(n * n), K(n * n);
  for (int c = 0; c < m->n_cells; ++c) {
    orc2d_cell_temperature_matrix(&m->ph, &m->geom[32 * size_t(c)], M.data(), K.data());
    const int* d = &m->cell_T[size_t(n) * c];
    distribute_local_to_global(m->cT, n, d, M.data(), nullptr, &m->Tmass, nullptr);
    distribute_local_to_global(m->cT, n, d, K.data(), nullptr, &m->Tstiff, nullptr);
  }
}

void orc2d_assemble_temperature_rhs(orc_model* m, const double* old_T, const double* nse_solution) {
  const int n = m->tdpc;
  std::vector<double> Tl(n), ul(22), rhs(n), mfbc(n * n);
  std::vector<int> mask(n);
  for (int c = 0; c < m->n_cells; ++c) {
    const int* d = &m->cell_T[size_t(n) * c];
    gather(m->cell_T, c, n, old_T, Tl.data());
    gather(m->cell_nse, c, 22, nse_solution, ul.data());
    for (int i = 0; i < n; ++i)
      mask[i] = m->cT.constrained(d[i]) && m->cT.inhom[m->cT.line_of[d[i]]] != 0.0;
    orc2d_cell_temperature_rhs(&m->ph, &m->geom[32 * size_t(c)], Tl.data(), ul.data(), mask.data(),
                               rhs.data(), mfbc.data());
    distribute_rhs_with_bc(m->cT, n, d, rhs.data(), mfbc.data(), m->T_rhs.data());
  }
}

// get_maximal_velocity / get_cfl_number (:1023-1101) at dim = 2: the 9 Q2
// support points (QIterated<QTrapez>(2)); diam == null: the maximal velocity
double orc2d_max_velocity(const orc_model* m, const double* sol, const double* diam) {
  double out = 0;
  for (int c = 0; c < m->n_cells; ++c) {
    double mx = diam ? 1e-10 : 0.0;
    for (int t = 0; t < 9; ++t) {
      const int* d = &m->cell_nse[22 * size_t(c) + (t < 4 ? 3 * t : 12 + 2 * (t - 4))];
      mx = std::max(mx, std::sqrt(sol[d[0]] * sol[d[0]] + sol[d[1]] * sol[d[1]]));
    }
    out = std::max(out, diam ? mx / diam[c] : mx);
  }
  return out;
}
