// deal.II geometry rules the reference's mesh and mapping rely on, restated
// from deal.II's published algorithms (deal.II >= 9.2 is not in this image):
//
//   SphericalManifold<3>::get_intermediate_point  — line midpoints on refinement
//   SphericalManifold<3>::get_new_points          — quad / hex centres on
//       refinement (TriaAccessor::center(true, true) weights) and the
//       MappingQGeneric(3) support points of every cell
//   MappingQ<3>(3) (boussinesq_model.tpp:20, boussinesq_model.h:211) — in
//       deal.II 9.2 the cubic map is used on cells with boundary lines only
//       (use_mapping_q_on_all_cells = false), MappingQ1 elsewhere.
//
// The reference builds its shell with GridGenerator::hyper_shell(6 cells,
// colorize) (planet_geometry.tpp:60-66), which attaches a SphericalManifold
// (centre = origin) to every cell, face and line.
#include <cmath>
#include <stdexcept>
#include <vector>

#include "fe_tables.h"
#include "mesh.h"

namespace dcp {

namespace {

inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// internal::compute_normal(vector, normalize = true): a unit vector normal to
// `v` (zero in none of the components but built from the dominant one).
void compute_normal(const double* v, double* n) {
  const double a0 = std::fabs(v[0]), a1 = std::fabs(v[1]), a2 = std::fabs(v[2]);
  if (a0 >= a1 && a0 >= a2) {
    n[1] = -1.0; n[2] = -1.0; n[0] = (v[1] + v[2]) / v[0];
  } else if (a1 >= a0 && a1 >= a2) {
    n[0] = -1.0; n[2] = -1.0; n[1] = (v[0] + v[2]) / v[1];
  } else {
    n[0] = -1.0; n[1] = -1.0; n[2] = (v[0] + v[1]) / v[2];
  }
  const double s = std::sqrt(dot3(n, n));
  for (int d = 0; d < 3; ++d) n[d] /= s;
}

// SphericalManifold's Newton iteration for the weighted spherical average of
// unit directions (the minimiser of sum_i w_i theta_i^2 on the unit sphere),
// started from `cand` (unit). Exact Hessian in the exponential chart at the
// candidate; stops when a step moves the candidate by less than 1e-10, at
// most 10 steps.
void spherical_average(int n, const double* dirs, const double* w, double* cand) {
  const double tol = 1e-10;
  for (int i = 0; i < n; ++i) {
    double d2 = 0;
    for (int d = 0; d < 3; ++d) d2 += (cand[d] - dirs[3 * i + d]) * (cand[d] - dirs[3 * i + d]);
    if (d2 < tol * tol) return;
  }
  if (n == 2) {
    double out[3];
    const double o[3] = {0, 0, 0};
    spherical_intermediate(o, dirs, dirs + 3, w[1], out);
    for (int d = 0; d < 3; ++d) cand[d] = out[d];
    return;
  }
  for (int it = 0; it < 10; ++it) {
    double ex[3], ey[3];
    compute_normal(cand, ex);
    cross3(cand, ex, ey);
    double g0 = 0, g1 = 0, H00 = 0, H01 = 0, H11 = 0;
    for (int i = 0; i < n; ++i) {
      if (!(std::fabs(w[i]) > 1e-15)) continue;
      const double* di = dirs + 3 * i;
      const double c = dot3(di, cand);
      double vp[3];
      for (int d = 0; d < 3; ++d) vp[d] = di[d] - c * cand[d];
      const double s = std::sqrt(dot3(vp, vp));
      if (s < tol) {
        H00 += w[i];
        H11 += w[i];
        continue;
      }
      const double theta = std::atan2(s, c);
      const double sinc_inv = theta / s;
      const double cphi = dot3(vp, ex), sphi = dot3(vp, ey);
      g0 += w[i] * sinc_inv * cphi;
      g1 += w[i] * sinc_inv * sphi;
      const double wt = w[i] / s / s;
      const double tt = sinc_inv * c;
      const double off = cphi * sphi * wt * (1.0 - tt);
      H00 += wt * (cphi * cphi + tt * sphi * sphi);
      H01 += off;
      H11 += wt * (sphi * sphi + tt * cphi * cphi);
    }
    const double det = H00 * H11 - H01 * H01;
    if (!(det > tol)) throw std::runtime_error("SphericalManifold: singular Hessian");
    const double x0 = (H11 * g0 - H01 * g1) / det, x1 = (H00 * g1 - H01 * g0) / det;
    double disp[3];
    for (int d = 0; d < 3; ++d) disp[d] = x0 * ex[d] + x1 * ey[d];
    const double th = std::sqrt(dot3(disp, disp));
    double old[3] = {cand[0], cand[1], cand[2]};
    if (th >= 1e-10)
      for (int d = 0; d < 3; ++d) cand[d] = std::cos(th) * old[d] + std::sin(th) * disp[d] / th;
    double m2 = 0;
    for (int d = 0; d < 3; ++d) m2 += (cand[d] - old[d]) * (cand[d] - old[d]);
    if (m2 < tol * tol) break;
  }
}

}  // namespace

void spherical_intermediate(const double* center, const double* p1, const double* p2, double w,
                            double* out) {
  const double tol = 1e-10;
  double dp2 = 0;
  for (int d = 0; d < 3; ++d) dp2 += (p1[d] - p2[d]) * (p1[d] - p2[d]);
  if (dp2 < tol * tol || std::fabs(w) < tol) {
    for (int d = 0; d < 3; ++d) out[d] = p1[d];
    return;
  }
  if (std::fabs(w - 1.0) < tol) {
    for (int d = 0; d < 3; ++d) out[d] = p2[d];
    return;
  }
  double v1[3], v2[3];
  for (int d = 0; d < 3; ++d) {
    v1[d] = p1[d] - center[d];
    v2[d] = p2[d] - center[d];
  }
  const double r1 = std::sqrt(dot3(v1, v1)), r2 = std::sqrt(dot3(v2, v2));
  double e1[3], e2[3];
  for (int d = 0; d < 3; ++d) {
    e1[d] = v1[d] / r1;
    e2[d] = v2[d] / r2;
  }
  const double cosg = dot3(e1, e2);
  const double eps = 2.220446049250313e-16;
  if (cosg < -1 + 8 * eps) {
    for (int d = 0; d < 3; ++d) out[d] = center[d];
    return;
  }
  if (cosg > 1 - 8 * eps) {
    for (int d = 0; d < 3; ++d) out[d] = center[d] + w * v2[d] + (1 - w) * v1[d];
    return;
  }
  const double sigma = w * std::acos(cosg);
  double n[3];
  const double v2e1 = dot3(v2, e1);
  for (int d = 0; d < 3; ++d) n[d] = v2[d] - v2e1 * e1[d];
  const double nn = std::sqrt(dot3(n, n));
  for (int d = 0; d < 3; ++d) n[d] /= nn;
  const double r = w * r2 + (1.0 - w) * r1;
  for (int d = 0; d < 3; ++d) out[d] = center[d] + r * (std::cos(sigma) * e1[d] + std::sin(sigma) * n[d]);
}

void spherical_new_points(const double* center, int n_src, const double* src, int n_rows,
                          const double* weights, double* out) {
  std::vector<double> dir(3 * size_t(n_src)), dist(n_src);
  double max_distance = 0;
  for (int i = 0; i < n_src; ++i) {
    double* di = &dir[3 * i];
    for (int d = 0; d < 3; ++d) di[d] = src[3 * i + d] - center[d];
    dist[i] = std::sqrt(dot3(di, di));
    if (dist[i] == 0.0) throw std::runtime_error("SphericalManifold: point at the centre");
    for (int d = 0; d < 3; ++d) di[d] /= dist[i];
    for (int k = 0; k < i; ++k) {
      double s = 0;
      for (int d = 0; d < 3; ++d) s += (di[d] - dir[3 * k + d]) * (di[d] - dir[3 * k + d]);
      max_distance = std::max(max_distance, s);
    }
  }
  // step 1: the linear guess (radius = weighted radii, direction = normalised
  // weighted directions)
  std::vector<double> rho(n_rows), cand(3 * size_t(n_rows));
  std::vector<char> found(n_rows, 0);
  for (int r = 0; r < n_rows; ++r) {
    const double* w = weights + size_t(r) * n_src;
    double c[3] = {0, 0, 0}, R = 0;
    for (int i = 0; i < n_src; ++i) {
      R += dist[i] * w[i];
      for (int d = 0; d < 3; ++d) c[d] += dir[3 * i + d] * w[i];
    }
    const double nc = std::sqrt(dot3(c, c));
    rho[r] = R;
    if (nc == 0.0) {
      rho[r] = 0.0;
      found[r] = 1;
      for (int d = 0; d < 3; ++d) cand[3 * r + d] = 0.0;
    } else {
      for (int d = 0; d < 3; ++d) cand[3 * r + d] = c[d] / nc;
    }
  }
  if (max_distance >= 2e-2) {
    // step 2: merge coinciding directions, then the Newton iteration
    std::vector<double> mdir;
    std::vector<int> slot(n_src);
    int nu = 0;
    for (int i = 0; i < n_src; ++i) {
      int hit = -1;
      for (int j = 0; j < nu && hit < 0; ++j) {
        double s = 0;
        for (int d = 0; d < 3; ++d) s += (dir[3 * i + d] - mdir[3 * j + d]) * (dir[3 * i + d] - mdir[3 * j + d]);
        if (s < 1e-28) hit = j;
      }
      if (hit < 0) {
        for (int d = 0; d < 3; ++d) mdir.push_back(dir[3 * i + d]);
        hit = nu++;
      }
      slot[i] = hit;
    }
    std::vector<double> mw(nu);
    for (int r = 0; r < n_rows; ++r) {
      if (found[r]) continue;
      std::fill(mw.begin(), mw.end(), 0.0);
      for (int i = 0; i < n_src; ++i) mw[slot[i]] += weights[size_t(r) * n_src + i];
      spherical_average(nu, mdir.data(), mw.data(), &cand[3 * r]);
    }
  }
  for (int r = 0; r < n_rows; ++r)
    for (int d = 0; d < 3; ++d) out[3 * r + d] = center[d] + rho[r] * cand[3 * r + d];
}

void mapping_support_points(const double* vertices, bool spherical, double* X) {
  // MappingQGeneric::compute_mapping_support_points: vertices, then every
  // other support point from the cell's manifold with the trilinear weights
  // of its unit position (support_point_weights_cell; all manifold ids of the
  // hyper_shell are equal, so one get_new_points call per cell).
  std::vector<double> w;
  std::vector<int> rows;
  for (int k = 0; k < 4; ++k)
    for (int j = 0; j < 4; ++j)
      for (int i = 0; i < 4; ++i) {
        const int t = i + 4 * j + 16 * k;
        const bool vx = (i == 0 || i == 3) && (j == 0 || j == 3) && (k == 0 || k == 3);
        if (vx) {
          const int v = (i == 3) + 2 * (j == 3) + 4 * (k == 3);
          for (int d = 0; d < 3; ++d) X[3 * t + d] = vertices[3 * v + d];
          continue;
        }
        const double x = kGL3[i], y = kGL3[j], z = kGL3[k];
        for (int v = 0; v < 8; ++v)
          w.push_back(((v & 1) ? x : 1 - x) * ((v & 2) ? y : 1 - y) * ((v & 4) ? z : 1 - z));
        rows.push_back(t);
      }
  const int nr = int(rows.size());
  std::vector<double> pts(3 * size_t(nr));
  if (spherical) {
    const double o[3] = {0, 0, 0};
    spherical_new_points(o, 8, vertices, nr, w.data(), pts.data());
  } else {
    // FlatManifold / MappingQ1: the weighted sum of the vertices
    for (int r = 0; r < nr; ++r)
      for (int d = 0; d < 3; ++d) {
        double s = 0;
        for (int v = 0; v < 8; ++v) s += w[8 * size_t(r) + v] * vertices[3 * v + d];
        pts[3 * r + d] = s;
      }
  }
  for (int r = 0; r < nr; ++r)
    for (int d = 0; d < 3; ++d) X[3 * rows[r] + d] = pts[3 * r + d];
}

void mapping_eval(const double* X, const double* xi, double* x, double J[3][3]) {
  double l[3][4], g[3][4];
  for (int e = 0; e < 3; ++e)
    for (int a = 0; a < 4; ++a) {
      l[e][a] = map_lag(a, xi[e]);
      g[e][a] = map_dlag(a, xi[e]);
    }
  for (int i = 0; i < 3; ++i) {
    x[i] = 0;
    for (int j = 0; j < 3; ++j) J[i][j] = 0;
  }
  for (int t = 0; t < kMapPts; ++t) {
    const int a = t % 4, b = (t / 4) % 4, c = t / 16;
    const double s = l[0][a] * l[1][b] * l[2][c];
    const double d0 = g[0][a] * l[1][b] * l[2][c], d1 = l[0][a] * g[1][b] * l[2][c],
                 d2 = l[0][a] * l[1][b] * g[2][c];
    for (int i = 0; i < 3; ++i) {
      const double Xi = X[3 * t + i];
      x[i] += s * Xi;
      J[i][0] += d0 * Xi;
      J[i][1] += d1 * Xi;
      J[i][2] += d2 * Xi;
    }
  }
}

}  // namespace dcp
