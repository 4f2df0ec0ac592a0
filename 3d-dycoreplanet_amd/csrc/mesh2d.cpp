// The 2D hyper_shell model setup (see mesh2d.h for the deal.II calls it
// restates).
#include "mesh2d.h"

#include <algorithm>
#include <cmath>
#include <map>
#include <numeric>
#include <stdexcept>
#include <utility>

namespace dcp {
namespace {

constexpr double kPi2D = 3.14159265358979323846;

// a 2D point through the spherical manifold helpers (z = 0 plane)
void mid_line(const double* p, const double* q, double* out) {
  const double o[3] = {0, 0, 0};
  const double a[3] = {p[0], p[1], 0}, b[3] = {q[0], q[1], 0};
  double r[3];
  spherical_intermediate(o, a, b, 0.5, r);
  out[0] = r[0];
  out[1] = r[1];
}

void new_point(int n, const double* pts2, const double* w, double* out) {
  std::vector<double> p3(3 * size_t(n));
  for (int i = 0; i < n; ++i) {
    p3[3 * i] = pts2[2 * i];
    p3[3 * i + 1] = pts2[2 * i + 1];
    p3[3 * i + 2] = 0;
  }
  const double o[3] = {0, 0, 0};
  double r[3];
  spherical_new_points(o, n, p3.data(), 1, w, r);
  out[0] = r[0];
  out[1] = r[1];
}

// MappingQGeneric(3) support points of a quad: vertices, then every other
// point as get_new_points(4 vertices, bilinear weights) of the cell's manifold
// (spherical) or the bilinear combination (MappingQ1)
void support_points_2d(const double* V /*[4][2]*/, bool spherical, double* X /*[16][2]*/) {
  std::vector<double> w;
  std::vector<int> rows;
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 4; ++i) {
      const int t = i + 4 * j;
      if ((i == 0 || i == 3) && (j == 0 || j == 3)) {
        const int v = (i == 3) + 2 * (j == 3);
        X[2 * t] = V[2 * v];
        X[2 * t + 1] = V[2 * v + 1];
        continue;
      }
      const double x = kGL3[i], y = kGL3[j];
      for (int v = 0; v < 4; ++v) w.push_back(((v & 1) ? x : 1 - x) * ((v & 2) ? y : 1 - y));
      rows.push_back(t);
    }
  const int nr = int(rows.size());
  if (spherical) {
    std::vector<double> p3(12);
    for (int v = 0; v < 4; ++v) {
      p3[3 * v] = V[2 * v];
      p3[3 * v + 1] = V[2 * v + 1];
      p3[3 * v + 2] = 0;
    }
    std::vector<double> out(3 * size_t(nr));
    const double o[3] = {0, 0, 0};
    spherical_new_points(o, 4, p3.data(), nr, w.data(), out.data());
    for (int r = 0; r < nr; ++r) {
      X[2 * rows[r]] = out[3 * r];
      X[2 * rows[r] + 1] = out[3 * r + 1];
    }
  } else {
    for (int r = 0; r < nr; ++r)
      for (int d = 0; d < 2; ++d) {
        double s = 0;
        for (int v = 0; v < 4; ++v) s += w[4 * size_t(r) + v] * V[2 * v + d];
        X[2 * rows[r] + d] = s;
      }
  }
}

struct Builder2D {
  std::vector<int> has;
  std::vector<std::map<int, double>> entries;
  std::vector<double> inhom;
  explicit Builder2D(int n) : has(n, 0), entries(n), inhom(n, 0.0) {}
  Constraints close() const {
    // no chains here: targets of the no-normal-flux lines are unconstrained
    Constraints c;
    const int n = int(has.size());
    c.n_dofs = n;
    c.line_of.assign(n, -1);
    c.entry_ptr.push_back(0);
    for (int d = 0; d < n; ++d) {
      if (!has[d]) continue;
      c.line_of[d] = c.n_lines();
      c.line_dof.push_back(d);
      c.inhomogeneity.push_back(inhom[d]);
      for (const auto& e : entries[d]) {
        if (has[e.first]) throw std::runtime_error("2D constraints: chained line");
        c.entry_dof.push_back(e.first);
        c.entry_w.push_back(e.second);
      }
      c.entry_ptr.push_back(int32_t(c.entry_dof.size()));
    }
    return c;
  }
};

}  // namespace

void mapping_eval_2d(const double* X, const double* xi, double* x, double J[2][2]) {
  double l[2][4], g[2][4];
  for (int e = 0; e < 2; ++e)
    for (int a = 0; a < 4; ++a) {
      l[e][a] = map_lag(a, xi[e]);
      g[e][a] = map_dlag(a, xi[e]);
    }
  x[0] = x[1] = 0;
  J[0][0] = J[0][1] = J[1][0] = J[1][1] = 0;
  for (int t = 0; t < kMapPts2D; ++t) {
    const int a = t % 4, b = t / 4;
    const double s = l[0][a] * l[1][b], d0 = g[0][a] * l[1][b], d1 = l[0][a] * g[1][b];
    for (int i = 0; i < 2; ++i) {
      const double Xi = X[2 * t + i];
      x[i] += s * Xi;
      J[i][0] += d0 * Xi;
      J[i][1] += d1 * Xi;
    }
  }
}

Mesh2D build_shell_2d(int refine, double R0, double R1, bool mapping_q_on_all_cells) {
  if (refine < 0 || refine > 10) throw std::invalid_argument("2D refinement must be in [0,10]");
  if (!(R0 > 0 && R1 > R0)) throw std::invalid_argument("2D shell radii: 0 < R0 < R1");
  Mesh2D m;
  m.refine = refine;
  m.R0 = R0;
  m.R1 = R1;
  // ---- coarse hyper_shell: 12 cells, outer ring first (GridGenerator::hyper_shell<2>)
  const int N0 = 12;
  std::vector<double> V;  // vertex coordinates
  for (int i = 0; i < N0; ++i) {
    V.push_back(std::cos(2 * kPi2D * i / N0) * R1);
    V.push_back(std::sin(2 * kPi2D * i / N0) * R1);
  }
  for (int i = 0; i < N0; ++i) {
    V.push_back(V[2 * i] * (R0 / R1));
    V.push_back(V[2 * i + 1] * (R0 / R1));
  }
  std::vector<std::array<int, 4>> cells;
  // per cell: which of its 4 lines (deal.II order x=0, x=1, y=0, y=1) lies on
  // the inner (bit 1) / outer (bit 2) boundary, as 2 bits per line
  std::vector<std::array<uint8_t, 4>> cell_bnd;
  for (int i = 0; i < N0; ++i) {
    cells.push_back({i, (i + 1) % N0, N0 + i, N0 + (i + 1) % N0});
    // v0 v1 outer (line y=0), v2 v3 inner (line y=1)
    cell_bnd.push_back({0, 0, kBndOuter, kBndInner});
  }
  // ---- refinement in tree order (children lexicographic)
  for (int l = 0; l < refine; ++l) {
    std::map<std::pair<int, int>, int> mid;
    auto line_mid = [&](int a, int b) {
      const auto key = std::make_pair(std::min(a, b), std::max(a, b));
      auto it = mid.find(key);
      if (it != mid.end()) return it->second;
      double p[2];
      mid_line(&V[2 * a], &V[2 * b], p);
      const int id = int(V.size() / 2);
      V.push_back(p[0]);
      V.push_back(p[1]);
      mid.emplace(key, id);
      return id;
    };
    std::vector<std::array<int, 4>> nc;
    std::vector<std::array<uint8_t, 4>> nb;
    nc.reserve(4 * cells.size());
    for (size_t c = 0; c < cells.size(); ++c) {
      const auto& v = cells[c];
      // lines: 0 = (v0, v2), 1 = (v1, v3), 2 = (v0, v1), 3 = (v2, v3)
      const int m0 = line_mid(v[0], v[2]), m1 = line_mid(v[1], v[3]);
      const int m2 = line_mid(v[0], v[1]), m3 = line_mid(v[2], v[3]);
      double pts[16];
      const int ids[8] = {v[0], v[1], v[2], v[3], m0, m1, m2, m3};
      for (int k = 0; k < 8; ++k) {
        pts[2 * k] = V[2 * ids[k]];
        pts[2 * k + 1] = V[2 * ids[k] + 1];
      }
      const double w[8] = {-0.25, -0.25, -0.25, -0.25, 0.5, 0.5, 0.5, 0.5};
      double ctr[2];
      new_point(8, pts, w, ctr);
      const int ce = int(V.size() / 2);
      V.push_back(ctr[0]);
      V.push_back(ctr[1]);
      const auto& b = cell_bnd[c];
      // child 0 (lower left), 1 (lower right), 2 (upper left), 3 (upper right)
      nc.push_back({v[0], m2, m0, ce});
      nb.push_back({b[0], 0, b[2], 0});
      nc.push_back({m2, v[1], ce, m1});
      nb.push_back({0, b[1], b[2], 0});
      nc.push_back({m0, ce, v[2], m3});
      nb.push_back({b[0], 0, 0, b[3]});
      nc.push_back({ce, m1, m3, v[3]});
      nb.push_back({0, b[1], 0, b[3]});
    }
    cells.swap(nc);
    cell_bnd.swap(nb);
  }
  m.n_cells = int(cells.size());
  // ---- MappingQ(3) support points; boundary cells: spherical
  m.cell_map.resize(size_t(m.n_cells) * 2 * kMapPts2D);
  std::vector<uint8_t> has_bnd(m.n_cells, 0);
  for (int c = 0; c < m.n_cells; ++c) {
    double Vc[8];
    for (int k = 0; k < 4; ++k) {
      Vc[2 * k] = V[2 * cells[c][k]];
      Vc[2 * k + 1] = V[2 * cells[c][k] + 1];
    }
    for (int k = 0; k < 4; ++k) has_bnd[c] |= cell_bnd[c][k];
    support_points_2d(Vc, mapping_q_on_all_cells || has_bnd[c] != 0,
                      &m.cell_map[size_t(c) * 2 * kMapPts2D]);
  }
  // ---- DoF numbering: first-encounter support points, objects in deal.II order
  const int n_vtx_total = int(V.size() / 2);
  std::vector<int32_t> vtx_node(n_vtx_total, -1), vtx_num(n_vtx_total, -1);
  std::map<std::pair<int, int>, int> line_node;
  m.cell_q2.assign(size_t(m.n_cells) * 9, -1);
  m.cell_q1.assign(size_t(m.n_cells) * 4, -1);
  int nn = 0, nv = 0;
  std::vector<int32_t> node_line_a, node_line_b;  // for line nodes: end vertices (else -1)
  std::vector<int32_t> node_cell, node_lex;       // first cell / position of each node
  auto add_node = [&](int c, int lex, int a, int b) {
    node_cell.push_back(c);
    node_lex.push_back(lex);
    node_line_a.push_back(a);
    node_line_b.push_back(b);
    return nn++;
  };
  for (int c = 0; c < m.n_cells; ++c) {
    const auto& v = cells[c];
    for (int k = 0; k < 4; ++k) {
      const int vt = v[k];
      if (vtx_node[vt] < 0) {
        vtx_node[vt] = add_node(c, kQ1VertexToQ2Lex2D[k], -1, -1);
        vtx_num[vt] = nv++;
      }
      m.cell_q2[9 * size_t(c) + kQ1VertexToQ2Lex2D[k]] = vtx_node[vt];
      m.cell_q1[4 * size_t(c) + k] = vtx_num[vt];
    }
    const int lv[4][2] = {{v[0], v[2]}, {v[1], v[3]}, {v[0], v[1]}, {v[2], v[3]}};
    for (int k = 0; k < 4; ++k) {
      const auto key = std::make_pair(std::min(lv[k][0], lv[k][1]), std::max(lv[k][0], lv[k][1]));
      auto it = line_node.find(key);
      int id;
      if (it == line_node.end()) {
        id = add_node(c, kQ2HierToLex2D[4 + k], lv[k][0], lv[k][1]);
        line_node.emplace(key, id);
      } else {
        id = it->second;
      }
      m.cell_q2[9 * size_t(c) + kQ2HierToLex2D[4 + k]] = id;
    }
    m.cell_q2[9 * size_t(c) + 4] = add_node(c, 4, -1, -1);
  }
  m.n_vnodes = nn;
  m.n_vertices = nv;
  m.vertex_vnode.assign(nv, -1);
  m.vnode_vertex.assign(nn, -1);
  for (int vt = 0; vt < n_vtx_total; ++vt)
    if (vtx_num[vt] >= 0) {
      m.vertex_vnode[vtx_num[vt]] = vtx_node[vt];
      m.vnode_vertex[vtx_node[vt]] = vtx_num[vt];
    }
  // ---- support point coordinates: MappingQ(3) and MappingQ1 images
  m.xy.assign(size_t(nn) * 2, 0.0);
  m.xy_q1.assign(size_t(nn) * 2, 0.0);
  for (int n = 0; n < nn; ++n) {
    const int c = node_cell[n], lex = node_lex[n];
    const double xi[2] = {0.5 * (lex % 3), 0.5 * (lex / 3)};
    const auto& v = cells[c];
    // bilinear image from the cell's vertices (MappingQ1)
    for (int d = 0; d < 2; ++d) {
      double s = 0;
      for (int k = 0; k < 4; ++k)
        s += ((k & 1) ? xi[0] : 1 - xi[0]) * ((k & 2) ? xi[1] : 1 - xi[1]) * V[2 * v[k] + d];
      m.xy_q1[2 * size_t(n) + d] = s;
    }
    if (m.vnode_vertex[n] >= 0) {
      // a vertex: exact
      int vt = -1;
      for (int k = 0; k < 4; ++k)
        if (kQ1VertexToQ2Lex2D[k] == lex) vt = v[k];
      m.xy[2 * size_t(n)] = V[2 * vt];
      m.xy[2 * size_t(n) + 1] = V[2 * vt + 1];
    } else {
      double x[2], J[2][2];
      mapping_eval_2d(&m.cell_map[size_t(c) * 2 * kMapPts2D], xi, x, J);
      m.xy[2 * size_t(n)] = x[0];
      m.xy[2 * size_t(n) + 1] = x[1];
    }
  }
  // ---- boundary flags: the support points of boundary lines
  m.vnode_bnd.assign(nn, 0);
  for (int c = 0; c < m.n_cells; ++c)
    for (int k = 0; k < 4; ++k) {
      const uint8_t bit = cell_bnd[c][k];
      if (!bit) continue;
      // lex points of line k: x=0: a=0; x=1: a=2; y=0: b=0; y=1: b=2
      for (int t = 0; t < 3; ++t) {
        const int lex = k == 0 ? 3 * t : k == 1 ? 2 + 3 * t : k == 2 ? t : 6 + t;
        m.vnode_bnd[m.cell_q2[9 * size_t(c) + lex]] |= bit;
      }
    }
  // ---- CellAccessor::diameter: the longer vertex diagonal
  m.cell_diameter.resize(m.n_cells);
  for (int c = 0; c < m.n_cells; ++c) {
    const auto& v = cells[c];
    auto dist = [&](int a, int b) {
      const double dx = V[2 * a] - V[2 * b], dy = V[2 * a + 1] - V[2 * b + 1];
      return std::sqrt(dx * dx + dy * dy);
    };
    m.cell_diameter[c] = std::max(dist(v[0], v[3]), dist(v[1], v[2]));
  }
  (void)node_line_a;
  (void)node_line_b;
  return m;
}

std::vector<int32_t> nse_cell_dofs_2d(const Mesh2D& m) {
  std::vector<int32_t> out(size_t(m.n_cells) * kNseDofs2D);
  const int nu = m.n_u();
  for (int c = 0; c < m.n_cells; ++c)
    for (int i = 0; i < kNseDofs2D; ++i) {
      const SysDof s = system_dof_2d(i);
      out[size_t(c) * kNseDofs2D + i] = s.comp < 2 ? 2 * m.cell_q2[9 * size_t(c) + s.lex] + s.comp
                                                   : nu + m.cell_q1[4 * size_t(c) + s.lex];
    }
  return out;
}

std::vector<int32_t> temperature_cell_dofs_2d(const Mesh2D& m) {
  std::vector<int32_t> out(size_t(m.n_cells) * 9);
  for (int c = 0; c < m.n_cells; ++c)
    for (int i = 0; i < 9; ++i) out[9 * size_t(c) + i] = m.cell_q2[9 * size_t(c) + kQ2HierToLex2D[i]];
  return out;
}

namespace {
// unit outward normal of every outer boundary line through the cell's
// MappingQ(3) at its support points, summed per point and normalised
// (compute_no_normal_flux_constraints with the reference's mapping)
std::vector<double> mapping_normals_2d(const Mesh2D& m, uint8_t bit) {
  std::vector<double> nrm(size_t(m.n_vnodes) * 2, 0.0);
  for (int c = 0; c < m.n_cells; ++c) {
    const double* X = &m.cell_map[size_t(c) * 2 * kMapPts2D];
    for (int f = 0; f < 4; ++f) {
      const int axis = f / 2, side = f % 2;  // faces x=0, x=1, y=0, y=1
      bool on = true;
      for (int l = 0; l < 9 && on; ++l) {
        const int ab[2] = {l % 3, l / 3};
        if (ab[axis] == 2 * side) on = (m.vnode_bnd[m.cell_q2[9 * size_t(c) + l]] & bit) != 0;
      }
      if (!on) continue;
      for (int l = 0; l < 9; ++l) {
        const int ab[2] = {l % 3, l / 3};
        if (ab[axis] != 2 * side) continue;
        const double xi[2] = {0.5 * ab[0], 0.5 * ab[1]};
        double x[2], J[2][2];
        mapping_eval_2d(X, xi, x, J);
        // tangent along the other axis t = J[:, 1 - axis]; outward normal
        const int t = 1 - axis;
        double n[2] = {J[1][t], -J[0][t]};  // t rotated by -90 degrees
        // orient outward: face at side 1 of axis 0 has outward +xi_0, etc.
        const double dir = (side ? 1.0 : -1.0);
        const double o = (axis == 0 ? J[0][0] * n[0] + J[1][0] * n[1] : J[0][1] * n[0] + J[1][1] * n[1]);
        const double s = (o * dir >= 0 ? 1.0 : -1.0) / std::sqrt(n[0] * n[0] + n[1] * n[1]);
        double* out = &nrm[2 * size_t(m.cell_q2[9 * size_t(c) + l])];
        out[0] += s * n[0];
        out[1] += s * n[1];
      }
    }
  }
  return nrm;
}
}  // namespace

Constraints nse_constraints_2d(const Mesh2D& m) {
  const int nu = m.n_u(), np = m.n_p();
  Builder2D b(nu + np);
  for (int n = 0; n < m.n_vnodes; ++n)
    if (m.vnode_bnd[n] & kBndInner)
      for (int c = 0; c < 2; ++c) b.has[2 * n + c] = 1;
  const std::vector<double> cn = mapping_normals_2d(m, kBndOuter);
  const double eps = 2.220446049250313e-16;
  for (int n = 0; n < m.n_vnodes; ++n) {
    if (!(m.vnode_bnd[n] & kBndOuter) || (m.vnode_bnd[n] & kBndInner)) continue;
    const double* x = &cn[2 * size_t(n)];
    const double r = std::sqrt(x[0] * x[0] + x[1] * x[1]);
    const double nrm[2] = {x[0] / r, x[1] / r};
    // deal.II: the component of the largest normal entry is constrained
    const int k = std::fabs(nrm[1]) > std::fabs(nrm[0]) + 1e-10 ? 1 : 0;
    const int dk = 2 * n + k, dot = 2 * n + (1 - k);
    b.has[dk] = 1;
    const double w = nrm[1 - k] / nrm[k];
    if (std::fabs(w) > eps) b.entries[dk][dot] += -w;
  }
  return b.close();
}

double temperature_initial_2d(const double* p, double R0, double R1) {
  // TemperatureInitialValues<2>: rotate = true, alpha = pi / 3; the centres
  // are formed as rotation * c * transpose(rotation), i.e. R (R c): the
  // Gaussians sit at the base centres rotated by 2 alpha
  const double a = kPi2D / 3;
  const double Rm[2][2] = {{std::cos(a), -std::sin(a)}, {std::sin(a), std::cos(a)}};
  auto rot2 = [&](const double* cin, double* out) {
    const double t[2] = {Rm[0][0] * cin[0] + Rm[0][1] * cin[1], Rm[1][0] * cin[0] + Rm[1][1] * cin[1]};
    // (t * R^T)_j = sum_i t_i R_ji
    out[0] = t[0] * Rm[0][0] + t[1] * Rm[0][1];
    out[1] = t[0] * Rm[1][0] + t[1] * Rm[1][1];
  };
  const double b1[2] = {R0 + (R1 - R0) * 0.35, 0}, b2[2] = {0, R0 + (R1 - R0) * 0.65};
  double c1[2], c2[2];
  rot2(b1, c1);
  rot2(b2, c2);
  const double cov = 20.0 / ((R1 - R0) / 2.0);
  const double sqrt_det = std::sqrt(cov * cov);
  const double norm = std::sqrt(std::pow(2 * kPi2D, 2));
  double q1 = 0, q2 = 0;
  for (int d = 0; d < 2; ++d) {
    q1 += (p[d] - c1[d]) * cov * (p[d] - c1[d]);
    q2 += (p[d] - c2[d]) * cov * (p[d] - c2[d]);
  }
  return sqrt_det * std::exp(-0.5 * q1) / norm + sqrt_det * std::exp(-0.5 * q2) / norm;
}

Constraints temperature_constraints_2d(const Mesh2D& m) {
  Builder2D b(m.n_vnodes);
  for (int n = 0; n < m.n_vnodes; ++n)
    if (m.vnode_bnd[n] & kBndInner) {
      b.has[n] = 1;
      b.inhom[n] = temperature_initial_2d(&m.xy_q1[2 * size_t(n)], m.R0, m.R1);
    }
  return b.close();
}

}  // namespace dcp
