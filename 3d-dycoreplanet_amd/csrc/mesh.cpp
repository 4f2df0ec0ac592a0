// Host setup: refined mesh, DoF numbering, constraints. See mesh.h.
#include "mesh.h"

#include <algorithm>
#include <cmath>
#include <functional>
#include <map>
#include <stdexcept>
#include <array>
#include <tuple>
#include <unordered_map>

#include "fe_tables.h"

namespace dcp {

namespace {

constexpr double kPi = 3.14159265358979323846;

// Morton decode with x in the lowest bit: deal.II's child index c = cx + 2cy + 4cz
// applied recursively, so tree order of the refined cells = increasing code.
void demorton(uint32_t m, int refine, int& i, int& j, int& k) {
  i = j = k = 0;
  for (int b = 0; b < refine; ++b) {
    i |= ((m >> (3 * b)) & 1u) << b;
    j |= ((m >> (3 * b + 1)) & 1u) << b;
    k |= ((m >> (3 * b + 2)) & 1u) << b;
  }
}

double cell_diameter_of(const Mesh& m, int c) {
  // CellAccessor::diameter for hexes: longest of the 4 space diagonals.
  static const int diag[4][2] = {{0, 7}, {1, 6}, {2, 5}, {3, 4}};
  double d = 0;
  for (const auto& dg : diag) {
    const double* a = &m.xyz[3 * m.cell_q2[27 * c + kQ1VertexToQ2Lex[dg[0]]]];
    const double* b = &m.xyz[3 * m.cell_q2[27 * c + kQ1VertexToQ2Lex[dg[1]]]];
    const double s = std::sqrt((a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) +
                               (a[2] - b[2]) * (a[2] - b[2]));
    d = std::max(d, s);
  }
  return d;
}

// Numbers nodes in deal.II first-encounter order: per cell (tree order),
// vertices, lines, faces, interior (hierarchic order), and vertices separately
// (the Q1 / pressure numbering). `key_of(cell, lex)` gives a global key.
template <class KeyFn>
void number_nodes(Mesh& m, size_t n_keys, KeyFn key_of, std::vector<int32_t>& key_node) {
  key_node.assign(n_keys, -1);
  std::vector<int32_t> key_vertex(n_keys, -1);
  m.cell_q2.assign(size_t(m.n_cells) * 27, -1);
  m.cell_q1.assign(size_t(m.n_cells) * 8, -1);
  int nn = 0, nv = 0;
  for (int c = 0; c < m.n_cells; ++c) {
    for (int h = 0; h < 27; ++h) {
      const int lex = kQ2HierToLex[h];
      const size_t key = key_of(c, lex);
      if (key_node[key] < 0) key_node[key] = nn++;
      m.cell_q2[27 * size_t(c) + lex] = key_node[key];
      if (h < 8) {
        if (key_vertex[key] < 0) key_vertex[key] = nv++;
        m.cell_q1[8 * size_t(c) + h] = key_vertex[key];
      }
    }
  }
  m.n_vnodes = nn;
  m.n_vertices = nv;
  m.vertex_vnode.assign(nv, -1);
  m.vnode_vertex.assign(nn, -1);
  for (int c = 0; c < m.n_cells; ++c)
    for (int v = 0; v < 8; ++v) {
      const int vid = m.cell_q1[8 * size_t(c) + v];
      const int nid = m.cell_q2[27 * size_t(c) + kQ1VertexToQ2Lex[v]];
      m.vertex_vnode[vid] = nid;
      m.vnode_vertex[nid] = vid;
    }
}

// Panels of the cube (outward normal n, tangents e1, e2 with e1 x e2 = n), so
// that (xi, eta, zeta) = (e1, e2, radial) is right-handed in every cell.
constexpr int kShellPanel[6][3][3] = {
    {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}},    // +x
    {{-1, 0, 0}, {0, 0, 1}, {0, 1, 0}},   // -x
    {{0, 1, 0}, {0, 0, 1}, {1, 0, 0}},    // +y
    {{0, -1, 0}, {1, 0, 0}, {0, 0, 1}},   // -y
    {{0, 0, 1}, {1, 0, 0}, {0, 1, 0}},    // +z
    {{0, 0, -1}, {0, 1, 0}, {1, 0, 0}}};  // -z

size_t shell_key_of_point(int N, const int P[3], int t) {
  const size_t L2 = size_t(2 * N + 1);
  return ((size_t(P[0] + N) * L2 + size_t(P[1] + N)) * L2 + size_t(P[2] + N)) * L2 + size_t(t);
}

// Global key of Q2 lattice node `lex` of shell cell c: the integer point P on
// the cube surface [-N,N]^3 (Q2 lattice units) the node's direction comes
// from, plus its radial lattice index t (0 = inner sphere).
void shell_surf_point(int N, int refine, int c, int lex, int P[3], int& t) {
  const int p = c / (N * N * N);
  int i, j, k;
  demorton(uint32_t(c % (N * N * N)), refine, i, j, k);
  const int a = 2 * i + lex % 3, b = 2 * j + (lex / 3) % 3;
  t = 2 * k + lex / 9;
  for (int d = 0; d < 3; ++d)
    P[d] = N * kShellPanel[p][0][d] + (a - N) * kShellPanel[p][1][d] + (b - N) * kShellPanel[p][2][d];
}

size_t shell_node_key(int N, int refine, int c, int lex) {
  int P[3], t;
  shell_surf_point(N, refine, c, lex, P, t);
  return shell_key_of_point(N, P, t);
}

}  // namespace

Mesh build_shell(int refine, double R0, double R1, bool mapping_q_on_all_cells) {
  if (refine < 0 || refine > 8) throw std::invalid_argument("shell refinement must be in [0,8]");
  Mesh m;
  m.cuboid = false;
  m.refine = refine;
  m.N = 1 << refine;
  m.R0 = R0;
  m.R1 = R1;
  const int N = m.N, L2 = 2 * N + 1;  // Q2 lattice points per edge
  m.n_cells = 6 * N * N * N;
  const int (&panel)[6][3][3] = kShellPanel;
  // Global key: integer point P on the cube surface [-N,N]^3 plus radial index t.
  const size_t n_keys = size_t(L2) * L2 * L2 * L2;
  auto surf_point = [&](int c, int lex, int P[3], int& t) {
    shell_surf_point(N, refine, c, lex, P, t);
  };
  auto key_of = [&](int c, int lex) { return shell_node_key(N, refine, c, lex); };
  std::vector<int32_t> key_node;
  number_nodes(m, n_keys, key_of, key_node);
  m.cell_coarse.resize(m.n_cells);
  for (int c = 0; c < m.n_cells; ++c) m.cell_coarse[c] = c / (N * N * N);
  // ---- vertex directions: hyper_shell's coarse corners (+-1,+-1,+-1)/sqrt(3),
  // then per refinement level every line midpoint by get_intermediate_point
  // (geodesic, w = 1/2) and every quad centre by get_new_point over its 4
  // vertices (weight -1/4) and 4 line midpoints (+1/2) — TriaAccessor::
  // center(true, true). Shell refinement is a radial extrusion: radial lines
  // keep the direction (collinear case of get_intermediate_point), hex centres
  // take their spherical faces' centre direction, so directions live on the
  // unit sphere and are keyed by the surface lattice point P (Q2 lattice units).
  std::unordered_map<int64_t, std::array<double, 3>> dir_of;
  auto skey = [&](const int P[3]) {
    return (int64_t(P[0] + N) * L2 + (P[1] + N)) * L2 + (P[2] + N);
  };
  const double o[3] = {0, 0, 0};
  for (int p = 0; p < 6; ++p) {
    // panel lattice (i, j) in [0, N]^2 of vertices -> surface point
    auto P_of = [&](int i, int j, int P[3]) {
      for (int d = 0; d < 3; ++d)
        P[d] = N * panel[p][0][d] + (2 * i - N) * panel[p][1][d] + (2 * j - N) * panel[p][2][d];
    };
    auto get = [&](int i, int j) -> const std::array<double, 3>& {
      int P[3];
      P_of(i, j, P);
      return dir_of.at(skey(P));
    };
    auto has = [&](int i, int j, int64_t& k) {
      int P[3];
      P_of(i, j, P);
      k = skey(P);
      return dir_of.count(k) != 0;
    };
    for (int j = 0; j <= N; j += N)
      for (int i = 0; i <= N; i += N) {
        int P[3];
        P_of(i, j, P);
        const int64_t k = skey(P);
        if (dir_of.count(k)) continue;
        std::array<double, 3> d;
        for (int e = 0; e < 3; ++e) d[e] = (P[e] > 0 ? 1.0 : -1.0) / std::sqrt(3.0);
        dir_of[k] = d;
      }
    auto midpoint = [&](int i0, int j0, int i1, int j1, int im, int jm) {
      int64_t k;
      if (has(im, jm, k)) return;
      int Pa[3], Pb[3];
      P_of(i0, j0, Pa);
      P_of(i1, j1, Pb);
      // canonical line orientation: lower surface key first
      const bool sw = skey(Pb) < skey(Pa);
      const auto& a = sw ? get(i1, j1) : get(i0, j0);
      const auto& b = sw ? get(i0, j0) : get(i1, j1);
      std::array<double, 3> out;
      spherical_intermediate(o, a.data(), b.data(), 0.5, out.data());
      dir_of[k] = out;
    };
    for (int s = N; s > 1; s /= 2) {
      const int h = s / 2;
      for (int j = 0; j <= N; j += s)
        for (int i = 0; i < N; i += s) midpoint(i, j, i + s, j, i + h, j);
      for (int i = 0; i <= N; i += s)
        for (int j = 0; j < N; j += s) midpoint(i, j, i, j + s, i, j + h);
      for (int j = 0; j < N; j += s)
        for (int i = 0; i < N; i += s) {
          int64_t k;
          if (has(i + h, j + h, k)) continue;
          const int pi[8][2] = {{i, j},     {i + s, j},     {i, j + s},     {i + s, j + s},
                                {i, j + h}, {i + s, j + h}, {i + h, j}, {i + h, j + s}};
          double src[24];
          for (int t = 0; t < 8; ++t) {
            const auto& d = get(pi[t][0], pi[t][1]);
            for (int e = 0; e < 3; ++e) src[3 * t + e] = d[e];
          }
          const double w[8] = {-0.25, -0.25, -0.25, -0.25, 0.5, 0.5, 0.5, 0.5};
          std::array<double, 3> out;
          spherical_new_points(o, 8, src, 1, w, out.data());
          dir_of[k] = out;
        }
    }
  }
  // radial levels: collinear get_intermediate_point = arithmetic midpoints
  std::vector<double> rad(N + 1, 0.0);
  rad[0] = R0;
  rad[N] = R1;
  for (int s = N; s > 1; s /= 2)
    for (int k = 0; k < N; k += s) rad[k + s / 2] = 0.5 * rad[k + s] + 0.5 * rad[k];
  // ---- MappingQ(3) support points of every cell from its 8 vertices
  m.mapping_q_on_all_cells = mapping_q_on_all_cells;
  m.cell_map.assign(size_t(m.n_cells) * 3 * kMapPts, 0.0);
  for (int c = 0; c < m.n_cells; ++c) {
    double V[24];
    int kz = 0;
    for (int v = 0; v < 8; ++v) {
      int P[3], t;
      surf_point(c, kQ1VertexToQ2Lex[v], P, t);
      const auto& d = dir_of.at(skey(P));
      for (int e = 0; e < 3; ++e) V[3 * v + e] = rad[t / 2] * d[e];
      if (v == 0) kz = t / 2;
    }
    // CellAccessor::has_boundary_lines(): the innermost and outermost layers
    const bool boundary = kz == 0 || kz == N - 1;
    mapping_support_points(V, mapping_q_on_all_cells || boundary, &m.cell_map[size_t(c) * 3 * kMapPts]);
  }
  // ---- Q2 support points = the cell's map at (a, b, c) / 2 (first cell)
  m.xyz.assign(size_t(m.n_vnodes) * 3, 0.0);
  m.vnode_bnd.assign(m.n_vnodes, 0);
  std::vector<char> done(m.n_vnodes, 0);
  for (int c = 0; c < m.n_cells; ++c)
    for (int lex = 0; lex < 27; ++lex) {
      const int n = m.cell_q2[27 * size_t(c) + lex];
      if (done[n]) continue;
      done[n] = 1;
      int P[3], t;
      surf_point(c, lex, P, t);
      double* x = &m.xyz[3 * size_t(n)];
      if (lex % 3 != 1 && (lex / 3) % 3 != 1 && lex / 9 != 1) {
        const auto& d = dir_of.at(skey(P));  // a vertex: exact
        for (int e = 0; e < 3; ++e) x[e] = rad[t / 2] * d[e];
      } else {
        const double xi[3] = {0.5 * (lex % 3), 0.5 * ((lex / 3) % 3), 0.5 * (lex / 9)};
        double J[3][3];
        mapping_eval(&m.cell_map[size_t(c) * 3 * kMapPts], xi, x, J);
      }
      if (t == 0) m.vnode_bnd[n] |= kBndInner;
      if (t == 2 * N) m.vnode_bnd[n] |= kBndOuter;
    }
  m.cell_diameter.resize(m.n_cells);
  for (int c = 0; c < m.n_cells; ++c) m.cell_diameter[c] = cell_diameter_of(m, c);
  m.global_diameter = 2 * R1;
  return m;
}

Mesh build_cube(int refine, double length) {
  if (refine < 0 || refine > 9) throw std::invalid_argument("cube refinement must be in [0,9]");
  Mesh m;
  m.cuboid = true;
  m.refine = refine;
  m.N = 1 << refine;
  const int N = m.N, L2 = 2 * N + 1;
  m.n_cells = N * N * N;
  auto lattice = [&](int c, int lex, int& a, int& b, int& d) {
    int i, j, k;
    demorton(uint32_t(c), refine, i, j, k);
    a = 2 * i + lex % 3;
    b = 2 * j + (lex / 3) % 3;
    d = 2 * k + lex / 9;
  };
  auto key_of = [&](int c, int lex) {
    int a, b, d;
    lattice(c, lex, a, b, d);
    return (size_t(d) * L2 + size_t(b)) * L2 + size_t(a);
  };
  std::vector<int32_t> key_node;
  number_nodes(m, size_t(L2) * L2 * L2, key_of, key_node);
  m.cell_coarse.assign(m.n_cells, 0);
  m.xyz.assign(size_t(m.n_vnodes) * 3, 0.0);
  m.vnode_bnd.assign(m.n_vnodes, 0);
  const double h = 1.0 / (2.0 * N) / length;
  for (int c = 0; c < m.n_cells; ++c)
    for (int lex = 0; lex < 27; ++lex) {
      const int n = m.cell_q2[27 * size_t(c) + lex];
      int a, b, d;
      lattice(c, lex, a, b, d);
      m.xyz[3 * size_t(n) + 0] = a * h;
      m.xyz[3 * size_t(n) + 1] = b * h;
      m.xyz[3 * size_t(n) + 2] = d * h;
      uint8_t bits = 0;
      if (a == 0) bits |= kBndX0;
      if (a == 2 * N) bits |= kBndX1;
      if (b == 0) bits |= kBndY0;
      if (b == 2 * N) bits |= kBndY1;
      if (d == 0) bits |= kBndZ0;
      if (d == 2 * N) bits |= kBndZ1;
      m.vnode_bnd[n] = bits;
    }
  m.cell_diameter.resize(m.n_cells);
  for (int c = 0; c < m.n_cells; ++c) m.cell_diameter[c] = cell_diameter_of(m, c);
  // MappingQ(3) on a FlatManifold box = the trilinear map of its vertices
  m.cell_map.assign(size_t(m.n_cells) * 3 * kMapPts, 0.0);
  for (int c = 0; c < m.n_cells; ++c) {
    double V[24];
    for (int v = 0; v < 8; ++v)
      for (int e = 0; e < 3; ++e)
        V[3 * v + e] = m.xyz[3 * size_t(m.cell_q2[27 * size_t(c) + kQ1VertexToQ2Lex[v]]) + e];
    mapping_support_points(V, false, &m.cell_map[size_t(c) * 3 * kMapPts]);
  }
  // planet_geometry.tpp:35 center = (p0+p1)/2, rescaled with 1/L (boussinesq_model.tpp:54)
  for (int d = 0; d < 3; ++d) m.center[d] = 0.5 / length;
  m.global_diameter = std::sqrt(3.0) / length;
  return m;
}

Mesh build_mesh(const Parameters& prm) {
  if (prm.space_dimension != 3) throw std::invalid_argument("only space dimension 3 is built");
  const double L = prm.reference_quantities.length;
  if (prm.cuboid_geometry) return build_cube(int(prm.initial_global_refinement), L);
  return build_shell(int(prm.initial_global_refinement), prm.physical_constants.R0 / L,
                     prm.physical_constants.R1 / L);
}

// ---------------------------------------------------------------------------
// Constraints

namespace {

struct Builder {
  // dof -> (entries, inhomogeneity); std::map keeps entries sorted by dof.
  std::vector<int> has;
  std::vector<std::map<int, double>> entries;
  std::vector<double> inhom;
  explicit Builder(int n) : has(n, 0), entries(n), inhom(n, 0.0) {}
  bool is_constrained(int d) const { return has[d] != 0; }
  void add_line(int d) { has[d] = 1; }
  void add_entry(int d, int t, double w) { entries[d][t] += w; }

  // AffineConstraints::close(): resolve chains (targets that are themselves
  // constrained are replaced by their expansion), sort entries.
  Constraints close() {
    const int n = int(has.size());
    std::vector<int> state(n, 0);  // 0 = unresolved, 1 = in progress, 2 = resolved
    std::function<void(int)> resolve = [&](int d) {
      if (state[d] == 2) return;
      if (state[d] == 1) throw std::runtime_error("cyclic constraints");
      state[d] = 1;
      std::map<int, double> out;
      double g = inhom[d];
      for (const auto& e : entries[d]) {
        if (has[e.first]) {
          resolve(e.first);
          for (const auto& e2 : entries[e.first]) out[e2.first] += e.second * e2.second;
          g += e.second * inhom[e.first];
        } else {
          out[e.first] += e.second;
        }
      }
      entries[d].swap(out);
      inhom[d] = g;
      state[d] = 2;
    };
    Constraints c;
    c.n_dofs = n;
    c.line_of.assign(n, -1);
    c.entry_ptr.push_back(0);
    for (int d = 0; d < n; ++d) {
      if (!has[d]) continue;
      resolve(d);
      c.line_of[d] = c.n_lines();
      c.line_dof.push_back(d);
      for (const auto& e : entries[d]) {
        c.entry_dof.push_back(e.first);
        c.entry_w.push_back(e.second);
      }
      c.entry_ptr.push_back(int(c.entry_dof.size()));
      c.inhomogeneity.push_back(inhom[d]);
    }
    return c;
  }
};

// VectorTools::compute_no_normal_flux_constraints, one normal per support
// point (deal.II internal::add_constraint, dim = 3): the constrained component
// is the dominant one with the 1e-10 / 2e-10 tie-breaking offsets, entries with
// |ratio| <= eps are dropped; already constrained dofs are left alone.
void add_no_normal_flux(Builder& b, const int dofs[3], const double n[3]) {
  const double eps = 2.220446049250313e-16;
  int k;
  if (std::fabs(n[0]) >= std::fabs(n[1]) + 1e-10 && std::fabs(n[0]) >= std::fabs(n[2]) + 2e-10)
    k = 0;
  else if (std::fabs(n[1]) + 1e-10 >= std::fabs(n[0]) && std::fabs(n[1]) >= std::fabs(n[2]) + 1e-10)
    k = 1;
  else
    k = 2;
  if (b.is_constrained(dofs[k])) return;
  b.add_line(dofs[k]);
  for (int d = 0; d < 3; ++d) {
    if (d == k) continue;
    const double r = n[d] / n[k];
    if (std::fabs(r) > eps) b.add_entry(dofs[k], dofs[d], -r);
  }
}

// Periodic identification of the x = 1 face onto x = 0 and y = 1 onto y = 0
// (DoFTools::make_periodicity_constraints, boussinesq_model.tpp:265-285). The
// partner node is found from the lattice position. `dof_of(vnode)` < 0 skips.
template <class DofFn>
void add_periodic(const Mesh& m, Builder& b, DofFn dof_of, int n_comp) {
  std::map<std::tuple<long, long, long>, int> at;
  auto key = [&](int n) {
    // xyz = lattice * h with h = 1/(2N L) and global_diameter = sqrt(3)/L
    const double s = 2.0 * m.N * std::sqrt(3.0) / m.global_diameter;
    return std::make_tuple(std::lround(m.xyz[3 * n] * s), std::lround(m.xyz[3 * n + 1] * s),
                           std::lround(m.xyz[3 * n + 2] * s));
  };
  for (int n = 0; n < m.n_vnodes; ++n) at[key(n)] = n;
  const long full = 2L * m.N;
  for (int dir = 0; dir < 2; ++dir) {
    const uint8_t hi = dir == 0 ? kBndX1 : kBndY1;
    for (int n = 0; n < m.n_vnodes; ++n) {
      if (!(m.vnode_bnd[n] & hi)) continue;
      auto k = key(n);
      if (dir == 0) std::get<0>(k) -= full; else std::get<1>(k) -= full;
      const int partner = at.at(k);
      for (int comp = 0; comp < n_comp; ++comp) {
        const int ds = dof_of(n, comp), dm = dof_of(partner, comp);
        if (ds < 0 || dm < 0 || b.is_constrained(ds)) continue;
        b.add_line(ds);
        b.add_entry(ds, dm, 1.0);
      }
    }
  }
}

double lag2(int a, double x) {
  return a == 0 ? 2 * (x - 0.5) * (x - 1) : a == 1 ? -4 * x * (x - 1) : 2 * x * (x - 0.5);
}
double dlag2(int a, double x) { return a == 0 ? 4 * x - 3 : a == 1 ? -8 * x + 4 : 4 * x - 1; }

}  // namespace

std::vector<double> consistent_normals(const Mesh& m, uint8_t boundary_bit) {
  // n_i = sum_cells int grad(phi_i) dx with the cell's MappingQ(3) and
  // QGauss(3), i.e. minus the row of B^T 1 of node i. Interior rows vanish to
  // roundoff, so constraining u_i . n_i = 0 on the boundary makes C^T B^T 1 = 0
  // exactly (consistent normals, Engelman, Sani & Gresho 1982).
  std::vector<double> nrm(size_t(m.n_vnodes) * 3, 0.0);
  for (int c = 0; c < m.n_cells; ++c) {
    bool touches = false;
    for (int l = 0; l < 27; ++l) touches |= (m.vnode_bnd[m.cell_q2[27 * size_t(c) + l]] & boundary_bit) != 0;
    if (!touches) continue;
    const double* X = &m.cell_map[size_t(c) * 3 * kMapPts];
    for (int q = 0; q < 27; ++q) {
      const double p[3] = {kGaussX[q % 3], kGaussX[(q / 3) % 3], kGaussX[q / 9]};
      const double w = kGaussW[q % 3] * kGaussW[(q / 3) % 3] * kGaussW[q / 9];
      double x[3], J[3][3], gref[27][3];
      mapping_eval(X, p, x, J);
      for (int n = 0; n < 27; ++n) {
        const int a = n % 3, b = (n / 3) % 3, cc = n / 9;
        gref[n][0] = dlag2(a, p[0]) * lag2(b, p[1]) * lag2(cc, p[2]);
        gref[n][1] = lag2(a, p[0]) * dlag2(b, p[1]) * lag2(cc, p[2]);
        gref[n][2] = lag2(a, p[0]) * lag2(b, p[1]) * dlag2(cc, p[2]);
      }
      // cofactor matrix: det(J) J^-T = cof(J); grad phi JxW = cof(J) gref w
      double cof[3][3];
      for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
          const int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
          cof[i][j] = J[i1][j1] * J[i2][j2] - J[i1][j2] * J[i2][j1];
        }
      for (int n = 0; n < 27; ++n) {
        double* out = &nrm[3 * size_t(m.cell_q2[27 * size_t(c) + n])];
        for (int i = 0; i < 3; ++i)
          out[i] += (cof[i][0] * gref[n][0] + cof[i][1] * gref[n][1] + cof[i][2] * gref[n][2]) * w;
      }
    }
  }
  return nrm;
}

std::vector<double> mapping_normals(const Mesh& m, uint8_t boundary_bit) {
  // VectorTools::compute_no_normal_flux_constraints (deal.II, called with the
  // reference's mapping at boussinesq_model.tpp:324-329): the unit outward
  // normal of each boundary face through the cell's mapping at the face's
  // support points; a support point shared by several faces gets the
  // normalised sum (the faces of a smooth sphere are all "close").
  std::vector<double> nrm(size_t(m.n_vnodes) * 3, 0.0);
  for (int c = 0; c < m.n_cells; ++c) {
    const double* X = &m.cell_map[size_t(c) * 3 * kMapPts];
    for (int f = 0; f < 6; ++f) {
      const int axis = f / 2, side = f % 2;
      bool on = true;
      for (int l = 0; l < 27 && on; ++l) {
        const int ab[3] = {l % 3, (l / 3) % 3, l / 9};
        if (ab[axis] == 2 * side) on = (m.vnode_bnd[m.cell_q2[27 * size_t(c) + l]] & boundary_bit) != 0;
      }
      if (!on) continue;
      for (int l = 0; l < 27; ++l) {
        const int ab[3] = {l % 3, (l / 3) % 3, l / 9};
        if (ab[axis] != 2 * side) continue;
        const double xi[3] = {0.5 * ab[0], 0.5 * ab[1], 0.5 * ab[2]};
        double x[3], J[3][3];
        mapping_eval(X, xi, x, J);
        // outward normal = +-(column t1 x column t2), t1, t2 the other two axes
        const int t1 = (axis + 1) % 3, t2 = (axis + 2) % 3;
        double n[3] = {J[1][t1] * J[2][t2] - J[2][t1] * J[1][t2], J[2][t1] * J[0][t2] - J[0][t1] * J[2][t2],
                       J[0][t1] * J[1][t2] - J[1][t1] * J[0][t2]};
        const double s = (side ? 1.0 : -1.0) / std::sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        double* out = &nrm[3 * size_t(m.cell_q2[27 * size_t(c) + l])];
        for (int d = 0; d < 3; ++d) out[d] += s * n[d];
      }
    }
  }
  return nrm;
}

Constraints nse_constraints(const Mesh& m, NormalMode mode) {
  const int nu = m.n_u(), np = m.n_p();
  Builder b(nu + np);
  if (m.cuboid) {
    add_periodic(m, b, [&](int n, int comp) {
      if (comp < 3) return 3 * n + comp;
      return m.vnode_vertex[n] >= 0 ? nu + m.vnode_vertex[n] : -1;
    }, 4);
    for (int n = 0; n < m.n_vnodes; ++n)
      if (m.vnode_bnd[n] & kBndZ0)
        for (int c = 0; c < 3; ++c)
          if (!b.is_constrained(3 * n + c)) b.add_line(3 * n + c);
    const double nz[3] = {0, 0, 1};
    for (int n = 0; n < m.n_vnodes; ++n)
      if ((m.vnode_bnd[n] & kBndZ1) && !(m.vnode_bnd[n] & kBndZ0)) {
        const int dofs[3] = {3 * n, 3 * n + 1, 3 * n + 2};
        add_no_normal_flux(b, dofs, nz);
      }
  } else {
    for (int n = 0; n < m.n_vnodes; ++n)
      if (m.vnode_bnd[n] & kBndInner)
        for (int c = 0; c < 3; ++c) b.add_line(3 * n + c);
    const std::vector<double> cn = mode == NormalMode::Consistent ? consistent_normals(m, kBndOuter)
                                   : mode == NormalMode::Mapping  ? mapping_normals(m, kBndOuter)
                                                                  : std::vector<double>();
    for (int n = 0; n < m.n_vnodes; ++n)
      if (m.vnode_bnd[n] & kBndOuter) {
        const double* x = mode == NormalMode::Radial ? &m.xyz[3 * size_t(n)] : &cn[3 * size_t(n)];
        const double r = std::sqrt(x[0] * x[0] + x[1] * x[1] + x[2] * x[2]);
        const double nn[3] = {x[0] / r, x[1] / r, x[2] / r};
        const int dofs[3] = {3 * n, 3 * n + 1, 3 * n + 2};
        add_no_normal_flux(b, dofs, nn);
      }
  }
  return b.close();
}

double temperature_initial_shell(const double* p, double R0, double R1) {
  // TemperatureInitialValues<3> (rotate = false): two Gaussians with
  // covariance diag(20 / ((R1-R0)/2)), centres (R0+0.35h,0,0), (0,R0+0.65h,0).
  const double cov = 20.0 / ((R1 - R0) / 2.0);
  const double c1[3] = {R0 + (R1 - R0) * 0.35, 0, 0};
  const double c2[3] = {0, R0 + (R1 - R0) * 0.65, 0};
  const double sqrt_det = std::sqrt(cov * cov * cov);
  const double norm = std::sqrt(std::pow(2 * kPi, 3));
  double q1 = 0, q2 = 0;
  for (int d = 0; d < 3; ++d) {
    q1 += (p[d] - c1[d]) * cov * (p[d] - c1[d]);
    q2 += (p[d] - c2[d]) * cov * (p[d] - c2[d]);
  }
  return sqrt_det * std::exp(-0.5 * q1) / norm + sqrt_det * std::exp(-0.5 * q2) / norm;
}

double temperature_initial_cuboid(const double* p, const double* center, double diameter) {
  // TemperatureInitialValuesCuboid<3>: covariance diag(1/(0.1 d)^2)
  const double cov = 1.0 / std::pow(diameter * 0.1, 2);
  double q = 0;
  for (int d = 0; d < 3; ++d) q += (p[d] - center[d]) * cov * (p[d] - center[d]);
  return std::sqrt(cov * cov * cov) * std::exp(-0.5 * q) / (2 * std::sqrt(std::pow(2 * kPi, 2)));
}

double temperature_initial(const Mesh& m, const double* p) {
  return m.cuboid ? temperature_initial_cuboid(p, m.center, m.global_diameter)
                  : temperature_initial_shell(p, m.R0, m.R1);
}

TemperatureDofs temperature_dofs(const Mesh& m, int degree) {
  TemperatureDofs t;
  t.degree = degree;
  if (degree == 1) {
    t.n_dofs = m.n_vertices;
    t.dofs_per_cell = 8;
    t.cell_dofs = m.cell_q1;
    t.dof_vnode = m.vertex_vnode;
  } else if (degree == 2) {
    t.n_dofs = m.n_vnodes;
    t.dofs_per_cell = 27;
    t.cell_dofs = m.cell_q2;
    t.dof_vnode.resize(m.n_vnodes);
    for (int n = 0; n < m.n_vnodes; ++n) t.dof_vnode[n] = n;
  } else {
    throw std::invalid_argument("temperature degree must be 1 or 2");
  }
  return t;
}

Constraints temperature_constraints(const Mesh& m, int degree) {
  const TemperatureDofs td = temperature_dofs(m, degree);
  std::vector<int> vnode_dof(m.n_vnodes, -1);
  for (int d = 0; d < td.n_dofs; ++d) vnode_dof[td.dof_vnode[d]] = d;
  Builder b(td.n_dofs);
  const uint8_t dirichlet_bit = m.cuboid ? kBndZ0 : kBndInner;
  if (m.cuboid) add_periodic(m, b, [&](int n, int) { return vnode_dof[n]; }, 1);
  for (int d = 0; d < td.n_dofs; ++d) {
    const int n = td.dof_vnode[d];
    if (!(m.vnode_bnd[n] & dirichlet_bit) || b.is_constrained(d)) continue;
    b.add_line(d);
    b.inhom[d] = temperature_initial(m, &m.xyz[3 * size_t(n)]);
  }
  return b.close();
}

std::vector<int32_t> nse_cell_dofs_dealii(const Mesh& m) {
  std::vector<int32_t> out(size_t(m.n_cells) * kNseDofs);
  const int nu = m.n_u();
  for (int c = 0; c < m.n_cells; ++c)
    for (int i = 0; i < kNseDofs; ++i) {
      const SysDof s = system_dof(i);
      out[size_t(c) * kNseDofs + i] = s.comp < 3 ? 3 * m.cell_q2[27 * size_t(c) + s.lex] + s.comp
                                                 : nu + m.cell_q1[8 * size_t(c) + s.lex];
    }
  return out;
}

// deal.II's DoF order on the 6-cell hyper_shell (setup_dofs,
// boussinesq_model.tpp:197-206): GridGenerator::hyper_shell(n_cells = 6) of
// deal.II 9.2 (grid_generator.cc, not in this image; restated, unpinned) takes
// the 8 corners of [-1,1]^3 (x fastest) scaled to the inner radius as vertices
// 0-7 and to the outer radius as 8-15, and the cells
//   bottom {8,9,10,11,0,1,2,3}, right {9,11,1,3,13,15,5,7}, top {12,13,4,5,14,15,6,7},
//   left {8,0,10,2,12,4,14,6}, front {8,9,0,1,12,13,4,5}, back {10,2,11,3,14,6,15,7}.
// refine_global puts the 8 children of a cell (child index x + 2y + 4z in the
// parent's frame) consecutively on the next level in parent order, so the
// active cells of level r are each coarse cell's Morton order. distribute_dofs
// numbers a cell's unseen vertices, lines, faces, interior in that order
// (FE_Q(2)'s hierarchic order); component_wise({0,0,0,1}) then keeps the
// velocity dofs in that order (3 per node) and moves the pressure behind them.
std::vector<int32_t> dealii_shell_node_order(const Mesh& m, std::vector<int32_t>* cell_order) {
  if (m.cuboid) throw std::invalid_argument("deal.II order: the 6-cell shell only");
  static const int kCells[6][8] = {{8, 9, 10, 11, 0, 1, 2, 3},   {9, 11, 1, 3, 13, 15, 5, 7},
                                   {12, 13, 4, 5, 14, 15, 6, 7}, {8, 0, 10, 2, 12, 4, 14, 6},
                                   {8, 9, 0, 1, 12, 13, 4, 5},   {10, 2, 11, 3, 14, 6, 15, 7}};
  const int N = m.N, refine = m.refine, N3 = N * N * N;
  std::unordered_map<size_t, int32_t> key_node, key_cell;
  key_node.reserve(size_t(m.n_vnodes));
  key_cell.reserve(size_t(m.n_cells));
  for (int c = 0; c < m.n_cells; ++c) {
    for (int lex = 0; lex < 27; ++lex)
      key_node.emplace(shell_node_key(N, refine, c, lex), m.cell_q2[27 * size_t(c) + lex]);
    key_cell.emplace(shell_node_key(N, refine, c, 13), c);
  }
  const int64_t den = int64_t(2 * N) * (2 * N) * (2 * N);
  auto dealii_key = [&](int q, int X, int Y, int Z) {
    int64_t num[4] = {0, 0, 0, 0};
    for (int v = 0; v < 8; ++v) {
      const int64_t w = int64_t((v & 1) ? X : 2 * N - X) * ((v & 2) ? Y : 2 * N - Y) *
                        ((v & 4) ? Z : 2 * N - Z);
      const int gv = kCells[q][v], corner = gv % 8;
      num[0] += w * ((corner & 1) ? N : -N);
      num[1] += w * ((corner & 2) ? N : -N);
      num[2] += w * ((corner & 4) ? N : -N);
      num[3] += w * (gv >= 8 ? 2 * N : 0);
    }
    int P[3];
    for (int d = 0; d < 3; ++d) {
      if (num[d] % den) throw std::logic_error("deal.II order: off-lattice point");
      P[d] = int(num[d] / den);
    }
    if (num[3] % den) throw std::logic_error("deal.II order: off-lattice radius");
    return shell_key_of_point(N, P, int(num[3] / den));
  };
  std::vector<int32_t> order(size_t(m.n_vnodes), -1);
  if (cell_order) cell_order->assign(size_t(m.n_cells), -1);
  int32_t next = 0;
  for (int q = 0; q < 6; ++q)
    for (int code = 0; code < N3; ++code) {
      int i, j, k;
      demorton(uint32_t(code), refine, i, j, k);
      if (cell_order) {
        const auto it = key_cell.find(dealii_key(q, 2 * i + 1, 2 * j + 1, 2 * k + 1));
        if (it == key_cell.end()) throw std::logic_error("deal.II order: cell not found");
        (*cell_order)[size_t(q) * N3 + code] = it->second;
      }
      for (int h = 0; h < 27; ++h) {
        const int lex = kQ2HierToLex[h];
        const auto it = key_node.find(dealii_key(q, 2 * i + lex % 3, 2 * j + (lex / 3) % 3, 2 * k + lex / 9));
        if (it == key_node.end()) throw std::logic_error("deal.II order: node not found");
        if (order[it->second] < 0) order[it->second] = next++;
      }
    }
  if (next != m.n_vnodes) throw std::logic_error("deal.II order: nodes not covered");
  return order;
}

}  // namespace dcp
