// FEEC DoF topology (ExteriorCalculus::BoussinesqModel<3>, config 4):
// lowest-order Nedelec on edges (vorticity w), Raviart-Thomas on faces
// (velocity u), DGQ0 on cells (pressure p), boussineq_model_FEEC.tpp:21-30.
//
// Orientation (documented convention; parity with deal.II unpinned):
//   edge: global direction from the lower to the higher global vertex id; a
//         cell's local edge function points along the local +axis (deal.II
//         line vertex order), sign = +1 if that matches the global direction;
//   face: global DoF = flux through the face in the outward direction of the
//         first cell (tree order) that has the face; a cell's local function
//         carries unit flux along its local +axis, sign accordingly.
// With these signs the assembled spaces are H(curl)/H(div) conforming, which
// is what the reference's RT face-sign fix (utilities.cc:20-45) restores.
//
// Cuboid (periodic in x and y, FEEC.tpp:313-333): edges and faces are keyed by
// the lattice position of their midpoint reduced modulo the box in x and y, so
// an edge or face on x = 1 (y = 1) IS its partner on x = 0 (y = 0). That is
// make_periodicity_constraints with unit weights in condensed form: the
// partner's row holds both sides' cell contributions and the image has no row
// of its own. Edges point along +axis (the cells are lattice aligned); only
// the z faces (boundary ids 4, 5) stay boundary faces.
#include <algorithm>
#include <cmath>
#include <stdexcept>
#include <unordered_map>

#include "mesh.h"

namespace dcp {

const int kFeecLineVertex[12][2] = {{0, 2}, {1, 3}, {0, 1}, {2, 3}, {4, 6}, {5, 7},
                                    {4, 5}, {6, 7}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
const int kFeecFaceVertex[6][4] = {{0, 2, 4, 6}, {1, 3, 5, 7}, {0, 1, 4, 5},
                                   {2, 3, 6, 7}, {0, 1, 2, 3}, {4, 5, 6, 7}};

FeecDofs feec_dofs(const Mesh& m) {
  if (m.cuboid && m.N < 2)
    throw std::runtime_error("feec_dofs: the periodic cuboid needs two cells per periodic direction");
  FeecDofs f;
  const int nc = m.n_cells;
  f.cell_w.assign(size_t(nc) * 12, -1);
  f.sign_w.assign(size_t(nc) * 12, 0);
  f.cell_u.assign(size_t(nc) * 6, -1);
  f.sign_u.assign(size_t(nc) * 6, 0);
  f.cell_vertices.assign(size_t(nc) * 24, 0.0);
  std::unordered_map<uint64_t, int32_t> edge_id, face_id;
  edge_id.reserve(size_t(nc) * 4);
  face_id.reserve(size_t(nc) * 4);
  std::vector<int32_t> face_cells;  // number of cells per face
  const uint64_t NV = uint64_t(m.n_vertices);
  // cuboid: lattice position (xyz = lattice / (2N L), global_diameter = sqrt(3)/L)
  const long full = 2L * m.N, L2 = full + 1;
  const double lat = 2.0 * m.N * std::sqrt(3.0) / (m.cuboid ? m.global_diameter : 1.0);
  auto lattice = [&](int vert, int d) {
    return std::lround(m.xyz[3 * size_t(m.vertex_vnode[vert]) + d] * lat);
  };
  // key of the point (sum of k vertices' lattice positions) / k, periodic in x, y
  auto periodic_key = [&](const int* vs, int k) {
    long p[3];
    for (int d = 0; d < 3; ++d) {
      long s = 0;
      for (int i = 0; i < k; ++i) s += lattice(vs[i], d);
      p[d] = s / k;
      if (d < 2) p[d] %= full;
    }
    return uint64_t((p[2] * L2 + p[1]) * L2 + p[0]);
  };
  for (int c = 0; c < nc; ++c) {
    const int32_t* v = &m.cell_q1[8 * size_t(c)];
    for (int k = 0; k < 8; ++k)
      for (int d = 0; d < 3; ++d)
        f.cell_vertices[24 * size_t(c) + 3 * k + d] = m.xyz[3 * size_t(m.vertex_vnode[v[k]]) + d];
    for (int l = 0; l < 12; ++l) {
      const int a = v[kFeecLineVertex[l][0]], b = v[kFeecLineVertex[l][1]];
      const int ab[2] = {a, b};
      const uint64_t key = m.cuboid ? periodic_key(ab, 2)
                                    : uint64_t(std::min(a, b)) * NV + uint64_t(std::max(a, b));
      auto it = edge_id.find(key);
      int32_t id;
      if (it == edge_id.end()) {
        id = int32_t(edge_id.size());
        edge_id.emplace(key, id);
      } else {
        id = it->second;
      }
      f.cell_w[12 * size_t(c) + l] = id;
      if (m.cuboid) {
        long step = 0;
        for (int d = 0; d < 3; ++d) step += lattice(b, d) - lattice(a, d);
        f.sign_w[12 * size_t(c) + l] = step > 0 ? 1 : -1;
      } else {
        f.sign_w[12 * size_t(c) + l] = a < b ? 1 : -1;
      }
    }
    for (int q = 0; q < 6; ++q) {
      // key: the smallest vertex and the vertex diagonally opposite to it
      int lo = 0;
      for (int k = 1; k < 4; ++k)
        if (v[kFeecFaceVertex[q][k]] < v[kFeecFaceVertex[q][lo]]) lo = k;
      const int opp = v[kFeecFaceVertex[q][3 - lo]];
      int fv[4];
      for (int k = 0; k < 4; ++k) fv[k] = v[kFeecFaceVertex[q][k]];
      const uint64_t key = m.cuboid ? periodic_key(fv, 4)
                                    : uint64_t(v[kFeecFaceVertex[q][lo]]) * NV + uint64_t(opp);
      auto it = face_id.find(key);
      const int s_out = (q % 2 == 1) ? 1 : -1;  // local +axis is outward on the max side
      int32_t id;
      if (it == face_id.end()) {
        id = int32_t(face_id.size());
        face_id.emplace(key, id);
        face_cells.push_back(1);
        f.sign_u[6 * size_t(c) + q] = int8_t(s_out);   // first cell: its outward normal
      } else {
        id = it->second;
        face_cells[id]++;
        f.sign_u[6 * size_t(c) + q] = int8_t(-s_out);  // the other cell sees it inward
      }
      f.cell_u[6 * size_t(c) + q] = id;
    }
  }
  f.n_w = int(edge_id.size());
  f.n_u = int(face_id.size());
  f.n_p = nc;
  f.u_boundary.assign(f.n_u, 0);
  f.w_boundary.assign(f.n_w, 0);
  for (int u = 0; u < f.n_u; ++u) {
    if (face_cells[u] > 2) throw std::runtime_error("feec_dofs: face shared by more than 2 cells");
    f.u_boundary[u] = face_cells[u] == 1;
  }
  // edges of boundary faces are boundary edges
  static const int kFaceLines[6][4] = {{0, 4, 8, 10}, {1, 5, 9, 11}, {2, 6, 8, 9},
                                       {3, 7, 10, 11}, {0, 1, 2, 3}, {4, 5, 6, 7}};
  for (int c = 0; c < nc; ++c)
    for (int q = 0; q < 6; ++q)
      if (f.u_boundary[f.cell_u[6 * size_t(c) + q]])
        for (int k = 0; k < 4; ++k) f.w_boundary[f.cell_w[12 * size_t(c) + kFaceLines[q][k]]] = 1;
  return f;
}

}  // namespace dcp
