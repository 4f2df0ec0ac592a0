// DoFRenumbering::Cuthill_McKee followed by component_wise on the NSE dofs, the
// numbering setup_dofs() gives when the Schur-complement solver is selected
// (boussinesq_model.tpp:198-204). ILU(0) of the velocity block (the A^-1 and
// S^-1 preconditioners of that solver) depends on the order: at the refine-3
// cube the factor's dependency chain falls from 5,937 levels in the mesh's
// first-encounter numbering to 1,698, which is what the device's level-by-level
// factorisation and triangular solves walk.
//
// deal.II's SparsityTools::reorder_Cuthill_McKee on the cell-coupling pattern
// without constraints: start at the first dof of least coordination (row
// length); each round numbers the not-yet-numbered neighbours of the previous
// round in order of (coordination, index); an empty round with dofs left
// restarts at the least-coordinated unnumbered dof. All dofs at one support
// point couple alike (same row length, same neighbours) and deal.II's initial
// numbering keeps them consecutive, so the rounds are run on support points
// (velocity nodes, with the pressure dof of the vertex nodes riding along) in
// node-id order; component_wise then lays the velocity block out as 3 n + c and
// the pressure block in the order of the nodes' new numbers.
#include <algorithm>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "mesh.h"
#include "mesh2d.h"
#include "renumber.h"

namespace dcp {
namespace {

// The FESystem(FE_Q(2)^dim, FE_Q(1)) cell layout: dofs per cell, support
// points per cell (hierarchic), vertices, velocity components; local index of
// the x velocity dof at support point t (dim + 1 dofs per vertex, dim per
// other point) and of the pressure dof at vertex v.
struct Layout {
  int dpc, npc, nv, dim;
  int vel_x(int t) const { return t < nv ? (dim + 1) * t : (dim + 1) * nv + dim * (t - nv); }
  int p_local(int v) const { return (dim + 1) * v + dim; }
};
constexpr Layout kLayout3D{89, 27, 8, 3};
constexpr Layout kLayout2D{kNseDofs2D, 9, 4, 2};

std::vector<int32_t> cm_nodes(const Layout& L, int n_cells, const int32_t* cell_nse, int n_vnodes) {
  const int P = L.npc;
  std::vector<int32_t> cn(size_t(n_cells) * P);
  std::vector<uint8_t> has_p(n_vnodes, 0);
  for (int c = 0; c < n_cells; ++c)
    for (int t = 0; t < P; ++t) {
      const int n = cell_nse[size_t(c) * L.dpc + L.vel_x(t)] / L.dim;
      if (n < 0 || n >= n_vnodes) throw std::invalid_argument("cuthill_mckee: velocity dof out of range");
      cn[size_t(c) * P + t] = n;
      if (t < L.nv) has_p[n] = 1;
    }
  // node -> cells
  std::vector<int32_t> nptr(n_vnodes + 1, 0), ncell(cn.size());
  for (int32_t n : cn) ++nptr[n + 1];
  std::partial_sum(nptr.begin(), nptr.end(), nptr.begin());
  {
    std::vector<int32_t> fill(nptr.begin(), nptr.end() - 1);
    for (int c = 0; c < n_cells; ++c)
      for (int t = 0; t < P; ++t) ncell[fill[cn[size_t(c) * P + t]]++] = c;
  }
  std::vector<int32_t> stamp(n_vnodes, -1);
  auto neighbours = [&](int n, std::vector<int32_t>& out) {
    for (int k = nptr[n]; k < nptr[n + 1]; ++k)
      for (int t = 0; t < P; ++t) {
        const int m = cn[size_t(ncell[k]) * P + t];
        if (stamp[m] != n) {
          stamp[m] = n;
          out.push_back(m);
        }
      }
  };
  // coordination of every dof at node n = its row length
  std::vector<int64_t> coord(n_vnodes, 0);
  {
    std::vector<int32_t> nb;
    for (int n = 0; n < n_vnodes; ++n) {
      nb.clear();
      neighbours(n, nb);
      for (int m : nb) coord[n] += L.dim + has_p[m];
    }
  }
  std::fill(stamp.begin(), stamp.end(), -1);
  std::vector<int32_t> nw(n_vnodes, -1);
  int next = 0;
  auto start = [&] {
    int best = -1;
    for (int n = 0; n < n_vnodes; ++n)
      if (nw[n] < 0 && (best < 0 || coord[n] < coord[best])) best = n;
    return best;
  };
  std::vector<int32_t> last, round;
  if (n_vnodes > 0) {
    last.push_back(start());
    nw[last[0]] = next++;
  }
  while (next < n_vnodes) {
    round.clear();
    for (int n : last) neighbours(n, round);
    round.erase(std::remove_if(round.begin(), round.end(), [&](int m) { return nw[m] >= 0; }),
                round.end());
    std::sort(round.begin(), round.end());
    round.erase(std::unique(round.begin(), round.end()), round.end());
    if (round.empty()) round.push_back(start());
    std::stable_sort(round.begin(), round.end(),
                     [&](int a, int b) { return coord[a] < coord[b]; });
    for (int m : round) nw[m] = next++;
    last.swap(round);
  }
  return nw;
}

std::vector<int32_t> dof_map(const Layout& L, int n_cells, const int32_t* cell_nse, int n_vnodes,
                             int n_p, const std::vector<int32_t>& node_new) {
  const int D = L.dim;
  const int n_u = D * n_vnodes;
  std::vector<int32_t> map(size_t(n_u) + n_p, -1);
  for (int n = 0; n < n_vnodes; ++n)
    for (int c = 0; c < D; ++c) map[D * size_t(n) + c] = D * node_new[n] + c;
  // pressure dofs in the order of their vertex node's new number
  std::vector<int32_t> pnode(n_p, -1);
  for (int c = 0; c < n_cells; ++c)
    for (int v = 0; v < L.nv; ++v) {
      const int p = cell_nse[size_t(c) * L.dpc + L.p_local(v)] - n_u;
      if (p < 0 || p >= n_p) throw std::invalid_argument("cuthill_mckee: pressure dof out of range");
      pnode[p] = cell_nse[size_t(c) * L.dpc + L.vel_x(v)] / D;
    }
  std::vector<int32_t> order(n_p);
  std::iota(order.begin(), order.end(), 0);
  for (int p = 0; p < n_p; ++p)
    if (pnode[p] < 0) throw std::invalid_argument("cuthill_mckee: pressure dof on no cell");
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return node_new[pnode[a]] < node_new[pnode[b]]; });
  for (int k = 0; k < n_p; ++k) map[size_t(n_u) + order[k]] = n_u + k;
  return map;
}

}  // namespace

std::vector<int32_t> cuthill_mckee_nodes(int n_cells, const int32_t* cell_nse, int n_vnodes) {
  return cm_nodes(kLayout3D, n_cells, cell_nse, n_vnodes);
}

std::vector<int32_t> nse_dof_map(int n_cells, const int32_t* cell_nse, int n_vnodes, int n_p,
                                 const std::vector<int32_t>& node_new) {
  return dof_map(kLayout3D, n_cells, cell_nse, n_vnodes, n_p, node_new);
}

std::vector<int32_t> cuthill_mckee_map_2d(const Mesh2D& m, const std::vector<int32_t>& cell_nse) {
  const std::vector<int32_t> nw = cm_nodes(kLayout2D, m.n_cells, cell_nse.data(), m.n_vnodes);
  return dof_map(kLayout2D, m.n_cells, cell_nse.data(), m.n_vnodes, m.n_p(), nw);
}

Constraints renumber_constraints(const Constraints& in, const std::vector<int32_t>& map) {
  Constraints out;
  out.n_dofs = in.n_dofs;
  out.line_of.assign(in.line_of.size(), -1);
  const int nl = in.n_lines();
  std::vector<int32_t> lines(nl);
  std::iota(lines.begin(), lines.end(), 0);
  std::sort(lines.begin(), lines.end(),
            [&](int a, int b) { return map[in.line_dof[a]] < map[in.line_dof[b]]; });
  out.entry_ptr.push_back(0);
  std::vector<int32_t> e;
  for (int l : lines) {
    out.line_of[map[in.line_dof[l]]] = out.n_lines();
    out.line_dof.push_back(map[in.line_dof[l]]);
    out.inhomogeneity.push_back(in.inhomogeneity[l]);
    e.resize(in.entry_ptr[l + 1] - in.entry_ptr[l]);
    std::iota(e.begin(), e.end(), in.entry_ptr[l]);
    std::stable_sort(e.begin(), e.end(),
                     [&](int a, int b) { return map[in.entry_dof[a]] < map[in.entry_dof[b]]; });
    for (int k : e) {
      out.entry_dof.push_back(map[in.entry_dof[k]]);
      out.entry_w.push_back(in.entry_w[k]);
    }
    out.entry_ptr.push_back(int32_t(out.entry_dof.size()));
  }
  return out;
}

}  // namespace dcp
