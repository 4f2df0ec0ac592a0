// Host-side setup of the two-dimensional model, Standard::BoussinesqModel<2>
// (boussinesq_model.inst.cc:8; data/aqua_planet_test_2d.prm, BASELINE config
// C1): what PlanetGeometry<2> and setup_dofs() build once per run.
//
//   hyper_shell(center 0, R0, R1, 12 cells, colorize) (planet_geometry.tpp:63-68):
//     vertex i = R1 (cos 2 pi i/12, sin 2 pi i/12), vertex 12 + i = R0 (same
//     direction); cell i = {i, i+1, 12+i, 12+i+1 (mod 12)}; boundary id 0 on
//     the inner circle, 1 on the outer one; SphericalManifold on all objects.
//   refine_global: every cell splits into its 4 children in lexicographic
//     child order; line midpoints by SphericalManifold::get_intermediate_point,
//     cell centres by get_new_point over the 4 vertices (weight -1/4) and the 4
//     line midpoints (+1/2), TriaAccessor::center(true, true) (manifold.cpp,
//     the 2D points embedded in the z = 0 plane).
//   MappingQ(3) (boussinesq_model.tpp:20): 16 support points per cell (Gauss-
//     Lobatto 4 x 4, lexicographic), spherical on cells with boundary lines,
//     bilinear (MappingQ1) elsewhere as deal.II 9.2 does (or everywhere, >= 9.3).
//   distribute_dofs(FESystem(FE_Q(2)^2, FE_Q(1))) + component_wise({0,0,1}):
//     support points numbered in first-encounter order over the cells, each
//     cell's objects in deal.II order (vertices 0-3, lines 0-3, interior);
//     velocity dof 2 node + c, pressure n_u + vertex number; the temperature
//     FE_Q(2) handler numbers the same support points the same way.
//   constraints (boussinesq_model.tpp:308-330, 356-380): no-slip on the inner
//     circle, no-normal-flux (normals of the mapped faces, averaged at shared
//     points) on the outer one; temperature Dirichlet on the inner circle with
//     TemperatureInitialValues<2> at the MappingQ1 support points
//     (interpolate_boundary_values without a mapping argument).
// Parity with deal.II itself is unpinned (deal.II is not in this image).
#pragma once
#include <cstdint>
#include <vector>

#include "fe_tables.h"
#include "mesh.h"

namespace dcp {

// FE_Q(2) hierarchic local index -> lexicographic (a + 3 b) support point:
// vertices (0,0) (1,0) (0,1) (1,1), lines x=0, x=1, y=0, y=1, interior
constexpr int kQ2HierToLex2D[9] = {0, 2, 6, 8, 3, 5, 1, 7, 4};
constexpr int kQ1VertexToQ2Lex2D[4] = {0, 2, 6, 8};
// FESystem(FE_Q(2)^2, FE_Q(1)) in 2D: 22 dofs per cell
constexpr int kNseDofs2D = 22;
constexpr int kMapPts2D = 16;
// local dof i -> (component 0,1 velocity / 2 pressure, lexicographic point
// (velocity) or vertex (pressure))
inline SysDof system_dof_2d(int i) {
  if (i < 12) return SysDof{i % 3, i % 3 == 2 ? i / 3 : kQ2HierToLex2D[i / 3]};
  if (i < 20) return SysDof{(i - 12) % 2, kQ2HierToLex2D[4 + (i - 12) / 2]};
  return SysDof{i - 20, 4};
}

struct Mesh2D {
  int refine = 0;
  double R0 = 0, R1 = 0;
  int n_cells = 0, n_vnodes = 0, n_vertices = 0;
  std::vector<int32_t> cell_q2;        // [n_cells][9] node ids, lexicographic
  std::vector<int32_t> cell_q1;        // [n_cells][4] vertex ids (lexicographic = deal.II order)
  std::vector<double> xy;              // [n_vnodes][2] MappingQ(3) image of the support points
  std::vector<double> xy_q1;           // [n_vnodes][2] MappingQ1 image (boundary values)
  std::vector<int32_t> vertex_vnode;   // vertex -> node
  std::vector<int32_t> vnode_vertex;   // node -> vertex or -1
  std::vector<uint8_t> vnode_bnd;      // kBndInner / kBndOuter
  std::vector<double> cell_diameter;   // CellAccessor::diameter (longest vertex diagonal)
  std::vector<double> cell_map;        // [n_cells][16][2] MappingQ(3) support points
  int n_u() const { return 2 * n_vnodes; }
  int n_p() const { return n_vertices; }
};

Mesh2D build_shell_2d(int refine, double R0, double R1, bool mapping_q_on_all_cells);
// cell dofs in FESystem local order, as cell->get_dof_indices() returns them
std::vector<int32_t> nse_cell_dofs_2d(const Mesh2D& m);
// temperature FE_Q(2) cell dofs in its local (hierarchic) order
std::vector<int32_t> temperature_cell_dofs_2d(const Mesh2D& m);
Constraints nse_constraints_2d(const Mesh2D& m);
Constraints temperature_constraints_2d(const Mesh2D& m);
// TemperatureInitialValues<2> (boussinesq_model_data.tpp:12-48, 120-141)
double temperature_initial_2d(const double* p, double R0, double R1);
// 2D MappingQ(3) map x(xi) and Jacobian J[i][e] = dx_i / dxi_e from 16 support points
void mapping_eval_2d(const double* X, const double* xi, double* x, double J[2][2]);
// DoFRenumbering::Cuthill_McKee + component_wise of the 2D NSE dofs:
// old -> new dof map (renumber.cpp's rule on the 2D cell layout)
std::vector<int32_t> cuthill_mckee_map_2d(const Mesh2D& m, const std::vector<int32_t>& cell_nse);

}  // namespace dcp
