// Host-side setup for the hot path: the refined mesh, the DoF numbering and the
// AffineConstraints of the NSE and temperature systems.
//
// This restates, without deal.II, what the reference builds once per run
// before the time loop:
//   PlanetGeometry ctor: hyper_shell(6 cells) / hyper_rectangle (planet_geometry.tpp:7-99)
//   refine_global (planet_geometry.tpp:109-120), GridTools::scale(1/L) (boussinesq_model.tpp:42-63)
//   setup_dofs: distribute_dofs + component_wise({0,0,0,1}) (boussinesq_model.tpp:194-206),
//               constraints (:259-387)
// Geometry: the shell's 6 coarse cells are hyper_shell's (corners
// (+-1,+-1,+-1) R/sqrt(3)); refinement places new vertices by
// SphericalManifold's rules (manifold.cpp): line midpoints by
// get_intermediate_point, quad / hex centres by get_new_point over the
// vertices and line / face midpoints with TriaAccessor::center(true, true)'s
// weights. Every cell carries the 64 support points of MappingQ(3)
// (boussinesq_model.tpp:20): spherical on cells with boundary lines, trilinear
// (MappingQ1) elsewhere unless mapping_q_on_all_cells (deal.II >= 9.3
// behaviour). Parity with deal.II itself is unpinned (not in this image);
// topology (panel frames, numbering) follows mesh.cpp's own convention.
#pragma once
#include <cstdint>
#include <vector>

#include "prm.h"

namespace dcp {

enum BoundaryBits : uint8_t {
  kBndInner = 1,  // shell r = R0 (boundary id 0)
  kBndOuter = 2,  // shell r = R1 (boundary id 1)
  kBndX0 = 4,     // cube faces (boundary ids 0..5 with colorize)
  kBndX1 = 8,
  kBndY0 = 16,
  kBndY1 = 32,
  kBndZ0 = 64,
  kBndZ1 = 128,
};

struct Mesh {
  bool cuboid = false;
  int refine = 0;
  int N = 1;  // cells per coarse-cell edge = 2^refine
  double R0 = 0, R1 = 0;
  double center[3] = {0, 0, 0};
  double global_diameter = 0;
  int n_cells = 0;
  int n_vnodes = 0;     // Q2 nodes (velocity support points = geometry nodes)
  int n_vertices = 0;   // Q1 nodes (pressure, Q1 temperature)
  // cell -> 27 vnode ids, lexicographic local order (a + 3b + 9c)
  std::vector<int32_t> cell_q2;
  // cell -> 8 vertex ids in deal.II vertex order (lexicographic)
  std::vector<int32_t> cell_q1;
  std::vector<double> xyz;              // [n_vnodes][3]
  std::vector<int32_t> vertex_vnode;    // vertex id -> vnode id
  std::vector<int32_t> vnode_vertex;    // vnode id -> vertex id or -1
  std::vector<uint8_t> vnode_bnd;       // BoundaryBits
  std::vector<double> cell_diameter;    // max vertex diagonal (CellAccessor::diameter)
  // MappingQ(3) support points per cell, [n_cells][64][3] lexicographic
  // (fe_tables.h kGL3); xyz above = their image of the Q2 support points.
  std::vector<double> cell_map;
  bool mapping_q_on_all_cells = false;
  std::vector<int32_t> cell_coarse;     // coarse cell (tree) of each cell

  int n_u() const { return 3 * n_vnodes; }
  int n_p() const { return n_vertices; }
};

// Builds the refined hyper shell (6 coarse cells) with radii already divided
// by the reference length. mapping_q_on_all_cells: false = deal.II 9.2's
// MappingQ (cubic map on boundary cells only, the version CMakeLists.txt:26
// pins), true = deal.II >= 9.3 (cubic map on every cell).
Mesh build_shell(int refine, double R0, double R1, bool mapping_q_on_all_cells = false);
// Builds the refined unit cube [0,1]^3 / L (hyper_rectangle, colorize).
Mesh build_cube(int refine, double length);
// Dispatch on Parameters (cuboid geometry flag, refinement, scaling by L).
Mesh build_mesh(const Parameters& prm);

// Closed AffineConstraints in CSR form over one DoF space.
struct Constraints {
  int n_dofs = 0;
  std::vector<int32_t> line_of;    // dof -> line or -1
  std::vector<int32_t> line_dof;   // constrained dof of each line
  std::vector<int32_t> entry_ptr;  // CSR over lines
  std::vector<int32_t> entry_dof;
  std::vector<double> entry_w;
  std::vector<double> inhomogeneity;
  int n_lines() const { return static_cast<int>(line_dof.size()); }
  bool constrained(int dof) const { return line_of[dof] >= 0; }
  bool inhomogeneous(int dof) const {
    return line_of[dof] >= 0 && inhomogeneity[line_of[dof]] != 0.0;
  }
};

// Normal used by the no-normal-flux constraint on the outer sphere.
//   Mapping (default): deal.II's compute_no_normal_flux_constraints rule, as
//     the reference calls it with its mapping (boussinesq_model.tpp:324-329) —
//     the unit normal of every adjacent mapped boundary face at the support
//     point (MappingQ(3) of the cell), summed over the faces and normalised.
//   Radial: the exact sphere normal at the support point.
//   Consistent: n_i = sum_cells int grad(phi_i) dx, minus the boundary row of
//     B^T 1 (Engelman, Sani & Gresho 1982). Under MappingQ(3) + QGauss(3) the
//     interior rows of B^T 1 no longer vanish (the quadrature is not exact for
//     a cubic map), so no choice of normals makes the constant pressure an
//     exact null vector of S; see DESIGN.md "no-normal-flux normals".
enum class NormalMode { Consistent, Radial, Mapping };
std::vector<double> consistent_normals(const Mesh& m, uint8_t boundary_bit);
std::vector<double> mapping_normals(const Mesh& m, uint8_t boundary_bit);

// deal.II geometry rules (manifold.cpp), centre = `center`:
// SphericalManifold::get_intermediate_point(p1, p2, w)
void spherical_intermediate(const double* center, const double* p1, const double* p2, double w,
                            double* out);
// SphericalManifold::get_new_points(src[n_src], weights[n_rows][n_src]) -> out[n_rows]
void spherical_new_points(const double* center, int n_src, const double* src, int n_rows,
                          const double* weights, double* out);
// MappingQGeneric(3)::compute_mapping_support_points from the 8 vertices
// (lexicographic): spherical (SphericalManifold, centre 0) or flat (trilinear).
void mapping_support_points(const double* vertices, bool spherical, double* X /*[64][3]*/);
// x(xi) and J = dx/dxi of the cubic map with support points X.
void mapping_eval(const double* X, const double* xi, double* x, double J[3][3]);

// NSE constraints (boussinesq_model.tpp:259-333): shell -> no-slip on the
// inner sphere, no-normal-flux on the outer sphere; cube -> periodic x/y,
// no-slip z=0, no-normal-flux z=1. DoF space: [3*n_vnodes velocity | n_p pressure].
Constraints nse_constraints(const Mesh& m, NormalMode mode = NormalMode::Mapping);

// Temperature constraints (:338-387): Dirichlet with the initial temperature on
// the inner sphere (shell) or on z=0 (cube, + periodic x/y). degree 1 or 2.
Constraints temperature_constraints(const Mesh& m, int degree);

// Initial temperature functions (boussinesq_model_data.tpp:61-147, :168-196).
double temperature_initial_shell(const double* p, double R0, double R1);
double temperature_initial_cuboid(const double* p, const double* center, double diameter);
double temperature_initial(const Mesh& m, const double* p);

// Temperature DoF numbering for degree 1 (= vertices) or 2 (= vnodes).
struct TemperatureDofs {
  int degree = 1;
  int n_dofs = 0;
  int dofs_per_cell = 8;
  std::vector<int32_t> cell_dofs;    // [n_cells][dofs_per_cell], lexicographic local order
  std::vector<int32_t> dof_vnode;    // support point of each dof (vnode id)
};
TemperatureDofs temperature_dofs(const Mesh& m, int degree);

// FEEC DoF topology (feec_mesh.cpp): lowest-order Nedelec (w, edges),
// Raviart-Thomas (u, faces), DGQ0 (p, cells); local order = deal.II line /
// face order. Signs orient each cell's local functions to the global DoFs.
struct FeecDofs {
  int n_w = 0, n_u = 0, n_p = 0;
  std::vector<int32_t> cell_w;         // [n_cells][12] edge ids
  std::vector<int8_t> sign_w;          // [n_cells][12]
  std::vector<int32_t> cell_u;         // [n_cells][6] face ids
  std::vector<int8_t> sign_u;          // [n_cells][6]
  std::vector<uint8_t> w_boundary;     // [n_w] edge on the domain boundary
  std::vector<uint8_t> u_boundary;     // [n_u] face on the domain boundary
  std::vector<double> cell_vertices;   // [n_cells][8][3] (MappingQ1 geometry)
};
FeecDofs feec_dofs(const Mesh& m);
extern const int kFeecLineVertex[12][2];
extern const int kFeecFaceVertex[6][4];

// FESystem-ordered (deal.II local order, 89 per cell) global NSE dof indices,
// i.e. what cell->get_dof_indices() returns in the reference.
std::vector<int32_t> nse_cell_dofs_dealii(const Mesh& m);

// New number of every velocity node in deal.II's distribute_dofs order on the
// 6-cell hyper_shell (see mesh.cpp); cell_order (optional): the mesh cell of
// each deal.II active cell, in deal.II's order.
std::vector<int32_t> dealii_shell_node_order(const Mesh& m, std::vector<int32_t>* cell_order);

}  // namespace dcp
