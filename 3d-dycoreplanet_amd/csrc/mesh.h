// Host-side setup for the hot path: the refined mesh, the DoF numbering and the
// AffineConstraints of the NSE and temperature systems.
//
// This restates, without deal.II, what the reference builds once per run
// before the time loop:
//   PlanetGeometry ctor: hyper_shell(6 cells) / hyper_rectangle (planet_geometry.tpp:7-99)
//   refine_global (planet_geometry.tpp:109-120), GridTools::scale(1/L) (boussinesq_model.tpp:42-63)
//   setup_dofs: distribute_dofs + component_wise({0,0,0,1}) (boussinesq_model.tpp:194-206),
//               constraints (:259-387)
// Geometry convention (documented deviation, parity vs deal.II unpinned): the
// shell's coarse cells are the 6 panels of an equiangular cube-sphere with the
// radius linear in the third reference coordinate; every refined cell carries
// a Q2 isoparametric geometry whose 27 nodes are exactly the Q2 velocity
// support points (nodes on the inner/outer boundary lie on the spheres).
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
  std::vector<int32_t> cell_coarse;     // coarse cell (tree) of each cell

  int n_u() const { return 3 * n_vnodes; }
  int n_p() const { return n_vertices; }
};

// Builds the refined hyper shell (6 coarse cells) with radii already divided
// by the reference length.
Mesh build_shell(int refine, double R0, double R1);
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
//   Consistent: n_i = sum_cells int grad(phi_i) dx (discretely consistent with
//     the divergence block, so B^T 1 lies in the constrained space and the
//     Schur complement's constant-pressure mode is exactly singular and never
//     excited). Default; see DESIGN.md "no-normal-flux normals".
//   Radial: the exact sphere normal at the support point (closest to deal.II's
//     mapping normal); leaves S with a near-null eigenvalue ~ h^5.6 that the
//     reference's identity-preconditioned Schur GMRES cannot resolve for r >= 3.
enum class NormalMode { Consistent, Radial };
std::vector<double> consistent_normals(const Mesh& m, uint8_t boundary_bit);

// NSE constraints (boussinesq_model.tpp:259-333): shell -> no-slip on the
// inner sphere, no-normal-flux on the outer sphere; cube -> periodic x/y,
// no-slip z=0, no-normal-flux z=1. DoF space: [3*n_vnodes velocity | n_p pressure].
Constraints nse_constraints(const Mesh& m, NormalMode mode = NormalMode::Consistent);

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

}  // namespace dcp
