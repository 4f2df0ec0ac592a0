// Cell partition + ghost layers + halo plans for the multi-GPU path.
//
// The reference distributes the mesh with parallel::distributed::Triangulation
// (p4est; planet_geometry.h:67): every rank owns a contiguous range of cells
// in tree (Morton) order, DoFs on partition interfaces belong to one of the
// touching ranks, and each rank keeps ghost cells plus ghost DoF values
// (locally_relevant_dofs, boussinesq_model.tpp:237-252) refreshed by
// Trilinos Import before every operator apply. This file restates that on the
// host, without deal.II, for a rank of a P-way split of the global mesh:
//
//   owned cells   [rank*n/P, (rank+1)*n/P)          (p4est's equal split)
//   DoF owner     rank of the lowest-index cell touching the DoF
//   ghost cells   two vertex-neighbour layers around the owned cells: layer 1
//                 makes every owned matrix row complete (owner computes, no
//                 reverse halo, unlike compress(add) at :736-737); layer 2
//                 makes the B^T rows and Jacobi diagonals of layer-1 nodes
//                 complete, so S = B D_A^-1 B^T is formed for owned rows
//                 without communication.
//
// Local numbering, per field (velocity support points, pressure, temperature):
// owned entities first (ascending global id), then ghosts (ascending global
// id). The local NSE vector is [u_own u_ghost | p_own p_ghost] with velocity
// dof 3*node + c, i.e. a standalone mesh to the rest of the library.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/dcp.h"

namespace dcp {

// Forward halo of one field: entity values (width doubles each) go from the
// owner to every rank that holds the entity as a ghost.
struct HaloPlan {
  int width = 1;
  std::vector<int> peers;                    // ranks exchanged with (ascending)
  std::vector<int32_t> send_ptr, send_idx;   // per peer: local indices of owned entities
  std::vector<int32_t> recv_ptr, recv_idx;   // per peer: local indices of ghost entities
  std::vector<int64_t> send_gid, recv_gid;   // global ids of the same (host checks / tests)
};

struct LocalMesh {
  int rank = 0, world = 1;
  int n_cells = 0, n_owned_cells = 0;
  int nvo = 0, nvg = 0, npo = 0, npg = 0, nTo = 0, nTg = 0;
  std::vector<int32_t> cells_g;              // local cell -> global cell
  std::vector<int32_t> cell_nse_dofs;        // [n_cells][89], local numbering
  std::vector<int32_t> cell_T_dofs;          // [n_cells][8 or 27] (FE_Q(1) / FE_Q(2))
  std::vector<double> geometry;              // [n_cells][64][3] (MappingQ(3) support points)
  std::vector<double> diameter;              // [n_cells]
  std::vector<int32_t> vnode_g, p_g, T_g;    // local -> global id per field
  // local constraints (CSR lines as dcp_constraints expects)
  std::vector<int> nse_line, nse_ptr, nse_edof, T_line, T_ptr, T_edof;
  std::vector<double> nse_w, nse_inh, T_w, T_inh;
  HaloPlan hv, hp, hT;                       // velocity nodes (width 3), pressure, temperature

  int n_u() const { return 3 * (nvo + nvg); }
  int n_p() const { return npo + npg; }
  int n_T() const { return nTo + nTg; }
  dcp_constraints nse_view() const;
  dcp_constraints T_view() const;
};

// FEEC variant (config 4): the same split and two ghost layers; fields w
// (edges), u (faces), p (cells: DGQ0), T (Q1 vertices), each numbered owned
// first then ghosts. The local NSE vector is [w_l | u_l | p_l].
struct FeecLocal {
  int rank = 0, world = 1;
  int n_cells = 0, n_owned_cells = 0;
  int nwo = 0, nwg = 0, nuo = 0, nug = 0, nTo = 0, nTg = 0;
  std::vector<int32_t> cells_g, w_g, u_g, T_g;  // local -> global (p_g = cells_g)
  std::vector<int32_t> cell_w, cell_u, cell_T;  // local ids
  std::vector<int8_t> sign_w, sign_u;
  std::vector<double> vertices, diameter;
  std::vector<uint8_t> w_fixed, u_fixed;
  std::vector<int> T_line, T_ptr, T_edof;
  std::vector<double> T_w, T_inh;
  HaloPlan hw, hu, hp, hT;
  int n_w() const { return nwo + nwg; }
  int n_u() const { return nuo + nug; }
  int n_T() const { return nTo + nTg; }
  dcp_feec_mesh view() const;  // points into this object
};
FeecLocal localize_feec(const dcp_feec_mesh& m, int rank, int world);

// The 2D model (Standard::BoussinesqModel<2>): the same split and two ghost
// layers (cells sharing a vertex = a pressure dof); fields u (scalar velocity
// dofs), p, T, each numbered owned first then ghosts, ascending global id.
// The local NSE vector is [u_l | p_l].
struct Local2D {
  int rank = 0, world = 1, tdpc = 4;
  int n_cells = 0, n_owned_cells = 0;
  int nuo = 0, nug = 0, npo = 0, npg = 0, nTo = 0, nTg = 0;
  std::vector<int32_t> cells_g, u_g, p_g, T_g;  // local -> global id per field
  std::vector<int32_t> cell_dofs, cell_T;       // [n][22] (u local, n_u_l + p local), [n][tdpc]
  std::vector<double> geometry, diameter;       // [n][16][2], [n]
  std::vector<int> nse_line, nse_ptr, nse_edof, T_line, T_ptr, T_edof;
  std::vector<double> nse_w, nse_inh, T_w, T_inh;
  HaloPlan hu, hp, hT;
  int n_u() const { return nuo + nug; }
  int n_p() const { return npo + npg; }
  int n_T() const { return nTo + nTg; }
  dcp_mesh2d view() const;  // points into this object
};
Local2D localize_2d(const dcp_mesh2d& m, int rank, int world);

// Builds rank `rank`'s local mesh of a `world`-way split of the global mesh
// (arguments as dcp_mesh_upload). Throws std::runtime_error on bad input.
LocalMesh localize(int n_cells, const int32_t* cell_nse_dofs, const int32_t* cell_T_dofs,
                   const double* cell_geometry, const double* cell_diameter, int n_u, int n_p,
                   int n_T, const dcp_constraints* nse_c, const dcp_constraints* T_c, int rank,
                   int world);

// Rank hc.rank's local mesh from what that rank holds in a distributed run
// (dcp_mesh_upload_distributed; distributed.cpp): the caller's ownership, the
// second ghost layer fetched from the ghost cells' owners through hc.
LocalMesh localize_distributed(const dcp_dist_mesh& m, const dcp_host_comm& hc);

}  // namespace dcp
