// Cuthill-McKee renumbering of the NSE dofs (boussinesq_model.tpp:198-204),
// see renumber.cpp.
#pragma once

#include <cstdint>
#include <vector>

#include "mesh.h"

namespace dcp {

// New number of every velocity node (support point) in the Cuthill-McKee
// order of the unconstrained cell-coupling pattern; cell_nse: [n_cells][89].
std::vector<int32_t> cuthill_mckee_nodes(int n_cells, const int32_t* cell_nse, int n_vnodes);

// Old -> new NSE dof map for a node order, component_wise: velocity 3 n + c,
// pressure in the order of the new numbers of the vertex nodes carrying it.
std::vector<int32_t> nse_dof_map(int n_cells, const int32_t* cell_nse, int n_vnodes, int n_p,
                                 const std::vector<int32_t>& node_new);

// The same constraints over the renumbered dofs (lines and entries in the
// new dof order, as AffineConstraints::close() keeps them).
Constraints renumber_constraints(const Constraints& in, const std::vector<int32_t>& map);

}  // namespace dcp
