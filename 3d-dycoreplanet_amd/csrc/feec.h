// Device interface of the FEEC variant (ExteriorCalculus::BoussinesqModel<3>,
// config 4): kernels in kernels/feec.hip, orchestration in api.cpp / solver.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "device.h"
#include "fe_tables.h"

namespace dcp {

// Local DoFs per cell: 12 Nedelec (w, edges) + 6 Raviart-Thomas (u, faces) +
// 1 DGQ0 (p), global NSE vector [w | u | p].
constexpr int kFeecDofs = 19;

struct FeecCellData {
  int n_cells;
  const int32_t* cell_dofs;   // [n][19] global dofs in [w | u | p]
  const int8_t* sign;         // [n][19] orientation signs (p: +1)
  const double* X;            // [n][8][3] vertices (MappingQ1)
  const double* diameter;     // [n]
  const uint8_t* fixed;       // [n_w + n_u + n_p] homogeneous boundary constraint
  const int32_t* cell_T;      // [n][8] temperature dofs
};

void launch_feec_system(const FeecCellData& cd, const int32_t* cells, int n, const int32_t* pos,
                        const double* old_nse, const double* T_old, const PhysicsDev& ph, double* A,
                        double* rhs, hipStream_t s);
void launch_feec_elements(const FeecCellData& cd, int first, int n, const double* old_nse,
                          const double* T_old, const PhysicsDev& ph, double* K, double* f,
                          hipStream_t s);
void launch_feec_precond(const FeecCellData& cd, const int32_t* cells, int n, const int32_t* pos,
                         const PhysicsDev& ph, double* P, hipStream_t s);
void launch_feec_T_rhs(const FeecCellData& cd, const int32_t* cells, int n, const double* T_old,
                       const double* nse, const PhysicsDev& ph, const uint8_t* T_fixed,
                       const double* T_bc, double* rhs, hipStream_t s);
void feec_velocity_stats(const FeecCellData& cd, int n_cells, const double* nse, double* out2,
                         hipStream_t s);
// npt = 1: QGauss(1) JxW (det J at the centre); 2: QGauss(2) JxW sum (the cell volume)
void feec_cell_weights(const FeecCellData& cd, int n_cells, double* w, hipStream_t s, int npt);
void feec_positions(const FeecCellData& cd, int n_cells, const int32_t* ptr, const int32_t* col,
                    int32_t* pos, hipStream_t s);

}  // namespace dcp
