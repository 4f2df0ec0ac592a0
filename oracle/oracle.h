/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference hot path (konsim83/3D-DyCorePlanet,
 * include/core/boussinesq_model.tpp, include/linear_algebra) used as
 * the checker for the HIP implementation. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product library
 * (3d-dycoreplanet_amd) never links or calls it.
 *
 * Parity status: UNPINNED against deal.II. The reference ships no golden
 * vectors (its only test prints a string, test/test_dummy.cc:19-41) and its
 * dependencies (deal.II >= 9.2, Trilinos, p4est) are absent from this image,
 * so it cannot be built here. This file restates the cited reference code
 * line by line, and the deal.II/Trilinos algorithms it calls (FEValues
 * arithmetic, AffineConstraints::distribute_local_to_global, SolverGMRES,
 * SolverFGMRES, SolverCG, SolverControl, Ifpack point Jacobi) from their
 * published behaviour; see oracle.cpp for the per-function citations.
 *
 * Conventions:
 *   - NSE local dofs in FESystem(FE_Q(2)^3, FE_Q(1)) order (89);
 *   - cell geometry = the 64 MappingQ(3) support points (Gauss-Lobatto,
 *     lexicographic) of the reference's mapping(3) (boussinesq_model.tpp:20);
 *   - temperature local dofs in FE_Q(k) hierarchic order (k = 1: vertex order);
 *   - global NSE vector = [velocity (n_u) | pressure (n_p)].
 */
#ifndef DCP_ORACLE_H
#define DCP_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  double time_step;          /* parameters.time_step */
  double one_over_reynolds;  /* 1/Re, core_model_data.cc:7-13 */
  double one_over_peclet;    /* 1/Pe, core_model_data.cc:16-22 */
  double expansion_coefficient;
  double temperature_ref;    /* reference_quantities.temperature_ref */
  double gravity_scale;      /* L / U^2 (boussinesq_model.tpp:640-643) */
  double gravity_constant;
  double coriolis_scale;     /* L / U (boussinesq_model.tpp:617-621) */
  double omega;
  int cuboid;                /* parameters.cuboid_geometry */
  int nse_solver_interval;   /* parameters.NSE_solver_interval */
  int temperature_degree;    /* 1 or 2 */
} orc_physics;

typedef struct {
  int n_lines;
  const int* line_dof;
  const int* entry_ptr;   /* n_lines + 1 */
  const int* entry_dof;
  const double* entry_w;
  const double* inhomogeneity;
} orc_constraints;

/* ---- element level (one cell) ------------------------------------------ */
/* local_assemble_nse_system (boussinesq_model.tpp:550-673). u_local: 89 NSE
 * coefficients (pressure ignored); T_local: temperature coefficients. */
void orc_cell_nse_system(const orc_physics* ph, const double* geom64,
                         const double* u_local, const double* T_local,
                         double* K /*89x89 row-major*/, double* f /*89*/);
/* local_assemble_nse_preconditioner (:421-464) */
void orc_cell_nse_preconditioner(const orc_physics* ph, const double* geom64, double* P);
/* The same two element matrices with every 89 x 89 term of the reference
 * loops evaluated (the functions above skip the FESystem's structural zeros
 * and are bitwise these, up to the sign of exact zeros). */
void orc_cell_nse_system_literal(const orc_physics* ph, const double* geom64,
                                 const double* u_local, const double* T_local, double* K,
                                 double* f);
void orc_cell_nse_preconditioner_literal(const orc_physics* ph, const double* geom64, double* P);
/* Threads of the oracle's cell loops (copier by row ranges, bitwise the
 * serial cell-order copier) and row-parallel operator applies; default 1. */
void orc_set_threads(int n);
/* local_assemble_temperature_matrix (:748-800) */
void orc_cell_temperature_matrix(const orc_physics* ph, const double* geom64, double* M,
                                 double* K);
/* local_assemble_temperature_rhs (:873-952). inhom_mask[i] != 0 marks an
 * inhomogeneously constrained local dof (fills matrix_for_bc column i). */
void orc_cell_temperature_rhs(const orc_physics* ph, const double* geom64,
                              const double* T_local, const double* u_local,
                              const int* inhom_mask, double* rhs, double* matrix_for_bc);

/* ---- global model ------------------------------------------------------- */
typedef struct orc_model orc_model;
/* parity hook: the Schur-complement solver's A^-1 and preconditioner CGs run
 * exactly k steps (0 = the reference's 1e-6 relative rule) */
void orc_set_schur_fixed_inner(orc_model* m, int k);
/* the Schur solver's ILU as on P ranks: owner[n_u] = the rank owning each
 * velocity dof, couplings between ranks dropped (block Jacobi); NULL: one rank */
void orc_set_ilu_blocks(orc_model* m, const int* owner);
/* Standard::BoussinesqModel<2>: element level (22 NSE dofs, 16 support points
 * per cell as [16][2]) and a 2D model whose other orc_* calls (schur solver,
 * temperature solve, exports, cfl) work as for the 3D one. */
void orc2d_cell_nse_system(const orc_physics* ph, const double* geom16, const double* u_local,
                           const double* T_local, double* K, double* f);
void orc2d_cell_nse_preconditioner(const orc_physics* ph, const double* geom16, double* P);
void orc2d_cell_temperature_matrix(const orc_physics* ph, const double* geom16, double* M,
                                   double* Kt);
void orc2d_cell_temperature_rhs(const orc_physics* ph, const double* geom16,
                                const double* T_local, const double* u_local,
                                const int* inhom_mask, double* rhs, double* mfbc);
orc_model* orc2d_create(const orc_physics* ph, int n_cells, const int* cell_nse_dofs,
                        const int* cell_T_dofs, const double* cell_geom, int n_u, int n_p,
                        int n_T, const orc_constraints* nse_c, const orc_constraints* T_c);

orc_model* orc_create(const orc_physics* ph, int n_cells, const int* cell_nse_dofs /*89*/,
                      const int* cell_T_dofs, const double* cell_geom /*64x3*/, int n_u,
                      int n_p, int n_T, const orc_constraints* nse_c,
                      const orc_constraints* T_c);
void orc_destroy(orc_model* m);
void orc_set_time_step(orc_model* m, double dt);

/* assemble_nse_system (:691-740) into the internal CSR nse_matrix + nse_rhs */
void orc_assemble_nse_system(orc_model* m, const double* old_nse, const double* old_T);
/* The same with WorkStream's structure: element work on `threads` threads,
 * copier serialized in cell order (bitwise the serial result; CPU baseline). */
void orc_assemble_nse_system_threads(orc_model* m, const double* old_nse, const double* old_T,
                                     int threads);
/* Timing hook: iteration cap of the inner Schur GMRES (the reference's 5000). */
void orc_set_inner_max_steps(orc_model* m, int n);
/* assemble_nse_preconditioner + build_nse_preconditioner (:479-542) */
void orc_build_nse_preconditioner(orc_model* m);
/* assemble_temperature_matrix (:821-864) */
void orc_assemble_temperature_matrix(orc_model* m);
/* assemble_temperature_rhs (:966-1020): nse_solution = the current NSE state (Q5) */
void orc_assemble_temperature_rhs(orc_model* m, const double* old_T, const double* nse_solution);

/* Accessors for parity checks. */
long orc_nse_matrix_nnz(const orc_model* m);
void orc_nse_matrix_csr(const orc_model* m, int* rowptr, int* cols, double* vals);
void orc_nse_rhs(const orc_model* m, double* out);
/* one block of nse_matrix (0: A, 1: B^T, 2: B), block-local columns; rowptr
 * NULL: returns the block's nnz only */
long orc_nse_block_csr(const orc_model* m, int which, int* rowptr, int* cols, double* vals);
void orc_precond_diagonals(const orc_model* m, double* A_diag /*n_u*/, double* Mp_diag /*n_p*/);
long orc_T_matrix_nnz(const orc_model* m);
void orc_T_matrix_csr(const orc_model* m, int* rowptr, int* cols, double* vals);
void orc_T_rhs(const orc_model* m, double* out);

/* Operators (for apply-level parity). */
void orc_nse_vmult(const orc_model* m, const double* src, double* dst);
void orc_schur_vmult(const orc_model* m, const double* src_p, double* dst_p);
void orc_block_preconditioner_vmult(orc_model* m, const double* src, double* dst,
                                    int do_solve_A, int* inner_iterations);

/* Solvers. Return 0 on success, 1 on NoConvergence (after the reference fallback). */
int orc_solve_nse(orc_model* m, double* nse_solution /*inout*/, int* outer_iterations,
                  int* inner_iterations, int max_outer /* 40 in the reference */);
int orc_solve_temperature(orc_model* m, double* T_solution /*inout*/, int* iterations);
/* solve_NSE_Schur_complement (boussinesq_model.tpp:1248-1414): GMRES on
 * B A^-1 B^T (A^-1: CG + ILU(0)) preconditioned by CG on B ILU^-1 B^T, then
 * u = A^-1 (f - B^T p). Returns 1 on NoConvergence of the Schur GMRES. */
int orc_solve_nse_schur(orc_model* m, double* nse_solution /*inout*/, int* schur_iterations,
                        int* a_solves);
/* AztecOO A-GMRES iterations of the last orc_solve_nse (do_solve_A fallback). */
long orc_a_solve_iterations(const orc_model* m);

/* CPU baseline sample: deal.II's SolverGMRES on S = B (D_A^-1 (B^T p)) from given
 * coupling blocks (block-local CSR columns), exactly k steps on orc_set_threads
 * threads; returns the wall seconds, dst_p the iterate. */
double orc_schur_gmres_sample(int n_u, int n_p, const int* bt_ptr, const int* bt_col,
                              const double* bt_val, const int* b_ptr, const int* b_col,
                              const double* b_val, const double* A_inv, const double* src_p,
                              double* dst_p, int k);

/* Step control (get_maximal_velocity / get_cfl_number, :1023-1101). */
double orc_max_velocity(const orc_model* m, const double* nse_solution);
double orc_cfl(const orc_model* m, const double* nse_solution, const double* cell_diameter);

/* ---- FEEC variant (ExteriorCalculus::BoussinesqModel<3>, config 4) ------ */
/* local dofs: 12 Nedelec (edges) + 6 RT (faces) + 1 DGQ0; X: 8 vertices x 3 */
void orc_feec_cell_system(const orc_physics* ph, const double* X, const signed char* sign19,
                          const double* dofv19, const double* T_local, double* K, double* f);
void orc_feec_cell_preconditioner(const orc_physics* ph, const double* X,
                                  const signed char* sign19, double* P);
typedef struct orc_feec orc_feec;
orc_feec* orc_feec_create(const orc_physics* ph, int n_cells, const int* cell_dofs19,
                          const signed char* sign19, const double* X24,
                          const unsigned char* fixed, int n_w, int n_u, int n_p,
                          const int* cell_T, int n_T, const orc_constraints* T_c,
                          const double* diameter);
void orc_feec_destroy(orc_feec* m);
void orc_feec_set_zero_mean(orc_feec* m, int on);
/* test hook: both inner GMRES of the FEEC preconditioner run exactly k steps */
void orc_feec_set_fixed_inner(orc_feec* m, int k);
/* use_block_preconditioner_feec (default 1); 0: identity-preconditioned GMRES(100) */
void orc_feec_set_block_preconditioner(orc_feec* m, int on);
void orc_feec_assemble_nse_system(orc_feec* m, const double* old_nse, const double* old_T);
void orc_feec_assemble_preconditioner(orc_feec* m);
long orc_feec_matrix_nnz(const orc_feec* m, int which);
void orc_feec_matrix_csr(const orc_feec* m, int which, int* rowptr, int* cols, double* vals);
void orc_feec_rhs(const orc_feec* m, double* out);
void orc_feec_assemble_temperature(orc_feec* m, const double* old_T, const double* nse_solution);
void orc_feec_T_rhs(const orc_feec* m, double* out);
int orc_feec_solve_nse(orc_feec* m, double* sol, int* iterations);
int orc_feec_solve_temperature(orc_feec* m, double* T, int* iterations);
void orc_feec_velocity_stats(const orc_feec* m, const double* sol, double* out2);

#ifdef __cplusplus
}
#endif
#endif
