/*
 * dcp.h — C ABI of the MI355X-native Boussinesq dynamical-core hot path
 * (libdcp.so). Drop-in boundary for the per-time-step work of
 * konsim83/3D-DyCorePlanet's Standard::BoussinesqModel<3>
 * (include/core/boussinesq_model.tpp). Every entry point below names the
 * reference member whose body it replaces.
 *
 * Conventions
 *   - Plain C types only; no exceptions cross the boundary. Every call returns
 *     DCP_OK (0), DCP_NOT_CONVERGED (1) or a negative error code; the message
 *     of the last failure is available from dcp_last_error().
 *   - Ownership: the caller owns every host buffer it passes; the library owns
 *     all device buffers. Outputs are caller-allocated.
 *   - Threading: one context per GPU / rank, calls on one context are not
 *     re-entrant.
 *   - DoF layout is the reference's after DoFRenumbering::component_wise(
 *     {0,0,0,1}) (boussinesq_model.tpp:204): NSE vector = [velocity (n_u) |
 *     pressure (n_p)], cell dof indices in FESystem(FE_Q(2)^3, FE_Q(1)) local
 *     order (89 per cell), exactly what cell->get_dof_indices() returns.
 *   - Geometry: per cell the 64 support points of the reference's mapping,
 *     MappingQ(3) (boussinesq_model.tpp:20; boussinesq_model.h:211), in
 *     lexicographic order over the 4 Gauss-Lobatto points {0, (1-1/sqrt5)/2,
 *     (1+1/sqrt5)/2, 1} per direction (x fastest), already divided by the
 *     reference length: what MappingQGeneric<3>(3)::compute_mapping_support_points
 *     returns for the cell. A cell deal.II maps with MappingQ1 (deal.II 9.2
 *     MappingQ: cells without boundary lines) is passed as its trilinear
 *     interpolant at those points, which the cubic basis reproduces exactly.
 *   - Arithmetic: IEEE FP64 throughout.
 */
#ifndef DCP_H
#define DCP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  DCP_OK = 0,
  DCP_NOT_CONVERGED = 1,      /* SolverControl::NoConvergence (boussinesq_model.tpp:1203) */
  DCP_ERR_INVALID = -1,       /* bad argument / shape mismatch */
  DCP_ERR_UNSUPPORTED = -2,   /* input the device path does not implement */
  DCP_ERR_DEVICE = -3,        /* HIP / RCCL failure or no GPU */
  DCP_ERR_STATE = -4          /* call out of order (e.g. solve before assemble) */
};

/* Version of this interface. It changes whenever a struct layout, an array
 * shape or a signature below changes (round 2 widened cell_geometry from
 * [n][27][3] to [n][64][3] and added a dcp_host_mesh_create parameter without
 * one). A caller compiled against another header must refuse to run:
 * dcp_abi_version() != DCP_ABI_VERSION. */
#define DCP_ABI_VERSION 5
int dcp_abi_version(void);
/* Support points per cell in cell_geometry (MappingQ(3): 4^3). */
#define DCP_CELL_SUPPORT_POINTS 64

typedef struct dcp_ctx dcp_ctx;

/* Derived, non-dimensional model constants (CoreModelData::Parameters after
 * parse + rescaling, boussinesq_model.tpp:14-65, core_model_data.cc:7-22). */
typedef struct {
  double time_step;             /* parameters.time_step */
  double one_over_reynolds;     /* 1 / Re */
  double one_over_peclet;       /* 1 / Pe */
  double expansion_coefficient; /* beta */
  double temperature_ref;       /* reference_quantities.temperature_ref */
  double gravity_scale;         /* L / U^2 */
  double gravity_constant;      /* g */
  double coriolis_scale;        /* L / U */
  double omega;                 /* planetary angular velocity */
  int cuboid;                   /* parameters.cuboid_geometry */
  int nse_solver_interval;      /* parameters.NSE_solver_interval */
  int temperature_degree;       /* 3D: 1; 2D model: 1 or 2 (set by dcp_mesh2d) */
} dcp_physics;

/* A closed AffineConstraints object in CSR form (one line per constrained dof). */
typedef struct {
  int n_lines;
  const int* line_dof;          /* [n_lines] */
  const int* entry_ptr;         /* [n_lines + 1] */
  const int* entry_dof;         /* [entry_ptr[n_lines]] */
  const double* entry_w;
  const double* inhomogeneity;  /* [n_lines] */
} dcp_constraints;

/* In-process group of world_size contexts on one device, each driven by its
 * own host thread (tests of the multi-rank path on a single GPU). */
typedef struct dcp_group dcp_group;

typedef struct {
  int device;           /* HIP device ordinal (local rank) */
  int rank;             /* rank in the node-local communicator */
  int world_size;       /* number of ranks / GPUs */
  const void* nccl_id;  /* ncclUniqueId (128 bytes) when world_size > 1, else NULL; with
                           world_size == 1 a non-NULL id still builds a one-rank RCCL
                           communicator, so the multi-GPU code path (partitioned
                           layout, all-reduces, halos) runs on a single GPU */
  dcp_group* group;     /* instead of nccl_id: in-process group (dcp_group_create) */
} dcp_config;

/* Multi-GPU ---------------------------------------------------------------
 * Several GPUs split the cells p4est-style (planet_geometry.h:67): rank r owns
 * cells [r n/P, (r+1) n/P) of the tree order, a DoF belongs to the rank of
 * the lowest-index cell touching it, and every rank keeps two layers of ghost
 * cells. Every rank passes the same GLOBAL mesh to dcp_mesh_upload and global
 * vectors to dcp_state_set; dcp_state_get fills the rank's owned entries.
 * Ghost DoFs are refreshed by RCCL send/recv (forward halo, the Trilinos
 * Import of the reference) and Krylov partial sums are all-reduced. */
int dcp_nccl_unique_id(void* out128);          /* rank 0; broadcast the 128 bytes */
dcp_group* dcp_group_create(int world_size);   /* in-process group (tests) */
void dcp_group_destroy(dcp_group* g);
/* Host-only partition summary of rank/world (no device): cells, owned/ghost
 * sizes per field, and the halo plan's global ids per peer for consistency
 * checks. info[12] = {n_cells_local, n_owned_cells, nvo, nvg, npo, npg, nTo,
 * nTg, n_peers_v, n_send_v, n_recv_v, n_colors}. Optional gid arrays
 * (sizes n_send_v, n_recv_v) receive the velocity-node halo lists in peer
 * order; peers (n_peers_v) the peer ranks, send_ptr/recv_ptr (n_peers_v+1). */
int dcp_partition_info(int n_cells, const int32_t* cell_nse_dofs, const int32_t* cell_T_dofs,
                       const double* cell_geometry, const double* cell_diameter, int n_u,
                       int n_p, int n_T, const dcp_constraints* nse_constraints,
                       const dcp_constraints* T_constraints, int rank, int world, int64_t* info,
                       int32_t* peers, int32_t* send_ptr, int64_t* send_gid, int32_t* recv_ptr,
                       int64_t* recv_gid);

/* Distributed upload (the reference's MPI layout) -----------------------------
 * What one deal.II rank holds after setup_dofs() on a
 * parallel::distributed::Triangulation (planet_geometry.h:67,
 * boussinesq_model.tpp:237-252): its locally owned cells and its ghost cells
 * (one vertex-neighbour layer), DoF indices in the GLOBAL numbering
 * (cell->get_dof_indices), its locally_owned_dofs() as one contiguous range per
 * block (velocity, pressure, temperature; what component_wise gives), and the
 * constraint lines of its locally relevant dofs. The library keeps this
 * ownership (each rank computes the rows of the dofs the caller owns), fetches
 * the second ghost layer the explicit Schur complement needs from the owners
 * of the caller's ghost cells, and builds the halos; the host-side exchanges
 * go through the caller's communicator (dcp_host_comm, e.g. MPI_Allgather /
 * MPI_Alltoallv on MPI_COMM_WORLD), the solver's through RCCL (dcp_config). */
typedef struct {
  void* user;
  int rank, world;
  /* every rank's `bytes` bytes, in rank order, into recv (world * bytes) */
  int (*allgather)(void* user, const void* send, size_t bytes, void* recv);
  /* send_bytes[s] bytes of send (packed in rank order) to rank s; recv gets
   * recv_bytes[s] bytes from rank s (packed in rank order) */
  int (*alltoallv)(void* user, const void* send, const size_t* send_bytes, void* recv,
                   const size_t* recv_bytes);
} dcp_host_comm;

typedef struct {
  int64_t n_lines;
  const int64_t* line_dof;      /* global dof of each line */
  const int64_t* entry_ptr;     /* [n_lines + 1] */
  const int64_t* entry_dof;     /* global dofs */
  const double* entry_w;
  const double* inhomogeneity;
} dcp_constraints64;

typedef struct {
  int n_cells;                  /* locally owned + ghost cells */
  int n_owned_cells;            /* the first n_owned_cells are the locally owned ones */
  const int64_t* cell_id;       /* [n_cells] unique global cell id (e.g. the global active index) */
  const int32_t* cell_owner;    /* [n_cells] subdomain id (rank) of each cell */
  const int64_t* cell_nse_dofs; /* [n_cells][89] global NSE dofs, FESystem local order */
  const int64_t* cell_T_dofs;   /* [n_cells][8 or 27] global temperature dofs */
  const double* cell_geometry;  /* [n_cells][64][3] */
  const double* cell_diameter;  /* [n_cells] */
  int64_t n_u, n_p, n_T;        /* global sizes */
  /* locally_owned_dofs(): [u_begin, u_end) velocity, [n_u + p_begin, n_u + p_end)
   * pressure, [T_begin, T_end) temperature (global indices) */
  int64_t u_begin, u_end, p_begin, p_end, T_begin, T_end;
  dcp_constraints64 nse, T;     /* lines of the locally relevant dofs */
} dcp_dist_mesh;
int dcp_mesh_upload_distributed(dcp_ctx* ctx, const dcp_dist_mesh* m, const dcp_host_comm* comm);
/* Host-only dry run of the distributed localisation (no device): info[12] as
 * dcp_partition_info, and the velocity halo in global node ids. Every rank of
 * `comm` must call it. */
int dcp_dist_partition_info(const dcp_dist_mesh* m, const dcp_host_comm* comm, int64_t* info,
                            int32_t* peers, int32_t* send_ptr, int64_t* send_gid,
                            int32_t* recv_ptr, int64_t* recv_gid);
/* dcp_partition_info / dcp_dist_partition_info with the halo of `field`: 0 =
 * velocity support points, 1 = pressure dofs, 2 = temperature dofs (peer
 * lists in global ids; the counts as in the velocity form). */
int dcp_partition_info_field(int n_cells, const int32_t* cell_nse_dofs, const int32_t* cell_T_dofs,
                             const double* cell_geometry, const double* cell_diameter, int n_u,
                             int n_p, int n_T, const dcp_constraints* nse_constraints,
                             const dcp_constraints* T_constraints, int rank, int world, int field,
                             int64_t* info, int32_t* peers, int32_t* send_ptr, int64_t* send_gid,
                             int32_t* recv_ptr, int64_t* recv_gid);
int dcp_dist_partition_info_field(const dcp_dist_mesh* m, const dcp_host_comm* comm, int field,
                                  int64_t* info, int32_t* peers, int32_t* send_ptr,
                                  int64_t* send_gid, int32_t* recv_ptr, int64_t* recv_gid);
/* The rank's locally owned entries of a state field, ascending global index
 * (NSE: owned velocity, then owned pressure; the Trilinos vector's local part).
 * Ghost entries are refreshed internally. Works after either upload. */
int dcp_state_set_owned(dcp_ctx* ctx, int field, const double* host, size_t n);
int dcp_state_get_owned(dcp_ctx* ctx, int field, double* host, size_t n);

/* Context / errors ------------------------------------------------------- */
int dcp_ctx_create(const dcp_config* cfg, dcp_ctx** out);
void dcp_ctx_destroy(dcp_ctx* ctx);
const char* dcp_last_error(const dcp_ctx* ctx);   /* ctx may be NULL */
int dcp_device_count(void);

/* Replaces the Parameters-derived scalars read inside the local_assemble_*
 * workers (boussinesq_model.tpp:434-438, 564-568, 760-764, 907-911). */
int dcp_set_physics(dcp_ctx* ctx, const dcp_physics* ph);
/* parameters.time_step (changed by recompute_time_step, :1104-1125). */
int dcp_set_time_step(dcp_ctx* ctx, double dt);

/* Execution options (no effect on the mathematics beyond rounding).
 * DCP_OPT_SCHUR_EXPLICIT: 1 (default) = form S = B D_A^-1 B^T once per
 *   build_nse_preconditioner and apply it as one CSR SpMV; 0 = apply it as
 *   B^T, Jacobi, B like SchurComplement::vmult (schur_complement.hpp:143-150). */
enum { DCP_OPT_SCHUR_EXPLICIT = 1 };
/* DCP_OPT_MATRIX_FREE: 1 (default) = every [A B^T; B 0] and A product of the
 *   solve (nse_matrix.vmult in SolverFGMRES, the A-GMRES of the do_solve_A
 *   fallback) is evaluated matrix-free from the mesh (kernels/matfree.hip) with
 *   the assembled diagonal for constrained dofs; 0 = block-CSR SpMV of the
 *   assembled matrix. Same operator, different rounding. */
enum { DCP_OPT_MATRIX_FREE = 3 };
/* DCP_OPT_FUSED_CHAIN: 1 (default) = on one GPU every modified Gram-Schmidt
 *   chain of the Krylov solvers (SolverGMRES's add_and_dot sequence) runs as
 *   one launch whose workgroups hand each step's reduction to each other on the
 *   device; 0 = one launch per step. Bitwise the same results. */
enum { DCP_OPT_FUSED_CHAIN = 4 };
/* DCP_OPT_ASSEMBLE_VELOCITY_BLOCK: 0 (default with DCP_OPT_MATRIX_FREE) =
 *   dcp_assemble_nse_system assembles nse_matrix in operator form: the B^T / B
 *   blocks, the rhs and the diagonal entries of the constrained velocity rows,
 *   which is everything the solve reads, while every product with the
 *   velocity-velocity block A is matrix-free; A itself is materialised
 *   (bitwise the same entries) only when something reads it
 *   (dcp_nse_matrix_export, DCP_OPT_MATRIX_FREE = 0). 1 = scatter A on every
 *   assembly too, as the reference's distribute_local_to_global does
 *   (boussinesq_model.tpp:677-687). */
enum { DCP_OPT_ASSEMBLE_VELOCITY_BLOCK = 6 };
/* DCP_OPT_GRAM_SCHMIDT: 0 (default) = the inner Schur-complement GMRES
 *   orthogonalises like deal.II SolverGMRES (modified Gram-Schmidt, one
 *   reduction per basis vector, re-orthogonalisation after a loss-of-
 *   orthogonality test); 1 = classical Gram-Schmidt applied twice (CGS2: two
 *   block reductions per Arnoldi step); 2 = DCGS2, classical Gram-Schmidt with
 *   the second pass delayed into the next step (one block reduction per
 *   Arnoldi step; each column's Givens rotation and check one step later);
 *   3 = s-step: blocks of 4 columns from a Chebyshev-shifted Newton basis (4
 *   SpMVs), orthogonalised by one launch (block CGS twice + Cholesky QR, two
 *   reductions per block), Hessenberg columns from the change of basis, then
 *   the 4 Givens steps and checks column by column (restart must be a
 *   multiple of 4). 1-3 run the Givens updates and the SolverControl check on the device
 *   so a restart cycle runs without host round trips. Same Krylov space and
 *   stopping rule; rounding differs. */
enum { DCP_OPT_GRAM_SCHMIDT = 7 };
/* DCP_OPT_FGMRES_MAX_OUTER (test hook, default 40): the iteration cap of the
 *   first FGMRES(30) (SolverControl(40, ...), boussinesq_model.tpp:1166); a
 *   lower cap sends small meshes through the do_solve_A / FGMRES(50) fallback
 *   (:1203-1232) that the reference takes when the cap is hit. */
enum { DCP_OPT_FGMRES_MAX_OUTER = 5 };
/* DCP_OPT_INNER_MAX_STEPS (probe hook, default 5000): the iteration cap of the
 *   inner Schur GMRES, SolverControl(5000, 1e-6 |src_p|) in
 *   BlockSchurPreconditioner::vmult (block_schur_preconditioner.hpp:46-51),
 *   so a large mesh can be probed for a bounded number of steps. */
enum { DCP_OPT_INNER_MAX_STEPS = 11 };
/* DCP_OPT_SCHUR_FIXED_INNER (parity hook, default 0 = the reference's rule): k
 *   > 0 runs both inner CGs of dcp_solve_nse_schur (InverseMatrix's A^-1,
 *   inverse_matrix.hpp:93-120, and the ApproximateInverseMatrix
 *   preconditioner) for exactly k steps with tolerance 0, so the solver is a
 *   smooth map of its input with no early-stop decisions for rounding to flip;
 *   the oracle has the same switch (orc_set_schur_fixed_inner). */
enum { DCP_OPT_SCHUR_FIXED_INNER = 12 };
/* DCP_OPT_ELEMENT_MFMA: 0 (default) = the velocity-velocity node-pair sums of
 *   the NSE element matrix (local_assemble_nse_system, boussinesq_model.tpp:
 *   597-640: mass + eps:eps over the 27 QGauss points) run as FP64 VALU
 *   register tiles; 1 = as v_mfma_f64_16x16x4_f64 Gram tiles (D^T W D,
 *   S^T W S). Same element matrix up to rounding; used by the full scatter
 *   (DCP_OPT_ASSEMBLE_VELOCITY_BLOCK, dcp_nse_matrix_export) and
 *   dcp_cell_nse_system. DESIGN.md section 4e has the measurement. */
enum { DCP_OPT_ELEMENT_MFMA = 9 };
/* DCP_OPT_LOG_HISTORY: 1 = record every SolverControl::check of the two
 *   FGMRES solves of dcp_solve_nse, as SolverControl(..., log_history = true,
 *   log_result = true) logs them to deallog (boussinesq_model.tpp:1166-1169,
 *   1215-1218); read back with dcp_solver_history. Default 0. */
enum { DCP_OPT_LOG_HISTORY = 10 };
/* DCP_OPT_HANDOFF_SPIN_LIMIT (test hook, process-wide, <= 0 = the default
 * 2^19): polls before a one-launch kernel's hand-off counts as timed out; a
 * tiny value makes the timeout path (rerun on the multi-launch kernels) run. */
enum { DCP_OPT_HANDOFF_SPIN_LIMIT = 13 };
/* DCP_OPT_BLOCK_FIXED_INNER (parity hook, default 0 = the reference's rule):
 * k > 0 runs the inner Schur GMRES of BlockSchurPreconditioner::vmult
 * (block_schur_preconditioner.hpp:47-51) for exactly k steps with no
 * tolerance test and uses the k-step iterate (no NoConvergence), so runs whose
 * dot products are summed in different orders (1 vs P GPUs) take the same
 * control decisions. */
enum { DCP_OPT_BLOCK_FIXED_INNER = 14 };
/* DCP_OPT_MATRIX_POWERS: 1 (default) = on several GPUs the s-step inner Schur
 * GMRES (DCP_OPT_GRAM_SCHMIDT = 3) receives each block's start vector once on
 * every pressure dof within S-graph distance 4 of the owned rows and computes
 * the next three basis vectors on the ghost rows itself (rows of S copied from
 * their owners after each formation): one halo exchange per block of 4 SpMVs
 * instead of 4. Bitwise the same iterates; 0 = one exchange per SpMV. No
 * effect on one GPU or with another DCP_OPT_GRAM_SCHMIDT. */
enum { DCP_OPT_MATRIX_POWERS = 15 };
/* DCP_OPT_T_FIXED_CG (test hook, default 0 = the reference's rule): k > 0 runs
 *   the temperature CG (dcp_solve_temperature) for exactly k steps (tolerance
 *   0, counted as converged at k), so partitioned sums cannot move its stopping
 *   step; k below the CG's convergence (steps past it divide round-off). */
enum { DCP_OPT_T_FIXED_CG = 17 };
int dcp_set_option(dcp_ctx* ctx, int option, int value);

/* The SolverControl log of the last dcp_solve_nse (DCP_OPT_LOG_HISTORY):
 * attempt 0 = the FGMRES(30) of :1166-1199, 1 = the do_solve_A FGMRES(50)
 * fallback of :1203-1232. steps/values (capacity cap, may be NULL) receive
 * (step, residual) of every check in order, deallog's "Check <step>\t<value>"
 * lines; *n their count; *result 0 = no verdict (not run), 1 = "Convergence
 * step ...", 2 = "Failure step ..." (the last check). */
int dcp_solver_history(dcp_ctx* ctx, int attempt, int* steps, double* values, int cap, int* n,
                       int* result);

/* TimerOutput of the reference (computing_timer with its section names, e.g.
 * "   Assemble NSE system", "   Solve Stokes system", "   Solve NSE system"
 * with its two nested sections; boussinesq_model.tpp:483-1572): wall time
 * (stream synchronised at the section end) and call count per section,
 * accumulated since context creation or dcp_timer_reset. dcp_timer_summary
 * writes TimerOutput::print_summary's table into buf (DCP_ERR_INVALID if len
 * is too small); dcp_timer_record adds host work of the caller under a
 * section name (e.g. "Postprocessing and output"). */
int dcp_timer_summary(dcp_ctx* ctx, char* buf, int len);
int dcp_timer_section(dcp_ctx* ctx, const char* section, long* calls, double* seconds);
int dcp_timer_record(dcp_ctx* ctx, const char* section, double seconds);
int dcp_timer_reset(dcp_ctx* ctx);

/* Mesh / DoF upload (the data setup_dofs() produces, :184-412). Builds the
 * device sparsity patterns, cell colouring and scatter maps once. */
int dcp_mesh_upload(dcp_ctx* ctx, int n_cells, const int32_t* cell_nse_dofs /*[n][89]*/,
                    const int32_t* cell_T_dofs /*[n][8]*/, const double* cell_geometry /*[n][64][3]*/,
                    const double* cell_diameter /*[n]*/, int n_u, int n_p, int n_T,
                    const dcp_constraints* nse_constraints,
                    const dcp_constraints* T_constraints);

/* Host-only dry run of dcp_mesh_upload's validation / conversion (node map,
 * node-local constraints, colouring, patterns); no device needed. */
int dcp_mesh_check(int n_cells, const int32_t* cell_nse_dofs, const int32_t* cell_T_dofs,
                   const double* cell_geometry, const double* cell_diameter, int n_u, int n_p,
                   int n_T, const dcp_constraints* nse_constraints,
                   const dcp_constraints* T_constraints, int* n_colors);

/* Host-only: is the MappingQ(3) geometry radially separable (support point
 * (a,b,c) of every cell at rho_c * Phi_ab, local c radial: the hyper_shell
 * under SphericalManifold, both for cubic and trilinear cells)?
 * Then the matrix-free operator takes J^-1 / JxW from n_columns 2D tables and
 * n_layers radial tables instead of recomputing the mapping per cell. */
int dcp_mesh_geometry_info(int n_cells, const double* cell_geometry, int* separable,
                           int* n_columns, int* n_layers);

/* Device-resident state vectors ----------------------------------------- */
enum {
  DCP_NSE_SOLUTION = 0,      /* nse_solution (n_u + n_p) */
  DCP_OLD_NSE_SOLUTION = 1,  /* old_nse_solution */
  DCP_T_SOLUTION = 2,        /* temperature_solution (n_T) */
  DCP_OLD_T_SOLUTION = 3,    /* old_temperature_solution */
  DCP_NSE_RHS = 4,           /* nse_rhs */
  DCP_T_RHS = 5              /* temperature_rhs */
};
int dcp_state_set(dcp_ctx* ctx, int field, const double* host, size_t n);
int dcp_state_get(dcp_ctx* ctx, int field, double* host, size_t n);
/* dst <- src (device copy), e.g. nse_solution <- old_nse_solution. */
int dcp_state_copy(dcp_ctx* ctx, int dst_field, int src_field);
/* Device pointer of a state field (for zero-copy interop). */
double* dcp_state_device_ptr(dcp_ctx* ctx, int field);

/* Hot path (one call per reference member) ------------------------------ */
/* assemble_nse_system (:691-740): nse_matrix + nse_rhs from old_nse_solution
 * and old_temperature_solution. flags: DCP_ASSEMBLE_MATRIX | DCP_ASSEMBLE_RHS. */
enum { DCP_ASSEMBLE_MATRIX = 1, DCP_ASSEMBLE_RHS = 2 };
int dcp_assemble_nse_system(dcp_ctx* ctx, int flags);
/* assemble_nse_preconditioner + build_nse_preconditioner (:479-542): the
 * point-Jacobi diagonals of P.block(0,0) and P.block(1,1). */
int dcp_build_nse_preconditioner(dcp_ctx* ctx);
/* assemble_temperature_matrix (:821-864). */
int dcp_assemble_temperature_matrix(dcp_ctx* ctx);
/* assemble_temperature_rhs (:966-1020); uses nse_solution (Q5). */
int dcp_assemble_temperature_rhs(dcp_ctx* ctx);
/* solve_NSE_block_preconditioned (:1131-1245) incl. the NoConvergence
 * fallback; returns DCP_NOT_CONVERGED only if the fallback fails too. */
int dcp_solve_nse(dcp_ctx* ctx, int* outer_iterations, int* inner_iterations);
/* solve_NSE_Schur_complement (:1248-1414), the use_schur_complement_solver
 * path (no build_nse_preconditioner): GMRES on B A^-1 B^T with A^-1 = CG +
 * ILU(0) of A (InverseMatrix, LA::PreconditionILU), preconditioned by CG on
 * B ILU^-1 B^T (ApproximateInverseMatrix of ApproximateSchurComplement), then
 * u = A^-1 (f - B^T p). One GPU. schur_iterations: the Schur GMRES steps;
 * a_solves: the A^-1 applications. DCP_NOT_CONVERGED if the GMRES fails. */
int dcp_solve_nse_schur(dcp_ctx* ctx, int* schur_iterations, int* a_solves);
/* solve_temperature (:1417-1476). T_range may be NULL or double[2]. */
int dcp_solve_temperature(dcp_ctx* ctx, int* iterations, double* T_range);
/* get_maximal_velocity / get_cfl_number (:1023-1101) on nse_solution. */
int dcp_max_velocity(dcp_ctx* ctx, double* out);
int dcp_cfl_number(dcp_ctx* ctx, double* out);
/* old <- current for both fields (:1921-1922). */
int dcp_advance_state(dcp_ctx* ctx);

/* Operators on device vectors (LinearAlgebra vmult seam) ----------------- */
int dcp_nse_vmult(dcp_ctx* ctx, const double* d_src, double* d_dst);          /* nse_matrix */
/* nse_matrix.block(0,0) on a velocity vector: the A products of the do_solve_A
 * GMRES (block_schur_preconditioner.hpp:59-67). */
int dcp_velocity_vmult(dcp_ctx* ctx, const double* d_src_u, double* d_dst_u);
int dcp_schur_vmult(dcp_ctx* ctx, const double* d_src_p, double* d_dst_p);    /* schur_complement.hpp:143-150 */
/* Diagnostic (no reference counterpart): `reps` back-to-back applies of an
 * operator on the context's stream between one pair of HIP events, device
 * vectors only; *ms_per_apply = elapsed / reps. which: 0 nse_matrix (the
 * matrix-free [A B^T; B 0] when DCP_OPT_MATRIX_FREE), 1 its velocity block,
 * 2 the Schur complement. Apply k reads vector k mod nvec of d_src and writes
 * the same of d_dst (nvec consecutive vectors of the operator's length each):
 * nvec vectors larger together than the 256 MB Infinity Cache keep every
 * source cold, as the Krylov vectors of a solve are. */
int dcp_time_operator(dcp_ctx* ctx, int which, int reps, int nvec, const double* d_src,
                      double* d_dst, double* ms_per_apply);
/* BlockSchurPreconditioner::vmult (block_schur_preconditioner.hpp:42-70).
 * As there, d_dst's pressure block is the inner Schur GMRES's initial guess
 * (and its velocity block the A-GMRES's when do_solve_A): pass it zeroed, or
 * holding what the caller's Krylov space left there. */
int dcp_block_preconditioner_vmult(dcp_ctx* ctx, const double* d_src, double* d_dst,
                                   int do_solve_A, int* inner_iterations);

/* Parity / export ------------------------------------------------------- */
/* nse_matrix as scalar CSR (rows n_u+n_p); call with NULL arrays to get nnz. */
int dcp_nse_matrix_export(dcp_ctx* ctx, int64_t* nnz, int32_t* rowptr, int32_t* cols, double* vals);
int dcp_T_matrix_export(dcp_ctx* ctx, int64_t* nnz, int32_t* rowptr, int32_t* cols, double* vals);
int dcp_precond_diagonals(dcp_ctx* ctx, double* A_diag, double* Mp_diag);
/* Element matrices of local_assemble_nse_system for cells [first, first+n):
 * K [n][89][89], f [n][89] in FESystem order (CopyData::NSESystem). */
int dcp_cell_nse_system(dcp_ctx* ctx, int first, int n, double* K, double* f);

/* Sizes of the device block patterns: A (3x3 blocks), B^T (3x1), B (1x3), T (scalar). */
int dcp_pattern_info(dcp_ctx* ctx, int64_t* nnzb_A, int64_t* nnzb_Bt, int64_t* nnzb_B,
                     int64_t* nnz_T, int64_t* nnz_S);

/* Storage of the explicit Schur complement (SELL-64): bytes per column index
 * (0: structured columns formed from the row's radial level and a lateral
 * neighbour table, one GPU on the layered shell; 2: 16-bit offsets from a
 * slice base; 4: int32), stored entries incl. padding, whether rows/columns
 * are permuted (level-major with structured columns, else reverse
 * Cuthill-McKee). */
int dcp_schur_layout(dcp_ctx* ctx, int* col_bytes, int64_t* stored, int* permuted);

/* The forms the assembly runs in. Temperature (assemble_temperature_matrix /
 * _rhs, boussinesq_model.tpp:748-1020): info[0] = 1 when the separable
 * Kronecker form runs (the layered shell, one product of columns and layers,
 * FE_Q(1), no periodic identity; DCP_T_SEPARABLE=0 disables it), 0 for the
 * colour kernels; [1] column ids, [2] radial layers, [3] layer kinds, [4]
 * lateral pattern entries. B^T of nse_matrix (:626-637, :677-687): [5] = 1
 * when the operator-form assembly writes it in Kronecker form (one GPU,
 * layered shell; DCP_BT_KRON=0 keeps the row tasks), [6] lateral
 * (node, vertex) pairs, [7] entries of constrained rows. */
int dcp_assembly_layout(dcp_ctx* ctx, int64_t info[8]);

/* Communicator self-test (no mesh needed): the solver's forward halo (gather
 * of vec[send_pos], grouped send/recv, scatter into vec[recv_pos]) with every
 * peer this rank itself, the n_list entries split over n_peers self-peers. On
 * a one-rank RCCL communicator this runs ncclSend/ncclRecv to its own rank. */
int dcp_halo_selftest(dcp_ctx* ctx, int n, double* vec, int n_list, const int32_t* send_pos,
                      const int32_t* recv_pos, int n_peers);

/* Communicator self-test of the all-reduce (every rank of the communicator
 * must call it with the same n and reps): vec (n doubles) is summed over the
 * ranks in place (the solver's partial-sum all-reduce; the result returned in
 * vec), then reps - 1 further all-reduces (max, so values stay finite) run
 * back to back between one HIP event pair: *ms_per_call is their average. */
int dcp_allreduce_selftest(dcp_ctx* ctx, double* vec, size_t n, int reps, double* ms_per_call);

/* Scatter bookkeeping of the assembly (copy_local_to_global_nse_system,
 * boussinesq_model.tpp:677-687): per block pattern A, B^T, B ([3] each) the
 * blocks some cell's scatter position reaches, the pattern size, and whether
 * the assembly stores at first touch (1) or zero-fills and adds (0). */
int dcp_scatter_info(dcp_ctx* ctx, int64_t* touched, int64_t* nnzb, int* first_touch);

/* The matrix powers of the last s-step inner solve (DCP_OPT_MATRIX_POWERS,
 * several GPUs): info[0] = 1 if built, [1] the extended pressure vector length
 * (local dofs + the further dofs the ghost rows reach), [2..4] ghost rows of
 * depth <= 1, 2, 3, [5] entries received per block (the depth-4 halo), [6]
 * ghost-row values received per formation of S, [7] the per-SpMV halo's
 * receive count. Zeros on one GPU or before the first such solve. */
int dcp_matrix_powers_info(dcp_ctx* ctx, int64_t info[8]);

/* The context's communicator as the transport reports it: info[0] = 0 (none,
 * one GPU), 1 (RCCL: [1] ncclCommCount, [2] ncclCommUserRank, [3]
 * ncclCommCuDevice), 2 (in-process group: size, rank, current device) or 3
 * (in-process group with device-initiated all-reduces, DCP_PEER_COMM=1 at
 * dcp_ctx_create: size, rank, device). */
int dcp_comm_info(dcp_ctx* ctx, int32_t info[4]);

/* Local sizes of the context's mesh: [0] local cells (owned + ghost layers),
 * [1] owned cells, [2] local velocity dofs, [3] local pressure dofs, [4] local
 * temperature dofs, [5] owned velocity dofs, [6] owned pressure dofs, [7]
 * owned temperature dofs (one GPU: local = owned = global). */
int dcp_local_sizes(dcp_ctx* ctx, int64_t out[8]);

/* Device bytes held by the buffers the CALLING host thread allocated through
 * the library (context state, operators, Krylov pools): live now and the peak.
 * One context per thread (one rank per process, or one rank per thread in an
 * in-process group) makes these the context's own footprint. Diagnostic; it
 * replaces no reference interface (deal.II's MemoryConsumption has no
 * counterpart on this path). */
int dcp_device_memory(int64_t* live_bytes, int64_t* peak_bytes);

/* The operator form's coupling blocks of nse_matrix as scalar CSR, without
 * materialising the velocity block: which = 0 -> B^T (3 n_vnodes rows, pressure
 * columns), 1 -> B (n_p rows, velocity columns 3 n + c), the B the Schur
 * complement reads. nnz first (rowptr NULL), then the arrays. */
int dcp_nse_coupling_export(dcp_ctx* ctx, int which, int64_t* nnz, int32_t* rowptr, int32_t* cols,
                            double* vals);

/* Timing of the last hot-path calls (device time, milliseconds). */
typedef struct {
  double assemble_nse_ms, build_precond_ms, assemble_T_matrix_ms, assemble_T_rhs_ms;
  double solve_nse_ms, solve_T_ms;
  double schur_apply_ms_avg; /* average device time of one Schur-complement apply */
  long schur_applies;
  /* matrix-free applies of the last solve (DCP_OPT_MATRIX_FREE): [A B^T; B 0]
   * (nse_matrix.vmult) and A alone (do_solve_A fallback); sampled device time */
  double stokes_apply_ms_avg, velocity_apply_ms_avg;
  long stokes_applies, velocity_applies;
  /* AztecOO A-GMRES iterations of the do_solve_A fallback (not reported by
   * the reference; block_schur_preconditioner.hpp:59-67) */
  long a_solve_iterations;
  /* one-launch Gram-Schmidt hand-offs that timed out since the context was
   * created (each reran its inner solve on the multi-launch kernels and turned
   * DCP_OPT_FUSED_CHAIN off; 0 on a healthy GPU) */
  long handoff_timeouts;
} dcp_timings;
int dcp_get_timings(dcp_ctx* ctx, dcp_timings* out);

/* FEEC variant --------------------------------------------------------------
 * ExteriorCalculus::BoussinesqModel<3> (boussineq_model_FEEC.tpp, config 4):
 * lowest-order Nedelec vorticity w (edges), Raviart-Thomas velocity u (faces),
 * DGQ0 pressure p (cells), MappingQ1. NSE state vector = [w | u | p]
 * (n_w + n_u + n_p); temperature as in the classic model (Q1). A context
 * holds either a classic or an FEEC mesh; the temperature calls, CFL / max
 * velocity and state calls dispatch on it. Several GPUs: every rank passes
 * the global mesh and keeps its cells + two ghost layers (as for
 * dcp_mesh_upload); state calls take global vectors. */
typedef struct {
  int n_cells, n_w, n_u, n_p, n_T;
  const int32_t* cell_w;          /* [n_cells][12] edge dofs, deal.II line order */
  const int8_t* sign_w;           /* [n_cells][12] +-1 local edge direction vs global */
  const int32_t* cell_u;          /* [n_cells][6] face dofs, deal.II face order */
  const int8_t* sign_u;           /* [n_cells][6] +-1 local flux direction vs global */
  const double* cell_vertices;    /* [n_cells][8][3] (lexicographic vertices) */
  const double* cell_diameter;    /* [n_cells] */
  const int32_t* cell_T_dofs;     /* [n_cells][8] */
  const uint8_t* w_fixed;         /* [n_w] boundary edge: w = 0 (FEEC.tpp:311-350) */
  const uint8_t* u_fixed;         /* [n_u] boundary face: u.n = 0 */
  dcp_constraints T;              /* temperature constraints: Dirichlet lines and
                                   * periodic identities (one entry, weight 1, no
                                   * inhomogeneity: the image is folded into its
                                   * partner, one GPU) */
} dcp_feec_mesh;
/* On the periodic cuboid (FEEC.tpp:313-333) the x = 1 / y = 1 edges and faces
 * ARE their x = 0 / y = 0 partners in cell_w / cell_u (make_periodicity_
 * constraints with unit weights, condensed): no NSE constraint lines beyond
 * the fixed flags of the z faces. A cell must not hold a dof twice. */
int dcp_feec_mesh_upload(dcp_ctx* ctx, const dcp_feec_mesh* m);
/* Host-only summary of rank's FEEC partition (no GPU): info[11] = {n_cells
 * local, n_owned_cells, nwo, nwg, nuo, nug, nTo, nTg, n_peers, n_send,
 * n_recv} for the halo of `field` (0 edges w, 1 faces u, 2 cells p, 3 T
 * vertices); optional arrays as in dcp_partition_info. */
int dcp_feec_partition_info(const dcp_feec_mesh* m, int rank, int world, int field,
                            int64_t* info, int32_t* peers, int32_t* send_ptr, int64_t* send_gid,
                            int32_t* recv_ptr, int64_t* recv_gid);
/* assemble_nse_system (FEEC.tpp:669-873) */
int dcp_feec_assemble_nse_system(dcp_ctx* ctx);
/* assemble_nse_preconditioner / build_nse_preconditioner (FEEC.tpp:509-660) */
int dcp_feec_build_nse_preconditioner(dcp_ctx* ctx);
/* solve_NSE_block_preconditioned (FEEC.tpp:1268-1477): GMRES(100) <= 500 with
 * BlockSchurPreconditionerFEEC (or, DCP_OPT_FEEC_BLOCK_PRECONDITIONER = 0,
 * <= 15000 with the block identity); DCP_NOT_CONVERGED if it does not converge. */
int dcp_feec_solve_nse(dcp_ctx* ctx, int* iterations);
/* DCP_OPT_FEEC_ZERO_MEAN (default 1): parameters.correct_pressure_to_zero_mean */
enum { DCP_OPT_FEEC_ZERO_MEAN = 2 };
/* DCP_OPT_FEEC_FIXED_INNER (test hook, default 0 = the reference's rule): k > 0
 *   runs both inner GMRES of BlockSchurPreconditionerFEEC for exactly k steps
 *   (tolerance 0, the NoConvergence swallowed as the reference does), so the
 *   preconditioner is a smooth map of its input with no early-stop decisions
 *   for rounding to flip; the oracle has the same switch. */
enum { DCP_OPT_FEEC_FIXED_INNER = 8 };
/* DCP_OPT_FEEC_BLOCK_PRECONDITIONER (default 1): parameters.use_block_preconditioner_feec.
 *   0: dcp_feec_solve_nse runs the reference's other branch
 *   (boussineq_model_FEEC.tpp:1420-1431): SolverGMRES(100) <= 15000 iterations,
 *   tol 1e-8 |rhs|, with PreconditionerBlockIdentity (dst = src, then the pressure
 *   block minus its QGauss(2) mean value if correct_pressure_to_zero_mean,
 *   preconditioner_block_identity.hpp:31-53); no preconditioner build needed. */
enum { DCP_OPT_FEEC_BLOCK_PRECONDITIONER = 16 };
/* element matrices / rhs of cells [first, first+n): K [n][19][19], f [n][19] */
int dcp_feec_cell_system(dcp_ctx* ctx, int first, int n, double* K, double* f);
/* which = 0: nse_matrix, 1: nse_preconditioner_matrix (CSR, n_w+n_u+n_p rows) */
int dcp_feec_matrix_export(dcp_ctx* ctx, int which, int64_t* nnz, int32_t* rowptr, int32_t* cols,
                           double* vals);

/* Two-dimensional model ---------------------------------------------------
 * Standard::BoussinesqModel<2> (boussinesq_model.inst.cc:8; the 2D test
 * configuration data/aqua_planet_test_2d.prm). FESystem(FE_Q(2)^2, FE_Q(1)):
 * 22 dofs per cell in FESystem local order (per vertex u_x u_y p, per line
 * u_x u_y, interior u_x u_y; deal.II vertex and line order); NSE vector =
 * [u (n_u) | p (n_p)] after component_wise({0,0,1}); temperature
 * FE_Q(temperature_degree), degree 1 or 2, in FE_Q local order (4 or 9 dofs
 * per cell); geometry: the 16 MappingQ(3) support points per cell
 * ([n][16][2], 4 x 4 Gauss-Lobatto, x fastest). The NSE constraint lines must
 * be homogeneous with at most one entry on a dof of the same cells (the
 * no-slip / no-normal-flux lines of the shell are), the temperature lines
 * Dirichlet. Several GPUs: every rank passes the global mesh and keeps its
 * cells + two ghost layers (as dcp_mesh_upload). After the upload the hot-path calls above (assemble,
 * preconditioner, dcp_solve_nse / dcp_solve_nse_schur, temperature, CFL,
 * state, vmults, exports; dcp_cell_nse_system returns [n][22][22] / [n][22])
 * act on the 2D model. */
typedef struct {
  int n_cells, n_u, n_p, n_T;
  int temperature_degree;          /* 1 or 2 */
  const int32_t* cell_nse_dofs;    /* [n_cells][22] */
  const int32_t* cell_T_dofs;      /* [n_cells][(degree + 1)^2] */
  const double* cell_geometry;     /* [n_cells][16][2] */
  const double* cell_diameter;     /* [n_cells] */
  dcp_constraints nse, T;
} dcp_mesh2d;
int dcp_mesh2d_upload(dcp_ctx* ctx, const dcp_mesh2d* m);
/* Host-only dry run of dcp_mesh2d_upload's validation, patterns and colouring. */
int dcp_mesh2d_check(const dcp_mesh2d* m, int* n_colors);
/* Host-only summary of rank's 2D partition (no GPU; several GPUs take the
 * global mesh in dcp_mesh2d_upload and keep their cells + two ghost layers):
 * info[11] = {n_cells, n_owned_cells, owned / ghost velocity dofs, owned /
 * ghost pressure, owned / ghost temperature, peers, send, recv} and the halo
 * lists (global ids) of field 0 (velocity), 1 (pressure), 2 (temperature);
 * the local mesh is run through dcp_mesh2d_check's validation as well. */
int dcp_mesh2d_partition_info(const dcp_mesh2d* m, int rank, int world, int field, int64_t* info,
                              int32_t* peers, int32_t* send_ptr, int64_t* send_gid,
                              int32_t* recv_ptr, int64_t* recv_gid);

/* Host setup helpers (mesh generator, .prm) ----------------------------- */
typedef struct dcp_host_mesh dcp_host_mesh;
/* Builds the refined shell (cuboid = 0) or cube, DoFs and constraints the way
 * setup_dofs() does (see mesh.h for the geometry convention: hyper_shell +
 * SphericalManifold refinement, MappingQ(3) support points per cell).
 * normal_mode of the no-normal-flux constraint: 0 = deal.II's
 * compute_no_normal_flux_constraints rule (normals of the mapped boundary
 * faces at the support point, averaged; default), 1 = radial (exact sphere
 * normal), 2 = consistent (minus the B^T 1 row, Engelman et al.). mapping_q_on_all_cells: 0 =
 * deal.II 9.2 MappingQ (cubic map on boundary cells, MappingQ1 inside), 1 =
 * deal.II >= 9.3 (cubic everywhere). */
dcp_host_mesh* dcp_host_mesh_create(int cuboid, int refine, double R0, double R1, double length,
                                    int temperature_degree, int normal_mode,
                                    int mapping_q_on_all_cells);
void dcp_host_mesh_destroy(dcp_host_mesh* m);
/* DoFRenumbering::Cuthill_McKee + component_wise of the NSE dofs, what
 * setup_dofs() does when use_schur_complement_solver is set
 * (boussinesq_model.tpp:198-204): cell dofs, NSE constraints and node_xyz of
 * later views follow the new numbering (velocity 3 n + c stays node-major). */
int dcp_host_mesh_renumber_cuthill_mckee(dcp_host_mesh* m);
/* deal.II's own DoF order on the 6-cell shell (setup_dofs,
 * boussinesq_model.tpp:197-206: distribute_dofs over GridGenerator::
 * hyper_shell's cells refined refine_global times, then component_wise
 * {0,0,0,1}; the temperature dof handler's distribute_dofs likewise): NSE and
 * temperature dofs, constraints and node_xyz of later views follow it; the
 * cells themselves keep the mesh's order. cell_order (optional, [n_cells]):
 * the mesh cell of each deal.II active cell, in deal.II's order. Call before
 * dcp_host_mesh_renumber_cuthill_mckee (the Schur configs renumber from this
 * order, as the reference does). 3D shell only. */
int dcp_host_mesh_renumber_dealii(dcp_host_mesh* m, int32_t* cell_order);
typedef struct {
  int n_cells, n_u, n_p, n_T, n_vnodes;
  const int32_t* cell_nse_dofs;   /* [n_cells][89] */
  const int32_t* cell_T_dofs;     /* [n_cells][8] */
  const double* cell_geometry;    /* [n_cells][64][3] MappingQ(3) support points */
  const double* cell_diameter;    /* [n_cells] */
  const double* node_xyz;         /* [n_vnodes][3] */
  dcp_constraints nse, T;
} dcp_host_mesh_view;
int dcp_host_mesh_view_get(const dcp_host_mesh* m, dcp_host_mesh_view* out);
/* FEEC topology of the host mesh (edges, faces, signs, boundary flags); the
 * arrays stay owned by the host mesh. */
int dcp_host_feec_view_get(dcp_host_mesh* m, dcp_feec_mesh* out);
/* T dof values of the initial temperature at the support points. */
int dcp_host_mesh_initial_temperature(const dcp_host_mesh* m, double* T);
/* The 2D shell: GridGenerator::hyper_shell<2>(0, R0, R1, 12 cells, colorize)
 * under SphericalManifold, refine_global(refine) (planet_geometry.tpp:63-68),
 * the DoFs of distribute_dofs + component_wise, the no-slip / no-normal-flux
 * and temperature constraints of setup_dofs() (:255-387) with
 * TemperatureInitialValues<2>. dcp_host_mesh_renumber_cuthill_mckee and
 * dcp_host_mesh_initial_temperature accept it; dcp_host_mesh_view_get does
 * not (use dcp_host_mesh2d_view_get: the arrays stay owned by the mesh). */
dcp_host_mesh* dcp_host_mesh2d_create(int refine, double R0, double R1, double length,
                                      int temperature_degree, int mapping_q_on_all_cells);
int dcp_host_mesh2d_view_get(const dcp_host_mesh* m, dcp_mesh2d* out, const double** node_xy,
                             int* n_vnodes);

/* output_results (boussinesq_model.tpp:1566-1680), classic model, host-only:
 * DataOut::build_patches(nse_velocity_degree = 2) of the joint [u p T] solution
 * -- per cell the 27 lattice points of {0, 1/2, 1}^3 under DataOut's default
 * MappingQ1 and 8 sub-hexahedra -- with the Postprocessor's point data
 * "velocity", "p", "T", "partition" (:1492-1554), written as a VTU file
 * (XML, ASCII data arrays). nse: n_u + n_p global values, T: n_T. */
int dcp_write_vtu(const dcp_host_mesh_view* mesh, const double* nse, const double* T,
                  int partition, const char* vtu_path);
/* write_pvtu_record: the .pvtu naming the n_pieces per-rank .vtu files. */
int dcp_write_pvtu_record(const char* pvtu_path, int n_pieces, const char* const* piece_files);
/* FEEC output_results (boussineq_model_FEEC.tpp:1917-2030): DataOut::
 * build_patches(min(nse_velocity_degree, temperature_degree) = 1) of the joint
 * [w u p T] solution -- one hexahedron per cell on its 8 vertices -- with the
 * Postprocessor's point data "vorticity" (Nedelec(0), covariant Piola),
 * "velocity" (RT(0), contravariant Piola), "p" (DGQ0), "T", "partition"
 * (:1808-1912). nse: n_w + n_u + n_p global values [w | u | p], T: n_T. */
int dcp_write_feec_vtu(const dcp_feec_mesh* mesh, const double* nse, const double* T,
                       int partition, const char* vtu_path);
int dcp_write_feec_pvtu_record(const char* pvtu_path, int n_pieces, const char* const* piece_files);

/* .prm -> dcp_physics (+ refinement etc.), CoreModelData::Parameters(file). */
typedef struct {
  dcp_physics physics;
  int initial_global_refinement, space_dimension, nse_velocity_degree;
  int use_schur_complement_solver, use_FEEC_solver, adapt_time_step;
  double final_time, R0, R1, length;
  int use_block_preconditioner_feec, correct_pressure_to_zero_mean;
  int solver_diagnostics_level;     /* deallog.depth_console level (main.cxx:89) */
  int use_direct_solver;            /* MUMPS branch: the reference throws (:1886-1893) */
} dcp_run_params;
int dcp_prm_load(const char* path, dcp_run_params* out, char* err, int err_len);

/* Time-step driver: the do-while loop of BoussinesqModel<dim>::run
 * (boussinesq_model.tpp:1841-1926, FEEC: boussineq_model_FEEC.tpp:2236-2310)
 * over the calls above, after the caller has uploaded the mesh and the initial
 * state: per step the CFL / max-velocity step control (recompute_time_step
 * every NSE interval when adapt_time_step, :1104-1125), NSE (re)assembly and
 * preconditioner on step 0 and every NSE interval, temperature matrix and
 * rhs, the NSE and temperature solves, the callback (output_results; a
 * non-zero return stops), time_index += dt / interval, old_* = *; until
 * time_index > final_time or max_steps (> 0) steps. Returns DCP_NOT_CONVERGED
 * where the reference's solve throws. use_schur_complement_solver selects
 * dcp_solve_nse_schur (one GPU); with use_FEEC_solver it selects the FEEC
 * model's solve_NSE_Schur_complement, whose body is commented out
 * (boussineq_model_FEEC.tpp:1480-1500): no preconditioner build and no NSE
 * solve, nse_solution keeps its value (FEEC.tpp:2264-2298). Returns
 * DCP_ERR_UNSUPPORTED where the reference throws (use_direct_solver,
 * :1886-1893, FEEC.tpp:2282-2290) and for what the device path does not
 * implement: nse_velocity_degree other than 2 (classic) / 1 (FEEC), FEEC
 * without its block preconditioner (the identity-preconditioned GMRES branch,
 * FEEC.tpp:1420-1431), FEEC on the periodic cuboid. */
typedef struct {
  int timestep_number, steps;       /* current step; steps completed */
  double time_index, time_step;     /* t at the step's start; dt */
  double cfl, max_velocity;         /* get_cfl_number / get_maximal_velocity */
  int fgmres_outer, schur_inner, T_cg;           /* this step */
  long total_outer, total_inner, total_T_cg;     /* whole run */
  double T_min, T_max;              /* solve_temperature range */
} dcp_run_report;
typedef int (*dcp_step_callback)(void* user, const dcp_run_report* step);
int dcp_run(dcp_ctx* ctx, const dcp_run_params* rp, int max_steps, dcp_step_callback cb,
            void* user, dcp_run_report* report);

#ifdef __cplusplus
}
#endif
#endif
