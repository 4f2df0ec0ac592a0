// Time-step driver: the do-while loop of BoussinesqModel<dim>::run
// (Standard: include/core/boussinesq_model.tpp:1841-1926; ExteriorCalculus:
// include/core/boussineq_model_FEEC.tpp:2236-2310) restated over the C ABI, so a
// host program gets the reference's step sequence, step control and stopping
// rule without re-implementing them. Mesh upload and the initial state
// (setup_dofs, VectorTools::project of T0, :1793-1834) stay with the caller;
// output_results is the callback.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <string>

#include "../../include/dcp.h"

namespace dcp {
void set_ctx_error(dcp_ctx* ctx, const char* msg);  // api.cpp: dcp_last_error(ctx)
}

namespace {

// recompute_time_step (boussinesq_model.tpp:1104-1125; FEEC.tpp:1241-1261):
// step-32's CFL rule, scaling 1/4, with the model's dimension
double recomputed_time_step(const dcp_run_params* rp, double cfl) {
  const double dim = rp->space_dimension == 2 ? 2.0 : 3.0;
  const double scaling = 0.25;
  const int deg = std::max(rp->physics.temperature_degree, rp->nse_velocity_degree);
  return (scaling / (2.1 * dim * std::sqrt(dim))) / (double(deg) * cfl);
}

}  // namespace

extern "C" int dcp_run(dcp_ctx* ctx, const dcp_run_params* rp, int max_steps,
                       dcp_step_callback cb, void* user, dcp_run_report* rep) {
  if (!ctx || !rp) return DCP_ERR_INVALID;
  // TimerOutput sections of run() and output_results (:1789, :1572)
  using clock = std::chrono::steady_clock;
  const auto t_run = clock::now();
  struct RunSection {
    dcp_ctx* c;
    clock::time_point t0;
    ~RunSection() {
      dcp_timer_record(c, "BoussinesqModel - global run function",
                       std::chrono::duration<double>(clock::now() - t0).count());
    }
  } run_section{ctx, t_run};
  const bool feec = rp->use_FEEC_solver != 0;
  // solve_NSE_Schur_complement instead of the block preconditioner (:1896-1902;
  // FEEC.tpp:2292-2298)
  const bool schur = rp->use_schur_complement_solver != 0;
  auto unsupported = [&](const char* what) {
    dcp::set_ctx_error(ctx, what);
    return DCP_ERR_UNSUPPORTED;
  };
  if (rp->use_direct_solver)  // the reference throws at its first step (:1886-1893)
    return unsupported("Solver not implemented: MUMPS does not work on "
                       "TrilinosWrappers::MPI::BlockSparseMatrix classes.");
  int rc0 = DCP_OK;
  if (feec) {
    if (rp->nse_velocity_degree != 1)
      return unsupported("FEEC: only nse velocity degree = 1 (Nedelec(0) / RT(0) / DGQ(0))");
    // use block preconditioner feec = false: the identity-preconditioned
    // GMRES(100) branch (FEEC.tpp:1420-1431)
    if ((rc0 = dcp_set_option(ctx, DCP_OPT_FEEC_BLOCK_PRECONDITIONER,
                              rp->use_block_preconditioner_feec ? 1 : 0)) < 0)
      return rc0;
    // correct pressure to zero mean (both preconditioners' mean corrections)
    if ((rc0 = dcp_set_option(ctx, DCP_OPT_FEEC_ZERO_MEAN,
                              rp->correct_pressure_to_zero_mean ? 1 : 0)) < 0)
      return rc0;
  } else if (rp->nse_velocity_degree != 2) {
    return unsupported("classic model: only nse velocity degree = 2 (Q2/Q1)");
  }
  const int interval = std::max(1, rp->physics.nse_solver_interval);
  dcp_run_report r{};
  r.time_step = rp->physics.time_step;
  int rc = dcp_set_time_step(ctx, r.time_step);
  if (rc < 0) return rc;
  double time_index = 0.0;
  int n = 0;
  do {
    // step control (:1843-1856): a new dt every NSE interval when adaptive,
    // otherwise CFL and max velocity are informative only
    if ((rc = dcp_cfl_number(ctx, &r.cfl)) < 0) return rc;
    if (n > 0 && n % interval == 0 && rp->adapt_time_step) {
      r.time_step = recomputed_time_step(rp, r.cfl);
      if ((rc = dcp_set_time_step(ctx, r.time_step)) < 0) return rc;
    }
    if ((rc = dcp_max_velocity(ctx, &r.max_velocity)) < 0) return rc;
    r.time_index = time_index;
    r.timestep_number = n;
    // NSE system (re)assembly on step 0 and every NSE interval (:1865-1881)
    if (n == 0 || n % interval == 0) {
      if (feec) {
        if ((rc = dcp_feec_assemble_nse_system(ctx)) < 0) return rc;
        // FEEC.tpp:2264-2276: only without the Schur-complement solver
        if (!schur && rp->use_block_preconditioner_feec &&
            (rc = dcp_feec_build_nse_preconditioner(ctx)) < 0)
          return rc;
      } else {
        if ((rc = dcp_assemble_nse_system(ctx, DCP_ASSEMBLE_MATRIX | DCP_ASSEMBLE_RHS)) < 0)
          return rc;
        // no preconditioner with the Schur-complement solver (:1871-1881)
        if (!schur && (rc = dcp_build_nse_preconditioner(ctx)) < 0) return rc;
      }
    }
    if ((rc = dcp_assemble_temperature_matrix(ctx)) < 0) return rc;
    if ((rc = dcp_assemble_temperature_rhs(ctx)) < 0) return rc;
    // solve_NSE_block_preconditioned is called every step (:1895-1902) but
    // solves only on step 0 and every NSE interval (its own guard, :1135-1137;
    // FEEC.tpp:1272-1274); otherwise nse_solution stays as it is
    r.fgmres_outer = r.schur_inner = 0;
    rc = DCP_OK;
    if (n == 0 || n % interval == 0) {
      if (feec && schur) {
        // FEEC's solve_NSE_Schur_complement is commented out (FEEC.tpp:1480-
        // 1500): nothing is solved, nse_solution keeps its value
      } else if (feec) {
        int it = 0;
        rc = dcp_feec_solve_nse(ctx, &it);
        r.fgmres_outer = it;
      } else if (schur) {
        int a_solves = 0;  // schur_inner: the Schur GMRES steps
        rc = dcp_solve_nse_schur(ctx, &r.schur_inner, &a_solves);
      } else {
        rc = dcp_solve_nse(ctx, &r.fgmres_outer, &r.schur_inner);
      }
    }
    if (rc < 0) return rc;
    if (rc == DCP_NOT_CONVERGED) {  // the reference throws out of run()
      if (rep) *rep = r;
      return rc;
    }
    r.total_outer += r.fgmres_outer;
    r.total_inner += r.schur_inner;
    double range[2] = {0.0, 0.0};
    if ((rc = dcp_solve_temperature(ctx, &r.T_cg, range)) < 0) return rc;
    r.T_min = range[0];
    r.T_max = range[1];
    r.total_T_cg += r.T_cg;
    r.steps = n + 1;
    int stop = 0;
    if (cb) {  // output_results (:1907); non-zero stops the run
      const auto t0 = clock::now();
      stop = cb(user, &r);
      dcp_timer_record(ctx, "Postprocessing and output",
                       std::chrono::duration<double>(clock::now() - t0).count());
    }
    if (stop != 0) {
      if ((rc = dcp_advance_state(ctx)) < 0) return rc;
      break;
    }
    time_index += r.time_step / interval;  // :1918
    ++n;
    if ((rc = dcp_advance_state(ctx)) < 0) return rc;  // old_* = * (:1921-1922)
    r.time_index = time_index;
  } while (time_index <= rp->final_time && (max_steps <= 0 || n < max_steps));
  if (rep) *rep = r;
  return DCP_OK;
}
