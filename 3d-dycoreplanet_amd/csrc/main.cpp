// dcp_aquaplanet -p <file.prm> [--refine R] [--max-steps N] [--device D]
//                [--output DIR [--output-stem NAME]] [--dof-order dealii|mesh]
//
// The reference executable (source/main.cxx: parse -p, construct the model
// from the parameter file, run()) over libdcp.so: CoreModelData::Parameters
// from the same .prm (dcp_prm_load), the refined shell / cube with its DoFs
// and constraints (setup_dofs, dcp_host_mesh_create; Cuthill-McKee for the
// Schur-complement solver), the initial temperature,
// then the time loop (dcp_run) with the reference's per-step log lines.
// --dof-order: the 3D shell's dofs in deal.II's distribute_dofs order
// (default; dcp_host_mesh_renumber_dealii) or the mesh's own tree order.
// --output: output_results (boussinesq_model.tpp:1566-1680) before the loop
// and after every step, DIR/NAME-XXXXX.0000.vtu + NAME-XXXXX.pvtu (classic;
// FEEC: boussineq_model_FEEC.tpp:1917-2030, vorticity / velocity / p / T).
// Single GPU; the multi-GPU path is driven through the same ABI by one process
// per GPU (bench.py).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/dcp.h"

namespace {

int fail(const char* what, dcp_ctx* ctx) {
  std::fprintf(stderr, "Error: %s: %s\n", what, dcp_last_error(ctx));
  return 1;
}

struct Output {
  dcp_ctx* ctx = nullptr;
  const dcp_host_mesh_view* view = nullptr;
  const dcp_feec_mesh* feec = nullptr;  // FEEC model: its own output_results
  std::string dir, stem;
  int index = 0;
  size_t n_nse = 0;
};

// output_results: the joint solution of this step as VTU + the pvtu record
int write_output(Output& o) {
  std::vector<double> u(o.n_nse), T(size_t(o.view->n_T));
  int rc = dcp_state_get(o.ctx, DCP_NSE_SOLUTION, u.data(), u.size());
  if (rc == DCP_OK) rc = dcp_state_get(o.ctx, DCP_T_SOLUTION, T.data(), T.size());
  char idx[16];
  std::snprintf(idx, sizeof(idx), "%05d", o.index++);
  const std::string piece = o.stem + "-" + idx + ".0000.vtu";
  const std::string vtu = o.dir + "/" + piece, pvtu = o.dir + "/" + o.stem + "-" + idx + ".pvtu";
  if (rc == DCP_OK)
    rc = o.feec ? dcp_write_feec_vtu(o.feec, u.data(), T.data(), 0, vtu.c_str())
                : dcp_write_vtu(o.view, u.data(), T.data(), 0, vtu.c_str());
  const char* pieces[1] = {piece.c_str()};
  if (rc == DCP_OK)
    rc = o.feec ? dcp_write_feec_pvtu_record(pvtu.c_str(), 1, pieces)
                : dcp_write_pvtu_record(pvtu.c_str(), 1, pieces);
  if (rc != DCP_OK) std::fprintf(stderr, "Error: writing %s/%s\n", o.dir.c_str(), piece.c_str());
  return rc;
}

struct Runner {
  dcp_ctx* ctx = nullptr;
  Output* out = nullptr;
  int diagnostics = 1;  // deallog.depth_console(solver diagnostics level), main.cxx:89
  int interval = 1;
};

// deallog at depth 2: SolverFGMRES's prefix and SolverControl's log_history /
// log_result lines of the step's NSE solve (boussinesq_model.tpp:1166-1169)
void print_solver_log(dcp_ctx* ctx) {
  for (int attempt = 0; attempt < 2; ++attempt) {
    int n = 0, result = 0;
    if (dcp_solver_history(ctx, attempt, nullptr, nullptr, 0, &n, &result) != DCP_OK || n == 0)
      continue;
    std::vector<int> steps(static_cast<size_t>(n));
    std::vector<double> vals(static_cast<size_t>(n));
    dcp_solver_history(ctx, attempt, steps.data(), vals.data(), n, &n, &result);
    for (int i = 0; i < n; ++i) std::printf("DEAL:FGMRES::Check %d\t%g\n", steps[size_t(i)], vals[size_t(i)]);
    if (result)
      std::printf("DEAL:FGMRES::%s step %d value %g\n", result == 1 ? "Convergence" : "Failure",
                  steps.back(), vals.back());
  }
}

int print_step(void* user, const dcp_run_report* r) {
  std::printf("----------------------------------------\n");
  std::printf("Time step %d:  t=%g -> t=%g  (dt=%g)\n", r->timestep_number, r->time_index,
              r->time_index + r->time_step, r->time_step);
  std::printf("   Max velocity (dimensionsless): %g\n", r->max_velocity);
  std::printf("   Max of local CFL numbers: %g\n", r->cfl);
  if (r->schur_inner > 0)
    std::printf("   Solved (outer / inner Schur GMRES): %d / %d\n", r->fgmres_outer, r->schur_inner);
  else
    std::printf("   Solved (GMRES): %d\n", r->fgmres_outer);
  std::printf("   Temperature: %d CG iterations, range %g %g\n", r->T_cg, r->T_min, r->T_max);
  Runner* run = static_cast<Runner*>(user);
  if (run->diagnostics >= 2) print_solver_log(run->ctx);
  if (run->out && write_output(*run->out) != DCP_OK) return 1;  // stop the run
  // computing_timer.print_summary() after every NSE interval (:1912-1916)
  if (r->timestep_number > 0 && r->timestep_number % run->interval == 0) {
    std::vector<char> buf(1 << 16);
    if (dcp_timer_summary(run->ctx, buf.data(), int(buf.size())) == DCP_OK)
      std::printf("%s", buf.data());
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  std::string prm, out_dir, out_stem = "boussinesq";
  int refine = -1, max_steps = 0, device = 0;
  bool dealii_order = true;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    if (a == "-p" && i + 1 < argc) {
      prm = argv[++i];
    } else if (a == "--refine" && i + 1 < argc) {
      refine = std::atoi(argv[++i]);
    } else if (a == "--max-steps" && i + 1 < argc) {
      max_steps = std::atoi(argv[++i]);
    } else if (a == "--device" && i + 1 < argc) {
      device = std::atoi(argv[++i]);
    } else if (a == "--output" && i + 1 < argc) {
      out_dir = argv[++i];
    } else if (a == "--output-stem" && i + 1 < argc) {
      out_stem = argv[++i];
    } else if (a == "--dof-order" && i + 1 < argc) {
      const std::string o = argv[++i];
      if (o != "dealii" && o != "mesh") {
        std::fprintf(stderr, "Error: --dof-order must be dealii or mesh\n");
        return 1;
      }
      dealii_order = o == "dealii";
    } else {
      std::fprintf(stderr, "Unknown command line option: %s\n", a.c_str());
      return 1;
    }
  }
  if (prm.empty()) {
    std::fprintf(stderr, "Error: flag '-p' must be followed by the name of a parameter file.\n");
    return 1;
  }
  dcp_run_params rp{};
  char err[512] = {0};
  if (dcp_prm_load(prm.c_str(), &rp, err, sizeof(err)) != DCP_OK) {
    std::fprintf(stderr, "Error: %s\n", err);
    return 1;
  }
  if (refine >= 0) rp.initial_global_refinement = refine;
  if (rp.space_dimension != 2 && rp.space_dimension != 3) {
    std::fprintf(stderr, "Error: space dimension must be 2 or 3\n");
    return 1;
  }
  const bool two_d = rp.space_dimension == 2;
  const bool feec = rp.use_FEEC_solver != 0;
  if (two_d && (feec || rp.physics.cuboid)) {
    std::fprintf(stderr, "Error: the 2D model runs the classic solver on the shell\n");
    return 1;
  }
  // Standard::BoussinesqModel<2> / <3> (boussinesq_model.inst.cc)
  dcp_host_mesh* m =
      two_d ? dcp_host_mesh2d_create(rp.initial_global_refinement, rp.R0, rp.R1, rp.length,
                                     rp.physics.temperature_degree, 0)
            : dcp_host_mesh_create(rp.physics.cuboid, rp.initial_global_refinement, rp.R0, rp.R1,
                                   rp.length, rp.physics.temperature_degree, 0, 0);
  if (!m) return fail("mesh", nullptr);
  // setup_dofs (:197-206): distribute_dofs in deal.II's cell order (the 2D
  // shell is built in it; the 3D shell is renumbered to it)
  if (!two_d && !rp.physics.cuboid && dealii_order && dcp_host_mesh_renumber_dealii(m, nullptr) != DCP_OK)
    return fail("deal.II dof order", nullptr);
  // setup_dofs (:198-204): Cuthill_McKee before component_wise for the Schur solver
  if (!feec && rp.use_schur_complement_solver && dcp_host_mesh_renumber_cuthill_mckee(m) != DCP_OK)
    return fail("renumbering", nullptr);
  dcp_host_mesh_view v{};
  dcp_mesh2d v2{};
  if (two_d) {
    dcp_host_mesh2d_view_get(m, &v2, nullptr, nullptr);
    v.n_cells = v2.n_cells;
    v.n_u = v2.n_u;
    v.n_p = v2.n_p;
    v.n_T = v2.n_T;
  } else {
    dcp_host_mesh_view_get(m, &v);
  }
  dcp_config cfg{device, 0, 1, nullptr, nullptr};
  dcp_ctx* ctx = nullptr;
  if (dcp_ctx_create(&cfg, &ctx) != DCP_OK) return fail("context", nullptr);
  int rc = dcp_set_physics(ctx, &rp.physics);
  size_t n_nse = size_t(v.n_u) + size_t(v.n_p);
  dcp_feec_mesh fm{};
  if (rc == DCP_OK) {
    if (two_d) {
      rc = dcp_mesh2d_upload(ctx, &v2);
    } else if (feec) {
      rc = dcp_host_feec_view_get(m, &fm);
      if (rc == DCP_OK) rc = dcp_feec_mesh_upload(ctx, &fm);
      n_nse = size_t(fm.n_w) + size_t(fm.n_u) + size_t(fm.n_p);
      if (rc == DCP_OK)
        rc = dcp_set_option(ctx, DCP_OPT_FEEC_ZERO_MEAN, rp.correct_pressure_to_zero_mean);
    } else {
      rc = dcp_mesh_upload(ctx, v.n_cells, v.cell_nse_dofs, v.cell_T_dofs, v.cell_geometry,
                           v.cell_diameter, v.n_u, v.n_p, v.n_T, &v.nse, &v.T);
    }
  }
  if (rc != DCP_OK) return fail("upload", ctx);
  std::printf("Number of active cells: %d\nNumber of degrees of freedom: %zu (NSE) + %d (T)\n",
              v.n_cells, n_nse, v.n_T);
  // initial values (run(), :1801-1834): u = 0, T = the projected initial field
  std::vector<double> u(n_nse, 0.0), T(size_t(v.n_T), 0.0);
  dcp_host_mesh_initial_temperature(m, T.data());
  for (int f : {DCP_NSE_SOLUTION, DCP_OLD_NSE_SOLUTION})
    if ((rc = dcp_state_set(ctx, f, u.data(), u.size())) != DCP_OK) return fail("state", ctx);
  for (int f : {DCP_T_SOLUTION, DCP_OLD_T_SOLUTION})
    if ((rc = dcp_state_set(ctx, f, T.data(), T.size())) != DCP_OK) return fail("state", ctx);
  Output out;
  Output* outp = nullptr;
  if (!out_dir.empty()) {
    if (two_d) {
      std::fprintf(stderr, "Error: --output writes the 3D models' fields only\n");
      return 1;
    }
    out.ctx = ctx;
    out.view = &v;
    out.feec = feec ? &fm : nullptr;
    out.dir = out_dir;
    out.stem = out_stem;
    out.n_nse = n_nse;
    outp = &out;
    if (write_output(out) != DCP_OK) return fail("output", ctx);  // before the loop (:1840)
  }
  Runner runner;
  runner.ctx = ctx;
  runner.out = outp;
  runner.diagnostics = rp.solver_diagnostics_level;
  runner.interval = rp.physics.nse_solver_interval > 0 ? rp.physics.nse_solver_interval : 1;
  if (runner.diagnostics >= 2) dcp_set_option(ctx, DCP_OPT_LOG_HISTORY, 1);
  dcp_run_report rep{};
  rc = dcp_run(ctx, &rp, max_steps, print_step, &runner, &rep);
  if (rc < 0) return fail("run", ctx);
  dcp_timings t{};
  dcp_get_timings(ctx, &t);
  std::printf("----------------------------------------\n");
  std::printf("%d steps to t=%g: %ld outer / %ld inner NSE iterations, %ld T CG iterations%s\n",
              rep.steps, rep.time_index, rep.total_outer, rep.total_inner, rep.total_T_cg,
              rc == DCP_NOT_CONVERGED ? " (NSE solve did not converge)" : "");
  std::printf("last step (device ms): assemble NSE %.3f | NSE precond %.3f | T matrix %.3f | "
              "T rhs %.3f | NSE solve %.1f | T solve %.3f\n",
              t.assemble_nse_ms, t.build_precond_ms, t.assemble_T_matrix_ms, t.assemble_T_rhs_ms,
              t.solve_nse_ms, t.solve_T_ms);
  dcp_ctx_destroy(ctx);
  dcp_host_mesh_destroy(m);
  return rc == DCP_OK ? 0 : 2;
}
