// The two-dimensional model, Standard::BoussinesqModel<2>
// (boussinesq_model.inst.cc:8; data/aqua_planet_test_2d.prm, BASELINE config
// C1), on the device: the upload of what setup_dofs() produces and the
// per-step members that differ from the 3D ones (assembly, preconditioner
// diagonals, temperature matrices and rhs, constraint distribute, exports).
// The solvers (solver.cpp) and the temperature CG are shared; the 2D
// nse_matrix [u | p] is one scalar CSR whose blocks are row/column windows.
#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "context.h"

namespace dcp {
namespace {

[[noreturn]] void fail2d(int code, const std::string& msg) { throw ApiError{code, msg}; }
void need(bool ok, int code, const std::string& msg) {
  if (!ok) fail2d(code, msg);
}

// FESystem(FE_Q(2)^2, FE_Q(1)) local dof -> component (0, 1 velocity, 2 pressure)
inline int comp2d(int i) { return i < 12 ? i % 3 : i < 20 ? (i - 12) % 2 : i - 20; }

struct Prep2D {
  int tdpc = 4;
  std::vector<int32_t> dofs, tdofs;
  std::vector<int8_t> src;
  std::vector<double> srcw;
  std::vector<uint8_t> fixed;
  std::vector<int32_t> ptr, col, Tp, Tc;
  std::vector<uint8_t> Tfix;
  std::vector<double> Tbc;
  std::vector<int> color_ptr;
  std::vector<int32_t> ccells;
  std::vector<int32_t> ldof, lptr, lent;
  std::vector<double> lw, linh;
};

void sort_unique(std::vector<int32_t>& v) {
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
}

void to_csr(std::vector<std::vector<int32_t>>& rows, std::vector<int32_t>& ptr,
            std::vector<int32_t>& col) {
  ptr.assign(rows.size() + 1, 0);
  for (size_t r = 0; r < rows.size(); ++r) {
    sort_unique(rows[r]);
    ptr[r + 1] = ptr[r] + int32_t(rows[r].size());
  }
  col.clear();
  col.reserve(size_t(ptr.back()));
  for (const auto& r : rows) col.insert(col.end(), r.begin(), r.end());
}

// Validation, the per-cell condensation table, patterns
// (make_sparsity_pattern with the constraints, keep_constrained_dofs = false:
// boussinesq_model.tpp:79-112 / 153-180) and the colouring.
void prepare2d(const dcp_mesh2d* m, Prep2D& h) {
  need(m != nullptr, DCP_ERR_INVALID, "NULL mesh");
  need(m->cell_nse_dofs && m->cell_T_dofs && m->cell_geometry && m->cell_diameter, DCP_ERR_INVALID,
       "NULL array");
  const int nc = m->n_cells, nu = m->n_u, np = m->n_p, nT = m->n_T, n = nu + np;
  need(nc > 0 && nu > 0 && np > 0 && nT > 0, DCP_ERR_INVALID, "empty 2D mesh");
  need(m->temperature_degree == 1 || m->temperature_degree == 2, DCP_ERR_UNSUPPORTED,
       "2D temperature degree must be 1 or 2");
  const int tdpc = m->temperature_degree == 1 ? 4 : 9;
  h.tdpc = tdpc;
  h.dofs.assign(m->cell_nse_dofs, m->cell_nse_dofs + size_t(nc) * 22);
  h.tdofs.assign(m->cell_T_dofs, m->cell_T_dofs + size_t(nc) * tdpc);
  for (int c = 0; c < nc; ++c) {
    for (int i = 0; i < 22; ++i) {
      const int d = h.dofs[22 * size_t(c) + i];
      if (comp2d(i) < 2) need(d >= 0 && d < nu, DCP_ERR_INVALID, "velocity dof out of range");
      else need(d >= nu && d < n, DCP_ERR_INVALID, "pressure dof out of range");
    }
    for (int i = 0; i < tdpc; ++i) {
      const int d = h.tdofs[size_t(tdpc) * c + i];
      need(d >= 0 && d < nT, DCP_ERR_INVALID, "temperature dof out of range");
    }
    need(m->cell_diameter[c] > 0, DCP_ERR_INVALID, "non-positive cell diameter");
  }
  // ---- NSE constraints: node-local, homogeneous
  std::vector<int32_t> line_of(n, -1);
  const dcp_constraints& C = m->nse;
  need(C.n_lines == 0 || (C.line_dof && C.entry_ptr && C.inhomogeneity), DCP_ERR_INVALID,
       "NULL constraint array");
  for (int l = 0; l < C.n_lines; ++l) {
    const int d = C.line_dof[l];
    need(d >= 0 && d < n, DCP_ERR_INVALID, "constrained dof out of range");
    need(line_of[d] < 0, DCP_ERR_INVALID, "dof constrained twice");
    line_of[d] = l;
  }
  h.lptr.assign(1, 0);
  for (int l = 0; l < C.n_lines; ++l) {
    const int ne = C.entry_ptr[l + 1] - C.entry_ptr[l];
    need(ne <= 1, DCP_ERR_UNSUPPORTED, "2D constraint lines with more than one entry");
    need(C.inhomogeneity[l] == 0.0, DCP_ERR_UNSUPPORTED, "inhomogeneous NSE constraints");
    for (int k = C.entry_ptr[l]; k < C.entry_ptr[l + 1]; ++k) {
      const int t = C.entry_dof[k];
      need(t >= 0 && t < n && line_of[t] < 0, DCP_ERR_UNSUPPORTED,
           "constraint entries must be unconstrained dofs (closed constraints)");
      h.lent.push_back(t);
      h.lw.push_back(C.entry_w[k]);
    }
    h.ldof.push_back(C.line_dof[l]);
    h.linh.push_back(0.0);
    h.lptr.push_back(int32_t(h.lent.size()));
  }
  // ---- per cell: constrained flags and the source of every local dof
  h.fixed.assign(size_t(nc) * 22, 0);
  h.src.assign(size_t(nc) * 22, int8_t(-1));
  h.srcw.assign(size_t(nc) * 22, 0.0);
  for (int c = 0; c < nc; ++c) {
    const int32_t* d = &h.dofs[22 * size_t(c)];
    for (int i = 0; i < 22; ++i) {
      const int l = line_of[d[i]];
      if (l < 0) continue;
      h.fixed[22 * size_t(c) + i] = 1;
      if (C.entry_ptr[l + 1] == C.entry_ptr[l]) continue;
      const int t = C.entry_dof[C.entry_ptr[l]];
      int j = -1;
      for (int k = 0; k < 22; ++k)
        if (d[k] == t) j = k;
      need(j >= 0, DCP_ERR_UNSUPPORTED, "constraint target outside the cell (not node-local)");
      need(h.src[22 * size_t(c) + j] < 0, DCP_ERR_UNSUPPORTED,
           "a dof receives two constraint lines in one cell");
      h.src[22 * size_t(c) + j] = int8_t(i);
      h.srcw[22 * size_t(c) + j] = C.entry_w[C.entry_ptr[l]];
    }
  }
  // ---- NSE pattern: everything but p-p, expanded through the constraints
  {
    std::vector<std::vector<int32_t>> rows(n);
    for (int c = 0; c < nc; ++c) {
      const int32_t* d = &h.dofs[22 * size_t(c)];
      int ex[22];
      for (int i = 0; i < 22; ++i) {
        const int l = line_of[d[i]];
        ex[i] = l < 0 ? d[i] : C.entry_ptr[l + 1] > C.entry_ptr[l] ? C.entry_dof[C.entry_ptr[l]] : -1;
      }
      for (int i = 0; i < 22; ++i) {
        if (ex[i] < 0) continue;
        for (int j = 0; j < 22; ++j)
          if (ex[j] >= 0 && !(comp2d(i) == 2 && comp2d(j) == 2)) rows[ex[i]].push_back(ex[j]);
      }
    }
    for (int r = 0; r < n; ++r)
      if (line_of[r] >= 0) rows[r].push_back(r);
    to_csr(rows, h.ptr, h.col);
  }
  // ---- temperature: Dirichlet lines; full coupling, constrained rows/columns diagonal only
  h.Tfix.assign(nT, 0);
  h.Tbc.assign(nT, 0.0);
  const dcp_constraints& TC = m->T;
  for (int l = 0; l < TC.n_lines; ++l) {
    const int d = TC.line_dof[l];
    need(d >= 0 && d < nT, DCP_ERR_INVALID, "temperature constraint out of range");
    need(TC.entry_ptr[l] == TC.entry_ptr[l + 1], DCP_ERR_UNSUPPORTED,
         "temperature constraints must be Dirichlet lines");
    h.Tfix[d] = 1;
    h.Tbc[d] = TC.inhomogeneity[l];
  }
  {
    std::vector<std::vector<int32_t>> rows(nT);
    for (int c = 0; c < nc; ++c) {
      const int32_t* t = &h.tdofs[size_t(tdpc) * c];
      for (int i = 0; i < tdpc; ++i) {
        if (h.Tfix[t[i]]) continue;
        for (int j = 0; j < tdpc; ++j)
          if (!h.Tfix[t[j]]) rows[t[i]].push_back(t[j]);
      }
    }
    for (int r = 0; r < nT; ++r)
      if (h.Tfix[r]) rows[r].push_back(r);
    to_csr(rows, h.Tp, h.Tc);
  }
  // ---- colouring: cells sharing a support point share a vertex = a pressure dof
  {
    std::vector<std::vector<int32_t>> vcells(np);
    const int pl[4] = {2, 5, 8, 11};
    for (int c = 0; c < nc; ++c)
      for (int v : pl) vcells[h.dofs[22 * size_t(c) + v] - nu].push_back(c);
    std::vector<int> color(nc, -1);
    int n_colors = 0;
    for (int c = 0; c < nc; ++c) {
      uint64_t used = 0;
      for (int v : pl)
        for (int o : vcells[h.dofs[22 * size_t(c) + v] - nu])
          if (color[o] >= 0) used |= uint64_t(1) << color[o];
      int k = 0;
      while (k < 64 && ((used >> k) & 1)) ++k;
      need(k < 64, DCP_ERR_UNSUPPORTED, "cell colouring needs more than 64 colours");
      color[c] = k;
      n_colors = std::max(n_colors, k + 1);
    }
    // the temperature dofs must be covered by the same colouring: every T dof
    // of a cell is one of its support points, so it suffices that no two cells
    // of a colour share one (checked)
    std::vector<int> seen(nT, -1);
    h.color_ptr.assign(n_colors + 1, 0);
    for (int c = 0; c < nc; ++c) h.color_ptr[color[c] + 1]++;
    for (int k = 0; k < n_colors; ++k) h.color_ptr[k + 1] += h.color_ptr[k];
    h.ccells.assign(nc, 0);
    std::vector<int> f(h.color_ptr.begin(), h.color_ptr.end() - 1);
    for (int c = 0; c < nc; ++c) h.ccells[f[color[c]]++] = c;
    for (int k = 0; k < n_colors; ++k)
      for (int e = h.color_ptr[k]; e < h.color_ptr[k + 1]; ++e) {
        const int c = h.ccells[e];
        for (int i = 0; i < tdpc; ++i) {
          int& s = seen[h.tdofs[size_t(tdpc) * c + i]];
          need(s != k, DCP_ERR_UNSUPPORTED, "temperature dofs shared across a vertex colour");
          s = k;
        }
      }
  }
}

}  // namespace

void mesh2d_check(const dcp_mesh2d* m, int* n_colors) {
  Prep2D h;
  prepare2d(m, h);
  if (n_colors) *n_colors = int(h.color_ptr.size()) - 1;
}

void mesh2d_upload(Ctx& c, const dcp_mesh2d* m) {
  // several GPUs: m is the rank's local mesh (localize_2d) and the caller
  // (dcp_mesh2d_upload) then sets the owned sizes, global ids and halos
  Prep2D h;
  prepare2d(m, h);
  DCP_HIP_CHECK(hipSetDevice(c.cfg.device));
  const int nc = m->n_cells, nu = m->n_u, np = m->n_p, nT = m->n_T, n = nu + np;
  c.have_mesh = false;
  c.feec = false;
  c.dim2 = true;
  c.vdim = 2;
  c.periodic = false;
  c.schur_explicit = false;  // S = B D_A^-1 B^T applied as three products
  c.m2_tdpc = h.tdpc;
  c.n_cells = c.n_owned_cells = nc;
  c.n_u = nu;
  c.n_p = np;
  c.n_T = nT;
  c.n_vnodes = nu / 2;
  c.n_u_g = nu;
  c.n_p_g = np;
  c.n_T_g = nT;
  c.nvo = nu / 2;
  c.npo = np;
  c.nTo = nT;
  c.vnode_g.clear();
  c.p_g.clear();
  c.T_g.clear();
  c.color_ptr = h.color_ptr;
  c.color_cells.upload(h.ccells);
  c.m2_dofs.upload(h.dofs);
  c.m2_tdofs.upload(h.tdofs);
  c.m2_X.upload(std::vector<double>(m->cell_geometry, m->cell_geometry + size_t(nc) * 32));
  c.diameter.upload(std::vector<double>(m->cell_diameter, m->cell_diameter + nc));
  c.m2_src.upload(h.src);
  c.m2_srcw.upload(h.srcw);
  c.m2_fixed.upload(h.fixed);
  c.m2_ptr.upload(h.ptr);
  c.m2_col.upload(h.col);
  c.m2_val.alloc(h.col.size());
  c.m2_pos.alloc(size_t(nc) * 484);
  positions_2d(nc, 22, c.m2_dofs.p, c.m2_ptr.p, c.m2_col.p, c.m2_pos.p, c.stream);
  c.m2_nlines = int(h.ldof.size());
  c.m2_ldof.upload(h.ldof);
  c.m2_lptr.upload(h.lptr);
  c.m2_lent.upload(h.lent);
  c.m2_lw.upload(h.lw);
  c.m2_linh.upload(h.linh);
  c.T_fixed.upload(h.Tfix);
  c.T_bc.upload(h.Tbc);
  c.T_ptr.upload(h.Tp);
  c.T_col.upload(h.Tc);
  c.Tmass.alloc(h.Tc.size());
  c.Tstiff.alloc(h.Tc.size());
  c.Tmat.alloc(h.Tc.size());
  c.m2_posT.alloc(size_t(nc) * h.tdpc * h.tdpc);
  positions_2d(nc, h.tdpc, c.m2_tdofs.p, c.T_ptr.p, c.T_col.p, c.m2_posT.p, c.stream);
  c.nse_sol.alloc(n);
  c.old_nse.alloc(n);
  c.nse_rhs.alloc(n);
  c.T_sol.alloc(nT);
  c.old_T.alloc(nT);
  c.T_rhs.alloc(nT);
  for (auto* b : {&c.nse_sol, &c.old_nse, &c.nse_rhs, &c.T_sol, &c.old_T, &c.T_rhs}) b->zero(c.stream);
  c.A_diag.alloc(nu);
  c.Mp_diag.alloc(np);
  c.A_inv.alloc(nu);
  c.Mp_inv.alloc(np);
  c.T_inv.alloc(nT);
  c.schur_tmp1.alloc(nu);
  c.schur_tmp2.alloc(nu);
  c.utmp.alloc(nu);
  c.fg_aux.alloc(n);
  free_workspaces(c);
  c.max_owned[0] = n;
  c.max_owned[1] = np;
  c.max_owned[2] = nu;
  c.max_owned[3] = nT;
  DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
  c.have_mesh = true;
  c.nse_assembled = c.precond_built = c.T_matrix_ok = c.T_rhs_ok = false;
}

void assemble_nse_2d(Ctx& c, int flags) {
  // assemble_nse_system (boussinesq_model.tpp:691-740) at dim = 2
  const bool matrix = (flags & DCP_ASSEMBLE_MATRIX) != 0;
  if (matrix) c.m2_val.zero(c.stream);
  if (flags & DCP_ASSEMBLE_RHS) c.nse_rhs.zero(c.stream);
  const Mesh2DDev md = c.m2();
  for (int k = 0; k < c.n_colors(); ++k)
    launch2d_nse_system(md, c.color_begin(k), c.color_size(k), c.old_nse.p, c.old_T.p, c.ph,
                        matrix ? c.m2_val.p : nullptr,
                        (flags & DCP_ASSEMBLE_RHS) ? c.nse_rhs.p : nullptr, c.stream);
  if (matrix) {
    c.nse_assembled = true;
    c.nse_ph = c.ph;
  }
}

void build_precond_2d(Ctx& c) {
  // assemble_nse_preconditioner + build_nse_preconditioner (:479-542): the
  // point-Jacobi diagonals of P(0,0) and P(1,1)
  c.A_diag.zero(c.stream);
  c.Mp_diag.zero(c.stream);
  const Mesh2DDev md = c.m2();
  for (int k = 0; k < c.n_colors(); ++k)
    launch2d_precond_diag(md, c.color_begin(k), c.color_size(k), c.ph, c.A_diag.p, c.Mp_diag.p,
                          c.stream);
  reciprocal(c.n_u, c.A_diag.p, c.A_inv.p, c.stream);
  reciprocal(c.n_p, c.Mp_diag.p, c.Mp_inv.p, c.stream);
}

void assemble_T_matrix_2d(Ctx& c) {
  c.Tmass.zero(c.stream);
  c.Tstiff.zero(c.stream);
  const Mesh2DDev md = c.m2();
  for (int k = 0; k < c.n_colors(); ++k)
    launch2d_T_matrix(md, c.color_begin(k), c.color_size(k), c.ph, c.Tmass.p, c.Tstiff.p, c.stream);
}

void assemble_T_rhs_2d(Ctx& c) {
  const Mesh2DDev md = c.m2();
  for (int k = 0; k < c.n_colors(); ++k)
    launch2d_T_rhs(md, c.color_begin(k), c.color_size(k), c.old_T.p, c.nse_sol.p, c.ph, c.T_rhs.p,
                   c.stream);
}

void distribute_nse_2d(Ctx& c, double* x) {
  distribute_2d(c.m2_nlines, c.m2_ldof.p, c.m2_lptr.p, c.m2_lent.p, c.m2_lw.p, c.m2_linh.p, x,
                c.stream);
}

void nse_matrix_export_2d(Ctx& c, int64_t* nnz, int32_t* rowptr, int32_t* cols, double* vals) {
  const int n = c.n_u + c.n_p;
  *nnz = int64_t(c.m2_col.n);
  if (!rowptr) return;
  need(cols && vals, DCP_ERR_INVALID, "NULL cols/vals");
  need(c.nse_assembled, DCP_ERR_STATE, "nse_matrix not assembled");
  DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
  DCP_HIP_CHECK(hipMemcpy(rowptr, c.m2_ptr.p, size_t(n + 1) * sizeof(int32_t), hipMemcpyDeviceToHost));
  DCP_HIP_CHECK(hipMemcpy(cols, c.m2_col.p, c.m2_col.n * sizeof(int32_t), hipMemcpyDeviceToHost));
  DCP_HIP_CHECK(hipMemcpy(vals, c.m2_val.p, c.m2_val.n * sizeof(double), hipMemcpyDeviceToHost));
}

void cell_nse_system_2d(Ctx& c, int first, int n, double* K, double* f) {
  DBuf<double> dK, df;
  dK.alloc(size_t(n) * 484);
  df.alloc(size_t(n) * 22);
  launch2d_nse_elements(c.m2(), first, n, c.old_nse.p, c.old_T.p, c.ph, dK.p, df.p, c.stream);
  DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
  DCP_HIP_CHECK(hipMemcpy(K, dK.p, dK.n * sizeof(double), hipMemcpyDeviceToHost));
  DCP_HIP_CHECK(hipMemcpy(f, df.p, df.n * sizeof(double), hipMemcpyDeviceToHost));
}

}  // namespace dcp
