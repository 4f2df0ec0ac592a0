// C ABI implementation (include/dcp.h): context management, the one-off
// mesh/DoF upload (patterns, colouring, scatter maps) and the hot-path calls.
#include <algorithm>
#include <queue>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <numeric>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/dcp.h"
#include "context.h"
#include "fe_tables.h"
#include "mesh.h"
#include "mesh2d.h"
#include "partition.h"
#include "prm.h"
#include "renumber.h"

using namespace dcp;

struct dcp_ctx : Ctx {};
struct dcp_group : dcp::LocalGroup {
  explicit dcp_group(int n) : dcp::LocalGroup(n) {}
};

namespace dcp {
Ctx::~Ctx() {
  free_workspaces(*this);
  if (hpinned) (void)hipHostFree(hpinned);
  if (hmapped) (void)hipHostFree(hmapped);
  if (gm_report) (void)hipHostFree(gm_report);
  for (auto& ev : gm_ev)
    if (ev) (void)hipEventDestroy(ev);
  ev_total.destroy();
  for (auto& t : schur_ev) t.destroy();
  for (auto& v : mf_ev)
    for (auto& t : v) t.destroy();
  for (auto& ev : mf_chunk_ev)
    if (ev) (void)hipEventDestroy(ev);
  if (mf_join_ev) (void)hipEventDestroy(mf_join_ev);
  if (mf_stream) (void)hipStreamDestroy(mf_stream);
  if (stream) (void)hipStreamDestroy(stream);
}
}  // namespace dcp

namespace {

thread_local std::string g_last_error;

template <class F>
int guarded(dcp_ctx* ctx, F&& f) {
  try {
    const int rc = f();
    // a device-side collective that timed out (PeerComm) fails the call that
    // observes it, not a later one (host-mapped flag; work still in flight is
    // caught by the next call)
    if (ctx && ctx->comm) ctx->comm->check();
    return rc;
  } catch (const ApiError& e) {
    if (ctx) ctx->err = e.msg;
    g_last_error = e.msg;
    return e.code;
  } catch (const DeviceError& e) {
    std::string m = std::string("HIP error ") + hipGetErrorString(e.code) + " in " + e.what_expr +
                    " (" + e.file + ":" + std::to_string(e.line) + ")";
    if (ctx) ctx->err = m;
    g_last_error = m;
    return DCP_ERR_DEVICE;
  } catch (const std::exception& e) {
    if (ctx) ctx->err = e.what();
    g_last_error = e.what();
    return DCP_ERR_INVALID;
  }
}

[[noreturn]] void fail(int code, const std::string& msg) { throw ApiError{code, msg}; }

void require(bool ok, int code, const std::string& msg) {
  if (!ok) fail(code, msg);
}

// Sorted, de-duplicated union pattern: row r collects the `cols` entries of
// every cell in which r appears among the `rows` entries.
void union_pattern(int n_rows, int n_cells, const int32_t* rows, int kr, const int32_t* cols, int kc,
                   std::vector<int32_t>& ptr, std::vector<int32_t>& col) {
  std::vector<int64_t> cnt(size_t(n_rows) + 1, 0);
  for (size_t i = 0; i < size_t(n_cells) * kr; ++i) cnt[rows[i] + 1] += kc;
  for (int r = 0; r < n_rows; ++r) cnt[r + 1] += cnt[r];
  std::vector<int32_t> tmp(static_cast<size_t>(cnt[n_rows]));
  std::vector<int64_t> fillp(cnt.begin(), cnt.end() - 1);
  for (int c = 0; c < n_cells; ++c)
    for (int a = 0; a < kr; ++a) {
      const int r = rows[size_t(c) * kr + a];
      std::memcpy(&tmp[fillp[r]], &cols[size_t(c) * kc], kc * sizeof(int32_t));
      fillp[r] += kc;
    }
  ptr.assign(size_t(n_rows) + 1, 0);
  std::vector<int32_t> len(n_rows);
#pragma omp parallel for schedule(dynamic, 1024)
  for (int r = 0; r < n_rows; ++r) {
    auto b = tmp.begin() + cnt[r], e = tmp.begin() + cnt[r + 1];
    std::sort(b, e);
    len[r] = int32_t(std::unique(b, e) - b);
  }
  for (int r = 0; r < n_rows; ++r) ptr[r + 1] = ptr[r] + len[r];
  col.resize(size_t(ptr[n_rows]));
#pragma omp parallel for schedule(dynamic, 1024)
  for (int r = 0; r < n_rows; ++r)
    std::copy(tmp.begin() + cnt[r], tmp.begin() + cnt[r] + len[r], col.begin() + ptr[r]);
}

void set_physics_dev(Ctx& c) {
  const dcp_physics& p = c.hph;
  c.ph.dt = p.time_step;
  c.ph.nu_sys = p.time_step * p.one_over_reynolds;
  c.ph.nu_pre = p.time_step * p.one_over_reynolds;
  c.ph.beta = p.expansion_coefficient;
  c.ph.T_ref = p.temperature_ref;
  c.ph.grav_scale = p.gravity_scale;
  c.ph.g = p.gravity_constant;
  c.ph.coriolis_z = p.cuboid ? p.coriolis_scale * p.omega : 0.0;
  c.ph.one_over_peclet = p.one_over_peclet;
  c.ph.dt_T = p.time_step / p.nse_solver_interval;
  c.ph.cuboid = p.cuboid;
}

// write = true: the caller changes the field, so an old field's ghost entries
// are no longer known to be current (reads leave the flags alone)
double* field_ptr(Ctx& c, int field, size_t& n, bool write) {
  if (write && field == DCP_OLD_NSE_SOLUTION) c.old_nse_ghosted = false;
  if (write && field == DCP_OLD_T_SOLUTION) c.old_T_ghosted = false;
  switch (field) {
    case DCP_NSE_SOLUTION: n = size_t(c.n_u + c.n_p); return c.nse_sol.p;
    case DCP_OLD_NSE_SOLUTION: n = size_t(c.n_u + c.n_p); return c.old_nse.p;
    case DCP_T_SOLUTION: n = size_t(c.n_T); return c.T_sol.p;
    case DCP_OLD_T_SOLUTION: n = size_t(c.n_T); return c.old_T.p;
    case DCP_NSE_RHS: n = size_t(c.n_u + c.n_p); return c.nse_rhs.p;
    case DCP_T_RHS: n = size_t(c.n_T); return c.T_rhs.p;
    default: fail(DCP_ERR_INVALID, "unknown state field " + std::to_string(field));
  }
}

// the ghost entries of an old field were just made current (see Ctx)
void mark_old_ghosted(Ctx& c, int field) {
  if (c.old_external) return;
  if (field == DCP_OLD_NSE_SOLUTION) c.old_nse_ghosted = true;
  if (field == DCP_OLD_T_SOLUTION) c.old_T_ghosted = true;
}

struct PhaseTimer {
  Ctx& c;
  double* out;
  explicit PhaseTimer(Ctx& ctx, double* o) : c(ctx), out(o) {
    DCP_HIP_CHECK(hipEventRecord(c.ev_total.a, c.stream));
  }
  void stop() {
    DCP_HIP_CHECK(hipEventRecord(c.ev_total.b, c.stream));
    DCP_HIP_CHECK(hipEventSynchronize(c.ev_total.b));
    float ms = 0;
    DCP_HIP_CHECK(hipEventElapsedTime(&ms, c.ev_total.a, c.ev_total.b));
    *out = ms;
  }
};

// get_maximal_velocity / get_cfl_number over the owned cells (+ MPI max)
void velocity_stats_global(Ctx& c) {
  halo_exchange(c, c.halo_nse, c.nse_sol.p);
  if (c.feec)
    feec_velocity_stats(c.fcd(), c.n_owned_cells, c.nse_sol.p, c.dscal.p + 262, c.stream);
  else if (c.dim2)
    velocity_stats_2d(c.m2(), c.nse_sol.p, c.dscal.p + 262, c.stream);
  else
    velocity_stats(c.cd(), c.n_owned_cells, c.nse_sol.p, c.dscal.p + 262, c.stream);
  allreduce(c, c.dscal.p + 262, 2, true);
  DCP_HIP_CHECK(hipMemcpyAsync(c.hpinned, c.dscal.p + 262, 2 * sizeof(double),
                               hipMemcpyDeviceToHost, c.stream));
  DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
}

void need_ready(Ctx& c) {
  require(c.have_physics, DCP_ERR_STATE, "dcp_set_physics has not been called");
  require(c.have_mesh, DCP_ERR_STATE, "dcp_mesh_upload has not been called");
  const int mesh_deg = c.dim2 ? (c.m2_tdpc == 9 ? 2 : 1) : (c.tdpc3 == 27 ? 2 : 1);
  require(!c.feec || c.hph.temperature_degree == 1, DCP_ERR_UNSUPPORTED,
          "the FEEC device temperature path implements FE_Q(1)");
  require(c.feec || c.hph.temperature_degree == mesh_deg, DCP_ERR_INVALID,
          "physics temperature degree differs from the uploaded mesh's");
}

struct HostPrep {
  int nv = 0;
  int tdpc = 8;  // temperature dofs per cell: 8 (FE_Q(1)) or 27 (FE_Q(2), stored lexicographic)
  std::vector<int32_t> q2, pd, td;
  std::vector<double> geo;  // [n_cells][64][3] MappingQ(3) support points
  std::vector<NodeConstraint> vc;
  std::vector<uint8_t> Tfix;
  std::vector<double> Tbc;
  std::vector<int> color_ptr;
  std::vector<int32_t> ccells;
  std::vector<int32_t> Ap, Ac, Btp, Btc, Bp, Bc, Tp, Tc, Sp, Sc;
  int S_max_row = 0;
  // periodic identification (DoFTools::make_periodicity_constraints): a dof
  // whose closed constraint line is "= its partner" is replaced by the partner
  // in the cell maps; the original maps (empty when nothing is identified)
  // route the constrained-diagonal entries to the identified dof itself
  std::vector<int32_t> q2o, pdo, tdo;
  std::vector<int32_t> vmaster, pmaster, tmaster;  // -1 or the partner
  int n_vslave = 0, n_pslave = 0, n_tslave = 0;
};

// Eight colours on the hyper_shell (the greedy colouring of the tree order
// needs 14 at refine 5, 6 of them small launches holding 2.3 % of the cells:
// latency the colour launches pay six times). The shell is columns x radial
// layers, the columns the cubed sphere's 6 patches of 2^r x 2^r quads; a
// vertex-sharing colouring is (layer parity) x a lateral 4-colouring. On each
// patch the lateral colour is a function of the quad's index parities
// (p_b, p_c) along the patch's two tangential cube axes b, c (found by a
// breadth-first walk from the patch's corner quad). The three ways of
// splitting 4 colours into two pairs are tied to the three cube axes (split
// pi_x: L & 1, pi_y: L >> 1, pi_z: the xor of both): the quads along a patch
// edge parallel to axis b then use one pair of pi_b and the quads across it
// the other pair, which holds on every edge and corner for one choice of the
// 12 per-patch parity offsets (searched). Anything else (cube, partitions,
// other manifolds) fails one of the checks and keeps the greedy colouring;
// the result is checked against every vertex-sharing pair before use.
bool shell_colouring(int n_cells, const double* geo, const std::vector<int32_t>& pd,
                     const std::vector<int32_t>& vptr, const std::vector<int32_t>& vcells,
                     std::vector<int>& color) {
  constexpr int kP = 64;
  const int corner[4] = {0, 3, 12, 15};  // lateral corners of the inner face
  std::map<std::array<long long, 3>, int> vkey;
  std::vector<std::array<int, 4>> cv(n_cells);
  std::vector<double> rad(n_cells);
  std::vector<std::array<double, 3>> cdir(n_cells);
  for (int c = 0; c < n_cells; ++c) {
    std::array<double, 3> cen{0, 0, 0};
    for (int k = 0; k < 4; ++k) {
      const double* X = geo + (size_t(c) * kP + corner[k]) * 3;
      const double r = std::sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
      if (!(r > 0)) return false;
      if (k == 0) rad[c] = r;
      std::array<long long, 3> key;
      for (int d = 0; d < 3; ++d) {
        key[d] = std::llround(X[d] / r * 1e9);
        cen[d] += X[d] / r;
      }
      cv[c][k] = vkey.emplace(key, int(vkey.size())).first->second;
    }
    cdir[c] = cen;
    std::sort(cv[c].begin(), cv[c].end());
  }
  std::map<std::array<int, 4>, int> ckey;
  std::vector<int> col(n_cells);
  std::vector<std::array<int, 4>> ccv;
  std::vector<std::array<double, 3>> cen;
  for (int c = 0; c < n_cells; ++c) {
    auto it = ckey.emplace(cv[c], int(ccv.size()));
    if (it.second) {
      ccv.push_back(cv[c]);
      cen.push_back(cdir[c]);
    }
    col[c] = it.first->second;
  }
  const int ncol = int(ccv.size());
  // layer parity: rank of the inner radius among the distinct ones
  std::vector<double> ur(rad);
  std::sort(ur.begin(), ur.end());
  std::vector<double> lev;
  for (double r : ur)
    if (lev.empty() || r > lev.back() * (1 + 1e-10)) lev.push_back(r);
  std::vector<int> lpar(n_cells);
  for (int c = 0; c < n_cells; ++c) {
    const auto it = std::lower_bound(lev.begin(), lev.end(), rad[c] * (1 - 1e-10));
    if (it == lev.end()) return false;
    lpar[c] = int(it - lev.begin()) & 1;
  }
  // patch (face) of a column and its tangential axes
  std::vector<int> face(ncol);
  for (int k = 0; k < ncol; ++k) {
    int a = 0;
    for (int d = 1; d < 3; ++d)
      if (std::fabs(cen[k][d]) > std::fabs(cen[k][a])) a = d;
    face[k] = 2 * a + (cen[k][a] > 0);
  }
  // columns sharing an edge (two corner vertices) / a vertex
  std::map<std::pair<int, int>, std::vector<int>> ecols;
  std::vector<std::vector<int>> vcols(vkey.size());
  for (int k = 0; k < ncol; ++k)
    for (int i = 0; i < 4; ++i) {
      vcols[ccv[k][i]].push_back(k);
      for (int j = i + 1; j < 4; ++j) ecols[{ccv[k][i], ccv[k][j]}].push_back(k);
    }
  std::vector<std::vector<int>> eadj(ncol);
  for (const auto& e : ecols)
    if (e.second.size() == 2) {
      eadj[e.second[0]].push_back(e.second[1]);
      eadj[e.second[1]].push_back(e.second[0]);
    }
  // index parities along the tangential cube axes, walking each patch from
  // its corner quad (smallest gnomonic coordinates)
  std::vector<std::array<int, 3>> par(ncol, {-1, -1, -1});
  for (int f = 0; f < 6; ++f) {
    const int a = f / 2, t0 = a == 0 ? 1 : 0, t1 = a == 2 ? 1 : 2;
    int anchor = -1, count = 0;
    double best = 0;
    for (int k = 0; k < ncol; ++k) {
      if (face[k] != f) continue;
      ++count;
      const double g = (cen[k][t0] + cen[k][t1]) / std::fabs(cen[k][a]);
      if (anchor < 0 || g < best) {
        anchor = k;
        best = g;
      }
    }
    if (anchor < 0) return false;
    par[anchor][t0] = par[anchor][t1] = 0;
    std::deque<int> q{anchor};
    int seen = 1;
    while (!q.empty()) {
      const int x = q.front();
      q.pop_front();
      for (int y : eadj[x]) {
        if (face[y] != f || par[y][t0] >= 0) continue;
        const double d0 = cen[y][t0] / std::fabs(cen[y][a]) - cen[x][t0] / std::fabs(cen[x][a]);
        const double d1 = cen[y][t1] / std::fabs(cen[y][a]) - cen[x][t1] / std::fabs(cen[x][a]);
        par[y] = par[x];
        par[y][std::fabs(d0) > std::fabs(d1) ? t0 : t1] ^= 1;
        ++seen;
        q.push_back(y);
      }
    }
    if (seen != count) return false;
  }
  auto split = [](int axis, int L) { return axis == 0 ? (L & 1) : axis == 1 ? ((L >> 1) & 1) : ((L ^ (L >> 1)) & 1); };
  std::vector<int> lab(ncol);
  bool found = false;
  for (int offs = 0; offs < 4096 && !found; ++offs) {
    bool ok = true;
    for (int k = 0; k < ncol && ok; ++k) {
      const int f = face[k], a = f / 2, b = a == 0 ? 1 : 0, c = a == 2 ? 1 : 2;
      const int o0 = (offs >> (2 * f)) & 1, o1 = (offs >> (2 * f + 1)) & 1;
      lab[k] = -1;
      for (int L = 0; L < 4; ++L)
        if (split(b, L) == (par[k][c] ^ o0) && split(c, L) == (par[k][b] ^ o1)) lab[k] = L;
      ok = lab[k] >= 0;
    }
    if (!ok) return false;
    for (int k = 0; k < ncol && ok; ++k)
      for (int i = 0; i < 4 && ok; ++i)
        for (int o : vcols[ccv[k][i]])
          if (o != k && lab[o] == lab[k]) {
            ok = false;
            break;
          }
    found = ok;
  }
  if (!found) return false;
  std::vector<int> out(n_cells);
  for (int c = 0; c < n_cells; ++c) out[c] = lab[col[c]] + 4 * lpar[c];
  // every pair of cells sharing a vertex differs
  for (int c = 0; c < n_cells; ++c)
    for (int v = 0; v < 8; ++v) {
      const int p = pd[size_t(c) * 8 + v];
      for (int k = vptr[p]; k < vptr[p + 1]; ++k)
        if (vcells[k] != c && out[vcells[k]] == out[c]) return false;
    }
  color.swap(out);
  return true;
}

// The whole mesh's 8-colour shell colouring restricted to a partition's cells
// (localize: local cell -> global cell); empty when the mesh is no shell.
std::vector<int> partition_colour_hint(int n_cells, const int32_t* cell_nse_dofs,
                                       const double* cell_geometry, int n_u, int n_p,
                                       const std::vector<int32_t>& cells_g) {
  std::vector<int32_t> pd(size_t(n_cells) * 8);
  for (int c = 0; c < n_cells; ++c)
    for (int v = 0; v < 8; ++v) {
      const int p = cell_nse_dofs[size_t(c) * 89 + 4 * v + 3] - n_u;
      if (p < 0 || p >= n_p) return {};
      pd[size_t(c) * 8 + v] = p;
    }
  std::vector<int32_t> vptr(size_t(n_p) + 1, 0), vcells(pd.size());
  for (int32_t p : pd) vptr[p + 1]++;
  for (int v = 0; v < n_p; ++v) vptr[v + 1] += vptr[v];
  std::vector<int32_t> f(vptr.begin(), vptr.end() - 1);
  for (int c = 0; c < n_cells; ++c)
    for (int v = 0; v < 8; ++v) vcells[f[pd[size_t(c) * 8 + v]]++] = c;
  std::vector<int> colour;
  if (!shell_colouring(n_cells, cell_geometry, pd, vptr, vcells, colour)) return {};
  std::vector<int> out(cells_g.size());
  for (size_t i = 0; i < cells_g.size(); ++i) out[i] = colour[cells_g[i]];
  return out;
}

// Host half of dcp_mesh_upload: validation, node map, node-local constraints,
// colouring and block patterns (no device access, so it is testable on CPU).
// The fused matrix-free apply's schedule (k_mf_fused):
// the pencil batches keep the two-launch kernel's XCD placement (XCD x works
// its contiguous batch range in order; workgroup id = XCD + 8 k), and every
// gather window is placed at least `lag` ids after the last batch it reads
// records from, so by the time an XCD dispatches it its inputs are usually
// complete and the poll costs one load. Only meshes whose apply runs as one
// chunk of one-wave batches (the default) get a schedule.
void build_mf_fused(Ctx& c, int n_cells, int nv, int n_p, const std::vector<int32_t>& vptr, const std::vector<int32_t>& pptr,
                    const std::vector<int32_t>& vslot, const std::vector<int32_t>& pslot,
                    int32_t pbase) {
  c.mf_fused = false;
  c.mf_ntasks = 0;
  // off by default: measured slower than the two launches;
  // tested on one-GPU shells only, so partitioned and periodic meshes keep the
  // two launches
  const char* env = std::getenv("DCP_MF_FUSED");
  if (!(env && *env == '1') || c.mf_chunks != 1 || kMfGroupCells != 7 || n_cells <= 0 ||
      c.comm || c.periodic)
    return;
  const int n_pen = (n_cells + 6) / 7;
  const int nvw = (nv + 63) / 64, npw = (n_p + 63) / 64, nw = nvw + npw;
  // slot -> batch of the records
  std::vector<int32_t> vb(size_t(vptr[nv]), -1), pb(size_t(pptr[n_p]), -1);
  for (int cell = 0; cell < n_cells; ++cell) {
    for (int t = 0; t < 27; ++t) {
      const int32_t sl = vslot[27 * size_t(cell) + t];
      if (sl >= 0) vb[size_t(sl / 3)] = cell / 7;
    }
    for (int v = 0; v < 8; ++v) pb[size_t(pslot[8 * size_t(cell) + v] - pbase)] = cell / 7;
  }
  // per window its distinct batches
  std::vector<int32_t> dep_ptr(size_t(nw) + 1, 0), dep;
  dep.reserve(size_t(nw) * 24);
  std::vector<int32_t> tmp;
  for (int w = 0; w < nw; ++w) {
    tmp.clear();
    if (w < nvw) {
      const int n0 = 64 * w, n1 = std::min(n0 + 64, nv);
      for (int k = vptr[n0]; k < vptr[n1]; ++k) tmp.push_back(vb[size_t(k)]);
    } else {
      const int j0 = 64 * (w - nvw), j1 = std::min(j0 + 64, n_p);
      for (int k = pptr[j0]; k < pptr[j1]; ++k) tmp.push_back(pb[size_t(k)]);
    }
    std::sort(tmp.begin(), tmp.end());
    tmp.erase(std::unique(tmp.begin(), tmp.end()), tmp.end());
    for (int32_t b : tmp)
      if (b < 0) return;  // a slot no batch writes: no schedule
    dep.insert(dep.end(), tmp.begin(), tmp.end());
    dep_ptr[size_t(w) + 1] = int32_t(dep.size());
  }
  // batch -> dependent windows
  std::vector<int32_t> rptr(size_t(n_pen) + 1, 0), rw(dep.size());
  for (int32_t b : dep) rptr[size_t(b) + 1]++;
  for (int b = 0; b < n_pen; ++b) rptr[b + 1] += rptr[b];
  {
    std::vector<int32_t> f(rptr.begin(), rptr.end() - 1);
    for (int w = 0; w < nw; ++w)
      for (int k = dep_ptr[w]; k < dep_ptr[w + 1]; ++k) rw[size_t(f[size_t(dep[k])]++)] = w;
  }
  // the two-launch kernel's XCD ranges (xcd_block)
  const int q = n_pen >> 3, r = n_pen & 7;
  int start[8], cnt[8], pos[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int x = 0; x < 8; ++x) {
    cnt[x] = q + (x < r ? 1 : 0);
    start[x] = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  }
  const char* env_lag = std::getenv("DCP_MF_FUSED_LAG");
  const long lag = env_lag ? std::atol(env_lag) : 3072;
  std::vector<int32_t> left(static_cast<size_t>(nw));
  for (int w = 0; w < nw; ++w) left[w] = dep_ptr[w + 1] - dep_ptr[w];
  using Ready = std::pair<long, int32_t>;  // (ready id, window)
  std::priority_queue<Ready, std::vector<Ready>, std::greater<Ready>> ready;
  std::vector<int32_t> sched;
  sched.reserve(size_t(n_pen) + size_t(nw) + 64);
  int pen_done = 0, win_done = 0;
  for (long id = 0; pen_done < n_pen || win_done < nw; ++id) {
    const int x = int(id & 7);
    if (!ready.empty() && ready.top().first <= id) {
      sched.push_back((ready.top().second < nvw ? 1 << 30 : 2 << 30) |
                      (ready.top().second < nvw ? ready.top().second : ready.top().second - nvw));
      ready.pop();
      ++win_done;
    } else if (pos[x] < cnt[x]) {
      const int b = start[x] + pos[x]++;
      sched.push_back(b);
      ++pen_done;
      for (int k = rptr[b]; k < rptr[b + 1]; ++k) {
        const int w = rw[size_t(k)];
        if (--left[w] == 0) ready.push({id + lag, w});
      }
    } else if (!ready.empty()) {
      sched.push_back((ready.top().second < nvw ? 1 << 30 : 2 << 30) |
                      (ready.top().second < nvw ? ready.top().second : ready.top().second - nvw));
      ready.pop();
      ++win_done;
    } else {
      sched.push_back(3 << 30);  // padding: this XCD's batches are out, no window ready
    }
  }
  c.mf_sched.upload(sched);
  c.mf_dep_ptr.upload(dep_ptr);
  c.mf_dep.upload(dep);
  c.mf_done.alloc(size_t(n_pen));
  c.mf_done.zero(c.stream);
  c.mf_seq = 0;
  c.mf_ntasks = int(sched.size());
  c.mf_nvwin = nvw;
  c.mf_fused = true;
}

void prepare_mesh(HostPrep& h, int n_cells, const int32_t* cell_nse_dofs,
                  const int32_t* cell_T_dofs, const double* cell_geometry,
                  const double* cell_diameter, int n_u, int n_p, int n_T,
                  const dcp_constraints* nse_c, const dcp_constraints* T_c,
                  const std::vector<int>* colour_hint = nullptr) {
  require(cell_nse_dofs && cell_T_dofs && cell_geometry && cell_diameter, DCP_ERR_INVALID,
          "NULL argument");
  require(n_cells > 0 && n_u > 0 && n_u % 3 == 0 && n_p > 0 && n_T > 0, DCP_ERR_INVALID,
          "invalid sizes");
  const int nv = n_u / 3;
  h.nv = nv;
  // FE_Q(2) temperature: one dof per velocity support point (n_T = n_u / 3),
  // FE_Q(1): one per vertex (n_T = n_p)
  const int tdpc = (n_T == nv && n_T != n_p) ? 27 : 8;
  require(tdpc == 27 || n_T == n_p, DCP_ERR_INVALID,
          "n_T must be the vertex count (FE_Q(1)) or the Q2 support-point count (FE_Q(2))");
  h.tdpc = tdpc;
  auto& q2 = h.q2;
  auto& pd = h.pd;
  auto& td = h.td;
  q2.assign(size_t(n_cells) * 27, 0);
  pd.assign(size_t(n_cells) * 8, 0);
  td.assign(size_t(n_cells) * tdpc, 0);
  h.geo.assign(cell_geometry, cell_geometry + size_t(n_cells) * 3 * kMapPts);
  for (double x : h.geo) require(std::isfinite(x), DCP_ERR_INVALID, "non-finite cell geometry");
  std::vector<char> seen(nv, 0);
  for (int cell = 0; cell < n_cells; ++cell) {
    const int32_t* d = cell_nse_dofs + size_t(cell) * kNseDofs;
    for (int i = 0; i < kNseDofs; ++i) {
      const SysDof s = system_dof(i);
      if (s.comp < 3) {
        require(d[i] >= 0 && d[i] < n_u && d[i] % 3 == s.comp, DCP_ERR_UNSUPPORTED,
                "velocity dofs must be node-interleaved (3*node + component), as after "
                "DoFRenumbering::component_wise({0,0,0,1})");
        const int node = d[i] / 3;
        if (s.comp == 0) {
          q2[size_t(cell) * 27 + s.lex] = node;
          seen[node] = 1;
        } else {
          require(q2[size_t(cell) * 27 + s.lex] == node, DCP_ERR_UNSUPPORTED,
                  "velocity components of one support point must share a node");
        }
      } else {
        require(d[i] >= n_u && d[i] < n_u + n_p, DCP_ERR_INVALID, "pressure dof out of range");
        pd[size_t(cell) * 8 + s.lex] = d[i] - n_u;
      }
    }
    for (int v = 0; v < tdpc; ++v) {
      const int t = cell_T_dofs[size_t(cell) * tdpc + v];
      require(t >= 0 && t < n_T, DCP_ERR_INVALID, "temperature dof out of range");
      // FE_Q(2): hierarchic local order -> lexicographic (the kernels' order)
      td[size_t(cell) * tdpc + (tdpc == 27 ? kQ2HierToLex[v] : v)] = t;
    }
  }
  // ---- periodic identification. An identity line "dof = partner" (one
  // entry, weight 1, homogeneous: a closed make_periodicity_constraints line)
  // makes the dof an image of its partner. A velocity node is an image of node
  // m when each component's line is the identity to m's component or equals
  // m's own line (e.g. both fixed, where the partner's boundary condition was
  // closed into the image's line).
  auto identity_target = [](const dcp_constraints* c, int l) {
    const int b = c->entry_ptr[l];
    return (c->entry_ptr[l + 1] - b == 1 && c->entry_w[b] == 1.0 && c->inhomogeneity[l] == 0.0)
               ? c->entry_dof[b]
               : -1;
  };
  h.vmaster.assign(nv, -1);
  h.pmaster.assign(n_p, -1);
  h.tmaster.assign(n_T, -1);
  std::vector<int> nse_line(size_t(n_u) + n_p, -1);
  if (nse_c)
    for (int l = 0; l < nse_c->n_lines; ++l) {
      const int dof = nse_c->line_dof[l];
      require(dof >= 0 && dof < n_u + n_p, DCP_ERR_INVALID, "constraint dof out of range");
      nse_line[dof] = l;
    }
  auto same_line = [&](int a, int b) {
    const int la = nse_line[a], lb = nse_line[b];
    if (la < 0 || lb < 0) return la == lb;
    const int na = nse_c->entry_ptr[la + 1] - nse_c->entry_ptr[la];
    if (na != nse_c->entry_ptr[lb + 1] - nse_c->entry_ptr[lb]) return false;
    if (nse_c->inhomogeneity[la] != nse_c->inhomogeneity[lb]) return false;
    for (int k = 0; k < na; ++k) {
      const int ea = nse_c->entry_ptr[la] + k, eb = nse_c->entry_ptr[lb] + k;
      // entries on the partner's other components, translated to a's node
      if (nse_c->entry_dof[ea] % 3 != nse_c->entry_dof[eb] % 3 ||
          nse_c->entry_w[ea] != nse_c->entry_w[eb])
        return false;
    }
    return true;
  };
  if (nse_c) {
    for (int n = 0; n < nv; ++n) {
      int m = -1;
      for (int c = 0; c < 3 && m < 0; ++c) {
        const int l = nse_line[3 * n + c];
        const int t = l >= 0 ? identity_target(nse_c, l) : -1;
        if (t >= 0 && t < n_u && t / 3 != n && t % 3 == c) m = t / 3;
      }
      if (m < 0) continue;
      for (int c = 0; c < 3; ++c) {
        const int l = nse_line[3 * n + c];
        require(l >= 0, DCP_ERR_UNSUPPORTED, "partly periodic velocity node");
        const bool ident = identity_target(nse_c, l) == 3 * m + c;
        require(ident || same_line(3 * n + c, 3 * m + c),
                DCP_ERR_UNSUPPORTED,
                "velocity node " + std::to_string(n) + " is neither free, node-local nor an "
                "image of one partner node");
      }
      h.vmaster[n] = m;
      h.n_vslave++;
    }
    for (int p = 0; p < n_p; ++p) {
      const int l = nse_line[n_u + p];
      if (l < 0) continue;
      const int t = identity_target(nse_c, l);
      require(t >= n_u && t < n_u + n_p && t != n_u + p, DCP_ERR_UNSUPPORTED,
              "pressure constraints other than periodic identities are not supported");
      h.pmaster[p] = t - n_u;
      h.n_pslave++;
    }
    for (int n = 0; n < nv; ++n)
      require(h.vmaster[n] < 0 || h.vmaster[h.vmaster[n]] < 0, DCP_ERR_UNSUPPORTED,
              "periodic chain not closed");
    // a rank's local mesh may hold a partner only through its images' cells
    for (int n = 0; n < nv; ++n)
      if (h.vmaster[n] >= 0 && seen[n]) seen[h.vmaster[n]] = 1;
    for (int p = 0; p < n_p; ++p)
      require(h.pmaster[p] < 0 || h.pmaster[h.pmaster[p]] < 0, DCP_ERR_UNSUPPORTED,
              "periodic chain not closed");
  }
  for (int k = 0; k < nv; ++k) require(seen[k], DCP_ERR_INVALID, "velocity node without a cell");
  // ---- constraints -> node-local form. A line without entries is a fixed
  // component; three of them on one node form a no-slip node; a single one is
  // a no-normal-flux line whose weights all vanished (normal along an axis).
  // A periodic image is type 3 (every component constrained to its partner).
  auto& vc = h.vc;
  vc.assign(nv, NodeConstraint{{0, 0, 0}, 0, -1});
  std::vector<int> n_lines(nv, 0), fixed(nv, 0), fixed_comp(nv, -1);
  if (nse_c) {
    for (int l = 0; l < nse_c->n_lines; ++l) {
      const int dof = nse_c->line_dof[l];
      if (dof >= n_u) continue;  // periodic pressure identities (above)
      require(nse_c->inhomogeneity[l] == 0.0, DCP_ERR_UNSUPPORTED,
              "inhomogeneous velocity constraints are not supported");
      const int node = dof / 3, comp = dof % 3;
      if (h.vmaster[node] >= 0) continue;
      n_lines[node]++;
      const int b = nse_c->entry_ptr[l], e = nse_c->entry_ptr[l + 1];
      if (b == e) {
        fixed[node]++;
        fixed_comp[node] = comp;
        continue;
      }
      vc[node].type = 2;
      vc[node].k = comp;
      for (int k = b; k < e; ++k) {
        const int t = nse_c->entry_dof[k];
        require(t / 3 == node && t % 3 != comp, DCP_ERR_UNSUPPORTED,
                "constraint couples dofs of different support points (periodic / hanging "
                "nodes are not supported by the device path)");
        vc[node].w[t % 3] = nse_c->entry_w[k];
      }
    }
    for (int k = 0; k < nv; ++k) {
      if (h.vmaster[k] >= 0) {
        vc[k] = NodeConstraint{{0, 0, 0}, 3, -1};
        continue;
      }
      if (n_lines[k] == 0) continue;
      if (n_lines[k] == 3 && fixed[k] == 3) {
        vc[k].type = 1;
      } else if (n_lines[k] == 1 && fixed[k] == 1) {
        vc[k] = NodeConstraint{{0, 0, 0}, 2, fixed_comp[k]};
      } else if (n_lines[k] == 1) {
        // no-normal-flux line with entries, set above
      } else {
        fail(DCP_ERR_UNSUPPORTED, "velocity constraints of node " + std::to_string(k) +
                                      " are neither no-slip nor a single no-normal-flux line");
      }
    }
  }
  h.Tfix.assign(n_T, 0);
  h.Tbc.assign(n_T, 0.0);
  if (T_c)
    for (int l = 0; l < T_c->n_lines; ++l) {
      const int dof = T_c->line_dof[l];
      require(dof >= 0 && dof < n_T, DCP_ERR_INVALID, "temperature constraint out of range");
      const int t = identity_target(T_c, l);
      if (t >= 0 && t != dof) {  // periodic image
        require(t < n_T, DCP_ERR_INVALID, "temperature constraint out of range");
        h.tmaster[dof] = t;
        h.n_tslave++;
        continue;
      }
      require(T_c->entry_ptr[l] == T_c->entry_ptr[l + 1], DCP_ERR_UNSUPPORTED,
              "temperature constraints must be Dirichlet lines or periodic identities");
      h.Tfix[dof] = 1;
      h.Tbc[dof] = T_c->inhomogeneity[l];
    }
  for (int t = 0; t < n_T; ++t)
    require(h.tmaster[t] < 0 || (h.tmaster[h.tmaster[t]] < 0 && !h.Tfix[h.tmaster[t]]),
            DCP_ERR_UNSUPPORTED, "periodic temperature chain not closed");
  require(tdpc == 8 || h.n_tslave == 0, DCP_ERR_UNSUPPORTED,
          "periodic FE_Q(2) temperature is not supported");
  // identified cell maps (the originals kept for the constrained diagonals)
  if (h.n_vslave || h.n_pslave || h.n_tslave) {
    h.q2o = q2;
    h.pdo = pd;
    h.tdo = td;
    for (auto& n : q2)
      if (h.vmaster[n] >= 0) n = h.vmaster[n];
    for (auto& p : pd)
      if (h.pmaster[p] >= 0) p = h.pmaster[p];
    for (auto& t : td)
      if (h.tmaster[t] >= 0) t = h.tmaster[t];
  }
  // ---- colouring (greedy over vertex-sharing cells; tree order)
  std::vector<int32_t> vptr, vcells;
  {
    std::vector<int32_t> cnt(size_t(n_p) + 1, 0);
    for (size_t i = 0; i < pd.size(); ++i) cnt[pd[i] + 1]++;
    for (int v = 0; v < n_p; ++v) cnt[v + 1] += cnt[v];
    vcells.resize(pd.size());
    std::vector<int32_t> f(cnt.begin(), cnt.end() - 1);
    for (int cell = 0; cell < n_cells; ++cell)
      for (int v = 0; v < 8; ++v) vcells[f[pd[size_t(cell) * 8 + v]]++] = cell;
    vptr.swap(cnt);
  }
  std::vector<int> color(n_cells, -1);
  int n_colors = 0;
  for (int cell = 0; cell < n_cells; ++cell) {
    uint64_t used = 0;
    for (int v = 0; v < 8; ++v) {
      const int p = pd[size_t(cell) * 8 + v];
      for (int k = vptr[p]; k < vptr[p + 1]; ++k) {
        const int o = vcells[k];
        if (color[o] >= 0) used |= (uint64_t(1) << color[o]);
      }
    }
    int col = 0;
    while (col < 64 && (used >> col) & 1) ++col;
    require(col < 64, DCP_ERR_UNSUPPORTED, "cell colouring needs more than 64 colours");
    color[cell] = col;
    n_colors = std::max(n_colors, col + 1);
  }
  if (colour_hint && int(colour_hint->size()) == n_cells) {
    // a partition of the whole mesh keeps the whole mesh's colouring when it
    // has fewer classes (checked again on the local cells)
    const std::vector<int>& hc = *colour_hint;
    const int nh = *std::max_element(hc.begin(), hc.end()) + 1;
    bool ok = nh < n_colors && nh <= 64;
    for (int c = 0; c < n_cells && ok; ++c)
      for (int v = 0; v < 8 && ok; ++v) {
        const int p = pd[size_t(c) * 8 + v];
        for (int k = vptr[p]; k < vptr[p + 1]; ++k)
          if (vcells[k] != c && hc[vcells[k]] == hc[c]) ok = false;
      }
    if (ok) {
      color = hc;
      n_colors = nh;
    }
  }
  if (n_colors > 8 && shell_colouring(n_cells, cell_geometry, pd, vptr, vcells, color)) n_colors = 8;
  h.color_ptr.assign(n_colors + 1, 0);
  for (int cell = 0; cell < n_cells; ++cell) h.color_ptr[color[cell] + 1]++;
  for (int k = 0; k < n_colors; ++k) h.color_ptr[k + 1] += h.color_ptr[k];
  h.ccells.assign(n_cells, 0);
  auto& ccells = h.ccells;
  {
    std::vector<int> f(h.color_ptr.begin(), h.color_ptr.end() - 1);
    for (int cell = 0; cell < n_cells; ++cell) ccells[f[color[cell]]++] = cell;
  }
  // ---- patterns (an identified dof keeps only its diagonal, as a constrained
  // row of make_sparsity_pattern)
  union_pattern(nv, n_cells, q2.data(), 27, q2.data(), 27, h.Ap, h.Ac);
  union_pattern(nv, n_cells, q2.data(), 27, pd.data(), 8, h.Btp, h.Btc);
  union_pattern(n_p, n_cells, pd.data(), 8, q2.data(), 27, h.Bp, h.Bc);
  union_pattern(n_T, n_cells, td.data(), tdpc, td.data(), tdpc, h.Tp, h.Tc);
  auto add_diagonals = [](std::vector<int32_t>& ptr, std::vector<int32_t>& col,
                          const std::vector<int32_t>& master) {
    std::vector<int32_t> np(ptr.size(), 0), nc;
    nc.reserve(col.size() + master.size());
    for (size_t r = 0; r + 1 < ptr.size(); ++r) {
      if (master[r] >= 0) nc.push_back(int32_t(r));  // empty row: the diagonal only
      else nc.insert(nc.end(), col.begin() + ptr[r], col.begin() + ptr[r + 1]);
      np[r + 1] = int32_t(nc.size());
    }
    ptr.swap(np);
    col.swap(nc);
  };
  if (h.n_vslave) add_diagonals(h.Ap, h.Ac, h.vmaster);
  if (h.n_tslave) add_diagonals(h.Tp, h.Tc, h.tmaster);
  // Pattern of the explicit Schur complement S = B D^-1 B^T: row p couples the
  // vertices reachable through one velocity node (the 2-cell vertex patch).
  h.Sp.assign(size_t(n_p) + 1, 0);
  std::vector<std::vector<int32_t>> srow(n_p);
#pragma omp parallel
  {
    std::vector<int32_t> mark(n_p, -1);
#pragma omp for schedule(dynamic, 256)
    for (int p = 0; p < n_p; ++p) {
      std::vector<int32_t>& r = srow[p];
      for (int k = h.Bp[p]; k < h.Bp[p + 1]; ++k) {
        const int n = h.Bc[k];
        for (int j = h.Btp[n]; j < h.Btp[n + 1]; ++j) {
          const int q = h.Btc[j];
          if (mark[q] != p) {
            mark[q] = p;
            r.push_back(q);
          }
        }
      }
      std::sort(r.begin(), r.end());
    }
  }
  for (int p = 0; p < n_p; ++p) h.Sp[p + 1] = h.Sp[p] + int32_t(srow[p].size());
  h.Sc.resize(size_t(h.Sp[n_p]));
  // S_max_row also bounds the B rows' node counts: k_schur_form stages a
  // row's nodes in LDS (one wave per row, one half-wave lane per B^T row entry)
  h.S_max_row = 0;
  for (int p = 0; p < n_p; ++p) {
    std::copy(srow[p].begin(), srow[p].end(), h.Sc.begin() + h.Sp[p]);
    h.S_max_row = std::max({h.S_max_row, int(srow[p].size()), h.Bp[p + 1] - h.Bp[p]});
  }
  for (size_t n = 0; n + 1 < h.Btp.size(); ++n)
    require(h.Btp[n + 1] - h.Btp[n] <= 32, DCP_ERR_UNSUPPORTED, "B^T rows above 32 entries");
}

}  // namespace

namespace dcp {
// Device halo of one vector family from per-peer position lists (also the
// matrix powers' halos, matpow.cpp).
void make_halo(Ctx::Halo& h, const std::vector<int>& peers,
               const std::vector<std::vector<int32_t>>& spos,
               const std::vector<std::vector<int32_t>>& rpos) {
  h.peers = peers;
  h.sn.clear();
  h.rn.clear();
  h.soff.clear();
  h.roff.clear();
  std::vector<int32_t> sp, rp;
  for (size_t i = 0; i < peers.size(); ++i) {
    h.soff.push_back(sp.size());
    h.roff.push_back(rp.size());
    h.sn.push_back(spos[i].size());
    h.rn.push_back(rpos[i].size());
    sp.insert(sp.end(), spos[i].begin(), spos[i].end());
    rp.insert(rp.end(), rpos[i].begin(), rpos[i].end());
  }
  h.ns = int(sp.size());
  h.nr = int(rp.size());
  h.spos.upload(sp);
  h.rpos.upload(rp);
  h.sbuf.alloc(sp.size());
  h.rbuf.alloc(rp.size());
}
}  // namespace dcp

namespace {

// positions of a HaloPlan's entities in a vector: entity e -> off + w*e + j
void plan_positions(const HaloPlan& p, int off, std::vector<int>& peers,
                    std::vector<std::vector<int32_t>>& s, std::vector<std::vector<int32_t>>& r) {
  for (size_t i = 0; i < p.peers.size(); ++i) {
    size_t k = 0;
    while (k < peers.size() && peers[k] != p.peers[i]) ++k;
    if (k == peers.size()) {
      // keep peers ascending
      k = std::lower_bound(peers.begin(), peers.end(), p.peers[i]) - peers.begin();
      peers.insert(peers.begin() + k, p.peers[i]);
      s.insert(s.begin() + k, std::vector<int32_t>());
      r.insert(r.begin() + k, std::vector<int32_t>());
    }
    for (int j = p.send_ptr[i]; j < p.send_ptr[i + 1]; ++j)
      for (int c = 0; c < p.width; ++c) s[k].push_back(off + p.width * p.send_idx[j] + c);
    for (int j = p.recv_ptr[i]; j < p.recv_ptr[i + 1]; ++j)
      for (int c = 0; c < p.width; ++c) r[k].push_back(off + p.width * p.recv_idx[j] + c);
  }
}

void build_halos(Ctx& c, const LocalMesh& L) {
  auto one = [&](Ctx::Halo& h, std::initializer_list<std::pair<const HaloPlan*, int>> parts) {
    std::vector<int> peers;
    std::vector<std::vector<int32_t>> s, r;
    for (auto& pr : parts) plan_positions(*pr.first, pr.second, peers, s, r);
    make_halo(h, peers, s, r);
  };
  one(c.halo_v, {{&L.hv, 0}});
  one(c.halo_p, {{&L.hp, 0}});
  one(c.halo_nse, {{&L.hv, 0}, {&L.hp, c.n_u}});
  one(c.halo_T, {{&L.hT, 0}});
}

// global position of every local entry of a state field (identity on one GPU)
std::vector<int64_t> global_positions(const Ctx& c, int field) {
  std::vector<int64_t> g;
  if (field == DCP_T_SOLUTION || field == DCP_OLD_T_SOLUTION || field == DCP_T_RHS) {
    g.assign(c.T_g.begin(), c.T_g.end());
  } else if (c.feec) {
    // [w | u | p]: edges, faces, cells
    const int nw = c.fe_nw, nu = c.fe_nu;
    g.resize(size_t(c.n_u) + c.n_p);
    for (int i = 0; i < nw; ++i) g[i] = c.fe_w_g[i];
    for (int i = 0; i < nu; ++i) g[size_t(nw) + i] = int64_t(c.fe_nw_g) + c.fe_u_g[i];
    for (int i = 0; i < c.n_p; ++i)
      g[size_t(nw + nu) + i] = int64_t(c.fe_nw_g) + c.fe_nu_g + c.p_g[i];
  } else {
    g.resize(size_t(c.n_u) + c.n_p);
    const int vd = c.vdim;
    for (int i = 0; i < c.n_u; ++i) g[i] = vd * int64_t(c.vnode_g[i / vd]) + i % vd;
    for (int i = 0; i < c.n_p; ++i) g[size_t(c.n_u) + i] = int64_t(c.n_u_g) + c.p_g[i];
  }
  return g;
}

// is local entry i of the field owned by this rank
bool owned_entry(const Ctx& c, int field, size_t i) {
  if (field == DCP_T_SOLUTION || field == DCP_OLD_T_SOLUTION || field == DCP_T_RHS)
    return int(i) < c.nTo;
  if (c.feec) {
    const int k = int(i);
    if (k < c.fe_nw) return k < c.fe_nwo;
    if (k < c.fe_nw + c.fe_nu) return k - c.fe_nw < c.fe_nuo;
    return k - c.fe_nw - c.fe_nu < c.fe_npo;
  }
  if (int(i) < c.n_u) return int(i) < c.vdim * c.nvo;
  return int(i) - c.n_u < c.npo;
}

}  // namespace

namespace {

// Reverse Cuthill-McKee order of a symmetric pattern (rows [0, n), columns
// < n kept): BFS from a minimum-degree vertex of every component, neighbours
// by ascending degree, reversed. Returns perm[new] = old.
std::vector<int32_t> rcm_order(int n, const std::vector<int32_t>& ptr,
                               const std::vector<int32_t>& col) {
  std::vector<int32_t> deg(n), order;
  order.reserve(n);
  for (int i = 0; i < n; ++i) {
    int d = 0;
    for (int k = ptr[i]; k < ptr[i + 1]; ++k) d += col[k] < n;
    deg[i] = d;
  }
  std::vector<int32_t> byd(n);
  for (int i = 0; i < n; ++i) byd[i] = i;
  std::stable_sort(byd.begin(), byd.end(), [&](int a, int b) { return deg[a] < deg[b]; });
  std::vector<uint8_t> seen(n, 0);
  std::vector<int32_t> nb;
  for (int start : byd) {
    if (seen[start]) continue;
    seen[start] = 1;
    size_t head = order.size();
    order.push_back(start);
    while (head < order.size()) {
      const int v = order[head++];
      nb.clear();
      for (int k = ptr[v]; k < ptr[v + 1]; ++k) {
        const int u = col[k];
        if (u < n && !seen[u]) {
          seen[u] = 1;
          nb.push_back(u);
        }
      }
      std::stable_sort(nb.begin(), nb.end(), [&](int a, int b) { return deg[a] < deg[b]; });
      order.insert(order.end(), nb.begin(), nb.end());
    }
  }
  std::reverse(order.begin(), order.end());
  return order;
}

// SELL-64 storage of the owned rows of the S pattern (sell_spmv): slice width
// = longest row of the slice, rounded to column pairs. One GPU: rows and
// columns in reverse Cuthill-McKee order, so every slice's columns span less
// than 2^16 and are stored as 16-bit offsets from a per-slice base (10 instead
// of 12 bytes per entry); the inner Schur GMRES then runs in that order.
// pmap: CSR entry -> SELL position (k_schur_form writes through it).
// Radially separable MappingQ(3) geometry (the hyper_shell under
// SphericalManifold: support point (a,b,c) of every cell at rho_c Phi_ab, c
// the radial index; the cubic cells have |Phi_ab| = 1, the trilinear (9.2
// MappingQ1) cells the bilinear blend of the corner directions). Then
//   X = R(zeta) Phi(xi, eta),  J = [R Phi_xi | R Phi_eta | R' Phi],
//   J^-1 rows = m0 / R, m1 / R, m2 / R',  det J = R^2 R' D2,
// with m0 = Phi_eta x Phi / D2, m1 = Phi x Phi_xi / D2, m2 = Phi_xi x Phi_eta / D2,
// D2 = (Phi_xi x Phi_eta) . Phi at the 9 tangential Gauss points: one table per
// column of cells (and mapping kind), four radii per cell. Returns false
// (general streamed geometry) unless every cell fits within 1e-13 relative.
// node(cell, t): the coordinates of lexicographic support point t of a cell.
// Also groups the cells into radial layers (same support radii) with, per
// layer and Gauss point, 1/R, 1/R' and R^2 R' of R(zeta) = sum_c L_c(zeta) rho_c.
template <class NodeFn>
bool separable_geometry(int n_cells, NodeFn node, std::vector<int32_t>& col,
                        std::vector<double>& colgeo, std::vector<int32_t>& layer,
                        std::vector<double>& laygeo, std::vector<double>* colphi = nullptr,
                        std::vector<double>* layR = nullptr) {
  std::vector<double> rad;
  constexpr double tol = 1e-13;
  constexpr int kP = kMapPts1, kP2 = kMapPts1 * kMapPts1;
  col.assign(n_cells, -1);
  rad.assign(kP * size_t(n_cells), 0.0);
  colgeo.clear();
  std::vector<std::vector<double>> col_phi;  // [col][16 * 3] Phi_ab of the column
  struct Key {
    int64_t k[6];
    bool operator==(const Key& o) const {
      for (int i = 0; i < 6; ++i)
        if (k[i] != o.k[i]) return false;
      return true;
    }
  };
  struct KeyHash {
    size_t operator()(const Key& a) const {
      size_t h = 0;
      for (int i = 0; i < 6; ++i) h = h * 1000003u ^ size_t(a.k[i]);
      return h;
    }
  };
  std::unordered_map<Key, std::vector<int>, KeyHash> cols;
  for (int cell = 0; cell < n_cells; ++cell) {
    double phi[kP2][3], r[kP];
    for (int c = 0; c < kP; ++c) {
      const double* X0 = node(cell, kP2 * c);
      const double rc = std::sqrt(X0[0] * X0[0] + X0[1] * X0[1] + X0[2] * X0[2]);
      if (!(rc > 0)) return false;
      for (int ab = 0; ab < kP2; ++ab) {
        const double* X = node(cell, ab + kP2 * c);
        for (int d = 0; d < 3; ++d) {
          if (c == 0) phi[ab][d] = X[d] / rc;
          else if (!(std::fabs(X[d] / rc - phi[ab][d]) <= tol)) return false;
        }
      }
      r[c] = rc;
    }
    for (int c = 1; c < kP; ++c)
      if (!(r[c - 1] < r[c])) return false;
    for (int c = 0; c < kP; ++c) rad[kP * size_t(cell) + c] = r[c];
    Key key{{std::llround(phi[0][0] * 1e9), std::llround(phi[0][1] * 1e9),
             std::llround(phi[0][2] * 1e9), std::llround(phi[5][0] * 1e9),
             std::llround(phi[5][1] * 1e9), std::llround(phi[5][2] * 1e9)}};
    auto& cand = cols[key];
    int id = -1;
    for (int k : cand) {
      const auto& ph = col_phi[k];
      bool same = true;
      for (int i = 0; i < 3 * kP2 && same; ++i) same = std::fabs(ph[i] - (&phi[0][0])[i]) <= tol;
      if (same) {
        id = k;
        break;
      }
    }
    if (id < 0) {
      id = int(col_phi.size());
      cand.push_back(id);
      col_phi.emplace_back(&phi[0][0], &phi[0][0] + 3 * kP2);
    }
    col[cell] = id;
  }
  colgeo.assign(col_phi.size() * 90, 0.0);
  if (colphi) colphi->assign(col_phi.size() * 27, 0.0);
  for (size_t k = 0; k < col_phi.size(); ++k) {
    const double* ph = col_phi[k].data();
    for (int q1 = 0; q1 < 3; ++q1)
      for (int q0 = 0; q0 < 3; ++q0) {
        double F[3] = {0, 0, 0}, Fx[3] = {0, 0, 0}, Fy[3] = {0, 0, 0};
        for (int b = 0; b < kP; ++b)
          for (int a = 0; a < kP; ++a) {
            const double la = map_lag(a, kGaussX[q0]), lb = map_lag(b, kGaussX[q1]);
            const double da = map_dlag(a, kGaussX[q0]), db = map_dlag(b, kGaussX[q1]);
            for (int d = 0; d < 3; ++d) {
              const double v = ph[3 * (a + kP * b) + d];
              F[d] += la * lb * v;
              Fx[d] += da * lb * v;
              Fy[d] += la * db * v;
            }
          }
        auto cross = [](const double* u, const double* v, double* w) {
          w[0] = u[1] * v[2] - u[2] * v[1];
          w[1] = u[2] * v[0] - u[0] * v[2];
          w[2] = u[0] * v[1] - u[1] * v[0];
        };
        double m0[3], m1[3], m2[3];
        cross(Fy, F, m0);
        cross(F, Fx, m1);
        cross(Fx, Fy, m2);
        const double D2 = m2[0] * F[0] + m2[1] * F[1] + m2[2] * F[2];
        double* g = &colgeo[90 * k + 10 * (q0 + 3 * q1)];
        for (int d = 0; d < 3; ++d) {
          g[d] = m0[d] / D2;
          g[3 + d] = m1[d] / D2;
          g[6 + d] = m2[d] / D2;
        }
        g[9] = D2;
        if (colphi)
          for (int d = 0; d < 3; ++d) (*colphi)[27 * k + 3 * (q0 + 3 * q1) + d] = F[d];
      }
  }
  // radial layers
  layer.assign(n_cells, 0);
  laygeo.clear();
  if (layR) layR->clear();
  std::unordered_map<int64_t, int> ids;
  for (int cell = 0; cell < n_cells; ++cell) {
    const double* r = &rad[kP * size_t(cell)];
    const int64_t key = std::llround(r[0] * 1e12) * 1000003 + std::llround(r[kP - 1] * 1e12);
    auto it = ids.find(key);
    if (it == ids.end()) {
      it = ids.emplace(key, int(laygeo.size() / 9)).first;
      for (int q = 0; q < 3; ++q) {
        double R = 0, Rp = 0;
        for (int k = 0; k < kP; ++k) {
          R += map_lag(k, kGaussX[q]) * r[k];
          Rp += map_dlag(k, kGaussX[q]) * r[k];
        }
        laygeo.push_back(1.0 / R);
        laygeo.push_back(1.0 / Rp);
        laygeo.push_back(R * R * Rp);
        if (layR) layR->push_back(R);
      }
    }
    layer[cell] = it->second;
  }
  return true;
}

void build_sell(Ctx& c, const std::vector<int32_t>& Sp, const std::vector<int32_t>& Sc,
                bool permute) {
  c.S_nbr.release();
  const int rows = c.npo;
  const int n_sl = (rows + 63) / 64;
  std::vector<int32_t> perm, iperm;
  if (permute && rows > 0) {
    perm = rcm_order(rows, Sp, Sc);
    iperm.assign(rows, 0);
    for (int r = 0; r < rows; ++r) iperm[perm[r]] = r;
  }
  auto orow = [&](int r) { return perm.empty() ? r : perm[r]; };
  auto ncol = [&](int q) { return iperm.empty() || q >= rows ? q : iperm[q]; };
  std::vector<int64_t> off(size_t(n_sl) + 1, 0);
  std::vector<int32_t> base(n_sl, 0);
  // 16-bit column offsets wherever every slice's columns span < 2^16: the
  // RCM order on one GPU, and any rank's local S on several GPUs (local
  // columns, owned + ghost, ~30 k at refine 5 on 8 ranks)
  bool c16 = true;
  for (int sl = 0; sl < n_sl; ++sl) {
    int w = 0, lo = INT32_MAX, hi = 0;
    for (int r = 64 * sl; r < std::min(rows, 64 * sl + 64); ++r) {
      const int p = orow(r);
      w = std::max(w, Sp[p + 1] - Sp[p]);
      for (int k = Sp[p]; k < Sp[p + 1]; ++k) {
        lo = std::min(lo, ncol(Sc[k]));
        hi = std::max(hi, ncol(Sc[k]));
      }
      lo = std::min(lo, r);  // padding points at the own row
      hi = std::max(hi, r);
    }
    base[sl] = lo == INT32_MAX ? 0 : lo;
    if (hi - base[sl] >= 65536) c16 = false;
    w += w & 1;  // column pairs
    off[sl + 1] = off[sl] + 64 * int64_t(w);
  }
  const size_t len = size_t(off[n_sl]);
  std::vector<int32_t> scol(len, 0), pmap(Sp[rows], 0);
  std::vector<std::pair<int32_t, int32_t>> ent;
  for (int sl = 0; sl < n_sl; ++sl) {
    const int w = int((off[sl + 1] - off[sl]) / 64);
    for (int i = 0; i < 64; ++i) {
      const int r = 64 * sl + i;
      ent.clear();
      if (r < rows) {
        const int p = orow(r);
        for (int k = Sp[p]; k < Sp[p + 1]; ++k) ent.emplace_back(ncol(Sc[k]), k);
        std::sort(ent.begin(), ent.end());
      }
      for (int k = 0; k < w; ++k) {
        const int64_t pos = sell_pos(off.data(), r, k);
        if (k < int(ent.size())) {
          scol[pos] = ent[k].first;
          pmap[ent[k].second] = int32_t(pos);
        } else {
          scol[pos] = r < rows ? r : base[sl];
        }
      }
    }
  }
  require(len < size_t(INT32_MAX), DCP_ERR_UNSUPPORTED, "SELL storage of S above 2^31 entries");
  c.S_sell_off.upload(off);
  if (c16) {
    std::vector<uint16_t> s16(len);
    for (int sl = 0; sl < n_sl; ++sl)
      for (int64_t e = off[sl]; e < off[sl + 1]; ++e) s16[e] = uint16_t(scol[e] - base[sl]);
    c.S_sell_c16.upload(s16);
    c.S_sell_base.upload(base);
    c.S_sell_col.release();
  } else {
    c.S_sell_col.upload(scol);
    c.S_sell_c16.release();
    c.S_sell_base.release();
  }
  c.S_pmap.upload(pmap);
  if (!perm.empty() && c16) {
    c.S_perm.upload(perm);
  } else {
    // permutation only pays with the 16-bit columns: keep the identity order
    c.S_perm.release();
    if (!perm.empty()) return build_sell(c, Sp, Sc, false);
  }
  c.S_val.alloc(len);
  c.S_val.zero(c.stream);  // padding entries stay 0
  c.mp.reset();            // the matrix powers follow the pattern of S
  c.sell_part_len = sell_fused_blocks(rows);
  c.sperm_x.alloc(std::max(rows, 1));
  c.sperm_b.alloc(std::max(rows, 1));
}

// S with structured columns (one GPU, SellView::nbr). On a radially layered
// shell the Q1 pressure dofs form a grid of levels (radial vertex layers) x
// lateral vertices, and S = B D^-1 B^T couples (l, c) with (l', c') exactly
// when |l' - l| <= 2 and c' is in c's lateral two-ring N(c) (cells are
// products of a lateral quad and a radial interval, so the coupling through a
// shared velocity node factors): the pattern of row (l, c) is {l-2..l+2} x N(c).
// Rows are ordered level-major, laterals in reverse Cuthill-McKee order of the
// two-ring graph; with nd the levels of [l - 2, l + 2] inside the mesh from
// l + dlo on, entry k = nd j + d of row (l, c) is column (l + dlo + d, N(c)_j).
// The kernel then streams the values only (8 instead of 10 bytes per entry)
// and forms the column from the row's level and the L2-resident neighbour
// table. Returns
// false (and changes nothing) unless every check holds; DCP_S_STRUCT=0 turns
// it off.
bool build_sell_structured(Ctx& c, const std::vector<int32_t>& Sp, const std::vector<int32_t>& Sc,
                           const std::vector<int32_t>& pd, const std::vector<double>& geo,
                           int n_cells) {
  const char* env = std::getenv("DCP_S_STRUCT");
  if (env && *env == '0') return false;
  const int n = c.npo;
  if (n <= 0 || n != c.n_p || n_cells <= 0 || geo.size() < size_t(n_cells) * 3 * kMapPts ||
      pd.size() != size_t(n_cells) * 8)
    return false;
  // radius of every pressure dof (its vertex: lexicographic support point
  // 3a + 12b + 48c of the cubic map); vertices v and v + 4 one level apart
  std::vector<double> rad(size_t(n), -1.0);
  for (int cell = 0; cell < n_cells; ++cell)
    for (int v = 0; v < 8; ++v) {
      const int t = 3 * (v & 1) + 12 * ((v >> 1) & 1) + 48 * (v >> 2);
      const double* X = &geo[3 * (size_t(kMapPts) * cell + t)];
      const double r = std::sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2]);
      const int p = pd[8 * size_t(cell) + v];
      if (p < 0 || p >= n) return false;
      if (rad[p] < 0) rad[p] = r;
      else if (std::fabs(rad[p] - r) > 1e-12 * r) return false;
    }
  std::vector<double> ur(rad);
  std::sort(ur.begin(), ur.end());
  if (!(ur[0] > 0)) return false;
  std::vector<double> lev;
  for (double r : ur)
    if (lev.empty() || r > lev.back() * (1 + 1e-10)) lev.push_back(r);
  const int nl = int(lev.size());
  // the structured SpMV steps through a row's slots with at most 3 wraps per
  // step (linalg.hip SlotPos), which needs >= 3 levels in reach of every row
  if (nl < 3) return false;
  std::vector<int32_t> level(static_cast<size_t>(n));
  for (int p = 0; p < n; ++p)
    level[p] = int32_t(std::lower_bound(lev.begin(), lev.end(), rad[p] * (1 - 1e-10)) - lev.begin());
  // lateral vertices: dofs v and v + 4 of a cell lie on one radial line
  std::vector<int32_t> par(static_cast<size_t>(n));
  std::iota(par.begin(), par.end(), 0);
  auto find = [&](int32_t a) {
    while (par[a] != a) a = par[a] = par[par[a]];
    return a;
  };
  for (int cell = 0; cell < n_cells; ++cell)
    for (int v = 0; v < 4; ++v) {
      const int32_t a = pd[8 * size_t(cell) + v], b = pd[8 * size_t(cell) + v + 4];
      if (std::abs(level[b] - level[a]) != 1) return false;
      const int32_t ra = find(a), rb = find(b);
      if (ra != rb) par[std::max(ra, rb)] = std::min(ra, rb);
    }
  std::vector<int32_t> lat(size_t(n), -1), rootid(size_t(n), -1);
  int nc = 0;
  for (int p = 0; p < n; ++p) {
    const int32_t r = find(p);
    if (rootid[r] < 0) rootid[r] = nc++;
    lat[p] = rootid[r];
  }
  if (int64_t(nc) * nl != n) return false;
  std::vector<int32_t> dof_at(size_t(n), -1);  // [l * nc + lateral] -> dof
  for (int p = 0; p < n; ++p) {
    int32_t& d = dof_at[size_t(level[p]) * nc + lat[p]];
    if (d >= 0) return false;
    d = p;
  }
  // lateral two-ring sets from the pattern; every coupling within two levels
  std::vector<std::vector<int32_t>> ring(nc);
  for (int p = 0; p < n; ++p)
    for (int k = Sp[p]; k < Sp[p + 1]; ++k) {
      const int q = Sc[k];
      if (std::abs(level[q] - level[p]) > 2) return false;
      ring[lat[p]].push_back(lat[q]);
    }
  size_t ring_nnz = 0;
  for (auto& r : ring) {
    std::sort(r.begin(), r.end());
    r.erase(std::unique(r.begin(), r.end()), r.end());
    ring_nnz += r.size();
  }
  // lateral order: reverse Cuthill-McKee of the two-ring graph
  std::vector<int32_t> rp(size_t(nc) + 1, 0), rc;
  rc.reserve(ring_nnz);
  for (int a = 0; a < nc; ++a) {
    rc.insert(rc.end(), ring[a].begin(), ring[a].end());
    rp[a + 1] = int32_t(rc.size());
  }
  const std::vector<int32_t> lperm = rcm_order(nc, rp, rc);  // new lateral -> old
  std::vector<int32_t> lrank(static_cast<size_t>(nc));
  for (int i = 0; i < nc; ++i) lrank[lperm[i]] = i;
  // neighbour lists in the new lateral order, ascending
  std::vector<std::vector<int32_t>> nbl(nc);
  int jmax = 0;
  for (int i = 0; i < nc; ++i) {
    for (int32_t q : ring[lperm[i]]) nbl[i].push_back(lrank[q]);
    std::sort(nbl[i].begin(), nbl[i].end());
    jmax = std::max(jmax, int(nbl[i].size()));
  }
  // rows: r = l * nc + i
  std::vector<int32_t> perm(static_cast<size_t>(n)), iperm(static_cast<size_t>(n));
  for (int l = 0; l < nl; ++l)
    for (int i = 0; i < nc; ++i) {
      const int r = l * nc + i;
      perm[r] = dof_at[size_t(l) * nc + lperm[i]];
      iperm[perm[r]] = r;
    }
  // levels in reach of level l: l + dlo .. l + dlo + nd - 1 (as the kernel)
  auto reach = [&](int l, int& dlo) {
    dlo = l < 2 ? -l : -2;
    return std::min(l + 2, nl - 1) - (l + dlo) + 1;
  };
  const int n_sl = (n + 63) / 64;
  std::vector<int64_t> off(size_t(n_sl) + 1, 0);
  for (int sl = 0; sl < n_sl; ++sl) {
    int w = 0, dlo;
    for (int r = 64 * sl; r < std::min(n, 64 * sl + 64); ++r)
      w = std::max(w, reach(r / nc, dlo) * int(nbl[r % nc].size()));
    w += w & 1;
    off[sl + 1] = off[sl] + 64 * int64_t(w);
  }
  const size_t len = size_t(off[n_sl]);
  if (len >= size_t(INT32_MAX)) return false;
  std::vector<int32_t> pmap(size_t(Sp[n]), -1);
  for (int p = 0; p < n; ++p) {
    const int r = iperm[p], l = r / nc, i = r - l * nc;
    const std::vector<int32_t>& nb = nbl[i];
    for (int k = Sp[p]; k < Sp[p + 1]; ++k) {
      const int rq = iperm[Sc[k]], lq = rq / nc, iq = rq - lq * nc;
      const auto it = std::lower_bound(nb.begin(), nb.end(), iq);
      if (it == nb.end() || *it != iq) return false;
      int dlo;
      const int nd = reach(l, dlo);
      pmap[k] = int32_t(sell_pos(off.data(), r, nd * int(it - nb.begin()) + (lq - l - dlo)));
    }
  }
  // jmax + 1 rows, the last one the lateral itself: the kernel reads padding
  // entries (value 0; a narrower row of the slice, or the even round-up)
  // through row min(j, jmax)
  const int jrows = jmax + 1;
  std::vector<int32_t> tab(size_t(jrows) * nc);
  for (int j = 0; j < jrows; ++j)
    for (int i = 0; i < nc; ++i)
      tab[size_t(j) * nc + i] = j < int(nbl[i].size()) ? nbl[i][j] : i;
  // every column the kernel forms (k_sell_spmv<.., 2>, lanes past the last
  // row as the last row) must index the vector
  for (int sl = 0; sl < n_sl; ++sl) {
    const int w = int((off[sl + 1] - off[sl]) / 64);
    for (int i = 0; i < 64; ++i) {
      const int r = std::min(64 * sl + i, n - 1), l = r / nc, cc = r - l * nc;
      int dlo;
      const int nd = reach(l, dlo);
      for (int k = 0; k < w; ++k) {
        const int lv = l + dlo + k % nd;
        const int64_t col = int64_t(lv) * nc + tab[size_t(std::min(k / nd, jmax)) * nc + cc];
        if (lv < 0 || lv >= nl || col < 0 || col >= n) return false;
      }
    }
  }
  c.S_sell_off.upload(off);
  c.S_sell_col.release();
  c.S_sell_c16.release();
  c.S_sell_base.release();
  c.S_nbr.upload(tab);
  c.S_nc = nc;
  c.S_nl = nl;
  c.S_nj = jrows;
  c.S_pmap.upload(pmap);
  c.S_perm.upload(perm);
  c.S_val.alloc(len);
  c.S_val.zero(c.stream);  // entries outside the pattern stay 0
  c.mp.reset();
  c.sell_part_len = sell_fused_blocks(n);
  c.sperm_x.alloc(size_t(n));
  c.sperm_b.alloc(size_t(n));
  return true;
}

}  // namespace

namespace dcp {
// nse_matrix.block(0,0) of the last assemble_nse_system (its dt, nse_ph) into
// A_val: the full MODE 0 scatter, which rewrites B^T / B / con_diag with the
// same values and leaves the rhs alone.
void ensure_A_val(Ctx& c) {
  // the velocity block's values (9 doubles per 3x3 block, 58 GB at r=6) exist
  // only once something reads the block
  if (!c.A_val.p) c.A_val.alloc(c.A_nnzb * 9);
}

void materialize_velocity_block(Ctx& c) {
  if (c.A_current) return;
  ensure_A_val(c);
  if (!c.first_touch_A) c.A_val.zero(c.stream);
  if (!c.first_touch_Bt) c.Bt_val.zero(c.stream);
  if (!c.first_touch_B) c.B_val.zero(c.stream);
  c.con_diag.zero(c.stream);
  NseOut out{};
  out.A = c.A_val.p;
  out.Bt = c.Bt_val.p;
  out.B = c.B_val.p;
  out.cdiag = c.con_diag.p;
  out.cidx = c.mf_cidx.p;
  out.pcdiag = c.con_diag.p + 3 * size_t(c.n_con);
  out.pcidx = c.periodic ? c.pcidx.p : nullptr;
  for (int k = 0; k < c.n_colors(); ++k)
    launch_nse_system(c.cd(), c.maps(), c.color_begin(k), c.color_size(k), c.old_nse.p, c.old_T.p,
                      c.nse_ph, out, c.stream, c.element_mfma);
  image_diagonal_blocks(c.n_img_node, c.img_node.p, c.img_blk.p, c.mf_cidx.p, c.con_diag.p,
                        c.A_val.p, c.stream);
  c.A_current = true;
  c.B_current = true;
}

void set_ctx_error(dcp_ctx* ctx, const char* msg) {
  if (ctx) ctx->err = msg;
  g_last_error = msg;
}

// nse_matrix.block(1,0) of the last operator-form assembly: the transpose of
// B^T, block by block (bitwise the B the full scatter produces)
void materialize_B(Ctx& c) {
  if (c.B_current) return;
  transpose_blocks3(long(c.B_tperm.n), c.B_tperm.p, c.Bt_val.p, c.B_val.p, c.stream);
  c.B_current = true;
}
}  // namespace dcp

extern "C" {

int dcp_nccl_unique_id(void* out128) {
  return guarded(nullptr, [&] {
    require(out128 != nullptr, DCP_ERR_INVALID, "NULL out");
    rccl_unique_id(out128);
    return DCP_OK;
  });
}

dcp_group* dcp_group_create(int world_size) {
  try {
    return new dcp_group(world_size);
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return nullptr;
  } catch (const DeviceError& e) {
    g_last_error = std::string("HIP error in ") + e.what_expr;
    return nullptr;
  }
}

void dcp_group_destroy(dcp_group* g) { delete g; }

namespace dcp {
// counts (the halo of `field`: 0 velocity nodes, 1 pressure, 2 temperature)
// and that halo's peer lists in global ids (dcp_partition_info[_field],
// dcp_dist_partition_info[_field])
void partition_info_out(const LocalMesh& L, int n_colors, int field, int64_t* info, int32_t* peers,
                        int32_t* send_ptr, int64_t* send_gid, int32_t* recv_ptr,
                        int64_t* recv_gid) {
  const HaloPlan& hp = field == 0 ? L.hv : field == 1 ? L.hp : L.hT;
  const int64_t v[12] = {L.n_cells, L.n_owned_cells, L.nvo, L.nvg, L.npo, L.npg, L.nTo, L.nTg,
                         int64_t(hp.peers.size()), int64_t(hp.send_idx.size()),
                         int64_t(hp.recv_idx.size()), int64_t(n_colors)};
  std::copy(v, v + 12, info);
  if (peers) std::copy(hp.peers.begin(), hp.peers.end(), peers);
  if (send_ptr) std::copy(hp.send_ptr.begin(), hp.send_ptr.end(), send_ptr);
  if (recv_ptr) std::copy(hp.recv_ptr.begin(), hp.recv_ptr.end(), recv_ptr);
  if (send_gid) std::copy(hp.send_gid.begin(), hp.send_gid.end(), send_gid);
  if (recv_gid) std::copy(hp.recv_gid.begin(), hp.recv_gid.end(), recv_gid);
}
}  // namespace dcp

int dcp_partition_info_field(int n_cells, const int32_t* cell_nse_dofs, const int32_t* cell_T_dofs,
                             const double* cell_geometry, const double* cell_diameter, int n_u,
                             int n_p, int n_T, const dcp_constraints* nse_c,
                             const dcp_constraints* T_c, int rank, int world, int field,
                             int64_t* info, int32_t* peers, int32_t* send_ptr, int64_t* send_gid,
                             int32_t* recv_ptr, int64_t* recv_gid) {
  return guarded(nullptr, [&] {
    require(info != nullptr, DCP_ERR_INVALID, "NULL info");
    require(field >= 0 && field <= 2, DCP_ERR_INVALID, "field must be 0..2");
    LocalMesh L;
    try {
      L = localize(n_cells, cell_nse_dofs, cell_T_dofs, cell_geometry, cell_diameter, n_u, n_p,
                   n_T, nse_c, T_c, rank, world);
    } catch (const std::runtime_error& e) {
      fail(DCP_ERR_INVALID, e.what());
    }
    const dcp_constraints lnc = L.nse_view(), ltc = L.T_view();
    HostPrep h;
    const std::vector<int> hint =
        partition_colour_hint(n_cells, cell_nse_dofs, cell_geometry, n_u, n_p, L.cells_g);
    prepare_mesh(h, L.n_cells, L.cell_nse_dofs.data(), L.cell_T_dofs.data(), L.geometry.data(),
                 L.diameter.data(), L.n_u(), L.n_p(), L.n_T(), &lnc, &ltc, &hint);
    partition_info_out(L, int(h.color_ptr.size()) - 1, field, info, peers, send_ptr, send_gid,
                       recv_ptr, recv_gid);
    return DCP_OK;
  });
}

int dcp_partition_info(int n_cells, const int32_t* cell_nse_dofs, const int32_t* cell_T_dofs,
                       const double* cell_geometry, const double* cell_diameter, int n_u, int n_p,
                       int n_T, const dcp_constraints* nse_c, const dcp_constraints* T_c, int rank,
                       int world, int64_t* info, int32_t* peers, int32_t* send_ptr,
                       int64_t* send_gid, int32_t* recv_ptr, int64_t* recv_gid) {
  return dcp_partition_info_field(n_cells, cell_nse_dofs, cell_T_dofs, cell_geometry, cell_diameter,
                                  n_u, n_p, n_T, nse_c, T_c, rank, world, 0, info, peers, send_ptr,
                                  send_gid, recv_ptr, recv_gid);
}

int dcp_dist_partition_info_field(const dcp_dist_mesh* m, const dcp_host_comm* comm, int field,
                                  int64_t* info, int32_t* peers, int32_t* send_ptr,
                                  int64_t* send_gid, int32_t* recv_ptr, int64_t* recv_gid) {
  return guarded(nullptr, [&] {
    require(m && comm && info, DCP_ERR_INVALID, "NULL argument");
    require(field >= 0 && field <= 2, DCP_ERR_INVALID, "field must be 0..2");
    LocalMesh L;
    try {
      L = localize_distributed(*m, *comm);
    } catch (const std::runtime_error& e) {
      fail(DCP_ERR_INVALID, e.what());
    }
    const dcp_constraints lnc = L.nse_view(), ltc = L.T_view();
    HostPrep h;
    prepare_mesh(h, L.n_cells, L.cell_nse_dofs.data(), L.cell_T_dofs.data(), L.geometry.data(),
                 L.diameter.data(), L.n_u(), L.n_p(), L.n_T(), &lnc, &ltc);
    partition_info_out(L, int(h.color_ptr.size()) - 1, field, info, peers, send_ptr, send_gid,
                       recv_ptr, recv_gid);
    return DCP_OK;
  });
}

int dcp_dist_partition_info(const dcp_dist_mesh* m, const dcp_host_comm* comm, int64_t* info,
                            int32_t* peers, int32_t* send_ptr, int64_t* send_gid,
                            int32_t* recv_ptr, int64_t* recv_gid) {
  return dcp_dist_partition_info_field(m, comm, 0, info, peers, send_ptr, send_gid, recv_ptr,
                                       recv_gid);
}

int dcp_feec_partition_info(const dcp_feec_mesh* m, int rank, int world, int field,
                            int64_t* info, int32_t* peers, int32_t* send_ptr, int64_t* send_gid,
                            int32_t* recv_ptr, int64_t* recv_gid) {
  return guarded(nullptr, [&] {
    require(m != nullptr && info != nullptr, DCP_ERR_INVALID, "NULL argument");
    require(field >= 0 && field < 4, DCP_ERR_INVALID, "field must be 0..3");
    FeecLocal L;
    try {
      L = localize_feec(*m, rank, world);
    } catch (const std::runtime_error& e) {
      fail(DCP_ERR_INVALID, e.what());
    }
    const HaloPlan& h = field == 0 ? L.hw : field == 1 ? L.hu : field == 2 ? L.hp : L.hT;
    const int64_t v[11] = {L.n_cells, L.n_owned_cells, L.nwo, L.nwg, L.nuo, L.nug, L.nTo, L.nTg,
                           int64_t(h.peers.size()), int64_t(h.send_idx.size()),
                           int64_t(h.recv_idx.size())};
    std::copy(v, v + 11, info);
    if (peers) std::copy(h.peers.begin(), h.peers.end(), peers);
    if (send_ptr) std::copy(h.send_ptr.begin(), h.send_ptr.end(), send_ptr);
    if (recv_ptr) std::copy(h.recv_ptr.begin(), h.recv_ptr.end(), recv_ptr);
    if (send_gid) std::copy(h.send_gid.begin(), h.send_gid.end(), send_gid);
    if (recv_gid) std::copy(h.recv_gid.begin(), h.recv_gid.end(), recv_gid);
    return DCP_OK;
  });
}

int dcp_abi_version(void) { return DCP_ABI_VERSION; }

// ---- TimerOutput / SolverControl log ---------------------------------------
int dcp_timer_record(dcp_ctx* ctx, const char* section, double seconds) {
  return guarded(ctx, [&] {
    require(ctx && section, DCP_ERR_INVALID, "NULL argument");
    ctx->section_add(section, seconds);
    return DCP_OK;
  });
}

int dcp_timer_section(dcp_ctx* ctx, const char* section, long* calls, double* seconds) {
  return guarded(ctx, [&] {
    require(ctx && section, DCP_ERR_INVALID, "NULL argument");
    for (const auto& s : ctx->sections)
      if (s.name == section) {
        if (calls) *calls = s.calls;
        if (seconds) *seconds = s.seconds;
        return DCP_OK;
      }
    fail(DCP_ERR_INVALID, std::string("no timer section \"") + section + "\"");
    return DCP_ERR_INVALID;
  });
}

int dcp_timer_reset(dcp_ctx* ctx) {
  return guarded(ctx, [&] {
    require(ctx != nullptr, DCP_ERR_INVALID, "NULL ctx");
    ctx->sections.clear();
    ctx->t_created = std::chrono::steady_clock::now();
    return DCP_OK;
  });
}

int dcp_timer_summary(dcp_ctx* ctx, char* buf, int len) {
  return guarded(ctx, [&] {
    require(ctx != nullptr, DCP_ERR_INVALID, "NULL ctx");
    // TimerOutput::print_summary (wall times)
    const double total =
        std::chrono::duration<double>(std::chrono::steady_clock::now() - ctx->t_created).count();
    std::string out, line(71, '-');
    char row[256];
    out += "\n+" + std::string(45, '-') + "+" + std::string(12, '-') + "+" + std::string(12, '-') +
           "+\n";
    std::snprintf(row, sizeof row, "| Total wallclock time elapsed since start    |%10.3gs |            |\n",
                  total);
    out += row;
    out += "|                                             |            |            |\n";
    out += "| Section                         | no. calls |  wall time | % of total |\n";
    const std::string sep = "+" + std::string(33, '-') + "+" + std::string(11, '-') + "+" +
                            std::string(12, '-') + "+" + std::string(12, '-') + "+\n";
    out += sep;
    std::vector<const Ctx::Section*> order;
    for (const auto& s : ctx->sections) order.push_back(&s);
    std::sort(order.begin(), order.end(),
              [](const Ctx::Section* x, const Ctx::Section* y) { return x->name < y->name; });
    for (const auto* s : order) {
      std::snprintf(row, sizeof row, "| %-32s| %9ld |%10.3gs |%10.3g%% |\n", s->name.c_str(),
                    s->calls, s->seconds, total > 0 ? 100.0 * s->seconds / total : 0.0);
      out += row;
    }
    out += sep;
    (void)line;
    require(buf != nullptr && len > 0, DCP_ERR_INVALID, "NULL buffer");
    std::snprintf(buf, size_t(len), "%s", out.c_str());
    return int(out.size()) < len ? DCP_OK : DCP_ERR_INVALID;
  });
}

int dcp_solver_history(dcp_ctx* ctx, int attempt, int* steps, double* values, int cap, int* n,
                       int* result) {
  return guarded(ctx, [&] {
    require(ctx != nullptr && n != nullptr, DCP_ERR_INVALID, "NULL argument");
    require(attempt == 0 || attempt == 1, DCP_ERR_INVALID, "attempt must be 0 or 1");
    const Ctx::SolverLog& l = ctx->solver_log[attempt];
    *n = int(l.checks.size());
    if (result) *result = l.result;
    for (int i = 0; i < std::min(cap, *n); ++i) {
      if (steps) steps[i] = int(l.checks[size_t(i)].first);
      if (values) values[i] = l.checks[size_t(i)].second;
    }
    return DCP_OK;
  });
}

int dcp_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* dcp_last_error(const dcp_ctx* ctx) {
  return ctx ? ctx->err.c_str() : g_last_error.c_str();
}

int dcp_ctx_create(const dcp_config* cfg, dcp_ctx** out) {
  return guarded(nullptr, [&] {
    require(out != nullptr, DCP_ERR_INVALID, "out is NULL");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
      fail(DCP_ERR_DEVICE, "no HIP device available: the dcp hot path runs on MI355X only");
    std::unique_ptr<dcp_ctx> c(new dcp_ctx());
    if (cfg) c->cfg = *cfg;
    if (c->cfg.world_size <= 0) c->cfg.world_size = 1;
    require(c->cfg.device >= 0 && c->cfg.device < ndev, DCP_ERR_INVALID, "device ordinal out of range");
    require(c->cfg.rank >= 0 && c->cfg.rank < c->cfg.world_size, DCP_ERR_INVALID, "rank out of range");
    DCP_HIP_CHECK(hipSetDevice(c->cfg.device));
    if (c->cfg.world_size > 1 || c->cfg.nccl_id) {
      if (c->cfg.group) {
        require(c->cfg.group->size == c->cfg.world_size, DCP_ERR_INVALID, "group size != world_size");
        c->comm = make_local_comm(c->cfg.group, c->cfg.rank);
        // DCP_PEER_COMM=1: the all-reduces device-initiated over the group's
        // mailboxes (comm.h PeerComm); every rank of the group must agree
        const char* env_pc = std::getenv("DCP_PEER_COMM");
        if (env_pc && *env_pc == '1')
          c->comm = make_peer_comm(std::move(c->comm), c->cfg.group, c->cfg.rank);
      } else {
        require(c->cfg.nccl_id != nullptr, DCP_ERR_INVALID,
                "world_size > 1 needs nccl_id (dcp_nccl_unique_id on rank 0) or a dcp_group");
        c->comm = make_rccl_comm(c->cfg.nccl_id, c->cfg.rank, c->cfg.world_size);
      }
    }
    DCP_HIP_CHECK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    c->ev_total.init();
    c->schur_ev.resize(Ctx::kSchurEvents);
    for (auto& t : c->schur_ev) t.init();
    for (auto& v : c->mf_ev) {
      v.resize(Ctx::kMfEvents);
      for (auto& t : v) t.init();
    }
    ensure_workspaces(*c);
    if (const char* e = std::getenv("DCP_TEST_FORCE_REORTH_AT"))
      c->test_force_reorth_at = std::atoi(e);
    *out = c.release();
    return DCP_OK;
  });
}

void dcp_ctx_destroy(dcp_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->cfg.device);
  delete ctx;
}

int dcp_set_physics(dcp_ctx* ctx, const dcp_physics* ph) {
  return guarded(ctx, [&] {
    require(ctx && ph, DCP_ERR_INVALID, "NULL argument");
    require(ph->temperature_degree == 1 || ph->temperature_degree == 2, DCP_ERR_UNSUPPORTED,
            "temperature degree must be 1 or 2");
    require(ph->nse_solver_interval >= 1, DCP_ERR_INVALID, "NSE solver interval must be >= 1");
    ctx->hph = *ph;
    set_physics_dev(*ctx);
    ctx->have_physics = true;
    return DCP_OK;
  });
}

int dcp_set_option(dcp_ctx* ctx, int option, int value) {
  return guarded(ctx, [&] {
    require(ctx != nullptr, DCP_ERR_INVALID, "NULL context");
    if (option == DCP_OPT_SCHUR_EXPLICIT) {
      ctx->schur_explicit = value != 0;
      ctx->precond_built = false;  // S must be (re)formed
      return DCP_OK;
    }
    if (option == DCP_OPT_MATRIX_FREE) {
      require(value >= 0 && value <= 2, DCP_ERR_INVALID, "DCP_OPT_MATRIX_FREE must be 0, 1 or 2");
      ctx->matrix_free = value;
      return DCP_OK;
    }
    if (option == DCP_OPT_FUSED_CHAIN) {
      ctx->fused_chain = value != 0;
      return DCP_OK;
    }
    if (option == DCP_OPT_FEEC_ZERO_MEAN) {
      ctx->feec_zero_mean = value != 0;
      return DCP_OK;
    }
    if (option == DCP_OPT_FEEC_BLOCK_PRECONDITIONER) {
      ctx->feec_block_prec = value != 0;
      return DCP_OK;
    }
    if (option == DCP_OPT_FEEC_FIXED_INNER) {
      require(value >= 0 && value <= 100, DCP_ERR_INVALID,
              "DCP_OPT_FEEC_FIXED_INNER must be in [0, 100]");
      ctx->feec_fixed_inner = value;
      return DCP_OK;
    }
    if (option == DCP_OPT_LOG_HISTORY) {
      ctx->log_history = value != 0;
      return DCP_OK;
    }
    if (option == DCP_OPT_GRAM_SCHMIDT) {
      require(value >= 0 && value <= 3, DCP_ERR_INVALID, "DCP_OPT_GRAM_SCHMIDT must be 0..3");
      ctx->gram_schmidt = value;
      return DCP_OK;
    }
    if (option == DCP_OPT_ASSEMBLE_VELOCITY_BLOCK) {
      ctx->assemble_A = value != 0;
      return DCP_OK;
    }
    if (option == DCP_OPT_ELEMENT_MFMA) {
      require(value == 0 || value == 1, DCP_ERR_INVALID, "DCP_OPT_ELEMENT_MFMA must be 0 or 1");
      ctx->element_mfma = value != 0;
      return DCP_OK;
    }
    if (option == DCP_OPT_T_FIXED_CG) {
      require(value >= 0, DCP_ERR_INVALID, "DCP_OPT_T_FIXED_CG must be >= 0");
      ctx->T_fixed_cg = value;
      return DCP_OK;
    }
    if (option == DCP_OPT_SCHUR_FIXED_INNER) {
      require(value >= 0, DCP_ERR_INVALID, "DCP_OPT_SCHUR_FIXED_INNER must be >= 0");
      ctx->schur_fixed_inner = value;
      return DCP_OK;
    }
    if (option == DCP_OPT_INNER_MAX_STEPS) {
      require(value >= 1, DCP_ERR_INVALID, "DCP_OPT_INNER_MAX_STEPS must be >= 1");
      ctx->inner_max_steps = value;
      return DCP_OK;
    }
    if (option == DCP_OPT_MATRIX_POWERS) {
      ctx->matrix_powers = value != 0;
      return DCP_OK;
    }
    if (option == DCP_OPT_BLOCK_FIXED_INNER) {
      require(value >= 0, DCP_ERR_INVALID, "DCP_OPT_BLOCK_FIXED_INNER must be >= 0");
      ctx->block_fixed_inner = value;
      return DCP_OK;
    }
    if (option == DCP_OPT_HANDOFF_SPIN_LIMIT) {
      set_handoff_spin_limit(value);
      return DCP_OK;
    }
    if (option == DCP_OPT_FGMRES_MAX_OUTER) {
      require(value >= 1, DCP_ERR_INVALID, "DCP_OPT_FGMRES_MAX_OUTER must be >= 1");
      ctx->fgmres_max_outer = value;
      return DCP_OK;
    }
    fail(DCP_ERR_INVALID, "unknown option " + std::to_string(option));
  });
}

int dcp_set_time_step(dcp_ctx* ctx, double dt) {
  return guarded(ctx, [&] {
    require(ctx && ctx->have_physics, DCP_ERR_STATE, "physics not set");
    ctx->hph.time_step = dt;
    set_physics_dev(*ctx);
    return DCP_OK;
  });
}

int dcp_mesh_check(int n_cells, const int32_t* cell_nse_dofs, const int32_t* cell_T_dofs,
                   const double* cell_geometry, const double* cell_diameter, int n_u, int n_p,
                   int n_T, const dcp_constraints* nse_c, const dcp_constraints* T_c,
                   int* n_colors) {
  return guarded(nullptr, [&] {
    HostPrep h;
    prepare_mesh(h, n_cells, cell_nse_dofs, cell_T_dofs, cell_geometry, cell_diameter, n_u, n_p,
                 n_T, nse_c, T_c);
    if (n_colors) *n_colors = int(h.color_ptr.size()) - 1;
    return DCP_OK;
  });
}

int dcp_mesh_geometry_info(int n_cells, const double* cell_geometry, int* separable,
                           int* n_columns, int* n_layers) {
  return guarded(nullptr, [&] {
    require(n_cells > 0 && cell_geometry != nullptr, DCP_ERR_INVALID, "empty mesh");
    std::vector<int32_t> col, layer;
    std::vector<double> colgeo, laygeo;
    const bool sep = separable_geometry(
        n_cells, [&](int cell, int t) { return cell_geometry + 3 * kMapPts * size_t(cell) + 3 * t; },
        col, colgeo, layer, laygeo);
    if (separable) *separable = sep ? 1 : 0;
    if (n_columns) *n_columns = sep ? int(colgeo.size() / 90) : 0;
    if (n_layers) *n_layers = sep ? int(laygeo.size() / 9) : 0;
    return DCP_OK;
  });
}

}  // extern "C"

// The device half of a mesh upload (one GPU, or this rank's LocalMesh `L`
// when dist): buffers, patterns, scatter maps, the explicit Schur complement
// layout, the matrix-free tables, halos.
void upload_prepared(Ctx& c, HostPrep& h, const LocalMesh& L, bool dist, int n_cells,
                     const double* cell_diameter, int n_u, int n_p, int n_T, int n_u_g, int n_p_g,
                     int n_T_g) {
    DCP_HIP_CHECK(hipSetDevice(c.cfg.device));
    c.old_nse_ghosted = c.old_T_ghosted = false;
    c.feec = false;
    c.dim2 = false;
    c.vdim = 3;
    c.tdpc3 = h.tdpc;
    c.tsep = false;
    c.ts_tmat_valid = false;
    c.btk = false;
    c.cdk = false;
    const int nv = h.nv;
    c.color_ptr = h.color_ptr;
    const auto &q2 = h.q2, &pd = h.pd, &td = h.td;
    const auto& vc = h.vc;
    const auto &Ap = h.Ap, &Ac = h.Ac, &Btp = h.Btp, &Btc = h.Btc, &Bp = h.Bp, &Bc = h.Bc,
               &Tp = h.Tp, &Tc = h.Tc;
    const auto& ccells = h.ccells;
    const auto& Tfix = h.Tfix;
    const auto& Tbc = h.Tbc;
    // ---- upload
    c.n_cells = n_cells;
    c.n_u = n_u;
    c.n_p = n_p;
    c.n_T = n_T;
    c.n_vnodes = nv;
    c.n_u_g = n_u_g;
    c.n_p_g = n_p_g;
    c.n_T_g = n_T_g;
    c.n_owned_cells = dist ? L.n_owned_cells : n_cells;
    c.nvo = dist ? L.nvo : nv;
    c.npo = dist ? L.npo : n_p;
    c.nTo = dist ? L.nTo : n_T;
    c.vnode_g = L.vnode_g;
    c.p_g = L.p_g;
    c.T_g = L.T_g;
    c.cell_q2.upload(q2);
    c.cell_p.upload(pd);
    c.cell_T.upload(td);
    c.cell_geo.upload(h.geo);
    c.diameter.upload(std::vector<double>(cell_diameter, cell_diameter + n_cells));
    c.vcon.upload(vc);
    c.T_fixed.upload(Tfix);
    c.T_bc.upload(Tbc);
    c.color_cells.upload(ccells);
    c.A_ptr.upload(Ap);
    c.A_col.upload(Ac);
    c.Bt_ptr.upload(Btp);
    c.Bt_col.upload(Btc);
    c.B_ptr.upload(Bp);
    c.B_col.upload(Bc);
    c.T_ptr.upload(Tp);
    c.T_col.upload(Tc);
    c.S_ptr.upload(h.Sp);
    c.S_col.upload(h.Sc);
    if (dist || !build_sell_structured(c, h.Sp, h.Sc, pd, h.geo, n_cells))
      build_sell(c, h.Sp, h.Sc, !dist);
    c.S_max_row = h.S_max_row;
    c.A_val.release();  // allocated on first use (ensure_A_val)
    c.A_nnzb = Ac.size();
    c.Bt_val.alloc(Btc.size() * 3);
    c.B_val.alloc(Bc.size() * 3);
    {
      // B entry (p, n) -> B^T entry (n, p), if every one exists locally
      const int rows = int(Bp.size()) - 1;
      std::vector<int32_t> tperm(Bc.size());
      int missing = 0;
#pragma omp parallel for schedule(static) reduction(+ : missing)
      for (int p = 0; p < rows; ++p)
        for (int k = Bp[p]; k < Bp[p + 1]; ++k) {
          const int n = Bc[k];
          // B^T holds the rows of the local (owned) velocity nodes only
          const bool local = n >= 0 && n + 1 < int(Btp.size());
          const int32_t* b = local ? Btc.data() + Btp[n] : nullptr;
          const int32_t* e = local ? Btc.data() + Btp[n + 1] : nullptr;
          const int32_t* f = local ? std::lower_bound(b, e, p) : nullptr;
          if (!local || f == e || *f != p) {
            ++missing;
            tperm[k] = -1;
          } else {
            tperm[k] = int32_t(f - Btc.data());
          }
        }
      c.B_transpose = missing == 0 && !Bc.empty();
      if (c.B_transpose) c.B_tperm.upload(tperm);
      else c.B_tperm.release();
    }
    c.Tmass.alloc(Tc.size());
    c.Tstiff.alloc(Tc.size());
    c.Tmat.alloc(Tc.size());
    c.posA.alloc(size_t(n_cells) * 729);
    c.posBt.alloc(size_t(n_cells) * 216);
    c.posB.alloc(size_t(n_cells) * 216);
    c.posT.alloc(size_t(n_cells) * h.tdpc * h.tdpc);
    launch_build_scatter_maps(c.cd(), c.A_ptr.p, c.A_col.p, c.Bt_ptr.p, c.Bt_col.p, c.B_ptr.p,
                              c.B_col.p, c.T_ptr.p, c.T_col.p, c.posA.p, c.posBt.p, c.posB.p,
                              c.posT.p, c.stream);
    c.first_touch_A = mark_first_touch(c.color_cells.p, c.color_ptr, 729, c.posA.p, n_cells,
                                       Ac.size(), c.stream, &c.touched_A);
    c.first_touch_Bt = mark_first_touch(c.color_cells.p, c.color_ptr, 216, c.posBt.p, n_cells,
                                        Btc.size(), c.stream, &c.touched_Bt);
    c.first_touch_B = mark_first_touch(c.color_cells.p, c.color_ptr, 216, c.posB.p, n_cells,
                                       Bc.size(), c.stream, &c.touched_B);
    {
      // matrix-free operator: first-touch bits in colour order, constrained
      // velocity dofs with the position of their assembled diagonal entry,
      // per-point geometry
      std::vector<uint64_t> first(n_cells, 0);
      std::vector<int32_t> oq2(size_t(n_cells) * 27), op(size_t(n_cells) * 8);
      std::vector<uint8_t> vt(nv, 0), pt(n_p, 0);
      for (size_t e = 0; e < ccells.size(); ++e) {
        const int cell = ccells[e];
        uint64_t bits = 0;
        for (int t = 0; t < 27; ++t) {
          const int n = q2[27 * size_t(cell) + t];
          oq2[27 * e + t] = n;
          if (!vt[n]) { vt[n] = 1; bits |= uint64_t(1) << t; }
        }
        for (int v = 0; v < 8; ++v) {
          const int p = pd[8 * size_t(cell) + v];
          op[8 * e + v] = p;
          if (!pt[p]) { pt[p] = 1; bits |= uint64_t(1) << (32 + v); }
        }
        first[e] = bits;
      }
      c.mf_q2.upload(oq2);
      c.mf_p.upload(op);
      // constrained velocity nodes: index into con_diag (3 per node)
      std::vector<int32_t> cdof, cidx(nv, -1), img_node;
      std::vector<int64_t> cpos, img_blk;
      int n_con = 0;
      for (int n = 0; n < nv; ++n) {
        if (vc[n].type == 0) continue;
        const auto* b = std::lower_bound(Ac.data() + Ap[n], Ac.data() + Ap[n + 1], n);
        require(b != Ac.data() + Ap[n + 1] && *b == n, DCP_ERR_INVALID, "A pattern lacks a diagonal block");
        cidx[n] = n_con;
        for (int comp = 0; comp < 3; ++comp)
          if (vc[n].type == 1 || vc[n].type == 3 || comp == vc[n].k) {
            cdof.push_back(3 * n + comp);
            cpos.push_back(3 * int64_t(n_con) + comp);
          }
        if (vc[n].type == 3) {
          img_node.push_back(n);
          img_blk.push_back(b - Ac.data());
        }
        ++n_con;
      }
      // periodic pressure images after the velocity nodes in con_diag (and in
      // the colour path's fix-up list, which the velocity-only apply cuts short)
      c.mf_ncon_v = int(cdof.size());
      std::vector<int32_t> pcidx(n_p, -1);
      int n_pimg = 0;
      for (int i = 0; i < n_p; ++i)
        if (h.pmaster[i] >= 0) {
          pcidx[i] = n_pimg;
          cdof.push_back(n_u + i);
          cpos.push_back(3 * int64_t(n_con) + n_pimg);
          ++n_pimg;
        }
      c.mf_cidx.upload(cidx);
      c.n_con = n_con;
      c.con_diag.alloc(3 * size_t(n_con) + n_pimg);
      c.periodic = h.n_vslave || h.n_pslave || h.n_tslave;
      if (c.periodic) {
        c.pcidx.upload(pcidx);
        c.cell_q2o.upload(h.q2o);
        c.cell_po.upload(h.pdo);
        c.cell_To.upload(h.tdo);
        std::vector<int32_t> iu, mu, ip, mp, iT, mT;
        for (int n = 0; n < nv; ++n)
          if (h.vmaster[n] >= 0)
            for (int comp = 0; comp < 3; ++comp) {
              iu.push_back(3 * n + comp);
              mu.push_back(3 * h.vmaster[n] + comp);
            }
        for (int i = 0; i < n_p; ++i)
          if (h.pmaster[i] >= 0) {
            ip.push_back(n_u + i);
            mp.push_back(n_u + h.pmaster[i]);
          }
        for (int t = 0; t < n_T; ++t)
          if (h.tmaster[t] >= 0) {
            iT.push_back(t);
            mT.push_back(h.tmaster[t]);
          }
        c.img_u.upload(iu);
        c.mst_u.upload(mu);
        c.img_p.upload(ip);
        c.mst_p.upload(mp);
        c.img_T.upload(iT);
        c.mst_T.upload(mT);
        c.n_img_u = int(iu.size());
        c.n_img_p = int(ip.size());
        c.n_img_T = int(iT.size());
        c.img_node.upload(img_node);
        c.img_blk.upload(img_blk);
        c.n_img_node = int(img_node.size());
        std::vector<int32_t> pts(size_t(n_cells) * 8, -1);
        for (int cell = 0; cell < n_cells; ++cell)
          for (int v = 0; v < 8; ++v) {
            const int o = h.tdo[8 * size_t(cell) + v];
            if (o == td[8 * size_t(cell) + v]) continue;
            const auto* b = std::lower_bound(Tc.data() + Tp[o], Tc.data() + Tp[o + 1], o);
            pts[8 * size_t(cell) + v] = int32_t(b - Tc.data());
          }
        c.posTs.upload(pts);
      }
      c.mf_first.upload(first);
      c.mf_cdof.upload(cdof);
      c.mf_cpos.upload(cpos);
      c.mf_ncon = int(cdof.size());
      c.mf_geo.release();  // colour-launch mode only: computed on its first use
      // cell-order path: constrained-node masks, per-dof lists of partial sums
      // (velocity: one per cell group touching the node, pressure: one per
      // cell; ascending cell order = the gather's summation order)
      // chunks of the cell range; a dof is gathered after the chunk of its last cell
      if (const char* e = std::getenv("DCP_MF_CHUNKS"))
        c.mf_chunks = std::max(1, std::min(Ctx::kMfChunksMax, std::atoi(e)));
      const int K = c.mf_chunks;
      c.mf_cell_cut.assign(K + 1, 0);
      for (int k = 0; k <= K; ++k) c.mf_cell_cut[k] = int(int64_t(n_cells) * k / K);
      // cell groups: kMfGroupCells consecutive cells from each chunk's first cell
      std::vector<int32_t> group_first(n_cells);  // first cell of the cell's group
      for (int k = 0; k < K; ++k)
        for (int cell = c.mf_cell_cut[k]; cell < c.mf_cell_cut[k + 1]; ++cell)
          group_first[cell] = cell - (cell - c.mf_cell_cut[k]) % kMfGroupCells;
      // per (cell, t): the owner is the node's first occurrence in its group (one
      // partial sum per group, gathered in group order); later occurrences are
      // chained to it in (cell, t) order by their group-local index 27 (cell - first) + t
      std::vector<uint32_t> cmask(n_cells, 0);
      std::vector<int32_t> vptr(nv + 1, 0), pptr(n_p + 1, 0);
      std::vector<MfLink> vnext(27 * size_t(n_cells), kMfLinkEnd);
      std::vector<char> vowner(27 * size_t(n_cells), 0);
      {
        std::vector<int> prev(nv, -1), prev_group(nv, -1);
        for (int cell = 0; cell < n_cells; ++cell) {
          const int g = group_first[cell];
          for (int t = 0; t < 27; ++t) {
            const size_t occ = 27 * size_t(cell) + t;
            const int n = q2[occ];
            if (vc[n].type != 0) cmask[cell] |= 1u << t;
            if (prev_group[n] == g) {
              vnext[size_t(prev[n])] = MfLink(27 * (cell - g) + t);
            } else {
              vowner[occ] = 1;
              vptr[n + 1]++;
              prev_group[n] = g;
            }
            prev[n] = int(occ);
          }
          for (int v = 0; v < 8; ++v) pptr[pd[8 * size_t(cell) + v] + 1]++;
        }
      }
      for (int n = 0; n < nv; ++n) vptr[n + 1] += vptr[n];
      for (int i = 0; i < n_p; ++i) pptr[i + 1] += pptr[i];
      std::vector<int> vlast(nv, 0), plast(n_p, 0);
      for (int k = 0; k < K; ++k)
        for (int cell = c.mf_cell_cut[k]; cell < c.mf_cell_cut[k + 1]; ++cell) {
          for (int t = 0; t < 27; ++t) vlast[q2[27 * size_t(cell) + t]] = k;
          for (int v = 0; v < 8; ++v) plast[pd[8 * size_t(cell) + v]] = k;
        }
      // gather order: by last chunk, then id (stable counting sort)
      auto order_of = [&](const std::vector<int>& last, std::vector<int32_t>& order,
                          std::vector<int>& cut) {
        cut.assign(K + 1, 0);
        for (int l : last) cut[l + 1]++;
        for (int k = 0; k < K; ++k) cut[k + 1] += cut[k];
        order.assign(last.size(), 0);
        std::vector<int> f(cut.begin(), cut.end() - 1);
        for (size_t i = 0; i < last.size(); ++i) order[f[last[i]]++] = int32_t(i);
      };
      std::vector<int32_t> vorder, porder;
      order_of(vlast, vorder, c.mf_vcut);
      order_of(plast, porder, c.mf_pcut);
      // slot ranges per gather position
      std::vector<int32_t> vptr_o(nv + 1, 0), pptr_o(n_p + 1, 0), vpos(nv), ppos(n_p);
      for (int i = 0; i < nv; ++i) {
        vpos[vorder[i]] = i;
        vptr_o[i + 1] = vptr_o[i] + (vptr[vorder[i] + 1] - vptr[vorder[i]]);
      }
      for (int i = 0; i < n_p; ++i) {
        ppos[porder[i]] = i;
        pptr_o[i + 1] = pptr_o[i] + (pptr[porder[i] + 1] - pptr[porder[i]]);
      }
      vptr.swap(vptr_o);
      pptr.swap(pptr_o);
      require(int64_t(n_cells) * 89 < (int64_t(1) << 31), DCP_ERR_UNSUPPORTED,
              "mesh too large for 32-bit incidence slots");
      const int32_t pbase = 3 * vptr[nv];
      std::vector<int32_t> vslot(27 * size_t(n_cells)), pslot(8 * size_t(n_cells));
      {
        std::vector<int32_t> vf(nv), pf(n_p);
        for (int n = 0; n < nv; ++n) vf[n] = vptr[vpos[n]];
        for (int i = 0; i < n_p; ++i) pf[i] = pptr[ppos[i]];
        for (int cell = 0; cell < n_cells; ++cell) {
          for (int t = 0; t < 27; ++t) {
            const size_t occ = 27 * size_t(cell) + t;
            vslot[occ] = vowner[occ] ? 3 * vf[q2[occ]]++ : -1;
          }
          for (int v = 0; v < 8; ++v)
            pslot[8 * size_t(cell) + v] = pbase + pf[pd[8 * size_t(cell) + v]]++;
        }
      }
      c.mf_vorder.upload(vorder);
      c.mf_porder.upload(porder);
      {
        // 64-position blocks of the gather order that hold a constrained node
        std::vector<uint8_t> wcon((size_t(nv) + 63) / 64, 0);
        for (int i = 0; i < nv; ++i)
          if (cidx[size_t(vorder[i])] >= 0) wcon[size_t(i) >> 6] = 1;
        c.mf_wcon.upload(wcon);
      }
      if (!c.mf_stream) {
        DCP_HIP_CHECK(hipStreamCreateWithFlags(&c.mf_stream, hipStreamNonBlocking));
        for (auto& ev : c.mf_chunk_ev)
          DCP_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        DCP_HIP_CHECK(hipEventCreateWithFlags(&c.mf_join_ev, hipEventDisableTiming));
      }
      build_mf_fused(c, n_cells, nv, n_p, vptr, pptr, vslot, pslot, pbase);
      c.mf_cmask.upload(cmask);
      c.mf_vptr.upload(vptr);
      c.mf_vslot.upload(vslot);
      c.mf_vnext.upload(vnext);
      c.mf_pbase = pbase;
      c.mf_pptr.upload(pptr);
      c.mf_pslot.upload(pslot);
      c.mf_buf.alloc(size_t(pbase) + size_t(pptr[n_p]));
      {
        std::vector<int32_t> col, layer;
        std::vector<double> colgeo, laygeo, colphi, layR;
        c.mf_separable = separable_geometry(
            n_cells, [&](int cell, int t) { return &h.geo[3 * kMapPts * size_t(cell) + 3 * t]; },
            col, colgeo, layer, laygeo, &colphi, &layR);
        if (c.mf_separable) {
          c.mf_col.upload(col);
          c.mf_colgeo.upload(colgeo);
          c.mf_layer.upload(layer);
          c.mf_laygeo.upload(laygeo);
          c.mf_colphi.upload(colphi);
          c.mf_layR.upload(layR);
          // the rhs gravity -g x / den(|x|), x = R Phi, den(r) = r (r > 1) or
          // sqrt(r): per column point |Phi|, 1 / |Phi|, 1 / sqrt|Phi|, per
          // layer point sqrt(R) (k_mf_pencil<.., RHS>: no square root or
          // division on the device)
          std::vector<double> pn(colphi.size()), rs(layR.size());
          for (size_t i = 0; i < colphi.size() / 3; ++i) {
            const double* f = &colphi[3 * i];
            const double a = std::sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
            pn[3 * i] = a;
            pn[3 * i + 1] = 1.0 / a;
            pn[3 * i + 2] = 1.0 / std::sqrt(a);
          }
          for (size_t i = 0; i < layR.size(); ++i) rs[i] = std::sqrt(layR[i]);
          c.mf_colphin.upload(pn);
          c.mf_layRs.upload(rs);
          // the temperature system in Kronecker form (kernels/temperature_sep.hip);
          // DCP_T_SEPARABLE=0 keeps the colour kernels
          const char* env_ts = std::getenv("DCP_T_SEPARABLE");
          if (!c.periodic && h.tdpc == 8 && !(env_ts && *env_ts == '0'))
            build_tsep(c, n_cells, td, col, layer, layR, Tfix, Tbc, Tp, Tc, n_T);
        } else {
          // general mesh: J^-1 / JxW per Gauss point, tree order (2160 B per cell)
          c.mf_geo_tree.alloc(size_t(n_cells) * 270);
          mf_geometry(c.cd(), nullptr, c.mf_geo_tree.p, c.stream);
        }
        // B^T by tasks of rows (k_bt_tasks) on the separable shell: per velocity
        // node row its cells in colour order (cell << 5 | lexicographic position)
        c.bt_rows = false;
        c.rhs_cell_order = false;
        const char* env = std::getenv("DCP_BT_ROWS");
        const char* env_rhs = std::getenv("DCP_ASM_RHS_CELL_ORDER");
        // (B is then read as the transpose of B^T: every local B entry must have
        // its B^T entry, c.B_transpose)
        if (c.mf_separable && !c.periodic && c.B_transpose && !(env && *env == '0') &&
            n_cells < (1 << 26)) {
          const int nrows = int(Btp.size()) - 1;
          std::vector<int32_t> rp(size_t(nrows) + 1, 0);
          for (const int cell : ccells)
            for (int t = 0; t < 27; ++t) {
              const int n = q2[27 * size_t(cell) + t];
              if (n < nrows) rp[n + 1]++;
            }
          int most = 0;
          for (int n = 0; n < nrows; ++n) {
            most = std::max(most, rp[n + 1]);
            rp[n + 1] += rp[n];
          }
          if (most <= 8 && *std::max_element(layer.begin(), layer.end()) < 65536) {
            // one wave: 8 cells x 8 vertices (27 nodes)
            std::vector<int32_t> inc(static_cast<size_t>(rp[nrows]));
            std::vector<int32_t> f(rp.begin(), rp.end() - 1);
            for (const int cell : ccells)
              for (int t = 0; t < 27; ++t) {
                const int n = q2[27 * size_t(cell) + t];
                if (n < nrows) inc[size_t(f[n]++)] = int32_t(cell) << 5 | t;
              }
            // tasks: runs of consecutive rows with <= SL slots and <= 64
            // entries (SL = 16: two records per lane; DCP_BT_SLOTS=8: one; =32: four, 128 entries)
            const char* env_sl = std::getenv("DCP_BT_SLOTS");
            const int SL = env_sl && (std::atoi(env_sl) == 8 || std::atoi(env_sl) == 32)
                               ? std::atoi(env_sl) : 16;
            const int NE = SL == 32 ? 128 : 64, FB = SL == 32 ? 7 : 6;  // entries, field bits
            std::vector<int32_t> hdr, rec;
            int first = 0, ns = 0, ne = 0, rec0 = 0;
            // SL slot records per task (unused ones zero): a lane loads its
            // records at SL task + slot without waiting for the header
            auto flush = [&](int next_row) {
              if (next_row > first) {
                hdr.insert(hdr.end(), {Btp[first], first, ns | ne << 8, rec0});
                rec.resize(size_t(rec0 + SL) * 4, 0);
              }
              first = next_row;
              ns = ne = 0;
              rec0 = int32_t(rec.size() / 4);
            };
            for (int n = 0; n < nrows; ++n) {
              const int cnt = rp[n + 1] - rp[n], len = Btp[n + 1] - Btp[n];
              require(cnt <= 8 && len <= 64, DCP_ERR_INVALID, "B^T task sizes");
              if (ns + cnt > SL || ne + len > NE) flush(n);
              for (int k = rp[n]; k < rp[n + 1]; ++k) {
                const int cell = inc[size_t(k)] >> 5, lex = inc[size_t(k)] & 31;
                uint64_t dm = 0;
                int dest[8];
                for (int v = 0; v < 8; ++v) {
                  const int q = pd[8 * size_t(cell) + v];
                  const int32_t* b = Btc.data() + Btp[n];
                  const int32_t* e = Btc.data() + Btp[n + 1];
                  const int32_t* it = std::lower_bound(b, e, q);
                  require(it != e && *it == q, DCP_ERR_INVALID, "B^T pattern lacks a cell's entry");
                  dest[v] = int(ne + (it - b));
                  // k_bt_tasks keeps one vertex per (slot, entry): a cell whose
                  // vertices share a pressure dof (identified vertices) would
                  // lose a contribution, so refuse it here
                  for (int w = 0; w < v; ++w)
                    require(dest[w] != dest[v], DCP_ERR_INVALID,
                            "B^T task: two vertices of a cell map to one entry");
                  dm |= uint64_t(dest[v]) << (FB * v);
                }
                // bit 15: the row's node is constrained (the entry lanes load its
                // NodeConstraint only then; unconstrained rows condense by identity)
                const int con = vc[n].type != 0 ? 1 << 15 : 0;
                rec.insert(rec.end(), {col[size_t(cell)], layer[size_t(cell)] << 16 | con | lex << 8 | (n - first),
                                       int32_t(uint32_t(dm)), int32_t(uint32_t(dm >> 32))});
                ++ns;
              }
              ne += len;
            }
            flush(nrows);
            c.bt_task_hdr.upload(hdr);
            c.bt_slot_rec.upload(rec);
            c.bt_ntasks = int(hdr.size() / 4);
            c.bt_slots = SL;
            // several GPUs: the rhs / constrained diagonal are read on owned rows
            // only, so the cell kernel runs over the cells with an owned
            // velocity node (owned cells + the first ghost layer), per colour
            c.rhs_color_ptr.clear();
            c.rhs_color_cells.release();
            if (dist || nrows < nv) {
              std::vector<int32_t> sub;
              c.rhs_color_ptr.assign(1, 0);
              for (size_t k = 0; k + 1 < h.color_ptr.size(); ++k) {
                for (int e = h.color_ptr[k]; e < h.color_ptr[k + 1]; ++e) {
                  const int cell = ccells[size_t(e)];
                  bool own = false;
                  for (int t = 0; t < 27 && !own; ++t) own = q2[27 * size_t(cell) + t] < nrows;
                  if (own) sub.push_back(cell);
                }
                c.rhs_color_ptr.push_back(int(sub.size()));
              }
              c.rhs_color_cells.upload(sub);
            }
            // the rhs in cell order (mf_rhs_cells + the velocity gather) with
            // FE_Q(1) temperature; the cell kernel then only forms the
            // constrained-row diagonals, on the cells with a constrained node
            // (and an owned node, several GPUs)
            c.con_color_ptr.clear();
            c.con_color_cells.release();
            c.rhs_cell_order = h.tdpc == 8 && !(env_rhs && *env_rhs == '0');
            // per slot: (lateral, radial) table indices; per node: constrained components
            std::vector<int32_t> cdk_rec, cdk_mask;
            if (c.rhs_cell_order) {
              std::vector<int32_t> sub;
              c.con_color_ptr.assign(1, 0);
              for (size_t k = 0; k + 1 < h.color_ptr.size(); ++k) {
                for (int e = h.color_ptr[k]; e < h.color_ptr[k + 1]; ++e) {
                  const int cell = ccells[size_t(e)];
                  bool own = false;
                  for (int t = 0; t < 27 && !own; ++t) own = q2[27 * size_t(cell) + t] < nrows;
                  if (cmask[size_t(cell)] != 0 && own) sub.push_back(cell);
                }
                c.con_color_ptr.push_back(int(sub.size()));
              }
              c.con_color_cells.upload(sub);
              // one launch over the list: per (list cell, node) of a constrained
              // node its slot, slots of a node in list (= colour) order
              std::vector<int32_t> cptr(size_t(n_con) + 1, 0), cslot(27 * sub.size(), -1);
              for (const int cell : sub)
                for (int t = 0; t < 27; ++t) {
                  const int ci = cidx[size_t(q2[27 * size_t(cell) + t])];
                  if (ci >= 0) cptr[size_t(ci) + 1]++;
                }
              for (int i = 0; i < n_con; ++i) cptr[i + 1] += cptr[i];
              std::vector<int32_t> fill(cptr.begin(), cptr.end() - 1);
              for (size_t k = 0; k < sub.size(); ++k)
                for (int t = 0; t < 27; ++t) {
                  const int ci = cidx[size_t(q2[27 * size_t(sub[k]) + t])];
                  if (ci >= 0) cslot[27 * k + t] = fill[size_t(ci)]++;
                }
              c.con_cptr.upload(cptr);
              c.con_cslot.upload(cslot);
              c.con_cbuf.alloc(3 * size_t(std::max(cptr[n_con], 1)));
              cdk_rec.assign(2 * size_t(cptr[n_con]), 0);
              cdk_mask.assign(size_t(n_con), 0);
              for (size_t k = 0; k < sub.size(); ++k)
                for (int t = 0; t < 27; ++t) {
                  const int sl = cslot[27 * k + t];
                  if (sl < 0) continue;
                  cdk_rec[2 * size_t(sl)] = 9 * col[size_t(sub[k])] + t % 9;
                  cdk_rec[2 * size_t(sl) + 1] = 3 * layer[size_t(sub[k])] + t / 9;
                  const int nd = q2[27 * size_t(sub[k]) + t];
                  const NodeConstraint& nc = vc[size_t(nd)];
                  cdk_mask[size_t(cidx[size_t(nd)])] =
                      nc.type == 1 || nc.type == 3 ? 7 : (nc.type == 2 ? 1 << nc.k : 0);
                }
            }
            // the column factors P of the B^T entries are mesh geometry
            // (the column tables, reference functions): formed once here
            c.bt_ncols = int(c.mf_colgeo.n / 90);
            const int nlay = int(c.mf_laygeo.n / 9);
            c.bt_P.alloc(size_t(216) * c.bt_ncols + size_t(12) * nlay);
            c.bt_Q = c.bt_P.p + size_t(216) * c.bt_ncols;
            launch_bt_rows(c.cd(), c.bt_ncols, nlay, c.bt_P.p, c.bt_Q, 0, c.bt_slots, nullptr,
                           nullptr, nullptr, c.stream);
            c.bt_rows = true;
            // one GPU: B^T in Kronecker form instead of the tasks
            // (kernels/bt_kron.hip; DCP_BT_KRON=0 keeps the tasks)
            const char* env_bk = std::getenv("DCP_BT_KRON");
            c.btk = false;
            if (!dist && nrows == nv && c.B_transpose && !(env_bk && *env_bk == '0'))
              build_btk(c, n_cells, q2, pd, col, layer, layR, vc, Btp, Btc, nv, n_p);
            // with it the constrained diagonals in Kronecker form (k_cdk_*;
            // DCP_CDIAG_KRON=0 keeps the cell pass + con_gather)
            const char* env_cd = std::getenv("DCP_CDIAG_KRON");
            if (c.btk && c.rhs_cell_order && !cdk_rec.empty() && !(env_cd && *env_cd == '0')) {
              c.cdk_rec.upload(cdk_rec);
              c.cdk_mask.upload(cdk_mask);
              c.cdk_L.alloc(size_t(90) * c.bt_ncols);
              c.cdk_R.alloc(size_t(12) * nlay);
              cdk_tables(c.mf_colgeo.p, c.bt_ncols, c.mf_laygeo.p, nlay, c.cdk_L.p, c.cdk_R.p,
                         c.stream);
              c.cdk = true;
            }
          }
        }
      }
    }
    const size_t nn = size_t(n_u + n_p);
    c.nse_sol.alloc(nn);
    c.old_nse.alloc(nn);
    c.nse_rhs.alloc(nn);
    c.T_sol.alloc(n_T);
    c.old_T.alloc(n_T);
    c.T_rhs.alloc(n_T);
    for (auto* b : {&c.nse_sol, &c.old_nse, &c.nse_rhs, &c.T_sol, &c.old_T, &c.T_rhs}) b->zero(c.stream);
    c.A_diag.alloc(n_u);
    c.Mp_diag.alloc(n_p);
    c.A_inv.alloc(n_u);
    c.Mp_inv.alloc(n_p);
    c.T_inv.alloc(n_T);
    c.schur_tmp1.alloc(n_u);
    c.schur_tmp2.alloc(n_u);
    c.utmp.alloc(n_u);
    c.fg_aux.alloc(nn);
    free_workspaces(c);
    // ---- multi-GPU: halo plans and the common widths of all-reduced partials
    c.max_owned[0] = 3 * c.nvo + c.npo;
    c.max_owned[1] = c.npo;
    c.max_owned[2] = 3 * c.nvo;
    c.max_owned[3] = c.nTo;
    if (dist) {
      build_halos(c, L);
      double m[5] = {double(c.max_owned[0]), double(c.max_owned[1]), double(c.max_owned[2]),
                     double(c.max_owned[3]), double(c.sell_part_len)};
      double* d = c.dscal.p + 3500;
      DCP_HIP_CHECK(hipMemcpyAsync(d, m, sizeof(m), hipMemcpyHostToDevice, c.stream));
      c.comm->allreduce(d, 5, true, c.stream);
      DCP_HIP_CHECK(hipMemcpyAsync(m, d, sizeof(m), hipMemcpyDeviceToHost, c.stream));
      DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
      for (int k = 0; k < 4; ++k) c.max_owned[k] = int(m[k]);
      c.sell_part_len = int(m[4]);
    }
    c.sell_part.alloc(2 * size_t(std::max(c.sell_part_len, 1)));
    c.sell_part.zero(c.stream);  // entries past this rank's slices stay 0
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    c.have_mesh = true;
    c.nse_assembled = c.precond_built = c.T_matrix_ok = c.T_rhs_ok = false;
}

extern "C" {

int dcp_mesh_upload(dcp_ctx* ctx, int n_cells, const int32_t* cell_nse_dofs,
                    const int32_t* cell_T_dofs, const double* cell_geometry,
                    const double* cell_diameter, int n_u, int n_p, int n_T,
                    const dcp_constraints* nse_c, const dcp_constraints* T_c) {
  return guarded(ctx, [&] {
    require(ctx != nullptr, DCP_ERR_INVALID, "NULL context");
    Ctx& c = *ctx;
    HostPrep h;
    const bool dist = c.comm != nullptr;
    LocalMesh L;
    const int n_u_g = n_u, n_p_g = n_p, n_T_g = n_T;
    if (dist) {
      // this rank's cells + two ghost layers in local numbering (partition.h)
      try {
        L = localize(n_cells, cell_nse_dofs, cell_T_dofs, cell_geometry, cell_diameter, n_u, n_p,
                     n_T, nse_c, T_c, c.cfg.rank, c.cfg.world_size);
      } catch (const std::runtime_error& e) {
        fail(DCP_ERR_INVALID, e.what());
      }
      const dcp_constraints lnc = L.nse_view(), ltc = L.T_view();
      const std::vector<int> hint =
          partition_colour_hint(n_cells, cell_nse_dofs, cell_geometry, n_u, n_p, L.cells_g);
      n_cells = L.n_cells;
      n_u = L.n_u();
      n_p = L.n_p();
      n_T = L.n_T();
      cell_diameter = L.diameter.data();
      prepare_mesh(h, n_cells, L.cell_nse_dofs.data(), L.cell_T_dofs.data(), L.geometry.data(),
                   cell_diameter, n_u, n_p, n_T, &lnc, &ltc, &hint);
    } else {
      prepare_mesh(h, n_cells, cell_nse_dofs, cell_T_dofs, cell_geometry, cell_diameter, n_u,
                   n_p, n_T, nse_c, T_c);
    }
    upload_prepared(c, h, L, dist, n_cells, cell_diameter, n_u, n_p, n_T, n_u_g, n_p_g, n_T_g);
    return DCP_OK;
  });
}

int dcp_mesh_upload_distributed(dcp_ctx* ctx, const dcp_dist_mesh* m, const dcp_host_comm* comm) {
  return guarded(ctx, [&] {
    require(ctx && m && comm, DCP_ERR_INVALID, "NULL argument");
    Ctx& c = *ctx;
    require(comm->world == c.cfg.world_size && comm->rank == c.cfg.rank, DCP_ERR_INVALID,
            "host communicator rank/world differ from the context's");
    LocalMesh L;
    try {
      L = localize_distributed(*m, *comm);
    } catch (const std::runtime_error& e) {
      fail(DCP_ERR_INVALID, e.what());
    }
    const dcp_constraints lnc = L.nse_view(), ltc = L.T_view();
    HostPrep h;
    prepare_mesh(h, L.n_cells, L.cell_nse_dofs.data(), L.cell_T_dofs.data(), L.geometry.data(),
                 L.diameter.data(), L.n_u(), L.n_p(), L.n_T(), &lnc, &ltc);
    require(!(h.n_vslave || h.n_pslave || h.n_tslave), DCP_ERR_UNSUPPORTED,
            "periodic constraints on several GPUs are not supported");
    // one GPU (world 1): the caller's whole mesh, no halos
    upload_prepared(c, h, L, c.comm != nullptr, L.n_cells, L.diameter.data(), L.n_u(), L.n_p(),
                    L.n_T(), int(m->n_u), int(m->n_p), int(m->n_T));
    return DCP_OK;
  });
}

// the owned segments [offset, offset + count) of a state field's local vector
static std::vector<std::pair<size_t, size_t>> owned_segments(const Ctx& c, int field) {
  if (field == DCP_T_SOLUTION || field == DCP_OLD_T_SOLUTION || field == DCP_T_RHS)
    return {{0, size_t(c.nTo)}};
  if (c.feec)
    return {{0, size_t(c.fe_nwo)}, {size_t(c.fe_nw), size_t(c.fe_nuo)},
            {size_t(c.fe_nw + c.fe_nu), size_t(c.fe_npo)}};
  return {{0, size_t(c.vdim) * c.nvo}, {size_t(c.n_u), size_t(c.npo)}};
}

int dcp_state_set_owned(dcp_ctx* ctx, int field, const double* host, size_t n) {
  return guarded(ctx, [&] {
    require(ctx && host && ctx->have_mesh, DCP_ERR_STATE, "mesh not uploaded");
    Ctx& c = *ctx;
    size_t want = 0;
    double* p = field_ptr(c, field, want, true);
    const auto segs = owned_segments(c, field);
    size_t total = 0;
    for (auto& sgm : segs) total += sgm.second;
    require(n == total, DCP_ERR_INVALID, "owned state size mismatch");
    size_t o = 0;
    for (auto& sgm : segs) {
      if (sgm.second)
        DCP_HIP_CHECK(hipMemcpyAsync(p + sgm.first, host + o, sgm.second * sizeof(double),
                                     hipMemcpyHostToDevice, c.stream));
      o += sgm.second;
    }
    // ghost entries from their owners (the Trilinos ghosted copy)
    const bool T = field == DCP_T_SOLUTION || field == DCP_OLD_T_SOLUTION || field == DCP_T_RHS;
    if (c.comm) halo_exchange(c, T ? c.halo_T : c.halo_nse, p);
    mark_old_ghosted(c, field);
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    return DCP_OK;
  });
}

int dcp_state_get_owned(dcp_ctx* ctx, int field, double* host, size_t n) {
  return guarded(ctx, [&] {
    require(ctx && host && ctx->have_mesh, DCP_ERR_STATE, "mesh not uploaded");
    Ctx& c = *ctx;
    size_t want = 0;
    double* p = field_ptr(c, field, want, false);
    const auto segs = owned_segments(c, field);
    size_t total = 0;
    for (auto& sgm : segs) total += sgm.second;
    require(n == total, DCP_ERR_INVALID, "owned state size mismatch");
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    size_t o = 0;
    for (auto& sgm : segs) {
      if (sgm.second)
        DCP_HIP_CHECK(hipMemcpy(host + o, p + sgm.first, sgm.second * sizeof(double),
                                hipMemcpyDeviceToHost));
      o += sgm.second;
    }
    return DCP_OK;
  });
}

int dcp_state_set(dcp_ctx* ctx, int field, const double* host, size_t n) {
  return guarded(ctx, [&] {
    require(ctx && host && ctx->have_mesh, DCP_ERR_STATE, "mesh not uploaded");
    size_t want = 0;
    double* p = field_ptr(*ctx, field, want, true);
    if (ctx->comm) {
      // global vector in, local (owned + ghost) entries uploaded
      const bool T = field == DCP_T_SOLUTION || field == DCP_OLD_T_SOLUTION || field == DCP_T_RHS;
      require(n == size_t(T ? ctx->n_T_g : ctx->n_u_g + ctx->n_p_g), DCP_ERR_INVALID,
              "state size mismatch (several GPUs: pass the global vector)");
      const std::vector<int64_t> g = global_positions(*ctx, field);
      std::vector<double> loc(want);
      for (size_t i = 0; i < want; ++i) loc[i] = host[g[i]];
      DCP_HIP_CHECK(hipMemcpy(p, loc.data(), want * sizeof(double), hipMemcpyHostToDevice));
      mark_old_ghosted(*ctx, field);
      return DCP_OK;
    }
    require(n == want, DCP_ERR_INVALID, "state size mismatch");
    DCP_HIP_CHECK(hipMemcpyAsync(p, host, n * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    DCP_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return DCP_OK;
  });
}

int dcp_state_get(dcp_ctx* ctx, int field, double* host, size_t n) {
  return guarded(ctx, [&] {
    require(ctx && host && ctx->have_mesh, DCP_ERR_STATE, "mesh not uploaded");
    size_t want = 0;
    double* p = field_ptr(*ctx, field, want, false);
    if (ctx->comm) {
      // owned entries written into the global vector, the rest untouched
      const bool T = field == DCP_T_SOLUTION || field == DCP_OLD_T_SOLUTION || field == DCP_T_RHS;
      require(n == size_t(T ? ctx->n_T_g : ctx->n_u_g + ctx->n_p_g), DCP_ERR_INVALID,
              "state size mismatch (several GPUs: pass the global vector)");
      DCP_HIP_CHECK(hipStreamSynchronize(ctx->stream));
      std::vector<double> loc(want);
      DCP_HIP_CHECK(hipMemcpy(loc.data(), p, want * sizeof(double), hipMemcpyDeviceToHost));
      const std::vector<int64_t> g = global_positions(*ctx, field);
      for (size_t i = 0; i < want; ++i)
        if (owned_entry(*ctx, field, i)) host[g[i]] = loc[i];
      return DCP_OK;
    }
    require(n == want, DCP_ERR_INVALID, "state size mismatch");
    DCP_HIP_CHECK(hipMemcpyAsync(host, p, n * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
    DCP_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    return DCP_OK;
  });
}

int dcp_state_copy(dcp_ctx* ctx, int dst_field, int src_field) {
  return guarded(ctx, [&] {
    require(ctx && ctx->have_mesh, DCP_ERR_STATE, "mesh not uploaded");
    size_t nd = 0, ns = 0;
    double* d = field_ptr(*ctx, dst_field, nd, true);
    double* s = field_ptr(*ctx, src_field, ns, false);
    require(nd == ns, DCP_ERR_INVALID, "state size mismatch");
    copy(int(nd), s, d, ctx->stream);
    if (dst_field == DCP_OLD_NSE_SOLUTION || dst_field == DCP_OLD_T_SOLUTION) {
      // old = new as the reference's ghosted assignment: owned entries copied,
      // ghosts imported from their owners (several GPUs)
      Ctx& c = *ctx;
      halo_exchange(c, dst_field == DCP_OLD_T_SOLUTION ? c.halo_T : c.halo_nse, d);
      mark_old_ghosted(c, dst_field);
    }
    return DCP_OK;
  });
}

double* dcp_state_device_ptr(dcp_ctx* ctx, int field) {
  if (!ctx || !ctx->have_mesh) return nullptr;
  if (field == DCP_OLD_NSE_SOLUTION || field == DCP_OLD_T_SOLUTION) ctx->old_external = true;
  size_t n = 0;
  try {
    return field_ptr(*ctx, field, n, true);
  } catch (...) {
    return nullptr;
  }
}

int dcp_assemble_nse_system(dcp_ctx* ctx, int flags) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(!ctx->feec, DCP_ERR_STATE, "FEEC mesh uploaded: use the dcp_feec_* calls");
    Ctx& c = *ctx;
    SectionScope sec(c, "   Assemble NSE system");
    PhaseTimer t(c, &c.timings.assemble_nse_ms);
    if (c.dim2) {
      if (!c.old_nse_ghosted) halo_exchange(c, c.halo_nse, c.old_nse.p);
      if (!c.old_T_ghosted) halo_exchange(c, c.halo_T, c.old_T.p);
      assemble_nse_2d(c, flags);
      t.stop();
      return DCP_OK;
    }
    const bool matrix = (flags & DCP_ASSEMBLE_MATRIX) != 0;
    // the velocity block is materialised only when something reads it
    const bool full = matrix && (c.assemble_A || c.matrix_free == 0);
    NseOut out{};
    bool bt_rows = false;
    if (matrix) {
      // first-touch scatter positions store instead of adding: no zero fill
      if (full) ensure_A_val(c);
      if (full && !c.first_touch_A) c.A_val.zero(c.stream);
      // operator form: B copied from B^T after the cell loop (c.B_transpose)
      const bool scatter_B = full || !c.B_transpose;
      // operator form on the separable shell: B^T by rows (k_bt_rows), the
      // cell kernel only the rhs and the constrained diagonals
      bt_rows = c.bt_rows && !full;
      if (!bt_rows && !c.first_touch_Bt) c.Bt_val.zero(c.stream);
      if (!bt_rows && scatter_B && !c.first_touch_B) c.B_val.zero(c.stream);
      // k_cdk_diag (below) assigns every constrained diagonal: no zero fill
      const bool cdk_all = c.cdk && bt_rows && c.rhs_cell_order && (flags & DCP_ASSEMBLE_RHS) &&
                           c.con_diag.n == 3 * size_t(c.n_con);
      if (!cdk_all) c.con_diag.zero(c.stream);
      out.A = full ? c.A_val.p : nullptr;
      out.Bt = bt_rows ? nullptr : c.Bt_val.p;
      out.B = scatter_B && !bt_rows ? c.B_val.p : nullptr;
      out.cdiag = c.con_diag.p;
      out.cidx = c.mf_cidx.p;
      out.pcdiag = c.con_diag.p + 3 * size_t(c.n_con);
      out.pcidx = c.periodic ? c.pcidx.p : nullptr;
    }
    // the rhs in cell order (operator form on the separable shell, FE_Q(1)
    // temperature): the pencil kernel + the velocity gather write every
    // velocity entry; the cell kernel forms only the constrained diagonals
    const bool rhs_co = (flags & DCP_ASSEMBLE_RHS) && c.bt_rows && c.rhs_cell_order && !full;
    if (flags & DCP_ASSEMBLE_RHS) {
      if (rhs_co)
        fill(c.n_p, 0.0, c.nse_rhs.p + c.n_u, c.stream);  // B rows: no rhs
      else
        c.nse_rhs.zero(c.stream);
      out.rhs = rhs_co ? nullptr : c.nse_rhs.p;
    }
    // ghosted old solutions (the reference reads the ghosted vectors, :583-589,
    // which its time loop imported at old = new): exchanged here only if the
    // old fields were written some other way since
    if (!c.old_nse_ghosted) halo_exchange(c, c.halo_nse, c.old_nse.p);
    if (!c.old_T_ghosted) halo_exchange(c, c.halo_T, c.old_T.p);
    const bool rhs_subset = bt_rows && !c.rhs_color_ptr.empty();
    // B^T (geometry only), the constrained diagonals and the rhs (state) are
    // independent: with DCP_ASM_OVERLAP the B^T tasks run on the second stream
    // beside the rhs launches (1: B^T launched first, 2: after the rhs
    // launches), or (3) the constrained-diagonal pass runs there while B^T
    // (launched first) and the rhs run on the main stream
    const char* env_ov = std::getenv("DCP_ASM_OVERLAP");
    const int overlap = bt_rows && rhs_co && c.mf_stream && env_ov ? std::atoi(env_ov) : 0;
    const hipStream_t bt_stream = overlap == 1 || overlap == 2 ? c.mf_stream : c.stream;
    const hipStream_t con_stream = overlap == 3 ? c.mf_stream : c.stream;
    auto launch_bt = [&] {
      if (c.btk)
        btk_assemble(c.btkd(), long(c.Bt_val.n / 3), c.vcon.p, c.Bt_val.p, bt_stream);
      else
        launch_bt_rows(c.cd(), 0, 0, c.bt_P.p, c.bt_Q, c.bt_ntasks, c.bt_slots, c.bt_task_hdr.p,
                       c.bt_slot_rec.p, c.Bt_val.p, bt_stream);
    };
    if (overlap) {
      DCP_HIP_CHECK(hipEventRecord(c.mf_chunk_ev[0], c.stream));
      DCP_HIP_CHECK(hipStreamWaitEvent(c.mf_stream, c.mf_chunk_ev[0], 0));
      if (overlap == 1) launch_bt();
    }
    if (overlap == 3 && !out.cdiag) launch_bt();  // nothing to overlap: B^T first anyway
    if (rhs_co && out.cdiag && c.cdk) {
      cdk_diag(c.n_con, c.con_cptr.p, c.cdk_rec.p, c.cdk_mask.p, c.cdk_L.p, c.cdk_R.p,
               c.ph.nu_sys, c.con_diag.p, con_stream);
      if (overlap == 3) launch_bt();
    } else if (rhs_co && out.cdiag) {
      // the constrained-row diagonals only: the cells with a constrained node
      // in one launch, per (cell, node) slots, summed per node in colour order
      NseOut oc = out;
      oc.cbuf = c.con_cbuf.p;
      oc.cslot = c.con_cslot.p;
      launch_nse_operator(c.cd(), c.maps(), c.con_color_cells.p, c.con_color_ptr.back(),
                          c.old_nse.p, c.old_T.p, c.ph, oc, con_stream);
      con_gather(c.n_con, c.con_cptr.p, c.con_cbuf.p, c.con_diag.p, con_stream);
      if (overlap == 3) launch_bt();
    }
    for (int k = 0; k < c.n_colors() && !rhs_co; ++k) {
      if (full)
        launch_nse_system(c.cd(), c.maps(), c.color_begin(k), c.color_size(k), c.old_nse.p,
                          c.old_T.p, c.ph, out, c.stream, c.element_mfma);
      else if (rhs_subset)
        launch_nse_operator(c.cd(), c.maps(), c.rhs_color_cells.p + c.rhs_color_ptr[k],
                            c.rhs_color_ptr[k + 1] - c.rhs_color_ptr[k], c.old_nse.p, c.old_T.p,
                            c.ph, out, c.stream);
      else
        launch_nse_operator(c.cd(), c.maps(), c.color_begin(k), c.color_size(k), c.old_nse.p,
                            c.old_T.p, c.ph, out, c.stream);
    }
    if (rhs_co) {
      const MfCells mc = c.mfc();
      MfGather g = c.mfg();
      g.cdiag = nullptr;  // condensation only
      g.pcidx = nullptr;
      if (c.mf_fused && c.hmapped) {
        if (++c.mf_seq == 0) ++c.mf_seq;
        mf_rhs_fused(mc, g, c.mff(c.hmapped + kMfErrSlot), c.mf_ntasks, c.old_nse.p, c.old_T.p,
                     c.ph, c.mf_buf.p, c.nse_rhs.p, c.mf_seq, c.stream);
      } else {
        for (int k = 0; k < c.mf_chunks; ++k)
          mf_rhs_cells(mc, c.mf_cell_cut[k], c.mf_cell_cut[k + 1], c.old_nse.p, c.old_T.p, c.ph,
                       c.mf_buf.p, c.nse_rhs.p, c.stream);
        mf_gather(g, 0, c.n_vnodes, 0, 0, false, c.mf_buf.p, nullptr, c.nse_rhs.p, c.stream);
      }
    }
    if (bt_rows && overlap != 1 && overlap != 3) launch_bt();
    if (overlap) {
      DCP_HIP_CHECK(hipEventRecord(c.mf_join_ev, c.mf_stream));
      DCP_HIP_CHECK(hipStreamWaitEvent(c.stream, c.mf_join_ev, 0));
    }
    if (full)
      image_diagonal_blocks(c.n_img_node, c.img_node.p, c.img_blk.p, c.mf_cidx.p, c.con_diag.p,
                            c.A_val.p, c.stream);
    t.stop();
    if (rhs_co && c.mf_fused && c.hmapped) {
      // the fused rhs's poll-timeout flag belongs to this call, not a later one
      DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
      check_mf_err(c);
    }
    if (matrix) {
      // else B = (B^T)^T, materialised when read
      c.B_current = out.B != nullptr;
      c.nse_assembled = true;
      c.A_current = full;
      c.nse_ph = c.ph;
    }
    return DCP_OK;
  });
}

int dcp_build_nse_preconditioner(dcp_ctx* ctx) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(!ctx->feec, DCP_ERR_STATE, "FEEC mesh uploaded: use the dcp_feec_* calls");
    Ctx& c = *ctx;
    SectionScope sec(c, "   Build NSE preconditioner");
    PhaseTimer t(c, &c.timings.build_precond_ms);
    if (c.dim2) {
      build_precond_2d(c);
      t.stop();
      c.precond_built = true;
      return DCP_OK;
    }
    {
      SectionScope sub(c, "   Assembly NSE preconditioner");
      c.A_diag.zero(c.stream);
      c.Mp_diag.zero(c.stream);
      for (int k = 0; k < c.n_colors(); ++k)
        launch_nse_precond_diag(c.cd(), c.color_begin(k), c.color_size(k), c.ph, c.A_diag.p,
                                c.Mp_diag.p, c.stream);
    }
    reciprocal(c.n_u, c.A_diag.p, c.A_inv.p, c.stream);
    reciprocal(c.n_p, c.Mp_diag.p, c.Mp_inv.p, c.stream);
    if (c.schur_explicit) {
      require(c.nse_assembled, DCP_ERR_STATE,
              "the explicit Schur complement needs the assembled B blocks: call "
              "dcp_assemble_nse_system first");
      // B read through B^T's transpose map unless B is materialised
      c.S_lambda = 0;  // the s-step shifts follow the new S
      form_schur_complement(c.npo, c.B_ptr.p, c.B_col.p, c.B_current ? c.B_val.p : nullptr,
                            c.B_current ? nullptr : c.B_tperm.p, c.Bt_ptr.p, c.Bt_col.p,
                            c.Bt_val.p, c.A_inv.p, c.S_ptr.p, c.S_col.p, c.S_pmap.p,
                            c.S_val.p, c.S_max_row, c.stream);
      ++c.S_version;
    }
    t.stop();
    c.precond_built = true;
    return DCP_OK;
  });
}

int dcp_assemble_temperature_matrix(dcp_ctx* ctx) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    SectionScope sec(c, "   Assemble temperature matrices");
    PhaseTimer t(c, &c.timings.assemble_T_matrix_ms);
    if (c.dim2) {
      assemble_T_matrix_2d(c);
      t.stop();
      c.T_matrix_ok = true;
      return DCP_OK;
    }
    c.ts_tmat_valid = false;
    if (c.tsep && !c.feec) {
      // Kronecker form: M, K, and T_matrix = M + dt K with its Jacobi inverse
      // (the first lines of assemble_temperature_rhs, :975-986) in one pass
      tsep_matrix(c.tsd(), long(c.Tmat.n), c.ph, c.Tmass.p, c.Tstiff.p, c.Tmat.p, c.T_inv.p,
                  c.stream);
      c.ts_tmat_valid = true;
      c.ts_tmat_dt = c.ph.dt_T;
    } else {
      c.Tmass.zero(c.stream);
      c.Tstiff.zero(c.stream);
      for (int k = 0; k < c.n_colors(); ++k)
        launch_T_matrix(c.cd(), c.maps(), c.color_begin(k), c.color_size(k), c.ph, c.Tmass.p,
                        c.Tstiff.p, c.periodic ? c.posTs.p : nullptr, c.stream);
    }
    t.stop();
    c.T_matrix_ok = true;
    return DCP_OK;
  });
}

int dcp_assemble_temperature_rhs(dcp_ctx* ctx) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(c.T_matrix_ok, DCP_ERR_STATE, "assemble the temperature matrices first");
    SectionScope sec(c, "   Assemble temperature RHS");
    PhaseTimer t(c, &c.timings.assemble_T_rhs_ms);
    // T_matrix = M + dt/interval K ; Jacobi rebuilt (:975-986), unless the
    // separable matrix assembly formed both with this dt
    if (!(c.ts_tmat_valid && c.ts_tmat_dt == c.ph.dt_T)) {
      lincomb(int(c.Tmat.n), c.Tmass.p, c.ph.dt_T, c.Tstiff.p, c.Tmat.p, c.stream);
      csr_diag_inverse(c.n_T, c.T_ptr.p, c.T_col.p, c.Tmat.p, c.T_inv.p, c.stream);
    }
    if (!c.old_T_ghosted) halo_exchange(c, c.halo_T, c.old_T.p);
    halo_exchange(c, c.halo_nse, c.nse_sol.p);
    if (c.tsep && !c.feec && !c.dim2) {
      tsep_rhs(c.tsd(), c.cd(), c.n_T, c.old_T.p, c.nse_sol.p, c.ph, c.T_rhs.p, c.stream);
      t.stop();
      c.T_rhs_ok = true;
      return DCP_OK;
    }
    c.T_rhs.zero(c.stream);
    if (c.dim2) {
      assemble_T_rhs_2d(c);
      t.stop();
      c.T_rhs_ok = true;
      return DCP_OK;
    }
    if (c.feec) {
      // velocity from the Raviart-Thomas field of nse_solution (FEEC.tpp:1000-1062)
      for (int k = 0; k < c.n_colors(); ++k)
        launch_feec_T_rhs(c.fcd(), c.color_begin(k), c.color_size(k), c.old_T.p, c.nse_sol.p, c.ph,
                          c.T_fixed.p, c.T_bc.p, c.T_rhs.p, c.stream);
      t.stop();
      c.T_rhs_ok = true;
      return DCP_OK;
    }
    for (int k = 0; k < c.n_colors(); ++k)
      launch_T_rhs(c.cd(), c.color_begin(k), c.color_size(k), c.old_T.p, c.nse_sol.p, c.ph,
                   c.T_rhs.p, c.stream);
    t.stop();
    c.T_rhs_ok = true;
    return DCP_OK;
  });
}

int dcp_solve_nse_schur(dcp_ctx* ctx, int* schur_iterations, int* a_solves) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(!ctx->feec, DCP_ERR_STATE, "FEEC mesh uploaded: use the dcp_feec_* calls");
    Ctx& c = *ctx;
    require(c.nse_assembled, DCP_ERR_STATE, "assemble_nse_system must run first");
    SectionScope sec(c, "   Solve NSE system");
    PhaseTimer t(c, &c.timings.solve_nse_ms);
    const int rc = solve_nse_schur(c, schur_iterations, a_solves);
    if (c.mf_fused) {
      DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
      check_mf_err(c);
    }
    return rc;
  });
}

int dcp_solve_nse(dcp_ctx* ctx, int* outer, int* inner) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(!ctx->feec, DCP_ERR_STATE, "FEEC mesh uploaded: use the dcp_feec_* calls");
    Ctx& c = *ctx;
    require(c.nse_assembled && c.precond_built, DCP_ERR_STATE,
            "assemble_nse_system and build_nse_preconditioner must run first");
    SectionScope sec(c, "   Solve Stokes system");
    PhaseTimer t(c, &c.timings.solve_nse_ms);
    c.time_schur = true;
    c.schur_ev_used = 0;
    c.schur_calls = 0;
    c.mf_ev_used[0] = c.mf_ev_used[1] = 0;
    c.mf_calls[0] = c.mf_calls[1] = 0;
    const int rc = solve_nse(c, outer, inner);
    c.time_schur = false;
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    check_mf_err(c);
    if (c.comm) c.comm->check();
    double sum = 0;
    int napp = 0;
    for (int k = 0; k < c.schur_ev_used; ++k) {
      float ms = 0;
      DCP_HIP_CHECK(hipEventElapsedTime(&ms, c.schur_ev[k].a, c.schur_ev[k].b));
      sum += ms;
      napp += c.schur_ev[k].count;
    }
    c.timings.schur_apply_ms_avg = napp ? sum / napp : 0.0;
    c.timings.schur_applies = c.schur_calls;
    double mf_ms[2] = {0, 0};
    for (int v = 0; v < 2; ++v) {
      double sm = 0;
      for (int k = 0; k < c.mf_ev_used[v]; ++k) {
        float ms = 0;
        DCP_HIP_CHECK(hipEventElapsedTime(&ms, c.mf_ev[v][k].a, c.mf_ev[v][k].b));
        sm += ms;
      }
      mf_ms[v] = c.mf_ev_used[v] ? sm / c.mf_ev_used[v] : 0.0;
    }
    c.timings.stokes_apply_ms_avg = mf_ms[0];
    c.timings.velocity_apply_ms_avg = mf_ms[1];
    c.timings.stokes_applies = c.mf_calls[0];
    c.timings.velocity_applies = c.mf_calls[1];
    c.timings.a_solve_iterations = c.a_solve_its;
    t.stop();
    return rc;
  });
}

int dcp_solve_temperature(dcp_ctx* ctx, int* iters, double* T_range) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(c.T_rhs_ok, DCP_ERR_STATE, "assemble_temperature_rhs must run first");
    SectionScope sec(c, "   Solve temperature system");
    PhaseTimer t(c, &c.timings.solve_T_ms);
    const int rc = solve_temperature(c, iters, T_range);
    t.stop();
    return rc;
  });
}

int dcp_max_velocity(dcp_ctx* ctx, double* out) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(out != nullptr, DCP_ERR_INVALID, "NULL out");
    Ctx& c = *ctx;
    velocity_stats_global(c);
    *out = c.hpinned[0];
    return DCP_OK;
  });
}

int dcp_cfl_number(dcp_ctx* ctx, double* out) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(out != nullptr, DCP_ERR_INVALID, "NULL out");
    Ctx& c = *ctx;
    velocity_stats_global(c);
    *out = c.hpinned[1];
    return DCP_OK;
  });
}

int dcp_advance_state(dcp_ctx* ctx) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    copy(c.n_u + c.n_p, c.nse_sol.p, c.old_nse.p, c.stream);
    copy(c.n_T, c.T_sol.p, c.old_T.p, c.stream);
    halo_exchange(c, c.halo_nse, c.old_nse.p);
    halo_exchange(c, c.halo_T, c.old_T.p);
    mark_old_ghosted(c, DCP_OLD_NSE_SOLUTION);
    mark_old_ghosted(c, DCP_OLD_T_SOLUTION);
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    return DCP_OK;
  });
}

int dcp_nse_vmult(dcp_ctx* ctx, const double* src, double* dst) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(ctx->nse_assembled, DCP_ERR_STATE, "nse_matrix not assembled");
    nse_vmult(*ctx, src, dst);
    DCP_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    check_mf_err(*ctx);
    return DCP_OK;
  });
}

int dcp_velocity_vmult(dcp_ctx* ctx, const double* src, double* dst) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(ctx->nse_assembled, DCP_ERR_STATE, "nse_matrix not assembled");
    require(!ctx->feec, DCP_ERR_UNSUPPORTED, "classic Q2/Q1 system only");
    velocity_vmult(*ctx, src, dst);
    DCP_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    check_mf_err(*ctx);
    return DCP_OK;
  });
}

int dcp_time_operator(dcp_ctx* ctx, int which, int reps, int nvec, const double* src,
                      double* dst, double* ms_per_apply) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(src && dst && ms_per_apply && reps > 0 && nvec > 0 && which >= 0 && which <= 2,
            DCP_ERR_INVALID, "bad arguments");
    require(c.nse_assembled && !c.feec, DCP_ERR_STATE, "nse_matrix not assembled");
    require(which != 2 || c.precond_built, DCP_ERR_STATE, "build_nse_preconditioner first");
    const size_t len = which == 0 ? size_t(c.n_u) + c.n_p : which == 1 ? size_t(c.n_u) : size_t(c.n_p);
    auto apply = [&](int k) {
      const double* s = src + len * size_t(k % nvec);
      double* d = dst + len * size_t(k % nvec);
      if (which == 0) nse_vmult(c, s, d);
      else if (which == 1) velocity_vmult(c, s, d);
      else schur_vmult(c, s, d);
    };
    apply(0);  // the first apply may build tables (B^T transpose map, S layout)
    hipEvent_t a, b;
    DCP_HIP_CHECK(hipEventCreate(&a));
    DCP_HIP_CHECK(hipEventCreate(&b));
    DCP_HIP_CHECK(hipEventRecord(a, c.stream));
    for (int k = 0; k < reps; ++k) apply(k + 1);
    DCP_HIP_CHECK(hipEventRecord(b, c.stream));
    DCP_HIP_CHECK(hipEventSynchronize(b));
    float ms = 0;
    DCP_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    check_mf_err(c);
    *ms_per_apply = double(ms) / reps;
    return DCP_OK;
  });
}

int dcp_schur_vmult(dcp_ctx* ctx, const double* src, double* dst) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(ctx->nse_assembled && ctx->precond_built, DCP_ERR_STATE, "operator not ready");
    schur_vmult(*ctx, src, dst);
    DCP_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    check_mf_err(*ctx);
    return DCP_OK;
  });
}

int dcp_block_preconditioner_vmult(dcp_ctx* ctx, const double* src, double* dst, int do_solve_A,
                                   int* inner) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(ctx->nse_assembled && ctx->precond_built, DCP_ERR_STATE, "operator not ready");
    const int rc = block_preconditioner_vmult(*ctx, src, dst, do_solve_A != 0, inner);
    DCP_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    check_mf_err(*ctx);
    return rc;
  });
}

int dcp_nse_matrix_export(dcp_ctx* ctx, int64_t* nnz, int32_t* rowptr, int32_t* cols, double* vals) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(nnz != nullptr, DCP_ERR_INVALID, "NULL nnz");
    if (c.dim2) {
      nse_matrix_export_2d(c, nnz, rowptr, cols, vals);
      return DCP_OK;
    }
    auto down_i = [&](const DBuf<int32_t>& b) {
      std::vector<int32_t> h(b.n);
      DCP_HIP_CHECK(hipMemcpy(h.data(), b.p, b.n * sizeof(int32_t), hipMemcpyDeviceToHost));
      return h;
    };
    auto down_d = [&](const DBuf<double>& b) {
      std::vector<double> h(b.n);
      DCP_HIP_CHECK(hipMemcpy(h.data(), b.p, b.n * sizeof(double), hipMemcpyDeviceToHost));
      return h;
    };
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    const auto Ap = down_i(c.A_ptr), Ac = down_i(c.A_col), Btp = down_i(c.Bt_ptr),
               Btc = down_i(c.Bt_col), Bp = down_i(c.B_ptr), Bc = down_i(c.B_col);
    const int64_t total = int64_t(Ap[c.n_vnodes]) * 9 + int64_t(Btp[c.n_vnodes]) * 3 +
                          int64_t(Bp[c.n_p]) * 3 + (c.periodic ? c.n_img_p : 0);
    *nnz = total;
    if (!rowptr) return DCP_OK;
    require(cols && vals, DCP_ERR_INVALID, "NULL cols/vals");
    require(c.nse_assembled, DCP_ERR_STATE, "nse_matrix not assembled");
    materialize_velocity_block(c);
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    const auto Av = down_d(c.A_val), Btv = down_d(c.Bt_val), Bv = down_d(c.B_val);
    const auto cdg = down_d(c.con_diag);
    std::vector<int32_t> pci;
    if (c.periodic) pci = down_i(c.pcidx);
    int64_t k = 0;
    rowptr[0] = 0;
    for (int n = 0; n < c.n_vnodes; ++n)
      for (int r = 0; r < 3; ++r) {
        for (int b = Ap[n]; b < Ap[n + 1]; ++b)
          for (int cc = 0; cc < 3; ++cc) {
            cols[k] = 3 * Ac[b] + cc;
            vals[k++] = Av[9 * size_t(b) + 3 * r + cc];
          }
        for (int b = Btp[n]; b < Btp[n + 1]; ++b) {
          cols[k] = c.n_u + Btc[b];
          vals[k++] = Btv[3 * size_t(b) + r];
        }
        rowptr[3 * n + r + 1] = int32_t(k);
      }
    for (int v = 0; v < c.n_p; ++v) {
      for (int b = Bp[v]; b < Bp[v + 1]; ++b)
        for (int cc = 0; cc < 3; ++cc) {
          cols[k] = 3 * Bc[b] + cc;
          vals[k++] = Bv[3 * size_t(b) + cc];
        }
      if (c.periodic && pci[v] >= 0) {  // a periodic pressure image: its diagonal only
        cols[k] = c.n_u + v;
        vals[k++] = cdg[3 * size_t(c.n_con) + pci[v]];
      }
      rowptr[c.n_u + v + 1] = int32_t(k);
    }
    return DCP_OK;
  });
}

int dcp_T_matrix_export(dcp_ctx* ctx, int64_t* nnz, int32_t* rowptr, int32_t* cols, double* vals) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(nnz != nullptr, DCP_ERR_INVALID, "NULL nnz");
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    std::vector<int32_t> Tp(c.T_ptr.n);
    DCP_HIP_CHECK(hipMemcpy(Tp.data(), c.T_ptr.p, Tp.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
    *nnz = Tp[c.n_T];
    if (!rowptr) return DCP_OK;
    require(cols && vals, DCP_ERR_INVALID, "NULL cols/vals");
    std::copy(Tp.begin(), Tp.begin() + c.n_T + 1, rowptr);
    DCP_HIP_CHECK(hipMemcpy(cols, c.T_col.p, size_t(Tp[c.n_T]) * sizeof(int32_t), hipMemcpyDeviceToHost));
    DCP_HIP_CHECK(hipMemcpy(vals, c.Tmat.p, size_t(Tp[c.n_T]) * sizeof(double), hipMemcpyDeviceToHost));
    return DCP_OK;
  });
}

int dcp_precond_diagonals(dcp_ctx* ctx, double* A_diag, double* Mp_diag) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(ctx->precond_built, DCP_ERR_STATE, "preconditioner not built");
    DCP_HIP_CHECK(hipStreamSynchronize(ctx->stream));
    if (A_diag)
      DCP_HIP_CHECK(hipMemcpy(A_diag, ctx->A_diag.p, ctx->n_u * sizeof(double), hipMemcpyDeviceToHost));
    if (Mp_diag)
      DCP_HIP_CHECK(hipMemcpy(Mp_diag, ctx->Mp_diag.p, ctx->n_p * sizeof(double), hipMemcpyDeviceToHost));
    return DCP_OK;
  });
}

int dcp_cell_nse_system(dcp_ctx* ctx, int first, int n, double* K, double* f) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(K && f && first >= 0 && n > 0 && first + n <= c.n_cells, DCP_ERR_INVALID,
            "bad cell range");
    if (c.dim2) {
      cell_nse_system_2d(c, first, n, K, f);
      return DCP_OK;
    }
    DBuf<double> dK, df;
    dK.alloc(size_t(n) * 89 * 89);
    df.alloc(size_t(n) * 89);
    launch_nse_system_elements(c.cd(), first, n, c.old_nse.p, c.old_T.p, c.ph, dK.p, df.p, c.stream,
                               c.element_mfma);
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    DCP_HIP_CHECK(hipMemcpy(K, dK.p, dK.n * sizeof(double), hipMemcpyDeviceToHost));
    DCP_HIP_CHECK(hipMemcpy(f, df.p, df.n * sizeof(double), hipMemcpyDeviceToHost));
    return DCP_OK;
  });
}

int dcp_pattern_info(dcp_ctx* ctx, int64_t* nA, int64_t* nBt, int64_t* nB, int64_t* nT,
                     int64_t* nS) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    if (nA) *nA = int64_t(ctx->A_col.n);
    if (nBt) *nBt = int64_t(ctx->Bt_col.n);
    if (nB) *nB = int64_t(ctx->B_col.n);
    if (nT) *nT = int64_t(ctx->T_col.n);
    if (nS) *nS = int64_t(ctx->S_col.n);
    return DCP_OK;
  });
}

int dcp_halo_selftest(dcp_ctx* ctx, int n, double* vec, int n_list, const int32_t* send_pos,
                      const int32_t* recv_pos, int n_peers) {
  return guarded(ctx, [&] {
    require(ctx && vec && send_pos && recv_pos, DCP_ERR_INVALID, "NULL argument");
    Ctx& c = *ctx;
    require(c.comm != nullptr, DCP_ERR_STATE, "no communicator (nccl_id or group)");
    require(n > 0 && n_list >= 0 && n_peers >= 1 && n_peers <= n_list + 1, DCP_ERR_INVALID,
            "bad sizes");
    for (int i = 0; i < n_list; ++i)
      require(send_pos[i] >= 0 && send_pos[i] < n && recv_pos[i] >= 0 && recv_pos[i] < n,
              DCP_ERR_INVALID, "position out of range");
    // the forward halo of the solver (gather, grouped send/recv, scatter) with
    // every peer this rank itself: the list split into n_peers chunks
    Ctx::Halo h;
    h.ns = h.nr = n_list;
    for (int k = 0; k < n_peers; ++k) {
      const size_t b = size_t(n_list) * k / n_peers, e = size_t(n_list) * (k + 1) / n_peers;
      h.peers.push_back(c.comm->rank);
      h.soff.push_back(b);
      h.roff.push_back(b);
      h.sn.push_back(e - b);
      h.rn.push_back(e - b);
    }
    h.spos.upload(std::vector<int32_t>(send_pos, send_pos + n_list));
    h.rpos.upload(std::vector<int32_t>(recv_pos, recv_pos + n_list));
    h.sbuf.alloc(std::max(n_list, 1));
    h.rbuf.alloc(std::max(n_list, 1));
    DBuf<double> v;
    v.upload(std::vector<double>(vec, vec + n));
    halo_exchange(c, h, v.p);
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    DCP_HIP_CHECK(hipMemcpy(vec, v.p, size_t(n) * sizeof(double), hipMemcpyDeviceToHost));
    return DCP_OK;
  });
}

int dcp_allreduce_selftest(dcp_ctx* ctx, double* vec, size_t n, int reps, double* ms_per_call) {
  return guarded(ctx, [&] {
    require(ctx && vec && n > 0 && reps >= 1, DCP_ERR_INVALID, "bad arguments");
    Ctx& c = *ctx;
    require(c.comm != nullptr, DCP_ERR_STATE, "no communicator (nccl_id or group)");
    DBuf<double> v;
    v.upload(std::vector<double>(vec, vec + n));
    hipEvent_t a, b;
    DCP_HIP_CHECK(hipEventCreate(&a));
    DCP_HIP_CHECK(hipEventCreate(&b));
    c.comm->allreduce(v.p, n, false, c.stream);  // warm-up: the result is this one's
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    DCP_HIP_CHECK(hipMemcpy(vec, v.p, n * sizeof(double), hipMemcpyDeviceToHost));
    DCP_HIP_CHECK(hipEventRecord(a, c.stream));
    for (int k = 1; k < reps; ++k) c.comm->allreduce(v.p, n, true, c.stream);  // max: stays finite
    DCP_HIP_CHECK(hipEventRecord(b, c.stream));
    DCP_HIP_CHECK(hipEventSynchronize(b));
    float ms = 0.0f;
    DCP_HIP_CHECK(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    c.comm->check();
    if (ms_per_call) *ms_per_call = reps > 1 ? double(ms) / (reps - 1) : 0.0;
    return DCP_OK;
  });
}

int dcp_scatter_info(dcp_ctx* ctx, int64_t* touched, int64_t* nnzb, int* first_touch) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    const Ctx& c = *ctx;
    require(!c.dim2 && !c.feec, DCP_ERR_UNSUPPORTED, "3D classic mesh only");
    const int64_t t[3] = {int64_t(c.touched_A), int64_t(c.touched_Bt), int64_t(c.touched_B)};
    const int64_t n[3] = {int64_t(c.A_col.n), int64_t(c.Bt_col.n), int64_t(c.B_col.n)};
    const int f[3] = {c.first_touch_A, c.first_touch_Bt, c.first_touch_B};
    for (int i = 0; i < 3; ++i) {
      if (touched) touched[i] = t[i];
      if (nnzb) nnzb[i] = n[i];
      if (first_touch) first_touch[i] = f[i];
    }
    return DCP_OK;
  });
}

int dcp_matrix_powers_info(dcp_ctx* ctx, int64_t info[8]) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(info != nullptr, DCP_ERR_INVALID, "NULL info");
    const Ctx& c = *ctx;
    const Ctx::MatPow& m = c.mp;
    const int64_t v[8] = {m.built ? 1 : 0, m.n_ext, m.rows[1], m.rows[2], m.rows[3],
                          m.halo.nr, m.vals.nr, c.halo_p.nr};
    for (int i = 0; i < 8; ++i) info[i] = m.built || i == 7 ? v[i] : 0;
    return DCP_OK;
  });
}

int dcp_comm_info(dcp_ctx* ctx, int32_t info[4]) {
  return guarded(ctx, [&] {
    require(info != nullptr, DCP_ERR_INVALID, "NULL info");
    int v[4] = {0, 1, 0, -1};
    if (ctx->comm) {
      ctx->comm->describe(v);
    } else {
      (void)hipGetDevice(&v[3]);
    }
    for (int i = 0; i < 4; ++i) info[i] = v[i];
    return DCP_OK;
  });
}

int dcp_local_sizes(dcp_ctx* ctx, int64_t out[8]) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(out != nullptr, DCP_ERR_INVALID, "NULL out");
    const Ctx& c = *ctx;
    const bool part = c.comm != nullptr;
    const int64_t v[8] = {c.n_cells, part ? c.n_owned_cells : c.n_cells, c.n_u, c.n_p, c.n_T,
                          part ? int64_t(c.vdim) * c.nvo : c.n_u, part ? c.npo : c.n_p,
                          part ? c.nTo : c.n_T};
    for (int i = 0; i < 8; ++i) out[i] = v[i];
    return DCP_OK;
  });
}

int dcp_device_memory(int64_t* live_bytes, int64_t* peak_bytes) {
  if (live_bytes) *live_bytes = dev_mem().live;
  if (peak_bytes) *peak_bytes = dev_mem().peak;
  return DCP_OK;
}

int dcp_nse_coupling_export(dcp_ctx* ctx, int which, int64_t* nnz, int32_t* rowptr, int32_t* cols,
                            double* vals) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(!c.dim2 && !c.feec, DCP_ERR_UNSUPPORTED, "3D classic mesh only");
    require(nnz != nullptr && (which == 0 || which == 1), DCP_ERR_INVALID, "bad arguments");
    const DBuf<int32_t>& P = which == 0 ? c.Bt_ptr : c.B_ptr;
    const DBuf<int32_t>& C = which == 0 ? c.Bt_col : c.B_col;
    const int rows = int(P.n) - 1;  // local rows (the owned nodes' on several GPUs)
    *nnz = int64_t(C.n) * 3;
    if (!rowptr) return DCP_OK;
    require(cols && vals, DCP_ERR_INVALID, "NULL cols/vals");
    require(c.nse_assembled, DCP_ERR_STATE, "nse_matrix not assembled");
    // the operator form's own blocks: B^T as scattered, B as the solve reads it
    // (materialised from B^T unless scattered); the velocity block untouched
    if (which == 1) materialize_B(c);
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    std::vector<int32_t> p(P.n), cl(C.n);
    std::vector<double> v(C.n * 3);
    DCP_HIP_CHECK(hipMemcpy(p.data(), P.p, P.n * sizeof(int32_t), hipMemcpyDeviceToHost));
    DCP_HIP_CHECK(hipMemcpy(cl.data(), C.p, C.n * sizeof(int32_t), hipMemcpyDeviceToHost));
    DCP_HIP_CHECK(hipMemcpy(v.data(), which == 0 ? c.Bt_val.p : c.B_val.p, v.size() * sizeof(double),
                            hipMemcpyDeviceToHost));
    int64_t k = 0;
    rowptr[0] = 0;
    if (which == 0) {  // scalar rows 3 n + r, columns the pressure dofs
      for (int n = 0; n < rows; ++n)
        for (int r = 0; r < 3; ++r) {
          for (int b = p[n]; b < p[n + 1]; ++b) {
            cols[k] = cl[b];
            vals[k++] = v[3 * size_t(b) + r];
          }
          rowptr[3 * n + r + 1] = int32_t(k);
        }
    } else {  // pressure rows, columns the velocity dofs 3 n + c
      for (int q = 0; q < rows; ++q) {
        for (int b = p[q]; b < p[q + 1]; ++b)
          for (int cc = 0; cc < 3; ++cc) {
            cols[k] = 3 * cl[b] + cc;
            vals[k++] = v[3 * size_t(b) + cc];
          }
        rowptr[q + 1] = int32_t(k);
      }
    }
    return DCP_OK;
  });
}

int dcp_schur_layout(dcp_ctx* ctx, int* col_bytes, int64_t* stored, int* permuted) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    const Ctx& c = *ctx;
    if (col_bytes) *col_bytes = c.S_nbr.p ? 0 : c.S_sell_c16.p ? 2 : 4;
    if (stored) *stored = int64_t(c.S_val.n);
    if (permuted) *permuted = c.S_perm.p != nullptr;
    return DCP_OK;
  });
}

int dcp_assembly_layout(dcp_ctx* ctx, int64_t info[8]) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    require(info != nullptr, DCP_ERR_INVALID, "NULL info");
    const Ctx& c = *ctx;
    const bool on = c.tsep && !c.feec && !c.dim2;
    const bool bk = c.btk && !c.feec && !c.dim2;
    const int64_t v[8] = {on ? 1 : 0, on ? c.ts_n_colids : 0, on ? c.ts_n_layers : 0,
                          on ? c.ts_n_kinds : 0, on ? c.ts_n_latnnz : 0, bk ? 1 : 0,
                          bk ? c.btk_n_pairs : 0, bk ? c.btk_n_conent : 0};
    for (int i = 0; i < 8; ++i) info[i] = v[i];
    return DCP_OK;
  });
}

int dcp_get_timings(dcp_ctx* ctx, dcp_timings* out) {
  if (!ctx || !out) return DCP_ERR_INVALID;
  ctx->timings.handoff_timeouts = ctx->handoff_timeouts;
  *out = ctx->timings;
  return DCP_OK;
}

// ---------------------------------------------------------------------------
}  // extern "C"

// ---------------------------------------------------------------------------
// FEEC variant (ExteriorCalculus::BoussinesqModel<3>, config 4)

namespace {

// rows -> sorted unique columns
void build_csr(const std::vector<std::vector<int32_t>>& rows, std::vector<int32_t>& ptr,
               std::vector<int32_t>& col) {
  ptr.assign(rows.size() + 1, 0);
  for (size_t r = 0; r < rows.size(); ++r) ptr[r + 1] = ptr[r] + int32_t(rows[r].size());
  col.clear();
  col.reserve(size_t(ptr.back()));
  for (const auto& r : rows) col.insert(col.end(), r.begin(), r.end());
}

// make_sparsity_pattern(dof_handler, coupling, sp, constraints, false) for the
// 19-dof FEEC cells: constrained rows/columns keep only the diagonal
// (FEEC.tpp:82-130 system coupling, :146-185 preconditioner coupling).
template <class Couple>
void feec_pattern(int n, int n_cells, const std::vector<int32_t>& dofs,
                  const std::vector<uint8_t>& fixed, Couple couple, std::vector<int32_t>& ptr,
                  std::vector<int32_t>& col) {
  std::vector<std::vector<int32_t>> rows(n);
  for (int c = 0; c < n_cells; ++c) {
    const int32_t* d = &dofs[19 * size_t(c)];
    for (int i = 0; i < 19; ++i) {
      if (fixed[d[i]]) continue;
      for (int j = 0; j < 19; ++j)
        if (!fixed[d[j]] && couple(i, j)) rows[d[i]].push_back(d[j]);
    }
  }
  for (int r = 0; r < n; ++r) {
    if (fixed[r]) rows[r].push_back(r);
    std::sort(rows[r].begin(), rows[r].end());
    rows[r].erase(std::unique(rows[r].begin(), rows[r].end()), rows[r].end());
  }
  build_csr(rows, ptr, col);
}

inline int feec_type(int i) { return i < 12 ? 0 : i < 18 ? 1 : 2; }

}  // namespace

extern "C" {

int dcp_feec_mesh_upload(dcp_ctx* ctx, const dcp_feec_mesh* gm) {
  return guarded(ctx, [&] {
    require(ctx != nullptr && gm != nullptr, DCP_ERR_INVALID, "NULL argument");
    Ctx& c = *ctx;
    require(gm->cell_w && gm->sign_w && gm->cell_u && gm->sign_u && gm->cell_vertices &&
                gm->cell_diameter && gm->cell_T_dofs && gm->w_fixed && gm->u_fixed,
            DCP_ERR_INVALID, "NULL array");
    require(gm->n_cells > 0 && gm->n_p == gm->n_cells, DCP_ERR_INVALID,
            "invalid FEEC sizes (DGQ0: n_p == n_cells)");
    // several GPUs: this rank's cells + two ghost layers (partition.h)
    const bool dist = c.comm != nullptr;
    FeecLocal L;
    dcp_feec_mesh lv{};
    if (dist) {
      try {
        L = localize_feec(*gm, c.cfg.rank, c.cfg.world_size);
      } catch (const std::runtime_error& e) {
        fail(DCP_ERR_INVALID, e.what());
      }
      lv = L.view();
    }
    const dcp_feec_mesh* m = dist ? &lv : gm;
    const int nc = m->n_cells, nw = m->n_w, nu = m->n_u, np = m->n_p, nT = m->n_T;
    require(nc > 0 && nw > 0 && nu > 0 && np == nc && nT > 0, DCP_ERR_INVALID,
            "invalid FEEC sizes");
    const int n = nw + nu + np;
    std::vector<int32_t> dofs(size_t(nc) * 19), td(size_t(nc) * 8);
    std::vector<int8_t> sg(size_t(nc) * 19, 1);
    for (int cell = 0; cell < nc; ++cell) {
      for (int l = 0; l < 12; ++l) {
        const int e = m->cell_w[12 * size_t(cell) + l];
        const int s = m->sign_w[12 * size_t(cell) + l];
        require(e >= 0 && e < nw && (s == 1 || s == -1), DCP_ERR_INVALID, "bad edge dof / sign");
        dofs[19 * size_t(cell) + l] = e;
        sg[19 * size_t(cell) + l] = int8_t(s);
      }
      for (int f = 0; f < 6; ++f) {
        const int u = m->cell_u[6 * size_t(cell) + f];
        const int s = m->sign_u[6 * size_t(cell) + f];
        require(u >= 0 && u < nu && (s == 1 || s == -1), DCP_ERR_INVALID, "bad face dof / sign");
        dofs[19 * size_t(cell) + 12 + f] = nw + u;
        sg[19 * size_t(cell) + 12 + f] = int8_t(s);
      }
      dofs[19 * size_t(cell) + 18] = nw + nu + cell;
      for (int v = 0; v < 8; ++v) {
        const int t = m->cell_T_dofs[8 * size_t(cell) + v];
        require(t >= 0 && t < nT, DCP_ERR_INVALID, "temperature dof out of range");
        td[8 * size_t(cell) + v] = t;
      }
    }
    std::vector<uint8_t> fixed(n, 0);
    for (int e = 0; e < nw; ++e) fixed[e] = m->w_fixed[e] != 0;
    for (int u = 0; u < nu; ++u) fixed[nw + u] = m->u_fixed[u] != 0;
    // temperature constraints: Dirichlet lines and, on the cuboid, the
    // periodic identities of make_periodicity_constraints (FEEC.tpp:435-455).
    // An image is folded into its partner in the cell maps (the partner's row
    // receives the image's cell contributions, as distribute_local_to_global
    // does) and keeps a diagonal-only row, copied from the partner after the
    // solve; the same treatment as the classic upload (prepare_host above).
    std::vector<uint8_t> Tfix(nT, 0);
    std::vector<double> Tbc(nT, 0.0);
    std::vector<int32_t> tmaster(nT, -1);
    int n_timg = 0;
    for (int l = 0; l < m->T.n_lines; ++l) {
      const int d = m->T.line_dof[l];
      require(d >= 0 && d < nT, DCP_ERR_INVALID, "temperature constraint out of range");
      const int b = m->T.entry_ptr[l];
      if (m->T.entry_ptr[l + 1] - b == 1 && m->T.entry_w[b] == 1.0 && m->T.inhomogeneity[l] == 0.0 &&
          m->T.entry_dof[b] != d) {
        require(m->T.entry_dof[b] >= 0 && m->T.entry_dof[b] < nT, DCP_ERR_INVALID,
                "temperature constraint out of range");
        tmaster[d] = m->T.entry_dof[b];
        ++n_timg;
        continue;
      }
      require(m->T.entry_ptr[l] == m->T.entry_ptr[l + 1], DCP_ERR_UNSUPPORTED,
              "temperature constraints must be Dirichlet lines or periodic identities");
      Tfix[d] = 1;
      Tbc[d] = m->T.inhomogeneity[l];
    }
    for (int t = 0; t < nT; ++t)
      require(tmaster[t] < 0 || (tmaster[tmaster[t]] < 0 && !Tfix[tmaster[t]]), DCP_ERR_UNSUPPORTED,
              "periodic temperature chain not closed");
    const std::vector<int32_t> tdo = td;
    if (n_timg)
      for (auto& t : td)
        if (tmaster[t] >= 0) t = tmaster[t];
    // one global dof per local dof of a cell: the scatter kernels add a
    // cell's entries concurrently
    for (int cell = 0; cell < nc; ++cell) {
      const int32_t* d = &dofs[19 * size_t(cell)];
      const int32_t* t = &td[8 * size_t(cell)];
      for (int i = 0; i < 19; ++i)
        for (int j = 0; j < i; ++j)
          require(d[i] != d[j] && (i >= 8 || t[i] != t[j]), DCP_ERR_UNSUPPORTED,
                  "a cell holds a global dof twice (periodic box with one cell across?)");
    }
    // patterns: system (w:{w,u}, u:{w,u,p}, p:{u}), preconditioner (w:{w,u}, u:{w,u}, p:{w,p})
    std::vector<int32_t> Sp, Sc, Pp, Pc;
    feec_pattern(n, nc, dofs, fixed,
                 [](int i, int j) {
                   const int a = feec_type(i), b = feec_type(j);
                   return a == 0 ? b < 2 : a == 1 ? true : b == 1;
                 },
                 Sp, Sc);
    feec_pattern(n, nc, dofs, fixed,
                 [](int i, int j) {
                   const int a = feec_type(i), b = feec_type(j);
                   return a < 2 ? b < 2 : b != 1;
                 },
                 Pp, Pc);
    // temperature pattern
    std::vector<std::vector<int32_t>> trows(nT);
    for (int cell = 0; cell < nc; ++cell)
      for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) trows[td[8 * size_t(cell) + i]].push_back(td[8 * size_t(cell) + j]);
    for (int t = 0; t < nT; ++t)
      if (tmaster[t] >= 0) trows[t].push_back(t);  // an image: its diagonal only
    for (auto& r : trows) {
      std::sort(r.begin(), r.end());
      r.erase(std::unique(r.begin(), r.end()), r.end());
    }
    std::vector<int32_t> Tp, Tc;
    build_csr(trows, Tp, Tc);
    // position of an image's diagonal per (cell, vertex), -1 if not an image
    std::vector<int32_t> posTs(n_timg ? size_t(nc) * 8 : 0, -1);
    std::vector<int32_t> iT, mT;
    if (n_timg) {
      for (size_t k = 0; k < posTs.size(); ++k)
        if (tdo[k] != td[k]) {
          const int o = tdo[k];
          posTs[k] = int32_t(std::lower_bound(Tc.begin() + Tp[o], Tc.begin() + Tp[o + 1], o) - Tc.begin());
        }
      for (int t = 0; t < nT; ++t)
        if (tmaster[t] >= 0) {
          iT.push_back(t);
          mT.push_back(tmaster[t]);
        }
    }
    std::vector<int32_t> posT(size_t(nc) * 64);
    for (int cell = 0; cell < nc; ++cell)
      for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) {
          const int r = td[8 * size_t(cell) + i], col = td[8 * size_t(cell) + j];
          const auto b = Tc.begin() + Tp[r], e = Tc.begin() + Tp[r + 1];
          posT[64 * size_t(cell) + 8 * i + j] = int32_t(std::lower_bound(b, e, col) - Tc.begin());
        }
    // colouring over vertex-sharing cells (Q1 temperature dofs are the vertices)
    std::vector<std::vector<int32_t>> vcells(nT);
    for (int cell = 0; cell < nc; ++cell)
      for (int v = 0; v < 8; ++v) vcells[td[8 * size_t(cell) + v]].push_back(cell);
    std::vector<int> color(nc, -1);
    int n_colors = 0;
    for (int cell = 0; cell < nc; ++cell) {
      uint64_t used = 0;
      for (int v = 0; v < 8; ++v)
        for (int o : vcells[td[8 * size_t(cell) + v]])
          if (color[o] >= 0) used |= uint64_t(1) << color[o];
      int col = 0;
      while (col < 64 && ((used >> col) & 1)) ++col;
      require(col < 64, DCP_ERR_UNSUPPORTED, "cell colouring needs more than 64 colours");
      color[cell] = col;
      n_colors = std::max(n_colors, col + 1);
    }
    c.color_ptr.assign(n_colors + 1, 0);
    for (int cell = 0; cell < nc; ++cell) c.color_ptr[color[cell] + 1]++;
    for (int k = 0; k < n_colors; ++k) c.color_ptr[k + 1] += c.color_ptr[k];
    std::vector<int32_t> ccells(nc);
    {
      std::vector<int> f(c.color_ptr.begin(), c.color_ptr.end() - 1);
      for (int cell = 0; cell < nc; ++cell) ccells[f[color[cell]]++] = cell;
    }
    // cell geometry = the trilinear map of the vertices at the 64 support
    // points: the classic temperature kernels then integrate on MappingQ1
    // (temperature_mapping(1), FEEC.tpp:20) exactly
    std::vector<int32_t> q2(size_t(nc) * 27);
    std::vector<double> geo(size_t(nc) * 3 * kMapPts);
    for (int cell = 0; cell < nc; ++cell) {
      for (int k = 0; k < 27; ++k) q2[27 * size_t(cell) + k] = 27 * cell + k;
      for (int k = 0; k < kMapPts; ++k) {
        const double t[3] = {kGL3[k % 4], kGL3[(k / 4) % 4], kGL3[k / 16]};
        for (int d = 0; d < 3; ++d) {
          double x = 0;
          for (int v = 0; v < 8; ++v) {
            const double w = ((v & 1) ? t[0] : 1 - t[0]) * (((v >> 1) & 1) ? t[1] : 1 - t[1]) *
                             ((v >> 2) ? t[2] : 1 - t[2]);
            x += w * m->cell_vertices[24 * size_t(cell) + 3 * v + d];
          }
          geo[3 * kMapPts * size_t(cell) + 3 * k + d] = x;
        }
      }
    }
    DCP_HIP_CHECK(hipSetDevice(c.cfg.device));
    c.feec = true;
    c.dim2 = false;
    c.vdim = 3;
    c.tdpc3 = 8;
    c.have_mesh = false;
    c.n_cells = nc;
    c.n_owned_cells = dist ? L.n_owned_cells : nc;
    c.fe_nw = nw;
    c.fe_nu = nu;
    c.fe_np = np;
    c.fe_nwo = dist ? L.nwo : nw;
    c.fe_nuo = dist ? L.nuo : nu;
    c.fe_npo = c.n_owned_cells;
    c.fe_nw_g = gm->n_w;
    c.fe_nu_g = gm->n_u;
    c.n_u = nw + nu;  // state API: NSE vector = [w u | p]
    c.n_p = np;
    c.n_T = nT;
    c.n_u_g = gm->n_w + gm->n_u;
    c.n_p_g = gm->n_p;
    c.n_T_g = gm->n_T;
    c.nTo = dist ? L.nTo : nT;
    c.n_vnodes = 0;
    c.fe_w_g = L.w_g;
    c.fe_u_g = L.u_g;
    c.p_g = L.cells_g;
    c.T_g = L.T_g;
    c.max_owned[3] = c.nTo;
    c.max_owned[4] = c.fe_nwo + c.fe_nuo + c.fe_npo;
    c.max_owned[5] = c.fe_nwo;
    c.max_owned[6] = c.fe_nuo;
    c.max_owned[7] = c.fe_npo;
    c.fe_dofs.upload(dofs);
    c.fe_sign.upload(sg);
    c.fe_X.upload(std::vector<double>(m->cell_vertices, m->cell_vertices + 24 * size_t(nc)));
    c.diameter.upload(std::vector<double>(m->cell_diameter, m->cell_diameter + nc));
    c.fe_fixed.upload(fixed);
    c.cell_T.upload(td);
    c.cell_q2.upload(q2);
    c.cell_geo.upload(geo);
    c.T_fixed.upload(Tfix);
    c.T_bc.upload(Tbc);
    c.color_cells.upload(ccells);
    c.fe_ptr.upload(Sp);
    c.fe_col.upload(Sc);
    c.fe_val.alloc(Sc.size());
    c.fp_ptr.upload(Pp);
    c.fp_col.upload(Pc);
    c.fp_val.alloc(Pc.size());
    c.fe_pos.alloc(size_t(nc) * 361);
    c.fp_pos.alloc(size_t(nc) * 361);
    feec_positions(c.fcd(), nc, c.fe_ptr.p, c.fe_col.p, c.fe_pos.p, c.stream);
    feec_positions(c.fcd(), nc, c.fp_ptr.p, c.fp_col.p, c.fp_pos.p, c.stream);
    c.T_ptr.upload(Tp);
    c.T_col.upload(Tc);
    c.Tmass.alloc(Tc.size());
    c.Tstiff.alloc(Tc.size());
    c.Tmat.alloc(Tc.size());
    c.posT.upload(posT);
    c.periodic = n_timg > 0;
    c.n_img_u = c.n_img_p = c.n_img_node = 0;
    c.n_img_T = n_timg;
    if (c.periodic) {
      c.posTs.upload(posTs);
      c.img_T.upload(iT);
      c.mst_T.upload(mT);
    }
    c.T_inv.alloc(nT);
    c.fe_cellw.alloc(nc);
    feec_cell_weights(c.fcd(), nc, c.fe_cellw.p, c.stream, 1);
    c.fe_cellw2.alloc(nc);
    feec_cell_weights(c.fcd(), nc, c.fe_cellw2.p, c.stream, 2);
    c.fe_dinv.alloc(nw + nu);
    for (auto* b : {&c.fe_t1, &c.fe_t2, &c.fe_t3, &c.fe_t4}) b->alloc(n);
    c.nse_sol.alloc(n);
    c.old_nse.alloc(n);
    c.nse_rhs.alloc(n);
    c.T_sol.alloc(nT);
    c.old_T.alloc(nT);
    c.T_rhs.alloc(nT);
    for (auto* b : {&c.nse_sol, &c.old_nse, &c.nse_rhs, &c.T_sol, &c.old_T, &c.T_rhs}) b->zero(c.stream);
    free_workspaces(c);
    {
      // sum of the mean-value weights over the owned cells (all ranks)
      std::vector<double> w(nc), w2(nc);
      DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
      DCP_HIP_CHECK(hipMemcpy(w.data(), c.fe_cellw.p, nc * sizeof(double), hipMemcpyDeviceToHost));
      DCP_HIP_CHECK(hipMemcpy(w2.data(), c.fe_cellw2.p, nc * sizeof(double), hipMemcpyDeviceToHost));
      double ws = 0, ws2 = 0;
      for (int k = 0; k < c.fe_npo; ++k) ws += w[k];
      for (int k = 0; k < c.fe_npo; ++k) ws2 += w2[k];
      c.fe_wsum = ws;
      c.fe_wsum2 = ws2;
    }
    if (dist) {
      auto one = [&](Ctx::Halo& h, std::initializer_list<std::pair<const HaloPlan*, int>> parts) {
        std::vector<int> peers;
        std::vector<std::vector<int32_t>> sp, rp;
        for (auto& pr : parts) plan_positions(*pr.first, pr.second, peers, sp, rp);
        make_halo(h, peers, sp, rp);
      };
      one(c.halo_fw, {{&L.hw, 0}});
      one(c.halo_fu, {{&L.hu, 0}});
      one(c.halo_fp, {{&L.hp, 0}});
      one(c.halo_nse, {{&L.hw, 0}, {&L.hu, nw}, {&L.hp, nw + nu}});
      one(c.halo_T, {{&L.hT, 0}});
      double mx[5] = {double(c.max_owned[3]), double(c.max_owned[4]), double(c.max_owned[5]),
                      double(c.max_owned[6]), double(c.max_owned[7])};
      double* d = c.dscal.p + 3500;
      DCP_HIP_CHECK(hipMemcpyAsync(d, mx, sizeof(mx), hipMemcpyHostToDevice, c.stream));
      c.comm->allreduce(d, 5, true, c.stream);
      DCP_HIP_CHECK(hipMemcpyAsync(mx, d, sizeof(mx), hipMemcpyDeviceToHost, c.stream));
      const double wsums[2] = {c.fe_wsum, c.fe_wsum2};
      DCP_HIP_CHECK(hipMemcpyAsync(d, wsums, sizeof(wsums), hipMemcpyHostToDevice, c.stream));
      c.comm->allreduce(d, 2, false, c.stream);
      double wsum_all[2];
      DCP_HIP_CHECK(hipMemcpyAsync(wsum_all, d, sizeof(wsum_all), hipMemcpyDeviceToHost, c.stream));
      DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
      for (int k = 0; k < 5; ++k) c.max_owned[3 + k] = int(mx[k]);
      c.fe_wsum = wsum_all[0];
      c.fe_wsum2 = wsum_all[1];
    }
    c.have_mesh = true;
    c.fe_assembled = c.fe_precond = c.T_matrix_ok = c.T_rhs_ok = false;
    return DCP_OK;
  });
}

int dcp_feec_assemble_nse_system(dcp_ctx* ctx) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(c.feec, DCP_ERR_STATE, "no FEEC mesh uploaded");
    SectionScope sec(c, "   Assemble NSE system");  // FEEC.tpp:831
    PhaseTimer t(c, &c.timings.assemble_nse_ms);
    halo_exchange(c, c.halo_nse, c.old_nse.p);
    halo_exchange(c, c.halo_T, c.old_T.p);
    c.fe_val.zero(c.stream);
    c.nse_rhs.zero(c.stream);
    for (int k = 0; k < c.n_colors(); ++k)
      launch_feec_system(c.fcd(), c.color_begin(k), c.color_size(k), c.fe_pos.p, c.old_nse.p,
                         c.old_T.p, c.ph, c.fe_val.p, c.nse_rhs.p, c.stream);
    t.stop();
    c.fe_assembled = true;
    return DCP_OK;
  });
}

int dcp_feec_build_nse_preconditioner(dcp_ctx* ctx) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(c.feec, DCP_ERR_STATE, "no FEEC mesh uploaded");
    SectionScope sec(c, "   Build NSE FEEC preconditioner");  // FEEC.tpp:630
    PhaseTimer t(c, &c.timings.build_precond_ms);
    {
      SectionScope sub(c, "   Assembly NSE preconditioner");  // FEEC.tpp:592
      c.fp_val.zero(c.stream);
      for (int k = 0; k < c.n_colors(); ++k)
        launch_feec_precond(c.fcd(), c.color_begin(k), c.color_size(k), c.fp_pos.p, c.ph,
                            c.fp_val.p, c.stream);
    }
    t.stop();
    c.fe_precond = true;
    return DCP_OK;
  });
}

int dcp_feec_solve_nse(dcp_ctx* ctx, int* iterations) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(c.feec && c.fe_assembled, DCP_ERR_STATE, "assemble the FEEC system first");
    SectionScope sec(c, "   Solve NSE system");  // FEEC.tpp:1277
    PhaseTimer t(c, &c.timings.solve_nse_ms);
    const int rc = feec_solve_nse(c, iterations);
    t.stop();
    return rc;
  });
}

int dcp_feec_cell_system(dcp_ctx* ctx, int first, int n, double* K, double* f) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(c.feec, DCP_ERR_STATE, "no FEEC mesh uploaded");
    require(K && f && first >= 0 && n > 0 && first + n <= c.n_cells, DCP_ERR_INVALID,
            "bad cell range");
    DBuf<double> dK, df;
    dK.alloc(size_t(n) * 361);
    df.alloc(size_t(n) * 19);
    launch_feec_elements(c.fcd(), first, n, c.old_nse.p, c.old_T.p, c.ph, dK.p, df.p, c.stream);
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    DCP_HIP_CHECK(hipMemcpy(K, dK.p, dK.n * sizeof(double), hipMemcpyDeviceToHost));
    DCP_HIP_CHECK(hipMemcpy(f, df.p, df.n * sizeof(double), hipMemcpyDeviceToHost));
    return DCP_OK;
  });
}

int dcp_feec_matrix_export(dcp_ctx* ctx, int which, int64_t* nnz, int32_t* rowptr, int32_t* cols,
                           double* vals) {
  return guarded(ctx, [&] {
    need_ready(*ctx);
    Ctx& c = *ctx;
    require(c.feec && nnz, DCP_ERR_INVALID, "no FEEC mesh / NULL nnz");
    const DBuf<int32_t>& P = which == 0 ? c.fe_ptr : c.fp_ptr;
    const DBuf<int32_t>& C = which == 0 ? c.fe_col : c.fp_col;
    const DBuf<double>& V = which == 0 ? c.fe_val : c.fp_val;
    *nnz = int64_t(C.n);
    if (!rowptr) return DCP_OK;
    require(cols && vals, DCP_ERR_INVALID, "NULL cols/vals");
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    DCP_HIP_CHECK(hipMemcpy(rowptr, P.p, P.n * sizeof(int32_t), hipMemcpyDeviceToHost));
    DCP_HIP_CHECK(hipMemcpy(cols, C.p, C.n * sizeof(int32_t), hipMemcpyDeviceToHost));
    DCP_HIP_CHECK(hipMemcpy(vals, V.p, V.n * sizeof(double), hipMemcpyDeviceToHost));
    return DCP_OK;
  });
}

}  // extern "C"

extern "C" {

// ---------------------------------------------------------------------------
// Host setup helpers

struct dcp_host_mesh {
  Mesh mesh;
  Constraints nse, T;
  TemperatureDofs tdofs;
  std::vector<int32_t> cell_nse;
  std::vector<double> nse_xyz;     // support point of each velocity node once renumbered
  bool renumbered = false;         // the NSE dofs no longer follow the mesh's node ids
  std::unique_ptr<FeecDofs> feec;  // built on first request
  // the 2D shell (dcp_host_mesh2d_create); the members above stay empty
  struct Two {
    Mesh2D mesh;
    int tdeg = 2, n_T = 0;
    Constraints nse, T;
    std::vector<int32_t> cell_nse, cell_T;
    std::vector<double> node_xy;   // support point of each velocity node (current numbering)
  };
  std::unique_ptr<Two> two;
};

dcp_host_mesh* dcp_host_mesh_create(int cuboid, int refine, double R0, double R1, double length,
                                    int temperature_degree, int normal_mode,
                                    int mapping_q_on_all_cells) {
  try {
    auto h = std::make_unique<dcp_host_mesh>();
    h->mesh = cuboid ? build_cube(refine, length)
                     : build_shell(refine, R0 / length, R1 / length, mapping_q_on_all_cells != 0);
    h->nse = nse_constraints(h->mesh, normal_mode == 1   ? NormalMode::Radial
                                      : normal_mode == 2 ? NormalMode::Consistent
                                                         : NormalMode::Mapping);
    h->T = temperature_constraints(h->mesh, temperature_degree);
    h->tdofs = temperature_dofs(h->mesh, temperature_degree);
    h->cell_nse = nse_cell_dofs_dealii(h->mesh);
    return h.release();
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return nullptr;
  }
}

void dcp_host_mesh_destroy(dcp_host_mesh* m) { delete m; }

int dcp_host_mesh_renumber_cuthill_mckee(dcp_host_mesh* h) {
  if (!h) return DCP_ERR_INVALID;
  if (h->two) {
    try {
      dcp_host_mesh::Two& t = *h->two;
      const std::vector<int32_t> map = cuthill_mckee_map_2d(t.mesh, t.cell_nse);
      for (int32_t& d : t.cell_nse) d = map[d];
      t.nse = renumber_constraints(t.nse, map);
      std::vector<double> xy(t.node_xy.size());
      for (int n = 0; n < t.mesh.n_vnodes; ++n)
        for (int k = 0; k < 2; ++k) xy[2 * size_t(map[2 * n] / 2) + k] = t.node_xy[2 * size_t(n) + k];
      t.node_xy.swap(xy);
      return DCP_OK;
    } catch (const std::exception& e) {
      g_last_error = e.what();
      return DCP_ERR_INVALID;
    }
  }
  try {
    const Mesh& m = h->mesh;
    const std::vector<int32_t> nw = cuthill_mckee_nodes(m.n_cells, h->cell_nse.data(), m.n_vnodes);
    const std::vector<int32_t> map =
        nse_dof_map(m.n_cells, h->cell_nse.data(), m.n_vnodes, m.n_p(), nw);
    for (int32_t& d : h->cell_nse) d = map[d];
    h->nse = renumber_constraints(h->nse, map);
    const std::vector<double>& src = h->nse_xyz.empty() ? m.xyz : h->nse_xyz;
    std::vector<double> xyz(src.size());
    for (int n = 0; n < m.n_vnodes; ++n)
      for (int k = 0; k < 3; ++k) xyz[3 * size_t(nw[n]) + k] = src[3 * size_t(n) + k];
    h->nse_xyz.swap(xyz);
    h->renumbered = true;
    return DCP_OK;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return DCP_ERR_INVALID;
  }
}

int dcp_host_mesh_renumber_dealii(dcp_host_mesh* h, int32_t* cell_order) {
  if (!h) return DCP_ERR_INVALID;
  try {
    if (h->two)
      throw std::invalid_argument("the 2D shell is already in deal.II's order (hyper_shell<2>)");
    if (h->renumbered) throw std::invalid_argument("renumber to deal.II's order before Cuthill-McKee");
    if (h->feec) throw std::invalid_argument("renumber before requesting the FEEC topology");
    const Mesh& m = h->mesh;
    std::vector<int32_t> cells;
    const std::vector<int32_t> nw = dealii_shell_node_order(m, cell_order ? &cells : nullptr);
    const std::vector<int32_t> map = nse_dof_map(m.n_cells, h->cell_nse.data(), m.n_vnodes, m.n_p(), nw);
    for (int32_t& d : h->cell_nse) d = map[d];
    h->nse = renumber_constraints(h->nse, map);
    std::vector<double> xyz(m.xyz.size());
    for (int n = 0; n < m.n_vnodes; ++n)
      for (int k = 0; k < 3; ++k) xyz[3 * size_t(nw[n]) + k] = m.xyz[3 * size_t(n) + k];
    h->nse_xyz.swap(xyz);
    // temperature: distribute_dofs of FE_Q(1|2) alone, the same first-encounter
    // order over the same cells, i.e. the order of the support points' new numbers
    TemperatureDofs& td = h->tdofs;
    std::vector<int32_t> byn(size_t(td.n_dofs));
    for (int d = 0; d < td.n_dofs; ++d) byn[d] = d;
    std::sort(byn.begin(), byn.end(),
              [&](int32_t a, int32_t b) { return nw[td.dof_vnode[a]] < nw[td.dof_vnode[b]]; });
    std::vector<int32_t> tmap(size_t(td.n_dofs)), vn(size_t(td.n_dofs));
    for (int r = 0; r < td.n_dofs; ++r) {
      tmap[byn[r]] = r;
      vn[r] = td.dof_vnode[byn[r]];
    }
    for (int32_t& d : td.cell_dofs) d = tmap[d];
    td.dof_vnode.swap(vn);
    h->T = renumber_constraints(h->T, tmap);
    if (cell_order) std::copy(cells.begin(), cells.end(), cell_order);
    return DCP_OK;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return DCP_ERR_INVALID;
  }
}

static dcp_constraints view_of(const Constraints& c) {
  dcp_constraints v;
  v.n_lines = c.n_lines();
  v.line_dof = c.line_dof.data();
  v.entry_ptr = c.entry_ptr.data();
  v.entry_dof = c.entry_dof.data();
  v.entry_w = c.entry_w.data();
  v.inhomogeneity = c.inhomogeneity.data();
  return v;
}

int dcp_host_mesh_view_get(const dcp_host_mesh* h, dcp_host_mesh_view* out) {
  if (!h || !out) return DCP_ERR_INVALID;
  if (h->two) {
    g_last_error = "a 2D host mesh: use dcp_host_mesh2d_view_get";
    return DCP_ERR_INVALID;
  }
  const Mesh& m = h->mesh;
  out->n_cells = m.n_cells;
  out->n_u = m.n_u();
  out->n_p = m.n_p();
  out->n_T = h->tdofs.n_dofs;
  out->n_vnodes = m.n_vnodes;
  out->cell_nse_dofs = h->cell_nse.data();
  out->cell_T_dofs = h->tdofs.cell_dofs.data();
  out->cell_geometry = m.cell_map.data();
  out->cell_diameter = m.cell_diameter.data();
  out->node_xyz = h->nse_xyz.empty() ? m.xyz.data() : h->nse_xyz.data();
  out->nse = view_of(h->nse);
  out->T = view_of(h->T);
  return DCP_OK;
}

int dcp_host_feec_view_get(dcp_host_mesh* h, dcp_feec_mesh* out) {
  if (!h || !out) return DCP_ERR_INVALID;
  // the cuboid's x/y periodicity is in the topology (feec_mesh.cpp) and in
  // the temperature constraints' identity lines (folded at upload)
  if (h->mesh.cuboid && h->mesh.N < 2) {
    // one cell across: a cell would hold the same edge / face dof twice
    g_last_error = "FEEC on the periodic cuboid needs refinement >= 1 (two cells per direction)";
    return DCP_ERR_UNSUPPORTED;
  }
  try {
    if (!h->feec) h->feec = std::make_unique<FeecDofs>(feec_dofs(h->mesh));
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return DCP_ERR_INVALID;
  }
  const FeecDofs& f = *h->feec;
  out->n_cells = h->mesh.n_cells;
  out->n_w = f.n_w;
  out->n_u = f.n_u;
  out->n_p = f.n_p;
  out->n_T = h->tdofs.n_dofs;
  out->cell_w = f.cell_w.data();
  out->sign_w = f.sign_w.data();
  out->cell_u = f.cell_u.data();
  out->sign_u = f.sign_u.data();
  out->cell_vertices = f.cell_vertices.data();
  out->cell_diameter = h->mesh.cell_diameter.data();
  out->cell_T_dofs = h->tdofs.cell_dofs.data();
  out->w_fixed = f.w_boundary.data();
  out->u_fixed = f.u_boundary.data();
  out->T = view_of(h->T);
  return DCP_OK;
}

int dcp_host_mesh_initial_temperature(const dcp_host_mesh* h, double* T) {
  if (!h || !T) return DCP_ERR_INVALID;
  if (h->two) {
    // TemperatureInitialValues<2> at the MappingQ1 support points
    const Mesh2D& m = h->two->mesh;
    for (int d = 0; d < h->two->n_T; ++d) {
      const int n = h->two->tdeg == 2 ? d : m.vertex_vnode[d];
      T[d] = temperature_initial_2d(&m.xy_q1[2 * size_t(n)], m.R0, m.R1);
    }
    return DCP_OK;
  }
  for (int d = 0; d < h->tdofs.n_dofs; ++d)
    T[d] = temperature_initial(h->mesh, &h->mesh.xyz[3 * size_t(h->tdofs.dof_vnode[d])]);
  return DCP_OK;
}

dcp_host_mesh* dcp_host_mesh2d_create(int refine, double R0, double R1, double length,
                                      int temperature_degree, int mapping_q_on_all_cells) {
  try {
    if (temperature_degree != 1 && temperature_degree != 2)
      throw std::invalid_argument("2D temperature degree must be 1 or 2");
    if (!(length > 0)) throw std::invalid_argument("reference length must be positive");
    auto h = std::make_unique<dcp_host_mesh>();
    h->two = std::make_unique<dcp_host_mesh::Two>();
    dcp_host_mesh::Two& t = *h->two;
    t.mesh = build_shell_2d(refine, R0 / length, R1 / length, mapping_q_on_all_cells != 0);
    const Mesh2D& m = t.mesh;
    t.tdeg = temperature_degree;
    t.cell_nse = nse_cell_dofs_2d(m);
    t.nse = nse_constraints_2d(m);
    t.node_xy = m.xy;
    if (temperature_degree == 2) {
      t.cell_T = temperature_cell_dofs_2d(m);
      t.T = temperature_constraints_2d(m);
      t.n_T = m.n_vnodes;
    } else {
      // FE_Q(1): the vertices in first-encounter order, Dirichlet on the inner circle
      t.cell_T = m.cell_q1;
      t.n_T = m.n_vertices;
      Constraints c;
      c.n_dofs = t.n_T;
      c.line_of.assign(t.n_T, -1);
      c.entry_ptr.push_back(0);
      for (int v = 0; v < t.n_T; ++v) {
        const int n = m.vertex_vnode[v];
        if (!(m.vnode_bnd[n] & kBndInner)) continue;
        c.line_of[v] = c.n_lines();
        c.line_dof.push_back(v);
        c.inhomogeneity.push_back(temperature_initial_2d(&m.xy_q1[2 * size_t(n)], m.R0, m.R1));
        c.entry_ptr.push_back(0);
      }
      t.T = std::move(c);
    }
    return h.release();
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return nullptr;
  }
}

int dcp_host_mesh2d_view_get(const dcp_host_mesh* h, dcp_mesh2d* out, const double** node_xy,
                             int* n_vnodes) {
  if (!h || !out || !h->two) return DCP_ERR_INVALID;
  const dcp_host_mesh::Two& t = *h->two;
  out->n_cells = t.mesh.n_cells;
  out->n_u = t.mesh.n_u();
  out->n_p = t.mesh.n_p();
  out->n_T = t.n_T;
  out->temperature_degree = t.tdeg;
  out->cell_nse_dofs = t.cell_nse.data();
  out->cell_T_dofs = t.cell_T.data();
  out->cell_geometry = t.mesh.cell_map.data();
  out->cell_diameter = t.mesh.cell_diameter.data();
  out->nse = view_of(t.nse);
  out->T = view_of(t.T);
  if (node_xy) *node_xy = t.node_xy.data();
  if (n_vnodes) *n_vnodes = t.mesh.n_vnodes;
  return DCP_OK;
}

int dcp_mesh2d_upload(dcp_ctx* ctx, const dcp_mesh2d* m) {
  return guarded(ctx, [&] {
    require(ctx != nullptr && m != nullptr, DCP_ERR_INVALID, "NULL argument");
    Ctx& c = *ctx;
    if (!c.comm) {
      mesh2d_upload(c, m);
      return DCP_OK;
    }
    // several GPUs: this rank's cells + two ghost layers (partition.h), the
    // velocity as scalar dofs (vdim 1: the support points' two components
    // are two owned-or-ghost entries of their own)
    Local2D L;
    try {
      L = localize_2d(*m, c.cfg.rank, c.cfg.world_size);
    } catch (const std::runtime_error& e) {
      fail(DCP_ERR_INVALID, e.what());
    }
    const dcp_mesh2d lv = L.view();
    mesh2d_upload(c, &lv);
    c.have_mesh = false;
    c.vdim = 1;
    c.n_owned_cells = L.n_owned_cells;
    c.n_vnodes = L.n_u();
    c.nvo = L.nuo;
    c.npo = L.npo;
    c.nTo = L.nTo;
    c.n_u_g = m->n_u;
    c.n_p_g = m->n_p;
    c.n_T_g = m->n_T;
    c.vnode_g = L.u_g;
    c.p_g = L.p_g;
    c.T_g = L.T_g;
    auto one = [&](Ctx::Halo& h, std::initializer_list<std::pair<const HaloPlan*, int>> parts) {
      std::vector<int> peers;
      std::vector<std::vector<int32_t>> sp, rp;
      for (auto& pr : parts) plan_positions(*pr.first, pr.second, peers, sp, rp);
      make_halo(h, peers, sp, rp);
    };
    one(c.halo_v, {{&L.hu, 0}});
    one(c.halo_p, {{&L.hp, 0}});
    one(c.halo_nse, {{&L.hu, 0}, {&L.hp, c.n_u}});
    one(c.halo_T, {{&L.hT, 0}});
    double mx[4] = {double(c.nvo + c.npo), double(c.npo), double(c.nvo), double(c.nTo)};
    double* d = c.dscal.p + 3500;
    DCP_HIP_CHECK(hipMemcpyAsync(d, mx, sizeof(mx), hipMemcpyHostToDevice, c.stream));
    c.comm->allreduce(d, 4, true, c.stream);
    DCP_HIP_CHECK(hipMemcpyAsync(mx, d, sizeof(mx), hipMemcpyDeviceToHost, c.stream));
    DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
    for (int k = 0; k < 4; ++k) c.max_owned[k] = int(mx[k]);
    c.old_nse_ghosted = c.old_T_ghosted = false;
    c.have_mesh = true;
    return DCP_OK;
  });
}

int dcp_mesh2d_partition_info(const dcp_mesh2d* m, int rank, int world, int field, int64_t* info,
                              int32_t* peers, int32_t* send_ptr, int64_t* send_gid,
                              int32_t* recv_ptr, int64_t* recv_gid) {
  return guarded(nullptr, [&] {
    require(m != nullptr && info != nullptr, DCP_ERR_INVALID, "NULL argument");
    require(field >= 0 && field < 3, DCP_ERR_INVALID, "field must be 0..2");
    Local2D L;
    try {
      L = localize_2d(*m, rank, world);
    } catch (const std::runtime_error& e) {
      fail(DCP_ERR_INVALID, e.what());
    }
    // the local mesh passes the upload's own checks
    int n_colors = 0;
    const dcp_mesh2d lv = L.view();
    mesh2d_check(&lv, &n_colors);
    const HaloPlan& h = field == 0 ? L.hu : field == 1 ? L.hp : L.hT;
    const int64_t v[11] = {L.n_cells, L.n_owned_cells, L.nuo, L.nug, L.npo, L.npg, L.nTo, L.nTg,
                           int64_t(h.peers.size()), int64_t(h.send_idx.size()),
                           int64_t(h.recv_idx.size())};
    std::copy(v, v + 11, info);
    if (peers) std::copy(h.peers.begin(), h.peers.end(), peers);
    if (send_ptr) std::copy(h.send_ptr.begin(), h.send_ptr.end(), send_ptr);
    if (recv_ptr) std::copy(h.recv_ptr.begin(), h.recv_ptr.end(), recv_ptr);
    if (send_gid) std::copy(h.send_gid.begin(), h.send_gid.end(), send_gid);
    if (recv_gid) std::copy(h.recv_gid.begin(), h.recv_gid.end(), recv_gid);
    return DCP_OK;
  });
}

int dcp_mesh2d_check(const dcp_mesh2d* m, int* n_colors) {
  return guarded(nullptr, [&] {
    mesh2d_check(m, n_colors);
    return DCP_OK;
  });
}

int dcp_prm_load(const char* path, dcp_run_params* out, char* err, int err_len) {
  try {
    if (!path || !out) throw std::invalid_argument("NULL argument");
    Parameters p;
    p.parse(PrmFile::read(path));
    const double L = p.reference_quantities.length, U = p.reference_quantities.velocity;
    dcp_physics& ph = out->physics;
    ph.time_step = p.time_step;
    ph.one_over_reynolds = 1.0 / p.reynolds();
    ph.one_over_peclet = 1.0 / p.peclet();
    ph.expansion_coefficient = p.physical_constants.expansion_coefficient;
    ph.temperature_ref = p.reference_quantities.temperature_ref;
    ph.gravity_scale = L / (U * U);
    ph.gravity_constant = p.physical_constants.gravity_constant;
    ph.coriolis_scale = L / U;
    ph.omega = p.physical_constants.omega;
    ph.cuboid = p.cuboid_geometry ? 1 : 0;
    ph.nse_solver_interval = int(p.NSE_solver_interval);
    ph.temperature_degree = int(p.temperature_degree);
    out->initial_global_refinement = int(p.initial_global_refinement);
    out->space_dimension = int(p.space_dimension);
    out->nse_velocity_degree = int(p.nse_velocity_degree);
    out->use_schur_complement_solver = p.use_schur_complement_solver;
    out->use_FEEC_solver = p.use_FEEC_solver;
    out->adapt_time_step = p.adapt_time_step;
    out->final_time = p.final_time;
    out->R0 = p.physical_constants.R0;
    out->R1 = p.physical_constants.R1;
    out->length = L;
    out->use_block_preconditioner_feec = p.use_block_preconditioner_feec ? 1 : 0;
    out->correct_pressure_to_zero_mean = p.correct_pressure_to_zero_mean ? 1 : 0;
    out->solver_diagnostics_level = int(p.solver_diagnostics_print_level);
    out->use_direct_solver = p.use_direct_solver ? 1 : 0;
    return DCP_OK;
  } catch (const std::exception& e) {
    if (err && err_len > 0) {
      std::strncpy(err, e.what(), size_t(err_len) - 1);
      err[err_len - 1] = 0;
    }
    return DCP_ERR_INVALID;
  }
}

}  // extern "C"
