// Host partitioning for the multi-GPU path (see partition.h).
#include "partition.h"

#include "fe_tables.h"

#include <algorithm>
#include <stdexcept>
#include <string>

namespace dcp {

dcp_constraints LocalMesh::nse_view() const {
  return dcp_constraints{int(nse_line.size()), nse_line.data(), nse_ptr.data(), nse_edof.data(),
                         nse_w.data(), nse_inh.data()};
}
dcp_constraints LocalMesh::T_view() const {
  return dcp_constraints{int(T_line.size()), T_line.data(), T_ptr.data(), T_edof.data(),
                         T_w.data(), T_inh.data()};
}

namespace {

struct Global {
  int n_cells, nv, n_p, n_T, world;
  const int32_t* nse;   // [n][89] global dofs
  const int32_t* Td;    // [n][8]
  int n_u;
  std::vector<int64_t> start;                 // cell range of each rank
  std::vector<int32_t> vown, pown, Town;      // owner rank per entity
  std::vector<int32_t> pc_ptr, pc_cells;      // pressure dof (partner) -> cells
  // periodic partner per entity (itself if none): make_periodicity_constraints'
  // identity lines. Ghost layers grow across them (the partner's cells are
  // neighbours, as p4est's periodic ghost layer has them) and every local
  // image brings its partner, so each rank's constraint lines stay local.
  std::vector<int32_t> vfold, pfold, Tfold;

  int rank_of(int c) const {
    return int(std::upper_bound(start.begin(), start.end(), int64_t(c)) - start.begin()) - 1;
  }
};

// Owned cells of rank s followed by its two ghost layers (ascending).
std::vector<int32_t> local_cells(const Global& g, int s, std::vector<int>& stamp, int token) {
  std::vector<int32_t> owned, ghosts, frontier, next;
  for (int64_t c = g.start[s]; c < g.start[s + 1]; ++c) {
    owned.push_back(int32_t(c));
    stamp[c] = token;
  }
  frontier = owned;
  for (int layer = 0; layer < 2; ++layer) {
    next.clear();
    for (int32_t c : frontier)
      for (int k = 0; k < 89; ++k) {
        const int d = g.nse[size_t(c) * 89 + k];
        if (d < g.n_u) continue;
        const int p = g.pfold[d - g.n_u];
        for (int j = g.pc_ptr[p]; j < g.pc_ptr[p + 1]; ++j) {
          const int o = g.pc_cells[j];
          if (stamp[o] != token) {
            stamp[o] = token;
            next.push_back(o);
          }
        }
      }
    ghosts.insert(ghosts.end(), next.begin(), next.end());
    frontier.swap(next);
  }
  std::sort(ghosts.begin(), ghosts.end());
  owned.insert(owned.end(), ghosts.begin(), ghosts.end());
  return owned;
}

// Entities of one field present in a cell list, split owned / ghost by rank.
template <class F>
void collect(const std::vector<int32_t>& cells, F&& for_each_entity, std::vector<int>& stamp,
             int token, std::vector<int32_t>& out) {
  out.clear();
  for (int32_t c : cells)
    for_each_entity(c, [&](int e) {
      if (stamp[e] != token) {
        stamp[e] = token;
        out.push_back(e);
      }
    });
  std::sort(out.begin(), out.end());
}

}  // namespace

LocalMesh localize(int n_cells, const int32_t* cell_nse_dofs, const int32_t* cell_T_dofs,
                   const double* cell_geometry, const double* cell_diameter, int n_u, int n_p,
                   int n_T, const dcp_constraints* nse_c, const dcp_constraints* T_c, int rank,
                   int world) {
  if (!cell_nse_dofs || !cell_T_dofs || !cell_geometry || !cell_diameter)
    throw std::runtime_error("localize: NULL argument");
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("localize: bad rank/world");
  if (n_cells < world) throw std::runtime_error("localize: fewer cells than ranks");
  if (n_u <= 0 || n_u % 3 || n_p <= 0 || n_T <= 0) throw std::runtime_error("localize: bad sizes");
  // FE_Q(2) temperature: n_T = the Q2 support points (27 dofs per cell), else vertices (8)
  const int tdpc = (n_T == n_u / 3 && n_T != n_p) ? 27 : 8;
  Global g;
  g.n_cells = n_cells;
  g.n_u = n_u;
  g.nv = n_u / 3;
  g.n_p = n_p;
  g.n_T = n_T;
  g.world = world;
  g.nse = cell_nse_dofs;
  g.Td = cell_T_dofs;
  g.start.resize(size_t(world) + 1);
  for (int r = 0; r <= world; ++r) g.start[r] = int64_t(r) * n_cells / world;
  g.vown.assign(g.nv, -1);
  g.pown.assign(n_p, -1);
  g.Town.assign(n_T, -1);
  std::vector<int32_t> cnt(size_t(n_p) + 1, 0);
  for (int c = 0; c < n_cells; ++c) {
    const int rc = g.rank_of(c);
    for (int k = 0; k < 89; ++k) {
      const int d = cell_nse_dofs[size_t(c) * 89 + k];
      if (d < 0 || d >= n_u + n_p) throw std::runtime_error("localize: NSE dof out of range");
      if (d < n_u) {
        if (g.vown[d / 3] < 0) g.vown[d / 3] = rc;
      } else {
        if (g.pown[d - n_u] < 0) g.pown[d - n_u] = rc;
        cnt[d - n_u + 1]++;
      }
    }
    for (int v = 0; v < tdpc; ++v) {
      const int t = cell_T_dofs[size_t(c) * tdpc + v];
      if (t < 0 || t >= n_T) throw std::runtime_error("localize: T dof out of range");
      if (g.Town[t] < 0) g.Town[t] = rc;
    }
  }
  // periodic partners: lines "dof = partner" (one entry, weight 1, homogeneous)
  auto identity = [](const dcp_constraints* cs, int l) {
    const int b = cs->entry_ptr[l];
    return (cs->entry_ptr[l + 1] - b == 1 && cs->entry_w[b] == 1.0 && cs->inhomogeneity[l] == 0.0)
               ? cs->entry_dof[b]
               : -1;
  };
  g.vfold.resize(g.nv);
  g.pfold.resize(n_p);
  g.Tfold.resize(n_T);
  for (int i = 0; i < g.nv; ++i) g.vfold[i] = i;
  for (int i = 0; i < n_p; ++i) g.pfold[i] = i;
  for (int i = 0; i < n_T; ++i) g.Tfold[i] = i;
  if (nse_c)
    for (int l = 0; l < nse_c->n_lines; ++l) {
      const int d = nse_c->line_dof[l], t = identity(nse_c, l);
      if (d < 0 || d >= n_u + n_p || t < 0 || t >= n_u + n_p || t == d) continue;
      if (d < n_u && t < n_u && t / 3 != d / 3 && t % 3 == d % 3) g.vfold[d / 3] = t / 3;
      if (d >= n_u && t >= n_u) g.pfold[d - n_u] = t - n_u;
    }
  // Q1 temperature: the partner vertex's dof (via the pressure partner of
  // the same vertex, local dof 4v + 3), also where the image's identity line
  // was closed into a Dirichlet line: local T and p then cover the same
  // vertices, as prepare_mesh requires
  if (tdpc == 8) {
    std::vector<int32_t> pT(n_p, -1);
    for (int c = 0; c < n_cells; ++c)
      for (int v = 0; v < 8; ++v) {
        const int d = cell_nse_dofs[size_t(c) * 89 + 4 * v + 3];
        if (d >= n_u && d < n_u + n_p) pT[d - n_u] = cell_T_dofs[size_t(c) * 8 + v];
      }
    for (int c = 0; c < n_cells; ++c)
      for (int v = 0; v < 8; ++v) {
        const int d = cell_nse_dofs[size_t(c) * 89 + 4 * v + 3];
        const int t = cell_T_dofs[size_t(c) * 8 + v];
        if (d < n_u || d >= n_u + n_p || t < 0 || t >= n_T) continue;
        const int pf = g.pfold[d - n_u];
        if (pf != d - n_u && pT[pf] >= 0) g.Tfold[t] = pT[pf];
      }
  }
  if (T_c)
    for (int l = 0; l < T_c->n_lines; ++l) {
      const int d = T_c->line_dof[l], t = identity(T_c, l);
      if (d >= 0 && d < n_T && t >= 0 && t < n_T && t != d) g.Tfold[d] = t;
    }
  // cells per pressure partner (a periodic image's cells join its partner's)
  std::fill(cnt.begin(), cnt.end(), 0);
  for (int c = 0; c < n_cells; ++c)
    for (int k = 0; k < 89; ++k) {
      const int d = cell_nse_dofs[size_t(c) * 89 + k];
      if (d >= n_u) cnt[g.pfold[d - n_u] + 1]++;
    }
  for (int p = 0; p < n_p; ++p) cnt[p + 1] += cnt[p];
  g.pc_ptr = cnt;
  g.pc_cells.resize(size_t(cnt[n_p]));
  {
    std::vector<int32_t> f(cnt.begin(), cnt.end() - 1);
    for (int c = 0; c < n_cells; ++c)
      for (int k = 0; k < 89; ++k) {
        const int d = cell_nse_dofs[size_t(c) * 89 + k];
        if (d >= n_u) g.pc_cells[f[g.pfold[d - n_u]]++] = c;
      }
  }
  std::vector<int> cstamp(n_cells, -1), vstamp(g.nv, -1), pstamp(n_p, -1), Tstamp(n_T, -1);
  int token = 0;
  // a cell's entities and their periodic partners
  auto vnodes_of = [&](int c, auto&& emit) {
    for (int k = 0; k < 89; ++k) {
      const int d = cell_nse_dofs[size_t(c) * 89 + k];
      if (d < n_u && d % 3 == 0) {
        emit(d / 3);
        if (g.vfold[d / 3] != d / 3) emit(g.vfold[d / 3]);
      }
    }
  };
  auto pdofs_of = [&](int c, auto&& emit) {
    for (int k = 0; k < 89; ++k) {
      const int d = cell_nse_dofs[size_t(c) * 89 + k];
      if (d >= n_u) {
        emit(d - n_u);
        if (g.pfold[d - n_u] != d - n_u) emit(g.pfold[d - n_u]);
      }
    }
  };
  auto Tdofs_of = [&](int c, auto&& emit) {
    for (int v = 0; v < tdpc; ++v) {
      const int t = cell_T_dofs[size_t(c) * tdpc + v];
      emit(t);
      if (g.Tfold[t] != t) emit(g.Tfold[t]);
    }
  };

  LocalMesh L;
  L.rank = rank;
  L.world = world;
  L.cells_g = local_cells(g, rank, cstamp, token++);
  L.n_cells = int(L.cells_g.size());
  L.n_owned_cells = int(g.start[rank + 1] - g.start[rank]);
  // per-field entity lists: owned first, then ghosts (ascending global id)
  auto order = [&](std::vector<int32_t>& ents, const std::vector<int32_t>& own, int& no, int& ng) {
    std::stable_partition(ents.begin(), ents.end(), [&](int32_t e) { return own[e] == rank; });
    no = int(std::count_if(ents.begin(), ents.end(), [&](int32_t e) { return own[e] == rank; }));
    ng = int(ents.size()) - no;
  };
  collect(L.cells_g, vnodes_of, vstamp, token++, L.vnode_g);
  collect(L.cells_g, pdofs_of, pstamp, token++, L.p_g);
  collect(L.cells_g, Tdofs_of, Tstamp, token++, L.T_g);
  order(L.vnode_g, g.vown, L.nvo, L.nvg);
  order(L.p_g, g.pown, L.npo, L.npg);
  order(L.T_g, g.Town, L.nTo, L.nTg);
  std::vector<int32_t> vl(g.nv, -1), pl(n_p, -1), Tl(n_T, -1);
  for (size_t i = 0; i < L.vnode_g.size(); ++i) vl[L.vnode_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.p_g.size(); ++i) pl[L.p_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.T_g.size(); ++i) Tl[L.T_g[i]] = int32_t(i);
  const int nu_loc = L.n_u();
  L.cell_nse_dofs.resize(size_t(L.n_cells) * 89);
  L.cell_T_dofs.resize(size_t(L.n_cells) * tdpc);
  L.geometry.resize(size_t(L.n_cells) * 3 * kMapPts);
  L.diameter.resize(L.n_cells);
  for (int lc = 0; lc < L.n_cells; ++lc) {
    const int c = L.cells_g[lc];
    for (int k = 0; k < 89; ++k) {
      const int d = cell_nse_dofs[size_t(c) * 89 + k];
      L.cell_nse_dofs[size_t(lc) * 89 + k] =
          d < n_u ? 3 * vl[d / 3] + d % 3 : nu_loc + pl[d - n_u];
    }
    for (int v = 0; v < tdpc; ++v)
      L.cell_T_dofs[size_t(lc) * tdpc + v] = Tl[cell_T_dofs[size_t(c) * tdpc + v]];
    std::copy(cell_geometry + size_t(c) * 3 * kMapPts, cell_geometry + size_t(c) * 3 * kMapPts + 3 * kMapPts,
              L.geometry.begin() + size_t(lc) * 3 * kMapPts);
    L.diameter[lc] = cell_diameter[c];
  }
  // constraints restricted to local dofs
  L.nse_ptr.push_back(0);
  if (nse_c)
    for (int l = 0; l < nse_c->n_lines; ++l) {
      const int d = nse_c->line_dof[l];
      if (d >= n_u || vl[d / 3] < 0) {
        if (d >= n_u && pl[d - n_u] >= 0) {  // pressure lines (periodic identities)
          L.nse_line.push_back(nu_loc + pl[d - n_u]);
          L.nse_inh.push_back(nse_c->inhomogeneity[l]);
          for (int k = nse_c->entry_ptr[l]; k < nse_c->entry_ptr[l + 1]; ++k) {
            const int e = nse_c->entry_dof[k];
            const int le = e >= n_u && e < n_u + n_p && pl[e - n_u] >= 0 ? nu_loc + pl[e - n_u] : -1;
            if (le < 0) throw std::runtime_error("localize: constraint entry outside the local mesh");
            L.nse_edof.push_back(le);
            L.nse_w.push_back(nse_c->entry_w[k]);
          }
          L.nse_ptr.push_back(int(L.nse_edof.size()));
        }
        continue;
      }
      L.nse_line.push_back(3 * vl[d / 3] + d % 3);
      L.nse_inh.push_back(nse_c->inhomogeneity[l]);
      for (int k = nse_c->entry_ptr[l]; k < nse_c->entry_ptr[l + 1]; ++k) {
        const int e = nse_c->entry_dof[k];
        const int le = e < n_u && vl[e / 3] >= 0 ? 3 * vl[e / 3] + e % 3 : -1;
        if (le < 0) throw std::runtime_error("localize: constraint entry outside the local mesh");
        L.nse_edof.push_back(le);
        L.nse_w.push_back(nse_c->entry_w[k]);
      }
      L.nse_ptr.push_back(int(L.nse_edof.size()));
    }
  L.T_ptr.push_back(0);
  if (T_c)
    for (int l = 0; l < T_c->n_lines; ++l) {
      const int d = T_c->line_dof[l];
      if (d < 0 || d >= n_T || Tl[d] < 0) continue;
      L.T_line.push_back(Tl[d]);
      L.T_inh.push_back(T_c->inhomogeneity[l]);
      for (int k = T_c->entry_ptr[l]; k < T_c->entry_ptr[l + 1]; ++k) {
        const int e = T_c->entry_dof[k];
        if (e < 0 || e >= n_T || Tl[e] < 0)
          throw std::runtime_error("localize: constraint entry outside the local mesh");
        L.T_edof.push_back(Tl[e]);
        L.T_w.push_back(T_c->entry_w[k]);
      }
      L.T_ptr.push_back(int(L.T_edof.size()));
    }
  // halo plans. Receive: my ghosts grouped by owner. Send: my owned entities
  // present in another rank's local cells.
  L.hv.width = 3;
  struct Field {
    HaloPlan* plan;
    const std::vector<int32_t>* ents;
    const std::vector<int32_t>* own;
    const std::vector<int32_t>* lidx;
    int no;
    std::vector<int>* stamp;
    int kind;
  };
  Field fields[3] = {{&L.hv, &L.vnode_g, &g.vown, &vl, L.nvo, &vstamp, 0},
                     {&L.hp, &L.p_g, &g.pown, &pl, L.npo, &pstamp, 1},
                     {&L.hT, &L.T_g, &g.Town, &Tl, L.nTo, &Tstamp, 2}};
  std::vector<std::vector<std::vector<int32_t>>> sends(3, std::vector<std::vector<int32_t>>(world));
  for (int s = 0; s < world; ++s) {
    if (s == rank) continue;
    const std::vector<int32_t> cs = local_cells(g, s, cstamp, token++);
    for (auto& f : fields) {
      std::vector<int32_t> ents;
      if (f.kind == 0) collect(cs, vnodes_of, *f.stamp, token++, ents);
      else if (f.kind == 1) collect(cs, pdofs_of, *f.stamp, token++, ents);
      else collect(cs, Tdofs_of, *f.stamp, token++, ents);
      auto& out = sends[f.kind][s];
      for (int32_t e : ents)
        if ((*f.own)[e] == rank) out.push_back(e);
    }
  }
  for (auto& f : fields) {
    std::vector<std::vector<int32_t>> recv(world);
    for (size_t i = size_t(f.no); i < f.ents->size(); ++i) {
      const int32_t e = (*f.ents)[i];
      recv[(*f.own)[e]].push_back(e);
    }
    HaloPlan& h = *f.plan;
    h.send_ptr.push_back(0);
    h.recv_ptr.push_back(0);
    for (int s = 0; s < world; ++s) {
      if (s == rank || (sends[f.kind][s].empty() && recv[s].empty())) continue;
      h.peers.push_back(s);
      for (int32_t e : sends[f.kind][s]) {
        h.send_idx.push_back((*f.lidx)[e]);
        h.send_gid.push_back(e);
      }
      for (int32_t e : recv[s]) {
        h.recv_idx.push_back((*f.lidx)[e]);
        h.recv_gid.push_back(e);
      }
      h.send_ptr.push_back(int32_t(h.send_idx.size()));
      h.recv_ptr.push_back(int32_t(h.recv_idx.size()));
    }
  }
  return L;
}

dcp_feec_mesh FeecLocal::view() const {
  dcp_feec_mesh v{};
  v.n_cells = n_cells;
  v.n_w = n_w();
  v.n_u = n_u();
  v.n_p = n_cells;
  v.n_T = n_T();
  v.cell_w = cell_w.data();
  v.sign_w = sign_w.data();
  v.cell_u = cell_u.data();
  v.sign_u = sign_u.data();
  v.cell_vertices = vertices.data();
  v.cell_diameter = diameter.data();
  v.cell_T_dofs = cell_T.data();
  v.w_fixed = w_fixed.data();
  v.u_fixed = u_fixed.data();
  v.T = dcp_constraints{int(T_line.size()), T_line.data(), T_ptr.data(), T_edof.data(),
                        T_w.data(), T_inh.data()};
  return v;
}

FeecLocal localize_feec(const dcp_feec_mesh& m, int rank, int world) {
  const int nc = m.n_cells;
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("localize: bad rank/world");
  if (nc < world) throw std::runtime_error("localize: fewer cells than ranks");
  std::vector<int64_t> start(size_t(world) + 1);
  for (int r = 0; r <= world; ++r) start[r] = int64_t(r) * nc / world;
  auto rank_of = [&](int c) {
    return int(std::upper_bound(start.begin(), start.end(), int64_t(c)) - start.begin()) - 1;
  };
  // owners: rank of the lowest-index cell touching the entity
  std::vector<int32_t> wown(m.n_w, -1), uown(m.n_u, -1), Town(m.n_T, -1);
  for (int c = 0; c < nc; ++c) {
    const int rc = rank_of(c);
    for (int l = 0; l < 12; ++l) {
      const int e = m.cell_w[12 * size_t(c) + l];
      if (e < 0 || e >= m.n_w) throw std::runtime_error("localize: edge dof out of range");
      if (wown[e] < 0) wown[e] = rc;
    }
    for (int f = 0; f < 6; ++f) {
      const int u = m.cell_u[6 * size_t(c) + f];
      if (u < 0 || u >= m.n_u) throw std::runtime_error("localize: face dof out of range");
      if (uown[u] < 0) uown[u] = rc;
    }
    for (int v = 0; v < 8; ++v) {
      const int t = m.cell_T_dofs[8 * size_t(c) + v];
      if (t < 0 || t >= m.n_T) throw std::runtime_error("localize: T dof out of range");
      if (Town[t] < 0) Town[t] = rc;
    }
  }
  // periodic temperature partners (the cuboid's identity lines): a local
  // image brings its partner, so the rank's constraint lines stay local
  std::vector<int32_t> Tfold(m.n_T);
  for (int t = 0; t < m.n_T; ++t) Tfold[t] = t;
  for (int l = 0; l < m.T.n_lines; ++l) {
    const int d = m.T.line_dof[l], b = m.T.entry_ptr[l];
    if (d >= 0 && d < m.n_T && m.T.entry_ptr[l + 1] - b == 1 && m.T.entry_w[b] == 1.0 &&
        m.T.inhomogeneity[l] == 0.0 && m.T.entry_dof[b] >= 0 && m.T.entry_dof[b] < m.n_T)
      Tfold[d] = m.T.entry_dof[b];
  }
  // vertex (T dof) -> cells and edge -> cells, for the ghost layers: cells
  // sharing a vertex or an edge are neighbours (the periodic cuboid's edges are
  // identified across x = 0 / 1, y = 0 / 1, so its layers cross them)
  std::vector<int32_t> vptr(size_t(m.n_T) + 1, 0), vcells;
  for (int c = 0; c < nc; ++c)
    for (int v = 0; v < 8; ++v) vptr[m.cell_T_dofs[8 * size_t(c) + v] + 1]++;
  for (int t = 0; t < m.n_T; ++t) vptr[t + 1] += vptr[t];
  vcells.resize(size_t(vptr[m.n_T]));
  {
    std::vector<int32_t> f(vptr.begin(), vptr.end() - 1);
    for (int c = 0; c < nc; ++c)
      for (int v = 0; v < 8; ++v) vcells[f[m.cell_T_dofs[8 * size_t(c) + v]]++] = c;
  }
  std::vector<int32_t> eptr(size_t(m.n_w) + 1, 0), ecells;
  for (int c = 0; c < nc; ++c)
    for (int l = 0; l < 12; ++l) eptr[m.cell_w[12 * size_t(c) + l] + 1]++;
  for (int e = 0; e < m.n_w; ++e) eptr[e + 1] += eptr[e];
  ecells.resize(size_t(eptr[m.n_w]));
  {
    std::vector<int32_t> f(eptr.begin(), eptr.end() - 1);
    for (int c = 0; c < nc; ++c)
      for (int l = 0; l < 12; ++l) ecells[f[m.cell_w[12 * size_t(c) + l]]++] = c;
  }
  std::vector<int> cstamp(nc, -1), wstamp(m.n_w, -1), ustamp(m.n_u, -1), Tstamp(m.n_T, -1);
  int token = 0;
  auto cells_of = [&](int s) {
    const int tok = token++;
    std::vector<int32_t> owned, ghosts, frontier, next;
    for (int64_t c = start[s]; c < start[s + 1]; ++c) {
      owned.push_back(int32_t(c));
      cstamp[c] = tok;
    }
    frontier = owned;
    for (int layer = 0; layer < 2; ++layer) {
      next.clear();
      auto visit = [&](int o) {
        if (cstamp[o] != tok) {
          cstamp[o] = tok;
          next.push_back(o);
        }
      };
      for (int32_t c : frontier) {
        for (int v = 0; v < 8; ++v) {
          const int t = m.cell_T_dofs[8 * size_t(c) + v];
          for (int j = vptr[t]; j < vptr[t + 1]; ++j) visit(vcells[j]);
        }
        for (int l = 0; l < 12; ++l) {
          const int e = m.cell_w[12 * size_t(c) + l];
          for (int j = eptr[e]; j < eptr[e + 1]; ++j) visit(ecells[j]);
        }
      }
      ghosts.insert(ghosts.end(), next.begin(), next.end());
      frontier.swap(next);
    }
    std::sort(ghosts.begin(), ghosts.end());
    owned.insert(owned.end(), ghosts.begin(), ghosts.end());
    return owned;
  };
  auto w_of = [&](int c, auto&& emit) {
    for (int l = 0; l < 12; ++l) emit(m.cell_w[12 * size_t(c) + l]);
  };
  auto u_of = [&](int c, auto&& emit) {
    for (int f = 0; f < 6; ++f) emit(m.cell_u[6 * size_t(c) + f]);
  };
  auto T_of = [&](int c, auto&& emit) {
    for (int v = 0; v < 8; ++v) {
      const int t = m.cell_T_dofs[8 * size_t(c) + v];
      emit(t);
      if (Tfold[t] != t) emit(Tfold[t]);
    }
  };
  FeecLocal L;
  L.rank = rank;
  L.world = world;
  L.cells_g = cells_of(rank);
  L.n_cells = int(L.cells_g.size());
  L.n_owned_cells = int(start[rank + 1] - start[rank]);
  auto order = [&](std::vector<int32_t>& ents, const std::vector<int32_t>& own, int& no, int& ng) {
    std::stable_partition(ents.begin(), ents.end(), [&](int32_t e) { return own[e] == rank; });
    no = int(std::count_if(ents.begin(), ents.end(), [&](int32_t e) { return own[e] == rank; }));
    ng = int(ents.size()) - no;
  };
  collect(L.cells_g, w_of, wstamp, token++, L.w_g);
  collect(L.cells_g, u_of, ustamp, token++, L.u_g);
  collect(L.cells_g, T_of, Tstamp, token++, L.T_g);
  order(L.w_g, wown, L.nwo, L.nwg);
  order(L.u_g, uown, L.nuo, L.nug);
  order(L.T_g, Town, L.nTo, L.nTg);
  std::vector<int32_t> wl(m.n_w, -1), ul(m.n_u, -1), Tl(m.n_T, -1), cl(nc, -1);
  for (size_t i = 0; i < L.w_g.size(); ++i) wl[L.w_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.u_g.size(); ++i) ul[L.u_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.T_g.size(); ++i) Tl[L.T_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.cells_g.size(); ++i) cl[L.cells_g[i]] = int32_t(i);
  const int lc_n = L.n_cells;
  L.cell_w.resize(size_t(lc_n) * 12);
  L.sign_w.resize(size_t(lc_n) * 12);
  L.cell_u.resize(size_t(lc_n) * 6);
  L.sign_u.resize(size_t(lc_n) * 6);
  L.cell_T.resize(size_t(lc_n) * 8);
  L.vertices.resize(size_t(lc_n) * 24);
  L.diameter.resize(lc_n);
  for (int lc = 0; lc < lc_n; ++lc) {
    const size_t c = size_t(L.cells_g[lc]);
    for (int l = 0; l < 12; ++l) {
      L.cell_w[12 * size_t(lc) + l] = wl[m.cell_w[12 * c + l]];
      L.sign_w[12 * size_t(lc) + l] = m.sign_w[12 * c + l];
    }
    for (int f = 0; f < 6; ++f) {
      L.cell_u[6 * size_t(lc) + f] = ul[m.cell_u[6 * c + f]];
      L.sign_u[6 * size_t(lc) + f] = m.sign_u[6 * c + f];
    }
    for (int v = 0; v < 8; ++v) L.cell_T[8 * size_t(lc) + v] = Tl[m.cell_T_dofs[8 * c + v]];
    std::copy(m.cell_vertices + 24 * c, m.cell_vertices + 24 * c + 24,
              L.vertices.begin() + 24 * size_t(lc));
    L.diameter[lc] = m.cell_diameter[c];
  }
  L.w_fixed.resize(L.w_g.size());
  L.u_fixed.resize(L.u_g.size());
  for (size_t i = 0; i < L.w_g.size(); ++i) L.w_fixed[i] = m.w_fixed[L.w_g[i]];
  for (size_t i = 0; i < L.u_g.size(); ++i) L.u_fixed[i] = m.u_fixed[L.u_g[i]];
  L.T_ptr.push_back(0);
  for (int l = 0; l < m.T.n_lines; ++l) {
    const int d = m.T.line_dof[l];
    if (d < 0 || d >= m.n_T || Tl[d] < 0) continue;
    L.T_line.push_back(Tl[d]);
    L.T_inh.push_back(m.T.inhomogeneity[l]);
    for (int k = m.T.entry_ptr[l]; k < m.T.entry_ptr[l + 1]; ++k) {
      const int e = m.T.entry_dof[k];
      if (e < 0 || e >= m.n_T || Tl[e] < 0)
        throw std::runtime_error("localize: constraint entry outside the local mesh");
      L.T_edof.push_back(Tl[e]);
      L.T_w.push_back(m.T.entry_w[k]);
    }
    L.T_ptr.push_back(int(L.T_edof.size()));
  }
  // halo plans: my ghosts grouped by owner; my owned entities in other
  // ranks' local cells
  std::vector<int32_t> cown(nc);
  for (int c = 0; c < nc; ++c) cown[c] = rank_of(c);
  std::vector<int32_t> pg_sorted;  // p: entities are cells
  struct Field {
    HaloPlan* plan;
    const std::vector<int32_t>* ents;
    const std::vector<int32_t>* own;
    const std::vector<int32_t>* lidx;
    int no;
  };
  const int npo = L.n_owned_cells;
  Field fields[4] = {{&L.hw, &L.w_g, &wown, &wl, L.nwo},
                     {&L.hu, &L.u_g, &uown, &ul, L.nuo},
                     {&L.hp, &L.cells_g, &cown, &cl, npo},
                     {&L.hT, &L.T_g, &Town, &Tl, L.nTo}};
  std::vector<std::vector<std::vector<int32_t>>> sends(4, std::vector<std::vector<int32_t>>(world));
  for (int s = 0; s < world; ++s) {
    if (s == rank) continue;
    const std::vector<int32_t> cs = cells_of(s);
    for (int f = 0; f < 4; ++f) {
      std::vector<int32_t> ents;
      if (f == 0) collect(cs, w_of, wstamp, token++, ents);
      else if (f == 1) collect(cs, u_of, ustamp, token++, ents);
      else if (f == 2) { ents = cs; std::sort(ents.begin(), ents.end()); }
      else collect(cs, T_of, Tstamp, token++, ents);
      for (int32_t e : ents)
        if ((*fields[f].own)[e] == rank) sends[f][s].push_back(e);
    }
  }
  for (int f = 0; f < 4; ++f) {
    const Field& F = fields[f];
    std::vector<std::vector<int32_t>> recv(world);
    for (size_t i = size_t(F.no); i < F.ents->size(); ++i) {
      const int32_t e = (*F.ents)[i];
      recv[(*F.own)[e]].push_back(e);
    }
    HaloPlan& h = *F.plan;
    h.send_ptr.push_back(0);
    h.recv_ptr.push_back(0);
    for (int s = 0; s < world; ++s) {
      if (s == rank || (sends[f][s].empty() && recv[s].empty())) continue;
      h.peers.push_back(s);
      for (int32_t e : sends[f][s]) {
        h.send_idx.push_back((*F.lidx)[e]);
        h.send_gid.push_back(e);
      }
      for (int32_t e : recv[s]) {
        h.recv_idx.push_back((*F.lidx)[e]);
        h.recv_gid.push_back(e);
      }
      h.send_ptr.push_back(int32_t(h.send_idx.size()));
      h.recv_ptr.push_back(int32_t(h.recv_idx.size()));
    }
  }
  return L;
}

dcp_mesh2d Local2D::view() const {
  dcp_mesh2d v{};
  v.n_cells = n_cells;
  v.n_u = n_u();
  v.n_p = n_p();
  v.n_T = n_T();
  v.temperature_degree = tdpc == 9 ? 2 : 1;
  v.cell_nse_dofs = cell_dofs.data();
  v.cell_T_dofs = cell_T.data();
  v.cell_geometry = geometry.data();
  v.cell_diameter = diameter.data();
  v.nse = dcp_constraints{int(nse_line.size()), nse_line.data(), nse_ptr.data(), nse_edof.data(),
                          nse_w.data(), nse_inh.data()};
  v.T = dcp_constraints{int(T_line.size()), T_line.data(), T_ptr.data(), T_edof.data(), T_w.data(),
                        T_inh.data()};
  return v;
}

Local2D localize_2d(const dcp_mesh2d& m, int rank, int world) {
  const int nc = m.n_cells, nu = m.n_u, np = m.n_p, nT = m.n_T;
  if (world < 1 || rank < 0 || rank >= world) throw std::runtime_error("localize: bad rank/world");
  if (nc < world) throw std::runtime_error("localize: fewer cells than ranks");
  if (!m.cell_nse_dofs || !m.cell_T_dofs || !m.cell_geometry || !m.cell_diameter)
    throw std::runtime_error("localize: NULL array");
  if (m.temperature_degree != 1 && m.temperature_degree != 2)
    throw std::runtime_error("localize: 2D temperature degree must be 1 or 2");
  const int tdpc = m.temperature_degree == 1 ? 4 : 9;
  // FESystem(FE_Q(2)^2, FE_Q(1)) local dof: pressure at 2, 5, 8, 11 (the vertices)
  auto is_p = [](int i) { return i < 12 && i % 3 == 2; };
  std::vector<int64_t> start(size_t(world) + 1);
  for (int r = 0; r <= world; ++r) start[r] = int64_t(r) * nc / world;
  auto rank_of = [&](int c) {
    return int(std::upper_bound(start.begin(), start.end(), int64_t(c)) - start.begin()) - 1;
  };
  std::vector<int32_t> uown(nu, -1), pown(np, -1), Town(nT, -1);
  std::vector<int32_t> pptr(size_t(np) + 1, 0), pcells;
  for (int c = 0; c < nc; ++c) {
    const int rc = rank_of(c);
    for (int i = 0; i < 22; ++i) {
      const int d = m.cell_nse_dofs[22 * size_t(c) + i];
      if (is_p(i)) {
        if (d < nu || d >= nu + np) throw std::runtime_error("localize: pressure dof out of range");
        if (pown[d - nu] < 0) pown[d - nu] = rc;
        pptr[d - nu + 1]++;
      } else {
        if (d < 0 || d >= nu) throw std::runtime_error("localize: velocity dof out of range");
        if (uown[d] < 0) uown[d] = rc;
      }
    }
    for (int v = 0; v < tdpc; ++v) {
      const int t = m.cell_T_dofs[size_t(tdpc) * c + v];
      if (t < 0 || t >= nT) throw std::runtime_error("localize: T dof out of range");
      if (Town[t] < 0) Town[t] = rc;
    }
  }
  for (int p = 0; p < np; ++p) pptr[p + 1] += pptr[p];
  pcells.resize(size_t(pptr[np]));
  {
    std::vector<int32_t> f(pptr.begin(), pptr.end() - 1);
    for (int c = 0; c < nc; ++c)
      for (int i = 2; i < 12; i += 3) pcells[f[m.cell_nse_dofs[22 * size_t(c) + i] - nu]++] = c;
  }
  std::vector<int> cstamp(nc, -1), ustamp(nu, -1), pstamp(np, -1), Tstamp(nT, -1);
  int token = 0;
  auto cells_of = [&](int s) {
    const int tok = token++;
    std::vector<int32_t> owned, ghosts, frontier, next;
    for (int64_t c = start[s]; c < start[s + 1]; ++c) {
      owned.push_back(int32_t(c));
      cstamp[c] = tok;
    }
    frontier = owned;
    for (int layer = 0; layer < 2; ++layer) {
      next.clear();
      for (int32_t c : frontier)
        for (int i = 2; i < 12; i += 3) {
          const int p = m.cell_nse_dofs[22 * size_t(c) + i] - nu;
          for (int j = pptr[p]; j < pptr[p + 1]; ++j)
            if (cstamp[pcells[j]] != tok) {
              cstamp[pcells[j]] = tok;
              next.push_back(pcells[j]);
            }
        }
      ghosts.insert(ghosts.end(), next.begin(), next.end());
      frontier.swap(next);
    }
    std::sort(ghosts.begin(), ghosts.end());
    owned.insert(owned.end(), ghosts.begin(), ghosts.end());
    return owned;
  };
  auto u_of = [&](int c, auto&& emit) {
    for (int i = 0; i < 22; ++i)
      if (!is_p(i)) emit(m.cell_nse_dofs[22 * size_t(c) + i]);
  };
  auto p_of = [&](int c, auto&& emit) {
    for (int i = 2; i < 12; i += 3) emit(m.cell_nse_dofs[22 * size_t(c) + i] - nu);
  };
  auto T_of = [&](int c, auto&& emit) {
    for (int v = 0; v < tdpc; ++v) emit(m.cell_T_dofs[size_t(tdpc) * c + v]);
  };
  Local2D L;
  L.rank = rank;
  L.world = world;
  L.tdpc = tdpc;
  L.cells_g = cells_of(rank);
  L.n_cells = int(L.cells_g.size());
  L.n_owned_cells = int(start[rank + 1] - start[rank]);
  auto order = [&](std::vector<int32_t>& ents, const std::vector<int32_t>& own, int& no, int& ng) {
    std::stable_partition(ents.begin(), ents.end(), [&](int32_t e) { return own[e] == rank; });
    no = int(std::count_if(ents.begin(), ents.end(), [&](int32_t e) { return own[e] == rank; }));
    ng = int(ents.size()) - no;
  };
  collect(L.cells_g, u_of, ustamp, token++, L.u_g);
  collect(L.cells_g, p_of, pstamp, token++, L.p_g);
  collect(L.cells_g, T_of, Tstamp, token++, L.T_g);
  order(L.u_g, uown, L.nuo, L.nug);
  order(L.p_g, pown, L.npo, L.npg);
  order(L.T_g, Town, L.nTo, L.nTg);
  std::vector<int32_t> ul(nu, -1), pl(np, -1), Tl(nT, -1);
  for (size_t i = 0; i < L.u_g.size(); ++i) ul[L.u_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.p_g.size(); ++i) pl[L.p_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.T_g.size(); ++i) Tl[L.T_g[i]] = int32_t(i);
  const int nul = L.n_u();
  auto local_nse = [&](int d) { return d < nu ? ul[d] : (pl[d - nu] < 0 ? -1 : nul + pl[d - nu]); };
  L.cell_dofs.resize(size_t(L.n_cells) * 22);
  L.cell_T.resize(size_t(L.n_cells) * tdpc);
  L.geometry.resize(size_t(L.n_cells) * 32);
  L.diameter.resize(L.n_cells);
  for (int lc = 0; lc < L.n_cells; ++lc) {
    const size_t c = size_t(L.cells_g[lc]);
    for (int i = 0; i < 22; ++i) L.cell_dofs[22 * size_t(lc) + i] = local_nse(m.cell_nse_dofs[22 * c + i]);
    for (int v = 0; v < tdpc; ++v) L.cell_T[size_t(tdpc) * lc + v] = Tl[m.cell_T_dofs[tdpc * c + v]];
    std::copy(m.cell_geometry + 32 * c, m.cell_geometry + 32 * c + 32, L.geometry.begin() + 32 * size_t(lc));
    L.diameter[lc] = m.cell_diameter[c];
  }
  // constraint lines of the local dofs (entries must be local: node-local lines)
  L.nse_ptr.push_back(0);
  for (int l = 0; l < m.nse.n_lines; ++l) {
    const int d = m.nse.line_dof[l];
    if (d < 0 || d >= nu + np || local_nse(d) < 0) continue;
    L.nse_line.push_back(local_nse(d));
    L.nse_inh.push_back(m.nse.inhomogeneity[l]);
    for (int k = m.nse.entry_ptr[l]; k < m.nse.entry_ptr[l + 1]; ++k) {
      const int e = m.nse.entry_dof[k];
      const int le = e >= 0 && e < nu + np ? local_nse(e) : -1;
      if (le < 0) throw std::runtime_error("localize: constraint entry outside the local mesh");
      L.nse_edof.push_back(le);
      L.nse_w.push_back(m.nse.entry_w[k]);
    }
    L.nse_ptr.push_back(int(L.nse_edof.size()));
  }
  L.T_ptr.push_back(0);
  for (int l = 0; l < m.T.n_lines; ++l) {
    const int d = m.T.line_dof[l];
    if (d < 0 || d >= nT || Tl[d] < 0) continue;
    L.T_line.push_back(Tl[d]);
    L.T_inh.push_back(m.T.inhomogeneity[l]);
    for (int k = m.T.entry_ptr[l]; k < m.T.entry_ptr[l + 1]; ++k) {
      const int e = m.T.entry_dof[k];
      if (e < 0 || e >= nT || Tl[e] < 0)
        throw std::runtime_error("localize: constraint entry outside the local mesh");
      L.T_edof.push_back(Tl[e]);
      L.T_w.push_back(m.T.entry_w[k]);
    }
    L.T_ptr.push_back(int(L.T_edof.size()));
  }
  // halo plans: my ghosts grouped by owner; my owned entities in other ranks' cells
  struct Field {
    HaloPlan* plan;
    const std::vector<int32_t>* ents;
    const std::vector<int32_t>* own;
    const std::vector<int32_t>* lidx;
    int no;
  };
  Field fields[3] = {{&L.hu, &L.u_g, &uown, &ul, L.nuo},
                     {&L.hp, &L.p_g, &pown, &pl, L.npo},
                     {&L.hT, &L.T_g, &Town, &Tl, L.nTo}};
  std::vector<std::vector<std::vector<int32_t>>> sends(3, std::vector<std::vector<int32_t>>(world));
  for (int s = 0; s < world; ++s) {
    if (s == rank) continue;
    const std::vector<int32_t> cs = cells_of(s);
    for (int f = 0; f < 3; ++f) {
      std::vector<int32_t> ents;
      if (f == 0) collect(cs, u_of, ustamp, token++, ents);
      else if (f == 1) collect(cs, p_of, pstamp, token++, ents);
      else collect(cs, T_of, Tstamp, token++, ents);
      for (int32_t e : ents)
        if ((*fields[f].own)[e] == rank) sends[f][s].push_back(e);
    }
  }
  for (int f = 0; f < 3; ++f) {
    const Field& F = fields[f];
    std::vector<std::vector<int32_t>> recv(world);
    for (size_t i = size_t(F.no); i < F.ents->size(); ++i) {
      const int32_t e = (*F.ents)[i];
      recv[(*F.own)[e]].push_back(e);
    }
    HaloPlan& h = *F.plan;
    h.send_ptr.push_back(0);
    h.recv_ptr.push_back(0);
    for (int s = 0; s < world; ++s) {
      if (s == rank || (sends[f][s].empty() && recv[s].empty())) continue;
      h.peers.push_back(s);
      for (int32_t e : sends[f][s]) {
        h.send_idx.push_back((*F.lidx)[e]);
        h.send_gid.push_back(e);
      }
      for (int32_t e : recv[s]) {
        h.recv_idx.push_back((*F.lidx)[e]);
        h.recv_gid.push_back(e);
      }
      h.send_ptr.push_back(int32_t(h.send_idx.size()));
      h.recv_ptr.push_back(int32_t(h.recv_idx.size()));
    }
  }
  return L;
}

}  // namespace dcp
