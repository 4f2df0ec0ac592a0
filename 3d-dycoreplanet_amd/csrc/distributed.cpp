// Distributed localisation (dcp_mesh_upload_distributed): a rank's LocalMesh
// built from what that rank holds in the reference's MPI run instead of from
// the global mesh (partition.h's localize). See include/dcp.h for the input.
//
//   ownership   the caller's locally_owned_dofs() ranges, all-gathered once;
//               the owner of a ghost dof is the rank whose range holds it
//   cells       the caller's owned cells and ghost layer; the second ghost
//               layer (neighbours of the ghost cells, which S = B D_A^-1 B^T
//               and the Jacobi diagonals of layer-1 nodes need) is requested
//               from the owners of the ghost cells, who hold every neighbour
//               of their owned cells, together with the constraint lines of
//               those cells' dofs
//   numbering   per field owned entities first, then ghosts, each ascending
//               by global id (as localize), so a caller that owns what
//               localize's rule assigns gets the same LocalMesh
//   halos       receive lists = my ghosts grouped by owner; send lists = the
//               receive lists the peers send me
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <unordered_set>

#include "fe_tables.h"
#include "partition.h"

namespace dcp {
namespace {

struct HostComm {
  const dcp_host_comm& c;
  void check(int rc, const char* what) const {
    if (rc != 0) throw std::runtime_error(std::string("dcp_host_comm ") + what + " failed");
  }
  std::vector<int64_t> allgather(const std::vector<int64_t>& mine) const {
    std::vector<int64_t> out(mine.size() * size_t(c.world));
    check(c.allgather(c.user, mine.data(), mine.size() * sizeof(int64_t), out.data()), "allgather");
    return out;
  }
  // per-destination int64 messages -> per-source messages
  std::vector<std::vector<int64_t>> exchange(const std::vector<std::vector<int64_t>>& out) const {
    const int W = c.world;
    std::vector<int64_t> counts(W);
    for (int s = 0; s < W; ++s) counts[s] = int64_t(out[s].size());
    const std::vector<int64_t> all = allgather(counts);  // all[q * W + s]: q sends s
    std::vector<size_t> sb(W), rb(W);
    size_t ns = 0, nr = 0;
    for (int s = 0; s < W; ++s) {
      sb[s] = out[s].size() * sizeof(int64_t);
      rb[s] = size_t(all[size_t(s) * W + c.rank]) * sizeof(int64_t);
      ns += sb[s];
      nr += rb[s];
    }
    std::vector<int64_t> send(ns / sizeof(int64_t) + 1), recv(nr / sizeof(int64_t) + 1);
    size_t o = 0;
    for (int s = 0; s < W; ++s) {
      std::copy(out[s].begin(), out[s].end(), send.begin() + o);
      o += out[s].size();
    }
    check(c.alltoallv(c.user, send.data(), sb.data(), recv.data(), rb.data()), "alltoallv");
    std::vector<std::vector<int64_t>> in(W);
    o = 0;
    for (int s = 0; s < W; ++s) {
      const size_t n = rb[s] / sizeof(int64_t);
      in[s].assign(recv.begin() + o, recv.begin() + o + n);
      o += n;
    }
    return in;
  }
};

// owner rank of a global index from the all-gathered [begin, end) ranges
struct Ranges {
  std::vector<int64_t> b, e;
  std::vector<int> rank;
  void build(const std::vector<int64_t>& all, int W, int k) {  // all[s * 6 + 2k], +1
    std::vector<int> order(W);
    for (int s = 0; s < W; ++s) order[s] = s;
    std::sort(order.begin(), order.end(), [&](int x, int y) { return all[6 * x + 2 * k] < all[6 * y + 2 * k]; });
    for (int s : order) {
      if (all[6 * s + 2 * k + 1] <= all[6 * s + 2 * k]) continue;  // empty range
      b.push_back(all[6 * s + 2 * k]);
      e.push_back(all[6 * s + 2 * k + 1]);
      rank.push_back(s);
    }
    for (size_t i = 1; i < b.size(); ++i)
      if (b[i] < e[i - 1]) throw std::runtime_error("distributed upload: owned ranges overlap");
  }
  int owner(int64_t g) const {
    const size_t i = size_t(std::upper_bound(b.begin(), b.end(), g) - b.begin());
    if (i == 0 || g >= e[i - 1]) throw std::runtime_error("distributed upload: dof owned by no rank");
    return rank[i - 1];
  }
};

struct Line {
  double inh;
  std::vector<std::pair<int64_t, double>> ent;
};
using LineMap = std::unordered_map<int64_t, Line>;

void read_lines(const dcp_constraints64& c, LineMap& out) {
  if (c.n_lines > 0 && (!c.line_dof || !c.entry_ptr || !c.inhomogeneity))
    throw std::runtime_error("distributed upload: NULL constraint array");
  for (int64_t l = 0; l < c.n_lines; ++l) {
    Line L{c.inhomogeneity[l], {}};
    for (int64_t k = c.entry_ptr[l]; k < c.entry_ptr[l + 1]; ++k) L.ent.push_back({c.entry_dof[k], c.entry_w[k]});
    out[c.line_dof[l]] = std::move(L);
  }
}

// a cell with its dofs' constraint lines, as exchanged between ranks
struct CellRec {
  int64_t id;
  int owner;
  std::vector<int64_t> nse, T;
  std::vector<double> geo;
  double diam;
};

void pack_lines(const LineMap& lines, const std::vector<int64_t>& dofs, std::vector<int64_t>& o) {
  size_t at = o.size();
  o.push_back(0);
  int64_t n = 0;
  for (int64_t d : dofs) {
    auto it = lines.find(d);
    if (it == lines.end()) continue;
    ++n;
    o.push_back(d);
    double inh = it->second.inh;
    int64_t bits;
    std::memcpy(&bits, &inh, 8);
    o.push_back(bits);
    o.push_back(int64_t(it->second.ent.size()));
    for (auto& e : it->second.ent) {
      o.push_back(e.first);
      std::memcpy(&bits, &e.second, 8);
      o.push_back(bits);
    }
  }
  o[at] = n;
}

size_t unpack_lines(const std::vector<int64_t>& in, size_t at, LineMap& lines) {
  const int64_t n = in[at++];
  for (int64_t k = 0; k < n; ++k) {
    const int64_t d = in[at++];
    Line L;
    std::memcpy(&L.inh, &in[at++], 8);
    const int64_t ne = in[at++];
    for (int64_t j = 0; j < ne; ++j) {
      double w;
      const int64_t e = in[at++];
      std::memcpy(&w, &in[at++], 8);
      L.ent.push_back({e, w});
    }
    lines.emplace(d, std::move(L));
  }
  return at;
}

void pack_cell(const CellRec& r, const LineMap& nl, const LineMap& tl, std::vector<int64_t>& o) {
  o.push_back(r.id);
  o.push_back(r.owner);
  o.insert(o.end(), r.nse.begin(), r.nse.end());
  o.insert(o.end(), r.T.begin(), r.T.end());
  for (double x : r.geo) {
    int64_t b;
    std::memcpy(&b, &x, 8);
    o.push_back(b);
  }
  int64_t b;
  std::memcpy(&b, &r.diam, 8);
  o.push_back(b);
  pack_lines(nl, r.nse, o);
  pack_lines(tl, r.T, o);
}

size_t unpack_cell(const std::vector<int64_t>& in, size_t at, int tdpc, CellRec& r, LineMap& nl,
                   LineMap& tl) {
  r.id = in[at++];
  r.owner = int(in[at++]);
  r.nse.assign(in.begin() + at, in.begin() + at + kNseDofs);
  at += kNseDofs;
  r.T.assign(in.begin() + at, in.begin() + at + tdpc);
  at += tdpc;
  r.geo.resize(3 * kMapPts);
  for (int i = 0; i < 3 * kMapPts; ++i) std::memcpy(&r.geo[i], &in[at++], 8);
  std::memcpy(&r.diam, &in[at++], 8);
  at = unpack_lines(in, at, nl);
  return unpack_lines(in, at, tl);
}

}  // namespace

LocalMesh localize_distributed(const dcp_dist_mesh& m, const dcp_host_comm& hc) {
  if (!hc.allgather || !hc.alltoallv) throw std::runtime_error("distributed upload: NULL communicator");
  const int W = hc.world, R = hc.rank;
  if (W < 1 || R < 0 || R >= W) throw std::runtime_error("distributed upload: bad rank/world");
  const HostComm comm{hc};
  // ---- the caller's input, checked locally first; the verdict is all-gathered
  // before any other exchange, so a bad input on one rank fails every rank
  // instead of leaving the others blocked in a collective
  std::string bad;
  auto check = [&](bool ok, const char* msg) {
    if (!ok && bad.empty()) bad = std::string("distributed upload: ") + msg;
    return ok;
  };
  check(m.cell_id && m.cell_owner && m.cell_nse_dofs && m.cell_T_dofs && m.cell_geometry &&
            m.cell_diameter,
        "NULL array");
  check(m.n_cells >= 1 && m.n_owned_cells >= 1 && m.n_owned_cells <= m.n_cells, "bad cell counts");
  check(m.n_u > 0 && m.n_u % 3 == 0 && m.n_p > 0 && m.n_T > 0 &&
            m.n_u + m.n_p < (int64_t(1) << 31) && m.n_T < (int64_t(1) << 31),
        "bad global sizes (32-bit global ids)");
  check(m.u_begin % 3 == 0 && m.u_end % 3 == 0 && m.u_begin >= 0 && m.u_end <= m.n_u &&
            m.p_begin >= m.n_u && m.p_end <= m.n_u + m.n_p && m.T_begin >= 0 && m.T_end <= m.n_T,
        "owned ranges outside the blocks (velocity range aligned to support points)");
  const int64_t n_u = m.n_u, n_p = m.n_p, n_T = m.n_T, nvg = n_u / 3;
  const int tdpc = (n_T == nvg && n_T != n_p) ? 27 : 8;
  std::vector<CellRec> cells;
  std::unordered_map<int64_t, int> by_id;
  if (bad.empty()) {
    cells.resize(m.n_cells);
    for (int c = 0; c < m.n_cells && bad.empty(); ++c) {
      CellRec& r = cells[c];
      r.id = m.cell_id[c];
      r.owner = m.cell_owner[c];
      if (!check((c < m.n_owned_cells) == (r.owner == R),
                 "the first n_owned_cells cells must be the owned ones") ||
          !check(r.owner >= 0 && r.owner < W, "bad cell owner"))
        break;
      r.nse.assign(m.cell_nse_dofs + size_t(c) * kNseDofs, m.cell_nse_dofs + size_t(c + 1) * kNseDofs);
      r.T.assign(m.cell_T_dofs + size_t(c) * tdpc, m.cell_T_dofs + size_t(c + 1) * tdpc);
      r.geo.assign(m.cell_geometry + size_t(c) * 3 * kMapPts,
                   m.cell_geometry + size_t(c + 1) * 3 * kMapPts);
      r.diam = m.cell_diameter[c];
      for (int64_t d : r.nse) check(d >= 0 && d < n_u + n_p, "NSE dof out of range");
      for (int64_t d : r.T) check(d >= 0 && d < n_T, "T dof out of range");
      check(by_id.emplace(r.id, c).second, "duplicate cell id");
    }
  }
  LineMap nlines, tlines;
  if (bad.empty()) {
    try {
      read_lines(m.nse, nlines);
      read_lines(m.T, tlines);
    } catch (const std::exception& e) {
      bad = e.what();
    }
  }
  for (int64_t f : comm.allgather({bad.empty() ? 0 : 1}))
    if (f) throw std::runtime_error(bad.empty() ? "distributed upload: another rank's input is invalid"
                                                : bad);
  // ---- ownership ranges of every rank: velocity nodes, pressure, temperature
  const std::vector<int64_t> all =
      comm.allgather({m.u_begin / 3, m.u_end / 3, m.p_begin - n_u, m.p_end - n_u, m.T_begin, m.T_end});
  Ranges rv, rp, rt;
  rv.build(all, W, 0);
  rp.build(all, W, 1);
  rt.build(all, W, 2);
  // ---- second ghost layer: ask the owner of each ghost cell for its neighbours
  std::vector<std::vector<int64_t>> req(W);
  for (int c = m.n_owned_cells; c < m.n_cells; ++c) req[cells[c].owner].push_back(cells[c].id);
  const std::vector<std::vector<int64_t>> asked = comm.exchange(req);
  // vertex (pressure dof) -> my cells
  std::unordered_map<int64_t, std::vector<int>> vcells;
  for (int c = 0; c < m.n_cells; ++c)
    for (int k = 0; k < kNseDofs; ++k)
      if (cells[c].nse[k] >= n_u) vcells[cells[c].nse[k]].push_back(c);
  std::vector<std::vector<int64_t>> reply(W);
  for (int q = 0; q < W; ++q) {
    std::unordered_set<int> sent;
    std::vector<int> list;
    for (int64_t id : asked[q]) {
      auto it = by_id.find(id);
      if (it == by_id.end() || cells[it->second].owner != R)
        throw std::runtime_error("distributed upload: a rank asked for a cell this rank does not own");
      const CellRec& g = cells[it->second];
      for (int k = 0; k < kNseDofs; ++k)
        if (g.nse[k] >= n_u)
          for (int o : vcells[g.nse[k]])
            if (sent.insert(o).second) list.push_back(o);
    }
    std::sort(list.begin(), list.end());
    for (int o : list) pack_cell(cells[o], nlines, tlines, reply[q]);
  }
  const std::vector<std::vector<int64_t>> got = comm.exchange(reply);
  for (int s = 0; s < W; ++s) {
    size_t at = 0;
    while (at < got[s].size()) {
      CellRec r;
      at = unpack_cell(got[s], at, tdpc, r, nlines, tlines);
      if (by_id.count(r.id)) continue;
      by_id.emplace(r.id, int(cells.size()));
      cells.push_back(std::move(r));
    }
  }
  // ---- local cells: owned (caller's order), then ghosts ascending by id
  std::vector<int> order;
  for (int c = 0; c < m.n_owned_cells; ++c) order.push_back(c);
  std::vector<int> ghosts;
  for (int c = m.n_owned_cells; c < int(cells.size()); ++c) ghosts.push_back(c);
  std::sort(ghosts.begin(), ghosts.end(), [&](int a, int b) { return cells[a].id < cells[b].id; });
  order.insert(order.end(), ghosts.begin(), ghosts.end());
  LocalMesh L;
  L.rank = R;
  L.world = W;
  L.n_cells = int(order.size());
  L.n_owned_cells = m.n_owned_cells;
  for (int c : order) {
    if (cells[c].id < 0 || cells[c].id >= (int64_t(1) << 31))
      throw std::runtime_error("distributed upload: cell ids must fit 32 bits");
    L.cells_g.push_back(int32_t(cells[c].id));
  }
  // ---- entities per field, owned first then ghosts (ascending)
  auto split = [&](std::vector<int32_t>& ents, auto&& own, int& no, int& ng) {
    std::sort(ents.begin(), ents.end());
    ents.erase(std::unique(ents.begin(), ents.end()), ents.end());
    std::stable_partition(ents.begin(), ents.end(), [&](int32_t e) { return own(e) == R; });
    no = int(std::count_if(ents.begin(), ents.end(), [&](int32_t e) { return own(e) == R; }));
    ng = int(ents.size()) - no;
  };
  for (int c : order) {
    for (int k = 0; k < kNseDofs; ++k) {
      const int64_t d = cells[c].nse[k];
      if (d < n_u) {
        if (d % 3 == 0) L.vnode_g.push_back(int32_t(d / 3));
      } else {
        L.p_g.push_back(int32_t(d - n_u));
      }
    }
    for (int64_t t : cells[c].T) L.T_g.push_back(int32_t(t));
  }
  split(L.vnode_g, [&](int32_t e) { return rv.owner(e); }, L.nvo, L.nvg);
  split(L.p_g, [&](int32_t e) { return rp.owner(e); }, L.npo, L.npg);
  split(L.T_g, [&](int32_t e) { return rt.owner(e); }, L.nTo, L.nTg);
  std::unordered_map<int32_t, int32_t> vl, pl, Tl;
  for (size_t i = 0; i < L.vnode_g.size(); ++i) vl[L.vnode_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.p_g.size(); ++i) pl[L.p_g[i]] = int32_t(i);
  for (size_t i = 0; i < L.T_g.size(); ++i) Tl[L.T_g[i]] = int32_t(i);
  const int nu_loc = L.n_u();
  L.cell_nse_dofs.resize(size_t(L.n_cells) * kNseDofs);
  L.cell_T_dofs.resize(size_t(L.n_cells) * tdpc);
  L.geometry.resize(size_t(L.n_cells) * 3 * kMapPts);
  L.diameter.resize(L.n_cells);
  for (int lc = 0; lc < L.n_cells; ++lc) {
    const CellRec& r = cells[order[lc]];
    for (int k = 0; k < kNseDofs; ++k) {
      const int64_t d = r.nse[k];
      L.cell_nse_dofs[size_t(lc) * kNseDofs + k] =
          d < n_u ? 3 * vl.at(int32_t(d / 3)) + int32_t(d % 3) : nu_loc + pl.at(int32_t(d - n_u));
    }
    for (int v = 0; v < tdpc; ++v) L.cell_T_dofs[size_t(lc) * tdpc + v] = Tl.at(int32_t(r.T[v]));
    std::copy(r.geo.begin(), r.geo.end(), L.geometry.begin() + size_t(lc) * 3 * kMapPts);
    L.diameter[lc] = r.diam;
  }
  // ---- constraint lines of the local dofs (ascending global dof, as the
  // global localize visits them)
  auto local_nse = [&](int64_t d) -> int {
    if (d < n_u) {
      auto it = vl.find(int32_t(d / 3));
      return it == vl.end() ? -1 : 3 * it->second + int(d % 3);
    }
    auto it = pl.find(int32_t(d - n_u));
    return it == pl.end() ? -1 : nu_loc + it->second;
  };
  std::vector<int64_t> keys;
  for (auto& kv : nlines) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());
  L.nse_ptr.push_back(0);
  for (int64_t d : keys) {
    const int ld = local_nse(d);
    if (ld < 0) continue;
    const Line& ln = nlines[d];
    L.nse_line.push_back(ld);
    L.nse_inh.push_back(ln.inh);
    if (d < n_u)
      for (auto& e : ln.ent) {
        const int le = e.first < n_u ? local_nse(e.first) : -1;
        if (le < 0) throw std::runtime_error("distributed upload: constraint entry outside the local mesh");
        L.nse_edof.push_back(le);
        L.nse_w.push_back(e.second);
      }
    L.nse_ptr.push_back(int(L.nse_edof.size()));
  }
  keys.clear();
  for (auto& kv : tlines) keys.push_back(kv.first);
  std::sort(keys.begin(), keys.end());
  L.T_ptr.push_back(0);
  for (int64_t d : keys) {
    auto it = Tl.find(int32_t(d));
    if (it == Tl.end()) continue;
    const Line& ln = tlines[d];
    L.T_line.push_back(it->second);
    L.T_inh.push_back(ln.inh);
    for (auto& e : ln.ent) {
      auto jt = Tl.find(int32_t(e.first));
      if (jt == Tl.end()) throw std::runtime_error("distributed upload: constraint entry outside the local mesh");
      L.T_edof.push_back(jt->second);
      L.T_w.push_back(e.second);
    }
    L.T_ptr.push_back(int(L.T_edof.size()));
  }
  // ---- halos: my ghosts grouped by owner; the peers' ghost lists are my sends
  L.hv.width = 3;
  struct Field {
    HaloPlan* plan;
    const std::vector<int32_t>* ents;
    int no;
    const Ranges* own;
    const std::unordered_map<int32_t, int32_t>* lidx;
  };
  const Field fields[3] = {{&L.hv, &L.vnode_g, L.nvo, &rv, &vl},
                           {&L.hp, &L.p_g, L.npo, &rp, &pl},
                           {&L.hT, &L.T_g, L.nTo, &rt, &Tl}};
  for (const Field& f : fields) {
    std::vector<std::vector<int64_t>> recv(W);
    for (size_t i = size_t(f.no); i < f.ents->size(); ++i) {
      const int32_t e = (*f.ents)[i];
      recv[f.own->owner(e)].push_back(e);
    }
    const std::vector<std::vector<int64_t>> sends = comm.exchange(recv);
    HaloPlan& h = *f.plan;
    h.send_ptr.push_back(0);
    h.recv_ptr.push_back(0);
    for (int s = 0; s < W; ++s) {
      if (s == R || (sends[s].empty() && recv[s].empty())) continue;
      h.peers.push_back(s);
      for (int64_t e : sends[s]) {
        auto it = f.lidx->find(int32_t(e));
        if (it == f.lidx->end() || it->second >= f.no)
          throw std::runtime_error("distributed upload: a peer expects an entity this rank does not own");
        h.send_idx.push_back(it->second);
        h.send_gid.push_back(e);
      }
      for (int64_t e : recv[s]) {
        h.recv_idx.push_back(f.lidx->at(int32_t(e)));
        h.recv_gid.push_back(e);
      }
      h.send_ptr.push_back(int32_t(h.send_idx.size()));
      h.recv_ptr.push_back(int32_t(h.recv_idx.size()));
    }
  }
  return L;
}

}  // namespace dcp
