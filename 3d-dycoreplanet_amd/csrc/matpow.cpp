// Matrix powers of the multi-GPU s-step inner solve (DCP_OPT_MATRIX_POWERS).
//
// An s-step block of the inner Schur GMRES (solver.cpp gmres_schur_sstep,
// DCP_OPT_GRAM_SCHMIDT = 3) forms the Newton basis w_i = (S - theta_i)
// w_{i-1} / sigma, i = 1..4, from the block's start vector w_0. Per SpMV, each
// rank needs the ghost entries of w_{i-1} its owned rows reach: four halo
// exchanges per block, each a latency-bound RCCL round (the reference's
// ghosted-vector Import before every operator apply). With the
// matrix powers a rank instead receives w_0 once, on every pressure dof within
// S-graph distance 4 of its owned rows, and computes w_1, w_2, w_3 itself on
// the ghost rows of depth <= 3, <= 2, <= 1: one exchange per block.
//
// The ghost rows are the owners' rows of S, entry for entry in the owner's
// order, their values copied from the owners after every formation of S. The
// SELL kernel sums a row's entries in an order that depends on the row only
// (kernels/linalg.hip k_sell_spmv: column pairs round robin over the four
// waves), so a ghost row computed here has the bits its owner computes, and
// the basis -- and the whole solve -- is bitwise the one of the per-SpMV
// exchanges (tests/test_multi_rank.py matrix-powers tests).
//
// Setup (collective, once per mesh): breadth-first over the S graph through
// the owners -- round t asks the owners of the depth-t dofs for their rows
// (column global ids and owners, in SELL order), the columns not yet seen are
// depth t + 1 -- then the depth-4 halo plan. Dofs that are not in the local
// mesh (depth >= 3 on the two-layer ghost mesh) get vector entries past n_p.
#include <algorithm>
#include <cstdint>
#include <numeric>
#include <stdexcept>
#include <unordered_map>
#include <vector>

#include "comm.h"
#include "context.h"
#include "device.h"

namespace dcp {

void make_halo(Ctx::Halo& h, const std::vector<int>& peers,
               const std::vector<std::vector<int32_t>>& spos,
               const std::vector<std::vector<int32_t>>& rpos);

namespace {

template <class T>
std::vector<T> download(const DBuf<T>& b, size_t n) {
  std::vector<T> h(n);
  if (n) DCP_HIP_CHECK(hipMemcpy(h.data(), b.p, n * sizeof(T), hipMemcpyDeviceToHost));
  return h;
}

// every rank sends send[r] to rank r and receives recv[r] from it (doubles;
// the ids sent are < 2^31, exact). Collective over all ranks.
std::vector<std::vector<double>> alltoallv(Ctx& c, const std::vector<std::vector<double>>& send) {
  const int P = c.comm->size, me = c.comm->rank;
  std::vector<int> peers;
  for (int r = 0; r < P; ++r)
    if (r != me) peers.push_back(r);
  const int np = int(peers.size());
  std::vector<std::vector<double>> recv(P);
  // counts
  std::vector<double> cnt(np);
  for (int i = 0; i < np; ++i) cnt[i] = double(send[peers[i]].size());
  DBuf<double> dc, dr;
  dc.upload(cnt);
  dr.alloc(size_t(np));
  std::vector<double*> sb(np), rb(np);
  std::vector<size_t> one(np, 1);
  for (int i = 0; i < np; ++i) {
    sb[i] = dc.p + i;
    rb[i] = dr.p + i;
  }
  c.comm->exchange(np, peers.data(), sb.data(), one.data(), rb.data(), one.data(), c.stream);
  DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
  const std::vector<double> rc = download(dr, size_t(np));
  // payloads
  std::vector<double> flat;
  std::vector<size_t> sn(np), rn(np), so(np), ro(np);
  size_t rtot = 0;
  for (int i = 0; i < np; ++i) {
    so[i] = flat.size();
    sn[i] = send[peers[i]].size();
    flat.insert(flat.end(), send[peers[i]].begin(), send[peers[i]].end());
    ro[i] = rtot;
    rn[i] = size_t(rc[i]);
    rtot += rn[i];
  }
  DBuf<double> ds, drr;
  ds.upload(flat);
  drr.alloc(rtot);
  for (int i = 0; i < np; ++i) {
    sb[i] = ds.p + so[i];
    rb[i] = drr.p + ro[i];
  }
  c.comm->exchange(np, peers.data(), sb.data(), sn.data(), rb.data(), rn.data(), c.stream);
  DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
  const std::vector<double> all = download(drr, rtot);
  for (int i = 0; i < np; ++i)
    recv[peers[i]].assign(all.begin() + long(ro[i]), all.begin() + long(ro[i] + rn[i]));
  recv[me] = send[me];
  return recv;
}

}  // namespace

void Ctx::MatPow::reset() {
  built = false;
  n_ext = 0;
  for (int& r : rows) r = 0;
  off.release();
  col.release();
  rowmap.release();
  val.release();
  version = -1;
}

void matpow_setup(Ctx& c) {
  if (!c.comm) throw std::runtime_error("matrix powers: one GPU has no ghost rows");
  if (c.S_perm.p) throw std::runtime_error("matrix powers: S in a permuted order");
  DCP_HIP_CHECK(hipStreamSynchronize(c.stream));
  const int me = c.comm->rank, P = c.comm->size;
  const int npo = c.npo, n_p = c.n_p;
  // this rank's rows of S in SELL order: row r, entry k = k-th smallest local
  // column (build_sell), SELL position sell_pos(off, r, k)
  const std::vector<int32_t> Sp = download(c.S_ptr, size_t(npo) + 1);
  std::vector<int32_t> Sc = download(c.S_col, size_t(Sp[npo]));
  for (int r = 0; r < npo; ++r) std::sort(Sc.begin() + Sp[r], Sc.begin() + Sp[r + 1]);
  const std::vector<int64_t> off = download(c.S_sell_off, size_t((npo + 63) / 64) + 1);
  // owners of the local ghosts (the receive lists of the pressure halo)
  std::vector<int> lowner(size_t(n_p), me);
  {
    const std::vector<int32_t> rp = download(c.halo_p.rpos, size_t(c.halo_p.nr));
    for (size_t i = 0; i < c.halo_p.peers.size(); ++i)
      for (size_t j = 0; j < c.halo_p.rn[i]; ++j) lowner[rp[c.halo_p.roff[i] + j]] = c.halo_p.peers[i];
  }
  std::unordered_map<int32_t, int32_t> lid;  // global id -> local id
  for (int i = 0; i < n_p; ++i) lid[c.p_g[i]] = i;
  // what this rank knows of a dof: depth from the owned rows, owner
  struct Dof {
    int depth, owner;
  };
  std::unordered_map<int32_t, Dof> seen;
  for (int i = 0; i < npo; ++i) seen[c.p_g[i]] = Dof{0, me};
  std::vector<std::vector<int32_t>> level(5);  // global ids per depth 1..4
  for (int r = 0; r < npo; ++r)
    for (int k = Sp[r]; k < Sp[r + 1]; ++k) {
      const int32_t g = c.p_g[Sc[k]];
      if (seen.emplace(g, Dof{1, lowner[Sc[k]]}).second) level[1].push_back(g);
    }
  // ghost rows: per depth-1..3 dof its entries (column global ids, SELL order)
  std::unordered_map<int32_t, std::vector<int32_t>> grow;
  // owner side: per requesting rank the SELL positions of the entries it
  // receives, in the order its ghost rows list them
  std::vector<std::vector<int32_t>> vsend(P);
  // requester side: per owner the rows asked for, in request order
  std::vector<std::vector<int32_t>> asked(P);
  for (int t = 1; t <= 3; ++t) {
    std::sort(level[t].begin(), level[t].end());
    std::vector<std::vector<double>> req(P);
    for (int32_t g : level[t]) {
      req[seen[g].owner].push_back(double(g));
      asked[seen[g].owner].push_back(g);
    }
    const auto in = alltoallv(c, req);
    // answer: per row [length, (column global id, column owner) ...]
    std::vector<std::vector<double>> ans(P);
    for (int q = 0; q < P; ++q)
      for (double dg : in[q]) {
        const auto it = lid.find(int32_t(dg));
        if (it == lid.end() || it->second >= npo)
          throw std::runtime_error("matrix powers: row requested from a rank that does not own it");
        const int r = it->second;
        ans[q].push_back(double(Sp[r + 1] - Sp[r]));
        for (int k = Sp[r]; k < Sp[r + 1]; ++k) {
          ans[q].push_back(double(c.p_g[Sc[k]]));
          ans[q].push_back(double(lowner[Sc[k]]));
          vsend[q].push_back(int32_t(sell_pos(off.data(), r, k - Sp[r])));
        }
      }
    const auto back = alltoallv(c, ans);
    for (int q = 0; q < P; ++q) {
      const std::vector<double>& a = back[q];
      size_t pos = 0;
      for (double dg : req[q]) {
        const int32_t g = int32_t(dg);
        if (pos >= a.size()) throw std::runtime_error("matrix powers: short row answer");
        const int len = int(a[pos++]);
        std::vector<int32_t>& row = grow[g];
        row.resize(size_t(len));
        for (int k = 0; k < len; ++k) {
          const int32_t cg = int32_t(a[pos]);
          const int co = int(a[pos + 1]);
          pos += 2;
          row[k] = cg;
          if (seen.emplace(cg, Dof{t + 1, co}).second) level[t + 1].push_back(cg);
        }
      }
    }
  }
  std::sort(level[4].begin(), level[4].end());
  // vector entries: the local mesh's dofs keep their local ids, the further
  // ones follow in ascending global id
  std::vector<int32_t> extra;
  for (int t = 1; t <= 4; ++t)
    for (int32_t g : level[t])
      if (!lid.count(g)) extra.push_back(g);
  std::sort(extra.begin(), extra.end());
  std::unordered_map<int32_t, int32_t> ext(lid);
  for (size_t j = 0; j < extra.size(); ++j) ext[extra[j]] = int32_t(n_p + j);
  auto mp = &c.mp;
  mp->reset();
  mp->n_ext = n_p + int(extra.size());
  // ghost rows by depth, then vector entry
  std::vector<int32_t> rowsg;
  mp->rows[0] = 0;
  for (int t = 1; t <= 3; ++t) {
    std::vector<int32_t> lv = level[t];
    std::sort(lv.begin(), lv.end(), [&](int32_t a, int32_t b) { return ext[a] < ext[b]; });
    rowsg.insert(rowsg.end(), lv.begin(), lv.end());
    mp->rows[t] = int(rowsg.size());
  }
  const int ng = int(rowsg.size());
  const int n_sl = (ng + 63) / 64;
  std::vector<int64_t> goff(size_t(n_sl) + 1, 0);
  for (int sl = 0; sl < n_sl; ++sl) {
    int w = 0;
    for (int r = 64 * sl; r < std::min(ng, 64 * sl + 64); ++r)
      w = std::max(w, int(grow[rowsg[r]].size()));
    w += w & 1;
    goff[sl + 1] = goff[sl] + 64 * int64_t(w);
  }
  const size_t len = size_t(goff[n_sl]);
  if (len >= size_t(INT32_MAX)) throw std::runtime_error("matrix powers: ghost rows above 2^31 entries");
  std::vector<int32_t> gcol(len, 0);
  std::vector<int32_t> gmap(static_cast<size_t>(ng));
  std::unordered_map<int32_t, int32_t> growidx;
  for (int r = 0; r < ng; ++r) {
    gmap[r] = ext[rowsg[r]];
    growidx[rowsg[r]] = r;
  }
  for (int sl = 0; sl < n_sl; ++sl) {
    const int w = int((goff[sl + 1] - goff[sl]) / 64);
    for (int i = 0; i < 64; ++i) {
      const int r = 64 * sl + i;
      for (int k = 0; k < w; ++k) {
        const int64_t pos = sell_pos(goff.data(), r, k);
        if (r >= ng) {
          gcol[pos] = gmap[ng - 1];
          continue;
        }
        const std::vector<int32_t>& row = grow[rowsg[r]];
        // padding: the row's own entry (valid whenever the row is computed)
        gcol[pos] = k < int(row.size()) ? ext[row[k]] : gmap[r];
      }
    }
  }
  mp->off.upload(goff);
  mp->col.upload(gcol);
  mp->rowmap.upload(gmap);
  mp->val.alloc(std::max<size_t>(len, 1));
  mp->val.zero(c.stream);  // padding entries stay 0
  // value plan: owner SELL positions -> ghost SELL positions
  {
    std::vector<int> peers;
    std::vector<std::vector<int32_t>> s, r;
    for (int q = 0; q < P; ++q) {
      if (q == me) continue;
      std::vector<int32_t> rp;
      for (int32_t g : asked[q]) {
        const int gr = growidx.at(g);
        const int L = int(grow[g].size());
        for (int k = 0; k < L; ++k) rp.push_back(int32_t(sell_pos(goff.data(), gr, k)));
      }
      if (vsend[q].empty() && rp.empty()) continue;
      peers.push_back(q);
      s.push_back(vsend[q]);
      r.push_back(std::move(rp));
    }
    make_halo(mp->vals, peers, s, r);
  }
  // depth-4 halo: every dof of depth 1..4 from its owner
  {
    std::vector<std::vector<double>> req(P);
    std::vector<std::vector<int32_t>> rpos(P);
    for (int t = 1; t <= 4; ++t)
      for (int32_t g : level[t]) {
        const int o = seen[g].owner;
        req[o].push_back(double(g));
        rpos[o].push_back(ext[g]);
      }
    const auto in = alltoallv(c, req);
    std::vector<int> peers;
    std::vector<std::vector<int32_t>> s, r;
    for (int q = 0; q < P; ++q) {
      if (q == me || (in[q].empty() && rpos[q].empty())) continue;
      std::vector<int32_t> sp;
      for (double dg : in[q]) {
        const auto it = lid.find(int32_t(dg));
        if (it == lid.end() || it->second >= npo)
          throw std::runtime_error("matrix powers: value requested from a rank that does not own it");
        sp.push_back(it->second);
      }
      peers.push_back(q);
      s.push_back(std::move(sp));
      r.push_back(std::move(rpos[q]));
    }
    make_halo(mp->halo, peers, s, r);
  }
  mp->built = true;
}

void matpow_prepare(Ctx& c) {
  if (!c.mp.built) matpow_setup(c);
  if (c.mp.version == c.S_version) return;
  // the ghost rows' values from their owners (after every formation of S)
  Ctx::Halo& h = c.mp.vals;
  gather(h.ns, h.spos.p, c.S_val.p, h.sbuf.p, c.stream);
  const int np = int(h.peers.size());
  std::vector<double*> sb(np), rb(np);
  for (int i = 0; i < np; ++i) {
    sb[i] = h.sbuf.p + h.soff[i];
    rb[i] = h.rbuf.p + h.roff[i];
  }
  c.comm->exchange(np, h.peers.data(), sb.data(), h.sn.data(), rb.data(), h.rn.data(), c.stream);
  scatter(h.nr, h.rpos.p, h.rbuf.p, c.mp.val.p, c.stream);
  c.mp.version = c.S_version;
}

}  // namespace dcp
