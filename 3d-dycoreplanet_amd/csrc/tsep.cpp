// Upload-time tables of the separable temperature assembly (kernels/temperature_sep.hip).
//
// The classic shell's cells are the full product (lateral column) x (radial
// layer) and its FE_Q(1) temperature dofs the product (lateral vertex) x
// (radial level), so the reference's assembled temperature matrices
// (local_assemble_temperature_matrix + copy, boussinesq_model.tpp:748-817)
// are sums of Kronecker products of lateral and radial matrices (see the
// kernel file). This builds, from the cell -> dof map alone:
//   * the radial order of the layers and the lateral vertex / level of
//     every dof (radial edges of the cells joined by union-find);
//   * the lateral columns, the column id of every (column, layer kind) and the
//     kind of every layer (layers are of one kind when every column uses the
//     same column id in them: MappingQ(3) boundary layers, MappingQ1 inside);
//   * the lateral pattern with its contributions (column, alpha, beta);
//   * one 32-bit code per CSR entry of T (lateral entry, row level, level
//     step, Dirichlet zero / diagonal flags);
//   * per dof its rhs records (8 cell + local vertex, ascending cell).
// Anything that does not fit (a partition, a periodic identity, another
// manifold) returns false and the colour kernels stay in use.
#include <algorithm>
#include <array>
#include <cstdint>
#include <map>
#include <numeric>
#include <vector>

#include "context.h"

namespace dcp {

namespace {
int find_root(std::vector<int32_t>& par, int x) {
  while (par[x] != x) {
    par[x] = par[par[x]];
    x = par[x];
  }
  return x;
}
}  // namespace

bool build_tsep(Ctx& c, int n_cells, const std::vector<int32_t>& td,
                const std::vector<int32_t>& col, const std::vector<int32_t>& layer,
                const std::vector<double>& layR, const std::vector<uint8_t>& Tfix,
                const std::vector<double>& Tbc, const std::vector<int32_t>& Tp,
                const std::vector<int32_t>& Tc, int n_T) {
  c.tsep = false;
  c.ts_tmat_valid = false;
  if (n_cells <= 0 || n_T <= 0 || td.size() != size_t(n_cells) * 8 || col.size() != size_t(n_cells) ||
      layer.size() != size_t(n_cells) || layR.empty())
    return false;
  const int n_colids = *std::max_element(col.begin(), col.end()) + 1;
  const int NL = int(layR.size() / 3);
  if (NL < 1 || NL > 254) return false;
  // radial order of the layers
  std::vector<int32_t> ord2lay(NL), lay2ord(NL);
  std::iota(ord2lay.begin(), ord2lay.end(), 0);
  std::stable_sort(ord2lay.begin(), ord2lay.end(),
                   [&](int a, int b) { return layR[3 * size_t(a)] < layR[3 * size_t(b)]; });
  for (int o = 0; o < NL; ++o) lay2ord[ord2lay[o]] = o;
  // lateral vertices: dofs joined along the radial edges of the cells
  std::vector<int32_t> par(n_T);
  std::iota(par.begin(), par.end(), 0);
  for (int cell = 0; cell < n_cells; ++cell)
    for (int al = 0; al < 4; ++al) {
      const int a = find_root(par, td[8 * size_t(cell) + al]);
      const int b = find_root(par, td[8 * size_t(cell) + al + 4]);
      if (a != b) par[std::max(a, b)] = std::min(a, b);
    }
  std::vector<int32_t> lat(n_T), lev(n_T, -1);
  int NV = 0;
  {
    std::vector<int32_t> id(n_T, -1);
    for (int i = 0; i < n_T; ++i) {
      const int r = find_root(par, i);
      if (id[r] < 0) id[r] = NV++;
      lat[i] = id[r];
    }
  }
  for (int cell = 0; cell < n_cells; ++cell)
    for (int a = 0; a < 8; ++a) {
      const int i = td[8 * size_t(cell) + a];
      const int l = lay2ord[layer[cell]] + (a >> 2);
      if (lev[i] >= 0 && lev[i] != l) return false;
      lev[i] = l;
    }
  if (int64_t(NV) * (NL + 1) != n_T) return false;
  {
    std::vector<uint8_t> seen(size_t(NV) * (NL + 1), 0);
    for (int i = 0; i < n_T; ++i) {
      if (lev[i] < 0) return false;
      uint8_t& s = seen[size_t(lat[i]) * (NL + 1) + lev[i]];
      if (s) return false;
      s = 1;
    }
  }
  // lateral columns (sorted lateral vertex quadruple) and the alpha order of each column id
  std::map<std::array<int32_t, 4>, int> colkey;
  std::vector<int32_t> latcol(n_cells);
  std::vector<std::array<int32_t, 4>> id_lat(n_colids, {-1, -1, -1, -1});
  for (int cell = 0; cell < n_cells; ++cell) {
    std::array<int32_t, 4> t;
    for (int al = 0; al < 4; ++al) t[al] = lat[td[8 * size_t(cell) + al]];
    auto& il = id_lat[col[cell]];
    if (il[0] < 0) il = t;
    else if (il != t) return false;
    std::array<int32_t, 4> k = t;
    std::sort(k.begin(), k.end());
    if (k[0] == k[1] || k[1] == k[2] || k[2] == k[3]) return false;
    latcol[cell] = colkey.emplace(k, int(colkey.size())).first->second;
  }
  const int NC = int(colkey.size());
  if (int64_t(NC) * NL != n_cells || NC >= (1 << 27)) return false;
  std::vector<int32_t> grid(size_t(NC) * NL, -1);
  for (int cell = 0; cell < n_cells; ++cell) {
    int32_t& g = grid[size_t(latcol[cell]) * NL + lay2ord[layer[cell]]];
    if (g >= 0) return false;
    g = col[cell];
  }
  // layer kinds: equal column ids in every column
  std::vector<int32_t> kind(NL, -1), rep;
  for (int o = 0; o < NL; ++o) {
    for (size_t k = 0; k < rep.size() && kind[o] < 0; ++k) {
      bool same = true;
      for (int C = 0; C < NC && same; ++C) same = grid[size_t(C) * NL + o] == grid[size_t(C) * NL + rep[k]];
      if (same) kind[o] = int(k);
    }
    if (kind[o] < 0) {
      kind[o] = int(rep.size());
      rep.push_back(o);
    }
  }
  const int NK = int(rep.size());
  std::vector<int32_t> kc(size_t(NC) * NK);
  for (int C = 0; C < NC; ++C)
    for (int k = 0; k < NK; ++k) {
      kc[size_t(C) * NK + k] = grid[size_t(C) * NL + rep[k]];
      if (id_lat[kc[size_t(C) * NK + k]] != id_lat[kc[size_t(C) * NK]]) return false;
    }
  // lateral pattern: (v, v') -> contributions (C, alpha, beta), ascending C
  struct Con {
    int32_t v, w, C, ab;
  };
  std::vector<Con> cons;
  cons.reserve(size_t(NC) * 16);
  for (int C = 0; C < NC; ++C) {
    const auto& t = id_lat[kc[size_t(C) * NK]];
    for (int al = 0; al < 4; ++al)
      for (int be = 0; be < 4; ++be) cons.push_back({t[al], t[be], C, (al << 2) | be});
  }
  std::stable_sort(cons.begin(), cons.end(), [](const Con& a, const Con& b) {
    return a.v != b.v ? a.v < b.v : a.w != b.w ? a.w < b.w : a.C < b.C;
  });
  std::vector<int32_t> lptr(1, 0), lcon, lrow(size_t(NV) + 1, 0), lcolv;
  for (size_t k = 0; k < cons.size(); ++k) {
    if (k > 0 && (cons[k].v != cons[k - 1].v || cons[k].w != cons[k - 1].w)) lptr.push_back(int32_t(k));
    if (k == 0 || cons[k].v != cons[k - 1].v || cons[k].w != cons[k - 1].w) {
      lcolv.push_back(cons[k].w);
      lrow[size_t(cons[k].v) + 1]++;
    }
    lcon.push_back(k);  // filled per kind below
  }
  // contributions as (column id of the kind) << 4 | alpha << 2 | beta, per kind
  {
    const size_t ncon = cons.size();
    lcon.assign(ncon * NK, 0);
    for (int k = 0; k < NK; ++k)
      for (size_t j = 0; j < ncon; ++j)
        lcon[k * ncon + j] = (kc[size_t(cons[j].C) * NK + k] << 4) | cons[j].ab;
  }
  lptr.push_back(int32_t(cons.size()));
  const int NLAT = int(lcolv.size());
  if (NLAT >= (1 << 20)) return false;
  for (int v = 0; v < NV; ++v) lrow[v + 1] += lrow[v];
  // per CSR entry of T its code
  std::vector<uint32_t> code(Tc.size());
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
  for (int i = 0; i < n_T; ++i)
    for (int e = Tp[i]; e < Tp[i + 1]; ++e) {
      const int j = Tc[e];
      const int dl = lev[j] - lev[i] + 1;
      const int32_t* b = lcolv.data() + lrow[lat[i]];
      const int32_t* en = lcolv.data() + lrow[lat[i] + 1];
      const int32_t* f = std::lower_bound(b, en, lat[j]);
      if (dl < 0 || dl > 2 || f == en || *f != lat[j]) {
        ++bad;
        continue;
      }
      const uint32_t p = uint32_t(f - lcolv.data());
      const bool zero = (Tfix[i] || Tfix[j]) && i != j;
      code[e] = p | (uint32_t(lev[i]) << 20) | (uint32_t(dl) << 28) | (zero ? 1u << 30 : 0u) |
                (i == j ? 1u << 31 : 0u);
    }
  if (bad) return false;
  // per block of pt x 256 entries (k_tsep_matrix_lds) the sorted distinct A
  // records (kind n_latnnz + p) of its terms, the entries coded by slot; the
  // larger block when every list fits the 10-bit slots
  auto terms = [&](uint32_t cd, int32_t rec[2]) {
    rec[0] = rec[1] = -1;
    if ((cd >> 30) & 1u) return;
    const int p = int(cd & 0xFFFFFu), l = int((cd >> 20) & 0xFFu), dl = int((cd >> 28) & 3u);
    const int oa = dl == 2 ? l : l - 1;
    if (oa >= 0) rec[0] = kind[oa] * NLAT + p;
    if (dl == 1 && l < NL) rec[1] = kind[l] * NLAT + p;
  };
  const long nnz = long(Tc.size());
  std::vector<uint32_t> rcode;
  std::vector<int32_t> blk_ptr, blk_rec;
  int blk_pt = 0, max_rec = 0;
  for (const int pt : {8, 4}) {
    if (int64_t(NK) * NLAT >= (int64_t(1) << 31)) break;
    const long B = long(pt) * 256, nblk = (nnz + B - 1) / B;
    std::vector<std::vector<int32_t>> lists(static_cast<size_t>(nblk));
    std::vector<uint32_t> rc(code.size());
    int worst = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(max : worst)
    for (long bi = 0; bi < nblk; ++bi) {
      const long e0 = bi * B, e1 = std::min(nnz, e0 + B);
      std::vector<int32_t>& L = lists[size_t(bi)];
      for (long e = e0; e < e1; ++e) {
        int32_t r[2];
        terms(code[e], r);
        for (int t = 0; t < 2; ++t)
          if (r[t] >= 0) L.push_back(r[t]);
      }
      std::sort(L.begin(), L.end());
      L.erase(std::unique(L.begin(), L.end()), L.end());
      if (L.empty()) L.push_back(0);  // every block stages at least one record
      worst = std::max(worst, int(L.size()));
      for (long e = e0; e < e1; ++e) {
        int32_t r[2];
        terms(code[e], r);
        uint32_t sl[2] = {0, 0};
        for (int t = 0; t < 2; ++t)
          if (r[t] >= 0) sl[t] = uint32_t(std::lower_bound(L.begin(), L.end(), r[t]) - L.begin());
        rc[e] = (sl[0] & 1023u) | ((sl[1] & 1023u) << 10) | (code[e] & 0xFFF00000u);
      }
    }
    if (worst > 1023) continue;
    blk_ptr.assign(size_t(nblk) + 1, 0);
    for (long bi = 0; bi < nblk; ++bi) blk_ptr[bi + 1] = blk_ptr[bi] + int32_t(lists[bi].size());
    blk_rec.clear();
    for (const auto& L : lists) blk_rec.insert(blk_rec.end(), L.begin(), L.end());
    rcode.swap(rc);
    blk_pt = pt;
    max_rec = worst;
    break;
  }
  // rhs records per dof, ascending cell
  std::vector<int32_t> sptr(size_t(n_T) + 1, 0), slot(size_t(n_cells) * 8);
  for (int cell = 0; cell < n_cells; ++cell)
    for (int a = 0; a < 8; ++a) sptr[td[8 * size_t(cell) + a] + 1]++;
  for (int i = 0; i < n_T; ++i) sptr[i + 1] += sptr[i];
  {
    std::vector<int32_t> fill(sptr.begin(), sptr.end() - 1);
    for (int cell = 0; cell < n_cells; ++cell)
      for (int a = 0; a < 8; ++a) slot[fill[td[8 * size_t(cell) + a]]++] = 8 * cell + a;
  }
  if (int64_t(n_cells) * 8 >= (int64_t(1) << 31) || n_colids >= (1 << 27)) return false;
  // per cell: bit a = vertex a fixed, bit 8 + a = fixed with a nonzero value (lifted)
  std::vector<uint16_t> cmask(n_cells, 0);
  for (int cell = 0; cell < n_cells; ++cell)
    for (int a = 0; a < 8; ++a) {
      const int i = td[8 * size_t(cell) + a];
      if (Tfix[i]) cmask[cell] |= uint16_t(1u << a);
      if (Tfix[i] && Tbc[i] != 0.0) cmask[cell] |= uint16_t(1u << (8 + a));
    }
  c.ts_n_colids = n_colids;
  c.ts_n_layers = NL;
  c.ts_n_kinds = NK;
  c.ts_n_latnnz = NLAT;
  c.ts_n_con = int(cons.size());
  c.ts_cmask.upload(cmask);
  c.ts_ord2lay.upload(ord2lay);
  c.ts_lay2ord.upload(lay2ord);
  c.ts_kind.upload(kind);
  c.ts_lptr.upload(lptr);
  c.ts_lcon.upload(lcon);
  c.ts_code.upload(code);
  c.ts_blk_pt = blk_pt;
  c.ts_max_rec = max_rec;
  if (blk_pt) {
    c.ts_rcode.upload(rcode);
    c.ts_blk_ptr.upload(blk_ptr);
    c.ts_blk_rec.upload(blk_rec);
  }
  c.ts_sptr.upload(sptr);
  c.ts_slot.upload(slot);
  c.ts_loc.alloc(size_t(n_colids) * 64);
  c.ts_rad.alloc(size_t(NL) * 16);
  c.ts_A.alloc(size_t(NK) * NLAT * 6);
  c.ts_rec.alloc(size_t(n_cells) * 8);
  c.tsep = true;
  tsep_tables(c.tsd(), c.stream);
  return true;
}

}  // namespace dcp
