// Upload-time tables of the Kronecker-form B^T (kernels/bt_kron.hip).
//
// On the one-GPU layered shell the cells are (lateral column) x (radial
// layer), the Q2 velocity nodes (lateral node, level 0..2 NL) and the Q1
// pressure dofs (lateral vertex, level 0..NL), so the assembled (0,1) block of
// nse_matrix (boussinesq_model.tpp:626-637 scattered at :677-687) is a sum of
// Kronecker products of lateral matrices (column factors P summed over the
// columns) and the layer factors Q. This builds, from the cell maps alone:
//   * the radial order of the layers, the lateral node / level of every
//     velocity node and the lateral vertex / level of every pressure dof
//     (radial edges of the cells joined by union-find);
//   * the lateral columns, the column id of every (column, layer kind), the
//     kind of every layer (tsep.cpp's rule);
//   * the lateral (node, vertex) pairs with their contributions (column,
//     a b, i j), per kind as offsets into P;
//   * per block of kBtkBlock consecutive B^T entries (one workgroup of
//     k_btk_entries) the sorted list of the distinct A records (kind, pair)
//     its entries read, and one 32-bit code per entry: the slots of its one or
//     two terms in that list, the node level and the level step;
//   * per block the constrained (no-normal-flux) rows its entries lie in, the
//     entries of such rows carrying the row's local index in the free slot.
// Anything that does not fit returns false and the B^T tasks stay in use.
#include <algorithm>
#include <array>
#include <cstdint>
#include <map>
#include <numeric>
#include <vector>

#include "context.h"

namespace dcp {

namespace {
int root_of(std::vector<int32_t>& par, int x) {
  while (par[x] != x) {
    par[x] = par[par[x]];
    x = par[x];
  }
  return x;
}
void join(std::vector<int32_t>& par, int a, int b) {
  a = root_of(par, a);
  b = root_of(par, b);
  if (a != b) par[std::max(a, b)] = std::min(a, b);
}
// compact ids of the union-find roots
int compact(std::vector<int32_t>& par, std::vector<int32_t>& id_of) {
  const int n = int(par.size());
  std::vector<int32_t> id(n, -1);
  id_of.assign(n, -1);
  int k = 0;
  for (int i = 0; i < n; ++i) {
    const int r = root_of(par, i);
    if (id[r] < 0) id[r] = k++;
    id_of[i] = id[r];
  }
  return k;
}
}  // namespace

bool build_btk(Ctx& c, int n_cells, const std::vector<int32_t>& q2, const std::vector<int32_t>& pd,
               const std::vector<int32_t>& col, const std::vector<int32_t>& layer,
               const std::vector<double>& layR, const std::vector<NodeConstraint>& vc,
               const std::vector<int32_t>& Btp, const std::vector<int32_t>& Btc, int nv, int n_p) {
  c.btk = false;
  if (n_cells <= 0 || q2.size() != size_t(n_cells) * 27 || pd.size() != size_t(n_cells) * 8 ||
      col.size() != size_t(n_cells) || layer.size() != size_t(n_cells) || layR.empty() ||
      int(Btp.size()) != nv + 1 || int(vc.size()) < nv)
    return false;
  const int n_colids = *std::max_element(col.begin(), col.end()) + 1;
  const int NL = int(layR.size() / 3);
  if (NL < 1 || 2 * NL > 255) return false;
  std::vector<int32_t> ord2lay(NL), lay2ord(NL);
  std::iota(ord2lay.begin(), ord2lay.end(), 0);
  std::stable_sort(ord2lay.begin(), ord2lay.end(),
                   [&](int a, int b) { return layR[3 * size_t(a)] < layR[3 * size_t(b)]; });
  for (int o = 0; o < NL; ++o) lay2ord[ord2lay[o]] = o;
  // pressure: lateral vertex / level
  std::vector<int32_t> par(n_p);
  std::iota(par.begin(), par.end(), 0);
  for (int cell = 0; cell < n_cells; ++cell)
    for (int v = 0; v < 4; ++v) join(par, pd[8 * size_t(cell) + v], pd[8 * size_t(cell) + v + 4]);
  std::vector<int32_t> plat, plev(n_p, -1);
  const int NPV = compact(par, plat);
  // velocity: lateral node / level
  par.resize(nv);
  std::iota(par.begin(), par.end(), 0);
  for (int cell = 0; cell < n_cells; ++cell)
    for (int ab = 0; ab < 9; ++ab) {
      join(par, q2[27 * size_t(cell) + ab], q2[27 * size_t(cell) + ab + 9]);
      join(par, q2[27 * size_t(cell) + ab + 9], q2[27 * size_t(cell) + ab + 18]);
    }
  std::vector<int32_t> vlat, vlev(nv, -1);
  const int NVL = compact(par, vlat);
  for (int cell = 0; cell < n_cells; ++cell) {
    const int L = lay2ord[layer[cell]];
    for (int v = 0; v < 8; ++v) {
      int32_t& l = plev[pd[8 * size_t(cell) + v]];
      if (l >= 0 && l != L + (v >> 2)) return false;
      l = L + (v >> 2);
    }
    for (int t = 0; t < 27; ++t) {
      int32_t& l = vlev[q2[27 * size_t(cell) + t]];
      if (l >= 0 && l != 2 * L + t / 9) return false;
      l = 2 * L + t / 9;
    }
  }
  if (int64_t(NPV) * (NL + 1) != n_p || int64_t(NVL) * (2 * NL + 1) != nv) return false;
  for (int i = 0; i < n_p; ++i)
    if (plev[i] < 0) return false;
  for (int i = 0; i < nv; ++i)
    if (vlev[i] < 0) return false;
  // lateral columns and the lateral node / vertex tuples of every column id
  std::map<std::array<int32_t, 4>, int> colkey;
  std::vector<int32_t> latcol(n_cells);
  std::vector<std::array<int32_t, 13>> id_tuple(n_colids);
  std::vector<uint8_t> id_seen(n_colids, 0);
  for (int cell = 0; cell < n_cells; ++cell) {
    std::array<int32_t, 13> t;
    for (int ab = 0; ab < 9; ++ab) t[ab] = vlat[q2[27 * size_t(cell) + ab]];
    for (int v = 0; v < 4; ++v) t[9 + v] = plat[pd[8 * size_t(cell) + v]];
    if (!id_seen[col[cell]]) {
      id_tuple[col[cell]] = t;
      id_seen[col[cell]] = 1;
    } else if (id_tuple[col[cell]] != t) {
      return false;
    }
    std::array<int32_t, 4> k = {t[9], t[10], t[11], t[12]};
    std::sort(k.begin(), k.end());
    if (k[0] == k[1] || k[1] == k[2] || k[2] == k[3]) return false;
    latcol[cell] = colkey.emplace(k, int(colkey.size())).first->second;
  }
  const int NC = int(colkey.size());
  if (int64_t(NC) * NL != n_cells) return false;
  std::vector<int32_t> grid(size_t(NC) * NL, -1);
  for (int cell = 0; cell < n_cells; ++cell) {
    int32_t& g = grid[size_t(latcol[cell]) * NL + lay2ord[layer[cell]]];
    if (g >= 0) return false;
    g = col[cell];
  }
  std::vector<int32_t> kind(NL, -1), rep;
  for (int o = 0; o < NL; ++o) {
    for (size_t k = 0; k < rep.size() && kind[o] < 0; ++k) {
      bool same = true;
      for (int C = 0; C < NC && same; ++C)
        same = grid[size_t(C) * NL + o] == grid[size_t(C) * NL + rep[k]];
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
      if (id_tuple[kc[size_t(C) * NK + k]] != id_tuple[kc[size_t(C) * NK]]) return false;
    }
  // lateral (node, vertex) pairs and their contributions, ascending column
  struct Con {
    int32_t nu, v, C, abij;
  };
  std::vector<Con> cons;
  cons.reserve(size_t(NC) * 36);
  for (int C = 0; C < NC; ++C) {
    const auto& t = id_tuple[kc[size_t(C) * NK]];
    for (int ab = 0; ab < 9; ++ab)
      for (int ij = 0; ij < 4; ++ij) cons.push_back({t[ab], t[9 + ij], C, ab << 2 | ij});
  }
  std::stable_sort(cons.begin(), cons.end(), [](const Con& a, const Con& b) {
    return a.nu != b.nu ? a.nu < b.nu : a.v != b.v ? a.v < b.v : a.C < b.C;
  });
  std::vector<int32_t> lptr(1, 0), lrow(size_t(NVL) + 1, 0), lcolv;
  for (size_t k = 0; k < cons.size(); ++k) {
    const bool fresh = k == 0 || cons[k].nu != cons[k - 1].nu || cons[k].v != cons[k - 1].v;
    if (fresh && k > 0) lptr.push_back(int32_t(k));
    if (fresh) {
      lcolv.push_back(cons[k].v);
      lrow[size_t(cons[k].nu) + 1]++;
    }
  }
  lptr.push_back(int32_t(cons.size()));
  const int NPAIR = int(lcolv.size());
  if (NPAIR >= (1 << 20)) return false;
  for (int i = 0; i < NVL; ++i) lrow[i + 1] += lrow[i];
  // per kind: offset of the contribution's P entry (colid 216 + a 36 + b 12 + i 6 + j 3)
  const size_t ncon = cons.size();
  std::vector<int32_t> lcon(ncon * NK);
  for (int k = 0; k < NK; ++k)
    for (size_t j = 0; j < ncon; ++j) {
      const int ab = cons[j].abij >> 2, ij = cons[j].abij & 3;
      const int a = ab % 3, b = ab / 3, i = ij & 1, jj = ij >> 1;
      lcon[k * ncon + j] = kc[size_t(cons[j].C) * NK + k] * 216 + 36 * a + 12 * b + 6 * i + 3 * jj;
    }
  if (int64_t(n_colids) * 216 >= (int64_t(1) << 31)) return false;
  // per B^T entry its code; the entries of constrained rows
  std::vector<uint32_t> code(Btc.size());
  int bad = 0;
#pragma omp parallel for schedule(static) reduction(+ : bad)
  for (int n = 0; n < nv; ++n)
    for (int e = Btp[n]; e < Btp[n + 1]; ++e) {
      const int p = Btc[e];
      const int lam = vlev[n], l = plev[p], dl = l - (lam >> 1) + 1;
      const int32_t* b = lcolv.data() + lrow[vlat[n]];
      const int32_t* en = lcolv.data() + lrow[vlat[n] + 1];
      const int32_t* f = std::lower_bound(b, en, plat[p]);
      const bool ok_level = (lam & 1) ? (dl == 1 || dl == 2) : (dl >= 0 && dl <= 2);
      if (!ok_level || f == en || *f != plat[p]) {
        ++bad;
        continue;
      }
      code[e] = uint32_t(f - lcolv.data()) | (uint32_t(lam) << 20) | (uint32_t(dl) << 28) |
                (vc[n].type != 0 ? 1u << 30 : 0u);
    }
  if (bad) return false;
  // the row of every entry of a constrained row (-1 elsewhere)
  std::vector<int32_t> erow(Btc.size(), -1);
  long n_conent = 0;
  for (int n = 0; n < nv; ++n)
    if (vc[n].type != 0)
      for (int e = Btp[n]; e < Btp[n + 1]; ++e) {
        erow[size_t(e)] = n;
        ++n_conent;
      }
  // the records of an entry's terms, in the order of btk_terms (bt_kron.hip)
  auto terms = [&](uint32_t cd, int32_t rec[2]) {
    const int p = int(cd & 0xFFFFFu), lam = int((cd >> 20) & 0xFFu), dl = int((cd >> 28) & 3u);
    const int m = lam >> 1;
    int L0 = -1, L1 = -1;
    if (lam & 1)
      L0 = m;
    else if (dl == 0)
      L0 = m >= 1 ? m - 1 : -1;
    else if (dl == 2)
      L0 = m;
    else {
      L0 = m >= 1 ? m - 1 : -1;
      L1 = m < NL ? m : -1;
    }
    rec[0] = L0 >= 0 && L0 < NL ? kind[L0] * NPAIR + p : -1;
    rec[1] = L1 >= 0 ? kind[L1] * NPAIR + p : -1;
  };
  const long nnz = long(Btc.size());
  const long nblk = (nnz + kBtkBlock - 1) / kBtkBlock;
  if (int64_t(NK) * NPAIR >= (int64_t(1) << 31) || nblk >= (1L << 31)) return false;
  std::vector<std::vector<int32_t>> blk_list(nblk), blk_cons(nblk);
  int worst = 0, worst_con = 0, bad_con = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(max : worst, worst_con) reduction(+ : bad_con)
  for (long bi = 0; bi < nblk; ++bi) {
    const long e0 = bi * kBtkBlock, e1 = std::min(nnz, e0 + kBtkBlock);
    std::vector<int32_t>& L = blk_list[bi];
    // the block's constrained rows (their NodeConstraints staged beside the
    // records); an entry of such a row carries its local index in the slot
    // field its terms leave free (one of the two on the shell's boundary levels)
    std::vector<int32_t>& CR = blk_cons[bi];
    for (long e = e0; e < e1; ++e)
      if (erow[size_t(e)] >= 0) CR.push_back(erow[size_t(e)]);
    std::sort(CR.begin(), CR.end());
    CR.erase(std::unique(CR.begin(), CR.end()), CR.end());
    worst_con = std::max(worst_con, int(CR.size()));
    for (long e = e0; e < e1; ++e) {
      int32_t r[2];
      terms(code[e], r);
      for (int t = 0; t < 2; ++t)
        if (r[t] >= 0) L.push_back(r[t]);
    }
    std::sort(L.begin(), L.end());
    L.erase(std::unique(L.begin(), L.end()), L.end());
    worst = std::max(worst, int(L.size()));
    for (long e = e0; e < e1; ++e) {
      int32_t r[2];
      terms(code[e], r);
      uint32_t slot[2] = {0, 0};
      for (int t = 0; t < 2; ++t)
        if (r[t] >= 0) slot[t] = uint32_t(std::lower_bound(L.begin(), L.end(), r[t]) - L.begin());
      if (erow[size_t(e)] >= 0) {
        const int free_t = r[0] < 0 ? 0 : (r[1] < 0 ? 1 : -1);
        if (free_t < 0) {
          ++bad_con;
        } else {
          slot[free_t] = uint32_t(std::lower_bound(CR.begin(), CR.end(), erow[size_t(e)]) - CR.begin());
        }
      }
      code[e] = (slot[0] & 1023u) | ((slot[1] & 1023u) << 10) | (code[e] & 0x7FF00000u);
    }
  }
  if (worst > kBtkMaxRec || worst_con > 1023 || bad_con) return false;
  std::vector<int32_t> blk_cptr(size_t(nblk) + 1, 0), blk_crow;
  for (long bi = 0; bi < nblk; ++bi) blk_cptr[bi + 1] = blk_cptr[bi] + int32_t(blk_cons[bi].size());
  blk_crow.reserve(size_t(blk_cptr[nblk]));
  for (long bi = 0; bi < nblk; ++bi) blk_crow.insert(blk_crow.end(), blk_cons[bi].begin(), blk_cons[bi].end());
  if (blk_crow.empty()) blk_crow.push_back(0);
  std::vector<int32_t> blk_ptr(size_t(nblk) + 1, 0), blk_rec;
  for (long bi = 0; bi < nblk; ++bi) blk_ptr[bi + 1] = blk_ptr[bi] + int32_t(blk_list[bi].size());
  blk_rec.reserve(size_t(blk_ptr[nblk]));
  for (long bi = 0; bi < nblk; ++bi) blk_rec.insert(blk_rec.end(), blk_list[bi].begin(), blk_list[bi].end());
  c.btk_n_layers = NL;
  c.btk_n_kinds = NK;
  c.btk_n_pairs = NPAIR;
  c.btk_n_con = int(ncon);
  c.btk_n_conent = int(n_conent);
  c.btk_ord2lay.upload(ord2lay);
  c.btk_kind.upload(kind);
  c.btk_lptr.upload(lptr);
  c.btk_lcon.upload(lcon);
  c.btk_code.upload(code);
  c.btk_blk_ptr.upload(blk_ptr);
  c.btk_blk_rec.upload(blk_rec);
  c.btk_max_rec = worst;
  c.btk_blk_cptr.upload(blk_cptr);
  c.btk_blk_crow.upload(blk_crow);
  c.btk_max_con = worst_con;
  c.btk_A.alloc(size_t(NK) * NPAIR * 6);
  c.btk = true;
  return true;
}

}  // namespace dcp
