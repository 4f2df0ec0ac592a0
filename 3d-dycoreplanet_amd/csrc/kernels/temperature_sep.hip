// Temperature system on a radially separable mesh (the hyper_shell), FP64.
//
// Replaces, for the classic model's FE_Q(1) temperature, the colour launches
// of k_T_matrix / k_T_rhs (assembly.hip) that stand for the reference's
//   local_assemble_temperature_matrix + copy      boussinesq_model.tpp:748-817
//   assemble_temperature_rhs: T_matrix = M + dt K, Jacobi           :966-986
//   local_assemble_temperature_rhs + copy (matrix_for_bc lift)      :873-964
//
// On the shell every cell is (column of the cubed sphere) x (radial layer),
// X = R(zeta) Phi(xi, eta) (api.cpp separable_geometry), so J^-1 rows are
// m_e / R (e = 0, 1) and m_2 / R', JxW = R^2 R' D2 w. With the Q1 shape
// phi_a = psi_alpha(xi, eta) chi_rho(zeta) every term of the element mass and
// stiffness matrices splits into a lateral integral (9 points, per column)
// times a radial one (3 points, per layer):
//   M_ab = LM[al][be] RM[ro][so]
//   K_ab / (1/Pe) = Lll[al][be] Rll[ro][so] + Lx[al][be] Rx[ro][so]
//                 + Lx[be][al] Rx[so][ro] + L22[al][be] R22[ro][so]
//   LM  = sum psi psi D2 w,   Lll = sum_{e,f<2} d_e psi d_f psi (m_e.m_f) D2 w,
//   Lx  = sum_{e<2} d_e psi psi (m_e.m_2) D2 w,   L22 = sum psi psi (m_2.m_2) D2 w,
//   RM  = sum chi chi R^2 R' w,  Rll = sum chi chi R' w,  Rx = sum chi chi' R w,
//   R22 = sum chi' chi' R^2 / R' w.
// And since the cells are the full product of columns and layers, the
// assembled matrices are sums of Kronecker products: entry ((v, l), (v', l'))
// = sum over the (one or two) layers holding levels l and l' of
// A_t^{kind(layer)}(v, v') x R_t,layer, where A_t^kind is the lateral matrix
// assembled over the columns (kind: the mapping of the layer, MappingQ(3) on
// the boundary layers, MappingQ1 inside, deal.II 9.2). So one assembly is
//   k_tsep_local   the 4 lateral 4x4 tables per column id, the 4 radial 2x2
//                  tables per layer: integrals of the mesh geometry alone,
//                  formed once at upload (as k_bt_coltab / k_bt_laytab form
//                  the B^T column and layer factors); then per assembly
//   k_tsep_lateral the lateral matrices A_t^kind (tiny: 2 x 55 k entries at r=5),
//   k_tsep_matrix  one thread per CSR entry of T: M, K, T_matrix = M + dt K
//                  and the Jacobi inverse at the diagonal, written once each
//                  (Dirichlet rows / columns as the AffineConstraints copy:
//                  an off-diagonal entry with a fixed row or column is 0, the
//                  diagonal of a fixed row the sum of |local diagonals| = the
//                  assembled diagonal, every local diagonal being positive).
// The rhs (advection of T by the Q2 velocity is not separable) runs in cell
// order, eight cells per workgroup, geometry from the same tables, into one
// record of 8 values per cell (the matrix_for_bc lift from the local tables),
// then k_tsep_gather sums each dof's records in ascending cell order: no
// colours, no atomics, deterministic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "../device.h"
#include "../fe_tables.h"

namespace dcp {
namespace {

constexpr int kTB = 256;

// Gauss point / weight / 1D bases by arithmetic: a lane-dependent index into a
// __constant__ table is a vector memory load per use, a select is not.
__device__ __forceinline__ double gx(int q) {
  return q == 0 ? kGaussX[0] : (q == 1 ? kGaussX[1] : kGaussX[2]);
}
__device__ __forceinline__ double gw(int q) { return q == 1 ? kGaussW[1] : kGaussW[0]; }
__device__ __forceinline__ double l1(int v, double x) { return v ? x : 1.0 - x; }
__device__ __forceinline__ double d1(int v) { return v ? 1.0 : -1.0; }
__device__ __forceinline__ void l2(double x, double* p) {
  p[0] = 2 * (x - 0.5) * (x - 1);
  p[1] = -4 * x * (x - 1);
  p[2] = 2 * x * (x - 0.5);
}

// Lateral tables of one column id (16 threads per column id, one per (alpha,
// beta)): loc[64 id + 16 t + 4 alpha + beta], t = LM, Lll, Lx, L22. Radial
// tables of ordinal layer o (threads after the columns):
// rad[16 o + 4 t + 2 rho + sigma], t = RM, Rll, Rx, R22.
__global__ __launch_bounds__(kTB) void k_tsep_local(TSepDev t) {
  const int gid = int(blockIdx.x) * kTB + int(threadIdx.x);
  if (gid < 16 * t.n_colids) {
    const int id = gid >> 4, al = (gid >> 2) & 3, be = gid & 3;
    const int va = al & 1, vb = al >> 1, wa = be & 1, wb = be >> 1;
    const double* g0 = t.colgeo + 90 * size_t(id);
    double LM = 0, Lll = 0, Lx = 0, L22 = 0;
#pragma unroll
    for (int q1 = 0; q1 < 3; ++q1)
#pragma unroll
      for (int q0 = 0; q0 < 3; ++q0) {
        const double* g = g0 + 10 * (q0 + 3 * q1);
        const double x0 = gx(q0), x1 = gx(q1);
        const double W = g[9] * gw(q0) * gw(q1);
        const double d00 = g[0] * g[0] + g[1] * g[1] + g[2] * g[2];
        const double d01 = g[0] * g[3] + g[1] * g[4] + g[2] * g[5];
        const double d11 = g[3] * g[3] + g[4] * g[4] + g[5] * g[5];
        const double d02 = g[0] * g[6] + g[1] * g[7] + g[2] * g[8];
        const double d12 = g[3] * g[6] + g[4] * g[7] + g[5] * g[8];
        const double d22 = g[6] * g[6] + g[7] * g[7] + g[8] * g[8];
        const double pa = l1(va, x0) * l1(vb, x1);
        const double a0 = d1(va) * l1(vb, x1), a1 = l1(va, x0) * d1(vb);
        const double pb = l1(wa, x0) * l1(wb, x1);
        const double b0 = d1(wa) * l1(wb, x1), b1 = l1(wa, x0) * d1(wb);
        LM += pa * pb * W;
        Lll += (a0 * b0 * d00 + a0 * b1 * d01 + a1 * b0 * d01 + a1 * b1 * d11) * W;
        Lx += (a0 * d02 + a1 * d12) * pb * W;
        L22 += pa * pb * d22 * W;
      }
    double* o = t.loc + 64 * size_t(id) + 4 * al + be;
    o[0] = LM;
    o[16] = Lll;
    o[32] = Lx;
    o[48] = L22;
    return;
  }
  const int o = gid - 16 * t.n_colids;
  if (o >= t.n_layers) return;
  const int lid = t.ord2lay[o];
  double r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = 0.0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double* lg = t.laygeo + 9 * size_t(lid) + 3 * q;
    const double R = t.layR[3 * size_t(lid) + q], Rp = 1.0 / lg[1], R2Rp = lg[2];
    const double w = gw(q), x = gx(q);
#pragma unroll
    for (int ro = 0; ro < 2; ++ro)
#pragma unroll
      for (int so = 0; so < 2; ++so) {
        const double cc = l1(ro, x) * l1(so, x);
        r[2 * ro + so] += cc * R2Rp * w;
        r[4 + 2 * ro + so] += cc * Rp * w;
        r[8 + 2 * ro + so] += l1(ro, x) * d1(so) * R * w;
        r[12 + 2 * ro + so] += d1(ro) * d1(so) * (R * R / Rp) * w;
      }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) t.rad[16 * size_t(o) + i] = r[i];
}

// A[(kind n_latnnz + p) 6 + t], t = M, ll, x, x^T, 22 (6: pad): the column
// sums of the lateral tables in the contribution order of the upload
// (ascending column).
__global__ __launch_bounds__(kTB) void k_tsep_lateral(TSepDev t) {
  const int gid = int(blockIdx.x) * kTB + int(threadIdx.x);
  if (gid >= t.n_kinds * t.n_latnnz) return;
  const int k = gid / t.n_latnnz, p = gid - k * t.n_latnnz;
  const int32_t* con = t.lcon + size_t(k) * t.n_con;
  double s[5] = {0, 0, 0, 0, 0};
  for (int j = t.lptr[p]; j < t.lptr[p + 1]; ++j) {
    const int c = con[j];
    const int al = (c >> 2) & 3, be = c & 3;
    const double* L = t.loc + 64 * size_t(c >> 4);
    s[0] += L[4 * al + be];
    s[1] += L[16 + 4 * al + be];
    s[2] += L[32 + 4 * al + be];
    s[3] += L[32 + 4 * be + al];
    s[4] += L[48 + 4 * al + be];
  }
  double* a = t.A + 6 * size_t(gid);
#pragma unroll
  for (int i = 0; i < 5; ++i) a[i] = s[i];
  a[5] = 0.0;
}

// code: bits 0-19 lateral entry p, 20-27 row level l, 28-29 l' - l + 1,
// 30 "zero" (off-diagonal entry of a fixed row or column), 31 diagonal.
// kPerThread entries per thread, kTB apart (every load and store coalesced,
// independent chains in flight); the radial tables and layer kinds in LDS.
template <int kPerThread>
__global__ __launch_bounds__(kTB) void k_tsep_matrix(TSepDev t, long nnz, double one_over_pe,
                                                     double dt_T, double* __restrict__ M,
                                                     double* __restrict__ K,
                                                     double* __restrict__ Tmat,
                                                     double* __restrict__ Tinv) {
  extern __shared__ __attribute__((aligned(16))) double srad[];
  int* skind = reinterpret_cast<int*>(srad + 16 * t.n_layers);
  for (int i = threadIdx.x; i < 16 * t.n_layers; i += kTB) srad[i] = t.rad[i];
  for (int i = threadIdx.x; i < t.n_layers; i += kTB) skind[i] = t.kind[i];
  // each XCD one contiguous range of entries: the lateral rows its entries
  // read stay in its own L2 (A is 5.3 MB at r=5, more than one XCD's 4 MB)
  const long base = long(xcd_block(int(blockIdx.x), int(gridDim.x))) * (kPerThread * kTB) +
                    threadIdx.x;
  uint32_t code[kPerThread];
#pragma unroll
  for (int u = 0; u < kPerThread; ++u) {
    const long e = base + long(u) * kTB;
    code[u] = e < nnz ? __builtin_nontemporal_load(t.code + e) : (1u << 30);
  }
  __syncthreads();
  double m[kPerThread], k[kPerThread];
#pragma unroll
  for (int u = 0; u < kPerThread; ++u) {
    m[u] = k[u] = 0.0;
    const uint32_t c = code[u];
    if ((c >> 30) & 1u) continue;
    if (t.probe & 1) {  // probe: no lateral / radial reads
      m[u] = double(c);
      continue;
    }
    const int p = int(c & 0xFFFFFu), l = int((c >> 20) & 0xFFu), dl = int((c >> 28) & 3u);
    // the (one or two) layers: ordinal and radial index 2 rho + sigma
    const int oa = dl == 2 ? l : l - 1;
    const int ra = dl == 2 ? 1 : (dl == 0 ? 2 : 3);
    const bool has_a = oa >= 0;
    const bool has_b = dl == 1 && l < t.n_layers;
    double mm = 0.0, kk = 0.0;
    if (has_a) {
      const double2* a2 = reinterpret_cast<const double2*>(
          t.A + 6 * (size_t(skind[oa]) * t.n_latnnz + p));
      const double2 A0 = a2[0], A1 = a2[1], A2 = a2[2];
      const double* r = srad + 16 * oa;
      const int rt = ((ra & 1) << 1) | (ra >> 1);
      mm += A0.x * r[ra];
      kk += A0.y * r[4 + ra] + A1.x * r[8 + ra] + A1.y * r[8 + rt] + A2.x * r[12 + ra];
    }
    if (has_b) {
      const double2* a2 = reinterpret_cast<const double2*>(
          t.A + 6 * (size_t(skind[l]) * t.n_latnnz + p));
      const double2 A0 = a2[0], A1 = a2[1], A2 = a2[2];
      const double* r = srad + 16 * l;
      mm += A0.x * r[0];
      kk += A0.y * r[4] + A1.x * r[8] + A1.y * r[8] + A2.x * r[12];
    }
    m[u] = mm;
    k[u] = kk * one_over_pe;
  }
#pragma unroll
  for (int u = 0; u < kPerThread; ++u) {
    const long e = base + long(u) * kTB;
    if (e >= nnz) break;
    const double tm = m[u] + dt_T * k[u];
    if (t.probe & 4) {  // probe: plain stores
      if (!(t.probe & 2)) {
        M[e] = m[u];
        K[e] = k[u];
      }
      Tmat[e] = tm;
    } else {
      if (!(t.probe & 2)) {  // probe 2: T_matrix only
        __builtin_nontemporal_store(m[u], M + e);
        __builtin_nontemporal_store(k[u], K + e);
      }
      __builtin_nontemporal_store(tm, Tmat + e);
    }
    if (code[u] >> 31) Tinv[t.T_col[e]] = 1.0 / tm;
  }
}

// The same entries from per-block records (tsep.cpp): the block's distinct A
// records staged into LDS with coalesced loads (the per-entry A loads above
// are 3 scattered 16-byte reads per term, bound by the vector memory pipe's
// line rate, as k_btk_entries was), then both terms of every entry from LDS,
// branch-free: an absent term (or a zero entry) with radial factors 0, which
// leaves mm / kk bitwise as without it (x + A 0 = x).
template <int PT>
__global__ __launch_bounds__(kTB) void k_tsep_matrix_lds(TSepDev t, long nnz, double one_over_pe,
                                                         double dt_T, double* __restrict__ M,
                                                         double* __restrict__ K,
                                                         double* __restrict__ Tmat,
                                                         double* __restrict__ Tinv) {
  extern __shared__ __attribute__((aligned(16))) double srad[];
  double2* srec = reinterpret_cast<double2*>(srad + 16 * t.n_layers);
  const int blk = xcd_block(int(blockIdx.x), int(gridDim.x));
  const long base = long(blk) * (PT * kTB) + threadIdx.x;
  const int r0 = t.blk_ptr[blk], nr = t.blk_ptr[blk + 1] - r0;  // nr >= 1
  constexpr int kU = 4;  // 4 kTB double2 = 341 records without the loop below
  int rid[kU];
#pragma unroll
  for (int q = 0; q < kU; ++q) rid[q] = t.blk_rec[r0 + min((int(threadIdx.x) + q * kTB) / 3, nr - 1)];
  uint32_t code[PT];
#pragma unroll
  for (int u = 0; u < PT; ++u)
    code[u] = __builtin_nontemporal_load(t.rcode + min(base + long(u) * kTB, nnz - 1));
  const double2* A2 = reinterpret_cast<const double2*>(t.A);
  double2 ra[kU];
#pragma unroll
  for (int q = 0; q < kU; ++q) {
    const int i = int(threadIdx.x) + q * kTB;
    ra[q] = A2[3 * size_t(rid[q]) + (i - 3 * (i / 3))];
  }
#pragma unroll
  for (int q = 0; q < kU; ++q) {
    const int i = int(threadIdx.x) + q * kTB;
    if (i < 3 * nr) srec[i] = ra[q];
  }
  for (int i = threadIdx.x + kU * kTB; i < 3 * nr; i += kTB) {
    const int j = i / 3;
    srec[i] = A2[3 * size_t(t.blk_rec[r0 + j]) + (i - 3 * j)];
  }
  for (int i = threadIdx.x; i < 16 * t.n_layers; i += kTB) srad[i] = t.rad[i];
  __syncthreads();
#pragma unroll
  for (int u = 0; u < PT; ++u) {
    const long e = base + long(u) * kTB;
    const uint32_t c = code[u];
    const int sa = int(c & 1023u), sb = int((c >> 10) & 1023u);
    const int l = int((c >> 20) & 0xFFu), dl = int((c >> 28) & 3u);
    const bool zero = (c >> 30) & 1u;
    const int oa = dl == 2 ? l : l - 1;
    const int ra_ = dl == 2 ? 1 : (dl == 0 ? 2 : 3);
    const int rt = ((ra_ & 1) << 1) | (ra_ >> 1);
    const bool has_a = !zero && oa >= 0;
    const bool has_b = !zero && dl == 1 && l < t.n_layers;
    const double* qa = srad + 16 * (oa >= 0 ? oa : 0);
    const double* qb = srad + 16 * (l < t.n_layers ? l : 0);
    const double fa0 = has_a ? qa[ra_] : 0.0, fa1 = has_a ? qa[4 + ra_] : 0.0;
    const double fa2 = has_a ? qa[8 + ra_] : 0.0, fa3 = has_a ? qa[8 + rt] : 0.0;
    const double fa4 = has_a ? qa[12 + ra_] : 0.0;
    const double fb0 = has_b ? qb[0] : 0.0, fb1 = has_b ? qb[4] : 0.0;
    const double fb2 = has_b ? qb[8] : 0.0, fb4 = has_b ? qb[12] : 0.0;
    const double2 A0 = srec[3 * sa], A1 = srec[3 * sa + 1], A2v = srec[3 * sa + 2];
    const double2 B0 = srec[3 * sb], B1 = srec[3 * sb + 1], B2 = srec[3 * sb + 2];
    double mm = 0.0, kk = 0.0;
    mm += A0.x * fa0;
    kk += A0.y * fa1 + A1.x * fa2 + A1.y * fa3 + A2v.x * fa4;
    mm += B0.x * fb0;
    kk += B0.y * fb1 + B1.x * fb2 + B1.y * fb2 + B2.x * fb4;
    const double m = mm, k = kk * one_over_pe;
    if (e < nnz) {
      const double tm = m + dt_T * k;
      __builtin_nontemporal_store(m, M + e);
      __builtin_nontemporal_store(k, K + e);
      __builtin_nontemporal_store(tm, Tmat + e);
      if (c >> 31) Tinv[t.T_col[e]] = 1.0 / tm;
    }
  }
}

// wave-level LDS hand-off (the two cells of a wave never leave it)
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Records of the temperature rhs, 8 cells per workgroup, two per wave (lanes
// 0-26 and 32-58): f_a = sum_q phi_a (T w - dt u.grad T w) for the free rows
// a, minus the lift sum_{b fixed, g_b != 0} g_b (M + dt K)_ab
// (boussinesq_model.tpp:922-949); 0 for fixed rows. The Q2 velocity at the 27
// points and the Q1 test sums both by sum factorisation over the cell's lanes
// (one 1D direction per step, LDS between steps): 9 + 9 instead of 81 products
// per point, and 6 + 6 + 6 instead of 27 per test function. (A persistent
// form, each wave a run of cells with the next cells' loads issued ahead,
// measured slower: 124 against 102 us per rhs at r=5; the loop-carried
// prefetch registers (220 VGPRs) cost the occupancy and the register copies
// at the back edge wait for the prefetched loads.)
__global__ __launch_bounds__(kTB) void k_tsep_rhs_cells(TSepDev t, CellData cd,
                                                        const double* __restrict__ T_old,
                                                        const double* __restrict__ u,
                                                        double one_over_pe, double dt_T) {
  __shared__ double U[8][81];   // velocity nodes, then the second interpolation step
  __shared__ double V[8][81];   // first interpolation step, then the test-sum steps
  __shared__ double S[8][28];   // integrand at the 27 points
  __shared__ double Tn[8][8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lc = 2 * wave + (lane >> 5), i = lane & 31;
  // each XCD one contiguous range of cells: shared velocity nodes meet in its L2
  const int cell = 8 * xcd_block(int(blockIdx.x), int(gridDim.x)) + lc;
  const bool live = cell < cd.n_cells;
  const bool qlane = live && i < 27;
  const bool vel = !(t.probe & 8);
  const int i0 = i % 3, i1 = (i / 3) % 3, i2 = i / 9;  // this lane's (q0|a, q1|b, q2|c)
  if (qlane && vel) {
    const int n = cd.cell_q2[27 * size_t(cell) + i];
    const double u0 = u[3 * size_t(n)], u1 = u[3 * size_t(n) + 1], u2 = u[3 * size_t(n) + 2];
    U[lc][3 * i] = u0;
    U[lc][3 * i + 1] = u1;
    U[lc][3 * i + 2] = u2;
  }
  unsigned mask = 0;
  if (live && i < 8) {
    Tn[lc][i] = T_old[cd.cell_T[8 * size_t(cell) + i]];
    mask = t.cmask[cell];
  }
  double geo[10], iR = 0, iRp = 0, R2Rp = 0;
  if (qlane) {
    const double* g = t.colgeo + 90 * size_t(cd.sep_col[cell]) + 10 * (i0 + 3 * i1);
#pragma unroll
    for (int k = 0; k < 10; ++k) geo[k] = g[k];
    const double* lg = t.laygeo + 9 * size_t(cd.sep_layer[cell]) + 3 * i2;
    iR = lg[0];
    iRp = lg[1];
    R2Rp = lg[2];
  }
  wsync();
  double p[3];
  // step 1: (q0, b, c) = sum_a L_a(q0) U(a, b, c)
  if (qlane && vel) {
    l2(gx(i0), p);
    double s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      const int n = a + 3 * i1 + 9 * i2;
      s0 += p[a] * U[lc][3 * n];
      s1 += p[a] * U[lc][3 * n + 1];
      s2 += p[a] * U[lc][3 * n + 2];
    }
    V[lc][3 * i] = s0;
    V[lc][3 * i + 1] = s1;
    V[lc][3 * i + 2] = s2;
  }
  wsync();
  // step 2: (q0, q1, c) = sum_b L_b(q1) V(q0, b, c), into U (step 1 read it all)
  if (qlane && vel) {
    l2(gx(i1), p);
    double s0 = 0, s1 = 0, s2 = 0;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const int n = i0 + 3 * b + 9 * i2;
      s0 += p[b] * V[lc][3 * n];
      s1 += p[b] * V[lc][3 * n + 1];
      s2 += p[b] * V[lc][3 * n + 2];
    }
    U[lc][3 * i] = s0;
    U[lc][3 * i + 1] = s1;
    U[lc][3 * i + 2] = s2;
  }
  wsync();
  // step 3: u(q0, q1, q2) = sum_c L_c(q2) U(q0, q1, c), then the integrand
  if (qlane) {
    double uq[3] = {0, 0, 0};
    if (vel) {
      l2(gx(i2), p);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int n = i0 + 3 * i1 + 9 * c;
        uq[0] += p[c] * U[lc][3 * n];
        uq[1] += p[c] * U[lc][3 * n + 1];
        uq[2] += p[c] * U[lc][3 * n + 2];
      }
    }
    const double x0 = gx(i0), x1 = gx(i1), x2 = gx(i2);
    double T = 0, r0 = 0, r1 = 0, r2 = 0;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int ka = v & 1, kb = (v >> 1) & 1, kc = v >> 2;
      const double la = l1(ka, x0), lb = l1(kb, x1), lc3 = l1(kc, x2);
      const double tv = Tn[lc][v];
      T += tv * (la * lb * lc3);
      r0 += tv * (d1(ka) * lb * lc3);
      r1 += tv * (la * d1(kb) * lc3);
      r2 += tv * (la * lb * d1(kc));
    }
    double gT[3];
#pragma unroll
    for (int d = 0; d < 3; ++d)
      gT[d] = r0 * (geo[d] * iR) + r1 * (geo[3 + d] * iR) + r2 * (geo[6 + d] * iRp);
    const double w = R2Rp * geo[9] * (gw(i0) * gw(i1) * gw(i2));
    S[lc][i] = T * w - dt_T * (uq[0] * gT[0] + uq[1] * gT[1] + uq[2] * gT[2]) * w;
  }
  wsync();
  // test sums f_a = sum_q phi_a(q) S(q), one direction per step (V reused):
  // (ka, q1, q2) -> (ka, kb, q2) -> (ka, kb, kc)
  if (live && i < 18 && !(t.probe & 32)) {
    const int ka = i & 1, r = i >> 1;  // r = q1 + 3 q2
    V[lc][i] = l1(ka, gx(0)) * S[lc][3 * r] + l1(ka, gx(1)) * S[lc][3 * r + 1] +
               l1(ka, gx(2)) * S[lc][3 * r + 2];
  }
  wsync();
  if (live && i < 12 && !(t.probe & 32)) {
    const int ka = i & 1, kb = (i >> 1) & 1, q2 = i >> 2;
    V[lc][32 + i] = l1(kb, gx(0)) * V[lc][ka + 6 * q2] + l1(kb, gx(1)) * V[lc][ka + 2 + 6 * q2] +
                    l1(kb, gx(2)) * V[lc][ka + 4 + 6 * q2];
  }
  wsync();
  if (!live || i >= 8) return;
  const int a = i;
  double f = 0.0;
  if (!((mask >> a) & 1u)) {
    const int kc = a >> 2;
    if (t.probe & 32)
      f = S[lc][a];  // probe: no test-function sums
    else
      f = l1(kc, gx(0)) * V[lc][32 + (a & 3)] + l1(kc, gx(1)) * V[lc][36 + (a & 3)] +
          l1(kc, gx(2)) * V[lc][40 + (a & 3)];
    if (mask >> 8) {
      const double* L = t.loc + 64 * size_t(cd.sep_col[cell]);
      const double* r = t.rad + 16 * size_t(t.lay2ord[cd.sep_layer[cell]]);
      const int al = a & 3, ro = a >> 2;
      for (int b = 0; b < 8; ++b) {
        if (!((mask >> (8 + b)) & 1u)) continue;
        const double gb = cd.T_bc[cd.cell_T[8 * size_t(cell) + b]];
        const int be = b & 3, so = b >> 2;
        const double mab = L[4 * al + be] * r[2 * ro + so];
        const double kab = one_over_pe * (L[16 + 4 * al + be] * r[4 + 2 * ro + so] +
                                          L[32 + 4 * al + be] * r[8 + 2 * ro + so] +
                                          L[32 + 4 * be + al] * r[8 + 2 * so + ro] +
                                          L[48 + 4 * al + be] * r[12 + 2 * ro + so]);
        f -= gb * (mab + dt_T * kab);
      }
    }
  }
  t.rec[8 * size_t(cell) + a] = f;
}

// rhs[i] = sum of dof i's records in ascending cell order (<= 8 on the shell:
// the slot loads issued together, then the record loads)
__global__ __launch_bounds__(kTB) void k_tsep_gather(TSepDev t, int n_T, double* __restrict__ rhs) {
  const int i = xcd_block(int(blockIdx.x), int(gridDim.x)) * kTB + int(threadIdx.x);
  if (i >= n_T) return;
  const int b = t.sptr[i], e = t.sptr[i + 1];
  double s = 0.0;
  if (e - b <= 8) {
    int sl[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) sl[k] = b + k < e ? t.slot[b + k] : -1;
    double v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = sl[k] >= 0 ? t.rec[sl[k]] : 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (b + k < e) s += v[k];
  } else {
    for (int k = b; k < e; ++k) s += t.rec[t.slot[k]];
  }
  rhs[i] = s;
}

int blocks(long n) { return int((n + kTB - 1) / kTB); }

}  // namespace

void tsep_tables(const TSepDev& t, hipStream_t s) {
  hipLaunchKernelGGL(k_tsep_local, dim3(blocks(16L * t.n_colids + t.n_layers)), dim3(kTB), 0, s, t);
  DCP_HIP_CHECK(hipGetLastError());
}

void tsep_matrix(const TSepDev& t, long nnz, const PhysicsDev& ph, double* M, double* K,
                 double* Tmat, double* Tinv, hipStream_t s) {
  hipLaunchKernelGGL(k_tsep_lateral, dim3(blocks(long(t.n_kinds) * t.n_latnnz)), dim3(kTB), 0, s,
                     t);
  if (t.blk_pt && !(t.probe & 64)) {  // records staged in LDS (probe 64: per-entry A loads)
    const size_t lds_r = sizeof(double) * 16 * size_t(t.n_layers) + 48 * size_t(t.max_rec);
    const long B = long(t.blk_pt) * kTB;
    const unsigned nb = unsigned((nnz + B - 1) / B);
    if (t.blk_pt == 8)
      hipLaunchKernelGGL(k_tsep_matrix_lds<8>, dim3(nb), dim3(kTB), lds_r, s, t, nnz,
                         ph.one_over_peclet, ph.dt_T, M, K, Tmat, Tinv);
    else
      hipLaunchKernelGGL(k_tsep_matrix_lds<4>, dim3(nb), dim3(kTB), lds_r, s, t, nnz,
                         ph.one_over_peclet, ph.dt_T, M, K, Tmat, Tinv);
    DCP_HIP_CHECK(hipGetLastError());
    return;
  }
  const size_t lds = sizeof(double) * 16 * size_t(t.n_layers) + sizeof(int) * size_t(t.n_layers);
  // CSR entries per thread (DCP_TSEP_PT: 4 or 8; default 4)
  const char* env = std::getenv("DCP_TSEP_PT");
  const int pt = env && std::atoi(env) == 8 ? 8 : 4;
  const unsigned nb = unsigned((nnz + long(pt) * kTB - 1) / (long(pt) * kTB));
  if (pt == 8)
    hipLaunchKernelGGL(k_tsep_matrix<8>, dim3(nb), dim3(kTB), lds, s, t, nnz, ph.one_over_peclet,
                       ph.dt_T, M, K, Tmat, Tinv);
  else
    hipLaunchKernelGGL(k_tsep_matrix<4>, dim3(nb), dim3(kTB), lds, s, t, nnz, ph.one_over_peclet,
                       ph.dt_T, M, K, Tmat, Tinv);
  DCP_HIP_CHECK(hipGetLastError());
}

void tsep_rhs(const TSepDev& t, const CellData& cd, int n_T, const double* T_old,
              const double* u, const PhysicsDev& ph, double* rhs, hipStream_t s) {
  hipLaunchKernelGGL(k_tsep_rhs_cells, dim3((cd.n_cells + 7) / 8), dim3(kTB), 0, s, t, cd, T_old,
                     u, ph.one_over_peclet, ph.dt_T);
  hipLaunchKernelGGL(k_tsep_gather, dim3(blocks(n_T)), dim3(kTB), 0, s, t, n_T, rhs);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
