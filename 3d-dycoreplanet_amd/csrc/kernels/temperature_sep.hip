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
//                  tables per layer (geometry tables of the upload, no cache
//                  of any result),
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

#include "../device.h"
#include "../fe_tables.h"

namespace dcp {
namespace {

constexpr int kTB = 256;

__constant__ double tW[3] = {kGaussW[0], kGaussW[1], kGaussW[2]};
// Q1 1D basis and derivative at the 3 Gauss points: [basis][point]
__constant__ double tL1[2][3] = {{1 - kGaussX[0], 1 - kGaussX[1], 1 - kGaussX[2]},
                                 {kGaussX[0], kGaussX[1], kGaussX[2]}};
__constant__ double tD1[2] = {-1.0, 1.0};
// Q2 1D basis at the 3 Gauss points: [basis][point]
__constant__ double tL2[3][3] = {
    {2 * (kGaussX[0] - 0.5) * (kGaussX[0] - 1), 2 * (kGaussX[1] - 0.5) * (kGaussX[1] - 1),
     2 * (kGaussX[2] - 0.5) * (kGaussX[2] - 1)},
    {-4 * kGaussX[0] * (kGaussX[0] - 1), -4 * kGaussX[1] * (kGaussX[1] - 1),
     -4 * kGaussX[2] * (kGaussX[2] - 1)},
    {2 * kGaussX[0] * (kGaussX[0] - 0.5), 2 * kGaussX[1] * (kGaussX[1] - 0.5),
     2 * kGaussX[2] * (kGaussX[2] - 0.5)}};

// Lateral tables of one column id (4 threads per column id, one per alpha):
// loc[64 id + 16 t + 4 alpha + beta], t = LM, Lll, Lx, L22. Radial tables of
// ordinal layer o (threads after the columns): rad[16 o + 4 t + 2 rho + sigma],
// t = RM, Rll, Rx, R22.
__global__ __launch_bounds__(kTB) void k_tsep_local(TSepDev t) {
  const int gid = int(blockIdx.x) * kTB + int(threadIdx.x);
  if (gid < 4 * t.n_colids) {
    const int id = gid >> 2, al = gid & 3;
    const int va = al & 1, vb = al >> 1;
    double LM[4] = {0, 0, 0, 0}, Lll[4] = {0, 0, 0, 0}, Lx[4] = {0, 0, 0, 0},
           L22[4] = {0, 0, 0, 0};
    for (int q1 = 0; q1 < 3; ++q1)
      for (int q0 = 0; q0 < 3; ++q0) {
        const double* g = t.colgeo + 90 * size_t(id) + 10 * (q0 + 3 * q1);
        const double W = g[9] * tW[q0] * tW[q1];
        const double d00 = g[0] * g[0] + g[1] * g[1] + g[2] * g[2];
        const double d01 = g[0] * g[3] + g[1] * g[4] + g[2] * g[5];
        const double d11 = g[3] * g[3] + g[4] * g[4] + g[5] * g[5];
        const double d02 = g[0] * g[6] + g[1] * g[7] + g[2] * g[8];
        const double d12 = g[3] * g[6] + g[4] * g[7] + g[5] * g[8];
        const double d22 = g[6] * g[6] + g[7] * g[7] + g[8] * g[8];
        const double pa = tL1[va][q0] * tL1[vb][q1];
        const double a0 = tD1[va] * tL1[vb][q1], a1 = tL1[va][q0] * tD1[vb];
#pragma unroll
        for (int be = 0; be < 4; ++be) {
          const int wa = be & 1, wb = be >> 1;
          const double pb = tL1[wa][q0] * tL1[wb][q1];
          const double b0 = tD1[wa] * tL1[wb][q1], b1 = tL1[wa][q0] * tD1[wb];
          LM[be] += pa * pb * W;
          Lll[be] += (a0 * b0 * d00 + a0 * b1 * d01 + a1 * b0 * d01 + a1 * b1 * d11) * W;
          Lx[be] += (a0 * d02 + a1 * d12) * pb * W;
          L22[be] += pa * pb * d22 * W;
        }
      }
    double* o = t.loc + 64 * size_t(id) + 4 * al;
#pragma unroll
    for (int be = 0; be < 4; ++be) {
      o[be] = LM[be];
      o[16 + be] = Lll[be];
      o[32 + be] = Lx[be];
      o[48 + be] = L22[be];
    }
    return;
  }
  const int o = gid - 4 * t.n_colids;
  if (o >= t.n_layers) return;
  const int lid = t.ord2lay[o];
  double r[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = 0.0;
  for (int q = 0; q < 3; ++q) {
    const double* lg = t.laygeo + 9 * size_t(lid) + 3 * q;
    const double R = t.layR[3 * size_t(lid) + q], Rp = 1.0 / lg[1], R2Rp = lg[2];
    const double w = tW[q];
#pragma unroll
    for (int ro = 0; ro < 2; ++ro)
#pragma unroll
      for (int so = 0; so < 2; ++so) {
        const double cc = tL1[ro][q] * tL1[so][q];
        r[2 * ro + so] += cc * R2Rp * w;
        r[4 + 2 * ro + so] += cc * Rp * w;
        r[8 + 2 * ro + so] += tL1[ro][q] * tD1[so] * R * w;
        r[12 + 2 * ro + so] += tD1[ro] * tD1[so] * (R * R / Rp) * w;
      }
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) t.rad[16 * size_t(o) + i] = r[i];
}

// A[(kind n_latnnz + p) 5 + t], t = M, ll, x, x^T, 22: the column sums of the
// lateral tables in the contribution order of the upload (ascending column).
__global__ __launch_bounds__(kTB) void k_tsep_lateral(TSepDev t) {
  const int gid = int(blockIdx.x) * kTB + int(threadIdx.x);
  if (gid >= t.n_kinds * t.n_latnnz) return;
  const int k = gid / t.n_latnnz, p = gid - k * t.n_latnnz;
  double s[5] = {0, 0, 0, 0, 0};
  for (int j = t.lptr[p]; j < t.lptr[p + 1]; ++j) {
    const int c = t.lcon[j];
    const int C = c >> 4, al = (c >> 2) & 3, be = c & 3;
    const double* L = t.loc + 64 * size_t(t.kc[size_t(C) * t.n_kinds + k]);
    s[0] += L[4 * al + be];
    s[1] += L[16 + 4 * al + be];
    s[2] += L[32 + 4 * al + be];
    s[3] += L[32 + 4 * be + al];
    s[4] += L[48 + 4 * al + be];
  }
  double* a = t.A + 5 * size_t(gid);
#pragma unroll
  for (int i = 0; i < 5; ++i) a[i] = s[i];
}

// code: bits 0-19 lateral entry p, 20-27 row level l, 28-29 l' - l + 1,
// 30 "zero" (off-diagonal entry of a fixed row or column), 31 diagonal.
__global__ __launch_bounds__(kTB) void k_tsep_matrix(TSepDev t, long nnz, double one_over_pe,
                                                     double dt_T, double* __restrict__ M,
                                                     double* __restrict__ K,
                                                     double* __restrict__ Tmat,
                                                     double* __restrict__ Tinv) {
  const long e = long(blockIdx.x) * kTB + threadIdx.x;
  if (e >= nnz) return;
  const uint32_t code = __builtin_nontemporal_load(t.code + e);
  double m = 0.0, k = 0.0;
  if (!((code >> 30) & 1u)) {
    const int p = int(code & 0xFFFFFu), l = int((code >> 20) & 0xFFu), dl = int((code >> 28) & 3u);
    auto add = [&](int o, int ro, int so) {
      const double* a = t.A + 5 * (size_t(t.kind[o]) * t.n_latnnz + p);
      const double* r = t.rad + 16 * size_t(o);
      m += a[0] * r[2 * ro + so];
      k += a[1] * r[4 + 2 * ro + so] + a[2] * r[8 + 2 * ro + so] + a[3] * r[8 + 2 * so + ro] +
           a[4] * r[12 + 2 * ro + so];
    };
    if (dl == 2) {
      add(l, 0, 1);
    } else if (dl == 0) {
      add(l - 1, 1, 0);
    } else {
      if (l >= 1) add(l - 1, 1, 1);
      if (l < t.n_layers) add(l, 0, 0);
    }
    k *= one_over_pe;
  }
  const double tm = m + dt_T * k;
  __builtin_nontemporal_store(m, M + e);
  __builtin_nontemporal_store(k, K + e);
  __builtin_nontemporal_store(tm, Tmat + e);
  if (code >> 31) Tinv[t.T_col[e]] = 1.0 / tm;
}

// Records of the temperature rhs, 8 cells per workgroup (two per wave, lanes
// 0-26 and 32-58 one Gauss point each): f_a = sum_q phi_a (T w - dt u.grad T w)
// for the free rows a, minus the lift sum_{b fixed, g_b != 0} g_b (M + dt K)_ab
// (boussinesq_model.tpp:922-949); 0 for fixed rows.
__global__ __launch_bounds__(kTB) void k_tsep_rhs_cells(TSepDev t, CellData cd,
                                                        const double* __restrict__ T_old,
                                                        const double* __restrict__ u,
                                                        double one_over_pe, double dt_T) {
  __shared__ double U[8][81];
  __shared__ double Tn[8][8];
  __shared__ double S[8][27];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lc = 2 * wave + (lane >> 5), i = lane & 31;
  const int cell = 8 * int(blockIdx.x) + lc;
  const bool live = cell < cd.n_cells;
  if (live && i < 27) {
    const int n = cd.cell_q2[27 * size_t(cell) + i];
#pragma unroll
    for (int d = 0; d < 3; ++d) U[lc][3 * i + d] = u[3 * size_t(n) + d];
    if (i < 8) Tn[lc][i] = T_old[cd.cell_T[8 * size_t(cell) + i]];
  }
  __syncthreads();
  if (live && i < 27) {
    const int q = i, q0 = q % 3, q1 = (q / 3) % 3, q2 = q / 9;
    const double* g = t.colgeo + 90 * size_t(cd.sep_col[cell]) + 10 * (q0 + 3 * q1);
    const double* lg = t.laygeo + 9 * size_t(cd.sep_layer[cell]) + 3 * q2;
    const double iR = lg[0], iRp = lg[1];
    // T and its reference derivatives at q
    double T = 0, r0 = 0, r1 = 0, r2 = 0;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int va = v & 1, vb = (v >> 1) & 1, vc = v >> 2;
      const double la = tL1[va][q0], lb = tL1[vb][q1], lc3 = tL1[vc][q2];
      const double tv = Tn[lc][v];
      T += tv * (la * lb * lc3);
      r0 += tv * (tD1[va] * lb * lc3);
      r1 += tv * (la * tD1[vb] * lc3);
      r2 += tv * (la * lb * tD1[vc]);
    }
    double gT[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) gT[d] = r0 * (g[d] * iR) + r1 * (g[3 + d] * iR) + r2 * (g[6 + d] * iRp);
    double uq[3] = {0, 0, 0};
    for (int c = 0; c < 3; ++c) {
      const double lcq = tL2[c][q2];
#pragma unroll
      for (int b = 0; b < 3; ++b) {
        const double lbc = tL2[b][q1] * lcq;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          const double s = tL2[a][q0] * lbc;
          const int n = a + 3 * b + 9 * c;
          uq[0] += U[lc][3 * n] * s;
          uq[1] += U[lc][3 * n + 1] * s;
          uq[2] += U[lc][3 * n + 2] * s;
        }
      }
    }
    const double w = lg[2] * g[9] * (tW[q0] * tW[q1] * tW[q2]);
    S[lc][q] = T * w - dt_T * (uq[0] * gT[0] + uq[1] * gT[1] + uq[2] * gT[2]) * w;
  }
  __syncthreads();
  if (!live || i >= 8) return;
  const int a = i;
  const int32_t* dofs = cd.cell_T + 8 * size_t(cell);
  double f = 0.0;
  if (!cd.T_fixed[dofs[a]]) {
    const int va = a & 1, vb = (a >> 1) & 1, vc = a >> 2;
    for (int q = 0; q < 27; ++q)
      f += (tL1[va][q % 3] * tL1[vb][(q / 3) % 3] * tL1[vc][q / 9]) * S[lc][q];
    const double* L = t.loc + 64 * size_t(cd.sep_col[cell]);
    const double* r = t.rad + 16 * size_t(t.lay2ord[cd.sep_layer[cell]]);
    const int al = a & 3, ro = a >> 2;
    for (int b = 0; b < 8; ++b) {
      const int db = dofs[b];
      if (!cd.T_fixed[db]) continue;
      const double gb = cd.T_bc[db];
      if (gb == 0.0) continue;
      const int be = b & 3, so = b >> 2;
      const double mab = L[4 * al + be] * r[2 * ro + so];
      const double kab = one_over_pe * (L[16 + 4 * al + be] * r[4 + 2 * ro + so] +
                                        L[32 + 4 * al + be] * r[8 + 2 * ro + so] +
                                        L[32 + 4 * be + al] * r[8 + 2 * so + ro] +
                                        L[48 + 4 * al + be] * r[12 + 2 * ro + so]);
      f -= gb * (mab + dt_T * kab);
    }
  }
  t.rec[8 * size_t(cell) + a] = f;
}

__global__ __launch_bounds__(kTB) void k_tsep_gather(TSepDev t, int n_T, double* __restrict__ rhs) {
  const int i = int(blockIdx.x) * kTB + int(threadIdx.x);
  if (i >= n_T) return;
  double s = 0.0;
  for (int k = t.sptr[i]; k < t.sptr[i + 1]; ++k) s += t.rec[t.slot[k]];
  rhs[i] = s;
}

int blocks(long n) { return int((n + kTB - 1) / kTB); }

}  // namespace

void tsep_matrix(const TSepDev& t, long nnz, const PhysicsDev& ph, double* M, double* K,
                 double* Tmat, double* Tinv, hipStream_t s) {
  hipLaunchKernelGGL(k_tsep_local, dim3(blocks(4L * t.n_colids + t.n_layers)), dim3(kTB), 0, s, t);
  hipLaunchKernelGGL(k_tsep_lateral, dim3(blocks(long(t.n_kinds) * t.n_latnnz)), dim3(kTB), 0, s,
                     t);
  hipLaunchKernelGGL(k_tsep_matrix, dim3(blocks(nnz)), dim3(kTB), 0, s, t, nnz, ph.one_over_peclet,
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
