// Temperature FE_Q(2) of the 3D classic model (temperature_fe(2),
// boussinesq_model.tpp:30; data/aqua_planet.prm, aqua_planet_test_3d.prm),
// hand-written HIP for gfx950, FP64.
//
//   k_T2_matrix   local_assemble_temperature_matrix (:748-800), QGauss(4)
//                 + distribute_local_to_global with the constrained diagonal
//   k_T2_rhs      local_assemble_temperature_rhs (:873-952), QGauss(4), the
//                 velocity of nse_solution (Q5), the matrix_for_bc lift
//
// One 64-lane wavefront per cell and one QGauss(4) point per lane: lane q
// evaluates the MappingQ(3) map from the 64 support points (cd.geo), JxW and
// the 27 physical Q2 shape gradients into LDS; then lanes sum the local
// entries (729 of them for the matrices, 27 rows for the rhs) over the 64
// points. Cell temperature dofs arrive in lexicographic order (api.cpp
// converts FE_Q(2)'s hierarchic local order on upload).
#include <hip/hip_runtime.h>

#include "../device.h"
#include "../fe_tables.h"

namespace dcp {
namespace {

__constant__ double cG4[4] = {0.069431844202973712388, 0.33000947820757186760,
                              0.66999052179242813240, 0.93056815579702628761};
__constant__ double cW4[4] = {0.17392742256872692869, 0.32607257743127307131,
                              0.32607257743127307131, 0.17392742256872692869};
__constant__ double cGLq[4] = {0.0, 0.27639320225002103036, 0.72360679774997896964, 1.0};

__device__ inline double l2(int i, double x) {
  return i == 0 ? 2.0 * (x - 0.5) * (x - 1.0) : i == 1 ? -4.0 * x * (x - 1.0) : 2.0 * x * (x - 0.5);
}
__device__ inline double d2(int i, double x) {
  return i == 0 ? 4.0 * x - 3.0 : i == 1 ? -8.0 * x + 4.0 : 4.0 * x - 1.0;
}
__device__ inline void l3(double x, double v[4], double d[4]) {
  for (int i = 0; i < 4; ++i) {
    double p = 1.0, s = 0.0;
    for (int j = 0; j < 4; ++j) {
      if (j == i) continue;
      p *= (x - cGLq[j]) / (cGLq[i] - cGLq[j]);
    }
    for (int k = 0; k < 4; ++k) {
      if (k == i) continue;
      double t = 1.0 / (cGLq[i] - cGLq[k]);
      for (int j = 0; j < 4; ++j)
        if (j != i && j != k) t *= (x - cGLq[j]) / (cGLq[i] - cGLq[j]);
      s += t;
    }
    v[i] = p;
    d[i] = s;
  }
}

struct T2Smem {
  double X[3 * kMapPts];
  double V[64][27];
  double G[64][27][3];
  double JxW[64];
  double Tq[64], Fq[64];
  double U[81];
  double Tn[27];
  double dM[27], dK[27];
  int dof[27];
  int fixed[27];
};

// lane q: mapping, JxW and the Q2 basis at QGauss(4) point q
__device__ inline void t2_point(T2Smem& sh, int q) {
  const double xi[3] = {cG4[q & 3], cG4[(q >> 2) & 3], cG4[q >> 4]};
  double lv[3][4], ld[3][4];
  for (int e = 0; e < 3; ++e) l3(xi[e], lv[e], ld[e]);
  double J[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
  for (int t = 0; t < kMapPts; ++t) {
    const int a = t & 3, b = (t >> 2) & 3, c = t >> 4;
    const double g0 = ld[0][a] * lv[1][b] * lv[2][c];
    const double g1 = lv[0][a] * ld[1][b] * lv[2][c];
    const double g2 = lv[0][a] * lv[1][b] * ld[2][c];
    for (int i = 0; i < 3; ++i) {
      const double Xi = sh.X[3 * t + i];
      J[i][0] += Xi * g0;
      J[i][1] += Xi * g1;
      J[i][2] += Xi * g2;
    }
  }
  const double c00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
  const double c01 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
  const double c02 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
  const double det = J[0][0] * c00 + J[0][1] * c01 + J[0][2] * c02;
  const double id = 1.0 / det;
  double Ji[3][3];
  Ji[0][0] = c00 * id;
  Ji[0][1] = (J[0][2] * J[2][1] - J[0][1] * J[2][2]) * id;
  Ji[0][2] = (J[0][1] * J[1][2] - J[0][2] * J[1][1]) * id;
  Ji[1][0] = c01 * id;
  Ji[1][1] = (J[0][0] * J[2][2] - J[0][2] * J[2][0]) * id;
  Ji[1][2] = (J[0][2] * J[1][0] - J[0][0] * J[1][2]) * id;
  Ji[2][0] = c02 * id;
  Ji[2][1] = (J[0][1] * J[2][0] - J[0][0] * J[2][1]) * id;
  Ji[2][2] = (J[0][0] * J[1][1] - J[0][1] * J[1][0]) * id;
  sh.JxW[q] = det * cW4[q & 3] * cW4[(q >> 2) & 3] * cW4[q >> 4];
  for (int n = 0; n < 27; ++n) {
    const int a = n % 3, b = (n / 3) % 3, c = n / 9;
    const double va = l2(a, xi[0]), vb = l2(b, xi[1]), vc = l2(c, xi[2]);
    sh.V[q][n] = va * vb * vc;
    const double r[3] = {d2(a, xi[0]) * vb * vc, va * d2(b, xi[1]) * vc, va * vb * d2(c, xi[2])};
    for (int i = 0; i < 3; ++i) sh.G[q][n][i] = Ji[0][i] * r[0] + Ji[1][i] * r[1] + Ji[2][i] * r[2];
  }
}

__device__ inline double gdot(const double* a, const double* b) {
  return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

__global__ __launch_bounds__(64) void k_T2_matrix(CellData cd, ScatterMaps sm,
                                                  const int32_t* __restrict__ cells, PhysicsDev ph,
                                                  double* __restrict__ Tmass,
                                                  double* __restrict__ Tstiff) {
  __shared__ T2Smem sh;
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  for (int i = tid; i < 3 * kMapPts; i += 64) sh.X[i] = cd.geo[3 * kMapPts * size_t(cell) + i];
  if (tid < 27) {
    const int d = cd.cell_T[27 * size_t(cell) + tid];
    sh.dof[tid] = d;
    sh.fixed[tid] = cd.T_fixed[d];
  }
  __syncthreads();
  t2_point(sh, tid);
  __syncthreads();
  auto entry = [&](int i, int j, double& M, double& K) {
    M = K = 0;
    for (int q = 0; q < 64; ++q) {
      M += sh.V[q][i] * sh.V[q][j] * sh.JxW[q];
      K += gdot(sh.G[q][i], sh.G[q][j]) * ph.one_over_peclet * sh.JxW[q];
    }
  };
  if (tid < 27) {
    double M, K;
    entry(tid, tid, M, K);
    sh.dM[tid] = fabs(M);
    sh.dK[tid] = fabs(K);
  }
  __syncthreads();
  double aM = 0, aK = 0;
  for (int k = 0; k < 27; ++k) {
    aM += sh.dM[k];
    aK += sh.dK[k];
  }
  aM /= 27.0;
  aK /= 27.0;
  for (int e = tid; e < 729; e += 64) {
    const int i = e / 27, j = e % 27;
    const size_t p = size_t(sm.posT[729 * size_t(cell) + e]);
    if (sh.fixed[i] || sh.fixed[j]) {
      // constrained row / column: the diagonal only, |K_ii| or the mean
      if (i == j) {
        Tmass[p] += sh.dM[i] != 0.0 ? sh.dM[i] : aM;
        Tstiff[p] += sh.dK[i] != 0.0 ? sh.dK[i] : aK;
      }
      continue;
    }
    double M, K;
    entry(i, j, M, K);
    Tmass[p] += M;
    Tstiff[p] += K;
  }
}

__global__ __launch_bounds__(64) void k_T2_rhs(CellData cd, const int32_t* __restrict__ cells,
                                               const double* __restrict__ T_old,
                                               const double* __restrict__ u_cur, PhysicsDev ph,
                                               double* __restrict__ rhs) {
  __shared__ T2Smem sh;
  const int tid = threadIdx.x;
  const int cell = cells[blockIdx.x];
  for (int i = tid; i < 3 * kMapPts; i += 64) sh.X[i] = cd.geo[3 * kMapPts * size_t(cell) + i];
  if (tid < 27) {
    const int d = cd.cell_T[27 * size_t(cell) + tid];
    sh.dof[tid] = d;
    sh.fixed[tid] = cd.T_fixed[d];
    sh.Tn[tid] = T_old[d];
    const int n = cd.cell_q2[27 * size_t(cell) + tid];
#pragma unroll
    for (int c = 0; c < 3; ++c) sh.U[3 * tid + c] = u_cur[3 * size_t(n) + c];
  }
  __syncthreads();
  t2_point(sh, tid);
  {
    // lane q: T, grad T (old temperature) and u (nse_solution, Q5) at point q
    const int q = tid;
    double T = 0, gT[3] = {0, 0, 0}, u[3] = {0, 0, 0};
    for (int n = 0; n < 27; ++n) {
      const double v = sh.V[q][n];
      T += sh.Tn[n] * v;
      for (int i = 0; i < 3; ++i) {
        gT[i] += sh.Tn[n] * sh.G[q][n][i];
        u[i] += sh.U[3 * n + i] * v;
      }
    }
    sh.Tq[q] = T * sh.JxW[q];
    sh.Fq[q] = ph.dt_T * gdot(u, gT) * sh.JxW[q];
  }
  __syncthreads();
  if (tid >= 27) return;
  const int j = tid;
  if (sh.fixed[j]) return;  // constrained rows receive nothing
  double f = 0;
  for (int q = 0; q < 64; ++q) f += sh.V[q][j] * (sh.Tq[q] - sh.Fq[q]);
  // lift: - sum_{i inhomogeneous} g_i (M + dt_T K)_ji
  for (int i = 0; i < 27; ++i) {
    if (!sh.fixed[i]) continue;
    const double g = cd.T_bc[sh.dof[i]];
    if (g == 0.0) continue;
    double mb = 0;
    for (int q = 0; q < 64; ++q)
      mb += (sh.V[q][i] * sh.V[q][j] + ph.dt_T * ph.one_over_peclet * gdot(sh.G[q][i], sh.G[q][j])) *
            sh.JxW[q];
    f -= g * mb;
  }
  rhs[sh.dof[j]] += f;
}

}  // namespace

void launch_T2_matrix(const CellData& cd, const ScatterMaps& sm, const int32_t* cells, int n,
                      const PhysicsDev& ph, double* Tmass, double* Tstiff, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_T2_matrix, dim3(n), dim3(64), 0, s, cd, sm, cells, ph, Tmass, Tstiff);
  DCP_HIP_CHECK(hipGetLastError());
}

void launch_T2_rhs(const CellData& cd, const int32_t* cells, int n, const double* T_old,
                   const double* u_cur, const PhysicsDev& ph, double* rhs, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_T2_rhs, dim3(n), dim3(64), 0, s, cd, cells, T_old, u_cur, ph, rhs);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
