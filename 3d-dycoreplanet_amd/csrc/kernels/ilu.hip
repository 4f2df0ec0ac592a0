// ILU(0) of the velocity block for the Schur-complement solver
// (solve_NSE_Schur_complement, boussinesq_model.tpp:1248-1414; LA::PreconditionILU,
// linear_algebra/preconditioner.h:40) on CDNA4 (gfx950), FP64.
//
// The factor lives on the scalar pattern of nse_matrix.block(0,0): scalar row
// 3n + c holds, for every block (n, m) of the block-CSR A in column order, the
// columns 3m + c' (c' = 0..2), so the scalar pattern is sorted and entry k's
// value starts as A_val[pos[k]]. Rows are processed in dependency levels
// built on the host (a row's level is one more than the deepest row it reads):
// the elimination runs one launch per level, one thread per row, each row the
// IKJ form of the oracle's restatement (oracle/oracle.cpp Ilu0) in the same
// operation order, so the factors agree bit for bit. The triangular solves are
// one workgroup that walks the levels with a barrier between them: the solver
// is the reference's choice for its small configs (the 2D shell, the cube), where
// a level holds tens of rows and launch latency would dominate.
#include <hip/hip_runtime.h>

#include "../device.h"

namespace dcp {
namespace {

__global__ void k_ilu_load(long nnz, const int32_t* __restrict__ pos, const double* __restrict__ A,
                           double* __restrict__ lu) {
  for (long k = long(blockIdx.x) * blockDim.x + threadIdx.x; k < nnz;
       k += long(gridDim.x) * blockDim.x)
    lu[k] = A[pos[k]];
}

// the rows of one level: l_ik = a_ik / u_kk in column order k < i, then
// a_ij -= l_ik u_kj on row i's pattern (rows k are final: earlier levels)
__global__ void k_ilu_factor(int nrows, const int32_t* __restrict__ rows,
                             const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
                             const int32_t* __restrict__ diag, double* __restrict__ lu) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= nrows) return;
  const int i = rows[t];
  const int e = ptr[i + 1];
  for (int p = ptr[i]; p < e && col[p] < i; ++p) {
    const int k = col[p];
    lu[p] /= lu[diag[k]];
    const double lik = lu[p];
    int r = p + 1;
    for (int q = diag[k] + 1; q < ptr[k + 1]; ++q) {
      const int cq = col[q];
      while (r < e && col[r] < cq) ++r;
      if (r == e) break;
      if (col[r] == cq) lu[r] -= lik * lu[q];
    }
  }
}

// x = U^-1 L^-1 b: forward over the lower levels (unit diagonal), backward over
// the upper ones, each row's sum in column order (the oracle's order: the
// nested 1e-6 solves amplify any other rounding to ~1e-10 of the result; a
// wave per row with a butterfly sum measured 1.2e-10 against the oracle).
// The dependency chains of ILU(0) on this pattern are long (~2,000 levels for
// 10 k rows), so the solve is latency-bound whatever the row mapping.
constexpr int kIluThreads = 1024;
__global__ __launch_bounds__(kIluThreads) void k_ilu_solve(
    int n_lf, const int32_t* __restrict__ lf_ptr, const int32_t* __restrict__ lf_rows, int n_lb,
    const int32_t* __restrict__ lb_ptr, const int32_t* __restrict__ lb_rows,
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const int32_t* __restrict__ diag, const double* __restrict__ lu, const double* __restrict__ b,
    double* x) {
  for (int l = 0; l < n_lf; ++l) {
    for (int t = lf_ptr[l] + threadIdx.x; t < lf_ptr[l + 1]; t += kIluThreads) {
      const int i = lf_rows[t];
      double s = b[i];
      for (int p = ptr[i]; p < diag[i]; ++p) s -= lu[p] * x[col[p]];
      x[i] = s;
    }
    __syncthreads();
  }
  for (int l = 0; l < n_lb; ++l) {
    for (int t = lb_ptr[l] + threadIdx.x; t < lb_ptr[l + 1]; t += kIluThreads) {
      const int i = lb_rows[t];
      double s = x[i];
      for (int p = diag[i] + 1; p < ptr[i + 1]; ++p) s -= lu[p] * x[col[p]];
      x[i] = s / lu[diag[i]];
    }
    __syncthreads();
  }
}

__global__ void k_zero_at(int n, const int32_t* __restrict__ idx, double* __restrict__ x) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) x[idx[t]] = 0.0;
}

}  // namespace

void ilu_factor(const IluView& f, const double* A_val, const int* lf_host_ptr, double* lu,
                hipStream_t s) {
  if (f.nnz > 0) {
    const long g = std::min<long>((f.nnz + 255) / 256, 4096);
    hipLaunchKernelGGL(k_ilu_load, dim3(unsigned(g)), dim3(256), 0, s, f.nnz, f.pos, A_val, lu);
    DCP_HIP_CHECK(hipGetLastError());
  }
  for (int l = 0; l < f.n_lf; ++l) {
    const int nr = lf_host_ptr[l + 1] - lf_host_ptr[l];
    hipLaunchKernelGGL(k_ilu_factor, dim3((nr + 63) / 64), dim3(64), 0, s, nr,
                       f.lf_rows + lf_host_ptr[l], f.ptr, f.col, f.diag, lu);
    DCP_HIP_CHECK(hipGetLastError());
  }
}

void ilu_apply(const IluView& f, const double* lu, const double* b, double* x, hipStream_t s) {
  hipLaunchKernelGGL(k_ilu_solve, dim3(1), dim3(kIluThreads), 0, s, f.n_lf, f.lf_ptr, f.lf_rows,
                     f.n_lb, f.lb_ptr, f.lb_rows, f.ptr, f.col, f.diag, lu, b, x);
  DCP_HIP_CHECK(hipGetLastError());
}

void zero_at(int n, const int32_t* idx, double* x, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_zero_at, dim3((n + 255) / 256), dim3(256), 0, s, n, idx, x);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
