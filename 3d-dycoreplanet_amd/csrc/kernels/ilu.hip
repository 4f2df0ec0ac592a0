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

// The same elimination with a wave per row (rows of up to kIluRowMax
// entries): the row is staged in LDS; for each k of its lower part in column
// order the lanes split row k's upper entries, each finding its column in the
// row by binary search. Every entry receives its updates in k order with the
// same arithmetic as the one-thread form (bitwise the same factor).
constexpr int kIluRowMax = 512;
__device__ inline void wsync64() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__global__ __launch_bounds__(64) void k_ilu_factor_wave(int nrows, const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ ptr,
                                                        const int32_t* __restrict__ col,
                                                        const int32_t* __restrict__ diag,
                                                        double* __restrict__ lu) {
  __shared__ double rv[kIluRowMax];
  __shared__ int rc[kIluRowMax];
  const int t = blockIdx.x;
  if (t >= nrows) return;
  const int lane = threadIdx.x;
  const int i = rows[t];
  const int b = ptr[i], len = ptr[i + 1] - b;
  for (int j = lane; j < len; j += 64) {
    rv[j] = lu[b + j];
    rc[j] = col[b + j];
  }
  wsync64();
  for (int pj = 0; pj < len && rc[pj] < i; ++pj) {
    const int k = rc[pj];
    const double lik = rv[pj] / lu[diag[k]];
    wsync64();  // every lane has read rv[pj]
    if (lane == 0) rv[pj] = lik;
    for (int q = diag[k] + 1 + lane; q < ptr[k + 1]; q += 64) {
      const int cq = col[q];
      int lo = pj + 1, hi = len;
      while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (rc[m] < cq) lo = m + 1; else hi = m;
      }
      if (lo < len && rc[lo] == cq) rv[lo] -= lik * lu[q];
    }
    wsync64();
  }
  for (int j = lane; j < len; j += 64) lu[b + j] = rv[j];
}

// x = U^-1 L^-1 b: forward over the lower levels (unit diagonal), backward over
// the upper ones. The dependency chains of ILU(0) on this pattern are long
// (~2,000 levels for 10 k rows, a handful of rows each), so each row gets a
// wave: 64 lane-strided partial sums combined by an xor butterfly, the order
// the oracle's restatement uses too (oracle.cpp row_sum64).
constexpr int kIluThreads = 1024;
constexpr int kIluWaves = kIluThreads / 64;
__device__ inline double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__global__ __launch_bounds__(kIluThreads) void k_ilu_solve(
    int n_lf, const int32_t* __restrict__ lf_ptr, const int32_t* __restrict__ lf_rows, int n_lb,
    const int32_t* __restrict__ lb_ptr, const int32_t* __restrict__ lb_rows,
    const int32_t* __restrict__ ptr, const int32_t* __restrict__ col,
    const int32_t* __restrict__ diag, const double* __restrict__ lu, const double* __restrict__ b,
    double* x) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  for (int l = 0; l < n_lf; ++l) {
    for (int t = lf_ptr[l] + wave; t < lf_ptr[l + 1]; t += kIluWaves) {
      const int i = lf_rows[t];
      double s = 0.0;
      for (int p = ptr[i] + lane; p < diag[i]; p += 64) s += lu[p] * x[col[p]];
      s = wave_sum(s);
      if (lane == 0) x[i] = b[i] - s;
    }
    __syncthreads();
  }
  for (int l = 0; l < n_lb; ++l) {
    for (int t = lb_ptr[l] + wave; t < lb_ptr[l + 1]; t += kIluWaves) {
      const int i = lb_rows[t];
      double s = 0.0;
      for (int p = diag[i] + 1 + lane; p < ptr[i + 1]; p += 64) s += lu[p] * x[col[p]];
      s = wave_sum(s);
      if (lane == 0) x[i] = (x[i] - s) / lu[diag[i]];
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
                int max_row, hipStream_t s) {
  if (f.nnz > 0) {
    const long g = std::min<long>((f.nnz + 255) / 256, 4096);
    hipLaunchKernelGGL(k_ilu_load, dim3(unsigned(g)), dim3(256), 0, s, f.nnz, f.pos, A_val, lu);
    DCP_HIP_CHECK(hipGetLastError());
  }
  for (int l = 0; l < f.n_lf; ++l) {
    const int nr = lf_host_ptr[l + 1] - lf_host_ptr[l];
    if (max_row <= kIluRowMax)
      hipLaunchKernelGGL(k_ilu_factor_wave, dim3(nr), dim3(64), 0, s, nr,
                         f.lf_rows + lf_host_ptr[l], f.ptr, f.col, f.diag, lu);
    else
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
