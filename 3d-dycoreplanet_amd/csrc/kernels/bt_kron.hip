// B^T of nse_matrix in Kronecker form on the layered shell, FP64.
//
// Replaces k_bt_tasks (assembly.hip) for one GPU: the (0,1) block of the
// reference's local_assemble_nse_system (boussinesq_model.tpp:626-637,
// -phi_p div phi_u) scattered by copy_local_to_global (:677-687).
//
// A cell's entry of velocity node (a, b, c) and pressure vertex (i, j, k) is
//   -(P01[col][a b i j][d] Q01[layer][c][k] + P2[col][a b i j][d] Q2[layer][c][k])
// (k_bt_coltab / k_bt_laytab: column and layer factors of the separable map,
// formed at upload). The cells are the full product of lateral columns and
// radial layers, and the node / dof sets the products (lateral node, level),
// so the assembled entry of node (nu, lambda) and pressure dof (v, l) is
//   -sum_{layers L holding both} (A01^{kind L}(nu, v)[d] Q01[L][c][k]
//                               + A2^{kind L}(nu, v)[d] Q2[L][c][k]),
//   c = lambda - 2 L, k = l - L,
// A_t^kind(nu, v) = sum over the (one to four) columns holding nu and v of
// that kind's P_t: the lateral matrices. Per assembly:
//   k_btk_lateral  A^kind from P (2 kinds x ~154 k lateral pairs at r=5),
//   k_btk_entries  one thread per B^T entry (4 per thread, kTB apart, each XCD
//                  a contiguous range): the one or two layer terms, written
//                  once (no zero fill, no colouring, no atomics),
//   k_btk_con      the entries of constrained rows (no-normal-flux nodes):
//                  the same value condensed with the row's constraint C^T.
#include <hip/hip_runtime.h>

#include "../device.h"

namespace dcp {
namespace {

constexpr int kTB = 256;
#ifndef DCP_BTK_PT
#define DCP_BTK_PT 4
#endif
constexpr int kPT = DCP_BTK_PT;  // entries per thread

// A[(kind n_pairs + pair) 6 + (t 3 + d)], t = 01, 2
__global__ __launch_bounds__(kTB) void k_btk_lateral(BtkDev b) {
  const int gid = int(blockIdx.x) * kTB + int(threadIdx.x);
  if (gid >= b.n_kinds * b.n_pairs) return;
  const int k = gid / b.n_pairs, p = gid - k * b.n_pairs;
  const int32_t* con = b.lcon + size_t(k) * b.n_con;
  double s[6] = {0, 0, 0, 0, 0, 0};
  for (int j = b.lptr[p]; j < b.lptr[p + 1]; ++j) {
    const double* P = b.P + con[j];  // colid 216 + a 36 + b 12 + i 6 + j 3
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      s[d] += P[d];
      s[3 + d] += P[108 + d];
    }
  }
  double* a = b.A + 6 * size_t(gid);
#pragma unroll
  for (int i = 0; i < 6; ++i) a[i] = s[i];
}

// code: bits 0-19 lateral pair, 20-27 node level lambda, 28-29 l - lambda / 2 + 1,
// 30 constrained row (k_btk_con writes it)
__device__ __forceinline__ void btk_value(const BtkDev& b, const int* skind, const double* sq,
                                          uint32_t code, double v[3]) {
  int p = int(code & 0xFFFFFu);
  const int lam = int((code >> 20) & 0xFFu), dl = int((code >> 28) & 3u);
  if (b.probe & 1) p &= 4095;  // probe: a 4096-pair window of A (L2-resident)
  if (b.probe & 2) {           // probe: no A / Q reads
    v[0] = double(p);
    v[1] = double(lam);
    v[2] = double(dl);
    return;
  }
  const int m = lam >> 1;
  v[0] = v[1] = v[2] = 0.0;
  auto add = [&](int L, int c, int k) {
    const double2* a2 = reinterpret_cast<const double2*>(b.A + 6 * (size_t(skind[L]) * b.n_pairs + p));
    const double2 A0 = a2[0], A1 = a2[1], A2 = a2[2];
    const double q01 = sq[12 * L + 4 * c + 2 * k], q2 = sq[12 * L + 4 * c + 2 * k + 1];
    v[0] -= A0.x * q01 + A1.y * q2;
    v[1] -= A0.y * q01 + A2.x * q2;
    v[2] -= A1.x * q01 + A2.y * q2;
  };
  if (lam & 1) {
    add(m, 1, dl - 1);
  } else if (dl == 0) {
    if (m >= 1) add(m - 1, 2, 0);
  } else if (dl == 2) {
    add(m, 0, 1);
  } else {
    if (m >= 1) add(m - 1, 2, 1);
    if (m < b.n_layers) add(m, 0, 0);
  }
}

__device__ __forceinline__ void btk_stage(const BtkDev& b, double* sq, int* skind) {
  for (int i = threadIdx.x; i < 12 * b.n_layers; i += kTB)
    sq[i] = b.Q[12 * size_t(b.ord2lay[i / 12]) + i % 12];
  for (int i = threadIdx.x; i < b.n_layers; i += kTB) skind[i] = b.kind[i];
}

// The 64 entries of a wave (per u) are 192 consecutive doubles of B^T: staged
// in LDS so each store instruction writes 512 contiguous bytes. Entries of
// constrained rows are written unconstrained here and overwritten by k_btk_con
// (same stream, after).
__global__ __launch_bounds__(kTB) void k_btk_entries(BtkDev b, long nnz, double* __restrict__ Bt) {
  extern __shared__ __attribute__((aligned(16))) double sq[];
  int* skind = reinterpret_cast<int*>(sq + 12 * b.n_layers);
  __shared__ double stage[kTB / 64][192];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long base = long(xcd_block(int(blockIdx.x), int(gridDim.x))) * (kPT * kTB) + threadIdx.x;
  uint32_t code[kPT];
#pragma unroll
  for (int u = 0; u < kPT; ++u) {
    const long e = base + long(u) * kTB;
    code[u] = e < nnz ? __builtin_nontemporal_load(b.code + e) : 0u;
  }
  btk_stage(b, sq, skind);
  __syncthreads();
  // every entry's A loads issued before the first LDS hand-off (the fences of
  // the hand-off would keep the next entry's loads behind this one's stores)
  double v[kPT][3];
#pragma unroll
  for (int u = 0; u < kPT; ++u) btk_value(b, skind, sq, code[u], v[u]);
#pragma unroll
  for (int u = 0; u < kPT; ++u) {
    stage[wave][3 * lane] = v[u][0];
    stage[wave][3 * lane + 1] = v[u][1];
    stage[wave][3 * lane + 2] = v[u][2];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const long e0 = base - lane + long(u) * kTB;  // the wave's first entry
    const long left = 3 * (nnz - e0);             // doubles of B^T left from there
    double* dst = Bt + 3 * e0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int k = lane + 64 * r;
      if (k < left && !(b.probe & 4)) __builtin_nontemporal_store(stage[wave][k], dst + k);
      if (k < left && (b.probe & 4) && stage[wave][k] == 12345.0) dst[k] = 0.0;  // probe: no stores
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// entries of constrained rows: out = C^T v (condensation(), type 2: the
// normal component eliminated; types 1 / 3: zero rows)
__global__ __launch_bounds__(kTB) void k_btk_con(BtkDev b, const NodeConstraint* __restrict__ vcon,
                                                 double* __restrict__ Bt) {
  extern __shared__ __attribute__((aligned(16))) double sq[];
  int* skind = reinterpret_cast<int*>(sq + 12 * b.n_layers);
  btk_stage(b, sq, skind);
  __syncthreads();
  const int i = int(blockIdx.x) * kTB + int(threadIdx.x);
  if (i >= b.n_conent) return;
  const long e = b.con_entry[i];
  double v[3];
  btk_value(b, skind, sq, b.code[e], v);
  const NodeConstraint nc = vcon[b.con_row[i]];
  double C[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int s = 0; s < 3; ++s) C[r][s] = 0.0;
  if (nc.type == 0) {
    C[0][0] = C[1][1] = C[2][2] = 1.0;
  } else if (nc.type == 2) {
#pragma unroll
    for (int d = 0; d < 3; ++d)
      if (d != nc.k) {
        C[d][d] = 1.0;
        C[nc.k][d] = nc.w[d];
      }
  }
  double* dst = Bt + 3 * e;
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) dst[jj] = C[0][jj] * v[0] + C[1][jj] * v[1] + C[2][jj] * v[2];
}

}  // namespace

void btk_assemble(const BtkDev& b, long nnz, const NodeConstraint* vcon, double* Bt,
                  hipStream_t s) {
  const size_t lds = sizeof(double) * 12 * size_t(b.n_layers) + sizeof(int) * size_t(b.n_layers);
  hipLaunchKernelGGL(k_btk_lateral, dim3((b.n_kinds * b.n_pairs + kTB - 1) / kTB), dim3(kTB), 0, s,
                     b);
  hipLaunchKernelGGL(k_btk_entries, dim3(unsigned((nnz + long(kPT) * kTB - 1) / (long(kPT) * kTB))),
                     dim3(kTB), lds, s, b, nnz, Bt);
  if (b.n_conent > 0)
    hipLaunchKernelGGL(k_btk_con, dim3((b.n_conent + kTB - 1) / kTB), dim3(kTB), lds, s, b, vcon,
                       Bt);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
