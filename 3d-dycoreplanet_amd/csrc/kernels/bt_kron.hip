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
//   k_btk_entries  one workgroup per kBtkPT x 256 consecutive B^T entries:
//                  the block's distinct lateral records (kind, pair; ~160 of
//                  them per 1024 entries at r=5, listed at upload) staged from
//                  A into LDS with coalesced loads, then per entry the one or
//                  two layer terms from LDS, written once (no zero fill, no
//                  colouring, no atomics) through an LDS stage so each store
//                  instruction writes 512 contiguous bytes,
//                  An entry of a constrained row (no-normal-flux node) is
//                  condensed with the row's constraint C^T before its store
//                  (the block's constraints staged in LDS beside the records).
// (Reading A per entry from L2 instead -- 3 16-byte loads per term at 64
// scattered lines per wave instruction -- cost 150 of the kernel's 270 us.)
#include <hip/hip_runtime.h>

#include "../device.h"

namespace dcp {
namespace {

constexpr int kTB = kBtkTB;
constexpr int kPT = kBtkPT;  // entries per thread

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

// The one or two layer terms of an entry (node level lambda, l - lambda / 2 + 1
// = dl), records r0 / r1 of terms 0 / 1:
//   lambda odd         term 0: layer m, c 1, k dl - 1
//   dl = 0             term 0: layer m - 1, c 2, k 0          (m >= 1)
//   dl = 2             term 0: layer m, c 0, k 1
//   dl = 1             term 0: layer m - 1, c 2, k 1 (m >= 1); term 1: layer m, c 0, k 0 (m < NL)
// Branch-free (the lanes of a wave hold every case; as branches each case
// took its own pass of LDS reads): both terms always, an absent one with
// factors q = 0, which leaves v bitwise as without it (v - (A 0 + A 0) = v).
__device__ __forceinline__ bool btk_terms(int n_layers, const double* sq, int lam, int dl,
                                          const double2* srec, int s0, int s1, double v[3]) {
  const int m = lam >> 1;
  const bool odd = lam & 1;
  const int L0 = odd || dl == 2 ? m : m - 1;
  const int c0 = odd ? 1 : (dl == 2 ? 0 : 2);
  const int k0 = odd ? dl - 1 : (dl == 0 ? 0 : 1);
  const bool p0 = L0 >= 0;
  const bool p1 = !odd && dl == 1 && m < n_layers;
  const int i0 = 12 * (p0 ? L0 : 0) + 4 * c0 + 2 * k0, i1 = 12 * (p1 ? m : 0);
  const double2 Q0 = *reinterpret_cast<const double2*>(sq + i0);
  const double2 Q1 = *reinterpret_cast<const double2*>(sq + i1);
  const double q01a = p0 ? Q0.x : 0.0, q2a = p0 ? Q0.y : 0.0;
  const double q01b = p1 ? Q1.x : 0.0, q2b = p1 ? Q1.y : 0.0;
  // an absent term's slot may hold a constrained-row index: read record 0
  const double2* r0 = srec + 3 * (p0 ? s0 : 0);
  const double2* r1 = srec + 3 * (p1 ? s1 : 0);
  const double2 A0 = r0[0], A1 = r0[1], A2 = r0[2];
  const double2 B0 = r1[0], B1 = r1[1], B2 = r1[2];
  v[0] = 0.0 - (A0.x * q01a + A1.y * q2a);
  v[1] = 0.0 - (A0.y * q01a + A2.x * q2a);
  v[2] = 0.0 - (A1.x * q01a + A2.y * q2a);
  v[0] -= B0.x * q01b + B1.y * q2b;
  v[1] -= B0.y * q01b + B2.x * q2b;
  v[2] -= B1.x * q01b + B2.y * q2b;
  return p0;
}

// an entry of a constrained row: C^T v (condensation(); type 2: the normal
// component k eliminated, C[d][d] = 1 and C[k][d] = w[d] for d != k; types 1 /
// 3: zero rows), the sums in the order of the former k_btk_con
__device__ __forceinline__ void btk_condense(const NodeConstraint& nc, double v[3]) {
  double C[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) C[r][c] = 0.0;
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
  double o[3];
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) o[jj] = C[0][jj] * v[0] + C[1][jj] * v[1] + C[2][jj] * v[2];
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) v[jj] = o[jj];
}

// The block's records are staged into LDS first. The 64 entries of a wave
// (per u) are 192 consecutive doubles of B^T: staged in LDS so each store
// instruction writes 512 contiguous bytes (every lane storing its own 24 bytes
// instead: 392 against 382 us per assembly, profiles/r06/r06al_direct_store.log).
// Entries of constrained rows are condensed before the store.
__global__ __launch_bounds__(kTB) void k_btk_entries(BtkDev b, long nnz,
                                                     const NodeConstraint* __restrict__ vcon,
                                                     double* __restrict__ Bt) {
  extern __shared__ __attribute__((aligned(16))) double sq[];
  double2* srec = reinterpret_cast<double2*>(sq + 12 * b.n_layers);
  __shared__ double stage[kTB / 64][192];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int blk = xcd_block(int(blockIdx.x), int(gridDim.x));
  const long base = long(blk) * kBtkBlock + threadIdx.x;
  // the block's records into LDS, 3 double2 each, consecutive threads on
  // consecutive double2 (coalesced, the records are sorted): every global
  // load issued up front and unpredicated (indices clamped; predicated loads
  // each got a wait of their own), so the staging costs two dependent
  // latencies (record id, record), not two per trip. Measured at r=5
  // (profiles/r06/r06ae_btk_staging_variants.log): a loop over the doubles 384 us per
  // assembly, this 370 us, a thread per record (48-byte strided loads) 532 us.
  const int r0 = b.blk_ptr[blk], nr = b.blk_ptr[blk + 1] - r0;  // nr >= 1
  const double2* A2 = reinterpret_cast<const double2*>(b.A);
  constexpr int kU = 4;  // 4 kTB double2 = 341 records without the loop below
  int rid[kU];
#pragma unroll
  for (int q = 0; q < kU; ++q) rid[q] = b.blk_rec[r0 + min((int(threadIdx.x) + q * kTB) / 3, nr - 1)];
  uint32_t code[kPT];
#pragma unroll
  for (int u = 0; u < kPT; ++u)
    code[u] = __builtin_nontemporal_load(b.code + min(base + long(u) * kTB, nnz - 1));
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
  for (int i = threadIdx.x + kU * kTB; i < 3 * nr; i += kTB) {  // blocks of > 341 records
    const int j = i / 3;
    srec[i] = A2[3 * size_t(b.blk_rec[r0 + j]) + (i - 3 * j)];
  }
  // the block's constrained rows (k_btk_con folded in: 11 us at r=5)
  NodeConstraint* scon = reinterpret_cast<NodeConstraint*>(srec + 3 * size_t(b.max_rec));
  {
    const int c0 = b.blk_cptr[blk], nc = b.blk_cptr[blk + 1] - c0;
    for (int i = threadIdx.x; i < nc; i += kTB) scon[i] = vcon[b.blk_crow[c0 + i]];
  }
  for (int i = threadIdx.x; i < 12 * b.n_layers; i += kTB)
    sq[i] = b.Q[12 * size_t(b.ord2lay[i / 12]) + i % 12];
  __syncthreads();
  // per u: the entry from LDS, then straight through the stage to the stores
  // (all kPT entries first held 8 x 12 double2 of records: 252 VGPRs)
#pragma unroll
  for (int u = 0; u < kPT; ++u) {
    const uint32_t cu = code[u];
    const int s0 = int(cu & 1023u), s1 = int((cu >> 10) & 1023u);
    double v[3];
    const bool p0 = btk_terms(b.n_layers, sq, int((cu >> 20) & 0xFFu), int((cu >> 28) & 3u), srec,
                              s0, s1, v);
    if ((cu >> 30) & 1u) btk_condense(scon[p0 ? s1 : s0], v);
    stage[wave][3 * lane] = v[0];
    stage[wave][3 * lane + 1] = v[1];
    stage[wave][3 * lane + 2] = v[2];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const long e0 = base - lane + long(u) * kTB;  // the wave's first entry
    const long left = 3 * (nnz - e0);             // doubles of B^T left from there
    double* dst = Bt + 3 * e0;
    // the three LDS reads before the stores: one wait, not one per store
    double o[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) o[r] = stage[wave][lane + 64 * r];
    if (left >= 192) {
#pragma unroll
      for (int r = 0; r < 3; ++r) __builtin_nontemporal_store(o[r], dst + lane + 64 * r);
    } else {
#pragma unroll
      for (int r = 0; r < 3; ++r)
        if (lane + 64 * r < left) __builtin_nontemporal_store(o[r], dst + lane + 64 * r);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

}  // namespace

void btk_assemble(const BtkDev& b, long nnz, const NodeConstraint* vcon, double* Bt,
                  hipStream_t s) {
  const size_t lds_e = sizeof(double) * 12 * size_t(b.n_layers) + 48 * size_t(b.max_rec) +
                       sizeof(NodeConstraint) * size_t(b.max_con);
  hipLaunchKernelGGL(k_btk_lateral, dim3((b.n_kinds * b.n_pairs + kTB - 1) / kTB), dim3(kTB), 0, s,
                     b);
  hipLaunchKernelGGL(k_btk_entries, dim3(unsigned((nnz + kBtkBlock - 1) / kBtkBlock)), dim3(kTB),
                     lds_e, s, b, nnz, vcon, Bt);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
