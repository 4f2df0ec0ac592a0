// Sparse operator applies and Krylov BLAS-1 for CDNA4 (gfx950), FP64.
//
// Replaces the Trilinos/Epetra work under the reference's solvers
// (boussinesq_model.tpp:1131-1245, 1417-1476; block_schur_preconditioner.hpp;
// schur_complement.hpp): CSR SpMV of the nse_matrix blocks, Ifpack point
// Jacobi, dot / add_and_dot / norms of deal.II's Krylov solvers.
//
// SpMV: block-CSR with RxC blocks; a group of G lanes (G | 64) owns one block
// row, lanes stride over the row's blocks (contiguous RxC*8-byte loads),
// shuffles reduce the R partial sums in a fixed order (deterministic).
// Reductions: fixed-shape two-pass (kReduceBlocks partials, then one block),
// so every dot product is bitwise reproducible run to run.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../comm.h"
#include "../device.h"
#include "granule.h"
#include "resident.h"

namespace dcp {
namespace {

constexpr int kBlock = 256;

template <int R, int C, int G>
__global__ __launch_bounds__(kBlock) void k_spmv_bsr(int rows, const int32_t* __restrict__ ptr,
                                                     const int32_t* __restrict__ col,
                                                     const double* __restrict__ val,
                                                     const double* __restrict__ x,
                                                     double* __restrict__ y, int add) {
  const int lane = threadIdx.x % G;
  const long row = (long(blockIdx.x) * kBlock + threadIdx.x) / G;
  if (row >= rows) return;  // whole group leaves together
  double acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = 0.0;
  const int e = ptr[row + 1];
  for (int k = ptr[row] + lane; k < e; k += G) {
    const size_t c = size_t(col[k]);
    const double* v = val + size_t(k) * (R * C);
    double xv[C];
#pragma unroll
    for (int j = 0; j < C; ++j) xv[j] = x[c * C + j];
#pragma unroll
    for (int i = 0; i < R; ++i)
#pragma unroll
      for (int j = 0; j < C; ++j) acc[i] += v[i * C + j] * xv[j];
  }
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1)
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] += __shfl_xor(acc[i], off, G);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      double* yp = y + size_t(row) * R + i;
      *yp = add ? *yp + acc[i] : acc[i];
    }
  }
}

template <int R, int C, int G>
void spmv(int rows, const int32_t* ptr, const int32_t* col, const double* val, const double* x,
          double* y, bool add, hipStream_t s) {
  if (rows <= 0) return;
  const long threads = long(rows) * G;
  const int grid = int((threads + kBlock - 1) / kBlock);
  hipLaunchKernelGGL((k_spmv_bsr<R, C, G>), dim3(grid), dim3(kBlock), 0, s, rows, ptr, col, val, x,
                     y, add ? 1 : 0);
  DCP_HIP_CHECK(hipGetLastError());
}

// position of the i-th owned entry of a two-segment vector (device.h Seg)
__device__ inline long seg_pos(const Seg& g, long i) {
  return i < g.n1 ? i : (i < g.n12 ? g.off2 + (i - g.n1) : g.off3 + (i - g.n12));
}

__device__ inline double block_sum(double v, double* sm) {
  // wave reduce then LDS across the 4 waves; fixed order
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) sm[w] = v;
  __syncthreads();
  double r = 0;
  if (threadIdx.x == 0) r = sm[0] + sm[1] + sm[2] + sm[3];
  return r;
}

__global__ __launch_bounds__(kBlock) void k_dot_partial(Seg g, const double* __restrict__ a,
                                                        const double* __restrict__ b,
                                                        double* __restrict__ partials) {
  __shared__ double sm[4];
  double s = 0;
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < g.n; i += long(gridDim.x) * kBlock) {
    const long j = seg_pos(g, i);
    s += a[j] * b[j];
  }
  const double r = block_sum(s, sm);
  if (threadIdx.x == 0) partials[blockIdx.x] = r;
}

// v += c x ; partial dot(v, w) (w may alias v)
__global__ __launch_bounds__(kBlock) void k_add_and_dot(Seg g, double* v, DScal c,
                                                        const double* __restrict__ x,
                                                        const double* w, double* partials) {
  __shared__ double sm[4];
  const double cf = c.p ? c.m * (*c.p) : c.m;
  double s = 0;
  for (long k = long(blockIdx.x) * kBlock + threadIdx.x; k < g.n; k += long(gridDim.x) * kBlock) {
    const long i = seg_pos(g, k);
    const double nv = v[i] + cf * x[i];
    v[i] = nv;
    s += nv * (w == v ? nv : w[i]);
  }
  const double r = block_sum(s, sm);
  if (threadIdx.x == 0) partials[blockIdx.x] = r;
}

// Chained Gram-Schmidt step without a separate reduction launch: every block
// first sums the previous step's nb_prev partials in the same fixed order (so
// all blocks agree bitwise), block 0 stores that coefficient, then
// v += mult * coef * x and the partial dot(v, w) of this block is written.
// The block's first kChainPrefetch elements of v, x, w are loaded before the
// partials, so the two dependent memory latencies overlap.
constexpr int kChainPrefetch = 4;
__global__ __launch_bounds__(kBlock) void k_chain_add_and_dot(
    Seg g, double* v, const double* __restrict__ prev, int nb_prev, double mult,
    const double* __restrict__ x, const double* w, double* __restrict__ partials,
    double* coef_store, const double* __restrict__ prev2, double* store2,
    double* partials_host) {
  __shared__ double sm[4];
  __shared__ double coef_sh;
  const bool self = (w == v);
  const long stride = long(gridDim.x) * kBlock;
  const long i0 = long(blockIdx.x) * kBlock + threadIdx.x;
  double rv[kChainPrefetch], rx[kChainPrefetch], rw[kChainPrefetch];
#pragma unroll
  for (int e = 0; e < kChainPrefetch; ++e) {
    const long k = i0 + e * stride;
    const long i = seg_pos(g, k);
    rv[e] = rx[e] = rw[e] = 0.0;
    if (k < g.n) {
      rv[e] = v[i];
      rx[e] = x[i];
      if (!self) rw[e] = w[i];
    }
  }
  double s = 0;
  for (int i = threadIdx.x; i < nb_prev; i += kBlock) s += prev[i];
  const double tot = block_sum(s, sm);
  if (threadIdx.x == 0) {
    coef_sh = tot;
    if (blockIdx.x == 0) *coef_store = tot;
  }
  __syncthreads();
  if (prev2) {
    double s2 = 0;
    for (int i = threadIdx.x; i < nb_prev; i += kBlock) s2 += prev2[i];
    const double t2 = block_sum(s2, sm);
    if (threadIdx.x == 0 && blockIdx.x == 0) *store2 = t2;
    __syncthreads();
  }
  const double cf = mult * coef_sh;
  double d = 0;
#pragma unroll
  for (int e = 0; e < kChainPrefetch; ++e) {
    const long k = i0 + e * stride;
    if (k < g.n) {
      const long i = seg_pos(g, k);
      const double nv = rv[e] + cf * rx[e];
      v[i] = nv;
      d += nv * (self ? nv : rw[e]);
    }
  }
  for (long k = i0 + kChainPrefetch * stride; k < g.n; k += stride) {
    const long i = seg_pos(g, k);
    const double nv = v[i] + cf * x[i];
    v[i] = nv;
    d += nv * (self ? nv : w[i]);
  }
  const double r = block_sum(d, sm);
  if (threadIdx.x == 0) {
    partials[blockIdx.x] = r;
    if (partials_host) partials_host[blockIdx.x] = r;
  }
}

// ---------------------------------------------------------------------------
// Whole modified-Gram-Schmidt chain in one launch (one GPU). The grid is the
// chain's nb workgroups, all resident (nb <= the CU count, checked by the
// launcher), and every workgroup keeps its <= kMgsElems entries of w in
// registers for the whole chain. A step's nb block sums are handed to every
// workgroup as 16-byte granules {sum, tag ^ mix(sum)} written by one `sc1`
// store and polled with `sc1` loads (agent-coherent, no fences; the value
// checksum in the tag half rejects a torn read); the tag = launch sequence *
// 64 + step is never reused, so the granule array needs no clearing. Every
// workgroup then forms the coefficient from the nb sums in exactly the order
// k_chain_add_and_dot uses, so the chain is bitwise the per-step one.
// Spins are bounded (an unbounded wait would hang the device): a workgroup
// that gives up writes 1 to *err and the host throws.
#ifndef DCP_MGS_ELEMS
#define DCP_MGS_ELEMS 8
#endif
constexpr int kMgsElems = DCP_MGS_ELEMS;
// h_0 = w.V[0] (from prev: nb_prev partials, e.g. the fused SpMV's; or, with
// prev == null, computed here), then for i = 1..d-1:
//   w -= h_{i-1} V[i-1];  h_i = w.V[i]
// and finally w -= h_{d-1} V[d-1]; partials of |w|^2. Coefficients -> coef
// (block 0), optional fixed-order sum of prev2 -> *store2 (block 0), the final
// partials -> partials (+ partials_host), w written back once at the end.
__global__ __launch_bounds__(kBlock) void k_mgs_chain(
    Seg g, double* w, ChainVecs V, int d, const double* __restrict__ prev, int nb_prev,
    const double* __restrict__ prev2, double* store2, double* coef, double* partials,
    double* partials_host, double* gran, unsigned long long seq, double* err) {
  __shared__ double sm[4];
  __shared__ double coef_sh;
  const int nb = gridDim.x;
  const long stride = long(nb) * kBlock;
  const long i0 = long(blockIdx.x) * kBlock + threadIdx.x;
  // rx: the vector subtracted at step i (V[i-1]), ry: the one dotted (V[i]),
  // rz: V[i+1], loaded before step i's hand-off wait so it lands meanwhile
  double rw[kMgsElems], rx[kMgsElems], ry[kMgsElems], rz[kMgsElems];
  long pos[kMgsElems];
#pragma unroll
  for (int e = 0; e < kMgsElems; ++e) {
    const long k = i0 + e * stride;
    pos[e] = k < g.n ? seg_pos(g, k) : -1;
    rw[e] = pos[e] >= 0 ? w[pos[e]] : 0.0;
    rx[e] = pos[e] >= 0 ? V.v[0][pos[e]] : 0.0;
    ry[e] = pos[e] >= 0 && d > 1 ? V.v[1][pos[e]] : 0.0;
  }
  if (prev) {
    double s = 0;
    for (int i = threadIdx.x; i < nb_prev; i += kBlock) s += prev[i];
    const double tot = block_sum(s, sm);
    if (threadIdx.x == 0) {
      coef_sh = tot;
      if (blockIdx.x == 0) coef[0] = tot;
    }
  } else {
    // h_0 = w.V0 here: the same per-thread order as k_dot_partial's grid stride
    double p0 = 0;
#pragma unroll
    for (int e = 0; e < kMgsElems; ++e)
      if (pos[e] >= 0) p0 += rw[e] * rx[e];
    const double r0 = block_sum(p0, sm);
    if (threadIdx.x == 0) granule_store(gran + 2 * size_t(blockIdx.x), r0, seq * 64);
    if (threadIdx.x < 64) {
      const double tot = granule_coef(gran, nb, seq * 64, err);
      if (threadIdx.x == 0) {
        coef_sh = tot;
        if (blockIdx.x == 0) coef[0] = tot;
      }
    }
  }
  __syncthreads();
  if (prev2) {
    double s2 = 0;
    for (int i = threadIdx.x; i < nb_prev; i += kBlock) s2 += prev2[i];
    const double t2 = block_sum(s2, sm);
    if (threadIdx.x == 0 && blockIdx.x == 0) *store2 = t2;
    __syncthreads();
  }
  for (int i = 1; i <= d; ++i) {
    const bool last = i == d;
    const double cf = -1.0 * coef_sh;
    double dd = 0;
#pragma unroll
    for (int e = 0; e < kMgsElems; ++e) {
      if (pos[e] >= 0) {
        const double nv = rw[e] + cf * rx[e];
        rw[e] = nv;
        dd += nv * (last ? nv : ry[e]);
      }
    }
    const double r = block_sum(dd, sm);
    if (last) {
      if (threadIdx.x == 0) {
        partials[blockIdx.x] = r;
        if (partials_host) partials_host[blockIdx.x] = r;
      }
      break;
    }
    const unsigned long long tag = seq * 64 + unsigned(i);
    double* gi = gran + 2 * size_t(i) * kChainMaxBlocks;
    if (threadIdx.x == 0) granule_store(gi + 2 * size_t(blockIdx.x), r, tag);
    if (i + 1 < d) {
#pragma unroll
      for (int e = 0; e < kMgsElems; ++e) rz[e] = pos[e] >= 0 ? V.v[i + 1][pos[e]] : 0.0;
    }
#pragma unroll
    for (int e = 0; e < kMgsElems; ++e) {
      rx[e] = ry[e];
      ry[e] = rz[e];
    }
    if (threadIdx.x < 64) {
      const double tot = granule_coef(gi, nb, tag, err);
      if (threadIdx.x == 0) {
        coef_sh = tot;
        if (blockIdx.x == 0) coef[i] = tot;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int e = 0; e < kMgsElems; ++e)
    if (pos[e] >= 0) w[pos[e]] = rw[e];
}

// SELL-64 SpMV (see device.h). One 256-thread workgroup per slice: lane i of
// every wave owns row 64s+i; wave j sums the column pairs j, j+4, j+8, ... of
// the slice (round robin; 4 waves per slice keep enough loads in flight: one
// wave per slice leaves ~3 waves per SIMD on a 2e5-row matrix, latency-bound),
// then wave 0 adds the 4 partial sums in order (fixed summation order). A
// row's sum depends only on its entries and their order, not on the slice's
// width (padding pairs add exact zeros), so a row gives the same bits in any
// slice: the matrix powers of the multi-GPU s-step basis evaluate ghost rows
// on a rank other than their owner (solver.cpp).
// Four column pairs per iteration, all value / column loads issued before the
// gathers; r=5 inner probe (tools/inner_probe.py, rocprofv3): 39.65 -> 38.50 us
// per S apply against the two-pair loop; DCP_SELL_NT (nontemporal values)
// 43.3 us.
#ifndef DCP_SELL_NT
#define DCP_SELL_NT 0
#endif
typedef double sell_d2v __attribute__((ext_vector_type(2)));
// DCP_SELL_NT (timing variant): the value stream as nontemporal loads, so it
// does not evict the gathered x from L2
__device__ inline double2 sell_ld(const double2* p) {
  if (DCP_SELL_NT) {
    const sell_d2v t = __builtin_nontemporal_load(reinterpret_cast<const sell_d2v*>(p));
    return double2{t.x, t.y};
  }
  return *p;
}
#define SELL_LD(p) sell_ld(p)
// CM: column mode, 0 = 32-bit columns, 1 = 16-bit offsets, 2 = structured
// (SellView::nbr: only values stream from HBM, the column of entry k = nd j + d
// comes from the level of the row and the L2-resident neighbour table)
struct SlotPos {  // entry k = nd j + d of a structured row (nd levels in reach)
  int j, d, nd;
  __device__ void step(int n) {  // k += n, 0 <= n <= 8
    // nd >= 3 and d <= 6 before a step, so at most 3 wraps: three selects
    // (a while loop here put a branch between the slice's address
    // computations and cost 0.7 us per S apply, profiles/r05/r05ae_*)
    d += n;
#pragma unroll
    for (int w = 0; w < 3; ++w) {
      const bool wr = d >= nd;
      d = wr ? d - nd : d;
      j = wr ? j + 1 : j;
    }
  }
};
template <bool EPI, int CM>
__global__ __launch_bounds__(kBlock) void k_sell_spmv(SellView m, const double* __restrict__ x,
                                                      double cf, double* xs,
                                                      double* __restrict__ y,
                                                      const double* v0,
                                                      double* __restrict__ part0,
                                                      double* __restrict__ part1,
                                                      const double* __restrict__ cf_dev,
                                                      const int* __restrict__ status,
                                                      double theta = 0.0, double sscale = 1.0,
                                                      const double* __restrict__ bsub = nullptr) {
  __shared__ double quarter[3][64];
  if (status && *status) return;  // device-resident GMRES cycle already stopped
  if (cf_dev) cf = *cf_dev;
  const int rows = m.rows;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const long sl = blockIdx.x;
  const long row = sl * 64 + lane;
  if (sl * 64 >= rows) {
    // padding workgroup of the common partial length (several GPUs): the
    // all-reduced partial arrays must hold zeros past this rank's slices
    if (EPI && threadIdx.x == 0) {
      if (part0) part0[sl] = 0.0;
      if (part1) part1[sl] = 0.0;
    }
    return;
  }
  const int64_t b = m.off[sl];
  const int np = int((m.off[sl + 1] - b) >> 7);  // column pairs of the slice
  const double2* vp = reinterpret_cast<const double2*>(m.val + b) + 64 * wave + lane;
  double acc = 0.0;
  int k = wave;
  if (CM == 2) {
    const int nc = m.nc, nl = m.nl;
    const long rr = row < rows ? row : rows - 1;  // lanes past the end: any valid row
    const int l = int(rr / nc), cc = int(rr - long(l) * nc);
    // levels l + dlo .. l + dlo + nd - 1 within [l - 2, l + 2] and the mesh
    const int dlo = l < 2 ? -l : -2;
    const int nd = min(l + 2, nl - 1) - (l + dlo) + 1;
    const int32_t* nb = m.nbr + cc;
    const int jlast = m.nj - 1;  // padding entries (value 0): the spare row, own lateral
    auto xat = [&](SlotPos p) {
      return x[(l + dlo + p.d) * nc + nb[min(p.j, jlast) * nc]] * cf;
    };
    SlotPos p0{0, 2 * k, nd};
    p0.step(0);
    for (; k + 12 < np; k += 16, vp += 1024) {
      // pairs k, k + 4, k + 8, k + 12: slots 2k .. 2k + 1 and 8, 16, 24 on
      SlotPos q[8];
      q[0] = p0;
#pragma unroll
      for (int i = 1; i < 8; ++i) {
        q[i] = q[i - 1];
        q[i].step((i & 1) ? 1 : 7);
      }
      const double2 a0 = SELL_LD(vp), a1 = SELL_LD(vp + 256), a2 = SELL_LD(vp + 512),
                    a3 = SELL_LD(vp + 768);
      const double x0 = xat(q[0]), x1 = xat(q[1]), x2 = xat(q[2]), x3 = xat(q[3]);
      const double x4 = xat(q[4]), x5 = xat(q[5]), x6 = xat(q[6]), x7 = xat(q[7]);
      acc += a0.x * x0;
      acc += a0.y * x1;
      acc += a1.x * x2;
      acc += a1.y * x3;
      acc += a2.x * x4;
      acc += a2.y * x5;
      acc += a3.x * x6;
      acc += a3.y * x7;
      p0 = q[7];
      p0.step(7);
    }
    for (; k < np; k += 4, vp += 256) {
      SlotPos p1 = p0;
      p1.step(1);
      const double2 a0 = SELL_LD(vp);
      acc += a0.x * xat(p0);
      acc += a0.y * xat(p1);
      p0.step(8);
    }
  } else if (CM == 1) {
    const int cb = m.base[sl];
    const ushort2* cp = reinterpret_cast<const ushort2*>(m.col16 + b) + 64 * wave + lane;
    for (; k + 12 < np; k += 16, cp += 1024, vp += 1024) {
      // pairs k, k + 4, k + 8, k + 12: all loads before the gathers
      const ushort2 c0 = cp[0], c1 = cp[256], c2 = cp[512], c3 = cp[768];
      const double2 a0 = SELL_LD(vp), a1 = SELL_LD(vp + 256), a2 = SELL_LD(vp + 512),
                    a3 = SELL_LD(vp + 768);
      const double x0 = x[cb + c0.x] * cf, x1 = x[cb + c0.y] * cf;
      const double x2 = x[cb + c1.x] * cf, x3 = x[cb + c1.y] * cf;
      const double x4 = x[cb + c2.x] * cf, x5 = x[cb + c2.y] * cf;
      const double x6 = x[cb + c3.x] * cf, x7 = x[cb + c3.y] * cf;
      acc += a0.x * x0;
      acc += a0.y * x1;
      acc += a1.x * x2;
      acc += a1.y * x3;
      acc += a2.x * x4;
      acc += a2.y * x5;
      acc += a3.x * x6;
      acc += a3.y * x7;
    }
    for (; k < np; k += 4, cp += 256, vp += 256) {
      const ushort2 c0 = cp[0];
      const double2 a0 = SELL_LD(vp);
      acc += a0.x * (x[cb + c0.x] * cf);
      acc += a0.y * (x[cb + c0.y] * cf);
    }
  } else {
    const int2* cp = reinterpret_cast<const int2*>(m.col + b) + 64 * wave + lane;
    for (; k + 12 < np; k += 16, cp += 1024, vp += 1024) {
      const int2 c0 = cp[0], c1 = cp[256], c2 = cp[512], c3 = cp[768];
      const double2 a0 = SELL_LD(vp), a1 = SELL_LD(vp + 256), a2 = SELL_LD(vp + 512),
                    a3 = SELL_LD(vp + 768);
      const double x0 = x[c0.x] * cf, x1 = x[c0.y] * cf, x2 = x[c1.x] * cf, x3 = x[c1.y] * cf;
      const double x4 = x[c2.x] * cf, x5 = x[c2.y] * cf, x6 = x[c3.x] * cf, x7 = x[c3.y] * cf;
      acc += a0.x * x0;
      acc += a0.y * x1;
      acc += a1.x * x2;
      acc += a1.y * x3;
      acc += a2.x * x4;
      acc += a2.y * x5;
      acc += a3.x * x6;
      acc += a3.y * x7;
    }
    for (; k < np; k += 4, cp += 256, vp += 256) {
      const int2 c0 = cp[0];
      const double2 a0 = SELL_LD(vp);
      acc += a0.x * (x[c0.x] * cf);
      acc += a0.y * (x[c0.y] * cf);
    }
  }
  if (wave > 0) quarter[wave - 1][lane] = acc;
  __syncthreads();
  if (wave > 0) return;
  acc += quarter[0][lane];
  acc += quarter[1][lane];
  acc += quarter[2][lane];
  // the vector entry of the row (m.rowmap: rows kept apart from the vector
  // order, the ghost rows of the matrix powers)
  const long orow = (m.rowmap && row < rows) ? long(m.rowmap[row]) : row;
  if (!EPI) {
    if (row < rows) y[orow] = acc;
    return;
  }
  double d0 = 0, d1 = 0;
  if (row < rows) {
    const double xv = x[orow] * cf;
    // s-step Newton basis: y = (S x - theta x) / sigma (sscale = 1 / sigma)
    if (theta != 0.0 || sscale != 1.0) acc = (acc - theta * xv) * sscale;
    // GMRES restart head: the residual y = b - S x
    if (bsub) acc = bsub[orow] - acc;
    y[orow] = acc;
    if (xs) xs[orow] = xv;
    if (part0) d0 = acc * (v0 == xs ? xv : v0[orow]);  // v0 == xs: the first Arnoldi vector
    if (part1) d1 = acc * acc;
  }
  if (!part0 && !part1) return;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    d0 += __shfl_xor(d0, o, 64);
    d1 += __shfl_xor(d1, o, 64);
  }
  if (lane == 0) {
    if (part0) part0[sl] = d0;
    if (part1) part1[sl] = d1;
  }
}

__global__ __launch_bounds__(kBlock) void k_reduce_final(int nb, const double* __restrict__ partials,
                                                         double* out) {
  __shared__ double sm[4];
  double s = 0;
  for (int i = threadIdx.x; i < nb; i += kBlock) s += partials[i];
  const double r = block_sum(s, sm);
  if (threadIdx.x == 0) *out = r;
}

__global__ void k_axpy(int n, DScal c, const double* __restrict__ x, double* __restrict__ y) {
  const double cf = c.p ? c.m * (*c.p) : c.m;
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] += cf * x[i];
}
__global__ void k_scale(int n, DScal c, double* x) {
  const double cf = c.p ? c.m * (*c.p) : c.m;
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    x[i] *= cf;
}
__global__ void k_sadd(int n, double s, double a, const double* __restrict__ x, double* y) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] = s * y[i] + a * x[i];
}
__global__ void k_copy(int n, const double* __restrict__ x, double* __restrict__ y) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] = x[i];
}
__global__ void k_equ(int n, DScal c, const double* __restrict__ x, double* __restrict__ y) {
  const double cf = c.p ? c.m * (*c.p) : c.m;
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] = cf * x[i];
}
__global__ void k_axpby(int n, DScal a, const double* __restrict__ x, DScal b, double* y) {
  const double ca = a.p ? a.m * (*a.p) : a.m;
  const double cb = b.p ? b.m * (*b.p) : b.m;
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] = cb * y[i] + ca * x[i];
}
__global__ void k_scalar_div(const double* num, const double* den, double* out) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *out = *num / *den;
}
__global__ void k_fill(int n, double v, double* y) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] = v;
}
__global__ void k_mul(int n, const double* __restrict__ a, const double* __restrict__ x,
                      double* __restrict__ y) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] = x[i] * a[i];
}
__global__ void k_recip(int n, const double* __restrict__ a, double* __restrict__ y) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] = 1.0 / a[i];
}
__global__ void k_csr_diag_inv(int rows, const int32_t* __restrict__ ptr,
                               const int32_t* __restrict__ col, const double* __restrict__ val,
                               double* __restrict__ inv) {
  for (long r = long(blockIdx.x) * kBlock + threadIdx.x; r < rows; r += long(gridDim.x) * kBlock) {
    int b = ptr[r], e = ptr[r + 1];
    while (b < e) {
      const int m = (b + e) >> 1;
      if (col[m] < r) b = m + 1; else e = m;
    }
    inv[r] = 1.0 / val[b];
  }
}
__global__ void k_lincomb(int n, const double* __restrict__ a, double alpha,
                          const double* __restrict__ b, double* __restrict__ z) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    z[i] = a[i] + alpha * b[i];
}
__global__ void k_multi_axpy(int n, int k, const double* __restrict__ coef,
                             const double* const* __restrict__ X, double* __restrict__ y) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock) {
    double v = y[i];
    for (int j = 0; j < k; ++j) v += coef[j] * X[j][i];
    y[i] = v;
  }
}

__global__ void k_multi_axpy_args(int n, int k, CombineArgs a, double* __restrict__ y) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock) {
    double v = y[i];
    for (int j = 0; j < k; ++j) v += a.c[j] * a.x[j][i];
    y[i] = v;
  }
}

__global__ void k_distribute_velocity(int n, const NodeConstraint* __restrict__ vc, double* u) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock) {
    const NodeConstraint c = vc[i];
    if (c.type == 1) {
      u[3 * i] = u[3 * i + 1] = u[3 * i + 2] = 0.0;
    } else if (c.type == 2) {
      double v = 0;
      for (int d = 0; d < 3; ++d)
        if (d != c.k) v += c.w[d] * u[3 * i + d];
      u[3 * i + c.k] = v;
    }
  }
}

__global__ void k_copy_images(int n, const int32_t* __restrict__ img,
                              const int32_t* __restrict__ master, double* x) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n) x[img[k]] = x[master[k]];
}

__global__ void k_distribute_T(int n, const uint8_t* __restrict__ fixed, const double* __restrict__ bc,
                               double* T) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    if (fixed[i]) T[i] = bc[i];
}

// non-negative doubles order like their bit patterns
__device__ inline void atomic_max_nonneg(double* addr, double v) {
  atomicMax(reinterpret_cast<unsigned long long*>(addr), __double_as_longlong(v));
}

__global__ __launch_bounds__(kBlock) void k_velocity_stats(CellData cd, int n_cells,
                                                           const double* __restrict__ u,
                                                           double* out2) {
  __shared__ double sm[2][4];
  const long c = long(blockIdx.x) * kBlock + threadIdx.x;
  double mx = 0, cfl = 0;
  if (c < n_cells) {
    double cm = 1e-10;  // get_cfl_number initialises the cell max with 1e-10
    for (int n = 0; n < 27; ++n) {
      // the cell's own dof values (a periodic image's, not its partner's)
      const size_t b = 3 * size_t((cd.cell_q2o ? cd.cell_q2o : cd.cell_q2)[27 * c + n]);
      const double v = sqrt(u[b] * u[b] + u[b + 1] * u[b + 1] + u[b + 2] * u[b + 2]);
      mx = fmax(mx, v);
      cm = fmax(cm, v);
    }
    cfl = cm / cd.diameter[c];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    mx = fmax(mx, __shfl_xor(mx, off, 64));
    cfl = fmax(cfl, __shfl_xor(cfl, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    sm[0][threadIdx.x / 64] = mx;
    sm[1][threadIdx.x / 64] = cfl;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomic_max_nonneg(&out2[0], fmax(fmax(sm[0][0], sm[0][1]), fmax(sm[0][2], sm[0][3])));
    atomic_max_nonneg(&out2[1], fmax(fmax(sm[1][0], sm[1][1]), fmax(sm[1][2], sm[1][3])));
  }
}

__global__ __launch_bounds__(kBlock) void k_minmax_partial(int n, const double* __restrict__ x,
                                                           double* partials) {
  __shared__ double sm[2][4];
  double lo = 1.7976931348623157e308, hi = -1.7976931348623157e308;
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock) {
    lo = fmin(lo, x[i]);
    hi = fmax(hi, x[i]);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, off, 64));
    hi = fmax(hi, __shfl_xor(hi, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    sm[0][threadIdx.x / 64] = lo;
    sm[1][threadIdx.x / 64] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    partials[2 * blockIdx.x] = fmin(fmin(sm[0][0], sm[0][1]), fmin(sm[0][2], sm[0][3]));
    partials[2 * blockIdx.x + 1] = fmax(fmax(sm[1][0], sm[1][1]), fmax(sm[1][2], sm[1][3]));
  }
}

__global__ void k_minmax_final(int nb, const double* partials, double* out2) {
  if (threadIdx.x != 0) return;
  double lo = partials[0], hi = partials[1];
  for (int i = 1; i < nb; ++i) {
    lo = fmin(lo, partials[2 * i]);
    hi = fmax(hi, partials[2 * i + 1]);
  }
  out2[0] = lo;
  out2[1] = hi;
}

// rows [r0, r1) x columns [c0, c1) of a CSR matrix: y[r - r0] (+)= sum val x[col - c0]
// (one 16-lane group per row, fixed-order shuffle reduction)
__global__ __launch_bounds__(kBlock) void k_spmv_block(int r0, int r1, int c0, int c1,
                                                       const int32_t* __restrict__ ptr,
                                                       const int32_t* __restrict__ col,
                                                       const double* __restrict__ val,
                                                       const double* __restrict__ x,
                                                       double* __restrict__ y, int add) {
  constexpr int G = 16;
  const int lane = threadIdx.x % G;
  const long row = r0 + (long(blockIdx.x) * kBlock + threadIdx.x) / G;
  if (row >= r1) return;
  double acc = 0;
  for (int k = ptr[row] + lane; k < ptr[row + 1]; k += G) {
    const int c = col[k];
    if (c >= c0 && c < c1) acc += val[k] * x[c - c0];
  }
#pragma unroll
  for (int off = G / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, G);
  if (lane == 0) {
    double* yp = y + (row - r0);
    *yp = add ? *yp + acc : acc;
  }
}
__global__ void k_shift(int n, DScal c, double* y) {
  const double cf = c.p ? c.m * (*c.p) : c.m;
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    y[i] += cf;
}
__global__ void k_zero_fixed(int n, const uint8_t* __restrict__ fixed, double* y) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    if (fixed[i]) y[i] = 0.0;
}

__global__ void k_group_reduce(size_t n, int nbufs, BufTable t, double* __restrict__ out, int mx) {
  for (size_t i = size_t(blockIdx.x) * kBlock + threadIdx.x; i < n; i += size_t(gridDim.x) * kBlock) {
    double v = t.p[0][i];
    for (int r = 1; r < nbufs; ++r) v = mx ? fmax(v, t.p[r][i]) : v + t.p[r][i];
    out[i] = v;
  }
}
__global__ void k_gather(int n, const int32_t* __restrict__ pos, const double* __restrict__ v,
                         double* __restrict__ buf) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    buf[i] = v[pos[i]];
}
__global__ void k_scatter(int n, const int32_t* __restrict__ pos, const double* __restrict__ buf,
                          double* __restrict__ v) {
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock)
    v[pos[i]] = buf[i];
}

inline int grid_for(long n) {
  long g = (n + kBlock - 1) / kBlock;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  return int(g);
}

}  // namespace

void spmv_bsr33(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                const double* x, double* y, bool add, hipStream_t s) {
  spmv<3, 3, 32>(rows, ptr, col, val, x, y, add, s);
}
void spmv_bsr31(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                const double* x, double* y, bool add, hipStream_t s) {
  spmv<3, 1, 8>(rows, ptr, col, val, x, y, add, s);
}
void spmv_bsr13(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                const double* x, double* y, bool add, hipStream_t s) {
  spmv<1, 3, 32>(rows, ptr, col, val, x, y, add, s);
}
void spmv_csr(int rows, const int32_t* ptr, const int32_t* col, const double* val,
              const double* x, double* y, bool add, hipStream_t s) {
  spmv<1, 1, 16>(rows, ptr, col, val, x, y, add, s);
}

void spmv_csr_long(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                   const double* x, double* y, bool add, hipStream_t s) {
  spmv<1, 1, 32>(rows, ptr, col, val, x, y, add, s);
}

void dot(Seg g, const double* a, const double* b, double* partials, double* out, hipStream_t s) {
  dot_partials(g, a, b, partials, s);
  reduce_final(kReduceBlocks, partials, out, s);
}
void dot_partials(Seg g, const double* a, const double* b, double* partials, hipStream_t s) {
  hipLaunchKernelGGL(k_dot_partial, dim3(kReduceBlocks), dim3(kBlock), 0, s, g, a, b, partials);
  DCP_HIP_CHECK(hipGetLastError());
}
void reduce_final(int nb, const double* partials, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_reduce_final, dim3(1), dim3(kBlock), 0, s, nb, partials, out);
  DCP_HIP_CHECK(hipGetLastError());
}

int chain_blocks(int n) {
  // >= 256 workgroups (one per CU) even for the 2e5-long pressure vectors: the
  // chain steps are latency-bound, so width beats the cost of each block
  // re-summing the previous step's nb partials.
#ifndef DCP_CHAIN_MIN_BLOCKS
#define DCP_CHAIN_MIN_BLOCKS 256
#endif
#ifndef DCP_CHAIN_PER_BLOCK
#define DCP_CHAIN_PER_BLOCK 2048
#endif
  int nb = (n + DCP_CHAIN_PER_BLOCK - 1) / DCP_CHAIN_PER_BLOCK;
  nb = ((nb + 63) / 64) * 64;
  return nb < DCP_CHAIN_MIN_BLOCKS ? DCP_CHAIN_MIN_BLOCKS
                                   : (nb > kChainMaxBlocks ? kChainMaxBlocks : nb);
}

void dot_partial(Seg g, const double* a, const double* b, double* partials, int nb, hipStream_t s) {
  hipLaunchKernelGGL(k_dot_partial, dim3(nb), dim3(kBlock), 0, s, g, a, b, partials);
  DCP_HIP_CHECK(hipGetLastError());
}

void chain_add_and_dot(Seg g, double* v, const double* prev, double mult, const double* x,
                       const double* w, double* partials, double* coef_store, int nb,
                       hipStream_t s) {
  chain_add_and_dot_ex(g, v, prev, nb, mult, x, w, partials, coef_store, nb, nullptr, nullptr,
                       nullptr, s);
}

void chain_add_and_dot_ex(Seg g, double* v, const double* prev, int nb_prev, double mult,
                          const double* x, const double* w, double* partials,
                          double* coef_store, int nb, const double* prev2, double* store2,
                          double* partials_host, hipStream_t s) {
  hipLaunchKernelGGL(k_chain_add_and_dot, dim3(nb), dim3(kBlock), 0, s, g, v, prev, nb_prev, mult,
                     x, w, partials, coef_store, prev2, store2, partials_host);
  DCP_HIP_CHECK(hipGetLastError());
}

bool mgs_chain_fits(long n, int nb, int d, int n_cus) {
  return d >= 1 && d < kMgsMaxVecs && nb >= 1 && nb <= n_cus && nb <= kBlock &&
         n <= long(kMgsElems) * nb * kBlock &&
         nb <= resident_capacity(reinterpret_cast<const void*>(&k_mgs_chain), kBlock);
}

void mgs_chain(Seg g, double* w, const ChainVecs& V, int d, const double* prev, int nb_prev,
               const double* prev2, double* store2, double* coef, double* partials,
               double* partials_host, int nb, double* gran, unsigned long long seq, double* err,
               hipStream_t s) {
  launch_resident(k_mgs_chain, nb, kBlock, s, g, w, V, d, prev, nb_prev, prev2, store2, coef,
                  partials, partials_host, gran, seq, err);
}

int sell_fused_blocks(int rows) { return int((long(rows) + 63) / 64); }

namespace {
// the instantiation for the view's column mode
template <bool EPI>
decltype(&k_sell_spmv<EPI, 0>) sell_kernel(const SellView& m) {
  if (m.nbr) return k_sell_spmv<EPI, 2>;
  return m.col16 ? k_sell_spmv<EPI, 1> : k_sell_spmv<EPI, 0>;
}
}  // namespace

void sell_spmv(const SellView& m, const double* x, double cf, double* y, hipStream_t s) {
  if (m.rows <= 0) return;
  const dim3 grid(sell_fused_blocks(m.rows));
  hipLaunchKernelGGL(sell_kernel<false>(m), grid, dim3(kBlock), 0, s, m, x, cf, nullptr, y, nullptr,
                     nullptr, nullptr, nullptr, nullptr, 0.0, 1.0, nullptr);
  DCP_HIP_CHECK(hipGetLastError());
}

void sell_spmv_fused(const SellView& m, const double* x, double cf, double* xs, double* y,
                     const double* v0, double* part0, double* part1, int n_part, hipStream_t s) {
  const int nb = std::max(sell_fused_blocks(m.rows), n_part);
  if (nb <= 0) return;
  hipLaunchKernelGGL(sell_kernel<true>(m), dim3(nb), dim3(kBlock), 0, s, m, x, cf, xs, y, v0,
                     part0, part1, nullptr, nullptr, 0.0, 1.0, nullptr);
  DCP_HIP_CHECK(hipGetLastError());
}

void sell_spmv_step(const SellView& m, const double* x, const double* cf_dev, double* xs,
                    double* y, const int* status, hipStream_t s) {
  if (m.rows <= 0) return;
  const dim3 grid(sell_fused_blocks(m.rows));
  hipLaunchKernelGGL(sell_kernel<true>(m), grid, dim3(kBlock), 0, s, m, x, 1.0, xs, y, nullptr,
                     nullptr, nullptr, cf_dev, status, 0.0, 1.0, nullptr);
  DCP_HIP_CHECK(hipGetLastError());
}

void sell_spmv_shifted(const SellView& m, const double* x, double theta, double sscale, double* y,
                       const int* status, hipStream_t s) {
  if (m.rows <= 0) return;
  const dim3 grid(sell_fused_blocks(m.rows));
  hipLaunchKernelGGL(sell_kernel<true>(m), grid, dim3(kBlock), 0, s, m, x, 1.0, nullptr, y,
                     nullptr, nullptr, nullptr, nullptr, status, theta, sscale, nullptr);
  DCP_HIP_CHECK(hipGetLastError());
}

void sell_spmv_residual(const SellView& m, const double* x, const double* b, double* y,
                        double* part, hipStream_t s) {
  if (m.rows <= 0) return;
  const dim3 grid(sell_fused_blocks(m.rows));
  hipLaunchKernelGGL(sell_kernel<true>(m), grid, dim3(kBlock), 0, s, m, x, 1.0, nullptr, y,
                     nullptr, nullptr, part, nullptr, nullptr, 0.0, 1.0, b);
  DCP_HIP_CHECK(hipGetLastError());
}

namespace {
// Gershgorin bound of the stored S: max over rows of sum |s_ij| (padding
// entries are zero), as a non-negative double through its bit pattern
__global__ __launch_bounds__(64) void k_sell_rowabs(SellView m, double* out) {
  const long sl = blockIdx.x;
  const long row = sl * 64 + threadIdx.x;
  const int64_t b = m.off[sl];
  const int np = int((m.off[sl + 1] - b) >> 7);
  const double2* vp = reinterpret_cast<const double2*>(m.val + b) + threadIdx.x;
  double s = 0.0;
  for (int k = 0; k < np; ++k, vp += 64) s += fabs(vp->x) + fabs(vp->y);
  if (row >= m.rows) s = 0.0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s = fmax(s, __shfl_xor(s, o, 64));
  if (threadIdx.x == 0)
    atomicMax(reinterpret_cast<unsigned long long*>(out), (unsigned long long)__double_as_longlong(s));
}
}  // namespace

void sell_gershgorin(const SellView& m, double* out, hipStream_t s) {
  DCP_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(double), s));
  if (m.rows <= 0) return;
  hipLaunchKernelGGL(k_sell_rowabs, dim3((m.rows + 63) / 64), dim3(64), 0, s, m, out);
  DCP_HIP_CHECK(hipGetLastError());
}

void add_and_dot(Seg g, double* v, DScal c, const double* x, const double* w, double* partials,
                 double* out, hipStream_t s) {
  add_and_dot_partials(g, v, c, x, w, partials, s);
  reduce_final(kReduceBlocks, partials, out, s);
}
void add_and_dot_partials(Seg g, double* v, DScal c, const double* x, const double* w,
                          double* partials, hipStream_t s) {
  hipLaunchKernelGGL(k_add_and_dot, dim3(kReduceBlocks), dim3(kBlock), 0, s, g, v, c, x, w,
                     partials);
  DCP_HIP_CHECK(hipGetLastError());
}

void axpy(int n, DScal c, const double* x, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_axpy, dim3(grid_for(n)), dim3(kBlock), 0, s, n, c, x, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void scale(int n, DScal c, double* x, hipStream_t s) {
  hipLaunchKernelGGL(k_scale, dim3(grid_for(n)), dim3(kBlock), 0, s, n, c, x);
  DCP_HIP_CHECK(hipGetLastError());
}
void sadd(int n, double s_, double a, const double* x, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_sadd, dim3(grid_for(n)), dim3(kBlock), 0, s, n, s_, a, x, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void copy(int n, const double* x, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_copy, dim3(grid_for(n)), dim3(kBlock), 0, s, n, x, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void equ(int n, DScal c, const double* x, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_equ, dim3(grid_for(n)), dim3(kBlock), 0, s, n, c, x, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void axpby(int n, DScal a, const double* x, DScal b, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_axpby, dim3(grid_for(n)), dim3(kBlock), 0, s, n, a, x, b, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void scalar_div(const double* num, const double* den, double* out, hipStream_t s) {
  hipLaunchKernelGGL(k_scalar_div, dim3(1), dim3(64), 0, s, num, den, out);
  DCP_HIP_CHECK(hipGetLastError());
}
void fill(int n, double v, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_fill, dim3(grid_for(n)), dim3(kBlock), 0, s, n, v, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void mul(int n, const double* a, const double* x, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_mul, dim3(grid_for(n)), dim3(kBlock), 0, s, n, a, x, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void reciprocal(int n, const double* a, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_recip, dim3(grid_for(n)), dim3(kBlock), 0, s, n, a, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void csr_diag_inverse(int rows, const int32_t* ptr, const int32_t* col, const double* val,
                      double* inv, hipStream_t s) {
  hipLaunchKernelGGL(k_csr_diag_inv, dim3(grid_for(rows)), dim3(kBlock), 0, s, rows, ptr, col, val,
                     inv);
  DCP_HIP_CHECK(hipGetLastError());
}
void multi_axpy(int n, int k, const double* coef, const double* const* X, double* y,
                hipStream_t s) {
  if (k <= 0) return;
  hipLaunchKernelGGL(k_multi_axpy, dim3(grid_for(n)), dim3(kBlock), 0, s, n, k, coef, X, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void multi_axpy_args(int n, int k, const CombineArgs& a, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_multi_axpy_args, dim3(grid_for(n)), dim3(kBlock), 0, s, n, k, a, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void lincomb(int n, const double* a, double alpha, const double* b, double* z, hipStream_t s) {
  hipLaunchKernelGGL(k_lincomb, dim3(grid_for(n)), dim3(kBlock), 0, s, n, a, alpha, b, z);
  DCP_HIP_CHECK(hipGetLastError());
}
void distribute_velocity(int n_vnodes, const NodeConstraint* vcon, double* u, hipStream_t s) {
  hipLaunchKernelGGL(k_distribute_velocity, dim3(grid_for(n_vnodes)), dim3(kBlock), 0, s, n_vnodes,
                     vcon, u);
  DCP_HIP_CHECK(hipGetLastError());
}
void copy_images(int n, const int32_t* img, const int32_t* master, double* x, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_copy_images, dim3(grid_for(n)), dim3(kBlock), 0, s, n, img, master, x);
  DCP_HIP_CHECK(hipGetLastError());
}
void distribute_temperature(int n_T, const uint8_t* fixed, const double* bc, double* T,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_distribute_T, dim3(grid_for(n_T)), dim3(kBlock), 0, s, n_T, fixed, bc, T);
  DCP_HIP_CHECK(hipGetLastError());
}
void velocity_stats(const CellData& cd, int n_cells, const double* u, double* out2, hipStream_t s) {
  DCP_HIP_CHECK(hipMemsetAsync(out2, 0, 2 * sizeof(double), s));
  const int grid = (n_cells + kBlock - 1) / kBlock;
  if (grid == 0) return;
  hipLaunchKernelGGL(k_velocity_stats, dim3(grid), dim3(kBlock), 0, s, cd, n_cells, u, out2);
  DCP_HIP_CHECK(hipGetLastError());
}
void minmax(int n, const double* x, double* out2, hipStream_t s) {
  // partial buffer: the caller's out2 must point at >= 2 + 2*kReduceBlocks doubles
  double* partials = out2 + 2;
  hipLaunchKernelGGL(k_minmax_partial, dim3(kReduceBlocks), dim3(kBlock), 0, s, n, x, partials);
  hipLaunchKernelGGL(k_minmax_final, dim3(1), dim3(64), 0, s, kReduceBlocks, partials, out2);
  DCP_HIP_CHECK(hipGetLastError());
}

void spmv_block(int r0, int r1, int c0, int c1, const int32_t* ptr, const int32_t* col,
                const double* val, const double* x, double* y, bool add, hipStream_t s) {
  if (r1 <= r0) return;
  const long threads = long(r1 - r0) * 16;
  hipLaunchKernelGGL(k_spmv_block, dim3(int((threads + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, r0,
                     r1, c0, c1, ptr, col, val, x, y, add ? 1 : 0);
  DCP_HIP_CHECK(hipGetLastError());
}
void shift(int n, DScal c, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_shift, dim3(grid_for(n)), dim3(kBlock), 0, s, n, c, y);
  DCP_HIP_CHECK(hipGetLastError());
}
void zero_fixed(int n, const uint8_t* fixed, double* y, hipStream_t s) {
  hipLaunchKernelGGL(k_zero_fixed, dim3(grid_for(n)), dim3(kBlock), 0, s, n, fixed, y);
  DCP_HIP_CHECK(hipGetLastError());
}

void group_reduce(size_t n, int nbufs, const BufTable& t, double* out, bool max, hipStream_t s) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_group_reduce, dim3(grid_for(long(n))), dim3(kBlock), 0, s, n, nbufs, t, out,
                     max ? 1 : 0);
  DCP_HIP_CHECK(hipGetLastError());
}
void gather(int n, const int32_t* pos, const double* v, double* buf, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_gather, dim3(grid_for(n)), dim3(kBlock), 0, s, n, pos, v, buf);
  DCP_HIP_CHECK(hipGetLastError());
}
void scatter(int n, const int32_t* pos, const double* buf, double* v, hipStream_t s) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_scatter, dim3(grid_for(n)), dim3(kBlock), 0, s, n, pos, buf, v);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
