// Device-resident GMRES cycle with classical Gram-Schmidt applied twice
// (CGS2) for CDNA4 (gfx950), FP64.
//
// The inner Schur-complement GMRES of BlockSchurPreconditioner::vmult
// (block_schur_preconditioner.hpp:47-51: SolverGMRES on S, identity
// preconditioner, restart 28) dominates the reference's time step. deal.II's
// modified Gram-Schmidt needs one global reduction per basis vector (a chain
// of d dependent reductions per Arnoldi step); CGS2 orthogonalises against all
// d vectors at once, twice, so a step is a fixed four launches with three
// reductions whatever d is:
//   k_sell_spmv (linalg.hip)  v_k = w_{k-1} / |w_{k-1}|, w_k = S v_k
//   k_cgs_dot                 h1 = V^T w                         (pass 1)
//   k_cgs_update<0>           w -= V h1; h2 = V^T w              (pass 2)
//   k_cgs_update<1>           w -= V h2; |w|; then the host-side step of
//                             SolverGMRES: h = h1 + h2, Givens rotation,
//                             residual estimate, SolverControl check
// Two vector entries per thread, all their loads issued up front (the 2e5-long
// pressure vectors are only a few loads per CU deep, so width, not depth,
// hides the latency); every block hands its d partial sums over as tagged
// granules (kernels/granule.h: `sc1` stores, no cache write-back fences), the
// last block to bump a device counter polls all of them, sums them in block
// order and publishes the d results, so the next launch reads d numbers
// instead of re-reducing. The Hessenberg
// column, the rotations and the convergence decision live in device memory
// (GmresDev): the host enqueues a whole restart cycle without reading
// anything back, and once a step sets the status every later launch of the
// cycle returns at entry. Every sum has a fixed shape and order, so a cycle
// is bitwise reproducible run to run. Several GPUs: the published sums are
// all-reduced between the launches and the Givens step is its own launch.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cmath>
#include <stdexcept>
#include <string>

#include "../comm.h"
#include "../device.h"
#include "granule.h"

namespace dcp {
namespace {

constexpr int kBlock = 256;

__device__ inline long seg_pos(const Seg& g, long i) {
  return i < g.n1 ? i : (i < g.n12 ? g.off2 + (i - g.n1) : g.off3 + (i - g.n12));
}

// d <= K block sums of s[j] (xor butterfly per wave, then the four wave sums
// left to right): thread j < d returns sum j. sm: [4][K] doubles.
template <int K>
__device__ inline double block_sums(double (&s)[K], int d, double* sm) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    if (j < d) {
      double v = s[j];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if (l == 0) sm[w * K + j] = v;
    }
  }
  __syncthreads();
  const int j = threadIdx.x;
  return j < d ? sm[j] + sm[K + j] + sm[2 * K + j] + sm[3 * K + j] : 0.0;
}

constexpr int kCgsElems = 2;          // vector entries per thread
constexpr long kCgsMaxSpins = 1L << 22;

// Thread 0 bumps the launch's counter; true in the block that comes last
// (which resets the counter for the next launch). No fence: the partials
// travel as self-validating granules.
__device__ inline bool last_block(unsigned* cnt, int* flag) {
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = atomicAdd(cnt, 1u);
    *flag = t == gridDim.x - 1;
    if (*flag) atomicExch(cnt, 0u);
  }
  __syncthreads();
  return *flag != 0;
}

__device__ inline double granule_poll(const double* p, unsigned long long tag, double* err) {
  const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
  for (long spins = 0;; ++spins) {
    const unsigned long long v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long t = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == (tag ^ granule_mix(v))) return __longlong_as_double((long long)v);
    if (spins >= kCgsMaxSpins) {
      *err = 1.0;
      return 0.0;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// Last block: out[j] = sum_b of the granules (j, b) in block order
// (per-thread strided sums, then block_sums), j < d. First every granule is
// loaded once (many loads in flight); only stale ones are polled again.
template <int K>
__device__ inline void reduce_granules(const double* gran, int nb, int d, unsigned long long seq,
                                       double* out, double* sm, double* err) {
  double s[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    s[j] = 0.0;
    if (j < d)
      for (int b = threadIdx.x; b < nb; b += kBlock) {
        const double* p = gran + 2 * (size_t(j) * nb + b);
        const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
        const unsigned long long v = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long t =
            __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long tag = seq * 64 + unsigned(j);
        s[j] += t == (tag ^ granule_mix(v)) ? __longlong_as_double((long long)v)
                                            : granule_poll(p, tag, err);
      }
  }
  const double r = block_sums<K>(s, d, sm);
  if (threadIdx.x < d) out[threadIdx.x] = r;
}

// The host-side step of deal.II SolverGMRES after Arnoldi step k, on the
// device state (one workgroup): h = h1 + h2, h_{k+1} = |w| = sqrt(nrm2), the
// previous rotations, the new Givens rotation (solver_gmres.h
// givens_rotation), residual estimate |gamma_{k+1}|, SolverControl::check.
__device__ void gmres_step(GmresDev* st, double nrm2, int k) {
  __shared__ double h[kGmMaxDim + 1], cs[kGmMaxDim], sn[kGmMaxDim];
  __shared__ double g0;
  __shared__ int acc0;
  const int t = threadIdx.x;
  if (t <= k) h[t] = st->coef[t] + st->coef[kGmMaxDim + t];
  if (t < k) {
    cs[t] = st->ci[t];
    sn[t] = st->si[t];
  }
  if (t == kBlock - 1) {
    g0 = st->gamma[k];
    acc0 = st->accumulated;
  }
  __syncthreads();
  if (t == 0) {
    const double nrm = sqrt(nrm2);
    h[k + 1] = nrm;
    for (int i = 0; i < k; i++) {
      const double dummy = h[i];
      h[i] = cs[i] * dummy + sn[i] * h[i + 1];
      h[i + 1] = -sn[i] * dummy + cs[i] * h[i + 1];
    }
    const double r = 1. / sqrt(h[k] * h[k] + h[k + 1] * h[k + 1]);
    const double s = h[k + 1] * r, c = h[k] * r;
    st->si[k] = s;
    st->ci[k] = c;
    h[k] = c * h[k] + s * h[k + 1];
    const double gk1 = -s * g0;
    st->gamma[k + 1] = gk1;
    st->gamma[k] = g0 * c;
    const int acc = acc0 + 1;
    st->accumulated = acc;
    st->dim = k + 1;
    const double rho = fabs(gk1);
    st->rho = rho;
    st->inv_norm = nrm != 0 ? 1.0 / nrm : 1.0;
    st->status = rho <= st->tol ? 1 : ((acc >= st->max_steps || isnan(rho)) ? 2 : 0);
  }
  __syncthreads();
  if (t <= k) st->H[t][k] = h[t];
}

// h1 = V^T w (j < d): block partials as granules, the last block sums them
// -> hout.
template <int K>
__global__ __launch_bounds__(kBlock) void k_cgs_dot(Seg g, const double* __restrict__ w,
                                                    ChainVecs V, int d, double* gran,
                                                    unsigned* cnt, double* hout,
                                                    unsigned long long seq, double* err,
                                                    const int* __restrict__ status) {
  __shared__ double sm[4 * K];
  __shared__ int is_last;
  if (*status) return;
  double s[K];
#pragma unroll
  for (int j = 0; j < K; ++j) s[j] = 0.0;
  const long k0 = long(blockIdx.x) * (kBlock * kCgsElems) + threadIdx.x;
  double wv[kCgsElems], v[kCgsElems][K];
#pragma unroll
  for (int e = 0; e < kCgsElems; ++e) {
    const long k = k0 + e * kBlock;
    const bool live = k < g.n;
    const long i = live ? seg_pos(g, k) : 0;
    wv[e] = live ? w[i] : 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) v[e][j] = live && j < d ? V.v[j][i] : 0.0;
  }
#pragma unroll
  for (int e = 0; e < kCgsElems; ++e)
#pragma unroll
    for (int j = 0; j < K; ++j) s[j] += v[e][j] * wv[e];
  const double r = block_sums<K>(s, d, sm);
  const int nb = gridDim.x;
  if (threadIdx.x < d)
    granule_store(gran + 2 * (size_t(threadIdx.x) * nb + blockIdx.x), r, seq * 64 + threadIdx.x);
  if (!last_block(cnt, &is_last)) return;
  reduce_granules<K>(gran, nb, d, seq, hout, sm, err);
}

// w -= V h (h = hin[0..d), fixed order j = 0..d-1), then PASS 0: h2 = V^T w
// -> hout; PASS 1: |w|^2 -> *hout, and with st != null (one GPU) the Givens
// step kstep in the last block.
template <int K, int PASS>
__global__ __launch_bounds__(kBlock) void k_cgs_update(Seg g, double* __restrict__ w, ChainVecs V,
                                                       int d, const double* hin, double* gran,
                                                       unsigned* cnt, double* hout,
                                                       GmresDev* st, int kstep,
                                                       unsigned long long seq, double* err,
                                                       const int* __restrict__ status) {
  __shared__ double sm[4 * K];
  __shared__ double hs[K];
  __shared__ int is_last;
  if (*status) return;
  if (threadIdx.x < d) hs[threadIdx.x] = hin[threadIdx.x];
  const long k0 = long(blockIdx.x) * (kBlock * kCgsElems) + threadIdx.x;
  double wv[kCgsElems], v[kCgsElems][K];
  long pos[kCgsElems];
#pragma unroll
  for (int e = 0; e < kCgsElems; ++e) {
    const long k = k0 + e * kBlock;
    pos[e] = k < g.n ? seg_pos(g, k) : -1;
    wv[e] = pos[e] >= 0 ? w[pos[e]] : 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) v[e][j] = pos[e] >= 0 && j < d ? V.v[j][pos[e]] : 0.0;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kCgsElems; ++e) {
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (j < d) wv[e] -= hs[j] * v[e][j];
    if (pos[e] >= 0) w[pos[e]] = wv[e];
  }
  const int nb = gridDim.x;
  if (PASS == 0) {
    double s[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
      s[j] = 0.0;
#pragma unroll
      for (int e = 0; e < kCgsElems; ++e) s[j] += v[e][j] * wv[e];
    }
    const double r = block_sums<K>(s, d, sm);
    if (threadIdx.x < d)
      granule_store(gran + 2 * (size_t(threadIdx.x) * nb + blockIdx.x), r, seq * 64 + threadIdx.x);
    if (!last_block(cnt, &is_last)) return;
    reduce_granules<K>(gran, nb, d, seq, hout, sm, err);
  } else {
    double s1[1] = {0.0};
#pragma unroll
    for (int e = 0; e < kCgsElems; ++e) s1[0] += wv[e] * wv[e];
    const double r = block_sums<1>(s1, 1, sm);
    if (threadIdx.x == 0) granule_store(gran + 2 * size_t(blockIdx.x), r, seq * 64);
    if (!last_block(cnt, &is_last)) return;
    reduce_granules<1>(gran, nb, 1, seq, hs, sm, err);
    __syncthreads();
    if (threadIdx.x == 0) *hout = hs[0];
    if (st) gmres_step(st, hs[0], kstep);
  }
}

// One GPU: the whole CGS2 step in one launch of nb resident 512-thread
// workgroups (nb <= the CU count, like k_mgs_chain), two vector entries per
// thread: every basis load of the step is issued at once and the 2 d basis
// entries stay in registers for all three passes (<= 210 VGPRs at d = 28,
// two waves per SIMD). A reduction is two granule hops: every workgroup
// publishes its d block sums (column j of the partial area), workgroup j sums
// column j in block_sum order and publishes the result, and every workgroup
// reads the d results. Two reductions per step (V^T w, then V^T w and |w|^2
// after the first update; the norm of the result is |w|^2 - |V^T w|^2), after
// which workgroup 0 does the Givens step. Overwriting a partial granule of the next reduction
// is safe: a workgroup only gets there after every reducer has published,
// i.e. finished reading.
constexpr int kChainThreads = 512;
constexpr int kChainWaves = kChainThreads / 64;
constexpr int kChainEntries = 2;   // vector entries per thread (registers: 2 x d basis entries)
constexpr int kCgsRes = 2 * kGmMaxDim * 256;  // result granules after the partial area

// Reduce-scatter of the K products v[j] * x over the 64 lanes of a wave:
// log2 K halving exchanges (the first one forms the products, so only K / 2
// accumulators are live next to v) then full butterflies over the remaining
// lane bits; lane l ends with the wave sum of value l >> (6 - log2 K).
// Fixed tree, deterministic.
// The products of one thread are v[0][j] x[0] + v[1][j] x[1] (its two entries).
template <int K>
__device__ inline double wave_reduce_scatter(const double (&v)[kChainEntries][K],
                                             const double (&x)[kChainEntries]) {
  const int l = threadIdx.x & 63;
  if constexpr (K == 1) {
    double r = v[0][0] * x[0] + v[1][0] * x[1];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
    return r;
  } else {
    double s[K / 2];
    {
      const bool up = (l & 32) != 0;
#pragma unroll
      for (int i = 0; i < K / 2; ++i) {
        const double lo = v[0][i] * x[0] + v[1][i] * x[1];
        const double hi = v[0][i + K / 2] * x[0] + v[1][i + K / 2] * x[1];
        const double send = up ? lo : hi;
        const double keep = up ? hi : lo;
        s[i] = keep + __shfl_xor(send, 32, 64);
      }
    }
    int o = 16;
#pragma unroll
    for (int c = K / 2; c > 1; c >>= 1, o >>= 1) {
      const bool up = (l & o) != 0;
#pragma unroll
      for (int i = 0; i < c / 2; ++i) {
        const double send = up ? s[i] : s[i + c / 2];
        const double keep = up ? s[i + c / 2] : s[i];
        s[i] = keep + __shfl_xor(send, o, 64);
      }
    }
    double r = s[0];
    for (; o > 0; o >>= 1) r += __shfl_xor(r, o, 64);
    return r;
  }
}
template <int K>
constexpr int log2i() { return K <= 1 ? 0 : 1 + log2i<K / 2>(); }

// d <= K block sums of v[j] * x over the 16 waves (wave reduce-scatter, then
// the wave sums in wave order): thread j < d returns sum j. sm: [kChainWaves][K].
template <int K>
__device__ inline double chain_block_sums(const double (&v)[kChainEntries][K],
                                          const double (&x)[kChainEntries], int d, double* sm) {
  const double r = wave_reduce_scatter<K>(v, x);
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int sh = 6 - log2i<K>();
  if ((l & ((1 << sh) - 1)) == 0) sm[w * K + (l >> sh)] = r;
  __syncthreads();
  double t = 0.0;
  if (int(threadIdx.x) < d)
    for (int i = 0; i < kChainWaves; ++i) t += sm[i * K + threadIdx.x];
  return t;
}

template <int KL>
constexpr int pow2_at_least() { return KL <= 1 ? 1 : 2 * pow2_at_least<(KL + 1) / 2>(); }
// KL: basis vectors loaded (d <= KL); the reductions run over the next power
// of two K with the entries past KL compile-time zero.
template <int KL, bool WIDE>
__global__ __launch_bounds__(kChainThreads) void k_cgs2_chain(Seg g, double* w, ChainVecs V,
                                                              int d, GmresDev* st, int kstep,
                                                              double* gran,
                                                              unsigned long long seq,
                                                              double* err) {
  constexpr int K = pow2_at_least<KL>();
  static_assert(kChainEntries == 2, "wide loads pair the two entries of a thread");
  __shared__ double sm[kChainWaves * K];
  __shared__ double hs[K];
  __shared__ double nrm_sh;
  if (st->status) return;
  const int nb = gridDim.x, b = blockIdx.x;
#ifndef DCP_CGS_NOLOAD
#define DCP_CGS_NOLOAD 0
#endif
#ifndef DCP_CGS_NOWAIT
#define DCP_CGS_NOWAIT 0
#endif
  // (timing probes only: DCP_CGS_NOLOAD replaces the basis loads, DCP_CGS_NOWAIT
  // the granule hand-offs; both give wrong results)
  // entries b * 1024 + e * 512 + t of the owned vector; branch-free loads
  // (V.v[j] for j >= d points at V.v[0]) all issued before the first use
  // WIDE (one segment, n even, 16-byte aligned vectors): a thread owns the adjacent
  // entries 2 t, 2 t + 1 of its block and reads each basis vector with one
  // 16-byte load (8-byte loads leave the chain's load phase at ~2.9 TB/s)
  double x[kChainEntries], v[kChainEntries][K];
  unsigned pos[kChainEntries];
  bool live[kChainEntries];
  const long kb = long(b) * (kChainThreads * kChainEntries);
  if (WIDE) {
    const long k0 = kb + 2 * long(threadIdx.x);
    live[0] = live[1] = k0 < g.n;  // n even: a pair is all in or all out
    pos[0] = live[0] ? unsigned(k0) : 0u;
    pos[1] = pos[0] + 1;
    const double2 xw = *reinterpret_cast<const double2*>(w + pos[0]);
    x[0] = xw.x;
    x[1] = xw.y;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      double2 t = {0.0, 0.0};
      if (j < KL) t = *reinterpret_cast<const double2*>(V.v[j] + pos[0]);
      v[0][j] = t.x;
      v[1][j] = t.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < kChainEntries; ++e) {
      const long k = kb + e * kChainThreads + threadIdx.x;
      live[e] = k < g.n;
      pos[e] = live[e] ? unsigned(seg_pos(g, k)) : 0u;
      x[e] = w[pos[e]];
#pragma unroll
      for (int j = 0; j < K; ++j)
        v[e][j] = j >= KL ? 0.0 : (DCP_CGS_NOLOAD ? x[e] * (j + 1) : V.v[j][pos[e]]);
    }
  }
#pragma unroll
  for (int e = 0; e < kChainEntries; ++e) {
    x[e] = live[e] ? x[e] : 0.0;
#pragma unroll
    for (int j = 0; j < KL; ++j) v[e][j] = live[e] && j < d ? v[e][j] : 0.0;
  }
  double* part = gran;
  double* res = gran + kCgsRes;
  // The second pass also reduces |x|^2 of its input (entry K - 1 of the
  // reduce-scatter, free since d < K; granule column d), so the norm of the
  // result follows without a third reduction: |x - V h|^2 = |x|^2 - |h|^2
  // for orthonormal V (h = V^T x).
  for (int pass = 0; pass < 2; ++pass) {
    const unsigned long long tag = seq * 64 + 4 * unsigned(pass);
    double r;
    if (pass == 1) {
      double v2[kChainEntries][K];
#pragma unroll
      for (int e = 0; e < kChainEntries; ++e)
#pragma unroll
        for (int j = 0; j < K; ++j) v2[e][j] = j == K - 1 ? x[e] : v[e][j];
      r = chain_block_sums<K>(v2, x, K, sm);
    } else {
      r = chain_block_sums<K>(v, x, d, sm);
    }
    const int ncol = d + pass;  // pass 1: column d = |x|^2
    const bool pub = int(threadIdx.x) < d || (pass == 1 && int(threadIdx.x) == K - 1);
    const int col = int(threadIdx.x) < d ? int(threadIdx.x) : d;
    if (DCP_CGS_NOWAIT) {
      if (int(threadIdx.x) < ncol) hs[threadIdx.x] = r * 1e-3;
    } else {
    if (pub) granule_store(part + 2 * (size_t(col) * nb + b), r, tag);
    if (b < ncol && threadIdx.x < 64) {
      const double tot = granule_coef(part + 2 * size_t(b) * nb, nb, tag, err);
      if (threadIdx.x == 0) granule_store(res + 2 * b, tot, tag + 1);
    }
    if (int(threadIdx.x) < ncol) {
      const double* p = res + 2 * threadIdx.x;
      mgs_u4 q = granule_load(p);
      for (long spins = 0; !tag_is(q, tag + 1); ++spins) {
        if (spins >= kMgsMaxSpins) {
          *err = 1.0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        q = granule_load(p);
      }
      hs[threadIdx.x] = granule_value(q);
      if (b == 0 && int(threadIdx.x) < d) st->coef[pass * kGmMaxDim + threadIdx.x] = granule_value(q);
    }
    }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < kChainEntries; ++e)
#pragma unroll
      for (int j = 0; j < KL; ++j)
        if (j < d) x[e] -= hs[j] * v[e][j];
    __syncthreads();  // hs / sm reused by the next reduction
  }
#pragma unroll
  for (int e = 0; e < kChainEntries; ++e)
    if (live[e]) w[pos[e]] = x[e];
  if (b != 0) return;
  if (threadIdx.x == 0) {
    double n2 = hs[d];
    for (int j = 0; j < d; ++j) n2 -= hs[j] * hs[j];
    nrm_sh = fmax(n2, 0.0);
    st->nrm2 = nrm_sh;
  }
  __syncthreads();
  gmres_step(st, nrm_sh, kstep);
}

// Several GPUs: the Givens step after the all-reduce of |w|^2.
__global__ __launch_bounds__(kBlock) void k_gmres_step(GmresDev* st, const double* nrm2, int k) {
  if (st->status) return;
  gmres_step(st, *nrm2, k);
}

// H y = gamma (upper triangular, dim x dim), as SolverGMRES's H1.backward:
// H and gamma staged in LDS by the whole workgroup, then one thread.
__global__ __launch_bounds__(kBlock) void k_gmres_backsub(GmresDev* st) {
  __shared__ double H[kGmMaxDim][kGmMaxDim + 1], gam[kGmMaxDim], y[kGmMaxDim];
  const int dim = st->dim;
  for (int t = threadIdx.x; t < dim * dim; t += kBlock) H[t / dim][t % dim] = st->H[t / dim][t % dim];
  if (int(threadIdx.x) < dim) gam[threadIdx.x] = st->gamma[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = dim - 1; i >= 0; --i) {
      double sum = gam[i];
      for (int j = i + 1; j < dim; ++j) sum -= y[j] * H[i][j];
      y[i] = sum / H[i][i];
    }
  }
  __syncthreads();
  if (int(threadIdx.x) < dim) st->y[threadIdx.x] = y[threadIdx.x];
}

template <int K>
void cgs_step_k(Seg g, double* w, const ChainVecs& V, int d, double* gran, unsigned* cnt,
                GmresDev* st, unsigned long long& seq, double* err, Comm* comm, hipStream_t s) {
  const int* status = &st->status;
  const int nb = int((long(g.n) + kBlock * kCgsElems - 1) / (kBlock * kCgsElems));
  if (nb <= 0) return;
  hipLaunchKernelGGL((k_cgs_dot<K>), dim3(nb), dim3(kBlock), 0, s, g, w, V, d, gran, cnt,
                     st->coef, ++seq, err, status);
  DCP_HIP_CHECK(hipGetLastError());
  if (comm) comm->allreduce(st->coef, size_t(d), false, s);
  hipLaunchKernelGGL((k_cgs_update<K, 0>), dim3(nb), dim3(kBlock), 0, s, g, w, V, d, st->coef,
                     gran, cnt, st->coef + kGmMaxDim, nullptr, d - 1, ++seq, err, status);
  DCP_HIP_CHECK(hipGetLastError());
  if (comm) comm->allreduce(st->coef + kGmMaxDim, size_t(d), false, s);
  hipLaunchKernelGGL((k_cgs_update<K, 1>), dim3(nb), dim3(kBlock), 0, s, g, w, V, d,
                     st->coef + kGmMaxDim, gran, cnt, &st->nrm2, comm ? nullptr : st, d - 1,
                     ++seq, err, status);
  DCP_HIP_CHECK(hipGetLastError());
  if (comm) {
    comm->allreduce(&st->nrm2, 1, false, s);
    hipLaunchKernelGGL(k_gmres_step, dim3(1), dim3(kBlock), 0, s, st, &st->nrm2, d - 1);
    DCP_HIP_CHECK(hipGetLastError());
  }
}

}  // namespace

bool cgs2_chain_fits(long n, int nb, int n_cus) {
  return nb >= kGmMaxDim && nb <= n_cus && nb <= 256 &&
         n <= long(nb) * kChainThreads * kChainEntries;
}

void cgs2_chain_step(Seg g, double* w, const ChainVecs& V, int d, GmresDev* st, double* gran,
                     int nb, unsigned long long seq, double* err, hipStream_t s) {
  ChainVecs Vp = V;  // unused slots point at V[0]: the kernel's loads are unconditional
  for (int j = d; j < kGmMaxDim; ++j) Vp.v[j] = V.v[0];
  bool wide = g.n1 == g.n && g.n % 2 == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0;
  for (int j = 0; j < d; ++j) wide = wide && (reinterpret_cast<uintptr_t>(V.v[j]) & 15) == 0;
  const dim3 grid(nb), block(kChainThreads);
  // KL > d: the chain's second reduction keeps its |w|^2 entry at K - 1 >= d
#define DCP_CGS_CASE(KL)                                                                       \
  if (d < KL) {                                                                                \
    if (wide)                                                                                  \
      hipLaunchKernelGGL((k_cgs2_chain<KL, true>), grid, block, 0, s, g, w, Vp, d, st, d - 1,  \
                         gran, seq, err);                                                      \
    else                                                                                       \
      hipLaunchKernelGGL((k_cgs2_chain<KL, false>), grid, block, 0, s, g, w, Vp, d, st, d - 1, \
                         gran, seq, err);                                                      \
    DCP_HIP_CHECK(hipGetLastError());                                                          \
    return;                                                                                    \
  }
  DCP_CGS_CASE(4) DCP_CGS_CASE(8) DCP_CGS_CASE(12) DCP_CGS_CASE(16) DCP_CGS_CASE(20)
  DCP_CGS_CASE(24) DCP_CGS_CASE(28) DCP_CGS_CASE(32)
#undef DCP_CGS_CASE
  throw std::runtime_error("cgs2_chain_step: " + std::to_string(d) + " basis vectors (at most " +
                           std::to_string(kGmMaxDim - 1) + ")");
}

size_t cgs2_granules(long n) {
  return 2 * size_t(kGmMaxDim) * size_t((n + kBlock * kCgsElems - 1) / (kBlock * kCgsElems)) + 2;
}

void cgs2_gmres_step(Seg g, double* w, const ChainVecs& V, int d, double* gran, unsigned* cnt,
                     GmresDev* st, unsigned long long& seq, double* err, Comm* comm,
                     hipStream_t s) {
  if (d <= 8)
    cgs_step_k<8>(g, w, V, d, gran, cnt, st, seq, err, comm, s);
  else if (d <= 16)
    cgs_step_k<16>(g, w, V, d, gran, cnt, st, seq, err, comm, s);
  else
    cgs_step_k<kGmMaxDim>(g, w, V, d, gran, cnt, st, seq, err, comm, s);
}

__global__ void k_gmres_cycle_init(GmresDev* st, const double* __restrict__ rho2, double tol,
                                   int max_steps, int first) {
  if (threadIdx.x != 0) return;
  if (first) {
    st->status = 0;
    st->accumulated = 0;
    st->tol = tol;
    st->max_steps = max_steps;
  }
  st->dim = 0;
  if (st->status != 0) return;
  const double rho = sqrt(*rho2);
  const int acc = st->accumulated;
  st->rho = rho;
  // SolverControl::check(accumulated, rho) at the head of the cycle
  const int status = rho <= st->tol ? 1 : ((acc >= st->max_steps || isnan(rho)) ? 2 : 0);
  st->status = status;
  if (status != 0) return;
  st->gamma[0] = rho;
  st->inv_rho = 1.0 / rho;
  st->inv_norm = 1.0;
}

// x += sum_{j < dim} y_j V_j, dim read on the device (0: nothing)
__global__ void k_gmres_update(const GmresDev* __restrict__ st, int n, const double* const* V,
                               double* __restrict__ x) {
  const int dim = st->dim;
  if (dim <= 0) return;
  for (long i = long(blockIdx.x) * kBlock + threadIdx.x; i < n; i += long(gridDim.x) * kBlock) {
    double v = x[i];
    for (int j = 0; j < dim; ++j) v += st->y[j] * V[j][i];
    x[i] = v;
  }
}

__global__ void k_gmres_report(const GmresDev* __restrict__ st, GmresReport* report) {
  if (threadIdx.x != 0) return;
  // plain vector stores into the pinned host record; the host reads it after
  // an event recorded behind this launch
  report->rho = st->rho;
  report->status = st->status;
  report->accumulated = st->accumulated;
}

void gmres_cycle_init(GmresDev* st, const double* rho2, double tol, int max_steps, bool first,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_gmres_cycle_init, dim3(1), dim3(64), 0, s, st, rho2, tol, max_steps,
                     int(first));
  DCP_HIP_CHECK(hipGetLastError());
}

void gmres_cycle_end(GmresDev* st, int n, const double* const* V, double* x, GmresReport* report,
                     hipStream_t s) {
  hipLaunchKernelGGL(k_gmres_backsub, dim3(1), dim3(kBlock), 0, s, st);
  DCP_HIP_CHECK(hipGetLastError());
  const long blocks = std::min<long>((long(n) + kBlock - 1) / kBlock, 2048);
  hipLaunchKernelGGL(k_gmres_update, dim3(unsigned(std::max<long>(blocks, 1))), dim3(kBlock), 0, s,
                     st, n, V, x);
  DCP_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(k_gmres_report, dim3(1), dim3(64), 0, s, st, report);
  DCP_HIP_CHECK(hipGetLastError());
}

void gmres_backsub(GmresDev* st, hipStream_t s) {
  hipLaunchKernelGGL(k_gmres_backsub, dim3(1), dim3(kBlock), 0, s, st);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
