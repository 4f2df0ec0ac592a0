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
#include "resident.h"

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
      const double v = wave_allsum(s[j]);
      if (l == 0) sm[w * K + j] = v;
    }
  }
  __syncthreads();
  const int j = threadIdx.x;
  return j < d ? sm[j] + sm[K + j] + sm[2 * K + j] + sm[3 * K + j] : 0.0;
}

// hand-off poll bound of the one-launch kernels below (kMgsMaxSpins; a test
// hook lowers it to make the timeout path run, set_handoff_spin_limit)
__constant__ long g_spin_limit = kMgsMaxSpins;

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
    atomicMax(&st->status, rho <= st->tol ? 1 : ((acc >= st->max_steps || isnan(rho)) ? 2 : 0));
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

template <int C, int O>
__device__ inline void rs_step(double* s, int l) {
  // C live accumulators -> C / 2: lanes with bit O clear keep [0, C/2), the
  // others [C/2, C)
  if constexpr (O >= 16) {
#pragma unroll
    for (int i = 0; i < C / 2; ++i) {
      double a = s[i], b = s[i + C / 2];
      xch_swap<O>(a, b);
      s[i] = a + b;
    }
  } else {
    const bool up = (l & O) != 0;
#pragma unroll
    for (int i = 0; i < C / 2; ++i) {
      const double send = up ? s[i] : s[i + C / 2];
      const double keep = up ? s[i + C / 2] : s[i];
      s[i] = keep + xch_xor<O>(send);
    }
  }
}
template <int C, int O>
__device__ inline void rs_steps(double* s, int l) {
  if constexpr (C > 1) {
    rs_step<C, O>(s, l);
    rs_steps<C / 2, O / 2>(s, l);
  }
}
template <int K>
__device__ inline double wave_reduce_scatter(const double (&v)[kChainEntries][K],
                                             const double (&x)[kChainEntries]) {
  const int l = threadIdx.x & 63;
  if constexpr (K == 1) {
    return butterfly_from<32>(v[0][0] * x[0] + v[1][0] * x[1]);
  } else {
    double s[K / 2];
#pragma unroll
    for (int i = 0; i < K / 2; ++i) {
      double lo = v[0][i] * x[0] + v[1][i] * x[1];
      double hi = v[0][i + K / 2] * x[0] + v[1][i + K / 2] * x[1];
      xch_swap<32>(lo, hi);
      s[i] = lo + hi;
    }
    // K / 2 live at lane bit 16, down to one value, then butterflies below
    rs_steps<K / 2, 16>(s, l);
    return butterfly_from<32 / K>(s[0]);  // the lane bits below the halving steps
  }
}
// Reduce-scatter over a wave of the K products prod(j) (j compile-time after
// unrolling), as wave_reduce_scatter: lane l ends with the wave sum of slot
// l >> (6 - log2 K).
template <int K, class F>
__device__ inline double wave_rs(F prod) {
  const int l = threadIdx.x & 63;
  double s[K / 2];
#pragma unroll
  for (int i = 0; i < K / 2; ++i) {
    double lo = prod(i), hi = prod(i + K / 2);
    xch_swap<32>(lo, hi);
    s[i] = lo + hi;
  }
  rs_steps<K / 2, 16>(s, l);
  return butterfly_from<32 / K>(s[0]);
}

template <int K>
constexpr int log2i() { return K <= 1 ? 0 : 1 + log2i<K / 2>(); }

// d <= K block sums of v[j] * x over the 16 waves (wave reduce-scatter, then
// the wave sums in wave order): thread j < d returns sum j. sm: [kChainWaves][K].
// (in two halves, chain_wave_sums / chain_sum_waves around the caller's
// barrier, so several reductions share one)
template <int K>
__device__ inline void chain_wave_sums(const double (&v)[kChainEntries][K],
                                       const double (&x)[kChainEntries], double* sm) {
  const double r = wave_reduce_scatter<K>(v, x);
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int sh = 6 - log2i<K>();
  if ((l & ((1 << sh) - 1)) == 0) sm[w * K + (l >> sh)] = r;
}
template <int K>
__device__ inline double chain_sum_waves(int d, const double* sm) {
  double t = 0.0;
  if (int(threadIdx.x) < d)
    for (int i = 0; i < kChainWaves; ++i) t += sm[i * K + threadIdx.x];
  return t;
}
template <int K>
__device__ inline double chain_block_sums(const double (&v)[kChainEntries][K],
                                          const double (&x)[kChainEntries], int d, double* sm) {
  chain_wave_sums<K>(v, x, sm);
  __syncthreads();
  return chain_sum_waves<K>(d, sm);
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
      const double tot = granule_coef(part + 2 * size_t(b) * nb, nb, tag, err, &st->status, g_spin_limit);
      if (threadIdx.x == 0) granule_store(res + 2 * b, tot, tag + 1);
    }
    if (int(threadIdx.x) < ncol) {
      const double* p = res + 2 * threadIdx.x;
      mgs_u4 q = granule_load(p);
      for (long spins = 0; !tag_is(q, tag + 1); ++spins) {
        if (spins >= g_spin_limit) {
          handoff_timeout(err, &st->status);
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
  // a rank with no owned pressure rows still runs one (empty) block per launch:
  // it must join every all-reduce and run the Givens step like the others
  const int nb = std::max(1, int((long(g.n) + kBlock * kCgsElems - 1) / (kBlock * kCgsElems)));
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

void set_handoff_spin_limit(long spins) {
  const long v = spins > 0 ? spins : kMgsMaxSpins;
  DCP_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_spin_limit), &v, sizeof(v)));
}

namespace {
// co-resident workgroups of every instance of a one-launch kernel family
// (resident.h; the smallest over the instances the launchers may pick)
template <class F, size_t N>
int family_capacity(const F (&fs)[N]) {
  int cap = 1 << 30;
  for (const F f : fs) cap = std::min(cap, resident_capacity(reinterpret_cast<const void*>(f), kChainThreads));
  return cap;
}
int cgs2_capacity() {
  static const int cap = [] {
    decltype(&k_cgs2_chain<4, true>) fs[] = {
        k_cgs2_chain<4, true>, k_cgs2_chain<8, true>, k_cgs2_chain<12, true>,
        k_cgs2_chain<16, true>, k_cgs2_chain<20, true>, k_cgs2_chain<24, true>,
        k_cgs2_chain<28, true>, k_cgs2_chain<32, true>, k_cgs2_chain<4, false>,
        k_cgs2_chain<8, false>, k_cgs2_chain<12, false>, k_cgs2_chain<16, false>,
        k_cgs2_chain<20, false>, k_cgs2_chain<24, false>, k_cgs2_chain<28, false>,
        k_cgs2_chain<32, false>};
    return family_capacity(fs);
  }();
  return cap;
}
}  // namespace

bool cgs2_chain_fits(long n, int nb, int n_cus) {
  return nb >= kGmMaxDim && nb <= n_cus && nb <= 256 &&
         n <= long(nb) * kChainThreads * kChainEntries && nb <= cgs2_capacity();
}

void cgs2_chain_step(Seg g, double* w, const ChainVecs& V, int d, GmresDev* st, double* gran,
                     int nb, unsigned long long seq, double* err, hipStream_t s) {
  ChainVecs Vp = V;  // unused slots point at V[0]: the kernel's loads are unconditional
  for (int j = d; j < kGmMaxDim; ++j) Vp.v[j] = V.v[0];
  bool wide = g.n1 == g.n && g.n % 2 == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0;
  for (int j = 0; j < d; ++j) wide = wide && (reinterpret_cast<uintptr_t>(V.v[j]) & 15) == 0;
  // KL > d: the chain's second reduction keeps its |w|^2 entry at K - 1 >= d
#define DCP_CGS_CASE(KL)                                                                       \
  if (d < KL) {                                                                                \
    if (wide)                                                                                  \
      launch_resident(k_cgs2_chain<KL, true>, nb, kChainThreads, s, g, w, Vp, d, st, d - 1,    \
                      gran, seq, err);                                                         \
    else                                                                                       \
      launch_resident(k_cgs2_chain<KL, false>, nb, kChainThreads, s, g, w, Vp, d, st, d - 1,   \
                      gran, seq, err);                                                         \
    return;                                                                                    \
  }
  DCP_CGS_CASE(4) DCP_CGS_CASE(8) DCP_CGS_CASE(12) DCP_CGS_CASE(16) DCP_CGS_CASE(20)
  DCP_CGS_CASE(24) DCP_CGS_CASE(28) DCP_CGS_CASE(32)
#undef DCP_CGS_CASE
  throw std::runtime_error("cgs2_chain_step: " + std::to_string(d) + " basis vectors (at most " +
                           std::to_string(kGmMaxDim - 1) + ")");
}

// ---------------------------------------------------------------------------
// s-step (communication-avoiding) Arnoldi block, s = kSStep: the host has
// formed the raw Newton basis w_i = (S - theta_i) w_{i-1} / sigma, w_0 = q_k,
// i = 1..s (sell_spmv_shifted, s back-to-back SpMVs); this launch
//   1. C1 = Q^T W against the basis q_0..q_k, W -= Q C1          (reduction 1)
//   2. C2 = Q^T W and G = W^T W, W -= Q C2, G' = G - C2^T C2      (reduction 2)
//   3. R = chol(G'), q_{k+1..k+s} = W R^-1 (block Gram-Schmidt twice, then
//      Cholesky QR; no further reduction)
// and one workgroup (an idle one when the grid has one) turns the change of
// basis into the s new Hessenberg columns
// k..k+s-1 (A [w_0..w_{s-1}] = [w_0..w_s] B, B = theta on the diagonal, sigma
// below it; H_new = (Rhat B - H_old T_top) U^-1) and runs SolverGMRES's Givens
// step and SolverControl check column by column, so the iteration count and
// the stopping column are those of the one-vector-per-step Arnoldi process.
// Two reductions per s steps instead of two per step; the same registers /
// granule hand-off scheme as k_cgs2_chain (nb resident 512-thread workgroups,
// two entries per thread). The wave reductions run on lane swaps / DPP
// (lanes.h), the four (eight) block sums of a pass share one barrier, and the
// Gram corrections run one thread per entry: the same arithmetic in the same
// order as before, bit for bit.
namespace {

constexpr int kSsRes = 2 * 128 * 256;  // result granules after the partial area

// DCP_SS_PROBE bit 32 (timing probe): thread 0 of the s-step block's
// Hessenberg workgroup stamps the wall clock (100 MHz) at the phase boundaries
// and prints every 64th launch
#ifndef DCP_SS_PROBE
#define DCP_SS_PROBE 0
#endif
#if DCP_SS_PROBE & 32
#define SS_STAMP(i) \
  if (ss_ts && threadIdx.x == 0) ss_ts[i] = wall_clock64()
#else
#define SS_STAMP(i)
#endif


// G' = G - C2^T C2 (G: pass-2 Gram sums after C2's d * S coefficients at
// c2[ncol1..]), upper-triangle entry p = (i, l >= i) in row order, one thread
// per entry
__device__ inline double sstep_gram_entry(const double* c2, int d, int ncol1, int p) {
  constexpr int S = kSStep;
  int i = 0, l = p;
  while (l >= S - i) {
    l -= S - i;
    ++i;
  }
  l += i;
  double gv = c2[ncol1 + p];
  for (int j = 0; j < d; ++j) gv -= c2[i * d + j] * c2[l * d + j];
  return gv;
}

// R = chol(G') upper triangular from the packed entries of sstep_gram_entry;
// false if G' is not positive definite (the block lost rank)
__device__ bool sstep_chol(const double* Gp, double (*Rm)[kSStep]) {
  constexpr int S = kSStep;
  double G[S][S];
  int p = 0;
  for (int i = 0; i < S; ++i)
    for (int l = i; l < S; ++l, ++p) G[i][l] = G[l][i] = Gp[p];
  bool ok = true;
  for (int i = 0; i < S; ++i) {
    double dd = G[i][i];
    for (int l = 0; l < i; ++l) dd -= Rm[l][i] * Rm[l][i];
    if (!(dd > 0)) {
      ok = false;
      dd = 1.0;
    }
    Rm[i][i] = sqrt(dd);
    for (int l = i + 1; l < S; ++l) {
      double o = G[i][l];
      for (int m = 0; m < i; ++m) o -= Rm[m][i] * Rm[m][l];
      Rm[i][l] = o / Rm[i][i];
    }
    for (int l = 0; l < i; ++l) Rm[i][l] = 0.0;
  }
  return ok;
}

// G' entries (threads < nG) and R (thread 0) into the workgroup's LDS; every
// thread of the workgroup calls it, ends with a barrier
__device__ inline void sstep_factor(const double* c2, int d, int ncol1, double* Gp,
                                    double (*Rm)[kSStep], int* bad) {
  constexpr int nG = kSStep * (kSStep + 1) / 2;
  if (threadIdx.x < nG) Gp[threadIdx.x] = sstep_gram_entry(c2, d, ncol1, threadIdx.x);
  __syncthreads();
  if (threadIdx.x == 0) *bad = !sstep_chol(Gp, Rm);
  __syncthreads();
}

// The Hessenberg state workgroup 0 reads (old raw columns, rotations, gamma_k,
// step count, tolerance), staged in LDS by sstep_hess_stage at the start of the
// launch so the global-memory latency overlaps the block's reductions (only
// workgroup 0 of the launch writes these fields, at its very end)
struct SsHess {
  double Hs[kGmMaxDim + 1][kGmMaxDim];
  double cs[kGmMaxDim], sn[kGmMaxDim], gam[kGmMaxDim + 1];
  double tol;
  int acc0, max_steps;
};
__device__ inline void sstep_hess_stage(SsHess& h, const GmresDev* st, int k) {
  const int d = k + 1, t = threadIdx.x, nt = blockDim.x;
  for (int e = t; e < d * k; e += nt) h.Hs[e / k][e % k] = st->Hr[e / k][e % k];
  for (int i = t; i < k; i += nt) {
    h.cs[i] = st->ci[i];
    h.sn[i] = st->si[i];
  }
  if (t == 0) {
    h.gam[k] = st->gamma[k];
    h.acc0 = st->accumulated;
    h.tol = st->tol;
    h.max_steps = st->max_steps;
  }
}

// Hessenberg columns k..k+s-1 from the block's change of basis (c1 + c2 the
// coefficients on q_0..q_k, Rm the Cholesky factor) into Hr, then their
// Givens steps / checks. Called by every thread of one workgroup: the old
// columns, rotations and gamma are staged in LDS (SsHess, staged and synchronised by the caller); X (old columns weighted by
// the change of basis) one thread per entry, the triangular solve
// H_new U = X one thread per row, the k earlier rotations one thread per new
// column, and one thread the block's own rotations and checks column by
// column (a column after the converged one is never used).
__device__ void sstep_hessenberg(GmresDev* st, SsHess& h, const SStepArgs& a, int k,
                                 const double* c1, const double* c2, const double (*Rm)[kSStep],
                                 long long* ss_ts = nullptr) {
  constexpr int S = kSStep;
  __shared__ double Hn[kGmMaxDim + 1][S];
  __shared__ double Hrot[kGmMaxDim + 1][S];
  __shared__ int last_col;
  auto& Hs = h.Hs;
  double* cs = h.cs;
  double* sn = h.sn;
  double* gam = h.gam;
  const int d = k + 1;
  const int rows = k + S + 1;
  const int t = threadIdx.x, nt = blockDim.x;
  SS_STAMP(8);
  auto rhat = [&](int r, int c) -> double {  // Rhat (rows x (S+1)): [e_k | [C; R]]
    if (c == 0) return r == k ? 1.0 : 0.0;
    if (r <= k) return c1[(c - 1) * d + r] + c2[(c - 1) * d + r];
    return Rm[r - k - 1][c - 1];
  };
  // X = Rhat-weighted old columns, one thread per (row, column) pair
  __shared__ double Xs[kGmMaxDim + 1][S];
  __shared__ double hk[S];
  for (int e = t; e < rows * S; e += nt) {
    const int r = e / S, c = e % S;
    double x = a.theta[c] * rhat(r, c) + a.sigma * rhat(r, c + 1);
    if (r <= k && c > 0)
      for (int i = (r > 0 ? r - 1 : 0); i < k; ++i) x -= Hs[r][i] * rhat(i, c);
    Xs[r][c] = x;
  }
  __syncthreads();
  SS_STAMP(9);
  // H_new U = X with U[l][c] = Rhat[k + l][c] (upper triangular), row by row
  if (t < rows) {
    const int r = t;
    double hrow[S];
#pragma unroll
    for (int c = 0; c < S; ++c) {
      double x = Xs[r][c];
      for (int l = 0; l < c; ++l) x -= hrow[l] * rhat(k + l, c);
      hrow[c] = x / rhat(k + c, c);
      Hn[r][c] = hrow[c];
    }
  }
  __syncthreads();
  SS_STAMP(10);
  // the k rotations of the earlier columns, one thread per new column
  if (t < S) {
    const int c = t;
    double hi = Hn[0][c];
#pragma unroll 4
    for (int i = 0; i < k; i++) {
      const double hn = Hn[i + 1][c];
      Hrot[i][c] = cs[i] * hi + sn[i] * hn;
      hi = -sn[i] * hi + cs[i] * hn;
    }
    hk[c] = hi;
  }
  __syncthreads();
  SS_STAMP(11);
  if (t == 0) {
    int acc = h.acc0;
    const double tol = h.tol;
    const int max_steps = h.max_steps;
    // the block's S x S corner of new columns, hk and gamma_k in registers up
    // front, the block's own rotations kept in registers (the loop is fully
    // unrolled; LDS round trips on the serial chain were its cost)
    double hnr[S][S], hkr[S], csr[S], snr[S];
#pragma unroll
    for (int c = 0; c < S; ++c) {
      hkr[c] = hk[c];
#pragma unroll
      for (int i = 0; i < S; ++i) hnr[i][c] = Hn[k + 1 + i][c];  // Hn[kk + 1] for kk = k + i
    }
    double g0 = gam[k];
    last_col = S - 1;
#pragma unroll
    for (int c = 0; c < S; ++c) {
      const int kk = k + c;
      // then the block's own rotations, carrying h[i+1] in a register
      double hi = hkr[c];
#pragma unroll
      for (int i = 0; i < c; i++) {
        const double hn = hnr[i][c];
        Hrot[k + i][c] = csr[i] * hi + snr[i] * hn;
        hi = -snr[i] * hi + csr[i] * hn;
      }
      const double hk1 = hnr[c][c];
      const double r = 1. / sqrt(hi * hi + hk1 * hk1);
      const double s_ = hk1 * r, c_ = hi * r;
      snr[c] = s_;
      csr[c] = c_;
      sn[kk] = s_;
      cs[kk] = c_;
      Hrot[kk][c] = c_ * hi + s_ * hk1;
      const double g1 = -s_ * g0;
      gam[kk + 1] = g1;
      gam[kk] = g0 * c_;
      g0 = g1;
      ++acc;
      const double rho = fabs(g1);
      const int status = rho <= tol ? 1 : ((acc >= max_steps || isnan(rho)) ? 2 : 0);
      if (status || c == S - 1) {
        st->accumulated = acc;
        st->dim = kk + 1;
        st->rho = rho;
        atomicMax(&st->status, status);
        last_col = c;
        break;
      }
    }
  }
  __syncthreads();
  SS_STAMP(12);
  const int nc = last_col + 1;
  // write back: raw and rotated columns, rotations, gamma
  for (int e = t; e < rows * nc; e += nt) {
    const int r = e / nc, c = e % nc, kk = k + c;
    if (r <= kk + 1) st->Hr[r][kk] = Hn[r][c];
    if (r <= kk) st->H[r][kk] = Hrot[r][c];
  }
  for (int c = t; c < nc; c += nt) {
    st->ci[k + c] = cs[k + c];
    st->si[k + c] = sn[k + c];
  }
  for (int i = t; i <= nc; i += nt) st->gamma[k + i] = gam[k + i];
  SS_STAMP(13);
#if DCP_SS_PROBE & 32
  if (t == 0 && ss_ts) {
    const unsigned ph = unsigned(ss_ts[15]) & 63;
    if (ph == 0)
      printf("ssprobe k=%d %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld %lld\n", k,
             ss_ts[1] - ss_ts[0], ss_ts[2] - ss_ts[1], ss_ts[3] - ss_ts[2], ss_ts[4] - ss_ts[3],
             ss_ts[5] - ss_ts[4], ss_ts[6] - ss_ts[5], ss_ts[7] - ss_ts[6], ss_ts[8] - ss_ts[7],
             ss_ts[9] - ss_ts[8], ss_ts[10] - ss_ts[9], ss_ts[11] - ss_ts[10],
             ss_ts[12] - ss_ts[11], ss_ts[13] - ss_ts[12]);
  }
#endif
}

// DCP_SS_NT (timing variant): the block's basis (1) and basis + W (2) loads
// as nontemporal loads, so the up to 28 basis vectors the block streams do not
// push the Schur complement (250 MB at refine 5) out of the 256 MiB Infinity
// Cache between the block's four SpMVs
#ifndef DCP_SS_NT
#define DCP_SS_NT 2
#endif
__device__ inline double ss_ldv(const double* p) {
  if (DCP_SS_NT >= 1) return __builtin_nontemporal_load(p);
  return *p;
}
__device__ inline double ss_ldw(const double* p) {
  if (DCP_SS_NT >= 2) return __builtin_nontemporal_load(p);
  return *p;
}
typedef double ss_d2 __attribute__((ext_vector_type(2)));
__device__ inline ss_d2 ss_ldv2(const double* p) {
  if (DCP_SS_NT >= 1) return __builtin_nontemporal_load(reinterpret_cast<const ss_d2*>(p));
  return *reinterpret_cast<const ss_d2*>(p);
}
__device__ inline ss_d2 ss_ldw2(const double* p) {
  if (DCP_SS_NT >= 2) return __builtin_nontemporal_load(reinterpret_cast<const ss_d2*>(p));
  return *reinterpret_cast<const ss_d2*>(p);
}
// WIDE (one segment, n even, 16-byte aligned vectors): a thread owns the
// adjacent entries b * 1024 + 2 t, + 1 and reads / writes each vector with one
// 16-byte access, else entries b * 1024 + e * 512 + t
template <int KL, bool WIDE>
__global__ __launch_bounds__(kChainThreads) void k_sstep_block(Seg g, ChainVecs V, SStepArgs a,
                                                               int k, GmresDev* st, double* gran,
                                                               unsigned long long seq, double* err) {
  constexpr int K = pow2_at_least<KL>();
  constexpr int S = kSStep;
  static_assert(kChainEntries == 2, "two entries per thread");
  constexpr int G = (KL + 7) / 8;  // slot groups: basis vectors 8 g .. 8 g + 7
  __shared__ double smg[G][kChainWaves * 32];
  __shared__ double sm16[kChainWaves * 16];
  __shared__ double c1[S * 32], c2[S * 32 + 16];
  __shared__ double Rm[S][S];
  __shared__ double Gp[S * (S + 1) / 2];
  __shared__ SsHess hs;
  __shared__ int bad;
  const int nb = gridDim.x, b = blockIdx.x;
  // the Hessenberg workgroup: the last one when it owns no vector entries (a
  // grid of min(CUs, 256) workgroups covers n <= 256 Ki with idle ones at the
  // end), so the Hessenberg columns and Givens steps overlap the other
  // workgroups' last update and q stores; else workgroup 0
  const int hb = long(nb - 1) * (kChainThreads * kChainEntries) >= g.n ? nb - 1 : 0;
#if DCP_SS_PROBE & 32
  __shared__ long long ss_buf[16];
  long long* ss_ts = b == hb ? ss_buf : nullptr;
  if (threadIdx.x == 0) ss_buf[15] = (long long)seq;
#else
  long long* ss_ts = nullptr;
#endif
  SS_STAMP(0);
  if (st->status) return;
  const int d = k + 1;              // basis vectors q_0..q_k
  const int ncol1 = S * d;          // C columns (i * d + j)
  constexpr int nG = S * (S + 1) / 2;
  // two entries per thread (WIDE: adjacent)
  double v[kChainEntries][K], w[kChainEntries][S];
  unsigned pos[kChainEntries];
  bool live[kChainEntries];
  const long kb = long(b) * (kChainThreads * kChainEntries);
  if (WIDE) {
    const long k0 = kb + 2 * long(threadIdx.x);
    live[0] = live[1] = k0 < g.n;  // n even: a pair is all in or all out
    pos[0] = live[0] ? unsigned(k0) : 0u;
    pos[1] = pos[0] + 1;
#pragma unroll
    for (int i = 0; i < S; ++i) {
      const ss_d2 t = live[0] ? ss_ldw2(a.w[i] + pos[0]) : ss_d2{0.0, 0.0};
      w[0][i] = t.x;
      w[1][i] = t.y;
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
      const ss_d2 t = (j < KL && j < d && live[0]) ? ss_ldv2(V.v[j] + pos[0]) : ss_d2{0.0, 0.0};
      v[0][j] = t.x;
      v[1][j] = t.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < kChainEntries; ++e) {
      const long kk = kb + e * kChainThreads + threadIdx.x;
      live[e] = kk < g.n;
      pos[e] = live[e] ? unsigned(seg_pos(g, kk)) : 0u;
#pragma unroll
      for (int i = 0; i < S; ++i) w[e][i] = live[e] ? ss_ldw(a.w[i] + pos[e]) : 0.0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        v[e][j] = (j < KL && j < d && live[e]) ? ss_ldv(V.v[j] + pos[e]) : 0.0;
    }
  }
  if (b == hb) sstep_hess_stage(hs, st, k);  // synchronised by the passes' barriers
  const bool idle = kb >= g.n;  // the workgroup owns no entries
  double* part = gran;
  double* res = gran + kSsRes;
  for (int pass = 0; pass < 2; ++pass) {
    const unsigned long long tag = seq * 256 + 2 * unsigned(pass);
    const int ncol = pass == 0 ? ncol1 : ncol1 + nG;
    if (pass == 1) SS_STAMP(3);
    // block sums of V^T w_i (and, pass 1, of w_a w_b): the wave sums of all
    // of them, one barrier, then the sums over the waves. The products are
    // reduced in groups of 32 slots (w_i . q_j for i < 4 and 8 consecutive j),
    // so group g needs only basis vectors 8 g .. 8 g + 7 and starts while the
    // later ones are still loading; the 10 Gram sums are one 16-slot group.
    // A workgroup that owns no entries publishes +0.0, what those reductions
    // give over its zero entries, without running them.
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (!idle) {
#pragma unroll
      for (int gr = 0; gr < G; ++gr) {
        // every group, without a branch on d (the launch takes the smallest KL
        // >= d = k + 1, so 8 gr < d anyway): one basic block, in which the
        // scheduler overlaps the groups' exchange trees (-0.2 us per column)
        {
          const double r = wave_rs<32>([&](int sl) {
            const int i = sl >> 3, j = 8 * gr + (sl & 7);
            return j < KL ? v[0][j] * w[0][i] + v[1][j] * w[1][i] : 0.0;
          });
          if ((lane & 1) == 0) smg[gr][wv * 32 + (lane >> 1)] = r;
        }
      }
      if (pass == 1) {
        const double r = wave_rs<16>([&](int p) {
          int i = 0, l = p;  // p -> (i, l >= i), row-major upper triangle
          while (l >= S - i) {
            l -= S - i;
            ++i;
          }
          l += i;
          return p < nG ? w[0][i] * w[0][l] + w[1][i] * w[1][l] : 0.0;
        });
        if ((lane & 3) == 0) sm16[wv * 16 + (lane >> 2)] = r;
      }
      __syncthreads();
    }
    for (int c = threadIdx.x; c < ncol1; c += kChainThreads) {
      const int i = c / d, j = c - i * d;
      const double* sp = &smg[j >> 3][i * 8 + (j & 7)];
      double t = 0.0;
      if (!idle)
        for (int q = 0; q < kChainWaves; ++q) t += sp[q * 32];
      granule_store(part + 2 * (size_t(c) * nb + b), t, tag);
    }
    if (pass == 1 && int(threadIdx.x) < nG) {
      double t = 0.0;
      if (!idle)
        for (int q = 0; q < kChainWaves; ++q) t += sm16[q * 16 + threadIdx.x];
      granule_store(part + 2 * (size_t(ncol1 + threadIdx.x) * nb + b), t, tag);
    }
    SS_STAMP(pass == 0 ? 1 : 4);
    // workgroup c reduces column c and publishes the total
    if (b < ncol && threadIdx.x < 64) {
      const double tot = granule_coef(part + 2 * size_t(b) * nb, nb, tag, err, &st->status, g_spin_limit);
      if (threadIdx.x == 0) granule_store(res + 2 * b, tot, tag + 1);
    }
    // an idle workgroup other than the Hessenberg one is done after its last
    // publications (it read the first pass's results, so every reducer of that
    // pass had read the partials its second-pass granules overwrite)
    if (pass == 1 && idle && b != hb) return;
    for (int c = threadIdx.x; c < ncol; c += kChainThreads) {
      const double* p = res + 2 * c;
      mgs_u4 q = granule_load(p);
      for (long spins = 0; !tag_is(q, tag + 1); ++spins) {
        if (spins >= g_spin_limit) {
          handoff_timeout(err, &st->status);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        q = granule_load(p);
      }
      if (pass == 0) c1[c] = granule_value(q);
      else c2[c] = granule_value(q);
    }
    __syncthreads();
    SS_STAMP(pass == 0 ? 2 : 5);
    if (idle) continue;  // no entries to update
    const double* h = pass == 0 ? c1 : c2;
    // basis vector by basis vector: the compiler barrier keeps the LDS loads of
    // the 4 coefficients of vector j next to their use (hoisting all 4 KL of
    // them spills the basis out of registers)
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      if (j < d) {
        double hj[S];
#pragma unroll
        for (int i = 0; i < S; ++i) hj[i] = h[i * d + j];
#pragma unroll
        for (int e = 0; e < kChainEntries; ++e)
#pragma unroll
          for (int i = 0; i < S; ++i) w[e][i] -= hj[i] * v[e][j];
      }
      asm volatile("" ::: "memory");
    }
    __syncthreads();
  }
  // G' = G - C2^T C2 and its Cholesky factor (every workgroup, the same
  // arithmetic in the same order); the idle Hessenberg workgroup gets here
  // straight from the second hand-off, so its Hessenberg columns overlap the
  // others' update and stores
  sstep_factor(c2, d, ncol1, Gp, Rm, &bad);
  SS_STAMP(6);
  // q_{k+1+i} = (w_i - sum_{l<i} q_{k+1+l} R[l][i]) / R[i][i]
#pragma unroll
  for (int e = 0; e < kChainEntries; ++e) {
#pragma unroll
    for (int i = 0; i < S; ++i) {
      double q = w[e][i];
#pragma unroll
      for (int l = 0; l < i; ++l) q -= w[e][l] * Rm[l][i];
      w[e][i] = q / Rm[i][i];
      if (!WIDE && live[e]) a.q[i][pos[e]] = w[e][i];
    }
  }
  if (WIDE && live[0])
#pragma unroll
    for (int i = 0; i < S; ++i)
      *reinterpret_cast<ss_d2*>(a.q[i] + pos[0]) = ss_d2{w[0][i], w[1][i]};
  SS_STAMP(7);
  if (b != hb) return;
  if (bad) {  // the block lost rank: a breakdown the one-vector process would not see
    if (threadIdx.x == 0) {
      atomicMax(&st->status, 2);
      st->rho = __longlong_as_double(0x7ff8000000000000LL);
    }
    return;
  }
  sstep_hessenberg(st, hs, a, k, c1, c2, Rm, ss_ts);
}

// Several GPUs / large meshes: the same block as five launches around two
// all-reduces of the per-rank sums (one reduction per pass, over the owned
// entries of Seg g). PASS 0: c1 = V^T w_i; PASS 1: w_i -= V c1 (written back),
// c2 = V^T w_i and the Gram sums. Each block publishes its sums as granules;
// k_ss_colsum adds them per column in block order.
template <int KL, int PASS>
__global__ __launch_bounds__(kBlock) void k_ss_dots(Seg g, ChainVecs V, SStepArgs a, int k,
                                                    const double* __restrict__ cin, double* gran,
                                                    unsigned long long seq,
                                                    const int* __restrict__ status) {
  constexpr int K = pow2_at_least<KL>();
  constexpr int S = kSStep;
  constexpr int nG = S * (S + 1) / 2;
  __shared__ double sm[4 * (K > 16 ? K : 16)];
  if (*status) return;
  const int d = k + 1, ncol1 = S * d;
  const long k0 = long(blockIdx.x) * (kBlock * kCgsElems) + threadIdx.x;
  double v[kCgsElems][K], w[kCgsElems][S];
  long pos[kCgsElems];
  bool live[kCgsElems];
#pragma unroll
  for (int e = 0; e < kCgsElems; ++e) {
    const long kk = k0 + e * kBlock;
    live[e] = kk < g.n;
    pos[e] = live[e] ? seg_pos(g, kk) : 0;
#pragma unroll
    for (int i = 0; i < S; ++i) w[e][i] = live[e] ? a.w[i][pos[e]] : 0.0;
#pragma unroll
    for (int j = 0; j < K; ++j) v[e][j] = (j < KL && j < d && live[e]) ? V.v[j][pos[e]] : 0.0;
  }
  if (PASS == 1) {
#pragma unroll
    for (int e = 0; e < kCgsElems; ++e) {
#pragma unroll
      for (int i = 0; i < S; ++i) {
#pragma unroll
        for (int j = 0; j < KL; ++j)
          if (j < d) w[e][i] -= cin[i * d + j] * v[e][j];
        if (live[e]) const_cast<double*>(a.w[i])[pos[e]] = w[e][i];
      }
    }
  }
  const int nb = gridDim.x;
  const unsigned long long tag = seq * 256;
#pragma unroll
  for (int i = 0; i < S; ++i) {
    double sj[K];
#pragma unroll
    for (int j = 0; j < K; ++j) sj[j] = v[0][j] * w[0][i] + v[1][j] * w[1][i];
    const double r = block_sums<K>(sj, d, sm);
    if (int(threadIdx.x) < d)
      granule_store(gran + 2 * (size_t(i * d + threadIdx.x) * nb + blockIdx.x), r, tag + 1);
    __syncthreads();
  }
  if (PASS == 1) {
    double sg[16];
    int p = 0;
#pragma unroll
    for (int i = 0; i < S; ++i)
#pragma unroll
      for (int l = i; l < S; ++l, ++p) sg[p] = w[0][i] * w[0][l] + w[1][i] * w[1][l];
#pragma unroll
    for (; p < 16; ++p) sg[p] = 0.0;
    const double r = block_sums<16>(sg, nG, sm);
    if (int(threadIdx.x) < nG)
      granule_store(gran + 2 * (size_t(ncol1 + threadIdx.x) * nb + blockIdx.x), r, tag + 1);
  }
}

// out[c] = the column-c granules of k_ss_dots summed over its nb blocks in a
// fixed order (thread-strided sums, then block_sums): one workgroup per column,
// so the granule reads of all columns are in flight at once (a single
// reducing workgroup reads ~6 MB at refine 6 and is load-latency bound).
__global__ __launch_bounds__(kBlock) void k_ss_colsum(const double* __restrict__ gran, int nb,
                                                      double* out, unsigned long long seq,
                                                      double* err, const int* __restrict__ status,
                                                      int* status_in) {
  __shared__ double sm[4];
  if (blockIdx.x == 0 && threadIdx.x == 0) *status_in = *status;  // for k_ss_final
  if (*status) return;
  const int c = blockIdx.x;
  const unsigned long long tag = seq * 256 + 1;
  double t[1] = {0.0};
  for (int b = threadIdx.x; b < nb; b += kBlock) {
    const double* q = gran + 2 * (size_t(c) * nb + b);
    const unsigned long long* u = reinterpret_cast<const unsigned long long*>(q);
    const unsigned long long vv = __hip_atomic_load(u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long tt = __hip_atomic_load(u + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t[0] += tt == (tag ^ granule_mix(vv)) ? __longlong_as_double((long long)vv)
                                          : granule_poll(q, tag, err);
  }
  const double r = block_sums<1>(t, 1, sm);
  if (threadIdx.x == 0) out[c] = r;
}

// the last of the five launches: w_i -= V c2, the Cholesky factor of the
// corrected Gram matrix, q = W R^-1 (owned entries), block 0 the Hessenberg
// columns and Givens steps
template <int KL>
__global__ __launch_bounds__(kBlock) void k_ss_final(Seg g, ChainVecs V, SStepArgs a, int k,
                                                     const double* __restrict__ c1g,
                                                     const double* __restrict__ c2g, GmresDev* st) {
  constexpr int S = kSStep;
  __shared__ double c1[S * 32], c2[S * 32 + 16];
  __shared__ double Rm[S][S];
  __shared__ double Gp[S * (S + 1) / 2];
  __shared__ SsHess hs;
  __shared__ int bad;
  // not st->status: block 0 sets it below (a stop at this block) while other
  // blocks may not have started; every block must still write its rows of q
  if (st->status_in) return;
  const int d = k + 1, ncol1 = S * d;
  if (blockIdx.x == 0) sstep_hess_stage(hs, st, k);
  for (int c = threadIdx.x; c < ncol1 + S * (S + 1) / 2; c += kBlock) {
    if (c < ncol1) c1[c] = c1g[c];
    c2[c] = c2g[c];
  }
  __syncthreads();
  sstep_factor(c2, d, ncol1, Gp, Rm, &bad);
  const long k0 = long(blockIdx.x) * (kBlock * kCgsElems) + threadIdx.x;
#pragma unroll
  for (int e = 0; e < kCgsElems; ++e) {
    const long kk = k0 + e * kBlock;
    if (kk >= g.n) continue;
    const long pos = seg_pos(g, kk);
    double w[S];
#pragma unroll
    for (int i = 0; i < S; ++i) {
      w[i] = a.w[i][pos];
#pragma unroll
      for (int j = 0; j < KL; ++j)
        if (j < d) w[i] -= c2[i * d + j] * V.v[j][pos];
    }
#pragma unroll
    for (int i = 0; i < S; ++i) {
      double q = w[i];
#pragma unroll
      for (int l = 0; l < i; ++l) q -= w[l] * Rm[l][i];
      w[i] = q / Rm[i][i];
      a.q[i][pos] = w[i];
    }
  }
  if (blockIdx.x != 0) return;
  if (bad) {
    if (threadIdx.x == 0) {
      atomicMax(&st->status, 2);
      st->rho = __longlong_as_double(0x7ff8000000000000LL);
    }
    return;
  }
  sstep_hessenberg(st, hs, a, k, c1, c2, Rm);
}

}  // namespace

int sstep_block_capacity() {
  static const int cap = [] {
    decltype(&k_sstep_block<4, true>) fs[] = {
        k_sstep_block<4, true>,   k_sstep_block<8, true>,   k_sstep_block<12, true>,
        k_sstep_block<16, true>,  k_sstep_block<20, true>,  k_sstep_block<24, true>,
        k_sstep_block<28, true>,  k_sstep_block<4, false>,  k_sstep_block<8, false>,
        k_sstep_block<12, false>, k_sstep_block<16, false>, k_sstep_block<20, false>,
        k_sstep_block<24, false>, k_sstep_block<28, false>};
    return family_capacity(fs);
  }();
  return cap;
}

void sstep_block(Seg g, const ChainVecs& V, const SStepArgs& a, int k, GmresDev* st, double* gran,
                 int nb, unsigned long long seq, double* err, hipStream_t s) {
  ChainVecs Vp = V;
  for (int j = k + 1; j < kGmMaxDim; ++j) Vp.v[j] = V.v[0];
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  bool wide = g.n1 == g.n && g.n % 2 == 0;
  for (int j = 0; j <= k; ++j) wide = wide && al16(V.v[j]);
  for (int i = 0; i < kSStep; ++i) wide = wide && al16(a.w[i]) && al16(a.q[i]);
#define DCP_SS_CASE(KL)                                                                          \
  if (k + 1 <= KL) {                                                                             \
    if (wide)                                                                                    \
      launch_resident(k_sstep_block<KL, true>, nb, kChainThreads, s, g, Vp, a, k, st, gran, seq,  \
                      err);                                                                      \
    else                                                                                         \
      launch_resident(k_sstep_block<KL, false>, nb, kChainThreads, s, g, Vp, a, k, st, gran, seq, \
                      err);                                                                      \
    return;                                                                                      \
  }
  DCP_SS_CASE(4) DCP_SS_CASE(8) DCP_SS_CASE(12) DCP_SS_CASE(16) DCP_SS_CASE(20) DCP_SS_CASE(24)
  DCP_SS_CASE(28)
#undef DCP_SS_CASE
  throw std::runtime_error("sstep_block: basis too long");
}

void sstep_block_multi(Seg g, const ChainVecs& V, const SStepArgs& a, int k, GmresDev* st,
                       double* gran, unsigned* cnt, double* c1, double* c2,
                       unsigned long long& seq, double* err, Comm* comm, hipStream_t s) {
  ChainVecs Vp = V;
  for (int j = k + 1; j < kGmMaxDim; ++j) Vp.v[j] = V.v[0];
  // a rank with no owned pressure rows still runs one (empty) block per launch:
  // it joins both all-reduces and block 0 of k_ss_final runs the Hessenberg
  // columns, Givens steps and status like every other rank
  const int nb = std::max(1, int((long(g.n) + kBlock * kCgsElems - 1) / (kBlock * kCgsElems)));
  const int ncol1 = kSStep * (k + 1), ncol2 = ncol1 + kSStep * (kSStep + 1) / 2;
  const int* status = &st->status;
  {
#define DCP_SSM(KL)                                                                              \
  if (k + 1 <= KL) {                                                                             \
    hipLaunchKernelGGL((k_ss_dots<KL, 0>), dim3(nb), dim3(kBlock), 0, s, g, Vp, a, k, nullptr,   \
                       gran, ++seq, status);                                                     \
    DCP_HIP_CHECK(hipGetLastError());                                                            \
    hipLaunchKernelGGL(k_ss_colsum, dim3(ncol1), dim3(kBlock), 0, s, gran, nb, c1, seq, err,     \
                       status, &st->status_in);                                                  \
    DCP_HIP_CHECK(hipGetLastError());                                                            \
    if (comm) comm->allreduce(c1, size_t(ncol1), false, s);                                      \
    hipLaunchKernelGGL((k_ss_dots<KL, 1>), dim3(nb), dim3(kBlock), 0, s, g, Vp, a, k, c1, gran, \
                       ++seq, status);                                                           \
    DCP_HIP_CHECK(hipGetLastError());                                                            \
    hipLaunchKernelGGL(k_ss_colsum, dim3(ncol2), dim3(kBlock), 0, s, gran, nb, c2, seq, err,     \
                       status, &st->status_in);                                                  \
    DCP_HIP_CHECK(hipGetLastError());                                                            \
    if (comm) comm->allreduce(c2, size_t(ncol2), false, s);                                      \
    hipLaunchKernelGGL((k_ss_final<KL>), dim3(nb), dim3(kBlock), 0, s, g, Vp, a, k, c1, c2, st); \
    DCP_HIP_CHECK(hipGetLastError());                                                            \
    return;                                                                                      \
  }
    DCP_SSM(4) DCP_SSM(8) DCP_SSM(12) DCP_SSM(16) DCP_SSM(20) DCP_SSM(24) DCP_SSM(28)
#undef DCP_SSM
    throw std::runtime_error("sstep_block_multi: basis too long");
  }
}

size_t cgs2_granules(long n) {
  return 2 * size_t(kGmMaxDim) *
             std::max<size_t>(1, size_t((n + kBlock * kCgsElems - 1) / (kBlock * kCgsElems))) +
         2;
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

// ---------------------------------------------------------------------------
// DCGS2: delayed classical Gram-Schmidt, one reduction per Arnoldi step.
// Step k holds the final basis q_0..q_{k-1} (V[0..k)), the tentative t_k
// (V[k]: once orthogonalised at step k - 1 and scaled by the Pythagorean
// norm estimate) and w = S t_k. Its one reduction is
//   slots [0, k): a_i = q_i.t      slot KP - 1: alpha = t.t
//   slots [KP, KP + k): z_i = q_i.w   2 KP - 2: zeta = t.w   2 KP - 1: omega = w.w
// (KP a power of two >= KL + 2, K = 2 KP slots, unused slots idle). Then, with
// beta = sqrt(alpha - |a|^2) (k > 0; q_0 = t_0 is exact: beta = 1),
//   q_k = (t - V a) / beta                       (the delayed second pass)
//   g = [z; (zeta - a.z) / beta] = Q_{k+1}^T w
//   u = w - V z - g_k q_k,  nu^2 = omega - |g|^2, t_{k+1} = u / nu
// and the Arnoldi relation S q_k = (w - S V a) / beta gives the provisional
// column H[:k+1, k] = (g - H[:k+1, :k] a) / beta, corrected one step later by
// the reorthogonalisation of t_{k+1}: H[:k+1, k] += (nu/beta) a',
// H[k+1, k] = (nu/beta) beta'. The column's Givens rotation and SolverControl
// check therefore run one step late (its residual estimate is exactly the
// one deal.II checks after step k; only one extra S apply at the end of a
// solve is wasted), and the cycle ends with a tail launch that only corrects
// its last column.
template <int KL>
constexpr int dcgs_kp() { return pow2_at_least<KL + 2>(); }

// Timing probe builds only (-DDCP_DCGS_TIMING=k, tools/dcgs_timing.py): the
// step with basis size k records per-workgroup realtime stamps (100 MHz) at
// its phase boundaries.
#ifdef DCP_DCGS_TIMING
__device__ unsigned long long g_dcgs_ts[256 * 8];
#define DCGS_TS(slot)                                                                  \
  do {                                                                                 \
    if (k == DCP_DCGS_TIMING && threadIdx.x == 0) g_dcgs_ts[8 * blockIdx.x + (slot)] = \
        wall_clock64();                                                                \
  } while (0)
#else
#define DCGS_TS(slot) \
  do {                \
  } while (0)
#endif
// result granules after the partial area (2 K nb <= 2 * 64 * 256 doubles)
constexpr int kDcgsRes = 2 * 64 * 256;

template <int KP>
__device__ inline bool dcgs_used(int j, int k, bool tail) {
  if (j < KP) return j < k || j == KP - 1;
  return !tail && (j - KP < k || j >= 2 * KP - 2);
}

// The scalars of the step from the reduced slots r[] (every workgroup computes
// them identically): beta, g_k, 1/nu.
struct DcgsScalars {
  double beta, gk, inv_nu, nu;
};
template <int KP>
__device__ inline DcgsScalars dcgs_scalars(const double* r, int k, bool tail) {
  DcgsScalars c;
  double aa = 0, az = 0, zz = 0;
  for (int i = 0; i < k; ++i) {
    aa += r[i] * r[i];
    az += r[i] * r[KP + i];
    zz += r[KP + i] * r[KP + i];
  }
  c.beta = k > 0 ? sqrt(fmax(r[KP - 1] - aa, 0.0)) : 1.0;
  if (tail) {
    c.gk = 0;
    c.nu = 0;
    c.inv_nu = 1;
    return c;
  }
  c.gk = (r[2 * KP - 2] - az) / c.beta;
  const double nu2 = r[2 * KP - 1] - zz - c.gk * c.gk;
  c.nu = sqrt(fmax(nu2, 0.0));
  c.inv_nu = c.nu != 0 ? 1.0 / c.nu : 1.0;
  return c;
}

// Workgroup 0 after the reduction: correct column k - 1 of the raw Hessenberg,
// its Givens rotation (solver_gmres.h givens_rotation) on the rotated copy,
// the residual estimate and SolverControl::check; then the provisional column
// k. r[] in LDS (the reduced slots), every thread of the workgroup calls.
template <int KP>
__device__ void dcgs_bookkeeping(GmresDev* st, const double* r, int k, bool tail,
                                 const DcgsScalars& c) {
  __shared__ double h[kGmMaxDim + 1], hp[kGmMaxDim + 1];
  __shared__ int stop;
  const int t = threadIdx.x;
  if (k > 0) {
    const int col = k - 1;
    const double cp = st->c_pend;
    if (t < k) h[t] = st->Hr[t][col] + cp * r[t];
    if (t == k) h[t] = cp * c.beta;
    __syncthreads();
    if (t <= k) st->Hr[t][col] = h[t];
    if (t == 0) {
      for (int i = 0; i < col; i++) {
        const double cs = st->ci[i], sn = st->si[i], dummy = h[i];
        h[i] = cs * dummy + sn * h[i + 1];
        h[i + 1] = -sn * dummy + cs * h[i + 1];
      }
      const double rr = 1. / sqrt(h[col] * h[col] + h[col + 1] * h[col + 1]);
      const double sn = h[col + 1] * rr, cs = h[col] * rr;
      st->si[col] = sn;
      st->ci[col] = cs;
      h[col] = cs * h[col] + sn * h[col + 1];
      const double g0 = st->gamma[col];
      const double gk1 = -sn * g0;
      st->gamma[col + 1] = gk1;
      st->gamma[col] = g0 * cs;
      const int acc = st->accumulated + 1;
      st->accumulated = acc;
      st->dim = k;
      const double rho = fabs(gk1);
      st->rho = rho;
      const int status = rho <= st->tol ? 1 : ((acc >= st->max_steps || isnan(rho)) ? 2 : 0);
      atomicMax(&st->status, status);
      stop = status;
    }
    __syncthreads();
    if (t <= col) st->H[t][col] = h[t];
  } else if (t == 0) {
    stop = 0;
  }
  __syncthreads();
  if (tail || stop) return;
  // provisional column k: (g - H[:k+1, :k] a) / beta, rows i <= k (Hessenberg:
  // H[i][j] = 0 for i > j + 1)
  if (t <= k) {
    double s = t < k ? r[KP + t] : c.gk;
    for (int j = t > 0 ? t - 1 : 0; j < k; ++j) s -= st->Hr[t][j] * r[j];
    hp[t] = s / c.beta;
  }
  __syncthreads();
  if (t <= k) st->Hr[t][k] = hp[t];
  if (t == 0) st->c_pend = c.nu / c.beta;
}

// One GPU: the whole DCGS2 step in one launch of nb resident 512-thread
// workgroups, two vector entries per thread (16-byte loads when WIDE), the k
// basis entries in registers from the loads to the update. The reduction is
// two granule hops as in k_cgs2_chain (every workgroup publishes its slot
// sums, workgroup j sums slot j, every workgroup reads the results).
template <int KL, bool WIDE>
__global__ __launch_bounds__(kChainThreads) void k_dcgs2_step(Seg g, const double* w, ChainVecs V,
                                                              int k, double* tnext, GmresDev* st,
                                                              double* gran, unsigned long long seq,
                                                              double* err) {
  constexpr int KP = dcgs_kp<KL>();
  constexpr int K = 2 * KP;
  __shared__ double sm[kChainWaves * K];
  __shared__ double hs[K];
  DCGS_TS(0);
  if (st->status) return;
  const bool tail = tnext == nullptr;
  const int nb = gridDim.x, b = blockIdx.x;
  double tv[kChainEntries], wv[kChainEntries], v[kChainEntries][KL];
  unsigned pos[kChainEntries];
  bool live[kChainEntries];
  const double* t_in = V.v[k];
  const long kb = long(b) * (kChainThreads * kChainEntries);
  if (WIDE) {
    const long k0 = kb + 2 * long(threadIdx.x);
    live[0] = live[1] = k0 < g.n;
    pos[0] = live[0] ? unsigned(k0) : 0u;
    pos[1] = pos[0] + 1;
    const double2 tw = *reinterpret_cast<const double2*>(t_in + pos[0]);
    tv[0] = tw.x;
    tv[1] = tw.y;
    double2 ww = {0.0, 0.0};
    if (!tail) ww = *reinterpret_cast<const double2*>(w + pos[0]);
    wv[0] = ww.x;
    wv[1] = ww.y;
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      const double2 a = *reinterpret_cast<const double2*>(V.v[j] + pos[0]);
      v[0][j] = a.x;
      v[1][j] = a.y;
    }
  } else {
#pragma unroll
    for (int e = 0; e < kChainEntries; ++e) {
      const long kk = kb + e * kChainThreads + threadIdx.x;
      live[e] = kk < g.n;
      pos[e] = live[e] ? unsigned(seg_pos(g, kk)) : 0u;
      tv[e] = t_in[pos[e]];
      wv[e] = tail ? 0.0 : w[pos[e]];
#pragma unroll
      for (int j = 0; j < KL; ++j) v[e][j] = V.v[j][pos[e]];
    }
  }
#pragma unroll
  for (int e = 0; e < kChainEntries; ++e) {
    tv[e] = live[e] ? tv[e] : 0.0;
    wv[e] = live[e] ? wv[e] : 0.0;
#pragma unroll
    for (int j = 0; j < KL; ++j) v[e][j] = live[e] && j < k ? v[e][j] : 0.0;
  }
  auto prod = [&](int j) -> double {
    if (j < KL) return v[0][j] * tv[0] + v[1][j] * tv[1];
    if (j == KP - 1) return tv[0] * tv[0] + tv[1] * tv[1];
    if (j >= KP && j < KP + KL) return v[0][j - KP] * wv[0] + v[1][j - KP] * wv[1];
    if (j == 2 * KP - 2) return tv[0] * wv[0] + tv[1] * wv[1];
    if (j == 2 * KP - 1) return wv[0] * wv[0] + wv[1] * wv[1];
    return 0.0;
  };
  {
    const double r = wave_rs<K>(prod);
    const int l = threadIdx.x & 63, wv_ = threadIdx.x >> 6;
    constexpr int sh = 6 - log2i<K>();
    if ((l & ((1 << sh) - 1)) == 0) sm[wv_ * K + (l >> sh)] = r;
  }
  __syncthreads();
  DCGS_TS(1);
  double* part = gran;
  double* res = gran + kDcgsRes;
  const unsigned long long tag = seq * 128;
  const int j = threadIdx.x;
  const bool used = j < K && dcgs_used<KP>(j, k, tail);
  if (used) {
    double tot = 0.0;
    for (int i = 0; i < kChainWaves; ++i) tot += sm[i * K + j];
    granule_store(part + 2 * (size_t(j) * nb + b), tot, tag + j);
  }
  // reducer: workgroup b sums slot b over the nb workgroups
  DCGS_TS(2);
  if (b < K && dcgs_used<KP>(b, k, tail) && threadIdx.x < 64) {
    const double tot = granule_coef(part + 2 * size_t(b) * nb, nb, tag + b, err, &st->status, g_spin_limit);
    if (threadIdx.x == 0) granule_store(res + 2 * b, tot, tag + K + b);
  }
  DCGS_TS(3);
  if (used) {
    const double* p = res + 2 * j;
    mgs_u4 q = granule_load(p);
    for (long spins = 0; !tag_is(q, tag + K + j); ++spins) {
      if (spins >= g_spin_limit) {
        handoff_timeout(err, &st->status);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
      q = granule_load(p);
    }
    hs[j] = granule_value(q);
  } else if (j < K) {
    hs[j] = 0.0;
  }
  __syncthreads();
  DCGS_TS(4);
  const DcgsScalars c = dcgs_scalars<KP>(hs, k, tail);
  if (!tail || k > 0) {
    const double ib = 1.0 / c.beta;
#pragma unroll
    for (int e = 0; e < kChainEntries; ++e) {
      double q = tv[e];
      if (k > 0) {
#pragma unroll
        for (int i = 0; i < KL; ++i)
          if (i < k) q -= hs[i] * v[e][i];
        q *= ib;
      }
      if (!tail) {
        double u = wv[e];
#pragma unroll
        for (int i = 0; i < KL; ++i)
          if (i < k) u -= hs[KP + i] * v[e][i];
        u -= c.gk * q;
        if (live[e]) tnext[pos[e]] = u * c.inv_nu;
      }
      if (k > 0 && live[e]) const_cast<double*>(t_in)[pos[e]] = q;
    }
  }
  DCGS_TS(5);
  if (b != 0) return;
  dcgs_bookkeeping<KP>(st, hs, k, tail, c);
  DCGS_TS(6);
}

// Several GPUs (or vectors too long for one resident launch): block sums of
// the used slots as granules, the last block to arrive sums them in block
// order into st->coef[0, K) (all-reduced across ranks by the host before the
// update launch).
template <int KL>
__global__ __launch_bounds__(kBlock) void k_dcgs_partials(Seg g, const double* __restrict__ w,
                                                          ChainVecs V, int k, bool tail,
                                                          double* gran, unsigned* cnt,
                                                          GmresDev* st, unsigned long long seq,
                                                          double* err) {
  constexpr int KP = dcgs_kp<KL>();
  constexpr int K = 2 * KP;
  __shared__ double sm[4 * K];
  __shared__ int is_last;
  if (blockIdx.x == 0 && threadIdx.x == 0) st->status_in = st->status;  // for k_dcgs_update
  if (st->status) return;
  double s[K];
#pragma unroll
  for (int j = 0; j < K; ++j) s[j] = 0.0;
  const long k0 = long(blockIdx.x) * (kBlock * kCgsElems) + threadIdx.x;
#pragma unroll
  for (int e = 0; e < kCgsElems; ++e) {
    const long kk = k0 + e * kBlock;
    if (kk >= g.n) continue;
    const long i = seg_pos(g, kk);
    const double t = V.v[k][i];
    const double wv = tail ? 0.0 : w[i];
#pragma unroll
    for (int j = 0; j < KL; ++j) {
      const double vj = j < k ? V.v[j][i] : 0.0;
      s[j] += vj * t;
      s[KP + j] += vj * wv;
    }
    s[KP - 1] += t * t;
    s[2 * KP - 2] += t * wv;
    s[2 * KP - 1] += wv * wv;
  }
  const double r = block_sums<K>(s, K, sm);
  const int nb = gridDim.x;
  const int j = threadIdx.x;
  if (j < K && dcgs_used<KP>(j, k, tail))
    granule_store(gran + 2 * (size_t(j) * nb + blockIdx.x), r, seq * 128 + j);
  if (!last_block(cnt, &is_last)) return;
  // the last block: slot j summed over the blocks (per-thread strided sums,
  // then block_sums: a fixed order); unused slots stay 0
  double s2[K];
#pragma unroll
  for (int jj = 0; jj < K; ++jj) {
    s2[jj] = 0.0;
    if (dcgs_used<KP>(jj, k, tail))
      for (int bb = threadIdx.x; bb < nb; bb += kBlock) {
        const double* p = gran + 2 * (size_t(jj) * nb + bb);
        mgs_u4 q = granule_load(p);
        for (long spins = 0; !tag_is(q, seq * 128 + jj); ++spins) {
          if (spins >= kMgsMaxSpins) {
            *err = 1.0;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          q = granule_load(p);
        }
        s2[jj] += granule_value(q);
      }
  }
  __syncthreads();
  const double r2 = block_sums<K>(s2, K, sm);
  if (j < K) st->coef[j] = r2;
}

// The update and bookkeeping of a DCGS2 step from the (all-reduced) slots in
// st->coef.
template <int KL>
__global__ __launch_bounds__(kBlock) void k_dcgs_update(Seg g, const double* __restrict__ w,
                                                        ChainVecs V, int k, double* tnext,
                                                        GmresDev* st) {
  constexpr int KP = dcgs_kp<KL>();
  constexpr int K = 2 * KP;
  __shared__ double hs[K];
  // not st->status: block 0's bookkeeping may stop the cycle while other
  // blocks have not started; every block must still write its rows
  if (st->status_in) return;
  const bool tail = tnext == nullptr;
  if (int(threadIdx.x) < K) hs[threadIdx.x] = st->coef[threadIdx.x];
  __syncthreads();
  const DcgsScalars c = dcgs_scalars<KP>(hs, k, tail);
  const double ib = 1.0 / c.beta;
  double* t_io = const_cast<double*>(V.v[k]);
  for (long kk = long(blockIdx.x) * kBlock + threadIdx.x; kk < g.n;
       kk += long(gridDim.x) * kBlock) {
    const long i = seg_pos(g, kk);
    double q = t_io[i];
    if (k > 0) {
      for (int j = 0; j < k; ++j) q -= hs[j] * V.v[j][i];
      q *= ib;
    }
    if (!tail) {
      double u = w[i];
      for (int j = 0; j < k; ++j) u -= hs[KP + j] * V.v[j][i];
      u -= c.gk * q;
      tnext[i] = u * c.inv_nu;
    }
    if (k > 0) t_io[i] = q;
  }
  if (blockIdx.x != 0) return;
  dcgs_bookkeeping<KP>(st, hs, k, tail, c);
}

namespace {
int dcgs2_capacity() {
  static const int cap = [] {
    decltype(&k_dcgs2_step<4, true>) fs[] = {
        k_dcgs2_step<4, true>,   k_dcgs2_step<8, true>,   k_dcgs2_step<12, true>,
        k_dcgs2_step<16, true>,  k_dcgs2_step<20, true>,  k_dcgs2_step<24, true>,
        k_dcgs2_step<28, true>,  k_dcgs2_step<4, false>,  k_dcgs2_step<8, false>,
        k_dcgs2_step<12, false>, k_dcgs2_step<16, false>, k_dcgs2_step<20, false>,
        k_dcgs2_step<24, false>, k_dcgs2_step<28, false>};
    return family_capacity(fs);
  }();
  return cap;
}
}  // namespace

bool dcgs2_fits(long n, int nb, int n_cus) {
  return cgs2_chain_fits(n, nb, n_cus) && nb <= dcgs2_capacity();
}

#ifdef DCP_DCGS_TIMING
extern "C" int dcp_probe_dcgs_timestamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dcgs_ts), sizeof(g_dcgs_ts)) == hipSuccess ? 0 : -1;
}
#endif

size_t dcgs2_granules(long n) {
  const size_t nbp = std::max<size_t>(1, size_t((n + kBlock * kCgsElems - 1) / (kBlock * kCgsElems)));
  return std::max<size_t>(kDcgsRes + 2 * 64 + 64, 2 * 64 * nbp + 64);
}

void dcgs2_step(Seg g, const double* w, const ChainVecs& V, int k, double* tnext, GmresDev* st,
                double* gran, unsigned* cnt, int nb, unsigned long long& seq, double* err,
                Comm* comm, bool one_launch, hipStream_t s) {
  ChainVecs Vp = V;  // slots past k point at V[0]: the one-launch kernel loads them unconditionally
  for (int j = k + 1; j < kGmMaxDim; ++j) Vp.v[j] = V.v[0];
  const bool tail = tnext == nullptr;
  if (one_launch) {
    bool wide = g.n1 == g.n && g.n % 2 == 0 && (reinterpret_cast<uintptr_t>(tnext) & 15) == 0 &&
                (reinterpret_cast<uintptr_t>(w) & 15) == 0;
    for (int j = 0; j <= k; ++j) wide = wide && (reinterpret_cast<uintptr_t>(V.v[j]) & 15) == 0;
    ++seq;
#define DCP_DCGS_CASE(KL)                                                                       \
    if (k <= KL) {                                                                              \
      if (wide)                                                                                 \
        launch_resident(k_dcgs2_step<KL, true>, nb, kChainThreads, s, g, w, Vp, k, tnext, st,   \
                        gran, seq, err);                                                        \
      else                                                                                      \
        launch_resident(k_dcgs2_step<KL, false>, nb, kChainThreads, s, g, w, Vp, k, tnext, st,  \
                        gran, seq, err);                                                        \
      return;                                                                                   \
    }
    DCP_DCGS_CASE(4) DCP_DCGS_CASE(8) DCP_DCGS_CASE(12) DCP_DCGS_CASE(16) DCP_DCGS_CASE(20)
    DCP_DCGS_CASE(24) DCP_DCGS_CASE(28)
#undef DCP_DCGS_CASE
    throw std::runtime_error("dcgs2_step: basis of " + std::to_string(k) + " vectors");
  }
  // at least one (empty) block on a rank without owned rows: it joins the
  // all-reduce and does the bookkeeping like the others
  const int nbp = std::max(1, int((long(g.n) + kBlock * kCgsElems - 1) / (kBlock * kCgsElems)));
  const int nbu = int(std::min<long>((long(g.n) + kBlock - 1) / kBlock, 2048));
  ++seq;
#define DCP_DCGS_CASE2(KL)                                                                       \
  if (k <= KL) {                                                                                 \
    hipLaunchKernelGGL((k_dcgs_partials<KL>), dim3(nbp), dim3(kBlock), 0, s, g, w, Vp, k, tail,  \
                       gran, cnt, st, seq, err);                                                 \
    DCP_HIP_CHECK(hipGetLastError());                                                            \
    if (comm) comm->allreduce(st->coef, size_t(2 * dcgs_kp<KL>()), false, s);                    \
    hipLaunchKernelGGL((k_dcgs_update<KL>), dim3(std::max(nbu, 1)), dim3(kBlock), 0, s, g, w, Vp, \
                       k, tnext, st);                                                            \
    DCP_HIP_CHECK(hipGetLastError());                                                            \
    return;                                                                                      \
  }
  DCP_DCGS_CASE2(8) DCP_DCGS_CASE2(16) DCP_DCGS_CASE2(28)
#undef DCP_DCGS_CASE2
  throw std::runtime_error("dcgs2_step: basis of " + std::to_string(k) + " vectors");
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

__global__ __launch_bounds__(kBlock) void k_gmres_head(GmresDev* st, const double* __restrict__ part,
                                                       int n_part, double tol, int max_steps,
                                                       int first, int n,
                                                       const double* __restrict__ p,
                                                       double* __restrict__ v0) {
  __shared__ double red[kBlock];
  const int t = threadIdx.x;
  double sum = 0.0;
  for (int i = t; i < n_part; i += kBlock) sum += part[i];
  red[t] = sum;
  __syncthreads();
#pragma unroll
  for (int o = kBlock / 2; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  const double rho = sqrt(red[0]);
  // workgroup 0 may already have moved status 0 -> s; a reader that sees s
  // skips v0, which the stopped cycle never uses
  const int s0 = first ? 0 : st->status;
  const int acc = first ? 0 : st->accumulated;
  const int status = s0 != 0 ? s0 : (rho <= tol ? 1 : ((acc >= max_steps || isnan(rho)) ? 2 : 0));
  if (blockIdx.x == 0 && t == 0) {
    if (first) {
      st->accumulated = 0;
      st->tol = tol;
      st->max_steps = max_steps;
    }
    st->dim = 0;
    if (s0 == 0) {
      st->rho = rho;
      st->status = status;
      if (status == 0) {
        st->gamma[0] = rho;
        st->inv_rho = 1.0 / rho;
        st->inv_norm = 1.0;
      }
    }
  }
  if (status != 0) return;
  const double cf = 1.0 * (1.0 / rho);
  for (long i = long(blockIdx.x) * kBlock + t; i < n; i += long(gridDim.x) * kBlock) v0[i] = cf * p[i];
}

__global__ __launch_bounds__(kBlock) void k_gmres_finish(GmresDev* st, int n,
                                                         const double* const* V,
                                                         double* __restrict__ x,
                                                         GmresReport* report) {
  __shared__ double H[kGmMaxDim][kGmMaxDim + 1], gam[kGmMaxDim], y[kGmMaxDim];
  const int dim = st->dim;
  const int t = threadIdx.x;
  if (blockIdx.x == 0 && t == 0) {
    report->rho = st->rho;
    report->status = st->status;
    report->accumulated = st->accumulated;
  }
  if (dim <= 0) return;
  for (int e = t; e < dim * dim; e += kBlock) H[e / dim][e % dim] = st->H[e / dim][e % dim];
  if (t < dim) gam[t] = st->gamma[t];
  __syncthreads();
  if (t == 0) {
    // k_gmres_backsub's order, y in registers (the LDS round trips of the
    // one-thread loop were its whole cost)
    double yr[kGmMaxDim];
#pragma unroll
    for (int i = kGmMaxDim - 1; i >= 0; --i) {
      if (i < dim) {
        double sum = gam[i];
#pragma unroll
        for (int j = i + 1; j < kGmMaxDim; ++j)
          if (j < dim) sum -= yr[j] * H[i][j];
        yr[i] = sum / H[i][i];
      } else {
        yr[i] = 0.0;
      }
    }
#pragma unroll
    for (int i = 0; i < kGmMaxDim; ++i) y[i] = yr[i];
  }
  __syncthreads();
  if (blockIdx.x == 0 && t < dim) st->y[t] = y[t];
  for (long i = long(blockIdx.x) * kBlock + t; i < n; i += long(gridDim.x) * kBlock) {
    double v = x[i];
    for (int j = 0; j < dim; ++j) v += y[j] * V[j][i];
    x[i] = v;
  }
}


void gmres_cycle_init(GmresDev* st, const double* rho2, double tol, int max_steps, bool first,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_gmres_cycle_init, dim3(1), dim3(64), 0, s, st, rho2, tol, max_steps,
                     int(first));
  DCP_HIP_CHECK(hipGetLastError());
}

void gmres_cycle_end(GmresDev* st, int n, const double* const* V, double* x, GmresReport* report,
                     hipStream_t s) {
  gmres_cycle_finish(st, n, V, x, report, s);
}

void gmres_cycle_head(GmresDev* st, const double* part, int n_part, double tol, int max_steps,
                      bool first, int n, const double* p, double* v0, hipStream_t s) {
  const long blocks = std::min<long>((long(n) + kBlock - 1) / kBlock, 1024);
  hipLaunchKernelGGL(k_gmres_head, dim3(unsigned(std::max<long>(blocks, 1))), dim3(kBlock), 0, s,
                     st, part, n_part, tol, max_steps, int(first), n, p, v0);
  DCP_HIP_CHECK(hipGetLastError());
}

void gmres_cycle_finish(GmresDev* st, int n, const double* const* V, double* x,
                        GmresReport* report, hipStream_t s) {
  const long blocks = std::min<long>((long(n) + kBlock - 1) / kBlock, 1024);
  hipLaunchKernelGGL(k_gmres_finish, dim3(unsigned(std::max<long>(blocks, 1))), dim3(kBlock), 0, s,
                     st, n, V, x, report);
  DCP_HIP_CHECK(hipGetLastError());
}

void gmres_backsub(GmresDev* st, hipStream_t s) {
  hipLaunchKernelGGL(k_gmres_backsub, dim3(1), dim3(kBlock), 0, s, st);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
