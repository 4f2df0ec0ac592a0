// Tagged 16-byte hand-off granules {value, tag ^ mix(value)} between
// workgroups of one launch (kernels/linalg.hip k_mgs_chain, kernels/krylov.hip):
// written by one `sc1` vector store, read by `sc1` vector loads (agent-
// coherent without fences); the tag is never reused, so a reader simply polls
// until the tag it expects appears.
#pragma once
#include <hip/hip_runtime.h>

#include "lanes.h"

namespace dcp {

typedef unsigned int mgs_u4 __attribute__((ext_vector_type(4)));

// The tag half of a granule carries tag ^ mix(value bits): the memory model
// guarantees single-copy atomicity only up to 64 bits, so a reader could see
// the two halves of a 16-byte access from different writes; such a torn read
// (new tag with an old value, or the reverse) fails the check below and is
// simply polled again (a false match needs a 64-bit hash collision).
__device__ inline unsigned long long granule_mix(unsigned long long x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}
__device__ inline void granule_store(double* p, double v, unsigned long long tag) {
  const unsigned long long b = __double_as_longlong(v);
  const unsigned long long t = tag ^ granule_mix(b);
  mgs_u4 q;
  q.x = unsigned(b);
  q.y = unsigned(b >> 32);
  q.z = unsigned(t);
  q.w = unsigned(t >> 32);
  asm volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(q) : "memory");
}

__device__ inline bool tag_is(const mgs_u4& q, unsigned long long tag) {
  const unsigned long long t = tag ^ granule_mix(((unsigned long long)q.y << 32) | q.x);
  return q.z == unsigned(t) && q.w == unsigned(t >> 32);
}
__device__ inline double granule_value(const mgs_u4& q) {
  return __longlong_as_double((long long)(((unsigned long long)q.y << 32) | q.x));
}

#ifndef DCP_MGS_SLEEP
#define DCP_MGS_SLEEP 1
#endif
// A hand-off normally completes in microseconds; ~2^19 polls (tenths of a
// second) mean a producer never ran (the grid was not all resident).
constexpr long kMgsMaxSpins = 1L << 19;

// Timed out waiting for a hand-off: the host flag (err, mapped memory) and,
// with a device GMRES state, status 3 so every later launch of the solve
// returns at entry and the host's cycle loop stops at the next report instead
// of spinning through thousands of stuck launches.
__device__ inline void handoff_timeout(double* err, int* status) {
  *err = 1.0;
  if (status) atomicMax(status, 3);
}

// Wave 0 only: waits for the nb <= 256 granules of one step (lane l polls
// granules l, l+64, l+128, l+192, four `sc1` loads in flight) and returns, in
// every lane, their sum in exactly block_sum's order (thread t holds granule
// t; xor butterfly per 64-thread wave; the four wave sums left to right).
__device__ inline double granule_coef(const double* gran, int nb, unsigned long long tag,
                                      double* err, int* status = nullptr,
                                      long max_spins = kMgsMaxSpins) {
  const int l = threadIdx.x & 63;
  const double* p = gran + 2 * size_t(l);
  mgs_u4 q0, q1, q2, q3;
  long spins = 0;
  for (;;) {
    asm volatile(
        "global_load_dwordx4 %0, %4, off sc1\n\t"
        "global_load_dwordx4 %1, %4, off offset:1024 sc1\n\t"
        "global_load_dwordx4 %2, %4, off offset:2048 sc1\n\t"
        "global_load_dwordx4 %3, %4, off offset:3072 sc1\n\t"
        "s_waitcnt vmcnt(0)"
        : "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3)
        : "v"(p)
        : "memory");
    const bool ok = (l >= nb || tag_is(q0, tag)) && (l + 64 >= nb || tag_is(q1, tag)) &&
                    (l + 128 >= nb || tag_is(q2, tag)) && (l + 192 >= nb || tag_is(q3, tag));
    if (__all(ok)) break;
    if (++spins >= max_spins) {
      if (l == 0) handoff_timeout(err, status);
      break;
    }
    if (DCP_MGS_SLEEP) __builtin_amdgcn_s_sleep(DCP_MGS_SLEEP);
  }
  double v[4] = {l < nb ? granule_value(q0) : 0.0, l + 64 < nb ? granule_value(q1) : 0.0,
                 l + 128 < nb ? granule_value(q2) : 0.0, l + 192 < nb ? granule_value(q3) : 0.0};
#pragma unroll
  for (int w = 0; w < 4; ++w) v[w] = wave_allsum(v[w]);
  return v[0] + v[1] + v[2] + v[3];
}

// one `sc1` load of a granule
__device__ inline mgs_u4 granule_load(const double* p) {
  mgs_u4 q;
  asm volatile("global_load_dwordx4 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(q) : "v"(p) : "memory");
  return q;
}

}  // namespace dcp
