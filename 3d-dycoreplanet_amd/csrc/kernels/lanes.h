// Lane exchanges of doubles over a wave without the LDS crossbar
// (ds_bpermute), for the deterministic reduction trees of the Krylov kernels.
#pragma once
#include <hip/hip_runtime.h>

namespace dcp {

// Every lane of the wave must be active.
//   xch_swap<32 | 16>(a, b): v_permlane32_swap / v_permlane16_swap, then
//     a + b: lanes with the exchange bit clear hold a_l + a_{l^o}, the others
//     b_{l^o} + b_l (the reduce-scatter step of the pair (a, b) in one go);
//   xch_xor<o>(x), o <= 8: x of lane l ^ o (DPP row_ror:8, quad_perm for 2
//     and 1, ds_swizzle's xor mode for 4).
// IEEE addition commutes, so the sums equal the __shfl_xor forms bit for bit.
template <int O>
__device__ inline void xch_swap(double& a, double& b) {
  const unsigned long long ua = __double_as_longlong(a), ub = __double_as_longlong(b);
  unsigned l0, l1, h0, h1;
  if constexpr (O == 32) {
    const auto lo = __builtin_amdgcn_permlane32_swap(unsigned(ua), unsigned(ub), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(unsigned(ua >> 32), unsigned(ub >> 32), false, false);
    l0 = lo[0], l1 = lo[1], h0 = hi[0], h1 = hi[1];
  } else {
    static_assert(O == 16, "lane swaps exist for 32 and 16");
    const auto lo = __builtin_amdgcn_permlane16_swap(unsigned(ua), unsigned(ub), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(unsigned(ua >> 32), unsigned(ub >> 32), false, false);
    l0 = lo[0], l1 = lo[1], h0 = hi[0], h1 = hi[1];
  }
  a = __longlong_as_double((long long)((unsigned long long)h0 << 32 | l0));
  b = __longlong_as_double((long long)((unsigned long long)h1 << 32 | l1));
}
template <int O>
__device__ inline int xch_xor_b32(int x) {
  if constexpr (O == 8) return __builtin_amdgcn_update_dpp(0, x, 0x128, 0xf, 0xf, false);  // row_ror:8
  else if constexpr (O == 4) return __builtin_amdgcn_ds_swizzle(x, 0x1f | (4 << 10));       // xor 4
  else if constexpr (O == 2) return __builtin_amdgcn_update_dpp(0, x, 0x4e, 0xf, 0xf, false);  // [2,3,0,1]
  else {
    static_assert(O == 1, "DPP / swizzle exchanges for 8, 4, 2, 1");
    return __builtin_amdgcn_update_dpp(0, x, 0xb1, 0xf, 0xf, false);  // quad_perm [1,0,3,2]
  }
}
template <int O>
__device__ inline double xch_xor(double x) {
  const unsigned long long u = __double_as_longlong(x);
  const unsigned lo = unsigned(xch_xor_b32<O>(int(unsigned(u))));
  const unsigned hi = unsigned(xch_xor_b32<O>(int(unsigned(u >> 32))));
  return __longlong_as_double((long long)((unsigned long long)hi << 32 | lo));
}
// r + r_{l^o} on every lane
template <int O>
__device__ inline double xch_allsum(double r) {
  if constexpr (O >= 16) {
    double a = r, b = r;
    xch_swap<O>(a, b);
    return a + b;
  } else {
    return r + xch_xor<O>(r);
  }
}

// Reduce-scatter of the K products v[j] * x over the 64 lanes of a wave:
// log2 K halving exchanges (the first one forms the products, so only K / 2
// accumulators are live next to v) then full butterflies over the remaining
// lane bits; lane l ends with the wave sum of value l >> (6 - log2 K).
// Fixed tree, deterministic.
// The products of one thread are v[0][j] x[0] + v[1][j] x[1] (its two entries).
template <int O>
__device__ inline double butterfly_from(double r) {
  if constexpr (O >= 1) return butterfly_from<O / 2>(xch_allsum<O>(r));
  else return r;
}
// the xor butterfly r + r_{l^32}, + r_{l^16}, ..., + r_{l^1}: every lane ends
// with the wave sum, the same value and order as the __shfl_xor loop
__device__ inline double wave_allsum(double r) { return butterfly_from<32>(r); }

}  // namespace dcp
