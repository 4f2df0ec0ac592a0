// Launches of the one-launch Gram-Schmidt / s-step kernels (k_mgs_chain,
// k_cgs2_chain, k_dcgs2_step, k_sstep_block): their workgroups hand partial
// sums to each other through granules (granule.h), so every workgroup of the
// grid must be resident at once. Two guarantees instead of an assumption:
//   * resident_capacity(f, threads): the device's co-resident workgroups of
//     kernel f (hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs), queried
//     once per kernel; the callers' *_fits predicates refuse a grid larger than
//     it up front and take the multi-launch kernels instead;
//   * launch_resident(...): with DCP_COOP_LAUNCH=1, hipLaunchCooperativeKernel,
//     which the runtime only starts with the whole grid resident (or
//     rejects), even with other streams' kernels on the device. Measured at
//     refine 5 it costs ~23 us per launch (s-step inner iteration 44.9 ->
//     50.7 us, profiles/r05/r05c_*), so the default is an ordinary launch of
//     a grid the occupancy query admitted, on the context's stream (the
//     library runs nothing beside it); the bounded hand-off polls stay as the
//     last guard either way.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdexcept>
#include <string>
#include <tuple>
#include <unordered_map>
#include <utility>

namespace dcp {

inline bool coop_launch_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("DCP_COOP_LAUNCH");
    return e && *e == '1';
  }();
  return on;
}

inline int resident_capacity(const void* f, int threads) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;
  std::lock_guard<std::mutex> lock(mu);
  auto it = cache.find(f);
  if (it != cache.end()) return it->second;
  int dev = 0, cus = 0, per_cu = 0, coop = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, threads, 0) != hipSuccess)
    per_cu = cus = 0;
  if (coop_launch_enabled() &&
      (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess || !coop))
    per_cu = 0;  // no cooperative launch: nothing is guaranteed resident
  const int cap = per_cu * cus;
  cache.emplace(f, cap);
  return cap;
}

template <class... P, class... A>
void launch_resident(void (*f)(P...), int nb, int threads, hipStream_t s, A&&... a) {
  const void* fp = reinterpret_cast<const void*>(f);
  if (nb > resident_capacity(fp, threads))
    throw std::runtime_error("launch_resident: " + std::to_string(nb) +
                             " workgroups exceed the co-resident capacity " +
                             std::to_string(resident_capacity(fp, threads)));
  std::tuple<P...> args(std::forward<A>(a)...);
  void* ptrs[sizeof...(P) > 0 ? sizeof...(P) : 1];
  std::apply([&](auto&... x) {
    int i = 0;
    ((ptrs[i++] = static_cast<void*>(&x)), ...);
  }, args);
  const hipError_t e = coop_launch_enabled()
                           ? hipLaunchCooperativeKernel(fp, dim3(nb), dim3(threads), ptrs, 0, s)
                           : hipLaunchKernel(fp, dim3(nb), dim3(threads), ptrs, 0, s);
  if (e != hipSuccess)
    throw std::runtime_error(std::string("launch_resident: ") + hipGetErrorString(e));
}

}  // namespace dcp
