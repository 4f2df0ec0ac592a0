// Measured bandwidth ceilings of this MI355X for the roofline fractions the
// bench reports (BASELINE.md section 4 asks for a measured STREAM-triad ceiling
// beside the 8 TB/s datasheet figure). Timing probe, not product.
//   copy / triad / read: 1 GiB arrays (HBM), best of 10 passes, 16-byte loads
//   resident read: a working set of S MB swept 10 times back to back (the first
//   sweep from HBM, later ones from the 256 MiB Infinity Cache as far as the set
//   stays resident), per-sweep rate of sweeps 2..10
// Output: one JSON object.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      std::printf("{\"error\": \"%s\"}\n", hipGetErrorString(e));      \
      return 1;                                                        \
    }                                                                  \
  } while (0)

__global__ void k_copy(const double2* __restrict__ a, double2* __restrict__ b, long n) {
  for (long i = long(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x)
    b[i] = a[i];
}
__global__ void k_triad(const double2* __restrict__ b, const double2* __restrict__ c,
                        double2* __restrict__ a, double s, long n) {
  for (long i = long(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x) {
    const double2 x = b[i], y = c[i];
    a[i] = make_double2(x.x + s * y.x, x.y + s * y.y);
  }
}
__global__ void k_read(const double2* __restrict__ a, long n, double* out) {
  double s = 0.0;
  for (long i = long(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x) {
    const double2 x = a[i];
    s += x.x + x.y;
  }
  if (s == 1234.5) out[0] = s;  // keeps the loads
}

int main() {
  const long n = (1L << 30) / 16;  // 1 GiB of double2
  double2 *a, *b, *c;
  double* out;
  CK(hipMalloc(&a, n * 16));
  CK(hipMalloc(&b, n * 16));
  CK(hipMalloc(&c, n * 16));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(a, 0, n * 16));
  CK(hipMemset(b, 0, n * 16));
  CK(hipMemset(c, 0, n * 16));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const dim3 grid(ncu * 8), block(256);
  auto best = [&](auto launch, int reps) {
    float bestms = 1e30f;
    for (int r = 0; r < reps; ++r) {
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      bestms = std::min(bestms, ms);
    }
    return double(bestms);
  };
  const double gb = 1e9;
  const double t_copy = best([&] { hipLaunchKernelGGL(k_copy, grid, block, 0, 0, a, b, n); }, 10);
  const double t_triad =
      best([&] { hipLaunchKernelGGL(k_triad, grid, block, 0, 0, b, c, a, 3.0, n); }, 10);
  const double t_read = best([&] { hipLaunchKernelGGL(k_read, grid, block, 0, 0, a, n, out); }, 10);
  std::printf("{\"copy_TBps\": %.3f, \"triad_TBps\": %.3f, \"read_TBps\": %.3f, \"resident_read\": [",
              2.0 * n * 16 / (t_copy * 1e-3) / gb / 1e3, 3.0 * n * 16 / (t_triad * 1e-3) / gb / 1e3,
              1.0 * n * 16 / (t_read * 1e-3) / gb / 1e3);
  const int sizes_mb[] = {16, 32, 64, 128, 192, 240, 320};
  bool first = true;
  for (int mb : sizes_mb) {
    const long m = long(mb) * (1L << 20) / 16;
    // evict: sweep 1 GiB of other data first
    hipLaunchKernelGGL(k_read, grid, block, 0, 0, c, n, out);
    std::vector<float> ms(10);
    for (int r = 0; r < 10; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(k_read, grid, block, 0, 0, a, m, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms[r], e0, e1);
    }
    std::vector<float> warm(ms.begin() + 1, ms.end());
    std::sort(warm.begin(), warm.end());
    const double med = warm[warm.size() / 2];
    std::printf("%s{\"MB\": %d, \"first_TBps\": %.3f, \"warm_median_TBps\": %.3f}", first ? "" : ", ",
                mb, double(m) * 16 / (ms[0] * 1e-3) / 1e12, double(m) * 16 / (med * 1e-3) / 1e12);
    first = false;
  }
  std::printf("], \"cus\": %d}\n", ncu);
  CK(hipDeviceSynchronize());
  return 0;
}
