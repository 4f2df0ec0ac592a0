// Kernel-boundary probe: what a kernel that writes mapped host memory, and an
// event recorded between two kernels, cost at the next kernel's start.
// Build: hipcc --offload-arch=gfx950 -O2 tools/gap_probe.hip -o tools/gap_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__);    \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

// ~T µs of work per block (wall clock at 100 MHz)
__global__ void k_busy(double* out, int us) {
  const long t0 = wall_clock64();
  while (wall_clock64() - t0 < long(us) * 100) __builtin_amdgcn_s_sleep(4);
  if (threadIdx.x == 0) out[blockIdx.x] = double(t0);
}

__global__ void k_write(double* dev, double* host, int nhost) {
  if (threadIdx.x == 0) {
    dev[blockIdx.x] = 1.0;
    if (host && int(blockIdx.x) < nhost) host[blockIdx.x] = 2.0;
  }
}

int main() {
  double *dev, *host;
  CK(hipMalloc(&dev, 1 << 20));
  CK(hipHostMalloc(&host, 1 << 20, hipHostMallocMapped | hipHostMallocCoherent));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t a, b, mid[2];
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto& e : mid) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  const int N = 2000, busy = 30;
  struct Case {
    const char* name;
    int nhost;
    bool event;
    bool host_sync;
  } cases[] = {{"device writes only", 0, false, false},
               {"+ 1 mapped-host write (block 0)", 1, false, false},
               {"+ 256 mapped-host writes", 256, false, false},
               {"device writes + event", 0, true, false},
               {"256 mapped writes + event", 256, true, false},
               {"256 mapped writes + event + host sync one behind", 256, true, true},
               {"device writes + event + host sync one behind", 0, true, true}};
  for (int rep = 0; rep < 2; ++rep)
    for (const Case& c : cases) {
      CK(hipStreamSynchronize(s));
      CK(hipEventRecord(a, s));
      for (int i = 0; i < N; ++i) {
        hipLaunchKernelGGL(k_busy, dim3(3169), dim3(256), 0, s, dev + 4096, busy);
        hipLaunchKernelGGL(k_write, dim3(256), dim3(256), 0, s, dev, c.nhost ? host : nullptr,
                           c.nhost);
        if (c.event) CK(hipEventRecord(mid[i & 1], s));
        if (c.host_sync && i > 0) CK(hipEventSynchronize(mid[(i - 1) & 1]));
      }
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (rep) std::printf("%-50s %.2f us per pair\n", c.name, 1e3 * ms / N);
    }
  return 0;
}
