// Bandwidth of the Krylov-basis read pattern of the inner Schur GMRES chain
// (K vectors of n = 202,818 doubles, the r=5 pressure space) after a flush of
// the Infinity Cache, for several launch shapes. Timing probe, not product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

struct Vecs { const double* v[32]; };
static double* g_vb = nullptr;

// every thread: E entries (pairs of 16-B loads when E=2), all K vectors loaded up front
template <int K, int E>
__global__ void k_read(Vecs V, long n, double* out) {
  const long base = (long(blockIdx.x) * blockDim.x + threadIdx.x) * E;
  double s = 0;
  if (E == 2) {
    if (base + 1 < n) {
      double2 a[K];
#pragma unroll
      for (int j = 0; j < K; ++j) a[j] = *reinterpret_cast<const double2*>(V.v[j] + base);
#pragma unroll
      for (int j = 0; j < K; ++j) s += a[j].x * (j + 1) + a[j].y;
    }
  } else {
    if (base < n) {
      double a[K];
#pragma unroll
      for (int j = 0; j < K; ++j) a[j] = V.v[j][base];
#pragma unroll
      for (int j = 0; j < K; ++j) s += a[j] * (j + 1);
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// grid-stride: each thread walks the vectors one at a time (streaming), 16-B loads
template <int K>
__global__ void k_stream(Vecs V, long n, double* out) {
  double s = 0;
  for (int j = 0; j < K; ++j)
    for (long i = (long(blockIdx.x) * blockDim.x + threadIdx.x) * 2; i + 1 < n;
         i += long(gridDim.x) * blockDim.x * 2) {
      const double2 a = *reinterpret_cast<const double2*>(V.v[j] + i);
      s += a.x + a.y * j;
    }
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// blocked basis layout [n / B][K][B] (B = 1024 entries = 8 KB): workgroup b
// reads block b of all K vectors, one contiguous K * 8 KB region
template <int K>
__global__ void k_read_blocked(const double* Vb, long n, int kstride, double* out) {
  const long blk = blockIdx.x;
  const double* base = Vb + blk * long(kstride) * 1024 + 2 * threadIdx.x;
  double2 a[K];
#pragma unroll
  for (int j = 0; j < K; ++j) a[j] = *reinterpret_cast<const double2*>(base + long(j) * 1024);
  double s = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) s += a[j].x * (j + 1) + a[j].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// read-only flush (the inner GMRES's SpMV only reads between two chain launches)
__global__ void k_flush(double* f, long n) {
  double s = 0;
  for (long i = long(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x)
    s += f[i];
  if (s == 12345.678) f[0] = s;
}

template <class F>
float timeit(F launch, double* flush, long nf, hipEvent_t a, hipEvent_t b) {
  float best = 1e30f, tot = 0;
  for (int r = 0; r < 20; ++r) {
    hipLaunchKernelGGL(k_flush, dim3(4096), dim3(256), 0, 0, flush, nf);
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (r >= 2) tot += ms;
    if (ms < best) best = ms;
  }
  return tot / 18 * 1000.f;
}

template <int K>
int run(Vecs V, long n, double* out, double* flush, long nf, hipEvent_t a, hipEvent_t b) {
  const double mb = K * n * 8.0 / 1e6;
  const long thr2 = (n + 1) / 2;
  float t;
  t = timeit([&] { hipLaunchKernelGGL((k_read<K, 2>), dim3((thr2 + 511) / 512), dim3(512), 0, 0, V, n, out); }, flush, nf, a, b);
  printf("K=%2d chain-like 512thr x2 (%ld WGs): %7.2f us  %6.2f TB/s\n", K, (thr2 + 511) / 512, t, mb / t);
  t = timeit([&] { hipLaunchKernelGGL((k_read<K, 2>), dim3((thr2 + 255) / 256), dim3(256), 0, 0, V, n, out); }, flush, nf, a, b);
  printf("K=%2d 256thr x2 (%ld WGs):            %7.2f us  %6.2f TB/s\n", K, (thr2 + 255) / 256, t, mb / t);
  t = timeit([&] { hipLaunchKernelGGL((k_read<K, 1>), dim3((n + 1023) / 1024), dim3(1024), 0, 0, V, n, out); }, flush, nf, a, b);
  printf("K=%2d 1024thr x1 (%ld WGs):           %7.2f us  %6.2f TB/s\n", K, (n + 1023) / 1024, t, mb / t);
  t = timeit([&] { hipLaunchKernelGGL((k_read<K, 1>), dim3((n + 255) / 256), dim3(256), 0, 0, V, n, out); }, flush, nf, a, b);
  printf("K=%2d 256thr x1 (%ld WGs):            %7.2f us  %6.2f TB/s\n", K, (n + 255) / 256, t, mb / t);
  {
    const long nblk = (n + 1023) / 1024;
    t = timeit([&] { hipLaunchKernelGGL((k_read_blocked<K>), dim3(nblk), dim3(512), 0, 0, g_vb, n, 32, out); }, flush, nf, a, b);
    printf("K=%2d blocked [n/1024][32][1024] (%ld WGs): %7.2f us  %6.2f TB/s\n", K, nblk, t, mb / t);
  }
  for (int g : {256, 1024, 2048}) {
    t = timeit([&] { hipLaunchKernelGGL((k_stream<K>), dim3(g), dim3(256), 0, 0, V, n, out); }, flush, nf, a, b);
    printf("K=%2d grid-stride %4d x 256:          %7.2f us  %6.2f TB/s\n", K, g, t, mb / t);
  }
  return 0;
}

int main() {
  const long n = 202818;
  std::vector<double*> vs(32);
  for (auto& p : vs) { CK(hipMalloc(&p, n * 8)); CK(hipMemset(p, 0, n * 8)); }
  Vecs V;
  for (int j = 0; j < 32; ++j) V.v[j] = vs[j];
  CK(hipMalloc(&g_vb, ((n + 1023) / 1024) * 32L * 1024 * 8));
  CK(hipMemset(g_vb, 0, ((n + 1023) / 1024) * 32L * 1024 * 8));
  double *out, *flush;
  const long nf = 512L << 20 >> 3;  // 512 MB
  CK(hipMalloc(&out, 8 << 20));
  CK(hipMalloc(&flush, nf * 8));
  CK(hipMemset(flush, 0, nf * 8));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  run<4>(V, n, out, flush, nf, a, b);
  run<16>(V, n, out, flush, nf, a, b);
  run<28>(V, n, out, flush, nf, a, b);
  CK(hipDeviceSynchronize());
  printf("done\n");
  return 0;
}
