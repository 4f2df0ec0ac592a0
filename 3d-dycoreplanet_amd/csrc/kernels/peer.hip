// Device side of PeerComm (comm.h): the all-reduce of Krylov partial sums
// (the reference's MPI_Allreduce behind every Trilinos dot,
// block_schur_preconditioner.hpp:46-51, boussinesq_model.tpp:1145-1146) as
// one kernel per call, no host rendezvous:
//   1. this rank's partial into slot [parity][rank] of every rank's mailbox
//      (remote stores), release at system scope, then the call's tag into
//      every rank's flag [parity][rank];
//   2. one lane per rank polls this rank's flag of that rank (acquire,
//      bounded by the wall clock: a timeout raises the host-mapped error word
//      and the result is refused by PeerComm::check);
//   3. the slots summed in rank order 0..size-1 -- the order of LocalComm's
//      group_reduce, so every rank holds bitwise the same, and LocalComm's, sum.
#include <hip/hip_runtime.h>

#include "../comm.h"
#include "../device.h"

namespace dcp {
namespace {

constexpr int kPeerThreads = 256;

__global__ __launch_bounds__(kPeerThreads) void k_peer_allreduce(PeerBoxes b, int rank, int size,
                                                                 int n, double* __restrict__ buf,
                                                                 unsigned long long seq, int mx,
                                                                 unsigned* err, long limit) {
  const int par = int(seq & 1ull);
  for (int r = 0; r < size; ++r) {
    double* dst = b.box[r] + (size_t(par) * size + rank) * kPeerArCap;
    for (int i = threadIdx.x; i < n; i += kPeerThreads) dst[i] = buf[i];
  }
  __threadfence_system();
  __syncthreads();
  if (int(threadIdx.x) < size)
    __hip_atomic_store(b.flag[threadIdx.x] + par * size + rank, seq, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  if (int(threadIdx.x) < size) {
    const unsigned long long* f = b.flag[rank] + par * size + threadIdx.x;
    const long t0 = long(wall_clock64());
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
      if (long(wall_clock64()) - t0 > limit) {
        __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const double* mine = b.box[rank] + size_t(par) * size * kPeerArCap;
  for (int i = threadIdx.x; i < n; i += kPeerThreads) {
    double v = mine[i];
    for (int r = 1; r < size; ++r) v = mx ? fmax(v, mine[size_t(r) * kPeerArCap + i]) : v + mine[size_t(r) * kPeerArCap + i];
    buf[i] = v;
  }
}

}  // namespace

void peer_allreduce(const PeerBoxes& b, int rank, int size, size_t n, double* buf,
                    unsigned long long seq, bool max, unsigned* err, long spin_limit,
                    hipStream_t s) {
  hipLaunchKernelGGL(k_peer_allreduce, dim3(1), dim3(kPeerThreads), 0, s, b, rank, size, int(n),
                     buf, seq, max ? 1 : 0, err, spin_limit);
  DCP_HIP_CHECK(hipGetLastError());
}

}  // namespace dcp
