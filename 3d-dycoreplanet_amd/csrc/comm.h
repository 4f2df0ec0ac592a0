// Inter-GPU communication of the multi-GPU path: the forward ghost-DoF halo
// (Trilinos Import behind every ghosted-vector copy / operator apply in the
// reference, boussinesq_model.tpp:1145-1146, 1241, 1433-1444) and the
// Allreduce of Krylov partial sums. Everything is
// stream-ordered on the context stream; no host synchronisation.
//
// Transports:
//   RcclComm  one process per GPU, RCCL over xGMI (the production path):
//             grouped ncclSend/ncclRecv per neighbour, ncclAllReduce;
//   LocalComm P contexts of ONE process, each driven by its own host thread
//             (tests on a single GPU: the partition, halo and reduction logic
//             of the P-rank path without P devices). Collectives rendezvous on
//             a host barrier and move data with device copies / one reduction
//             kernel; results are identical on every rank;
//   PeerComm  device-initiated all-reduce over peer-mapped mailboxes
//             (DCP_PEER_COMM=1 on an in-process group): one kernel per
//             all-reduce stores this rank's partial into every rank's mailbox
//             slot, then a tagged flag, polls its own mailbox for every
//             rank's flag and sums the slots in rank order -- no host
//             rendezvous, bitwise LocalComm's sums. Halos and all-reduces
//             longer than the mailbox go to the wrapped transport.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstddef>
#include <memory>
#include <mutex>
#include <vector>

namespace dcp {

struct Comm {
  int rank = 0, size = 1;
  virtual ~Comm() = default;
  // For every i: send sn[i] doubles from sbuf[i] to peers[i], receive rn[i]
  // doubles from peers[i] into rbuf[i] (device buffers). Collective over the
  // ranks that appear in each other's peer lists.
  virtual void exchange(int npeers, const int* peers, double* const* sbuf, const size_t* sn,
                        double* const* rbuf, const size_t* rn, hipStream_t s) = 0;
  // In-place element-wise sum (or max) over all ranks; identical result on
  // every rank. Collective over all ranks.
  virtual void allreduce(double* buf, size_t n, bool max, hipStream_t s) = 0;
  // What the transport itself reports: kind (1 RCCL, 2 in-process group), its
  // rank count, this rank, and the device it drives (RCCL: ncclCommCount /
  // ncclCommUserRank / ncclCommCuDevice).
  virtual void describe(int out[4]) const = 0;
  // Raise if a device-side collective timed out (PeerComm; call after a
  // stream synchronisation).
  virtual void check() {}
};

// ncclUniqueId (128 bytes) from rank 0, passed in dcp_config.nccl_id.
std::unique_ptr<Comm> make_rccl_comm(const void* nccl_id, int rank, int size);
void rccl_unique_id(void* out128);

struct LocalGroup {
  explicit LocalGroup(int n);
  ~LocalGroup();
  int size;
  std::mutex m;
  std::condition_variable cv;
  int arrived = 0;
  long generation = 0;
  void barrier();
  // per-rank posts of the current collective
  struct Post {
    std::vector<int> dest;
    std::vector<const double*> ptr;
    std::vector<size_t> n;
    double* buf = nullptr;
    size_t len = 0;
    double* peer_box = nullptr;  // PeerComm mailboxes, shared at creation
    unsigned long long* peer_flag = nullptr;
  };
  std::vector<Post> post;
  std::vector<hipEvent_t> ready, done;
  std::vector<double*> tmp;      // per-rank reduction scratch
  std::vector<size_t> tmp_len;
};
std::unique_ptr<Comm> make_local_comm(LocalGroup* g, int rank);
// linalg.hip: out[i] = sum (or max) over r < nbufs of bufs[r][i], r ascending.
constexpr int kMaxLocalRanks = 16;
struct BufTable {
  const double* p[kMaxLocalRanks];
};
void group_reduce(size_t n, int nbufs, const BufTable& t, double* out, bool max, hipStream_t s);

// PeerComm over an in-process group (every rank must call it: the mailbox
// pointers are shared under the group's barrier); `base` keeps the halos
std::unique_ptr<Comm> make_peer_comm(std::unique_ptr<Comm> base, LocalGroup* g, int rank);

// kernels/peer.hip: the device side of PeerComm
constexpr int kPeerArCap = 4096;  // doubles per all-reduce slot
struct PeerBoxes {
  double* box[kMaxLocalRanks];              // [2 parity][size][kPeerArCap] slots per rank
  unsigned long long* flag[kMaxLocalRanks];  // [2 parity][size] tags per rank
};
void peer_allreduce(const PeerBoxes& b, int rank, int size, size_t n, double* buf,
                    unsigned long long seq, bool max, unsigned* err, long spin_limit,
                    hipStream_t s);


}  // namespace dcp
