// RCCL and in-process transports of comm.h.
#include "comm.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>

#include "device.h"

namespace dcp {
namespace {

void nccl_check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess)
    throw std::runtime_error(std::string("RCCL ") + what + ": " + ncclGetErrorString(r));
}

struct RcclComm : Comm {
  ncclComm_t comm = nullptr;
  ~RcclComm() override {
    if (comm) (void)ncclCommDestroy(comm);
  }
  void exchange(int npeers, const int* peers, double* const* sbuf, const size_t* sn,
                double* const* rbuf, const size_t* rn, hipStream_t s) override {
    if (npeers == 0) return;
    nccl_check(ncclGroupStart(), "ncclGroupStart");
    for (int i = 0; i < npeers; ++i) {
      if (sn[i]) nccl_check(ncclSend(sbuf[i], sn[i], ncclDouble, peers[i], comm, s), "ncclSend");
      if (rn[i]) nccl_check(ncclRecv(rbuf[i], rn[i], ncclDouble, peers[i], comm, s), "ncclRecv");
    }
    nccl_check(ncclGroupEnd(), "ncclGroupEnd");
  }
  void allreduce(double* buf, size_t n, bool max, hipStream_t s) override {
    if (n == 0) return;
    nccl_check(ncclAllReduce(buf, buf, n, ncclDouble, max ? ncclMax : ncclSum, comm, s),
               "ncclAllReduce");
  }
  void describe(int out[4]) const override {
    int count = -1, user = -1, dev = -1;
    nccl_check(ncclCommCount(comm, &count), "ncclCommCount");
    nccl_check(ncclCommUserRank(comm, &user), "ncclCommUserRank");
    nccl_check(ncclCommCuDevice(comm, &dev), "ncclCommCuDevice");
    out[0] = 1;
    out[1] = count;
    out[2] = user;
    out[3] = dev;
  }
};

struct LocalComm : Comm {
  LocalGroup* g;
  void describe(int out[4]) const override {
    int dev = -1;
    (void)hipGetDevice(&dev);
    out[0] = 2;
    out[1] = g->size;
    out[2] = rank;
    out[3] = dev;
  }
  void exchange(int npeers, const int* peers, double* const* sbuf, const size_t* sn,
                double* const* rbuf, const size_t* rn, hipStream_t s) override {
    LocalGroup::Post& me = g->post[rank];
    me.dest.assign(peers, peers + npeers);
    me.ptr.assign(sbuf, sbuf + npeers);
    me.n.assign(sn, sn + npeers);
    DCP_HIP_CHECK(hipEventRecord(g->ready[rank], s));
    g->barrier();
    for (int i = 0; i < npeers; ++i) {
      const LocalGroup::Post& o = g->post[peers[i]];
      size_t k = 0;
      while (k < o.dest.size() && o.dest[k] != rank) ++k;
      if (k == o.dest.size() || o.n[k] != rn[i])
        throw std::runtime_error("LocalComm: halo plans of ranks " + std::to_string(rank) +
                                 " and " + std::to_string(peers[i]) + " disagree");
      DCP_HIP_CHECK(hipStreamWaitEvent(s, g->ready[peers[i]], 0));
      if (rn[i])
        DCP_HIP_CHECK(hipMemcpyAsync(rbuf[i], o.ptr[k], rn[i] * sizeof(double),
                                     hipMemcpyDeviceToDevice, s));
    }
    DCP_HIP_CHECK(hipEventRecord(g->done[rank], s));
    g->barrier();
    // a peer reuses its send buffer only after our copies out of it ran
    for (int i = 0; i < npeers; ++i) DCP_HIP_CHECK(hipStreamWaitEvent(s, g->done[peers[i]], 0));
  }
  void allreduce(double* buf, size_t n, bool max, hipStream_t s) override {
    LocalGroup::Post& me = g->post[rank];
    me.buf = buf;
    me.len = n;
    if (g->tmp_len[rank] < n) {
      if (g->tmp[rank]) DCP_HIP_CHECK(hipFree(g->tmp[rank]));
      DCP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&g->tmp[rank]), n * sizeof(double)));
      g->tmp_len[rank] = n;
    }
    DCP_HIP_CHECK(hipEventRecord(g->ready[rank], s));
    g->barrier();
    BufTable t{};
    for (int r = 0; r < size; ++r) {
      if (g->post[r].len != n) throw std::runtime_error("LocalComm: allreduce length mismatch");
      DCP_HIP_CHECK(hipStreamWaitEvent(s, g->ready[r], 0));
      t.p[r] = g->post[r].buf;
    }
    group_reduce(n, size, t, g->tmp[rank], max, s);
    DCP_HIP_CHECK(hipEventRecord(g->done[rank], s));
    g->barrier();
    for (int r = 0; r < size; ++r) DCP_HIP_CHECK(hipStreamWaitEvent(s, g->done[r], 0));
    DCP_HIP_CHECK(hipMemcpyAsync(buf, g->tmp[rank], n * sizeof(double), hipMemcpyDeviceToDevice, s));
    // nobody may overwrite its buffer before every rank has read it: the
    // copies above are ordered after all ranks' reductions (done events)
  }
};

// Device-initiated all-reduce over the group's mailboxes (comm.h). Each call
// takes the next tag; tags alternate between two slot sets (parity), and a
// rank cannot start call k + 2 before every rank has finished call k (call
// k + 1 waits for all ranks' tags of k + 1, posted after their k), so a slot
// set is never overwritten while a rank still reads it.
struct PeerComm : Comm {
  std::unique_ptr<Comm> base;
  LocalGroup* g = nullptr;
  PeerBoxes boxes{};
  double* box = nullptr;
  unsigned long long* flag = nullptr;
  unsigned* err = nullptr;  // host-mapped timeout flag
  unsigned long long seq = 0;
  ~PeerComm() override {
    if (box) (void)hipFree(box);
    if (flag) (void)hipFree(flag);
    if (err) (void)hipHostFree(err);
  }
  void exchange(int npeers, const int* peers, double* const* sbuf, const size_t* sn,
                double* const* rbuf, const size_t* rn, hipStream_t s) override {
    base->exchange(npeers, peers, sbuf, sn, rbuf, rn, s);
  }
  // diagnostics (DCP_PEER_MAXN: the longest all-reduce taken by the peer
  // kernel; DCP_PEER_SYNC=1: a stream synchronisation after each)
  size_t max_n = kPeerArCap;
  bool sync_each = false;
  void allreduce(double* buf, size_t n, bool max, hipStream_t s) override {
    if (n == 0) return;
    if (n > max_n) {
      base->allreduce(buf, n, max, s);
      return;
    }
    peer_allreduce(boxes, rank, size, n, buf, ++seq, max, err, 3000000000L, s);  // 30 s
    if (sync_each) DCP_HIP_CHECK(hipStreamSynchronize(s));
  }
  void describe(int out[4]) const override {
    base->describe(out);
    out[0] = 3;
  }
  void check() override {
    if (err && *reinterpret_cast<volatile unsigned*>(err))
      throw std::runtime_error("PeerComm: an all-reduce timed out waiting for a rank's tag");
  }
};

}  // namespace

std::unique_ptr<Comm> make_peer_comm(std::unique_ptr<Comm> base, LocalGroup* g, int rank) {
  // Every rank's polling kernel must run beside the others: in one process
  // their streams need hardware queues of their own (HIP shares
  // GPU_MAX_HW_QUEUES, default 4, among all streams of the process; two ranks'
  // streams on one queue would run their all-reduces in order and deadlock).
  // Each context holds two streams.
  const char* q = std::getenv("GPU_MAX_HW_QUEUES");
  const int queues = q ? std::atoi(q) : 4;
  if (queues < 2 * g->size + 1)
    throw std::runtime_error("PeerComm: " + std::to_string(g->size) +
                             " in-process ranks need GPU_MAX_HW_QUEUES >= " +
                             std::to_string(2 * g->size + 1) + " (is " + std::to_string(queues) +
                             "): ranks sharing a hardware queue would deadlock");
  auto c = std::make_unique<PeerComm>();
  c->rank = rank;
  c->size = g->size;
  c->g = g;
  c->base = std::move(base);
  if (const char* e = std::getenv("DCP_PEER_MAXN"))
    c->max_n = std::min<size_t>(size_t(std::atol(e)), size_t(kPeerArCap));
  if (const char* e = std::getenv("DCP_PEER_SYNC")) c->sync_each = *e == '1';
  DCP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&c->box),
                          sizeof(double) * 2 * size_t(g->size) * kPeerArCap));
  DCP_HIP_CHECK(hipMalloc(reinterpret_cast<void**>(&c->flag),
                          sizeof(unsigned long long) * 2 * size_t(g->size)));
  DCP_HIP_CHECK(hipMemset(c->flag, 0, sizeof(unsigned long long) * 2 * size_t(g->size)));
  DCP_HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&c->err), sizeof(unsigned),
                              hipHostMallocMapped | hipHostMallocCoherent));
  *c->err = 0;
  DCP_HIP_CHECK(hipDeviceSynchronize());
  g->post[rank].peer_box = c->box;
  g->post[rank].peer_flag = c->flag;
  g->barrier();  // every rank's mailbox posted
  for (int r = 0; r < g->size; ++r) {
    c->boxes.box[r] = g->post[r].peer_box;
    c->boxes.flag[r] = g->post[r].peer_flag;
  }
  g->barrier();  // the posts may be reused
  return c;
}

std::unique_ptr<Comm> make_rccl_comm(const void* nccl_id, int rank, int size) {
  auto c = std::make_unique<RcclComm>();
  c->rank = rank;
  c->size = size;
  ncclUniqueId id;
  std::memcpy(&id, nccl_id, sizeof(id));
  nccl_check(ncclCommInitRank(&c->comm, size, id, rank), "ncclCommInitRank");
  return c;
}

void rccl_unique_id(void* out128) {
  ncclUniqueId id;
  nccl_check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  std::memcpy(out128, &id, sizeof(id));
}

LocalGroup::LocalGroup(int n) : size(n), post(n), ready(n), done(n), tmp(n, nullptr), tmp_len(n, 0) {
  if (n < 1 || n > kMaxLocalRanks) throw std::runtime_error("LocalGroup: 1..16 ranks");
  for (int r = 0; r < n; ++r) {
    DCP_HIP_CHECK(hipEventCreateWithFlags(&ready[r], hipEventDisableTiming));
    DCP_HIP_CHECK(hipEventCreateWithFlags(&done[r], hipEventDisableTiming));
  }
}

LocalGroup::~LocalGroup() {
  for (int r = 0; r < size; ++r) {
    (void)hipEventDestroy(ready[r]);
    (void)hipEventDestroy(done[r]);
    if (tmp[r]) (void)hipFree(tmp[r]);
  }
}

void LocalGroup::barrier() {
  std::unique_lock<std::mutex> lk(m);
  const long gen = generation;
  if (++arrived == size) {
    arrived = 0;
    ++generation;
    cv.notify_all();
  } else if (!cv.wait_for(lk, std::chrono::seconds(120), [&] { return generation != gen; })) {
    throw std::runtime_error("LocalGroup: a rank did not reach the collective within 120 s");
  }
}

std::unique_ptr<Comm> make_local_comm(LocalGroup* g, int rank) {
  auto c = std::make_unique<LocalComm>();
  c->g = g;
  c->rank = rank;
  c->size = g->size;
  return c;
}

}  // namespace dcp
