// Collective transports of the partitioned engine.
//
// The reference fans a GetNeighbors request out to every storaged host that leads one of the
// frontier's parts (StorageClient::getNeighbors, src/storage/client/StorageClient.cpp:94-124)
// and graphd merges the responses into one dst set (GoExecutor::getDstIdsFromResp,
// src/graph/GoExecutor.cpp:501-541).  Here the hosts are GPUs (part p is served by rank
// p % G, CreateSpaceProcessor.cpp:84-95) and that merge is one collective per hop:
//
//   RcclComm   one process per GPU; RCCL over xGMI.  Every collective is enqueued on the
//              engine's stream, so a GO query still needs no host synchronisation until its end.
//   LocalComm  several engines in ONE process (one host thread per engine), copies between the
//              engines' buffers with hipMemcpyAsync.  Used to exercise the partitioned path on a
//              single-GPU box (several ranks on device 0) and by hosts that drive all GPUs of
//              a node from one process.  Each collective synchronises the calling stream.
#include <rccl/rccl.h>

#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>

#include "engine.h"

namespace nbg {

// ----------------------------------------------------------------------------- RCCL
namespace {

struct RcclComm final : Comm {
  ncclComm_t comm = nullptr;
  ~RcclComm() override {
    if (comm) (void)ncclCommDestroy(comm);
  }
  const char* kind() const override { return "rccl"; }
  int check(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return 0;
    last = std::string(what) + ": " + ncclGetErrorString(r);
    return -1;
  }
  int alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    return check(ncclAllToAll(send, recv, bytes, ncclUint8, comm, s), "ncclAllToAll");
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    return check(ncclAllGather(send, recv, bytes, ncclUint8, comm, s), "ncclAllGather");
  }
  int allreduce_sum_u64(unsigned long long* buf, size_t n, hipStream_t s) override {
    return check(ncclAllReduce(buf, buf, n, ncclUint64, ncclSum, comm, s), "ncclAllReduce");
  }
  Comm* split(std::string* err) override {
    ncclComm_t nc = nullptr;
    const ncclResult_t r = ncclCommSplit(comm, 0, rank, &nc, nullptr);
    if (r != ncclSuccess || !nc) {
      if (err) *err = std::string("ncclCommSplit: ") + ncclGetErrorString(r);
      return nullptr;
    }
    auto* c = new RcclComm();
    c->comm = nc;
    c->world = world;
    c->rank = rank;
    return c;
  }
};

// ----------------------------------------------------------------------------- in-process group
struct LocalGroup {
  int world;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  std::vector<const void*> send;
  std::vector<std::vector<unsigned long long>> red;
  explicit LocalGroup(int w) : world(w), send(w, nullptr), red(w) {}
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
};

struct LocalComm final : Comm {
  std::shared_ptr<LocalGroup> g;
  const char* kind() const override { return "local"; }
  int hip(hipError_t e, const char* what) {
    if (e == hipSuccess) return 0;
    last = std::string(what) + ": " + hipGetErrorString(e);
    return -1;
  }
  // Every rank reaches both barriers even after a local failure, so the group never deadlocks.
  int exchange(const void* send, void* recv, size_t bytes, hipStream_t s, bool all_to_all) {
    int rc = hip(hipStreamSynchronize(s), "local collective (producer)");
    g->send[rank] = send;
    g->barrier();
    for (int q = 0; q < world && !rc; ++q) {
      const char* src = static_cast<const char*>(g->send[q]) + (all_to_all ? (size_t)rank * bytes : 0);
      rc = hip(hipMemcpyAsync(static_cast<char*>(recv) + (size_t)q * bytes, src, bytes, hipMemcpyDeviceToDevice, s),
               "local collective copy");
    }
    if (!rc) rc = hip(hipStreamSynchronize(s), "local collective (consumer)");
    g->barrier();
    return rc;
  }
  int alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    return exchange(send, recv, bytes, s, true);
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    return exchange(send, recv, bytes, s, false);
  }
  int allreduce_sum_u64(unsigned long long* buf, size_t n, hipStream_t s) override {
    auto& mine = g->red[rank];
    mine.assign(n, 0);
    int rc = hip(hipMemcpyAsync(mine.data(), buf, n * 8, hipMemcpyDeviceToHost, s), "local allreduce d2h");
    if (!rc) rc = hip(hipStreamSynchronize(s), "local allreduce d2h");
    g->barrier();
    std::vector<unsigned long long> sum(n, 0);
    for (int q = 0; q < world; ++q)
      for (size_t i = 0; i < n && i < g->red[q].size(); ++i) sum[i] += g->red[q][i];
    g->barrier();   // every rank has read every contribution
    if (!rc) rc = hip(hipMemcpyAsync(buf, sum.data(), n * 8, hipMemcpyHostToDevice, s), "local allreduce h2d");
    if (!rc) rc = hip(hipStreamSynchronize(s), "local allreduce h2d");
    return rc;
  }
};

}  // namespace

Comm* comm_rccl(const uint8_t id[NBG_UNIQUE_ID_BYTES], int world, int rank, std::string* err) {
  static_assert(NBG_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId uid;
  memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  auto* c = new RcclComm();
  c->world = world;
  c->rank = rank;
  ncclResult_t r = ncclCommInitRank(&c->comm, world, uid, rank);
  if (r != ncclSuccess) {
    if (err) *err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    c->comm = nullptr;
    delete c;
    return nullptr;
  }
  return c;
}

std::vector<Comm*> comm_local_group(int world) {
  auto g = std::make_shared<LocalGroup>(world);
  std::vector<Comm*> out;
  for (int r = 0; r < world; ++r) {
    auto* c = new LocalComm();
    c->world = world;
    c->rank = r;
    c->g = g;
    out.push_back(c);
  }
  return out;
}

}  // namespace nbg

// ============================================================================= C ABI
extern "C" int32_t nbg_comm_unique_id(uint8_t out[NBG_UNIQUE_ID_BYTES]) {
  if (!out) return NBG_E_INVALID_ARGUMENT;
  ncclUniqueId uid;
  if (ncclGetUniqueId(&uid) != ncclSuccess) return NBG_E_DEVICE;
  memcpy(out, uid.internal, NBG_UNIQUE_ID_BYTES);
  return NBG_OK;
}

static int32_t check_comm_target(nbg_engine* h, int32_t world, int32_t rank) {
  nbg::Engine& E = h->e;
  if (E.finalized) return E.fail(NBG_E_STATE, "nbg_comm_init must precede nbg_finalize");
  if (E.comm) return E.fail(NBG_E_STATE, "communicator already initialised");
  if (world != E.cfg.num_gpus || rank != E.cfg.rank)
    return E.fail(NBG_E_INVALID_ARGUMENT, "world/rank must equal nbg_config.num_gpus/rank");
  return NBG_OK;
}

extern "C" int32_t nbg_comm_init(nbg_engine* h, const uint8_t id[NBG_UNIQUE_ID_BYTES], int32_t world, int32_t rank) {
  if (!h || !id || world < 1 || rank < 0 || rank >= world) return NBG_E_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> lg(h->e.mu);
  if (int32_t rc = check_comm_target(h, world, rank)) return rc;
  if (hipSetDevice(h->e.cfg.device) != hipSuccess) return h->e.fail(NBG_E_DEVICE, "hipSetDevice failed");
  std::string err;
  nbg::Comm* c = nbg::comm_rccl(id, world, rank, &err);
  if (!c) return h->e.fail(NBG_E_DEVICE, err);
  h->e.comm.reset(c);
  return NBG_OK;
}

extern "C" int32_t nbg_comm_init_local(nbg_engine* const* engines, int32_t n) {
  if (!engines || n < 1) return NBG_E_INVALID_ARGUMENT;
  for (int32_t r = 0; r < n; ++r) {
    if (!engines[r]) return NBG_E_INVALID_ARGUMENT;
    std::lock_guard<std::mutex> lg(engines[r]->e.mu);
    if (int32_t rc = check_comm_target(engines[r], n, r)) return rc;
  }
  auto comms = nbg::comm_local_group(n);
  for (int32_t r = 0; r < n; ++r) {
    std::lock_guard<std::mutex> lg(engines[r]->e.mu);
    engines[r]->e.comm.reset(comms[r]);
  }
  return NBG_OK;
}
