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
//
// Failure handling (nbg_internal.h, struct Comm): agree() for rank-local failures before a
// query's first collective; abort() + a bounded host wait for failures after it.  The
// reference's storaged fan-out keeps a query alive on a partial failure and reports the failed
// parts (StorageClient.inl:112-136, GoExecutor.cpp:424-442); a collective engine cannot run a
// hop without one of its ranks, so the query fails on every rank with the same code instead.
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>

#include "engine.h"

namespace nbg {

double comm_timeout_s() {
  const char* v = getenv("NBG_COMM_TIMEOUT_S");
  const double t = v ? atof(v) : 120.0;
  return t > 0 ? t : 120.0;
}

Comm::~Comm() {
  if (agree_dev) (void)hipFree(agree_dev);
  if (agree_host) (void)hipHostFree(agree_host);
}

bool Comm::agree_ready(std::string* err) {
  if (agree_dev) return true;
  if (hipMalloc((void**)&agree_dev, GATHER_WORDS * 8) != hipSuccess ||
      hipHostMalloc((void**)&agree_host, GATHER_WORDS * 8, hipHostMallocDefault) != hipSuccess) {
    if (err) *err = "communicator scratch allocation failed";
    return false;
  }
  return true;
}

// Host polling budget of a collective wait: spin on the stream for NBG_COMM_SPIN_US (default
// 200 us: a hop's all-to-all over xGMI completes well inside it), then yield the core between
// polls up to 2 ms, then sleep 50 us between polls.  Eight ranks share a node's host cores with
// their RCCL proxy threads; a long spin on every rank's slot streams starves those threads.
static double comm_spin_s() {
  static const double v = [] {
    const char* e = getenv("NBG_COMM_SPIN_US");
    const double us = e ? atof(e) : 200.0;
    return (us >= 0 ? us : 200.0) * 1e-6;
  }();
  return v;
}

int Comm::wait(hipStream_t s) {
  // poll: a query's latency ends here (a blocking wait would add the wake-up latency), with a
  // bound so that a peer that never arrives cannot hold this rank forever
  const auto t0 = std::chrono::steady_clock::now();
  const double limit = comm_timeout_s();
  const double spin_s = comm_spin_s();
  for (uint64_t spin = 0;; ++spin) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) return 0;
    if (e != hipErrorNotReady) {
      last = std::string("stream: ") + hipGetErrorString(e);
      abort();
      return -1;
    }
    const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (el > limit) {
      last = "collective timed out after " + std::to_string((int)limit) + " s (a peer rank failed or never arrived)";
      abort();
      return -1;
    }
    if (el > 0.002 && el > spin_s) std::this_thread::sleep_for(std::chrono::microseconds(50));
    else if (el > spin_s) std::this_thread::yield();
  }
}

int Comm::agree(hipStream_t s, int32_t local, int32_t* out) {
  *out = NBG_OK;
  if (aborted) {
    last = "communicator aborted by an earlier failure";
    *out = NBG_E_DEVICE;
    return -1;
  }
  if (!agree_dev || world > AGREE_WORDS) {
    last = "agreement scratch missing";
    *out = NBG_E_STATE;
    return -1;
  }
  memset(agree_host, 0, AGREE_WORDS * 8);
  agree_host[rank] = (unsigned long long)(int64_t)local;
  const size_t n = (size_t)world;
  int rc = hipMemcpyAsync(agree_dev, agree_host, n * 8, hipMemcpyHostToDevice, s) == hipSuccess ? 0 : -1;
  if (!rc) rc = allreduce_sum_u64(agree_dev, n, s);
  if (!rc) rc = hipMemcpyAsync(agree_host, agree_dev, n * 8, hipMemcpyDeviceToHost, s) == hipSuccess ? 0 : -1;
  if (!rc) rc = wait(s);
  if (rc) {
    if (last.empty()) last = "agreement exchange failed";
    abort();
    *out = NBG_E_DEVICE;
    return -1;
  }
  for (size_t q = 0; q < n; ++q)
    if (agree_host[q]) {
      *out = (int32_t)(int64_t)agree_host[q];
      break;
    }
  return 0;
}

int Comm::gather_u64(hipStream_t s, const uint64_t* mine, size_t k, std::vector<uint64_t>* out) {
  const size_t n = (size_t)world * k;
  if (aborted) {
    last = "communicator aborted by an earlier failure";
    return -1;
  }
  if (!agree_dev || n > GATHER_WORDS) {   // (the same on every rank: nobody enters the exchange)
    last = "gather scratch missing or too small";
    return -1;
  }
  memset(agree_host, 0, n * 8);
  for (size_t i = 0; i < k; ++i) agree_host[(size_t)rank * k + i] = mine[i];
  int rc = hipMemcpyAsync(agree_dev, agree_host, n * 8, hipMemcpyHostToDevice, s) == hipSuccess ? 0 : -1;
  if (!rc) rc = allreduce_sum_u64(agree_dev, n, s);
  if (!rc) rc = hipMemcpyAsync(agree_host, agree_dev, n * 8, hipMemcpyDeviceToHost, s) == hipSuccess ? 0 : -1;
  if (!rc) rc = wait(s);
  if (rc) {
    if (last.empty()) last = "gather exchange failed";
    abort();
    return -1;
  }
  out->assign(agree_host, agree_host + n);
  return 0;
}

// ----------------------------------------------------------------------------- RCCL
namespace {

struct RcclComm final : Comm {
  ncclComm_t comm = nullptr;
  ~RcclComm() override {
    if (comm) (void)(aborted ? ncclCommAbort(comm) : ncclCommDestroy(comm));
  }
  const char* kind() const override { return "rccl"; }
  int check(ncclResult_t r, const char* what) {
    if (aborted) {
      last = std::string(what) + ": communicator aborted";
      return -1;
    }
    if (r == ncclSuccess) return 0;
    last = std::string(what) + ": " + ncclGetErrorString(r);
    return -1;
  }
  void abort() override {
    if (aborted) return;
    aborted = true;
    // ncclCommAbort makes this rank's pending collectives return; the peers' own waits time out
    // (or see their transport fail) and abort in turn
    if (comm) (void)ncclCommAbort(comm);
    comm = nullptr;
  }
  int alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (aborted) return check(ncclSuccess, "ncclAllToAll");
    return check(ncclAllToAll(send, recv, bytes, ncclUint8, comm, s), "ncclAllToAll");
  }
  int alltoallv(const void* send, const uint64_t* scount, const uint64_t* sdisp, void* recv, const uint64_t* rcount,
                const uint64_t* rdisp, size_t elem, hipStream_t s) override {
    if (aborted) return check(ncclSuccess, "ncclSend/ncclRecv");
    const char* sp = static_cast<const char*>(send);
    char* rp = static_cast<char*>(recv);
    int rc = check(ncclGroupStart(), "ncclGroupStart");
    for (int q = 0; q < world && !rc; ++q) {
      if (scount[q]) rc = check(ncclSend(sp + sdisp[q] * elem, scount[q] * elem, ncclUint8, q, comm, s), "ncclSend");
      if (!rc && rcount[q])
        rc = check(ncclRecv(rp + rdisp[q] * elem, rcount[q] * elem, ncclUint8, q, comm, s), "ncclRecv");
    }
    const int end = check(ncclGroupEnd(), "ncclGroupEnd");
    return rc ? rc : end;
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (aborted) return check(ncclSuccess, "ncclAllGather");
    return check(ncclAllGather(send, recv, bytes, ncclUint8, comm, s), "ncclAllGather");
  }
  int allreduce_sum_u64(unsigned long long* buf, size_t n, hipStream_t s) override {
    if (aborted) return check(ncclSuccess, "ncclAllReduce");
    return check(ncclAllReduce(buf, buf, n, ncclUint64, ncclSum, comm, s), "ncclAllReduce");
  }
  Comm* split(std::string* err) override {
    if (aborted) {
      if (err) *err = "communicator aborted";
      return nullptr;
    }
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
    if (!c->agree_ready(err)) {
      delete c;
      return nullptr;
    }
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
  bool aborted = false;
  std::vector<const void*> send;
  std::vector<const uint64_t*> vcount, vdisp;   // alltoallv: each rank's send counts / displacements
  std::vector<std::vector<unsigned long long>> red;
  explicit LocalGroup(int w) : world(w), send(w, nullptr), vcount(w, nullptr), vdisp(w, nullptr), red(w) {}
  // false: the group was aborted (by a failing rank, or a peer that did not arrive in time)
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const uint64_t gen = generation;
    if (++arrived == world) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return true;
    }
    const auto limit = std::chrono::duration<double>(comm_timeout_s());
    if (!cv.wait_for(lk, limit, [&] { return generation != gen || aborted; })) aborted = true;
    if (aborted) {
      cv.notify_all();
      return false;
    }
    return true;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
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
  int gone(const char* what) {
    aborted = true;
    last = std::string(what) + ": in-process group aborted (a rank failed or did not arrive)";
    return -1;
  }
  void abort() override {
    aborted = true;
    g->abort();
  }
  // Every rank reaches both barriers even after a local copy failure, so the group never
  // deadlocks; an aborted group fails every collective at once.
  int exchange(const void* send, void* recv, size_t bytes, hipStream_t s, bool all_to_all) {
    int rc = hip(hipStreamSynchronize(s), "local collective (producer)");
    g->send[rank] = send;
    if (!g->barrier()) return gone("local collective");
    for (int q = 0; q < world && !rc; ++q) {
      const char* src = static_cast<const char*>(g->send[q]) + (all_to_all ? (size_t)rank * bytes : 0);
      rc = hip(hipMemcpyAsync(static_cast<char*>(recv) + (size_t)q * bytes, src, bytes, hipMemcpyDeviceToDevice, s),
               "local collective copy");
    }
    if (!rc) rc = hip(hipStreamSynchronize(s), "local collective (consumer)");
    if (!g->barrier()) return gone("local collective");
    return rc;
  }
  int alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    return exchange(send, recv, bytes, s, true);
  }
  int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    return exchange(send, recv, bytes, s, false);
  }
  int alltoallv(const void* send, const uint64_t* scount, const uint64_t* sdisp, void* recv, const uint64_t* rcount,
                const uint64_t* rdisp, size_t elem, hipStream_t s) override {
    int rc = hip(hipStreamSynchronize(s), "local alltoallv (producer)");
    g->send[rank] = send;
    g->vcount[rank] = scount;
    g->vdisp[rank] = sdisp;
    if (!g->barrier()) return gone("local alltoallv");
    for (int q = 0; q < world && !rc; ++q) {
      const uint64_t n = g->vcount[q][rank];
      if (n != rcount[q]) {
        last = "local alltoallv: count mismatch";
        rc = -1;
        break;
      }
      if (!n) continue;
      const char* src = static_cast<const char*>(g->send[q]) + g->vdisp[q][rank] * elem;
      rc = hip(hipMemcpyAsync(static_cast<char*>(recv) + rdisp[q] * elem, src, n * elem, hipMemcpyDeviceToDevice, s),
               "local alltoallv copy");
    }
    if (!rc) rc = hip(hipStreamSynchronize(s), "local alltoallv (consumer)");
    if (!g->barrier()) return gone("local alltoallv");
    return rc;
  }
  int allreduce_sum_u64(unsigned long long* buf, size_t n, hipStream_t s) override {
    auto& mine = g->red[rank];
    mine.assign(n, 0);
    int rc = hip(hipMemcpyAsync(mine.data(), buf, n * 8, hipMemcpyDeviceToHost, s), "local allreduce d2h");
    if (!rc) rc = hip(hipStreamSynchronize(s), "local allreduce d2h");
    if (!g->barrier()) return gone("local allreduce");
    std::vector<unsigned long long> sum(n, 0);
    for (int q = 0; q < world; ++q)
      for (size_t i = 0; i < n && i < g->red[q].size(); ++i) sum[i] += g->red[q][i];
    if (!g->barrier()) return gone("local allreduce");   // every rank has read every contribution
    if (!rc) rc = hip(hipMemcpyAsync(buf, sum.data(), n * 8, hipMemcpyHostToDevice, s), "local allreduce h2d");
    if (!rc) rc = hip(hipStreamSynchronize(s), "local allreduce h2d");
    return rc;
  }
};

}  // namespace

Comm* comm_rccl(const uint8_t id[NBG_UNIQUE_ID_BYTES], int world, int rank, std::string* err) {
  static_assert(NBG_UNIQUE_ID_BYTES == NCCL_UNIQUE_ID_BYTES, "unique id size");
  if (world > AGREE_WORDS) {
    if (err) *err = "at most 256 ranks";
    return nullptr;
  }
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
  if (!c->agree_ready(err)) {
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
  if (world > nbg::AGREE_WORDS) return E.fail(NBG_E_UNSUPPORTED, "at most 256 ranks");
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
    (void)hipSetDevice(engines[r]->e.cfg.device);
    std::string err;
    if (!comms[r]->agree_ready(&err)) {
      for (int32_t q = r; q < n; ++q) delete comms[q];
      return engines[r]->e.fail(NBG_E_OUT_OF_MEMORY, err);
    }
    engines[r]->e.comm.reset(comms[r]);
  }
  return NBG_OK;
}

// Not under the engine lock: another thread may be blocked inside a collective of this engine
// while holding it (the abort is what releases it).
extern "C" int32_t nbg_comm_abort(nbg_engine* h) {
  if (!h) return NBG_E_INVALID_ARGUMENT;
  nbg::Engine& E = h->e;
  if (!E.comm) return NBG_OK;
  E.comm->abort();
  for (auto& q : E.slots)
    if (q.comm) q.comm->abort();
  return NBG_OK;
}

extern "C" int32_t nbg_comm_aborted(const nbg_engine* h) {
  if (!h || !h->e.comm) return 0;
  return h->e.comm->is_aborted() ? 1 : 0;
}
