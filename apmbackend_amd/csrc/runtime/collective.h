// Collective backend of the engine's node-wide exchanges (lock-step clocks, fleet moments,
// node-wide alert candidates).  Production: one RCCL communicator per rank over xGMI
// (RcclCollective).  Tests: LocalCollective -- N engines of ONE process (one GPU) joined through
// a host rendezvous, so a 2/4-rank node can be checked against a 1-rank run without 2/4 GPUs.
//
// Every call is issued by the engine's ingest thread in a fixed per-batch sequence (see
// Engine::fleet_exchange_upto), which makes the call order identical on every rank.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <memory>
#include <string>
#include <vector>

namespace apm {

class Collective {
 public:
  virtual ~Collective() = default;
  virtual int nranks() const = 0;
  virtual int rank() const = 0;
  // stream-ordered on `s`, device buffers; `max` selects MAX, else SUM
  virtual void all_reduce_f64(double* buf, size_t n, bool max, hipStream_t s) = 0;
  // recv[r * bytes, (r + 1) * bytes) = rank r's send
  virtual void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // asynchronous failure (peer gone, network fault): returns a message, "" when healthy
  virtual std::string async_error() = 0;
  // unblock / release a wedged communicator; later calls throw
  virtual void abort() = 0;
  virtual bool aborted() const = 0;
};

std::vector<uint8_t> rccl_unique_id();
std::unique_ptr<Collective> make_rccl_collective(const std::vector<uint8_t>& uid, int nranks, int rank);

// In-process group of `n` ranks (test backend).  Each rank's engine runs on its own host thread;
// a call blocks until all n ranks made it (timeout -> throws).
// A generation-counted rendezvous: every rank deposits its contribution, the last arrival
// advances the generation, everybody reads all contributions, and a second rendezvous keeps the
// slots alive until every rank has read them.
struct LocalGroup {
  int n;
  double timeout_ms;
  std::mutex mu;
  std::condition_variable cv;
  uint64_t gen = 0;
  int arrived = 0;
  bool broken = false;
  std::vector<std::vector<uint8_t>> slot;
  LocalGroup(int n_, double t) : n(n_), timeout_ms(t), slot((size_t)n_) {}
  void rendezvous(std::unique_lock<std::mutex>& lk);  // blocks until all n ranks called it
};
std::shared_ptr<LocalGroup> make_local_group(int n, double timeout_ms = 120000.0);
std::unique_ptr<Collective> make_local_collective(std::shared_ptr<LocalGroup> g, int rank);

}  // namespace apm
