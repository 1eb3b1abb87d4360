// Collective backend of the engine's node-wide exchanges (lock-step clocks, fleet moments,
// node-wide alert candidates).  Production: one RCCL communicator per rank over xGMI
// (RcclCollective).  Host transport: HostCollective -- one process per rank joined by TCP
// through rank 0 (ranks sharing one GPU, or nodes without a working RCCL path); it is how the
// multi-PROCESS node is exercised on a one-GPU box.  Tests: LocalCollective -- N engines of ONE
// process (one GPU) joined through a host rendezvous.
//
// Every call is issued by the engine's ingest thread in a fixed per-batch sequence (see
// Engine::fleet_exchange_upto), which makes the call order identical on every rank.
#pragma once
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdint>
#include <mutex>
#include <memory>
#include <stdexcept>
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
  // host-buffer variants (HostCollective: CPU tests of the transport without a GPU)
  virtual std::vector<double> all_reduce_host(const std::vector<double>&, bool) {
    throw std::runtime_error("host-buffer collectives: HostCollective only");
  }
  virtual std::vector<uint8_t> all_gather_host(const std::vector<uint8_t>&) {
    throw std::runtime_error("host-buffer collectives: HostCollective only");
  }
};

std::vector<uint8_t> rccl_unique_id();
// ncclCommInitRank under a deadline: a rank whose peers never arrive (a rank that crashed before
// its init, mismatched world sizes, two ranks on one device) throws a clear error after
// `init_timeout_ms` instead of blocking forever.  The blocked init thread is abandoned; the
// caller is expected to exit the process.
std::unique_ptr<Collective> make_rccl_collective(const std::vector<uint8_t>& uid, int nranks, int rank,
                                                 double init_timeout_ms = 120000.0);

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

// TCP star through rank 0 (`addr`:`port`): rank 0 listens, the others connect (retrying until
// `timeout_ms`).  Every call is synchronous on the host: the stream is drained, the buffer copied
// to the host, exchanged, reduced by rank 0 in rank order (deterministic) and copied back.  A peer
// that closes its connection (process gone) or does not arrive within `timeout_ms` makes the call
// throw after shutting every connection down, so the remaining ranks fail the same way.
std::unique_ptr<Collective> make_host_collective(const std::string& addr, int port, int nranks, int rank,
                                                 double timeout_ms);
std::unique_ptr<Collective> make_local_collective(std::shared_ptr<LocalGroup> g, int rank);

}  // namespace apm
