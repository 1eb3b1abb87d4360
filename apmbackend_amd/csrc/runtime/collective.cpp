// Collective backends: RCCL (production), TCP host transport (multi-process on one GPU), and an
// in-process rendezvous (tests).
#include "collective.h"

#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <fcntl.h>
#include <immintrin.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <cstdlib>
#include <cerrno>
#include <thread>

#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <stdexcept>

#include "../kernels/common.h"

namespace apm {

// ------------------------------------------------------------------------------------ RCCL
namespace {

class RcclCollective final : public Collective {
 public:
  RcclCollective(const std::vector<uint8_t>& uid, int nranks, int rank, double init_timeout_ms)
      : n_(nranks), r_(rank) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad RCCL unique id size");
    if (rank < 0 || rank >= nranks) throw std::runtime_error("RCCL: rank out of range");
    // The blocking init runs on a helper thread bound to this thread's device; the caller waits
    // on a deadline.  State lives in a shared block so an abandoned init can still finish (or
    // stay blocked) without touching this object.
    struct Init {
      std::mutex mu;
      std::condition_variable cv;
      bool done = false;
      ncclResult_t res = ncclInternalError;
      ncclComm_t comm = nullptr;
    };
    auto st = std::make_shared<Init>();
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    int dev = 0;
    HIP_OK(hipGetDevice(&dev));
    std::thread([st, id, nranks, rank, dev]() {
      ncclComm_t c = nullptr;
      ncclResult_t r = hipSetDevice(dev) == hipSuccess ? ncclCommInitRank(&c, nranks, id, rank) : ncclUnhandledCudaError;
      std::lock_guard<std::mutex> g(st->mu);
      st->res = r;
      st->comm = c;
      st->done = true;
      st->cv.notify_all();
    }).detach();
    std::unique_lock<std::mutex> lk(st->mu);
    const bool ok = st->cv.wait_for(lk, std::chrono::microseconds((int64_t)(init_timeout_ms * 1000)),
                                    [&]() { return st->done; });
    if (!ok)
      throw std::runtime_error("RCCL communicator init did not complete within " +
                               std::to_string((long long)(init_timeout_ms / 1000)) + " s (rank " +
                               std::to_string(rank) + " of " + std::to_string(nranks) +
                               "): a peer rank never joined (crashed before init, different world size, "
                               "or two ranks on one GPU -- use gpu.collectiveBackend=host for that)");
    if (st->res != ncclSuccess)
      throw std::runtime_error(std::string("ncclCommInitRank failed (rank ") + std::to_string(rank) + " of " +
                               std::to_string(nranks) + "): " + ncclGetErrorString(st->res));
    comm_ = st->comm;
    int cnt = 0;
    if (ncclCommCount(comm_, &cnt) != ncclSuccess || cnt != nranks)
      throw std::runtime_error("RCCL communicator has " + std::to_string(cnt) + " ranks, expected " +
                               std::to_string(nranks));
  }
  ~RcclCollective() override {
    if (comm_ && !aborted_) ncclCommDestroy(comm_);  // an aborted communicator is already freed
  }
  int nranks() const override { return n_; }
  int rank() const override { return r_; }
  void all_reduce_f64(double* buf, size_t n, bool max, hipStream_t s) override {
    check(ncclAllReduce(buf, buf, n, ncclDouble, max ? ncclMax : ncclSum, comm_, s), "all-reduce");
  }
  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    check(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s), "all-gather");
  }
  std::string async_error() override {
    if (aborted_) return "communicator aborted";
    ncclResult_t ar = ncclSuccess;
    if (ncclCommGetAsyncError(comm_, &ar) != ncclSuccess) return "";
    if (ar != ncclSuccess && ar != ncclInProgress) return ncclGetErrorString(ar);
    return "";
  }
  void abort() override {
    if (!aborted_) ncclCommAbort(comm_);
    aborted_ = true;
  }
  bool aborted() const override { return aborted_; }

 private:
  void check(ncclResult_t r, const char* what) {
    if (aborted_) throw std::runtime_error("RCCL communicator was aborted");
    if (r == ncclSuccess || r == ncclInProgress) return;
    abort();
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(r));
  }
  ncclComm_t comm_ = nullptr;
  int n_, r_;
  bool aborted_ = false;
};

}  // namespace

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) throw std::runtime_error("ncclGetUniqueId failed");
  return std::vector<uint8_t>((uint8_t*)&id, (uint8_t*)&id + sizeof(id));
}

std::unique_ptr<Collective> make_rccl_collective(const std::vector<uint8_t>& uid, int nranks, int rank,
                                                 double init_timeout_ms) {
  return std::unique_ptr<Collective>(new RcclCollective(uid, nranks, rank, init_timeout_ms));
}

// ----------------------------------------------------------------------- in-process group
void LocalGroup::rendezvous(std::unique_lock<std::mutex>& lk) {
  if (broken) throw std::runtime_error("local collective group broken (a rank failed)");
  const uint64_t g = gen;
  if (++arrived == n) {
    arrived = 0;
    ++gen;
    cv.notify_all();
    return;
  }
  const bool ok = cv.wait_for(lk, std::chrono::microseconds((int64_t)(timeout_ms * 1000)),
                              [&]() { return gen != g || broken; });
  if (broken) throw std::runtime_error("local collective group broken (a rank failed)");
  if (!ok) {
    broken = true;
    cv.notify_all();
    throw std::runtime_error("local collective: peer ranks did not arrive (timeout)");
  }
}

std::shared_ptr<LocalGroup> make_local_group(int n, double timeout_ms) {
  if (n <= 0) throw std::runtime_error("local group size must be > 0");
  return std::make_shared<LocalGroup>(n, timeout_ms);
}

namespace {

class LocalCollective final : public Collective {
 public:
  LocalCollective(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)), r_(rank) {
    if (rank < 0 || rank >= g_->n) throw std::runtime_error("local collective: rank out of range");
  }
  int nranks() const override { return g_->n; }
  int rank() const override { return r_; }

  void all_reduce_f64(double* buf, size_t n, bool max, hipStream_t s) override {
    std::vector<uint8_t> mine(n * 8);
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipMemcpy(mine.data(), buf, n * 8, hipMemcpyDeviceToHost));
    std::vector<double> out(n);
    exchange(std::move(mine), [&](const std::vector<std::vector<uint8_t>>& all) {
      const double* a0 = (const double*)all[0].data();
      for (size_t i = 0; i < n; ++i) out[i] = a0[i];
      for (size_t r = 1; r < all.size(); ++r) {
        const double* a = (const double*)all[r].data();
        for (size_t i = 0; i < n; ++i) out[i] = max ? (a[i] > out[i] ? a[i] : out[i]) : out[i] + a[i];
      }
    });
    HIP_OK(hipMemcpy(buf, out.data(), n * 8, hipMemcpyHostToDevice));
  }

  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    std::vector<uint8_t> mine(bytes);
    HIP_OK(hipStreamSynchronize(s));
    HIP_OK(hipMemcpy(mine.data(), send, bytes, hipMemcpyDeviceToHost));
    std::vector<uint8_t> out(bytes * (size_t)g_->n);
    exchange(std::move(mine), [&](const std::vector<std::vector<uint8_t>>& all) {
      for (size_t r = 0; r < all.size(); ++r) std::memcpy(out.data() + r * bytes, all[r].data(), bytes);
    });
    HIP_OK(hipMemcpy(recv, out.data(), out.size(), hipMemcpyHostToDevice));
  }

  std::string async_error() override { return aborted_ ? "local collective aborted" : ""; }
  void abort() override {
    aborted_ = true;
    std::lock_guard<std::mutex> lk(g_->mu);
    g_->broken = true;
    g_->cv.notify_all();
  }
  bool aborted() const override { return aborted_; }

 private:
  template <class F>
  void exchange(std::vector<uint8_t>&& mine, F&& combine) {
    if (aborted_) throw std::runtime_error("local collective aborted");
    std::unique_lock<std::mutex> lk(g_->mu);
    g_->slot[(size_t)r_] = std::move(mine);
    g_->rendezvous(lk);
    combine(g_->slot);
    g_->rendezvous(lk);  // nobody overwrites a slot before every rank has read it
  }
  std::shared_ptr<LocalGroup> g_;
  int r_;
  bool aborted_ = false;
};

}  // namespace

std::unique_ptr<Collective> make_local_collective(std::shared_ptr<LocalGroup> g, int rank) {
  return std::unique_ptr<Collective>(new LocalCollective(std::move(g), rank));
}

}  // namespace apm

// --------------------------------------------------------------------- host transport (TCP)

namespace apm {
namespace {

double mono_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

class HostCollective final : public Collective {
 public:
  HostCollective(const std::string& addr, int port, int nranks, int rank, double timeout_ms)
      : n_(nranks), r_(rank), timeout_ms_(timeout_ms), fd_((size_t)std::max(nranks, 1), -1) {
    if (rank < 0 || rank >= nranks) throw std::runtime_error("host collective: rank out of range");
    if (nranks == 1) return;
    sockaddr_in sa{};
    sa.sin_family = AF_INET;
    sa.sin_port = htons((uint16_t)port);
    if (inet_pton(AF_INET, addr.c_str(), &sa.sin_addr) != 1) throw std::runtime_error("host collective: bad address " + addr);
    const double t_end = mono_ms() + timeout_ms_;
    if (rank == 0) {
      const int ls = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
      if (ls < 0) throw std::runtime_error("host collective: socket failed");
      const int one = 1;
      ::setsockopt(ls, SOL_SOCKET, SO_REUSEADDR, &one, sizeof one);
      if (::bind(ls, (sockaddr*)&sa, sizeof sa) != 0 || ::listen(ls, nranks) != 0) {
        const std::string e = std::strerror(errno);
        ::close(ls);
        throw std::runtime_error("host collective: cannot listen on " + addr + ":" + std::to_string(port) + ": " + e);
      }
      for (int got = 1; got < nranks;) {
        pollfd p{ls, POLLIN, 0};
        const double left = t_end - mono_ms();
        if (left <= 0 || ::poll(&p, 1, (int)left) <= 0) {
          ::close(ls);
          shutdown_all();
          throw std::runtime_error("host collective: only " + std::to_string(got) + " of " + std::to_string(nranks) +
                                   " ranks connected in time");
        }
        const int c = ::accept4(ls, nullptr, nullptr, SOCK_CLOEXEC);
        if (c < 0) continue;
        int32_t peer = -1;
        if (!recv_all(c, &peer, 4, t_end) || peer <= 0 || peer >= nranks || fd_[(size_t)peer] >= 0) {
          ::close(c);
          continue;
        }
        tune(c);
        fd_[(size_t)peer] = c;
        ++got;
      }
      ::close(ls);
    } else {
      for (;;) {
        const int c = ::socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
        if (c < 0) throw std::runtime_error("host collective: socket failed");
        if (::connect(c, (sockaddr*)&sa, sizeof sa) == 0) {
          tune(c);
          const int32_t me = rank;
          if (!send_all(c, &me, 4)) { ::close(c); throw std::runtime_error("host collective: hello failed"); }
          fd_[0] = c;
          break;
        }
        ::close(c);
        if (mono_ms() > t_end) throw std::runtime_error("host collective: rank 0 not reachable at " + addr + ":" + std::to_string(port));
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
      }
    }
    shm_handshake(port, t_end);
  }
  ~HostCollective() override {
    shutdown_all();
    if (shm_) ::munmap(shm_, shm_len_);
    for (Staged* st : pool_) {
      if (st->done) { hipEventSynchronize(st->done); hipEventDestroy(st->done); }
      if (st->in) hipHostFree(st->in);
      if (st->out) hipHostFree(st->out);
      delete st;
    }
  }
  int nranks() const override { return n_; }
  int rank() const override { return r_; }

  // APM_HOSTCOLL_ASYNC=1: stream-ordered like RCCL, the calling thread only enqueues.  On stream `s`: D2H of the
  // contribution into a pinned stage, a host function (HIP's callback thread) that runs the TCP
  // exchange, H2D of the result.  The stream -- and nothing else -- waits for the peers, so the
  // engine's split lock-step rounds overlap the join here exactly as they do over RCCL.  Every
  // collective of an engine is on its one collective stream, so the callbacks run in issue
  // order on every rank.  One rank: MAX / SUM over one rank is the identity, nothing to do.
  void all_reduce_f64(double* buf, size_t n, bool max, hipStream_t s) override {
    if (aborted_.load()) throw std::runtime_error("host collective aborted: " + error());
    if (n_ == 1 || n == 0) return;
    if (sync_mode()) {  // the caller waits (default; see sync_mode)
      std::vector<double> mine(n);
      HIP_OK(hipStreamSynchronize(s));
      HIP_OK(hipMemcpy(mine.data(), buf, n * 8, hipMemcpyDeviceToHost));
      const std::vector<double> out = all_reduce_host(mine, max);
      HIP_OK(hipMemcpy(buf, out.data(), n * 8, hipMemcpyHostToDevice));
      return;
    }
    enqueue(s, max ? 1u : 2u, buf, buf, n * 8, n * 8);
  }

  void all_gather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (aborted_.load()) throw std::runtime_error("host collective aborted: " + error());
    if (n_ == 1) {
      if (bytes && send != recv) HIP_OK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
      return;
    }
    if (sync_mode()) {
      std::vector<uint8_t> mine(bytes);
      HIP_OK(hipStreamSynchronize(s));
      HIP_OK(hipMemcpy(mine.data(), send, bytes, hipMemcpyDeviceToHost));
      const std::vector<uint8_t> out = all_gather_host(mine);
      HIP_OK(hipMemcpy(recv, out.data(), out.size(), hipMemcpyHostToDevice));
      return;
    }
    enqueue(s, 3u, send, recv, bytes, bytes * (size_t)n_);
  }
  // The stream-ordered form (host functions on HIP's callback thread) measured slower on the
  // 2-rank one-GPU rehearsal: 119 M lines/s, lock-step 1.6 ms/step, against 156 M / 0.18 ms for
  // the synchronous form (profiles/r6_d) -- the callback thread's wake-up latency lands on every
  // collective.  Synchronous is the default; APM_HOSTCOLL_ASYNC=1 selects the stream-ordered form.
  static bool sync_mode() {
    static const bool v = [] { const char* e = std::getenv("APM_HOSTCOLL_ASYNC"); return !(e && e[0] == '1'); }();
    return v;
  }

  // rank 0 reduces in rank order: the same bits on every rank, every run
  std::vector<double> all_reduce_host(const std::vector<double>& v, bool max) override {
    const size_t n = v.size();
    std::vector<uint8_t> mine(n * 8);
    std::memcpy(mine.data(), v.data(), n * 8);
    const std::vector<uint8_t> out = exchange(max ? 1u : 2u, std::move(mine), [&](std::vector<std::vector<uint8_t>>& all) {
      std::vector<uint8_t> r(all[0]);
      double* o = (double*)r.data();
      for (size_t k = 1; k < all.size(); ++k) {
        const double* a = (const double*)all[k].data();
        for (size_t i = 0; i < n; ++i) o[i] = max ? (a[i] > o[i] ? a[i] : o[i]) : o[i] + a[i];
      }
      return r;
    });
    std::vector<double> res(n);
    std::memcpy(res.data(), out.data(), n * 8);
    return res;
  }

  std::vector<uint8_t> all_gather_host(const std::vector<uint8_t>& v) override {
    const size_t bytes = v.size();
    return exchange(3u, std::vector<uint8_t>(v), [&](std::vector<std::vector<uint8_t>>& all) {
      std::vector<uint8_t> r(bytes * all.size());
      for (size_t k = 0; k < all.size(); ++k) std::memcpy(r.data() + k * bytes, all[k].data(), bytes);
      return r;
    });
  }

  std::string async_error() override { return aborted_.load() ? "host collective aborted: " + error() : ""; }
  void abort() override {
    {
      std::lock_guard<std::mutex> g(err_mu_);
      if (err_.empty()) err_ = "aborted";
    }
    aborted_ = true;
    if (shm_) shm_hdr()->abort.store(1, std::memory_order_release);
    shutdown_all();
  }
  bool aborted() const override { return aborted_.load(); }

 private:
  // pinned in / out stages, reused once the H2D that read `out` has completed (`done`)
  struct Staged {
    size_t cap = 0;
    void *in = nullptr, *out = nullptr;
    hipEvent_t done = nullptr;
    bool used = false;
  };
  struct Op {
    HostCollective* self;
    uint32_t kind;
    Staged* st;
    size_t in_bytes, out_bytes;
  };
  Staged* stage(size_t bytes) {
    for (Staged* st : pool_) {
      if (st->cap < bytes) continue;
      if (!st->used || hipEventQuery(st->done) == hipSuccess) return st;
    }
    Staged* st = new Staged();
    st->cap = std::max<size_t>(4096, bytes);
    HIP_OK(hipHostMalloc(&st->in, st->cap, hipHostMallocDefault));
    HIP_OK(hipHostMalloc(&st->out, st->cap * (size_t)n_, hipHostMallocDefault));
    HIP_OK(hipEventCreateWithFlags(&st->done, hipEventDisableTiming));
    pool_.push_back(st);
    return st;
  }
  void enqueue(hipStream_t s, uint32_t kind, const void* send, void* recv, size_t in_bytes, size_t out_bytes) {
    Staged* st = stage(in_bytes);
    HIP_OK(hipMemcpyAsync(st->in, send, in_bytes, hipMemcpyDeviceToHost, s));
    Op* op = new Op{this, kind, st, in_bytes, out_bytes};
    const hipError_t e = hipLaunchHostFunc(s, &HostCollective::run_op, op);
    if (e != hipSuccess) { delete op; HIP_OK(e); }
    HIP_OK(hipMemcpyAsync(recv, st->out, out_bytes, hipMemcpyHostToDevice, s));
    HIP_OK(hipEventRecord(st->done, s));
    st->used = true;
  }
  // HIP callback thread: no HIP calls here.  A failure marks the communicator aborted (the
  // engine's coll_wait sees async_error() and throws); the stream goes on with zeros.
  static void run_op(void* p) {
    Op* op = (Op*)p;
    HostCollective* self = op->self;
    try {
      if (self->aborted_.load()) throw std::runtime_error("aborted");
      std::vector<uint8_t> out;
      if (op->kind == 3u) {
        out = self->all_gather_host(std::vector<uint8_t>((uint8_t*)op->st->in, (uint8_t*)op->st->in + op->in_bytes));
      } else {
        std::vector<double> v(op->in_bytes / 8);
        std::memcpy(v.data(), op->st->in, op->in_bytes);
        const std::vector<double> r = self->all_reduce_host(v, op->kind == 1u);
        out.resize(op->in_bytes);
        std::memcpy(out.data(), r.data(), op->in_bytes);
      }
      if (out.size() != op->out_bytes) throw std::runtime_error("reply of unexpected size");
      std::memcpy(op->st->out, out.data(), out.size());
    } catch (const std::exception& e) {
      {
        std::lock_guard<std::mutex> g(self->err_mu_);
        if (self->err_.empty()) self->err_ = e.what();
      }
      self->aborted_ = true;
      std::memset(op->st->out, 0, op->out_bytes);
    }
    delete op;
  }
  std::string error() {
    std::lock_guard<std::mutex> g(err_mu_);
    return err_;
  }

  struct Hdr { uint32_t magic, op; uint64_t seq, bytes; };
  static constexpr uint32_t kMagic = 0x41504d43;  // "APMC"

  static void tune(int fd) {
    const int one = 1;
    ::setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
  }
  static bool send_all(int fd, const void* p, size_t n) {
    const char* c = (const char*)p;
    while (n) {
      const ssize_t w = ::send(fd, c, n, MSG_NOSIGNAL);
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) return false;
      c += w;
      n -= (size_t)w;
    }
    return true;
  }
  // false on EOF / error / deadline
  static bool recv_all(int fd, void* p, size_t n, double t_end) {
    char* c = (char*)p;
    while (n) {
      pollfd q{fd, POLLIN, 0};
      const double left = t_end - mono_ms();
      if (left <= 0) return false;
      const int pr = ::poll(&q, 1, (int)std::min(left, 1000.0));
      if (pr < 0 && errno == EINTR) continue;
      if (pr <= 0) continue;
      const ssize_t r = ::recv(fd, c, n, 0);
      if (r < 0 && (errno == EINTR || errno == EAGAIN)) continue;
      if (r <= 0) return false;
      c += r;
      n -= (size_t)r;
    }
    return true;
  }
  void shutdown_all() {
    for (int& f : fd_) {
      if (f >= 0) { ::shutdown(f, SHUT_RDWR); ::close(f); f = -1; }
    }
  }
  [[noreturn]] void fail(const std::string& why) {
    {
      std::lock_guard<std::mutex> g(err_mu_);
      err_ = why;
    }
    aborted_ = true;
    if (shm_) shm_hdr()->abort.store(1, std::memory_order_release);
    shutdown_all();
    throw std::runtime_error("host collective: " + why);
  }

  // ---- shared-memory data plane (ranks on one host: the rehearsal transport's usual case).
  // The TCP star stays for the rendezvous and for liveness: a dead peer's socket reads EOF.  Each
  // rank writes its contribution into its slot of the current parity, publishes the sequence
  // number, waits for every rank's, and combines all of them itself in rank order -- the same
  // bits on every rank, no round trip through rank 0.  A rank reuses a parity only two
  // collectives later, after every rank has published the one in between, which it does only
  // after reading this one.  Contributions over kShmSlot bytes go through TCP (every rank
  // decides alike: equal sizes per collective).  APM_HOSTCOLL_SHM=0: TCP only.
  static constexpr size_t kShmSlot = (size_t)1 << 20;
  static constexpr size_t kShmHead = 64;
  struct ShmHdr {
    uint64_t nonce;
    std::atomic<uint32_t> abort;
  };
  struct ShmSlot {
    std::atomic<uint64_t> seq;
    uint32_t op;
    uint32_t pad;
    uint64_t bytes;
  };
  ShmHdr* shm_hdr() { return (ShmHdr*)shm_; }
  char* shm_slot(int parity, int r) {
    return (char*)shm_ + kShmHead + ((size_t)parity * (size_t)n_ + (size_t)r) * (kShmHead + kShmSlot);
  }

  void shm_handshake(int port, double t_end) {
    const char* env = std::getenv("APM_HOSTCOLL_SHM");
    const bool want = !(env && env[0] == '0');
    const size_t len = kShmHead + 2 * (size_t)n_ * (kShmHead + kShmSlot);
    if (r_ == 0) {
      std::string name;
      uint64_t nonce = 0;
      void* m = MAP_FAILED;
      int fd = -1;
      if (want) {
        nonce = (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^ ((uint64_t)::getpid() << 32);
        name = "/apm_hc_" + std::to_string(port) + "_" + std::to_string(::getpid()) + "_" + std::to_string(nonce & 0xffffff);
        fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
        if (fd >= 0 && ::ftruncate(fd, (off_t)len) == 0)
          m = ::mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (m != MAP_FAILED) ((ShmHdr*)m)->nonce = nonce;
      }
      // the segment's name goes away on every path (a peer lost mid-handshake throws from fail())
      struct Unlink {
        const std::string& n;
        int fd;
        ~Unlink() {
          if (fd >= 0) { ::shm_unlink(n.c_str()); ::close(fd); }
        }
      } unlink_guard{name, fd};
      struct Unmap {
        void*& m;
        size_t len;
        bool keep = false;
        ~Unmap() {
          if (!keep && m != MAP_FAILED) ::munmap(m, len);
        }
      } unmap_guard{m, len};
      const uint32_t nl = m != MAP_FAILED ? (uint32_t)name.size() : 0u;
      bool all = nl > 0;
      for (int r = 1; r < n_; ++r) {
        if (!send_all(fd_[(size_t)r], &nl, 4) || (nl && (!send_all(fd_[(size_t)r], name.data(), nl) ||
                                                       !send_all(fd_[(size_t)r], &nonce, 8))))
          fail("shared-memory handshake: rank " + std::to_string(r) + " gone");
      }
      for (int r = 1; r < n_; ++r) {
        uint8_t ok = 0;
        if (!recv_all(fd_[(size_t)r], &ok, 1, t_end)) fail("shared-memory handshake: no reply from rank " + std::to_string(r));
        all = all && ok;
      }
      const uint8_t on = all ? 1 : 0;
      for (int r = 1; r < n_; ++r)
        if (!send_all(fd_[(size_t)r], &on, 1)) fail("shared-memory handshake: rank " + std::to_string(r) + " gone");
      // (unlink_guard: every rank has it mapped or gave up -- nothing is left behind in /dev/shm)
      if (on) { shm_ = m; shm_len_ = len; unmap_guard.keep = true; }
    } else {
      uint32_t nl = 0;
      if (!recv_all(fd_[0], &nl, 4, t_end)) fail("shared-memory handshake: rank 0 gone");
      void* m = MAP_FAILED;
      uint8_t ok = 0;
      if (nl) {
        std::string name(nl, '\0');
        uint64_t nonce = 0;
        if (!recv_all(fd_[0], &name[0], nl, t_end) || !recv_all(fd_[0], &nonce, 8, t_end))
          fail("shared-memory handshake: rank 0 gone");
        const int fd = want ? ::shm_open(name.c_str(), O_RDWR, 0600) : -1;
        if (fd >= 0) {
          m = ::mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
          ::close(fd);
        }
        ok = m != MAP_FAILED && ((ShmHdr*)m)->nonce == nonce;  // (another host's segment of that name: no)
      }
      if (!send_all(fd_[0], &ok, 1)) fail("shared-memory handshake: rank 0 gone");
      uint8_t on = 0;
      if (!recv_all(fd_[0], &on, 1, t_end)) fail("shared-memory handshake: rank 0 gone");
      if (on && ok) { shm_ = m; shm_len_ = len; }
      else if (m != MAP_FAILED) ::munmap(m, len);
    }
  }

  // a peer's socket reading EOF (or an error) = that process is gone
  bool peer_gone(int fd) {
    if (fd < 0) return true;
    pollfd q{fd, POLLIN, 0};
    if (::poll(&q, 1, 0) <= 0) return false;
    if (q.revents & (POLLHUP | POLLERR | POLLNVAL)) return true;
    char c;
    const ssize_t r = ::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
    return r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR);
  }

  template <class F>
  std::vector<uint8_t> shm_exchange(uint32_t op, uint64_t seq, const std::vector<uint8_t>& mine, F&& combine) {
    const int par = (int)(seq & 1);
    char* my = shm_slot(par, r_);
    ShmSlot* h = (ShmSlot*)my;
    if (!mine.empty()) std::memcpy(my + kShmHead, mine.data(), mine.size());
    h->op = op;
    h->bytes = mine.size();
    h->seq.store(seq, std::memory_order_release);
    const double t_end = mono_ms() + timeout_ms_;
    std::vector<std::vector<uint8_t>> all((size_t)n_);
    for (int q = 0; q < n_; ++q) {
      ShmSlot* hq = (ShmSlot*)shm_slot(par, q);
      double next_check = 0;
      for (uint32_t spin = 0; hq->seq.load(std::memory_order_acquire) != seq; ++spin) {
        if (spin < 4096) { _mm_pause(); continue; }
        if (shm_hdr()->abort.load(std::memory_order_acquire)) fail("a rank closed its connection: the collective was aborted (peer process gone)");
        const double now = mono_ms();
        if (now >= next_check) {
          if (r_ == 0) {
            for (int r = 1; r < n_; ++r)
              if (peer_gone(fd_[(size_t)r])) fail("rank " + std::to_string(r) + " closed its connection (peer process gone)");
          } else if (peer_gone(fd_[0])) {
            fail("rank 0 closed its connection (peer process gone)");
          }
          next_check = now + 1.0;
        }
        if (now >= t_end) fail("rank " + std::to_string(q) + " did not arrive within the collective timeout");
        std::this_thread::yield();
      }
      if (hq->op != op || hq->bytes != mine.size())
        fail("protocol mismatch with rank " + std::to_string(q) + " (ranks issued different collectives)");
      const char* d = shm_slot(par, q) + kShmHead;
      all[(size_t)q].assign(d, d + hq->bytes);
    }
    return combine(all);
  }

  template <class F>
  std::vector<uint8_t> exchange(uint32_t op, std::vector<uint8_t>&& mine, F&& combine) {
    if (aborted_.load()) throw std::runtime_error("host collective aborted: " + error());
    const uint64_t seq = ++seq_;
    if (n_ == 1) {
      std::vector<std::vector<uint8_t>> all(1);
      all[0] = std::move(mine);
      return combine(all);
    }
    if (shm_ && mine.size() <= kShmSlot) return shm_exchange(op, seq, mine, combine);
    const double t_end = mono_ms() + timeout_ms_;
    const Hdr h{kMagic, op, seq, (uint64_t)mine.size()};
    if (r_ != 0) {
      if (!send_all(fd_[0], &h, sizeof h) || !send_all(fd_[0], mine.data(), mine.size()))
        fail("rank 0 closed its connection (peer process gone)");
      Hdr rh{};
      if (!recv_all(fd_[0], &rh, sizeof rh, t_end))
        fail(mono_ms() >= t_end ? "no reply from rank 0 within the collective timeout"
                                : "rank 0 closed its connection (peer process gone)");
      if (rh.magic != kMagic || rh.op != op || rh.seq != seq) fail("protocol mismatch (ranks issued different collectives)");
      std::vector<uint8_t> out(rh.bytes);
      if (!recv_all(fd_[0], out.data(), out.size(), t_end)) fail("rank 0 connection lost mid-message");
      return out;
    }
    std::vector<std::vector<uint8_t>> all((size_t)n_);
    all[0] = std::move(mine);
    for (int r = 1; r < n_; ++r) {
      Hdr ph{};
      if (!recv_all(fd_[(size_t)r], &ph, sizeof ph, t_end))
        fail(mono_ms() >= t_end ? "rank " + std::to_string(r) + " did not arrive within the collective timeout"
                                : "rank " + std::to_string(r) + " closed its connection (peer process gone)");
      if (ph.magic != kMagic || ph.op != op || ph.seq != seq || ph.bytes != h.bytes)
        fail("protocol mismatch with rank " + std::to_string(r) + " (ranks issued different collectives)");
      all[(size_t)r].resize(ph.bytes);
      if (!recv_all(fd_[(size_t)r], all[(size_t)r].data(), ph.bytes, t_end))
        fail("rank " + std::to_string(r) + " connection lost mid-message");
    }
    std::vector<uint8_t> out = combine(all);
    const Hdr oh{kMagic, op, seq, (uint64_t)out.size()};
    for (int r = 1; r < n_; ++r)
      if (!send_all(fd_[(size_t)r], &oh, sizeof oh) || !send_all(fd_[(size_t)r], out.data(), out.size()))
        fail("rank " + std::to_string(r) + " closed its connection (peer process gone)");
    return out;
  }

  int n_, r_;
  double timeout_ms_;
  std::vector<int> fd_;  // rank 0: one per peer; others: [0] = rank 0
  uint64_t seq_ = 0;
  std::atomic<bool> aborted_{false};
  std::mutex err_mu_;
  std::string err_;
  std::vector<Staged*> pool_;  // enqueue side (the engine's ingest thread)
  void* shm_ = nullptr;        // shared-memory data plane (shm_handshake), or none
  size_t shm_len_ = 0;
};

}  // namespace

std::unique_ptr<Collective> make_host_collective(const std::string& addr, int port, int nranks, int rank,
                                                 double timeout_ms) {
  return std::unique_ptr<Collective>(new HostCollective(addr, port, nranks, rank, timeout_ms));
}

}  // namespace apm
