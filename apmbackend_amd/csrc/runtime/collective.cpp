// Collective backends: RCCL (production) and an in-process rendezvous (tests).
#include "collective.h"

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
  RcclCollective(const std::vector<uint8_t>& uid, int nranks, int rank) : n_(nranks), r_(rank) {
    if (uid.size() != sizeof(ncclUniqueId)) throw std::runtime_error("bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    if (ncclCommInitRank(&comm_, nranks, id, rank) != ncclSuccess) throw std::runtime_error("ncclCommInitRank failed");
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

std::unique_ptr<Collective> make_rccl_collective(const std::vector<uint8_t>& uid, int nranks, int rank) {
  return std::unique_ptr<Collective>(new RcclCollective(uid, nranks, rank));
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
