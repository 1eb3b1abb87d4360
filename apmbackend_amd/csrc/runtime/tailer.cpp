// Native log tailer: the MI355X-native replacement of perl_tail.pl + File::Tail
// (perl_tail.pl:13-42, stream_parse_transactions.js:902-975).
//
//  * One Tailer follows many files and produces whole-line batches laid out exactly as the
//    engine's canonical fast path wants them (engine.cpp launch_parse): chunks grouped by server,
//    contiguous from byte 0, every chunk ending in '\n' -- so the batch is DMA'd to the GPU
//    straight from the buffer it was read into, with no host re-layout.
//  * Batches can be read straight into caller-owned pinned slots (`poll_into`) and, with
//    `start()`, by a read-ahead thread that keeps a ring of pinned slots full while the engine
//    processes the previous batch.  Per-file reads of one batch run on a small pread pool.
//  * Each file's cut point (its last complete line inside the budget) is found first with a
//    small tail probe, so the preads land at their final offsets (no compaction copy).
//  * Lines longer than the per-file budget are still read whole (the budget stretches to the
//    next newline, up to the batch size); a line longer than a whole batch is skipped and counted
//    instead of stalling its file forever.
//  * Rotation (inode change): the old inode stays open and is drained to EOF -- its complete
//    lines first, then (once it stops growing) an unterminated last line closed with '\n' --
//    before the tailer moves to the new file.  Truncation (same inode, size < offset) restarts
//    the file at 0 (File::Tail resetafter, without the NFS inode assertion the reference patched).
//  * The pause-file contract is kept: while `pause_file` exists nothing is read (perl_tail.pl:36-41).
//  * Offsets are committed per batch (`commit(batch_id)`) after the engine consumed it, and are
//    persisted as JSON with escaped paths, fsync'd file + directory and an atomic rename.  The
//    reference lacked persisted offsets altogether (restart = data gap).
//  * `wait()` blocks on inotify (parent directories: modify / create / move) instead of polling.
#include <fcntl.h>
#include <poll.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/inotify.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

namespace py = pybind11;

namespace apm {

namespace {

constexpr uint64_t kProbe = 64 * 1024;

std::string json_escape(const std::string& s) {
  std::string o;
  o.reserve(s.size() + 2);
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += (char)c;
        }
    }
  }
  return o;
}

ssize_t pread_full(int fd, char* dst, uint64_t len, uint64_t off) {
  uint64_t got = 0;
  while (got < len) {
    const ssize_t r = ::pread(fd, dst + got, len - got, (off_t)(off + got));
    if (r < 0) {
      if (errno == EINTR) continue;
      return got ? (ssize_t)got : -1;
    }
    if (r == 0) break;
    got += (uint64_t)r;
  }
  return (ssize_t)got;
}

// Fixed pool running one parallel-for at a time (the per-file preads of a batch).
class ReadPool {
 public:
  explicit ReadPool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~ReadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size(); }
  void run(size_t n, const std::function<void(size_t)>& f) {
    if (th_.empty() || n <= 1) {
      for (size_t i = 0; i < n; ++i) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &f;
      n_ = n;
      next_.store(0);
      busy_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    for (size_t i; (i = next_.fetch_add(1)) < n;) f(i);  // the caller works too
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return busy_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(size_t)>* f;
      size_t n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        f = fn_;
        n = n_;
      }
      for (size_t i; (i = next_.fetch_add(1)) < n;) (*f)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--busy_ == 0) done_cv_.notify_all();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(size_t)>* fn_ = nullptr;
  size_t n_ = 0;
  std::atomic<size_t> next_{0};
  int busy_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace

struct TailFile {
  std::string path;
  int32_t file_id = 0;
  int32_t group = 0;  // server rank: batches are laid out grouped by it
  int fd = -1;
  uint64_t ino = 0;
  uint64_t offset = 0;        // read position (read-ahead)
  uint64_t committed = 0;     // position of the last batch the caller committed
  uint64_t committed_ino = 0;
  bool starved = false;       // its next line did not fit the last batch: planned first next time
  // rotation: the previous inode, drained before the tailer reads the new one
  int old_fd = -1;
  uint64_t old_ino = 0, old_offset = 0, old_last_size = UINT64_MAX;
};

class Tailer {
 public:
  using ChunkList = std::vector<std::tuple<int32_t, uint64_t, uint64_t>>;

  Tailer(std::string pause_file, uint64_t max_batch_bytes, int read_threads)
      : pause_file_(std::move(pause_file)), max_batch_(max_batch_bytes), pool_(std::max(0, read_threads)) {
    ino_fd_ = inotify_init1(IN_NONBLOCK | IN_CLOEXEC);
  }
  ~Tailer() {
    stop();
    for (auto& f : files_) {
      if (f.fd >= 0) ::close(f.fd);
      if (f.old_fd >= 0) ::close(f.old_fd);
    }
    if (ino_fd_ >= 0) ::close(ino_fd_);
  }

  void add(const std::string& path, int32_t file_id, bool from_start, int32_t group) {
    std::lock_guard<std::mutex> lk(mu_);
    std::lock_guard<std::mutex> ck(cmu_);
    TailFile f;
    f.path = path;
    f.file_id = file_id;
    f.group = group;
    struct stat st;
    if (::stat(path.c_str(), &st) == 0) {
      f.ino = st.st_ino;
      f.offset = from_start ? 0 : (uint64_t)st.st_size;
    }
    f.committed = f.offset;
    f.committed_ino = f.ino;
    files_.push_back(f);
    order_.resize(files_.size());
    for (size_t i = 0; i < order_.size(); ++i) order_[i] = i;
    std::stable_sort(order_.begin(), order_.end(), [&](size_t a, size_t b) { return files_[a].group < files_[b].group; });
    if (ino_fd_ >= 0) {
      const size_t slash = path.rfind('/');
      const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
      if (dirs_.insert(dir).second)
        inotify_add_watch(ino_fd_, dir.c_str(), IN_MODIFY | IN_CREATE | IN_MOVED_TO | IN_CLOSE_WRITE);
    }
  }

  bool paused() const {
    struct stat st;
    return !pause_file_.empty() && ::stat(pause_file_.c_str(), &st) == 0;
  }

  // Synchronous poll into an internal buffer; offsets are committed at once.
  std::pair<py::bytes, ChunkList> poll() {
    std::string buf;
    ChunkList chunks;
    uint64_t n = 0;
    int64_t id;
    {
      py::gil_scoped_release rel;
      buf.resize(max_batch_ + 64);
      std::lock_guard<std::mutex> lk(mu_);
      id = read_batch(&buf[0], max_batch_, chunks, n);
      std::lock_guard<std::mutex> ck(cmu_);
      commit_locked(id);
    }
    buf.resize(n);
    return {py::bytes(buf), chunks};
  }

  // Reads the next batch into dst (cap bytes).  Returns (n_bytes, chunks, batch_id); the
  // batch's offsets become the persisted ones only at commit(batch_id).
  std::tuple<uint64_t, ChunkList, int64_t> poll_into(uintptr_t dst, uint64_t cap) {
    ChunkList chunks;
    uint64_t n = 0;
    py::gil_scoped_release rel;
    std::lock_guard<std::mutex> lk(mu_);
    const int64_t id = read_batch((char*)dst, std::min(cap, max_batch_), chunks, n);
    return {n, chunks, id};
  }

  // (the commit lock only: the read-ahead thread holds mu_ through a whole batch read, ~0.7 ms,
  // which the ingest loop's per-batch commit waited out)
  void commit(int64_t id) {
    std::lock_guard<std::mutex> lk(cmu_);
    commit_locked(id);
  }

  // ---- read-ahead ring over caller-owned (pinned) slots
  void start(const std::vector<uintptr_t>& slots, uint64_t slot_bytes, double idle_ms) {
    stop();
    {
      std::lock_guard<std::mutex> lk(ra_mu_);
      free_.clear();
      ready_.clear();
      slots_ = slots;
      slot_bytes_ = slot_bytes;
      for (size_t i = 0; i < slots.size(); ++i) free_.push_back((int)i);
      ra_stop_ = false;
      ra_error_.clear();
    }
    idle_ms_ = idle_ms;
    ra_ = std::thread([this] { readahead_loop(); });
  }

  void stop() {
    {
      std::lock_guard<std::mutex> lk(ra_mu_);
      ra_stop_ = true;
    }
    ra_cv_.notify_all();
    if (ra_.joinable()) ra_.join();
  }

  // Next ready batch: (slot, ptr, n_bytes, chunks, batch_id), or None after timeout_ms.
  py::object next(double timeout_ms) {
    Ready r;
    std::string err;
    bool got = false;
    {
      py::gil_scoped_release rel;
      std::unique_lock<std::mutex> lk(ra_mu_);
      ra_cv_.wait_for(lk, std::chrono::microseconds((int64_t)(timeout_ms * 1000)),
                      [&] { return !ready_.empty() || !ra_error_.empty() || ra_stop_; });
      if (!ra_error_.empty()) {
        err = ra_error_;
      } else if (!ready_.empty()) {
        r = std::move(ready_.front());
        ready_.pop_front();
        got = true;
      }
    }
    if (!err.empty()) throw std::runtime_error("tailer read-ahead: " + err);
    if (!got) return py::none();
    return py::make_tuple(r.slot, slots_[r.slot], r.n, r.chunks, r.id);
  }

  // Peek at the batch after the one just taken (for the engine's speculative next-parse).
  py::object peek() {
    std::lock_guard<std::mutex> lk(ra_mu_);
    if (ready_.empty()) return py::none();
    const Ready& r = ready_.front();
    return py::make_tuple(r.slot, slots_[r.slot], r.n, r.chunks, r.id);
  }

  void release(int slot) {
    {
      std::lock_guard<std::mutex> lk(ra_mu_);
      free_.push_back(slot);
    }
    ra_cv_.notify_all();
  }

  // Blocks until a watched directory reports a change (or timeout).  Returns true on a change.
  bool wait(double timeout_ms) {
    py::gil_scoped_release rel;
    return wait_change(timeout_ms);
  }

  std::string offsets_json() const {
    std::lock_guard<std::mutex> lk(cmu_);
    std::string o = "{";
    for (size_t i = 0; i < files_.size(); ++i) {
      if (i) o += ",";
      o += "\"" + json_escape(files_[i].path) + "\":[" + std::to_string(files_[i].committed) + "," +
           std::to_string(files_[i].committed_ino) + "]";
    }
    return o + "}";
  }

  void save_offsets(const std::string& path) const {
    const std::string body = offsets_json();
    const std::string tmp = path + ".tmp";
    const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) throw std::runtime_error("save_offsets: cannot open " + tmp);
    const char* p = body.data();
    size_t left = body.size();
    while (left) {
      const ssize_t w = ::write(fd, p, left);
      if (w < 0) {
        if (errno == EINTR) continue;
        ::close(fd);
        throw std::runtime_error("save_offsets: write failed");
      }
      p += w;
      left -= (size_t)w;
    }
    ::fsync(fd);
    ::close(fd);
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("save_offsets: rename failed");
    const size_t slash = path.rfind('/');
    const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
    const int dfd = ::open(dir.c_str(), O_RDONLY | O_DIRECTORY | O_CLOEXEC);
    if (dfd >= 0) {
      ::fsync(dfd);
      ::close(dfd);
    }
  }

  void set_offset(const std::string& path, uint64_t offset, uint64_t inode) {
    std::lock_guard<std::mutex> lk(mu_);
    std::lock_guard<std::mutex> ck(cmu_);
    for (auto& f : files_) {
      if (f.path != path) continue;
      struct stat st;
      const bool same = ::stat(path.c_str(), &st) == 0 && (uint64_t)st.st_ino == inode;
      // a checkpoint taken before a rotation names the old inode, which is gone: new file from 0
      f.offset = same || inode == 0 ? offset : 0;
      f.ino = same || inode == 0 ? inode : (uint64_t)st.st_ino;
      if (f.fd >= 0) { ::close(f.fd); f.fd = -1; }
      f.committed = f.offset;
      f.committed_ino = f.ino;
    }
  }

  std::vector<std::tuple<std::string, uint64_t, uint64_t>> offsets() const {
    std::lock_guard<std::mutex> lk(cmu_);
    std::vector<std::tuple<std::string, uint64_t, uint64_t>> r;
    for (auto& f : files_) r.emplace_back(f.path, f.committed, f.committed_ino);
    return r;
  }

  py::dict stats() const {
    std::lock_guard<std::mutex> lk(mu_);
    py::dict d;
    d["bytes_read"] = bytes_read_;
    d["batches"] = batches_;
    d["rotations"] = rotations_;
    d["truncations"] = truncations_;
    d["overlong_lines_skipped"] = overlong_;
    d["unterminated_lines_closed"] = closed_partial_;
    d["read_threads"] = pool_.size() + 1;
    d["plan_ms"] = plan_ms_;
    d["read_ms"] = read_ms_;
    return d;
  }
  uint64_t bytes_read() const { return bytes_read_; }

 private:
  struct Part {  // one pread of a batch
    size_t file;
    bool old;
    uint64_t src, len, dst;
    bool add_nl;  // closing an unterminated last line of a rotated-away inode
  };
  struct Ready {
    int slot = -1;
    uint64_t n = 0;
    ChunkList chunks;
    int64_t id = -1;
  };

  bool wait_change(double timeout_ms) {
    if (ino_fd_ < 0) {
      std::this_thread::sleep_for(std::chrono::microseconds((int64_t)(timeout_ms * 1000)));
      return false;
    }
    struct pollfd p{ino_fd_, POLLIN, 0};
    const int r = ::poll(&p, 1, (int)timeout_ms);
    if (r <= 0) return false;
    alignas(struct inotify_event) char buf[16384];
    while (::read(ino_fd_, buf, sizeof buf) > 0) {
    }
    return true;
  }

  static uint64_t fd_size(int fd) {
    struct stat st;
    return ::fstat(fd, &st) == 0 ? (uint64_t)st.st_size : 0;
  }

  // Offset just past the last '\n' in [lo, hi) of fd, or UINT64_MAX.
  static uint64_t last_newline_end(int fd, uint64_t lo, uint64_t hi, std::vector<char>& scratch) {
    scratch.resize(kProbe);
    while (hi > lo) {
      const uint64_t a = hi - lo > kProbe ? hi - kProbe : lo;
      const ssize_t got = pread_full(fd, scratch.data(), hi - a, a);
      if (got <= 0) return UINT64_MAX;
      const void* q = memrchr(scratch.data(), '\n', (size_t)got);
      if (q) return a + (uint64_t)((const char*)q - scratch.data()) + 1;
      hi = a;
    }
    return UINT64_MAX;
  }

  // Offset just past the first '\n' in [lo, limit) of fd, or UINT64_MAX.
  static uint64_t first_newline_end(int fd, uint64_t lo, uint64_t limit, std::vector<char>& scratch) {
    scratch.resize(kProbe);
    while (lo < limit) {
      const uint64_t n = std::min<uint64_t>(kProbe, limit - lo);
      const ssize_t got = pread_full(fd, scratch.data(), n, lo);
      if (got <= 0) return UINT64_MAX;
      const void* q = memchr(scratch.data(), '\n', (size_t)got);
      if (q) return lo + (uint64_t)((const char*)q - scratch.data()) + 1;
      lo += (uint64_t)got;
    }
    return UINT64_MAX;
  }

  void check_rotation(TailFile& f) {
    struct stat st;
    if (::stat(f.path.c_str(), &st) != 0) return;  // moved away, new one not created yet
    if (f.fd >= 0 && (uint64_t)st.st_ino != f.ino) {
      // rotated: keep draining the old inode before switching
      if (f.old_fd >= 0) ::close(f.old_fd);  // rotated twice before the first drained: give up on it
      f.old_fd = f.fd;
      f.old_ino = f.ino;
      f.old_offset = f.offset;
      f.old_last_size = UINT64_MAX;
      f.fd = -1;
      f.ino = st.st_ino;
      f.offset = 0;
      ++rotations_;
    } else if (f.fd < 0 && f.ino && (uint64_t)st.st_ino != f.ino) {
      f.ino = st.st_ino;  // rotated while closed (restart): start the new file
      f.offset = 0;
    }
    if (f.fd < 0) {
      f.fd = ::open(f.path.c_str(), O_RDONLY | O_CLOEXEC);
      if (f.fd < 0) return;
      f.ino = st.st_ino;
    }
    const uint64_t size = fd_size(f.fd);
    if (size < f.offset) {
      f.offset = 0;  // truncated in place
      ++truncations_;
    }
  }

  // Plans how many bytes of fd [off, size) go into this batch: the cut is the end of the last
  // complete line within `budget`; if the first line alone is longer, the budget stretches to
  // its end (up to `room`).  Returns the byte count (0 = nothing ready) and sets `skip_to` when
  // a line longer than a whole batch has to be skipped.
  uint64_t plan_file(int fd, uint64_t off, uint64_t size, uint64_t budget, uint64_t room, uint64_t& skip_to,
                     bool& starved, std::vector<char>& scratch) {
    skip_to = 0;
    starved = false;
    if (size <= off) return 0;
    const uint64_t want = std::min(size - off, std::min(budget, room));
    uint64_t cut = want ? last_newline_end(fd, off, off + want, scratch) : UINT64_MAX;
    if (cut != UINT64_MAX) return cut - off;
    // no newline inside the budget: one long line
    const uint64_t lim = std::min(size, off + max_batch_);
    cut = first_newline_end(fd, off + want, lim, scratch);
    if (cut == UINT64_MAX) {
      if (size - off >= max_batch_) {  // longer than any batch can hold: skip it
        const uint64_t e = first_newline_end(fd, lim, size, scratch);
        if (e != UINT64_MAX) skip_to = e;
      }
      return 0;  // still being written
    }
    if (cut - off <= room) return cut - off;
    starved = true;  // fits a batch, but not what is left of this one
    return 0;
  }

  int64_t read_batch(char* dst, uint64_t cap, ChunkList& chunks, uint64_t& n_out) {
    n_out = 0;
    const int64_t id = next_id_++;
    std::vector<std::pair<size_t, std::pair<uint64_t, uint64_t>>> ends;  // file -> (offset, ino)
    if (paused() || files_.empty()) {
      std::lock_guard<std::mutex> ck(cmu_);
      pending_[id] = ends;
      return id;
    }
    const auto tp0 = std::chrono::steady_clock::now();
    for (auto& f : files_) check_rotation(f);
    // budgets: starved files first (their whole next line), then a fair share for everyone
    const size_t nf = files_.size();
    std::vector<uint64_t> take_old(nf, 0), take(nf, 0);
    std::vector<char> close_old(nf, 0), add_nl(nf, 0);
    uint64_t room = cap;
    const uint64_t share = std::max<uint64_t>(kProbe, cap / std::max<size_t>(1, nf));
    std::vector<size_t> plan_order;
    for (size_t i = 0; i < nf; ++i)
      if (files_[i].starved) plan_order.push_back(i);
    for (size_t i = 0; i < nf; ++i)
      if (!files_[i].starved) plan_order.push_back(i);
    std::vector<char>& scratch = scratch_;
    for (size_t i : plan_order) {
      TailFile& f = files_[i];
      bool starved = false;
      uint64_t skip = 0;
      if (f.old_fd >= 0) {  // drain the rotated inode first
        const uint64_t osz = fd_size(f.old_fd);
        uint64_t t;
        for (;;) {  // a skipped over-long line: plan again from behind it
          t = plan_file(f.old_fd, f.old_offset, osz, osz - std::min(osz, f.old_offset), room, skip, starved, scratch);
          if (!skip) break;
          f.old_offset = skip;
          ++overlong_;
        }
        take_old[i] = t;
        room -= t;
        if (t == 0 && !starved) {
          const uint64_t rest = osz - std::min(osz, f.old_offset);
          if (rest == 0 || (osz == f.old_last_size && rest + 1 <= room)) {
            // drained (or its unterminated last line stopped growing): close it with '\n'
            if (rest) { take_old[i] = rest + 1; room -= rest + 1; add_nl[i] = 1; ++closed_partial_; }
            close_old[i] = 1;
          }
        }
        f.old_last_size = osz;
        if (starved || (f.old_fd >= 0 && !close_old[i])) {  // the new inode waits for the old one
          f.starved = starved;
          continue;
        }
      }
      if (f.fd < 0) continue;
      const uint64_t sz = fd_size(f.fd);
      uint64_t t;
      for (;;) {
        t = plan_file(f.fd, f.offset, sz, f.starved ? room : share, room, skip, starved, scratch);
        if (!skip) break;
        f.offset = skip;
        ++overlong_;
      }
      take[i] = t;
      room -= t;
      f.starved = starved;
    }
    // layout in canonical order (grouped by server), then the preads in parallel
    std::vector<Part> parts;
    uint64_t pos = 0;
    for (size_t i : order_) {
      TailFile& f = files_[i];
      const uint64_t begin = pos;
      if (take_old[i]) {
        const bool nl = add_nl[i] != 0;
        parts.push_back({i, true, f.old_offset, take_old[i] - (nl ? 1 : 0), pos, nl});
        pos += take_old[i];
      }
      if (take[i]) {
        parts.push_back({i, false, f.offset, take[i], pos, false});
        pos += take[i];
      }
      if (pos > begin) chunks.emplace_back(f.file_id, begin, pos);
    }
    // A busy log (the SOAP / app logs of a JVM) is most of a batch: one pread per file left a
    // few threads copying megabytes each while the rest idled (7-8 GB/s whatever the pool size).
    // Large reads are split into kSplit pieces, so the pool copies the page cache in parallel.
    {
      constexpr uint64_t kSplit = 1ull << 20;
      std::vector<Part> split;
      split.reserve(parts.size() + pos / kSplit + 1);
      for (const Part& p : parts) {
        if (p.len <= kSplit + kSplit / 2) { split.push_back(p); continue; }
        for (uint64_t o = 0; o < p.len; o += kSplit) {
          const uint64_t n = std::min(kSplit, p.len - o);
          split.push_back({p.file, p.old, p.src + o, n, p.dst + o, p.add_nl && o + n == p.len});
        }
      }
      parts.swap(split);
    }
    std::atomic<int> short_reads{0};
    const auto tp1 = std::chrono::steady_clock::now();
    pool_.run(parts.size(), [&](size_t k) {
      const Part& p = parts[k];
      const TailFile& f = files_[p.file];
      const ssize_t got = pread_full(p.old ? f.old_fd : f.fd, dst + p.dst, p.len, p.src);
      if (got != (ssize_t)p.len) short_reads.fetch_add(1);
      if (p.add_nl) dst[p.dst + p.len] = '\n';
    });
    if (short_reads.load()) {
      // a file shrank between the probe and the read (truncation race): keep nothing of this
      // batch; the next poll re-plans from the same offsets
      chunks.clear();
      std::lock_guard<std::mutex> ck(cmu_);
      pending_[id] = ends;
      return id;
    }
    for (const Part& p : parts) {
      TailFile& f = files_[p.file];
      if (p.old) f.old_offset += p.len;
      else f.offset += p.len;
    }
    for (size_t i = 0; i < nf; ++i) {
      TailFile& f = files_[i];
      if (close_old[i] && f.old_fd >= 0) {
        ::close(f.old_fd);
        f.old_fd = -1;
      }
      // committed position after this batch: the old inode while it is being drained
      if (f.old_fd >= 0) ends.push_back({i, {f.old_offset, f.old_ino}});
      else ends.push_back({i, {f.offset, f.ino}});
    }
    {
      std::lock_guard<std::mutex> ck(cmu_);
      pending_[id] = std::move(ends);
    }
    n_out = pos;
    if (pos) std::memset(dst + pos, 0, std::min<uint64_t>(64, cap + 64 - pos));
    bytes_read_ += pos;
    ++batches_;
    const auto tp2 = std::chrono::steady_clock::now();
    plan_ms_ += std::chrono::duration<double, std::milli>(tp1 - tp0).count();
    read_ms_ += std::chrono::duration<double, std::milli>(tp2 - tp1).count();
    return id;
  }

  void commit_locked(int64_t id) {  // cmu_ held
    for (auto it = pending_.begin(); it != pending_.end() && it->first <= id;) {
      for (const auto& e : it->second) {
        files_[e.first].committed = e.second.first;
        files_[e.first].committed_ino = e.second.second;
      }
      it = pending_.erase(it);
    }
  }

  void readahead_loop() {
    for (;;) {
      int slot;
      {
        std::unique_lock<std::mutex> lk(ra_mu_);
        ra_cv_.wait(lk, [&] { return ra_stop_ || !free_.empty(); });
        if (ra_stop_) return;
        slot = free_.front();
        free_.pop_front();
      }
      Ready r;
      r.slot = slot;
      try {
        for (;;) {
          {
            std::lock_guard<std::mutex> lk(mu_);
            r.chunks.clear();
            r.id = read_batch((char*)slots_[slot], std::min(slot_bytes_, max_batch_), r.chunks, r.n);
            // An empty read only restates positions of earlier batches (or moves a drained
            // rotation to the new inode).  Committing it would commit every earlier batch still
            // waiting in a slot, before the engine has its lines -- a checkpoint would then store
            // offsets past state it does not hold.  So it commits only when nothing is pending.
            if (r.n == 0) {
              std::lock_guard<std::mutex> ck(cmu_);
              if (pending_.begin()->first == r.id) commit_locked(r.id);
              else pending_.erase(r.id);
            }
          }
          if (r.n > 0) break;
          {
            std::lock_guard<std::mutex> lk(ra_mu_);
            if (ra_stop_) return;
          }
          wait_change(idle_ms_);
        }
      } catch (const std::exception& e) {
        std::lock_guard<std::mutex> lk(ra_mu_);
        ra_error_ = e.what();
        ra_cv_.notify_all();
        return;
      }
      {
        std::lock_guard<std::mutex> lk(ra_mu_);
        ready_.push_back(std::move(r));
      }
      ra_cv_.notify_all();
    }
  }

  std::string pause_file_;
  uint64_t max_batch_;
  // mu_: the read state (files_' read positions and fds, the read-ahead's batch reads);
  // cmu_: the commit state (pending_, files_' committed positions).  Order: mu_ before cmu_.
  mutable std::mutex mu_;
  mutable std::mutex cmu_;
  std::vector<TailFile> files_;
  std::vector<size_t> order_;
  std::vector<char> scratch_;
  std::map<int64_t, std::vector<std::pair<size_t, std::pair<uint64_t, uint64_t>>>> pending_;
  int64_t next_id_ = 0;
  uint64_t bytes_read_ = 0, batches_ = 0, rotations_ = 0, truncations_ = 0, overlong_ = 0, closed_partial_ = 0;
  double plan_ms_ = 0, read_ms_ = 0;  // read_batch: planning (sizes, tail probes) / the parallel preads
  ReadPool pool_;
  int ino_fd_ = -1;
  std::set<std::string> dirs_;
  // read-ahead
  std::thread ra_;
  std::mutex ra_mu_;
  std::condition_variable ra_cv_;
  std::vector<uintptr_t> slots_;
  uint64_t slot_bytes_ = 0;
  std::deque<int> free_;
  std::deque<Ready> ready_;
  bool ra_stop_ = true;
  std::string ra_error_;
  double idle_ms_ = 50.0;
};

}  // namespace apm

void register_tailer(py::module_& m) {
  using apm::Tailer;
  py::class_<Tailer>(m, "Tailer")
      .def(py::init<std::string, uint64_t, int>(), py::arg("pause_file"), py::arg("max_batch_bytes") = 32ull << 20,
           py::arg("read_threads") = 3)
      .def("add", &Tailer::add, py::arg("path"), py::arg("file_id"), py::arg("from_start") = false,
           py::arg("group") = 0)
      .def("poll", &Tailer::poll)
      .def("poll_into", &Tailer::poll_into, py::arg("dst"), py::arg("cap"))
      .def("commit", &Tailer::commit)
      .def("start", &Tailer::start, py::arg("slots"), py::arg("slot_bytes"), py::arg("idle_ms") = 50.0)
      .def("stop", &Tailer::stop, py::call_guard<py::gil_scoped_release>())
      .def("next", &Tailer::next, py::arg("timeout_ms") = 0.0)
      .def("peek", &Tailer::peek)
      .def("release", &Tailer::release)
      .def("wait", &Tailer::wait, py::arg("timeout_ms"))
      .def("paused", &Tailer::paused)
      .def("save_offsets", &Tailer::save_offsets, py::call_guard<py::gil_scoped_release>())
      .def("offsets_json", &Tailer::offsets_json)
      .def("set_offset", &Tailer::set_offset)
      .def("offsets", &Tailer::offsets)
      .def("stats", &Tailer::stats)
      .def("bytes_read", &Tailer::bytes_read);
}
