// Native DB insert stage: the MI355X-native replacement of stream_insert_db.js's buffering +
// pg-promise multi-row INSERT path (stream_insert_db.js:277-353, dbstats.js:1-45).
//
// Semantics kept from the reference:
//  * one buffer per record type (tx / fs / al / jx, entries.js toPostgresObject types);
//  * a buffer already holding `limit` rows is flushed *before* the next row is appended (so one
//    flush carries at most `limit` rows, :341-345), and `max_wait_ms` after the first row entered
//    an empty buffer it is flushed by the timer (:333-339);
//  * a failed flush puts its rows back at the *front* of the buffer, retried with the next flush
//    (:310-320); DBStats rows / ms are kept per interval (dbstats.js).
// Changed for throughput:
//  * rows travel as wire lines until a flush; the COPY text encoding (copyenc.cpp) runs on a pool
//    of encoder threads, and one writer thread loads the encoded flushes in submission order;
//  * loading is `COPY table (cols) FROM STDIN` -- through one long-lived `psql` process per sink
//    (each flush one COPY, acknowledged with an `\echo` marker carrying psql's :ERROR), or as
//    append-only COPY spool files (`<table>.copy`, rotated by size; load with \copy), or null.
//  * The caller's thread only splits lines into the per-type buffers (memchr speed).
#include <fcntl.h>
#include <poll.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <signal.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/uio.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <string_view>
#include <thread>
#include <vector>

#include "engine.h"

extern char** environ;

namespace py = pybind11;

namespace apm {
namespace copyenc {
void encode_blob(std::string_view blob, std::string* out, int64_t* counts);
}

namespace {

constexpr int NT = 5;  // tx, fs, al, jx, fb

double mono_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int type_of(std::string_view line) {
  if (line.size() < 3 || line[2] != '|') return -1;
  const char a = line[0], b = line[1];
  if (a == 't' && b == 'x') return 0;
  if (a == 'f' && b == 's') return 1;
  if (a == 'a' && b == 'l') return 2;
  if (a == 'j' && b == 'x') return 3;
  if (a == 'f' && b == 'b') return 4;
  return -1;
}

bool write_all(int fd, const char* p, size_t n) {
  while (n) {
    const ssize_t w = ::write(fd, p, n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return false;
    }
    p += w;
    n -= (size_t)w;
  }
  return true;
}

// ----------------------------------------------------------------------------- writers
struct Writer {
  virtual ~Writer() = default;
  // returns "" on success, else the error text
  virtual std::string write(int type, const std::string& table, const std::string& columns, std::string_view rows) = 0;
  // Several consecutive flushes of one type, in order; returns how many were written (the rest
  // failed with `err`).  Default: one at a time.
  virtual size_t write_run(int type, const std::string& table, const std::string& columns,
                           const std::vector<std::string_view>& rows, std::string& err) {
    for (size_t i = 0; i < rows.size(); ++i) {
      err = write(type, table, columns, rows[i]);
      if (!err.empty()) return i;
    }
    return rows.size();
  }
};

struct NullWriter : Writer {
  std::string write(int, const std::string&, const std::string&, std::string_view) override { return ""; }
};

// Append-only COPY text files, one per table, rotated by size.
struct SpoolWriter : Writer {
  std::string dir;
  uint64_t rotate;
  std::string suffix;  // "" for lane 0, ".lane<k>" for writer lane k
  int fd[NT] = {-1, -1, -1, -1, -1};
  uint64_t size[NT] = {0, 0, 0, 0, 0};
  SpoolWriter(std::string d, uint64_t r, std::string sfx = "") : dir(std::move(d)), rotate(r), suffix(std::move(sfx)) {
    ::mkdir(dir.c_str(), 0755);
  }
  ~SpoolWriter() override {
    for (int f : fd)
      if (f >= 0) ::close(f);
  }
  std::string write(int type, const std::string& table, const std::string& columns, std::string_view rows) override {
    const std::string path = dir + "/" + table + suffix + ".copy";
    if (fd[type] >= 0 && rotate && size[type] >= rotate) {
      ::close(fd[type]);
      fd[type] = -1;
      const auto ms = (long long)std::chrono::duration_cast<std::chrono::milliseconds>(
                          std::chrono::system_clock::now().time_since_epoch()).count();
      ::rename(path.c_str(), (dir + "/" + table + suffix + "." + std::to_string(ms) + ".copy").c_str());
    }
    if (fd[type] < 0) {
      // <table>.columns, shared by the lanes' files: written under a per-lane name and renamed
      // into place (every lane writes the same text, so concurrent renames are harmless)
      const std::string cpath = dir + "/" + table + ".columns";
      const std::string tpath = cpath + suffix + ".tmp";
      const int cf = ::open(tpath.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
      if (cf >= 0) {
        const std::string c = columns + "\n";
        const bool ok = write_all(cf, c.data(), c.size());
        ::close(cf);
        if (!ok || ::rename(tpath.c_str(), cpath.c_str()) != 0) ::unlink(tpath.c_str());
      }
      // not O_APPEND: pwrite on an O_APPEND fd ignores its offset on Linux (write_run)
      fd[type] = ::open(path.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
      if (fd[type] < 0) return "cannot open " + path + ": " + std::strerror(errno);
      struct stat st;
      size[type] = ::fstat(fd[type], &st) == 0 ? (uint64_t)st.st_size : 0;
    }
    if (rows.empty()) return "";
    if (::lseek(fd[type], (off_t)size[type], SEEK_SET) < 0 || !write_all(fd[type], rows.data(), rows.size()))
      return std::string("spool write failed: ") + std::strerror(errno);
    size[type] += rows.size();
    return "";
  }
  // A run of flushes: one writev per run (tmpfs serialises writers on the inode, so copying a
  // run on several threads measured slower: 174-191 ms vs 115 ms for 0.5 GB).
  size_t write_run(int type, const std::string& table, const std::string& columns,
                   const std::vector<std::string_view>& rows, std::string& err) override {
    err = write(type, table, columns, std::string());  // rotation / open, no bytes
    if (!err.empty()) return 0;
    size_t done = 0;
    while (done < rows.size()) {
      struct iovec iov[64];
      int k = 0;
      size_t bytes = 0;
      for (size_t i = done; i < rows.size() && k < 64; ++i, ++k) {
        iov[k].iov_base = const_cast<char*>(rows[i].data());
        iov[k].iov_len = rows[i].size();
        bytes += rows[i].size();
      }
      if (::lseek(fd[type], (off_t)size[type], SEEK_SET) < 0) { err = std::strerror(errno); return done; }
      size_t left = bytes;
      int first = 0;
      while (left) {
        const ssize_t w = ::writev(fd[type], iov + first, k - first);
        if (w < 0) {
          if (errno == EINTR) continue;
          err = std::string("spool write failed: ") + std::strerror(errno);
          if (::ftruncate(fd[type], (off_t)size[type]) != 0) err += " (and the truncate back failed)";
          return done;
        }
        left -= (size_t)w;
        size_t adv = (size_t)w;
        while (first < k && adv >= iov[first].iov_len) { adv -= iov[first].iov_len; ++first; }
        if (first < k && adv) {
          iov[first].iov_base = (char*)iov[first].iov_base + adv;
          iov[first].iov_len -= adv;
        }
      }
      size[type] += bytes;
      done += (size_t)k;
    }
    return done;
  }
};

// One long-lived psql process: every flush is `COPY t (cols) FROM STDIN;` + rows + `\.`, then
// `\echo APMACK <seq> :ERROR` -- psql prints `APMACK <seq> false` when the COPY committed.  A
// dead process is restarted by the next flush (that flush fails and is re-buffered).
struct PsqlWriter : Writer {
  std::vector<std::string> argv;
  pid_t pid = -1;
  int in = -1, out = -1;
  uint64_t seq = 0;
  std::string rbuf;
  double timeout_ms;
  explicit PsqlWriter(std::vector<std::string> a, double t) : argv(std::move(a)), timeout_ms(t) {}
  ~PsqlWriter() override { stop(); }
  void stop() {
    if (in >= 0) { ::close(in); in = -1; }
    if (out >= 0) { ::close(out); out = -1; }
    if (pid > 0) {
      int st = 0;
      for (int i = 0; i < 50 && ::waitpid(pid, &st, WNOHANG) == 0; ++i) ::usleep(20000);
      if (::waitpid(pid, &st, WNOHANG) == 0) { ::kill(pid, SIGTERM); ::waitpid(pid, &st, 0); }
      pid = -1;
    }
    rbuf.clear();
  }
  std::string start() {
    int pin[2], pout[2];
    if (::pipe2(pin, O_CLOEXEC) != 0 || ::pipe2(pout, O_CLOEXEC) != 0) return "pipe failed";
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_adddup2(&fa, pin[0], 0);
    posix_spawn_file_actions_adddup2(&fa, pout[1], 1);
    std::vector<char*> av;
    for (auto& s : argv) av.push_back(const_cast<char*>(s.c_str()));
    av.push_back(nullptr);
    const int rc = posix_spawnp(&pid, av[0], &fa, nullptr, av.data(), environ);
    posix_spawn_file_actions_destroy(&fa);
    ::close(pin[0]);
    ::close(pout[1]);
    if (rc != 0) {
      ::close(pin[1]);
      ::close(pout[0]);
      pid = -1;
      return std::string("cannot start ") + argv[0] + ": " + std::strerror(rc);
    }
    in = pin[1];
    out = pout[0];
    return "";
  }
  std::string write(int, const std::string& table, const std::string& columns, std::string_view rows) override {
    if (pid < 0) {
      std::string e = start();
      if (!e.empty()) return e;
    }
    const uint64_t s = ++seq;
    std::string head = "COPY " + table + " (" + columns + ") FROM STDIN;\n";
    std::string tail = "\\.\n\\echo APMACK " + std::to_string(s) + " :ERROR\n";
    if (!write_all(in, head.data(), head.size()) || !write_all(in, rows.data(), rows.size()) ||
        !write_all(in, tail.data(), tail.size())) {
      stop();
      return "psql pipe closed";
    }
    const std::string want = "APMACK " + std::to_string(s) + " ";
    const double t_end = mono_ms() + timeout_ms;
    for (;;) {
      size_t nl;
      while ((nl = rbuf.find('\n')) != std::string::npos) {
        std::string line = rbuf.substr(0, nl);
        rbuf.erase(0, nl + 1);
        if (line.compare(0, want.size(), want) == 0) {
          const std::string v = line.substr(want.size());
          return v == "false" ? "" : "COPY into " + table + " failed (psql :ERROR=" + v + ")";
        }
      }
      const double left = t_end - mono_ms();
      // the whole COPY (with its terminator) was sent: it may have committed.  A retry could
      // duplicate every row, so the outcome is reported as unknown ('?') and not retried.
      if (left <= 0) {
        stop();
        return "?psql did not acknowledge the COPY into " + table + " within " + std::to_string((int)(timeout_ms / 1000)) +
               " s: outcome unknown, not retried (would risk duplicate rows)";
      }
      struct pollfd p{out, POLLIN, 0};
      if (::poll(&p, 1, (int)left) <= 0) continue;
      char b[4096];
      const ssize_t r = ::read(out, b, sizeof b);
      if (r <= 0) { stop(); return "?psql exited before acknowledging the COPY into " + table + ": outcome unknown, not retried"; }
      rbuf.append(b, (size_t)r);
    }
  }
};

}  // namespace

class DbSink : public ByteSink {
  struct Job;

 public:
  DbSink(int64_t limit, double max_wait_ms, std::vector<std::string> tables, std::vector<std::string> columns,
         const std::string& writer, const std::vector<std::string>& arg, uint64_t rotate_bytes, int encoders,
         int lanes = 1, double ack_timeout_ms = 120000.0)
      : limit_(std::max<int64_t>(1, limit)), max_wait_ms_(max_wait_ms), tables_(std::move(tables)),
        columns_(std::move(columns)), lanes_(std::max(1, std::min(lanes, 64))), order_((size_t)lanes_) {
    if (tables_.size() != NT || columns_.size() != NT) throw std::runtime_error("DbSink: 5 tables / column lists");
    // Writer lanes: `lanes` independent writers (own spool files / own psql connection), each
    // writing its share of the flushes in submission order -- the reference's pg Pool likewise
    // keeps several INSERTs in flight (stream_insert_db.js:277-327).
    for (int l = 0; l < lanes_; ++l) {
      if (writer == "null") w_.emplace_back(new NullWriter());
      else if (writer == "spool") w_.emplace_back(new SpoolWriter(arg.at(0), rotate_bytes, l ? ".lane" + std::to_string(l) : ""));
      else if (writer == "psql") w_.emplace_back(new PsqlWriter(arg, ack_timeout_ms));
      else throw std::runtime_error("DbSink: unknown writer " + writer);
    }
    for (int i = 0; i < std::max(1, encoders); ++i) enc_.emplace_back([this] { encode_loop(); });
    for (int l = 0; l < lanes_; ++l) wr_.emplace_back([this, l] { write_loop(l); });
  }
  ~DbSink() override { shutdown(); }

  // engine output lane -> sink (Engine::set_byte_sink)
  void write_bytes(int, const char* p, size_t n) override { consume(std::string_view(p, n)); }

  // Splits a newline-separated blob of wire lines into the type buffers (runs of one type are
  // appended with one copy); returns accepted lines.
  int64_t consume(std::string_view blob) {
    const double now = mono_ms();
    int64_t n = 0;
    std::lock_guard<std::mutex> lk(mu_);
    size_t i = 0;
    int run_t = -1;
    size_t run_b = 0;
    int64_t run_n = 0;
    auto close_run = [&](size_t end) {
      if (run_t >= 0 && run_n) append_run_locked(run_t, blob.data() + run_b, end - run_b, run_n, now, false);
      run_t = -1;
      run_n = 0;
    };
    while (i < blob.size()) {
      const char* q = (const char*)std::memchr(blob.data() + i, '\n', blob.size() - i);
      const size_t j = q ? (size_t)(q - blob.data()) : blob.size();
      if (j > i) {
        const int t = type_of(blob.substr(i, j - i));
        if (t != run_t || buf_[t < 0 ? 0 : t].n + run_n >= limit_) close_run(i);
        if (t < 0) {
          ++not_db_;
        } else {
          if (run_t < 0) { run_t = t; run_b = i; }
          ++run_n;
          ++n;
        }
      } else {
        close_run(i);
      }
      i = j + 1;
    }
    close_run(std::min(i, blob.size()));
    return n;
  }

  // Rows already in COPY text for `type` (the engine's fs stream in COPY mode): buffered and
  // flushed with the same limit / timer rules, written without encoding.  A rollover's fs rows
  // (tens of MB) are cut at the flush limit and copied into their flush jobs by several threads;
  // the resulting buffers and jobs are exactly those of the serial path.
  int64_t consume_encoded(int type, std::string_view blob, std::shared_ptr<const void> hold = nullptr) {
    if (blob.size() >= kParallelBytes && blob.size() < (1ull << 32))
      return consume_encoded_parallel(type, blob, std::move(hold));
    const double now = mono_ms();
    std::lock_guard<std::mutex> lk(mu_);
    encoded_[type] = true;
    if (buf_[type].n > 0 && !buf_[type].enc) submit_locked(type);
    int64_t n = 0;
    size_t i = 0;
    while (i < blob.size()) {
      // the rows that fit the buffer before its limit
      const int64_t room = std::max<int64_t>(1, limit_ - buf_[type].n);
      size_t j = i;
      int64_t k = 0;
      while (k < room && j < blob.size()) {
        const char* q = (const char*)std::memchr(blob.data() + j, '\n', blob.size() - j);
        j = q ? (size_t)(q - blob.data()) + 1 : blob.size();
        ++k;
      }
      append_run_locked(type, blob.data() + i, j - i, k, now, true);
      n += k;
      i = j;
    }
    return n;
  }

  static constexpr size_t kParallelBytes = 4u << 20;
  static constexpr size_t kSpares = 256;

  // Flush buffers are recycled: a rollover's COPY rows are tens of MB in ~250 KB flushes, and
  // fresh allocations of that size are mmap'd and page-faulted in on every batch.
  std::string take_spare_locked() {
    if (spare_.empty()) return std::string();
    std::string s = std::move(spare_.back());
    spare_.pop_back();
    s.clear();
    return s;
  }
  void give_spare_locked(std::string&& s) {
    if (spare_.size() < kSpares && s.capacity() >= (64u << 10)) spare_.push_back(std::move(s));
  }

  // A few long-lived helper threads for the row scan of large COPY blobs (spawning 2 x 8 threads
  // per hand-off cost ~0.5 ms of the output lane per batch).  One run at a time; the caller works too.
  struct Helpers {
    std::mutex run_mu, mu;
    std::condition_variable cv, done_cv;
    std::vector<std::thread> th;
    const std::function<void(int)>* fn = nullptr;
    int n = 0, next = 0, finished = 0;
    uint64_t gen = 0;
    bool stop = false;
    void take_and_run() {  // (mu held on entry and exit)
      while (next < n) {
        const int i = next++;
        const std::function<void(int)>* f = fn;
        mu.unlock();
        (*f)(i);
        mu.lock();
        if (++finished == n) done_cv.notify_all();
      }
    }
    void loop() {
      std::unique_lock<std::mutex> lk(mu);
      uint64_t seen = 0;
      for (;;) {
        cv.wait(lk, [&] { return stop || gen != seen; });
        if (stop) return;
        seen = gen;
        take_and_run();
      }
    }
    void run(int count, const std::function<void(int)>& f) {
      std::lock_guard<std::mutex> rg(run_mu);
      std::unique_lock<std::mutex> lk(mu);
      if (th.empty())
        for (int i = 0; i < 7; ++i) th.emplace_back([this] { loop(); });
      fn = &f;
      n = count;
      next = 0;
      finished = 0;
      ++gen;
      cv.notify_all();
      take_and_run();
      done_cv.wait(lk, [&] { return finished == n; });
      fn = nullptr;
    }
    ~Helpers() {
      {
        std::lock_guard<std::mutex> lk(mu);
        stop = true;
      }
      cv.notify_all();
      for (auto& t : th) t.join();
    }
  };
  Helpers helpers_;
  template <class F>
  void parallel_for(int n, const F& fn) {
    const std::function<void(int)> f = [&fn](int i) { fn(i); };
    helpers_.run(n, f);
  }

  // With `hold` (the caller's buffer stays valid until released) the middle flushes reference the
  // blob instead of copying it: a firehose rollover hands ~80 MB of COPY rows per batch, and the
  // copy into flush strings was most of the output lane's time.
  int64_t consume_encoded_parallel(int type, std::string_view blob, std::shared_ptr<const void> hold = nullptr) {
    const double now = mono_ms();
    const char* d = blob.data();
    const size_t size = blob.size();
    const int P = (int)std::max<size_t>(2, std::min<size_t>(8, size >> 20));
    // parts start at line starts
    std::vector<size_t> b(P + 1, size);
    b[0] = 0;
    for (int p = 1; p < P; ++p) {
      const size_t x = std::max(b[p - 1], size * (size_t)p / (size_t)P);
      const char* q = x < size ? (const char*)std::memchr(d + x, '\n', size - x) : nullptr;
      b[p] = q ? (size_t)(q - d) + 1 : size;
    }
    // one pass per part: the end offset of every row (a row is a line; an unterminated tail
    // counts as one, as on the serial path)
    std::vector<std::vector<uint32_t>> ends(P);
    parallel_for(P, [&](int p) {
      std::vector<uint32_t>& e = ends[p];
      e.reserve((b[p + 1] - b[p]) / 128 + 16);
      size_t i = b[p];
      while (i < b[p + 1]) {
        const char* q = (const char*)std::memchr(d + i, '\n', b[p + 1] - i);
        i = q ? (size_t)(q - d) + 1 : b[p + 1];
        e.push_back((uint32_t)(i - b[p]));
      }
    });
    std::vector<int64_t> r0(P + 1, 0);
    for (int p = 0; p < P; ++p) r0[p + 1] = r0[p] + (int64_t)ends[p].size();
    const int64_t total = r0[P];
    if (total == 0) return 0;
    // the blob offset where each cut (a row count from the blob start) ends
    int pi = 0;
    auto end_of = [&](int64_t c) {
      while (c > r0[pi + 1]) ++pi;
      return b[pi] + ends[pi][(size_t)(c - r0[pi] - 1)];
    };
    return cut_and_submit(type, d, total, end_of, hold, now, P);
  }

  // Rows whose boundaries the producer already knows (the engine's fs COPY rows: K12's exclusive
  // scan of the row lengths): row r is [row_off[r], row_off[r + 1]) of the blob, empty rows are
  // skipped.  No scan of the text -- the flushes are exactly those of consume_encoded.
  int64_t consume_encoded_rows(int type, std::string_view blob, const uint32_t* row_off, size_t nrows,
                               std::shared_ptr<const void> hold = nullptr) {
    if (blob.size() >= (1ull << 32) || nrows == 0 || row_off[nrows] != blob.size() || row_off[0] != 0)
      return consume_encoded(type, blob, std::move(hold));
    const double now = mono_ms();
    std::vector<uint32_t> ends;
    ends.reserve(nrows);
    for (size_t r = 0; r < nrows; ++r)
      if (row_off[r + 1] > row_off[r]) ends.push_back(row_off[r + 1]);
    const int64_t total = (int64_t)ends.size();
    if (total == 0) return 0;
    auto end_of = [&](int64_t c) { return (size_t)ends[(size_t)c - 1]; };
    return cut_and_submit(type, blob.data(), total, end_of, hold, now,
                          (int)std::max<size_t>(2, std::min<size_t>(8, blob.size() >> 20)));
  }

  // `total` rows starting at d; end_of(c) = blob offset where the first c rows end (c ascending).
  template <class EndOf>
  int64_t cut_and_submit(int type, const char* d, int64_t total, EndOf& end_of,
                         const std::shared_ptr<const void>& hold, double now, int P) {
    std::lock_guard<std::mutex> lk(mu_);
    encoded_[type] = true;
    if (buf_[type].n > 0 && !buf_[type].enc) submit_locked(type);
    // a full buffer is flushed before anything is added (as append_run_locked does); then the
    // serial path's flushes hold `limit` consecutive rows each: A0 tops the buffer up to the
    // limit, every later flush is `limit` rows of the blob, the remainder stays buffered
    if (buf_[type].n >= limit_) submit_locked(type);
    const int64_t room = limit_ - buf_[type].n;
    std::vector<int64_t> cut;  // row index (from the blob start) where each append ends
    for (int64_t c = std::min(room, total); ; c = std::min(c + limit_, total)) {
      cut.push_back(c);
      if (c == total) break;
    }
    std::vector<size_t> off(cut.size());
    for (size_t k = 0; k < cut.size(); ++k) off[k] = end_of(cut[k]);
    // flushes: [buffer + A0], A1, ..., A(m-1); Am stays buffered
    const size_t m = cut.size() - 1;
    append_run_locked(type, d, off[0], cut[0], now, true);
    if (m == 0) return total;
    submit_locked(type);
    std::vector<std::shared_ptr<Job>> mid(m - 1);
    for (size_t k = 1; k < m; ++k) {
      auto j = std::make_shared<Job>();
      j->type = type;
      j->n = cut[k] - cut[k - 1];
      if (hold) {
        j->ext = std::string_view(d + off[k - 1], off[k] - off[k - 1]);
        j->hold = hold;
      } else {
        j->encoded = take_spare_locked();  // recycled capacity: no page faults, no zero fill
      }
      mid[k - 1] = std::move(j);
    }
    if (!mid.empty()) {
      if (!hold) {
        const int T = (int)std::min<size_t>((size_t)P, mid.size());
        parallel_for(T, [&](int t) {
          for (size_t k = (size_t)t; k < mid.size(); k += (size_t)T)
            mid[k]->encoded.assign(d + off[k], off[k + 1] - off[k]);
        });
      }
      for (auto& j : mid) {
        j->seq = next_seq_++;
        j->ready = true;
        enqueue_locked(j);
      }
      cv_.notify_all();
    }
    append_run_locked(type, d + off[m - 1], off[m] - off[m - 1], cut[m] - cut[m - 1], now, true);
    return total;
  }

  // Rows already in COPY text (e.g. re-loaded from a resume file) queued as one flush.
  void add_encoded(int type, std::string rows, int64_t n) {
    auto j = std::make_shared<Job>();
    j->type = type;
    j->n = n;
    j->encoded = std::move(rows);
    j->ready = true;
    std::lock_guard<std::mutex> lk(mu_);
    j->seq = next_seq_++;
    enqueue_locked(j);
    cv_.notify_all();
  }

  int tick() {
    const double now = mono_ms();
    int k = 0;
    std::lock_guard<std::mutex> lk(mu_);
    for (int t = 0; t < NT; ++t)
      if (buf_[t].n > 0 && now >= buf_[t].deadline) { submit_locked(t); ++k; }
    return k;
  }

  void flush_all() {
    std::lock_guard<std::mutex> lk(mu_);
    for (int t = 0; t < NT; ++t)
      if (buf_[t].n > 0) submit_locked(t);
  }

  // Waits until every submitted flush was written (or failed and re-buffered).
  void drain() {
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return queued_locked() == 0; });
  }

  // Final flush; returns what could not be written, per type, as wire lines (the caller keeps
  // it in the resume file).
  std::vector<std::string> close() {
    flush_all();
    drain();
    shutdown();
    std::vector<std::string> left(NT);
    for (int t = 0; t < NT; ++t) left[t] = buf_[t].lines;
    return left;
  }

  py::dict stats() {
    std::lock_guard<std::mutex> lk(mu_);
    py::dict d;
    d["rows"] = rows_;
    d["ms"] = ms_;
    d["flushes"] = flushes_;
    d["failures"] = failures_;
    d["queued"] = queued_locked();
    d["lanes"] = lanes_;
    d["not_db_lines"] = not_db_;
    d["bytes"] = bytes_;
    int64_t buffered = 0;
    for (auto& b : buf_) buffered += b.n;
    d["buffered"] = buffered;
    d["last_error"] = last_error_;
    d["doubtful_rows"] = doubtful_rows_;
    d["doubtful_flushes"] = doubtful_flushes_;
    return d;
  }

  // (rows, ms) since the previous call -- DBStats' per-interval line
  std::pair<int64_t, double> take_interval() {
    std::lock_guard<std::mutex> lk(mu_);
    auto r = std::make_pair(rows_ - rows_mark_, ms_ - ms_mark_);
    rows_mark_ = rows_;
    ms_mark_ = ms_;
    return r;
  }

  // the format of what type t's buffer holds (close() returns it as is)
  bool is_encoded(int t) {
    std::lock_guard<std::mutex> lk(mu_);
    return buf_[t].n > 0 ? buf_[t].enc : encoded_[t];
  }

  // ---- checkpoint support: an acknowledged-flush watermark instead of a drain.
  // Every flush gets a sequence number when it is submitted; `acked` = the smallest sequence not
  // yet written (all earlier flushes are in the database / spool).  set_ack_file() makes each
  // writer lane record {incarnation, acked} in a 16-byte file after every write (no fsync: it
  // survives a process crash, like the spool files themselves).  snapshot_pending() submits the
  // partial buffers and copies every flush not yet acknowledged -- without waiting for a writer --
  // so a checkpoint can carry them: on restore, the flushes at or above the file's watermark are
  // submitted again (the ones written after the snapshot were acknowledged in the file).
  struct PendingJob { uint64_t seq; int type; bool encoded; int64_t n; std::string data; };
  void set_ack_file(const std::string& path, uint64_t incarnation) {
    std::lock_guard<std::mutex> lk(mu_);
    if (ack_fd_ >= 0) ::close(ack_fd_);
    ack_fd_ = ::open(path.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC, 0644);
    if (ack_fd_ < 0) throw std::runtime_error("DbSink: cannot open ack file " + path);
    incarnation_ = incarnation;
    write_ack_locked();
  }
  // Rows that failed go back to their buffer and keep their first sequence as a floor (`floor`
  // of the job that carries them next), so the watermark never passes rows not yet written.
  uint64_t acked_locked() const {
    uint64_t a = next_seq_;
    for (auto& kv : live_) a = std::min(a, kv.second->floor);
    for (int t = 0; t < NT; ++t)
      if (buf_[t].n > 0) a = std::min(a, rebuf_floor_[t]);
    return a;
  }
  uint64_t acked() {
    std::lock_guard<std::mutex> lk(mu_);
    return acked_locked();
  }
  std::pair<uint64_t, std::vector<PendingJob>> snapshot_pending() {
    std::lock_guard<std::mutex> lk(mu_);
    for (int t = 0; t < NT; ++t)
      if (buf_[t].n > 0) submit_locked(t);
    std::vector<PendingJob> out;
    out.reserve(live_.size());
    for (auto& kv : live_) {
      const Job& j = *kv.second;
      // (a flush may still be on its way through an encoder: its wire lines are the payload then)
      const bool enc = j.ready;
      out.push_back(PendingJob{j.seq, j.type, enc, j.n, std::string(enc ? j.data() : std::string_view(j.lines))});
    }
    return {acked_locked(), std::move(out)};
  }

  // Asynchronous form of snapshot_pending for the checkpoint writer: the capture (ingest thread,
  // sink lock held for microseconds) takes references to the unacknowledged flushes instead of
  // copying them; snapshot_write (the engine's checkpoint writer thread) writes them to `path`
  // -- the layout runtime/sinks.py write_sink_snapshot uses -- fsyncs, renames, and releases the
  // references.  Until then the writer lanes keep those flushes' buffers (zero-copy engine
  // buffers stay held).
  struct Snapshot {
    uint64_t acked = 0;
    int64_t rows = 0;
    std::vector<std::shared_ptr<Job>> jobs;
    std::vector<uint8_t> enc;
    bool released = false;
  };
  std::shared_ptr<Snapshot> snapshot_capture() {
    auto snap = std::make_shared<Snapshot>();
    std::lock_guard<std::mutex> lk(mu_);
    for (int t = 0; t < NT; ++t)
      if (buf_[t].n > 0) submit_locked(t);
    snap->jobs.reserve(live_.size());
    for (auto& kv : live_) {
      const std::shared_ptr<Job>& j = kv.second;
      ++j->snap_refs;
      snap->jobs.push_back(j);
      snap->enc.push_back(j->ready ? 1 : 0);  // (a flush still in an encoder: its wire lines)
      snap->rows += j->n;
    }
    snap->acked = acked_locked();
    return snap;
  }
  void snapshot_release(Snapshot& snap) {
    std::lock_guard<std::mutex> lk(mu_);
    if (snap.released) return;
    snap.released = true;
    for (auto& j : snap.jobs)
      if (--j->snap_refs == 0 && j->written) release_job_locked(*j);
  }
  void snapshot_write(Snapshot& snap, const std::string& path) {
    const std::string tmp = path + ".tmp";
    const int fd = ::open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) { snapshot_release(snap); throw std::runtime_error("sink snapshot: cannot create " + tmp); }
    std::string head;
    auto put = [&head](const void* p, size_t n) { head.append((const char*)p, n); };
    bool ok = true;
    auto flush_head = [&]() {
      if (!head.empty() && !write_all(fd, head.data(), head.size())) ok = false;
      head.clear();
    };
    const uint64_t count = snap.jobs.size();
    put("APMSINK1", 8);
    put(&count, 8);
    for (size_t k = 0; k < snap.jobs.size() && ok; ++k) {
      const Job& j = *snap.jobs[k];
      // (read without the lock: snap_refs keeps the writer lanes and encoders off these fields)
      const std::string_view d = snap.enc[k] ? j.data() : std::string_view(j.lines);
      const uint64_t seq = j.seq, len = d.size();
      const uint32_t ti = (uint32_t)j.type;
      const uint8_t e = snap.enc[k];
      const int64_t rows = j.n;
      put(&seq, 8); put(&ti, 4); put(&e, 1); put(&rows, 8); put(&len, 8);  // struct "<QIBqQ"
      if (len >= (1u << 16)) {
        flush_head();
        if (ok && !write_all(fd, d.data(), d.size())) ok = false;
      } else {
        head.append(d.data(), d.size());
        if (head.size() >= (4u << 20)) flush_head();
      }
    }
    flush_head();
    snapshot_release(snap);
    if (!ok || ::fdatasync(fd) != 0) {
      ::close(fd);
      throw std::runtime_error("sink snapshot: write failed: " + tmp);
    }
    ::close(fd);
    if (std::rename(tmp.c_str(), path.c_str()) != 0) throw std::runtime_error("sink snapshot: rename failed: " + path);
  }

  void set_limit(int64_t limit, double max_wait_ms) {
    std::lock_guard<std::mutex> lk(mu_);
    limit_ = std::max<int64_t>(1, limit);
    max_wait_ms_ = max_wait_ms;
  }

 private:
  struct Buf {
    std::string lines;
    int64_t n = 0;
    double deadline = 0;
    bool enc = false;  // lines are COPY rows (else wire lines, encoded at submit)
  };
  struct Job {
    int type = 0;
    int64_t n = 0;
    uint64_t seq = 0;
    std::string lines, encoded;
    // zero-copy flush: COPY rows in the caller's (engine's pinned) buffer, kept alive and unchanged
    // until `hold` is released (the engine reuses the buffer only then)
    std::string_view ext;
    std::shared_ptr<const void> hold;
    uint64_t floor = UINT64_MAX;  // smallest sequence whose rows this flush carries (re-buffered rows)
    bool taken = false, ready = false;
    // a checkpoint snapshot is writing this flush's rows (snapshot_capture .. snapshot_write):
    // the writer lane leaves its buffers alone and `written` defers their release
    int snap_refs = 0;
    bool written = false;
    std::string_view data() const { return ext.data() ? ext : std::string_view(encoded); }
  };

  // Appends `nrows` complete lines of type t (COPY rows if enc, else wire lines); the buffer is
  // flushed first when it is full or holds the other format (one table may get engine-encoded
  // rows from one stream and wire lines from another: the db and audit_db streams).
  void append_run_locked(int t, const char* p, size_t len, int64_t nrows, double now, bool enc) {
    Buf& b = buf_[t];
    if (b.n >= limit_ || (b.n > 0 && b.enc != enc)) submit_locked(t);
    if (b.n == 0) { b.deadline = now + max_wait_ms_; b.enc = enc; }
    b.lines.append(p, len);
    if (len && p[len - 1] != '\n') b.lines += '\n';
    b.n += nrows;
  }

  void submit_locked(int t) {
    auto j = std::make_shared<Job>();
    j->type = t;
    j->n = buf_[t].n;
    j->seq = next_seq_++;
    j->floor = std::min(j->seq, rebuf_floor_[t]);
    rebuf_floor_[t] = UINT64_MAX;
    if (buf_[t].enc) {  // COPY text already: straight to the writer
      j->encoded.swap(buf_[t].lines);
      j->ready = true;
    } else {
      j->lines.swap(buf_[t].lines);
      to_encode_.push_back(j);
    }
    buf_[t].lines = take_spare_locked();
    buf_[t].n = 0;
    enqueue_locked(j);
    cv_.notify_all();
  }

  void release_job_locked(Job& j) {
    give_spare_locked(std::move(j.encoded));
    give_spare_locked(std::move(j.lines));
    j.ext = std::string_view();
    j.hold.reset();
  }
  static bool write_all(int fd, const char* p, size_t n) {
    while (n) {
      const ssize_t w = ::write(fd, p, n);
      if (w < 0) {
        if (errno == EINTR) continue;
        return false;
      }
      p += w;
      n -= (size_t)w;
    }
    return true;
  }

  // A flush goes to the next writer lane; lanes take their jobs in order.  Round robin over
  // blocks of kLaneBlock flushes, so a lane still sees runs of one type to write with one writev.
  static constexpr uint64_t kLaneBlock = 16;
  void enqueue_locked(const std::shared_ptr<Job>& j) {
    order_[(size_t)((rr_++ / kLaneBlock) % (uint64_t)lanes_)].push_back(j);
    if (j->floor == UINT64_MAX) j->floor = j->seq;
    live_[j->seq] = j;
  }
  void write_ack_locked() {
    if (ack_fd_ < 0) return;
    const uint64_t v[2] = {incarnation_, acked_locked()};
    if (::pwrite(ack_fd_, v, sizeof v, 0) != (ssize_t)sizeof v) last_error_ = "ack file write failed";
  }
  int64_t queued_locked() const {
    int64_t q = 0;
    for (auto& o : order_) q += (int64_t)o.size();
    return q;
  }

  void encode_loop() {
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !to_encode_.empty(); });
        if (to_encode_.empty()) return;  // stop_ and nothing left
        j = to_encode_.front();
        to_encode_.pop_front();
      }
      std::string out[NT];
      int64_t counts[NT] = {0, 0, 0, 0, 0};
      copyenc::encode_blob(j->lines, out, counts);
      {
        std::lock_guard<std::mutex> lk(mu_);
        j->encoded.swap(out[j->type]);
        j->ready = true;
      }
      cv_.notify_all();
    }
  }

  void write_loop(int lane) {
    std::deque<std::shared_ptr<Job>>& order = order_[(size_t)lane];
    Writer& w = *w_[(size_t)lane];
    for (;;) {
      std::vector<std::shared_ptr<Job>> run;  // consecutive ready flushes of one type
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return (!order.empty() && order.front()->ready) || (stop_ && order.empty()); });
        if (order.empty()) return;
        const int t = order.front()->type;
        for (size_t i = 0; i < order.size() && i < 256 && order[i]->ready && order[i]->type == t; ++i)
          run.push_back(order[i]);
      }
      const int t = run[0]->type;
      std::vector<std::string_view> rows;
      for (auto& j : run) rows.push_back(j->data());
      std::string err;
      const double t0 = mono_ms();
      const size_t ok = w.write_run(t, tables_[t], columns_[t], rows, err);
      const double dt = mono_ms() - t0;
      {
        std::lock_guard<std::mutex> lk(mu_);
        for (size_t i = 0; i < run.size(); ++i) {
          order.pop_front();
          live_.erase(run[i]->seq);  // written, doubtful (not retried) or back in its buffer
        }
        for (size_t i = 0; i < ok; ++i) {
          Job& j = *run[i];
          rows_ += j.n;
          bytes_ += (int64_t)j.data().size();
          ++flushes_;
          if (j.snap_refs) { j.written = true; continue; }  // released by snapshot_write
          release_job_locked(j);
        }
        ms_ = std::max(ms_, lane_ms_[lane] += dt);  // wall time of the busiest lane
        if (ok < run.size()) {
          failures_ += (int64_t)(run.size() - ok);
          last_error_ = err;
          size_t retry_from = ok;
          if (!err.empty() && err[0] == '?') {  // outcome unknown: that flush is not retried
            doubtful_rows_ += run[ok]->n;
            ++doubtful_flushes_;
            retry_from = ok + 1;
          }
          // back to the front of its buffer, in order (:310-320)
          // (wire lines stay wire lines; if COPY rows are involved -- a flush that came in
          // encoded, or a buffer holding them -- everything goes back as COPY rows: a written
          // flush always has its COPY text)
          Buf& b = buf_[t];
          bool as_copy = b.n > 0 && b.enc;
          for (size_t i = retry_from; i < run.size(); ++i) as_copy |= run[i]->lines.empty();
          std::string back;
          int64_t n = 0;
          for (size_t i = retry_from; i < run.size(); ++i) {
            if (as_copy) back.append(run[i]->data());
            else back += run[i]->lines;
            if (!run[i]->snap_refs) run[i]->hold.reset();
            n += run[i]->n;
            rebuf_floor_[t] = std::min(rebuf_floor_[t], run[i]->floor);
          }
          if (!back.empty()) {
            if (as_copy && b.n > 0 && !b.enc) {  // the buffer's wire lines -> COPY rows
              std::string out[NT];
              int64_t counts[NT] = {0, 0, 0, 0, 0};
              copyenc::encode_blob(b.lines, out, counts);
              b.lines.swap(out[t]);
            }
            if (b.n == 0) b.deadline = mono_ms() + max_wait_ms_;
            b.enc = as_copy;
            b.lines.insert(0, back);
            b.n += n;
          }
        }
        write_ack_locked();
      }
      done_cv_.notify_all();
    }
  }

  void shutdown() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (stop_) return;
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : enc_) t.join();
    for (auto& t : wr_)
      if (t.joinable()) t.join();
    w_.clear();
    if (ack_fd_ >= 0) { ::close(ack_fd_); ack_fd_ = -1; }
  }

  int64_t limit_;
  double max_wait_ms_;
  std::vector<std::string> tables_, columns_;
  int lanes_;
  std::vector<std::unique_ptr<Writer>> w_;  // one per lane
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  Buf buf_[NT];
  bool encoded_[NT] = {false, false, false, false, false};  // type buffered as COPY rows (engine-encoded)
  std::vector<std::deque<std::shared_ptr<Job>>> order_;  // per writer lane, submission order
  std::deque<std::shared_ptr<Job>> to_encode_;
  uint64_t rr_ = 0;
  double lane_ms_[64] = {};
  std::vector<std::string> spare_;
  uint64_t next_seq_ = 0;
  std::map<uint64_t, std::shared_ptr<Job>> live_;  // submitted, not yet written (by sequence)
  uint64_t rebuf_floor_[NT] = {UINT64_MAX, UINT64_MAX, UINT64_MAX, UINT64_MAX, UINT64_MAX};
  int ack_fd_ = -1;
  uint64_t incarnation_ = 0;
  bool stop_ = false;
  std::vector<std::thread> enc_;
  std::vector<std::thread> wr_;
  int64_t rows_ = 0, flushes_ = 0, failures_ = 0, not_db_ = 0, bytes_ = 0, rows_mark_ = 0;
  int64_t doubtful_rows_ = 0, doubtful_flushes_ = 0;  // psql flushes whose commit is unknown (not retried)
  double ms_ = 0, ms_mark_ = 0;
  std::string last_error_;
};

// Engine output stream -> sink, as wire lines or (type >= 0) as COPY rows of that type.
struct SinkRoute : ByteSink {
  std::shared_ptr<DbSink> sink;
  int type;
  SinkRoute(std::shared_ptr<DbSink> s, int t) : sink(std::move(s)), type(t) {}
  void write_bytes(int kind, const char* p, size_t n) override {
    if (type >= 0) sink->consume_encoded(type, std::string_view(p, n));
    else sink->write_bytes(kind, p, n);
  }
  void write_bytes_held(int kind, const char* p, size_t n, std::shared_ptr<const void> hold) override {
    if (type >= 0) sink->consume_encoded(type, std::string_view(p, n), std::move(hold));
    else sink->write_bytes(kind, p, n);
  }
  void write_rows_held(int kind, const char* p, size_t n, const uint32_t* row_off, size_t nrows,
                       std::shared_ptr<const void> hold) override {
    if (type >= 0) sink->consume_encoded_rows(type, std::string_view(p, n), row_off, nrows, std::move(hold));
    else sink->write_bytes(kind, p, n);
  }
};

// A captured sink snapshot held by Python until the engine's checkpoint takes it; releases the
// flushes' references if it is never written (busy checkpoint, failed write).
struct SinkSnapHandle {
  std::shared_ptr<DbSink> sink;
  std::shared_ptr<DbSink::Snapshot> snap;
  ~SinkSnapHandle() {
    if (sink && snap) sink->snapshot_release(*snap);
  }
};

}  // namespace apm

void register_dbsink(py::module_& m) {
  using apm::DbSink;
  using apm::Engine;
  using apm::SinkSnapHandle;
  py::class_<SinkSnapHandle, std::shared_ptr<SinkSnapHandle>>(m, "SinkSnapshot")
      .def_property_readonly("acked", [](const SinkSnapHandle& h) { return h.snap->acked; })
      .def_property_readonly("jobs", [](const SinkSnapHandle& h) { return h.snap->jobs.size(); })
      .def_property_readonly("rows", [](const SinkSnapHandle& h) { return h.snap->rows; })
      .def("write", [](SinkSnapHandle& h, const std::string& path) {
        py::gil_scoped_release rel;  // (synchronous form: tests, the sync checkpoint fallback)
        h.sink->snapshot_write(*h.snap, path);
      });
  m.def("checkpoint_async_sink", [](Engine& e, const std::string& prefix, py::bytes extra, bool force_base,
                                    std::shared_ptr<SinkSnapHandle> h, const std::string& path) {
    // the engine's checkpoint writer writes the sink snapshot after the checkpoint file is
    // durable and before the manifest names it (both or neither become the restore point)
    std::string x = extra;
    py::gil_scoped_release rel;
    return e.checkpoint_async(prefix, x, force_base, [h, path]() { h->sink->snapshot_write(*h->snap, path); });
  }, py::arg("engine"), py::arg("prefix"), py::arg("extra"), py::arg("force_base"), py::arg("snapshot"), py::arg("path"));
  py::class_<DbSink, std::shared_ptr<DbSink>>(m, "DbSink")
      .def(py::init<int64_t, double, std::vector<std::string>, std::vector<std::string>, std::string,
                    std::vector<std::string>, uint64_t, int, int, double>(),
           py::arg("limit"), py::arg("max_wait_ms"), py::arg("tables"), py::arg("columns"), py::arg("writer"),
           py::arg("arg"), py::arg("rotate_bytes") = 1ull << 30, py::arg("encoders") = 2, py::arg("lanes") = 1,
           py::arg("ack_timeout_ms") = 120000.0)
      .def("consume", [](DbSink& s, py::bytes b) {
        std::string_view v = b;
        py::gil_scoped_release rel;
        return s.consume(v);
      })
      .def("add_encoded", [](DbSink& s, int type, py::bytes rows, int64_t n) { s.add_encoded(type, rows, n); })
      .def("tick", &DbSink::tick, py::call_guard<py::gil_scoped_release>())
      .def("flush_all", &DbSink::flush_all, py::call_guard<py::gil_scoped_release>())
      .def("drain", &DbSink::drain, py::call_guard<py::gil_scoped_release>())
      .def("close", [](DbSink& s) {
        std::vector<std::string> left;
        { py::gil_scoped_release rel; left = s.close(); }
        py::list out;
        for (auto& l : left) out.append(py::bytes(l));
        return out;
      })
      .def("stats", &DbSink::stats)
      .def("take_interval", &DbSink::take_interval)
      .def("set_limit", &DbSink::set_limit)
      .def("is_encoded", &DbSink::is_encoded)
      .def("set_ack_file", &DbSink::set_ack_file)
      .def("acked", &DbSink::acked)
      .def("snapshot_capture", [](std::shared_ptr<DbSink> s) {
        auto h = std::make_shared<SinkSnapHandle>();
        h->sink = s;
        {
          py::gil_scoped_release rel;
          h->snap = s->snapshot_capture();
        }
        return h;
      })
      .def("snapshot_pending", [](DbSink& s) {
        std::pair<uint64_t, std::vector<DbSink::PendingJob>> r;
        { py::gil_scoped_release rel; r = s.snapshot_pending(); }
        py::list jobs;
        for (auto& j : r.second) jobs.append(py::make_tuple(j.seq, j.type, j.encoded, j.n, py::bytes(j.data)));
        return py::make_tuple(r.first, jobs);
      })
      .def("consume_encoded", [](DbSink& s, int type, py::bytes b) {
        std::string_view v = b;
        py::gil_scoped_release rel;
        return s.consume_encoded(type, v);
      })
      .def("consume_encoded_rows", [](DbSink& s, int type, py::bytes b, std::vector<uint32_t> off) {
        std::string_view v = b;
        if (off.empty()) throw std::invalid_argument("row offsets: nrows + 1 entries");
        py::gil_scoped_release rel;
        return s.consume_encoded_rows(type, v, off.data(), off.size() - 1);
      })
      .def("consume_encoded_ptr", [](DbSink& s, int type, uintptr_t p, size_t n) {
        py::gil_scoped_release rel;  // rows in caller-owned (e.g. pinned) memory
        return s.consume_encoded(type, std::string_view(reinterpret_cast<const char*>(p), n));
      });
  m.def("attach_sink", [](Engine& e, const std::string& kind, std::shared_ptr<DbSink> s, int encoded_type) {
    py::gil_scoped_release rel;
    e.set_byte_sink(kind, std::make_shared<apm::SinkRoute>(std::move(s), encoded_type));
  }, py::arg("engine"), py::arg("kind"), py::arg("sink"), py::arg("encoded_type") = -1);
  m.def("detach_sink", [](Engine& e, const std::string& kind) {
    py::gil_scoped_release rel;
    e.set_byte_sink(kind, nullptr);
  }, py::arg("engine"), py::arg("kind"));
}
