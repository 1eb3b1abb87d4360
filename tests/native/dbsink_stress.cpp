// DbSink under the sanitizers: producers feeding pre-encoded COPY rows of two types (rollover-
// sized blobs through the parallel cutter, small ones through the serial path) while another
// thread ticks and flushes, with the encoder pool and the ordered spool writer running.  Every
// row must reach its spool file exactly once and in order.  The class is compiled from its
// source; its Python bindings are linked but never called.
#include "runtime/dbsink.cpp"

#include <atomic>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <thread>

namespace {

std::string rows(int type, int64_t lo, int64_t n, int pad) {
  std::string s;
  s.reserve((size_t)n * (size_t)(pad + 24));
  for (int64_t i = lo; i < lo + n; ++i) {
    s += std::to_string(type);
    s += '\t';
    s += std::to_string(i);
    s += '\t';
    s.append((size_t)(pad + (int)(i % 97)), 'x');
    s += '\n';
  }
  return s;
}

bool check(const std::string& path, int type, int64_t total) {
  std::ifstream f(path);
  std::string line;
  int64_t want = 0;
  while (std::getline(f, line)) {
    std::istringstream is(line);
    int t = -1;
    int64_t i = -1;
    char tab;
    is >> t >> std::noskipws >> tab >> std::skipws >> i;
    if (t != type || i != want) {
      std::printf("%s: row %lld is type %d id %lld\n", path.c_str(), (long long)want, t, (long long)i);
      return false;
    }
    ++want;
  }
  if (want != total) {
    std::printf("%s: %lld rows, want %lld\n", path.c_str(), (long long)want, (long long)total);
    return false;
  }
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string dir = argv[1];
  const std::vector<std::string> tables = {"t_tx", "t_fs", "t_al", "t_jx", "t_fb"};
  const std::vector<std::string> cols = {"a", "b", "c", "d", "e"};
  apm::DbSink sink(1000, 5.0, tables, cols, "spool", {dir}, 1ull << 62, 4);
  const int64_t big = 24000, small = 700;  // rows per blob: ~5 MB (parallel cut) and ~0.1 MB
  std::atomic<bool> done{false};
  int64_t total[2] = {0, 0};
  auto producer = [&](int slot, int type, int rounds) {
    int64_t next = 0;
    for (int r = 0; r < rounds; ++r) {
      const int64_t n = (r % 3 == 0) ? big : small;
      const std::string b = rows(type, next, n, 150);
      sink.consume_encoded(type, b);
      next += n;
    }
    total[slot] = next;
  };
  std::thread ticker([&] {
    int k = 0;
    while (!done.load()) {
      sink.tick();
      if (++k % 16 == 0) sink.flush_all();
      std::this_thread::sleep_for(std::chrono::microseconds(500));
    }
  });
  std::thread p1(producer, 0, 1, 12);
  std::thread p2(producer, 1, 4, 12);
  p1.join();
  p2.join();
  done = true;
  ticker.join();
  const std::vector<std::string> left = sink.close();
  for (const auto& l : left)
    if (!l.empty()) { std::printf("leftover rows after close\n"); return 1; }
  if (!check(dir + "/t_fs.copy", 1, total[0]) || !check(dir + "/t_fb.copy", 4, total[1])) return 1;
  std::printf("ok %lld %lld\n", (long long)total[0], (long long)total[1]);
  return 0;
}
