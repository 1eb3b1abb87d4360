// Host-only replay driver for the join workers, built with AddressSanitizer + UBSan by
// tests/test_sanitizers.py (GPU sanitizers are not available; the join is host code).
//
// Input directory:
//   files.txt          one "<path>\t<kind>\t<server>" per file id
//   batch_<i>.meta     "<now_ms>" then one chunk->file id per line
//   batch_<i>.events   raw Event records (parse kernel layout, produced by ops/parse_ref.py)
//   batch_<i>.bytes    the batch bytes the events point into
// Output: the tx lines in the engine's merge order ("<queue>\t<line>").
#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <thread>
#include <string>
#include <unordered_map>
#include <vector>

#include "runtime/join.h"

#ifdef JOIN_REPLAY_HIP
#include <hip/hip_runtime.h>
#endif

using namespace apm;

static std::string slurp(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main(int argc, char** argv) {
  if (argc < 3) { std::fprintf(stderr, "usage: join_replay DIR NBATCHES\n"); return 2; }
  const std::string dir = argv[1];
  const int nb = std::atoi(argv[2]);
  std::vector<FileInfo> files;
  std::vector<std::string> servers;
  std::unordered_map<std::string, int32_t> server_ids;
  {
    std::istringstream in(slurp(dir + "/files.txt"));
    std::string line;
    while (std::getline(in, line)) {
      if (line.empty()) continue;
      const size_t a = line.find('\t'), b = line.find('\t', a + 1);
      const std::string path = line.substr(0, a), srv = line.substr(b + 1);
      const int kind = std::atoi(line.substr(a + 1, b - a - 1).c_str());
      auto it = server_ids.find(srv);
      int32_t sid;
      if (it == server_ids.end()) { sid = (int32_t)servers.size(); servers.push_back(srv); server_ids[srv] = sid; }
      else sid = it->second;
      files.push_back(FileInfo{path, sid, (uint8_t)kind});
    }
  }
  JoinConfig cfg;  // UTC table: n = 0 -> offset 0
  Dictionary dict;
  const bool quiet = std::getenv("JOIN_REPLAY_QUIET") != nullptr;  // timing mode (tools/join_prof.py)
  // JOIN_REPLAY_THREADS=1: every shard of a batch is joined on its own thread, as in the engine
  // (shared Dictionary, concurrent interning) -- the ThreadSanitizer configuration
  const bool threaded = std::getenv("JOIN_REPLAY_THREADS") != nullptr;
  double t_total = 0;
  size_t ev_total = 0;
  std::vector<std::unique_ptr<JoinShard>> shards;
  for (size_t i = 0; i < servers.size(); ++i) shards.emplace_back(new JoinShard(cfg, &dict, &files, &servers));
  for (int b = 0; b < nb; ++b) {
    const std::string pre = dir + "/batch_" + std::to_string(b);
    std::istringstream meta(slurp(pre + ".meta"));
    double now;
    meta >> now;
    std::vector<int32_t> chunk_file;
    int32_t cf;
    while (meta >> cf) chunk_file.push_back(cf);
    const std::string ev_s = slurp(pre + ".events");
    const std::string by_s = slurp(pre + ".bytes");
    const char* ev_p = ev_s.data();
    const char* by_p = by_s.data();
#ifdef JOIN_REPLAY_HIP
    // JOIN_REPLAY_PINNED=1: replay out of hipHostMalloc'd buffers, as the engine does
    static char *pin_ev = nullptr, *pin_by = nullptr;
    if (std::getenv("JOIN_REPLAY_PINNED")) {
      if (!pin_ev) {
        if (hipHostMalloc((void**)&pin_ev, 64 << 20, hipHostMallocDefault) != hipSuccess ||
            hipHostMalloc((void**)&pin_by, 64 << 20, hipHostMallocDefault) != hipSuccess) return 3;
      }
      std::memcpy(pin_ev, ev_s.data(), ev_s.size());
      std::memcpy(pin_by, by_s.data(), by_s.size());
      ev_p = pin_ev;
      by_p = pin_by;
    }
#endif
    const Event* e = reinterpret_cast<const Event*>(ev_p);
    const size_t n = ev_s.size() / sizeof(Event);
    std::vector<TxOut> all;
    for (size_t s = 0; s < shards.size(); ++s) {
      shards[s]->out().clear();
      shards[s]->begin_batch(now, (uint64_t)b);
    }
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::vector<std::pair<size_t, size_t>>> range(shards.size());
    size_t i = 0;
    while (i < n) {
      const int32_t srv = files[chunk_file[e[i].chunk]].server;
      size_t j = i;
      while (j < n && files[chunk_file[e[j].chunk]].server == srv) ++j;
      range[srv].push_back({i, j});
      i = j;
    }
    auto run = [&](size_t s) {
      for (auto& r : range[s]) shards[s]->process(e + r.first, r.second - r.first, (const uint8_t*)by_p, chunk_file);
    };
    if (threaded) {
      std::vector<std::thread> th;
      for (size_t s = 0; s < shards.size(); ++s) th.emplace_back(run, s);
      for (auto& t : th) t.join();
    } else {
      for (size_t s = 0; s < shards.size(); ++s) run(s);
    }
    const double dt = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (quiet) {
      size_t tx = 0;
      for (auto& sh : shards) tx += sh->out().size();
      std::fprintf(stderr, "batch %d: events=%zu tx=%zu join=%.3f ms\n", b, n, tx, dt);
      if (b > 0) { t_total += dt; ev_total += n; }
      continue;
    }
    for (auto& sh : shards)
      for (auto& t : sh->out()) all.push_back(t);
    std::stable_sort(all.begin(), all.end(), [](const TxOut& x, const TxOut& y) { return x.seq < y.seq; });
    for (auto& t : all)
      std::cout << (t.to_db ? "db_insert" : "transactions") << '\t'
                << shards[t.server]->text().substr(t.line_off, t.line_len) << '\n';
  }
  if (quiet && ev_total) std::fprintf(stderr, "steady: %.1f ns/event\n", t_total * 1e6 / ev_total);
  return 0;
}
