// Host test of the checkpoint writer (runtime/binio.h): sections serialised by the in-memory
// writer (MemBlob, in-place fills, patched section lengths) and spliced into a file after the
// header -- the asynchronous checkpoint path -- must be byte-identical to the same sections
// written straight to a file, and read back by BinReader.  Run under ASan/UBSan.
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "runtime/binio.h"

using namespace apm;

static void sections(BinWriter& w, uint32_t seed) {
  std::mt19937 rng(seed);
  for (uint32_t tag = 1; tag <= 6; ++tag) {
    w.begin(tag);
    const size_t n = rng() % 200000;
    std::vector<int32_t> v(n);
    for (auto& x : v) x = (int32_t)rng();
    w.vec(v);
    w.str(std::string(rng() % 5000, (char)('a' + tag)));
    const size_t m = rng() % 300000;
    w.pod<uint64_t>(m);
    w.raw_fill(m, [&](char* dst) { for (size_t i = 0; i < m; ++i) dst[i] = (char)(i * 31 + tag); });
    w.end();
  }
}

static std::string slurp(const std::string& p) {
  FILE* f = std::fopen(p.c_str(), "rb");
  std::string s;
  char buf[1 << 16];
  size_t k;
  while ((k = std::fread(buf, 1, sizeof buf, f)) > 0) s.append(buf, k);
  std::fclose(f);
  return s;
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : ".";
  for (uint32_t seed = 1; seed <= 3; ++seed) {
    const std::string a = dir + "/direct.ckpt", b = dir + "/spliced.ckpt";
    {
      BinWriter w(a);
      sections(w, seed);
      w.commit();
    }
    MemBlob blob;
    {
      BinWriter mw{BinWriter::Memory{}, seed == 2 ? (size_t)1 << 24 : 0};  // with and without a reserve
      sections(mw, seed);
      blob = mw.take_memory();
    }
    MemBlob moved(std::move(blob));  // ownership moves; the source is empty
    if (blob.data() != nullptr || blob.size() != 0) { std::printf("FAIL moved-from blob not empty\n"); return 1; }
    {
      BinWriter w(b);
      w.raw(moved.data(), moved.size());
      w.commit();
    }
    const std::string da = slurp(a), db = slurp(b);
    if (da != db) { std::printf("FAIL seed %u: %zu vs %zu bytes\n", seed, da.size(), db.size()); return 1; }
    BinReader rd(b);
    std::printf("seed %u ok: %zu bytes\n", seed, da.size());
  }
  std::printf("ALL OK\n");
  return 0;
}
