// Randomised equivalence checks for the JS string helpers the join relies on (jsutil.h):
// js::trim (ASCII fast path for the right trim) against the exact code-point walk over random
// mixes of ASCII, JS Unicode whitespace and broken UTF-8.  Exit 0 = equal on every input.
#include "runtime/jsutil.h"

#include <cstdio>
#include <random>
#include <string>

using namespace apm::js;

static std::string_view trim_walk(std::string_view s) {
  const uint8_t* p = (const uint8_t*)s.data();
  const uint8_t* e = p + s.size();
  while (p < e) { int w = ws_len(p, e); if (!w) break; p += w; }
  const uint8_t* q = p;
  const uint8_t* last = p;
  while (q < e) { int w = ws_len(q, e); if (w) q += w; else { ++q; last = q; } }
  return std::string_view((const char*)p, last - p);
}

int main(int argc, char** argv) {
  const long iters = argc > 1 ? std::atol(argv[1]) : 1000000;
  std::mt19937 rng(1);
  static const char* pieces[] = {" ", "\t", "\n", "\r", "\v", "a", "x", "9", "<", "\xC2\xA0", "\xE2\x80\x80",
                                 "\xE2\x80\xAF", "\xEF\xBB\xBF", "\xE3\x80\x80", "\xE1\x9A\x80", "\xC2", "\xE2\x80",
                                 "\xA0", "\xBF"};
  const int np = sizeof(pieces) / sizeof(pieces[0]);
  for (long it = 0; it < iters; ++it) {
    std::string s;
    const int n = (int)(rng() % 9);
    for (int i = 0; i < n; ++i) s += pieces[rng() % np];
    const std::string_view a = trim(s), b = trim_walk(s);
    if (a.data() != b.data() || a.size() != b.size()) {
      std::printf("trim mismatch at iteration %ld (len %zu)\n", it, s.size());
      return 1;
    }
  }
  std::printf("ok %ld\n", iters);
  return 0;
}
