// Wire-format encoders (entries.js toCSVString): st (:71-73), fs (:116-118), al (:214-216).  Numbers go through the JS-exact helpers in jsutil.h.
#pragma once
#include <string>
#include <vector>

#include "../apm_types.h"
#include "join.h"
#include "jsutil.h"

namespace apm {
namespace fmt {

inline const char* cause_text(int i) {
  static const char* t[5] = {"average exceeded hard ms threshold", "per75 exceeded hard ms threshold",
                             "average UB exceeded", "per75 UB exceeded", "average and per75 UB exceeded"};
  return t[i];
}

// tx lines are formatted by the join workers (join.cpp JoinShard::output).

inline std::string st_line(int64_t ts, const std::string& server, const std::string& service, const WinStat& w) {
  std::string s = "st|" + std::to_string(ts) + "|" + server + "|" + service + "|";
  s += js::nf(w.tpm, 2) + "|" + js::nf(w.avg) + "|" + js::nf(w.p75) + "|" + js::nf(w.p95);
  return s;
}

inline std::string fs_line(int64_t ts, const std::string& server, const std::string& service, int lag,
                           const WinStat& w, const ZOut& z) {
  const double x[3] = {w.avg, w.p75, w.p95};
  std::string s = "fs|" + std::to_string(ts) + "|" + server + "|" + service + "|" + std::to_string(lag) + "|";
  s += js::nf(w.tpm, 2);
  for (int k = 0; k < 3; ++k) {
    s += '|';
    s += js::nf(x[k]) + ":" + js::nf(z.mean[k]) + ":" + js::nf(z.lb[k]) + ":" + js::nf(z.ub[k]) + ":";
    // averageSignal is printed raw; the percentile signals go through nf (entries.js:117)
    s += k == 0 ? std::to_string((int)z.sig[k]) : js::nf((double)z.sig[k]);
  }
  return s;
}

inline std::string al_line(double alert_ts, int64_t entry_ts, const std::string& server, const std::string& service,
                           uint32_t causes, const std::string& fs) {
  std::string c;
  for (int i = 0; i < 5; ++i)
    if (causes & (1u << i)) { if (!c.empty()) c += ','; c += cause_text(i); }
  std::string e = fs;
  for (char& ch : e) if (ch == '|') ch = '&';
  return "al|" + js::num_str(alert_ts) + "|" + std::to_string(entry_ts) + "|" + server + "|" + service + "|" + c +
         "|" + e;
}

}  // namespace fmt
}  // namespace apm
