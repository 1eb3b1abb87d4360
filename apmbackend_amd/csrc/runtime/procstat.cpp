// Process memory probe: the native replacement of pid_stats.py (ps_mem fork) as used by the
// supervisor (config pidInspectionCommand, apm_manager.js:359-370).  Reads
// /proc/<pid>/smaps_rollup (falling back to /proc/<pid>/smaps) and reports PSS and SwapPss in
// bytes; the CLI (apmbackend_amd/cli/pid_stats.py) prints the reference's quiet format
// "<ram> MiB <swap> MiB" (pid_stats.py:573-583).
#include <pybind11/pybind11.h>

#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>
#include <utility>

namespace py = pybind11;

namespace apm {

std::pair<long long, long long> pid_pss_swap(int pid) {
  long long pss = -1, swap = 0, rss = -1;
  for (const char* name : {"smaps_rollup", "smaps"}) {
    std::ifstream f(std::string("/proc/") + std::to_string(pid) + "/" + name);
    if (!f) continue;
    std::string line;
    long long p = 0, s = 0, r = 0;
    bool any = false;
    while (std::getline(f, line)) {
      long long v;
      if (sscanf(line.c_str(), "Pss: %lld kB", &v) == 1) { p += v; any = true; }
      else if (sscanf(line.c_str(), "SwapPss: %lld kB", &v) == 1) { s += v; }
      else if (sscanf(line.c_str(), "Rss: %lld kB", &v) == 1) { r += v; }
    }
    if (any) { pss = p * 1024; swap = s * 1024; rss = r * 1024; break; }
  }
  if (pss < 0) {  // no smaps access: fall back to statm RSS
    std::ifstream f(std::string("/proc/") + std::to_string(pid) + "/statm");
    long long size = 0, res = 0;
    if (f >> size >> res) pss = res * 4096;
  }
  (void)rss;
  return {pss, swap};
}

}  // namespace apm

void register_procstat(py::module_& m) {
  m.def("pid_pss_swap", &apm::pid_pss_swap, "PSS and SwapPss of a pid in bytes (-1 if unknown)");
}
