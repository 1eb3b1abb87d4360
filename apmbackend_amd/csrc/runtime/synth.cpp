// Native synthetic WildFly log generator (same grammar as apmbackend_amd/utils/synth.py,
// SURVEY Appendix A), used by bench.py to build multi-GB corpora quickly: one generator per JVM
// host, hosts generated in parallel threads, lines kept in per-file min-heaps so every file is
// emitted in timestamp order, output as whole-line chunks ready for Engine::process_batch.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cmath>
#include <cstdint>
#include <cstring>
#include <queue>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace apm {
namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed * 0x9E3779B97F4A7C15ULL + 0x1234567ULL) { next(); }
  uint64_t next() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  int range(int lo, int hi) { return lo + (int)(uni() * (hi - lo + 1)); }
  double normal() {
    double u1 = uni(), u2 = uni();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
  double expo(double rate) { double u = uni(); if (u < 1e-300) u = 1e-300; return -std::log(u) / rate; }
};

void days_to_civil(int64_t z, int& y, unsigned& m, unsigned& d) {
  z += 719468;
  const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
  const unsigned doe = (unsigned)(z - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const int64_t yy = (int64_t)yoe + era * 400;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp < 10 ? mp + 3 : mp - 9;
  y = (int)(yy + (m <= 2));
}

struct TsCache {
  int64_t sec = INT64_MIN;
  char prefix[24];  // "YYYY-MM-DD HH:MM:SS,"
  void fmt(int64_t ms, std::string& out) {
    const int64_t s = ms >= 0 ? ms / 1000 : (ms - 999) / 1000;
    if (s != sec) {
      sec = s;
      int64_t days = s >= 0 ? s / 86400 : (s - 86399) / 86400;
      int64_t rem = s - days * 86400;
      int y; unsigned mo, d;
      days_to_civil(days, y, mo, d);
      snprintf(prefix, sizeof(prefix), "%04d-%02u-%02u %02d:%02d:%02d,", y, mo, d, (int)(rem / 3600),
               (int)(rem / 60 % 60), (int)(rem % 60));
    }
    out.append(prefix, 20);
    const int msr = (int)(ms - sec * 1000);
    char b[3] = {(char)('0' + msr / 100), (char)('0' + msr / 10 % 10), (char)('0' + msr % 10)};
    out.append(b, 3);
  }
  void iso(int64_t ms, std::string& out) {  // -06:00 offset form used by audit trails
    const int64_t l = ms - 6 * 3600000LL;
    const int64_t s = l >= 0 ? l / 1000 : (l - 999) / 1000;
    int64_t days = s >= 0 ? s / 86400 : (s - 86399) / 86400;
    int64_t rem = s - days * 86400;
    int y; unsigned mo, d;
    days_to_civil(days, y, mo, d);
    char b[48];
    snprintf(b, sizeof(b), "%04d-%02u-%02uT%02d:%02d:%02d.%03d-06:00", y, mo, d, (int)(rem / 3600),
             (int)(rem / 60 % 60), (int)(rem % 60), (int)(l - s * 1000));
    out.append(b);
  }
};

inline void app_int(std::string& o, int64_t v) {
  char b[24];
  int n = 0;
  if (v < 0) { o.push_back('-'); v = -v; }
  do { b[n++] = (char)('0' + v % 10); v /= 10; } while (v);
  while (n) o.push_back(b[--n]);
}

struct Line {
  int64_t ts;
  uint64_t seq;
  std::string text;
  bool operator>(const Line& o) const { return ts != o.ts ? ts > o.ts : seq > o.seq; }
};

struct Params {
  int servers = 8;
  int ejb_services = 6000;
  int provider_services = 4000;
  double tx_per_sec_per_server = 50.0;
  int64_t start_ms = 1578391200000LL;
  int noise_per_tx = 3;
  double riskid = 0.15, baf = 0.3, audit = 0.02, missing = 0.01, late = 0.05, no_acct = 0.01;
  int sub_min = 1, sub_max = 3;
  uint64_t seed = 1;
  int server_offset = 0;  // rank * servers: distinct JVM names per GPU shard
  // planted incident: EJB services getSvc0000 .. getSvc(anomaly_services-1) run anomaly_factor
  // times slower on every JVM from anomaly_start_ms on (the bench's alert rows)
  int anomaly_services = 0;
  double anomaly_factor = 1.0;
  int64_t anomaly_start_ms = INT64_MAX;
  // distinct service pools (BASELINE config 5: 100k services over 256 JVMs): JVM g draws its
  // ejb_services / provider_services names from a window of the pool starting at g * count, so
  // neighbouring JVMs share part of their services and the node holds ejb_pool + provider_pool
  // distinct names.  0 = every JVM uses the same names.
  int ejb_pool = 0;
  int provider_pool = 0;
  // capacity stress (see utils/synth.py): overlapping provider calls, longer logIds
  bool overlap_subs = false;
  int logid_pad = 0;
};

class ServerGen {
 public:
  ServerGen(const Params& p, int idx) : p_(p), idx_(idx), rng_(p.seed * 1000003ULL + idx + 1) {
    char b[32];
    snprintf(b, sizeof(b), "jvm%03d", idx + p.server_offset);
    name_ = b;
    for (char c : name_) upper_.push_back((char)toupper(c));
    next_tx_ = (double)p.start_ms + rng_.expo(p.tx_per_sec_per_server) * 1000.0;
  }
  const std::string& name() const { return name_; }

  // Appends all lines with ts < t1 for file kind k (0 soap, 1 server, 2 app) to `out`.
  void advance(int64_t t1) {
    while (next_tx_ < (double)t1) {
      tx((int64_t)next_tx_);
      next_tx_ += rng_.expo(p_.tx_per_sec_per_server) * 1000.0;
    }
  }
  void drain(int k, int64_t t1, std::string& out) {
    auto& h = heap_[k];
    while (!h.empty() && h.top().ts < t1) {
      out += h.top().text;
      out.push_back('\n');
      h.pop();
    }
  }

 private:
  double base_elapsed(uint64_t svc_hash) {
    Rng r(svc_hash);
    return 60.0 + r.uni() * 840.0;
  }
  int64_t elapsed(double base) { return std::max<int64_t>(1, (int64_t)(base * std::exp(0.25 * rng_.normal()))); }
  void emit(int k, int64_t ts, std::string&& s) { heap_[k].push(Line{ts, seq_++, std::move(s)}); }
  void prefix(std::string& s, const std::string& lid, int64_t ts) {
    s.push_back('['); s += lid; s += "] ";
    tsc_.fmt(ts, s);
    s.push_back(' ');
  }
  void noise(int k, int64_t ts, const std::string& lid) {
    std::string s;
    const uint64_t r = rng_.next();
    if (k == 0) {
      s = "    <ns2:field";
      app_int(s, r % 9); s += ">value"; app_int(s, (r >> 8) % 1000); s += "</ns2:field"; app_int(s, r % 9); s += ">";
    } else {
      prefix(s, lid, ts);
      s += (r & 7) < 5 ? "DEBUG [com.acme.svc.Handler" : "INFO  [com.acme.svc.Handler";
      app_int(s, (r >> 4) % 50);
      s += "] processed step ";
      app_int(s, (int64_t)((r >> 12) % 1000000));
    }
    emit(k, ts, std::move(s));
  }
  void tx(int64_t t0) {
    ++n_;
    std::string log_id = upper_ + "-";
    {
      char b[16];
      snprintf(b, sizeof(b), "%08llu", (unsigned long long)n_);
      log_id += b;
      if (p_.logid_pad > 0) {
        static const char pad[] = "ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789abcdefghijklmnopqrstuvwxyz";
        log_id.push_back('-');
        for (int i = 0; i < p_.logid_pad; ++i) log_id.push_back(pad[i % 62]);
      }
    }
    const bool missing = rng_.uni() < p_.missing;
    const std::string lid = missing ? std::string() : log_id;
    std::string acct;
    app_int(acct, 1000000000000000LL + (int64_t)(rng_.next() % 8999999999999999ULL));
    const int ejb = (int)(rng_.next() % (uint64_t)p_.ejb_services);
    char svc[32];
    if (p_.ejb_pool > 0)
      snprintf(svc, sizeof(svc), "getSvc%05d",
               (int)(((int64_t)(idx_ + p_.server_offset) * p_.ejb_services + ejb) % p_.ejb_pool));
    else
      snprintf(svc, sizeof(svc), "getSvc%04d", ejb);
    int64_t total = elapsed(base_elapsed(0xABCDEFULL + ejb));
    if (ejb < p_.anomaly_services && t0 >= p_.anomaly_start_ms) total = (int64_t)((double)total * p_.anomaly_factor);
    const int64_t t_end = t0 + total;
    const bool late = rng_.uni() < p_.late;
    const bool no_acct = rng_.uni() < p_.no_acct;
    const int64_t soap_t = late ? t_end + rng_.range(50, 15000) : t0;
    { std::string s = "=== jbossId=" + log_id + " IO=I"; emit(0, soap_t, std::move(s)); }
    noise(0, soap_t, log_id);
    if (!no_acct) {
      if (rng_.uni() < p_.riskid) {
        emit(0, soap_t, std::string("      <key>AccountNumber</key>"));
        emit(0, soap_t, "      <value>" + acct + "</value>");
      } else {
        emit(0, soap_t, "      <accountNumber>" + acct + "</accountNumber>");
      }
    }
    { std::string s = "=== jbossId=" + log_id + " IO=O"; emit(0, soap_t + 1, std::move(s)); }
    {
      std::string s;
      prefix(s, lid, t0);
      s += "INFO  [CommonTiming] The EJB call started for bean Delegation method: ";
      s += svc;
      emit(1, t0, std::move(s));
    }
    for (int i = 0; i < p_.noise_per_tx; ++i) {
      const int k = (rng_.next() % 3) == 0 ? 1 : 2;
      noise(k, t0 + (int64_t)(rng_.uni() * (double)total), lid);
    }
    const int nsub = rng_.range(p_.sub_min, p_.sub_max);
    const bool audit = !missing && rng_.uni() < p_.audit;
    struct Sub { std::string svc; int64_t s, e, el; };
    std::vector<Sub> subs;
    int64_t cursor = t0 + 1;
    for (int i = 0; i < nsub; ++i) {
      const int pv = (int)(rng_.next() % (uint64_t)p_.provider_services);
      char pn[48];
      if (p_.provider_pool > 0)
        snprintf(pn, sizeof(pn), "Provider[cb-util-%05d]",
                 (int)(((int64_t)(idx_ + p_.server_offset) * p_.provider_services + pv) % p_.provider_pool));
      else
        snprintf(pn, sizeof(pn), "Provider[cb-util-%03d]", pv);
      int64_t el = elapsed(base_elapsed(0x55AA55ULL + pv) * 0.4);
      int64_t s_t, e_t;
      if (p_.overlap_subs) {
        s_t = std::min<int64_t>(t0 + 1 + i, t_end - 1);
        e_t = std::min<int64_t>(std::max<int64_t>(s_t + el, t0 + 1 + nsub), t_end - 1);
      } else {
        s_t = std::min(cursor, t_end - 1);
        e_t = std::min(s_t + el, t_end - 1);
      }
      el = std::max<int64_t>(0, e_t - s_t);
      subs.push_back(Sub{pn, s_t, e_t, el});
      cursor = e_t + 1;
      if (audit) continue;
      const bool baf = rng_.uni() < p_.baf;
      std::string a, b;
      prefix(a, lid, s_t);
      prefix(b, lid, e_t);
      if (baf) { a += "[baf][x:y:" + acct + "] "; b += "[baf][x:y:" + acct + "] "; }
      a += "INFO  CommonTiming::Start: "; a += pn; a += " begin";
      b += "INFO  CommonTiming::Stop: "; b += pn; b += " - total time "; app_int(b, el); b += " ms";
      emit(2, s_t, std::move(a));
      emit(2, e_t, std::move(b));
    }
    if (audit) {
      std::string autr = "A" + log_id;
      std::string s;
      prefix(s, log_id, t0 + 2);
      s += "[baf][x:" + acct + "] INFO  auditTrailId=" + autr;
      emit(2, t0 + 2, std::move(s));
      const int64_t tb = t_end - 1;
      emit(2, tb, "Audit Trail id : " + autr);
      { std::string h; prefix(h, log_id, tb); h += "INFO  com.acme.Audit: RequestTrace [stopWatchList="; emit(2, tb, std::move(h)); }
      const int64_t rules = rng_.range(1, 40);
      for (auto& sb : subs) { std::string e = "  " + sb.svc + ":["; app_int(e, sb.el); e += " millis] ok"; emit(2, tb, std::move(e)); }
      { std::string e = "  RulesEngine:["; app_int(e, rules); e += " millis] ok"; emit(2, tb, std::move(e)); }
      emit(2, tb, std::string("]"));
      emit(2, tb, std::string("<stopWatchList>"));
      for (auto& sb : subs) {
        emit(2, tb, "  <name>" + sb.svc + "</name>");
        std::string a = "  <startTime>"; tsc_.iso(sb.s, a); a += "</startTime>"; emit(2, tb, std::move(a));
        std::string b = "  <stopTime>"; tsc_.iso(sb.e, b); b += "</stopTime>"; emit(2, tb, std::move(b));
      }
      emit(2, tb, std::string("  <name>RulesEngine</name>"));
      { std::string a = "  <startTime>"; tsc_.iso(t0 + 1, a); a += "</startTime>"; emit(2, tb, std::move(a)); }
      { std::string b = "  <stopTime>"; tsc_.iso(t0 + 1 + rules, b); b += "</stopTime>"; emit(2, tb, std::move(b)); }
      emit(2, tb, std::string("</stopWatchList>"));
    }
    {
      std::string s;
      prefix(s, lid, t_end);
      s += "INFO  [CommonTiming] Total time taken for: ";
      s += svc;
      s += " - ";
      app_int(s, total);
      s += " ms";
      emit(1, t_end, std::move(s));
    }
  }

  Params p_;
  int idx_;
  Rng rng_;
  std::string name_, upper_;
  double next_tx_;
  uint64_t n_ = 0, seq_ = 0;
  std::priority_queue<Line, std::vector<Line>, std::greater<Line>> heap_[3];
  TsCache tsc_;
};

class SynthGen {
 public:
  explicit SynthGen(const Params& p) : p_(p) {
    for (int i = 0; i < p.servers; ++i) gens_.emplace_back(new ServerGen(p, i));
  }
  // (path, kind, server) for every file; file id = index
  std::vector<std::tuple<std::string, int, std::string>> files() const {
    std::vector<std::tuple<std::string, int, std::string>> f;
    static const char* names[3] = {"soap_io.log", "server.log", "app.log"};
    for (auto& g : gens_)
      for (int k = 0; k < 3; ++k)
        f.emplace_back("/net/" + g->name() + "/export/jvm1/log/" + names[k], k, g->name());
    return f;
  }
  // Generates all lines with ts < t1 into `out`, appending chunks (file_id, begin, end).
  void generate(int64_t t1, std::string& out, std::vector<std::tuple<int32_t, uint64_t, uint64_t>>& chunks, int threads) {
    const int n = (int)gens_.size();
    std::vector<std::string> parts((size_t)n * 3);
    auto work = [&](int i) {
      gens_[i]->advance(t1);
      for (int k = 0; k < 3; ++k) gens_[i]->drain(k, t1, parts[(size_t)i * 3 + k]);
    };
    if (threads <= 1) {
      for (int i = 0; i < n; ++i) work(i);
    } else {
      std::vector<std::thread> th;
      for (int t = 0; t < threads; ++t)
        th.emplace_back([&, t]() { for (int i = t; i < n; i += threads) work(i); });
      for (auto& x : th) x.join();
    }
    for (int i = 0; i < n * 3; ++i) {
      if (parts[i].empty()) continue;
      const uint64_t b = out.size();
      out += parts[i];
      chunks.emplace_back(i, b, (uint64_t)out.size());
    }
  }

 private:
  Params p_;
  std::vector<std::unique_ptr<ServerGen>> gens_;
};

}  // namespace
}  // namespace apm

void register_synth(py::module_& m) {
  using namespace apm;
  py::class_<SynthGen>(m, "SynthGen")
      .def(py::init([](const py::dict& d) {
        Params p;
        auto g = [&](const char* k, auto& v) { if (d.contains(k)) v = d[k].cast<std::decay_t<decltype(v)>>(); };
        g("servers", p.servers); g("ejb_services", p.ejb_services); g("provider_services", p.provider_services);
        g("tx_per_sec_per_server", p.tx_per_sec_per_server); g("start_ms", p.start_ms);
        g("noise_per_tx", p.noise_per_tx); g("riskid", p.riskid); g("baf", p.baf); g("audit", p.audit);
        g("missing", p.missing); g("late", p.late); g("no_acct", p.no_acct); g("sub_min", p.sub_min);
        g("sub_max", p.sub_max); g("seed", p.seed); g("server_offset", p.server_offset);
        g("anomaly_services", p.anomaly_services); g("anomaly_factor", p.anomaly_factor);
        g("anomaly_start_ms", p.anomaly_start_ms); g("ejb_pool", p.ejb_pool); g("provider_pool", p.provider_pool);
        g("overlap_subs", p.overlap_subs); g("logid_pad", p.logid_pad);
        return new SynthGen(p);
      }))
      .def("files", &SynthGen::files)
      .def("generate", [](SynthGen& s, int64_t t1, int threads) {
        std::string out;
        std::vector<std::tuple<int32_t, uint64_t, uint64_t>> chunks;
        {
          py::gil_scoped_release rel;
          s.generate(t1, out, chunks, threads);
        }
        return std::make_pair(py::bytes(out), chunks);
      }, py::arg("t1"), py::arg("threads") = 8);
}
