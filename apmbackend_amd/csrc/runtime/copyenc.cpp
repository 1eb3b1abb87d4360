// K13: wire records -> Postgres COPY text rows (host, C++).
//
// The reference converts every db_insert message to a row object (entries.js toPostgresObject
// :23-42, :120-151, :218-240, :310-331) and ships them with multi-row INSERTs built by
// pg-promise (stream_insert_db.js:298).  At the fused engine's output rate (one fs row per
// series per LAG every 10 s: ~160k rows per interval per GPU) that per-row object path would
// dominate, so the sink encodes COPY text directly from the wire lines here.  The Python
// definition is runtime/sinks.py (copy_encode_lines); tests/test_sinks.py checks both agree
// byte for byte.
//
// Field rules (as the Python/JS path produces them):
//   timestamps      parseInt -> 'YYYY-MM-DD HH:MM:SS.mmm+00' (UTC), NaN -> \N
//   numbers         parseInt / parseFloat, printed as String(x); NaN/Infinity -> \N (JSON null)
//   strings         COPY-escaped (\\, \t, \n, \r); missing field -> \N
//   fs.lag          kept as the string it was on the wire (JSON: a string)
//   stats / entry   JSON.stringify text (jsonb), dates as toISOString()
#include <cmath>
#include <cstdint>
#include <cstring>
#include <string>
#include <string_view>
#include <vector>

#include "../kernels/common.h"
#include "jsutil.h"

namespace apm {
namespace copyenc {

namespace {

constexpr std::string_view kNull = "\\N";

// JS parseFloat
double parse_float(std::string_view s) {
  const uint8_t* p = (const uint8_t*)s.data();
  const uint8_t* e = p + s.size();
  while (p < e) { int w = js::ws_len(p, e); if (!w) break; p += w; }
  const char* b = (const char*)p;
  const char* q = b;
  const char* end = (const char*)e;
  if (q < end && (*q == '+' || *q == '-')) ++q;
  if ((size_t)(end - q) >= 8 && std::memcmp(q, "Infinity", 8) == 0)
    return *b == '-' ? -INFINITY : INFINITY;
  const char* d0 = q;
  while (q < end && *q >= '0' && *q <= '9') ++q;
  bool digits = q > d0;
  if (q < end && *q == '.') {
    ++q;
    const char* f0 = q;
    while (q < end && *q >= '0' && *q <= '9') ++q;
    digits |= q > f0;
  }
  if (!digits) return js::nan();
  if (q < end && (*q == 'e' || *q == 'E')) {
    const char* x = q + 1;
    if (x < end && (*x == '+' || *x == '-')) ++x;
    const char* x0 = x;
    while (x < end && *x >= '0' && *x <= '9') ++x;
    if (x > x0) q = x;
  }
  return std::strtod(std::string(b, q).c_str(), nullptr);
}

void civil(int64_t days, int& y, unsigned& m, unsigned& d) {
  days += 719468;
  const int64_t era = (days >= 0 ? days : days - 146096) / 146097;
  const unsigned doe = (unsigned)(days - era * 146097);
  const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
  const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
  const unsigned mp = (5 * doy + 2) / 153;
  d = doy - (153 * mp + 2) / 5 + 1;
  m = mp < 10 ? mp + 3 : mp - 9;
  y = (int)(yoe + era * 400) + (m <= 2);
}

// ms since epoch -> "YYYY-MM-DD?HH:MM:SS.mmm" (sep ' ' or 'T')
bool ts_text(double ms, char sep, std::string& out) {
  if (!(ms == ms) || std::isinf(ms) || std::fabs(ms) > 8.64e15) return false;
  const int64_t t = (int64_t)ms;
  int64_t days = t / 86400000, rem = t % 86400000;
  if (rem < 0) { rem += 86400000; --days; }
  int y;
  unsigned mo, d;
  civil(days, y, mo, d);
  char buf[40];
  std::snprintf(buf, sizeof(buf), "%04d-%02u-%02u%c%02d:%02d:%02d.%03d", y, mo, d, sep, (int)(rem / 3600000),
                (int)(rem / 60000 % 60), (int)(rem / 1000 % 60), (int)(rem % 1000));
  out += buf;
  return true;
}

void copy_escape(std::string& out, std::string_view s) {
  for (char c : s) {
    switch (c) {
      case '\\': out += "\\\\"; break;
      case '\t': out += "\\t"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      default: out += c;
    }
  }
}

void json_str(std::string& out, std::string_view s) {
  out += '"';
  for (unsigned char c : s) {
    switch (c) {
      case '"': out += "\\\""; break;
      case '\\': out += "\\\\"; break;
      case '\n': out += "\\n"; break;
      case '\r': out += "\\r"; break;
      case '\t': out += "\\t"; break;
      case '\b': out += "\\b"; break;
      case '\f': out += "\\f"; break;
      default:
        if (c < 0x20) {
          char b[8];
          std::snprintf(b, sizeof(b), "\\u%04x", c);
          out += b;
        } else {
          out += (char)c;
        }
    }
  }
  out += '"';
}

struct Fields {
  std::string_view f[32];
  int n = 0;
  bool has(int i) const { return i < n; }
};

void split(std::string_view s, char d, Fields& o) {
  o.n = 0;
  size_t i = 0;
  for (;;) {
    size_t j = s.find(d, i);
    if (o.n < 32) o.f[o.n++] = s.substr(i, j == std::string_view::npos ? std::string_view::npos : j - i);
    if (j == std::string_view::npos) break;
    i = j + 1;
  }
}

void c_str(std::string& out, const Fields& a, int i) {
  if (a.has(i)) copy_escape(out, a.f[i]); else out += kNull;
}
void c_num(std::string& out, double v) {
  if (v == v && !std::isinf(v)) js::append_num(out, v); else out += kNull;
}
void c_ts(std::string& out, const Fields& a, int i) {
  if (!a.has(i) || !ts_text(js::parse_int(a.f[i]), ' ', out)) { out += kNull; return; }
  out += "+00";
}
void j_num(std::string& out, double v) {
  if (v == v && !std::isinf(v)) js::append_num(out, v); else out += "null";
}

// stats object of FullStatEntry.toPostgresObject (entries.js:120-151)
void fs_stats_json(std::string& out, const Fields& a) {
  static const char* names[3] = {"average", "per75", "per95"};
  static const char* suff[5] = {"", "avg", "lb", "ub", "signal"};
  out += '{';
  for (int k = 0; k < 3; ++k) {
    Fields p;
    if (a.has(6 + k)) split(a.f[6 + k], ':', p);
    for (int j = 0; j < 5; ++j) {
      if (k || j) out += ',';
      out += '"';
      out += names[k];
      out += suff[j];
      out += "\":";
      const double v = !p.has(j) ? js::nan() : (j == 4 ? js::parse_int(p.f[j]) : parse_float(p.f[j]));
      j_num(out, v);
    }
  }
  out += '}';
}

void fs_row_json(std::string& out, const Fields& a) {
  out += "{\"timestamp\":";
  std::string ts;
  if (a.has(1) && ts_text(js::parse_int(a.f[1]), 'T', ts)) { out += '"'; out += ts; out += "Z\""; }
  else out += "null";
  out += ",\"server\":";
  if (a.has(2)) json_str(out, a.f[2]); else out += "null";
  out += ",\"service\":";
  if (a.has(3)) json_str(out, a.f[3]); else out += "null";
  out += ",\"tpm\":";
  j_num(out, a.has(5) ? parse_float(a.f[5]) : js::nan());
  out += ",\"lag\":";
  if (a.has(4)) json_str(out, a.f[4]); else out += "null";
  out += ",\"stats\":";
  fs_stats_json(out, a);
  out += '}';
}

}  // namespace

// Returns the type index (0 tx, 1 fs, 2 al, 3 jx, 4 fb) the row was appended to, or -1.
int encode_line(std::string_view line, std::string* out /*[5]*/) {
  Fields a;
  split(line, '|', a);
  const std::string_view t = a.f[0];
  if (t == "tx") {
    std::string& o = out[0];
    c_ts(o, a, 6); o += '\t';
    c_ts(o, a, 5); o += '\t';
    c_str(o, a, 1); o += '\t';
    c_str(o, a, 2); o += '\t';
    c_str(o, a, 3); o += '\t';
    c_num(o, a.has(4) ? js::parse_int(a.f[4]) : js::nan()); o += '\t';
    c_num(o, a.has(7) ? js::parse_int(a.f[7]) : js::nan()); o += '\t';
    c_str(o, a, 8); o += '\n';
    return 0;
  }
  if (t == "fs") {
    std::string& o = out[1];
    c_ts(o, a, 1); o += '\t';
    c_str(o, a, 2); o += '\t';
    c_str(o, a, 3); o += '\t';
    c_num(o, a.has(5) ? parse_float(a.f[5]) : js::nan()); o += '\t';
    c_str(o, a, 4); o += '\t';
    std::string js;
    fs_stats_json(js, a);
    copy_escape(o, js);
    o += '\n';
    return 1;
  }
  if (t == "al") {
    std::string& o = out[2];
    c_ts(o, a, 2); o += '\t';
    c_ts(o, a, 1); o += '\t';
    c_str(o, a, 3); o += '\t';
    c_str(o, a, 4); o += '\t';
    c_str(o, a, 5); o += '\t';
    Fields e;
    split(a.has(6) ? a.f[6] : std::string_view(), '&', e);
    std::string js;
    fs_row_json(js, e);
    copy_escape(o, js);
    o += '\n';
    return 2;
  }
  if (t == "fb") {  // fleet baseline: timestamp, service, lag, nseries, stats json
    std::string& o = out[4];
    c_ts(o, a, 1); o += '\t';
    c_str(o, a, 2); o += '\t';
    c_str(o, a, 3); o += '\t';
    c_num(o, a.has(4) ? js::parse_int(a.f[4]) : js::nan()); o += '\t';
    static const char* names[3] = {"average", "per75", "per95"};
    std::string js = "{";
    for (int k = 0; k < 3; ++k) {
      Fields p;
      if (a.has(5 + k)) split(a.f[5 + k], ':', p);
      for (int j = 0; j < 2; ++j) {
        if (k || j) js += ',';
        js += '"';
        js += names[k];
        js += j ? "std\":" : "mean\":";
        j_num(js, p.has(j) ? parse_float(p.f[j]) : js::nan());
      }
    }
    js += '}';
    copy_escape(o, js);
    o += '\n';
    return 4;
  }
  if (t == "jx") {
    std::string& o = out[3];
    c_ts(o, a, 1); o += '\t';
    c_str(o, a, 2);
    for (int k = 0; k < 16; ++k) {
      o += '\t';
      const int i = 3 + k;
      c_num(o, !a.has(i) ? js::nan() : (k == 9 ? parse_float(a.f[i]) : js::parse_int(a.f[i])));
    }
    o += '\n';
    return 3;
  }
  return -1;
}

// Encode a newline-separated blob; counts[k] rows appended to out[k].
void encode_blob(std::string_view blob, std::string* out, int64_t* counts) {
  size_t i = 0;
  while (i < blob.size()) {
    size_t j = blob.find('\n', i);
    if (j == std::string_view::npos) j = blob.size();
    if (j > i) {
      const int k = encode_line(blob.substr(i, j - i), out);
      if (k >= 0) ++counts[k];
    }
    i = j + 1;
  }
}

}  // namespace copyenc
}  // namespace apm
