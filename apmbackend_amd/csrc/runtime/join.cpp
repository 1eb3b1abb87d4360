// Host join workers -- see join.h for the contract.  Each handler below cites the reference
// lines whose behaviour it reproduces; tests/test_engine_parity.py checks the produced tx
// stream byte-for-byte against the oracle (which itself is checked against the reference JS).
#include "join.h"

#include <algorithm>
#include <cctype>

namespace apm {

namespace {

std::string_view tok_or_undef(const std::vector<std::string_view>& t, size_t i) {
  return i < t.size() ? t[i] : std::string_view("undefined");
}
bool has_tok(const std::vector<std::string_view>& t, size_t i) { return i < t.size(); }

std::string strip_brackets(std::string_view s) {  // .replace(/[[\]]/g, '')
  std::string r;
  r.reserve(s.size());
  for (char c : s) if (c != '[' && c != ']') r.push_back(c);
  return r;
}

bool all_digits(std::string_view s) {
  if (s.empty()) return false;
  for (char c : s) if (c < '0' || c > '9') return false;
  return true;
}

bool icontains(std::string_view hay, std::string_view needle) {
  if (needle.size() > hay.size()) return false;
  for (size_t i = 0; i + needle.size() <= hay.size(); ++i) {
    size_t k = 0;
    for (; k < needle.size(); ++k)
      if (std::tolower((unsigned char)hay[i + k]) != std::tolower((unsigned char)needle[k])) break;
    if (k == needle.size()) return true;
  }
  return false;
}

// service.replace(/Provider\[/i, 'Provider:').replace(']', '')
std::string normalize_service(std::string_view raw) {
  std::string s(raw);
  for (size_t i = 0; i + 9 <= s.size(); ++i) {
    static const char pat[] = "provider[";
    size_t k = 0;
    for (; k < 9; ++k) if (std::tolower((unsigned char)s[i + k]) != pat[k]) break;
    if (k == 9) { s.replace(i, 9, "Provider:"); break; }
  }
  size_t b = s.find(']');
  if (b != std::string::npos) s.erase(b, 1);
  return s;
}

// line.replace(/<\/.*/,'').replace(/.*>/,'')
std::string xml_inner(std::string_view line) {
  std::string_view s = line;
  size_t p = s.find("</");
  if (p != std::string_view::npos) s = s.substr(0, p);
  size_t q = s.rfind('>');
  if (q != std::string_view::npos) s = s.substr(q + 1);
  return std::string(s);
}

// split(/<|>/)[2] of trim(line)
std::string_view angle_field2(std::string_view line) {
  std::string_view t = js::trim(line);
  int field = 0;
  size_t start = 0;
  for (size_t i = 0; i <= t.size(); ++i) {
    if (i == t.size() || t[i] == '<' || t[i] == '>') {
      if (field == 2) return t.substr(start, i - start);
      ++field;
      start = i + 1;
    }
  }
  return std::string_view();
}

std::vector<std::string_view> info_segment_tokens(std::string_view line) {
  // line.split(/INFO/)[1].trim().split(/[\s]+/)
  size_t p1 = line.find("INFO");
  if (p1 == std::string_view::npos) return {std::string_view()};
  size_t p2 = line.find("INFO", p1 + 4);
  std::string_view seg = line.substr(p1 + 4, p2 == std::string_view::npos ? std::string_view::npos : p2 - p1 - 4);
  return js::split_ws(js::trim(seg));
}

bool baf_match(std::string_view line) {  // /\[[^ ]+] +INFO /
  for (size_t i = 1; i < line.size(); ++i) {
    if (line[i] != ']') continue;
    size_t j = i + 1;
    if (j >= line.size() || line[j] != ' ') continue;
    while (j < line.size() && line[j] == ' ') ++j;
    if (line.compare(j, 5, "INFO ") != 0) continue;
    for (size_t k = i; k-- > 0;) {
      if (line[k] == ' ') break;
      if (line[k] == '[' && k + 1 < i) return true;
    }
  }
  return false;
}

}  // namespace

int32_t Dictionary::service_id(std::string_view normalized) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = svc_map_.find(std::string(normalized));
  if (it != svc_map_.end()) return it->second;
  int32_t id = (int32_t)services_.size();
  services_.emplace_back(normalized);
  svc_map_.emplace(services_.back(), id);
  return id;
}

// ----------------------------------------------------------------------------- clock / caches

void JoinShard::begin_batch(double now_ms, uint64_t batch_no) {
  now_ = now_ms;
  batch_no_ = batch_no;
  sweep();
}

JoinShard::NeedMap& JoinShard::need_map(const std::string& log_id) {
  auto nit = need_.find(log_id);
  if (nit == need_.end()) {
    nit = need_.emplace(log_id, TtlEntry<NeedMap>{NeedMap{}, now_ + cfg_.need_ttl_ms}).first;
    nit->second.v.created = (batch_no_ << 28) | (cur_line_ & 0xfffffff);
    need_order_.emplace_back(log_id, nit->second.exp);
  }
  return nit->second.v;
}

void JoinShard::sweep() {
  // recordCache: expired partial maps are discarded (error log in the reference, :220-224)
  for (auto it = record_.begin(); it != record_.end();) {
    if (it->second.exp < now_) { counters.expired_partials += it->second.v.items.size(); it = record_.erase(it); }
    else ++it;
  }
  // needNumRecordCache: expiry emits every parked record with altAcctNum or '' (:226-239).
  // Creation order == expiry order (the clock never goes back), so a FIFO gives NodeCache's
  // insertion-ordered sweep.
  while (!need_order_.empty() && need_order_.front().second < now_) {
    auto key = need_order_.front();
    need_order_.pop_front();
    auto it = need_.find(key.first);
    if (it == need_.end() || it->second.exp != key.second) continue;
    NeedMap nm = std::move(it->second.v);
    need_.erase(it);
    expire_need(key.first, nm);
  }
  for (auto it = acct_.begin(); it != acct_.end();) {
    if (it->second.exp < now_) it = acct_.erase(it); else ++it;
  }
}

void JoinShard::expire_need(const std::string& log_id, NeedMap& nm) {
  sub_ = 0;
  for (auto& r : nm.items) {
    ++counters.need_expired;
    const double acct = r.alt_acct.empty() ? js::nan() : js::parse_int(r.alt_acct);
    output(r.server, r.service_raw, log_id, acct, r.start_ms, r.start_empty, r.end_ms, r.end_empty, r.elapsed,
           r.insert_to_db, nm.created);
  }
}

// outputRecord (:264-290)
void JoinShard::output(int32_t server, std::string_view service_raw, std::string_view log_id, double acct,
                       double start_ms, bool start_empty, double end_ms, bool end_empty, double elapsed,
                       bool to_db, uint64_t seq) {
  TxOut t;
  t.seq = (seq << 12) | (sub_++ & 0xfff);
  t.server = server;
  const std::string svc = normalize_service(service_raw);
  t.service = dict_->service_id(svc);
  t.log_id.assign(log_id);
  t.acct = acct;
  double s = start_empty ? js::nan() : start_ms;
  const double e_for_sub = end_empty ? 0.0 : end_ms;  // JS: '' - n === -n
  if (!(s == s) || s == 0) s = e_for_sub - elapsed;
  // TxEntry parseInt's numbers through their string form: integral values pass unchanged
  t.start_ms = std::isfinite(s) ? std::trunc(s) : js::nan();
  t.end_ms = end_empty ? js::nan() : (std::isfinite(end_ms) ? std::trunc(end_ms) : js::nan());
  t.elapsed = elapsed;
  t.to_db = to_db;
  t.toplevel = svc.size() >= 2 && svc[0] == 'S' && svc[1] == ':';
  ++counters.tx;
  if (to_db) ++counters.tx_db;
  out_.push_back(std::move(t));
}

// saveAcctNum (:294-327). source: 0 standard, 1 riskStrategy, 2 bafmetainfo.
void JoinShard::save_acct(std::string_view acct_raw, int32_t file, int source, std::string_view alt_log_id,
                          uint64_t seq) {
  std::string_view acct = js::trim(acct_raw);
  if (!all_digits(acct)) {
    ++counters.invalid_acct;  // reference logs (and throws via the $currLogFp typo, Q16: fixed)
    return;
  }
  std::string log_id;
  if (source == 2) {
    if (alt_log_id.empty()) return;
    log_id.assign(alt_log_id);
  } else {
    auto it = soap_.find(file);
    log_id = (it != soap_.end() && it->second.has_log_id) ? it->second.log_id : std::string("undefined");
  }
  auto& ae = acct_[log_id];
  ae.v.assign(acct);
  ae.exp = now_ + cfg_.acct_ttl_ms;
  if (source != 2) soap_.erase(file);
  auto nit = need_.find(log_id);
  if (nit != need_.end()) {
    const double a = js::parse_int(acct);
    const int32_t server = (*files_)[file].server;
    for (auto& r : nit->second.v.items)
      output(server, r.service_raw, log_id, a, r.start_ms, r.start_empty, r.end_ms, r.end_empty, r.elapsed, false,
             seq);
    nit->second.v.items.clear();
  }
}

// attemptReadAccountNumberFromBAFInfo (:486-497)
std::string JoinShard::baf_acct(std::string_view line, const std::vector<std::string_view>& toks, int32_t file,
                                std::string_view log_id, uint64_t seq) {
  if (!baf_match(line)) return std::string();
  std::string_view t3 = has_tok(toks, 3) ? toks[3] : std::string_view();
  // .replace(/.*]\[/,'') -> drop through the last "]["
  size_t p = std::string_view::npos;
  for (size_t i = 0; i + 1 < t3.size(); ++i) if (t3[i] == ']' && t3[i + 1] == '[') p = i;
  if (p != std::string_view::npos) t3 = t3.substr(p + 2);
  std::string s = strip_brackets(t3);
  size_t c = s.rfind(':');
  std::string acct = c == std::string::npos ? s : s.substr(c + 1);
  if (!acct.empty()) save_acct(acct, file, 2, log_id, seq);
  return acct;
}

// ----------------------------------------------------------------------------- handlers

void JoinShard::on_soap(const Event& e, std::string_view line, int32_t file, uint64_t seq) {
  const uint32_t m = e.mask;
  if (m & PM_SOAP_IN) {
    auto toks = js::split_ws(line, 4);
    SoapCtx c;
    if (has_tok(toks, 1)) {
      std::string_view t1 = toks[1];
      size_t eq = t1.find('=');
      if (eq != std::string_view::npos) {
        size_t eq2 = t1.find('=', eq + 1);
        c.log_id.assign(t1.substr(eq + 1, eq2 == std::string_view::npos ? std::string_view::npos : eq2 - eq - 1));
        c.has_log_id = true;
      }
    }
    soap_[file] = c;
  } else if (m & PM_SOAP_OUT) {
    soap_.erase(file);
  } else {
    auto it = soap_.find(file);
    if (it == soap_.end()) return;
    if (m & PM_SOAP_ACCT) {
      save_acct(angle_field2(line), file, 0, {}, seq);
    } else if (m & PM_SOAP_KEY) {
      it->second.pull_next = true;
    } else if ((m & PM_SOAP_VALUE) && it->second.pull_next) {
      save_acct(angle_field2(line), file, 1, {}, seq);
    }
  }
}

void JoinShard::on_ejb(const Event& e, std::string_view line, int32_t file, bool entry, uint64_t seq) {
  const int32_t server = (*files_)[file].server;
  auto toks = js::split_ws(line, 16);
  const std::string log_id = strip_brackets(toks[0]);
  double ts;
  bool ts_empty = false;
  if (!(e.mask & PM_HOST) && has_tok(toks, 2)) {
    ts = e.ts;
  } else {
    std::string tsstr = std::string(tok_or_undef(toks, 1)) + " " + std::string(tok_or_undef(toks, 2));
    if (!js::convert_date(tsstr, cfg_.tz, ts)) { ts_empty = true; ts = js::nan(); }
  }
  if (entry) {  // parseEjbCommonTimingEntry (:378-401)
    if (log_id.empty()) return;
    std::string service = "S:" + std::string(tok_or_undef(toks, 13));
    auto it = record_.find(log_id);
    if (it == record_.end()) {
      it = record_.emplace(log_id, TtlEntry<RecordMap>{RecordMap{}, now_ + cfg_.record_ttl_ms}).first;
    }
    auto& items = it->second.v.items;
    auto f = std::find_if(items.begin(), items.end(), [&](const Partial& p) { return p.service_raw == service; });
    if (f != items.end()) { f->server = server; f->start_ms = ts; f->start_empty = ts_empty; }
    else items.push_back(Partial{service, server, ts, ts_empty});
    return;
  }
  // parseEjbCommonTimingExit (:403-446)
  std::string service = "S:" + std::string(tok_or_undef(toks, 9));
  double elapsed;
  if (!(e.mask & PM_HOST) && has_tok(toks, 11)) elapsed = e.num;
  else elapsed = has_tok(toks, 11) ? js::parse_int(toks[11]) : js::nan();
  if (log_id.empty()) {
    output(server, service, "", js::nan(), 0, true, ts, ts_empty, elapsed, false, seq);
    return;
  }
  auto it = record_.find(log_id);
  if (it == record_.end()) { ++counters.ejb_exit_unmatched; return; }
  auto& items = it->second.v.items;
  auto f = std::find_if(items.begin(), items.end(), [&](const Partial& p) { return p.service_raw == service; });
  if (f == items.end()) { ++counters.ejb_exit_unmatched; return; }
  Partial part = *f;
  items.erase(f);
  auto ait = acct_.find(log_id);
  if (ait != acct_.end()) {
    output(server, service, log_id, js::parse_int(ait->second.v), part.start_ms, part.start_empty, ts, ts_empty,
           elapsed, false, seq);
  } else {
    Need n{service, part.server, part.start_ms, part.start_empty, ts, ts_empty, elapsed, std::string(), false};
    auto& ni = need_map(log_id).items;
    auto g = std::find_if(ni.begin(), ni.end(), [&](const Need& x) { return x.service_raw == service; });
    if (g != ni.end()) *g = n; else ni.push_back(n);
  }
}

void JoinShard::on_ct(const Event& e, std::string_view line, int32_t file, bool entry, uint64_t seq) {
  const int32_t server = (*files_)[file].server;
  auto toks = js::split_ws(line, 8);
  const std::string log_id = strip_brackets(toks[0]);
  double ts;
  bool ts_empty = false;
  if (!(e.mask & PM_HOST) && has_tok(toks, 2)) {
    ts = e.ts;
  } else {
    std::string tsstr = std::string(tok_or_undef(toks, 1)) + " " + std::string(tok_or_undef(toks, 2));
    if (!js::convert_date(tsstr, cfg_.tz, ts)) { ts_empty = true; ts = js::nan(); }
  }
  std::vector<std::string_view> seg;
  std::string_view service_v, elapsed_v;
  bool has_service, has_elapsed;
  if (!(e.mask & PM_HOST)) {
    has_service = e.tAs != 0xffff;
    has_elapsed = e.tBs != 0xffff;
    if (has_service) service_v = line.substr(e.tAs, e.tAe - e.tAs);
    if (has_elapsed) elapsed_v = line.substr(e.tBs, e.tBe - e.tBs);
  } else {
    seg = info_segment_tokens(line);
    has_service = has_tok(seg, 1);
    has_elapsed = has_tok(seg, 5);
    if (has_service) service_v = seg[1];
    if (has_elapsed) elapsed_v = seg[5];
  }
  const std::string service = has_service ? std::string(service_v) : std::string("undefined");
  if (entry) {  // parseCommonTimingEntry (:451-483)
    if (log_id.empty()) return;
    auto it = record_.find(log_id);
    if (it == record_.end())
      it = record_.emplace(log_id, TtlEntry<RecordMap>{RecordMap{}, now_ + cfg_.record_ttl_ms}).first;
    auto& items = it->second.v.items;
    auto f = std::find_if(items.begin(), items.end(), [&](const Partial& p) { return p.service_raw == service; });
    if (f != items.end()) { f->server = server; f->start_ms = ts; f->start_empty = ts_empty; }
    else items.push_back(Partial{service, server, ts, ts_empty});
    return;
  }
  // parseCommonTimingExit (:506-565)
  double elapsed = js::nan();
  if (has_elapsed) elapsed = (!(e.mask & PM_HOST)) ? e.num : js::parse_int(elapsed_v);
  auto salvage = [&]() {  // salvageRecordAndOutput (:500-504)
    std::string acct = baf_acct(line, toks, file, log_id, seq);
    output(server, service, "", acct.empty() ? js::nan() : js::parse_int(acct), 0, true, ts, ts_empty, elapsed,
           false, seq);
  };
  if (log_id.empty()) { salvage(); return; }
  auto it = record_.find(log_id);
  if (it == record_.end()) { salvage(); return; }
  auto& items = it->second.v.items;
  auto f = std::find_if(items.begin(), items.end(), [&](const Partial& p) { return p.service_raw == service; });
  if (f == items.end()) { salvage(); return; }
  Partial part = *f;
  auto ait = acct_.find(log_id);
  if (ait != acct_.end()) {
    items.erase(f);
    output(server, service, log_id, js::parse_int(ait->second.v), part.start_ms, part.start_empty, ts, ts_empty,
           elapsed, false, seq);
    return;
  }
  need_map(log_id);
  std::string alt = baf_acct(line, toks, file, log_id, seq);  // may drain the need map first
  Need n{service, part.server, part.start_ms, part.start_empty, ts, ts_empty, elapsed, alt, false};
  auto& ni = need_map(log_id).items;
  auto g = std::find_if(ni.begin(), ni.end(), [&](const Need& x) { return x.service_raw == service; });
  if (g != ni.end()) *g = n; else ni.push_back(n);
  // map.delete(service): the partial was looked up before baf_acct; re-find (vector may move)
  auto it2 = record_.find(log_id);
  if (it2 != record_.end()) {
    auto& it2i = it2->second.v.items;
    auto f2 = std::find_if(it2i.begin(), it2i.end(), [&](const Partial& p) { return p.service_raw == service; });
    if (f2 != it2i.end()) it2i.erase(f2);
  }
}

// parseAppLine (:578-731)
void JoinShard::on_app(const Event& e, std::string_view line, int32_t file, uint64_t seq) {
  const uint32_t m = e.mask;
  const int32_t server = (*files_)[file].server;
  if (m & PM_AUTR_MAP) {
    auto toks = js::split_ws(line, 8);
    std::string log_id = strip_brackets(toks[0]);
    std::string_view t5 = has_tok(toks, 5) ? toks[5] : std::string_view();
    size_t eq = t5.find('=');
    std::string autr;
    if (eq != std::string_view::npos) {
      size_t eq2 = t5.find('=', eq + 1);
      autr.assign(t5.substr(eq + 1, eq2 == std::string_view::npos ? std::string_view::npos : eq2 - eq - 1));
    } else {
      autr = "undefined";
    }
    AuditCtx& ctx = audit_[file];
    std::string alt = baf_acct(line, toks, file, log_id, seq);
    auto f = std::find_if(ctx.autr_map.begin(), ctx.autr_map.end(), [&](auto& p) { return p.first == autr; });
    if (f != ctx.autr_map.end()) f->second = {log_id, alt};
    else ctx.autr_map.push_back({autr, {log_id, alt}});
    return;
  }
  if (m & PM_AUTR_HDR) {
    auto cit = audit_.find(file);
    if (cit == audit_.end()) { ++counters.audit_errors; return; }
    AuditCtx& ctx = cit->second;
    size_t c1 = line.find(':');
    size_t c2 = line.find(':', c1 + 1);
    std::string autr(js::trim(line.substr(c1 + 1, c2 == std::string_view::npos ? std::string_view::npos : c2 - c1 - 1)));
    auto f = std::find_if(ctx.autr_map.begin(), ctx.autr_map.end(), [&](auto& p) { return p.first == autr; });
    if (f == ctx.autr_map.end() || f->second.first.empty()) { ++counters.audit_errors; return; }
    ctx.service_map.clear();
    ctx.active = true;
    ctx.active_log_id = f->second.first;
    ctx.active_alt = f->second.second;
    ctx.elapsed_flag = false;
    ctx.sw_flag = false;
    ctx.has_active_service = false;
    ctx.autr_map.erase(f);
    return;
  }
  auto cit = audit_.find(file);
  if (cit == audit_.end() || !cit->second.active) return;
  AuditCtx& ctx = cit->second;
  if (m & PM_EL_START) { ctx.elapsed_flag = true; return; }
  if (ctx.elapsed_flag) {
    if (m & PM_EL_END) { ctx.elapsed_flag = false; return; }
    size_t c1 = line.find(':');
    std::string service(js::trim(line.substr(0, c1)));
    std::string elapsed;
    if (c1 != std::string_view::npos) {
      size_t c2 = line.find(':', c1 + 1);
      std::string_view a1 = line.substr(c1 + 1, c2 == std::string_view::npos ? std::string_view::npos : c2 - c1 - 1);
      auto st = js::split_ws(a1, 2);
      elapsed = strip_brackets(st[0]);
    }
    auto f = std::find_if(ctx.service_map.begin(), ctx.service_map.end(), [&](auto& p) { return p.first == service; });
    if (f == ctx.service_map.end()) { ctx.service_map.push_back({service, {}}); f = ctx.service_map.end() - 1; }
    f->second.push_back(AuditItem{elapsed, false, std::string()});
    return;
  }
  if (m & PM_SW_START) { ctx.sw_flag = true; return; }
  if (!ctx.sw_flag) return;
  if (m & PM_SW_END) {
    ctx.active = false;
    ctx.active_log_id.clear();
    ctx.active_alt.clear();
    ctx.has_active_service = false;
    ctx.elapsed_flag = false;
    ctx.sw_flag = false;
    ctx.service_map.clear();
    return;
  }
  if (m & PM_SW_NAME) { ctx.active_service = xml_inner(line); ctx.has_active_service = true; return; }
  if (!ctx.has_active_service || ctx.active_service.empty()) return;
  const std::string& svc = ctx.active_service;
  auto f = std::find_if(ctx.service_map.begin(), ctx.service_map.end(), [&](auto& p) { return p.first == svc; });
  if (m & PM_SW_STARTTS) {
    if (f == ctx.service_map.end() || f->second.empty()) { ++counters.audit_errors; return; }
    f->second.front().has_start = true;
    f->second.front().start_ts = xml_inner(line);
    return;
  }
  if (m & PM_SW_STOPTS) {
    std::string end_ts = xml_inner(line);
    if (f == ctx.service_map.end() || f->second.empty()) { ++counters.audit_errors; return; }
    AuditItem obj = f->second.front();
    f->second.pop_front();
    const std::string& log_id = ctx.active_log_id;
    const bool to_db = !icontains(svc, "Provider[");
    double s_ms = js::nan(), e_ms = js::nan();
    bool s_empty = !obj.has_start || !js::convert_date(obj.start_ts, cfg_.tz, s_ms);
    bool e_empty = !js::convert_date(end_ts, cfg_.tz, e_ms);
    const double elapsed = js::parse_int(obj.elapsed);
    auto ait = acct_.find(log_id);
    if (ait != acct_.end()) {
      output(server, svc, log_id, js::parse_int(ait->second.v), s_ms, s_empty, e_ms, e_empty, elapsed, to_db, seq);
    } else {
      Need n{svc, server, s_ms, s_empty, e_ms, e_empty, elapsed, ctx.active_alt, to_db};
      auto& ni = need_map(log_id).items;
      auto g = std::find_if(ni.begin(), ni.end(), [&](const Need& x) { return x.service_raw == svc; });
      if (g != ni.end()) *g = n; else ni.push_back(n);
    }
  }
}

void JoinShard::process(const Event* ev, size_t n, const uint8_t* bytes, const std::vector<int32_t>& chunk_file) {
  for (size_t i = 0; i < n; ++i) {
    const Event& e = ev[i];
    ++counters.events;
    if (e.mask & PM_HOST) ++counters.host_fallback;
    const int32_t file = chunk_file[e.chunk];
    std::string_view line((const char*)bytes + e.off, e.len);
    const uint64_t seq = (1ULL << 51) | e.line;  // << 12 in output(): bit 63 marks line emissions
    cur_line_ = e.line;
    sub_ = 0;
    switch (e.kind) {
      case LK_SOAP: on_soap(e, line, file, seq); break;
      case LK_EJB_ENTRY: on_ejb(e, line, file, true, seq); break;
      case LK_EJB_EXIT: on_ejb(e, line, file, false, seq); break;
      case LK_CT_ENTRY: on_ct(e, line, file, true, seq); break;
      case LK_CT_EXIT: on_ct(e, line, file, false, seq); break;
      case LK_APP: on_app(e, line, file, seq); break;
      default: break;
    }
  }
}

}  // namespace apm
