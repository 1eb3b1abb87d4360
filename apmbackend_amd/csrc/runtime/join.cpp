// Host join workers -- see join.h for the contract.  Each handler cites the reference lines
// whose behaviour it reproduces; tests/test_join_native.py checks the produced tx stream
// byte-for-byte against the oracle (itself checked against the reference JS).
#include "join.h"
#include "join_util.h"

#include <algorithm>
#include <cctype>
#include <cstring>
#ifdef APM_JOIN_PROF
#include <x86intrin.h>
#include <cstdio>
uint64_t prof_cyc[16], prof_n[16];
struct ProfDump { ~ProfDump() { for (int i = 0; i < 16; ++i) if (prof_n[i]) fprintf(stderr, "kind %d: n=%lu avg=%.0f cyc\n", i, prof_n[i], (double)prof_cyc[i] / prof_n[i]); } } prof_dump;
#endif

namespace apm {

namespace {

using namespace jstr;

// Token views for one event: GPU-provided offsets on the fast path, a JS-exact re-split when
// the kernel deferred the line to the host (PM_HOST: non-ASCII whitespace, exotic numbers).
struct Toks {
  std::string_view t[16];
  int n = 0;
  void from_event(const Event& e, std::string_view line) {
    n = e.ntok;
    const uint16_t* se = &e.t0s;
    for (int k = 0; k < 4 && k < n; ++k) t[k] = line.substr(se[2 * k], se[2 * k + 1] - se[2 * k]);
  }
  void from_line(std::string_view line) {
    auto v = js::split_ws(line, 16);
    n = (int)v.size();
    for (int k = 0; k < n && k < 16; ++k) t[k] = v[k];
  }
  bool has(int i) const { return i < n; }
  std::string_view get(int i) const { return i < n ? t[i] : kUndef; }
};

}  // namespace

int32_t Dictionary::service_id(std::string_view normalized) {
  std::lock_guard<std::mutex> g(mu_);
  std::string key(normalized);
  auto it = svc_map_.find(key);
  if (it != svc_map_.end()) return it->second;
  int32_t id = (int32_t)services_.size();
  services_.push_back(key);
  svc_map_.emplace(std::move(key), id);
  return id;
}

int32_t JoinShard::raw_service(uint64_t h, bool ejb, std::string_view name) {
  const size_t raw_len = name.size() + (ejb ? 2 : 0);
  if (const int32_t* slot = raw_svc_map_.find(h)) {
    if (svc_info_[*slot - 1].raw_len == raw_len) return *slot - 1;
  }
  std::string raw(ejb ? "S:" : "");
  raw += name;
  return intern_service(std::move(raw), h);
}

int32_t JoinShard::intern_service(std::string raw, uint64_t h) {
  std::string norm = normalize_service(raw);
  const int32_t id = (int32_t)raw_svc_.size();
  const bool top = norm.size() >= 2 && norm[0] == 'S' && norm[1] == ':';
  const int32_t nid = dict_->service_id(norm);
  svc_info_.push_back(SvcInfo{(uint32_t)svc_text_.size(), (uint32_t)norm.size(), nid, (uint32_t)raw.size(), top});
  svc_text_ += norm;
  raw_svc_.push_back(RawService{std::move(raw), std::move(norm), nid, top, h});
  int32_t* slot = raw_svc_map_.find(h);
  if (!slot) raw_svc_map_[h] = id + 1;  // a colliding name is re-interned on every call (correct, slow)
  return id;
}

// ----------------------------------------------------------------------------- clock / caches

void JoinShard::begin_batch(double now_ms, uint64_t batch_no) {
  text_.clear();
  if (text_.capacity() < (1u << 20)) text_.reserve(1u << 20);  // arenas move into release blocks
  now_ = now_ms;
  batch_no_ = batch_no;
  sweep();
}

JoinShard::NeedEntry& JoinShard::need_map(uint64_t key, std::string_view log_id) {
  auto r = need_.emplace(key);
  NeedEntry& ne = *r.first;
  if (r.second) {
    ne.exp = now_ + cfg_.need_ttl_ms;
    ne.created = (batch_no_ << 28) | (cur_line_ & 0xfffffff);
    ne.log_id.assign(log_id);
    need_fifo_.emplace_back(key, ne.exp);
  }
  return ne;
}

JoinShard::RecordEntry& JoinShard::record_map(uint64_t key) {
  auto r = record_.emplace(key);
  if (r.second) {
    r.first->exp = now_ + cfg_.record_ttl_ms;
    record_fifo_.emplace_back(key, r.first->exp);
  }
  return *r.first;
}

void JoinShard::sweep() {
  // every expiry is a random map access: request the slots a few entries ahead
  constexpr size_t kAhead = 8;
  for (size_t i = 0; i < kAhead && i < record_fifo_.size() && record_fifo_[i].second < now_; ++i)
    record_.prefetch(record_fifo_[i].first);
  for (size_t i = 0; i < kAhead && i < acct_fifo_.size() && acct_fifo_[i].second < now_; ++i)
    acct_.prefetch(acct_fifo_[i].first);
  // recordCache: expired partial maps are discarded (error log in the reference, :220-224)
  while (!record_fifo_.empty() && record_fifo_.front().second < now_) {
    if (record_fifo_.size() > kAhead && record_fifo_[kAhead].second < now_) record_.prefetch(record_fifo_[kAhead].first);
    auto k = record_fifo_.front();
    record_fifo_.pop_front();
    RecordEntry* it = record_.find(k.first);
    if (!it || it->exp != k.second) continue;
    counters.expired_partials += it->items.size();
    record_.erase(k.first);
  }
  // needNumRecordCache: expiry emits every parked record with altAcctNum or '' (:226-239).
  // Creation order == expiry order (the clock never goes back): the FIFO is NodeCache's
  // insertion-ordered sweep.
  while (!need_fifo_.empty() && need_fifo_.front().second < now_) {
    auto k = need_fifo_.front();
    need_fifo_.pop_front();
    NeedEntry* it = need_.find(k.first);
    if (!it || it->exp != k.second) continue;
    NeedEntry ne = std::move(*it);
    need_.erase(k.first);
    expire_need(ne);
  }
  while (!acct_fifo_.empty() && acct_fifo_.front().second < now_) {
    if (acct_fifo_.size() > kAhead && acct_fifo_[kAhead].second < now_) acct_.prefetch(acct_fifo_[kAhead].first);
    auto k = acct_fifo_.front();
    acct_fifo_.pop_front();
    AcctEntry* it = acct_.find(k.first);
    if (it && it->exp == k.second) acct_.erase(k.first);
  }
}

void JoinShard::expire_need(NeedEntry& nm) {
  sub_ = 0;
  for (auto& r : nm.items) {
    ++counters.need_expired;
    output(r.server, r.svc, nm.log_id, r.alt_acct, r.start_ms, r.start_empty, r.end_ms, r.end_empty, r.elapsed,
           r.insert_to_db, nm.created);
  }
}

// outputRecord (:264-290)
void JoinShard::output(int32_t server, int32_t svc, std::string_view log_id, double acct, double start_ms,
                       bool start_empty, double end_ms, bool end_empty, double elapsed, bool to_db, uint64_t seq) {
  out_.emplace_back();
  TxOut& t = out_.back();
  t.seq = (seq << 12) | (sub_++ & 0xfff);
  t.server = server;
  const SvcInfo& rs = svc_info_[svc];
  const std::string_view norm(svc_text_.data() + rs.norm_off, rs.norm_len);
  t.service = rs.norm_id;
  t.raw_svc = svc;
  double s = start_empty ? js::nan() : start_ms;
  const double e_for_sub = end_empty ? 0.0 : end_ms;  // JS: '' - n === -n
  if (!(s == s) || s == 0) s = e_for_sub - elapsed;
  // TxEntry parseInt's numbers through their string form: integral values pass unchanged
  const double start = std::isfinite(s) ? std::trunc(s) : js::nan();
  t.end_ms = end_empty ? js::nan() : (std::isfinite(end_ms) ? std::trunc(end_ms) : js::nan());
  t.elapsed = elapsed;
  t.to_db = to_db;
  t.toplevel = rs.toplevel;
  // wire line, formatted here on the join worker (parallel across shards): one append of a
  // stack-built line on the common path
  t.line_off = (uint32_t)text_.size();
  const std::string& srv = (*servers_)[server];
  char buf[512];
  const size_t fixed = srv.size() + norm.size() + log_id.size() + 3 + 8 + 4 * 32 + 2;
  if (fixed <= sizeof(buf)) {
    char* p = buf;
    auto put = [&](const char* q, size_t n) { std::memcpy(p, q, n); p += n; };
    put("tx|", 3);
    put(srv.data(), srv.size());
    *p++ = '|';
    put(norm.data(), norm.size());
    *p++ = '|';
    put(log_id.data(), log_id.size());
    *p++ = '|';
    p = js::put_num(p, acct);
    *p++ = '|';
    p = js::put_num(p, start);
    *p++ = '|';
    p = js::put_num(p, t.end_ms);
    *p++ = '|';
    p = js::put_num(p, elapsed);
    *p++ = '|';
    *p++ = rs.toplevel ? 'Y' : 'N';
    t.line_len = (uint32_t)(p - buf);
    *p++ = '\n';
    text_.append(buf, (size_t)(p - buf));
  } else {
    text_ += "tx|";
    text_ += srv;
    text_ += '|';
    text_ += norm;
    text_ += '|';
    text_ += log_id;
    text_ += '|';
    js::append_num(text_, acct);
    text_ += '|';
    js::append_num(text_, start);
    text_ += '|';
    js::append_num(text_, t.end_ms);
    text_ += '|';
    js::append_num(text_, elapsed);
    text_ += '|';
    text_ += rs.toplevel ? 'Y' : 'N';
    t.line_len = (uint32_t)(text_.size() - t.line_off);
    text_ += '\n';  // lines stay newline-terminated in the arena (zero-copy release, engine.cpp)
  }
  ++counters.tx;
  if (to_db) ++counters.tx_db;
}

// saveAcctNum (:294-327). source: 0 standard, 1 riskStrategy, 2 bafmetainfo.
void JoinShard::save_acct(std::string_view acct_raw, int32_t file, int source, std::string_view alt_log_id,
                          uint64_t seq) {
  std::string_view acct = js::trim(acct_raw);
  if (!all_digits(acct)) {
    ++counters.invalid_acct;  // reference logs (and throws via the $currLogFp typo, Q16: fixed)
    return;
  }
  std::string_view log_id;
  if (source == 2) {
    if (alt_log_id.empty()) return;
    log_id = alt_log_id;
  } else {
    SoapCtx* sc = soap_.find(file);
    if (sc && sc->has_log_id) log_id = sc->log_id;  // storage survives soap_.erase below
    else log_id = kUndef;
  }
  const uint64_t key = key_of(log_id);
  const double a = js::parse_int(acct);
  auto& ae = acct_[key];
  ae.acct = a;
  ae.exp = now_ + cfg_.acct_ttl_ms;
  acct_fifo_.emplace_back(key, ae.exp);
  if (source != 2) soap_.erase(file);
  NeedEntry* nit = need_.find(key);
  if (nit && !nit->items.empty()) {
    const int32_t server = (*files_)[file].server;
    std::vector<Need> items;
    items.swap(nit->items);  // the (now empty) map stays until it expires
    for (auto& r : items)
      output(server, r.svc, log_id, a, r.start_ms, r.start_empty, r.end_ms, r.end_empty, r.elapsed, false, seq);
  }
}

// attemptReadAccountNumberFromBAFInfo (:486-497)
std::string_view JoinShard::baf_acct(const Event& e, std::string_view line, std::string_view t3, int32_t file,
                                     std::string_view log_id, uint64_t seq, std::string& scratch) {
  // the parse kernel already tested the pattern (PM_BAF) unless it deferred the line to the host
  if (!((e.mask & PM_HOST) ? baf_match(line) : (e.mask & PM_BAF) != 0)) return std::string_view();
  // .replace(/.*]\[/,'') -> drop through the last "]["
  size_t p = std::string_view::npos;
  for (size_t i = 0; i + 1 < t3.size(); ++i) if (t3[i] == ']' && t3[i + 1] == '[') p = i;
  if (p != std::string_view::npos) t3 = t3.substr(p + 2);
  scratch.clear();
  for (char c : t3) if (c != '[' && c != ']') scratch.push_back(c);
  size_t c = scratch.rfind(':');
  std::string_view acct = c == std::string::npos ? std::string_view(scratch) : std::string_view(scratch).substr(c + 1);
  if (!acct.empty()) save_acct(acct, file, 2, log_id, seq);
  return acct;
}

// ----------------------------------------------------------------------------- handlers

void JoinShard::on_soap(const Event& e, std::string_view line, int32_t file, uint64_t seq) {
  const uint32_t m = e.mask;
  if (m & PM_SOAP_IN) {
    Toks tk;
    if (e.mask & PM_HOST) tk.from_line(line); else tk.from_event(e, line);
    // the context is reused per file: assigning into it keeps the logId string's capacity
    SoapCtx& dst = soap_.put(file);
    dst.has_log_id = false;
    dst.pull_next = false;
    if (tk.has(1)) {
      std::string_view t1 = tk.t[1];
      size_t eq = t1.find('=');
      if (eq != std::string_view::npos) {
        size_t eq2 = t1.find('=', eq + 1);
        dst.log_id.assign(t1.substr(eq + 1, eq2 == std::string_view::npos ? std::string_view::npos : eq2 - eq - 1));
        dst.has_log_id = true;
      }
    }
    if (!dst.has_log_id) dst.log_id.clear();
  } else if (m & PM_SOAP_OUT) {
    soap_.erase(file);
  } else {
    SoapCtx* it = soap_.find(file);
    if (!it) return;
    if (m & PM_SOAP_ACCT) {
      save_acct(angle_field2(line), file, 0, {}, seq);
    } else if (m & PM_SOAP_KEY) {
      it->pull_next = true;
    } else if ((m & PM_SOAP_VALUE) && it->pull_next) {
      save_acct(angle_field2(line), file, 1, {}, seq);
    }
  }
}

void JoinShard::on_ejb(const Event& e, std::string_view line, int32_t file, bool entry, uint64_t seq) {
  const int32_t server = (*files_)[file].server;
  const bool host = e.mask & PM_HOST;
  Toks tk;
  std::vector<std::string_view> all;
  if (host) { all = js::split_ws(line, 16); tk.n = (int)all.size(); for (int k = 0; k < tk.n && k < 16; ++k) tk.t[k] = all[k]; }
  else tk.from_event(e, line);
  std::string scratch;
  const bool keyed = e.mask & PM_KEYS;  // t0 already stripped, key / svc hashed by the kernel
  const std::string_view log_id = keyed ? tk.t[0] : strip_brackets(tk.t[0], scratch);
  double ts;
  bool ts_empty = false;
  if (!host && tk.has(2)) {
    ts = e.ts;
  } else {
    std::string tsstr = std::string(tk.get(1)) + " " + std::string(tk.get(2));
    if (!js::convert_date(tsstr, cfg_.tz, ts)) { ts_empty = true; ts = js::nan(); }
  }
  if (entry) {  // parseEjbCommonTimingEntry (:378-401)
    if (log_id.empty()) return;
    const std::string_view nm = host ? tk.get(13) : (e.tAs != 0xffff ? line.substr(e.tAs, e.tAe - e.tAs) : kUndef);
    const int32_t svc = keyed ? raw_service(e.svc, true, nm) : raw_service(true, nm);
    auto& items = record_map(keyed ? e.key : key_of(log_id)).items;
    auto f = std::find_if(items.begin(), items.end(), [&](const Partial& p) { return p.svc == svc; });
    if (f != items.end()) { f->server = server; f->start_ms = ts; }
    else items.push_back(Partial{svc, server, ts});
    return;
  }
  // parseEjbCommonTimingExit (:403-446)
  double elapsed;
  std::string_view nm;
  if (host) {
    nm = tk.get(9);
    elapsed = tk.has(11) ? js::parse_int(tk.t[11]) : js::nan();
  } else {
    nm = e.tAs != 0xffff ? line.substr(e.tAs, e.tAe - e.tAs) : kUndef;
    elapsed = e.num;
  }
  const int32_t svc = keyed ? raw_service(e.svc, true, nm) : raw_service(true, nm);
  if (log_id.empty()) {
    output(server, svc, "", js::nan(), 0, true, ts, ts_empty, elapsed, false, seq);
    return;
  }
  const uint64_t key = keyed ? e.key : key_of(log_id);
  RecordEntry* it = record_.find(key);
  if (!it) { ++counters.ejb_exit_unmatched; return; }
  auto& items = it->items;
  auto f = std::find_if(items.begin(), items.end(), [&](const Partial& p) { return p.svc == svc; });
  if (f == items.end()) { ++counters.ejb_exit_unmatched; return; }
  const Partial part = *f;
  items.erase(f);
  AcctEntry* ait = acct_.find(key);
  if (ait) {
    output(server, svc, log_id, ait->acct, part.start_ms, false, ts, ts_empty, elapsed, false, seq);
  } else {
    Need n{svc, part.server, part.start_ms, false, ts, ts_empty, elapsed, js::nan(), false};
    auto& ni = need_map(key, log_id).items;
    auto g = std::find_if(ni.begin(), ni.end(), [&](const Need& x) { return x.svc == svc; });
    if (g != ni.end()) *g = n; else ni.push_back(n);
  }
}

void JoinShard::on_ct(const Event& e, std::string_view line, int32_t file, bool entry, uint64_t seq) {
  const int32_t server = (*files_)[file].server;
  const bool host = e.mask & PM_HOST;
  Toks tk;
  if (host) tk.from_line(line); else tk.from_event(e, line);
  std::string scratch;
  const bool keyed = e.mask & PM_KEYS;
  const std::string_view log_id = keyed ? tk.t[0] : strip_brackets(tk.t[0], scratch);
  double ts;
  bool ts_empty = false;
  if (!host && tk.has(2)) {
    ts = e.ts;
  } else {
    std::string tsstr = std::string(tk.get(1)) + " " + std::string(tk.get(2));
    if (!js::convert_date(tsstr, cfg_.tz, ts)) { ts_empty = true; ts = js::nan(); }
  }
  std::string_view service_v = kUndef, elapsed_v;
  bool has_elapsed;
  std::vector<std::string_view> seg;
  if (!host) {
    if (e.tAs != 0xffff) service_v = line.substr(e.tAs, e.tAe - e.tAs);
    has_elapsed = e.tBs != 0xffff;
  } else {
    seg = info_segment_tokens(line);
    if (seg.size() > 1) service_v = seg[1];
    has_elapsed = seg.size() > 5;
    if (has_elapsed) elapsed_v = seg[5];
  }
  const int32_t svc = keyed ? raw_service(e.svc, false, service_v) : raw_service(service_v);
  if (entry) {  // parseCommonTimingEntry (:451-483)
    if (log_id.empty()) return;
    auto& items = record_map(keyed ? e.key : key_of(log_id)).items;
    auto f = std::find_if(items.begin(), items.end(), [&](const Partial& p) { return p.svc == svc; });
    if (f != items.end()) { f->server = server; f->start_ms = ts; }
    else items.push_back(Partial{svc, server, ts});
    return;
  }
  // parseCommonTimingExit (:506-565)
  double elapsed = js::nan();
  if (has_elapsed) elapsed = host ? js::parse_int(elapsed_v) : e.num;
  std::string baf_scratch;
  auto salvage = [&]() {  // salvageRecordAndOutput (:500-504)
    std::string_view acct = baf_acct(e, line, tk.get(3), file, log_id, seq, baf_scratch);
    output(server, svc, "", acct.empty() ? js::nan() : js::parse_int(acct), 0, true, ts, ts_empty, elapsed, false,
           seq);
  };
  if (log_id.empty()) { salvage(); return; }
  const uint64_t key = keyed ? e.key : key_of(log_id);
  RecordEntry* it = record_.find(key);
  if (!it) { salvage(); return; }
  auto* items = &it->items;
  auto f = std::find_if(items->begin(), items->end(), [&](const Partial& p) { return p.svc == svc; });
  if (f == items->end()) { salvage(); return; }
  const Partial part = *f;
  AcctEntry* ait = acct_.find(key);
  if (ait) {
    items->erase(f);
    output(server, svc, log_id, ait->acct, part.start_ms, false, ts, ts_empty, elapsed, false, seq);
    return;
  }
  need_map(key, log_id);
  std::string_view alt = baf_acct(e, line, tk.get(3), file, log_id, seq, baf_scratch);  // may drain the map first
  Need n{svc, part.server, part.start_ms, false, ts, ts_empty, elapsed,
         alt.empty() ? js::nan() : js::parse_int(alt), false};
  auto& ni = need_map(key, log_id).items;
  auto g = std::find_if(ni.begin(), ni.end(), [&](const Need& x) { return x.svc == svc; });
  if (g != ni.end()) *g = n; else ni.push_back(n);
  // map.delete(service)
  RecordEntry* it2 = record_.find(key);
  if (it2) {
    auto& v = it2->items;
    auto f2 = std::find_if(v.begin(), v.end(), [&](const Partial& p) { return p.svc == svc; });
    if (f2 != v.end()) v.erase(f2);
  }
}

// parseAppLine (:578-731) -- rare lines, kept simple
void JoinShard::on_app(const Event& e, std::string_view line, int32_t file, uint64_t seq) {
  const uint32_t m = e.mask;
  const int32_t server = (*files_)[file].server;
  if (m & PM_AUTR_MAP) {
    auto toks = js::split_ws(line, 8);
    std::string scratch;
    std::string log_id(strip_brackets(toks[0], scratch));
    std::string_view t5 = toks.size() > 5 ? toks[5] : std::string_view();
    size_t eq = t5.find('=');
    std::string autr;
    if (eq != std::string_view::npos) {
      size_t eq2 = t5.find('=', eq + 1);
      autr.assign(t5.substr(eq + 1, eq2 == std::string_view::npos ? std::string_view::npos : eq2 - eq - 1));
    } else {
      autr = "undefined";
    }
    AuditCtx& ctx = audit_[file];
    std::string baf_scratch;
    std::string alt(baf_acct(e, line, toks.size() > 3 ? toks[3] : std::string_view(), file, log_id, seq, baf_scratch));
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
      std::string scratch;
      elapsed.assign(strip_brackets(st[0], scratch));
      for (char& ch : elapsed) (void)ch;
      // strip_brackets keeps inner-only views; make sure *all* brackets are gone
      elapsed.erase(std::remove_if(elapsed.begin(), elapsed.end(), [](char c) { return c == '[' || c == ']'; }), elapsed.end());
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
  const std::string& svcname = ctx.active_service;
  auto f = std::find_if(ctx.service_map.begin(), ctx.service_map.end(), [&](auto& p) { return p.first == svcname; });
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
    const bool to_db = !icontains(svcname, "Provider[");
    double s_ms = js::nan(), e_ms = js::nan();
    bool s_empty = !obj.has_start || !js::convert_date(obj.start_ts, cfg_.tz, s_ms);
    bool e_empty = !js::convert_date(end_ts, cfg_.tz, e_ms);
    const double elapsed = js::parse_int(obj.elapsed);
    const int32_t svc = raw_service(svcname);
    const uint64_t key = key_of(log_id);
    AcctEntry* ait = acct_.find(key);
    if (ait) {
      output(server, svc, log_id, ait->acct, s_ms, s_empty, e_ms, e_empty, elapsed, to_db, seq);
    } else {
      const double alt = ctx.active_alt.empty() ? js::nan() : js::parse_int(ctx.active_alt);
      Need n{svc, server, s_ms, s_empty, e_ms, e_empty, elapsed, alt, to_db};
      auto& ni = need_map(key, log_id).items;
      auto g = std::find_if(ni.begin(), ni.end(), [&](const Need& x) { return x.svc == svc; });
      if (g != ni.end()) *g = n; else ni.push_back(n);
    }
  }
}

// Lookahead half of process(): the slots of the logId maps and the service map an EJB /
// CommonTiming event will probe, requested kLookahead events before the event is handled.
void JoinShard::prefetch_event(const Event& e, const uint8_t* bytes) {
  const uint8_t k = e.kind;
  if (k == LK_SOAP) {
    // A request line opens the SOAP context whose account line (a few lines later) writes
    // acct_[logId] and probes need_[logId]: two random misses that nothing else prefetches
    if ((e.mask & (PM_SOAP_IN | PM_HOST)) != PM_SOAP_IN || e.ntok < 2) return;
    const std::string_view t1((const char*)bytes + e.off + e.t1s, (size_t)(e.t1e - e.t1s));
    const size_t eq = t1.find('=');
    if (eq == std::string_view::npos) return;
    const size_t eq2 = t1.find('=', eq + 1);
    const uint64_t key = key_of(t1.substr(eq + 1, eq2 == std::string_view::npos ? std::string_view::npos : eq2 - eq - 1));
    acct_.prefetch(key);
    need_.prefetch(key);
    return;
  }
  if (k < LK_EJB_ENTRY || k > LK_CT_EXIT || (e.mask & PM_HOST) || e.ntok == 0) return;
  if (e.mask & PM_KEYS) {  // hashed on the GPU
    record_.prefetch(e.key);
    raw_svc_map_.prefetch(e.svc);
    if (k == LK_EJB_EXIT || k == LK_CT_EXIT) {
      acct_.prefetch(e.key);
      __builtin_prefetch(bytes + e.off + e.t0s);  // the logId is copied into the tx line
    }
    return;
  }
  const char* l = (const char*)bytes + e.off;
  const char* a = l + e.t0s;
  const char* b = l + e.t0e;
  if (a < b && *a == '[') ++a;
  if (b > a && b[-1] == ']') --b;
  const uint64_t key = key_of(std::string_view(a, (size_t)(b - a)));
  record_.prefetch(key);
  if (k == LK_EJB_EXIT || k == LK_CT_EXIT) acct_.prefetch(key);
  if (e.tAs != 0xffff)
    raw_svc_map_.prefetch(svc_hash(k <= LK_EJB_EXIT, std::string_view(l + e.tAs, (size_t)(e.tAe - e.tAs))));
}

void JoinShard::process(const Event* ev, size_t n, const uint8_t* bytes, const std::vector<int32_t>& chunk_file) {
  constexpr size_t kLookahead = 10;
  out_.reserve(out_.size() + n / 2);
  for (size_t i = 0; i < n && i < kLookahead; ++i) prefetch_event(ev[i], bytes);
  for (size_t i = 0; i < n; ++i) {
    if (i + kLookahead < n) prefetch_event(ev[i + kLookahead], bytes);
    const Event& e = ev[i];
    ++counters.events;
    if (e.mask & PM_HOST) ++counters.host_fallback;
    const int32_t file = chunk_file[e.chunk];
    std::string_view line((const char*)bytes + e.off, e.len);
    const uint64_t seq = (1ULL << 51) | e.line;  // << 12 in output(): bit 63 marks line emissions
    cur_line_ = e.line;
    sub_ = 0;
#ifdef APM_JOIN_PROF
    const uint64_t t0 = __rdtsc();
#endif
#ifndef APM_JOIN_NOOP
    switch (e.kind) {
      case LK_SOAP: on_soap(e, line, file, seq); break;
      case LK_EJB_ENTRY: on_ejb(e, line, file, true, seq); break;
      case LK_EJB_EXIT: on_ejb(e, line, file, false, seq); break;
      case LK_CT_ENTRY: on_ct(e, line, file, true, seq); break;
      case LK_CT_EXIT: on_ct(e, line, file, false, seq); break;
      case LK_APP: on_app(e, line, file, seq); break;
      default: break;
    }
#endif
#ifdef APM_JOIN_PROF
    prof_cyc[e.kind & 15] += __rdtsc() - t0;
    prof_n[e.kind & 15]++;
#endif
  }
}

}  // namespace apm
