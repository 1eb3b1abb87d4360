// Re-shard merge of engine checkpoints on the host (see merge.h for what and why).
//
// Every input is read section by section in the layout Engine::write_small_sections /
// DeviceJoin::save / the ring writers produce (checkpoint.cpp, devjoin.cpp); the merged state is
// renumbered into the new rank's ids and written as one full checkpoint in the same layout.
#include "merge.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string_view>
#include <unordered_map>

#include "../apm_types.h"
#include "../kernels/devjoin_types.h"
#include "binio.h"
#include "engine.h"

namespace apm {

namespace {

struct SeriesRec { int32_t server, service; uint64_t emit_key; };  // checkpoint.cpp SEC_SERIES
struct I64Pair { int64_t a, b; };
struct RawRec { int32_t server; int32_t norm_id; uint64_t svc; };  // DeviceJoin::RawInfo
struct Region { uint64_t lo, hi; double exp; };
struct Blk { uint8_t b[CHAIN_BLK]; };
struct FileRec { std::string path; int32_t server; uint8_t kind; };
struct SlotRec { std::vector<int32_t> counts, packed; int32_t spill_n = 0; std::vector<int32_t> sp_series, sp_val; };
struct LagRec {
  std::vector<int32_t> len, counter;
  std::vector<double> sum, comp, sumsq, sqcomp;  // [NSTAT][n]
  std::vector<int32_t> cnt;                       // [NSTAT][n]
};

std::string dir_of(const std::string& path) {
  const size_t slash = path.rfind('/');
  return slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
}

bool is_manifest(const std::string& path) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) throw std::runtime_error("merge: cannot open " + path);
  char m[8] = {0};
  const size_t got = std::fread(m, 1, 8, f);
  std::fclose(f);
  return got == 8 && std::memcmp(m, "APMCHAIN", 8) == 0;
}

std::vector<std::string> chain_files(const std::string& path) {
  if (!is_manifest(path)) return {path};
  FILE* f = std::fopen(path.c_str(), "rb");
  std::vector<std::string> out;
  char line[4096];
  bool first = true;
  while (std::fgets(line, sizeof line, f)) {
    std::string l(line);
    while (!l.empty() && (l.back() == '\n' || l.back() == '\r')) l.pop_back();
    if (first) { first = false; continue; }
    if (!l.empty()) out.push_back(dir_of(path) + "/" + l);
  }
  std::fclose(f);
  if (out.empty()) throw std::runtime_error("merge: empty chain manifest " + path);
  return out;
}

uint64_t file_batch(const std::string& f) {
  BinReader rd(f);
  rd.skip_to(SEC_CLOCK);
  rd.pod<double>();
  return rd.pod<uint64_t>();
}

// One old rank's state at the chosen batch: the small sections of that chain file, parsed.
struct Input {
  std::vector<std::string> chain;  // base .. the chosen file
  // config
  int32_t max_series = 0, cell_cap = 0, spill_cap = 0, window = 0, buffer = 0;
  int n_lags = 0, ring_bytes = 0;
  int32_t lags[MAX_LAGS] = {};
  int64_t pool_cap = 0;
  // topology
  std::vector<std::string> servers, services;
  std::vector<FileRec> files;
  // series
  std::vector<SeriesRec> sr;
  std::vector<int32_t> server_rank, server_next_service, server_gidx;
  int32_t next_server_rank = 0;
  std::vector<int64_t> server_first_batch;
  std::vector<double> thr, infl, hard_max;
  std::vector<uint8_t> suppressed;
  std::vector<uint64_t> emit_key;
  std::vector<int32_t> zscore_seen;
  std::vector<uint8_t> active_h;
  std::vector<int32_t> unseen;
  double alias_thr[MAX_LAGS] = {}, alias_infl[MAX_LAGS] = {};
  // clock
  double watermark = 0;
  uint64_t batch_no = 0;
  int64_t latest = 0, rollover_idx = 0, next_gid = 0;
  std::vector<int64_t> slot_bucket;  // the saver's ring (its slot count)
  uint32_t line_block_seq = 0;
  // join
  JoinCounts jc{};
  uint64_t jcount[7] = {};
  std::vector<KeyState> keys;
  uint32_t arena_cap = 0;
  uint64_t arena_head = 0;
  std::vector<Region> regions;
  std::vector<NeedEnt> ents;
  std::vector<Blk> blocks;
  std::vector<SoapState> soap;
  std::vector<RawRec> raw;
  std::vector<int32_t> raw_top;
  std::vector<AudCarry> carry;
  std::vector<AutrEnt> autr;
  std::vector<AudItem> items;
  std::string aud_txt;
  std::vector<int32_t> raw_series;
  // parse
  std::vector<uint8_t> file_open;
  // buckets
  std::vector<uint8_t> active_d;
  std::map<int32_t, SlotRec> slots;
  std::vector<int32_t> nan_until;
  // z-score
  std::vector<LagRec> lag;
  // pool
  std::vector<I64Pair> bucket_count, exact_edge;
  std::vector<int64_t> pool_end, tail_end, gids;
  std::string pend_text;
  // alerts / outputs / metrics
  std::vector<std::pair<std::string, double>> cool;
  std::string blob[N_OUT];
  uint64_t metrics[11] = {};
  std::string extra;
  int64_t n() const { return (int64_t)sr.size(); }
};

void read_small(Input& in, const std::string& path) {
  BinReader rd(path);
  rd.begin(SEC_CONFIG);
  rd.pod(in.max_series); rd.pod(in.n_lags); rd.raw(in.lags, sizeof(in.lags)); rd.pod(in.ring_bytes);
  rd.pod(in.cell_cap); rd.pod(in.spill_cap); rd.pod(in.pool_cap); rd.pod(in.window); rd.pod(in.buffer);

  rd.begin(SEC_TOPOLOGY);
  in.servers = rd.strs();
  for (uint64_t nf = rd.pod<uint64_t>(); nf; --nf) {
    FileRec f;
    f.path = rd.str();
    rd.pod(f.server);
    rd.pod(f.kind);
    in.files.push_back(f);
  }
  in.services = rd.strs();

  rd.begin(SEC_SERIES);
  in.sr = rd.vec<SeriesRec>();
  in.server_rank = rd.vec<int32_t>();
  in.server_next_service = rd.vec<int32_t>();
  rd.pod(in.next_server_rank);
  in.server_gidx = rd.vec<int32_t>();
  in.server_first_batch = rd.vec<int64_t>();
  in.thr = rd.vec<double>(); in.infl = rd.vec<double>(); in.hard_max = rd.vec<double>();
  in.suppressed = rd.vec<uint8_t>(); in.emit_key = rd.vec<uint64_t>();
  in.zscore_seen = rd.vec<int32_t>(); in.active_h = rd.vec<uint8_t>(); in.unseen = rd.vec<int32_t>();
  rd.raw(in.alias_thr, sizeof(in.alias_thr)); rd.raw(in.alias_infl, sizeof(in.alias_infl));
  const int64_t n = in.n();

  rd.begin(SEC_CLOCK);
  rd.pod(in.watermark); rd.pod(in.batch_no); rd.pod(in.latest); rd.pod(in.rollover_idx);
  in.slot_bucket = rd.vec<int64_t>();
  rd.pod(in.next_gid); rd.pod(in.line_block_seq);

  rd.begin(SEC_JOIN);
  if (rd.pod<uint8_t>() != 1) throw std::runtime_error("merge: re-shard needs gpu.joinOnDevice checkpoints");
  rd.pod(in.jc);
  for (auto& v : in.jcount) rd.pod(v);
  in.keys = rd.vec<KeyState>();
  rd.pod(in.arena_cap);
  rd.pod(in.arena_head);
  for (uint64_t k = rd.pod<uint64_t>(); k; --k) {
    Region r;
    rd.pod(r.lo); rd.pod(r.hi); rd.pod(r.exp);
    in.regions.push_back(r);
  }
  in.ents = rd.vec<NeedEnt>();
  in.blocks = rd.vec<Blk>();
  in.soap = rd.vec<SoapState>();
  in.raw = rd.vec<RawRec>();
  in.raw_top = rd.vec<int32_t>();
  in.carry = rd.vec<AudCarry>();
  in.autr = rd.vec<AutrEnt>();
  in.items = rd.vec<AudItem>();
  in.aud_txt = rd.str();
  in.raw_series = rd.vec<int32_t>();

  rd.begin(SEC_PARSE);
  in.file_open = rd.vec<uint8_t>();

  rd.begin(SEC_BUCKETS);
  in.active_d = rd.vec<uint8_t>();
  for (;;) {
    const int32_t slot = rd.pod<int32_t>();
    if (slot < 0) break;
    SlotRec& s = in.slots[slot];
    s.counts = rd.vec<int32_t>();
    s.packed = rd.vec<int32_t>();
    rd.pod(s.spill_n);
    s.sp_series = rd.vec<int32_t>();
    s.sp_val = rd.vec<int32_t>();
  }
  in.nan_until = rd.vec<int32_t>();

  rd.begin(SEC_ZSCORE);
  in.lag.resize((size_t)in.n_lags);
  for (auto& L : in.lag) {
    L.len = rd.vec<int32_t>();
    L.counter = rd.vec<int32_t>();
    for (std::vector<double>* a : {&L.sum, &L.comp, &L.sumsq, &L.sqcomp}) {
      a->resize((size_t)NSTAT * n);
      rd.raw(a->data(), a->size() * 8);
    }
    L.cnt.resize((size_t)NSTAT * n);
    rd.raw(L.cnt.data(), L.cnt.size() * 4);
  }

  rd.begin(SEC_POOL);
  {
    int64_t off, pn, tn;
    rd.pod(off); rd.pod(pn); rd.pod(tn);
    in.bucket_count = rd.vec<I64Pair>();
    in.exact_edge = rd.vec<I64Pair>();
    in.pool_end = rd.vec<int64_t>();
    rd.vec<int64_t>();  // ring positions of the saving engine (the rebased gids below replace them)
    in.tail_end = rd.vec<int64_t>();
    in.gids = rd.vec<int64_t>();
    in.pend_text.resize(rd.pod<uint64_t>());
    rd.raw(&in.pend_text[0], in.pend_text.size());
    if ((int64_t)in.pool_end.size() != pn || (int64_t)in.tail_end.size() != tn ||
        (int64_t)in.gids.size() != pn + tn)
      throw std::runtime_error("merge: pool section sizes differ");
  }

  rd.begin(SEC_ALERTS);
  for (uint64_t k = rd.pod<uint64_t>(); k; --k) {
    std::string key = rd.str();
    in.cool.emplace_back(std::move(key), rd.pod<double>());
  }
  rd.begin(SEC_OUTPUTS);
  for (auto& b : in.blob) b = rd.str();
  rd.begin(SEC_METRICS);
  for (auto& v : in.metrics) rd.pod(v);
  rd.skip_to(SEC_EXTRA);
  in.extra = rd.str();
}

// The rings of one LAG as the chain has them: the base's rows overwritten by every increment's
// dirty rows, in order.  [NSTAT][L][n] of `rb`-byte elements (n: the chosen file's series).
std::vector<char> read_ring(const Input& in, int l, size_t rb) {
  const int32_t L = in.lags[l];
  const size_t n = (size_t)in.n();
  std::vector<char> ring((size_t)NSTAT * L * n * rb, 0);
  std::vector<char> row;
  for (const auto& f : in.chain) {
    BinReader rd(f);
    rd.skip_to(SEC_RING);
    for (int q = 0; q < in.n_lags; ++q) {
      int32_t nc = rd.pod<int32_t>();
      const bool row_major = nc < 0;  // a streamed snapshot (checkpoint.cpp write_streamed_ring)
      if (row_major) nc = -nc - 1;
      const std::vector<int32_t> heads = rd.vec<int32_t>();
      if ((size_t)nc > n) throw std::runtime_error("merge: ring rows wider than the series table");
      const size_t w = (size_t)nc * rb;
      if (q != l) {
        rd.skip((uint64_t)NSTAT * heads.size() * w);
        continue;
      }
      row.resize(w);
      if (row_major) {
        for (int32_t h : heads) {
          if (h < 0 || h >= L) throw std::runtime_error("merge: bad ring row");
          for (int k = 0; k < NSTAT; ++k) {
            rd.raw(row.data(), w);
            std::memcpy(ring.data() + ((size_t)k * L + (size_t)h) * n * rb, row.data(), w);
          }
        }
        continue;
      }
      for (int k = 0; k < NSTAT; ++k)
        for (int32_t h : heads) {  // (runs of consecutive rows are contiguous: row order is file order)
          if (h < 0 || h >= L) throw std::runtime_error("merge: bad ring row");
          rd.raw(row.data(), w);
          std::memcpy(ring.data() + ((size_t)k * L + (size_t)h) * n * rb, row.data(), w);
        }
    }
  }
  return ring;
}

int32_t server_of_line(const std::string& text, uint64_t gid, const std::unordered_map<std::string, int32_t>& srv) {
  const uint64_t off = gid >> 20, len = gid & 0xfffffu;
  if (off + len > text.size()) throw std::runtime_error("merge: pending line outside the text");
  const std::string_view ln(text.data() + off, len);
  const size_t a = ln.find('|');
  if (a == std::string_view::npos) return -1;
  const size_t b = ln.find('|', a + 1);
  const std::string s(ln.substr(a + 1, b == std::string_view::npos ? std::string_view::npos : b - a - 1));
  auto it = srv.find(s);
  return it == srv.end() ? -1 : it->second;
}

uint64_t pow2_at_least(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

}  // namespace

std::vector<std::pair<uint64_t, std::string>> checkpoint_batches(const std::string& path) {
  std::vector<std::pair<uint64_t, std::string>> out;
  for (const auto& f : chain_files(path)) out.emplace_back(file_batch(f), f);
  return out;
}

MergeResult merge_checkpoints(const std::vector<std::string>& inputs, const std::vector<std::string>& keep_servers,
                              const std::string& out_path, const std::string& extra, uint64_t batch_no) {
  if (inputs.empty()) throw std::runtime_error("merge: no input checkpoints");
  // ---- the common batch and each input's chain prefix ending at it
  std::vector<std::vector<std::pair<uint64_t, std::string>>> chains;
  for (const auto& p : inputs) chains.push_back(checkpoint_batches(p));
  if (batch_no == 0) {
    std::map<uint64_t, int> seen;
    for (const auto& c : chains) {
      std::vector<uint64_t> b;
      for (const auto& x : c) b.push_back(x.first);
      std::sort(b.begin(), b.end());
      b.erase(std::unique(b.begin(), b.end()), b.end());
      for (uint64_t v : b) ++seen[v];
    }
    for (auto it = seen.rbegin(); it != seen.rend(); ++it)
      if (it->second == (int)chains.size()) { batch_no = it->first; break; }
    if (batch_no == 0) throw std::runtime_error("merge: the input checkpoints share no batch");
  }
  std::vector<Input> in(inputs.size());
  MergeResult res;
  res.batch_no = batch_no;
  for (size_t j = 0; j < inputs.size(); ++j) {
    const auto& c = chains[j];
    size_t last = c.size();
    for (size_t i = 0; i < c.size(); ++i)
      if (c[i].first == batch_no) last = i;
    if (last == c.size())
      throw std::runtime_error("merge: " + inputs[j] + " has no checkpoint at batch " + std::to_string(batch_no));
    for (size_t i = 0; i <= last; ++i) in[j].chain.push_back(c[i].second);
    read_small(in[j], c[last].second);
    res.used.push_back(c[last].second);
    res.extras.push_back(in[j].extra);
  }
  const Input& I0 = in[0];
  for (const Input& x : in) {
    if (x.n_lags != I0.n_lags || std::memcmp(x.lags, I0.lags, sizeof(x.lags)) != 0 || x.ring_bytes != I0.ring_bytes ||
        x.cell_cap != I0.cell_cap || x.window != I0.window || x.buffer != I0.buffer)
      throw std::runtime_error("merge: the input checkpoints were written with different configurations");
    if (x.batch_no != I0.batch_no || x.latest != I0.latest || x.rollover_idx != I0.rollover_idx ||
        x.slot_bucket != I0.slot_bucket)
      throw std::runtime_error("merge: the inputs are not one lock-step batch (clocks / bucket slots differ)");
  }
  const size_t rb = (size_t)I0.ring_bytes;
  const int n_lags = I0.n_lags;

  // ---- topology: kept servers (input order), their files, the union of the service names
  std::unordered_map<std::string, int32_t> keep;
  for (const auto& s : keep_servers) keep.emplace(s, -1);
  std::vector<std::string> servers, services;
  std::vector<FileRec> files;
  std::unordered_map<std::string, int32_t> svc_id;
  std::vector<std::vector<int32_t>> smap(in.size()), fmap(in.size()), vmap(in.size());
  for (size_t j = 0; j < in.size(); ++j) {
    for (const auto& s : in[j].servers) {
      auto it = keep.find(s);
      int32_t id = -1;
      if (it != keep.end()) {
        if (it->second < 0) { it->second = (int32_t)servers.size(); servers.push_back(s); }
        id = it->second;
      }
      smap[j].push_back(id);
    }
    for (const auto& f : in[j].files) {
      const int32_t ns = smap[j].at((size_t)f.server);
      if (ns < 0) { fmap[j].push_back(-1); continue; }
      fmap[j].push_back((int32_t)files.size());
      files.push_back(FileRec{f.path, ns, f.kind});
    }
    for (const auto& v : in[j].services) {
      auto it = svc_id.find(v);
      if (it == svc_id.end()) { it = svc_id.emplace(v, (int32_t)services.size()).first; services.push_back(v); }
      vmap[j].push_back(it->second);
    }
  }
  if (files.size() > (1u << 16)) throw std::runtime_error("merge: too many files");
  // inputs holding at least one of the kept servers (the others contribute nothing)
  std::vector<char> contrib(in.size(), 0);
  for (size_t j = 0; j < in.size(); ++j)
    for (int32_t ns : smap[j]) contrib[j] |= ns >= 0;
  res.servers = (int64_t)servers.size();
  res.files = (int64_t)files.size();

  // ---- series (input order), server emission ranks re-drawn in first-appearance order
  std::vector<std::vector<int32_t>> ser(in.size());
  std::vector<SeriesRec> sr;
  const size_t NS = servers.size();
  std::vector<int32_t> server_rank(NS, -1), server_next(NS, 0), server_gidx(NS, 0);
  std::vector<int64_t> server_first(NS, -1);
  for (size_t j = 0; j < in.size(); ++j)
    for (size_t s = 0; s < in[j].servers.size(); ++s) {
      const int32_t ns = smap[j][s];
      if (ns < 0) continue;
      server_next[ns] = in[j].server_next_service.at(s);
      server_gidx[ns] = in[j].server_gidx.at(s);
      server_first[ns] = in[j].server_first_batch.at(s);
    }
  {
    struct R { int64_t first; size_t j; int32_t old_rank; int32_t ns; };
    std::vector<R> ranked;
    for (size_t j = 0; j < in.size(); ++j)
      for (size_t s = 0; s < in[j].servers.size(); ++s)
        if (smap[j][s] >= 0 && in[j].server_rank.at(s) >= 0)
          ranked.push_back(R{in[j].server_first_batch.at(s), j, in[j].server_rank.at(s), smap[j][s]});
    std::sort(ranked.begin(), ranked.end(), [](const R& a, const R& b) {
      return a.first != b.first ? a.first < b.first : (a.j != b.j ? a.j < b.j : a.old_rank < b.old_rank);
    });
    for (size_t r = 0; r < ranked.size(); ++r) server_rank[ranked[r].ns] = (int32_t)r;
  }
  std::vector<double> thr, infl, hard_max;
  std::vector<uint8_t> suppressed, active_h, active_d;
  std::vector<uint64_t> emit_key;
  std::vector<int32_t> zscore_seen, unseen, nan_until;
  for (size_t j = 0; j < in.size(); ++j) {
    const Input& x = in[j];
    ser[j].assign((size_t)x.n(), -1);
    for (int64_t s = 0; s < x.n(); ++s) {
      const int32_t ns = smap[j][(size_t)x.sr[s].server];
      if (ns < 0) continue;
      ser[j][s] = (int32_t)sr.size();
      const uint64_t ek = ((uint64_t)server_rank[ns] << 24) | (x.sr[s].emit_key & 0xFFFFFFull);
      sr.push_back(SeriesRec{ns, vmap[j].at((size_t)x.sr[s].service), ek});
      thr.insert(thr.end(), x.thr.begin() + s * MAX_LAGS, x.thr.begin() + (s + 1) * MAX_LAGS);
      infl.insert(infl.end(), x.infl.begin() + s * MAX_LAGS, x.infl.begin() + (s + 1) * MAX_LAGS);
      hard_max.push_back(x.hard_max[s]);
      suppressed.push_back(x.suppressed[s]);
      emit_key.push_back(ek);
      zscore_seen.push_back(x.zscore_seen[s]);
      active_h.push_back(x.active_h[s]);
      active_d.push_back(x.active_d.at((size_t)s));
      nan_until.push_back(x.nan_until.at((size_t)s));
    }
    for (int32_t s : x.unseen)
      if (ser[j].at((size_t)s) >= 0) unseen.push_back(ser[j][s]);
  }
  const int64_t N = (int64_t)sr.size();
  if (N > I0.max_series)  // (every input shares one config, so its maxSeries holds the merged table)
    throw std::runtime_error("merge: " + std::to_string(N) + " merged series exceed gpu.maxSeries " +
                             std::to_string(I0.max_series));
  res.series = N;
  auto per_series = [&](auto getter, auto& out) {  // concat of the kept columns of an [n] array
    for (size_t j = 0; j < in.size(); ++j) {
      const auto& v = getter(in[j]);
      for (int64_t s = 0; s < in[j].n(); ++s)
        if (ser[j][s] >= 0) out.push_back(v.at((size_t)s));
    }
  };

  // ---- raw service registry
  std::vector<std::vector<int32_t>> rmap(in.size());
  std::vector<RawRec> raw;
  std::vector<int32_t> raw_top, raw_series;
  for (size_t j = 0; j < in.size(); ++j)
    for (size_t r = 0; r < in[j].raw.size(); ++r) {
      const RawRec& x = in[j].raw[r];
      const int32_t ns = smap[j].at((size_t)x.server);
      if (ns < 0) { rmap[j].push_back(-1); continue; }
      rmap[j].push_back((int32_t)raw.size());
      raw.push_back(RawRec{ns, vmap[j].at((size_t)x.norm_id), x.svc});
      raw_top.push_back(in[j].raw_top.at(r));
      const int32_t os = r < in[j].raw_series.size() ? in[j].raw_series[r] : -1;
      raw_series.push_back(os >= 0 ? ser[j].at((size_t)os) : -1);
    }
  res.raw = (int64_t)raw.size();

  // ---- join: need arena (regions re-laid out by expiry), chain blocks, key table
  std::vector<Blk> blocks;
  std::vector<int32_t> blk_base(in.size(), 0);
  for (size_t j = 0; j < in.size(); ++j) {
    blk_base[j] = (int32_t)blocks.size();
    for (Blk b : in[j].blocks) {
      int32_t next;
      std::memcpy(&next, b.b, 4);
      if (next) next += blk_base[j];
      std::memcpy(b.b, &next, 4);
      blocks.push_back(b);
    }
  }
  auto shift_blk = [](int32_t v, int32_t base) { return v ? v + base : 0; };
  std::vector<std::vector<uint64_t>> newv(in.size());  // entry index -> new virtual index
  std::vector<NeedEnt> ents;
  std::vector<Region> regions;
  {
    struct RR { double exp; size_t j; size_t r; };
    std::vector<RR> order;
    for (size_t j = 0; j < in.size(); ++j) {
      newv[j].assign(in[j].ents.size(), 0);
      for (size_t r = 0; r < in[j].regions.size(); ++r) order.push_back(RR{in[j].regions[r].exp, j, r});
    }
    std::stable_sort(order.begin(), order.end(), [](const RR& a, const RR& b) {
      return a.exp != b.exp ? a.exp < b.exp : a.j < b.j;
    });
    uint64_t cur = 0;
    for (const RR& o : order) {
      const Input& x = in[o.j];
      const Region& g = x.regions[o.r];
      const uint64_t lo0 = x.regions.front().lo;
      const uint64_t start = cur;
      for (uint64_t v = g.lo; v < g.hi; ++v) {
        const size_t e = (size_t)(v - lo0);
        NeedEnt ne = x.ents.at(e);
        newv[o.j][e] = cur;
        ne.vidx = cur;
        // The expiry emits every entry of an expiring region that still holds records, whatever its
        // key (k_exp_keys / k_exp_emit), under the entry's server: an entry of a server this rank
        // does not own must hold nothing (else its records are emitted here too, under whatever
        // server its old id now names), and an empty one nothing to free.
        const int32_t ns = ne.key && ne.server >= 0 ? smap[o.j].at((size_t)ne.server) : -1;
        if (ns < 0) {
          ne.key = 0;  // not this rank's (or already gone): a dead slot (keeps the region contiguous)
          ne.n = 0;
          ne.iblk = ne.lblk = 0;
        } else {
          ne.server = ns;
          ne.iblk = shift_blk(ne.iblk, blk_base[o.j]);
          ne.lblk = shift_blk(ne.lblk, blk_base[o.j]);
          ++res.need;
        }
        ents.push_back(ne);
        ++cur;
      }
      regions.push_back(Region{start, cur, g.exp});
    }
  }
  uint32_t arena_cap = 0;
  for (const Input& x : in) arena_cap = std::max(arena_cap, x.arena_cap);
  arena_cap = (uint32_t)std::max<uint64_t>(arena_cap, pow2_at_least(ents.size() + 1));
  std::vector<KeyState> keys;
  for (size_t j = 0; j < in.size(); ++j) {
    const Input& x = in[j];
    const uint64_t lo = x.regions.empty() ? x.arena_head : x.regions.front().lo;
    const uint64_t cap = x.arena_cap;
    for (KeyState k : x.keys) {
      if (k.server < 0 || (size_t)k.server >= smap[j].size()) throw std::runtime_error("merge: key without a server");
      const int32_t ns = smap[j][(size_t)k.server];
      if (ns < 0) continue;
      k.server = ns;
      if (k.need >= 0) {
        // A link past the live range is stale (its region expired, or the slot was reused): the
        // join checks the entry's key and TTL before it follows a link (k_group_walk), so a stale
        // link is simply no link.  One inside the range keeps its entry (the key check still
        // applies after the move).
        const uint64_t e = ((uint64_t)k.need - (lo & (cap - 1))) & (cap - 1);  // entry index in [lo, head)
        k.need = e < newv[j].size() ? (int32_t)(newv[j][e] & (arena_cap - 1)) : -1;
      }
      k.pblk = shift_blk(k.pblk, blk_base[j]);
      keys.push_back(k);
    }
  }
  res.keys = (int64_t)keys.size();

  // ---- audit carry (per new file), SOAP contexts, parse carry
  std::vector<SoapState> soap(files.size());
  std::vector<AudCarry> carry(files.size());
  std::vector<AutrEnt> autr;
  std::vector<AudItem> items;
  std::string aud_txt;
  std::vector<uint8_t> file_open((size_t)1 << 16, 0);
  for (size_t j = 0; j < in.size(); ++j) {
    const Input& x = in[j];
    if (!contrib[j]) continue;
    const uint32_t tb = (uint32_t)aud_txt.size(), ib = (uint32_t)items.size();
    aud_txt += x.aud_txt;
    items.insert(items.end(), x.items.begin(), x.items.end());
    for (AutrEnt a : x.autr) { a.lid_off += tb; autr.push_back(a); }
    for (size_t f = 0; f < x.files.size(); ++f) {
      const int32_t nf = fmap[j][f];
      if (nf < 0) continue;
      if (f < x.soap.size()) soap[nf] = x.soap[f];
      if (f < x.carry.size()) {
        AudCarry c = x.carry[f];
        c.lid_off += tb;
        c.svc_off += tb;
        c.items_off += ib;
        carry[nf] = c;
      }
      if (f < x.file_open.size()) file_open[nf] = x.file_open[f];
    }
  }

  // ---- pending release lines: the owned servers', pool merged by endTs, tails concatenated
  std::unordered_map<std::string, int32_t> kept_srv;
  for (size_t i = 0; i < servers.size(); ++i) kept_srv.emplace(servers[i], (int32_t)i);
  std::vector<int64_t> pool_end, tail_end, gids;
  std::string pend_text;
  {
    struct P { int64_t end; size_t j; size_t i; };
    std::vector<P> pool, tail;
    for (size_t j = 0; j < in.size(); ++j) {
      const Input& x = in[j];
      for (size_t i = 0; i < x.pool_end.size(); ++i)
        if (server_of_line(x.pend_text, (uint64_t)x.gids[i], kept_srv) >= 0) pool.push_back(P{x.pool_end[i], j, i});
      for (size_t i = 0; i < x.tail_end.size(); ++i)
        if (server_of_line(x.pend_text, (uint64_t)x.gids[x.pool_end.size() + i], kept_srv) >= 0)
          tail.push_back(P{x.tail_end[i], j, x.pool_end.size() + i});
    }
    std::stable_sort(pool.begin(), pool.end(), [](const P& a, const P& b) { return a.end < b.end; });
    auto put = [&](const P& p) {
      const uint64_t g = (uint64_t)in[p.j].gids[p.i];
      const uint64_t off = g >> 20, len = g & 0xfffffu;
      gids.push_back((int64_t)(((uint64_t)pend_text.size() << 20) | len));
      pend_text.append(in[p.j].pend_text, off, len);
      pend_text.push_back('\n');
    };
    for (const P& p : pool) { pool_end.push_back(p.end); put(p); }
    for (const P& p : tail) { tail_end.push_back(p.end); put(p); }
    res.pending = (int64_t)gids.size();
  }

  // ---- write
  BinWriter w(out_path);
  int32_t spill_cap = 0;
  {
    std::map<int32_t, int64_t> need;
    for (size_t j = 0; j < in.size(); ++j) {
      spill_cap = std::max(spill_cap, in[j].spill_cap);
      for (const auto& kv : in[j].slots) need[kv.first] += (int64_t)kv.second.sp_series.size();
    }
    for (const auto& kv : need) spill_cap = (int32_t)std::max<int64_t>(spill_cap, kv.second);
  }
  w.begin(SEC_CONFIG);
  w.pod((int32_t)std::max<int64_t>(I0.max_series, N)); w.pod(I0.n_lags); w.raw(I0.lags, sizeof(I0.lags));
  w.pod(I0.ring_bytes); w.pod(I0.cell_cap); w.pod(spill_cap); w.pod(I0.pool_cap); w.pod(I0.window); w.pod(I0.buffer);
  w.end();

  w.begin(SEC_TOPOLOGY);
  w.strs(servers);
  w.pod<uint64_t>(files.size());
  for (const auto& f : files) { w.str(f.path); w.pod(f.server); w.pod(f.kind); }
  w.strs(services);
  w.end();

  w.begin(SEC_SERIES);
  w.vec(sr);
  w.vec(server_rank); w.vec(server_next);
  int32_t next_rank = 0;
  for (int32_t r : server_rank) next_rank = std::max(next_rank, r + 1);
  w.pod(next_rank);
  w.vec(server_gidx); w.vec(server_first);
  w.vec(thr); w.vec(infl); w.vec(hard_max); w.vec(suppressed); w.vec(emit_key);
  w.vec(zscore_seen); w.vec(active_h); w.vec(unseen);
  w.raw(I0.alias_thr, sizeof(I0.alias_thr)); w.raw(I0.alias_infl, sizeof(I0.alias_infl));
  w.end();

  w.begin(SEC_CLOCK);
  {
    double wm = I0.watermark;
    int64_t ng = I0.next_gid;
    uint32_t lbs = I0.line_block_seq;
    for (const Input& x : in) { wm = std::max(wm, x.watermark); ng = std::max(ng, x.next_gid); lbs = std::max(lbs, x.line_block_seq); }
    w.pod(wm); w.pod(I0.batch_no); w.pod(I0.latest); w.pod(I0.rollover_idx);
    w.vec(I0.slot_bucket);
    w.pod(ng); w.pod(lbs);
  }
  w.end();

  w.begin(SEC_JOIN);
  w.pod<uint8_t>(1);
  {
    size_t j0 = 0;
    while (j0 + 1 < in.size() && !contrib[j0]) ++j0;
    JoinCounts c = in[j0].jc;
    for (size_t j = j0 + 1; j < in.size(); ++j) {
      if (!contrib[j]) continue;
      const JoinCounts& d = in[j].jc;
      c.ejb_unmatched += d.ejb_unmatched; c.partial_overflow += d.partial_overflow; c.need_overflow += d.need_overflow;
      c.expired_partials += d.expired_partials; c.need_expired += d.need_expired; c.invalid_acct += d.invalid_acct;
      c.table_full += d.table_full; c.key_probe_max = std::max(c.key_probe_max, d.key_probe_max);
      c.audit_errors += d.audit_errors;
      c.chain_parts += d.chain_parts; c.chain_items += d.chain_items; c.chain_lids += d.chain_lids;
    }
    w.pod(c);
    for (int k = 0; k < 7; ++k) {
      uint64_t s = 0;
      for (size_t j = 0; j < in.size(); ++j) s += contrib[j] ? in[j].jcount[k] : 0;
      w.pod(s);
    }
  }
  w.vec(keys);
  w.pod(arena_cap);
  w.pod<uint64_t>(ents.size());  // arena head (virtual): the entries are laid out from 0
  w.pod<uint64_t>(regions.size());
  for (const Region& r : regions) { w.pod(r.lo); w.pod(r.hi); w.pod(r.exp); }
  w.vec(ents);
  w.vec(blocks);
  w.vec(soap);
  w.vec(raw);
  w.vec(raw_top);
  w.vec(carry);
  w.vec(autr);
  w.vec(items);
  w.str(aud_txt);
  w.vec(raw_series);
  w.end();

  w.begin(SEC_PARSE);
  w.vec(file_open);
  w.end();

  w.begin(SEC_BUCKETS);
  w.vec(active_d);
  {
    std::map<int32_t, int> live;
    for (const Input& x : in)
      for (const auto& kv : x.slots) live[kv.first] = 1;
    for (const auto& kv : live) {
      const int32_t slot = kv.first;
      std::vector<int32_t> counts, packed, sp_series, sp_val;
      for (size_t j = 0; j < in.size(); ++j) {
        const Input& x = in[j];
        auto it = x.slots.find(slot);
        const SlotRec* s = it == x.slots.end() ? nullptr : &it->second;
        size_t p = 0;
        for (int64_t q = 0; q < x.n(); ++q) {
          const int32_t c = s ? s->counts.at((size_t)q) : 0;
          const int32_t m = std::max(0, std::min(c, x.cell_cap));
          if (ser[j][q] >= 0) {
            counts.push_back(c);
            if (s && m > 0)
              packed.insert(packed.end(), s->packed.begin() + (ptrdiff_t)p, s->packed.begin() + (ptrdiff_t)(p + m));
          }
          p += (size_t)m;
        }
        if (s)
          for (size_t i = 0; i < s->sp_series.size(); ++i) {
            const int32_t os = s->sp_series[i];
            if (os >= 0 && os < x.n() && ser[j][os] >= 0) { sp_series.push_back(ser[j][os]); sp_val.push_back(s->sp_val[i]); }
          }
      }
      w.pod<int32_t>(slot);
      w.vec(counts);
      w.vec(packed);
      w.pod<int32_t>((int32_t)sp_series.size());
      w.vec(sp_series);
      w.vec(sp_val);
    }
    w.pod<int32_t>(-1);
  }
  w.vec(nan_until);
  w.end();

  w.begin(SEC_ZSCORE);
  for (int l = 0; l < n_lags; ++l) {
    std::vector<int32_t> len, counter;
    per_series([&](const Input& x) -> const std::vector<int32_t>& { return x.lag[l].len; }, len);
    per_series([&](const Input& x) -> const std::vector<int32_t>& { return x.lag[l].counter; }, counter);
    w.vec(len);
    w.vec(counter);
    auto rows = [&](auto member, size_t esz) {  // [NSTAT][N]
      for (int k = 0; k < NSTAT; ++k)
        for (size_t j = 0; j < in.size(); ++j) {
          const auto& v = in[j].lag[l].*member;
          const int64_t n = in[j].n();
          for (int64_t s = 0; s < n; ++s)
            if (ser[j][s] >= 0) w.raw(&v[(size_t)k * n + s], esz);
        }
    };
    rows(&LagRec::sum, 8); rows(&LagRec::comp, 8); rows(&LagRec::sumsq, 8); rows(&LagRec::sqcomp, 8);
    rows(&LagRec::cnt, 4);
  }
  w.end();

  w.begin(SEC_POOL);
  w.pod<int64_t>(0); w.pod<int64_t>((int64_t)pool_end.size()); w.pod<int64_t>((int64_t)tail_end.size());
  {
    std::map<int64_t, int64_t> bc, ee;  // (host-join release accounting; unused by the device join)
    for (const Input& x : in) {
      for (const auto& p : x.bucket_count) bc[p.a] += p.b;
      for (const auto& p : x.exact_edge) ee[p.a] += p.b;
    }
    std::vector<I64Pair> vb, ve;
    for (auto& kv : bc) vb.push_back({kv.first, kv.second});
    for (auto& kv : ee) ve.push_back({kv.first, kv.second});
    w.vec(vb);
    w.vec(ve);
  }
  w.vec(pool_end);
  w.vec(std::vector<int64_t>(gids.begin(), gids.begin() + (ptrdiff_t)pool_end.size()));
  w.vec(tail_end);
  w.vec(gids);
  w.pod<uint64_t>(pend_text.size());
  w.raw(pend_text.data(), pend_text.size());
  w.end();

  w.begin(SEC_ALERTS);
  {
    std::map<std::string, double> cool;
    for (const Input& x : in)
      for (const auto& kv : x.cool) {
        auto it = cool.find(kv.first);
        if (it == cool.end() || kv.second > it->second) cool[kv.first] = kv.second;
      }
    w.pod<uint64_t>(cool.size());
    for (const auto& kv : cool) { w.str(kv.first); w.pod(kv.second); }
  }
  w.end();

  // undelivered output: the lines of the kept servers (the server field of each record type);
  // fb rows (node-wide, no server) from the inputs whose first server this rank keeps
  w.begin(SEC_OUTPUTS);
  for (int k = 0; k < N_OUT; ++k) {
    const int field = (k == OUT_TRANSACTIONS || k == OUT_AUDIT_DB || k == OUT_DB) ? 1
                    : (k == OUT_ST || k == OUT_FS || k == OUT_SX) ? 2 : (k == OUT_AL ? 3 : -1);
    std::string b;
    for (size_t j = 0; j < in.size(); ++j) {
      const std::string& src = in[j].blob[k];
      if (field < 0) {
        if (!smap[j].empty() && smap[j][0] >= 0) b += src;
        continue;
      }
      for (size_t a = 0; a < src.size();) {
        size_t e = src.find('\n', a);
        e = e == std::string::npos ? src.size() : e + 1;
        const std::string_view ln(src.data() + a, e - a);
        size_t p = 0;
        for (int f = 0; f < field && p != std::string_view::npos; ++f) {
          p = ln.find('|', p);
          if (p != std::string_view::npos) ++p;
        }
        if (p != std::string_view::npos) {
          size_t q = ln.find('|', p);
          if (q == std::string_view::npos) q = ln.size();
          if (kept_srv.count(std::string(ln.substr(p, q - p)))) b.append(ln.data(), ln.size());
        } else if (!smap[j].empty() && smap[j][0] >= 0) {
          b.append(ln.data(), ln.size());  // (not a wire line, e.g. COPY text: the input's first owner)
        }
        a = e;
      }
    }
    w.str(b);
  }
  w.end();

  w.begin(SEC_METRICS);
  for (int k = 0; k < 11; ++k) {
    uint64_t s = 0;
    for (size_t j = 0; j < in.size(); ++j) s += contrib[j] ? in[j].metrics[k] : 0;
    w.pod(s);
  }
  w.end();

  // rings: every row of every LAG, the kept columns of each input side by side
  w.begin(SEC_RING);
  for (int l = 0; l < n_lags; ++l) {
    const int32_t L = I0.lags[l];
    std::vector<std::vector<char>> rings;
    for (const Input& x : in) rings.push_back(read_ring(x, l, rb));
    w.pod<int32_t>((int32_t)N);
    std::vector<int32_t> heads((size_t)L);
    for (int32_t h = 0; h < L; ++h) heads[(size_t)h] = h;
    w.vec(heads);
    std::vector<char> row((size_t)N * rb);
    for (int k = 0; k < NSTAT; ++k)
      for (int32_t h = 0; h < L; ++h) {
        size_t o = 0;
        for (size_t j = 0; j < in.size(); ++j) {
          const int64_t n = in[j].n();
          const char* src = rings[j].data() + ((size_t)k * L + (size_t)h) * (size_t)n * rb;
          for (int64_t s = 0; s < n; ++s)
            if (ser[j][s] >= 0) { std::memcpy(row.data() + o, src + (size_t)s * rb, rb); o += rb; }
        }
        w.raw(row.data(), row.size());
      }
  }
  w.end();
  w.begin(SEC_EXTRA);
  w.str(extra);
  w.end();
  w.commit();
  return res;
}

}  // namespace apm
