// Launch-side API of the GPU join (devjoin.hip), used by runtime/devjoin.cpp.
#pragma once
#include <vector>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../apm_types.h"
#include "devjoin_types.h"

namespace apm {

constexpr int SOAP_SEGS = 16;            // scan segments per SOAP chunk
constexpr uint32_t DJ_OVF_CAP = 1u << 16; // outputs beyond the first two of one op

// The plan's write verdict (JoinCounts::pad[1]): the write pass runs only on DJ_WRITE_OK.
enum : uint32_t {
  DJ_WRITE_OK = 0,
  DJ_WRITE_TXT = 1,       // the tx / audit_db text exceeds the staging (host: grow, write again)
  DJ_WRITE_TOO_BIG = 2,   // one batch's ring text over a quarter of the ring
  DJ_WRITE_RING_FULL = 3, // the pending released-tx lines would be overwritten
};

// Where a batch of `bytes` ring text goes (virtual position): after `head`, moved to the next
// ring start when it would wrap (the region stays contiguous).  Device (k_plan_totals) and host
// (DeviceJoin::run, after sync C) compute it alike.
__host__ __device__ inline uint64_t ring_place(uint64_t head, uint64_t bytes, uint64_t cap) {
  return ((head & (cap - 1)) + bytes > cap) ? (head + cap - 1) & ~(cap - 1) : head;
}

struct DJOverflow {
  uint32_t ev, sub;
  uint32_t pad[14];
  TxDev t;
};

// One generation of the audit carry (devjoin_types.h AudCarry / AutrEnt / AudItem); batch k reads
// generation k % 2 and writes the other one.
struct AudGen {
  AudCarry* carry;    // [max files]
  AutrEnt* autr;
  AudItem* items;
  char* txt;
  uint32_t n_autr, n_items, n_txt;  // host-known sizes (input generation)
  uint32_t cap_autr, cap_items, cap_txt;
};

// Per-event selection counts of the parse-side pass (one exclusive scan of these)
struct SelCount {
  uint32_t host;      // events the host resolves
  uint32_t mh;        // audit map lines + block headers
  uint32_t walk;      // audit lines of the block walks (every LK_APP event but map lines)
  uint32_t aud_bytes; // bytes of map / stopWatch name lines (bound of the carry text they add)
};

// Everything one batch of the device join touches.  Device pointers unless noted.
struct DJArgs {
  // ---- batch inputs
  const Event* ev;
  uint32_t n_ev;                  // host-known (parse counts)
  const uint8_t* bytes;
  const uint32_t* chunk_file;
  const uint8_t* chunk_kind;
  uint32_t n_chunks;
  const int32_t* chunk_next;      // next chunk of the same file in this batch (-1)
  const uint8_t* chunk_first;     // 1: first chunk of its file in this batch
  const int32_t* file_server;     // global file id -> server id
  // world-invariant keys (hash of the server name / of the file path) that the join's table keys
  // mix in instead of the engine-local ids: a checkpoint's key table, need arena and audit carry
  // stay valid when a re-sharded engine numbers its servers and files differently (merge.cpp)
  const uint64_t* file_skey;      // global file id -> key of its server
  const uint64_t* file_fkey;      // global file id -> key of the file
  const HostOp* hops;
  uint32_t n_hops;
  const uint8_t* hbuf;            // host op string bytes
  double now;
  uint64_t batch_no;
  double rec_ttl, acct_ttl, need_ttl;
  // ---- host-event selection (run right after the parse kernels)
  uint8_t* host_flag;             // [n_ev] SEL_* bits
  uint64_t* sel_val;              // [n_ev + 1] per-event counts, packed (devjoin.hip sel_unpack)
  uint64_t* sel_pos;              // [n_ev + 1] exclusive scan
  Event* host_ev;                 // compacted host events
  uint32_t* host_ev_idx;
  uint32_t* mh_idx;               // compacted audit map / header events (event indices)
  uint32_t* walk_idx;             // compacted audit walk events (event indices, line order per file)
  SelCount* n_host;               // device totals
  // ---- audit trail (K5)
  uint32_t n_mh, n_walk;          // host-known totals
  uint32_t n_files;
  AudF* aud;                      // [n_ev]
  AudGen gin, gout;               // carry in (read) / out (written)
  uint64_t* aud_key;              // [gin.n_autr + n_mh] sort keys
  uint64_t* aud_key_sorted;
  uint32_t* aud_ord;              // values: < gin.n_autr carried entry, else mh position
  uint32_t* aud_ord_sorted;
  uint32_t* walk_lo;              // [n_chunks + 1] first walk position per chunk
  int32_t* file_first_chunk;      // [n_files]
  AudItem* aud_slots;             // [n_walk + gin.n_items] item slot space of the walks
  // ---- op build + SOAP scan
  JOp* ops;                       // [n_ev]
  uint8_t* soap_code;             // [n_ev]
  double* soap_num;
  uint64_t* soap_hash;
  uint32_t* chunk_ev_lo;          // [n_chunks + 1]
  uint32_t* seg_f;                // [n_chunks][SOAP_SEGS] composed transition function
  uint32_t* seg_in;               // incoming state per segment
  uint64_t* chain_hash;           // per chunk: carried context hash of its file
  SoapState* soap_state;          // [max files] carried per file
  // ---- grouping.  Default (slot lists): k_claim pushes each op onto its key's list
  // (slot_head[slot] <- op, op_idx[op] = the previous head); the op that found the list empty
  // leads the group -- it collects and orders the members (k_group_walk; groups of more than
  // GW_SMALL ops go to k_group_walk_big, one workgroup each) and empties the list again.
  // APM_OPSORT=sort: the stable radix sort of (slot, op) pairs (the round-4 form, for A/B).
  uint32_t* op_slot;              // [n_ev] table slot / DIRECT / NONE
  uint32_t* op_slot_sorted;       // sort: sorted slots; lists: the big groups' leaders
  uint32_t* op_idx;               // sort: op indices; lists: the next (earlier-pushed) member
  uint32_t* op_idx_sorted;        // sort: sorted op indices; lists: the big groups' members
  uint32_t* slot_head;            // lists: [table cap] list heads, ~0u between batches
  uint32_t* big;                  // lists: [2] big groups, their members (zeroed by k_claim)
  int group_sort;                 // 1: the radix-sort grouping
  void* tmp;                      // rocprim scratch
  size_t tmp_bytes;
  KeyState* table;
  // dense copy of table[i].key (8 B per slot): k_claim probes it, so a probe sequence stays in
  // one or two cache lines instead of touching a 128-byte KeyState per step (2M slots: 16 MB
  // against 256 MB); only the winning slot's payload is read or initialised
  uint64_t* keys;
  uint32_t table_mask;
  int table_bits;
  RegSlot* reg;
  uint32_t reg_mask;
  RegMiss* miss;
  uint32_t miss_cap;
  NeedEnt* arena;
  uint32_t arena_cap;             // power of two
  uint64_t arena_base;            // virtual index of this batch's region start
  uint32_t arena_limit;           // entries this batch may allocate
  uint8_t* pool;                  // chain blocks (CHAIN_BLK bytes each)
  uint32_t* pool_ring;            // free block indices (ring of pool_mask + 1)
  uint32_t pool_mask;
  // expiring need entries: virtual ranges [lo, hi) of the regions that expire now
  const uint64_t* exp_lo;         // device
  const uint64_t* exp_hi;
  uint32_t n_exp_regions;
  uint32_t n_exp_entries;         // host-known total
  uint64_t* exp_key;              // [n_exp_entries] created (or max for empty)
  uint64_t* exp_key_sorted;
  uint32_t* exp_idx;
  uint32_t* exp_idx_sorted;
  uint32_t* exp_cnt;
  uint32_t* exp_pos;
  // ---- outputs
  uint32_t* out_cnt;              // [n_ev + 1]
  uint32_t* out_pos;
  TxDev* stage;                   // [n_ev][2]
  DJOverflow* ovf;
  TxDev* out;                     // merged order
  uint32_t out_cap;
  JoinCounts* counts;
};

// Resolve / format / stats hand-off of the joined tx (after the host registered new services).
struct DJFormatArgs {
  TxDev* out;
  uint32_t n_out;
  const RegSlot* reg;
  uint32_t reg_mask;
  const RawSvc* raw;              // [raw id]
  const int32_t* raw_series;      // [raw id] -> series (-1: none yet)
  int32_t* raw_first;             // [raw id] scratch, INT_MAX between batches
  const char* names;              // join names table
  const uint8_t* bytes;
  const uint8_t* hbuf;
  const char* aud_txt;            // audit carry text of this batch (LID_AUD)
  const NeedEnt* arena;
  uint32_t arena_cap;
  const uint8_t* pool;            // chain blocks (long logIds of need entries)
  // per tx {line length, stats flag, length if not to_db, length if to_db} and their scans
  uint32_t* lens;                 // [n_out + 1] x 4
  uint32_t* offs;                 // [n_out + 1] x 4 (exclusive)
  // ring
  char* ring;
  uint64_t ring_cap;              // power of two
  // The batch's ring region is placed on the device (k_plan_totals: ring_place from the head the
  // host knows at launch), so no host round trip sits between the plan and the write pass.
  uint64_t ring_head;             // virtual ring head before this batch (host's, at launch)
  uint64_t ring_low;              // oldest pending ring byte (host's, at launch; only grows)
  uint64_t* ring_pos;             // [1] device: this batch's ring base (written by k_plan_totals)
  uint64_t txt_cap;               // bytes of txt_tx and of txt_db
  // stats hand-off
  TxRec* tx;                      // [n_stats]
  int32_t* tx_raw;
  int64_t* tx_gid;                // ring pos << 20 | len
  int64_t* tx_bucket;
  int64_t* tx_bmax;               // inclusive max scan
  uint32_t* cand;                 // [n] rollover candidates (positions)
  int64_t* cand_bucket;
  uint32_t* unresolved;           // first appearances of raw ids with no series
  char* txt_tx;                   // "transactions" stream (optional)
  char* txt_db;                   // "audit_db" stream (optional)
  int want_tx, want_db;
  JoinCounts* counts;
  void* tmp;
  size_t tmp_bytes;
};

}  // namespace apm

extern "C" {
size_t apm_dj_tmp_bytes(uint32_t max_ev, uint32_t max_out, int table_bits);
// APM_DJ_MARKS=1: host clock (ms, steady clock) after each launch of the join chain since the
// last call, with the launch names; returns the count (at most cap)
int apm_dj_take_marks(double* t, const char** names, int cap);
// a 4-byte field (words = 1) or 8-byte field (words = 2) at `base` (offset included) of n records
// of `stride` bytes, packed into out (checkpoint: the chain heads of the key table / arena)
void apm_dj_gather_field(const void* base, size_t stride, uint32_t n, int words, uint32_t* out, hipStream_t s);
// parse stream, right after apm_parse_batch: select the events the host resolves and copy
// them to a compact buffer (count in *a->n_host).
int apm_dj_select_host(apm::DJArgs* a, const uint32_t* d_n_ev, uint32_t max_ev, hipStream_t s);
// join stream: ops, SOAP scan, grouping, expiry, group walk, placement; counts -> a->counts.
int apm_dj_join(apm::DJArgs* a, hipStream_t s);
// after the host filled the PENDING registry slots: resolve raw ids, line lengths, scans, the
// ring placement and the write verdict (counts->pad[1], DJ_WRITE_*).
int apm_dj_plan(apm::DJFormatArgs* f, hipStream_t s);
// text into the ring, stats arrays, rollover candidates, unresolved series, optional streams.
// Nothing is written unless the plan's verdict was DJ_WRITE_OK (n_out: the tx count, a bound of
// the stats count the kernels read from counts).
int apm_dj_write(apm::DJFormatArgs* f, hipStream_t s);
// key-table rebuild: live entries of `old` reinserted into `fresh` (zeroed by the caller).
// Dropped keys / expired partials free their chain blocks into the pool (pool may be null when
// `now` is -inf: nothing is dropped).
void apm_dj_rebuild(const apm::KeyState* old, uint32_t old_cap, apm::KeyState* fresh, uint32_t fresh_mask,
                    const apm::NeedEnt* arena, uint32_t arena_cap, double now, apm::JoinCounts* counts,
                    unsigned long long* live, uint8_t* pool, uint32_t* pool_ring, uint32_t pool_mask, hipStream_t s);
// The same rebuild in place (same size; cap a power of two >= 8): each cluster of the linear-
// probing table keeps its live keys, slid back towards their homes.  scratch:
// apm_dj_rebuild_scratch_bytes(cap) bytes of device memory.
size_t apm_dj_rebuild_scratch_bytes(uint32_t cap);
// test entry: the rebuild on a synthetic table, checked on the host (see devjoin.hip)
std::vector<double> apm_dj_rebuild_selftest(uint32_t cap, double load, double dead, uint64_t seed, bool copy);
void apm_dj_rebuild_inplace(apm::KeyState* table, uint32_t cap, uint32_t* scratch, const apm::NeedEnt* arena,
                            uint32_t arena_cap, double now, apm::JoinCounts* counts, unsigned long long* live,
                            uint8_t* pool, uint32_t* pool_ring, uint32_t pool_mask, hipStream_t s);
// Checkpoint: the occupied slots (key != 0) of the key table, in slot order, into `out`;
// *d_n = their count.  tmp: apm_dj_live_tmp_bytes(cap) bytes.
size_t apm_dj_live_tmp_bytes(uint32_t cap);
void apm_dj_live_compact(const apm::KeyState* table, uint32_t cap, apm::KeyState* out, uint32_t* d_n, void* tmp,
                         size_t tmp_bytes, hipStream_t s);
// checkpoint: chain blocks idx[0..n) (1-based block numbers, device) gathered into out (device)
void apm_dj_gather_blocks(const uint8_t* pool, const int32_t* idx, uint32_t n, uint8_t* out, hipStream_t s);
// chain-block pool: ring = identity (all `n` blocks free), counters head = 0, tail = ptail = n
void apm_dj_pool_init(uint32_t* ring, uint32_t n, apm::JoinCounts* counts, hipStream_t s);
// pool growth: the free entries of the old ring, then blocks [old_n, new_n), into `fresh_ring`
void apm_dj_pool_grow(const uint32_t* old_ring, uint32_t old_mask, uint32_t* fresh_ring, uint32_t old_n, uint32_t new_n,
                      apm::JoinCounts* counts, hipStream_t s);
// need-arena growth: live entries [lo, hi) (virtual) move to their slots in the bigger arena, and
// every key's `need` index follows its entry
void apm_dj_arena_grow(const apm::NeedEnt* old, uint32_t old_cap, apm::NeedEnt* fresh, uint32_t fresh_cap, uint64_t lo,
                       uint64_t hi, apm::KeyState* table, uint32_t table_cap, hipStream_t s);
// released lines (gids = ring pos << 20 | len): line lengths + offsets of the first *d_n of
// n_upper gids (d_n null: all; offs[n_upper] = total bytes), then the copy into `out`
int apm_dj_gather_plan(const int64_t* gid, int64_t n_upper, const int64_t* d_n, uint32_t* lens, uint32_t* offs,
                       void* tmp, size_t tmp_bytes, hipStream_t s);
// The same for the transactions table's COPY rows (txcopy.hip): lens / offs of the rows the
// released wire lines encode to; fb_count += lines outside the GPU encoder's domain
int apm_dj_txcopy_plan(const int64_t* gid, int64_t n_upper, const int64_t* d_n, const char* ring, uint64_t ring_cap,
                       uint32_t* lens, uint32_t* offs, uint32_t* fb_count, void* tmp, size_t tmp_bytes, hipStream_t s);
void apm_dj_txcopy_write(const int64_t* gid, int64_t n, const char* ring, uint64_t ring_cap, const uint32_t* offs,
                         char* out, hipStream_t s);
// `out` must hold offs[n] = total_bytes bytes (16-byte aligned)
void apm_dj_gather_copy(const int64_t* gid, int64_t n, const char* ring, uint64_t ring_cap, const uint32_t* offs,
                        char* out, uint64_t total_bytes, hipStream_t s);
// checkpoint: gid i -> ((base + offs[i]) << 20) | its length, the line's offset in the saved text
// blob (offs = apm_dj_gather_plan's scan of length + 1)
void apm_dj_rebase_gids(const int64_t* gid, int64_t n, const uint32_t* offs, uint64_t base, int64_t* out,
                        hipStream_t s);
// min ring position among gids (for ring reuse); writes UINT64_MAX when n == 0
void apm_dj_min_pos(const int64_t* gid, int64_t n, unsigned long long* out, hipStream_t s);
// relocate gids below `below` (virtual ring pos): copy their lines to dst_base.. and rewrite
void apm_dj_reg_fill(apm::RegSlot* reg, const int32_t* pairs, uint32_t n, hipStream_t s);
void apm_dj_scatter_i32(int32_t* dst, const int32_t* pairs, uint32_t n, hipStream_t s);
// stats thread: TxRec.series of tx whose raw service got its series after the batch was joined
void apm_dj_fill_series(apm::TxRec* tx, const int32_t* raw, uint32_t n, const int32_t* raw_series,
                        unsigned long long* unmapped, hipStream_t s);
void apm_dj_gather_u8(const uint8_t* src, const int32_t* idx, uint32_t n, uint8_t* out, hipStream_t s);
void apm_dj_cache_stats(const apm::KeyState* table, uint32_t cap, double now, unsigned long long* out, hipStream_t s);
// keys[i] = table[i].key for every slot (after any rewrite of the table other than k_claim's)
void apm_dj_keys_sync(const apm::KeyState* table, uint32_t cap, uint64_t* keys, hipStream_t s);
void apm_dj_count_le(const int64_t* end, int64_t n, int64_t edge, int64_t* out, hipStream_t s);
void apm_dj_relocate(int64_t* gid, int64_t n, char* ring, uint64_t ring_cap, uint64_t below, uint64_t dst_base,
                     unsigned long long* cursor, hipStream_t s);
}
