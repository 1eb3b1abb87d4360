// Device join (K4/K5/K6 on the GPU): record layouts shared by devjoin.hip and the host driver
// (runtime/devjoin.cpp).
//
// The reference joins a logId's entry, exit and account lines through three TTL caches
// (stream_parse_transactions.js:211-239 recordCache / acctCache / needNumRecordCache,
// saveAcctNum :294-327, EJB exit :403-446, CT exit :506-565).  Every cache is keyed by the
// logId of one JVM, so the join is independent per (server, logId): the GPU groups a batch's
// join operations by that key (table slot), and one lane replays each group's operations in
// line order against the key's state, which lives in HBM between batches:
//   KeyState  -- acct cache entry + recordCache partial map of one key (128 B, one table slot)
//   NeedEnt   -- needNumRecordCache entry (parked exits waiting for an account), arena-allocated
//                per batch so a batch's entries expire together (their TTL clock is the batch's)
// SOAP request contexts (per file) are resolved by a segmented scan over state-transition
// functions, the audit-trail state machine (K5) by key-grouped and block-parallel walks (below);
// the host only re-derives the fields of lines the parser deferred (PM_HOST) as HostOps.
#pragma once
#include <stdint.h>

namespace apm {

// ------------------------------------------------------------------------------ join ops
enum JOpKind : uint8_t {
  JOP_NONE = 0,
  JOP_ENTRY = 1,      // EJB / CommonTiming entry: recordCache[logId][svc] = start
  JOP_EJB_EXIT = 2,   // EJB exit (logId non-empty)
  JOP_CT_EXIT = 3,    // CommonTiming exit (logId non-empty), optional BAF account
  JOP_ACCT = 4,       // saveAcctNum (SOAP account / value line, auditTrailId BAF account)
  JOP_AUDIT_TX = 5,   // audit-trail stopTime record (parseAppLine :688-729)
  JOP_DIRECT = 6,     // immediate output, no cache state (EJB exit / CT exit with an empty logId)
};

enum JOpFlags : uint16_t {
  JF_TS_EMPTY = 1u << 0,     // end timestamp '' (convertStringDateToMs falsy)
  JF_START_EMPTY = 1u << 1,  // audit: start timestamp ''
  JF_BAF = 1u << 2,          // CT exit: BAF account string present (non-empty)
  JF_BAF_VALID = 1u << 3,    // ... and it is all digits (saveAcctNum accepts it)
  JF_TO_DB = 1u << 4,        // audit: insertToDb (non-Provider service, Q18)
  JF_LID_HOST = 1u << 5,     // logId bytes live in the host op buffer (else: the batch bytes)
  JF_SVC_UNDEF = 1u << 6,    // service token missing: the name is "undefined"
  JF_SVC_HOST = 1u << 7,     // service name bytes in the host op buffer
  JF_EJB = 1u << 8,          // EJB service ("S:" prefix, kHashSeedEjb)
  JF_HAS_SVC = 1u << 9,      // op names a service (registry claim)
  JF_LID_AUD = 1u << 10,     // logId bytes in the audit carry text (AudGen::txt of this batch)
  JF_SVC_AUD = 1u << 11,     // service name bytes in the audit carry text
};

// One join operation per relevant event (line order), 80 B.
struct JOp {
  uint64_t gkey;     // join key = mix(hash(logId), server) (0: JOP_DIRECT)
  uint64_t svc;      // raw service hash (seeded by kind)
  double ts;         // ENTRY: start; EXIT / AUDIT: end (NaN = unparseable)
  double num;        // EXIT / AUDIT: elapsed; ACCT: account value
  double aux;        // CT exit: BAF account as output (parseInt); AUDIT: start
  double aux2;       // CT exit: BAF account as saved; AUDIT: alt account (NaN none)
  uint32_t line;     // line index in the batch (need-entry creation order)
  uint32_t lid;      // logId bytes offset (batch bytes, or host buffer with JF_LID_HOST)
  uint32_t svc_ref;  // service name bytes offset (batch bytes, or host buffer with JF_SVC_HOST)
  uint16_t lid_len;
  uint16_t svc_len;
  int32_t server;
  uint16_t flags;
  uint8_t op;
  uint8_t pad;
  uint32_t pad2[2];
};
static_assert(sizeof(JOp) == 80, "JOp layout");

// Host-resolved op for an event the GPU cannot resolve alone (audit lines, PM_HOST lines, SOAP
// lines whose fields the host re-derived).  `ev` = event index; sorted by ev.
enum HostOpKind : uint8_t {
  HOP_JOIN = 1,       // a full JOp (op.op != JOP_NONE)
  HOP_SOAP_IN = 2,    // SOAP request start; lid bytes in the host buffer (lid_len 0 + num=1: "undefined")
  HOP_SOAP_OUT = 3,
  HOP_SOAP_ACCT = 4,  // op.num = account, flags JF_BAF_VALID when valid
  HOP_SOAP_KEY = 5,
  HOP_SOAP_VALUE = 6,
  HOP_SKIP = 7,       // event produces nothing
  HOP_AUD = 8,        // audit line the GPU cannot read alone: its AudF fields (in `op`), strings in hbuf
};
struct HostOp {
  uint32_t ev;
  uint8_t kind;
  uint8_t pad[3];
  uint64_t lid_hash;  // HOP_SOAP_IN: hash of the logId (or of "undefined")
  JOp op;
};
static_assert(sizeof(HostOp) == 96, "HostOp layout");

// ------------------------------------------------------------------------------ state
// The reference caches are unbounded JS Maps (recordCache / needNumRecordCache `maxKeys: -1`,
// :211-218): a logId may hold any number of open partials and parked records, and logIds have
// any length.  The common case lives inline in the table slot / arena entry; everything beyond
// it goes to chains of 256-byte blocks in a device block pool (index + 1 links, 0 = none),
// allocated and freed by the join kernels (ChainPool below).  Nothing is dropped.
constexpr int KS_PARTS = 5;
struct KeyState {  // 128 B, one hash-table slot
  uint64_t key;    // gkey, 0 = empty
  double acct;
  double acct_exp;  // acctCache entry live iff acct_exp >= now (-inf: none)
  double rec_exp;   // recordCache entry live iff rec_exp >= now
  int32_t need;     // NeedEnt arena index (-1 none)
  int32_t n_part;   // open partials: [0, KS_PARTS) inline, the rest in the PartBlk chain
  uint64_t part_svc[KS_PARTS];
  double part_start[KS_PARTS];
  int32_t pblk;     // PartBlk chain (block index + 1, 0 none)
  int32_t server;   // engine server id of the key (a re-shard keeps the keys of the servers it owns)
};
static_assert(sizeof(KeyState) == 128, "KeyState layout");

constexpr int NEED_ITEMS = 7;
constexpr int NEED_LID = 80;
struct NeedItem {   // 48 B
  uint64_t svc;
  double start, end, elapsed, alt;
  uint32_t flags;   // JF_START_EMPTY | JF_TS_EMPTY | JF_TO_DB
  int32_t pad;
};
struct NeedEnt {    // 512 B
  uint64_t key;
  double exp;
  uint64_t created;  // (batch_no << 28) | line
  int32_t server;
  int32_t n;         // items: [0, NEED_ITEMS) inline, the rest in the NeedBlk chain (insertion order)
  int32_t lid_len;   // full logId length: [0, NEED_LID) inline, the rest in the LidBlk chain
  int32_t pad;
  char lid[NEED_LID];
  NeedItem items[NEED_ITEMS];
  int32_t iblk;      // NeedBlk chain (block index + 1, 0 none)
  int32_t lblk;      // LidBlk chain
  uint64_t vidx;     // virtual arena index (arena growth remaps the table's `need` through it)
  uint8_t tail[40];
};
static_assert(sizeof(NeedEnt) == 512, "NeedEnt layout");

// ---- chain blocks (256 B, one pool)
constexpr int CHAIN_BLK = 256;
constexpr int PBLK_N = 15;   // partials per block
constexpr int NBLK_N = 5;    // parked records per block
constexpr int LBLK_N = 240;  // logId bytes per block
struct PartBlk {
  int32_t next;
  int32_t pad[3];
  uint64_t svc[PBLK_N];
  double start[PBLK_N];
};
struct NeedBlk {
  int32_t next;
  int32_t pad[3];
  NeedItem items[NBLK_N];
};
struct LidBlk {
  int32_t next;
  int32_t pad[3];
  char b[LBLK_N];
};
static_assert(sizeof(PartBlk) == CHAIN_BLK && sizeof(NeedBlk) == CHAIN_BLK && sizeof(LidBlk) == CHAIN_BLK,
              "chain block layout");

// A completed transaction (outputRecord :264-290) before formatting, 64 B.
enum : uint8_t { LID_NONE = 0, LID_BATCH = 1, LID_HOST = 2, LID_NEED = 3, LID_AUD = 4 };
struct TxDev {
  double end;       // endTs after parseInt (NaN: '')
  double start;     // startTs after the start = end - elapsed fallback and parseInt
  double acct;
  double elapsed;
  uint64_t svc;
  int32_t server;
  uint32_t lid;     // logId location (see lid_src)
  uint16_t lid_len;
  uint8_t lid_src;
  uint8_t to_db;
  int32_t raw;      // raw service id (registry), filled by the resolve pass
  uint32_t pad[2];
};
static_assert(sizeof(TxDev) == 64, "TxDev layout");

// Registry of (server, raw service hash) -> raw service id.  Slot value RAW_PENDING: claimed by
// the GPU in this batch, the host assigns the id (names are interned on the host).
constexpr int32_t RAW_EMPTY = -1;
constexpr int32_t RAW_PENDING = -2;
struct RegSlot {
  uint64_t key;     // mix(svc, server) (0 empty)
  int32_t raw;
  int32_t pad;
};
struct RegMiss {    // a service seen for the first time (name bytes for the host)
  uint64_t svc;
  int32_t server;
  uint32_t name;    // offset (batch bytes, or host buffer with JF_SVC_HOST)
  uint16_t name_len;
  uint16_t flags;   // JF_EJB | JF_SVC_UNDEF | JF_SVC_HOST
  int32_t slot;
};

// Raw service table (host-filled): names for the tx line and the toplevel flag.
struct RawSvc {
  int32_t srv_off, srv_len;   // server name in the join names table
  int32_t norm_off, norm_len; // normalized service name (Provider[x] -> Provider:x)
  int32_t toplevel;           // normalized name starts with "S:"
  int32_t pad;
};

// Per-file SOAP request context carried across batches.
struct SoapState {
  int32_t tag;        // 0 none, 1 present, 2 present + pull_next
  int32_t undef;      // has_log_id false -> "undefined"
  uint64_t lid_hash;  // hash(logId) of the context
};

// ------------------------------------------------------------------------------ audit trail (K5)
// parseAppLine (stream_parse_transactions.js:578-731) keeps, per log file, an auditTrailId ->
// {logId, alt account} map and one open audit block (the service -> elapsed queues of its
// RequestTrace section, then the stopWatchList that pops them).  On the GPU:
//   * every audit line gets its fields extracted once (AudF, one lane per event; lines the GPU
//     cannot read alone -- non-ASCII, exotic numbers / dates -- get them from the host, HOP_AUD);
//   * map lines and block headers are matched per (file, auditTrailId) key: the carried map
//     entries and this batch's MAP / HDR events are sorted by key (stable: carried first, then
//     line order) and one lane per key replays them -- a header consumes the live entry;
//   * each block (a header that found its entry, up to the next such header of its file) is
//     walked by one lane in line order: the service queues live in a per-batch slot space, a
//     stopTime pops the front of its service's queue and becomes a JOP_AUDIT_TX op;
//   * what is still open at the end of the batch (map entries, one block per file) is written to
//     the next generation of the carry (AudGen, double-buffered): strings into its text arena.
// The result equals the host state machine (runtime/join.cpp on_app) line for line.
enum AudFlags : uint8_t {
  AF_SRC_HOST = 1u << 0,  // ref/len point into the host op buffer (else the batch bytes)
  AF_SRC_AUD = 1u << 1,   // ... into the carry text of this batch (HDR results only)
  AF_TS_EMPTY = 1u << 2,  // STARTTS / STOPTS: convertStringDateToMs returned ''
  AF_TO_DB = 1u << 3,     // SW_NAME: the name has no "Provider[" (insertToDb)
  AF_HDR_OK = 1u << 4,    // HDR: found a live map entry with a non-empty logId (block start)
  AF_ACCT = 1u << 5,      // MAP: the alt account is non-empty
  AF_ACCT_VALID = 1u << 6,  // ... and all digits (saveAcctNum accepts it)
};
struct AudF {        // 48 B per event
  uint64_t h_item;   // item role: hash(service); MAP / HDR: (file, auditTrailId) key
  double el;         // item role: parseInt(elapsed); MAP / HDR-ok: parseInt(alt account) (NaN: '')
  uint64_t h_sw;     // SW_NAME: hash(name); MAP / HDR-ok: hash(logId)
  double ts;         // STARTTS / STOPTS: ms
  uint32_t ref;      // SW_NAME: name; MAP / HDR-ok: logId (see AF_SRC_*)
  uint16_t len;
  uint8_t flags;
  uint8_t pad;
  uint32_t pad2[2];
};
struct AutrEnt {     // a live auditTrailId map entry carried to the next batch, 32 B
  uint64_t key;      // (file, auditTrailId)
  uint64_t lid_hash;
  double alt;
  uint32_t lid_off;  // carry text
  uint32_t lid_len;
};
struct AudItem {     // one queued elapsed entry of a service, 32 B
  uint64_t svc;      // hash(service)
  double el;
  double start;      // startTime ms (valid when AI_START and not AI_START_EMPTY)
  uint32_t flags;
  uint32_t next;     // slot list link (walk kernels only)
};
enum : uint32_t { AI_START = 1u, AI_START_EMPTY = 2u };
struct AudCarry {    // the open block of one file, 64 B
  uint8_t active, elapsed, sw, has_svc;
  uint8_t svc_to_db, pad0[3];
  uint64_t lid_hash;
  uint64_t svc_hash;
  double alt;
  uint32_t lid_off, lid_len;    // carry text
  uint32_t svc_off, svc_len;    // carry text
  uint32_t items_off, n_items;  // carry items, queue order
  uint32_t pad1[2];
};
static_assert(sizeof(AudF) == 48 && sizeof(AutrEnt) == 32 && sizeof(AudItem) == 32 && sizeof(AudCarry) == 64,
              "audit layouts");

// Batch counters written by the join kernels (D2H once per batch).
struct JoinCounts {
  uint32_t n_ops;
  uint32_t n_out;          // tx produced (expiries + line emissions)
  uint32_t n_exp_out;      // of which from expired need entries
  uint32_t n_miss;         // new raw services
  uint32_t n_need_new;     // need entries created
  uint32_t n_keys_new;     // key-table slots claimed
  uint32_t text_bytes;     // formatted tx text
  uint32_t n_stats;        // tx handed to the stats stage (non-db, usable endTs)
  uint32_t n_db;           // audit non-Provider tx (to_db)
  uint32_t n_dropped;      // NaN / short endTs
  uint32_t n_cand;         // rollover candidates
  uint32_t n_unresolved;   // stats tx whose raw service has no series yet (first appearances)
  uint32_t tx_text_bytes;  // "transactions" stream bytes
  uint32_t db_text_bytes;  // "audit_db" stream bytes
  uint32_t pad[2];
  // audit carry written for the next batch (sizes of its generation)
  uint32_t aud_autr_n, aud_items_n, aud_txt_n, aud_pad;
  // sticky counters
  unsigned long long ejb_unmatched, partial_overflow, need_overflow, expired_partials, need_expired,
      invalid_acct, table_full, key_probe_max;
  unsigned long long audit_errors;  // header without a live map entry, start/stop without a queued entry
  // chain-block pool: free-index ring positions (virtual).  Allocation takes [head, tail); frees
  // append at ptail; k_pool_fix publishes them (tail = ptail) after the kernels that allocate.
  unsigned long long pool_head, pool_tail, pool_ptail, pool_fail;
  unsigned long long chain_parts, chain_items, chain_lids;  // blocks ever allocated, by kind
};

}  // namespace apm
