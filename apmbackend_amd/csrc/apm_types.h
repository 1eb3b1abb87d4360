// Shared host/device record layouts for the apm-mi355x engine.
//
// Everything that crosses a stage boundary inside one GPU process is a fixed-layout POD
// defined here (SoA where a kernel streams it, AoS where the host walks it).  The text wire
// formats of the reference (entries.js) are produced from these only at the sinks.
#pragma once
#include <stdint.h>

namespace apm {

// ----------------------------------------------------------------------------- log files
enum FileKind : uint8_t { FILE_SOAP = 0, FILE_SERVER = 1, FILE_APP = 2 };

// ----------------------------------------------------------------------------- parse events
// Line kinds reported by the classify kernel (stream_parse_transactions.js:734-791).
enum LineKind : uint8_t {
  LK_NONE = 0,
  LK_EJB_ENTRY = 1,   // INFO *\[CommonTiming] The EJB            (server.log)
  LK_EJB_EXIT = 2,    // INFO *\[CommonTiming] Total time         (server.log)
  LK_CT_ENTRY = 3,    // INFO *CommonTiming::Start                (server/app)
  LK_CT_EXIT = 4,     // INFO *CommonTiming::Stop                 (server/app)
  LK_SOAP = 5,        // any soap_io line matching a SOAP pattern (mask says which)
  LK_APP = 6,         // app line matching an audit pattern or inside an elapsed section
};

// Pattern bits (Event::mask).  SOAP bits:
enum : uint32_t {
  PM_SOAP_IN = 1u << 0,       // ^=== jbossId.*IO=I
  PM_SOAP_OUT = 1u << 1,      // ^=== jbossId.*IO=O
  PM_SOAP_ACCT = 1u << 2,     // <accountNumber>  (case-insensitive)
  PM_SOAP_KEY = 1u << 3,      // <key>AccountNumber</key> (case-insensitive)
  PM_SOAP_VALUE = 1u << 4,    // <value>
  // app / audit bits
  PM_AUTR_MAP = 1u << 8,      // INFO  auditTrailId=
  PM_AUTR_HDR = 1u << 9,      // ^Audit Trail id *:
  PM_EL_START = 1u << 10,     // : RequestTrace \[stopWatchList=
  PM_EL_END = 1u << 11,       // ^]
  PM_SW_START = 1u << 12,     // <stopWatchList>
  PM_SW_END = 1u << 13,       // </stopWatchList>
  PM_SW_NAME = 1u << 14,      // <name>
  PM_SW_STARTTS = 1u << 15,   // <startTime>
  PM_SW_STOPTS = 1u << 16,    // <stopTime>
  PM_IN_SECTION = 1u << 17,   // line lies inside an elapsed section (over-approximation)
  // misc
  PM_BAF = 1u << 24,          // \[[^ ]+] +INFO   (BAF metadata present)
  PM_HOST = 1u << 25,         // non-ASCII / exotic number forms: host re-derives the fields
  PM_HAS_INFO2 = 1u << 26,    // a second "INFO" occurrence bounds the INFO segment
  PM_KEYS = 1u << 27,         // EJB/CT: t0 is the bracket-stripped logId, key / svc hold its hashes
};

// One event per relevant line, in line order (ordered stream compaction).
struct Event {
  uint32_t line;        // line index within the batch
  uint32_t chunk;       // chunk (file) index within the batch
  uint32_t off;         // byte offset of the line within the batch
  uint32_t len;         // line length (without '\n' / trailing '\r')
  uint32_t mask;        // PM_* bits
  uint8_t kind;         // LineKind
  uint8_t ntok;         // whitespace tokens found (capped at 15)
  uint16_t pad0;
  // whitespace-token byte offsets relative to the line start (0xffff = missing)
  uint16_t t0s, t0e, t1s, t1e, t2s, t2e, t3s, t3e;
  uint16_t tAs, tAe;    // ejb: token 13 (entry) / token 9 (exit); ct: INFO-segment token 1
  uint16_t tBs, tBe;    // ejb exit: token 11; ct exit: INFO-segment token 5
  double ts;            // parsed "t1 t2" timestamp in UTC ms (NaN if unparseable)
  double num;           // parseInt(elapsed token) (NaN if none)
  // PM_KEYS events: the join's map keys, hashed on the GPU so the host never touches the line
  // bytes of an entry event: key = hash_bytes(logId), svc = hash_bytes(service name, seed by
  // kind: kHashSeedEjb for the "S:"-prefixed EJB names, kHashSeed for CommonTiming)
  uint64_t key;
  uint64_t svc;
};

static_assert(sizeof(Event) == 80, "Event layout");

// ----------------------------------------------------------------------------- transactions
// A completed transaction handed from the join to the stats stage.
struct TxRec {
  int64_t end_ms;       // endTs
  int32_t series;       // (server, service) series id
  int32_t elapsed;      // parseInt(elapsed) clamped to int32 (INT32_MIN = NaN)
};
static_assert(sizeof(TxRec) == 16, "TxRec layout");

constexpr int32_t ELAPSED_NAN = (int32_t)0x80000000;

// ----------------------------------------------------------------------------- stats / z-score
// Bucket ring slots per series: config-sized (gpu.bucketRingSlots, at least window + buffer + 1:
// removeOldBuckets keeps window + buffer buckets plus the one being filled); this is the default
// floor (window 31 + buffer 6 + slack).  A live reload to a longer window grows the ring.
constexpr int NSLOT_MIN = 40;
constexpr int K8_INLINE_SLOTS = 64;  // window buckets passed to K8 as kernel arguments (more: a device array)
constexpr int NSTAT = 3;           // avg, p75, p95
// LAG settings per engine.  The reference takes any number; here it is a capacity: every LAG is an
// HBM ring of LAG x NSTAT x maxSeries values (LAG 8640 at fp64 and 131k series: 27 GB), so HBM,
// not this table, is what bounds it -- 16 daily LAGs would not fit a 288 GB MI355X.
constexpr int MAX_LAGS = 16;

// Per-series window statistics produced at a rollover (values already rounded the way the
// z-score stage sees them after the `st` wire format: tpm 2 dp, the rest 1 dp).
struct WinStat {
  double tpm;
  double avg;           // NaN = undefined
  double p75;
  double p95;
  int32_t n;            // samples in the window
  int32_t active;       // series existed at this rollover
};

// z-score outputs per (series, lag) for one rollover -> `fs` fields.
struct ZOut {
  double mean[NSTAT];   // avgAvg / per75Avg / per95Avg (NaN = undefined)
  double lb[NSTAT];
  double ub[NSTAT];
  int8_t sig[NSTAT];
  uint8_t valid;        // row produced
  uint8_t pad[4];
};

// Alert candidate (compacted).
struct AlertRec {
  int32_t series;
  int32_t lag_idx;
  uint32_t causes;      // bit i = cause i in check order (stream_process_alerts.js:401-423)
  uint32_t pad;
  uint64_t order;       // emission order (series emit key * nlags + lag_idx)
};

}  // namespace apm
