"""Record types and wire codecs (reference ``entries.js:1-342``).

Five record kinds travel between stages, pipe-delimited UTF-8 text:

====  =====================================================================================
tx    ``tx|server|service|logId|acctNum|startTs|endTs|elapsed|topLevel``        (entries.js:19)
st    ``st|ts|server|service|tpm(.2)|avg(.1)|p75(.1)|p95(.1)``                  (entries.js:72)
fs    ``fs|ts|server|service|lag|tpm|avg:avgAvg:avgLB:avgUB:avgSig|p75:...|p95:...`` (:117)
al    ``al|alertTs|entryTs|server|service|cause|<fs with '|' -> '&'>``            (:215)
jx    ``jx|ts|server|<16 JVM gauges>``                                             (:307)
====  =====================================================================================

Every numeric field is parsed with JS ``parseInt``/``parseFloat`` semantics and printed
with JS ``toFixed``/``String`` semantics (``jsfmt``), so a record that round-trips through
this module is byte-identical to what the reference stages produce.
``to_pg_row`` mirrors ``toPostgresObject`` (the inferred Postgres schema).
"""
from __future__ import annotations

import datetime as _dt
import math
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

from .jsfmt import js_str, nf, parse_float, parse_int

Num = Union[int, float]


def _ms_to_dt(ms: Num) -> Optional[_dt.datetime]:
    if ms is None or (isinstance(ms, float) and math.isnan(ms)):
        return None
    return _dt.datetime.fromtimestamp(float(ms) / 1000.0, tz=_dt.timezone.utc)


def _num_or_none(x):
    if x is None or (isinstance(x, float) and math.isnan(x)):
        return None
    return x


@dataclass
class TxEntry:
    server: str
    service: str
    logId: str
    acctNum: Num
    startTs: Num
    endTs: Num
    elapsed: Num
    topLevel: str
    type: str = "tx"

    @classmethod
    def make(cls, server, service, logId, acctNum, startTs, endTs, elapsed, topLevel) -> "TxEntry":
        return cls(server, service, logId, parse_int(acctNum), parse_int(startTs),
                   parse_int(endTs), parse_int(elapsed), topLevel)

    def to_csv(self) -> str:
        return (f"tx|{self.server}|{self.service}|{self.logId}|{js_str(self.acctNum)}|"
                f"{js_str(self.startTs)}|{js_str(self.endTs)}|{js_str(self.elapsed)}|{self.topLevel}")

    def to_pg_row(self) -> Dict[str, Any]:
        return {
            "endts": _ms_to_dt(self.endTs),
            "startts": _ms_to_dt(self.startTs),
            "server": self.server,
            "service": self.service,
            "logid": self.logId,
            "acctnum": _num_or_none(self.acctNum),
            "elapsed": _num_or_none(self.elapsed),
            "toplevel": self.topLevel,
        }


@dataclass
class StatEntry:
    timestamp: Num
    server: str
    service: str
    tpm: float
    average: float
    per75: float
    per95: float
    type: str = "st"

    @classmethod
    def make(cls, timestamp, server, service, tpm, average, per75, per95) -> "StatEntry":
        return cls(parse_int(timestamp), server, service, parse_float(tpm), parse_float(average),
                   parse_float(per75), parse_float(per95))

    def to_csv(self) -> str:
        return (f"st|{js_str(self.timestamp)}|{self.server}|{self.service}|{nf(self.tpm, 2)}|"
                f"{nf(self.average)}|{nf(self.per75)}|{nf(self.per95)}")


@dataclass
class FullStatEntry:
    timestamp: Num
    server: str
    service: str
    tpm: float
    lag: Any
    average: float
    averageAvg: float
    averageLB: float
    averageUB: float
    averageSignal: Num
    per75: float
    per75Avg: float
    per75LB: float
    per75UB: float
    per75Signal: Num
    per95: float
    per95Avg: float
    per95LB: float
    per95UB: float
    per95Signal: Num
    type: str = "fs"

    @classmethod
    def make(cls, timestamp, server, service, tpm, lag, average, averageAvg, averageLB, averageUB,
             averageSignal, per75, per75Avg, per75LB, per75UB, per75Signal, per95, per95Avg,
             per95LB, per95UB, per95Signal) -> "FullStatEntry":
        pf, pi = parse_float, parse_int
        return cls(pi(timestamp), server, service, pf(tpm), lag,
                   pf(average), pf(averageAvg), pf(averageLB), pf(averageUB), pi(averageSignal),
                   pf(per75), pf(per75Avg), pf(per75LB), pf(per75UB), pi(per75Signal),
                   pf(per95), pf(per95Avg), pf(per95LB), pf(per95UB), pi(per95Signal))

    def to_csv(self) -> str:
        # averageSignal is printed raw, the percentile signals through nf (entries.js:117, Q22)
        return (f"fs|{js_str(self.timestamp)}|{self.server}|{self.service}|{self.lag}|{nf(self.tpm, 2)}|"
                f"{nf(self.average)}:{nf(self.averageAvg)}:{nf(self.averageLB)}:{nf(self.averageUB)}:"
                f"{js_str(self.averageSignal)}|"
                f"{nf(self.per75)}:{nf(self.per75Avg)}:{nf(self.per75LB)}:{nf(self.per75UB)}:"
                f"{nf(self.per75Signal)}|"
                f"{nf(self.per95)}:{nf(self.per95Avg)}:{nf(self.per95LB)}:{nf(self.per95UB)}:"
                f"{nf(self.per95Signal)}")

    def to_pg_row(self) -> Dict[str, Any]:
        n = _num_or_none
        return {
            "timestamp": _ms_to_dt(self.timestamp),
            "server": self.server,
            "service": self.service,
            "tpm": n(self.tpm),
            "lag": self.lag,
            "stats": {
                "average": n(self.average), "averageavg": n(self.averageAvg),
                "averagelb": n(self.averageLB), "averageub": n(self.averageUB),
                "averagesignal": n(self.averageSignal),
                "per75": n(self.per75), "per75avg": n(self.per75Avg), "per75lb": n(self.per75LB),
                "per75ub": n(self.per75UB), "per75signal": n(self.per75Signal),
                "per95": n(self.per95), "per95avg": n(self.per95Avg), "per95lb": n(self.per95LB),
                "per95ub": n(self.per95UB), "per95signal": n(self.per95Signal),
            },
        }


@dataclass
class AlertEntry:
    alertTimestamp: Num
    entryTimestamp: Num
    server: str
    service: str
    cause: str
    entry: str  # fs CSV with '|' replaced by '&'
    type: str = "al"

    @classmethod
    def make(cls, alertTimestamp, entryTimestamp, server, service, cause, entry) -> "AlertEntry":
        return cls(parse_int(alertTimestamp), parse_int(entryTimestamp), server, service, cause,
                   entry.replace("|", "&"))

    def to_csv(self) -> str:
        return (f"al|{js_str(self.alertTimestamp)}|{js_str(self.entryTimestamp)}|{self.server}|"
                f"{self.service}|{self.cause}|{self.entry}")

    def fs_entry(self) -> "FullStatEntry":
        return entry_from_csv(self.entry, "&")  # type: ignore[return-value]

    def to_pg_row(self) -> Dict[str, Any]:
        return {
            "alerttimestamp": _ms_to_dt(self.alertTimestamp),
            "entrytimestamp": _ms_to_dt(self.entryTimestamp),
            "server": self.server,
            "service": self.service,
            "cause": self.cause,
            "entry": self.fs_entry().to_pg_row(),
        }


JMX_FIELDS = ["dsInUseNodes", "dsActiveNodes", "dsAvailableNodes", "heapUsed", "heapCommitted",
              "heapMax", "metaUsed", "metaCommitted", "metaMax", "sysLoad", "classCnt",
              "threadCnt", "daemonThreadCnt", "beanPoolAvailableCount", "beanPoolCurrentSize",
              "beanPoolMaxSize"]
JMX_PG = ["dsinusenodes", "dsactivenodes", "dsavailablenodes", "heapused", "heapcommitted",
          "heapmax", "metaused", "metacommitted", "metamax", "sysload", "classcnt", "threadcnt",
          "daemonthreadcnt", "beanpoolavailablecnt", "beanpoolcurrentsize", "beanpoolmaxsize"]


@dataclass
class JmxEntry:
    timestamp: Num
    server: str
    values: List[Num] = field(default_factory=list)
    type: str = "jx"

    @classmethod
    def from_stats(cls, timestamp, server, stats: Dict[str, Any]) -> "JmxEntry":
        """Constructor used by the poller (entries.js:246-273)."""
        pi = parse_int
        r = lambda k: stats[k]["result"]
        vals = [
            pi(r("ds")["InUseCount"]), pi(r("ds")["ActiveCount"]), pi(r("ds")["AvailableCount"]),
            pi(r("heap")["used"]), pi(r("heap")["committed"]), pi(r("heap")["max"]),
            pi(r("meta")["used"]), pi(r("meta")["committed"]), pi(r("meta")["max"]),
            parse_float(r("sysload")),
            pi(r("classcnt")),
            pi(r("threading")["thread-count"]), pi(r("threading")["daemon-thread-count"]),
            pi(r("bean")[0]["result"]["pool-available-count"]),
            pi(r("bean")[0]["result"]["pool-current-size"]),
            pi(r("bean")[0]["result"]["pool-max-size"]),
        ]
        return cls(pi(timestamp), server, vals)

    @classmethod
    def make(cls, timestamp, server, *vals) -> "JmxEntry":
        out = []
        for name, v in zip(JMX_FIELDS, vals):
            out.append(parse_float(v) if name == "sysLoad" else parse_int(v))
        return cls(parse_int(timestamp), server, out)

    def to_csv(self) -> str:
        return "jx|" + "|".join([js_str(self.timestamp), self.server] + [js_str(v) for v in self.values])

    def to_pg_row(self) -> Dict[str, Any]:
        row = {"timestamp": _ms_to_dt(self.timestamp), "server": self.server}
        for k, v in zip(JMX_PG, self.values):
            row[k] = _num_or_none(v)
        return row


def _pad(arr: List[str], n: int) -> List[Optional[str]]:
    return list(arr) + [None] * max(0, n - len(arr))


@dataclass
class FleetEntry:
    """``fb|ts|service|lag|nseries|avgMean:avgStd|p75Mean:p75Std|p95Mean:p95Std`` -- the
    fleet-merged per-service baseline (no reference counterpart: the reference has one process
    per stage and no cross-JVM view).  Emitted by rank 0 after each interval's RCCL merge."""
    timestamp: Num
    service: str
    lag: str
    nseries: Num
    stats: List[Num]  # [avg mean, avg std, p75 mean, p75 std, p95 mean, p95 std]
    type: str = "fb"

    def to_csv(self) -> str:
        g = [f"{nf(self.stats[2 * k], 1)}:{nf(self.stats[2 * k + 1], 1)}" for k in range(3)]
        return f"fb|{js_str(self.timestamp)}|{self.service}|{self.lag}|{js_str(self.nseries)}|" + "|".join(g)

    def to_pg_row(self) -> Dict[str, Any]:
        keys = ("averagemean", "averagestd", "per75mean", "per75std", "per95mean", "per95std")
        return {"timestamp": _ms_to_dt(self.timestamp), "service": self.service, "lag": self.lag,
                "nseries": _num_or_none(self.nseries),
                "stats": {k: _num_or_none(v) for k, v in zip(keys, self.stats)}}


def entry_from_csv(line: Union[str, bytes], delim: str = "|"):
    """EntryFactory.getEntryFromCSV (entries.js:174-193). Returns None for unknown types."""
    if isinstance(line, bytes):
        line = line.decode("utf-8")
    arr = line.split(delim)
    t = arr[0]
    if t == "tx":
        a = _pad(arr, 9)
        return TxEntry.make(a[1], a[2], a[3], a[4], a[5], a[6], a[7], a[8])
    if t == "st":
        a = _pad(arr, 8)
        return StatEntry.make(a[1], a[2], a[3], a[4], a[5], a[6], a[7])
    if t == "fs":
        a = _pad(arr, 9)
        # a truncated record throws in entries.js (undefined.split); here missing groups are
        # read as all-undefined so one bad line cannot take the consumer down
        av = _pad(a[6].split(":") if a[6] is not None else [], 5)
        p75 = _pad(a[7].split(":") if a[7] is not None else [], 5)
        p95 = _pad(a[8].split(":") if a[8] is not None else [], 5)
        return FullStatEntry.make(a[1], a[2], a[3], a[5], a[4], *av, *p75, *p95)
    if t == "al":
        a = _pad(arr, 7)
        return AlertEntry(parse_int(a[1]), parse_int(a[2]), a[3], a[4], a[5], a[6])
    if t == "jx":
        a = _pad(arr, 19)
        return JmxEntry.make(a[1], a[2], *a[3:19])
    if t == "fb":
        a = _pad(arr, 8)
        st: List[Num] = []
        for g in a[5:8]:
            p = _pad(g.split(":") if g is not None else [], 2)
            st += [parse_float(p[0]), parse_float(p[1])]
        return FleetEntry(parse_int(a[1]), a[2], a[3], parse_int(a[4]), st)
    return None


RECORD_TYPES = ("tx", "st", "fs", "al", "jx", "fb")
