"""Exact sequential CPU model of the reference pipeline semantics ("the oracle").

This module is the executable specification that every GPU kernel is tested against.  It
models *behaviour* of the reference stages, record-at-a-time, in double precision:

* ``ParseOracle``  -- log line -> ``tx`` records (``stream_parse_transactions.js:210-812``):
  SOAP account capture, EJB / standard CommonTiming entry-exit joins, BAF account salvage,
  the audit-trail state machine, and the three TTL caches (``NodeCache`` semantics with an
  injectable clock; expiry is lazy on ``get``/``has`` plus a sweep at every batch boundary).
* ``StatsOracle``  -- ``tx`` -> ``st`` + released ``tx`` (``stream_calc_stats.js:28-204,331-371``):
  10 s buckets, rollover on a newer bucket, the 31-bucket window / 30-bucket TPM divisor (Q2),
  the reference percentile formula (Q3), ordered release through a port of the JS binary heap.
* ``ZScoreOracle`` -- ``st`` -> ``fs`` (``stream_calc_z_score.js:66-311``): smoothed z-score per
  LAG with ``sqrt(mean)`` as sigma (Q1) and influence on the previous stored value.
* ``AlertsOracle`` -- ``fs`` -> ``al`` (``stream_process_alerts.js:348-471``): hard max, signal
  gates, alertOnBothOnly, the leaky counter (Q6) and the per-service cooldown (Q7).

Where the reference depends on wall-clock time (NodeCache TTLs, alert timestamps) the oracle
takes an explicit clock, which is what makes GPU-vs-oracle comparisons deterministic.
"""
from __future__ import annotations

import math
import re
from collections import OrderedDict
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

from ..utils import jsfmt
from ..utils.config import zscore_lag_settings
from ..utils.records import AlertEntry, FullStatEntry, StatEntry, TxEntry, entry_from_csv
from ..utils.timeparse import TzOffset, convert_string_date_to_ms, default_tz

NAN = float("nan")


# ----------------------------------------------------------------------------- JS helpers

def _valid(v) -> bool:
    return v is not None and not (isinstance(v, float) and math.isnan(v))


def js_average(values: Iterable) -> Optional[float]:
    """Array.prototype.average (util_methods.js:10-24): mean of defined, non-NaN entries,
    summed left to right from 0 in double precision; ``None`` when there are none.

    A history list that offers ``float_view()`` (a float64 array, NaN = undefined; used by the
    bench-scale tests for LAG 8640) is summed by ``np.add.accumulate``: the same sequential
    left-to-right double additions, in C."""
    view = getattr(values, "float_view", None)
    if view is not None:
        import numpy as np
        a = view()
        a = a[~np.isnan(a)]
        return float(np.add.accumulate(a)[-1] / a.size) if a.size else None
    cnt = 0
    s = 0
    for v in values:
        if _valid(v):
            cnt += 1
            s = s + float(v)
    if cnt > 0:
        return s / cnt
    return None


def js_stddev(values: Iterable) -> Optional[float]:
    """Array.prototype.standardDeviation *as the reference computes it* (Q1):
    ``average()`` ignores its argument, so the result is ``sqrt(mean)`` (``None`` if the mean
    is 0/undefined, NaN if negative)."""
    vals = values if hasattr(values, "float_view") else list(values)
    avg = js_average(vals)
    if avg is None or (isinstance(avg, float) and math.isnan(avg)):
        return None
    avg_sq = avg  # the bug: this.average(squareDiffs) === this.average()
    if avg_sq and avg_sq != 0:
        return math.sqrt(avg_sq) if avg_sq > 0 else NAN
    return None


def true_stddev(values: Iterable) -> Optional[float]:
    vals = [float(v) for v in values if _valid(v)]
    if not vals:
        return None
    m = sum(vals) / len(vals)
    var = sum((v - m) ** 2 for v in vals) / len(vals)
    return math.sqrt(var) if var != 0 else None


def js_binary_insert(arr: List[float], v: float) -> None:
    """Array.prototype.binaryInsert(v, duplicate=true) (util_methods.js:57-95) with the default
    comparator.  NaN compares 'equal' to everything, so once a NaN is in the array the result
    is no longer sorted and depends on the insertion order -- reproduced exactly here."""
    lo, hi = 0, len(arr) - 1
    while lo <= hi:
        m = (lo + hi) >> 1
        a = arr[m]
        if a < v:
            lo = m + 1
        elif a > v:
            hi = m - 1
        else:  # equal, or either side NaN
            arr.insert(m, v)
            return
    arr.insert(lo, v)


def js_window_array(bucket_arrays) -> List[float]:
    """windowSortedElapTimes of generateAllStatsToQueue (stream_calc_stats.js:172-178): the
    window buckets binaryConcat'ed in key order.  Without NaN this is just the sorted union."""
    out: List[float] = []
    if not any(v != v for arr in bucket_arrays for v in arr):
        for arr in bucket_arrays:
            out.extend(arr)
        out.sort()
        return out
    for arr in bucket_arrays:
        for v in arr:
            js_binary_insert(out, v)
    return out


def calc_percentile(arr: List[float], percentile: float):
    """Array.prototype.calcPercentile (util_methods.js:112-142) on a sorted array."""
    n = len(arr)
    if n == 0:
        return None
    if percentile == 0:
        return arr[0]
    if percentile == 100:
        return arr[-1]
    index = (percentile / 100.0) * n - 1.0
    if n == 1 or index % 1 == 0:
        return arr[int(index)]
    index = int(math.ceil(index))
    if index == n - 1:
        return arr[index]
    return (arr[index] + arr[index + 1]) / 2


def percentile_ranks(n: int, percentile: float) -> Tuple[int, int]:
    """The (lo, hi) sorted ranks calc_percentile reads for a window of n samples; the value is
    ``(a[lo] + a[hi]) / 2`` when ``lo != hi`` else ``a[lo]``.  Shared with the GPU kernel."""
    if n <= 0:
        return (-1, -1)
    if percentile == 0:
        return (0, 0)
    if percentile == 100:
        return (n - 1, n - 1)
    index = (percentile / 100.0) * n - 1.0
    if n == 1 or index % 1 == 0:
        i = int(index)
        return (i, i)
    i = int(math.ceil(index))
    if i == n - 1:
        return (i, i)
    return (i, i + 1)


class JsBinaryHeap:
    """Port of binary_heap.js (min-heap by score) -- kept so the oracle reproduces the
    reference release order exactly, including the order of equal scores."""

    def __init__(self, score: Callable[[Any], float]):
        self.content: List[Any] = []
        self.score = score

    def push(self, el):
        self.content.append(el)
        self._bubble_up(len(self.content) - 1)

    def pop(self):
        result = self.content[0]
        end = self.content.pop()
        if self.content:
            self.content[0] = end
            self._sink_down(0)
        return result

    def peek(self):
        return self.content[0]

    def size(self):
        return len(self.content)

    def pop_all_le(self, score):
        out = []
        while self.content and self.score(self.peek()) <= score:
            out.append(self.pop())
        return out

    def _bubble_up(self, n):
        el = self.content[n]
        sc = self.score(el)
        while n > 0:
            pn = (n + 1) // 2 - 1
            parent = self.content[pn]
            if sc >= self.score(parent):
                break
            self.content[pn] = el
            self.content[n] = parent
            n = pn

    def _sink_down(self, n):
        length = len(self.content)
        el = self.content[n]
        es = self.score(el)
        while True:
            c2 = (n + 1) * 2
            c1 = c2 - 1
            swap = None
            c1s = None
            if c1 < length:
                c1s = self.score(self.content[c1])
                if c1s < es:
                    swap = c1
            if c2 < length:
                c2s = self.score(self.content[c2])
                if c2s < (es if swap is None else c1s):
                    swap = c2
            if swap is None:
                break
            self.content[n] = self.content[swap]
            self.content[swap] = el
            n = swap


# ----------------------------------------------------------------------------- TTL cache

class TTLCache:
    """NodeCache (v5) semantics with an injectable clock.

    ``set`` stamps expiry = now + ttl; ``get``/``has`` lazily expire (strict ``expiry < now``),
    emitting ``on_expired(key, value)``; ``sweep`` is the periodic ``_checkData``.
    """

    def __init__(self, ttl_s: float, clock: Callable[[], float],
                 on_expired: Optional[Callable[[str, Any], None]] = None):
        self.ttl_ms = ttl_s * 1000.0
        self.clock = clock
        self.on_expired = on_expired
        self.data: "OrderedDict[str, Tuple[Any, float]]" = OrderedDict()
        self.stats = {"hits": 0, "misses": 0, "keys": 0}

    def _check(self, key) -> bool:
        val, t = self.data[key]
        if t != 0 and t < self.clock():
            del self.data[key]
            if self.on_expired:
                self.on_expired(key, val)
            return False
        return True

    def set(self, key, value):
        # JS object semantics: re-setting an existing key keeps its position
        self.data[key] = (value, self.clock() + self.ttl_ms)
        return True

    def get(self, key):
        if key in self.data and self._check(key):
            self.stats["hits"] += 1
            return self.data[key][0]
        self.stats["misses"] += 1
        return None

    def has(self, key) -> bool:
        return key in self.data and self._check(key)

    def sweep(self):
        for key in list(self.data.keys()):
            if key in self.data:
                self._check(key)

    def __len__(self):
        return len(self.data)


# ----------------------------------------------------------------------------- parse oracle

_WS_SPLIT = re.compile(r"\s+")
_SOAP_LOG = re.compile(r"soap_io")
_SERVER_LOG = re.compile(r"server\.log")
_EJB_ENTRY = re.compile(r"INFO *\[CommonTiming] The EJB")
_EJB_EXIT = re.compile(r"INFO *\[CommonTiming] Total time")
_CT_ENTRY = re.compile(r"INFO *CommonTiming::Start")
_CT_EXIT = re.compile(r"INFO *CommonTiming::Stop")
_SOAP_IN = re.compile(r"^=== jbossId.*IO=I")
_SOAP_OUT = re.compile(r"^=== jbossId.*IO=O")
_SOAP_ACCT = re.compile(r"<accountNumber>", re.I)
_SOAP_ALT_KEY = re.compile(r"<key>AccountNumber</key>", re.I)
_SOAP_ALT_VALUE = re.compile(r"<value>")
_BAF_RX = re.compile(r"\[[^ ]+] +INFO ")
_AUTR_MAP = re.compile(r"INFO  auditTrailId=")
_AUTR_HDR = re.compile(r"^Audit Trail id *:")
_EL_START = re.compile(r": RequestTrace \[stopWatchList=")
_EL_END = re.compile(r"^]")
_SW_START = re.compile(r"<stopWatchList>")
_SW_END = re.compile(r"</stopWatchList>")
_SW_NAME = re.compile(r"<name>")
_SW_START_TS = re.compile(r"<startTime>")
_SW_STOP_TS = re.compile(r"<stopTime>")
_TOPLEVEL = re.compile(r"^S:")
_PROVIDER = re.compile(r"Provider\[", re.I)
_DIGITS = re.compile(r"^[0-9]+$")
_BRACKETS = re.compile(r"[\[\]]")


def _tok(arr: List[str], i: int) -> Optional[str]:
    return arr[i] if 0 <= i < len(arr) else None


def _s(x: Optional[str]) -> str:
    """Template-literal interpolation: undefined -> 'undefined'."""
    return "undefined" if x is None else x


def js_split_ws(s: str) -> List[str]:
    return _WS_SPLIT.split(s)


def xml_inner(line: str) -> str:
    """``line.replace(/<\\/.*/,'').replace(/.*>/,'')``"""
    return re.sub(r".*>", "", re.sub(r"</.*", "", line, count=1), count=1)


def normalize_service(service: str) -> str:
    """outputRecord's rewrite: first ``Provider[`` (any case) -> ``Provider:``, then the first ``]``
    removed (stream_parse_transactions.js:274)."""
    service = _PROVIDER.sub("Provider:", service, count=1)
    return service.replace("]", "", 1)


def file_kind(path: str) -> str:
    name = path.split("/")[-1]
    if _SOAP_LOG.search(name):
        return "SOAP"
    if _SERVER_LOG.search(name):
        return "SERVER"
    return "APP"


def server_of(path: str) -> str:
    parts = path.split("/")
    return parts[2] if len(parts) > 2 else "undefined"


class ParseOracle:
    """Sequential model of the transaction parser.

    ``emit(queue, csv_line)`` receives every produced record; ``queue`` is ``'transactions'``
    (the stats stage) or ``'db_insert'`` (non-Provider audit records, Q18).
    The clock is set with ``begin_batch(now_ms)``, which also performs the periodic sweep.
    """

    def __init__(self, emit: Callable[[str, str], None], tz: Optional[TzOffset] = None,
                 record_ttl=120, acct_ttl=120, need_ttl=30, server_fn: Callable[[str], str] = None):
        self.emit = emit
        self.server_fn = server_fn or server_of  # path -> server (reference: split('/')[2])
        self.tz = tz or default_tz()
        self.now = 0.0
        clock = lambda: self.now
        self.context: Dict[str, Dict[str, Any]] = {}
        self.acct_cache = TTLCache(acct_ttl, clock)
        self.record_cache = TTLCache(record_ttl, clock, self._record_expired)
        self.need_cache = TTLCache(need_ttl, clock, self._need_expired)
        self.counters = {"lines": 0, "expired_partials": 0, "need_expired": 0,
                         "ejb_exit_unmatched": 0, "invalid_acct": 0, "audit_errors": 0}

    # -- clock
    def begin_batch(self, now_ms: float):
        self.now = float(now_ms)
        # periodic check: need-cache checkperiod 10 s, others 30 s -- modelled as a sweep at
        # every batch boundary (the engine does the same).
        self.record_cache.sweep()
        self.need_cache.sweep()
        self.acct_cache.sweep()

    def _record_expired(self, log_id, m):
        self.counters["expired_partials"] += len(m)

    def _need_expired(self, log_id, need_map):
        for service, rec in list(need_map.items()):
            self.counters["need_expired"] += 1
            alt = rec.get("altAcctNum") or ""
            self.output_record(rec.get("server"), service, log_id, alt, rec.get("startTs"),
                               rec.get("endTs"), rec.get("elapsed"), rec.get("insertToDb") or False)

    # -- output
    def output_record(self, server, service, log_id, acct_num, start_ts, end_ts, elapsed,
                      insert_to_db=False):
        start_ms = convert_string_date_to_ms(start_ts, self.tz) if isinstance(start_ts, str) else start_ts
        end_ms = convert_string_date_to_ms(end_ts, self.tz) if isinstance(end_ts, str) else end_ts
        service = normalize_service(_s(service))
        if not jsfmt.js_truthy_num(start_ms):
            e = 0.0 if end_ms is None else end_ms  # JS: '' - n === -n
            start_ms = e - jsfmt.parse_int(elapsed)
        tx = TxEntry.make(server, service, _s(log_id) if log_id is not None else "undefined",
                          acct_num if acct_num is not None else "undefined",
                          start_ms, end_ms if end_ms is not None else "", elapsed,
                          "Y" if _TOPLEVEL.search(service) else "N")
        self.emit("db_insert" if insert_to_db else "transactions", tx.to_csv())

    # -- account handling
    def save_acct_num(self, acct: str, fp: str, source: str, alt_log_id: Optional[str] = None):
        acct = acct.strip()
        if not _DIGITS.match(acct):
            # reference: logs (and, through the $currLogFp typo, throws -- Q16 fixed)
            self.counters["invalid_acct"] += 1
            return
        if source == "bafmetainfo":
            log_id = alt_log_id
            if not log_id:
                return
        else:
            log_id = self.context[fp]["logId"]
        self.acct_cache.set(log_id, acct)
        if source != "bafmetainfo":
            self.context.pop(fp, None)
        need_map = self.need_cache.get(log_id)
        if need_map:
            srv = self.server_fn(fp)
            for service, rec in list(need_map.items()):
                self.output_record(srv, service, log_id, acct, rec.get("startTs"), rec.get("endTs"),
                                   rec.get("elapsed"))
                del need_map[service]

    def _baf_acct(self, line: str, fp: str, log_id: str, arr: List[str]) -> str:
        acct = ""
        if _BAF_RX.search(line):
            t = _tok(arr, 3) or ""
            t = re.sub(r".*]\[", "", t, count=1)
            t = _BRACKETS.sub("", t)
            parts = t.split(":")
            acct = parts[-1]
            if acct:
                self.save_acct_num(acct, fp, "bafmetainfo", log_id)
        return acct

    # -- SOAP
    def _soap(self, line: str, fp: str):
        if _SOAP_IN.search(line):
            tok = _tok(js_split_ws(line), 1)
            parts = (tok or "").split("=")
            self.context[fp] = {"logId": parts[1] if len(parts) > 1 else None}
        elif _SOAP_OUT.search(line):
            self.context.pop(fp, None)
        elif fp in self.context:
            if _SOAP_ACCT.search(line):
                parts = re.split(r"<|>", line.strip())
                self.save_acct_num(parts[2] if len(parts) > 2 else "", fp, "standard")
            elif _SOAP_ALT_KEY.search(line):
                self.context[fp] = dict(self.context[fp], pullNextValueFlag=True)
            elif _SOAP_ALT_VALUE.search(line) and self.context[fp].get("pullNextValueFlag"):
                parts = re.split(r"<|>", line.strip())
                self.save_acct_num(parts[2] if len(parts) > 2 else "", fp, "riskStrategy")

    # -- CommonTiming
    def _ejb_entry(self, line: str, server: str):
        arr = js_split_ws(line)
        log_id = _BRACKETS.sub("", arr[0])
        start_ts = f"{_s(_tok(arr, 1))} {_s(_tok(arr, 2))}"
        if log_id == "":
            return
        service = f"S:{_s(_tok(arr, 13))}"
        if not self.record_cache.has(log_id):
            self.record_cache.set(log_id, OrderedDict())
        m = self.record_cache.get(log_id)
        m[service] = {"server": server, "startTs": start_ts}  # Map.set keeps position

    def _ejb_exit(self, line: str, server: str):
        arr = js_split_ws(line)
        log_id = _BRACKETS.sub("", arr[0])
        end_ts = f"{_s(_tok(arr, 1))} {_s(_tok(arr, 2))}"
        service = f"S:{_s(_tok(arr, 9))}"
        elapsed = _tok(arr, 11)
        if log_id == "":
            self.output_record(server, service, "", "", "", end_ts, elapsed)
            return
        m = self.record_cache.get(log_id)
        if m is None:
            self.counters["ejb_exit_unmatched"] += 1
            return
        part = m.get(service)
        if part is None:
            self.counters["ejb_exit_unmatched"] += 1
            return
        acct = self.acct_cache.get(log_id)
        if acct:
            self.output_record(server, service, log_id, acct, part["startTs"], end_ts, elapsed)
        else:
            if not self.need_cache.has(log_id):
                self.need_cache.set(log_id, OrderedDict())
            nm = self.need_cache.get(log_id)
            nm[service] = dict(part, endTs=end_ts, elapsed=elapsed)
        del m[service]

    @staticmethod
    def _after_info(line: str) -> List[str]:
        parts = line.split("INFO")
        seg = parts[1] if len(parts) > 1 else ""
        return js_split_ws(seg.strip())

    def _ct_entry(self, line: str, server: str):
        arr = js_split_ws(line)
        log_id = _BRACKETS.sub("", arr[0])
        start_ts = f"{_s(_tok(arr, 1))} {_s(_tok(arr, 2))}"
        service = _s(_tok(self._after_info(line), 1))
        if log_id == "":
            return
        if not self.record_cache.has(log_id):
            self.record_cache.set(log_id, OrderedDict())
        m = self.record_cache.get(log_id)
        m[service] = {"server": server, "startTs": start_ts}  # Map.set keeps position

    def _salvage(self, line, fp, log_id, arr, server, service, end_ts, elapsed):
        acct = self._baf_acct(line, fp, log_id, arr)
        self.output_record(server, service, "", acct, "", end_ts, elapsed)

    def _ct_exit(self, line: str, fp: str, server: str):
        arr = js_split_ws(line)
        second = self._after_info(line)
        log_id = _BRACKETS.sub("", arr[0])
        end_ts = f"{_s(_tok(arr, 1))} {_s(_tok(arr, 2))}"
        service = _s(_tok(second, 1))
        elapsed = _tok(second, 5)
        m = self.record_cache.get(log_id)
        if log_id == "":
            self._salvage(line, fp, log_id, arr, server, service, end_ts, elapsed)
            return
        if m is None:
            self._salvage(line, fp, log_id, arr, server, service, end_ts, elapsed)
            return
        part = m.get(service)
        if part is None:
            self._salvage(line, fp, log_id, arr, server, service, end_ts, elapsed)
            return
        acct = self.acct_cache.get(log_id)
        if acct:
            self.output_record(server, service, log_id, acct, part["startTs"], end_ts, elapsed)
        else:
            if not self.need_cache.has(log_id):
                self.need_cache.set(log_id, OrderedDict())
            alt = self._baf_acct(line, fp, log_id, arr)
            nm = self.need_cache.get(log_id)
            if nm is None:  # expired between has() and get() cannot happen with a fixed clock
                nm = OrderedDict()
            nm[service] = dict(part, endTs=end_ts, elapsed=elapsed, altAcctNum=alt)
        del m[service]

    # -- audit trail
    def _app(self, line: str, fp: str, server: str):
        if _AUTR_MAP.search(line):
            arr = js_split_ws(line)
            log_id = _BRACKETS.sub("", arr[0])
            t5 = _tok(arr, 5) or ""
            parts = t5.split("=")
            autr_id = parts[1] if len(parts) > 1 else None
            if fp not in self.context:
                self.context[fp] = {"autrIdMap": OrderedDict()}
            ctx = self.context[fp]
            ctx.setdefault("autrIdMap", OrderedDict())
            alt = self._baf_acct(line, fp, log_id, arr)
            ctx["autrIdMap"][autr_id] = {"logId": log_id, "altAcctNum": alt}
        elif _AUTR_HDR.search(line):
            if fp in self.context:
                autr_id = line.split(":")[1].strip()
                ctx = self.context[fp]
                obj = (ctx.get("autrIdMap") or {}).get(autr_id)
                if not obj or not obj.get("logId"):
                    self.counters["audit_errors"] += 1
                else:
                    ctx["serviceMap"] = OrderedDict()
                    ctx["activeAutrId"] = autr_id
                    ctx["activeLogId"] = obj["logId"]
                    ctx["activeAltAcctNum"] = obj["altAcctNum"]
                    ctx["elapsedFlag"] = False
                    ctx["swFlag"] = False
                    ctx["activeService"] = None
                    del ctx["autrIdMap"][autr_id]
            else:
                self.counters["audit_errors"] += 1
        elif fp in self.context and self.context[fp].get("activeLogId"):
            ctx = self.context[fp]
            if _EL_START.search(line):
                ctx["elapsedFlag"] = True
            elif ctx.get("elapsedFlag"):
                if _EL_END.search(line):
                    ctx["elapsedFlag"] = False
                else:
                    arr = line.split(":")
                    service = arr[0].strip()
                    el_tok = js_split_ws(arr[1])[0] if len(arr) > 1 else ""
                    elapsed = _BRACKETS.sub("", el_tok)
                    ctx["serviceMap"].setdefault(service, []).append({"elapsed": elapsed})
            elif _SW_START.search(line):
                ctx["swFlag"] = True
            elif ctx.get("swFlag"):
                if _SW_END.search(line):
                    for k in ("activeAutrId", "activeLogId", "activeAltAcctNum", "activeService",
                              "serviceMap"):
                        ctx[k] = None
                    ctx["elapsedFlag"] = False
                    ctx["swFlag"] = False
                elif _SW_NAME.search(line):
                    ctx["activeService"] = xml_inner(line)
                elif ctx.get("activeService"):
                    svc = ctx["activeService"]
                    if _SW_START_TS.search(line):
                        lst = ctx["serviceMap"].get(svc)
                        if not lst:
                            self.counters["audit_errors"] += 1
                            return
                        lst[0]["startTs"] = xml_inner(line)
                    elif _SW_STOP_TS.search(line):
                        end_ts = xml_inner(line)
                        lst = ctx["serviceMap"].get(svc)
                        if not lst:
                            self.counters["audit_errors"] += 1
                            return
                        obj = lst.pop(0)
                        log_id = ctx["activeLogId"]
                        acct = self.acct_cache.get(log_id)
                        insert_to_db = not _PROVIDER.search(svc)
                        if acct:
                            self.output_record(server, svc, log_id, acct, obj.get("startTs"), end_ts,
                                               obj.get("elapsed"), insert_to_db)
                        else:
                            if not self.need_cache.has(log_id):
                                self.need_cache.set(log_id, OrderedDict())
                            nm = self.need_cache.get(log_id)
                            nm[svc] = {"server": server, "logId": log_id,
                                       "startTs": obj.get("startTs"), "endTs": end_ts,
                                       "elapsed": obj.get("elapsed"),
                                       "altAcctNum": ctx.get("activeAltAcctNum"),
                                       "insertToDb": insert_to_db}

    # -- dispatcher
    def read_line(self, fp: str, line: str):
        if not line:
            return
        self.counters["lines"] += 1
        server = self.server_fn(fp)
        kind = file_kind(fp)
        if kind == "SOAP":
            self._soap(line, fp)
        elif kind == "SERVER":
            if _EJB_ENTRY.search(line):
                self._ejb_entry(line, server)
            elif _EJB_EXIT.search(line):
                self._ejb_exit(line, server)
            elif _CT_ENTRY.search(line):
                self._ct_entry(line, server)
            elif _CT_EXIT.search(line):
                self._ct_exit(line, fp, server)
        else:
            if _CT_ENTRY.search(line):
                self._ct_entry(line, server)
            elif _CT_EXIT.search(line):
                self._ct_exit(line, fp, server)
            else:
                self._app(line, fp, server)


# ----------------------------------------------------------------------------- stats oracle

class StatsOracle:
    """``StatParser`` + ``consumeMsg`` of stream_calc_stats.js."""

    def __init__(self, emit_stat: Callable[[str], None], emit_db: Callable[[str], None],
                 interval_len=10, window=30, buffer=6):
        self.emit_stat = emit_stat
        self.emit_db = emit_db
        self.interval_len = interval_len
        self.window = window
        self.buffer = buffer
        self.keep = window + buffer
        self.servers: "OrderedDict[str, OrderedDict[str, Dict[int, List[int]]]]" = OrderedDict()
        self.latest = 0
        self.heap = JsBinaryHeap(lambda tx: tx.endTs)
        self.rollovers = 0

    @staticmethod
    def bucket_label(end_ts) -> Optional[int]:
        s = jsfmt.js_str(end_ts)
        lab = s[:-4] if len(s) > 4 else ""
        try:
            return int(lab)
        except ValueError:
            return None

    def consume(self, csv_line: str):
        tx = entry_from_csv(csv_line)
        self.consume_tx(tx)

    def consume_tx(self, tx: TxEntry):
        lab = self.bucket_label(tx.endTs)
        if lab is None:
            return  # NaN/short endTs: the reference would wedge its heap (fix)
        if lab > self.latest:
            self.latest = lab
            self.rollover()
        srv = self.servers.setdefault(tx.server, OrderedDict())
        svc = srv.setdefault(tx.service, {})
        svc.setdefault(lab, []).append(jsfmt.parse_int(tx.elapsed))
        self.heap.push(tx)

    def advance_to(self, latest: int):
        """Multi-rank lock-step (parallel/dist): another rank saw bucket ``latest`` -- roll
        over as the single reference stats process would have at that tx."""
        if latest > self.latest:
            self.latest = latest
            self.rollover()

    def rollover(self):
        self.rollovers += 1
        for srv in self.servers.values():
            for svc in srv.values():
                for b in [b for b in svc if b < self.latest - self.keep]:
                    del svc[b]
        edge_ts = (self.latest - self.buffer - 1) * 10000
        for tx in self.heap.pop_all_le(edge_ts):
            self.emit_db(tx.to_csv())
        for server, srv in self.servers.items():
            for service, svc in srv.items():
                win: List[List[int]] = []
                cnt = 0
                total = 0
                # bucket keys are integer-like, so Object.entries visits them ascending
                for b in sorted(svc):
                    arr = svc[b]
                    if self.latest - self.keep <= b <= self.latest - self.buffer:
                        cnt += len(arr)
                        for v in arr:
                            total += v
                        win.append(arr)
                avg = p75 = p95 = None
                if cnt != 0:
                    vals = js_window_array(win)
                    avg = total / cnt
                    p75 = calc_percentile(vals, 75)
                    p95 = calc_percentile(vals, 95)
                tpm = cnt / (self.window * self.interval_len / 60.0)
                st = StatEntry.make(edge_ts, server, service, tpm, avg, p75, p95)
                self.emit_stat(st.to_csv())


# ----------------------------------------------------------------------------- z-score oracle

def process_zscore_stats(lag: int, threshold: float, influence: float, x: float,
                         prev: List[float], sigma_mode: str = "sqrt_mean"):
    """processZScoreStats (stream_calc_z_score.js:66-104). Returns (stored, avg, lb, ub, signal)."""
    infl = x
    avg = sd = lb = ub = None
    signal = 0
    if len(prev) >= lag:
        avg = js_average(prev)
        sd = js_stddev(prev) if sigma_mode == "sqrt_mean" else true_stddev(prev)
        ok = lambda v: v is not None and not (isinstance(v, float) and math.isnan(v))
        if ok(avg) and ok(sd):
            lb = avg - threshold * sd
            ub = avg + threshold * sd
        if not ok(avg) or not ok(sd):
            signal = 0
        elif not _valid(x):
            signal = 0
        elif abs(x - avg) > threshold * sd:
            signal = 1 if x > avg else -1
            last = prev[-1]
            if _valid(last):
                infl = influence * x + (1 - influence) * last
        else:
            signal = 0
    return infl, avg, lb, ub, signal


class ZScoreOracle:
    def __init__(self, cfg: Dict[str, Any], emit: Callable[[str], None],
                 emulate_aliasing: bool = False, sigma_mode: str = "sqrt_mean"):
        self.cfg = cfg
        self.emit = emit
        self.emulate_aliasing = emulate_aliasing
        self.sigma_mode = sigma_mode
        self.servers: "OrderedDict[str, OrderedDict[str, Dict[int, Dict[str, Any]]]]" = OrderedDict()

    def settings(self, service):
        return zscore_lag_settings(self.cfg, service, self.emulate_aliasing)

    def reload(self, cfg: Dict[str, Any]):
        """The watcher callback (stream_calc_z_score.js:362-382): updateAllServiceSettings --
        every series gets the new THRESHOLD / INFLUENCE of every configured LAG, a new LAG an
        empty history -- then removeStaleLagData drops the LAGs no longer configured."""
        self.cfg = cfg
        for srv in self.servers.values():
            for service, lags in srv.items():
                settings = self.settings(service)
                for el in settings:
                    lag = int(el["LAG"])
                    if lag in lags:
                        lags[lag]["THRESHOLD"], lags[lag]["INFLUENCE"] = el["THRESHOLD"], el["INFLUENCE"]
                    else:
                        lags[lag] = {"THRESHOLD": el["THRESHOLD"], "INFLUENCE": el["INFLUENCE"],
                                     "avgList": [], "per75List": [], "per95List": []}
                keep = {int(el["LAG"]) for el in settings}
                for lag in [x for x in lags if x not in keep]:
                    del lags[lag]

    def consume(self, csv_line: str):
        e = entry_from_csv(csv_line)
        if e is not None and e.type == "st":
            for fs in self.process(e):
                self.emit(fs.to_csv())

    def process(self, st: StatEntry) -> List[FullStatEntry]:
        srv = self.servers.setdefault(st.server, OrderedDict())
        if st.service not in srv:
            lags: Dict[int, Dict[str, Any]] = {}
            for el in self.settings(st.service):
                lags[int(el["LAG"])] = {"THRESHOLD": el["THRESHOLD"], "INFLUENCE": el["INFLUENCE"],
                                        "avgList": [], "per75List": [], "per95List": []}
            srv[st.service] = lags
        out = []
        for lag in sorted(srv[st.service].keys()):
            o = srv[st.service][lag]
            T, I = o["THRESHOLD"], o["INFLUENCE"]
            a = process_zscore_stats(lag, T, I, st.average, o["avgList"], self.sigma_mode)
            p = process_zscore_stats(lag, T, I, st.per75, o["per75List"], self.sigma_mode)
            q = process_zscore_stats(lag, T, I, st.per95, o["per95List"], self.sigma_mode)
            for key in ("avgList", "per75List", "per95List"):
                if len(o[key]) >= lag:
                    o[key].pop(0)
            f = lambda v: NAN if v is None else v
            out.append(FullStatEntry.make(
                st.timestamp, st.server, st.service, st.tpm, str(lag),
                st.average, f(a[1]), f(a[2]), f(a[3]), a[4],
                st.per75, f(p[1]), f(p[2]), f(p[3]), p[4],
                st.per95, f(q[1]), f(q[2]), f(q[3]), q[4]))
            o["avgList"].append(a[0])
            o["per75List"].append(p[0])
            o["per95List"].append(q[0])
        return out


# ----------------------------------------------------------------------------- alerts oracle

ALERT_CAUSES = ["average exceeded hard ms threshold", "per75 exceeded hard ms threshold",
                "average UB exceeded", "per75 UB exceeded", "average and per75 UB exceeded"]


class AlertsOracle:
    def __init__(self, cfg: Dict[str, Any], clock: str = "entry",
                 wall: Callable[[], float] = None, cooldown_key: str = "service"):
        self.cfg = cfg
        self.clock = clock
        self.wall = wall
        self.cooldown_key = cooldown_key
        self.recent: Dict[Tuple[str, str, str], int] = {}
        self.alerts: Dict[str, AlertEntry] = {}
        self.alert_buffer: List[AlertEntry] = []

    def process(self, en: FullStatEntry) -> Optional[AlertEntry]:
        ac = self.cfg["streamProcessAlerts"]
        key = (en.server, en.service, str(en.lag))
        cnt = self.recent.get(key, 0)
        window = int(ac["rollingAlertWindowSizeInIntervals"])
        thresh = int(ac["requiredNumberBadIntervalsInAlertWindowToTrigger"])
        state = {"cnt": cnt, "inc": False, "trigger": False}
        causes: List[str] = []

        def alert(cause):
            if not state["inc"]:
                if state["cnt"] <= window:
                    state["cnt"] += 1
                state["inc"] = True
            if window and window > 1 and thresh and thresh > 1:
                if state["cnt"] >= thresh:
                    state["trigger"] = True
                    causes.append(cause)
            else:
                state["trigger"] = True
                causes.append(cause)

        ovr = ((ac.get("overrides") or {}).get("services") or {}).get(en.service)
        lag_i = jsfmt.parse_int(en.lag)
        if lag_i not in [int(x) for x in ac.get("suppressedLags", [])]:
            if en.service not in ac.get("suppressedServices", []):
                hard_max = ac["hardMaxMsAlertThreshold"]
                if ovr is not None and ovr.get("hardMaxMsAlertThreshold"):
                    hard_max = ovr["hardMaxMsAlertThreshold"]
                gt = lambda a, b: _valid(a) and a > b
                if gt(en.average, hard_max):
                    alert(ALERT_CAUSES[0])
                if gt(en.per75, hard_max):
                    alert(ALERT_CAUSES[1])
                both = 0
                mn, mt = ac["hardMinMsAlertThreshold"], ac["hardMinTpmAlertThreshold"]
                if gt(en.averageSignal, 0) and gt(en.average, mn) and gt(en.tpm, mt):
                    if not ac["alertOnBothOnly"]:
                        alert(ALERT_CAUSES[2])
                    else:
                        both += 1
                if gt(en.per75Signal, 0) and gt(en.per75, mn) and gt(en.tpm, mt):
                    if not ac["alertOnBothOnly"]:
                        alert(ALERT_CAUSES[3])
                    else:
                        both += 1
                if ac["alertOnBothOnly"] and both >= 2:
                    alert(ALERT_CAUSES[4])
        if not state["inc"] and state["cnt"] > 0:
            state["cnt"] -= 1
        if state["cnt"] < 0:
            state["cnt"] = 0
        self.recent[key] = state["cnt"]
        if not state["trigger"]:
            return None
        now = en.timestamp if self.clock == "entry" else self.wall()
        al = AlertEntry.make(now, en.timestamp, en.server, en.service, ",".join(causes), en.to_csv())
        return al if self.admit(al) else None

    def cooldown_key_of(self, server: str, service: str) -> str:
        return service if self.cooldown_key == "service" else f"{server}\x00{service}"

    def admit(self, al: AlertEntry) -> bool:
        """The per-service cooldown (:436-468): the first candidate in emission order wins."""
        ac = self.cfg["streamProcessAlerts"]
        ck = self.cooldown_key_of(al.server, al.service)
        last = self.alerts.get(ck)
        if last is None or (al.alertTimestamp - last.alertTimestamp) / 1000 > ac["perServiceAlertCooldownInMinutes"] * 60:
            self.alerts[ck] = al
            self.alert_buffer.append(al)
            return True
        return False

    def evaluate(self, en: FullStatEntry) -> Optional[AlertEntry]:
        """The leaky counter alone: the candidate an fs row raises, before the cooldown."""
        saved, self.admit = self.admit, (lambda al: True)
        try:
            return self.process(en)
        finally:
            self.admit = saved


# ----------------------------------------------------------------------------- full chain

class PipelineOracle:
    """parse -> stats -> z-score -> alerts, with the queues modelled as in-order FIFOs."""

    def __init__(self, cfg: Dict[str, Any], tz: Optional[TzOffset] = None, alert_clock="entry",
                 server_fn: Callable[[str], str] = None,
                 node_exchange: Optional[Callable[[list], list]] = None,
                 server_index: Optional[Dict[str, int]] = None):
        """``node_exchange`` (multi-rank, servers sharded over ranks): the cooldown is decided
        node-wide.  Alert candidates are queued with their global emission-order key and, after
        every batch, ``node_exchange(mine)`` returns every rank's candidates; each rank applies
        the same cooldown in the same order and keeps its own winners (engine.cpp "node-wide
        cooldown").  ``server_index``: node-wide server positions (the key's tie-break within
        one batch)."""
        self.cfg = cfg
        self.node_exchange = node_exchange
        self.server_index = server_index or {}
        self._batch_no = 0
        self._first_batch: Dict[str, int] = {}
        self._svc_seq: Dict[Tuple[str, str], int] = {}
        self._node_q: list = []
        self._fs_no = 0
        self.tx_db: List[str] = []
        self.audit_db: List[str] = []
        self.stats: List[str] = []
        self.fs: List[str] = []
        self.al: List[str] = []
        self.tx_out: List[str] = []
        g = cfg.get("gpu", {})
        self.zs = ZScoreOracle(cfg, self._on_fs, g.get("emulateOverrideAliasing", False),
                               g.get("zscoreSigma", "sqrt_mean"))
        self.alerts = AlertsOracle(cfg, alert_clock, cooldown_key=g.get("cooldownKey", "service"))
        sc = cfg["streamCalcStats"]
        self.st = StatsOracle(self._on_st, self.tx_db.append, int(sc["intervalLengthInSeconds"]),
                              int(sc["windowSizeInIntervals"]), int(sc["bufferSizeInIntervals"]))
        self.parse = ParseOracle(self._on_tx, tz, g.get("recordTtlSeconds", 120),
                                 g.get("acctTtlSeconds", 120), g.get("needTtlSeconds", 30), server_fn=server_fn)

    def reload(self, cfg: Dict[str, Any]):
        """Config hot reload between two batches: z-score settings / LAG set (ZScoreOracle.reload)
        and every alert gate (read from the config per fs entry)."""
        self.cfg = cfg
        self.zs.reload(cfg)
        self.alerts.cfg = cfg
        # stream_calc_stats.js watcher (:228-261): getParseSettings re-read, used from the next
        # rollover (removeOldBuckets / window / TPM divisor / edge)
        sc = cfg["streamCalcStats"]
        st = self.st
        st.interval_len = int(sc["intervalLengthInSeconds"])
        st.window = int(sc["windowSizeInIntervals"])
        st.buffer = int(sc["bufferSizeInIntervals"])
        st.keep = st.window + st.buffer

    def _on_tx(self, queue, line):
        if queue == "db_insert":
            self.audit_db.append(line)
        else:
            self.tx_out.append(line)
            n = len(self.st.servers)
            self.st.consume(line)
            if len(self.st.servers) != n:  # a server's first series: its node-wide order key
                for srv in list(self.st.servers)[n:]:
                    self._first_batch.setdefault(srv, self._batch_no)

    def _on_st(self, line):
        self.stats.append(line)
        self.zs.consume(line)

    def _on_fs(self, line):
        self.fs.append(line)
        en = entry_from_csv(line)
        if self.node_exchange is not None:
            al = self.alerts.evaluate(en)
            if al is not None:
                sk = (en.server, en.service)
                if sk not in self._svc_seq:
                    self._svc_seq[sk] = list(self.st.servers[en.server]).index(en.service)
                self._fs_no += 1
                key = (int(en.timestamp), self._first_batch.get(en.server, -1),
                       self.server_index.get(en.server, 0), self._svc_seq[sk], self._fs_no)
                self._node_q.append((key, al.to_csv()))
            return
        al = self.alerts.process(en)
        if al is not None:
            self.al.append(al.to_csv())

    def _node_resolve(self):
        mine = set(c for _k, c in self._node_q)
        every = self.node_exchange(self._node_q)
        self._node_q = []
        for _key, csv in sorted(every):
            al = entry_from_csv(csv)
            if self.alerts.admit(al) and csv in mine:
                self.al.append(csv)

    def run_batches(self, batches: Iterable[Tuple[float, List[Tuple[str, List[str]]]]],
                    sync_latest: Optional[Callable[[int], int]] = None):
        """batches: (now_ms, [(file_path, [lines...]), ...]).  ``sync_latest`` (multi-rank)
        maps this rank's latest bucket to the global one after every batch."""
        for now, chunks in batches:
            self.parse.begin_batch(now)
            for fp, lines in chunks:
                for ln in lines:
                    self.parse.read_line(fp, ln)
            if sync_latest is not None:
                self.st.advance_to(sync_latest(self.st.latest))
            if self.node_exchange is not None:
                self._node_resolve()
            self._batch_no += 1
