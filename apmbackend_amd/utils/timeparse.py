"""Timestamp parsing with JS ``Date`` semantics (reference ``stream_parse_transactions.js:242-256``).

* ``YYYY-MM-DD HH:MM:SS,mmm`` -> ``new Date(y, m-1, d, h, mi, s, ms)`` in the configured zone
  (the reference uses the process-local zone).  Field values go through ``Number()``
  conversion and out-of-range fields normalise arithmetically, exactly as ``MakeDay``/
  ``MakeTime`` do.
* strings matching ``/T.*-/`` (audit-trail ISO stamps such as ``2020-01-07T10:00:01.959-06:00``)
  -> ``Date`` parse of the ISO form.
* empty / falsy -> ``''`` (represented here as ``None``); unparseable -> NaN.

The device kernel (``csrc/kernels/parse.hip``) implements the same arithmetic with a host-built
UTC-offset table, so both sides agree bit-for-bit on the integer millisecond results.
"""
from __future__ import annotations

import math
import os
import re
import time
from typing import Optional

_SPLIT_RE = re.compile(r"-|\s+|:|,")
_ISO_RE = re.compile(
    r"^\s*([+-]\d{6}|\d{4})-(\d{2})-(\d{2})T(\d{2}):(\d{2})(?::(\d{2})(?:\.(\d+))?)?\s*(Z|[+-]\d{2}:?\d{2})?\s*$")
_JSNUM_RE = re.compile(r"^[+-]?(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?$")

NAN = float("nan")


def js_number(s: Optional[str]) -> float:
    """``Number(s)`` for the strings that reach ``new Date(...)``."""
    if s is None:
        return NAN
    t = s.strip()
    if t == "":
        return 0.0
    if _JSNUM_RE.match(t):
        return float(t)
    if t.lower().startswith(("0x",)):
        try:
            return float(int(t, 16))
        except ValueError:
            return NAN
    return NAN


def days_from_civil(y: int, m: int, d: int) -> int:
    """Days since 1970-01-01 for proleptic Gregorian y-m-d (m 1..12)."""
    y -= m <= 2
    era = (y if y >= 0 else y - 399) // 400
    yoe = y - era * 400
    mp = (m + 9) % 12
    doy = (153 * mp + 2) // 5 + d - 1
    doe = yoe * 365 + yoe // 4 - yoe // 100 + doy
    return era * 146097 + doe - 719468


def make_date_ms(y: float, mon0: float, d: float, h: float, mi: float, s: float, ms: float) -> float:
    """ECMAScript MakeDate(MakeDay(y, mon0, d), MakeTime(h, mi, s, ms)) in UTC."""
    vals = (y, mon0, d, h, mi, s, ms)
    if any(math.isnan(v) or math.isinf(v) for v in vals):
        return NAN
    y, mon0, d, h, mi, s, ms = (math.trunc(v) for v in vals)
    ym = y + math.floor(mon0 / 12)
    mn = int(mon0 % 12)
    day = days_from_civil(int(ym), mn + 1, 1) + d - 1
    t = ((h * 60 + mi) * 60 + s) * 1000 + ms
    return float(day * 86400000 + t)


class TzOffset:
    """UTC offset provider. ``local`` uses the process zone at parse time; ``UTC``/``+HH:MM``
    are fixed; IANA names use zoneinfo (first occurrence in a DST overlap)."""

    def __init__(self, spec: str = "local"):
        self.spec = spec or "local"
        self.fixed_ms: Optional[int] = None
        self.zone = None
        if self.spec.upper() in ("UTC", "Z", "GMT"):
            self.fixed_ms = 0
        elif re.match(r"^[+-]\d{2}:?\d{2}$", self.spec):
            sgn = -1 if self.spec[0] == "-" else 1
            hh, mm = int(self.spec[1:3]), int(self.spec[-2:])
            self.fixed_ms = sgn * (hh * 60 + mm) * 60000
        elif self.spec != "local":
            from zoneinfo import ZoneInfo
            self.zone = ZoneInfo(self.spec)

    def local_to_utc(self, local_ms: float) -> float:
        if math.isnan(local_ms):
            return NAN
        if self.fixed_ms is not None:
            return local_ms - self.fixed_ms
        if self.zone is not None:
            import datetime as dt
            base = dt.datetime(1970, 1, 1) + dt.timedelta(milliseconds=local_ms)
            off = self.zone.utcoffset(base.replace(fold=0))
            return local_ms - off.total_seconds() * 1000.0
        # process-local zone: JS uses the offset in effect at that local time
        guess = local_ms / 1000.0
        off = -time.altzone if time.localtime(guess).tm_isdst > 0 else -time.timezone
        return local_ms - off * 1000.0

    def offset_ms_for_utc(self, utc_ms: float) -> int:
        if self.fixed_ms is not None:
            return self.fixed_ms
        if self.zone is not None:
            import datetime as dt
            t = dt.datetime.fromtimestamp(utc_ms / 1000.0, tz=dt.timezone.utc)
            return int(self.zone.utcoffset(t.replace(tzinfo=None)).total_seconds() * 1000)
        lt = time.localtime(utc_ms / 1000.0)
        return int(lt.tm_gmtoff * 1000)


_DEFAULT_TZ: Optional[TzOffset] = None


def default_tz() -> TzOffset:
    global _DEFAULT_TZ
    if _DEFAULT_TZ is None:
        _DEFAULT_TZ = TzOffset(os.environ.get("APM_TZ", "local"))
    return _DEFAULT_TZ


def parse_iso(s: str) -> float:
    m = _ISO_RE.match(s)
    if not m:
        return NAN
    y, mo, d, h, mi, sec, frac, tz = m.groups()
    y, mo, d, h, mi = int(y), int(mo), int(d), int(h), int(mi)
    sec = int(sec) if sec else 0
    ms = int((frac or "0")[:3].ljust(3, "0"))
    if not (1 <= mo <= 12 and 1 <= d <= 31 and h <= 24 and mi <= 59 and sec <= 59):
        return NAN
    t = make_date_ms(y, mo - 1, d, h, mi, sec, ms)
    if tz is None:
        # ES2015+: date-time forms without offset are local time
        return default_tz().local_to_utc(t)
    if tz == "Z":
        return t
    sgn = -1 if tz[0] == "-" else 1
    tzd = tz[1:].replace(":", "")
    off = (int(tzd[:2]) * 60 + int(tzd[2:])) * 60000
    return t - sgn * off


def convert_string_date_to_ms(date_str: Optional[str], tz: Optional[TzOffset] = None):
    """Returns ``None`` for the reference's ``''`` result, else a float (possibly NaN)."""
    if not date_str:
        return None
    if re.search(r"T.*-", date_str):
        return parse_iso(date_str)
    arr = _SPLIT_RE.split(date_str.strip())
    get = lambda i: arr[i] if i < len(arr) else None
    nums = [js_number(get(i)) if get(i) is not None else NAN for i in range(7)]
    # new Date(y, m) with fewer args: missing args default (d=1, rest 0) -- but the reference
    # always passes 7 args, undefined -> NaN.
    y = nums[0]
    if not math.isnan(y) and 0 <= math.trunc(y) <= 99:
        y = 1900 + math.trunc(y)  # Date(y, m, ...) maps two-digit years to 19xx
    local = make_date_ms(y, nums[1] - 1, nums[2], nums[3], nums[4], nums[5], nums[6])
    return (tz or default_tz()).local_to_utc(local)


_LINE_TS_RE = re.compile(r"^\S*\s+(\d{4}-\d{2}-\d{2})\s+(\d{2}:\d{2}:\d{2},\d{1,3})(\s|$)")


def leading_line_ts(line: str, tz: Optional[TzOffset] = None) -> Optional[float]:
    """Watermark rule shared by the engine and the oracles: a line whose whitespace tokens 1
    and 2 are ``YYYY-MM-DD`` and ``HH:MM:SS,mmm`` carries a log timestamp."""
    m = _LINE_TS_RE.match(line)
    if not m:
        return None
    v = convert_string_date_to_ms(m.group(1) + " " + m.group(2), tz)
    if v is None or math.isnan(v):
        return None
    return v
