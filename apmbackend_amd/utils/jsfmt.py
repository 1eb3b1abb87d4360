"""JavaScript-exact number parsing and formatting.

The reference writes every record through JS template strings, ``Number.prototype.toFixed``
and ``parseInt``/``parseFloat`` (``entries.js:8-11,58-61,65-69,110-117``).  Wire-format and
database parity therefore needs the exact ECMAScript algorithms, not Python's ``%.1f``
(which rounds half-to-even on the binary value and differs on ties such as ``0.25``).

* ``to_fixed(x, f)``     -- ECMA-262 ``Number.prototype.toFixed`` (ties go to the larger n,
  computed on the exact binary value of the double).
* ``js_str(x)``          -- ``String(x)`` / template-literal formatting of a number
  (shortest round-trip digits, JS exponent rules).
* ``parse_int(s)``       -- ``parseInt(s)`` (radix 10); returns ``float('nan')`` on failure.
* ``parse_float(s)``     -- ``parseFloat(s)``.
* ``nf(x, f)``           -- the ``nf`` helper of ``StatEntry``/``FullStatEntry``
  (``entries.js:65-69``): ``undefined`` for NaN/None, else ``toFixed``.
"""
from __future__ import annotations

import math
import re
from decimal import Decimal, ROUND_HALF_UP
from typing import Optional, Union

Num = Union[int, float, None]

_WS = " \t\n\r\x0b\x0c ﻿  "

_INT_RE = re.compile(r"[+-]?\d+")
_FLOAT_RE = re.compile(r"[+-]?(Infinity|(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?)")


def is_nan(x: Num) -> bool:
    return x is None or (isinstance(x, float) and math.isnan(x))


def to_fixed(x: float, f: int = 1) -> str:
    """ECMA-262 Number.prototype.toFixed for finite |x| < 1e21."""
    if x is None:
        return "undefined"
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if abs(x) >= 1e21 or math.isinf(x):
        return js_str(x)
    neg = x < 0
    d = Decimal(abs(x)).quantize(Decimal(1).scaleb(-f), rounding=ROUND_HALF_UP)
    s = format(d, "f")
    if neg and d != 0:
        return "-" + s
    if neg and d == 0:
        # toFixed(-0.04, 1) === "-0.0" in JS (x < 0 -> "-" prefix) ; -0.0 itself -> "0.0"
        return "-" + s
    return s


def nf(x: Num, f: int = 1) -> str:
    """``nf`` from entries.js:65-69 / 110-114: undefined when falsy-but-not-zero."""
    if x is None:
        return "undefined"
    xf = float(x)
    if math.isnan(xf):
        return "undefined"
    return to_fixed(xf, f)


def js_str(x: Num) -> str:
    """String(x) for a JS number (or ``undefined`` for None)."""
    if x is None:
        return "undefined"
    if isinstance(x, bool):
        return "true" if x else "false"
    if isinstance(x, int):
        x = float(x) if abs(x) > 2 ** 53 else x
        if isinstance(x, int):
            return str(x)
    x = float(x)
    if math.isnan(x):
        return "NaN"
    if math.isinf(x):
        return "Infinity" if x > 0 else "-Infinity"
    if x == 0:
        return "0"
    sign = "-" if x < 0 else ""
    r = repr(abs(x))
    # decompose python repr into digits and exponent
    if "e" in r:
        mant, exp = r.split("e")
        exp = int(exp)
    else:
        mant, exp = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    digits = (ip + fp).lstrip("0")
    # position of decimal point relative to start of `digits`
    lead_zeros = len(ip + fp) - len((ip + fp).lstrip("0"))
    n = len(ip) - lead_zeros + exp
    digits = digits.rstrip("0") or "0"
    k = len(digits)
    if k <= n <= 21:
        return sign + digits + "0" * (n - k)
    if 0 < n <= 21:
        return sign + digits[:n] + "." + digits[n:]
    if -6 < n <= 0:
        return sign + "0." + "0" * (-n) + digits
    e = n - 1
    es = ("+" if e >= 0 else "-") + str(abs(e))
    if k == 1:
        return sign + digits + "e" + es
    return sign + digits[0] + "." + digits[1:] + "e" + es


def parse_int(s) -> float:
    """JS parseInt(s, 10). Numbers are stringified first, as JS does."""
    if s is None:
        return float("nan")
    if isinstance(s, (int, float)) and not isinstance(s, bool):
        if isinstance(s, float) and (math.isnan(s) or math.isinf(s)):
            return float("nan")
        s = js_str(s)
    s = str(s).lstrip(_WS)
    hm = re.match(r"([+-]?)0[xX]([0-9a-fA-F]+)", s)
    if hm:  # radix undefined + "0x" prefix -> hexadecimal
        v = int(hm.group(2), 16) * (-1 if hm.group(1) == "-" else 1)
        return v if abs(v) <= 2 ** 53 else float(v)
    m = _INT_RE.match(s)
    if not m:
        return float("nan")
    v = int(m.group(0))
    if abs(v) <= 2 ** 53:
        return v
    return float(v)


def parse_float(s) -> float:
    """JS parseFloat(s)."""
    if s is None:
        return float("nan")
    if isinstance(s, (int, float)) and not isinstance(s, bool):
        return float(s)
    s = str(s).lstrip(_WS)
    m = _FLOAT_RE.match(s)
    if not m:
        return float("nan")
    t = m.group(0)
    if t.lstrip("+-") == "Infinity":
        return float("-inf") if t.startswith("-") else float("inf")
    return float(t)


def js_truthy_num(x: Num) -> bool:
    """``if (x)`` for a number: false for 0, NaN, None."""
    if x is None:
        return False
    if isinstance(x, str):
        return len(x) > 0
    return not (x == 0 or (isinstance(x, float) and math.isnan(x)))


def round_js_1dp(x: Optional[float]) -> float:
    """parseFloat(x.toFixed(1)) -- the value a downstream stage sees after the wire."""
    if x is None or math.isnan(x):
        return float("nan")
    return float(to_fixed(x, 1))


def round_js_2dp(x: Optional[float]) -> float:
    if x is None or math.isnan(x):
        return float("nan")
    return float(to_fixed(x, 2))
