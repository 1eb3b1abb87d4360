"""Pure-Python model of the K1/K2 parse kernels (csrc/kernels/parse.hip).

It produces the exact ``apm::Event`` records the GPU emits (same line order, kinds, pattern
masks, token offsets, parsed timestamps and elapsed values), so that:

* the C++ host join can be tested on a CPU-only machine (events -> ``_apm_native.JoinHarness``),
* GPU tests can compare the device event stream field-by-field against this model.

It is deliberately a line-by-line transliteration of the kernel's single pass, not a regex
implementation: the regex semantics are covered by the oracle tests.
"""
from __future__ import annotations

import math
from typing import List, Sequence, Tuple

import numpy as np

from ..utils.timeparse import TzOffset, make_date_ms

FILE_SOAP, FILE_SERVER, FILE_APP = 0, 1, 2
LK_NONE, LK_EJB_ENTRY, LK_EJB_EXIT, LK_CT_ENTRY, LK_CT_EXIT, LK_SOAP, LK_APP = range(7)

PM_SOAP_IN, PM_SOAP_OUT, PM_SOAP_ACCT, PM_SOAP_KEY, PM_SOAP_VALUE = (1 << i for i in range(5))
PM_AUTR_MAP = 1 << 8
PM_AUTR_HDR = 1 << 9
PM_EL_START = 1 << 10
PM_EL_END = 1 << 11
PM_SW_START = 1 << 12
PM_SW_END = 1 << 13
PM_SW_NAME = 1 << 14
PM_SW_STARTTS = 1 << 15
PM_SW_STOPTS = 1 << 16
PM_IN_SECTION = 1 << 17
PM_BAF = 1 << 24
PM_HOST = 1 << 25
PM_HAS_INFO2 = 1 << 26
PM_KEYS = 1 << 27
SOAP_BITS = PM_SOAP_IN | PM_SOAP_OUT | PM_SOAP_ACCT | PM_SOAP_KEY | PM_SOAP_VALUE
AUDIT_BITS = (PM_AUTR_MAP | PM_AUTR_HDR | PM_EL_START | PM_EL_END | PM_SW_START | PM_SW_END | PM_SW_NAME
              | PM_SW_STARTTS | PM_SW_STOPTS)
NOTOK = 0xFFFF

EVENT_DTYPE = np.dtype([
    ("line", "<u4"), ("chunk", "<u4"), ("off", "<u4"), ("len", "<u4"), ("mask", "<u4"),
    ("kind", "u1"), ("ntok", "u1"), ("pad0", "<u2"),
    ("t0s", "<u2"), ("t0e", "<u2"), ("t1s", "<u2"), ("t1e", "<u2"), ("t2s", "<u2"), ("t2e", "<u2"),
    ("t3s", "<u2"), ("t3e", "<u2"), ("tAs", "<u2"), ("tAe", "<u2"), ("tBs", "<u2"), ("tBe", "<u2"),
    ("ts", "<f8"), ("num", "<f8"), ("key", "<u8"), ("svc", "<u8"),
])
assert EVENT_DTYPE.itemsize == 80

_M64 = (1 << 64) - 1
HASH_SEED = 0x243f6a8885a308d3
HASH_SEED_EJB = 0x13198a2e03707344


def _mix(a: int, b: int) -> int:
    r = (a & _M64) * (b & _M64)
    return (r ^ (r >> 64)) & _M64


def hash_bytes(data: bytes, seed: int = HASH_SEED) -> int:
    """kernels/common.h::hash_bytes (join keys: logIds and service names)."""
    n = len(data)
    h = seed ^ _mix(n ^ 0xa0761d6478bd642f, 0xe7037ed1a0b428db)
    i = 0
    while n - i >= 8:
        h = _mix(h ^ int.from_bytes(data[i:i + 8], "little"), 0x8ebc6af09c88c6e3)
        i += 8
    r = n - i
    if r:
        h = _mix(h ^ int.from_bytes(data[i:], "little") ^ ((r << 59) & _M64), 0x589965cc75374cc3)
    return _mix(h, 0x1d8e4e27c47d124f)

_WS = b" \t\n\r\x0b\x0c"


def _is_ws(c: int) -> bool:
    return c in (32, 9, 10, 13, 11, 12)


def _match(p: bytes, i: int, lit: bytes) -> bool:
    return p[i:i + len(lit)] == lit


def _parse_int_tok(p: bytes, s: int, e: int):
    i = s
    neg = False
    if i < e and p[i] in b"+-":
        neg = p[i] == ord("-")
        i += 1
    if i + 1 < e and p[i] == ord("0") and p[i + 1] in b"xX":
        return None
    v = 0
    nd = 0
    while i < e and 48 <= p[i] <= 57:
        v = v * 10 + (p[i] - 48)
        i += 1
        nd += 1
        if nd > 15:
            return None
    if nd == 0:
        return float("nan")
    return -float(v) if neg else float(v)


def _parse_log_ts(p: bytes, s1, e1, s2, e2, tz: TzOffset):
    vals, nds = [], []
    for s, e in ((s1, e1), (s2, e2)):
        cur, cnt = 0, 0
        i = s
        while i <= e:
            end = i == e
            c = ord("-") if end else p[i]
            if c in (45, 58, 44):  # - : ,
                if len(vals) >= 8:
                    return None, False
                vals.append(cur)
                nds.append(cnt)
                cur, cnt = 0, 0
                if end:
                    break
            elif 48 <= c <= 57:
                cur = cur * 10 + (c - 48)
                cnt += 1
                if cnt > 12:
                    return None, False
            else:
                return None, False
            i += 1
    if len(vals) < 7:
        return float("nan"), False
    y = vals[0] + 1900 if 0 <= vals[0] <= 99 else vals[0]
    local = make_date_ms(y, vals[1] - 1, vals[2], vals[3], vals[4], vals[5], vals[6])
    t = tz.local_to_utc(local)
    strict = (len(vals) == 7 and nds[0] == 4 and nds[1] == 2 and nds[2] == 2 and nds[3] == 2
              and nds[4] == 2 and nds[5] == 2 and 1 <= nds[6] <= 3)
    return t, strict


def parse_line(p: bytes, fk: int, tz: TzOffset):
    """Returns (kind, mask, ntok, toks(list of (s,e)), tA, tB, ts, num, wm_ts)."""
    n = len(p)
    ts_, te_ = [], []
    ntok = 0
    in_tok = False
    if n > 0 and _is_ws(p[0]):
        ts_.append(0); te_.append(0); ntok = 1
    info1 = info2 = -1
    ejb_entry = ejb_exit = ct_start = ct_stop = False
    baf = nonascii = False
    m = 0
    for i in range(n):
        c = p[i]
        nonascii |= c >= 0x80
        w = _is_ws(c)
        if not w and not in_tok:
            if ntok < 16:
                ts_.append(i)
            in_tok = True
        if w and in_tok:
            if ntok < 16:
                te_.append(i)
            ntok += 1
            in_tok = False
        if c == 73 and _match(p, i, b"INFO"):
            if info1 < 0:
                info1 = i
            elif info2 < 0 and i >= info1 + 4:
                info2 = i
            j = i + 4
            while j < n and p[j] == 32:
                j += 1
            ejb_entry |= _match(p, j, b"[CommonTiming] The EJB")
            ejb_exit |= _match(p, j, b"[CommonTiming] Total time")
            ct_start |= _match(p, j, b"CommonTiming::Start")
            ct_stop |= _match(p, j, b"CommonTiming::Stop")
            if _match(p, i, b"INFO  auditTrailId="):
                m |= PM_AUTR_MAP
        elif c == 93:  # ']'
            if not baf and i + 1 < n and p[i + 1] == 32:
                j = i + 1
                while j < n and p[j] == 32:
                    j += 1
                if _match(p, j, b"INFO "):
                    k = i - 2
                    while k >= 0 and p[k] != 32:
                        if p[k] == 91:
                            baf = True
                            break
                        k -= 1
        elif c == 60:  # '<'
            if _match(p, i, b"<stopWatchList>"): m |= PM_SW_START
            if _match(p, i, b"</stopWatchList>"): m |= PM_SW_END
            if _match(p, i, b"<name>"): m |= PM_SW_NAME
            if _match(p, i, b"<startTime>"): m |= PM_SW_STARTTS
            if _match(p, i, b"<stopTime>"): m |= PM_SW_STOPTS
            if _match(p, i, b"<value>"): m |= PM_SOAP_VALUE
            if p[i:i + 15].lower() == b"<accountnumber>": m |= PM_SOAP_ACCT
            if p[i:i + 24].lower() == b"<key>accountnumber</key>": m |= PM_SOAP_KEY
        elif c == 58:  # ':'
            if _match(p, i, b": RequestTrace [stopWatchList="): m |= PM_EL_START
    if in_tok:
        if ntok < 16:
            te_.append(n)
        ntok += 1
    elif n > 0 and _is_ws(p[n - 1]) and ntok < 16:
        ts_.append(n); te_.append(n); ntok += 1
    if n > 0 and p[0] == 93:
        m |= PM_EL_END
    if _match(p, 0, b"Audit Trail id"):
        j = 14
        while j < n and p[j] == 32:
            j += 1
        if j < n and p[j] == 58:
            m |= PM_AUTR_HDR
    if _match(p, 0, b"=== jbossId"):
        for i in range(11, n - 3):
            if p[i] == 73 and p[i + 1] == 79 and p[i + 2] == 61:
                if p[i + 3] == 73: m |= PM_SOAP_IN
                if p[i + 3] == 79: m |= PM_SOAP_OUT
    if baf: m |= PM_BAF
    if nonascii: m |= PM_HOST
    toks = [(ts_[k], te_[k]) for k in range(min(ntok, 16))]
    ts = float("nan")
    num = float("nan")
    wm = None
    ts_host = False
    if ntok >= 3:
        t, strict = _parse_log_ts(p, toks[1][0], toks[1][1], toks[2][0], toks[2][1], tz)
        if t is None:
            ts_host = True
        else:
            ts = t
            if strict and t == t:
                wm = t
    kind = LK_NONE
    tA = tB = (NOTOK, NOTOK)
    if fk == FILE_SOAP:
        if m & SOAP_BITS:
            kind = LK_SOAP
        m &= SOAP_BITS | PM_HOST
    else:
        if fk == FILE_SERVER and ejb_entry:
            kind = LK_EJB_ENTRY
        elif fk == FILE_SERVER and ejb_exit:
            kind = LK_EJB_EXIT
        elif ct_start:
            kind = LK_CT_ENTRY
        elif ct_stop:
            kind = LK_CT_EXIT
        elif fk == FILE_APP:
            m &= ~SOAP_BITS
            if m & AUDIT_BITS:
                kind = LK_APP
        if kind == LK_EJB_ENTRY:
            if 13 < ntok:
                tA = toks[13]
        elif kind == LK_EJB_EXIT:
            if 9 < ntok:
                tA = toks[9]
            if 11 < ntok:
                tB = toks[11]
                v = _parse_int_tok(p, toks[11][0], toks[11][1])
                if v is None:
                    m |= PM_HOST
                else:
                    num = v
        elif kind in (LK_CT_ENTRY, LK_CT_EXIT):
            s0 = info1 + 4
            e0 = info2 if info2 >= 0 else n
            if info2 >= 0:
                m |= PM_HAS_INFO2
            k = 0
            it = False
            cs = 0
            i = s0
            while i <= e0:
                w = (i == e0) or _is_ws(p[i])
                if not w and not it:
                    it = True
                    cs = i
                if w and it:
                    it = False
                    if k == 1:
                        tA = (cs, i)
                    if k == 5:
                        tB = (cs, i)
                    k += 1
                    if k > 5:
                        break
                i += 1
            if kind == LK_CT_EXIT and tB[0] != NOTOK:
                v = _parse_int_tok(p, tB[0], tB[1])
                if v is None:
                    m |= PM_HOST
                else:
                    num = v
    if ts_host and LK_EJB_ENTRY <= kind <= LK_CT_EXIT:
        m |= PM_HOST
    key = svc = 0
    if LK_EJB_ENTRY <= kind <= LK_CT_EXIT and not (m & PM_HOST) and ntok >= 1:
        a0, b0 = toks[0]
        if a0 < b0 and p[a0] == ord("["):
            a0 += 1
        if b0 > a0 and p[b0 - 1] == ord("]"):
            b0 -= 1
        if b"[" not in p[a0:b0] and b"]" not in p[a0:b0]:
            toks = [(a0, b0)] + toks[1:]
            key = hash_bytes(p[a0:b0])
            seed = HASH_SEED_EJB if kind <= LK_EJB_EXIT else HASH_SEED
            svc = hash_bytes(p[tA[0]:tA[1]] if tA[0] != NOTOK else b"undefined", seed)
            m |= PM_KEYS
    return kind, m, min(ntok, 15), toks, tA, tB, ts, num, wm, key, svc


def parse_batch(chunks: Sequence[Tuple[int, bytes]], tz: TzOffset, file_open: dict = None,
                chunk_files: Sequence[int] = None):
    """chunks: [(file_kind, bytes)] in batch order.  Returns (events ndarray, n_lines, watermark,
    batch_bytes).  ``file_open`` carries the elapsed-section state per file id across batches."""
    file_open = {} if file_open is None else file_open
    buf = b"".join(b for _, b in chunks)
    rows = []
    masks = []
    line_idx = 0
    wm = None
    off = 0
    for ci, (fk, data) in enumerate(chunks):
        pos = 0
        chunk_rows = []
        while pos < len(data):
            nl = data.index(b"\n", pos)
            raw = data[pos:nl]
            ln_off = off + pos
            ln = raw[:-1] if raw.endswith(b"\r") else raw
            rec = {"line": line_idx, "chunk": ci, "off": ln_off, "len": len(ln), "keep": False}
            if 0 < len(ln) <= 65000:
                kind, m, ntok, toks, tA, tB, ts, num, w, key, svc = parse_line(ln, fk, tz)
                if w is not None and (wm is None or w > wm):
                    wm = w
                rec.update(kind=kind, mask=m, ntok=ntok, toks=toks, tA=tA, tB=tB, ts=ts, num=num,
                           keep=kind != LK_NONE, key=key, svc=svc)
            elif len(ln) > 65000:
                rec.update(kind=LK_SOAP if fk == FILE_SOAP else LK_APP, mask=PM_HOST, ntok=0, toks=[],
                           tA=(NOTOK, NOTOK), tB=(NOTOK, NOTOK), ts=float("nan"), num=float("nan"), keep=True)
            else:
                rec.update(kind=LK_NONE, mask=0, ntok=0, toks=[], tA=(NOTOK, NOTOK), tB=(NOTOK, NOTOK),
                           ts=float("nan"), num=float("nan"))
            chunk_rows.append(rec)
            line_idx += 1
            pos = nl + 1
        # elapsed-section scan for app chunks
        if fk == FILE_APP:
            fid = chunk_files[ci] if chunk_files is not None else ci
            opened = file_open.get(fid, False)
            for rec in chunk_rows:
                m = rec["mask"]
                is_open = bool(m & PM_EL_START)
                is_close = bool(m & PM_EL_END) and not (m & PM_AUTR_MAP) and not is_open
                if opened and not is_open:
                    rec["mask"] |= PM_IN_SECTION
                    if not rec["keep"]:
                        rec["keep"] = True
                        rec["kind"] = LK_APP
                if is_open:
                    opened = True
                elif is_close:
                    opened = False
            file_open[fid] = opened
        rows.extend(chunk_rows)
        off += len(data)
    keep = [r for r in rows if r["keep"]]
    ev = np.zeros(len(keep), dtype=EVENT_DTYPE)
    for i, r in enumerate(keep):
        ev[i]["line"] = r["line"]; ev[i]["chunk"] = r["chunk"]; ev[i]["off"] = r["off"]
        ev[i]["len"] = r["len"]; ev[i]["mask"] = r["mask"]; ev[i]["kind"] = r["kind"]
        ev[i]["ntok"] = r["ntok"]
        toks = r["toks"]
        for k, nm in enumerate(("t0", "t1", "t2", "t3")):
            s, e = toks[k] if k < len(toks) else (NOTOK, NOTOK)
            ev[i][nm + "s"] = s; ev[i][nm + "e"] = e
        ev[i]["tAs"], ev[i]["tAe"] = r["tA"]
        ev[i]["tBs"], ev[i]["tBe"] = r["tB"]
        ev[i]["ts"] = r["ts"]; ev[i]["num"] = r["num"]
        ev[i]["key"] = r.get("key", 0); ev[i]["svc"] = r.get("svc", 0)
    return ev, line_idx, wm, buf


def tz_table(tz: TzOffset, years=(1990, 2100)) -> List[Tuple[int, int]]:
    """(local_start_ms, offset_ms) rows for the device/host TzTable (fixed zones: one row)."""
    if tz.fixed_ms is not None:
        return [(-(1 << 61), tz.fixed_ms)]
    import datetime as dt
    rows = []
    prev = None
    t = dt.datetime(years[0], 1, 1, tzinfo=dt.timezone.utc)
    end = dt.datetime(years[1], 1, 1, tzinfo=dt.timezone.utc)
    step = dt.timedelta(hours=1)
    while t < end and len(rows) < 64:
        ms = int(t.timestamp() * 1000)
        off = tz.offset_ms_for_utc(ms)
        if off != prev:
            rows.append((ms + off if rows else -(1 << 61), off))
            prev = off
        t += step if rows and len(rows) > 1 else dt.timedelta(days=7)
    return rows
