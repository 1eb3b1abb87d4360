"""Synthetic WildFly log generator (SURVEY Appendix A grammar).

Produces, per JVM host, the three log kinds the parser understands -- ``server.log`` (EJB
CommonTiming), ``app.log`` (standard CommonTiming, BAF metadata, audit trails) and
``soap_io.log`` (request/response with account numbers, incl. the riskStrategy key/value
form) -- plus configurable noise lines, with a seeded RNG and a planted-anomaly schedule so
that alerts are known a priori.  Paths follow ``/net/<server>/export/jvm1/log/<file>`` so
``path.split('/')[2]`` is the server, as the reference requires.

``generate()`` returns timestamped lines per file; ``batches()`` slices them into the
``(now_ms, [(path, lines)])`` batches consumed by both the oracle and the engine.  The bench
uses the native generator (``csrc/runtime/synth.cpp``) which emits the same grammar.
"""
from __future__ import annotations

import dataclasses
import datetime as dt
import math
import random
from typing import Dict, List, Optional, Sequence, Tuple

LOG_DIR = "/net/{server}/export/jvm1/log/{file}"
_PAD = "ABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789abcdefghijklmnopqrstuvwxyz"


@dataclasses.dataclass
class Anomaly:
    server: str
    service: str            # full service name as emitted, e.g. "getFoo" or "Provider[cb-util-3]"
    start_ms: int
    end_ms: int
    factor: float = 20.0


@dataclasses.dataclass
class SynthConfig:
    servers: int = 2
    ejb_services: int = 8             # top-level services (S:<name>)
    provider_services: int = 6        # sub-services Provider[<name>]
    tx_per_sec_per_server: float = 2.0
    start_ms: int = 1578391200000     # 2020-01-07 10:00:00 UTC
    duration_s: float = 600.0
    sub_calls: Tuple[int, int] = (1, 3)
    base_elapsed_ms: Tuple[float, float] = (60.0, 900.0)
    noise_lines_per_tx: int = 3
    riskid_fraction: float = 0.15
    baf_fraction: float = 0.3
    audit_fraction: float = 0.05
    missing_logid_fraction: float = 0.02
    soap_late_fraction: float = 0.1   # account arrives after the exits (exercises need cache)
    no_acct_fraction: float = 0.03    # never gets an account (exercises expiry)
    anomalies: Sequence[Anomaly] = ()
    # capacity stress: every provider call of a request opens before any closes (many open
    # partials per logId, many parked records when the account is late), and logIds get this
    # many extra characters (the device join keeps 80 inline)
    overlap_subs: bool = False
    logid_pad: int = 0
    seed: int = 1234
    tz_offset_ms: int = 0             # log timestamps written in this offset (UTC default)


def fmt_ts(ms: int, tz_offset_ms: int = 0) -> str:
    t = dt.datetime(1970, 1, 1) + dt.timedelta(milliseconds=ms + tz_offset_ms)
    return t.strftime("%Y-%m-%d %H:%M:%S,") + f"{t.microsecond // 1000:03d}"


def fmt_iso(ms: int, tz_offset_ms: int = -6 * 3600000) -> str:
    t = dt.datetime(1970, 1, 1) + dt.timedelta(milliseconds=ms + tz_offset_ms)
    sign = "-" if tz_offset_ms < 0 else "+"
    off = abs(tz_offset_ms) // 60000
    return t.strftime("%Y-%m-%dT%H:%M:%S.") + f"{t.microsecond // 1000:03d}{sign}{off // 60:02d}:{off % 60:02d}"


class Generator:
    def __init__(self, cfg: SynthConfig):
        self.cfg = cfg
        self.rng = random.Random(cfg.seed)
        self.server_names = [f"jvm{i:02d}" for i in range(cfg.servers)]
        self.ejb = [f"getSvc{i:04d}" for i in range(cfg.ejb_services)]
        self.prov = [f"cb-util-{i:03d}" for i in range(cfg.provider_services)]
        self.base = {}
        for s in self.ejb:
            self.base[s] = self.rng.uniform(*cfg.base_elapsed_ms)
        for s in self.prov:
            self.base[f"Provider[{s}]"] = self.rng.uniform(*cfg.base_elapsed_ms) * 0.4
        self.lines: Dict[str, List[Tuple[int, int, str]]] = {}
        self._seq = 0

    def path(self, server: str, kind: str) -> str:
        return LOG_DIR.format(server=server, file=kind)

    def _emit(self, server: str, kind: str, ts: int, text: str):
        self._seq += 1
        self.lines.setdefault(self.path(server, kind), []).append((ts, self._seq, text))

    def _elapsed(self, server: str, service: str, t: int) -> int:
        b = self.base[service]
        v = self.rng.lognormvariate(math.log(b), 0.25)
        for a in self.cfg.anomalies:
            if a.server == server and a.service == service and a.start_ms <= t < a.end_ms:
                v *= a.factor
        return max(1, int(v))

    def _noise(self, server: str, kind: str, ts: int, log_id: str):
        r = self.rng.random()
        if kind == "soap_io.log":
            self._emit(server, kind, ts, f"    <ns2:field{int(r * 9)}>value{int(r * 1000)}</ns2:field{int(r * 9)}>")
        else:
            lvl = "DEBUG" if r < 0.6 else "INFO "
            self._emit(server, kind, ts, f"[{log_id}] {fmt_ts(ts, self.cfg.tz_offset_ms)} {lvl} "
                                         f"[com.acme.svc.Handler{int(r * 50)}] processed step {int(r * 1e6)}")

    def transaction(self, server: str, t0: int, idx: int):
        c, rng = self.cfg, self.rng
        tz = c.tz_offset_ms
        log_id = f"{server.upper()}-{idx:08d}"
        if c.logid_pad:
            log_id += "-" + (_PAD * (c.logid_pad // len(_PAD) + 1))[:c.logid_pad]
        missing = rng.random() < c.missing_logid_fraction
        lid = "" if missing else log_id
        acct = str(rng.randint(10 ** 15, 10 ** 16 - 1))
        ejb = rng.choice(self.ejb)
        total = self._elapsed(server, ejb, t0)
        t_end = t0 + total
        # SOAP request with account
        late = rng.random() < c.soap_late_fraction
        no_acct = rng.random() < c.no_acct_fraction
        soap_t = t_end + rng.randint(50, 15000) if late else t0
        self._emit(server, "soap_io.log", soap_t, f"=== jbossId={log_id} IO=I")
        self._noise(server, "soap_io.log", soap_t, log_id)
        if not no_acct:
            if rng.random() < c.riskid_fraction:
                self._emit(server, "soap_io.log", soap_t, "      <key>AccountNumber</key>")
                self._emit(server, "soap_io.log", soap_t, f"      <value>{acct}</value>")
            else:
                self._emit(server, "soap_io.log", soap_t, f"      <accountNumber>{acct}</accountNumber>")
        self._emit(server, "soap_io.log", soap_t + 1, f"=== jbossId={log_id} IO=O")
        # top-level EJB timing
        self._emit(server, "server.log", t0,
                   f"[{lid}] {fmt_ts(t0, tz)} INFO  [CommonTiming] The EJB call started for bean "
                   f"Delegation method: {ejb}")
        for _ in range(c.noise_lines_per_tx):
            kind = rng.choice(["server.log", "app.log", "app.log"])
            self._noise(server, kind, rng.randint(t0, t_end), lid)
        # provider sub calls
        n_sub = rng.randint(*c.sub_calls)
        use_audit = rng.random() < c.audit_fraction and not missing
        sub_records = []
        cursor = t0 + 1
        for i in range(n_sub):
            p = rng.choice(self.prov)
            svc = f"Provider[{p}]"
            el = self._elapsed(server, svc, cursor)
            if c.overlap_subs:  # all starts (t0+1 .. t0+n_sub) before all stops
                s_t = min(t0 + 1 + i, t_end - 1)
                e_t = min(max(s_t + el, t0 + 1 + n_sub), t_end - 1)
            else:
                s_t = min(cursor, t_end - 1)
                e_t = min(s_t + el, t_end - 1)
            el = max(0, e_t - s_t)
            sub_records.append((svc, s_t, e_t, el))
            cursor = e_t + 1
            if use_audit:
                continue
            baf = rng.random() < c.baf_fraction
            pre = f"[baf][x:y:{acct}] " if baf else ""
            self._emit(server, "app.log", s_t,
                       f"[{lid}] {fmt_ts(s_t, tz)} {pre}INFO  CommonTiming::Start: {svc} begin")
            self._emit(server, "app.log", e_t,
                       f"[{lid}] {fmt_ts(e_t, tz)} {pre}INFO  CommonTiming::Stop: {svc} - total time {el} ms")
        if use_audit:
            autr = f"A{idx:07d}{server}"
            ta = t0 + 2
            self._emit(server, "app.log", ta, f"[{log_id}] {fmt_ts(ta, tz)} [baf][x:{acct}] INFO  auditTrailId={autr}")
            tb = t_end - 1
            block = [f"Audit Trail id : {autr}",
                     f"[{log_id}] {fmt_ts(tb, tz)} INFO  com.acme.Audit: RequestTrace [stopWatchList="]
            rules_el = rng.randint(1, 40)
            for svc, s_t, e_t, el in sub_records:
                block.append(f"  {svc}:[{el} millis] ok")
            block.append(f"  RulesEngine:[{rules_el} millis] ok")
            block.append("]")
            block.append("<stopWatchList>")
            for svc, s_t, e_t, el in sub_records:
                block += [f"  <name>{svc}</name>", f"  <startTime>{fmt_iso(s_t)}</startTime>",
                          f"  <stopTime>{fmt_iso(e_t)}</stopTime>"]
            block += ["  <name>RulesEngine</name>", f"  <startTime>{fmt_iso(t0 + 1)}</startTime>",
                      f"  <stopTime>{fmt_iso(t0 + 1 + rules_el)}</stopTime>", "</stopWatchList>"]
            for ln in block:
                self._emit(server, "app.log", tb, ln)
        self._emit(server, "server.log", t_end,
                   f"[{lid}] {fmt_ts(t_end, tz)} INFO  [CommonTiming] Total time taken for: {ejb} - {total} ms")

    def generate(self) -> Dict[str, List[Tuple[int, int, str]]]:
        c = self.cfg
        idx = 0
        for server in self.server_names:
            t = float(c.start_ms)
            end = c.start_ms + c.duration_s * 1000
            while True:
                t += self.rng.expovariate(c.tx_per_sec_per_server) * 1000.0
                if t >= end:
                    break
                idx += 1
                self.transaction(server, int(t), idx)
        for fp in self.lines:
            self.lines[fp].sort(key=lambda x: (x[0], x[1]))
        return self.lines


def batches(lines: Dict[str, List[Tuple[int, int, str]]], start_ms: int, batch_s: float,
            end_ms: Optional[int] = None):
    """Slice per-file timestamped lines into batches of ``batch_s`` seconds of log time.
    Each batch's clock is the watermark rule: max line timestamp of previous batches."""
    files = sorted(lines)
    if end_ms is None:
        end_ms = max((v[-1][0] for v in lines.values() if v), default=start_ms) + 1
    pos = {f: 0 for f in files}
    out = []
    t = start_ms
    while t < end_ms:
        hi = t + int(batch_s * 1000)
        chunks = []
        for f in files:
            arr = lines[f]
            i = pos[f]
            j = i
            while j < len(arr) and arr[j][0] < hi:
                j += 1
            if j > i:
                chunks.append((f, [x[2] for x in arr[i:j]]))
            pos[f] = j
        out.append(chunks)
        t = hi
    return out


def with_watermarks(batch_list, tz=None):
    """Attach the engine's watermark clock to every batch: now(b) = max leading line timestamp
    over batches < b (0 for the first)."""
    from .timeparse import leading_line_ts
    res = []
    w = 0.0
    for chunks in batch_list:
        res.append((w, chunks))
        for _, ls in chunks:
            for ln in ls:
                v = leading_line_ts(ln, tz)
                if v is not None and v > w:
                    w = v
    return res


def to_bytes(chunks) -> List[Tuple[str, bytes]]:
    return [(fp, ("\n".join(ls) + "\n").encode("utf-8")) for fp, ls in chunks]
