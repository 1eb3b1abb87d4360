"""CPU stand-in for the native engine, built on the sequential oracle (models/oracle.py).

It exposes the subset of ``_apm_native.Engine`` the host runtime uses (add_file,
process_batch, take / take_bytes, flush, metrics, n_series, files) with the same semantics,
including the watermark clock (now = max leading line timestamp of earlier batches).  It exists
so that the service, sinks, queue bridge and supervisor can be tested in containers without a
GPU; it is never selected implicitly -- ``IngestService(engine="cpu-oracle")`` must ask for it.
"""
from __future__ import annotations

import copy
from typing import Any, Dict, List, Optional, Sequence, Tuple

from ..utils.timeparse import TzOffset, leading_line_ts
from .oracle import PipelineOracle

_KIND_NAMES = {0: "SOAP", 1: "SERVER", 2: "APP"}


class CpuOracleEngine:
    def __init__(self, cfg: Dict[str, Any]):
        g = cfg.get("gpu", {})
        self.tz = TzOffset(g.get("timezone", "local"))
        self.files_: List[Tuple[str, int, str]] = []
        self._server = {}
        self.P = PipelineOracle(copy.deepcopy(cfg), self.tz, alert_clock=g.get("alertClock", "entry"),
                                server_fn=lambda p: self._server.get(p, "undefined"))
        self.watermark = 0.0
        self._taken = {"transactions": 0, "audit_db": 0, "db": 0, "st": 0, "fs": 0, "al": 0}
        self.lines = 0
        self.batches = 0

    # --- native Engine API subset
    def add_file(self, path: str, kind: int, server: str) -> int:
        self.files_.append((path, kind, server))
        self._server[path] = server
        return len(self.files_) - 1

    def files(self):
        return list(self.files_)

    def process_batch(self, buf: bytes, table: Sequence[Tuple[int, int, int]], now: float = -1.0):
        clock = self.watermark if now is None or now < 0 else now
        self.P.parse.begin_batch(clock)
        wm = self.watermark
        for fid, lo, hi in table:
            path = self.files_[fid][0]
            for ln in buf[lo:hi].decode("utf-8", "replace").split("\n"):
                if ln == "" :
                    continue
                self.lines += 1
                self.P.parse.read_line(path, ln)
                v = leading_line_ts(ln, self.tz)
                if v is not None and v > wm:
                    wm = v
        self.watermark = wm
        self.batches += 1

    def _stream(self, kind: str) -> List[str]:
        P = self.P
        return {"transactions": P.tx_out, "audit_db": P.audit_db, "db": P.tx_db, "st": P.stats, "fs": P.fs,
                "al": P.al}[kind]

    def take(self, kind: str) -> List[str]:
        s = self._stream(kind)
        out = s[self._taken[kind]:]
        self._taken[kind] = len(s)
        return out

    def take_bytes(self, kind: str) -> bytes:
        out = self.take(kind)
        return ("\n".join(out) + "\n").encode("utf-8") if out else b""

    def flush(self):
        pass

    def n_series(self) -> int:
        return sum(len(s["services"]) for s in self.P.st.servers.values()) if hasattr(self.P.st, "servers") else 0

    def metrics(self) -> Dict[str, Any]:
        return {"batches": self.batches, "lines": self.lines, "tx": len(self.P.tx_out) + len(self.P.audit_db),
                "alerts": len(self.P.al), "rollovers": len(self.P.stats), "rollover_latency_ms": []}

    def refresh_series_settings(self):
        pass

    def clear_overrides(self):
        pass

    def set_override(self, svc, o):
        pass

    def save_state(self, path: str) -> int:
        raise NotImplementedError("the CPU oracle engine has no binary checkpoint")

    def load_state(self, path: str):
        raise NotImplementedError("the CPU oracle engine has no binary checkpoint")
