"""Daily-rolling file logger (reference ``logger.js:1-127``, simple-node-logger settings).

Files are ``<logDir>/<prefix>.log.YYYYMMDD`` (``fileNamePattern`` / ``dateFormat``), each line
``YYYYMMDD HH:mm:ss <LEVEL> <message>`` (``timestampFormat``), with the level colourised the
same way when ``colorize`` is on (cyan info, yellow warn, red error, green debug).  The
supervisor prunes files older than ``appLogRetentionDays`` (apm_manager.js:532-566; see
``prune_logs``).
"""
from __future__ import annotations

import datetime as _dt
import glob
import logging
import os
import re
import threading
import time
from typing import Optional

_COLORS = {"INFO": "\x1b[36m", "WARNING": "\x1b[33m", "ERROR": "\x1b[31m", "CRITICAL": "\x1b[31m",
           "DEBUG": "\x1b[32m"}
_RESET = "\x1b[39m"
_LEVEL_NAMES = {"WARNING": "WARN", "CRITICAL": "FATAL"}


class DailyRollingHandler(logging.Handler):
    def __init__(self, log_dir: str, prefix: str, colorize: bool = True, clock=time.time):
        super().__init__()
        self.dir = log_dir
        self.prefix = prefix
        self.colorize = colorize
        self.clock = clock
        self._day = None
        self._fh = None
        self._lock2 = threading.Lock()
        os.makedirs(log_dir, exist_ok=True)

    def path_for(self, t: float) -> str:
        return os.path.join(self.dir, f"{self.prefix}.log.{_dt.datetime.fromtimestamp(t).strftime('%Y%m%d')}")

    def _stream(self, t: float):
        day = _dt.datetime.fromtimestamp(t).strftime("%Y%m%d")
        if day != self._day:
            if self._fh:
                self._fh.close()
            self._fh = open(self.path_for(t), "a", encoding="utf-8")
            self._day = day
        return self._fh

    def format_line(self, record: logging.LogRecord) -> str:
        ts = _dt.datetime.fromtimestamp(record.created).strftime("%Y%m%d %H:%M:%S")
        lvl = _LEVEL_NAMES.get(record.levelname, record.levelname)
        msg = record.getMessage()
        if record.exc_info:
            msg += "\n" + logging.Formatter().formatException(record.exc_info)
        if self.colorize and record.levelname in _COLORS:
            msg = _COLORS[record.levelname] + msg + _RESET
        return f"{ts} {lvl} {msg}\n"

    def emit(self, record):
        try:
            with self._lock2:
                fh = self._stream(record.created)
                fh.write(self.format_line(record))
                fh.flush()
        except Exception:  # pragma: no cover
            self.handleError(record)

    def close(self):
        with self._lock2:
            if self._fh:
                self._fh.close()
                self._fh = None
        super().close()


def set_global_logger(log_dir: Optional[str], prefix: str, level=logging.INFO, colorize: bool = True,
                      also_stderr: bool = False) -> logging.Logger:
    """setGlobalLogger (util_methods.js:419-428): (re)point the root 'apm' logger at
    ``<log_dir>/<prefix>.log.<date>``; called again on config reload."""
    lg = logging.getLogger("apm")
    lg.setLevel(level)
    for h in list(lg.handlers):
        if isinstance(h, DailyRollingHandler) or getattr(h, "_apm_stderr", False):
            lg.removeHandler(h)
            h.close()
    if log_dir:
        lg.addHandler(DailyRollingHandler(log_dir, prefix, colorize))
    if also_stderr or not log_dir:
        sh = logging.StreamHandler()
        sh._apm_stderr = True  # type: ignore[attr-defined]
        sh.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
        lg.addHandler(sh)
    lg.propagate = False
    return lg


_DATE_SUFFIX = re.compile(r"\.log\.(\d{8})$")


def prune_logs(log_dir: str, retention_days: int, now: Optional[float] = None) -> list:
    """removeOldLogs (apm_manager.js:532-566): delete ``*.log.YYYYMMDD`` older than the
    retention window.  Returns the removed paths."""
    now = time.time() if now is None else now
    cutoff = (_dt.datetime.fromtimestamp(now) - _dt.timedelta(days=retention_days)).strftime("%Y%m%d")
    removed = []
    for p in glob.glob(os.path.join(log_dir, "*.log.*")):
        m = _DATE_SUFFIX.search(p)
        if m and m.group(1) < cutoff:
            try:
                os.remove(p)
                removed.append(p)
            except OSError:
                pass
    return sorted(removed)
